"""A/B: LifeStable Propagate (LifeStable.hpp:718-729; PASS=stabilise:
StabiliseOptions, :677-693) with every iteration
on the whole columns against the steps after the first on a 32-row window
around the cells the step before changed (stable_kernels.hpp
stable_iter_window; tuning build k_stable<4, false / true>, k_stable_dma<5, ...>,
k_stable<5, true, false / true>), and the
product's launch, on 1M LifeStables of tools/rows_bench.py's two inputs
(fresh options on still lifes; a search's next node).  Per form: planes
and flags checked equal to the whole-column form; times back to back (4
launches, each on its own fresh copy, median of 7) and alone after a scrub.
One JSON line per input."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip as tune  # noqa: E402
from rows_bench import stable_inputs, stable_next_node  # noqa: E402


class RT:
    kind = "hip"

    def __init__(self):
        self.device = torch.device("cuda", 0)
        self.stream = torch.cuda.current_stream()


def main():
    n = int(os.environ.get("N", str(1 << 20)))
    scrub = bench.Scrub(RT())
    st = stable_inputs(n)
    inputs = {"fresh options": st, "next node": stable_next_node(st)}
    which = os.environ.get("PASS", "propagate")
    if which == "propagate":
        forms = {"whole": lambda w: tune.stable_pass(w, 14, 0, xcd_chunk=True),
                 "window": lambda w: tune.stable_pass(w, 15, 0, xcd_chunk=True),
                 "shipped": lambda w: hip.stable_pass(w, "propagate")}
    else:  # StabiliseOptions: the shipped LDS-DMA form, whole columns against the window
        forms = {"whole": lambda w: tune.stable_pass(w, 37, 0, upw=1),
                 "window": lambda w: tune.stable_pass(w, 38, 0, upw=1),
                 # k_stable (no LDS-DMA), whole columns / the later rounds on
                 # the window with the columns stashed in LDS
                 "k_whole": lambda w: tune.stable_pass(w, 6, 0, xcd_chunk=True),
                 "k_window": lambda w: tune.stable_pass(w, 7, 0, xcd_chunk=True),
                 "shipped": lambda w: hip.stable_pass(w, "stabilise")}
    works = [st.clone() for _ in range(4)]
    for iname, src in inputs.items():
        ref = src.clone()
        ref_flags = forms["whole"](ref).clone()
        row = {"pass": which, "input": iname, "objects": n}
        for fname, fn in forms.items():
            w = src.clone()
            fl = fn(w)
            torch.cuda.synchronize()
            row[fname] = {"equal": bool(torch.equal(w, ref)) and bool(torch.equal(fl, ref_flags))}
            ms = []
            for _ in range(7):
                for wk in works:
                    wk.copy_(src)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for wk in works:
                    fn(wk)
                b.record()
                b.synchronize()
                ms.append(a.elapsed_time(b) / len(works))
            alone = []
            for k in range(10):
                works[0].copy_(src)
                scrub()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                fn(works[0])
                b.record()
                b.synchronize()
                if k >= 2:
                    alone.append(a.elapsed_time(b))
            row[fname].update(ms=statistics.median(ms), ms_alone=statistics.median(alone))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
