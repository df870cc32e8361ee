"""What Propagate's write-backs cost: the shipped
windowed Propagate (tuning build k_stable<4, true>, pass 15) on a search's
next node against the same launch storing no plane (mode bit 3: a timing
probe whose planes are left wrong), the same storing a plane's dirty line
only where that plane changed (pass 40, the unmodified object re-read at
the end to compare), and against SynchroniseStateKnown and
SignalNeighbours on the same input (read-mostly passes).  1M LifeStables,
each launch on its own fresh copy, back to back (4 per timing, median of 7)
and alone after a 768 MiB scrub (median of 8).  One JSON line."""
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
    inputs = {"next node": stable_next_node(st), "fresh options": st}
    which = os.environ.get("INPUT", "next node")
    src = inputs[which]
    forms = {"shipped": lambda w: hip.stable_pass(w, "propagate"),
             "window": lambda w: tune.stable_pass(w, 15, 0, xcd_chunk=True),
             "window_no_store": lambda w: tune.stable_pass(w, 15, 0, xcd_chunk=True, no_store=True),
             "window_plane_stores": lambda w: tune.stable_pass(w, 40, 0, xcd_chunk=True),
             "whole_no_store": lambda w: tune.stable_pass(w, 14, 0, xcd_chunk=True, no_store=True),
             "sync": lambda w: hip.stable_pass(w, "sync"),
             "signal": lambda w: hip.stable_pass(w, "signal")}
    works = [src.clone() for _ in range(4)]
    row = {"input": which, "objects": n}
    for name, fn in forms.items():
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
        row[name] = {"ms": statistics.median(ms), "ms_alone": statistics.median(alone)}
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
