"""A/B: PropagateStep and Propagate with no branch between their passes
(stable_kernels.hpp stable_step_nb, tuning build passes 6 / 7) against the
same kernels with the reference's early returns (passes 3 / 4), on a search's
next node (rows_bench.stable_next_node, 1M) and on fresh options
(rows_bench.stable_inputs).  Forms: k_stable one wave per LifeStable
("plain"), and the LDS-prefetch k_stable_dma with U = 1 / 2 LifeStables per
wave.  Each launch on a fresh copy, 4 back to back between one pair of events
(/ 4), median of 7, forms interleaved rep by rep; planes and flags checked
against the shipped pass.  One JSON line per (input, pass)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip  # noqa: E402
from rows_bench import stable_inputs, stable_next_node  # noqa: E402


def main():
    n = int(os.environ.get("N", str(1 << 20)))
    st = stable_inputs(n)
    inputs = {"next": stable_next_node(st), "still": st}
    works = [torch.empty_like(st) for _ in range(4)]
    chk = torch.empty_like(st)
    for iname, src in inputs.items():
        for pname, p_ref, p_nb in (("step", 3, 6), ("propagate", 4, 7)):
            forms = {"shipped": lambda x: hip.stable_pass(x, pname)}
            for label, p in (("ref", p_ref), ("nb", p_nb)):
                forms[f"{label}_plain"] = lambda x, p=p: tune_hip.stable_pass(x, p, 0)
                forms[f"{label}_dma_u1"] = lambda x, p=p: tune_hip.stable_pass(x, 16 + p, 0, upw=1)
                forms[f"{label}_dma_u2"] = lambda x, p=p: tune_hip.stable_pass(x, 16 + p, 0, upw=2)
            chk.copy_(src)
            want_flags = hip.stable_pass(chk, pname)
            want = chk.clone()
            row = {"input": iname, "pass": pname, "objects": n}
            for name, fn in forms.items():
                chk.copy_(src)
                f = fn(chk)
                torch.cuda.synchronize()
                row[f"{name}_exact"] = bool(torch.equal(chk, want)) and bool(torch.equal(f, want_flags))
            ms = {k: [] for k in forms}
            for _ in range(7):
                for name, fn in forms.items():
                    for w in works:
                        w.copy_(src)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for w in works:
                        fn(w)
                    b.record()
                    b.synchronize()
                    ms[name].append(a.elapsed_time(b) / len(works))
            for name, v in ms.items():
                row[f"{name}_ms"] = sorted(v)[len(v) // 2]
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
