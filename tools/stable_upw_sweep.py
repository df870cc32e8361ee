"""Sweep: LifeStables per wave of the LDS-prefetch pass (k_stable_dma, tuning
build: a grid of n / U waves, each a contiguous run of U LifeStables with the
next one fetched into LDS while the wave works on the current one) for
PropagateStep and Propagate on a search's next node (rows_bench.stable_next_node,
1M), against the shipped pass.  U = 128 on 1M is one wave per resident slot
(8 blocks of 4 waves per CU, 256 CUs), each running through its own eighth of
an XCD's share.  Per (pass, form): each launch on a fresh copy, 4 back to back
between one pair of events (/ 4), median of 7, forms interleaved rep by rep;
answers checked against the shipped pass.  One JSON line per pass."""
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
    upws = [int(v) for v in os.environ.get("UPW", "1,2,8,32,128").split(",")]
    src = stable_next_node(stable_inputs(n))
    works = [torch.empty_like(src) for _ in range(4)]
    chk = torch.empty_like(src)
    for pname in os.environ.get("PASSES", "step,propagate").split(","):
        p = hip.STABLE_PASSES.index(pname)
        forms = {"shipped": lambda x: hip.stable_pass(x, pname)}
        for u in upws:
            forms[f"dma_u{u}"] = lambda x, u=u: tune_hip.stable_pass(x, 16 + p, 0, upw=u)
        chk.copy_(src)
        want_flags = hip.stable_pass(chk, pname)
        want = chk.clone()
        row = {"input": "next", "pass": pname, "objects": n}
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
