"""How fast the LifeStable passes issue their VALU with the memory side
amortised: k_stable_rep (tuning build) runs a pass R times per LifeStable on
its planes in VGPRs (every repetition on the same input, so the same work),
one load and one store per LifeStable.  1M LifeStables (rows_bench inputs:
`next` = a search's next node).  The slope between R = 1 and R = 5 is the
pass's compute time per launch-equivalent; against SQ_INSTS_VALU per
LifeStable (profiles/r05/pmc_rows.json) and the clock that gives the issue
rate, in wave64 VALU instructions per SIMD-clock.  One JSON line per pass."""
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


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return sorted(ms)[len(ms) // 2]


def main():
    n = 1 << 20
    st = stable_inputs(n)
    nxt = stable_next_node(st)
    with open(os.path.join(ROOT, "profiles", "r05", "pmc_rows.json")) as f:
        pmc = json.load(f)["rows"]
    w = torch.empty_like(nxt)
    for pname in ("sync", "signal", "step", "propagate"):
        which = hip.STABLE_PASSES.index(pname)
        t = {}
        for r in (1, 3, 5):
            def run():
                w.copy_(nxt)
                tune_hip.stable_rep(w, which, r)
            # the copy's own time, to subtract
            t[r] = timed(run)
        cp = timed(lambda: w.copy_(nxt))
        slope = (t[5] - t[1]) / 4
        valu = pmc[f"k_stable {pname} (next)"]["valu_per_object"]
        print(json.dumps({"pass": pname, "objects": n, "ms_r1": t[1] - cp, "ms_r3": t[3] - cp, "ms_r5": t[5] - cp,
                          "compute_ms_per_rep": slope, "valu_per_object": valu,
                          "valu_per_simd_clock_at_2.1GHz": valu * n / 1024 / (slope / 1e3) / 2.1e9,
                          "note": "peak is 0.5 (one wave64 VALU per 2 clocks)"}), flush=True)


if __name__ == "__main__":
    main()
