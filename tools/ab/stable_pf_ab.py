#!/usr/bin/env python3
"""Same-process A/B of the LifeStable passes on 1M LifeStables (the
rows_bench input: block still lifes around an unknown window): the shipped
launch (one wave per LifeStable, stencils.hip's caps) against the
prefetching loop (k_stable<PASS, true>: each wave loads the next
LifeStable's planes before it works on the current one) on grids of 3..8
blocks per CU.  Each timing runs KS passes back to back, each on its own
fresh copy of the input; planes and flags are checked equal to the shipped
pass's.  One JSON line per variant, median over rounds.

Usage: python tools/ab/stable_pf_ab.py [--n N] [--rounds R]"""
import json
import os
import statistics
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip as tune  # noqa: E402
from rows_bench import stable_inputs  # noqa: E402

PEAK = 8000.0
NAMES = {0: "sync", 3: "step", 4: "propagate"}


def arg(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    n, rounds, ks = arg("--n", 1 << 20), arg("--rounds", 5), 4
    st = stable_inputs(n)
    works = [st.clone() for _ in range(ks)]
    cases = {}
    for p in (4, 3, 0):
        cases[f"{NAMES[p]} shipped"] = (p, lambda wk, p=p: hip.stable_pass(wk, NAMES[p]))
        for cap in (3, 4, 5, 6, 8):
            cases[f"{NAMES[p]} prefetch grid={cap}/CU"] = (
                p, lambda wk, p=p, cap=cap: tune.stable_pass(wk, 8 + p, cap))
    ref = {}
    for p in (4, 3, 0):
        w = st.clone()
        f = hip.stable_pass(w, NAMES[p])
        ref[p] = (w, f)
    res = {c: [] for c in cases}
    for _ in range(rounds):
        for c, (p, fn) in cases.items():
            for wk in works:
                wk.copy_(st)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for wk in works:
                fn(wk)
            b.record()
            b.synchronize()
            res[c].append(a.elapsed_time(b) / ks)
    for c, (p, fn) in cases.items():
        w = st.clone()
        f = fn(w)
        f = f[1] if isinstance(f, tuple) else f
        rf = ref[p][1][1] if isinstance(ref[p][1], tuple) else ref[p][1]
        ok = torch.equal(w, ref[p][0]) and torch.equal(f.to(torch.uint8), rf.to(torch.uint8))
        ms = statistics.median(res[c])
        print(json.dumps({"variant": c, "objects": n, "bytes_per_object": 10241, "ms": ms,
                          "GBps": n * 10241 / ms / 1e6, "hbm_frac": n * 10241 / ms / 1e6 / PEAK,
                          "ms_rounds": res[c], "equal_to_shipped": ok}), flush=True)


if __name__ == "__main__":
    main()
