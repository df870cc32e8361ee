#!/usr/bin/env python3
"""Same-process A/B of the LifeStable passes on 1M LifeStables (the
rows_bench input): each pass's shipped launch shape (stencils.hip
kStablePassResident) with the plain block mapping against the XCD-chunked
one (k_stable's reverse bit 1: XCD k streams one contiguous eighth of the
batch; tools/ab/xcd_ab.hip for the bare access shapes).  Each timing runs KS
passes back to back on fresh copies; planes and flags are checked equal to
the shipped pass's.  One JSON line per variant, median over rounds.

Usage: python tools/ab/stable_xcd_ab.py [--n N] [--rounds R]"""
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
CAPS = {0: -3, 1: -3, 2: -3, 3: -3, 4: 0, 5: -4}   # stencils.hip kStablePassResident


def arg(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    n, rounds, ks = arg("--n", 1 << 20), arg("--rounds", 5), 4
    st = stable_inputs(n)
    works = [st.clone() for _ in range(ks)]
    cases = {}
    for p, name in enumerate(hip.STABLE_PASSES):
        cases[f"{name} shipped"] = (p, lambda wk, name=name: hip.stable_pass(wk, name))
        for chunk in (False, True):
            cases[f"{name} {'xcd_chunk' if chunk else 'plain'}"] = (
                p, lambda wk, p=p, chunk=chunk: tune.stable_pass(wk, p, CAPS[p], xcd_chunk=chunk))
    ref = {}
    for p, name in enumerate(hip.STABLE_PASSES):
        w = st.clone()
        ref[p] = (w, hip.stable_pass(w, name))
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
        ok = torch.equal(w, ref[p][0]) and torch.equal(f, ref[p][1])
        ms = statistics.median(res[c])
        print(json.dumps({"variant": c, "objects": n, "bytes_per_object": 10241, "ms": ms,
                          "GBps": n * 10241 / ms / 1e6, "hbm_frac": n * 10241 / ms / 1e6 / PEAK,
                          "ms_rounds": res[c], "equal_to_shipped": ok}), flush=True)


if __name__ == "__main__":
    main()
