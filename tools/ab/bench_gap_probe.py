#!/usr/bin/env python3
"""Why does bench.py's timed region give a slower per-launch time for the
same shipped config-2 launch than tools/ab/order_policy_ab.py on the same box
(0.160 against 0.151 ms)?  One process, alternating: (A) the A/B's sequence
(4 untimed launches right before, then 50 back to back between events) and
(B) the bench's (9 untimed, a synchronize, then 50 between events), on the
same buffers; then (C) B with a fresh pair of buffers allocated the bench's
way, and (D) A on bench-style buffers.

Usage: python tools/ab/bench_gap_probe.py"""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import lifeapi_amd.hip as hip  # noqa: E402


def run(bufs, warm, sync, k=50):
    cur = 0
    for _ in range(warm):
        hip.step(bufs[cur], out=bufs[1 - cur], generations=1)
        cur = 1 - cur
    if sync:
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        hip.step(bufs[cur], out=bufs[1 - cur], generations=1)
        cur = 1 - cur
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / k


def main():
    n = 1 << 20
    ab = [hip.fill_random(n, seed=2), torch.empty((n, 64), dtype=torch.int64, device="cuda")]
    a = hip.fill_random(n, seed=2, first_universe=0)
    be = [a, torch.empty_like(a)]
    res = {"A (4 warm, no sync)": [], "B (9 warm, sync)": [], "C (B, bench buffers)": [], "D (A, bench buffers)": [],
           "E (0 warm, sync)": []}
    for _ in range(5):
        res["A (4 warm, no sync)"].append(run(ab, 4, False))
        res["B (9 warm, sync)"].append(run(ab, 9, True))
        res["C (B, bench buffers)"].append(run(be, 9, True))
        res["D (A, bench buffers)"].append(run(be, 4, False))
        res["E (0 warm, sync)"].append(run(ab, 0, True))
    for c, v in res.items():
        print(json.dumps({"case": c, "ms": sorted(v)[len(v) // 2], "all": v}), flush=True)
    # the bench also loads the tuning build (its side launches): does that change the launch?
    sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
    import tune_hip  # noqa: F401
    v = [run(ab, 4, False) for _ in range(5)]
    print(json.dumps({"case": "A after importing tune_hip", "ms": sorted(v)[2], "all": v}), flush=True)
    x = torch.empty((n, 64), dtype=torch.int64, device="cuda")
    tune_hip.step_order(ab[0], x, 1, nts=True, resident=0)
    torch.cuda.synchronize()
    v = [run(ab, 4, False) for _ in range(5)]
    print(json.dumps({"case": "A after one tuning-build launch", "ms": sorted(v)[2], "all": v}), flush=True)


if __name__ == "__main__":
    main()
