#!/usr/bin/env python3
"""Is the pair layout's deficit on config 3 (tools/gen_pair_asm.py, round 2:
7-17 % slower) the single round of waves it has at 64K universes (8 per
wave, 8192 waves = one per slot)?  Same process: the shipped gens > 2 step
and the pair loop's schedules at 64K, 128K and 256K universes x 1024
generations; ns per universe-generation, median of 5 launches after 2.

Usage: python tools/ab/pair_rounds_ab.py"""
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
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip as tune  # noqa: E402


def timed(fn, reps=5, warm=2):
    for _ in range(warm):
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
    return statistics.median(ms)


def main():
    g = 1024
    for n in (1 << 16, 1 << 17, 1 << 18):
        x = hip.fill_random(n, seed=3)
        y = torch.empty_like(x)
        ref = hip.step(x, generations=g)
        cases = {"shipped": lambda: hip.step(x, out=y, generations=g)}
        for v in range(6):
            cases[f"pair v{v}"] = lambda v=v: tune.step_pair(x, y, g, v)
        res = {c: [] for c in cases}
        for _ in range(3):
            for c, fn in cases.items():
                res[c].append(timed(fn))
        for c, fn in cases.items():
            fn()
            torch.cuda.synchronize()
            ms = statistics.median(res[c])
            print(json.dumps({"universes": n, "variant": c, "ms": ms, "ns_per_universe_gen": ms * 1e6 / (n * g),
                              "frac_16slot": n * g * 16 / (ms / 1e3) / 1.2288e12,
                              "equal": bool(torch.equal(y, ref))}), flush=True)


if __name__ == "__main__":
    main()
