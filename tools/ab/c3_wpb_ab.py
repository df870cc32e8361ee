#!/usr/bin/env python3
"""Config 3 (64K universes x 1024 generations, two rounds of waves) with 1,
2 or 4 (shipped) waves per block: with finer blocks the dispatcher can hand
the last round's waves to whichever SIMD frees up first, so a slower CU
holds back less of the tail (at 256K universes the same loop runs 3 % faster
per universe than at 64K, tools/ab/pair_rounds_ab.py).  Same process,
interleaved; median of 5 launches after 2, over 3 rounds; outputs checked
against the shipped launch.

Usage: python tools/ab/c3_wpb_ab.py"""
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

from pair_rounds_ab import timed  # noqa: E402


def main():
    g = 1024
    for n in (1 << 16, 1 << 18):
        x = hip.fill_random(n, seed=3)
        y = torch.empty_like(x)
        ref = hip.step(x, generations=g)
        cases = {"shipped": lambda: hip.step(x, out=y, generations=g)}
        for w in (1, 2, 4):
            cases[f"wpb={w}"] = lambda w=w: tune.step_split_wpb(x, y, g, w)
        res = {c: [] for c in cases}
        for _ in range(4):
            for c, fn in cases.items():
                res[c].append(timed(fn))
        for c, fn in cases.items():
            fn()
            torch.cuda.synchronize()
            ms = statistics.median(res[c])
            print(json.dumps({"universes": n, "variant": c, "ms": ms, "frac_16slot": n * g * 16 / (ms / 1e3) / 1.2288e12,
                              "ms_rounds": res[c], "equal": bool(torch.equal(y, ref))}), flush=True)


if __name__ == "__main__":
    main()
