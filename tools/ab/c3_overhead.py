#!/usr/bin/env python3
"""Config 3's fixed per-launch cost: the shipped gens > 2 step on 64K
universes at 1024 and 2048 generations, and on 32K / 128K universes at 1024
(one / four rounds of waves); median of 7 launches after 3, interleaved.
t(64K, 2048) - t(64K, 1024) is 1024 generations of loop; the rest of
t(64K, 1024) is what a launch costs besides the loop.

Usage: python tools/ab/c3_overhead.py"""
import json
import os
import statistics
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import lifeapi_amd.hip as hip  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from pair_rounds_ab import timed  # noqa: E402


def main():
    cases = [(1 << 16, 1024), (1 << 16, 2048), (1 << 16, 512), (1 << 15, 1024), (1 << 17, 1024), (1 << 16, 64)]
    bufs = {n: (hip.fill_random(n, seed=3), torch.empty((n, 64), dtype=torch.int64, device="cuda"))
            for n in {c[0] for c in cases}}
    res = {c: [] for c in cases}
    for _ in range(4):
        for n, g in cases:
            x, y = bufs[n]
            res[(n, g)].append(timed(lambda: hip.step(x, out=y, generations=g), reps=7, warm=3))
    for n, g in cases:
        ms = statistics.median(res[(n, g)])
        print(json.dumps({"universes": n, "gens": g, "ms": ms, "ns_per_universe_gen": ms * 1e6 / (n * g),
                          "frac_16slot": n * g * 16 / (ms / 1e3) / 1.2288e12, "ms_rounds": res[(n, g)]}), flush=True)


if __name__ == "__main__":
    main()
