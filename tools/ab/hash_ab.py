#!/usr/bin/env python3
"""A/B of the per-universe hash kernels (tools/tune/tune_reduce.hip) against
the shipped k_hash on 1M and 16M universes: median launch time, algorithmic
GB/s (512 B read + 8 B written per universe) and bit-equality.  One JSON
line per (variant, grid cap, n)."""
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
import tune_hip  # noqa: E402


def t(fn, reps=15):
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    return statistics.median(ms)


for n in (1 << 20, 1 << 24):
    a = hip.fill_random(n, seed=4)
    ref = hip.hashes(a)
    out = torch.empty_like(ref)
    for _ in range(3):
        hip.hashes(a)
    ms = t(lambda: hip.hashes(a))
    print(json.dumps({"n": n, "variant": "shipped", "ms": ms, "GBps": n * 520 / ms / 1e6}), flush=True)
    for v, caps in ((0, (0, 32)), (1, (0, 32)), (2, (0, 16)), (4, (0, 8, 16, 32)), (5, (0, 8, 16, 32))):
        for cap in caps:
            tune_hip.hash_variant(a, v, cap, out)
            ok = bool(torch.equal(out, ref))
            ms = t(lambda: tune_hip.hash_variant(a, v, cap, out))
            print(json.dumps({"n": n, "variant": v, "blocks_per_cu": cap, "ms": ms, "GBps": n * 520 / ms / 1e6,
                              "equal": ok}), flush=True)
    del a, ref, out
    torch.cuda.empty_cache()
