#!/usr/bin/env python3
"""Occupancy A/B of the shipped one-generation step (config 2 / config 4
shapes): the tuning build's launch of the shipped kernel with no grid cap
(as shipped), with grid caps (blocks per CU, grid-strided), and with at most
k blocks resident per CU (unused dynamic LDS; cfg.blocks_per_cu = -k).
Ping-pong between two buffers as bench.py does, launches interleaved, 30
each after a warm-up; results must equal the shipped entry point's.
usage: python tools/step_occupancy_ab.py [universes ...]"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip  # noqa: E402

CAPS = [int(c) for c in os.environ.get("CAPS", "0,8,32,-2,-3,-4,-6,-8").split(",")]
for n in [int(a) for a in sys.argv[1:]] or [1 << 20, 1 << 24]:
    a = hip.fill_random(n, seed=2)
    b = torch.empty_like(a)
    ref = hip.step(a, generations=1)
    cfgs = {}
    for cap in CAPS:
        c = tune_hip.default_cfg(1)
        c.blocks_per_cu = cap
        cfgs[cap] = c
        tune_hip.step(a, out=b, generations=1, cfg=c)
        assert torch.equal(b, ref), cap
    ms = {cap: [] for cap in CAPS}
    bufs = [a, b]
    for rep in range(40):
        for i, cap in enumerate(CAPS[rep % len(CAPS):] + CAPS[:rep % len(CAPS)]):
            src, dst = bufs[i & 1], bufs[(i + 1) & 1]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            tune_hip.step(src, out=dst, generations=1, cfg=cfgs[cap])
            e1.record()
            e1.synchronize()
            if rep >= 10:
                ms[cap].append(e0.elapsed_time(e1))
    for cap in CAPS:
        med = statistics.median(ms[cap])
        print(json.dumps({"universes": n, "cap": cap, "ms_median": med, "ms_min": min(ms[cap]),
                          "GBps": n * 1024 / (med * 1e-3) / 1e9}), flush=True)
    del a, b, ref
    torch.cuda.empty_cache()
