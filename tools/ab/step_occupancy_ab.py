#!/usr/bin/env python3
"""Occupancy A/B of the shipped one-generation step (config 2 / config 4
shapes): the tuning build's launch of the shipped kernel with no grid cap
(as shipped), with grid caps (blocks per CU, grid-strided), and with at most
k blocks resident per CU (unused dynamic LDS; cfg.blocks_per_cu = -k).
Ping-pong between two buffers as bench.py does, launches interleaved, 30
each after a warm-up; results must equal the shipped entry point's.
usage: [CAPS=0,-6,...] [UPW=2,4,8] [GENS=1] python tools/ab/step_occupancy_ab.py [universes ...]
(GENS > 2: the split-layout kernel, where UPW counts groups of 4 universes)"""
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

CAPS = [int(c) for c in os.environ.get("CAPS", "0,8,32,-2,-3,-4,-6,-8").split(",")]
UPW = [int(u) for u in os.environ.get("UPW", "4").split(",")]  # universes per wave (shipped: 4)
KEYS = [(u, c) for u in UPW for c in CAPS]
GENS = int(os.environ.get("GENS", "1"))  # 1024: the config-3 kernel (VALU-bound split layout)
for n in [int(a) for a in sys.argv[1:]] or [1 << 20, 1 << 24]:
    a = hip.fill_random(n, seed=2)
    b = torch.empty_like(a)
    ref = hip.step(a, generations=GENS)
    cfgs = {}
    for key in KEYS:
        c = tune_hip.default_cfg(GENS)
        c.universes_per_wave, c.blocks_per_cu = key
        cfgs[key] = c
        tune_hip.step(a, out=b, generations=GENS, cfg=c)
        assert torch.equal(b, ref), key
    ms = {key: [] for key in KEYS}
    bufs = [a, b]
    for rep in range(40):
        for i, key in enumerate(KEYS[rep % len(KEYS):] + KEYS[:rep % len(KEYS)]):
            src, dst = bufs[i & 1], bufs[(i + 1) & 1]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            tune_hip.step(src, out=dst, generations=GENS, cfg=cfgs[key])
            e1.record()
            e1.synchronize()
            if rep >= 10:
                ms[key].append(e0.elapsed_time(e1))
    for key in KEYS:
        med = statistics.median(ms[key])
        print(json.dumps({"universes": n, "generations": GENS, "universes_per_wave": key[0], "cap": key[1],
                          "ms_median": med, "ms_min": min(ms[key]),
                          "GBps": n * 1024 / (med * 1e-3) / 1e9 if GENS == 1 else None}), flush=True)
    del a, b, ref
    torch.cuda.empty_cache()
