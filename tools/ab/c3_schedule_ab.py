#!/usr/bin/env python3
"""Config 3 (64K universes x 1024 generations) on the assembly loop's
schedules (tools/gen_split_asm.py VARIANTS: 0 = shipped pipe_prio, 1..3 the
others) through the tuning build, launches interleaved, 30 each after
warm-up; outputs equal to the shipped entry point's."""
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

n, g = 1 << 16, 1024
x = hip.fill_random(n, seed=3)
ref = hip.step(x, generations=g)
out = torch.empty_like(x)
cfgs = {}
for k in range(4):
    c = tune_hip.default_cfg(g)
    if k:
        c.xchg = 24 + k          # LIFEAPI_XCHG_ASM_V(k)
    cfgs[k] = c
    tune_hip.step(x, out=out, generations=g, cfg=c)
    assert torch.equal(out, ref), k
ms = {k: [] for k in cfgs}
keys = list(cfgs)
for rep in range(40):
    for k in keys[rep % len(keys):] + keys[:rep % len(keys)]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        tune_hip.step(x, out=out, generations=g, cfg=cfgs[k])
        e1.record()
        e1.synchronize()
        if rep >= 10:
            ms[k].append(e0.elapsed_time(e1))
for k in keys:
    print(json.dumps({"schedule": k, "ms_median": statistics.median(ms[k]), "ms_min": min(ms[k])}), flush=True)
