#!/usr/bin/env python3
"""GetPop / Contains launch shapes through the tuning build: universes per
wave x grid (cap 32 per CU as shipped, none, or at most k blocks resident);
interleaved, 30 launches each after warm-up, results equal to the shipped
entry points'.  usage: python tools/ab/reduce_ab.py [universes]"""
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
x = hip.fill_random(n, seed=7)
w = x[:1].clone()
pop_ref, con_ref = hip.pop(x), hip.contains(x, w, w)
outs = {0: torch.empty(n, dtype=torch.int32, device="cuda"), 1: torch.empty(n, dtype=torch.uint8, device="cuda")}
CAPS = [int(c) for c in os.environ.get("CAPS", "32,0,-4,-6").split(",")]
KEYS = [(kind, upw, cap) for kind in (0, 1) for upw in (4, 8) for cap in CAPS]
for k in KEYS:
    tune_hip.reduce(k[0], x, outs[k[0]], k[1], k[2], w, w)
    torch.cuda.synchronize()
    assert torch.equal(outs[k[0]].view(-1).to(torch.int64), (pop_ref if k[0] == 0 else con_ref).view(-1).to(torch.int64)), k
ms = {k: [] for k in KEYS}
for rep in range(40):
    for k in KEYS[rep % len(KEYS):] + KEYS[:rep % len(KEYS)]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        tune_hip.reduce(k[0], x, outs[k[0]], k[1], k[2], w, w)
        e1.record()
        e1.synchronize()
        if rep >= 10:
            ms[k].append(e0.elapsed_time(e1))
for k in KEYS:
    med = statistics.median(ms[k])
    nb = 516 if k[0] == 0 else 513
    print(json.dumps({"kernel": "k_pop" if k[0] == 0 else "k_contains", "universes": n, "universes_per_wave": k[1],
                      "grid": k[2], "ms_median": med, "GBps": n * nb / (med * 1e-3) / 1e9}), flush=True)
