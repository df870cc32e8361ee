#!/usr/bin/env python3
"""The one-generation search filter (Step + Contains, natural layout,
SURVEY 8(f) row 1) through the tuning build: universes per wave x resident
blocks per CU (RES: > 0 resident blocks, < 0 a grid-stride grid of that
many blocks per CU), with and without final states; launches interleaved, 30 each
after warm-up; results equal to the shipped entry point's.
usage: python tools/ab/filter_ab.py [universes]"""
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
fin = torch.empty_like(x)
w = torch.zeros((1, 64), dtype=torch.int64, device="cuda")
w[0, 10] = w[0, 11] = 3 << 40
u = torch.zeros((1, 64), dtype=torch.int64, device="cuda")
for c in (9, 10, 11, 12):
    u[0, c] = 15 << 39
u &= ~w
ref, _ = hip.step_contains(x, w, u, 1)
RES = [int(c) for c in os.environ.get("RES", "0,4,6").split(",")]  # > 0 resident blocks, < 0 grid-stride cap
UPWS = [int(c) for c in os.environ.get("UPW", "1,2,4,8").split(",")]
KEYS = [(upw, res, wf) for upw in UPWS for res in RES for wf in (False, True)]
for k in KEYS:
    got = tune_hip.step_contains_nat(x, w, u, 1, k[0], k[1], final=fin if k[2] else None)
    assert torch.equal(got, ref), k
ms = {k: [] for k in KEYS}
for rep in range(40):
    for k in KEYS[rep % len(KEYS):] + KEYS[:rep % len(KEYS)]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        tune_hip.step_contains_nat(x, w, u, 1, k[0], k[1], final=fin if k[2] else None)
        e1.record()
        e1.synchronize()
        if rep >= 10:
            ms[k].append(e0.elapsed_time(e1))
for k in KEYS:
    med = statistics.median(ms[k])
    nb = 1028 if k[2] else 516
    print(json.dumps({"universes": n, "universes_per_wave": k[0], "resident_blocks": k[1], "final": k[2],
                      "ms_median": med, "GBps": n * nb / (med * 1e-3) / 1e9}), flush=True)
