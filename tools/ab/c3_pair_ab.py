#!/usr/bin/env python3
"""Config-3 A/B: the shipped rule-11 kernel against the pair layout
(tools/gen_pair_asm.py, tuning build) in the same process, launches
interleaved, after >= 2 s of warm-up.  One JSON line per kernel: median /
min ms over rounds, and bit-equality with the shipped kernel's output."""
import json
import os
import statistics
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip  # noqa: E402

gens = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 16
a = hip.fill_random(n, seed=3)
ref = hip.step(a, generations=gens)
outs = {}
kern = {"shipped": lambda o: hip.step(a, out=o, generations=gens)}
for v in range(6):
    kern[f"pair_v{v}"] = (lambda vv: (lambda o: tune_hip.step_pair(a, o, gens, vv)))(v)
for k in kern:
    outs[k] = torch.empty_like(a)
t0 = time.time()
while time.time() - t0 < 2.0:
    for k, f in kern.items():
        f(outs[k])
    torch.cuda.synchronize()
ms = {k: [] for k in kern}
for _ in range(12):
    for k, f in kern.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f(outs[k])
        e1.record()
        e1.synchronize()
        ms[k].append(e0.elapsed_time(e1))
for k in kern:
    print(json.dumps({"gens": gens, "n": n, "kernel": k, "ms_median": statistics.median(ms[k]), "ms_min": min(ms[k]),
                      "equal_to_reference_path": bool(torch.equal(outs[k], ref))}), flush=True)
