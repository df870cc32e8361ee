#!/usr/bin/env python3
"""Fused Step + Contains A/B on the config-3 shape (64K universes x 1024
gens; and 4K x 4096 with hits): the plain shipped step, the shipped fused
kernel, and the tuning build's variants (step_kernels.hpp: 0 compiled loop,
1 assembly loop, 2 lean SALU bookkeeping, 3 on the target's row window, 4 its
scalar test late, 5 batched over four generations, 6 / 7 = 3 / 5 in the low
register layout, 8 = the wider windows (shipped: 7 then 8); argv: the
variants to run, default
0..7, and "six" for a 6-row target (a loaf in its 6 x 6 box) instead), launches
interleaved after a 2 s warm-up.  Results must equal the shipped fused
kernel's."""
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

n, g = 1 << 16, 1024
x = hip.fill_random(n, seed=3)
SIX = "six" in sys.argv[1:]
w = torch.zeros((1, 64), dtype=torch.int64, device="cuda")
u = torch.zeros((1, 64), dtype=torch.int64, device="cuda")
if SIX:                                              # a loaf in its 6 x 6 box
    for c, rows in zip(range(21, 25), ((1,), (0, 2), (0, 3), (1, 2))):
        w[0, c] = sum(1 << (31 + r) for r in rows)
    for c in range(20, 26):
        u[0, c] = 0x3F << 30
else:
    w[0, 10] = w[0, 11] = 3 << 40                   # a block ...
    for c in (9, 10, 11, 12):
        u[0, c] = 15 << 39
u &= ~w                                              # ... and its empty ring
VARS = [int(a) for a in sys.argv[1:] if a.isdigit()] or list(range(8))
CAPS = [tuple(int(c) for c in a[4:].split("/")) for a in sys.argv[1:] if a.startswith("cap=")]  # cap=lo/hi
outs = {k: torch.empty_like(x) for k in ["step", "ship"] + [f"v{v}" for v in VARS] + [f"pair{c}" for c in CAPS]}
firsts = {}
kern = {
    "step": lambda: hip.step(x, out=outs["step"], generations=g),
    "ship": lambda: firsts.__setitem__("ship", hip.step_contains(x, w, u, g, final=outs["ship"])[0]),
}
for v in VARS:
    kern[f"v{v}"] = (lambda vv: lambda: firsts.__setitem__(
        f"v{vv}", tune_hip.step_contains(x, w, u, g, vv, final=outs[f"v{vv}"])))(v)
for cap in CAPS:
    kern[f"pair{cap}"] = (lambda cc: lambda: firsts.__setitem__(
        f"pair{cc}", tune_hip.step_contains_pair(x, w, u, g, cc[0], cc[1], final=outs[f"pair{cc}"])))(cap)
t0 = time.time()
while time.time() - t0 < 2.0:
    for f in kern.values():
        f()
    torch.cuda.synchronize()
ms = {k: [] for k in kern}
REPS = 30
for rep in range(REPS):
    order = list(kern.items())
    for k, f in order[rep % len(order):] + order[:rep % len(order)]:  # rotate who runs first
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        e1.synchronize()
        ms[k].append(e0.elapsed_time(e1))
hits = int((firsts["ship"] > 0).sum().item())
for k in kern:
    same = None if k == "step" else bool(torch.equal(firsts[k], firsts["ship"]) and torch.equal(outs[k], outs["ship"]))
    print(json.dumps({"kernel": k, "ms_median": statistics.median(ms[k]), "ms_min": min(ms[k]),
                      "over_step": statistics.median(ms[k]) / statistics.median(ms["step"]),
                      "equal_to_shipped": same, "universes_with_hit": hits,
                      "target": "loaf + 6x6 box (6 rows)" if SIX else "2x2 block + ring (4 rows)"}), flush=True)
