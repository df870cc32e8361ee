#!/usr/bin/env python3
"""Occupancy A/B of the streaming stencils (stencil_kernels.hpp): k_counts
(3 modes), k_weld (1 generation) and k_refined (config 5), each with as many
blocks resident per CU as fit (as shipped) and with at most k (unused
dynamic LDS), through the tuning build; launches interleaved, 30 each after
warm-up, outputs checked equal to the shipped entry points'.
usage: python tools/ab/stencil_occupancy_ab.py [objects]"""
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

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
RES = [int(c) for c in os.environ.get("CAPS", "0,4,5,6,8").split(",")]
x = hip.fill_random(N, seed=11)
cases = {  # name: (kind, input, output, bytes per object, shipped result)
    "NeighbourCount": (0, x, torch.empty((N, 4 * 64), dtype=torch.int64, device="cuda"), 512 * 5,
                       hip.neighbour_count(x)),
    "InteractionCounts": (1, x, torch.empty((N, 3 * 64), dtype=torch.int64, device="cuda"), 512 * 4,
                          hip.interaction_counts(x, with_next=False)),
    "InteractionCountsAndNext": (2, x, torch.empty((N, 4 * 64), dtype=torch.int64, device="cuda"), 512 * 5,
                                 hip.interaction_counts(x, with_next=True)),
}
p11 = hip.fill_random(N * 11, seed=12).reshape(N, 11 * 64)
cases["refined (config 5)"] = (4, p11, torch.empty((N, 3 * 64), dtype=torch.int64, device="cuda"), 512 * 14,
                               hip.refined_step(p11))
for name, (kind, inp, out, nbytes, ref) in cases.items():
    for r in RES:
        tune_hip.stencil(kind, inp, out, N, r)
        torch.cuda.synchronize()
        assert torch.equal(out.view(ref.shape), ref), (name, r)
welds = hip.fill_random(N * 4, seed=13).reshape(N, 256)
ms = {(name, r): [] for name in list(cases) + ["LifeWeld::Step (1 gen)"] for r in RES}
for rep in range(40):
    for name, (kind, inp, out, nbytes, ref) in cases.items():
        for r in RES[rep % len(RES):] + RES[:rep % len(RES)]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            tune_hip.stencil(kind, inp, out, N, r)
            e1.record()
            e1.synchronize()
            if rep >= 10:
                ms[(name, r)].append(e0.elapsed_time(e1))
    for r in RES[rep % len(RES):] + RES[:rep % len(RES)]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        tune_hip.stencil(3, welds, None, N, r)
        e1.record()
        e1.synchronize()
        if rep >= 10:
            ms[("LifeWeld::Step (1 gen)", r)].append(e0.elapsed_time(e1))
nb = {name: c[3] for name, c in cases.items()}
nb["LifeWeld::Step (1 gen)"] = 2560  # LifeWeld.hpp: 4 planes in, state written: DESIGN.md 5.4
for (name, r), v in ms.items():
    med = statistics.median(v)
    print(json.dumps({"kernel": name, "objects": N, "resident_blocks": r, "ms_median": med,
                      "GBps": N * nb[name] / (med * 1e-3) / 1e9}), flush=True)
