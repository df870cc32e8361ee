#!/usr/bin/env python3
"""Launch-order A/B of the one-generation search filter with final states
(Step + Contains, LifeTarget.hpp:44-51), run as a loop would run it: each
call filters the states the previous call wrote (ping-pong between two
arrays).  "round2" = the tuning build's launch of the same kernel in one
order with nontemporal stores (8 universes per wave, every block slot, as
shipped before); "shipped" = lifeapi_step_contains_batch_dev, which
alternates the order and stores the last min(256 MiB, half the batch) of
final states plain.  Runs of 40 launches between one pair of events, the two
interleaved, 6 runs each; both must give the same first-hit generations.
usage: python tools/ab/filter_order_ab.py [universes ...]"""
import json
import os
import statistics
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip  # noqa: E402

RUN = 40
# the bench's search-loop target: a 2 x 2 block with its empty ring
with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
    gold = json.load(f)["digests"]["config3_contains"]
tw, tu = (torch.from_numpy(np.array([[int(v, 16) for v in gold[k]]], dtype=np.uint64).view(np.int64)).cuda()
          for k in ("wanted", "unwanted"))

modes = {
    "round2": lambda s, d: tune_hip.step_contains_nat(s, tw, tu, 1, 8, 0, final=d),
    "shipped": lambda s, d: hip.step_contains(s, tw, tu, 1, final=d)[0],
}


def run(bufs, launch):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(RUN):
        launch(bufs[i & 1], bufs[(i + 1) & 1])
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / RUN


for n in [int(a) for a in sys.argv[1:]] or [1 << 19, 1 << 20, 1 << 21, 1 << 22]:
    a = hip.fill_random(n, seed=3)
    b, c = torch.empty_like(a), torch.empty_like(a)
    f0 = modes["round2"](a, b)
    f1 = modes["shipped"](a, c)
    assert torch.equal(f0, f1) and torch.equal(b, c)
    ms = {k: [] for k in modes}
    bufs = [a, b]
    for k in modes:
        run(bufs, modes[k])
    for rep in range(6):
        for k in (list(modes) if rep % 2 == 0 else list(modes)[::-1]):
            ms[k].append(run(bufs, modes[k]))
    for k in modes:
        med = statistics.median(ms[k])
        print(json.dumps({"universes": n, "launch": k, "ms_per_launch_median": med, "ms_all": ms[k],
                          "GBps": n * 1028 / (med * 1e-3) / 1e9}), flush=True)
    del a, b, c
    torch.cuda.empty_cache()
