#!/usr/bin/env python3
"""Launch-order A/B of LifeWeld::Step (LifeWeld.hpp:169-186), one generation
per launch in place, as a loop steps a batch of welds: "round2" = the tuning
build's launch in one order, nontemporal throughout (as shipped before);
"alt-pK" = the order alternated between launches and the last K welds of
each launch loaded and stored plain; "shipped" = lifeapi_weld_step_batch_dev.
Runs of 40 launches between one pair of events, modes interleaved, 6 runs
each; every mode must step the same welds to the same states.
usage: python tools/ab/weld_order_ab.py [welds ...]"""
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

RUN = 40


def make(n):
    w = torch.cat([hip.fill_random(n, seed=s).view(n, 1, 64) for s in (11, 12, 13, 14)], 1).reshape(n, 256)
    w[:, 64:] &= hip.fill_random(3 * n, seed=15).view(n, 192)
    return w


for n in [int(a) for a in sys.argv[1:]] or [1 << 18, 1 << 19, 1 << 20, 1 << 21]:
    welds = make(n)
    modes = {"round2": lambda i: tune_hip.stencil(3, welds, None, n, 0),
             "shipped": lambda i: hip.weld_step(welds, 1)}
    for k in (0, 1 << 16, 1 << 17, 1 << 18, n // 2):
        modes[f"alt-p{k}"] = lambda i, k=k: tune_hip.weld_order(welds, reverse=bool(i & 1), plain_welds=k)
    # parity: every mode, the same two generations from the same start
    ref = welds.clone()
    hip.weld_step(ref, 2)
    for name, f in modes.items():
        w0 = make(n)
        welds.copy_(w0)
        f(0)
        f(1)
        assert torch.equal(welds, ref), name
    ms = {k: [] for k in modes}

    def run(f):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(RUN):
            f(i)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / RUN

    for k in modes:
        run(modes[k])
    for rep in range(6):
        for k in (list(modes) if rep % 2 == 0 else list(modes)[::-1]):
            ms[k].append(run(modes[k]))
    for k in modes:
        med = statistics.median(ms[k])
        print(json.dumps({"welds": n, "launch": k, "ms_per_launch_median": med, "ms_all": ms[k],
                          "GBps": n * 2560 / (med * 1e-3) / 1e9}), flush=True)
    del welds, ref
    torch.cuda.empty_cache()
