#!/usr/bin/env python3
"""Launch-order A/B of the in-place LifeStable passes (LifeStable.hpp:526-729;
stable_kernels.hpp), as a search runs them: the same pass over the same batch
call after call.  "fixed" = the tuning build's launch in one order (with the
shipped occupancy: at most 4 blocks resident per CU, Propagate uncapped),
"alternate" = the same with the order reversed on every other launch,
"shipped" = lifeapi_stable_pass_batch_dev.  Random planes (the rows-bench
input); runs of 20 launches between one pair of events, modes interleaved,
5 runs each; all modes must leave the same planes and flags.
usage: python tools/ab/stable_order_ab.py [lifestables ...]"""
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

RUN = 20
PASSES = {0: "sync", 3: "step", 4: "propagate"}

for n in [int(a) for a in sys.argv[1:]] or [1 << 16, 1 << 18, 1 << 20]:
    pristine = hip.fill_random(n * 10, seed=21).reshape(n, 640)
    work = pristine.clone()
    for p, name in PASSES.items():
        cap = 0 if p == 4 else -4
        modes = {"fixed": lambda i, p=p, cap=cap: tune_hip.stable_pass(work, p, cap),
                 "alternate": lambda i, p=p, cap=cap: tune_hip.stable_pass(work, p, cap, reverse=bool(i & 1)),
                 "shipped": lambda i, p=p: hip.stable_pass(work, p)}
        outs = {}
        for k, f in modes.items():
            work.copy_(pristine)
            fl = f(0)
            fl2 = f(1)
            outs[k] = (work.clone(), fl.clone(), fl2.clone())
        for k in modes:
            assert all(torch.equal(a, b) for a, b in zip(outs[k], outs["fixed"])), (name, k)
        del outs

        def run(f):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(RUN):
                f(i)
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / RUN

        work.copy_(pristine)
        ms = {k: [] for k in modes}
        for k in modes:
            run(modes[k])
        for rep in range(5):
            for k in (list(modes) if rep % 2 == 0 else list(modes)[::-1]):
                ms[k].append(run(modes[k]))
        for k in modes:
            med = statistics.median(ms[k])
            print(json.dumps({"lifestables": n, "pass": name, "launch": k, "ms_per_launch_median": med,
                              "ms_all": ms[k], "GBps": n * 10241 / (med * 1e-3) / 1e9}), flush=True)
    del pristine, work
    torch.cuda.empty_cache()
