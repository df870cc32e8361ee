#!/usr/bin/env python3
"""Launch-configuration sweep for the step kernel (measurement tool).

Times every lifeapi_launch_cfg variant on the config-2 (1M x 1 gen) and
config-3 (64K x 1024 gens) workloads in ONE process, interleaving rounds so
that clock drift hits all variants alike (cdna_hip_programming.md rule 24),
and checks each variant's output against the default variant bit-for-bit.
Prints one JSON line per (workload, variant) with best/median kernel time.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import lifeapi_amd.hip as hip  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tune"))
import tune_hip  # noqa: E402  (tools/tune/liblifeapi_tune.so: explicit launch configurations)


def timeit(fn, reps):
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        out.append(e0.elapsed_time(e1))
    return out


def tune_c5(args):
    """Config 5 (refined ternary step): prefetch x grid cap x occupancy bound."""
    raise SystemExit("the config-5 launch variants were measured in round 1 (profiles/r01/tune_c5.jsonl); "
                     "their tuning form is no longer built -- the shipped k_refined<1, 0> is fixed")
    import ctypes
    n = 1 << 18
    planes = hip.fill_random(n * 11, seed=6).reshape(n, 11 * 64)
    ref = hip.refined_step(planes)
    out = torch.empty_like(ref)
    s = torch.cuda.current_stream().cuda_stream
    cfgs = list(itertools.product([1, 2], [4, 6, 8, 12, 0], [0, 4, 6]))
    ms = {c: [] for c in cfgs}
    ok = {}
    for r in range(args.rounds):
        for c in cfgs:
            cfg = tune_hip.LaunchCfg(0, c[0], c[1], 1, c[2])
            run = lambda: hip._check(hip.lib.lifeapi_refined_step_batch_dev_cfg(  # noqa: E731
                planes.data_ptr(), out.data_ptr(), n, s, ctypes.byref(cfg)))
            ms[c] += timeit(run, args.reps)
            if r == 0:
                torch.cuda.synchronize()
                ok[c] = bool(torch.equal(out, ref))
    for c in cfgs:
        t = sorted(ms[c])
        med = t[len(t) // 2]
        print(json.dumps({"workload": "c5", "n": n, "prefetch": c[0] - 1, "blocks_per_cu": c[1],
                          "occ": c[2], "ms_best": t[0], "ms_median": med,
                          "GBps_median": n * 7168 / (med / 1e3) / 1e9, "bit_exact": ok[c]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["c2", "c3", "c3net", "c3mix", "c3pipe", "c3asm", "c5", "gsweep", "both", "all"], default="both")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()

    if args.workload in ("c5", "all"):
        tune_c5(args)
        if args.workload == "c5":
            return
    work = []
    if args.workload in ("c2", "both", "all"):
        n, g = 1 << 20, 1
        xs = [0, 2]
        us = [2, 4, 8]
        bpcs = [0]
        nts = [1]
        rules = [0, 2]
        work.append(("c2", n, g, list(itertools.product(xs, us, bpcs, nts, rules))))
    if args.workload == "gsweep":  # where the split layouts start to pay
        cfgs = [(0, 4, 0, 1, 2), (0, 4, 0, 1, 3), (0, 1, 0, 0, 3), (1, 1, 0, 0, 6), (1, 2, 0, 0, 6),
                (1, 2, 0, 1, 6)]
        for g in (1, 2, 4, 8, 16, 32):
            work.append((f"g{g}", 1 << 18, g, cfgs))
    if args.workload in ("c3", "both", "all"):
        n, g = 1 << 16, 1024
        work.append(("c3", n, g, [(1, 1, 0, 0, 6), (1, 2, 0, 0, 6), (1, 1, 0, 0, 7), (1, 1, 0, 0, 8),
                                  (0, 1, 0, 0, 8), (1, 1, 0, 0, 9), (8, 1, 0, 0, 8), (8, 1, 0, 1, 8)]))
    if args.workload == "c3asm":  # the hand-allocated rule-11 loop against the compiled one
        n, g = 1 << 16, 1024
        work.append(("c3", n, g, [(1, 1, 0, 0, 11), (8, 1, 0, 0, 11), (25, 1, 0, 0, 11), (26, 1, 0, 0, 11),
                                  (27, 1, 0, 0, 11), (8, 2, 0, 0, 11)]))
        for gg in (4, 16, 64):
            work.append((f"g{gg}", 1 << 18, gg, [(1, 1, 0, 1, 11), (8, 1, 0, 1, 11)]))
    if args.workload == "c3pipe":  # software-pipelined LDS loop against the plain one
        n, g = 1 << 16, 1024
        work.append(("c3", n, g, [(1, 1, 0, 0, 11), (9, 1, 0, 0, 11), (9, 2, 0, 0, 11), (1, 1, 0, 0, 6),
                                  (9, 1, 0, 0, 6), (1, 1, 0, 0, 12), (9, 1, 0, 0, 12)]))
        for gg in (4, 16):
            work.append((f"g{gg}", 1 << 18, gg, [(1, 1, 0, 1, 11), (9, 1, 0, 1, 11)]))
    if args.workload == "c3mix":  # rule 11 with d registers exchanged by DPP
        n, g = 1 << 16, 1024
        work.append(("c3", n, g, [(1, 1, 0, 0, 11)] + [(16 + d, u, 0, 0, 11) for d in (1, 2, 3, 4) for u in (1, 2)]
                     + [(1, 1, 0, 0, 12), (18, 1, 0, 0, 12), (20, 1, 0, 0, 12)]))
    if args.workload == "c3net":  # 6-LUT tail (rules 10-13) against the 7-LUT one
        n, g = 1 << 16, 1024
        work.append(("c3", n, g, [(1, 1, 0, 0, 6), (1, 1, 0, 0, 11), (1, 2, 0, 0, 6), (1, 2, 0, 0, 11),
                                  (1, 1, 0, 0, 7), (1, 1, 0, 0, 12), (1, 1, 0, 0, 10),
                                  (1, 1, 0, 0, 8), (1, 1, 0, 0, 13), (0, 1, 0, 0, 8), (0, 1, 0, 0, 13)]))
        for gg in (4, 16, 64):
            work.append((f"g{gg}", 1 << 18, gg, [(1, 1, 0, 1, 6), (1, 1, 0, 1, 11), (1, 1, 0, 0, 6),
                                                  (1, 1, 0, 0, 11)]))

    for name, n, g, cfgs in work:
        a = hip.fill_random(n, seed=2)
        ref = hip.step(a, generations=g)
        b = torch.empty_like(a)
        ms = {c: [] for c in cfgs}
        ok = {}
        if name == "c2":  # stream-copy ceiling of the same bytes, for context
            copy_ms = []
        for r in range(args.rounds):
            for c in cfgs:
                cfg = tune_hip.LaunchCfg(*c)
                ms[c] += timeit(lambda: tune_hip.step(a, out=b, generations=g, cfg=cfg), args.reps)
                if r == 0:
                    torch.cuda.synchronize()
                    ok[c] = bool(torch.equal(b, ref))
            if name == "c2":
                copy_ms += timeit(lambda: b.copy_(a), args.reps)
        for c in cfgs:
            t = sorted(ms[c])
            best, med = t[0], t[len(t) // 2]
            rec = {"workload": name, "n": n, "gens": g, "xchg": c[0], "universes_per_wave": c[1],
                   "blocks_per_cu": c[2], "nontemporal": c[3], "rule": c[4], "ms_best": best,
                   "ms_median": med, "gen_per_s_median": n * g / (med / 1e3), "bit_exact": ok[c]}
            if name == "c2":
                rec["GBps_median"] = n * 1024 / (med / 1e3) / 1e9
            print(json.dumps(rec), flush=True)
        if name == "c2":
            t = sorted(copy_ms)
            print(json.dumps({"workload": "c2-torch-copy", "ms_best": t[0], "ms_median": t[len(t) // 2],
                              "GBps_median": n * 1024 / (t[len(t) // 2] / 1e3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
