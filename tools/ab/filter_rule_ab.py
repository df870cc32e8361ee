#!/usr/bin/env python3
"""Same-process A/B of the natural-layout generation (gens <= 2) on 1M
universes: RULE 3 (7-LUT tail, shipped) against RULE 14 (the 6-LUT tail,
device.hpp life_tail6), each with the DPP or the LDS neighbour exchange, in
  - the 1-generation search filter, first hits only (k_step_contains, 516 B
    per universe) and with final states (1028 B);
  - the streaming step (k_step, 1024 B), one fixed order, nt loads/stores;
and the filter with the prefetching loop (k_step_contains<..., PF>: each wave
loads its next group before working on the current one) on capped grids.
Every variant's output is checked equal to the shipped kernel's.  Rounds
interleave the variants; a timing is K back-to-back launches between two
events (per launch: / K); one JSON line per variant, median over rounds.

Usage: python tools/ab/filter_rule_ab.py [--n N] [--rounds R] [--k K]"""
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
import tune_hip as tune  # noqa: E402

PEAK = 8000.0


def timed(fn, k):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(k):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / k


def arg(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    n, rounds, k = arg("--n", 1 << 20), arg("--rounds", 7), arg("--k", 20)
    x = hip.fill_random(n, seed=7)
    w = x[:1].clone()
    fin = torch.empty_like(x)
    y = torch.empty_like(x)
    ref_first = hip.step_contains(x, w, w, 1)[0]
    ref_next = hip.step(x, generations=1)

    cases = {}  # name -> (bytes per object, fn, check)
    cases["filter shipped"] = (516, lambda: hip.step_contains(x, w, w, 1), None)
    names = {8: "dpp rule3", 40: "lds rule3", 72: "dpp rule14", 104: "lds rule14",
             4: "dpp rule3 upw4", 36: "lds rule3 upw4", 68: "dpp rule14 upw4", 100: "lds rule14 upw4"}
    for code, nm in names.items():
        cases[f"filter {nm}"] = (516, lambda code=code: tune.step_contains_nat(x, w, w, 1, code, 0), None)
    for code, nm in ((136, "dpp rule3 prefetch"), (200, "dpp rule14 prefetch"), (132, "dpp rule3 upw4 prefetch")):
        for cap in (4, 6, 8):
            cases[f"filter {nm} grid={cap}/CU"] = (
                516, lambda code=code, cap=cap: tune.step_contains_nat(x, w, w, 1, code, -cap), None)
    for cap in (4, 8):
        cases[f"filter+final dpp rule3 prefetch grid={cap}/CU"] = (
            1028, lambda cap=cap: tune.step_contains_nat(x, w, w, 1, 136, -cap, final=fin),
            lambda: torch.equal(fin, ref_next))
    for code in (8, 40, 72, 104):
        cases[f"filter+final {names[code]}"] = (
            1028, lambda code=code: tune.step_contains_nat(x, w, w, 1, code, 0, final=fin),
            lambda: torch.equal(fin, ref_next))
    for rule in (3, 14):
        for xchg, xn in ((tune.XCHG_DPP, "dpp"), (tune.XCHG_LDS, "lds")):
            cfg = tune.LaunchCfg(xchg=xchg, universes_per_wave=4, blocks_per_cu=0, nontemporal=1, rule=rule)
            cases[f"step {xn} rule{rule}"] = (
                1024, lambda cfg=cfg: tune.step(x, out=y, generations=1, cfg=cfg),
                lambda: torch.equal(y, ref_next))

    res = {c: [] for c in cases}
    for _ in range(rounds):
        for c, (_, fn, _) in cases.items():
            res[c].append(timed(fn, k))
    for c, (nb, fn, check) in cases.items():
        if check is None:
            out = fn()
            ok = torch.equal(out[0] if isinstance(out, tuple) else out, ref_first)
        else:
            fn()
            torch.cuda.synchronize()
            ok = bool(check())
        ms = statistics.median(res[c])
        print(json.dumps({"variant": c, "objects": n, "bytes_per_object": nb, "ms": ms,
                          "GBps": n * nb / ms / 1e6, "hbm_frac": n * nb / ms / 1e6 / PEAK,
                          "ms_rounds": res[c], "equal_to_shipped": ok}), flush=True)


if __name__ == "__main__":
    main()
