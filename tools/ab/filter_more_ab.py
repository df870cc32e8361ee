#!/usr/bin/env python3
"""Same-process A/B of the 1-generation search filter (first hits only,
516 B per universe): the shipped launch against the tuning build's
k_step_contains with 8 / 12 / 16 universes per wave and the XCD-chunked
block mapping, at 1M and 4M universes; 20 launches back to back per timing,
median over rounds; first hits checked equal to the shipped launch's.

Usage: python tools/ab/filter_more_ab.py [--rounds R]"""
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
sys.path.insert(0, os.path.join(ROOT, "tools"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip as tune  # noqa: E402
from filter_rule_ab import arg, timed  # noqa: E402


def main():
    rounds, k = arg("--rounds", 5), 20
    for n in (1 << 20, 1 << 22):
        x = hip.fill_random(n, seed=7)
        w = x[:1].clone()
        ref = hip.step_contains(x, w, w, 1)[0]
        cases = {"shipped": lambda: hip.step_contains(x, w, w, 1)[0]}
        for code, name in ((8, "upw8"), (1024 + 8, "upw8 xcd_chunk"), (12, "upw12"), (16, "upw16"),
                           (1024 + 16, "upw16 xcd_chunk")):
            cases[name] = lambda code=code: tune.step_contains_nat(x, w, w, 1, code, 0)
        res = {c: [] for c in cases}
        for _ in range(rounds):
            for c, fn in cases.items():
                res[c].append(timed(fn, k))
        for c, fn in cases.items():
            ok = bool(torch.equal(fn(), ref))
            ms = statistics.median(res[c])
            print(json.dumps({"universes": n, "variant": c, "ms": ms, "hbm_frac": n * 516 / ms / 1e6 / 8000.0,
                              "ms_rounds": res[c], "equal_to_shipped": ok}), flush=True)
        del x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
