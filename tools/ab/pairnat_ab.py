#!/usr/bin/env python3
"""Same-process A/B of the streaming step's layout (1 generation, ping-pong,
50 launches back to back per timing, rounds interleaved): the shipped
one-column-per-lane kernel (k_step, DPP exchange) against the column-pair
form (k_step_pairnat: two adjacent columns per lane, 16-byte accesses, the
outer columns by ds_bpermute), both under the product's policy (the order
alternating per launch, the last min(256 MiB, half) stored plain) and in one
fixed order with every store nontemporal; 4 and 8 universes per wave; 1M
and 2M universes.  Outputs checked against the shipped step.

Usage: python tools/ab/pairnat_ab.py [--rounds R]"""
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


def arg(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    rounds, k = arg("--rounds", 5), 50
    for n in (1 << 20, 1 << 21):
        a, b = hip.fill_random(n, seed=2), torch.empty((n, 64), dtype=torch.int64, device="cuda")
        ref = hip.step(a, generations=1)

        def policy(upw):
            flip = [False]

            def fn(s, d):
                rev = flip[0]
                flip[0] = not flip[0]
                tune.step_order(s, d, 1, reverse=rev, nts=True, resident=0, upw=upw, plain_bytes=min(256 << 20, n * 256))
            return fn

        cases = {"shipped": lambda s, d: hip.step(s, out=d, generations=1),
                 "1 col/lane, policy (tune)": policy(4),
                 "pair, policy, 4/wave": policy(36),
                 "pair, policy, 8/wave": policy(40),
                 "1 col/lane, fixed nt": lambda s, d: tune.step_order(s, d, 1, nts=True, resident=0, upw=4),
                 "pair, fixed nt, 4/wave": lambda s, d: tune.step_order(s, d, 1, nts=True, resident=0, upw=36),
                 "pair, fixed nt, 8/wave": lambda s, d: tune.step_order(s, d, 1, nts=True, resident=0, upw=40)}
        res = {c: [] for c in cases}
        for _ in range(rounds):
            for c, fn in cases.items():
                for i in range(4):
                    fn(a if i % 2 == 0 else b, b if i % 2 == 0 else a)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(k):
                    fn(a if i % 2 == 0 else b, b if i % 2 == 0 else a)
                e1.record()
                e1.synchronize()
                res[c].append(e0.elapsed_time(e1) / k)
        x = hip.fill_random(n, seed=2)
        for c, fn in cases.items():
            y = torch.empty_like(x)
            fn(x, y)
            torch.cuda.synchronize()
            ms = statistics.median(res[c])
            print(json.dumps({"universes": n, "variant": c, "ms": ms, "hbm_frac": n * 1024 / ms / 1e9 / 8,
                              "ms_rounds": res[c], "equal": bool(torch.equal(y, ref))}), flush=True)
        del a, b, x, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
