#!/usr/bin/env python3
"""Is the batch-keyed order + plain-stored tail still worth it at 1M
universes?  Same process, ping-pong as the bench (K launches between two
events), rounds interleaved: the shipped launch (hip.step: reversed order on
a batch the last launch wrote, the last min(256 MiB, half) stored plain) and
through the tuning build the same kernel code in one fixed order with every
store nontemporal (the bench's cache-neutral form), uncapped and at 7 blocks
per CU, and the alternating policy itself; at 1M and 2M universes.

Usage: python tools/ab/order_policy_ab.py [--rounds R]"""
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
    rounds, k = arg("--rounds", 7), 50
    for n in (1 << 20, 1 << 21):
        a, b = hip.fill_random(n, seed=2), torch.empty((n, 64), dtype=torch.int64, device="cuda")
        flip = [False]

        def alt(s, d, n=n):
            rev = flip[0]
            flip[0] = not flip[0]
            tune.step_order(s, d, 1, reverse=rev, nts=True, resident=0, plain_bytes=min(256 << 20, n * 256))

        cases = {
            "shipped": lambda s, d: hip.step(s, out=d, generations=1),
            "fixed nt uncapped (neutral)": lambda s, d: tune.step_order(s, d, 1, nts=True, resident=0, plain_bytes=0),
            "fixed nt 7 blocks": lambda s, d: tune.step_order(s, d, 1, nts=True, resident=7, plain_bytes=0),
            "alternating + plain tail (tune)": alt,
        }
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
        for c in cases:
            ms = statistics.median(res[c])
            print(json.dumps({"universes": n, "variant": c, "ms": ms, "TBps": n * 1024 / ms / 1e9,
                              "hbm_frac": n * 1024 / ms / 1e9 / 8, "ms_rounds": res[c]}), flush=True)
        del a, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
