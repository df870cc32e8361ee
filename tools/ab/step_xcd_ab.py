#!/usr/bin/env python3
"""Same-process A/B of the streaming step (1 generation, ping-pong) with the
plain block mapping against the XCD-chunked one (kXcdChunk: XCD k streams
one contiguous eighth of the batch), one fixed order, nontemporal stores,
4 universes per wave, uncapped or at most 7 blocks per CU; the shipped launch
(batch-keyed order, plain-stored tail, caps) alongside.  Outputs checked
against the shipped step.  One JSON line per (size, variant): median over
rounds of 10 back-to-back launches.

Usage: python tools/ab/step_xcd_ab.py [--rounds R]"""
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
    rounds, k = arg("--rounds", 5), 10
    for n in (1 << 24, 1 << 23, 1 << 22, 1 << 20):
        bufs = [hip.fill_random(n, seed=2), torch.empty(n * 64, dtype=torch.int64, device="cuda").view(n, 64)]
        ref = hip.step(bufs[0], generations=1)
        cases = {"shipped": lambda s, d: hip.step(s, out=d, generations=1)}
        for res in (0, 7):
            for chunk in (False, True):
                cases[f"fixed nt resident={res} {'xcd_chunk' if chunk else 'plain'}"] = (
                    lambda s, d, res=res, chunk=chunk: tune.step_order(s, d, 1, resident=res, xcd_chunk=chunk))
        out = {c: [] for c in cases}
        for _ in range(rounds):
            for c, fn in cases.items():
                fn(bufs[0], bufs[1])
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for i in range(k):
                    fn(bufs[i & 1], bufs[1 - (i & 1)])
                b.record()
                b.synchronize()
                out[c].append(a.elapsed_time(b) / k)
        x = hip.fill_random(n, seed=2)
        for c, fn in cases.items():
            y = torch.empty_like(x)
            fn(x, y)
            torch.cuda.synchronize()
            ms = statistics.median(out[c])
            print(json.dumps({"universes": n, "variant": c, "ms": ms, "TBps": n * 1024 / ms / 1e9,
                              "hbm_frac": n * 1024 / ms / 1e9 / 8.0, "ms_rounds": out[c],
                              "equal_to_shipped": bool(torch.equal(y, ref))}), flush=True)
        del bufs, ref, x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
