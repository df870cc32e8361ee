#!/usr/bin/env python3
"""Same-process A/B of the other multi-plane kernels with the plain block
mapping against the XCD-chunked one (CHUNK = true: XCD k streams one
contiguous eighth of the batch), each at the product's launch shape:
NeighbourCount / InteractionCounts(AndNext) (k_counts), LifeWeld::Step one
generation in place (k_weld, 7 blocks per CU), the config-5 refined step
(k_refined) and Vulnerable (k_stable_vulnerable, 4 blocks per CU), on 1M
objects (config 5: 256K, its BASELINE size, and 1M).  Outputs checked equal
between the two mappings.  One JSON line per variant: median over rounds of
10 back-to-back launches.

Usage: python tools/ab/stencil_xcd_ab.py [--rounds R]"""
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
from rows_bench import stable_inputs  # noqa: E402


def arg(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    rounds, k = arg("--rounds", 5), 10
    n = 1 << 20
    x = hip.fill_random(n, seed=7)
    welds = torch.cat([hip.fill_random(n, seed=s).view(n, 1, 64) for s in (11, 12, 13, 14)], 1).reshape(n, 256)
    welds[:, 64:] &= hip.fill_random(3 * n, seed=15).view(n, 192)
    st = stable_inputs(n)
    cases = {}
    for kind, name, planes, nb in ((0, "NeighbourCount", 4, 2560), (1, "InteractionCounts", 3, 2048),
                                   (2, "InteractionCountsAndNext", 4, 2560)):
        out = {c: torch.empty((n, planes * 64), dtype=torch.int64, device="cuda") for c in (False, True)}
        for c in (False, True):
            cases[f"{name} {'xcd_chunk' if c else 'plain'}"] = (
                n, nb, lambda kind=kind, c=c, o=out[c]: tune.stencil(kind + (8 if c else 0), x, o, n, 0), out[c])
    wk = {c: welds.clone() for c in (False, True)}
    for c in (False, True):
        cases[f"LifeWeld::Step 1 gen {'xcd_chunk' if c else 'plain'}"] = (
            n, 2560, lambda c=c: tune.stencil(3 + (8 if c else 0), wk[c], None, n, 7), None)
    for nr in (1 << 18, 1 << 20):
        planes = hip.fill_random(11 * nr, seed=21).view(nr, 11 * 64)
        out = {c: torch.empty((nr, 3 * 64), dtype=torch.int64, device="cuda") for c in (False, True)}
        for c in (False, True):
            cases[f"refined {nr} {'xcd_chunk' if c else 'plain'}"] = (
                nr, 7168, lambda c=c, p=planes, o=out[c], nr=nr: tune.stencil(4 + (8 if c else 0), p, o, nr, 0), out[c])
    vout = {c: torch.empty((n, 64), dtype=torch.int64, device="cuda") for c in (False, True)}
    for c in (False, True):
        cases[f"Vulnerable {'xcd_chunk' if c else 'plain'}"] = (
            n, 5632, lambda c=c: tune.stable_vulnerable(st, -4 + (1000 if c else 0), out=vout[c]), vout[c])
    res = {c: [] for c in cases}
    for _ in range(rounds):
        for c, (m, nb, fn, _) in cases.items():
            fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(k):
                fn()
            b.record()
            b.synchronize()
            res[c].append(a.elapsed_time(b) / k)
    names = list(cases)
    for c in names:
        m, nb, fn, out = cases[c]
        ok = None
        if out is not None and c.endswith("xcd_chunk"):
            ok = bool(torch.equal(out, cases[c.replace("xcd_chunk", "plain")][3]))
        ms = statistics.median(res[c])
        print(json.dumps({"variant": c, "objects": m, "bytes_per_object": nb, "ms": ms,
                          "hbm_frac": m * nb / ms / 1e6 / 8000.0, "ms_rounds": res[c],
                          "equal_to_plain": ok}), flush=True)


if __name__ == "__main__":
    main()
