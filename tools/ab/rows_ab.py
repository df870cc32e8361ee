#!/usr/bin/env python3
"""Same-process A/B of the read-dominated SURVEY 8(f) rows on 1M objects
(VERDICT r02 item 4): GetPop, Contains, the 1-generation search filter
(first hits only), the seeded fill, and LifeStable Propagate, each shipped
form against alternatives from the tuning build (tools/tune): 16-byte loads
(k_pop16 / k_contains16) or stores (k_fill16), universes per wave, and exact
occupancy caps (host.hip occupancy_lds).  Every variant's output is checked
equal to the shipped one's.  Rounds interleave the variants; one JSON line per
variant with the median over rounds of each round's median launch time.

Usage: python tools/ab/rows_ab.py [--n N] [--rounds R]"""
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

sys.path.insert(0, os.path.join(ROOT, "tools"))
from rows_bench import stable_inputs  # noqa: E402

PEAK = 8000.0


def timed(fn, reps=9):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return statistics.median(ms)


def main():
    n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 1 << 20
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 3
    x = hip.fill_random(n, seed=7)
    w = x[:1].clone()
    pop_out = torch.empty(n, dtype=torch.int32, device="cuda")
    con_out = torch.empty(n, dtype=torch.uint8, device="cuda")
    fill_out = torch.empty_like(x)
    ref_pop, ref_con = hip.pop(x), hip.contains(x, w, w)
    ref_filter = hip.step_contains(x, w, w, 1)[0]
    ref_fill = hip.fill_random(n, seed=9)

    cases = {}  # name -> (bytes per object, fn, check)
    cases["pop shipped"] = (516, lambda: hip.pop(x), lambda: True)
    for upw in (4, 8):
        for cap in (32, 0):
            cases[f"pop8 upw={upw} cap={cap}"] = (
                516, lambda upw=upw, cap=cap: tune.reduce(0, x, pop_out, upw, cap),
                lambda: torch.equal(pop_out, ref_pop))
    for upw in (4, 8):
        for cap in (32, 0, -6, -7):
            cases[f"pop16 upw={upw} cap={cap}"] = (
                516, lambda upw=upw, cap=cap: tune.reduce(2, x, pop_out, upw, cap),
                lambda: torch.equal(pop_out, ref_pop))
    cases["contains shipped"] = (513, lambda: hip.contains(x, w, w), lambda: True)
    for upw in (4, 8):
        cases[f"contains8 upw={upw} cap=0"] = (
            513, lambda upw=upw: tune.reduce(1, x, con_out, upw, 0, w, w),
            lambda: torch.equal(con_out.to(torch.bool), ref_con.to(torch.bool)))
    for upw in (4, 8):
        for cap in (0, 32, -6, -7):
            cases[f"contains16 upw={upw} cap={cap}"] = (
                513, lambda upw=upw, cap=cap: tune.reduce(3, x, con_out, upw, cap, w, w),
                lambda: torch.equal(con_out.to(torch.bool), ref_con.to(torch.bool)))
    cases["filter shipped (k_step_contains<8>, one-shot)"] = (516, lambda: hip.step_contains(x, w, w, 1),
                                                             lambda: True)
    for upw in (8, 20, 24):
        for res in (0, 6, 7):
            cases[f"filter upw={upw} resident={res}" + (" (16-byte staged)" if upw > 16 else "")] = (
                516, lambda upw=upw, res=res: tune.step_contains_nat(x, w, w, 1, upw, res), None)
    fin = torch.empty_like(x)
    ref_fin = torch.empty_like(x)
    hip.step(x, out=ref_fin, generations=1)
    for upw in (8, 24):
        cases[f"filter+final upw={upw}" + (" (16-byte staged)" if upw > 16 else "")] = (
            1028, lambda upw=upw: tune.step_contains_nat(x, w, w, 1, upw, 0, final=fin),
            lambda: torch.equal(fin, ref_fin))
    cases["fill shipped"] = (512, lambda: hip.fill_random(n, seed=9, out=fill_out), lambda: True)
    for cap in (0, 32):
        cases[f"fill16 cap={cap}"] = (512, lambda cap=cap: tune.fill16(fill_out, 9, blocks_per_cu=cap),
                                      lambda: torch.equal(fill_out, ref_fill))

    st = stable_inputs(n)
    work = st.clone()

    def prop(cap):
        work.copy_(st)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        if cap is None:
            hip.stable_pass(work, "propagate")
        else:
            tune.stable_pass(work, 4, cap)
        b.record()
        b.synchronize()
        return a.elapsed_time(b)

    res = {k: [] for k in cases}
    prop_caps = [None, -6, -7]
    pres = {c: [] for c in prop_caps}
    for _ in range(rounds):
        for k, (_, fn, _) in cases.items():
            res[k].append(timed(fn))
        for c in prop_caps:
            pres[c].append(statistics.median(prop(c) for _ in range(7)))
    for k, (nb, fn, check) in cases.items():
        if check is None:  # the filter: first-hit generations equal the shipped kernel's
            ok = torch.equal(fn(), ref_filter)
        else:
            fn()
            torch.cuda.synchronize()
            ok = bool(check())
        ms = statistics.median(res[k])
        print(json.dumps({"variant": k, "objects": n, "bytes_per_object": nb, "ms": ms,
                          "GBps": n * nb / ms / 1e6, "hbm_frac": n * nb / ms / 1e6 / PEAK,
                          "ms_rounds": res[k], "equal_to_shipped": ok}), flush=True)
    for c in prop_caps:
        ms = statistics.median(pres[c])
        print(json.dumps({"variant": "propagate " + ("shipped (every wave slot)" if c is None else f"cap={c}"),
                          "objects": n, "bytes_per_object": 10241, "ms": ms, "GBps": n * 10241 / ms / 1e6,
                          "hbm_frac": n * 10241 / ms / 1e6 / PEAK, "ms_rounds": pres[c]}), flush=True)


if __name__ == "__main__":
    main()
