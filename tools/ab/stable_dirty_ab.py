#!/usr/bin/env python3
"""Same-process A/B of the LifeStable passes storing only the 128-byte lines
that hold a changed column (shipped) against storing every line (round 3's
k_stable: the tuning build with mode bit 2), each pass's shipped launch shape
(stencils.hip kStablePassResident, XCD-chunked).  Inputs: the rows_bench
still lifes around an unknown window with fresh options (the state a search
propagates from), the next node of such a search (those propagated to their
fixpoint, then one unknown cell decided ON) and random planes.  Each timing runs KS passes back to back
on fresh copies; planes and flags are checked equal between the forms and
to the shipped pass.  One JSON line per (input, pass, form), median over rounds.

Usage: python tools/ab/stable_dirty_ab.py [--n N] [--rounds R]"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip as tune  # noqa: E402
from rows_bench import stable_inputs, stable_next_node  # noqa: E402

PEAK = 8000.0
CAPS = {0: -3, 1: -3, 2: -3, 3: -3, 4: 0, 5: -4}   # stencils.hip kStablePassResident


def arg(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    n, rounds, ks = arg("--n", 1 << 20), arg("--rounds", 5), 4
    still = stable_inputs(n)
    nxt = stable_next_node(still)
    families = {"still_lifes": still, "next_node": nxt,
                "random": hip.fill_random(10 * n, seed=31).view(n, 640)}
    for fam, st in families.items():
        works = [st.clone() for _ in range(ks)]
        for p, name in enumerate(hip.STABLE_PASSES):
            forms = {"dirty_lines": lambda wk, name=name: hip.stable_pass(wk, name),
                     "every_line": lambda wk, p=p: tune.stable_pass(wk, p, CAPS[p], xcd_chunk=True,
                                                                     store_all=True)}
            outs = {}
            for f, fn in forms.items():
                w = st.clone()
                outs[f] = (w, fn(w))
            ok = torch.equal(outs["dirty_lines"][0], outs["every_line"][0]) and \
                torch.equal(outs["dirty_lines"][1], outs["every_line"][1])
            changed_cols = int(((outs["every_line"][0] != st).view(n, 10, 64).any(1)).sum().item())
            del outs
            res = {f: [] for f in forms}
            for _ in range(rounds):
                for f, fn in forms.items():
                    for wk in works:
                        wk.copy_(st)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for wk in works:
                        fn(wk)
                    b.record()
                    b.synchronize()
                    res[f].append(a.elapsed_time(b) / ks)
            for f in forms:
                ms = statistics.median(res[f])
                print(json.dumps({"input": fam, "pass": name, "form": f, "objects": n, "ms": ms,
                                  "hbm_frac_algorithmic": n * 10241 / ms / 1e6 / PEAK,
                                  "changed_columns_per_object": changed_cols / n,
                                  "ms_rounds": res[f], "equal": ok}), flush=True)
        del works


if __name__ == "__main__":
    main()
