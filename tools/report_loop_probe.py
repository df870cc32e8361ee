"""The search filter's launch report in a loop that rewrites its target
(ADVICE r05 items 1-2).

Round 5's filter picked its launch form from the report word of the last
call on the same target buffers (keyed on the wanted / unwanted pointers and
the generation count); a loop that writes a new target into one pair of
device buffers before every call always read the previous target's report
(profiles/r06/report_loop_reported.jsonl: +13-20 % per call).  Round 6 reads
no report (step.hip), so the three loops should match
(profiles/r06/report_loop_unified.jsonl).  This probe times three loops over the same
sequence of calls -- 1M config-2 universes, targets cycling block (4 x 4
window), one-row whole board, full height (bench.py's), at 1, 2, 5 and 8
generations:

  fixed:   every target in buffers of its own (its report always current)
  rewrite: one pair of buffers, the next target copied in before each call
  fresh:   a new pair of tensors for every call (pointers the allocator
           hands out again and again, or new ones)

Per loop: the time of the whole cycle (events, median of 7 cycles of 9
calls each, the copies included in every loop: `fixed` copies into a scratch
pair), and the answers of every call checked against the fixed loop's.

  python tools/report_loop_probe.py  -> one JSON line per generation count
"""
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import lifeapi_amd.hip as hip  # noqa: E402
from filter_iter_probe import targets  # noqa: E402


def main():
    n = int(os.environ.get("N", str(1 << 20)))
    x = hip.fill_random(n, seed=2)
    tg = targets(x)
    names = ["block", "one_row", "full_height"]
    seq = [names[i % 3] for i in range(9)]
    for gens in [int(g) for g in os.environ.get("GENS", "1,2,5,8").split(",")]:
        own = {k: (tg[k][0].clone(), tg[k][1].clone()) for k in names}
        shared = (torch.empty_like(own["block"][0]), torch.empty_like(own["block"][1]))
        scratch = (torch.empty_like(shared[0]), torch.empty_like(shared[1]))

        def fixed():
            outs = []
            for k in seq:
                scratch[0].copy_(own[k][0])
                scratch[1].copy_(own[k][1])
                outs.append(hip.step_contains(x, own[k][0], own[k][1], gens)[0])
            return outs

        def rewrite():
            outs = []
            for k in seq:
                shared[0].copy_(own[k][0])
                shared[1].copy_(own[k][1])
                outs.append(hip.step_contains(x, shared[0], shared[1], gens)[0])
            return outs

        def fresh():
            outs = []
            for k in seq:
                w, u = own[k][0].clone(), own[k][1].clone()
                outs.append(hip.step_contains(x, w, u, gens)[0])
            return outs

        loops = {"fixed": fixed, "rewrite": rewrite, "fresh": fresh}
        ref = [o.clone() for o in fixed()]
        row = {"gens": gens, "universes": n, "sequence": seq, "ms_per_cycle": {}, "ms_per_call": {}, "ok": {}}
        for name, fn in loops.items():
            got = fn()
            fn()
            torch.cuda.synchronize()
            row["ok"][name] = all(bool(torch.equal(a, b)) for a, b in zip(got, ref))
            ts = []
            for _ in range(7):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                fn()
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b))
            row["ms_per_cycle"][name] = statistics.median(ts)
            row["ms_per_call"][name] = statistics.median(ts) / len(seq)
        row["rewrite_over_fixed"] = row["ms_per_cycle"]["rewrite"] / row["ms_per_cycle"]["fixed"]
        row["fresh_over_fixed"] = row["ms_per_cycle"]["fresh"] / row["ms_per_cycle"]["fixed"]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
