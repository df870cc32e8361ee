#!/usr/bin/env python3
"""A/B of the launch-order policy on interleaved batches:
two batches A and B ping-ponged in turn (step A, step B, step A, ...), one
generation per launch, with the shipped kernel and store policy (the last
min(256 MiB, half the batch) of each launch stored plain), the group order
chosen by

  book      the product (host.hip launch_reverse): reverse exactly when the
            input is a batch written forward, so each batch alternates on its
            own -- A, B, A, B gives A: F, R, F ... and B: F, R, F ...
  device    round 2's rule: the order flips on every launch on the device,
            whatever the batch -- A, B, A, B gives F, R, F, R, so A always
            reads in forward and B in reverse, and neither reuses its tail
  fixed     one order, every launch

Same process, rounds interleaved; TB/s of algorithmic bytes (1 KiB per
universe-generation).  The book and device rules are emulated with the
tuning build's launcher (tools/tune step_order) so all three run the same
kernel; the product path is timed too.  Usage: python tools/ab/order_interleave_ab.py"""
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


def run(policy, bufs, n, launches=40, batches="AB", resident=None):
    """`launches` launches alternating A and B (launches/2 each), ping-pong
    within each batch; returns TB/s over the whole sequence.  resident: the
    occupancy cap of the emulated policies (None: the product's rule)"""
    plain = min(256 << 20, n * 512 // 2)
    if resident is None:
        resident = 0 if n <= (1 << 22) else 7
    cur = {"A": 0, "B": 0}
    wrote = {"A": False, "B": False}  # order the batch's current input was written in
    flip = False
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(launches):
        b = batches[k % len(batches)]
        src, dst = bufs[b][cur[b]], bufs[b][1 - cur[b]]
        if policy == "product":
            hip.step(src, out=dst, generations=1)
        else:
            if policy == "book":
                rev = not wrote[b]
                rev = rev if k >= len(batches) else False  # a batch's first launch: nothing recorded yet
            elif policy == "device":
                rev = flip
                flip = not flip
            else:
                rev = False
            tune.step_order(src, dst, 1, reverse=rev, nts=True, resident=resident, upw=4, plain_bytes=plain)
            wrote[b] = rev
        cur[b] = 1 - cur[b]
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1)
    return launches * n * 1024 / (ms / 1e3) / 1e12


def caps_main(sizes):
    """--caps: one batch, the book's order, occupancy caps 0 / 6 / 7"""
    for n in sizes:
        bufs = {"A": [hip.fill_random(n, seed=1), torch.empty((n, 64), dtype=torch.int64, device="cuda")]}
        res = {c: [] for c in ("product", 0, 6, 7)}
        for _ in range(6):
            for c in res:
                if c == "product":
                    res[c].append(run("product", bufs, n, batches="A"))
                else:
                    res[c].append(run("book", bufs, n, batches="A", resident=c))
        print(json.dumps({"universes": n, "order": "book (one batch)",
                          **{f"TBps_{'product' if c == 'product' else f'cap{c}'}": statistics.median(v)
                             for c, v in res.items()}}), flush=True)
        del bufs
        torch.cuda.empty_cache()


def main():
    if "--caps" in sys.argv:
        return caps_main([int(a) for a in sys.argv[1:] if a != "--caps"])
    sizes = [int(a) for a in sys.argv[1:]] or [1 << 16, 1 << 17, 3 << 16, 1 << 18, 3 << 17, 1 << 19, 1 << 20]
    for n in sizes:
        bufs = {b: [hip.fill_random(n, seed=s), torch.empty((n, 64), dtype=torch.int64, device="cuda")]
                for b, s in (("A", 1), ("B", 2))}
        for batches in ("A", "AB"):
            pols = ("product", "book", "fixed") if batches == "A" else ("product", "book", "device", "fixed")
            res = {p: [] for p in pols}
            for _ in range(6):
                for p in res:
                    res[p].append(run(p, bufs, n, batches=batches))
            print(json.dumps({"universes_per_batch": n, "batches": len(batches), "launches": 40,
                              **{f"TBps_{p}": statistics.median(v) for p, v in res.items()},
                              "rounds": res}), flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
