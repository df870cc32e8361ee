#!/usr/bin/env python3
"""Group-order and store-policy A/B of the one-generation step (config 2 /
config 4 shapes), ping-ponged between two buffers as bench.py does: every
launch in the same order ("fixed") against the order reversed on every other
launch ("alternate", k_step kReverse), so that each launch first reads what
the previous one wrote last, each with nontemporal ("nts") or plain stores.
The tuning build's launch of the streaming kernel (at most 6 blocks resident
per CU); runs of 40 back-to-back launches between one pair of events, the
modes interleaved, 6 runs each.  Results must equal the shipped entry
point's in every mode.  Also times the shipped entry point itself.
usage: [RESIDENT=0,4,5,8] [UPW=2,4,8] [LATE=128,256] [LATE_RESIDENT=0,6] python tools/ab/order_ab.py [universes ...]
(RESIDENT: also the alternating plain-store launch with those occupancy caps,
for each UPW universes per wave; LATE: nontemporal stores but plain for
the groups that store the last LATE MiB of each launch, alternating, with
each LATE_RESIDENT occupancy cap and LATE_UPW universes per wave)"""
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
import tune_hip  # noqa: E402

REV = 1 << 31
RUN = 40
RESIDENT = [int(r) for r in os.environ.get("RESIDENT", "").split(",") if r]  # e.g. 0,4,5,8
UPW = [int(u) for u in os.environ.get("UPW", "4").split(",") if u]  # universes per wave for RESIDENT
LATE = [int(e) for e in os.environ.get("LATE", "").split(",") if e]  # MiB stored plain at each launch's end
LATE_RESIDENT = [int(r) for r in os.environ.get("LATE_RESIDENT", "0").split(",") if r]
LATE_UPW = [int(u) for u in os.environ.get("LATE_UPW", "4").split(",") if u]


def run(bufs, launch):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(RUN):
        launch(bufs[i & 1], bufs[(i + 1) & 1], i)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / RUN


for n in [int(a) for a in sys.argv[1:]] or [1 << 18, 1 << 19, 1 << 20, 1 << 21, 1 << 22, 1 << 24]:
    a = hip.fill_random(n, seed=2)
    b = torch.empty_like(a)
    ref = hip.step(a, generations=1)
    modes = {"shipped": lambda s, d, i: hip.step(s, out=d, generations=1)}
    for nts in (True, False):
        for alt in (False, True):
            def f(s, d, i, nts=nts, alt=alt):
                tune_hip.step_order(s, d, 1, reverse=alt and bool(i & 1), nts=nts)
            modes[f"{'nts' if nts else 'plain'}-{'alternate' if alt else 'fixed'}"] = f
            for rev in (False, True):
                tune_hip.step_order(a, b, 1, reverse=rev, nts=nts)
                assert torch.equal(b, ref), (nts, rev)
    for r in RESIDENT:  # other occupancy caps for the alternating plain-store launch
        for u in UPW:
            modes[f"plain-alternate-r{r}-u{u}"] = (
                lambda s, d, i, r=r, u=u: tune_hip.step_order(s, d, 1, reverse=bool(i & 1), nts=False, resident=r,
                                                              upw=u))
            for rev in (False, True):
                tune_hip.step_order(a, b, 1, reverse=rev, nts=False, resident=r, upw=u)
                assert torch.equal(b, ref), (r, u, rev)
    for mb in LATE:  # nontemporal stores but the last `mb` MiB plain, alternating, per occupancy
        for r in LATE_RESIDENT:
            for u in LATE_UPW:
                modes[f"late{mb}M-alternate-r{r}" + (f"-u{u}" if u != 4 else "")] = (
                    lambda s, d, i, mb=mb, r=r, u=u: tune_hip.step_order(s, d, 1, reverse=bool(i & 1), resident=r,
                                                                         upw=u, plain_bytes=mb << 20))
                for rev in (False, True):
                    tune_hip.step_order(a, b, 1, reverse=rev, resident=r, upw=u, plain_bytes=mb << 20)
                    assert torch.equal(b, ref), (mb, r, u, rev)
    ms = {k: [] for k in modes}
    bufs = [a, b]
    for k in modes:  # warm
        run(bufs, modes[k])
    for rep in range(6):
        for k in (list(modes) if rep % 2 == 0 else list(modes)[::-1]):
            ms[k].append(run(bufs, modes[k]))
    for k in modes:
        med = statistics.median(ms[k])
        print(json.dumps({"universes": n, "order": k, "ms_per_launch_median": med, "ms_all": ms[k],
                          "GBps": n * 1024 / (med * 1e-3) / 1e9}), flush=True)
    del a, b, ref
    torch.cuda.empty_cache()
