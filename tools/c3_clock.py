#!/usr/bin/env python3
"""In-kernel clock of the shipped config-3 kernel (64K universes x 1024
generations): >= 2 s of back-to-back launches of the product kernel first
(MI355X_MICROARCH.md, DVFS item 6), then the diagnostic build of the same
kernel (tools/tune: k_step_split_clock, stamps around the generation loop)
and the product kernel timed alternately.  Prints one JSON line: median
held clock over waves, both kernels' median launch times, and whether the
diagnostic output equals the product's."""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip  # noqa: E402

n, gens = 1 << 16, 1024
a = hip.fill_random(n, seed=3)
b = torch.empty_like(a)
c = torch.empty_like(a)
t0 = time.time()
while time.time() - t0 < 2.5:
    for _ in range(50):
        hip.step(a, out=b, generations=gens)
    torch.cuda.synchronize()


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1), r


prod, diag, clocks = [], [], []
for _ in range(10):
    prod.append(timed(lambda: hip.step(a, out=b, generations=gens))[0])
    ms, (_, st) = timed(lambda: tune_hip.step_clock(a, c, gens))
    diag.append(ms)
    s = st.cpu()
    dt, dq = (s[:, 2] - s[:, 0]).double(), (s[:, 3] - s[:, 1]).double()
    ok = dq > 0
    clocks.append(float((dt[ok] / dq[ok]).median()) * 0.1)  # GHz (100 MHz real-time counter)
loop_ms = (s[:, 3].max() - s[:, 1].min()).item() / 1e5
torch.cuda.synchronize()
print(json.dumps({
    "workload": "config3: 64K universes x 1024 gens", "kernel": hip.step_kernel_name(gens),
    "held_clock_GHz_median": statistics.median(clocks), "held_clock_GHz_all": clocks,
    "product_ms_median": statistics.median(prod), "diagnostic_ms_median": statistics.median(diag),
    "diagnostic_equals_product": bool(torch.equal(b, c)),
    "method": "median over waves of (s_memtime delta / s_memrealtime delta) x 100 MHz around the "
              "generation loop, after >= 2.5 s of back-to-back launches",
}), flush=True)
