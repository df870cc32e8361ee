#!/usr/bin/env python3
"""Launch overhead of the bench loop: K back-to-back ping-pong launches of
the shipped one-generation step issued one by one, against the same K
launches captured once into a HIP graph (torch.cuda.CUDAGraph over the
library's launches on the capture stream) and replayed; interleaved, per-step
time from events around the K launches.  Results must be identical.
usage: python tools/ab/graph_ab.py [universes] [K]"""
import json
import os
import statistics
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import lifeapi_amd.hip as hip  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
x0 = hip.fill_random(n, seed=2)
a, b = x0.clone(), torch.empty_like(x0)
bufs = [a, b]


def launches(stream):
    for k in range(K):
        hip.step(bufs[k & 1], out=bufs[(k + 1) & 1], generations=1, stream=stream)


launches(torch.cuda.current_stream())  # warm, and the library's per-device state
torch.cuda.synchronize()
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    launches(s)
torch.cuda.synchronize()
# same result: K steps from the same start, either way
a.copy_(x0)
launches(torch.cuda.current_stream())
torch.cuda.synchronize()
plain = bufs[K & 1].clone()
a.copy_(x0)
g.replay()
torch.cuda.synchronize()
assert torch.equal(bufs[K & 1], plain)
ms = {"plain": [], "graph": []}
cur = torch.cuda.current_stream()
for rep in range(24):
    for kind in (("plain", "graph") if rep % 2 else ("graph", "plain")):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        if kind == "plain":
            launches(cur)
        else:
            g.replay()
        e1.record(cur)
        e1.synchronize()
        if rep >= 4:
            ms[kind].append(e0.elapsed_time(e1) / K)
for kind, v in ms.items():
    print(json.dumps({"universes": n, "K": K, "launch": kind, "ms_per_step_median": statistics.median(v),
                      "ms_per_step_min": min(v)}), flush=True)
