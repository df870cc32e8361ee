#!/usr/bin/env python3
"""Config 2 (1M universes x 1 gen per launch): K back-to-back ping-pong
launches issued eagerly against the same K launches captured once in a HIP
graph (torch.cuda.CUDAGraph around the C-ABI launches) and replayed; HIP-event
time per launch, interleaved rounds.  One JSON line per mode."""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import lifeapi_amd.hip as hip  # noqa: E402


def main():
    n, K = 1 << 20, 50
    a = hip.fill_random(n, seed=2)
    b = torch.empty_like(a)
    s = torch.cuda.Stream()

    def issue(stream):
        bufs = [a, b]
        for k in range(K):
            hip.step(bufs[k % 2], out=bufs[1 - k % 2], generations=1, stream=stream)

    with torch.cuda.stream(s):
        issue(s)  # warm (and fills the library's per-device caches before capture)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        issue(s)
    torch.cuda.synchronize()
    res = {"eager": [], "graph": []}
    for _ in range(7):
        for mode in ("eager", "graph"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                e0.record(s)
                if mode == "eager":
                    issue(s)
                else:
                    g.replay()
                e1.record(s)
            e1.synchronize()
            res[mode].append(e0.elapsed_time(e1) / K)
    for mode, ts in res.items():
        t = sorted(ts)[len(ts) // 2]
        print(json.dumps({"mode": mode, "launches": K, "ms_per_launch_median": t, "ms_all": ts,
                          "GBps": n * 1024 / (t / 1e3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
