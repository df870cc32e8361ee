#!/usr/bin/env python3
"""Config 2 (1M universes x 1 gen): in-place Step() (out == in, the
reference's own Step() semantics) against ping-pong buffers, for a few launch
configurations; interleaved rounds, HIP-event timing of 20 back-to-back
launches.  Prints one JSON line per variant."""
import itertools
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import lifeapi_amd.hip as hip  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tune"))
import tune_hip  # noqa: E402  (tools/tune/liblifeapi_tune.so: explicit launch configurations)


def main():
    n = 1 << 20
    a = hip.fill_random(n, seed=2)
    b = torch.empty_like(a)
    cfgs = [None] + [tune_hip.LaunchCfg(0, u, 0, nt, 3) for u, nt in itertools.product((2, 4, 8), (0, 1))]
    res = {}
    for rnd in range(5):
        for ci, cfg in enumerate(cfgs):
            for mode in ("pingpong", "inplace"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for k in range(20):
                    if mode == "inplace":
                        tune_hip.step(a, out=a, generations=1, cfg=cfg)
                    else:
                        src, dst = (a, b) if k % 2 == 0 else (b, a)
                        tune_hip.step(src, out=dst, generations=1, cfg=cfg)
                e1.record()
                e1.synchronize()
                res.setdefault((ci, mode), []).append(e0.elapsed_time(e1) / 20)
    for (ci, mode), ts in sorted(res.items()):
        t = sorted(ts)[len(ts) // 2]
        cfg = cfgs[ci]
        print(json.dumps({"cfg": "default" if cfg is None else cfg.as_dict(), "mode": mode,
                          "ms_median": t, "GBps": n * 1024 / (t / 1e3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
