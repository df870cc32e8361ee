#!/usr/bin/env python3
"""Config 3 (64K universes x 1024 generations, default launch cfg) run a few
times: the target program of the PMC passes in tools/ab/gpu_pmc_c3.sh."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lifeapi_amd.hip as hip  # noqa: E402

if __name__ == "__main__":
    a = hip.fill_random(1 << 16, seed=2)
    b = torch.empty_like(a)
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        hip.step(a, out=b, generations=1024)
    torch.cuda.synchronize()
    print("ok")
