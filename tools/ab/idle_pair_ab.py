"""What an idle launch costs: the shipped fused search loop for gens > 2
launches two kernels whose waves each find the target's row window, and the
one that does not own it returns at once.  The shipped pair against its
working kernel alone (tuning variant 7, windows of <= 4 rows) on 64K and 1M
universes, 8 and 64 generations, no final states: the difference is the
idle kernel (n / 4 waves that exit after the window search)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip as tune  # noqa: E402


class RT:
    kind = "hip"

    def __init__(self):
        self.device = torch.device("cuda", 0)
        self.stream = torch.cuda.current_stream()

    @staticmethod
    def event():
        return torch.cuda.Event(enable_timing=True)


def main():
    rt = RT()
    w, u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    w[10] = w[11] = np.uint64(3 << 40)
    for c in (9, 10, 11, 12):
        u[c] = np.uint64(15 << 39)
    u &= ~w
    dw, du = (torch.from_numpy(v.view(np.int64)[None].copy()).cuda() for v in (w, u))
    for n in (1 << 16, 1 << 20):
        x = hip.fill_random(n, seed=3)
        for gens in (8, 64):
            pair = lambda a, b, gens=gens: hip.step_contains(x, dw, du, gens)  # noqa: E731
            lo = lambda a, b, gens=gens: tune.step_contains(x, dw, du, gens, 7)  # noqa: E731
            assert (pair(0, 0)[0] == lo(0, 0)).all()
            r = {"universes": n, "gens": gens}
            for name, fn in (("pair", pair), ("lo_only", lo), ("pair2", pair), ("lo_only2", lo)):
                r[name + "_ms"] = bench.back_to_back_ms(rt, fn, x, x)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
