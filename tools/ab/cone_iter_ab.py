"""The iterated search loop without final states (gens > 2) on the light
cone: the shipped entry point (the cone kernel with 8 universes per wave for
cones of <= 32 columns, the split pair's waves skipping them) against the
split-layout kernel that answered before (tuning variant 7, the low-layout
kernel for windows of <= 4 rows) and against cone shapes alone (universes per
wave 8 / 16 / 32 / 64), 64K and 1M universes, a 2 x 2 block + ring target
(4 columns, 4 rows), gens 3 / 5 / 8 / 13 (cone 10 / 14 / 20 / 30 columns);
back to back, median of 3 x 20.  Results equal (checked per case)."""
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
        for gens in (3, 5, 8, 13):
            forms = {"shipped": lambda a, b, g=gens: hip.step_contains(x, dw, du, g)[0],
                     "split_lo": lambda a, b, g=gens: tune.step_contains(x, dw, du, g, 7)}
            for upw in (8, 16, 32, 64):
                forms[f"cone{upw}"] = lambda a, b, g=gens, upw=upw: tune.cone(x, dw, du, g, upw, 8)
            ref = forms["split_lo"](0, 0)
            r = {"universes": n, "gens": gens}
            for name, fn in forms.items():
                r[name + "_equal"] = bool((fn(0, 0) == ref).all().item())
                r[name + "_ms"] = bench.back_to_back_ms(rt, fn, x, x)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
