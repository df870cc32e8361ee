"""Light-cone filter / Contains: one-shot grid (shipped, every wave finds the
window, loads and exits) against capped grids whose waves find the window
once and loop over the batch, and 64 universes per wave; 1M config-2
universes, the 4-column target and a loaf box, the whole-board target;
each launch alone after a 768 MiB read-only scrub (median of 10; the
realistic case: a filter's input is fresh) and back to back (median of 3 x
20).  One JSON line per (target, op, shape)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip as tune  # noqa: E402
from cone_ab import targets  # noqa: E402


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
    scrub = bench.Scrub(rt)
    n = 1 << 20
    x = hip.fill_random(n, seed=2)
    shapes = [(32, 8), (64, 8), (64, 16), (1000 * 4 + 32, 8), (1000 * 8 + 32, 8), (1000 * 16 + 32, 8),
              (1000 * 8 + 64, 8), (1000 * 4 + 64, 16)]
    for name in ("block", "loaf", "full"):
        w, u = targets()[name]
        dw, du = (torch.from_numpy(v.view(np.int64)[None].copy()).cuda() for v in (w, u))
        want_f = hip.step_contains(x, dw, du, 1)[0]
        want_c = hip.contains(x, dw, du)
        for op in ("filter1", "contains"):
            for upw, rmax in shapes:
                first = op == "filter1"
                fn = (lambda a, b, upw=upw, rmax=rmax, first=first:
                      tune.cone(x, dw, du, 1 if first else 0, upw, rmax, first=first))
                got = fn(None, None)
                ok = bool((got == (want_f if first else want_c)).all().item())
                scr, _ = bench.scrubbed_ms(rt, fn, x, x, scrub)
                b2b = bench.back_to_back_ms(rt, fn, x, x)
                print(json.dumps({"target": name, "op": op, "upw": upw % 1000, "blocks_per_cu": upw // 1000,
                                  "rmax": rmax, "scrubbed_ms": scr, "b2b_ms": b2b, "equal": ok}), flush=True)


if __name__ == "__main__":
    main()
