"""The split pair with final states (config 3's launch, the search loop that
keeps Stepped(gens)): both grids uncapped (shipped) against capped at c blocks
per CU, looping over the batch, as the no-final-states form ships
(tools/ab/search_iter_caps_ab.py).  A 4-column block target and a whole-board
target, 64K / 256K / 1M universes, 8 and 64 generations (and config 3's 1024
at 64K); back to back (median of 3 x 20); results and final states equal."""
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
    bw, bu = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    bw[10] = bw[11] = np.uint64(3 << 40)
    for c in (9, 10, 11, 12):
        bu[c] = np.uint64(15 << 39)
    bu &= ~bw
    ww, wu = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    wu[0::3] = np.uint64(1 << 10)
    for tname, (w, u) in (("block", (bw, bu)), ("whole", (ww, wu))):
        dw, du = (torch.from_numpy(v.view(np.int64)[None].copy()).cuda() for v in (w, u))
        for n in (1 << 16, 1 << 18, 1 << 20):
            x = hip.fill_random(n, seed=3)
            fin = torch.empty_like(x)
            for gens in ((8, 64, 1024) if n == 1 << 16 else (8, 64)):
                ref = tune.step_contains_pair(x, dw, du, gens, 0, 0, final=fin)
                ref_fin = fin.clone()
                r = {"target": tname, "universes": n, "gens": gens}
                for c in (0, 16, 32, 64):
                    fn = lambda a, b, g=gens, c=c: tune.step_contains_pair(x, dw, du, g, c, c, final=fin)  # noqa: E731
                    got = fn(0, 0)
                    r[f"cap{c}_equal"] = bool((got == ref).all().item() and (fin == ref_fin).all().item())
                    r[f"cap{c}_ms"] = bench.back_to_back_ms(rt, fn, x, x)
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
