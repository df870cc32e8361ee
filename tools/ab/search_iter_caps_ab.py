"""The iterated search loop without final states: round 4's first form (the
cone kernel launched alone, then the split pair, whose low-layout kernel
now steps the cone as well), with the cone grid and the split grids capped
at c blocks per CU (0 = one-shot); round 3's launch (the uncapped pair, no
cone); the product (kContainsLo stepping the cone, capped pair); and the
cone kernel alone (8 universes per wave, a lower bound for narrow cones): a
4-column block target (the cone answers up to 13 generations) and a
whole-board target (the split pair answers); cone cap + 1000 * u: u universes
per cone wave, 64K and 1M universes, gens 3,
8, 13, 64; back to back, median of 3 x 20; results equal across caps."""
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
    caps = []
    for tname, (w, u) in (("block", (bw, bu)), ("whole", (ww, wu))):
        dw, du = (torch.from_numpy(v.view(np.int64)[None].copy()).cuda() for v in (w, u))
        sizes = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1 << 16, 1 << 20]
        gens_list = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [3, 4, 5, 6, 8, 13, 64]
        for n in sizes:
            x = hip.fill_random(n, seed=3)
            for gens in gens_list:
                ref = tune.step_contains(x, dw, du, gens, 7)  # both targets' windows are <= 4 rows
                r = {"target": tname, "universes": n, "gens": gens}
                for cc, sc in caps:
                    fn = lambda a, b, g=gens, cc=cc, sc=sc: tune.search_iter(x, dw, du, g, cc, sc)  # noqa: E731
                    r[f"c{cc}_s{sc}_equal"] = bool((fn(0, 0) == ref).all().item())
                    r[f"c{cc}_s{sc}_ms"] = bench.back_to_back_ms(rt, fn, x, x)
                # round 3's launch (the uncapped split pair, no cone) and the product
                forms = {"round3": lambda a, b, g=gens: tune.step_contains_pair(x, dw, du, g, 0, 0),
                         "product": lambda a, b, g=gens: hip.step_contains(x, dw, du, generations=g)[0],
                         "cone8_alone": lambda a, b, g=gens: tune.cone(x, dw, du, g, 8, 8),
                         # k_cone_adapt alone (the 1-2 generation filter's kernel), 16 blocks per CU
                         "adapt_alone": lambda a, b, g=gens: tune.cone(x, dw, du, g, 16000, 8)}
                for k, fn in forms.items():
                    r[k + "_equal"] = bool((fn(0, 0) == ref).all().item())
                    r[k + "_ms"] = bench.back_to_back_ms(rt, fn, x, x)
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
