"""A/B: the search filter and Contains, shipped (launch form by the target's
last report) against the tuning build's fixed forms, same process, 1M
config-2 universes (seed 2), bench.py's two targets (golden.json
digests.config2_filter: block = 4 care columns; whole board = row 10 of every
third column) and a whole-board target with five care rows spread over the
column (rows 0, 12, 29, 46, 63: no row window).  Forms: dma_r8 = the LDS form
on the uncapped grid (cone shape upw 1), dma_r8_norows = the same without
the packed row-window pass (upw 2), capped = the capped form (upw 0, 16 blocks
per CU).  Per (target, op, form): back to back (20 launches between one pair
of events, median of 7) and each launch alone after a 768 MiB scrub (median
of 10, bench.py's secondary.filter timing); answers checked against the
shipped kernel's.  One JSON line per row."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        gold = json.load(f)["digests"]["config2_filter"]
    n = gold["universes"]
    x = hip.fill_random(n, seed=gold["seed"])
    scrub = bench.Scrub(rt)
    forms = {"shipped": None, "dma_r8": (1, 8), "dma_r8_norows": (2, 8), "capped": (16000, 8)}
    targets = {k: tuple(np.array([int(v, 16) for v in t[k2]], dtype=np.uint64) for k2 in ("wanted", "unwanted"))
               for k, t in gold["targets"].items()}
    full_u = np.zeros(64, np.uint64)
    full_u[0::3] = np.uint64(0x8000400020001001)  # five care rows spread over the column: the full pass
    targets["whole_board_5rows"] = (np.zeros(64, np.uint64), full_u)
    ops = [("filter_1gen", 1), ("filter_2gen", 2), ("filter_4gen", 4), ("contains", 0)]
    if os.environ.get("FILTER_AB_OPS"):
        ops = [o for o in ops if o[0] in os.environ["FILTER_AB_OPS"].split(",")]
    for name, (w, u) in targets.items():
        if os.environ.get("FILTER_AB_TARGETS") and name not in os.environ["FILTER_AB_TARGETS"].split(","):
            continue
        tw, tu = (torch.from_numpy(v.view(np.int64)[None].copy()).cuda() for v in (w, u))
        for op, gens in ops:
            row = {"target": name, "op": op, "universes": n}
            ref = None
            for form, shape in forms.items():
                if shape is None:
                    fn = (lambda: hip.step_contains(x, tw, tu, gens)[0]) if gens else (lambda: hip.contains(x, tw, tu))
                else:
                    fn = lambda s=shape: tune.cone(x, tw, tu, gens, s[0], s[1], first=gens > 0)  # noqa: E731
                got = fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = got.clone()
                    row["hits"] = int((ref > 0).sum())
                row[f"{form}_exact"] = bool(torch.equal(got.to(ref.dtype), ref))
                row[f"{form}_b2b_ms"] = bench.back_to_back_ms(rt, lambda a, b: fn(), x, x)
                row[f"{form}_scrubbed_ms"], _ = bench.scrubbed_ms(rt, lambda a, b: fn(), x, x, scrub)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
