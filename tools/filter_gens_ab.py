"""A/B: the search filter without final states at 3-12 generations on
whole-board targets, shipped (k_cone_adapt up to 4 generations, 6 for
batches <= 256K; beyond, the split-layout pair) against the natural layout
at every generation count (tuning build k_cone_adapt, LDS form: `rows` =
with the packed row-window pass, `norows` = the full pass).  1M config-2
universes (seed 2); targets: bench.py's whole-board one (row 10 of every third
column must be dead: one care row), one with five care rows spread over
the column (0, 12, 29, 46, 63 of every third column: no row window), and
bench.py's block target (4 columns x 4 rows), and 40 columns x 3 rows.  `capped` / `capped_norows`:
the capped form (cone shape upw 0 / 7, 16 blocks per CU) with and without
the row-window passes (for a column window: cone_wave_rows).  Per
rep every form in turn, each launch alone after a 768 MiB scrub; medians.
Answers checked against the shipped path."""
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
    reps = int(os.environ.get("REPS", "15"))
    n = int(os.environ.get("N", str(1 << 20)))
    x = hip.fill_random(n, seed=2)
    scrub = bench.Scrub(rt)
    targets = {}
    for name, rowmask in (("one_row", 1 << 10), ("five_rows", 0x8000400020001001)):
        u = np.zeros(64, np.uint64)
        u[0::3] = np.uint64(rowmask)
        targets[name] = (torch.zeros((1, 64), dtype=torch.int64, device="cuda"),
                         torch.from_numpy(u.view(np.int64)[None].copy()).cuda())
    # bench.py's block target: a 2x2 block and its ring, columns 9-12, rows 39-42
    bw, bu = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    bw[10] = bw[11] = np.uint64(3 << 40)
    bu[9:13] = np.uint64(15 << 39)
    bu &= ~bw
    targets["block"] = tuple(torch.from_numpy(v.view(np.int64)[None].copy()).cuda() for v in (bw, bu))
    # 40 columns x 3 rows (rows 20-22 must be dead): a column window wider than 32
    wu = np.zeros(64, np.uint64)
    wu[:40] = np.uint64(7 << 20)
    targets["wide"] = (torch.zeros((1, 64), dtype=torch.int64, device="cuda"),
                       torch.from_numpy(wu.view(np.int64)[None].copy()).cuda())
    only = os.environ.get("TARGETS")
    gens_list = [int(v) for v in os.environ.get("GENS", "3,4,5,6,8,12").split(",")]
    for tname, (tw, tu) in targets.items():
        if only and tname not in only.split(","):
            continue
        for gens in gens_list:
            forms = {
                "shipped": lambda: hip.step_contains(x, tw, tu, gens)[0],
                "rows": lambda: tune.cone(x, tw, tu, gens, 1, 8, first=True),
                "norows": lambda: tune.cone(x, tw, tu, gens, 2, 8, first=True),
                "capped": lambda: tune.cone(x, tw, tu, gens, 16000, 8, first=True),
                "capped_norows": lambda: tune.cone(x, tw, tu, gens, 16007, 8, first=True),
            }
            ref = forms["shipped"]().clone()
            torch.cuda.synchronize()
            row = {"target": tname, "generations": gens, "universes": n, "reps": reps,
                   "hits": int((ref > 0).sum()), "shipped_path": "k_cone_adapt" if gens <= (6 if n <= 1 << 18 else 4) else "split pair"}
            for name, fn in forms.items():
                got = fn()
                torch.cuda.synchronize()
                row[f"{name}_exact"] = bool(torch.equal(got.to(ref.dtype), ref))
            ms = {k: [] for k in forms}
            for r in range(reps + 2):
                for name, fn in forms.items():
                    scrub()
                    e0, e1 = rt.event(), rt.event()
                    e0.record(rt.stream)
                    fn()
                    e1.record(rt.stream)
                    e1.synchronize()
                    if r >= 2:
                        ms[name].append(e0.elapsed_time(e1))
            for name, v in ms.items():
                row[f"{name}_ms"] = float(np.median(v))
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
