"""Interleaved per-launch timing of the whole-board search filter's forms and
of Contains on the same bytes: 1M config-2 universes (seed 2), bench.py's
whole-board target (golden.json digests.config2_filter: row 10 of every third
column) at 1, 2 and 4 generations.  Per rep, every form in turn: a 768 MiB
scrub (bench.Scrub), then the launch alone between a pair of events; the
forms alternate launch by launch, so that a clock or fabric state that drifts
over a series falls on all of them alike.  Forms: shipped,
rows / norows (tuning build cone shapes upw 1 / 2: the LDS form with and
without the packed row-window pass), rows_capC (upw 3: rows on a grid of at
most C blocks per CU looping over the batch), probe_sS (with PROBE=1: the pass with no
window search and s_sleep(S) after each next-pass fetch, tune_cone.hip
k_rows_probe), capped (upw 0, 16 blocks per CU), and
Contains (shipped, and the LDS form).  One JSON line per generation count:
median, 10th and 90th percentile per form, answers checked against the
shipped form."""
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
    reps = int(os.environ.get("REPS", "40"))
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        gold = json.load(f)["digests"]["config2_filter"]
    n = gold["universes"]
    x = hip.fill_random(n, seed=gold["seed"])
    t = gold["targets"]["whole_board"]
    tw, tu = (torch.from_numpy(np.array([[int(v, 16) for v in t[k]]], dtype=np.uint64).view(np.int64)).cuda()
              for k in ("wanted", "unwanted"))
    scrub = bench.Scrub(rt)
    runs = [(int(v), None) for v in os.environ.get("GENS", "1,2,4").split(",")]
    if os.environ.get("ROWS"):  # GENS x ROWS: the bench target's care row moved to each row given
        runs = [(g, int(r)) for r in os.environ["ROWS"].split(",") for g, _ in runs]
    for gens, row10 in runs:
        if row10 is not None:
            u = np.zeros(64, np.uint64)
            u[0::3] = np.uint64(1) << np.uint64(row10)
            tw.zero_()
            tu.copy_(torch.from_numpy(u.view(np.int64)[None].copy()))
        r = 10 if row10 is None else row10  # the care row (the probe's window starts gens above it)
        forms = {
            "shipped": lambda: hip.step_contains(x, tw, tu, gens)[0],
            "rows": lambda: tune.cone(x, tw, tu, gens, 1, 8, first=True),
            "rows_cap16": lambda: tune.cone(x, tw, tu, gens, 16003, 8, first=True),
            "norows": lambda: tune.cone(x, tw, tu, gens, 2, 8, first=True),
            "capped": lambda: tune.cone(x, tw, tu, gens, 16000, 8, first=True),
            **({f"probe_s{sl}": (lambda sl=sl: tune.rows_probe(x, tw, tu, gens, (r - gens) & 63, sl))
                for sl in (0, 2, 8)} if os.environ.get("PROBE") else {}),
            "contains": lambda: hip.contains(x, tw, tu),
            "contains_lds": lambda: tune.cone(x, tw, tu, 0, 1, 8, first=False),
        }
        ref = forms["shipped"]().clone()
        torch.cuda.synchronize()
        row = {"generations": gens, "care_row": 10 if row10 is None else row10, "universes": n, "reps": reps, "hits": int((ref > 0).sum())}
        for name, fn in forms.items():
            if name.startswith("contains"):
                continue
            got = fn()
            torch.cuda.synchronize()
            row[f"{name}_exact"] = bool(torch.equal(got.to(ref.dtype), ref))
        ms = {k: [] for k in forms}
        for r in range(reps + 3):
            for name, fn in forms.items():
                scrub()
                e0, e1 = rt.event(), rt.event()
                e0.record(rt.stream)
                fn()
                e1.record(rt.stream)
                e1.synchronize()
                if r >= 3:
                    ms[name].append(e0.elapsed_time(e1))
        for name, v in ms.items():
            row[name] = {"median": float(np.median(v)), "p10": float(np.percentile(v, 10)),
                         "p90": float(np.percentile(v, 90))}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
