#!/usr/bin/env python3
"""Grid-cap A/B of the LifeStable kernels (stable_kernels.hpp) on three input
families of 64K LifeStables each:
  still -- still lifes around an unknown window, fresh options (the state a
           LifeStable search starts a propagation from),
  soup  -- sparse random soups around an unknown window, fresh options,
  random -- random planes (the round-1 A/B's input).
Every pass (0 sync .. 5 stabilise) and Vulnerable, at grid caps 0 (one wave
per LifeStable), 16 and 32 blocks per CU (or argv[2]; -k = one wave per
LifeStable, at most k blocks resident per CU), through the tuning build; each
timed launch starts from the same pristine planes.  One JSON line per
(family, pass, cap): median ms over 7 launches, and whether the result
equals the cap-0 result."""
import json
import os
import statistics
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip  # noqa: E402


def fill(n, seed):
    """n seeded universes from the product's own fill (lifeapi_fill_random_dev)"""
    return hip.fill_random(n, seed=seed).cpu().numpy().view(np.uint64)

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
# grid caps (blocks per CU; 0 = one wave per LifeStable; -k = that, with at
# most k blocks resident per CU): argv[2], comma-separated
CAPS = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 16, 32]
DISTINCT = 2048


def rect(x0, y0, w, h):
    s = np.zeros(64, np.uint64)
    col = np.uint64(((1 << h) - 1) << y0)
    s[x0:x0 + w] = col
    return s


def moved(s, dx, dy):
    s = np.roll(s, dx)
    dy %= 64
    return (s << np.uint64(dy)) | (s >> np.uint64((64 - dy) % 64)) if dy else s


def family(kind, rng):
    lifes = list(hip.parse_rle_host(["2o$2o!", "b2o$o2bo$b2o!", "2o$obo$bo!", "2b2o$bobo$bo$2o!",
                                     "b2o$o2bo$bobo$2bo!", "bo$obo$bo!"])[0])
    out = np.zeros((DISTINCT, 10, 64), np.uint64)
    for u in range(DISTINCT):
        w, h = int(rng.integers(6, 24)), int(rng.integers(6, 24))
        unk = rect(int(rng.integers(0, 64 - w)), int(rng.integers(0, 64 - h)), w, h)
        if kind == "still":
            st = np.zeros(64, np.uint64)
            for _ in range(int(rng.integers(4, 12))):
                st |= moved(lifes[int(rng.integers(len(lifes)))], int(rng.integers(64)), int(rng.integers(64)))
            out[u, 0], out[u, 1] = st & ~unk, unk
        elif kind == "soup":
            f = fill(2, seed=int(rng.integers(1 << 30)))
            out[u, 0], out[u, 1] = f[0] & f[1] & ~unk, unk
        else:
            f, g, k = (fill(10, seed=int(rng.integers(1 << 30))) for _ in range(3))
            out[u, 0], out[u, 1], out[u, 2:] = f[0], g[1] & unk, f[2:] & g[2:] & k[2:]
    return np.tile(out.reshape(DISTINCT, 640), (N // DISTINCT, 1))


def timed(fn, reps=7):
    ms = []
    for _ in range(reps):
        fn(prep=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn(prep=False)
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    return statistics.median(ms), r


rng = np.random.default_rng(77)
for kind in ("still", "soup", "random"):
    pristine = torch.from_numpy(family(kind, rng).view(np.int64)).cuda()
    work = torch.empty_like(pristine)
    for which in list(range(6)) + ["vulnerable"]:
        base = None
        for cap in CAPS:
            def run(prep, which=which, cap=cap):
                if prep:
                    work.copy_(pristine)
                    return None
                if which == "vulnerable":
                    return tune_hip.stable_vulnerable(work, cap)
                return tune_hip.stable_pass(work, which, cap)
            ms, r = timed(run)
            res = (r.clone(), work.clone()) if which != "vulnerable" else (r.clone(),)
            same = None if base is None else all(torch.equal(a, b) for a, b in zip(res, base))
            if base is None:
                base = res
            print(json.dumps({"family": kind, "pass": which, "blocks_per_cu": cap, "ms": ms,
                              "equal_to_cap0": same}), flush=True)
    del pristine, work
    torch.cuda.empty_cache()
