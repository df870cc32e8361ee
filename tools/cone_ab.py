"""A/B of the light-cone Contains / search filter (k_cone, cone_kernels.hpp)
against the full-universe kernels it replaces, one process, 1M universes
(--n): objects/s and HBM fraction on the algorithmic bytes of the FULL read
(512 B per universe + the output), so the gain shows as objects/s.

Targets (care-column window w, light cone K = w + 2g):
  block  2x2 block + ring, 4 columns      (K = 4 / 6 at g = 0 / 1)
  loaf   loaf + 6x6 box, 6 columns         (K = 6 / 8)
  w14    14 columns                        (K = 14 / 16)
  w30    30 columns                        (K = 30 / 32)
  full   64 columns                        (the whole board)
One JSON line per (target, kernel, shape)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip as tune  # noqa: E402

PEAK = 8000.0
K = 20


def timed(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(K):
            fn()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b) / K)
    return sorted(ms)[len(ms) // 2]


def targets():
    def box(x0, w, rows):
        t = np.zeros(64, np.uint64)
        for i in range(w):
            t[(x0 + i) % 64] = np.uint64(rows)
        return t
    out = {}
    bw = np.zeros(64, np.uint64)
    bw[10] = bw[11] = np.uint64(3 << 40)
    out["block"] = (bw, box(9, 4, 15 << 39) & ~bw)
    lw = np.zeros(64, np.uint64)
    for c, rows in zip(range(21, 25), ((1,), (0, 2), (0, 3), (1, 2))):
        lw[c] = np.uint64(sum(1 << (31 + r) for r in rows))
    out["loaf"] = (lw, box(20, 6, 0x3F << 30) & ~lw)
    for name, w in (("w14", 14), ("w30", 30), ("full", 64)):
        b = box(3, w, 0xFF << 20)
        t = b & np.uint64(0x5555555555555555)
        out[name] = (t, b & ~t)
    return out


def line(**d):
    print(json.dumps(d), flush=True)


def main():
    n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 1 << 20
    x = hip.fill_random(n, seed=7)
    for name, (w, u) in targets().items():
        dw = torch.from_numpy(w.view(np.int64)[None].copy()).cuda()
        du = torch.from_numpy(u.view(np.int64)[None].copy()).cuda()
        out8 = torch.empty(n, dtype=torch.uint8, device="cuda")
        ref_c = tune.reduce(3, x, out8.clone(), 8, 0, wanted=dw, unwanted=du)
        ref_f = tune.step_contains_nat(x, dw, du, 1, 8, 0)
        assert (hip.contains(x, dw, du) == ref_c).all() and (hip.step_contains(x, dw, du, 1)[0] == ref_f).all()
        rows = [("contains", "k_contains16<8> (round 3)", 513, lambda: tune.reduce(3, x, out8, 8, 0, dw, du)),
                ("contains", "shipped", 513, lambda: hip.contains(x, dw, du)),
                ("filter1", "k_step_contains<8> (round 3)", 516, lambda: tune.step_contains_nat(x, dw, du, 1, 8, 0)),
                ("filter1", "shipped", 516, lambda: hip.step_contains(x, dw, du, 1)),
                ("filter2", "k_step_contains<8> (round 3)", 516, lambda: tune.step_contains_nat(x, dw, du, 2, 8, 0)),
                ("filter2", "shipped", 516, lambda: hip.step_contains(x, dw, du, 2))]
        for upw, rmax in ((16, 8), (32, 4), (32, 8), (32, 16), (64, 8), (64, 16), (32, 104), (32, 108), (64, 108), (64, 116),
                           (0, 8), (4000, 8), (8000, 8), (16000, 8), (32000, 8), (8000, 16), (0, 16)):
            # upw 0 + 1000 c: k_cone_adapt (chunk 64 / 16 by the window) capped at c blocks per CU
            # rmax + 100: the pipelined pass (the next pass's loads before this pass's steps)
            label = f"k_cone<{upw},{rmax % 100}{' pipelined' if rmax > 100 else ''}>"
            if upw % 1000 == 0:
                label = f"k_cone_adapt<{rmax}> cap {upw // 1000}"
            rows.append(("contains", label, 513,
                         lambda upw=upw, rmax=rmax: tune.cone(x, dw, du, 0, upw, rmax, first=False)))
            rows.append(("filter1", label, 516,
                         lambda upw=upw, rmax=rmax: tune.cone(x, dw, du, 1, upw, rmax)))
        for what, kern, nbytes, fn in rows:
            ms = timed(fn)
            line(target=name, op=what, kernel=kern, n=n, ms=ms, objects_per_s=n / ms * 1e3,
                 full_read_GBps=n * nbytes / ms / 1e6, full_read_frac=n * nbytes / ms / 1e6 / PEAK)


if __name__ == "__main__":
    main()
