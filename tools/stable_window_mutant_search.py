"""Search for LifeStables on which Propagate's window width matters: the
shipped library against a build whose window trusts only RHO = 1 row
(`MUTANT`: a .so built from lifeapi_amd/csrc with stable_kernels.hpp's
RHO for PropagateStep set to 1), on N candidates of the cascade family of
tests/test_ref_gpu.py (still lifes on an 8-cell lattice under a large unknown
region with a few decided cells; here also denser lattices and taller
regions), propagated and then with unknown cells decided (next nodes: their
later steps take the window).  Writes the inputs on which the two differ (at most 64) to
OUT (.npy): tests/golden/make_golden.py turns them into a fixture with the
reference's answers.

  MUTANT=build/abs/liblifeapi_hip_mut.so OUT=gpurun_out/x.npy python tools/stable_window_mutant_search.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lifeapi_amd.hip as hip  # noqa: E402
from oracle.oracle import Port  # noqa: E402  (the parser only: test infrastructure)


def candidates(n, seed):
    rng = np.random.default_rng(seed)
    port = Port()
    pats = [port.parse(t) for t in ("2o$2o!", "b2o$o2bo$b2o!", "b2o$o2bo$bobo$2bo!", "2o$obo$bo!", "bo$obo$bo!")]
    st = np.zeros((n, 64), np.uint64)
    dens = rng.uniform(0.3, 0.9, n)
    for gx in range(8):
        for gy in range(8):
            pick = rng.integers(len(pats), size=n)
            on = rng.random(n) < dens
            for k, pt in enumerate(pats):
                sel = on & (pick == k)
                for c in range(4):
                    st[sel, (8 * gx + 1 + c) % 64] |= np.uint64(int(pt[c]) << (8 * gy + 1)) if c < len(pt) else np.uint64(0)
    y0 = rng.integers(64, size=n)
    h = rng.integers(10, 56, size=n)
    x0 = rng.integers(64, size=n)
    w = rng.integers(10, 64, size=n)
    rows = np.zeros(n, np.uint64)
    for i in range(64):
        rows |= np.where(i < h, np.uint64(1) << ((y0 + i) % 64).astype(np.uint64), np.uint64(0))
    unk = np.zeros((n, 64), np.uint64)
    for c in range(64):
        unk[:, c] = np.where(((c - x0) % 64) < w, rows, np.uint64(0))
    state = st & ~unk
    for _ in range(3):
        c = (x0 + (rng.random(n) * w).astype(np.int64)) % 64
        b = ((y0 + (rng.random(n) * h).astype(np.int64)) % 64).astype(np.uint64)
        use = rng.random(n) < 0.8
        bit = np.uint64(1) << b
        idx = np.arange(n)
        unk[idx[use], c[use]] &= ~bit[use]
        on = use & (rng.random(n) < 0.5)
        state[idx[on], c[on]] |= bit[on]
    x = np.zeros((n, 10, 64), np.uint64)
    x[:, 0], x[:, 1] = state, unk
    return x.reshape(n, 640)


def main():
    n = int(os.environ.get("N", str(1 << 18)))
    x = candidates(n, int(os.environ.get("SEED", "11")))
    mut = ctypes.CDLL(os.environ["MUTANT"])
    mut.lifeapi_stable_pass_batch_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                                  ctypes.c_uint32, ctypes.c_void_p]
    # the parents propagated to their fixpoint (the shipped kernel), then one
    # to three of their unknown cells decided: next nodes, whose later steps
    # run on the window
    rng = np.random.default_rng(int(os.environ.get("SEED", "11")) + 1)
    par = torch.from_numpy(x.view(np.int64)).cuda()
    hip.stable_pass(par, "propagate")
    x = par.cpu().numpy().view(np.uint64).reshape(n, 10, 64).copy()
    for _ in range(int(os.environ.get("DECIDE", "2"))):
        unk = x[:, 1]
        cols_any = unk != 0
        has = cols_any.any(axis=1)
        # a random unknown column per object, then its lowest or highest unknown bit
        r = rng.random((n, 64)) * cols_any
        c = r.argmax(axis=1)
        u = unk[np.arange(n), c]
        low = u & (~u + np.uint64(1))
        hi = np.where(u != 0, np.uint64(1) << (np.floor(np.log2(np.maximum(u, 1).astype(np.float64))).astype(np.uint64)), np.uint64(0))
        bit = np.where(rng.random(n) < 0.5, low, hi)
        bit = np.where(has, bit, np.uint64(0))
        idx = np.arange(n)
        x[idx, 1, c] &= ~bit
        on = rng.random(n) < 0.5
        x[idx[on], 0, c[on]] |= bit[on]
    x = x.reshape(n, 640)
    a = torch.from_numpy(x.view(np.int64)).cuda()
    b = a.clone()
    fa = hip.stable_pass(a, "propagate")
    fb = torch.empty(n, dtype=torch.uint8, device="cuda")
    rc = mut.lifeapi_stable_pass_batch_dev(b.data_ptr(), fb.data_ptr(), n, 4, 0, None)
    assert rc == 0, rc
    torch.cuda.synchronize()
    diff = ((a != b).any(dim=1) | (fa != fb)).cpu().numpy()
    idx = np.nonzero(diff)[0]
    print(f"{n} candidates, {int((fa & 1).sum())} consistent, {idx.size} differ", flush=True)
    np.save(os.environ.get("OUT", "gpurun_out/stable_window_cases.npy"), x[idx[:64]])


if __name__ == "__main__":
    main()
