"""GPU parity of the TUNING build (tools/tune/liblifeapi_tune.so): every
measured alternative to the shipped step kernels -- other networks, exchanges,
layouts, tiles and assembly-loop schedules -- against the oracle, bit-exact.
These configurations are not in the product library; the shipped ones are
covered by tests/test_gpu_parity.py and tests/test_ref_gpu.py."""
import itertools
import os
import sys

import numpy as np
import pytest

from test_gpu_parity import seam_cases, to_dev, to_host

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "tune"))

ALL_CFGS = list(itertools.product(range(8), (1, 2, 4, 8), (0, 1), (0, 1, 2, 3, 4)))
# the hand-allocated loop exists for rule 4 only
ALL_CFGS += list(itertools.product((8,), (1, 2, 4, 8), (0, 1), (4,)))
# the row-split layouts: LDS exchange, 1 or 2 groups of 2 / 4 universes
ALL_CFGS += list(itertools.product((1,), (1, 2), (0, 1), (5, 6, 7)))
# the tile layouts (4 / 2 columns per lane): one tile per wave
ALL_CFGS += [(x, 1, nt, r) for r, xs in ((8, (0, 1, 8)), (9, (1,))) for x in xs for nt in (0, 1)]
# the 6-LUT tail: split layouts (rules 10-12) and the 4-column tile (rule 13)
ALL_CFGS += list(itertools.product((1,), (1, 2), (0, 1), (10, 11, 12)))
ALL_CFGS += [(x, 1, nt, 13) for x in (0, 1) for nt in (0, 1)]
# split layouts with part of the exchange by DPP (LIFEAPI_XCHG_LDS_DPP(d) = 16 + d)
ALL_CFGS += [(16 + d, u, nt, 11) for d in (1, 2, 3, 4) for u in (1, 2) for nt in (0, 1)]
ALL_CFGS += [(16 + d, 1, nt, 12) for d in (2, 4) for nt in (0, 1)]
# the hand-allocated rule-11 loop (LIFEAPI_XCHG_ASM = 8)
ALL_CFGS += [(8, u, nt, 11) for u in (1, 2) for nt in (0, 1)]
ALL_CFGS += [(24 + k, 1, nt, 11) for k in (1, 2, 3) for nt in (0, 1)]  # its other schedules
# the software-pipelined LDS loop (LIFEAPI_XCHG_LDS_PIPE = 9)
ALL_CFGS += [(9, u, nt, r) for r in (6, 11, 12) for u in (1, 2) for nt in (0, 1)]




@pytest.fixture(scope="module")
def tune(hip):
    import tune_hip
    return tune_hip


def test_tune_default_is_shipped(tune):
    for g in (1, 2, 3, 31, 32, 1024):
        c = tune.default_cfg(g)
        assert (c.xchg, c.rule) == ((0, 3) if g <= 2 else (8, 11))


@pytest.mark.parametrize("xchg,upw,nt,rule", ALL_CFGS)
def test_step_all_cfgs(tune, port, xchg, upw, nt, rule):
    n = 2048 + 3                               # ragged vs every U
    x = port.fill(n, seed=1000 + xchg * 100 + upw * 10 + nt * 2 + rule)
    x = np.concatenate([seam_cases(port), x])
    cfg = tune.LaunchCfg(xchg, upw, 1, nt, rule)  # 1 block/CU: forces grid-striding
    d = to_dev(x)
    for gens in (1, 5):
        got = to_host(tune.step(d, generations=gens, cfg=cfg))
        want = port.step_batch(x, gens)
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, f"gens={gens}: {bad.size} universes differ, first {bad[:8]}"




@pytest.mark.parametrize("nts", [False, True])
@pytest.mark.parametrize("reverse", [False, True])
def test_step_order(tune, port, nts, reverse):
    """The streaming step in either group order, plain or nontemporal
    stores (tools/ab/order_ab.py), 2, 4 or 8 universes per wave, ragged against
    each, 1 and 2 generations."""
    import torch
    n = 4096 + 3
    x = np.concatenate([seam_cases(port), port.fill(n, seed=4242)])
    d = to_dev(x)
    out = torch.empty_like(d)
    for gens in (1, 2):
        for upw in (2, 4, 8):
            for plain in (0, 1, 300 * 512, 1 << 40):  # no, one, some and all groups store plain
                tune.step_order(d, out, gens, reverse=reverse, nts=nts, upw=upw, plain_bytes=plain)
                assert (to_host(out) == port.step_batch(x, gens)).all(), (gens, upw, plain)


def test_bad_cfgs_rejected(tune, hip):
    import torch
    d = torch.zeros((4, 64), dtype=torch.int64, device="cuda")
    for bad in [(10, 4, 8, 0, 0), (0, 3, 8, 0, 0), (0, 1, 8, 0, 5), (8, 1, 8, 0, 2)]:
        with pytest.raises(hip.LifeApiError):
            tune.step(d, generations=1, cfg=tune.LaunchCfg(*bad))


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("gens", [3, 6, 8, 9, 37])
@pytest.mark.parametrize("with_final", [False, True])
def test_step_contains_variants(tune, port, variant, gens, with_final):
    """The fused Step + Contains kernels of the tuning build (step_kernels.hpp
    kContainsAsm: 0 compiled loop ... 7 batched, low layout) against the
    oracle's step-then-Contains loop (LifeTarget.hpp:44-51), ragged n,
    planted hits; gens 3 / 6 / 8 / 9 / 37 = 0 / 0 / 1 / 1 / 4 blocks of
    eight after 3 / 6 / 0 / 1 / 5 single generations for the batched test.
    (Variant 8 takes only windows wider than this 4-row target: see
    test_step_contains_row_window.)"""
    import torch
    n = 1003
    x = port.fill(n, seed=223) & port.fill(n, seed=224) & port.fill(n, seed=225)
    blk = np.zeros(64, np.uint64)
    blk[10] = blk[11] = np.uint64(0b11 << 40)
    ring = np.zeros(64, np.uint64)
    for c in (9, 10, 11, 12):
        ring[c] = np.uint64(0b1111 << 39)
    ring &= ~blk
    x[::5] &= ~ring & ~blk
    x[::10] |= blk
    fin = torch.empty((n, 64), dtype=torch.int64, device="cuda") if with_final else None
    got = tune.step_contains(to_dev(x), to_dev(blk[None]), to_dev(ring[None]), gens, variant, final=fin)
    got = got.cpu().numpy()
    exp = np.zeros(n, np.int64)
    s = x.copy()
    for g in range(1, gens + 1):
        s = port.step_batch(s, 1)
        hit = (((s ^ blk) & (blk | ring)) == 0).all(axis=1)
        exp[(exp == 0) & hit] = g
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert (exp > 0).any()
    if with_final:
        assert (to_host(fin) == port.step_batch(x, gens)).all()



def _target(kind):
    """(wanted, unwanted) with care rows: a block + ring straddling the row
    seam (rows 62..1: window 4 across 63 -> 0), a tall one (12 rows: no
    window <= 8), a one-row target, and an empty target (always contained)"""
    w, u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    if kind == "seam":
        for c in (30, 31):
            w[c] = np.uint64((1 << 63) | 1)
        for c in (29, 30, 31, 32):
            u[c] = np.uint64((3 << 62) | 3)
        u &= ~w
    elif kind == "tall":
        w[5] = np.uint64(0b111 << 20)
        for c in (4, 5, 6):
            u[c] = np.uint64(0xFFF << 16)
        u &= ~w
    elif kind == "row":
        for c in range(10, 20):
            u[c] = np.uint64(1 << 7)
    elif kind == "six":   # a loaf (still life) in its 6 x 6 box
        for c, rows in zip(range(21, 25), ((1,), (0, 2), (0, 3), (1, 2))):
            w[c] = np.uint64(sum(1 << (31 + r) for r in rows))
        for c in range(20, 26):
            u[c] = np.uint64(0x3F << 30)
        u &= ~w
    return w, u


# the windows each variant takes: 3..5 any; 6 and 7 (<= 4 rows) the seam,
# one-row and empty targets; 8 (the wider windows) the tall and six-row ones
_WINDOW_CASES = [(k, v) for v in (3, 4, 5) for k in ("seam", "tall", "row", "empty", "six")]
_WINDOW_CASES += [(k, v) for v in (6, 7) for k in ("seam", "row", "empty")] + [(k, 8) for k in ("tall", "six")]


@pytest.mark.parametrize("kind,variant", _WINDOW_CASES)
@pytest.mark.parametrize("with_final", [False, True])
def test_step_contains_row_window(tune, hip, port, kind, with_final, variant):
    """variants 3..8 (the target's row window, universes rotated into it
    and back) against the oracle and against the shipped kernels, for
    targets whose window wraps the row seam, exceeds 8 rows, is one row, is
    empty, or is six rows (batched in the full layout)."""
    import torch
    n, gens = 2001, 9
    w, u = _target(kind)
    x = port.fill(n, seed=501) & port.fill(n, seed=502)
    x[::3] &= ~(w | u)
    x[::6] |= w
    fin = torch.empty((n, 64), dtype=torch.int64, device="cuda") if with_final else None
    got = tune.step_contains(to_dev(x), to_dev(w[None]), to_dev(u[None]), gens, variant, final=fin).cpu().numpy()
    exp = np.zeros(n, np.int64)
    s = x.copy()
    for g in range(1, gens + 1):
        s = port.step_batch(s, 1)
        hit = (((s ^ w) & (w | u)) == 0).all(axis=1)
        exp[(exp == 0) & hit] = g
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    if kind == "empty":
        assert (exp == 1).all()
    if with_final:
        assert (to_host(fin) == port.step_batch(x, gens)).all()
    ship, _ = hip.step_contains(to_dev(x), to_dev(w[None]), to_dev(u[None]), gens)
    assert (ship.cpu().numpy() == exp).all()


@pytest.mark.parametrize("caps", [(1, 1), (8, 5), (0, 0)])
@pytest.mark.parametrize("kind", ["seam", "six", "tall"])
def test_step_contains_pair_capped_grid(tune, hip, port, caps, kind):
    """the two-kernel form (7 then 8) with capped grids: every wave strides
    over several groups of universes, and the kernel with nothing to do
    returns"""
    import torch
    n, gens = 3001, 11
    w, u = _target(kind)
    x = port.fill(n, seed=601) & port.fill(n, seed=602)
    x[::4] &= ~(w | u)
    x[::8] |= w
    fin = torch.empty((n, 64), dtype=torch.int64, device="cuda")
    got = tune.step_contains_pair(to_dev(x), to_dev(w[None]), to_dev(u[None]), gens, *caps, final=fin)
    ship, shipfin = hip.step_contains(to_dev(x), to_dev(w[None]), to_dev(u[None]), gens, final=torch.empty_like(fin))
    assert torch.equal(got, ship) and torch.equal(fin, shipfin)
    assert (to_host(fin) == port.step_batch(x, gens)).all()


CONE_SHAPES = [(16, 4), (16, 8), (16, 16), (32, 4), (32, 8), (32, 16), (32, 32), (64, 8), (64, 16), (64, 32),
               (1000 + 32, 8), (2000 + 64, 16), (8000 + 32, 8),  # + 1000 c: at most c blocks per CU, grid-stride
               (1, 4), (1, 8), (2000 + 1, 8)]  # upw 1: k_cone_adapt, the whole board through LDS (cone_wave_full_dma)


@pytest.mark.parametrize("upw,rmax", CONE_SHAPES)
def test_cone_shapes(tune, port, upw, rmax):
    """every measured shape of the light-cone kernel (tune_cone.hip) against
    the oracle: Contains and the 1-2 generation filter, windows of 1..64
    columns anywhere on the board, a ragged batch"""
    rng = np.random.default_rng(upw * 100 + rmax)
    n = 1031
    x = port.fill(n, seed=upw + rmax) & port.fill(n, seed=7 * upw + rmax)
    x[::3] = x[0]
    d = to_dev(x)
    for w in (1, 3, 6, 13, 29, 31, 60, 64):
        x0 = int(rng.integers(64))
        box = np.zeros(64, np.uint64)
        for c in {x0 % 64, (x0 + w - 1) % 64}:
            box[c] = np.uint64(int(rng.integers(1, 1 << 63)))
        for gens in (0, 1, 2):
            ahead = port.step_batch(x[:1], gens)[0] if gens else x[0]
            tw, tu = ahead & box, box & ~ahead
            want = np.zeros(n, np.uint32)
            s = x.copy()
            if gens == 0:
                want = (((x ^ tw) & (tw | tu)) == 0).all(axis=1).astype(np.uint8)
                got = tune.cone(d, to_dev(tw[None]), to_dev(tu[None]), 0, upw, rmax, first=False).cpu().numpy()
            else:
                for g in range(1, gens + 1):
                    s = port.step_batch(s, 1)
                    hit = (((s ^ tw) & (tw | tu)) == 0).all(axis=1)
                    want[(want == 0) & hit] = g
                got = tune.cone(d, to_dev(tw[None]), to_dev(tu[None]), gens, upw, rmax).cpu().numpy()
            assert (got.astype(np.uint32) == want).all(), (w, x0, gens, np.nonzero(got != want)[0][:8])
            assert want[0] != 0


# k_stable_dma (stable_kernels.hpp) on the tuning build's grids: the looping
# grid (U = 0: each XCD an eighth, waves striding, the next LifeStable
# prefetched into LDS), U LifeStables per wave (U = 2, 3: the prefetch within
# a run), the wide stores (pass offset 32, U = 1) and a resident-block cap.
# The shipped SignalNeighbours is the U = 1 form (tests/test_gpu_parity.py).
@pytest.mark.parametrize("off,upw,cap", [(16, 0, 0), (16, 2, 0), (16, 3, 0), (16, 2, 3), (32, 1, 0), (32, 1, 5)])
@pytest.mark.parametrize("n", [5, 20003])
def test_stable_dma_forms(tune, hip, port, off, upw, cap, n):
    from test_gpu_parity import _stable_cases
    x = _stable_cases(port, n, seed=17 + n % 7)
    for w, name in enumerate(hip.STABLE_PASSES):
        want, wfl = port.stable_pass(x, w)
        d = to_dev(x).reshape(n, 640)
        fl = tune.stable_pass(d, off + w, cap, upw=upw).cpu().numpy()
        assert (to_host(d).reshape(n, 640) == want).all(), (name, off, upw, cap)
        assert (fl == wfl).all(), (name, off, upw, cap)


@pytest.mark.parametrize("rmax", [4, 8])
@pytest.mark.parametrize("n", [1, 3, 17, 33, 100])
def test_cone_full_dma_ragged(tune, port, rmax, n):
    """cone_wave_full_dma on batches that end inside a pass or a chunk (its
    loads clamp to the last universe, its stores stop at n): the whole-board
    filter at 1 and 2 generations and whole-board Contains against the oracle"""
    x = port.fill(n, seed=n + rmax)
    x[::2] &= port.fill(n, seed=n + 99)[::2]
    tw, tu = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    tu[0::3] = np.uint64(1 << 10)  # row 10 of every third column dead: a 62-column window
    d = to_dev(x)
    for gens in (0, 1, 2):
        if gens == 0:
            want = (((x ^ tw) & (tw | tu)) == 0).all(axis=1).astype(np.uint8)
            got = tune.cone(d, to_dev(tw[None]), to_dev(tu[None]), 0, 1, rmax, first=False).cpu().numpy()
        else:
            want, s = np.zeros(n, np.uint32), x.copy()
            for g in range(1, gens + 1):
                s = port.step_batch(s, 1)
                hit = (((s ^ tw) & (tw | tu)) == 0).all(axis=1)
                want[(want == 0) & hit] = g
            got = tune.cone(d, to_dev(tw[None]), to_dev(tu[None]), gens, 1, rmax).cpu().numpy()
        assert (got.astype(want.dtype) == want).all(), (gens, np.nonzero(got != want)[0][:8])


# k_stable's measured alternatives (stable_kernels.hpp): StabiliseOptions with
# every round on the whole columns / the later rounds on the 32-row window
# (tuning passes 6 / 7), Propagate whole / windowed (14 / 15, the product
# ships 15's form) and windowed with plane-selective stores (40)
@pytest.mark.parametrize("which,pname", [(6, "stabilise"), (7, "stabilise"), (14, "propagate"), (15, "propagate"),
                                         (40, "propagate")])
@pytest.mark.parametrize("n", [5, 20003])
def test_stable_window_forms(tune, hip, port, which, pname, n):
    from test_gpu_parity import _stable_cases
    x = _stable_cases(port, n, seed=23 + n % 7)
    w = hip.STABLE_PASSES.index(pname)
    want, wfl = port.stable_pass(x, w)
    d = to_dev(x).reshape(n, 640)
    fl = tune.stable_pass(d, which, 0, xcd_chunk=True).cpu().numpy()
    assert (to_host(d).reshape(n, 640) == want).all(), (which, pname)
    assert (fl == wfl).all(), (which, pname)
