"""CPU: the generated rule-11 assembly loop (tools/gen_split_asm.py ->
lifeapi_amd/csrc/split_asm.inc) is up to date, keeps its bank rules, and -- run
on numpy lanes -- computes gen_split's network (the oracle's Step() on the
8-way split layout)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_split_asm as g  # noqa: E402


def test_inc_is_generated():
    assert open(g.OUT).read() == g.emit()
    assert open(g.OUT_TUNE).read() == g.emit_tune()


def test_bank_rules():
    n, bad = g.check_banks(g.body())
    assert n == 68 and len(bad) == 16
    assert all(l.split()[-1] in ("bitop3:0x96", "bitop3:0xe8") for l in bad)  # the h-layer only


def _to_split(states):
    """4 universes (4 x 64 uint64) -> r[8][64] of the 8-way split: bit 4k + u of
    R_j = universe u, row 8k + j (split_layout.hpp)."""
    r = np.zeros((8, 64), np.uint32)
    for u in range(4):
        for j in range(8):
            for k in range(8):
                bit = (states[u] >> np.uint64(8 * k + j)) & np.uint64(1)
                r[j] |= (bit.astype(np.uint32) << np.uint32(4 * k + u))
    return r


def test_simulated_loop_is_step(port):
    x = port.fill(4, seed=77)
    for v in g.VARIANTS:
        n, bad = g.check_banks(g.body(v))
        assert n == 68 and len(bad) == 16, v
        for gens in (1, 3):
            got = g.simulate(_to_split(x), gens, variant=v)
            assert (got == _to_split(port.step_batch(x, gens))).all(), (v, gens)


def test_simulated_two_group_loop_is_step(port):
    """split_gens_asm2: two groups per wave, each one's exchange in flight
    behind the other's generation."""
    x, y = port.fill(4, seed=78), port.fill(4, seed=79)
    for gens in (1, 2, 5):
        ga, gb = g.simulate(_to_split(x), gens, two=_to_split(y))
        assert (ga == _to_split(port.step_batch(x, gens))).all(), gens
        assert (gb == _to_split(port.step_batch(y, gens))).all(), gens


@pytest.mark.parametrize("lean", [False, True])
def test_simulated_contains_loop(port, lean):
    """split_contains_asm[_lean]: the same generations plus, after each, the
    first generation at which each universe contains the target
    (LifeTarget.hpp:44-51)."""
    x = port.fill(4, seed=80) & port.fill(4, seed=81)
    blk = np.zeros(64, np.uint64)
    blk[20] = blk[21] = np.uint64(0b11 << 30)
    ring = np.zeros(64, np.uint64)
    for c in (19, 20, 21, 22):
        ring[c] = np.uint64(0b1111 << 29)
    ring &= ~blk
    x[0] = (x[0] & ~ring & ~blk) | blk               # contained at once (still life)
    x[2] = np.zeros(64, np.uint64)
    x[2][20] = np.uint64(0b111 << 30)                 # no block
    w = _to_split(np.stack([blk] * 4))
    m = _to_split(np.stack([blk | ring] * 4))
    for gens in (1, 4, 9):
        got, hits = g.simulate_contains(_to_split(x), w, m, gens, lean)
        s, exp = x.copy(), [0] * 4
        for k in range(1, gens + 1):
            s = port.step_batch(s, 1)
            for u in range(4):
                if not exp[u] and (((s[u] ^ blk) & (blk | ring)) == 0).all():
                    exp[u] = k
        assert (got == _to_split(s)).all() and hits == exp, (gens, hits, exp)


def _rot_rows(states, k):
    """rotate every column word down by k rows (row k becomes row 0)"""
    k %= 64
    s = np.asarray(states, dtype=np.uint64)
    if k == 0:
        return s.copy()
    return (s >> np.uint64(k)) | (s << np.uint64(64 - k))


@pytest.mark.parametrize("late", [False, True])
@pytest.mark.parametrize("h", range(1, 9))
def test_simulated_windowed_contains(port, h, late):
    """split_contains_asm_lean_h<h>: with the universes and the target rotated
    so that the target's care rows lie in rows 0..h-1 (residues 0..h-1 of the
    8-way split), differencing only registers 0..h-1 gives the same first-hit
    generations as the full test on the unrotated states."""
    rng = np.random.default_rng(100 + h)
    y0 = int(rng.integers(64))
    rows = np.uint64(((((1 << h) - 1) << y0) | (((1 << h) - 1) >> (64 - y0))) & ((1 << 64) - 1))  # rows y0.. (mod 64)
    wanted = np.zeros(64, np.uint64)
    care = np.zeros(64, np.uint64)
    for c in range(20, 26):
        care[c] = rows
        wanted[c] = rows & np.uint64(int(rng.integers(1 << 62)))
    unwanted = care & ~wanted
    x = port.fill(4, seed=300 + h) & port.fill(4, seed=400 + h)
    x[1] = (x[1] & ~care) | wanted                      # contained at generation 0 ...
    x[3] = wanted.copy()                                # ... and a bare copy of the wanted cells
    gens = 6
    exp, s = [0] * 4, x.copy()
    for k in range(1, gens + 1):
        s = port.step_batch(s, 1)
        for u in range(4):
            if not exp[u] and (((s[u] ^ wanted) & (wanted | unwanted)) == 0).all():
                exp[u] = k
    xr, wr, mr = _rot_rows(x, y0), _rot_rows(wanted, y0), _rot_rows(wanted | unwanted, y0)
    assert (_rot_rows(care, y0) >> np.uint64(h) == 0).all()   # care rows now in 0..h-1
    got, hits = g.simulate_contains(_to_split(xr), _to_split(np.stack([wr] * 4)),
                                    _to_split(np.stack([mr] * 4)), gens, lean=True, h=h, late=late)
    assert hits == exp, (h, y0, hits, exp)
    assert (got == _to_split(_rot_rows(s, y0))).all()


@pytest.mark.parametrize("lay,h", [("high", h) for h in range(1, 9)] + [("low", h) for h in range(1, g.LOW_H + 1)])
def test_simulated_batched_contains(port, h, lay):
    """split_contains_asm_batch_h<h> / _batch_lo (the test batched over eight
    generations: a nibble per generation, one DPP lane OR and one scalar
    test per block, gens % 8 leading single generations; the full and low
    register layouts)
    against the oracle's step-then-Contains loop, for generation counts with
    every remainder and hits at every position of a block."""
    rng = np.random.default_rng(700 + h)
    y0 = int(rng.integers(64))
    rows = np.uint64(((((1 << h) - 1) << y0) | (((1 << h) - 1) >> (64 - y0))) & ((1 << 64) - 1))
    care = np.zeros(64, np.uint64)
    for c in range(30, 33):
        care[c] = rows
    # the target is universe 0's window at generation 13; universes 1 and 2
    # start 5 and 9 generations ahead, so the hits land at different places
    # in a block (and earlier, if the window matches by chance)
    for seed in range(800 + 16 * h, 816 + 16 * h):  # a soup whose window at generation 13 is busy
        base = port.fill(1, seed=seed)[0]
        wanted = port.step_batch(base[None], 13)[0] & care
        if sum(bin(int(v)).count("1") for v in wanted) >= max(2, h):
            break
    unwanted = care & ~wanted
    x = np.stack([base, port.step_batch(base[None], 5)[0], port.step_batch(base[None], 9)[0],
                  port.fill(1, seed=950 + h)[0]])
    xr, wr, mr = _rot_rows(x, y0), _rot_rows(wanted, y0), _rot_rows(wanted | unwanted, y0)
    W, M = _to_split(np.stack([wr] * 4)), _to_split(np.stack([mr] * 4))
    with g.layout(lay):
        for gens in (0, 1, 2, 3, 7, 8, 9, 15, 16, 21):
            exp, s = [0] * 4, x.copy()
            for k in range(1, gens + 1):
                s = port.step_batch(s, 1)
                for u in range(4):
                    if not exp[u] and (((s[u] ^ wanted) & (wanted | unwanted)) == 0).all():
                        exp[u] = k
            got, hits = g.simulate_batch(_to_split(xr), W, M, gens, g.LOW_H if lay == "low" else h)
            assert hits == exp, (h, gens, hits, exp)
            assert (got == _to_split(_rot_rows(s, y0))).all()
        assert len({e for e in exp[:3] if e}) >= 2, exp  # hits at two or more distinct generations


def test_batched_dpp_chain_reaches_lane_63():
    """the six in-place DPP ORs leave the OR of all 64 lanes in lane 63, for
    single-lane words at every lane (the simulator's DPP model: row_shr
    within rows of 16 lanes, row_bcast 15 / 31 into the masked rows)"""
    a = g.ACC_HI
    for lane in range(64):
        v = np.zeros((g.N_VGPR_C, 64), np.uint32)
        v[a, lane] = 1 << (lane % 32)
        for line in g.batch_chain():
            g._dpp(v, line)
        assert v[a, 63] == 1 << (lane % 32), lane


@pytest.mark.parametrize("rows", [0x1111111111111111, 0x8000400020001001, (1 << 64) - 1])
def test_simulated_batched_contains_any_target(port, rows):
    """split_contains_asm_batch_h8 on targets with no row window (care rows
    every fourth row, five scattered rows, every row): each generation's OR
    of differences folded onto a nibble before the block's lane OR; against
    the oracle's step-then-Contains loop at every remainder of 8"""
    care = np.zeros(64, np.uint64)
    for c in (3, 17, 40, 63):
        care[c] = np.uint64(rows)
    base = port.fill(1, seed=4242)[0]
    wanted = port.step_batch(base[None], 11)[0] & care
    unwanted = care & ~wanted
    x = np.stack([base, port.step_batch(base[None], 3)[0], port.step_batch(base[None], 8)[0],
                  port.fill(1, seed=4343)[0]])
    W, M = _to_split(np.stack([wanted] * 4)), _to_split(np.stack([wanted | unwanted] * 4))
    for gens in (0, 1, 5, 8, 9, 11, 16, 19):
        exp, s = [0] * 4, x.copy()
        for k in range(1, gens + 1):
            s = port.step_batch(s, 1)
            for u in range(4):
                if not exp[u] and (((s[u] ^ wanted) & (wanted | unwanted)) == 0).all():
                    exp[u] = k
        got, hits = g.simulate_batch(_to_split(x), W, M, gens, g.S)
        assert hits == exp, (hex(rows), gens, hits, exp)
        assert (got == _to_split(s)).all()
    assert exp[0] == 11 and exp[1] == 8 and exp[2] == 3, exp
