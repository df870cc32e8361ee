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
