"""CPU: the generated pair-layout loop (tools/gen_pair_asm.py ->
tools/tune/pair_asm.inc) is up to date and -- run on numpy lanes -- computes
the oracle's Step() for 8 universes (2 groups x 4, two columns per lane)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_pair_asm as g  # noqa: E402
from test_split_asm import _to_split  # noqa: E402


def _pack(x8):
    ga, gb = _to_split(x8[:4]), _to_split(x8[4:])
    a, b = np.zeros((8, 64), np.uint32), np.zeros((8, 64), np.uint32)
    for lane in range(64):
        src, i = (ga if lane < 32 else gb), lane & 31
        a[:, lane], b[:, lane] = src[:, 2 * i], src[:, 2 * i + 1]
    return a, b


def test_inc_is_generated():
    assert open(g.OUT).read() == g.emit()


def test_register_budget_and_banks():
    for v in g.VARIANTS:
        body = g.alt_gen(2, False) if v.startswith("alt") else g.body(v)
        n, bad = g.check_banks(body)
        assert n == 136 and len(bad) == 32, v      # 128 bitop3 + 8 alignbit; the h-layer only
        assert all(ln.split()[-1] in ("bitop3:0x96", "bitop3:0xe8") for ln in bad)
    text = open(g.OUT).read()
    assert max(int(x) for x in __import__("re").findall(r"\bv(\d+)\b", text)) < 62  # + 2 for the kernel: 8 waves per SIMD


@pytest.mark.parametrize("variant", g.VARIANTS)
def test_simulated_loop_is_step(port, variant):
    x = port.fill(8, seed=91)
    x[3] = port.parse("bo$2bo$3o!")          # a glider crossing the seams
    x[6] = np.roll(port.parse("2o$2o!"), 63)
    for gens in (1, 2, 3, 7, 8):
        got = g.simulate(*_pack(x), gens, variant)
        want = _pack(port.step_batch(x, gens))
        assert (got[0] == want[0]).all() and (got[1] == want[1]).all(), (variant, gens)
