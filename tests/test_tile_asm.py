"""The generated tile-layout generation loop (tools/tune/tile_asm.inc,
tools/gen_tile_asm.py) on CPU: the committed file is what the generator
emits, no VALU reads two sources from one VGPR bank, and executing the
assembly text on 64 simulated lanes steps 16 universes exactly as the oracle
does (the register layout is Split<8>'s: register j, bit 4k + u = universe u,
row 8k + j; lane i of group g owns columns 4(i mod 16) .. +3 of universes
4g .. 4g+3)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_tile_asm as G  # noqa: E402


def test_generated_file_is_current():
    assert open(G.OUT).read() == G.emit()


def test_no_bank_conflicts_and_no_temp_leak():
    prog, gen = G.program()
    G.check_banks(prog)
    n_valu = sum(o[0] in ("bitop3", "alignbit") for o in gen)
    assert n_valu == 288 + 16


def to_regs(univ):
    """16 universes (uint64[16, 64]) -> regs[32, 64] in the tile layout"""
    regs = np.zeros((G.N_VGPR, 64), np.uint32)
    for lane in range(64):
        g, li = divmod(lane, 16)
        for c in range(4):
            x = 4 * li + c
            for j in range(8):
                w = 0
                for k in range(8):
                    for u in range(4):
                        w |= ((int(univ[4 * g + u, x]) >> (8 * k + j)) & 1) << (4 * k + u)
                regs[G.ST(c, j), lane] = w
    return regs


def from_regs(regs):
    univ = np.zeros((16, 64), np.uint64)
    for lane in range(64):
        g, li = divmod(lane, 16)
        for c in range(4):
            x = 4 * li + c
            for u in range(4):
                col = 0
                for j in range(8):
                    w = int(regs[G.ST(c, j), lane])
                    for k in range(8):
                        col |= ((w >> (4 * k + u)) & 1) << (8 * k + j)
                univ[4 * g + u, x] = np.uint64(col)
    return univ


@pytest.mark.parametrize("gens", [0, 1, 2, 3, 4])
def test_simulated_asm_matches_oracle(port, gens):
    x = port.fill(16, seed=77 + gens)
    x[0] = 0
    x[0][0] = x[0][63] = x[0][1] = np.uint64(0x8000000000000003)  # seam cells
    regs = to_regs(x)
    lanes = np.arange(64)
    grp = lanes & ~15
    regs[G.A_SELF] = lanes * 16
    regs[G.A_PREV] = (grp | ((lanes + 15) & 15)) * 16
    regs[G.A_NEXT] = (grp | ((lanes + 1) & 15)) * 16
    lds = np.zeros(4 * G.PLANE, np.uint8)
    body = G.parse_program(open(G.OUT).read())
    G.simulate(body, regs, lds, gens)
    got = from_regs(regs)
    want = port.step_batch(x, gens)
    assert (got == want).all()
