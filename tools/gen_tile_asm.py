#!/usr/bin/env python3
"""Generate the hand-allocated generation loop of the tile layout (RULE 8 with
LIFEAPI_XCHG_ASM: 8-way row split, 4 columns per lane, LDS edge exchange) as
inline gfx950 assembly: tools/tune/tile_asm.inc (tuning build only).

Why: a v_bitop3_b32 whose sources sit in two or three VGPRs of one bank (bank =
vN mod 4) issues at about half rate on gfx950 (tools/ab/bank_probe.hip:
1.8 vs 1.0 ns per instruction per SIMD), and the compiler's allocation of the
tile loop puts 60 % of its VALU in that case (tools/vbank.py).  Here every
instruction reads distinct banks by construction:

  state   column c, row-register j  -> bank (c + j) mod 4, so a horizontal
          triple (c-1, c, c+1) always spans three banks; the exchanged edge
          columns play columns -1 and 4
  h0/h1   of row-register j          -> bank j mod 4 (vertical triples j-1, j, j+1)
  tail    s0 a+1, s1 a+2, s2 a+1, s3 a+3, t1 a+3, t2 a    (a = bank of the centre)

The network is RULE 3's (device.hpp kLe1 .. kT3) exactly as gen_tile computes it
(split_layout.hpp).  `simulate()` executes the generated text on numpy lanes;
tests/test_tile_asm.py checks it against the oracle on CPU.

Usage: python tools/gen_tile_asm.py [--check]   (--check: fail if the .inc differs)
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "tune", "tile_asm.inc")

S, C, P = 8, 4, 4            # row split, columns per lane, universes per group
XOR3, MAJ, LE1, NAE, EVEN = 0x96, 0xE8, 0x17, 0x7E, 0x69
T1, T2, T3 = 0x34, 0x58, 0x28
PLANE = 1024                 # bytes of one 16-B-per-lane LDS plane


def col_map(c, base):
    """register of row-register j of a column-c register set at `base`
    (base = 0 mod 4): bank (c + j) mod 4; the tuples v[base..+3], v[base+4..+7]
    hold rows (c, c+1, c+2, c+3 mod 4) + 4 * (tuple index)"""
    return lambda j: base + ((j + c) % 4) + 4 * (j >> 2)


def ST(c, j):  # state register of column c at entry / exit of the asm block
    return col_map(c, 8 * c)(j)


E0, E3 = col_map(0, 32), col_map(3, 40)   # new edge columns (ping-pong with ST 0 / 3)
LV = col_map(3, 48)  # left edge: column 3 of lane i-1 ("column -1", bank (j+3) % 4)
RV = col_map(0, 56)  # right edge: column 0 of lane i+1 ("column 4", bank j % 4)
H_SLOTS = (64, 80)   # h0 at base + j, h1 at base + 8 + j
TEMPS = list(range(96, 120))  # 6 per bank
A_SELF, A_PREV, A_NEXT = 120, 121, 122
N_VGPR = 123


class Alloc:
    """Temps by bank; a register is free again after the last read of its value."""

    def __init__(self):
        self.free = {b: [r for r in TEMPS if r % 4 == b] for b in range(4)}

    def get(self, bank):
        return self.free[bank % 4].pop(0)

    def put(self, r):
        self.free[r % 4].append(r)


def hcol(c, cols, slot):
    """h0/h1 of column c (register maps `cols`, LV/RV at the ends) into `slot`"""
    base = H_SLOTS[slot]
    ops = []
    for j in range(S):
        L = LV(j) if c == 0 else cols[c - 1](j)
        R = RV(j) if c == C - 1 else cols[c + 1](j)
        a = cols[c](j)
        ops.append(("bitop3", base + j, (L, a, R), XOR3))
        ops.append(("bitop3", base + 8 + j, (L, a, R), MAJ))
    return ops


def out_col(c, a_reg, dst, slot, al: Alloc):
    """the rule tail of column c from H slot `slot`: centre a_reg(j), result
    to dst(j) (dst may be a_reg: a is dead after t2).  Temps from `al`."""
    base = H_SLOTS[slot]
    h0 = [base + j for j in range(S)]
    h1 = [base + 8 + j for j in range(S)]
    ops = []
    h0u, h1u = al.get(2), al.get(3)  # beside banks 0, 1 (row 0)
    ops.append(("alignbit", h0u, (h0[S - 1], h0[S - 1]), 32 - P))
    ops.append(("alignbit", h1u, (h1[S - 1], h1[S - 1]), 32 - P))
    h0d = h1d = None
    for pair in ((0, 1), (2, 3), (4, 5), (6, 7)):
        if pair[1] == S - 1:
            h0d, h1d = al.get(0), al.get(1)  # beside banks 2, 3 (row 7)
            ops.append(("alignbit", h0d, (h0[0], h0[0]), P))
            ops.append(("alignbit", h1d, (h1[0], h1[0]), P))
        s = {}
        for j in pair:
            a = (c + j) % 4
            x0 = h0u if j == 0 else h0[j - 1]
            z0 = h0d if j == S - 1 else h0[j + 1]
            x1 = h1u if j == 0 else h1[j - 1]
            z1 = h1d if j == S - 1 else h1[j + 1]
            s0, s1, s2, s3 = al.get(a + 1), al.get(a + 2), al.get(a + 1), al.get(a + 3)
            s[j] = (s0, s1, s2, s3)
            ops.append(("bitop3", s0, (x0, h0[j], z0), LE1))
            ops.append(("bitop3", s1, (x0, h0[j], z0), NAE))
            ops.append(("bitop3", s2, (x1, h1[j], z1), LE1))
            ops.append(("bitop3", s3, (x1, h1[j], z1), EVEN))
        if pair[0] == 0:
            al.put(h0u), al.put(h1u)
        if pair[1] == S - 1:
            al.put(h0d), al.put(h1d)
        t = {}
        for j in pair:
            a = (c + j) % 4
            s0, s1, s2, s3 = s[j]
            t1 = al.get(a + 3)
            ops.append(("bitop3", t1, (s0, s1, a_reg(j)), T1))
            al.put(s0)
            t[j] = t1
        for j in pair:
            a = (c + j) % 4
            s0, s1, s2, s3 = s[j]
            t2 = al.get(a)
            ops.append(("bitop3", t2, (s2, a_reg(j), t[j]), T2))
            al.put(s2), al.put(t[j])
            t[j] = t2
        for j in pair:
            s0, s1, s2, s3 = s[j]
            ops.append(("bitop3", dst(j), (s1, s3, t[j]), T3))
            al.put(s1), al.put(s3), al.put(t[j])
    return ops


def out_col_skew(c, a_reg, dst, slot, al: Alloc):
    """out_col with the rows software-pipelined: step k issues row k's four
    s-functions interleaved with t1 of row k-1, t2 of row k-2 and T3 of row
    k-3, so every dependent pair is about six instructions apart"""
    base = H_SLOTS[slot]
    h0 = [base + j for j in range(S)]
    h1 = [base + 8 + j for j in range(S)]
    ops = []
    h0u, h1u = al.get(2), al.get(3)  # beside banks 0, 1 (row 0)
    ops.append(("alignbit", h0u, (h0[S - 1], h0[S - 1]), 32 - P))
    ops.append(("alignbit", h1u, (h1[S - 1], h1[S - 1]), 32 - P))
    h0d = h1d = None
    sv, t1v, t2v = {}, {}, {}

    def s_op(k, i):
        j = k
        a = (c + j) % 4
        x0 = h0u if j == 0 else h0[j - 1]
        z0 = h0d if j == S - 1 else h0[j + 1]
        x1 = h1u if j == 0 else h1[j - 1]
        z1 = h1d if j == S - 1 else h1[j + 1]
        bank = (a + 1, a + 2, a + 1, a + 3)[i]
        r = al.get(bank)
        sv.setdefault(j, [None] * 4)[i] = r
        src = (x0, h0[j], z0) if i < 2 else (x1, h1[j], z1)
        ops.append(("bitop3", r, src, (LE1, NAE, LE1, EVEN)[i]))

    for k in range(S + 3):
        if k == S - 1:
            h0d, h1d = al.get(0), al.get(1)  # beside banks 2, 3 (row 7)
            ops.append(("alignbit", h0d, (h0[0], h0[0]), P))
            ops.append(("alignbit", h1d, (h1[0], h1[0]), P))
        if k < S:
            s_op(k, 0)
        j = k - 1
        if 0 <= j < S:  # t1 of row k-1
            a = (c + j) % 4
            t1v[j] = al.get(a + 3)
            ops.append(("bitop3", t1v[j], (sv[j][0], sv[j][1], a_reg(j)), T1))
            al.put(sv[j][0])
        if k < S:
            s_op(k, 1)
        j = k - 2
        if 0 <= j < S:  # t2 of row k-2
            a = (c + j) % 4
            t2v[j] = al.get(a)
            ops.append(("bitop3", t2v[j], (sv[j][2], a_reg(j), t1v[j]), T2))
            al.put(sv[j][2]), al.put(t1v[j])
        if k < S:
            s_op(k, 2)
        j = k - 3
        if 0 <= j < S:  # T3 of row k-3
            ops.append(("bitop3", dst(j), (sv[j][1], sv[j][3], t2v[j]), T3))
            al.put(sv[j][1]), al.put(sv[j][3]), al.put(t2v[j])
        if k < S:
            s_op(k, 3)
        if k == 0:
            al.put(h0u), al.put(h1u)
        if k == S - 1:
            al.put(h0d), al.put(h1d)
    return ops


TAIL = out_col_skew


def publish(c0, c3):
    """edge columns to LDS: planes 0/1 = column 0's tuples (rows 0-3 / 4-7),
    planes 2/3 = column 3's tuples (rows 1,2,3,0 / 5,6,7,4)"""
    return [("ds_write", A_SELF, c0(0), 0 * PLANE), ("ds_write", A_SELF, c0(4), 1 * PLANE),
            ("ds_write", A_SELF, c3(1), 2 * PLANE), ("ds_write", A_SELF, c3(5), 3 * PLANE)]


def fetch():
    """lane i-1's column 3 -> LV, lane i+1's column 0 -> RV"""
    return [("ds_read", LV(1), A_PREV, 2 * PLANE), ("ds_read", LV(5), A_PREV, 3 * PLANE),
            ("ds_read", RV(0), A_NEXT, 0 * PLANE), ("ds_read", RV(4), A_NEXT, 1 * PLANE)]


def generation(cols, e0, e3, lds=True):
    """One generation, software-pipelined around the exchange: on entry LV/RV
    hold this generation's edges (reads in flight).  The edge columns are
    computed first into the spare sets e0 / e3 and published, the next
    generation's edges are fetched, and the interior columns (about 150 VALU)
    cover the LDS round trip.  Returns (ops, new column maps)."""
    al = Alloc()
    ops = [("waitcnt",)]
    ops += hcol(0, cols, 0)                     # A: LV, c0, c1
    ops += TAIL(0, cols[0], e0, 0, al)          # new column 0 -> e0 (c0 kept for hcol 1)
    ops += hcol(C - 1, cols, 1)                 # B: c2, c3, RV
    ops += TAIL(C - 1, cols[C - 1], e3, 1, al)
    if lds:
        ops += publish(e0, e3)
        ops += fetch()                          # next generation's edges
    ops += hcol(1, cols, 0)                     # A: c0 (old), c1, c2
    ops += hcol(2, cols, 1)                     # B: c1, c2, c3 (old)
    ops += TAIL(1, cols[1], cols[1], 0, al)     # in place
    ops += TAIL(2, cols[2], cols[2], 1, al)
    assert all(len(v) == len(TEMPS) // 4 for v in al.free.values()), "temp leak"
    return ops, [e0, cols[1], cols[2], e3]


def check_banks(ops):
    for op in ops:
        if op[0] == "bitop3":
            srcs = set(op[2])
            assert len({r % 4 for r in srcs}) == len(srcs), f"bank conflict in {op}"


def render(op):
    k = op[0]
    if k == "bitop3":
        d, (a, b, c), t = op[1], op[2], op[3]
        return f"v_bitop3_b32 v{d}, v{a}, v{b}, v{c} bitop3:0x{t:x}"
    if k == "alignbit":
        d, (a, b), s = op[1], op[2], op[3]
        return f"v_alignbit_b32 v{d}, v{a}, v{b}, {s}"
    if k == "ds_write":
        return f"ds_write_b128 v{op[1]}, v[{op[2]}:{op[2] + 3}] offset:{op[3]}"
    if k == "ds_read":
        return f"ds_read_b128 v[{op[1]}:{op[1] + 3}], v{op[2]} offset:{op[3]}"
    if k == "waitcnt":
        return "s_waitcnt lgkmcnt(0)"
    if k == "mov":
        return f"v_mov_b32 v{op[1]}, v{op[2]}"
    if k == "raw":
        return op[1]
    raise ValueError(op)


def program(lds=True):
    """the whole asm block: prologue (publish, fetch), a loop of generation
    pairs (the spare edge sets swap back after two), an odd generation, and
    the final copy of the edge columns home"""
    cols0 = [col_map(c, 8 * c) for c in range(C)]
    gA, cols1 = generation(cols0, E0, E3, lds)
    gB, cols2 = generation(cols1, cols0[0], cols0[C - 1], lds)
    assert [f(j) for f in cols2 for j in range(S)] == [f(j) for f in cols0 for j in range(S)]
    prog = [("raw", "s_cmp_eq_u32 %[g], 0"), ("raw", "s_cbranch_scc1 4f")]
    prog += publish(cols0[0], cols0[C - 1]) + fetch()
    prog += [("raw", "s_lshr_b32 %[p], %[g], 1"), ("raw", "s_cmp_eq_u32 %[p], 0"),
             ("raw", "s_cbranch_scc1 2f"), ("raw", "1:"), ("raw", "s_sub_u32 %[p], %[p], 1")]
    prog += gA + gB
    prog += [("raw", "s_cmp_lg_u32 %[p], 0"), ("raw", "s_cbranch_scc1 1b"), ("raw", "2:"),
             ("raw", "s_bitcmp1_b32 %[g], 0"), ("raw", "s_cbranch_scc0 3f")]
    prog += gA
    prog += [("mov", cols0[0](j), E0(j)) for j in range(S)]
    prog += [("mov", cols0[C - 1](j), E3(j)) for j in range(S)]
    prog += [("raw", "3:"), ("waitcnt",), ("raw", "4:")]
    return prog, gA


def emit(lds=True, name="tile_gens_asm") -> str:
    prog, gen = program(lds)
    check_banks(prog)
    body = [render(op) for op in prog]
    n_valu = sum(op[0] in ("bitop3", "alignbit") for op in gen)
    state = [f'"+{{v{ST(c, j)}}}"(r[{c}][{j}])' for c in range(C) for j in range(S)]
    clob = [r for r in range(32, N_VGPR) if r not in (A_SELF, A_PREV, A_NEXT)]
    lines = [
        "// tile_asm.inc -- GENERATED by tools/gen_tile_asm.py; do not edit.",
        "// The generation loop of the tile layout (RULE 8, 8-way row split, 4 columns",
        "// per lane, LDS edge exchange) with every VALU source in a distinct VGPR",
        "// bank, software-pipelined around the exchange.",
        f"// {n_valu} VALU + 8 LDS per generation for 16 universes; {N_VGPR} VGPRs pinned.",
        "#pragma once",
        "",
        "namespace lifeapi_impl {",
        "",
        "// r: the tile's state (gen_tile's r[c][j]); a_self / a_prev / a_next: LDS",
        "// byte addresses of this lane's / lane i-1's / lane i+1's 16-B slot in the",
        "// wave's four 1-KiB planes (lanes of the lane's 16-lane group, mod 16)",
        f"__device__ __forceinline__ void {name}(uint32_t (&r)[4][8], uint32_t gens, uint32_t a_self,",
        "                                              uint32_t a_prev, uint32_t a_next) {",
        "  uint32_t pairs;",
        "  asm volatile(",
    ]
    lines += [f'      "{b}\\n"' for b in body]
    lines += [
        "      : " + ",\n        ".join(state) + ",",
        '        [p] "=&s"(pairs)',
        f'      : [g] "s"(gens), "{{v{A_SELF}}}"(a_self), "{{v{A_PREV}}}"(a_prev), "{{v{A_NEXT}}}"(a_next)',
        "      : " + ", ".join(f'"v{r}"' for r in clob) + ', "scc", "memory");',
        "}",
        "",
        "}  // namespace lifeapi_impl",
        "",
    ]
    return "\n".join(lines)


# ---------------------------------------------------------------------------
# simulator of the generated text (64 lanes, numpy) for the CPU tests
# ---------------------------------------------------------------------------

def parse_program(text: str):
    """the instruction lines of the asm block, in order"""
    out = []
    for line in text.split("\n"):
        line = line.strip()
        if line.startswith('"') and line.endswith('\\n"'):
            out.append(line[1:-3].strip())
    return out


def _v(tok):
    return int(tok.strip().lstrip("v").split(":")[0].lstrip("["))


def simulate(prog, regs: np.ndarray, lds: np.ndarray, gens: int):
    """execute the asm block on 64 lanes: regs uint32 [N_VGPR, 64]; lds uint8"""
    sreg = {"%[g]": gens, "%[p]": 0}
    scc = 0
    labels = {ins[:-1]: i for i, ins in enumerate(prog) if ins.endswith(":")}
    pc = 0
    while pc < len(prog):
        ins = prog[pc]
        pc += 1
        if ins.endswith(":"):
            continue
        op, _, rest = ins.partition(" ")
        args = [a.strip() for a in rest.split(",")]
        if op == "v_bitop3_b32":
            d, a, b = _v(args[0]), _v(args[1]), _v(args[2])
            c_tok, t_tok = args[3].split()
            t = int(t_tok.split(":")[1], 16)
            A, B, Cc = regs[a].copy(), regs[b].copy(), regs[_v(c_tok)].copy()
            res = np.zeros(64, np.uint32)
            for idx in range(8):  # minterm idx = (src0, src1, src2) bits
                if (t >> idx) & 1:
                    res |= ((A if idx & 4 else ~A) & (B if idx & 2 else ~B) & (Cc if idx & 1 else ~Cc))
            regs[d] = res
        elif op == "v_alignbit_b32":
            d, a, b, sh = _v(args[0]), _v(args[1]), _v(args[2]), int(args[3])
            wide = (regs[a].astype(np.uint64) << 32) | regs[b].astype(np.uint64)
            regs[d] = ((wide >> np.uint64(sh)) & 0xFFFFFFFF).astype(np.uint32)
        elif op == "v_mov_b32":
            regs[_v(args[0])] = regs[_v(args[1])]
        elif op == "ds_write_b128":
            addr, base = _v(args[0]), _v(args[1].split()[0])
            off = int(args[1].split("offset:")[1])
            for lane in range(64):
                at = int(regs[addr][lane]) + off
                lds[at:at + 16] = np.ascontiguousarray(regs[base:base + 4, lane]).view(np.uint8)
        elif op == "ds_read_b128":
            base = _v(args[0])
            addr, off = _v(args[1].split()[0]), int(args[1].split("offset:")[1])
            vals = np.zeros((4, 64), np.uint32)
            for lane in range(64):
                at = int(regs[addr][lane]) + off
                vals[:, lane] = lds[at:at + 16].view(np.uint32)
            regs[base:base + 4] = vals
        elif op == "s_waitcnt":
            pass
        elif op == "s_cmp_eq_u32":
            scc = int(sreg[args[0]] == int(args[1]))
        elif op == "s_cmp_lg_u32":
            scc = int(sreg[args[0]] != int(args[1]))
        elif op == "s_bitcmp1_b32":
            scc = (sreg[args[0]] >> int(args[1])) & 1
        elif op == "s_lshr_b32":
            sreg[args[0]] = sreg[args[1]] >> int(args[2])
        elif op == "s_sub_u32":
            sreg[args[0]] = sreg[args[1]] - int(args[2])
        elif op in ("s_cbranch_scc0", "s_cbranch_scc1"):
            if scc == (op == "s_cbranch_scc1"):
                pc = labels[args[0][:-1]]
        else:
            raise ValueError(ins)


def main():
    text = emit()
    if "--check" in sys.argv:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        if cur != text:
            sys.exit(f"{OUT} is stale: run python tools/gen_tile_asm.py")
        print("tile_asm.inc up to date")
        return
    with open(OUT, "w") as f:
        f.write(text)
    _, ops = program()
    print(f"wrote {OUT}: {sum(o[0] in ('bitop3', 'alignbit') for o in ops)} VALU, "
          f"{sum(o[0].startswith('ds') for o in ops)} LDS per generation")


if __name__ == "__main__":
    main()
