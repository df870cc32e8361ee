#!/usr/bin/env python3
"""Generate the hand-allocated generation loop of the PAIR layout: the 8-way
row split with 4 universes interleaved bit by bit per register (as rule 11,
tools/gen_split_asm.py), but each lane holds TWO adjacent columns (2i, 2i+1)
of its group's universes, 32 lanes per group, 2 groups (8 universes) per
wave.  Only a lane's outer columns cross lanes, so per universe-generation
the LDS exchange reads half the bytes of rule 11's (writes are unchanged):

  per wave and generation: write A (column 2i, 8 registers) and B (2i+1),
  read L = B of lane i-1 and R = A of lane i+1 (within the 32-lane group,
  wrapping) -- 4 ds_write_b128 + 4 ds_read_b128 for 8 universes, against
  2 + 4 for rule 11's 4 universes: 6 instead of 8 LDS-array cycles per
  universe-generation.

VALU is unchanged per universe (h-layer 2, 6-LUT tail, 4 ring rotates per
column).  VGPR banks (vN mod 4), as gen_split_asm.py:
  A[j] v0..v7 bank j, B[j] v8..v15 bank j  (the ds_write_b128 tuples)
  L[j] v18..v25 bank j+2, R[j] v26..v33 bank j+2  (ds_read_b128 tuples);
      h1A[j] overwrites L[j], h1B[j] overwrites R[j]
  h0A[j], h0B[j] bank j+1; tail temps g1/g4 j+1, g2 j+2, g3 j+3, g5 j+2
The h-layer (xor3/maj of L, A, B and of A, B, R) keeps one conflict per
instruction (three even-aligned tuples leave two bank classes), like rule 11.

`simulate()` runs the text on numpy lanes; tests/test_pair_asm.py checks it
against the oracle's Step().  Usage: python tools/gen_pair_asm.py [--check]
"""
from __future__ import annotations

import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "tune", "pair_asm.inc")

S, P = 8, 4
XOR3, MAJ, N1, NAE, N4, N6 = 0x96, 0xE8, 0xE9, 0x7E, 0x52, 0xE0

A = list(range(0, 8))
B = list(range(8, 16))
L = list(range(18, 26))
R = list(range(26, 34))
H1A, H1B = L, R                      # h1 overwrites the read buffers
FREE = [16, 17] + list(range(34, 59))
A_SELF, A_PREV, A_NEXT = 59, 60, 61
N_VGPR = 62
# LDS regions (bytes) of one wave: A rows 0-3 / 4-7, B rows 0-3 / 4-7
OFF_A, OFF_B = (0, 1024), (2048, 3072)


class Pool:
    def __init__(self, regs):
        self.free = {b: [r for r in regs if r % 4 == b] for b in range(4)}

    def get(self, bank):
        return self.free[bank % 4].pop(0)

    def put(self, r):
        self.free[r % 4].append(r)


_pool = Pool(FREE)
H0A = [_pool.get(j + 1) for j in range(S)]
H0B = [_pool.get(j + 1) for j in range(S)]
# the ring-rotation registers (rows -1 and 8 of h0 / h1) are taken from the
# temp pool only around rows 0 and 7; their banks are those of h0[-1], h1[-1],
# h0[8], h1[8]
BANK_H0U, BANK_H1U, BANK_H0D, BANK_H1D = 0, 1, 1, 2
TEMPS = [r for b in range(4) for r in _pool.free[b]]


def temps_for(j, al):
    """registers for g1 (also g4), g2, g3, g5 of row j: banks(g1, g2, g3)
    distinct (g4 = N4(g3, g2, g1)) and banks(g1, g5, r[j] = j) distinct
    (next = N6(g4, g5, r)); the default is g1 j+1, g2 j+2, g3 j+3, g5 j+2."""
    import itertools
    prefs = [(j + 1, j + 2, j + 3, j + 2)] + list(itertools.product(range(4), repeat=4))
    for b1, b2, b3, b5 in prefs:
        b1, b2, b3, b5 = b1 % 4, b2 % 4, b3 % 4, b5 % 4
        if len({b1, b2, b3}) < 3 or len({b1, b5, j % 4}) < 3:
            continue
        need = {}
        for b in (b1, b2, b3, b5):
            need[b] = need.get(b, 0) + 1
        if all(len(al.free[b]) >= k for b, k in need.items()):
            return al.get(b1), al.get(b2), al.get(b3), al.get(b5)
    raise RuntimeError(f"no temps for row {j}")


def op(dst, a, b, c, tt):
    return f"v_bitop3_b32 v{dst}, v{a}, v{b}, v{c} bitop3:0x{tt:02x}"


def hlayer(col, js):
    out = []
    for j in js:
        if col == 0:
            out += [op(H0A[j], L[j], A[j], B[j], XOR3), op(H1A[j], L[j], A[j], B[j], MAJ)]
        else:
            out += [op(H0B[j], A[j], B[j], R[j], XOR3), op(H1B[j], A[j], B[j], R[j], MAJ)]
    return out


def tail_ops(j, r, h0, h1, rot, al):
    a0 = rot["h0u"] if j == 0 else h0[j - 1]
    c0 = rot["h0d"] if j == S - 1 else h0[j + 1]
    a1 = rot["h1u"] if j == 0 else h1[j - 1]
    c1 = rot["h1d"] if j == S - 1 else h1[j + 1]
    g1, g2, g3, g5 = temps_for(j, al)
    return [op(g1, h1[j], a1, c1, N1),        # SB in {0,2,3}
            op(g2, c1, a1, c0, MAJ),
            op(g3, c0, a0, h0[j], NAE),       # SA in {1,2}
            op(g5, h0[j], c0, a0, XOR3),      # SA odd
            op(g1, g3, g2, g1, N4),           # g4
            op(r[j], g1, g5, r[j], N6)], (g1, g2, g3, g5)   # next = g4 & (g5 | a)


def tails(col, h1set=None):
    r, h0, h1 = (A, H0A, H1A) if col == 0 else (B, H0B, H1B)
    if h1set is not None:
        h1 = h1set
    al = Pool(TEMPS)
    out = []
    for j in range(0, S, 2):
        rot = {}
        if j == 0:   # rows -1 (rotl P of row 7's h)
            rot["h0u"], rot["h1u"] = al.get(BANK_H0U), al.get(BANK_H1U)
            out += [f"v_alignbit_b32 v{rot['h0u']}, v{h0[S - 1]}, v{h0[S - 1]}, {32 - P}",
                    f"v_alignbit_b32 v{rot['h1u']}, v{h1[S - 1]}, v{h1[S - 1]}, {32 - P}"]
        if j + 1 == S - 1:   # row 8 (rotr P of row 0's h)
            rot["h0d"], rot["h1d"] = al.get(BANK_H0D), al.get(BANK_H1D)
            out += [f"v_alignbit_b32 v{rot['h0d']}, v{h0[0]}, v{h0[0]}, {P}",
                    f"v_alignbit_b32 v{rot['h1d']}, v{h1[0]}, v{h1[0]}, {P}"]
        (x, rx), (y, ry) = tail_ops(j, r, h0, h1, rot, al), tail_ops(j + 1, r, h0, h1, rot, al)
        out += [v for xy in zip(x, y) for v in xy]
        for t in list(rx) + list(ry) + list(rot.values()):
            al.put(t)
    return out


def writes(col):
    regs, offs = (A, OFF_A) if col == 0 else (B, OFF_B)
    return [f"ds_write_b128 v{A_SELF}, v[{regs[4 * k]}:{regs[4 * k] + 3}]" + (f" offset:{offs[k]}" if offs[k] else "")
            for k in range(2)]


def reads(col):
    """col 0: L (B of lane i-1); col 1: R (A of lane i+1)"""
    regs, offs, addr = (L, OFF_B, A_PREV) if col == 0 else (R, OFF_A, A_NEXT)
    return [f"ds_read_b128 v[{regs[4 * k]}:{regs[4 * k] + 3}], v{addr}" + (f" offset:{offs[k]}" if offs[k] else "")
            for k in range(2)]


# schedules: "plain" -- the whole exchange at the top of each generation;
# "pipeA" -- A is published right after its tails (B's tails overlap it);
# "*_prio" -- s_setprio 2 from the arrival of the exchange until A is
# published (as rule 11's default);
# "alt" -- the read buffers X (v18..25) and Y (v26..33) swap roles every
# generation (loop unrolled by two): the column whose tails finish first is
# published at once and the next generation's read of it goes into the
# buffer its h1 just vacated, so each generation's first exchange is in
# flight behind the other column's tails; "alt_prio" adds s_setprio 2 from
# the arrival of the exchange until the next reads are issued.
VARIANTS = ("plain", "pipeA", "pipeA_prio", "plain_prio", "alt", "alt_prio")
X, Y = L, R


def hl(col, lin, js):
    """h-layer of column col with the neighbour column in lin; h1 overwrites lin"""
    out = []
    for j in js:
        if col == 0:
            out += [op(H0A[j], lin[j], A[j], B[j], XOR3), op(lin[j], lin[j], A[j], B[j], MAJ)]
        else:
            out += [op(H0B[j], A[j], B[j], lin[j], XOR3), op(lin[j], A[j], B[j], lin[j], MAJ)]
    return out


def rd(kind, regs):
    """kind "L": B of lane i-1; "R": A of lane i+1"""
    offs, addr = (OFF_B, A_PREV) if kind == "L" else (OFF_A, A_NEXT)
    return [f"ds_read_b128 v[{regs[4 * k]}:{regs[4 * k] + 3}], v{addr}" + (f" offset:{offs[k]}" if offs[k] else "")
            for k in range(2)]


def alt_gen(kind, prio):
    """one generation of the alternating schedule.  kind 2: L data pending in
    X (issued first), R data in Y; kind 1: R data in X first, L data in Y.
    Outstanding at entry, in order: a write pair, the first read pair, a
    write pair, the second read pair."""
    first_col = 0 if kind == 2 else 1          # the column whose neighbour data arrives first
    other = 1 - first_col
    lines = ["s_waitcnt lgkmcnt(5)"]
    if prio:
        lines.append("s_setprio 2")
    lines += hl(first_col, X, range(4)) + ["s_waitcnt lgkmcnt(4)"] + hl(first_col, X, range(4, 8))
    lines += ["s_waitcnt lgkmcnt(1)"] + hl(other, Y, range(4)) + ["s_waitcnt lgkmcnt(0)"] + hl(other, Y, range(4, 8))
    # the first column's tails (h1 in X), publish it, read its next-gen
    # neighbour copy into X; then the other column (h1 in Y) and Y
    lines += tails(first_col, X) + writes(first_col) + rd("R" if first_col == 0 else "L", X)
    if prio:
        lines.append("s_setprio 0")
    lines += tails(other, Y) + writes(other) + rd("L" if first_col == 0 else "R", Y)
    return lines


def alt_prologue():
    # entering kind 2: W_B, L -> X, W_A, R -> Y
    return writes(1) + rd("L", X) + writes(0) + rd("R", Y)


def alt_text(prio):
    return (["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 2f"] + alt_prologue() +
            ["s_lshr_b32 %[p], %[g], 1", "s_cmp_eq_u32 %[p], 0", "s_cbranch_scc1 3f", "1:",
             "s_sub_u32 %[p], %[p], 1"] + alt_gen(2, prio) + alt_gen(1, prio) +
            ["s_cmp_lg_u32 %[p], 0", "s_cbranch_scc1 1b", "3:", "s_bitcmp1_b32 %[g], 0", "s_cbranch_scc0 4f"] +
            alt_gen(2, prio) + ["4:", "s_waitcnt lgkmcnt(0)", "2:"])


def alt_seq(gens, prio):
    """the straight-line instruction sequence alt_text executes for `gens`"""
    if gens == 0:
        return []
    return alt_prologue() + (alt_gen(2, prio) + alt_gen(1, prio)) * (gens // 2) + \
        (alt_gen(2, prio) if gens % 2 else [])


def prologue(variant):
    return writes(0) if variant.startswith("pipeA") else []


def body(variant):
    pipe, prio = variant.startswith("pipeA"), variant.endswith("prio")
    x = ([] if pipe else writes(0)) + writes(1) + reads(0) + reads(1)
    lines = ["s_sub_u32 %[g], %[g], 1"] + x + ["s_waitcnt lgkmcnt(3)"]
    if prio:
        lines.append("s_setprio 2")
    lines += hlayer(0, range(4)) + ["s_waitcnt lgkmcnt(2)"] + hlayer(0, range(4, 8))
    lines += ["s_waitcnt lgkmcnt(1)"] + hlayer(1, range(4)) + ["s_waitcnt lgkmcnt(0)"] + hlayer(1, range(4, 8))
    lines += tails(0)
    if pipe:
        lines += writes(0)
    if prio:
        lines.append("s_setprio 0")
    lines += tails(1)
    return lines


def asm_text(variant):
    if variant.startswith("alt"):
        return alt_text(variant.endswith("prio"))
    return ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 2f"] + prologue(variant) + ["1:"] + body(variant) + \
        ["s_cmp_lg_u32 %[g], 0", "s_cbranch_scc1 1b", "s_waitcnt lgkmcnt(0)", "2:"]


def check_banks(lines):
    n, bad = 0, []
    for ln in lines:
        if not ln.startswith("v_"):
            continue
        n += 1
        srcs = {int(x) for x in re.findall(r"v(\d+)", ln.split(",", 1)[1])}
        banks = [s % 4 for s in srcs]
        if len(banks) != len(set(banks)):
            bad.append(ln)
    return n, bad


def simulate(a, b, gens, variant=VARIANTS[0]):
    """a, b: uint32 [8, 64] (register j, lane) = columns 2i / 2i+1 of lane i's
    group (lanes 0-31 group 0, 32-63 group 1).  Returns (a, b)."""
    v = np.zeros((N_VGPR, 64), np.uint32)
    v[A], v[B] = a, b
    lds = {}
    lane = np.arange(64)
    prev = (lane & 32) | ((lane + 31) & 31)
    nxt = (lane & 32) | ((lane + 1) & 31)
    if variant.startswith("alt"):
        seq = alt_seq(gens, variant.endswith("prio"))
    else:
        seq = prologue(variant) + body(variant) * gens if gens else []
    for ln in seq:
        if ln.startswith("ds_write_b128"):
            off = int(re.search(r"offset:(\d+)", ln)[1]) if "offset" in ln else 0
            base = int(re.search(r"v\[(\d+):", ln)[1])
            lds[off] = v[base:base + 4].copy()
        elif ln.startswith("ds_read_b128"):
            off = int(re.search(r"offset:(\d+)", ln)[1]) if "offset" in ln else 0
            base = int(re.search(r"v\[(\d+):", ln)[1])
            src = int(re.search(r"\], v(\d+)", ln)[1])
            v[base:base + 4] = lds[off][:, prev if src == A_PREV else nxt]
        elif ln.startswith("v_bitop3_b32"):
            d, x, y, z = (int(t) for t in re.findall(r"v(\d+)", ln))
            tt = int(ln.rsplit(":", 1)[1], 16)
            out = np.zeros(64, np.uint32)
            for k in range(8):
                if tt >> k & 1:
                    out |= (v[x] if k & 4 else ~v[x]) & (v[y] if k & 2 else ~v[y]) & (v[z] if k & 1 else ~v[z])
            v[d] = out
        elif ln.startswith("v_alignbit_b32"):
            d, x, y = (int(t) for t in re.findall(r"v(\d+)", ln)[:3])
            sh = int(ln.rsplit(",", 1)[1])
            w = (v[x].astype(np.uint64) << np.uint64(32)) | v[y].astype(np.uint64)
            v[d] = ((w >> np.uint64(sh)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    return v[A].copy(), v[B].copy()


def fn_text(name, variant):
    asm = "\n".join(f'      "{ln}\\n"' for ln in asm_text(variant))
    outs = ",\n".join([f'        "+{{v{A[j]}}}"(a[{j}])' for j in range(S)] +
                      [f'        "+{{v{B[j]}}}"(b[{j}])' for j in range(S)])
    pinned = sorted(set(L + R + H0A + H0B + TEMPS))
    clob = ", ".join(f'"v{x}"' for x in pinned)
    return f"""
// schedule "{variant}" (see tools/gen_pair_asm.py)
__device__ __forceinline__ void {name}(uint32_t (&a)[8], uint32_t (&b)[8], uint32_t gens, uint32_t a_self,
                                       uint32_t a_prev, uint32_t a_next) {{
  uint32_t p;
  asm volatile(
{asm}
      : {outs.strip()},
        [g] "+s"(gens), [p] "=&s"(p)
      : "{{v{A_SELF}}}"(a_self), "{{v{A_PREV}}}"(a_prev), "{{v{A_NEXT}}}"(a_next)
      : {clob}, "scc", "memory");
}}
"""


def emit():
    n, bad = check_banks(body(VARIANTS[0]))
    fns = "".join(fn_text(f"pair_gens_asm_v{k}", v) for k, v in enumerate(VARIANTS))
    return f"""// pair_asm.inc -- GENERATED by tools/gen_pair_asm.py; do not edit.
// The pair-layout generation loop (8-way row split, 4 universes per register,
// two adjacent columns per lane, 32 lanes and 4 universes per group, two
// groups per wave; LDS exchange of the outer columns only; the 6-LUT tail)
// with hand-allocated VGPRs: {n} VALU per generation, {len(bad)} of them
// (the h-layer) with two sources in one bank.  {N_VGPR} VGPRs.
//
// pair_gens_asm_v<k>(a, b, gens, a_self, a_prev, a_next): a / b = columns
// 2i / 2i+1 as gen_split's r[j]; a_self, a_prev, a_next = LDS byte addresses
// of this lane's, lane i-1's and lane i+1's 16-B slot (within the group) in
// the wave's 4 KiB (A rows 0-3, A rows 4-7, B rows 0-3, B rows 4-7).
// Schedules: {", ".join(f"v{k} = {v}" for k, v in enumerate(VARIANTS))}.
#pragma once

namespace lifeapi_impl {{
{fns}
}}  // namespace lifeapi_impl
"""


if __name__ == "__main__":
    text = emit()
    if "--check" in sys.argv:
        sys.exit(0 if open(OUT).read() == text else 1)
    with open(OUT, "w") as f:
        f.write(text)
    n, bad = check_banks(body(VARIANTS[0]))
    print(f"{OUT}: {n} VALU, {len(bad)} with a bank conflict; {len(TEMPS)} temps {TEMPS}")
