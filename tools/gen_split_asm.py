#!/usr/bin/env python3
"""Generate the hand-allocated generation loop of rule 11 (8-way row split, 4
universes per wave interleaved bit by bit, LDS exchange, the 6-LUT tail of
device.hpp's life_tail6) as inline gfx950 assembly:
lifeapi_amd/csrc/split_asm.inc, used by k_step_split with LIFEAPI_XCHG_ASM.

Why: the compiler's allocation of the rule-11 loop puts 30 of its 68 VALU on
two sources in one VGPR bank (bank = vN mod 4, tools/vbank.py), and such a
v_bitop3 issues at about half rate (tools/ab/bank_probe.hip).  16 of them are the
h-layer xor3 / maj(L, r, R), which cannot avoid it: r, L and R all live in
even-aligned b128 tuples (ds_write_b128 / ds_read_b128), so word j sits at the
same position parity in each and only two banks are left for three operands.
The other 52 (the tails and the ring rotates) are conflict-free here:

  r[j]  bank j        (v0..v7, the ds_write_b128 tuples)
  L[j]  bank j + 2    (ds_read_b128 at v[10:13], v[14:17])
  R[j]  bank j        (ds_read_b128 at v[20:23], v[24:27]); h1[j] overwrites R[j]
                      (h1[3] in v51: see H1)
  h0[j] bank j + 1,  h1[j] bank j  (vertical triples j-1, j, j+1 span 3 banks;
        maj(h1[j+1], h1[j-1], h0[j+1]) needs h0's offset odd against h1's)
  tail temps by bank: g1/g4 j+1, g2 j+2, g3 j+3, g5 j+2 (g4, g5 and r[j]
        distinct for the last LUT)

`simulate()` runs the generated text on numpy lanes (LDS exchange = lane
rotate); tests/test_split_asm.py checks it against gen_split's network on
random states and that the bank rules hold.

Usage: python tools/gen_split_asm.py [--check]
"""
from __future__ import annotations

import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "lifeapi_amd", "csrc", "split_asm.inc")

S, P = 8, 4
XOR3, MAJ, N1, NAE, N4, N6 = 0x96, 0xE8, 0xE9, 0x7E, 0x52, 0xE0

R = [j for j in range(8)]                       # r[j]: v0..v7
L = [10 + j for j in range(4)] + [14 + j - 4 for j in range(4, 8)]
RR = [20 + j for j in range(4)] + [24 + j - 4 for j in range(4, 8)]
# h1[j] overwrites R[j], except h1[3]: rows 4..7's tails still read it after
# the next generation's plane-0 reads have refilled v[20:23] (PIPE)
H1 = RR[:3] + [51] + RR[4:]
H0 = [29 + j for j in range(8)]                 # bank j + 1
H0U, H0D, H1U, H1D = 40, 41, 39, 44              # banks 0, 1, 3, 0 (as h0[-1], h0[8], h1[-1], h1[8])
# three per bank: a pair of interleaved tails needs at most three of one bank
TEMPS = [8, 9, 18, 19, 28, 37, 38, 42, 43, 45, 47, 48]
A_SELF, A_PREV, A_NEXT = 46, 49, 50
N_VGPR = 52


class Alloc:
    def __init__(self):
        self.free = {b: [r for r in TEMPS if r % 4 == b] for b in range(4)}

    def get(self, bank):
        return self.free[bank % 4].pop(0)

    def put(self, r):
        self.free[r % 4].append(r)


def op(dst, a, b, c, tt):
    return f"v_bitop3_b32 v{dst}, v{a}, v{b}, v{c} bitop3:0x{tt:02x}"


def tail_ops(j, al: Alloc):
    a0 = H0U if j == 0 else H0[j - 1]
    c0 = H0D if j == S - 1 else H0[j + 1]
    a1 = H1U if j == 0 else H1[j - 1]
    c1 = H1D if j == S - 1 else H1[j + 1]
    g1, g2, g3, g5 = al.get(j + 1), al.get(j + 2), al.get(j + 3), al.get(j + 2)
    ops = [
        op(g1, H1[j], a1, c1, N1),        # SB in {0,2,3}
        op(g2, c1, a1, c0, MAJ),
        op(g3, c0, a0, H0[j], NAE),       # SA in {1,2}
        op(g5, H0[j], c0, a0, XOR3),      # SA odd
        op(g1, g3, g2, g1, N4),           # g4 (in g1's register)
        op(R[j], g1, g5, R[j], N6),       # next = g4 & (g5 | a)
    ]
    return ops, (g1, g2, g3, g5)


# Variants of the loop's schedule (same instructions, different order):
#   "plain"      plane by plane (write, then its two reads) at the top of each
#                generation; lgkmcnt(3) before plane 0's h-layer, as the
#                compiler orders the compiled loop
#   "pipe"       the NEXT generation's exchange is issued inside this one:
#                plane 0 right after rows 0..3's tails, plane 1 at the end
#   "early"      "plain", and rows 1 and 2 (which read only plane-0 h values)
#                run their tails before waiting for plane 1
#   "pipe_prio"  "pipe", with the wave's priority raised (s_setprio 2) from
#                the arrival of its exchange until it has published the next
#                generation's plane 0, so that a wave with data in hand keeps
#                the LDS pipe fed before the others' tails
#   "pipe_prio_e"  "pipe_prio", and raised again for rows 6..7 and the
#                  plane-1 exchange (low only during rows 4..5)
#   "pipe_prio_m"  priority dropped after rows 0..1's tails
#   "pipe_prio1"   "pipe_prio" with s_setprio 1
# v0 (LIFEAPI_XCHG_ASM) is VARIANTS[0]; the others are LIFEAPI_XCHG_ASM_V(k).
# Measured on config 3 (profiles/r01/tune_c3asm_*.jsonl): "plain" 1.349 ms,
# "early" 1.363, "pipe" 1.330-1.373, the compiled loop 1.370-1.392;
# "pipe_prio" 1.287-1.307, dropping the priority right after the h-layer
# 1.361, s_setprio 3 instead of 2 1.320.
VARIANTS = ("pipe_prio", "pipe_prio_e", "pipe_prio_m", "pipe_prio1")
DEFAULT = VARIANTS[0]


def exchange(plane):
    off = " offset:1024" if plane else ""
    lo = 4 * plane
    return [f"ds_write_b128 v{A_SELF}, v[{lo}:{lo + 3}]{off}",
            f"ds_read_b128 v[{L[lo]}:{L[lo] + 3}], v{A_PREV}{off}",
            f"ds_read_b128 v[{RR[lo]}:{RR[lo] + 3}], v{A_NEXT}{off}"]


def prologue(variant=DEFAULT):
    return exchange(0) + exchange(1) if variant.startswith("pipe") else []


def body(variant=DEFAULT):
    pipe, early = variant.startswith("pipe"), variant.endswith("early")
    prio = 3 if variant.endswith("prio3") else 1 if variant.endswith("prio1") else 2 if "prio" in variant else 0
    drop_after_h = variant.endswith("prio_h")
    again, mid = variant.endswith("prio_e"), variant.endswith("prio_m")
    lines = [] if pipe else exchange(0) + exchange(1)
    lines += ["s_sub_u32 %[g], %[g], 1", "s_waitcnt lgkmcnt(3)"]
    if prio:
        lines.append(f"s_setprio {prio}")

    def hlayer(js):
        out = []
        for j in js:
            out.append(op(H0[j], L[j], R[j], RR[j], XOR3))
            out.append(op(H1[j], L[j], R[j], RR[j], MAJ))
        return out

    rot_d = [f"v_alignbit_b32 v{H0D}, v{H0[0]}, v{H0[0]}, {P}",                 # rotr P
             f"v_alignbit_b32 v{H1D}, v{H1[0]}, v{H1[0]}, {P}"]
    rot_u = [f"v_alignbit_b32 v{H0U}, v{H0[S - 1]}, v{H0[S - 1]}, {32 - P}",   # rotl P
             f"v_alignbit_b32 v{H1U}, v{H1[S - 1]}, v{H1[S - 1]}, {32 - P}"]
    al = Alloc()

    def pair(j, k):
        (a, ra), (b, rb) = tail_ops(j, al), tail_ops(k, al)
        out = [x for xy in zip(a, b) for x in xy]
        for r in ra + rb:  # free only after both interleaved rows are emitted
            al.put(r)
        return out

    lines += hlayer(range(4))
    if early:
        lines += rot_d + pair(1, 2) + ["s_waitcnt lgkmcnt(0)"] + hlayer(range(4, 8)) + rot_u + pair(0, 3)
    else:
        lines += ["s_waitcnt lgkmcnt(0)"] + hlayer(range(4, 8)) + rot_u + rot_d
        if drop_after_h:
            lines.append("s_setprio 0")
        lines += pair(0, 1)
        if mid:
            lines.append("s_setprio 0")
        lines += pair(2, 3)
    if pipe:
        lines += exchange(0)   # rows 0..3 are final: publish plane 0
    if prio and not (drop_after_h or mid):
        lines.append("s_setprio 0")
    lines += pair(4, 5)
    if again:
        lines.append(f"s_setprio {prio}")
    lines += pair(6, 7)
    if pipe:
        lines += exchange(1)
    return lines


# ---- two groups per wave (G = 2): each group's exchange hides behind the
# other group's h-layer and tails; 8 more universes per wave in flight.
RB_REGS = list(range(56, 64))                    # group B's r[j]: bank j
LB2 = [66 + j for j in range(4)] + [70 + j - 4 for j in range(4, 8)]    # bank j + 2
RRB2 = [76 + j for j in range(4)] + [80 + j - 4 for j in range(4, 8)]   # bank j
N_VGPR2 = 84


def exchange2(grp, plane):
    off = 2048 * grp + 1024 * plane
    o = f" offset:{off}" if off else ""
    r = R if grp == 0 else RB_REGS
    l = L if grp == 0 else LB2
    rr = RR if grp == 0 else RRB2
    lo = 4 * plane
    return [f"ds_write_b128 v{A_SELF}, v[{r[lo]}:{r[lo] + 3}]{o}",
            f"ds_read_b128 v[{l[lo]}:{l[lo] + 3}], v{A_PREV}{o}",
            f"ds_read_b128 v[{rr[lo]}:{rr[lo] + 3}], v{A_NEXT}{o}"]


def group_gen(grp):
    """one generation of group grp (its exchange already landed)"""
    r = R if grp == 0 else RB_REGS
    l = L if grp == 0 else LB2
    rr = RR if grp == 0 else RRB2
    h1 = rr                                      # h1[j] overwrites R[j]
    lines = []
    for j in range(S):
        lines.append(op(H0[j], l[j], r[j], rr[j], XOR3))
        lines.append(op(h1[j], l[j], r[j], rr[j], MAJ))
    lines += [
        f"v_alignbit_b32 v{H0U}, v{H0[S - 1]}, v{H0[S - 1]}, {32 - P}",
        f"v_alignbit_b32 v{H1U}, v{h1[S - 1]}, v{h1[S - 1]}, {32 - P}",
        f"v_alignbit_b32 v{H0D}, v{H0[0]}, v{H0[0]}, {P}",
        f"v_alignbit_b32 v{H1D}, v{h1[0]}, v{h1[0]}, {P}",
    ]
    al = Alloc()

    def tail(j):
        a0 = H0U if j == 0 else H0[j - 1]
        c0 = H0D if j == S - 1 else H0[j + 1]
        a1 = H1U if j == 0 else h1[j - 1]
        c1 = H1D if j == S - 1 else h1[j + 1]
        g1, g2, g3, g5 = al.get(j + 1), al.get(j + 2), al.get(j + 3), al.get(j + 2)
        return [op(g1, h1[j], a1, c1, N1), op(g2, c1, a1, c0, MAJ), op(g3, c0, a0, H0[j], NAE),
                op(g5, H0[j], c0, a0, XOR3), op(g1, g3, g2, g1, N4), op(r[j], g1, g5, r[j], N6)], \
            (g1, g2, g3, g5)

    for j in range(0, S, 2):
        (a, ra), (b, rb) = tail(j), tail(j + 1)
        for x, y in zip(a, b):
            lines += [x, y]
        for x in ra + rb:
            al.put(x)
    return lines


def prologue2():
    return exchange2(0, 0) + exchange2(0, 1) + exchange2(1, 0) + exchange2(1, 1)


def body2():
    # in order: A's 6 LDS ops, then B's 6 are outstanding at the top
    lines = ["s_sub_u32 %[g], %[g], 1", "s_waitcnt lgkmcnt(6)"] + group_gen(0) + \
        exchange2(0, 0) + exchange2(0, 1) + ["s_waitcnt lgkmcnt(6)"] + group_gen(1) + \
        exchange2(1, 0) + exchange2(1, 1)
    return lines


def emit2():
    lines = ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 2f"] + prologue2() + ["1:"] + body2() + \
        ["s_cmp_lg_u32 %[g], 0", "s_cbranch_scc1 1b", "s_waitcnt lgkmcnt(0)", "2:"]
    asm = "\n".join(f'      "{l}\\n"' for l in lines)
    outs = ",\n".join([f'        "+{{v{R[j]}}}"(a[{j}])' for j in range(S)] +
                      [f'        "+{{v{RB_REGS[j]}}}"(b[{j}])' for j in range(S)])
    pinned = sorted({x for x in L + RR + LB2 + RRB2 + H0 + [H0U, H0D, H1U, H1D] + TEMPS})
    clob = ", ".join(f'"v{x}"' for x in pinned)
    return f"""
// Two groups per wave (G = 2): a / b are the groups' r[j]; group b's planes
// sit 2 KiB after group a's.  Each group's exchange is in flight while the
// other group's generation runs.  {N_VGPR2} VGPRs pinned.
__device__ __forceinline__ void split_gens_asm2(uint32_t (&a)[8], uint32_t (&b)[8], uint32_t gens,
                                                uint32_t a_self, uint32_t a_prev, uint32_t a_next) {{
  asm volatile(
{asm}
      : {outs.strip()},
        [g] "+s"(gens)
      : "{{v{A_SELF}}}"(a_self), "{{v{A_PREV}}}"(a_prev), "{{v{A_NEXT}}}"(a_next)
      : {clob}, "scc", "memory");
}}
"""


# ---- fused Step + Contains(LifeTarget) on the same loop (k_step_contains_split):
# after each generation, d = OR_j (r_j ^ w_j) & m_j (m = wanted | unwanted,
# LifeTarget.hpp:44-51), one ballot per universe (its bits are every 4th),
# and the first generation with an empty ballot is kept per universe in SGPRs.
W_REGS = [53, 54, 55, 56, 57, 58, 59, 60]        # w_j: bank j + 1
M_REGS = [62, 63, 52, 61, 66, 67, 64, 65]        # m_j: bank j + 2
N_VGPR_C = 68
# the "low" layout for targets of at most 4 rows: w_0..3 / m_0..3 in v52..v59
# (same banks) and the batched test's block word in v60, so that the
# kernel's VGPR count, and with it the waves per SIMD, stays at the plain
# step's 8 (at most 64 VGPRs) instead of 5 (87 VGPRs with all eight rows)
W_LO = [53, 54, 55, 56]
M_LO = [58, 59, 52, 57]
LOW_H = 4
DIFF = 0x28        # (r ^ w) & m
OR3 = 0xFE         # a | b | c
ORAND = 0xA8       # (a | b) & c


def _or_to_two(d, al):
    """OR-reduce the difference registers d to two values (y, z) with
    y | z = OR(d), in as few OR3 as possible; (lines, y, z)"""
    h = len(d)
    if h == 1:
        return [], d[0], d[0]
    if h == 2:
        return [], d[0], d[1]
    x = al.get(1)
    lines = [op(x, d[0], d[1], d[2], OR3)]
    if h == 3:
        return lines, x, x
    if h == 4:
        return lines, x, d[3]
    y = al.get(2)
    if h == 5:
        return lines + [op(y, d[3], d[4], d[4], OR3)], x, y
    lines.append(op(y, d[3], d[4], d[5], OR3))
    if h == 6:
        return lines, x, y
    z = al.get(3)
    if h == 7:
        return lines + [op(z, d[6], x, x, OR3)], y, z
    return lines + [op(z, d[6], d[7], x, OR3)], y, z


_LAYOUT = {"name": "high"}


def _wm():
    return {"low": (W_LO, M_LO), "high": (W_REGS, M_REGS)}[_LAYOUT["name"]]


class layout:
    """with layout(name): the generators use register layout name ("high",
    "low"; True / False = "low" / "high")"""
    def __init__(self, name):
        self.name = {True: "low", False: "high"}.get(name, name)

    def __enter__(self):
        self.prev, _LAYOUT["name"] = _LAYOUT["name"], self.name

    def __exit__(self, *a):
        _LAYOUT["name"] = self.prev


def contains_check(lean=False, h=S):
    """lean: the per-universe bookkeeping on the fast path is 2 SALU per
    universe (s_cmp_eq_u64 + s_addc_u32 building the clean mask, universe 0
    in bit 3) and one s_andn2 + branch; a hit (rare) branches to a slow path
    that records it.  Otherwise 8 SALU per universe per generation.
    h < 8 (lean only): the target's care rows all lie in residues 0..h-1 of
    the 8-way split (the kernel rotates universes and target so), so only
    registers 0..h-1 are differenced."""
    al = Alloc()
    d = []
    for j in range(h):
        t = al.get(j)
        d.append(t)
    wr, mr = _wm()
    lines = [op(d[j], R[j], wr[j], mr[j], DIFF) for j in range(h)]
    if lean:
        red, y, z = _or_to_two(d, al)
        lines += red
        for t in set(d) - {y, z}:  # consumed: the masked ORs may reuse them
            al.put(t)
        lines.append("s_add_u32 %[gc], %[gc], 1")
        ts = [al.get(b) for b in range(P)]
        for u in range(P):
            lines += [f"v_bitop3_b32 v{ts[u]}, v{y}, v{z}, %[m{u}] bitop3:0x{ORAND:02x}",
                      f"v_cmp_ne_u32_e64 %[cmp{u}], 0, v{ts[u]}"]
        return lines + contains_salu()
    assert h == S
    x, y = al.get(1), al.get(2)
    z = al.get(3)
    lines += [op(x, d[0], d[1], d[2], OR3), op(y, d[3], d[4], d[5], OR3), op(z, d[6], d[7], x, OR3)]
    t = al.get(0)
    lines.append("s_add_u32 %[gc], %[gc], 1")
    for u in range(P):
        lines += [f"v_bitop3_b32 v{t}, v{y}, v{z}, %[m{u}] bitop3:0x{ORAND:02x}",
                  f"v_cmp_ne_u32_e64 %[cmp], 0, v{t}",
                  "s_cmp_eq_u64 %[cmp], 0",                 # SCC = universe u clean
                  f"s_cselect_b32 %[c], {1 << u}, 0",
                  "s_andn2_b32 %[c], %[c], %[found]",      # fresh hit
                  "s_cmp_lg_u32 %[c], 0",
                  f"s_cselect_b32 %[h{u}], %[gc], %[h{u}]",
                  "s_or_b32 %[found], %[found], %[c]"]
    return lines


def contains_salu():
    """the lean check's scalar part: the clean mask from the four compares
    (universe 0 in bit 3), fresh hits, and the branch to the slow path"""
    lines = ["s_mov_b32 %[c], 0"]
    for u in range(P):
        lines += [f"s_cmp_eq_u64 %[cmp{u}], 0",       # SCC = universe u clean
                  "s_addc_u32 %[c], %[c], %[c]"]      # c = 2c + SCC
    return lines + ["s_andn2_b32 %[c], %[c], %[found]",     # fresh hits; SCC = any
                    "s_cbranch_scc1 3f",
                    "4:"]


def contains_slowpath():
    """the lean check's hit handler, placed after the loop: record gc for
    every fresh universe (bit 3 - u of c) and jump back"""
    lines = ["3:", "s_or_b32 %[found], %[found], %[c]"]
    for u in range(P):
        lines += [f"s_bitcmp1_b32 %[c], {P - 1 - u}",
                  f"s_cselect_b32 %[h{u}], %[gc], %[h{u}]"]
    return lines + ["s_branch 4b"]


def contains_body(lean=False, h=S, late=False):
    """the default schedule's body with the check after rows 6..7 (all eight
    rows final), before the plane-1 exchange; late (lean only): the check's
    scalar part after that exchange, so the compares' results have landed
    in their SGPRs when the SALU reads them"""
    b = body(DEFAULT)
    k = b.index(exchange(1)[0])
    chk = contains_check(lean, h)
    if not late:
        return b[:k] + chk + b[k:]
    sal = contains_salu()
    assert chk[-len(sal):] == sal
    return b[:k] + chk[:-len(sal)] + b[k:] + sal


def contains_text(lean=False, h=S, late=False):
    lines = ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 2f"] + prologue(DEFAULT) + ["1:"] + \
        contains_body(lean, h, late) + \
        ["s_cmp_lg_u32 %[g], 0", "s_cbranch_scc1 1b", "s_waitcnt lgkmcnt(0)"]
    if lean:
        lines += ["s_branch 2f"] + contains_slowpath()
    return lines + ["2:"]


def emit_contains(lean=False, h=S, late=False):
    low = _LAYOUT["name"] == "low"
    wr, mr = _wm()
    lines = contains_text(lean, h, late)
    asm = "\n".join(f'      "{l}\\n"' for l in lines)
    outs = ",\n".join([f'        "+{{v{R[j]}}}"(r[{j}])' for j in range(S)] +
                      [f'        [h{u}] "+s"(hit[{u}])' for u in range(P)])
    nt = h if low else S
    ins = ", ".join([f'"{{v{wr[j]}}}"(w[{j}])' for j in range(nt)] +
                    [f'"{{v{mr[j]}}}"(m[{j}])' for j in range(nt)] +
                    [f'[m{u}] "s"(0x11111111u << {u})' for u in range(P)])
    pinned = sorted({x for x in L + RR + H1 + H0 + [H0U, H0D, H1U, H1D] + TEMPS})
    clob = ", ".join(f'"v{x}"' for x in pinned)
    if lean:
        name = "split_contains_asm_lean" + ("_late" if late else "") + ("_lo" if low else "" if h == S else f"_h{h}")
        cmps = "uint64_t cmp0, cmp1, cmp2, cmp3;"
        cmp_outs = "[cmp0] \"=&s\"(cmp0), [cmp1] \"=&s\"(cmp1), [cmp2] \"=&s\"(cmp2), [cmp3] \"=&s\"(cmp3)"
        doc = ("// The same with the per-universe bookkeeping cut to two SALU per universe on\n"
               "// the fast path (the clean mask built by s_cmp + s_addc; hits branch to a\n"
               "// slow path after the loop)" +
               ("." if h == S else f", differencing only registers 0..{h - 1} (a target whose\n"
                f"// care rows the kernel has rotated into residues 0..{h - 1})."))
    else:
        name, cmps = "split_contains_asm", "uint64_t cmp;"
        cmp_outs = "[cmp] \"=&s\"(cmp)"
        doc = ("// Fused Step + Contains on the default schedule: after every generation the\n"
               "// containment test of all four universes (hit[u] = first generation whose\n"
               "// state contains the target, 0 = none yet).  w / m: the target's wanted and\n"
               f"// wanted | unwanted planes in the same register layout.  {N_VGPR_C} VGPRs pinned.")
    return f"""
{doc}
__device__ __forceinline__ void {name}(uint32_t (&r)[8], const uint32_t (&w)[8],
                                   const uint32_t (&m)[8], uint32_t gens, uint32_t a_self,
                                   uint32_t a_prev, uint32_t a_next, uint32_t (&hit)[4]) {{
  uint32_t gc = 0, found = 0, c;
  {cmps}
  asm volatile(
{asm}
      : {outs.strip()},
        [g] "+s"(gens), [gc] "+s"(gc), [found] "+s"(found), [c] "=&s"(c), {cmp_outs}
      : "{{v{A_SELF}}}"(a_self), "{{v{A_PREV}}}"(a_prev), "{{v{A_NEXT}}}"(a_next),
        {ins}
      : {clob}, "scc", "memory");
}}
"""


def simulate_contains(r, w, m, gens, lean=False, h=S, late=False):
    """numpy run of split_contains_asm[_lean[_h<h>]]: returns (r, hits[4])"""
    v = np.zeros((72, 64), np.uint32)
    v[:8] = r
    wr, mr = _wm()
    v[wr] = w[:len(wr)]
    v[mr] = m[:len(mr)]
    hits, found = [0] * P, 0
    lds_plane = {}
    seq = prologue(DEFAULT) + (contains_body(lean, h, late) * gens if gens else [])
    gc, c, scc = 0, 0, 0
    cmp = {}
    for l in seq:
        if l.startswith("s_add_u32 %[gc]"):
            gc += 1
        elif l.startswith("v_bitop3_b32") and "%[m" in l:
            d, a, b = (int(x) for x in re.findall(r"v(\d+)", l)[:3])
            u = int(re.search(r"%\[m(\d)\]", l)[1])
            v[d] = (v[a] | v[b]) & np.uint32(0x11111111 << u)
        elif l.startswith("v_cmp_ne_u32_e64"):
            t = int(re.findall(r"v(\d+)", l)[-1])
            key = re.search(r"%\[(cmp\d?)\]", l)[1]
            cmp[key] = int((v[t] != 0).any())
        elif l.startswith("s_cmp_eq_u64"):
            scc = int(cmp[re.search(r"%\[(cmp\d?)\]", l)[1]] == 0)
        elif l.startswith("s_mov_b32 %[c], 0"):
            c = 0
        elif l.startswith("s_addc_u32 %[c]"):
            c = 2 * c + scc
        elif l.startswith("s_cselect_b32 %[c]"):
            bit = int(l.split(",")[1])
            c = bit if scc else 0
        elif l.startswith("s_andn2_b32 %[c]"):
            c &= ~found
            scc = int(c != 0)
        elif l.startswith("s_cbranch_scc1 3f"):
            if scc:                       # the slow path (contains_slowpath)
                found |= c
                for u in range(P):
                    if c >> (P - 1 - u) & 1:
                        hits[u] = gc
        elif l.startswith("s_cmp_lg_u32 %[c]"):
            scc = int(c != 0)
        elif l.startswith("s_cselect_b32 %[h"):
            u = int(re.search(r"%\[h(\d)\]", l)[1])
            if scc:
                hits[u] = gc
        elif l.startswith("s_or_b32 %[found]"):
            found |= c
        elif l == "4:":
            pass
        else:
            _exec(v, l, lds_plane)
    return v[:8].copy(), hits


# ---- the batched test (split_contains_asm_batch_h<h>, h <= 7): the same
# differences, but the cross-lane part runs once per EIGHT generations.  With
# the target's care rows rotated into rows 0..h-1, every difference register
# is zero outside its bits 0..3 (row j of the four universes), and so is
# their OR x_k; generation k of a block therefore packs into bits 4k..4k+3 of
# one word with a single v_lshl_or_b32 (x_0 is written as is).  The OR of that
# word over the 64 lanes is a DPP chain (row_shr 1/2/4/8, row_bcast 15/31)
# issued inside the next block's first h-layer, so that its two-wait-state
# hazards are filled by independent work, then one v_readlane and one s_nor:
# universe u is clean at generation k iff bit 4k + u is clear in every lane.
# Per wave-generation (h = 4): 4 differences, 2 ORs, 1 shift-OR and 7 / 8
# for the chain = 7.9 VALU against 13, and 3 SALU per block instead of 12 per
# generation.  gens % 8 leading generations run the lean per-generation loop.
# The block word needs one register, free in both layouts: w[7] (h <= 7) or
# v60 (low).
ACC_HI, ACC_LO = 60, 60
# h = 8 (any target: every register differenced, w[7] in v60 taken): the
# block word in v68, one VGPR past the lean loop's 68; each generation's OR
# of differences is folded onto its low nibble first (rotates by 16, 8, 4:
# the universe index, bit & 3, is kept), 6 VALU, then packed as above
ACC_H8 = 68
KB = 8             # generations per block
BATCH_MAX_H = 7
OR2 = 0xFC         # a | b


def _acc(h=None):
    if _LAYOUT["name"] == "high" and h == S:
        return ACC_H8
    return {"low": ACC_LO, "high": ACC_HI}[_LAYOUT["name"]]


def _or_into(d, dst, al):
    """dst = OR of registers d (OR3 tree, the last OR writing dst)"""
    lines, d = [], list(d)
    while len(d) > 3:
        t = al.get(len(lines) + 1)
        lines.append(op(t, d[0], d[1], d[2], OR3))
        d = d[3:] + [t]
    a, b, c = (d + d[-1:] * 2)[:3]
    return lines + [op(dst, a, b, c, OR3)]


def batch_x_full(k, al):
    """batch_x for h = 8: the eight differences OR-ed in place (their
    temps reused), folded onto the low nibble, then packed"""
    acc = _acc(S)
    wr, mr = _wm()
    d = [al.get(j) for j in range(S)]
    lines = [op(d[j], R[j], wr[j], mr[j], DIFF) for j in range(S)]
    x, t = d[6], d[7]
    lines += [op(d[0], d[0], d[1], d[2], OR3), op(d[3], d[3], d[4], d[5], OR3), op(x, d[6], t, d[0], OR3),
              op(x, x, d[3], d[3], OR3)]
    for sh in (16, 8, 4):
        lines += [f"v_alignbit_b32 v{t}, v{x}, v{x}, {sh}", op(x, x, t, t, OR3)]
    if k == 0:
        return lines + [f"v_and_b32 v{acc}, 15, v{x}"]
    return lines + [f"v_and_b32 v{t}, 15, v{x}", f"v_lshl_or_b32 v{acc}, v{t}, {4 * k}, v{acc}"]


def batch_x(h, k, al):
    """generation k of the block: ACC = x_k (k = 0) or ACC |= x_k << 4k,
    x_k = OR_j (r_j ^ w_j) & m_j over the h care registers"""
    if h == S:
        return batch_x_full(k, al)
    acc = _acc()
    wr, mr = _wm()
    if h == 1 and k == 0:
        return [op(acc, R[0], wr[0], mr[0], DIFF)]
    d = [al.get(j) for j in range(h)]
    lines = [op(d[j], R[j], wr[j], mr[j], DIFF) for j in range(h)]
    if k == 0:
        return lines + _or_into(d, acc, al)
    if h == 1:
        return lines + [f"v_lshl_or_b32 v{acc}, v{d[0]}, {4 * k}, v{acc}"]
    x = al.get(3)
    return lines + _or_into(d, x, al) + [f"v_lshl_or_b32 v{acc}, v{x}, {4 * k}, v{acc}"]


def batch_chain(h=None):
    """the lane OR of the block word into lane 63 (six in-place DPP ORs)"""
    a = _acc(h)
    return [f"v_or_b32_dpp v{a}, v{a}, v{a} row_shr:{n} row_mask:0xf bank_mask:0xf" for n in (1, 2, 4, 8)] + \
           [f"v_or_b32_dpp v{a}, v{a}, v{a} row_bcast:15 row_mask:0xa bank_mask:0xf",
            f"v_or_b32_dpp v{a}, v{a}, v{a} row_bcast:31 row_mask:0xc bank_mask:0xf"]


def batch_check(slow, back):
    """the pending block's scalar test: c = generations x universes clean and
    not yet found (nibble k, bit u); any -> the slow path"""
    return ["s_nor_b32 %[c], %[rl], %[fm]",            # SCC = c != 0
            f"s_cbranch_scc1 {slow}f",
            f"{back}:"]


def batch_slowpath(lbl, back):
    """record the first clean generation of every fresh universe: nibble k of
    c is generation gc - 7 + k (gc already counts the pending block)"""
    lines = [f"{lbl}:", f"s_sub_u32 %[gk], %[gc], {KB - 1}"]
    for k in range(KB):
        lines += [f"s_bfe_u32 %[t], %[c], 0x{(4 << 16) | (4 * k):x}",
                  "s_andn2_b32 %[t], %[t], %[fu]",
                  "s_or_b32 %[fu], %[fu], %[t]"]
        for u in range(P):
            lines += [f"s_bitcmp1_b32 %[t], {u}",
                      f"s_cselect_b32 %[h{u}], %[gk], %[h{u}]"]
        lines.append("s_add_u32 %[gk], %[gk], 1")
    return lines + ["s_mul_i32 %[fm], %[fu], 0x11111111", f"s_branch {back}b"]


def batch_block(h):
    """eight generations; the first carries the previous block's lane OR and
    scalar test between its h-layer's VALU"""
    acc = _acc(h)
    out = []
    for k in range(KB):
        b = body(DEFAULT)
        if k:
            b.remove("s_sub_u32 %[g], %[g], 1")
        else:   # the pending chain, two VALU apart (DPP reads a fresh VGPR after 2 wait states)
            chain = batch_chain(h) + [f"v_readlane_b32 %[rl], v{acc}, 63"]
            valu = [i for i, l in enumerate(b) if l.startswith("v_")]
            pos = {valu[2 * i]: c for i, c in enumerate(chain[:6])}
            pos[valu[13]] = chain[6]
            nb = []
            for i, l in enumerate(b):
                if i in pos:
                    nb.append(pos[i])
                nb.append(l)
                if i == valu[15]:
                    nb += batch_check(8, 9)
            b = nb
        ex = b.index(exchange(1)[0])
        chk = batch_x(h, k, Alloc())
        if k == KB - 1:
            chk.append(f"s_add_u32 %[gc], %[gc], {KB}")
        out += b[:ex] + chk + b[ex:]
    return out


def batch_text(h):
    acc = _acc(h)
    assert 1 <= h <= {"low": LOW_H, "high": S}[_LAYOUT["name"]]
    lean = [l.replace("%[g]", "%[rem]") for l in contains_body(True, h)]
    flush = []
    for c in batch_chain(h):
        flush += [c, "s_nop 1"]
    flush += [f"v_readlane_b32 %[rl], v{acc}, 63"] + batch_check(10, 11)
    return (["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 2f"] + prologue(DEFAULT) +
            [f"s_and_b32 %[rem], %[g], {KB - 1}", "s_lshr_b32 %[g], %[g], 3",
             "s_cmp_eq_u32 %[rem], 0", "s_cbranch_scc1 5f", "1:"] + lean +
            ["s_cmp_lg_u32 %[rem], 0", "s_cbranch_scc1 1b",
             "5:", "s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 7f",
             f"v_mov_b32 v{acc}, -1",                   # no pending block
             "s_brev_b32 %[fu], %[found]", "s_lshr_b32 %[fu], %[fu], 28",  # bit 3 - u -> bit u
             "s_mul_i32 %[fm], %[fu], 0x11111111", "6:"] + batch_block(h) +
            ["s_cmp_lg_u32 %[g], 0", "s_cbranch_scc1 6b"] + flush +
            ["7:", "s_waitcnt lgkmcnt(0)", "s_branch 2f"] + contains_slowpath() +
            batch_slowpath(8, 9) + batch_slowpath(10, 11) + ["2:"])


def emit_batch(h):
    lay = _LAYOUT["name"]
    wr, mr = _wm()
    asm = "\n".join(f'      "{l}\\n"' for l in batch_text(h))
    outs = ",\n".join([f'        "+{{v{R[j]}}}"(r[{j}])' for j in range(S)] +
                      [f'        [h{u}] "+s"(hit[{u}])' for u in range(P)])
    nt = h
    ins = ", ".join([f'"{{v{wr[j]}}}"(w[{j}])' for j in range(nt)] +
                    [f'"{{v{mr[j]}}}"(m[{j}])' for j in range(nt)] +
                    [f'[m{u}] "s"(0x11111111u << {u})' for u in range(P)])
    used = set(wr[:nt] + mr[:nt])
    extra = {"low": [ACC_LO], "high": W_REGS + M_REGS + ([ACC_H8] if h == S else [])}[lay]
    pinned = sorted({x for x in L + RR + H1 + H0 + [H0U, H0D, H1U, H1D] + TEMPS + extra} - used)
    clob = ", ".join(f'"v{x}"' for x in pinned)
    name = {"low": "split_contains_asm_batch_lo", "high": f"split_contains_asm_batch_h{h}"}[lay]
    note = {"low": ";\n// the low register layout (any target of at most 4 rows)", "high": ""}[lay]
    return f"""
// The lean test batched over eight generations ({"any target" if h == S else f"rows 0..{h - 1}"}): per block one
// lane OR (DPP) and one scalar test of a word holding a nibble per generation{note}.
__device__ __forceinline__ void {name}(uint32_t (&r)[8], const uint32_t (&w)[8],
                                   const uint32_t (&m)[8], uint32_t gens, uint32_t a_self,
                                   uint32_t a_prev, uint32_t a_next, uint32_t (&hit)[4]) {{
  uint32_t gc = 0, found = 0, c, rem, fu, fm, rl, t, gk;
  uint64_t cmp0, cmp1, cmp2, cmp3;
  asm volatile(
{asm}
      : {outs.strip()},
        [g] "+s"(gens), [gc] "+s"(gc), [found] "+s"(found), [c] "=&s"(c), [rem] "=&s"(rem),
        [fu] "=&s"(fu), [fm] "=&s"(fm), [rl] "=&s"(rl), [t] "=&s"(t), [gk] "=&s"(gk),
        [cmp0] "=&s"(cmp0), [cmp1] "=&s"(cmp1), [cmp2] "=&s"(cmp2), [cmp3] "=&s"(cmp3)
      : "{{v{A_SELF}}}"(a_self), "{{v{A_PREV}}}"(a_prev), "{{v{A_NEXT}}}"(a_next),
        {ins}
      : {clob}, "scc", "memory");
}}
"""


def _dpp(v, l):
    d = int(re.search(r"v_or_b32_dpp v(\d+)", l)[1])
    a, b = (int(x) for x in re.findall(r"v(\d+)", l)[1:3])
    rm = int(re.search(r"row_mask:0x([0-9a-f]+)", l)[1], 16)
    src, ok = np.zeros(64, np.uint32), np.zeros(64, bool)
    lane = np.arange(64)
    if "row_shr" in l:
        n = int(re.search(r"row_shr:(\d+)", l)[1])
        ok = lane % 16 >= n
        src[ok] = v[a][lane[ok] - n]
    else:
        n = int(re.search(r"row_bcast:(\d+)", l)[1])
        ok = lane >= 16 if n == 15 else lane >= 32
        src[ok] = v[a][(lane[ok] // 16) * 16 - 1] if n == 15 else v[a][31]
    ok &= (rm >> (lane // 16)) & 1 == 1
    out = v[d].copy()
    out[ok] = src[ok] | v[b][ok]
    v[d] = out


def simulate_batch(r, w, m, gens, h):
    """numpy run of split_contains_asm_batch_h<h>: returns (r, hits[4])"""
    v = np.zeros((72, 64), np.uint32)
    v[:8] = r
    wr, mr = _wm()
    v[wr[:h]] = w[:h]
    v[mr[:h]] = m[:h]
    text = batch_text(h)
    lbl = {l[:-1]: i for i, l in enumerate(text) if re.fullmatch(r"\d+:", l)}
    sg = {"g": gens, "gc": 0, "found": 0, "hits": [0] * P}
    sgk = {f"m{u}": 0x11111111 << u for u in range(P)}
    scc, lds_plane, pc, steps = 0, {}, 0, 0

    def val(x):
        x = x.strip()
        if x.startswith("%[h"):
            return sg["hits"][int(x[3])]
        if x.startswith("%["):
            k = x[2:-1]
            return sgk[k] if k in sgk else sg[k]
        return int(x, 0) & 0xFFFFFFFF

    def setv(x, y):
        x = x.strip()
        if x.startswith("%[h"):
            sg["hits"][int(x[3])] = y & 0xFFFFFFFF
        else:
            sg[x[2:-1]] = y & 0xFFFFFFFF

    def jump(t):
        n, d = t[:-1], t[-1]
        cands = [i for i, l in enumerate(text) if l == n + ":"]
        return min(i for i in cands if i > pc) if d == "f" else max(i for i in cands if i < pc)

    while pc < len(text):
        l = text[pc]
        steps += 1
        assert steps < 10 ** 7
        npc = pc + 1
        ops = l.split(None, 1)
        mn, args = ops[0], (ops[1].split(",") if len(ops) > 1 else [])
        if re.fullmatch(r"\d+:", l) or mn in ("s_waitcnt", "s_setprio", "s_nop"):
            pass
        elif mn == "s_cbranch_scc1":
            if scc:
                npc = jump(args[0].strip())
        elif mn == "s_branch":
            npc = jump(args[0].strip())
        elif mn == "s_cmp_eq_u32":
            scc = int(val(args[0]) == val(args[1]))
        elif mn == "s_cmp_lg_u32":
            scc = int(val(args[0]) != val(args[1]))
        elif mn == "s_cmp_eq_u64":
            scc = int(sg[args[0].strip()[2:-1]] == 0)
        elif mn in ("s_add_u32", "s_sub_u32", "s_and_b32", "s_lshr_b32", "s_or_b32", "s_andn2_b32", "s_mul_i32",
                    "s_addc_u32", "s_nor_b32"):
            a, b = val(args[1]), val(args[2])
            y = {"s_add_u32": a + b, "s_sub_u32": a - b, "s_and_b32": a & b, "s_lshr_b32": a >> b,
                 "s_or_b32": a | b, "s_andn2_b32": a & ~b, "s_mul_i32": a * b, "s_addc_u32": a + b + scc,
                 "s_nor_b32": ~(a | b)}[mn]
            if mn in ("s_and_b32", "s_lshr_b32", "s_or_b32", "s_andn2_b32", "s_nor_b32"):
                scc = int(y & 0xFFFFFFFF != 0)
            setv(args[0], y)
        elif mn == "s_mov_b32":
            setv(args[0], val(args[1]))
        elif mn == "s_brev_b32":
            setv(args[0], int(f"{val(args[1]):032b}"[::-1], 2))
        elif mn == "s_bfe_u32":
            a, sel = val(args[1]), val(args[2])
            setv(args[0], (a >> (sel & 31)) & ((1 << (sel >> 16)) - 1))
        elif mn == "s_bitcmp1_b32":
            scc = val(args[0]) >> val(args[1]) & 1
        elif mn == "s_cselect_b32":
            setv(args[0], val(args[1]) if scc else val(args[2]))
        elif mn == "v_cmp_ne_u32_e64":
            sg[args[0].strip()[2:-1]] = int((v[int(args[2].strip()[1:])] != 0).any())
        elif mn == "v_bitop3_b32" and "%[" in l:
            d, a, b = (int(x) for x in re.findall(r"v(\d+)", l)[:3])
            c = np.uint32(val(re.search(r"(%\[\w+\])", l)[1]))
            tt = int(l.rsplit(":", 1)[1], 16)
            out = np.zeros(64, np.uint32)
            for k in range(8):
                if tt >> k & 1:
                    out |= (v[a] if k & 4 else ~v[a]) & (v[b] if k & 2 else ~v[b]) & (c if k & 1 else ~c)
            v[d] = out
        elif mn == "v_perm_b32":
            d, s0, s1 = (int(x) for x in re.findall(r"v(\d+)", l)[:3])
            sel = val(args[3])
            src = (v[s0].astype(np.uint64) << np.uint64(32)) | v[s1].astype(np.uint64)
            out = np.zeros(64, np.uint64)
            for i in range(4):
                bsel = sel >> (8 * i) & 0xFF
                assert bsel < 8
                out |= ((src >> np.uint64(8 * bsel)) & np.uint64(0xFF)) << np.uint64(8 * i)
            v[d] = out.astype(np.uint32)
        elif mn == "v_and_b32":
            d, a = int(args[0].strip()[1:]), int(args[2].strip()[1:])
            v[d] = v[a] & np.uint32(int(args[1]))
        elif mn == "v_lshl_or_b32":
            d, a = (int(x) for x in re.findall(r"v(\d+)", l)[:2])
            c = int(re.findall(r"v(\d+)", l)[2])
            v[d] = (v[a] << np.uint32(int(args[2]))) | v[c]
        elif mn == "v_or_b32_dpp":
            _dpp(v, l)
        elif mn == "v_readlane_b32":
            setv(args[0], int(v[int(args[1].strip()[1:])][int(args[2])]))
        elif mn == "v_mov_b32":
            v[int(args[0].strip()[1:])] = np.uint32(val(args[1]))
        else:
            _exec(v, l, lds_plane)
        pc = npc
    return v[:8].copy(), sg["hits"]


def _exec(v, l, lds_plane):
    if l.startswith("ds_write_b128"):
        off = int(re.search(r"offset:(\d+)", l)[1]) if "offset" in l else 0
        base = int(re.search(r"v\[(\d+):", l)[1])
        lds_plane[off] = v[base:base + 4].copy()
    elif l.startswith("ds_read_b128"):
        off = int(re.search(r"offset:(\d+)", l)[1]) if "offset" in l else 0
        base = int(re.search(r"v\[(\d+):", l)[1])
        src = int(re.search(r"v(\d+)(?: offset|$)", l.split(",", 1)[1].strip())[1])
        v[base:base + 4] = np.roll(lds_plane[off], 1 if src == A_PREV else -1, axis=1)
    elif l.startswith("v_bitop3_b32"):
        d, a, b, c = (int(x) for x in re.findall(r"v(\d+)", l))
        tt = int(l.rsplit(":", 1)[1], 16)
        out = np.zeros(64, np.uint32)
        for k in range(8):
            if tt >> k & 1:
                out |= (v[a] if k & 4 else ~v[a]) & (v[b] if k & 2 else ~v[b]) & (v[c] if k & 1 else ~v[c])
        v[d] = out
    elif l.startswith("v_alignbit_b32"):
        d, a, b = (int(x) for x in re.findall(r"v(\d+)", l)[:3])
        sh = int(l.rsplit(",", 1)[1])
        x = (v[a].astype(np.uint64) << np.uint64(32)) | v[b].astype(np.uint64)
        v[d] = ((x >> np.uint64(sh)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def asm_text(variant=DEFAULT):
    return ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 2f"] + prologue(variant) + ["1:"] + body(variant) + \
        ["s_cmp_lg_u32 %[g], 0", "s_cbranch_scc1 1b", "s_waitcnt lgkmcnt(0)", "2:"]


def check_banks(lines):
    """(VALU instructions, those with two sources in one bank)"""
    n, bad = 0, []
    for l in lines:
        if not l.startswith("v_"):
            continue
        n += 1
        srcs = {int(x) for x in re.findall(r"v(\d+)", l.split(",", 1)[1])}
        banks = [s % 4 for s in srcs]
        if len(banks) != len(set(banks)):
            bad.append(l)
    return n, bad


def simulate(r, gens, two=None, variant=DEFAULT):
    """Run the generated loop on numpy: r = uint32 [8, 64] (register j, lane);
    with `two` (a second group), the two-group loop; returns r (and two)."""
    v = np.zeros((max(N_VGPR, N_VGPR2), 64), np.uint32)
    v[:8] = r
    if two is not None:
        v[RB_REGS] = two
        seq = prologue2() + body2() * gens if gens else []
    else:
        seq = prologue(variant) + body(variant) * gens if gens else []
    lds_plane = {}
    for _ in range(1):
        for l in seq:
            if l.startswith("ds_write_b128"):
                off = int(re.search(r"offset:(\d+)", l)[1]) if "offset" in l else 0
                base = int(re.search(r"v\[(\d+):", l)[1])
                lds_plane[off] = v[base:base + 4].copy()
            elif l.startswith("ds_read_b128"):
                off = int(re.search(r"offset:(\d+)", l)[1]) if "offset" in l else 0
                base = int(re.search(r"v\[(\d+):", l)[1])
                src = int(re.search(r"v(\d+)(?: offset|$)", l.split(",", 1)[1].strip())[1])
                shift = 1 if src == A_PREV else -1          # lane i reads lane i-1 / i+1
                v[base:base + 4] = np.roll(lds_plane[off], shift, axis=1)
            elif l.startswith("v_bitop3_b32"):
                d, a, b, c = (int(x) for x in re.findall(r"v(\d+)", l))
                tt = int(l.rsplit(":", 1)[1], 16)
                out = np.zeros(64, np.uint32)
                for k in range(8):
                    if tt >> k & 1:
                        out |= ((v[a] if k & 4 else ~v[a]) & (v[b] if k & 2 else ~v[b]) &
                                (v[c] if k & 1 else ~v[c]))
                v[d] = out
            elif l.startswith("v_alignbit_b32"):
                d, a, b = (int(x) for x in re.findall(r"v(\d+)", l)[:3])
                sh = int(l.rsplit(",", 1)[1])
                x = (v[a].astype(np.uint64) << np.uint64(32)) | v[b].astype(np.uint64)
                v[d] = ((x >> np.uint64(sh)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    if two is not None:
        return v[:8].copy(), v[RB_REGS].copy()
    return v[:8].copy()


def fn_text(name, variant):
    asm = "\n".join(f'      "{l}\\n"' for l in asm_text(variant))
    outs = ",\n".join(f'        "+{{v{R[j]}}}"(r[{j}])' for j in range(S))
    pinned = sorted({x for x in L + RR + H1 + H0 + [H0U, H0D, H1U, H1D] + TEMPS})
    clob = ", ".join(f'"v{x}"' for x in pinned)
    return f"""
// schedule "{variant}" (see tools/gen_split_asm.py)
__device__ __forceinline__ void {name}(uint32_t (&r)[8], uint32_t gens, uint32_t a_self, uint32_t a_prev,
{" " * (len(name) + 32)}uint32_t a_next) {{
  asm volatile(
{asm}
      : {outs.strip()},
        [g] "+s"(gens)
      : "{{v{A_SELF}}}"(a_self), "{{v{A_PREV}}}"(a_prev), "{{v{A_NEXT}}}"(a_next)
      : {clob}, "scc", "memory");
}}
"""


OUT_TUNE = os.path.join(ROOT, "tools", "tune", "split_asm_tune.inc")

_SIG_LOOP = "(uint32_t (&r)[8], uint32_t gens, uint32_t a_self, uint32_t a_prev, uint32_t a_next)"
_SIG_CONT = ("(uint32_t (&r)[8], const uint32_t (&w)[8], const uint32_t (&m)[8], uint32_t gens, "
             "uint32_t a_self, uint32_t a_prev, uint32_t a_next, uint32_t (&hit)[4])")
_SIG_TWO = "(uint32_t (&a)[8], uint32_t (&b)[8], uint32_t gens, uint32_t a_self, uint32_t a_prev, uint32_t a_next)"


# what the product include defines: the step loop, the full lean test (any
# target), the batched test for windows of 5..7 rows and, in the low layout,
# for windows of at most 4 rows; everything else is the tuning build's
PRODUCT_BATCH_H = range(LOW_H + 1, BATCH_MAX_H + 1)


def _ablation_decls():
    """forward declarations of the tuning build's loops: step_kernels.hpp
    names them in template branches the product never instantiates"""
    names = [(f"split_gens_asm_v{k}", _SIG_LOOP) for k in range(1, len(VARIANTS))]
    names += [("split_gens_asm2", _SIG_TWO), ("split_contains_asm", _SIG_CONT)]
    names += [(f"split_contains_asm_lean_h{h}", _SIG_CONT) for h in range(1, S)]
    names += [("split_contains_asm_lean_late" + ("" if h == S else f"_h{h}"), _SIG_CONT) for h in range(1, S + 1)]
    names += [(f"split_contains_asm_batch_h{h}", _SIG_CONT) for h in range(1, LOW_H + 1)]
    names += [("split_contains_asm_lean_lo", _SIG_CONT)]
    return "".join(f"__device__ __forceinline__ void {n}{sig};\n" for n, sig in names)


def _low_batch():
    with layout("low"):
        return emit_batch(LOW_H)


def emit():
    n, bad = check_banks(body())
    return f"""// split_asm.inc -- GENERATED by tools/gen_split_asm.py; do not edit.
// The generation loop of rule 11 (8-way row split, 4 universes per wave,
// LDS exchange, the 6-LUT tail) with hand-allocated VGPRs: of its {n} VALU
// per generation only the {len(bad)} h-layer ones read two sources from one
// bank (see the generator).  {N_VGPR} VGPRs pinned.
//
// split_gens_asm_v0(r, gens, a_self, a_prev, a_next): r is gen_split's r[j]
// for S = 8; a_self / a_prev / a_next are the LDS byte addresses of this
// lane's / lane i-1's / lane i+1's 16-B slot in the wave's two 1-KiB planes
// (schedule "{VARIANTS[0]}").  The same loop with the fused Contains test
// (k_step_contains_split): split_contains_asm_batch_lo (a target window of at
// most 4 rows, the test batched over eight generations, 61 VGPRs pinned),
// split_contains_asm_batch_h<5..7> (windows of 5..7 rows, 68 pinned) and
// split_contains_asm_lean (any target, per generation, 68 pinned).  The measured
// alternatives (other schedules, two groups per wave, the round-1 contains
// bookkeeping, the per-generation test on narrower windows, a late scalar
// test) are generated into tools/tune/split_asm_tune.inc for the tuning
// build; they are only declared here.
#pragma once

namespace lifeapi_impl {{
{fn_text("split_gens_asm_v0", VARIANTS[0])}{emit_contains(lean=True)}{"".join(emit_batch(h) for h in PRODUCT_BATCH_H)}{_low_batch()}
{_ablation_decls()}
}}  // namespace lifeapi_impl
"""


def _low_lean():
    with layout(True):
        return emit_contains(True, LOW_H)


def emit_tune():
    fns = "".join(fn_text(f"split_gens_asm_v{k}", v) for k, v in enumerate(VARIANTS) if k)
    return f"""// split_asm_tune.inc -- GENERATED by tools/gen_split_asm.py; do not edit.
// The tuning build's variants of the rule-11 assembly loop (see
// lifeapi_amd/csrc/split_asm.inc and the generator): schedules
// {", ".join(f"v{k} = {v}" for k, v in enumerate(VARIANTS) if k)}; two groups per wave
// (split_gens_asm2); the round-1 fused-Contains bookkeeping
// (split_contains_asm); the per-generation lean test on windows of 1..7 rows
// (split_contains_asm_lean_h<h>, and _lo in the low layout), with its scalar
// part late (split_contains_asm_lean_late[_h<h>]); the batched test in the
// full layout on windows of 1..4 rows (split_contains_asm_batch_h<1..4>) and
// on any target, differences folded onto a nibble (split_contains_asm_batch_h8:
// no gain over the lean test, profiles/r06/batch_h8_ab/).
#pragma once

namespace lifeapi_impl {{
{fns}{emit2()}{emit_contains()}{"".join(emit_contains(True, h) for h in range(1, S))}{"".join(emit_contains(True, h, True) for h in range(1, S + 1))}{"".join(emit_batch(h) for h in list(range(1, LOW_H + 1)) + [S])}{_low_lean()}
}}  // namespace lifeapi_impl
"""


if __name__ == "__main__":
    texts = {OUT: emit(), OUT_TUNE: emit_tune()}
    if "--check" in sys.argv:
        sys.exit(0 if all(open(p).read() == t for p, t in texts.items()) else 1)
    for p, t in texts.items():
        with open(p, "w") as f:
            f.write(t)
    n, bad = check_banks(body())
    print(f"{OUT} (+ {OUT_TUNE}): {n} VALU, {len(bad)} with a bank conflict")
