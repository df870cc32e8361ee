#!/usr/bin/env python3
"""Schedules of the config-3 assembly loop (tools/gen_split_asm.py, rule 11)
beyond the generator's VARIANTS: the same 68 VALU + 6 LDS per generation in
other orders.  Writes build/c3_sched.inc (one diag_<name> function per
schedule, in the shape of tools/ab/c3_diag.py's) for tools/ab/c3_sched.hip, after
checking every schedule on numpy lanes against the shipped one.

  shipped     gen_split_asm's DEFAULT ("pipe_prio")
  early       rows 1 and 2 (which read only plane-0 h values) run their tails
              before the wait for plane 1, so that plane 1's round trip has
              the h-layer of rows 0..3, the rotates of h[0] and two tails of
              cover instead of the h-layer alone
  early_np    early without the priority toggling
  rotd        shipped, with the two rotates of h[0] before the plane-1 wait
  early_hi    early, priority kept up until plane 1 has been published

Usage: python tools/ab/c3_sched.py   (writes build/c3_sched.inc)
"""
from __future__ import annotations

import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_split_asm as g  # noqa: E402


def _body(early=False, prio=2, rotd_first=False, hold_prio=False):
    S, P = g.S, g.P
    lines = ["s_sub_u32 %[g], %[g], 1", "s_waitcnt lgkmcnt(3)"]
    if prio:
        lines.append(f"s_setprio {prio}")

    def hlayer(js):
        out = []
        for j in js:
            out.append(g.op(g.H0[j], g.L[j], g.R[j], g.RR[j], g.XOR3))
            out.append(g.op(g.H1[j], g.L[j], g.R[j], g.RR[j], g.MAJ))
        return out

    rot_d = [f"v_alignbit_b32 v{g.H0D}, v{g.H0[0]}, v{g.H0[0]}, {P}",
             f"v_alignbit_b32 v{g.H1D}, v{g.H1[0]}, v{g.H1[0]}, {P}"]
    rot_u = [f"v_alignbit_b32 v{g.H0U}, v{g.H0[S - 1]}, v{g.H0[S - 1]}, {32 - P}",
             f"v_alignbit_b32 v{g.H1U}, v{g.H1[S - 1]}, v{g.H1[S - 1]}, {32 - P}"]
    al = g.Alloc()

    def pair(j, k):
        (a, ra), (b, rb) = g.tail_ops(j, al), g.tail_ops(k, al)
        out = [x for xy in zip(a, b) for x in xy]
        for r in ra + rb:
            al.put(r)
        return out

    lines += hlayer(range(4))
    if early:
        lines += rot_d + pair(1, 2) + ["s_waitcnt lgkmcnt(0)"] + hlayer(range(4, 8)) + rot_u + pair(0, 3)
    elif rotd_first:
        lines += rot_d + ["s_waitcnt lgkmcnt(0)"] + hlayer(range(4, 8)) + rot_u + pair(0, 1) + pair(2, 3)
    else:
        lines += ["s_waitcnt lgkmcnt(0)"] + hlayer(range(4, 8)) + rot_u + rot_d + pair(0, 1) + pair(2, 3)
    lines += g.exchange(0)
    if prio and not hold_prio:
        lines.append("s_setprio 0")
    lines += pair(4, 5) + pair(6, 7) + g.exchange(1)
    if prio and hold_prio:
        lines.append("s_setprio 0")
    return lines


SCHEDS = {
    "shipped": lambda: g.body(g.DEFAULT),
    "early": lambda: _body(early=True),
    "early_np": lambda: _body(early=True, prio=0),
    "rotd": lambda: _body(rotd_first=True),
    "early_hi": lambda: _body(early=True, hold_prio=True),
    "early_p1": lambda: _body(early=True, prio=1),
}


def text(name):
    body = SCHEDS[name]()
    return ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 2f"] + g.prologue(g.DEFAULT) + ["1:"] + body + \
        ["s_cmp_lg_u32 %[g], 0", "s_cbranch_scc1 1b", "s_waitcnt lgkmcnt(0)", "2:"]


def simulate(name, r, gens):
    v = np.zeros((g.N_VGPR, 64), np.uint32)
    v[:8] = r
    lds = {}
    seq = g.prologue(g.DEFAULT) + SCHEDS[name]() * gens if gens else []
    for l in seq:
        g._exec(v, l, lds)
    return v[:8].copy()


def check():
    rng = np.random.default_rng(11)
    r = rng.integers(0, 2 ** 32, (8, 64), dtype=np.uint64).astype(np.uint32)
    ref = simulate("shipped", r, 5)
    for name in SCHEDS:
        body = SCHEDS[name]()
        assert sorted(l.split()[0] for l in body if l.startswith(("v_", "ds_"))) == \
            sorted(l.split()[0] for l in g.body(g.DEFAULT) if l.startswith(("v_", "ds_"))), name
        assert np.array_equal(simulate(name, r, 5), ref), name


def fn(name):
    asm = "\n".join(f'      "{l}\\n"' for l in text(name))
    outs = ",\n".join(f'        "+{{v{g.R[j]}}}"(r[{j}])' for j in range(g.S))
    pinned = sorted({x for x in g.L + g.RR + g.H1 + g.H0 + [g.H0U, g.H0D, g.H1U, g.H1D] + g.TEMPS})
    clob = ", ".join(f'"v{x}"' for x in pinned)
    return f"""
__device__ __forceinline__ void diag_{name}(uint32_t (&r)[8], uint32_t gens, uint32_t a_self, uint32_t a_prev,
                                           uint32_t a_next) {{
  asm volatile(
{asm}
      : {outs.strip()},
        [g] "+s"(gens)
      : "{{v{g.A_SELF}}}"(a_self), "{{v{g.A_PREV}}}"(a_prev), "{{v{g.A_NEXT}}}"(a_next)
      : {clob}, "scc", "memory");
}}
"""


def main():
    check()
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    names = list(SCHEDS)
    out = "#pragma once\nnamespace lifeapi_impl {\n" + "".join(fn(n) for n in names) + "}\n"
    out += "#define C3_SCHEDS(X) " + " ".join(f"X({n})" for n in names) + "\n"
    with open(os.path.join(ROOT, "build", "c3_sched.inc"), "w") as f:
        f.write(out)
    print("schedules:", ", ".join(names))


if __name__ == "__main__":
    main()
