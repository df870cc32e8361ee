#!/usr/bin/env python3
"""Generate build/c3_diag.inc for tools/ab/c3_diag.hip: the shipped config-3
assembly loop (tools/gen_split_asm.py, schedule VARIANTS[0]) and diagnostic
cuts of it, to split a generation's time between its parts.  The cuts compute
garbage; only their time and in-kernel clock are read.

  full      the shipped loop
  nolds     the LDS exchange removed (68 VALU, no ds_* op)
  norot     the four ring rotates removed (64 VALU + 6 LDS)
  valu_only both removed (64 VALU)
  lds_only  the exchange and the scalar loop only (no VALU)

Usage: python tools/ab/c3_diag.py   (writes build/c3_diag.inc)
"""
from __future__ import annotations

import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_split_asm as g  # noqa: E402

CUTS = {
    "full": lambda l: True,
    "nolds": lambda l: not l.startswith("ds_"),
    "norot": lambda l: not l.startswith("v_alignbit"),
    "valu_only": lambda l: not l.startswith(("ds_", "v_alignbit")),
    "lds_only": lambda l: not l.startswith("v_"),
    "half_write": lambda l: not l.startswith("ds_write_b128 v46, v[4:7]"),
    "half_read": lambda l: not l.startswith(("ds_read_b128 v[20:23]", "ds_read_b128 v[24:27]")),
    "no_write": lambda l: not l.startswith("ds_write"),
    "no_read": lambda l: not l.startswith("ds_read"),
}


def b64_writes(lines):
    """each ds_write_b128 as two ds_write_b64 (the transfer costs 2 cycles
    per dword plus the address: 2 x 6 against 13, MI355X_MICROARCH.md LDS);
    the lgkmcnt waits count one more op per plane"""
    out = []
    for l in lines:
        if l.startswith("ds_write_b128"):
            base = int(l.split("v[")[1].split(":")[0])
            off = int(l.split("offset:")[1]) if "offset:" in l else 0
            out.append(f"ds_write_b64 v{g.A_SELF}, v[{base}:{base + 1}]" + (f" offset:{off}" if off else ""))
            out.append(f"ds_write_b64 v{g.A_SELF}, v[{base + 2}:{base + 3}] offset:{off + 8}")
        elif l == "s_waitcnt lgkmcnt(3)":
            out.append("s_waitcnt lgkmcnt(4)")
        else:
            out.append(l)
    return out


def prio_shift(lines, k):
    """every s_setprio raised by k (the wave's static class on top of the
    schedule's own 2 / 0 toggling)"""
    return [f"s_setprio {int(l.split()[1]) + k}" if l.startswith("s_setprio") else l for l in lines]


VARIANT_TEXT = {
    "hi": lambda: prio_shift(g.asm_text(g.DEFAULT), 1),
    "b64": lambda: b64_writes(g.asm_text(g.DEFAULT)),
    "prio1": lambda: g.asm_text("pipe_prio1"),
    "prio_e": lambda: g.asm_text("pipe_prio_e"),
}


def fn(name, keep, text=None):
    lines = [l for l in (text or g.asm_text(g.DEFAULT)) if keep(l)]
    asm = "\n".join(f'      "{l}\\n"' for l in lines)
    outs = ",\n".join(f'        "+{{v{g.R[j]}}}"(r[{j}])' for j in range(g.S))
    pinned = sorted({x for x in g.L + g.RR + g.H1 + g.H0 + [g.H0U, g.H0D, g.H1U, g.H1D] + g.TEMPS})
    clob = ", ".join(f'"v{x}"' for x in pinned)
    n_valu = sum(l.startswith("v_") for l in g.body(g.DEFAULT) if keep(l))
    n_lds = sum(l.startswith("ds_") for l in g.body(g.DEFAULT) if keep(l))
    return f"""
// cut "{name}": {n_valu} VALU, {n_lds} LDS per generation
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


import gen_pair_asm as gp  # noqa: E402

PAIR_CUTS = ("full", "nolds", "lds_only")
PAIR_VARIANTS = ("plain", "pipeA")


def pair_fn(variant, name, keep):
    lines = [l for l in gp.asm_text(variant) if keep(l)]
    asm = "\n".join(f'      "{l}\\n"' for l in lines)
    outs = ",\n".join([f'        "+{{v{gp.A[j]}}}"(a[{j}])' for j in range(gp.S)] +
                      [f'        "+{{v{gp.B[j]}}}"(b[{j}])' for j in range(gp.S)])
    clob = ", ".join(f'"v{x}"' for x in range(16, gp.N_VGPR) if x not in (gp.A_SELF, gp.A_PREV, gp.A_NEXT))
    return f"""
__device__ __forceinline__ void diag_pair_{variant}_{name}(uint32_t (&a)[8], uint32_t (&b)[8], uint32_t gens,
    uint32_t a_self, uint32_t a_prev, uint32_t a_next) {{
  asm volatile(
{asm}
      : {outs.strip()},
        [g] "+s"(gens)
      : "{{v{gp.A_SELF}}}"(a_self), "{{v{gp.A_PREV}}}"(a_prev), "{{v{gp.A_NEXT}}}"(a_next)
      : {clob}, "scc", "memory");
}}
"""


def main():
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    text = "#pragma once\nnamespace lifeapi_impl {\n" + "".join(fn(k, v) for k, v in CUTS.items())
    text += "".join(fn(k, CUTS["full"], v()) for k, v in VARIANT_TEXT.items())
    text += "}\n"
    with open(os.path.join(ROOT, "build", "c3_diag.inc"), "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
