#!/usr/bin/env python3
"""Generate build/issue_probe.inc for tools/ab/issue_probe.hip: VALU issue
probes on gfx950 (the issue model behind the config-3 loop's layout choice).
Each probe is a loop of 64 VALU instructions on v32..v95, repeated `iters`
times; probes differ in dependency distance, encoding and operand banks.

  indep     64 v_bitop3_b32, sources in three distinct banks, no result read
            within the next 16 instructions
  chainK    K interleaved dependent chains (K = 1, 2, 4, 8): each
            instruction reads the result of the instruction K before it
  xor2      64 v_xor_b32 (VOP2, 4-byte encoding), independent
  conflict  as indep, but two of the three sources in one bank
  alignbit  64 v_alignbit_b32 (rotate), independent

Usage: python tools/ab/issue_probe.py
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BASE, NREG = 32, 64


def reg(bank, k):
    """k-th register of bank `bank` in v32..v95"""
    return BASE + 4 * (k % 16) + bank


def indep():
    out = []
    for i in range(64):
        d = reg(i % 4, (i // 4) % 16)
        a, b, c = reg((i + 1) % 4, (i // 4 + 5) % 16), reg((i + 2) % 4, (i // 4 + 9) % 16), reg((i + 3) % 4, (i // 4 + 13) % 16)
        out.append(f"v_bitop3_b32 v{d}, v{a}, v{b}, v{c} bitop3:0x96")
    return out


def chain(k):
    out = []
    for i in range(64):
        d = reg(i % 4, (i // 4) % 16)
        p = i - k if i >= k else 64 + i - k     # the instruction k before (cyclic)
        src = reg(p % 4, (p // 4) % 16)
        b1 = [x for x in range(4) if x != src % 4]
        a = reg(b1[0], (i + 7) % 16)
        c = reg(b1[1], (i + 11) % 16)
        out.append(f"v_bitop3_b32 v{d}, v{src}, v{a}, v{c} bitop3:0x96")
    return out


def xor2():
    out = []
    for i in range(64):
        d = reg(i % 4, (i // 4) % 16)
        a, b = reg((i + 1) % 4, (i // 4 + 5) % 16), reg((i + 2) % 4, (i // 4 + 9) % 16)
        out.append(f"v_xor_b32 v{d}, v{a}, v{b}")
    return out


def conflict():
    out = []
    for i in range(64):
        d = reg(i % 4, (i // 4) % 16)
        a, b, c = reg((i + 1) % 4, (i // 4 + 5) % 16), reg((i + 1) % 4, (i // 4 + 9) % 16), reg((i + 3) % 4, (i // 4 + 13) % 16)
        out.append(f"v_bitop3_b32 v{d}, v{a}, v{b}, v{c} bitop3:0x96")
    return out


def alignbit():
    out = []
    for i in range(64):
        d = reg(i % 4, (i // 4) % 16)
        a = reg((i + 1) % 4, (i // 4 + 5) % 16)
        out.append(f"v_alignbit_b32 v{d}, v{a}, v{a}, 4")
    return out


PROBES = {"indep": indep(), "chain1": chain(1), "chain2": chain(2), "chain4": chain(4), "chain8": chain(8),
          "xor2": xor2(), "conflict": conflict(), "alignbit": alignbit()}


def fn(name, body):
    init = [f"v_mul_u32_u24 v{r}, {hex(0x9E3779 * (r + 1) & 0xFFFFFF | 1)}, %[seed]" for r in range(BASE, BASE + NREG)]
    lines = init + ["1:"] + body + ["s_sub_u32 %[n], %[n], 1", "s_cmp_lg_u32 %[n], 0", "s_cbranch_scc1 1b"]
    asm = "\n".join(f'      "{l}\\n"' for l in lines)
    clob = ", ".join(f'"v{r}"' for r in range(BASE, BASE + NREG))
    return f"""
__device__ __forceinline__ void probe_{name}(uint32_t iters, uint32_t seed) {{
  asm volatile(
{asm}
      : [n] "+s"(iters)
      : [seed] "v"(seed)
      : {clob}, "scc");
}}
"""


def main():
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    text = "#pragma once\n" + "".join(fn(k, v) for k, v in PROBES.items())
    text += "#define ISSUE_PROBES(X) " + " ".join(f"X({k})" for k in PROBES) + "\n"
    with open(os.path.join(ROOT, "build", "issue_probe.inc"), "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
