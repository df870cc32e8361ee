"""Count VGPR bank conflicts (two or more distinct source VGPRs of one VALU
instruction in the same bank, bank = vN mod 4) in the inner loop of a kernel
in build/asm/*.s.  Usage: python tools/vbank.py <mangled-kernel-name>"""
import re
import sys

ASM_GLOB = "build/asm/*-hip-amdgcn-amd-amdhsa-gfx950.s"


def loop_body(name):
    import glob
    lines = [l for f in sorted(glob.glob(ASM_GLOB)) for l in open(f).read().split("\n")]
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = lines[start:end]
    # the generation loop: the backward branch whose body holds the most v_bitop3
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
    best = None
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", l)
        if m and m[1] in labels and labels[m[1]] < i:
            k = sum("v_bitop3" in x for x in body[labels[m[1]]:i])
            # the innermost loop that holds a generation (>= 32 v_bitop3)
            if k >= 32 and (best is None or i - labels[m[1]] < best[1] - best[0]):
                best = (labels[m[1]], i, k)
    return body[best[0]:best[1] + 1]


def conflicts(body):
    n = 0
    out = []
    for l in body:
        l = l.split(";")[0].strip()
        if not l.startswith("v_") or "dpp" in l.split()[0]:
            continue
        ops = [o.strip() for o in l.split(None, 1)[1].split(",")]
        srcs = set()
        for o in ops[1:]:
            o = o.split()[0]
            m = re.match(r"v(\d+)$", o) or re.match(r"v\[(\d+):\d+\]$", o)
            if m:
                srcs.add(int(m[1]))
        banks = [s % 4 for s in srcs]
        if len(banks) != len(set(banks)):
            n += 1
            out.append(l)
    return n, out


if __name__ == "__main__":
    body = loop_body(sys.argv[1])
    n, bad = conflicts(body)
    valu = sum(1 for l in body if l.strip().startswith("v_"))
    print(f"{valu} VALU in loop, {n} with a source bank conflict")
    for l in bad:
        print("  ", l)
