"""Instruction mix of the innermost loops of a kernel in build/asm/*.s (a loop
= a label up to the backward branch that targets it):
python tools/ab/kloop.py <kernel-name-regex>."""
import collections
import glob
import re
import sys

pat = re.compile(sys.argv[1])
for f in sorted(glob.glob("build/asm/*gfx950.s")):
    s = open(f).read()
    for m in re.finditer(r"^(_Z\w+):\s*;", s, re.M):
        if not pat.search(m.group(1)):
            continue
        body = s[m.end():s.find(".end_amdhsa_kernel", m.end())]
        lines = body.split("\n")
        labels = {l.split(":")[0]: i for i, l in enumerate(lines) if re.match(r"^\.LBB\w+:", l)}
        print(m.group(1))
        for i, l in enumerate(lines):
            b = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)", l) or re.match(r"\s+s_branch\s+(\.LBB\w+)", l)
            if b and b.group(1) in labels and labels[b.group(1)] < i:
                seg = [x.split()[0] for x in lines[labels[b.group(1)] + 1:i + 1]
                       if x.startswith("\t") and not x.strip().startswith(";") and x.strip()]
                c = collections.Counter(seg)
                print(f"  loop {b.group(1)}: {len(seg)} instrs:",
                      ", ".join(f"{k}={v}" for k, v in c.most_common(14)))
