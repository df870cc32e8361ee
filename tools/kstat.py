"""Per-kernel register use and instruction mix from the saved device assembly
(build/asm/*.s): python tools/kstat.py [kernel-name-regex]."""
import glob
import re
import sys

pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
KEYS = ("v_bitop3", "_dpp", "row_ror", "v_alignbit", "ds_read", "ds_write", "v_mov_b32", "v_perm",
        "s_cbranch", "global_load", "global_store", "scratch_")
for f in sorted(glob.glob("build/asm/*gfx950.s")):
    s = open(f).read()
    for m in re.finditer(r"^(_Z\w+):\s*;", s, re.M):
        name = m.group(1)
        if not pat.search(name):
            continue
        end = s.find(".end_amdhsa_kernel", m.end())
        seg = s[m.end():end]
        body = seg[:seg.find(".amdhsa_kernel")]
        v = re.search(r"\.amdhsa_next_free_vgpr (\d+)", seg)
        a = re.search(r"\.amdhsa_accum_offset (\d+)", seg)
        sp = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", seg)
        counts = " ".join(f"{k.strip('_')}={body.count(k)}" for k in KEYS if body.count(k))
        print(f"{name[:70]:70s} vgpr={v and v.group(1)} acc_off={a and a.group(1)} "
              f"scratch={sp and sp.group(1)} {counts}")
