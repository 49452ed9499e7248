"""Per-kernel MFMA count and scratch (spill) instructions, split into inside/outside the span between the first
and last MFMA. usage: python tools/asm_spills.py file.s [name-filter]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
heads = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):[^\n]*$", s, re.M)]
for k, (i, name) in enumerate(heads):
    if flt not in name:
        continue
    f = s[i: heads[k + 1][0] if k + 1 < len(heads) else len(s)]
    lines = f.split("\n")
    mf = [j for j, l in enumerate(lines) if "v_mfma" in l]
    sc = [j for j, l in enumerate(lines) if "scratch_" in l]
    inside = [j for j in sc if mf and mf[0] < j < mf[-1]]
    print(f"{name[:80]:80s} lines {len(lines):6d} mfma {len(mf):4d} scratch {len(sc):3d} in-mfma-span {len(inside):3d}")
