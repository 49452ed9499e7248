"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: one line per kernel (VGPRs, spills, scratch, LDS).
usage: python tools/kres.py <file.hip> [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
       "-I/root/repo/include", "-I/root/repo/simlingo_amd/csrc", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
for a in sys.argv[3:]:
    cmd.append(a)
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, {}
for line in out.splitlines():
    m = re.search(r"remark: (?:\s*)([A-Za-z ]+?)(?: \[[^\]]*\])?: (.*?) \[-Rpass", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, r in rows.items():
    if flt in name:
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('AGPRs','0'):>3} agpr spill {r.get('VGPRs Spill','?'):>3} "
              f"scratch {r.get('ScratchSize','?'):>4} lds {r.get('LDS Size','?'):>6}  {dem[:150]}")
