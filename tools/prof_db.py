"""Summarise a rocprofv3 SQLite output (rocpd): per-kernel (and optionally per-grid) time per step.
usage: python tools/prof_db.py <dir-or-db> <steps> [top] [--grid]"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict

path = sys.argv[1]
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 and not sys.argv[3].startswith("--") else 40
by_grid = "--grid" in sys.argv
c = sqlite3.connect(path)
agg = defaultdict(lambda: [0, 0.0])
for name, dur, gx, gy, gz, wx in c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels"):
    short = name.replace("void ", "").replace("slx::", "")[:110]
    key = (short, (gx // max(wx, 1), gy, gz)) if by_grid else (short, None)  # blocks
    agg[key][0] += 1
    agg[key][1] += dur
tot = sum(v[1] for v in agg.values())
print(f"total {tot / 1e6:.2f} ms over {steps:g} steps -> {tot / 1e6 / steps:.2f} ms/step")
for (n, g), (cnt, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    gs = f" grid {g}" if g else ""
    print(f"{d / 1e6 / steps:8.2f} ms/step calls/step {cnt / steps:6.1f} avg {d / cnt / 1e3:8.1f} us{gs}  {n}")
