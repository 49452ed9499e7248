"""Steady-state per-step kernel summary from a rocprofv3 SQLite output (rocpd).

The optimizer kernel (adamw_kernel) runs exactly once at the end of every training step, so the kernels
launched after the W-th adamw_kernel and up to the last one are W' = (#adamw - W) whole steps: setup work
(parameter init, first-touch allocations, warmup) is excluded, unlike a plain --stats summary.

usage: python tools/prof_steps.py <dir-or-db> [--warmup W] [--top N] [--grid] [--marker NAME]
"""
import argparse
import glob
import os
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("path")
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--top", type=int, default=45)
ap.add_argument("--grid", action="store_true", help="split kernels by launch grid (GEMM shape attribution)")
ap.add_argument("--marker", default="adamw_kernel")
ap.add_argument("--gaps", type=int, default=0, help="also list the N largest idle gaps between kernels")
ap.add_argument("--dump", default="", help="write the first steady step's dispatch sequence (name, us, grid) to FILE")
ap.add_argument("--alternate", default="", help="split the calls of kernels whose name contains this string by "
                "occurrence parity within the steady steps (#0, #1): the two InternViT weight-gradient pairs share one "
                "kernel and one grid, and alternate fc2.w+fc1.w (#0), proj.w+qkv.w (#1) in every layer's backward")
args = ap.parse_args()
path = args.path
if os.path.isdir(path):
    path = sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))[0]
c = sqlite3.connect(path)
cols = [r[1] for r in c.execute("PRAGMA table_info(kernels)")]
start = next((k for k in ("start", "start_ts", "beginNs", "begin") if k in cols), None)
end = next((k for k in ("end", "end_ts", "endNs") if k in cols), None)
if start is None:
    raise SystemExit(f"no start column in kernels: {cols}")
rows = list(c.execute(f"select name, {start}, {end if end else start}, duration, grid_x, grid_y, grid_z, workgroup_x "
                      f"from kernels order by {start}"))
marks = [r[1] for r in rows if args.marker in r[0]]
if len(marks) <= args.warmup:
    raise SystemExit(f"only {len(marks)} '{args.marker}' launches; need > warmup={args.warmup}")
t0, t1 = marks[args.warmup - 1] if args.warmup > 0 else rows[0][1] - 1, marks[-1]
steps = len(marks) - args.warmup
sel = [r for r in rows if t0 < r[1] <= t1]
agg = defaultdict(lambda: [0, 0.0])
alt = 0
for name, s, e, dur, gx, gy, gz, wx in sel:
    short = name.replace("void ", "").replace("slx::", "")[:120]
    if args.alternate and args.alternate in name:
        short = f"#{alt % 2} " + short
        alt += 1
    key = (short, (gx // max(wx, 1), gy, gz)) if args.grid else (short, None)
    agg[key][0] += 1
    agg[key][1] += dur
busy = sum(v[1] for v in agg.values())
wall = (sel[-1][2] - sel[0][1]) if sel else 0
print(f"{steps} steady steps: kernel-busy {busy / 1e6 / steps:.2f} ms/step, first-to-last span {wall / 1e6 / steps:.2f} "
      f"ms/step ({len(sel) / steps:.0f} launches/step)")
for (n, g), (cnt, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
    gs = f" grid {g}" if g else ""
    print(f"{d / 1e6 / steps:8.3f} ms/step calls/step {cnt / steps:6.1f} avg {d / cnt / 1e3:8.1f} us{gs}  {n}")

if args.gaps:
    # idle time between kernels of the steady steps (a kernel may overlap the previous: track the running max end)
    gaps = []
    run_end = sel[0][2]
    prev = sel[0][0]
    for name, s_, e_, *_ in sel[1:]:
        if s_ > run_end:
            gaps.append((s_ - run_end, prev, name))
        if e_ > run_end:
            run_end, prev = e_, name
    idle = sum(g for g, _, _ in gaps)
    print(f"idle between kernels: {idle / 1e6 / steps:.2f} ms/step over {len(gaps) / steps:.0f} gaps/step")
    hist = defaultdict(lambda: [0, 0.0])
    for g, a, b in gaps:
        k = (a.replace("void ", "").replace("slx::", "")[:60], b.replace("void ", "").replace("slx::", "")[:60])
        hist[k][0] += 1
        hist[k][1] += g
    for (a, b), (n, g) in sorted(hist.items(), key=lambda kv: -kv[1][1])[:args.gaps]:
        print(f"{g / 1e6 / steps:7.3f} ms/step {n / steps:5.1f}x avg {g / n / 1e3:6.1f} us  {a}  ->  {b}")

if args.dump:
    # the first steady step in dispatch order: site attribution by position (kernels are shared by many sites)
    t_end = marks[args.warmup] if len(marks) > args.warmup else t1
    with open(args.dump, "w") as f:
        for i, (name, s_, e_, dur, gx, gy, gz, wx) in enumerate(r for r in sel if r[1] <= t_end):
            f.write(f"{i:5d} {dur / 1e3:9.1f} us grid ({gx // max(wx, 1)},{gy},{gz})  "
                    f"{name.replace('void ', '').replace('slx::', '')[:110]}\n")
