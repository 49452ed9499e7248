"""Per-kernel averages of every counter in a rocprofv3 --pmc output directory (any counter set).
usage: python tools/pmc_kernels.py DIR [name-substring ...]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
keys = sys.argv[2:]
disp = {}
for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(path)):
        e = disp.setdefault(row["Dispatch_Id"], {"name": row["Kernel_Name"]})
        e[row["Counter_Name"]] = e.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for e in disp.values():
    n = e["name"]
    if keys and not any(k in n for k in keys):
        continue
    cnt[n] += 1
    for k, v in e.items():
        if k != "name":
            agg[n][k] += v
for n in sorted(agg, key=lambda n: -cnt[n]):
    vals = "  ".join(f"{k}={v / cnt[n]:.4g}" for k, v in sorted(agg[n].items()))
    print(f"[{cnt[n]}] {n[:110]}\n    {vals}")
