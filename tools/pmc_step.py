"""Per-kernel hardware counters of the steady-state VLA training step (rocprofv3 --pmc, one pass per counter group).

  python tools/pmc_step.py parse --sq DIR --fetch DIR --write DIR [--out JSON] [--top N]

The three directories come from tools/pmc_step.sh (separate rocprofv3 --pmc runs of `bench.py --steps 2 --warmup 1`;
counters cannot share a pass: FETCH_SIZE takes 3 of the 4 TCC slots, WRITE_SIZE 2). Dispatches after the first
adamw_kernel (the end of the first timed step) are grouped by (kernel, grid) and reported per launch:
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)   (GUI_ACTIVE sums the 8 XCDs)
  hbm_read    = 2 x FETCH_SIZE KiB (gfx950 tallies a wide coalesced read at half its bytes, MI355X_MICROARCH.md
                'HBM/rocprofv3'); hbm_write = WRITE_SIZE KiB
  wait/active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY as fractions of SQ_WAVE_CYCLES.
Durations under --pmc are serialised per dispatch; the kernel-trace profile gives the real ones.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

SQ = ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
      "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU"]


def load(d):
    """{dispatch_id: {"name", "grid", "wg", "t0", "t1", counters...}}"""
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            did = int(row["Dispatch_Id"])
            e = out.setdefault(did, {"name": row["Kernel_Name"], "grid": int(row["Grid_Size"]),
                                     "wg": int(row["Workgroup_Size"]), "t0": int(row["Start_Timestamp"]),
                                     "t1": int(row["End_Timestamp"])})
            e[row["Counter_Name"]] = e.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return out


def short(name):
    n = re.sub(r"^void ", "", name).replace("slx::", "")
    return n[:110]


def steady(ds):
    ids = sorted(ds)
    marks = [i for i in ids if "adamw_kernel" in ds[i]["name"]]
    first = marks[0] if marks else ids[0]
    last = marks[-1] if len(marks) > 1 else ids[-1]
    return [i for i in ids if first < i <= last]


def parse(a):
    runs = {k: load(getattr(a, k)) for k in ("sq", "fetch", "write")}
    groups = defaultdict(lambda: defaultdict(float))
    for kind, ds in runs.items():
        for i in steady(ds):
            e = ds[i]
            key = (short(e["name"]), e["grid"] // max(e["wg"], 1))
            g = groups[key]
            if kind == "sq":
                g["n"] += 1
                g["us"] += (e["t1"] - e["t0"]) / 1e3
            for c, v in e.items():
                if c.isupper() or c.startswith("SQ_") or c in ("FETCH_SIZE", "WRITE_SIZE"):
                    g[c] += v
    rows = []
    for (name, grid), g in groups.items():
        n = max(g["n"], 1)
        gui = g.get("GRBM_GUI_ACTIVE", 0.0)
        wave = g.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        rows.append({"kernel": name, "grid": grid, "launches": int(g["n"]), "us_per_launch_pmc": g["us"] / n,
                     "mfma_busy": 8 * g.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * gui) if gui else None,
                     "hbm_read_MB": 2 * g.get("FETCH_SIZE", 0.0) * 1024 / 1e6 / n,
                     "hbm_write_MB": g.get("WRITE_SIZE", 0.0) * 1024 / 1e6 / n,
                     "wait_any": g.get("SQ_WAIT_ANY", 0.0) / wave, "wait_inst": g.get("SQ_WAIT_INST_ANY", 0.0) / wave,
                     "active_inst": g.get("SQ_ACTIVE_INST_ANY", 0.0) / wave,
                     "active_valu": g.get("SQ_ACTIVE_INST_VALU", 0.0) / wave,
                     "valu_insts_per_launch": g.get("SQ_INSTS_VALU", 0.0) / n})
    rows.sort(key=lambda r: -r["us_per_launch_pmc"] * r["launches"])
    rows = rows[: a.top]
    print(f"{'us/launch':>9} {'n':>4} {'mfma':>5} {'rd MB':>8} {'wr MB':>8} {'wait':>5} {'winst':>5} {'act':>5}  kernel (grid)")
    for r in rows:
        mb = f"{r['mfma_busy']:.2f}" if r["mfma_busy"] is not None else "  -  "
        print(f"{r['us_per_launch_pmc']:9.1f} {r['launches']:4d} {mb:>5} {r['hbm_read_MB']:8.1f} {r['hbm_write_MB']:8.1f} "
              f"{r['wait_any']:5.2f} {r['wait_inst']:5.2f} {r['active_inst']:5.2f}  {r['kernel']} ({r['grid']})")
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["parse"])
    ap.add_argument("--sq")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out")
    ap.add_argument("--top", type=int, default=40)
    parse(ap.parse_args())
