"""Per-dispatch PMC records, grouped by (kernel, grid) and named by call site: every rocprofv3 --pmc pass directory
given is merged on (Dispatch_Id order within each pass is the same program order), so counters from separate passes
line up per dispatch. Prints one JSON record per (kernel, grid) with the mean of every counter, the kernel cycles per XCD
(GRBM_GUI_ACTIVE / 8, rocprofv3 sums the 8 XCDs) and, when present, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
kernel cycles), LDS instructions per wave, and the wave-cycle split (SQ_* wave counters count quad-cycles).
usage: python tools/pmc_dispatch.py SITES.json PASS_DIR [PASS_DIR ...]
SITES.json: {"kernel-substring@grid_x": "site name", ...} (grid_x optional)"""
import collections
import csv
import glob
import json
import os
import sys

sites = json.load(open(sys.argv[1]))
rows = collections.OrderedDict()
for d in sys.argv[2:]:
    per = collections.OrderedDict()
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            e = per.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0),
                                                       "wg": int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 0)})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for i, (_, e) in enumerate(sorted(per.items())):
        tgt = rows.setdefault(i, {"name": e["name"], "grid": e["grid"], "wg": e["wg"]})
        if tgt["name"] != e["name"]:
            raise SystemExit(f"pass {d}: dispatch {i} is {e['name']}, another pass has {tgt['name']}")
        tgt.update({k: v for k, v in e.items() if k not in ("name", "grid", "wg")})


def site_of(e):
    nblk = e["grid"] // max(e["wg"], 1)
    for key, name in sites.items():
        k, _, g = key.partition("@")
        if k in e["name"] and (not g or int(g) == nblk):
            return name
    return None


agg = collections.OrderedDict()
for e in rows.values():
    s = site_of(e)
    if s is None:
        continue
    a = agg.setdefault(s, {"kernel": e["name"][:90], "blocks": e["grid"] // max(e["wg"], 1), "n": 0, "sum": collections.Counter()})
    a["n"] += 1
    for k, v in e.items():
        if k not in ("name", "grid", "wg"):
            a["sum"][k] += v
for s, a in agg.items():
    m = {k: v / a["n"] for k, v in a["sum"].items()}
    rec = {"site": s, "kernel": a["kernel"], "blocks": a["blocks"], "dispatches": a["n"]}
    cyc = m.get("GRBM_GUI_ACTIVE")
    if cyc:
        rec["kernel_cycles_per_xcd"] = round(cyc / 8)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            rec["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc / 8), 4)
    waves = m.get("SQ_WAVES")
    if waves:
        for k in ("SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU"):
            if k in m:
                rec[k.lower() + "_per_wave"] = round(m[k] / waves, 1)
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU"):
            if k in m:
                rec[k.lower() + "_frac_of_wave_cycles"] = round(m[k] / wc, 4)
    rec["counters"] = {k: round(v, 1) for k, v in sorted(m.items())}
    print(json.dumps(rec))
