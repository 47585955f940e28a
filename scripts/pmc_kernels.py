#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 directory laid out by scripts/profile_g81.sh: the kernel
trace's stats and resources (VGPRs, workgroup, grid), and every counter pass's mean value per
dispatch.  Usage: pmc_kernels.py <dir>"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
out = ["# rocprofv3 per-kernel summary: " + os.path.basename(d.rstrip("/")), ""]
stats = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))
if stats:
    out += ["## kernel trace (--kernel-trace --stats)", "", "| kernel | calls | avg us | % |", "|---|---|---|---|"]
    for r in csv.DictReader(open(stats[0])):
        out.append(f"| `{r['Name'][:70]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                   f"{float(r['Percentage']):.1f} |")
kt = glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))
if kt:
    res = {}
    for r in csv.DictReader(open(kt[0])):
        k = r.get("Kernel_Name", "")
        if k not in res:
            res[k] = (r.get("Arch_VGPR_Count", "?"), r.get("Accum_VGPR_Count", "?"), r.get("SGPR_Count", "?"),
                      r.get("LDS_Block_Size", r.get("Lds_Size", "?")), r.get("Workgroup_Size", "?"),
                      r.get("Grid_Size", "?"))
    out += ["", "## resources (first dispatch)", "", "| kernel | VGPR | AGPR | SGPR | LDS | workgroup | grid |",
            "|---|---|---|---|---|---|---|"]
    for k, v in res.items():
        out.append(f"| `{k[:70]}` | " + " | ".join(str(x) for x in v) + " |")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ("sq", "fetch", "write"):
    for f in glob.glob(os.path.join(d, sub, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
if agg:
    names = sorted({c for v in agg.values() for c in v})
    out += ["", "## counters (mean per dispatch; FETCH_SIZE / WRITE_SIZE in KB, FETCH uncorrected)", "",
            "| kernel | dispatches | " + " | ".join(names) + " |", "|---|---|" + "---|" * len(names)]
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
        n = max(len(x) for x in v.values())
        out.append(f"| `{k[:60]}` | {n} | " + " | ".join(
            f"{sum(v[c]) / len(v[c]):.4g}" if v.get(c) else "" for c in names) + " |")
print("\n".join(out))
