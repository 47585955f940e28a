#!/usr/bin/env python3
"""Summarise a scripts/profile_*.sh run (rocprofv3 CSVs under gpurun_out/prof_<tag>)
into profiles/<tag>_*.  Usage: python scripts/summarize_prof.py <tag>"""
import collections
import csv
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
dst = os.environ.get("PROF_DST") or os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))

lines = [f"# rocprofv3 summary `{tag}`", "", "Command: `scripts/profile_r01.sh` (bench.py headline run; separate --pmc passes).", "", "## kernel trace (--kernel-trace --stats)", "",
         "| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
    lines.append(f"| `{r['Name'][:60]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                 f"{float(r['MinNs'])/1e3:.2f} | {float(r['MaxNs'])/1e3:.2f} | {float(r['Percentage']):.2f} |")
pmc = {}
for f, cname in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    p = os.path.join(src, f, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        pmc.setdefault(k, {})[cname] = (len(v), sum(v) / len(v))
if pmc:
    lines += ["", "## HBM-side bytes per dispatch (separate --pmc passes; KB as reported, FETCH_SIZE uncorrected)", "",
              "| kernel | dispatches | FETCH_SIZE KB | x2 (gfx950 wide-read correction) KB | WRITE_SIZE KB |",
              "|---|---|---|---|---|"]
    for k, d in sorted(pmc.items(), key=lambda kv: -kv[1].get("FETCH_SIZE", (0, 0))[1]):
        fz = d.get("FETCH_SIZE", (0, float("nan")))
        wz = d.get("WRITE_SIZE", (0, float("nan")))
        lines.append(f"| `{k[:60]}` | {fz[0]} | {fz[1]:.1f} | {2 * fz[1]:.1f} | {wz[1]:.1f} |")
for log in ("trace.log",):
    p = os.path.join(src, log)
    if os.path.exists(p):
        js = [l[l.index("{"):] for l in open(p) if "{\"metric\"" in l]
        if js:
            lines += ["", "## bench line under the profiler", "", "```", js[-1].strip(), "```"]
open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
# per-dispatch HBM-side bytes for bench.py's roofline.traffic: FETCH_SIZE doubled (the gfx950
# correction for wide streaming reads, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, KB -> bytes
import json
pmc_out = {}
for k, d in pmc.items():
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        pmc_out[k.split("(")[0].replace("void ", "").strip()] = {
            "dispatches": d["FETCH_SIZE"][0], "fetch_bytes": 2 * d["FETCH_SIZE"][1] * 1024,
            "write_bytes": d["WRITE_SIZE"][1] * 1024, "source": f"profiles/{tag}_summary.md"}
json.dump(pmc_out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1, sort_keys=True)
print("\n".join(lines))
