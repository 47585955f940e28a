#!/usr/bin/env python3
"""Gaps between the single-workgroup inner-loop launches of one solve, from a rocprofv3
`--kernel-trace --hip-trace --output-format csv` run (argv: the directory holding
<name>_kernel_trace.csv and <name>_hip_api_trace.csv, and the name): the gaps' total, median and
largest, and the HIP calls inside the largest ones (profiles/r06zd_theta3_summary.md)."""
import collections
import csv
import os
import statistics
import sys

d, name = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "theta3"
K = sorted(csv.DictReader(open(os.path.join(d, f"{name}_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
H = sorted(csv.DictReader(open(os.path.join(d, f"{name}_hip_api_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
alm = [r for r in K if "k_small_alm" in r["Kernel_Name"]]
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]), int(a["End_Timestamp"]), int(b["Start_Timestamp"]))
        for a, b in zip(alm, alm[1:])]
print(f"{len(alm)} launches; gaps {sum(g for g, _, _ in gaps) / 1e6:.2f} ms, median "
      f"{statistics.median(g for g, _, _ in gaps) / 1e3:.0f} us")
for g, e, s in sorted(gaps, reverse=True)[:6]:
    agg, cnt = collections.Counter(), collections.Counter()
    for r in H:
        t = int(r["Start_Timestamp"])
        if e < t < s:
            agg[r["Function"]] += int(r["End_Timestamp"]) - t
            cnt[r["Function"]] += 1
    print(f"  {g / 1e3:.0f} us:", ", ".join(f"{f} x{cnt[f]} {v / 1e3:.0f} us" for f, v in agg.most_common(5)))
