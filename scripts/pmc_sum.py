#!/usr/bin/env python3
"""Average a rocprofv3 --pmc counter per kernel (argv[1] = counter_collection.csv, argv[2] =
counter name, argv[3] = kernel-name substring filter)."""
import collections
import csv
import sys

tot, cnt = collections.defaultdict(float), collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if r.get("Counter_Name") != sys.argv[2] or sys.argv[3] not in r["Kernel_Name"]:
        continue
    key = r["Kernel_Name"].split("(")[0]
    tot[key] += float(r["Counter_Value"])
    cnt[key].add(r["Dispatch_Id"])
for k in sorted(tot):
    print(f"{k}: {sys.argv[2]} {tot[k] / len(cnt[k]):.1f} per dispatch over {len(cnt[k])}")
