#!/usr/bin/env python3
"""Average per-dispatch counter values of one kernel over every CSV under a directory.
Usage: tools/pmc_summary.py DIR KERNEL_SUBSTRING"""
import csv
import glob
import os
import sys

d, kern = sys.argv[1], sys.argv[2]
acc = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    per = {}
    for row in csv.DictReader(open(f)):
        if kern not in row["Kernel_Name"]:
            continue
        per.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
        per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    for c, v in per.items():
        acc[c] = sum(v.values()) / len(v)
for c in sorted(acc):
    print(f"{c:45s} {acc[c]:.6g}")
