#!/usr/bin/env python3
"""Per-kernel PMC summary of scripts/pmc_step_kernel.sh output: counter totals per
dispatch of the longest kernel.  usage: pmc_summary.py <outdir>"""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
tot = defaultdict(float)
n = defaultdict(set)
kern = None
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "gemm" not in name and "slab" not in name:
            continue
        key = (name[:60], r["Counter_Name"])
        tot[key] += float(r["Counter_Value"])
        n[key].add(r["Dispatch_Id"])
for (k, c), v in sorted(tot.items()):
    print(f"{k:60s} {c:28s} {v / max(1, len(n[(k, c)])):16.1f} per dispatch ({len(n[(k, c)])} disp)")
