#!/usr/bin/env python3
"""Per-kernel mean (per dispatch) of every counter in rocprofv3 --pmc output
directories: a quick look at one kernel's counters across several passes.

    python scripts/pmc_kernels.py <pmc dir> [<pmc dir> ...] [--match FRAGMENT]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    match = None
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1]
        args = args[:i] + args[i + 2:]
    vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name", "")
                    if match and match not in k:
                        continue
                    vals[k[:90]][row["Counter_Name"]][row.get("Dispatch_Id")] += float(row["Counter_Value"])
    for k, per in sorted(vals.items()):
        print(k)
        for c, disp in sorted(per.items()):
            v = sum(disp.values()) / len(disp)
            print(f"   {c:32s} {v:16.0f}   ({len(disp)} dispatches)")


if __name__ == "__main__":
    main()
