#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats directory: the kernels with the largest total time."""
import csv
import glob
import sys


def main(d, top=25):
    f = sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True))
    if not f:
        print("no kernel_stats.csv under", d)
        return
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {tot / 1e6:.3f} ms")
    for r in rows[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e3:10.1f} us {int(r['Calls']):6d} x {float(r['AverageNs']) / 1e3:8.1f} us  "
              f"{r['Name'][:100]}")


if __name__ == "__main__":
    main(sys.argv[1])
