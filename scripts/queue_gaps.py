#!/usr/bin/env python3
"""Idle gaps (> 1 us) on the main queue of one timed-region step of a
rocprofv3 kernel trace of bench.py (the step starting at the sixth-last
encoder forward launch), with the kernels either side, and the median step
period.  usage: queue_gaps.py run_kernel_trace.csv"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "enc_fwd_persist" in r["Kernel_Name"]]
s, e = idx[-6], idx[-5]
q = rows[s]["Queue_Id"]
lst = [r for r in rows[s - 4:e + 1] if r["Queue_Id"] == q]
t0 = int(rows[s]["Start_Timestamp"])
tot = 0.0
for a, b in zip(lst, lst[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    if g > 1:
        tot += g
        print(f"{(int(a['End_Timestamp']) - t0) / 1e3:9.1f} {g:6.1f}  {a['Kernel_Name'][:40]} -> {b['Kernel_Name'][:40]}")
per = [(int(rows[j]["Start_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3 for i, j in zip(idx, idx[1:])]
print(f"gaps {tot:.1f} us; step period median {statistics.median(per):.1f} us over {len(per)}")
