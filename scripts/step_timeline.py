#!/usr/bin/env python3
"""Prints one training step's kernel timeline (start, end, duration in us,
queue) from a rocprofv3 kernel trace of bench.py: a step of the timed region,
the one starting at the sixth-last encoder forward launch (bench.py's last
three steps run with the per-launch HIP-event timing on, whose event records
add ~7 us in front of every persistent launch; the step after this one is the
last timed step).  usage: step_timeline.py run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "enc_fwd_persist" in r["Kernel_Name"]]
s, e = (idx[-6], idx[-5]) if len(idx) >= 6 else (idx[-3], idx[-2])
t0 = int(rows[s]["Start_Timestamp"])
for r in rows[s - 3:e]:
    st = (int(r["Start_Timestamp"]) - t0) / 1e3
    en = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{st:9.1f} {en:9.1f} {en - st:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:80]}")
