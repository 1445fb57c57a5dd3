#!/usr/bin/env python3
"""Gaps between consecutive kernels of the last full step in a rocprofv3
kernel trace (the step boundary = the last `sample_kernel` dispatch):

    python tools/trace_gaps.py gpurun_out/X/prof/run_kernel_trace.csv [min_gap_us]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
starts = [i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"]]
a, b = starts[-2], starts[-1]
t0 = int(rows[a]["Start_Timestamp"])
tot_gap = 0.0
for i in range(a, b):
    r, n = rows[i], rows[i + 1]
    gap = (int(n["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3
    tot_gap += max(gap, 0.0)
    if gap >= thr:
        print(f"{(int(r['End_Timestamp']) - t0) / 1e3:9.1f} us  gap {gap:6.1f} us  after {r['Kernel_Name'][:60]}  before {n['Kernel_Name'][:50]}")
print(f"step {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us, idle between kernels {tot_gap:.1f} us")
