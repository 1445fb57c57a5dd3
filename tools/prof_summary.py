#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv / kernel_trace.csv: per-kernel time,
calls, share, and (from the trace) VGPR/LDS/scratch per kernel."""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("mcc::gpu::", "")
    name = re.sub(r"^void ", "", name)
    i = name.rfind("(")
    if i > 0 and name.endswith(")"):
        name = name[:i]
    return name[:110]


def main(d):
    rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
    res = {}
    try:
        for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
            res.setdefault(r["Kernel_Name"], (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"]))
    except FileNotFoundError:
        pass
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':<112} {'calls':>6} {'avg_us':>9} {'pct':>6}  vgpr/agpr/lds/scratch")
    for r in rows:
        k = r["Name"]
        v = res.get(k, ("", "", "", ""))
        print(f"{short(k):<112} {r['Calls']:>6} {float(r['AverageNs'])/1e3:>9.1f} {float(r['Percentage']):>6.2f}  {'/'.join(v)}")
    print(f"total {total/1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
