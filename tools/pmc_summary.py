#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter_collection.csv per kernel (mean over dispatches)."""
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
    return name[:120]


def main(paths):
    agg = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = sorted({c for k in agg for c in agg[k]})
    for k, cs in agg.items():
        print(k)
        for c in names:
            if c in cs:
                v = cs[c]
                print(f"    {c:<28} {sum(v)/len(v):>16.0f}")


if __name__ == "__main__":
    main(sys.argv[1:])
