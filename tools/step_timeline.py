#!/usr/bin/env python3
"""Per-dispatch timeline (us, grid, kernel) of the last full step in a rocprofv3
kernel trace; steps are delimited by the device sampler (sample_kernel / sample_advance_kernel)."""
import csv
import sys


def main(path, marker="sample"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    start, end = idx[-2], idx[-1]
    t0 = int(rows[start]["Start_Timestamp"])
    for r in rows[start:end]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        t = (int(r["Start_Timestamp"]) - t0) / 1000
        print(f"{t:9.1f} {d:8.1f} q{r['Queue_Id']:>2} {r['Grid_Size_X']:>10} {r['Kernel_Name'][:80]}")
    print(f"step {(int(rows[end]['Start_Timestamp']) - t0) / 1000:.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])
