#!/usr/bin/env python3
"""Comm/compute overlap from a rocprofv3 kernel trace (run_kernel_trace.csv).

For every collective kernel (RCCL: name contains nccl / rccl / OneRank) it
prints its HIP stream and hardware queue, its duration, and which kernels on
OTHER hardware queues ran concurrently with it (intersection of [start, end)
intervals) — the evidence that a bucket's all-reduce runs on the comm stream
while the compute stream continues with the earlier stages' backward.  (A
replayed hipGraph reports one stream id for all its nodes; the executor runs
independent branches on different hardware queues, so concurrency is judged
by Queue_Id.)  Usage:
    overlap_report.py <trace dir> [max steps to print]
"""
import csv
import glob
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("mcc::gpu::", "")
    name = re.sub(r"^void ", "", name)
    i = name.find("(")
    return (name[:i] if i > 0 else name)[:70]


def is_coll(name):
    n = name.lower()
    return "nccl" in n or "rccl" in n or "onerank" in n


def main(d, max_show=6):
    paths = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not paths:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = list(csv.DictReader(open(paths[0])))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"), r.get("Stream_Id", "?"),
                   r["Kernel_Name"]))
    ks.sort()
    coll = [k for k in ks if is_coll(k[4])]
    print(f"trace: {paths[0]}")
    print(f"kernels: {len(ks)}, collective kernels: {len(coll)}")
    if not coll:
        return
    qs = sorted({k[2] for k in coll})
    print(f"collective hw queues: {qs}; compute hw queues: {sorted({k[2] for k in ks if not is_coll(k[4])})}")
    tot_c = sum(e - s for s, e, *_ in coll)
    ov_tot = 0
    shown = 0
    for i, (s, e, q, hs, n) in enumerate(coll):
        over = [(max(s, s2), min(e, e2), n2, q2) for s2, e2, q2, hq2, n2 in ks if q2 != q and s2 < e and e2 > s]
        ov = 0
        # union of overlapping intervals
        iv = sorted((a, b) for a, b, *_ in over)
        cur = None
        for a, b in iv:
            if cur is None or a > cur[1]:
                if cur:
                    ov += cur[1] - cur[0]
                cur = [a, b]
            else:
                cur[1] = max(cur[1], b)
        if cur:
            ov += cur[1] - cur[0]
        ov_tot += ov
        if shown < max_show and (ov > 0 or i + max_show >= len(coll)):
            shown += 1
            names = sorted({short(n2) for *_, n2, q2 in over})
            print(f"  [{i}] {short(n)} hw queue {q} (stream {hs}): {(e - s) / 1e3:.1f} us, "
                  f"{100.0 * ov / max(1, e - s):.0f}% overlapped by: {', '.join(names) or '-'}")
    print(f"collective time {tot_c / 1e3:.1f} us total, {100.0 * ov_tot / max(1, tot_c):.1f}% of it concurrent "
          f"with compute kernels on other hardware queues")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 6)
