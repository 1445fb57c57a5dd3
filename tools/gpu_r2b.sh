#!/bin/bash
# HW-queue probe: which streams run concurrently on the box (GPU_MAX_HW_QUEUES=4)
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/q0 -o run --output-format csv -- python $R/tools/probes/queue_probe.py > $O/q0.log 2>&1 || { tail -20 $O/q0.log; exit 1; }
cat $O/q0.log | grep -v "^W\|warn" | tail -8
HP=1 timeout -k 10 120 rocprofv3 --kernel-trace -d $O/q1 -o run --output-format csv -- python $R/tools/probes/queue_probe.py > $O/q1.log 2>&1 || { tail -20 $O/q1.log; exit 1; }
cat $O/q1.log | grep -v "^W\|warn" | tail -3
for d in q0 q1; do python - $O/$d <<'PY'
import csv,glob,sys
p=glob.glob(sys.argv[1]+"/**/*kernel_trace.csv",recursive=True)[0]
for r in csv.DictReader(open(p)):
    n=r["Kernel_Name"]
    if "ncclDevKernel" in n or "oneRank" in n or "sleep" in n.lower() or "spin" in n.lower():
        print(sys.argv[1][-2:], "stream", r["Stream_Id"], "queue", r["Queue_Id"], n[:60])
PY
done
