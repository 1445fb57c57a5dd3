#!/bin/bash
# LeNet-5 headline step: kernel summary + per-dispatch timeline (eager launches and graph replay)
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for g in off auto; do
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_$g -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --graph $g > $O/prof_$g.log 2>&1 || { tail $O/prof_$g.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof_$g > $O/summary_$g.txt 2>&1
python3 $R/tools/step_timeline.py $O/prof_$g/run_kernel_trace.csv > $O/timeline_$g.txt
done
head -24 $O/summary_off.txt
cat $O/timeline_auto.txt
