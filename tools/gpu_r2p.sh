#!/bin/bash
# Round-2 final-state measurement: full GPU suite, every model's bench line, kernel summaries
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2p
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
: > $O/bench.jsonl
b() { timeout -k 10 200 python bench.py "$@" >> $O/bench.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }; }
b
b --dtype fp32 --batch-per-gpu 65536
b --model cifar3
b --model vgg11 --steps 10 --warmup 3
b --model ref
grep metric $O/bench.jsonl | python -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['config']['model'], d['dtype'], d['config']['batch_per_gpu'], d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
for m in lenet5 cifar3 vgg11; do
  st=10; [ $m = vgg11 ] && st=6
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python3 $R/bench.py --model $m --steps $st --warmup 2 > $O/prof_$m.log 2>&1 || { tail $O/prof_$m.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/prof_$m > $O/${m}_summary.txt 2>&1
  python3 $R/tools/step_timeline.py $O/prof_$m/run_kernel_trace.csv > $O/${m}_timeline.txt 2>&1 || true
done
head -12 $O/lenet5_summary.txt
