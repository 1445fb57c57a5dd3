#!/bin/bash
# Graph-capture robustness at world 1 (watchdog / captured-event fix): 12 short bench runs, stop at
# the first failure; then the side-stream A/B that crashed before.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2r
mkdir -p $O
: > $O/runs.jsonl
for i in 1 2 3 4 5 6; do
  for m in ref lenet5; do
    timeout -k 10 120 python bench.py --model $m --steps 10 --warmup 3 >> $O/runs.jsonl 2>$O/err.log || { echo "run $i $m failed"; grep -v "^frame" $O/err.log | tail -20; exit 1; }
  done
done
grep -c metric $O/runs.jsonl
: > $O/ab.jsonl
for m in ref; do
  for ss in 0 1 0 1; do
    MCC_SIDE_STREAM=$ss timeout -k 10 180 python bench.py --model $m --steps 30 --warmup 5 >> $O/ab.jsonl 2>$O/err.log || { grep -v "^frame" $O/err.log | tail; exit 1; }
    echo "$m side=$ss $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
  done
done
for ss in 0 1; do
  MCC_SIDE_STREAM=$ss timeout -k 10 180 python bench.py --model vgg11 --steps 6 --warmup 2 >> $O/ab.jsonl 2>$O/err.log || { grep -v "^frame" $O/err.log | tail; exit 1; }
  echo "vgg11 side=$ss $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
