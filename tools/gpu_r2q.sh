#!/bin/bash
# dW side-stream A/B at the round-2 batches (LeNet-5 131072, VGG-11 512, ref 65536)
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2q
mkdir -p $O
: > $O/ab.jsonl
for m in lenet5 ref; do
  for ss in 0 1 0 1; do
    MCC_SIDE_STREAM=$ss timeout -k 10 180 python bench.py --model $m --steps 30 --warmup 5 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
    echo "$m side=$ss $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
  done
done
for ss in 0 1; do
  MCC_SIDE_STREAM=$ss timeout -k 10 180 python bench.py --model vgg11 --steps 6 --warmup 2 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "vgg11 side=$ss $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
