#!/bin/bash
# CIFAR-3conv: 256-pixel x 128-channel tiles for conv3 (MCC_IGEMM_BIG=128) vs 128x128
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3c
mkdir -p $O
: > $O/ab.jsonl
for m in 1 128 1 128; do
  MCC_IGEMM_BIG=$m timeout -k 10 180 python bench.py --model cifar3 --steps 20 --warmup 5 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "cifar3 big=$m $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
