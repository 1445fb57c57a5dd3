#!/bin/bash
# LeNet-5 batch 163840 (96% of the 32-bit activation bound) vs 131072
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2x
mkdir -p $O
: > $O/ab.jsonl
for b in 131072 163840 131072 163840; do
  timeout -k 10 180 python bench.py --batch-per-gpu $b --steps 30 --warmup 5 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "B=$b $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['config']['train_loss_last'])")"
done
