#!/bin/bash
# VGG-11 per-GPU batch 512 vs 640 (95.7 % of the 32-bit activation bound)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3g
mkdir -p $O
: > $O/ab.jsonl
for b in 512 640 512 640; do
  timeout -k 10 200 python bench.py --model vgg11 --batch-per-gpu $b --steps 6 --warmup 2 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "B=$b $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['config']['train_loss_last'])")"
done
