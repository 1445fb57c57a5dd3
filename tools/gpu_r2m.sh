#!/bin/bash
# per-GPU batch sweep for the 288 GB HBM sizing (LeNet-5, CIFAR-3conv, VGG-11)
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2m
mkdir -p $O
: > $O/sweep.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_igemm.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { timeout -k 10 180 python bench.py "$@" >> $O/sweep.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }; }
for b in 65536 131072; do run --batch-per-gpu $b --steps 20 --warmup 5; done
for b in 16384 32768 65536; do run --model cifar3 --batch-per-gpu $b --steps 20 --warmup 5; done
for b in 256 512; do run --model vgg11 --batch-per-gpu $b --steps 8 --warmup 3; done
grep metric $O/sweep.jsonl | python -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['config']['model'], d['config']['batch_per_gpu'], d['value'], d['ms_per_step'])"
