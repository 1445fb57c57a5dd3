#!/bin/bash
# every BASELINE.json model config at its bench.py default batch (+ a cifar3 batch sweep)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/models_r1g.jsonl
run() {
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/m.log 2>&1 || { echo "FAIL $*"; tail -3 gpurun_out/m.log; exit 1; }
  grep metric gpurun_out/m.log >> gpurun_out/models_r1g.jsonl
  echo "$* :: $(grep -o '"value": [0-9.]*' gpurun_out/m.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/m.log)"
}
run --model lenet5 --dtype fp32
run --model ref
run --model ref --dtype fp32
run --model cifar3
run --model cifar3 --batch-per-gpu 8192
run --model cifar3 --batch-per-gpu 16384
run --model cifar3 --dtype fp32
run --model vgg11 --steps 10 --warmup 3
run --model vgg11 --batch-per-gpu 384 --steps 10 --warmup 3
