#!/bin/bash
# One short bench.py run per model / dtype (1 GPU) -> gpurun_out/bench_models.jsonl
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/bench_models.jsonl
for cfg in "lenet5 bf16" "lenet5 fp32" "ref bf16" "ref fp32" "cifar3 bf16" "vgg11 bf16"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --model $1 --dtype $2 --steps 20 --warmup 5 > gpurun_out/bm_$1_$2.log 2>&1 || { echo "FAILED $cfg"; tail -5 gpurun_out/bm_$1_$2.log; exit 1; }
  grep metric gpurun_out/bm_$1_$2.log >> gpurun_out/bench_models.jsonl
  echo "$cfg ok"
done
