#!/bin/bash
# fused classifier head: engine/program tests, A/B bench (MCC_NO_HEAD=1 = unfused), kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_programs.py -x -v --timeout 120 --timeout-method thread > gpurun_out/head_tests.log 2>&1 || { tail -30 gpurun_out/head_tests.log; exit 1; }
tail -2 gpurun_out/head_tests.log
for m in lenet5 cifar3; do
  for nh in 1 0 1 0; do
    MCC_NO_HEAD=$nh timeout -k 10 200 python bench.py --model $m > gpurun_out/head_b.log 2>&1 || { tail -5 gpurun_out/head_b.log; exit 1; }
    echo "$m no_head=$nh $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/head_b.log') if l.startswith('{')][-1]);print(d['value'],d['ms_per_step'],d['config']['train_loss_last'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_head -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 > $R/gpurun_out/prof_head.log 2>&1
