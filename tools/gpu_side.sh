#!/bin/bash
# A/B of the weight-gradient side stream (MCC_NO_SIDE=1 = single stream) + engine/program tests
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_programs.py -x -v --timeout 120 --timeout-method thread > gpurun_out/side_tests.log 2>&1 || { tail -30 gpurun_out/side_tests.log; exit 1; }
tail -2 gpurun_out/side_tests.log
for m in "lenet5" "ref" "cifar3" "vgg11 --batch-per-gpu 128 --steps 10 --warmup 3"; do
  for ns in 0 1; do
    MCC_SIDE_STREAM=$ns timeout -k 10 200 python bench.py --model $m > gpurun_out/side_b.log 2>&1 || { tail -5 gpurun_out/side_b.log; exit 1; }
    echo "$m side=$ns $(python3 -c "import json,sys;d=json.loads([l for l in open('gpurun_out/side_b.log') if l.startswith('{')][-1]);print(d['value'],d['ms_per_step'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_side -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 > $R/gpurun_out/prof_side.log 2>&1
