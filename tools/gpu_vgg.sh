#!/bin/bash
# large-image path: engine tests, VGG-11 bench + kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k "igemm or vgg or im2col or step_matches" > gpurun_out/vgg_tests.log 2>&1 || { tail -30 gpurun_out/vgg_tests.log; exit 1; }
tail -3 gpurun_out/vgg_tests.log
for b in ${VGG_BATCHES:-128}; do
  timeout -k 10 200 python bench.py --model vgg11 --batch-per-gpu $b --steps 10 --warmup 3 > gpurun_out/vgg_$b.log 2>&1 || { tail -5 gpurun_out/vgg_$b.log; exit 1; }
  grep metric gpurun_out/vgg_$b.log
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_vgg -o run --output-format csv -- python3 $R/bench.py --model vgg11 --batch-per-gpu 128 --steps 5 --warmup 2 > $R/gpurun_out/prof_vgg.log 2>&1
