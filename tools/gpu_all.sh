#!/bin/bash
# full GPU test suite, headline bench, VGG bench + profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
grep metric gpurun_out/bench.log
for b in ${VGG_BATCHES:-128}; do
  timeout -k 10 200 python bench.py --model vgg11 --batch-per-gpu $b --steps 10 --warmup 3 > gpurun_out/vgg_$b.log 2>&1 || { tail -5 gpurun_out/vgg_$b.log; exit 1; }
  grep metric gpurun_out/vgg_$b.log
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_vgg -o run --output-format csv -- python3 $R/bench.py --model vgg11 --batch-per-gpu 128 --steps 5 --warmup 2 > $R/gpurun_out/prof_vgg.log 2>&1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_lenet -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 > $R/gpurun_out/prof_lenet.log 2>&1
