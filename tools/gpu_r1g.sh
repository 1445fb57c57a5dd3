#!/bin/bash
# LeNet-5 per-GPU batch sweep + roctx phase ranges of the native trainer
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
for b in ${SWEEP:-65536 98304 131072}; do
  timeout -k 10 120 python bench.py --batch-per-gpu $b --steps 40 --warmup 8 --dataset 131072 > gpurun_out/sweep_$b.log 2>&1 || { tail -5 gpurun_out/sweep_$b.log; exit 1; }
  grep metric gpurun_out/sweep_$b.log
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --marker-trace --kernel-trace --stats -d $R/gpurun_out/prof_roctx -o run --output-format csv -- $R/build/bin/cnn_hip --synthetic 65536 --model lenet5 --batch 4096 --epochs 1 --profile --json - > $R/gpurun_out/prof_roctx.log 2>&1 || { tail -5 $R/gpurun_out/prof_roctx.log; exit 1; }
tail -3 $R/gpurun_out/prof_roctx.log
find $R/gpurun_out/prof_roctx -name "*marker*" | head
