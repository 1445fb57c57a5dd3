#!/bin/bash
# kernel stats for the large-image configs
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
for cfg in "vgg11 32" "vgg11 128" "cifar3 4096"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --model $1 --batch-per-gpu $2 --steps 10 --warmup 3 > gpurun_out/pm_$1_$2.log 2>&1 || { tail -5 gpurun_out/pm_$1_$2.log; exit 1; }
  grep metric gpurun_out/pm_$1_$2.log
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$1_$2 -o run --output-format csv -- python3 $R/bench.py --model $1 --batch-per-gpu $2 --steps 5 --warmup 2 > $R/gpurun_out/prof_$1_$2.log 2>&1) || exit 1
done
