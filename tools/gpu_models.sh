#!/bin/bash
# Throughput + kernel summaries of the other configs: LeNet-5 fp32, VGG-11 bf16
# B=256, CIFAR-3conv bf16 (one MI355X).
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/models
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 240 python $R/bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  echo "$n: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/$n.json | tr '\n' ' ')"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/p_$n -o run --output-format csv -- python $R/bench.py "$@" --steps 6 --warmup 2 > $O/p_$n.log 2>&1 || { tail -5 $O/p_$n.log; return 1; }
  python $R/tools/prof_summary.py $O/p_$n > $O/${n}_kernels.txt && head -${TOPK:-12} $O/${n}_kernels.txt
}
for c in ${CONFIGS:-lenet_fp32 vgg11 cifar3}; do
  case $c in
    lenet_fp32) run lenet_fp32 --dtype fp32 --steps 20 --warmup 5 --no-dist ;;
    vgg11) run vgg11 --model vgg11 --batch-per-gpu 256 --steps 10 --warmup 3 --no-dist ;;
    cifar3) run cifar3 --model cifar3 --steps 20 --warmup 5 --no-dist ;;
  esac || exit 1
done
