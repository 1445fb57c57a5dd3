#!/bin/bash
# Re-validation of HEAD after a container restore: GPU tests, every model's
# bench line, VGG-11 kernel summary.  Every GPU step has its own time limit;
# the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2h
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python bench.py > $O/bench.jsonl 2>$O/bench.err || { tail $O/bench.err; exit 1; }
timeout -k 10 120 python bench.py --dtype fp32 >> $O/bench.jsonl 2>>$O/bench.err || exit 1
timeout -k 10 120 python bench.py --model cifar3 >> $O/bench.jsonl 2>>$O/bench.err || exit 1
timeout -k 10 180 python bench.py --model vgg11 --batch-per-gpu 256 --steps 10 --warmup 3 >> $O/bench.jsonl 2>>$O/bench.err || exit 1
cat $O/bench.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_vgg -o run --output-format csv -- python3 $R/bench.py --model vgg11 --batch-per-gpu 256 --steps 8 --warmup 2 --graph off > $O/prof_vgg.log 2>&1 || { tail $O/prof_vgg.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof_vgg > $O/vgg_summary.txt 2>&1
head -30 $O/vgg_summary.txt
