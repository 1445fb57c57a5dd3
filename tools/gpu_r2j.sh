#!/bin/bash
# Full GPU suite + LeNet-5 / VGG-11 bench after the 256-tile kernels and the SUM all-reduce.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2j
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python bench.py > $O/bench.jsonl 2>$O/bench.err || { tail $O/bench.err; exit 1; }
timeout -k 10 180 python bench.py --model vgg11 --batch-per-gpu 256 --steps 10 --warmup 3 >> $O/bench.jsonl 2>>$O/bench.err || exit 1
timeout -k 10 120 python bench.py --model cifar3 >> $O/bench.jsonl 2>>$O/bench.err || exit 1
grep metric $O/bench.jsonl | python -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['config']['model'], d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_vgg -o run --output-format csv -- python3 $R/bench.py --model vgg11 --batch-per-gpu 256 --steps 8 --warmup 2 --graph off > $O/prof_vgg.log 2>&1 || { tail $O/prof_vgg.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof_vgg > $O/vgg_summary.txt 2>&1
python3 $R/tools/step_timeline.py $O/prof_vgg/run_kernel_trace.csv > $O/vgg_timeline.txt
head -16 $O/vgg_summary.txt
tail -1 $O/vgg_timeline.txt
