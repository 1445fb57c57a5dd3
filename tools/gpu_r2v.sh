#!/bin/bash
# fused-dZ variants A/B on VGG-11 (B=512) + step timeline of mode 2
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2v
mkdir -p $O
: > $O/ab.jsonl
for f in 0 2 0 2; do
  MCC_DZ_FUSE=$f timeout -k 10 180 python bench.py --model vgg11 --steps 6 --warmup 2 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "dzfuse=$f $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
MCC_DZ_FUSE=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --model vgg11 --steps 4 --warmup 2 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python3 $R/tools/step_timeline.py $O/prof/run_kernel_trace.csv > $O/timeline_fuse1.txt
