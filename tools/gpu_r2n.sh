#!/bin/bash
# CIFAR-3conv: implicit GEMM for the wide small-image conv (MCC_IGEMM_SMALL) numerics + A/B; VGG batch 512
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2n
mkdir -p $O
MCC_IGEMM_SMALL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.jsonl
for m in 0 1 0 1; do
  MCC_IGEMM_SMALL=$m timeout -k 10 180 python bench.py --model cifar3 --steps 20 --warmup 5 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "small=$m $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 180 python bench.py --model vgg11 --batch-per-gpu 512 --steps 6 --warmup 2 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
echo "vgg512 $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
cd /tmp && export TMPDIR=/tmp
MCC_IGEMM_SMALL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c -o run --output-format csv -- python3 $R/bench.py --model cifar3 --steps 8 --warmup 2 --graph off > $O/prof_c.log 2>&1 || { tail $O/prof_c.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof_c > $O/cifar_summary.txt 2>&1
head -16 $O/cifar_summary.txt
