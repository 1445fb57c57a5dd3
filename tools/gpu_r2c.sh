#!/bin/bash
# RCCL world-1 with the high-priority comm stream: bench A/B and overlap traces
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2c
mkdir -p $O
export MCC_COMM_TIMEOUT=120
timeout -k 10 180 python bench.py --steps 40 --warmup 10 > $O/bench_rccl.log 2>&1 || { tail -5 $O/bench_rccl.log; exit 1; }
grep metric $O/bench_rccl.log
timeout -k 10 180 python bench.py --steps 40 --warmup 10 --no-dist > $O/bench_local.log 2>&1 || { tail -5 $O/bench_local.log; exit 1; }
grep metric $O/bench_local.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_rccl.py > $O/pytest_rccl.log 2>&1 || { tail -30 $O/pytest_rccl.log; exit 1; }
tail -2 $O/pytest_rccl.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace_bench -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 3 --bucket-mb 0.01 > $O/trace_bench.log 2>&1 || { tail -5 $O/trace_bench.log; exit 1; }
python $R/tools/overlap_report.py $O/trace_bench 8 > $O/overlap_bench.txt 2>&1; cat $O/overlap_bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_vgg -o run --output-format csv -- $R/build/bin/cnn_dist --synthetic 640 --model vgg11 --batch 128 --epochs 1 --bucket-mb 32 --json - > $O/trace_vgg.log 2>&1 || { tail -5 $O/trace_vgg.log; exit 1; }
tail -2 $O/trace_vgg.log
python $R/tools/overlap_report.py $O/trace_vgg 12 > $O/overlap_vgg.txt 2>&1; cat $O/overlap_vgg.txt
