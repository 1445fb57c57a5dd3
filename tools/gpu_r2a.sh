#!/bin/bash
# Round 2 (a): RCCL at world 1 on the hardware path — GPU tests, bench with
# and without the RCCL process group, and a kernel trace of cnn_dist with
# many buckets (comm/compute overlap).
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2a
mkdir -p $O
export MCC_COMM_TIMEOUT=120
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_rccl.py tests/test_gpu_programs.py > $O/pytest_rccl.log 2>&1 || { tail -30 $O/pytest_rccl.log; exit 1; }
tail -3 $O/pytest_rccl.log
timeout -k 10 180 python bench.py --steps 40 --warmup 10 > $O/bench_rccl.log 2>&1 || { tail -5 $O/bench_rccl.log; exit 1; }
grep metric $O/bench_rccl.log
timeout -k 10 180 python bench.py --steps 40 --warmup 10 --no-dist > $O/bench_local.log 2>&1 || { tail -5 $O/bench_local.log; exit 1; }
grep metric $O/bench_local.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace_dist -o run --output-format csv -- $R/build/bin/cnn_dist --synthetic 262144 --model lenet5 --batch 65536 --epochs 1 --bucket-mb 0.01 --json - > $O/trace_dist.log 2>&1 || { tail -5 $O/trace_dist.log; exit 1; }
tail -2 $O/trace_dist.log
python $R/tools/overlap_report.py $O/trace_dist 8 > $O/overlap_dist.txt 2>&1; cat $O/overlap_dist.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace_bench -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 3 --bucket-mb 0.01 > $O/trace_bench.log 2>&1 || { tail -5 $O/trace_bench.log; exit 1; }
python $R/tools/overlap_report.py $O/trace_bench 8 > $O/overlap_bench.txt 2>&1; cat $O/overlap_bench.txt
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_all.log 2>&1 || { tail -30 $O/pytest_all.log; exit 1; }
tail -3 $O/pytest_all.log
