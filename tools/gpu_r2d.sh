#!/bin/bash
# conv1 dW on the row-chunked kernel: numerics, bench, kernel stats
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gpu_kernels.py tests/test_gpu_igemm.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
timeout -k 10 180 python bench.py --steps 40 --warmup 10 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench.log | tr '\n' ' '; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python $R/tools/prof_summary.py $O/prof | head -24
