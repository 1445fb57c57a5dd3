#!/bin/bash
# conv_rows v2 (unconditional buffer loads, one-group-ahead index gather): tests, bench, profile, ablation
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; }
tail -1 $O/pytest.log
timeout -k 10 180 python bench.py --steps 40 --warmup 10 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench.log | tr '\n' ' '; echo
cd /tmp && export TMPDIR=/tmp
for a in 0 1 2; do
  MCC_ABLATE=$a timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/abl$a -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 2 --no-dist > $O/abl$a.log 2>&1 || { tail -5 $O/abl$a.log; exit 1; }
  echo "ablate=$a"; python $R/tools/prof_summary.py $O/abl$a | grep -E "conv_dw_rows|conv_pipe_fwd_kernel<0|conv_pipe_fwd_kernel<3|conv_dw_pipe|conv_pipe_fwd_kernel<1|total"
done
