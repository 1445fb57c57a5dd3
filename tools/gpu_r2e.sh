#!/bin/bash
# conv_rows dW ablation: staging vs MFMA loop (MCC_ABLATE 1/2), kernel times
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for a in 0 1 2 3; do
  MCC_ABLATE=$a timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/abl$a -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 2 --no-dist > $O/abl$a.log 2>&1 || { tail -5 $O/abl$a.log; exit 1; }
  echo "ablate=$a"; python $R/tools/prof_summary.py $O/abl$a | grep -E "conv_dw_rows|conv_pipe_fwd_kernel<0|conv_pipe_fwd_kernel<3|conv_dw_pipe|conv_pipe_fwd_kernel<1"
done
