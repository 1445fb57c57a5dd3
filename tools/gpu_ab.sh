#!/bin/bash
# Same-box A/B of the LeNet-5 bench kernels: new tree vs build/ab_old
# (tools/ab_build.sh), each with MCC_ABLATE in $ABL (default "0 1 2").
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  B=$R/bench.py; [ $v = old ] && B=$R/build/ab_old/bench.py
  timeout -k 10 180 python $B --steps 30 --warmup 10 > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; exit 1; }
  echo "$v: $(grep -o '"value": [0-9.]*' $O/bench_$v.log)"
  for a in ${ABL:-0 1 2}; do
    MCC_ABLATE=$a timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${v}_$a -o run --output-format csv -- python $B --steps 10 --warmup 2 --no-dist > $O/${v}_$a.log 2>&1 || { tail -5 $O/${v}_$a.log; exit 1; }
    echo "$v ablate=$a"; python $R/tools/prof_summary.py $O/${v}_$a | grep -E "${KPAT:-conv_dw_rows|conv_pipe_fwd_kernel<0}"
  done
done
