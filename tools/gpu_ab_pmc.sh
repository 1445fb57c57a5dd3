#!/bin/bash
# PMC A/B (one pass of 8 SQ counters): new tree vs build/ab_old, MCC_ABLATE=$ABL
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/abpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CTR=${CTR:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"}
for v in old new; do
  B=$R/bench.py; [ $v = old ] && B=$R/build/ab_old/bench.py
  MCC_ABLATE=${ABL:-0} timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTR -d $O/$v -o run --output-format csv -- python $B --steps 4 --warmup 2 --no-dist > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  python $R/tools/pmc_summary.py $O/$v/run_counter_collection.csv > $O/$v.txt
  echo "== $v"; grep -A9 "${KPAT:-conv_pipe_fwd_kernel<0, 0, 1, 2}" $O/$v.txt
done
