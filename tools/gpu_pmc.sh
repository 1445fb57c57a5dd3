#!/bin/bash
# One PMC pass over a bench config: CTR="counters" ARGS="bench args" KPAT=regex
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/pmc_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CTR=${CTR:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"}
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR -d $O/run -o run --output-format csv -- python $R/bench.py $ARGS --no-dist > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
python $R/tools/pmc_summary.py $O/run/run_counter_collection.csv > $O/summary.txt
grep -A12 -E "${KPAT:-igemm}" $O/summary.txt | head -${LINES_OUT:-60}
