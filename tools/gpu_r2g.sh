#!/bin/bash
# PMC counters of the conv kernels (LeNet-5 bench step), two passes
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d $O/pmc$i -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 2 --no-dist > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 1; }
done
python $R/tools/pmc_summary.py $O/pmc1/run_counter_collection.csv $O/pmc2/run_counter_collection.csv > $O/pmc_summary.txt
grep -A16 "conv_dw_rows\|conv_pipe_fwd_kernel<" $O/pmc_summary.txt | head -80
