#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/probes/lds_unaligned > gpurun_out/lds_unaligned.txt 2>&1; cat gpurun_out/lds_unaligned.txt
R=$PWD
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/base_bench.json 2>gpurun_out/base_bench.err || exit 1
cat gpurun_out/base_bench.json
CTR="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" TAG=base1 ARGS="--steps 3 --warmup 1" KPAT=conv LINES_OUT=5 bash tools/gpu_pmc.sh || exit 1
CTR="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" TAG=base2 ARGS="--steps 3 --warmup 1" KPAT=conv LINES_OUT=5 bash tools/gpu_pmc.sh || exit 1
