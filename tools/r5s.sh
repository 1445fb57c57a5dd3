#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_MISC"
OUT=r5s_lenet PROF="--steps 3 --warmup 1 --fp32-extra off" PMC="$P1;$P2" KPAT="lenet" PMC_LINES=200 bash tools/gpu_job.sh || exit 1
OUT=r5s_ref PROF="--model ref --steps 3 --warmup 1 --fp32-extra off" PMC="$P1;$P2" KPAT="ref_" PMC_LINES=200 bash tools/gpu_job.sh
