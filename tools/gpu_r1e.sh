#!/bin/bash
# every model config (1 GPU), VGG PMC passes (MFMA busy, LDS), hipBLASLt ceiling probe
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
bash tools/bench_models.sh || exit 1
timeout -k 10 200 python tools/probes/blas_ceiling.py > gpurun_out/blas_ceiling.log 2>&1 || { tail -5 gpurun_out/blas_ceiling.log; exit 1; }
BENCH_ARGS="--model vgg11 --batch-per-gpu 128" bash tools/pmc.sh \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA"
