#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=r5n TESTS="tests/test_gpu_refnet.py tests/test_gpu_engine.py::test_bf16_grads_per_channel_vs_rounded_oracle" \
BENCH="--model ref --steps 20 --warmup 5 --fp32-extra off;MCC_AB=ref_bwd1 --model ref --steps 20 --warmup 5 --fp32-extra off" \
PROF="--model ref --steps 5 --warmup 2 --fp32-extra off" bash tools/gpu_job.sh
