#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=r5p TESTS="tests/test_gpu_refnet.py tests/test_gpu_engine.py" TEST_LINES=10 \
BENCH="--model ref --dtype fp32 --steps 10 --warmup 3 --fp32-extra off;--dtype fp32 --steps 10 --warmup 3 --fp32-extra off;MCC_AB=no_fc_dw32 --dtype fp32 --steps 10 --warmup 3 --fp32-extra off" \
PROF="--model ref --dtype fp32 --steps 3 --warmup 1 --fp32-extra off" bash tools/gpu_job.sh
