#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=r5r TESTS="tests/test_gpu_engine.py tests/test_gpu_programs.py" TEST_LINES=8 \
BENCH="--dtype fp32 --steps 20 --warmup 5 --fp32-extra off;MCC_AB=no_head32 --dtype fp32 --steps 20 --warmup 5 --fp32-extra off;--model ref --dtype fp32 --steps 10 --warmup 3 --fp32-extra off" \
PROF="--dtype fp32 --steps 3 --warmup 1 --fp32-extra off" PROF_LINES=30 bash tools/gpu_job.sh
