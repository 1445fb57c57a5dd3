#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=r5w TESTS="tests/test_gpu_engine.py::test_vgg11_bench_batch_matches_small_batches tests/test_gpu_engine.py::test_step_matches_torch" TEST_LINES=4 \
BENCH="--model vgg11 --steps 5 --warmup 2;MCC_AB=big128pool --model vgg11 --steps 5 --warmup 2" PROF="--model vgg11 --steps 2 --warmup 1" PROF_LINES=50 bash tools/gpu_job.sh
