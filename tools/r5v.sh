#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=r5v TESTS="tests/test_gpu_igemm.py tests/test_gpu_engine.py::test_bf16_grads_per_channel_vs_rounded_oracle tests/test_gpu_engine.py::test_vgg11_bench_batch_matches_small_batches tests/test_gpu_engine.py::test_igemm_conv_path_matches_torch" TEST_LINES=6 \
BENCH="--model vgg11 --steps 5 --warmup 2;MCC_AB=big128 --model vgg11 --steps 5 --warmup 2" PROF="--model vgg11 --steps 2 --warmup 1" PROF_LINES=60 bash tools/gpu_job.sh
