#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5q
timeout -k 10 400 python -u -m pytest -m gpu -x -v -s --timeout 200 --timeout-method thread \
  "tests/test_gpu_engine.py::test_bench_batch_step_matches_small_batches" \
  "tests/test_gpu_engine.py::test_fc_igemm_bench_batch_matches_small_batches" \
  "tests/test_gpu_engine.py::test_bf16_grads_per_channel_vs_rounded_oracle[vgg224]" > gpurun_out/r5q/pytest.log 2>&1 || { tail -40 gpurun_out/r5q/pytest.log; exit 1; }
grep -E "PASSED|FAILED|per-channel|passed|failed" gpurun_out/r5q/pytest.log | head -80
OUT=r5q PROF="--dtype fp32 --steps 3 --warmup 1 --fp32-extra off" PROF_LINES=40 bash tools/gpu_job.sh
