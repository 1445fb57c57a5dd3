#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=r5u TESTS="tests/test_gpu_igemm.py tests/test_gpu_engine.py" TEST_LINES=6 TEST_TIMEOUT=700 \
BENCH="--model vgg11 --steps 5 --warmup 2;--model cifar3 --steps 10 --warmup 3" bash tools/gpu_job.sh || exit 1
PROBE_MODEL=vgg11 PROBE_B=640 timeout -k 10 300 python tools/probes/lenet_phase_probe.py
