set -o pipefail
OUT=r5h TESTS="tests/test_gpu_lenet.py tests/test_gpu_engine.py tests/test_gpu_lenet_fc.py tests/test_gpu_rccl.py tests/test_gpu_ddp.py" bash tools/gpu_job.sh || exit 1
OUT=r5h BENCH="--steps 20 --warmup 5;--steps 20 --warmup 5" PROF="--steps 3 --warmup 2 --fp32-extra off" bash tools/gpu_job.sh
