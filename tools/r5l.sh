set -o pipefail
OUT=r5l TESTS="tests/test_gpu_fp64.py" bash tools/gpu_job.sh || exit 1
OUT=r5l BENCH="--model ref --dtype fp64 --steps 10 --warmup 2 --batch-per-gpu 8192;--model ref --dtype fp64 --steps 10 --warmup 2;--model ref --dtype fp64 --steps 5 --warmup 2 --batch-per-gpu 65536;--model lenet5 --dtype fp64 --steps 10 --warmup 2" PROF="--model ref --dtype fp64 --steps 3 --warmup 1" PROF_LINES=45 bash tools/gpu_job.sh
