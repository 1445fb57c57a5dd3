set -o pipefail
OUT=r5m TESTS="tests" TEST_TIMEOUT=800 TEST_LINES=5 bash tools/gpu_job.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 || exit 1
OUT=r5m BENCH="--steps 20 --warmup 5" bash tools/gpu_job.sh && cat gpurun_out/r5m/bench_1.json
