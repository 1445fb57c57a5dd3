#!/bin/bash
# One GPU session: tests, bench sweep, rocprof kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
for b in 4096 16384 65536; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --batch-per-gpu $b >> gpurun_out/bench_sweep.log 2>&1 || { echo "bench $b failed"; exit 1; }
done
cat gpurun_out/bench_sweep.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1; echo "prof rc=$?"
