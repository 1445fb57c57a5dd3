#!/bin/bash
# Round-end rehearsal: full GPU suite, smoke(), default bench exactly as the driver runs it, fp32 bench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2t
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
