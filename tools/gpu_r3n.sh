#!/bin/bash
# Round-end rehearsal on the final tree: full GPU suite, smoke(), default bench, LeNet-5 kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r3n
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
grep -h '^{' $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 2 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python3 $R/tools/step_timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt && tail -1 $O/timeline.txt
