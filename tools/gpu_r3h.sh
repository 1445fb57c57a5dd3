#!/bin/bash
# xent head LDS sized by input width: numerics + bench + timeline
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/${OUT:-r3h}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.jsonl
for i in 1 2 3; do
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "run $i $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 2 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python3 $R/tools/step_timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt
grep -E "fc_|xent|dw_reduce_kernel|step" $O/timeline.txt | cut -c1-110
