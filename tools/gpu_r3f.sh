#!/bin/bash
# FC column split on the data gradient only (default 2) vs off; engine numerics with the default
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.jsonl
for f in 0 2 0 2 0 2; do
  MCC_FC_SPLIT=$f timeout -k 10 180 python bench.py --steps 30 --warmup 5 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "fcsplit=$f $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
