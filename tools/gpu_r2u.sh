#!/bin/bash
# dZ fused into the next stage's data-gradient epilogue: numerics + VGG-11 A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_igemm.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.jsonl
for f in 0 1 0 1; do
  MCC_DZ_FUSE=$f timeout -k 10 180 python bench.py --model vgg11 --steps 6 --warmup 2 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "dzfuse=$f $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
