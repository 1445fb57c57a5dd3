#!/bin/bash
# generic-activation convs (tanh, pool after a non-ReLU conv) + engine regression
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2s
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_igemm.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
grep -E "generic" $O/pytest.log; tail -1 $O/pytest.log
