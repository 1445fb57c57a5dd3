#!/bin/bash
# LeNet-5 FC-path knobs at B=131072: weights-resident FC kernel vs tiled GEMM, fused head vs split
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r3d
for cfg in "MCC_X=0" "MCC_NO_FC=1" "MCC_NO_HEAD=1" "MCC_X=0"; do
  env $cfg timeout -k 10 100 python bench.py --steps 30 --warmup 5 > gpurun_out/r3d/knob.log 2>&1 || { echo "FAIL $cfg"; tail -3 gpurun_out/r3d/knob.log; exit 1; }
  echo "$cfg :: $(tail -1 gpurun_out/r3d/knob.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
