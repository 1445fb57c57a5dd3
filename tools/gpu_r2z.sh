#!/bin/bash
# pipelined-conv occupancy knobs re-tuned at the round-2 LeNet-5 batch (131072)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2z
for cfg in "MCC_X=0" "MCC_DW_WGS=3" "MCC_DW_WGS=4" "MCC_FWD_WGS=3" "MCC_FWD_WGS=6" "MCC_FWD_LDS_KB=48" "MCC_FWD_LDS_KB=80" "MCC_DW_LDS_KB=48" "MCC_DW_LDS_KB=96" "MCC_X=0"; do
  env $cfg timeout -k 10 100 python bench.py --steps 30 --warmup 5 > gpurun_out/r2z/knob.log 2>&1 || { echo "FAIL $cfg"; tail -3 gpurun_out/r2z/knob.log; exit 1; }
  echo "$cfg :: $(tail -1 gpurun_out/r2z/knob.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
