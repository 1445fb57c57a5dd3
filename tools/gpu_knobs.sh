#!/bin/bash
# A/B of the pipelined-conv occupancy knobs (MCC_{DW,FWD}_{LDS_KB,WGS}) on the headline bench
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for cfg in "${@}"; do
  env $cfg timeout -k 10 100 python bench.py --steps 30 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/knob.log 2>&1 || { echo "FAIL $cfg"; tail -3 gpurun_out/knob.log; exit 1; }
  echo "$cfg :: $(grep -o '"value": [0-9.]*, [^,]*, [^,]*, [^,]*, [^,]*, "ms_per_step": [0-9.]*' gpurun_out/knob.log | sed 's/"unit.*ms_per/ms_per/')"
done
