#!/bin/bash
# One-factor sweep of the pipelined-conv planner knobs on the LeNet-5 bench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/sweep; mkdir -p $O
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 30 --warmup 8 --no-dist > $O/$l.json 2> $O/$l.err || { echo "$l FAILED"; tail -3 $O/$l.err; return 0; }
  echo "$l $(grep -o '"value": [0-9.]*' $O/$l.json)"
}
run base
for v in 32 48 96; do run fwdlds$v MCC_FWD_LDS_KB=$v; done
for v in 2 3 6; do run fwdwgs$v MCC_FWD_WGS=$v; done
for v in 32 48 96; do run dwlds$v MCC_DW_LDS_KB=$v; done
for v in 1 3; do run dwwgs$v MCC_DW_WGS=$v; done
