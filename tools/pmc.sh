#!/bin/bash
# PMC counter passes over a short bench run (no trace domains other than kernel-trace).
cd "$(dirname "$0")/.."
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc $set -d $R/gpurun_out/pmc$i -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 ${BENCH_ARGS:-} > $R/gpurun_out/pmc$i.log 2>&1
  echo "pmc set $i ($set) rc=$?"
done
