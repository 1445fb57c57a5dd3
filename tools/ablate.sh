#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for a in 0 1 2; do
  MCC_ABLATE=$a timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abl$a -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 > $R/gpurun_out/abl$a.log 2>&1 || exit 1
done
