#!/bin/bash
# Per-kernel time with MCC_ABLATE bit sets (1 no staging, 2 no MFMA loop, 4 no epilogue)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for a in ${ABLATE_SETS:-0 1 2 4}; do
  MCC_ABLATE=$a timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abl$a -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 > $R/gpurun_out/abl$a.log 2>&1 || exit 1
  python3 $R/tools/prof_summary.py $R/gpurun_out/abl$a > $R/gpurun_out/abl${a}_sum.txt
done
