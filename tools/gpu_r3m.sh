#!/bin/bash
# 8-wave FC kernel: column split mode A/B (MCC_FC_SPLIT 0 never / 1 fwd+dgrad / 2 dgrad only)
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r3m
mkdir -p $O
for m in 2 0 1 2; do
  export MCC_FC_SPLIT=$m
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 > $O/b_$m.json 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "split=$m $(grep -h '^{' $O/b_$m.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
for m in 0 1 2; do
  export MCC_FC_SPLIT=$m
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof$m -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 2 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv
for m in (0, 1, 2):
    print("split", m)
    for r in csv.DictReader(open(f"gpurun_out/r3m/prof{m}/run_kernel_stats.csv")):
        if "fc_kernel" in r["Name"]: print("  ", r["Name"][40:90], r["AverageNs"])
PY
