#!/bin/bash
# FC persistent: next row block A loads issued right after the last MFMAs
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r3r
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 > $O/b_$i.json 2>$O/err.log || { tail $O/err.log; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 2 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
cd $R && for i in 1 2 3; do grep -h '^{' $O/b_$i.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])"; done
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r3r/prof/run_kernel_stats.csv")):
    if "fc_kernel" in r["Name"] or "xent" in r["Name"]: print(r["Name"][40:90], r["Calls"], r["AverageNs"])
PY
