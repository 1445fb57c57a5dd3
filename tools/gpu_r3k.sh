#!/bin/bash
# LeNet-5 FC1 data gradient: column parts 2 / 3 / 4 (MCC_FC_PARTS), kernel time + step time
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r3k
mkdir -p $O
MCC_FC_PARTS=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for parts in 2 3 4 2; do
  export MCC_FC_PARTS=$parts
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 > $O/b_$parts.json 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "parts=$parts $(python -c "import json;d=json.load(open('$O/b_$parts.json'));print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
for parts in 2 3 4; do
  export MCC_FC_PARTS=$parts
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof$parts -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 2 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
  echo "parts=$parts $(grep -h 'fc_kernel<2, 0' $O/prof$parts/run_kernel_stats.csv | cut -d, -f1-4)"
done
