#!/bin/bash
# CIFAR-3conv side-stream A/B with the round-2 kernels and batch; the 2-rank bench rehearsal test
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3b
mkdir -p $O
: > $O/ab.jsonl
for ss in 1 0 1 0; do
  MCC_SIDE_STREAM=$ss timeout -k 10 180 python bench.py --model cifar3 --steps 20 --warmup 5 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "cifar3 side=$ss $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_programs.py -m gpu -x -q --timeout 150 --timeout-method thread -k "rehearsal or two_ranks" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
