#!/bin/bash
# Python GpuTrainer (bench.py, per-kernel launches) vs the native hipGraph
# trainer (cnn_hip) on the same LeNet-5 step, at the headline batch and a
# small batch where host launch cost could matter.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/nvp; mkdir -p $O
for B in 65536 8192; do
  timeout -k 10 120 python bench.py --batch-per-gpu $B --steps 40 --warmup 10 > $O/py_$B.json 2> $O/py_$B.err || { tail -3 $O/py_$B.err; exit 1; }
  echo "python bench B=$B: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/py_$B.json | tr '\n' ' ')"
  for g in "" "--no-graph"; do
    timeout -k 10 200 build/bin/cnn_hip --synthetic 1200000 --model lenet5 --batch $B --epochs 2 --quiet $g --json $O/native_${B}${g}.json > $O/native_${B}${g}.log 2>&1 || { tail -3 $O/native_${B}${g}.log; exit 1; }
    echo "cnn_hip B=$B ${g:-graph}: $(python -c "import json;d=json.load(open('$O/native_${B}${g}.json'));print({k:d[k] for k in d if k in ('train_img_per_s','steps','train_s','hipgraph','comm')})")"
  done
done
