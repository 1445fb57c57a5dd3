#!/bin/bash
# Final-tree bench of every model (1 GPU, default batches)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3q
mkdir -p $O
: > $O/models.jsonl
for args in "--model lenet5" "--model lenet5 --dtype fp32 --batch-per-gpu 65536" "--model ref" "--model cifar3" "--model vgg11 --steps 10 --warmup 3"; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 $args > $O/one.json 2>$O/err.log || { tail $O/err.log; exit 1; }
  grep -h '^{' $O/one.json >> $O/models.jsonl
  python3 -c "import json;d=json.loads(open('$O/models.jsonl').read().splitlines()[-1]);print(d['config']['model'], d['dtype'], d['config']['batch_per_gpu'], d['value'], d['ms_per_step'])"
done
