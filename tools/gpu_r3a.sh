#!/bin/bash
# Rehearsal of bench.py's multi-rank logic (barriers, MAX of rank times, rank-0 JSON) with gloo,
# 2 and 4 ranks sharing the box's one GPU, as the driver launches it (torch.distributed.run).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3a
mkdir -p $O
for n in 2 4; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 2 --batch-per-gpu 16384 --dist-backend gloo \
    > $O/n$n.out 2> $O/n$n.err || { tail -20 $O/n$n.err; exit 1; }
  grep -c metric $O/n$n.out
  tail -1 $O/n$n.out | cut -c1-400
done
