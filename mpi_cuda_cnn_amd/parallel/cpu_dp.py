"""CPU data-parallel trainer (torch.distributed "gloo") over the native fp32 /
fp64 CPU executor.

Same synchronisation semantics as the GPU path (``parallel.ddp``): identical
initial weights broadcast from rank 0, per-rank share of the global batch,
gradients pre-scaled by 1/(global batch), bucketed SUM all-reduce in reverse
stage order (``_C.plan_buckets``), then SGD.  It lets the distributed logic be
tested with world_size > 1 on machines without GPUs, and is the Python-side
twin of the native ``cnnmpi`` program.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .. import _C


class CpuDataParallel:
    def __init__(self, spec, params=None, dtype="fp64", group=None, bucket_bytes: int = 4 << 20, lr: float = 0.1):
        self.spec = spec
        self.net = (_C.CpuNet64 if dtype == "fp64" else _C.CpuNet32)(spec)
        self.np_dtype = np.float64 if dtype == "fp64" else np.float32
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.lr = lr
        if params is None:
            params = _C.init_params(spec, 0)
        p = torch.from_numpy(np.asarray(params, dtype=self.np_dtype).copy())
        if self.world > 1:
            dist.broadcast(p, src=0, group=group)
        self.net.set_params(p.numpy())
        self.buckets = _C.plan_buckets(spec, int(bucket_bytes))

    def step(self, x: np.ndarray, labels: np.ndarray, global_batch: int):
        """x: this rank's [b, C*H*W] (CHW, /255), labels: [b] int. Returns stats."""
        self.net.forward(np.ascontiguousarray(x, dtype=self.np_dtype))
        st = self.net.backward(np.ascontiguousarray(labels, dtype=np.int32), 1.0 / global_batch)
        g = torch.from_numpy(self.net.get_grads())
        if self.world > 1:
            works = [
                dist.all_reduce(g[off : off + cnt], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                for _hi, _lo, off, cnt in self.buckets
            ]
            for w in works:
                w.wait()
            self.net.set_grads(g.numpy())
        self.net.sgd(self.lr)
        return st

    def params(self) -> np.ndarray:
        return self.net.get_params()
