"""Data-parallel gradient synchronisation over RCCL (torch.distributed "nccl").

Replaces the reference's per-sample, per-layer blocking ``MPI_Allreduce`` of
the wrong buffer (cnnmpi.c:487-498, defects D4/D5) with:

* one flat fp32 gradient buffer owned by the native engine, aliased into torch
  via DLPack — no copies, the collective runs in place;
* buckets = contiguous suffix ranges of that buffer in reverse stage order, so
  bucket 0 is complete as soon as the last stages' backward kernels finish;
* each bucket's all-reduce is issued with ``async_op=True`` right after its
  stages' backward kernels are enqueued: RCCL runs it on its own HIP stream
  (ordered after the producing kernels by an event) while the compute stream
  continues with the earlier stages' backward — comm/compute overlap on xGMI;
* the loss gradient is pre-scaled by 1/(global batch), so SUM == mean;
* initial weights are broadcast from rank 0 (fixes D6: ``srand(rank)``).

Bucket size: xGMI is point-to-point (7 links x ~153 GB/s per MI355X); a ring
all-reduce is per-link bound and tiny messages are latency bound.  LeNet-5's
whole gradient is 247 KB, so the default (4 MiB) gives ONE collective per step;
VGG-11's 532 MB splits into ~25 MB buckets that overlap with backward.
"""

from __future__ import annotations

import torch
import torch.distributed as dist


class BucketedAllReduce:
    def __init__(self, net, grads: torch.Tensor, group=None, bucket_bytes: int = 4 << 20):
        self.net = net
        self.grads = grads
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.buckets = [tuple(b) for b in net.buckets(int(bucket_bytes))]
        covered = sum(b[3] for b in self.buckets)
        assert covered == grads.numel(), "buckets must cover the whole gradient buffer"

    def backward(self, stream_handle: int):
        """Run the engine backward bucket by bucket, launching each bucket's
        all-reduce as soon as its gradients are enqueued; returns when every
        collective has been ordered before subsequent work on the current
        stream (host does not block)."""
        works = []
        for hi, lo, off, cnt in self.buckets:
            self.net.backward(hi, lo, stream_handle)
            if self.world > 1:
                works.append(
                    dist.all_reduce(self.grads[off : off + cnt], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                )
        for w in works:
            w.wait()


def broadcast_params(params: torch.Tensor, src: int = 0, group=None):
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(params, src=src, group=group)
