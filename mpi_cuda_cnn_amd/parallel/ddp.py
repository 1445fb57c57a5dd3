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
* the collective is SUM and the loss gradient is pre-scaled by 1/(global
  batch), so the update uses the global-batch mean gradient.  (ncclAvg would
  scale inside the reduction, but RCCL implements it as a pre-multiplied sum
  that, at one rank, still launches a full read+write "oneRankReduce" pass
  over the buffer: 0.96 ms per VGG-11 step for nothing; an in-place one-rank
  SUM is elided by RCCL while the same call path still runs.)
* initial weights are broadcast from rank 0 (fixes D6: ``srand(rank)``).

Bucket size: xGMI is point-to-point (7 links x ~153 GB/s per MI355X); a ring
all-reduce is per-link bound and tiny messages are latency bound.  LeNet-5's
whole gradient is 247 KB, so the default (4 MiB) gives ONE collective per step;
VGG-11's 532 MB splits into ~25 MB buckets that overlap with backward.
"""

from __future__ import annotations

import datetime
import os
import socket

import torch
import torch.distributed as dist


def comm_timeout() -> datetime.timedelta:
    """Deadline of every collective (MCC_COMM_TIMEOUT seconds, default 300):
    a rank that dies mid-step makes its peers' collectives fail after this
    long instead of hanging forever (reference defect D9, cnnmpi.c:443-453)."""
    try:
        t = float(os.environ.get("MCC_COMM_TIMEOUT", "300"))
    except ValueError:
        t = 300.0
    return datetime.timedelta(seconds=t if t > 0 else 300.0)


def init_process_group(backend: str, device: torch.device | None = None):
    """torch.distributed init with the framework's defaults: env:// rendezvous
    on 127.0.0.1 (a free port when launched without a launcher, world 1), the
    collective deadline of comm_timeout(), and for "nccl" (= RCCL) the device
    bound eagerly so the communicator is created now, not at the first
    collective.  World 1 is a real process group too: the single-GPU run
    executes the same RCCL broadcast and bucketed all-reduce as an 8-GPU one."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    own_port = "MASTER_PORT" not in os.environ

    def pick_port():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])

    if own_port:
        pick_port()
    kw = {"timeout": comm_timeout()}
    if backend == "nccl":
        # No recycled HIP events between collectives: with the cache on, the
        # events of collectives captured into a HIP graph (bench.py --graph)
        # return to the cache "last recorded in a capturing stream", a later
        # eager collective inherits one, and the process-group watchdog's
        # query of it fails (hipErrorCapturedEvent -> abort; seen 1 in 7 runs).
        os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
        if device is not None:
            kw["device_id"] = device
        # RCCL's stream from the high-priority pool: HIP maps streams onto
        # GPU_MAX_HW_QUEUES (4) hardware queues per priority, and a
        # normal-priority pool stream can land on the compute stream's queue,
        # which serialises every all-reduce behind the backward kernels
        # (measured: tools/probes/queue_probe.py, profiles/rccl_world1_r2.txt).
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        kw["pg_options"] = opts
    # A port we picked ourselves is free when probed but can be taken before
    # the store binds it (seen once on a GPU box: EADDRINUSE between two
    # back-to-back bench runs): pick another and retry.  A launcher-given
    # port is shared with the other ranks and is never changed here.
    for attempt in range(5 if own_port else 1):
        try:
            dist.init_process_group(backend, **kw)
            return
        except dist.DistNetworkError as e:
            if not own_port or "EADDRINUSE" not in str(e) or attempt == 4:
                raise
            pick_port()


class BucketedAllReduce:
    """Issues one SUM all-reduce per bucket whenever a process group exists
    (any world size, 1 included: with the "nccl" backend that is a real RCCL
    collective on RCCL's stream)."""

    def __init__(self, net, grads: torch.Tensor, group=None, bucket_bytes: int = 4 << 20,
                 force_kernel: bool = False):
        self.net = net
        self.grads = grads
        self.group = group
        self.active = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.active else 1
        self.op = dist.ReduceOp.SUM
        # force_kernel: make the one-rank collective a real reduction kernel
        # (AVG = a pre-multiplied sum; x * 1 is exact, so the result is
        # bit-identical) to measure comm/compute contention on one GPU.  At
        # world > 1 the SUM already runs RCCL's ring kernels.
        self.elided = self.active and self.world == 1 and not force_kernel
        if self.active and self.world == 1 and force_kernel:
            self.op = dist.ReduceOp.AVG
        self.buckets = [tuple(b) for b in net.buckets(int(bucket_bytes))]
        self.issued = 0  # collectives issued so far (introspection / tests)
        covered = sum(b[3] for b in self.buckets)
        assert covered == grads.numel(), "buckets must cover the whole gradient buffer"

    def loss_scale(self, local_batch: int) -> float:
        """Gradient scale for the loss of `local_batch` samples on this rank."""
        return 1.0 / (local_batch * self.world)

    def backward(self, stream_handle: int):
        """Run the engine backward bucket by bucket, launching each bucket's
        all-reduce as soon as its gradients are enqueued; returns when every
        collective has been ordered before subsequent work on the current
        stream (host does not block)."""
        works = []
        for hi, lo, off, cnt in self.buckets:
            self.net.backward(hi, lo, stream_handle)
            if self.active:
                works.append(
                    dist.all_reduce(self.grads[off : off + cnt], op=self.op, group=self.group, async_op=True)
                )
        self.issued += len(works)
        for w in works:
            w.wait()

    def backward_update(self, stream_handle: int, update):
        """backward() with the update split per bucket: every bucket's
        all-reduce is issued as in backward(), then, in issue order, the
        compute stream joins bucket k's collective and calls
        ``update(off, count)`` for its parameter range (GpuNet.sgd_range).
        The update of the early buckets (LeNet-5: the FC stages, 96 % of the
        bytes) runs while the last bucket's collective -- the one issued after
        the fused conv-block backward -- is still in flight, so only the
        small conv-parameter update waits for it.  Bit-identical to
        backward() + a whole-buffer SGD (the update is elementwise)."""
        works = []
        for hi, lo, off, cnt in self.buckets:
            self.net.backward(hi, lo, stream_handle)
            works.append(dist.all_reduce(self.grads[off : off + cnt], op=self.op, group=self.group, async_op=True)
                         if self.active else None)
        self.issued += sum(w is not None for w in works)
        for (hi, lo, off, cnt), w in zip(self.buckets, works):
            if w is not None:
                w.wait()
            update(off, cnt)


def broadcast_params(params: torch.Tensor, src: int = 0, group=None):
    if dist.is_initialized():
        dist.broadcast(params, src=src, group=group)
