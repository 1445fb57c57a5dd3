"""High-level GPU trainer over the native engine.

One process per GPU.  The dataset (u8 NHWC images + labels) is resident in
HBM (MNIST is 47 MB; a 288 GB MI355X holds any of the configs' datasets many
times over), minibatches are sampled on the device and gathered by index
inside the first conv kernel, so there is no host data path in the step.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist
import torch.utils.dlpack

from . import _C
from .parallel.ddp import BucketedAllReduce, broadcast_params


def _alias(ptr: int, numel: int, dtype: str, device: int) -> torch.Tensor:
    return torch.utils.dlpack.from_dlpack(_C.dlpack_wrap(ptr, numel, dtype, device))


class GpuTrainer:
    def __init__(
        self,
        model="lenet5",
        dtype: str = "bf16",
        batch: int = 256,
        device: int | None = None,
        seed: int = 0,
        lr: float = 0.1,
        momentum: float = 0.0,
        weight_decay: float = 0.0,
        init: str = "glibc",
        params=None,
        group=None,
        bucket_bytes: int = 4 << 20,
        force_reduce: bool = False,
        split_sgd: bool | None = None,
    ):
        self.spec = _C.make_model(model) if isinstance(model, str) else model
        self.device = torch.cuda.current_device() if device is None else device
        torch.cuda.set_device(self.device)
        self.batch = batch
        self.lr, self.momentum, self.weight_decay = lr, momentum, weight_decay
        self.net = _C.GpuNet(self.spec, dtype, batch, self.device)
        n = self.spec.nparams
        if params is None:
            params = _C.init_params(self.spec, seed, init)
        self.net.set_params(np.asarray(params, dtype=np.float32))
        self.params = _alias(self.net.params_ptr, n, "float32", self.device)
        self.grads = _alias(self.net.grads_ptr, n, "float32", self.device)
        self.stats = _alias(self.net.stats_ptr, 4, "int64", self.device)  # u64 fixed point (get_stats decodes)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if dist.is_initialized():  # identical replicas (fixes D6: srand(rank), no broadcast)
            broadcast_params(self.params, 0, group)
            self.net.pack(self.stream)
        self.sync = BucketedAllReduce(self.net, self.grads, group, bucket_bytes, force_reduce)
        # per-bucket SGD (BucketedAllReduce.backward_update): default where a
        # collective can be in flight after the backward, i.e. world > 1
        self.split_sgd = (self.world > 1) if split_sgd is None else bool(split_sgd)

    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def step(self, images: torch.Tensor, labels: torch.Tensor, idx: torch.Tensor | None, batch: int | None = None):
        """One synchronous data-parallel SGD step (asynchronous w.r.t. the host)."""
        B = self.batch if batch is None else batch
        s = self.stream
        idx_ptr = 0 if idx is None else idx.data_ptr()
        self.net.forward(images.data_ptr(), idx_ptr, B, s)
        self.net.loss(labels.data_ptr(), idx_ptr, self.sync.loss_scale(B), True, s)
        if self.split_sgd and len(self.sync.buckets) > 1:
            self.sync.backward_update(
                s, lambda off, cnt: self.net.sgd_range(self.lr, self.momentum, self.weight_decay, off, cnt, s))
        else:
            self.sync.backward(s)
            self.net.sgd(self.lr, self.momentum, self.weight_decay, s)

    def zero_stats(self):
        self.net.zero_stats(self.stream)

    def evaluate(self, images: torch.Tensor, labels: torch.Tensor) -> tuple[int, int]:
        """Returns (ntests, ncorrect) over the whole (device-resident) set."""
        n = images.shape[0]
        s = self.stream
        self.net.zero_stats(s)
        for i in range(0, n, self.batch):
            nb = min(self.batch, n - i)
            idx = torch.arange(i, i + nb, device=images.device, dtype=torch.int32)
            self.net.forward(images.data_ptr(), idx.data_ptr(), nb, s)
            self.net.loss(labels.data_ptr(), idx.data_ptr(), 1.0, False, s)
        st = self.net.get_stats()
        return n, int(round(st["correct"]))

    def state_dict(self) -> np.ndarray:
        return self.net.get_params()


def drain_collective_watchdog(group=None) -> bool:
    """Block until the RCCL process group's watchdog holds no eager work.

    The watchdog thread polls the end event of every eager collective until it
    sees it complete, and HIP fails that query once the event's RCCL stream is
    capturing (hipErrorCapturedEvent: the watchdog then aborts the whole
    process -- seen once on the LeNet-5 bench in round 3).  Collectives issued
    during a capture are never handed to the watchdog, so the condition for a
    safe capture is exactly "its work list is empty", which
    ``ProcessGroup._wait_for_pending_works`` waits for (it takes the
    watchdog's own locks).  Returns False when there is no RCCL group."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_backend(group) != "nccl":
        return False
    pg = group if group is not None else dist.group.WORLD
    pg._wait_for_pending_works()
    return True


def capture_step(fn):
    """Capture ``fn()`` -- a training step that launches everything on the
    current stream (engine kernels, the device sampler, the bucketed RCCL
    all-reduces) -- into a HIP graph via ``torch.cuda.CUDAGraph`` and return
    ``(graph, None)``; ``(None, reason)`` if capture is not possible here.

    A replay re-issues every kernel and collective of the step with the
    captured pointers: callers keep their buffers (batch indices, sampler
    counter) alive and fixed.  Run ``fn`` eagerly at least once before (code
    objects loaded, RCCL communicator set up)."""
    torch.cuda.synchronize()
    drain_collective_watchdog()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            fn()
    except Exception as e:  # capture unsupported by a component: caller falls back to eager
        torch.cuda.synchronize()
        return None, f"{type(e).__name__}: {str(e)[:120]}"
    return g, None

