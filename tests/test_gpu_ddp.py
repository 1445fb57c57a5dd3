"""Data-parallel GpuTrainer on the real GPU: two ranks sharing the one MI355X
of the test box (torch.distributed over gloo, since RCCL rejects two ranks on
one device) must end bit-for-bit identical to each other and equal, to fp32
rounding, to one process stepping the full batch.

This runs the exact multi-GPU code path of bench.py — GpuTrainer's
broadcast of rank 0's weights (fixes the reference's srand(rank) / no
broadcast, cnnmpi.c:423), BucketedAllReduce issuing one async all-reduce per
reverse-order bucket between the engine's backward stage ranges, the
1/(global batch) loss pre-scale and SGD with momentum — only the transport
differs from the driver's RCCL runs.
"""

import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import mpi_cuda_cnn_amd as mcc

STEPS, B, LR, MOM = 3, 64, 0.05, 0.9


def _data(spec):
    C, H, W = spec.input_shape()
    return mcc.synth_dataset(STEPS * B, C, H, W, spec.num_classes(), seed=5)


def _worker(rank, world, port, model, bucket_bytes, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from mpi_cuda_cnn_amd.trainer import GpuTrainer

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = mcc.make_model(model)
    imgs, labels = _data(spec)
    dev = torch.device("cuda", 0)
    d_img, d_lab = torch.from_numpy(imgs).to(dev), torch.from_numpy(labels).to(dev)
    b = B // world
    # different initial weights per rank on purpose: the broadcast must fix it
    tr = GpuTrainer(spec, dtype="fp32", batch=b, device=0, lr=LR, momentum=MOM,
                    params=mcc.init_params(spec, seed=rank * 17), bucket_bytes=bucket_bytes)
    assert len(tr.sync.buckets) >= 1
    for s in range(STEPS):
        idx = torch.arange(s * B + rank * b, s * B + (rank + 1) * b, device=dev, dtype=torch.int32)
        tr.step(d_img, d_lab, idx)
    torch.cuda.synchronize()
    np.save(os.path.join(out, f"p{rank}.npy"), tr.state_dict())
    np.save(os.path.join(out, f"nb{rank}.npy"), np.array(len(tr.sync.buckets)))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("model,bucket_bytes", [("lenet5", 4 << 20), ("lenet5", 16 << 10), ("cifar3", 64 << 10)])
def test_gpu_dp_two_ranks_equals_single_process(cuda, model, bucket_bytes, tmp_path):
    from mpi_cuda_cnn_amd.trainer import GpuTrainer

    mp.spawn(_worker, args=(2, _free_port(), model, bucket_bytes, str(tmp_path)), nprocs=2, join=True)
    p0, p1 = np.load(tmp_path / "p0.npy"), np.load(tmp_path / "p1.npy")
    np.testing.assert_array_equal(p0, p1)
    if bucket_bytes < (1 << 20):
        assert int(np.load(tmp_path / "nb0.npy")) > 1, "expected several buckets"

    spec = mcc.make_model(model)
    imgs, labels = _data(spec)
    d_img, d_lab = torch.from_numpy(imgs).to(cuda), torch.from_numpy(labels).to(cuda)
    tr = GpuTrainer(spec, dtype="fp32", batch=B, device=0, lr=LR, momentum=MOM,
                    params=mcc.init_params(spec, seed=0))
    for s in range(STEPS):
        idx = torch.arange(s * B, (s + 1) * B, device=cuda, dtype=torch.int32)
        tr.step(d_img, d_lab, idx)
    torch.cuda.synchronize()
    ref = tr.state_dict()
    p0_init = mcc.init_params(spec, seed=0).astype(np.float32)
    moved = np.linalg.norm(ref - p0_init)
    assert moved > 0
    assert np.linalg.norm(p0 - ref) < 2e-3 * max(moved, 1e-3) + 1e-6, (np.abs(p0 - ref).max(), moved)
