"""Multi-process data-parallel semantics on CPU (gloo, world_size 2), the
launcher's failure propagation, and the native MPI program.

The GPU path (RCCL over xGMI) uses the same bucket plan, the same loss
pre-scaling and the same broadcast-then-train protocol; the 8-GPU runs are
done by the driver's scaling bench.
"""

import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import mpi_cuda_cnn_amd as mcc
from mpi_cuda_cnn_amd.parallel.cpu_dp import CpuDataParallel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _batches(spec, steps, B, seed=0):
    C, H, W = spec.input_shape()
    imgs, labels = mcc.synth_dataset(steps * B, C, H, W, 10, seed=seed)
    x = (imgs.transpose(0, 3, 1, 2).reshape(steps * B, -1) / 255.0).astype(np.float64)
    return x.reshape(steps, B, -1), labels.reshape(steps, B).astype(np.int32)


def _worker(rank, world, port, model, steps, B, bucket_bytes, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = mcc.make_model(model)
    p0 = mcc.init_params(spec, seed=rank * 17)  # different per rank on purpose: broadcast must fix it
    dp = CpuDataParallel(spec, p0, group=None, bucket_bytes=bucket_bytes, lr=0.1)
    xs, ls = _batches(spec, steps, B)
    b = B // world
    for s in range(steps):
        dp.step(xs[s, rank * b : (rank + 1) * b], ls[s, rank * b : (rank + 1) * b], B)
    np.save(os.path.join(out, f"p{rank}.npy"), dp.params())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("model,bucket_bytes", [("lenet5", 4 << 20), ("lenet5", 4096), ("ref", 64 << 10)])
def test_dp_two_ranks_equals_single_process(model, bucket_bytes, tmp_path):
    steps, B = 3, 8
    mp.spawn(_worker, args=(2, _free_port(), model, steps, B, bucket_bytes, str(tmp_path)), nprocs=2, join=True)
    p0, p1 = np.load(tmp_path / "p0.npy"), np.load(tmp_path / "p1.npy")
    np.testing.assert_array_equal(p0, p1)  # replicas identical (defect D6 fixed)
    # single process, full batch
    spec = mcc.make_model(model)
    dp = CpuDataParallel(spec, mcc.init_params(spec, seed=0), lr=0.1)
    xs, ls = _batches(spec, steps, B)
    for s in range(steps):
        dp.step(xs[s], ls[s], B)
    np.testing.assert_allclose(p0, dp.params(), rtol=0, atol=1e-12)


def test_launcher_propagates_failure(tmp_path):
    from mpi_cuda_cnn_amd.launch import launch

    script = tmp_path / "w.py"
    script.write_text(
        "import os, sys, time\n"
        "r = int(os.environ['RANK'])\n"
        "assert os.environ['WORLD_SIZE'] == '3' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
        "if r == 1: sys.exit(7)\n"
        "time.sleep(60)\n"
    )
    rc = launch(3, [sys.executable, str(script)], timeout=30)
    assert rc == 7


def test_launcher_gloo_allreduce(tmp_path):
    from mpi_cuda_cnn_amd.launch import launch

    script = tmp_path / "ar.py"
    script.write_text(
        "import torch, torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "t = torch.tensor([float(dist.get_rank() + 1)])\n"
        "dist.all_reduce(t)\n"
        "assert t.item() == 3.0, t\n"
        "dist.destroy_process_group()\n"
    )
    assert launch(2, [sys.executable, str(script)], timeout=120) == 0


MPIEXEC = shutil.which("mpiexec") or ("/opt/conda/bin/mpiexec" if os.path.exists("/opt/conda/bin/mpiexec") else None)


@pytest.mark.skipif(MPIEXEC is None, reason="no MPI")
def test_cnnmpi_trains_and_replicas_agree(tmp_path):
    binp = os.path.join(ROOT, "build", "bin", "cnnmpi")
    if not os.path.exists(binp):
        r = subprocess.run(["make", "-C", ROOT, "build/bin/cnnmpi"], capture_output=True)
        if r.returncode != 0:
            pytest.skip("cnnmpi not buildable here")
    d = str(tmp_path)
    for n, s, p in ((400, 1, "train"), (100, 2, "test")):
        i, l = mcc.synth_dataset(n, 1, 28, 28, 10, seed=s)
        mcc.idx_write(os.path.join(d, p + "-images"), i.reshape(n, 28, 28))
        mcc.idx_write(os.path.join(d, p + "-labels"), l)
    args = [os.path.join(d, x) for x in ("train-images", "train-labels", "test-images", "test-labels")]
    w = os.path.join(d, "w.mcnnw")
    r = subprocess.run([MPIEXEC, "-n", "2", binp] + args + ["--epochs", "2", "--save", w], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "0 0 200" in r.stderr and "1 200 400" in r.stderr  # shard lines (cnnmpi.c:459)
    assert "epoch = 1" in r.stderr
    last = r.stderr.strip().splitlines()[-1]
    assert last.startswith("ntests=100, ncorrect=")
    assert int(last.split("=")[-1]) >= 95
    spec, p = mcc.load_weights(w)
    assert np.isfinite(p).all()


def test_rank_death_mid_training_fails_every_rank(tmp_path):
    """Failure detection (reference defect D9, cnnmpi.c:443-453): rank 1 dies
    abruptly mid-training; with NO launcher to kill the survivor, rank 0 must
    leave its collective and exit non-zero (111) within the deadline."""
    import time

    d = str(tmp_path)
    for n, s, p in ((512, 1, "train"), (64, 2, "test")):
        i, l = mcc.synth_dataset(n, 1, 28, 28, 10, seed=s)
        mcc.idx_write(os.path.join(d, p + "-images"), i.reshape(n, 28, 28))
        mcc.idx_write(os.path.join(d, p + "-labels"), l)
    args = [os.path.join(d, x) for x in ("train-images", "train-labels", "test-images", "test-labels")]
    port = str(_free_port())
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, MCC_COMM_TIMEOUT="30", MCC_FAULT_RANK="1", MCC_FAULT_STEP="3")
        procs.append(subprocess.Popen([sys.executable, "-m", "mpi_cuda_cnn_amd.train"] + args +
                                      ["--model", "lenet5", "--epochs", "4", "--batch", "16", "--device", "cpu"],
                                      cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    try:
        outs = [p.communicate(timeout=120) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.time() - t0
    assert procs[1].returncode == 17, outs[1][1]
    assert procs[0].returncode == 111, outs[0][1]
    assert elapsed < 100
