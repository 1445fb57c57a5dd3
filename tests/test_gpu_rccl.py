"""RCCL on the hardware path at one rank (the box has one MI355X; RCCL refuses
two ranks on one device).  A world-1 RCCL communicator executes the same
broadcast, bucketed all-reduce on a separate stream and (native) graph-captured
collectives as the 8-GPU runs; at one rank the sum is the identity, so the
trained weights must be BIT-equal to the collective-free path.

  * Python: GpuTrainer under a world-1 "nccl" process group (bench.py's N=1
    path) vs no process group.
  * Native: cnn_dist with its RcclComm (hipGraph replay, eager, --profile)
    vs --comm local.
"""

import json
import os
import subprocess

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import mpi_cuda_cnn_amd as mcc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS, B, LR, MOM, BUCKET = 4, 256, 0.05, 0.9, 16 << 10


def _train(model, dtype, force=False):
    from mpi_cuda_cnn_amd.trainer import GpuTrainer

    dev = torch.device("cuda", 0)
    spec = mcc.make_model(model)
    C, H, W = spec.input_shape()
    imgs, labels = mcc.synth_dataset(STEPS * B, C, H, W, spec.num_classes(), seed=9)
    d_img, d_lab = torch.from_numpy(imgs).to(dev), torch.from_numpy(labels).to(dev)
    tr = GpuTrainer(spec, dtype=dtype, batch=B, device=0, lr=LR, momentum=MOM,
                    params=mcc.init_params(spec, seed=3, mode="fast"), bucket_bytes=BUCKET, force_reduce=force)
    for s in range(STEPS):
        idx = torch.arange(s * B, (s + 1) * B, device=dev, dtype=torch.int32)
        tr.step(d_img, d_lab, idx)
    torch.cuda.synchronize()
    return tr.state_dict(), len(tr.sync.buckets), tr.sync.issued


def _rccl_worker(rank, model, dtype, out, force=False):
    import torch.distributed as dist

    from mpi_cuda_cnn_amd.parallel.ddp import init_process_group

    os.environ.pop("MASTER_PORT", None)
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    init_process_group("nccl", torch.device("cuda", 0))
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    p, nb, issued = _train(model, dtype, force)
    np.save(os.path.join(out, "p.npy"), p)
    np.save(os.path.join(out, "n.npy"), np.array([nb, issued]))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("model,dtype,force", [("lenet5", "bf16", False), ("cifar3", "bf16", False),
                                               ("ref", "fp32", False), ("lenet5", "bf16", True)])
def test_python_rccl_world1_bit_equal(cuda, model, dtype, force, tmp_path):
    """force: bench.py --force-reduce (a real one-rank AVG reduction kernel per bucket) is bit-equal too."""
    mp.spawn(_rccl_worker, args=(model, dtype, str(tmp_path), force), nprocs=1, join=True)
    p_rccl = np.load(tmp_path / "p.npy")
    nb, issued = np.load(tmp_path / "n.npy")
    assert nb > 1, "expected several buckets"
    assert issued == STEPS * nb, "one RCCL all-reduce per bucket per step"
    import torch.distributed as dist

    assert not dist.is_initialized()
    p_local, nb2, issued2 = _train(model, dtype)
    assert issued2 == 0 and nb2 == nb
    np.testing.assert_array_equal(p_rccl, p_local)


@pytest.fixture(scope="module")
def idx_files(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("rcclidx"))
    for n, s, p in ((4096, 1, "train"), (512, 2, "test")):
        i, l = mcc.synth_dataset(n, 1, 28, 28, 10, seed=s)
        mcc.idx_write(os.path.join(d, p + "-images"), i.reshape(n, 28, 28))
        mcc.idx_write(os.path.join(d, p + "-labels"), l)
    return [os.path.join(d, x) for x in ("train-images", "train-labels", "test-images", "test-labels")]


def _cnn_dist(idx_files, w, extra, env_extra=None):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MCC_COMM_TIMEOUT="120")
    env.pop("MCC_AB", None)
    env.update(env_extra or {})
    r = subprocess.run([os.path.join(ROOT, "build/bin/cnn_dist")] + idx_files +
                       ["--model", "lenet5", "--batch", "512", "--epochs", "1", "--lr", "0.05", "--momentum", "0.9",
                        "--bucket-mb", "0.01", "--json", "-", "--save", w] + extra,
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1]), mcc.load_weights(w)[1]


@pytest.mark.gpu
def test_cnn_dist_rccl_world1_bit_equal(idx_files, tmp_path):
    js_g, p_g = _cnn_dist(idx_files, str(tmp_path / "g.w"), [])
    assert js_g["comm"] == "rccl" and js_g["hipgraph"] is True and js_g["buckets"] > 1
    js_e, p_e = _cnn_dist(idx_files, str(tmp_path / "e.w"), ["--no-graph"])
    assert js_e["comm"] == "rccl" and js_e["hipgraph"] is False
    js_p, p_p = _cnn_dist(idx_files, str(tmp_path / "p.w"), ["--profile"])
    assert js_p["comm"] == "rccl" and "phase_ms" in js_p
    js_l, p_l = _cnn_dist(idx_files, str(tmp_path / "l.w"), ["--comm", "local"])
    assert js_l["comm"] == "local" and js_l["hipgraph"] is True
    np.testing.assert_array_equal(p_g, p_l)  # RCCL world-1 == no collectives
    np.testing.assert_array_equal(p_g, p_e)  # graph replay == eager
    np.testing.assert_array_equal(p_g, p_p)  # --profile (event-timed phases) == graph
    assert js_g["ncorrect"] >= 0.9 * js_g["ntests"]


def _graph_worker(rank, out):
    """Eager steps vs one eager step + HIP-graph replays of the captured step
    (bench.py --graph), both under the world-1 RCCL group, same init."""
    import torch.distributed as dist

    from mpi_cuda_cnn_amd.parallel.ddp import init_process_group
    from mpi_cuda_cnn_amd.trainer import GpuTrainer, capture_step

    os.environ.pop("MASTER_PORT", None)
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    init_process_group("nccl", dev)
    spec = mcc.make_model("lenet5")
    imgs, labels = mcc.synth_dataset(4096, 1, 28, 28, 10, seed=9)
    d_img, d_lab = torch.from_numpy(imgs).to(dev), torch.from_numpy(labels).to(dev)
    K = mcc._C.kernels
    res = []
    for graphed in (False, True):
        tr = GpuTrainer(spec, dtype="bf16", batch=B, device=0, lr=LR, momentum=MOM,
                        params=mcc.init_params(spec, seed=3, mode="fast"), bucket_bytes=BUCKET)
        idx = torch.empty(B, dtype=torch.int32, device=dev)
        ctr = torch.zeros(1, dtype=torch.int64, device=dev)

        def launch():
            s = torch.cuda.current_stream().cuda_stream
            K.sample_indices(idx.data_ptr(), B, 0, 4096, 77, ctr.data_ptr(), s)
            tr.step(d_img, d_lab, idx)
            K.advance_counter(ctr.data_ptr(), s)

        launch()
        torch.cuda.synchronize()
        if graphed:
            g, why = capture_step(launch)
            assert g is not None, why
            for _ in range(STEPS):
                g.replay()
        else:
            for _ in range(STEPS):
                launch()
        torch.cuda.synchronize()
        res.append((tr.state_dict(), int(ctr.item()), tr.sync.issued, len(tr.sync.buckets)))
    (pe, ce, ie, nb), (pg, cg, ig, _) = res
    np.save(os.path.join(out, "pe.npy"), pe)
    np.save(os.path.join(out, "pg.npy"), pg)
    np.save(os.path.join(out, "meta.npy"), np.array([ce, cg, ie, ig, nb]))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_python_graph_replay_bit_equal(cuda, tmp_path):
    """bench.py's graph mode: a captured step (device sampler, engine kernels,
    bucketed RCCL all-reduces, fused SGD) replayed K times gives BIT-equal
    weights to K eager steps, and every replay really advances the sampler."""
    mp.spawn(_graph_worker, args=(str(tmp_path),), nprocs=1, join=True)
    pe, pg = np.load(tmp_path / "pe.npy"), np.load(tmp_path / "pg.npy")
    ce, cg, ie, ig, nb = np.load(tmp_path / "meta.npy")
    assert ce == cg == STEPS + 1, (ce, cg)
    assert ie == (STEPS + 1) * nb and ig == 2 * nb, (ie, ig, nb)  # eager: every step; graph: eager + capture
    assert not np.array_equal(pe, mcc.init_params(mcc.make_model("lenet5"), seed=3, mode="fast"))
    np.testing.assert_array_equal(pe, pg)


def _capture_cycles_worker(rank, out):
    """Eager step (its collectives go to the process-group watchdog) and a
    graph capture right after it, several times over, with no pause between:
    capture_step must wait for the watchdog to retire the eager work
    (drain_collective_watchdog) instead of racing it."""
    import torch.distributed as dist

    from mpi_cuda_cnn_amd.parallel.ddp import init_process_group
    from mpi_cuda_cnn_amd.trainer import GpuTrainer, capture_step, drain_collective_watchdog

    os.environ.pop("MASTER_PORT", None)
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    init_process_group("nccl", dev)
    spec = mcc.make_model("lenet5")
    imgs, labels = mcc.synth_dataset(2048, 1, 28, 28, 10, seed=5)
    d_img, d_lab = torch.from_numpy(imgs).to(dev), torch.from_numpy(labels).to(dev)
    tr = GpuTrainer(spec, dtype="bf16", batch=B, device=0, lr=LR, momentum=MOM,
                    params=mcc.init_params(spec, seed=3, mode="fast"), bucket_bytes=BUCKET)
    idx = torch.arange(B, dtype=torch.int32, device=dev)
    ok = 0
    for _ in range(6):
        tr.step(d_img, d_lab, idx)  # eager: RCCL works queued on the watchdog
        g, why = capture_step(lambda: tr.step(d_img, d_lab, idx))
        assert g is not None, why
        g.replay()
        torch.cuda.synchronize()
        ok += 1
    assert drain_collective_watchdog() is True
    np.save(os.path.join(out, "ok.npy"), np.array([ok, tr.sync.issued]))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_capture_right_after_eager_collectives(cuda, tmp_path):
    mp.spawn(_capture_cycles_worker, args=(str(tmp_path),), nprocs=1, join=True)
    ok, issued = np.load(tmp_path / "ok.npy")
    assert ok == 6 and issued > 0
