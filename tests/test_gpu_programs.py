"""End-to-end GPU programs on the MI355X: the native `cnn_hip` / `cnn_dist`
drivers (hipGraph-captured step) and the Python trainer, on synthetic
MNIST-shaped IDX data with the reference CLI."""

import json
import os
import subprocess
import sys

import pytest

import mpi_cuda_cnn_amd as mcc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def idx_files(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("gpuidx"))
    for n, s, p in ((4000, 1, "train"), (1000, 2, "test")):
        i, l = mcc.synth_dataset(n, 1, 28, 28, 10, seed=s)
        mcc.idx_write(os.path.join(d, p + "-images"), i.reshape(n, 28, 28))
        mcc.idx_write(os.path.join(d, p + "-labels"), l)
    return [os.path.join(d, x) for x in ("train-images", "train-labels", "test-images", "test-labels")]


def _run(cmd, **kw):
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("model,dtype,batch", [("lenet5", "bf16", 256), ("ref", "fp32", 32)])
def test_cnn_hip_trains(idx_files, model, dtype, batch, tmp_path):
    w = str(tmp_path / "w.mcnnw")
    r = _run([os.path.join(ROOT, "build/bin/cnn_hip")] + idx_files +
             ["--model", model, "--dtype", dtype, "--batch", str(batch), "--epochs", "2", "--lr", "0.05",
              "--momentum", "0.5", "--json", "-", "--save", w])
    assert r.returncode == 0, r.stderr
    lines = r.stderr.strip().splitlines()
    assert lines[0] == "training..." and lines[1].startswith("i=0, error=")
    assert lines[-1].startswith("ntests=1000, ncorrect=")
    assert int(lines[-1].split("=")[-1]) >= 950, r.stderr
    js = json.loads(r.stdout.strip().splitlines()[-1])
    assert js["hipgraph"] is True and js["train_img_per_s"] > 0
    spec, p = mcc.load_weights(w)
    assert spec.nparams == mcc.make_model(model).nparams


@pytest.mark.gpu
def test_cnn_hip_profile_phases(idx_files):
    r = _run([os.path.join(ROOT, "build/bin/cnn_hip")] + idx_files +
             ["--model", "lenet5", "--batch", "512", "--epochs", "1", "--profile", "--json", "-"])
    assert r.returncode == 0, r.stderr
    js = json.loads(r.stdout.strip().splitlines()[-1])
    assert set(js["phase_ms"]) == {"forward_loss", "backward_allreduce_issue", "allreduce_wait", "sgd"}


@pytest.mark.gpu
def test_cnn_dist_single_rank(idx_files):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = _run([os.path.join(ROOT, "build/bin/cnn_dist")] + idx_files +
             ["--model", "lenet5", "--batch", "256", "--epochs", "1", "--lr", "0.05"], env=env)
    assert r.returncode == 0, r.stderr
    assert int(r.stderr.strip().splitlines()[-1].split("=")[-1]) >= 900


@pytest.mark.gpu
def test_python_train_gpu(idx_files):
    r = _run([sys.executable, "-m", "mpi_cuda_cnn_amd.train"] + idx_files +
             ["--model", "lenet5", "--batch", "256", "--epochs", "2", "--lr", "0.05", "--momentum", "0.5",
              "--device", "gpu"], cwd=ROOT)
    assert r.returncode == 0, r.stderr
    assert int(r.stderr.strip().splitlines()[-1].split("=")[-1]) >= 950, r.stderr


@pytest.mark.gpu
def test_python_train_gpu_two_ranks(idx_files):
    """The train CLI under torch.distributed.run with two ranks sharing the
    box's one GPU (gloo transport; RCCL needs a GPU per rank): per-rank shard
    lines, rank-0 log and test accuracy, the same GpuTrainer DP path as the
    driver's multi-GPU runs."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
              "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "-m", "mpi_cuda_cnn_amd.train"] +
             idx_files + ["--model", "lenet5", "--batch", "512", "--epochs", "2", "--lr", "0.05",
                          "--momentum", "0.5", "--device", "gpu", "--dist-backend", "gloo"], cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr
    lines = r.stderr.strip().splitlines()
    assert "0 0 2000" in lines and "1 2000 4000" in lines, r.stderr
    last = [l for l in lines if l.startswith("ntests=")]
    assert len(last) == 1 and int(last[0].split("=")[-1]) >= 950, r.stderr


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_exit_codes_gpu_programs(idx_files):
    for prog in ("cnn_hip", "cnn_dist"):
        assert _run([os.path.join(ROOT, "build/bin", prog)]).returncode == 100
        assert _run([os.path.join(ROOT, "build/bin", prog), "/nonexistent"] + idx_files[1:]).returncode == 111


@pytest.mark.gpu
def test_bench_two_ranks_gloo_rehearsal():
    """bench.py's multi-rank logic as the driver launches it (torch.distributed.run,
    one JSON line from rank 0, barriers + MAX of the rank times, n_gpus = world),
    rehearsed with two gloo ranks sharing the box's one GPU (RCCL needs a GPU per
    rank; the 8-GPU RCCL run is the driver's)."""
    import json

    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
              "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "bench.py", "--gpus", "2",
              "--steps", "3", "--warmup", "2", "--batch-per-gpu", "4096", "--dist-backend", "gloo"],
             cwd=ROOT, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["config"]["global_batch"] == 8192, d
    assert d["config"]["parallelism"] == "dp2" and d["value"] > 0, d


@pytest.mark.gpu
def test_bench_self_launch_without_launcher():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts torch.distributed.run
    itself (child process, before any GPU call) instead of measuring one rank."""
    import json

    r = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
              "--batch-per-gpu", "2048", "--dist-backend", "gloo"], cwd=ROOT,
             env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert r.returncode == 0, r.stderr
    assert "launching 2 ranks" in r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2", d


@pytest.mark.gpu
def test_bench_one_gpu_reports_fp32_config():
    """At N = 1 the headline (bf16) line also carries BASELINE config 2 (LeNet-5
    fp32 on one MI355X) as a second timed region of the same run, and both
    regions report the reference optimizer (plain SGD, lr 0.1)."""
    import json

    r = _run([sys.executable, "bench.py", "--steps", "3", "--warmup", "2", "--batch-per-gpu", "4096"], cwd=ROOT)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["dtype"] == "bf16" and d["n_gpus"] == 1 and d["value"] > 0, d
    assert "plain SGD" in d["config"]["optimizer"] and "lr=0.1" in d["config"]["optimizer"], d
    f = d["fp32"]
    assert f["steps"] == 3 and f["warmup"] == 2 and f["value"] > 0 and f["ms_per_step"] > 0, f
    assert abs(f["value"] * f["ms_per_step"] / 1000.0 - 4096) < 1.0, f
