"""Multi-rank rehearsal of the native data-parallel driver on ONE GPU.

RCCL refuses two ranks on one device, so `cnn_dist --comm host` runs 2 and 4
ranks on the test box's MI355X with host shared-memory collectives
(csrc/apps/host_comm.cpp, shm_group.cpp; CPU-tested by build/bin/test_comm).
Everything else is the multi-rank code path the 8-GPU RCCL run takes
(reference: /root/reference/cnnmpi.c:443-498): the TCP bootstrap at world > 1,
per-rank shards and sampler ranges, the bucketed fork/join on the comm stream
inside the captured hipGraph, the multi-rank log reduction, the time and
exit-code MAX, and rank-death detection (exit 111 instead of a hang, D9).

Checked: every rank's final weights are bit-identical (the sum is taken in
one fixed rank order), graph replay == eager at world 2, the run trains, and
a rank killed mid-training ends every survivor with 111 within the deadline.
"""

import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import mpi_cuda_cnn_amd as mcc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CNN_DIST = os.path.join(ROOT, "build/bin/cnn_dist")


@pytest.fixture(scope="module")
def idx_files(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("hostidx"))
    for n, s, p in ((4096, 1, "train"), (512, 2, "test")):
        i, l = mcc.synth_dataset(n, 1, 28, 28, 10, seed=s)
        mcc.idx_write(os.path.join(d, p + "-images"), i.reshape(n, 28, 28))
        mcc.idx_write(os.path.join(d, p + "-labels"), l)
    return [os.path.join(d, x) for x in ("train-images", "train-labels", "test-images", "test-labels")]


def _launch(n, idx_files, wpat, extra=(), env_extra=None, timeout=240):
    env = dict(os.environ, MCC_COMM_TIMEOUT="60", MCC_BOOTSTRAP_TIMEOUT="60")
    env.pop("MCC_AB", None)
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "mpi_cuda_cnn_amd.launch", "-n", str(n), CNN_DIST] + idx_files + [
        "--comm", "host", "--model", "lenet5", "--batch", "512", "--epochs", "1", "--lr", "0.05",
        "--momentum", "0.9", "--bucket-mb", "0.01", "--json", "-", "--save", wpat] + list(extra)
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    return r, time.time() - t0


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_cnn_dist_host_comm_replicas_bit_equal(idx_files, tmp_path, world):
    wpat = str(tmp_path / "w{rank}.bin")
    r, _ = _launch(world, idx_files, wpat)
    assert r.returncode == 0, r.stderr[-3000:]
    js = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert js["world"] == world and js["comm"] == "host" and js["hipgraph"] is True and js["buckets"] > 1
    assert js["global_batch"] == 512
    # shard lines "rank lo hi" (cnnmpi.c:457-458), one per rank, contiguous
    shards = sorted(tuple(map(int, ln.split())) for ln in r.stderr.splitlines()
                    if len(ln.split()) == 3 and all(t.isdigit() for t in ln.split()))
    assert [s[0] for s in shards] == list(range(world))
    assert shards[0][1] == 0 and all(shards[i][2] == shards[i + 1][1] for i in range(world - 1))
    reps = [mcc.load_weights(wpat.replace("{rank}", str(k)))[1] for k in range(world)]
    for k in range(1, world):
        np.testing.assert_array_equal(reps[0], reps[k], err_msg=f"rank {k} replica differs from rank 0")
    assert js["ncorrect"] >= 0.9 * js["ntests"], js


def _world1(idx_files, w, extra):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MCC_COMM_TIMEOUT="60")
    env.pop("MCC_AB", None)
    r = subprocess.run([CNN_DIST] + idx_files + [
        "--comm", "local", "--model", "lenet5", "--batch", "512", "--epochs", "1", "--lr", "0.05",
        "--momentum", "0.9", "--json", "-", "--save", w] + list(extra),
        capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return mcc.load_weights(w)[1]


@pytest.mark.gpu
@pytest.mark.parametrize("world,dtype", [(2, "fp32"), (4, "fp32"), (2, "bf16")])
def test_cnn_dist_world_n_equals_one_process(idx_files, tmp_path, world, dtype):
    """World N at global batch 512 (b = 512/N per rank, bucketed sums over the
    host collectives) ends where ONE process stepping the same global batches
    ends, to fp32 rounding of the different summation order (reference DP
    semantics to beat: cnnmpi.c:487-499 all-reduced the wrong buffer).  Both
    runs use --sampler seq, so step t's global batch is the same 512 images."""
    extra = ["--sampler", "seq", "--dtype", dtype]
    r, _ = _launch(world, idx_files, str(tmp_path / "n{rank}.bin"), extra)
    assert r.returncode == 0, r.stderr[-3000:]
    pn = mcc.load_weights(str(tmp_path / "n0.bin"))[1]
    p1 = _world1(idx_files, str(tmp_path / "one.bin"), extra)
    spec = mcc.make_model("lenet5")
    p0 = np.asarray(mcc.init_params(spec, seed=0), dtype=np.float64)
    moved = np.linalg.norm(p1 - p0)
    assert moved > 1e-2, moved
    # fp32: only the summation order differs; bf16: additionally a weight's
    # bf16 compute copy can round the other way after a step
    tol = 2e-3 if dtype == "fp32" else 3e-2
    err = np.linalg.norm(pn - p1)
    assert err < tol * moved, (err, moved)


@pytest.mark.gpu
def test_cnn_dist_host_comm_graph_equals_eager(idx_files, tmp_path):
    r1, _ = _launch(2, idx_files, str(tmp_path / "g{rank}.bin"))
    r2, _ = _launch(2, idx_files, str(tmp_path / "e{rank}.bin"), ["--no-graph"])
    assert r1.returncode == 0 and r2.returncode == 0, (r1.stderr[-2000:], r2.stderr[-2000:])
    g = mcc.load_weights(str(tmp_path / "g0.bin"))[1]
    e = mcc.load_weights(str(tmp_path / "e0.bin"))[1]
    np.testing.assert_array_equal(g, e)


@pytest.mark.gpu
def test_cnn_dist_host_comm_rank_death_exits_111(idx_files, tmp_path):
    """Ranks started directly (no launcher that would kill the survivors): rank
    1 dies abruptly before step 3; ranks 0 and 2 must detect it through the
    collective watchdog / the poisoned group and exit 111 -- not hang."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(3):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="3", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MCC_COMM_TIMEOUT="15", MCC_BOOTSTRAP_TIMEOUT="60",
                   MCC_FAULT_RANK="1", MCC_FAULT_STEP="3")
        env.pop("MCC_AB", None)
        procs.append(subprocess.Popen(
            [CNN_DIST] + idx_files + ["--comm", "host", "--model", "lenet5", "--batch", "512", "--epochs", "4",
                                      "--lr", "0.05", "--bucket-mb", "0.01"],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=ROOT))
    t0 = time.time()
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=150))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    dt = time.time() - t0
    rcs = [p.returncode for p in procs]
    assert rcs[1] != 0 and "injected fault" in outs[1][1]
    assert rcs[0] == 111 and rcs[2] == 111, (rcs, outs[0][1][-1500:], outs[2][1][-1500:])
    assert "aborting" in outs[0][1] + outs[2][1]
    assert dt < 120


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_cnn_dist_split_sgd_equals_joined(idx_files, tmp_path, world):
    """Per-bucket SGD (the default at world > 1: bucket k's parameters are
    updated as soon as ITS all-reduce landed, so the FC update overlaps the
    conv block's collective) ends bit-identical to the joined update (one
    whole-buffer SGD after every bucket's all-reduce), inside the captured
    hipGraph, with momentum and several buckets (--bucket-mb 0.01)."""
    r1, _ = _launch(world, idx_files, str(tmp_path / "s{rank}.bin"), ["--split-sgd", "on"])
    r2, _ = _launch(world, idx_files, str(tmp_path / "j{rank}.bin"), ["--split-sgd", "off"])
    assert r1.returncode == 0 and r2.returncode == 0, (r1.stderr[-2000:], r2.stderr[-2000:])
    js = json.loads([ln for ln in r1.stdout.splitlines() if ln.startswith("{")][-1])
    assert js["buckets"] > 1 and js["hipgraph"] is True
    for k in range(world):
        s = mcc.load_weights(str(tmp_path / f"s{k}.bin"))[1]
        j = mcc.load_weights(str(tmp_path / f"j{k}.bin"))[1]
        np.testing.assert_array_equal(s, j, err_msg=f"rank {k}")


@pytest.mark.gpu
def test_cnn_dist_rccl_world1_split_sgd_equals_joined(idx_files, tmp_path):
    """The same equivalence on the real RCCL communicator at world 1 (the only
    RCCL world one GPU allows): split vs joined update, bit-identical."""
    def run(w, mode):
        env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MCC_COMM_TIMEOUT="60",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29500 + os.getpid() % 1000))
        env.pop("MCC_AB", None)
        r = subprocess.run([CNN_DIST] + idx_files + [
            "--comm", "rccl", "--model", "lenet5", "--batch", "512", "--epochs", "1", "--lr", "0.05",
            "--momentum", "0.9", "--bucket-mb", "0.01", "--split-sgd", mode, "--json", "-", "--save", w],
            capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        return mcc.load_weights(w)[1]

    s = run(str(tmp_path / "s.bin"), "on")
    j = run(str(tmp_path / "j.bin"), "off")
    np.testing.assert_array_equal(s, j)
