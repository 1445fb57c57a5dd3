"""GpuNet64: the reference's precision (fp64, /root/reference/cnn.c:22-30) on
the GPU.

Oracle: the CPU executor CpuNet64 (csrc/core/cpu_net.cpp), whose --ref-compat
program log is byte-identical to the reference cnn.c (tests/test_cli.py).
  * forward probabilities, every parameter gradient and the parameters after
    SGD steps agree to fp64 rounding (summation order differs: MFMA GEMM vs
    the CPU's blocked loops), in default and --ref-compat (D1 shared-slice
    conv weights, D10 softmax max) modes, over the zoo models and a spec with
    overlapping pools, tanh convs and odd sizes;
  * `cnn_hip --dtype fp64 --ref-compat` prints the same log as `cnn
    --ref-compat` (the reference program: per-sample backprop, update every
    32 samples, rand() % N sampling) -- the reference's own GPU offload
    (CUDAcnn.cu:167-218) at its own precision, whole program.
"""

import os
import re
import subprocess

import numpy as np
import pytest

import mpi_cuda_cnn_amd as mcc
from mpi_cuda_cnn_amd import _C

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CNN = os.path.join(ROOT, "build", "bin", "cnn")
CNN_HIP = os.path.join(ROOT, "build", "bin", "cnn_hip")

ODD = "input 2 13 11; conv 5 k3 s1 p1 tanh; pool 3 2; conv 7 k2 s2 p1 relu; fc 9 tanh; fc 6 softmax"


def _spec(name):
    return _C.parse_model_spec(ODD, "odd") if name == "odd" else mcc.make_model(name)


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.mark.parametrize("compat", [False, True], ids=["fixed", "ref_compat"])
@pytest.mark.parametrize("model,B", [("ref", 37), ("lenet5", 19), ("cifar3", 6), ("odd", 23)])
def test_gpunet64_matches_cpu_executor(model, B, compat):
    spec = _spec(model)
    C, H, W = spec.input_shape()
    rng = np.random.default_rng(3)
    p0 = np.asarray(_C.init_params(spec, 5, "fast"), dtype=np.float64)
    cpu = _C.CpuNet64(spec, compat)
    gpu = _C.GpuNet64(spec, compat, 64)
    cpu.set_params(p0)
    gpu.set_params(p0)
    for step in range(3):
        x = rng.random((B, C * H * W))
        lab = rng.integers(0, spec.num_classes(), B).astype(np.int32)
        pc, pg = cpu.forward(x), gpu.forward(x)
        assert _rel(pg, pc) < 1e-12, (step, _rel(pg, pc))
        sc, sg = cpu.backward(lab, 1.0 / B), gpu.backward(lab, 1.0 / B)
        assert sg["correct"] == sc["correct"] and sg["count"] == sc["count"] == B
        assert abs(sg["loss_sum"] - sc["loss_sum"]) <= 1e-10 * abs(sc["loss_sum"])
        assert abs(sg["mse_sum"] - sc["mse_sum"]) <= 1e-10 * abs(sc["mse_sum"])
        gc, gg = cpu.get_grads(), gpu.get_grads()
        for L in spec.layers()[1:]:
            if L["nweights"] == 0:
                continue
            for off, n in ((L["w_off"], L["nweights"]), (L["b_off"], L["nbiases"])):
                a, b = gg[off:off + n], gc[off:off + n]
                assert np.max(np.abs(a - b)) <= 1e-11 * max(np.max(np.abs(b)), 1e-30), (step, L["kind"], off)
        if compat:  # D1: only the [o][0] slice of a conv weight ever receives gradient
            for L in spec.layers()[1:]:
                if L["kind"] == "conv" and L["inC"] > 1:
                    g = gg[L["w_off"]:L["w_off"] + L["nweights"]].reshape(L["C"], L["inC"], -1)
                    assert np.all(g[:, 1:] == 0)
        cpu.sgd(0.05)
        gpu.sgd(0.05)
    assert _rel(gpu.get_params(), cpu.get_params()) < 1e-11
    assert np.all(gpu.get_grads() == 0)


def test_gpunet64_is_deterministic():
    spec = mcc.make_model("lenet5")
    rng = np.random.default_rng(0)
    x = rng.random((200, 784))
    lab = rng.integers(0, 10, 200).astype(np.int32)
    p0 = np.asarray(_C.init_params(spec, 1, "fast"), dtype=np.float64)
    out = []
    for _ in range(2):
        g = _C.GpuNet64(spec, False, 256)
        g.set_params(p0)
        g.forward(x)
        g.backward(lab, 1.0 / 200)
        out.append(g.get_grads())
    assert np.array_equal(out[0], out[1])


def _write_set(d, n, seed, prefix):
    imgs, labels = mcc.synth_dataset(n, 1, 28, 28, 10, seed=seed)
    pi, pl = os.path.join(d, prefix + "-images"), os.path.join(d, prefix + "-labels")
    mcc.idx_write(pi, imgs.reshape(n, 28, 28))
    mcc.idx_write(pl, labels)
    return pi, pl


def _log_numbers(text):
    lines = text.strip().splitlines()
    errs = [float(m.group(1)) for m in (re.fullmatch(r"i=\d+, error=(\d+\.\d+)", s) for s in lines) if m]
    return lines, errs


@pytest.mark.parametrize("mode", [["--ref-compat"], ["--batch", "16", "--epochs", "2"]], ids=["ref_compat", "minibatch"])
def test_cnn_hip_fp64_log_matches_cnn(tmp_path, mode):
    for b in (CNN, CNN_HIP):
        assert os.path.exists(b), f"{b} not built (make bins)"
    d = str(tmp_path)
    data = list(_write_set(d, 1200, 1, "train") + _write_set(d, 300, 2, "test"))
    args = data + ["--max-train", "1200", "--epochs", "1"] + mode
    cpu = subprocess.run([CNN] + args, capture_output=True, text=True, timeout=300)
    assert cpu.returncode == 0, cpu.stderr
    gpu = subprocess.run([CNN_HIP] + args + ["--dtype", "fp64", "--json", "-"], capture_output=True, text=True,
                         timeout=300)
    assert gpu.returncode == 0, gpu.stderr
    lc, ec = _log_numbers(cpu.stderr)
    lg, eg = _log_numbers(gpu.stderr)
    assert len(lc) == len(lg) and len(ec) == len(eg) > 0
    # same samples, same updates: the logged errors agree to the printed digits
    # (at most a last-digit flip from fp64 rounding of the summation order)
    assert max(abs(a - b) for a, b in zip(ec, eg)) <= 1e-4
    assert lc[-1] == lg[-1], (lc[-1], lg[-1])  # ntests=..., ncorrect=...
    assert '"program": "cnn_hip"' in gpu.stdout and '"dtype": "fp64"' in gpu.stdout
