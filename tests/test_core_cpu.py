"""CPU-only tests of the native core: model zoo / shape inference, the fp64
CPU executor vs PyTorch, the reference-compat (defect D1) conv indexing, IDX
and weight-file I/O, synthetic data, gradient bucket planning."""

import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import mpi_cuda_cnn_amd as mcc
from mpi_cuda_cnn_amd.models.torch_reference import TorchReference, images_to_nchw


# ----------------------------------------------------------------- models


def test_model_zoo_param_counts():
    # ref: cnn.c:416-428 -> 360,810 params
    assert mcc.make_model("ref").nparams == 360810
    assert mcc.make_model("lenet5").nparams == 61706
    assert mcc.make_model("vgg11").nparams == 132863336
    assert set(mcc.model_names()) >= {"ref", "lenet5", "cifar3", "vgg11"}


def test_ref_shapes_match_reference():
    L = mcc.make_model("ref").layers()
    # conv1 16x14x14, conv2 32x7x7 (cnn.c:419-422), fc 200/200/10
    assert [(l["kind"], l["C"], l["H"], l["W"]) for l in L] == [
        ("input", 1, 28, 28),
        ("conv", 16, 14, 14),
        ("conv", 32, 7, 7),
        ("fc", 200, 1, 1),
        ("fc", 200, 1, 1),
        ("fc", 10, 1, 1),
    ]
    assert L[3]["nweights"] == 200 * 1568


def test_spec_parser_roundtrip():
    s = mcc.parse_model_spec("input 1 28 28; conv 6 k5 s1 p2 relu; pool 2; conv 16 k5 relu; pool 2; "
                             "fc 120 relu; fc 84 relu; fc 10 softmax")
    assert s.nparams == mcc.make_model("lenet5").nparams
    with pytest.raises(RuntimeError):
        mcc.parse_model_spec("input 1 28 28; fc 10 relu")  # last layer must be softmax
    with pytest.raises(RuntimeError):
        mcc.make_model("nope")


def test_plan_buckets_cover_reverse_order():
    for name in mcc.model_names():
        spec = mcc.make_model(name)
        for mb in (0.001, 1, 4, 64):
            b = mcc._C.plan_buckets(spec, int(mb * (1 << 20)))
            assert sum(x[3] for x in b) == spec.nparams
            # contiguous, descending ranges, first bucket ends at nparams
            end = spec.nparams
            hi_prev = None
            for hi, lo, off, cnt in b:
                assert off + cnt == end and hi >= lo
                if hi_prev is not None:
                    assert hi == hi_prev - 1
                hi_prev = lo
                end = off
            assert end == 0
            # the last stage to finish in backward (stage 0) is reduced alone
            assert b[-1][0] == 0 and b[-1][1] == 0
            if mb >= 4 and name in ("ref", "lenet5", "cifar3"):
                assert len(b) == 2  # small models: one big collective + the stage-0 tail


# ------------------------------------------------------------ CPU oracle


@pytest.mark.parametrize("name", ["ref", "lenet5", "cifar3"])
def test_cpu_net_matches_torch_fp64(name):
    spec = mcc.make_model(name)
    C, H, W = spec.input_shape()
    B = 6
    imgs, labels = mcc.synth_dataset(B, C, H, W, 10, seed=7)
    p = mcc.init_params(spec, seed=3)
    net = mcc.CpuNet64(spec)
    net.set_params(p)
    x = images_to_nchw(imgs, torch.float64)
    probs = net.forward(x.numpy().reshape(B, -1))
    st = net.backward(labels.astype(np.int32), 1.0 / B)
    ref = TorchReference(spec, torch.float64)
    ref.load_flat(torch.from_numpy(p))
    logits = ref(x)
    loss = F.cross_entropy(logits, torch.from_numpy(labels.astype(np.int64)))
    loss.backward()
    np.testing.assert_allclose(probs, torch.softmax(logits, 1).detach().numpy(), atol=1e-13)
    np.testing.assert_allclose(net.get_grads(), ref.flat_grads().numpy(), atol=1e-12)
    assert abs(st["loss_sum"] / B - loss.item()) < 1e-12
    assert st["count"] == B


def test_ref_compat_is_shared_slice_conv():
    """Defect D1 (cnn.c:181,193): every input channel uses filter slice [o][0].
    ref_compat reproduces it; equivalently a standard conv whose weight is
    w[:, :1].expand(...) (measured <= 2e-15)."""
    spec = mcc.make_model("ref")
    B = 3
    imgs, labels = mcc.synth_dataset(B, 1, 28, 28, 10, seed=2)
    p = mcc.init_params(spec, seed=0)
    net = mcc.CpuNet64(spec, ref_compat=True)
    net.set_params(p)
    x = images_to_nchw(imgs, torch.float64)
    probs = net.forward(x.numpy().reshape(B, -1))
    L = spec.layers()
    q = p.copy()
    w2 = q[L[2]["w_off"] : L[2]["w_off"] + L[2]["nweights"]].reshape(32, 16, 3, 3)
    # reference index q = o*Cin*9 + kh*3 + kw  ->  flat slice [o][0][kh][kw]
    w2[:] = w2[:, :1].copy()
    ref = TorchReference(spec, torch.float64)
    ref.load_flat(torch.from_numpy(q))
    logits = ref(x)
    # the softmax max starts at -1 in compat mode (D10): identical in exact math
    np.testing.assert_allclose(probs, torch.softmax(logits, 1).detach().numpy(), atol=1e-12)


def test_cpu_sgd_update():
    spec = mcc.make_model("lenet5")
    net = mcc.CpuNet64(spec)
    p = mcc.init_params(spec, seed=1)
    g = np.random.default_rng(0).standard_normal(spec.nparams)
    net.set_params(p)
    net.set_grads(g)
    net.sgd(0.25)
    np.testing.assert_allclose(net.get_params(), p - 0.25 * g)
    assert not net.get_grads().any()


def test_glibc_init_matches_reference_rng():
    """init 'glibc' = srand(seed); std * (4 rand()/RAND_MAX - 2) * 1.724 in layer
    order (cnn.c:46-49,320-341).  Check statistics and determinism."""
    spec = mcc.make_model("ref")
    a = mcc.init_params(spec, seed=0)
    b = mcc.init_params(spec, seed=0)
    np.testing.assert_array_equal(a, b)
    L = spec.layers()
    w = a[L[3]["w_off"] : L[3]["w_off"] + L[3]["nweights"]]
    assert abs(w.std() - 0.1 * 0.995) < 0.002 and abs(w.mean()) < 0.002
    assert not a[L[3]["b_off"] : L[3]["b_off"] + 200].any()  # zero biases (calloc)
    fast = mcc.init_params(spec, seed=0, mode="fast")
    assert abs(fast[L[3]["w_off"] : L[3]["w_off"] + L[3]["nweights"]].std() - 0.0995) < 0.002


# -------------------------------------------------------------------- I/O


def test_idx_roundtrip_and_validation(tmp_path):
    imgs, labels = mcc.synth_dataset(17, 1, 28, 28, 10, seed=5)
    pi, pl = str(tmp_path / "img"), str(tmp_path / "lbl")
    mcc.idx_write(pi, imgs.reshape(17, 28, 28))
    mcc.idx_write(pl, labels)
    a = mcc.idx_read(pi)
    b = mcc.idx_read(pl)
    assert a.shape == (17, 28, 28) and b.shape == (17,)
    np.testing.assert_array_equal(a.reshape(-1), imgs.reshape(-1))
    np.testing.assert_array_equal(b, labels)
    raw = open(pi, "rb").read()
    assert raw[:4] == b"\x00\x00\x08\x03" and raw[4:8] == (17).to_bytes(4, "big")
    bad = tmp_path / "bad"
    bad.write_bytes(b"\x00\x01\x08\x01" + (3).to_bytes(4, "big") + b"abc")
    with pytest.raises(RuntimeError):
        mcc.idx_read(str(bad))
    short = tmp_path / "short"
    short.write_bytes(raw[:100])
    with pytest.raises(RuntimeError):  # payload is always read (defect D3 fixed)
        mcc.idx_read(str(short))
    with pytest.raises(RuntimeError):
        mcc.idx_read(str(tmp_path / "missing"))


def test_synthetic_data_is_class_striped():
    imgs, labels = mcc.synth_dataset(200, 1, 28, 28, 10, seed=1)
    for i in range(20):
        l = labels[i]
        rows = imgs[i, :, :, 0]
        assert (rows[2 + 2 * l : 4 + 2 * l] == 220).all()
        assert rows.max() == 220 and (rows[rows != 220] < 40).all()
    assert len(set(labels.tolist())) == 10


def test_weight_file_roundtrip(tmp_path):
    for name in ("ref", "lenet5"):
        spec = mcc.make_model(name)
        p = mcc.init_params(spec, seed=9)
        path = str(tmp_path / f"{name}.mcnnw")
        mcc.save_weights(path, spec, p)
        spec2, p2 = mcc.load_weights(path)
        assert spec2.nparams == spec.nparams
        assert [l["kind"] for l in spec2.layers()] == [l["kind"] for l in spec.layers()]
        np.testing.assert_array_equal(p, p2)
        raw = open(path, "rb").read()
        assert raw[:5] == b"MCNNW"
    with pytest.raises(RuntimeError):
        mcc.load_weights(str(tmp_path / "nope"))


def test_weight_file_validation(tmp_path):
    """The loader re-derives every layer's shape and parameter counts and
    rejects disagreeing stored counts, a bad activation, a big-endian file
    and trailing bytes; version-1 files (no byte-order mark) still load."""
    import struct

    spec = mcc.make_model("lenet5")
    p = mcc.init_params(spec, seed=2)
    path = tmp_path / "w.mcnnw"
    mcc.save_weights(str(path), spec, p)
    raw = bytearray(path.read_bytes())
    assert struct.unpack_from("<II", raw, 8) == (2, 0x01020304)
    nl = struct.unpack_from("<I", raw, 16)[0]
    hdr, rec = 28, 48  # magic+version+bom+nlayers+nparams; per layer 8 x i32 + 2 x i64

    def bad(mut):
        b = bytearray(raw)
        mut(b)
        q = tmp_path / "bad.mcnnw"
        q.write_bytes(bytes(b))
        with pytest.raises(RuntimeError):
            mcc.load_weights(str(q))

    bad(lambda b: struct.pack_into("<q", b, hdr + rec * 1 + 40, 7))      # conv1 stored nweights
    bad(lambda b: struct.pack_into("<q", b, hdr + rec * 1 + 32, 5))      # conv1 stored nbiases
    bad(lambda b: struct.pack_into("<i", b, hdr + rec * 1 + 28, 9))      # activation out of range
    bad(lambda b: struct.pack_into("<i", b, hdr + rec * 2 + 8, 13))      # pool stored width
    bad(lambda b: struct.pack_into(">II", b, 8, 2, 0x01020304))          # big-endian header
    bad(lambda b: struct.pack_into("<I", b, 12, 0x04030201))             # byte-order mark
    bad(lambda b: b.extend(b"\0" * 8))                                    # trailing bytes
    bad(lambda b: b.__delitem__(slice(len(b) - 8, len(b))))               # truncated payload
    # version 1 (round-1 files): no byte-order mark
    v1 = bytearray(raw[:8]) + struct.pack("<I", 1) + raw[16:]
    q = tmp_path / "v1.mcnnw"
    q.write_bytes(bytes(v1))
    spec1, p1 = mcc.load_weights(str(q))
    assert nl == len(spec.layers()) and spec1.nparams == spec.nparams
    np.testing.assert_array_equal(p1, p)


def test_watchdog_policy():
    """Collective watchdog of cnn_dist (csrc/apps/watchdog.h): completion,
    async-error and deadline branches, as a native CPU test binary."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    binp = os.path.join(root, "build", "bin", "test_watchdog")
    if not os.path.exists(binp):
        subprocess.run(["make", "-C", root, "build/bin/test_watchdog"], check=True, capture_output=True)
    r = subprocess.run([binp], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "watchdog ok" in r.stdout, r.stderr


def test_native_bootstrap_and_host_collectives():
    """TCP rendezvous of cnn_dist (csrc/apps/bootstrap.cpp) serving 4 forked
    processes, both of its timeout branches, and the shared-memory
    collectives of `cnn_dist --comm host` (csrc/apps/shm_group.cpp): bit-equal
    sums on every rank in fixed rank order, max with NaN, broadcast, a dead
    peer / a poisoned group / a rank that never attaches -- as a native CPU
    test binary (csrc/tests/test_comm.cpp)."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    binp = os.path.join(root, "build", "bin", "test_comm")
    subprocess.run(["make", "-C", root, "build/bin/test_comm"], check=True, capture_output=True)
    r = subprocess.run([binp], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "comm ok" in r.stdout, r.stdout + r.stderr
