"""GPU engine numerics: one full training step (fwd + softmax-CE + bwd) of the
native HIP engine vs the plain-PyTorch fp64 oracle of the same model.

Covers every conv/pool/fc/loss kernel in both compute dtypes on the real
MI355X: conv_small fwd (scalar + 8-channel gathers, fused ReLU+maxpool),
the zero-inserted strided data-gradient path (ref model), conv dW slabs +
reduce, the FC GEMM epilogues, split-K weight gradients and the fused
softmax-cross-entropy.
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import mpi_cuda_cnn_amd as mcc
from mpi_cuda_cnn_amd.models.torch_reference import TorchReference, images_to_nchw

TOL = {"fp32": dict(logit=2e-4, grad=1e-3), "bf16": dict(logit=4e-2, grad=5e-2)}


def _oracle(spec, params, imgs, labels):
    ref = TorchReference(spec, dtype=torch.float64)
    ref.load_flat(torch.from_numpy(params.astype(np.float64)))
    x = images_to_nchw(imgs, torch.float64)
    logits = ref(x)
    loss = F.cross_entropy(logits, torch.from_numpy(labels.astype(np.int64)))
    loss.backward()
    return logits.detach().numpy(), ref.flat_grads().numpy(), loss.item()


def _relerr(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("model", ["lenet5", "ref", "cifar3"])
def test_step_matches_torch(cuda, model, dtype):
    _check_step(cuda, model, dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("model", ["lenet5", "cifar3"])
def test_step_matches_torch_side_stream(cuda, model, dtype, monkeypatch):
    """Weight gradients on the engine's side stream (MCC_SIDE_STREAM=1), data
    gradients on the caller's: same numbers as the single-stream step."""
    monkeypatch.setenv("MCC_SIDE_STREAM", "1")
    _check_step(cuda, model, dtype)


def _check_step(cuda, model, dtype):
    spec = mcc.make_model(model)
    C, H, W = spec.input_shape()
    B = 96  # not a multiple of the per-workgroup image count on purpose
    imgs, labels = mcc.synth_dataset(B, C, H, W, spec.num_classes(), seed=3)
    params = mcc.init_params(spec, seed=1).astype(np.float32)

    net = mcc.GpuNet(spec, dtype, B)
    net.set_params(params)
    d_img = torch.from_numpy(imgs).to(cuda)
    d_lab = torch.from_numpy(labels).to(cuda)
    s = torch.cuda.current_stream().cuda_stream
    net.zero_stats(s)
    net.forward(d_img.data_ptr(), 0, B, s)
    net.loss(d_lab.data_ptr(), 0, 1.0 / B, True, s)
    net.backward_all(s)
    torch.cuda.synchronize()

    logits = net.get_logits(B)
    grads = net.get_grads()
    stats = net.get_stats()
    ref_logits, ref_grads, ref_loss = _oracle(spec, params, imgs, labels)

    tol = TOL[dtype]
    assert _relerr(logits, ref_logits) < tol["logit"], "logits mismatch"
    assert abs(stats["loss_sum"] / B - ref_loss) < 5 * tol["logit"] * max(1.0, abs(ref_loss))
    # per-layer gradient check (weights and biases separately)
    for L in spec.layers():
        if L["nweights"] == 0:
            continue
        for off, n, what in ((L["w_off"], L["nweights"], "W"), (L["b_off"], L["nbiases"], "b")):
            g, r = grads[off : off + n], ref_grads[off : off + n]
            err = _relerr(g, r)
            assert err < tol["grad"], f"{model} {dtype} layer {L['kind']} {what} grad rel err {err:.3e}"


@pytest.mark.gpu
def test_sgd_and_pack_roundtrip(cuda):
    spec = mcc.make_model("lenet5")
    params = mcc.init_params(spec, seed=5).astype(np.float32)
    net = mcc.GpuNet(spec, "fp32", 32)
    net.set_params(params)
    np.testing.assert_array_equal(net.get_params(), params)
    g = torch.randn(spec.nparams, device=cuda, dtype=torch.float32)
    p = torch.from_numpy(params).to(cuda)
    mcc._C.kernels.sgd_update(p.data_ptr(), g.data_ptr(), 0, spec.nparams, 0.1, 0.0, 0.0,
                              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_allclose(p.cpu().numpy(), params - 0.1 * g.cpu().numpy(), rtol=1e-6, atol=1e-6)


def _sgd_steps(cuda, spec, dtype, B, steps=2):
    C, H, W = spec.input_shape()
    imgs, labels = mcc.synth_dataset(B, C, H, W, spec.num_classes(), seed=13)
    net = mcc.GpuNet(spec, dtype, B)
    net.set_params(mcc.init_params(spec, seed=6, mode="fast").astype(np.float32))
    d_img = torch.from_numpy(imgs).to(cuda)
    d_lab = torch.from_numpy(labels).to(cuda)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(steps):
        net.forward(d_img.data_ptr(), 0, B, s)
        net.loss(d_lab.data_ptr(), 0, 1.0 / B, True, s)
        net.backward_all(s)
        net.sgd(0.05, 0.9, 1e-3, s)
    net.forward(d_img.data_ptr(), 0, B, s)  # reads the refreshed packed copies
    torch.cuda.synchronize()
    return net.plan(), net.get_params(), net.get_logits(B)


@pytest.mark.gpu
@pytest.mark.parametrize("model,dtype", [("lenet5", "bf16"), ("lenet5", "fp32"), ("ref", "bf16"), ("cifar3", "bf16"),
                                         ("big", "bf16"), ("big", "fp32")])
def test_fused_sgd_pack_matches_table(cuda, model, dtype, monkeypatch):
    """One-pass SGD + packed-copy refresh (analytic per-stage maps, no index
    table) vs the gather-table path (MCC_NO_FUSED_PACK=1): bit-identical
    parameters after SGD with momentum + weight decay, and bit-identical
    logits from the refreshed bf16/fp32 compute copies (every packed layout:
    S1 pair, C8, flipped data-gradient copies, im2col, FC and FC^T)."""
    spec = (mcc.parse_model_spec("input 3 72 72; conv 16 k3 s1 p1 relu; pool 2; conv 24 k3 s2 p1 relu; "
                                 "fc 32 relu; fc 10 softmax", "big") if model == "big" else mcc.make_model(model))
    B = 8 if model == "big" else 64
    plan, p_fused, l_fused = _sgd_steps(cuda, spec, dtype, B)
    assert "fused sgd+pack" in plan, plan
    monkeypatch.setenv("MCC_NO_FUSED_PACK", "1")
    plan2, p_tab, l_tab = _sgd_steps(cuda, spec, dtype, B)
    assert "pack table" in plan2
    np.testing.assert_array_equal(p_fused, p_tab)
    np.testing.assert_array_equal(l_fused, l_tab)


@pytest.mark.gpu
def test_training_reduces_loss(cuda):
    spec = mcc.make_model("lenet5")
    B = 256
    imgs, labels = mcc.synth_dataset(4096, 1, 28, 28, 10, seed=11)
    net = mcc.GpuNet(spec, "bf16", B)
    net.set_params(mcc.init_params(spec, seed=2).astype(np.float32))
    d_img = torch.from_numpy(imgs).to(cuda)
    d_lab = torch.from_numpy(labels).to(cuda)
    s = torch.cuda.current_stream().cuda_stream
    gen = torch.Generator(device="cpu").manual_seed(0)
    losses = []
    for step in range(60):
        idx = torch.randint(0, 4096, (B,), generator=gen, dtype=torch.int32).to(cuda)
        net.zero_stats(s)
        net.forward(d_img.data_ptr(), idx.data_ptr(), B, s)
        net.loss(d_lab.data_ptr(), idx.data_ptr(), 1.0 / B, True, s)
        net.backward_all(s)
        net.sgd(0.05, 0.5, 0.0, s)
        losses.append(net.get_stats()["loss_sum"] / B)
    assert min(losses[-10:]) < 0.5 * losses[0], losses


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_im2col_gemm_conv_path_matches_torch(cuda, dtype):
    """Large-image path (explicit im2col + MFMA GEMM, standalone max-pool,
    materialised dZ): forced by a 96x96 input (conv output > 64x64)."""
    spec = mcc.parse_model_spec("input 3 96 96; conv 16 k3 s1 p1 relu; pool 2; conv 32 k3 s2 p1 relu; "
                                "conv 32 k3 s1 p1 relu; pool 2; fc 64 relu; fc 10 softmax", "big96")
    B = 6
    imgs, labels = mcc.synth_dataset(B, 3, 96, 96, 10, seed=4)
    params = mcc.init_params(spec, seed=2).astype(np.float32)
    net = mcc.GpuNet(spec, dtype, B)
    assert "im2col+gemm" in net.plan()
    net.set_params(params)
    d_img = torch.from_numpy(imgs).to(cuda)
    d_lab = torch.from_numpy(labels).to(cuda)
    s = torch.cuda.current_stream().cuda_stream
    net.zero_stats(s)
    net.forward(d_img.data_ptr(), 0, B, s)
    net.loss(d_lab.data_ptr(), 0, 1.0 / B, True, s)
    net.backward_all(s)
    torch.cuda.synchronize()
    ref_logits, ref_grads, _ = _oracle(spec, params, imgs, labels)
    # bf16 activations/gradients between layers + long (B*96*96) cancelling
    # reductions: looser gradient bound than the small models; fp32 stays tight.
    tol = dict(TOL[dtype])
    if dtype == "bf16":
        tol["grad"] = 0.15
    assert _relerr(net.get_logits(B), ref_logits) < tol["logit"]
    grads = net.get_grads()
    for L in spec.layers():
        if L["nweights"] == 0:
            continue
        for off, n, what in ((L["w_off"], L["nweights"], "W"), (L["b_off"], L["nbiases"], "b")):
            err = _relerr(grads[off : off + n], ref_grads[off : off + n])
            assert err < tol["grad"], f"{dtype} {L['kind']} {what} rel err {err:.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("no_igemm", [False, True])
def test_igemm_conv_path_matches_torch(cuda, no_igemm, monkeypatch):
    """Large-image path on implicit-GEMM kernels (bf16, C % 64 == 0 layers:
    forward with the bias+ReLU epilogue, the flipped-weight data gradient and
    the split-K weight gradient) vs the fp64 oracle; the same model with
    MCC_NO_IGEMM=1 runs the explicit im2col + GEMM path."""
    if no_igemm:
        monkeypatch.setenv("MCC_NO_IGEMM", "1")
    spec = mcc.parse_model_spec("input 3 80 80; conv 64 k3 s1 p1 relu; pool 2; conv 64 k3 s1 p1 relu; "
                                "conv 128 k3 s1 p1 relu; pool 2; fc 32 relu; fc 10 softmax", "big80")
    B = 5
    imgs, labels = mcc.synth_dataset(B, 3, 80, 80, 10, seed=5)
    params = mcc.init_params(spec, seed=3).astype(np.float32)
    net = mcc.GpuNet(spec, "bf16", B)
    plan = net.plan()
    assert ("igemm" in plan) != no_igemm, plan
    net.set_params(params)
    d_img = torch.from_numpy(imgs).to(cuda)
    d_lab = torch.from_numpy(labels).to(cuda)
    s = torch.cuda.current_stream().cuda_stream
    net.zero_stats(s)
    net.forward(d_img.data_ptr(), 0, B, s)
    net.loss(d_lab.data_ptr(), 0, 1.0 / B, True, s)
    net.backward_all(s)
    torch.cuda.synchronize()
    ref_logits, ref_grads, _ = _oracle(spec, params, imgs, labels)
    assert _relerr(net.get_logits(B), ref_logits) < TOL["bf16"]["logit"]
    grads = net.get_grads()
    for L in spec.layers():
        if L["nweights"] == 0:
            continue
        for off, n, what in ((L["w_off"], L["nweights"], "W"), (L["b_off"], L["nbiases"], "b")):
            err = _relerr(grads[off : off + n], ref_grads[off : off + n])
            assert err < 0.15, f"{L['kind']} {what} rel err {err:.3e}"


@pytest.mark.gpu
def test_vgg11_step_runs(cuda):
    spec = mcc.make_model("vgg11")
    B = 4
    imgs, labels = mcc.synth_dataset(B, 3, 224, 224, 1000, seed=1)
    net = mcc.GpuNet(spec, "bf16", B)
    net.set_params(mcc.init_params(spec, seed=0, mode="fast").astype(np.float32))
    d_img = torch.from_numpy(imgs).to(cuda)
    d_lab = torch.from_numpy(labels).to(cuda)
    s = torch.cuda.current_stream().cuda_stream
    net.zero_stats(s)
    net.forward(d_img.data_ptr(), 0, B, s)
    net.loss(d_lab.data_ptr(), 0, 1.0 / B, True, s)
    net.backward_all(s)
    net.sgd(0.01, 0.0, 0.0, s)
    torch.cuda.synchronize()
    st = net.get_stats()
    assert np.isfinite(st["loss_sum"]) and 0 < st["loss_sum"] / B < 20
    g = net.get_grads()
    assert np.isfinite(g).all() and np.abs(g).max() > 0


@pytest.mark.gpu
def test_bench_batch_step_matches_small_batches(cuda):
    """bench.py's per-GPU batch (65,536, plus a ragged tail): the persistent
    kernels' many-group loops and 32-bit activation offsets at full size must
    give the same logits and summed gradients as 1,024-image chunks through
    the small-batch path (which test_step_matches_torch pins to PyTorch).
    A PyTorch reference at this size would spend minutes in MIOpen's first
    backward-convolution search on a fresh box."""
    spec = mcc.make_model("lenet5")
    B, b = 65536 + 37, 1024
    imgs, labels = mcc.synth_dataset(B, 1, 28, 28, 10, seed=21)
    params = mcc.init_params(spec, seed=4).astype(np.float32)
    d_img = torch.from_numpy(imgs).to(cuda)
    d_lab = torch.from_numpy(labels).to(cuda)
    s = torch.cuda.current_stream().cuda_stream

    big = mcc.GpuNet(spec, "bf16", B)
    big.set_params(params)
    big.zero_stats(s)
    big.forward(d_img.data_ptr(), 0, B, s)
    big.loss(d_lab.data_ptr(), 0, 1.0 / B, True, s)
    big.backward_all(s)
    torch.cuda.synchronize()
    logits, grads = big.get_logits(B), big.get_grads()
    del big

    small = mcc.GpuNet(spec, "bf16", b)
    small.set_params(params)
    ref_logits = np.empty_like(logits)
    ref_grads = np.zeros_like(grads, dtype=np.float64)
    for i in range(0, B, b):
        nb = min(b, B - i)
        idx = torch.arange(i, i + nb, device=cuda, dtype=torch.int32)
        small.forward(d_img.data_ptr(), idx.data_ptr(), nb, s)
        small.loss(d_lab.data_ptr(), idx.data_ptr(), 1.0 / B, True, s)
        small.backward_all(s)
        torch.cuda.synchronize()
        ref_logits[i : i + nb] = small.get_logits(nb)
        ref_grads += small.get_grads()
    assert _relerr(logits, ref_logits) < 1e-2
    for L in spec.layers():
        if L["nweights"] == 0:
            continue
        for off, n, what in ((L["w_off"], L["nweights"], "W"), (L["b_off"], L["nbiases"], "b")):
            err = _relerr(grads[off : off + n], ref_grads[off : off + n])
            assert err < 2e-2, f"layer {L['kind']} {what} grad rel err {err:.3e}"


@pytest.mark.gpu
def test_max_batch_guard(cuda):
    spec = mcc.make_model("lenet5")
    with pytest.raises(Exception, match="32-bit activation indexing"):
        mcc.GpuNet(spec, "bf16", 1 << 20)


def _lenet_grads(cuda, B, seed=7):
    spec = mcc.make_model("lenet5")
    imgs, labels = mcc.synth_dataset(B, 1, 28, 28, 10, seed=seed)
    params = mcc.init_params(spec, seed=seed).astype(np.float32)
    net = mcc.GpuNet(spec, "bf16", B)
    net.set_params(params)
    d_img = torch.from_numpy(imgs).to(cuda)
    d_lab = torch.from_numpy(labels).to(cuda)
    s = torch.cuda.current_stream().cuda_stream
    net.forward(d_img.data_ptr(), 0, B, s)
    net.loss(d_lab.data_ptr(), 0, 1.0 / B, True, s)
    net.backward_all(s)
    torch.cuda.synchronize()
    return spec, net.plan(), net.get_grads()


@pytest.mark.gpu
@pytest.mark.parametrize("B", [96, 4099])
def test_rows_dw_matches_pipe_dw(cuda, B, monkeypatch):
    """conv1 weight gradient on the row-chunked kernel (conv_rows.hip) vs the
    pixel-major conv_dw_pipe kernel (MCC_NO_ROWS=1).  Same bf16 dZ; the
    pixels differ only in rounding (conv_rows stages the exact integers
    0..255 and applies 1/255 in fp32 at the end, conv_dw_pipe rounds x/255 to
    bf16: <= 2^-9 relative per pixel), so every output channel agrees to a
    few 1e-3 and the bias (no pixel operand) to ~1e-5."""
    spec, plan, g_rows = _lenet_grads(cuda, B)
    assert "dw:rows" in plan, plan
    monkeypatch.setenv("MCC_NO_ROWS", "1")
    _, plan2, g_pipe = _lenet_grads(cuda, B)
    assert "dw:rows" not in plan2
    L = spec.layers()[1]
    w0, nb = L["w_off"], L["nbiases"]
    W = g_rows[w0 : w0 + L["nweights"]].reshape(nb, -1)
    Wp = g_pipe[w0 : w0 + L["nweights"]].reshape(nb, -1)
    for c in range(nb):
        assert _relerr(W[c], Wp[c]) < 4e-3, (c, W[c], Wp[c])
    bo = L["b_off"]
    np.testing.assert_allclose(g_rows[bo : bo + nb], g_pipe[bo : bo + nb], rtol=1e-4, atol=1e-7)
    # the other layers are untouched by the switch
    rest = np.ones_like(g_rows, dtype=bool)
    rest[w0 : w0 + L["nweights"]] = False
    rest[bo : bo + nb] = False
    np.testing.assert_array_equal(g_rows[rest], g_pipe[rest])
