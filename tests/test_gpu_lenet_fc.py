"""The fused LeNet-5 classifier chain (csrc/kernels/lenet_fc.hip: FC 400 ->
120 -> 84 -> 10, softmax-CE, the three layers' backward in one kernel) against
the per-layer FC kernels + fused head of the same engine (MCC_AB=no_fcchain),
which test_gpu_engine.py pins to the PyTorch fp64 oracle -- and against the
oracle directly, per output channel.

Both paths round at the same points (bf16 activations, fp32 logits, bf16
dlogits / dH), so logits agree to fp32 accumulation order and gradients to a
rare bf16 rounding flip; an indexing error (a wrong row permutation, a
misplaced tile, a dropped padding mask) is O(1).
Reference semantics: /root/reference/cnn.c:113-173 (FC forward / backward),
cnn.c:125-143 and 284-286 (softmax, output error), cnn.c:275-282 (metric).
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import mpi_cuda_cnn_amd as mcc
from mpi_cuda_cnn_amd.models.torch_reference import TorchReference, images_to_nchw


def _relerr(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _step(cuda, B, ab, seed=3, idx=None):
    import os

    os.environ["MCC_AB"] = ab
    try:
        spec = mcc.make_model("lenet5")
        imgs, labels = mcc.synth_dataset(max(B, 64), 1, 28, 28, 10, seed=seed)
        params = mcc.init_params(spec, seed=1).astype(np.float32)
        net = mcc.GpuNet(spec, "bf16", B)
        assert ("lenet_fc" in net.plan()) == (ab == ""), net.plan()
        net.set_params(params)
        d_img = torch.from_numpy(imgs).to(cuda)
        d_lab = torch.from_numpy(labels).to(cuda)
        d_idx = None if idx is None else torch.from_numpy(idx).to(cuda)
        ip = 0 if d_idx is None else d_idx.data_ptr()
        pred = torch.full((B,), -1, dtype=torch.int32, device=cuda)
        s = torch.cuda.current_stream().cuda_stream
        net.zero_stats(s)
        net.forward(d_img.data_ptr(), ip, B, s)
        net.loss(d_lab.data_ptr(), ip, 1.0 / B, True, s, pred.data_ptr())
        net.backward_all(s)
        torch.cuda.synchronize()
        out = dict(logits=net.get_logits(B), grads=net.get_grads(), stats=net.get_stats(), pred=pred.cpu().numpy())
        del net
        return spec, params, imgs, labels, out
    finally:
        os.environ.pop("MCC_AB", None)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 31, 96, 1000, 4096 + 13])
def test_fused_fc_chain_matches_per_layer_path(cuda, B):
    rng = np.random.default_rng(B)
    idx = rng.integers(0, max(B, 64), size=B).astype(np.int32)  # label gather through the sampler's indices
    spec, _, _, labels, f = _step(cuda, B, "", idx=idx)
    _, _, _, _, u = _step(cuda, B, "no_fcchain", idx=idx)
    assert _relerr(f["logits"][:, :10], u["logits"][:, :10]) < 1e-5
    np.testing.assert_array_equal(f["pred"], u["pred"])
    assert f["stats"]["correct"] == u["stats"]["correct"]
    assert abs(f["stats"]["loss_sum"] - u["stats"]["loss_sum"]) < 1e-4 * max(1.0, abs(u["stats"]["loss_sum"]))
    assert abs(f["stats"]["mse_sum"] - u["stats"]["mse_sum"]) < 1e-4 * max(1.0, abs(u["stats"]["mse_sum"]))
    for L in spec.layers():
        if L["nweights"] == 0:
            continue
        for off, n, what in ((L["w_off"], L["nweights"], "W"), (L["b_off"], L["nbiases"], "b")):
            err = _relerr(f["grads"][off : off + n], u["grads"][off : off + n])
            # conv layers see the FC input gradient (bf16 either way)
            assert err < 1e-2, f"B={B} layer {L['kind']} {what}: fused vs per-layer rel err {err:.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("B", [37, 300])
def test_fused_fc_chain_per_channel_vs_oracle(cuda, B):
    """Per output feature of every FC layer against the fp64 oracle fed the
    engine's bf16 rounding points (as test_gpu_engine's per-channel tests)."""
    spec, params, imgs, labels, f = _step(cuda, B, "")
    ref = TorchReference(spec, torch.float64, mimic_bf16=True)
    ref.load_flat(torch.from_numpy(params.astype(np.float64)))
    rl = ref(images_to_nchw(imgs[:B], torch.float64))
    F.cross_entropy(rl, torch.from_numpy(labels[:B].astype(np.int64))).backward()
    rg = ref.flat_grads().numpy()
    assert _relerr(f["logits"][:, :10], rl.detach().numpy()) < 1e-2
    for L in spec.layers():
        if L["kind"] != "fc":
            continue
        C = L["C"]
        g = f["grads"][L["w_off"] : L["w_off"] + L["nweights"]].reshape(C, -1).astype(np.float64)
        r = rg[L["w_off"] : L["w_off"] + L["nweights"]].reshape(C, -1)
        floor = 1e-2 * np.linalg.norm(r) / np.sqrt(C)
        e = np.linalg.norm(g - r, axis=1) / np.maximum(np.linalg.norm(r, axis=1), max(floor, 1e-30))
        assert e.max() < 6e-2, (C, float(e.max()), int(e.argmax()))
        gb = f["grads"][L["b_off"] : L["b_off"] + C]
        rb = rg[L["b_off"] : L["b_off"] + C]
        assert _relerr(gb, rb) < 6e-2, (C, _relerr(gb, rb))


@pytest.mark.gpu
def test_fused_fc_chain_eval_and_logits_without_backward(cuda):
    """forward() defers the FC chain to loss(); a forward-only loss
    (evaluation) and get_logits() after forward() alone still see the
    per-layer FC forward, with the same numbers."""
    spec = mcc.make_model("lenet5")
    B = 200
    imgs, labels = mcc.synth_dataset(B, 1, 28, 28, 10, seed=8)
    params = mcc.init_params(spec, seed=2).astype(np.float32)
    d_img = torch.from_numpy(imgs).to(cuda)
    d_lab = torch.from_numpy(labels).to(cuda)
    s = torch.cuda.current_stream().cuda_stream
    net = mcc.GpuNet(spec, "bf16", B)
    net.set_params(params)
    net.forward(d_img.data_ptr(), 0, B, s)
    l_fwd = net.get_logits(B)  # flushes the deferred FC forward
    net.zero_stats(s)
    net.forward(d_img.data_ptr(), 0, B, s)
    net.loss(d_lab.data_ptr(), 0, 1.0, False, s)
    torch.cuda.synchronize()
    st_eval = net.get_stats()
    l_eval = net.get_logits(B)
    net.zero_stats(s)
    net.forward(d_img.data_ptr(), 0, B, s)
    net.loss(d_lab.data_ptr(), 0, 1.0 / B, True, s)
    torch.cuda.synchronize()
    st_train = net.get_stats()
    l_train = net.get_logits(B)
    np.testing.assert_array_equal(l_fwd, l_eval)
    assert _relerr(l_train[:, :10], l_eval[:, :10]) < 1e-5
    assert st_eval["correct"] == st_train["correct"]
    assert abs(st_eval["loss_sum"] - st_train["loss_sum"]) < 1e-4 * max(1.0, st_eval["loss_sum"])
    # forward() on a non-blocking side stream: get_logits() / stage_output()
    # order the deferred FC forward after it (device-wide synchronisation)
    side = torch.cuda.Stream()
    for k in range(3):
        net.forward(d_img.data_ptr(), 0, B, side.cuda_stream)
        l_side = net.get_logits(B)
        np.testing.assert_array_equal(l_side, l_fwd)
    net.forward(d_img.data_ptr(), 0, B, side.cuda_stream)
    y3, _ = net.stage_output(3, B)
    assert np.isfinite(y3).all() and np.abs(y3).max() > 0
