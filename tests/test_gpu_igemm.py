"""Implicit-GEMM convolution kernels (igemm.hip) vs plain PyTorch fp32 conv2d.

Forward (bias + ReLU epilogue), data gradient (stride-1 conv of dY with the
flipped weights) and weight/bias gradient (split-K slabs + deterministic
reduce), on bf16 NHWC tensors.  Shapes cover VGG-style layers, image sizes
that leave partial 128-pixel tiles, channel counts below one 128 tile, strided
and padding-free convs and an asymmetric kernel (a symmetric one hides a
flipped-tap bug)."""

import pytest
import torch
import torch.nn.functional as F

from mpi_cuda_cnn_amd import ops

CASES = [
    # B, H, W, C, O, KS, stride, pad
    (2, 56, 56, 64, 128, 3, 1, 1),
    (3, 28, 28, 128, 256, 3, 1, 1),
    (1, 14, 14, 512, 512, 3, 1, 1),
    (4, 13, 11, 64, 64, 3, 1, 1),
    (2, 17, 19, 128, 72, 3, 2, 1),
    (2, 9, 9, 64, 136, 5, 1, 0),
    (3, 16, 16, 32, 64, 3, 1, 1),    # C = 32: a K-step spans two taps, K = 288 (tail K-step half zero)
    (2, 14, 14, 32, 48, 5, 1, 2),    # C = 32, 5x5: K = 800
    (2, 12, 10, 96, 40, 3, 1, 1),    # C = 96: channel wrap at c0 = 64
    (4, 8, 8, 96, 200, 1, 1, 0),     # 129..256 output channels: the 256-channel dW tile (ref FC1 shape class)
    (3, 7, 7, 32, 160, 3, 1, 1),     # ... with taps
]


def _rand(shape, g, dev, scale=1.0):
    return (torch.randn(*shape, generator=g, device=dev) * scale).to(torch.bfloat16)


def _relerr(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W,C,O,KS,stride,pad", CASES)
def test_igemm_forward(cuda, B, H, W, C, O, KS, stride, pad):
    g = torch.Generator(device=cuda).manual_seed(B * 1000 + C + O)
    x = _rand((B, H, W, C), g, cuda)
    w = _rand((O, C, KS, KS), g, cuda, (2.0 / (C * KS * KS)) ** 0.5)
    w[:, :, 0, KS - 1] *= 3.0  # asymmetric taps
    b = torch.randn(O, generator=g, device=cuda) * 0.1
    y = ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu")
    ref = F.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), b, stride=stride, padding=pad)).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert _relerr(y, ref) < 1e-2
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W,C,O,KS,stride,pad", [c for c in CASES if c[6] == 1 and c[4] % 32 == 0])
def test_igemm_dgrad(cuda, B, H, W, C, O, KS, stride, pad):
    g = torch.Generator(device=cuda).manual_seed(7 + B + C)
    OH, OW = (H + 2 * pad - KS) + 1, (W + 2 * pad - KS) + 1
    dy = _rand((B, OH, OW, O), g, cuda)
    w = _rand((O, C, KS, KS), g, cuda, (1.0 / (O * KS * KS)) ** 0.5)
    w[:, :, KS - 1, 0] *= 2.0
    dx = ops.conv2d_dgrad_nhwc(dy, w, pad=pad)
    ref = torch.nn.grad.conv2d_input((B, C, H, W), w.float(), dy.float().permute(0, 3, 1, 2), padding=pad)
    ref = ref.permute(0, 2, 3, 1)
    assert dx.shape == ref.shape
    assert _relerr(dx, ref) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W,C,O,KS,stride,pad", CASES)
def test_igemm_wgrad(cuda, B, H, W, C, O, KS, stride, pad):
    g = torch.Generator(device=cuda).manual_seed(99 + H + O)
    OH, OW = (H + 2 * pad - KS) // stride + 1, (W + 2 * pad - KS) // stride + 1
    x = _rand((B, H, W, C), g, cuda)
    dy = _rand((B, OH, OW, O), g, cuda, 0.1)
    gw, gb = ops.conv2d_wgrad_nhwc(dy, x, KS, stride=stride, pad=pad)
    xr = x.float().permute(0, 3, 1, 2)
    dyr = dy.float().permute(0, 3, 1, 2)
    ref_w = torch.nn.grad.conv2d_weight(xr, (O, C, KS, KS), dyr, stride=stride, padding=pad)
    ref_b = dyr.sum((0, 2, 3))
    assert _relerr(gw, ref_w) < 1e-3
    assert _relerr(gb, ref_b) < 1e-3
    # deterministic: a second run is bitwise identical; the split count does not change the math
    gw2, gb2 = ops.conv2d_wgrad_nhwc(dy, x, KS, stride=stride, pad=pad)
    assert torch.equal(gw, gw2) and torch.equal(gb, gb2)
    gw1, _ = ops.conv2d_wgrad_nhwc(dy, x, KS, stride=stride, pad=pad, splitk=1)
    assert _relerr(gw1, ref_w) < 1e-3


@pytest.mark.gpu
def test_igemm_rejects_unsupported(cuda):
    x = torch.zeros(1, 8, 8, 48, dtype=torch.bfloat16, device=cuda)
    w = torch.zeros(64, 48, 3, 3, device=cuda)
    with pytest.raises(RuntimeError):
        ops.conv2d_nhwc(x, w)
    with pytest.raises(RuntimeError):
        ops.conv2d_nhwc(x.cpu(), w.cpu())


# 256-pixel phase-pipelined kernel (igemm_big_kernel): every tile variant vs
# fp32 F.conv2d and vs the 128x128 kernel; pixel counts that leave partial
# 256-row tiles (and a whole grid smaller than one tile), fused pool.
BIG_CASES = [
    # B, H, W, C, O, KS, stride, pad
    (2, 30, 26, 128, 256, 3, 1, 1),   # M = 1560: partial last tile
    (1, 14, 14, 512, 512, 3, 1, 1),   # M = 196 < 256
    (2, 28, 28, 64, 128, 3, 1, 1),    # BC = 128 only
    (3, 20, 12, 256, 384, 3, 1, 1),   # N % 256 != 0 -> 128-channel tiles
    (2, 19, 17, 128, 256, 3, 2, 1),   # strided
]


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W,C,O,KS,stride,pad", BIG_CASES)
@pytest.mark.parametrize("tile", [128, 256])
def test_igemm_big_forward(cuda, B, H, W, C, O, KS, stride, pad, tile):
    g = torch.Generator(device=cuda).manual_seed(B * 31 + C + O + tile)
    x = _rand((B, H, W, C), g, cuda)
    w = _rand((O, C, KS, KS), g, cuda, (2.0 / (C * KS * KS)) ** 0.5)
    w[:, :, 0, KS - 1] *= 3.0
    b = torch.randn(O, generator=g, device=cuda) * 0.1
    y = ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu", tile=tile)
    ref = F.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), b, stride=stride, padding=pad)).permute(0, 2, 3, 1)
    assert _relerr(y, ref) < 1e-2
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)
    # same fp32 accumulation order per fragment as the 128x128 kernel: equal bits
    y0 = ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu", tile=0)
    assert torch.equal(y, y0)


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [0, 128, 256])
def test_igemm_big_pool(cuda, tile):
    B, H, W, C, O = 3, 22, 18, 128, 256
    g = torch.Generator(device=cuda).manual_seed(5 + tile)
    x = _rand((B, H, W, C), g, cuda)
    w = _rand((O, C, 3, 3), g, cuda, (2.0 / (C * 9)) ** 0.5)
    b = torch.randn(O, generator=g, device=cuda) * 0.1
    y, arg = ops.conv2d_nhwc(x, w, b, stride=1, pad=1, act="relu", pool=True, tile=tile)
    z = ops.conv2d_nhwc(x, w, b, stride=1, pad=1, act="relu", tile=tile)  # pre-pool, same kernel family
    zr = z.float().reshape(B, H // 2, 2, W // 2, 2, O).permute(0, 1, 3, 5, 2, 4).reshape(B, H // 2, W // 2, O, 4)
    assert torch.equal(y.float(), zr.max(-1).values)
    live = y.float() > 0
    a = arg.long()
    assert bool((a[live] < 4).all())
    # the argmax names a position holding the max (ties after bf16 rounding may pick either)
    picked = zr.gather(-1, a.clamp(max=3).unsqueeze(-1)).squeeze(-1)
    assert torch.equal(picked[live], y.float()[live])
    assert bool((a[~live] == 4).all())  # ReLU-inactive windows: byte 4
    if tile:
        y0, arg0 = ops.conv2d_nhwc(x, w, b, stride=1, pad=1, act="relu", pool=True, tile=0)
        assert torch.equal(y, y0) and torch.equal(arg, arg0)


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W,C,O", [(2, 28, 28, 128, 128), (1, 14, 14, 512, 512), (2, 15, 13, 256, 256)])
def test_igemm_big_dgrad(cuda, B, H, W, C, O):
    g = torch.Generator(device=cuda).manual_seed(11 + B + C)
    dy = _rand((B, H, W, O), g, cuda)
    w = _rand((O, C, 3, 3), g, cuda, (1.0 / (O * 9)) ** 0.5)
    w[:, :, 2, 0] *= 2.0
    ref = torch.nn.grad.conv2d_input((B, C, H, W), w.float(), dy.float().permute(0, 3, 1, 2), padding=1)
    ref = ref.permute(0, 2, 3, 1)
    dx0 = ops.conv2d_dgrad_nhwc(dy, w, pad=1, tile=0)
    for tile in (128, 256):
        dx = ops.conv2d_dgrad_nhwc(dy, w, pad=1, tile=tile)
        assert _relerr(dx, ref) < 1e-2
        assert torch.equal(dx, dx0)


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W,C,O,KS,stride,pad", [
    (2, 30, 26, 128, 256, 3, 1, 1),   # kf = 1152: partial last 256-column tile
    (1, 14, 14, 512, 512, 3, 1, 1),   # M = 196: partial K-step
    (2, 28, 28, 64, 128, 3, 1, 1),    # 128-channel tiles (128-byte transposed rows)
    (3, 20, 12, 256, 384, 3, 1, 1),   # O % 256 != 0
    (2, 19, 17, 128, 256, 3, 2, 1),   # strided
    (4, 8, 8, 512, 256, 1, 1, 0),     # 1x1, one split: direct write (FC-style)
])
@pytest.mark.parametrize("tile", [128, 256])
def test_igemm_big_wgrad(cuda, B, H, W, C, O, KS, stride, pad, tile):
    g = torch.Generator(device=cuda).manual_seed(3 + H + O + tile)
    OH, OW = (H + 2 * pad - KS) // stride + 1, (W + 2 * pad - KS) // stride + 1
    x = _rand((B, H, W, C), g, cuda)
    dy = _rand((B, OH, OW, O), g, cuda, 0.1)
    xr = x.float().permute(0, 3, 1, 2)
    dyr = dy.float().permute(0, 3, 1, 2)
    ref_w = torch.nn.grad.conv2d_weight(xr, (O, C, KS, KS), dyr, stride=stride, padding=pad)
    ref_b = dyr.sum((0, 2, 3))
    gw, gb = ops.conv2d_wgrad_nhwc(dy, x, KS, stride=stride, pad=pad, tile=tile)
    assert _relerr(gw, ref_w) < 1e-3
    assert _relerr(gb, ref_b) < 1e-3
    # per output channel: a wrong channel fragment cannot hide in the whole-tensor norm
    cw = ((gw - ref_w).flatten(1).norm(dim=1) / ref_w.flatten(1).norm(dim=1).clamp_min(1e-12))
    assert float(cw.max()) < 3e-3
    assert float(((gb - ref_b).abs() / ref_b.abs().clamp_min(1e-3)).max()) < 1e-2
    gw2, gb2 = ops.conv2d_wgrad_nhwc(dy, x, KS, stride=stride, pad=pad, tile=tile)
    assert torch.equal(gw, gw2) and torch.equal(gb, gb2)
    gw1, gb1 = ops.conv2d_wgrad_nhwc(dy, x, KS, stride=stride, pad=pad, splitk=1, tile=tile)
    assert _relerr(gw1, ref_w) < 1e-3 and _relerr(gb1, ref_b) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("hw", [80, 66])  # 66: rows not dword-aligned -> byte path in both
def test_u8_first_layer_runs_match_bytes(cuda, monkeypatch, hw):
    """First-layer u8 staging from dword image-row runs (C=3, 3x3, pad 1) vs
    the single-byte gather: bit-identical logits and gradients through the
    engine (same bf16 rounding of byte/255), incl. the left/right/top/bottom
    zero padding and a sample-index gather."""
    import numpy as np
    import mpi_cuda_cnn_amd as mcc

    spec = mcc.parse_model_spec(f"input 3 {hw} {hw}; conv 64 k3 s1 p1 relu; pool 2; conv 64 k3 s1 p1 relu; "
                                "fc 32 relu; fc 10 softmax", "u8runs")
    B = 6
    imgs, labels = mcc.synth_dataset(3 * B, 3, hw, hw, 10, seed=4)
    imgs = np.random.default_rng(1).integers(0, 256, imgs.shape, dtype=np.uint8)  # every byte position matters
    params = mcc.init_params(spec, seed=3).astype(np.float32)
    d_img = torch.from_numpy(imgs).to(cuda)
    d_lab = torch.from_numpy(labels).to(cuda)
    idx = torch.tensor([5, 0, 17, 3, 3, 9], dtype=torch.int32, device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MCC_AB", "" if mode == "1" else "u8_bytes")
        net = mcc.GpuNet(spec, "bf16", B)
        net.set_params(params)
        net.zero_stats(s)
        net.forward(d_img.data_ptr(), idx.data_ptr(), B, s)
        net.loss(d_lab.data_ptr(), idx.data_ptr(), 1.0 / B, True, s)
        net.backward_all(s)
        torch.cuda.synchronize()
        out[mode] = (net.plan(), net.get_logits(B), net.get_grads())
        del net
    assert "igemm" in out["1"][0], out["1"][0]
    np.testing.assert_array_equal(out["1"][1], out["0"][1])
    np.testing.assert_array_equal(out["1"][2], out["0"][2])
