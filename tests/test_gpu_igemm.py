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
@pytest.mark.parametrize("B,H,W,C,O,KS,stride,pad", [c for c in CASES if c[6] == 1 and c[4] % 64 == 0])
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
