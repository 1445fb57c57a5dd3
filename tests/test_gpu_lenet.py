"""Unit tests of the LeNet-5 conv block kernels (csrc/kernels/lenet.hip).

lenet_forward (conv1 + ReLU + pool + conv2 + ReLU + pool in one kernel) is
checked tensor by tensor against a PyTorch oracle fed the same bf16 rounding
points (bf16 weights, exact-integer pixels, the bf16 pooled conv1 output);
lenet_backward (conv2 dW + conv2 dX + conv1 dW in one kernel) against an fp64
oracle built from the kernel's own forward tensors and argmax codes, so a
tie broken differently cannot route a gradient elsewhere.  Reference
semantics: /root/reference/cnn.c:175-247 (conv fwd/bwd, D1 fixed).
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mpi_cuda_cnn_amd import _C

K = _C.kernels


def _bf16(t):
    return t.to(torch.bfloat16).to(torch.float64)


def _case(B, seed, dev):
    g = torch.Generator().manual_seed(seed)
    N = B + 11
    x = torch.randint(0, 256, (N, 28, 28), generator=g, dtype=torch.uint8)
    x[:, :, :3] = 0  # flat regions (pooling ties)
    idx = torch.randperm(N, generator=g)[:B].to(torch.int32)
    w1 = torch.randn(6, 1, 5, 5, generator=g) * 0.3
    b1 = torch.randn(6, generator=g) * 0.1
    w2 = torch.randn(16, 6, 5, 5, generator=g) * 0.1
    b2 = torch.randn(16, generator=g) * 0.1
    d = dict(x=x.to(dev), idx=idx.to(dev), w1=w1.to(dev), b1=b1.to(dev), w2=w2.to(dev), b2=b2.to(dev))
    d["y1"] = torch.zeros(B, 14, 14, 8, dtype=torch.bfloat16, device=dev)
    d["a1"] = torch.full((B, 6, 14, 16), 77, dtype=torch.uint8, device=dev)
    d["y2"] = torch.zeros(B, 25, 16, dtype=torch.bfloat16, device=dev)
    d["a2"] = torch.full((B, 25, 16), 77, dtype=torch.uint8, device=dev)
    return d


def _run_fwd(d, B):
    s = torch.cuda.current_stream().cuda_stream
    K.lenet_forward(B, d["x"].data_ptr(), d["idx"].data_ptr(), d["w1"].data_ptr(), d["b1"].data_ptr(),
                    d["w2"].data_ptr(), d["b2"].data_ptr(), d["y1"].data_ptr(), d["a1"].data_ptr(),
                    d["y2"].data_ptr(), d["a2"].data_ptr(), s)
    torch.cuda.synchronize()


def _pool_codes(z):
    """2x2 max-pool of NCHW z: values and the window position (first max wins)."""
    Bn, C, H, W = z.shape
    win = z.reshape(Bn, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(Bn, C, H // 2, W // 2, 4)
    v, pos = win.max(dim=-1)  # torch returns the first max
    srt = win.sort(dim=-1, descending=True).values
    gap = srt[..., 0] - srt[..., 1]
    return v, pos, gap


@pytest.fixture(params=["", "bwd4_twobar", "lenet_fwd1,lenet_bwd2"], ids=["round6", "round5", "round4"])
def kernel_gen(request, monkeypatch):
    """The default kernels (window-in-lane forward lenet_fwd2, four-wave
    backward lenet_bwd4 on the one-barrier schedule), the round-5 two-barrier
    schedule of lenet_bwd4 (MCC_AB=bwd4_twobar) and, under
    MCC_AB=lenet_fwd1,lenet_bwd2, the round-4 pair: all against the same
    oracle."""
    monkeypatch.setenv("MCC_AB", request.param)
    return request.param


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 37, 300, 5000])
def test_lenet_forward_matches_oracle(cuda, B, kernel_gen):
    """(B = 5000 > the 4096-wave grid: waves that take a second image reuse
    their LDS tiles and the prefetched pixels)"""
    d = _case(B, 7 + B, cuda)
    _run_fwd(d, B)
    xs = d["x"].cpu()[d["idx"].cpu().long()].to(torch.float64)[:, None] / 255.0
    z1 = F.conv2d(xs, _bf16(d["w1"].cpu()), d["b1"].cpu().double(), padding=2)
    v1, pos1, gap1 = _pool_codes(z1)
    y1r = F.relu(v1)
    y1 = d["y1"].cpu().double()
    assert torch.all(y1[..., 6:] == 0), "Y1 channel padding must be zero"
    y1k = y1[..., :6].permute(0, 3, 1, 2)
    err = (y1k - y1r).abs() / (y1r.abs() + 1e-2)
    assert err.max() < 1.5e-2, f"Y1 max rel err {err.max():.3e}"
    a1 = d["a1"].cpu()[:, :, :, :14].long()
    code1 = torch.where(_bf16(y1r) > 0, pos1, torch.full_like(pos1, 4))
    sure = (gap1 > 1e-3 * (v1.abs() + 1e-3)) | (code1 == 4)
    assert torch.all((a1 == code1) | ~sure), f"A1 codes: {int(((a1 != code1) & sure).sum())} mismatches"
    # conv2 on the kernel's own bf16 Y1
    z2 = F.conv2d(y1k, _bf16(d["w2"].cpu()), d["b2"].cpu().double())
    v2, pos2, gap2 = _pool_codes(z2)
    y2r = F.relu(v2)
    y2 = d["y2"].cpu().double().reshape(B, 5, 5, 16).permute(0, 3, 1, 2)
    err2 = (y2 - y2r).abs() / (y2r.abs() + 1e-2)
    assert err2.max() < 1.5e-2, f"Y2 max rel err {err2.max():.3e}"
    a2 = d["a2"].cpu().reshape(B, 5, 5, 16).permute(0, 3, 1, 2).long()
    code2 = torch.where(_bf16(y2r) > 0, pos2, torch.full_like(pos2, 4))
    sure2 = (gap2 > 1e-3 * (v2.abs() + 1e-3)) | (code2 == 4)
    assert torch.all((a2 == code2) | ~sure2), f"A2 codes: {int(((a2 != code2) & sure2).sum())} mismatches"


def _unpool(dy, codes):
    """dy [B,C,h,w], codes [B,C,h,w] (0..3 or 4) -> [B,C,2h,2w]"""
    Bn, C, h, w = dy.shape
    out = torch.zeros(Bn, C, h, w, 4, dtype=dy.dtype)
    act = codes < 4
    out.scatter_(-1, codes.clamp(max=3)[..., None], torch.where(act, dy, torch.zeros_like(dy))[..., None])
    return out.reshape(Bn, C, h, w, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(Bn, C, 2 * h, 2 * w)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 37, 300, 1500, 2900])
def test_lenet_backward_matches_oracle(cuda, B, kernel_gen):
    """(B > 512: several images per workgroup of the four-wave kernel, so its
    one-image conv1-dW lag and double-buffered dZ1 / X0 are exercised, with a
    ragged tail)"""
    d = _case(B, 100 + B, cuda)
    _run_fwd(d, B)
    g = torch.Generator().manual_seed(B)
    dy2 = (torch.randn(B, 25, 16, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    slab = torch.empty(K.lenet_slab_bytes() // 4, dtype=torch.float32, device=cuda)
    gw1 = torch.full((6, 1, 5, 5), 123.0, device=cuda)
    gb1 = torch.full((6,), 123.0, device=cuda)
    gw2 = torch.full((16, 6, 5, 5), 123.0, device=cuda)
    gb2 = torch.full((16,), 123.0, device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    K.lenet_backward(B, d["x"].data_ptr(), d["idx"].data_ptr(), d["w2"].data_ptr(), dy2.data_ptr(),
                     d["a2"].data_ptr(), d["y1"].data_ptr(), d["a1"].data_ptr(), slab.data_ptr(),
                     gw1.data_ptr(), gb1.data_ptr(), gw2.data_ptr(), gb2.data_ptr(), s)
    torch.cuda.synchronize()
    # fp64 oracle on the kernel's tensors
    y1 = d["y1"].cpu().double()[..., :6].permute(0, 3, 1, 2)
    a1 = d["a1"].cpu()[:, :, :, :14].long()
    a2 = d["a2"].cpu().reshape(B, 5, 5, 16).permute(0, 3, 1, 2).long()
    dY2 = dy2.cpu().double().reshape(B, 5, 5, 16).permute(0, 3, 1, 2)
    dz2 = _unpool(dY2, a2)
    w2 = _bf16(d["w2"].cpu())
    rgw2 = torch.nn.grad.conv2d_weight(y1, w2.shape, dz2)
    rgb2 = dz2.sum(dim=(0, 2, 3))
    dy1 = torch.nn.grad.conv2d_input(y1.shape, w2, dz2)
    dz1 = _unpool(_bf16(dy1), a1)
    xs = d["x"].cpu()[d["idx"].cpu().long()].to(torch.float64)[:, None] / 255.0
    rgw1 = torch.nn.grad.conv2d_weight(xs, (6, 1, 5, 5), dz1, padding=2)
    rgb1 = dz1.sum(dim=(0, 2, 3))
    for name, got, ref in (("gw2", gw2, rgw2), ("gb2", gb2, rgb2), ("gw1", gw1, rgw1), ("gb1", gb1, rgb1)):
        got = got.cpu().double()
        rel = float((got - ref).norm() / max(ref.norm(), 1e-12))
        assert rel < 1e-2, f"{name} rel err {rel:.3e}"
        # per output channel as well (a wrong channel must not hide in the norm)
        gc, rc = got.reshape(got.shape[0], -1), ref.reshape(ref.shape[0], -1)
        pc = (gc - rc).norm(dim=1) / (rc.norm(dim=1) + 1e-3 * ref.norm() + 1e-12)
        assert pc.max() < 2e-2, f"{name} per-channel rel err {pc.max():.3e} (channel {int(pc.argmax())})"
