"""Unit tests of the reference-model conv block kernels (csrc/kernels/refnet.hip,
fp32: refnet_f32.hip).

ref_forward (conv1 1->16 + ReLU + conv2 16->32 + ReLU, 3x3 stride 2 pad 1,
cnn.c:416-428) is checked against a PyTorch oracle fed the same bf16 rounding
points (bf16 weights, exact-integer pixels, bf16 Y1); ref_backward (recomputed
conv1, conv2 dW, sub-pixel conv2 dX, conv1 dW) against an fp64 oracle built
from the kernel's own Y2 and the same rounding points (bf16 Y1, bf16 dZ1).
The fp32 kernels are checked against the same oracles without the bf16
rounding points (fp32 products and accumulation vs fp64: ~1e-6 relative).
Reference semantics: /root/reference/cnn.c:175-247 (conv fwd/bwd, D1 fixed).
"""

import pytest
import torch
import torch.nn.functional as F

from mpi_cuda_cnn_amd import _C

K = _C.kernels


def _bf16(t):
    return t.to(torch.bfloat16).to(torch.float64)


def _round(t, f32):
    return t.to(torch.float64) if f32 else _bf16(t)


def _case(B, seed, dev, f32=False):
    g = torch.Generator().manual_seed(seed)
    N = B + 7
    x = torch.randint(0, 256, (N, 28, 28), generator=g, dtype=torch.uint8)
    x[:, :, :4] = 0
    idx = torch.randperm(N, generator=g)[:B].to(torch.int32)
    w1 = torch.randn(16, 1, 3, 3, generator=g) * 0.4
    b1 = torch.randn(16, generator=g) * 0.1
    w2 = torch.randn(32, 16, 3, 3, generator=g) * 0.15
    b2 = torch.randn(32, generator=g) * 0.1
    d = dict(x=x.to(dev), idx=idx.to(dev), w1=w1.to(dev), b1=b1.to(dev), w2=w2.to(dev), b2=b2.to(dev))
    d["y2"] = torch.full((B, 49, 32), 7.0, dtype=torch.float32 if f32 else torch.bfloat16, device=dev)
    d["f32"] = f32
    return d


def _run_fwd(d, B):
    s = torch.cuda.current_stream().cuda_stream
    K.ref_forward(B, d["x"].data_ptr(), d["idx"].data_ptr(), d["w1"].data_ptr(), d["b1"].data_ptr(),
                  d["w2"].data_ptr(), d["b2"].data_ptr(), d["y2"].data_ptr(), s, f32=d["f32"])
    torch.cuda.synchronize()


def _oracle_y1(d):
    xs = d["x"].cpu()[d["idx"].cpu().long()].to(torch.float64)[:, None] / 255.0
    z1 = F.conv2d(xs, _round(d["w1"].cpu(), d["f32"]), d["b1"].cpu().double(), stride=2, padding=1)
    return xs, _round(F.relu(z1), d["f32"])


DTYPES = [pytest.param(False, id="bf16"), pytest.param(True, id="fp32")]


@pytest.mark.gpu
@pytest.mark.parametrize("f32", DTYPES)
@pytest.mark.parametrize("B", [1, 37, 300])
def test_ref_forward_matches_oracle(cuda, B, f32):
    d = _case(B, 11 + B, cuda, f32)
    _run_fwd(d, B)
    _, y1 = _oracle_y1(d)
    z2 = F.conv2d(y1, _round(d["w2"].cpu(), f32), d["b2"].cpu().double(), stride=2, padding=1)
    y2r = F.relu(z2)  # [B, 32, 7, 7]
    y2 = d["y2"].cpu().double().reshape(B, 7, 7, 32).permute(0, 3, 1, 2)
    # elementwise bound loose enough for a Y1 element whose bf16 rounding flips
    # between the fp32 kernel and the fp64 oracle; the L2 bound is tight
    err = (y2 - y2r).abs() / (y2r.abs() + 1e-2)
    assert err.max() < (1e-4 if f32 else 3e-2), f"Y2 max rel err {err.max():.3e}"
    rel = float((y2 - y2r).norm() / y2r.norm())
    assert rel < (1e-5 if f32 else 4e-3), f"Y2 rel L2 err {rel:.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("f32", DTYPES)
@pytest.mark.parametrize("B", [1, 37, 300, 2900])  # 2900: several images per workgroup of the
def test_ref_backward_matches_oracle(cuda, B, f32):  # 1,024-group two-wave grid, ragged tail
    d = _case(B, 200 + B, cuda, f32)
    _run_fwd(d, B)
    g = torch.Generator().manual_seed(B)
    dy2 = (torch.randn(B, 49, 32, generator=g) * 0.05).to(torch.float32 if f32 else torch.bfloat16).to(cuda)
    slab = torch.empty(K.ref_slab_bytes(f32) // 4, dtype=torch.float32, device=cuda)
    gw1 = torch.full((16, 1, 3, 3), 123.0, device=cuda)
    gb1 = torch.full((16,), 123.0, device=cuda)
    gw2 = torch.full((32, 16, 3, 3), 123.0, device=cuda)
    gb2 = torch.full((32,), 123.0, device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    K.ref_backward(B, d["x"].data_ptr(), d["idx"].data_ptr(), d["w1"].data_ptr(), d["b1"].data_ptr(),
                   d["w2"].data_ptr(), d["y2"].data_ptr(), dy2.data_ptr(), slab.data_ptr(),
                   gw1.data_ptr(), gb1.data_ptr(), gw2.data_ptr(), gb2.data_ptr(), s, f32=f32)
    torch.cuda.synchronize()
    xs, y1 = _oracle_y1(d)
    y2 = d["y2"].cpu().double().reshape(B, 7, 7, 32).permute(0, 3, 1, 2)
    dz2 = dy2.cpu().double().reshape(B, 7, 7, 32).permute(0, 3, 1, 2) * (y2 > 0)
    w2 = _round(d["w2"].cpu(), f32)
    rgw2 = torch.nn.grad.conv2d_weight(y1, w2.shape, dz2, stride=2, padding=1)
    rgb2 = dz2.sum(dim=(0, 2, 3))
    dy1 = torch.nn.grad.conv2d_input(y1.shape, w2, dz2, stride=2, padding=1)
    dz1 = _round(dy1, f32) * (y1 > 0)
    rgw1 = torch.nn.grad.conv2d_weight(xs, (16, 1, 3, 3), dz1, stride=2, padding=1)
    rgb1 = dz1.sum(dim=(0, 2, 3))
    for name, got, ref in (("gw2", gw2, rgw2), ("gb2", gb2, rgb2), ("gw1", gw1, rgw1), ("gb1", gb1, rgb1)):
        got = got.cpu().double()
        rel = float((got - ref).norm() / max(ref.norm(), 1e-12))
        assert rel < (1e-5 if f32 else 1e-2), f"{name} rel err {rel:.3e}"
        gc, rc = got.reshape(got.shape[0], -1), ref.reshape(ref.shape[0], -1)
        pc = (gc - rc).norm(dim=1) / (rc.norm(dim=1) + 1e-3 * ref.norm() + 1e-12)
        assert pc.max() < (1e-4 if f32 else 2e-2), f"{name} per-channel rel err {pc.max():.3e} (channel {int(pc.argmax())})"
