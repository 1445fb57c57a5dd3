"""Per-kernel numerics on the MI355X vs plain PyTorch fp32 references.

GEMM: every operand orientation (A/B row- or K-major — the K-major bf16 path
uses the ds_read_b64_tr_b16 hardware transpose), every tile configuration the
dispatcher can pick, every epilogue, split-K partials, the ones-column bias
trick, and an asymmetric B (a symmetric one hides a transposed C write).
"""

import numpy as np
import pytest
import torch

import mpi_cuda_cnn_amd as mcc

K_ = mcc._C.kernels
TDT = {"bf16": torch.bfloat16, "fp32": torch.float32}


def _s():
    return torch.cuda.current_stream().cuda_stream


def _stored(x, trans, ld):
    """x: logical [R][K]; returns storage tensor and pointer with leading dim ld."""
    R, K = x.shape
    if not trans:
        buf = torch.zeros(R, ld, dtype=x.dtype, device=x.device)
        buf[:, :K] = x
    else:
        buf = torch.zeros(K, ld, dtype=x.dtype, device=x.device)
        buf[:, :R] = x.t()
    return buf


SHAPES = [(96, 120, 400), (16384, 120, 400), (1000, 84, 120), (257, 10, 84), (120, 401, 2048), (64, 200, 1568),
          (4096, 256, 2048), (48, 1000, 4096), (2048, 64, 27)]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_gemm_orientations_and_tiles(cuda, dtype, ta, tb):
    g = torch.Generator(device=cuda).manual_seed(0)
    for M, N, K in SHAPES:
        A = torch.randn(M, K, device=cuda, generator=g).to(TDT[dtype])
        Bm = (torch.randn(N, K, device=cuda, generator=g) + torch.arange(N, device=cuda)[:, None] * 0.01).to(TDT[dtype])
        lda = ((M if ta else K) + 7) // 8 * 8
        ldb = ((N if tb else K) + 7) // 8 * 8
        As, Bs = _stored(A, ta, lda), _stored(Bm, tb, ldb)
        ldc = (N + 7) // 8 * 8
        Cf = torch.zeros(M, ldc, device=cuda)
        bias = torch.randn(N, device=cuda, generator=g)
        K_.gemm(dtype, M, N, K, As.data_ptr(), lda, ta, Bs.data_ptr(), ldb, tb, epi=K_.EPI_LOGITS,
                bias=bias.data_ptr(), ldc=ldc, Cf=Cf.data_ptr(), stream=_s())
        torch.cuda.synchronize()
        ref = A.float() @ Bm.float().t() + bias
        err = (Cf[:, :N] - ref).abs().max().item() / max(1e-6, ref.abs().max().item())
        tol = 2e-5 if dtype == "fp32" else 2e-2
        assert err < tol, (M, N, K, ta, tb, err)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_gemm_epilogues(cuda, dtype):
    g = torch.Generator(device=cuda).manual_seed(1)
    M, N, K = 300, 120, 256
    A = torch.randn(M, K, device=cuda, generator=g).to(TDT[dtype])
    Bm = torch.randn(N, K, device=cuda, generator=g).to(TDT[dtype])
    bias = torch.randn(N, device=cuda, generator=g)
    ref = A.float() @ Bm.float().t()
    tol = 2e-5 if dtype == "fp32" else 3e-2
    for act, fn in ((K_.ACT_RELU, torch.relu), (K_.ACT_TANH, torch.tanh), (K_.ACT_NONE, lambda x: x)):
        C = torch.zeros(M, 120, device=cuda, dtype=TDT[dtype])
        K_.gemm(dtype, M, N, K, A.data_ptr(), K, False, Bm.data_ptr(), K, False, epi=K_.EPI_BIAS_ACT, act=act,
                bias=bias.data_ptr(), C=C.data_ptr(), ldc=120, stream=_s())
        torch.cuda.synchronize()
        torch.testing.assert_close(C.float(), fn(ref + bias), atol=tol * 10, rtol=tol)
    # EPI_DACT: acc * act'(aux) with aux = activation output
    aux = torch.tanh(torch.randn(M, N, device=cuda, generator=g)).to(TDT[dtype])
    for act, d in ((K_.ACT_TANH, 1 - aux.float() ** 2), (K_.ACT_RELU, (aux.float() > 0).float())):
        C = torch.zeros(M, 120, device=cuda, dtype=TDT[dtype])
        K_.gemm(dtype, M, N, K, A.data_ptr(), K, False, Bm.data_ptr(), K, False, epi=K_.EPI_DACT, act=act,
                aux=aux.data_ptr(), ldaux=120, C=C.data_ptr(), ldc=120, stream=_s())
        torch.cuda.synchronize()
        torch.testing.assert_close(C.float(), ref * d, atol=tol * 10, rtol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_gemm_splitk_partials_with_ones_column(cuda, dtype):
    """dW = dY^T [X | 1]: both operands K-major (batch-major storage)."""
    g = torch.Generator(device=cuda).manual_seed(2)
    Bt, Nout, Kin = 4096, 120, 400
    dY = torch.randn(Bt, Nout, device=cuda, generator=g).to(TDT[dtype])
    X = torch.randn(Bt, Kin, device=cuda, generator=g).to(TDT[dtype])
    S = 8
    ldp = (Kin + 1 + 7) // 8 * 8
    part = torch.zeros(S, Nout, ldp, device=cuda)
    K_.gemm(dtype, Nout, Kin + 1, Bt, dY.data_ptr(), Nout, True, X.data_ptr(), Kin, True, ones_col=Kin,
            epi=K_.EPI_PARTIAL, Cf=part.data_ptr(), ldc=ldp, splitk=S, pstride=Nout * ldp, stream=_s())
    torch.cuda.synchronize()
    tot = part.sum(0)
    refW = dY.float().t() @ X.float()
    refb = dY.float().sum(0)
    tol = 1e-4 if dtype == "fp32" else 2e-2
    assert ((tot[:, :Kin] - refW).abs().max() / refW.abs().max()).item() < tol
    assert ((tot[:, Kin] - refb).abs().max() / refb.abs().max()).item() < tol


@pytest.mark.gpu
def test_softmax_xent_kernel(cuda):
    g = torch.Generator(device=cuda).manual_seed(3)
    M, N = 1000, 10
    logits = torch.randn(M, 16, device=cuda, generator=g) * 3
    labels = torch.randint(0, N, (M,), device=cuda, generator=g).to(torch.uint8)
    dl = torch.zeros(M, 16, device=cuda)
    stats = torch.zeros(4, dtype=torch.int64, device=cuda)  # u64 fixed point
    pred = torch.zeros(M, dtype=torch.int32, device=cuda)
    K_.softmax_xent("fp32", M, N, logits.data_ptr(), 16, labels.data_ptr(), dlogits=dl.data_ptr(), ldd=16,
                    scale=0.5, stats=stats.data_ptr(), pred=pred.data_ptr(), stream=_s())
    torch.cuda.synchronize()
    lg = logits[:, :N]
    p = torch.softmax(lg, 1)
    y = torch.nn.functional.one_hot(labels.long(), N).float()
    torch.testing.assert_close(dl[:, :N], (p - y) * 0.5, atol=1e-5, rtol=1e-4)
    ce = torch.nn.functional.cross_entropy(lg, labels.long(), reduction="sum")
    st = stats.double().cpu() / torch.tensor([2.0**32, 2.0**32, 1.0, 1.0], dtype=torch.float64)
    assert abs(st[0].item() - ce.item()) < 1e-3 * ce.item()
    assert abs(st[1].item() - ((p - y) ** 2).mean(1).sum().item()) < 1e-3
    assert int(stats[2].item()) == int((lg.argmax(1) == labels.long()).sum().item())
    assert torch.equal(pred.long(), lg.argmax(1))


# ---- mpi_cuda_cnn_amd.ops: the kernels on ordinary torch tensors ----

import mpi_cuda_cnn_amd.ops as ops  # noqa: E402


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("act", ["none", "relu", "tanh"])
def test_ops_linear_family(cuda, dtype, act):
    g = torch.Generator(device=cuda).manual_seed(7)
    M, N, K = 777, 84, 120  # odd shapes: ld padding paths
    x = torch.randn(M, K, device=cuda, generator=g).to(TDT[dtype])
    w = (torch.randn(N, K, device=cuda, generator=g) * 0.1).to(TDT[dtype])
    b = torch.randn(N, device=cuda, generator=g)
    fn = {"none": lambda t: t, "relu": torch.relu, "tanh": torch.tanh}[act]
    y = ops.linear(x, w, b, act)
    ref = fn(x.float() @ w.float().t() + b)
    tol = 1e-4 if dtype == "fp32" else 3e-2
    torch.testing.assert_close(y.float(), ref, atol=tol * 4, rtol=tol)
    dy = torch.randn(M, N, device=cuda, generator=g).to(TDT[dtype])
    dx = ops.linear_dgrad(dy, w, x if act != "none" else None, act)
    d = {"none": torch.ones_like, "relu": lambda t: (t > 0).float(), "tanh": lambda t: 1 - t * t}[act](x.float())
    torch.testing.assert_close(dx.float(), (dy.float() @ w.float()) * d, atol=tol * 10, rtol=tol * 2)
    dw, db = ops.linear_wgrad(dy, x)
    rw = dy.float().t() @ x.float()
    assert ((dw - rw).abs().max() / rw.abs().max()).item() < (1e-4 if dtype == "fp32" else 2e-2)
    torch.testing.assert_close(db, dy.float().sum(0), atol=1e-2, rtol=1e-2)


@pytest.mark.gpu
def test_ops_softmax_xent_and_sgd(cuda):
    g = torch.Generator(device=cuda).manual_seed(8)
    logits = torch.randn(513, 10, device=cuda, generator=g) * 2
    labels = torch.randint(0, 10, (513,), device=cuda, generator=g)
    d, loss, mse, correct = ops.softmax_xent(logits, labels, scale=1.0 / 513)
    p = torch.softmax(logits, 1)
    y = torch.nn.functional.one_hot(labels, 10).float()
    torch.testing.assert_close(d, (p - y) / 513, atol=1e-6, rtol=1e-4)
    assert abs(loss.item() - torch.nn.functional.cross_entropy(logits, labels, reduction="sum").item()) < 1e-2
    assert int(correct.item()) == int((logits.argmax(1) == labels).sum().item())
    w = torch.randn(1001, device=cuda, generator=g)
    gr = torch.randn(1001, device=cuda, generator=g)
    v = torch.zeros_like(w)
    w0 = w.clone()
    ops.sgd_(w, gr, v, lr=0.1, momentum=0.9, weight_decay=0.01)
    torch.testing.assert_close(w, w0 - 0.1 * (gr + 0.01 * w0), atol=1e-6, rtol=1e-6)
    with pytest.raises(RuntimeError):
        ops.linear(torch.zeros(4, 8), torch.zeros(4, 8))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("M,N,K,act", [(1000, 200, 1568, "tanh"), (4096 + 37, 200, 1568, "none"),
                                       (300, 1568, 200, "nobias"), (2 * 128 + 5, 224 + 8, 64 + 8, "nobias"),
                                       (2 * 128 + 5, 216, 64 + 8, "relu")])
def test_fc_tall_kernel(cuda, M, N, K, act, dtype):
    """fc_tall.hip (the reference model's FC1 forward and data gradient): every
    epilogue, ragged batch rows, a K tail, N spanning two column tiles (the
    data-gradient form; the bias epilogue covers one tile), several tiles per
    persistent workgroup (1568 = 7 column tiles);
    fp32 is exact f32 MFMA (checked tight against an fp64 product)."""
    g = torch.Generator().manual_seed(M + N)
    t = TDT[dtype]
    a = torch.randn(M, K, generator=g).to(t).to(cuda)
    w = (torch.randn(N, K, generator=g) / K**0.5).to(t).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    out = torch.full((M, N), 7.0, dtype=t, device=cuda)
    code = {"none": K_.ACT_NONE, "relu": K_.ACT_RELU, "tanh": K_.ACT_TANH, "nobias": K_.ACT_NONE}[act]
    K_.fc_tall(M, N, K, a.data_ptr(), K, w.data_ptr(), K, 0 if act == "nobias" else b.data_ptr(), code,
               out.data_ptr(), N, _s(), f32=dtype == "fp32")
    torch.cuda.synchronize()
    ref = a.double() @ w.double().t()
    if act != "nobias":
        ref = ref + b.double()
    ref = {"relu": torch.relu, "tanh": torch.tanh}.get(act, lambda x: x)(ref)
    err = float((out.double() - ref).norm() / ref.norm())
    assert err < (1e-5 if dtype == "fp32" else 1e-2), err
    assert float((out.double() - ref).abs().max()) < (1e-4 if dtype == "fp32" else 0.05) * float(ref.abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,M,N,K,act", [
    ("bf16", 4096 + 37, 1568, 200, "none"),   # ref FC1 data gradient (7 column slabs)
    ("bf16", 1000, 200, 200, "tanh"),         # ref FC2 data gradient x tanh'
    ("bf16", 3, 1568, 200, "none"),           # fewer rows than one block
    ("fp32", 2048 + 11, 1568, 200, "none"),   # ref fp32 FC1 (14 slabs of 112)
    ("fp32", 777, 200, 200, "tanh"),
    ("fp32", 4096 + 5, 400, 120, "none"),     # LeNet-5 fp32 FC1 data gradient (208 + 192)
    ("fp32", 1000, 120, 84, "relu"),          # LeNet-5 fp32 FC2 data gradient x ReLU'
])
def test_fc_wres_kernel(cuda, dtype, M, N, K, act):
    """fc_wres.hip (FC data gradient, W resident in LDS): out = (A W^T) x
    act'(aux) against an fp64 product; ragged rows, K tails inside the last
    64-byte k-step (K = 200 bf16 / 84 fp32), a partial last column slab, the
    aux epilogue.  The padding columns of A and W hold NaN: the kernel must
    never read them (its k tail uses clamped in-row addresses)."""
    g = torch.Generator().manual_seed(M + N + K)
    t = TDT[dtype]
    f32 = dtype == "fp32"
    code = {"none": K_.ACT_NONE, "relu": K_.ACT_RELU, "tanh": K_.ACT_TANH}[act]
    assert K_.fc_wres_supported(f32, M, N, K, code)
    lda, ldw, ldo = K + 8, K + 8, N + 8
    a = torch.full((M, lda), float("nan"), dtype=t)
    a[:, :K] = torch.randn(M, K, generator=g).to(t)
    a = a.to(cuda)
    w = torch.full((N, ldw), float("nan"), dtype=t)
    w[:, :K] = (torch.randn(N, K, generator=g) / K**0.5).to(t)
    w = w.to(cuda)
    y = torch.randn(M, N, generator=g)
    y = (torch.relu(y) if act == "relu" else torch.tanh(y)).to(t).to(cuda)
    out = torch.full((M, ldo), 7.0, dtype=t, device=cuda)
    K_.fc_wres(M, N, K, a.data_ptr(), lda, w.data_ptr(), ldw, code, y.data_ptr(), N, out.data_ptr(), ldo, _s(), f32=f32)
    torch.cuda.synchronize()
    ref = a[:, :K].double() @ w[:, :K].double().t()
    if act == "relu":
        ref = ref * (y.double() > 0)
    elif act == "tanh":
        ref = ref * (1 - y.double() ** 2)
    o = out[:, :N].double()
    assert bool(torch.isfinite(o).all())
    err = float((o - ref).norm() / ref.norm())
    assert err < (1e-6 if f32 else 1e-2), err
    assert float((o - ref).abs().max()) < (1e-5 if f32 else 0.05) * float(ref.abs().max())
    assert bool((out[:, N:] == 7.0).all())  # nothing written past N


@pytest.mark.gpu
@pytest.mark.parametrize("M", [640, 768, 896, 2])
def test_fc1_splitk_forward_vgg_shape(cuda, M):
    """VGG-11 FC1 (25,088 -> 4,096, bias + ReLU) on the engine's long-K
    forward: split-K 128x128 partials + the finishing bias/ReLU pass, at the
    bench batch (640) and the batches whose split count differs (768 -> 6,
    896 -> 5; 2 -> no split), against torch's fp32 matmul of the same bf16
    operands, per output channel (reference semantics: cnn.c:113-152)."""
    N, K = 4096, 25088
    g = torch.Generator(device=cuda).manual_seed(7)
    A = (torch.rand(M, K, device=cuda, generator=g) * 0.1).to(torch.bfloat16)  # ReLU'd activations
    W = (torch.randn(N, K, device=cuda, generator=g) * 0.01).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda, generator=g) * 0.05
    C = torch.zeros(M, N, device=cuda, dtype=torch.bfloat16)
    sk = K_.gemm_fwd_splitk(M, N, K)
    scratch = torch.empty(max(1, sk) * M * N, device=cuda, dtype=torch.float32)
    used = K_.gemm_splitk_fwd("bf16", M, N, K, A.data_ptr(), K, W.data_ptr(), K, K_.ACT_RELU, bias.data_ptr(),
                              C.data_ptr(), N, scratch.data_ptr(), splitk=0, stream=_s())
    torch.cuda.synchronize()
    assert used == sk >= 1, (M, sk)
    ref = torch.relu(A.float() @ W.float().t() + bias)
    err = (C.float() - ref).norm(dim=0) / ref.norm(dim=0).clamp_min(1e-3 * ref.norm() / N ** 0.5)
    # bf16 output rounding (2^-9 relative) dominates; a dropped split or K
    # slice would be O(1) on every channel
    assert err.max().item() < 1e-2, (err.max().item(), int(err.argmax()))


@pytest.mark.gpu
def test_sample_indices_advance_matches_two_launches(cuda):
    """The fused sampler (sample_indices_advance: one launch, the last
    workgroup advances the counter) draws the same index stream as
    sample_indices + advance_counter, eagerly and replayed from a graph."""
    K = mcc._C.kernels
    B, lo, hi, seed = 50_000, 3, 60_003, 0x5EED0007
    s = torch.cuda.current_stream().cuda_stream
    c2 = torch.zeros(1, dtype=torch.int64, device=cuda)
    ref = torch.empty(B, dtype=torch.int32, device=cuda)
    want = []
    for _ in range(6):
        K.sample_indices(ref.data_ptr(), B, lo, hi, seed, c2.data_ptr(), s)
        K.advance_counter(c2.data_ptr(), s)
        want.append(ref.clone())
    c1 = torch.zeros(2, dtype=torch.int64, device=cuda)
    got = torch.empty(B, dtype=torch.int32, device=cuda)
    out = []
    for _ in range(3):
        K.sample_indices_advance(got.data_ptr(), B, lo, hi, seed, c1.data_ptr(), s)
        out.append(got.clone())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        K.sample_indices_advance(got.data_ptr(), B, lo, hi, seed, c1.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
    for _ in range(2):  # the capture did not run the kernel; replays do
        g.replay()
        out.append(got.clone())
    torch.cuda.synchronize()
    assert c1.tolist() == [5, 0]
    for i, (a, b) in enumerate(zip(out, want)):
        assert torch.equal(a, b), f"step {i}"
    assert int(want[0].min()) >= lo and int(want[0].max()) < hi
