"""Torch-tensor entry points for the gfx950 kernels.

The training engine (``GpuNet``) calls the kernels on its own arena; these
wrappers make the same kernels usable on ordinary torch tensors (CUDA/HIP
device tensors, contiguous, bf16 or fp32), e.g. to build other models or to
test a kernel in isolation.  They launch on the current torch stream and
fail loudly on CPU tensors: there is no eager fallback.

    linear(x, w, b, act)            y = act(x @ w.T + b)            (MFMA GEMM, fused epilogue)
    linear_dgrad(dy, w, y_prev, act) dx = (dy @ w) * act'(y_prev)
    linear_wgrad(dy, x)             (dW, db) = (dy.T @ x, dy.sum(0)) (split-K, ones-column bias)
    softmax_xent(logits, labels)    dlogits, loss_sum, mse_sum, correct
    sgd_(p, g, mom, lr, mu, wd)     in-place SGD / momentum / weight decay
    conv2d_nhwc(x, w, b, s, p, act) y = act(conv2d(x, w) + b), NHWC bf16 (implicit-GEMM MFMA)
    conv2d_dgrad_nhwc(dy, w, ...)   dx of a stride-1 conv (the same kernel on flipped weights)
    conv2d_wgrad_nhwc(dy, x, ...)   (dW OIHW fp32, db fp32) split-K implicit GEMM

Reference counterparts: Layer_feedForw_full / Layer_feedBack_full
(cnn.c:113-173), Layer_feedForw_conv / Layer_feedBack_conv (cnn.c:175-247) and
the CUDA offload forward_convolution_layer (CUDAcnn.cu:167-218), the softmax + error of cnn.c:125-143,275-287 and
Layer_update (cnn.c:303-314).
"""

from __future__ import annotations

import torch

from .. import _C

_K = _C.kernels
_ACT = {"none": _K.ACT_NONE, "relu": _K.ACT_RELU, "tanh": _K.ACT_TANH}
_DT = {torch.bfloat16: "bf16", torch.float32: "fp32"}



STAT_SCALE = float(2**32)  # loss / mse statistics: u64 fixed point (kernels.h kStatScale)

def _check(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("mpi_cuda_cnn_amd.ops: tensors must be on the GPU (no CPU fallback)")
        if not t.is_contiguous():
            raise RuntimeError("mpi_cuda_cnn_amd.ops: tensors must be contiguous")


def _dtype(t):
    if t.dtype not in _DT:
        raise RuntimeError(f"mpi_cuda_cnn_amd.ops: unsupported dtype {t.dtype} (bf16 / fp32)")
    return _DT[t.dtype]


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _ld8(n):
    return (n + 7) // 8 * 8


def _pad_cols(t, ld):
    if t.shape[1] == ld:
        return t
    out = torch.zeros(t.shape[0], ld, dtype=t.dtype, device=t.device)
    out[:, : t.shape[1]] = t
    return out


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, act: str = "none") -> torch.Tensor:
    """y = act(x @ w.T + b); x [M, K], w [N, K] (same dtype), b fp32 [N]."""
    _check(x, w, b)
    dt = _dtype(x)
    M, K = x.shape
    N = w.shape[0]
    ldk = _ld8(K)
    xa, wa = _pad_cols(x, ldk), _pad_cols(w, ldk)
    ldc = _ld8(N)
    y = torch.empty(M, ldc, dtype=x.dtype, device=x.device)
    bias = b.float().contiguous() if b is not None else None
    _K.gemm(dt, M, N, K, xa.data_ptr(), ldk, False, wa.data_ptr(), ldk, False, epi=_K.EPI_BIAS_ACT,
            act=_ACT[act], bias=bias.data_ptr() if bias is not None else 0, C=y.data_ptr(), ldc=ldc,
            stream=_stream())
    return y[:, :N] if ldc != N else y


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, y_prev: torch.Tensor | None = None,
                 act: str = "none") -> torch.Tensor:
    """dx = (dy @ w) * act'(y_prev); dy [M, N], w [N, K]; act' from the activation OUTPUT y_prev [M, K]."""
    _check(dy, w, y_prev)
    dt = _dtype(dy)
    M, N = dy.shape
    K = w.shape[1]
    wt = _pad_cols(w.t().contiguous(), _ld8(N))  # [K, N]: the B operand stays K(=N)-contiguous
    ldn = _ld8(N)
    dya = _pad_cols(dy, ldn)
    ldc = _ld8(K)
    dx = torch.empty(M, ldc, dtype=dy.dtype, device=dy.device)
    aux = _pad_cols(y_prev.contiguous(), ldc) if (y_prev is not None and act != "none") else None
    _K.gemm(dt, M, K, N, dya.data_ptr(), ldn, False, wt.data_ptr(), ldn, False, epi=_K.EPI_DACT,
            act=_ACT[act] if aux is not None else _K.ACT_NONE, aux=aux.data_ptr() if aux is not None else 0,
            ldaux=ldc, C=dx.data_ptr(), ldc=ldc, stream=_stream())
    return dx[:, :K] if ldc != K else dx


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, splitk: int = 0):
    """(dW [N, K] fp32, db [N] fp32) = (dy.T @ x, dy.sum(0)): split-K over the batch, the
    bias gradient as a ones-column appended to x (one GEMM, no separate reduction pass)."""
    _check(dy, x)
    dt = _dtype(dy)
    M, N = dy.shape
    K = x.shape[1]
    ldn, ldk = _ld8(N), _ld8(K)
    dya, xa = _pad_cols(dy, ldn), _pad_cols(x, ldk)
    ldp = _ld8(K + 1)
    if splitk <= 0:
        tiles = ((N + 63) // 64) * ((K + 64) // 64)
        splitk = max(1, min(64, 512 // max(1, tiles), M // 128))
    part = torch.empty(splitk, N, ldp, dtype=torch.float32, device=dy.device)
    _K.gemm(dt, N, K + 1, M, dya.data_ptr(), ldn, True, xa.data_ptr(), ldk, True, ones_col=K,
            epi=_K.EPI_PARTIAL, Cf=part.data_ptr(), ldc=ldp, splitk=splitk, pstride=N * ldp, stream=_stream())
    tot = part.sum(0)
    return tot[:, :K].contiguous(), tot[:, K].contiguous()


def softmax_xent(logits: torch.Tensor, labels: torch.Tensor, scale: float = 1.0, grad_dtype=torch.float32):
    """Fused softmax-cross-entropy forward + backward on fp32 logits [M, N] and u8 labels [M].

    Returns (dlogits = (softmax - onehot) * scale [M, N], loss_sum, mse_sum, correct) where mse is
    the reference's logged error, mean((p - y)^2) per sample (cnn.c:275-282), and correct counts
    argmax == label with the first maximum winning (cnn.c:508-513)."""
    _check(logits, labels)
    if logits.dtype != torch.float32:
        raise RuntimeError("softmax_xent: logits must be fp32")
    M, N = logits.shape
    lab = labels.to(torch.uint8).contiguous()
    ldd = _ld8(N)
    d = torch.empty(M, ldd, dtype=grad_dtype, device=logits.device)
    stats = torch.zeros(4, dtype=torch.int64, device=logits.device)  # fixed point, see kStatScale
    _K.softmax_xent(_DT[grad_dtype], M, N, logits.data_ptr(), N, lab.data_ptr(), dlogits=d.data_ptr(), ldd=ldd,
                    scale=scale, stats=stats.data_ptr(), stream=_stream())
    f = stats.to(torch.float64)
    return d[:, :N], f[0] / STAT_SCALE, f[1] / STAT_SCALE, f[2]


def sgd_(param: torch.Tensor, grad: torch.Tensor, mom: torch.Tensor | None = None, lr: float = 0.1,
         momentum: float = 0.0, weight_decay: float = 0.0) -> torch.Tensor:
    """In place on fp32 tensors: v = mu*v + (g + wd*p); p -= lr*v (plain SGD when mom is None)."""
    _check(param, grad, mom)
    if param.dtype != torch.float32 or grad.dtype != torch.float32:
        raise RuntimeError("sgd_: fp32 master parameters and gradients")
    _K.sgd_update(param.data_ptr(), grad.data_ptr(), mom.data_ptr() if mom is not None else 0, param.numel(), lr,
                  momentum=momentum if mom is not None else 0.0, weight_decay=weight_decay, stream=_stream())
    return param


def _conv_geom(H, W, KS, stride, pad):
    return (H + 2 * pad - KS) // stride + 1, (W + 2 * pad - KS) // stride + 1


def pack_conv_weight(w: torch.Tensor) -> torch.Tensor:
    """OIHW -> [O][(kh*KS + kw)*I + i] bf16 (the implicit-GEMM K order)."""
    O, I, KH, KW = w.shape
    return w.permute(0, 2, 3, 1).reshape(O, KH * KW * I).to(torch.bfloat16).contiguous()


def conv2d_nhwc(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, stride: int = 1, pad: int = 0,
                act: str = "none", pool: bool = False, tile: int = -1):
    """y = act(conv2d(x, w, b)) on channels-last bf16: x [B, H, W, C] (C % 32 == 0), w OIHW -> y [B, OH, OW, O].

    pool=True fuses a 2x2/2 max-pool (returns (y_pooled, argmax bytes [B, OH/2, OW/2, O])).
    tile selects the kernel (igemm.hip): -1 auto, 0 the 128x128 kernel, 128 / 256 the
    256-pixel x 128 / 256-channel phase-pipelined kernel (where O allows it)."""
    _check(x, b)
    if x.dtype != torch.bfloat16:
        raise RuntimeError("conv2d_nhwc: bf16 activations")
    B, H, W, C = x.shape
    O, I, KS, KS2 = w.shape
    if I != C or KS != KS2 or not _K.igemm_conv_supported(C, O, KS):
        raise RuntimeError("conv2d_nhwc: needs square kernels, C % 32 == 0 and O % 8 == 0")
    wp = pack_conv_weight(w)
    OH, OW = _conv_geom(H, W, KS, stride, pad)
    if pool and (OH % 2 or OW % 2):
        raise RuntimeError("conv2d_nhwc: the fused pool needs even output dims")
    PH, PW = (OH // 2, OW // 2) if pool else (OH, OW)
    y = torch.empty(B, PH, PW, O, dtype=torch.bfloat16, device=x.device)
    arg = torch.empty(B, PH, PW, O, dtype=torch.uint8, device=x.device) if pool else None
    bias = b.float().contiguous() if b is not None else None
    _K.igemm_conv(B, H, W, C, O, KS, stride, pad, x.data_ptr(), wp.data_ptr(), wp.shape[1],
                  bias=bias.data_ptr() if bias is not None else 0, bias_act=True, act=_ACT[act], out=y.data_ptr(),
                  ldo=O, out_arg=arg.data_ptr() if pool else 0, tile=tile, stream=_stream())
    return (y, arg) if pool else y


def conv2d_dgrad_nhwc(dy: torch.Tensor, w: torch.Tensor, pad: int = 0, tile: int = -1) -> torch.Tensor:
    """dx of a stride-1 conv: dy [B, OH, OW, O] bf16 (O % 32 == 0), w OIHW -> dx [B, H, W, I]."""
    _check(dy)
    B, OH, OW, O = dy.shape
    Oc, I, KS, _ = w.shape
    if Oc != O or not _K.igemm_conv_supported(O, I, KS):
        raise RuntimeError("conv2d_dgrad_nhwc: needs O % 32 == 0 and I % 8 == 0")
    wf = w.flip(2, 3).permute(1, 2, 3, 0).reshape(I, KS * KS * O).to(torch.bfloat16).contiguous()
    pd = KS - 1 - pad
    H, W = _conv_geom(OH, OW, KS, 1, pd)
    dx = torch.empty(B, H, W, I, dtype=torch.bfloat16, device=dy.device)
    _K.igemm_conv(B, OH, OW, O, I, KS, 1, pd, dy.data_ptr(), wf.data_ptr(), wf.shape[1], bias_act=False,
                  out=dx.data_ptr(), ldo=I, tile=tile, stream=_stream())
    return dx


def conv2d_wgrad_nhwc(dy: torch.Tensor, x: torch.Tensor, KS: int, stride: int = 1, pad: int = 0, splitk: int = 0,
                      tile: int = -1):
    """(dW [O, I, KS, KS] fp32, db [O] fp32) for dy [B, OH, OW, O], x [B, H, W, I] bf16 NHWC.

    tile: -1 auto, 0 the 128x128 kernel, 128 / 256 the phase-pipelined O-tile x 256 kernel (O % 128 == 0)."""
    _check(dy, x)
    B, H, W, C = x.shape
    O = dy.shape[3]
    OH, OW = _conv_geom(H, W, KS, stride, pad)
    if tuple(dy.shape) != (B, OH, OW, O) or C % 8 or O % 8:
        raise RuntimeError("conv2d_wgrad_nhwc: shape mismatch or channels not multiples of 8")
    kf = KS * KS * C
    M = B * OH * OW
    if splitk <= 0:
        splitk = _K.igemm_dw_splitk(M, O, kf, tile)
    slab = torch.empty(splitk, kf + 1, O, dtype=torch.float32, device=x.device)
    gw = torch.empty(O, C, KS, KS, dtype=torch.float32, device=x.device)
    gb = torch.empty(O, dtype=torch.float32, device=x.device)
    _K.igemm_dw(B, H, W, C, O, KS, stride, pad, dy.data_ptr(), O, x.data_ptr(), slab.data_ptr(), (kf + 1) * O,
                splitk, gw.data_ptr(), gb.data_ptr(), tile=tile, stream=_stream())
    return gw, gb


__all__ = ["linear", "linear_dgrad", "linear_wgrad", "softmax_xent", "sgd_", "conv2d_nhwc", "conv2d_dgrad_nhwc",
           "conv2d_wgrad_nhwc", "pack_conv_weight"]
