"""Plain-PyTorch fp32/fp64 oracle of a model spec.

Used only by tests and validation: it builds the same network as the native
engine from a ``ModelSpec`` (NCHW, canonical parameter layouts) and loads the
framework's flat canonical parameter vector, so kernel outputs and gradients
can be compared against ``torch.nn`` reference ops.
"""

from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class _RoundBF16(torch.autograd.Function):
    """Round to bf16 in the forward AND the backward (a stored activation and
    the gradient that flows back into it are both bf16 in the engine)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


class _RoundBF16Weight(torch.autograd.Function):
    """bf16 compute copy of a parameter: rounded forward, gradient passed to
    the fp32/fp64 master unchanged."""

    @staticmethod
    def forward(ctx, w):
        return w.to(torch.bfloat16).to(w.dtype)

    @staticmethod
    def backward(ctx, g):
        return g


class TorchReference(nn.Module):
    """``mimic_bf16``: the oracle of the bf16 engine's rounding points --
    bf16 weight copies, every stored hidden activation (a conv fused with its
    max-pool stores only the pooled value) and the gradient flowing back into
    it rounded to bf16, fp64 everywhere else (accumulation, logits,
    loss).  Fed the same rounded operands, the engine's per-channel errors
    are then only its fp32 accumulation order, so tests can bound them
    tightly per output channel.

    ``u8_fp32_first``: the first layer's VALUE as the exact-integer u8 kernels
    compute it -- the integer sum (exact), x (1/255) and + bias in fp32 --
    while its gradient stays the fp64 one of conv(x/255).  Without it the
    fp64 oracle and the fp32 scale land on different sides of a bf16
    rounding boundary a few times per 10^5 activations, and in a batch of a
    few images one flipped pool / ReLU decision moves a sparse channel's
    gradient by O(0.1)."""

    def __init__(self, spec, dtype=torch.float32, mimic_bf16=False, u8_fp32_first=False):
        super().__init__()
        self.u8_fp32_first = u8_fp32_first
        self.spec = spec
        self.mimic_bf16 = mimic_bf16
        self.layer_info = spec.layers()
        mods = []
        for L in self.layer_info[1:]:
            if L["kind"] == "conv":
                mods.append(nn.Conv2d(L["inC"], L["C"], L["ks"], L["stride"], L["pad"], dtype=dtype))
            elif L["kind"] == "maxpool":
                mods.append(nn.MaxPool2d(L["ks"], L["stride"]))
            elif L["kind"] == "fc":
                nin = L["inC"] * L["inH"] * L["inW"]
                mods.append(nn.Linear(nin, L["C"], dtype=dtype))
            else:
                raise ValueError(L["kind"])
        self.mods = nn.ModuleList(mods)

    @torch.no_grad()
    def load_flat(self, flat):
        flat = torch.as_tensor(flat)
        for L, m in zip(self.layer_info[1:], self.mods):
            if L["nweights"] == 0:
                continue
            w = flat[L["w_off"] : L["w_off"] + L["nweights"]].reshape(m.weight.shape)
            b = flat[L["b_off"] : L["b_off"] + L["nbiases"]]
            m.weight.copy_(w.to(m.weight.dtype))
            m.bias.copy_(b.to(m.bias.dtype))

    def flat_grads(self):
        parts = []
        for L, m in zip(self.layer_info[1:], self.mods):
            if L["nweights"] == 0:
                continue
            parts.append(m.weight.grad.reshape(-1))
            parts.append(m.bias.grad.reshape(-1))
        return torch.cat(parts)

    def flat_params(self):
        parts = []
        for L, m in zip(self.layer_info[1:], self.mods):
            if L["nweights"] == 0:
                continue
            parts.append(m.weight.detach().reshape(-1))
            parts.append(m.bias.detach().reshape(-1))
        return torch.cat(parts)

    def forward(self, x, forced=None):
        """x: NCHW float in [0,1]. Returns logits (pre-softmax).

        ``forced`` (mimic_bf16 only): per fused stage (a conv with its max-pool,
        or an fc), None or the VALUE the engine stored for that stage's output
        (NCHW / [B, N]).  The oracle then continues from the engine's own
        activations (straight-through: the value is replaced, the gradient
        flows through the oracle's graph), so each layer's gradient is checked
        on the engine's forward state: in a deep bf16 net, one-ulp differences
        otherwise grow through the layers until ReLU / pool decisions near 0
        flip between engine and oracle."""
        n = len(self.mods)
        stage = 0
        for i, (L, m) in enumerate(zip(self.layer_info[1:], self.mods)):
            if L["kind"] == "fc" and x.dim() > 2:
                x = x.reshape(x.shape[0], -1)
            if self.mimic_bf16 and L["kind"] in ("conv", "fc"):
                w, b = _RoundBF16Weight.apply(m.weight), m.bias
                xin = x
                x = (F.conv2d(x, w, b, m.stride, m.padding) if L["kind"] == "conv" else F.linear(x, w, b))
                if i == 0 and self.u8_fp32_first and L["kind"] == "conv":
                    with torch.no_grad():  # integer sum, then fp32 scale and bias (value only)
                        s_int = F.conv2d(torch.round(xin * 255.0), w, None, m.stride, m.padding)
                        v = (s_int.float() * torch.tensor(1.0 / 255.0, dtype=torch.float32)
                             + b.detach().float().view(1, -1, 1, 1))
                    x = x + (v.to(x.dtype) - x).detach()
            else:
                x = m(x)
            if i == n - 1:
                break
            act = L["act"]
            if L["kind"] != "maxpool":
                if act == "relu":
                    x = F.relu(x)
                elif act == "tanh":
                    x = torch.tanh(x)
            # a conv fused with the following max-pool stores only the pooled
            # value (the max is taken on the unrounded sums)
            nxt = self.layer_info[i + 2] if i + 2 < len(self.layer_info) else None
            if self.mimic_bf16 and not (nxt is not None and nxt["kind"] == "maxpool"):
                x = _RoundBF16.apply(x)
                if forced is not None and stage < len(forced) and forced[stage] is not None:
                    f = forced[stage].to(x.dtype).reshape(x.shape)
                    x = x + (f - x).detach()
                stage += 1
        return x


def images_to_nchw(images_u8, dtype=torch.float32):
    """[N,H,W,C] uint8 -> [N,C,H,W] float / 255 (cnn.c:457)."""
    t = torch.as_tensor(images_u8)
    return t.permute(0, 3, 1, 2).to(dtype) / 255.0
