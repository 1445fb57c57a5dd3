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


class TorchReference(nn.Module):
    def __init__(self, spec, dtype=torch.float32):
        super().__init__()
        self.spec = spec
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

    def forward(self, x):
        """x: NCHW float in [0,1]. Returns logits (pre-softmax)."""
        n = len(self.mods)
        for i, (L, m) in enumerate(zip(self.layer_info[1:], self.mods)):
            if L["kind"] == "fc" and x.dim() > 2:
                x = x.reshape(x.shape[0], -1)
            x = m(x)
            if i == n - 1:
                break
            act = L["act"]
            if L["kind"] == "maxpool":
                continue
            if act == "relu":
                x = F.relu(x)
            elif act == "tanh":
                x = torch.tanh(x)
        return x


def images_to_nchw(images_u8, dtype=torch.float32):
    """[N,H,W,C] uint8 -> [N,C,H,W] float / 255 (cnn.c:457)."""
    t = torch.as_tensor(images_u8)
    return t.permute(0, 3, 1, 2).to(dtype) / 255.0
