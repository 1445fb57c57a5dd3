#!/usr/bin/env python3
"""Per-phase timing of lenet_bwd4 from a diagnostic build with s_memtime
stamps (tools/build_variant.sh stamp -DMCC_LENET_STAMP=1):

    PYTHONPATH=build/var_stamp python tools/probes/lenet_stamp_probe.py

Runs lenet_forward + lenet_backward at B = 163,840 through the kernel-level
bindings and prints, per wave role, the mean cycles of: barrier A wait,
compute (phase A), barrier B wait, staging (phase B), for images 2..15."""
import os
import sys

import numpy as np
import torch

from mpi_cuda_cnn_amd import _C

K = _C.kernels
assert "var_" in os.path.dirname(_C.__file__), _C.__file__
dev = torch.device("cuda", 0)
B = int(os.environ.get("PROBE_B", "163840"))
g = torch.Generator().manual_seed(0)
N = 65536
x = torch.randint(0, 256, (N, 28, 28), generator=g, dtype=torch.uint8).to(dev)
idx = torch.randint(0, N, (B,), generator=g, dtype=torch.int32).to(dev)
w1 = (torch.randn(6, 1, 5, 5, generator=g) * 0.3).to(dev)
b1 = (torch.randn(6, generator=g) * 0.1).to(dev)
w2 = (torch.randn(16, 6, 5, 5, generator=g) * 0.1).to(dev)
b2 = (torch.randn(16, generator=g) * 0.1).to(dev)
y1 = torch.zeros(B, 14, 14, 8, dtype=torch.bfloat16, device=dev)
a1 = torch.zeros(B, 6, 14, 16, dtype=torch.uint8, device=dev)
y2 = torch.zeros(B, 25, 16, dtype=torch.bfloat16, device=dev)
a2 = torch.zeros(B, 25, 16, dtype=torch.uint8, device=dev)
dy2 = (torch.randn(B, 25, 16, generator=g) * 0.05).to(torch.bfloat16).to(dev)
slab = torch.zeros(K.lenet_slab_bytes() // 4, dtype=torch.float32, device=dev)
gw1 = torch.zeros(6, 1, 5, 5, device=dev)
gb1 = torch.zeros(6, device=dev)
gw2 = torch.zeros(16, 6, 5, 5, device=dev)
gb2 = torch.zeros(16, device=dev)
s = torch.cuda.current_stream().cuda_stream
for it in range(3):
    K.lenet_forward(B, x.data_ptr(), idx.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
                    y1.data_ptr(), a1.data_ptr(), y2.data_ptr(), a2.data_ptr(), s)
    K.lenet_backward(B, x.data_ptr(), idx.data_ptr(), w2.data_ptr(), dy2.data_ptr(), a2.data_ptr(), y1.data_ptr(),
                     a1.data_ptr(), slab.data_ptr(), gw1.data_ptr(), gb1.data_ptr(), gw2.data_ptr(), gb2.data_ptr(), s)
torch.cuda.synchronize()
kslab = 13 * 4 * 64 + 4 * 64
raw = slab.view(torch.int64)[(512 * kslab) // 2:(512 * kslab) // 2 + 512 * 4 * 5].cpu().numpy()
st = raw.reshape(512, 4, 5).astype(np.float64)
names = ["w0", "w1", "w2", "w3"]
n = st[:, 0, 4].sum()
tot = st[:, 0, :4].sum() / n
print(f"{os.path.basename(os.path.dirname(os.path.dirname(_C.__file__)))} B={B}: image period {tot:.0f} cycles (s_memtime), "
      f"{int(n)} images over {512} workgroups")
for w in range(4):
    m = st[:, w, :4].sum(axis=0) / n
    print(f"  {names[w]:3s} barrierA {m[0]:7.0f}  compute {m[1]:7.0f}  barrierB {m[2]:7.0f}  stage {m[3]:7.0f}")
