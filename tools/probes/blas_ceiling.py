#!/usr/bin/env python3
"""Library ceiling for the VGG-11 conv GEMM shapes: hipBLASLt (torch.matmul,
bf16) TFLOP/s on the implicit-GEMM problem sizes of each layer at B=128, for
comparison with igemm_conv / igemm_dw (not on the training path)."""
import torch

B = 128
layers = [(112, 64, 128), (56, 128, 256), (56, 256, 256), (28, 256, 512), (28, 512, 512), (14, 512, 512), (14, 512, 512)]
dev = torch.device("cuda")
for HW, C, O in layers:
    M, N, K = B * HW * HW, O, 9 * C
    for name, (m, n, k) in {"fwd": (M, N, K), "dw": (N, K, M)}.items():
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        b = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(a, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            torch.matmul(a, b)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{name} HW={HW} C={C} O={O}  M={m} N={n} K={k}: {ms*1e3:8.1f} us  {2*m*n*k/ms/1e9:7.1f} TFLOP/s", flush=True)
        del a, b
