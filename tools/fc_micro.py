"""Microbenchmark: weights-resident FC kernel (mcc.ops.linear) vs torch/hipBLASLt."""
import sys
import time

import torch

sys.path.insert(0, ".")
import mpi_cuda_cnn_amd.ops as ops  # noqa: E402


def bench(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000.0  # us


dev = torch.device("cuda")
for (M, N, K) in [(16384, 120, 400), (16384, 84, 120), (16384, 400, 120), (4096, 120, 400), (65536, 120, 400),
                  (16384, 10, 84)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16) * 0.05
    b = torch.randn(N, device=dev)
    t_mcc = bench(lambda: ops.linear(x, w, b, "relu"))
    t_torch = bench(lambda: torch.relu(torch.nn.functional.linear(x, w, b.to(torch.bfloat16))))
    t_mm = bench(lambda: x @ w.t())
    gb = (M * K * 2 + M * N * 2) / 1e9
    print(f"M={M:6d} N={N:4d} K={K:4d}  mcc {t_mcc:7.1f} us  torch(linear+relu) {t_torch:7.1f} us  "
          f"torch mm {t_mm:7.1f} us   bytes-roofline@5TB/s {gb / 5e12 * 1e15:6.1f} us")
