"""hipBLASLt (torch.matmul, bf16) on the FC GEMM shapes of the bench models,
to price the engine's own FC / GEMM kernels against the vendor library.

    python tools/probes/blas_fc_shapes.py
"""
import torch

dev = torch.device("cuda", 0)
torch.backends.cuda.matmul.allow_bf16_reduced_precision_reduction = False
SHAPES = [  # (name, M, N, K): C[M,N] = A[M,K] @ B[K,N]
    ("ref fc1 fwd", 65536, 200, 1568),
    ("ref fc1 dX", 65536, 1568, 200),
    ("ref fc1 dW", 200, 1568, 65536),
    ("ref fc2 fwd", 65536, 200, 200),
    ("lenet fc1 fwd", 131072, 120, 400),
    ("lenet fc1 dX", 131072, 400, 120),
    ("lenet fc1 dW", 120, 400, 131072),
    ("lenet fc2 fwd", 131072, 84, 120),
    ("cifar fc1 fwd", 32768, 256, 2048),
    ("vgg fc1 fwd", 640, 4096, 25088),
]


def bench(f, it=30):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1000.0


for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    bt = b.t().contiguous()
    us = bench(lambda: torch.matmul(a, b))
    us_t = bench(lambda: torch.matmul(a, bt.t()))
    tf = 2.0 * M * N * K / (min(us, us_t) * 1e-6) / 1e12
    gb = (M * K + K * N + M * N) * 2 / 1e9
    print(f"{name:<16} M={M:>6} N={N:>5} K={K:>6}: {us:8.1f} us (B^T {us_t:8.1f} us)  {tf:7.1f} TF/s  "
          f"mem floor {gb / 8.0 * 1e3:6.1f} us")
