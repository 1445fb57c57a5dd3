"""Phase timestamps (100 MHz realtime clock) of the weights-resident FC kernel."""
import sys

import torch

sys.path.insert(0, ".")
import mpi_cuda_cnn_amd as mcc  # noqa: E402

K_ = mcc._C.kernels
dev = torch.device("cuda")
for (M, N, K, ab) in [(16384, 120, 400, 0), (16384, 400, 120, 0), (16384, 84, 120, 0), (16384, 400, 120, 1),
                      (16384, 400, 120, 2), (16384, 400, 120, 3), (4096, 400, 120, 0)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    ldc = (N + 7) // 8 * 8
    y = torch.empty(M, ldc, device=dev, dtype=torch.bfloat16)
    grid = (M + 63) // 64
    dbg = torch.zeros(grid * 16, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for it in range(3):
        K_.fc(M, N, K, x.data_ptr(), K, w.data_ptr(), K, epi=K_.EPI_BIAS_ACT, act=K_.ACT_RELU, bias=b.data_ptr(),
              C=y.data_ptr(), ldc=ldc, dbg=dbg.data_ptr(), ablate=ab, stream=s)
    torch.cuda.synchronize()
    t = dbg.view(grid, 4, 4).double() * 10.0 / 1000.0  # us (100 MHz clock)
    t0 = t[:, :, 0].min()
    start = t[:, :, 0] - t0
    copy = t[:, :, 1] - t[:, :, 0]
    bar = t[:, :, 2] - t[:, :, 1]
    comp = t[:, :, 3] - t[:, :, 2]
    span = t[:, :, 3].max() - t0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for it in range(20):
        K_.fc(M, N, K, x.data_ptr(), K, w.data_ptr(), K, epi=K_.EPI_BIAS_ACT, act=K_.ACT_RELU, bias=b.data_ptr(),
              C=y.data_ptr(), ldc=ldc, ablate=ab, stream=s)
    e1.record()
    torch.cuda.synchronize()
    print(f"ablate={ab} event-avg {e0.elapsed_time(e1) / 20 * 1000:.2f} us  ", end="")
    print(f"M={M} N={N} K={K}: span {span:.2f} us | start skew max {start.max():.2f} | W+A load mean {copy.mean():.2f} "
          f"max {copy.max():.2f} | barrier wait mean {bar.mean():.2f} | compute+store mean {comp.mean():.2f} max {comp.max():.2f}")
