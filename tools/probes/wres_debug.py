"""Error structure of fc_wres (fp32, tanh) against fp64: which rows / columns are off."""
import torch
from mpi_cuda_cnn_amd import _C
K_ = _C.kernels
cuda = torch.device("cuda:0")
s = torch.cuda.current_stream().cuda_stream
for (M, N, K, act) in [(777, 200, 200, 2), (777, 200, 200, 1), (777, 200, 200, 0), (256, 112, 200, 2), (777, 400, 120, 2), (777, 120, 84, 2)]:
    g = torch.Generator().manual_seed(1)
    a = torch.randn(M, K, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / K**0.5).to(cuda)
    y = torch.tanh(torch.randn(M, N, generator=g)).to(cuda)
    out = torch.full((M, N), 7.0, device=cuda)
    K_.fc_wres(M, N, K, a.data_ptr(), K, w.data_ptr(), K, act, y.data_ptr(), N, out.data_ptr(), N, s, f32=True)
    torch.cuda.synchronize()
    ref = a.double() @ w.double().t()
    if act == 2: ref = ref * (1 - y.double() ** 2)
    if act == 1: ref = ref * (y.double() > 0)
    e = (out.double() - ref).abs()
    bad = e > 1e-4 * ref.abs().max()
    print(M, N, K, act, "bad", int(bad.sum()), "of", M * N)
    if bad.any():
        r = bad.any(1).nonzero().flatten()
        c = bad.any(0).nonzero().flatten()
        print("  rows", r[:20].tolist(), "... n", len(r), " cols", c[:40].tolist(), "n", len(c))
        i, j = int(r[0]), int(c[0])
        print("  sample out/ref/plain", float(out[i, j]), float(ref[i, j]), float((a.double() @ w.double().t())[i, j]), float(y[i, j]))
