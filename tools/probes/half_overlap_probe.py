"""Would two half-batch steps on two streams overlap?  (LeNet-5 bf16)

Times, on one GPU:
  full   one GpuNet at B, one stream                        (the bench step)
  seq    two GpuNets at B/2, one after the other on one stream
  conc   the same two, B's step on a second stream, started after A's forward
         (staggered: A's FC chain / backward against B's conv kernels)
Prints ms per (pair of half) steps.  No correctness: the two nets train
independently; this only bounds what a two-stream half-batch pipeline could
gain from co-running latency-bound and LDS-bound kernels.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
import mpi_cuda_cnn_amd as mcc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 163840
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
spec = mcc.make_model("lenet5")
N = 65536
imgs, labels = mcc.synth_dataset(N, 1, 28, 28, 10, seed=3)
params = mcc.init_params(spec, seed=1).astype(np.float32)
d_img = torch.from_numpy(imgs).cuda()
d_lab = torch.from_numpy(labels).cuda()
g = torch.Generator(device="cuda").manual_seed(5)


def make(b):
    n = mcc.GpuNet(spec, "bf16", b)
    n.set_params(params)
    idx = torch.randint(0, N, (b,), device="cuda", dtype=torch.int32, generator=g)
    return n, idx


def fwd(n, idx, b, s):
    n.forward(d_img.data_ptr(), idx.data_ptr(), b, s)


def rest(n, idx, b, s):
    n.loss(d_lab.data_ptr(), idx.data_ptr(), 1.0 / b, True, s)
    n.backward_all(s)
    n.sgd(0.01, 0.0, 0.0, s)


def timeit(fn, k):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3 / k


full, fidx = make(B)
s0 = torch.cuda.current_stream()
sB = torch.cuda.Stream()
h = B // 2
a, aidx = make(h)
b, bidx = make(h)
ev = torch.cuda.Event()


def step_full():
    fwd(full, fidx, B, s0.cuda_stream)
    rest(full, fidx, B, s0.cuda_stream)


def step_seq():
    for n, i in ((a, aidx), (b, bidx)):
        fwd(n, i, h, s0.cuda_stream)
        rest(n, i, h, s0.cuda_stream)


def step_conc():
    fwd(a, aidx, h, s0.cuda_stream)
    ev.record(s0)
    rest(a, aidx, h, s0.cuda_stream)
    sB.wait_event(ev)
    fwd(b, bidx, h, sB.cuda_stream)
    rest(b, bidx, h, sB.cuda_stream)
    s0.wait_stream(sB)


for rep in range(2):
    print(f"rep {rep}: full {timeit(step_full, steps):.3f} ms   seq {timeit(step_seq, steps):.3f} ms   "
          f"conc {timeit(step_conc, steps):.3f} ms", flush=True)
