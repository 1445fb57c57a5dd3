#!/usr/bin/env python3
"""Per-step time of the graph-replayed LeNet-5 bench step over the first N
steps after capture (HIP events around each replay), to tell a warm-up that
follows the step count (training state) from one that follows wall time
(clocks): PROBE_SLEEP_MS inserts an idle gap after capture.

    python tools/probes/step_warmup_probe.py [lr]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import mpi_cuda_cnn_amd as mcc  # noqa: E402
from mpi_cuda_cnn_amd.trainer import GpuTrainer, capture_step  # noqa: E402


def main():
    lr = float(sys.argv[1]) if len(sys.argv) > 1 else 0.1
    B = 163840
    dev = torch.device("cuda", 0)
    spec = mcc.make_model("lenet5")
    imgs, labels = mcc.synth_dataset(65536, 1, 28, 28, 10, seed=1)
    d_img, d_lab = torch.from_numpy(imgs).to(dev), torch.from_numpy(labels).to(dev)
    tr = GpuTrainer(spec, dtype="bf16", batch=B, device=0, seed=0, lr=lr, momentum=0.0, init="fast")
    K = mcc._C.kernels
    idx = torch.empty(B, dtype=torch.int32, device=dev)
    counter = torch.zeros(1, dtype=torch.int64, device=dev)

    def step():
        s = torch.cuda.current_stream(dev).cuda_stream
        K.sample_indices(idx.data_ptr(), B, 0, 65536, 0x5EED0000, counter.data_ptr(), s)
        tr.step(d_img, d_lab, idx)
        K.advance_counter(counter.data_ptr(), s)

    step()
    torch.cuda.synchronize()
    g, why = capture_step(step)
    assert g is not None, why
    time.sleep(float(os.environ.get("PROBE_SLEEP_MS", "0")) / 1000)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(41)]
    ev[0].record()
    for i in range(40):
        g.replay()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(40)]
    print(f"lr {lr} sleep {os.environ.get('PROBE_SLEEP_MS', '0')} ms: per-step us " + " ".join(f"{t:.0f}" for t in ts))


if __name__ == "__main__":
    main()
