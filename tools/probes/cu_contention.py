"""CU-contention probe for the persistent LeNet-5 kernels (VERDICT r3, next
round item 3b).

At world > 1 an RCCL kernel that waits for its peers holds CUs (and LDS)
while the step's compute kernels run.  lenet_fwd / lenet_bwd split the batch
statically over a grid sized to fill every SIMD, so a workgroup that cannot
become resident delays the whole kernel.  This probe reproduces that on one
GPU: `kernels.cu_hold` launches `nwg` workgroups that each hold `lds` bytes of
LDS and spin for `usec` on a high-priority stream, released by an event at
the point where the collective would be issued, and reports the step time
against an undisturbed step.

    python tools/probes/cu_contention.py [--batch 163840] [--steps 20]

Output: one line per configuration (mean ms/step over `steps`, delta vs the
undisturbed step).  profiles/cu_contention_r4.txt holds a run.
"""

from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpi_cuda_cnn_amd as mcc  # noqa: E402
from mpi_cuda_cnn_amd import _C  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=163840)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--model", default="lenet5")
    ap.add_argument("--reserve-sweep", action="store_true",
                    help="sweep MCC_AB=bwd_reserve_cus over 0/2/4/8 with holds during the backward")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    spec = mcc.make_model(a.model)
    C, H, W = spec.input_shape()
    n = 60000
    imgs, labels = mcc.synth_dataset(n, C, H, W, 10, seed=1)
    d_img = torch.from_numpy(imgs).to(dev)
    d_lab = torch.from_numpy(labels).to(dev)
    idx = torch.randint(0, n, (a.batch,), dtype=torch.int32, device=dev)
    B = a.batch
    net = _C.GpuNet(spec, "bf16", B)
    net.set_params(np.asarray(_C.init_params(spec, 0, "glibc"), dtype=np.float32))
    main_s = torch.cuda.current_stream(dev)
    hog = torch.cuda.Stream(dev, priority=-1)
    ev = torch.cuda.Event()
    s = main_s.cuda_stream

    def step(cfg):
        where, nwg, lds, us = cfg if cfg else (None, 0, 0, 0.0)
        if where == "fwd":
            main_s.record_event(ev)
            hog.wait_event(ev)
            _C.kernels.cu_hold(nwg, lds, us, hog.cuda_stream)
        net.forward(d_img.data_ptr(), idx.data_ptr(), B, s)
        net.loss(d_lab.data_ptr(), idx.data_ptr(), 1.0 / B, True, s)
        if where == "bwd":  # the FC gradient is complete here: where a bucket's all-reduce would start
            main_s.record_event(ev)
            hog.wait_event(ev)
            _C.kernels.cu_hold(nwg, lds, us, hog.cuda_stream)
        net.backward_all(s)
        net.sgd(0.01, 0.0, 0.0, s)
        main_s.wait_stream(hog)

    def timed(cfg):
        for _ in range(3):
            step(cfg)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(main_s)
        for _ in range(a.steps):
            step(cfg)
        t1.record(main_s)
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) / a.steps

    # hold-kernel sanity: its own duration with nothing else running
    for us in (20.0, 50.0):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        _C.kernels.cu_hold(32, 40960, us, s)
        e1.record(main_s)
        torch.cuda.synchronize()
        print(f"cu_hold alone: 32 WG x 40 KB, {us:.0f} us requested -> {e0.elapsed_time(e1) * 1e3:.1f} us", flush=True)

    if a.reserve_sweep:
        # round 5: the FC bucket's all-reduce is issued before lenet_bwd; a
        # backward grid that leaves k CUs free keeps a peer-waiting RCCL
        # kernel off the static partition.  Per k: undisturbed step, holds
        # during the backward.
        for k in (0, 2, 4, 8):
            os.environ["MCC_AB"] = f"bwd_reserve_cus={k}"
            base = min(timed(None) for _ in range(3))
            line = f"reserve {k} CUs: undisturbed {base:.4f} ms"
            for nwg, us in ((4, 20.0), (4, 50.0), (16, 50.0)):
                t = timed(("bwd", nwg, 40960, us))
                line += f" | hold {nwg:2d} WG x {us:.0f} us {t:.4f} ({(t - base) * 1e3:+.1f} us)"
            print(line, flush=True)
        os.environ.pop("MCC_AB", None)
        return 0
    base = [timed(None) for _ in range(2)]
    ref = min(base)
    print(f"model {a.model} batch {B}: undisturbed step {base[0]:.4f} / {base[1]:.4f} ms", flush=True)
    cfgs = [(w, nwg, lds, us) for w in ("bwd", "fwd") for nwg in (16, 32) for lds, us in ((40960, 20.0), (40960, 50.0))]
    cfgs.append(("bwd", 32, 4096, 50.0))
    for cfg in cfgs:
        t = timed(cfg)
        w, nwg, lds, us = cfg
        print(
            f"hold during {w:3s}: {nwg:2d} WG x {lds // 1024:2d} KB LDS x {us:4.0f} us -> {t:.4f} ms/step "
            f"({(t - ref) * 1e3:+7.1f} us, {100 * (t - ref) / ref:+5.2f}%)",
            flush=True,
        )
    again = timed(None)
    print(f"undisturbed again: {again:.4f} ms", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
