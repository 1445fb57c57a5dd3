#!/usr/bin/env python3
"""Time the LeNet-5 step's three parts (forward() = lenet_fwd, loss() = the
fused FC chain, backward_all() = lenet_bwd) with HIP events, for the
in-tree module or ablation builds (tools/build_variant.sh); PROBE_MODEL picks
another model (e.g. ref: fwd = ref_fwd, bwd = FC backward + ref_bwd), PROBE_DTYPE
the compute dtype (bf16 default, fp32):

    python tools/probes/lenet_phase_probe.py [variant_dir ...]

Each variant runs in its own subprocess (a module is loaded once per process)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_one(path):
    sys.path.insert(0, path)
    import numpy as np
    import torch

    import mpi_cuda_cnn_amd as mcc

    assert os.path.dirname(mcc.__file__).startswith(os.path.abspath(path)), mcc.__file__
    B = int(os.environ.get("PROBE_B", "163840"))
    spec = mcc.make_model(os.environ.get("PROBE_MODEL", "lenet5"))
    C, H, W = spec.input_shape()
    ndata = min(65536, max(B, 1024))
    imgs, labels = mcc.synth_dataset(ndata, C, H, W, spec.num_classes(), seed=1)
    dev = torch.device("cuda", 0)
    d_img, d_lab = torch.from_numpy(imgs).to(dev), torch.from_numpy(labels).to(dev)
    idx = torch.randint(0, ndata, (B,), dtype=torch.int32, device=dev)
    net = mcc.GpuNet(spec, os.environ.get("PROBE_DTYPE", "bf16"), B)
    net.set_params(mcc.init_params(spec, seed=0, mode="fast").astype(np.float32))
    s = torch.cuda.current_stream().cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    acc = np.zeros(3)
    n = 10
    for it in range(n + 3):
        ev[0].record()
        net.forward(d_img.data_ptr(), idx.data_ptr(), B, s)
        ev[1].record()
        net.loss(d_lab.data_ptr(), idx.data_ptr(), 1.0 / B, True, s)
        ev[2].record()
        net.backward_all(s)
        ev[3].record()
        torch.cuda.synchronize()
        if it >= 3:
            acc += [ev[i].elapsed_time(ev[i + 1]) for i in range(3)]
    acc /= n
    print(f"{os.path.basename(path.rstrip('/')) or 'tree'}: fwd {acc[0]*1e3:.1f} us  loss+fc {acc[1]*1e3:.1f} us  "
          f"bwd {acc[2]*1e3:.1f} us  total {acc.sum()*1e3:.1f} us", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        run_one(sys.argv[2])
        sys.exit(0)
    paths = sys.argv[1:] or [ROOT]
    for p in [ROOT] + [x for x in paths if x != ROOT]:
        r = subprocess.run([sys.executable, __file__, "--one", p], timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)
