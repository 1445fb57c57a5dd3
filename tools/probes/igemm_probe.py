#!/usr/bin/env python3
"""Time the 256-tile implicit-GEMM kernels (igemm.hip: igemm_big_kernel
forward / pooled forward / data gradient, igemm_dwbig_kernel weight gradient)
on VGG-11 layer shapes, for the in-tree module and ablation builds
(tools/build_variant.sh with SRC=csrc/kernels/igemm.hip), in interleaved rounds
(one subprocess per variant per round: a module is loaded once per process):

    python tools/probes/igemm_probe.py [rounds] [variant_dir ...]

Prints per variant and op the median / min time (us) and TFLOP/s over rounds."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# B, H, W, C, O, KS: VGG-11 conv4 (56x56x256, 3x3) and conv6 (28x28x512) at the
# B = 640 bench batch (whole 256-pixel-tile rounds: a 64-image slice leaves a
# 2 % fourth round at 56x56), and a 1x1 "conv" of the same K = 2304 (a plain
# GEMM through the same kernel: no im2col bounds); PROBE_SHAPES="0,2" picks
SHAPES = [(640, 56, 56, 256, 256, 3), (640, 28, 28, 512, 512, 3), (640, 28, 28, 2304, 256, 1)]
SHAPES = [SHAPES[int(i)] for i in os.environ.get("PROBE_SHAPES", "0,1,2").split(",")]
OPS = os.environ.get("PROBE_OPS", "fwd,fwd_pool,dgrad,wgrad").split(",")


def run_one(path):
    sys.path.insert(0, path)
    import torch

    import mpi_cuda_cnn_amd as mcc
    from mpi_cuda_cnn_amd import ops

    assert os.path.dirname(mcc.__file__).startswith(os.path.abspath(path)), mcc.__file__
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for B, H, W, C, O, KS in SHAPES:
        pd = KS // 2
        x = (torch.rand(B, H, W, C, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.randn(O, C, KS, KS, generator=g, device=dev) * (2.0 / (KS * KS * C)) ** 0.5).to(torch.bfloat16)
        b = torch.randn(O, generator=g, device=dev) * 0.1
        dy = (torch.rand(B, H, W, O, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        flop = 2.0 * B * H * W * C * O * KS * KS
        ops_ = {
            "fwd": lambda: ops.conv2d_nhwc(x, w, b, stride=1, pad=pd, act="relu"),
            "fwd_pool": lambda: ops.conv2d_nhwc(x, w, b, stride=1, pad=pd, act="relu", pool=True),
            "dgrad": lambda: ops.conv2d_dgrad_nhwc(dy, w, pad=pd),
            "wgrad": lambda: ops.conv2d_wgrad_nhwc(dy, x, KS, stride=1, pad=pd),
        }
        for name in OPS:
            if KS == 1 and name == "dgrad" and O % 64:
                continue
            fn = ops_[name]
            for _ in range(3):
                fn()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            n = 10
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(n):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            us = ev[0].elapsed_time(ev[1]) * 1e3 / n
            res[f"{name}_{H}x{C}k{KS}"] = (us, flop / us * 1e-6)
        del x, w, dy
    print("RESULT " + json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        run_one(sys.argv[2])
        sys.exit(0)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    paths = [ROOT] + [p for p in sys.argv[2:] if p != ROOT]
    acc = {p: {} for p in paths}
    for r in range(rounds):
        for p in paths:
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", p], capture_output=True,
                                 text=True, timeout=300)
            if out.returncode != 0:
                print(out.stdout[-2000:], out.stderr[-3000:])
                sys.exit(out.returncode)
            line = next(l for l in out.stdout.splitlines() if l.startswith("RESULT "))
            for k, v in json.loads(line[7:]).items():
                acc[p].setdefault(k, []).append(v[0])
        print(f"round {r + 1}/{rounds} done", flush=True)
    for p in paths:
        name = os.path.basename(p.rstrip("/")) if p != ROOT else "tree"
        for k, v in acc[p].items():
            v = sorted(v)
            B, H, W, C, O, KS = next(s for s in SHAPES if k.endswith(f"_{s[1]}x{s[3]}k{s[5]}"))
            flop = 2.0 * B * H * W * C * O * KS * KS
            print(f"{name:>14} {k:>18}: median {v[len(v) // 2]:8.1f} us  min {v[0]:8.1f} us  "
                  f"{flop / v[0] * 1e-6:7.1f} TF/s")
