#!/usr/bin/env python3
"""Headline benchmark: LeNet-5 training throughput on MNIST-shaped data.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch-per-gpu B]
    torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)

Metric (BASELINE.json): images/sec for the whole node, LeNet-5, 28x28x1
input, synchronous data-parallel SGD over RCCL (weak scaling: fixed per-GPU
batch).  Synthetic data of the MNIST shape, random-init weights; every step
does the full work: device-side sampling, forward, softmax-CE, backward, the
bucketed gradient all-reduce and the SGD update.  The timed region is K
steps bracketed by barrier + device synchronize on both sides; the reported
time is the max over ranks.

At N = 1 the same run also times LeNet-5 in fp32 (BASELINE.json config 2,
"LeNet-5 fp32 on one MI355X") as a second region with the same K / W and
reports it under "fp32" in the one JSON line.  The optimizer defaults to the
reference's plain SGD at lr 0.1 (cnn.c:303-314, 446).
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_IMG_S = 2510.0  # best reference number (8-rank MPI CPU)
METRIC = "images/sec (whole node), LeNet-5 MNIST-shaped, at 1/2/4/8 MI355X"
# Per-GPU batch sized for 288 GB HBM3E: LeNet-5 throughput keeps rising with
# batch as the persistent conv kernels' per-step prologue/tail and the launch
# chain amortise (round 1: 36.7 M img/s at 16,384 -> 45.3 M at 65,536 -> 47.3 M
# at 131,072, profiles/lenet5_batch_sweep_r1g.txt; round 2 kernels: 59.1 M at
# 65,536 -> 64.9 M at 131,072, profiles/batch_sweep_r2.txt; round 3 fused
# conv-block kernels: 109.3 M at 131,072, 111.2 M at 155,648, 112.6-113.2 M at
# 163,840, 111.9-112.1 M at 167,936 / 170,496, profiles/batch_sweep_r3.txt).
# The engine's 32-bit activation-index bound is B * 16 padded channels * 28 *
# 28 < 2^31 (B < 171,196).
# CIFAR-3conv: 1.88 M img/s at 4,096 -> 2.58 M at 16,384 (profiles/bench_models_r1g.jsonl);
# round 2: 3.64 M at 16,384 -> 3.91 M at 32,768 (65,536 exceeds the 32-bit bound);
# round 3: 5.47 M at 32,768, 5.57-5.59 M at 49,152, 5.59 M at 57,344, 5.61 M at
# 61,440, 5.64 M at 65,000 -> 65,024 (just under the B * 32 * 32 * 32 < 2^31 bound).
# reference CNN, round 3 fused block: 50.6 M at 65,536, 55.7 M at 131,072, 56.3 M at
# 163,840 (profiles/batch_sweep_r3.txt).
# VGG-11: 15.0 k img/s at 256 -> 15.7 k at 512 -> 16.26 k at 640 (640 x 64 x 224^2 is 95.7 % of the
# 32-bit activation bound; the 224^2 x 64 pre-pool conv1 tensor is never materialised).
DEFAULT_BATCH = {"lenet5": 163840, "ref": 163840, "cifar3": 65024, "vgg11": 640}
# models whose step is faster with the dW side stream (engine.cpp, measured A/B): none with the
# round-2 kernels (CIFAR-3conv at 32768: 4.38 M img/s without, 4.27 M with; LeNet-5 / VGG-11 / ref
# also faster without, profiles/side_stream_ab_r2.txt)
SIDE_STREAM: set = set()


def metric_for(model):
    # the BASELINE.json metric is defined on LeNet-5; other models report the
    # same quantity under their own name and without a baseline ratio
    return METRIC if model == "lenet5" else f"images/sec (whole node), {model}, at 1/2/4/8 MI355X"


def timed_run(args, spec, dtype, B, d_img, d_lab, dev, dev_idx, rank, world, multi, eager_anchor=False):
    """Build a trainer, warm up, time exactly args.steps steps between
    barrier + device synchronize on both sides (max over ranks), free it."""
    import torch
    import torch.distributed as dist

    import mpi_cuda_cnn_amd as mcc
    from mpi_cuda_cnn_amd.trainer import GpuTrainer

    tr = GpuTrainer(
        spec,
        dtype=dtype,
        batch=B,
        device=dev_idx,
        seed=0,
        lr=args.lr,
        momentum=args.momentum,
        init="fast",
        bucket_bytes=int(args.bucket_mb * (1 << 20)),
        force_reduce=args.force_reduce,
    )
    # device minibatch sampler (rand() % N semantics, cnn.c:455): indices and
    # its step counter live on the GPU, so a graph replay draws a fresh batch
    K = mcc._C.kernels
    idx_buf = torch.empty(B, dtype=torch.int32, device=dev)
    counter = torch.zeros(2, dtype=torch.int64, device=dev)  # (step, ticket of the fused sampler)
    seed = 0x5EED0000 + rank

    def step_launch():
        s = torch.cuda.current_stream(dev).cuda_stream
        # indices of this step + the counter advance in one launch
        K.sample_indices_advance(idx_buf.data_ptr(), B, 0, args.dataset, seed, counter.data_ptr(), s)
        tr.step(d_img, d_lab, idx_buf)

    # host-side rank agreement (capture consensus, the barriers around the
    # timed loop, the MAX of the per-rank times) only where there are ranks
    # to agree with: at world 1 a barrier / MAX is the identity, and no eager
    # collective then follows the graph capture (see ddp.init_process_group)
    step = step_launch
    graph_note = "per-kernel launches" + (" (--graph off)" if args.graph == "off" else "")
    coll_graph = None
    g = None
    tr.zero_stats()
    step_launch()  # eager first: code objects loaded, RCCL communicator warmed up
    torch.cuda.synchronize()
    if args.graph == "on" or (args.graph == "auto" and world == 1):
        from mpi_cuda_cnn_amd.trainer import capture_step

        issued_before = tr.sync.issued
        g, why = capture_step(step_launch)
        ok = torch.tensor([1 if g is not None else 0], device=dev, dtype=torch.int32)
        if multi:  # every rank replays or none does (collectives inside)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 1:
            coll_graph = tr.sync.issued - issued_before
            step = g.replay
            graph_note = "hip graph: whole step captured once (torch.cuda.CUDAGraph), replayed per step"
        else:
            if args.graph == "on":
                raise RuntimeError(f"--graph on: capture failed: {why}")
            graph_note = f"off (capture failed: {why})"
    def timed(fn, warmup, counted):
        """`warmup` untimed calls, then exactly args.steps timed ones bracketed
        by barrier + device synchronize on both sides; returns (seconds, MAX
        over ranks; collectives issued per timed step, from the host counter
        when `counted`)"""
        for _ in range(max(0, warmup)):
            fn()
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
        torch.cuda.synchronize()
        tr.zero_stats()
        issued0 = tr.sync.issued
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        per = (tr.sync.issued - issued0) / max(1, args.steps) if counted else None
        if multi:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, per

    # (the eager first step above is warmup step 1 of the headline region)
    elapsed, per = timed(step, args.warmup - 1, coll_graph is None)
    coll_per_step = per if coll_graph is None else coll_graph
    st = tr.net.get_stats()
    # Same-path anchor for the N > 1 points, which run per-kernel launches: at
    # N = 1 the same trainer is timed again with eager launches, same K / W,
    # AFTER the headline region (whose warmup is therefore unchanged)
    eager = None
    if eager_anchor and step is not step_launch:
        e_el, _ = timed(step_launch, args.warmup, True)
        eager = {"value": round(B * world * args.steps / e_el, 1), "ms_per_step": round(1000.0 * e_el / args.steps, 4),
                 "steps": args.steps, "warmup": args.warmup,
                 "train_loss_mean": round(tr.net.get_stats()["loss_sum"] / (B * args.steps), 4),
                 "launch": "per-kernel launches (the N > 1 launch mode, --graph off semantics), same trainer, "
                           "timed after the graph region"}
    nb = len(tr.sync.buckets)
    res = {
        "elapsed": elapsed,
        "eager": eager,
        "loss_key": "train_loss_mean",  # mean over the K timed steps
        "loss": round(st["loss_sum"] / (B * args.steps), 4),
        "launch": graph_note,
        "optimizer": ("sgd lr={} (plain SGD, the reference's Layer_update, cnn.c:303-314)".format(args.lr)
                      if args.momentum == 0 else f"sgd lr={args.lr} momentum={args.momentum}"),
        "allreduce": (f"{'rccl' if args.dist_backend == 'nccl' else 'gloo (rehearsal)'}: {coll_per_step:g} "
                      f"all-reduce(s)/step over {nb} bucket(s) <= {args.bucket_mb} MiB, async on RCCL's stream, "
                      "joined before its SGD"
                      + ("; at one rank RCCL elides the in-place SUM: no reduction kernel runs"
                         " (--force-reduce runs one)" if tr.sync.elided else "")
                      + ("; forced one-rank reduction kernel (AVG)" if args.force_reduce and world == 1 else "")
                      + ("; SGD split per bucket: each bucket's update joins only its own all-reduce"
                         if tr.split_sgd and nb > 1 else "")
                      if coll_per_step else "none (--no-dist)"),
    }
    del step, g, tr
    torch.cuda.synchronize()
    return res


def timed_run64(args, spec, B, d_img, d_lab, dev):
    """The reference precision (fp64 throughout, cnn.c:22-30) on the GPU:
    GpuNet64 (v_mfma_f64_16x16x4_f64 GEMMs, f64.hip) with a device-resident
    batch (u8 gather by the device sampler's indices, /255 in fp64), forward,
    softmax-CE, backward and SGD per step; no collectives (one GPU)."""
    import torch

    import mpi_cuda_cnn_amd as mcc

    net = mcc._C.GpuNet64(spec, False, B)
    net.set_params(mcc.init_params(spec, seed=0, mode="fast").astype("float64"))
    K = mcc._C.kernels
    idx_buf = torch.empty(B, dtype=torch.int32, device=dev)
    counter = torch.zeros(1, dtype=torch.int64, device=dev)
    s = net.stream  # GpuNet64's own stream: the sampler runs there too

    def step():
        K.sample_indices(idx_buf.data_ptr(), B, 0, args.dataset, 0x5EED0000, counter.data_ptr(), s)
        net.forward_u8(d_img.data_ptr(), d_lab.data_ptr(), idx_buf.data_ptr(), B)
        net.backward_device(1.0 / B)
        net.sgd(args.lr)
        K.advance_counter(counter.data_ptr(), s)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    loss = net.loss_sum() / B
    del net
    return {
        "elapsed": elapsed,
        "loss_key": "train_loss_last",  # the last timed step's mean loss (read once: no per-step host sync)
        "loss": round(loss, 4),
        "launch": "per-kernel launches on GpuNet64's stream (fp64 GEMMs on v_mfma_f64_16x16x4_f64)",
        "optimizer": f"sgd lr={args.lr} (plain SGD, the reference's Layer_update, cnn.c:303-314)",
        "allreduce": "none (fp64 reference-precision path: one GPU)",
    }


def _self_launch(n: int) -> int:
    """Run this script under torch.distributed.run with n ranks on this node
    (rendezvous on 127.0.0.1, a free port) as a child process; rank 0's JSON
    line reaches our stdout directly.  Returns the launcher's exit code."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1")).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="lenet5")
    ap.add_argument("--batch-per-gpu", type=int, default=0, help="default: per-model (163840 for LeNet-5)")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--dataset", type=int, default=0,
                    help="synthetic samples resident per GPU (default 65536; 8 batches for large images)")
    ap.add_argument("--bucket-mb", type=float, default=4.0)
    # the reference's optimizer: plain SGD at lr 0.1 (cnn.c:303-314,446)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--momentum", type=float, default=0.0)
    ap.add_argument("--fp32-extra", choices=["auto", "on", "off"], default="auto",
                    help="also time LeNet-5 fp32 (BASELINE config 2) in the same run and report it under "
                         "\"fp32\" in the JSON line; auto = on at N=1 for a bf16 LeNet-5 run")
    ap.add_argument("--eager-anchor", choices=["auto", "on", "off"], default="auto",
                    help="also time the headline trainer with per-kernel launches (the launch mode of the N > 1 "
                         "points) after the graph region and report it under \"eager\"; auto = on at N=1")
    ap.add_argument("--no-dist", action="store_true",
                    help="N=1 only: no process group, no collectives (A/B against the RCCL path)")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="replay the whole step (sampler, fwd, loss, bwd, bucketed RCCL all-reduce, SGD) "
                         "from a HIP graph; auto = on at N=1 (bit-equal to eager: tests/test_gpu_rccl.py) "
                         "with a fallback to per-kernel launches if capture fails, off at N>1 (multi-rank "
                         "capture of the collectives is not verifiable on a one-GPU box)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl (= RCCL, the measured path) or gloo: a rehearsal of the multi-rank bench logic "
                         "with more ranks than GPUs (ranks share GPUs round-robin; not a performance number)")
    ap.add_argument("--force-reduce", action="store_true",
                    help="N=1: make each bucket's collective a real RCCL reduction kernel (AVG; bit-identical "
                         "result) instead of the in-place SUM RCCL elides at one rank -- measures comm/compute "
                         "contention (profiles/comm_contention_r3.txt)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start one rank per GPU
        # as CHILD processes (before this process touches the GPU) and relay
        # their result -- never silently measure one rank for an N-GPU request
        return _self_launch(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: the JSON line would not describe "
                         "the requested run")

    # Native libraries write banners to stdout (RCCL prints its version block
    # at communicator init): route fd 1 to stderr for the run and keep a
    # duplicate of the real stdout for the one JSON line.
    json_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()  # (counting does not initialise the GPU)
    if args.dist_backend == "nccl" and world > ndev:
        raise SystemExit(f"bench: {world} ranks but {ndev} GPU(s): RCCL needs one GPU per rank (--dist-backend gloo "
                         "rehearses more ranks than GPUs)")
    dev_idx = local_rank % max(1, ndev)
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    if (world > 1 or not args.no_dist) and args.dtype != "fp64":
        # RCCL process group at every N, 1 included: the N=1 step runs the
        # same broadcast + bucketed all-reduce on RCCL's stream as N=8
        from mpi_cuda_cnn_amd.parallel.ddp import init_process_group

        init_process_group(args.dist_backend, dev)

    import mpi_cuda_cnn_amd as mcc

    spec = mcc.make_model(args.model)
    C, H, W = spec.input_shape()
    if args.model in SIDE_STREAM:
        ab = os.environ.get("MCC_AB", "")
        os.environ["MCC_AB"] = ",".join(x for x in (ab, "side_stream") if x)
    B = args.batch_per_gpu or (16384 if args.dtype == "fp64" else DEFAULT_BATCH.get(args.model, 1024))
    if not args.dataset:
        args.dataset = max(65536, B) if H * W <= 32 * 32 else max(256, 8 * B)
    imgs, labels = mcc.synth_dataset(args.dataset, C, H, W, spec.num_classes(), seed=1234 + rank)
    d_img = torch.from_numpy(imgs).to(dev)
    d_lab = torch.from_numpy(labels).to(dev)
    multi = dist.is_initialized() and world > 1

    if args.dtype == "fp64":
        if args.momentum != 0:
            raise SystemExit("bench: --dtype fp64 runs the reference's plain SGD (GpuNet64.sgd): --momentum 0 only")
        if world > 1:
            raise SystemExit("bench: --dtype fp64 (the reference precision, GpuNet64) runs on one GPU")
        head = timed_run64(args, spec, B, d_img, d_lab, dev)
        args.fp32_extra = "off"
    else:
        head = timed_run(args, spec, args.dtype, B, d_img, d_lab, dev, dev_idx, rank, world, multi,
                         eager_anchor=args.eager_anchor == "on" or (args.eager_anchor == "auto" and world == 1))
    # BASELINE config 2 ("LeNet-5 fp32 on one MI355X") in the same run: a
    # second trainer after the first is freed, same graph replay, same K / W
    extra = None
    if args.fp32_extra == "on" or (args.fp32_extra == "auto" and world == 1 and args.model == "lenet5"
                                   and args.dtype != "fp32"):
        extra = timed_run(args, spec, "fp32", B, d_img, d_lab, dev, dev_idx, rank, world, multi)

    if rank == 0:
        value = B * world * args.steps / head["elapsed"]
        out = {
            "metric": metric_for(args.model),
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * head["elapsed"] / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_IMG_S, 2) if args.model == "lenet5" else None,
            "dtype": args.dtype,
            "data": f"synthetic ({C}x{H}x{W} u8 stripe images, device-resident, random-init weights)",
            "config": {
                "model": args.model,
                "global_batch": B * world,
                "seq_len": H * W,
                "parallelism": f"dp{world}",
                "batch_per_gpu": B,
                "input_shape": f"{C}x{H}x{W}",
                "optimizer": head["optimizer"],
                "allreduce": head["allreduce"],
                head["loss_key"]: head["loss"],
                "launch": head["launch"],
            },
        }
        if head.get("eager"):
            out["eager"] = head["eager"]
        if extra is not None:
            v32 = B * world * args.steps / extra["elapsed"]
            out["fp32"] = {
                "config": f"BASELINE config 2: {args.model} fp32 (exact f32 MFMA / fp32 VALU), dp{world}, "
                          f"batch_per_gpu {B}, same data, second timed region of this run",
                "value": round(v32, 1),
                "unit": "images/s",
                "ms_per_step": round(1000.0 * extra["elapsed"] / args.steps, 4),
                "steps": args.steps,
                "warmup": args.warmup,
                "vs_baseline": round(v32 / BASELINE_IMG_S, 2) if args.model == "lenet5" else None,
                extra["loss_key"]: extra["loss"],
                "launch": extra["launch"],
            }
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
