"""Python training entry point with the reference CLI (cnn.c:406-531).

    python -m mpi_cuda_cnn_amd.train train-images train-labels test-images test-labels \
        [--model ref|lenet5|cifar3|vgg11] [--epochs 10] [--batch 32] [--lr 0.1] [--dtype bf16|fp32]
        [--device gpu|cpu] [--save W] [--load W] [--json PATH|-]
    torchrun --nproc-per-node 8 -m mpi_cuda_cnn_amd.train ...      (data parallel, RCCL)

Exit codes and stderr lines follow the reference: 100 for too few arguments,
111 for unreadable/mismatched IDX files; "training...", "i=%d, error=%.4f",
"testing...", "i=%d", "ntests=%d, ncorrect=%d".  GPU runs use the native HIP
engine (``trainer.GpuTrainer``), CPU runs the native fp64 executor with the
same data-parallel protocol over gloo (``parallel.cpu_dp``).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def _parse(argv):
    ap = argparse.ArgumentParser(prog="mpi_cuda_cnn_amd.train", add_help=True)
    ap.add_argument("paths", nargs="*")
    ap.add_argument("--model", default="ref")
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--momentum", type=float, default=0.0)
    ap.add_argument("--weight-decay", type=float, default=0.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--device", default="auto", choices=["auto", "gpu", "cpu"])
    ap.add_argument("--bucket-mb", type=float, default=4.0)
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo", "none"],
                    help="torch.distributed backend (auto: nccl = RCCL on GPUs at any world size, "
                         "gloo on CPU when world > 1; none: no process group, world 1 only)")
    ap.add_argument("--log-every", type=int, default=1000)
    ap.add_argument("--save", default="")
    ap.add_argument("--load", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--synthetic", type=int, default=0,
                    help="generated stripe data (N train / N/5 test images) instead of IDX files")
    return ap.parse_args(argv)


def _load_idx(path, spec):
    """An IDX file or 'synthetic:<N>:<seed>:images|labels' (same syntax as the
    native binaries, csrc/apps/cli.h load_idx)."""
    from . import _C

    if not path.startswith("synthetic:"):
        arr = _C.idx_read(path)
        if arr.ndim == 1 and arr.size and int(arr.max()) >= spec.num_classes():
            # labels index the loss kernels (the reference only compared j == label, cnn.c:462)
            raise RuntimeError(f"{path}: label {int(arr.max())} is not a class of the model "
                               f"({spec.num_classes()} classes)")
        return arr
    _, n, seed, kind = path.split(":")
    C, H, W = spec.input_shape()
    imgs, labels = _C.synth_dataset(int(n), C, H, W, spec.num_classes(), seed=int(seed))
    return labels if kind == "labels" else imgs.reshape(int(n), H, W, C)


def _log(rank, msg):
    if rank == 0:
        sys.stderr.write(f"{msg}\n")  # one write per line (see the shard line)
        sys.stderr.flush()


def main(argv=None) -> int:
    a = _parse(sys.argv[1:] if argv is None else argv)
    if a.synthetic > 0 and not a.paths:
        n, m = a.synthetic, max(1, a.synthetic // 5)
        a.paths = [f"synthetic:{n}:1:images", f"synthetic:{n}:1:labels", f"synthetic:{m}:2:images",
                   f"synthetic:{m}:2:labels"]
    if len(a.paths) < 4:
        return 100
    import torch
    import torch.distributed as dist

    from . import _C

    use_gpu = a.device == "gpu" or (a.device == "auto" and torch.cuda.is_available())
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if use_gpu:
        # more ranks than GPUs (rehearsal on a small box, gloo only): share devices
        local_rank %= max(1, torch.cuda.device_count())
    backend = a.dist_backend
    if backend == "auto":
        backend = "nccl" if use_gpu else ("gloo" if world > 1 else "none")
    if backend == "none" and world > 1:
        backend = "nccl" if use_gpu else "gloo"
    if use_gpu:
        torch.cuda.set_device(local_rank)
    if backend != "none":
        from .parallel.ddp import init_process_group

        init_process_group(backend, torch.device("cuda", local_rank) if use_gpu else None)
    try:
        return _train(a, world, rank, local_rank, use_gpu)
    except (RuntimeError, dist.DistBackendError) as e:  # a failed collective (peer gone, deadline passed)
        print(f"rank {rank}: {e}", file=sys.stderr, flush=True)
        if not dist.is_initialized():
            return 111
        _exit_now(111)


def _exit_now(rc: int):
    """Leave the process with ``rc`` without interpreter teardown.

    After a failed collective the process group cannot be destroyed cleanly
    (its peer is gone), and returning through ``sys.exit`` lets the backend's
    background threads run into the teardown: gloo's pair thread calls
    ``std::terminate`` on the read error (rc -6 instead of 111, roughly every
    other run).  Reference contract: a failing rank exits 111 and its peers
    must not hang (defect D9, cnnmpi.c:443-453) -- so flush and ``_exit``."""
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(rc)


def _fault(rank, it):
    """Fault injection for the failure-detection tests: MCC_FAULT_RANK=r
    MCC_FAULT_STEP=k makes rank r die abruptly before step k."""
    if os.environ.get("MCC_FAULT_RANK") == str(rank) and os.environ.get("MCC_FAULT_STEP") == str(it):
        print(f"rank {rank}: injected fault at step {it}", file=sys.stderr, flush=True)
        os._exit(17)


def _train(a, world, rank, local_rank, use_gpu) -> int:
    import torch
    import torch.distributed as dist

    from . import _C

    try:
        if a.load:
            spec, params = _C.load_weights(a.load)
        else:
            spec = _C.make_model(a.model)
            params = _C.init_params(spec, a.seed)
        tr_img = _load_idx(a.paths[0], spec)
        tr_lab = _load_idx(a.paths[1], spec)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        return 111
    C, H, W = spec.input_shape()
    N = tr_img.shape[0]
    if tr_img[0].size != C * H * W or tr_lab.shape[0] < N:
        return 111
    tr_img = tr_img.reshape(N, H, W, C)
    lo, hi = N // world * rank, N // world * (rank + 1)
    if world > 1:
        # one write per line: ranks share the stderr pipe, and print() writes
        # the text and the newline separately (lines interleaved under load)
        sys.stderr.write(f"{rank} {lo} {hi}\n")
        sys.stderr.flush()
    b = max(1, a.batch // world)
    B = b * world  # effective global batch (SGD mean, sample count, img/s)
    total = a.epochs * N
    steps = (total + B - 1) // B
    rng = np.random.default_rng(a.seed * 7919 + rank)
    _log(rank, "training...")
    t0 = time.time()
    etotal, ecount, seen = 0.0, 0, 0

    if use_gpu:
        from .trainer import GpuTrainer

        dev = torch.device("cuda", local_rank)
        d_img = torch.from_numpy(np.ascontiguousarray(tr_img)).to(dev)
        d_lab = torch.from_numpy(tr_lab[:N]).to(dev)
        tr = GpuTrainer(spec, dtype=a.dtype, batch=max(b, 1024), device=local_rank, lr=a.lr, momentum=a.momentum,
                        weight_decay=a.weight_decay, params=params, bucket_bytes=int(a.bucket_mb * (1 << 20)))
        gen = torch.Generator(device=dev)
        gen.manual_seed(a.seed * 7919 + rank)
        tr.zero_stats()
        for it in range(steps):
            _fault(rank, it)
            idx = torch.randint(lo, hi, (b,), device=dev, dtype=torch.int32, generator=gen)
            tr.step(d_img, d_lab, idx, b)
            prev, seen = seen, seen + B
            mark = (prev + a.log_every - 1) // a.log_every * a.log_every
            if mark < seen:
                st = tr.net.get_stats()
                # [this rank's MSE sum, this rank's samples], summed over ranks
                mse = torch.tensor([st["mse_sum"], float((seen - ecount) // world)], dtype=torch.float64, device=dev)
                if dist.is_initialized():
                    dist.all_reduce(mse)
                _log(rank, f"i={mark}, error={mse[0].item() / max(1.0, mse[1].item()):.4f}")
                ecount = seen
                tr.zero_stats()
        torch.cuda.synchronize()
        final = tr.state_dict().astype(np.float64)

        def evaluate(img, lab):
            n = img.shape[0]
            ti = torch.from_numpy(np.ascontiguousarray(img)).to(dev)
            tl = torch.from_numpy(lab[:n]).to(dev)
            return tr.evaluate(ti, tl)
    else:
        from .parallel.cpu_dp import CpuDataParallel

        dp = CpuDataParallel(spec, params, dtype="fp64", bucket_bytes=int(a.bucket_mb * (1 << 20)), lr=a.lr)
        for it in range(steps):
            _fault(rank, it)
            sel = rng.integers(lo, hi, size=b)
            x = tr_img[sel].transpose(0, 3, 1, 2).reshape(b, -1) / 255.0
            st = dp.step(x, tr_lab[sel].astype(np.int32), b * world)
            etotal += st["mse_sum"]
            prev, seen = seen, seen + B
            mark = (prev + a.log_every - 1) // a.log_every * a.log_every
            if mark < seen:
                _log(rank, f"i={mark}, error={etotal / max(1, (seen - ecount) // world):.4f}")
                etotal, ecount = 0.0, seen
        final = dp.params().astype(np.float64)

        def evaluate(img, lab):
            net = _C.CpuNet64(spec)
            net.set_params(final)
            n = img.shape[0]
            correct = 0
            for i in range(0, n, 256):
                x = img[i : i + 256].transpose(0, 3, 1, 2).reshape(-1, C * H * W) / 255.0
                net.forward(x)
                correct += net.evaluate(lab[i : i + x.shape[0]].astype(np.int32))["correct"]
            return n, correct

    train_s = time.time() - t0
    rc = 0
    if rank == 0:
        try:
            te_img = _load_idx(a.paths[2], spec)
            te_lab = _load_idx(a.paths[3], spec)
        except RuntimeError as e:
            print(e, file=sys.stderr)
            rc = 111
        if rc == 0:
            n = te_img.shape[0]
            if te_img[0].size != C * H * W or te_lab.shape[0] < n:
                rc = 111
            else:
                _log(rank, "testing...")
                for i in range(0, n, 1000):
                    _log(rank, f"i={i}")
                ntests, ncorrect = evaluate(te_img.reshape(n, H, W, C), te_lab)
                _log(rank, f"ntests={ntests}, ncorrect={ncorrect}")
                if a.save:
                    _C.save_weights(a.save, spec, final)
                if a.json:
                    out = {"program": "mpi_cuda_cnn_amd.train", "model": spec.name, "device": "gpu" if use_gpu else "cpu",
                           "world": world, "train_img_per_s": steps * B / max(train_s, 1e-9), "ntests": ntests,
                           "ncorrect": ncorrect}
                    if a.json == "-":
                        print(json.dumps(out))
                    else:
                        with open(a.json, "w") as f:
                            json.dump(out, f)
    if dist.is_initialized():
        # every rank leaves with rank 0's verdict (no rank waits on a failed peer)
        v = torch.tensor([rc], dtype=torch.int64, device=torch.device("cuda", local_rank) if use_gpu else None)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        rc = int(v.item())
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
