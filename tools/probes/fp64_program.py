"""The reference program at the reference precision on the GPU: `cnn_hip
--dtype fp64` (GpuNet64) vs the CPU executor `cnn`, same synthetic MNIST-shaped
IDX set, same CLI (reference hyper-parameters: lr 0.1, batch 32).

    python tools/probes/fp64_program.py [--train 60000] [--test 10000] [--epochs 1]

Prints one line per run with the program's own --json summary (train img/s,
accuracy).  profiles/fp64_program_r4.txt holds a run.
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import mpi_cuda_cnn_amd as mcc  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--train", type=int, default=60000)
    ap.add_argument("--test", type=int, default=10000)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--cpu-train", type=int, default=6000, help="samples for the (slow) CPU runs")
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="fp64_")
    paths = []
    for n, seed, pre in ((a.train, 1, "train"), (a.test, 2, "test")):
        imgs, labels = mcc.synth_dataset(n, 1, 28, 28, 10, seed=seed)
        pi, pl = os.path.join(d, pre + "-images"), os.path.join(d, pre + "-labels")
        mcc.idx_write(pi, imgs.reshape(n, 28, 28))
        mcc.idx_write(pl, labels)
        paths += [pi, pl]
    runs = [
        ("cnn_hip fp64 (GPU)", "cnn_hip", ["--dtype", "fp64"], a.train),
        ("cnn_hip fp64 --ref-compat (GPU)", "cnn_hip", ["--dtype", "fp64", "--ref-compat"], a.train),
        ("cnn fp64 (CPU, 1 thread)", "cnn", [], a.cpu_train),
        ("cnn fp64 --ref-compat (CPU, 1 thread)", "cnn", ["--ref-compat"], a.cpu_train),
    ]
    for name, prog, extra, ntrain in runs:
        cmd = [os.path.join(ROOT, "build", "bin", prog)] + paths + ["--epochs", str(a.epochs), "--max-train",
                                                                    str(ntrain), "--json", "-"] + extra
        t0 = time.time()
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        wall = time.time() - t0
        if r.returncode != 0:
            print(f"{name}: rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
            return 1
        js = json.loads([s for s in r.stdout.splitlines() if s.startswith("{")][-1])
        print(f"{name}: train {js['train_img_per_s']:.0f} img/s over {js['train_samples']} samples, "
              f"test {js['ncorrect']}/{js['ntests']}, wall {wall:.1f} s", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
