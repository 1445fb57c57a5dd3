"""Put the four MNIST IDX files the programs take into one directory
(the reference's `get_mnist` Makefile rule, Makefile:12-35, which needed dnf,
pip and a Google-Drive download, and left `make` without a rule when the files
were missing).

    python tools/get_mnist.py [--src DIR] [--out data] [--synthetic N]

* --src DIR: take MNIST files already on this machine, in any of the usual
  spellings (train-images-idx3-ubyte, train-images.idx3-ubyte, either
  gzipped), check their IDX headers and write them under --out with the
  names `make run_* DATA=...` uses.  Nothing is downloaded: there is no
  network here, and a fetch would run code and data from outside the tree.
* otherwise (or with --synthetic N): write the framework's synthetic
  MNIST-shaped set (N training / N/5 test images, the same generator as
  `--synthetic`) as IDX files under the same names.

Prints the four paths, in the programs' argument order.
"""

from __future__ import annotations

import argparse
import gzip
import os
import shutil
import struct
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

NAMES = ["train-images-idx3-ubyte", "train-labels-idx1-ubyte", "t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"]


def _candidates(src: str, name: str):
    dotted = name.replace("-idx", ".idx")
    for base in (name, dotted):
        for ext in ("", ".gz"):
            yield os.path.join(src, base + ext)


def _check_idx(path: str, want_dims: int) -> None:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        head = f.read(4)
    if len(head) != 4 or head[0] != 0 or head[1] != 0 or head[2] != 0x08 or head[3] != want_dims:
        raise SystemExit(f"{path}: not an unsigned-byte IDX file with {want_dims} dims")


def from_local(src: str, out: str) -> list[str]:
    paths = []
    copied = False
    for name in NAMES:
        found = next((p for p in _candidates(src, name) if os.path.exists(p)), None)
        if found is None:
            raise SystemExit(f"{name} not found under {src}")
        _check_idx(found, 3 if "images" in name else 1)
        dst = os.path.join(out, name)
        if found.endswith(".gz"):
            with gzip.open(found, "rb") as fi, open(dst, "wb") as fo:
                shutil.copyfileobj(fi, fo)
            copied = True
        elif not (os.path.exists(dst) and os.path.samefile(found, dst)):
            shutil.copyfile(found, dst)
            copied = True
        paths.append(dst)
    marker = os.path.join(out, "SYNTHETIC")
    if copied and os.path.exists(marker):  # files from elsewhere replace an earlier synthetic set
        os.remove(marker)
    return paths


def synthetic(out: str, n: int) -> list[str]:
    import mpi_cuda_cnn_amd as mcc

    paths = []
    for (count, seed), (img_name, lab_name) in zip(((n, 1), (max(1, n // 5), 2)), (NAMES[:2], NAMES[2:])):
        imgs, labels = mcc.synth_dataset(count, 1, 28, 28, 10, seed=seed)
        pi, pl = os.path.join(out, img_name), os.path.join(out, lab_name)
        mcc.idx_write(pi, imgs.reshape(count, 28, 28))
        mcc.idx_write(pl, labels)
        paths += [pi, pl]
    # the synthetic set uses the real MNIST file names: leave a marker so a
    # later run's accuracy / loss log is not mistaken for a real-MNIST one
    with open(os.path.join(out, "SYNTHETIC"), "w") as f:
        f.write(f"synthetic MNIST-shaped stripe images (mcc.synth_dataset), {n} train / {max(1, n // 5)} test;"
                " not real MNIST\n")
    print(f"get_mnist: no --src given: wrote a SYNTHETIC MNIST-shaped set under {out} "
          f"(marker {os.path.join(out, 'SYNTHETIC')})", file=sys.stderr)
    return paths


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="", help="directory holding MNIST files (raw or .gz)")
    ap.add_argument("--out", default="data")
    ap.add_argument("--synthetic", type=int, default=60000, help="images when no --src is given")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    paths = from_local(a.src, a.out) if a.src else synthetic(a.out, a.synthetic)
    for p in paths:  # header sanity of what was written
        with open(p, "rb") as f:
            magic, = struct.unpack(">I", f.read(4))
        assert magic >> 8 == 0x08, p
    print(" ".join(paths))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
