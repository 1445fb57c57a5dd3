"""Minimal single-node launcher: one process per GPU (or per CPU rank).

    python -m mpi_cuda_cnn_amd.launch -n 8 build/bin/cnn_dist <4 IDX files> [flags]
    python -m mpi_cuda_cnn_amd.launch -n 8 --python bench.py --gpus 8

Sets RANK / WORLD_SIZE / LOCAL_RANK / LOCAL_WORLD_SIZE / MASTER_ADDR /
MASTER_PORT for each child (the same contract torchrun uses, so the native
`cnn_dist` and the torch.distributed path read one environment), forwards
signals, and if any rank exits non-zero terminates the others — a failed
rank never leaves its peers hanging in a collective (reference defect D9).
Replaces ``mpirun -np 8`` from the reference Makefile (Makefile:44).
"""

from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(nproc: int, cmd: list[str], master_addr: str = "127.0.0.1", master_port: int | None = None,
           env_extra: dict | None = None, timeout: float | None = None) -> int:
    port = master_port or _free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update(
            RANK=str(r),
            WORLD_SIZE=str(nproc),
            LOCAL_RANK=str(r),
            LOCAL_WORLD_SIZE=str(nproc),
            MASTER_ADDR=master_addr,
            MASTER_PORT=str(port),
        )
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen(cmd, env=env))

    def kill_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass

    signal.signal(signal.SIGINT, lambda *_: kill_all(signal.SIGINT))
    signal.signal(signal.SIGTERM, lambda *_: kill_all())
    t0 = time.time()
    rc = 0
    while any(p.poll() is None for p in procs):
        for p in procs:
            code = p.poll()
            if code not in (None, 0):
                rc = rc or code
                kill_all()
        if timeout is not None and time.time() - t0 > timeout:
            rc = rc or 124
            kill_all(signal.SIGKILL)
        time.sleep(0.05)
    for p in procs:
        rc = rc or p.returncode
    return rc


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-n", "--nproc", type=int, required=True)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("--python", action="store_true", help="run the program with this interpreter")
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd
    if cmd and cmd[0] == "--":
        cmd = cmd[1:]
    if not cmd:
        ap.error("missing command")
    if a.python:
        cmd = [sys.executable] + cmd
    sys.exit(launch(a.nproc, cmd, a.master_addr, a.master_port, timeout=a.timeout))


if __name__ == "__main__":
    main()
