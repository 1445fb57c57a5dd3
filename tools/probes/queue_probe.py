"""Which HIP streams share a hardware queue (GPU_MAX_HW_QUEUES=4 on the box)?
Launches a long spin kernel on the default stream, then a short kernel on a
second stream, for several ways of creating that second stream, and reports
whether the short kernel finished while the spin was still running.  Also
issues an RCCL all-reduce from a world-1 process group created with and
without a high-priority stream (run under rocprofv3 --kernel-trace to read
the Queue_Id of each kernel)."""
import os
import time

import torch
import torch.distributed as dist


def concurrent(s2):
    s1 = torch.cuda.current_stream()
    x = torch.ones(1024, device="cuda")
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e2 = torch.cuda.Event(enable_timing=True)
    e0.record(s1)
    torch.cuda._sleep(200_000_000)  # ~100 ms spin on s1
    e1.record(s1)
    with torch.cuda.stream(s2):
        y = x * 2
        e2.record(s2)
    torch.cuda.synchronize()
    t_spin = e0.elapsed_time(e1)
    t_other = e0.elapsed_time(e2)
    return t_spin, t_other, t_other < 0.5 * t_spin


for name, mk in [
    ("pool stream prio 0", lambda: torch.cuda.Stream()),
    ("pool stream prio -1 (high)", lambda: torch.cuda.Stream(priority=-1)),
    ("2nd pool stream prio 0", lambda: torch.cuda.Stream()),
    ("3rd pool stream prio 0", lambda: torch.cuda.Stream()),
]:
    s = mk()
    ts, to, ok = concurrent(s)
    print(f"{name:32s} spin {ts:7.1f} ms, other done at {to:7.1f} ms -> {'CONCURRENT' if ok else 'serialized'}", flush=True)

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29633", RANK="0", WORLD_SIZE="1")
hp = os.environ.get("HP", "0") == "1"
opts = dist.ProcessGroupNCCL.Options()
opts.is_high_priority_stream = hp
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), pg_options=opts)
g = torch.ones(1 << 20, device="cuda")
torch.cuda.synchronize()
e0 = torch.cuda.Event(enable_timing=True)
e1 = torch.cuda.Event(enable_timing=True)
e0.record()
torch.cuda._sleep(200_000_000)
e1.record()
t0 = time.time()
w = dist.all_reduce(g[: 1 << 10], op=dist.ReduceOp.AVG, async_op=True)  # waits for the spin (producer order)
h = torch.ones(1 << 20, device="cuda")
w2 = dist.all_reduce(h, op=dist.ReduceOp.AVG, async_op=True)
torch.cuda.synchronize()
print(f"rccl high-priority stream={hp}: done", flush=True)
dist.destroy_process_group()
