"""Time the C4 exchange buffers' RCCL all-reduce (torch.distributed "nccl" = RCCL) on this box.

Run under torch.distributed.run (any world size; on the one-GPU box world size 1):
  python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 tools/rccl_allreduce_time.py
Buffers: all-reduce #1 = [S (m_p^2), t (m_p), r'r + pad] = 1024^2 + 1024 + 8 doubles (8.4 MB at
C3/C4), all-reduce #2 = L + 5 = 13 doubles.  Prints one JSON line (rank 0): mean / min time per
all-reduce over 50 repetitions, timed with HIP events on the current stream after 5 warm-ups.
"""
import json
import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    out = {"world_size": dist.get_world_size(), "backend": "nccl (RCCL)"}
    for name, count in (("red1_8.4MB", 1024 * 1024 + 1024 + 8), ("red2_13", 13)):
        buf = torch.ones(count, dtype=torch.float64, device=dev)
        for _ in range(5):
            dist.all_reduce(buf)
        torch.cuda.synchronize(dev)
        times = []
        for _ in range(50):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            dist.all_reduce(buf)
            b.record()
            b.synchronize()
            times.append(a.elapsed_time(b))
        out[name] = {"bytes": count * 8, "mean_ms": sum(times) / len(times), "min_ms": min(times)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
