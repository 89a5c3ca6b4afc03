#!/usr/bin/env python3
"""gather_cost.py -- cost of the per-frame framebuffer gather of bench.py's N-rank path.

Payloads: one rank's packed tiles (the buffer rank 0 receives from every peer each frame):
1024^2 split 8 ways = 32 tiles x 64^2 px x 12 B = 1.5 MiB (4-way 3 MiB, 2-way 6 MiB), 4096^2
8-way (C5) = 25.2 MiB.  One GPU cannot exercise xGMI, so three figures are measured / stated:
  * d2d_ms       -- a device-to-device copy of the payload (the local HBM part),
  * gather_ms    -- one torch.distributed.gather of the payload at world size 1 over the nccl
                    (RCCL) backend on this GPU, bracketed by torch.cuda.synchronize() the way
                    bench.py's step is: the collective's fixed launch / synchronisation cost,
                    which a bandwidth model misses,
  * xgmi_est_ms  -- the payload over one point-to-point xGMI link (~150 GB/s; rank 0 receives
                    every peer over its own link, concurrently).
The multi-GPU prediction (tools/shares_summary.py) adds gather_ms + xgmi_est_ms to the slowest
rank's frame.  Run: python3 tools/gather_cost.py [out.json]
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

PAYLOADS = (("head_8way", 256 // 8), ("head_4way", 256 // 4), ("head_2way", 256 // 2), ("c5_8way", 4096 // 8))


def time_copy(nbytes: int, reps: int = 50) -> float:
    src = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda:0")
    dst = torch.empty_like(src)
    for _ in range(5):
        dst.copy_(src)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        dst.copy_(src)
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def time_gather(nbytes: int, reps: int = 50) -> tuple[float, float]:
    """(mean, min) wall ms of one gather to rank 0 with a synchronize before and after."""
    buf = torch.ones(nbytes // 4, dtype=torch.float32, device="cuda:0")
    out = [torch.empty_like(buf)]
    for _ in range(5):
        dist.gather(buf, out, dst=0)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dist.gather(buf, out, dst=0)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    assert torch.equal(out[0], buf)
    return sum(ts) / len(ts), min(ts)


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    res = {"world_size": 1, "backend": "nccl (RCCL)", "xgmi_link_gbs": 150.0}
    for name, tiles in PAYLOADS:
        nb = tiles * 64 * 64 * 12
        g_mean, g_min = time_gather(nb)
        res[name] = {"bytes": nb, "d2d_ms": round(time_copy(nb), 4), "gather_ms": round(g_mean, 4),
                     "gather_min_ms": round(g_min, 4), "xgmi_est_ms": round(nb / 150e9 * 1e3, 4)}
    dist.destroy_process_group()
    line = json.dumps(res)
    print(line)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(line + "\n")


if __name__ == "__main__":
    main()
