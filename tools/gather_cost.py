#!/usr/bin/env python3
"""gather_cost.py -- device-to-device copy time of one rank's packed tiles (the payload the
RCCL gather moves to rank 0 each frame): 1024^2 frame split 8 ways = 32 tiles x 64^2 px x 12 B
= 1.5 MiB (the bench's buffer holds tiles_per_rank tiles: 4 MiB at 2-way), 4096^2 8-way =
25.2 MiB.  One GPU cannot exercise xGMI, so this is the local HBM copy cost; the xGMI transfer
of the same bytes over one point-to-point link (~150 GB/s) is added as an estimate: rank 0 receives
every peer over its own link, concurrently."""
import json

import torch


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


out = {}
for name, tiles in (("head_8way", 256 // 8), ("head_4way", 256 // 4), ("head_2way", 256 // 2), ("c5_8way", 4096 // 8)):
    nb = tiles * 64 * 64 * 12
    ms = time_copy(nb)
    out[name] = {"bytes": nb, "d2d_ms": round(ms, 4), "xgmi_estimate_ms": round(nb / 150e9 * 1e3, 4)}
print(json.dumps(out))
