"""Image-tile data parallelism across GPUs (one process per GPU, torch.distributed).

The reference renders serially (raytracer.cpp:433-476) and has no parallel path; with the
counter RNG every pixel/sample is independent, so the frame is split into tiles, dealt
round-robin to ranks (scene content is spatially uneven, so interleaving balances load),
rendered independently, and the packed tiles are gathered to rank 0 -- over RCCL/xGMI on
MI355X (backend "nccl"), over gloo in the CPU tests.  The result is bit-identical for any
world size (tests/test_distributed.py, tests/test_gpu_parity.py).
"""
from __future__ import annotations

import numpy as np


def tile_grid(width: int, height: int, tile: int) -> tuple[int, int]:
    return (width + tile - 1) // tile, (height + tile - 1) // tile


def assign_tiles(n_tiles: int, world: int, rank: int) -> np.ndarray:
    """Round-robin deal: tile t -> rank t % world."""
    ids = np.arange(n_tiles, dtype=np.int32)
    return ids[ids % world == rank]


def tiles_per_rank(n_tiles: int, world: int) -> int:
    return (n_tiles + world - 1) // world


def unpack(packed_per_rank, world: int, n_tiles: int, tile: int, width: int, height: int) -> np.ndarray:
    """Assemble an image from each rank's packed tiles (rank r holds tiles r, r+world, ...)."""
    img = np.zeros((height, width, 3), dtype=np.float32)
    tiles_x, _ = tile_grid(width, height, tile)
    for r in range(world):
        buf = np.asarray(packed_per_rank[r], dtype=np.float32).reshape(-1, tile, tile, 3)
        for k, tid in enumerate(assign_tiles(n_tiles, world, r)):
            x0, y0 = (tid % tiles_x) * tile, (tid // tiles_x) * tile
            w, h = min(tile, width - x0), min(tile, height - y0)
            img[y0:y0 + h, x0:x0 + w] = buf[k, :h, :w]
    return img


def gather_to_root(dist, local, rank: int, world: int):
    """dist.gather of equally sized per-rank buffers to rank 0 (RCCL on GPU tensors)."""
    if world == 1:
        return [local]
    out = [local.new_empty(local.shape) for _ in range(world)] if rank == 0 else None
    dist.gather(local, out, dst=0)
    return out
