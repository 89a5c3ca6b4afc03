"""N>1 path on CPU: world_size-2 gloo run of the tile partition + gather + unpack used by
bench.py (ray_tracying_amd/tiles.py).  Each rank renders ONLY its tiles (with the oracle as
the per-tile renderer -- the GPU kernel is covered by test_gpu_parity); rank 0 gathers over
torch.distributed and must reassemble a frame identical to the single-process render."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, scene_path, args, tile, q, balanced=False):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind as ob
    from ray_tracying_amd import tiles as tl
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W, H, _, _ = ob.scene_info(scene_path)
    tx, ty = tl.tile_grid(W, H, tile)
    n = tx * ty
    # balanced: the cost-balanced deal bench.py uses, from costs every rank derives alike
    deal = tl.balanced_deal(np.random.default_rng(7).random(n), world) if balanced else None
    mine = tl.assign_tiles(n, world, rank, tx, deal)
    packed = np.zeros((tl.tiles_per_rank(n, world, tx, deal), tile, tile, 3), np.float32)
    for k, tid in enumerate(mine):
        x0, y0 = (tid % tx) * tile, (tid // tx) * tile
        w, h = min(tile, W - x0), min(tile, H - y0)
        rgb, _, _ = ob.render(scene_path, rng=ob.RNG_COUNTER, seed=5, region=(x0, y0, w, h), **args)
        packed[k, :h, :w] = rgb
    got = tl.gather_to_root(dist, torch.from_numpy(packed.reshape(-1)), rank, world)
    if rank == 0:
        q.put(tl.unpack([g.numpy() for g in got], world, n, tile, W, H, deal))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,balanced", [(2, False), (3, False), (2, True), (3, True)])
def test_tiles_gather_equals_single_render(world, balanced, tmp_path):
    import multiprocessing as mp
    import socket
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind as ob
    import scenes
    path, args = scenes.materialise("soup_s3", str(tmp_path))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, args, 8, q, balanced)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full, _, _ = ob.render(path, rng=ob.RNG_COUNTER, seed=5, **args)
    assert np.array_equal(img.view(np.uint32), full.view(np.uint32))


def test_assign_tiles_is_a_partition():
    from ray_tracying_amd import tiles as tl
    for n, tx in ((1, 1), (7, 7), (12, 4), (256, 16), (1024, 32)):
        for world in (1, 2, 3, 4, 6, 8):
            parts = [tl.assign_tiles(n, world, r, tx) for r in range(world)]
            allt = np.sort(np.concatenate(parts))
            assert np.array_equal(allt, np.arange(n))
            assert max(len(p) for p in parts) == tl.tiles_per_rank(n, world, tx)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_lattice_deal_balances_a_centred_object(world):
    """The headline frame's work sits in the centre (the soup); plain t mod world would give
    2 of 8 ranks the central columns.  With the lattice deal every rank's share of a centred
    disc of tiles stays within 20% of the mean."""
    from ray_tracying_amd import tiles as tl
    tx = 16
    yy, xx = np.mgrid[0:tx, 0:tx]
    heavy = ((xx - 7.5) ** 2 + (yy - 7.5) ** 2 <= 5.5 ** 2).reshape(-1)
    load = [heavy[tl.assign_tiles(tx * tx, world, r, tx)].sum() for r in range(world)]
    assert max(load) <= 1.2 * np.mean(load), load
    naive = [heavy[np.arange(tx * tx) % world == r].sum() for r in range(world)]
    assert max(load) <= max(naive)


def test_balanced_deal_is_an_even_partition():
    from ray_tracying_amd import tiles as tl
    rng = np.random.default_rng(3)
    for n in (1, 7, 12, 256, 1024):
        costs = rng.random(n) * (rng.random(n) < 0.4)  # many zero-cost (background) tiles
        for world in (1, 2, 3, 4, 6, 8):
            deal = tl.balanced_deal(costs, world)
            parts = [tl.assign_tiles(n, world, r, None if world == 1 else 1, deal) for r in range(world)]
            assert np.array_equal(np.sort(np.concatenate(parts)), np.arange(n))
            sizes = [len(p) for p in parts]
            assert max(sizes) - min(sizes) <= 1 and max(sizes) == tl.tiles_per_rank(n, world, 1, deal)
            assert np.array_equal(deal, tl.balanced_deal(costs, world))  # deterministic


@pytest.mark.parametrize("world", [2, 4, 8])
def test_balanced_deal_beats_the_lattice_on_a_centred_object(world):
    """A centred, peaked cost (the soup's projected centres): the cost-balanced deal's busiest
    rank is within 1 % of the mean and never worse than the lattice's."""
    from ray_tracying_amd import tiles as tl
    tx = 16
    yy, xx = np.mgrid[0:tx, 0:tx]
    cost = np.exp(-((xx - 7.5) ** 2 + (yy - 7.5) ** 2) / 18.0).reshape(-1) * 1000.0
    deal = tl.balanced_deal(cost, world)
    bal = [cost[tl.assign_tiles(tx * tx, world, r, tx, deal)].sum() for r in range(world)]
    lat = [cost[tl.assign_tiles(tx * tx, world, r, tx)].sum() for r in range(world)]
    assert max(bal) <= 1.01 * np.mean(bal), bal
    assert max(bal) <= max(lat) + 1e-9
