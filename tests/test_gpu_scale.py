"""GPU parity at the measured scale: the headline 1M-triangle soup (bench.py's workload,
SURVEY.md 8(d) C5 scene; Plane::intersect shapes.cpp:444-494 over the reference's
median-split leaves acceleration.cpp:20-118).

What only this size exercises: spatial-split duplicate parts (~1.1M primitive records), the
24-bit leaf packing, depth-12+ trees (the 64K-slot rerun also cuts the LDS stack to 2
entries, so deeper entries spill to HBM), and a frame whose units outnumber the slots, so
every slot-wave claims many batches.  The GPU
renders a subset of the frame's 64x64 tiles through rt_render_tiles (the path bench.py
times); the oracle renders the same regions in counter-RNG mode after one scene load
(oracle_render_regions, rows over host threads).  Bar: every float bit-identical and the
ray counts equal.
"""
import os

import numpy as np
import pytest

import oracle_bind as ob
import ray_tracying_amd as rt

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]
SOUP_SEED = 20251226   # bench.py / SURVEY.md 8(d) C5 generator seed
N_TRIS = 1_000_000
T = 64


@pytest.fixture(scope="module")
def soup_path(tmp_path_factory):
    p = str(tmp_path_factory.mktemp("soup") / "soup1m.json")
    rt.make_soup(p, N_TRIS, seed=SOUP_SEED, width=1024, height=1024)
    return p


def _render_tiles(scene, tiles, spp_sqrt, seed):
    import torch
    ds = rt.DeviceScene(scene, 0)
    try:
        buf = torch.zeros(len(tiles) * T * T * 3, dtype=torch.float32, device="cuda:0")
        st = ds.render_tiles(np.asarray(tiles, dtype=np.int32), T, T, buf.data_ptr(),
                             rt.RenderParams(spp_sqrt=spp_sqrt, light_samples=1, use_bvh=True, seed=seed))
        torch.cuda.synchronize()
        return buf.cpu().numpy().reshape(len(tiles), T, T, 3), st
    finally:
        ds.close()


def _check(path, res, tiles, spp_sqrt, seed, slot_variants=()):
    tiles_x = res // T
    regions = [((t % tiles_x) * T, (t // tiles_x) * T, T, T) for t in tiles]
    ref, ost = ob.render_regions(path, regions, use_bvh=True, spp_sqrt=spp_sqrt, light_samples=1, seed=seed,
                                 resolution=(res, res))
    sc = rt.Scene(path, resolution=(res, res))
    try:
        assert sc.desc().n_prims > N_TRIS, "expected spatial-split duplicates at this size"
        assert sc.info.tree_depth >= 10
        for env in ({},) + tuple(slot_variants):
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                img, st = _render_tiles(sc, tiles, spp_sqrt, seed)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            for i, t in enumerate(tiles):
                bad = int((img[i].view(np.uint32) != ref[i].view(np.uint32)).sum())
                assert bad == 0, f"{env} tile {t}: {bad} channels differ from the oracle"
            assert st.rays == ost["rays"], (env, st.rays, ost["rays"])
    finally:
        sc.close()


def test_headline_soup_tiles_1024_100spp(soup_path, gpu):
    """bench.py's frame (1024^2, -s 10): the dense centre, the corners, an edge and two
    off-centre tiles (one-pass); then the same tiles through the step pipeline with only 64K
    slots (every wave claims ~37 batches), and with one and three slot pipelines -- the
    scheduling must not change a bit."""
    tiles = [7 * 16 + 7, 8 * 16 + 8, 0, 15 * 16 + 15, 8 * 16 + 15, 3 * 16 + 12, 12 * 16 + 4]
    _check(soup_path, 1024, tiles, 10, seed=SOUP_SEED,
           slot_variants=({"RT_ONE_PASS": "0", "RT_SLOTS": "65536", "RT_LDS_STACK": "2"},
                          {"RT_ONE_PASS": "0", "RT_PIPES": "1"},
                          {"RT_ONE_PASS": "0", "RT_PIPES": "3", "RT_LDS_STACK": "4"}))


def test_c5_tile_4096_64spp(soup_path, gpu):
    """C5's frame (4096^2, -s 8 = 64 spp): two tiles of the 64x64 grid (centre and edge)."""
    _check(soup_path, 4096, [32 * 64 + 32, 20 * 64 + 63], 8, seed=7)
