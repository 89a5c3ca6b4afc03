"""GPU parity at the C3 / C4 bench configurations (bench.py --scene ...):
1024^2 at -s 10 (100 jittered spp), C4 with light radius 1.0 and -light_sample 4.

At these settings a frame runs many steps, every slot-wave claims many batches, the tracing
lane continues soft-shadow samples (kSoft, soft_start) and reflection chains go 10 deep
(Code/raytracer.cpp:18-70 compute_pixel_color, :180-274 shade, :280-351 Trace).  The GPU
renders four 64x64 tiles of the frame through rt_render_tiles -- the call bench.py times --
chosen to cover the spheres, the cube, the floor and their reflections; the oracle renders
the same regions in counter-RNG mode.  Bar: every float bit-identical and the ray counts
equal, by default (C3 one-pass, C4 the step pipeline) and through the step pipeline with two
slot pipelines (RT_ONE_PASS=0 RT_PIPES=2, which an explicit request allows at any call size:
the multi-pipeline scheduler at the full configurations).
"""
import os

import numpy as np
import pytest

import oracle_bind as ob
import ray_tracying_amd as rt
import scenes

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]
T = 64
RES = 1024


def _render(sc, tiles, spp_sqrt, light_samples, seed, env):
    import torch
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    ds = rt.DeviceScene(sc, 0)
    try:
        buf = torch.zeros(len(tiles) * T * T * 3, dtype=torch.float32, device="cuda:0")
        st = ds.render_tiles(np.asarray(tiles, dtype=np.int32), T, T, buf.data_ptr(),
                             rt.RenderParams(spp_sqrt=spp_sqrt, light_samples=light_samples, use_bvh=True, seed=seed))
        torch.cuda.synchronize()
        return buf.cpu().numpy().reshape(len(tiles), T, T, 3), st
    finally:
        ds.close()
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _check(path, tiles, spp_sqrt, light_samples, seed):
    tiles_x = RES // T
    regions = [((t % tiles_x) * T, (t // tiles_x) * T, T, T) for t in tiles]
    ref, ost = ob.render_regions(path, regions, use_bvh=True, spp_sqrt=spp_sqrt, light_samples=light_samples,
                                 seed=seed, texture_root=scenes.TEXTURES, resolution=(RES, RES))
    sc = rt.Scene(path, resolution=(RES, RES), texture_root=scenes.TEXTURES)
    try:
        for env in ({}, {"RT_ONE_PASS": "0", "RT_PIPES": "2"}):
            img, st = _render(sc, tiles, spp_sqrt, light_samples, seed, env)
            for i, t in enumerate(tiles):
                bad = int((img[i].view(np.uint32) != ref[i].view(np.uint32)).sum())
                assert bad == 0, f"{env} tile {t}: {bad} channels differ from the oracle"
            assert st.rays == ost["rays"], (env, st.rays, ost["rays"])
    finally:
        sc.close()


def test_c3_antialiasing_tiles_1024_100spp(tmp_path, gpu):
    """C3: Antialiasing.blend (cube + plane, point light), -s 10."""
    p = scenes.write(scenes.blend("Antialiasing", (RES, RES)), str(tmp_path / "c3.json"))
    # the cube's top and side faces, its silhouette, and the lit floor
    _check(p, [9 * 16 + 7, 12 * 16 + 6, 7 * 16 + 6, 3 * 16 + 12], 10, 1, seed=20251226)


def test_c4_glossy_soft_tiles_1024_100spp(tmp_path, gpu):
    """C4: glossy_reflection.blend with light radius 1.0, -s 10 -light_sample 4 (soft shadows,
    rough and mirror-like metal spheres, the red cube)."""
    p = scenes.write(scenes.blend("glossy_reflection", (RES, RES), light_radius=1.0), str(tmp_path / "c4.json"))
    _check(p, [14 * 16 + 7, 10 * 16 + 4, 11 * 16 + 12, 7 * 16 + 9], 10, 4, seed=20251226)
