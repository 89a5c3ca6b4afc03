"""rt_render_frames (r06): several frames of the same tiles in ONE call -- every sample of them in
one camera pass, one traversal launch and one shading pass for one-pass scenes -- each frame
keyed by its own seed.  bench.py renders a rank's share of an N-way split this way (N frames per
call: launches of the whole frame's size).

Every frame of a multi-frame call must equal the single-frame call with its seed bit for bit,
with the summed ray count; the single-frame calls are pinned to the oracle elsewhere, and one
frame here is checked against the oracle directly.  Cases: the planes instance with fused
point-light shadows, transformed shapes under a thin lens with a moving sphere (stored origins
and ray times), tiles reaching past the image (the kind word), a rank-like tile subset in
costliest-first order, frames split over several passes (RT_ONE_PASS_MAX), and a step-pipeline
scene (reflection: its frames are rendered one after another).
The loop this replaces, once per frame: /root/reference/Code/raytracer.cpp:433-476.
"""
import os

import numpy as np
import pytest

import oracle_bind as ob
import ray_tracying_amd as rt
import scenes
from test_gpu_one_pass import _flat

pytestmark = pytest.mark.gpu
T = 32


def _case_scene(name):
    if name == "soup_lit":
        return scenes.soup(3000, seed=11, res=(128, 96)), 2
    if name == "shapes_thin_lens":
        return _flat(scenes.features(res=(96, 64), aperture=0.4, focus=5.0)), 2
    if name == "soup_edge":  # 100 x 70: tiles reach past the image
        return scenes.soup(2000, seed=5, res=(100, 70)), 2
    if name == "features_steps":  # reflection / refraction / soft lights: the step pipeline
        return scenes.features(res=(64, 64)), 1
    raise KeyError(name)


def _frames_vs_single(path, spp_sqrt, ids, seeds, env=None, light_samples=1):
    import torch
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    sc = rt.Scene(path, texture_root=scenes.TEXTURES)
    ds = rt.DeviceScene(sc, 0)
    try:
        n = ids.size * T * T * 3
        p = rt.RenderParams(spp_sqrt=spp_sqrt, light_samples=light_samples, use_bvh=True, seed=999)
        single, rays = [], 0
        buf = torch.zeros(n, dtype=torch.float32, device="cuda:0")
        for sd in seeds:
            p.seed = sd
            st = ds.render_tiles(ids, T, T, buf.data_ptr(), p)
            single.append(buf.cpu().numpy().copy())
            rays += st.rays
        # (pixels of edge tiles outside the image are left untouched: zero in both buffers)
        multi = torch.zeros(len(seeds) * n, dtype=torch.float32, device="cuda:0")
        p.seed = 12345  # not used by rt_render_frames
        st = ds.render_frames(seeds, ids, T, T, multi.data_ptr(), p)
        got = multi.cpu().numpy().reshape(len(seeds), n)
        for f in range(len(seeds)):
            bad = int((got[f].view(np.uint32) != single[f].view(np.uint32)).sum())
            assert bad == 0, f"frame {f} (seed {seeds[f]}): {bad} channels differ from its single-frame call"
        assert st.rays == rays, (st.rays, rays)
        return st, got
    finally:
        ds.close()
        sc.close()
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("name", ["soup_lit", "shapes_thin_lens", "soup_edge", "features_steps"])
def test_frames_equal_single_frames(name, tmp_path, gpu):
    sc, spp_sqrt = _case_scene(name)
    path = scenes.write(sc, str(tmp_path / f"{name}.json"))
    info = rt.Scene(path, texture_root=scenes.TEXTURES)
    W, H = info.width, info.height
    info.close()
    tx, ty = -(-W // T), -(-H // T)
    ids = np.arange(tx * ty, dtype=np.int32)
    seeds = [7, 8, 1 << 40, 20251226]
    ls = 2 if name == "features_steps" else 1
    st, got = _frames_vs_single(path, spp_sqrt, ids, seeds, light_samples=ls)
    assert st.path == (rt.PATH_STEPS if name == "features_steps" else rt.PATH_ONE_PASS)
    if name != "features_steps":  # one launch for all the frames
        assert st.iterations == 1
    # the last frame against the oracle directly
    ref, _, _ = ob.render(path, rng=ob.RNG_COUNTER, seed=seeds[-1], spp_sqrt=spp_sqrt, light_samples=ls,
                          use_bvh=True, texture_root=scenes.TEXTURES)
    img = rt.unpack_tiles(got[-1], ids, T, T, W, H)
    assert int((img.view(np.uint32) != ref.view(np.uint32)).sum()) == 0


def test_rank_share_frames(tmp_path, gpu):
    """A rank-like share (every third tile of a 4 x 3 grid, costliest first inside the call) in
    8 frames per call, and the same frames split over passes of 3 frames and of single tiles
    (RT_ONE_PASS_MAX)."""
    path = scenes.write(scenes.soup(4000, seed=9, res=(128, 96)), str(tmp_path / "s.json"))
    ids = np.array([2, 5, 8, 11], dtype=np.int32)
    seeds = list(range(300, 308))
    st, _ = _frames_vs_single(path, 3, ids, seeds)
    assert st.iterations == 1 and st.path == rt.PATH_ONE_PASS
    per_frame = ids.size * T * T * 9
    st, _ = _frames_vs_single(path, 3, ids, seeds, env={"RT_ONE_PASS_MAX": str(3 * per_frame)})
    assert st.iterations == 3  # passes of 3 + 3 + 2 frames
    st, _ = _frames_vs_single(path, 3, ids, seeds[:3], env={"RT_ONE_PASS_MAX": str(T * T * 9)})
    assert st.iterations == 3 * ids.size  # one tile per pass


def test_frames_arguments(tmp_path, gpu):
    import torch
    path = scenes.write(scenes.soup(500, seed=3, res=(32, 32)), str(tmp_path / "a.json"))
    sc = rt.Scene(path)
    ds = rt.DeviceScene(sc, 0)
    try:
        buf = torch.zeros(4 * T * T * 3, dtype=torch.float32, device="cuda:0")
        p = rt.RenderParams(spp_sqrt=1)
        with pytest.raises(rt.NativeError, match="frames"):
            ds.render_frames([], [0], T, T, buf.data_ptr(), p)
        with pytest.raises(rt.NativeError, match="count_work"):
            ds.render_frames([1, 2], [0], T, T, buf.data_ptr(), rt.RenderParams(spp_sqrt=1, count_work=True))
        st = ds.render_frames([5], [0], T, T, buf.data_ptr(), p)  # one frame: seed 5, not params.seed
        one = buf[:T * T * 3].cpu().numpy().copy()
        p.seed = 5
        ds.render_tiles([0], T, T, buf.data_ptr(), p)
        assert np.array_equal(one.view(np.uint32), buf[:T * T * 3].cpu().numpy().view(np.uint32)) and st.rays > 0
    finally:
        ds.close()
        sc.close()
