"""Fused shadow rays (trace_refill_kernel<.., kFuse>): in a scene lit by point lights only
(planes, or untextured transformed shapes), the lane that finds a closest hit traces its
lights' shadow rays right after it and leaves occlusion bits for the logic step.  Fused and unfused renders must both match the
oracle bit for bit (and in ray count): with reflection, refraction and glossy fuzz after the
shade (raytracer.cpp:180-350), in BVH and linear modes, and with 24 lights (the last bit of the
occlusion word).  RT_FUSE is read per call, so each setting renders in a child process like
the other knobs (tests/test_gpu_knobs.py); RT_ONE_PASS=0 keeps the point-lit planes scenes,
one-pass otherwise (tests/test_gpu_one_pass.py), on the step pipeline whose fusion this tests."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_bind as ob
import scenes

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import ray_tracying_amd as rt
sc = rt.Scene(sys.argv[2], texture_root=sys.argv[7])
img, st = sc.render(rt.RenderParams(spp_sqrt=int(sys.argv[4]), light_samples=int(sys.argv[6]), use_bvh=sys.argv[5] == "1",
                                    seed=9))
np.save(sys.argv[3], img)
print(st.rays)
"""


def render_child(path, out, spp, bvh, fuse, light_samples=1, env=None):
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, path, out, str(spp), "1" if bvh else "0", str(light_samples),
                        scenes.TEXTURES], env={**os.environ, "RT_ONE_PASS": "0", "RT_FUSE": fuse, **(env or {})},
                       capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(out), int(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("bvh", [True, False])
def test_fused_shadows_match_oracle(tmp_path, gpu, bvh):
    p = scenes.write(scenes.planes_lit(), str(tmp_path / "p.json"))
    ref, _, ost = ob.render(p, rng=ob.RNG_COUNTER, seed=9, spp_sqrt=2, light_samples=1, use_bvh=bvh)
    for fuse in ("1", "0"):
        img, rays = render_child(p, str(tmp_path / f"img{fuse}.npy"), 2, bvh, fuse)
        diff = int((img.view(np.uint32) != ref.view(np.uint32)).sum())
        assert diff == 0, f"RT_FUSE={fuse}: {diff} channels differ"
        assert rays == ost["rays"], fuse


def point_lit_features():
    """features() (spheres incl. a moving one, cubes, rectangles, planes; mirror, glass, glossy)
    with point lights and no textures: the fused path for transformed shapes, whose hit
    record the tracing lane computes (prim_hit with attributes) before the shadow rays."""
    sc = scenes.features(res=(40, 32))
    for light in sc["lights"]:
        light["radius"] = 0.0
    for k in ("spheres", "cubes", "rectangles", "planes"):
        for o in sc.get(k, []):
            if isinstance(o.get("material"), dict):
                o["material"].pop("texture_file", None)
    return sc


@pytest.mark.parametrize("bvh", [True, False])
def test_fused_shadows_transformed_shapes(tmp_path, gpu, bvh):
    p = scenes.write(point_lit_features(), str(tmp_path / "f.json"))
    ref, _, ost = ob.render(p, rng=ob.RNG_COUNTER, seed=9, spp_sqrt=2, light_samples=1, use_bvh=bvh)
    for fuse in ("1", "0"):
        img, rays = render_child(p, str(tmp_path / f"img{fuse}.npy"), 2, bvh, fuse)
        diff = int((img.view(np.uint32) != ref.view(np.uint32)).sum())
        assert diff == 0, f"RT_FUSE={fuse}: {diff} channels differ"
        assert rays == ost["rays"], fuse


def test_fused_24_lights(tmp_path, gpu):
    p = scenes.write(scenes.planes_lit(n=150, res=(24, 16), n_lights=24), str(tmp_path / "p24.json"))
    ref, _, ost = ob.render(p, rng=ob.RNG_COUNTER, seed=9, spp_sqrt=1, light_samples=1, use_bvh=True)
    img, rays = render_child(p, str(tmp_path / "img.npy"), 1, True, "1")
    assert int((img.view(np.uint32) != ref.view(np.uint32)).sum()) == 0
    assert rays == ost["rays"]


def test_fused_textured_planes(tmp_path, gpu):
    """Fused shadows on textured planes: the closest hit's (u, v) go to the uv array."""
    sc = scenes.planes_lit()
    for k, pl in enumerate(sc["planes"]):
        if k % 3 == 0:
            pl["material"]["texture_file"] = "checker.jpg"
    p = scenes.write(sc, str(tmp_path / "t.json"))
    ref, _, ost = ob.render(p, rng=ob.RNG_COUNTER, seed=9, spp_sqrt=2, light_samples=1, use_bvh=True,
                            texture_root=scenes.TEXTURES)
    for fuse in ("1", "0"):
        img, rays = render_child(p, str(tmp_path / f"img{fuse}.npy"), 2, True, fuse)
        assert int((img.view(np.uint32) != ref.view(np.uint32)).sum()) == 0, fuse
        assert rays == ost["rays"], fuse


@pytest.mark.parametrize("start", ["1", "0"])
def test_soft_samples_in_lane_planes(tmp_path, gpu, start):
    """Soft-light samples drawn and traced by the tracing lane on a planes-only scene (kSoft),
    the first one started by the closest hit itself or by the logic step (RT_SOFT_START)."""
    sc = scenes.planes_lit(n_lights=2)
    sc["lights"][0]["radius"] = 0.4
    p = scenes.write(sc, str(tmp_path / "s.json"))
    ref, _, ost = ob.render(p, rng=ob.RNG_COUNTER, seed=9, spp_sqrt=2, light_samples=3, use_bvh=True)
    img, rays = render_child(p, str(tmp_path / "img.npy"), 2, True, "1", light_samples=3,
                             env={"RT_SOFT_START": start})
    assert int((img.view(np.uint32) != ref.view(np.uint32)).sum()) == 0
    assert rays == ost["rays"]


def _reflective_scenes():
    """Reflective scenes lit by one soft light: C4's glossy_reflection (metal spheres of roughness
    0 / 0.2 / 0.5, a diffuse cube, a slightly reflective floor), the mirror corridor without its
    glass cube (chains to MAX_RECURSION_DEPTH, raytracer.hpp:11) and a planes-only soup of mirror
    / glossy / diffuse triangles."""
    c4 = scenes.blend("glossy_reflection", (40, 32), light_radius=1.0)
    corridor = scenes.mirror_corridor()
    corridor["cubes"][0]["material"] = {"diffuse_color": [0.8, 0.9, 1.0], "reflectivity": 0.3, "roughness": 0.1}
    planes = scenes.planes_lit(n_lights=1)
    for pl in planes["planes"]:
        pl["material"]["transparency"] = 0.0
    planes["lights"][0]["radius"] = 0.4
    return {"c4": c4, "corridor": corridor, "planes": planes}


@pytest.mark.parametrize("name", ["c4", "corridor", "planes"])
def test_reflection_chains_soft_light(tmp_path, gpu, name):
    """Reflection chains under a soft light (Code/raytracer.cpp:180-274 shade, :303-331 Trace's
    reflection): the tracing lane draws and traces every soft sample of a hit, the first started
    by the closest hit itself or by the logic step (RT_SOFT_START) -- every float and the ray count
    equal to the oracle's.  (r05: continuing the chain itself in the lane -- shade and reflection
    ray -- was measured 34 % slower on C4 and is not built)"""
    p = scenes.write(_reflective_scenes()[name], str(tmp_path / f"{name}.json"))
    ref, _, ost = ob.render(p, rng=ob.RNG_COUNTER, seed=9, spp_sqrt=2, light_samples=3, use_bvh=True)
    for start in ("1", "0"):
        img, rays = render_child(p, str(tmp_path / f"img{start}.npy"), 2, True, "1", light_samples=3,
                                 env={"RT_SOFT_START": start})
        assert int((img.view(np.uint32) != ref.view(np.uint32)).sum()) == 0, start
        assert rays == ost["rays"], start
