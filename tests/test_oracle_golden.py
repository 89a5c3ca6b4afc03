"""The oracle (CPU restatement, oracle/rt_oracle.cpp) against the compiled reference.

Golden vectors were produced by tests/golden/make_golden.py from the reference's own
sources (oracle/_ref/ref_driver: compute_pixel_color/Trace/shade/BVH untouched, serial
std::mt19937 seeded with 42).  In mt19937-serial mode the oracle must reproduce every float
of every framebuffer, the P3 bytes, and the reference's ray / AABB-test counts exactly.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_bind as ob
import scenes

MANIFEST = json.load(open(os.path.join(scenes.GOLDEN, "manifest.json")))


@pytest.mark.parametrize("name", sorted(MANIFEST["cases"]))
def test_oracle_matches_reference_bit_exact(name, tmp_path):
    case = MANIFEST["cases"][name]
    path, args = scenes.materialise(name, str(tmp_path))
    assert args == case["args"]
    rgb, u8, st = ob.render(path, rng=ob.RNG_MT19937, seed=MANIFEST["seed"], texture_root=scenes.TEXTURES, **args)
    ref = np.fromfile(os.path.join(scenes.GOLDEN, "ref", name + ".f32"), dtype=np.float32).reshape(rgb.shape)
    assert np.array_equal(rgb.view(np.uint32), ref.view(np.uint32)), f"{name}: framebuffer differs from the reference"
    assert hashlib.md5(ob.ppm_bytes(u8)).hexdigest() == case["ppm_md5"]
    assert st["rays"] == case["rays"]
    assert st["box_tests"] == case["box_tests"]


def test_known_answer_k1_k4(tmp_path):
    """deterministic configs, md5 of the untouched reference binary."""
    ka = MANIFEST["known_answer"]
    for key, scene in (("K1", scenes.ascii((256, 256), roughness=0.0)),
                       ("K4", scenes.ascii((1024, 1024), primary_only=True))):
        path = scenes.write(scene, str(tmp_path / f"{key}.json"))
        _, u8, _ = ob.render(path, use_bvh=True, spp_sqrt=1, rng=ob.RNG_COUNTER, seed=1)  # RNG unused here
        assert hashlib.md5(ob.ppm_bytes(u8)).hexdigest() == ka[key]["md5"] == ka[key]["survey_md5"]


def test_bvh_and_linear_agree_on_reference_scenes(tmp_path):
    """on these scenes -bvh == linear (the BVH never drops a hit)."""
    for name in ("features_s1", "soup_s1"):
        path, args = scenes.materialise(name, str(tmp_path))
        a, _, _ = ob.render(path, rng=ob.RNG_COUNTER, seed=3, texture_root=scenes.TEXTURES,
                            **{**args, "use_bvh": True})
        b, _, _ = ob.render(path, rng=ob.RNG_COUNTER, seed=3, texture_root=scenes.TEXTURES,
                            **{**args, "use_bvh": False})
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_counter_rng_partition_independent(tmp_path):
    """Counter mode: a region rendered alone equals the same region of the full frame."""
    path, args = scenes.materialise("features_s2_ls3", str(tmp_path))
    full, _, _ = ob.render(path, rng=ob.RNG_COUNTER, seed=9, texture_root=scenes.TEXTURES, **args)
    part, _, _ = ob.render(path, rng=ob.RNG_COUNTER, seed=9, texture_root=scenes.TEXTURES, region=(8, 5, 20, 11), **args)
    assert np.array_equal(full[5:16, 8:28].view(np.uint32), part.view(np.uint32))


def test_counter_rng_stream():
    """generate_canonical-style draws: in [0,1), deterministic, keyed by (seed, pixel, sample)."""
    lib = ob.lib()
    v = [lib.oracle_counter_draw(7, p, s, n) for p in range(40) for s in range(5) for n in range(6)]
    assert all(0.0 <= x < 1.0 for x in v)
    assert abs(np.mean(v) - 0.5) < 0.05
    assert lib.oracle_counter_draw(7, 3, 1, 2) == lib.oracle_counter_draw(7, 3, 1, 2)
    assert lib.oracle_counter_draw(7, 3, 1, 2) != lib.oracle_counter_draw(8, 3, 1, 2)
    assert lib.oracle_counter_draw(7, 3, 1, 2) != lib.oracle_counter_draw(7, 4, 1, 2)
