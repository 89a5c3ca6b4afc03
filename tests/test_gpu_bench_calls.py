"""Parity of the exact calls bench.py times.

The other full-scale parity tests render a few tiles per call.  The timed calls differ: the
headline step is one one-pass call over all 256 tiles of the 1024^2 x 100 spp frame (104.9M
units, costliest tiles first, their outputs remapped to the caller's order); C5 is one call of
2^30 units over the whole 4096^2 x 64 spp frame (64-bit query offsets, ~56 GB of workspace);
a rank's share of an 8-way split is rendered eight frames per rt_render_frames call (r06; two
frames in flight on two scene handles and streams until r05).  Each test runs bench.py itself (`--dump-frame`: after the timed steps the
frame at --seed is rendered by the same calls -- same frames in flight, issued behind another
frame still in flight -- and saved) and compares it with the oracle (counter RNG) bit for bit
(r05: the C3 and C4 frames as timed too -- C4 on the step pipeline's two slot pipelines):
the whole headline frame and the whole rank share, with equal ray counts (the timed frame with
--steps 1 is the frame at --seed: config.rays_per_step); for C5 a spread of tiles (the whole
frame is ~1.5G rays, hours for the CPU restatement), so its ray count is not compared.

The loop these calls replace: /root/reference/Code/raytracer.cpp:433-476 (compute_pixel_color
per pixel, :18-70); the traversal: Code/acceleration.cpp:67-118.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_bind as ob
import ray_tracying_amd as rt
from ray_tracying_amd import tiles as tl

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 20251226  # bench.py's --seed and soup seed
T = 64


def _soup(tmp_path_factory, res):
    p = str(tmp_path_factory.mktemp(f"soup{res}") / "soup1m.json")
    rt.make_soup(p, 1_000_000, seed=SEED, width=res, height=res)
    return p


@pytest.fixture(scope="module")
def soup1024(tmp_path_factory):
    return _soup(tmp_path_factory, 1024)


def _bench(tmp_path, tag, *args):
    frame = str(tmp_path / f"{tag}.npy")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--pmc-traffic", "",
           "--pmc-valu", "", "--dump-frame", frame, *args]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    return np.load(frame), line


def _compare(img, path, res, spp_sqrt, tiles):
    tiles_x = res // T
    regions = [((t % tiles_x) * T, (t // tiles_x) * T, T, T) for t in tiles]
    ref, ost = ob.render_regions(path, regions, use_bvh=True, spp_sqrt=spp_sqrt, light_samples=1, seed=SEED,
                                 resolution=(res, res))
    for k, t in enumerate(tiles):
        x0, y0 = (t % tiles_x) * T, (t // tiles_x) * T
        got = np.ascontiguousarray(img[y0:y0 + T, x0:x0 + T])
        bad = int((got.view(np.uint32) != ref[k].view(np.uint32)).sum())
        assert bad == 0, f"tile {t}: {bad} channels differ from the oracle"
    return ost["rays"]


def test_headline_frame_as_timed(soup1024, tmp_path, gpu):
    """bench.py's default step: the whole 1024^2 x 100 spp frame, rendered as the last of eight
    frames of one rt_render_frames call (r06: one camera pass, one traversal launch, one shading
    pass for the eight)."""
    img, line = _bench(tmp_path, "head")
    assert line["config"]["frames_in_flight"] == 1 and line["config"]["pipeline"].startswith("one-pass")
    assert line["config"]["frames_per_call"] == 8
    assert np.isfinite(img).all()
    rays = _compare(img, soup1024, 1024, 10, list(range(16 * 16)))
    assert rays == line["config"]["rays_per_step"]


def test_rank_share_as_timed(soup1024, tmp_path, gpu):
    """One rank's share of the 8-way split (rank 7: 32 tiles of the lattice deal) rendered as its
    rank does (r06): 64 frames per rt_render_frames call -- one camera pass, one traversal
    launch of the whole-frame run's size (eight whole frames' samples), one shading pass -- the
    frame at --seed the last of them."""
    img, line = _bench(tmp_path, "em8", "--emulate", "8", "--emulate-rank", "7")
    assert line["config"]["frames_per_call"] == 64 and line["config"]["frames_in_flight"] == 1
    mine = [int(t) for t in tl.assign_tiles(256, 8, 7, 16)]
    assert len(mine) == 32
    done = np.isfinite(img).all(axis=2)
    for t in range(256):  # exactly the share's tiles were rendered
        assert bool(done[(t // 16) * T, (t % 16) * T]) == (t in mine), t
    rays = _compare(img, soup1024, 1024, 10, mine)
    assert rays == line["config"]["rays_per_step"]


def test_c2_frame_as_timed(tmp_path_factory, tmp_path, gpu):
    """C2 as timed (r06): the 1024^2 x 1 spp primary-only soup frame rendered 64 frames per
    rt_render_frames call (small frames: as many as make 64M samples), the frame at --seed the last
    of them; the whole frame against the oracle with an equal ray count."""
    path = str(tmp_path_factory.mktemp("soupc2") / "soup1m.json")
    rt.make_soup(path, 1_000_000, seed=SEED, width=1024, height=1024)
    txt = open(path).read()  # the soup with "lights": [] as bench.py writes it for --primary-only
    i = txt.index('"lights": [')
    j = txt.index("\n", i)
    open(path, "w").write(txt[:i] + '"lights": [],' + txt[j:])
    img, line = _bench(tmp_path, "c2", "--primary-only", "--spp-sqrt", "1")
    assert line["config"]["frames_per_call"] == 64 and line["config"]["pipeline"].startswith("one-pass")
    assert np.isfinite(img).all()
    tiles_x = 1024 // T
    regions = [((t % tiles_x) * T, (t // tiles_x) * T, T, T) for t in range(256)]
    ref, ost = ob.render_regions(path, regions, use_bvh=True, spp_sqrt=1, light_samples=1, seed=SEED,
                                 resolution=(1024, 1024))
    for k, (x0, y0, _, _) in enumerate(regions):
        got = np.ascontiguousarray(img[y0:y0 + T, x0:x0 + T])
        assert int((got.view(np.uint32) != ref[k].view(np.uint32)).sum()) == 0, f"tile {k}"
    assert ost["rays"] == line["config"]["rays_per_step"]


def test_c5_frame_as_timed(tmp_path_factory, tmp_path, gpu):
    """C5 as timed: the whole 4096^2 x 64 spp frame (2^30 units) in one one-pass call; tiles at
    the centre, the corners, the edges and across the soup's silhouette (64 x 64 tile grid)."""
    path = _soup(tmp_path_factory, 4096)
    img, line = _bench(tmp_path, "c5", "--res", "4096", "--spp-sqrt", "8")
    assert line["config"]["pipeline"].startswith("one-pass") and line["config"]["resolution"] == "4096x4096"
    assert np.isfinite(img).all()
    tiles = [32 * 64 + 32, 0, 63, 63 * 64, 63 * 64 + 63, 32 * 64 + 11, 32 * 64 + 52, 11 * 64 + 32, 52 * 64 + 20,
             44 * 64 + 47]
    _compare(img, path, 4096, 8, tiles)


def _scene_as_bench_writes(tmp_path, name, light_radius=None):
    """The scene file bench.py renders for --scene NAME (--light-radius): resolution 1024^2 and
    the light radius set, as bench.py writes it (bench.py:389-401)."""
    src = os.path.join(ROOT, "tests", "golden", "scenes", "blend", name + ".json")
    sc = json.load(open(src))
    sc["render"] = {"resolution_x": 1024, "resolution_y": 1024}
    if light_radius is not None:
        for light in sc.get("lights", []):
            light["radius"] = light_radius
    p = str(tmp_path / (name + "_bench.json"))
    with open(p, "w") as f:
        json.dump(sc, f)
    return src, p


def test_c3_frame_as_timed(tmp_path, gpu):
    """C3 as timed: the whole Antialiasing frame (1024^2 x 100 spp) as the last of eight frames of
    one one-pass rt_render_frames call over all 256 tiles (transformed shapes: byte-code nodes,
    fused point-light shadows in the tracing lane, the hit recomputed by the shading); the cube's
    faces and silhouette and the lit floor against the oracle."""
    src, path = _scene_as_bench_writes(tmp_path, "Antialiasing")
    img, line = _bench(tmp_path, "c3", "--scene", src)
    assert line["config"]["pipeline"].startswith("one-pass, few primitives") and line["config"]["frames_in_flight"] == 1
    assert line["config"]["frames_per_call"] == 8 and line["roofline"]["kernel"] == "flat_render_kernel"
    assert np.isfinite(img).all()
    _compare(img, path, 1024, 10, [9 * 16 + 7, 12 * 16 + 6, 7 * 16 + 6, 3 * 16 + 12, 0, 255])


def test_c4_frame_as_timed(tmp_path, gpu):
    """C4 as timed: the whole glossy_reflection frame (light radius 1.0, -light_sample 4) on the
    step pipeline with its defaults for scenes with Trace frames -- two slot pipelines on two
    streams, 8M slots between them, and (five primitives, r06) the logic step answering every
    query itself, ~13 steps per pipeline and no traversal launch; tiles over the spheres, the cube
    and their reflections against the oracle."""
    src, path = _scene_as_bench_writes(tmp_path, "glossy_reflection", light_radius=1.0)
    img, line = _bench(tmp_path, "c4", "--scene", src, "--light-radius", "1.0", "--light-samples", "4")
    assert line["config"]["pipeline"].startswith("steps, few primitives")  # the logic step answers its queries
    assert np.isfinite(img).all()
    tiles_x = 16
    regions = [((t % tiles_x) * T, (t // tiles_x) * T, T, T) for t in [14 * 16 + 7, 10 * 16 + 4, 11 * 16 + 12, 7 * 16 + 9]]
    ref, _ = ob.render_regions(path, regions, use_bvh=True, spp_sqrt=10, light_samples=4, seed=SEED,
                               resolution=(1024, 1024))
    for k, (x0, y0, _, _) in enumerate(regions):
        got = np.ascontiguousarray(img[y0:y0 + T, x0:x0 + T])
        bad = int((got.view(np.uint32) != ref[k].view(np.uint32)).sum())
        assert bad == 0, f"region {regions[k]}: {bad} channels differ from the oracle"


def test_step_pipeline_scene_frames_in_flight(tmp_path, gpu):
    """frames in flight on a step-pipeline scene (C4's glossy reflection with soft
    lights).  Its calls complete before returning, so by default bench.py keeps one frame in
    flight; forced to two, every frame's statistics still reach the line (DeviceScene.wait hands
    out the held stats) -- never a silent 0 Mrays/s -- and the frame is the same."""
    scene = os.path.join(ROOT, "tests", "golden", "scenes", "blend", "glossy_reflection.json")
    common = ("--scene", scene, "--res", "128", "--spp-sqrt", "2", "--light-radius", "1.0", "--light-samples", "2")
    auto_img, auto = _bench(tmp_path, "c4auto", *common)
    assert auto["config"]["frames_in_flight"] == 1 and auto["config"]["pipeline"].startswith("steps")
    two_img, two = _bench(tmp_path, "c4two", *common, "--frames-in-flight", "2")
    assert two["config"]["frames_in_flight"] == 2
    assert two["value"] > 0 and two["config"]["rays_per_step"] == auto["config"]["rays_per_step"] > 0
    assert int((auto_img.view(np.uint32) != two_img.view(np.uint32)).sum()) == 0
