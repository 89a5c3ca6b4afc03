"""The scheduling knobs of the trace / logic kernels never change a result.

Each knob is read once per process (environment), so every configuration renders in a fresh
child process and must match the oracle bit for bit: the LDS traversal stack cut to 2
entries (every deeper entry spills to HBM), extreme refill / leaf-phase thresholds, one and
many work-counter shards, a slot count so small that a frame takes dozens of steps, and the
slots split into two pipelines on two streams, soft-shadow samples advanced by
shadow_step_kernel or by the logic kernel instead of the tracing lane, the greedy BVH4
collapse instead of the SAH-optimal one, point-light shadow rays left unfused in a small
call, two or four slot pipelines instead of the default one, and the tiles rendered in the
caller's order instead of costliest first (small calls' default), and the lanes still
traversing when a launch's queue runs dry left alone instead of helped by the free lanes.
"""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import oracle_bind as ob
import ray_tracying_amd as rt
import scenes

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import ray_tracying_amd as rt
sc = rt.Scene(sys.argv[2], texture_root=sys.argv[4])
img, st = sc.render(rt.RenderParams(spp_sqrt=2, light_samples=2, use_bvh=True, seed=5))
np.save(sys.argv[3], img)
print(st.path)
print(st.rays)
"""

# RT_ONE_PASS=0 runs one-pass scenes (the soup) through the step pipeline, whose knobs the
# entries below exercise; without it a one-pass call ignores the step pipeline's knobs (last
# entries: it must stay one-pass and bit-exact -- VERDICT r04 item 7)
STEPS = {"RT_ONE_PASS": "0"}
KNOBS = [
    {"RT_LDS_STACK": "2"},
    {"RT_LEAF_MIN": "1", "RT_REFILL": "64"},
    {"RT_LEAF_MIN": "64", "RT_REFILL": "1"},
    {"RT_BATCH_SHARDS": "1", "RT_FETCH_SHARDS": "64", "RT_SLOTS": "4096", **STEPS},
    {"RT_BATCH_SHARDS": "1024", "RT_FETCH_SHARDS": "1"},
    {"RT_BATCH_SHARDS": "1024", "RT_SLOTS": "4096", **STEPS},  # more shards than slot-waves: clamped
    {"RT_MAX_UNITS": "3000"},  # the call runs as many tile chunks
    {"RT_PIPES": "2", "RT_SLOTS": "4096", "RT_BATCH_SHARDS": "64", **STEPS},
    {"RT_SOFT_START": "0"},  # a closest hit's first shadow sample emitted by the logic step
    {"RT_SOFT_FUSE": "0"},  # soft-shadow samples advanced by shadow_step_kernel, not the tracing lane
    {"RT_SOFT_FUSE": "0", "RT_SHADOW_STEP": "0"},  # ... or by the logic kernel itself
    {"RT_COLLAPSE": "greedy"},  # the round-1 BVH2 -> BVH4 collapse instead of the SAH-optimal one
    {"RT_FUSE": "0", **STEPS},  # point-light shadow rays as their own queries (small calls fuse them by default)
    {"RT_PIPES": "2", **STEPS},  # two slot pipelines on two streams (the default is one)
    {"RT_TILE_ORDER": "0"},  # tiles in the caller's order (small calls render costliest tiles first)
    {"RT_PIPES": "4", "RT_SLOTS": "8192", **STEPS},  # four pipelines of two slot blocks each
    {"RT_DRAIN_HELP": "0"},  # no drain helpers: each query traversed by its own lane alone
    {"RT_DRAIN_HELP": "1", "RT_LDS_STACK": "2", "RT_LEAF_MIN": "1"},  # helpers take entries from the HBM spill area
    {"RT_DRAIN_HELP": "0", **STEPS},  # the step pipeline without helpers
    {"RT_TRACE_SEVEN": "1"},  # the 7-wave planes instances (whole frames' default) on a small call
    {"RT_TRACE_SEVEN": "1", **STEPS},  # ... through the step pipeline (fused shadows: the soup is small)
    {"RT_XCD_CHUNK": "0"},  # the round-robin deal of the work queue (group g to shard g % 32)
    {"RT_XCD_CHUNK": "4", **STEPS},  # the smallest XCD chunks, through the step pipeline
    {"RT_XCD_CHUNK": "100000"},  # one chunk larger than the call: one XCD's shards, the rest stolen
    {"RT_XCD_CHUNK": "1048576"},  # the clamp bound (2^20 groups per chunk)
    {"RT_COMPACT_HIT": "0"},  # one-pass planes calls store the 32-B hit record instead of the hit's t
    {"RT_FLAT_PRIMS": "127"},  # scenes of <= 127 primitives (features) test them all from one leaf item
    {"RT_FLAT_PRIMS": "127", **STEPS},  # ... through the step pipeline (the logic step answers its own queries)
    {"RT_FLAT_PRIMS": "127", "RT_FLAT_RENDER": "0"},  # ... every query through the traversal launches
    {"RT_FLAT_PRIMS": "127", "RT_FLAT_RENDER": "0", **STEPS},
    # step-pipeline knobs on a one-pass scene: ignored (one message each), still one-pass
    {"RT_FUSE": "1"},
    {"RT_FUSE": "0", "RT_SLOTS": "4096", "RT_PIPES": "2", "RT_DIAG": "1"},
]


def _untextured(sc):
    """features() without its textures: the step pipeline's untextured logic instances, whose
    few-primitive form (RT_FLAT_PRIMS=127 here) answers its own queries (kInline, r06)."""
    for kind in ("spheres", "cubes", "rectangles", "planes"):
        for o in sc.get(kind, []):
            if o.get("material"):
                o["material"].pop("texture_file", None)
    return sc


@pytest.mark.parametrize("scene", ["soup", "features", "features_untextured"])
def test_knobs_do_not_change_results(scene, tmp_path, gpu):
    if scene == "soup":
        p = scenes.write(scenes.soup(3000, seed=11, res=(48, 48)), str(tmp_path / "s.json"))
    elif scene == "features":  # reflection, refraction, soft shadows, textures, every primitive kind
        p = scenes.write(scenes.features(res=(40, 32)), str(tmp_path / "f.json"))
    else:
        p = scenes.write(_untextured(scenes.features(res=(40, 32))), str(tmp_path / "fu.json"))
    ref, _, ost = ob.render(p, rng=ob.RNG_COUNTER, seed=5, spp_sqrt=2, light_samples=2, use_bvh=True,
                            texture_root=scenes.TEXTURES)
    for i, env in enumerate(KNOBS):
        out = str(tmp_path / f"img{i}.npy")
        r = subprocess.run([sys.executable, "-c", CHILD, ROOT, p, out, scenes.TEXTURES],
                           env={**os.environ, **env}, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (env, r.stderr[-2000:])
        img = np.load(out)
        diff = int((img.view(np.uint32) != ref.view(np.uint32)).sum())
        assert diff == 0, f"{env}: {diff} channels differ"
        path, rays = map(int, r.stdout.strip().splitlines()[-2:])
        assert rays == ost["rays"], env
        one_pass_scene = scene == "soup"  # features: reflection, refraction, soft lights -> steps
        assert path == (rt.PATH_ONE_PASS if one_pass_scene and "RT_ONE_PASS" not in env else rt.PATH_STEPS), env
        if one_pass_scene and "RT_ONE_PASS" not in env:  # an ignored knob says so once
            for k in ("RT_SLOTS", "RT_PIPES", "RT_FUSE", "RT_DIAG"):
                if k in env:
                    assert f"librt_hip: {k} applies to the step pipeline only" in r.stderr, (env, k)


def test_seven_wave_unfused_instance(tmp_path, gpu):
    """the non-fused 7-wave planes instance (trace_refill_kernel<false, true, false,
    false, true, true>) -- production launches it for light-less whole frames and for step-pipeline
    planes calls whose shadows are not fused -- through the step pipeline with RT_FUSE=0 and
    RT_TRACE_SEVEN=1, on a 60K-triangle soup whose tree is deeper than the instance's 11 LDS rows
    (entries past them go to the HBM spill area), and a light-less soup through the one-pass path;
    the instance log (RT_LOG_INSTANCE) must show the 7-wave unfused launch, and the frame must equal
    the oracle's."""
    cases = [(scenes.soup(60000, seed=31, res=(48, 40)), {"RT_ONE_PASS": "0", "RT_FUSE": "0"}, "steps"),
             (scenes.soup(60000, seed=32, res=(48, 40), light=False), {}, "one-pass")]
    for k, (sc, env, kind) in enumerate(cases):
        p = scenes.write(sc, str(tmp_path / f"deep{k}.json"))
        ref, _, ost = ob.render(p, rng=ob.RNG_COUNTER, seed=5, spp_sqrt=2, light_samples=2, use_bvh=True,
                                texture_root=scenes.TEXTURES)
        out = str(tmp_path / f"deep{k}.npy")
        r = subprocess.run([sys.executable, "-c", CHILD, ROOT, p, out, scenes.TEXTURES],
                           env={**os.environ, **env, "RT_TRACE_SEVEN": "1", "RT_LOG_INSTANCE": "1"},
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        inst = [ln for ln in r.stderr.splitlines() if ln.startswith("[rt instance]")]
        assert inst and all(f"[rt instance] {kind}," in ln for ln in inst), r.stderr[-2000:]
        assert all("waves 7, lds rows 11" in ln and "planes," in ln and "fused" not in ln and "soft" not in ln
                   for ln in inst), inst
        spill = [int(re.search(r"stack bound \d+: (\d+) rows spill", ln).group(1)) for ln in inst]
        assert min(spill) > 0, inst  # the tree's stack bound exceeds the 11 LDS rows
        img = np.load(out)
        assert int((img.view(np.uint32) != ref.view(np.uint32)).sum()) == 0, kind
        assert int(r.stdout.strip().splitlines()[-1]) == ost["rays"]
