"""Scene fixtures for the parity tests.

* ``ascii(...)``      -- the reference's own input scene (/root/reference/ASCII/scene.json,
  committed as data under tests/golden/scenes/ascii_scene.json: 140 cubes + 1 rectangle +
  2 lights), with the edits the survey's known-answer tests use (SURVEY.md section 4:
  K1 = roughness 0, K4 = primary-only).
* ``features(...)``   -- a hand-written scene that exercises every primitive kind and every
  feature of the hot path: mirror / glass (refraction + TIR) / glossy spheres, a moving
  (motion-blurred) ellipsoid, rotated cubes (one with default material), a reflective
  floor rectangle, a textured quad plane and two triangles (planes with c3 == c0), a hard
  and a soft (radius > 0) light, optional thin-lens depth of field.
* ``soup(...)``       -- a seeded triangle soup written as ``planes`` with c3 == c0.
* ``blend(name, ...)`` -- the reference's own Blender scenes (/root/reference/Blend/*.blend),
  exported by tools/blend_export.py (byte-identical to the reference exporter's output on
  Test2.blend -> ASCII/scene.json) and committed under tests/golden/scenes/blend/: the
  BASELINE configs C3 (Antialiasing) and C4 (glossy_reflection + soft shadows), and the DOF,
  motion-blur, soft-shadow and sphere scenes, at small resolutions.
Scenes are plain dicts; ``write(scene, path)`` dumps JSON whose floats round-trip exactly.
"""
from __future__ import annotations

import copy
import json
import os
import random

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ASCII_PATH = os.path.join(GOLDEN, "scenes", "ascii_scene.json")
TEXTURES = os.path.join(GOLDEN, "textures") + os.sep


def write(scene: dict, path: str) -> str:
    with open(path, "w") as f:
        json.dump(scene, f, indent=1)
    return path


def ascii(res=(64, 64), roughness=None, primary_only=False, texture=None) -> dict:
    with open(ASCII_PATH) as f:
        s = json.load(f)
    s["render"] = {"resolution_x": res[0], "resolution_y": res[1]}
    for k in ("cubes", "rectangles"):
        for o in s.get(k, []):
            m = o["material"]
            if roughness is not None:
                m["roughness"] = roughness
            if primary_only:
                m["reflectivity"] = 0.0
                m["transparency"] = 0.0
            if texture is not None:
                m["texture_file"] = texture
    if primary_only:
        s["lights"] = []
    return s


def features(res=(64, 48), aperture=0.0, focus=6.0, soft_radius=0.5, texture="checker.jpg") -> dict:
    def mat(**kw):
        m = {"diffuse_color": [0.7, 0.7, 0.7], "specular_color": [1.0, 1.0, 1.0], "roughness": 0.2,
             "k_ambient": 0.1, "k_diffuse": 0.6, "k_specular": 0.4, "reflectivity": 0.0,
             "transparency": 0.0, "refractive_index": 1.0}
        m.update(kw)
        return m

    return {
        "cameras": [{"location": [0.3, -6.0, 2.2], "gaze_vector": [0.0, 1.0, -0.28],
                     "up_vector": [0.0, 0.28, 1.0], "focal_length": 35.0, "sensor_width": 36.0,
                     "sensor_height": 24.0, "aperture": aperture, "focus_dist": focus}],
        "render": {"resolution_x": res[0], "resolution_y": res[1]},
        "lights": [
            {"location": [4.0, -4.0, 6.0], "intensity": 800.0, "color": [1.0, 0.9, 0.8], "radius": 0.0},
            {"location": [-3.0, -2.0, 5.0], "intensity": 500.0, "color": [0.6, 0.7, 1.0], "radius": soft_radius},
            {"location": [0.0, 0.0, 9.0], "intensity": -5.0, "color": [1, 1, 1]},   # skipped: intensity <= 0
            {"location": [0.0, 0.0, 9.0], "color": [1, 1, 1]},                       # skipped: no intensity
        ],
        "spheres": [
            {"location": [-1.3, 0.2, 0.85], "radius": 0.8,
             "material": mat(diffuse_color=[0.9, 0.9, 0.95], reflectivity=0.85, roughness=0.0)},
            {"location": [1.0, -0.6, 0.7], "radius": 0.7,
             "material": mat(diffuse_color=[0.8, 1.0, 0.9], transparency=0.85, refractive_index=1.5,
                             reflectivity=0.1, roughness=0.0)},
            {"location": [0.1, 1.6, 0.6], "rotation": [0.3, 0.2, 0.1], "scale": [0.5, 0.7, 0.45],
             "velocity": [1.5, 0.0, 0.5],
             "material": mat(diffuse_color=[0.2, 0.4, 0.9], reflectivity=0.3, roughness=0.3)},
            {"location": [-0.4, -1.8, 0.35], "radius": 0.35},                       # default Material()
        ],
        "cubes": [
            {"translation": [2.3, 1.0, 0.6], "rotation": [0.4, 0.2, 0.7], "scale": [0.8, 0.6, 1.0],
             "material": mat(diffuse_color=[0.9, 0.2, 0.1], roughness=0.5)},
            {"translation": [-2.4, 1.4, 0.5], "rotation": [0.0, 0.0, 0.6], "scale": 0.9},
            {"translation": [0.0, 0.0, 9.0]},                                        # skipped: no rotation
        ],
        "rectangles": [
            {"translation": [0.0, 0.0, 0.0], "rotation": [0.0, 0.0, 0.0], "scale": [12.0, 12.0, 1.0],
             "material": mat(diffuse_color=[0.6, 0.6, 0.55], reflectivity=0.25, roughness=0.05)},
        ],
        "planes": [
            {"corners": [[-3.0, 3.0, 0.01], [-1.0, 3.0, 0.01], [-1.0, 3.0, 2.0], [-3.0, 3.0, 2.0]],
             "material": mat(diffuse_color=[1.0, 1.0, 1.0], texture_file=texture)},
            {"corners": [[1.4, 2.6, 0.02], [2.9, 2.2, 0.02], [2.0, 2.4, 1.9], [1.4, 2.6, 0.02]],
             "material": mat(diffuse_color=[0.95, 0.8, 0.2], reflectivity=0.2)},
            {"corners": [[-0.5, 2.8, 1.4], [0.6, 2.9, 1.6], [0.0, 3.0, 2.6], [-0.5, 2.8, 1.4]]},
            {"corners": [[0, 0, 0], [1, 1, 1], [2, 2, 2]]},                          # skipped: 3 corners
        ],
    }


def soup(n=200, seed=5, res=(48, 48), light=True) -> dict:
    rnd = random.Random(seed)
    s = n ** (-1.0 / 3.0)
    planes = []
    for _ in range(n):
        c = [rnd.uniform(-1, 1) for _ in range(3)]
        v = [[c[k] + rnd.uniform(-s, s) for k in range(3)] for _ in range(3)]
        planes.append({"corners": [v[0], v[1], v[2], v[0]]})
    return {
        "cameras": [{"location": [0.0, -4.0, 0.0], "gaze_vector": [0.0, 1.0, 0.0], "up_vector": [0.0, 0.0, 1.0],
                     "focal_length": 35.0, "sensor_width": 36.0, "sensor_height": 36.0}],
        "render": {"resolution_x": res[0], "resolution_y": res[1]},
        "lights": [{"location": [2.0, -3.0, 3.0], "intensity": 600.0, "color": [1.0, 1.0, 1.0], "radius": 0.0}]
        if light else [],
        "planes": planes,
    }


def planes_lit(n=400, seed=17, res=(40, 32), n_lights=3) -> dict:
    """A planes-only scene (the trace kernel's fused shadow-ray case) with point lights only:
    a soup whose triangles cycle through a mirror, a glass (refraction, total internal
    reflection), a glossy (random fuzz draws after the shadow rays) and a plain diffuse
    material, lit by `n_lights` point lights around and inside the soup."""
    sc = soup(n, seed=seed, res=res)
    mats = [{"diffuse_color": [0.9, 0.9, 0.9], "reflectivity": 0.9, "roughness": 0.0, "k_ambient": 0.05},
            {"diffuse_color": [0.8, 0.9, 1.0], "transparency": 0.85, "refractive_index": 1.5, "reflectivity": 0.1},
            {"diffuse_color": [0.2, 0.4, 0.9], "reflectivity": 0.4, "roughness": 0.3},
            {"diffuse_color": [0.9, 0.3, 0.2]}]
    for k, pl in enumerate(sc["planes"]):
        pl["material"] = dict(mats[k % len(mats)])
    rnd = random.Random(seed + 1)
    sc["lights"] = [{"location": [rnd.uniform(-2.5, 2.5), rnd.uniform(-3.5, 1.5), rnd.uniform(-2.5, 2.5)],
                     "intensity": 200.0 + 20.0 * i, "color": [1.0, 0.9 - 0.01 * i, 0.8], "radius": 0.0}
                    for i in range(n_lights)]
    return sc


def soup_degenerate(n=300, seed=13, res=(48, 48), every=7) -> dict:
    """A soup in which every `every`-th plane repeats its third corner (c3 == c2): the
    reference's trap (shapes.cpp:485-494) -- the degenerate sub-triangle
    (c1, c2, c2) accepts a thin band along the infinite line c1c2 that only the reference's
    leaf AABB clips, so -bvh and linear disagree and the kernel's unbounded-primitive list is
    non-empty.  Every `every`-th other plane is a true quad (parallelogram c0, c1, c2, c0+c2-c1)."""
    sc = soup(n, seed=seed, res=res)
    for k, pl in enumerate(sc["planes"]):
        c = pl["corners"]
        if k % every == 0:
            c[3] = list(c[2])
        elif k % every == 3:
            c[3] = [c[0][i] + c[2][i] - c[1][i] for i in range(3)]
    return sc


def sphere_textured(res=(48, 40)) -> dict:
    """features() with the checker texture on the spheres (UV from double atan2 / asin,
    shapes.cpp:257-259; material.hpp:99-134) and on a cube."""
    sc = features(res=res)
    for o in sc["spheres"] + sc["cubes"][:1]:
        if "material" in o:
            o["material"]["texture_file"] = "checker.jpg"
    return sc


# name -> (scene builder, CLI-equivalent render args).  These are the golden-vector cases.
def blend(name: str, res=(48, 32), light_radius=None) -> dict:
    with open(os.path.join(GOLDEN, "scenes", "blend", name + ".json")) as f:
        s = json.load(f)
    s["render"] = {"resolution_x": res[0], "resolution_y": res[1]}
    if light_radius is not None:  # soft shadows via light radius > 0
        for light in s["lights"]:
            light["radius"] = light_radius
    return s


def cases() -> dict:
    return {
        "ascii_k1_bvh": (lambda: ascii((64, 64), roughness=0.0), dict(use_bvh=True, spp_sqrt=1, light_samples=1)),
        "ascii_glossy_bvh": (lambda: ascii((48, 48)), dict(use_bvh=True, spp_sqrt=1, light_samples=1)),
        "ascii_glossy_s2_linear": (lambda: ascii((32, 32)), dict(use_bvh=False, spp_sqrt=2, light_samples=1)),
        "ascii_primary": (lambda: ascii((64, 64), primary_only=True), dict(use_bvh=True, spp_sqrt=1, light_samples=1)),
        "ascii_textured": (lambda: ascii((48, 48), texture="checker.jpg"), dict(use_bvh=True, spp_sqrt=1, light_samples=1)),
        "features_s1": (lambda: features(), dict(use_bvh=True, spp_sqrt=1, light_samples=1)),
        "features_s2_ls3": (lambda: features(), dict(use_bvh=True, spp_sqrt=2, light_samples=3)),
        "features_linear": (lambda: features((40, 30)), dict(use_bvh=False, spp_sqrt=1, light_samples=2)),
        "features_dof": (lambda: features(aperture=0.25, focus=5.5), dict(use_bvh=True, spp_sqrt=2, light_samples=1)),
        "soup_s1": (lambda: soup(300, seed=11), dict(use_bvh=True, spp_sqrt=1, light_samples=1)),
        "soup_s3": (lambda: soup(120, seed=3, res=(32, 32)), dict(use_bvh=True, spp_sqrt=3, light_samples=1)),
        "soup_linear": (lambda: soup(80, seed=4, res=(32, 32)), dict(use_bvh=False, spp_sqrt=1, light_samples=1)),
        "soup_c3c2_bvh": (lambda: soup_degenerate(400, seed=13), dict(use_bvh=True, spp_sqrt=2, light_samples=1)),
        "soup_c3c2_linear": (lambda: soup_degenerate(150, seed=14, res=(32, 32)),
                             dict(use_bvh=False, spp_sqrt=1, light_samples=1)),
        "sphere_textured": (lambda: sphere_textured(), dict(use_bvh=True, spp_sqrt=2, light_samples=2)),
        "blend_c3_antialiasing": (lambda: blend("Antialiasing", (64, 48)), dict(use_bvh=True, spp_sqrt=2, light_samples=1)),
        "blend_c4_glossy_soft": (lambda: blend("glossy_reflection", (64, 48), light_radius=1.0),
                                 dict(use_bvh=True, spp_sqrt=2, light_samples=2)),
        # C3 / C4 at the bench's sample settings (-s 10 = 100 spp; C4 -light_sample 4, light radius
        # 1), 128^2: SURVEY.md 8(c) parity chain item (4) at 100 spp
        "blend_c3_s10": (lambda: blend("Antialiasing", (128, 128)), dict(use_bvh=True, spp_sqrt=10, light_samples=1)),
        "blend_c4_s10": (lambda: blend("glossy_reflection", (128, 128), light_radius=1.0),
                         dict(use_bvh=True, spp_sqrt=10, light_samples=4)),
        "blend_dop": (lambda: blend("dop"), dict(use_bvh=True, spp_sqrt=2, light_samples=1)),
        "blend_motion_blur": (lambda: blend("motion_blur"), dict(use_bvh=True, spp_sqrt=2, light_samples=1)),
        "blend_distributed": (lambda: blend("Distributed"), dict(use_bvh=True, spp_sqrt=1, light_samples=2)),
        "blend_test1": (lambda: blend("Test1"), dict(use_bvh=True, spp_sqrt=1, light_samples=1)),
        "blend_test3": (lambda: blend("Test3"), dict(use_bvh=True, spp_sqrt=1, light_samples=1)),
    }


def materialise(name: str, directory: str) -> tuple[str, dict]:
    builder, args = cases()[name]
    return write(copy.deepcopy(builder()), os.path.join(directory, name + ".json")), dict(args)


def mirror_corridor(res=(40, 32)) -> dict:
    """Two facing perfect mirrors + a glass cube (total internal reflection) and a glossy
    sphere: drives the Trace recursion into MAX_RECURSION_DEPTH (raytracer.hpp:11)."""
    mirror = {"diffuse_color": [0.9, 0.9, 0.9], "reflectivity": 0.95, "roughness": 0.0, "k_ambient": 0.05}
    return {
        "cameras": [{"location": [0.0, -1.0, 0.2], "gaze_vector": [0.35, 1.0, 0.05], "up_vector": [0, 0, 1],
                     "focal_length": 30.0, "sensor_width": 36, "sensor_height": 24}],
        "render": {"resolution_x": res[0], "resolution_y": res[1]},
        "lights": [{"location": [0.0, 2.0, 1.5], "intensity": 300.0, "color": [1, 1, 1], "radius": 0.2}],
        "rectangles": [
            {"translation": [-1.0, 2.0, 0.0], "rotation": [0.0, 1.5707963, 0.0], "scale": [4.0, 8.0, 1.0], "material": mirror},
            {"translation": [1.0, 2.0, 0.0], "rotation": [0.0, -1.5707963, 0.0], "scale": [4.0, 8.0, 1.0], "material": mirror},
        ],
        "cubes": [{"translation": [0.2, 3.0, 0.1], "rotation": [0.3, 0.5, 0.2], "scale": [0.5, 0.5, 0.5],
                   "material": {"diffuse_color": [0.8, 0.9, 1.0], "transparency": 0.9, "refractive_index": 2.4,
                                "reflectivity": 0.05}}],
        "spheres": [{"location": [-0.3, 4.0, 0.3], "radius": 0.3,
                     "material": {"reflectivity": 0.5, "roughness": 0.4}}],
    }


def tiny(n_prims=3, res=(21, 13)) -> dict:
    """<= 4 primitives: the reference's BVH root is itself a leaf."""
    s = soup(n_prims, seed=2, res=res)
    s["spheres"] = [{"location": [0.0, 0.0, 0.0], "radius": 0.3}]
    return s


def empty(res=(16, 16)) -> dict:
    return {"cameras": [{"location": [0, -4, 0], "gaze_vector": [0, 1, 0], "up_vector": [0, 0, 1],
                         "focal_length": 35, "sensor_width": 36, "sensor_height": 36}],
            "render": {"resolution_x": res[0], "resolution_y": res[1]},
            "lights": [{"location": [0, 0, 3], "intensity": 100, "color": [1, 1, 1]}]}
