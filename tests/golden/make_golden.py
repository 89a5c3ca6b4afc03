#!/usr/bin/env python3
"""Generate the golden vectors from the COMPILED REFERENCE (run here, where /root/reference
exists; the outputs are committed, the reference is not).

For every case in tests/scenes.py:cases() this writes the scene JSON to a scratch tree laid
out like the reference expects (X/Code/build = cwd, X/Textures/ holds the test texture),
runs oracle/_ref/ref_driver -- the reference's own compute_pixel_color/Trace/shade/BVH code,
serial std::mt19937 seeded with SEED -- and stores:
  tests/golden/ref/<case>.f32   linear float RGB framebuffer (pre-gamma), row-major
  tests/golden/ref/<case>.md5   md5 of the reference's P3 image bytes
  tests/golden/manifest.json    args, sizes, ray / AABB-test counts
It also runs the unmodified reference binary (oracle/_ref/Raytracer, main() untouched) on
the survey's deterministic known-answer configs K1 (256^2) and K4 (1024^2) and records the
md5 of its output next to the survey's published value.

usage: python tests/golden/make_golden.py   (after `make ref`)
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import scenes  # noqa: E402

SEED = 42
REF_DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "Raytracer")
SURVEY_MD5 = {"K1": "a9620c1ca16d531329760ed7a855f0e6", "K4": "a442c6561ac94d5db981ac01745b0405"}


def main():
    for p in (REF_DRIVER, REF_BIN):
        if not os.path.exists(p):
            sys.exit(f"{p} missing: run `make ref` first")
    out_dir = os.path.join(HERE, "ref")
    os.makedirs(out_dir, exist_ok=True)
    manifest = {"seed": SEED, "generator": "oracle/_ref/ref_driver (reference sources, serial mt19937)",
                "cases": {}, "known_answer": {}}
    with tempfile.TemporaryDirectory() as tmp:
        build = os.path.join(tmp, "Code", "build")
        os.makedirs(build)
        os.makedirs(os.path.join(tmp, "ASCII"))
        os.makedirs(os.path.join(tmp, "Output"))
        shutil.copytree(os.path.join(HERE, "textures"), os.path.join(tmp, "Textures"))
        for name in scenes.cases():
            path, args = scenes.materialise(name, os.path.join(tmp, "ASCII"))
            cmd = [REF_DRIVER, "-input", path, "-s", str(args["spp_sqrt"]), "-light_sample", str(args["light_samples"]),
                   "-seed", str(SEED), "-float-out", os.path.join(out_dir, name + ".f32"),
                   "-ppm-out", os.path.join(tmp, name + ".ppm")]
            if args["use_bvh"]:
                cmd.append("-bvh")
            r = subprocess.run(cmd, cwd=build, capture_output=True, text=True, check=True)
            stats = json.loads(r.stdout.strip().splitlines()[-1])
            md5 = hashlib.md5(open(os.path.join(tmp, name + ".ppm"), "rb").read()).hexdigest()
            with open(os.path.join(out_dir, name + ".md5"), "w") as f:
                f.write(md5 + "\n")
            manifest["cases"][name] = {"args": args, "width": stats["width"], "height": stats["height"],
                                       "rays": stats["rays"], "box_tests": stats["box_tests"],
                                       "n_shapes": stats["n_shapes"], "n_lights": stats["n_lights"], "ppm_md5": md5}
            print(name, stats["width"], stats["height"], stats["rays"], md5)
        # K1 / K4 with the untouched reference main() (deterministic: no RNG effect)
        for key, scene, args in (("K1", scenes.ascii((256, 256), roughness=0.0), ["-bvh", "-s", "1"]),
                                 ("K4", scenes.ascii((1024, 1024), primary_only=True), ["-bvh", "-s", "1"])):
            scenes.write(scene, os.path.join(tmp, "ASCII", key + ".json"))
            subprocess.run([REF_BIN, "-input", key + ".json", "-output", key + ".ppm"] + args, cwd=build,
                           capture_output=True, check=True)
            md5 = hashlib.md5(open(os.path.join(tmp, "Output", key + ".ppm"), "rb").read()).hexdigest()
            manifest["known_answer"][key] = {"md5": md5, "survey_md5": SURVEY_MD5[key], "args": args,
                                             "resolution": scene["render"]}
            print(key, md5, "(survey", SURVEY_MD5[key] + ")")
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
