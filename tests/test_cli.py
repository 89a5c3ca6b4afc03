"""The drop-in CLI `ray_tracying_amd/bin/raytracer` against the reference's main()
(Code/raytracer.cpp:356-488): same flags, the same ../../ASCII/ and ../../Output/ layout
relative to the working directory, the same messages and exit codes, the same P3 bytes.

CPU tests cover the paths that end before any rendering (no scene name, unreadable or
malformed file, zero resolution: camera.cpp:14-58, 240-252 and raytracer.cpp:389-402).  When
the compiled reference (oracle/_ref/Raytracer, built from the reference's own sources by
oracle/Makefile) is present, its output is the expectation; otherwise the reference's literal
messages are.  The GPU test renders K1 through the CLI and checks the
image md5 against the reference's and the stdout lines against the reference binary's.
"""
import hashlib
import json
import os
import shutil
import subprocess

import pytest

import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "ray_tracying_amd", "bin", "raytracer")
REF = os.path.join(ROOT, "oracle", "_ref", "Raytracer")
RES0 = "Error: Camera resolution is 0. Check scene.json."
CAM_FAIL = "Camera configuration failed to load. Using default values."


@pytest.fixture
def tree(tmp_path):
    """X/Code/build (cwd), X/ASCII (scenes), X/Output (images), X/Textures."""
    build = tmp_path / "Code" / "build"
    build.mkdir(parents=True)
    (tmp_path / "ASCII").mkdir()
    (tmp_path / "Output").mkdir()
    shutil.copytree(scenes.TEXTURES, tmp_path / "Textures")
    return tmp_path


def run(binary, args, cwd):
    r = subprocess.run([binary] + args, cwd=cwd, capture_output=True, text=True, timeout=300)
    return r.returncode, r.stdout.splitlines(), r.stderr.splitlines()


def _error_cases(tree):
    res0 = scenes.ascii((64, 64))
    res0["render"] = {"resolution_x": 0, "resolution_y": 0}
    scenes.write(res0, str(tree / "ASCII" / "res0.json"))
    (tree / "ASCII" / "bad.json").write_text('{"cameras": [')
    keys = scenes.ascii((64, 64))
    del keys["render"]
    scenes.write(keys, str(tree / "ASCII" / "nokeys.json"))
    return {
        "no_input": ([], 1, ["Correct usage: ./Raytracer -name {scene_file_name.json}"],
                     ["Error: Please specify scene file name"]),
        "missing": (["-input", "missing.json"], 1, [],
                    ["Error: Could not open file ../../ASCII/missing.json", CAM_FAIL, RES0]),
        "res0": (["-input", "res0.json", "-bvh"], 1, [], [RES0]),
        "nokeys": (["-input", "nokeys.json"], 1, [], ["Error: JSON file is missing required keys.", RES0]),
        "bad_json": (["-input", "bad.json", "-s", "2"], 1, [], ["JSON Parse Error: *", CAM_FAIL, RES0]),
    }


def _match(lines, expected):
    assert len(lines) == len(expected), (lines, expected)
    for got, want in zip(lines, expected):
        if want.endswith("*"):  # nlohmann's parse-error text is not restated
            assert got.startswith(want[:-1]), (got, want)
        else:
            assert got == want, (got, want)


@pytest.mark.parametrize("case", ["no_input", "missing", "res0", "nokeys", "bad_json"])
def test_cli_error_paths(tree, case):
    args, rc, out, err = _error_cases(tree)[case]
    cwd = str(tree / "Code" / "build")
    got = run(CLI, args, cwd)
    assert got[0] == rc
    _match(got[1], out)
    _match(got[2], err)
    if os.path.exists(REF):  # the reference binary itself prints the same lines
        ref = run(REF, args, cwd)
        assert ref[0] == rc
        _match(ref[1], out)
        _match(ref[2], err)
    assert not os.listdir(tree / "Output")


@pytest.mark.gpu
def test_cli_k1_matches_reference(tree, gpu):
    """K1 (ASCII scene 256^2, roughness 0, -bvh -s 1: deterministic) through the drop-in CLI:
    the P3 file equals the reference's byte for byte, and stdout carries the reference's lines."""
    man = json.load(open(os.path.join(scenes.GOLDEN, "manifest.json")))
    scenes.write(scenes.ascii((256, 256), roughness=0.0), str(tree / "ASCII" / "K1.json"))
    cwd = str(tree / "Code" / "build")
    rc, out, err = run(CLI, ["-input", "K1.json", "-bvh", "-s", "1", "-output", "k1.ppm"], cwd)
    assert rc == 0, err[-3:]
    md5 = hashlib.md5((tree / "Output" / "k1.ppm").read_bytes()).hexdigest()
    assert md5 == man["known_answer"]["K1"]["md5"]
    assert out == ["BVH built. Mode: ON", "Rendering 256x256 with 1x1 samples and 1 light sampling points ...",
                   "Progress: 39%", "Progress: 78%", "Rendering complete.",
                   "Image written to ../../Output/k1.ppm"]  # Image::write, image.cpp:82
    if os.path.exists(REF):
        ref = run(REF, ["-input", "K1.json", "-bvh", "-s", "1", "-output", "k1_ref.ppm"], cwd)
        assert ref[0] == 0 and ref[1] == out[:-1] + ["Image written to ../../Output/k1_ref.ppm"]
        assert (tree / "Output" / "k1_ref.ppm").read_bytes() == (tree / "Output" / "k1.ppm").read_bytes()
    # default output name, the image-tile path on one device (-gpus 1 renders in one call)
    rc, _, err = run(CLI, ["-input", "K1.json", "-bvh", "-s", "1", "-gpus", "1"], cwd)
    assert rc == 0, err[-3:]
    assert hashlib.md5((tree / "Output" / "output.ppm").read_bytes()).hexdigest() == md5


@pytest.mark.gpu
def test_cli_multi_device_tiles(tree, gpu):
    """-gpus 2: tiles dealt to two devices and gathered over RCCL (main.cpp).  With fewer
    devices than asked for the CLI fails cleanly (exit 1, a message, no image)."""
    scenes.write(scenes.ascii((128, 96), roughness=0.0), str(tree / "ASCII" / "K.json"))
    cwd = str(tree / "Code" / "build")
    rc1, _, err1 = run(CLI, ["-input", "K.json", "-bvh", "-s", "1", "-output", "one.ppm"], cwd)
    assert rc1 == 0, err1
    rc2, _, err2 = run(CLI, ["-input", "K.json", "-bvh", "-s", "1", "-gpus", "2", "-output", "two.ppm"], cwd)
    if gpu >= 2:
        assert rc2 == 0, err2
        assert (tree / "Output" / "two.ppm").read_bytes() == (tree / "Output" / "one.ppm").read_bytes()
    else:
        assert rc2 == 1 and any(line.startswith("An error occurred: ") for line in err2)
        assert not (tree / "Output" / "two.ppm").exists()
