"""The scene loader (json_dom.cpp + scene.cpp) on damaged input: truncated files, flipped
bytes, wrong value types and absurd numbers must end in a loaded scene or a clean
NativeError -- never a crash.  Run it under the sanitizer build (`make asan`, see Makefile)
to check memory safety as well (profiles/r02_asan_ubsan_cpu_suite.log)."""
import json
import random

import pytest

import ray_tracying_amd as rt
import scenes


def _load(path):
    try:
        sc = rt.Scene(path, texture_root=scenes.TEXTURES)
    except rt.NativeError:
        return False
    sc.close()
    return True


def test_truncated_and_mutated_scenes(tmp_path):
    base = json.dumps(scenes.features(res=(16, 12)), indent=1).encode()
    rnd = random.Random(1234)
    p = str(tmp_path / "m.json")
    outcomes = set()
    for k in range(300):
        data = bytearray(base)
        mode = k % 3
        if mode == 0:
            data = data[:rnd.randrange(len(data))]
        elif mode == 1:
            for _ in range(rnd.randint(1, 8)):
                data[rnd.randrange(len(data))] = rnd.choice(b'{}[],:"0123456789.eE-+ \\nul')
        else:
            i = rnd.randrange(len(data))
            data[i:i] = rnd.choice([b'1e999', b'-', b'"', b'\\u00', b'[[[[[', b'null', b'true'])
        open(p, "wb").write(bytes(data))
        outcomes.add(_load(p))
    assert outcomes == {True, False}


@pytest.mark.parametrize("edit", ["str_vector", "nested", "huge", "negative_res", "empty_arrays"])
def test_wrong_types(tmp_path, edit):
    sc = scenes.features(res=(16, 12))
    if edit == "str_vector":
        sc["spheres"][0]["location"] = "abc"
        sc["planes"][0]["corners"][1] = [1, 2]
    elif edit == "nested":
        sc["cubes"][0]["scale"] = [[1, 2, 3]]
        sc["lights"][0]["color"] = {"r": 1}
    elif edit == "huge":
        sc["spheres"][1]["radius"] = 1e300
        sc["cameras"][0]["focal_length"] = 1e-300
    elif edit == "negative_res":
        sc["render"] = {"resolution_x": -5, "resolution_y": 12}
    else:
        sc["spheres"], sc["cubes"], sc["planes"], sc["lights"] = [], [], [], []
    p = scenes.write(sc, str(tmp_path / "w.json"))
    _load(p)  # either outcome is fine; no crash
