"""Host layer (librt_host.so) and the C ABI surface -- CPU only, no GPU calls."""
import ctypes
import hashlib
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_bind as ob
import ray_tracying_amd as rt
import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?[a-z_]+\**\s+\**(rth?_[a-z0-9_]+)\s*\(", txt, flags=re.M))


@pytest.mark.parametrize("lib,header", [("librt_hip.so", "rt_hip.h"), ("librt_host.so", "rt_host.h"),
                                        ("librt_comm.so", "rt_comm.h")])
def test_c_abi_exports_every_declared_symbol(lib, header):
    path = os.path.join(rt.LIB_DIR, lib)
    syms = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in syms.splitlines() if " T " in l}
    want = declared(header)
    assert want, header
    assert want <= exported, want - exported
    # and the library loads / resolves them
    L = ctypes.CDLL(path)
    for s in want:
        getattr(L, s)


def test_python_symbol_lists_match_headers():
    assert set(rt.HIP_SYMBOLS) == declared("rt_hip.h")
    assert set(rt.HOST_SYMBOLS) == declared("rt_host.h")


@pytest.mark.parametrize("name", sorted(scenes.cases()))
def test_scene_loading_matches_oracle(name, tmp_path):
    path, _ = scenes.materialise(name, str(tmp_path))
    W, H, ns, nl = ob.scene_info(path)
    sc = rt.Scene(path, texture_root=scenes.TEXTURES)
    assert (sc.width, sc.height, sc.info.n_shapes, sc.info.n_lights) == (W, H, ns, nl)
    assert sc.info.tree_depth <= 64 and (ns == 0 or sc.info.n_nodes >= 1)
    sc.close()


def test_quantise_matches_reference_formula():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.random(20000, dtype=np.float32) * 1.3 - 0.1,
                        np.array([0, 1, 1e-30, 0.5, 0.999, 1.0001, 2.0, -0.0], dtype=np.float32)]).astype(np.float32)
    got = rt.quantise(x)
    lib = ob.lib()
    want = np.array([lib.oracle_quantise(ctypes.c_float(v)) for v in x.tolist()], dtype=np.uint8)
    assert np.array_equal(got, want)


def test_ppm_writer_byte_identical(tmp_path):
    rng = np.random.default_rng(1)
    u8 = rng.integers(0, 256, size=(7, 5, 3), dtype=np.uint8)
    p = str(tmp_path / "x.ppm")
    rt.write_ppm(p, u8)
    assert open(p, "rb").read() == ob.ppm_bytes(u8)


def test_unpack_tiles_roundtrip():
    W, H, T = 37, 21, 8
    img = np.random.default_rng(2).random((H, W, 3), dtype=np.float32)
    tx, ty = (W + T - 1) // T, (H + T - 1) // T
    ids = np.array([5, 0, 3, 1, 2, 4] + list(range(6, tx * ty)), dtype=np.int32)
    packed = np.zeros((len(ids), T, T, 3), np.float32)
    for k, t in enumerate(ids):
        x0, y0 = (t % tx) * T, (t // tx) * T
        blk = img[y0:y0 + T, x0:x0 + T]
        packed[k, :blk.shape[0], :blk.shape[1]] = blk
    out = rt.unpack_tiles(packed, ids, T, T, W, H)
    assert np.array_equal(out, img)


def test_soup_generator_and_loader(tmp_path):
    p = str(tmp_path / "soup.json")
    rt.make_soup(p, 1000, seed=3, width=64, height=32)
    sc = rt.Scene(p)
    assert (sc.width, sc.height, sc.info.n_shapes, sc.info.n_lights) == (64, 32, 1000, 1)
    assert sc.info.prim_stride == 64  # planes only -> 64-byte records
    assert ob.scene_info(p) == (64, 32, 1000, 1)


def test_resolution_override(tmp_path):
    path, _ = scenes.materialise("features_s1", str(tmp_path))
    sc = rt.Scene(path, resolution=(100, 30))
    assert (sc.width, sc.height) == (100, 30)


def test_missing_scene_raises():
    with pytest.raises(rt.NativeError):
        rt.Scene("/nonexistent/scene.json")


def test_malformed_json_raises(tmp_path):
    p = tmp_path / "bad.json"
    p.write_text('{"cameras": [ {"focal_length": 1.0,, } ]')
    with pytest.raises(rt.NativeError):
        rt.Scene(str(p))


def test_edge_scenes_match_oracle_counts(tmp_path):
    """Skip rules of json_loader.cpp: invalid lights/cubes/planes are dropped with warnings,
    materials that fail to parse fall back to Material() -- same counts as the oracle."""
    s = scenes.features()
    s["spheres"].append({"location": [0, 0, 0], "radius": 1.0, "material": {"k_ambient": "x"}})
    s["spheres"].append({"location": [0, 1]})        # short array -> skipped
    s["cubes"].append("not an object")
    s["lights"].append({"location": [1, 2, 3], "color": [1, 1, 1], "intensity": True})
    s["render"] = {"resolution_x": 16.9, "resolution_y": 8}
    p = scenes.write(s, str(tmp_path / "edge.json"))
    sc = rt.Scene(p, texture_root=scenes.TEXTURES)
    assert (sc.width, sc.height, sc.info.n_shapes, sc.info.n_lights) == ob.scene_info(p)


def test_render_without_gpu_fails_loudly(tmp_path):
    """No silent CPU fallback: on a machine without a HIP device render() raises."""
    if rt.device_count() > 0:
        pytest.skip("a HIP device is present")
    path, _ = scenes.materialise("soup_s1", str(tmp_path))
    sc = rt.Scene(path)
    with pytest.raises(rt.NativeError):
        sc.render()


def test_scene_create_rejects_misused_tri1_never_tag(tmp_path):
    """RT_TAG_TRI1_NEVER turns a[12] into a squared radius; rt_scene_create must
    reject the bit on anything but a valid Plane record with a finite a[12] >= 0.  The check
    runs before any device call, so it holds on a machine without a GPU too."""
    rt._load()
    sc = rt.Scene(scenes.write(scenes.soup(300, seed=2), str(tmp_path / "s.json")))
    d = sc.desc()
    w = d.prim_stride // 4
    prims = np.ctypeslib.as_array(ctypes.cast(d.prims, ctypes.POINTER(ctypes.c_float)), shape=(d.n_prims * w,))
    recs = prims.reshape(d.n_prims, w).copy()
    tags = recs[:, 15].view(np.uint32)
    tri1 = np.flatnonzero(tags & 16)
    assert len(tri1) > 0, "the soup's triangles carry RT_TAG_TRI1_NEVER"
    k = int(tri1[0])

    def create(bad):
        dd = rt.rt_scene_desc.from_buffer_copy(d)
        dd.prims = bad.ctypes.data
        h = ctypes.c_void_p()
        rc = rt._hip.rt_scene_create(0, ctypes.byref(dd), ctypes.byref(h))
        if rc == 0:
            rt._hip.rt_scene_destroy(h)
        return rc, rt._hip.rt_last_error().decode()

    for mutate in (lambda r: r.__setitem__((k, 12), -1.0),                      # negative radius
                   lambda r: r.__setitem__((k, 12), np.float32("nan")),         # NaN radius
                   lambda r: r[k, 15:16].view(np.uint32).__iand__(np.uint32(~4 & 0xffffffff)),  # not a valid plane
                   lambda r: r[k, 15:16].view(np.uint32).__iand__(np.uint32(~3 & 0xffffffff))):  # kind: sphere
        bad = recs.copy()
        mutate(bad)
        rc, msg = create(bad)
        assert rc == -1 and "TRI1_NEVER" in msg, (rc, msg)
    rc, msg = create(recs.copy())  # the untouched records pass the check (then need a device)
    assert "TRI1_NEVER" not in msg
    sc.close()
