"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference's path (oracle/rt_oracle.cpp).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.environ.get("ORACLE_SO") or os.path.join(ROOT, "oracle", "liboracle.so")  # ORACLE_SO: sanitizer build
RNG_MT19937, RNG_COUNTER = 0, 1


class oracle_params(ctypes.Structure):
    _fields_ = [("use_bvh", ctypes.c_int), ("spp_sqrt", ctypes.c_int), ("light_samples", ctypes.c_int),
                ("rng_mode", ctypes.c_int), ("seed", ctypes.c_ulonglong), ("res_w", ctypes.c_int),
                ("res_h", ctypes.c_int), ("x0", ctypes.c_int), ("y0", ctypes.c_int), ("w", ctypes.c_int),
                ("h", ctypes.c_int)]


class oracle_stats(ctypes.Structure):
    _fields_ = [("rays", ctypes.c_ulonglong), ("box_tests", ctypes.c_ulonglong), ("prim_tests", ctypes.c_ulonglong),
                ("width", ctypes.c_int), ("height", ctypes.c_int), ("n_shapes", ctypes.c_int),
                ("n_lights", ctypes.c_int), ("render_seconds", ctypes.c_double), ("load_seconds", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            raise FileNotFoundError(f"{ORACLE_SO} missing: run `make -C oracle`")
        _lib = ctypes.CDLL(ORACLE_SO)
        _lib.oracle_render.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(oracle_params),
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(oracle_stats)]
        _lib.oracle_render_regions.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(oracle_params),
                                               ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.POINTER(oracle_stats), ctypes.c_int]
        _lib.oracle_scene_info.argtypes = [ctypes.c_char_p] + [ctypes.POINTER(ctypes.c_int)] * 4
        _lib.oracle_powf.argtypes = [ctypes.c_float, ctypes.c_float]
        _lib.oracle_powf.restype = ctypes.c_float
        _lib.oracle_quantise.argtypes = [ctypes.c_float]
        _lib.oracle_counter_draw.argtypes = [ctypes.c_ulonglong, ctypes.c_ulonglong, ctypes.c_ulonglong, ctypes.c_int]
        _lib.oracle_counter_draw.restype = ctypes.c_double
    return _lib


def scene_info(path: str):
    w, h, ns, nl = (ctypes.c_int() for _ in range(4))
    rc = lib().oracle_scene_info(path.encode(), ctypes.byref(w), ctypes.byref(h), ctypes.byref(ns), ctypes.byref(nl))
    if rc:
        raise RuntimeError(f"oracle_scene_info({path}) -> {rc}")
    return w.value, h.value, ns.value, nl.value


def render(path: str, *, use_bvh=True, spp_sqrt=1, light_samples=1, rng=RNG_COUNTER, seed=20251226,
           texture_root=None, region=None, resolution=None):
    """-> (float32 (h, w, 3) linear RGB, uint8 (h, w, 3), stats dict)."""
    W, H, _, _ = scene_info(path)
    if resolution:
        W, H = resolution
    x0, y0, w, h = region if region else (0, 0, W, H)
    p = oracle_params(int(use_bvh), int(spp_sqrt), int(light_samples), int(rng), int(seed),
                      resolution[0] if resolution else 0, resolution[1] if resolution else 0,
                      x0, y0, 0 if not region else w, 0 if not region else h)
    rgb = np.zeros((h, w, 3), dtype=np.float32)
    u8 = np.zeros((h, w, 3), dtype=np.uint8)
    st = oracle_stats()
    rc = lib().oracle_render(path.encode(), texture_root.encode() if texture_root else None, ctypes.byref(p),
                             rgb.ctypes.data, u8.ctypes.data, ctypes.byref(st))
    if rc:
        raise RuntimeError(f"oracle_render({path}) -> {rc}")
    return rgb, u8, {"rays": st.rays, "box_tests": st.box_tests, "prim_tests": st.prim_tests,
                     "render_seconds": st.render_seconds, "load_seconds": st.load_seconds}


def render_regions(path: str, regions, *, use_bvh=True, spp_sqrt=1, light_samples=1, seed=20251226,
                   texture_root=None, resolution=None, threads=None):
    """Counter-RNG render of several (x0, y0, w, h) regions after ONE scene load, rows spread
    over `threads` threads -> (list of float32 (h, w, 3) arrays, stats dict)."""
    reg = np.ascontiguousarray(np.asarray(regions, dtype=np.int32).reshape(-1, 4))
    total = int((reg[:, 2] * reg[:, 3]).sum()) * 3
    out = np.zeros(total, dtype=np.float32)
    p = oracle_params(int(use_bvh), int(spp_sqrt), int(light_samples), RNG_COUNTER, int(seed),
                      resolution[0] if resolution else 0, resolution[1] if resolution else 0, 0, 0, 0, 0)
    st = oracle_stats()
    nt = threads or min(16, os.cpu_count() or 1)
    rc = lib().oracle_render_regions(path.encode(), texture_root.encode() if texture_root else None, ctypes.byref(p),
                                     len(reg), reg.ctypes.data, out.ctypes.data, ctypes.byref(st), int(nt))
    if rc:
        raise RuntimeError(f"oracle_render_regions({path}) -> {rc}")
    imgs, off = [], 0
    for x0, y0, w, h in reg.tolist():
        imgs.append(out[off:off + w * h * 3].reshape(h, w, 3))
        off += w * h * 3
    return imgs, {"rays": st.rays, "box_tests": st.box_tests, "prim_tests": st.prim_tests,
                  "render_seconds": st.render_seconds, "load_seconds": st.load_seconds}


def ppm_bytes(u8: np.ndarray) -> bytes:
    """Image::write's exact P3 layout (image.cpp:62-79)."""
    h, w = u8.shape[:2]
    lines = [f"P3\n{w} {h}\n255\n"]
    for y in range(h):
        lines.append("  ".join(f"{r} {g} {b}" for r, g, b in u8[y].tolist()) + "\n")
    return "".join(lines).encode()
