"""ray_tracying_amd -- MI355X-native drop-in for the Ray_Tracying per-pixel hot path.

Python mirror of the reference's host surface over the C ABI in ``include/rt_hip.h``
(device) and ``include/rt_host.h`` (host).  Names follow the reference:

    Scene(path)              Camera(path) + load_lights_from_json + load_shapes_from_json
                             + BVH(shapes)   (camera.cpp:240-252, json_loader.cpp:103-338,
                                              acceleration.cpp:7-64)
    Scene.render(...)        main()'s y/x loop over compute_pixel_color (raytracer.cpp:433-476)
    quantise(rgb)            gamma 1/1.1, clamp, *255.999 (raytracer.cpp:446-457)
    write_ppm(path, u8)      Image::write (image.cpp:53-83)

The compute path is the hand-written HIP kernels in ``librt_hip.so``; there is no CPU
fallback: if the native libraries are missing or no HIP device is present, ``render``
raises.  (The CPU restatement under ``oracle/`` is test infrastructure only.)
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RT_LIB_DIR overrides the library directory (A/B builds of the same sources); default in-tree
LIB_DIR = os.environ.get("RT_LIB_DIR") or os.path.join(_HERE, "lib")

__all__ = [
    "Scene", "RenderParams", "RenderStats", "quantise", "write_ppm", "make_soup",
    "device_count", "native_loaded", "LIB_DIR", "NativeError",
]


class NativeError(RuntimeError):
    """A C-ABI call returned a negative RT_E* code."""


# ---------------------------------------------------------------- C structs (rt_hip.h)
class rt_scene_desc(ctypes.Structure):
    _fields_ = [
        ("n_prims", ctypes.c_int32), ("prim_stride", ctypes.c_int32), ("prims", ctypes.c_void_p),
        ("prim_refs", ctypes.c_void_p), ("n_unbounded", ctypes.c_int32),
        ("n_nodes", ctypes.c_int32), ("tree_depth", ctypes.c_int32), ("stack_bound", ctypes.c_int32),
        ("nodes", ctypes.c_void_p),
        ("n_ref_leaves", ctypes.c_int32), ("ref_leaf_boxes", ctypes.c_void_p),
        ("n_materials", ctypes.c_int32), ("materials", ctypes.c_void_p),
        ("n_lights", ctypes.c_int32), ("lights", ctypes.c_void_p),
        ("n_textures", ctypes.c_int32), ("textures", ctypes.c_void_p),
        ("n_texel_bytes", ctypes.c_int64), ("texels", ctypes.c_void_p),
        ("scene_scale", ctypes.c_float), ("flags", ctypes.c_int32),
    ]


class rt_camera_desc(ctypes.Structure):
    _fields_ = [
        ("res_x", ctypes.c_int32), ("res_y", ctypes.c_int32),
        ("half_sensor_w", ctypes.c_float), ("half_sensor_h", ctypes.c_float),
        ("location", ctypes.c_float * 3), ("focal_length", ctypes.c_float),
        ("x_dir", ctypes.c_float * 3), ("aperture", ctypes.c_float),
        ("y_dir", ctypes.c_float * 3), ("focus_dist", ctypes.c_float),
        ("z_dir", ctypes.c_float * 3), ("pad", ctypes.c_float),
    ]


class rt_render_params(ctypes.Structure):
    _fields_ = [
        ("spp_sqrt", ctypes.c_int32), ("light_samples", ctypes.c_int32),
        ("use_bvh", ctypes.c_int32), ("count_work", ctypes.c_int32),
        ("seed", ctypes.c_uint64), ("sync", ctypes.c_int32), ("pad", ctypes.c_int32),
    ]


class rt_stats(ctypes.Structure):
    _fields_ = [
        ("rays", ctypes.c_uint64), ("box_tests", ctypes.c_uint64), ("prim_tests", ctypes.c_uint64),
        ("kernel_ms", ctypes.c_double), ("trace_ms", ctypes.c_double),
        ("iterations", ctypes.c_int32), ("path", ctypes.c_int32), ("node_visits", ctypes.c_uint64),
        ("trace_busy_ms", ctypes.c_double),
    ]


class rth_scene_info(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("n_shapes", ctypes.c_int32), ("n_lights", ctypes.c_int32),
        ("n_nodes", ctypes.c_int32), ("tree_depth", ctypes.c_int32),
        ("n_materials", ctypes.c_int32), ("n_textures", ctypes.c_int32),
        ("prim_stride", ctypes.c_int32), ("flags", ctypes.c_int32),
        ("load_seconds", ctypes.c_double), ("build_seconds", ctypes.c_double),
    ]


# ---------------------------------------------------------------- library loading
_hip = None
_host = None

# exported symbols each library must provide (tests check this list against include/*.h)
HIP_SYMBOLS = [
    "rt_device_count", "rt_scene_create", "rt_scene_destroy", "rt_render_tiles", "rt_malloc",
    "rt_free", "rt_memcpy_d2h", "rt_memcpy_h2d", "rt_synchronize", "rt_build_info", "rt_last_error",
    "rt_quantise_device", "rt_tile_costs", "rt_tile_costs_measured", "rt_render_wait", "rt_render_frames",
]
HOST_SYMBOLS = [
    "rth_scene_load", "rth_scene_free", "rth_scene_get_info", "rth_scene_desc", "rth_scene_camera",
    "rth_render", "rth_unpack_tiles", "rth_quantise", "rth_write_ppm", "rth_make_soup", "rth_last_error",
]


def _load():
    """Load librt_hip.so / librt_host.so (RTLD_GLOBAL).  If torch is importable it is imported
    first so that its HIP runtime (same SONAME libamdhip64.so.7) is the one both share."""
    global _hip, _host
    if _host is not None:
        return
    try:  # share one HIP runtime with torch when both are used in a process
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the C ABI
        pass
    hip_path = os.path.join(LIB_DIR, "librt_hip.so")
    host_path = os.path.join(LIB_DIR, "librt_host.so")
    for p in (hip_path, host_path):
        if not os.path.exists(p):
            raise NativeError(f"native library missing: {p} (run `make` or __graft_entry__.build())")
    _hip = ctypes.CDLL(hip_path, mode=ctypes.RTLD_GLOBAL)
    _host = ctypes.CDLL(host_path, mode=ctypes.RTLD_GLOBAL)
    c = ctypes
    _hip.rt_last_error.restype = c.c_char_p
    _hip.rt_build_info.restype = c.c_char_p
    _hip.rt_device_count.argtypes = [c.POINTER(c.c_int32)]
    _hip.rt_scene_create.argtypes = [c.c_int32, c.POINTER(rt_scene_desc), c.POINTER(c.c_void_p)]
    _hip.rt_scene_destroy.argtypes = [c.c_void_p]
    _hip.rt_render_tiles.argtypes = [c.c_void_p, c.POINTER(rt_camera_desc), c.POINTER(rt_render_params),
                                     c.POINTER(c.c_int32), c.c_int32, c.c_int32, c.c_int32, c.c_void_p,
                                     c.c_void_p, c.POINTER(rt_stats)]
    _hip.rt_render_frames.argtypes = [c.c_void_p, c.POINTER(rt_camera_desc), c.POINTER(rt_render_params),
                                      c.POINTER(c.c_uint64), c.c_int32, c.POINTER(c.c_int32), c.c_int32, c.c_int32,
                                      c.c_int32, c.c_void_p, c.c_void_p, c.POINTER(rt_stats)]
    _hip.rt_malloc.argtypes = [c.c_int32, c.c_size_t, c.POINTER(c.c_void_p)]
    _hip.rt_free.argtypes = [c.c_void_p]
    _hip.rt_memcpy_d2h.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t]
    _hip.rt_memcpy_h2d.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t]
    _hip.rt_quantise_device.argtypes = [c.c_void_p, c.c_int64, c.c_void_p, c.c_void_p]
    _hip.rt_tile_costs.argtypes = [c.c_void_p, c.POINTER(rt_camera_desc), c.c_int32, c.c_int32, c.POINTER(c.c_float)]
    _hip.rt_tile_costs_measured.argtypes = [c.c_void_p, c.POINTER(rt_camera_desc), c.c_int32, c.c_int32, c.c_int32,
                                            c.POINTER(c.c_float)]
    _hip.rt_render_wait.argtypes = [c.c_void_p, c.POINTER(rt_stats)]
    _hip.rt_synchronize.argtypes = [c.c_int32]
    _host.rth_last_error.restype = c.c_char_p
    _host.rth_scene_load.argtypes = [c.c_char_p, c.c_char_p, c.c_int32, c.c_int32, c.POINTER(c.c_void_p)]
    _host.rth_scene_free.argtypes = [c.c_void_p]
    _host.rth_scene_get_info.argtypes = [c.c_void_p, c.POINTER(rth_scene_info)]
    _host.rth_scene_desc.argtypes = [c.c_void_p, c.POINTER(rt_scene_desc)]
    _host.rth_scene_camera.argtypes = [c.c_void_p, c.POINTER(rt_camera_desc)]
    _host.rth_render.argtypes = [c.c_void_p, c.c_int32, c.POINTER(rt_render_params), c.c_void_p,
                                 c.POINTER(rt_stats)]
    _host.rth_unpack_tiles.argtypes = [c.c_void_p, c.POINTER(c.c_int32), c.c_int32, c.c_int32, c.c_int32,
                                       c.c_int32, c.c_int32, c.c_void_p]
    _host.rth_quantise.argtypes = [c.c_void_p, c.c_int64, c.c_void_p]
    _host.rth_write_ppm.argtypes = [c.c_char_p, c.c_int32, c.c_int32, c.c_void_p]
    _host.rth_make_soup.argtypes = [c.c_char_p, c.c_int64, c.c_uint64, c.c_int32, c.c_int32]


def native_loaded() -> bool:
    try:
        _load()
        return True
    except NativeError:
        return False


def hip_lib():
    _load()
    return _hip


def host_lib():
    _load()
    return _host


def _check_hip(rc: int, what: str):
    if rc != 0:
        raise NativeError(f"{what} failed ({rc}): {_hip.rt_last_error().decode(errors='replace')}")


def _check_host(rc: int, what: str):
    if rc != 0:
        raise NativeError(f"{what} failed ({rc}): {_host.rth_last_error().decode(errors='replace')}")


def device_count() -> int:
    _load()
    n = ctypes.c_int32(0)
    rc = _hip.rt_device_count(ctypes.byref(n))
    return int(n.value) if rc == 0 else 0


# ---------------------------------------------------------------- public API
@dataclass
class RenderParams:
    """The reference's CLI knobs (raytracer.cpp:361-390) + the counter-RNG seed."""
    spp_sqrt: int = 4          # -s
    light_samples: int = 1     # -light_sample
    use_bvh: bool = True       # -bvh
    seed: int = 20251226
    count_work: bool = False   # instrumented run: fill box_tests / prim_tests
    sync: bool = True          # False: a one-pass call returns once enqueued (DeviceScene.wait finishes it)

    def c(self) -> rt_render_params:
        return rt_render_params(int(self.spp_sqrt), int(self.light_samples), 1 if self.use_bvh else 0,
                                1 if self.count_work else 0, int(self.seed) & (2**64 - 1), 1 if self.sync else 0, 0)


PATH_STEPS, PATH_ONE_PASS = 0, 1  # rt_stats.path (include/rt_hip.h)


@dataclass
class RenderStats:
    rays: int
    box_tests: int
    prim_tests: int
    kernel_ms: float
    trace_ms: float
    iterations: int
    node_visits: int = 0
    trace_busy_ms: float = 0.0
    path: int = 0  # PATH_ONE_PASS: camera rays, one trace launch, shading + reduction; PATH_STEPS: the step pipeline

    @staticmethod
    def of(st: rt_stats) -> "RenderStats":
        return RenderStats(int(st.rays), int(st.box_tests), int(st.prim_tests), float(st.kernel_ms),
                           float(st.trace_ms), int(st.iterations), int(st.node_visits), float(st.trace_busy_ms),
                           int(st.path))


class Scene:
    """A loaded, BVH-built, flattened scene (host side) -- see rt_host.h."""

    def __init__(self, path: str, texture_root: str | None = None, resolution: tuple[int, int] | None = None):
        _load()
        h = ctypes.c_void_p()
        w, hgt = resolution if resolution else (0, 0)
        _check_host(_host.rth_scene_load(path.encode(), texture_root.encode() if texture_root else None,
                                         int(w), int(hgt), ctypes.byref(h)), "rth_scene_load")
        self._h = h
        info = rth_scene_info()
        _check_host(_host.rth_scene_get_info(h, ctypes.byref(info)), "rth_scene_get_info")
        self.info = info
        self.width, self.height = int(info.width), int(info.height)

    def close(self):
        if getattr(self, "_h", None):
            _host.rth_scene_free(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def desc(self) -> rt_scene_desc:
        d = rt_scene_desc()
        _check_host(_host.rth_scene_desc(self._h, ctypes.byref(d)), "rth_scene_desc")
        return d

    def camera(self) -> rt_camera_desc:
        c = rt_camera_desc()
        _check_host(_host.rth_scene_camera(self._h, ctypes.byref(c)), "rth_scene_camera")
        return c

    def render(self, params: RenderParams | None = None, device: int = 0) -> tuple[np.ndarray, RenderStats]:
        """Whole frame on one GPU -> (H, W, 3) float32 linear RGB (== compute_pixel_color)."""
        p = (params or RenderParams()).c()
        if self.width <= 0 or self.height <= 0:
            raise NativeError("Error: Camera resolution is 0. Check scene.json.")
        if device_count() <= device:
            raise NativeError(f"no HIP device {device} (visible: {device_count()})")
        out = np.zeros((self.height, self.width, 3), dtype=np.float32)
        st = rt_stats()
        _check_host(_host.rth_render(self._h, int(device), ctypes.byref(p), out.ctypes.data, ctypes.byref(st)),
                    "rth_render")
        return out, RenderStats.of(st)


class DeviceScene:
    """A scene uploaded to one device (rt_scene_t), for tile-level rendering."""

    def __init__(self, scene: Scene, device: int = 0):
        _load()
        self.device = device
        self.cam = scene.camera()
        d = scene.desc()
        h = ctypes.c_void_p()
        _check_hip(_hip.rt_scene_create(int(device), ctypes.byref(d), ctypes.byref(h)), "rt_scene_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _hip.rt_scene_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def render_tiles(self, tile_ids, tile_w: int, tile_h: int, d_out: int, params: RenderParams,
                     stream: int | None = None) -> RenderStats:
        """rt_render_tiles into a caller-owned DEVICE buffer (e.g. a torch tensor's data_ptr)."""
        ids = np.ascontiguousarray(np.asarray(tile_ids, dtype=np.int32))
        p = params.c()
        st = rt_stats()
        _check_hip(_hip.rt_render_tiles(self._h, ctypes.byref(self.cam), ctypes.byref(p),
                                        ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), int(ids.size),
                                        int(tile_w), int(tile_h), ctypes.c_void_p(int(d_out)),
                                        ctypes.c_void_p(int(stream) if stream else 0), ctypes.byref(st)),
                   "rt_render_tiles")
        return RenderStats.of(st)

    def render_frames(self, seeds, tile_ids, tile_w: int, tile_h: int, d_out: int, params: RenderParams,
                      stream: int | None = None) -> RenderStats:
        """rt_render_frames: len(seeds) frames of the same tiles in one call (frame f with seed
        seeds[f]; params.seed unused) into a DEVICE buffer of len(seeds) * len(tile_ids) tiles,
        frame-major; frame f == render_tiles with seed seeds[f], bit for bit."""
        ids = np.ascontiguousarray(np.asarray(tile_ids, dtype=np.int32))
        sd = np.ascontiguousarray(np.asarray([int(x) & (2**64 - 1) for x in seeds], dtype=np.uint64))
        p = params.c()
        st = rt_stats()
        _check_hip(_hip.rt_render_frames(self._h, ctypes.byref(self.cam), ctypes.byref(p),
                                         sd.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), int(sd.size),
                                         ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), int(ids.size),
                                         int(tile_w), int(tile_h), ctypes.c_void_p(int(d_out)),
                                         ctypes.c_void_p(int(stream) if stream else 0), ctypes.byref(st)),
                   "rt_render_frames")
        return RenderStats.of(st)

    def tile_costs(self, tile_w: int, tile_h: int) -> np.ndarray:
        """rt_tile_costs: per-tile cost estimate (projected primitive centres), tile id order."""
        if int(tile_w) <= 0 or int(tile_h) <= 0:
            raise NativeError(f"rt_tile_costs: tile size must be positive (got {tile_w}x{tile_h})")
        tx =(self.cam.res_x + tile_w - 1) // tile_w
        ty = (self.cam.res_y + tile_h - 1) // tile_h
        out = np.zeros(tx * ty, dtype=np.float32)
        _check_hip(_hip.rt_tile_costs(self._h, ctypes.byref(self.cam), int(tile_w), int(tile_h),
                                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))), "rt_tile_costs")
        return out


    def wait(self) -> RenderStats:
        """rt_render_wait: finish this scene's deferred call (RenderParams(sync=False)) and return
        its statistics (zeros when nothing is deferred)."""
        st = rt_stats()
        _check_hip(_hip.rt_render_wait(self._h, ctypes.byref(st)), "rt_render_wait")
        return RenderStats.of(st)

    def tile_costs_measured(self, tile_w: int, tile_h: int, spp_sqrt: int) -> np.ndarray:
        """rt_tile_costs_measured: BVH4 node visits per tile (tile id order) of the last
        instrumented (count_work) one-pass render of this camera / tile size / spp; -1 where
        that render did not cover the tile (or there was none)."""
        if int(tile_w) <= 0 or int(tile_h) <= 0:
            raise NativeError(f"rt_tile_costs_measured: tile size must be positive (got {tile_w}x{tile_h})")
        tx = (self.cam.res_x + tile_w - 1) // tile_w
        ty = (self.cam.res_y + tile_h - 1) // tile_h
        out = np.zeros(tx * ty, dtype=np.float32)
        _check_hip(_hip.rt_tile_costs_measured(self._h, ctypes.byref(self.cam), int(tile_w), int(tile_h), int(spp_sqrt),
                                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))), "rt_tile_costs_measured")
        return out


def unpack_tiles(packed: np.ndarray, tile_ids, tile_w: int, tile_h: int, width: int, height: int) -> np.ndarray:
    _load()
    ids = np.ascontiguousarray(np.asarray(tile_ids, dtype=np.int32))
    img = np.zeros((height, width, 3), dtype=np.float32)
    packed = np.ascontiguousarray(packed, dtype=np.float32)
    _check_host(_host.rth_unpack_tiles(packed.ctypes.data, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                       int(ids.size), int(tile_w), int(tile_h), int(width), int(height),
                                       img.ctypes.data), "rth_unpack_tiles")
    return img


def quantise(rgb: np.ndarray) -> np.ndarray:
    """Gamma 1/1.1 (glibc-exact powf), clamp, *255.999 -> uint8, same shape."""
    _load()
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    out = np.empty(a.shape, dtype=np.uint8)
    _check_host(_host.rth_quantise(a.ctypes.data, int(a.size), out.ctypes.data), "rth_quantise")
    return out


def quantise_device(d_rgb: int, n: int, d_u8: int, stream: int = 0):
    """Device-side quantise (rt_quantise_device): n floats at device pointer d_rgb -> n bytes
    at d_u8, byte-identical to quantise(); enqueued on `stream` (0 = default)."""
    _load()
    _check_hip(_hip.rt_quantise_device(d_rgb, int(n), d_u8, stream or None), "rt_quantise_device")


def write_ppm(path: str, u8: np.ndarray):
    _load()
    a = np.ascontiguousarray(u8, dtype=np.uint8)
    h, w = a.shape[:2]
    _check_host(_host.rth_write_ppm(path.encode(), int(w), int(h), a.ctypes.data), "rth_write_ppm")


def make_soup(path: str, n_triangles: int, seed: int = 20251226, width: int = 1024, height: int = 1024):
    """Synthetic triangle-soup scene.json."""
    _load()
    _check_host(_host.rth_make_soup(path.encode(), int(n_triangles), int(seed), int(width), int(height)),
                "rth_make_soup")
