"""rt_tile_costs (the cost estimate behind the costliest-tiles-first order and bench.py
--deal balanced) against the renderer's own camera: its inverse projection of a primitive's
centre must land in the tile where camera_ray (Code/camera.cpp:98-179, the forward mapping
the kernels use) actually sees the primitive.

Scene: small triangles (planes with c3 == c0) placed on camera rays through chosen pixel
centres -- the rays built here from the camera basis the library exports -- plus one
triangle behind the camera and one outside the frustum.  A 1-spp primary render (no lights:
ambient 0.08 against the 0.1 background) shows which tiles the triangles cover; the non-zero
costs must be exactly those tiles, one centre each, and sum to the centres inside the frame.
"""
import numpy as np
import pytest

import ray_tracying_amd as rt
import scenes

pytestmark = pytest.mark.gpu
RES, T = 256, 32
TARGETS = [(1, 2), (5, 5), (6, 1), (3, 6), (0, 7)]  # (tile x, tile y)


def _scene(tmp_path):
    base = scenes.soup(1, seed=1, res=(RES, RES), light=False)
    p0 = scenes.write(base, str(tmp_path / "cam.json"))
    sc = rt.Scene(p0)
    cam = sc.camera()
    sc.close()
    L = np.array(cam.location, dtype=np.float64)
    X, Y, Z = (np.array(v, dtype=np.float64) for v in (cam.x_dir, cam.y_dir, cam.z_dir))
    planes = []
    for tx, ty in TARGETS:
        px, py = tx * T + T / 2, ty * T + T / 2
        nx, ny = 1 - (px / RES) * 2, 1 - (py / RES) * 2  # camera.cpp:104-105
        d = X * nx * cam.half_sensor_w + Y * ny * cam.half_sensor_h + Z * cam.focal_length
        P = L + 3.0 * d / np.linalg.norm(d)
        a = 0.03  # ~2.5 px at distance 3
        c0, c1, c2 = P + a * X, P - a / 2 * X + a * Y, P - a / 2 * X - a * Y  # centroid = P
        planes.append({"corners": [c0.tolist(), c1.tolist(), c2.tolist(), c0.tolist()]})
    behind = L - 2.0 * Z
    aside = L + 3.0 * Z + 5.0 * X
    for P in (behind, aside):
        planes.append({"corners": [(P + [0.03, 0, 0]).tolist(), (P + [0, 0, 0.03]).tolist(),
                                   (P - [0.03, 0, 0.03]).tolist(), (P + [0.03, 0, 0]).tolist()]})
    base["planes"] = planes
    return scenes.write(base, str(tmp_path / "targets.json"))


def test_tile_costs_match_camera_rays(tmp_path, gpu):
    sc = rt.Scene(_scene(tmp_path))
    try:
        img, _ = sc.render(rt.RenderParams(spp_sqrt=1, light_samples=1, use_bvh=True, seed=1))
        ds = rt.DeviceScene(sc, 0)
        try:
            cost = ds.tile_costs(T, T)
            tiles_x = RES // T
            assert cost.shape == (tiles_x * tiles_x,)
            hit = np.abs(img - np.float32(0.1)).max(axis=2) > 1e-6
            seen = {(x // T, y // T) for y, x in zip(*np.nonzero(hit))}
            assert seen == set(TARGETS)
            costly = {(int(t) % tiles_x, int(t) // tiles_x) for t in np.nonzero(cost)[0]}
            assert costly == set(TARGETS)
            assert all(cost[ty * tiles_x + tx] == 1.0 for tx, ty in TARGETS)
            assert cost.sum() == len(TARGETS)  # behind the camera / outside the frustum: not counted
            # ragged grid: length from the grid size, same centres counted
            c2 = ds.tile_costs(48, 40)
            assert c2.shape == (((RES + 47) // 48) * ((RES + 39) // 40),) and c2.sum() == len(TARGETS)
            with pytest.raises(rt.NativeError):
                ds.tile_costs(0, T)
        finally:
            ds.close()
    finally:
        sc.close()


def test_measured_tile_costs_sum_to_node_visits(tmp_path, gpu):
    """rt_tile_costs_measured: an instrumented (count_work) one-pass render leaves each tile's
    BVH4 node visits; over a whole frame they sum to the call's node_visits, and a tile left
    out of the call reads -1.  Before any instrumented call every tile reads -1."""
    import torch
    sc = rt.Scene(scenes.write(scenes.soup(3000, seed=4, res=(192, 128)), str(tmp_path / "s.json")))
    ds = rt.DeviceScene(sc, 0)
    try:
        T = 32
        n = (192 // T) * (128 // T)
        assert (ds.tile_costs_measured(T, T, 2) == -1).all()
        buf = torch.zeros(n * T * T * 3, dtype=torch.float32, device="cuda:0")
        ids = np.arange(n, dtype=np.int32)
        p = rt.RenderParams(spp_sqrt=2, light_samples=1, use_bvh=True, seed=3, count_work=True)
        st = ds.render_tiles(ids[1:], T, T, buf.data_ptr(), p)  # every tile but tile 0
        assert st.path == rt.PATH_ONE_PASS
        m = ds.tile_costs_measured(T, T, 2)
        assert m[0] == -1 and (m[1:] >= 0).all()
        assert int(m[1:].sum()) == st.node_visits and st.node_visits > 0
        assert (ds.tile_costs_measured(T, T, 3) == -1).all()  # another sample count: not measured
        st = ds.render_tiles(ids, T, T, buf.data_ptr(), p)
        m = ds.tile_costs_measured(T, T, 2)
        assert (m >= 0).all() and int(m.sum()) == st.node_visits
    finally:
        ds.close()
        sc.close()
