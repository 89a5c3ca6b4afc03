"""The 64-byte rt_node4 tree the host builds (bvh_wide.cpp, layout in include/rt_hip.h), read
back through rth_scene_desc and checked on the CPU -- the kernel follows these indices
unchecked, and its culling is only exact if every box is conservative:
  * meta bytes are 0, 0x01 (internal child, index after its parent) or 0x80 | n (leaf);
    every node but the root has exactly one parent;
  * the leaf ranges (child[k], n) cover every bounded primitive exactly once (except planes
    that accept no point, kept only for indexing);
  * every Plane primitive's corners lie inside the dequantised grid box of every ancestor slot
    on the path of one of its parts (origin + q * 2^(e - 127), evaluated in double); spatial
    splits store a primitive once per part.
rt_scene_create repeats the structural part as its input validation.
"""
import ctypes

import numpy as np
import pytest

import scenes

NODE = np.dtype([("origin", "<f4", 3), ("exps", "<u4"), ("q", "<u4", 6), ("meta", "<u4"), ("child", "<i4", 4),
                 ("pad", "<u4")])
assert NODE.itemsize == 64


def _arrays(sc):
    d = sc.desc()
    nodes = np.frombuffer(ctypes.string_at(d.nodes, d.n_nodes * 64), dtype=NODE) if d.n_nodes else None
    prims = np.frombuffer(ctypes.string_at(d.prims, d.n_prims * d.prim_stride), dtype="<f4").reshape(
        d.n_prims, d.prim_stride // 4)
    refs = np.frombuffer(ctypes.string_at(d.prim_refs, d.n_prims * 8), dtype="<i4").reshape(d.n_prims, 2)
    return d, nodes, prims, refs


def _slot_box(nd, k):
    lo, hi = np.empty(3), np.empty(3)
    for a in range(3):
        step = 2.0 ** (int((nd["exps"] >> (8 * a)) & 255) - 127)
        lo[a] = float(nd["origin"][a]) + ((int(nd["q"][2 * a]) >> (8 * k)) & 255) * step
        hi[a] = float(nd["origin"][a]) + ((int(nd["q"][2 * a + 1]) >> (8 * k)) & 255) * step
    return lo, hi


def check_tree(sc):
    d, nodes, prims, refs = _arrays(sc)
    n_bounded = d.n_prims - d.n_unbounded
    if d.n_nodes == 0:
        assert n_bounded == 0
        return 0
    parents = np.zeros(d.n_nodes, np.int64)
    covered = np.zeros(d.n_prims, np.int64)
    is_plane = (prims[:, 15].view(np.uint32) & 3) == 3
    corners = prims[:, [0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14]].reshape(-1, 4, 3).astype(np.float64)
    tri1 = (prims[:, 15].view(np.uint32) & 16) != 0  # RT_TAG_TRI1_NEVER: c3 == c0, a[12] holds a radius
    corners[tri1, 3] = corners[tri1, 0]
    checked = 0
    # spatial splits: a primitive may sit in several leaves (parts); every corner of a plane
    # must lie inside all ancestor boxes of at least one of its parts
    corner_ok = {}
    stack = [(0, [])]  # (node, ancestor boxes)
    while stack:
        i, boxes = stack.pop()
        nd = nodes[i]
        meta = int(nd["meta"])
        for k in range(4):
            m = (meta >> (8 * k)) & 255
            c = int(nd["child"][k])
            if m == 0:
                continue
            box = _slot_box(nd, k)
            assert (box[0] <= box[1]).all()
            if m == 0x01:
                assert i < c < d.n_nodes
                parents[c] += 1
                stack.append((c, boxes + [box]))
            else:
                n = m & 0x7F
                cu = c & 0xFFFFFFFF  # leaf entry: 0x80000000 | first << 7 | n
                assert m & 0x80 and n >= 1 and cu & 0x80000000 and (cu & 0x7F) == n
                c = (cu & 0x7FFFFFFF) >> 7
                assert c + n <= n_bounded
                covered[c:c + n] += 1
                for p in range(c, c + n):
                    if not is_plane[p]:
                        continue
                    inside = np.ones(4, bool)
                    for lo, hi in boxes + [box]:
                        inside &= ((corners[p] >= lo) & (corners[p] <= hi)).all(axis=1)
                    r = int(refs[p, 0])
                    corner_ok[r] = corner_ok.get(r, np.zeros(4, bool)) | inside
                    checked += 1
    for r, ok in corner_ok.items():
        assert ok.all(), (r, ok)
    assert parents[0] == 0 and (parents[1:] == 1).all()
    # uncovered bounded slots may only be planes that accept no point (kept for indexing)
    assert (covered <= 1).all() and (covered[n_bounded:] == 0).all()
    assert is_plane[:n_bounded][covered[:n_bounded] == 0].all()
    return checked


@pytest.mark.parametrize("name", ["soup_s1", "features_s1", "ascii_k1_bvh", "blend_c3_antialiasing",
                                  "blend_c4_glossy_soft", "blend_test1"])
def test_node_tree_invariants(name, tmp_path):
    import ray_tracying_amd as rt
    path, _ = scenes.materialise(name, str(tmp_path))
    sc = rt.Scene(path, texture_root=scenes.TEXTURES)
    try:
        check_tree(sc)
    finally:
        sc.close()


def test_node_tree_soup_large(tmp_path):
    import ray_tracying_amd as rt
    path = str(tmp_path / "soup.json")
    rt.make_soup(path, 20000, seed=7, width=64, height=64)
    sc = rt.Scene(path)
    try:
        assert check_tree(sc) > 15000  # nearly every triangle is a bounded Plane
    finally:
        sc.close()


def test_spatial_splits_store_parts(tmp_path, monkeypatch):
    """Spatial splits (bvh_wide.cpp) store some primitives once per part; every primitive
    stays reachable, the tree invariants hold, and RT_SBVH_DUP=0 turns them off."""
    import ray_tracying_amd as rt
    p = scenes.write(scenes.soup(3000, seed=11, res=(48, 48)), str(tmp_path / "s.json"))
    counts = {}
    for dup in ("0", "0.3"):
        monkeypatch.setenv("RT_SBVH_DUP", dup)
        sc = rt.Scene(p)
        try:
            check_tree(sc)
            d, _, _, refs = _arrays(sc)
            counts[dup] = d.n_prims
            assert set(np.unique(refs[:, 0]).tolist()) == set(range(3000))
        finally:
            sc.close()
    assert counts["0"] == 3000 and 3000 < counts["0.3"] <= 3900
