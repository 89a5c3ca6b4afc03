#!/usr/bin/env python3
"""width_study.py -- node visits per ray of the headline soup's traversal tree at 4 and 8
children per node, before building an 8-wide kernel ("measure before
building").

The BVH4 is the one the kernel walks (rth_scene_desc: bvh_wide.cpp's SAH BVH2 with spatial
splits, collapsed to 4 wide; child boxes decoded from the 8-bit grid codes exactly as the host
wrote them).  The BVH8 is collapsed from it: every 4-wide node takes in the children of its
largest-area internal children while it has slots (at most 8), and the internal children left
become 8-wide nodes in turn -- the greedy collapse that halves the levels of a balanced tree.
Both trees are walked on the CPU by the kernel's algorithm -- near-first (children entered
within the bound ordered by entry distance), pruned by the best hit, closest hit for camera rays
and any hit within the light distance for the shadow ray of every camera hit -- over camera rays
through random pixels of the headline frame (1024^2, the soup's own camera; one jittered sample
per pixel).  Triangle tests are Moller-Trumbore in binary64: the visit counts need the
traversal's pruning, not the reference's bits.

Usage: python3 tools/width_study.py [--rays 3000] [--tris 1000000] [--out profiles/x.json]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ray_tracying_amd as rt  # noqa: E402

NODE = np.dtype([("origin", "<f4", 3), ("exps", "<u4"), ("q", "<u4", 6), ("meta", "<u4"), ("child", "<i4", 4),
                 ("pad", "<u4")])


def load_tree(sc):
    d = sc.desc()
    nodes = np.frombuffer(ctypes.string_at(d.nodes, d.n_nodes * 64), dtype=NODE)
    prims = np.frombuffer(ctypes.string_at(d.prims, d.n_prims * d.prim_stride), dtype="<f4").reshape(
        d.n_prims, d.prim_stride // 4).astype(np.float64)
    n = len(nodes)
    lo = np.zeros((n, 4, 3))
    hi = np.zeros((n, 4, 3))
    for a in range(3):
        step = np.ldexp(1.0, ((nodes["exps"] >> (8 * a)) & 255).astype(np.int64) - 127)
        org = nodes["origin"][:, a].astype(np.float64)
        for k in range(4):
            lo[:, k, a] = org + ((nodes["q"][:, 2 * a] >> (8 * k)) & 255) * step
            hi[:, k, a] = org + ((nodes["q"][:, 2 * a + 1] >> (8 * k)) & 255) * step
    meta = nodes["meta"].astype(np.int64)
    kind = np.stack([(meta >> (8 * k)) & 255 for k in range(4)], axis=1)  # 0 none, 1 internal, 0x80|n leaf
    child = nodes["child"].astype(np.int64)
    return d, lo, hi, kind, child, prims


def children4(lo, hi, kind, child):
    """Per BVH4 node: list of (lo, hi, is_internal, ref) -- ref = node index or (first, count)."""
    out = []
    for i in range(len(kind)):
        ch = []
        for k in range(4):
            m = kind[i, k]
            if m == 0:
                continue
            if m == 1:
                ch.append((lo[i, k], hi[i, k], True, int(child[i, k])))
            else:
                cu = int(child[i, k]) & 0xFFFFFFFF
                ch.append((lo[i, k], hi[i, k], False, ((cu & 0x7FFFFFFF) >> 7, m & 0x7F)))
        out.append(ch)
    return out


def area(lo, hi):
    e = np.maximum(hi - lo, 0.0)
    return e[0] * e[1] + e[1] * e[2] + e[2] * e[0]


def collapse(ch4, width):
    """Greedy collapse of the BVH4 into `width`-wide nodes (see the module docstring)."""
    nodes, index = [], {}

    def build(i):
        if i in index:
            return index[i]
        slots = list(ch4[i])
        while True:
            best, bk = -1.0, -1
            for k, (l, h, internal, ref) in enumerate(slots):
                if internal and len(slots) - 1 + len(ch4[ref]) <= width:
                    a = area(l, h)
                    if a > best:
                        best, bk = a, k
            if bk < 0:
                break
            ref = slots[bk][3]
            slots = slots[:bk] + list(ch4[ref]) + slots[bk + 1:]
        me = len(nodes)
        index[i] = me
        nodes.append(None)
        nodes[me] = [(l, h, internal, build(ref) if internal else ref) for (l, h, internal, ref) in slots]
        return me

    sys.setrecursionlimit(100000)
    build(0)
    packed = []
    for ch in nodes:
        L = np.array([c[0] for c in ch])
        H = np.array([c[1] for c in ch])
        packed.append((L, H, [c[2] for c in ch], [c[3] for c in ch]))
    return packed


def tri_hit(prims, first, count, o, d, tmax):
    """Closest Moller-Trumbore hit among the leaf's planes (c0, c1, c2; the soup's c3 == c0)."""
    P = prims[first:first + count]
    c0, c1, c2 = P[:, 0:3], P[:, 4:7], P[:, 8:11]
    e1, e2 = c1 - c0, c2 - c0
    p = np.cross(d, e2)
    det = np.einsum("ij,ij->i", e1, p)
    ok = np.abs(det) > 1e-12
    inv = np.where(ok, 1.0 / np.where(ok, det, 1.0), 0.0)
    s = o - c0
    u = np.einsum("ij,ij->i", s, p) * inv
    qv = np.cross(s, e1)
    v = (qv @ d) * inv
    t = np.einsum("ij,ij->i", e2, qv) * inv
    hit = ok & (u >= 0) & (v >= 0) & (u + v <= 1) & (t > 1e-6) & (t <= tmax)
    return float(t[hit].min()) if hit.any() else None


def traverse(tree, prims, o, d, tmax, any_hit):
    """Near-first traversal; returns (closest t or None, internal node visits, leaf visits)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / np.where(np.abs(d) < 1e-12, np.copysign(1e-12, d), d)
    best = tmax
    found = None
    visits = leaves = 0
    stack = [(True, 0, 0.0)]  # (internal, node index or (first, count), entry distance)
    while stack:
        internal, ref, tn = stack.pop()
        if tn > best:
            continue
        if not internal:  # a leaf: its primitives
            leaves += 1
            t = tri_hit(prims, ref[0], ref[1], o, d, best)
            if t is not None and t < best:
                best = found = t
                if any_hit:
                    return found, visits, leaves
            continue
        visits += 1
        L, H, kinds, refs = tree[ref]
        t1 = (L - o) * inv
        t2 = (H - o) * inv
        tnear = np.maximum(np.minimum(t1, t2).max(axis=1), 0.0)
        tfar = np.minimum(np.maximum(t1, t2).min(axis=1), best)
        enter = np.nonzero(tnear <= tfar)[0]
        for k in enter[np.argsort(-tnear[enter], kind="stable")]:  # far first: the nearest is popped next
            stack.append((kinds[k], refs[k], float(tnear[k])))
    return found, visits, leaves


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=3000)
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    path = f"/tmp/width_study_soup_{a.tris}.json"
    if not os.path.exists(path):
        rt.make_soup(path, a.tris, seed=20251226, width=1024, height=1024)
    sc = rt.Scene(path, resolution=(1024, 1024))
    d, lo, hi, kind, child, prims = load_tree(sc)
    cam = sc.camera()
    ch4 = children4(lo, hi, kind, child)
    t0 = time.time()
    tree4 = [(np.array([c[0] for c in ch]), np.array([c[1] for c in ch]), [c[2] for c in ch], [c[3] for c in ch])
             for ch in ch4]
    tree8 = collapse(ch4, 8)
    build_s = time.time() - t0
    light = np.array(json.load(open(path))["lights"][0]["location"], dtype=np.float64)
    rng = np.random.default_rng(a.seed)
    loc = np.array(cam.location[:], dtype=np.float64)
    X, Y, Z = (np.array(v[:], dtype=np.float64) for v in (cam.x_dir, cam.y_dir, cam.z_dir))
    stats = {4: [0, 0, 0, 0], 8: [0, 0, 0, 0]}  # visits, leaves, rays, hits
    for _ in range(a.rays):
        px, py = rng.uniform(0, cam.res_x), rng.uniform(0, cam.res_y)
        nx, ny = 1.0 - 2.0 * px / cam.res_x, 1.0 - 2.0 * py / cam.res_y
        dw = X * nx * cam.half_sensor_w + Y * ny * cam.half_sensor_h + Z * cam.focal_length
        dw /= np.linalg.norm(dw)
        for w, tree in ((4, tree4), (8, tree8)):
            t, v, lv = traverse(tree, prims, loc, dw, np.inf, False)
            s = stats[w]
            s[0] += v
            s[1] += lv
            s[2] += 1
            if t is not None:
                s[3] += 1
                hp = loc + t * dw
                lvv = light - hp
                dist = float(np.linalg.norm(lvv))
                _, v2, l2 = traverse(tree, prims, hp + 1e-4 * (lvv / dist), lvv / dist, dist, True)
                s[0] += v2
                s[1] += l2
                s[2] += 1
    res = {"label": "width study (tools/width_study.py)", "tris": a.tris, "camera_rays": a.rays,
           "bvh4_nodes": len(tree4), "bvh8_nodes": len(tree8), "collapse_seconds": round(build_s, 1)}
    for w in (4, 8):
        v, lv, n, h = stats[w]
        res[f"bvh{w}"] = {"rays": n, "camera_hits": h, "node_visits_per_ray": round(v / n, 3),
                          "leaf_visits_per_ray": round(lv / n, 3)}
    res["visit_ratio_8_to_4"] = round(res["bvh8"]["node_visits_per_ray"] / res["bvh4"]["node_visits_per_ray"], 4)
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
