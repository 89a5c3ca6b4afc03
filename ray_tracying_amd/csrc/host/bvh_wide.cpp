// bvh_wide.cpp -- traversal BVH for the MI355X kernel: binned-SAH BVH2 collapsed to 4-wide
// nodes (rt_node4, 64 B, 8-bit conservative child grids), built over conservative per-primitive HIT boxes.
//
// Exactness contract: the reference accepts a primitive hit only
// if the primitive's leaf box in the REFERENCE's median-split tree passes the exact slab test
// (acceleration.cpp:67-100 + shapes.cpp:55-72); the kernel re-checks exactly that box for every
// candidate hit, so this tree only has to be conservative: every point a primitive test can
// report as a hit must lie inside every box on its path (pruning by t_near relies on it).
//   * Plane (shapes.cpp:444-494): isPointInQuad accepts P iff one of two sub-triangles'
//     edge functions are all >= -1e-6; each sub-triangle's acceptance region is the
//     intersection of three offset half-planes, computed exactly (tri_region, with a 2x
//     tolerance for float rounding).  The box is the union of the two regions.  Regions that
//     are unbounded (parallel or zero-length edges, e.g. the `c3 == c2` trap of SURVEY.md 8(a)
//     a13) send the plane to the "unbounded" list that every ray tests; planes that accept
//     nothing (invalid normal, empty regions) are never traversed.
//   * Sphere / Cube / Rectangle: the reference's own bbox (swept over time for moving spheres)
//     + rounding margin.  Non-finite boxes (zero scale) -> unbounded list.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <vector>

#include "scene.hpp"

namespace rth {

namespace {

struct BuildPrim {
  Box box;
  V3 c;  // centroid
  int id;
};

inline float area(const Box& b) {
  float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0f;
  return 2.0f * (dx * dy + dy * dz + dz * dx);
}

struct Node2 {
  Box box;
  int left = -1, right = -1;  // internal: children
  int start = 0, count = 0;   // leaf: range in `order`
};

struct SAHBuilder {
  std::vector<BuildPrim>& P;
  std::vector<Node2> nodes;
  static constexpr int kBinsMax = 64;
  int kBins = 32;          // RT_SAH_BINS (tuning knob; 16 -> 32 and node 1.0 -> 0.5: +1.2%)
  int kMaxLeaf = 4;        // RT_SAH_LEAF
  float kNodeCost = 0.5f;  // RT_SAH_NODE: traversal step cost relative to one primitive test

  int build(int start, int end, int depth) {
    int id = (int)nodes.size();
    nodes.emplace_back();
    Box b, cb;
    for (int i = start; i < end; ++i) {
      b.merge(P[i].box);
      cb.merge(P[i].c);
    }
    nodes[id].box = b;
    const int n = end - start;
    if (n <= 1 || depth > 60) {
      nodes[id].start = start;
      nodes[id].count = n;
      if (n <= kMaxLeaf) return id;
    }
    // binned SAH over all three axes
    float best_cost = INFINITY;
    int best_axis = -1, best_bin = -1;
    for (int ax = 0; ax < 3; ++ax) {
      float lo = cb.lo[ax], hi = cb.hi[ax];
      if (!(hi > lo)) continue;
      float scale = kBins / (hi - lo);
      Box bb[kBinsMax];
      int cnt[kBinsMax] = {0};
      for (int i = start; i < end; ++i) {
        int k = std::min(kBins - 1, (int)((P[i].c[ax] - lo) * scale));
        bb[k].merge(P[i].box);
        cnt[k]++;
      }
      float ra[kBinsMax];
      int rc[kBinsMax];
      Box acc;
      int c = 0;
      for (int k = kBins - 1; k > 0; --k) {
        acc.merge(bb[k]);
        c += cnt[k];
        ra[k] = area(acc);
        rc[k] = c;
      }
      Box accl;
      int cl = 0;
      for (int k = 0; k < kBins - 1; ++k) {
        accl.merge(bb[k]);
        cl += cnt[k];
        if (cl == 0 || rc[k + 1] == 0) continue;
        float cost = area(accl) * cl + ra[k + 1] * rc[k + 1];
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = ax;
          best_bin = k;
        }
      }
    }
    const float leaf_cost = area(b) * n;
    const float node_cost = area(b) * kNodeCost;  // traversal step relative to one primitive test
    if (n <= kMaxLeaf && (best_axis < 0 || best_cost * 1.0f + node_cost >= leaf_cost)) {
      nodes[id].start = start;
      nodes[id].count = n;
      return id;
    }
    int mid;
    if (best_axis < 0) {  // all centroids coincide: split the index range
      mid = start + n / 2;
    } else {
      float lo = cb.lo[best_axis], scale = kBins / (cb.hi[best_axis] - lo);
      auto it = std::partition(P.begin() + start, P.begin() + end, [&](const BuildPrim& p) {
        return std::min(kBins - 1, (int)((p.c[best_axis] - lo) * scale)) <= best_bin;
      });
      mid = (int)(it - P.begin());
      if (mid == start || mid == end) mid = start + n / 2;
    }
    int l = build(start, mid, depth + 1);
    int r = build(mid, end, depth + 1);
    nodes[id].left = l;
    nodes[id].right = r;
    nodes[id].count = 0;
    return id;
  }
};

// Accepted region of isPointInTriangle(P, A, B, C, n) (shapes.cpp:24-40) for P in the plane:
// dot(cross(E_i, P - V_i), n) >= -tol for the three edges (E_1 = B-A at A, E_2 = C-B at B,
// E_3 = A-C at C).  With w_i = cross(n, E_i) each is the half-plane dot(P, w_i) >= dot(V_i, w_i)
// - tol; three half-planes whose normals positively span the plane intersect in a bounded
// triangle (possibly empty) whose vertices are pairwise line intersections.  Works for either
// winding.  Returns false if the region is unbounded (parallel / zero-length edges).
bool tri_region(const double A[3], const double B[3], const double C[3], const double n[3], double tol,
                Box& box, bool& nonempty) {
  auto sub = [](const double* a, const double* b, double* o) { o[0] = a[0] - b[0]; o[1] = a[1] - b[1]; o[2] = a[2] - b[2]; };
  auto cross = [](const double* a, const double* b, double* o) {
    o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0];
  };
  auto dot = [](const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
  const double* V[3] = {A, B, C};
  double E[3][3], W[3][3], c[3];
  sub(B, A, E[0]);
  sub(C, B, E[1]);
  sub(A, C, E[2]);
  // in-plane orthonormal basis (u, v) around A
  double u[3], v[3];
  {
    double t[3] = {std::fabs(n[0]) < 0.9 ? 1.0 : 0.0, std::fabs(n[0]) < 0.9 ? 0.0 : 1.0, 0.0};
    cross(n, t, u);
    double lu = std::sqrt(dot(u, u));
    if (!(lu > 0)) return false;
    for (double& x : u) x /= lu;
    cross(n, u, v);
  }
  double w2[3][2];
  for (int i = 0; i < 3; ++i) {
    cross(n, E[i], W[i]);
    w2[i][0] = dot(W[i], u);
    w2[i][1] = dot(W[i], v);
    double d[3];
    sub(V[i], A, d);
    c[i] = dot(d, W[i]) - tol;  // constraint: w2_i . (a, b) >= c_i, with P = A + a u + b v
  }
  auto cr = [&](int i, int j) { return w2[i][0] * w2[j][1] - w2[i][1] * w2[j][0]; };
  const double k01 = cr(0, 1), k12 = cr(1, 2), k20 = cr(2, 0);
  const double scale = std::max({std::fabs(k01), std::fabs(k12), std::fabs(k20)});
  if (!(scale > 0) || !((k01 > 1e-9 * scale && k12 > 1e-9 * scale && k20 > 1e-9 * scale) ||
                        (k01 < -1e-9 * scale && k12 < -1e-9 * scale && k20 < -1e-9 * scale)))
    return false;
  nonempty = false;
  const int pr[3][3] = {{0, 1, 2}, {1, 2, 0}, {2, 0, 1}};
  for (auto& q : pr) {
    const int i = q[0], j = q[1], k = q[2];
    const double det = cr(i, j);
    const double a = (c[i] * w2[j][1] - c[j] * w2[i][1]) / det;
    const double b = (w2[i][0] * c[j] - w2[j][0] * c[i]) / det;
    if (w2[k][0] * a + w2[k][1] * b < c[k] - 1e-9 * (std::fabs(c[k]) + 1e-30)) continue;
    nonempty = true;
    V3 P;
    for (int m = 0; m < 3; ++m) P[m] = (float)(A[m] + a * u[m] + b * v[m]);
    box.merge(P);
  }
  return true;
}

}  // namespace

// Grid coordinate origin + q * step as a real number (double: exact for the 8-bit code and a
// power-of-two step unless the exponents are ~29 apart, and then off by < 2^-53 relative).
// The trace kernel never rounds this value: it folds it into the slab as
// fma(q, step * inv, (origin - o) * inv) (rt_hip.hip), whose rounding, like the plain
// slab form's, is orders of magnitude inside the 1e-5 * scale box padding.
static inline double grid_value(float origin, uint32_t q, float step) { return (double)origin + (double)q * (double)step; }

// Per-axis 8-bit grid codes for the first n child boxes of `out` (rt_hip.h, rt_node4): every
// grid lo is <= the box's lo and every grid hi >= its hi.
// Unused slots get an empty box (lo code 255, hi code 0; their meta byte is 0 anyway).
static void quantise_children(rt_node4& out, const Box* cb, int n) {
  uint32_t qlo[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, qhi[3] = {0, 0, 0};
  uint32_t exps = 0;
  for (int a = 0; a < 3; ++a) {
    float lo = cb[0].lo[a], hi = cb[0].hi[a];
    for (int k = 1; k < n; ++k) {
      lo = std::min(lo, cb[k].lo[a]);
      hi = std::max(hi, cb[k].hi[a]);
    }
    const float origin = lo;
    // smallest power-of-two step whose 255 steps span the extent; grown until every
    // child bound is representable conservatively
    const double ext = (double)hi - (double)lo;
    int e = ext > 0 ? (int)std::ceil(std::log2(ext / 255.0)) : -126;
    e = std::max(e, -126);
    uint32_t codes_lo = 0, codes_hi = 0;
    for (;; ++e) {
      if (e > 80) throw std::runtime_error("BVH node grid: scene extent too large (> 2^88)");
      const float step = std::ldexp(1.0f, e);
      bool ok = true;
      codes_lo = codes_hi = 0;
      for (int k = 0; k < 4 && ok; ++k) {
        uint32_t ql = 255, qh = 0;
        if (k < n) {
          const double fl = std::floor(((double)cb[k].lo[a] - (double)origin) / (double)step);
          ql = (uint32_t)std::max(0.0, std::min(255.0, fl));
          while (ql > 0 && grid_value(origin, ql, step) > cb[k].lo[a]) --ql;
          if (grid_value(origin, ql, step) > cb[k].lo[a]) ok = false;
          const double ch = std::ceil(((double)cb[k].hi[a] - (double)origin) / (double)step);
          qh = (uint32_t)std::max(0.0, std::min(255.0, ch));
          while (qh < 255 && grid_value(origin, qh, step) < cb[k].hi[a]) ++qh;
          if (grid_value(origin, qh, step) < cb[k].hi[a]) ok = false;
        }
        codes_lo |= ql << (8 * k);
        codes_hi |= qh << (8 * k);
      }
      if (ok) break;
    }
    out.origin[a] = origin;
    exps |= (uint32_t)(e + 127) << (8 * a);
    qlo[a] = codes_lo;
    qhi[a] = codes_hi;
  }
  out.exps = exps;
  out.q_lo_x = qlo[0]; out.q_hi_x = qhi[0];
  out.q_lo_y = qlo[1]; out.q_hi_y = qhi[1];
  out.q_lo_z = qlo[2]; out.q_hi_z = qhi[2];
}

// Fills sc.node4 / sc.prims order / prim_refs / ref_leaf_boxes / n_unbounded.
// `ref_order` = the reference's BVH-sorted shape order, `ref_leaf_of` = reference leaf id per
// sorted position, `ref_leaf_boxes` = the exact reference leaf boxes.
void build_wide(Scene& sc, const std::vector<Box>& shape_box, const std::vector<int>& ref_leaf_of) {
  const int n = (int)sc.order.size();
  const float margin = 1e-5f * sc.scene_scale;
  std::vector<BuildPrim> bounded;
  std::vector<Box> accept_box(n);          // unpadded acceptance region (planes)
  std::vector<uint8_t> has_accept(n, 0);
  std::vector<int> unbounded;  // sorted positions
  std::vector<int> never;      // planes that accept no point: kept for indexing, never traversed
  bounded.reserve(n);
  for (int r = 0; r < n; ++r) {
    const Shape& s = sc.shapes[sc.order[r]];
    Box b = shape_box[sc.order[r]];
    bool ok = true;
    float pad = margin;
    if (s.kind == RT_PRIM_PLANE) {
      // isPointInQuad = triangle (c1,c3,c2) OR triangle (c0,c1,c2) (shapes.cpp:485-494); the
      // acceptance regions (2x the reference's 1e-6 tolerance for float rounding) bound every
      // hit point.  Invalid planes (|cross| < 1e-6f) never hit and are left out entirely.
      uint32_t tag;
      std::memcpy(&tag, &sc.prims[r].a[15], 4);
      if (!(tag & RT_TAG_PLANE_VALID)) { never.push_back(r); continue; }
      const V3* c = s.corners;
      double C[4][3], nn[3];
      for (int q = 0; q < 4; ++q)
        for (int m = 0; m < 3; ++m) C[q][m] = c[q][m];
      double e1[3] = {C[1][0] - C[0][0], C[1][1] - C[0][1], C[1][2] - C[0][2]};
      double e2[3] = {C[2][0] - C[0][0], C[2][1] - C[0][1], C[2][2] - C[0][2]};
      nn[0] = e1[1] * e2[2] - e1[2] * e2[1];
      nn[1] = e1[2] * e2[0] - e1[0] * e2[2];
      nn[2] = e1[0] * e2[1] - e1[1] * e2[0];
      double ln = std::sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
      for (double& x : nn) x /= ln;
      Box region;
      bool ne1 = false, ne2 = false;
      ok = tri_region(C[1], C[3], C[2], nn, 2e-6, region, ne1) && tri_region(C[0], C[1], C[2], nn, 2e-6, region, ne2);
      if (ok && !ne1 && !ne2) { never.push_back(r); continue; }  // accepts nothing
      if (ok) {
        b = region;
        accept_box[r] = region;
        has_accept[r] = 1;
      }
    }
    for (int i = 0; i < 3; ++i) {
      b.lo[i] -= pad + std::fabs(b.lo[i]) * 2e-6f;
      b.hi[i] += pad + std::fabs(b.hi[i]) * 2e-6f;
      if (!std::isfinite(b.lo[i]) || !std::isfinite(b.hi[i])) ok = false;
    }
    if (!ok) {
      unbounded.push_back(r);
      continue;
    }
    BuildPrim bp;
    bp.box = b;
    bp.c = {0.5f * (b.lo[0] + b.hi[0]), 0.5f * (b.lo[1] + b.hi[1]), 0.5f * (b.lo[2] + b.hi[2])};
    bp.id = r;
    bounded.push_back(bp);
  }
  SAHBuilder B{bounded, {}};
  if (const char* e = std::getenv("RT_SAH_BINS")) B.kBins = std::max(2, std::min(SAHBuilder::kBinsMax, std::atoi(e)));
  if (const char* e = std::getenv("RT_SAH_LEAF")) B.kMaxLeaf = std::max(1, std::min(15, std::atoi(e)));
  if (const char* e = std::getenv("RT_SAH_NODE")) B.kNodeCost = (float)std::atof(e);
  B.nodes.reserve(bounded.size() + 1);
  if (!bounded.empty()) B.build(0, (int)bounded.size(), 0);

  // new primitive order: leaves of the SAH tree (DFS), then the unbounded list
  std::vector<int> new_order;  // new index -> sorted reference position r
  new_order.reserve(n);
  for (auto& bp : bounded) new_order.push_back(bp.id);  // leaves are contiguous ranges of `bounded`
  for (int r : never) new_order.push_back(r);
  for (int r : unbounded) new_order.push_back(r);  // the last n_unbounded, tested by every ray
  sc.n_unbounded = (int)unbounded.size();

  // collapse BVH2 -> BVH4
  sc.node4.clear();
  sc.stack_bound = 1;
  if (!bounded.empty()) {
    struct Item { int n2; int slot; int depth; };
    std::vector<Item> todo;
    auto emit = [&](int n2, int depth) -> int {
      int id = (int)sc.node4.size();
      sc.node4.emplace_back();
      todo.push_back({n2, id, depth});
      return id;
    };
    // a root that is a leaf becomes a single-child node
    emit(0, 1);
    int max_depth = 1;
    while (!todo.empty()) {
      Item it = todo.back();
      todo.pop_back();
      max_depth = std::max(max_depth, it.depth);
      std::vector<int> kids;
      const Node2& root = B.nodes[it.n2];
      if (root.left < 0) {
        kids.push_back(it.n2);
      } else {
        kids = {root.left, root.right};
        while (kids.size() < 4) {
          int best = -1;
          float ba = -1;
          for (int k = 0; k < (int)kids.size(); ++k) {
            const Node2& c = B.nodes[kids[k]];
            if (c.left >= 0 && area(c.box) > ba) { ba = area(c.box); best = k; }
          }
          if (best < 0) break;
          int nb = kids[best];
          kids.erase(kids.begin() + best);
          kids.push_back(B.nodes[nb].left);
          kids.push_back(B.nodes[nb].right);
        }
      }
      rt_node4 out{};
      uint32_t meta = 0;
      Box cb[4];
      int nk = 0;
      for (int k = 0; k < 4; ++k) {
        if (k >= (int)kids.size()) {
          out.child[k] = -1;
          continue;
        }
        const Node2& c = B.nodes[kids[k]];
        cb[nk++] = c.box;
        if (c.left < 0) {
          // leaf entry: 0x80000000 | first primitive << 7 | count (new order == bounded order)
          out.child[k] = (int32_t)(0x80000000u | ((uint32_t)c.start << 7) | (uint32_t)c.count);
          meta |= (0x80u | (uint32_t)c.count) << (8 * k);
        } else {
          out.child[k] = emit(kids[k], it.depth + 1);
          meta |= 0x01u << (8 * k);
        }
      }
      quantise_children(out, cb, nk);
      out.meta = meta;
      sc.node4[it.slot] = out;
    }
    sc.stack_bound = 3 * max_depth + 2;
    sc.tree_depth = max_depth;
  }

  // reorder primitive records; keep (reference index, reference leaf) per primitive
  std::vector<rt_prim> prims(n);
  sc.prim_refs.assign(n, rt_prim_ref{});
  for (int i = 0; i < n; ++i) {
    int r = new_order[i];
    prims[i] = sc.prims[r];
    sc.prim_refs[i].ref_index = r;
    sc.prim_refs[i].ref_leaf = ref_leaf_of[r];
    // The reference-leaf filter (AABB::intersect on the primitive's leaf box, shapes.cpp:55-72)
    // is provably true for every hit this primitive can report when its acceptance region
    // lies inside the leaf box shrunk by delta: along an axis with |d| >= 1e-6 the computed
    // slab bounds are off by at most |bound - o| * 2^-23 <= 2 * scale * 2^-23 << delta, and
    // along a near-parallel axis the origin is within |P - o| * 1e-6 <= 2e-6 * scale of the
    // hit point (unit directions, |P - o| <= 2 * scale).  Such primitives carry ref_leaf = -1
    // and the kernel skips the check (for c3 == c0 triangles the reference pads every plane
    // box by 1e-4, so triangle soups qualify).
    if (has_accept[r]) {
      const double delta = 1e-5 * std::max(1.0, (double)sc.scene_scale);
      const float* lb = &sc.ref_leaf_boxes[(size_t)ref_leaf_of[r] * 8];
      bool inside = true;
      for (int a = 0; a < 3; ++a)
        inside = inside && (double)accept_box[r].lo[a] >= (double)lb[a] + delta &&
                 (double)accept_box[r].hi[a] <= (double)lb[4 + a] - delta;
      if (inside) sc.prim_refs[i].ref_leaf = -1;
    }
  }
  sc.prims.swap(prims);
}

}  // namespace rth
