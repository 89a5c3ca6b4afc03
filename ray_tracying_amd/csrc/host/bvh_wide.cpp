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
#include <array>
#include <functional>
#include <string>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <system_error>
#include <thread>
#include <utility>
#include <stdexcept>
#include <vector>

#include "scene.hpp"

namespace rth {

namespace {

// spatial splits (SBVH-style): extra references allowed, as a fraction of the bounded
// primitives (RT_SBVH_DUP; 0 = object splits only)
constexpr double kSbvhDup = 0.3;

struct BuildPrim {
  Box box;  // padded box of the whole primitive
  V3 c;     // centroid
  int id;
};

inline float area(const Box& b) {
  float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0f;
  return 2.0f * (dx * dy + dy * dz + dz * dx);
}

inline Box intersect(const Box& a, const Box& b) {
  Box r;
  for (int i = 0; i < 3; ++i) {
    r.lo[i] = std::max(a.lo[i], b.lo[i]);
    r.hi[i] = std::min(a.hi[i], b.hi[i]);
  }
  return r;
}

struct Node2 {
  Box box;
  int left = -1, right = -1;  // internal: children
  int start = 0, count = 0;   // leaf: range in `leaf_refs`
};

// A reference: a primitive, or the part of it inside `clip` (spatial splits).  `box` is the
// padded box of the primitive's acceptance polygon clipped to `clip` -- every point the
// primitive test can report inside `clip` (to within rounding) lies in `box`, and the parts
// of one primitive cover its whole acceptance region, so near-first pruning stays exact.
struct Ref {
  Box box;
  Box clip;  // accumulated split slabs (unpadded), initially unbounded
  int p;     // index into the BuildPrim table
};

// Acceptance polygons of the planes (two triangles each, double; tri_region's vertices).
// Primitives without one (spheres, cubes, rectangles, degenerate regions) are never split.
struct Polys {
  std::vector<double> v;    // 9 doubles per triangle
  std::vector<int> off, n;  // per BuildPrim: first triangle, triangle count (0: no polygon)
};

// Sutherland-Hodgman against one axis-aligned plane: keeps x[axis] >= v (ge) or <= v.
static int clip_plane(const double (*in)[3], int n, double (*out)[3], int axis, double v, bool ge) {
  int m = 0;
  for (int i = 0; i < n; ++i) {
    const double* a = in[i];
    const double* b = in[(i + 1) % n];
    const double da = ge ? a[axis] - v : v - a[axis];
    const double db = ge ? b[axis] - v : v - b[axis];
    if (da >= 0) {
      for (int k = 0; k < 3; ++k) out[m][k] = a[k];
      ++m;
    }
    if ((da >= 0) != (db >= 0)) {
      const double t = da / (da - db);
      for (int k = 0; k < 3; ++k) out[m][k] = a[k] + t * (b[k] - a[k]);
      out[m][axis] = v;
      ++m;
    }
  }
  return m;
}

// Output of one (sub)tree build: nodes in DFS pre-order (children after their parent, the
// left subtree before the right one) and the leaf references in DFS order.  Subtrees built on
// other threads are appended with their indices shifted, which yields exactly the numbering
// of a sequential build: the tree does not depend on the thread count.
struct BuildOut {
  std::vector<Node2> nodes;
  std::vector<Ref> leaf_refs;
  void append(BuildOut&& o) {
    const int dn = (int)nodes.size(), dl = (int)leaf_refs.size();
    for (Node2& nd : o.nodes) {
      if (nd.left >= 0) {
        nd.left += dn;
        nd.right += dn;
      } else {
        nd.start += dl;
      }
      nodes.push_back(nd);
    }
    leaf_refs.insert(leaf_refs.end(), o.leaf_refs.begin(), o.leaf_refs.end());
    std::vector<Node2>().swap(o.nodes);
    std::vector<Ref>().swap(o.leaf_refs);
  }
};

// Run fn(chunk, begin, end) over `n` items in `chunks` contiguous chunks on their own threads
// (a chunk whose thread cannot be created runs on the calling thread).
template <class F>
static void parallel_chunks(size_t n, int chunks, F&& fn) {
  std::vector<std::thread> th;
  const size_t per = (n + chunks - 1) / chunks;
  for (int c = 1; c < chunks; ++c) {
    const size_t b = std::min(n, c * per), e = std::min(n, (c + 1) * per);
    try {
      th.emplace_back([&fn, c, b, e] { fn(c, b, e); });
    } catch (const std::system_error&) {
      fn(c, b, e);
    }
  }
  fn(0, 0, std::min(n, per));
  for (auto& t : th) t.join();
}

struct SAHBuilder {
  std::vector<BuildPrim>& P;
  const Polys& polys;
  float pad_abs;  // 1e-5 * scene scale
  static constexpr int kBinsMax = 64;
  int kBins = 32;          // RT_SAH_BINS (tuning knob; 16 -> 32 and node 1.0 -> 0.5: +1.2%)
  int kMaxLeaf = 4;        // RT_SAH_LEAF
  float kNodeCost = 0.5f;  // RT_SAH_NODE: traversal step cost relative to one primitive test
  float kSplitAlpha = 1e-5f;  // RT_SBVH_ALPHA: try spatial splits when children overlap > alpha * root area
  float root_area = 0.0f;
  int threads = 1;                    // RT_BUILD_THREADS
  std::atomic<int> spare{0};          // threads free to take a subtree
  static constexpr size_t kSpawnMin = 2048;     // smallest subtree handed to another thread
  static constexpr size_t kChunkMin = 65536;    // nodes this large bin / partition on all threads

  Box pad(Box b) const {
    for (int i = 0; i < 3; ++i) {
      b.lo[i] -= pad_abs + std::fabs(b.lo[i]) * 2e-6f;
      b.hi[i] += pad_abs + std::fabs(b.hi[i]) * 2e-6f;
    }
    return b;
  }

  // the reference `r` restricted to clip `c`; false if nothing of the primitive is left
  bool clipped(const Ref& r, const Box& c, Ref& out) const {
    out.p = r.p;
    out.clip = c;
    const int nt = polys.n[r.p];
    if (nt == 0) {  // no polygon: the whole box, trimmed to the padded slab
      out.box = intersect(P[r.p].box, pad(c));
      return true;
    }
    Box b;
    bool any = false;
    for (int t = 0; t < nt; ++t) {
      double A[16][3], B[16][3];
      const double* tv = &polys.v[(size_t)(polys.off[r.p] + t) * 9];
      for (int k = 0; k < 3; ++k)
        for (int m = 0; m < 3; ++m) A[k][m] = tv[k * 3 + m];
      int n = 3;
      for (int ax = 0; ax < 3 && n > 0; ++ax) {
        if (std::isfinite(c.lo[ax])) {
          n = clip_plane(A, n, B, ax, c.lo[ax], true);
          for (int k = 0; k < n; ++k) std::memcpy(A[k], B[k], sizeof A[k]);
        }
        if (n > 0 && std::isfinite(c.hi[ax])) {
          n = clip_plane(A, n, B, ax, c.hi[ax], false);
          for (int k = 0; k < n; ++k) std::memcpy(A[k], B[k], sizeof A[k]);
        }
      }
      for (int k = 0; k < n; ++k) {
        b.merge(V3{(float)A[k][0], (float)A[k][1], (float)A[k][2]});
        any = true;
      }
    }
    if (!any) return false;
    out.box = intersect(pad(b), P[r.p].box);
    return true;
  }

  // binning of a spatial split: the reference's polygon cut at each bin plane in turn (the
  // remainder carried on), each piece's padded box (within the reference's box) into its bin
  void sweep_bins(const Ref& r, int ax, float lo, float w, int b0, int b1, Box* bb) const {
    Box part[kBinsMax];
    for (int t = 0; t < polys.n[r.p]; ++t) {
      double A[16][3], L[16][3], Rm[16][3];
      const double* tv = &polys.v[(size_t)(polys.off[r.p] + t) * 9];
      for (int k = 0; k < 3; ++k)
        for (int m = 0; m < 3; ++m) A[k][m] = tv[k * 3 + m];
      int n = 3;
      for (int k = b0; k < b1 && n > 0; ++k) {
        const double plane = (double)lo + (double)w * (k + 1);
        const int nl = clip_plane(A, n, L, ax, plane, false);
        for (int q = 0; q < nl; ++q) part[k].merge(V3{(float)L[q][0], (float)L[q][1], (float)L[q][2]});
        n = clip_plane(A, n, Rm, ax, plane, true);
        for (int q = 0; q < n; ++q) std::memcpy(A[q], Rm[q], sizeof A[q]);
      }
      for (int q = 0; q < n; ++q) part[b1].merge(V3{(float)A[q][0], (float)A[q][1], (float)A[q][2]});
    }
    for (int k = b0; k <= b1; ++k)
      if (part[k].lo[0] <= part[k].hi[0]) bb[k].merge(intersect(pad(part[k]), r.box));
  }

  static void make_leaf(BuildOut& out, int id, std::vector<Ref>& refs) {
    out.nodes[id].start = (int)out.leaf_refs.size();
    out.nodes[id].count = (int)refs.size();
    out.leaf_refs.insert(out.leaf_refs.end(), refs.begin(), refs.end());
  }

  static float centroid(const Ref& r, int ax) { return 0.5f * (r.box.lo[ax] + r.box.hi[ax]); }

  // Object-split bins of refs[b, e) on all three axes (centroid bins over `cb`).
  struct ObjBins {
    Box bb[3][kBinsMax];
    int cnt[3][kBinsMax] = {};
  };
  void object_bins(const std::vector<Ref>& refs, size_t b, size_t e, const Box& cb, ObjBins& o) const {
    for (int ax = 0; ax < 3; ++ax) {
      const float lo = cb.lo[ax], hi = cb.hi[ax];
      if (!(hi > lo)) continue;
      const float scale = kBins / (hi - lo);
      for (size_t i = b; i < e; ++i) {
        const Ref& r = refs[i];
        const int k = std::min(kBins - 1, (int)((centroid(r, ax) - lo) * scale));
        o.bb[ax][k].merge(r.box);
        o.cnt[ax][k]++;
      }
    }
  }

  // Spatial-split bins of refs[b, e) on axis `ax` over the node box: each reference clipped
  // into every bin it spans (entering / leaving counts as in SBVH).
  struct SpBins {
    Box bb[kBinsMax];
    int enter[kBinsMax] = {}, leave[kBinsMax] = {};
  };
  void spatial_bins(const std::vector<Ref>& refs, size_t b, size_t e, int ax, float lo, float w, SpBins& o) const {
    for (size_t i = b; i < e; ++i) {
      const Ref& r = refs[i];
      int b0 = std::min(kBins - 1, std::max(0, (int)((r.box.lo[ax] - lo) / w)));
      int b1 = std::min(kBins - 1, std::max(0, (int)((r.box.hi[ax] - lo) / w)));
      if (polys.n[r.p] == 0) b0 = b1 = std::min(kBins - 1, std::max(0, (int)((centroid(r, ax) - lo) / w)));
      if (b0 == b1)
        o.bb[b0].merge(r.box);
      else
        sweep_bins(r, ax, lo, w, b0, b1, o.bb);
      o.enter[b0]++;
      o.leave[b1]++;
    }
  }

  // Partition refs[b, e) by the chosen split into L / R (spatial: straddlers clipped into
  // both sides); returns the number of references duplicated.
  long long partition(const std::vector<Ref>& refs, size_t b, size_t e, int sp_axis, float sp_pos, int best_axis,
                      int best_bin, float obj_lo, float obj_scale, std::vector<Ref>& L, std::vector<Ref>& R) const {
    long long dup = 0;
    for (size_t i = b; i < e; ++i) {
      const Ref& r = refs[i];
      if (sp_axis < 0) {
        (std::min(kBins - 1, (int)((centroid(r, best_axis) - obj_lo) * obj_scale)) <= best_bin ? L : R).push_back(r);
        continue;
      }
      if (polys.n[r.p] == 0) {
        (centroid(r, sp_axis) < sp_pos ? L : R).push_back(r);
        continue;
      }
      if (r.box.hi[sp_axis] <= sp_pos) { L.push_back(r); continue; }
      if (r.box.lo[sp_axis] >= sp_pos) { R.push_back(r); continue; }
      Box cl = r.clip, cr = r.clip;
      cl.hi[sp_axis] = std::min(cl.hi[sp_axis], sp_pos);
      cr.lo[sp_axis] = std::max(cr.lo[sp_axis], sp_pos);
      Ref a, c;
      const bool ha = clipped(r, cl, a), hc = clipped(r, cr, c);
      if (ha) L.push_back(a);
      if (hc) R.push_back(c);
      if (ha && hc) ++dup;
      if (!ha && !hc) L.push_back(r);  // cannot happen for a nonempty polygon; keep it anyway
    }
    return dup;
  }

  // Builds the subtree over `refs` into `out` (its root is out.nodes[returned id]).
  // `budget` = duplicate references this subtree may still create by spatial splits; it is
  // shared between the two children in proportion to their sizes, so the tree is the same
  // for every thread count (and a chosen split never exceeds it: candidates whose straddling
  // references outnumber the budget are skipped).
  int build(std::vector<Ref> refs, int depth, long long budget, BuildOut& out) {
    const int id = (int)out.nodes.size();
    out.nodes.emplace_back();
    Box b, cb;
    for (const Ref& r : refs) {
      b.merge(r.box);
      cb.merge(V3{centroid(r, 0), centroid(r, 1), centroid(r, 2)});
    }
    out.nodes[id].box = b;
    if (depth == 0) root_area = area(b);
    const int n = (int)refs.size();
    if (n <= 1 || depth > 60) {
      make_leaf(out, id, refs);
      return id;
    }
    // chunk threads are bounded by the idle build threads (subtrees running on spawned threads
    // hold the others), so the process never runs much more than `threads` threads at once
    const int idle = 1 + std::max(0, spare.load());
    const bool wide = (size_t)n >= kChunkMin && threads > 1 && idle > 1;
    const int chunks = wide ? std::min(threads, idle) : 1;
    // object split: binned SAH over all three axes
    ObjBins ob;
    if (wide) {
      std::vector<ObjBins> part(chunks);
      parallel_chunks(refs.size(), chunks, [&](int c, size_t s, size_t e) { object_bins(refs, s, e, cb, part[c]); });
      for (const ObjBins& p : part)
        for (int ax = 0; ax < 3; ++ax)
          for (int k = 0; k < kBins; ++k) {
            ob.bb[ax][k].merge(p.bb[ax][k]);
            ob.cnt[ax][k] += p.cnt[ax][k];
          }
    } else {
      object_bins(refs, 0, refs.size(), cb, ob);
    }
    float best_cost = INFINITY;
    int best_axis = -1, best_bin = -1;
    Box best_l, best_r;
    for (int ax = 0; ax < 3; ++ax) {
      if (!(cb.hi[ax] > cb.lo[ax])) continue;
      Box rb[kBinsMax];
      int rc[kBinsMax];
      Box acc;
      int c = 0;
      for (int k = kBins - 1; k > 0; --k) {
        acc.merge(ob.bb[ax][k]);
        c += ob.cnt[ax][k];
        rb[k] = acc;
        rc[k] = c;
      }
      Box accl;
      int cl = 0;
      for (int k = 0; k < kBins - 1; ++k) {
        accl.merge(ob.bb[ax][k]);
        cl += ob.cnt[ax][k];
        if (cl == 0 || rc[k + 1] == 0) continue;
        float cost = area(accl) * cl + area(rb[k + 1]) * rc[k + 1];
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = ax;
          best_bin = k;
          best_l = accl;
          best_r = rb[k + 1];
        }
      }
    }
    // spatial split: bins over the node box, references clipped into every bin they span
    int sp_axis = -1;
    float sp_pos = 0.0f;
    if (budget > 0 && best_axis >= 0 && area(intersect(best_l, best_r)) > kSplitAlpha * root_area) {
      for (int ax = 0; ax < 3; ++ax) {
        const float lo = b.lo[ax], hi = b.hi[ax];
        if (!(hi > lo)) continue;
        const float w = (hi - lo) / kBins;
        SpBins sb;
        if (wide) {
          std::vector<SpBins> part(chunks);
          parallel_chunks(refs.size(), chunks,
                          [&](int c, size_t s, size_t e) { spatial_bins(refs, s, e, ax, lo, w, part[c]); });
          for (const SpBins& p : part)
            for (int k = 0; k < kBins; ++k) {
              sb.bb[k].merge(p.bb[k]);
              sb.enter[k] += p.enter[k];
              sb.leave[k] += p.leave[k];
            }
        } else {
          spatial_bins(refs, 0, refs.size(), ax, lo, w, sb);
        }
        Box rb[kBinsMax];
        int rc[kBinsMax];
        Box acc;
        int c = 0;
        for (int k = kBins - 1; k > 0; --k) {
          acc.merge(sb.bb[k]);
          c += sb.leave[k];
          rb[k] = acc;
          rc[k] = c;
        }
        Box accl;
        int cl = 0;
        for (int k = 0; k < kBins - 1; ++k) {
          accl.merge(sb.bb[k]);
          cl += sb.enter[k];
          if (cl == 0 || rc[k + 1] == 0) continue;
          if ((long long)cl + rc[k + 1] - n > budget) continue;  // straddlers past the budget
          float cost = area(accl) * cl + area(rb[k + 1]) * rc[k + 1];
          if (cost < best_cost) {
            best_cost = cost;
            sp_axis = ax;
            sp_pos = lo + w * (k + 1);
          }
        }
      }
    }
    const float leaf_cost = area(b) * n;
    const float node_cost = area(b) * kNodeCost;  // traversal step relative to one primitive test
    if (n <= kMaxLeaf && ((best_axis < 0 && sp_axis < 0) || best_cost * 1.0f + node_cost >= leaf_cost)) {
      make_leaf(out, id, refs);
      return id;
    }
    std::vector<Ref> L, R;
    long long dup = 0;
    const float obj_lo = best_axis >= 0 ? cb.lo[best_axis] : 0.0f;
    const float obj_scale = best_axis >= 0 ? kBins / (cb.hi[best_axis] - obj_lo) : 0.0f;
    auto split = [&](int axis) {
      if (wide) {
        std::vector<std::vector<Ref>> pl(chunks), pr(chunks);
        std::vector<long long> pd(chunks, 0);
        parallel_chunks(refs.size(), chunks, [&](int c, size_t s, size_t e) {
          pd[c] = partition(refs, s, e, axis, sp_pos, best_axis, best_bin, obj_lo, obj_scale, pl[c], pr[c]);
        });
        for (int c = 0; c < chunks; ++c) {  // chunk order == sequential order
          L.insert(L.end(), pl[c].begin(), pl[c].end());
          R.insert(R.end(), pr[c].begin(), pr[c].end());
          dup += pd[c];
        }
      } else {
        dup = partition(refs, 0, refs.size(), axis, sp_pos, best_axis, best_bin, obj_lo, obj_scale, L, R);
      }
    };
    if (sp_axis >= 0) {
      split(sp_axis);
      if (L.empty() || R.empty()) {  // degenerate: fall back to the object split below
        L.clear();
        R.clear();
        dup = 0;
        sp_axis = -1;
      }
    }
    if (sp_axis < 0) {
      if (best_axis < 0) {  // all centroids coincide: split the list
        L.assign(refs.begin(), refs.begin() + n / 2);
        R.assign(refs.begin() + n / 2, refs.end());
      } else {
        split(-1);
        if (L.empty() || R.empty()) {
          L.assign(refs.begin(), refs.begin() + n / 2);
          R.assign(refs.begin() + n / 2, refs.end());
        }
      }
    }
    std::vector<Ref>().swap(refs);
    const long long left_budget = std::max(0LL, budget - dup);
    const long long bl = (long long)((double)left_budget * (double)L.size() / (double)(L.size() + R.size()));
    const long long br = left_budget - bl;
    int l, r;
    int tok = spare.load();
    const bool spawn = L.size() >= kSpawnMin && R.size() >= kSpawnMin && tok > 0 &&
                       spare.compare_exchange_strong(tok, tok - 1);
    if (spawn) {  // left subtree on another thread, right here; appended in DFS order
      BuildOut lo, ro;
      std::thread t;
      try {
        t = std::thread([&] { build(std::move(L), depth + 1, bl, lo); });
      } catch (const std::system_error&) {  // no thread: the left subtree runs here first
        build(std::move(L), depth + 1, bl, lo);
      }
      build(std::move(R), depth + 1, br, ro);
      if (t.joinable()) t.join();
      spare.fetch_add(1);
      l = (int)out.nodes.size();
      out.append(std::move(lo));
      r = (int)out.nodes.size();
      out.append(std::move(ro));
    } else {
      l = build(std::move(L), depth + 1, bl, out);
      r = build(std::move(R), depth + 1, br, out);
    }
    out.nodes[id].left = l;
    out.nodes[id].right = r;
    out.nodes[id].count = 0;
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
                Box& box, bool& nonempty, std::vector<double>* verts = nullptr) {
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
    if (verts)
      for (int m = 0; m < 3; ++m) verts->push_back(A[m] + a * u[m] + b * v[m]);
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
  BuildTimer tm("build_wide");
  const int n = (int)sc.order.size();
  const float margin = 1e-5f * sc.scene_scale;
  std::vector<BuildPrim> bounded;
  std::vector<Box> accept_box(n);          // unpadded acceptance region (planes)
  std::vector<uint8_t> has_accept(n, 0);
  std::vector<int> unbounded;  // sorted positions
  std::vector<int> never;      // planes that accept no point: kept for indexing, never traversed
  Polys polys;                 // per bounded primitive: acceptance triangles (spatial splits)
  bounded.reserve(n);
  // per-primitive classification on all build threads (chunks of the sorted positions),
  // concatenated in chunk order == the sequential order
  struct Part {
    std::vector<BuildPrim> bounded;
    std::vector<int> never, unbounded;
    Polys polys;
  };
  const int nchunks = n >= 65536 ? build_threads() : 1;
  std::vector<Part> parts(nchunks);
  parallel_chunks((size_t)n, nchunks, [&](int ci, size_t rb, size_t re) {
    Part& pt = parts[ci];
    for (int r = (int)rb; r < (int)re; ++r) {
      const Shape& s = sc.shapes[sc.order[r]];
      Box b = shape_box[sc.order[r]];
      bool ok = true;
      float pad = margin;
      std::vector<double> tv1, tv2;  // the two sub-triangles' acceptance regions (3 vertices each)
      if (s.kind == RT_PRIM_PLANE) {
        // isPointInQuad = triangle (c1,c3,c2) OR triangle (c0,c1,c2) (shapes.cpp:485-494); the
        // acceptance regions (2x the reference's 1e-6 tolerance for float rounding) bound every
        // hit point.  Invalid planes (|cross| < 1e-6f) never hit and are left out entirely.
        uint32_t tag;
        std::memcpy(&tag, &sc.prims[r].a[15], 4);
        if (!(tag & RT_TAG_PLANE_VALID)) { pt.never.push_back(r); continue; }
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
        ok = tri_region(C[1], C[3], C[2], nn, 2e-6, region, ne1, &tv1) &&
             tri_region(C[0], C[1], C[2], nn, 2e-6, region, ne2, &tv2);
        if (ok && !ne1 && !ne2) { pt.never.push_back(r); continue; }  // accepts nothing
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
        pt.unbounded.push_back(r);
        continue;
      }
      // polygons only when both regions are whole triangles or empty (otherwise: never split)
      int ntri = 0;
      if ((tv1.size() == 9 || tv1.empty()) && (tv2.size() == 9 || tv2.empty()) && !(tv1.empty() && tv2.empty())) {
        // c3 == c0 makes both sub-triangles the same triangle: keep one copy
        bool same = tv1.size() == 9 && tv2.size() == 9;
        for (int k = 0; k < 3 && same; ++k) {
          bool found = false;
          for (int m = 0; m < 3 && !found; ++m)
            found = std::fabs(tv1[k * 3] - tv2[m * 3]) + std::fabs(tv1[k * 3 + 1] - tv2[m * 3 + 1]) +
                        std::fabs(tv1[k * 3 + 2] - tv2[m * 3 + 2]) <= 1e-12 * (1.0 + std::fabs(tv1[k * 3]));
          same = found;
        }
        pt.polys.off.push_back((int)(pt.polys.v.size() / 9));
        pt.polys.v.insert(pt.polys.v.end(), tv1.begin(), tv1.end());
        if (!same) pt.polys.v.insert(pt.polys.v.end(), tv2.begin(), tv2.end());
        ntri = (int)(pt.polys.v.size() / 9) - pt.polys.off.back();
      } else {
        pt.polys.off.push_back((int)(pt.polys.v.size() / 9));
      }
      pt.polys.n.push_back(ntri);
      BuildPrim bp;
      bp.box = b;
      bp.c = {0.5f * (b.lo[0] + b.hi[0]), 0.5f * (b.lo[1] + b.hi[1]), 0.5f * (b.lo[2] + b.hi[2])};
      bp.id = r;
      pt.bounded.push_back(bp);
    }
  });
  for (Part& pt : parts) {
    const int voff = (int)(polys.v.size() / 9);
    bounded.insert(bounded.end(), pt.bounded.begin(), pt.bounded.end());
    never.insert(never.end(), pt.never.begin(), pt.never.end());
    unbounded.insert(unbounded.end(), pt.unbounded.begin(), pt.unbounded.end());
    polys.v.insert(polys.v.end(), pt.polys.v.begin(), pt.polys.v.end());
    for (int o : pt.polys.off) polys.off.push_back(o + voff);
    polys.n.insert(polys.n.end(), pt.polys.n.begin(), pt.polys.n.end());
    Part().bounded.swap(pt.bounded);
  }
  std::vector<Part>().swap(parts);
  tm.lap("acceptance regions");
  SAHBuilder B{bounded, polys, margin};
  if (const char* e = std::getenv("RT_SAH_BINS")) B.kBins = std::max(2, std::min(SAHBuilder::kBinsMax, std::atoi(e)));
  if (const char* e = std::getenv("RT_SAH_LEAF")) B.kMaxLeaf = std::max(1, std::min(15, std::atoi(e)));
  if (const char* e = std::getenv("RT_SAH_NODE")) B.kNodeCost = (float)std::atof(e);
  if (const char* e = std::getenv("RT_SBVH_ALPHA")) B.kSplitAlpha = (float)std::atof(e);
  double dup = kSbvhDup;
  if (const char* e = std::getenv("RT_SBVH_DUP")) dup = std::max(0.0, std::min(4.0, std::atof(e)));
  B.threads = build_threads();
  B.spare = B.threads - 1;
  // duplicates allowed: the RT_SBVH_DUP fraction, and never past the 24-bit leaf packing
  const long long ref_cap = (1LL << 24) - 1 - (long long)(n - (int)bounded.size());
  const long long budget = std::max(0LL, std::min((long long)(dup * (double)bounded.size()),
                                                  ref_cap - (long long)bounded.size()));
  BuildOut T;
  T.nodes.reserve(bounded.size() + 1);
  if (!bounded.empty()) {
    std::vector<Ref> refs(bounded.size());
    Box open;  // no clip yet
    for (int a = 0; a < 3; ++a) {
      open.lo[a] = -INFINITY;
      open.hi[a] = INFINITY;
    }
    for (size_t i = 0; i < bounded.size(); ++i) refs[i] = Ref{bounded[i].box, open, (int)i};
    B.build(std::move(refs), 0, budget, T);
  }

  tm.lap("SAH/SBVH BVH2");
  // new primitive order: leaf references of the SAH tree (DFS; a primitive split by spatial
  // splits appears once per part), then the never-hit and the unbounded lists
  std::vector<int> new_order;  // new index -> sorted reference position r
  new_order.reserve(T.leaf_refs.size() + never.size() + unbounded.size());
  for (const Ref& r : T.leaf_refs) new_order.push_back(bounded[r.p].id);
  for (int r : never) new_order.push_back(r);
  for (int r : unbounded) new_order.push_back(r);  // the last n_unbounded, tested by every ray
  sc.n_unbounded = (int)unbounded.size();

  // collapse BVH2 -> BVH4.  Default: SAH-optimal by dynamic programming over the BVH2
  // (bottom-up: cost[i][k] = the least SAH cost of node i's subtree given k child slots of its
  // parent -- one slot as a leaf or as a 4-wide node of its own, or split between its two
  // children; the 4-wide node of BVH2 node i takes its children's best 4-slot split).
  // RT_COLLAPSE=greedy: expand the largest-area internal child until four (round 1).
  const bool dp_collapse = !(std::getenv("RT_COLLAPSE") && std::string(std::getenv("RT_COLLAPSE")) == "greedy");
  const int n2 = (int)T.nodes.size();
  std::vector<std::array<float, 5>> dpc(dp_collapse ? n2 : 0);     // cost by slots (1..4)
  std::vector<std::array<uint8_t, 5>> dps(dp_collapse ? n2 : 0);   // 0: one slot; j: j slots to the left child
  for (int i = (int)dpc.size() - 1; i >= 0; --i) {  // children follow their parent (DFS pre-order)
    const Node2& nd = T.nodes[i];
    const float A = area(nd.box);
    if (nd.left < 0) {
      for (int k = 1; k <= 4; ++k) { dpc[i][k] = A * (float)nd.count; dps[i][k] = 0; }
      continue;
    }
    float dist[5] = {0, 0, 0, 0, 0};
    uint8_t dj[5] = {0, 0, 0, 0, 0};
    for (int k = 2; k <= 4; ++k) {
      dist[k] = INFINITY;
      for (int j = 1; j < k; ++j) {
        const float c = dpc[nd.left][j] + dpc[nd.right][k - j];
        if (c < dist[k]) { dist[k] = c; dj[k] = (uint8_t)j; }
      }
    }
    dpc[i][1] = A * B.kNodeCost + dist[4];
    dps[i][1] = 0;
    for (int k = 2; k <= 4; ++k) {
      if (dist[k] < dpc[i][1]) { dpc[i][k] = dist[k]; dps[i][k] = dj[k]; }
      else { dpc[i][k] = dpc[i][1]; dps[i][k] = 0; }
    }
    dps[i][0] = dj[4];  // the 4-slot split of i's own children, used when i becomes a node
  }
  // the BVH2 nodes that become the child slots of the 4-wide node made from internal node n
  std::function<void(int, int, std::vector<int>&)> gather = [&](int n, int k, std::vector<int>& out) {
    const uint8_t j = dps[n][k];
    if (k == 1 || j == 0) { out.push_back(n); return; }
    gather(T.nodes[n].left, j, out);
    gather(T.nodes[n].right, k - j, out);
  };
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
      const Node2& root = T.nodes[it.n2];
      if (root.left < 0) {
        kids.push_back(it.n2);
      } else if (dp_collapse) {
        const int j = dps[it.n2][0];
        gather(root.left, j, kids);
        gather(root.right, 4 - j, kids);
      } else {
        kids = {root.left, root.right};
        while (kids.size() < 4) {
          int best = -1;
          float ba = -1;
          for (int k = 0; k < (int)kids.size(); ++k) {
            const Node2& c = T.nodes[kids[k]];
            if (c.left >= 0 && area(c.box) > ba) { ba = area(c.box); best = k; }
          }
          if (best < 0) break;
          int nb = kids[best];
          kids.erase(kids.begin() + best);
          kids.push_back(T.nodes[nb].left);
          kids.push_back(T.nodes[nb].right);
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
        const Node2& c = T.nodes[kids[k]];
        cb[nk++] = c.box;
        if (c.left < 0) {
          // leaf entry: 0x80000000 | first primitive << 7 | count (new order == leaf_refs order)
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

  tm.lap("BVH4 collapse + quantise");
  // reorder primitive records; keep (reference index, reference leaf) per primitive
  const int n_out = (int)new_order.size();
  if (n_out >= (1 << 24)) throw std::runtime_error("BVH: 2^24 or more primitive references");
  std::vector<rt_prim> prims(n_out);
  sc.prim_refs.assign(n_out, rt_prim_ref{});
  for (int i = 0; i < n_out; ++i) {
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
  tm.lap("reorder + reference-leaf filter");
}

}  // namespace rth
