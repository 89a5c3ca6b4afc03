// rt_device.h -- device-side math of the MI355X ray-trace path (gfx950).
//
// Every function restates a reference function with the reference's IEEE binary32 operand
// order (hipcc -ffp-contract=off, correctly rounded div/sqrt), so the kernel reproduces the
// reference's hit points, normals and colours bit for bit.  References are to
// /root/reference/Code/<file>:<line>.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/rt_hip.h"

#define RT_HD __device__
#define RT_TABLE_QUAL static __constant__
#define RT_FMA64 __builtin_fma
#define RT_FMA32 __builtin_fmaf
#include "../common/rt_powf.h"
#include "../common/rt_div.h"

namespace rtd {

struct V3 {
  float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 mul(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
// vecDot / VecMath::dot: ((a0*b0 + a1*b1) + a2*b2)
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// vecCross (shapes.cpp:12-18)
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// VecMath::normalize (raytracer.cpp:75-79) == Camera::normalize (camera.cpp:60-68)
__device__ __forceinline__ V3 normalize(V3 v) {
  float m = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
  if (m == 0.0f) return V3{0.0f, 0.0f, 0.0f};
  return V3{((v.x) / (m)), ((v.y) / (m)), ((v.z) / (m))};
}
// normalize() with one correctly rounded reciprocal and three Markstein quotients where they
// give the same bits as the three divisions by m (rt_normalize3, rt_div.h; otherwise the
// divisions themselves)
__device__ __forceinline__ V3 normalize_rcp(V3 v) {
  rt_normalize3(v.x, v.y, v.z);
  return v;
}
// std::max / std::min on floats: (a < b) ? b : a  and  (b < a) ? b : a
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }

// Shapes::transformPoint (shapes.cpp:151-158); row 3 of every matrix built by
// buildTransformationMatrices is exactly (0,0,0,1), so w == 1 and the divide never runs.
__device__ __forceinline__ V3 xpoint(const float* m, V3 p) {
  return V3{m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3],
            m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7],
            m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11]};
}
// Shapes::transformVector (shapes.cpp:160-165)
__device__ __forceinline__ V3 xvec(const float* m, V3 v) {
  return V3{m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
            m[8] * v.x + m[9] * v.y + m[10] * v.z};
}
// Shapes::transformNormal (shapes.cpp:167-187): world_to_object transposed, renormalised
__device__ __forceinline__ V3 xnormal(const float* w, V3 n) {
  V3 r{w[0] * n.x + w[4] * n.y + w[8] * n.z, w[1] * n.x + w[5] * n.y + w[9] * n.z,
       w[2] * n.x + w[6] * n.y + w[10] * n.z};
  float len = sqrtf(r.x * r.x + r.y * r.y + r.z * r.z);
  if (len > 1e-6f) r = V3{((r.x) / (len)), ((r.y) / (len)), ((r.z) / (len))};
  return r;
}

struct Ray {
  V3 o, d;
  float time;
};

// A primitive record as loaded from HBM (first 64 bytes; the second half -- object_to_world
// -- is fetched only when a transformed primitive is actually hit).
struct PrimA {
  float a[16];
};
__device__ __forceinline__ void load_prim_a(const float4* rec, PrimA& p) {
  float4 q0 = rec[0], q1 = rec[1], q2 = rec[2], q3 = rec[3];
  p.a[0] = q0.x; p.a[1] = q0.y; p.a[2] = q0.z; p.a[3] = q0.w;
  p.a[4] = q1.x; p.a[5] = q1.y; p.a[6] = q1.z; p.a[7] = q1.w;
  p.a[8] = q2.x; p.a[9] = q2.y; p.a[10] = q2.z; p.a[11] = q2.w;
  p.a[12] = q3.x; p.a[13] = q3.y; p.a[14] = q3.z; p.a[15] = q3.w;
}
__device__ __forceinline__ void load_o2w(const float4* rec, float* m) {
  float4 q0 = rec[4], q1 = rec[5], q2 = rec[6];
  m[0] = q0.x; m[1] = q0.y; m[2] = q0.z; m[3] = q0.w;
  m[4] = q1.x; m[5] = q1.y; m[6] = q1.z; m[7] = q1.w;
  m[8] = q2.x; m[9] = q2.y; m[10] = q2.z; m[11] = q2.w;
}
__device__ __forceinline__ uint32_t prim_tag(const PrimA& p) { return __float_as_uint(p.a[15]); }

// Full hit record (shapes.hpp:15-23); only produced for the winning primitive.
struct HitAttr {
  V3 p, n;
  float u, v;
};

// ---- Sphere::intersect (shapes.cpp:200-262): unit sphere in object space, motion blur
template <bool kAttr, bool kUV = true>
__device__ __forceinline__ bool sphere_hit(const PrimA& P, const float4* rec, const Ray& ray,
                                           float& t_out, HitAttr* at) {
  V3 vel{P.a[12], P.a[13], P.a[14]};
  V3 mo{ray.o.x - vel.x * ray.time, ray.o.y - vel.y * ray.time, ray.o.z - vel.z * ray.time};
  V3 o = xpoint(P.a, mo), d = xvec(P.a, ray.d);
  float a = dot(d, d);
  float b = 2.0f * dot(o, d);
  float c = dot(o, o) - 1.0f;
  float disc = b * b - 4.0f * a * c;
  if (disc < 0) return false;
  float sq = sqrtf(disc);
  float t1 = ((-b - sq) / (2.0f * a));
  float t2 = ((-b + sq) / (2.0f * a));
  float tl = (t1 > 0.001f) ? t1 : ((t2 > 0.001f) ? t2 : -1.0f);
  if (tl < 0) return false;
  V3 pl{o.x + tl * d.x, o.y + tl * d.y, o.z + tl * d.z};
  float m[12];
  load_o2w(rec, m);
  V3 hp = xpoint(m, pl);
  hp = V3{hp.x + vel.x * ray.time, hp.y + vel.y * ray.time, hp.z + vel.z * ray.time};
  V3 dv = sub(hp, ray.o);
  t_out = sqrtf(dot(dv, dv));
  if (kAttr) {
    at->p = hp;
    at->n = xnormal(P.a, pl);
    if (kUV) {
      const float PI = 3.1415926535f;
      // double atan2/asin as in the reference; ocml, not glibc: UVs only feed textures.
      at->u = (float)(0.5 + atan2((double)pl.z, (double)pl.x) / (double)(2.0f * PI));
      at->v = (float)(0.5 - asin((double)pl.y) / (double)PI);
    } else {
      at->u = 0.0f;
      at->v = 0.0f;
    }
  }
  return true;
}

// ---- Rectangle::intersect (shapes.cpp:299-333): unit square on z = 0
template <bool kAttr>
__device__ __forceinline__ bool rect_hit(const PrimA& P, const float4* rec, const Ray& ray,
                                         float& t_out, HitAttr* at) {
  V3 o = xpoint(P.a, ray.o), d = xvec(P.a, ray.d);
  if (fabsf(d.z) < 1e-6f) return false;
  float tl = ((-o.z) / (d.z));
  if (tl < 0.001f) return false;
  float hx = o.x + tl * d.x;
  float hy = o.y + tl * d.y;
  if (hx < -0.5f || hx > 0.5f || hy < -0.5f || hy > 0.5f) return false;
  float m[12];
  load_o2w(rec, m);
  V3 hp = xpoint(m, V3{hx, hy, 0.0f});
  V3 dv = sub(hp, ray.o);
  t_out = sqrtf(dot(dv, dv));
  if (kAttr) {
    at->p = hp;
    at->n = xnormal(P.a, V3{0.0f, 0.0f, 1.0f});
    at->u = hx + 0.5f;
    at->v = hy + 0.5f;
  }
  return true;
}

// ---- Cube::intersect (shapes.cpp:355-423): unit cube [-0.5,0.5]^3, slab with entry axis
template <bool kAttr>
__device__ __forceinline__ bool cube_hit(const PrimA& P, const float4* rec, const Ray& ray,
                                         float& t_out, HitAttr* at) {
  V3 o = xpoint(P.a, ray.o), d = xvec(P.a, ray.d);
  const float tmin = -0.5f, tmax = 0.5f;
  float tn = -3.40282347e+38f, tf = 3.40282347e+38f;
  int axis = -1, sign = 0;
  float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
#pragma unroll
  for (int i = 0; i < 3; i++) {
    if (fabsf(dd[i]) < 1e-6f) {
      if (oo[i] < tmin || oo[i] > tmax) return false;
    } else {
      float t1 = ((tmin - oo[i]) / (dd[i]));
      float t2 = ((tmax - oo[i]) / (dd[i]));
      float te = smin(t1, t2), tx = smax(t1, t2);
      if (te > tn) { tn = te; axis = i; sign = (t1 < t2) ? -1 : 1; }
      if (tx < tf) tf = tx;
      if (tn > tf || tf < 0) return false;
    }
  }
  float tl = (tn > 0) ? tn : tf;
  if (tl < 0) return false;
  V3 pl{o.x + tl * d.x, o.y + tl * d.y, o.z + tl * d.z};
  float m[12];
  load_o2w(rec, m);
  V3 hp = xpoint(m, pl);
  V3 dv = sub(hp, ray.o);
  t_out = sqrtf(dot(dv, dv));
  if (kAttr) {
    V3 nl{0.0f, 0.0f, 0.0f};
    if (axis == 0) nl.x = (float)sign;
    else if (axis == 1) nl.y = (float)sign;
    else if (axis == 2) nl.z = (float)sign;
    at->p = hp;
    at->n = xnormal(P.a, nl);
    float uc = pl.x + 0.5f, vc = pl.y + 0.5f, wc = pl.z + 0.5f;
    if (axis == 0) { at->u = (sign > 0) ? wc : (1.0f - wc); at->v = vc; }
    else if (axis == 1) { at->u = uc; at->v = (sign > 0) ? wc : (1.0f - wc); }
    else { at->u = (sign > 0) ? uc : (1.0f - uc); at->v = vc; }
  }
  return true;
}

// isPointInTriangle (shapes.cpp:24-40)
__device__ __forceinline__ bool in_tri(V3 P, V3 A, V3 B, V3 C, V3 n) {
  if (dot(cross(sub(B, A), sub(P, A)), n) < -1e-6f) return false;
  if (dot(cross(sub(C, B), sub(P, B)), n) < -1e-6f) return false;
  if (dot(cross(sub(A, C), sub(P, C)), n) < -1e-6f) return false;
  return true;
}

// ---- Plane::intersect (shapes.cpp:444-494); normal precomputed on the host with the
// identical ops (the reference recomputes it per call, same bits).
template <bool kAttr>
__device__ __forceinline__ bool plane_hit(const PrimA& P, const Ray& ray, float& t_out, HitAttr* at,
                                          V3* x_out = nullptr) {
  if (!(prim_tag(P) & RT_TAG_PLANE_VALID)) return false;
  const bool tri = (prim_tag(P) & RT_TAG_TRI1_NEVER) != 0u;
  V3 c0{P.a[0], P.a[1], P.a[2]}, c1{P.a[4], P.a[5], P.a[6]}, c2{P.a[8], P.a[9], P.a[10]};
  V3 c3 = tri ? c0 : V3{P.a[12], P.a[13], P.a[14]};
  V3 n{P.a[3], P.a[7], P.a[11]};
  float denom = dot(n, ray.d);
  if (fabsf(denom) < 1e-6f) return false;
  float t = ((dot(sub(c0, ray.o), n)) / (denom));
  if (t < 0) return false;
  V3 X{ray.o.x + t * ray.d.x, ray.o.y + t * ray.d.y, ray.o.z + t * ray.d.z};
  // isPointInQuad: (c1, c3, c2) || (c0, c1, c2); the OR of two pure tests in either order.  With
  // RT_TAG_TRI1_NEVER the first cannot accept a point within sqrt(a[12]) of c0 (scene.cpp).
  if (!in_tri(X, c0, c1, c2, n)) {
    const V3 dx = sub(X, c0);
    if (tri && dot(dx, dx) <= P.a[12]) return false;
    if (!in_tri(X, c1, c3, c2, n)) return false;
  }
  t_out = t;
  if (x_out) *x_out = X;
  if (kAttr) {
    V3 vu = sub(c1, c0), vv = sub(c3, c0), hv = sub(X, c0);
    float u = ((dot(hv, vu)) / (dot(vu, vu)));
    float v = ((dot(hv, vv)) / (dot(vv, vv)));
    at->u = smax(0.0f, smin(1.0f, u));
    at->v = smax(0.0f, smin(1.0f, v));
    at->p = X;
    at->n = n;
  }
  return true;
}

template <bool kAttr, bool kPlanesOnly = false, bool kUV = true>
__device__ __forceinline__ bool prim_hit(const PrimA& P, const float4* rec, const Ray& ray,
                                         float& t, HitAttr* at) {
  if (kPlanesOnly) return plane_hit<kAttr>(P, ray, t, at);
  switch (RT_TAG_KIND(prim_tag(P))) {
    case RT_PRIM_PLANE: return plane_hit<kAttr>(P, ray, t, at);
    case RT_PRIM_CUBE: return cube_hit<kAttr>(P, rec, ray, t, at);
    case RT_PRIM_RECTANGLE: return rect_hit<kAttr>(P, rec, ray, t, at);
    default: return sphere_hit<kAttr, kUV>(P, rec, ray, t, at);
  }
}

// ---- AABB::intersect (shapes.cpp:55-72), exact: used for every leaf box so the set of
// candidate primitives equals the reference's.  `par` bit i = fabs(d_i) < 1e-6 (double).
// The per-axis early exits are folded into one final test (t_near only grows and t_far only
// shrinks, so a failure at any axis persists).  Returns t_near for pruning.
__device__ __forceinline__ bool aabb_exact(const float* lo, const float* hi, const Ray& r,
                                           uint32_t par, float& tnear) {
  float tn = -3.40282347e+38f, tf = 3.40282347e+38f;
  bool ok = true;
  const float o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (par & (1u << i)) {
      ok = ok && !(o[i] < lo[i] || o[i] > hi[i]);
    } else {
      float t1 = ((lo[i] - o[i]) / (d[i]));
      float t2 = ((hi[i] - o[i]) / (d[i]));
      float a = (t1 > t2) ? t2 : t1, b = (t1 > t2) ? t1 : t2;
      tn = smax(tn, a);
      tf = smin(tf, b);
    }
  }
  tnear = tn;
  return ok && !(tn > tf || tf < 0);
}

// Conservative slab test for internal nodes (boxes padded on the host by far more than the
// reciprocal-multiply error), so it never rejects a subtree whose exact leaf test passes.
__device__ __forceinline__ bool aabb_fast(const float* lo, const float* hi, V3 o, V3 inv, float& tnear) {
  float tx1 = (lo[0] - o.x) * inv.x, tx2 = (hi[0] - o.x) * inv.x;
  float ty1 = (lo[1] - o.y) * inv.y, ty2 = (hi[1] - o.y) * inv.y;
  float tz1 = (lo[2] - o.z) * inv.z, tz2 = (hi[2] - o.z) * inv.z;
  float tn = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
  float tf = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
  tnear = tn;
  return tn <= tf && tf >= 0.0f;
}

// ---- counter RNG: one dist(gen) draw == generate_canonical<double,53> of two 32-bit words
// (libstdc++), words from splitmix64(key + n * C).  Identical to oracle/rt_oracle.cpp Rng.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27; z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}
struct Rng {
  uint64_t key;
  uint32_t ctr;
  __device__ __forceinline__ void begin(uint64_t seed_key, uint64_t pixel, uint64_t sample) {
    uint64_t pk = mix64(seed_key ^ (pixel * 0xD1B54A32D192ED03ull));
    key = mix64(pk + (sample + 1) * 0x9E3779B97F4A7C15ull);
    ctr = 0;
  }
  __device__ __forceinline__ double next() {
    uint64_t w = mix64(key + (uint64_t)(++ctr) * 0xDA942042E4DD58B5ull);
    double sum = (double)(uint32_t)w + (double)(uint32_t)(w >> 32) * 4294967296.0;
    double ret = sum / 18446744073709551616.0;
    return ret >= 1.0 ? 0x1.fffffffffffffp-1 : ret;
  }
  // VecMath::random_in_unit_sphere (raytracer.cpp:153-171)
  __device__ __forceinline__ V3 in_unit_sphere() {
    for (;;) {
      float r1 = (float)next(), r2 = (float)next(), r3 = (float)next();
      V3 p{2.0f * r1 - 1.0f, 2.0f * r2 - 1.0f, 2.0f * r3 - 1.0f};
      if (dot(p, p) < 1.0f) return p;
    }
  }
};

}  // namespace rtd
