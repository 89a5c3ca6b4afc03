// rt_powf.h -- bit-exact restatement of glibc 2.35 powf (x86_64 FMA ifunc variant).
//
// The reference evaluates std::pow(float, float) == glibc powf in two places:
//   * specular term  pow(N_dot_H, shininess)    /root/reference/Code/raytracer.cpp:258
//   * gamma          pow(c, 1.0f / 1.1f)        /root/reference/Code/raytracer.cpp:447-449
// glibc >= 2.28 powf is the ARM optimized-routines algorithm (e_powf.c): log2(x) from a
// 16-entry table + degree-5 polynomial, y*log2(x) in double, exp2 from a 32-entry table +
// degree-3 polynomial, one final double->float rounding.  On CPUs with FMA+AVX2 glibc
// selects the copy built with -mfma, where gcc contracted every a*b+c of the polynomial
// evaluation into a fused multiply-add; the operation order below is read off that copy's
// machine code (libm.so.6 +0x7aef0) and each fma() here is one vfmadd there.  The result
// must be identical bit for bit (tests/test_powf.py sweeps it against the live libm).
//
// The includer defines RT_HD (empty on the host, __device__ in HIP code) and RT_FMA64
// (std::fma / __builtin_fma); both map to one correctly rounded IEEE binary64 fma.
#pragma once
#include <stdint.h>
#include <string.h>
#include "glibc_powf_data.h"

#ifndef RT_HD
#define RT_HD
#endif
// Storage class for the lookup tables: plain static const on the host; the HIP
// translation unit defines it as `static __constant__` so the tables live in device
// read-only memory (runtime-indexed, so they cannot be folded into registers).
#ifndef RT_TABLE_QUAL
#define RT_TABLE_QUAL static const
#endif

namespace rtpow {

RT_TABLE_QUAL double kLog2Invc[16] = RT_POWF_LOG2_INVC;
RT_TABLE_QUAL double kLog2Logc[16] = RT_POWF_LOG2_LOGC;
RT_TABLE_QUAL uint64_t kExp2Tab[32] = RT_EXP2F_TAB;

RT_HD inline uint32_t asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
RT_HD inline float asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
RT_HD inline uint64_t asuint64(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
RT_HD inline double asdouble(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

// e_powf.c: zeroinfnan / checkint / issignalingf_inline
RT_HD inline int zeroinfnan(uint32_t ix) { return 2u * ix - 1u >= 2u * 0x7f800000u - 1u; }
RT_HD inline int checkint(uint32_t iy) {
  int e = (int)(iy >> 23 & 0xff);
  if (e < 0x7f) return 0;
  if (e > 0x7f + 23) return 2;
  if (iy & ((1u << (0x7f + 23 - e)) - 1u)) return 0;
  if (iy & (1u << (0x7f + 23 - e))) return 1;
  return 2;
}
RT_HD inline int is_snan(float x) {
  uint32_t ix = asuint(x);
  return 2u * (ix ^ 0x00400000u) > 2u * 0x7fc00000u;
}
// math_err.c: __math_oflowf / __math_uflowf / __math_may_uflowf / __math_invalidf
RT_HD inline float xflow(uint32_t sign, float y) { float s = sign ? -y : y; return s * y; }

// log2_inline (e_powf.c), POWF_SCALE_BITS == 0 on x86_64.
RT_HD inline double log2_inline(uint32_t ix) {
  const double A[5] = RT_POWF_LOG2_POLY;
  uint32_t tmp = ix - 0x3f330000u;
  int i = (int)((tmp >> (23 - 4)) % 16);
  uint32_t top = tmp & 0xff800000u;
  uint32_t iz = ix - top;
  int k = (int32_t)top >> 23;
  double invc = kLog2Invc[i];
  double logc = kLog2Logc[i];
  double z = (double)asfloat(iz);
  double r = RT_FMA64(z, invc, -1.0);
  double y0 = logc + (double)k;
  double r2 = r * r;
  double y = RT_FMA64(A[0], r, A[1]);
  double p = RT_FMA64(A[2], r, A[3]);
  double r4 = r2 * r2;
  double q = RT_FMA64(A[4], r, y0);
  q = RT_FMA64(p, r2, q);
  y = RT_FMA64(y, r4, q);
  return y;
}

// exp2_inline (e_powf.c), non-TOINT_INTRINSICS branch.
RT_HD inline float exp2_inline(double xd, uint32_t sign_bias) {
  const double C[3] = RT_EXP2F_POLY;
  const double SHIFT = RT_EXP2F_SHIFT_SCALED;
  double kd = xd + SHIFT;
  uint64_t ki = asuint64(kd);
  kd -= SHIFT;
  double r = xd - kd;
  uint64_t t = kExp2Tab[ki % 32];
  uint64_t ski = ki + sign_bias;
  t += ski << (52 - 5);
  double s = asdouble(t);
  double z = RT_FMA64(C[0], r, C[1]);
  double r2 = r * r;
  double y = RT_FMA64(C[2], r, 1.0);
  y = RT_FMA64(z, r2, y);
  y = y * s;
  return (float)y;
}

}  // namespace rtpow

RT_HD inline float rt_powf(float x, float y) {
  using namespace rtpow;
  const uint32_t SIGN_BIAS = 1u << (5 + 11);
  uint32_t sign_bias = 0;
  uint32_t ix = asuint(x);
  uint32_t iy = asuint(y);
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || zeroinfnan(iy)) {
    if (zeroinfnan(iy)) {
      if (2u * iy == 0) return rtpow::is_snan(x) ? x + y : 1.0f;
      if (ix == 0x3f800000u) return rtpow::is_snan(y) ? x + y : 1.0f;
      if (2u * ix > 2u * 0x7f800000u || 2u * iy > 2u * 0x7f800000u) return x + y;
      if (2u * ix == 2u * 0x3f800000u) return 1.0f;
      if ((2u * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
      return y * y;
    }
    if (zeroinfnan(ix)) {
      float x2 = x * x;
      if ((ix & 0x80000000u) && checkint(iy) == 1) x2 = -x2;
      return (iy & 0x80000000u) ? 1.0f / x2 : x2;
    }
    if (ix & 0x80000000u) {
      int yint = checkint(iy);
      if (yint == 0) return (x - x) / (x - x);
      if (yint == 1) sign_bias = SIGN_BIAS;
      ix &= 0x7fffffffu;
    }
    if (ix < 0x00800000u) {
      ix = asuint(x * 0x1p23f);
      ix &= 0x7fffffffu;
      ix -= 23u << 23;
    }
  }
  double logx = log2_inline(ix);
  double ylogx = (double)y * logx;
  if ((asuint64(ylogx) >> 47 & 0xffff) >= asuint64(126.0) >> 47) {
    if (ylogx > 0x1.fffffffd1d571p+6) return xflow(sign_bias, 0x1p97f);
    // ylogx > 0x1.fffffffa3aae2p+6: glibc re-checks rounding direction; under
    // round-to-nearest 1.0f + 0x1p-25f == 1.0f, so it falls through to exp2_inline.
    if (ylogx <= -150.0) return xflow(sign_bias, 0x1p-95f);
    if (ylogx < -149.0) return xflow(sign_bias, 0x1.4p-75f);
  }
  return exp2_inline(ylogx, sign_bias);
}
