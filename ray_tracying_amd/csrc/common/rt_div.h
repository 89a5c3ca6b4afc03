// rt_div.h -- correctly rounded division by a value whose reciprocal is known.
//
// q = a / b (IEEE round to nearest) from y = RN(1 / b), the correctly rounded reciprocal,
// by Markstein's correction (P. Markstein, IBM J. Res. Dev. 34(1), 1990; J.-M. Muller et al.,
// Handbook of Floating-Point Arithmetic, "Markstein's theorem"): q0 = RN(a * y) is within
// one ulp of a / b, the remainder r = a - b * q0 is exact in one fma, and RN(q0 + r * y) is
// RN(a / b) -- provided nothing over- or underflows (|a|, |b|, |a / b| and 1 / b normal).
// Three operations instead of the division's scale / reciprocal / refinement sequence
// (~10 on gfx950, twice as many issue cycles in binary64).  The kernels use it only where
// the divisor is the same for many quotients and its range is known (the jitter's s, the
// image resolution, a camera ray's length); tests/test_div.py checks it against the
// hardware division on random and swept operands.
//
// The includer defines RT_HD (empty on the host, __device__ in HIP code) and RT_FMA32 /
// RT_FMA64 (one correctly rounded fma each).
#pragma once

#ifndef RT_HD
#define RT_HD
#endif

RT_HD inline float rt_div_by(float a, float b, float y) {
  const float q0 = a * y;
  const float r = RT_FMA32(-q0, b, a);
  return RT_FMA32(r, y, q0);
}
RT_HD inline double rt_div_by(double a, double b, double y) {
  const double q0 = a * y;
  const double r = RT_FMA64(-q0, b, a);
  return RT_FMA64(r, y, q0);
}

// normalize() (raytracer.cpp:75-79: x / m per component, m = sqrtf(x*x + y*y + z*z)) through
// one correctly rounded reciprocal and three Markstein quotients where those are RN(x / m):
// m and 1 / m normal, and every component x with |x| >= 2^-100 and |x| >= m * 2^-120 -- then
// the remainder x - m * q0 is exact (x at least 2^(emin + 26)) and x / m is normal.  Any other
// vector -- a zero component (whose sign the correction could lose: -0 / m is -0), a subnormal
// or tiny one, an extreme length -- takes the three divisions.  tests/test_div.py checks it
// against the divisions on vectors with zero, signed-zero, subnormal and tiny components.
RT_HD inline bool rt_quot_by_len_ok(float x, float m) {
  const float ax = x < 0.0f ? -x : x;
  return ax >= 0x1p-100f && ax >= m * 0x1p-120f;
}
RT_HD inline void rt_normalize3(float& x, float& y, float& z) {
  const float m = sqrtf(x * x + y * y + z * z);
  if (m == 0.0f) {
    x = y = z = 0.0f;
    return;
  }
  if (!(m > 0x1p-120f && m < 0x1p120f) || !(rt_quot_by_len_ok(x, m) && rt_quot_by_len_ok(y, m) && rt_quot_by_len_ok(z, m))) {
    x = x / m;
    y = y / m;
    z = z / m;
    return;
  }
  const float r = 1.0f / m;
  x = rt_div_by(x, m, r);
  y = rt_div_by(y, m, r);
  z = rt_div_by(z, m, r);
}
