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
