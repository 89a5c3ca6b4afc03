// Sweep rt_powf (ray_tracying_amd/csrc/common/rt_powf.h) against the live glibc powf.
// usage: powf_check <y> <x_lo_bits> <x_hi_bits> <stride>   -> prints "<checked> <mismatches>"
//        powf_check random <n> <seed>                       -> random (x,y) pairs
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#define RT_FMA64 std::fma
#include "../../ray_tracying_amd/csrc/common/rt_powf.h"

static int same(float a, float b) {
  uint32_t ua, ub; memcpy(&ua, &a, 4); memcpy(&ub, &b, 4);
  if (std::isnan(a) && std::isnan(b)) return 1;
  return ua == ub;
}

int main(int argc, char** argv) {
  unsigned long long checked = 0, bad = 0;
  if (argc >= 4 && !strcmp(argv[1], "random")) {
    unsigned long long n = strtoull(argv[2], 0, 10);
    uint64_t s = strtoull(argv[3], 0, 10) * 0x9E3779B97F4A7C15ull + 1;
    for (unsigned long long i = 0; i < n; ++i) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      uint32_t xb = (uint32_t)s, yb = (uint32_t)(s >> 32);
      float x, y; memcpy(&x, &xb, 4); memcpy(&y, &yb, 4);
      if ((i & 3) == 0) { x = std::fabs(x); y = std::fabs(y); }   // bias to x>=0
      float a = rt_powf(x, y), b = powf(x, y);
      ++checked; if (!same(a, b)) { if (bad < 5) fprintf(stderr, "x=%a y=%a mine=%a libm=%a\n", x, y, a, b); ++bad; }
    }
  } else if (argc >= 5) {
    float y = strtof(argv[1], 0);
    uint32_t lo = strtoul(argv[2], 0, 0), hi = strtoul(argv[3], 0, 0), st = strtoul(argv[4], 0, 0);
    for (uint64_t b = lo; b <= hi; b += st) {
      uint32_t xb = (uint32_t)b; float x; memcpy(&x, &xb, 4);
      float a = rt_powf(x, y), c = powf(x, y);
      ++checked; if (!same(a, c)) { if (bad < 5) fprintf(stderr, "x=%a y=%a mine=%a libm=%a\n", x, y, a, c); ++bad; }
    }
  } else { fprintf(stderr, "usage\n"); return 2; }
  printf("%llu %llu\n", checked, bad);
  return 0;
}
