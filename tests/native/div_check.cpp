// tests/native/div_check.cpp -- rt_div_by (ray_tracying_amd/csrc/common/rt_div.h) against the
// hardware's correctly rounded division.  Prints "<checked> <mismatches>".
//   div_check f32 random N SEED        random a, b (exponents -60..60)
//   div_check f32 sweep B E0 E1        every binary32 a in [2^E0, 2^E1) against divisor B
//   div_check f64 random N SEED
//   div_check f64 jitter S N SEED      a = si + U[0,1) (the stratified jitter), divisor S
//   div_check f32 norm N SEED          rt_normalize3 against three divisions by the length, on
//                                      vectors mixing normal, zero, -0, subnormal, tiny and huge
//                                      components (bit patterns compared: the sign of a zero counts)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#define RT_FMA32 std::fmaf
#define RT_FMA64 std::fma
#include "../../ray_tracying_amd/csrc/common/rt_div.h"

static float rf(std::mt19937_64& g) {
  std::uniform_int_distribution<int> e(-60, 60);
  std::uniform_real_distribution<float> m(1.0f, 2.0f);
  float v = std::ldexp(m(g), e(g));
  return (g() & 1) ? -v : v;
}
static double rd(std::mt19937_64& g) {
  std::uniform_int_distribution<int> e(-300, 300);
  std::uniform_real_distribution<double> m(1.0, 2.0);
  double v = std::ldexp(m(g), e(g));
  return (g() & 1) ? -v : v;
}
int main(int argc, char** argv) {
  if (argc < 3) return 2;
  unsigned long long checked = 0, bad = 0;
  const bool f32 = !strcmp(argv[1], "f32");
  if (!strcmp(argv[2], "random")) {
    const long long n = atoll(argv[3]);
    std::mt19937_64 g(strtoull(argv[4], 0, 10));
    for (long long i = 0; i < n; ++i) {
      if (f32) {
        volatile float a = rf(g), b = rf(g);
        const float y = 1.0f / b;
        if (rt_div_by((float)a, (float)b, y) != a / b) ++bad;
      } else {
        volatile double a = rd(g), b = rd(g);
        const double y = 1.0 / b;
        if (rt_div_by((double)a, (double)b, y) != a / b) ++bad;
      }
      ++checked;
    }
  } else if (!strcmp(argv[2], "sweep")) {
    const float b = strtof(argv[3], 0), y = 1.0f / b;
    uint32_t lo, hi;
    float flo = std::ldexp(1.0f, atoi(argv[4])), fhi = std::ldexp(1.0f, atoi(argv[5]));
    memcpy(&lo, &flo, 4);
    memcpy(&hi, &fhi, 4);
    for (uint32_t u = lo; u < hi; ++u) {
      float a;
      memcpy(&a, &u, 4);
      volatile float va = a, vb = b;
      if (rt_div_by((float)va, (float)vb, y) != va / vb) ++bad;
      ++checked;
    }
  } else if (!strcmp(argv[2], "norm")) {
    const long long n = atoll(argv[3]);
    std::mt19937_64 g(strtoull(argv[4], 0, 10));
    auto comp = [&]() -> float {
      const unsigned k = (unsigned)(g() % 8);
      const bool neg = g() & 1;
      float v;
      if (k == 0) v = 0.0f;
      else if (k == 1) {  // subnormal
        const uint32_t u = 1u + (uint32_t)(g() % 0x7fffffu);
        memcpy(&v, &u, 4);
      } else if (k == 2) v = std::ldexp(1.0f + (float)(g() >> 40) * 0x1p-24f, -126 + (int)(g() % 40));  // tiny normal
      else if (k == 3) v = std::ldexp(1.0f + (float)(g() >> 40) * 0x1p-24f, 40 + (int)(g() % 88));     // huge
      else v = std::ldexp(1.0f + (float)(g() >> 40) * 0x1p-24f, -8 + (int)(g() % 12));                // camera-like
      return neg ? -v : v;
    };
    for (long long i = 0; i < n; ++i) {
      volatile float x = comp(), y = comp(), z = comp();
      float a = x, b = y, c = z;
      rt_normalize3(a, b, c);
      const float m = sqrtf(x * x + y * y + z * z);
      float r[3] = {0.0f, 0.0f, 0.0f};
      if (m != 0.0f) {
        r[0] = x / m;
        r[1] = y / m;
        r[2] = z / m;
      }
      const float q[3] = {a, b, c};
      if (memcmp(q, r, sizeof q) != 0) ++bad;
      ++checked;
    }
  } else if (!strcmp(argv[2], "jitter")) {
    const int s = atoi(argv[3]);
    const long long n = atoll(argv[4]);
    std::mt19937_64 g(strtoull(argv[5], 0, 10));
    const double y = 1.0 / (double)s;
    for (long long i = 0; i < n; ++i) {
      const double u = (double)(g() >> 11) * 0x1p-53;
      volatile double a = (double)(i % s) + u, vs = (double)s;
      if (rt_div_by((double)a, (double)vs, y) != a / vs) ++bad;
      ++checked;
    }
  }
  printf("%llu %llu\n", checked, bad);
  return 0;
}
