// Microbenchmark (diagnostic, not product): VALU issue rate of the instruction kinds the trace
// kernel's node visit is made of, at 1..8 waves per SIMD, to pin the real VALU peak of gfx950
// (wave64 instructions per CU-cycle) for the roofline.  Each lane runs 8 independent chains of
// one instruction kind.  The printed rate counts the SOURCE-level operations at 2.4 GHz; the
// authoritative figure is the counter one -- run it under
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- tools/bin/ubench_valu
// and divide SQ_INSTS_VALU (what the compiler emitted, issued) by 256 CUs x GRBM_GUI_ACTIVE / 8
// (tools/pmc_ubench.py); dispatches run >= 1 ms so the GRBM clock is accurate.
// hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/ubench_valu.hip -o tools/bin/ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kIters = 32768;
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(256) void spin(float* out, unsigned* cyc, float seed) {
  float a[8];
  unsigned u[8];
  f32x2 p[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = seed + threadIdx.x * 1e-3f + k;
    u[k] = threadIdx.x * 2654435761u + k * 977u;
    p[k] = f32x2{a[k], a[k] + 1.0f};
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (KIND == 0) a[k] = __builtin_fmaf(a[k], 1.0001f, 0.5f);                       // v_fma_f32
      if (KIND == 1) a[k] = __builtin_amdgcn_fmed3f(a[k], a[k] * 0.5f, 3.0f);             // v_med3 + mul
      if (KIND == 2) a[k] = fmaxf(fmaxf(a[k], seed), a[(k + 1) & 7]);                      // v_max3_f32
      if (KIND == 3) u[k] = __builtin_amdgcn_perm(u[k], u[(k + 3) & 7], 0x07030501u);    // v_perm_b32
      if (KIND == 4) { u[k] += 0x01010101u; a[k] += (float)((u[k] >> (8 * (k & 3))) & 0xffu); }  // add_u32 + cvt_f32_ubyte + add_f32
      if (KIND == 5) p[k] = __builtin_elementwise_fma(p[k], f32x2{1.0001f, 0.9999f}, f32x2{0.5f, 0.25f});  // v_pk_fma_f32
      if (KIND == 6) u[k] = u[k] * 0x9E3779B1u + (unsigned)k;                              // v_mad_u32_u24 / mul_lo
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k] + (float)u[k] + p[k].x + p[k].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = (unsigned)(t1 - t0);
}

template <int KIND>
static void run(const char* name, int ops_per_iter_k, int ncu) {
  const int waves_per_simd[] = {1, 2, 4, 8};
  for (int w : waves_per_simd) {
    const int blocks = ncu * w;  // 256-thread blocks = 4 waves = 1 per SIMD each
    float* out;
    unsigned* cyc;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&cyc, (size_t)blocks * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    spin<KIND><<<blocks, 256>>>(out, cyc, 1.0f);
    (void)hipEventRecord(e0);
    spin<KIND><<<blocks, 256>>>(out, cyc, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double wave_instr = (double)blocks * 4 * kIters * 8 * ops_per_iter_k;
    const double cu_cycles = ms * 1e-3 * 2.4e9 * ncu;  // at the 2.4 GHz max clock
    std::printf("%-28s waves/SIMD %d: %.3f wave64 VALU instr per CU-cycle (%.3f ms)\n", name, w,
                wave_instr / cu_cycles, ms);
    (void)hipFree(out);
    (void)hipFree(cyc);
  }
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  run<0>("v_fma_f32", 1, ncu);
  run<2>("v_max3_f32", 1, ncu);
  run<3>("v_perm_b32", 1, ncu);
  run<4>("add_u32+cvt_f32_ubyte+add_f32", 3, ncu);
  run<5>("v_pk_fma_f32", 1, ncu);
  run<6>("v_mul_lo_u32 + v_add", 2, ncu);
  return 0;
}
