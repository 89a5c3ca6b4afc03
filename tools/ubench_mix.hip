// Microbenchmark (diagnostic, not product): which VALU instruction kinds of the traversal's
// node visit share an issue slot.  Each lane runs 8 independent chains of an exact
// instruction stream (inline asm, so the compiler neither rewrites nor packs it); the
// kernel's HIP-event time at 1, 2, 4 and 8 waves per SIMD gives wave64 instructions per
// CU-cycle at the 2.4 GHz clock.  A mix reaching ~2 while its parts alone reach ~1 issues
// its two kinds in parallel.
// hipcc --offload-arch=gfx950 -O3 tools/ubench_mix.hip -o tools/bin/ubench_mix
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 16384;

#define A1(op) asm volatile(op : "+v"(x[k]) : "v"(y[k]), "v"(z[k]))
#define U1(op) asm volatile(op : "+v"(u[k]) : "v"(v[k]), "v"(w[k]))

template <int KIND>
__global__ __launch_bounds__(256) void spin(float* out, float seed) {
  float x[8], y[8], z[8];
  unsigned u[8], v[8], w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    x[k] = seed + threadIdx.x * 1e-3f + k;
    y[k] = 1.0001f + k * 1e-4f;
    z[k] = 0.25f * k;
    u[k] = threadIdx.x * 2654435761u + k * 977u;
    v[k] = 0x01010101u * (k + 1);
    w[k] = 0x07030501u;
  }
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (KIND == 0) A1("v_fma_f32 %0, %0, %1, %2");
      if (KIND == 1) A1("v_max3_f32 %0, %0, %1, %2");
      if (KIND == 2) U1("v_max3_i32 %0, %0, %1, %2");
      if (KIND == 3) U1("v_min_u32 %0, %0, %1");
      if (KIND == 4) U1("v_cndmask_b32 %0, %0, %1, vcc");
      if (KIND == 5) asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(x[k]) : "v"(u[k]));
      if (KIND == 6) U1("v_perm_b32 %0, %0, %1, %2");
      if (KIND == 7) U1("v_add_u32 %0, %0, %1");
      if (KIND == 8) { A1("v_fma_f32 %0, %0, %1, %2"); U1("v_max3_i32 %0, %0, %1, %2"); }
      if (KIND == 9) { A1("v_fma_f32 %0, %0, %1, %2"); asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(y[k]) : "v"(u[k])); }
      if (KIND == 10) { A1("v_fma_f32 %0, %0, %1, %2"); U1("v_cndmask_b32 %0, %0, %1, vcc"); }
      if (KIND == 11) { A1("v_max3_f32 %0, %0, %1, %2"); U1("v_max3_i32 %0, %0, %1, %2"); }
      if (KIND == 12) { A1("v_fma_f32 %0, %0, %1, %2"); U1("v_perm_b32 %0, %0, %1, %2"); }
      if (KIND == 13) { A1("v_fma_f32 %0, %0, %1, %2"); U1("v_add_u32 %0, %0, %1"); }
      if (KIND == 14) U1("v_min3_u32 %0, %0, %1, %2");
      if (KIND == 15) { A1("v_fma_f32 %0, %0, %1, %2"); U1("v_min_u32 %0, %0, %1"); }
      if (KIND == 16) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double*)&x[k & 6]) : "v"(*(double*)&y[k & 6]), "v"(*(double*)&z[k & 6]));
      if (KIND == 17) { asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double*)&x[k & 6]) : "v"(*(double*)&y[k & 6]), "v"(*(double*)&z[k & 6])); U1("v_max3_i32 %0, %0, %1, %2"); }
      if (KIND == 18) asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(x[k]), "v"(y[k]) : "vcc");
      if (KIND == 19) asm volatile("v_cmp_lt_u32 vcc, %0, %1" : : "v"(u[k]), "v"(v[k]) : "vcc");
      if (KIND == 20) { A1("v_fma_f32 %0, %0, %1, %2"); asm volatile("v_cmp_lt_u32 vcc, %0, %1" : : "v"(u[k]), "v"(v[k]) : "vcc"); }
      if (KIND == 21) A1("v_sub_f32 %0, %0, %1");
      if (KIND == 22) { A1("v_max3_f32 %0, %0, %1, %2"); asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(y[k]) : "v"(u[k])); }
      // r05: the node visit's remaining kinds and the mixes a restructured visit would issue
      if (KIND == 23) A1("v_max_f32 %0, %0, %1");
      if (KIND == 24) U1("v_max_i32 %0, %0, %1");
      if (KIND == 25) { A1("v_fma_f32 %0, %0, %1, %2"); U1("v_max_i32 %0, %0, %1"); }
      if (KIND == 26) U1("v_cndmask_b32_e64 %0, %0, %1, s[20:21]");
      if (KIND == 27) { A1("v_fma_f32 %0, %0, %1, %2"); U1("v_cndmask_b32_e64 %0, %0, %1, s[20:21]"); }
      if (KIND == 28) A1("v_mul_f32 %0, %0, %1");
      if (KIND == 29) U1("v_and_b32 %0, %0, %1");
      if (KIND == 30) U1("v_lshlrev_b32 %0, %1, %0");
      if (KIND == 31) {  // the node visit's planes as issued now: two byte converts per packed fma
        asm volatile("v_cvt_f32_ubyte0 %0, %1" : "=v"(y[k]) : "v"(u[k]));
        asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(z[k]) : "v"(u[k]));
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double*)&x[k & 6]) : "v"(*(double*)&y[k & 6]), "v"(*(double*)&z[k & 6]));
      }
      if (KIND == 32) {  // ... and with one scalar fma per converted byte
        asm volatile("v_cvt_f32_ubyte0 %0, %1" : "=v"(y[k]) : "v"(u[k]));
        A1("v_fma_f32 %0, %0, %1, %2");
      }
      if (KIND == 33) { A1("v_min_f32 %0, %0, %1"); U1("v_max_i32 %0, %0, %1"); }
      if (KIND == 34) { A1("v_fma_f32 %0, %0, %1, %2"); A1("v_max_f32 %0, %0, %1"); }
      if (KIND == 35) U1("v_med3_i32 %0, %0, %1, %2");
      if (KIND == 36) { A1("v_fma_f32 %0, %0, %1, %2"); U1("v_max3_i32 %0, %0, %1, %2"); U1("v_perm_b32 %0, %0, %1, %2"); }
      if (KIND == 37) U1("v_mul_u32_u24 %0, %0, %1");
      if (KIND == 38) { A1("v_fma_f32 %0, %0, %1, %2"); U1("v_mul_u32_u24 %0, %0, %1"); }
      if (KIND == 39) U1("v_or_b32 %0, %0, %1");
      if (KIND == 40) U1("v_alignbit_b32 %0, %0, %1, %2");
      if (KIND == 41) U1("v_bfe_u32 %0, %0, %1, %2");
      if (KIND == 42) U1("v_lshrrev_b32 %0, %1, %0");
      if (KIND == 43) A1("v_add_f32 %0, %0, %1");
      if (KIND == 44) { A1("v_fma_f32 %0, %0, %1, %2"); U1("v_and_b32 %0, %0, %1"); }
      if (KIND == 45) A1("v_ldexp_f32 %0, %0, %1");
      if (KIND == 46) U1("v_xor_b32 %0, %0, %1");
      if (KIND == 47) U1("v_sub_u32 %0, %0, %1");
      if (KIND == 48) {  // bf16 plane pairs: one select, two extracts, two fmas per child-axis
        U1("v_perm_b32 %0, %0, %1, %2");
        asm volatile("v_and_b32 %0, 0xffff0000, %1" : "=v"(y[k]) : "v"(u[k]));
        asm volatile("v_mul_u32_u24 %0, 0x10000, %1" : "=v"(z[k]) : "v"(u[k]));
        A1("v_fma_f32 %0, %0, %1, %2");
        A1("v_fma_f32 %0, %0, %2, %1");
      }
      if (KIND == 49) {  // byte planes as now (scalar): half a perm, two converts, two fmas per child-axis
        if (k & 1) U1("v_perm_b32 %0, %0, %1, %2");
        asm volatile("v_cvt_f32_ubyte0 %0, %1" : "=v"(y[k]) : "v"(u[k]));
        asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(z[k]) : "v"(u[k]));
        A1("v_fma_f32 %0, %0, %1, %2");
        A1("v_fma_f32 %0, %0, %2, %1");
      }
      if (KIND == 50) { U1("v_sub_u32 %0, %0, %1"); U1("v_ashrrev_i32 %0, 31, %0"); U1("v_or_b32 %0, %0, %1"); }
      if (KIND == 51) U1("v_ashrrev_i32 %0, 31, %0");
      // fp16 plane codes: v_fma_mix_f32 converts its f16 operand (either half) inside the fma
#define MIX(sel) asm volatile("v_fma_mix_f32 %0, %1, %0, %2 " sel : "+v"(x[k]) : "v"(u[k]), "v"(z[k]))
      if (KIND == 52) MIX("op_sel_hi:[1,0,0]");
      if (KIND == 53) MIX("op_sel:[1,0,0] op_sel_hi:[1,0,0]");
      if (KIND == 54) { MIX("op_sel_hi:[1,0,0]"); U1("v_max3_i32 %0, %0, %1, %2"); }
      if (KIND == 55) { MIX("op_sel_hi:[1,0,0]"); U1("v_perm_b32 %0, %0, %1, %2"); }
      if (KIND == 56) { MIX("op_sel_hi:[1,0,0]"); U1("v_add_u32 %0, %0, %1"); }
      if (KIND == 57) { MIX("op_sel_hi:[1,0,0]"); asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(y[k]) : "v"(v[k])); }
      if (KIND == 58) { MIX("op_sel_hi:[1,0,0]"); A1("v_fma_f32 %0, %0, %1, %2"); }
      if (KIND == 59) {  // f16 plane pairs selected by perm: one perm, two mixed fmas per child-axis pair
        U1("v_perm_b32 %0, %0, %1, %2");
        MIX("op_sel_hi:[1,0,0]");
        MIX("op_sel:[1,0,0] op_sel_hi:[1,0,0]");
      }
#undef MIX
    }
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k] + y[k] + (float)u[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int KIND>
static void run(const char* name, double instr_per_k, int ncu) {
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = ncu * wps;  // 256-thread blocks: one wave per SIMD each
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    spin<KIND><<<blocks, 256>>>(out, 1.0f);
    (void)hipEventRecord(e0);
    spin<KIND><<<blocks, 256>>>(out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double wi = (double)blocks * 4 * kIters * 8 * instr_per_k;
    std::printf("%-34s waves/SIMD %d: %.3f wave64 instr per CU-cycle\n", name, wps, wi / (ms * 1e-3 * 2.4e9 * ncu));
    (void)hipFree(out);
  }
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  run<0>("v_fma_f32", 1, ncu);
  run<21>("v_sub_f32", 1, ncu);
  run<1>("v_max3_f32", 1, ncu);
  run<16>("v_pk_fma_f32", 1, ncu);
  run<2>("v_max3_i32", 1, ncu);
  run<14>("v_min3_u32", 1, ncu);
  run<3>("v_min_u32", 1, ncu);
  run<7>("v_add_u32", 1, ncu);
  run<4>("v_cndmask_b32", 1, ncu);
  run<5>("v_cvt_f32_ubyte1", 1, ncu);
  run<6>("v_perm_b32", 1, ncu);
  run<18>("v_cmp_lt_f32", 1, ncu);
  run<19>("v_cmp_lt_u32", 1, ncu);
  run<8>("fma_f32 + max3_i32", 2, ncu);
  run<9>("fma_f32 + cvt_f32_ubyte1", 2, ncu);
  run<10>("fma_f32 + cndmask", 2, ncu);
  run<11>("max3_f32 + max3_i32", 2, ncu);
  run<12>("fma_f32 + perm", 2, ncu);
  run<13>("fma_f32 + add_u32", 2, ncu);
  run<15>("fma_f32 + min_u32", 2, ncu);
  run<17>("pk_fma_f32 + max3_i32", 2, ncu);
  run<20>("fma_f32 + cmp_lt_u32", 2, ncu);
  run<22>("max3_f32 + cvt_f32_ubyte1", 2, ncu);
  run<23>("v_max_f32", 1, ncu);
  run<24>("v_max_i32", 1, ncu);
  run<25>("fma_f32 + max_i32", 2, ncu);
  run<26>("v_cndmask_b32_e64 (sgpr pair)", 1, ncu);
  run<27>("fma_f32 + cndmask_e64", 2, ncu);
  run<28>("v_mul_f32", 1, ncu);
  run<29>("v_and_b32", 1, ncu);
  run<30>("v_lshlrev_b32", 1, ncu);
  run<31>("2 cvt_ubyte + pk_fma (planes now)", 3, ncu);
  run<32>("cvt_ubyte + fma_f32 (scalar planes)", 2, ncu);
  run<33>("min_f32 + max_i32", 2, ncu);
  run<34>("fma_f32 + max_f32", 2, ncu);
  run<35>("v_med3_i32", 1, ncu);
  run<36>("fma_f32 + max3_i32 + perm", 3, ncu);
  run<37>("v_mul_u32_u24", 1, ncu);
  run<38>("fma_f32 + mul_u32_u24", 2, ncu);
  run<39>("v_or_b32", 1, ncu);
  run<40>("v_alignbit_b32", 1, ncu);
  run<41>("v_bfe_u32", 1, ncu);
  run<42>("v_lshrrev_b32", 1, ncu);
  run<43>("v_add_f32", 1, ncu);
  run<44>("fma_f32 + and_b32", 2, ncu);
  run<45>("v_ldexp_f32", 1, ncu);
  run<46>("v_xor_b32", 1, ncu);
  run<47>("v_sub_u32", 1, ncu);
  run<48>("bf16 pair: perm+and+mul_u24+2 fma", 5, ncu);
  run<49>("bytes: 0.5 perm+2 cvt+2 fma", 4.5, ncu);
  run<50>("sub_u32 + ashr + or (cull mask)", 3, ncu);
  run<51>("v_ashrrev_i32", 1, ncu);
  run<52>("v_fma_mix_f32 (lo half)", 1, ncu);
  run<53>("v_fma_mix_f32 (hi half)", 1, ncu);
  run<54>("fma_mix + max3_i32", 2, ncu);
  run<55>("fma_mix + perm", 2, ncu);
  run<56>("fma_mix + add_u32", 2, ncu);
  run<57>("fma_mix + cvt_f32_ubyte1", 2, ncu);
  run<58>("fma_mix + fma_f32", 2, ncu);
  run<59>("f16 pair: perm + 2 fma_mix", 3, ncu);
  return 0;
}
