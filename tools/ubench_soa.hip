// Microbenchmark (diagnostic, not product): a pass over n slots of SoA fields
// ([field][slot], 4-B words) reading R fields and writing W fields per slot, as the logic
// step does; reports the rate for several (R, W) and for a [slot][field] (AoS) layout.
// hipcc --offload-arch=gfx950 -O3 tools/ubench_soa.hip -o tools/bin/ubench_soa
#include <hip/hip_runtime.h>
#include <cstdio>

template <int R, int W>
__global__ __launch_bounds__(256) void soa_pass(const unsigned* __restrict__ in, unsigned* __restrict__ out, int n) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= n) return;
  unsigned acc = 0;
#pragma unroll
  for (int f = 0; f < R; ++f) acc += in[(size_t)f * n + s] * (f + 1);
#pragma unroll
  for (int f = 0; f < W; ++f) out[(size_t)f * n + s] = acc + f;
}

// [slot][field] records of F words: each thread loads/stores its own record (dwordx4 pieces)
template <int F>
__global__ __launch_bounds__(256) void aos_pass(const uint4* __restrict__ in, uint4* __restrict__ out, int n) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= n) return;
  uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < F / 4; ++k) {
    uint4 v = in[(size_t)s * (F / 4) + k];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
#pragma unroll
  for (int k = 0; k < F / 4; ++k) out[(size_t)s * (F / 4) + k] = acc;
}

int main() {
  const int n = 16 << 20;
  unsigned *in, *out;
  hipMalloc(&in, (size_t)n * 32 * 4);
  hipMalloc(&out, (size_t)n * 32 * 4);
  hipMemset(in, 1, (size_t)n * 32 * 4);
  hipMemset(out, 0, (size_t)n * 32 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char* name, auto launch, double bytes) {
    launch();
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    std::printf("%-28s %.3f ms  %.2f TB/s\n", name, ms, bytes / (ms * 1e9));
  };
  const dim3 g(n / 256), t(256);
#define SOA(R, W) run("soa R=" #R " W=" #W, [&] { hipLaunchKernelGGL((soa_pass<R, W>), g, t, 0, 0, in, out, n); }, (double)n * 4 * (R + W))
  SOA(1, 0); SOA(4, 0); SOA(11, 0); SOA(20, 0);
  SOA(0, 1); SOA(0, 4); SOA(0, 11);
  SOA(1, 1); SOA(11, 11); SOA(11, 16); SOA(4, 8);
#define AOS(F) run("aos F=" #F " (r+w)", [&] { hipLaunchKernelGGL((aos_pass<F>), g, t, 0, 0, (const uint4*)in, (uint4*)out, n); }, (double)n * 4 * 2 * F)
  AOS(4); AOS(8); AOS(16); AOS(32);
  return 0;
}
