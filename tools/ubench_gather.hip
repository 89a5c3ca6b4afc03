// Microbenchmark (diagnostic, not product): cost of per-lane dependent record fetches as the
// trace kernel does them, by record size (dwordx4 loads per step) and lane divergence.
// Each lane walks a dependent chain: idx' = hash(record words, idx) over a table of n records;
// groups of G lanes share one chain (G = 64: wave-uniform address, G = 1: 64 distinct lines).
// hipcc --offload-arch=gfx950 -O3 tools/ubench_gather.hip -o /tmp/ubench_gather
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int NL>
__global__ __launch_bounds__(256) void walk(const uint4* __restrict__ tab, unsigned n, int steps, int group,
                                            unsigned* out) {
  const unsigned lane = threadIdx.x & 63;
  const unsigned gid = blockIdx.x * 256 + threadIdx.x;
  unsigned idx = ((gid - lane) + lane / group) * 2654435761u % n;
  unsigned acc = 0;
  for (int s = 0; s < steps; ++s) {
    const uint4* r = tab + (size_t)idx * NL;
    uint4 v[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) v[k] = r[k];
    unsigned h = idx;
#pragma unroll
    for (int k = 0; k < NL; ++k) h = (h ^ v[k].x ^ v[k].y ^ v[k].z ^ v[k].w) * 0x9E3779B1u;
    idx = (h >> 3) % n;
    acc += h;
  }
  out[gid] = acc;
}

int main(int argc, char** argv) {
  const size_t bytes = argc > 1 ? std::atoll(argv[1]) : (28u << 20);
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint4* tab;
  unsigned* out;
  hipMalloc(&tab, bytes);
  std::vector<unsigned> h(bytes / 4);
  unsigned x = 12345;
  for (auto& w : h) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; w = x; }
  hipMemcpy(tab, h.data(), bytes, hipMemcpyHostToDevice);
  const int steps = 2000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int wps : {2, 4}) {  // waves per SIMD
    const int blocks = ncu * wps;  // 256-thread blocks = 4 waves -> wps waves per SIMD
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    for (int group : {64, 16, 4, 1}) {
      for (int nl : {1, 2, 3, 4, 5, 8}) {
        const unsigned n = (unsigned)(bytes / (16 * nl));
        auto launch = [&]() {
          switch (nl) {
            case 1: hipLaunchKernelGGL(walk<1>, dim3(blocks), dim3(256), 0, 0, tab, n, steps, group, out); break;
            case 2: hipLaunchKernelGGL(walk<2>, dim3(blocks), dim3(256), 0, 0, tab, n, steps, group, out); break;
            case 3: hipLaunchKernelGGL(walk<3>, dim3(blocks), dim3(256), 0, 0, tab, n, steps, group, out); break;
            case 4: hipLaunchKernelGGL(walk<4>, dim3(blocks), dim3(256), 0, 0, tab, n, steps, group, out); break;
            case 5: hipLaunchKernelGGL(walk<5>, dim3(blocks), dim3(256), 0, 0, tab, n, steps, group, out); break;
            case 8: hipLaunchKernelGGL(walk<8>, dim3(blocks), dim3(256), 0, 0, tab, n, steps, group, out); break;
          }
        };
        launch();
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double wave_steps = (double)blocks * 4 * steps;
        const double ns_per_wave_step_per_cu = ms * 1e6 / (wave_steps / ncu);
        std::printf("waves/SIMD %d group %2d rec %3d B: %.3f ms, %.2f G lane-steps/s, %.1f CU-ns per wave-step (%.0f clk @2.4GHz)\n",
                    wps, group, 16 * nl, ms, wave_steps * 64 / (ms * 1e6), ns_per_wave_step_per_cu,
                    ns_per_wave_step_per_cu * 2.4);
      }
    }
    hipFree(out);
  }
  return 0;
}
