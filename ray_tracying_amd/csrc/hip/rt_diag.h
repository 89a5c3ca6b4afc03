// rt_diag.h -- diagnostic builds of the traversal (`make variant VDEFS=-DRT_...`), kept out of
// rt_hip.hip: the product build defines every hook below as nothing (device) or a no-op (host),
// so the production kernels are the same instructions with or without this header's options.
//
//   RT_EXIT_TIMING  per wave of a trace launch: start, work-queue exhausted and exit times
//                   (s_memrealtime, 100 MHz), printed per launch as percentiles (DESIGN.md 4:
//                   the launch tail / drain measurements)
//   RT_PHASE_TIMING per wave: s_memtime cycles in the refill, leaf, node and loop-control phases
//                   and the lanes doing useful work in the leaf and node phases, summed into
//                   control-block counters 64..79 and printed per call
//   RT_WRITE_DIAG   the traversal's HBM stores by kind -- stack entries past the LDS rows (8 B),
//                   result words (4 B), hit records (32 B), occlusion words (4 B) -- counted into
//                   control-block counters 80..83 and printed per one-pass call (the PMC
//                   WRITE_SIZE attribution)
//
// Device hooks are macros over the trace kernel's own names (a, ta, lane, item, gtid); host hooks
// are templates over TraceArgs, instantiated where rt_hip.hip calls them.
#ifndef RT_DIAG_H
#define RT_DIAG_H

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#if defined(RT_EXIT_TIMING) || defined(RT_PHASE_TIMING) || defined(RT_WRITE_DIAG)
constexpr bool kDiagBuild = true;
#else
constexpr bool kDiagBuild = false;
#endif

// ---------------------------------------------------------------- RT_WRITE_DIAG
#ifdef RT_WRITE_DIAG
#define RT_WD(k) atomicAdd(a.counters + 80 + (k), 1ull)
#else
#define RT_WD(k)
#endif

// ---------------------------------------------------------------- RT_PHASE_TIMING
#ifdef RT_PHASE_TIMING
// pt_c[k] cycles and pt_n[k] executions of phase k (0 refill, 1 leaf, 2 node, 3 loop control);
// pt_l[k] lane-iterations of useful work and pt_w[k] the wave's capacity -- 64 per node phase, 64
// x the longest leaf per leaf phase, whose useful work is the primitive tests
#define RT_PT_DECL                                                                                   \
  unsigned long long pt_c[4] = {0, 0, 0, 0}, pt_n[4] = {0, 0, 0, 0}, pt_l[4] = {0, 0, 0, 0},        \
                     pt_w[4] = {0, 0, 0, 0}, pt_t = __builtin_amdgcn_s_memtime();
#define RT_PT_MARK(k)                                               \
  do {                                                              \
    const unsigned long long pt_now = __builtin_amdgcn_s_memtime(); \
    pt_c[k] += pt_now - pt_t;                                       \
    pt_n[k] += 1;                                                   \
    pt_t = pt_now;                                                  \
  } while (0)
#define RT_PT_LEAF_LANES                                                          \
  do {                                                                            \
    const int pt_cnt = is_leaf_item(item) ? (int)((uint32_t)item & 0x7fu) : 0;   \
    int pt_mx = pt_cnt, pt_sm = pt_cnt;                                           \
    for (int off = 32; off > 0; off >>= 1) {                                      \
      pt_mx = max(pt_mx, __shfl_xor(pt_mx, off));                                 \
      pt_sm += __shfl_xor(pt_sm, off);                                            \
    }                                                                             \
    pt_l[1] += (unsigned long long)pt_sm;                                         \
    pt_w[1] += 64ull * (unsigned long long)pt_mx;                                 \
  } while (0)
// the node phase: counted (and timed) only when some lane visits a node
#define RT_PT_NODE_BEGIN                          \
  {                                               \
    const uint64_t pt_nm = __ballot(item >= 0);   \
    if (pt_nm) {                                  \
      pt_l[2] += (unsigned long long)__popcll(pt_nm); \
      pt_w[2] += 64ull;                           \
    }
#define RT_PT_NODE_END      \
    if (pt_nm) RT_PT_MARK(2); \
  }
#define RT_PT_FLUSH                                 \
  if (lane == 0)                                    \
    for (int k = 0; k < 4; ++k) {                   \
      atomicAdd(ta.counters + 64 + k, pt_c[k]);     \
      atomicAdd(ta.counters + 68 + k, pt_n[k]);     \
      atomicAdd(ta.counters + 72 + k, pt_l[k]);     \
      atomicAdd(ta.counters + 76 + k, pt_w[k]);     \
    }
#else
#define RT_PT_DECL
#define RT_PT_MARK(k)
#define RT_PT_LEAF_LANES
#define RT_PT_NODE_BEGIN
#define RT_PT_NODE_END
#define RT_PT_FLUSH
#endif

// ---------------------------------------------------------------- RT_EXIT_TIMING
#ifdef RT_EXIT_TIMING
#define RT_ET_BEGIN                                                    \
  const unsigned long long et_begin = __builtin_amdgcn_s_memrealtime(); \
  unsigned long long et_exh = 0;
#define RT_ET_EXHAUSTED et_exh = __builtin_amdgcn_s_memrealtime()
#define RT_ET_END                                                        \
  if (lane == 0) {                                                       \
    unsigned long long* et_e = ta.exit_log + (size_t)(gtid >> 6) * 3;    \
    et_e[0] = et_begin;                                                  \
    et_e[1] = et_exh;                                                    \
    et_e[2] = __builtin_amdgcn_s_memrealtime();                          \
  }
#else
#define RT_ET_BEGIN
#define RT_ET_EXHAUSTED (void)0
#define RT_ET_END
#endif

// ---------------------------------------------------------------- host side
// Every trace launch of a diagnostic build waits for its step (one pipeline, per-step reports).
constexpr bool kDiagStepSync =
#ifdef RT_EXIT_TIMING
    true;
#else
    false;
#endif

// The exit-log buffer of RT_EXIT_TIMING builds (512 K u64: 170 K waves), set on every launch's
// arguments; nothing in the product build.
template <class TA>
inline bool diag_prepare(TA* tas, int n) {
#ifdef RT_EXIT_TIMING
  static unsigned long long* exit_log = nullptr;
  if (!exit_log && hipMalloc(&exit_log, (size_t)1 << 22) != hipSuccess) return false;
  for (int h = 0; h < n; ++h) tas[h].exit_log = exit_log;
#else
  (void)tas;
  (void)n;
#endif
  return true;
}

// After a trace launch `step` of `ms` (its stream synchronised): the exit-time percentiles.
template <class TA>
inline void diag_after_launch(const TA& ta, float ms, int step) {
#ifdef RT_EXIT_TIMING
  const int nw = (int)ta.n_threads / 64;
  std::vector<unsigned long long> lg((size_t)nw * 3);
  if (nw <= 0 || hipMemcpy(lg.data(), ta.exit_log, lg.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  unsigned long long b0 = ~0ull, x0 = ~0ull;
  std::vector<double> ex;
  for (int w = 0; w < nw; ++w) {
    b0 = std::min(b0, lg[(size_t)w * 3]);
    if (lg[(size_t)w * 3 + 1]) x0 = std::min(x0, lg[(size_t)w * 3 + 1]);
  }
  for (int w = 0; w < nw; ++w) ex.push_back((double)(lg[(size_t)w * 3 + 2] - b0) * 1e-5);  // ms
  std::sort(ex.begin(), ex.end());
  std::fprintf(stderr, "[rt exit] step %2d: trace %.3f ms; queue exhausted at %.3f ms; waves exit: 10%% %.3f, 50%% %.3f, "
               "90%% %.3f, 99%% %.3f, last %.3f ms\n",
               step, ms, x0 == ~0ull ? -1.0 : (double)(x0 - b0) * 1e-5, ex[nw / 10], ex[nw / 2], ex[nw * 9 / 10],
               ex[nw * 99 / 100], ex[nw - 1]);
#else
  (void)ta;
  (void)ms;
  (void)step;
#endif
}

// After a call (its control block at `counters`, device): the phase split and the store counts.
inline void diag_after_call(const unsigned long long* counters, bool one_pass) {
#ifdef RT_PHASE_TIMING
  unsigned long long pt[16] = {};
  if (hipMemcpy(pt, counters + 64, sizeof(pt), hipMemcpyDeviceToHost) == hipSuccess) {
    const double tot = (double)(pt[0] + pt[1] + pt[2] + pt[3]);
    std::fprintf(stderr, "[rt phase] refill %.3f (%llu), leaf %.3f (%llu), node %.3f (%llu), control %.3f (%llu) of %.3g "
                 "wave-ticks; lane utilisation: leaf %.3f (%.4g prim tests), node %.3f (%.4g visits)\n",
                 pt[0] / tot, pt[4], pt[1] / tot, pt[5], pt[2] / tot, pt[6], pt[3] / tot, pt[7], tot,
                 pt[13] ? (double)pt[9] / (double)pt[13] : 0.0, (double)pt[9],
                 pt[14] ? (double)pt[10] / (double)pt[14] : 0.0, (double)pt[10]);
  }
#endif
#ifdef RT_WRITE_DIAG
  unsigned long long wd[4] = {};
  if (one_pass && hipMemcpy(wd, counters + 80, sizeof(wd), hipMemcpyDeviceToHost) == hipSuccess)
    std::fprintf(stderr, "[rt writes] HBM stack entries %llu (%.3f GB), result words %llu (%.3f GB), hit records %llu "
                 "(%.3f GB), occlusion words %llu (%.3f GB)\n", wd[0], wd[0] * 8e-9, wd[1], wd[1] * 4e-9, wd[2],
                 wd[2] * 32e-9, wd[3], wd[3] * 4e-9);
#endif
  (void)counters;
  (void)one_pass;
}

#endif  // RT_DIAG_H
