// rt_hip.hip -- MI355X (gfx950) kernels + C ABI for the reference's per-pixel ray-trace path.
//
// Wavefront structure (two kernels per step, iterated until every pixel is done):
//
//   logic_kernel  one thread per SLOT (one sample of one pixel in flight).  Runs the
//                 reference's Trace -> shade recursion for that sample as an explicit state
//                 machine whose state lives in SoA HBM buffers between steps; consumes the
//                 previous query's answer and advances until the slot needs the next scene
//                 query, which it writes to the slot's query record.  A finished sample writes
//                 its colour to the sample buffer; when all 64 slots of a wave are done the
//                 wave claims the next batch of 64 consecutive units (one pixel's samples:
//                 coherent rays) from sharded counters, one 128-B line each.
//   reduce_kernel one thread per pixel (samples staged through LDS): compute_pixel_color sum over the s*s samples in
//                 the reference's order, then the division (raytracer.cpp:46-69).
//   trace_refill_kernel  one lane per query.  BVH::get_intersection (acceleration.cpp:142):
//                 closest-hit for camera/reflection/refraction rays, any-hit-within-tmax for
//                 shadow rays (== the reference's `!hit.shape || t > light_dist`,
//                 raytracer.cpp:233).  Persistent waves; a lane whose query finished takes a
//                 new one when fewer than 48 of 64 still traverse; 4-wide BVH with 64-B nodes
//                 (8-bit conservative child grids), near-first order with t-pruning over an
//                 (entry, t_near) stack in LDS (lane-minor, HBM spill), leaves postponed until
//                 enough lanes wait on one.
//
// Splitting them keeps the heavy recursion/shading state out of the traversal's registers
// (fused, the allocator needed ~250 VGPRs = 1 wave/SIMD).  Leaf boxes are tested with the
// reference's exact AABB::intersect (shapes.cpp:55-72) so the candidate set is the
// reference's; internal boxes are padded on the host and tested by reciprocal slabs.
// Ties on t resolve to the lowest primitive index == the reference's BVH-sorted order
// (std::min_element, acceleration.cpp:112; strict < in intersect_linear, :133).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_device.h"
#include "rt_diag.h"  // diagnostic builds' hooks (RT_WD, RT_PT_*, RT_ET_*, diag_*): nothing in the product
#include "rt_knobs.h"  // the runtime knobs (RT_* environment variables): one table, one snapshot per call

using namespace rtd;

namespace {

constexpr int kMaxDepth = 10;  // MAX_RECURSION_DEPTH, raytracer.hpp:11
constexpr int kBlock = 256;
// default LDS stack entries per lane (RT_LDS_STACK overrides), by the instance's waves/SIMD
// (instance_waves): 12 at 6 waves (6 blocks x 24 KB of LDS per CU) -- every instance but the two
// below -- 11 at 7 (7 x 22 KB: the planes instances of whole frames), 16 at 5 (the soft-light
// chains over transformed shapes; they keep runtime values capped at the tree's depth bound,
// call_lds_entries)
// the production traversal instances (kFixed) take the three loop parameters as constants
// -- the defaults, the LDS stack per waves/SIMD -- so they hold no SGPRs of their own;
// render_tiles launches them when a call's values are exactly these (any tree depth: a shallow
// tree leaves the rows past its depth unused), else the runtime-knob instances (RT_REFILL,
// RT_LEAF_MIN, RT_LDS_STACK, and the soft-light chains)
#ifndef RT_REFILL_DEFAULT
#define RT_REFILL_DEFAULT 48
#endif
#ifndef RT_LEAF_DEFAULT
#define RT_LEAF_DEFAULT 24
#endif
constexpr int kSevenStack = 11, kRefillDefault = RT_REFILL_DEFAULT, kLeafDefault = RT_LEAF_DEFAULT;
constexpr int default_stack(int waves) { return waves >= 7 ? kSevenStack : waves == 6 ? 12 : 16; }
static int lds_stack_entries(int waves) { return (int)knob(K_LDS_STACK, default_stack(waves)); }
// LDS stack entries of a launch: the instance's default rows even for a tree shallower than
// them (the rows past its depth stay unused; the kFixed instances assume the default), an
// RT_LDS_STACK request -- and the soft-light chain instances, which keep runtime values and
// whose 16 default rows at 5 waves/SIMD would fill a CU's LDS (C4 -0.9 %) -- capped at the
// tree's depth bound
static int call_lds_entries(int stack_bound, int waves, bool soft) {
  return knob_set(K_LDS_STACK) || soft ? std::min(stack_bound, lds_stack_entries(waves)) : default_stack(waves);
}
constexpr int kMaxFetchShards = 256;  // trace work counters (slot slices), one 128-B line each
constexpr int kFetchStride = 32;      // u32 words between counters
constexpr int kCtlBytes = 4096;    // control block (cleared by init_kernel)
constexpr int kStatsBytes = 512;  // its head, copied to the host after each batch: counters at bytes 16..32, 488
// scenes with fewer primitives spend their frame in the per-step passes over the slots, not in
// traversal: their shadow rays are fused whatever the call size
constexpr int kFuseFewPrims = 65536;
// scenes of at most this many bounded primitives skip the traversal (TraceArgs::root_item;
// RT_FLAT_PRIMS overrides, 0 = always traverse).  r06 sweep with the one-kernel paths
// (profiles/r06ao_flat_prims_sweep.txt, exported Blender scenes on the step pipeline):
// Distributed (10 bounded) 8,608 -> 19,202 Mrays/s flat, Test1 (21) 9,706 -> 8,413 -- 16
// sits between the two
constexpr int kFlatPrims = 16;
// Batch-claim counters of the logic step: one per 128-B line (kCtrStride words apart) --
// atomics on one line serialise at the memory side, so the shards must not share lines.
constexpr int kMaxBatchShards = 1024;
constexpr int kCtrStride = 32;
// Host batches: up to this many logic -> trace steps are enqueued before the host waits and
// reads their any_query copies.  Steps after the frame's last query find every slot-wave
// retired (logic) and no query (trace) and return at once, so a batch may overshoot.
constexpr int kMaxHostBatch = 16;
constexpr int kMaxFrames = 1024;  // frames of one rt_render_frames call
// Slot pipelines: the slots are split into independent logic -> trace pipelines on their own
// streams, so one pipeline's logic step and launch tail overlap the other's traversal.
constexpr int kPipes = 4;  // at most (RT_PIPES); the default is pipes_env()
constexpr size_t kFetchLines = (size_t)kMaxFetchShards + 2;  // fetch counters + two any_query lines, per pipeline

// ---------------------------------------------------------------- slot state (SoA, HBM)
// field f of slot s lives at state[f * n_slots + s] (32-bit words; floats bit-cast)
// A word is read or written only where it carries information: the logic
// step is bound by these bytes.  The hit being shaded is NOT copied here -- the trace
// kernel's hit record stays intact while the slot traces only shadow queries.
enum Field : int {
  F_UNIT = 0,  // work unit = launch-local pixel * n_samples + sample; -1 = slot retired
  F_CTRL,      // st | depth << 4
  F_LIGHT,     // light index in shade | shadow sample index for that light << 16
  F_VIS,       // visibility accumulator of the current light (kept only while sample index > 0)
  F_FIN,       // 3: shade's final_color (kept only from light 1 on: at light 0 it is the ambient term)
  F_RNG = F_FIN + 3,  // draws consumed in the current sample  } only when a step after the
  F_KEY,              // 2: the sample's RNG stream key        } sample's start can draw
  F_RAY = F_KEY + 2,  // 7: o, d, time of the Trace at `depth` (without frames: o only, and
                      // nothing for a pinhole camera, whose primary rays start at its location)
  F_COUNT = F_RAY + 7
};
// closest-hit record written by the trace kernel, one per slot, AoS (32 B: stored from one
// address by the trace kernel -- no per-field base pointers held in the traversal loop --
// and read as two float4 by the logic step): point, normal, material; the (u, v) of
// textured scenes live in a float2 array of their own (a 48-B record cost every untextured
// scene 16 B per load)
enum HitField : int { HIT_P = 0, HIT_N = 3, HIT_MAT = 6, HIT_STRIDE = 8 };
struct HitRec {
  V3 p, n;
  float u, v;
  uint32_t mat;
};
__device__ __forceinline__ float* hit_rec(float* hit, int slot) { return hit + (size_t)slot * HIT_STRIDE; }
// TraceArgs::has_tex: what a closest hit leaves for the shading (finish_query / settle):
// the 32-B record, the record and (u, v), the hit's t alone (one-pass planes calls), or
// nothing beyond the result index (kHitRecompute: one-pass calls of transformed shapes, whose
// shading recomputes the hit -- compact_hit)
constexpr int kHitRecord = 0, kHitTex = 1, kHitCompact = 2, kHitRecompute = 3;
__device__ __forceinline__ const float* hit_rec(const float* hit, int slot) { return hit + (size_t)slot * HIT_STRIDE; }
__device__ __forceinline__ const float* hit_rec_u(const float* hit, size_t unit) { return hit + unit * HIT_STRIDE; }
// point + normal + material
__device__ __forceinline__ void store_hit_pnm(float* R, V3 p, V3 n, uint32_t mat) {
  *reinterpret_cast<float4*>(R) = make_float4(p.x, p.y, p.z, n.x);
  *reinterpret_cast<float4*>(R + 4) = make_float4(n.y, n.z, __uint_as_float(mat), 0.0f);
}
// point + normal + material (u, v: from the uv array, textured scenes only)
__device__ __forceinline__ HitRec load_hit(const float* R) {
  const float4 a = *reinterpret_cast<const float4*>(R), b = *reinterpret_cast<const float4*>(R + 4);
  return HitRec{V3{a.x, a.y, a.z}, V3{a.w, b.x, b.y}, 0.0f, 0.0f, __float_as_uint(b.z)};
}
// query record, one per slot: o(3) d(3); TMAX = light distance (shadow) or ray time
// (closest); KIND bit 0 = shadow any-hit
// SoA [field][slot] (an AoS record of two float4 measured no faster for the trace kernel and
// cost the logic kernel registers: 132 VGPRs at the same occupancy target)
enum QField : int { Q_O = 0, Q_D = 3, Q_TMAX = 6, Q_KIND = 7, Q_COUNT = 8 };
struct QueryRec {
  V3 o, d;
  float tq;
  int kind;
};
// KIND bit 1: a pinhole camera's primary ray, whose origin (the camera location) is not
// stored -- 12 B less per camera ray for start_kernel to write and the traversal to read
constexpr int kQueryCamOrigin = 2;
__device__ __forceinline__ QueryRec load_query(const float* Q, int N, int slot, const float* cam_loc) {
  const int kind = __float_as_int(Q[Q_KIND * N + slot]);
  const V3 o = (kind & kQueryCamOrigin) ? V3{cam_loc[0], cam_loc[1], cam_loc[2]}
                                        : V3{Q[(Q_O + 0) * N + slot], Q[(Q_O + 1) * N + slot], Q[(Q_O + 2) * N + slot]};
  return QueryRec{o, V3{Q[(Q_D + 0) * N + slot], Q[(Q_D + 1) * N + slot], Q[(Q_D + 2) * N + slot]}, Q[Q_TMAX * N + slot],
                  kind};
}
__device__ __forceinline__ void store_query(float* Q, int N, int slot, V3 o, V3 d, float tq, int kind) {
  Q[(Q_O + 0) * N + slot] = o.x; Q[(Q_O + 1) * N + slot] = o.y; Q[(Q_O + 2) * N + slot] = o.z;
  Q[(Q_D + 0) * N + slot] = d.x; Q[(Q_D + 1) * N + slot] = d.y; Q[(Q_D + 2) * N + slot] = d.z;
  Q[Q_TMAX * N + slot] = tq;
  Q[Q_KIND * N + slot] = __int_as_float(kind);
}
__device__ __forceinline__ void store_cam_query(float* Q, int N, int slot, V3 d, float tq) {
  Q[(Q_D + 0) * N + slot] = d.x; Q[(Q_D + 1) * N + slot] = d.y; Q[(Q_D + 2) * N + slot] = d.z;
  Q[Q_TMAX * N + slot] = tq;
  Q[Q_KIND * N + slot] = __int_as_float(kQueryCamOrigin);
}
__device__ __forceinline__ void store_no_query(float* Q, int N, int slot) { Q[Q_KIND * N + slot] = __int_as_float(-1); }
// frames for depths 0..kMaxDepth-1: A(3) + meta, and the pending refraction ray (6)
enum FrField : int { FR_A = 0, FR_META = 3, FR_COUNT = 4 };

enum : int { ST_SAMPLE = 0, ST_CLOSEST = 1, ST_SHADOW = 2 };
constexpr unsigned int kWaveIdle = 2u;  // wave_done value: every slot of the wave idle (start_kernel's work)
// result word of a shadow query that shadow_step_kernel consumed in this step (results are
// otherwise >= -1: a primitive index, -1 for a miss, or 0 / 1 for a shadow query)
constexpr int kResAdvanced = -2;

struct Common {
  const float4* prims;
  int prim_stride4;
  int n_prims;
  const float4* nodes;
  int use_bvh;
  float eps_abs;
};

// Division by a call-invariant divisor (n / d for any 32-bit n; n % d from it): one mul_hi and
// three ALU ops instead of the ~20-instruction expansion of an integer division.  m =
// floor(2^32 (2^l - d) / d) + 1 with l = ceil(log2 d); q = (t + ((n - t) >> min(l, 1))) >> max(l - 1, 0)
// where t = mul_hi(n, m) (Granlund-Montgomery round-up method).
struct FastDiv {
  uint32_t m, s1, s2;
};
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& d) {
  const uint32_t t = __umulhi(n, d.m);
  return (t + ((n - t) >> d.s1)) >> d.s2;
}
static FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return FastDiv{(uint32_t)m, l < 1 ? l : 1u, l > 1 ? l - 1 : 0u};
}

struct LogicArgs {
  Common c;
  const rt_material* mats;
  const rt_light* lights;
  int n_lights;
  const rt_texture* textures;
  const uint8_t* texels;
  rt_camera_desc cam;
  int spp_sqrt, light_samples;
  uint64_t seed_key;
  // multi-frame calls (rt_render_frames): the call's tile list is the frames' lists end to end,
  // frame f's output tiles at [f * frame_tiles, (f + 1) * frame_tiles) -- and frame f's samples
  // keyed by seed_keys[f] instead of seed_key
  int n_frames;
  const uint64_t* seed_keys;
  FastDiv fd_frame_tiles;
  FastDiv fd_s;              // sample -> (sj, si): division by spp_sqrt
  double inv_s;                 // RN(1 / spp_sqrt): the jitter's quotients (rt_div_by)
  float inv_res_x, inv_res_y;   // RN(1 / res): the camera's pixel -> NDC quotients
  // work
  const int* tile_ids;         // the call's tiles in render order (costliest first, see tile_cost_order)
  const int* tile_out;         // render-order index -> the caller's index (output position); null: identity
  int tile_affine;            // tile_ids[i] == tile_first + i * tile_step (no table lookup)
  int tile_first, tile_step;
  int tile_w, tile_h, tiles_x, sub_x;
  FastDiv fd_tile_px, fd_sub_x, fd_tiles_x, fd_samples;  // the divisions of pixel_coords / unit_coords
  int n_pixels;  // n_tiles * tile_w * tile_h (launch-local pixel space)
  int n_samples; // s*s (1 when s <= 1)
  long long n_units;  // n_pixels * n_samples
  unsigned int* batch_ctr;  // batch_shards counters, kCtrStride words apart; wave w pulls from w % batch_shards
  int batch_shards;
  float* samples;  // [n_units][3] per-sample Trace colours
  float* out;
  // buffers
  int n_slots;           // field stride of every per-slot array (all pipelines' slots)
  int slot_base, slot_end;  // this pipeline's slots [slot_base, slot_end) (multiples of kBlock)
  uint32_t* state;
  uint32_t* frames;      // [kMaxDepth][FR_COUNT][n_slots] (null if no reflection/refraction)
  float* refr;           // [kMaxDepth][6][n_slots] (null if no refraction)
  float* query;          // [Q_COUNT][n_slots]
  int* result;           // [n_slots] (shadow_step_kernel marks consumed results)
  float* hit;            // [n_slots][HIT_STRIDE] (closest hits; written here for transformed shapes)
  float2* hit_uv;        // [n_slots] (u, v) of closest hits in textured scenes
  const float4* prim_shade;  // planes-only scenes: per primitive (normal, material) -- compact hits (compact_hit)
  int late_draws;        // some step after a sample's start draws random numbers (soft lights, glossy)
  int pinhole;           // camera aperture <= 0: primary rays start at the camera location
  int multi_shadow;      // soft lights, light_samples > 1, RT_SOFT_FUSE=0: shadow_step_kernel runs first
  unsigned int* any_query;  // set to 1 by every wave that emits a query (plain store)
  // per-step resets done by start_kernel's first block (no fill launches between kernels):
  // the trace work counters of this step and the other any_query line (the next step's flag;
  // the two lines alternate by step parity)
  unsigned int* any_query_next;
  unsigned int* fetch_reset;
  int fetch_reset_n;
  int first_step;        // the call's first step: slot-wave w takes batch w (no claim atomics)
  int n_fuse;            // > 0: every closest hit's point-light shadow rays were traced with it (occl bits)
  const unsigned int* occl;
  unsigned int* wave_done;  // per slot-wave: 1 once all its slots retired (later steps skip it);
                            // kWaveIdle from logic_kernel to start_kernel: every slot is idle
  // one-pass calls (camera_kernel -> one trace launch -> shade_reduce_kernel; slot == unit): the
  // query record holds only what the call needs, field k of unit u at query[k * n_slots + u] --
  // the direction in fields 0..2, then (-1: absent) the origin (thin lens), the ray time
  // (transformed shapes: moving spheres) and a kind word (some tile reaches past the image)
  int op_fo, op_ft, op_fk;
  // step-pipeline calls of few-primitive scenes (kInline logic instances, r06): the logic step
  // answers the queries it emits itself -- one leaf item of the flat_n bounded primitives and the
  // unbounded ones, as the trace kernel's flat root item does -- and counts them in *rays
  const int2* prim_refs;
  const float4* ref_boxes;
  int n_unbounded;
  int flat_n;
  unsigned long long* rays;
};

#ifndef RT_XCD_CHUNK_DEFAULT
#define RT_XCD_CHUNK_DEFAULT 64  // r05 A/B (same box, 3 reps interleaved): headline +0.9 %, one rank's eighth +0.4 %, C5 +-0
#endif
struct TraceArgs {
  Common c;
  const int2* prim_refs;      // (reference index, reference leaf) per primitive
  const float4* ref_boxes;    // 2 float4 per reference leaf: lo, hi
  int n_unbounded;
  int n_nodes;
  const float* query;
  int* result;
  unsigned int* fetch;        // fetch_shards work counters over slot slices (zeroed per step)
  int fetch_shards;
  int xcd_chunk;              // > 0: XCD-aware deal of chunks of this many groups (fetch loop)
  const unsigned int* any_query;  // logic's "some slot has a query" flag for this step
  float cam_loc[3];           // origin of the queries marked kQueryCamOrigin
  unsigned int* host_flag;    // pinned host word: any_query of this step, for the host's loop
  unsigned long long* rays;   // queries traced (one atomic per wave at exit)
  int n_slots;                // field stride of the per-slot arrays
  int slot_base, n_work;      // this pipeline's query slots: [slot_base, slot_base + n_work)
  int lds_entries;            // traversal stack entries kept in LDS per lane
  int* spill;                 // deeper entries: [entry - lds_entries][n_threads]
  int n_threads;              // threads of the persistent grid
  unsigned long long* counters;  // box tests, prim tests (count_work)
  float* hit;                 // [n_slots][HIT_STRIDE]: attributes of a closest hit (for the logic step)
  float2* hit_uv;             // [n_slots]: (u, v) of a closest hit, textured scenes
  int has_tex;                // hit output: kHitRecord (32-B record), kHitTex (some material is textured:
                              // the record and (u, v)), kHitCompact (one-pass planes calls: t alone),
                              // kHitRecompute (one-pass transformed-shape calls: nothing)
  int refill_min;             // refill kernel: refill finished lanes when fewer than this many traverse
  int leaf_min;               // refill kernel: test postponed leaves once this many lanes wait on one
  int diag;                   // count_work under RT_DIAG: wave-level utilisation counters
  // fused shadow rays (kFuse launches): point lights whose shadow rays a closest hit's lane
  // traces right after the hit, and the per-slot occlusion bits it leaves for the logic step
  const rt_light* lights;
  int n_fuse;
  unsigned int* occl;
  // kSoft launches: a finished soft-light shadow sample with samples left draws and traces
  // the next one in the same lane (shadow_step_kernel's ops on the slot's state)
  uint32_t* state;
  int light_samples;
  // kSoft launches with soft_start: a closest hit also starts its shade loop -- the first
  // shadow sample of light 0, as the logic step would emit it (then continued as above);
  // frames / pinhole tell which of the closest ray's words the shading step reads back
  int soft_start;
  int frames, pinhole;
  const unsigned int* wave_done;  // per 64-slot group: all slots retired (nothing to fetch)
  int drain_help;             // once the queue is dry, free lanes search subtrees of busy lanes' queries
  int one_pass;               // one-pass call: every query is its unit's camera ray (camera_kernel), no slot state
  // the first item of every traversal (render_tiles): the root node, kNoItem (linear mode, no
  // bounded primitive) or -- -bvh on a scene of at most kFlatPrims bounded primitives -- one leaf
  // item of all of them, so the leaf phase tests every bounded primitive, each candidate hit
  // through the reference-leaf filter: the minimum the traversal finds (the tree prunes only
  // subtrees that cannot hold a closer accepted hit), without the node visit and its stack
  int root_item;
  int op_fo, op_ft, op_fk;    // one-pass query fields (LogicArgs): origin, time, kind; -1 absent
  // instrumented one-pass calls: node visits per render-order tile (unit / units per tile),
  // summed per wave at each work fetch -- the measured cost later calls of this camera order
  // their tiles by
  unsigned int* tile_cost;
  FastDiv fd_tile_units;
  unsigned long long* exit_log;  // RT_EXIT_TIMING builds (rt_diag.h): per wave (start, queue exhausted, exit)
};

// ---------------------------------------------------------------- traversal
// The closest-hit / any-hit state of one query.
struct HitState {
  float best_t;
  int best_ref;   // reference index of the best hit (tie-break, acceleration.cpp:112)
  int best_idx;   // primitive index (traversal order) of the best hit, -1 = miss
  bool done;      // any-hit: occluded
};

// The reference accepts a primitive's hit only if its reference leaf box passes the exact
// AABB::intersect (acceleration.cpp:71-75); checked lazily, for candidate hits only.
__device__ __forceinline__ bool ref_leaf_ok(const TraceArgs& a, int leaf, const Ray& r, uint32_t par) {
  const float4 lo = a.ref_boxes[2 * leaf], hi = a.ref_boxes[2 * leaf + 1];
  const float blo[3] = {lo.x, lo.y, lo.z}, bhi[3] = {hi.x, hi.y, hi.z};
  float tn;
  return aabb_exact(blo, bhi, r, par, tn);
}

// Plane hit at parameter t.  The primitive's reference leaf box contains the plane's own box,
// corners -/+ 1e-4f (Plane::get_bounding_box, shapes.cpp:496-503).  A hit point inside that
// box by 2 * eps_abs (eps_abs = 1e-5 * scale) passes the reference's exact slab test on the
// leaf box: along an axis with |d| >= 1e-6 its computed slab bounds err by at most
// |bound - o| * 2^-23 <= 2 * scale * 2^-23, along a near-parallel axis the origin lies within
// |P - o| * 1e-6 <= 2e-6 * scale of the hit point (unit directions; P and o inside the scene
// bound) -- both far below the margin.  Such hits skip ref_leaf_ok's six divisions and its
// extra memory round trip; every other hit takes the exact test.
__device__ __forceinline__ bool plane_leaf_fast_ok(const PrimA& P, const Ray& r, float t, float eps) {
  const float m = 2.0f * eps;
  const float o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float c0 = P.a[k], c1 = P.a[4 + k], c2 = P.a[8 + k];
    const float c3 = (prim_tag(P) & RT_TAG_TRI1_NEVER) ? c0 : P.a[12 + k];  // a[12] is a radius then
    const float lo = fminf(fminf(c0, c1), fminf(c2, c3)) - 1e-4f;
    const float hi = fmaxf(fmaxf(c0, c1), fmaxf(c2, c3)) + 1e-4f;
    const float p = o[k] + t * d[k];
    ok = ok && (p - lo >= m) && (hi - p >= m);
  }
  return ok;
}

// A scene array element at a 32-bit byte offset from its base: global loads with the base in
// SGPRs and the offset in one VGPR, no 64-bit address arithmetic per access (node indices <
// 2^26 and primitive indices < 2^24 are enforced by rt_scene_create).
__device__ __forceinline__ const float4* at_byte(const float4* base, uint32_t off) {
  return reinterpret_cast<const float4*>(reinterpret_cast<const char*>(base) + off);
}

// Tests primitives [first, first + cnt) against the lane's query: only (t, reference index,
// primitive index) of the best hit are kept; its hit record is written once, when the query
// settles (finish_query).
template <bool kCount, bool kPlanesOnly>
__device__ __forceinline__ void test_prims(const TraceArgs& a, int first, int cnt, const Ray& r, bool any, float tmax,
                                           uint32_t par, bool check_leaf, HitState& h, unsigned int& nprim) {
  for (int k = 0; k < cnt; ++k) {
    const int pi = first + k;
    const float4* rec = at_byte(a.c.prims, (uint32_t)pi * ((uint32_t)a.c.prim_stride4 << 4));  // pi < 2^24
    PrimA P;
    load_prim_a(rec, P);
    float t;
    if (kCount) {
      ++nprim;
      if (a.diag && __lane_id() == __ffsll((long long)__ballot(1)) - 1) atomicAdd(a.counters + 61, 1ull);  // wave-level prim tests
    }
    if (kPlanesOnly) {
      if (!plane_hit<false>(P, r, t, nullptr)) continue;
    } else if (!prim_hit<false, false>(P, rec, r, t, nullptr)) {
      continue;
    }
    const int2 ref = a.prim_refs[pi];
    auto leaf_ok = [&]() {
      if (!check_leaf || ref.y < 0) return true;
      if ((kPlanesOnly || RT_TAG_KIND(prim_tag(P)) == RT_PRIM_PLANE) && plane_leaf_fast_ok(P, r, t, a.c.eps_abs))
        return true;
      return ref_leaf_ok(a, ref.y, r, par);
    };
    if (any) {  // occluder iff t <= light_dist (raytracer.cpp:233)
      if (!(t > tmax) && leaf_ok()) {
        h.done = true;
        return;
      }
    } else if ((t < h.best_t || (t == h.best_t && ref.x < h.best_ref)) && leaf_ok()) {
      h.best_t = t;
      h.best_ref = ref.x;
      h.best_idx = pi;
    }
  }
}

// Lanes set in a wave-uniform mask, as a 32-bit SGPR value: with __popcll the compiler kept
// the i64 popcount and compared it in 64 bits -- a VALU v_cmp_gt_u64 (gfx9 has no 64-bit
// scalar ordered compare) at the loop head and the leaf check of every iteration
__device__ __forceinline__ int popc_s(uint64_t m) {
  int c;
  asm("s_bcnt1_i32_b64 %0, %1" : "=s"(c) : "s"(m));
  return c;
}

// a wave-uniform value in an SGPR of its own (opaque to the optimiser: not re-fused with the
// wide load it came from)
__device__ __forceinline__ int sgpr_copy(int v) {
  int r;
  asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "s"(__builtin_amdgcn_readfirstlane(v)));
  return r;
}

// cswap on non-negative (or +inf) floats compared as integers (node_visit's child order)
__device__ __forceinline__ void cswap_bits(float& ta, int& ca, float& tb, int& cb) {
  const int ia = __float_as_int(ta), ib = __float_as_int(tb);
  const bool sw = ib < ia;
  ta = __int_as_float(sw ? ib : ia);
  tb = __int_as_float(sw ? ia : ib);
  const int c = sw ? cb : ca;
  cb = sw ? ca : cb;
  ca = c;
}

// One query's traversal state between node steps.
struct Query {
  Ray r;
  V3 inv;       // reciprocal direction for the culling slabs (|d| clamped away from 0)
  float tmax;   // shadow: light distance
  bool any;     // shadow query: any hit with t <= tmax
  uint32_t par; // bit i: fabs(d_i) < 1e-6 (double), the exact slab's parallel test
  uint32_t sel[3];  // per axis, v_perm_b32 selector of the near-plane code word: 0x03020100
                    // picks the lo word (inv_i >= 0), 0x07060504 the hi word
};

// The traversal form of a query: origin, direction, light distance (shadow) or ray time.
__device__ __forceinline__ void setup_query(Query& q, V3 o, V3 d, float tq, bool any) {
  q.r.o = o;
  q.r.d = d;
  q.any = any;
  q.tmax = q.any ? tq : 0.0f;
  q.r.time = q.any ? 0.0f : tq;  // shadow rays have time 0 (raytracer.cpp:225, shapes.hpp:28)
  uint32_t par = 0;
  par |= ((double)fabsf(q.r.d.x) < 1e-6) ? 1u : 0u;
  par |= ((double)fabsf(q.r.d.y) < 1e-6) ? 2u : 0u;
  par |= ((double)fabsf(q.r.d.z) < 1e-6) ? 4u : 0u;
  q.par = par;
  // culling only: v_rcp_f32 (1 ulp) instead of a correctly rounded division -- a relative
  // 2^-23 error in t is far inside the boxes' 1e-5 * scale padding and the pruning margin
  auto safe_inv = [](float d) {
    float dd = fabsf(d) < 1e-12f ? copysignf(1e-12f, d) : d;
    return __builtin_amdgcn_rcpf(dd);
  };
  q.inv = V3{safe_inv(q.r.d.x), safe_inv(q.r.d.y), safe_inv(q.r.d.z)};
  q.sel[0] = q.inv.x < 0.0f ? 0x07060504u : 0x03020100u;
  q.sel[1] = q.inv.y < 0.0f ? 0x07060504u : 0x03020100u;
  q.sel[2] = q.inv.z < 0.0f ? 0x07060504u : 0x03020100u;
}

// Camera::pixelToRay_thin_lens (camera.cpp:98-179), basis precomputed on the host.
// The divisions px / res and those of the normalisations are correctly rounded quotients by
// a precomputed reciprocal (rt_div.h: the same bits, a third of the instructions).
__device__ __forceinline__ Ray camera_ray(const rt_camera_desc& c, float px, float py, Rng& rng, float inv_rx,
                                          float inv_ry) {
  float nx = 1.0f - rt_div_by(px, (float)c.res_x, inv_rx) * 2.0f;
  float ny = 1.0f - rt_div_by(py, (float)c.res_y, inv_ry) * 2.0f;
  float nxr = nx * c.half_sensor_w, nyr = ny * c.half_sensor_h;
  V3 dw{c.x_dir[0] * nxr + c.y_dir[0] * nyr + c.z_dir[0] * c.focal_length,
        c.x_dir[1] * nxr + c.y_dir[1] * nyr + c.z_dir[1] * c.focal_length,
        c.x_dir[2] * nxr + c.y_dir[2] * nyr + c.z_dir[2] * c.focal_length};
  dw = normalize_rcp(dw);
  Ray r;
  r.time = 0.0f;
  V3 loc{c.location[0], c.location[1], c.location[2]};
  if (c.aperture <= 0.0f) {
    r.o = loc;
    r.d = dw;
    return r;
  }
  V3 fp{loc.x + dw.x * c.focus_dist, loc.y + dw.y * c.focus_dist, loc.z + dw.z * c.focus_dist};
  float rx, ry;
  for (;;) {  // random_in_unit_disk (camera.cpp:90-96)
    rx = (float)rng.next() * 2.0f - 1.0f;
    ry = (float)rng.next() * 2.0f - 1.0f;
    if (rx * rx + ry * ry < 1.0f) break;
  }
  float lr = c.aperture / 2.0f;
  rx *= lr;
  ry *= lr;
  V3 off{c.x_dir[0] * rx + c.y_dir[0] * ry, c.x_dir[1] * rx + c.y_dir[1] * ry,
         c.x_dir[2] * rx + c.y_dir[2] * ry};
  r.o = add(loc, off);
  r.d = normalize_rcp(sub(fp, r.o));
  return r;
}

// launch-local pixel index -> image (x, y) and output offset; 8x8 blocks inside tiles so
// consecutive slots trace spatially coherent rays.
__device__ __forceinline__ bool pixel_coords(const LogicArgs& a, int p, int& x, int& y, size_t& out_off) {
  const int tile_px = a.tile_w * a.tile_h;
  const int tl = (int)fdiv((uint32_t)p, a.fd_tile_px), r = p - tl * tile_px;
  const int b = r >> 6, l = r & 63;
  const int by = (int)fdiv((uint32_t)b, a.fd_sub_x), bx = b - by * a.sub_x;
  const int lx = bx * 8 + (l & 7), ly = by * 8 + (l >> 3);
  const int tid = a.tile_affine ? a.tile_first + tl * a.tile_step : a.tile_ids[tl];
  const int ty = (int)fdiv((uint32_t)tid, a.fd_tiles_x), tx = tid - ty * a.tiles_x;
  x = tx * a.tile_w + lx;
  y = ty * a.tile_h + ly;
  const int to = a.tile_out ? a.tile_out[tl] : tl;
  out_off = ((size_t)to * tile_px + (size_t)ly * a.tile_w + lx) * 3;
  return x < a.cam.res_x && y < a.cam.res_y;
}

// shade's specular term is m.specular * powf(ndh, shininess) (raytracer.cpp:245-250): with
// every component of the specular colour zero it is +0 (or -0 for a -0 component) whenever the
// power is finite -- ndh = max(0, dot) is never NaN and at most 1 + a few ulps, so any shininess
// in [0, 5e6] (the JSON loader's 5 / r^2, json_loader.cpp:56-61, lies in [5, 5e6]) -- and the
// glibc powf restatement (~100 instructions, much of it binary64) can be skipped: same bits.
// The Blender scenes' materials (C3, C4) are all such.  rt_scene_create decides it per
// material on the host and marks the device copy (kMatSpecSkip in rt_material.pad): a C-ABI
// caller's NaN, negative or huge shininess keeps the powf, and with it the reference's
// 0 * inf = NaN.
constexpr int32_t kMatSpecSkip = 1;
__device__ __forceinline__ bool spec_zero(const rt_material& m) { return (m.pad & kMatSpecSkip) != 0; }

// ---------------------------------------------------------------- logic kernel
// unit -> (launch-local pixel, sample) and the counter-RNG key of its frame; false if the pixel
// lies outside the image
// (frames = false: the step pipeline, whose calls render one frame -- rt_render_frames runs
// them one after another)
__device__ __forceinline__ bool unit_coords(const LogicArgs& a, long long unit, int& px, int& py, int& sample,
                                            uint64_t& key, bool frames = true) {
  // units < 2^31 (checked on the host): 32-bit unsigned division
  const unsigned u = (unsigned)unit, ns = (unsigned)a.n_samples;
  const int p = (int)fdiv(u, a.fd_samples);
  sample = (int)(u - (unsigned)p * ns);
  key = a.seed_key;
  if (frames && a.n_frames > 1) {  // the frame of the unit's output tile
    const int tl = (int)fdiv((uint32_t)p, a.fd_tile_px);
    const int to = a.tile_out ? a.tile_out[tl] : tl;
    key = a.seed_keys[fdiv((uint32_t)to, a.fd_frame_tiles)];
  }
  size_t off;
  return pixel_coords(a, p, px, py, off);
}

// compute_pixel_color (raytracer.cpp:18-70): the camera ray of sample `sample` of pixel (px,
// py) -- its RNG stream (keyed by the frame's seed), the stratified jitter in double,
// Camera::pixelToRay_thin_lens (the lens draws for an aperture > 0).  The ray's time is the
// caller's next draw.
// (draws = false: the caller knows the sample draws nothing -- one spp, a pinhole, no ray time
// -- and the stream's key, two splitmix64 rounds of quarter-rate 64-bit multiplies, is skipped)
__device__ __forceinline__ Ray sample_ray(const LogicArgs& a, int px, int py, int sample, uint64_t key, Rng& rng,
                                          bool draws = true) {
  if (draws) rng.begin(key, (uint64_t)py * (uint64_t)a.cam.res_x + (uint64_t)px, (uint64_t)sample);
  const int s = a.spp_sqrt;
  float fx, fy;
  if (s <= 1) {
    fx = (float)px + 0.5f;
    fy = (float)py + 0.5f;
  } else {  // the divisions by s: fast invariant integer division, Markstein quotients (rt_div.h)
    const int sj = (int)fdiv((uint32_t)sample, a.fd_s), si = sample - sj * s;
    double ox = rng.next();
    double oy = rng.next();
    double sx = rt_div_by((double)si + ox, (double)s, a.inv_s);
    double sy = rt_div_by((double)sj + oy, (double)s, a.inv_s);
    fx = (float)((double)px + sx);
    fy = (float)((double)py + sy);
  }
  return camera_ray(a.cam, fx, fy, rng, a.inv_res_x, a.inv_res_y);
}

// Reads slot's query record; false if the slot emitted no query this step.
__device__ __forceinline__ bool begin_query(const TraceArgs& a, int slot, Query& q) {
  if (a.one_pass) {  // the unit's camera ray (camera_kernel): 64-bit field offsets (up to 2^30 slots)
    const size_t n = (size_t)(unsigned)a.n_slots, u = (size_t)(unsigned)slot;
    if (a.op_fk >= 0 && __float_as_int(a.query[(size_t)a.op_fk * n + u]) < 0) return false;
    V3 o{a.cam_loc[0], a.cam_loc[1], a.cam_loc[2]};
    if (a.op_fo >= 0) {
      const float* Qo = a.query + (size_t)a.op_fo * n + u;
      o = V3{Qo[0], Qo[n], Qo[2 * n]};
    }
    setup_query(q, o, V3{a.query[u], a.query[n + u], a.query[2 * n + u]},
                a.op_ft >= 0 ? a.query[(size_t)a.op_ft * n + u] : 0.0f, false);
    return true;
  }
  const int N = a.n_slots;
  const int kind = __float_as_int(a.query[Q_KIND * N + slot]);
  if (kind < 0) return false;
  const V3 o = (kind & kQueryCamOrigin)
                   ? V3{a.cam_loc[0], a.cam_loc[1], a.cam_loc[2]}
                   : V3{a.query[(Q_O + 0) * N + slot], a.query[(Q_O + 1) * N + slot], a.query[(Q_O + 2) * N + slot]};
  setup_query(q, o, V3{a.query[(Q_D + 0) * N + slot], a.query[(Q_D + 1) * N + slot], a.query[(Q_D + 2) * N + slot]},
              a.query[Q_TMAX * N + slot], (kind & 1) != 0);
  return true;
}

// After the traversal: the primitives whose region could not be boxed (tested by every ray).
template <bool kCount, bool kPlanesOnly>
__device__ __forceinline__ void complete_query(const TraceArgs& a, int slot, const Query& q, HitState& h,
                                               unsigned int& nprim) {
  if (a.c.use_bvh && !h.done && a.n_unbounded > 0)
    test_prims<kCount, kPlanesOnly>(a, a.c.n_prims - a.n_unbounded, a.n_unbounded, q.r, q.any, q.tmax, q.par, true, h, nprim);
}

// The result word and (closest hits of planes-only scenes) the hit record the shading reads,
// written once here: Plane::intersect's hit point o + t d from the best t (the same ops as the
// test, so the same bits) and the record's precomputed normal (shapes.cpp:472-480) and
// material -- in hp / hn too, for a fused shadow ray that follows (returns true then).
// kHitCompact (one-pass planes-only calls without textures, at most one fused light: r06): only
// the hit's t, 4 B instead of the 32-B record -- shade_reduce_kernel rebuilds the record from t,
// the unit's query record and the primitive (compact_hit) with the same ops.
// Transformed shapes get their record from the lane's settle (fused / soft-start instances) or
// the logic step.
template <bool kCount, bool kPlanesOnly>
__device__ __forceinline__ bool finish_query(const TraceArgs& a, int slot, const Query& q, HitState& h,
                                             unsigned int& nprim, V3& hp, V3& hn) {
  const Ray& r = q.r;
  complete_query<kCount, kPlanesOnly>(a, slot, q, h, nprim);
  a.result[slot] = q.any ? (h.done ? 1 : 0) : h.best_idx;
  RT_WD(1);
  // (an opaque copy, compared here: compares hoisted to the kernel's entry stay live across the
  // traversal loop in SGPRs of their own -- 2 to 6 more spilled)
  const int hit_mode = kPlanesOnly ? sgpr_copy(a.has_tex) : a.has_tex;
  if (kPlanesOnly && hit_mode != kHitTex && !q.any && h.best_idx >= 0) {
    RT_WD(2);
    const float4* rec = at_byte(a.c.prims, (uint32_t)h.best_idx * ((uint32_t)a.c.prim_stride4 << 4));  // < 2^24
    const float* w = reinterpret_cast<const float*>(rec);
    hn = V3{w[3], w[7], w[11]};
    const uint32_t tag = __float_as_uint(w[15]);
    hp = V3{r.o.x + h.best_t * r.d.x, r.o.y + h.best_t * r.d.y, r.o.z + h.best_t * r.d.z};
    if (hit_mode == kHitCompact) a.hit[slot] = h.best_t;
    else store_hit_pnm(hit_rec(a.hit, slot), hp, hn, RT_TAG_MATERIAL(tag));
    return true;
  }
  if (kPlanesOnly && hit_mode == kHitTex && !q.any && h.best_idx >= 0) {
    // textured planes: the hit record with (u, v) -- the same primitive test with attributes,
    // on the primitive this lane just tested (cached).  Scenes with transformed shapes get
    // their record from the logic step (logic_kernel, ST_CLOSEST): sphere / cube / rectangle
    // attributes (double atan2 / asin UVs, object-to-world transforms) would push this
    // kernel past its 128 registers.
    const float4* rec = a.c.prims + (size_t)h.best_idx * a.c.prim_stride4;
    PrimA P;
    load_prim_a(rec, P);
    HitAttr at;
    float t;
    prim_hit<true, true, true>(P, rec, r, t, &at);
    store_hit_pnm(hit_rec(a.hit, slot), at.p, at.n, RT_TAG_MATERIAL(prim_tag(P)));
    a.hit_uv[slot] = make_float2(at.u, at.v);
    hp = at.p;
    hn = at.n;
    return true;
  }
  return false;
}

template <bool kCount>
__device__ __forceinline__ void trace_counters_out(const TraceArgs& ta, int lane, unsigned int nrays, unsigned int nbox,
                                                   unsigned int nprim, unsigned long long dg_any_rays,
                                                   unsigned long long dg_any_box, unsigned int nvisit) {
  unsigned long long nr = nrays;
  for (int off = 32; off > 0; off >>= 1) nr += __shfl_xor(nr, off);
  if (lane == 0 && nr) atomicAdd(ta.rays, nr);
  if (kCount) {
    unsigned long long b = nbox, p = nprim;
    for (int off = 32; off > 0; off >>= 1) {
      b += __shfl_xor(b, off);
      p += __shfl_xor(p, off);
    }
    if (lane == 0 && (b | p)) {
      atomicAdd(ta.counters + 0, b);
      atomicAdd(ta.counters + 1, p);
    }
    for (int off = 32; off > 0; off >>= 1) {
      dg_any_rays += __shfl_xor(dg_any_rays, off);
      dg_any_box += __shfl_xor(dg_any_box, off);
    }
    unsigned long long v = nvisit;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) {  // ctl byte 512
      atomicAdd(ta.counters + 62, dg_any_rays);
      atomicAdd(ta.counters + 63, dg_any_box);
      atomicAdd(ta.counters + 59, v);  // lane-level node visits
    }
  }
}

// Instrumented (count_work) one-pass calls: the wave's node visits since its last work fetch
// (its lanes' nvisit counts past their values then, `base`) added to the tile of the group it
// fetched then -- most of the wave's rays come from it.  Production instances count nothing
// (a per-visit count in the traversal loop cost 21 % through register pressure).
__device__ __forceinline__ void flush_tile_cost(const TraceArgs& a, int lane, int tile, unsigned int nvisit,
                                                unsigned int& base, unsigned int nrays, unsigned int& rbase) {
  unsigned int v = nvisit - base, r = nrays - rbase;
  base = nvisit;
  rbase = nrays;
  for (int off = 32; off > 0; off >>= 1) {
    v += __shfl_xor(v, off);
    r += __shfl_xor(r, off);
  }
  if (lane == 0 && tile >= 0 && (v | r)) {
    atomicAdd(a.tile_cost + 2 * tile, v);
    atomicAdd(a.tile_cost + 2 * tile + 1, r);
  }
}

// ---- refill kernel with postponed leaves
// Stack / item entries: a node index (>= 0), a leaf = kLeafBit | first << 7 | count (first <
// 2^24, count < 128), or kNoItem.  Each stack entry carries its t_near so it is re-culled
// against the bound current when it is popped.
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr int kNoItem = -1;
__device__ __forceinline__ bool is_leaf_item(int e) { return e != kNoItem && e < 0; }

// The lane's stack pointer is one word, the LDS byte offset of its next free entry:
// w = sp * kStackRow + threadIdx.x * 8 (entries are lane-minor rows of the block's 8-B
// (entry, t_near) pairs), so a push or pop is one add and the lane's own base never has to
// stay live across the traversal loop (r04: kept apart, the base was spilled to scratch and
// reloaded on every node visit and pop).  sp = w / kStackRow; w % kStackRow is the lane's
// column; entries from lds_entries on live in the HBM spill area at gtid.
constexpr int kStackRow = kBlock * 8;
static_assert((kStackRow & (kStackRow - 1)) == 0, "stack rows are a power of two");
__device__ __forceinline__ int stack_depth(int w) { return w / kStackRow; }
__device__ __forceinline__ int stack_empty_word(int w) { return w & (kStackRow - 1); }

struct LaneStack {
  char* lds;   // the block's LDS stack area
  int2* spill; // entries past lds_entries: spill[(i - lds) * n_threads + gtid]
};

__device__ __forceinline__ int2* stack_at(const TraceArgs& a, const LaneStack& S, int w_col, int i, int gtid) {
  return i < a.lds_entries ? reinterpret_cast<int2*>(S.lds + w_col + i * kStackRow)
                           : S.spill + (size_t)(i - a.lds_entries) * a.n_threads + gtid;
}

__device__ __forceinline__ void stack_push(const TraceArgs& a, const LaneStack& S, int& w, int gtid, int e, float t) {
  const int sp = stack_depth(w);
  if (sp < a.lds_entries) {
    *reinterpret_cast<int2*>(S.lds + w) = make_int2(e, __float_as_int(t));
  } else {
    S.spill[(size_t)(sp - a.lds_entries) * a.n_threads + gtid] = make_int2(e, __float_as_int(t));
    RT_WD(0);
  }
  w += kStackRow;
}

// Pops entries until one is still within the bound (each popped entry is re-culled against
// the bound current now); kNoItem when the stack empties.  Wave-uniform fast path when no
// lane's stack reaches into the HBM spill area.
__device__ __forceinline__ int stack_pop_live(const TraceArgs& a, const LaneStack& S, int& w, int gtid, float lim) {
  if (__ballot(w >= (a.lds_entries + 1) * kStackRow) == 0ull) {
    while (w >= kStackRow) {
      w -= kStackRow;
      const int2 v = *reinterpret_cast<const int2*>(S.lds + w);
      if (!(__int_as_float(v.y) > lim)) return v.x;
    }
    return kNoItem;
  }
  while (w >= kStackRow) {
    w -= kStackRow;
    const int2 v = *stack_at(a, S, stack_empty_word(w), stack_depth(w), gtid);
    if (!(__int_as_float(v.y) > lim)) return v.x;
  }
  return kNoItem;
}

// Drain: removes and returns the lane's bottom stack entry -- pushed first, so the farthest
// pending subtree of the query -- and moves the others down one, so sp never exceeds the
// serial traversal's depth bound (the order of the rest is kept).
__device__ __forceinline__ int2 stack_take_bottom(const TraceArgs& a, const LaneStack& S, int& w, int gtid) {
  const int col = stack_empty_word(w), sp = stack_depth(w);
  const int2 b = *stack_at(a, S, col, 0, gtid);
  for (int i = 1; i < sp; ++i) {
    *stack_at(a, S, col, i - 1, gtid) = *stack_at(a, S, col, i, gtid);
    if (i - 1 >= a.lds_entries) RT_WD(0);
  }
  w -= kStackRow;
  return b;
}

__device__ __forceinline__ float cull_limit(const TraceArgs& a, const Query& q, const HitState& h) {
  const float lim = q.any ? q.tmax : h.best_t;
  return lim + (lim * 1e-5f + a.c.eps_abs);
}

// Issue priority around the node fetch (r06): a wave that has decided its next node runs at
// s_setprio kVisitPrio until that node's loads are issued, then at 0 -- the SIMD's arbiter
// prefers the waves about to fetch, so more fetches are in flight while the others compute
// (same box, 3 reps: headline +1.1 % at 2, +1.3 % at 1; C3 +-0; level 3 and the leaf phase at
// priority 0 measured no better, profiles/r06l_ab_prio_variants.txt).  RT_SETPRIO=0 builds without.
#ifndef RT_SETPRIO
#define RT_SETPRIO 1
#endif
constexpr int kVisitPrio = RT_SETPRIO;

// One 4-wide node visit: every child box the ray enters within the bound -- internal nodes
// and leaves alike -- is ordered by t_near; the three farthest are pushed, the nearest
// becomes the lane's item (a leaf item waits for the next leaf phase).
//
// Per axis the ray's direction sign picks which of the two code words holds the near planes
// of all four children (inv > 0: lo, else hi; one v_perm_b32 with a per-ray byte selector,
// operands swapped for the far word; two per side with the fp16 codes of kF16, two planes
// per word), so each child needs one max3 and one min3
// instead of three min/max pairs.  Empty children carry inverted boxes (lo 255, hi 0) and
// always miss; child entries come precomputed from the host (node index, or the encoded
// leaf), so nothing is decoded here.  `lim` is the cull bound (cull_limit) of the query.
template <bool kCount, bool kF16>
__device__ __forceinline__ int node_visit(const TraceArgs& a, const Query& q, float lim, int node,
                                          const LaneStack& S, int& w, int gtid, unsigned int& nbox,
                                          unsigned long long& dg_any_box, unsigned int& nvisit) {
  const Ray& r = q.r;
  const V3& inv = q.inv;
  float tnx[4], tfx[4], tny[4], tfy[4], tnz[4], tfz[4];
  int cc[4];
  uint32_t meta;  // count_work: byte k nonzero for a child in slot k
  // the slab terms of the node's grid: plane = origin + code * 2^k per axis, so t = A + code * B
  // with A = (origin - o) * inv and B = inv * 2^k -- one v_ldexp_f32 from the node's signed
  // exponent byte k (upload_nodes), the bits the multiply by the power-of-two float gives
  auto g_terms = [&](const float4 g, float& ax, float& bx, float& ay, float& by, float& az, float& bz) {
    const int ex = __float_as_int(g.w);
    ax = (g.x - r.o.x) * inv.x, bx = __builtin_ldexpf(inv.x, (ex << 24) >> 24);
    ay = (g.y - r.o.y) * inv.y, by = __builtin_ldexpf(inv.y, (ex << 16) >> 24);
    az = (g.z - r.o.z) * inv.z, bz = __builtin_ldexpf(inv.z, (ex << 8) >> 24);
  };
  float ax, bx, ay, by, az, bz;
  if constexpr (kF16) {
    // planes-only scenes: 80-B device nodes with fp16 plane codes (upload_nodes); v_fma_mix_f32
    // converts each code inside its fma -- the value the byte convert gives, so the same bits --
    // and takes the 24 byte converts out of the visit (r05 A/B, same box: headline +2.9 %, one
    // rank's eighth +2.3 %, C5 +3.6 %; the code pairs picked by a per-lane load address
    // instead of the perms: -13 %, eight loads per visit).  Transformed-shape instances keep the
    // byte codes: there the wider node cost 10 more spilled VGPRs (C3 -4.5 %).
    const char* nb = reinterpret_cast<const char*>(a.c.nodes) + (uint32_t)node;  // entry = the node's byte offset
    const float4 g = *reinterpret_cast<const float4*>(nb);
    const int4 qc = *reinterpret_cast<const int4*>(nb + 64);
    uint32_t nx0, nx1, fx0, fx1, ny0, ny1, fy0, fy1, nz0, nz1, fz0, fz1;
    // words (lo01, lo23, hi01, hi23) per axis; perm(hi, lo, sel) is the near pair
    const uint4 px = *reinterpret_cast<const uint4*>(nb + 16);
    const uint4 py = *reinterpret_cast<const uint4*>(nb + 32);
    const uint4 pz = *reinterpret_cast<const uint4*>(nb + 48);
    if constexpr (kVisitPrio > 0) __builtin_amdgcn_s_setprio(0);  // the node's loads are out
    nx0 = __builtin_amdgcn_perm(px.z, px.x, q.sel[0]), nx1 = __builtin_amdgcn_perm(px.w, px.y, q.sel[0]);
    fx0 = __builtin_amdgcn_perm(px.x, px.z, q.sel[0]), fx1 = __builtin_amdgcn_perm(px.y, px.w, q.sel[0]);
    ny0 = __builtin_amdgcn_perm(py.z, py.x, q.sel[1]), ny1 = __builtin_amdgcn_perm(py.w, py.y, q.sel[1]);
    fy0 = __builtin_amdgcn_perm(py.x, py.z, q.sel[1]), fy1 = __builtin_amdgcn_perm(py.y, py.w, q.sel[1]);
    nz0 = __builtin_amdgcn_perm(pz.z, pz.x, q.sel[2]), nz1 = __builtin_amdgcn_perm(pz.w, pz.y, q.sel[2]);
    fz0 = __builtin_amdgcn_perm(pz.x, pz.z, q.sel[2]), fz1 = __builtin_amdgcn_perm(pz.y, pz.w, q.sel[2]);
    g_terms(g, ax, bx, ay, by, az, bz);
    cc[0] = qc.x, cc[1] = qc.y, cc[2] = qc.z, cc[3] = qc.w;
    auto lo = [](uint32_t w, float B, float A) {
      return __builtin_fmaf((float)__builtin_bit_cast(_Float16, (unsigned short)(w & 0xffffu)), B, A);
    };
    auto hi = [](uint32_t w, float B, float A) {
      return __builtin_fmaf((float)__builtin_bit_cast(_Float16, (unsigned short)(w >> 16)), B, A);
    };
    tnx[0] = lo(nx0, bx, ax), tnx[1] = hi(nx0, bx, ax), tnx[2] = lo(nx1, bx, ax), tnx[3] = hi(nx1, bx, ax);
    tfx[0] = lo(fx0, bx, ax), tfx[1] = hi(fx0, bx, ax), tfx[2] = lo(fx1, bx, ax), tfx[3] = hi(fx1, bx, ax);
    tny[0] = lo(ny0, by, ay), tny[1] = hi(ny0, by, ay), tny[2] = lo(ny1, by, ay), tny[3] = hi(ny1, by, ay);
    tfy[0] = lo(fy0, by, ay), tfy[1] = hi(fy0, by, ay), tfy[2] = lo(fy1, by, ay), tfy[3] = hi(fy1, by, ay);
    tnz[0] = lo(nz0, bz, az), tnz[1] = hi(nz0, bz, az), tnz[2] = lo(nz1, bz, az), tnz[3] = hi(nz1, bz, az);
    tfz[0] = lo(fz0, bz, az), tfz[1] = hi(fz0, bz, az), tfz[2] = lo(fz1, bz, az), tfz[3] = hi(fz1, bz, az);
    meta = (__float_as_uint(g.w) >> 24) * 0x00204081u & 0x01010101u;  // valid mask bit k -> byte k
  } else {
    const float4* nd = at_byte(a.c.nodes, (uint32_t)node << 6);  // node < 2^26 (rt_scene_create)
    const float4 g = nd[0];
    const uint4 qa = *reinterpret_cast<const uint4*>(nd + 1);
    const uint4 qb = *reinterpret_cast<const uint4*>(nd + 2);
    const int4 qc = *reinterpret_cast<const int4*>(nd + 3);
    if constexpr (kVisitPrio > 0) __builtin_amdgcn_s_setprio(0);  // the node's loads are out
    cc[0] = (int)qb.w, cc[1] = qc.x, cc[2] = qc.y, cc[3] = qc.z;
    g_terms(g, ax, bx, ay, by, az, bz);
    // perm(hi, lo, sel) is the near word; swapping the operands gives the far one
    const uint32_t nxw = __builtin_amdgcn_perm(qa.y, qa.x, q.sel[0]), fxw = __builtin_amdgcn_perm(qa.x, qa.y, q.sel[0]);
    const uint32_t nyw = __builtin_amdgcn_perm(qa.w, qa.z, q.sel[1]), fyw = __builtin_amdgcn_perm(qa.z, qa.w, q.sel[1]);
    const uint32_t nzw = __builtin_amdgcn_perm(qb.y, qb.x, q.sel[2]), fzw = __builtin_amdgcn_perm(qb.x, qb.y, q.sel[2]);
    // one v_fma_f32 per plane: on gfx950 it issues beside the byte converts, where a v_pk_fma_f32
    // (two planes) does not (tools/ubench_mix.hip; r05 A/B: headline +2.5 %, one rank's eighth
    // +2.6 %, C5 +3.6 %; the same fma per plane, so the same bits)
    auto pl = [](uint32_t w, int k, float B, float A) { return __builtin_fmaf((float)((w >> (8 * k)) & 0xffu), B, A); };
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      tnx[k] = pl(nxw, k, bx, ax), tfx[k] = pl(fxw, k, bx, ax);
      tny[k] = pl(nyw, k, by, ay), tfy[k] = pl(fyw, k, by, ay);
      tnz[k] = pl(nzw, k, bz, az), tfz[k] = pl(fzw, k, bz, az);
    }
    meta = qb.z;
  }
  if (kCount) {
    const uint64_t wm = __ballot(1);
    if (a.diag && __lane_id() == __ffsll((long long)wm) - 1) atomicAdd(a.counters + 60, 1ull);  // wave-level node visits
    if (a.diag) {  // ... of which every visiting lane's ray has the same direction octant
      const uint64_t sx = __ballot(q.inv.x < 0.0f), sy = __ballot(q.inv.y < 0.0f), sz = __ballot(q.inv.z < 0.0f);
      const bool uni = (sx == 0ull || sx == wm) && (sy == 0ull || sy == wm) && (sz == 0ull || sz == wm);
      if (uni && __lane_id() == __ffsll((long long)wm) - 1) atomicAdd(a.counters + 57, 1ull);
    }
    ++nvisit;
    const unsigned nb = __builtin_popcount((meta | (meta >> 1) | (meta >> 2) | (meta >> 3) | (meta >> 4) |
                                            (meta >> 5) | (meta >> 6) | (meta >> 7)) & 0x01010101u);
    nbox += nb;
    if (q.any) dg_any_box += nb;
  }
  // entered within the bound: max(t_near, 0) <= min(t_far, lim)  (lim > 0 always), i.e.
  // t_near <= t_far, t_far >= 0 and t_near <= lim; misses sort last as (inf, entry)
  float t[4];
  int c[4];
  // the test on the values' bit patterns as signed integers: for floats >= +0
  // integer order is float order, a negative float is a negative integer, so
  // max(tnx, tny, tnz, 0) is exact and a negative far distance still fails the test (its
  // value no longer matters); a far distance of exactly -0 now fails too -- conservative, as
  // no accepted hit lies there (the origin would sit on a padded box's far face)
  const int lim_b = __float_as_int(lim);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int nb = max(max(__float_as_int(tnx[k]), __float_as_int(tny[k])), max(__float_as_int(tnz[k]), 0));
    const int fb = min(min(__float_as_int(tfx[k]), __float_as_int(tfy[k])), min(__float_as_int(tfz[k]), lim_b));
    t[k] = __int_as_float(nb <= fb ? nb : 0x7f800000);
    c[k] = cc[k];
  }
  // Order the four (t, entry) pairs just enough: three compare-exchanges put the nearest
  // first (the lane's next item), the pushes below need no order among the other three (a
  // full sort, 5 exchanges, visits 0.7 % fewer nodes but was 1.3 % slower, round 2).  The t
  // values are >= +0 or +inf: integer order on their bits (v_min/max_u32, no canonicalising
  // of float operands).  r04 A/B of the integer cull + sort against the float one (same box,
  // two boxes): headline +0.9 / +1.3 %, one rank's eighth +3.8 / +2.5 %, C3 +1.9 %, C2 -1.2 / -2.4 %.
  cswap_bits(t[0], c[0], t[1], c[1]);
  cswap_bits(t[2], c[2], t[3], c[3]);
  cswap_bits(t[0], c[0], t[2], c[2]);
  const bool v3 = __float_as_int(t[3]) != 0x7f800000, v2 = __float_as_int(t[2]) != 0x7f800000,
             v1 = __float_as_int(t[1]) != 0x7f800000;
  // push the three other children (entries 3, 2, 1; far-to-near when fully sorted).  Writes
  // at sp, sp+v3, sp+v3+v2 -- offsets counting only the children entered -- leave exactly
  // those below the new top whatever the order (a missed one lands on the next slot and is
  // overwritten or abandoned).
  if (__ballot(w >= (a.lds_entries - 2) * kStackRow) == 0ull) {  // sp + 3 <= lds_entries in every lane
    char* st = S.lds + w;
    *reinterpret_cast<int2*>(st) = make_int2(c[3], __float_as_int(t[3]));
    *reinterpret_cast<int2*>(st + (int)v3 * kStackRow) = make_int2(c[2], __float_as_int(t[2]));
    *reinterpret_cast<int2*>(st + ((int)v3 + (int)v2) * kStackRow) = make_int2(c[1], __float_as_int(t[1]));
    w += ((int)v3 + (int)v2 + (int)v1) * kStackRow;
  } else {
    if (v3) stack_push(a, S, w, gtid, c[3], t[3]);
    if (v2) stack_push(a, S, w, gtid, c[2], t[2]);
    if (v1) stack_push(a, S, w, gtid, c[1], t[1]);
  }
  if constexpr (kVisitPrio > 0) __builtin_amdgcn_s_setprio(kVisitPrio);  // until the next node's loads
  if (__float_as_int(t[0]) != 0x7f800000) return c[0];
  return stack_pop_live(a, S, w, gtid, lim);
}

// Refill kernel.  Lanes that finished their query are handed new slots (from the wave's
// current 64-slot range, then the next one) whenever fewer than `refill_min` lanes of the
// wave still hold a query, so wave instructions keep most lanes busy instead of waiting for
// the longest traversal of a fixed batch; write-back of finished queries is batched into the
// same step.  Leaves are postponed: a lane whose nearest item is a leaf waits until at least
// `leaf_min` lanes wait on one (or no lane has a node to visit), then they all test their
// leaf's primitives together -- leaf hits are sparse (~1 per 8 node visits per lane), and
// testing them at once keeps the primitive code from running with a handful of lanes.
// (RT_PHASE_TIMING builds split the waves' time into these phases: rt_diag.h.)
#ifndef RT_TRACE_WAVES
#define RT_TRACE_WAVES 6  // fused shadows over transformed shapes (C3; r05 A/B: 6 waves +4.2 % over 5
                          // once the hit record moved to settle and the planes to scalar fmas)
#endif
#ifndef RT_TRACE_WAVES_PLAIN
#define RT_TRACE_WAVES_PLAIN 6  // every other instance: 6 waves/SIMD, 80 VGPRs (r03: plain headline
#endif                          // +1.7 %, C5 +1.1 %; fused planes / soft shadows +1-2 %)
// waves per SIMD of an instance: 5 only for fused shadows over transformed shapes (C3 -1..-3 % at
// 6), 7 for the planes instances of whole frames (kSeven, chosen per call: render_tiles), else 6
#ifndef RT_TRACE_WAVES_SOFT
#define RT_TRACE_WAVES_SOFT 5  // soft-light chains over transformed shapes (C4; r05 A/B: +2.3 % over 6,
                               // whose 30 spilled VGPRs sat in the chain code)
#endif
#define RT_INSTANCE_WAVES(kPlanesOnly, kFuse, kSeven) \
  (kSeven ? 7 : (kFuse && !kPlanesOnly) ? RT_TRACE_WAVES : (kSoft && !kPlanesOnly) ? RT_TRACE_WAVES_SOFT : RT_TRACE_WAVES_PLAIN)
// the same choice on the host (LDS stack entries and blocks per CU of a launch)
static int instance_waves(bool planes, bool fuse, bool soft, bool seven) {
  return seven ? 7 : (fuse && !planes) ? RT_TRACE_WAVES : (soft && !planes) ? RT_TRACE_WAVES_SOFT : RT_TRACE_WAVES_PLAIN;
}
template <bool kCount, bool kPlanesOnly, bool kFuse, bool kSoft, bool kSeven = false, bool kFixed = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(RT_INSTANCE_WAVES(kPlanesOnly, kFuse, kSeven), 8))) void trace_refill_kernel(TraceArgs ta) {
  extern __shared__ __attribute__((aligned(16))) int lds_stack[];
  const unsigned int nq = (unsigned)ta.n_work;
  const int lane = threadIdx.x & 63;
  const uint64_t lane_lt = (1ull << lane) - 1ull;
  unsigned int nrays = 0;
  const int gtid = blockIdx.x * kBlock + threadIdx.x;
  unsigned int nbox = 0, nprim = 0, nvisit = 0;
  unsigned long long dg_any_rays = 0, dg_any_box = 0;
  unsigned int nvc = 0, nrc = 0;  // count_work: nvisit / nrays at the wave's last work fetch (measured tile costs)
  int cost_tile = -1;    // render-order tile of the wave's last fetched group
  // the loop's scalar parameters as separate SGPRs: loaded as part of a wide kernel-argument
  // load, a field spilled to a VGPR lane is restored with its whole 8-dword tuple (8
  // v_readlane per use at the loop head; r04 A/B: headline +5 %, one rank's eighth +4 %, C5 +6 %)
  TraceArgs la = ta;
  if constexpr (kFixed || kSeven) {  // constants (render_tiles checks the call's values): three
    // SGPRs fewer live across the loop, whose spills were reloaded by a v_readlane each per
    // iteration (r05 A/B, 7 waves: headline +4.6 %, C5 +5.2 %)
    la.refill_min = kRefillDefault;
    la.leaf_min = kLeafDefault;
    la.lds_entries = default_stack(RT_INSTANCE_WAVES(kPlanesOnly, kFuse, kSeven));
  } else {
    la.refill_min = sgpr_copy(ta.refill_min);
    la.leaf_min = sgpr_copy(ta.leaf_min);
    la.lds_entries = sgpr_copy(ta.lds_entries);
  }
  const TraceArgs& a = la;
  const unsigned int any = *ta.any_query;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ta.host_flag = any;  // read by the host after the step
  if (any == 0u) return;
  // the work queue: 64-slot groups, dealt to fetch_shards counters round robin (group g to
  // shard g % shards), so the queue is consumed in slot order -- the call's costliest tiles
  // first (tile_cost_order) -- and the launch ends on cheap rays
  const unsigned nfs = (unsigned)ta.fetch_shards;
  // XCD-aware deal (32 shards; RT_XCD_CHUNK groups per chunk, 0: group g to shard g % 32):
  // chunks of xc consecutive groups -- 64 by default, 4096 samples, ~41 pixels at 100 spp --
  // go to the 4 shards of one XCD in turn (blocks are dispatched to the 8 XCDs round robin, so
  // block b runs on XCD b % 8 and starts on a shard of its own XCD), so each XCD's L2 holds
  // the nodes of its own image patches instead of every XCD caching every patch
  const unsigned xc = nfs == 32u ? (unsigned)ta.xcd_chunk : 0u;
  const unsigned n_groups = (nq + 63u) >> 6;
  // wave-uniform work queue: [q_next, q_end)
  int sk = 0;
  unsigned q_next = 0, q_end = 0;
  bool exhausted = false;
  // lane state
  int slot = -1;        // query owned by this lane (traversing, or finished awaiting write-back)
  int item = kNoItem;   // node to visit / leaf to test next; kNoItem: traversal finished
  float lim = 0.0f;     // cull bound of the query (cull_limit), refreshed after each leaf test
  Query q;
  HitState h{__builtin_inff(), 0x7fffffff, -1, false};
  int sw = (int)threadIdx.x * 8;  // the lane's stack word (LaneStack): empty
  const LaneStack S{reinterpret_cast<char*>(lds_stack), reinterpret_cast<int2*>(a.spill)};
  // the first item of every traversal (wave-uniform, in an SGPR of its own: as a VGPR constant
  // it was spilled and reloaded in the leaf loop)
  const int root_item = sgpr_copy(a.root_item);
  // a query was set up in q: start its traversal at the root (BVH::intersect_linear tests
  // every primitive at once, acceleration.cpp:124-139, and leaves nothing to traverse)
  auto start_traversal = [&]() {
    h = HitState{__builtin_inff(), 0x7fffffff, -1, false};
    lim = cull_limit(a, q, h);
    sw = stack_empty_word(sw);
    item = root_item;
    if (a.c.n_prims > 0 && !a.c.use_bvh)
      test_prims<kCount, kPlanesOnly>(a, 0, a.c.n_prims, q.r, q.any, q.tmax, q.par, false, h, nprim);
  };
  // kFuse: 0 while the lane traces the slot's own query; (occlusion bits << 8) | (light + 1)
  // while it traces the shadow ray of a point light for the closest hit it just found
  int fz = 0;
  // shade's shadow ray towards point light l from the slot's hit (raytracer.cpp:214-236; the
  // logic step's ops for it, on the hit record this kernel stored)
  // (the first light's: from the hit point / normal just computed; later lights reload them)
  auto fused_shadow = [&](int l, V3 hp, V3 hn) {
    const rt_light& L = a.lights[l];
    const V3 lv = sub(V3{L.location[0], L.location[1], L.location[2]}, hp);
    const float tmax = sqrtf(dot(lv, lv));
    setup_query(q, add(hp, mul(hn, 1e-4f)), normalize(lv), tmax, true);
    ++nrays;
    if (kCount) ++dg_any_rays;
    start_traversal();
  };
  // the lane's query is complete: write it back and free the lane (kFuse: a closest hit goes
  // on to its lights' shadow rays first; their occlusion bits are written after the last)
  // kSoft: the slot's light (a sphere light) still has samples to draw after this one: add
  // this sample's visibility, draw the next target and start its traversal (shade's loop,
  // raytracer.cpp:214-236, as shadow_step_kernel does it); false when the light is done
  auto soft_next = [&](bool occluded) -> bool {
    const int N = a.n_slots;
    uint32_t* S = a.state;
    const uint32_t lw = S[F_LIGHT * N + slot];
    const int light = (int)(lw & 0xffffu), ls = (int)(lw >> 16);
    const rt_light& L = a.lights[light];
    if (!(L.radius > 0.0f && ls + 1 < a.light_samples)) return false;
    float vis = ls > 0 ? __uint_as_float(S[F_VIS * N + slot]) : 0.0f;
    if (!occluded) vis += 1.0f;
    Rng rng;
    rng.key = (uint64_t)S[F_KEY * N + slot] | ((uint64_t)S[(F_KEY + 1) * N + slot] << 32);
    rng.ctr = S[F_RNG * N + slot];
    const HitRec hr = load_hit(hit_rec(a.hit, slot));
    V3 target{L.location[0], L.location[1], L.location[2]};
    target = add(target, mul(rng.in_unit_sphere(), L.radius));
    const V3 lv = sub(target, hr.p);
    const float tmax = sqrtf(dot(lv, lv));
    S[F_LIGHT * N + slot] = (uint32_t)light | ((uint32_t)(ls + 1) << 16);
    S[F_VIS * N + slot] = __float_as_uint(vis);
    S[F_RNG * N + slot] = rng.ctr;
    setup_query(q, add(hr.p, mul(hr.n, 1e-4f)), normalize(lv), tmax, true);
    ++nrays;
    if (kCount) ++dg_any_rays;
    start_traversal();
    return true;
  };
  // kSoft + soft_start: shade's first shadow ray for the closest hit just found (the logic
  // step's transition ST_CLOSEST -> ST_SHADOW, raytracer.cpp:180-236: light 0, sample 0)
  auto soft_first = [&](V3 hp, V3 hn) {
    const int N = a.n_slots;
    uint32_t* S = a.state;
    const uint32_t depth = S[F_CTRL * N + slot] >> 4;
    const rt_light& L = a.lights[0];
    V3 target{L.location[0], L.location[1], L.location[2]};
    if (L.radius > 0.0f) {
      Rng rng;
      rng.key = (uint64_t)S[F_KEY * N + slot] | ((uint64_t)S[(F_KEY + 1) * N + slot] << 32);
      rng.ctr = S[F_RNG * N + slot];
      target = add(target, mul(rng.in_unit_sphere(), L.radius));
      S[F_RNG * N + slot] = rng.ctr;
    }
    const V3 lv = sub(target, hp);
    const float tmax = sqrtf(dot(lv, lv));
    S[F_CTRL * N + slot] = (uint32_t)ST_SHADOW | (depth << 4);
    S[F_LIGHT * N + slot] = 0u;
    if (a.frames) {  // the traced ray, read back by the shading (view vector) and reflection
      S[(F_RAY + 0) * N + slot] = __float_as_uint(q.r.o.x);
      S[(F_RAY + 1) * N + slot] = __float_as_uint(q.r.o.y);
      S[(F_RAY + 2) * N + slot] = __float_as_uint(q.r.o.z);
      S[(F_RAY + 3) * N + slot] = __float_as_uint(q.r.d.x);
      S[(F_RAY + 4) * N + slot] = __float_as_uint(q.r.d.y);
      S[(F_RAY + 5) * N + slot] = __float_as_uint(q.r.d.z);
      S[(F_RAY + 6) * N + slot] = __float_as_uint(q.r.time);
    } else if (!a.pinhole) {
      S[(F_RAY + 0) * N + slot] = __float_as_uint(q.r.o.x);
      S[(F_RAY + 1) * N + slot] = __float_as_uint(q.r.o.y);
      S[(F_RAY + 2) * N + slot] = __float_as_uint(q.r.o.z);
    }
    setup_query(q, add(hp, mul(hn, 1e-4f)), normalize(lv), tmax, true);
    ++nrays;
    if (kCount) ++dg_any_rays;
    start_traversal();
  };
  auto settle = [&]() {
    int next = -1;  // kFuse: the light whose shadow ray the lane traces next
    V3 hp{0.0f, 0.0f, 0.0f}, hn{0.0f, 0.0f, 0.0f};
    bool have = false;  // hp / hn: the hit record just written (else the next shadow ray reloads it)
    if (kSoft && q.any) {
      complete_query<kCount, kPlanesOnly>(a, slot, q, h, nprim);
      if (soft_next(h.done)) return;
      a.result[slot] = h.done ? 1 : 0;
    } else if (kFuse && fz != 0) {
      complete_query<kCount, kPlanesOnly>(a, slot, q, h, nprim);
      const int l = (fz & 0xff) - 1;
      const unsigned bits = ((unsigned)fz >> 8) | (h.done ? 1u << l : 0u);
      if (l + 1 < a.n_fuse) {
        fz = (int)(bits << 8) | (l + 2);
        next = l + 1;
      } else {
        a.occl[slot] = bits;
        RT_WD(3);
        fz = 0;
      }
    } else {
      have = finish_query<kCount, kPlanesOnly>(a, slot, q, h, nprim, hp, hn);
      if ((kFuse || (kSoft && a.soft_start)) && !q.any && h.best_idx >= 0) {
        if (!kPlanesOnly) {  // transformed shapes: the hit record the logic step would compute
          const float4* rec = a.c.prims + (size_t)h.best_idx * a.c.prim_stride4;
          PrimA P;
          load_prim_a(rec, P);
          HitAttr at;
          float t;
          prim_hit<true, false, false>(P, rec, q.r, t, &at);
          if (a.has_tex != kHitRecompute) store_hit_pnm(hit_rec(a.hit, slot), at.p, at.n, RT_TAG_MATERIAL(prim_tag(P)));
          hp = at.p;
          hn = at.n;
          have = true;
        }
        if (kSoft) {
          soft_first(hp, hn);
          return;
        }
        if (a.n_fuse > 0) {  // (a one-pass call without lights launches this instance for the record alone)
          fz = 1;
          next = 0;
        }
      }
    }
    if (kFuse && next >= 0) {
      if (!have) {
        const HitRec hr = load_hit(hit_rec(a.hit, slot));
        hp = hr.p;
        hn = hr.n;
      }
      fused_shadow(next, hp, hn);
    } else {
      slot = -1;
    }
  };
  RT_PT_DECL
  RT_ET_BEGIN
  for (;;) {
    RT_PT_MARK(3);  // loop control (ballots) since the node phase
    uint64_t act = __ballot(item != kNoItem);
    if (popc_s(act) < a.refill_min) {
      if (slot >= 0 && item == kNoItem) settle();
      while (!exhausted) {
        const uint64_t freem = __ballot(slot < 0);
        if (freem == 0ull) break;
        if (q_next >= q_end) {  // next 64 slots: this shard's counter, then the other shards'
          for (;;) {
            int sh;
            // 7-wave instances: the deal's derived values recomputed here, in the cold fetch path,
            // from opaque copies -- hoisted to the kernel's entry they stayed live across the
            // whole loop (SGPRs spilled 111 -> 101; r05 A/B, 3 reps: headline +0.5 %, C5 +0.6 %;
            // in the 6-wave instances one rank's eighth lost 0.8 %, so they keep the hoisting)
            unsigned xcv = xc, bid = blockIdx.x;
            if constexpr (kSeven) {
              asm volatile("s_mov_b32 %0, %1" : "=s"(xcv) : "s"(xc));
              asm volatile("s_mov_b32 %0, %1" : "=s"(bid) : "s"((unsigned)blockIdx.x));
            }
            if (xcv > 0u) {  // this block's XCD's shards first, then the other XCDs'
              const unsigned xo = (unsigned)sk / 4u, po = (unsigned)sk % 4u;
              sh = (int)(((bid % 8u + xo) % 8u) + 8u * ((bid / 8u + po) % 4u));
            } else {
              sh = (int)((blockIdx.x + sk) % nfs);
            }
            unsigned j = 0;
            if (xc > 0u || (unsigned)sh < n_groups) {
              if (lane == 0) j = atomicAdd(ta.fetch + sh * kFetchStride, 1u);
              j = __shfl(j, 0);
            }
            unsigned g;
            if (xcv > 0u) {  // shard sh = XCD x + 8 p: the chunks k of XCD x (chunk % 8 == x), offsets == p (mod 4)
              const unsigned per = xcv / 4u, k = j / per;
              g = ((k * 8u + (unsigned)sh % 8u) * xcv) + (unsigned)sh / 8u + (j % per) * 4u;
            } else {
              g = (unsigned)sh + j * nfs;
            }
            if ((xc > 0u || (unsigned)sh < n_groups) && g < n_groups) {
              q_next = (unsigned)ta.slot_base + g * 64u;
              q_end = (unsigned)ta.slot_base + min(g * 64u + 64u, nq);
              // 64-slot groups are slot-waves of the logic step: skip one whose slots retired
              if (!a.one_pass && a.wave_done[q_next >> 6] != 0u) continue;
              if (kCount && a.tile_cost) {  // the wave's node visits since its last fetch go to that group's tile
                flush_tile_cost(a, lane, cost_tile, nvisit, nvc, nrays, nrc);
                cost_tile = (int)fdiv(q_next, a.fd_tile_units);
              }
              break;
            }
            if (++sk >= (int)nfs) {
              exhausted = true;
              RT_ET_EXHAUSTED;
              break;
            }
          }
          if (exhausted) break;
        }
        const unsigned rank = (unsigned)__popcll(freem & lane_lt);
        const unsigned avail = q_end - q_next;
        if (slot < 0 && rank < avail) {
          const int s = (int)(q_next + rank);
          if (begin_query(a, s, q)) {
            slot = s;
            ++nrays;
            if (kCount && q.any) ++dg_any_rays;
            start_traversal();  // nothing to traverse (linear mode): settled in the next refill phase
          }
        }
        q_next += min(avail, (unsigned)__popcll(freem));
      }
      act = __ballot(item != kNoItem);
      RT_PT_MARK(0);  // refill: write-back, work fetch, query setup
      // done when the queue is drained and every lane settled (a query with nothing to
      // traverse -- linear mode, empty scene -- is settled in the next refill phase)
      // (drain_help: the queries still traversing go on in the drain loop below)
      if (exhausted && (a.drain_help || __ballot(slot >= 0) == 0ull)) break;
    }
    // leaf phase: enough lanes wait on a leaf, or nothing else is left to do
    const uint64_t leafm = __ballot(is_leaf_item(item));
    if (leafm != 0ull && (popc_s(leafm) >= a.leaf_min || (act & ~leafm) == 0ull)) {
      RT_PT_LEAF_LANES;
      if (is_leaf_item(item)) {
        const uint32_t e = (uint32_t)item;
        test_prims<kCount, kPlanesOnly>(a, (int)((e & ~kLeafBit) >> 7), (int)(e & 0x7fu), q.r, q.any, q.tmax, q.par, true,
                                        h, nprim);
        lim = cull_limit(a, q, h);
        item = h.done ? kNoItem : stack_pop_live(a, S, sw, gtid, lim);
      }
      RT_PT_MARK(1);  // leaf phase
    }
    // node phase
    RT_PT_NODE_BEGIN
    if (item >= 0) item = node_visit<kCount, kPlanesOnly>(a, q, lim, item, S, sw, gtid, nbox, dg_any_box, nvisit);
    RT_PT_NODE_END
  }
  // ---- drain (drain_help: the queue is dry).  A query still traversing keeps its lane (its
  // owner); a free lane becomes a helper: it takes the bottom entry of a busy lane's stack --
  // pushed first, the farthest subtree pending there -- and searches it with the owner's ray
  // under the owner's bound, re-read every iteration.  A finished helper's best hit is folded
  // into its owner's (lower t, then lower reference index: the minimum the serial traversal
  // finds in any visiting order; any-hit: occluded), and an owner settles only once no helper
  // searches for it, so every result is the serial traversal's.  A soup ray that crosses the
  // scene without a hit visits hundreds of nodes; without help it alone holds its wave (and
  // the launch) long after the queue ran dry.
  if (a.drain_help) {
    int own = -1;  // helper: lane of the owner whose query it searches
    int nh = 0;    // owner: helpers searching for its query
    for (;;) {
      // fold finished helpers into their owners
      uint64_t fin = __ballot(own >= 0 && item == kNoItem);
      while (fin != 0ull) {
        const int hl = __ffsll((long long)fin) - 1;
        fin &= fin - 1ull;
        const int o = __builtin_amdgcn_readlane(own, hl);
        const float bt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h.best_t), hl));
        const int br = __builtin_amdgcn_readlane(h.best_ref, hl);
        const int bi = __builtin_amdgcn_readlane(h.best_idx, hl);
        const int bd = __builtin_amdgcn_readlane((int)h.done, hl);
        if (lane == o) {
          --nh;
          if (q.any) {
            if (bd) {
              h.done = true;
              item = kNoItem;
            }
          } else if (bi >= 0 && (bt < h.best_t || (bt == h.best_t && br < h.best_ref))) {
            h.best_t = bt;
            h.best_ref = br;
            h.best_idx = bi;
            lim = cull_limit(a, q, h);
          }
        }
      }
      if (own >= 0 && item == kNoItem) {
        own = -1;
        sw = stack_empty_word(sw);
      }
      // an owner whose traversal and helpers are done settles (and may start its next query)
      if (slot >= 0 && item == kNoItem && nh == 0) settle();
      if (__ballot(slot >= 0) == 0ull) break;
      // pair free lanes with lanes that have stack entries (k-th free lane, k-th donor)
      const bool can_give = item != kNoItem && sw >= kStackRow;
      const uint64_t D = __ballot(can_give), I = __ballot(slot < 0 && own < 0);
      if (D != 0ull && I != 0ull) {
        const int k = min(__popcll(D), __popcll(I));
        const int rootv = own >= 0 ? own : lane;
        int src = -1;
        uint64_t d = D, fr = I;
        for (int j = 0; j < k; ++j) {
          const int dl = __ffsll((long long)d) - 1, il = __ffsll((long long)fr) - 1;
          d &= d - 1ull;
          fr &= fr - 1ull;
          if (lane == il) src = dl;
          if (lane == __builtin_amdgcn_readlane(rootv, dl)) ++nh;
        }
        int2 ent = make_int2(kNoItem, 0);
        if (can_give && __popcll(D & lane_lt) < k) ent = stack_take_bottom(a, S, sw, gtid);
        const int s2 = src >= 0 ? src : lane;
        const int ge = __shfl(ent.x, s2), gt = __shfl(ent.y, s2), rs = __shfl(rootv, s2);
        const int qs = src >= 0 ? rs : lane;  // receivers copy their owner's query
        q.r.o.x = __shfl(q.r.o.x, qs);
        q.r.o.y = __shfl(q.r.o.y, qs);
        q.r.o.z = __shfl(q.r.o.z, qs);
        q.r.d.x = __shfl(q.r.d.x, qs);
        q.r.d.y = __shfl(q.r.d.y, qs);
        q.r.d.z = __shfl(q.r.d.z, qs);
        q.r.time = __shfl(q.r.time, qs);
        q.inv.x = __shfl(q.inv.x, qs);
        q.inv.y = __shfl(q.inv.y, qs);
        q.inv.z = __shfl(q.inv.z, qs);
        q.tmax = __shfl(q.tmax, qs);
        q.any = __shfl((int)q.any, qs) != 0;
        q.par = (uint32_t)__shfl((int)q.par, qs);
        q.sel[0] = (uint32_t)__shfl((int)q.sel[0], qs);
        q.sel[1] = (uint32_t)__shfl((int)q.sel[1], qs);
        q.sel[2] = (uint32_t)__shfl((int)q.sel[2], qs);
        const float rl = __shfl(lim, qs);
        if (src >= 0) {
          own = rs;
          h = HitState{__builtin_inff(), 0x7fffffff, -1, false};
          lim = rl;
          sw = stack_empty_word(sw);
          item = __int_as_float(gt) > rl ? kNoItem : ge;
        }
      }
      // helpers take their owner's bound (closest: its best so far; any-hit: occluded ends it)
      if (__ballot(own >= 0) != 0ull) {
        const int os = own >= 0 ? own : lane;
        const float ol = __shfl(lim, os);
        const int od = __shfl((int)h.done, os);
        if (own >= 0) {
          if (od) item = kNoItem;
          else if (ol < lim) lim = ol;
        }
      }
      const uint64_t act = __ballot(item != kNoItem);
      const uint64_t leafm = __ballot(is_leaf_item(item));
      if (leafm != 0ull && (popc_s(leafm) >= a.leaf_min || (act & ~leafm) == 0ull)) {
        if (is_leaf_item(item)) {
          const uint32_t e = (uint32_t)item;
          test_prims<kCount, kPlanesOnly>(a, (int)((e & ~kLeafBit) >> 7), (int)(e & 0x7fu), q.r, q.any, q.tmax, q.par,
                                          true, h, nprim);
          lim = cull_limit(a, q, h);
          item = h.done ? kNoItem : stack_pop_live(a, S, sw, gtid, lim);
        }
      }
      if (item >= 0) item = node_visit<kCount, kPlanesOnly>(a, q, lim, item, S, sw, gtid, nbox, dg_any_box, nvisit);
    }
  }
  RT_PT_FLUSH
  RT_ET_END
  if (kCount && a.tile_cost) flush_tile_cost(a, lane, cost_tile, nvisit, nvc, nrays, nrc);
  trace_counters_out<kCount>(ta, lane, nrays, nbox, nprim, dg_any_rays, dg_any_box, nvisit);
}

// ---------------------------------------------------------------- shading helpers
// Material::getDiffuseColor (material.hpp:99-134)
__device__ __forceinline__ V3 diffuse_color(const LogicArgs& a, const rt_material& m, float u, float v) {
  V3 dc{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
  if (m.texture < 0) return dc;
  rt_texture tx = a.textures[m.texture];
  int x = (int)(u * (float)(tx.width - 1));
  int y = (int)((1.0f - v) * (float)(tx.height - 1));
  int cr = 0, cg = 0, cb = 0;
  if (!(x < 0 || x >= tx.width || y < 0 || y >= tx.height)) {
    const uint8_t* p = a.texels + tx.offset + ((size_t)y * tx.width + x) * 3;
    cr = p[0]; cg = p[1]; cb = p[2];
  }
  V3 t{(((float)cr) / (255.0f)), (((float)cg) / (255.0f)), (((float)cb) / (255.0f))};
  return V3{t.x * dc.x, t.y * dc.y, t.z * dc.z};
}

// kFrames: some material reflects or refracts (Trace recursion frames needed)
// kTex: some material has a texture (hit UVs + texel fetch)
// kPlanes: every primitive is a Plane (no transformed-shape intersection code)
// Waves per SIMD the register allocation must allow (__launch_bounds__' second argument:
// blocks of 4 waves per CU = waves per SIMD).  The logic step is bound by the latency of its
// scattered state loads, so occupancy pays: without frames 4 waves (<= 128 VGPRs; the
// unconstrained allocation took 132 = 3 waves, 10 % slower frame); with recursion frames
// the state machine needs ~195 (2 waves).  A/B builds: make variant VDEFS=-DRT_LOGIC_WAVES=6
// r05, two slot pipelines: 5 waves for the reflection-frames instance (95-96 VGPRs, 4-6
// spilled; the frameless instances fit 5 at 87-89 either way) -- C4 +2.0 % (same box, 2 reps:
// 14296-14303 -> 14561-14597 Mrays/s; 6 waves spill 34-41)
#ifndef RT_LOGIC_WAVES
#define RT_LOGIC_WAVES 5
#endif
#ifndef RT_LOGIC_WAVES_F
#define RT_LOGIC_WAVES_F 2
#endif
// kRefr: the scene has refraction (pending refraction rays in the frames); the reflection-only
// instance of the frames variant drops that code and fits 4 waves/SIMD (121 VGPRs, 161 with it)
// kInline: a few-primitive scene (at most RT_FLAT_PRIMS bounded primitives: every traversal is
// one leaf item of all of them) -- the step answers every query itself, the camera query
// start_kernel emitted and every one it emits, against that leaf item and the unbounded
// primitives with the trace kernel's functions (test_prims, complete_query, the hit record of
// finish_query / the ST_CLOSEST entry below), and goes on with the sample: a slot's sample runs
// to its end in one step and the call launches no traversal at all.  The answers are the trace
// kernel's (same functions, same operands), the shadow rays the unfused ones (the RT_FUSE=0 /
// RT_SOFT_FUSE=0 / RT_SOFT_START=0 order of draws: the knob tests pin them equal), so the same bits.
#ifndef RT_LOGIC_WAVES_I
#define RT_LOGIC_WAVES_I 5
#endif
template <bool kFrames, bool kRefr, bool kTex, bool kPlanes, bool kInline = false>
__global__ __launch_bounds__(kBlock, kRefr ? RT_LOGIC_WAVES_F : kInline ? RT_LOGIC_WAVES_I : RT_LOGIC_WAVES) void logic_kernel(LogicArgs a) {
  const int slot = a.slot_base + (int)(blockIdx.x * kBlock + threadIdx.x);
  // a wave whose slots all retired has nothing left in this frame (one scalar load)
  if (a.wave_done[__builtin_amdgcn_readfirstlane(slot >> 6)] != 0u) return;
  // no batch left for this wave's shard: a wave whose slots all finish now retires at the end
  // of this step (below), so its finished slots need no idle marks
  const int wave = slot >> 6, shard = wave % a.batch_shards;
  const unsigned claimed = __hip_atomic_load(a.batch_ctr + shard * kCtrStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool no_batch = ((long long)claimed * a.batch_shards + shard) * 64 >= a.n_units;
  bool want = false;
  unsigned int n_inline = 0;  // kInline: queries answered by this step
  if (slot < a.slot_end) {
    const int N = a.n_slots;
    uint32_t* S = a.state;
    auto ld = [&](int f) { return S[f * N + slot]; };
    auto ldf = [&](int f) { return __uint_as_float(S[f * N + slot]); };
    auto stu = [&](int f, uint32_t v) { S[f * N + slot] = v; };
    auto stf = [&](int f, float v) { S[f * N + slot] = __float_as_uint(v); };

    // One round of independent loads: the control words, the trace result and the RNG
    // stream position are read for every slot whatever its state (a retired or idle slot
    // discards them), so no load waits on another's value before the state-specific round.
    long long unit = (long long)(int)ld(F_UNIT);  // >= 0 active, -2 idle (batch done), -1 retired
    const uint32_t ctrl0 = ld(F_CTRL);
    const int res_ld = kInline ? -1 : a.result[slot];  // kInline: no traversal launch answered anything
    uint32_t key_lo = 0, key_hi = 0, rng_ctr = 0;
    if (a.late_draws) {
      key_lo = ld(F_KEY);
      key_hi = ld(F_KEY + 1);
      rng_ctr = ld(F_RNG);
    }
    if (unit != -1) {
      const int s = a.spp_sqrt;
      uint32_t ctrl = ctrl0;
      int st = (int)(ctrl & 15u), depth = (int)(ctrl >> 4);
      // Only what the entry state reads is loaded: a closest-hit result needs the ray that
      // was traced (still in the query record) and the hit record (loaded before the result
      // is known: a miss ignores it); a shadow result needs the hit and the shade
      // accumulators; a new sample needs nothing.
      const int st0 = unit >= 0 ? st : -1;
      // A shadow result whose light still had soft-shadow samples to draw was advanced by
      // shadow_step_kernel earlier in this step (it marks the consumed result -2): such a
      // slot is left untouched here and only counts as a slot with a query.
      const bool fast = st0 == ST_SHADOW && res_ld == kResAdvanced;
      int light = 0, ls = 0, mat_id = 0;
      Ray ray;
      ray.o = V3{0.0f, 0.0f, 0.0f};
      ray.d = V3{0.0f, 0.0f, 0.0f};
      ray.time = 0.0f;
      V3 hp{0.0f, 0.0f, 0.0f}, hn{0.0f, 0.0f, 0.0f}, fin{0.0f, 0.0f, 0.0f};
      float vis = 0.0f, hu = 0.0f, hv = 0.0f;
      const V3 cam_o{a.cam.location[0], a.cam.location[1], a.cam.location[2]};
      if (fast) {
        want = true;
      } else if (!kInline && !kPlanes && st0 == ST_CLOSEST && res_ld >= 0 && a.n_fuse == 0) {
        // the hit being shaded (raytracer.cpp:293-303): the hit primitive's test with
        // attributes on the ray just traced (the query record), kept in the slot's hit record
        // for the shadow steps that follow
        const QueryRec qr = load_query(a.query, N, slot, a.cam.location);
        const Ray tr{qr.o, qr.d, qr.tq};
        const float4* rec = a.c.prims + (size_t)res_ld * a.c.prim_stride4;
        PrimA P;
        load_prim_a(rec, P);
        HitAttr at;
        float t;
        prim_hit<true, false, kTex>(P, rec, tr, t, &at);
        hp = at.p;
        hn = at.n;
        hu = at.u;
        hv = at.v;
        mat_id = (int)RT_TAG_MATERIAL(prim_tag(P));
        store_hit_pnm(hit_rec(a.hit, slot), hp, hn, (uint32_t)mat_id);
        if (kTex) a.hit_uv[slot] = make_float2(hu, hv);
      } else if (!kInline && (st0 == ST_SHADOW || (st0 == ST_CLOSEST && res_ld >= 0))) {
        // the hit being shaded: its record (written by the trace kernel for planes-only scenes,
        // by the ST_CLOSEST step above otherwise); a closest miss does not read it
        const HitRec hr = load_hit(hit_rec(a.hit, slot));
        hp = hr.p;
        hn = hr.n;
        if (kTex) {
          const float2 uv = a.hit_uv[slot];
          hu = uv.x;
          hv = uv.y;
        }
        mat_id = (int)hr.mat;
      }
      if (st0 == ST_SHADOW && !fast) {
        const uint32_t lw = ld(F_LIGHT);
        light = (int)(lw & 0xffffu);
        ls = (int)(lw >> 16);
        if (kFrames) {
          ray.o = V3{ldf(F_RAY), ldf(F_RAY + 1), ldf(F_RAY + 2)};
          ray.d = V3{ldf(F_RAY + 3), ldf(F_RAY + 4), ldf(F_RAY + 5)};
          ray.time = ldf(F_RAY + 6);
        } else {  // shading reads only the origin
          ray.o = a.pinhole ? cam_o : V3{ldf(F_RAY), ldf(F_RAY + 1), ldf(F_RAY + 2)};
        }
        if (ls > 0) vis = ldf(F_VIS);
        if (light > 0) fin = V3{ldf(F_FIN), ldf(F_FIN + 1), ldf(F_FIN + 2)};
      } else if (!kInline && st0 == ST_CLOSEST) {
        if (kFrames) {
          const QueryRec qr = load_query(a.query, N, slot, a.cam.location);
          ray.o = qr.o;
          ray.d = qr.d;
          ray.time = qr.tq;  // closest queries carry the ray time there
        } else if (!a.pinhole) {
          ray.o = load_query(a.query, N, slot, a.cam.location).o;
        } else {
          ray.o = cam_o;
        }
      }
      int res = st0 >= ST_CLOSEST ? res_ld : -1;
      // later steps of a sample continue its RNG stream from the stored key and counter
      Rng rng;
      rng.key = 0;
      rng.ctr = 0;
      if (st0 >= ST_CLOSEST) {
        rng.key = (uint64_t)key_lo | ((uint64_t)key_hi << 32);
        rng.ctr = rng_ctr;
      }
      bool idle = st0 < 0;  // idle (batch done, pixel outside the image): start_kernel's work
      // a closest hit whose point-light shadow rays the trace kernel traced along (kFuse)
      bool fused = !kInline && a.n_fuse > 0 && st0 == ST_CLOSEST && res >= 0;
      const unsigned occl_bits = fused ? a.occl[slot] : 0u;
      V3 qo{0, 0, 0}, qd{0, 0, 0};
      float qtmax = 0.0f;
      int qkind = 0;
      if (kInline && st0 == ST_CLOSEST) {  // the camera query start_kernel emitted: answered below
        const QueryRec qr = load_query(a.query, N, slot, a.cam.location);
        qo = qr.o;
        qd = qr.d;
        qtmax = qr.tq;
        want = true;
      }

      for (;;) {
      while (!want && !idle) {
        V3 ret{0, 0, 0};
        bool returning = false;
        bool shade_now = false;
        if (st == ST_CLOSEST) {  // Trace body after get_intersection (raytracer.cpp:293-303)
          if (res < 0) {
            ret = V3{0.1f, 0.1f, 0.1f};
            returning = true;
          } else {
            const rt_material& m = a.mats[mat_id];
            V3 base = kTex ? diffuse_color(a, m, hu, hv) : V3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
            fin = V3{base.x * m.k_ambient, base.y * m.k_ambient, base.z * m.k_ambient};
            light = 0;
            ls = 0;
            vis = 0.0f;
            shade_now = true;
          }
        } else if (st == ST_SHADOW) {
          if (res == 0) vis += 1.0f;
          ++ls;
          if (light == 0) {  // final_color before any light: the ambient term (same ops as above)
            const rt_material& m = a.mats[mat_id];
            V3 base = kTex ? diffuse_color(a, m, hu, hv) : V3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
            fin = V3{base.x * m.k_ambient, base.y * m.k_ambient, base.z * m.k_ambient};
          }
          shade_now = true;
        }
        if (shade_now) {  // shade (raytracer.cpp:180-274)
          const rt_material& m = a.mats[mat_id];
          while (light < a.n_lights) {
            const rt_light& L = a.lights[light];
            const int ns = (L.radius > 0.0f) ? a.light_samples : 1;
            if (ls < ns) {
              if (fused) {  // the trace kernel traced this shadow ray with the hit (result in occl bits)
                if (!((occl_bits >> light) & 1u)) vis += 1.0f;
                ++ls;
                continue;
              }
              V3 target{L.location[0], L.location[1], L.location[2]};
              if (L.radius > 0.0f) target = add(target, mul(rng.in_unit_sphere(), L.radius));
              V3 lv = sub(target, hp);
              qtmax = sqrtf(dot(lv, lv));
              qd = normalize(lv);
              qo = add(hp, mul(hn, 1e-4f));
              qkind = 1;
              st = ST_SHADOW;
              want = true;
              break;
            }
            vis = vis / (float)ns;
            if (!(vis <= 0.0f)) {
              V3 base = kTex ? diffuse_color(a, m, hu, hv) : V3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
              V3 lc = sub(V3{L.location[0], L.location[1], L.location[2]}, hp);
              float dsq = dot(lc, lc);
              float ldist = sqrtf(dsq);
              V3 Ld = normalize(lc);
              float ndl = smax(0.0f, dot(hn, Ld));
              V3 diff = mul(base, ndl);
              // a material without a specular colour adds 0 * si == +0 for every finite si >= 0
              // (ndh in [0, 1 + eps], shininess <= 5e6): the same bits without the powf -- and
              // without the view and half vectors, which feed nothing else (r06: their two
              // normalisations, six divisions, are skipped too)
              float si = 0.0f;
              if (!spec_zero(m)) {
                V3 V = normalize(sub(ray.o, hp));
                V3 H = normalize(add(Ld, V));
                float ndh = smax(0.0f, dot(hn, H));
                si = rt_powf(ndh, m.shininess);
              }
              V3 spec{m.specular[0] * si, m.specular[1] * si, m.specular[2] * si};
              float att = (10.0f * L.intensity) / (25.0f + 10.0f * ldist + 150.0f * dsq);
              V3 inner{diff.x * m.k_diffuse + spec.x * m.k_specular, diff.y * m.k_diffuse + spec.y * m.k_specular,
                       diff.z * m.k_diffuse + spec.z * m.k_specular};
              V3 contrib{L.color[0] * inner.x * att, L.color[1] * inner.y * att, L.color[2] * inner.z * att};
              fin = V3{fin.x + contrib.x * vis, fin.y + contrib.y * vis, fin.z + contrib.z * vis};
            }
            ++light;
            ls = 0;
            vis = 0.0f;
          }
          if (want) break;
          // Trace continues with reflection / refraction (raytracer.cpp:303-350)
          const float lcf = smax(0.0f, 1.0f - m.reflectivity - m.transparency);
          const V3 A{lcf * fin.x, lcf * fin.y, lcf * fin.z};
          bool refl_ok = false, refr_ok = false;
          Ray rr, tr;
          rr.time = 0.0f;
          tr.time = 0.0f;
          if (kFrames && m.reflectivity > 0.0f) {  // createReflectionRay (raytracer.cpp:101-115) + glossy fuzz
            float idn = dot(ray.d, hn);
            rr.d = sub(ray.d, mul(hn, 2.0f * idn));
            rr.o = add(hp, mul(hn, 1e-4f));
            if (m.roughness > 0.0f) {
              V3 fuzz = rng.in_unit_sphere();
              rr.d = normalize(add(rr.d, mul(fuzz, m.roughness)));
              if (dot(rr.d, hn) < 0.0f) rr.d = V3{0.0f, 0.0f, 0.0f};
            }
            refl_ok = dot(rr.d, rr.d) > 0.001f;
          }
          if (kRefr && m.transparency > 0.0f) {  // createRefractionRay (raytracer.cpp:118-150)
            V3 N = hn;
            float n_in = 1.0f, n_out = m.refractive_index;
            float cos_i = dot(ray.d, N);
            if (cos_i > 0) {
              float tmp = n_in;
              n_in = n_out;
              n_out = tmp;
              N = mul(N, -1.0f);
            }
            float eta = n_in / n_out;
            float ca = fabsf(cos_i);
            float disc = 1.0f - eta * eta * (1.0f - ca * ca);
            if (disc < 0) {
              tr.o = V3{0, 0, 0};
              tr.d = V3{0, 0, 0};
            } else {
              float cos_t = sqrtf(disc);
              V3 T = add(mul(ray.d, eta), mul(N, (eta * ca - cos_t)));
              tr.o = add(hp, mul(N, -1e-4f));
              tr.d = normalize(T);
            }
            refr_ok = dot(tr.d, tr.d) > 1e-6f;
          }
          // a child that is not traced (invalid ray, or depth+1 > MAX) contributes (0,0,0)
          const bool refl_go = refl_ok && depth + 1 <= kMaxDepth;
          const bool refr_go = refr_ok && depth + 1 <= kMaxDepth;
          if (!kFrames || (!refl_go && !refr_go)) {
            V3 part{A.x + m.reflectivity * 0.0f, A.y + m.reflectivity * 0.0f, A.z + m.reflectivity * 0.0f};
            ret = V3{part.x + m.transparency * 0.0f, part.y + m.transparency * 0.0f, part.z + m.transparency * 0.0f};
            returning = true;
          } else {
            uint32_t* F = a.frames + (size_t)depth * FR_COUNT * N;
            uint32_t meta = (uint32_t)mat_id << 2;
            if (refl_go) {
              F[(FR_A + 0) * N + slot] = __float_as_uint(A.x);
              F[(FR_A + 1) * N + slot] = __float_as_uint(A.y);
              F[(FR_A + 2) * N + slot] = __float_as_uint(A.z);
              if (refr_go) {
                meta |= 2;
                float* R = a.refr + (size_t)depth * 6 * N;
                R[0 * N + slot] = tr.o.x; R[1 * N + slot] = tr.o.y; R[2 * N + slot] = tr.o.z;
                R[3 * N + slot] = tr.d.x; R[4 * N + slot] = tr.d.y; R[5 * N + slot] = tr.d.z;
              }
              ray = rr;
            } else {  // reflection not traced: A + r*0, then straight into the refraction child
              F[(FR_A + 0) * N + slot] = __float_as_uint(A.x + m.reflectivity * 0.0f);
              F[(FR_A + 1) * N + slot] = __float_as_uint(A.y + m.reflectivity * 0.0f);
              F[(FR_A + 2) * N + slot] = __float_as_uint(A.z + m.reflectivity * 0.0f);
              meta |= 1;
              ray = tr;
            }
            F[FR_META * N + slot] = meta;
            ++depth;
            st = ST_CLOSEST;
            qo = ray.o;
            qd = ray.d;
            qtmax = 0.0f;  // secondary rays have time 0 (createReflectionRay returns {o, d})
            qkind = 0;
            want = true;
            break;
          }
        }
        // unwind finished Traces
        while (returning) {
          if (depth == 0) {  // the sample's Trace returned: store it, pull the next unit
            a.samples[unit * 3 + 0] = ret.x;
            a.samples[unit * 3 + 1] = ret.y;
            a.samples[unit * 3 + 2] = ret.z;
            idle = true;  // wait for the rest of the wave's batch
            unit = -2;
            break;
          }
          if (!kFrames) break;  // unreachable: without frames every Trace returns at depth 0
          --depth;
          const uint32_t* F = a.frames + (size_t)depth * FR_COUNT * N;
          uint32_t meta = F[FR_META * N + slot];
          const rt_material& pm = a.mats[meta >> 2];
          V3 A{__uint_as_float(F[(FR_A + 0) * N + slot]), __uint_as_float(F[(FR_A + 1) * N + slot]),
               __uint_as_float(F[(FR_A + 2) * N + slot])};
          if (!(meta & 1)) {  // the reflection child returned R
            V3 p{A.x + pm.reflectivity * ret.x, A.y + pm.reflectivity * ret.y, A.z + pm.reflectivity * ret.z};
            if (kRefr && (meta & 2)) {  // refraction pending: trace it as the next child
              uint32_t* Fw = a.frames + (size_t)depth * FR_COUNT * N;
              Fw[(FR_A + 0) * N + slot] = __float_as_uint(p.x);
              Fw[(FR_A + 1) * N + slot] = __float_as_uint(p.y);
              Fw[(FR_A + 2) * N + slot] = __float_as_uint(p.z);
              Fw[FR_META * N + slot] = meta | 1;
              const float* R = a.refr + (size_t)depth * 6 * N;
              ray.o = V3{R[0 * N + slot], R[1 * N + slot], R[2 * N + slot]};
              ray.d = V3{R[3 * N + slot], R[4 * N + slot], R[5 * N + slot]};
              ray.time = 0.0f;
              ++depth;
              st = ST_CLOSEST;
              qo = ray.o;
              qd = ray.d;
              qtmax = 0.0f;
              qkind = 0;
              want = true;
              break;
            }
            ret = V3{p.x + pm.transparency * 0.0f, p.y + pm.transparency * 0.0f, p.z + pm.transparency * 0.0f};
          } else {  // the refraction child returned T
            ret = V3{A.x + pm.transparency * ret.x, A.y + pm.transparency * ret.y, A.z + pm.transparency * ret.z};
          }
        }
      }
      if (!kInline || !want) break;
      if constexpr (kInline) {  // answer the query just emitted and go on with the sample
        TraceArgs tv{};  // what test_prims / complete_query read
        tv.c = a.c;
        tv.prim_refs = a.prim_refs;
        tv.ref_boxes = a.ref_boxes;
        tv.n_unbounded = a.n_unbounded;
        Query q;
        setup_query(q, qo, qd, qtmax, qkind == 1);
        ++n_inline;
        HitState h{__builtin_inff(), 0x7fffffff, -1, false};
        unsigned int np = 0;
        if (a.flat_n > 0) test_prims<false, kPlanes>(tv, 0, a.flat_n, q.r, q.any, q.tmax, q.par, true, h, np);
        complete_query<false, kPlanes>(tv, slot, q, h, np);
        want = false;
        if (qkind == 1) {  // shadow: occluded (st is ST_SHADOW)
          res = h.done ? 1 : 0;
        } else {  // closest (st is ST_CLOSEST): the hit record the entry above would read
          res = h.best_idx;
          fused = false;  // its shadow rays are this step's own queries
          ray = q.r;      // closest queries carry the ray time in qtmax (0 for secondary rays)
          if (res >= 0) {
            const float4* rec = a.c.prims + (size_t)res * a.c.prim_stride4;
            if constexpr (kPlanes && !kTex) {  // finish_query: o + t d, the plane's normal and tag
              const float* w = reinterpret_cast<const float*>(rec);
              hp = V3{q.r.o.x + h.best_t * q.r.d.x, q.r.o.y + h.best_t * q.r.d.y, q.r.o.z + h.best_t * q.r.d.z};
              hn = V3{w[3], w[7], w[11]};
              mat_id = (int)RT_TAG_MATERIAL(__float_as_uint(w[15]));
            } else {  // prim_hit with attributes (finish_query's textured planes, the entry's shapes)
              PrimA P;
              load_prim_a(rec, P);
              HitAttr at;
              float th;
              prim_hit<true, kPlanes, kTex>(P, rec, q.r, th, &at);
              hp = at.p;
              hn = at.n;
              hu = at.u;
              hv = at.v;
              mat_id = (int)RT_TAG_MATERIAL(prim_tag(P));
            }
          }
        }
      }
      }
      const bool wave_wants_here = __ballot(want) != 0ull;  // lanes outside this block want nothing
      if (fast || st0 < 0) {
        // advanced by shadow_step_kernel / idle since an earlier step: nothing changes
      } else if (!want) {  // the sample finished: idle until the wave's batch is done
        if (!no_batch || wave_wants_here) {  // (a wave that retires now is never read again)
          stu(F_UNIT, (uint32_t)-2);
          store_no_query(a.query, N, slot);
        }
      } else {
        stu(F_CTRL, (uint32_t)st | ((uint32_t)depth << 4));
        if (a.late_draws) stu(F_RNG, rng.ctr);
        if (st == ST_SHADOW) {  // a closest query's ray travels in the query record
          stu(F_LIGHT, (uint32_t)light | ((uint32_t)ls << 16));
          if (ls > 0) stf(F_VIS, vis);
          if (light > 0) { stf(F_FIN, fin.x); stf(F_FIN + 1, fin.y); stf(F_FIN + 2, fin.z); }
          if (st0 != ST_SHADOW) {  // shadow -> shadow steps never change the ray
            if (kFrames) {
              stf(F_RAY, ray.o.x); stf(F_RAY + 1, ray.o.y); stf(F_RAY + 2, ray.o.z);
              stf(F_RAY + 3, ray.d.x); stf(F_RAY + 4, ray.d.y); stf(F_RAY + 5, ray.d.z);
              stf(F_RAY + 6, ray.time);
            } else if (!a.pinhole) {
              stf(F_RAY, ray.o.x); stf(F_RAY + 1, ray.o.y); stf(F_RAY + 2, ray.o.z);
            }
          }
        }
        store_query(a.query, N, slot, qo, qd, qtmax, qkind);
      }
    }
  }
  // tell the host another step is needed: a plain store, no atomic (all writers store 1); a
  // slot-wave left with no query (every sample of its batch finished) is flagged for
  // start_kernel, which pulls its next batch in this same step -- or retired here when its
  // shard's claim counter is already past the call's units (start_kernel's claim could only
  // retire it: a call whose samples were all in flight skips that pass over every slot)
  const bool wave_wants = __ballot(want) != 0ull;
  if ((threadIdx.x & 63) == 0) {
    if (wave_wants) {
      *a.any_query = 1u;
    } else {
      a.wave_done[wave] = no_batch ? 1u : kWaveIdle;
    }
  }
  if constexpr (kInline) {  // the queries answered here, counted as the trace kernel counts its own
    unsigned long long nr = n_inline;
    for (int off = 32; off > 0; off >>= 1) nr += __shfl_xor(nr, off);
    if ((threadIdx.x & 63) == 0 && nr) atomicAdd(a.rays, nr);
  }
}

// One-pass calls (every sample of the call traced by one launch; no Trace recursion, point
// lights only, so no draw after a sample's start): each unit's camera ray -- start_kernel's
// ops -- written to the query record of the slot with the unit's own index, and nothing else:
// the direction; the origin for a thin-lens camera; the ray time for scenes with transformed
// shapes (moving spheres; a plane ignores it, so planes-only scenes skip that draw); a kind
// word only when some tile reaches past the image (those units: -1, and a miss result) -- in
// the compact field layout of LogicArgs::op_fo / op_ft / op_fk.
__global__ __launch_bounds__(kBlock) void camera_kernel(LogicArgs a) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.any_query = 1u;  // the trace launch runs
  const long long unit = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (unit >= a.n_units) return;
  const size_t N = (size_t)(unsigned)a.n_slots, u = (size_t)unit;
  float* Q = a.query;
  int px, py, sample;
  uint64_t key;
  if (!unit_coords(a, unit, px, py, sample, key)) {  // edge tile: pixel outside the image
    Q[(size_t)a.op_fk * N + u] = __int_as_float(-1);
    a.result[u] = -1;
    return;
  }
  Rng rng;
  const Ray ray = sample_ray(a, px, py, sample, key, rng, a.spp_sqrt > 1 || a.cam.aperture > 0.0f || a.op_ft >= 0);
  Q[u] = ray.d.x;
  Q[N + u] = ray.d.y;
  Q[2 * N + u] = ray.d.z;
  if (a.op_fo >= 0) {
    Q[(size_t)a.op_fo * N + u] = ray.o.x;
    Q[(size_t)(a.op_fo + 1) * N + u] = ray.o.y;
    Q[(size_t)(a.op_fo + 2) * N + u] = ray.o.z;
  }
  if (a.op_ft >= 0) Q[(size_t)a.op_ft * N + u] = (float)rng.next();
  if (a.op_fk >= 0) Q[(size_t)a.op_fk * N + u] = __int_as_float(0);
}

// New samples.  A slot-wave whose 64 slots are all idle (every sample of its batch finished,
// or the slots are fresh) pulls the next batch of 64 consecutive units -- one pixel's
// samples: coherent rays -- from its counter shard (one 128-B line per shard), and each
// slot starts its sample: compute_pixel_color's jittered sub-position and the camera ray
// (raytracer.cpp:18-70, camera.cpp:98-179), whose closest-hit query it emits.  Runs after
// logic_kernel in every step (the same step in which a wave's last sample finishes) and
// alone in the call's first step, where it visits every slot-wave and initialises every
// slot; 8 waves per SIMD: the sample-start code kept in logic_kernel cost it 36 registers.
__global__ __launch_bounds__(kBlock, 8) void start_kernel(LogicArgs a) {
  const int slot = a.slot_base + (int)(blockIdx.x * kBlock + threadIdx.x);
  if (blockIdx.x == 0) {  // this step's trace counters, and the next step's any_query line
    for (int i = (int)threadIdx.x; i < a.fetch_reset_n; i += kBlock) a.fetch_reset[i * kFetchStride] = 0u;
    if (threadIdx.x == 0) *a.any_query_next = 0u;
  }
  // only the slot-waves logic_kernel flagged in this step (one scalar load per wave); every
  // slot-wave in the call's first step, which also initialises every slot
  if (!a.first_step && a.wave_done[__builtin_amdgcn_readfirstlane(slot >> 6)] != kWaveIdle) return;
  const int N = a.n_slots;
  uint32_t* S = a.state;
  const int lane = (int)(threadIdx.x & 63);
  const int wave = slot >> 6;
  const int shard = wave % a.batch_shards;
  unsigned int j = 0;
  if (a.first_step) {  // batch w for wave w: init_kernel set each shard's counter past them
    j = (unsigned)(wave / a.batch_shards);
  } else {
    if (lane == 0) j = atomicAdd(a.batch_ctr + shard * kCtrStride, 1u);
    j = __shfl(j, 0);
  }
  const long long batch = (long long)j * a.batch_shards + shard;
  const long long unit = batch * 64 + lane;
  if (batch * 64 >= a.n_units) {  // every unit claimed: the slot-wave retires (n_units is a multiple of 64)
    S[F_UNIT * N + slot] = 0xFFFFFFFFu;
    if (lane == 0) a.wave_done[wave] = 1u;
    return;
  }
  if (lane == 0) {
    a.wave_done[wave] = 0u;
    // another step is needed even if every pixel of the batch lies outside the image (an edge
    // tile's bottom rows): the wave's slots stay idle, and the next step claims again
    *a.any_query = 1u;
  }
  int px, py, sample;
  uint64_t key;
  if (!unit_coords(a, unit, px, py, sample, key, false)) {  // edge tile: pixel outside the image (stays idle)
    if (a.first_step) {
      S[F_UNIT * N + slot] = (uint32_t)-2;
      store_no_query(a.query, N, slot);
    }
    return;
  }
  Rng rng;
  Ray ray = sample_ray(a, px, py, sample, key, rng);
  ray.time = (float)rng.next();
  S[F_UNIT * N + slot] = (uint32_t)unit;
  S[F_CTRL * N + slot] = (uint32_t)ST_CLOSEST;  // depth 0
  if (a.late_draws) {
    S[F_RNG * N + slot] = rng.ctr;
    S[F_KEY * N + slot] = (uint32_t)rng.key;
    S[(F_KEY + 1) * N + slot] = (uint32_t)(rng.key >> 32);
  }
  if (a.pinhole) store_cam_query(a.query, N, slot, ray.d, ray.time);
  else store_query(a.query, N, slot, ray.o, ray.d, ray.time, 0);
}

// The next soft-shadow sample of a light (shade, raytracer.cpp:214-236): a slot in ST_SHADOW
// whose light (radius > 0) still has samples to draw after this result adds the result to its
// visibility count and emits the next sample's shadow query -- the logic kernel's own ops
// for that transition, in a kernel light enough to run at 8 waves per SIMD (the logic
// kernel with recursion frames runs at 2).  It runs first in the step and marks the result
// word it consumed (kResAdvanced); the logic kernel then leaves exactly those slots alone.
__global__ __launch_bounds__(kBlock, 8) void shadow_step_kernel(LogicArgs a) {
  const int slot = a.slot_base + (int)(blockIdx.x * kBlock + threadIdx.x);
  if (a.wave_done[__builtin_amdgcn_readfirstlane(slot >> 6)] != 0u || slot >= a.slot_end) return;
  const int N = a.n_slots;
  const uint32_t* S = a.state;
  if ((int)S[F_UNIT * N + slot] < 0 || (S[F_CTRL * N + slot] & 15u) != (uint32_t)ST_SHADOW) return;
  const uint32_t lw = S[F_LIGHT * N + slot];
  const int light = (int)(lw & 0xffffu), ls = (int)(lw >> 16);
  const rt_light& L = a.lights[light];
  if (!(L.radius > 0.0f && ls + 1 < a.light_samples)) return;
  float vis = ls > 0 ? __uint_as_float(S[F_VIS * N + slot]) : 0.0f;
  if (a.result[slot] == 0) vis += 1.0f;
  Rng rng;
  rng.key = (uint64_t)S[F_KEY * N + slot] | ((uint64_t)S[(F_KEY + 1) * N + slot] << 32);
  rng.ctr = S[F_RNG * N + slot];
  const HitRec hr = load_hit(hit_rec(a.hit, slot));
  V3 target{L.location[0], L.location[1], L.location[2]};
  target = add(target, mul(rng.in_unit_sphere(), L.radius));
  const V3 lv = sub(target, hr.p);
  const float qtmax = sqrtf(dot(lv, lv));
  const V3 qd = normalize(lv);
  const V3 qo = add(hr.p, mul(hr.n, 1e-4f));
  uint32_t* W = a.state;
  W[F_LIGHT * N + slot] = (uint32_t)light | ((uint32_t)(ls + 1) << 16);
  W[F_VIS * N + slot] = __float_as_uint(vis);
  W[F_RNG * N + slot] = rng.ctr;
  store_query(a.query, N, slot, qo, qd, qtmax, 1);
  a.result[slot] = kResAdvanced;
}

// compute_pixel_color's accumulation (raytracer.cpp:46-69): totalColor starts at {0,0,0},
// adds every sample's Trace colour in (j, i) order, then divides by (float)(s*s); with
// s <= 1 the single Trace colour is returned as is.
#ifndef RT_RED_CHUNK
#define RT_RED_CHUNK 16
#endif
constexpr int kRedChunk = RT_RED_CHUNK;        // samples per pixel staged per pass (A/B: make variant)
constexpr int kRedStride = kRedChunk * 3 + 1;  // padded LDS row (odd: conflict-free column reads)
__global__ __launch_bounds__(kBlock) void reduce_kernel(LogicArgs a) {
  // The block's 256 pixels own a contiguous run of samples (unit = pixel * n_samples + s,
  // 3 floats each).  Each pass stages 16 samples of every pixel through LDS with coalesced
  // loads; every thread then adds its own pixel's samples in the reference's order.
  __shared__ float stage[kBlock * kRedStride];
  const int p0 = blockIdx.x * kBlock;
  const int np = min(kBlock, a.n_pixels - p0);
  const int p = p0 + (int)threadIdx.x;
  const size_t row = (size_t)a.n_samples * 3;
  const float* base = a.samples + (size_t)p0 * row;
  V3 acc{0.0f, 0.0f, 0.0f};
  const int ns = a.spp_sqrt <= 1 ? 1 : a.n_samples;
  for (int s0 = 0; s0 < ns; s0 += kRedChunk) {
    const int cw = min(kRedChunk, ns - s0) * 3;  // floats per pixel in this pass
    if ((row & 3) == 0 && (cw & 3) == 0) {  // 16-B aligned rows and chunks: float4 loads
      const int cw4 = cw >> 2;
      for (int i = (int)threadIdx.x; i < np * cw4; i += kBlock) {
        const int j = i / cw4, r = (i - j * cw4) * 4;
        const float4 v = *reinterpret_cast<const float4*>(base + (size_t)j * row + (size_t)s0 * 3 + r);
        float* d = stage + j * kRedStride + r;
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
      }
    } else {
      for (int i = (int)threadIdx.x; i < np * cw; i += kBlock) {
        const int j = i / cw, r = i - j * cw;
        stage[j * kRedStride + r] = base[(size_t)j * row + (size_t)s0 * 3 + r];
      }
    }
    __syncthreads();
    if ((int)threadIdx.x < np) {
      const float* q = stage + threadIdx.x * kRedStride;
      if (a.spp_sqrt <= 1) acc = V3{q[0], q[1], q[2]};
      else
        for (int k = 0; k < cw; k += 3) acc = V3{acc.x + q[k], acc.y + q[k + 1], acc.z + q[k + 2]};
    }
    __syncthreads();
  }
  if (p >= a.n_pixels) return;
  int x, y;
  size_t off;
  if (!pixel_coords(a, p, x, y, off)) return;
  V3 c = acc;
  if (a.spp_sqrt > 1) {  // compute_pixel_color: sum / (float)(s*s) (raytracer.cpp:46-69)
    const float tot = (float)a.n_samples;
    c = V3{acc.x / tot, acc.y / tot, acc.z / tot};
  }
  a.out[off] = c.x;
  a.out[off + 1] = c.y;
  a.out[off + 2] = c.z;
}

// One sample of a one-pass call, from the trace launch's answer: Trace's miss colour or the
// hit's shade with the occlusion bits the tracing lane left (raytracer.cpp:180-274, 293-303),
// then Trace's (lc * L + r * R) + t * T with no child traced (:303-350) -- the logic step's ops
// for these states, in its order (point lights: one shadow ray each, vis = count / 1).  `hr`
// is the unit's hit record (loaded by the caller; unused for a miss).
template <bool kTex>
__device__ __forceinline__ V3 one_pass_sample(const LogicArgs& a, size_t unit, int res, const HitRec& hr,
                                              unsigned occl_bits, const V3* ray_origin = nullptr) {
  if (res < 0) return V3{0.1f, 0.1f, 0.1f};
  const V3 hp = hr.p, hn = hr.n;
  const rt_material& m = a.mats[hr.mat];
  float hu = 0.0f, hv = 0.0f;
  if (kTex) {
    const float2 uv = a.hit_uv[unit];
    hu = uv.x;
    hv = uv.y;
  }
  const V3 base0 = kTex ? diffuse_color(a, m, hu, hv) : V3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
  V3 fin{base0.x * m.k_ambient, base0.y * m.k_ambient, base0.z * m.k_ambient};
  if (a.n_fuse > 0) {
    const size_t N = (size_t)(unsigned)a.n_slots;
    V3 ro{a.cam.location[0], a.cam.location[1], a.cam.location[2]};
    if (ray_origin) {  // flat_render_kernel: the camera ray it traced itself
      ro = *ray_origin;
    } else if (a.op_fo >= 0) {
      const float* Qo = a.query + (size_t)a.op_fo * N + unit;
      ro = V3{Qo[0], Qo[N], Qo[2 * N]};
    }
    for (int light = 0; light < a.n_lights; ++light) {
      const rt_light& L = a.lights[light];
      float vis = 0.0f;
      if (!((occl_bits >> light) & 1u)) vis += 1.0f;
      vis = vis / (float)1;  // ns = 1 (radius 0)
      if (!(vis <= 0.0f)) {
        V3 base = kTex ? diffuse_color(a, m, hu, hv) : V3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
        V3 lc = sub(V3{L.location[0], L.location[1], L.location[2]}, hp);
        float dsq = dot(lc, lc);
        float ldist = sqrtf(dsq);
        V3 Ld = normalize(lc);
        float ndl = smax(0.0f, dot(hn, Ld));
        V3 diff = mul(base, ndl);
        float si = 0.0f;  // as in logic_kernel: V and H only when the specular term is not +-0
        if (!spec_zero(m)) {
          V3 V = normalize(sub(ro, hp));
          V3 H = normalize(add(Ld, V));
          float ndh = smax(0.0f, dot(hn, H));
          si = rt_powf(ndh, m.shininess);
        }
        V3 spec{m.specular[0] * si, m.specular[1] * si, m.specular[2] * si};
        float att = (10.0f * L.intensity) / (25.0f + 10.0f * ldist + 150.0f * dsq);
        V3 inner{diff.x * m.k_diffuse + spec.x * m.k_specular, diff.y * m.k_diffuse + spec.y * m.k_specular,
                 diff.z * m.k_diffuse + spec.z * m.k_specular};
        V3 contrib{L.color[0] * inner.x * att, L.color[1] * inner.y * att, L.color[2] * inner.z * att};
        fin = V3{fin.x + contrib.x * vis, fin.y + contrib.y * vis, fin.z + contrib.z * vis};
      }
    }
  }
  const float lcf = smax(0.0f, 1.0f - m.reflectivity - m.transparency);
  const V3 A{lcf * fin.x, lcf * fin.y, lcf * fin.z};
  const V3 part{A.x + m.reflectivity * 0.0f, A.y + m.reflectivity * 0.0f, A.z + m.reflectivity * 0.0f};
  return V3{part.x + m.transparency * 0.0f, part.y + m.transparency * 0.0f, part.z + m.transparency * 0.0f};
}

// The one-pass call's last kernel: the logic step (one_pass_sample) and reduce_kernel in one
// pass, with no per-sample colour buffer.  A block owns 128 pixels; each pass shades 8 samples
// of every pixel into LDS -- 1024 units, 4 per thread, their result words, occlusion bits and
// hit records loaded together before any is used (the shading is bound by these dependent
// loads, not by its arithmetic) -- then each pixel's thread adds its samples in the
// reference's order (raytracer.cpp:46-69).  12.8 KB of LDS per block: 8 waves per SIMD.
#ifndef RT_SR_PIXELS
#define RT_SR_PIXELS 64  // r04 A/B (head / em8 / C3 Mrays/s): 128 px x 4 waves 7147 / 5850 / 27437, 64 x 6 7174 / 5901 / 28480, 64 x 8 7153 / 5904 / 28131
#endif
#ifndef RT_SR_WAVES
#define RT_SR_WAVES 6
#endif
#ifndef RT_SR_CHUNK
#define RT_SR_CHUNK 8
#endif
constexpr int kSrPixels = RT_SR_PIXELS, kSrChunk = RT_SR_CHUNK, kSrStride = kSrChunk * 3 + 1;  // odd row: conflict-free sums
constexpr int kSrUnits = kSrPixels * kSrChunk / kBlock;                     // units per thread per pass
// kHitCompact calls (r06): the hit record finish_query used to store, rebuilt here from what the
// trace kernel keeps -- the hit's t -- and what the call already holds: the unit's camera ray
// (origin the camera's location or the stored lens origin, direction from the query record) and
// the plane record's precomputed normal and tag.  The point is o + t d with the trace kernel's own
// ops on the same operands, so the same bits.
__device__ __forceinline__ HitRec compact_hit(const LogicArgs& a, size_t unit, int res) {
  const size_t N = (size_t)(unsigned)a.n_slots;
  const float t = a.hit[unit];
  const float4 ns = a.prim_shade[res];  // the plane's normal and material (rt_scene_create)
  V3 o{a.cam.location[0], a.cam.location[1], a.cam.location[2]};
  if (a.op_fo >= 0) {
    const float* Qo = a.query + (size_t)a.op_fo * N + unit;
    o = V3{Qo[0], Qo[N], Qo[2 * N]};
  }
  const V3 d{a.query[unit], a.query[N + unit], a.query[2 * N + unit]};
  return HitRec{V3{o.x + t * d.x, o.y + t * d.y, o.z + t * d.z}, V3{ns.x, ns.y, ns.z}, 0.0f, 0.0f, __float_as_uint(ns.w)};
}
// kHitRecompute calls (r06, transformed shapes): the record the trace kernel's settle computed
// for its fused shadow ray and no longer stores -- prim_hit with attributes on the same
// primitive and the same ray (the unit's camera ray and its time), so the same bits.
__device__ __forceinline__ HitRec recompute_hit(const LogicArgs& a, size_t unit, int res) {
  const size_t N = (size_t)(unsigned)a.n_slots;
  Ray r;
  r.o = V3{a.cam.location[0], a.cam.location[1], a.cam.location[2]};
  if (a.op_fo >= 0) {
    const float* Qo = a.query + (size_t)a.op_fo * N + unit;
    r.o = V3{Qo[0], Qo[N], Qo[2 * N]};
  }
  r.d = V3{a.query[unit], a.query[N + unit], a.query[2 * N + unit]};
  r.time = a.op_ft >= 0 ? a.query[(size_t)a.op_ft * N + unit] : 0.0f;
  const float4* rec = a.c.prims + (size_t)res * a.c.prim_stride4;
  PrimA P;
  load_prim_a(rec, P);
  HitAttr at;
  float t;
  prim_hit<true, false, false>(P, rec, r, t, &at);
  return HitRec{at.p, at.n, 0.0f, 0.0f, RT_TAG_MATERIAL(prim_tag(P))};
}
template <bool kTex, int kHit>
__global__ __launch_bounds__(kBlock, RT_SR_WAVES) void shade_reduce_kernel(LogicArgs a) {
  __shared__ float stage[kSrPixels * kSrStride];
  const int p0 = blockIdx.x * kSrPixels;
  const int np = min(kSrPixels, a.n_pixels - p0);
  const int ns = a.n_samples;
  V3 acc{0.0f, 0.0f, 0.0f};
  for (int s0 = 0; s0 < ns; s0 += kSrChunk) {
    const int cn = min(kSrChunk, ns - s0), total = np * cn;
    size_t u[kSrUnits];
    int res[kSrUnits], st[kSrUnits];
    unsigned ob[kSrUnits];
#pragma unroll
    for (int m = 0; m < kSrUnits; ++m) {
      const int i = (int)threadIdx.x + m * kBlock;
      const int j = cn == kSrChunk ? i / kSrChunk : i / cn, k = i - j * cn;
      st[m] = j * kSrStride + k * 3;
      u[m] = (size_t)(p0 + j) * (size_t)ns + (size_t)(s0 + k);
      res[m] = i < total ? a.result[u[m]] : -1;
      ob[m] = i < total && a.n_fuse > 0 ? a.occl[u[m]] : 0u;
    }
    HitRec hr[kSrUnits];
#pragma unroll
    for (int m = 0; m < kSrUnits; ++m) {
      if constexpr (kHit == kHitCompact)  // (no lights: the shading reads the material alone)
        hr[m] = res[m] < 0 ? HitRec{}
                : a.n_fuse > 0 ? compact_hit(a, u[m], res[m])
                               : HitRec{V3{}, V3{}, 0.0f, 0.0f, __float_as_uint(a.prim_shade[res[m]].w)};
      else if constexpr (kHit == kHitRecompute) hr[m] = res[m] >= 0 ? recompute_hit(a, u[m], res[m]) : HitRec{};
      else hr[m] = res[m] >= 0 ? load_hit(hit_rec_u(a.hit, u[m])) : HitRec{};
    }
#pragma unroll
    for (int m = 0; m < kSrUnits; ++m) {
      if ((int)threadIdx.x + m * kBlock < total) {
        const V3 c = one_pass_sample<kTex>(a, u[m], res[m], hr[m], ob[m]);
        float* d = stage + st[m];
        d[0] = c.x;
        d[1] = c.y;
        d[2] = c.z;
      }
    }
    __syncthreads();
    if ((int)threadIdx.x < np) {
      const float* q = stage + threadIdx.x * kSrStride;
      if (a.spp_sqrt <= 1) acc = V3{q[0], q[1], q[2]};
      else
        for (int k = 0; k < cn * 3; k += 3) acc = V3{acc.x + q[k], acc.y + q[k + 1], acc.z + q[k + 2]};
    }
    __syncthreads();
  }
  const int p = p0 + (int)threadIdx.x;
  if ((int)threadIdx.x >= np) return;
  int x, y;
  size_t off;
  if (!pixel_coords(a, p, x, y, off)) return;
  V3 c = acc;
  if (a.spp_sqrt > 1) {  // compute_pixel_color: sum / (float)(s*s) (raytracer.cpp:46-69)
    const float tot = (float)a.n_samples;
    c = V3{acc.x / tot, acc.y / tot, acc.z / tot};
  }
  a.out[off] = c.x;
  a.out[off + 1] = c.y;
  a.out[off + 2] = c.z;
}

// Few-primitive one-pass calls (r06): the whole sample in one thread -- the camera ray
// (camera_kernel's ops), its closest hit and its point-light shadow rays against the scene's
// primitives, and the shading -- with shade_reduce_kernel's per-pixel sums.  A scene of at most
// RT_FLAT_PRIMS bounded primitives gives every traversal one leaf item of all of them (the trace
// kernel's root_item), so the traversal kernel's queue, stacks and refill only move a handful of
// primitive tests around, and camera rays, results and hit records make three HBM round trips
// per sample.  Here each query runs test_prims over the same leaf item (the exact reference-leaf
// filter, closest hit by (t, reference index): no order dependence) and over the unbounded
// primitives (complete_query), the hit record is the fused settle's (finish_query / prim_hit)
// and the shadow rays are fused_shadow's: the same functions on the same operands, so the
// same bits.  Rays are counted as the trace kernel counts them (camera + shadow rays).
#ifndef RT_FLAT_WAVES
#define RT_FLAT_WAVES 1  // minimum blocks per CU the allocation must allow (1: the compiler's choice)
#endif
template <bool kPlanesOnly>
__global__ __launch_bounds__(kBlock, RT_FLAT_WAVES) void flat_render_kernel(LogicArgs a, TraceArgs t) {
  __shared__ float stage[kSrPixels * kSrStride];
  const int p0 = blockIdx.x * kSrPixels;
  const int np = min(kSrPixels, a.n_pixels - p0);
  const int ns = a.n_samples;
  const int nb = t.root_item < 0 && t.root_item != kNoItem ? (int)((uint32_t)t.root_item & 0x7fu) : 0;
  unsigned int nrays = 0, nprim = 0;
  auto flat_query = [&](const Query& q, HitState& h) {  // the leaf item of all bounded primitives, then the rest
    if (nb > 0) test_prims<false, kPlanesOnly>(t, 0, nb, q.r, q.any, q.tmax, q.par, true, h, nprim);
    complete_query<false, kPlanesOnly>(t, 0, q, h, nprim);
  };
  V3 acc{0.0f, 0.0f, 0.0f};
  for (int s0 = 0; s0 < ns; s0 += kSrChunk) {
    const int cn = min(kSrChunk, ns - s0), total = np * cn;
    for (int m = 0; m < kSrUnits; ++m) {
      const int i = (int)threadIdx.x + m * kBlock;
      if (i >= total) continue;
      const int j = cn == kSrChunk ? i / kSrChunk : i / cn, k = i - j * cn;
      const size_t u = (size_t)(p0 + j) * (size_t)ns + (size_t)(s0 + k);
      int px, py, sample;
      uint64_t key;
      int res = -1;
      unsigned ob = 0;
      HitRec hr{};
      V3 ro{0.0f, 0.0f, 0.0f};
      if (unit_coords(a, (long long)u, px, py, sample, key)) {
        Rng rng;
        const Ray cam = sample_ray(a, px, py, sample, key, rng);  // (a lazy key here: C3 -3.7 %, codegen)
        const float time = a.op_ft >= 0 ? (float)rng.next() : 0.0f;  // camera_kernel's ray-time draw
        ro = cam.o;
        Query q;
        setup_query(q, cam.o, cam.d, time, false);
        ++nrays;
        HitState h{__builtin_inff(), 0x7fffffff, -1, false};
        flat_query(q, h);
        res = h.best_idx;
        if (res >= 0) {
          const float4* rec = t.c.prims + (size_t)res * t.c.prim_stride4;
          if constexpr (kPlanesOnly) {  // finish_query's record: o + t d, the plane's normal and tag
            const float* w = reinterpret_cast<const float*>(rec);
            hr.p = V3{q.r.o.x + h.best_t * q.r.d.x, q.r.o.y + h.best_t * q.r.d.y, q.r.o.z + h.best_t * q.r.d.z};
            hr.n = V3{w[3], w[7], w[11]};
            hr.mat = RT_TAG_MATERIAL(__float_as_uint(w[15]));
          } else {  // the fused settle's record
            PrimA P;
            load_prim_a(rec, P);
            HitAttr at;
            float th;
            prim_hit<true, false, false>(P, rec, q.r, th, &at);
            hr.p = at.p;
            hr.n = at.n;
            hr.mat = RT_TAG_MATERIAL(prim_tag(P));
          }
          for (int l = 0; l < t.n_fuse; ++l) {  // fused_shadow
            const rt_light& L = t.lights[l];
            const V3 lv = sub(V3{L.location[0], L.location[1], L.location[2]}, hr.p);
            const float tmax = sqrtf(dot(lv, lv));
            Query sq;
            setup_query(sq, add(hr.p, mul(hr.n, 1e-4f)), normalize(lv), tmax, true);
            ++nrays;
            HitState sh{__builtin_inff(), 0x7fffffff, -1, false};
            flat_query(sq, sh);
            if (sh.done) ob |= 1u << l;
          }
        }
      }
      const V3 c = one_pass_sample<false>(a, u, res, hr, ob, &ro);
      float* d = stage + j * kSrStride + k * 3;
      d[0] = c.x;
      d[1] = c.y;
      d[2] = c.z;
    }
    __syncthreads();
    if ((int)threadIdx.x < np) {
      const float* q = stage + threadIdx.x * kSrStride;
      if (a.spp_sqrt <= 1) acc = V3{q[0], q[1], q[2]};
      else
        for (int k = 0; k < cn * 3; k += 3) acc = V3{acc.x + q[k], acc.y + q[k + 1], acc.z + q[k + 2]};
    }
    __syncthreads();
  }
  unsigned long long nr = nrays;
  for (int off = 32; off > 0; off >>= 1) nr += __shfl_xor(nr, off);
  if ((threadIdx.x & 63) == 0 && nr) atomicAdd(t.rays, nr);
  const int p = p0 + (int)threadIdx.x;
  if ((int)threadIdx.x >= np) return;
  int x, y;
  size_t off;
  if (!pixel_coords(a, p, x, y, off)) return;
  V3 c = acc;
  if (a.spp_sqrt > 1) {  // compute_pixel_color: sum / (float)(s*s) (raytracer.cpp:46-69)
    const float tot = (float)a.n_samples;
    c = V3{acc.x / tot, acc.y / tot, acc.z / tot};
  }
  a.out[off] = c.x;
  a.out[off + 1] = c.y;
  a.out[off + 2] = c.z;
}

// kInline calls launch no traversal: the host's per-step flag (the trace kernel's first store
// otherwise) -- start_kernel emitted camera queries, so the next step has samples to run
__global__ void step_flag_kernel(const unsigned int* any_query, unsigned int* host_flag) { *host_flag = *any_query; }

// pixel finalisation (raytracer.cpp:446-457, image.cpp:28-37), the same ops as rth_quantise
__global__ __launch_bounds__(kBlock) void quantise_kernel(const float* rgb, long long n, uint8_t* out) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const float gamma = 1.1f;
  const float g = rt_powf(rgb[i], 1.0f / gamma);
  const float c = smax(0.0f, smin(1.0f, g));
  const int v = static_cast<int>((double)c * 255.999);
  out[i] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// The call's control state, one block: the control block, the pipelines' trace counters and
// any_query lines, and each claim counter set past the first step's batches (in the first
// step slot-wave w takes batch w = j * shards + w % shards without a claim, so shard k's
// counter starts at the number of waves w with w % shards == k).  The slots themselves are
// initialised by that first start_kernel, which visits every slot-wave.
struct InitArgs {
  int n_slots;
  unsigned int* ctl;
  int ctl_words;
  unsigned int* fetch;
  int fetch_words;
  unsigned int* batch_ctr;
  int batch_shards;
  unsigned int* tile_cost;  // one-pass calls: the measured per-tile node visits, cleared
  int n_tiles;
};
__global__ __launch_bounds__(kBlock) void init_kernel(InitArgs a) {
  for (int i = (int)threadIdx.x; i < a.ctl_words; i += kBlock) a.ctl[i] = 0u;
  if (a.tile_cost)
    for (int i = (int)threadIdx.x; i < a.n_tiles; i += kBlock) a.tile_cost[i] = 0u;
  for (int i = (int)threadIdx.x; i < a.fetch_words; i += kBlock) a.fetch[i] = 0u;
  const int waves = a.n_slots >> 6;
  for (int k = (int)threadIdx.x; k < a.batch_shards; k += kBlock)
    a.batch_ctr[k * kCtrStride] = (unsigned)(waves / a.batch_shards + (k < waves % a.batch_shards ? 1 : 0));
}

template <bool F, bool R, bool T>
void launch_logic2(const LogicArgs& la, bool planes, bool inl, unsigned blocks, hipStream_t st) {
  if (inl && !T) {  // few-primitive scenes without textures: queries answered in the step
    if (planes) hipLaunchKernelGGL((logic_kernel<F, R, T, true, !T>), dim3(blocks), dim3(kBlock), 0, st, la);
    else hipLaunchKernelGGL((logic_kernel<F, R, T, false, !T>), dim3(blocks), dim3(kBlock), 0, st, la);
  } else if (planes) {
    hipLaunchKernelGGL((logic_kernel<F, R, T, true>), dim3(blocks), dim3(kBlock), 0, st, la);
  } else {
    hipLaunchKernelGGL((logic_kernel<F, R, T, false>), dim3(blocks), dim3(kBlock), 0, st, la);
  }
}
// trace launch (the refill kernel; count: the instrumented variant)
template <bool kCount, bool kFixed>
void launch_trace3(const TraceArgs& ta, bool planes, bool soft, bool seven, unsigned blocks, size_t lds, hipStream_t st) {
  if (!kCount && seven && planes && ta.n_fuse > 0)  // 7 waves/SIMD (whole frames; render_tiles)
    hipLaunchKernelGGL((trace_refill_kernel<false, true, true, false, true, true>), dim3(blocks), dim3(kBlock), lds, st, ta);
  else if (!kCount && seven && planes && !soft)
    hipLaunchKernelGGL((trace_refill_kernel<false, true, false, false, true, true>), dim3(blocks), dim3(kBlock), lds, st, ta);
  else if (ta.n_fuse > 0 && planes)  // point lights only (the host's choice)
    hipLaunchKernelGGL((trace_refill_kernel<kCount, true, true, false, false, kFixed>), dim3(blocks), dim3(kBlock), lds, st, ta);
  else if (ta.n_fuse > 0 || (ta.one_pass && !planes))  // ... and no textures: the fused path stores no (u, v);
                                                       // one-pass calls of transformed shapes: the lane computes
                                                       // the hit record (planes-only one-pass calls without
                                                       // lights take the plain planes instance below, whose
                                                       // finish_query writes a textured hit's (u, v))
    hipLaunchKernelGGL((trace_refill_kernel<kCount, false, true, false, false, kFixed>), dim3(blocks), dim3(kBlock), lds, st, ta);
  else if (soft && planes)
    hipLaunchKernelGGL((trace_refill_kernel<kCount, true, false, true, false, kFixed>), dim3(blocks), dim3(kBlock), lds, st, ta);
  else if (soft)
    hipLaunchKernelGGL((trace_refill_kernel<kCount, false, false, true, false, kFixed>), dim3(blocks), dim3(kBlock), lds, st, ta);
  else if (planes)
    hipLaunchKernelGGL((trace_refill_kernel<kCount, true, false, false, false, kFixed>), dim3(blocks), dim3(kBlock), lds, st, ta);
  else
    hipLaunchKernelGGL((trace_refill_kernel<kCount, false, false, false, false, kFixed>), dim3(blocks), dim3(kBlock), lds, st, ta);
}
// trace launch: soft = the lanes continue soft-light shadow samples themselves (kSoft)
// fixed: the call's loop parameters are the instance's defaults (kFixed instances; not for
// the instrumented count_work launches, which keep runtime values)
void launch_trace(const TraceArgs& ta, bool count, bool planes, bool soft, bool seven, bool fixed, unsigned blocks,
                  size_t lds, hipStream_t st) {
  if (count) launch_trace3<true, false>(ta, planes, soft, seven, blocks, lds, st);
  else if (fixed) launch_trace3<false, true>(ta, planes, soft, seven, blocks, lds, st);
  else launch_trace3<false, false>(ta, planes, soft, seven, blocks, lds, st);
}
static int pipes_env() { return (int)knob(K_PIPES, 1); }
// r03 sweep: 4 / 8 / 16 / 32 fetch shards: 5377 / 5542 / 5628 / 5769 Mrays/s (headline)
static int fetch_shards_env() { return (int)knob(K_FETCH_SHARDS, 32); }
static int batch_shards_env() { return (int)knob(K_BATCH_SHARDS, 128); }
// r03 sweep at 32M slots: leaf 12 / 16 / 24 / 32 (two pipelines); DESIGN.md 5
static int leaf_min_env() { return (int)knob(K_LEAF_MIN, kLeafDefault); }
static int refill_min_env() { return (int)knob(K_REFILL, kRefillDefault); }

void launch_logic(const LogicArgs& la, bool frames, bool refr, bool tex, bool planes, bool inl, unsigned blocks,
                  hipStream_t st) {
  if (frames && refr) {
    if (tex) launch_logic2<true, true, true>(la, planes, inl, blocks, st);
    else launch_logic2<true, true, false>(la, planes, inl, blocks, st);
  } else if (frames) {
    if (tex) launch_logic2<true, false, true>(la, planes, inl, blocks, st);
    else launch_logic2<true, false, false>(la, planes, inl, blocks, st);
  } else {
    if (tex) launch_logic2<false, false, true>(la, planes, inl, blocks, st);
    else launch_logic2<false, false, false>(la, planes, inl, blocks, st);
  }
}

// ---------------------------------------------------------------- C ABI support
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIP_TRY(expr, code)                                                                     \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) return fail(code, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

uint64_t mix64_host(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27; z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}

}  // namespace

struct rt_scene_s {
  int device = 0;
  rt_scene_desc desc{};
  void* d_prims = nullptr;
  void* d_nodes = nullptr;
  void* d_mats = nullptr;
  void* d_lights = nullptr;
  void* d_tex = nullptr;
  void* d_texels = nullptr;
  void* d_prim_refs = nullptr;
  float4* d_prim_shade = nullptr;  // planes-only scenes: per primitive (normal, material) for compact hits
  void* d_ref_boxes = nullptr;
  int n_cu = 0, trace_blocks_per_cu = 0;  // plain traversal instance
  int trace_blocks_per_cu_fuse = 0, trace_blocks_per_cu_soft = 0;  // shadow-chain instances (kFuse / kSoft)
  int trace_blocks_per_cu_seven = 0, trace_blocks_per_cu_fuse_seven = 0;  // 7-wave planes instances
  bool late_draws = false;  // a light with radius > 0 or a rough material: draws after a sample's start
  bool moving = false;      // some sphere has a non-zero velocity: the ray time matters
  bool soft_lights = false;  // a light with radius > 0 (several shadow samples with -light_sample > 1)
  int* d_spill = nullptr;
  size_t spill_cap = 0;
  // per-render workspace (grown on demand)
  void* d_ctl = nullptr;  // bytes 16/24: box/prim tests, 32: rays (u64), 240..: diagnostics, 488: node visits
  int* d_tiles = nullptr;
  size_t tiles_cap = 0;
  uint64_t* d_keys = nullptr;  // a multi-frame call's per-frame counter-RNG keys
  size_t cap_keys = 0;
  std::vector<uint64_t> keys_on_device;
  // (each array grown on demand by grow(); its byte capacity beside it: a one-pass call needs
  // only the query record, result, hit record and occlusion bits of its slots)
  uint32_t* d_state = nullptr;
  uint32_t* d_frames = nullptr;
  float* d_refr = nullptr;
  float* d_query = nullptr;
  float* d_samples = nullptr;
  int* d_result = nullptr;
  float* d_hit = nullptr;
  unsigned int* d_occl = nullptr;  // per slot: occlusion bits of fused shadow rays
  float2* d_hit_uv = nullptr;      // per slot: (u, v) of the closest hit (textured scenes)
  unsigned int* d_wave_done = nullptr;
  size_t cap_state = 0, cap_frames = 0, cap_refr = 0, cap_query = 0, cap_samples = 0, cap_result = 0, cap_hit = 0,
         cap_occl = 0, cap_hit_uv = 0, cap_wave_done = 0;
  unsigned int* h_flag = nullptr;  // pinned: per pipeline, one 128-B line per step of a host batch (any_query copies)
  unsigned long long* h_stats = nullptr;  // pinned: the first kStatsBytes of the control block, copied after each batch
  std::vector<int32_t> tiles_on_device;   // the tile list d_tiles holds
  unsigned int* d_batch_ctr = nullptr;  // kMaxBatchShards counters, one 128-B line each
  unsigned int* d_fetch = nullptr;      // per pipeline: trace fetch counters (one line each) + any_query line
  hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr, ev_fork = nullptr, ev_join = nullptr;
  // per pipeline and step of a host batch: around the trace launch
  hipEvent_t ev_a[kPipes][kMaxHostBatch] = {}, ev_b[kPipes][kMaxHostBatch] = {};
  hipStream_t aux[kPipes] = {};  // pipelines 1.. run on these non-blocking streams (0: the caller's)
  int last_iters = 0;  // steps the previous render took: the size of the next render's first host batch
  // tile cost model (tile_cost_order): a sample of primitive centres, and the per-tile cost of
  // the last camera / tile size it was projected for
  std::vector<float> cost_pts;
  std::vector<unsigned char> cost_key;
  std::vector<float> tile_cost;
  // measured tile costs (instrumented one-pass calls, rt_tile_costs_measured): lane node visits
  // per tile id of the last calls with this camera / tile size / sample count (-1: not measured
  // yet), and their device / pinned host counters
  std::vector<unsigned char> meas_key;
  std::vector<float> meas_visits;
  unsigned int* d_tile_cost = nullptr;
  unsigned int* h_tile_cost = nullptr;
  size_t cap_tile_cost = 0, cap_h_tile_cost = 0;
  // a deferred one-pass call (rt_render_params.sync == 0): enqueued, not yet waited for --
  // what rt_render_wait (or the scene's next call) needs to finish it
  struct Pending {
    bool active = false, count_work = false, measure_tiles = false;
    int n_tiles = 0, tiles_x = 0, tiles_y = 0;
    std::vector<int32_t> tl_dev;
    std::vector<unsigned char> meas_key;
    TraceArgs ta{};  // the launch's arguments (diagnostic builds' reports, rt_diag.h)
  } pending;
  // a call with rt_render_params.sync == 0 that completed before returning (the step pipeline,
  // or a call split into tile chunks): its statistics, handed out by the next rt_render_wait
  bool held = false;
  rt_stats held_stats{};
  int fuse_lights = 0;  // > 0: point lights whose shadow rays the trace kernel may fuse (see rt_scene_create)
};

static void free_workspace(rt_scene_s* s) {
  void* ptrs[] = {s->d_state, s->d_frames, s->d_refr, s->d_query, s->d_result, s->d_samples, s->d_hit, s->d_wave_done,
                  s->d_occl, s->d_hit_uv};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  s->d_wave_done = nullptr;
  s->d_occl = nullptr;
  s->d_hit_uv = nullptr;
  s->d_state = nullptr; s->d_frames = nullptr; s->d_refr = nullptr;
  s->d_query = nullptr; s->d_result = nullptr; s->d_samples = nullptr; s->d_hit = nullptr;
  s->cap_state = s->cap_frames = s->cap_refr = s->cap_query = s->cap_samples = s->cap_result = s->cap_hit = 0;
  s->cap_occl = s->cap_hit_uv = s->cap_wave_done = 0;
}

// A workspace array of at least `bytes` (contents undefined): reallocated only to grow.
template <class T>
static int grow(T*& ptr, size_t& cap, size_t bytes) {
  if (ptr && bytes <= cap) return RT_OK;
  if (ptr) (void)hipFree(ptr);
  ptr = nullptr;
  cap = 0;
  HIP_TRY(hipMalloc((void**)&ptr, std::max<size_t>(bytes, 4)), RT_ENOMEM);
  cap = std::max<size_t>(bytes, 4);
  return RT_OK;
}

// Render order of a call's tiles: costliest first.  A launch ends when its slowest rays do,
// so the work consumed last should be cheap: the tiles are ordered by a cost estimate --
// how many primitives (a sample of their centres) project into the tile -- so the
// background tiles come last, in every launch and at the end of the call.  Scheduling only:
// every sample is keyed by its pixel (counter RNG), so the order changes no value.  The
// per-tile costs are cached per camera and tile size.
// Per-tile cost estimate for `cam` and the tile size (cached on the scene): how many of the
// sampled primitive centres project into each tile of the grid.
static const std::vector<float>& tile_costs(rt_scene_s* s, const rt_camera_desc* cam, int tile_w, int tile_h, int tiles_x,
                                            int tiles_y) {
  std::vector<unsigned char> key(sizeof(rt_camera_desc) + 2 * sizeof(int));
  std::memcpy(key.data(), cam, sizeof(rt_camera_desc));
  std::memcpy(key.data() + sizeof(rt_camera_desc), &tile_w, sizeof(int));
  std::memcpy(key.data() + sizeof(rt_camera_desc) + sizeof(int), &tile_h, sizeof(int));
  if (key != s->cost_key) {
    s->cost_key = key;
    s->tile_cost.assign((size_t)tiles_x * tiles_y, 0.0f);
    const float* L = cam->location;
    for (size_t k = 0; k + 2 < s->cost_pts.size(); k += 3) {
      const float v[3] = {s->cost_pts[k] - L[0], s->cost_pts[k + 1] - L[1], s->cost_pts[k + 2] - L[2]};
      const float c = v[0] * cam->z_dir[0] + v[1] * cam->z_dir[1] + v[2] * cam->z_dir[2];
      if (!(c > 1e-6f)) continue;  // behind the camera
      const float a = v[0] * cam->x_dir[0] + v[1] * cam->x_dir[1] + v[2] * cam->x_dir[2];
      const float b = v[0] * cam->y_dir[0] + v[1] * cam->y_dir[1] + v[2] * cam->y_dir[2];
      // camera_ray's mapping inverted: n = 1 - 2 p / res, n * half_sensor = (a / c) * focal
      const float px = (1.0f - a / c * cam->focal_length / cam->half_sensor_w) * 0.5f * (float)cam->res_x;
      const float py = (1.0f - b / c * cam->focal_length / cam->half_sensor_h) * 0.5f * (float)cam->res_y;
      if (!(px >= 0.0f && py >= 0.0f && px < (float)cam->res_x && py < (float)cam->res_y)) continue;
      s->tile_cost[(size_t)((int)py / tile_h) * tiles_x + (int)px / tile_w] += 1.0f;
    }
  }
  return s->tile_cost;
}

// The key of measured tile costs: camera, tile size, samples per pixel.
static std::vector<unsigned char> meas_key_of(const rt_camera_desc* cam, int tile_w, int tile_h, int n_samples) {
  std::vector<unsigned char> key(sizeof(rt_camera_desc) + 3 * sizeof(int));
  std::memcpy(key.data(), cam, sizeof(rt_camera_desc));
  const int v[3] = {tile_w, tile_h, n_samples};
  std::memcpy(key.data() + sizeof(rt_camera_desc), v, sizeof(v));
  return key;
}

// Tiles are ordered by the projected-centre estimate (ordering by the node visits an
// instrumented call measured per tile was 4 % slower on one rank's eighth, r04: those
// measurements serve bench.py's `--deal measured` instead).
static void tile_cost_order(rt_scene_s* s, const rt_camera_desc* cam, int tile_w, int tile_h, int tiles_x, int tiles_y,
                            const int32_t* tile_ids, int n_tiles, bool wanted, std::vector<int32_t>& order) {
  order.resize((size_t)n_tiles);
  for (int i = 0; i < n_tiles; ++i) order[i] = i;
  wanted = knob(K_TILE_ORDER, wanted) != 0;  // 0 / 1: never / always
  if (!wanted || n_tiles < 2) return;
  if (s->cost_pts.empty()) return;
  const std::vector<float>& cost = tile_costs(s, cam, tile_w, tile_h, tiles_x, tiles_y);
  std::stable_sort(order.begin(), order.end(), [&](int i, int j) {
    return cost[(size_t)tile_ids[i]] > cost[(size_t)tile_ids[j]];
  });
}

extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }

const char* rt_build_info(void) {
  return "librt_hip: gfx950 hand-written HIP; wavefront logic+trace kernels; SAH BVH4 (quantised nodes: fp16 codes for planes-only scenes, 8-bit otherwise) + LDS stack; one-pass and step pipelines; no MFMA";
}

int rt_device_count(int32_t* count) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return fail(RT_ENODEV, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *count = n;
  return RT_OK;
}

static int upload(void** dst, const void* src, size_t bytes) {
  if (bytes == 0) {
    *dst = nullptr;
    return RT_OK;
  }
  HIP_TRY(hipMalloc(dst, bytes), RT_ENOMEM);
  HIP_TRY(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice), RT_EDEVICE);
  return RT_OK;
}

// The nodes as laid out in HBM: AoS, one node = consecutive 16-B words fetched by one lane (an
// SoA layout -- word k of every node in array k -- measured 2.3 % slower, r04).  Scenes with
// transformed shapes keep the 64-B rt_node4 records; planes-only scenes get 80-B device nodes
// -- origin + exponents (valid-child mask in the top byte), per axis the words (lo01, lo23,
// hi01, hi23) of fp16 plane codes (exact: codes < 256), the child entries with internal
// children as the node's byte offset (node index x 80: no shift per visit) -- for
// node_visit's mixed fmas
struct NodeF16 {
  float origin[3];
  uint32_t exps;
  uint32_t p[3][4];
  int32_t child[4];
};
static_assert(sizeof(NodeF16) == 80, "80-B device node");
static uint32_t f16_code(uint32_t c) {  // binary16 bits of the integer c < 2048
  if (c == 0) return 0;
  int e = 31 - __builtin_clz(c);
  return (uint32_t)(e + 15) << 10 | ((c << (10 - e)) & 0x3ffu);
}
// the grid steps' exponent bytes unbiased: int8 k = e - 127 (bvh_wide: e in [1, 207]), the
// device nodes' form (node_visit's v_ldexp_f32 takes k as it is; r06)
static uint32_t signed_exps(uint32_t exps) {
  uint32_t ks = 0;
  for (int a = 0; a < 3; ++a) ks |= (uint32_t)(uint8_t)(int8_t)((int)((exps >> (8 * a)) & 0xffu) - 127) << (8 * a);
  return ks;
}
static int upload_nodes(void** dst, const rt_node4* nodes, int32_t n, bool planes_only) {
  if (!planes_only) {
    std::vector<rt_node4> v(nodes, nodes + n);
    for (rt_node4& d : v) d.exps = signed_exps(d.exps);
    return upload(dst, v.data(), v.size() * sizeof(rt_node4));
  }
  std::vector<NodeF16> v((size_t)n);
  for (int32_t i = 0; i < n; ++i) {
    const rt_node4& s = nodes[i];
    NodeF16& d = v[(size_t)i];
    uint32_t valid = 0;
    for (int k = 0; k < 4; ++k) {
      const uint32_t m = (s.meta >> (8 * k)) & 0xffu;
      if (m) valid |= 1u << k;
      d.child[k] = m == 0x01u ? s.child[k] * 80 : s.child[k];  // < 2^31 (rt_scene_create)
    }
    for (int a = 0; a < 3; ++a) d.origin[a] = s.origin[a];
    d.exps = signed_exps(s.exps) | valid << 24;
    const uint32_t qlo[3] = {s.q_lo_x, s.q_lo_y, s.q_lo_z}, qhi[3] = {s.q_hi_x, s.q_hi_y, s.q_hi_z};
    for (int a = 0; a < 3; ++a) {
      auto pair = [](uint32_t w, int k) { return f16_code((w >> (8 * k)) & 0xffu) | f16_code((w >> (8 * k + 8)) & 0xffu) << 16; };
      d.p[a][0] = pair(qlo[a], 0);
      d.p[a][1] = pair(qlo[a], 2);
      d.p[a][2] = pair(qhi[a], 0);
      d.p[a][3] = pair(qhi[a], 2);
    }
  }
  return upload(dst, v.data(), v.size() * sizeof(NodeF16));
}

int rt_scene_destroy(rt_scene_t s) {
  if (!s) return RT_OK;
  (void)hipSetDevice(s->device);
  (void)hipDeviceSynchronize();
  free_workspace(s);
  void* ptrs[] = {s->d_prims, s->d_nodes, s->d_mats, s->d_lights, s->d_tex, s->d_texels, s->d_ctl, s->d_tiles,
                  s->d_prim_refs, s->d_ref_boxes, s->d_spill, s->d_batch_ctr, s->d_fetch, s->d_keys,
                  s->d_prim_shade};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (s->h_flag) (void)hipHostFree(s->h_flag);
  if (s->d_tile_cost) (void)hipFree(s->d_tile_cost);
  if (s->h_tile_cost) (void)hipHostFree(s->h_tile_cost);
  if (s->h_stats) (void)hipHostFree(s->h_stats);
  hipEvent_t evs[] = {s->ev_t0, s->ev_t1, s->ev_fork, s->ev_join};
  for (hipEvent_t e : evs)
    if (e) (void)hipEventDestroy(e);
  for (int h = 0; h < kPipes; ++h) {
    for (int k = 0; k < kMaxHostBatch; ++k) {
      if (s->ev_a[h][k]) (void)hipEventDestroy(s->ev_a[h][k]);
      if (s->ev_b[h][k]) (void)hipEventDestroy(s->ev_b[h][k]);
    }
    if (s->aux[h]) (void)hipStreamDestroy(s->aux[h]);
  }
  delete s;
  return RT_OK;
}

int rt_scene_create(int32_t device, const rt_scene_desc* d, rt_scene_t* out) {
  knobs_refresh();
  if (!d || !out) return fail(RT_EINVAL, "rt_scene_create: null argument");
  if (d->n_prims < 0 || d->n_prims >= (1 << 24) || (d->n_prims > 0 && (!d->prims || !d->prim_refs)) ||
      (d->n_prims > d->n_unbounded && (d->n_nodes <= 0 || !d->nodes)) || d->n_unbounded < 0 ||
      d->n_unbounded > d->n_prims || (d->n_prims > 0 && (d->n_ref_leaves <= 0 || !d->ref_leaf_boxes)))
    return fail(RT_EINVAL, "rt_scene_create: inconsistent primitive/node arrays (at most 2^24 - 1 primitives)");
  if (d->n_nodes < 0 || d->n_nodes >= (1 << 26))
    return fail(RT_EINVAL, "rt_scene_create: at most 2^26 - 1 BVH4 nodes");
  if (d->prim_stride == 64 && (int64_t)d->n_nodes * 80 > (int64_t)INT32_MAX)  // 80-B device nodes, entries = byte offsets
    return fail(RT_EINVAL, "rt_scene_create: at most 26843545 BVH4 nodes in a planes-only scene");
  if (d->stack_bound < 1 || d->stack_bound > 4096) return fail(RT_EINVAL, "rt_scene_create: stack_bound out of range");
  if (d->prim_stride != 64 && d->prim_stride != 128)
    return fail(RT_EINVAL, "rt_scene_create: prim_stride must be 64 or 128");
  if (d->n_materials <= 0 || !d->materials) return fail(RT_EINVAL, "rt_scene_create: need >= 1 material");
  if (d->n_lights < 0 || d->n_lights > 65535 || (d->n_lights > 0 && !d->lights))
    return fail(RT_EINVAL, "rt_scene_create: bad lights (at most 65535)");
  // every node reference in range and pointing forward (the kernel follows them unchecked)
  const int64_t n_bounded = (int64_t)d->n_prims - d->n_unbounded;
  for (int32_t i = 0; i < d->n_nodes; ++i) {
    const rt_node4& nd = d->nodes[i];
    for (int k = 0; k < 4; ++k) {
      const uint32_t m = (nd.meta >> (8 * k)) & 0xffu;
      const int64_t c = nd.child[k];
      // leaf entries: 0x80000000 | first << 7 | count (first < 2^24), count == the meta byte's
      const uint32_t cu = (uint32_t)nd.child[k];
      const int64_t first = (int64_t)((cu & 0x7fffffffu) >> 7);
      const bool ok = (m == 0 && nd.child[k] == -1) || (m == 0x01u && c > i && c < d->n_nodes) ||
                      ((m & 0x80u) && (m & 0x7fu) != 0 && (cu & 0x80000000u) && (cu & 0x7fu) == (m & 0x7fu) &&
                       first + (m & 0x7fu) <= n_bounded);
      if (!ok) return fail(RT_EINVAL, "rt_scene_create: node child out of range");
    }
  }
  // RT_TAG_TRI1_NEVER changes what a[12] means (a squared radius, not c3.x): only on a valid
  // Plane record, with a finite non-negative radius
  bool moving = false;
  for (int32_t i = 0; i < d->n_prims; ++i) {
    const float* a = reinterpret_cast<const float*>(d->prims) + (size_t)i * (d->prim_stride / 4);
    uint32_t tag;
    std::memcpy(&tag, a + 15, 4);
    // (from the velocity itself, not the tag: a caller's untagged moving sphere still gets its time)
    moving = moving || (d->prim_stride == 128 && RT_TAG_KIND(tag) == RT_PRIM_SPHERE &&
                        (a[12] != 0.0f || a[13] != 0.0f || a[14] != 0.0f));
    if ((tag & RT_TAG_TRI1_NEVER) &&
        !(RT_TAG_KIND(tag) == RT_PRIM_PLANE && (tag & RT_TAG_PLANE_VALID) && std::isfinite(a[12]) && a[12] >= 0.0f))
      return fail(RT_EINVAL, "rt_scene_create: RT_TAG_TRI1_NEVER on a record that is not a valid Plane with a[12] >= 0");
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(RT_ENODEV, "rt_scene_create: no such HIP device");
  HIP_TRY(hipSetDevice(device), RT_EDEVICE);
  rt_scene_s* s = new rt_scene_s();
  s->device = device;
  s->desc = *d;
  // the kernel variants follow these flags (recursion frames, refraction): derived from the
  // materials here as well, so a caller's desc cannot select a variant that drops a path
  for (int i = 0; i < d->n_materials; ++i) {
    if (d->materials[i].reflectivity > 0.0f) s->desc.flags |= RT_SCENE_HAS_REFLECTION;
    if (d->materials[i].transparency > 0.0f) s->desc.flags |= RT_SCENE_HAS_REFRACTION;
    if (d->materials[i].texture >= 0) s->desc.flags |= RT_SCENE_HAS_TEXTURE;
  }
  for (int i = 0; i < d->n_lights; ++i) s->soft_lights = s->soft_lights || d->lights[i].radius > 0.0f;
  // fused shadow rays: scenes whose lights are all points (one shadow ray each, no random
  // draws), at most 24 of them (occlusion bits of one word); with transformed shapes only
  // untextured ones (the tracing lane computes the hit's point and normal, not its (u, v))
  s->fuse_lights = (d->prim_stride == 64 || !(s->desc.flags & RT_SCENE_HAS_TEXTURE)) && !s->soft_lights &&
                   d->n_lights >= 1 && d->n_lights <= 24 ? d->n_lights : 0;
  s->late_draws = s->soft_lights;
  s->moving = moving;
  for (int i = 0; i < d->n_materials; ++i) s->late_draws = s->late_draws || d->materials[i].roughness > 0.0f;
  // planes-only scenes: what the shading of a compact hit needs of its plane, 16 B per primitive --
  // the precomputed normal and the material index (record words 3, 7, 11 and the tag's bits)
  std::vector<float4> prim_shade;
  if (d->prim_stride == 64) {
    prim_shade.resize((size_t)d->n_prims);
    const float* P = reinterpret_cast<const float*>(d->prims);
    for (int32_t i = 0; i < d->n_prims; ++i) {
      const float* a = P + (size_t)i * 16;
      uint32_t tag;
      std::memcpy(&tag, a + 15, 4);
      const uint32_t mat = RT_TAG_MATERIAL(tag);
      float matf;
      std::memcpy(&matf, &mat, 4);
      prim_shade[i] = make_float4(a[3], a[7], a[11], matf);
    }
  }
  // the device copy of the materials: pad = kMatSpecSkip where shade's specular term is +-0 for
  // any hit (spec_zero); the caller's pad is ignored
  std::vector<rt_material> mats(d->materials, d->materials + d->n_materials);
  for (rt_material& m : mats)
    m.pad = m.specular[0] == 0.0f && m.specular[1] == 0.0f && m.specular[2] == 0.0f && m.shininess >= 0.0f &&
                    m.shininess <= 5e6f
                ? kMatSpecSkip
                : 0;
  int rc = RT_OK;
  if ((rc = upload(&s->d_prims, d->prims, (size_t)d->n_prims * d->prim_stride)) ||
      (rc = upload_nodes(&s->d_nodes, d->nodes, d->n_nodes, d->prim_stride == 64)) ||
      (rc = upload(&s->d_prim_refs, d->prim_refs, (size_t)d->n_prims * sizeof(rt_prim_ref))) ||
      (rc = upload((void**)&s->d_prim_shade, prim_shade.data(), prim_shade.size() * sizeof(float4))) ||
      (rc = upload(&s->d_ref_boxes, d->ref_leaf_boxes, (size_t)d->n_ref_leaves * 8 * sizeof(float))) ||
      (rc = upload(&s->d_mats, mats.data(), mats.size() * sizeof(rt_material))) ||
      (rc = upload(&s->d_lights, d->lights, (size_t)d->n_lights * sizeof(rt_light))) ||
      (rc = upload(&s->d_tex, d->textures, (size_t)d->n_textures * sizeof(rt_texture))) ||
      (rc = upload(&s->d_texels, d->texels, (size_t)d->n_texel_bytes))) {
    rt_scene_destroy(s);
    return rc;
  }
  bool ev_ok = true;
  for (int h = 0; h < kPipes && ev_ok; ++h) {
    for (int k = 0; k < kMaxHostBatch && ev_ok; ++k)
      ev_ok = hipEventCreate(&s->ev_a[h][k]) == hipSuccess && hipEventCreate(&s->ev_b[h][k]) == hipSuccess;
    ev_ok = ev_ok && (h == 0 || hipStreamCreateWithFlags(&s->aux[h], hipStreamNonBlocking) == hipSuccess);
  }
  if (!ev_ok || hipMalloc(&s->d_ctl, kCtlBytes) != hipSuccess ||
      hipHostMalloc((void**)&s->h_flag, (size_t)kPipes * kMaxHostBatch * kFetchStride * 4) != hipSuccess ||
      hipHostMalloc((void**)&s->h_stats, kStatsBytes) != hipSuccess ||
      hipMalloc(&s->d_batch_ctr, (size_t)kMaxBatchShards * kCtrStride * 4) != hipSuccess ||
      hipMalloc(&s->d_fetch, (size_t)kPipes * kFetchLines * kFetchStride * 4) != hipSuccess ||
      hipEventCreate(&s->ev_t0) != hipSuccess || hipEventCreate(&s->ev_t1) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming) != hipSuccess) {
    rt_scene_destroy(s);
    return fail(RT_ENOMEM, "rt_scene_create: control block / events");
  }
  {  // persistent trace grid: blocks resident per CU x CUs
    int ncu = 0, bpc = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) ncu = 256;
    const bool planes = d->prim_stride == 64;
    auto occupancy = [&](const void* fn, int waves, bool soft = false) {
      const int lds_entries = call_lds_entries(d->stack_bound, waves, soft);
      const size_t lds_bytes = (size_t)lds_entries * kBlock * 2 * sizeof(int);  // (entry, t_near) per stack slot
      int b = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, fn, kBlock, lds_bytes) != hipSuccess || b < 1) b = 2;
      b = std::min(b, (int)knob(K_TRACE_BPC, b));  // diagnostic cap
      return b;
    };
    bpc = occupancy(planes ? (const void*)trace_refill_kernel<false, true, false, false>
                           : (const void*)trace_refill_kernel<false, false, false, false>,
                    instance_waves(planes, false, false, false));
    s->trace_blocks_per_cu_fuse = occupancy(planes ? (const void*)trace_refill_kernel<false, true, true, false>
                                                   : (const void*)trace_refill_kernel<false, false, true, false>,
                                            instance_waves(planes, true, false, false));
    s->trace_blocks_per_cu_soft = occupancy(planes ? (const void*)trace_refill_kernel<false, true, false, true>
                                                   : (const void*)trace_refill_kernel<false, false, false, true>,
                                            instance_waves(planes, false, true, false), true);
    if (planes) {
      s->trace_blocks_per_cu_seven = occupancy((const void*)trace_refill_kernel<false, true, false, false, true, true>, 7);
      s->trace_blocks_per_cu_fuse_seven = occupancy((const void*)trace_refill_kernel<false, true, true, false, true, true>, 7);
    }

    s->n_cu = ncu;
    s->trace_blocks_per_cu = bpc;
  }
  {  // tile cost model: up to 64K primitive centres (planes: the mean of c0, c1, c2; transformed
     // shapes: the object-to-world translation)
    const int32_t n = d->n_prims;
    const int32_t stride = std::max(1, n / 65536);
    const float* P = reinterpret_cast<const float*>(d->prims);
    const size_t w = (size_t)d->prim_stride / 4;
    for (int32_t i = 0; i < n; i += stride) {
      const float* a = P + (size_t)i * w;
      uint32_t tag;
      std::memcpy(&tag, a + 15, 4);
      if (d->prim_stride == 64 || RT_TAG_KIND(tag) == RT_PRIM_PLANE) {
        s->cost_pts.push_back((a[0] + a[4] + a[8]) / 3.0f);
        s->cost_pts.push_back((a[1] + a[5] + a[9]) / 3.0f);
        s->cost_pts.push_back((a[2] + a[6] + a[10]) / 3.0f);
      } else {
        s->cost_pts.push_back(a[16 + 3]);
        s->cost_pts.push_back(a[16 + 7]);
        s->cost_pts.push_back(a[16 + 11]);
      }
    }
  }
  s->desc.prims = nullptr; s->desc.nodes = nullptr; s->desc.materials = nullptr; s->desc.prim_refs = nullptr;
  s->desc.ref_leaf_boxes = nullptr;
  s->desc.lights = nullptr; s->desc.textures = nullptr; s->desc.texels = nullptr;
  *out = s;
  return RT_OK;
}

int rt_tile_costs(rt_scene_t s, const rt_camera_desc* cam, int32_t tile_w, int32_t tile_h, float* costs_out) {
  if (!s || !cam || !costs_out) return fail(RT_EINVAL, "rt_tile_costs: null argument");
  if (tile_w <= 0 || tile_h <= 0) return fail(RT_EINVAL, "rt_tile_costs: tile size must be positive");
  if (cam->res_x <= 0 || cam->res_y <= 0) return fail(RT_EINVAL, "rt_tile_costs: camera resolution is 0");
  const int tiles_x = (cam->res_x + tile_w - 1) / tile_w, tiles_y = (cam->res_y + tile_h - 1) / tile_h;
  const std::vector<float>& cost = tile_costs(s, cam, tile_w, tile_h, tiles_x, tiles_y);
  std::memcpy(costs_out, cost.data(), cost.size() * sizeof(float));
  return RT_OK;
}

}  // extern "C"

// RT_DIAG on an instrumented (count_work) call, either path: shadow / other rays' box tests,
// node and prim-test lane utilisation, and the wave node visits whose lanes share one
// direction octant (control-block counters, trace_counters_out / node_visit)
static int print_work_diag(const unsigned int* ctl) {
  unsigned long long cnt[3] = {0, 0, 0};  // box tests, prim tests, rays (ctl bytes 16..)
  HIP_TRY(hipMemcpy(cnt, ctl + 4, sizeof(cnt), hipMemcpyDeviceToHost), RT_EDEVICE);
  unsigned long long dg[2] = {0, 0};
  HIP_TRY(hipMemcpy(dg, ctl + 128, sizeof(dg), hipMemcpyDeviceToHost), RT_EDEVICE);
  const unsigned long long cr = cnt[2] - dg[0], cb = cnt[0] - dg[1];
  std::fprintf(stderr, "[rt diag] shadow rays %llu: %.1f box tests/ray; other rays %llu: %.1f box tests/ray\n", dg[0],
               (double)dg[1] / (double)std::max(dg[0], 1ull), cr, (double)cb / (double)std::max(cr, 1ull));
  unsigned long long wv[3] = {0, 0, 0};  // lane node visits, wave node visits, wave prim tests (ctl bytes 488..)
  HIP_TRY(hipMemcpy(wv, ctl + 122, sizeof(wv), hipMemcpyDeviceToHost), RT_EDEVICE);
  unsigned long long uo = 0;  // wave node visits with one direction octant (ctl byte 472)
  HIP_TRY(hipMemcpy(&uo, ctl + 118, sizeof(uo), hipMemcpyDeviceToHost), RT_EDEVICE);
  std::fprintf(stderr, "[rt diag] node visits: %.2f/ray, lane utilisation %.3f; prim tests: %.2f/ray, lane utilisation %.3f; "
               "wave prim-test iterations per wave node visit %.2f; wave node visits with one octant %.3f\n",
               (double)wv[0] / (double)std::max(cnt[2], 1ull), (double)wv[0] / (64.0 * (double)std::max(wv[1], 1ull)),
               (double)cnt[1] / (double)std::max(cnt[2], 1ull), (double)cnt[1] / (64.0 * (double)std::max(wv[2], 1ull)),
               (double)wv[2] / (double)std::max(wv[1], 1ull), (double)uo / (double)std::max(wv[1], 1ull));
  return RT_OK;
}

// Finishes the scene's enqueued one-pass call: waits for its last event, records its measured
// tile costs (instrumented calls) and fills `stats` (may be null).
static int finish_one_pass(rt_scene_s* s, rt_stats* stats) {
  rt_scene_s::Pending& q = s->pending;
  if (!q.active) {
    if (stats) *stats = rt_stats{};
    return RT_OK;
  }
  q.active = false;
  HIP_TRY(hipSetDevice(s->device), RT_EDEVICE);
  HIP_TRY(hipEventSynchronize(s->ev_t1), RT_EDEVICE);
  if (q.measure_tiles) {  // measured tile costs, by tile id (render-order index i holds tile tl_dev[i])
    if (s->meas_key != q.meas_key) {
      s->meas_key = q.meas_key;
      s->meas_visits.assign((size_t)q.tiles_x * q.tiles_y, -1.0f);
    }
    for (int i = 0; i < q.n_tiles; ++i) s->meas_visits[(size_t)q.tl_dev[i]] = (float)s->h_tile_cost[2 * i];
  }
  float ms = 0.f, t_a = 0.f, t_b = 0.f, k_ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, s->ev_a[0][0], s->ev_b[0][0]), RT_EDEVICE);
  if (kDiagBuild) {
    diag_after_launch(q.ta, ms, 0);
    diag_after_call(q.ta.counters, true);
  }
  s->last_iters = 1;
  if (q.count_work && knob(K_DIAG, 0) != 0)
    if (const int rc = print_work_diag((const unsigned int*)s->d_ctl)) return rc;
  if (!stats) return RT_OK;
  *stats = rt_stats{};
  const unsigned long long* h = s->h_stats;
  HIP_TRY(hipEventElapsedTime(&k_ms, s->ev_t0, s->ev_t1), RT_EDEVICE);
  HIP_TRY(hipEventElapsedTime(&t_a, s->ev_t0, s->ev_a[0][0]), RT_EDEVICE);
  HIP_TRY(hipEventElapsedTime(&t_b, s->ev_t0, s->ev_b[0][0]), RT_EDEVICE);
  stats->rays = h[4];  // ctl bytes 16, 24, 32: box tests, prim tests, rays
  stats->box_tests = h[2];
  stats->prim_tests = h[3];
  stats->kernel_ms = k_ms;
  stats->trace_ms = ms;
  stats->trace_busy_ms = t_b - t_a;
  stats->iterations = 1;
  stats->path = RT_PATH_ONE_PASS;
  stats->node_visits = q.count_work ? h[61] : 0;
  return RT_OK;
}

// One-pass calls: camera_kernel -> one trace launch -> shade_reduce_kernel, slot == unit and no
// slot state.  The scene must need nothing between a sample's camera ray and its colour but the
// closest hit and one shadow ray per light, traced by the tracing lane: no Trace recursion
// (reflection / refraction), lights all points (the fused shadow rays: at most 24) or none,
// and the hit's (u, v) from the trace kernel (planes) or no texture.  RT_ONE_PASS=0 selects the
// step pipeline for every call, and nothing else does: the step pipeline's own knobs (RT_SLOTS,
// RT_PIPES, RT_FUSE) and its per-step log (RT_DIAG) do not apply to a one-pass call, which ignores
// them and says so once per process (note_ignored_knobs).
static bool one_pass_scene(const rt_scene_s* s) {
  const bool frames = (s->desc.flags & (RT_SCENE_HAS_REFLECTION | RT_SCENE_HAS_REFRACTION)) != 0;
  const bool tex = (s->desc.flags & RT_SCENE_HAS_TEXTURE) != 0;
  return !frames && !s->soft_lights && (s->desc.n_lights == 0 || s->fuse_lights == s->desc.n_lights) &&
         (s->desc.prim_stride == 64 || !tex);
}
static bool one_pass_env() { return knob(K_ONE_PASS, 1) != 0; }
static void note_ignored_knobs() {
  static std::atomic<bool> said[4] = {};
  static const Knob knobs[4] = {K_SLOTS, K_PIPES, K_FUSE, K_DIAG};
  for (int k = 0; k < 4; ++k)
    if (knob_set(knobs[k]) && !said[k].exchange(true))
      std::fprintf(stderr, "librt_hip: %s applies to the step pipeline only; one-pass calls ignore it "
                   "(RT_ONE_PASS=0 selects the step pipeline)\n", kKnobDefs[knobs[k]].name);
}
// units of one one-pass call (larger calls run as tile chunks): 52 B of workspace per unit
// touched (query direction 12, result 4, hit record 32 on a hit, occlusion bits 4)
static long long one_pass_cap() { return knob(K_ONE_PASS_MAX, 1LL << 30); }

extern "C" {

int rt_render_wait(rt_scene_t s, rt_stats* stats) {
  if (!s) return fail(RT_EINVAL, "rt_render_wait: null scene");
  if (!s->pending.active && s->held) {  // a sync == 0 call that had completed already
    s->held = false;
    if (stats) *stats = s->held_stats;
    return RT_OK;
  }
  return finish_one_pass(s, stats);
}

int rt_tile_costs_measured(rt_scene_t s, const rt_camera_desc* cam, int32_t tile_w, int32_t tile_h, int32_t spp_sqrt,
                           float* costs_out) {
  if (!s || !cam || !costs_out) return fail(RT_EINVAL, "rt_tile_costs_measured: null argument");
  if (tile_w <= 0 || tile_h <= 0) return fail(RT_EINVAL, "rt_tile_costs_measured: tile size must be positive");
  if (cam->res_x <= 0 || cam->res_y <= 0) return fail(RT_EINVAL, "rt_tile_costs_measured: camera resolution is 0");
  const int tiles_x = (cam->res_x + tile_w - 1) / tile_w, tiles_y = (cam->res_y + tile_h - 1) / tile_h;
  const int n_samples = spp_sqrt <= 1 ? 1 : spp_sqrt * spp_sqrt;
  const bool have = s->meas_key == meas_key_of(cam, tile_w, tile_h, n_samples);
  for (int i = 0; i < tiles_x * tiles_y; ++i) costs_out[i] = have ? s->meas_visits[(size_t)i] : -1.0f;
  return RT_OK;
}

}  // extern "C"

static int render_tiles(rt_scene_t s, const rt_camera_desc* cam, const rt_render_params* p, const int32_t* tile_ids,
                        int32_t n_tiles, int32_t tile_w, int32_t tile_h, float* d_out, void* stream_ptr, rt_stats* stats,
                        const uint64_t* seeds, int n_frames);

extern "C" {

// A call with sync == 0 is finished by rt_render_wait, whichever path ran: a deferred one-pass
// call is waited for there; a call that completed before returning (the step pipeline, tile
// chunks) leaves its statistics for it (held), so the caller's wait never reads zeros.  The
// statistics are gathered only when someone reads them: the caller (stats) or that wait.
static int render_entry(rt_scene_t s, const rt_camera_desc* cam, const rt_render_params* p, const int32_t* tile_ids,
                        int32_t n_tiles, int32_t tile_w, int32_t tile_h, float* d_out, void* stream_ptr, rt_stats* stats,
                        const uint64_t* seeds, int n_frames) {
  knobs_refresh();
  if (s) s->held = false;
  rt_stats st{};
  const bool want = stats || (p && p->sync == 0);
  const int rc = render_tiles(s, cam, p, tile_ids, n_tiles, tile_w, tile_h, d_out, stream_ptr, want ? &st : nullptr,
                              seeds, n_frames);
  if (rc == RT_OK && p->sync == 0 && !s->pending.active) {
    s->held = true;
    s->held_stats = st;
  }
  if (stats) *stats = st;
  return rc;
}

int rt_render_tiles(rt_scene_t s, const rt_camera_desc* cam, const rt_render_params* p, const int32_t* tile_ids,
                    int32_t n_tiles, int32_t tile_w, int32_t tile_h, float* d_out, void* stream_ptr,
                    rt_stats* stats) {
  return render_entry(s, cam, p, tile_ids, n_tiles, tile_w, tile_h, d_out, stream_ptr, stats, nullptr, 1);
}

int rt_render_frames(rt_scene_t s, const rt_camera_desc* cam, const rt_render_params* p, const uint64_t* seeds,
                     int32_t n_frames, const int32_t* tile_ids, int32_t n_tiles, int32_t tile_w, int32_t tile_h,
                     float* d_out, void* stream_ptr, rt_stats* stats) {
  if (n_frames < 1 || n_frames > kMaxFrames || !seeds)
    return fail(RT_EINVAL, "rt_render_frames: need 1.." + std::to_string(kMaxFrames) + " frames and their seeds");
  return render_entry(s, cam, p, tile_ids, n_tiles, tile_w, tile_h, d_out, stream_ptr, stats, seeds, n_frames);
}

}  // extern "C"

static void add_stats(rt_stats& acc, const rt_stats& st) {
  acc.rays += st.rays;
  acc.box_tests += st.box_tests;
  acc.prim_tests += st.prim_tests;
  acc.node_visits += st.node_visits;
  acc.kernel_ms += st.kernel_ms;
  acc.trace_ms += st.trace_ms;
  acc.trace_busy_ms += st.trace_busy_ms;
  acc.iterations += st.iterations;
  if (st.path != RT_PATH_ONE_PASS) acc.path = RT_PATH_STEPS;
}

static int render_tiles(rt_scene_t s, const rt_camera_desc* cam, const rt_render_params* p, const int32_t* tile_ids,
                        int32_t n_tiles, int32_t tile_w, int32_t tile_h, float* d_out, void* stream_ptr,
                        rt_stats* stats, const uint64_t* seeds, int n_frames) {
  if (!s || !cam || !p || (!tile_ids && n_tiles > 0) || !d_out) return fail(RT_EINVAL, "rt_render_tiles: null argument");
  if (tile_w <= 0 || tile_h <= 0 || tile_w % 8 || tile_h % 8)
    return fail(RT_EINVAL, "rt_render_tiles: tile size must be a positive multiple of 8");
  if (cam->res_x <= 0 || cam->res_y <= 0) return fail(RT_EINVAL, "rt_render_tiles: camera resolution is 0");
  if (p->spp_sqrt > 4096 || p->light_samples < 0 || p->light_samples > 65535)
    return fail(RT_EINVAL, "rt_render_tiles: bad sample counts (light_samples at most 65535)");
  const int tiles_x = (cam->res_x + tile_w - 1) / tile_w, tiles_y = (cam->res_y + tile_h - 1) / tile_h;
  for (int i = 0; i < n_tiles; ++i)
    if (tile_ids[i] < 0 || tile_ids[i] >= tiles_x * tiles_y) return fail(RT_EINVAL, "rt_render_tiles: tile id out of range");
  if (s->pending.active)  // the scene's deferred call finishes first (its workspace is reused)
    if (const int rc = finish_one_pass(s, nullptr)) return rc;
  if (stats) *stats = rt_stats{};
  if (n_tiles == 0) return RT_OK;
  rt_render_params pf = *p;  // a multi-frame call's single frames: params with the frame's seed
  std::vector<int32_t> frame_list;  // a multi-frame call's tile list: the frames' lists end to end
  const int frame_tiles = n_tiles;
  {  // calls larger than the unit cap run as consecutive tile chunks (same pixels: the counter
     // RNG keys every sample by pixel, so the split changes no value); the per-sample colour
     // buffer (12 B per unit) stays bounded, and the frame-wide 2^31 unit limit goes away
    const long long per_tile = (long long)tile_w * tile_h * (p->spp_sqrt <= 1 ? 1LL : (long long)p->spp_sqrt * p->spp_sqrt);
    long long cap = 1LL << 30;
    cap = knob(K_MAX_UNITS, cap);
    const bool op = one_pass_scene(s) && one_pass_env();
    if (op) cap = std::min(cap, one_pass_cap());
    const size_t frame_floats = (size_t)n_tiles * tile_w * tile_h * 3;
    if (n_frames > 1) {
      // Multi-frame calls (rt_render_frames): a one-pass scene renders as many frames per pass as
      // the unit cap holds -- every one of their samples in one camera pass, one traversal launch
      // and one shading pass, so a rank's share of a split frame runs launches of the whole
      // frame's size.  The step pipeline renders the frames one after another.
      const int per_pass = op ? (int)std::max(1LL, std::min<long long>(n_frames, cap / ((long long)n_tiles * per_tile))) : 1;
      if (per_pass < n_frames) {
        rt_stats acc{};
        acc.path = RT_PATH_ONE_PASS;
        rt_render_params pc = *p;
        pc.sync = 1;  // the passes share the workspace: each one finishes before the next
        for (int f0 = 0; f0 < n_frames; f0 += per_pass) {
          const int nf = std::min(per_pass, n_frames - f0);
          rt_stats st{};
          pc.seed = seeds[f0];
          const int rc = render_tiles(s, cam, &pc, tile_ids, n_tiles, tile_w, tile_h, d_out + (size_t)f0 * frame_floats,
                                      stream_ptr, stats ? &st : nullptr, seeds + f0, nf);
          if (rc) return rc;
          add_stats(acc, st);
        }
        if (stats) *stats = acc;
        return RT_OK;
      }
      frame_list.resize((size_t)n_frames * n_tiles);
      for (int f = 0; f < n_frames; ++f) std::copy(tile_ids, tile_ids + n_tiles, frame_list.begin() + (size_t)f * n_tiles);
      tile_ids = frame_list.data();
      n_tiles *= n_frames;
    } else if (seeds) {
      pf.seed = seeds[0];
      p = &pf;
    }
    if (n_frames == 1 && n_tiles > 1 && (long long)n_tiles * per_tile > cap) {
      const int k = (int)std::max(1LL, std::min<long long>(n_tiles, cap / per_tile));
      rt_stats acc{};
      acc.path = RT_PATH_ONE_PASS;
      rt_render_params pc = *p;
      pc.sync = 1;  // chunks share the workspace: each one finishes before the next
      for (int t0 = 0; t0 < n_tiles; t0 += k) {
        rt_stats st{};
        const int rc = render_tiles(s, cam, &pc, tile_ids + t0, std::min(k, n_tiles - t0), tile_w, tile_h,
                                    d_out + (size_t)t0 * tile_w * tile_h * 3, stream_ptr, stats ? &st : nullptr,
                                    nullptr, 1);
        if (rc) return rc;
        add_stats(acc, st);
      }
      if (stats) *stats = acc;
      return RT_OK;
    }
  }
  if (n_frames > 1 && p->count_work)
    return fail(RT_EINVAL, "rt_render_frames: instrumented (count_work) calls render one frame");
  const long long n_pixels_ll = (long long)n_tiles * tile_w * tile_h;
  if (n_pixels_ll > 0x7fffffffLL) return fail(RT_EINVAL, "rt_render_tiles: too many pixels in one call");
  const int n_pixels = (int)n_pixels_ll;
  HIP_TRY(hipSetDevice(s->device), RT_EDEVICE);
  hipStream_t stream = (hipStream_t)stream_ptr;

  // ---- workspace
  const bool need_frames = (s->desc.flags & (RT_SCENE_HAS_REFLECTION | RT_SCENE_HAS_REFRACTION)) != 0;
  const bool need_refr = (s->desc.flags & RT_SCENE_HAS_REFRACTION) != 0;
  const bool planes_only = s->desc.prim_stride == 64;
  const int n_samples = p->spp_sqrt <= 1 ? 1 : p->spp_sqrt * p->spp_sqrt;
  const long long n_units = (long long)n_pixels * n_samples;
  if (n_units > 0x7ffffff0LL) return fail(RT_EINVAL, "rt_render_tiles: too many samples in one call (split the tiles)");
  // whole blocks of slots; a wave renders 64 consecutive samples per batch
  // Slots in flight (r03 sweep with one pipeline and drain helpers, one box; Mrays/s): every
  // sample of a call of at most 128M units -- the whole headline frame (105M: 32M 6167, 48M
  // 6263, 64M 6184, all 6319) or one rank's half of it (52M: 32M 5885, all 6225) -- else 128M
  // (C5 1.07G units: 96M 7666, 128M 7703, 192M 7705); scenes with reflection / refraction keep
  // 16M (C4: 8M 13043, 16M 13065, 32M 12791: their slots carry the Trace frames and take many
  // short steps) -- since r05 6M in two slot pipelines (below), since r06 8M (with the
  // few-primitive leaf item a C4 trace launch is 15 % shorter and the pipelines want more slots
  // per step: same box, 3 reps, 6M 15,829-15,836 Mrays/s, 7M 15,686-15,893, 8M 15,917-15,975,
  // 10M 15,926-15,959, profiles/r06q_c4_slots.txt).  ~180 B of HBM per slot: 128M slots ~23 GB.
  const bool frames_scene = (s->desc.flags & (RT_SCENE_HAS_REFLECTION | RT_SCENE_HAS_REFRACTION)) != 0;
  const bool tex_scene = (s->desc.flags & RT_SCENE_HAS_TEXTURE) != 0;
  const bool one_pass = one_pass_scene(s) && one_pass_env() && n_units <= one_pass_cap();
  if (one_pass) note_ignored_knobs();
  long long slots = frames_scene ? std::min(n_units, 8LL << 20) : std::min(n_units, 128LL << 20);
  slots = knob(K_SLOTS, slots);
  // slot-state words are addressed S[field * N + slot] in 32-bit int: (highest field + 1) * N
  // <= 2^31.  Scenes without Trace frames touch fields up to F_RAY + 2 (the ray origin), scenes
  // with frames all F_COUNT; RT_SLOTS is clamped to that bound (one-pass calls keep no slot
  // state and address their arrays with 64-bit offsets)
  static_assert((long long)(F_RAY + 3) * (128LL << 20) <= (1LL << 31), "default slot cap overflows the state index");
  static_assert((long long)F_COUNT * (16LL << 20) <= (1LL << 31), "frames-scene slot cap overflows the state index");
  slots = std::min(slots, ((1LL << 31) / (frames_scene ? F_COUNT : F_RAY + 3)) / kBlock * kBlock);
  if (one_pass) slots = n_units;  // every unit its own slot
  const int n_slots = (int)(((std::min<long long>(n_units, slots) + kBlock - 1) / kBlock) * kBlock);
  if ((size_t)n_tiles > s->tiles_cap) {  // render-order tile ids, then their output positions
    if (s->d_tiles) (void)hipFree(s->d_tiles);
    s->d_tiles = nullptr;
    s->tiles_cap = 0;
    s->tiles_on_device.clear();
    HIP_TRY(hipMalloc(&s->d_tiles, (size_t)n_tiles * 2 * sizeof(int32_t)), RT_ENOMEM);
    s->tiles_cap = (size_t)n_tiles;
  }
  // one-pass query record: the fields the call needs (LogicArgs::op_fo / op_ft / op_fk)
  int op_fields = 3, op_fo = -1, op_ft = -1, op_fk = -1;
  if (one_pass) {
    if (cam->aperture > 0.0f) op_fo = op_fields, op_fields += 3;  // thin lens: the origin
    // the ray time: only a moving sphere reads it (every other primitive, a static sphere included,
    // gives the same bits for any time >= 0: its velocity terms are +-0), and it is the sample's
    // last draw in a one-pass call -- so scenes without one skip the draw and its 4 B per unit
    // (r06: C3's camera rays)
    if (!planes_only && s->moving) op_ft = op_fields++;
    bool edge = false;  // some tile reaches past the image: its outside units are marked in a kind word
    for (int i = 0; i < n_tiles && !edge; ++i)
      edge = ((tile_ids[i] % tiles_x) + 1) * tile_w > cam->res_x || ((tile_ids[i] / tiles_x) + 1) * tile_h > cam->res_y;
    if (edge) op_fk = op_fields++;
  }
  {
    const size_t N = (size_t)std::max(n_slots, 1);
    int rc = RT_OK;
    if ((rc = grow(s->d_query, s->cap_query, N * (one_pass ? op_fields : Q_COUNT) * 4)) ||
        (rc = grow(s->d_result, s->cap_result, N * 4)) ||
        (rc = grow(s->d_hit, s->cap_hit, N * HIT_STRIDE * 4)) ||
        (tex_scene && (rc = grow(s->d_hit_uv, s->cap_hit_uv, N * sizeof(float2)))) ||
        (s->fuse_lights > 0 && (rc = grow(s->d_occl, s->cap_occl, N * 4))))
      return rc;
    if (!one_pass) {  // the step pipeline's slot state, Trace frames and per-sample colours
      if ((rc = grow(s->d_state, s->cap_state, N * F_COUNT * 4)) ||
          (rc = grow(s->d_wave_done, s->cap_wave_done, (N / 64 + 1) * 4)) ||
          (need_frames && (rc = grow(s->d_frames, s->cap_frames, N * kMaxDepth * FR_COUNT * 4))) ||
          (need_refr && (rc = grow(s->d_refr, s->cap_refr, N * kMaxDepth * 6 * 4))) ||
          (rc = grow(s->d_samples, s->cap_samples, (size_t)n_units * 3 * sizeof(float))))
        return rc;
    }
  }
  // render order and the tile list in that order + output positions; uploaded only when it
  // changed (a renderer's frames reuse one list).  Costliest tiles first for a call whose
  // samples are all in flight at once (one step per pipeline: one rank's share of a split
  // frame), where the call's last drain is exposed: one rank's eighth of the headline frame
  // 4509-4564 -> 4723-4727 Mrays/s.  Longer calls keep the caller's order (whole frames,
  // C4, C5: within -1.6 %..+0 % -- the other pipeline hides their drains).
  std::vector<int32_t> order;
  tile_cost_order(s, cam, tile_w, tile_h, tiles_x, tiles_y, tile_ids, n_tiles, n_units <= n_slots, order);
  std::vector<int32_t> tl_dev((size_t)n_tiles * 2);
  bool identity = true;
  for (int i = 0; i < n_tiles; ++i) {
    tl_dev[i] = tile_ids[order[i]];
    tl_dev[(size_t)n_tiles + i] = order[i];
    identity = identity && order[i] == i;
  }
  if (s->tiles_on_device != tl_dev) {
    s->tiles_on_device = tl_dev;
    HIP_TRY(hipMemcpyAsync(s->d_tiles, s->tiles_on_device.data(), tl_dev.size() * sizeof(int32_t),
                           hipMemcpyHostToDevice, stream), RT_EDEVICE);
  }
  unsigned int* ctl = (unsigned int*)s->d_ctl;  // cleared by init_kernel

  LogicArgs la{};
  Common c{};
  c.prims = (const float4*)s->d_prims;
  c.prim_stride4 = s->desc.prim_stride / 16;
  c.n_prims = s->desc.n_prims;
  c.nodes = (const float4*)s->d_nodes;
  c.use_bvh = p->use_bvh;
  c.eps_abs = 1e-5f * (s->desc.scene_scale > 1.0f ? s->desc.scene_scale : 1.0f);
  la.c = c;
  la.mats = (const rt_material*)s->d_mats;
  la.prim_shade = s->d_prim_shade;
  la.lights = (const rt_light*)s->d_lights;
  la.n_lights = s->desc.n_lights;
  la.textures = (const rt_texture*)s->d_tex;
  la.texels = (const uint8_t*)s->d_texels;
  la.cam = *cam;
  la.spp_sqrt = p->spp_sqrt;
  la.fd_s = make_fastdiv((uint32_t)std::max(1, p->spp_sqrt));
  la.inv_s = 1.0 / (double)std::max(1, p->spp_sqrt);
  {  // volatile: the correctly rounded reciprocals of the host's IEEE division
    volatile float rx = (float)cam->res_x, ry = (float)cam->res_y;
    la.inv_res_x = 1.0f / rx;
    la.inv_res_y = 1.0f / ry;
  }
  la.light_samples = p->light_samples;
  la.seed_key = mix64_host(p->seed + 0x9E3779B97F4A7C15ull);
  la.n_frames = n_frames;
  la.fd_frame_tiles = make_fastdiv((uint32_t)frame_tiles);
  la.seed_keys = nullptr;
  if (n_frames > 1) {  // frame f's key, as a single-frame call with seed seeds[f] derives it
    std::vector<uint64_t> keys((size_t)n_frames);
    for (int f = 0; f < n_frames; ++f) keys[f] = mix64_host(seeds[f] + 0x9E3779B97F4A7C15ull);
    if (keys.size() * 8 > s->cap_keys) s->keys_on_device.clear();
    if (const int rc = grow(s->d_keys, s->cap_keys, keys.size() * 8)) return rc;
    if (s->keys_on_device != keys) {
      s->keys_on_device = keys;
      HIP_TRY(hipMemcpyAsync(s->d_keys, s->keys_on_device.data(), keys.size() * 8, hipMemcpyHostToDevice, stream),
              RT_EDEVICE);
    }
    la.seed_keys = s->d_keys;
  }
  la.tile_ids = s->d_tiles;
  la.tile_out = identity ? nullptr : s->d_tiles + n_tiles;
  // affine tile lists (one GPU: 0, 1, 2 ...; round-robin ranks: r, r + N ...) need no lookup
  la.tile_first = tl_dev[0];
  la.tile_step = n_tiles > 1 ? tl_dev[1] - tl_dev[0] : 1;
  la.tile_affine = 1;
  for (int i = 0; i < n_tiles && la.tile_affine; ++i) la.tile_affine = tl_dev[i] == la.tile_first + i * la.tile_step;
  la.tile_w = tile_w;
  la.tile_h = tile_h;
  la.tiles_x = tiles_x;
  la.sub_x = tile_w / 8;
  la.fd_tile_px = make_fastdiv((uint32_t)(tile_w * tile_h));
  la.fd_sub_x = make_fastdiv((uint32_t)la.sub_x);
  la.fd_tiles_x = make_fastdiv((uint32_t)tiles_x);
  la.n_pixels = n_pixels;
  la.n_samples = n_samples;
  la.fd_samples = make_fastdiv((uint32_t)n_samples);
  la.n_units = n_units;
  la.samples = s->d_samples;
  la.out = d_out;
  la.n_slots = n_slots;
  la.state = s->d_state;
  la.frames = s->d_frames;
  la.refr = s->d_refr;
  la.query = s->d_query;
  la.result = s->d_result;
  la.hit = s->d_hit;
  la.hit_uv = s->d_hit_uv;
  la.late_draws = s->late_draws ? 1 : 0;
  la.pinhole = cam->aperture <= 0.0f ? 1 : 0;
  // Soft-light shadow samples after a light's first: drawn and traced by the lane that traced
  // the previous one (kSoft trace launches, default), or advanced by shadow_step_kernel
  // (RT_SOFT_FUSE=0), or by the logic kernel itself (RT_SOFT_FUSE=0 RT_SHADOW_STEP=0)
  const bool soft_scene = s->soft_lights && p->light_samples > 1;
  bool soft_trace = soft_scene;
  soft_trace = soft_trace && knob(K_SOFT_FUSE, 1) != 0;
  la.multi_shadow = soft_scene && !soft_trace ? 1 : 0;
  la.multi_shadow = la.multi_shadow && knob(K_SHADOW_STEP, 1) != 0;
  la.wave_done = s->d_wave_done;
  la.batch_ctr = s->d_batch_ctr;
  // every shard needs a slot-wave to drain it (wave w claims from shard w % batch_shards)
  la.batch_shards = std::max(1, std::min(batch_shards_env(), n_slots / 64));  // counters set by init_kernel

  TraceArgs ta{};
  ta.c = c;
  ta.prim_refs = (const int2*)s->d_prim_refs;
  ta.ref_boxes = (const float4*)s->d_ref_boxes;
  ta.n_unbounded = s->desc.n_unbounded;
  ta.n_nodes = s->desc.n_nodes;
  ta.query = s->d_query;
  ta.result = s->d_result;
  ta.hit = s->d_hit;
  ta.hit_uv = s->d_hit_uv;
  ta.has_tex = (s->desc.flags & RT_SCENE_HAS_TEXTURE) != 0 ? kHitTex : kHitRecord;
  ta.fetch_shards = fetch_shards_env();
  ta.xcd_chunk = RT_XCD_CHUNK_DEFAULT;
  ta.xcd_chunk = (int)knob(K_XCD_CHUNK, ta.xcd_chunk) & ~3;  // at most 2^20: 32-bit group indices
  ta.wave_done = s->d_wave_done;
  ta.rays = (unsigned long long*)(ctl + 8);  // byte 32
  ta.n_slots = n_slots;
  ta.lds_entries = call_lds_entries(s->desc.stack_bound, 6, false);  // set again below (instance)
  // the refill kernel's leaf items hold first << 7 in 31 bits
  ta.refill_min = refill_min_env();
  ta.leaf_min = leaf_min_env();
  ta.diag = knob(K_DIAG, 0) != 0 ? 1 : 0;
  // free lanes help the queries still traversing once a launch's queue is dry (RT_DRAIN_HELP=0 off)
  // The instrumented (count_work) frame runs without helpers: a helper searches a subtree under
  // a bound that lags its owner's, so its visits depend on scheduling; without them the counts
  // are the serial near-first traversal's (the algorithmic bytes bench.py reports)
  ta.drain_help = p->count_work ? 0 : 1;
  ta.drain_help = (int)knob(K_DRAIN_HELP, ta.drain_help);
  ta.lights = (const rt_light*)s->d_lights;
  ta.state = s->d_state;
  {  // few-primitive scenes test every bounded primitive instead of traversing (r06: a root node
     // and postponed leaves cost more than the few tests, and the lanes stay together)
    const int n_bounded = s->desc.n_prims - s->desc.n_unbounded;
    const bool flat = p->use_bvh && n_bounded > 0 && n_bounded <= std::min(127, (int)knob(K_FLAT_PRIMS, kFlatPrims));
    ta.root_item = flat ? (int)(0x80000000u | (uint32_t)n_bounded)  // a leaf item: kLeafBit | first 0 << 7 | count
                   : (s->desc.n_prims > 0 && p->use_bvh && s->desc.n_nodes > 0) ? 0 : -1;
  }
  // ... and on the step pipeline (no textures) the logic step answers the queries it emits itself
  // (kInline logic instances, r06; RT_FLAT_RENDER=0: every query through the traversal launches;
  // the instrumented frame keeps them for its counts)
  const bool flat_item = ta.root_item < 0 && ta.root_item != kNoItem;
  la.prim_refs = ta.prim_refs;
  la.ref_boxes = ta.ref_boxes;
  la.n_unbounded = ta.n_unbounded;
  la.rays = ta.rays;
  la.flat_n = flat_item ? (int)((uint32_t)ta.root_item & 0x7fu) : 0;
  const bool inline_queries = !one_pass && flat_item && !p->count_work && knob(K_FLAT_RENDER, 1) != 0 &&
                              (s->desc.flags & RT_SCENE_HAS_TEXTURE) == 0;  // (launch_logic2: untextured instances)
  for (int k = 0; k < 3; ++k) ta.cam_loc[k] = cam->location[k];
  ta.light_samples = p->light_samples;
  // the closest hit starts its shade loop in the tracing lane too: planes, or untextured
  // transformed shapes (that lane computes point and normal, not (u, v)); RT_SOFT_START=0 off
  ta.soft_start = soft_trace && s->desc.n_lights >= 1 && (planes_only || !(s->desc.flags & RT_SCENE_HAS_TEXTURE)) ? 1 : 0;
  ta.soft_start = ta.soft_start && knob(K_SOFT_START, 1) != 0;
  ta.frames = need_frames ? 1 : 0;
  ta.pinhole = cam->aperture <= 0.0f ? 1 : 0;
  // Fused shadow rays halve the steps of a sample.  They pay when the call is small (at most
  // two slot loads of samples: one rank's share of a split frame; each launch ends in a drain
  // of ~0.45 ms whatever its size) and when the scene has few primitives (its frame is spent
  // in the per-step passes over the slots); on a whole frame of a large scene the lanes'
  // camera and shadow rays interleave within a wave and lose coherence (headline -6.5 %).
  // RT_FUSE=0 / 1 overrides (1: whenever the scene allows it).
  ta.n_fuse = n_units <= 2LL * n_slots || s->desc.n_prims < kFuseFewPrims ? s->fuse_lights : 0;
  if (knob_set(K_FUSE) && !one_pass)  // (a one-pass call traces every point light's shadow ray fused)
    ta.n_fuse = knob(K_FUSE, 0) != 0 ? s->fuse_lights : 0;
  // the launched instance (launch_trace3): fused, soft or plain, at instance_waves() waves/SIMD
  // with default_stack() LDS rows (7 / 11 for whole planes-only frames, 5 / 16 for soft-light
  // chains over transformed shapes, else 6 / 12)
  ta.one_pass = one_pass ? 1 : 0;
  ta.tile_cost = nullptr;
  const bool measure_tiles = one_pass && p->count_work;
  if (measure_tiles) {  // the per-tile node visits later calls of this camera order their tiles by
    if (const int rc = grow(s->d_tile_cost, s->cap_tile_cost, (size_t)n_tiles * 8)) return rc;
    if ((size_t)n_tiles * 8 > s->cap_h_tile_cost) {
      if (s->h_tile_cost) (void)hipHostFree(s->h_tile_cost);
      s->h_tile_cost = nullptr;
      s->cap_h_tile_cost = 0;
      HIP_TRY(hipHostMalloc((void**)&s->h_tile_cost, (size_t)n_tiles * 8), RT_ENOMEM);
      s->cap_h_tile_cost = (size_t)n_tiles * 8;
    }
    ta.tile_cost = s->d_tile_cost;
    ta.fd_tile_units = make_fastdiv((uint32_t)(tile_w * tile_h * n_samples));
  }
  ta.op_fo = op_fo;
  ta.op_ft = op_ft;
  ta.op_fk = op_fk;
  la.op_fo = op_fo;
  la.op_ft = op_ft;
  la.op_fk = op_fk;
  const bool fuse_launch = ta.n_fuse > 0 || (one_pass && !planes_only), soft_launch = !fuse_launch && soft_trace;
  // Seven waves per SIMD (11 LDS stack entries) for the planes instances of synchronous calls of
  // more than 32M units -- whole frames (r05, same box: headline +2.9 %, C5 +2.8 %, their 12 / 10
  // spilled VGPRs outside the node visit); a deferred call (another frame in flight: one rank's
  // eighth -2.6 %) and smaller calls keep six.  RT_TRACE_SEVEN=0 / 1 overrides (1: every planes
  // call but soft-light and instrumented ones).
  bool seven = planes_only && !soft_launch && !p->count_work && p->sync != 0 && n_units > (32LL << 20);
  if (knob_set(K_TRACE_SEVEN)) seven = planes_only && !soft_launch && !p->count_work && knob(K_TRACE_SEVEN, 0) != 0;
  // the 7-wave instances have the default loop parameters built in: another stack depth
  // (RT_LDS_STACK) or threshold (RT_REFILL, RT_LEAF_MIN) takes the 6-wave runtime-knob ones (a
  // shallow tree keeps the default rows, call_lds_entries, and so keeps seven)
  if (seven && (call_lds_entries(s->desc.stack_bound, 7, false) != kSevenStack || ta.refill_min != kRefillDefault ||
                ta.leaf_min != kLeafDefault))
    seven = false;
  const int trace_waves = instance_waves(planes_only, fuse_launch, soft_launch, seven);
  ta.lds_entries = call_lds_entries(s->desc.stack_bound, trace_waves, soft_launch);
  // (soft-light chain launches keep the runtime-knob instance: their kFixed build spilled more
  // SGPRs, C4 -0.8 %)
  const bool fixed = !soft_launch && ta.lds_entries == default_stack(trace_waves) && ta.refill_min == kRefillDefault &&
                     ta.leaf_min == kLeafDefault;
  if (knob(K_LOG_INSTANCE, 0) != 0)  // which trace_refill_kernel instance this call launches (knob tests)
    std::fprintf(stderr, "[rt instance] %s, %lld units, %d frame(s): waves %d, lds rows %d (stack bound %d: %d rows "
                 "spill to HBM), %s%s, %s\n", one_pass ? "one-pass" : "steps", n_units, n_frames, trace_waves,
                 ta.lds_entries, s->desc.stack_bound, std::max(0, s->desc.stack_bound - ta.lds_entries),
                 planes_only ? "planes" : "transformed", fuse_launch ? " fused" : soft_launch ? " soft" : "",
                 fixed ? "constant loop parameters" : "runtime loop parameters");
  ta.occl = s->d_occl;
  la.n_fuse = ta.n_fuse;
  // one-pass calls without textures and with at most one fused light (a later light's shadow ray
  // would reload the full record) store no 32-B hit record: planes-only calls keep the hit's t
  // (kHitCompact), calls of transformed shapes nothing (kHitRecompute: the shading recomputes the
  // hit, r06 A/B same box: C3 +6.2 %, the trace launch -15 %; headline +-0); RT_COMPACT_HIT=0
  // keeps the record
  if (one_pass && ta.has_tex == kHitRecord && ta.n_fuse <= 1 && knob(K_COMPACT_HIT, 1) != 0)
    ta.has_tex = planes_only ? kHitCompact : kHitRecompute;
  la.occl = s->d_occl;
  ta.counters = (unsigned long long*)(ctl + 4);  // byte 16
  // entry + t_near per stack slot
  const size_t lds = (size_t)ta.lds_entries * kBlock * 2 * sizeof(int);

  const bool diag = knob(K_DIAG, 0) != 0 && !p->count_work;
  const bool steps_log = knob(K_STEPS_LOG, 0) != 0;  // diagnostic: every trace launch, any pipeline
  // the diagnostics wait on every step (one pipeline)
  const bool step_sync = diag || kDiagStepSync;

  // ---- pipelines: the slots may split into independent logic -> trace sequences, one per
  // stream (units are claimed from the shared batch counters, so the split changes no value):
  // one pipeline's trace launch drains and its logic and start steps run while the other
  // pipeline's traversal fills the machine.  Before the drain helpers two pipelines won
  // (headline 4967 vs 5521 Mrays/s); with them the drain is short and one pipeline wins
  // everywhere (r03, one box, RT_PIPES=2 vs 1): headline 6050 / 6251, one rank's half / quarter /
  // eighth 5535 / 5875, 5239 / 5948, 4961 / 5357, C3 19955 / 20374, C4 12782 / 12979, C5 7492 /
  // 7683 -- one by default, RT_PIPES=2..4 on request.  Scenes with Trace frames (reflection /
  // refraction: many short steps, a logic step ~25 % of each) take two since r05, with 6M slots
  // between them (C4, same box, 3 reps: one pipeline of 16M 13531-13563 Mrays/s, two of 6M
  // 14135-14190, two of 8M 14044-14185, two of 12M 13691-13721, three of 12M 13886-13963).
  int n_pipes = n_units <= (4LL << 20) ? 1 : frames_scene && !knob_set(K_PIPES) ? 2 : pipes_env();
  if (knob_set(K_PIPES)) n_pipes = pipes_env();  // an explicit request holds for any size
  if (step_sync || one_pass) n_pipes = 1;
  n_pipes = std::max(1, std::min(n_pipes, n_slots / kBlock));  // every pipeline gets whole blocks of slots
  struct Pipe {
    LogicArgs la;
    TraceArgs ta;
    hipStream_t st;
    unsigned logic_blocks, trace_blocks;
    int iters, steps;
    bool done;
  } pipes[kPipes];
  const int per_pipe = (n_slots / kBlock / n_pipes) * kBlock;
  const int spill_entries = std::max(0, s->desc.stack_bound - ta.lds_entries);
  // a call of at most 4M units runs one short launch: one block per CU fewer shortens each
  // ray's latency and so the launch's tail (C2, 1M units: 6 / 5 / 4 blocks 1679 / 1772 / 1790
  // Mrays/s; one rank's eighth, 13M units: 5 and 6 within 1 %)
  const int call_bpc = seven ? (fuse_launch ? s->trace_blocks_per_cu_fuse_seven : s->trace_blocks_per_cu_seven)
                       : fuse_launch ? s->trace_blocks_per_cu_fuse
                       : soft_launch ? s->trace_blocks_per_cu_soft
                                     : s->trace_blocks_per_cu;
  // A deferred one-pass call (another frame in flight) leaves one block per CU to the other
  // frame's camera and shading kernels, which cannot share a CU's registers with six traversal
  // waves per SIMD (r04, one box, two frames in flight, Mrays/s: one rank's eighth / quarter
  // 5220-5260 / 5182-5258 with all blocks, 5291-5316 / 5630 with one fewer; one frame in flight
  // 4918-4924 / 5404-5440).  RT_DEFER_BPC overrides.
  int defer_free = one_pass && p->sync == 0 ? 1 : 0;
  if (one_pass && p->sync == 0)
    defer_free = (int)knob(K_DEFER_BPC, defer_free);
  const unsigned grid_cap = (unsigned)std::max(
      1, s->n_cu * std::max(1, (n_units <= (4LL << 20) ? std::max(1, call_bpc - 1) : call_bpc) - defer_free));
  size_t spill_need = 0;
  for (int h = 0; h < n_pipes; ++h) {
    Pipe& P = pipes[h];
    const int base = h * per_pipe, count = h == n_pipes - 1 ? n_slots - base : per_pipe;
    P.st = h == 0 ? stream : s->aux[h];
    P.la = la;
    P.la.slot_base = base;
    P.la.slot_end = base + count;
    P.ta = ta;
    P.ta.slot_base = base;
    P.ta.n_work = count;
    P.ta.fetch = s->d_fetch + (size_t)h * kFetchLines * kFetchStride;
    P.la.fetch_reset = P.ta.fetch;
    P.la.fetch_reset_n = ta.fetch_shards;
    P.logic_blocks = (unsigned)(count / kBlock);
    P.trace_blocks = std::min(grid_cap, (unsigned)((count + kBlock - 1) / kBlock));
    P.ta.n_threads = (int)P.trace_blocks * kBlock;
    spill_need += (size_t)spill_entries * P.ta.n_threads;
    P.iters = 0;
    P.steps = 0;
    P.done = false;
  }
  if (spill_need > s->spill_cap) {
    if (s->d_spill) (void)hipFree(s->d_spill);
    s->d_spill = nullptr;
    s->spill_cap = 0;
    HIP_TRY(hipMalloc(&s->d_spill, spill_need * sizeof(int2)), RT_ENOMEM);
    s->spill_cap = spill_need;
  }
  for (int h = 0, off = 0; h < n_pipes; ++h) {  // each pipeline's traversal spills into its own range
    pipes[h].ta.spill = s->d_spill + (size_t)2 * off;
    off += spill_entries * pipes[h].ta.n_threads;
  }
  if (kDiagBuild) {
    TraceArgs tas[kPipes];
    for (int h = 0; h < n_pipes; ++h) tas[h] = pipes[h].ta;
    if (!diag_prepare(tas, n_pipes)) return fail(RT_ENOMEM, "diagnostic exit log");
    for (int h = 0; h < n_pipes; ++h) pipes[h].ta.exit_log = tas[h].exit_log;
  }

  {
    InitArgs ia{};
    ia.n_slots = n_slots;
    ia.ctl = ctl;
    ia.ctl_words = kCtlBytes / 4;
    ia.fetch = s->d_fetch;
    ia.fetch_words = (int)(kPipes * kFetchLines * kFetchStride);
    ia.batch_ctr = s->d_batch_ctr;
    ia.batch_shards = la.batch_shards;
    ia.tile_cost = pipes[0].ta.tile_cost;
    ia.n_tiles = 2 * n_tiles;
    hipLaunchKernelGGL(init_kernel, dim3(1), dim3(kBlock), 0, stream, ia);
    HIP_TRY(hipGetLastError(), RT_EDEVICE);
  }

  // ---- iterate logic -> trace per pipeline until none of its slots issues a query
  double trace_ms = 0.0;
  std::vector<std::pair<float, float>> busy;  // every trace launch's (start, end) after ev_t0
  int iters = 0;
  unsigned long long diag_prev = 0;
  // steps go out in host batches (one wait per batch, not per step); the first batch is
  // sized by the previous render's step count
  int batch = step_sync ? 1 : std::max(2, std::min(kMaxHostBatch, s->last_iters + 1));
  HIP_TRY(hipEventRecord(s->ev_t0, stream), RT_EDEVICE);
  if (n_pipes > 1) {  // the other pipelines start after init (and the resets before it)
    HIP_TRY(hipEventRecord(s->ev_fork, stream), RT_EDEVICE);
    for (int h = 1; h < n_pipes; ++h) HIP_TRY(hipStreamWaitEvent(pipes[h].st, s->ev_fork, 0), RT_EDEVICE);
  }
  const bool tex = (s->desc.flags & RT_SCENE_HAS_TEXTURE) != 0;
  // A host batch that should complete the call (by the previous call's step count) ends with
  // the reduce and the statistics copy, so the host waits once for the whole call; when it
  // falls short more steps follow and the reduce runs again.  Earlier batches of a long call
  // (C4: 92 steps in batches of 16) end without them.
  unsigned long long* h_stats = s->h_stats;
  bool reduced = false;
  auto finish = [&]() -> int {  // join the pipelines, reduce, copy the statistics, wait
    for (int h = 1; h < n_pipes; ++h) {
      HIP_TRY(hipEventRecord(s->ev_join, pipes[h].st), RT_EDEVICE);
      HIP_TRY(hipStreamWaitEvent(stream, s->ev_join, 0), RT_EDEVICE);
    }
    hipLaunchKernelGGL(reduce_kernel, dim3((unsigned)((n_pixels + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, la);
    HIP_TRY(hipGetLastError(), RT_EDEVICE);
    if (stats) HIP_TRY(hipMemcpyAsync(h_stats, ctl, kStatsBytes, hipMemcpyDeviceToHost, stream), RT_EDEVICE);
    HIP_TRY(hipEventRecord(s->ev_t1, stream), RT_EDEVICE);
    HIP_TRY(hipEventSynchronize(s->ev_t1), RT_EDEVICE);
    return RT_OK;
  };
  if (one_pass) {  // camera rays, one trace launch, shading + reduction: one host wait
    Pipe& P = pipes[0];
    unsigned int* aq = P.ta.fetch + (size_t)ta.fetch_shards * kFetchStride;  // cleared by init_kernel
    P.la.any_query = aq;
    P.ta.any_query = aq;
    P.ta.host_flag = s->h_flag;
    P.ta.n_work = (int)n_units;
    const unsigned rblocks = (unsigned)((n_pixels + kSrPixels - 1) / kSrPixels);
    // scenes whose every traversal is one leaf item of all their bounded primitives (root_item,
    // RT_FLAT_PRIMS) and no textures: the whole sample in one kernel (flat_render_kernel; its
    // time is the call's trace time); the instrumented and tile-measuring calls keep the launches
    const bool flat_render = !tex && !p->count_work && !measure_tiles && ta.c.use_bvh && ta.root_item < 0 &&
                             ta.root_item != kNoItem && knob(K_FLAT_RENDER, 1) != 0;
    if (flat_render) {
      HIP_TRY(hipEventRecord(s->ev_a[0][0], stream), RT_EDEVICE);
      if (planes_only) hipLaunchKernelGGL((flat_render_kernel<true>), dim3(rblocks), dim3(kBlock), 0, stream, la, P.ta);
      else hipLaunchKernelGGL((flat_render_kernel<false>), dim3(rblocks), dim3(kBlock), 0, stream, la, P.ta);
      HIP_TRY(hipGetLastError(), RT_EDEVICE);
      HIP_TRY(hipEventRecord(s->ev_b[0][0], stream), RT_EDEVICE);
    } else {
      hipLaunchKernelGGL(camera_kernel, dim3((unsigned)((n_units + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, P.la);
      HIP_TRY(hipGetLastError(), RT_EDEVICE);
      HIP_TRY(hipEventRecord(s->ev_a[0][0], stream), RT_EDEVICE);
      launch_trace(P.ta, p->count_work != 0, planes_only, false, seven, fixed, P.trace_blocks, lds, stream);
      HIP_TRY(hipGetLastError(), RT_EDEVICE);
      HIP_TRY(hipEventRecord(s->ev_b[0][0], stream), RT_EDEVICE);
      if (tex) hipLaunchKernelGGL((shade_reduce_kernel<true, kHitRecord>), dim3(rblocks), dim3(kBlock), 0, stream, la);
      else if (ta.has_tex == kHitCompact)
        hipLaunchKernelGGL((shade_reduce_kernel<false, kHitCompact>), dim3(rblocks), dim3(kBlock), 0, stream, la);
      else if (ta.has_tex == kHitRecompute)
        hipLaunchKernelGGL((shade_reduce_kernel<false, kHitRecompute>), dim3(rblocks), dim3(kBlock), 0, stream, la);
      else hipLaunchKernelGGL((shade_reduce_kernel<false, kHitRecord>), dim3(rblocks), dim3(kBlock), 0, stream, la);
      HIP_TRY(hipGetLastError(), RT_EDEVICE);
    }
    HIP_TRY(hipMemcpyAsync(h_stats, ctl, kStatsBytes, hipMemcpyDeviceToHost, stream), RT_EDEVICE);
    if (measure_tiles)
      HIP_TRY(hipMemcpyAsync(s->h_tile_cost, s->d_tile_cost, (size_t)n_tiles * 8, hipMemcpyDeviceToHost, stream),
              RT_EDEVICE);
    HIP_TRY(hipEventRecord(s->ev_t1, stream), RT_EDEVICE);
    rt_scene_s::Pending& q = s->pending;
    q.active = true;
    q.count_work = p->count_work != 0;
    q.measure_tiles = measure_tiles;
    q.n_tiles = n_tiles;
    q.tiles_x = tiles_x;
    q.tiles_y = tiles_y;
    q.tl_dev = tl_dev;
    q.meas_key = meas_key_of(cam, tile_w, tile_h, n_samples);
    q.ta = P.ta;
    // sync == 0: deferred -- rt_render_wait (or the scene's next call) finishes it, so the
    // caller can enqueue another frame (on another scene handle and stream) meanwhile
    if (p->sync == 0) {
      if (stats) stats->path = RT_PATH_ONE_PASS;  // enqueued: rt_render_wait fills the rest
      return RT_OK;
    }
    return finish_one_pass(s, stats);
  }
  for (int live = one_pass ? 0 : n_pipes; live > 0;) {
    for (int h = 0; h < n_pipes; ++h) {
      Pipe& P = pipes[h];
      if (P.done) continue;
      unsigned int* flag = s->h_flag + (size_t)h * kMaxHostBatch * kFetchStride;
      for (int k = 0; k < batch; ++k) {
        const int step = P.steps++;
        // any_query lines alternate by step parity (start_kernel clears the next step's)
        unsigned int* aq = P.ta.fetch + ((size_t)ta.fetch_shards + (step & 1)) * kFetchStride;
        unsigned int* aq_next = P.ta.fetch + ((size_t)ta.fetch_shards + ((step + 1) & 1)) * kFetchStride;
        P.la.any_query = aq;
        P.la.any_query_next = aq_next;
        P.la.first_step = step == 0 ? 1 : 0;
        P.ta.any_query = aq;
        P.ta.host_flag = flag + (size_t)k * kFetchStride;
        if (step > 0) {  // the first step has no result to consume: start_kernel alone
          if (P.la.multi_shadow) {  // first: the logic kernel skips the slots it advanced
            hipLaunchKernelGGL(shadow_step_kernel, dim3(P.logic_blocks), dim3(kBlock), 0, P.st, P.la);
            HIP_TRY(hipGetLastError(), RT_EDEVICE);
          }
          // (kInline: the logic step does the traversal work -- the step's logic, start and flag
          // launches are its trace time, and the host's wait on ev_b covers the flag's store)
          if (inline_queries) HIP_TRY(hipEventRecord(s->ev_a[h][k], P.st), RT_EDEVICE);
          launch_logic(P.la, need_frames, need_refr, tex, planes_only, inline_queries, P.logic_blocks, P.st);
          HIP_TRY(hipGetLastError(), RT_EDEVICE);
        } else if (inline_queries) {
          HIP_TRY(hipEventRecord(s->ev_a[h][k], P.st), RT_EDEVICE);
        }
        hipLaunchKernelGGL(start_kernel, dim3(P.logic_blocks), dim3(kBlock), 0, P.st, P.la);
        HIP_TRY(hipGetLastError(), RT_EDEVICE);
        if (inline_queries) {
          hipLaunchKernelGGL(step_flag_kernel, dim3(1), dim3(1), 0, P.st, (const unsigned int*)aq, P.ta.host_flag);
          HIP_TRY(hipGetLastError(), RT_EDEVICE);
          HIP_TRY(hipEventRecord(s->ev_b[h][k], P.st), RT_EDEVICE);
        } else {
          HIP_TRY(hipEventRecord(s->ev_a[h][k], P.st), RT_EDEVICE);
          launch_trace(P.ta, p->count_work != 0, planes_only, soft_trace, seven, fixed, P.trace_blocks, lds, P.st);
          HIP_TRY(hipGetLastError(), RT_EDEVICE);
          HIP_TRY(hipEventRecord(s->ev_b[h][k], P.st), RT_EDEVICE);
        }
      }
    }
    int enq = 0;
    for (int h = 0; h < n_pipes; ++h) enq = std::max(enq, pipes[h].steps);
    reduced = enq >= s->last_iters + 1;  // the previous call's steps plus its final (empty) one
    if (reduced) {
      if (const int rc = finish()) return rc;
    } else {
      for (int h = 0; h < n_pipes; ++h)
        if (!pipes[h].done) HIP_TRY(hipEventSynchronize(s->ev_b[h][batch - 1]), RT_EDEVICE);
    }
    for (int h = 0; h < n_pipes; ++h) {
      Pipe& P = pipes[h];
      if (P.done) continue;
      const unsigned int* flag = s->h_flag + (size_t)h * kMaxHostBatch * kFetchStride;
      for (int k = 0; k < batch && !P.done; ++k) {
        float ms = 0.f, t_a = 0.f, t_b = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, s->ev_a[h][k], s->ev_b[h][k]), RT_EDEVICE);
        if (stats && hipEventElapsedTime(&t_a, s->ev_t0, s->ev_a[h][k]) == hipSuccess &&
            hipEventElapsedTime(&t_b, s->ev_t0, s->ev_b[h][k]) == hipSuccess)
          busy.emplace_back(t_a, t_b);
        const bool more = flag[(size_t)k * kFetchStride] != 0;
        if (kDiagBuild && more) diag_after_launch(P.ta, ms, iters);
        if (diag && more) {
          unsigned long long rc = 0;
          HIP_TRY(hipMemcpy(&rc, ctl + 8, 8, hipMemcpyDeviceToHost), RT_EDEVICE);
          std::fprintf(stderr, "[rt diag] step %2d: %9llu queries, trace %.3f ms (%.2f Gq/s)\n", iters, rc - diag_prev, ms,
                       (double)(rc - diag_prev) / (ms * 1e6));
          diag_prev = rc;
        }
        if (steps_log)
          std::fprintf(stderr, "[rt steps] pipe %d step %d: any_query %d, trace %.3f ms\n", h, P.steps - batch + k,
                       (int)more, ms);
        if (more) {  // the final (empty) trace launch -- and any after it in the batch -- is not a traversal step
          trace_ms += ms;
          ++iters;
          ++P.iters;
        } else {
          P.done = true;
          --live;
        }
      }
    }
    // more steps: up to the previous call's count in full batches, past it in small ones
    batch = step_sync ? 1 : s->last_iters + 1 > enq ? std::max(2, std::min(kMaxHostBatch, s->last_iters + 1 - enq)) : 4;
  }
  if (!reduced)
    if (const int rc = finish()) return rc;
  s->last_iters = 0;
  for (int h = 0; h < n_pipes; ++h) s->last_iters = std::max(s->last_iters, pipes[h].iters);
  if (stats) {
    const unsigned long long* cnt = h_stats + 2;  // ctl bytes 16, 24, 32
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, s->ev_t0, s->ev_t1), RT_EDEVICE);
    stats->rays = cnt[2];
    stats->box_tests = cnt[0];
    stats->prim_tests = cnt[1];
    stats->kernel_ms = ms;
    stats->trace_ms = trace_ms;
    std::sort(busy.begin(), busy.end());  // union of the launches' intervals
    double un = 0.0, cur_a = -1.0, cur_b = -1.0;
    for (const auto& iv : busy) {
      if (iv.first > cur_b) {
        if (cur_b > cur_a) un += cur_b - cur_a;
        cur_a = iv.first;
        cur_b = iv.second;
      } else {
        cur_b = std::max(cur_b, (double)iv.second);
      }
    }
    if (cur_b > cur_a) un += cur_b - cur_a;
    stats->trace_busy_ms = un;
    stats->iterations = iters;
    stats->path = one_pass ? RT_PATH_ONE_PASS : RT_PATH_STEPS;
    if (kDiagBuild) diag_after_call((const unsigned long long*)(ctl + 4), false);
    stats->node_visits = 0;
    if (p->count_work) stats->node_visits = h_stats[61];  // lane-level node visits (trace_counters_out, ctl byte 488)
    if (p->count_work && knob(K_DIAG, 0) != 0)
      if (const int rc = print_work_diag(ctl)) return rc;
  }
  return RT_OK;
}

extern "C" {

int rt_malloc(int32_t device, size_t bytes, void** d_ptr) {
  if (!d_ptr) return fail(RT_EINVAL, "rt_malloc: null");
  HIP_TRY(hipSetDevice(device), RT_EDEVICE);
  HIP_TRY(hipMalloc(d_ptr, bytes), RT_ENOMEM);
  return RT_OK;
}
int rt_free(void* d_ptr) {
  if (d_ptr) HIP_TRY(hipFree(d_ptr), RT_EDEVICE);
  return RT_OK;
}
int rt_memcpy_d2h(void* h, const void* d, size_t bytes) {
  HIP_TRY(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost), RT_EDEVICE);
  return RT_OK;
}
int rt_memcpy_h2d(void* d, const void* h, size_t bytes) {
  HIP_TRY(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice), RT_EDEVICE);
  return RT_OK;
}
int rt_synchronize(int32_t device) {
  HIP_TRY(hipSetDevice(device), RT_EDEVICE);
  HIP_TRY(hipDeviceSynchronize(), RT_EDEVICE);
  return RT_OK;
}

int rt_quantise_device(const float* d_rgb, int64_t n, uint8_t* d_u8, void* stream) {
  if (n < 0 || (n > 0 && (!d_rgb || !d_u8))) return fail(RT_EINVAL, "rt_quantise_device: bad argument");
  if (n == 0) return RT_OK;
  const unsigned blocks = (unsigned)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(quantise_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, d_rgb, (long long)n, d_u8);
  HIP_TRY(hipGetLastError(), RT_EDEVICE);
  return RT_OK;
}

}  // extern "C"
