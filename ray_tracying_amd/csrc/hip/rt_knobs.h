// rt_knobs.h -- every runtime knob of librt_hip in one table (host code only).
//
// The knobs are environment variables for A/B measurement, sweeps and tests; none changes a
// result (tests/test_gpu_knobs.py renders every one against the oracle).  They are read into
// one snapshot at each entry of the C ABI (rt_scene_create, rt_render_tiles, rt_render_frames:
// knobs_refresh), so a call sees one consistent set and tests may vary them between calls of
// one process; everything else reads the snapshot (knob / knob_set), never the environment.
// Unset knobs take the defaults in rt_hip.hip (DESIGN.md 4 and 5 give the measurements behind
// them); a set value is clamped to the table's range.
#ifndef RT_KNOBS_H
#define RT_KNOBS_H

#include <algorithm>
#include <cstdlib>

enum Knob : int {
  // path and sizes
  K_ONE_PASS,       // 0: the step pipeline for every call (one-pass scenes too)
  K_ONE_PASS_MAX,   // units of one one-pass pass (default 2^30); larger calls run as tile / frame chunks
  K_MAX_UNITS,      // units of one call of any path (default 2^30); larger calls run as tile chunks
  K_SLOTS,          // step pipeline: slots in flight (default 128M, 6M with Trace frames)
  K_PIPES,          // step pipeline: slot pipelines on their own streams (default 1, 2 with Trace frames)
  K_FUSE,           // step pipeline: 0 / 1 point-light shadow rays traced by the closest hit's lane
  K_SOFT_FUSE,      // 0: soft-light shadow samples advanced by shadow_step_kernel, not the tracing lane
  K_SOFT_START,     // 0: a closest hit's first soft shadow sample emitted by the logic step
  K_SHADOW_STEP,    // 0 (with RT_SOFT_FUSE=0): soft samples advanced by the logic kernel itself
  K_COMPACT_HIT,    // 0: one-pass planes calls store the 32-B hit record instead of the hit's t
  K_FLAT_PRIMS,     // scenes of at most this many bounded primitives test them all, no traversal (default 8)
  K_FLAT_RENDER,    // 0: one-pass calls of such scenes keep camera / traversal / shading launches (default 1: one kernel)
  // traversal scheduling
  K_FETCH_SHARDS,   // trace work counters (default 32)
  K_BATCH_SHARDS,   // step pipeline: batch-claim counters (default 128)
  K_LEAF_MIN,       // lanes waiting on a leaf before the leaf phase runs (default 24)
  K_REFILL,         // refill finished lanes when fewer than this many traverse (default 48)
  K_LDS_STACK,      // traversal stack entries per lane kept in LDS (default by waves/SIMD: 11 / 12 / 16)
  K_TRACE_SEVEN,    // 0 / 1: the 7-wave planes instances (default: synchronous calls of > 32M units)
  K_DRAIN_HELP,     // 0: no drain helpers once a launch's queue is dry
  K_XCD_CHUNK,      // groups per XCD chunk of the work deal (default 64; 0 = round robin)
  K_TILE_ORDER,     // 0 / 1: render tiles costliest first never / always (default: one-step calls)
  K_DEFER_BPC,      // blocks per CU a deferred one-pass call leaves to the other frame (default 1)
  K_TRACE_BPC,      // cap on the traversal's blocks per CU (diagnostic)
  // logs
  K_DIAG,           // per-step query counts and rates (forces one pipeline, a wait per step)
  K_STEPS_LOG,      // every trace launch of every pipeline: any_query and its time
  K_LOG_INSTANCE,   // the traversal instance each call launches (waves/SIMD, LDS rows, variant)
  K_COUNT
};

struct KnobDef {
  const char* name;
  long long lo, hi;
};

// names and ranges, in Knob order
static constexpr KnobDef kKnobDefs[K_COUNT] = {
    {"RT_ONE_PASS", 0, 1},        {"RT_ONE_PASS_MAX", 1, 1LL << 30}, {"RT_MAX_UNITS", 1, 1LL << 30},
    {"RT_SLOTS", 1LL << 12, 1LL << 31}, {"RT_PIPES", 1, 4},          {"RT_FUSE", 0, 1},
    {"RT_SOFT_FUSE", 0, 1},       {"RT_SOFT_START", 0, 1},           {"RT_SHADOW_STEP", 0, 1},
    {"RT_COMPACT_HIT", 0, 1},     {"RT_FLAT_PRIMS", 0, 1 << 20},     {"RT_FLAT_RENDER", 0, 1},
    {"RT_FETCH_SHARDS", 1, 256},  {"RT_BATCH_SHARDS", 1, 1024},      {"RT_LEAF_MIN", 1, 64},
    {"RT_REFILL", 1, 64},         {"RT_LDS_STACK", 1, 64},           {"RT_TRACE_SEVEN", 0, 1},
    {"RT_DRAIN_HELP", 0, 1},      {"RT_XCD_CHUNK", 0, 1LL << 20},    {"RT_TILE_ORDER", 0, 1},
    {"RT_DEFER_BPC", 0, 64},      {"RT_TRACE_BPC", 1, 64},           {"RT_DIAG", 0, 1},
    {"RT_STEPS_LOG", 0, 1},       {"RT_LOG_INSTANCE", 0, 1},
};

struct Knobs {
  long long v[K_COUNT] = {};
  bool set[K_COUNT] = {};
};

// The snapshot of the calling thread (the CLI renders one device per host thread).
inline Knobs& knobs_snapshot() {
  static thread_local Knobs k;
  return k;
}

inline void knobs_refresh() {
  Knobs& k = knobs_snapshot();
  for (int i = 0; i < K_COUNT; ++i) {
    const char* e = std::getenv(kKnobDefs[i].name);
    k.set[i] = e != nullptr;
    long long x = e ? std::atoll(e) : 0;
    if (kKnobDefs[i].hi == 1 && kKnobDefs[i].lo == 0) x = x != 0;  // on / off knobs: any non-zero is on
    k.v[i] = std::max(kKnobDefs[i].lo, std::min(kKnobDefs[i].hi, x));
  }
}

inline bool knob_set(Knob k) { return knobs_snapshot().set[k]; }
// the knob's value when set, else `dflt`
inline long long knob(Knob k, long long dflt) { return knobs_snapshot().set[k] ? knobs_snapshot().v[k] : dflt; }

#endif  // RT_KNOBS_H
