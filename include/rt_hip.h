/* rt_hip.h -- C ABI of the MI355X ray-trace hot path (librt_hip.so).
 *
 * This is the drop-in boundary for the reference's per-pixel path.  The reference has no
 * FFI; its hot path is entered through C++ free functions and two internal seams, all of
 * which this ABI replaces for a whole frame (or a list of image tiles) at a time:
 *
 *   rt_render_tiles()  replaces the y/x loop of main() calling
 *                      compute_pixel_color(x, y, samples_sqrt, camera, bvh, lights,
 *                      use_bvh, gen, dist, light_samples)
 *                      (/root/reference/Code/raytracer.cpp:18-70, called at :433-476),
 *                      and with it Trace (:280-351), shade (:180-274),
 *                      BVH::get_intersection (/root/reference/Code/acceleration.cpp:142-150,
 *                      acceleration.hpp:23) and Shapes::intersect (shapes.hpp:62).
 *   rt_scene_create()  replaces BVH::BVH + the Shapes object graph as the thing traversal
 *                      reads (acceleration.cpp:7-64, shapes.cpp:92-138): it takes the scene
 *                      already flattened by the host (rt_host.h) into the records below.
 *
 * Conventions: plain pointers and sizes only; no C++ or torch types cross this ABI.
 * Every function returns 0 on success or a negative RT_E* code; rt_last_error() returns a
 * thread-local message for the last failure.  No C++ exception crosses the ABI.
 * Host input descriptors are read during the call only (copied to device memory).
 * Device output buffers are owned by the caller.
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK 0
#define RT_EINVAL -1   /* bad argument / descriptor */
#define RT_EDEVICE -2  /* HIP runtime error (message in rt_last_error) */
#define RT_ENOMEM -3   /* device allocation failed */
#define RT_ENODEV -4   /* no HIP device / extension unusable */

/* primitive kinds (tag bits 0..1) -- Sphere, Cube, Rectangle, Plane (shapes.hpp:89-140) */
#define RT_PRIM_SPHERE 0
#define RT_PRIM_CUBE 1
#define RT_PRIM_RECTANGLE 2
#define RT_PRIM_PLANE 3
#define RT_TAG_KIND(tag) ((tag) & 3u)
#define RT_TAG_PLANE_VALID 4u       /* Plane: |cross(c1-c0,c2-c0)| >= 1e-6f (shapes.cpp:450) */
#define RT_TAG_MOVING 8u            /* Sphere with non-zero velocity (shapes.cpp:207-209) */
#define RT_TAG_TRI1_NEVER 16u       /* Plane with c3 == c0 whose first sub-triangle (c1,c3,c2) cannot
                                       accept a hit point within sqrt(a[12]) of c0 (then a[12] holds
                                       that radius squared instead of c3.x; c3 = c0): scene.cpp */
#define RT_TAG_MATERIAL(tag) ((tag) >> 8)

/* One primitive, 128 bytes (64-byte stride when every primitive is a Plane).
 * Transformed kinds (Sphere/Cube/Rectangle):
 *   a[0..11]  world_to_object rows 0..2 (m[i][0..3])      shapes.hpp:68
 *   a[12..14] velocity (already /5, json_loader.cpp:221-223), a[15] = tag bits
 *   b[0..11]  object_to_world rows 0..2                      shapes.hpp:69
 * Plane (shapes.cpp:444-494; a triangle is a Plane with c3 == c0):
 *   a[0..2]=c0 a[3]=n.x  a[4..6]=c1 a[7]=n.y  a[8..10]=c2 a[11]=n.z  a[12..14]=c3 a[15]=tag
 *   (with RT_TAG_TRI1_NEVER: c3 = c0 and a[12] is a squared radius, finite and >= 0 -- only on
 *   a Plane record with RT_TAG_PLANE_VALID; rt_scene_create rejects any other use of the bit)
 *   n = normalize(cross(c1-c0, c2-c0)), computed on the host with the reference's ops.
 * Records are stored in traversal order; rt_prim_ref gives each one's reference order. */
typedef struct rt_prim {
  float a[16];
  float b[16];
} rt_prim;

/* Traversal node: 4-wide, 64 bytes (half a cache line).  Built on the host with binned SAH
 * over conservative per-primitive hit boxes (bvh_wide.cpp); the reference's own median-split
 * tree (acceleration.cpp:20-64) is NOT used for traversal -- its leaves survive as
 * rt_prim_ref.ref_leaf / ref_leaf_boxes, the exact filter every candidate hit must pass
 * (AABB::intersect, shapes.cpp:55-72).
 * Child boxes are 8-bit coordinates on a per-node grid: bound = origin[a] + q * 2^(e[a]-127).
 * The host picks every q so that this value is <= the child's lo (resp. >= its hi): the grid
 * box always contains the full-precision one, so culling stays conservative.  The kernel
 * evaluates the slab as fma(q, 2^k * inv, (origin - o) * inv) -- rounding of the same order
 * as the plain (lo - o) * inv form, far inside the boxes' 1e-5 * scale padding.
 *   exps: e_x | e_y << 8 | e_z << 16 (biased binary32 exponents of the grid steps)
 *   q_lo_x: byte k = child k's lo.x code (likewise q_hi_x .. q_hi_z)
 *   meta byte k: 0 = no child (child[k] = -1, codes lo 255 / hi 0: an inverted box);
 *                0x01 = internal child (child[k] = node index);
 *                0x80 | n = leaf child with n primitives starting at f:
 *                child[k] = 0x80000000 | f << 7 | n  (f < 2^24, n < 128).
 * rt_scene_create keeps its device copy in this layout for scenes with transformed shapes and
 * re-packs it for planes-only scenes (80-B device nodes, the codes as fp16 integers for the
 * kernel's mixed-precision fmas: the same values); the caller's array is not modified. */
typedef struct rt_node4 {
  float origin[3];
  uint32_t exps;
  uint32_t q_lo_x, q_hi_x, q_lo_y, q_hi_y;
  uint32_t q_lo_z, q_hi_z;
  uint32_t meta;
  int32_t child[4];
  uint32_t pad;
} rt_node4;

/* Per primitive (in traversal order): its position in the reference's BVH-sorted list
 * (the tie-break order for equal t, acceleration.cpp:112/133) and the reference leaf that
 * holds it (index into ref_leaf_boxes), or -1 when the host proved that the reference leaf
 * test passes for every hit the primitive can report (bvh_wide.cpp: acceptance region inside
 * the leaf box shrunk by 1e-5 * scale), so the kernel skips it. */
typedef struct rt_prim_ref {
  int32_t ref_index;
  int32_t ref_leaf;
} rt_prim_ref;

/* Material (material.hpp:47-93 after json_loader.cpp:30-97), 64 bytes. */
typedef struct rt_material {
  float diffuse[3], k_ambient;
  float specular[3], k_diffuse;
  float k_specular, shininess, roughness, reflectivity;
  float transparency, refractive_index;
  int32_t texture; /* index into rt_scene_desc.textures or -1 */
  int32_t pad;     /* ignored: rt_scene_create derives its device copy's flags here */
} rt_material;

/* Point light (light.hpp:5-13), 32 bytes. */
typedef struct rt_light {
  float location[3], intensity;
  float color[3], radius;
} rt_light;

/* P3 texture (image.hpp:8-11): width*height*3 bytes at texels + offset. */
typedef struct rt_texture {
  int32_t width, height;
  int64_t offset;
} rt_texture;

typedef struct rt_scene_desc {
  int32_t n_prims;
  int32_t prim_stride;          /* 64 (all planes) or 128 bytes */
  const rt_prim* prims;         /* n_prims records at prim_stride, traversal order */
  const rt_prim_ref* prim_refs; /* n_prims */
  int32_t n_unbounded;          /* the last n_unbounded prims are tested by every ray */
  int32_t n_nodes;              /* 0 when no bounded primitive */
  int32_t tree_depth;           /* node levels of the 4-wide tree */
  int32_t stack_bound;          /* max traversal stack entries (3 per level + 2) */
  const rt_node4* nodes;
  int32_t n_ref_leaves;
  const float* ref_leaf_boxes;  /* n_ref_leaves x {lo.x, lo.y, lo.z, 0, hi.x, hi.y, hi.z, 0} */
  int32_t n_materials;
  const rt_material* materials;
  int32_t n_lights;
  const rt_light* lights;
  int32_t n_textures;
  const rt_texture* textures;
  int64_t n_texel_bytes;
  const uint8_t* texels;
  float scene_scale; /* max |coordinate| of scene bounds and camera, for pruning margins */
  int32_t flags;     /* RT_SCENE_* feature bits; rt_scene_create also derives them from the
                        materials (reflectivity, transparency > 0, texture >= 0), so a desc
                        that omits one cannot select a kernel variant that drops its path */
} rt_scene_desc;

#define RT_SCENE_HAS_REFLECTION 1
#define RT_SCENE_HAS_REFRACTION 2
#define RT_SCENE_HAS_TEXTURE 4

/* Camera after Camera::readCameraSpec (camera.cpp:14-58); the basis is precomputed on the
 * host with the reference's own ops (camera.cpp:110-116): z = normalize(gaze),
 * x = normalize(up x z), y = normalize(z x x); half_sensor = sensor/2.0f. */
typedef struct rt_camera_desc {
  int32_t res_x, res_y;
  float half_sensor_w, half_sensor_h;
  float location[3], focal_length;
  float x_dir[3], aperture;
  float y_dir[3], focus_dist;
  float z_dir[3], pad;
} rt_camera_desc;

/* Render parameters: the reference's CLI flags (raytracer.cpp:361-390) + RNG key. */
typedef struct rt_render_params {
  int32_t spp_sqrt;      /* -s  (<=1: one ray through the pixel centre) */
  int32_t light_samples; /* -light_sample (0..65535; scenes hold at most 65535 lights) */
  int32_t use_bvh;       /* -bvh (0: linear search over all primitives, acceleration.cpp:124) */
  int32_t count_work;    /* 1: instrumented kernel, fills box_tests / prim_tests */
  uint64_t seed;         /* counter-RNG seed */
  int32_t sync;          /* 1: wait for the render and fill the stats before returning; 0: a one-pass
                            call (rt_stats.path) returns once enqueued on `stream` -- rt_render_wait
                            (or the scene's next call) finishes it; a step-pipeline or chunked call
                            completes before returning and rt_render_wait hands out its stats */
  int32_t pad;
} rt_render_params;

typedef struct rt_stats {
  uint64_t rays;       /* BVH::get_intersection calls: camera + reflection + refraction + shadow */
  uint64_t box_tests;  /* count_work only: AABB tests (32 B each in the roofline model) */
  uint64_t prim_tests; /* count_work only: primitive tests (64 B each) */
  double kernel_ms;    /* HIP-event time of the whole render (all logic+trace steps) */
  double trace_ms;     /* HIP-event time summed over the trace_kernel launches only */
  int32_t iterations;  /* logic->trace steps (== trace_kernel launches) */
  int32_t path;        /* RT_PATH_ONE_PASS when every chunk of the call ran one-pass (camera rays,
                          one trace launch, shading + reduction), RT_PATH_STEPS for the step
                          pipeline (logic -> trace steps over slot state) */
  uint64_t node_visits; /* count_work only: BVH4 node visits (one 64-B node fetch each) */
  double trace_busy_ms; /* HIP-event time during which at least one trace_kernel launch ran (the
                           union of the launches' intervals: slot pipelines overlap theirs) */
} rt_stats;

#define RT_PATH_STEPS 0
#define RT_PATH_ONE_PASS 1

typedef struct rt_scene_s* rt_scene_t;

/* Number of visible HIP devices. */
int rt_device_count(int32_t* count);

/* Copy a flattened scene to `device` and return a handle that owns the device memory. */
int rt_scene_create(int32_t device, const rt_scene_desc* desc, rt_scene_t* out);
int rt_scene_destroy(rt_scene_t scene);

/* Render the listed image tiles (tile id = ty * ceil(res_x/tile_w) + tx; tile_w, tile_h
 * multiples of 8) into d_rgb_out, a DEVICE buffer of n_tiles*tile_w*tile_h*3 floats:
 * tile k occupies [k*tile_w*tile_h*3, (k+1)*tile_w*tile_h*3), row-major RGB, linear
 * (pre-gamma) colour == the reference's compute_pixel_color() result.  Pixels of a tile
 * outside the image are left untouched.  `stream` is a hipStream_t (NULL = default).
 * tile_ids is a HOST array.  A call of more than 2^30 samples (RT_MAX_UNITS) runs as
 * consecutive tile chunks; stats are summed over them.  Replaces the pixel loop of
 * main() (Code/raytracer.cpp:433-443) calling compute_pixel_color (:18-70). */
int rt_render_tiles(rt_scene_t scene, const rt_camera_desc* cam, const rt_render_params* params,
                    const int32_t* tile_ids, int32_t n_tiles, int32_t tile_w, int32_t tile_h,
                    float* d_rgb_out, void* stream, rt_stats* stats);

/* Renders n_frames frames (1..1024) of the same tiles, frame f with counter-RNG seed seeds[f]
 * (params->seed is not used), into d_rgb_out: frame f's n_tiles tiles at
 * [f*n_tiles*tile_w*tile_h*3, (f+1)*n_tiles*tile_w*tile_h*3), each laid out as rt_render_tiles
 * lays out its tiles.  Frame f equals rt_render_tiles with params->seed = seeds[f] bit for bit.
 * One-pass scenes (rt_stats.path) render as many frames per pass as 2^30 samples hold -- every
 * sample of them in one camera pass, one traversal launch and one shading pass -- so a small
 * tile list (one rank's share of a frame split over GPUs) still runs launches of a whole frame's
 * size; the step pipeline renders the frames one after another.  Stats are summed over the
 * frames; sync as for rt_render_tiles; count_work calls must render one frame.  Replaces the
 * reference's render loop (Code/raytracer.cpp:433-476) run once per frame. */
int rt_render_frames(rt_scene_t scene, const rt_camera_desc* cam, const rt_render_params* params,
                     const uint64_t* seeds, int32_t n_frames, const int32_t* tile_ids, int32_t n_tiles,
                     int32_t tile_w, int32_t tile_h, float* d_rgb_out, void* stream, rt_stats* stats);

/* Finishes the scene's last call made with rt_render_params.sync == 0: waits for it if it was
 * deferred (one-pass) and fills `stats` (may be null) -- also when that call had completed
 * before returning (step pipeline, tile chunks: its stats are held for this wait).  With no such
 * call outstanding it returns zeroed stats.  Two scene handles of
 * one scene on two streams keep two frames in flight (bench.py --frames-in-flight 2): the
 * next frame's camera rays and the previous frame's shading run in the idle tail of the
 * other frame's trace launch. */
int rt_render_wait(rt_scene_t scene, rt_stats* stats);

/* Per-tile cost estimate of a frame (host only, no device work): for every tile of the
 * ceil(res_x/tile_w) x ceil(res_y/tile_h) grid (tile id order), how many of a sample of up to
 * 64K primitive centres project into it through `cam` -- the estimate rt_render_tiles orders
 * single-step calls by.  costs_out holds one float per tile.  Multi-GPU callers deal tiles to
 * ranks by it (ray_tracying_amd/tiles.py balanced_deal); every rank computes the same values
 * from the same scene.  No reference counterpart: the reference renders serially
 * (Code/raytracer.cpp:433-476). */
int rt_tile_costs(rt_scene_t scene, const rt_camera_desc* cam, int32_t tile_w, int32_t tile_h, float* costs_out);

/* Measured per-tile cost: the BVH4 node visits the trace kernel made for each tile of the grid
 * (tile id order) in the last instrumented (count_work) one-pass call of this camera, tile
 * size and spp_sqrt -- -1 for tiles that call did not render (or when there was none).  The
 * counts sum to that call's rt_stats.node_visits.  Multi-GPU callers deal tiles to ranks by
 * it (bench.py --deal measured: one instrumented render of the whole frame, then
 * tiles.balanced_deal); not deterministic in the last bits across runs (a wave's visits go to
 * the tile it fetched last), so one rank computes the deal and broadcasts it. */
int rt_tile_costs_measured(rt_scene_t scene, const rt_camera_desc* cam, int32_t tile_w, int32_t tile_h,
                           int32_t spp_sqrt, float* costs_out);

/* Small device-memory helpers so non-torch callers (ctypes tests, the C++ CLI) can drive
 * rt_render_tiles without their own HIP runtime bindings. */
int rt_malloc(int32_t device, size_t bytes, void** d_ptr);
int rt_free(void* d_ptr);
int rt_memcpy_d2h(void* h_dst, const void* d_src, size_t bytes);
int rt_memcpy_h2d(void* d_dst, const void* h_src, size_t bytes);
int rt_synchronize(int32_t device);

/* Device-side pixel finalisation (raytracer.cpp:446-457 + Image::setPixel, image.cpp:28-37):
 * out[i] = clamp((int)(clamp(powf(rgb[i], 1.0f/1.1f), 0, 1) * 255.999), 0, 255), with the
 * bit-exact glibc powf restatement -- equal to rth_quantise byte for byte.  d_rgb / d_u8 are
 * device pointers on the current device; stream may be NULL; returns after enqueueing. */
int rt_quantise_device(const float* d_rgb, int64_t n, uint8_t* d_u8, void* stream);

/* Identification of the compiled device code (e.g. "gfx950"). */
const char* rt_build_info(void);
const char* rt_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_H */
