/* rt_host.h -- C ABI of the host side (librt_host.so): scene.json loading, BVH build,
 * frame rendering through librt_hip.so, gamma/quantise and P3 PPM output.
 *
 * Mirrors the reference's host surface, which stays C++ (names kept where they map 1:1):
 *   rth_scene_load      Camera(const std::string&)            camera.cpp:240-252
 *                       load_lights_from_json / load_shapes_from_json / parse_material
 *                                                             json_loader.cpp:30-338
 *                       BVH::BVH(shapes)                      acceleration.cpp:7-64
 *   rth_render          main()'s render loop                  raytracer.cpp:433-476
 *   rth_quantise        gamma 1/1.1 + clamp + *255.999        raytracer.cpp:446-457
 *   rth_write_ppm       Image::write (P3, byte-identical)     image.cpp:53-83
 * All functions return 0 on success or a negative RT_E* code (rt_hip.h) and never throw;
 * rth_last_error() describes the last failure.  The reference's stderr warnings for
 * malformed scene entries are reproduced verbatim.
 */
#ifndef RT_HOST_H
#define RT_HOST_H

#include <stdint.h>

#include "rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rth_scene_s* rth_scene_t;

typedef struct rth_scene_info {
  int32_t width, height;       /* render.resolution_x/y (or the override) */
  int32_t n_shapes, n_lights;  /* after the reference's skip rules */
  int32_t n_nodes, tree_depth; /* flattened BVH2 */
  int32_t n_materials, n_textures;
  int32_t prim_stride, flags;
  double load_seconds, build_seconds;
} rth_scene_info;

/* Load scene.json exactly as the reference does.  texture_root replaces the reference's
 * hard-coded "../../Textures/" (NULL = that default); res_w/res_h > 0 override
 * render.resolution_x/y (the reference has no resolution flag). */
int rth_scene_load(const char* path, const char* texture_root, int32_t res_w, int32_t res_h,
                   rth_scene_t* out);
int rth_scene_free(rth_scene_t scene);
int rth_scene_get_info(rth_scene_t scene, rth_scene_info* info);
/* The flattened device records (pointers stay owned by the scene handle). */
int rth_scene_desc(rth_scene_t scene, rt_scene_desc* desc);
int rth_scene_camera(rth_scene_t scene, rt_camera_desc* cam);

/* Render the whole frame on `device` and copy the linear float RGB image (row-major,
 * width*height*3, == compute_pixel_color per pixel) to host_rgb. */
int rth_render(rth_scene_t scene, int32_t device, const rt_render_params* params, float* host_rgb,
               rt_stats* stats);
/* Unpack rt_render_tiles' packed-tile output (host copy) into a row-major image. */
int rth_unpack_tiles(const float* packed, const int32_t* tile_ids, int32_t n_tiles, int32_t tile_w,
                     int32_t tile_h, int32_t width, int32_t height, float* image);

/* raytracer.cpp:446-457 + Image::setPixel clamp (image.cpp:28-37), glibc-exact powf. */
int rth_quantise(const float* rgb, int64_t n_values, uint8_t* out);
/* Image::write (image.cpp:53-83): "P3\n{w} {h}\n255\n", pixels "r g b" joined by two
 * spaces, '\n' per row.  Prints "Image written to <path>" like the reference. */
int rth_write_ppm(const char* path, int32_t width, int32_t height, const uint8_t* rgb);

/* Synthetic triangle soup: n triangles written as
 * `planes` with c3 == c0, centres U[-1,1]^3, vertices centre + U[-s,s]^3, s = n^(-1/3),
 * splitmix64(seed); camera (0,-4,0) gaze (0,1,0) up (0,0,1) focal 35 sensor 36x36;
 * one light (2,-3,3) intensity 600 radius 0; default materials. */
int rth_make_soup(const char* path, int64_t n_triangles, uint64_t seed, int32_t width, int32_t height);

const char* rth_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_HOST_H */
