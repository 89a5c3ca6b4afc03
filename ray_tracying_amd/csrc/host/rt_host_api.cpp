// rt_host_api.cpp -- C ABI of the host layer (include/rt_host.h): scene handles, whole-frame
// rendering through librt_hip.so, gamma/quantise, P3 output, synthetic scenes.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/rt_host.h"
#include "scene.hpp"

#define RT_FMA64 std::fma
#include "../common/rt_powf.h"

namespace {

thread_local std::string g_err;
int fail(int code, const std::string& m) {
  g_err = m;
  return code;
}

template <class T> inline const T& smax(const T& a, const T& b) { return (a < b) ? b : a; }
template <class T> inline const T& smin(const T& a, const T& b) { return (b < a) ? b : a; }

// raytracer.cpp:446-457: pow(c, 1.0f/gamma) -> clamp [0,1] -> (int)(c * 255.999) (double)
// -> Image::setPixel clamp 0..255 (image.cpp:28-37)
inline uint8_t quantise_one(float c) {
  const float gamma = 1.1f;
  float g = rt_powf(c, 1.0f / gamma);
  int v = static_cast<int>(smax(0.0f, smin(1.0f, g)) * 255.999);
  return (uint8_t)std::max(0, std::min(v, 255));
}

uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

struct rth_scene_s {
  std::unique_ptr<rth::Scene> sc;
  std::map<int, rt_scene_t> dev;  // uploaded copies per device
};

extern "C" {

const char* rth_last_error(void) { return g_err.c_str(); }

int rth_scene_load(const char* path, const char* texture_root, int32_t res_w, int32_t res_h, rth_scene_t* out) {
  if (!path || !out) return fail(RT_EINVAL, "rth_scene_load: null argument");
  try {
    auto h = std::make_unique<rth_scene_s>();
    h->sc = rth::load_scene(path, texture_root ? texture_root : "../../Textures/", res_w, res_h);
    *out = h.release();
    return RT_OK;
  } catch (std::exception& e) {
    return fail(RT_EINVAL, e.what());
  }
}

int rth_scene_free(rth_scene_t h) {
  if (!h) return RT_OK;
  for (auto& kv : h->dev) rt_scene_destroy(kv.second);
  delete h;
  return RT_OK;
}

int rth_scene_get_info(rth_scene_t h, rth_scene_info* info) {
  if (!h || !info) return fail(RT_EINVAL, "rth_scene_get_info: null argument");
  const rth::Scene& s = *h->sc;
  *info = rth_scene_info{};
  info->width = s.camera.res_x;
  info->height = s.camera.res_y;
  info->n_shapes = (int32_t)s.shapes.size();
  info->n_lights = (int32_t)s.lights.size();
  info->n_nodes = (int32_t)s.node4.size();
  info->tree_depth = s.tree_depth;
  info->n_materials = (int32_t)s.materials.size();
  info->n_textures = (int32_t)s.textures.size();
  info->prim_stride = s.prim_stride;
  info->flags = s.flags;
  info->load_seconds = s.load_seconds;
  info->build_seconds = s.build_seconds;
  return RT_OK;
}

int rth_scene_desc(rth_scene_t h, rt_scene_desc* d) {
  if (!h || !d) return fail(RT_EINVAL, "rth_scene_desc: null argument");
  *d = rth::scene_desc(*h->sc);
  return RT_OK;
}

int rth_scene_camera(rth_scene_t h, rt_camera_desc* c) {
  if (!h || !c) return fail(RT_EINVAL, "rth_scene_camera: null argument");
  *c = rth::camera_desc(h->sc->camera);
  return RT_OK;
}

int rth_unpack_tiles(const float* packed, const int32_t* tile_ids, int32_t n_tiles, int32_t tw, int32_t th,
                     int32_t W, int32_t H, float* image) {
  if (!packed || !tile_ids || !image || tw <= 0 || th <= 0) return fail(RT_EINVAL, "rth_unpack_tiles: bad argument");
  const int tiles_x = (W + tw - 1) / tw;
  for (int k = 0; k < n_tiles; ++k) {
    const int tid = tile_ids[k];
    const int x0 = (tid % tiles_x) * tw, y0 = (tid / tiles_x) * th;
    for (int ly = 0; ly < th; ++ly) {
      const int y = y0 + ly;
      if (y >= H) break;
      const int w = std::min(tw, W - x0);
      if (w <= 0) continue;
      std::memcpy(image + ((size_t)y * W + x0) * 3, packed + ((size_t)k * tw * th + (size_t)ly * tw) * 3,
                  (size_t)w * 3 * sizeof(float));
    }
  }
  return RT_OK;
}

int rth_render(rth_scene_t h, int32_t device, const rt_render_params* p, float* host_rgb, rt_stats* stats) {
  if (!h || !p || !host_rgb) return fail(RT_EINVAL, "rth_render: null argument");
  const rth::Scene& s = *h->sc;
  rt_camera_desc cam = rth::camera_desc(s.camera);
  if (cam.res_x <= 0 || cam.res_y <= 0) return fail(RT_EINVAL, "Error: Camera resolution is 0. Check scene.json.");
  rt_scene_t ds = nullptr;
  auto it = h->dev.find(device);
  if (it == h->dev.end()) {
    rt_scene_desc d = rth::scene_desc(s);
    int rc = rt_scene_create(device, &d, &ds);
    if (rc) return fail(rc, rt_last_error());
    h->dev[device] = ds;
  } else {
    ds = it->second;
  }
  const int T = 64;
  const int tx = (cam.res_x + T - 1) / T, ty = (cam.res_y + T - 1) / T;
  std::vector<int32_t> tiles((size_t)tx * ty);
  for (size_t i = 0; i < tiles.size(); ++i) tiles[i] = (int32_t)i;
  const size_t n_vals = tiles.size() * T * T * 3;
  void* d_out = nullptr;
  int rc = rt_malloc(device, n_vals * sizeof(float), &d_out);
  if (rc) return fail(rc, rt_last_error());
  rt_stats st{};
  rc = rt_render_tiles(ds, &cam, p, tiles.data(), (int32_t)tiles.size(), T, T, (float*)d_out, nullptr, &st);
  if (!rc && p->sync == 0) rc = rt_render_wait(ds, &st);  // a deferred call: finished here
  if (rc) {
    std::string e = rt_last_error();
    rt_free(d_out);
    return fail(rc, e);
  }
  std::vector<float> packed(n_vals);
  rc = rt_memcpy_d2h(packed.data(), d_out, n_vals * sizeof(float));
  rt_free(d_out);
  if (rc) return fail(rc, rt_last_error());
  rth_unpack_tiles(packed.data(), tiles.data(), (int32_t)tiles.size(), T, T, cam.res_x, cam.res_y, host_rgb);
  if (stats) *stats = st;
  return RT_OK;
}

int rth_quantise(const float* rgb, int64_t n, uint8_t* out) {
  if ((!rgb || !out) && n > 0) return fail(RT_EINVAL, "rth_quantise: null argument");
  for (int64_t i = 0; i < n; ++i) out[i] = quantise_one(rgb[i]);
  return RT_OK;
}

int rth_write_ppm(const char* path, int32_t W, int32_t H, const uint8_t* rgb) {
  if (!path || (!rgb && W * H > 0)) return fail(RT_EINVAL, "rth_write_ppm: null argument");
  FILE* f = std::fopen(path, "wb");
  if (!f) {  // image.cpp:56-59: error message, not fatal
    std::cerr << "Error: Could not open file " << path << " for writing\n";
    return fail(RT_EINVAL, std::string("Error: Could not open file ") + path + " for writing");
  }
  std::string buf;
  buf.reserve((size_t)W * 12 + 16);
  std::fprintf(f, "P3\n%d %d\n255\n", W, H);
  char num[8];
  auto put = [&](unsigned v) {
    int n = 0;
    if (v >= 100) num[n++] = (char)('0' + v / 100);
    if (v >= 10) num[n++] = (char)('0' + (v / 10) % 10);
    num[n++] = (char)('0' + v % 10);
    buf.append(num, n);
  };
  for (int y = 0; y < H; ++y) {
    buf.clear();
    for (int x = 0; x < W; ++x) {
      const uint8_t* p = rgb + ((size_t)y * W + x) * 3;
      put(p[0]);
      buf += ' ';
      put(p[1]);
      buf += ' ';
      put(p[2]);
      if (x < W - 1) buf += "  ";
    }
    buf += '\n';
    std::fwrite(buf.data(), 1, buf.size(), f);
  }
  std::fclose(f);
  std::cout << "Image written to " << path << "\n";
  return RT_OK;
}

int rth_make_soup(const char* path, int64_t n, uint64_t seed, int32_t W, int32_t H) {
  if (!path || n < 0) return fail(RT_EINVAL, "rth_make_soup: bad argument");
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(RT_EINVAL, std::string("rth_make_soup: cannot open ") + path);
  uint64_t st = seed;
  auto u01 = [&]() { return (double)(splitmix(st) >> 11) * (1.0 / 9007199254740992.0); };
  const double s = n > 0 ? std::pow((double)n, -1.0 / 3.0) : 0.0;
  std::fprintf(f,
               "{\"cameras\": [{\"location\": [0.0, -4.0, 0.0], \"gaze_vector\": [0.0, 1.0, 0.0], "
               "\"up_vector\": [0.0, 0.0, 1.0], \"focal_length\": 35.0, \"sensor_width\": 36.0, "
               "\"sensor_height\": 36.0, \"aperture\": 0.0, \"focus_dist\": 10.0}],\n"
               "\"render\": {\"resolution_x\": %d, \"resolution_y\": %d},\n"
               "\"lights\": [{\"location\": [2.0, -3.0, 3.0], \"intensity\": 600.0, \"color\": [1.0, 1.0, 1.0], "
               "\"radius\": 0.0}],\n\"planes\": [\n",
               W, H);
  std::string line;
  char tmp[64];
  for (int64_t i = 0; i < n; ++i) {
    float c[3], v[3][3];
    for (int k = 0; k < 3; ++k) c[k] = (float)(u01() * 2.0 - 1.0);
    for (int q = 0; q < 3; ++q)
      for (int k = 0; k < 3; ++k) v[q][k] = (float)((double)c[k] + (u01() * 2.0 - 1.0) * s);
    line = "{\"corners\": [";
    // c3 == c0 (the only exact triangle encoding)
    const float* cs[4] = {v[0], v[1], v[2], v[0]};
    for (int q = 0; q < 4; ++q) {
      line += '[';
      for (int k = 0; k < 3; ++k) {
        std::snprintf(tmp, sizeof tmp, "%.9g", (double)cs[q][k]);
        line += tmp;
        if (k < 2) line += ", ";
      }
      line += q < 3 ? "], " : "]";
    }
    line += (i + 1 < n) ? "]},\n" : "]}\n";
    std::fwrite(line.data(), 1, line.size(), f);
  }
  std::fprintf(f, "]}\n");
  std::fclose(f);
  return RT_OK;
}

}  // extern "C"
