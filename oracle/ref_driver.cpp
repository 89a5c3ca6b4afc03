// oracle/ref_driver.cpp -- TEST INFRASTRUCTURE.  Drives the *unmodified* reference sources
// (/root/reference/Code/*.cpp, compiled in place by oracle/Makefile; raytracer.cpp with its
// main() renamed) to dump the reference's own linear float framebuffer.
//
// It replays main()'s render loop (/root/reference/Code/raytracer.cpp:400-480) with the one
// change that std::random_device is replaced by an explicit seed, so the serial mt19937
// stream is reproducible:   std::mt19937 gen(seed)   (raytracer.cpp:425-427).
// Rays are counted by link-time wrapping of BVH::get_intersection (acceleration.cpp:142)
// and AABB tests by wrapping AABB::intersect (shapes.cpp:55) -- no reference source edits.
//
// usage: ref_driver -input scene.json [-bvh] [-s N] [-light_sample N] [-seed S]
//                   [-float-out file.f32] [-ppm-out file.ppm] [-rows y0 y1] [-row-step k]
// -row-step k renders only rows y0, y0 + k, ... < y1 (a sample spread over the frame, for the
// CPU baseline; the float output then holds those rows in order)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "acceleration.hpp"
#include "camera.hpp"
#include "image.hpp"
#include "json_loader.hpp"
#include "light.hpp"
#include "raytracer.hpp"
#include "shapes.hpp"

Color compute_pixel_color(int x, int y, int samples_sqrt, Camera& camera, BVH& bvh,
                          const std::vector<Light>& lights, bool use_bvh, std::mt19937& gen,
                          std::uniform_real_distribution<double>& dist, int light_samples);

static unsigned long long g_rays = 0, g_boxes = 0;
extern "C" {
Hit __real__ZN3BVH16get_intersectionERK3Rayb(BVH* self, const Ray& r, bool b);
Hit __wrap__ZN3BVH16get_intersectionERK3Rayb(BVH* self, const Ray& r, bool b) {
  ++g_rays;
  return __real__ZN3BVH16get_intersectionERK3Rayb(self, r, b);
}
bool __real__ZNK4AABB9intersectERK3Ray(const AABB* self, const Ray& r);
bool __wrap__ZNK4AABB9intersectERK3Ray(const AABB* self, const Ray& r) {
  ++g_boxes;
  return __real__ZNK4AABB9intersectERK3Ray(self, r);
}
}

int main(int argc, char** argv) {
  std::string input, fout, pout;
  bool use_bvh = false;
  int s = 4, ls = 1, y0 = -1, y1 = -1, step = 1;
  unsigned long long seed = 1;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "-bvh")) use_bvh = true;
    else if (!strcmp(argv[i], "-s") && i + 1 < argc) s = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-light_sample") && i + 1 < argc) ls = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-input") && i + 1 < argc) input = argv[++i];
    else if (!strcmp(argv[i], "-seed") && i + 1 < argc) seed = strtoull(argv[++i], 0, 10);
    else if (!strcmp(argv[i], "-float-out") && i + 1 < argc) fout = argv[++i];
    else if (!strcmp(argv[i], "-ppm-out") && i + 1 < argc) pout = argv[++i];
    else if (!strcmp(argv[i], "-rows") && i + 2 < argc) { y0 = atoi(argv[++i]); y1 = atoi(argv[++i]); }
    else if (!strcmp(argv[i], "-row-step") && i + 1 < argc) step = std::max(1, atoi(argv[++i]));
  }
  if (input.empty()) { std::cerr << "ref_driver: -input required\n"; return 2; }
  auto t0 = std::chrono::steady_clock::now();
  Camera camera(input);
  auto [width, height] = camera.getResolution();
  if (width == 0 || height == 0) { std::cerr << "Error: Camera resolution is 0.\n"; return 1; }
  std::vector<Light> lights = load_lights_from_json(input);
  std::vector<std::unique_ptr<Shapes>> shapes = load_shapes_from_json(input);
  std::vector<Shapes*> ptrs;
  for (auto& sh : shapes) ptrs.push_back(sh.get());
  BVH bvh(ptrs);
  std::mt19937 gen((std::mt19937::result_type)seed);
  std::uniform_real_distribution<double> dist(0.0, 1.0);
  if (y0 < 0) { y0 = 0; y1 = height; }
  auto t1 = std::chrono::steady_clock::now();
  unsigned long long boxes_before = g_boxes;
  const int n_rows = (y1 - y0 + step - 1) / step;
  std::vector<float> fb((size_t)width * n_rows * 3);
  Image img(width, height);
  for (int y = y0; y < y1; y += step) {
    for (int x = 0; x < width; ++x) {
      Color c = compute_pixel_color(x, y, s, camera, bvh, lights, use_bvh, gen, dist, ls);
      size_t i = ((size_t)((y - y0) / step) * width + x) * 3;
      fb[i] = c.r; fb[i + 1] = c.g; fb[i + 2] = c.b;
      float gamma = 1.1f;  // raytracer.cpp:446-457
      float r = std::pow(c.r, 1.0f / gamma), g = std::pow(c.g, 1.0f / gamma), b = std::pow(c.b, 1.0f / gamma);
      img.setPixel(x, y, static_cast<int>(std::max(0.0f, std::min(1.0f, r)) * 255.999),
                   static_cast<int>(std::max(0.0f, std::min(1.0f, g)) * 255.999),
                   static_cast<int>(std::max(0.0f, std::min(1.0f, b)) * 255.999));
    }
  }
  auto t2 = std::chrono::steady_clock::now();
  if (!fout.empty()) {
    std::ofstream f(fout, std::ios::binary);
    f.write((const char*)fb.data(), fb.size() * sizeof(float));
  }
  if (!pout.empty()) img.write(pout);
  double ld = std::chrono::duration<double>(t1 - t0).count(), rd = std::chrono::duration<double>(t2 - t1).count();
  printf("{\"width\": %d, \"height\": %d, \"rows\": [%d, %d], \"row_step\": %d, \"n_rows\": %d, \"rays\": %llu, "
         "\"box_tests\": %llu, \"load_seconds\": %.6f, \"render_seconds\": %.6f, \"n_shapes\": %zu, \"n_lights\": %zu}\n",
         width, height, y0, y1, step, n_rows, g_rays, g_boxes - boxes_before, ld, rd, shapes.size(), lights.size());
  return 0;
}
