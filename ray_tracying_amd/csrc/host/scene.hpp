// scene.hpp -- host-side scene model: the reference's loaders, transforms and BVH build,
// flattened into the device records of include/rt_hip.h.
#pragma once
#include <array>
#include <chrono>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/rt_hip.h"

namespace rth {

using V3 = std::array<float, 3>;
using M4 = std::array<std::array<float, 4>, 4>;

struct Box {  // AABB (shapes.hpp:31-58); default = empty (max, lowest)
  V3 lo{3.40282347e+38f, 3.40282347e+38f, 3.40282347e+38f};
  V3 hi{-3.40282347e+38f, -3.40282347e+38f, -3.40282347e+38f};
  void merge(const Box& o);
  void merge(const V3& p);
  int longest_axis() const;
};

struct Texture {  // Image(const std::string&) (image.cpp:86-133)
  int width = 0, height = 0;
  bool loaded = false;
  std::vector<uint8_t> rgb;
};

struct MaterialDesc {  // Material (material.hpp:47-93)
  float diffuse[3] = {0.8f, 0.8f, 0.8f};
  float specular[3] = {1.0f, 1.0f, 1.0f};
  float k_ambient = 0.1f, k_diffuse = 0.9f, k_specular = 0.3f, shininess = 20.0f;
  float roughness = 0.0f, reflectivity = 0.0f, transparency = 0.0f, refractive_index = 1.0f;
  int texture = -1;  // index into Scene::textures
};

struct Shape {
  int kind = RT_PRIM_SPHERE;
  MaterialDesc mat;
  V3 velocity{0, 0, 0};
  M4 w2o{}, o2w{};
  V3 corners[4]{};
  Box bbox() const;  // get_bounding_box of each kind
};

struct CameraDesc {  // Camera members after readCameraSpec (camera.cpp:14-58)
  int res_x = 0, res_y = 0;
  float sensor_w = 0, sensor_h = 0, focal = 0, aperture = 0.0f, focus_dist = 10.0f;
  V3 location{0, 0, 0}, gaze{0, 0, 0}, up{0, 0, 0};
  bool ok = false;
};

struct Scene {
  CameraDesc camera;
  std::vector<rt_light> lights;
  std::vector<Shape> shapes;      // load order: spheres, cubes, rectangles, planes
  std::vector<Texture> textures;
  // flattened
  std::vector<int> order;          // BVH-sorted shape indices (acceleration.cpp:46-55)
  std::vector<rt_prim> prims;      // traversal order (after build_wide)
  std::vector<float> prim_blob;    // prims packed at prim_stride bytes (what the device reads)
  std::vector<rt_node4> node4;        // traversal tree (bvh_wide.cpp)
  std::vector<rt_prim_ref> prim_refs;  // per prim (traversal order)
  std::vector<float> ref_leaf_boxes;   // 8 floats per reference leaf
  int n_unbounded = 0;
  int stack_bound = 1;
  std::vector<rt_material> materials;
  std::vector<uint8_t> texels;
  std::vector<rt_texture> tex_desc;
  int tree_depth = 0;
  int prim_stride = 128;
  int flags = 0;
  float scene_scale = 1.0f;
  double load_seconds = 0, build_seconds = 0;
};

// Phase timings of the host build on stderr when RT_BUILD_TIMING is set (diagnostic).
struct BuildTimer {
  const char* what;
  bool on;
  double t0, last;
  explicit BuildTimer(const char* w);
  void lap(const char* phase);
};

// Worker threads for the host build: RT_BUILD_THREADS, else the hardware concurrency capped at 16.
int build_threads();

// Parse and flatten; throws std::runtime_error on unreadable files (the reference's
// fatal errors), prints the reference's warnings for skipped entries.
std::unique_ptr<Scene> load_scene(const std::string& path, const std::string& texture_root, int res_w, int res_h);
void build_bvh(Scene& sc);
void build_wide(Scene& sc, const std::vector<Box>& shape_box, const std::vector<int>& ref_leaf_of);
rt_camera_desc camera_desc(const CameraDesc& c);
rt_scene_desc scene_desc(const Scene& sc);
M4 build_o2w(const V3& t, const V3& r, const V3& s, M4* w2o);

}  // namespace rth
