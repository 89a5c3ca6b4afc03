// scene.cpp -- the reference's host surface, restated for the MI355X path:
//   Camera::readCameraSpec            /root/reference/Code/camera.cpp:14-58
//   parse_material                    /root/reference/Code/json_loader.cpp:30-97
//   load_lights_from_json             /root/reference/Code/json_loader.cpp:103-158
//   load_shapes_from_json             /root/reference/Code/json_loader.cpp:164-338
//   buildTransformationMatrices       /root/reference/Code/shapes.cpp:92-149
//   get_bounding_box (4 kinds)        /root/reference/Code/shapes.cpp:264-287,335-343,425-433,496-503
//   BVH::construct_tree               /root/reference/Code/acceleration.cpp:20-64
// plus the flattening into rt_prim / rt_node / rt_material records.
// Built with -ffp-contract=off: every float op keeps the reference's order and rounding.
#include "scene.hpp"

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <thread>

#include "json_dom.hpp"

namespace rth {

template <class T> static inline const T& smax(const T& a, const T& b) { return (a < b) ? b : a; }  // std::max
template <class T> static inline const T& smin(const T& a, const T& b) { return (b < a) ? b : a; }  // std::min

void Box::merge(const Box& o) {
  for (int i = 0; i < 3; ++i) { lo[i] = smin(lo[i], o.lo[i]); hi[i] = smax(hi[i], o.hi[i]); }
}
void Box::merge(const V3& p) {
  for (int i = 0; i < 3; ++i) { lo[i] = smin(lo[i], p[i]); hi[i] = smax(hi[i], p[i]); }
}
int Box::longest_axis() const {  // shapes.cpp:46-53
  float x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
  if (x > y && x > z) return 0;
  if (y > z) return 1;
  return 2;
}

static M4 mat_mul(const M4& A, const M4& B) {  // shapes.cpp:140-148
  M4 R{};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++)
      for (int k = 0; k < 4; k++) R[i][j] += A[i][k] * B[k][j];
  return R;
}

M4 build_o2w(const V3& t, const V3& r, const V3& s, M4* w2o) {  // shapes.cpp:92-138
  M4 S = {{{s[0], 0, 0, 0}, {0, s[1], 0, 0}, {0, 0, s[2], 0}, {0, 0, 0, 1}}};
  // cos/sin of the float angle promoted to double (shapes.cpp:101-103), narrowed to float
  float cx = (float)std::cos((double)r[0]), sx = (float)std::sin((double)r[0]);
  float cy = (float)std::cos((double)r[1]), sy = (float)std::sin((double)r[1]);
  float cz = (float)std::cos((double)r[2]), sz = (float)std::sin((double)r[2]);
  M4 R = {{{cy * cz, sx * sy * cz - cx * sz, cx * sy * cz + sx * sz, 0},
           {cy * sz, sx * sy * sz + cx * cz, cx * sy * sz - sx * cz, 0},
           {-sy, sx * cy, cx * cy, 0},
           {0, 0, 0, 1}}};
  M4 T = {{{1, 0, 0, t[0]}, {0, 1, 0, t[1]}, {0, 0, 1, t[2]}, {0, 0, 0, 1}}};
  M4 o2w = mat_mul(T, mat_mul(R, S));
  M4 iS = {{{1.0f / s[0], 0, 0, 0}, {0, 1.0f / s[1], 0, 0}, {0, 0, 1.0f / s[2], 0}, {0, 0, 0, 1}}};
  M4 iR = {{{R[0][0], R[1][0], R[2][0], 0}, {R[0][1], R[1][1], R[2][1], 0}, {R[0][2], R[1][2], R[2][2], 0}, {0, 0, 0, 1}}};
  M4 iT = {{{1, 0, 0, -t[0]}, {0, 1, 0, -t[1]}, {0, 0, 1, -t[2]}, {0, 0, 0, 1}}};
  *w2o = mat_mul(mat_mul(iS, iR), iT);
  return o2w;
}

static V3 xpoint(const M4& m, const V3& p) {  // shapes.cpp:151-158
  V3 r;
  float w = m[3][0] * p[0] + m[3][1] * p[1] + m[3][2] * p[2] + m[3][3];
  for (int i = 0; i < 3; i++) r[i] = m[i][0] * p[0] + m[i][1] * p[1] + m[i][2] * p[2] + m[i][3];
  if (std::fabs(w - 1.0f) > 1e-6f && w != 0) { r[0] /= w; r[1] /= w; r[2] /= w; }
  return r;
}

Box Shape::bbox() const {
  Box box;
  switch (kind) {
    case RT_PRIM_SPHERE: {  // shapes.cpp:264-287, swept over time 0..1
      static const float C[8][3] = {{-1, -1, -1}, {1, -1, -1}, {1, 1, -1}, {-1, 1, -1}, {-1, -1, 1}, {1, -1, 1}, {1, 1, 1}, {-1, 1, 1}};
      for (auto& c : C) {
        V3 p = xpoint(o2w, {c[0], c[1], c[2]});
        box.merge(p);
        box.merge(V3{p[0] + velocity[0], p[1] + velocity[1], p[2] + velocity[2]});
      }
      break;
    }
    case RT_PRIM_RECTANGLE: {  // shapes.cpp:335-343
      static const float C[4][3] = {{-0.5f, -0.5f, 0}, {0.5f, -0.5f, 0}, {0.5f, 0.5f, 0}, {-0.5f, 0.5f, 0}};
      for (auto& c : C) box.merge(xpoint(o2w, {c[0], c[1], c[2]}));
      break;
    }
    case RT_PRIM_CUBE: {  // shapes.cpp:425-433
      static const float C[8][3] = {{-0.5f, -0.5f, -0.5f}, {0.5f, -0.5f, -0.5f}, {0.5f, 0.5f, -0.5f}, {-0.5f, 0.5f, -0.5f},
                                    {-0.5f, -0.5f, 0.5f}, {0.5f, -0.5f, 0.5f}, {0.5f, 0.5f, 0.5f}, {-0.5f, 0.5f, 0.5f}};
      for (auto& c : C) box.merge(xpoint(o2w, {c[0], c[1], c[2]}));
      break;
    }
    default: {  // Plane, shapes.cpp:496-503
      const float pad = 1e-4f;
      for (int i = 0; i < 4; ++i) box.merge(corners[i]);
      for (int i = 0; i < 3; ++i) { box.lo[i] -= pad; box.hi[i] += pad; }
    }
  }
  return box;
}

// ---------------------------------------------------------------- loading
static std::string slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) throw std::runtime_error("Error: Could not open JSON file: " + path);
  std::string s;
  f.seekg(0, std::ios::end);
  std::streamoff n = f.tellg();
  f.seekg(0, std::ios::beg);
  if (n > 0) {
    s.resize((size_t)n);
    f.read(&s[0], n);
  }
  return s;
}

static void load_texture(const std::string& fn, Texture& t) {  // Image::read (image.cpp:86-133)
  std::ifstream file(fn);
  if (!file.is_open()) {
    std::cerr << "Error: Could not open file " << fn << " for reading\n";
    return;
  }
  std::string line, magic;
  file >> magic;
  if (magic != "P3") {
    std::cerr << "Error: Only P3 PPM format is supported\n";
    return;
  }
  file >> std::ws;
  while (file.peek() == '#') {
    std::getline(file, line);
    file >> std::ws;
  }
  file >> t.width >> t.height;
  int maxc = 255;
  file >> maxc;
  if (maxc != 255) std::cerr << "Warning: Max color value is " << maxc << ", expected 255\n";
  if (t.width < 0 || t.height < 0) { t.width = t.height = 0; }
  t.rgb.assign((size_t)t.width * t.height * 3, 0);
  for (size_t i = 0; i < t.rgb.size(); i++) {
    int v = 0;
    file >> v;
    t.rgb[i] = (uint8_t)std::max(0, std::min(v, 255));
  }
  std::cout << "Image read from " << fn << " (" << t.width << "x" << t.height << ")\n";
  t.loaded = true;
}

struct Loader {
  const JsonDoc& j;
  Scene& sc;
  std::string tex_root;
  std::string path;
  std::map<std::string, int> tex_cache;

  MaterialDesc parse_material(uint32_t m) {  // json_loader.cpp:30-97
    MaterialDesc mat;
    try {
      float tmp[3];
      if (j.contains(m, "diffuse_color")) { j.get_vec3(j.find(m, "diffuse_color"), tmp); std::copy(tmp, tmp + 3, mat.diffuse); }
      if (j.contains(m, "specular_color")) { j.get_vec3(j.find(m, "specular_color"), tmp); std::copy(tmp, tmp + 3, mat.specular); }
      mat.k_ambient = j.value_float(m, "k_ambient", 0.1f);
      mat.k_diffuse = j.value_float(m, "k_diffuse", 0.6f);
      mat.k_specular = j.value_float(m, "k_specular", 0.6f);
      float rough = j.value_float(m, "roughness", 0.001f);
      rough = smax(0.001f, rough);
      float r = smax(0.001f, smin(1.0f, rough));
      mat.shininess = 5.0f / (r * r);
      mat.roughness = j.value_float(m, "roughness", 0.0f);
      mat.reflectivity = j.value_float(m, "reflectivity", 0.0f);
      mat.transparency = j.value_float(m, "transparency", 0.0f);
      mat.refractive_index = j.value_float(m, "refractive_index", 1.0f);
      if (j.contains(m, "texture_file") && !j.empty(j.find(m, "texture_file"))) {
        std::string fn = j.get_string(j.find(m, "texture_file"));
        if (!fn.empty()) {
          std::string changed = std::string(fn.begin(), fn.end() - (fn.size() >= 3 ? 3 : fn.size())) + "ppm";
          changed = tex_root + changed;
          // successful loads are shared; failures are retried per material, as the
          // reference constructs one Image per material (json_loader.cpp:82-87)
          auto it = tex_cache.find(changed);
          if (it != tex_cache.end()) {
            mat.texture = it->second;
          } else {
            Texture t;
            load_texture(changed, t);
            if (t.width == 0 || !t.loaded) {
              std::cerr << "Warning: Failed to load texture file: " << changed << std::endl;
            } else {
              int idx = (int)sc.textures.size();
              sc.textures.push_back(std::move(t));
              tex_cache[changed] = idx;
              mat.texture = idx;
            }
          }
        }
      }
    } catch (JsonError& e) {
      std::cerr << "Warning: Error parsing material data: " << e.what() << std::endl;
      return MaterialDesc();
    }
    return mat;
  }

  // nlohmann non-const operator[] on a missing key / index reads as null (camera.cpp:26-43)
  uint32_t idx_or_null(uint32_t v, const char* k) {
    if (j.kind(v) == JsonDoc::Null) return v;
    if (!j.is_object(v)) throw JsonError("type_error.305: cannot use operator[] with a string argument");
    return j.find(v, k);
  }

  void camera() {  // Camera::readCameraSpec (camera.cpp:14-58)
    CameraDesc& c = sc.camera;
    uint32_t r = j.root();
    if (!(j.contains(r, "cameras") && j.contains(r, "render"))) {
      std::cerr << "Error: JSON file is missing required keys." << std::endl;
      return;
    }
    try {
      uint32_t cams = j.find(r, "cameras");
      uint32_t c0 = JsonDoc::kNone;
      if (j.is_array(cams)) {
        if (j.size(cams) > 0) c0 = j.at(cams, 0);
      } else if (j.kind(cams) != JsonDoc::Null) {
        throw JsonError("type_error.305: cannot use operator[] with a numeric argument");
      }
      auto member = [&](const char* k) -> uint32_t {
        if (c0 == JsonDoc::kNone) throw JsonError("type_error.302: type must be number, but is null");
        uint32_t v = idx_or_null(c0, k);
        if (v == JsonDoc::kNone) throw JsonError("type_error.302: type must be number, but is null");
        return v;
      };
      c.focal = j.get_float(member("focal_length"));
      if (c0 == JsonDoc::kNone) throw JsonError("type_error.306: cannot use value() with null");
      c.aperture = j.value_float(c0, "aperture", 0.0f);
      c.focus_dist = j.value_float(c0, "focus_dist", 10.0f);
      j.get_vec3(member("location"), c.location.data());
      j.get_vec3(member("gaze_vector"), c.gaze.data());
      j.get_vec3(member("up_vector"), c.up.data());
      c.sensor_w = (float)j.get_int(member("sensor_width"));
      c.sensor_h = (float)j.get_int(member("sensor_height"));
      uint32_t rn = j.find(r, "render");
      uint32_t rx = idx_or_null(rn, "resolution_x"), ry = idx_or_null(rn, "resolution_y");
      if (rx == JsonDoc::kNone || ry == JsonDoc::kNone) throw JsonError("type_error.302: type must be number, but is null");
      c.res_x = j.get_int(rx);
      c.res_y = j.get_int(ry);
      c.ok = true;
    } catch (JsonError& e) {
      std::cerr << "An unexpected error occurred: " << e.what() << std::endl;
      std::cerr << "Camera configuration failed to load. Using default values." << std::endl;
    }
  }

  void lights() {  // json_loader.cpp:103-158
    uint32_t r = j.root();
    if (j.contains(r, "lights") && j.is_array(j.find(r, "lights"))) {
      uint32_t arr = j.find(r, "lights");
      for (uint32_t i = 0; i < j.size(arr); ++i) {
        uint32_t lj = j.at(arr, i);
        if (!j.is_object(lj)) { std::cerr << "Warning: Skipping non-object entry in 'lights' array." << std::endl; continue; }
        try {
          if (!j.contains(lj, "location") || !j.contains(lj, "color") || !j.contains(lj, "intensity")) {
            std::cerr << "Warning: Skipping invalid light definition." << std::endl;
            continue;
          }
          rt_light L{};
          j.get_vec3(j.find(lj, "location"), L.location);
          j.get_vec3(j.find(lj, "color"), L.color);
          L.intensity = j.get_float(j.find(lj, "intensity"));
          L.radius = j.value_float(lj, "radius", 0.0f);
          if (L.intensity <= 0) { std::cerr << "Warning: Skipping light with non-positive intensity." << std::endl; continue; }
          sc.lights.push_back(L);
        } catch (JsonError& e) {
          std::cerr << "Warning: Error parsing light entry: " << e.what() << std::endl;
        }
      }
    } else if (j.contains(r, "lights")) {
      std::cerr << "Warning: 'lights' key found but is not an array in " << path << ". No lights loaded." << std::endl;
    }
    if (sc.lights.empty()) std::cerr << "Warning: No valid lights were loaded from " << path << "." << std::endl;
  }

  uint32_t shape_array(const char* k) {
    uint32_t r = j.root();
    if (j.contains(r, k) && j.is_array(j.find(r, k))) return j.find(r, k);
    return JsonDoc::kNone;
  }
  uint32_t need(uint32_t o, const char* k) {  // const operator[] on a present-or-not key
    uint32_t v = j.find(o, k);
    if (v == JsonDoc::kNone) throw JsonError(std::string("type_error.302: type must be array, but is null (") + k + ")");
    return v;
  }

  void shapes() {  // json_loader.cpp:164-338
    uint32_t a;
    if ((a = shape_array("spheres")) != JsonDoc::kNone) {
      for (uint32_t i = 0; i < j.size(a); ++i) {
        uint32_t s = j.at(a, i);
        if (!j.is_object(s)) continue;
        try {
          V3 t, r{0, 0, 0}, sc3{1, 1, 1}, vel{0, 0, 0};
          j.get_vec3(need(s, "location"), t.data());
          if (j.contains(s, "rotation")) j.get_vec3(j.find(s, "rotation"), r.data());
          if (j.contains(s, "scale") && j.is_array(j.find(s, "scale"))) j.get_vec3(j.find(s, "scale"), sc3.data());
          else if (j.contains(s, "radius")) { float rr = j.get_float(j.find(s, "radius")); sc3 = {rr, rr, rr}; }
          MaterialDesc mat;
          if (j.contains(s, "material")) mat = parse_material(j.find(s, "material"));
          if (j.contains(s, "velocity")) j.get_vec3(j.find(s, "velocity"), vel.data());
          vel[0] = vel[0] / 5; vel[1] = vel[1] / 5; vel[2] = vel[2] / 5;
          Shape sh;
          sh.kind = RT_PRIM_SPHERE;
          sh.mat = mat;
          sh.velocity = vel;
          sh.o2w = build_o2w(t, r, sc3, &sh.w2o);
          sc.shapes.push_back(sh);
        } catch (JsonError& e) { std::cerr << "Warning: Error parsing sphere: " << e.what() << std::endl; }
      }
    }
    if ((a = shape_array("cubes")) != JsonDoc::kNone) {
      for (uint32_t i = 0; i < j.size(a); ++i) {
        uint32_t s = j.at(a, i);
        if (!j.is_object(s)) continue;
        try {
          if (!j.contains(s, "translation") || !j.contains(s, "rotation")) {
            std::cerr << "Warning: Skipping invalid cube definition." << std::endl;
            continue;
          }
          V3 t, r, sc3{1, 1, 1};
          j.get_vec3(j.find(s, "translation"), t.data());
          j.get_vec3(j.find(s, "rotation"), r.data());
          if (j.contains(s, "scale")) {
            uint32_t sv = j.find(s, "scale");
            if (j.is_array(sv)) j.get_vec3(sv, sc3.data());
            else if (j.is_number(sv)) { float x = j.get_float(sv); sc3 = {x, x, x}; }
          }
          MaterialDesc mat;
          if (j.contains(s, "material")) mat = parse_material(j.find(s, "material"));
          Shape sh;
          sh.kind = RT_PRIM_CUBE;
          sh.mat = mat;
          sh.o2w = build_o2w(t, r, sc3, &sh.w2o);
          sc.shapes.push_back(sh);
        } catch (JsonError& e) { std::cerr << "Warning: Error parsing cube entry: " << e.what() << std::endl; }
      }
    }
    if ((a = shape_array("rectangles")) != JsonDoc::kNone) {
      for (uint32_t i = 0; i < j.size(a); ++i) {
        uint32_t s = j.at(a, i);
        if (!j.is_object(s)) continue;
        try {
          V3 t, r, sc3;
          j.get_vec3(need(s, "translation"), t.data());
          j.get_vec3(need(s, "rotation"), r.data());
          j.get_vec3(need(s, "scale"), sc3.data());
          MaterialDesc mat;
          if (j.contains(s, "material")) mat = parse_material(j.find(s, "material"));
          Shape sh;
          sh.kind = RT_PRIM_RECTANGLE;
          sh.mat = mat;
          sh.o2w = build_o2w(t, r, sc3, &sh.w2o);
          sc.shapes.push_back(sh);
        } catch (JsonError& e) { std::cerr << "Warning: Error parsing rectangle: " << e.what() << std::endl; }
      }
    }
    if ((a = shape_array("planes")) != JsonDoc::kNone) {
      for (uint32_t i = 0; i < j.size(a); ++i) {
        uint32_t s = j.at(a, i);
        if (!j.is_object(s)) continue;
        try {
          if (!j.contains(s, "corners") || !j.is_array(j.find(s, "corners")) || j.size(j.find(s, "corners")) != 4) {
            std::cerr << "Warning: Skipping invalid plane definition." << std::endl;
            continue;
          }
          uint32_t cs = j.find(s, "corners");
          Shape sh;
          sh.kind = RT_PRIM_PLANE;
          for (uint32_t k = 0; k < 4; ++k) j.get_vec3(j.at(cs, k), sh.corners[k].data());
          MaterialDesc mat;
          if (j.contains(s, "material")) mat = parse_material(j.find(s, "material"));
          sh.mat = mat;
          sc.shapes.push_back(sh);
        } catch (JsonError& e) { std::cerr << "Warning: Error parsing plane entry: " << e.what() << std::endl; }
      }
    }
    if (sc.shapes.empty()) std::cerr << "Warning: No valid shapes were loaded from " << path << "." << std::endl;
  }
};

std::unique_ptr<Scene> load_scene(const std::string& path, const std::string& texture_root, int res_w, int res_h) {
  auto t0 = std::chrono::steady_clock::now();
  auto sc = std::make_unique<Scene>();
  // main() reads the camera first (raytracer.cpp:396-404): Camera(path) reports an unreadable
  // or malformed file and falls back to resolution 0, which ends the run before the lights
  // and shapes are loaded (camera.cpp:14-58, 240-252); -res (no reference counterpart) skips
  // that stop, and the loaders' own errors then apply (json_loader.cpp:106-116)
  const bool res_override = res_w > 0 && res_h > 0;
  const char* kResZero = "Error: Camera resolution is 0. Check scene.json.";
  auto camera_failed = [&](const std::string& loader_error) {
    std::cerr << "Camera configuration failed to load. Using default values." << std::endl;
    throw std::runtime_error(res_override ? loader_error : std::string(kResZero));
  };
  std::string text;
  try {
    text = slurp(path);
  } catch (std::runtime_error& e) {
    std::cerr << "Error: Could not open file " << path << std::endl;
    camera_failed(e.what());
  }
  std::unique_ptr<JsonDoc> doc;
  try {
    doc = std::make_unique<JsonDoc>(text);
  } catch (JsonError& e) {
    std::cerr << "JSON Parse Error: " << e.what() << std::endl;
    camera_failed(std::string("Error: JSON parsing error: ") + e.what());
  }
  { std::string().swap(text); }
  Loader L{*doc, *sc, texture_root, path, {}};
  L.camera();
  if (res_override) {
    sc->camera.res_x = res_w;
    sc->camera.res_y = res_h;
  }
  if (sc->camera.res_x == 0 || sc->camera.res_y == 0) throw std::runtime_error(kResZero);
  L.lights();
  L.shapes();
  doc.reset();
  auto t1 = std::chrono::steady_clock::now();
  build_bvh(*sc);
  auto t2 = std::chrono::steady_clock::now();
  sc->load_seconds = std::chrono::duration<double>(t1 - t0).count();
  sc->build_seconds = std::chrono::duration<double>(t2 - t1).count();
  return sc;
}

// ---------------------------------------------------------------- BVH + flattening
static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
BuildTimer::BuildTimer(const char* w) : what(w), on(std::getenv("RT_BUILD_TIMING") != nullptr), t0(now_s()), last(t0) {}
void BuildTimer::lap(const char* phase) {
  if (!on) return;
  const double t = now_s();
  std::fprintf(stderr, "[%s] %-36s %8.3f s (total %.3f s)\n", what, phase, t - last, t - t0);
  last = t;
}

// Cores this process may use: its affinity mask capped by the cgroup v2 CPU quota (the job's
// share on a shared host; hardware_concurrency() is the whole machine) -- bench.py's usable_cpus()
static int usable_cores() {
  int n = 0;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
  if (n <= 0) {
    const unsigned hc = std::thread::hardware_concurrency();
    n = hc ? (int)hc : 1;
  }
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long per = 0;
    if (std::fscanf(f, "%31s %lld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0) {
      const long long quota = std::atoll(q) / per;
      if (quota >= 1) n = (int)std::min<long long>(n, quota);
    }
    std::fclose(f);
  }
  return std::max(1, n);
}

int build_threads() {
  const int cores = usable_cores();
  if (const char* e = std::getenv("RT_BUILD_THREADS")) return std::max(1, std::min(std::min(64, cores), std::atoi(e)));
  return std::min(16, cores);
}

namespace {

struct BNode {
  Box box;
  int left = -1, right = -1;
  int start = 0, end = 0;
  bool leaf() const { return left < 0; }
};

struct Builder {
  std::vector<int>& order;
  const std::vector<Box>& boxes;
  std::vector<float> cent;  // centroid along the current sort axis, per shape
  std::atomic<int> spare{0};  // threads free to take a subtree
  static constexpr int kSpawnMin = 16384;

  // Nodes in DFS pre-order (left subtree first).  A subtree built on another thread works on
  // its own disjoint range of `order` / `cent` and is appended with shifted indices, so the
  // node numbering (the reference-leaf ids) is the sequential build's for any thread count.
  static void append(std::vector<BNode>& dst, std::vector<BNode>&& src) {
    const int d = (int)dst.size();
    for (BNode& nd : src) {
      if (nd.left >= 0) {
        nd.left += d;
        nd.right += d;
      }
      dst.push_back(nd);
    }
    std::vector<BNode>().swap(src);
  }

  int build(int start, int end, std::vector<BNode>& nodes) {  // acceleration.cpp:20-64
    int id = (int)nodes.size();
    nodes.emplace_back();
    Box nb;
    for (int i = start; i < end; i++) nb.merge(boxes[order[i]]);
    nodes[id].box = nb;
    nodes[id].start = start;
    nodes[id].end = end;
    if (end - start <= 4) return id;
    int axis = nb.longest_axis();
    for (int i = start; i < end; ++i) {
      const Box& b = boxes[order[i]];
      cent[order[i]] = (b.lo[axis] + b.hi[axis]) / 2.0f;
    }
    const float* c = cent.data();
    // Same comparator results as the reference's lambda on the same sequence -> std::sort
    // (libstdc++ introsort) produces the same permutation.
    std::sort(order.begin() + start, order.begin() + end, [c](int a, int b) { return c[a] < c[b]; });
    int mid = (start + end) / 2;
    int l, r;
    int tok = spare.load();
    if (mid - start >= kSpawnMin && tok > 0 && spare.compare_exchange_strong(tok, tok - 1)) {
      std::vector<BNode> ln, rn;
      std::thread t([&] { build(start, mid, ln); });
      build(mid, end, rn);
      t.join();
      spare.fetch_add(1);
      l = (int)nodes.size();
      append(nodes, std::move(ln));
      r = (int)nodes.size();
      append(nodes, std::move(rn));
    } else {
      l = build(start, mid, nodes);
      r = build(mid, end, nodes);
    }
    nodes[id].left = l;
    nodes[id].right = r;
    return id;
  }
};

// isPointInQuad's first sub-triangle (c1, c3, c2) (shapes.cpp:485-494) with c3 == c0 has the
// opposite winding to the normal: its three edge functions e_i = dot(cross(B-A, P-A), n) sum to
// S = dot(A x B + B x C + C x A, n) < 0 for every point P.  isPointInTriangle (shapes.cpp:24-40)
// accepts only if all three float e_i >= -1e-6, i.e. (with float error |e_i - exact| <=
// 32 * 2^-24 * |E_i| * |P - A_i|) only if S >= -3e-6 - sum of the errors.  For |P - c0| <= R
// (|P - A_i| <= R + Emax) that is impossible when |S| - 3e-6 > 96 * 2^-24 * Emax * (R + Emax).
// Returns half of the largest such R (0 if none): the kernel skips the test for hit points
// within R of c0 -- same result, fewer instructions.
double tri1_never_radius(const V3& A, const V3& B, const V3& C, const V3& n) {
  auto d3 = [](const V3& v) { return std::array<double, 3>{v[0], v[1], v[2]}; };
  auto cross = [](const std::array<double, 3>& a, const std::array<double, 3>& b) {
    return std::array<double, 3>{a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  };
  const auto a = d3(A), b = d3(B), c = d3(C), nn = d3(n);
  const auto ab = cross(a, b), bc = cross(b, c), ca = cross(c, a);
  double S = 0, mag = 0;
  for (int k = 0; k < 3; ++k) {
    S += (ab[k] + bc[k] + ca[k]) * nn[k];
    mag += (std::fabs(ab[k]) + std::fabs(bc[k]) + std::fabs(ca[k])) * std::fabs(nn[k]);
  }
  if (!(S < 0)) return 0.0;
  auto len = [](const std::array<double, 3>& u, const std::array<double, 3>& v) {
    return std::sqrt((u[0] - v[0]) * (u[0] - v[0]) + (u[1] - v[1]) * (u[1] - v[1]) + (u[2] - v[2]) * (u[2] - v[2]));
  };
  const double emax = std::max({len(a, b), len(b, c), len(c, a)});
  const double slack = -S - 3e-6 - 1e-12 * mag;  // double rounding of S: far below 1e-12 * mag
  if (!(slack > 0) || !(emax > 0)) return 0.0;
  const double r = slack / (96.0 * std::ldexp(1.0, -24) * emax) - emax;
  return r > 0 ? 0.5 * r : 0.0;
}

float finite_abs_max(float a, float b) {
  if (!std::isfinite(b)) return a;
  return std::max(a, std::fabs(b));
}

}  // namespace

void build_bvh(Scene& sc) {
  BuildTimer tm("build_bvh");
  const int n = (int)sc.shapes.size();
  std::vector<Box> boxes(n);
  for (int i = 0; i < n; ++i) boxes[i] = sc.shapes[i].bbox();
  tm.lap("shape boxes");
  sc.order.resize(n);
  for (int i = 0; i < n; ++i) sc.order[i] = i;
  Builder B{sc.order, boxes, std::vector<float>(n)};
  B.spare = build_threads() - 1;
  std::vector<BNode> ref_nodes;
  if (n > 0) {
    ref_nodes.reserve((size_t)n);
    B.build(0, n, ref_nodes);
  }
  tm.lap("reference median-split tree");

  // materials (deduplicated) and primitive records in sorted order
  std::map<std::vector<char>, int> mat_ids;
  rt_material last_mat{};
  int last_mid = -1;
  sc.materials.clear();
  sc.prims.assign((size_t)n, rt_prim{});
  bool all_planes = true;
  int flags = 0;
  float scale = 1.0f;
  for (int k = 0; k < n; ++k) {
    const Shape& s = sc.shapes[sc.order[k]];
    rt_material m{};
    std::copy(s.mat.diffuse, s.mat.diffuse + 3, m.diffuse);
    m.k_ambient = s.mat.k_ambient;
    std::copy(s.mat.specular, s.mat.specular + 3, m.specular);
    m.k_diffuse = s.mat.k_diffuse;
    m.k_specular = s.mat.k_specular;
    m.shininess = s.mat.shininess;
    m.roughness = s.mat.roughness;
    m.reflectivity = s.mat.reflectivity;
    m.transparency = s.mat.transparency;
    m.refractive_index = s.mat.refractive_index;
    m.texture = s.mat.texture;
    int mid;
    if (last_mid >= 0 && std::memcmp(&last_mat, &m, sizeof m) == 0) {
      mid = last_mid;  // runs of one material (triangle soups): no map lookup
    } else if (auto it = mat_ids.find(std::vector<char>((const char*)&m, (const char*)&m + sizeof(m)));
               it == mat_ids.end()) {
      std::vector<char> key((const char*)&m, (const char*)&m + sizeof(m));
      mid = (int)sc.materials.size();
      mat_ids[key] = mid;
      sc.materials.push_back(m);
      if (m.reflectivity > 0.0f) flags |= RT_SCENE_HAS_REFLECTION;
      if (m.transparency > 0.0f) flags |= RT_SCENE_HAS_REFRACTION;
      if (m.texture >= 0) flags |= RT_SCENE_HAS_TEXTURE;
    } else {
      mid = it->second;
    }
    last_mat = m;
    last_mid = mid;
    rt_prim& p = sc.prims[k];
    uint32_t tag = (uint32_t)s.kind | ((uint32_t)mid << 8);
    if (s.kind == RT_PRIM_PLANE) {
      const V3* c = s.corners;
      // Plane::intersect's normal (shapes.cpp:446-451), identical ops
      V3 e1{c[1][0] - c[0][0], c[1][1] - c[0][1], c[1][2] - c[0][2]};
      V3 e2{c[2][0] - c[0][0], c[2][1] - c[0][1], c[2][2] - c[0][2]};
      V3 nn{e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
      float len = std::sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
      if (!(len < 1e-6f)) tag |= RT_TAG_PLANE_VALID;
      V3 un{nn[0] / len, nn[1] / len, nn[2] / len};
      for (int q = 0; q < 3; ++q) {
        p.a[4 * q + 0] = c[q][0];
        p.a[4 * q + 1] = c[q][1];
        p.a[4 * q + 2] = c[q][2];
        p.a[4 * q + 3] = un[q];
      }
      p.a[12] = c[3][0];
      p.a[13] = c[3][1];
      p.a[14] = c[3][2];
      if ((tag & RT_TAG_PLANE_VALID) && c[3] == c[0]) {
        const double r = tri1_never_radius(c[1], c[0], c[2], un);
        if (r > 0.0) {  // a[12] = R^2 (rounded down); c3 == c0 is implied by the tag
          tag |= RT_TAG_TRI1_NEVER;
          p.a[12] = std::nextafter((float)(r * r), 0.0f);
        }
      }
    } else {
      all_planes = false;
      for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 4; ++q) {
          p.a[4 * r + q] = s.w2o[r][q];
          p.b[4 * r + q] = s.o2w[r][q];
        }
      p.a[12] = s.velocity[0];
      p.a[13] = s.velocity[1];
      p.a[14] = s.velocity[2];
      if (s.kind == RT_PRIM_SPHERE && (s.velocity[0] != 0 || s.velocity[1] != 0 || s.velocity[2] != 0)) tag |= RT_TAG_MOVING;
    }
    std::memcpy(&p.a[15], &tag, 4);
  }
  tm.lap("materials + primitive records");
  if (sc.materials.empty()) sc.materials.push_back(rt_material{});  // placeholder for empty scenes
  sc.prim_stride = (n > 0 && all_planes) ? 64 : 128;

  // scale for pruning / padding margins: scene boxes and the camera
  for (const BNode& nd : ref_nodes)
    for (int i = 0; i < 3; ++i) scale = finite_abs_max(finite_abs_max(scale, nd.box.lo[i]), nd.box.hi[i]);
  for (int i = 0; i < 3; ++i) scale = finite_abs_max(scale, sc.camera.location[i]);
  sc.scene_scale = scale;

  // the reference's leaves: exact boxes + which leaf holds each sorted position
  std::vector<int> ref_leaf_of(n, 0);
  sc.ref_leaf_boxes.clear();
  for (const BNode& nd : ref_nodes) {
    if (!nd.leaf()) continue;
    int id = (int)(sc.ref_leaf_boxes.size() / 8);
    for (int i = nd.start; i < nd.end; ++i) ref_leaf_of[i] = id;
    const float v[8] = {nd.box.lo[0], nd.box.lo[1], nd.box.lo[2], 0.0f, nd.box.hi[0], nd.box.hi[1], nd.box.hi[2], 0.0f};
    sc.ref_leaf_boxes.insert(sc.ref_leaf_boxes.end(), v, v + 8);
  }
  sc.tree_depth = 0;
  tm.lap("reference leaves");
  build_wide(sc, boxes, ref_leaf_of);
  tm.lap("traversal tree (build_wide)");
  {
    const size_t fl = (size_t)sc.prim_stride / 4;
    const size_t np = sc.prims.size();  // spatial splits may duplicate primitives
    sc.prim_blob.assign(np * fl, 0.0f);
    for (size_t k = 0; k < np; ++k) std::memcpy(&sc.prim_blob[(size_t)k * fl], &sc.prims[k], (size_t)sc.prim_stride);
  }
  sc.flags = flags;

  // textures -> one byte array
  sc.tex_desc.clear();
  sc.texels.clear();
  for (const Texture& t : sc.textures) {
    rt_texture d{};
    d.width = t.loaded ? t.width : 0;
    d.height = t.loaded ? t.height : 0;
    d.offset = (int64_t)sc.texels.size();
    if (t.loaded) sc.texels.insert(sc.texels.end(), t.rgb.begin(), t.rgb.end());
    sc.tex_desc.push_back(d);
  }
}

rt_camera_desc camera_desc(const CameraDesc& c) {
  // Camera::normalize / cross_product (camera.cpp:60-87) and the basis (camera.cpp:110-116)
  auto norm = [](const V3& v) -> V3 {
    float m = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (m == 0.0f) return {0.0f, 0.0f, 0.0f};
    return {v[0] / m, v[1] / m, v[2] / m};
  };
  auto cross = [](const V3& a, const V3& b) -> V3 {
    return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  };
  V3 z = norm(c.gaze);
  V3 x = norm(cross(c.up, z));
  V3 y = norm(cross(z, x));
  rt_camera_desc d{};
  d.res_x = c.res_x;
  d.res_y = c.res_y;
  d.half_sensor_w = c.sensor_w / 2.0f;
  d.half_sensor_h = c.sensor_h / 2.0f;
  for (int i = 0; i < 3; ++i) {
    d.location[i] = c.location[i];
    d.x_dir[i] = x[i];
    d.y_dir[i] = y[i];
    d.z_dir[i] = z[i];
  }
  d.focal_length = c.focal;
  d.aperture = c.aperture;
  d.focus_dist = c.focus_dist;
  return d;
}

rt_scene_desc scene_desc(const Scene& sc) {
  rt_scene_desc d{};
  d.n_prims = (int32_t)sc.prims.size();
  d.prim_stride = sc.prim_stride;
  d.prims = reinterpret_cast<const rt_prim*>(sc.prim_blob.data());
  d.prim_refs = sc.prim_refs.data();
  d.n_unbounded = sc.n_unbounded;
  d.n_nodes = (int32_t)sc.node4.size();
  d.tree_depth = sc.tree_depth;
  d.stack_bound = sc.stack_bound;
  d.nodes = sc.node4.data();
  d.n_ref_leaves = (int32_t)(sc.ref_leaf_boxes.size() / 8);
  d.ref_leaf_boxes = sc.ref_leaf_boxes.data();
  d.n_materials = (int32_t)sc.materials.size();
  d.materials = sc.materials.data();
  d.n_lights = (int32_t)sc.lights.size();
  d.lights = sc.lights.data();
  d.n_textures = (int32_t)sc.tex_desc.size();
  d.textures = sc.tex_desc.data();
  d.n_texel_bytes = (int64_t)sc.texels.size();
  d.texels = sc.texels.data();
  d.scene_scale = sc.scene_scale;
  d.flags = sc.flags;
  return d;
}

}  // namespace rth
