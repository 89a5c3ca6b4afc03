// oracle/oracle_cli.cpp -- TEST INFRASTRUCTURE.  Command-line front end of liboracle.so.
// usage: oracle_cli -input scene.json [-bvh] [-s N] [-light_sample N] [-seed S]
//                   [-rng mt|counter] [-res WxH] [-region x0 y0 w h]
//                   [-float-out f.f32] [-ppm-out f.ppm] [-textures DIR/]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

extern "C" {
struct oracle_params { int use_bvh, spp_sqrt, light_samples, rng_mode; unsigned long long seed; int res_w, res_h, x0, y0, w, h; };
struct oracle_stats { unsigned long long rays, box_tests, prim_tests; int width, height, n_shapes, n_lights; double render_seconds, load_seconds; };
int oracle_render(const char*, const char*, const oracle_params*, float*, unsigned char*, oracle_stats*);
int oracle_scene_info(const char*, int*, int*, int*, int*);
}

int main(int argc, char** argv) {
  oracle_params p{0, 4, 1, 0, 1, 0, 0, 0, 0, 0, 0};
  std::string input, fout, pout, tex = "../../Textures/";
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "-bvh")) p.use_bvh = 1;
    else if (!strcmp(argv[i], "-s") && i + 1 < argc) p.spp_sqrt = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-light_sample") && i + 1 < argc) p.light_samples = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-seed") && i + 1 < argc) p.seed = strtoull(argv[++i], 0, 10);
    else if (!strcmp(argv[i], "-rng") && i + 1 < argc) p.rng_mode = strcmp(argv[++i], "counter") == 0 ? 1 : 0;
    else if (!strcmp(argv[i], "-res") && i + 1 < argc) sscanf(argv[++i], "%dx%d", &p.res_w, &p.res_h);
    else if (!strcmp(argv[i], "-region") && i + 4 < argc) { p.x0 = atoi(argv[++i]); p.y0 = atoi(argv[++i]); p.w = atoi(argv[++i]); p.h = atoi(argv[++i]); }
    else if (!strcmp(argv[i], "-input") && i + 1 < argc) input = argv[++i];
    else if (!strcmp(argv[i], "-float-out") && i + 1 < argc) fout = argv[++i];
    else if (!strcmp(argv[i], "-ppm-out") && i + 1 < argc) pout = argv[++i];
    else if (!strcmp(argv[i], "-textures") && i + 1 < argc) tex = argv[++i];
  }
  int W, H, ns, nl;
  if (input.empty() || oracle_scene_info(input.c_str(), &W, &H, &ns, &nl) != 0) { fprintf(stderr, "oracle_cli: bad input\n"); return 2; }
  if (p.res_w > 0) { W = p.res_w; H = p.res_h; }
  int w = p.w ? p.w : W, h = p.h ? p.h : H;
  std::vector<float> fb((size_t)w * h * 3);
  std::vector<unsigned char> u8((size_t)w * h * 3);
  oracle_stats st{};
  int rc = oracle_render(input.c_str(), tex.c_str(), &p, fb.data(), u8.data(), &st);
  if (rc) { fprintf(stderr, "oracle_cli: render failed (%d)\n", rc); return 1; }
  if (!fout.empty()) { std::ofstream f(fout, std::ios::binary); f.write((const char*)fb.data(), fb.size() * 4); }
  if (!pout.empty()) {  // image.cpp:53-83 P3 layout
    FILE* f = fopen(pout.c_str(), "w");
    fprintf(f, "P3\n%d %d\n255\n", w, h);
    for (int y = 0; y < h; ++y) {
      for (int x = 0; x < w; ++x) {
        size_t i = ((size_t)y * w + x) * 3;
        fprintf(f, "%d %d %d", u8[i], u8[i + 1], u8[i + 2]);
        if (x < w - 1) fputs("  ", f);
      }
      fputc('\n', f);
    }
    fclose(f);
  }
  printf("{\"width\": %d, \"height\": %d, \"rays\": %llu, \"box_tests\": %llu, \"prim_tests\": %llu, "
         "\"load_seconds\": %.6f, \"render_seconds\": %.6f, \"n_shapes\": %d, \"n_lights\": %d}\n",
         w, h, st.rays, st.box_tests, st.prim_tests, st.load_seconds, st.render_seconds, st.n_shapes, st.n_lights);
  return 0;
}
