// rt_main.cpp — the reference's main.cu (main.cu:8-45) rewritten against the C ABI: a C++ host
// program that owns the scene and calls draw() through include/rt_hip.h (one GPU) or
// include/rt_multi.h (the frame buffer tiled over several GPUs, one RCCL gather).
//
//   rt_main SCENE WIDTH SPP_PER_FB NO_FB OUT.ppm [options]
//     --devices 0,1,...     tile over these devices with rt_multi (default: one GPU, rt_draw)
//     --gather rccl|host    rt_multi's gather (default rccl; host lets ranks share a device)
//     --band-rows B         rows per band for rt_multi (default 4)
//     --repeat K            draw K times (the first draw is cold, later ones reuse the schedule)
//     --depth D             max_depth (default 50)
//     --obj PATH            mesh scenes: rt_obj_load (assimp's OBJ import, reference indexing)
//     --tex PATH            texture for the mesh / earth scenes: rt_image_load (stb_image bytes)
//
// Writes OUT.ppm (binary P6, top row first) and one JSON line per draw on stdout.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_hip.h"
#include "rt_multi.h"

namespace {

// render.h:21-50 (the reference's render_settings, unchanged in meaning)
struct render_settings {
  float aspect_ratio = 16.0f / 9.0f;
  int image_width = 1200;
  int image_height = 0;
  int samples_per_pixel_per_fb = 100;
  int no_fb = 10;
  int max_depth = 50;
  int rays_per_pixel = 0;
  void calc_all() {
    image_height = static_cast<int>(image_width / (double)aspect_ratio);  // H18
    rays_per_pixel = samples_per_pixel_per_fb * no_fb;
  }
};

int die(const char* what, const char* msg) {
  fprintf(stderr, "rt_main: %s: %s\n", what, msg ? msg : "");
  return 99;  // checkCudaErrors' exit code (common.h:30-38)
}

std::vector<int> parse_devices(const char* s) {
  std::vector<int> d;
  while (*s) {
    d.push_back(atoi(s));
    const char* c = strchr(s, ',');
    if (!c) break;
    s = c + 1;
  }
  return d;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: rt_main SCENE WIDTH SPP_PER_FB NO_FB OUT.ppm [--devices 0,1] [--gather rccl|host] "
                    "[--band-rows B] [--repeat K] [--depth D] [--obj PATH] [--tex PATH]\n");
    return 2;
  }
  const char* name = argv[1];
  render_settings s;
  s.image_width = atoi(argv[2]);
  s.samples_per_pixel_per_fb = atoi(argv[3]);
  s.no_fb = atoi(argv[4]);
  const char* out = argv[5];
  std::vector<int> devices;
  int gather = RT_GATHER_RCCL, band_rows = 4, repeat = 1;
  const char *obj_path = nullptr, *tex_path = nullptr;
  for (int k = 6; k < argc; ++k) {
    const std::string a = argv[k];
    const char* v = k + 1 < argc ? argv[k + 1] : "";
    if (a == "--devices") devices = parse_devices(v), ++k;
    else if (a == "--gather") gather = strcmp(v, "host") == 0 ? RT_GATHER_HOST : RT_GATHER_RCCL, ++k;
    else if (a == "--band-rows") band_rows = atoi(v), ++k;
    else if (a == "--repeat") repeat = atoi(v), ++k;
    else if (a == "--depth") s.max_depth = atoi(v), ++k;
    else if (a == "--obj") obj_path = v, ++k;
    else if (a == "--tex") tex_path = v, ++k;
    else return die("unknown option", argv[k]);
  }

  // ---- scene: the reference's `door_scene curr_scene;` etc. (main.cu:17-18) as the host library
  rt_scene_host* scene = nullptr;
  rt_obj_mesh* obj = nullptr;
  rt_image_host* tex = nullptr;
  if (obj_path || tex_path) {
    rt_image_asset img = {};
    rt_mesh_asset mesh = {};
    rt_scene_assets assets = {};
    if (tex_path) {  // make_image(): stbi_load(path, .., 0) bytes
      if (rt_image_load(tex_path, &tex)) return die("rt_image_load", tex_path);
      img = *rt_image_view(tex);
      assets.n_images = 1;
      assets.images = &img;
    }
    if (obj_path) {  // create_meshes(): assimp Triangulate | GenNormals, create_meshes_d indexing (H16)
      if (rt_obj_load(obj_path, RT_OBJ_INDEX_REFERENCE, &obj)) return die("rt_obj_load", obj_path);
      const rt_obj_info* oi = rt_obj_view(obj);
      mesh = rt_mesh_asset{oi->n_triangles, 1, 0, 0, oi->triangles};
      assets.n_meshes = 1;
      assets.meshes = &mesh;
    }
    if (rt_scene_build_ex(name, &assets, &scene)) return die("rt_scene_build_ex", name);
    if (obj) rt_obj_free(obj);  // the scene owns copies
    if (tex) rt_image_free(tex);
  } else if (rt_scene_build(name, &scene)) {
    return die("rt_scene_build", name);
  }
  const rt_scene_soa* soa = rt_scene_view(scene);
  s.aspect_ratio = soa->aspect;  // main.cu:27
  s.calc_all();

  rt_render_args a = {};
  a.width = s.image_width;
  a.height = s.image_height;
  a.spp = s.samples_per_pixel_per_fb;
  a.fb_first = 0;
  a.fb_count = s.no_fb;
  a.max_depth = s.max_depth;
  a.cam_mode = RT_CAM_REF_SLOT0;
  a.band_rows = devices.empty() ? a.height : band_rows;
  a.band_first = 0;
  a.band_stride = 1;
  a.seed = 1984;  // render.h:91
  std::vector<uint8_t> png(3 * (size_t)a.width * a.height);
  rt_counters c = {};

  rt_ctx* ctx = nullptr;
  rt_multi* multi = nullptr;
  if (devices.empty()) {
    if (rt_ctx_create(0, &ctx)) return die("rt_ctx_create", "device 0");
    if (rt_scene_upload(ctx, soa)) return die("rt_scene_upload", rt_last_error(ctx));
  } else {
    int rc = rt_multi_create((int)devices.size(), devices.data(), gather, &multi);
    if (rc) return die("rt_multi_create", gather == RT_GATHER_RCCL ? "RCCL communicator (distinct devices?)" : "");
    if (rt_multi_upload(multi, soa)) return die("rt_multi_upload", rt_multi_last_error(multi));
  }
  for (int k = 0; k < repeat; ++k) {
    const auto t0 = std::chrono::steady_clock::now();
    rt_multi_timing tm = {};
    if (ctx) {
      if (rt_draw(ctx, &a, png.data(), &c)) return die("rt_draw", rt_last_error(ctx));
    } else if (rt_multi_draw(multi, &a, png.data(), &c, &tm)) {
      return die("rt_multi_draw", rt_multi_last_error(multi));
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"draw\": %d, \"scene\": \"%s\", \"width\": %d, \"height\": %d, \"ranks\": %d, \"wall_ms\": %.3f, "
           "\"segments\": %llu, \"samples\": %llu",
           k, name, a.width, a.height, ctx ? 1 : (int)devices.size(), ms, (unsigned long long)c.segments,
           (unsigned long long)c.samples);
    if (multi) {
      printf(", \"warm\": %d, \"render_ms_max\": %.3f, \"gather_ms\": %.3f, \"gather_bytes\": %.0f, \"kernel_ms\": [",
             tm.warm, tm.render_ms_max, tm.gather_ms, tm.gather_bytes);
      for (size_t r = 0; r < devices.size(); ++r) printf("%s%.3f", r ? ", " : "", tm.kernel_ms[r]);
      printf("]");
    }
    printf("}\n");
    fflush(stdout);
  }
  // average_images wrote the PNG with png++ (color.h:125-170); a binary PPM carries the same bytes
  FILE* f = fopen(out, "wb");
  if (!f) return die("open", out);
  fprintf(f, "P6\n%d %d\n255\n", a.width, a.height);
  fwrite(png.data(), 1, png.size(), f);
  fclose(f);
  if (ctx) rt_ctx_destroy(ctx);
  if (multi) rt_multi_destroy(multi);
  rt_scene_free(scene);
  return 0;
}
