// ref_cpu_cli — command-line driver for the CPU oracle (test infrastructure only).
// usage: ref_cpu_cli scene W H spp_per_fb no_fb max_depth cam_mode threads out.ppm
// Renders the fbs in order, quantises and averages them like draw() (render.h:118-174) and
// writes a binary PPM of the averaged image.  Prints segments and wall time on stderr.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ref_cpu.h"

int main(int argc, char** argv) {
  if (argc < 10) {
    fprintf(stderr, "usage: %s scene W H spp no_fb depth cam_mode threads out.ppm\n", argv[0]);
    return 2;
  }
  ref_scene* s = nullptr;
  if (ref_scene_create(argv[1], 0, &s)) {
    fprintf(stderr, "unknown scene %s\n", argv[1]);
    return 2;
  }
  const int W = atoi(argv[2]), H = atoi(argv[3]), spp = atoi(argv[4]), nfb = atoi(argv[5]);
  const int depth = atoi(argv[6]), cam = atoi(argv[7]), th = atoi(argv[8]);
  std::vector<float> fb((size_t)W * H * 3);
  std::vector<std::vector<uint8_t>> q(nfb, std::vector<uint8_t>((size_t)W * H * 3));
  std::vector<const uint8_t*> qp;
  long long segs = 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int f = 0; f < nfb; ++f) {
    ref_counters c;
    ref_render(s, W, H, spp, f, depth, cam, 0, 1, th, fb.data(), nullptr, &c);
    segs += c.segments;
    ref_quantize_fb(fb.data(), W, H, q[f].data());
    qp.push_back(q[f].data());
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::vector<uint8_t> img((size_t)W * H * 3);
  ref_average(qp.data(), nfb, W, H, img.data());
  FILE* f = fopen(argv[9], "wb");
  fprintf(f, "P6\n%d %d\n255\n", W, H);
  fwrite(img.data(), 1, img.size(), f);
  fclose(f);
  fprintf(stderr, "segments %lld time %.3f s  %.3f Mrays/s  h20 %d\n", segs, dt, segs / dt * 1e-6,
          ref_scene_h20(s));
  ref_scene_destroy(s);
  return 0;
}
