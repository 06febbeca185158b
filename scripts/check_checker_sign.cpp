// Exhaustive check of rtm::sin_neg_fast against the sign of rtm::det_sinf for every float with
// 2^-20 <= |x| <= 2^17 (both signs).  Also checks |det_sinf| is never 0 or subnormal there, so the
// checker product cannot underflow.  usage: check_checker_sign [stride]  (stride 1 = exhaustive)
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../raytracing_gpu_amd/csrc/rt_detmath.h"

int main(int argc, char** argv) {
  const unsigned stride = argc > 1 ? (unsigned)atoi(argv[1]) : 1u;
  float lo = 9.5367431640625e-07f, hi = 131072.0f;
  uint32_t ulo, uhi;
  memcpy(&ulo, &lo, 4);
  memcpy(&uhi, &hi, 4);
  long long checked = 0, bad = 0;
  float minmag = 1.0f;
  for (uint32_t u = ulo; u <= uhi; u += stride) {
    for (int sgn = 0; sgn < 2; ++sgn) {
      float x;
      uint32_t w = u | (sgn ? 0x80000000u : 0u);
      memcpy(&x, &w, 4);
      bool ok;
      const bool neg = rtm::sin_neg_fast(x, ok);
      const float sv = rtm::det_sinf(x);
      const float mag = sv < 0 ? -sv : sv;
      if (mag < minmag) minmag = mag;
      if (!ok || neg != (sv < 0.0f) || mag < 1.1754944e-38f) {
        if (bad < 10) printf("mismatch x=%a det_sinf=%a fast_neg=%d ok=%d\n", x, sv, neg, ok);
        ++bad;
      }
      ++checked;
    }
  }
  printf("checked %lld floats, mismatches %lld, min |det_sinf| %g\n", checked, bad, minmag);
  return bad ? 1 : 0;
}
