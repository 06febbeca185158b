// Host check of Markstein division (rt_kernels.hip div_rn): q1 = fma(fma(-d, q, a), y, q) with q = a*y,
// y = RN(1/d), against a / d for random a, d with exponents in [2^-60, 2^60].
//   gcc -O2 -ffp-contract=off -mfma -o check_div scripts/check_div.c -lm && ./check_div
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline float fb(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
int main(void) {
  long bad = 0, n = 0;
  for (long k = 0; k < 2000000000L; ++k) {
    uint64_t v = xr();
    // exponents in [2^-40, 2^40] for both operands, random mantissas and signs
    uint32_t ea = 127 - 60 + (uint32_t)(v % 121), eb = 127 - 60 + (uint32_t)((v >> 8) % 121);
    float a = fb(((uint32_t)(v >> 16) & 0x807fffffu) | (ea << 23));
    float d = fb(((uint32_t)(v >> 40) & 0x807fffffu) | (eb << 23));
    float y = 1.0f / d;               // stands for rcp + Newton (== IEEE 1/d, verified exhaustively)
    float q = a * y;
    float r = fmaf(-d, q, a);
    float q1 = fmaf(r, y, q);
    float ref = a / d;
    ++n;
    if (memcmp(&q1, &ref, 4) != 0) { if (bad < 5) printf("a=%a d=%a got %a want %a\n", a, d, q1, ref); ++bad; }
  }
  printf("%ld of %ld differ\n", bad, n);
  return 0;
}
