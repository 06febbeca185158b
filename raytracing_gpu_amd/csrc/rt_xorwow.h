// rt_xorwow.h — cuRAND-compatible XORWOW for host scene generation and the gfx950 kernels.
//
// Semantics pinned in SURVEY.md §8c: curand_init's seed scrambling (salts 0xaad26b49 /
// 0xf7dcefdd, multipliers 1099087573 / 2591861531), the xorshift+Weyl recurrence, the 2^67
// subsequence stride, and curand_uniform(x) = float(x)*2^-32 + 2^-33 in (0, 1].
// (rocrand_init/rocrand_uniform differ in both the salts and the uniform mapping, so they are not
// used.)  The jump matrices are derived here from the recurrence itself.
#pragma once

#include <stdint.h>

#include "rt_detmath.h"

namespace rtx {

struct State {
  uint32_t d, v[5];
};

RT_HD uint32_t next(State& s) {
  const uint32_t t = s.v[0] ^ (s.v[0] >> 2);
  s.v[0] = s.v[1];
  s.v[1] = s.v[2];
  s.v[2] = s.v[3];
  s.v[3] = s.v[4];
  s.v[4] = (s.v[4] ^ (s.v[4] << 4)) ^ (t ^ (t << 1));
  s.d += 362437u;
  return s.v[4] + s.d;
}

// curand_uniform: exact scaling by 2^-32 of the RNE-converted word, plus 2^-33.
RT_HD float uniform(State& s) {
  return (float)next(s) * 2.3283064365386963e-10f + 1.1641532182693481e-10f;
}

// curand_init(seed, 0, 0).
RT_HD State seed_state(uint64_t seed) {
  const uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
  const uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
  const uint32_t t0 = 1099087573u * s0;
  const uint32_t t1 = 2591861531u * s1;
  State s;
  s.d = 6615241u + t1 + t0;
  s.v[0] = 123456789u + t0;
  s.v[1] = 362436069u ^ t0;
  s.v[2] = 521288629u + t1;
  s.v[3] = 88675123u ^ t1;
  s.v[4] = 5783321u + t0;
  return s;
}

// Linear map on GF(2)^160 as the images of the basis vectors: m[5*(32*word+bit)+k].
RT_HD void mat_apply(const uint32_t* m, const uint32_t in[5], uint32_t out[5]) {
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
  for (int b = 0; b < 160; ++b) {
    const uint32_t mask = 0u - ((in[b >> 5] >> (b & 31)) & 1u);
    const uint32_t* row = m + 5 * b;
    r0 ^= row[0] & mask;
    r1 ^= row[1] & mask;
    r2 ^= row[2] & mask;
    r3 ^= row[3] & mask;
    r4 ^= row[4] & mask;
  }
  out[0] = r0; out[1] = r1; out[2] = r2; out[3] = r3; out[4] = r4;
}

// Host: seq[i] = A^(4^i * 2^67) for i < 32 (32 x 800 words), the subsequence jump tables.
inline void build_sequence_jumps(uint32_t* seq /* 32*800 */) {
  static uint32_t a[800], t[800], u[800];
  for (int col = 0; col < 160; ++col) {
    State s{0, {0, 0, 0, 0, 0}};
    s.v[col >> 5] = 1u << (col & 31);
    next(s);
    for (int k = 0; k < 5; ++k) a[5 * col + k] = s.v[k];
  }
  auto square = [](const uint32_t* x, uint32_t* y) {
    for (int col = 0; col < 160; ++col) mat_apply(x, x + 5 * col, y + 5 * col);
  };
  for (int i = 0; i < 67; ++i) {
    square(a, t);
    for (int k = 0; k < 800; ++k) a[k] = t[k];
  }
  for (int k = 0; k < 800; ++k) seq[k] = a[k];
  for (int i = 1; i < 32; ++i) {
    square(seq + 800 * (i - 1), t);
    square(t, u);
    for (int k = 0; k < 800; ++k) seq[800 * i + k] = u[k];
  }
}

}  // namespace rtx
