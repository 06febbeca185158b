// rt_detmath.h — deterministic transcendentals shared by the gfx950 kernel and host code.
//
// The reference calls CUDA libdevice sinf/cosf/tanf/logf/acosf/atan2f/pow on the hot path
// (texture.h:38 checker sin, constant_medium.h:57 log, material.h:102 pow, sphere.h:25-26
// acosf/atan2f, camera.h:27 tan, hittable.h:80-81 sin/cos).  Their exact bit patterns are not
// reproducible off NVIDIA hardware, so this project DEFINES each function as the float rounding
// of a double-precision evaluation built only from IEEE +,-,*,/ and floor.  Those operations are
// correctly rounded on x86-64 SSE2 and on gfx950 (v_*_f64, div_scale/fmas/fixup), so the same
// source yields the same bits on host and device as long as FP contraction is off on both
// (-ffp-contract=off everywhere).  Accuracy is close to correctly rounded float results.
#pragma once

#ifdef __HIPCC__
#define RT_HD __host__ __device__ inline
#else
#define RT_HD inline
#endif

#include <stdint.h>
#include <string.h>

namespace rtm {

RT_HD uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
RT_HD float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

RT_HD double dfloor(double x) { return __builtin_floor(x); }

// sin / cos of a reduced argument |r| <= pi/4 (fdlibm kernel coefficients, plain Horner).
RT_HD double ksin(double x) {
  const double z = x * x;
  const double r = 8.33333333332248946124e-03 +
                   z * (-1.98412698298579493134e-04 +
                        z * (2.75573137070700676789e-06 +
                             z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
  return x + (z * x) * (-1.66666666666666324348e-01 + z * r);
}
RT_HD double kcos(double x) {
  const double z = x * x;
  const double r =
      z * (4.16666666666666019037e-02 +
           z * (-1.38888888888741095749e-03 +
                z * (2.48015872894767294178e-05 +
                     z * (-2.75573143513906633035e-07 +
                          z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
  return 1.0 - (0.5 * z - z * r);
}

// Cody-Waite reduction by pi/2 (three parts; exact products for |k| < 2^20).
// Returns quadrant in q and the reduced argument.
RT_HD double reduce_pio2(double x, int& q) {
  const double fn = dfloor(x * 6.36619772367581382433e-01 + 0.5);
  const double r = ((x - fn * 1.57079632673412561417e+00) - fn * 6.07710050630396597660e-11) -
                   fn * 2.02226624871116645580e-21;
  q = (int)(((long long)fn) & 3);
  return r;
}

RT_HD bool finite_small(float x) {
  const float a = x < 0 ? -x : x;
  return a <= 1.0e9f;  // also false for NaN
}

RT_HD double sin_d(double x, bool& ok) {
  int q;
  const double r = reduce_pio2(x, q);
  ok = true;
  switch (q) {
    case 0: return ksin(r);
    case 1: return kcos(r);
    case 2: return -ksin(r);
    default: return -kcos(r);
  }
}
RT_HD double cos_d(double x) {
  int q;
  const double r = reduce_pio2(x, q);
  switch (q) {
    case 0: return kcos(r);
    case 1: return -ksin(r);
    case 2: return -kcos(r);
    default: return ksin(r);
  }
}

RT_HD float det_sinf(float x) {
  if (!finite_small(x)) return u2f(0x7fc00000u);
  bool ok;
  return (float)sin_d((double)x, ok);
}
RT_HD float det_cosf(float x) {
  if (!finite_small(x)) return u2f(0x7fc00000u);
  return (float)cos_d((double)x);
}
RT_HD float det_tanf(float x) {
  if (!finite_small(x)) return u2f(0x7fc00000u);
  bool ok;
  return (float)(sin_d((double)x, ok) / cos_d((double)x));
}

// Natural log of a float via log(m) = 2 atanh(s), s = (m-1)/(m+1), m in [sqrt(1/2), sqrt(2)).
RT_HD float det_logf(float x) {
  const uint32_t u = f2u(x);
  if (x != x) return x;
  if (x == 0.0f) return u2f(0xff800000u);
  if (u & 0x80000000u) return u2f(0x7fc00000u);
  if (u == 0x7f800000u) return x;
  int e;
  double m;
  if ((u & 0x7f800000u) == 0) {  // subnormal: scale up by 2^32
    const double sx = (double)x * 4294967296.0;
    uint64_t b;
    memcpy(&b, &sx, 8);
    e = (int)((b >> 52) & 0x7ff) - 1023 - 32;
    b = (b & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
    memcpy(&m, &b, 8);
  } else {
    e = (int)((u >> 23) & 0xff) - 127;
    m = (double)u2f((u & 0x007fffffu) | 0x3f800000u);
  }
  if (m > 1.41421356237309504880) {
    m = m * 0.5;
    e += 1;
  }
  const double s = (m - 1.0) / (m + 1.0);
  const double z = s * s;
  double p = 1.0 / 23.0;
  p = 1.0 / 21.0 + z * p;
  p = 1.0 / 19.0 + z * p;
  p = 1.0 / 17.0 + z * p;
  p = 1.0 / 15.0 + z * p;
  p = 1.0 / 13.0 + z * p;
  p = 1.0 / 11.0 + z * p;
  p = 1.0 / 9.0 + z * p;
  p = 1.0 / 7.0 + z * p;
  p = 1.0 / 5.0 + z * p;
  p = 1.0 / 3.0 + z * p;
  p = 1.0 + z * p;
  const double lm = 2.0 * s * p;
  return (float)((double)e * 6.93147180559945286227e-01 + lm);
}

// x^5 (material.h:102 pow(1-cos, 5)).
RT_HD float det_pow5f(float x) {
  const double d = (double)x;
  const double d2 = d * d;
  return (float)(d2 * d2 * d);
}

// atan for 0 <= z <= tan(pi/8) by its Taylor series (21 terms).
RT_HD double katan(double u) {
  const double z = u * u;
  double p = -1.0 / 43.0;
  p = 1.0 / 41.0 + z * p;
  p = -1.0 / 39.0 + z * p;
  p = 1.0 / 37.0 + z * p;
  p = -1.0 / 35.0 + z * p;
  p = 1.0 / 33.0 + z * p;
  p = -1.0 / 31.0 + z * p;
  p = 1.0 / 29.0 + z * p;
  p = -1.0 / 27.0 + z * p;
  p = 1.0 / 25.0 + z * p;
  p = -1.0 / 23.0 + z * p;
  p = 1.0 / 21.0 + z * p;
  p = -1.0 / 19.0 + z * p;
  p = 1.0 / 17.0 + z * p;
  p = -1.0 / 15.0 + z * p;
  p = 1.0 / 13.0 + z * p;
  p = -1.0 / 11.0 + z * p;
  p = 1.0 / 9.0 + z * p;
  p = -1.0 / 7.0 + z * p;
  p = 1.0 / 5.0 + z * p;
  p = -1.0 / 3.0 + z * p;
  p = 1.0 + z * p;
  return u * p;
}
// atan of a non-negative finite double.
RT_HD double atan_pos(double z) {
  const double PIO2 = 1.57079632679489655800e+00;
  const double PIO4 = 7.85398163397448278999e-01;
  bool inv = false;
  if (z > 1.0) {
    z = 1.0 / z;
    inv = true;
  }
  double a;
  if (z > 4.14213562373095034e-01)
    a = PIO4 + katan((z - 1.0) / (z + 1.0));
  else
    a = katan(z);
  return inv ? PIO2 - a : a;
}
RT_HD double atan2_d(double y, double x) {
  const double PI = 3.14159265358979311600e+00;
  const double PIO2 = 1.57079632679489655800e+00;
  if (x != x || y != y) return x + y;
  const double ay = y < 0 ? -y : y;
  const double ax = x < 0 ? -x : x;
  const bool xneg = x < 0 || (x == 0 && (1.0 / x) < 0);
  const bool yneg = y < 0 || (y == 0 && (1.0 / y) < 0);
  double a;
  if (ay == 0.0) {
    a = xneg ? PI : 0.0;
  } else if (ax == 0.0) {
    a = PIO2;
  } else if (ax == ay && ax == __builtin_inf()) {
    a = xneg ? 3.0 * PIO2 * 0.5 : PIO2 * 0.5;
  } else if (ay == __builtin_inf()) {
    a = PIO2;
  } else if (ax == __builtin_inf()) {
    a = xneg ? PI : 0.0;
  } else {
    const double base = atan_pos(ay / ax);
    a = xneg ? PI - base : base;
  }
  return yneg ? -a : a;
}
RT_HD float det_atan2f(float y, float x) { return (float)atan2_d((double)y, (double)x); }

// acos(x) = atan2(sqrt(1-x^2), x); the square root is one Newton step in double from a
// correctly-rounded float seed (IEEE sqrtf on both sides) so no f64 sqrt lowering is involved.
RT_HD float det_acosf(float x) {
  if (x != x || x > 1.0f || x < -1.0f) return u2f(0x7fc00000u);
  const double d = (double)x;
  const double w = (1.0 - d) * (1.0 + d);
  double s = 0.0;
  if (w > 0.0) {
    s = (double)__builtin_sqrtf((float)w);
    if (s > 0.0) s = 0.5 * (s + w / s);
  }
  return (float)atan2_d(s, d);
}

// checker_texture's test det_sinf(a) * det_sinf(b) * det_sinf(c) < 0 (texture.h:38-40), same
// result at a fraction of the cost: for 2^-20 <= |x| <= 2^17 the sign of det_sinf(x) is the
// parity of floor(x / pi) (verified for every float in that range by scripts/check_checker_sign.cpp),
// no factor is zero and the float product cannot underflow, so the product is negative iff an
// odd number of factors are.  Outside that range (or NaN) the full product is evaluated.
RT_HD bool sin_neg_fast(float x, bool& ok) {
  const float a = x < 0 ? -x : x;
  ok = a >= 9.5367431640625e-07f && a <= 131072.0f;  // also false for NaN
  const double k = dfloor((double)x * 3.18309886183790671538e-01);
  return (((long long)k) & 1) != 0;
}
RT_HD bool checker_odd(float a, float b, float c) {
  bool oa, ob, oc;
  const bool na = sin_neg_fast(a, oa), nb = sin_neg_fast(b, ob), nc = sin_neg_fast(c, oc);
  if (oa && ob && oc) return (na ^ nb ^ nc);
  return det_sinf(a) * det_sinf(b) * det_sinf(c) < 0.0f;
}

}  // namespace rtm
