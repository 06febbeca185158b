// ref_cpu.cpp — CPU oracle for the per-pixel render path of daRoyalCacti/Raytracing_GPU.
//
// TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg as the checker.  Nothing in raytracing_gpu_amd/ links or calls it.
//
// A restatement (not a translation) of the reference semantics, cited per function.  The object
// graph keeps the reference's shape (virtual hit()/scatter()/value(), hittable_list, the
// complete-binary-tree BVH with its random split axes) because the oracle has to reproduce the
// reference's draw order and tie-breaking, not be fast.  Every hazard of SURVEY.md's ledger that
// changes bits is reproduced or defined here (H1, H2, H3, H6, H8, H9, H13, H18, H19, H20, H23-H25).
//
// Floating point: IEEE binary32 with no contraction (-ffp-contract=off), evaluation order as
// written in the reference C++.  Transcendentals follow the shared deterministic definitions in
// raytracing_gpu_amd/csrc/rt_detmath.h (the reference's CUDA libdevice results are unpinnable).
#include "ref_cpu.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../raytracing_gpu_amd/csrc/rt_detmath.h"

namespace oref {

// ---------------------------------------------------------------- XORWOW (cuRAND semantics)
// curand_init(seed, subsequence, offset) scrambling + skipahead_sequence (2^67 stride) +
// skipahead; curand() recurrence; curand_uniform = x*2^-32 + 2^-33.  Call sites: render.h:91,
// scenes.h:30, vec3.h:8.
struct Rng {
  uint32_t d, v[5];
};

static inline uint32_t rng_next(Rng& s) {
  const uint32_t t = s.v[0] ^ (s.v[0] >> 2);
  s.v[0] = s.v[1];
  s.v[1] = s.v[2];
  s.v[2] = s.v[3];
  s.v[3] = s.v[4];
  s.v[4] = (s.v[4] ^ (s.v[4] << 4)) ^ (t ^ (t << 1));
  s.d += 362437u;
  return s.v[4] + s.d;
}
static inline float rng_uniform(Rng& s) {
  const float two_m32 = 2.3283064e-10f;
  return (float)rng_next(s) * two_m32 + two_m32 / 2.0f;
}

// A linear map on GF(2)^160 stored as the images of the 160 basis vectors (5 words each):
// the same layout cuRAND/rocRAND use for their precalc tables, m[5*(32*i+j)+k].
struct Mat160 {
  uint32_t w[800];
};
static void mat_apply(const Mat160& m, const uint32_t in[5], uint32_t out[5]) {
  uint32_t r[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 32; ++j)
      if (in[i] >> j & 1u)
        for (int k = 0; k < 5; ++k) r[k] ^= m.w[5 * (32 * i + j) + k];
  memcpy(out, r, sizeof(r));
}
static Mat160 mat_mul(const Mat160& a, const Mat160& b) {  // a∘b
  Mat160 c;
  for (int col = 0; col < 160; ++col) mat_apply(a, &b.w[5 * col], &c.w[5 * col]);
  return c;
}
static Mat160 step_matrix() {
  Mat160 m;
  for (int col = 0; col < 160; ++col) {
    Rng s{0, {0, 0, 0, 0, 0}};
    s.v[col / 32] = 1u << (col % 32);
    rng_next(s);
    for (int k = 0; k < 5; ++k) m.w[5 * col + k] = s.v[k];
  }
  return m;
}
struct JumpTables {
  Mat160 seq[32];  // A^(4^i * 2^67)
  Mat160 off[32];  // A^(4^i)
  JumpTables() {
    Mat160 a = step_matrix();
    off[0] = a;
    for (int i = 1; i < 32; ++i) {
      Mat160 sq = mat_mul(off[i - 1], off[i - 1]);
      off[i] = mat_mul(sq, sq);
    }
    Mat160 p = a;
    for (int i = 0; i < 67; ++i) p = mat_mul(p, p);
    seq[0] = p;
    for (int i = 1; i < 32; ++i) {
      Mat160 sq = mat_mul(seq[i - 1], seq[i - 1]);
      seq[i] = mat_mul(sq, sq);
    }
  }
};
static const JumpTables& jump_tables() {
  static JumpTables t;
  return t;
}
static void jump(Rng& s, uint64_t n, const Mat160* tab) {
  int mi = 0;
  while (n) {
    const unsigned digit = (unsigned)(n & 3u);
    for (unsigned t = 0; t < digit; ++t) mat_apply(tab[mi], s.v, s.v);
    n >>= 2;
    ++mi;
  }
}
static Rng rng_init(uint64_t seed, uint64_t subseq, uint64_t offset) {
  const uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
  const uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
  const uint32_t t0 = 1099087573u * s0;
  const uint32_t t1 = 2591861531u * s1;
  Rng s;
  s.d = 6615241u + t1 + t0;
  s.v[0] = 123456789u + t0;
  s.v[1] = 362436069u ^ t0;
  s.v[2] = 521288629u + t1;
  s.v[3] = 88675123u ^ t1;
  s.v[4] = 5783321u + t0;
  const JumpTables& jt = jump_tables();
  jump(s, subseq, jt.seq);
  jump(s, offset, jt.off);
  s.d += (uint32_t)offset * 362437u;
  return s;
}

// ---------------------------------------------------------------- vec3 (vec3.h:16-158)
struct V3 {
  float x, y, z;
  V3() : x(0), y(0), z(0) {}
  V3(float a, float b, float c) : x(a), y(b), z(c) {}
  float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
  float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
  V3 operator-() const { return V3(-x, -y, -z); }
  V3& operator+=(const V3& o) { x += o.x; y += o.y; z += o.z; return *this; }
  V3& operator*=(float t) { x *= t; y *= t; z *= t; return *this; }
  V3& operator*=(const V3& o) { x *= o.x; y *= o.y; z *= o.z; return *this; }
  float len2() const { return x * x + y * y + z * z; }
  float len() const { return std::sqrt(len2()); }
  bool near_zero() const {
    const float s = 1e-6f;
    return std::fabs(x) < s && std::fabs(y) < s && std::fabs(z) < s;
  }
};
static inline V3 operator+(const V3& a, const V3& b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 operator-(const V3& a, const V3& b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 operator*(const V3& a, const V3& b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 operator*(float t, const V3& v) { return V3(t * v.x, t * v.y, t * v.z); }
static inline V3 operator*(const V3& v, float t) { return t * v; }
static inline V3 operator/(const V3& v, float t) { return (1.0f / t) * v; }
static inline float dot(const V3& a, const V3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 cross(const V3& a, const V3& b) {
  return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline V3 unit(const V3& v) { return v / v.len(); }
static inline V3 reflect(const V3& v, const V3& n) { return v - 2.0f * dot(v, n) * n; }
static inline V3 refract(const V3& uv, const V3& n, float eta) {  // vec3.h:152-158
  const float c = std::fmin(dot(-uv, n), 1.0f);
  const V3 perp = eta * (uv + c * n);
  const V3 par = -std::sqrt(std::fabs((float)(1.0 - (double)perp.len2()))) * n;
  return perp + par;
}

// H9: the reference passes several RNG draws as arguments of one call; C++ leaves their order
// unspecified.  The oracle pins left-to-right; `rtl` flips it for the layout pin test.
struct Draw {
  Rng* s;
  bool rtl;
  float u() { return rng_uniform(*s); }
  float u(float a, float b) { return a + (b - a) * u(); }
  V3 v3(float a, float b) {  // vec3::random(s, min, max)  vec3.h:62-69
    float c[3];
    for (int k = 0; k < 3; ++k) c[rtl ? 2 - k : k] = u(a, b);
    return V3(c[0], c[1], c[2]);
  }
  V3 v3() {
    float c[3];
    for (int k = 0; k < 3; ++k) c[rtl ? 2 - k : k] = u();
    return V3(c[0], c[1], c[2]);
  }
  V3 in_sphere() {  // vec3.h:129-134
    for (;;) {
      const V3 p = v3(-1.0f, 1.0f);
      if (p.len2() < 1.0f) return p;
    }
  }
  V3 in_disk() {  // vec3.h:136-141
    for (;;) {
      float c[2];
      for (int k = 0; k < 2; ++k) c[rtl ? 1 - k : k] = u(-1.0f, 1.0f);
      const V3 p(c[0], c[1], 0.0f);
      if (p.len2() < 1.0f) return p;
    }
  }
  V3 unit_vec() { return unit(in_sphere()); }
};

struct Ray {
  V3 o, d;
  float tm;
  Ray() : tm(0) {}
  Ray(const V3& a, const V3& b, float t) : o(a), d(b), tm(t) {}
  V3 at(float t) const { return o + t * d; }
};

struct Material;
struct Rec {  // hit_record  hittable.h:8-23
  V3 p, n;
  const Material* m = nullptr;
  float t = 0;
  bool front = false;
  float u = 0, v = 0;
  void face(const Ray& r, const V3& out) {
    front = dot(r.d, out) < 0;
    n = front ? out : -out;
  }
};

struct Counters {
  long long seg = 0, node = 0, prim = 0, samples = 0;
};
static thread_local Counters* tl_cnt = nullptr;
// Optional capture of world-query rays (o, d, tm) for offline tree experiments.
static std::atomic<long long> g_cap_n{0};
static long long g_cap_max = 0;
static float* g_cap = nullptr;
static thread_local bool tl_h20 = false;

static inline int rand_int(Draw& g, int lo, int hi) {  // common.h:49-52 (may return hi+1: H20)
  const int r = (int)g.u((float)lo, (float)(hi + 1));
  if (r > hi) tl_h20 = true;
  return r;
}

// ---------------------------------------------------------------- aabb (aabb.h:19-119)
struct Box {
  V3 lo, hi;
  bool hit(const Ray& r, float tmin, double tmax) const {
    for (int a = 0; a < 3; ++a) {
      const float inv = 1.0f / r.d[a];
      float t0 = (lo[a] - r.o[a]) * inv;
      float t1 = (hi[a] - r.o[a]) * inv;
      if (inv < 0.0f) std::swap(t0, t1);
      tmin = t0 > tmin ? t0 : tmin;
      tmax = t1 < tmax ? t1 : tmax;
      if (tmax <= tmin) return false;
    }
    return true;
  }
};
static Box enclose(const Box& a, const Box& b) {
  return Box{V3(std::fmin(a.lo.x, b.lo.x), std::fmin(a.lo.y, b.lo.y), std::fmin(a.lo.z, b.lo.z)),
             V3(std::fmax(a.hi.x, b.hi.x), std::fmax(a.hi.y, b.hi.y), std::fmax(a.hi.z, b.hi.z))};
}

// ---------------------------------------------------------------- textures (texture.h, perlin.h)
struct Texture {
  virtual V3 value(float u, float v, const V3& p) const = 0;
  virtual ~Texture() {}
};
struct Solid : Texture {
  V3 c;
  explicit Solid(V3 a) : c(a) {}
  V3 value(float, float, const V3&) const override { return c; }
};
struct Checker : Texture {  // texture.h:26-46
  const Texture *even, *odd;
  Checker(const Texture* e, const Texture* o) : even(e), odd(o) {}
  V3 value(float u, float v, const V3& p) const override {
    const float s = rtm::det_sinf(10.0f * p.x) * rtm::det_sinf(10.0f * p.y) *
                    rtm::det_sinf(10.0f * p.z);
    return s < 0 ? odd->value(u, v, p) : even->value(u, v, p);
  }
};
struct Perlin {  // perlin.h:9-127
  V3 ranvec[256];
  int px[256], py[256], pz[256];
  explicit Perlin(Draw& g) {
    for (int i = 0; i < 256; ++i) ranvec[i] = unit(g.v3(-1.0f, 1.0f));
    perm(g, px);
    perm(g, py);
    perm(g, pz);
  }
  static void perm(Draw& g, int* p) {
    for (int i = 0; i < 256; ++i) p[i] = i;
    for (int i = 255; i > 0; --i) {
      int tg = rand_int(g, 0, i);
      if (tg > i) tg = i;  // H20: the reference would read p[i+1]; recorded via tl_h20
      std::swap(p[i], p[tg]);
    }
  }
  float noise(const V3& p) const {
    const float u = p.x - std::floor(p.x), v = p.y - std::floor(p.y), w = p.z - std::floor(p.z);
    const int i = (int)std::floor(p.x), j = (int)std::floor(p.y), k = (int)std::floor(p.z);
    const float uu = u * u * (3.0f - 2.0f * u);
    const float vv = v * v * (3.0f - 2.0f * v);
    const float ww = w * w * (3.0f - 2.0f * w);
    float acc = 0.0f;
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b)
        for (int c = 0; c < 2; ++c) {
          const V3& g = ranvec[px[(i + a) & 255] ^ py[(j + b) & 255] ^ pz[(k + c) & 255]];
          const V3 wv(u - (float)a, v - (float)b, w - (float)c);
          acc += ((float)a * uu + (float)(1 - a) * (1.0f - uu)) *
                 ((float)b * vv + (float)(1 - b) * (1.0f - vv)) *
                 ((float)c * ww + (float)(1 - c) * (1.0f - ww)) * dot(g, wv);
        }
    return acc;
  }
  float turb(V3 p, int depth) const {
    double acc = 0.0, w = 1.0;
    for (int i = 0; i < depth; ++i) {
      acc += w * (double)noise(p);
      w *= 0.5;
      p *= 2.0f;
    }
    return (float)std::fabs(acc);
  }
};
struct NoiseTex : Texture {  // texture.h:49-62
  Perlin pn;
  float sc;
  NoiseTex(Draw& g, float s) : pn(g), sc(s) {}
  V3 value(float, float, const V3& p) const override {
    return V3(1, 1, 1) * 0.5f * (float)(1.0 + (double)pn.noise(sc * p));
  }
};
struct TurbTex : Texture {  // texture.h:65-77
  Perlin pn;
  float sc;
  int depth;
  TurbTex(Draw& g, float s, int d = 7) : pn(g), sc(s), depth(d) {}
  V3 value(float, float, const V3& p) const override { return V3(1, 1, 1) * pn.turb(sc * p, depth); }
};
struct MarbleTex : Texture {  // texture.h:80-91
  Perlin pn;
  float sc;
  MarbleTex(Draw& g, float s) : pn(g), sc(s) {}
  V3 value(float, float, const V3& p) const override {
    return V3(1, 1, 1) * 0.5f * (1.0f + rtm::det_sinf(sc * p.z + 10.0f * pn.turb(sc * p, 7)));
  }
};

// ---------------------------------------------------------------- materials (material.h)
struct ImageTex : Texture {  // texture.h:125-163 (decoded texels owned here)
  std::vector<uint8_t> data;
  int w = 0, h = 0, bpp = 0;
  ImageTex(const uint8_t* d, int ww, int hh, int bb) : w(ww), h(hh), bpp(bb) {
    if (d && ww > 0 && hh > 0) data.assign(d, d + (size_t)ww * hh * bb);
  }
  V3 value(float u, float v, const V3&) const override {
    if (data.empty()) return V3(0, 1, 1);  // texture.h:146-147
    const float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);  // clamp_d, common.h:62-67
    const float vc = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
    const double vv = 1.0 - vc;  // double (texture.h:150)
    int i = (int)(uu * w);       // float * int -> float
    int j = (int)(vv * h);       // double * int -> double
    if (i >= w) i = w - 1;
    if (j >= h) j = h - 1;
    const float cs = 1.0f / 255.0f;
    const uint8_t* px = data.data() + (size_t)j * (bpp * w) + (size_t)i * bpp;
    return V3(cs * px[0], cs * px[1], cs * px[2]);
  }
};

struct Material {
  virtual bool scatter(const Ray& in, const Rec& r, V3& att, Ray& out, Draw& g) const = 0;
  virtual V3 emitted(float, float, const V3&) const { return V3(0, 0, 0); }
  virtual ~Material() {}
};
struct Lambert : Material {  // material.h:16-36
  const Texture* alb;
  explicit Lambert(const Texture* a) : alb(a) {}
  bool scatter(const Ray& in, const Rec& r, V3& att, Ray& out, Draw& g) const override {
    V3 dir = r.n + g.unit_vec();
    if (dir.near_zero()) dir = r.n;
    out = Ray(r.p, dir, in.tm);
    att = alb->value(r.u, r.v, r.p);
    return true;
  }
};
struct Metal : Material {  // material.h:39-56 (draws even when fuzz == 0: H8)
  const Texture* alb;
  float fuzz;
  Metal(const Texture* a, float f) : alb(a), fuzz(f) {}
  bool scatter(const Ray& in, const Rec& r, V3& att, Ray& out, Draw& g) const override {
    const V3 refl = reflect(unit(in.d), r.n);
    out = Ray(r.p, refl + fuzz * g.in_sphere(), in.tm);
    att = alb->value(r.u, r.v, r.p);
    return dot(out.d, r.n) > 0;
  }
};
struct Dielectric : Material {  // material.h:59-104
  float ir;
  explicit Dielectric(float i) : ir(i) {}
  bool scatter(const Ray& in, const Rec& r, V3& att, Ray& out, Draw& g) const override {
    att = V3(1.0f, 1.0f, 1.0f);
    const float ratio = r.front ? (1.0f / ir) : ir;
    const V3 ud = unit(in.d);
    const float c = std::fmin(dot(-ud, r.n), 1.0f);
    const float s = std::sqrt(1.0f - c * c);
    const bool tir = ratio * s > 1.0f;
    V3 dir;
    if (tir || reflectance(c, ratio) > g.u())  // short-circuit skips the draw on TIR (H8)
      dir = reflect(ud, r.n);
    else
      dir = refract(ud, r.n, ratio);
    out = Ray(r.p, dir, in.tm);
    return true;
  }
  static float reflectance(float c, float ri) {
    const float sr = (1.0f - ri) / (1.0f + ri);
    const float r0 = sr * sr;
    return r0 + (1.0f - r0) * rtm::det_pow5f(1.0f - c);
  }
};
struct Light : Material {  // material.h:107-122
  const Texture* e;
  explicit Light(const Texture* t) : e(t) {}
  bool scatter(const Ray&, const Rec&, V3&, Ray&, Draw&) const override { return false; }
  V3 emitted(float u, float v, const V3& p) const override { return e->value(u, v, p); }
};
struct Isotropic : Material {  // material.h:125-138
  const Texture* alb;
  explicit Isotropic(const Texture* a) : alb(a) {}
  bool scatter(const Ray& in, const Rec& r, V3& att, Ray& out, Draw& g) const override {
    out = Ray(r.p, g.in_sphere(), in.tm);
    att = alb->value(r.u, r.v, r.p);
    return true;
  }
};

// ---------------------------------------------------------------- hittables
struct Hittable {
  virtual bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw& g) const = 0;
  virtual bool bbox(float t0, float t1, Box& out) const = 0;
  virtual bool is_prim() const { return true; }  // containers are not counted as prim tests
  virtual ~Hittable() {}
};
static inline bool prim_hit(const Hittable* h, const Ray& r, float a, float b, Rec& rec, Draw& g) {
  if (tl_cnt && h->is_prim()) tl_cnt->prim++;
  return h->hit(r, a, b, rec, g);
}

struct Sphere : Hittable {  // sphere.h:35-78
  V3 c;
  float rad;
  const Material* m;
  Sphere(V3 cc, float r, const Material* mm) : c(cc), rad(r), m(mm) {}
  bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw&) const override {
    const V3 oc = r.o - c;
    const float a = r.d.len2();
    const float hb = dot(oc, r.d);
    const float cc = oc.len2() - rad * rad;
    const float disc = hb * hb - a * cc;
    if (disc < 0) return false;
    const float sq = std::sqrt(disc);
    const float root = (-hb - sq) / a;  // the "second root" retest repeats this value (H1)
    if (root < tmin || tmax < root) return false;
    rec.t = root;
    rec.p = r.at(root);
    const V3 out = (rec.p - c) / rad;
    rec.face(r, out);
    rec.m = m;
    rec.u = (rtm::det_atan2f(-out.z, out.x) + 3.1415927f) / (2.0f * 3.1415927f);
    rec.v = rtm::det_acosf(-out.y) / 3.1415927f;
    return true;
  }
  bool bbox(float, float, Box& o) const override {
    o = Box{c - V3(rad, rad, rad), c + V3(rad, rad, rad)};
    return true;
  }
};
struct MovingSphere : Hittable {  // moving_sphere.h:20-66
  V3 c0, c1;
  float t0, t1, rad;
  const Material* m;
  MovingSphere(V3 a, V3 b, float ta, float tb, float r, const Material* mm)
      : c0(a), c1(b), t0(ta), t1(tb), rad(r), m(mm) {}
  V3 center(float t) const { return c0 + ((t - t0) / (t1 - t0)) * (c1 - c0); }
  bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw&) const override {
    const V3 oc = r.o - center(r.tm);
    const float a = r.d.len2();
    const float hb = dot(oc, r.d);
    const float cc = oc.len2() - rad * rad;
    const float disc = hb * hb - a * cc;
    if (disc < 0) return false;
    const float sq = std::sqrt(disc);
    const float root = (-hb - sq) / a;
    if (root < tmin || tmax < root) return false;
    rec.t = root;
    rec.p = r.at(root);
    rec.face(r, (rec.p - center(r.tm)) / rad);
    rec.m = m;
    rec.u = 0.0f;  // H13: the reference leaves u,v stale; defined as 0 here and in the kernel
    rec.v = 0.0f;
    return true;
  }
  bool bbox(float a, float b, Box& o) const override {
    const V3 rr(rad, rad, rad);
    const Box b0{center(a) - rr, center(a) + rr}, b1{center(b) - rr, center(b) + rr};
    o = enclose(b0, b1);
    return true;
  }
};
// Axis-aligned rectangles (aarect.h:8-150).  `ax` is the axis of the normal: 2 = xy, 1 = xz, 0 = yz.
struct Rect : Hittable {
  int ax;
  float a0, a1, b0, b1, k;
  const Material* m;
  Rect(int axis, float p0, float p1, float q0, float q1, float kk, const Material* mm)
      : ax(axis), a0(p0), a1(p1), b0(q0), b1(q1), k(kk), m(mm) {}
  bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw&) const override {
    // (a,b) = (x,y) for xy, (x,z) for xz, (y,z) for yz.
    const int ia = ax == 0 ? 1 : 0, ib = ax == 2 ? 1 : 2;
    const float t = (k - r.o[ax]) / r.d[ax];
    if (t < tmin || t > tmax) return false;
    const float a = r.o[ia] + t * r.d[ia];
    const float b = r.o[ib] + t * r.d[ib];
    if (a < a0 || a > a1 || b < b0 || b > b1) return false;
    if (ax == 0) {  // yz_rect stores u from y and v from z
      rec.v = (b - b0) / (b1 - b0);
      rec.u = (a - a0) / (a1 - a0);
    } else {
      rec.u = (a - a0) / (a1 - a0);
      rec.v = (b - b0) / (b1 - b0);
    }
    rec.t = t;
    V3 nrm(0, 0, 0);
    nrm[ax] = 1.0f;
    rec.face(r, nrm);
    rec.m = m;
    rec.p = r.at(t);
    return true;
  }
  bool bbox(float, float, Box& o) const override {
    const float e = 0.0001f;
    if (ax == 2) o = Box{V3(a0, b0, k - e), V3(a1, b1, k + e)};
    else if (ax == 1) o = Box{V3(a0, k - e, b1), V3(a1, k + e, b1)};  // H4: z1 twice
    else o = Box{V3(k - e, a0, b0), V3(k + e, a1, b1)};
    return true;
  }
};
struct Triangle : Hittable {  // triangle.h:6-178
  V3 p0, p1, p2, e0, e1, n0, n1, n2;
  float uv[6];
  float d00, d01, d11, inv;
  bool vn = false;
  const Material* m;
  Triangle(V3 a, V3 b, V3 c, const float* tuv, const V3* n, const Material* mm) : p0(a), p1(b), p2(c), m(mm) {
    for (int k = 0; k < 6; ++k) uv[k] = tuv[k];
    e0 = p1 - p0;  // "v0", "v1" of triangle.h:26-27
    e1 = p2 - p0;
    d00 = dot(e0, e0);
    d01 = dot(e0, e1);
    d11 = dot(e1, e1);
    inv = 1.0f / (d00 * d11 - d01 * d01);
    if (n) {
      n0 = n[0];
      n1 = n[1];
      n2 = n[2];
      vn = true;
    }
  }
  bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw&) const override {  // :120-178
    const float eps = 0.0000001f;
    const V3 hh = cross(r.d, e1);
    const float a = dot(e0, hh);
    if (a > -eps && a < eps) return false;
    const float f = 1.0f / a;
    const V3 sv = r.o - p0;
    const float u = f * dot(sv, hh);
    if (u < 0.0f || u > 1.0f) return false;
    const V3 q = cross(sv, e0);
    const float v = f * dot(r.d, q);
    if ((v < 0.0f) | (u + v > 1.0f)) return false;
    const float t = f * dot(e1, q);
    if (t < tmin || t > tmax || t < eps) return false;
    rec.t = t;
    rec.m = m;
    rec.p = r.at(t);
    const V3 v2 = rec.p - p0;
    const float d20 = dot(v2, e0), d21 = dot(v2, e1);
    const float b0 = (d11 * d20 - d01 * d21) * inv;
    const float b1 = (d00 * d21 - d01 * d20) * inv;
    const float b2 = 1.0f - b0 - b1;
    rec.u = b2 * uv[0] + b0 * uv[2] + b1 * uv[4];
    rec.v = b2 * uv[1] + b0 * uv[3] + b1 * uv[5];
    if (!vn) {
      rec.face(r, cross(e1, e0));  // unnormalised face normal (H12)
    } else {
      const V3 nn(b2 * n0.x + b0 * n1.x + b1 * n2.x, b2 * n0.y + b0 * n1.y + b1 * n2.y,
                  b2 * n0.z + b0 * n1.z + b1 * n2.z);
      rec.face(r, nn);
    }
    return true;
  }
  bool bbox(float, float, Box& o) const override {  // :46-98, flat extents padded by 1e-4
    const V3 vs[3] = {p0, p1, p2};
    for (int k = 0; k < 3; ++k) {
      float lo = vs[0][k], hi = vs[0][k];
      for (int q = 1; q < 3; ++q) {
        if (vs[q][k] < lo) lo = vs[q][k];
        if (vs[q][k] > hi) hi = vs[q][k];
      }
      if (std::fabs(lo - hi) < 0.000001f) {
        hi += 0.0001f;
        lo -= 0.0001f;
      }
      o.lo[k] = lo;
      o.hi[k] = hi;
    }
    return true;
  }
};

struct List : Hittable {
  bool is_prim() const override { return false; }  // hittable_list.h:23-59 (later object wins ties)
  std::vector<const Hittable*> objs;
  bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw& g) const override {
    Rec tmp;
    bool any = false;
    float best = tmax;
    for (const Hittable* o : objs)
      if (prim_hit(o, r, tmin, best, tmp, g)) {
        any = true;
        best = tmp.t;
        rec = tmp;
      }
    return any;
  }
  bool bbox(float t0, float t1, Box& out) const override {
    if (objs.empty()) return false;
    Box tmp;
    bool first = true;
    for (const Hittable* o : objs) {
      if (!o->bbox(t0, t1, tmp)) return false;
      out = first ? tmp : enclose(out, tmp);
      first = false;
    }
    return true;
  }
};
struct BoxShape : Hittable {
  bool is_prim() const override { return false; }  // box.h:8-40
  V3 lo, hi;
  List sides;
  std::vector<std::unique_ptr<Rect>> own;
  BoxShape(V3 p0, V3 p1, const Material* m) : lo(p0), hi(p1) {
    own.emplace_back(new Rect(2, p0.x, p1.x, p0.y, p1.y, p1.z, m));
    own.emplace_back(new Rect(2, p0.x, p1.x, p0.y, p1.y, p0.z, m));
    own.emplace_back(new Rect(1, p0.x, p1.x, p0.z, p1.z, p1.y, m));
    own.emplace_back(new Rect(1, p0.x, p1.x, p0.z, p1.z, p0.y, m));
    own.emplace_back(new Rect(0, p0.y, p1.y, p0.z, p1.z, p1.x, m));
    own.emplace_back(new Rect(0, p0.y, p1.y, p0.z, p1.z, p0.x, m));
    for (auto& r : own) sides.objs.push_back(r.get());
  }
  bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw& g) const override {
    return sides.hit(r, tmin, tmax, rec, g);
  }
  bool bbox(float, float, Box& o) const override {
    o = Box{lo, hi};
    return true;
  }
};
struct Translate : Hittable {
  bool is_prim() const override { return false; }  // hittable.h:31-59
  const Hittable* ch;
  V3 off;
  Translate(const Hittable* c, V3 o) : ch(c), off(o) {}
  bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw& g) const override {
    const Ray mr(r.o - off, r.d, r.tm);
    if (!ch->hit(mr, tmin, tmax, rec, g)) return false;
    rec.p += off;
    rec.face(mr, rec.n);
    return true;
  }
  bool bbox(float t0, float t1, Box& o) const override {
    if (!ch->bbox(t0, t1, o)) return false;
    o = Box{o.lo + off, o.hi + off};
    return true;
  }
};
struct RotateY : Hittable {
  bool is_prim() const override { return false; }  // hittable.h:62-143
  const Hittable* ch;
  float sn, cs;
  bool has;
  Box bb;
  RotateY(const Hittable* c, float deg) : ch(c) {
    const float rad = deg * 3.1415927f / 180.0f;
    sn = rtm::det_sinf(rad);
    cs = rtm::det_cosf(rad);
    has = ch->bbox(0, 1, bb);
    V3 mn(INFINITY, INFINITY, INFINITY), mx(-INFINITY, -INFINITY, -INFINITY);
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int k = 0; k < 2; ++k) {
          const float x = (float)i * bb.hi.x + (float)(1 - i) * bb.lo.x;
          const float y = (float)j * bb.hi.y + (float)(1 - j) * bb.lo.y;
          const float z = (float)k * bb.hi.z + (float)(1 - k) * bb.lo.z;
          const V3 t(cs * x + sn * z, y, -sn * x + cs * z);
          for (int q = 0; q < 3; ++q) {
            mn[q] = std::fmin(mn[q], t[q]);
            mx[q] = std::fmax(mx[q], t[q]);
          }
        }
    bb = Box{mn, mx};
  }
  bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw& g) const override {
    V3 o = r.o, d = r.d;
    o[0] = cs * r.o[0] - sn * r.o[2];
    o[2] = sn * r.o[0] + cs * r.o[2];
    d[0] = cs * r.d[0] - sn * r.d[2];
    d[2] = sn * r.d[0] + cs * r.d[2];
    const Ray rr(o, d, r.tm);
    if (!ch->hit(rr, tmin, tmax, rec, g)) return false;
    V3 p = rec.p, n = rec.n;
    p[0] = cs * rec.p[0] + sn * rec.p[2];
    p[2] = -sn * rec.p[0] + cs * rec.p[2];
    n[0] = cs * rec.n[0] + sn * rec.n[2];
    n[2] = -sn * rec.n[0] + cs * rec.n[2];
    rec.p = p;
    rec.face(rr, n);  // H25: rotated-frame ray against the world-frame normal
    return true;
  }
  bool bbox(float, float, Box& o) const override {
    o = bb;
    return has;
  }
};
struct Medium : Hittable {
  bool is_prim() const override { return false; }  // constant_medium.h:34-70 (one RNG draw inside hit())
  const Hittable* bnd;
  const Material* phase;
  float neg_inv;
  Medium(const Hittable* b, float dens, const Material* ph) : bnd(b), phase(ph), neg_inv(-1.0f / dens) {}
  bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw& g) const override {
    Rec r1, r2;
    if (!bnd->hit(r, -INFINITY, INFINITY, r1, g)) return false;
    if (!bnd->hit(r, r1.t + 0.0001f, INFINITY, r2, g)) return false;
    if (r1.t < tmin) r1.t = tmin;
    if (r2.t > tmax) r2.t = tmax;
    if (r1.t >= r2.t) return false;
    if (r1.t < 0) r1.t = 0;
    const float len = r.d.len();
    const float inside = (r2.t - r1.t) * len;
    const float hd = neg_inv * rtm::det_logf(g.u());
    if (hd > inside) return false;
    rec.t = r1.t + hd / len;
    rec.p = r.at(rec.t);
    rec.n = V3(1, 0, 0);
    rec.front = true;
    rec.m = phase;
    rec.u = 0.0f;  // stale in the reference; defined as 0
    rec.v = 0.0f;
    return true;
  }
  bool bbox(float t0, float t1, Box& o) const override { return bnd->bbox(t0, t1, o); }
};

// Complete-binary-tree BVH with random split axes (bvh.h:16-436).
struct RefBvh : Hittable {
  bool is_prim() const override { return false; }
  std::vector<const Hittable*> objs;
  int n = 0, rows = 0;                 // rows = number of inner levels = ceil(log2 n)
  std::vector<int> num;                // objects below each inner node (heap order)
  std::vector<int> leaf_a, leaf_b;     // last-row inner nodes: object of left / right leaf (-1)
  std::vector<Box> bounds;             // inner nodes
  std::vector<int> axes;               // split axis drawn per inner node (record for fixtures)

  RefBvh(const std::vector<const Hittable*>& in, float time0, float time1, Draw& g) : objs(in) {
    n = (int)objs.size();
    rows = 0;
    while ((1 << rows) < n) ++rows;
    if (n < 3) { fprintf(stderr, "RefBvh: n < 3 unsupported\n"); abort(); }
    const int inner = (1 << rows) - 1;
    const int last0 = (1 << (rows - 1)) - 1;  // first node of the last inner row
    num.assign(inner, 0);
    num[0] = n;
    for (int k = 1; k < inner; ++k) {  // bvh.h:163-267: left gets floor, right gets the rest
      const int par = (k - 1) / 2;
      num[k] = (k & 1) ? num[par] / 2 : num[par] / 2 + num[par] % 2;
    }
    for (int k = last0; k < inner; ++k)
      if (num[k] < 1 || num[k] > 2) { fprintf(stderr, "RefBvh: bad layout\n"); abort(); }
    // Stable ascending order of bbox(0,0).min[axis] per axis (the merge sort of bvh.h:28-116).
    std::vector<int> sorted[3];
    for (int a = 0; a < 3; ++a) {
      std::vector<float> key(n);
      for (int i = 0; i < n; ++i) {
        Box b;
        objs[i]->bbox(0, 0, b);
        key[i] = b.lo[a];
      }
      sorted[a].resize(n);
      for (int i = 0; i < n; ++i) sorted[a][i] = i;
      std::stable_sort(sorted[a].begin(), sorted[a].end(),
                       [&](int x, int y) { return key[x] < key[y]; });
    }
    // Distribute objects top-down (bvh.h:290-322): one random axis per inner node in index order.
    std::vector<std::vector<char>> member(inner, std::vector<char>(n, 0));
    for (int i = 0; i < n; ++i) member[0][i] = 1;
    leaf_a.assign(inner, -1);
    leaf_b.assign(inner, -1);
    for (int k = 0; k < inner; ++k) {
      int ax = rand_int(g, 0, 2);
      axes.push_back(ax);
      if (ax > 2) ax = 2;  // H20 (reference reads obj_s[3]); recorded via tl_h20
      const bool last = k >= last0;
      const int nl = last ? (num[k] == 2 ? 1 : 1) : num[2 * k + 1];
      int cnt = 0;
      for (int i = 0; i < n; ++i) {
        const int o = sorted[ax][i];
        if (!member[k][o]) continue;
        if (last) {
          if (cnt < nl) leaf_a[k] = o; else leaf_b[k] = o;
        } else {
          member[cnt < nl ? 2 * k + 1 : 2 * k + 2][o] = 1;
        }
        ++cnt;
      }
    }
    bounds.resize(inner);
    for (int k = last0; k < inner; ++k) {
      Box b0;
      objs[leaf_a[k]]->bbox(time0, time1, b0);
      if (num[k] == 2) {
        Box b1;
        objs[leaf_b[k]]->bbox(time0, time1, b1);
        b0 = enclose(b0, b1);
      }
      bounds[k] = b0;
    }
    for (int k = last0 - 1; k >= 0; --k) bounds[k] = enclose(bounds[2 * k + 1], bounds[2 * k + 2]);
  }
  // Depth-first, left child first; every box is tested against the caller's [tmin, tmax]; leaves
  // keep strictly smaller t (first hit wins ties).  Same visiting order as bvh.h:348-436.
  void visit(int k, const Ray& r, float tmin, float tmax, Rec& rec, float& best, bool& any,
             Draw& g) const {
    if (tl_cnt) tl_cnt->node++;
    if (!bounds[k].hit(r, tmin, tmax)) return;
    if (k >= (1 << (rows - 1)) - 1) {
      Rec tmp;
      const int ids[2] = {leaf_a[k], leaf_b[k]};
      for (int q = 0; q < num[k]; ++q)
        if (prim_hit(objs[ids[q]], r, tmin, tmax, tmp, g) && tmp.t < best) {
          best = tmp.t;
          rec = tmp;
          any = true;
        }
      return;
    }
    visit(2 * k + 1, r, tmin, tmax, rec, best, any, g);
    visit(2 * k + 2, r, tmin, tmax, rec, best, any, g);
  }
  bool hit(const Ray& r, float tmin, float tmax, Rec& rec, Draw& g) const override {
    float best = INFINITY;
    bool any = false;
    visit(0, r, tmin, tmax, rec, best, any, g);
    return any;
  }
  bool bbox(float, float, Box& o) const override {
    o = bounds[0];
    return true;
  }
};

// ---------------------------------------------------------------- camera (camera.h:18-58)
struct Camera {
  V3 origin, llc, horiz, vert, u, v, w;
  float lens, t0, t1;
  Camera() {}
  Camera(V3 from, V3 at, V3 up, float vfov, float aspect, float aperture, float focus, float ta,
         float tb)
      : t0(ta), t1(tb) {
    const float theta = vfov * 3.1415927f / 180.0f;
    const float h = rtm::det_tanf(theta / 2.0f);
    const float vh = 2.0f * h;
    const float vw = aspect * vh;
    w = unit(from - at);
    u = unit(cross(up, w));
    v = cross(w, u);
    origin = from;
    horiz = focus * vw * u;
    vert = focus * vh * v;
    llc = origin - horiz / 2.0f - vert / 2.0f - focus * w;
    lens = aperture / 2.0f;
  }
  Ray ray(Draw& g, float s, float t) const {
    const V3 rd = lens * g.in_disk();
    const V3 off = u * rd.x + v * rd.y;
    const V3 o = origin + off;
    const V3 d = llc + s * horiz + t * vert - origin - off;
    return Ray(o, d, g.u(t0, t1));
  }
};

}  // namespace oref

using namespace oref;

// ---------------------------------------------------------------- scenes (scenes.h)
struct ref_scene {
  std::string name;
  float aspect = 16.0f / 9.0f;
  V3 background;
  Camera cam;
  const Hittable* world = nullptr;
  std::vector<std::unique_ptr<Hittable>> hs;
  std::vector<std::unique_ptr<Material>> ms;
  std::vector<std::unique_ptr<Texture>> ts;
  std::vector<float> table;  // big_scene1 object table, 13 floats per object
  std::vector<int> axes;
  bool h20 = false;

  template <class T, class... A> T* H(A&&... a) { T* p = new T(std::forward<A>(a)...); hs.emplace_back(p); return p; }
  template <class T, class... A> T* M(A&&... a) { T* p = new T(std::forward<A>(a)...); ms.emplace_back(p); return p; }
  template <class T, class... A> T* X(A&&... a) { T* p = new T(std::forward<A>(a)...); ts.emplace_back(p); return p; }
  const Material* lam(V3 c) { return M<Lambert>(X<Solid>(c)); }
  List* list(std::initializer_list<const Hittable*> l) {
    List* L = H<List>();
    for (auto* o : l) L->objs.push_back(o);
    return L;
  }
};

static const V3 kSky(0.7f, 0.8f, 1.0f);
static const V3 kBlack(0.0f, 0.0f, 0.0f);

static void build_basic(ref_scene& s) {  // scenes.h:82-100
  s.background = kSky;
  s.world = s.list({s.H<Sphere>(V3(0, 0, -1), 0.5f, s.lam(V3(0, 1, 0))),
                    s.H<Sphere>(V3(0, -100.5f, -1), 100.0f, s.lam(V3(0, 0, 1)))});
  s.cam = Camera(V3(0, 0, -3), V3(0, 0, 0), V3(0, 1, 0), 40, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
}
static void build_first(ref_scene& s) {  // scenes.h:106-137
  s.background = kSky;
  auto* g = s.lam(V3(0.8f, 0.8f, 0.0f));
  auto* c = s.lam(V3(0.1f, 0.2f, 0.3f));
  auto* l = s.M<Dielectric>(2.5f);
  auto* r = s.M<Metal>(s.X<Solid>(V3(0.8f, 0.6f, 0.2f)), 0.2f);
  auto* f = s.M<Dielectric>(2.0f);
  s.world = s.list({s.H<Sphere>(V3(0, -100.5f, -1), 100.0f, g), s.H<Sphere>(V3(0, 0, -1), 0.5f, c),
                    s.H<Sphere>(V3(-1, 0, -1), 0.5f, l), s.H<Sphere>(V3(1, 0, -1), 0.5f, r),
                    s.H<Sphere>(V3(0, 1, -0.75f), 0.25f, f), s.H<Sphere>(V3(0, 1, -0.75f), -0.25f, f)});
  s.cam = Camera(V3(-2, 2, -3), V3(0, 0, -1), V3(0, 1, 0), 20, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
}
// Object table row: type (0 sphere, 1 moving), material (0 lambertian, 1 metal, 2 dielectric),
// centre0, centre1, radius, albedo, fuzz-or-ir.
static void push_row(ref_scene& s, int type, int mtype, V3 c0, V3 c1, float r, V3 alb, float p) {
  const float row[13] = {(float)type, (float)mtype, c0.x, c0.y, c0.z, c1.x, c1.y, c1.z, r, alb.x, alb.y, alb.z, p};
  s.table.insert(s.table.end(), row, row + 13);
}
static void build_big1(ref_scene& s, Draw& g) {  // scenes.h:140-222 (C2)
  s.background = kSky;
  std::vector<const Hittable*> L;
  auto* checker = s.X<Checker>(s.X<Solid>(V3(0.2f, 0.3f, 0.1f)), s.X<Solid>(V3(0.9f, 0.9f, 0.9f)));
  L.push_back(s.H<Sphere>(V3(0, -1000, 0), 1000.0f, s.M<Lambert>(checker)));
  push_row(s, 0, 0, V3(0, -1000, 0), V3(0, -1000, 0), 1000.0f, V3(), 0);
  for (int a = -11; a < 11; ++a)
    for (int b = -11; b < 11; ++b) {
      const float choose = g.u();
      float cx, cz;
      if (!g.rtl) { cx = (float)a + 0.9f * g.u(); cz = (float)b + 0.9f * g.u(); }
      else { cz = (float)b + 0.9f * g.u(); cx = (float)a + 0.9f * g.u(); }
      const V3 c(cx, 0.2f, cz);
      if ((c - V3(4, 0.2f, 0)).len2() > 0.9f * 0.9f) {
        if ((double)choose < 0.8) {
          V3 a1, a2;
          if (!g.rtl) { a1 = g.v3(); a2 = g.v3(); } else { a2 = g.v3(); a1 = g.v3(); }
          const V3 alb = a1 * a2;
          const V3 c2 = c + V3(0, g.u(0.0f, 0.5f), 0);
          L.push_back(s.H<MovingSphere>(c, c2, 0.0f, 1.0f, 0.2f, s.lam(alb)));
          push_row(s, 1, 0, c, c2, 0.2f, alb, 0.0f);
        } else if ((double)choose < 0.95) {
          const V3 alb = g.v3(0.5f, 1.0f);
          const float fuzz = g.u(0.0f, 0.5f);
          L.push_back(s.H<Sphere>(c, 0.2f, s.M<Metal>(s.X<Solid>(alb), fuzz)));
          push_row(s, 0, 1, c, c, 0.2f, alb, fuzz);
        } else {
          L.push_back(s.H<Sphere>(c, 0.2f, s.M<Dielectric>(1.5f)));
          push_row(s, 0, 2, c, c, 0.2f, V3(), 1.5f);
        }
      } else {
        L.push_back(s.H<Sphere>(V3(10000, -10000, 10000), 0.00001f, s.lam(V3(0, 0, 0))));
        push_row(s, 0, 0, V3(10000, -10000, 10000), V3(10000, -10000, 10000), 0.00001f, V3(), 0);
      }
    }
  L.push_back(s.H<Sphere>(V3(0, 1, 0), 1.0f, s.M<Dielectric>(1.5f)));
  push_row(s, 0, 2, V3(0, 1, 0), V3(0, 1, 0), 1.0f, V3(), 1.5f);
  L.push_back(s.H<Sphere>(V3(-4, 1, 0), 1.0f, s.lam(V3(0.4f, 0.2f, 0.1f))));
  push_row(s, 0, 0, V3(-4, 1, 0), V3(-4, 1, 0), 1.0f, V3(0.4f, 0.2f, 0.1f), 0.0f);
  L.push_back(s.H<Sphere>(V3(4, 1, 0), 1.0f, s.M<Metal>(s.X<Solid>(V3(0.7f, 0.6f, 0.5f)), 0.0f)));
  push_row(s, 0, 1, V3(4, 1, 0), V3(4, 1, 0), 1.0f, V3(0.7f, 0.6f, 0.5f), 0.0f);
  auto* bvh = s.H<RefBvh>(L, 0.0f, 1.0f, g);
  s.axes = bvh->axes;
  s.world = s.list({bvh});
  s.cam = Camera(V3(13.0f, 2.0f, -3.0f), V3(0, 0, 0), V3(0, 1, 0), 20, 16.0f / 9.0f, 0.1f, 10.0f, 0, 1);
}
static void build_two_spheres(ref_scene& s) {  // scenes.h:225-243
  s.background = kSky;
  auto* ck = s.X<Checker>(s.X<Solid>(V3(0.2f, 0.3f, 0.1f)), s.X<Solid>(V3(0.9f, 0.9f, 0.9f)));
  s.world = s.list({s.H<Sphere>(V3(0, -10, 0), 10.0f, s.M<Lambert>(ck)),
                    s.H<Sphere>(V3(0, 10, 0), 10.0f, s.M<Lambert>(ck))});
  s.cam = Camera(V3(13, 2, 3), V3(0, 0, 0), V3(0, 1, 0), 20, 16.0f / 9.0f, 0.1f, 10.0f, 0, 1);
}
static void build_two_perlin(ref_scene& s, Draw& g) {  // scenes.h:248-274
  // The reference copies a temporary perlin whose destructor frees the tables it keeps pointing
  // at (texture.h:56,71,85): undefined.  Defined here as each texture owning its own tables.
  s.background = kSky;
  auto* t1 = s.X<MarbleTex>(g, 4.0f);
  auto* t2 = s.X<TurbTex>(g, 5.0f);
  s.world = s.list({s.H<Sphere>(V3(0, -1000, 0), 1000.0f, s.M<Lambert>(t1)),
                    s.H<Sphere>(V3(0, 2, 0), 2.0f, s.M<Lambert>(t2))});
  s.cam = Camera(V3(13, 2, 3), V3(0, 0, 0), V3(0, 1, 0), 20, 16.0f / 9.0f, 0.1f, 10.0f, 0, 1);
}
static void build_cornell(ref_scene& s, bool smoke) {  // scenes.h:323-404
  s.background = kBlack;
  s.aspect = 1.0f;
  auto* red = s.lam(V3(0.65f, 0.05f, 0.05f));
  auto* white = s.lam(V3(0.73f, 0.73f, 0.73f));
  auto* green = s.lam(V3(0.12f, 0.45f, 0.15f));
  auto* light = s.M<Light>(s.X<Solid>(V3(15, 15, 15)));
  List* L = s.H<List>();
  L->objs.push_back(s.H<Rect>(0, 0.0f, 555.0f, 0.0f, 555.0f, 555.0f, green));
  L->objs.push_back(s.H<Rect>(0, 0.0f, 555.0f, 0.0f, 555.0f, 0.0f, red));
  if (smoke) L->objs.push_back(s.H<Rect>(1, 113.0f, 443.0f, 127.0f, 432.0f, 554.0f, light));
  else L->objs.push_back(s.H<Rect>(1, 213.0f, 343.0f, 227.0f, 332.0f, 554.0f, light));
  L->objs.push_back(s.H<Rect>(1, 0.0f, 555.0f, 0.0f, 555.0f, 0.0f, white));
  L->objs.push_back(s.H<Rect>(1, 0.0f, 555.0f, 0.0f, 555.0f, 555.0f, white));
  L->objs.push_back(s.H<Rect>(2, 0.0f, 555.0f, 0.0f, 555.0f, 555.0f, white));
  const Hittable* b1 = s.H<BoxShape>(V3(0, 0, 0), V3(165, 330, 165), white);
  b1 = s.H<RotateY>(b1, 15.0f);
  b1 = s.H<Translate>(b1, V3(265, 0, 295));
  const Hittable* b2 = s.H<BoxShape>(V3(0, 0, 0), V3(165, 165, 165), white);
  b2 = s.H<RotateY>(b2, -18.0f);
  b2 = s.H<Translate>(b2, V3(130, 0, 65));
  if (smoke) {
    b1 = s.H<Medium>(b1, 0.01f, s.M<Isotropic>(s.X<Solid>(V3(0, 0, 0))));
    b2 = s.H<Medium>(b2, 0.01f, s.M<Isotropic>(s.X<Solid>(V3(1, 1, 1))));
  }
  L->objs.push_back(b1);
  L->objs.push_back(b2);
  s.world = L;
  s.cam = Camera(V3(278, 278, -800), V3(278, 278, 0), V3(0, 1, 0), 40, 1.0f, 0.0f, 10.0f, 0, 1);
}

// triangle_scene, scenes.h:409-428.
static void build_triangle(ref_scene& s) {
  s.background = kSky;
  const float uv[6] = {0, 0, 0, 1, 1, 0};
  s.world = s.list({s.H<Triangle>(V3(-0.5f, 0, 0), V3(0, 1, 10), V3(0.0f, 0, 0), uv, nullptr, s.lam(V3(0, 1, 0))),
                    s.H<Sphere>(V3(0, -100.5f, -1), 100.0f, s.lam(V3(0, 0, 1)))});
  s.cam = Camera(V3(0, 0, -3), V3(0, 0, 0), V3(0, 1, 0), 40, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
}
// triangles_scene, scenes.h:432-475: triangle_mesh = bvh_node over 4 triangles (world_init state).
static void build_triangles(ref_scene& s, Draw& g) {
  s.background = kSky;
  const float uv[6] = {0, 0, 0, 1, 1, 0};
  std::vector<const Hittable*> t = {
      s.H<Triangle>(V3(-0.5f, 0, 0), V3(0, 1, 10), V3(0.5f, 0, 0), uv, nullptr, s.lam(V3(0, 1, 0))),
      s.H<Triangle>(V3(0.5f, 0, 0), V3(0, 1, 10), V3(0.5f, 1, 0), uv, nullptr, s.lam(V3(1, 1, 0))),
      s.H<Triangle>(V3(1.5f, 0, 0), V3(0, 2, 10), V3(1.5f, 1, 0), uv, nullptr, s.lam(V3(1, 1, 1))),
      s.H<Triangle>(V3(1.5f, 0, 0), V3(1.5f, 1, 10), V3(1.5f, 0, 2), uv, nullptr, s.lam(V3(1, 1, 1)))};
  s.world = s.list({s.H<RefBvh>(t, 0.0f, 1.0f, g), s.H<Sphere>(V3(0, -100.5f, -1), 100.0f, s.lam(V3(0, 0, 1)))});
  s.cam = Camera(V3(0, 0, -3), V3(0, 0, 0), V3(0, 1, 0), 40, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
}
// earth_scene, scenes.h:278-320.
static bool build_earth(ref_scene& s, const ref_assets* a) {
  if (!a || a->n_images < 1) return false;
  s.background = kBlack;
  const ref_image& im = a->images[0];
  auto* tex = s.X<ImageTex>(im.data, im.width, im.height, im.bytes_per_pixel);
  s.world = s.list({s.H<Sphere>(V3(0, 0, 0), 2.0f, s.M<Lambert>(tex)),
                    s.H<Rect>(2, -5.0f, 5.0f, -3.0f, 3.0f, 6.0f, s.M<Light>(s.X<Solid>(V3(4.0f, 4.0f, 4.0f))))});
  s.cam = Camera(V3(13.0f, 0.0f, 3.0f), V3(0.0f, 0.0f, 0.0f), V3(0, 1, 0), 20, 16.0f / 9.0f, 0.1f, 10.0f, 0, 1);
  return true;
}
// One triangle_mesh of create_meshes_d (triangle_mesh.h:147-204): lambertian(image_texture).
static const Hittable* build_mesh(ref_scene& s, const ref_assets* a, const ref_mesh& m, Draw& g) {
  const Texture* tex;
  if (m.image >= 0 && m.image < a->n_images) {
    const ref_image& im = a->images[m.image];
    tex = s.X<ImageTex>(im.data, im.width, im.height, im.bytes_per_pixel);
  } else {
    tex = s.X<ImageTex>(nullptr, 0, 0, 0);
  }
  const Material* mat = s.M<Lambert>(tex);
  std::vector<const Hittable*> t;
  for (int k = 0; k < m.n_triangles; ++k) {
    const float* d = m.data + 24 * (size_t)k;
    const V3 n[3] = {V3(d[9], d[10], d[11]), V3(d[12], d[13], d[14]), V3(d[15], d[16], d[17])};
    t.push_back(s.H<Triangle>(V3(d[0], d[1], d[2]), V3(d[3], d[4], d[5]), V3(d[6], d[7], d[8]), d + 18,
                              m.vertex_normals ? n : nullptr, mat));
  }
  return s.H<RefBvh>(t, 0.0f, 1.0f, g);
}
// door_scene / cup_scene, scenes.h:478-523,576-621.
static bool build_mesh_scene(ref_scene& s, const ref_assets* a, Draw& g, V3 from, V3 at) {
  if (!a || a->n_meshes < 1 || !a->meshes[0].data || a->meshes[0].n_triangles < 3) return false;
  s.background = kSky;
  s.world = s.list({build_mesh(s, a, a->meshes[0], g), s.H<Sphere>(V3(0, -100, -1), 100.0f, s.lam(V3(0, 1, 0)))});
  s.cam = Camera(from, at, V3(0, 1, 0), 20, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
  return true;
}
// backpack_scene, scenes.h:526-572: only the ground sphere remains (H17).
static void build_backpack(ref_scene& s) {
  s.background = kSky;
  s.world = s.list({s.H<Sphere>(V3(0, -100, -1), 100.0f, s.lam(V3(0, 1, 0)))});
  s.cam = Camera(V3(0, 0, -3), V3(0, 0, 0), V3(0, 1, 0), 20, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
}

// Config C5 final scene: the composition defined in rt_scene.cpp (scene_final) / DESIGN.md,
// restated with the reference's hittable types (box.h boxes under a bvh_node, constant_medium,
// translate(rotate_y(...)), triangle_mesh).
static bool build_final(ref_scene& s, const ref_assets* a, Draw& g) {
  if (!a || a->n_images < 1 || a->n_meshes < 1 || !a->meshes[0].data || a->meshes[0].n_triangles < 3) return false;
  s.background = kBlack;
  const Material* ground = s.lam(V3(0.48f, 0.83f, 0.53f));
  std::vector<const Hittable*> boxes;
  for (int i = 0; i < 20; ++i)
    for (int j = 0; j < 20; ++j) {
      const float w = 100.0f;
      const float x0 = -1000.0f + (float)i * w, z0 = -1000.0f + (float)j * w, y0 = 0.0f;
      const float x1 = x0 + w, y1 = g.u(1.0f, 101.0f), z1 = z0 + w;
      boxes.push_back(s.H<BoxShape>(V3(x0, y0, z0), V3(x1, y1, z1), ground));
    }
  List* L = s.H<List>();
  L->objs.push_back(s.H<RefBvh>(boxes, 0.0f, 1.0f, g));
  L->objs.push_back(s.H<Rect>(1, 123.0f, 423.0f, 147.0f, 412.0f, 554.0f, s.M<Light>(s.X<Solid>(V3(7, 7, 7)))));
  const V3 c1(400, 400, 200), c2 = c1 + V3(30, 0, 0);
  L->objs.push_back(s.H<MovingSphere>(c1, c2, 0.0f, 1.0f, 50.0f, s.lam(V3(0.7f, 0.3f, 0.1f))));
  L->objs.push_back(s.H<Sphere>(V3(260, 150, 45), 50.0f, s.M<Dielectric>(1.5f)));
  L->objs.push_back(s.H<Sphere>(V3(0, 150, 145), 50.0f, s.M<Metal>(s.X<Solid>(V3(0.8f, 0.8f, 0.9f)), 1.0f)));
  const Hittable* boundary = s.H<Sphere>(V3(360, 150, 145), 70.0f, s.M<Dielectric>(1.5f));
  L->objs.push_back(boundary);
  L->objs.push_back(s.H<Medium>(boundary, 0.2f, s.M<Isotropic>(s.X<Solid>(V3(0.2f, 0.4f, 0.9f)))));
  const Hittable* fog = s.H<Sphere>(V3(0, 0, 0), 5000.0f, s.M<Dielectric>(1.5f));
  L->objs.push_back(s.H<Medium>(fog, 0.0001f, s.M<Isotropic>(s.X<Solid>(V3(1, 1, 1)))));
  const ref_image& im = a->images[0];
  L->objs.push_back(s.H<Sphere>(V3(400, 200, 400), 100.0f,
                                s.M<Lambert>(s.X<ImageTex>(im.data, im.width, im.height, im.bytes_per_pixel))));
  L->objs.push_back(s.H<Sphere>(V3(220, 280, 300), 80.0f, s.M<Lambert>(s.X<NoiseTex>(g, 0.1f))));
  const Material* white = s.lam(V3(0.73f, 0.73f, 0.73f));
  std::vector<const Hittable*> balls;
  for (int k = 0; k < 1000; ++k) balls.push_back(s.H<Sphere>(g.v3(0.0f, 165.0f), 10.0f, white));
  L->objs.push_back(s.H<Translate>(s.H<RotateY>(s.H<RefBvh>(balls, 0.0f, 1.0f, g), 15.0f), V3(-100, 270, 395)));
  ref_mesh m = a->meshes[0];
  std::vector<float> scaled(m.data, m.data + 24 * (size_t)m.n_triangles);
  for (int t = 0; t < m.n_triangles; ++t)
    for (int q = 0; q < 9; ++q) scaled[24 * (size_t)t + q] *= 150.0f;
  m.data = scaled.data();
  L->objs.push_back(s.H<Translate>(s.H<RotateY>(build_mesh(s, a, m, g), -30.0f), V3(30, 101, 150)));
  s.world = L;
  s.cam = Camera(V3(478, 278, -600), V3(278, 278, 0), V3(0, 1, 0), 40, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
  return true;
}

// Test scenes "coincident" / "coincident_step" (not in scenes.h; parity fixtures of the list and BVH
// tie rules, the same compositions as rt_scene.cpp's scene_coincident).  "coincident": xy_rects lying
// in the plane z = 0 in three kinds of list entries -- a primitive, members of a bvh_node and a
// translate(rotate_y(.., 0)) instance (rotate_y by 0 and a translation in x, y leave the ray's z terms
// exact) -- so world queries meet exact ties across entries (hittable_list.h:23-39: t_max = the
// closest so far, inclusive, the later entry wins) and inside the BVH (bvh.h: strictly closer, the
// first visited wins); the BVH also holds an xz_rect (H4 box), spheres and a rect behind the plane.
// "coincident_step": a BVH, then primitives; a triangle repeated bit for bit inside the BVH and once
// more after it (triangle.h's t depends on v0, e0, e1 only, so equal triangles tie exactly).
static void build_coincident(ref_scene& s, Draw& g, bool step) {
  s.background = kSky;
  auto* red = s.lam(V3(0.8f, 0.1f, 0.1f));
  auto* green = s.lam(V3(0.1f, 0.8f, 0.1f));
  auto* yellow = s.lam(V3(0.8f, 0.8f, 0.1f));
  auto* blue = s.lam(V3(0.1f, 0.2f, 0.8f));
  auto* cyan = s.lam(V3(0.1f, 0.8f, 0.8f));
  auto* grey = s.lam(V3(0.5f, 0.5f, 0.5f));
  auto* metal = s.M<Metal>(s.X<Solid>(V3(0.8f, 0.8f, 0.8f)), 0.05f);
  auto* glass = s.M<Dielectric>(1.5f);
  const Hittable* ground = nullptr;
  if (step) {
    const float uv[6] = {0, 0, 1, 0, 0, 1};
    const V3 a(-1.0f, -1.5f, 0.0f), b(2.0f, -1.5f, 0.0f), c(-1.0f, 0.5f, 0.0f), d(2.0f, 0.5f, 0.0f);
    std::vector<const Hittable*> L = {
        s.H<Triangle>(a, b, c, uv, nullptr, green), s.H<Triangle>(b, d, c, uv, nullptr, blue),
        s.H<Sphere>(V3(2.2f, -0.3f, -0.8f), 0.5f, metal), s.H<Triangle>(a, b, c, uv, nullptr, yellow),
        s.H<Sphere>(V3(-2.0f, 0.2f, -1.0f), 0.6f, glass)};
    const Hittable* bvh = s.H<RefBvh>(L, 0.0f, 1.0f, g);
    const Hittable* again = s.H<Triangle>(a, b, c, uv, nullptr, red);
    ground = s.H<Sphere>(V3(0.0f, -101.7f, 0.0f), 100.0f, grey);
    s.world = s.list({bvh, again, ground});
  } else {
    std::vector<const Hittable*> L = {
        s.H<Rect>(2, -1.0f, 2.0f, -1.5f, 0.5f, 0.0f, green),
        s.H<Rect>(2, -3.0f, 3.0f, 0.8f, 2.0f, 0.5f, blue),
        s.H<Sphere>(V3(2.2f, -0.3f, -0.8f), 0.5f, metal),
        s.H<Rect>(2, -0.5f, 0.7f, -1.2f, -0.2f, 0.0f, yellow),
        s.H<Rect>(1, -3.0f, 3.0f, -3.0f, 3.0f, -1.6f, grey),
        s.H<Sphere>(V3(-2.0f, 0.2f, -1.0f), 0.6f, glass)};
    const Hittable* bvh = s.H<RefBvh>(L, 0.0f, 1.0f, g);
    const Hittable* prim = s.H<Rect>(2, -2.0f, 0.5f, -1.0f, 1.0f, 0.0f, red);
    ground = s.H<Sphere>(V3(0.0f, -101.7f, 0.0f), 100.0f, grey);
    const Hittable* inst = s.H<Translate>(s.H<RotateY>(s.H<Rect>(2, -0.75f, 1.25f, -0.6f, 1.1f, 0.0f, cyan), 0.0f),
                                          V3(0.25f, 0.1f, 0.0f));
    s.world = s.list({prim, bvh, inst, ground});
  }
  s.cam = Camera(V3(0.3f, 0.4f, -6.0f), V3(0, 0, 0), V3(0, 1, 0), 40, 16.0f / 9.0f, 0.1f, 6.0f, 0, 1);
}

// ---------------------------------------------------------------- integrator (render.h:55-113)
static V3 trace(const ref_scene& s, Ray r, Draw& g, int depth) {
  V3 att(1, 1, 1);
  for (int i = 0; i < depth; ++i) {
    Rec rec;
    if (tl_cnt) tl_cnt->seg++;
    if (g_cap) {
      const long long k = g_cap_n.fetch_add(1);
      if (k < g_cap_max) {
        float* e = g_cap + 8 * k;
        e[0] = r.o.x; e[1] = r.o.y; e[2] = r.o.z; e[3] = r.d.x; e[4] = r.d.y; e[5] = r.d.z; e[6] = r.tm; e[7] = (float)i;  // e[7]: bounce depth (0 = camera ray)
      }
    }
    if (!s.world->hit(r, 0.001f, INFINITY, rec, g)) return att * s.background;
    Ray sc;
    V3 a;
    const V3 em = rec.m->emitted(rec.u, rec.v, rec.p);
    if (rec.m->scatter(r, rec, a, sc, g)) {
      att *= a;
      r = sc;
    } else {
      return att * em;
    }
  }
  return V3(0, 0, 0);
}

static void render_pixel(const ref_scene& s, int i, int j, int W, int H, int spp, int fb_id,
                         int depth, int cam_mode, float* out) {
  const long long N = (long long)W * H;
  const long long p = (long long)j * W + i;
  const long long slot = ((long long)(fb_id + 1) * p + fb_id + 1) % N;  // render.h:101 (H3)
  Rng local = rng_init(1984, (uint64_t)slot, 0);
  Rng cam0 = rng_init(1984, 0, 0);  // H2 REF mode: private pristine copy of slot 0
  Draw gl{&local, false};
  Draw gc{cam_mode == REF_CAM_PER_PIXEL ? &local : &cam0, false};
  V3 col(0, 0, 0);
  for (int k = 0; k < spp; ++k) {
    const float u = ((float)i + gl.u()) / (float)W;
    const float v = ((float)j + gl.u()) / (float)H;
    const Ray r = s.cam.ray(gc, u, v);
    col += trace(s, r, gl, depth);
    if (tl_cnt) tl_cnt->samples++;
  }
  const V3 f = col / (float)spp;
  out[0] = f.x;
  out[1] = f.y;
  out[2] = f.z;
}

// ---------------------------------------------------------------- C API
extern "C" {

int ref_scene_create_ex(const char* name, int rtl, const ref_assets* a, ref_scene** out) {
  std::unique_ptr<ref_scene> s(new ref_scene);
  s->name = name;
  Rng st = rng_init(1984, 0, 0);  // world_init  scenes.h:28-32
  Draw g{&st, rtl != 0};
  tl_h20 = false;
  const std::string n(name);
  if (n == "basic") build_basic(*s);
  else if (n == "first") build_first(*s);
  else if (n == "big1" || n == "random") build_big1(*s, g);
  else if (n == "two_spheres") build_two_spheres(*s);
  else if (n == "two_perlin") build_two_perlin(*s, g);
  else if (n == "cornell") build_cornell(*s, false);
  else if (n == "cornell_smoke") build_cornell(*s, true);
  else if (n == "triangle") build_triangle(*s);
  else if (n == "triangles") build_triangles(*s, g);
  else if (n == "backpack") build_backpack(*s);
  else if (n == "earth") { if (!build_earth(*s, a)) return 1; }
  else if (n == "door") { if (!build_mesh_scene(*s, a, g, V3(-3, 4, -5), V3(0, 1, 0))) return 1; }
  else if (n == "cup") { if (!build_mesh_scene(*s, a, g, V3(0, 0, -1), V3(0, 0, 0))) return 1; }
  else if (n == "final") { if (!build_final(*s, a, g)) return 1; }
  else if (n == "coincident") build_coincident(*s, g, false);
  else if (n == "coincident_step") build_coincident(*s, g, true);
  else return 1;
  s->h20 = tl_h20;
  *out = s.release();
  return 0;
}
int ref_scene_create(const char* name, int rtl, ref_scene** out) { return ref_scene_create_ex(name, rtl, nullptr, out); }
void ref_scene_destroy(ref_scene* s) { delete s; }
long long ref_capture_rays(float* buf, long long max_rays) {  // buf = NULL stops capturing
  const long long n = g_cap_n.exchange(0);
  g_cap = buf;
  g_cap_max = buf ? max_rays : 0;
  return n;
}
float ref_scene_aspect(const ref_scene* s) { return s->aspect; }
void ref_scene_background(const ref_scene* s, float rgb[3]) {
  rgb[0] = s->background.x;
  rgb[1] = s->background.y;
  rgb[2] = s->background.z;
}
int ref_scene_h20(const ref_scene* s) { return s->h20 ? 1 : 0; }
void ref_scene_set_camera(ref_scene* s, const float from[3], const float at[3], float vfov,
                          float aperture, float focus) {
  s->cam = Camera(V3(from[0], from[1], from[2]), V3(at[0], at[1], at[2]), V3(0, 1, 0), vfov,
                  s->aspect, aperture, focus, 0, 1);
}
int ref_scene_table(const ref_scene* s, float* out, int max_rows) {
  const int rows = (int)s->table.size() / 13;
  if (out) memcpy(out, s->table.data(), sizeof(float) * 13 * std::min(rows, max_rows));
  return rows;
}
int ref_scene_bvh_axes(const ref_scene* s, int* out, int max_n) {
  const int n = (int)s->axes.size();
  if (out)
    for (int i = 0; i < max_n; ++i) out[i] = i < n ? s->axes[i] : -1;
  return n;
}

int ref_render(const ref_scene* s, int W, int H, int spp, int fb_id, int max_depth, int cam_mode,
               int row0, int row_step, int nthreads, float* fb, int* seg_per_pixel,
               ref_counters* counters) {
  if (!s || W <= 0 || H <= 0 || spp <= 0 || row_step <= 0 || row0 < 0) return 1;
  std::vector<int> rows;
  for (int j = row0; j < H; j += row_step) rows.push_back(j);
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
  nthreads = std::max(1, std::min<int>(nthreads, (int)rows.size()));
  std::vector<Counters> cs(nthreads);
  std::atomic<int> next{0};
  auto work = [&](int t) {
    tl_cnt = &cs[t];
    for (;;) {
      const int r = next.fetch_add(1);
      if (r >= (int)rows.size()) break;
      const int j = rows[r];
      for (int i = 0; i < W; ++i) {
        const long long before = cs[t].seg;
        render_pixel(*s, i, j, W, H, spp, fb_id, max_depth, cam_mode, fb + 3 * ((size_t)j * W + i));
        if (seg_per_pixel) seg_per_pixel[(size_t)j * W + i] = (int)(cs[t].seg - before);
      }
    }
    tl_cnt = nullptr;
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  if (counters) {
    memset(counters, 0, sizeof(*counters));
    for (auto& c : cs) {
      counters->segments += c.seg;
      counters->node_tests += c.node;
      counters->prim_tests += c.prim;
      counters->samples += c.samples;
    }
  }
  return 0;
}

static inline int quant(float x) {  // color.h:40-44 (NaN defined as 0)
  const float r = std::sqrt(x);
  if (!(r == r)) return 0;
  const float c = r < 0.0f ? 0.0f : (r > 0.999f ? 0.999f : r);
  return (int)(256.0f * c);
}
void ref_quantize_fb(const float* fb, int W, int H, uint8_t* out) {
  size_t o = 0;
  for (int j = H - 1; j >= 0; --j)
    for (int i = 0; i < W; ++i)
      for (int c = 0; c < 3; ++c) out[o++] = (uint8_t)quant(fb[3 * ((size_t)j * W + i) + c]);
}
void ref_average(const uint8_t* const* ppms, int nfb, int W, int H, uint8_t* out) {
  const size_t n = (size_t)W * H * 3;
  std::vector<float> acc(n, 0.0f);
  for (int f = 0; f < nfb; ++f)
    for (size_t k = 0; k < n; ++k) {
      const int c = ppms[f][k];
      acc[k] += (float)(c * c) / (255.0f * 255.0f);
    }
  for (size_t k = 0; k < n; ++k) out[k] = (uint8_t)quant(acc[k] / (float)nfb);
}

void ref_xorwow_init(uint64_t seed, uint64_t subsequence, uint64_t offset, uint32_t st[6]) {
  const Rng s = rng_init(seed, subsequence, offset);
  st[0] = s.d;
  for (int k = 0; k < 5; ++k) st[1 + k] = s.v[k];
}
uint32_t ref_xorwow_next(uint32_t st[6]) {
  Rng s;
  s.d = st[0];
  for (int k = 0; k < 5; ++k) s.v[k] = st[1 + k];
  const uint32_t r = rng_next(s);
  st[0] = s.d;
  for (int k = 0; k < 5; ++k) st[1 + k] = s.v[k];
  return r;
}
float ref_xorwow_uniform(uint32_t st[6]) {
  const float two_m32 = 2.3283064e-10f;
  return (float)ref_xorwow_next(st) * two_m32 + two_m32 / 2.0f;
}
void ref_xorwow_jump_matrix(int which, int i, uint32_t out[800]) {
  const JumpTables& t = jump_tables();
  memcpy(out, (which == 0 ? t.seq : t.off)[i].w, 800 * 4);
}

}  // extern "C"
