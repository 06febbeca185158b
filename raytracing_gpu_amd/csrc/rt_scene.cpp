// rt_scene.cpp — host-side scene library: builds the reference's scenes as flattened arrays.
//
// Replaces the <<<1,1>>> create_*_world kernels of scenes.h and the device-side bvh_node build
// (bvh.h:163-346).  The host owns camera, object list, materials, textures and the BVH as plain
// structs; rt_scene_upload() copies them to the device.  Scene content follows the reference's
// RNG draw order exactly (world_init = curand_init(1984,0,0), scenes.h:28-32; multi-draw argument
// lists evaluated left to right), so the flattened scene is the reference's scene.
//
// Compiled with -ffp-contract=off: every float expression keeps the reference's rounding.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_detmath.h"
#include "rt_host_geom.h"
#include "rt_xorwow.h"

namespace {

struct F3 {
  float x, y, z;
};
inline F3 mk(float x, float y, float z) { return F3{x, y, z}; }
inline F3 add(F3 a, F3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline F3 sub(F3 a, F3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline F3 mul(F3 a, F3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
inline F3 scale(float t, F3 v) { return mk(t * v.x, t * v.y, t * v.z); }
inline float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline F3 cross(F3 a, F3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
inline F3 unit(F3 v) { return scale(1.0f / std::sqrt(dot(v, v)), v); }
inline void put(float* d, F3 v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; }

struct Box3 {
  F3 lo, hi;
};
inline Box3 join(const Box3& a, const Box3& b) {
  return Box3{mk(std::fmin(a.lo.x, b.lo.x), std::fmin(a.lo.y, b.lo.y), std::fmin(a.lo.z, b.lo.z)),
              mk(std::fmax(a.hi.x, b.hi.x), std::fmax(a.hi.y, b.hi.y), std::fmax(a.hi.z, b.hi.z))};
}

// Scene RNG: curand_uniform-based helpers of vec3.h:7-13,62-69 and common.h:49-52.
struct SceneRng {
  rtx::State s = rtx::seed_state(1984);
  float u() { return rtx::uniform(s); }
  float u(float lo, float hi) { return lo + (hi - lo) * u(); }
  F3 v3() {
    const float a = u(), b = u(), c = u();
    return mk(a, b, c);
  }
  F3 v3(float lo, float hi) {
    const float a = u(lo, hi), b = u(lo, hi), c = u(lo, hi);
    return mk(a, b, c);
  }
  int rint(int lo, int hi) { return (int)u((float)lo, (float)(hi + 1)); }
};

}  // namespace

struct rt_scene_host {
  rt_scene_soa view{};
  std::vector<int32_t> world;
  std::vector<rt_object> objects;
  std::vector<rt_prim> prims;
  std::vector<rt_triangle> tris;
  std::vector<rt_bvh_node> nodes;
  std::vector<rt_material> mats;
  std::vector<rt_texture> texs;
  std::vector<rt_perlin> perlins;
  std::vector<rt_image> images;
  std::vector<uint8_t> texels;
  bool h20 = false;

  // ---- textures / materials
  int solid(F3 c) {
    rt_texture t{};
    t.type = RT_TEX_SOLID;
    put(t.color, c);
    texs.push_back(t);
    return (int)texs.size() - 1;
  }
  int checker(int even, int odd) {
    rt_texture t{};
    t.type = RT_TEX_CHECKER;
    t.a = even;
    t.b = odd;
    texs.push_back(t);
    return (int)texs.size() - 1;
  }
  int perlin(SceneRng& g) {  // perlin.h:63-76
    rt_perlin p{};
    for (int i = 0; i < 256; ++i) put(p.ranvec[i], unit(g.v3(-1.0f, 1.0f)));
    int32_t* perms[3] = {p.perm_x, p.perm_y, p.perm_z};
    for (int32_t* q : perms) {
      for (int i = 0; i < 256; ++i) q[i] = i;
      for (int i = 255; i > 0; --i) {
        int tg = g.rint(0, i);
        if (tg > i) { h20 = true; tg = i; }
        std::swap(q[i], q[tg]);
      }
    }
    perlins.push_back(p);
    return (int)perlins.size() - 1;
  }
  int noise_tex(int type, SceneRng& g, float sc, int depth) {
    rt_texture t{};
    t.type = type;
    t.a = perlin(g);
    t.b = depth;
    t.scale = sc;
    texs.push_back(t);
    return (int)texs.size() - 1;
  }
  int mat(int type, int tex, float param) {
    rt_material m{};
    m.type = type;
    m.texture = tex;
    m.param = param;
    mats.push_back(m);
    return (int)mats.size() - 1;
  }
  int lam(F3 c) { return mat(RT_MAT_LAMBERTIAN, solid(c), 0.0f); }
  // image_texture over a decoded image (texture.h:125-163); texels appended in upload order.
  int image_tex(const rt_image_asset& a) {
    rt_image im{};
    im.width = a.width;
    im.height = a.height;
    im.bytes_per_pixel = a.bytes_per_pixel;
    im.offset = (int32_t)texels.size();
    const size_t n = (size_t)a.width * a.height * a.bytes_per_pixel;
    if (a.data && n) texels.insert(texels.end(), a.data, a.data + n);
    else im.width = 0;  // no data: the reference's cyan fallback (texture.h:146-147)
    images.push_back(im);
    rt_texture t{};
    t.type = RT_TEX_IMAGE;
    t.a = (int)images.size() - 1;
    texs.push_back(t);
    return (int)texs.size() - 1;
  }

  // ---- primitives / objects
  int prim(int type, int m, std::initializer_list<float> p) {
    rt_prim r{};
    int k = 0;
    for (float v : p) r.p[k++] = v;
    r.type = type;
    r.material = m;
    prims.push_back(r);
    return (int)prims.size() - 1;
  }
  int sphere(F3 c, float r, int m) { return prim(RT_PRIM_SPHERE, m, {c.x, c.y, c.z, r}); }
  int moving(F3 c0, F3 c1, float t0, float t1, float r, int m) {
    const F3 d = sub(c1, c0);
    return prim(RT_PRIM_MOVING_SPHERE, m, {c0.x, c0.y, c0.z, r, d.x, d.y, d.z, t0, t1 - t0});
  }
  // triangle.h:19-41: edges, barycentric dot products and 1/denominator precomputed; vertex
  // normals only with the second constructor (n != nullptr).
  int tri(F3 a, F3 b, F3 c, const float uv[6], const F3* n, int m) {
    rt_triangle t{};
    put(t.v0, a);
    put(t.v1, b);
    put(t.v2, c);
    const F3 e0 = sub(b, a), e1 = sub(c, a);
    put(t.e0, e0);
    put(t.e1, e1);
    t.d00 = dot(e0, e0);
    t.d01 = dot(e0, e1);
    t.d11 = dot(e1, e1);
    t.inv_denom = 1.0f / (t.d00 * t.d11 - t.d01 * t.d01);
    for (int k = 0; k < 6; ++k) t.uv[k] = uv[k];
    if (n) {
      put(t.n0, n[0]);
      put(t.n1, n[1]);
      put(t.n2, n[2]);
      t.vertex_normals = 1;
    }
    tris.push_back(t);
    return prim(RT_PRIM_TRIANGLE, m, {(float)(tris.size() - 1)});
  }
  int rect(int type, float a0, float a1, float b0, float b1, float k, int m) {
    return prim(type, m, {a0, a1, b0, b1, k, a1 - a0, b1 - b0});
  }
  int object(int kind, int a, int b, std::initializer_list<float> f = {}) {
    rt_object o{};
    o.kind = kind;
    o.a = a;
    o.b = b;
    int k = 0;
    for (float v : f) o.f[k++] = v;
    objects.push_back(o);
    return (int)objects.size() - 1;
  }
  // box.h:8-40: the list of six rects as one primitive (same hit order and tie rule, box bbox).
  int box_prim(F3 p0, F3 p1, int m) { return prim(RT_PRIM_BOX, m, {p0.x, p0.y, p0.z, p1.x, p1.y, p1.z}); }
  int box(F3 p0, F3 p1, int m) { return object(RT_OBJ_PRIM, box_prim(p0, p1, m), 0); }
  // translate(rotate_y(child, deg), off): hittable.h:31-143.
  int xform(int child, float deg, F3 off) {
    const float rad = deg * 3.1415927f / 180.0f;
    return object(RT_OBJ_XFORM, child, 3, {off.x, off.y, off.z, rtm::det_sinf(rad), rtm::det_cosf(rad)});
  }

  // bounding_box(t0, t1) of a primitive (sphere.h:75-78, moving_sphere.h:61-66, aarect.h).
  Box3 pbox(int pi, float t0, float t1) const {
    const rth::Box b = rth::prim_box(prims[pi], tris.data(), t0, t1);
    return Box3{mk(b.lo[0], b.lo[1], b.lo[2]), mk(b.hi[0], b.hi[1], b.hi[2])};
  }

  // Reference-layout BVH over prims [first, first+n) (bvh.h:163-346): perfect tree of
  // rows = ceil(log2 n) inner levels; left child gets floor(num/2) objects; one split axis per
  // inner node drawn in node-index order; children take the node's objects in ascending stable
  // order of bbox(0,0).min[axis]; bounds from bbox(time0,time1), bottom-up.
  int bvh(int first, int n, float time0, float time1, SceneRng& g) {
    int rows = 0;
    while ((1 << rows) < n) ++rows;
    if (n < 3) return -1;
    const int inner = (1 << rows) - 1, last0 = (1 << (rows - 1)) - 1;
    std::vector<int> num(inner);
    num[0] = n;
    for (int k = 1; k < inner; ++k) {
      const int par = (k - 1) >> 1;
      num[k] = (k & 1) ? num[par] / 2 : num[par] / 2 + num[par] % 2;
    }
    for (int k = last0; k < inner; ++k)
      if (num[k] < 1 || num[k] > 2) return -1;
    std::vector<int> axis(inner);
    for (int k = 0; k < inner; ++k) {
      int a = g.rint(0, 2);
      if (a > 2) { h20 = true; a = 2; }
      axis[k] = a;
    }
    std::vector<int> rank[3];
    for (int a = 0; a < 3; ++a) {
      std::vector<int> ord(n);
      std::vector<float> key(n);
      for (int i = 0; i < n; ++i) {
        ord[i] = i;
        const Box3 b = pbox(first + i, 0.0f, 0.0f);
        key[i] = a == 0 ? b.lo.x : (a == 1 ? b.lo.y : b.lo.z);
      }
      std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return key[x] < key[y]; });
      rank[a].resize(n);
      for (int i = 0; i < n; ++i) rank[a][ord[i]] = i;
    }
    std::vector<std::vector<int>> members(inner);
    members[0].resize(n);
    for (int i = 0; i < n; ++i) members[0][i] = i;
    const int base = (int)nodes.size();
    nodes.resize(base + inner);
    for (int k = 0; k < inner; ++k) {
      std::vector<int>& m = members[k];
      const std::vector<int>& rk = rank[axis[k]];
      std::sort(m.begin(), m.end(), [&](int x, int y) { return rk[x] < rk[y]; });
      rt_bvh_node& nd = nodes[base + k];
      nd.leaf_a = axis[k];  // inner nodes keep their split axis (near-first ordering)
      nd.leaf_b = -1;
      if (k >= last0) {
        nd.leaf_a = first + m[0];
        if (num[k] == 2) nd.leaf_b = first + m[1];
      } else {
        const int nl = num[2 * k + 1];
        members[2 * k + 1].assign(m.begin(), m.begin() + nl);
        members[2 * k + 2].assign(m.begin() + nl, m.end());
      }
      std::vector<int>().swap(m);
    }
    std::vector<Box3> bb(inner);
    for (int k = inner - 1; k >= 0; --k) {
      rt_bvh_node& nd = nodes[base + k];
      if (k >= last0) {
        bb[k] = pbox(nd.leaf_a, time0, time1);
        if (nd.leaf_b >= 0) bb[k] = join(bb[k], pbox(nd.leaf_b, time0, time1));
      } else {
        bb[k] = join(bb[2 * k + 1], bb[2 * k + 2]);
      }
      put(nd.lo, bb[k].lo);
      put(nd.hi, bb[k].hi);
    }
    return object(RT_OBJ_BVH, base, rows);
  }

  // camera.h:18-47
  void camera(F3 from, F3 at, F3 up, float vfov, float aspect, float aperture, float focus,
              float t0, float t1) {
    rt_camera& c = view.camera;
    const float theta = vfov * 3.1415927f / 180.0f;
    const float h = rtm::det_tanf(theta / 2.0f);
    const float vh = 2.0f * h;
    const float vw = aspect * vh;
    const F3 w = unit(sub(from, at));
    const F3 u = unit(cross(up, w));
    const F3 v = cross(w, u);
    const F3 horiz = scale(focus * vw, u);
    const F3 vert = scale(focus * vh, v);
    const F3 llc = sub(sub(sub(from, scale(1.0f / 2.0f, horiz)), scale(1.0f / 2.0f, vert)), scale(focus, w));
    put(c.origin, from);
    put(c.lower_left, llc);
    put(c.horizontal, horiz);
    put(c.vertical, vert);
    put(c.u, u);
    put(c.v, v);
    put(c.w, w);
    c.lens_radius = aperture / 2.0f;
    c.time0 = t0;
    c.time1 = t1;
  }

  void finish() {
    view.world = world.data();           view.n_world = (int32_t)world.size();
    view.objects = objects.data();       view.n_objects = (int32_t)objects.size();
    view.prims = prims.data();           view.n_prims = (int32_t)prims.size();
    view.triangles = tris.data();        view.n_triangles = (int32_t)tris.size();
    view.nodes = nodes.data();           view.n_nodes = (int32_t)nodes.size();
    view.materials = mats.data();        view.n_materials = (int32_t)mats.size();
    view.textures = texs.data();         view.n_textures = (int32_t)texs.size();
    view.perlins = perlins.data();       view.n_perlins = (int32_t)perlins.size();
    view.images = images.data();         view.n_images = (int32_t)images.size();
    view.texels = texels.data();         view.n_texels = (int64_t)texels.size();
  }
};

namespace {

const F3 kSky = {0.7f, 0.8f, 1.0f};
const F3 kBlack = {0.0f, 0.0f, 0.0f};

void set_bg(rt_scene_host& s, F3 c, float aspect) {
  put(s.view.background, c);
  s.view.aspect = aspect;
}

void scene_basic(rt_scene_host& s) {  // scenes.h:82-100
  set_bg(s, kSky, 16.0f / 9.0f);
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, 0, -1), 0.5f, s.lam(mk(0, 1, 0))), 0));
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, -100.5f, -1), 100.0f, s.lam(mk(0, 0, 1))), 0));
  s.camera(mk(0, 0, -3), mk(0, 0, 0), mk(0, 1, 0), 40, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
}

void scene_first(rt_scene_host& s) {  // scenes.h:106-137
  set_bg(s, kSky, 16.0f / 9.0f);
  const int g = s.lam(mk(0.8f, 0.8f, 0.0f)), c = s.lam(mk(0.1f, 0.2f, 0.3f));
  const int l = s.mat(RT_MAT_DIELECTRIC, -1, 2.5f);
  const int r = s.mat(RT_MAT_METAL, s.solid(mk(0.8f, 0.6f, 0.2f)), 0.2f);
  const int f = s.mat(RT_MAT_DIELECTRIC, -1, 2.0f);
  const int ids[6] = {s.sphere(mk(0, -100.5f, -1), 100.0f, g), s.sphere(mk(0, 0, -1), 0.5f, c),
                      s.sphere(mk(-1, 0, -1), 0.5f, l),       s.sphere(mk(1, 0, -1), 0.5f, r),
                      s.sphere(mk(0, 1, -0.75f), 0.25f, f),   s.sphere(mk(0, 1, -0.75f), -0.25f, f)};
  for (int id : ids) s.world.push_back(s.object(RT_OBJ_PRIM, id, 0));
  s.camera(mk(-2, 2, -3), mk(0, 0, -1), mk(0, 1, 0), 20, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
}

// big_scene1, scenes.h:140-222 (config C2): 488 objects under one BVH.
void scene_big1(rt_scene_host& s) {
  set_bg(s, kSky, 16.0f / 9.0f);
  SceneRng g;
  const int first = (int)s.prims.size();
  const int checker = s.checker(s.solid(mk(0.2f, 0.3f, 0.1f)), s.solid(mk(0.9f, 0.9f, 0.9f)));
  s.sphere(mk(0, -1000, 0), 1000.0f, s.mat(RT_MAT_LAMBERTIAN, checker, 0.0f));
  for (int a = -11; a < 11; ++a)
    for (int b = -11; b < 11; ++b) {
      const float choose = g.u();
      const float cx = (float)a + 0.9f * g.u();
      const float cz = (float)b + 0.9f * g.u();
      const F3 c = mk(cx, 0.2f, cz);
      const F3 off = sub(c, mk(4, 0.2f, 0));
      if (dot(off, off) > 0.9f * 0.9f) {
        if ((double)choose < 0.8) {
          const F3 a1 = g.v3();
          const F3 a2 = g.v3();
          const int m = s.lam(mul(a1, a2));
          const F3 c2 = add(c, mk(0, g.u(0.0f, 0.5f), 0));
          s.moving(c, c2, 0.0f, 1.0f, 0.2f, m);
        } else if ((double)choose < 0.95) {
          const F3 alb = g.v3(0.5f, 1.0f);
          const float fuzz = g.u(0.0f, 0.5f);
          s.sphere(c, 0.2f, s.mat(RT_MAT_METAL, s.solid(alb), fuzz));
        } else {
          s.sphere(c, 0.2f, s.mat(RT_MAT_DIELECTRIC, -1, 1.5f));
        }
      } else {
        s.sphere(mk(10000, -10000, 10000), 0.00001f, s.lam(mk(0, 0, 0)));
      }
    }
  s.sphere(mk(0, 1, 0), 1.0f, s.mat(RT_MAT_DIELECTRIC, -1, 1.5f));
  s.sphere(mk(-4, 1, 0), 1.0f, s.lam(mk(0.4f, 0.2f, 0.1f)));
  s.sphere(mk(4, 1, 0), 1.0f, s.mat(RT_MAT_METAL, s.solid(mk(0.7f, 0.6f, 0.5f)), 0.0f));
  s.world.push_back(s.bvh(first, (int)s.prims.size() - first, 0.0f, 1.0f, g));
  s.camera(mk(13.0f, 2.0f, -3.0f), mk(0, 0, 0), mk(0, 1, 0), 20, 16.0f / 9.0f, 0.1f, 10.0f, 0, 1);
}

void scene_two_spheres(rt_scene_host& s) {  // scenes.h:225-243
  set_bg(s, kSky, 16.0f / 9.0f);
  const int ck = s.checker(s.solid(mk(0.2f, 0.3f, 0.1f)), s.solid(mk(0.9f, 0.9f, 0.9f)));
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, -10, 0), 10.0f, s.mat(RT_MAT_LAMBERTIAN, ck, 0)), 0));
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, 10, 0), 10.0f, s.mat(RT_MAT_LAMBERTIAN, ck, 0)), 0));
  s.camera(mk(13, 2, 3), mk(0, 0, 0), mk(0, 1, 0), 20, 16.0f / 9.0f, 0.1f, 10.0f, 0, 1);
}

void scene_two_perlin(rt_scene_host& s) {  // scenes.h:248-274
  set_bg(s, kSky, 16.0f / 9.0f);
  SceneRng g;
  const int t1 = s.noise_tex(RT_TEX_MARBLE, g, 4.0f, 7);
  const int t2 = s.noise_tex(RT_TEX_TURBULENT, g, 5.0f, 7);
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, -1000, 0), 1000.0f, s.mat(RT_MAT_LAMBERTIAN, t1, 0)), 0));
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, 2, 0), 2.0f, s.mat(RT_MAT_LAMBERTIAN, t2, 0)), 0));
  s.camera(mk(13, 2, 3), mk(0, 0, 0), mk(0, 1, 0), 20, 16.0f / 9.0f, 0.1f, 10.0f, 0, 1);
}

// cornell_box / cornell_smoke_box, scenes.h:323-404 (config C3 with smoke).
void scene_cornell(rt_scene_host& s, bool smoke) {
  set_bg(s, kBlack, 1.0f);
  const int red = s.lam(mk(0.65f, 0.05f, 0.05f)), white = s.lam(mk(0.73f, 0.73f, 0.73f));
  const int green = s.lam(mk(0.12f, 0.45f, 0.15f));
  const int light = s.mat(RT_MAT_DIFFUSE_LIGHT, s.solid(mk(15, 15, 15)), 0);
  auto top = [&](int prim) { s.world.push_back(s.object(RT_OBJ_PRIM, prim, 0)); };
  top(s.rect(RT_PRIM_RECT_YZ, 0, 555, 0, 555, 555, green));
  top(s.rect(RT_PRIM_RECT_YZ, 0, 555, 0, 555, 0, red));
  if (smoke) top(s.rect(RT_PRIM_RECT_XZ, 113, 443, 127, 432, 554, light));
  else top(s.rect(RT_PRIM_RECT_XZ, 213, 343, 227, 332, 554, light));
  top(s.rect(RT_PRIM_RECT_XZ, 0, 555, 0, 555, 0, white));
  top(s.rect(RT_PRIM_RECT_XZ, 0, 555, 0, 555, 555, white));
  top(s.rect(RT_PRIM_RECT_XY, 0, 555, 0, 555, 555, white));
  int b1 = s.xform(s.box(mk(0, 0, 0), mk(165, 330, 165), white), 15.0f, mk(265, 0, 295));
  int b2 = s.xform(s.box(mk(0, 0, 0), mk(165, 165, 165), white), -18.0f, mk(130, 0, 65));
  if (smoke) {
    b1 = s.object(RT_OBJ_MEDIUM, b1, s.mat(RT_MAT_ISOTROPIC, s.solid(mk(0, 0, 0)), 0), {-1.0f / 0.01f});
    b2 = s.object(RT_OBJ_MEDIUM, b2, s.mat(RT_MAT_ISOTROPIC, s.solid(mk(1, 1, 1)), 0), {-1.0f / 0.01f});
  }
  s.world.push_back(b1);
  s.world.push_back(b2);
  s.camera(mk(278, 278, -800), mk(278, 278, 0), mk(0, 1, 0), 40, 1.0f, 0.0f, 10.0f, 0, 1);
}

// triangle_scene, scenes.h:409-428: one triangle (face normal) and the ground sphere.
void scene_triangle(rt_scene_host& s) {
  set_bg(s, kSky, 16.0f / 9.0f);
  const float uv[6] = {0, 0, 0, 1, 1, 0};
  s.world.push_back(s.object(RT_OBJ_PRIM, s.tri(mk(-0.5f, 0, 0), mk(0, 1, 10), mk(0.0f, 0, 0), uv, nullptr,
                                                s.lam(mk(0, 1, 0))), 0));
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, -100.5f, -1), 100.0f, s.lam(mk(0, 0, 1))), 0));
  s.camera(mk(0, 0, -3), mk(0, 0, 0), mk(0, 1, 0), 40, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
}

// triangles_scene, scenes.h:432-475: four triangles in a triangle_mesh (a bvh_node built with
// the world_init state) and the ground sphere.
void scene_triangles(rt_scene_host& s) {
  set_bg(s, kSky, 16.0f / 9.0f);
  SceneRng g;
  const float uv[6] = {0, 0, 0, 1, 1, 0};
  const int first = (int)s.prims.size();
  s.tri(mk(-0.5f, 0, 0), mk(0, 1, 10), mk(0.5f, 0, 0), uv, nullptr, s.lam(mk(0, 1, 0)));
  s.tri(mk(0.5f, 0, 0), mk(0, 1, 10), mk(0.5f, 1, 0), uv, nullptr, s.lam(mk(1, 1, 0)));
  s.tri(mk(1.5f, 0, 0), mk(0, 2, 10), mk(1.5f, 1, 0), uv, nullptr, s.lam(mk(1, 1, 1)));
  s.tri(mk(1.5f, 0, 0), mk(1.5f, 1, 10), mk(1.5f, 0, 2), uv, nullptr, s.lam(mk(1, 1, 1)));
  s.world.push_back(s.bvh(first, 4, 0.0f, 1.0f, g));
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, -100.5f, -1), 100.0f, s.lam(mk(0, 0, 1))), 0));
  s.camera(mk(0, 0, -3), mk(0, 0, 0), mk(0, 1, 0), 40, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
}

// earth_scene, scenes.h:278-320: image-textured sphere and an emitting xy_rect, black background.
bool scene_earth(rt_scene_host& s, const rt_scene_assets* a) {
  if (!a || a->n_images < 1) return false;
  set_bg(s, kBlack, 16.0f / 9.0f);
  const int earth = s.mat(RT_MAT_LAMBERTIAN, s.image_tex(a->images[0]), 0.0f);
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, 0, 0), 2.0f, earth), 0));
  const int light = s.mat(RT_MAT_DIFFUSE_LIGHT, s.solid(mk(4.0f, 4.0f, 4.0f)), 0);
  s.world.push_back(s.object(RT_OBJ_PRIM, s.rect(RT_PRIM_RECT_XY, -5, 5, -3, 3, 6, light), 0));
  s.camera(mk(13.0f, 0.0f, 3.0f), mk(0.0f, 0.0f, 0.0f), mk(0, 1, 0), 20, 16.0f / 9.0f, 0.1f, 10.0f, 0, 1);
  return true;
}

// One triangle_mesh of create_meshes_d (triangle_mesh.h:147-204): lambertian(image_texture) on
// every triangle, a bvh_node over them built with the world_init state (triangle_mesh.h:27-35).
int add_mesh(rt_scene_host& s, const rt_scene_assets* a, const rt_mesh_asset& m, SceneRng& g) {
  int tex;
  if (m.image >= 0 && m.image < a->n_images) tex = s.image_tex(a->images[m.image]);
  else tex = s.image_tex(rt_image_asset{0, 0, 0, 0, nullptr});
  const int mat = s.mat(RT_MAT_LAMBERTIAN, tex, 0.0f);
  const int first = (int)s.prims.size();
  for (int k = 0; k < m.n_triangles; ++k) {
    const float* d = m.data + 24 * (size_t)k;
    const F3 n[3] = {mk(d[9], d[10], d[11]), mk(d[12], d[13], d[14]), mk(d[15], d[16], d[17])};
    s.tri(mk(d[0], d[1], d[2]), mk(d[3], d[4], d[5]), mk(d[6], d[7], d[8]), d + 18, m.vertex_normals ? n : nullptr,
          mat);
  }
  if (m.n_triangles < 3) return -1;
  return s.bvh(first, m.n_triangles, 0.0f, 1.0f, g);
}

// door_scene / cup_scene, scenes.h:478-523,576-621: the mesh and a ground sphere.
bool scene_mesh(rt_scene_host& s, const rt_scene_assets* a, F3 from, F3 at) {
  if (!a || a->n_meshes < 1 || !a->meshes[0].data) return false;
  set_bg(s, kSky, 16.0f / 9.0f);
  SceneRng g;
  s.world.push_back(add_mesh(s, a, a->meshes[0], g));
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, -100, -1), 100.0f, s.lam(mk(0, 1, 0))), 0));
  s.camera(from, at, mk(0, 1, 0), 20, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
  return true;
}

// backpack_scene, scenes.h:526-572: the mesh is overwritten by the ground sphere (H17), so the
// world is that sphere alone.
void scene_backpack(rt_scene_host& s) {
  set_bg(s, kSky, 16.0f / 9.0f);
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(0, -100, -1), 100.0f, s.lam(mk(0, 1, 0))), 0));
  s.camera(mk(0, 0, -3), mk(0, 0, 0), mk(0, 1, 0), 20, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
}

// Config C5, final_scene(): the reference has no definition; composed from its components after
// "Ray Tracing: The Next Week" section 10: 400 ground boxes under a BVH, a light,
// a moving sphere, glass / metal spheres, a glass sphere filled with a constant medium, a global
// fog medium, the earth-textured sphere, a perlin sphere, a rotated+translated BVH of 1000
// spheres and the door mesh (scaled 150x, translated) under its own BVH.  Scene RNG draws, from
// world_init: 400 box heights (row-major), the ground BVH, the perlin tables, 1000 sphere centres
// (x, y, z), the sphere BVH, the mesh BVH.
bool scene_final(rt_scene_host& s, const rt_scene_assets* a) {
  if (!a || a->n_images < 1 || a->n_meshes < 1 || !a->meshes[0].data || a->meshes[0].n_triangles < 3) return false;
  set_bg(s, kBlack, 16.0f / 9.0f);
  SceneRng g;
  const int ground = s.lam(mk(0.48f, 0.83f, 0.53f));
  const int gfirst = (int)s.prims.size();
  for (int i = 0; i < 20; ++i)
    for (int j = 0; j < 20; ++j) {
      const float w = 100.0f;
      const float x0 = -1000.0f + (float)i * w, z0 = -1000.0f + (float)j * w, y0 = 0.0f;
      const float x1 = x0 + w, y1 = g.u(1.0f, 101.0f), z1 = z0 + w;
      s.box_prim(mk(x0, y0, z0), mk(x1, y1, z1), ground);
    }
  s.world.push_back(s.bvh(gfirst, 400, 0.0f, 1.0f, g));
  const int light = s.mat(RT_MAT_DIFFUSE_LIGHT, s.solid(mk(7, 7, 7)), 0);
  s.world.push_back(s.object(RT_OBJ_PRIM, s.rect(RT_PRIM_RECT_XZ, 123, 423, 147, 412, 554, light), 0));
  const F3 c1 = mk(400, 400, 200), c2 = add(c1, mk(30, 0, 0));
  s.world.push_back(s.object(RT_OBJ_PRIM, s.moving(c1, c2, 0, 1, 50, s.lam(mk(0.7f, 0.3f, 0.1f))), 0));
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(260, 150, 45), 50, s.mat(RT_MAT_DIELECTRIC, -1, 1.5f)), 0));
  s.world.push_back(s.object(RT_OBJ_PRIM,
                             s.sphere(mk(0, 150, 145), 50, s.mat(RT_MAT_METAL, s.solid(mk(0.8f, 0.8f, 0.9f)), 1.0f)), 0));
  const int boundary = s.object(RT_OBJ_PRIM, s.sphere(mk(360, 150, 145), 70, s.mat(RT_MAT_DIELECTRIC, -1, 1.5f)), 0);
  s.world.push_back(boundary);
  s.world.push_back(s.object(RT_OBJ_MEDIUM, boundary, s.mat(RT_MAT_ISOTROPIC, s.solid(mk(0.2f, 0.4f, 0.9f)), 0),
                             {-1.0f / 0.2f}));
  const int fog = s.object(RT_OBJ_PRIM, s.sphere(mk(0, 0, 0), 5000, s.mat(RT_MAT_DIELECTRIC, -1, 1.5f)), 0);
  s.world.push_back(s.object(RT_OBJ_MEDIUM, fog, s.mat(RT_MAT_ISOTROPIC, s.solid(mk(1, 1, 1)), 0), {-1.0f / 0.0001f}));
  const int earth = s.mat(RT_MAT_LAMBERTIAN, s.image_tex(a->images[0]), 0.0f);
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(400, 200, 400), 100, earth), 0));
  const int pertext = s.noise_tex(RT_TEX_NOISE, g, 0.1f, 0);
  s.world.push_back(s.object(RT_OBJ_PRIM, s.sphere(mk(220, 280, 300), 80, s.mat(RT_MAT_LAMBERTIAN, pertext, 0)), 0));
  const int white = s.lam(mk(0.73f, 0.73f, 0.73f));
  const int sfirst = (int)s.prims.size();
  for (int k = 0; k < 1000; ++k) s.sphere(g.v3(0.0f, 165.0f), 10, white);
  s.world.push_back(s.xform(s.bvh(sfirst, 1000, 0.0f, 1.0f, g), 15.0f, mk(-100, 270, 395)));
  // the door: the mesh with its positions scaled by 150
  const rt_mesh_asset& m = a->meshes[0];
  std::vector<float> scaled(m.data, m.data + 24 * (size_t)m.n_triangles);
  for (int t = 0; t < m.n_triangles; ++t)
    for (int q = 0; q < 9; ++q) scaled[24 * (size_t)t + q] *= 150.0f;
  rt_mesh_asset ms = m;
  ms.data = scaled.data();
  s.world.push_back(s.xform(add_mesh(s, a, ms, g), -30.0f, mk(30, 101, 150)));
  s.camera(mk(478, 278, -600), mk(278, 278, 0), mk(0, 1, 0), 40, 16.0f / 9.0f, 0.0f, 10.0f, 0, 1);
  return true;
}

// Test scenes "coincident" / "coincident_step" (not in scenes.h): parity fixtures of the list and
// BVH tie rules, restated in the oracle (build_coincident).  "coincident": xy_rects in the plane z = 0
// in three kinds of list entries -- a primitive, members of a reference BVH and a translate(rotate_y(..,
// 0)) instance (rotate_y by 0 and a translation in x, y leave the ray's z terms exact) -- so world
// queries meet exact ties across entries (hittable_list.h:23-39: the later entry wins) and inside the
// BVH (the first visited wins).  "coincident_step": render_step_kernel's world shape (a BVH, then
// primitives): a triangle repeated bit for bit inside the BVH and once more after it (Moller-Trumbore's
// t depends on v0, e0, e1 only, so equal triangles tie exactly: the H16 duplicates' case).
void scene_coincident(rt_scene_host& s, bool step) {
  set_bg(s, kSky, 16.0f / 9.0f);
  SceneRng g;
  const int red = s.lam(mk(0.8f, 0.1f, 0.1f)), green = s.lam(mk(0.1f, 0.8f, 0.1f));
  const int yellow = s.lam(mk(0.8f, 0.8f, 0.1f)), blue = s.lam(mk(0.1f, 0.2f, 0.8f));
  const int cyan = s.lam(mk(0.1f, 0.8f, 0.8f)), grey = s.lam(mk(0.5f, 0.5f, 0.5f));
  const int metal = s.mat(RT_MAT_METAL, s.solid(mk(0.8f, 0.8f, 0.8f)), 0.05f);
  const int glass = s.mat(RT_MAT_DIELECTRIC, -1, 1.5f);
  const int first = (int)s.prims.size();
  if (step) {
    const float uv[6] = {0, 0, 1, 0, 0, 1};
    const F3 a = mk(-1.0f, -1.5f, 0.0f), b = mk(2.0f, -1.5f, 0.0f), c = mk(-1.0f, 0.5f, 0.0f), d = mk(2.0f, 0.5f, 0.0f);
    s.tri(a, b, c, uv, nullptr, green);
    s.tri(b, d, c, uv, nullptr, blue);
    s.sphere(mk(2.2f, -0.3f, -0.8f), 0.5f, metal);
    s.tri(a, b, c, uv, nullptr, yellow);  // the first triangle again
    s.sphere(mk(-2.0f, 0.2f, -1.0f), 0.6f, glass);
    const int bvh = s.bvh(first, 5, 0.0f, 1.0f, g);
    const int again = s.object(RT_OBJ_PRIM, s.tri(a, b, c, uv, nullptr, red), 0);  // and after the BVH
    const int ground = s.object(RT_OBJ_PRIM, s.sphere(mk(0.0f, -101.7f, 0.0f), 100.0f, grey), 0);
    s.world = {bvh, again, ground};
  } else {
    s.rect(RT_PRIM_RECT_XY, -1.0f, 2.0f, -1.5f, 0.5f, 0.0f, green);
    s.rect(RT_PRIM_RECT_XY, -3.0f, 3.0f, 0.8f, 2.0f, 0.5f, blue);
    s.sphere(mk(2.2f, -0.3f, -0.8f), 0.5f, metal);
    s.rect(RT_PRIM_RECT_XY, -0.5f, 0.7f, -1.2f, -0.2f, 0.0f, yellow);
    s.rect(RT_PRIM_RECT_XZ, -3.0f, 3.0f, -3.0f, 3.0f, -1.6f, grey);
    s.sphere(mk(-2.0f, 0.2f, -1.0f), 0.6f, glass);
    const int bvh = s.bvh(first, 6, 0.0f, 1.0f, g);
    const int prim = s.object(RT_OBJ_PRIM, s.rect(RT_PRIM_RECT_XY, -2.0f, 0.5f, -1.0f, 1.0f, 0.0f, red), 0);
    const int ground = s.object(RT_OBJ_PRIM, s.sphere(mk(0.0f, -101.7f, 0.0f), 100.0f, grey), 0);
    const int inst = s.xform(s.object(RT_OBJ_PRIM, s.rect(RT_PRIM_RECT_XY, -0.75f, 1.25f, -0.6f, 1.1f, 0.0f, cyan), 0),
                             0.0f, mk(0.25f, 0.1f, 0.0f));
    s.world = {prim, bvh, inst, ground};
  }
  s.camera(mk(0.3f, 0.4f, -6.0f), mk(0, 0, 0), mk(0, 1, 0), 40, 16.0f / 9.0f, 0.1f, 6.0f, 0, 1);
}

int build_named(rt_scene_host& s, const std::string& n, const rt_scene_assets* a) {
  if (n == "basic") scene_basic(s);
  else if (n == "first") scene_first(s);
  else if (n == "big1" || n == "random") scene_big1(s);
  else if (n == "two_spheres") scene_two_spheres(s);
  else if (n == "two_perlin") scene_two_perlin(s);
  else if (n == "cornell") scene_cornell(s, false);
  else if (n == "cornell_smoke") scene_cornell(s, true);
  else if (n == "triangle") scene_triangle(s);
  else if (n == "triangles") scene_triangles(s);
  else if (n == "backpack") scene_backpack(s);
  else if (n == "earth") { if (!scene_earth(s, a)) return RT_ERR_ARG; }
  else if (n == "door") { if (!scene_mesh(s, a, mk(-3, 4, -5), mk(0, 1, 0))) return RT_ERR_ARG; }
  else if (n == "cup") { if (!scene_mesh(s, a, mk(0, 0, -1), mk(0, 0, 0))) return RT_ERR_ARG; }
  else if (n == "final") { if (!scene_final(s, a)) return RT_ERR_ARG; }
  else if (n == "coincident") scene_coincident(s, false);
  else if (n == "coincident_step") scene_coincident(s, true);
  else return RT_ERR_ARG;
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_scene_build_ex(const char* name, const rt_scene_assets* assets, rt_scene_host** out) {
  if (!name || !out) return RT_ERR_ARG;
  *out = nullptr;
  std::unique_ptr<rt_scene_host> s(new rt_scene_host);
  const int rc = build_named(*s, std::string(name), assets);
  if (rc != RT_OK) return rc;
  for (int32_t w : s->world)
    if (w < 0) return RT_ERR_SCENE;
  s->finish();
  *out = s.release();
  return RT_OK;
}

int rt_scene_build(const char* name, rt_scene_host** out) { return rt_scene_build_ex(name, nullptr, out); }

const rt_scene_soa* rt_scene_view(const rt_scene_host* s) { return s ? &s->view : nullptr; }

void rt_scene_free(rt_scene_host* s) { delete s; }

}  // extern "C"
