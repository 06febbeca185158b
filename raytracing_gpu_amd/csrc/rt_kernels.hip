// rt_kernels.hip — gfx950 render path: RNG init, the persistent path-tracing megakernel and the
// frame-buffer resolve, plus the C ABI of include/rt_hip.h.
//
// Reference semantics (file:line in daRoyalCacti/Raytracing_GPU):
//   render_init            render.h:84-92
//   render / color_f       render.h:55-113
//   world list             hittable_list.h:23-39
//   BVH traversal          bvh.h:348-436      (same visiting order, stackless over the perfect tree)
//   AABB slab test         aabb.h:19-104
//   sphere / moving sphere sphere.h:35-73, moving_sphere.h:26-59
//   rects / box            aarect.h:63-150, box.h:29-32
//   translate / rotate_y   hittable.h:37-59, 112-143
//   constant medium        constant_medium.h:34-70
//   materials              material.h:16-138
//   textures / perlin      texture.h:12-164, perlin.h:37-126
//   output transform       color.h:19-170
//
// MI355X design: one lane owns one (frame buffer, pixel) work item and runs its samples
// sequentially (the pixel's RNG stream is consumed in order, so samples cannot be split), but a
// lane whose path ends starts its next sample immediately and a lane whose item ends takes a new
// one: waves refill idle lanes from a global work counter with one atomic per refill (ballot
// compaction), so divergent path lengths do not idle the wave.  Each loop iteration is one ray
// segment (one world query + one scatter).  Hit records are deferred: traversal keeps only
// (t, prim) and the winner is finalised once.  No FP contraction (-ffp-contract=off): every
// float op rounds like the reference's C++ source.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <set>
#include <type_traits>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_detmath.h"
#include "rt_diag.h"
#include "rt_host_geom.h"
#include "rt_xorwow.h"

#define RT_PRIM_TYPE_MASK 0xff
#define RT_PRIM_FLAG_UV 0x100      // material needs sphere u,v (image texture)
#define RT_PRIM_FLAG_UNIT_T 0x200  // moving sphere with time0 = 0, time1 - time0 = 1
#define RT_PRIM_FLAG_XF 0x400      // world-tree leaf under a translate/rotate_y instance (F_WORLD)
#define RT_WKEY_SHIFT 20           // world-tree tie key: (n_world - 1 - entry) << 20 | reference leaf rank

// Scene feature mask: the render kernel is instantiated per feature set so that a scene pays
// registers only for the primitive / object / texture kinds it contains.
enum : int {
  F_STATS = 1 << 0,
  F_MOVING = 1 << 1,
  F_RECT = 1 << 2,
  F_TRI = 1 << 3,
  F_LIST = 1 << 4,
  F_XFORM = 1 << 5,
  F_MEDIUM = 1 << 6,
  F_CHECKER = 1 << 7,
  F_NOISE = 1 << 8,
  F_IMAGE = 1 << 9,
  F_BVH = 1 << 10,
  F_EXACT = 1 << 11,  // reference BVH visit set (no culling): node/prim counts equal the oracle's
  F_CHECK = 1 << 12,  // culled search + exact re-run per query; disagreements logged (audit mode)
  F_LDS = 1 << 13,    // BVH nodes + primitives staged in LDS (1024-thread workgroups, 1 per CU)
  F_STEP = 1 << 14,   // world = one BVH object: render_step_kernel (one traversal step per loop trip)
  F_WORLD = 1 << 15,  // list world flattened into ONE traversal tree (render_step_kernel; rt_scene_upload)
  F_QLDS = 1 << 16,   // the world BVH's traversal tree quantized to 24-byte pair records in LDS (qpair)
  F_MERGE = 1 << 17,  // render_kernel answers world queries with world_search only (merge_ok scenes)
  F_PROBE = 1 << 18,  // the same code under its own symbol for the probe launches of a first launch
                      // (rt_render): rocprof then times the render launches apart from the probes
  F_ALL = (1 << 11) - 2,
  F_SPHERES = F_MOVING | F_CHECKER | F_BVH,           // basic, first, big1 (C2), two_spheres
  F_CORNELL = F_RECT | F_LIST | F_XFORM | F_MEDIUM,   // cornell, cornell_smoke (C3)
  F_MESH = F_TRI | F_IMAGE | F_BVH | F_LIST,            // triangle meshes with image textures (C4)
  F_FINAL = F_ALL & ~F_CHECKER,                         // final (C5): everything but the checker texture
};

namespace {

// ------------------------------------------------------------------ device scene view
struct DScene {
  const int32_t* world;
  const rt_object* objects;
  const float4* prims;  // 3 float4 per prim: p0..p3 | p4..p7 | p8 p9 type mat
  const rt_triangle* tris;
  const float4* nodes;  // 2 float4 per node: lo.xyz leaf_a | hi.xyz leaf_b
  const int4* mats;     // type, texture, param bits, pad
  const rt_texture* texs;
  const rt_perlin* perlins;
  const rt_image* images;
  const uint8_t* texels;
  const float2* pmargin; // per prim: reference-chain safety margins (see bvh_closest)
  const float4* pvalid;  // per prim, 3 float4: the chain check in one fetch (chain_ok's first test)
  float* dbg;            // audit log (F_CHECK): 16 floats per disagreeing BVH query
  unsigned* dbg_n;
  int32_t dbg_cap;
  int32_t n_world;
  int32_t lds_nodes;     // F_LDS: node slots staged (the primitives follow them)
  int32_t lds_fb;        // F_LDS|F_STEP: first node of the world BVH's traversal tree, staged in planes
  int32_t lds_pairs;     // ... and its pair records (<= kPlanePairs)
  int32_t lds_prims;     // F_LDS: primitive count staged (validation margins follow them)
  int32_t lds_mats;      // F_LDS: materials staged after the margins (one float4 each)
  int32_t lds_texs;      // F_LDS: textures staged after the materials (two float4 each; stacks follow)
  int32_t lds_imgs;      // F_QLDS: images staged after the textures (one float4 each)
  const float4* cam_tab; // REF camera mode: lens offset (xyz) and time (w) of sample s (camera_ray)
  // F_WORLD (list world as one traversal tree, see build_world_tree): 4 float4 per leaf -- the
  // primitive's record (c.y = tie key, RT_PRIM_FLAG_XF in the type word for instance members) and
  // {instance, world entry, reference BVH object or -1, primitive} as ints; 2 float4 per instance
  // {translate xyz, flags bits} {sin, cos}; world entries from w_media on are constant media queried
  // in list order after the tree; w_inert: inert sphere-bounded media sit between tree entries.
  const float4* wleaf;
  const float4* wxf;
  int32_t wt_fb;
  int32_t w_media;
  int32_t w_inert;
  int32_t merge_ok;      // render_kernel may answer world queries with world_search
  const int32_t* worder; // world_search's visiting order of the entries (a permutation of 0..n_world-1)
  // F_QLDS: the world BVH's traversal tree as 24-byte pair records (build_qtree), staged in LDS;
  // q_ebias: exponent bias of their 5-bit per-axis scales
  const uint32_t* qnodes;
  int32_t q_pairs;
  int32_t q_ebias;
  rt_camera cam;
  float bg[3];
};

// Read-only scene arrays through the constant address space: a load whose address is wave-uniform
// (a list entry's object and primitive records, the world list) becomes a scalar load into SGPRs
// instead of a vector load that fills a VGPR with 64 copies; a lane-dependent address still becomes
// a global_load.  The scene is never written while a kernel runs.
// Only in variants without BVHs or triangles (C3's list of rects and media, whose entry loop is all
// uniform loads: 118 -> 108 VGPRs): in C5's variant the records held in SGPRs raise its SGPR spills
// into VGPR lanes and its VGPR spills (39 -> 49).
#define RT_RO __attribute__((address_space(4)))
// (The host pass type-checks device bodies too, and x86 has no address space 4 to copy a record
// from: there ro is the plain pointer.)
template <int F, class T>
__device__ __forceinline__ auto ro(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr ((F & (F_BVH | F_TRI)) == 0) return (const RT_RO T*)p;
  else return p;
#else
  return p;
#endif
}

// LDS image of the scene for F_LDS variants: [nodes (2 float4 each) | prims (3 float4 each)].
extern __shared__ float4 rt_lds[];

// Node / primitive arrays: LDS for F_LDS variants, global memory otherwise.  Going through these
// (instead of storing an LDS pointer into the scene struct) keeps the address space visible to
// the compiler: ds_read for LDS, global_load for the kernel-argument pointers.
template <int F>
__device__ __forceinline__ const float4* nodes_of(const DScene& S) {
  if constexpr ((F & F_LDS) != 0) return rt_lds;
  else return S.nodes;
}
template <int F>
__device__ __forceinline__ const float4* prims_of(const DScene& S) {
  if constexpr ((F & F_LDS) != 0) return rt_lds + 2 * S.lds_nodes;
  else return S.prims;
}
template <int F>
constexpr int render_block() {
  return (F & (F_LDS | F_QLDS)) != 0 ? 1024 : 256;
}
// Validation margins (F_LDS: staged after the primitives, two per float4).
template <int F>
__device__ __forceinline__ const float2* pmargin_of(const DScene& S) {
  if constexpr ((F & F_LDS) != 0) return (const float2*)(rt_lds + 2 * S.lds_nodes + 3 * S.lds_prims);
  else return S.pmargin;
}
static_assert(sizeof(rt_material) == 16 && sizeof(rt_texture) == 32 && sizeof(rt_image) == 16,
              "LDS staging copies whole float4s");
constexpr int kStackDepthQ = 16;  // = kStackDepth (the F_QLDS stacks, 16-bit entries)
// Materials and textures (F_LDS: staged after the margins; read once per segment by scatter).
__device__ __forceinline__ int lds_mats_at(const DScene& S) {
  return 2 * S.lds_nodes + 3 * S.lds_prims + (S.lds_prims + 1) / 2;
}
// F_QLDS: materials, textures and images staged after the quantized tree and its 16-bit stacks (one,
// two and one float4 each), so the shading phase's dependent chain (material -> texture -> image ->
// texel) reads LDS instead of L2 until the texel itself.
__host__ __device__ __forceinline__ int qlds_mats_at(const DScene& S) {
  return ((6 * S.q_pairs + 1024 * kStackDepthQ / 2) + 3) / 4;  // float4 index, 16-byte aligned
}
// render_kernel's variants without BVHs or triangles (C3) stage them after their locker too, and so does
// the merged-search variant (C5): its stacks and locker leave 1 KB of a quarter CU's LDS, room for a
// scene's tables (materials, textures, images) of up to 1 KB (rt_render checks; else the entry-loop
// variant runs).
constexpr int stack_words(int mask);
constexpr int locker_words(int mask);
template <int F>
constexpr bool tables_after_locker() {
  return (F & (F_LDS | F_QLDS | F_STEP | F_BVH | F_TRI)) == 0 || (F & F_MERGE) != 0;
}
template <int F>
constexpr int locker_tables_at() {  // float4 index after the stacks and the locker (256-thread blocks)
  return 256 * (stack_words(F) + locker_words(F)) / 4;
}
template <int F>
__device__ __forceinline__ const int4* mats_of(const DScene& S) {
  if constexpr ((F & F_LDS) != 0) return (const int4*)(rt_lds + lds_mats_at(S));
  else if constexpr ((F & F_QLDS) != 0) return (const int4*)(rt_lds + qlds_mats_at(S));
  else if constexpr (tables_after_locker<F>()) return (const int4*)(rt_lds + locker_tables_at<F>());
  else return S.mats;
}
template <int F>
__device__ __forceinline__ const rt_texture* texs_of(const DScene& S) {
  if constexpr ((F & F_LDS) != 0) return (const rt_texture*)(rt_lds + lds_mats_at(S) + S.lds_mats);
  else if constexpr ((F & F_QLDS) != 0) return (const rt_texture*)(rt_lds + qlds_mats_at(S) + S.lds_mats);
  else if constexpr (tables_after_locker<F>()) return (const rt_texture*)(rt_lds + locker_tables_at<F>() + S.lds_mats);
  else return S.texs;
}
template <int F>
__device__ __forceinline__ const rt_image* imgs_of(const DScene& S) {
  if constexpr ((F & F_QLDS) != 0) return (const rt_image*)(rt_lds + qlds_mats_at(S) + S.lds_mats + 2 * S.lds_texs);
  else if constexpr (tables_after_locker<F>())
    return (const rt_image*)(rt_lds + locker_tables_at<F>() + S.lds_mats + 2 * S.lds_texs);
  else return S.images;
}
// Stack entries: child words (pair index, or -1 - primitive).  F_LDS scenes have < 32768 pairs and
// primitives (they fit in LDS), so their entries are 16-bit (32 KB of stacks per 1024 lanes).
template <int F>
using stack_t = std::conditional_t<(F & (F_LDS | F_QLDS)) != 0, short, int>;
template <int F>
__device__ __forceinline__ stack_t<F>* stack_of(const DScene& S) {
  if constexpr ((F & F_LDS) != 0)
    return (short*)(rt_lds + lds_mats_at(S) + S.lds_mats + 2 * S.lds_texs) + threadIdx.x;
  else if constexpr ((F & F_QLDS) != 0)
    return (short*)((uint32_t*)rt_lds + 6 * S.q_pairs) + threadIdx.x;
  else return (int*)rt_lds + threadIdx.x;
}
// Per-lane traversal stack in LDS (after the staged scene for F_LDS variants), lane-interleaved
// (entry d of thread t at [d * block + t]) so a wave's pushes/pops hit 64 distinct banks.
constexpr int kStackDepth = 16;
// Per-lane "locker" of render_kernel's global-memory variants: cold per-item / per-sample state
// (the sample sum, the item's fb and row) kept in LDS after the stacks,
// lane-interleaved (word k of thread t at [k * block + t]), instead of VGPRs: it is touched once
// per sample, and without it the variants' live state spills to scratch inside the traversal
// loops (F_FINAL: 744 B per lane, ~340 B of scratch stores per segment, missing L2).
constexpr int kLocker = 23;  // words 15..20: the lane's RNG state, lane-contiguous (6 words per lane);
                             // 21, 22: split-sample end and claim (s_end, ck)
constexpr int kLockerSmall = 5;  // variants that park only the sample sum, fb and row
// Variants that also park the per-segment state (locker words 5..20: column, row, sample, depth,
// counts, attenuation, RNG state): the widest global-memory variants, whose world query spills to
// scratch at the 4-wave floor.  C5 F_FINAL at 3840x2159 4x4 (MI355X): 86.0 ms with 200 B of
// scratch per lane; 81.6 ms with words 5..14 parked (140 B); 80.7 ms with the RNG state too (132 B).
// F_CORNELL (no spills) ran 1 % slower with words 5..14 parked, so it keeps the small locker (and at
// 5 waves/SIMD too: 26 270-26 300 vs 26 850-26 930 Mrays/s).
constexpr bool parks_segment_mask(int mask) {
  return (mask & (F_LDS | F_STEP)) == 0 && ((mask & F_ALL) == F_FINAL || (mask & F_ALL) == F_ALL);
}
// LDS words per lane of traversal stack: render_kernel's global-memory variants without BVHs (C3's
// list of rects and media) traverse nothing and keep none, so their locker starts at word 0.
constexpr int stack_words(int mask) {
  return (mask & (F_LDS | F_STEP | F_QLDS | F_BVH)) == 0 ? 0 : kStackDepth;
}
// render_step_kernel: the world-tree variants park their per-item / per-sample state in a locker
// of kLockerStep words (step_parks_mask); the others keep none (only the traversal stack is in LDS).
constexpr int kLockerStep = 24;  // 18 state words + the RNG state (6 words, lane-contiguous)
constexpr bool step_parks_mask(int mask) { return (mask & F_STEP) != 0 && (mask & F_WORLD) != 0; }
constexpr int locker_words(int mask) {
  return (mask & F_STEP) != 0 ? (step_parks_mask(mask) ? kLockerStep : 0)
                              : (parks_segment_mask(mask) ? kLocker : kLockerSmall);
}
// Word k of the locker as a T lvalue for parking variants, else the register copy `reg`.
template <bool PK, typename T>
__device__ __forceinline__ T& cold_ref(T& reg, uint32_t* slot) {
  if constexpr (PK) return *reinterpret_cast<T*>(slot);
  else return reg;
}
template <int F>
constexpr bool parks() {
  return (F & F_LDS) == 0;
}
template <int F>
__device__ __forceinline__ uint32_t* locker_of() {
  return (uint32_t*)rt_lds + render_block<F>() * stack_words(F) + threadIdx.x;
}

// The stepwise LDS variant stages the world BVH's traversal tree (node slots lds_fb ..) in four planes
// of kPlanePairs float4 each -- plane c holds float4 c of every 64-byte pair record -- instead of
// record after record: the four ds_read_b128 of a traversal step then read 16-byte slots (pair mod 16)
// of the 256-byte bank row instead of 4 slots (pair mod 4), so a 16-lane group's reads spread over all
// 64 banks (MI355X_MICROARCH.md, LDS), at the same address arithmetic (plane offsets are immediates).
constexpr int kPlanePairs = 512;
template <int F>
constexpr bool planes() {
  return (F & F_LDS) != 0 && (F & F_STEP) != 0;
}
// Stage the read-only scene arrays a F_LDS variant reads in LDS, once per workgroup.
template <int F>
__device__ __forceinline__ void stage_lds(const DScene& S) {
  constexpr int BS = render_block<F>();
  const int nn = 2 * S.lds_nodes, np = 3 * S.lds_prims, nm = (S.lds_prims + 1) / 2;
  if constexpr (planes<F>()) {
    const int nf = 2 * S.lds_fb;  // reference trees as they are, then the traversal tree in planes
    for (int q = threadIdx.x; q < nf; q += BS) rt_lds[q] = S.nodes[q];
    for (int q = threadIdx.x; q < 4 * kPlanePairs; q += BS) {
      const int c = q / kPlanePairs, k = q - c * kPlanePairs;
      rt_lds[nf + q] = k < S.lds_pairs ? S.nodes[nf + 4 * k + c] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
  } else {
    for (int q = threadIdx.x; q < nn; q += BS) rt_lds[q] = S.nodes[q];
  }
  for (int q = threadIdx.x; q < np; q += BS) rt_lds[nn + q] = S.prims[q];
  const float4* pm = (const float4*)S.pmargin;  // padded to an even count at upload
  for (int q = threadIdx.x; q < nm; q += BS) rt_lds[nn + np + q] = pm[q];
  const int m0 = nn + np + nm;
  for (int q = threadIdx.x; q < S.lds_mats; q += BS) rt_lds[m0 + q] = ((const float4*)S.mats)[q];
  const float4* tx = (const float4*)S.texs;
  for (int q = threadIdx.x; q < 2 * S.lds_texs; q += BS) rt_lds[m0 + S.lds_mats + q] = tx[q];
  __syncthreads();
}


struct V {
  float x, y, z;
};
__device__ __forceinline__ V mk(float x, float y, float z) { return V{x, y, z}; }
__device__ __forceinline__ V operator+(V a, V b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V operator-(V a, V b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V operator*(V a, V b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V operator*(float t, V v) { return mk(t * v.x, t * v.y, t * v.z); }
__device__ __forceinline__ V neg(V a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len2(V a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ V unit(V v) { return (1.0f / __builtin_sqrtf(len2(v))) * v; }
__device__ __forceinline__ V ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ float comp(V v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

struct Ray {
  V o, d;
  float tm;
};

struct Hit {
  V p, n;
  float t, u, v;
  int mat;
  bool front;
};

__device__ __forceinline__ void set_face(Hit& h, const Ray& r, V out) {  // hittable.h:17-22
  h.front = dot(r.d, out) < 0;
  h.n = h.front ? out : neg(out);
}

// translate(rotate_y(child)) ray into the child's frame (hittable.h:37-59, 112-143), from an
// instance record {translate xyz, flags bits} {sin, cos} (flags: 1 translate, 2 rotate_y); the same
// float operations as xform_ray on the rt_object.  moved = the ray after the translation only.
__device__ __forceinline__ Ray xform_ray_x(float4 x0, float4 x1, const Ray& r, Ray& moved) {
  const int fl = __float_as_int(x0.w);
  moved = r;
  if (fl & 1) moved.o = r.o - mk(x0.x, x0.y, x0.z);
  Ray rr = moved;
  if (fl & 2) {
    const float s = x1.x, c = x1.y;
    rr.o.x = c * moved.o.x - s * moved.o.z;
    rr.o.z = s * moved.o.x + c * moved.o.z;
    rr.d.x = c * moved.d.x - s * moved.d.z;
    rr.d.z = s * moved.d.x + c * moved.d.z;
  }
  return rr;
}

using Rng = rtx::State;

// vec3.h:129-141 (left-to-right argument order).
__device__ __forceinline__ float urange(Rng& s, float lo, float hi) { return lo + (hi - lo) * rtx::uniform(s); }
__device__ __forceinline__ V in_unit_sphere(Rng& s) {
  V p;
  bool inside;
  do {
    const float a = urange(s, -1.0f, 1.0f);
    const float b = urange(s, -1.0f, 1.0f);
    const float c = urange(s, -1.0f, 1.0f);
    p = mk(a, b, c);
    inside = len2(p) < 1.0f;
  } while (!inside);
  return p;
}
__device__ __forceinline__ V in_unit_disk(Rng& s) {
  V p;
  bool inside;
  do {
    const float a = urange(s, -1.0f, 1.0f);
    const float b = urange(s, -1.0f, 1.0f);
    p = mk(a, b, 0.0f);
    inside = len2(p) < 1.0f;
  } while (!inside);
  return p;
}

// ------------------------------------------------------------------ primitive tests (t only)
struct PrimRec {
  float4 a, b, c;
};
template <int F>
__device__ __forceinline__ PrimRec load_prim(const DScene& S, int i) {
  if constexpr ((F & (F_LDS | F_BVH | F_TRI)) == 0) {  // read-only scene memory (ro): s_load when i is wave-uniform
    const auto q = ro<F>(S.prims) + 3 * i;
    return PrimRec{q[0], q[1], q[2]};
  } else {
    const float4* q = prims_of<F>(S) + 3 * i;
    return PrimRec{q[0], q[1], q[2]};
  }
}
// A wave-uniform primitive index in any global-memory variant: the record through ro (s_load).
template <int F>
__device__ __forceinline__ PrimRec load_prim_u(const DScene& S, int i) {
  if constexpr ((F & F_LDS) != 0) return load_prim<F>(S, i);
  const auto q = ro<0>(S.prims) + 3 * i;
  return PrimRec{q[0], q[1], q[2]};
}
__device__ __forceinline__ int prim_type(const PrimRec& q) { return __float_as_int(q.c.z) & RT_PRIM_TYPE_MASK; }

__device__ __forceinline__ bool sphere_t(const Ray& r, V c, float rad, float tmin, float tmax, float& t) {
  const V oc = r.o - c;
  const float a = len2(r.d);
  const float hb = dot(oc, r.d);
  const float cc = len2(oc) - rad * rad;
  const float disc = hb * hb - a * cc;
  if (disc < 0) return false;
  const float sq = __builtin_sqrtf(disc);
  const float root = (-hb - sq) / a;  // the "second root" of sphere.h:51 is the same value (H1)
  if (root < tmin || tmax < root) return false;
  t = root;
  return true;
}
// moving_sphere::center (moving_sphere.h:20-22).  With time0 = 0 and time1 - time0 = 1 (flag
// set at upload) (tm - 0) / 1 is exactly tm, so the division is skipped.
__device__ __forceinline__ V moving_center(const PrimRec& q, float tm) {
  const float sc = (__float_as_int(q.c.z) & RT_PRIM_FLAG_UNIT_T) ? tm : (tm - q.b.w) / q.c.x;
  return mk(q.a.x, q.a.y, q.a.z) + sc * mk(q.b.x, q.b.y, q.b.z);
}
// Rect axis layout: normal axis ax, in-plane axes (ia, ib).
__device__ __forceinline__ void rect_axes(int type, int& ax, int& ia, int& ib) {
  ax = type == RT_PRIM_RECT_XY ? 2 : (type == RT_PRIM_RECT_XZ ? 1 : 0);
  ia = ax == 0 ? 1 : 0;
  ib = ax == 2 ? 1 : 2;
}
// aarect.h hit for the plane comp(ax) = k, a in [a0, a1], b in [b0, b1] over axes (ia, ib).
__device__ __forceinline__ bool rect_tt(const Ray& r, int ax, int ia, int ib, float a0, float a1, float b0, float b1,
                                        float k, float tmin, float tmax, float& t) {
  const float tt = (k - comp(r.o, ax)) / comp(r.d, ax);
  if (tt < tmin || tt > tmax) return false;
  const float a = comp(r.o, ia) + tt * comp(r.d, ia);
  const float b = comp(r.o, ib) + tt * comp(r.d, ib);
  if (a < a0 || a > a1 || b < b0 || b > b1) return false;
  t = tt;
  return true;
}
__device__ __forceinline__ bool rect_t(const Ray& r, const PrimRec& q, int type, float tmin, float tmax, float& t) {
  int ax, ia, ib;
  rect_axes(type, ax, ia, ib);
  return rect_tt(r, ax, ia, ib, q.a.x, q.a.y, q.a.z, q.a.w, q.b.x, tmin, tmax, t);
}
// Face f of box.h's side list (box.h:14-27): xy(z1), xy(z0), xz(y1), xz(y0), yz(x1), yz(x0).
// lo = (x0 y0 z0), hi = (x1 y1 z1).  Returns the rect type; a0..b1, k its extent and plane.
__device__ __forceinline__ int box_face(V lo, V hi, int f, float& a0, float& a1, float& b0, float& b1, float& k) {
  if (f < 2) {
    a0 = lo.x; a1 = hi.x; b0 = lo.y; b1 = hi.y; k = f == 0 ? hi.z : lo.z;
    return RT_PRIM_RECT_XY;
  }
  if (f < 4) {
    a0 = lo.x; a1 = hi.x; b0 = lo.z; b1 = hi.z; k = f == 2 ? hi.y : lo.y;
    return RT_PRIM_RECT_XZ;
  }
  a0 = lo.y; a1 = hi.y; b0 = lo.z; b1 = hi.z; k = f == 4 ? hi.x : lo.x;
  return RT_PRIM_RECT_YZ;
}
// box.h hit = hittable_list over the six faces: t_max shrinks, a later face wins ties.
// Returns the winning face (-1: miss).
__device__ __forceinline__ int box_t(const Ray& r, const PrimRec& q, float tmin, float tmax, float& t) {
  const V lo = mk(q.a.x, q.a.y, q.a.z), hi = mk(q.a.w, q.b.x, q.b.y);
  float closest = tmax;
  int face = -1;
  for (int f = 0; f < 6; ++f) {
    float a0, a1, b0, b1, k, tt;
    int ax, ia, ib;
    rect_axes(box_face(lo, hi, f, a0, a1, b0, b1, k), ax, ia, ib);
    if (rect_tt(r, ax, ia, ib, a0, a1, b0, b1, k, tmin, closest, tt)) {
      closest = tt;
      t = tt;
      face = f;
    }
  }
  return face;
}
__device__ __forceinline__ V cross(V a, V b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// Moller-Trumbore, triangle.h:120-147 (bitwise | of the reference kept as a non-short-circuit or),
// on the operands the device record carries: v0 = p[0..2], e0 = p[3..5], e1 = p[6..8].
__device__ __forceinline__ bool tri_t(const Ray& r, const PrimRec& q, float tmin, float tmax, float& t) {
  const float eps = 0.0000001f;
  const V v0 = mk(q.a.x, q.a.y, q.a.z), e0 = mk(q.a.w, q.b.x, q.b.y), e1 = mk(q.b.z, q.b.w, q.c.x);
  const V h = cross(r.d, e1);
  const float a = dot(e0, h);
  if (a > -eps && a < eps) return false;
  const float f = 1.0f / a;
  const V s = r.o - v0;
  const float u = f * dot(s, h);
  if (u < 0.0f || u > 1.0f) return false;
  const V qq = cross(s, e0);
  const float v = f * dot(r.d, qq);
  if ((v < 0.0f) | (u + v > 1.0f)) return false;
  const float tt = f * dot(e1, qq);
  if (tt < tmin || tt > tmax || tt < eps) return false;
  t = tt;
  return true;
}
// Index of a triangle primitive's 144-byte record (type word bits 12..31, set at upload).
__device__ __forceinline__ int tri_index(const PrimRec& q) { return __float_as_int(q.c.z) >> 12; }

template <int F>
__device__ __forceinline__ bool prim_t_q(const DScene& S, const PrimRec& q, const Ray& r, float tmin, float tmax,
                                         float& t, unsigned& nprim) {
  if constexpr ((F & F_STATS) != 0) ++nprim;
  const int type = prim_type(q);
  if (type <= RT_PRIM_MOVING_SPHERE) {  // one quadratic for both sphere kinds (lanes of a wave mix them)
    V c = mk(q.a.x, q.a.y, q.a.z);
    if constexpr ((F & F_MOVING) != 0)
      if (type == RT_PRIM_MOVING_SPHERE) c = moving_center(q, r.tm);
    return sphere_t(r, c, q.a.w, tmin, tmax, t);
  }
  if constexpr ((F & F_TRI) != 0)
    if (type == RT_PRIM_TRIANGLE) return tri_t(r, q, tmin, tmax, t);
  if constexpr ((F & F_RECT) != 0) {
    if (type >= RT_PRIM_RECT_XY && type <= RT_PRIM_RECT_YZ) return rect_t(r, q, type, tmin, tmax, t);
    if (type == RT_PRIM_BOX) {
      if constexpr ((F & F_STATS) != 0) nprim += 5;  // six rect hit() calls, as the list counts them
      return box_t(r, q, tmin, tmax, t) >= 0;
    }
  }
  return false;
}
template <int F>
__device__ __forceinline__ bool prim_t(const DScene& S, int pi, const Ray& r, float tmin, float tmax, float& t,
                                       unsigned& nprim) {
  return prim_t_q<F>(S, load_prim<F>(S, pi), r, tmin, tmax, t, nprim);
}

// Candidate range of primitive q for the culled BVH search: an interval [lo, hi] that contains the
// t the reference's hit() returns, or false when the reference certainly rejects the primitive.
// Spheres: the discriminant is the reference's own float value (same operations, so the miss
// test disc < 0 is exact), the root comes from the hardware sqrt and reciprocal (a few ulp)
// instead of the correctly rounded sqrt and divide; e bounds |root - reference root| with a
// margin of ~4x (each of sqrt, reciprocal, subtraction and product is within 2 ulp of exact, the
// reference's own roundings within 0.5 ulp).  The exact root of the winner is computed once, in
// bvh_settle.  rcpa = rcp(|d|^2) of the query.  Other primitives: their exact t (lo = hi).
template <int F>
__device__ __forceinline__ bool prim_range(const DScene& S, const PrimRec& q, const Ray& r, float a, float rcpa,
                                           float tmin, float tmax, float& lo, float& hi, unsigned& nprim) {
  const int type = prim_type(q);
  if (type <= RT_PRIM_MOVING_SPHERE) {
    if constexpr ((F & F_STATS) != 0) ++nprim;
    V c = mk(q.a.x, q.a.y, q.a.z);
    if constexpr ((F & F_MOVING) != 0)
      if (type == RT_PRIM_MOVING_SPHERE) c = moving_center(q, r.tm);
    const float rad = q.a.w;
    const V oc = r.o - c;
    const float hb = dot(oc, r.d);
    const float cc = len2(oc) - rad * rad;
    const float disc = hb * hb - a * cc;
    if (disc < 0) return false;
    const float sq = __builtin_amdgcn_sqrtf(disc);
    const float num = -hb - sq;
    const float ra = num * rcpa;
    const float e = __builtin_fmaf((sq + __builtin_fabsf(num)) * 0x1p-19f + 1e-12f, rcpa,
                                   __builtin_fabsf(ra) * 0x1p-20f);
    lo = ra - e;
    hi = ra + e;
    if (!(e < __builtin_inff())) {  // degenerate direction: no usable bound, the query goes exact
      lo = -__builtin_inff();
      hi = __builtin_inff();
      return true;
    }
    return !(hi < tmin || lo > tmax);
  }
  float t;
  if (!prim_t_q<F>(S, q, r, tmin, tmax, t, nprim)) return false;
  lo = t;
  hi = t;
  return true;
}

// Full hit record of primitive pi at parameter t (the fields hit() sets on success).
template <int F>
__device__ __forceinline__ void finalize(const DScene& S, int pi, const Ray& r, float tmin, float t, Hit& h) {
  const PrimRec q = load_prim<F>(S, pi);
  const int tw = __float_as_int(q.c.z);
  const int type = tw & RT_PRIM_TYPE_MASK;
  h.t = t;
  h.mat = __float_as_int(q.c.w);
  h.p = r.o + t * r.d;
  if (type == RT_PRIM_SPHERE || type == RT_PRIM_MOVING_SPHERE) {
    const V c = type == RT_PRIM_SPHERE ? mk(q.a.x, q.a.y, q.a.z) : moving_center(q, r.tm);
    const V out = (1.0f / q.a.w) * (h.p - c);
    set_face(h, r, out);
    h.u = 0.0f;  // moving_sphere leaves u,v stale (H13): defined as 0
    h.v = 0.0f;
    if constexpr ((F & F_IMAGE) != 0) {
      if (type == RT_PRIM_SPHERE && (tw & RT_PRIM_FLAG_UV)) {  // sphere.h:19-32
        const float pi_f = 3.1415927f;
        h.u = (rtm::det_atan2f(-out.z, out.x) + pi_f) / (2.0f * pi_f);
        h.v = rtm::det_acosf(-out.y) / pi_f;
      }
    }
    return;
  }
  if constexpr ((F & F_TRI) != 0) {
   if (type == RT_PRIM_TRIANGLE) {  // triangle.h:151-175
    const rt_triangle& T = S.tris[tri_index(q)];
    const V v2 = h.p - ld3(T.v0);
    const V e0 = ld3(T.e0), e1 = ld3(T.e1);
    const float d20 = dot(v2, e0), d21 = dot(v2, e1);
    const float b0 = (T.d11 * d20 - T.d01 * d21) * T.inv_denom;
    const float b1 = (T.d00 * d21 - T.d01 * d20) * T.inv_denom;
    const float b2 = 1.0f - b0 - b1;
    h.u = b2 * T.uv[0] + b0 * T.uv[2] + b1 * T.uv[4];
    h.v = b2 * T.uv[1] + b0 * T.uv[3] + b1 * T.uv[5];
    if (!T.vertex_normals) {
      set_face(h, r, cross(e1, e0));
    } else {
      const V n = mk(b2 * T.n0[0] + b0 * T.n1[0] + b1 * T.n2[0], b2 * T.n0[1] + b0 * T.n1[1] + b1 * T.n2[1],
                     b2 * T.n0[2] + b0 * T.n1[2] + b1 * T.n2[2]);
      set_face(h, r, n);
    }
    return;
   }
  }
  if constexpr ((F & F_RECT) != 0) {  // aarect.h
    float a0 = q.a.x, b0 = q.a.z, wa = q.b.y, wb = q.b.z;
    int rt = type;
    if (type == RT_PRIM_BOX) {  // the face that won: the last one at exactly t in [tmin, t]
      float tt, a1, b1, k;
      const int f = box_t(r, q, tmin, t, tt);
      rt = box_face(mk(q.a.x, q.a.y, q.a.z), mk(q.a.w, q.b.x, q.b.y), f < 0 ? 0 : f, a0, a1, b0, b1, k);
      wa = a1 - a0;
      wb = b1 - b0;
    }
    int ax, ia, ib;
    rect_axes(rt, ax, ia, ib);
    const float a = comp(r.o, ia) + t * comp(r.d, ia);
    const float b = comp(r.o, ib) + t * comp(r.d, ib);
    h.u = (a - a0) / wa;
    h.v = (b - b0) / wb;
    set_face(h, r, mk(ax == 0 ? 1.0f : 0.0f, ax == 1 ? 1.0f : 0.0f, ax == 2 ? 1.0f : 0.0f));
  }
}

// ------------------------------------------------------------------ BVH (bvh.h:348-436)
// Kensler slab test, aabb.h:19-104, with the reciprocal hoisted per ray (same value as the
// reference's per-node 1.0f/d).  Select-based min/max keep the reference's NaN behaviour.
__device__ __forceinline__ bool slab(float lo, float hi, float o, float inv, float& tmin, float& tmax) {
  float t0 = (lo - o) * inv;
  float t1 = (hi - o) * inv;
  if (inv < 0.0f) {
    const float tmp = t0;
    t0 = t1;
    t1 = tmp;
  }
  tmin = t0 > tmin ? t0 : tmin;
  tmax = t1 < tmax ? t1 : tmax;
  return !(tmax <= tmin);
}
__device__ __forceinline__ bool box_hit(float4 lo, float4 hi, const Ray& r, V inv, float tmin, float tmax) {
  if (!slab(lo.x, hi.x, r.o.x, inv.x, tmin, tmax)) return false;
  if (!slab(lo.y, hi.y, r.o.y, inv.y, tmin, tmax)) return false;
  return slab(lo.z, hi.z, r.o.z, inv.z, tmin, tmax);
}

// Conservative box test for the traversal tree: fma form, NaN-tolerant min/max, inclusive.
// Returns the entry distance in tn.
__device__ __forceinline__ bool fbox(float4 lo, float4 hi, V oi, V inv, float tmin, float tcut, float& tn) {
  const float x0 = __builtin_fmaf(lo.x, inv.x, -oi.x), x1 = __builtin_fmaf(hi.x, inv.x, -oi.x);
  const float y0 = __builtin_fmaf(lo.y, inv.y, -oi.y), y1 = __builtin_fmaf(hi.y, inv.y, -oi.y);
  const float z0 = __builtin_fmaf(lo.z, inv.z, -oi.z), z1 = __builtin_fmaf(hi.z, inv.z, -oi.z);
  const float tnear = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(x0, x1), __builtin_fminf(y0, y1)),
                                      __builtin_fmaxf(__builtin_fminf(z0, z1), tmin));
  const float tfar = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(x0, x1), __builtin_fmaxf(y0, y1)),
                                     __builtin_fminf(__builtin_fmaxf(z0, z1), tcut));
  tn = tnear;
  return tnear <= tfar;
}

// Closest primitive of a reference-layout BVH with the reference's exact visit set: a node's box
// is tested iff its parent's box passed (bvh.h:348-436), against the caller's [tmin, tmax],
// depth-first, left first; leaves keep strictly smaller t (first hit wins ties).  Both children
// of a node are tested from one 64-byte fetch (siblings are adjacent in heap order), halving the
// chain of dependent loads; `pending` keeps, per level, whether a right child is still to visit.
template <int F>
__device__ __forceinline__ bool bvh_exact(const DScene& S, int base, int rows, const Ray& r, V inv, float tmin, float tmax,
                          float& best, int& best_prim, unsigned& nnode, unsigned& nprim, unsigned& nfall) {
  const int last0 = (1 << (rows - 1)) - 1;
  best = __builtin_inff();
  best_prim = -1;
  if constexpr ((F & F_STATS) != 0) ++nnode;
  {
    const float4 lo = nodes_of<F>(S)[2 * base], hi = nodes_of<F>(S)[2 * base + 1];
    if (!box_hit(lo, hi, r, inv, tmin, tmax)) return false;
  }
  unsigned pending = 0;
  int level = 0, k = 0;
  for (;;) {
    // invariant: the box of node k passed
    if (k >= last0) {
      const float4 lo = nodes_of<F>(S)[2 * (base + k)], hi = nodes_of<F>(S)[2 * (base + k) + 1];
      float t;
      const int pa = __float_as_int(lo.w), pb = __float_as_int(hi.w);
      if (prim_t<F>(S, pa, r, tmin, tmax, t, nprim) && t < best) {
        best = t;
        best_prim = pa;
      }
      if (pb >= 0 && prim_t<F>(S, pb, r, tmin, tmax, t, nprim) && t < best) {
        best = t;
        best_prim = pb;
      }
    } else {
      const float4* c = nodes_of<F>(S) + 2 * (base + 2 * k + 1);
      const float4 l0 = c[0], l1 = c[1], r0 = c[2], r1 = c[3];
      if constexpr ((F & F_STATS) != 0) nnode += 2;
      const bool hl = box_hit(l0, l1, r, inv, tmin, tmax);
      const bool hr = box_hit(r0, r1, r, inv, tmin, tmax);
      if (hl || hr) {
        pending = (pending & ~(1u << level)) | ((hl && hr) ? (1u << level) : 0u);
        ++level;
        k = 2 * k + (hl ? 1 : 2);
        continue;
      }
    }
    for (;;) {  // climb to the deepest level with a pending right child
      if (level == 0) return best_prim >= 0;
      --level;
      k = (k - 1) >> 1;
      if (pending & (1u << level)) {
        pending &= ~(1u << level);
        ++level;
        k = 2 * k + 2;
        break;
      }
    }
  }
}

// One candidate of the culled search (a primitive whose range test passed): the lane keeps the
// candidate with the smallest lo as the winner [blo, bhi] and the smallest lo of every other
// candidate in `second`; the winner is certain when second > bhi (checked in bvh_settle).  Two exact
// candidates (lo = hi) of one BVH compare exactly, as bvh.h does (strictly smaller t, ties to the
// lower leaf rank), and the loser is not kept in `second`: an exact loser of an exact winner has
// t >= the winner's t, so when a range later displaces that winner, the winner's lo (added to
// `second`) covers it.
// World keys (WORLD: world_search, the world tree): candidates of different world entries carry
// different entry parts of the tie key (rk >> RT_WKEY_SHIFT).  An exact candidate of another entry is
// never dropped from `second`, whichever of the two arrives first: it bounds the closest-so-far that
// the reference's list passes to the winner's entry (world_settle, world_search), and an exact tie
// across entries leaves second == bhi, so the query is not certain -- whatever the visiting order.
template <bool WORLD = false>
__device__ __forceinline__ void take_candidate(float lo, float hi, int pi, int rk, float& blo, float& bhi,
                                               float& second, int& best_prim, int& best_rank) {
  if (lo == hi && blo == bhi) {  // both exact: the reference's rule, ties to the lower rank
    const bool other = WORLD && (rk >> RT_WKEY_SHIFT) != (best_rank >> RT_WKEY_SHIFT);
    if (lo < blo || (lo == blo && rk < best_rank)) {
      if (other) second = __builtin_fminf(second, blo);
      blo = lo;
      bhi = hi;
      best_prim = pi;
      best_rank = rk;
    } else if (other) {
      second = __builtin_fminf(second, lo);
    }
  } else if (lo < blo) {
    second = __builtin_fminf(second, blo);
    blo = lo;
    bhi = hi;
    best_prim = pi;
    best_rank = rk;
  } else {
    second = __builtin_fminf(second, lo);
  }
}

// One pair record of the quantized traversal tree (F_QLDS, build_qtree), 6 words in LDS:
//   w0 = origin x | y (binary16, rounded down), w1 = origin z | (ex | ey << 5 | ez << 10) << 16,
//   w2..w4 = child 0 lo xyz, hi xyz, child 1 lo xyz, hi xyz as bytes q (box coordinate origin +
//   q * 2^(e + q_ebias), lo rounded down and hi up from the padded box), w5 = child 0 | child 1 (16-bit
//   child words: pair index, or -1 - primitive).
// Slab values t = (origin + q 2^E - o) / d as fma(q, A, B) with A = 2^E finv, B = origin finv - oi per
// axis: two instructions per axis on top of fbox's one fma per bound.  The quantized boxes contain the
// padded ones (2^-16 relative), far wider than the few roundings of A, B and the fma.
__device__ __forceinline__ float q_half(uint32_t bits16) {
  const uint16_t b = (uint16_t)bits16;
  _Float16 h;
  __builtin_memcpy(&h, &b, 2);
  return (float)h;
}
__device__ __forceinline__ float q_byte(uint32_t w, int k) { return (float)((w >> (8 * k)) & 255u); }
__device__ __forceinline__ bool qbox(float lx, float ly, float lz, float hx, float hy, float hz, V A, V B, float tmin,
                                     float tcut, float& tn) {
  const float x0 = __builtin_fmaf(lx, A.x, B.x), x1 = __builtin_fmaf(hx, A.x, B.x);
  const float y0 = __builtin_fmaf(ly, A.y, B.y), y1 = __builtin_fmaf(hy, A.y, B.y);
  const float z0 = __builtin_fmaf(lz, A.z, B.z), z1 = __builtin_fmaf(hz, A.z, B.z);
  const float tnear = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(x0, x1), __builtin_fminf(y0, y1)),
                                      __builtin_fmaxf(__builtin_fminf(z0, z1), tmin));
  const float tfar = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(x0, x1), __builtin_fmaxf(y0, y1)),
                                     __builtin_fminf(__builtin_fmaxf(z0, z1), tcut));
  tn = tnear;
  return tnear <= tfar;
}
__device__ __forceinline__ void qpair(const DScene& S, int cur, V oi, V finv, float tmin, float tcut, bool& hl,
                                      bool& hr, float& tl, float& tr, int& c0, int& c1) {
  const uint2* rec = reinterpret_cast<const uint2*>((const uint32_t*)rt_lds + 6 * cur);
  const uint2 a = rec[0], b = rec[1], c = rec[2];
  const uint32_t ee = a.y >> 16;
  const V org = mk(q_half(a.x), q_half(a.x >> 16), q_half(a.y));
  const V sc = mk(__builtin_ldexpf(1.0f, (int)(ee & 31u) + S.q_ebias), __builtin_ldexpf(1.0f, (int)((ee >> 5) & 31u) + S.q_ebias),
                  __builtin_ldexpf(1.0f, (int)((ee >> 10) & 31u) + S.q_ebias));
  const V A = mk(sc.x * finv.x, sc.y * finv.y, sc.z * finv.z);
  const V B = mk(__builtin_fmaf(org.x, finv.x, -oi.x), __builtin_fmaf(org.y, finv.y, -oi.y),
                 __builtin_fmaf(org.z, finv.z, -oi.z));
  hl = qbox(q_byte(b.x, 0), q_byte(b.x, 1), q_byte(b.x, 2), q_byte(b.x, 3), q_byte(b.y, 0), q_byte(b.y, 1), A, B,
            tmin, tcut, tl);
  hr = qbox(q_byte(b.y, 2), q_byte(b.y, 3), q_byte(c.x, 0), q_byte(c.x, 1), q_byte(c.x, 2), q_byte(c.x, 3), A, B,
            tmin, tcut, tr);
  c0 = (int)(short)(c.y & 0xffffu);
  c1 = (int)(short)(c.y >> 16);
}

// KEYED (world_search): candidates carry the tie key kbase | reference leaf rank of their list entry
// and follow take_candidate<true>'s cross-entry rule.
template <int F, bool KEYED = false>
__device__ __forceinline__ bool trav_step(const DScene& S, int fb, const Ray& r, V oi, V finv, float a, float rcpa,
                                          float tmin, float tmax, int& cur, int& sp, float& blo, float& bhi,
                                          float& second, int& best_prim, int& best_rank, bool& overflow,
                                          unsigned& nnode, unsigned& nprim, int kbase = 0) {
  stack_t<F>* stk = stack_of<F>(S);
  constexpr int BS = render_block<F>();
  RT_STAMP(3);
  if constexpr ((F & F_STATS) != 0) nnode += 2;
  // bhi >= the winner's exact t: a box entered beyond bhi*(1+2^-8) holds no primitive that can win
  const float cut = __builtin_fminf(bhi * 1.00390625f, tmax);
  float tl, tr;
  bool hl, hr;
  int c0, c1;
  if constexpr ((F & F_QLDS) != 0) {
    qpair(S, cur, oi, finv, tmin, cut, hl, hr, tl, tr, c0, c1);
  } else {
    float4 l0, l1, r0, r1;
    if constexpr (planes<F>()) {  // the four planes of the staged tree (stage_lds)
      const float4* n = nodes_of<F>(S) + 2 * fb + cur;
      l0 = n[0];
      l1 = n[kPlanePairs];
      r0 = n[2 * kPlanePairs];
      r1 = n[3 * kPlanePairs];
    } else {
      const float4* n = nodes_of<F>(S) + 2 * (fb + 2 * cur);
      l0 = n[0];
      l1 = n[1];
      r0 = n[2];
      r1 = n[3];
    }
    hl = fbox(l0, l1, oi, finv, tmin, cut, tl);
    hr = fbox(r0, r1, oi, finv, tmin, cut, tr);
    c0 = __float_as_int(l0.w);
    c1 = __float_as_int(l1.w);
  }
  // Primitive children are tested right away (leaves hold one primitive): one pass for the lanes
  // with a hit leaf child on either side, a second only for lanes with two (the candidate kept does
  // not depend on the order, see take_candidate).  3 % faster on C2 than a pass per side.
  {
    const bool la = hl && c0 < 0, lb = hr && c1 < 0;
    const int p0 = la ? c0 : (lb ? c1 : 0);
    const int p1 = (la && lb) ? c1 : 0;
    if (la) hl = false;
    if (lb) hr = false;
    #pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int ch = pass == 0 ? p0 : p1;
      if (ch < 0) {
        RT_STAMP(4);
        const int pi = -ch - 1;
        if constexpr ((F & F_WORLD) != 0) {
          // world-tree leaf: its record, tested in its instance's frame (the reference's ray for
          // that entry, hittable.h:37-59, 112-143) when it belongs to a translate/rotate_y
          const float4* L = S.wleaf + 4 * pi;
          const PrimRec q{L[0], L[1], L[2]};
          float lo, hi;
          Ray rr = r;
          float a2 = a, rc2 = rcpa;
          if ((F & F_XFORM) != 0 && (__float_as_int(q.c.z) & RT_PRIM_FLAG_XF) != 0) {
            const int xf = __float_as_int(L[3].x);
            Ray moved;
            rr = xform_ray_x(S.wxf[2 * xf], S.wxf[2 * xf + 1], r, moved);
            a2 = len2(rr.d);
            rc2 = __builtin_amdgcn_rcpf(a2);
          }
          if (prim_range<F>(S, q, rr, a2, rc2, tmin, tmax, lo, hi, nprim))
            take_candidate<true>(lo, hi, pi, __float_as_int(q.c.y), blo, bhi, second, best_prim, best_rank);
        } else {
          const PrimRec q = load_prim<F>(S, pi);
          float lo, hi;
          if (prim_range<F>(S, q, r, a, rcpa, tmin, tmax, lo, hi, nprim)) {
            if constexpr (KEYED)
              take_candidate<true>(lo, hi, pi, kbase | __float_as_int(q.c.y), blo, bhi, second, best_prim, best_rank);
            else
              take_candidate(lo, hi, pi, __float_as_int(q.c.y), blo, bhi, second, best_prim, best_rank);
          }
        }
        RT_STAMP(3);
      }
    }
  }
  if (hl && hr) {
    const bool right_first = tr < tl;
    if (sp < kStackDepth) stk[BS * sp++] = (stack_t<F>)(right_first ? c0 : c1);
    else overflow = true;
    cur = right_first ? c1 : c0;
    return true;
  }
  if (hl || hr) {
    cur = hl ? c0 : c1;
    return true;
  }
  if (sp == 0) return false;
  cur = stk[BS * --sp];
  return true;
}

// Camera-ray candidates of a world BVH from the per-tile candidate list (bin_tiles_kernel): every
// primitive that any camera ray of the 8x8-pixel tile can hit, over the lens disk and the shutter,
// is in the list, so the candidates of the culled search are all tested here instead of traversing
// the tree; bvh_settle then decides the query exactly as after a traversal.  Entries are (primitive,
// nearest) pairs sorted by `nearest`, a lower bound on the distance from the ray origin to any
// point of the primitive: once nearest / |d| exceeds the winner's range end bhi (with the
// traversal's 2^-8 margin) the remaining candidates lie beyond it -- a lo above bhi changes neither
// the winner nor the certainty test second > bhi -- and the loop ends.  Two pairs per 16-byte load,
// the next load issued before the current pair's tests; g0 = the first pair(s), loaded by the
// caller together with the count.
template <int F>
__device__ __forceinline__ void tile_candidates(const DScene& S, const int32_t* __restrict__ ent, int cnt, int4 g0,
                                                const Ray& r, float a, float rcpa, float tmin, float tmax,
                                                float& blo, float& bhi, float& second, int& best_prim,
                                                int& best_rank, unsigned& nprim) {
  const float rlen = __builtin_amdgcn_rsqf(a) * 0.99951171875f;  // 1/|d|, rounded well down (1 - 2^-11)
  const int4* __restrict__ e4 = reinterpret_cast<const int4*>(ent);
  int4 gn = g0;
  for (int k = 0; k < cnt; k += 2) {
    const int4 g = gn;
    if (k + 2 < cnt) gn = e4[(k >> 1) + 1];
    if (__int_as_float(g.y) * rlen > bhi * 1.00390625f) break;  // sorted: the rest lie beyond the winner
    #pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (k + u < cnt) {
        const int pi = u == 0 ? g.x : g.z;
        if (u == 1 && __int_as_float(g.w) * rlen > bhi * 1.00390625f) break;
        const PrimRec q = load_prim<F>(S, pi);
        float lo, hi;
        if (prim_range<F>(S, q, r, a, rcpa, tmin, tmax, lo, hi, nprim))
          take_candidate(lo, hi, pi, __float_as_int(q.c.y), blo, bhi, second, best_prim, best_rank);
      }
    }
  }
}

// Reference-chain validation of a candidate search's winner (best_prim at exact t = best, reference
// leaf rank best_rank of the BVH at `base` with `rows` inner levels): true when the reference's
// visit set certainly reaches it, i.e. every reference ancestor passes the slab test against
// [tmin, tmax]; false when that is not certain (the caller re-runs the query exactly).
template <int F>
__device__ __forceinline__ bool chain_ok(const DScene& S, int base, int rows, const Ray& r, float tmin, float tmax,
                                         float best, int best_prim, int best_rank, unsigned& nnode) {
  const int last0 = (1 << (rows - 1)) - 1;
  // Reference ancestors whose box contains the winner's box with a margin wider than any
  // displacement of its computed hit point (hit-distance error up to ~4e-4 t for grazing
  // spheres, slab rounding 2^-22 of the distance) cannot reject this ray, so only the other
  // chain positions are tested.  pmargin = {bitmask of chain positions with margin < 0.05,
  // smallest margin among the rest} (computed at upload).
  const float dmax = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.d.x), __builtin_fabsf(r.d.y)),
                                     __builtin_fabsf(r.d.z));
  const float bound = 0.001953125f * best * dmax;  // 2^-9 * t * |d|_inf
  if constexpr ((F & (F_LDS | F_MEDIUM)) == 0 && (F & F_TRI) != 0) {
    // The loop below in one 48-byte fetch, in global-memory mesh variants, where every ancestor node
    // is an L2 round trip (C4 door: the loop's dependent fetches were ~19 % of a launch).  It comes
    // first there: 0.7 % faster on C4 than after the sphere test.  Not in C3's rect variant (no gain
    // measured) nor in C5's, which spills (0.6 % slower).  pvalid = {box of the LOWEST position of the
    // `must` set below, mask}, {its hi, safe}, {largest |coordinate| over the `must` boxes}.  Those boxes contain the lowest one
    // (checked at upload), so the computed hit point is at least as deep inside each as inside the
    // lowest, and each one's margin `need` (below) is at most the record's: a hit point deeper than that
    // inside the lowest one passes the loop's test at every position -- the loop's own answer, true.
    const float4 v0 = S.pvalid[3 * best_prim], v1 = S.pvalid[3 * best_prim + 1], v2 = S.pvalid[3 * best_prim + 2];
    if (bound < v1.w) {  // the loop's `must` is the mask (else every position is tested)
      if (__float_as_uint(v0.w) == 0u) return true;
      const V p = r.o + best * r.d;
      const float dx = __builtin_fminf(p.x - v0.x, v1.x - p.x);
      const float dy = __builtin_fminf(p.y - v0.y, v1.y - p.y);
      const float dz = __builtin_fminf(p.z - v0.z, v1.z - p.z);
      const float need_max = 0x1p-20f * (v2.x + 2.0f * (__builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.o.x),
                                                                                      __builtin_fabsf(r.o.y)),
                                                                       __builtin_fabsf(r.o.z)) + best * dmax));
      if (__builtin_fminf(__builtin_fminf(dx, dy), dz) > need_max) return true;
    }
  }
  {
    // Every reference ancestor contains the winner's box, so a computed hit point deeper inside
    // the winner's own box than `bound` passes all of them: a sphere touches its box only at
    // six points, so the chain is rarely tested at all.  (Moving spheres: the box at the ray's
    // time lies inside the box over the shutter.  A negative radius inverts the box: no skip.)
    const PrimRec q = load_prim<F>(S, best_prim);
    const int ty = prim_type(q);
    if (ty == RT_PRIM_SPHERE || ((F & F_MOVING) != 0 && ty == RT_PRIM_MOVING_SPHERE)) {
      V c = mk(q.a.x, q.a.y, q.a.z);
      if constexpr ((F & F_MOVING) != 0)
        if (ty == RT_PRIM_MOVING_SPHERE) c = moving_center(q, r.tm);
      const V p = r.o + best * r.d;
      const float rad = q.a.w;
      const float mx = __builtin_fminf(p.x - (c.x - rad), (c.x + rad) - p.x);
      const float my = __builtin_fminf(p.y - (c.y - rad), (c.y + rad) - p.y);
      const float mz = __builtin_fminf(p.z - (c.z - rad), (c.z + rad) - p.z);
      // the chain check's per-ancestor margin below, taken at its largest: the root box's magnitude
      const float4 rlo = nodes_of<F>(S)[2 * base], rhi = nodes_of<F>(S)[2 * base + 1];
      const float rmax = __builtin_fmaxf(
          __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(rlo.x), __builtin_fabsf(rlo.y)), __builtin_fabsf(rlo.z)),
          __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(rhi.x), __builtin_fabsf(rhi.y)), __builtin_fabsf(rhi.z)));
      const float need = 0x1p-20f * (rmax + 2.0f * (__builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.o.x),
                                                                                   __builtin_fabsf(r.o.y)),
                                                                    __builtin_fabsf(r.o.z)) + best * dmax));
      if (__builtin_fminf(__builtin_fminf(mx, my), mz) > __builtin_fminf(bound, need)) return true;

    }
  }
  const float2 pm = pmargin_of<F>(S)[best_prim];
  const unsigned must = bound < pm.y ? __float_as_uint(pm.x) : 0xffffffffu;
  // The remaining positions: an ancestor whose box holds the computed hit point deeper than
  // `bound` cannot reject the ray either (the same argument as for the winner's own box, on the
  // actual hit point instead of the primitive's box: triangles and rects touch their boxes along
  // whole faces, but a hit point rarely lies near an ancestor's faces); the others get the
  // reference's slab test, with its IEEE reciprocals.
  // Margin needed here: the reference's slab values (lo - o) * RN(1/d) carry ~3 roundings of
  // |lo - o| <= |lo| + |o| in distance terms, and p = o + t d (our float evaluation at the
  // reference's own t) is within a few ulp of |o| + t |d|: 2^-20 of their sum is > 4x both.
  const V p = r.o + best * r.d;
  const float obase = 2.0f * (__builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.o.x), __builtin_fabsf(r.o.y)),
                                              __builtin_fabsf(r.o.z)) + best * dmax);
  int pos = 0;
  for (int kr = last0 + (best_rank >> 1);; kr = (kr - 1) >> 1, ++pos) {
    if ((must >> pos) & 1u) {
      if constexpr ((F & F_STATS) != 0) ++nnode;
      const float4 lo = nodes_of<F>(S)[2 * (base + kr)], hi = nodes_of<F>(S)[2 * (base + kr) + 1];
      const float mx = __builtin_fminf(p.x - lo.x, hi.x - p.x);
      const float my = __builtin_fminf(p.y - lo.y, hi.y - p.y);
      const float mz = __builtin_fminf(p.z - lo.z, hi.z - p.z);
      const float bmax = __builtin_fmaxf(
          __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(lo.x), __builtin_fabsf(lo.y)), __builtin_fabsf(lo.z)),
          __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(hi.x), __builtin_fabsf(hi.y)), __builtin_fabsf(hi.z)));
      const float need = 0x1p-20f * (bmax + obase);
      if (!(__builtin_fminf(__builtin_fminf(mx, my), mz) > need)) {
        // the reference's reciprocals (three IEEE divides), only on this rare path
        if (!box_hit(lo, hi, r, mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z), tmin, tmax)) return false;
      }
    }
    if (kr == 0) return true;
  }
}

// Second half of bvh_closest once the candidate search has ended: overflow fallback, audit mode,
// and the reference-chain validation of the candidate (best_rank = its reference leaf rank).
template <int F>
__device__ __forceinline__ bool bvh_settle(const DScene& S, int base, int rows, const Ray& r, float tmin, float tmax,
                                           bool overflow, float bhi, float second, float& best, int& best_prim,
                                           int best_rank, unsigned& nnode, unsigned& nprim, unsigned& nfall) {
  // the reference's reciprocals (three IEEE divides), only on the rare paths that test boxes
  auto inv_of = [&r]() { return mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z); };
  // The candidate search keeps ranges: its winner is certain when every other candidate's range
  // lies above the winner's (second > bhi), and its exact t (the reference's hit() value) must
  // pass [tmin, tmax].  Otherwise -- a subtree dropped on stack overflow, overlapping ranges (near
  // ties), a range straddling tmin -- the query is answered on the exact visit set.
  // On entry best = the winner's lo (= its exact t when lo = hi).
  bool sure = !overflow && (best_prim < 0 || second > bhi);  // no candidate at all: a certain miss
  if (sure && best_prim >= 0 && best != bhi) {
    float t;
    unsigned np = 0;
    sure = prim_t<F>(S, best_prim, r, tmin, tmax, t, np);
    best = t;
  }
  if (!sure) {
    if constexpr ((F & F_STATS) != 0) ++nfall;
    return bvh_exact<F>(S, base, rows, r, inv_of(), tmin, tmax, best, best_prim, nnode, nprim, nfall);
  }
  if constexpr ((F & F_CHECK) != 0) {
    float te;
    int pe;
    bvh_exact<F>(S, base, rows, r, inv_of(), tmin, tmax, te, pe, nnode, nprim, nfall);
    if (pe != best_prim || (pe >= 0 && __float_as_uint(te) != __float_as_uint(best))) {
      const unsigned slot = atomicAdd(S.dbg_n, 1u);
      if ((int)slot < S.dbg_cap) {
        float* e = S.dbg + 16 * slot;
        e[0] = r.o.x; e[1] = r.o.y; e[2] = r.o.z; e[3] = r.d.x; e[4] = r.d.y; e[5] = r.d.z; e[6] = r.tm;
        e[7] = tmin; e[8] = tmax; e[9] = best; e[10] = __int_as_float(best_prim); e[11] = te;
        e[12] = __int_as_float(pe); e[13] = __int_as_float(best_rank); e[14] = 0.0f; e[15] = 0.0f;
      }
    }
    best = te;
    best_prim = pe;
    return pe >= 0;
  }
  if (best_prim < 0) return false;
  if (chain_ok<F>(S, base, rows, r, tmin, tmax, best, best_prim, best_rank, nnode)) return true;
  if constexpr ((F & F_STATS) != 0) ++nfall;
  return bvh_exact<F>(S, base, rows, r, inv_of(), tmin, tmax, best, best_prim, nnode, nprim, nfall);
}

// A ray whose sphere tests cannot produce a NaN root against the scene's inert media boundaries
// (spheres with coordinates and radii below 1e6, moving ones whose centre stays within 1e6 of c0 for
// |time| < 1024, checked at upload by medium_inert): finite, |o| < 1e7, |time| < 1024, 1e-12 < |d|^2
// < 1e8 -- then hb^2 and a*cc stay below ~1e23, and root = num / a is finite.  NaN and inf fail the
// comparisons.
__device__ __forceinline__ bool ray_sane(const Ray& r) {
  const float a = len2(r.d);
  const float om = __builtin_fabsf(r.o.x) + __builtin_fabsf(r.o.y) + __builtin_fabsf(r.o.z);
  return a > 1e-12f && a < 1e8f && om < 1e7f && __builtin_fabsf(r.tm) < 1024.0f;
}

// Outcome of the world tree's candidate search (F_WORLD; leaf = winning leaf, key its tie key):
// 0 = certain miss, 1 = certain hit (best = the reference's t; wobj / prim = its world object and
// primitive), 2 = not certain: the caller answers the query on the reference's sequential list.
// The reference's list (hittable_list.h:23-39) queries the winner's entry with t_max = the closest
// hit of the entries before it; that value is at least `lim`: every candidate of another entry lies
// at or above `second` (take_candidate<true>), and a box culled beyond the cut bhi*(1+2^-8) holds
// only primitives hit beyond bhi*(1+2^-9).  The winner's reference chain is validated against
// [tmin, lim]: a slab test that passes there passes for any larger t_max.
template <int F>
__device__ __forceinline__ int world_settle(const DScene& S, const Ray& r, float tmin, bool overflow, float bhi,
                                            float second, float& best, int leaf, int key, int& wobj, int& prim,
                                            unsigned& nnode) {
  if (overflow || (leaf >= 0 && !(second > bhi))) return 2;
  if (leaf < 0) return 0;
  const float4* L = S.wleaf + 4 * leaf;
  const PrimRec q{L[0], L[1], L[2]};
  const float4 dw = L[3];
  Ray rr = r;
  if ((F & F_XFORM) != 0 && (__float_as_int(q.c.z) & RT_PRIM_FLAG_XF) != 0) {
    const int xf = __float_as_int(dw.x);
    Ray moved;
    rr = xform_ray_x(S.wxf[2 * xf], S.wxf[2 * xf + 1], r, moved);
  }
  if (best != bhi) {  // a range: the exact root once, IEEE sqrt and divide
    float t;
    unsigned np = 0;
    if (!prim_t_q<F>(S, q, rr, tmin, __builtin_inff(), t, np)) return 2;
    best = t;
  }
  const int bobj = __float_as_int(dw.z);
  prim = __float_as_int(dw.w);
  if (bobj >= 0) {
    const int base = ro<F>(S.objects)[bobj].a, rows = ro<F>(S.objects)[bobj].b;
    const float lim = __builtin_fminf(second, bhi * 1.0009765625f);
    if (!chain_ok<F>(S, base, rows, rr, tmin, lim, best, prim, key & ((1 << RT_WKEY_SHIFT) - 1), nnode)) return 2;
  }
  wobj = ro<F>(S.world)[__float_as_int(dw.y)];
  return 1;
}

// Closest primitive of a reference BVH object, same result as bvh_exact.
//  1. Candidate search on the object's traversal tree (built at upload: same perfect-tree shape,
//     largest-extent median splits, boxes padded by 2^-16 relative): both children per 64-byte
//     fetch, nearer child first, boxes culled once their entry exceeds best*(1+2^-8).  Every
//     primitive lies inside its padded ancestors, so a culled primitive's hit distance exceeds
//     the box entry up to rounding (<= ~4e-4 relative for grazing spheres): strictly farther
//     than best, it could not have won.  Ties go to the lower rank in the reference's depth-first
//     left-first leaf order (first hit wins, bvh.h:375).
//  2. The candidate wins in the reference iff the reference visits it: its last-row node and every
//     ancestor pass the reference slab test against [tmin, tmax].  If that check fails (a
//     floating-point edge of the reference's own boxes), the query is re-run on the exact visit set.
template <int F>
__device__ __forceinline__ bool bvh_closest(const DScene& S, const rt_object& o, const Ray& r, float tmin, float tmax, float& best,
                            int& best_prim, unsigned& nnode, unsigned& nprim, unsigned& nfall) {
  const int base = o.a, rows = o.b;
  if constexpr ((F & F_EXACT) != 0) {
    const V inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);  // the reference's reciprocals
    return bvh_exact<F>(S, base, rows, r, inv, tmin, tmax, best, best_prim, nnode, nprim, nfall);
  } else {
    // traversal reciprocals from v_rcp_f32 (see render_step_kernel's query setup)
    const V inv = mk(__builtin_amdgcn_rcpf(r.d.x), __builtin_amdgcn_rcpf(r.d.y), __builtin_amdgcn_rcpf(r.d.z));
    const int fb = o.c;  // traversal tree: 64-byte records at nodes[fb + 2i], root i = 0
    // Finite reciprocals for the traversal tree: with d = 0 the fma form would give inf - inf.
    // Clamped to +-1e30 the slab of a parallel axis is (-huge, +huge) inside and empty outside.
    const V finv = mk(__builtin_fminf(__builtin_fmaxf(inv.x, -1e30f), 1e30f),
                      __builtin_fminf(__builtin_fmaxf(inv.y, -1e30f), 1e30f),
                      __builtin_fminf(__builtin_fmaxf(inv.z, -1e30f), 1e30f));
    const V oi = mk(r.o.x * finv.x, r.o.y * finv.y, r.o.z * finv.z);
    const float a = len2(r.d), rcpa = __builtin_amdgcn_rcpf(a);
    float blo = __builtin_inff(), bhi = __builtin_inff(), second = __builtin_inff();
    best_prim = -1;
    int best_rank = 0x7fffffff;
    int sp = 0, cur = 0;
    bool overflow = false;
    for (;;) {
      RT_STEP_COUNT(0);
      if (!trav_step<F>(S, fb, r, oi, finv, a, rcpa, tmin, tmax, cur, sp, blo, bhi, second, best_prim, best_rank,
                        overflow, nnode, nprim))
        break;
    }
    RT_STAMP(5);
    best = blo;
    return bvh_settle<F>(S, base, rows, r, tmin, tmax, overflow, bhi, second, best, best_prim, best_rank, nnode, nprim,
                         nfall);
  }
}

// Closest hit of a PRIM / LIST / BVH object: (t, prim).  LIST keeps the reference list rule:
// shrinking t_max, later object wins ties (hittable_list.h:23-39).
template <int F>
__device__ __forceinline__ bool leaf_closest(const DScene& S, const rt_object& o, const Ray& r, float tmin, float tmax, float& t,
                             int& prim, unsigned& nnode, unsigned& nprim, unsigned& nfall) {
  if constexpr ((F & F_BVH) != 0)
    if (o.kind == RT_OBJ_BVH) return bvh_closest<F>(S, o, r, tmin, tmax, t, prim, nnode, nprim, nfall);
  if (o.kind == RT_OBJ_PRIM || (F & F_LIST) == 0) {
    prim = o.a;
    return prim_t<F>(S, o.a, r, tmin, tmax, t, nprim);
  }
  bool any = false;
  float closest = tmax;
  for (int k = 0; k < o.b; ++k) {
    float tt;
    if (prim_t<F>(S, o.a + k, r, tmin, closest, tt, nprim)) {
      any = true;
      closest = tt;
      t = tt;
      prim = o.a + k;
    }
  }
  return any;
}

__device__ __forceinline__ Ray xform_ray(const rt_object& o, const Ray& r, Ray& moved) {
  moved = r;
  if (o.b & 1) moved.o = r.o - mk(o.f[0], o.f[1], o.f[2]);
  Ray rr = moved;
  if (o.b & 2) {
    const float s = o.f[3], c = o.f[4];
    rr.o.x = c * moved.o.x - s * moved.o.z;
    rr.o.z = s * moved.o.x + c * moved.o.z;
    rr.d.x = c * moved.d.x - s * moved.d.z;
    rr.d.z = s * moved.d.x + c * moved.d.z;
  }
  return rr;
}

// constant_medium::hit over a (moving) sphere boundary after its first boundary query returned
// t1: sphere.h's second root is its first (H1), so the query from t1 + 1e-4 returns nothing or
// t1 itself (when t1 + 1e-4 rounds to t1), and with t2 = t1 the clamps to [tmin, tmax] leave
// t1 >= t2: the medium returns before its RNG draw either way.  A NaN root (degenerate ray) does
// not, and keeps the reference's path.  Stats variants run the query to count it.
template <int F>
__device__ __forceinline__ bool sphere_boundary_no_hit(const DScene& S, int boundary, float t1) {
  if constexpr ((F & F_STATS) != 0) return false;
  const rt_object bo = ro<F>(S.objects)[boundary];
  return bo.kind == RT_OBJ_PRIM && t1 == t1 && prim_type(load_prim<F>(S, bo.a)) <= RT_PRIM_MOVING_SPHERE;
}

// Both boundary queries of constant_medium::hit (constant_medium.h:38-44) for a box boundary,
// optionally under translate/rotate_y, in one pass over the six faces: a face's t and its
// in-rectangle test do not depend on the query interval, so they are computed once and box.h's
// list acceptance (tmin <= t <= shrinking t_max, later face wins) is replayed for each interval
// -- the same float operations on the same operands as the two box_t calls.  Returns 0: the
// first query missed, 1: the second missed, 2: t1 and t2 set.
template <int F>
__device__ __forceinline__ int box_boundary_t12(const DScene& S, const rt_object& bo, const PrimRec& q, const Ray& r, float& t1,
                                float& t2) {
  Ray moved;
  const Ray rr = bo.kind == RT_OBJ_XFORM ? xform_ray(bo, r, moved) : r;
  const V lo = mk(q.a.x, q.a.y, q.a.z), hi = mk(q.a.w, q.b.x, q.b.y);
  float tt[6];
  unsigned in = 0;
#pragma unroll
  for (int f = 0; f < 6; ++f) {
    float a0, a1, b0, b1, k;
    int ax, ia, ib;
    rect_axes(box_face(lo, hi, f, a0, a1, b0, b1, k), ax, ia, ib);
    tt[f] = (k - comp(rr.o, ax)) / comp(rr.d, ax);
    const float a = comp(rr.o, ia) + tt[f] * comp(rr.d, ia);
    const float b = comp(rr.o, ib) + tt[f] * comp(rr.d, ib);
    if (!(a < a0 || a > a1 || b < b0 || b > b1)) in |= 1u << f;
  }
  const float inf = __builtin_inff();
  float c = inf;
  bool h = false;
#pragma unroll
  for (int f = 0; f < 6; ++f)
    if (((in >> f) & 1u) && !(tt[f] < -inf || tt[f] > c)) {
      c = tt[f];
      h = true;
    }
  if (!h) return 0;
  t1 = c;
  const float m = t1 + 0.0001f;
  c = inf;
  h = false;
#pragma unroll
  for (int f = 0; f < 6; ++f)
    if (((in >> f) & 1u) && !(tt[f] < m || tt[f] > c)) {
      c = tt[f];
      h = true;
    }
  if (!h) return 1;
  t2 = c;
  return 2;
}

// constant_medium::hit after its boundary queries (constant_medium.h:45-70): clamps, then one RNG
// draw per qualifying query (H8).  prim = -1 marks a volume hit.
template <int F>
__device__ __forceinline__ bool medium_hit(const rt_object& o, const Ray& r, float tmin, float tmax, float t1, float t2,
                                           Rng& rng, float& t, int& prim) {
  if (t1 < tmin) t1 = tmin;
  if (t2 > tmax) t2 = tmax;
  if (t1 >= t2) return false;
  if (t1 < 0) t1 = 0;
  const float len = __builtin_sqrtf(len2(r.d));
  const float inside = (t2 - t1) * len;
  const float hd = o.f[0] * rtm::det_logf(rtx::uniform(rng));
  if (hd > inside) return false;
  t = t1 + hd / len;
  prim = -1;
  return true;
}

// hittable::hit of one top-level object, split in two: object_query finds the hit's t and its
// primitive (-1: a medium's volume hit) and makes the RNG draws; object_record builds the hit
// record from them.  world_hit builds only the winning entry's record: the reference copies every
// closer entry's record (hittable_list.h:23-39), but only the last copy survives and a record is
// a pure function of (object, primitive, ray, t), so the result is the same bit for bit.
// Every query of the object goes through ONE leaf query (one inlined copy of the BVH traversal
// per kernel): a constant medium's two boundary queries (constant_medium.h:38-44: over (-inf, inf),
// then from t1 + 1e-4; phases 0 and 1) and a plain object's own query (phase 2), each through an
// optional translate/rotate_y (hittable.h:37-59, 112-143).  Primitive boundaries (C3's boxes, C5's
// spheres) are answered before that, without a traversal.  The query chain is inlined: an
// out-of-line call made the kernel copy its whole argument block to scratch and reload the scene
// pointers from there on every use (C5: ~160 scratch loads in the kernel body).
template <int F>
__device__ __forceinline__ bool object_query(const DScene& S, int oi, const Ray& r, float tmin, float tmax, float& t,
                                             int& prim, Rng& rng, unsigned& nnode, unsigned& nprim, unsigned& nfall) {
  const float inf = __builtin_inff();
  const rt_object o = ro<F>(S.objects)[oi];
  int phase = 2, target = oi;
  float lo = tmin, hi = tmax, t1 = 0.0f;
  if constexpr ((F & F_MEDIUM) != 0) if (o.kind == RT_OBJ_MEDIUM) {
      if constexpr ((F & F_STATS) == 0) {  // stats variants run the reference's two queries to count them
        // an inert medium (o.c = 1 at upload: a bounded sphere boundary, H1) returns before its draw
        // for every sane ray: its boundary query cannot produce the NaN root that would reach it
        if (o.c == 1 && ray_sane(r)) return false;
        const rt_object bo = ro<F>(S.objects)[o.a];
        const bool prim_leaf = bo.kind == RT_OBJ_XFORM ? ro<F>(S.objects)[bo.a].kind == RT_OBJ_PRIM : bo.kind == RT_OBJ_PRIM;
        if (prim_leaf) {
          const int pi = bo.kind == RT_OBJ_XFORM ? ro<F>(S.objects)[bo.a].a : bo.a;
          const PrimRec q = load_prim<F>(S, pi);
          float b1, b2;
          if ((F & F_RECT) != 0 && prim_type(q) == RT_PRIM_BOX)
            return box_boundary_t12<F>(S, bo, q, r, b1, b2) == 2 && medium_hit<F>(o, r, tmin, tmax, b1, b2, rng, t, prim);
          if (bo.kind == RT_OBJ_PRIM) {
            unsigned np = 0;
            if (!prim_t_q<F>(S, q, r, -inf, inf, b1, np)) return false;
            if (prim_type(q) <= RT_PRIM_MOVING_SPHERE && b1 == b1) return false;  // sphere_boundary_no_hit
            return prim_t_q<F>(S, q, r, b1 + 0.0001f, inf, b2, np) && medium_hit<F>(o, r, tmin, tmax, b1, b2, rng, t, prim);
          }
        }
      }
      phase = 0;
      target = o.a;
      lo = -inf;
      hi = inf;
  }
  if constexpr ((F & F_BVH) == 0) {  // no traversal to share (C3): straight-line queries measured faster
    auto leaf_q = [&](int ti, float qlo, float qhi, float& tq, int& pq) {
      rt_object x = ro<F>(S.objects)[ti];
      Ray rr = r;
      if constexpr ((F & F_XFORM) != 0) if (x.kind == RT_OBJ_XFORM) {
          Ray moved;
          rr = xform_ray(x, r, moved);
          x = ro<F>(S.objects)[x.a];
      }
      return leaf_closest<F>(S, x, rr, qlo, qhi, tq, pq, nnode, nprim, nfall);
    };
    if (phase == 2) return leaf_q(oi, tmin, tmax, t, prim);
    float b1, b2;
    int pq;
    if (!leaf_q(o.a, -inf, inf, b1, pq)) return false;
    if (sphere_boundary_no_hit<F>(S, o.a, b1)) return false;
    if (!leaf_q(o.a, b1 + 0.0001f, inf, b2, pq)) return false;
    return medium_hit<F>(o, r, tmin, tmax, b1, b2, rng, t, prim);
  }
  for (;;) {
    rt_object x = ro<F>(S.objects)[target];
    Ray rr = r;
    if constexpr ((F & F_XFORM) != 0) if (x.kind == RT_OBJ_XFORM) {
        Ray moved;
        rr = xform_ray(x, r, moved);
        x = ro<F>(S.objects)[x.a];
    }
    float tq;
    int pq;
    const bool hit = leaf_closest<F>(S, x, rr, lo, hi, tq, pq, nnode, nprim, nfall);
    if (phase == 2) {
      t = tq;
      prim = pq;
      return hit;
    }
    if (!hit) return false;
    // the medium's record again (an opaque index: not kept live in VGPRs across the leaf query)
    int oi2 = oi;
    asm volatile("" : "+v"(oi2));
    const rt_object o2 = ro<F>(S.objects)[oi2];
    if (phase == 1) return medium_hit<F>(o2, r, tmin, tmax, t1, tq, rng, t, prim);
    t1 = tq;
    if (sphere_boundary_no_hit<F>(S, o2.a, t1)) return false;
    lo = t1 + 0.0001f;
    phase = 1;
  }
}

template <int F>
__device__ __forceinline__ void object_record(const DScene& S, int oi, int prim, const Ray& r, float tmin, float t, Hit& h) {
  const rt_object o = ro<F>(S.objects)[oi];
  if constexpr ((F & F_XFORM) != 0) if (o.kind == RT_OBJ_XFORM) {
      Ray moved;
      const Ray rr = xform_ray(o, r, moved);
      finalize<F>(S, prim, rr, tmin, t, h);
      if (o.b & 2) {
        const float s = o.f[3], cs = o.f[4];
        const V p = mk(cs * h.p.x + s * h.p.z, h.p.y, -s * h.p.x + cs * h.p.z);
        const V n = mk(cs * h.n.x + s * h.n.z, h.n.y, -s * h.n.x + cs * h.n.z);
        h.p = p;
        set_face(h, rr, n);  // rotated-frame ray against the world-frame normal (H25)
      }
      if (o.b & 1) {
        h.p = h.p + mk(o.f[0], o.f[1], o.f[2]);
        set_face(h, moved, h.n);
      }
      return;
  }
  if constexpr ((F & F_MEDIUM) != 0) if (o.kind == RT_OBJ_MEDIUM) {
      h.t = t;
      h.p = r.o + h.t * r.d;
      h.n = mk(1.0f, 0.0f, 0.0f);
      h.front = true;
      h.mat = o.b;
      h.u = 0.0f;  // stale in the reference; defined as 0
      h.v = 0.0f;
      return;
  }
  finalize<F>(S, prim, r, tmin, t, h);
}

// World = hittable_list of top-level objects (render.h:63 with t in [0.001, inf)).
// mask: bit w clear = no ray of this query's set can reach entry w (w < 32; camera-ray tile masks).
template <int F>
__device__ __forceinline__ bool world_hit(const DScene& S, const Ray& r, Hit& h, Rng& rng, unsigned& nnode, unsigned& nprim, unsigned& nfall,
                          uint32_t mask) {
  float closest = __builtin_inff();
  int wobj = -1, wprim = -1;
  for (int w = 0; w < S.n_world; ++w) {
    if (w < 32 && ((mask >> w) & 1u) == 0) continue;
    float t;
    int pr;
    const int oi = ro<F>(S.world)[w];
    if (object_query<F>(S, oi, r, 0.001f, closest, t, pr, rng, nnode, nprim, nfall)) {
      closest = t;
      wobj = oi;
      wprim = pr;
    }
  }
  if (wobj < 0) return false;
  object_record<F>(S, wobj, wprim, r, 0.001f, closest, h);
  return true;
}

// List world as ONE candidate search (S.merge_ok: entries are primitives, BVHs and instances of
// them, plus inert media; render_kernel's variants without counters).  The entries are visited in
// list order as world_hit does -- an instance's ray transformed once per entry, a BVH entry through
// its own traversal tree -- but their candidates go into one (winner, second) pair with list tie keys
// (take_candidate<true>, key = (n_world - 1 - w) << RT_WKEY_SHIFT | reference leaf rank: a later entry
// wins an exact tie, inside a BVH the lower rank), every traversal culls against the best candidate
// of all entries so far, and only the final winner gets its exact root and its reference-chain
// check, against a lower bound of the t_max the list passes to its entry (world_settle's argument).
// A sphere entry is a candidate range instead of an IEEE sqrt and divide.  Returns 0: certain miss,
// 1: certain hit (best, wobj, prim), 2: not certain (the caller runs the exact sequential list).
template <int F>
__device__ __forceinline__ int world_search(const DScene& S, const Ray& r, uint32_t mask, float& best, int& wobj,
                                            int& prim, unsigned& nnode, unsigned& nprim) {
  const float tmin = 0.001f, inf = __builtin_inff();
  float blo = inf, bhi = inf, second = inf;
  int best_prim = -1, best_key = 0x7fffffff;
  bool overflow = false;
  const int NW = S.n_world;
  for (int k = 0; k < NW; ++k) {
    const int w = ro<0>(S.worder)[k];  // the visiting order does not change the winner (tie keys carry w)
    if (w < 32 && ((mask >> w) & 1u) == 0) continue;
    const rt_object o = ro<0>(S.objects)[ro<0>(S.world)[w]];
    if ((F & F_MEDIUM) != 0 && o.kind == RT_OBJ_MEDIUM) continue;  // inert (merge_ok), the ray is sane
    Ray rr = r;
    int xi = ro<0>(S.world)[w];
    if constexpr ((F & F_XFORM) != 0) if (o.kind == RT_OBJ_XFORM) {
      Ray moved;
      rr = xform_ray(o, r, moved);
      xi = o.a;
    }
    const rt_object x = ro<0>(S.objects)[xi];
    const int kbase = (NW - 1 - w) << RT_WKEY_SHIFT;
    const float a = len2(rr.d), rcpa = __builtin_amdgcn_rcpf(a);
    if ((F & F_BVH) != 0 && x.kind == RT_OBJ_BVH) {
      const V inv = mk(__builtin_amdgcn_rcpf(rr.d.x), __builtin_amdgcn_rcpf(rr.d.y), __builtin_amdgcn_rcpf(rr.d.z));
      const V finv = mk(__builtin_fminf(__builtin_fmaxf(inv.x, -1e30f), 1e30f),
                        __builtin_fminf(__builtin_fmaxf(inv.y, -1e30f), 1e30f),
                        __builtin_fminf(__builtin_fmaxf(inv.z, -1e30f), 1e30f));
      const V oi = mk(rr.o.x * finv.x, rr.o.y * finv.y, rr.o.z * finv.z);
      int sp = 0, cur = 0;
      for (;;) {
        if (!trav_step<F, true>(S, x.c, rr, oi, finv, a, rcpa, tmin, inf, cur, sp, blo, bhi, second, best_prim, best_key,
                                overflow, nnode, nprim, kbase))
          break;
      }
    } else {
      const PrimRec q = load_prim_u<F>(S, x.a);
      float lo, hi;
      if (prim_range<F>(S, q, rr, a, rcpa, tmin, inf, lo, hi, nprim))
        take_candidate<true>(lo, hi, x.a, kbase, blo, bhi, second, best_prim, best_key);
    }
  }
  if (overflow || (best_prim >= 0 && !(second > bhi))) return 2;
  if (best_prim < 0) return 0;
  wobj = ro<F>(S.world)[NW - 1 - (best_key >> RT_WKEY_SHIFT)];
  prim = best_prim;
  const rt_object o = ro<F>(S.objects)[wobj];
  Ray rr = r;
  int xi = wobj;
  if constexpr ((F & F_XFORM) != 0) if (o.kind == RT_OBJ_XFORM) {
    Ray moved;
    rr = xform_ray(o, r, moved);
    xi = o.a;
  }
  best = blo;
  if (blo != bhi) {  // a range: the exact root once
    unsigned np = 0;
    if (!prim_t<F>(S, best_prim, rr, tmin, inf, best, np)) return 2;
  }
  if constexpr ((F & F_BVH) != 0) {
    const rt_object x = ro<F>(S.objects)[xi];
    if (x.kind == RT_OBJ_BVH) {
      const float lim = __builtin_fminf(second, bhi * 1.0009765625f);
      if (!chain_ok<F>(S, x.a, x.b, rr, tmin, lim, best, best_prim, best_key & ((1 << RT_WKEY_SHIFT) - 1), nnode))
        return 2;
    }
  }
  return 1;
}

// render_kernel's world query on merge_ok lists: world_search, and when it is not certain the
// reference's list loop exactly (render_step_kernel's world branch: exact BVH visit sets, exact
// primitive roots, the media's own queries).
template <int F>
__device__ __forceinline__ bool world_query_merged(const DScene& S, const Ray& r, Hit& h, Rng& rng, unsigned& nnode,
                                                   unsigned& nprim, unsigned& nfall, uint32_t mask) {
  float best = 0.0f;
  int wobj = -1, wprim = -1;
  int st = ray_sane(r) ? world_search<F>(S, r, mask, best, wobj, wprim, nnode, nprim) : 2;
  if (S.merge_ok > 1) st = 2;  // RT_MERGE_FALLBACK (tests): every query through the exact list
  if (st == 0) return false;
  if (st == 2) {  // every entry in list order, exactly (render_step_kernel's world branch)
    constexpr int FM = F & ~F_BVH;  // media boundaries are primitives
    const float tmin = 0.001f;
    bool hit = false;
    for (int w = 0; w < S.n_world; ++w) {
      if (w < 32 && ((mask >> w) & 1u) == 0) continue;
      const int oi = ro<F>(S.world)[w];
      const rt_object o = ro<F>(S.objects)[oi];
      const float tcl = hit ? best : __builtin_inff();
      float tq;
      int pq;
      bool hq;
      if ((F & F_MEDIUM) != 0 && o.kind == RT_OBJ_MEDIUM) {
        hq = object_query<FM>(S, oi, r, tmin, tcl, tq, pq, rng, nnode, nprim, nfall);
      } else {
        Ray rr = r;
        int xi = oi;
        if constexpr ((F & F_XFORM) != 0) if (o.kind == RT_OBJ_XFORM) {
          Ray moved;
          rr = xform_ray(o, r, moved);
          xi = o.a;
        }
        const rt_object x = ro<F>(S.objects)[xi];
        if ((F & F_BVH) != 0 && x.kind == RT_OBJ_BVH) {
          hq = bvh_exact<F>(S, x.a, x.b, rr, mk(1.0f / rr.d.x, 1.0f / rr.d.y, 1.0f / rr.d.z), tmin, tcl, tq, pq, nnode,
                            nprim, nfall);
        } else {
          pq = x.a;
          hq = prim_t<F>(S, x.a, rr, tmin, tcl, tq, nprim);
        }
      }
      if (hq) {
        hit = true;
        best = tq;
        wobj = oi;
        wprim = pq;
      }
    }
    if (!hit) return false;
  }
  object_record<F>(S, wobj, wprim, r, 0.001f, best, h);
  return true;
}

// ------------------------------------------------------------------ textures (texture.h, perlin.h)
__device__ float perlin_noise(const rt_perlin& P, V p) {
  const float u = p.x - __builtin_floorf(p.x), v = p.y - __builtin_floorf(p.y), w = p.z - __builtin_floorf(p.z);
  const int i = (int)__builtin_floorf(p.x), j = (int)__builtin_floorf(p.y), k = (int)__builtin_floorf(p.z);
  const float uu = u * u * (3.0f - 2.0f * u);
  const float vv = v * v * (3.0f - 2.0f * v);
  const float ww = w * w * (3.0f - 2.0f * w);
  float acc = 0.0f;
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int c = 0; c < 2; ++c) {
        const int idx = P.perm_x[(i + a) & 255] ^ P.perm_y[(j + b) & 255] ^ P.perm_z[(k + c) & 255];
        const V g = ld3(P.ranvec[idx]);
        const V wv = mk(u - (float)a, v - (float)b, w - (float)c);
        acc += ((float)a * uu + (float)(1 - a) * (1.0f - uu)) * ((float)b * vv + (float)(1 - b) * (1.0f - vv)) *
               ((float)c * ww + (float)(1 - c) * (1.0f - ww)) * dot(g, wv);
      }
  return acc;
}
__device__ float perlin_turb(const rt_perlin& P, V p, int depth) {
  double acc = 0.0, w = 1.0;
  for (int i = 0; i < depth; ++i) {
    acc += w * (double)perlin_noise(P, p);
    w *= 0.5;
    p = 2.0f * p;
  }
  return (float)__builtin_fabs(acc);
}
template <int F>
__device__ __forceinline__ V tex_leaf(const DScene& S, const rt_texture& T, float u, float v, V p) {
  if constexpr ((F & F_NOISE) != 0) {
    if (T.type == RT_TEX_NOISE) {
      const float n = perlin_noise(S.perlins[T.a], T.scale * p);
      return (float)(1.0 + (double)n) * (0.5f * mk(1.0f, 1.0f, 1.0f));
    }
    if (T.type == RT_TEX_TURBULENT) return perlin_turb(S.perlins[T.a], T.scale * p, T.b) * mk(1.0f, 1.0f, 1.0f);
    if (T.type == RT_TEX_MARBLE) {
      const float tb = perlin_turb(S.perlins[T.a], T.scale * p, 7);
      const float s = 1.0f + rtm::det_sinf(T.scale * p.z + 10.0f * tb);
      return s * (0.5f * mk(1.0f, 1.0f, 1.0f));
    }
  }
  if constexpr ((F & F_IMAGE) != 0) {
    if (T.type == RT_TEX_IMAGE) {  // texture.h:145-163
      const rt_image im = imgs_of<F>(S)[T.a];
      if (im.width <= 0) return mk(0.0f, 1.0f, 1.0f);
      const float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);
      const float vc = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
      const double vv = 1.0 - (double)vc;
      int i = (int)(uu * (float)im.width);
      int j = (int)(vv * (double)im.height);
      if (i >= im.width) i = im.width - 1;
      if (j >= im.height) j = im.height - 1;
      // texel (i, j) in the tiled copy rt_scene_upload made: 8x8-texel tiles, row-major
      const unsigned t = ((unsigned)((j >> 3) * ((im.width + 7) >> 3) + (i >> 3)) << 6) + ((j & 7) << 3) + (i & 7);
      const uint8_t* px = S.texels + im.offset + (size_t)t * im.bytes_per_pixel;
      const float cs = 1.0f / 255.0f;
      return mk(cs * (float)px[0], cs * (float)px[1], cs * (float)px[2]);
    }
  }
  return ld3(T.color);  // solid
}
template <int F>
__device__ __forceinline__ V tex_value(const DScene& S, int ti, float u, float v, V p) {
  const rt_texture T = texs_of<F>(S)[ti];
  if constexpr ((F & F_CHECKER) != 0) {
    if (T.type == RT_TEX_CHECKER) {  // texture.h:37-45: sin(10x) sin(10y) sin(10z) < 0 -> odd
      return tex_leaf<F>(S, texs_of<F>(S)[rtm::checker_odd(10.0f * p.x, 10.0f * p.y, 10.0f * p.z) ? T.b : T.a], u, v, p);
    }
  }
  return tex_leaf<F>(S, T, u, v, p);
}

// ------------------------------------------------------------------ materials (material.h)
// Returns true when the path continues: att set and the scattered ray written over `ray` in place
// (origin h.p, time kept).  em = emitted colour.  The in-place write matters: with the query chain
// inlined, a conditional whole-struct copy of a separately built scattered ray (`ray = sc` under
// `if (scatter(...))`) was compiled into per-component selects of which some kept the incoming
// ray's values (widest variants, isotropic scatter: origin x/z and direction x of the old ray;
// found with scripts/diag_trace.py on cornell_smoke).
template <int F>
__device__ __forceinline__ bool scatter(const DScene& S, Ray& ray, const Hit& h, V& att, V& em, Rng& rng) {
  const int4 m = mats_of<F>(S)[h.mat];
  const int mt = m.x;
  em = mk(0.0f, 0.0f, 0.0f);
  // lambertian, metal and isotropic each draw exactly one random_in_unit_sphere and nothing else
  // (material.h:26,52,135): one shared rejection loop keeps every lane's draw order and lets
  // the wave run a single loop instead of one per material.
  V sp = mk(0.0f, 0.0f, 0.0f);
  if (mt == RT_MAT_LAMBERTIAN || mt == RT_MAT_METAL || mt == RT_MAT_ISOTROPIC) sp = in_unit_sphere(rng);
  if (mt == RT_MAT_DIFFUSE_LIGHT) {  // material.h:115-121
    em = tex_value<F>(S, m.y, h.u, h.v, h.p);
    return false;
  }
  // The materials differ only in the scattered direction (and attenuation): one direction chosen
  // per lane, then one write of the ray.
  V dir = sp;  // isotropic, material.h:133-137
  bool cont = true;
  if (mt == RT_MAT_DIELECTRIC) {  // material.h:64-104
    att = mk(1.0f, 1.0f, 1.0f);
    const float ir = __int_as_float(m.z);
    const float ratio = h.front ? (1.0f / ir) : ir;
    const V ud = unit(ray.d);
    const float c = __builtin_fminf(dot(neg(ud), h.n), 1.0f);
    const float sn = __builtin_sqrtf(1.0f - c * c);
    bool refl = ratio * sn > 1.0f;
    if (!refl) {
      const float sr = (1.0f - ratio) / (1.0f + ratio);
      const float r0 = sr * sr;
      const float rf = r0 + (1.0f - r0) * rtm::det_pow5f(1.0f - c);
      refl = rf > rtx::uniform(rng);
    }
    if (refl) {
      dir = ud - (2.0f * dot(ud, h.n)) * h.n;
    } else {  // vec3.h:152-158
      const float ct = __builtin_fminf(dot(neg(ud), h.n), 1.0f);
      const V perp = ratio * (ud + ct * h.n);
      const V par = (-__builtin_sqrtf(__builtin_fabsf(1.0f - len2(perp)))) * h.n;
      dir = perp + par;
    }
  } else {
    att = tex_value<F>(S, m.y, h.u, h.v, h.p);  // albedo
    if (mt == RT_MAT_LAMBERTIAN) {  // material.h:25-35
      dir = h.n + unit(sp);
      const float e = 1e-6f;
      if (__builtin_fabsf(dir.x) < e && __builtin_fabsf(dir.y) < e && __builtin_fabsf(dir.z) < e) dir = h.n;
    } else if (mt == RT_MAT_METAL) {  // material.h:50-55
      const V ud = unit(ray.d);
      dir = (ud - (2.0f * dot(ud, h.n)) * h.n) + __int_as_float(m.z) * sp;
      cont = dot(dir, h.n) > 0;
    }
  }
  ray.o = h.p;
  ray.d = dir;
  return cont;
}

// ------------------------------------------------------------------ kernels
struct RenderParams {
  DScene S;
  const uint4* states;  // 2 uint4 per slot: d v0 v1 v2 | v3 v4 - -
  float* fb;
  const int2* row_q;          // processing position q -> {owned row r (output layout order), image
                              // row j}: rows costliest first (one load at an item's start)
  unsigned long long* row_cost;  // per image row: segments of the finished items with i % 16 == 0
  unsigned long long* work;
  unsigned long long* counters;  // segments, node, prim, samples
  unsigned long long total_items;
  long long npix;  // W*H of the full image
  int W, H, rows, spp, fb_first, max_depth, cam_mode, fb_count;
  int shade_min;  // render_step_kernel: lanes waiting before a wave runs its shading phase
  int pstep;      // item grid step (1; a probe launch's grid of every pstep-th row position and pixel)
  long long per_row;  // items per row position: fb_count * W (a probe launch: its grid's width)
  // Item schedule (see rt_render): perm maps the claimed position to the item (null: identity);
  // positions below n_long hold the longest items of the previous launch, longest first, and the
  // waves holding one run at raised priority.  item_cost (measuring launch) receives each item's
  // segment count.
  const uint32_t* perm;
  uint16_t* item_cost;
  unsigned long long n_long;
  uint32_t cam_state[6];  // pristine slot-0 state curand_init(seed, 0, 0): REF camera draws of render_step_kernel
  // Split samples (render_step_kernel, warm launches of a small share; see rt_render): the first
  // n_split positions of perm are the longest items.  split_mode 1: those items record their RNG
  // state at every sample start into ckpt[pos * spp + s]; split_mode 2: their samples are separate
  // work items (claim k < n_split * spp: position k / spp, sample k % spp) that start from ckpt
  // (sample 0: from states) and write the sample's sum to contrib[3 k]; merge_split_kernel adds
  // them up in sample order.  cam_st[s]: the REF camera state at sample s's start.  order (split_mode
  // 2, may be null): claim k takes order[k] instead of k -- split samples and the other items in
  // one longest-first sequence by the recording launch's per-sample segment counts (split_mode 1
  // keeps them in ckpt's spare word: segments before sample s at [pos * spp + s], the item's
  // total at [pos * spp]).
  int split_mode;
  int pad5;
  unsigned long long n_split;
  uint4* ckpt;
  float* contrib;
  const uint4* cam_st;
  const uint32_t* order;
  // Camera-ray candidate lists (render_step_kernel; null: camera rays traverse the tree): per 8x8
  // tile of the image, tile_cnt[t] (id, nearest) pairs at tile_ent[2 * t * tile_cap] (-1: the tile
  // overflowed).
  const int32_t* tile_cnt;
  const int32_t* tile_ent;
  int tiles_x, tile_cap;
  // Camera-ray entry masks (render_kernel, list worlds; null: every entry is tested): bit w of
  // tile_mask[t] = a camera ray of tile t may hit top-level entry w.
  const uint32_t* tile_mask;
};

constexpr int kBlock = 256;
constexpr int kAuditCap = 4096;
constexpr int kTileShift = 3;  // camera-ray candidate lists per 8x8-pixel tile
constexpr int kTileCap = 32;   // entries per tile list (a fuller tile traverses the tree)
// render_kernel refills a wave once this many lanes are idle (same box, Mrays/s at 16 / 8 / 4 / 2 / 1:
// C3 18 854 / 20 165 / 20 590 / 20 571 / 20 645, C5 3 749 / 3 829 / 3 828 / 3 813 / 3 745)
constexpr int kRefill = 4;
// render_step_kernel refills a wave once this many lanes are idle (or none is busy): at every idle
// lane for the sphere variants (C2 at 4 / 8: 14 930 -> 14 796 / 14 498 Mrays/s), at 4 for the mesh
// variants, whose refill (state, row and tile-list loads from global memory behind the traversal's
// own global loads) stalls the whole wave (C4 at 1 / 2 / 3 / 4 / 6: 18 144 / 18 513 / 18 697 /
// 18 741 / 18 659 Mrays/s; profiles/r05/refill_ab.txt)
template <int F>
constexpr int step_refill() { return (F & F_TRI) != 0 ? 4 : 1; }
constexpr int kShadeMin = 60;  // render_step_kernel: default shading-phase threshold
constexpr int kShadeMinMesh = 48;  // ... for triangle-mesh variants (round 5, with step_refill 4: C4 at
                                   // 36 / 40 / 44 / 48 / 52 / 56 / 60: 18 845 / 18 971 / 19 048 / 19 079 /
                                   // 19 021 / 18 750 / 17 986 Mrays/s; profiles/r05/shade_ab.txt)
constexpr int kShadePasses = 2;    // render_step_kernel: shading passes per phase (1: C2 17.2 -> 20.4 ms, 3: +0.7 %)
constexpr unsigned kChunk = 64;  // items a wave claims per work-counter atomic
static_assert(kChunk >= 64, "claim_items: one claim must cover a refill of every lane of a wave");

// Camera ray of sample s of pixel (i, j) for render_kernel (render.h:105-108, camera.h:49-58).
// In the REF camera mode every pixel restarts a private copy of the pristine slot-0 state (H2), so
// the lens offset and time of sample s are the same for all pixels: they come from cam_tab, built
// on the host with the same float operations (camera_table): no camera RNG state per lane, no
// rejection loop (C3-C5 2 % faster).  PER_PIXEL draws them from the pixel's own state, after the
// jitter (render.h:105-108 order).
__device__ __forceinline__ void camera_ray(const RenderParams& P, const rt_camera& C, int i, int j, int s,
                                           bool per_pixel, Rng& loc, Ray& ray) {
  const float u = ((float)i + rtx::uniform(loc)) / (float)P.W;
  const float v = ((float)j + rtx::uniform(loc)) / (float)P.H;
  V off;
  float tm;
  if (per_pixel) {
    const V rd = C.lens_radius * in_unit_disk(loc);
    off = rd.x * ld3(C.u) + rd.y * ld3(C.v);
    tm = urange(loc, C.time0, C.time1);
  } else {
    const float4 e = P.S.cam_tab[s];
    off = mk(e.x, e.y, e.z);
    tm = e.w;
  }
  ray.o = ld3(C.origin) + off;
  ray.d = ld3(C.lower_left) + u * ld3(C.horizontal) + v * ld3(C.vertical) - ld3(C.origin) - off;
  ray.tm = tm;
}

__device__ __forceinline__ unsigned lane_rank(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

// Work items for the lanes in `idle` (lane order) from the wave's chunk [chunk_base, +chunk_left)
// of the global work counter; a chunk of kChunk items is claimed with ONE atomic when the current
// one runs short (all waves of the grid hit one counter: its atomics serialise in L2).
__device__ __forceinline__ unsigned long long claim_items(unsigned long long* work, unsigned long long idle,
                                                          unsigned long long& chunk_base, unsigned& chunk_left) {
  const unsigned nidle = (unsigned)__popcll(idle);
  const unsigned long long old_base = chunk_base;
  const unsigned old_left = chunk_left;
  unsigned long long fresh = 0;
  if (old_left < nidle) {
    const int leader = __ffsll((long long)idle) - 1;
    if ((int)__lane_id() == leader) fresh = atomicAdd(work, (unsigned long long)kChunk);
    fresh = __shfl(fresh, leader, 64);
    chunk_base = fresh + (nidle - old_left);
    chunk_left = kChunk - (nidle - old_left);
  } else {
    chunk_base = old_base + nidle;
    chunk_left = old_left - nidle;
  }
  const unsigned rk = lane_rank(idle);
  return rk < old_left ? old_base + rk : fresh + (rk - old_left);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

// Minimum waves per SIMD the compiler must fit (VGPR budget 512 / waves) for the variants that
// traverse from global memory, where latency hiding is the limiter: measured on MI355X (C3
// 800x800 10x100: F_CORNELL at 135 VGPRs / 3 waves 33.2 ms, capped at 128 / 4 waves 28.6 ms; C5
// 1280x720 8x8: F_ALL at 201 VGPRs / 2 waves 81.4 ms, at 168 / 3 waves 69.1 ms, at 128 / 4 waves
// with spills 73.2 ms; F_FINAL (no checker code) at 4 waves 66.7 ms, at 3 waves 69.5 ms; C4 door:
// F_MESH best uncapped, 166 VGPRs / 3 waves, at 4 after the deferred hit record; F_CORNELL at 5 with its
// list entries in SGPRs: 4 / 5 / 6 waves 24 470 / 26 890 / 25 290 Mrays/s).  LDS variants run
// 1024-thread workgroups, which already cap them at 128.
template <int F>
constexpr int render_wpe() {
  constexpr int feat = F & F_ALL;
  return (F & F_LDS) != 0 ? 1
                          : (feat == F_FINAL || feat == F_MESH ? 4 : (feat == F_CORNELL ? 5 : (feat == F_ALL ? 3 : 1)));
}
// The kernel arguments through an opaque pointer to the kernarg segment, once per loop trip: their
// fields are then re-read (scalar loads) in every trip instead of held in SGPRs across the whole loop.
// Only in the list variants without BVHs or triangles (C3's): their SGPR spills 64 -> 0 and VGPR spills
// 16 -> 8, 1.8-2.7 % faster (same box, profiles/r06/launder_ab.txt); the other variants measured slower
// with it (C2's stepwise 6.5 %, C4 1.4 %, C5 0.5 %: the reloads sit in their dependent chains).
template <int F>
constexpr bool launders() { return (F & (F_BVH | F_TRI)) == 0; }
template <int F>
__device__ __forceinline__ const RenderParams& loop_params(const RenderParams& P0) {
  if constexpr (launders<F>()) {
    const RT_RO RenderParams* p = (const RT_RO RenderParams*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const RenderParams*)p;
  } else {
    return P0;
  }
}
template <int F>
__global__ __launch_bounds__(render_block<F>()) __attribute__((amdgpu_waves_per_eu(render_wpe<F>())))
void render_kernel(const RenderParams P) {
  const DScene& S = P.S;
  if constexpr ((F & F_LDS) != 0) stage_lds<F>(S);  // nodes, primitives, margins, materials, textures
  if constexpr (tables_after_locker<F>()) {  // materials, textures and images after the locker
    static_assert(render_block<F>() == 256, "locker_tables_at assumes 256-thread blocks");
    float4* m = rt_lds + locker_tables_at<F>();
    const int nm = S.lds_mats, nt = 2 * S.lds_texs, ni = S.lds_imgs;
    for (int k = threadIdx.x; k < nm + nt + ni; k += 256)
      m[k] = k < nm ? ((const float4*)S.mats)[k]
                    : (k < nm + nt ? ((const float4*)S.texs)[k - nm] : ((const float4*)S.images)[k - nm - nt]);
    __syncthreads();
  }
  const unsigned lane = __lane_id();
  RT_STEP_COUNT_BEGIN();
  RT_STAMP_BEGIN();
  long long item = -1;  // -1: idle
  bool done = false;
  // cold state in the LDS locker (parks<F>): 0..2 sample sum, 3 fb, 4 owned row, 5 column,
  // 6 image row, 7 sample, 8 depth, 9 item segments, 10/11 segment / sample counts, 12..14
  // attenuation -- touched once per segment or sample, so none of it is live in VGPRs across
  // the world query (where the widest variants otherwise spill to scratch)
  uint32_t* const lk = locker_of<F>();
  constexpr int LB = render_block<F>();
  constexpr bool PK = parks_segment_mask(F);
  int f = 0, r = 0;
  int i_r = 0, j_r = 0, s_r = 0, depth_r = 0;
  unsigned item_segs_r = 0, nseg_r = 0, nsamp_r = 0;
  int& i = cold_ref<PK>(i_r, lk + 5 * LB);
  int& j = cold_ref<PK>(j_r, lk + 6 * LB);
  int& s = cold_ref<PK>(s_r, lk + 7 * LB);
  int& depth = cold_ref<PK>(depth_r, lk + 8 * LB);
  unsigned& item_segs = cold_ref<PK>(item_segs_r, lk + 9 * LB);
  unsigned& nseg = cold_ref<PK>(nseg_r, lk + 10 * LB);
  unsigned& nsamp = cold_ref<PK>(nsamp_r, lk + 11 * LB);
  // split samples (see render_step_kernel; the parking variants only -- C5's, whose shares run on 8
  // GPUs; C3's variant measured 2.6 % slower with the code and is a one-GPU config): the item ends
  // after sample s_end - 1; ck = the split claim
  constexpr bool SPL = PK;
  int s_end_r = 0, ck_r = -1;
  int& s_end = cold_ref<PK>(s_end_r, lk + 21 * LB);
  int& ck = cold_ref<PK>(ck_r, lk + 22 * LB);
  if constexpr (PK) {
    nseg = 0;
    nsamp = 0;
  }
  float* const lkf = reinterpret_cast<float*>(lk);
  V att_r = mk(1, 1, 1);
  auto att_get = [&]() -> V {
    if constexpr (PK) return mk(lkf[12 * LB], lkf[13 * LB], lkf[14 * LB]);
    else return att_r;
  };
  auto att_set = [&](V a) {
    if constexpr (PK) {
      lkf[12 * LB] = a.x;
      lkf[13 * LB] = a.y;
      lkf[14 * LB] = a.z;
    } else {
      att_r = a;
    }
  };
  // the RNG state: parked too; the world query (media draws) uses it in place, the camera ray and
  // scatter on a register copy
  Rng loc_r{};
  Rng& loc = cold_ref<PK>(loc_r, (uint32_t*)rt_lds + LB * (stack_words(F) + 15) + 6 * threadIdx.x);
  Ray ray{};
  V col = mk(0, 0, 0);
  unsigned nnode = 0, nprim = 0, nfall = 0;
  const bool per_pixel = P.cam_mode == RT_CAM_PER_PIXEL;
  const rt_camera& C = S.cam;
  unsigned long long chunk_base = 0;  // wave-uniform: next unclaimed item of the wave's chunk
  unsigned chunk_left = 0;

  const RenderParams& P0 = P;
  for (;;) {
    // the kernel arguments re-read every loop trip in the variants that launder them (loop_params)
    const RenderParams& P = loop_params<F>(P0);
    const DScene& S = P.S;
    const rt_camera& C = S.cam;
    // ---- refill idle lanes (one atomic per wave, ballot-compacted ranks)
    RT_STAMP(7);  // back-to-back pair: phase 7 = the cost of one stamp per loop trip
    RT_STAMP(0);
    const unsigned long long idle = __ballot(item < 0 && !done);
    const unsigned long long busy = __ballot(item >= 0);
    const int nidle = __popcll(idle);
    if (nidle > 0 && (nidle >= kRefill || busy == 0)) {
      const unsigned long long mine = claim_items(P.work, idle, chunk_base, chunk_left);
      if (item < 0 && !done) {
        if (mine >= P.total_items) {
          done = true;
        } else {
          unsigned long long pos = mine;
          int sa = 0;
          if constexpr (SPL) ck = -1;
          if (SPL && P.split_mode == 2) {  // split samples and the other items, claimed in one sequence
            const unsigned long long nsub = P.n_split * (unsigned long long)P.spp;
            const unsigned long long v = P.order ? (unsigned long long)P.order[mine] : mine;
            if (v < nsub) {
              pos = v / (unsigned)P.spp;
              sa = (int)(v - pos * (unsigned)P.spp);
              ck = (int)v;
            } else {
              pos = v - nsub + P.n_split;
            }
          } else if (SPL && P.split_mode == 1 && mine < P.n_split) {
            ck = (int)mine;
          }
          item = P.perm ? (long long)P.perm[pos] : (long long)pos;
          // Row-major, fb inside the row, rows in row_q order: the costliest rows of the previous
          // launch of this configuration first (else bottom to top), so a launch does not end
          // with a long item started late (a lane runs an item's samples serially).
          // (probe launches: items on a grid of every pstep-th row position and pixel, per_row = the
          // grid's width; otherwise pstep = 1, per_row = fb_count * W)
          const long long per_row = P.per_row;
          const int qi = (int)(item / per_row);
          const long long rem = item - (long long)qi * per_row;
          const int2 rj = P.row_q[qi * P.pstep];
          r = rj.x;
          f = (int)(rem / P.W);
          i = (int)(rem - (long long)f * P.W) * P.pstep;
          j = rj.y;
          const long long id = P.fb_first + f;
          const long long p = (long long)j * P.W + i;
          const long long slot = ((id + 1) * p + id + 1) % P.npix;  // render.h:101 (H3)
          const uint4* st = sa > 0 ? P.ckpt + 2 * (long long)ck : P.states + 2 * slot;
          const uint4 s0 = st[0], s1 = st[1];
          loc.d = s0.x; loc.v[0] = s0.y; loc.v[1] = s0.z; loc.v[2] = s0.w; loc.v[3] = s1.x; loc.v[4] = s1.y;
          s = sa;
          if constexpr (SPL) s_end = (P.split_mode == 2 && ck >= 0) ? sa + 1 : P.spp;
          depth = 0;
          item_segs = 0;
          if constexpr (parks<F>()) {
            lk[0 * LB] = 0u;
            lk[1 * LB] = 0u;
            lk[2 * LB] = 0u;
            lk[3 * LB] = (uint32_t)f;
            lk[4 * LB] = (uint32_t)r;
          } else {
            col = mk(0, 0, 0);
          }
        }
      }
    }
    if (__ballot(item >= 0) == 0) break;
    if (item >= 0) {  // idle lanes wait at the loop head (no divergent continue)
      // ---- begin a sample: jitter + camera ray (render.h:105-108, camera.h:49-58)
      if (depth == 0) {
        RT_STAMP(1);
        if (SPL && P.split_mode == 1 && ck >= 0 && s > 0) {  // record the sample-start state for split launches
          uint4* dst = P.ckpt + 2 * ((long long)ck * P.spp + s);
          dst[0] = make_uint4(loc.d, loc.v[0], loc.v[1], loc.v[2]);
          dst[1] = make_uint4(loc.v[3], loc.v[4], item_segs, 0u);
        }
        {
          Rng lr = loc;
          camera_ray(P, C, i, j, s, per_pixel, lr, ray);
          loc = lr;
        }
        att_set(mk(1.0f, 1.0f, 1.0f));
      }

      // ---- one segment (render.h:60-77)
      ++nseg;
      ++item_segs;
      Hit h;
      bool ended = false;
      V contrib;
      RT_STAMP(2);
      RT_STEP_COUNT(2);
      const uint32_t wmask = (depth == 0 && P.tile_mask) ? P.tile_mask[(j >> kTileShift) * P.tiles_x + (i >> kTileShift)]
                                                         : 0xffffffffu;
      // The merged candidate search on scenes rt_scene_upload marks merge_ok: only it in the F_MERGE
      // variants (C5: F_FINAL's entry loop costs 11 more spilled VGPRs), decided per scene in the
      // widest counter-free ones.
      constexpr bool kOnly = (F & F_MERGE) != 0;
      constexpr bool kDyn = !kOnly && (F & F_ALL) == F_ALL && (F & (F_STATS | F_EXACT | F_CHECK)) == 0;
      bool hit_any;
      if (kOnly || (kDyn && S.merge_ok))
        hit_any = world_query_merged<((kOnly || kDyn) ? F : 0)>(S, ray, h, loc, nnode, nprim, nfall, wmask);
      else
        hit_any = world_hit<F>(S, ray, h, loc, nnode, nprim, nfall, wmask);
      RT_STAMP(6);
      if (!hit_any) {
        contrib = att_get() * ld3(S.bg);
        ended = true;
      } else {
        V a, em;
        Rng lr = loc;
        const bool sc_ok = scatter<F>(S, ray, h, a, em, lr);
        loc = lr;
        if (sc_ok) {
          att_set(att_get() * a);
          if (++depth == P.max_depth) {
            contrib = mk(0.0f, 0.0f, 0.0f);
            ended = true;
          }
        } else {
          contrib = att_get() * em;
          ended = true;
        }
      }
      if (ended) {
        if constexpr (parks<F>()) col = mk(__uint_as_float(lk[0 * LB]), __uint_as_float(lk[1 * LB]), __uint_as_float(lk[2 * LB]));
        col = col + contrib;
        if constexpr (parks<F>()) {
          lk[0 * LB] = __float_as_uint(col.x);
          lk[1 * LB] = __float_as_uint(col.y);
          lk[2 * LB] = __float_as_uint(col.z);
        }
        depth = 0;
        ++nsamp;
        if (++s == (SPL ? s_end : P.spp)) {
          if (SPL && P.split_mode == 2 && ck >= 0) {  // one sample of a split item: its sum, merged later
            float* dst = P.contrib + 3 * (long long)ck;
            dst[0] = col.x;
            dst[1] = col.y;
            dst[2] = col.z;
          } else {
            const V out = (1.0f / (float)P.spp) * col;
            if constexpr (parks<F>()) {
              f = (int)lk[3 * LB];
              r = (int)lk[4 * LB];
            }
            float* dst = P.fb + 3 * (((long long)f * P.rows + r) * P.W + i);
            dst[0] = out.x;
            dst[1] = out.y;
            dst[2] = out.z;
          }
          if (SPL && P.split_mode == 1 && ck >= 0) P.ckpt[2 * (long long)ck * P.spp + 1] = make_uint4(0u, 0u, item_segs, 0u);
          if (P.row_cost && (i & 15) == 0) atomicAdd(&P.row_cost[j], (unsigned long long)item_segs);  // a sample ranks rows
          if (P.item_cost) P.item_cost[item] = (uint16_t)(item_segs < 65535u ? item_segs : 65535u);
          item = -1;
        }
      }
    }
  }

  RT_STAMP_END();
  RT_STEP_COUNT_END();
  const unsigned long long ws = wave_sum(nseg), wm = wave_sum(nsamp);
  unsigned long long wn = 0, wp = 0, wf = 0;
  if constexpr ((F & F_STATS) != 0) {
    wn = wave_sum(nnode);
    wp = wave_sum(nprim);
    wf = wave_sum(nfall);
  }
  if (lane == 0) {
    atomicAdd(&P.counters[0], ws);
    atomicAdd(&P.counters[3], wm);
    if constexpr ((F & F_STATS) != 0) {
      atomicAdd(&P.counters[1], wn);
      atomicAdd(&P.counters[2], wp);
      atomicAdd(&P.counters[4], wf);
    }
  }
}

// Stepwise megakernel for worlds that are ONE BVH object (C1/C2 sphere scenes).  render_kernel
// runs a whole world query per loop trip, so every lane of a wave stays in the traversal until
// the wave's longest query ends (~27 % lane utilisation on C2).  Here one loop trip is ONE
// traversal step (trav_step: a node pair and its primitive leaves) for the lanes that are
// traversing; a lane whose search has ended waits, and once `shade_min` lanes wait (or none is
// traversing) the wave runs its shading phase for all of them together: validation + hit record
// (bvh_settle, finalize), scatter, sample / item bookkeeping, refill from the work counter,
// the next camera ray and the next query's setup.  Per lane the sequence of RNG draws and float
// operations is exactly render_kernel's, so frame buffers are bit-identical.
template <int F>
__global__ __launch_bounds__(render_block<F>()) __attribute__((amdgpu_waves_per_eu(render_wpe<F>())))
void render_step_kernel(const RenderParams P) {
  const DScene& S = P.S;
  if constexpr ((F & F_LDS) != 0) stage_lds<F>(S);  // nodes, primitives, margins, materials, textures
  if constexpr ((F & F_QLDS) != 0) {  // the quantized traversal tree (24-byte pair records)
    uint32_t* q = (uint32_t*)rt_lds;
    for (int k = threadIdx.x; k < 6 * S.q_pairs; k += render_block<F>()) q[k] = S.qnodes[k];
    // ... and after its stacks the materials, textures and images (lds_mats / lds_texs / lds_imgs)
    float4* m = rt_lds + qlds_mats_at(S);
    const int nm = S.lds_mats, nt = 2 * S.lds_texs, ni = S.lds_imgs;
    for (int k = threadIdx.x; k < nm + nt + ni; k += render_block<F>())
      m[k] = k < nm ? ((const float4*)S.mats)[k]
                    : (k < nm + nt ? ((const float4*)S.texs)[k - nm] : ((const float4*)S.images)[k - nm - nt]);
    __syncthreads();
  }
  const unsigned lane = __lane_id();
  RT_STEP_COUNT_BEGIN();
  RT_STAMP_BEGIN();
  const rt_object obj = ro<F>(S.objects)[ro<F>(S.world)[0]];
  const int tbase = (F & F_WORLD) != 0 ? S.wt_fb : obj.c;  // traversal tree of the world's BVH / the world tree
  const float tmin = 0.001f, tmax = __builtin_inff();  // render.h:63
  long long item = -1;  // -1: no item
  bool done = false;
  int mode = 0;  // 0: between queries, 1: traversing, 2: search ended, shading pending
  // Per-item / per-sample state, touched only between queries.  The world-tree variants (PKS) keep it
  // in an LDS locker after the stacks (word k of thread t at [k * block + t]; the RNG state
  // lane-contiguous after them) instead of VGPRs, which the traversal loop needs (C5: the variant
  // needs ~190 VGPRs otherwise, far above the 128 of 4 waves/SIMD); their REF camera offsets come
  // from cam_tab, as in render_kernel, instead of a camera RNG copy.
  constexpr bool PKS = step_parks_mask(F);
  constexpr int LB = render_block<F>();
  uint32_t* const lk = (uint32_t*)rt_lds + LB * kStackDepth + threadIdx.x;
  int f_r = 0, i_r = 0, r_r = 0, j_r = 0, s_r = 0, depth_r = 0, ck_r = -1, lng_r = 0, fresh_r = 0;
  unsigned nseg_r = 0, nsamp_r = 0, item_segs_r = 0;
  int& f = cold_ref<PKS>(f_r, lk + 0 * LB);
  int& i = cold_ref<PKS>(i_r, lk + 1 * LB);
  int& r = cold_ref<PKS>(r_r, lk + 2 * LB);
  int& j = cold_ref<PKS>(j_r, lk + 3 * LB);
  int& s = cold_ref<PKS>(s_r, lk + 4 * LB);
  int& depth = cold_ref<PKS>(depth_r, lk + 5 * LB);
  unsigned& item_segs = cold_ref<PKS>(item_segs_r, lk + 6 * LB);
  unsigned& nseg = cold_ref<PKS>(nseg_r, lk + 7 * LB);
  unsigned& nsamp = cold_ref<PKS>(nsamp_r, lk + 8 * LB);
  int& ck = cold_ref<PKS>(ck_r, lk + 9 * LB);  // split_mode 1: perm position whose sample-start states are
                                               // recorded; 2: split sample (the item ends after it)
  int& lng = cold_ref<PKS>(lng_r, lk + 10 * LB);  // the item is one of the longest of the previous launch
  int& fresh = cold_ref<PKS>(fresh_r, lk + 11 * LB);  // the item's first sample is next (camera state)
  if constexpr (PKS) {
    nseg = 0;
    nsamp = 0;
    ck = -1;
    lng = 0;
  }
  float* const lkf = reinterpret_cast<float*>(lk);
  V att_r = mk(1, 1, 1), col_r = mk(0, 0, 0);
  auto vget = [&](V& reg, int w) -> V {
    if constexpr (PKS) return mk(lkf[w * LB], lkf[(w + 1) * LB], lkf[(w + 2) * LB]);
    else return reg;
  };
  auto vset = [&](V& reg, int w, V a) {
    if constexpr (PKS) {
      lkf[w * LB] = a.x;
      lkf[(w + 1) * LB] = a.y;
      lkf[(w + 2) * LB] = a.z;
    } else {
      reg = a;
    }
  };
  Rng loc_r{}, cam{};
  Rng& loc = cold_ref<PKS>(loc_r, (uint32_t*)rt_lds + LB * (kStackDepth + 18) + 6 * threadIdx.x);
  int s_end_r = 0;  // the lane's item ends after sample s_end - 1 (spp, or one sample of a split item)
  Ray ray{};
  V finv = mk(0, 0, 0), oi = mk(0, 0, 0);
  int cur = 0, sp = 0, best_prim = -1, best_rank = 0x7fffffff;
  float best = 0.0f, bhi = 0.0f, second = 0.0f, qa = 0.0f, rcpa = 0.0f;
  bool overflow = false;
  unsigned nnode = 0, nprim = 0, nfall = 0;
  const bool per_pixel = P.cam_mode == RT_CAM_PER_PIXEL;
  const rt_camera& C = S.cam;
  unsigned long long chunk_base = 0;  // wave-uniform: next unclaimed item of the wave's chunk
  unsigned chunk_left = 0;
  RT_WAVE_T0();

  for (;;) {
    // Shading passes: a camera ray answered by its tile's candidate list (mode 2 right after the
    // setup) is shaded in another pass of the same phase, so the traversal loop that follows
    // starts with every lane traversing.
    for (int pass = 0;; ++pass) {
      RT_STEP_COUNT(2);
      // ---- shading phase: finish the ended queries (render.h:60-77)
      RT_STAMP(7);  // back-to-back pair: phase 7 = the cost of one stamp per loop trip
      RT_STAMP(5);
      if (mode == 2) {
        ++nseg;
        ++item_segs;
        bool ended = false;
        V contrib;
        Hit h;
        bool hit;
        if constexpr ((F & F_WORLD) != 0) {
          // list world: the tree's winner, then the constant media that follow every tree entry in
          // the list, in list order with the closest hit so far (their RNG draws depend on it);
          // anything uncertain -- near ties, a chain the reference may reject, a ray that could
          // make an inert medium draw -- runs the reference's sequential list exactly
          constexpr int FM = F & ~(F_WORLD | F_STEP | F_BVH);  // media boundaries are primitives
          int wobj = -1, wprim = -1;
          int st = world_settle<F>(S, ray, tmin, overflow, bhi, second, best, best_prim, best_rank, wobj, wprim, nnode);
          if (S.w_inert && !ray_sane(ray)) st = 2;
          const bool exact = st == 2;
          if constexpr ((F & F_STATS) != 0) nfall += exact ? 1u : 0u;
          hit = st == 1;
          // exact: every entry in list order (the reference's visit sets); else the media after the tree
          for (int w = exact ? 0 : S.w_media; w < S.n_world; ++w) {
            const int oi = ro<F>(S.world)[w];
            const rt_object o = ro<F>(S.objects)[oi];
            float tq;
            int pq;
            bool hq;
            const float tcl = hit ? best : tmax;
            if (o.kind == RT_OBJ_MEDIUM) {
              hq = object_query<FM>(S, oi, ray, tmin, tcl, tq, pq, loc, nnode, nprim, nfall);
            } else {
              Ray rr = ray;
              int xi = oi;
              if constexpr ((F & F_XFORM) != 0) if (o.kind == RT_OBJ_XFORM) {
                Ray moved;
                rr = xform_ray(o, ray, moved);
                xi = o.a;
              }
              const rt_object x = ro<F>(S.objects)[xi];
              if ((F & F_BVH) != 0 && x.kind == RT_OBJ_BVH) {
                hq = bvh_exact<F>(S, x.a, x.b, rr, mk(1.0f / rr.d.x, 1.0f / rr.d.y, 1.0f / rr.d.z), tmin, tcl, tq, pq,
                                  nnode, nprim, nfall);
              } else {
                pq = x.a;
                hq = prim_t<F>(S, x.a, rr, tmin, tcl, tq, nprim);
              }
            }
            if (hq) {
              hit = true;
              best = tq;
              wobj = oi;
              wprim = pq;
            }
          }
          if (hit) object_record<FM>(S, wobj, wprim, ray, tmin, best, h);
        } else {
          hit = bvh_settle<F>(S, obj.a, obj.b, ray, tmin, tmax, overflow, bhi, second, best, best_prim, best_rank,
                              nnode, nprim, nfall);
          // primitive objects after the BVH in the world list (C4's ground sphere): hittable_list's
          // rule, t_max = the closest hit so far (inclusive), so a later entry wins a tie
          for (int w = 1; w < S.n_world; ++w) {
            const rt_object po = ro<0>(S.objects)[ro<0>(S.world)[w]];  // uniform: scalar loads
            float tq;
            if (prim_t_q<F>(S, load_prim_u<F>(S, po.a), ray, tmin, hit ? best : tmax, tq, nprim)) {
              hit = true;
              best = tq;
              best_prim = po.a;
            }
          }
          if (hit) finalize<F>(S, best_prim, ray, tmin, best, h);
        }
        if (!hit) {
          contrib = vget(att_r, 15) * ld3(S.bg);
          ended = true;
        } else {
          V a, em;
          RT_STAMP(6);
          bool sc;
          if constexpr (PKS) {  // on a register copy of the parked state
            Rng lr = loc;
            sc = scatter<F>(S, ray, h, a, em, lr);
            loc = lr;
          } else {
            sc = scatter<F>(S, ray, h, a, em, loc);
          }
          if (sc) {
            vset(att_r, 15, vget(att_r, 15) * a);
            if (++depth == P.max_depth) {
              contrib = mk(0.0f, 0.0f, 0.0f);
              ended = true;
            }
          } else {
            contrib = vget(att_r, 15) * em;
            ended = true;
          }
        }
        RT_STAMP(0);
        if (ended) {
          const V col = vget(col_r, 12) + contrib;
          vset(col_r, 12, col);
          depth = 0;
          ++nsamp;
          // the item ends after sample spp - 1, a split item's sample (split_mode 2) after itself
          // (parking variants derive it from ck: sample ck % spp)
          if constexpr (PKS) s_end_r = (P.split_mode == 2 && ck >= 0) ? ck - (ck / P.spp) * P.spp + 1 : P.spp;
          if (++s == s_end_r) {
            if (P.split_mode == 2 && ck >= 0) {  // one sample of a split item: its sum, merged later
              float* dst = P.contrib + 3 * (long long)ck;
              dst[0] = col.x;
              dst[1] = col.y;
              dst[2] = col.z;
            } else {
              const V out = (1.0f / (float)P.spp) * col;
              float* dst = P.fb + 3 * (((long long)f * P.rows + r) * P.W + i);
              dst[0] = out.x;
              dst[1] = out.y;
              dst[2] = out.z;
            }
            if (P.row_cost && (i & 15) == 0) atomicAdd(&P.row_cost[j], (unsigned long long)item_segs);
            if (P.item_cost) P.item_cost[item] = (uint16_t)(item_segs < 65535u ? item_segs : 65535u);
            if (P.split_mode == 1 && ck >= 0) P.ckpt[2 * (long long)ck * P.spp + 1] = make_uint4(0u, 0u, item_segs, 0u);
            item = -1;
          }
        }
        mode = 0;
      }
      RT_STAMP(0);
      // ---- refill lanes without an item from the wave's chunk of the work counter (one atomic
      // per kChunk items: a single counter serialises its atomics in L2)
      const unsigned long long idle = __ballot(item < 0 && !done);
      if (idle != 0 && (__popcll(idle) >= step_refill<F>() || __ballot(item >= 0) == 0)) {
        const unsigned long long mine = claim_items(P.work, idle, chunk_base, chunk_left);
        if (item < 0 && !done) {
          if (mine >= P.total_items) {
            done = true;
            RT_WAVE_EXHAUSTED();
          } else {
            unsigned long long pos = mine;
            int sa = 0;
            ck = -1;
            if (P.split_mode == 2) {  // split samples first, then the rest of perm
              const unsigned long long nsub = P.n_split * (unsigned long long)P.spp;
              const unsigned long long v = P.order ? (unsigned long long)P.order[mine] : mine;
              if (v < nsub) {
                pos = v / (unsigned)P.spp;
                sa = (int)(v - pos * (unsigned)P.spp);
                ck = (int)v;
              } else {
                pos = v - nsub + P.n_split;
              }
            } else if (P.split_mode == 1 && mine < P.n_split) {
              ck = (int)mine;
            }
            item = P.perm ? (long long)P.perm[pos] : (long long)pos;
            lng = pos < P.n_long ? 1 : 0;
            const long long per_row = P.per_row;  // same item order as render_kernel
            const int qi = (int)(item / per_row);
            const long long rem = item - (long long)qi * per_row;
            const int2 rj = P.row_q[qi * P.pstep];
            r = rj.x;
            f = (int)(rem / P.W);
            i = (int)(rem - (long long)f * P.W) * P.pstep;
            j = rj.y;
            const long long id = P.fb_first + f;
            const long long p = (long long)j * P.W + i;
            const long long slot = ((id + 1) * p + id + 1) % P.npix;  // render.h:101 (H3)
            const uint4* st = sa > 0 ? P.ckpt + 2 * (long long)ck : P.states + 2 * slot;
            const uint4 s0 = st[0], s1 = st[1];
            loc.d = s0.x; loc.v[0] = s0.y; loc.v[1] = s0.z; loc.v[2] = s0.w; loc.v[3] = s1.x; loc.v[4] = s1.y;
            s = sa;
            if constexpr (!PKS) s_end_r = (P.split_mode == 2 && ck >= 0) ? sa + 1 : P.spp;
            fresh = 1;
            depth = 0;
            item_segs = 0;
            vset(col_r, 12, mk(0, 0, 0));
          }
        }
      }
      // Waves holding one of the longest items (processed first) issue ahead of the others, so the
      // long items of a small multi-GPU share are not the last to finish.
      if (P.n_long > 0) {
        if (__ballot(item >= 0 && lng != 0) != 0) __builtin_amdgcn_s_setprio(3);
        else __builtin_amdgcn_s_setprio(0);
      }
      // ---- next query: camera ray at a sample's start (render.h:105-108, camera.h:49-58)
      RT_STAMP(1);
      if (item >= 0 && mode == 0) {
        // camera ray: its tile's candidate list (count + first entries) is loaded before the ray is
        // generated, so the loads overlap the camera arithmetic
        const bool listed = (F & F_WORLD) == 0 && depth == 0 && P.tile_cnt != nullptr;
        const int32_t* ent = nullptr;
        int tcnt = -1;
        int4 g0 = make_int4(0, 0, 0, 0);
        if (listed) {
          const int t = (j >> kTileShift) * P.tiles_x + (i >> kTileShift);
          ent = P.tile_ent + (size_t)t * P.tile_cap * 2;  // (id, nearest) pairs
          tcnt = P.tile_cnt[t];
          g0 = *reinterpret_cast<const int4*>(ent);
        }
        if (depth == 0 && PKS) {
          if (P.split_mode == 1 && ck >= 0 && s > 0) {  // record the sample-start state for split launches
            uint4* dst = P.ckpt + 2 * ((long long)ck * P.spp + s);
            dst[0] = make_uint4(loc.d, loc.v[0], loc.v[1], loc.v[2]);
            dst[1] = make_uint4(loc.v[3], loc.v[4], item_segs, 0u);
          }
          Rng lr = loc;
          camera_ray(P, C, i, j, s, per_pixel, lr, ray);  // REF offsets from cam_tab
          loc = lr;
          vset(att_r, 15, mk(1.0f, 1.0f, 1.0f));
        } else if (depth == 0) {
          // REF: the step kernel draws the per-sample lens offset and time from its own copy of the
          // pristine slot-0 state instead of cam_tab (measured faster here: the table read would sit
          // in the shading phase's dependent chain)
          if (fresh && !per_pixel) {
            if (s == 0) {
              cam.d = P.cam_state[0];
              for (int k = 0; k < 5; ++k) cam.v[k] = P.cam_state[1 + k];
            } else {  // a split sample: the camera state at its start
              const uint4 c0 = P.cam_st[2 * s], c1 = P.cam_st[2 * s + 1];
              cam.d = c0.x; cam.v[0] = c0.y; cam.v[1] = c0.z; cam.v[2] = c0.w; cam.v[3] = c1.x; cam.v[4] = c1.y;
            }
          }
          fresh = 0;
          if (P.split_mode == 1 && ck >= 0 && s > 0) {  // record the sample-start state for split launches
            uint4* dst = P.ckpt + 2 * ((long long)ck * P.spp + s);
            dst[0] = make_uint4(loc.d, loc.v[0], loc.v[1], loc.v[2]);
            dst[1] = make_uint4(loc.v[3], loc.v[4], item_segs, 0u);
          }
          const float u = ((float)i + rtx::uniform(loc)) / (float)P.W;
          const float v = ((float)j + rtx::uniform(loc)) / (float)P.H;
          Rng& cr = per_pixel ? loc : cam;
          const V rd = C.lens_radius * in_unit_disk(cr);
          const V off = rd.x * ld3(C.u) + rd.y * ld3(C.v);
          ray.o = ld3(C.origin) + off;
          ray.d = ld3(C.lower_left) + u * ld3(C.horizontal) + v * ld3(C.vertical) - ld3(C.origin) - off;
          ray.tm = urange(cr, C.time0, C.time1);
          vset(att_r, 15, mk(1.0f, 1.0f, 1.0f));
        }
        // traversal reciprocals: hardware v_rcp_f32 (1 ulp; the tree's boxes are padded by 2^-16
        // relative, far above either reciprocal's rounding) instead of three IEEE divides
        const V inv = mk(__builtin_amdgcn_rcpf(ray.d.x), __builtin_amdgcn_rcpf(ray.d.y), __builtin_amdgcn_rcpf(ray.d.z));
        finv = mk(__builtin_fminf(__builtin_fmaxf(inv.x, -1e30f), 1e30f),
                  __builtin_fminf(__builtin_fmaxf(inv.y, -1e30f), 1e30f),
                  __builtin_fminf(__builtin_fmaxf(inv.z, -1e30f), 1e30f));
        oi = mk(ray.o.x * finv.x, ray.o.y * finv.y, ray.o.z * finv.z);
        qa = len2(ray.d);
        rcpa = __builtin_amdgcn_rcpf(qa);
        best = __builtin_inff();
        bhi = __builtin_inff();
        second = __builtin_inff();
        best_prim = -1;
        best_rank = 0x7fffffff;
        cur = 0;
        sp = 0;
        overflow = false;
        mode = 1;
        if constexpr ((F & F_WORLD) == 0) {
          if (listed && tcnt >= 0) {  // camera ray: the tile's candidate list instead of the tree
            tile_candidates<F>(S, ent, tcnt, g0, ray, qa, rcpa, tmin, tmax, best, bhi, second, best_prim, best_rank,
                               nprim);
            mode = 2;
          }
        }
      }
      if (pass + 1 >= kShadePasses || __ballot(mode == 2) == 0) break;
    }
    RT_STAMP(3);
    if (__ballot(mode != 0) == 0) break;  // no item left for any lane of the wave (mode 2: a listed camera ray)
    // ---- traversal steps until shade_min lanes wait (or none traverses)
    for (;;) {
      RT_STEP_COUNT(3);
      // several traversal steps per check of the shading condition, same VGPRs (same box, Mrays/s at
      // 1 / 2 / 3 / 4 steps: C2 14 538 / 14 713 / 14 829 / 14 843, C4 11 180 / 11 247 (before the
      // triangle dedupe) and 14 095 / 14 051 / 13 990 after it); the opt-in world-tree variants keep
      // one (more spills with two)
      constexpr int kUnroll = (F & F_WORLD) != 0 ? 1 : ((F & F_TRI) != 0 ? 2 : 4);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
      if (mode == 1) {
        RT_STEP_COUNT(0);
        if (!trav_step<F>(S, tbase, ray, oi, finv, qa, rcpa, tmin, tmax, cur, sp, best, bhi, second, best_prim,
                          best_rank, overflow, nnode, nprim))
          mode = 2;
      }
      // (the threshold as a kernel argument measured 1.5 % faster than the compile-time constant)
      if (__ballot(mode == 1) == 0 || __popcll(__ballot(mode == 2)) >= P.shade_min) break;
    }
  }

  RT_STEP_COUNT_END();
  RT_STAMP_END();
  RT_WAVE_END();
  const unsigned long long ws = wave_sum(nseg), wm = wave_sum(nsamp);
  unsigned long long wn = 0, wp = 0, wf = 0;
  if constexpr ((F & F_STATS) != 0) {
    wn = wave_sum(nnode);
    wp = wave_sum(nprim);
    wf = wave_sum(nfall);
  }
  if (lane == 0) {
    atomicAdd(&P.counters[0], ws);
    atomicAdd(&P.counters[3], wm);
    if constexpr ((F & F_STATS) != 0) {
      atomicAdd(&P.counters[1], wn);
      atomicAdd(&P.counters[2], wp);
      atomicAdd(&P.counters[4], wf);
    }
  }
}

// curand_init(seed, slot, 0) for every slot < n (render.h:84-92).  Each lane owns `chunk`
// consecutive slots: one seed scramble + subsequence jump A^(first * 2^67) applied digit by digit
// in base 4 (as skipahead_sequence: digit d at position i applies (A^(4^i * 2^67))^d), then one
// mat-vec with A^(2^67) per following slot (state(s+1) = A^(2^67) state(s)).  Every mat-vec on
// GF(2)^160 goes through byte tables (rt_ctx::jump_tab, built once per context): the image of the
// state is the XOR of 20 table rows, one per state byte, instead of 160 masked row XORs.  The
// slot-step table (the one every following slot applies) is staged in LDS, one workgroup per CU:
// with every table read from L2 the kernel moved ~1 GB of table rows per C2 init (105 us).
constexpr int kInitBlock = 512;
constexpr int kStepRows = 20 * 256;           // rows of a byte table
constexpr int kTabRow = 8;                    // words per table row (5 used, 32-byte aligned)
constexpr int kTabMat = 20 * 256 * kTabRow;   // words per matrix table
__device__ __forceinline__ void tab_apply(const uint32_t* __restrict__ t, uint32_t v[5]) {
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
  #pragma unroll
  for (int b = 0; b < 20; ++b) {
    const uint32_t byte = (v[b >> 2] >> (8 * (b & 3))) & 0xffu;
    const uint4 x = *(const uint4*)(t + (b * 256 + byte) * kTabRow);
    const uint32_t y = t[(b * 256 + byte) * kTabRow + 4];
    r0 ^= x.x;
    r1 ^= x.y;
    r2 ^= x.z;
    r3 ^= x.w;
    r4 ^= y;
  }
  v[0] = r0; v[1] = r1; v[2] = r2; v[3] = r3; v[4] = r4;
}
// The slot-step table in LDS as five planes (word k of row r at [k * kStepRows + r]).
__device__ __forceinline__ void tab_apply_lds(const uint32_t* t, uint32_t v[5]) {
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
  #pragma unroll
  for (int b = 0; b < 20; ++b) {
    const int row = b * 256 + (int)((v[b >> 2] >> (8 * (b & 3))) & 0xffu);
    r0 ^= t[row];
    r1 ^= t[kStepRows + row];
    r2 ^= t[2 * kStepRows + row];
    r3 ^= t[3 * kStepRows + row];
    r4 ^= t[4 * kStepRows + row];
  }
  v[0] = r0; v[1] = r1; v[2] = r2; v[3] = r3; v[4] = r4;
}
// jump_tab: table (d - 1) * 32 + i = (A^(4^i * 2^67))^d, d = 1..3; table 0 is the slot step.
__global__ __launch_bounds__(kInitBlock) void init_states_kernel(uint4* states, long long n, uint64_t seed,
                                                                const uint32_t* __restrict__ jump_tab, int digits,
                                                                long long chunk) {
  extern __shared__ uint32_t step_lds[];  // 5 * kStepRows words
  for (int r = threadIdx.x; r < kStepRows; r += kInitBlock) {
    const uint4 x = *(const uint4*)(jump_tab + (size_t)r * kTabRow);
    step_lds[r] = x.x;
    step_lds[kStepRows + r] = x.y;
    step_lds[2 * kStepRows + r] = x.z;
    step_lds[3 * kStepRows + r] = x.w;
    step_lds[4 * kStepRows + r] = jump_tab[(size_t)r * kTabRow + 4];
  }
  __syncthreads();
  const long long first = ((long long)blockIdx.x * kInitBlock + threadIdx.x) * chunk;
  if (first >= n) return;
  rtx::State st = rtx::seed_state(seed);
  unsigned long long x = (unsigned long long)first;
  for (int d = 0; d < digits; ++d) {
    const unsigned dig = (unsigned)(x & 3u);
    x >>= 2;
    if (dig != 0) tab_apply(jump_tab + (size_t)((dig - 1) * 32 + d) * kTabMat, st.v);
  }
  for (long long c = 0; c < chunk && first + c < n; ++c) {
    if (c > 0) tab_apply_lds(step_lds, st.v);
    const long long slot = first + c;
    states[2 * slot] = make_uint4(st.d, st.v[0], st.v[1], st.v[2]);
    states[2 * slot + 1] = make_uint4(st.v[3], st.v[4], 0u, 0u);
  }
}

// write_frame_buffer quantisation (color.h:40-44); NaN defined as 0.
__device__ __forceinline__ int quant(float x) {
  const float r = __builtin_sqrtf(x);
  if (!(r == r)) return 0;
  const float c = r < 0.0f ? 0.0f : (r > 0.999f ? 0.999f : r);
  return (int)(256.0f * c);
}

// average_images (color.h:57-170) over fbs 0..nfb-1 in order, per owned pixel.
__global__ __launch_bounds__(kBlock) void resolve_kernel(const float* __restrict__ fb, uint8_t* __restrict__ out,
                                                        long long per_fb, int nfb) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (k >= per_fb) return;
  float acc = 0.0f;
  for (int f = 0; f < nfb; ++f) {
    const int c = quant(fb[(long long)f * per_fb + k]);
    acc += (float)(c * c) / (255.0f * 255.0f);
  }
  out[k] = (uint8_t)quant(acc / (float)nfb);
}

// Split items (render_step_kernel split_mode 2): the fb value of each of the first n_split items
// of perm from its samples' sums, added in sample order from 0 -- the same float additions as the
// item's own loop (col = 0; col += sample sum; (0 + x) + y == x + y for every x that is not -0,
// and a sample sum 0 + c is never -0) -- then scaled by 1 / spp as render.h:111 does.
__global__ __launch_bounds__(kBlock) void merge_split_kernel(const RenderParams P) {
  const long long p = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (p >= (long long)P.n_split) return;
  const long long item = P.perm[p];
  const long long per_row = (long long)P.fb_count * P.W;
  const int q = (int)(item / per_row);
  const long long rem = item - (long long)q * per_row;
  const int r = P.row_q[q].x;
  const int f = (int)(rem / P.W);
  const int i = (int)(rem - (long long)f * P.W);
  V col = mk(0.0f, 0.0f, 0.0f);
  for (int s = 0; s < P.spp; ++s) col = col + ld3(P.contrib + 3 * (p * P.spp + s));
  const V out = (1.0f / (float)P.spp) * col;
  float* dst = P.fb + 3 * (((long long)f * P.rows + r) * P.W + i);
  dst[0] = out.x;
  dst[1] = out.y;
  dst[2] = out.z;
}

// Segment count of every split sample k = pos * spp + s of the recording launch (split_mode 1):
// the difference of the item's segment counts at consecutive sample starts (ckpt's spare word),
// the last sample's up to the item's total (kept at sample 0's record).  Clamped to 255.
__global__ __launch_bounds__(kBlock) void split_len_kernel(const uint4* __restrict__ ckpt, unsigned long long nsub,
                                                           int spp, uint8_t* __restrict__ len) {
  const unsigned long long k = (unsigned long long)blockIdx.x * kBlock + threadIdx.x;
  if (k >= nsub) return;
  const unsigned long long pos = k / (unsigned)spp;
  const int s = (int)(k - pos * (unsigned)spp);
  const unsigned st = s > 0 ? ckpt[2 * k + 1].z : 0u;
  const unsigned en = s + 1 < spp ? ckpt[2 * (k + 1) + 1].z : ckpt[2 * pos * spp + 1].z;
  const unsigned d = en >= st ? en - st : 0u;
  len[k] = (uint8_t)(d < 255u ? d : 255u);
}

// Claim order of a split launch, built on the device from the sample lengths (split_len_kernel)
// and the unsplit positions' cost groups (host tables; `kOrderKeys` keys: a sample's length, an
// unsplit position's bucket midpoint clamped to 256 -- every sample key is < 256):
//   sample k of key v   -> sub_base[v] + its rank among the samples of key v, in k order (a
//                          stable counting sort: neighbouring samples keep their order, as the
//                          coherence of the claims needs -- an atomic-order scatter measured
//                          1.5-4 % slower launches)
//   unsplit position r  -> r + (samples with key >= key(r)), key(r) from rest_gt (unsplit
//                          positions with key > v, non-increasing in v; perm is longest first)
// so samples precede unsplit positions of an equal key.  Results do not depend on the order.
// The sort runs over tiles of kOrderTile samples, one wave per tile: per-tile histograms, a scan
// per key over the tiles, then each tile's samples ranked in order with ballots.
constexpr int kOrderKeys = 257;
constexpr int kOrderTile = 4096;
__global__ __launch_bounds__(64) void order_tile_hist_kernel(const uint8_t* __restrict__ len, unsigned long long n,
                                                             unsigned* __restrict__ tile_hist) {
  __shared__ unsigned h[256];
  for (int v = threadIdx.x; v < 256; v += 64) h[v] = 0;
  __syncthreads();
  const unsigned long long k0 = (unsigned long long)blockIdx.x * kOrderTile;
  for (int q = threadIdx.x; q < kOrderTile; q += 64)
    if (k0 + q < n) atomicAdd(&h[len[k0 + q]], 1u);
  __syncthreads();
  for (int v = threadIdx.x; v < 256; v += 64) tile_hist[(size_t)blockIdx.x * 256 + v] = h[v];
}
// One block per key: exclusive prefix over the tiles (in place), the key's total into total[v].
__global__ __launch_bounds__(256) void order_scan_kernel(unsigned* __restrict__ tile_hist, unsigned tiles,
                                                         unsigned* __restrict__ total) {
  __shared__ unsigned part[256];
  const unsigned v = blockIdx.x, per = (tiles + 255) / 256, t0 = threadIdx.x * per;
  unsigned sum = 0;
  for (unsigned t = t0; t < t0 + per && t < tiles; ++t) sum += tile_hist[(size_t)t * 256 + v];
  part[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned acc = 0;
    for (int q = 0; q < 256; ++q) {
      const unsigned x = part[q];
      part[q] = acc;
      acc += x;
    }
    total[v] = acc;
  }
  __syncthreads();
  unsigned acc = part[threadIdx.x];
  for (unsigned t = t0; t < t0 + per && t < tiles; ++t) {
    const unsigned x = tile_hist[(size_t)t * 256 + v];
    tile_hist[(size_t)t * 256 + v] = acc;
    acc += x;
  }
}
// tab: sub_base[256], sub_ge[kOrderKeys], rest_gt[kOrderKeys]
__global__ __launch_bounds__(64) void order_scatter_kernel(const uint8_t* __restrict__ len, unsigned long long need,
                                                           const unsigned* __restrict__ tile_off,
                                                           const unsigned* __restrict__ tab, uint32_t* __restrict__ order) {
  __shared__ unsigned cnt[256];
  for (int v = threadIdx.x; v < 256; v += 64) cnt[v] = tab[v] + tile_off[(size_t)blockIdx.x * 256 + v];
  __syncthreads();
  const unsigned long long k0 = (unsigned long long)blockIdx.x * kOrderTile;
  const unsigned lane = threadIdx.x;
  for (int q = 0; q < kOrderTile; q += 64) {
    const unsigned long long k = k0 + q + lane;
    if (k0 + q >= need) break;  // wave-uniform
    bool pending = k < need;
    const unsigned v = pending ? len[k] : 0u;
    while (__ballot(pending) != 0) {  // one pass per distinct key among the 64
      const unsigned long long act = __ballot(pending);
      const unsigned lead = __shfl(v, __ffsll((long long)act) - 1, 64);
      const unsigned long long m = __ballot(pending && v == lead);
      const unsigned base = cnt[lead];
      if (pending && v == lead) {
        order[base + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)k;
        pending = false;
      }
      __syncthreads();  // every lane has read cnt[lead] (one wave: a barrier of the wave)
      if (lane == 0) cnt[lead] = base + (unsigned)__popcll(m);
      __syncthreads();
    }
  }
}
// Sort keys of the item schedule: the measuring launch's segment count in buckets of 2^shift,
// clamped to the top bucket 255 (items of >= 255 * 2^shift segments keep their natural order).
__global__ __launch_bounds__(kBlock) void cost_key_kernel(const uint16_t* __restrict__ cost, unsigned long long n,
                                                          int shift, uint8_t* __restrict__ key) {
  const unsigned long long k = (unsigned long long)blockIdx.x * kBlock + threadIdx.x;
  if (k < n) key[k] = (uint8_t)min(255u, (unsigned)cost[k] >> shift);
}
// Largest measured item cost (build_schedule sizes the cost buckets from it).
__global__ __launch_bounds__(kBlock) void cost_max_kernel(const uint16_t* __restrict__ cost, unsigned long long n,
                                                          unsigned* __restrict__ out) {
  unsigned m = 0;
  for (unsigned long long k = (unsigned long long)blockIdx.x * kBlock + threadIdx.x; k < n;
       k += (unsigned long long)gridDim.x * kBlock)
    m = max(m, (unsigned)cost[k]);
  for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off, 64));
  if (__lane_id() == 0) atomicMax(out, m);
}
__global__ __launch_bounds__(kBlock) void order_rest_kernel(unsigned long long need, unsigned long long rest,
                                                            const unsigned* __restrict__ tab, uint32_t* __restrict__ order) {
  const unsigned long long r = (unsigned long long)blockIdx.x * kBlock + threadIdx.x;
  if (r >= rest) return;
  const unsigned* sub_ge = tab + 256;
  const unsigned* rest_gt = tab + 256 + kOrderKeys;
  int lo = 0, hi = kOrderKeys - 1;  // smallest key v with rest_gt[v] <= r (= r's key)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (rest_gt[mid] <= (unsigned)r) hi = mid;
    else lo = mid + 1;
  }
  order[r + sub_ge[lo]] = (uint32_t)(need + r);
}

// Camera-ray culling per 8x8-pixel tile.  A camera ray (render.h:105-108, camera.h:49-58) is
//   X(t) = O + off + t (F - O - off),  F = lower_left + u horizontal + v vertical,
// with (u, v) inside the tile (jitter in [0, 1] of a pixel), |off| <= lens_radius = L and its time
// in the shutter.  X(t) = Y(t) + (1 - t) off with Y(t) = O + t (F - O) inside the pinhole frustum of
// the tile, so a sphere (C, R) hit at parameter t >= 0 is within R + |1 - t| L of that frustum: it
// is kept unless it lies farther than that outside one of the frustum's four side planes.  (C, R)
// bounds a primitive's or an object's box over the shutter (rt_scene_upload); t <= (|C - O| + R +
// L) / (dmin - L) with dmin the distance from O to the focus plane; R is widened by 4e-3 (|C - O| +
// R + L) for the float rounding of the ray and of the reference's hit tests (a sphere's
// discriminant admits rays up to ~1e-3 |oc| beyond its radius).  Double precision throughout.
struct TileFrustum {
  double O[3], N[4][3], dmin, L;
  bool ok;
  __device__ void init(const rt_camera& cam, int W, int H, int t, int tx) {
    const int i0 = (t % tx) << kTileShift, j0 = (t / tx) << kTileShift;
    const int i1 = min(i0 + (1 << kTileShift), W), j1 = min(j0 + (1 << kTileShift), H);
    const double us[2] = {(i0 - 0.01) / W, (i1 + 0.01) / W}, vs[2] = {(j0 - 0.01) / H, (j1 + 0.01) / H};
    double D[4][3], Dc[3] = {0, 0, 0};
    for (int k = 0; k < 3; ++k) O[k] = cam.origin[k];
    const int cu[4] = {0, 1, 1, 0}, cv[4] = {0, 0, 1, 1};
    for (int c = 0; c < 4; ++c)
      for (int k = 0; k < 3; ++k) {
        D[c][k] = (double)cam.lower_left[k] + us[cu[c]] * cam.horizontal[k] + vs[cv[c]] * cam.vertical[k] - O[k];
        Dc[k] += 0.25 * D[c][k];
      }
    for (int c = 0; c < 4; ++c) {
      const double* a = D[c];
      const double* b = D[(c + 1) & 3];
      const double m[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
      const double len = sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
      const double sg = (m[0] * Dc[0] + m[1] * Dc[1] + m[2] * Dc[2]) < 0 ? -1.0 : 1.0;
      for (int k = 0; k < 3; ++k) N[c][k] = sg * m[k] / len;
    }
    const float* h = cam.horizontal;
    const float* v = cam.vertical;
    double nf[3] = {(double)h[1] * v[2] - (double)h[2] * v[1], (double)h[2] * v[0] - (double)h[0] * v[2],
                    (double)h[0] * v[1] - (double)h[1] * v[0]};
    const double nl = sqrt(nf[0] * nf[0] + nf[1] * nf[1] + nf[2] * nf[2]);
    dmin = fabs(D[0][0] * nf[0] + D[0][1] * nf[1] + D[0][2] * nf[2]) / nl;
    L = (double)fabsf(cam.lens_radius) * (1.0 + 1e-5) + 1e-7;
    ok = dmin > 2.0 * L && dmin < 1e30;  // else (degenerate camera) no culling
    for (int c = 0; c < 4; ++c)
      for (int k = 0; k < 3; ++k) ok = ok && N[c][k] == N[c][k];
  }
  // Lower bound on |p - o| for any point p of sphere s and any camera ray origin o = O + off
  // (|off| <= L): |C - O| - R - L, rounded down (cast and a 1e-5 relative margin).  A camera ray's
  // hit parameter t is then >= nearest / |d| (p = o + t d).
  __device__ float nearest(float4 s) const {
    const double C[3] = {s.x - O[0], s.y - O[1], s.z - O[2]};
    const double dist = sqrt(C[0] * C[0] + C[1] * C[1] + C[2] * C[2]);
    const double m = dist - s.w - L - 1e-5 * (dist + s.w + L) - 1e-6;
    if (!(m == m)) return -__builtin_inff();
    return __double2float_rd(m);
  }
  // May a camera ray of the tile hit something inside sphere s (xyz centre, w radius)?
  __device__ bool sees(float4 s) const {
    const double C[3] = {s.x - O[0], s.y - O[1], s.z - O[2]};
    const double dist = sqrt(C[0] * C[0] + C[1] * C[1] + C[2] * C[2]);
    const double reach = dist + s.w + L;
    const double m = s.w + 4e-3 * reach + L * fmax(1.0, reach / (dmin - L)) + 1e-6;
    if (!(m < 1e300)) return true;  // NaN or infinite bound: always kept
    for (int p = 0; p < 4; ++p)
      if (N[p][0] * C[0] + N[p][1] * C[1] + N[p][2] * C[2] < -m) return false;
    return true;
  }
};

// World = one BVH: every primitive of the BVH that a camera ray of tile t may hit (ids[q] for the
// bounding sphere sph[q]); cnt[t] = -1 when the tile overflows kTileCap (it traverses the tree).
__global__ __launch_bounds__(kBlock) void bin_tiles_kernel(const float4* __restrict__ sph, const int32_t* __restrict__ ids,
                                                          int n, rt_camera cam, int W, int H, int tx, int ty,
                                                          int32_t* __restrict__ cnt, int32_t* __restrict__ ent) {
  const int t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= tx * ty) return;
  TileFrustum fr;
  fr.init(cam, W, H, t, tx);
  int c = 0;
  int32_t* e = ent + (size_t)t * kTileCap * 2;  // (primitive id, nearest distance bits) pairs
  if (!fr.ok) {
    c = kTileCap + 1;
  } else {
    for (int q = 0; q < n; ++q)
      if (fr.sees(sph[q])) {
        if (c < kTileCap) {  // insertion by the nearest possible hit distance, ascending
          const float dn = fr.nearest(sph[q]);
          int k = c;
          for (; k > 0 && __int_as_float(e[2 * k - 1]) > dn; --k) {
            e[2 * k] = e[2 * k - 2];
            e[2 * k + 1] = e[2 * k - 1];
          }
          e[2 * k] = ids[q];
          e[2 * k + 1] = __float_as_int(dn);
        }
        ++c;
      }
  }
  cnt[t] = c <= kTileCap ? c : -1;
}

// World = a list: bit w of mask[t] is set when a camera ray of tile t may hit top-level entry w
// (w < 32; entries past 32 are always tested).  An entry that no ray of the tile can reach makes
// no RNG draw either: a constant medium draws only after its boundary is hit at t > t_min.
__global__ __launch_bounds__(kBlock) void bin_masks_kernel(const float4* __restrict__ sph, int n, rt_camera cam, int W,
                                                          int H, int tx, int ty, uint32_t* __restrict__ mask) {
  const int t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= tx * ty) return;
  TileFrustum fr;
  fr.init(cam, W, H, t, tx);
  uint32_t m = 0xffffffffu;
  if (fr.ok)
    for (int w = 0; w < n && w < 32; ++w)
      if (!fr.sees(sph[w])) m &= ~(1u << w);
  mask[t] = m;
}

}  // namespace

// ====================================================================== host side (C ABI)
struct rt_ctx {
  int device = 0;
  rt_ctx_options opt{};  // rt_ctx_set_options (defaults: rt_ctx_options_default)
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;  // render call start, its end; render kernel start
  std::string err;
  std::vector<void*> scene_bufs;
  DScene scene{};
  bool have_scene = false;
  uint4* states = nullptr;
  long long states_n = 0;
  uint64_t states_seed = 0;
  uint32_t* seq = nullptr;
  uint32_t* jump_tab = nullptr;  // byte tables of the subsequence jumps (init_states_kernel)
  unsigned long long* work = nullptr;  // [0] work counter, [1..4] counters
  int32_t* row_map = nullptr;  // [rows] {owned row r, image row j} in processing order (RenderParams::row_q)
  std::vector<int32_t> row_map_host;  // what row_map holds (uploaded only when it changes)
  int row_cap = 0;
  unsigned long long* row_cost = nullptr;  // device, per image row
  int row_cost_cap = 0;
  // Per-row cost of the last launch of (scene generation, W, H, spp, depth): the schedule of the
  // next launch of that configuration (no pixel result depends on the order).
  std::vector<unsigned long long> host_cost;
  long long cost_key[5] = {-1, -1, -1, -1, -1};
  // Item schedule of the last configuration (scene generation, size, spp, depth, fb range, tiling):
  // per-item segment counts of its measuring launch -> longest items first (perm).
  uint16_t* item_cost = nullptr;
  uint16_t* probe_cost = nullptr;  // per (owned row, pixel): the probe launch's segment counts
  long long probe_cap = 0;
  uint32_t* spread_tmp = nullptr;  // probe_schedule: a copy of perm's head, gathered back spread
  long long spread_cap = 0;
  uint32_t* perm = nullptr;
  long long item_cap = 0;
  static constexpr int kKey = 11;
  long long perm_key[kKey] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
  long long pending_key[kKey] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};  // measured, schedule not built yet
  unsigned long long pending_segs = 0;
  unsigned long long n_long = 0;
  // Split samples of the longest items (render_step_kernel; see rt_render): n_split perm positions,
  // split_state 0 = record on the next launch of perm_key, 1 = recorded for split_seed.
  unsigned long long n_split = 0;
  int split_state = -1;
  uint64_t split_seed = 0;
  uint4* ckpt = nullptr;
  long long ckpt_cap = 0;  // uint4 pairs
  float* contrib = nullptr;
  long long contrib_cap = 0;  // floats
  uint4* cam_st = nullptr;
  long long cam_st_cap = 0;  // uint4 pairs
  // Claim order of the split launches (RenderParams::order), built on the first one after a
  // recording (order_scatter_kernel); rest_gt[v]: unsplit perm positions (from n_split on) whose
  // key -- cost bucket midpoint, clamped to 256 -- exceeds v; order_tab: the kernel's tables, its
  // histogram and cursors (order_tab_host: the host copy of the tables).
  uint32_t* order = nullptr;
  long long order_cap = 0;
  bool order_ok = false;
  long long rest_n = -1;
  std::vector<unsigned> rest_gt;
  unsigned* order_tab = nullptr;
  std::vector<unsigned> order_tab_host;
  // scratch of the device sorts (sort_keys / sort_scatter): keys, then per-tile tables
  uint8_t* sort_scratch = nullptr;
  long long sort_scratch_cap = 0;
  long long cam_st_key[3] = {-1, -1, -1};
  long long scene_gen = 0;
  int cus = 0, blocks_per_cu[32] = {0};  // per kernel variant (kVariants)
  int features = 0;
  bool world_bvh = false;  // the world list is one BVH object (camera tile lists apply)
  bool world_step = false;  // one BVH object followed by primitive objects (render_step_kernel applies)
  bool world_tree = false;  // a list world flattened into the world tree (render_step_kernel<..|F_WORLD>)
  int dev_nodes = 0, dev_prims = 0, dev_mats = 0, dev_texs = 0, dev_imgs = 0;  // device array sizes (LDS staging)
  int plane_fb = -1, plane_pairs = 0;  // world tree staged in planes by the stepwise LDS variant (-1: not)
  float last_ms = 0.0f;         // the last rt_render's device time: probe + schedule + render kernel
  float last_kernel_ms = 0.0f;  // ... its render kernel (and split merge) alone
  int last_sched = 0;  // RT_SCHED_* of the last render launch
  char last_kernel[48] = "";  // rocprof name stem of the last render launch, e.g. render_step_kernel<25730>
  float* dbg = nullptr;  // audit log: [0] = count, then 16 floats per entry
  // Camera-ray candidate lists (world = one BVH): bounding spheres of the world BVH's primitives
  // over the shutter (scene buffers) and the per-tile lists of the last (scene, W, H).
  const float4* bin_sph = nullptr;
  const int32_t* bin_ids = nullptr;
  int bin_n = 0;
  // REF camera mode: per-sample lens offset + time of the last (scene, seed, spp) (camera_table)
  float4* cam_tab = nullptr;
  long long cam_cap = 0;
  long long cam_key[3] = {-1, -1, -1};
  std::vector<float4> cam_host;  // stays alive while the upload is in flight
  std::vector<uint4> cam_st_host;
  int32_t* tiles = nullptr;  // [ntiles] counts, then [ntiles * kTileCap] entries
  long long tiles_cap = 0;
  long long tiles_key[3] = {-1, -1, -1};
};

namespace {

struct Variant {
  int mask;
  const void* fn;
};
#define RT_VARIANT(m) {m, (const void*)render_kernel<m>}
#define RT_VARIANT_STEP(m) {m, (const void*)render_step_kernel<m>}
const Variant kVariants[] = {
    RT_VARIANT_STEP(F_SPHERES | F_LDS | F_STEP),
    RT_VARIANT_STEP(F_SPHERES | F_STEP),
    RT_VARIANT_STEP(F_MESH | F_STEP),
    RT_VARIANT_STEP(F_MESH | F_STEP | F_QLDS),
    RT_VARIANT_STEP(F_CORNELL | F_WORLD | F_STEP),
    RT_VARIANT_STEP(F_FINAL | F_WORLD | F_STEP),
    RT_VARIANT(F_SPHERES),
    RT_VARIANT(F_ALL),
    RT_VARIANT(F_SPHERES | F_STATS),
    RT_VARIANT(F_ALL | F_STATS),
    RT_VARIANT(F_SPHERES | F_EXACT),
    RT_VARIANT(F_ALL | F_EXACT),
    RT_VARIANT(F_SPHERES | F_EXACT | F_STATS),
    RT_VARIANT(F_ALL | F_EXACT | F_STATS),
    RT_VARIANT(F_SPHERES | F_CHECK),
    RT_VARIANT(F_ALL | F_CHECK),
    RT_VARIANT(F_SPHERES | F_LDS),
    RT_VARIANT(F_ALL | F_LDS),
    RT_VARIANT(F_CORNELL),
    RT_VARIANT(F_CORNELL | F_EXACT),
    RT_VARIANT(F_CORNELL | F_EXACT | F_STATS),
    RT_VARIANT(F_MESH),
    RT_VARIANT(F_MESH | F_STATS),
    RT_VARIANT(F_MESH | F_EXACT),
    RT_VARIANT(F_FINAL),
    RT_VARIANT(F_FINAL | F_MERGE),
    // the counting twin of C2's stepwise LDS variant: bench.py's untimed stats pass counts the node and
    // primitive tests of the traversal it times (culled search, camera tile lists)
    RT_VARIANT_STEP(F_SPHERES | F_LDS | F_STEP | F_STATS),
    // probe twins of the product variants of C2, C4 and C5 (F_PROBE changes no code)
    RT_VARIANT_STEP(F_SPHERES | F_LDS | F_STEP | F_PROBE),
    RT_VARIANT_STEP(F_MESH | F_STEP | F_QLDS | F_PROBE),
    RT_VARIANT(F_FINAL | F_MERGE | F_PROBE),
};
#undef RT_VARIANT
#undef RT_VARIANT_STEP
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
static_assert(kNumVariants <= 32, "rt_ctx::blocks_per_cu holds 32 variants");
constexpr int kLdsBudget = 156 * 1024;  // bytes of staged nodes + primitives + stacks per workgroup

// Smallest compiled variant that covers the scene's features and the requested mode.
int pick_variant(int features, bool stats, bool exact, bool check, bool lds, bool widest = false, bool step = false,
                 bool world = false, bool qlds = false, bool merge = false) {
  const int modes = F_STATS | F_EXACT | F_CHECK | F_LDS | F_STEP | F_WORLD | F_QLDS | F_MERGE;
  const int mode = check ? F_CHECK : ((stats ? F_STATS : 0) | (exact ? F_EXACT : 0));
  auto best_of = [&](int want) {  // covering variant with the fewest (widest: most) feature bits
    int best = -1;
    for (int v = 0; v < kNumVariants; ++v) {
      const int m = kVariants[v].mask;
      if ((m & modes) != want || (features & ~m) != 0 || (m & F_PROBE) != 0) continue;
      const int pm = __builtin_popcount(m), pb = best < 0 ? 0 : __builtin_popcount(kVariants[best].mask);
      if (best < 0 || (widest ? pm > pb : pm < pb)) best = v;
    }
    return best;
  };
  int v = best_of(mode);
  if (v >= 0 && lds && mode == 0)  // the LDS twin of that variant, when one is compiled
    for (int w = 0; w < kNumVariants; ++w)
      if (kVariants[w].mask == (kVariants[v].mask | F_LDS)) {
        v = w;
        break;
      }
  if (v >= 0 && step && mode == 0) {  // its stepwise twin (world = one BVH object, or the world tree)
    int sv = -1;
    for (int w = 0; w < kNumVariants; ++w)
      if (kVariants[w].mask == (kVariants[v].mask | F_STEP | (world ? F_WORLD : 0))) sv = w;
    if (sv >= 0 && qlds)  // ... with its traversal tree quantized in LDS
      for (int w = 0; w < kNumVariants; ++w)
        if (kVariants[w].mask == (kVariants[sv].mask | F_QLDS)) return w;
    if (sv >= 0) return sv;
  }
  if (v >= 0 && merge && mode == 0)  // its merged-search twin (render_kernel; merge_ok scenes)
    for (int w = 0; w < kNumVariants; ++w)
      if (kVariants[w].mask == (kVariants[v].mask | F_MERGE)) return w;
  if (v >= 0 && mode == F_STATS && lds && step && !world)  // the counting twin of the stepwise LDS variant
    for (int w = 0; w < kNumVariants; ++w)
      if (kVariants[w].mask == (kVariants[v].mask | F_LDS | F_STEP)) return w;
  return v;
}
// The probe twin of variant v (same code, own symbol), or v itself when none is compiled.
int probe_variant(int v) {
  for (int w = 0; w < kNumVariants; ++w)
    if (kVariants[w].mask == (kVariants[v].mask | F_PROBE)) return w;
  return v;
}
int variant_block(int v) { return (kVariants[v].mask & (F_LDS | F_QLDS)) != 0 ? 1024 : 256; }

int scene_features(const rt_scene_soa* s) {
  int f = 0;
  for (int k = 0; k < s->n_prims; ++k) {
    const int t = s->prims[k].type;
    if (t == RT_PRIM_MOVING_SPHERE) f |= F_MOVING;
    if ((t >= RT_PRIM_RECT_XY && t <= RT_PRIM_RECT_YZ) || t == RT_PRIM_BOX) f |= F_RECT;
    if (t == RT_PRIM_TRIANGLE) f |= F_TRI;
  }
  for (int k = 0; k < s->n_objects; ++k) {
    const int t = s->objects[k].kind;
    if (t == RT_OBJ_LIST) f |= F_LIST;
    if (t == RT_OBJ_BVH) f |= F_BVH;
    if (t == RT_OBJ_XFORM) f |= F_XFORM;
    if (t == RT_OBJ_MEDIUM) f |= F_MEDIUM;
  }
  for (int k = 0; k < s->n_textures; ++k) {
    const int t = s->textures[k].type;
    if (t == RT_TEX_CHECKER) f |= F_CHECKER;
    if (t == RT_TEX_NOISE || t == RT_TEX_TURBULENT || t == RT_TEX_MARBLE) f |= F_NOISE;
    if (t == RT_TEX_IMAGE) f |= F_IMAGE;
  }
  return f;
}

int fail(rt_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}
#define HIPCHK(ctx, call)                                                                          \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess) return fail(ctx, RT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

template <class T>
int upload(rt_ctx* c, const T* src, size_t n, const T** dst) {
  *dst = nullptr;
  if (n == 0) return RT_OK;
  void* p = nullptr;
  HIPCHK(c, hipMalloc(&p, n * sizeof(T)));
  c->scene_bufs.push_back(p);
  HIPCHK(c, hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice));
  *dst = (const T*)p;
  return RT_OK;
}

void free_scene(rt_ctx* c) {
  for (void* p : c->scene_bufs) (void)hipFree(p);
  c->scene_bufs.clear();
  c->have_scene = false;
}

bool tex_needs_uv(const rt_scene_soa* s, int ti) {
  if (ti < 0 || ti >= s->n_textures) return false;
  const rt_texture& t = s->textures[ti];
  if (t.type == RT_TEX_IMAGE) return true;
  if (t.type == RT_TEX_CHECKER) {
    for (int c : {t.a, t.b})
      if (c >= 0 && c < s->n_textures && s->textures[c].type == RT_TEX_IMAGE) return true;
  }
  return false;
}

// Traversal tree of a reference BVH (see bvh_closest): a binary SAH tree over the same
// primitives, one primitive per leaf, child boxes stored in the parent (padded by 2^-16 relative
// so a primitive hit is never outside its padded ancestors).  Record i = 2 rt_bvh_node slots at
// nodes[fb + 2i]: {lo0, child0}, {hi0, child1}, {lo1, -}, {hi1, -}; child >= 0 is a record,
// child < 0 the primitive -child-1.  Also writes each primitive's reference leaf rank (its
// position in the reference's depth-first left-first order) into prims[].p[9].
// Returns the first node index of the new tree in `nodes`, or -1 if the reference tree is malformed.
struct SahBuilder {
  const std::vector<rth::Box>& box;
  std::vector<rt_bvh_node>& nodes;
  int fb;
  static float area(const rth::Box& b) {
    const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    return dx < 0.0f ? 0.0f : 2.0f * (dx * dy + dy * dz + dz * dx);
  }
  static rth::Box pad(rth::Box b) {
    for (int a = 0; a < 3; ++a) {
      const float p = (std::max(std::fabs(b.lo[a]), std::fabs(b.hi[a])) + (b.hi[a] - b.lo[a])) * (1.0f / 65536.0f);
      b.lo[a] -= p;
      b.hi[a] += p;
    }
    return b;
  }
  rth::Box bounds(const int* ids, int n) const {
    rth::Box b = box[ids[0]];
    for (int i = 1; i < n; ++i) b = rth::join(b, box[ids[i]]);
    return b;
  }
  // Builds the subtree over ids[0..n) (n >= 2) as record `me`; returns nothing.
  void build(int* ids, int n, int me) {
    float best = INFINITY;
    int bax = 0, bsplit = n / 2;
    std::vector<float> right(n + 1);
    for (int ax = 0; ax < 3; ++ax) {
      auto key = [&](int id) { return box[id].lo[ax] + box[id].hi[ax]; };
      std::stable_sort(ids, ids + n, [&](int x, int y) { return key(x) < key(y); });
      rth::Box acc = box[ids[n - 1]];
      for (int i = n - 1; i >= 1; --i) {
        if (i < n - 1) acc = rth::join(acc, box[ids[i]]);
        right[i] = area(acc) * (float)(n - i);
      }
      rth::Box lacc = box[ids[0]];
      for (int i = 1; i < n; ++i) {
        if (i > 1) lacc = rth::join(lacc, box[ids[i - 1]]);
        const float cost = area(lacc) * (float)i + right[i];
        if (cost < best) {
          best = cost;
          bax = ax;
          bsplit = i;
        }
      }
    }
    auto key = [&](int id) { return box[id].lo[bax] + box[id].hi[bax]; };
    std::stable_sort(ids, ids + n, [&](int x, int y) { return key(x) < key(y); });
    int child[2];
    rth::Box cb[2];
    const int part[2][2] = {{0, bsplit}, {bsplit, n}};
    for (int c = 0; c < 2; ++c) {
      const int* cid = ids + part[c][0];
      const int cn = part[c][1] - part[c][0];
      cb[c] = pad(bounds(cid, cn));
      if (cn == 1) {
        child[c] = -cid[0] - 1;
      } else {
        child[c] = (int)(nodes.size() - fb) / 2;
        nodes.resize(nodes.size() + 2);
      }
    }
    rt_bvh_node* r = &nodes[fb + 2 * me];
    for (int a = 0; a < 3; ++a) {
      r[0].lo[a] = cb[0].lo[a];
      r[0].hi[a] = cb[0].hi[a];
      r[1].lo[a] = cb[1].lo[a];
      r[1].hi[a] = cb[1].hi[a];
    }
    r[0].leaf_a = child[0];
    r[0].leaf_b = child[1];
    r[1].leaf_a = 0;
    r[1].leaf_b = 0;
    for (int c = 0; c < 2; ++c)
      if (child[c] >= 0) build(ids + part[c][0], part[c][1] - part[c][0], child[c]);
  }
};

int build_traversal_tree(const rt_scene_soa* s, int base, int rows, std::vector<rt_prim>& prims,
                         std::vector<rt_bvh_node>& nodes, std::vector<float2>& pmargin, std::vector<float4>& pvalid,
                         int* n_pairs, bool dedup) {
  const int inner = (1 << rows) - 1, last0 = (1 << (rows - 1)) - 1;
  std::vector<int> members;
  for (int k = last0; k < inner; ++k) {
    const rt_bvh_node& nd = s->nodes[base + k];
    const int ids[2] = {nd.leaf_a, nd.leaf_b};
    for (int q = 0; q < 2; ++q) {
      if (ids[q] < 0) continue;
      if (ids[q] >= s->n_prims) return -1;
      const int32_t rank = 2 * (k - last0) + q;
      memcpy(&prims[ids[q]].p[9], &rank, 4);
      members.push_back(ids[q]);
    }
  }
  const int n = (int)members.size();
  if (n < 2 || n > (1 << rows)) return -1;
  const float t0 = s->camera.time0, t1 = s->camera.time1;
  std::vector<rth::Box> box(s->n_prims);
  for (int id : members) box[id] = rth::prim_box(prims[id], s->triangles, t0 < t1 ? t0 : t1, t0 < t1 ? t1 : t0);
  // Safety margins of each primitive's reference chain: margin of chain position j = smallest
  // distance from the primitive's box (over the camera shutter) to the faces of its j-th
  // reference ancestor (position 0 = its last-row node).  Stored as {bitmask of positions with
  // margin < 0.05 (always tested), smallest margin of the other positions}.
  for (int k = last0; k < inner; ++k) {
    const rt_bvh_node& nd = s->nodes[base + k];
    for (int id : {nd.leaf_a, nd.leaf_b}) {
      if (id < 0) continue;
      uint32_t mask = 0;
      float safe = INFINITY;
      int pos = 0;
      for (int a = k;; a = (a - 1) >> 1, ++pos) {
        const rt_bvh_node& an = s->nodes[base + a];
        float mm = INFINITY;
        for (int q = 0; q < 3; ++q) mm = std::min(mm, std::min(box[id].lo[q] - an.lo[q], an.hi[q] - box[id].hi[q]));
        if (!(mm >= 0.05f)) mask |= 1u << pos;
        else safe = std::min(safe, mm);
        if (a == 0) break;
      }
      float mbits;
      memcpy(&mbits, &mask, 4);
      pmargin[id] = make_float2(mbits, safe);
      // chain_ok's one-fetch record: the lowest `must` position's box, the mask, `safe`, and the largest
      // |coordinate| over the `must` ancestors' boxes.  Only when every `must` ancestor contains the
      // lowest one's box (the reference's surrounding boxes always do); else safe = -inf turns it off.
      int low = k;  // node of the lowest must position
      for (int q = 0; mask != 0u && q < __builtin_ctz(mask); ++q) low = (low - 1) >> 1;
      const rt_bvh_node& ln = s->nodes[base + low];
      float rmax = 0.0f, vsafe = safe;
      pos = 0;
      for (int a = k;; a = (a - 1) >> 1, ++pos) {
        if ((mask >> pos) & 1u) {
          const rt_bvh_node& an = s->nodes[base + a];
          for (int q = 0; q < 3; ++q) {
            rmax = std::fmax(rmax, std::fmax(std::fabs(an.lo[q]), std::fabs(an.hi[q])));
            if (!(an.lo[q] <= ln.lo[q] && an.hi[q] >= ln.hi[q])) vsafe = -INFINITY;
          }
        }
        if (a == 0) break;
      }
      if (!(rmax < INFINITY)) vsafe = -INFINITY;
      pvalid[3 * (size_t)id] = make_float4(ln.lo[0], ln.lo[1], ln.lo[2], mbits);
      pvalid[3 * (size_t)id + 1] = make_float4(ln.hi[0], ln.hi[1], ln.hi[2], vsafe);
      pvalid[3 * (size_t)id + 2] = make_float4(rmax, 0.0f, 0.0f, 0.0f);
    }
  }
  // Coincident triangles (the reference's mesh import indexes the concatenated vertex array with
  // per-mesh local indices, H16: 1 828 of the door's 4 330 triangles repeat an earlier one's v0, e0,
  // e1 bit for bit) hit every ray at the same t, so among them the reference keeps the first it
  // visits in its depth-first left-first order: the lowest leaf rank whose chain passes.  The
  // candidate search only needs that member; members are in rank order, so the first of each group
  // stays in the tree.  The settle validates the kept member's chain; if it fails the query re-runs
  // on the exact visit set, where a later member may win (options.dedup_triangles = 0 keeps every member).
  std::vector<int> kept;
  if (dedup) {
    std::set<std::array<uint32_t, 9>> seen;
    for (int id : members) {
      if ((prims[id].type & 0xff) == RT_PRIM_TRIANGLE) {
        const int ti = (int)prims[id].p[0];
        if (ti < 0 || ti >= s->n_triangles) return -1;
        const rt_triangle& t = s->triangles[ti];
        std::array<uint32_t, 9> key;
        memcpy(&key[0], t.v0, 12);
        memcpy(&key[3], t.e0, 12);
        memcpy(&key[6], t.e1, 12);
        if (!seen.insert(key).second) continue;
      }
      kept.push_back(id);
    }
  }
  std::vector<int>& leaves = kept.size() >= 2 ? kept : members;
  const int fb = (int)nodes.size();
  nodes.resize(fb + 2);  // record 0 = root
  SahBuilder sb{box, nodes, fb};
  sb.build(leaves.data(), (int)leaves.size(), 0);
  *n_pairs = (int)leaves.size() - 1;  // records of the tree (one per inner node): leaves - 1
  return fb;
}

// REF camera mode (H2): each pixel draws its lens offset and time from a private copy of the
// pristine slot-0 state curand_init(seed, 0, 0), restarted per item, so sample s of every pixel
// uses the same draws: in_unit_disk (vec3.h:136-142, left-to-right H9) scaled by lens_radius,
// offset = rd.x u + rd.y v, time = time0 + (time1 - time0) U (camera.h:49-58).  Same float
// operations as the device path (-ffp-contract=off on both sides), so the rays are bit-identical.
// states (optional): the camera RNG state at each sample's start, 2 uint4 per sample as the
// step kernel loads them (d v0 v1 v2 | v3 v4 - -).
void camera_table(const rt_camera& C, uint64_t seed, int spp, std::vector<float4>& out,
                  std::vector<uint4>* states = nullptr) {
  rtx::State cr = rtx::seed_state(seed);
  out.resize((size_t)spp);
  if (states) states->resize(2 * (size_t)spp);
  for (int s = 0; s < spp; ++s) {
    if (states) {
      (*states)[2 * (size_t)s] = make_uint4(cr.d, cr.v[0], cr.v[1], cr.v[2]);
      (*states)[2 * (size_t)s + 1] = make_uint4(cr.v[3], cr.v[4], 0u, 0u);
    }
    float a, b;
    bool inside;
    do {
      a = -1.0f + (1.0f - -1.0f) * rtx::uniform(cr);
      b = -1.0f + (1.0f - -1.0f) * rtx::uniform(cr);
      inside = a * a + b * b + 0.0f * 0.0f < 1.0f;
    } while (!inside);
    const float rx = C.lens_radius * a, ry = C.lens_radius * b;
    const float ox = rx * C.u[0] + ry * C.v[0], oy = rx * C.u[1] + ry * C.v[1], oz = rx * C.u[2] + ry * C.v[2];
    const float tm = C.time0 + (C.time1 - C.time0) * rtx::uniform(cr);
    out[(size_t)s] = make_float4(ox, oy, oz, tm);
  }
}

// Stable descending counting sort of n one-byte keys on the context's stream (order_*_kernel):
// sort_keys returns the scratch key array to fill; sort_hist leaves the per-tile offsets in scratch
// and returns the 256 key totals on the host; sort_scatter writes out[base[v] + rank] = k for every
// key v (base: device array of 256, the caller's layout).
constexpr int kOrderTabWords = 256 + 2 * kOrderKeys + 256;  // base, sub_ge, rest_gt, key totals
uint8_t* sort_keys(rt_ctx* c, long long n) {
  const long long tiles = (n + kOrderTile - 1) / kOrderTile;
  const long long need = ((n + 255) & ~255LL) + tiles * 256 * 4;
  if (need > c->sort_scratch_cap) {
    if (c->sort_scratch) (void)hipFree(c->sort_scratch);
    c->sort_scratch = nullptr;
    c->sort_scratch_cap = 0;
    if (hipMalloc((void**)&c->sort_scratch, (size_t)need) != hipSuccess) return nullptr;
    c->sort_scratch_cap = need;
  }
  if (!c->order_tab && hipMalloc((void**)&c->order_tab, kOrderTabWords * sizeof(unsigned)) != hipSuccess) return nullptr;
  return c->sort_scratch;
}
int sort_hist(rt_ctx* c, long long n, unsigned hist[256]) {
  const unsigned tiles = (unsigned)((n + kOrderTile - 1) / kOrderTile);
  unsigned* tile_tab = (unsigned*)(c->sort_scratch + ((n + 255) & ~255LL));
  unsigned* totals = c->order_tab + 256 + 2 * kOrderKeys;
  order_tile_hist_kernel<<<tiles, 64, 0, c->stream>>>(c->sort_scratch, (unsigned long long)n, tile_tab);
  HIPCHK(c, hipGetLastError());
  order_scan_kernel<<<256, 256, 0, c->stream>>>(tile_tab, tiles, totals);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(hist, totals, 256 * sizeof(unsigned), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return RT_OK;
}
int sort_scatter(rt_ctx* c, long long n, const unsigned* base, uint32_t* out) {
  const unsigned tiles = (unsigned)((n + kOrderTile - 1) / kOrderTile);
  const unsigned* tile_tab = (const unsigned*)(c->sort_scratch + ((n + 255) & ~255LL));
  order_scatter_kernel<<<tiles, 64, 0, c->stream>>>(c->sort_scratch, (unsigned long long)n, tile_tab, base, out);
  HIPCHK(c, hipGetLastError());
  return RT_OK;
}

// Mean of the probe counts within kProbeRadius grid points (rows and pixels, clipped at the edges), in
// 1/16 segment: one sample's count is a noisy estimate of a pixel's cost, a neighbourhood's mean is a
// steadier one.
// Measured (MI355X, one GPU rendering each rank's share, first launches, median of 3; probe of every
// pixel), cold share ms at N = 4 / 8: C2 10 x 10 no probe 5.87 / 4.17, radius 0 7.02 / 5.10, 2 5.64 /
// 4.02, 5 5.65 / 4.12; C4 no probe 32.86 / 26.70, radius 0 28.14 / 27.87, 2 27.49 / 27.08, 5 25.58 /
// 25.12 (profiles/r05/probe/psc_*.txt).
constexpr int kProbeRadius = 5;
__global__ __launch_bounds__(kBlock) void probe_smooth_kernel(const uint16_t* __restrict__ raw,
                                                              uint16_t* __restrict__ out, int prow, int pw) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (k >= (long long)prow * pw) return;
  const int q = (int)(k / pw), i = (int)(k - (long long)q * pw);
  unsigned sum = 0, n = 0;
  for (int dq = -kProbeRadius; dq <= kProbeRadius; ++dq) {
    const int qq = q + dq;
    if (qq < 0 || qq >= prow) continue;
    for (int di = -kProbeRadius; di <= kProbeRadius; ++di) {
      const int ii = i + di;
      if (ii < 0 || ii >= pw) continue;
      sum += raw[(long long)qq * pw + ii];
      ++n;
    }
  }
  out[k] = (uint16_t)((16 * sum + n / 2) / n);
}

// Sort key of every item from the probe: the smoothed probe count (1/16 segment) of its grid point (sample
// 0 of the first fb at row position ps * (q / ps), pixel ps * (i / ps)) times spp, in cost buckets of
// 2^shift segments, clamped to 255.  Items are row-major with the fb inside the row (render kernels); the
// probe launch's items are the grid's (row position, pixel) points.
__global__ __launch_bounds__(kBlock) void probe_keys_kernel(const uint16_t* __restrict__ probe, uint8_t* __restrict__ key,
                                                            unsigned long long items, int W, int fbc, int spp, int ps,
                                                            int pw, int shift) {
  const unsigned long long per_row = (unsigned long long)fbc * (unsigned)W;
  for (unsigned long long k = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; k < items;
       k += (unsigned long long)gridDim.x * blockDim.x) {
    const unsigned long long q = k / per_row, i = (k - q * per_row) % (unsigned)W;
    const unsigned long long v = (unsigned long long)probe[(q / (unsigned)ps) * (unsigned)pw + i / (unsigned)ps] * spp;
    key[k] = (uint8_t)min(255ull, v >> (4 + shift));
  }
}
// Bases of a descending counting sort from its key totals: base[v] = keys above v (one lane: 256 adds).
__global__ __launch_bounds__(64) void key_base_kernel(const unsigned* __restrict__ total, unsigned* __restrict__ base) {
  if (threadIdx.x != 0) return;
  unsigned acc = 0;
  for (int v = 255; v >= 0; --v) {
    base[v] = acc;
    acc += total[v];
  }
}

// Item schedule of a configuration from its measuring launch's per-item segment counts (c->item_cost,
// `segs` segments in all): perm, the long prefix and the split items.  Built when the configuration
// is rendered again, so a single draw() does not pay the host sort.
int build_schedule(rt_ctx* c, long long items, int spp, unsigned long long segs, bool step_kernel) {
  RT_DIAG_ITEM_COSTS(c, items);  // diagnostic builds only (rt_diag.h): per-item segment counts to a file
  // Every item in descending cost buckets of 8 segments, the natural (spatially coherent) order
  // inside a bucket (a stable counting sort on the device; the top bucket 255 holds every item of
  // >= 2040 segments); the top ~2 % by cost are the "long" prefix whose waves run at raised
  // priority.  (C2, one GPU as rank 0 of N: N = 8 share 3.89 -> 3.45 ms, N = 1 unchanged.)
  // Buckets of 8 segments unless the longest item would saturate the top bucket (>= 2040 segments:
  // high spp); then wider buckets, so the longest items stay ordered and splittable.
  uint8_t* keys = sort_keys(c, items);
  if (!keys) return fail(c, RT_ERR_HIP, "out of device memory (schedule sort)");
  unsigned cmax = 0;
  {
    unsigned* dmax = c->order_tab + 256 + 2 * kOrderKeys;  // key-total words, free until sort_hist
    HIPCHK(c, hipMemsetAsync(dmax, 0, sizeof(unsigned), c->stream));
    cost_max_kernel<<<(unsigned)std::min<long long>(1024, (items + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(
        c->item_cost, (unsigned long long)items, dmax);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(&cmax, dmax, sizeof(unsigned), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  // (render_kernel: exact counts, buckets of one segment, the longest quarter of the range saturating the
  // top bucket.  Its waves refill once 4 lanes are idle, and items of equal cost in a wave end together:
  // C5 warm 55.0 -> 51.8 ms per launch at N = 1, 7.86 -> 6.96 at N = 8 (profiles/r06/cost_shift/); the
  // stepwise kernel, which refills every idle lane, keeps buckets of 8)
  int shift = step_kernel ? 3 : 0;
  while (shift < 8 && (cmax >> shift) > (step_kernel ? 255u : 1023u)) ++shift;
  if (c->opt.cost_shift >= 0) shift = std::min(12, c->opt.cost_shift);  // tuning
  cost_key_kernel<<<(unsigned)((items + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(
      c->item_cost, (unsigned long long)items, shift, keys);
  HIPCHK(c, hipGetLastError());
  unsigned h[256];
  if (int rc = sort_hist(c, items, h)) return rc;
  std::vector<long long> hist(256);
  for (int v = 0; v < 256; ++v) hist[(size_t)v] = h[v];
  unsigned base[256];
  {
    unsigned acc = 0;
    for (int v = 255; v >= 0; --v) {
      base[v] = acc;
      acc += h[v];
    }
  }
  HIPCHK(c, hipMemcpyAsync(c->order_tab, base, sizeof(base), hipMemcpyHostToDevice, c->stream));
  if (int rc = sort_scatter(c, items, c->order_tab, c->perm)) return rc;
  // completed before returning (base is on this stack): the next launch (same stream) reads perm
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const double pct = c->opt.long_pct;
  const long long want = (long long)((double)items * pct / 100.0);
  long long nl = 0;  // whole buckets from the top while they fit in `want`
  for (int v = 255; v >= 0 && nl + hist[(size_t)v] <= want; --v) nl += hist[(size_t)v];
  c->n_long = (unsigned long long)nl;
  // Items that can decide when a launch ends have their samples split on later launches: the
  // items at or above a threshold set by the share's size (below).  They are the first positions
  // of perm (cost buckets descending).  (Round 2, samples still claimed in item order: C2's N = 8
  // share 3.59 -> 2.88 ms.)
  {
    // lanes of the stepwise kernel that runs the split launches (4 waves/SIMD: 1024 per CU),
    // whatever variant measured (bench.py measures with the counting variant)
    const double lanes = (double)c->cus * 1024.0;
    // Split launches claim everything longest first (RenderParams::order), so an unsplit item
    // only needs to be short against a lane's share; every split costs claims and state loads, and
    // a sky pixel (one segment per sample) gains nothing from it.  Measured, C2 warm by threshold
    // (camera lists on), 10 x 10: N = 8 (4.6 items and 117 segments per lane) 24: 2.53, 32: 2.34,
    // 48: 2.62 ms; N = 4 (9.2, 231) 24: 4.82, 32: 4.43, 48: 4.55, 115: 4.72; N = 2 (18, 462) 32:
    // 8.54, 48: 8.39, 231: 8.57; N = 1 (36, 925) 48: 16.56, 462: 16.53.  1 x 100: N = 8 85: 3.08,
    // 100: 2.81, 120: 2.79; N = 4 100: 5.39, 150: 5.28, 200: 5.31, 250: 6.27; N = 2 200: 10.93,
    // 300: 9.09, 400: 11.32; N = 1 200: 21.59, 300: 16.69, 400: 18.44.
    // Round 5: the 48-segment band reaches up to 48 items per lane (was 24).  C4 (door 1920x1079,
    // 16 x 16) as rank of N = 4 has 31.7 items per lane, and "half a lane's share" (~574 segments)
    // split almost nothing: its warm share ran 27.9 ms against an ideal 20; at 48 segments 20.7 ms
    // (N = 1 / 2 / 8 unchanged within 1 %).  C2's only case in the new band, N = 1 (36 per lane),
    // measured the same at 48 and 462 in round 3.
    const double share = (double)segs / lanes, per_lane = (double)items / lanes;
    double thr = spp <= 16 ? (per_lane < 6.0 ? 32.0 : per_lane < 48.0 ? 48.0 : std::max(32.0, 0.5 * share))
                           : std::min(3.0 * spp, std::max(1.04 * spp, 0.85 * share));
    if (c->opt.split_min_segments > 0.0f) thr = c->opt.split_min_segments;  // tuning, tests
    const long long bt = (long long)std::ceil(thr / (double)(1 << shift));
    long long ns = 0;
    for (long long v = 255; v >= bt && v >= 0; --v) ns += hist[(size_t)v];  // bt > 255: no split
    if (ns * (long long)spp >= (1LL << 30)) ns = 0;
    c->n_split = (unsigned long long)ns;
    c->split_state = ns > 0 ? 0 : -1;
    c->order_ok = false;
    c->rest_n = items - ns;
    c->rest_gt.assign(kOrderKeys, 0u);
    for (long long b = 0; b < bt && b < 256; ++b) {  // the unsplit buckets
      const long long key = std::min(256LL, (b << shift) + ((1LL << shift) >> 1));
      for (long long v = 0; v < key; ++v) c->rest_gt[(size_t)v] += (unsigned)hist[(size_t)b];
    }
  }
  return RT_OK;
}

// Position k < 64 * nw of chunk c = k / 64, lane l = k % 64 takes rank l * nw + c of the head (a copy of
// perm's first 64 * nw entries) for l < top, else rank top * nw + c * (64 - top) + l - top: the chunk of 64
// positions a wave claims first holds `top` items strided over the head's first top * nw ranks and
// 64 - top consecutive ones (neighbours in the order, spatially coherent inside a cost bucket).
__global__ __launch_bounds__(kBlock) void spread_head_kernel(const uint32_t* __restrict__ head, uint32_t* __restrict__ perm,
                                                             unsigned long long nw, unsigned top) {
  for (unsigned long long k = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; k < 64ull * nw;
       k += (unsigned long long)gridDim.x * blockDim.x) {
    const unsigned long long c = k >> 6, l = k & 63ull;
    perm[k] = head[l < top ? l * nw + c : top * nw + c * (64ull - top) + l - top];
  }
}

// Item schedule of a probe-scheduled first launch from the smoothed probe grid (c->probe_cost + pitems):
// every step on the device, no host round trip (the draw's critical path): per-item keys, the tile
// histograms and their scan, the bases, the stable scatter into perm.  The long prefix is the first
// long_pct % of the positions.  Cost buckets of 8 segments, as the measured schedule's (natural order
// inside a bucket keeps neighbouring claims coherent), wider where smoothed means of up to 32 segments
// per sample would saturate the top bucket (a grid point above that, rare, saturates it).
int probe_schedule(rt_ctx* c, long long items, int spp, int width, int fbc, int ps, int pw, long long pitems,
                   bool step_kernel, long long waves, int spread_top) {
  uint8_t* keys = sort_keys(c, items);
  if (!keys) return fail(c, RT_ERR_HIP, "out of device memory (probe schedule)");
  // (render_kernel: buckets of 2 segments.  C5 first launches at N = 1 / 2 / 4 / 8, buckets of 8 / 4 / 2 /
  // 1: 63.2 / 63.1 / 63.0 / 64.4 ms, 35.9 / 33.8 / 34.0 / 34.4, 22.1 / 20.4 / 20.2 / 20.3, 14.8 / 15.2 /
  // 14.5 / 14.4; profiles/r06/cost_shift/)
  int shift = step_kernel ? 3 : 1;
  while (shift < 12 && ((32LL * spp) >> shift) > 255) ++shift;
  if (c->opt.cost_shift >= 0) shift = c->opt.cost_shift;  // tuning
  probe_keys_kernel<<<(unsigned)std::min<long long>(4096, (items + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(
      c->probe_cost + pitems, keys, (unsigned long long)items, width, fbc, spp, ps, pw, shift);
  HIPCHK(c, hipGetLastError());
  const unsigned tiles = (unsigned)((items + kOrderTile - 1) / kOrderTile);
  unsigned* tile_tab = (unsigned*)(c->sort_scratch + ((items + 255) & ~255LL));
  unsigned* totals = c->order_tab + 256 + 2 * kOrderKeys;
  order_tile_hist_kernel<<<tiles, 64, 0, c->stream>>>(keys, (unsigned long long)items, tile_tab);
  HIPCHK(c, hipGetLastError());
  order_scan_kernel<<<256, 256, 0, c->stream>>>(tile_tab, tiles, totals);
  HIPCHK(c, hipGetLastError());
  key_base_kernel<<<1, 64, 0, c->stream>>>(totals, c->order_tab);
  HIPCHK(c, hipGetLastError());
  if (int rc = sort_scatter(c, items, c->order_tab, c->perm)) return rc;
  c->n_long = (unsigned long long)((double)items * c->opt.long_pct / 100.0);
  // Spread head (spread_top > 0, options.spread_first): longest first, the first claims would hand the
  // estimated-longest items 64 to a wave to the waves that claim first (one workgroup's); strided, every
  // wave starts with spread_top of the head's first spread_top * waves items
  const int sf = spread_top;
  if (sf > 0 && waves > 0 && items >= 64 * waves) {
    const long long n = 64 * waves;
    if (n > c->spread_cap) {
      if (c->spread_tmp) HIPCHK(c, hipFree(c->spread_tmp));
      c->spread_tmp = nullptr;
      c->spread_cap = 0;
      HIPCHK(c, hipMalloc((void**)&c->spread_tmp, (size_t)n * sizeof(uint32_t)));
      c->spread_cap = n;
    }
    HIPCHK(c, hipMemcpyAsync(c->spread_tmp, c->perm, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToDevice, c->stream));
    spread_head_kernel<<<(unsigned)std::min<long long>(4096, (n + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(
        c->spread_tmp, c->perm, (unsigned long long)waves, (unsigned)sf);
    HIPCHK(c, hipGetLastError());
  }
  return RT_OK;
}

int validate_args(rt_ctx* c, const rt_render_args* a) {
  if (!a) return fail(c, RT_ERR_ARG, "null args");
  if (a->width <= 0 || a->height <= 0 || a->spp <= 0 || a->fb_count <= 0 || a->fb_first < 0 || a->max_depth <= 0)
    return fail(c, RT_ERR_ARG, "bad render args");
  if (a->band_rows <= 0 || a->band_stride <= 0 || a->band_first < 0 || a->band_first >= a->band_stride)
    return fail(c, RT_ERR_ARG, "bad band tiling");
  if (a->cam_mode != RT_CAM_REF_SLOT0 && a->cam_mode != RT_CAM_PER_PIXEL) return fail(c, RT_ERR_ARG, "bad cam_mode");
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_ctx_create(int hip_device, rt_ctx** out) {
  if (!out) return RT_ERR_ARG;
  *out = nullptr;
  rt_ctx* c = new rt_ctx;
  c->device = hip_device;
  rt_ctx_options_default(&c->opt);
  int rc = RT_OK;
  auto chk = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && rc == RT_OK) rc = fail(c, RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  };
  chk(hipSetDevice(hip_device), "hipSetDevice");
  if (rc == RT_OK) chk(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
  if (rc == RT_OK) chk(hipEventCreate(&c->ev0), "hipEventCreate");
  if (rc == RT_OK) chk(hipEventCreate(&c->ev1), "hipEventCreate");
  if (rc == RT_OK) chk(hipEventCreate(&c->ev2), "hipEventCreate");
  if (rc == RT_OK) chk(hipMalloc((void**)&c->work, 8 * sizeof(unsigned long long)), "hipMalloc");
  if (rc == RT_OK) {
    std::vector<uint32_t> seq(32 * 800);
    rtx::build_sequence_jumps(seq.data());
    chk(hipMalloc((void**)&c->seq, seq.size() * 4), "hipMalloc");
    if (rc == RT_OK) chk(hipMemcpy(c->seq, seq.data(), seq.size() * 4, hipMemcpyHostToDevice), "hipMemcpy");
    // byte tables of M^d for the 32 digit positions M = seq[i], d = 1..3
    std::vector<uint32_t> tab((size_t)96 * kTabMat, 0u);
    std::vector<uint32_t> m2(800), m3(800);
    for (int i = 0; i < 32 && rc == RT_OK; ++i) {
      const uint32_t* m1 = seq.data() + 800 * i;
      for (int col = 0; col < 160; ++col) rtx::mat_apply(m1, m1 + 5 * col, m2.data() + 5 * col);  // M^2
      for (int col = 0; col < 160; ++col) rtx::mat_apply(m1, m2.data() + 5 * col, m3.data() + 5 * col);  // M^3
      const uint32_t* ms[3] = {m1, m2.data(), m3.data()};
      for (int d = 0; d < 3; ++d) {
        uint32_t* t = tab.data() + (size_t)(d * 32 + i) * kTabMat;
        for (int b = 0; b < 20; ++b)
          for (int v = 0; v < 256; ++v)
            for (int j = 0; j < 8; ++j)
              if ((v >> j) & 1)
                for (int k = 0; k < 5; ++k) t[(b * 256 + v) * kTabRow + k] ^= ms[d][5 * (8 * b + j) + k];
      }
    }
    if (rc == RT_OK) chk(hipMalloc((void**)&c->jump_tab, tab.size() * 4), "hipMalloc");
    if (rc == RT_OK) chk(hipMemcpy(c->jump_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice), "hipMemcpy");
  }
  if (rc == RT_OK) {
    hipDeviceProp_t prop;
    chk(hipGetDeviceProperties(&prop, hip_device), "hipGetDeviceProperties");
    c->cus = prop.multiProcessorCount;
    for (int v = 0; v < kNumVariants; ++v)
      chk(hipOccupancyMaxActiveBlocksPerMultiprocessor(&c->blocks_per_cu[v], kVariants[v].fn, variant_block(v),
                                                       (kVariants[v].mask & (F_LDS | F_QLDS)) ? kLdsBudget
                                                                                   : variant_block(v) * (stack_words(kVariants[v].mask) + locker_words(kVariants[v].mask)) * 4),
          "occupancy");
  }
  if (rc != RT_OK) {
    fprintf(stderr, "rt_ctx_create: %s\n", c->err.c_str());
    rt_ctx_destroy(c);
    return rc;
  }
  *out = c;
  return RT_OK;
}

int rt_ctx_destroy(rt_ctx* c) {
  if (!c) return RT_OK;
  (void)hipSetDevice(c->device);
  free_scene(c);
  if (c->states) (void)hipFree(c->states);
  if (c->seq) (void)hipFree(c->seq);
  if (c->jump_tab) (void)hipFree(c->jump_tab);
  if (c->work) (void)hipFree(c->work);
  if (c->row_map) (void)hipFree(c->row_map);
  if (c->row_cost) (void)hipFree(c->row_cost);
  if (c->item_cost) (void)hipFree(c->item_cost);
  if (c->probe_cost) (void)hipFree(c->probe_cost);
  if (c->spread_tmp) (void)hipFree(c->spread_tmp);
  if (c->perm) (void)hipFree(c->perm);
  if (c->dbg) (void)hipFree(c->dbg);
  if (c->tiles) (void)hipFree(c->tiles);
  if (c->cam_tab) (void)hipFree(c->cam_tab);
  if (c->ckpt) (void)hipFree(c->ckpt);
  if (c->order) (void)hipFree(c->order);
  if (c->order_tab) (void)hipFree(c->order_tab);
  if (c->sort_scratch) (void)hipFree(c->sort_scratch);
  if (c->contrib) (void)hipFree(c->contrib);
  if (c->cam_st) (void)hipFree(c->cam_st);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev2) (void)hipEventDestroy(c->ev2);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return RT_OK;
}

const char* rt_last_error(const rt_ctx* c) { return c ? c->err.c_str() : "null context"; }

void rt_ctx_options_default(rt_ctx_options* o) {
  if (!o) return;
  *o = rt_ctx_options{};
  o->world_tree = 0;
  o->quantized_tree = 1;
  o->merged_search = RT_MERGE_ON;
  o->merge_order = RT_ORDER_DISTANCE;
  o->dedup_triangles = 1;
  o->shade_min = 0;
  o->bins_min_items_per_lane = 6.0f;
  o->split_min_segments = 0.0f;
  o->split_order = 1;
  o->cost_shift = -1;
  o->long_pct = 2.0f;
  o->probe_schedule = -1;
  o->probe_max_items_per_lane = 0.0f;
  o->probe_depth = -1;
  o->spread_first = -1;
}

int rt_ctx_set_options(rt_ctx* c, const rt_ctx_options* o) {
  if (!c || !o) return RT_ERR_ARG;
  if (o->merged_search < RT_MERGE_ON || o->merged_search > RT_MERGE_FALLBACK_ALL ||
      o->merge_order < RT_ORDER_DISTANCE || o->merge_order > RT_ORDER_REVERSED || o->shade_min < 0 ||
      o->shade_min > 64 || !(o->bins_min_items_per_lane >= 0.0f) || !(o->split_min_segments >= 0.0f) ||
      o->cost_shift < -1 || o->cost_shift > 12 || !(o->long_pct >= 0.0f && o->long_pct <= 100.0f) ||
      o->probe_schedule < -1 || o->probe_schedule > 64 || !(o->probe_max_items_per_lane >= 0.0f) ||
      (o->world_tree & ~1) != 0 || (o->quantized_tree & ~1) != 0 || (o->dedup_triangles & ~1) != 0 ||
      (o->split_order & ~1) != 0 || o->probe_depth < -1 || o->spread_first < -1 ||
      o->spread_first > 64)
    return fail(c, RT_ERR_ARG, "bad context options");
  c->opt = *o;
  // the schedule and split thresholds come from the options: every configuration starts cold again
  std::fill(c->perm_key, c->perm_key + rt_ctx::kKey, -1LL);
  std::fill(c->pending_key, c->pending_key + rt_ctx::kKey, -1LL);
  c->split_state = -1;
  c->n_split = 0;
  c->order_ok = false;
  return RT_OK;
}

int rt_ctx_get_options(const rt_ctx* c, rt_ctx_options* o) {
  if (!c || !o) return RT_ERR_ARG;
  *o = c->opt;
  return RT_OK;
}

int32_t rt_owned_rows(const rt_render_args* a, int32_t* rows) {
  if (!a || a->band_rows <= 0 || a->band_stride <= 0) return 0;
  int32_t n = 0;
  for (int32_t b = a->band_first; (int64_t)b * a->band_rows < a->height; b += a->band_stride)
    for (int32_t j = b * a->band_rows; j < (b + 1) * a->band_rows && j < a->height; ++j) {
      if (rows) rows[n] = j;
      ++n;
    }
  return n;
}

// Bounding sphere (centre, radius) of a primitive box, rounded outward so that it contains the box.
float4 box_sphere(const rth::Box& b) {
  const double cx = 0.5 * ((double)b.lo[0] + b.hi[0]), cy = 0.5 * ((double)b.lo[1] + b.hi[1]),
               cz = 0.5 * ((double)b.lo[2] + b.hi[2]);
  const double hx = 0.5 * ((double)b.hi[0] - b.lo[0]), hy = 0.5 * ((double)b.hi[1] - b.lo[1]),
               hz = 0.5 * ((double)b.hi[2] - b.lo[2]);
  const double rad = std::sqrt(hx * hx + hy * hy + hz * hz) * (1.0 + 1e-6) +
                     1e-6 * (std::fabs(cx) + std::fabs(cy) + std::fabs(cz)) + 1e-30;
  return make_float4((float)cx, (float)cy, (float)cz, (float)(rad * (1.0 + 1e-6)));
}
// Geometric box of a primitive over the shutter: bounding_box() (rth::prim_box) except for the
// xz_rect, whose reference box spans z1 only (aarect.h:39, H4) and so does not bound the rect.
rth::Box geom_box(const rt_prim& q, const rt_triangle* tris, float t0, float t1) {
  rth::Box b = rth::prim_box(q, tris, t0, t1);
  if ((q.type & 0xff) == RT_PRIM_RECT_XZ) {
    b.lo[2] = std::fmin(q.p[2], q.p[3]);
    b.hi[2] = std::fmax(q.p[2], q.p[3]);
  }
  return b;
}
// World-space box of a child-frame box cb under instance o (translate(rotate_y(child))).
rth::Box xform_box(const rt_object& o, const rth::Box& cb) {
  // world = R^-1 (object) + offset, R^-1: x = c x' + s z', z = -s x' + c z' (hittable.h:112-143)
  const double sn = (o.b & 2) ? o.f[3] : 0.0, cs = (o.b & 2) ? o.f[4] : 1.0;
  const double off[3] = {(o.b & 1) ? o.f[0] : 0.0, (o.b & 1) ? o.f[1] : 0.0, (o.b & 1) ? o.f[2] : 0.0};
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  for (int q = 0; q < 8; ++q) {
    const double x = (q & 1) ? cb.hi[0] : cb.lo[0], y = (q & 2) ? cb.hi[1] : cb.lo[1], z = (q & 4) ? cb.hi[2] : cb.lo[2];
    const double w[3] = {cs * x + sn * z + off[0], y + off[1], -sn * x + cs * z + off[2]};
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], w[k]);
      hi[k] = std::max(hi[k], w[k]);
    }
  }
  rth::Box out;
  for (int k = 0; k < 3; ++k) {  // widened for the float rounding of the instance transform
    const double pad = 1e-5 * (std::fabs(lo[k]) + std::fabs(hi[k]) + (hi[k] - lo[k])) + 1e-6;
    out.lo[k] = (float)(lo[k] - pad);
    out.hi[k] = (float)(hi[k] + pad);
  }
  return out;
}

// World-space box over the shutter [t0, t1] of object oi (an instance's child box through its
// rotate_y + translate, a medium's boundary); false when it cannot be bounded.
bool object_box(const rt_scene_soa* s, int oi, float t0, float t1, rth::Box& out, int depth = 0) {
  const rt_prim* prims = s->prims;  // the scene's records (the device copies hold triangle operands)
  if (oi < 0 || oi >= s->n_objects || depth > 8) return false;
  const rt_object& o = s->objects[oi];
  auto pbox = [&](int id) { return geom_box(prims[id], s->triangles, t0, t1); };
  switch (o.kind) {
    case RT_OBJ_PRIM:
      out = pbox(o.a);
      return true;
    case RT_OBJ_LIST:
      if (o.b <= 0) return false;
      out = pbox(o.a);
      for (int k = 1; k < o.b; ++k) out = rth::join(out, pbox(o.a + k));
      return true;
    case RT_OBJ_BVH: {
      const int inner = (1 << o.b) - 1, last0 = (1 << (o.b - 1)) - 1;
      bool any = false;
      for (int k = last0; k < inner; ++k)
        for (int id : {s->nodes[o.a + k].leaf_a, s->nodes[o.a + k].leaf_b}) {
          if (id < 0) continue;
          out = any ? rth::join(out, pbox(id)) : pbox(id);
          any = true;
        }
      return any;
    }
    case RT_OBJ_MEDIUM:
      return object_box(s, o.a, t0, t1, out, depth + 1);
    case RT_OBJ_XFORM: {
      rth::Box cb;
      if (!object_box(s, o.a, t0, t1, cb, depth + 1)) return false;
      out = xform_box(o, cb);
      return true;
    }
  }
  return false;
}

// World tree (F_WORLD): a list world (hittable_list.h:23-39) of primitives, BVHs and translate /
// rotate_y instances of them, followed by constant media, flattened into ONE traversal tree over
// every primitive of every non-medium entry (world-space boxes over the shutter; an instance's
// primitives through its transform, padded), so the whole world query is one candidate search in
// render_step_kernel instead of a loop over entries with a traversal per BVH.  Each leaf keeps its
// entry's semantics: it is tested in its instance's frame, its tie key orders exact ties as the list
// does (a later entry wins) and, inside a BVH entry, as bvh.h does (the lower reference leaf rank
// wins), and a BVH member's winner is validated on that BVH's reference chain (world_settle).
// Media must follow every tree entry in the list (they draw from the RNG with the closest hit so far
// as their t_max), except inert ones: a medium bounded by a sphere never reaches its draw (H1: the
// second boundary query returns nothing or t1 itself) unless its boundary root is NaN, which a
// sane ray (ray_sane) cannot produce.  Leaves: 4 float4 each (see DScene::wleaf).
// A constant medium that never reaches its RNG draw for a sane ray (ray_sane): its boundary is a
// sphere with coordinates and radius below 1e6, whose second boundary query repeats the first root
// (H1, sphere.h:51) -- see sphere_boundary_no_hit -- or a moving sphere whose centre c0 + (tm - t0) /
// dt * d stays within 1e6 of c0 for every sane ray time (|tm| < 1024): a tiny shutter span dt would
// let the centre run off to where the boundary root overflows to NaN, and NaN reaches the draw.
static bool medium_inert(const rt_scene_soa* s, const rt_object& o) {
  if (o.kind != RT_OBJ_MEDIUM || o.a < 0 || o.a >= s->n_objects) return false;
  const rt_object& bo = s->objects[o.a];
  if (bo.kind != RT_OBJ_PRIM) return false;
  const rt_prim& q = s->prims[bo.a];
  const int ty = q.type & 0xff;
  if (ty != RT_PRIM_SPHERE && ty != RT_PRIM_MOVING_SPHERE) return false;
  const int np = ty == RT_PRIM_SPHERE ? 4 : 9;
  for (int k = 0; k < np; ++k)
    if (!(std::fabs(q.p[k]) < 1e6f)) return false;
  if (ty == RT_PRIM_SPHERE) return true;
  const double dmax = std::max(std::fabs((double)q.p[4]), std::max(std::fabs((double)q.p[5]), std::fabs((double)q.p[6])));
  return q.p[8] != 0.0f && (1024.0 + std::fabs((double)q.p[7])) / std::fabs((double)q.p[8]) * dmax < 1e6;
}

static bool build_world_tree(const rt_scene_soa* s, const std::vector<rt_prim>& prims, std::vector<rt_bvh_node>& nodes,
                             std::vector<float4>& wleaf, std::vector<float4>& wxf, int& wt_fb, int& w_media,
                             int& w_inert) {
  const int NW = s->n_world;
  if (NW < 2 || NW >= (1 << (31 - RT_WKEY_SHIFT))) return false;
  auto obj = [&](int k) -> const rt_object& { return s->objects[k]; };
  int last_tree = -1;
  for (int w = 0; w < NW; ++w)
    if (obj(s->world[w]).kind != RT_OBJ_MEDIUM) last_tree = w;
  if (last_tree < 0) return false;
  w_inert = 0;
  for (int w = 0; w < NW; ++w) {
    const rt_object& o = obj(s->world[w]);
    if (o.kind == RT_OBJ_MEDIUM) {
      const rt_object& bo = obj(o.a);
      if (w < last_tree) {  // must be inert
        if (!medium_inert(s, o)) return false;
        w_inert = 1;
      } else if (!(bo.kind == RT_OBJ_PRIM || (bo.kind == RT_OBJ_XFORM && obj(bo.a).kind == RT_OBJ_PRIM))) {
        return false;  // active media: primitive boundaries (object_query's direct path)
      }
    } else if (o.kind == RT_OBJ_XFORM) {
      const int ck = obj(o.a).kind;
      if (ck != RT_OBJ_PRIM && ck != RT_OBJ_BVH) return false;
    } else if (o.kind != RT_OBJ_PRIM && o.kind != RT_OBJ_BVH) {
      return false;
    }
  }
  w_media = last_tree + 1;
  struct Leaf {
    int prim, xf, w, bobj, rank;
  };
  std::vector<Leaf> leaves;
  std::vector<rth::Box> box;
  std::vector<int> xf_of(s->n_objects, -1);
  const float t0 = std::fmin(s->camera.time0, s->camera.time1), t1 = std::fmax(s->camera.time0, s->camera.time1);
  for (int w = 0; w < w_media; ++w) {
    int oi = s->world[w];
    if (obj(oi).kind == RT_OBJ_MEDIUM) continue;  // inert
    int xf = -1, xo = -1;
    if (obj(oi).kind == RT_OBJ_XFORM) {
      xo = oi;
      if (xf_of[oi] < 0) {
        const rt_object& o = obj(oi);
        int32_t bits = o.b;
        float fb;
        memcpy(&fb, &bits, 4);
        xf_of[oi] = (int)wxf.size() / 2;
        wxf.push_back(make_float4(o.f[0], o.f[1], o.f[2], fb));
        wxf.push_back(make_float4(o.f[3], o.f[4], 0.0f, 0.0f));
      }
      xf = xf_of[oi];
      oi = obj(oi).a;
    }
    auto add = [&](int pid, int bobj, int rank) {
      rth::Box b = geom_box(s->prims[pid], s->triangles, t0, t1);
      if (xo >= 0) b = xform_box(obj(xo), b);
      leaves.push_back(Leaf{pid, xf, w, bobj, rank});
      box.push_back(b);
    };
    const rt_object& o = obj(oi);
    if (o.kind == RT_OBJ_PRIM) {
      add(o.a, -1, 0);
    } else {  // BVH: its reference leaves, with their ranks in the reference's depth-first order
      if (o.b > RT_WKEY_SHIFT) return false;
      const int inner = (1 << o.b) - 1, last0 = (1 << (o.b - 1)) - 1;
      for (int k = last0; k < inner; ++k) {
        const int ids[2] = {s->nodes[o.a + k].leaf_a, s->nodes[o.a + k].leaf_b};
        for (int q = 0; q < 2; ++q)
          if (ids[q] >= 0) add(ids[q], oi, 2 * (k - last0) + q);
      }
    }
  }
  const int n = (int)leaves.size();
  if (n < 2 || n >= (1 << 24)) return false;
  wleaf.resize(4 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    const Leaf& L = leaves[(size_t)i];
    rt_prim q = prims[(size_t)L.prim];  // the device record: flags, triangle operands
    const int32_t key = ((NW - 1 - L.w) << RT_WKEY_SHIFT) | L.rank;
    memcpy(&q.p[9], &key, 4);
    if (L.xf >= 0) q.type |= RT_PRIM_FLAG_XF;
    memcpy(&wleaf[4 * (size_t)i], &q, sizeof(q));
    const int32_t d[4] = {L.xf, L.w, L.bobj, L.prim};
    memcpy(&wleaf[4 * (size_t)i + 3], d, sizeof(d));
  }
  std::vector<int> ids(n);
  for (int i = 0; i < n; ++i) ids[(size_t)i] = i;
  wt_fb = (int)nodes.size();
  nodes.resize(wt_fb + 2);  // record 0 = root
  SahBuilder sb{box, nodes, wt_fb};
  sb.build(ids.data(), n, 0);
  return true;
}

// Quantized traversal tree (F_QLDS; qpair): the world BVH's traversal-tree pair records, `npairs` of
// them from rt_bvh_node index fb, as 24-byte records that fit LDS next to 16-bit stacks (C4's door:
// 4 329 pairs = 104 KB + 32 KB of stacks, instead of 277 KB in L2).  Per pair and axis: an origin
// rounded down to binary16 below both children, a power-of-two scale 2^E with 255 * 2^E covering the
// pair's extent, and each child's padded box as bytes rounded outward.  False when a value does
// not fit (binary16 range, scales spread over more than 32 octaves, child words beyond 16 bits).
static bool build_qtree(const std::vector<rt_bvh_node>& nodes, int fb, int npairs, std::vector<uint32_t>& out,
                        int& ebias) {
  auto half_down = [](double x, uint16_t& bits) {
    if (!(std::fabs(x) < 60000.0)) return false;
    _Float16 h = (_Float16)(float)x;
    memcpy(&bits, &h, 2);
    while ((double)(float)h > x) {  // step down one binary16 ulp
      bits = (bits & 0x8000u) ? (uint16_t)(bits + 1) : (bits == 0 ? (uint16_t)0x8001u : (uint16_t)(bits - 1));
      memcpy(&h, &bits, 2);
    }
    return true;
  };
  std::vector<int> E((size_t)npairs * 3);
  std::vector<uint16_t> org((size_t)npairs * 3);
  int emax = -1000;
  for (int i = 0; i < npairs; ++i) {
    const rt_bvh_node* r = &nodes[(size_t)fb + 2 * (size_t)i];
    for (int a = 0; a < 3; ++a) {
      const double mn = std::min(r[0].lo[a], r[1].lo[a]), mx = std::max(r[0].hi[a], r[1].hi[a]);
      uint16_t ob;
      if (!half_down(mn, ob) || !(mx >= mn) || !(mx < 60000.0)) return false;
      _Float16 h;
      memcpy(&h, &ob, 2);
      const double ext = mx - (double)(float)h;
      int e = -60;
      while (255.0 * std::ldexp(1.0, e) < ext) ++e;
      org[3 * (size_t)i + a] = ob;
      E[3 * (size_t)i + a] = e;
      emax = std::max(emax, e);
    }
  }
  ebias = emax - 31;  // a scale below 2^ebias is widened to it: coarser, still covering
  if (ebias < -120 || emax > 100) return false;
  out.assign((size_t)npairs * 6, 0u);
  for (int i = 0; i < npairs; ++i) {
    const rt_bvh_node* r = &nodes[(size_t)fb + 2 * (size_t)i];
    uint32_t ee = 0;
    uint8_t q[2][6];
    for (int a = 0; a < 3; ++a) {
      const int e = std::max(E[3 * (size_t)i + a], ebias);
      ee |= (uint32_t)(e - ebias) << (5 * a);
      _Float16 h;
      memcpy(&h, &org[3 * (size_t)i + a], 2);
      const double o = (double)(float)h, sc = std::ldexp(1.0, e);
      for (int ch = 0; ch < 2; ++ch) {
        const double lo = std::floor(((double)r[ch].lo[a] - o) / sc), hi = std::ceil(((double)r[ch].hi[a] - o) / sc);
        if (!(lo >= 0.0 && hi <= 255.0 && lo <= hi)) return false;
        if (!(o + lo * sc <= (double)r[ch].lo[a] && o + hi * sc >= (double)r[ch].hi[a])) return false;
        q[ch][a] = (uint8_t)lo;
        q[ch][3 + a] = (uint8_t)hi;
      }
    }
    const int c0 = r[0].leaf_a, c1 = r[0].leaf_b;
    if (c0 < -32768 || c0 > 32767 || c1 < -32768 || c1 > 32767) return false;
    uint32_t* w = &out[6 * (size_t)i];
    w[0] = (uint32_t)org[3 * (size_t)i] | (uint32_t)org[3 * (size_t)i + 1] << 16;
    w[1] = (uint32_t)org[3 * (size_t)i + 2] | ee << 16;
    const uint8_t b[12] = {q[0][0], q[0][1], q[0][2], q[0][3], q[0][4], q[0][5],
                           q[1][0], q[1][1], q[1][2], q[1][3], q[1][4], q[1][5]};
    memcpy(&w[2], b, 12);
    w[5] = ((uint32_t)c0 & 0xffffu) | ((uint32_t)c1 << 16);
  }
  return true;
}

int rt_scene_upload(rt_ctx* c, const rt_scene_soa* s) {
  if (c) ++c->scene_gen;  // invalidates the row-cost schedule
  if (!c || !s) return RT_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  if (s->n_world <= 0 || !s->world || s->n_objects <= 0 || s->n_materials <= 0)
    return fail(c, RT_ERR_SCENE, "empty scene");
  for (int k = 0; k < s->n_world; ++k)
    if (s->world[k] < 0 || s->world[k] >= s->n_objects) return fail(c, RT_ERR_SCENE, "world index out of range");
  for (int k = 0; k < s->n_objects; ++k) {
    const rt_object& o = s->objects[k];
    if (o.kind == RT_OBJ_BVH && (o.b < 2 || o.b > 30 || o.a < 0 || o.a + (1 << o.b) - 1 > s->n_nodes))
      return fail(c, RT_ERR_SCENE, "bvh out of range");
    if ((o.kind == RT_OBJ_PRIM || o.kind == RT_OBJ_LIST) && (o.a < 0 || o.a + (o.kind == RT_OBJ_LIST ? o.b : 1) > s->n_prims))
      return fail(c, RT_ERR_SCENE, "prim index out of range");
    if ((o.kind == RT_OBJ_XFORM || o.kind == RT_OBJ_MEDIUM) && (o.a < 0 || o.a >= s->n_objects))
      return fail(c, RT_ERR_SCENE, "child object out of range");
  }
  for (int k = 0; k < s->n_prims; ++k)
    if (s->prims[k].material < 0 || s->prims[k].material >= s->n_materials)
      return fail(c, RT_ERR_SCENE, "prim material out of range");
  free_scene(c);
  // Device copies: primitives with the u,v flag folded into the type word and their reference
  // leaf rank in p[9]; nodes = reference trees followed by the traversal trees built here.
  std::vector<rt_prim> prims(s->prims, s->prims + s->n_prims);
  for (rt_prim& p : prims) {
    const rt_material& m = s->materials[p.material];
    if (p.type == RT_PRIM_SPHERE && m.type != RT_MAT_DIELECTRIC && tex_needs_uv(s, m.texture)) p.type |= RT_PRIM_FLAG_UV;
    if (p.type == RT_PRIM_MOVING_SPHERE && p.p[7] == 0.0f && p.p[8] == 1.0f) p.type |= RT_PRIM_FLAG_UNIT_T;
    int32_t none = -1;
    memcpy(&p.p[9], &none, 4);
  }
  std::vector<rt_bvh_node> nodes(s->nodes, s->nodes + s->n_nodes);
  std::vector<rt_object> objects(s->objects, s->objects + s->n_objects);
  std::vector<float2> pmargin(s->n_prims, make_float2(-INFINITY, -INFINITY));
  // (pvalid of a primitive outside every BVH: safe = -inf, so chain_ok's first test never applies)
  std::vector<float4> pvalid(3 * (size_t)s->n_prims, make_float4(0.0f, 0.0f, 0.0f, -INFINITY));
  std::vector<int> tree_pairs(objects.size(), 0);  // records of each BVH object's traversal tree
  for (size_t k = 0; k < objects.size(); ++k) {
    rt_object& o = objects[k];
    o.c = -1;
    if (o.kind == RT_OBJ_MEDIUM && medium_inert(s, o)) o.c = 1;  // object_query skips it for sane rays
    if (o.kind == RT_OBJ_BVH) {
      const int fast = build_traversal_tree(s, o.a, o.b, prims, nodes, pmargin, pvalid, &tree_pairs[k],
                                            c->opt.dedup_triangles != 0);
      if (fast < 0) return fail(c, RT_ERR_SCENE, "malformed reference bvh");
      o.c = fast;
    }
  }
  // Triangles: the Moller-Trumbore operands (v0, e0, e1) in p[0..8] of the device record and the
  // triangle's index in the type word's bits 12..31, so a hit test is one 48-byte fetch; the
  // 144-byte record is read only for the winner's hit record.
  for (rt_prim& p : prims) {
    if ((p.type & 0xff) != RT_PRIM_TRIANGLE) continue;
    const int ti = (int)p.p[0];
    if (ti < 0 || ti >= s->n_triangles || ti >= (1 << 19)) return fail(c, RT_ERR_SCENE, "triangle index out of range");
    const rt_triangle& t = s->triangles[ti];
    for (int k = 0; k < 3; ++k) {
      p.p[k] = t.v0[k];
      p.p[3 + k] = t.e0[k];
      p.p[6 + k] = t.e1[k];
    }
    p.type |= ti << 12;
  }
  bool world_step = s->n_world <= 8 && s->objects[s->world[0]].kind == RT_OBJ_BVH;
  for (int w = 1; w < s->n_world; ++w) world_step = world_step && s->objects[s->world[w]].kind == RT_OBJ_PRIM;
  std::vector<float4> wleaf, wxf;
  int wt_fb = -1, w_media = 0, w_inert = 0;
  // The world tree is opt-in (options.world_tree): measured slower than render_kernel's entry loop on
  // both list-world configs (MI355X: C5 3840x2159 4x4 97.2 ms vs 78.4; C3 800x800 10x10 24.7 vs 19.1)
  const bool world_tree = !world_step && c->opt.world_tree != 0 &&
                          build_world_tree(s, prims, nodes, wleaf, wxf, wt_fb, w_media, w_inert);
  std::vector<uint32_t> qnodes;
  int q_pairs = 0, q_ebias = 0;
  if (world_step && c->opt.quantized_tree != 0) {  // the world BVH's traversal tree, quantized (F_QLDS)
    // (the tree's own record count: coincident triangles are not leaves of it)
    const rt_object& wo = objects[(size_t)s->world[0]];
    const int np = tree_pairs[(size_t)s->world[0]];
    const size_t tables = 16 * ((size_t)s->n_materials + 2 * (size_t)s->n_textures + (size_t)s->n_images) + 16;
    if (np >= 1 && (size_t)np * 24 + 1024 * kStackDepth * 2 + tables <= (size_t)kLdsBudget &&
        build_qtree(nodes, wo.c, np, qnodes, q_ebias))
      q_pairs = np;
  }
  DScene& d = c->scene;
  d = DScene{};
  const rt_prim* dp;
  const rt_bvh_node* dn;
  const rt_material* dm;
  int rc;
  if ((rc = upload(c, s->world, (size_t)s->n_world, &d.world))) return rc;
  if ((rc = upload(c, objects.data(), objects.size(), &d.objects))) return rc;
  if ((rc = upload(c, prims.data(), prims.size(), &dp))) return rc;
  if ((rc = upload(c, s->triangles, (size_t)s->n_triangles, &d.tris))) return rc;
  if ((rc = upload(c, nodes.data(), nodes.size(), &dn))) return rc;
  if ((rc = upload(c, s->materials, (size_t)s->n_materials, &dm))) return rc;
  if (pmargin.size() & 1) pmargin.push_back(make_float2(-INFINITY, -INFINITY));  // whole float4s for LDS staging
  if ((rc = upload(c, pmargin.data(), pmargin.size(), &d.pmargin))) return rc;
  if ((rc = upload(c, pvalid.data(), pvalid.size(), &d.pvalid))) return rc;
  if ((rc = upload(c, s->textures, (size_t)s->n_textures, &d.texs))) return rc;
  if ((rc = upload(c, s->perlins, (size_t)s->n_perlins, &d.perlins))) return rc;
  // Image textures in 8x8-texel tiles (row-major tiles, row-major texels inside a tile): a texel's 2-D
  // neighbours share its cache lines, whichever way the texture's axes run across the image.  The
  // device image records point into the tiled copy; texel values are unchanged.
  std::vector<rt_image> dimages(s->images, s->images + s->n_images);
  std::vector<uint8_t> dtexels;
  for (rt_image& im : dimages) {
    if (im.width <= 0) continue;  // no data: the cyan fallback (texture.h:146-147)
    const long long n = (long long)im.width * im.height * im.bytes_per_pixel;
    if (im.height <= 0 || im.bytes_per_pixel < 1 || im.bytes_per_pixel > 4 || im.offset < 0 || im.offset + n > s->n_texels)
      return fail(c, RT_ERR_SCENE, "image texels out of range");
    if (dtexels.size() + ((size_t)n * 2) >= (size_t)1 << 31) return fail(c, RT_ERR_SCENE, "textures too large");
    const uint8_t* src = s->texels + im.offset;
    const int bpp = im.bytes_per_pixel, tpr = (im.width + 7) >> 3, tpc = (im.height + 7) >> 3;
    const size_t base = dtexels.size();
    dtexels.resize(base + (size_t)tpr * tpc * 64 * bpp, 0);
    for (int j = 0; j < im.height; ++j)
      for (int i = 0; i < im.width; ++i)
        memcpy(&dtexels[base + (((size_t)((j >> 3) * tpr + (i >> 3)) << 6) + ((j & 7) << 3) + (i & 7)) * bpp],
               src + ((size_t)j * im.width + i) * bpp, (size_t)bpp);
    im.offset = (int32_t)base;
  }
  if ((rc = upload(c, dimages.data(), dimages.size(), &d.images))) return rc;
  if ((rc = upload(c, dtexels.data(), dtexels.size(), &d.texels))) return rc;
  if ((rc = upload(c, wleaf.data(), wleaf.size(), &d.wleaf))) return rc;
  if ((rc = upload(c, wxf.data(), wxf.size(), &d.wxf))) return rc;
  d.wt_fb = wt_fb;
  d.w_media = w_media;
  d.w_inert = w_inert;
  // world_search applies: a list of primitives, BVHs (up to 2^20 leaves) and instances of them, and
  // inert media (options.merged_search: RT_MERGE_OFF keeps the entry loop; RT_MERGE_FALLBACK_ALL runs
  // the search, then every query takes the exact list -- tests)
  d.merge_ok = !world_step && s->n_world >= 2 && s->n_world < (1 << (31 - RT_WKEY_SHIFT)) &&
               c->opt.merged_search != RT_MERGE_OFF;
  for (int w = 0; w < s->n_world && d.merge_ok; ++w) {
    const rt_object& o = s->objects[s->world[w]];
    const rt_object& x = o.kind == RT_OBJ_XFORM ? s->objects[o.a] : o;
    if (o.kind == RT_OBJ_MEDIUM) d.merge_ok = medium_inert(s, o);
    else if (x.kind == RT_OBJ_BVH) d.merge_ok = x.b <= RT_WKEY_SHIFT;
    else d.merge_ok = x.kind == RT_OBJ_PRIM;
  }
  if (d.merge_ok && c->opt.merged_search == RT_MERGE_FALLBACK_ALL) d.merge_ok = 2;
  // world_search's visiting order (the winner does not depend on it: tie keys carry the list
  // position): the primitive entries first (one test each; their hits cull the traversals after
  // them), then the BVH and instance entries nearest first by the distance from the camera's origin
  // to their world-space box over the shutter, then the (inert) media.  C5, same box, Mrays/s: list
  // order 5 010-5 017, primitives first 5 036-5 044, primitives first + ground, door, instance (the
  // distance order) 5 093, + door, instance, ground 5 086, BVHs first 4 960.  options.merge_order:
  // RT_ORDER_LIST keeps list order, RT_ORDER_REVERSED reverses it (tests: both arrival orders of a tie).
  std::vector<int32_t> worder((size_t)s->n_world);
  for (int w = 0; w < s->n_world; ++w) worder[(size_t)w] = w;
  if (c->opt.merge_order == RT_ORDER_REVERSED) std::reverse(worder.begin(), worder.end());
  if (c->opt.merge_order == RT_ORDER_DISTANCE) {
    const float t0 = std::min(s->camera.time0, s->camera.time1), t1 = std::max(s->camera.time0, s->camera.time1);
    auto rank = [&](int w) -> double {  // < 0: primitive; distance: BVH / instance; +inf: medium / no box
      const rt_object& o = s->objects[s->world[w]];
      if (o.kind == RT_OBJ_PRIM) return -1.0;
      rth::Box b;
      if (o.kind == RT_OBJ_MEDIUM || !object_box(s, s->world[w], t0, t1, b)) return INFINITY;
      double d2 = 0.0;
      for (int a = 0; a < 3; ++a) {
        const double c = s->camera.origin[a], g = c < b.lo[a] ? b.lo[a] - c : (c > b.hi[a] ? c - b.hi[a] : 0.0);
        d2 += g * g;
      }
      return d2;
    };
    std::vector<double> key((size_t)s->n_world);
    for (int w = 0; w < s->n_world; ++w) key[(size_t)w] = rank(w);
    std::stable_sort(worder.begin(), worder.end(), [&](int x, int y) { return key[(size_t)x] < key[(size_t)y]; });
  }
  if ((rc = upload(c, worder.data(), worder.size(), &d.worder))) return rc;
  if (q_pairs > 0 && (rc = upload(c, qnodes.data(), qnodes.size(), &d.qnodes))) return rc;
  d.q_pairs = q_pairs;
  d.q_ebias = q_ebias;
  d.prims = (const float4*)dp;
  d.nodes = (const float4*)dn;
  d.mats = (const int4*)dm;
  d.n_world = s->n_world;
  d.cam = s->camera;
  d.bg[0] = s->background[0];
  d.bg[1] = s->background[1];
  d.bg[2] = s->background[2];
  c->features = scene_features(s);
  c->world_bvh = s->n_world == 1 && s->objects[s->world[0]].kind == RT_OBJ_BVH;
  c->world_step = world_step;
  c->world_tree = world_tree;
  c->bin_sph = nullptr;
  c->bin_ids = nullptr;
  c->bin_n = 0;
  if (c->world_bvh) {  // bounding spheres of the world BVH's primitives (boxes over the shutter)
    const rt_object& o = s->objects[s->world[0]];
    const int inner = (1 << o.b) - 1, last0 = (1 << (o.b - 1)) - 1;
    const float t0 = s->camera.time0, t1 = s->camera.time1;
    std::vector<float4> sph;
    std::vector<int32_t> ids;
    for (int k = last0; k < inner; ++k)
      for (int id : {s->nodes[o.a + k].leaf_a, s->nodes[o.a + k].leaf_b}) {
        if (id < 0) continue;
        sph.push_back(box_sphere(geom_box(s->prims[id], s->triangles, t0 < t1 ? t0 : t1, t0 < t1 ? t1 : t0)));
        ids.push_back(id);
      }
    if ((rc = upload(c, sph.data(), sph.size(), &c->bin_sph))) return rc;
    if ((rc = upload(c, ids.data(), ids.size(), &c->bin_ids))) return rc;
    c->bin_n = (int)ids.size();
  } else {  // list world: bounding spheres of the top-level entries (camera-ray entry masks)
    const float t0 = s->camera.time0, t1 = s->camera.time1;
    std::vector<float4> sph;
    for (int w = 0; w < s->n_world && w < 32; ++w) {
      rth::Box b;
      sph.push_back(object_box(s, s->world[w], t0 < t1 ? t0 : t1, t0 < t1 ? t1 : t0, b)
                        ? box_sphere(b) : make_float4(0.0f, 0.0f, 0.0f, INFINITY));
    }
    if ((rc = upload(c, sph.data(), sph.size(), &c->bin_sph))) return rc;
    c->bin_n = -(int)sph.size();  // negative: entry spheres (masks), not primitive spheres (lists)
  }
  c->dev_nodes = (int)nodes.size();
  // the stepwise LDS variant stages the world BVH's traversal tree in planes (stage_lds): it must be
  // the last tree of the node array and have at most kPlanePairs records.  A larger sphere tree (more
  // than 512 primitives) runs the stepwise kernel from global memory instead (documented cap: the
  // plane offsets are immediates, and every reference sphere scene fits; C2 has 487 pairs)
  c->plane_fb = -1;
  if (world_step) {
    const rt_object& wo = objects[(size_t)s->world[0]];
    const int np = tree_pairs[(size_t)s->world[0]];
    if (np >= 1 && np <= kPlanePairs && wo.c + 2 * np == (int)nodes.size()) {
      c->plane_fb = wo.c;
      c->plane_pairs = np;
    }
  }
  c->dev_prims = (int)prims.size();
  c->dev_mats = s->n_materials;
  c->dev_imgs = s->n_images;
  c->dev_texs = s->n_textures;
  c->have_scene = true;
  return RT_OK;
}

int rt_render_init(rt_ctx* c, int32_t width, int32_t height, uint64_t seed) {
  if (!c || width <= 0 || height <= 0) return fail(c, RT_ERR_ARG, "bad init args");
  HIPCHK(c, hipSetDevice(c->device));
  const long long n = (long long)width * height;
  if (n != c->states_n) {
    if (c->states) HIPCHK(c, hipFree(c->states));
    c->states = nullptr;
    c->states_n = 0;
    HIPCHK(c, hipMalloc((void**)&c->states, (size_t)n * 2 * sizeof(uint4)));
    c->states_n = n;
  }
  int digits = 0;
  for (unsigned long long x = (unsigned long long)(n - 1); x; x >>= 2) ++digits;
  // one workgroup per CU (its LDS holds the 100 KB slot-step table), every lane a run of slots
  const long long blocks = std::max(1LL, std::min<long long>(c->cus, (n + kInitBlock - 1) / kInitBlock));
  const long long chunk = (n + blocks * kInitBlock - 1) / (blocks * kInitBlock);
  hipLaunchKernelGGL(init_states_kernel, dim3((unsigned)blocks), dim3(kInitBlock), 5 * kStepRows * sizeof(uint32_t),
                     c->stream, c->states, n, seed, (const uint32_t*)c->jump_tab, digits, chunk);
  HIPCHK(c, hipGetLastError());
  // no host wait: every reader of the states (rt_render's kernels, rt_read_states) is ordered
  // after this launch on the context's stream
  c->states_seed = seed;
  return RT_OK;
}

namespace {
// A pointer the GPU kernels may write directly: device (or managed) memory.  Host memory, pinned
// or pageable, is staged through a temporary device buffer by rt_render / rt_resolve.
bool device_ptr(const void* p) {
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged || at.isManaged;
}
int render_dev(rt_ctx* c, const rt_render_args* a, float* fb_dev, rt_counters* counters);
}  // namespace

int rt_render(rt_ctx* c, const rt_render_args* a, float* fb, rt_counters* counters) {
  if (!c) return RT_ERR_ARG;
  int rc = validate_args(c, a);
  if (rc) return rc;
  if (!fb) return fail(c, RT_ERR_ARG, "null fb");
  HIPCHK(c, hipSetDevice(c->device));
  if (device_ptr(fb)) return render_dev(c, a, fb, counters);
  // host frame buffer: render into device memory, then copy the owned rows back
  const size_t n = (size_t)a->fb_count * rt_owned_rows(a, nullptr) * a->width * 3;
  float* tmp = nullptr;
  HIPCHK(c, hipMalloc((void**)&tmp, n * sizeof(float)));
  rc = render_dev(c, a, tmp, counters);
  if (!rc && hipMemcpy(fb, tmp, n * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(c, RT_ERR_HIP, "copy frame buffer to host");
  (void)hipFree(tmp);
  return rc;
}

namespace {
int render_dev(rt_ctx* c, const rt_render_args* a, float* fb_dev, rt_counters* counters) {
  int rc = RT_OK;
  if (!c->have_scene) return fail(c, RT_ERR_STATE, "no scene uploaded");
  if (!c->states || c->states_n != (long long)a->width * a->height || c->states_seed != a->seed)
    return fail(c, RT_ERR_STATE, "rt_render_init not called for this size/seed");
  if (!fb_dev) return fail(c, RT_ERR_ARG, "null fb");
  HIPCHK(c, hipSetDevice(c->device));
  const int rows = rt_owned_rows(a, nullptr);
  if (rows <= 0) return fail(c, RT_ERR_ARG, "no rows owned");
  if (rows > c->row_cap) {
    if (c->row_map) HIPCHK(c, hipFree(c->row_map));
    c->row_map = nullptr;
    HIPCHK(c, hipMalloc((void**)&c->row_map, 2 * (size_t)rows * sizeof(int32_t)));
    c->row_map_host.clear();
    c->row_cap = rows;
  }
  if (a->height > c->row_cost_cap) {
    if (c->row_cost) HIPCHK(c, hipFree(c->row_cost));
    c->row_cost = nullptr;
    HIPCHK(c, hipMalloc((void**)&c->row_cost, (size_t)a->height * sizeof(unsigned long long)));
    c->row_cost_cap = a->height;
  }
  std::vector<int32_t> rm(2 * (size_t)rows);
  rt_owned_rows(a, rm.data());
  const long long key[5] = {c->scene_gen, a->width, a->height, a->spp, a->max_depth};
  const bool have_cost = std::equal(key, key + 5, c->cost_key) && (int)c->host_cost.size() == a->height;
  for (int q = 0; q < rows; ++q) rm[rows + q] = q;
  // Costliest rows first only when lanes get few items each (a rank's share of a multi-GPU
  // image): there the launch ends with its last long item; with many items per lane bottom-to-top
  // order (sky last in the reference's scenes) measures faster.
  const long long items = (long long)a->fb_count * rows * a->width;
  // Item schedule: the first launch of a configuration records every item's segment count; later
  // launches process the items longest first (cost buckets of 8 segments, natural order inside a
  // bucket), and waves holding one of the top ~2 % run at raised priority.  A lane runs an item's samples serially, so
  // an item that starts late under full load (22 us per segment per lane on C2) decides when a
  // small share (a rank of a multi-GPU run) ends.  Pixel results do not depend on the order.
  // cam_mode is part of the key: the split samples' recorded sample-start states depend on it (the
  // PER_PIXEL camera draws come from the pixel's own state, REF ones from the slot-0 copy)
  constexpr int K = rt_ctx::kKey;
  // the launch runs render_step_kernel (as pick_variant decides below): the schedules' cost buckets
  const bool step_kernel = (c->world_step || c->world_tree) && (a->flags & (RT_FLAG_NO_STEP | RT_FLAG_WIDEST)) == 0;
  const long long pkey[K] = {c->scene_gen, a->width,   a->height,    a->spp,       a->max_depth, a->fb_first,
                             a->fb_count,  a->band_rows, a->band_first, a->band_stride, a->cam_mode};
  // (up to 2^31 items: 6 bytes of cost and position per item, C5's configured 100 fb x 100 spp draw
  // has 829 M; perm holds 32-bit positions)
  const bool sched = items <= (1LL << 31) && (a->flags & RT_FLAG_NO_SCHEDULE) == 0;
  if ((a->flags & RT_FLAG_FRESH) != 0) {  // as the configuration's first launch
    std::fill(c->perm_key, c->perm_key + K, -1LL);
    std::fill(c->pending_key, c->pending_key + K, -1LL);
    c->split_state = -1;
    c->n_split = 0;
    c->order_ok = false;
  }
  if (sched && !std::equal(pkey, pkey + K, c->perm_key) && std::equal(pkey, pkey + K, c->pending_key) &&
      items <= c->item_cap) {  // the configuration repeats: its schedule from the measured counts
    if ((rc = build_schedule(c, items, a->spp, c->pending_segs, step_kernel))) return rc;
    std::copy(pkey, pkey + K, c->perm_key);
    std::fill(c->pending_key, c->pending_key + K, -1LL);
  }
  const bool have_perm = sched && std::equal(pkey, pkey + K, c->perm_key);
  if (sched && items > c->item_cap) {
    if (c->item_cost) HIPCHK(c, hipFree(c->item_cost));
    if (c->perm) HIPCHK(c, hipFree(c->perm));
    c->item_cost = nullptr;
    c->perm = nullptr;
    c->item_cap = 0;
    std::fill(c->perm_key, c->perm_key + K, -1LL);
    std::fill(c->pending_key, c->pending_key + K, -1LL);
    HIPCHK(c, hipMalloc((void**)&c->item_cost, (size_t)items * sizeof(uint16_t)));
    HIPCHK(c, hipMalloc((void**)&c->perm, (size_t)items * sizeof(uint32_t)));
    c->item_cap = items;
  }
  const long long order_cap = 8LL * c->cus * 1024;
  if (!sched && have_cost && items < order_cap)
    std::stable_sort(rm.begin() + rows, rm.end(), [&](int x, int y) { return c->host_cost[rm[x]] > c->host_cost[rm[y]]; });
  // Per-launch host work kept off the repeat path: the row tables are uploaded only when they
  // change, the row costs are cleared and read back only on their measuring launch.
  std::vector<int32_t> rq(2 * (size_t)rows);
  for (int q = 0; q < rows; ++q) {
    rq[2 * (size_t)q] = rm[rows + q];
    rq[2 * (size_t)q + 1] = rm[rm[rows + q]];
  }
  if (rq != c->row_map_host) {
    c->row_map_host = rq;  // kept alive for the async copy
    HIPCHK(c, hipMemcpyAsync(c->row_map, c->row_map_host.data(), 2 * (size_t)rows * sizeof(int32_t),
                             hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(c, hipMemsetAsync(c->work, 0, 8 * sizeof(unsigned long long), c->stream));
  // row costs order the rows only when there is no item schedule: measured only then
  const bool measure_rows = !have_cost && !sched;
  if (measure_rows) HIPCHK(c, hipMemsetAsync(c->row_cost, 0, (size_t)a->height * sizeof(unsigned long long), c->stream));

  RenderParams P{};
  P.S = c->scene;
  P.states = c->states;
  P.fb = fb_dev;
  P.row_q = (const int2*)c->row_map;
  P.row_cost = measure_rows ? c->row_cost : nullptr;  // measured once per configuration
  P.work = c->work;
  P.counters = c->work + 1;
  P.total_items = (unsigned long long)a->fb_count * rows * a->width;
  P.npix = (long long)a->width * a->height;
  P.W = a->width;
  P.H = a->height;
  P.rows = rows;
  P.pstep = 1;
  P.per_row = (long long)a->fb_count * a->width;
  P.spp = a->spp;
  P.fb_first = a->fb_first;
  P.fb_count = a->fb_count;
  P.max_depth = a->max_depth;
  P.cam_mode = a->cam_mode;
  const rtx::State cs = rtx::seed_state(a->seed);  // pristine slot 0 = curand_init(seed, 0, 0)
  P.cam_state[0] = cs.d;
  for (int k = 0; k < 5; ++k) P.cam_state[1 + k] = cs.v[k];
  if (a->cam_mode == RT_CAM_REF_SLOT0) {
    const long long ckey[3] = {c->scene_gen, (long long)a->seed, a->spp};
    if (!std::equal(ckey, ckey + 3, c->cam_key)) {
      if (a->spp > c->cam_cap) {
        if (c->cam_tab) HIPCHK(c, hipFree(c->cam_tab));
        c->cam_tab = nullptr;
        c->cam_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->cam_tab, (size_t)a->spp * sizeof(float4)));
        c->cam_cap = a->spp;
      }
      camera_table(c->scene.cam, a->seed, a->spp, c->cam_host);
      HIPCHK(c, hipMemcpyAsync(c->cam_tab, c->cam_host.data(), (size_t)a->spp * sizeof(float4), hipMemcpyHostToDevice,
                               c->stream));
      std::copy(ckey, ckey + 3, c->cam_key);
    }
    P.S.cam_tab = c->cam_tab;
  }

  const bool stats = a->stats != 0;
  const bool check = (a->flags & RT_FLAG_AUDIT) != 0;
  const bool step = (c->world_step || c->world_tree) && (a->flags & (RT_FLAG_NO_STEP | RT_FLAG_WIDEST)) == 0;
  // node slots of the LDS image: the stepwise variant's world tree in planes of kPlanePairs records
  const int lds_node_slots = step && c->world_step ? (c->plane_fb >= 0 ? c->plane_fb + 2 * kPlanePairs : -1) : c->dev_nodes;
  const size_t lds_bytes =
      (size_t)(2 * lds_node_slots + 3 * c->dev_prims + (c->dev_prims + 1) / 2 + c->dev_mats + 2 * c->dev_texs) * sizeof(float4);
  const bool use_lds = lds_node_slots >= 0 && lds_bytes + 1024 * kStackDepth * 2 <= (size_t)kLdsBudget &&
                       c->dev_nodes / 2 < 32768 && c->dev_prims < 32768 && (a->flags & RT_FLAG_NO_LDS) == 0;
  // (the quantized tree applies to the variants that have a QLDS twin, whether or not the whole scene
  // would fit the LDS image of the F_LDS variants: no triangle-mesh variant has an F_LDS twin)
  const bool qlds = c->scene.q_pairs > 0 && (a->flags & RT_FLAG_NO_LDS) == 0;
  // the variants that stage their materials, textures and images after the locker (tables_after_locker)
  // need them to fit: a list world without BVHs whose tables exceed 32 KB runs the widest variant
  // instead, a merged-search scene whose tables exceed 1 KB the entry-loop variant
  const size_t table_bytes = (size_t)16 * ((size_t)c->dev_mats + 2 * (size_t)c->dev_texs + (size_t)c->dev_imgs);
  const bool big_tables = table_bytes > 32768;
  const bool merge_tables_fit = table_bytes <= 1024;
  int var = pick_variant(c->features, stats, (a->flags & RT_FLAG_EXACT_TRAVERSAL) != 0, check, use_lds,
                         (a->flags & RT_FLAG_WIDEST) != 0, step, c->world_tree, qlds,
                         c->scene.merge_ok != 0 && merge_tables_fit);
  if (var >= 0 && big_tables && (kVariants[var].mask & (F_LDS | F_QLDS | F_STEP | F_BVH | F_TRI)) == 0)
    var = pick_variant(c->features, stats, (a->flags & RT_FLAG_EXACT_TRAVERSAL) != 0, check, use_lds, true, step,
                       c->world_tree, qlds, c->scene.merge_ok != 0);
  if (var < 0) return fail(c, RT_ERR_SCENE, "no kernel variant covers the scene features");
  // shading phase of render_step_kernel once this many lanes of a wave wait (RT_SHADE_MIN: tuning)
  // (measured: C2 best at 60 of 64 lanes; C4's triangle-mesh steps at 48: 125.0 -> 119.7 ms, 40: 121.8)
  // (round 4, after the triangle dedupe and two steps per check, C4 Mrays/s at 40/48/52/56/60/62: 13 490 /
  // 13 922 / 14 052 / 14 090 / 13 932 / 13 618; C2 at 56/60/62: 14 659 / 14 747 / 14 605)
  P.shade_min = (kVariants[var].mask & F_TRI) != 0 ? kShadeMinMesh : kShadeMin;
  P.perm = have_perm ? c->perm : nullptr;
  P.n_long = have_perm ? c->n_long : 0;
  // Split samples of the longest items (stepwise kernel; scheduled launches of a configuration
  // with split items): the launch after the measuring one records their sample-start RNG states,
  // later launches with the same seed run each of their samples as a separate work item.
  // (split samples: the stepwise kernel, and render_kernel's parking variants)
  const bool split_ok = have_perm && c->n_split > 0 && a->spp > 1 && (a->flags & RT_FLAG_NO_SPLIT) == 0 &&
                        ((kVariants[var].mask & F_STEP) != 0 || parks_segment_mask(kVariants[var].mask));
  int split_mode = 0;
  if (split_ok && c->split_state == 1 && c->split_seed == a->seed) split_mode = 2;
  else if (split_ok) split_mode = 1;
  if (split_mode != 0) {
    const long long need = (long long)c->n_split * a->spp;
    if (need > c->ckpt_cap) {
      if (c->ckpt) HIPCHK(c, hipFree(c->ckpt));
      c->ckpt = nullptr;
      c->ckpt_cap = 0;
      c->split_state = -1;
      HIPCHK(c, hipMalloc((void**)&c->ckpt, (size_t)need * 2 * sizeof(uint4)));
      c->ckpt_cap = need;
      split_mode = 1;
    }
    if (split_mode == 2 && 3 * need > c->contrib_cap) {
      if (c->contrib) HIPCHK(c, hipFree(c->contrib));
      c->contrib = nullptr;
      c->contrib_cap = 0;
      HIPCHK(c, hipMalloc((void**)&c->contrib, (size_t)need * 3 * sizeof(float)));
      c->contrib_cap = 3 * need;
    }
    const long long skey[3] = {c->scene_gen, (long long)a->seed, a->spp};
    if (!std::equal(skey, skey + 3, c->cam_st_key)) {  // REF camera state at every sample start
      if (a->spp > c->cam_st_cap) {
        if (c->cam_st) HIPCHK(c, hipFree(c->cam_st));
        c->cam_st = nullptr;
        c->cam_st_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->cam_st, (size_t)a->spp * 2 * sizeof(uint4)));
        c->cam_st_cap = a->spp;
      }
      std::vector<float4> unused;
      camera_table(c->scene.cam, a->seed, a->spp, unused, &c->cam_st_host);
      HIPCHK(c, hipMemcpyAsync(c->cam_st, c->cam_st_host.data(), c->cam_st_host.size() * sizeof(uint4),
                               hipMemcpyHostToDevice, c->stream));
      std::copy(skey, skey + 3, c->cam_st_key);
    }
    // Split launches claim split samples and unsplit items in one sequence, longest first by the
    // recording launch's counts (the long samples of a small share start with the launch instead of
    // trailing it).  Built once per recording; results do not depend on the order.
    const long long rest = items - (long long)c->n_split;
    if (split_mode == 2 && c->rest_n == rest && c->opt.split_order != 0) {  // 0: samples in item order, then the rest
      const long long total = need + rest;
      if (!c->order_ok) {
        if (total > c->order_cap) {
          if (c->order) HIPCHK(c, hipFree(c->order));
          c->order = nullptr;
          c->order_cap = 0;
          HIPCHK(c, hipMalloc((void**)&c->order, (size_t)total * sizeof(uint32_t)));
          c->order_cap = total;
        }
        uint8_t* len = sort_keys(c, need);
        if (!len) return fail(c, RT_ERR_HIP, "out of device memory (split order)");
        split_len_kernel<<<(unsigned)((need + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(
            c->ckpt, (unsigned long long)need, a->spp, len);
        HIPCHK(c, hipGetLastError());
        unsigned hist[256];
        if ((rc = sort_hist(c, need, hist))) return rc;
        std::vector<unsigned>& t = c->order_tab_host;
        t.assign(256 + 2 * kOrderKeys, 0u);
        unsigned* sub_base = t.data();
        unsigned* sub_ge = t.data() + 256;
        unsigned* rest_gt = t.data() + 256 + kOrderKeys;
        for (int v = 255; v >= 0; --v) sub_ge[v] = sub_ge[v + 1] + hist[v];  // sub_ge[256] = 0
        for (int v = 0; v < 256; ++v) sub_base[v] = c->rest_gt[(size_t)v] + sub_ge[v + 1];
        std::copy(c->rest_gt.begin(), c->rest_gt.end(), rest_gt);
        HIPCHK(c, hipMemcpyAsync(c->order_tab, t.data(), t.size() * sizeof(unsigned), hipMemcpyHostToDevice, c->stream));
        if ((rc = sort_scatter(c, need, c->order_tab, c->order))) return rc;
        if (rest > 0) {
          order_rest_kernel<<<(unsigned)((rest + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(
              (unsigned long long)need, (unsigned long long)rest, c->order_tab, c->order);
          HIPCHK(c, hipGetLastError());
        }
        c->order_ok = true;
      }
      P.order = c->order;
    }
    P.split_mode = split_mode;
    P.n_split = c->n_split;
    P.ckpt = c->ckpt;
    P.contrib = c->contrib;
    P.cam_st = c->cam_st;
    if (split_mode == 2) P.total_items = (unsigned long long)need + (unsigned long long)(items - (long long)c->n_split);
  }
  P.item_cost = (sched && !have_perm) ? c->item_cost : nullptr;
  if (c->opt.shade_min > 0) P.shade_min = c->opt.shade_min;
  if (check) {
    if (!c->dbg) {
      HIPCHK(c, hipMalloc((void**)&c->dbg, 16 * sizeof(float) * kAuditCap + 64));
    }
    HIPCHK(c, hipMemsetAsync(c->dbg, 0, 16 * sizeof(float) * kAuditCap + 64, c->stream));
    P.S.dbg = c->dbg + 16;
    P.S.dbg_n = (unsigned*)c->dbg;
    P.S.dbg_cap = kAuditCap;
  }
  const int bs = variant_block(var);
  const bool lds_var = (kVariants[var].mask & F_LDS) != 0;
  const bool planes_var = lds_var && (kVariants[var].mask & F_STEP) != 0;
  if (planes_var && (c->plane_fb < 0 || lds_node_slots != c->plane_fb + 2 * kPlanePairs))
    return fail(c, RT_ERR_STATE, "stepwise LDS variant without a plane-staged world tree");
  P.S.lds_nodes = lds_var ? (planes_var ? lds_node_slots : c->dev_nodes) : 0;
  P.S.lds_fb = planes_var ? c->plane_fb : 0;
  P.S.lds_pairs = planes_var ? c->plane_pairs : 0;
  P.S.lds_prims = lds_var ? c->dev_prims : 0;
  const bool qlds_var = (kVariants[var].mask & F_QLDS) != 0;
  const int vmask = kVariants[var].mask;
  const bool tables_var = (vmask & (F_LDS | F_QLDS | F_STEP | F_BVH | F_TRI)) == 0 || (vmask & F_MERGE) != 0;
  P.S.lds_mats = (lds_var || qlds_var || tables_var) ? c->dev_mats : 0;
  P.S.lds_texs = (lds_var || qlds_var || tables_var) ? c->dev_texs : 0;
  P.S.lds_imgs = (qlds_var || tables_var) ? c->dev_imgs : 0;
  static_assert(kStackDepthQ == kStackDepth, "F_QLDS stacks");
  const size_t shmem = lds_var    ? lds_bytes + (size_t)bs * kStackDepth * 2
                       : qlds_var ? (size_t)16 * (qlds_mats_at(P.S) + c->dev_mats + 2 * c->dev_texs + c->dev_imgs)
                                  : (size_t)bs * (stack_words(vmask) + locker_words(vmask)) * 4 +
                                        (tables_var ? table_bytes : 0);
  // Camera-ray culling, built once per (scene, W, H): candidate lists for the stepwise kernel
  // (world = one BVH), top-level entry masks for list worlds.  Not in the exact / audit modes,
  // whose counters are the reference's.
  const int vm = kVariants[var].mask;
  const bool cull = (a->flags & RT_FLAG_NO_CAMERA_BINS) == 0 && (vm & (F_EXACT | F_CHECK)) == 0;
  const int tx = (a->width + (1 << kTileShift) - 1) >> kTileShift, ty = (a->height + (1 << kTileShift) - 1) >> kTileShift;
  const long long nt = (long long)tx * ty, ntp = (nt + 3) & ~3LL;  // tile lists: counts, then entries from ntp
  if (cull && (vm & F_STEP) == 0 && c->bin_n < 0) {
    const long long tkey[3] = {c->scene_gen, a->width, -1 - (long long)a->height};
    if (!std::equal(tkey, tkey + 3, c->tiles_key)) {
      if (nt > c->tiles_cap) {
        if (c->tiles) HIPCHK(c, hipFree(c->tiles));
        c->tiles = nullptr;
        c->tiles_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->tiles, (size_t)nt * sizeof(int32_t)));
        c->tiles_cap = nt;
      }
      bin_masks_kernel<<<(unsigned)((nt + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(
          c->bin_sph, -c->bin_n, c->scene.cam, a->width, a->height, tx, ty, (uint32_t*)c->tiles);
      HIPCHK(c, hipGetLastError());
      std::copy(tkey, tkey + 3, c->tiles_key);
    }
    P.tile_mask = (const uint32_t*)c->tiles;
    P.tiles_x = tx;
  }
  // Camera-ray candidate lists pay when lanes get many items each; for a small share (a rank of a
  // multi-GPU image) the launch ends with its longest items and the lists made that tail longer
  // (C2, one GPU rendering each rank's share: N = 4 (9.2 items per resident lane) 5.24 ms with
  // lists vs 5.94 without, N = 8 (4.6 per lane) 4.03 vs 3.51 ms).
  const double bins_min = c->opt.bins_min_items_per_lane;  // items per resident lane (default 6)
  // resident workgroups per CU: from the context's occupancy table, except for the variants whose
  // LDS holds the scene's tables after the locker (their size is the scene's)
  int bpc = std::max(1, c->blocks_per_cu[var]);
  if (tables_var) {
    int b = 0;
    HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kVariants[var].fn, bs, shmem));
    bpc = std::max(1, b);
  }
  const double lanes = (double)c->cus * bpc * bs;
  if (cull && (vm & F_STEP) != 0 && c->bin_n > 0 && (double)P.total_items >= bins_min * lanes) {
    const long long tkey[3] = {c->scene_gen, a->width, a->height};
    if (!std::equal(tkey, tkey + 3, c->tiles_key)) {
      if (ntp + nt * kTileCap * 2 > c->tiles_cap) {
        if (c->tiles) HIPCHK(c, hipFree(c->tiles));
        c->tiles = nullptr;
        c->tiles_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->tiles, (size_t)(ntp + nt * kTileCap * 2) * sizeof(int32_t)));
        c->tiles_cap = ntp + nt * kTileCap * 2;
      }
      bin_tiles_kernel<<<(unsigned)((nt + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(
          c->bin_sph, c->bin_ids, c->bin_n, c->scene.cam, a->width, a->height, tx, ty, c->tiles, c->tiles + ntp);
      HIPCHK(c, hipGetLastError());
      std::copy(tkey, tkey + 3, c->tiles_key);
    }
    P.tile_cnt = c->tiles;
    P.tile_ent = c->tiles + ntp;  // 16-byte aligned: tile_candidates reads int4 groups
    P.tiles_x = tx;
    P.tile_cap = kTileCap;
  }
  const long long resident = (long long)c->cus * bpc;
  // Persistent grid: every resident workgroup, even when there are fewer items than lanes (a
  // rank of a multi-GPU run): waves take items dynamically, so the items spread over all CUs
  // instead of packing into the first ceil(items / block) of them.
  const unsigned blocks = (unsigned)std::max(1LL, resident);
  // The first launch of a configuration has no measured item costs; a probe launch estimates them:
  // sample 0 of the first fb (the item's own first sample: same state, same camera draw) at every
  // ps-th owned row position and pixel, into the frame buffer's first fb slice, which the launch then
  // overwrites.  An item's estimate is the mean count of the grid points within kProbeRadius of its
  // own (rows and pixels) times spp; the launch claims items longest first by it (and records the
  // real counts, from which the next launch builds the schedule).  Inside the timed region: the
  // probe is part of the draw.  Grid step (options.probe_schedule < 0, the default): the smallest
  // with step^2 * spp * fb_count >= 200, a probe of at most ~0.5 % of the draw's samples.  Measured
  // (MI355X, cold first launches, no probe -> probe): whole frames C4 77.3 -> 67.0 ms (step 1; 4:
  // 69.6), C5 67.8 -> 64.0 (step 4; 2: 65.1, 8: 64.8), C2 17.02 -> 16.96 (step 4; 1: 17.28); not for
  // scenes without BVHs: C3's list of rects and media lost at every share size (N = 1 / 2 / 4 / 8
  // 14.73 / 8.10 / 4.93 / 3.23 -> 15.64 / 8.94 / 5.70 / 4.04 ms), its costs short and spatially
  // random, the natural order's coherence better (profiles/r05/probe/).
  int ps = c->opt.probe_schedule;  // probe grid step (0: no probe)
  if (ps < 0)
    for (ps = 1; ps < 64 && (long long)ps * ps * a->spp * a->fb_count < 200; ++ps) {
    }
  const bool probe = sched && !have_perm && ps > 0 && !check && (long long)a->spp * a->fb_count >= 4 &&
                     (vmask & (F_STEP | F_BVH)) != 0 && items <= c->item_cap &&
                     (c->opt.probe_max_items_per_lane <= 0.0f ||
                      (double)items < (double)c->opt.probe_max_items_per_lane * lanes);
  const int prow = (rows + ps - 1) / std::max(1, ps), pw = (a->width + ps - 1) / std::max(1, ps);
  const long long pitems = (long long)prow * pw;
  if (probe && pitems > c->probe_cap) {  // raw counts, then the smoothed grid
    if (c->probe_cost) HIPCHK(c, hipFree(c->probe_cost));
    c->probe_cost = nullptr;
    c->probe_cap = 0;
    HIPCHK(c, hipMalloc((void**)&c->probe_cost, 2 * (size_t)pitems * sizeof(uint16_t)));
    c->probe_cap = pitems;
  }
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  if (probe) {
    RenderParams Q = P;
    Q.spp = 1;
    Q.fb_count = 1;
    // a probe sample's path is cut after probe_depth segments: the launch (one sample per lane) lasts as
    // long as its longest path, and the estimate needs only the short ones' counts to rank regions.
    // Automatic (-1): 10 for the stepwise kernel, 20 for render_kernel.  Measured (MI355X, one GPU
    // rendering every rank's share, first launches, ms at N = 1 / 4 / 8; profiles/r06/probe_depth/):
    // C2 full depth 16.94 / 5.66 / 4.08, 10: 16.71 / 5.68 / 3.97, 6: 16.68 / 5.69 / 4.25; C4 full
    // 66.25 / 26.55 / 25.71, 10: 65.61 / 25.25 / 24.34, 16: 65.42 / 25.77 / 25.19; C5 full 64.26 /
    // 22.65 / 15.36, 10: 63.65 / 22.24 / 16.19, 20: 63.12 / 21.86 / 14.96
    const int pd = c->opt.probe_depth >= 0 ? c->opt.probe_depth : ((vmask & F_STEP) != 0 ? 10 : 20);
    if (pd > 0) Q.max_depth = std::min(a->max_depth, pd);
    Q.total_items = (unsigned long long)pitems;
    Q.pstep = ps;
    Q.per_row = pw;
    Q.perm = nullptr;
    Q.n_long = 0;
    Q.item_cost = c->probe_cost;
    Q.row_cost = nullptr;
    Q.split_mode = 0;
    void* qargs[] = {&Q};
    HIPCHK(c, hipLaunchKernel(kVariants[probe_variant(var)].fn, dim3(blocks), dim3(bs), qargs, shmem, c->stream));
    HIPCHK(c, hipGetLastError());
    RT_DIAG_PROBE_COSTS(c, pitems);  // diagnostic builds only (rt_diag.h): the raw probe counts to a file
    probe_smooth_kernel<<<(unsigned)((pitems + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(
        c->probe_cost, c->probe_cost + pitems, prow, pw);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemsetAsync(c->work, 0, 8 * sizeof(unsigned long long), c->stream));
    // The probe's schedule overwrites the context's one (perm, long prefix, split items): whatever
    // configuration perm_key named no longer has its schedule, so it runs cold again when it repeats
    // (A, A, probe of B, A must not claim A's items through B's perm).
    std::fill(c->perm_key, c->perm_key + K, -1LL);
    c->split_state = -1;
    c->n_split = 0;
    c->order_ok = false;
    // spread head (automatic: the stepwise triangle-mesh variants, every position of the first claims
    // strided).  Measured (MI355X, one GPU rendering each rank's share, first launches, ms at N = 1 / 2 /
    // 4 / 8; profiles/r06/spread/): C4 in order 65.54 / 36.87 / 24.42 / 24.20, spread 1 65.53 / 36.79 /
    // 24.61 / 23.93, 8 65.45 / 36.92 / 24.43 / 19.10, 64 65.56 / 36.89 / 24.64 / 18.33; C2 in order 16.77 /
    // 9.06 / 5.76 / 3.96, 1 16.74 / 9.09 / 5.46 / 3.99, 64 16.89 / 9.26 / 5.89 / 4.44 (its waves lose the
    // coherence of neighbouring items)
    const int spread_top =
        c->opt.spread_first >= 0 ? c->opt.spread_first : (step_kernel && (vmask & F_TRI) != 0 ? 64 : 0);
    if ((rc = probe_schedule(c, items, a->spp, a->width, a->fb_count, ps, pw, pitems, step_kernel,
                             (long long)blocks * (bs / 64), spread_top)))
      return rc;
    P.perm = c->perm;
    P.n_long = c->n_long;
  }
  RT_STEP_COUNT_HOST_RESET();
  RT_STAMP_HOST_RESET();
  RT_WAVE_HOST_RESET();
  void* kargs[] = {&P};
  // rt_last_kernel_ms: the render kernel (and the split merge), not the probe before it
  HIPCHK(c, hipEventRecord(c->ev2, c->stream));
  HIPCHK(c, hipLaunchKernel(kVariants[var].fn, dim3(blocks), dim3(bs), kargs, shmem, c->stream));
  HIPCHK(c, hipGetLastError());
  if (split_mode == 2) {
    merge_split_kernel<<<(unsigned)((c->n_split + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(P);
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  c->last_sched = (have_perm ? RT_SCHED_PREVIOUS : 0) | (split_mode == 2 ? RT_SCHED_SPLIT_REPLAY : 0) |
                  (probe ? RT_SCHED_PROBE : 0);
  snprintf(c->last_kernel, sizeof(c->last_kernel), "%s<%d>",
           (kVariants[var].mask & F_STEP) != 0 ? "render_step_kernel" : "render_kernel", kVariants[var].mask);
  unsigned long long host_cnt[8];
  HIPCHK(c, hipMemcpyAsync(host_cnt, c->work, sizeof(host_cnt), hipMemcpyDeviceToHost, c->stream));
  std::vector<unsigned long long> cost(measure_rows ? (size_t)a->height : 0);
  if (measure_rows)
    HIPCHK(c, hipMemcpyAsync(cost.data(), c->row_cost, cost.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                             c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (measure_rows) {
    c->host_cost.assign((size_t)a->height, 0ull);
    std::copy(key, key + 5, c->cost_key);
    for (int q = 0; q < rows; ++q) c->host_cost[rm[q]] = cost[rm[q]];
  }
  if (sched && !have_perm) {  // the schedule is built from these counts when the configuration repeats
    std::copy(pkey, pkey + K, c->pending_key);
    c->pending_segs = host_cnt[1];
  }
  if (split_mode == 1) {  // sample-start states recorded for this seed
    c->split_state = 1;
    c->order_ok = false;
    c->split_seed = a->seed;
  }
  HIPCHK(c, hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
  HIPCHK(c, hipEventElapsedTime(&c->last_kernel_ms, c->ev2, c->ev1));
  if (counters) {
    counters->segments = host_cnt[1];
    counters->node_tests = host_cnt[2];
    counters->prim_tests = host_cnt[3];
    counters->samples = host_cnt[4];
    counters->fallbacks = host_cnt[5];
  }
  RT_WAVE_HOST_WRITE();
  RT_STEP_COUNT_HOST_PRINT(var);
  RT_STAMP_HOST_WRITE();
  if (host_cnt[4] != (unsigned long long)a->spp * (unsigned long long)items)  // split samples: items != work items
    return fail(c, RT_ERR_HIP, "render kernel did not complete every sample");
  return RT_OK;
}
}  // namespace

float rt_last_render_ms(const rt_ctx* c) { return c ? c->last_ms : 0.0f; }
float rt_last_kernel_ms(const rt_ctx* c) { return c ? c->last_kernel_ms : 0.0f; }
const char* rt_last_render_kernel(const rt_ctx* c) { return c ? c->last_kernel : ""; }
int32_t rt_last_render_schedule(const rt_ctx* c) { return c ? c->last_sched : 0; }

int rt_read_states(rt_ctx* c, int64_t first, int64_t count, uint32_t* out) {
  if (!c || !out || first < 0 || count < 0) return fail(c, RT_ERR_ARG, "bad read_states args");
  if (!c->states || first + count > c->states_n) return fail(c, RT_ERR_STATE, "states not initialised");
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<uint4> tmp((size_t)count * 2);
  HIPCHK(c, hipMemcpyAsync(tmp.data(), c->states + 2 * first, tmp.size() * sizeof(uint4), hipMemcpyDeviceToHost,
                           c->stream));  // after rt_render_init's kernel on the same stream
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int64_t k = 0; k < count; ++k) {
    const uint4 a = tmp[2 * k], b = tmp[2 * k + 1];
    const uint32_t w[6] = {a.x, a.y, a.z, a.w, b.x, b.y};
    memcpy(out + 6 * k, w, sizeof(w));
  }
  return RT_OK;
}

int rt_audit_log(rt_ctx* c, float* out, int32_t cap) {
  if (!c) return -1;
  if (!c->dbg) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return -1;
  unsigned n = 0;
  if (hipMemcpy(&n, c->dbg, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  const int m = (int)std::min<unsigned>(n, (unsigned)std::min(cap, kAuditCap));
  if (out && m > 0 && hipMemcpy(out, c->dbg + 16, (size_t)m * 16 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return (int)n;
}

int rt_resolve(rt_ctx* c, const rt_render_args* a, const float* fb, uint8_t* out) {
  if (!c) return RT_ERR_ARG;
  int rc = validate_args(c, a);
  if (rc) return rc;
  if (!fb || !out) return fail(c, RT_ERR_ARG, "null buffer");
  HIPCHK(c, hipSetDevice(c->device));
  const long long per_fb = (long long)rt_owned_rows(a, nullptr) * a->width * 3;
  const long long blocks = (per_fb + kBlock - 1) / kBlock;
  // host buffers (either side) are staged through device memory
  const bool fb_host = !device_ptr(fb), out_host = !device_ptr(out);
  float* fb_tmp = nullptr;
  uint8_t* out_tmp = nullptr;
  if (fb_host) {
    HIPCHK(c, hipMalloc((void**)&fb_tmp, (size_t)per_fb * a->fb_count * sizeof(float)));
    if (hipMemcpy(fb_tmp, fb, (size_t)per_fb * a->fb_count * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
      rc = fail(c, RT_ERR_HIP, "copy frame buffer to device");
  }
  if (!rc && out_host && hipMalloc((void**)&out_tmp, (size_t)per_fb) != hipSuccess) rc = fail(c, RT_ERR_NOMEM, "hipMalloc out");
  if (!rc) {
    hipLaunchKernelGGL(resolve_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, c->stream, fb_host ? fb_tmp : fb,
                       out_host ? out_tmp : out, per_fb, a->fb_count);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess)
      rc = fail(c, RT_ERR_HIP, "resolve kernel");
  }
  if (!rc && out_host && hipMemcpy(out, out_tmp, (size_t)per_fb, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(c, RT_ERR_HIP, "copy image to host");
  if (fb_tmp) (void)hipFree(fb_tmp);
  if (out_tmp) (void)hipFree(out_tmp);
  return rc;
}

int rt_draw(rt_ctx* c, const rt_render_args* a, uint8_t* png_rgb_host, rt_counters* counters) {
  if (!c || !png_rgb_host) return RT_ERR_ARG;
  rt_render_args full = *a;
  full.band_rows = a->height;
  full.band_first = 0;
  full.band_stride = 1;
  int rc = validate_args(c, &full);
  if (rc) return rc;
  if ((rc = rt_render_init(c, a->width, a->height, a->seed))) return rc;
  const size_t npx = (size_t)a->width * a->height;
  float* fb = nullptr;
  uint8_t* img = nullptr;
  HIPCHK(c, hipMalloc((void**)&fb, npx * 3 * sizeof(float) * a->fb_count));
  if (hipMalloc((void**)&img, npx * 3) != hipSuccess) {
    (void)hipFree(fb);
    return fail(c, RT_ERR_NOMEM, "hipMalloc image");
  }
  rc = rt_render(c, &full, fb, counters);
  if (!rc) rc = rt_resolve(c, &full, fb, img);
  std::vector<uint8_t> tmp(npx * 3);
  if (!rc && hipMemcpy(tmp.data(), img, tmp.size(), hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(c, RT_ERR_HIP, "copy image");
  (void)hipFree(fb);
  (void)hipFree(img);
  if (rc) return rc;
  const size_t row = (size_t)a->width * 3;
  for (int j = 0; j < a->height; ++j) memcpy(png_rgb_host + (size_t)(a->height - 1 - j) * row, tmp.data() + j * row, row);
  return RT_OK;
}

}  // extern "C"
