// Reduced form of the round-2 "conditional ray copy" fault: a per-lane segment loop
// whose scatter builds the new ray in a separate struct and copies it under a divergent
// `if (scatter(...)) ray = sc;`, with per-material branches and rejection loops of lane-dependent
// trip counts.  Every lane's final ray is compared with the same code run on the host.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off [-DRT_COPY_INPLACE] -o raycopy_repro scripts/raycopy_repro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
struct V { float x, y, z; };
struct Ray { V o, d; float tm; };
__host__ __device__ inline V mk(float x, float y, float z) { return V{x, y, z}; }
__host__ __device__ inline V add(V a, V b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__host__ __device__ inline V mul(float t, V a) { return mk(t * a.x, t * a.y, t * a.z); }
__host__ __device__ inline float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ inline unsigned rnd(unsigned& s) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }
__host__ __device__ inline float uni(unsigned& s) { return (float)(rnd(s) >> 8) * (1.0f / 16777216.0f); }
__host__ __device__ inline V in_sphere(unsigned& s) {  // rejection loop: lane-dependent trip count
  V p;
  do p = mk(2 * uni(s) - 1, 2 * uni(s) - 1, 2 * uni(s) - 1); while (dot(p, p) >= 1.0f);
  return p;
}
// material m of the hit: 0 diffuse, 1 metal (may absorb), 2 glass (reflect / refract), 3 light, 4 fog
__host__ __device__ inline bool scatter(const Ray& r, V p, V n, int m, unsigned& s, Ray& out) {
  if (m == 3) return false;
  V dir;
  if (m == 0) {
    dir = add(n, in_sphere(s));
  } else if (m == 1) {
    dir = add(add(r.d, mul(-2.0f * dot(r.d, n), n)), mul(0.3f, in_sphere(s)));
    if (dot(dir, n) <= 0) return false;
  } else if (m == 2) {
    const float c = -dot(r.d, n);
    dir = uni(s) < 0.5f ? add(r.d, mul(2.0f * c, n)) : add(mul(0.66f, r.d), mul(0.66f * c - 0.5f, n));
  } else {
    dir = in_sphere(s);
  }
  out.o = p;
  out.d = dir;
  out.tm = r.tm;
  return true;
}
__host__ __device__ inline void trace(Ray& ray, unsigned s, int segs, float* att) {
  float a = 1.0f;
  for (int k = 0; k < segs; ++k) {
    const float t = 1.0f + (float)(rnd(s) & 7);  // a "hit" at t with a lane-dependent material
    const V p = add(ray.o, mul(t, ray.d));
    const V n = mul(1.0f / sqrtf(dot(p, p) + 1.0f), p);
    const int m = (int)(rnd(s) % 5u);
#ifdef RT_COPY_INPLACE
    if (!scatter(ray, p, n, m, s, ray)) break;
#else
    Ray sc;
    if (scatter(ray, p, n, m, s, sc)) {
      a *= 0.5f + 0.1f * (float)m;
      ray = sc;  // the conditional whole-struct copy
    } else {
      break;
    }
#endif
  }
  *att = a;
}
__global__ void k(Ray* rays, const unsigned* seeds, float* att, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Ray r = rays[i];
  trace(r, seeds[i], 3 + (int)(seeds[i] % 13u), att + i);
  rays[i] = r;
}
int main() {
  const int n = 1 << 16;
  Ray* h = new Ray[n];
  Ray* want = new Ray[n];
  unsigned* sd = new unsigned[n];
  float *ha = new float[n], *wa = new float[n];
  for (int i = 0; i < n; ++i) {
    sd[i] = 2654435761u * (unsigned)(i + 1);
    h[i] = Ray{mk(0.01f * (i % 97), 0.02f * (i % 31), -1.0f), mk(0.3f, 0.2f, 1.0f), 0.5f};
    want[i] = h[i];
    trace(want[i], sd[i], 3 + (int)(sd[i] % 13u), wa + i);
  }
  Ray* dr; unsigned* ds; float* da;
  if (hipMalloc(&dr, n * sizeof(Ray)) || hipMalloc(&ds, n * 4) || hipMalloc(&da, n * 4)) return 2;
  (void)hipMemcpy(dr, h, n * sizeof(Ray), hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, sd, n * 4, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dr, ds, da, n);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  (void)hipMemcpy(h, dr, n * sizeof(Ray), hipMemcpyDeviceToHost);
  (void)hipMemcpy(ha, da, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) bad += memcmp(&h[i], &want[i], sizeof(Ray)) != 0 || ha[i] != wa[i];
  printf("{\"lanes\": %d, \"mismatches\": %d}\n", n, bad);
  return 0;
}
