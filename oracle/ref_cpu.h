/* ref_cpu.h — C API of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * The oracle is a plain C++17 restatement of daRoyalCacti/Raytracing_GPU's render path
 * (render.h:55-113 and everything it calls).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product path never does.
 */
#ifndef REF_CPU_H
#define REF_CPU_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ref_scene ref_scene;

typedef struct ref_counters {
  long long segments;   /* top-level world->hit queries (render.h:63) */
  long long node_tests; /* BVH AABB tests (bvh.h:416) */
  long long prim_tests; /* primitive hit() calls issued by BVH leaves and lists */
  long long samples;
} ref_counters;

enum { REF_CAM_REF_SLOT0 = 0, REF_CAM_PER_PIXEL = 1 };

/* Build one of the reference's scenes (scenes.h).  rtl != 0 evaluates multi-draw argument lists
 * right-to-left instead of left-to-right (hazard H9; used only for the layout pin test). */
int ref_scene_create(const char* name, int rtl, ref_scene** out);
/* Scenes that read files in the reference take decoded assets: "earth" (images[0]), "door" /
 * "cup" (meshes[0], 24 floats per triangle: v0 v1 v2 n0 n1 n2 u0 v0 u1 v1 u2 v2). */
typedef struct ref_image { int width, height, bytes_per_pixel, pad; const uint8_t* data; } ref_image;
typedef struct ref_mesh { int n_triangles, vertex_normals, image, pad; const float* data; } ref_mesh;
typedef struct ref_assets { int n_images, n_meshes; const ref_image* images; const ref_mesh* meshes; } ref_assets;
int ref_scene_create_ex(const char* name, int rtl, const ref_assets* assets, ref_scene** out);
void ref_scene_destroy(ref_scene* s);
/* Capture world-query rays (8 floats: o, d, time, 0) into buf during later ref_render calls
 * (design experiments only); returns the number captured since the previous call. */
long long ref_capture_rays(float* buf, long long max_rays);
float ref_scene_aspect(const ref_scene* s);
void ref_scene_background(const ref_scene* s, float rgb[3]);
int ref_scene_h20(const ref_scene* s); /* 1 if random_int returned max+1 during the build */
/* Replace the scene camera (vup (0,1,0), shutter [0,1]); used to match older reference renders. */
void ref_scene_set_camera(ref_scene* s, const float from[3], const float at[3], float vfov,
                          float aperture, float focus);
/* Object table of big_scene1, 13 floats per row: type, material, centre0[3], centre1[3], radius,
 * albedo[3], fuzz-or-ir. */
int ref_scene_table(const ref_scene* s, float* out, int max_rows);
/* Sequence of BVH split axes drawn during the build (bvh.h:294), -1 padded. */
int ref_scene_bvh_axes(const ref_scene* s, int* out, int max_n);

/* Render frame buffer `fb_id` of a W x H image with `spp` samples per pixel, for the rows
 * j = row0, row0+row_step, ... (j = 0 is the bottom row, render.h:99).  fb is W*H*3 floats
 * indexed p = j*W + i; untouched rows are left alone.  seg_per_pixel (optional) gets the
 * segment count of each rendered pixel. */
int ref_render(const ref_scene* s, int W, int H, int spp, int fb_id, int max_depth, int cam_mode,
               int row0, int row_step, int nthreads, float* fb, int* seg_per_pixel,
               ref_counters* counters);

/* write_frame_buffer (color.h:19-49) quantisation of one fb, then average_images
 * (color.h:57-170) over nfb quantised fbs taken in order 0..nfb-1.  Output is the PNG raster:
 * row 0 = top = fb row H-1. */
void ref_quantize_fb(const float* fb, int W, int H, uint8_t* out_ppm_order);
void ref_average(const uint8_t* const* ppms, int nfb, int W, int H, uint8_t* out_png_order);

/* cuRAND-compatible XORWOW: state = {d, v0..v4}. */
void ref_xorwow_init(uint64_t seed, uint64_t subsequence, uint64_t offset, uint32_t state[6]);
uint32_t ref_xorwow_next(uint32_t state[6]);
float ref_xorwow_uniform(uint32_t state[6]);
/* Jump matrices A^(4^i * 2^67) (sequence, which=0) or A^(4^i) (offset, which=1), 800 words
 * each, derived from the XORWOW recurrence from first principles. */
void ref_xorwow_jump_matrix(int which, int i, uint32_t out[800]);

#ifdef __cplusplus
}
#endif
#endif
