/* rt_hip.h — C ABI of the MI355X (gfx950) path-tracing hot path.
 *
 * Drop-in replacement for the per-pixel render path of daRoyalCacti/Raytracing_GPU:
 *
 *   rt_render_init   replaces  __global__ render_init(W, H, curandState*)        render.h:84-92
 *   rt_render        replaces  __global__ render(fb, W, H, ns, cam, states, world,
 *                                                max_depth, id, background)     render.h:94-113
 *                              (and color_f, render.h:55-81, plus everything it calls:
 *                               bvh.h:348-436, aabb.h:19-104, hittable_list.h:23-39,
 *                               sphere.h, moving_sphere.h, aarect.h, box.h, hittable.h:31-143,
 *                               constant_medium.h, material.h, texture.h, perlin.h)
 *   rt_resolve       replaces  write_frame_buffer + average_images (the per-fb 8-bit quantise
 *                              and square-average of draw())            color.h:19-170
 *   rt_scene_upload  replaces  the device-side object graph that struct scene's constructor
 *                              builds with <<<1,1>>> kernels            scenes.h:36-79
 *   rt_draw          replaces  void draw(scene&, render_settings)       render.h:118-174
 *
 * Conventions (render.h:99): a frame buffer is row-major, p = j*W + i, j = 0 the BOTTOM row,
 * 3 floats per pixel.  Every call returns 0 on success or a nonzero rt_status; rt_last_error()
 * gives the message.  Nothing exits or throws across the boundary (the reference's
 * checkCudaErrors -> exit(99), common.h:30-38, becomes a status code).  A context belongs to one
 * device and one host thread at a time.  Calls are synchronous unless named _async.
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum rt_status {
  RT_OK = 0,
  RT_ERR_ARG = 1,     /* invalid argument / shape */
  RT_ERR_HIP = 2,     /* HIP runtime error */
  RT_ERR_STATE = 3,   /* call order (e.g. render before upload) */
  RT_ERR_SCENE = 4,   /* malformed scene arrays */
  RT_ERR_NOMEM = 5
};

/* ------------------------------------------------------------------ flattened scene (host) */
/* Camera as built by camera::camera(), camera.h:18-47. */
typedef struct rt_camera {
  float origin[3], lower_left[3], horizontal[3], vertical[3];
  float u[3], v[3], w[3];
  float lens_radius, time0, time1;
} rt_camera;

enum rt_prim_type {
  RT_PRIM_SPHERE = 0,        /* sphere.h          p = cx cy cz r                           */
  RT_PRIM_MOVING_SPHERE = 1, /* moving_sphere.h   p = c0x c0y c0z r  dx dy dz t0  dt
                                                  (d = center1-center0, dt = time1-time0)   */
  RT_PRIM_RECT_XY = 2,       /* aarect.h xy_rect  p = x0 x1 y0 y1 k  (x1-x0) (y1-y0)        */
  RT_PRIM_RECT_XZ = 3,       /* aarect.h xz_rect  p = x0 x1 z0 z1 k  (x1-x0) (z1-z0)        */
  RT_PRIM_RECT_YZ = 4,       /* aarect.h yz_rect  p = y0 y1 z0 z1 k  (y1-y0) (z1-z0)        */
  RT_PRIM_TRIANGLE = 5,      /* triangle.h        p[0] = index into rt_scene_soa.triangles  */
  RT_PRIM_BOX = 6            /* box.h: the list of six rects  p = x0 y0 z0 x1 y1 z1         */
};
/* 48-byte primitive record; three 16-byte loads on the device. */
typedef struct rt_prim {
  float p[10];
  int32_t type;
  int32_t material;
} rt_prim;

/* Triangle (triangle.h:19-41 constructor output), 144 bytes. */
typedef struct rt_triangle {
  float v0[3], v1[3], v2[3];
  float e0[3], e1[3];        /* vertex1-vertex0, vertex2-vertex0 (triangle.h:26-27) */
  float d00, d01, d11, inv_denom;
  float uv[6];               /* u0 v0 u1 v1 u2 v2 */
  float n0[3], n1[3], n2[3];
  int32_t vertex_normals;
  int32_t pad;
} rt_triangle;

/* Inner node of a reference-layout BVH (bvh.h:133-346): a perfect binary tree of `rows` inner
 * levels stored in heap order (children of k are 2k+1, 2k+2).  Nodes of the last inner level
 * carry the one or two primitives of their leaves in leaf_a / leaf_b (-1 = none); nodes above it
 * carry their split axis (0..2, drawn at build time) in leaf_a and -1 in leaf_b. */
typedef struct rt_bvh_node {
  float lo[3];
  int32_t leaf_a;
  float hi[3];
  int32_t leaf_b;
} rt_bvh_node;

enum rt_object_kind {
  RT_OBJ_PRIM = 0,   /* a = prim index                                                         */
  RT_OBJ_LIST = 1,   /* a = first prim, b = count; hittable_list semantics (box.h)             */
  RT_OBJ_BVH = 2,    /* a = first node, b = rows (inner levels)                                */
  RT_OBJ_XFORM = 3,  /* translate(rotate_y(child)), hittable.h:31-143; a = child object
                        (PRIM/LIST/BVH), b = flags (1 translate, 2 rotate_y);
                        f[0..2] = offset, f[3] = sin, f[4] = cos                               */
  RT_OBJ_MEDIUM = 4  /* constant_medium.h; a = boundary object (PRIM/LIST/BVH/XFORM),
                        b = phase material, f[0] = -1/density                                  */
};
typedef struct rt_object {
  int32_t kind, a, b, c;
  float f[8];
} rt_object;

enum rt_material_type {
  RT_MAT_LAMBERTIAN = 0, RT_MAT_METAL = 1, RT_MAT_DIELECTRIC = 2,
  RT_MAT_DIFFUSE_LIGHT = 3, RT_MAT_ISOTROPIC = 4
};
typedef struct rt_material {
  int32_t type;
  int32_t texture; /* albedo / emit texture (unused by dielectric) */
  float param;     /* metal fuzz or dielectric index of refraction */
  int32_t pad;
} rt_material;

enum rt_texture_type {
  RT_TEX_SOLID = 0, RT_TEX_CHECKER = 1, RT_TEX_NOISE = 2, RT_TEX_TURBULENT = 3,
  RT_TEX_MARBLE = 4, RT_TEX_IMAGE = 5
};
typedef struct rt_texture {
  int32_t type;
  int32_t a;       /* checker: even texture; noise/turb/marble: perlin table; image: image   */
  int32_t b;       /* checker: odd texture; turbulent: depth                                  */
  int32_t pad;
  float color[3];  /* solid colour                                                            */
  float scale;     /* noise scale                                                             */
} rt_texture;

/* Perlin tables (perlin.h:9-34). */
typedef struct rt_perlin {
  float ranvec[256][3];
  int32_t perm_x[256], perm_y[256], perm_z[256];
} rt_perlin;

/* Image texture (texture.h:97-164): width, height, bytes per pixel, byte offset into texels. */
typedef struct rt_image {
  int32_t width, height, bytes_per_pixel;
  int32_t offset;
} rt_image;

typedef struct rt_scene_soa {
  rt_camera camera;
  float background[3];
  float aspect;
  const int32_t* world;          int32_t n_world;   /* top-level hittable_list */
  const rt_object* objects;      int32_t n_objects;
  const rt_prim* prims;          int32_t n_prims;
  const rt_triangle* triangles;  int32_t n_triangles;
  const rt_bvh_node* nodes;      int32_t n_nodes;
  const rt_material* materials;  int32_t n_materials;
  const rt_texture* textures;    int32_t n_textures;
  const rt_perlin* perlins;      int32_t n_perlins;
  const rt_image* images;        int32_t n_images;
  const uint8_t* texels;         int64_t n_texels;
} rt_scene_soa;

/* ------------------------------------------------------------------ render arguments */
enum rt_cam_mode {
  RT_CAM_REF_SLOT0 = 0, /* reference mode: lens/time draws from a private copy of
                           the pristine slot-0 state, restarted per pixel and per fb        */
  RT_CAM_PER_PIXEL = 1  /* lens/time draws from the pixel's own state                       */
};

/* rt_render_args.flags */
#define RT_FLAG_EXACT_TRAVERSAL 1 /* visit exactly the reference's BVH node set (bvh.h:348-436)
                                     instead of the margin-culled near-first traversal; both give
                                     the same pixels, only node/prim test counts differ          */
#define RT_FLAG_NO_LDS 4          /* keep the scene in global memory even when it fits in LDS   */
#define RT_FLAG_AUDIT 2           /* run both traversals per BVH query, keep the exact result and
                                     log every disagreement (read back with rt_audit_log)       */
#define RT_FLAG_WIDEST 8          /* testing: run the widest compiled kernel variant that covers
                                     the scene instead of the narrowest (same pixels)           */
#define RT_FLAG_NO_STEP 16        /* testing: world = one BVH still runs the segment-per-trip
                                     kernel instead of the stepwise one (same pixels)           */
#define RT_FLAG_NO_SCHEDULE 32    /* natural item order on every launch (no longest-first
                                     schedule from the previous launch; same pixels)            */
#define RT_FLAG_NO_CAMERA_BINS 64 /* camera rays traverse the BVH instead of testing their 8x8
                                     tile's candidate list (world = one BVH; same pixels)       */
#define RT_FLAG_NO_SPLIT 128      /* never split the samples of the longest items over work items
                                     on warm launches (stepwise kernel; same pixels)            */
#define RT_FLAG_FRESH 256         /* forget the context's item schedule first: the launch runs as
                                     the first launch of its configuration does (benchmarks of a
                                     one-shot draw; same pixels)                                */

typedef struct rt_render_args {
  int32_t width, height;  /* full image size; N = width*height drives the RNG slots (H3)  */
  int32_t spp;            /* samples_per_pixel_per_fb (render.h:24)                      */
  int32_t fb_first;       /* first frame-buffer id `id` (render.h:154)                   */
  int32_t fb_count;       /* number of consecutive fb ids rendered by this call          */
  int32_t max_depth;      /* render.h:27                                                 */
  int32_t cam_mode;       /* rt_cam_mode                                                 */
  int32_t band_rows;      /* row tiling: rows grouped in bands of band_rows (>= 1)       */
  int32_t band_first;     /* this call renders bands b = band_first, +band_stride, ...   */
  int32_t band_stride;
  int32_t stats;          /* 1: also count BVH node and primitive tests                  */
  int32_t flags;          /* RT_FLAG_*                                                   */
  uint64_t seed;          /* 1984 in the reference (render.h:91)                         */
} rt_render_args;

typedef struct rt_counters {
  uint64_t segments;      /* top-level world->hit queries, primary + bounces (render.h:63) */
  uint64_t node_tests;    /* stats only: BVH box tests                                     */
  uint64_t prim_tests;    /* stats only: primitive hit() tests                             */
  uint64_t samples;
  uint64_t fallbacks;     /* stats only: culled BVH queries re-run on the reference visit set */
} rt_counters;

typedef struct rt_ctx rt_ctx;

/* ------------------------------------------------------------------ context */
int rt_ctx_create(int hip_device, rt_ctx** out);
int rt_ctx_destroy(rt_ctx* ctx);
const char* rt_last_error(const rt_ctx* ctx);

/* Implementation options of a context.  None of them changes a pixel or a segment count (every
 * setting is parity-tested against the oracle); they choose kernel variants, search algorithms and
 * schedule thresholds.  rt_ctx_options_default gives the measured product configuration, which a new
 * context starts with; the library reads no environment variable.  The upload-time fields apply from
 * the next rt_scene_upload; rt_ctx_set_options also drops the context's item schedule, so the next
 * launch of any configuration is a cold one. */
enum rt_merge_mode {
  RT_MERGE_ON = 0,           /* list worlds of primitives, BVHs, instances and inert media: one
                                candidate search over every entry (world_search)                 */
  RT_MERGE_OFF = 1,          /* the per-entry list loop of hittable_list.h:23-39 (world_hit)     */
  RT_MERGE_FALLBACK_ALL = 2  /* testing: run the search, then answer every query exactly         */
};
enum rt_merge_order {
  RT_ORDER_DISTANCE = 0,     /* merged search visits primitives, then BVHs / instances nearest the
                                camera first, then inert media                                    */
  RT_ORDER_LIST = 1,         /* the list's own order                                               */
  RT_ORDER_REVERSED = 2      /* testing: the list reversed                                         */
};
typedef struct rt_ctx_options {
  /* upload time (rt_scene_upload) */
  int32_t world_tree;        /* 1: a list world flattened into ONE traversal tree for the stepwise
                                kernel (measured slower than the merged search; default 0).  This
                                and the other 0/1 fields reject any other value                    */
  int32_t quantized_tree;    /* 1: the world BVH's traversal tree as 24-byte records in LDS when it
                                fits (C4's mesh; default 1)                                         */
  int32_t merged_search;     /* rt_merge_mode (default RT_MERGE_ON)                                */
  int32_t merge_order;       /* rt_merge_order (default RT_ORDER_DISTANCE)                         */
  int32_t dedup_triangles;   /* 1: coincident triangles leave the traversal trees, the first of a
                                group stands for it (default 1)                                     */
  /* per launch (rt_render) */
  int32_t shade_min;         /* stepwise kernel: lanes waiting before a wave shades; 0 = the
                                variant's measured value (60, 48 for triangle meshes)               */
  float bins_min_items_per_lane; /* camera-ray tile lists from this many items per resident lane
                                (default 6; 0 = always)                                             */
  float split_min_segments;  /* > 0: split the samples of items of at least this many segments;
                                0 = the share-size rule (default)                                   */
  int32_t split_order;       /* 1: split samples and unsplit items claimed in one longest-first
                                sequence (default); 0: split samples first, in item order          */
  int32_t cost_shift;        /* item-schedule cost buckets of 2^cost_shift segments, 0..12; -1 =
                                automatic                                                           */
  float long_pct;            /* share of the longest items whose waves run at raised priority
                                (default 2)                                                         */
  int32_t probe_schedule;    /* k > 0: the first launch of a configuration (>= 4 samples per pixel,
                                a scene with BVHs) claims its items longest first by a probe
                                launch's estimate: sample 0 of the first fb at every k-th row and
                                pixel (output discarded), smoothed over neighbouring grid points;
                                -1 (default): the smallest k with k*k*spp*fb_count >= 200; 0: natural
                                order; at most 64                                                   */
  float probe_max_items_per_lane; /* > 0: probe only launches with fewer items per resident lane (a
                                multi-GPU share); 0 (default): any launch                           */
  int32_t probe_depth;       /* k > 0: a probe sample's path ends after k segments (the probe launch
                                lasts as long as its longest path); 0: the launch's max_depth; -1
                                (default): 10 for the stepwise kernel, 20 for the others            */
  int32_t spread_first;      /* k = 1..64: a probe-ordered first launch gives each wave's first
                                claim k of the order's first k x waves items, strided (one wave
                                does not start with many of the longest), and 64 - k neighbours
                                in order; 0: the order as is; -1 (default): automatic              */
} rt_ctx_options;
void rt_ctx_options_default(rt_ctx_options* opts);
int rt_ctx_set_options(rt_ctx* ctx, const rt_ctx_options* opts);
int rt_ctx_get_options(const rt_ctx* ctx, rt_ctx_options* opts);
/* Rows of the image owned by a band tiling (ascending); returns the count. rows may be NULL. */
int32_t rt_owned_rows(const rt_render_args* a, int32_t* rows);

/* Copies the flattened scene to device memory owned by the context. */
int rt_scene_upload(rt_ctx* ctx, const rt_scene_soa* scene);

/* Per-slot XORWOW states curand_init(seed, slot, 0) for slot < width*height (render.h:84-92). */
int rt_render_init(rt_ctx* ctx, int32_t width, int32_t height, uint64_t seed);
/* Copies states [first, first+count) to host as 6 words each: d, v0..v4 (the curandStateXORWOW
 * words the reference's render_init leaves in its state array). */
int rt_read_states(rt_ctx* ctx, int64_t first, int64_t count, uint32_t* out);

/* Renders fb ids [fb_first, fb_first+fb_count) for the owned rows into fb: layout
 * [fb_count][owned_rows][width][3] floats, owned rows ascending.  fb may be a device (or managed)
 * pointer, written by the kernel directly, or a host pointer (pinned or pageable): then the frame
 * buffers are rendered into a temporary device buffer and copied back before the call returns.
 * counters may be NULL. */
int rt_render(rt_ctx* ctx, const rt_render_args* args, float* fb, rt_counters* counters);
/* Device time in ms of the last rt_render call, from HIP events recorded on the context stream: a first
 * launch's probe launch and item schedule (RT_SCHED_PROBE) included, the host staging of a host fb
 * excluded. */
float rt_last_render_ms(const rt_ctx* ctx);
/* ... of its render kernel alone (with the split-sample merge after it, RT_SCHED_SPLIT_REPLAY). */
float rt_last_kernel_ms(const rt_ctx* ctx);
/* Kernel of the last render launch as rocprof names it (stem, e.g. "render_step_kernel<25730>"):
 * the kernel variant the context picked for the scene's features and flags. */
const char* rt_last_render_kernel(const rt_ctx* ctx);
/* How the last render launch ordered its work (RT_SCHED_* bits; 0 = a cold launch: nothing from an
 * earlier launch of the same configuration was used). */
#define RT_SCHED_PREVIOUS 1     /* items claimed longest first by the segment counts of an earlier
                                   launch of this configuration (same scene, size, spp, depth, fb
                                   range, tiling and camera mode)                               */
#define RT_SCHED_SPLIT_REPLAY 2 /* split samples started from RNG states an earlier launch recorded */
#define RT_SCHED_PROBE 4        /* items claimed longest first by a probe launch's estimate (the
                                   first launch of a configuration, options.probe_schedule)     */
int32_t rt_last_render_schedule(const rt_ctx* ctx);
/* Audit log of the last RT_FLAG_AUDIT render: 16 floats per disagreeing BVH query (ray o[3] d[3]
 * time, tmin, tmax, culled t, culled prim (int bits), exact t, exact prim, culled rank, 0, 0).
 * Copies up to cap entries into out (may be NULL); returns the total number of disagreements. */
int rt_audit_log(rt_ctx* ctx, float* out, int32_t cap);

/* Quantise each fb (write_frame_buffer) and square-average them in fb order (average_images)
 * for the owned rows: out = [owned_rows][width][3] bytes, owned rows ascending (row 0 of a PNG is
 * image row height-1).  fb and out may each be a device or a host pointer (host buffers are
 * staged through temporary device memory). */
int rt_resolve(rt_ctx* ctx, const rt_render_args* args, const float* fb, uint8_t* out);

/* draw(): init + render every fb + resolve, whole image, host output in PNG row order
 * (top row first), W*H*3 bytes.  counters may be NULL. */
int rt_draw(rt_ctx* ctx, const rt_render_args* args, uint8_t* png_rgb_host, rt_counters* counters);

/* ------------------------------------------------------------------ host scene library */
/* Builds one of the reference scenes (scenes.h) on the host: "basic", "first", "big1" (alias
 * "random"), "two_spheres", "two_perlin", "cornell", "cornell_smoke", "triangle", "triangles",
 * "backpack" (renders only its ground, H17).  The returned handle owns the arrays its
 * rt_scene_soa points at. */
typedef struct rt_scene_host rt_scene_host;
int rt_scene_build(const char* name, rt_scene_host** out);
const rt_scene_soa* rt_scene_view(const rt_scene_host* s);
void rt_scene_free(rt_scene_host* s);

/* Decoded image, the stbi_load layout make_image() uploads (texture.h:166-203): rows top to
 * bottom, bytes_per_pixel interleaved channels. */
typedef struct rt_image_asset {
  int32_t width, height, bytes_per_pixel;
  int32_t pad;
  const uint8_t* data;
} rt_image_asset;
/* One mesh as create_meshes_d() builds it (triangle_mesh.h:147-204): 24 floats per triangle,
 * v0[3] v1[3] v2[3] n0[3] n1[3] n2[3] u0 v0 u1 v1 u2 v2.  vertex_normals = 0 uses the face
 * normal (triangle.h:166); image = index into the assets' images for its lambertian texture. */
typedef struct rt_mesh_asset {
  int32_t n_triangles;
  int32_t vertex_normals;
  int32_t image;
  int32_t pad;
  const float* data;
} rt_mesh_asset;
typedef struct rt_scene_assets {
  int32_t n_images;
  int32_t n_meshes;
  const rt_image_asset* images;
  const rt_mesh_asset* meshes;
} rt_scene_assets;
/* rt_scene_build with external assets (the files the reference reads at scene construction):
 * "earth" (images[0] = earthmap, scenes.h:278-320), "door" / "cup" (meshes[0] with its texture,
 * scenes.h:478-523,576-621), "final" (the composed book-2 final scene of config C5: images[0]
 * and meshes[0]), and every name rt_scene_build accepts (assets may be NULL). */
int rt_scene_build_ex(const char* name, const rt_scene_assets* assets, rt_scene_host** out);

/* OBJ mesh ingestion: create_meshes() (triangle_mesh.h:208-352) with assimp's OBJ import
 * (ReadFile(Triangulate | GenNormals), processNode order) restated, see csrc/rt_obj.cpp.
 * RT_OBJ_INDEX_REFERENCE reproduces create_meshes_d's indexing of the concatenated vertex array
 * with per-mesh local indices; RT_OBJ_INDEX_GLOBAL offsets each mesh's indices. */
enum { RT_OBJ_INDEX_REFERENCE = 0, RT_OBJ_INDEX_GLOBAL = 1 };
typedef struct rt_obj_mesh rt_obj_mesh;
typedef struct rt_obj_info {
  int32_t n_triangles;   /* rows of `triangles` (rt_mesh_asset layout, 24 floats each)         */
  int32_t n_meshes;      /* aiMeshes the import produced                                        */
  int32_t n_vertices;    /* concatenated vertex count                                            */
  int32_t n_textures;    /* distinct diffuse textures of the used materials (reference needs 1) */
  const float* triangles;
  const char* texture;   /* first diffuse texture path (OBJ directory + map_Kd), "" if none     */
} rt_obj_info;
int rt_obj_load(const char* path, int32_t index_mode, rt_obj_mesh** out);
/* Image decoding for textures: make_image()/imread() (texture.h:166-203) through the reference's
 * stb_image v2.26, restated for baseline JPEGs (csrc/rt_image.cpp): identical texel bytes.
 * Output = stbi_load(.., 0) layout (rows top to bottom, 1 or 3 channels). */
typedef struct rt_image_host rt_image_host;
int rt_image_decode(const uint8_t* bytes, int64_t n, rt_image_host** out);
int rt_image_load(const char* path, rt_image_host** out);
const rt_image_asset* rt_image_view(const rt_image_host* im);
void rt_image_free(rt_image_host* im);
const rt_obj_info* rt_obj_view(const rt_obj_mesh* m);
void rt_obj_free(rt_obj_mesh* m);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_H */
