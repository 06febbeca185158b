/* rt_multi.h — multi-GPU draw() for one node, C ABI (librt_multi.so, links librt_hip.so + RCCL).
 *
 * Replaces the reference's single-device `void draw(scene&, render_settings)` (render.h:118-174)
 * when the frame buffer is tiled over several GPUs (BASELINE configs C4/C5):
 *   - one rt_ctx (device copy of the scene, RNG states, stream) per rank;
 *   - image rows dealt in bands of args->band_rows round-robin over the ranks
 *     (band_first = rank, band_stride = n_ranks; rt_owned_rows gives each rank's rows);
 *   - each rank runs render_init + render (every fb) + resolve (per-fb quantise + square average,
 *     color.h:19-170: per pixel, hence rank-local) on its own host thread;
 *   - ONE collective: ncclGather of the ranks' 8-bit rows (padded to the largest share) to rank 0
 *     over xGMI, then rank 0's buffer is copied to the host and de-interleaved into PNG order.
 * Pixels depend only on global indices (RNG slot, seed), so the assembled image is byte-identical
 * to rt_draw's for every rank count and band size.
 *
 * Every function returns 0 (RT_OK) on success or an rt_status; nothing throws or exits.
 */
#ifndef RT_MULTI_H
#define RT_MULTI_H

#include "rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RT_GATHER_RCCL 0 /* ncclGather to rank 0 (one RCCL communicator, ncclCommInitAll; distinct devices) */
#define RT_GATHER_HOST 1 /* each rank's rows copied to the host instead (ranks may share a device: tests) */
#define RT_MULTI_MAX_RANKS 16

typedef struct rt_multi rt_multi;

typedef struct rt_multi_timing {
  float total_ms;                        /* whole draw, host clock                                  */
  float render_ms_max;                   /* slowest rank: render_init + render + resolve             */
  float gather_ms;                       /* the collective (or the host copies) + host assembly      */
  float gather_bytes;                    /* bytes gathered to rank 0 (n_ranks * padded rows * W * 3) */
  float render_ms[RT_MULTI_MAX_RANKS];   /* per rank, host clock around its render_init..resolve     */
  float kernel_ms[RT_MULTI_MAX_RANKS];   /* per rank, render kernel alone (HIP events)               */
  int32_t warm;                          /* 1: every rank's launch reused the item schedule of an
                                            earlier launch (rt_last_render_schedule & RT_SCHED_PREVIOUS) */
  int32_t pad;
} rt_multi_timing;

/* One context per rank on devices[rank]; RT_GATHER_RCCL also creates the RCCL communicator. */
int rt_multi_create(int32_t n_ranks, const int32_t* devices, int32_t gather_mode, rt_multi** out);
int rt_multi_destroy(rt_multi* m);
const char* rt_multi_last_error(const rt_multi* m);
/* Uploads the scene to every rank's context (rt_scene_upload). */
int rt_multi_upload(rt_multi* m, const rt_scene_soa* scene);
/* draw() over the ranks.  args: as rt_draw (band_rows = band size, >= 1; band_first / band_stride
 * are set per rank).  png_rgb_host: W*H*3 bytes, top row first.  counters / timing may be NULL
 * (counters are summed over ranks). */
int rt_multi_draw(rt_multi* m, const rt_render_args* args, uint8_t* png_rgb_host, rt_counters* counters,
                  rt_multi_timing* timing);

#ifdef __cplusplus
}
#endif

#endif /* RT_MULTI_H */
