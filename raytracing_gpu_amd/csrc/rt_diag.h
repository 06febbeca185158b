// rt_diag.h — instrumentation of the render megakernels, compiled only into diagnostic builds.
//
// The product library (raytracing_gpu_amd/_build.py) defines nothing here: every hook below is an
// empty macro, the kernels carry no timing code and the library reads no environment variable.
// A diagnostic build sets -DRT_DIAG=<bits> (scripts/build_ab.sh NAME src -DRT_DIAG=...):
//   1  per-wave counts of traversal-loop iterations, lane steps, shading phases and loop trips
//      (printed to stderr after each launch)
//   2  per-wave cycle shares of the loop's phases: s_memtime stamps, appended to $RT_STAMPS_OUT
//      (scripts/diag_stamps.py)
//   4  per-wave start / work-exhausted / end times (s_memrealtime), written to $RT_WAVE_TIMES_OUT
//      (scripts/diag_waves.py)
//   8  every measuring launch's per-item segment counts, written to $RT_ITEM_COST_OUT, and every probe
//      launch's raw per-grid-point counts, written to $RT_PROBE_OUT (scripts/diag_pace.py,
//      scripts/diag_order.py)
// Bits 2 and 4 perturb the timing they measure; use one at a time.
#pragma once

#ifndef RT_DIAG
#define RT_DIAG 0
#endif

// ---------------------------------------------------------------- 1: step counts
#if RT_DIAG & 1
__device__ unsigned long long rt_diag_steps[4];
__shared__ unsigned long long rt_diag_steps_acc[16][4];
__device__ __forceinline__ void rt_step_count(int k) {  // one count per wave (first active lane)
  const unsigned long long act = __ballot(1);
  if ((int)__lane_id() == __ffsll((long long)act) - 1) {
    rt_diag_steps_acc[threadIdx.x >> 6][k] += 1;
    if (k == 0) rt_diag_steps_acc[threadIdx.x >> 6][1] += __popcll(act);
  }
}
#define RT_STEP_COUNT(k) rt_step_count(k)
#define RT_STEP_COUNT_BEGIN() \
  if (__lane_id() < 4) rt_diag_steps_acc[threadIdx.x >> 6][__lane_id()] = 0
#define RT_STEP_COUNT_END() \
  if (__lane_id() < 4) atomicAdd(&rt_diag_steps[__lane_id()], rt_diag_steps_acc[threadIdx.x >> 6][__lane_id()])
#define RT_STEP_COUNT_HOST_RESET()                                   \
  do {                                                               \
    const unsigned long long z_[4] = {0, 0, 0, 0};                   \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(rt_diag_steps), z_, sizeof(z_)); \
  } while (0)
#define RT_STEP_COUNT_HOST_PRINT(var)                                                                       \
  do {                                                                                                      \
    unsigned long long h_[4];                                                                               \
    (void)hipMemcpyFromSymbol(h_, HIP_SYMBOL(rt_diag_steps), sizeof(h_));                                   \
    fprintf(stderr, "RT_STEP_DIAG var=%d trav_wave_iters=%llu trav_lane_steps=%llu shade_phases=%llu trips=%llu\n", \
            var, h_[0], h_[1], h_[2], h_[3]);                                                               \
  } while (0)
#else
#define RT_STEP_COUNT(k)
#define RT_STEP_COUNT_BEGIN()
#define RT_STEP_COUNT_END()
#define RT_STEP_COUNT_HOST_RESET()
#define RT_STEP_COUNT_HOST_PRINT(var)
#endif

// ---------------------------------------------------------------- 2: phase stamps
// Phase = code run after the stamp: 0 head, 1 camera, 2 world glue, 3 node tests, 4 primitive tests,
// 5 validation, 6 scatter, 7 one stamp (a back-to-back pair measures the stamp itself).
#if RT_DIAG & 2
constexpr int kStampPhases = 8;
__device__ unsigned long long rt_diag_stamps[kStampPhases];
__shared__ unsigned long long rt_stamp_acc[16][kStampPhases + 2];
__device__ __forceinline__ void rt_stamp(int ph) {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long act = __ballot(1);
  if ((int)__lane_id() == __ffsll((long long)act) - 1) {
    unsigned long long* a = rt_stamp_acc[threadIdx.x >> 6];
    if (a[0] != 0) a[2 + a[1]] += t - a[0];
    a[0] = t;
    a[1] = (unsigned long long)ph;
  }
}
#define RT_STAMP(ph) rt_stamp(ph)
#define RT_STAMP_BEGIN()                                                              \
  do {                                                                                \
    if (__lane_id() < kStampPhases + 2) rt_stamp_acc[threadIdx.x >> 6][__lane_id()] = 0; \
    __syncthreads();                                                                  \
    rt_stamp(0);                                                                      \
  } while (0)
#define RT_STAMP_END()                                                                                       \
  do {                                                                                                       \
    rt_stamp(0);                                                                                             \
    if (__lane_id() < kStampPhases) atomicAdd(&rt_diag_stamps[__lane_id()], rt_stamp_acc[threadIdx.x >> 6][2 + __lane_id()]); \
  } while (0)
#define RT_STAMP_HOST_RESET()                                                 \
  do {                                                                        \
    const unsigned long long z_[kStampPhases] = {};                           \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(rt_diag_stamps), z_, sizeof(z_));      \
  } while (0)
#define RT_STAMP_HOST_WRITE()                                                       \
  do {                                                                              \
    unsigned long long h_[kStampPhases];                                            \
    (void)hipMemcpyFromSymbol(h_, HIP_SYMBOL(rt_diag_stamps), sizeof(h_));          \
    if (const char* p_ = getenv("RT_STAMPS_OUT"))                                   \
      if (FILE* f_ = fopen(p_, "ab")) {                                             \
        fwrite(h_, sizeof(h_), 1, f_);                                              \
        fclose(f_);                                                                 \
      }                                                                             \
  } while (0)
#else
#define RT_STAMP(ph)
#define RT_STAMP_BEGIN()
#define RT_STAMP_END()
#define RT_STAMP_HOST_RESET()
#define RT_STAMP_HOST_WRITE()
#endif

// ---------------------------------------------------------------- 4: wave timeline
#if RT_DIAG & 4
__device__ unsigned long long rt_wave_times[3 * 8192];  // per wave: start, global work exhausted, end
__device__ unsigned rt_wave_count;
__device__ __forceinline__ unsigned long long rt_realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define RT_WAVE_T0() const unsigned long long rt_wt0 = rt_realtime(); unsigned long long rt_wt1 = 0
#define RT_WAVE_EXHAUSTED() \
  if (rt_wt1 == 0) rt_wt1 = rt_realtime()
#define RT_WAVE_END()                                                                   \
  do {                                                                                  \
    const unsigned long long wt2_ = rt_realtime();                                      \
    const unsigned long long any1_ = __ballot(rt_wt1 != 0);                             \
    const unsigned long long e1_ = any1_ ? __shfl(rt_wt1, __ffsll((long long)any1_) - 1, 64) : 0ull; \
    if (__lane_id() == 0) {                                                             \
      const unsigned k_ = atomicAdd(&rt_wave_count, 1u);                                \
      if (k_ < 8192) {                                                                  \
        rt_wave_times[3 * k_] = rt_wt0;                                                 \
        rt_wave_times[3 * k_ + 1] = e1_;                                                \
        rt_wave_times[3 * k_ + 2] = wt2_;                                               \
      }                                                                                 \
    }                                                                                   \
  } while (0)
#define RT_WAVE_HOST_RESET()                                               \
  do {                                                                     \
    const unsigned z_ = 0;                                                 \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(rt_wave_count), &z_, sizeof(z_));   \
  } while (0)
#define RT_WAVE_HOST_WRITE()                                                                          \
  do {                                                                                                \
    if (const char* p_ = getenv("RT_WAVE_TIMES_OUT")) {                                               \
      std::vector<unsigned long long> wt_(3 * 8192);                                                  \
      unsigned n_ = 0;                                                                                \
      (void)hipMemcpyFromSymbol(&n_, HIP_SYMBOL(rt_wave_count), sizeof(n_));                          \
      (void)hipMemcpyFromSymbol(wt_.data(), HIP_SYMBOL(rt_wave_times), wt_.size() * sizeof(unsigned long long)); \
      if (FILE* f_ = fopen(p_, "wb")) {                                                               \
        fwrite(wt_.data(), sizeof(unsigned long long), 3 * (size_t)std::min(n_, 8192u), f_);          \
        fclose(f_);                                                                                   \
      }                                                                                               \
    }                                                                                                 \
  } while (0)
#else
#define RT_WAVE_T0()
#define RT_WAVE_EXHAUSTED()
#define RT_WAVE_END()
#define RT_WAVE_HOST_RESET()
#define RT_WAVE_HOST_WRITE()
#endif

// ---------------------------------------------------------------- 8: item costs
#if RT_DIAG & 8
#define RT_DIAG_ITEM_COSTS(c, items)                                                                  \
  do {                                                                                                \
    if (const char* p_ = getenv("RT_ITEM_COST_OUT")) {                                                \
      std::vector<uint16_t> ic_((size_t)(items));                                                     \
      HIPCHK(c, hipMemcpyAsync(ic_.data(), (c)->item_cost, ic_.size() * sizeof(uint16_t), hipMemcpyDeviceToHost, \
                               (c)->stream));                                                         \
      HIPCHK(c, hipStreamSynchronize((c)->stream));                                                   \
      if (FILE* f_ = fopen(p_, "wb")) {                                                               \
        fwrite(ic_.data(), sizeof(uint16_t), ic_.size(), f_);                                         \
        fclose(f_);                                                                                   \
      }                                                                                               \
    }                                                                                                 \
  } while (0)
#define RT_DIAG_PROBE_COSTS(c, n)                                                                     \
  do {                                                                                                \
    if (const char* p_ = getenv("RT_PROBE_OUT")) {                                                    \
      std::vector<uint16_t> pc_((size_t)(n));                                                         \
      HIPCHK(c, hipMemcpyAsync(pc_.data(), (c)->probe_cost, pc_.size() * sizeof(uint16_t), hipMemcpyDeviceToHost, \
                               (c)->stream));                                                         \
      HIPCHK(c, hipStreamSynchronize((c)->stream));                                                   \
      if (FILE* f_ = fopen(p_, "wb")) {                                                               \
        fwrite(pc_.data(), sizeof(uint16_t), pc_.size(), f_);                                         \
        fclose(f_);                                                                                   \
      }                                                                                               \
    }                                                                                                 \
  } while (0)
#else
#define RT_DIAG_ITEM_COSTS(c, items)
#define RT_DIAG_PROBE_COSTS(c, n)
#endif
