// rt_multi.cpp — multi-GPU draw() over one node (include/rt_multi.h): one rt_ctx per rank, row
// bands dealt round-robin, each rank renders + resolves its rows on its own persistent host thread,
// one RCCL gather of the 8-bit rows to rank 0 over xGMI, one DMA copy into pinned host memory, and
// the ranks' threads assemble the image in PNG row order.
//
// Replaces render.h:118-174 (draw) for a frame buffer tiled across GPUs.  The
// reference has no multi-GPU path; its per-pixel independence (RNG slot ((id+1)p+id+1) mod N and
// curand_init(1984, slot, 0) depend only on global indices, render.h:91,101) is what makes the
// tiling exact.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_multi.h"

struct rt_multi {
  int n = 0;
  int mode = RT_GATHER_RCCL;
  std::vector<int> dev;
  std::vector<rt_ctx*> ctx;
  std::vector<ncclComm_t> comm;
  std::vector<hipStream_t> stream;
  // per-rank device buffers, grown on demand
  std::vector<float*> fb;
  std::vector<uint8_t*> rows8;   // padded to max_rows * W * 3 bytes
  std::vector<size_t> fb_cap, rows_cap;
  uint8_t* gathered = nullptr;   // rank 0: n * padded bytes
  size_t gathered_cap = 0;
  uint8_t* host = nullptr;       // pinned host copy of the gathered rows (DMA, not a staged copy)
  size_t host_cap = 0;
  bool broken = false;  // a collective failed: the communicator is not reused
  std::string err;
  // One persistent host thread per rank (its device set once): a draw posts one job per phase
  // instead of creating threads.
  std::vector<std::thread> workers;
  std::mutex mu;
  std::condition_variable go, done;
  std::function<void(int)> job;
  unsigned long long gen = 0;
  int pending = 0;
  bool quit = false;
};

namespace {

int fail(rt_multi* m, int code, const std::string& msg) {
  if (m) m->err = msg;
  return code;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Runs job(r) on every rank's thread and waits for all of them.
void run_ranks(rt_multi* m, std::function<void(int)> job) {
  std::unique_lock<std::mutex> lk(m->mu);
  m->job = std::move(job);
  m->pending = m->n;
  ++m->gen;
  m->go.notify_all();
  m->done.wait(lk, [m] { return m->pending == 0; });
}

void worker(rt_multi* m, int r) {
  (void)hipSetDevice(m->dev[r]);
  unsigned long long seen = 0;
  for (;;) {
    std::function<void(int)> job;
    {
      std::unique_lock<std::mutex> lk(m->mu);
      m->go.wait(lk, [&] { return m->quit || m->gen != seen; });
      if (m->quit) return;
      seen = m->gen;
      job = m->job;
    }
    job(r);
    std::lock_guard<std::mutex> lk(m->mu);
    if (--m->pending == 0) m->done.notify_one();
  }
}

// grow a device buffer on `dev`
int grow(rt_multi* m, int dev, void** p, size_t* cap, size_t need) {
  if (need <= *cap) return RT_OK;
  if (hipSetDevice(dev) != hipSuccess) return fail(m, RT_ERR_HIP, "hipSetDevice");
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc(p, need) != hipSuccess) return fail(m, RT_ERR_NOMEM, "hipMalloc in rt_multi");
  *cap = need;
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_multi_create(int32_t n_ranks, const int32_t* devices, int32_t gather_mode, rt_multi** out) {
  if (!out || !devices || n_ranks < 1 || n_ranks > RT_MULTI_MAX_RANKS ||
      (gather_mode != RT_GATHER_RCCL && gather_mode != RT_GATHER_HOST))
    return RT_ERR_ARG;
  *out = nullptr;
  rt_multi* m = new rt_multi();
  m->n = n_ranks;
  m->mode = gather_mode;
  m->dev.assign(devices, devices + n_ranks);
  if (gather_mode == RT_GATHER_RCCL) {
    std::vector<int> s(m->dev);
    std::sort(s.begin(), s.end());
    if (std::adjacent_find(s.begin(), s.end()) != s.end()) {
      delete m;
      return RT_ERR_ARG;  // RCCL: one rank per device
    }
  }
  m->ctx.assign(n_ranks, nullptr);
  m->stream.assign(n_ranks, nullptr);
  m->fb.assign(n_ranks, nullptr);
  m->rows8.assign(n_ranks, nullptr);
  m->fb_cap.assign(n_ranks, 0);
  m->rows_cap.assign(n_ranks, 0);
  for (int r = 0; r < n_ranks; ++r) {
    int rc = rt_ctx_create(m->dev[r], &m->ctx[r]);
    if (rc == RT_OK && (hipSetDevice(m->dev[r]) != hipSuccess ||
                        hipStreamCreateWithFlags(&m->stream[r], hipStreamNonBlocking) != hipSuccess))
      rc = RT_ERR_HIP;
    if (rc != RT_OK) {
      rt_multi_destroy(m);
      return rc;
    }
  }
  if (gather_mode == RT_GATHER_RCCL) {
    m->comm.assign(n_ranks, nullptr);
    if (ncclCommInitAll(m->comm.data(), n_ranks, m->dev.data()) != ncclSuccess) {
      m->comm.clear();
      rt_multi_destroy(m);
      return RT_ERR_HIP;
    }
  }
  for (int r = 0; r < n_ranks; ++r) m->workers.emplace_back(worker, m, r);
  *out = m;
  return RT_OK;
}

int rt_multi_destroy(rt_multi* m) {
  if (!m) return RT_ERR_ARG;
  {
    std::lock_guard<std::mutex> lk(m->mu);
    m->quit = true;
    m->go.notify_all();
  }
  for (std::thread& t : m->workers) t.join();
  if (m->host) (void)hipHostFree(m->host);
  for (ncclComm_t c : m->comm)
    if (c) ncclCommDestroy(c);
  for (int r = 0; r < m->n; ++r) {
    (void)hipSetDevice(m->dev[r]);
    if (r < (int)m->fb.size() && m->fb[r]) (void)hipFree(m->fb[r]);
    if (r < (int)m->rows8.size() && m->rows8[r]) (void)hipFree(m->rows8[r]);
    if (r < (int)m->stream.size() && m->stream[r]) (void)hipStreamDestroy(m->stream[r]);
    if (r < (int)m->ctx.size() && m->ctx[r]) rt_ctx_destroy(m->ctx[r]);
  }
  if (m->gathered) {
    (void)hipSetDevice(m->dev[0]);
    (void)hipFree(m->gathered);
  }
  delete m;
  return RT_OK;
}

const char* rt_multi_last_error(const rt_multi* m) { return m ? m->err.c_str() : "null rt_multi"; }

int rt_multi_upload(rt_multi* m, const rt_scene_soa* scene) {
  if (!m || !scene) return RT_ERR_ARG;
  for (int r = 0; r < m->n; ++r) {
    const int rc = rt_scene_upload(m->ctx[r], scene);
    if (rc != RT_OK) return fail(m, rc, std::string("rank ") + std::to_string(r) + ": " + rt_last_error(m->ctx[r]));
  }
  return RT_OK;
}

int rt_multi_draw(rt_multi* m, const rt_render_args* args, uint8_t* png_rgb_host, rt_counters* counters,
                  rt_multi_timing* timing) {
  if (!m || !args || !png_rgb_host) return RT_ERR_ARG;
  if (args->band_rows < 1 || args->width <= 0 || args->height <= 0) return fail(m, RT_ERR_ARG, "bad args");
  const double t0 = now_ms();
  const int n = m->n, W = args->width, H = args->height;
  std::vector<rt_render_args> ra(n, *args);
  std::vector<std::vector<int32_t>> rows(n);
  int max_rows = 0;
  for (int r = 0; r < n; ++r) {
    ra[r].band_first = r;
    ra[r].band_stride = n;
    const int k = rt_owned_rows(&ra[r], nullptr);
    rows[r].resize((size_t)std::max(k, 0));
    if (k > 0) rt_owned_rows(&ra[r], rows[r].data());
    max_rows = std::max(max_rows, k);
  }
  if (max_rows <= 0) return fail(m, RT_ERR_ARG, "no rows");
  const size_t padded = (size_t)max_rows * W * 3;
  for (int r = 0; r < n; ++r) {
    const size_t fbb = (size_t)args->fb_count * std::max<size_t>(rows[r].size(), 1) * W * 3 * sizeof(float);
    int rc = grow(m, m->dev[r], (void**)&m->fb[r], &m->fb_cap[r], fbb);
    if (!rc) rc = grow(m, m->dev[r], (void**)&m->rows8[r], &m->rows_cap[r], padded);
    if (rc) return rc;
  }
  if (m->mode == RT_GATHER_RCCL) {
    int rc = grow(m, m->dev[0], (void**)&m->gathered, &m->gathered_cap, padded * n);
    if (rc) return rc;
  }

  if (padded * n > m->host_cap) {
    if (m->host) (void)hipHostFree(m->host);
    m->host = nullptr;
    m->host_cap = 0;
    if (hipHostMalloc((void**)&m->host, padded * n, hipHostMallocDefault) != hipSuccess)
      return fail(m, RT_ERR_NOMEM, "hipHostMalloc in rt_multi");
    m->host_cap = padded * n;
  }

  // ---- every rank: render_init + render + resolve of its rows, on its own host thread (host
  // gather: its rows copied into the pinned buffer too)
  std::vector<int> status(n, RT_OK);
  std::vector<rt_counters> cnt(n);
  std::vector<double> rms(n, 0.0);
  std::vector<float> kms(n, 0.0f);
  std::vector<int> sched(n, 0);  // rt_last_render_schedule of each rank's launch
  run_ranks(m, [&](int r) {
    const double a = now_ms();
    rt_ctx* c = m->ctx[r];
    if (rows[r].empty()) {  // nothing to render: its (ignored) gather slot is zeros, not stale bytes
      status[r] = hipMemset(m->rows8[r], 0, padded) == hipSuccess ? RT_OK : RT_ERR_HIP;
      return;
    }
    int rc = rt_render_init(c, W, H, args->seed);
    if (!rc) rc = rt_render(c, &ra[r], m->fb[r], &cnt[r]);
    if (!rc) {
      kms[r] = rt_last_render_ms(c);
      sched[r] = rt_last_render_schedule(c);
    }
    if (!rc) rc = rt_resolve(c, &ra[r], m->fb[r], m->rows8[r]);
    if (!rc && m->mode == RT_GATHER_HOST &&
        hipMemcpy(m->host + padded * r, m->rows8[r], rows[r].size() * W * 3, hipMemcpyDeviceToHost) != hipSuccess)
      rc = RT_ERR_HIP;
    status[r] = rc;
    rms[r] = now_ms() - a;
  });
  for (int r = 0; r < n; ++r)
    if (status[r] != RT_OK)
      return fail(m, status[r], std::string("rank ") + std::to_string(r) + ": " + rt_last_error(m->ctx[r]));

  // ---- one gather of the padded 8-bit rows to rank 0
  const double g0 = now_ms();
  if (m->mode == RT_GATHER_RCCL) {
    if (m->broken) return fail(m, RT_ERR_STATE, "an earlier collective failed: destroy this rt_multi");
    if (ncclGroupStart() != ncclSuccess) return fail(m, RT_ERR_HIP, "ncclGroupStart");
    // the group is always closed, whatever fails inside it: a thread left inside an open RCCL group
    // would fold its next collectives into this one
    int gerr = -1;
    for (int r = 0; r < n && gerr < 0; ++r) {
      (void)hipSetDevice(m->dev[r]);
      if (ncclGather(m->rows8[r], r == 0 ? m->gathered : nullptr, padded, ncclUint8, 0, m->comm[r], m->stream[r]) !=
          ncclSuccess)
        gerr = r;
    }
    const bool end_ok = ncclGroupEnd() == ncclSuccess;
    bool sync_ok = true;
    for (int r = 0; r < n; ++r) {  // every rank's stream drained, also after a failure
      (void)hipSetDevice(m->dev[r]);
      if (hipStreamSynchronize(m->stream[r]) != hipSuccess) sync_ok = false;
    }
    if (gerr >= 0 || !end_ok || !sync_ok) {
      m->broken = true;  // the communicator's state is unknown after a failed collective
      return fail(m, RT_ERR_HIP, gerr >= 0 ? "ncclGather (rank " + std::to_string(gerr) + ")"
                                           : (!end_ok ? "ncclGroupEnd" : "gather sync"));
    }
    (void)hipSetDevice(m->dev[0]);
    if (hipMemcpy(m->host, m->gathered, padded * n, hipMemcpyDeviceToHost) != hipSuccess)
      return fail(m, RT_ERR_HIP, "copy gathered rows");
  }
  // ---- assembly: owned row j (0 = bottom) goes to PNG row H-1-j; each rank's thread copies its rows
  const size_t rowb = (size_t)W * 3;
  run_ranks(m, [&](int r) {
    for (size_t q = 0; q < rows[r].size(); ++q)
      memcpy(png_rgb_host + (size_t)(H - 1 - rows[r][q]) * rowb, m->host + padded * r + q * rowb, rowb);
  });
  const double g1 = now_ms();

  if (counters) {
    memset(counters, 0, sizeof(*counters));
    for (int r = 0; r < n; ++r) {
      counters->segments += cnt[r].segments;
      counters->node_tests += cnt[r].node_tests;
      counters->prim_tests += cnt[r].prim_tests;
      counters->samples += cnt[r].samples;
      counters->fallbacks += cnt[r].fallbacks;
    }
  }
  if (timing) {
    memset(timing, 0, sizeof(*timing));
    for (int r = 0; r < n; ++r) {
      timing->render_ms[r] = (float)rms[r];
      timing->kernel_ms[r] = kms[r];
      timing->render_ms_max = std::max(timing->render_ms_max, (float)rms[r]);
    }
    timing->gather_ms = (float)(g1 - g0);
    timing->gather_bytes = (float)(padded * n);
    timing->total_ms = (float)(now_ms() - t0);
    int warm = 1;
    for (int r = 0; r < n; ++r)
      if (!rows[r].empty() && (sched[r] & RT_SCHED_PREVIOUS) == 0) warm = 0;
    timing->warm = warm;
  }
  return RT_OK;
}

}  // extern "C"
