"""Diagnostic: strong-scaling estimate of bench.py's N-GPU step on one GPU.

For N in 1, 2, 4, 8 and every rank r < N, times rank r's step pieces as bench.py runs them
(render_init, the render of its 4-row bands, resolve) with HIP events; the N-GPU step is bounded
below by max over ranks.  "cold" is a rank's first launch of its configuration (no item schedule yet: the reference's single
draw(); the median of three RT_FLAG_FRESH launches), "warm" the best of the 2nd and 3rd launch after
them (the 1st records the split items' sample-start states).  The gather
is modelled from its bytes (N x the largest share's 8-bit rows) at XGMI_GBS (default 64 GB/s,
a conservative all-gather rate for a few MB over xGMI) plus 30 us of collective latency.

usage: diag_scale.py [scene W H spp nfb] [--opt KEY=VALUE ...]   (context options, include/rt_hip.h)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import raytracing_gpu_amd as rt

from bench import parse_opts, scene_assets  # noqa: E402  (door mesh fixture, synthetic textures for C4 / C5)

argv = [x for x in sys.argv[1:]]
opt_items = []
while "--opt" in argv:
    k = argv.index("--opt")
    opt_items.append(argv[k + 1])
    del argv[k:k + 2]
scene, W, H, spp, nfb = (argv[0], *[int(x) for x in argv[1:5]]) if argv else ("big1", 1200, 800, 10, 10)
ctx = rt.Context(0)
if opt_items:
    ctx.set_options(**parse_opts(opt_items))

ctx.upload(rt.Scene.builtin(scene, **scene_assets(scene)[0]))
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]


def timed(fn):
    torch.cuda.synchronize()
    ev[0].record()
    fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1])


def host_timed(fn):  # render_init runs on the context's own stream: time it to a device-wide sync
    import time

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


# module load + first allocations on a tiny image (a different configuration), as bench.py does
ctx.render_init(64, 36, 1984)
_tfb = torch.empty(64 * 36 * 3, dtype=torch.float32, device="cuda")
ctx.render(rt.make_args(64, 36, 1, 0, 1, 50, 0), _tfb.data_ptr())
t_init = min(host_timed(lambda: ctx.render_init(W, H, 1984)) for _ in range(5))
xgmi = float(os.environ.get("XGMI_GBS", "64"))
base = None
for n in (1, 2, 4, 8):
    worst = 0.0
    worst_cold = 0.0
    segs = 0
    share_rows = 0
    for r in range(n):
        args = rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=4, band_first=r, band_stride=n,
                            bins=os.environ.get("DIAG_BINS", "1") != "0")
        rows = rt.owned_rows(args)
        fb = torch.empty(nfb * len(rows) * W * 3, dtype=torch.float32, device="cuda")
        img = torch.empty(len(rows) * W * 3, dtype=torch.uint8, device="cuda")
        fargs = rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=4, band_first=r, band_stride=n,
                             bins=os.environ.get("DIAG_BINS", "1") != "0", fresh=True)
        cold_ms, bits = [], []
        for _ in range(3):  # first launches of the configuration (RT_FLAG_FRESH): the median
            ctx.render(fargs, fb.data_ptr())
            cold_ms.append(ctx.last_render_ms())
            bits.append(ctx.last_render_schedule())
        ms = [sorted(cold_ms)[1]]
        for _ in range(3):  # the 1st builds the schedule and records split states, 2nd+ are warm
            c = ctx.render(args, fb.data_ptr())
            ms.append(ctx.last_render_ms())
            bits.append(ctx.last_render_schedule())
        t_res = min(timed(lambda: ctx.resolve(args, fb.data_ptr(), img.data_ptr())) for _ in range(3))
        worst = max(worst, min(ms[2:]) + t_res)
        worst_cold = max(worst_cold, ms[0] + t_res)
        share_rows = max(share_rows, len(rows))
        segs += c["segments"]
        if os.environ.get("VERBOSE"):
            print(f"   N={n} rank {r}: warm {min(ms[2:]):.2f} ms, cold {ms[0]:.2f} ms {[round(x, 2) for x in cold_ms]}, "
                  f"1st scheduled {ms[1]:.2f} ms, "
                  f"{c['segments']} segments, {c['segments'] / min(ms[2:]) / 1e3:.0f} Mrays/s, schedule bits {bits}", flush=True)
    gbytes = n * share_rows * W * 3 if n > 1 else 0
    t_gather = (gbytes / (xgmi * 1e6) + 0.03) if n > 1 else 0.0
    step = worst + t_init + t_gather
    cold = worst_cold + t_init + t_gather
    base = base or step
    print(f"N={n}: max rank render+resolve warm {worst:.2f} / cold {worst_cold:.2f} ms + init {t_init:.2f} ms "
          f"+ gather {t_gather:.3f} ms ({gbytes} B) = warm {step:.2f} / cold {cold:.2f} ms/step, "
          f"{segs / step / 1e3:.0f} Mrays/s, x{base / step:.2f} (cold x{base / cold:.2f})", flush=True)
