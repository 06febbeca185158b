"""Diagnostic: cold (single draw) vs warm launches of one configuration, full frame (N = 1) and the
rank-0 share of N = 8; then the per-item segment-count distribution (the longest item bounds a
cold launch: a lane runs an item's samples serially).

The item-cost dump needs a diagnostic build (scripts/build_ab.sh cold raytracing_gpu_amd/csrc/rt_kernels.hip
-DRT_DIAG=8; RT_HIP_LIB=build/ab/libcold.so); the launch times do not.

usage: diag_cold.py [scene W H spp nfb]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import raytracing_gpu_amd as rt

scene, W, H, spp, nfb = (sys.argv[1], *[int(x) for x in sys.argv[2:6]]) if len(sys.argv) > 1 else ("big1", 1200, 800, 10, 10)
ctx = rt.Context(0)
ctx.upload(rt.Scene.builtin(scene))
ctx.render_init(W, H, 1984)
out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
os.makedirs(out, exist_ok=True)


def launch(args, env=None):
    env = env or {}
    for k, v in env.items():
        os.environ[k] = v
    fb = torch.empty(args.fb_count * len(rt.owned_rows(args)) * W * 3, dtype=torch.float32, device="cuda")
    c = ctx.render(args, fb.data_ptr())
    for k in env:
        del os.environ[k]
    return ctx.last_render_ms(), c


for n in (1, 8):
    band = dict(band_rows=4, band_first=0, band_stride=n)
    nat = rt.make_args(W, H, spp, 0, nfb, 50, 0, schedule=False, **band)
    res = {}
    res["cold"] = min(launch(nat)[0] for _ in range(2))
    warm = rt.make_args(W, H, spp, 0, nfb, 50, 0, **band)
    nosplit = rt.make_args(W, H, spp, 0, nfb, 50, 0, split=False, **band)
    ms = [launch(warm, {"RT_ITEM_COST_OUT": f"{out}/item_cost_n{n}.bin"})[0] for _ in range(4)]
    res["warm_first"] = ms[0]
    res["warm"] = min(ms[2:])
    res["warm_nosplit"] = min(launch(nosplit)[0] for _ in range(2))
    print(f"N={n} share ({scene} {W}x{H} {nfb}x{spp}): " + ", ".join(f"{k} {v:.2f}" for k, v in res.items()), flush=True)
    p = f"{out}/item_cost_n{n}.bin"
    if os.path.exists(p):
        ic = np.fromfile(p, dtype=np.uint16).astype(np.int64)
        q = np.percentile(ic, [50, 90, 99, 99.9, 99.99])
        top = np.sort(ic)[-8:]
        lanes = 256 * 1024
        print(f"   items {ic.size} ({ic.size / lanes:.2f} per resident lane), segments {ic.sum()} "
              f"({ic.sum() / lanes:.0f} per lane), item p50/p90/p99/p99.9/p99.99 {q.round(0).tolist()}, "
              f"longest {top.tolist()}", flush=True)
