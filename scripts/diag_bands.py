"""Diagnostic: render-kernel time of one rank's share of a multi-GPU run (band tiling) on one GPU.

usage: diag_bands.py [scene W H spp nfb]   prints ms and Mrays/s for band_stride 1, 2, 4, 8 (rank 0)
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import raytracing_gpu_amd as rt

scene, W, H, spp, nfb = (sys.argv[1], *[int(x) for x in sys.argv[2:6]]) if len(sys.argv) > 1 else ("big1", 1200, 800, 10, 10)
ctx = rt.Context(0); ctx.upload(rt.Scene.builtin(scene)); ctx.render_init(W, H, 1984)
for stride in (1, 2, 4, 8):
    args = rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=8, band_first=0, band_stride=stride)
    rows = rt.owned_rows(args)
    fb = torch.empty(nfb * len(rows) * W * 3, dtype=torch.float32, device="cuda")
    ms = []
    for _ in range(3):
        c = ctx.render(args, fb.data_ptr())
        ms.append(ctx.last_render_ms())
    t = min(ms)
    print(f"{os.environ.get('RT_HIP_LIB', 'default')} stride {stride}: rows {len(rows)} {t:.2f} ms "
          f"{c['segments'] / t / 1e3:.0f} Mrays/s per GPU, x{stride} = {stride * c['segments'] / t / 1e3:.0f}", flush=True)
