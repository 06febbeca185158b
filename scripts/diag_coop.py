"""Diagnostic: the cooperative tail search (context option coop_max, render_step_kernel<..|F_COOP> on
cold launches).  (1) Lone-lane pace: cold launches of tiny images (one wave or less) with many samples,
launch time per segment of the image's longest pixel chain, coop off and on.  (2) C2 shares (rank 0 of
N, 10 fb x 10 spp) cold, by coop_max.

usage: diag_coop.py [scene]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import raytracing_gpu_amd as rt
from bench import scene_assets  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "big1"
ctx = rt.Context(0)
ctx.upload(rt.Scene.builtin(scene, **scene_assets(scene)[0]))


def cold(W, H, spp, nfb, band=(4, 0, 1), coop=0, reps=3):
    ctx.set_options(coop_max=coop)
    ctx.render_init(W, H, 1984)
    args = rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=band[0], band_first=band[1], band_stride=band[2],
                        schedule=False)
    fb = torch.empty(nfb * len(rt.owned_rows(args)) * W * 3, dtype=torch.float32, device="cuda")
    ms = []
    for _ in range(reps):
        c = ctx.render(args, fb.data_ptr())
        ms.append(ctx.last_render_ms())
    return min(ms), c, ctx.last_render_kernel()


for W, H, spp in ((1, 1, 400), (8, 1, 100), (64, 1, 100), (640, 1, 50)):
    out = []
    for coop in (0, 64):
        ms, c, k = cold(W, H, spp, 1, band=(H, 0, 1), coop=coop)
        out.append(f"coop {coop}: {ms:.3f} ms, {c['segments']} segments ({k})")
    per = (f" -- 1x1: {out[0].split(' ms')[0].split(': ')[1]} / {out[1].split(' ms')[0].split(': ')[1]} ms for "
           f"{c['segments']} segments" if W * H == 1 else "")
    print(f"{W}x{H} x{spp}: " + "; ".join(out) + per, flush=True)

W, H = (1200, 800) if scene == "big1" else (1920, 1079)
spp, nfb = (10, 10) if scene == "big1" else (16, 16)
for n in (1, 4, 8):
    res = []
    for coop in (0, 1, 2, 4, 8, 16, 64):
        ms, c, k = cold(W, H, spp, nfb, band=(4, 0, n), coop=coop)
        res.append(f"{coop}: {ms:.2f}")
    print(f"{scene} N={n} rank 0 cold ms by coop_max: " + ", ".join(res), flush=True)
