"""Diagnostic: warm (split-sample replay) launch time of C2 against the split threshold
(context option split_min_segments), for the full frame and the rank-0 share of N = 8.

usage: diag_split.py [spp nfb thresholds...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import raytracing_gpu_amd as rt

spp, nfb = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (100, 1)
thr = sys.argv[3:] or ["default", "24", "100", "200", "400", "800", "100000"]
W, H = 1200, 800
ctx = rt.Context(0)
ctx.render_init(W, H, 1984)
sc = rt.Scene.builtin("big1")
for n in [int(x) for x in os.environ.get("DIAG_N", "1,8").split(",")]:
    args = rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=4, band_first=0, band_stride=n)
    fb = torch.empty(nfb * len(rt.owned_rows(args)) * W * 3, dtype=torch.float32, device="cuda")
    res = []
    for t in thr:
        ctx.set_options(split_min_segments=0.0 if t == "default" else float(t))
        ctx.upload(sc)  # new scene generation: the schedule (and its split set) is rebuilt
        ms = []
        for _ in range(5):
            ctx.render(args, fb.data_ptr())
            ms.append(ctx.last_render_ms())
        res.append(f"{t}: {min(ms[2:]):.2f}")
    print(f"N={n} {nfb}x{spp} warm ms by split threshold: " + ", ".join(res), flush=True)
