"""Diagnostic: wall-clock vs kernel time of the first launches of a configuration (host work per
launch: schedule build on launch 2, split claim order on launch 3).

usage: diag_launch.py [spp nfb]   (DIAG_N: shares, default 1,8)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import raytracing_gpu_amd as rt

spp, nfb = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (10, 10)
W, H = 1200, 800
ctx = rt.Context(0)
ctx.render_init(W, H, 1984)
sc = rt.Scene.builtin("big1")
for n in [int(x) for x in os.environ.get("DIAG_N", "1,8").split(",")]:
    args = rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=4, band_first=0, band_stride=n)
    fb = torch.empty(nfb * len(rt.owned_rows(args)) * W * 3, dtype=torch.float32, device="cuda")
    ctx.upload(sc)
    out = []
    for k in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.render(args, fb.data_ptr())
        torch.cuda.synchronize()
        out.append(f"{(time.perf_counter() - t0) * 1e3:.2f}/{ctx.last_render_ms():.2f}")
    print(f"N={n} {nfb}x{spp} launches wall/kernel ms: " + " ".join(out), flush=True)
