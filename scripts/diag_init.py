"""Diagnostic: rt_render_init alone, K times per image size (time it under rocprofv3 --kernel-trace
--stats, or read the host-timed average this prints).

usage: diag_init.py [K]   (RT_HIP_LIB selects the library)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import raytracing_gpu_amd as rt

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = rt.Context(0)
for W, H in ((1200, 800), (1920, 1079), (3840, 2159)):
    ctx.render_init(W, H, 1984)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        ctx.render_init(W, H, 1984)
    torch.cuda.synchronize()
    print(f"{W}x{H}: {(time.perf_counter() - t0) / K * 1e3:.3f} ms per render_init (host-timed)", flush=True)
