"""Diagnostic: wave timeline of one render launch from a -DRT_DIAG=4 build (RT_HIP_LIB=<that .so>).

usage: diag_waves.py [stride]   C2, rank 0 of `stride` ranks (4-row bands); prints when waves see the
global work counter exhausted and when they end, relative to the first wave's start.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import raytracing_gpu_amd as rt

stride = int(sys.argv[1]) if len(sys.argv) > 1 else 8
W, H, spp, nfb = 1200, 800, 10, 10
ctx = rt.Context(0)
ctx.upload(rt.Scene.builtin("big1"))
ctx.render_init(W, H, 1984)
args = rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=4, band_first=0, band_stride=stride)
rows = rt.owned_rows(args)
fb = torch.empty(nfb * len(rows) * W * 3, dtype=torch.float32, device="cuda")
out = "/tmp/wave_times.bin"
for k in range(4):
    if k == 3:
        os.environ["RT_WAVE_TIMES_OUT"] = out
    ctx.render(args, fb.data_ptr())
ms = ctx.last_render_ms()
t = np.fromfile(out, np.uint64).astype(np.float64).reshape(-1, 3)
t0 = t[:, 0].min()
st, ex, en = t[:, 0] - t0, t[:, 1] - t0, t[:, 2] - t0
hz = en.max() / (ms * 1e-3)  # s_memtime rate, taking the last wave's end as the launch end


def f(x):
    return x / hz * 1e3


print(f"stride {stride}: {len(t)} waves, kernel {ms:.2f} ms, memtime {hz / 1e6:.0f} MHz (derived)")
print(f"  start max {f(st.max()):.3f} ms; work exhausted: first {f(ex[t[:, 1] > 0].min()):.3f} ms, "
      f"median {f(np.median(ex[t[:, 1] > 0])):.3f} ms")
for q in (10, 50, 90, 99, 100):
    print(f"  wave end p{q}: {f(np.percentile(en, q)):.3f} ms")
