"""Diagnostic: phase shares of the render loop from a -DRT_DIAG=2 build (scripts/build_ab.sh stamps raytracing_gpu_amd/csrc/rt_kernels.hip -DRT_DIAG=2) (RT_HIP_LIB=<that .so>).

usage: diag_stamps.py scene W H spp nfb [nolds]
Shares only: the stamps' own fences change the run time (cdna_hip_programming.md section 7).
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import raytracing_gpu_amd as rt

PH = ["head/refill (step: sample end + refill)", "camera (step: camera + query setup)", "world glue", "node tests", "prim tests", "validation+finalize", "scatter", "one stamp (x trips)"]
scene = sys.argv[1]; W, H, spp, nfb = [int(x) for x in sys.argv[2:6]]
out = "/tmp/stamps.bin"
if os.path.exists(out):
    os.remove(out)
from bench import scene_assets
ctx = rt.Context(0); ctx.upload(rt.Scene.builtin(scene, **scene_assets(scene)[0])); ctx.render_init(W, H, 1984)
fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
os.environ["RT_STAMPS_OUT"] = out
c = ctx.render(rt.make_args(W, H, spp, 0, nfb, 50, 0, lds="nolds" not in sys.argv), fb.data_ptr())
a = np.fromfile(out, np.uint64).astype(np.float64)
tot = a.sum()
print(scene, W, H, spp, nfb, "segments", c["segments"], "stamp ticks/segment", round(tot / c["segments"], 1))
for k, n in enumerate(PH):
    print(f"  {n:22s} {100 * a[k] / tot:6.2f} %   {a[k] / c['segments']:9.1f} ticks/seg")
