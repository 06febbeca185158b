"""Diagnostic: segment-by-segment trace of one pixel, GPU (library built with -DRT_TRACE) vs oracle.

usage: diag_trace.py scene W H spp nfb [flags: exact widest nolds stats]
Finds the first pixel of fb 0 whose colour differs and prints both ray sequences.
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import raytracing_gpu_amd as rt
from oracle import ref_cpu

scene = sys.argv[1]; W, H, spp, nfb = [int(x) for x in sys.argv[2:6]]
fl = set(sys.argv[6:])
FB = int(next((x[3:] for x in fl if x.startswith("fb=")), "0"))  # fb id to compare
kw = dict(exact="exact" in fl, widest="widest" in fl, lds="nolds" not in fl, stats="stats" in fl)
ctx = rt.Context(0); ctx.upload(rt.Scene.builtin(scene)); ctx.render_init(W, H, 1984)
ref = ref_cpu.RefScene(scene)
want = ref.render(W, H, spp, FB, 50, 0)[0].reshape(H, W, 3)
fb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
ctx.render(rt.make_args(W, H, spp, FB, 1, 50, 0, **kw), fb.data_ptr())
got = fb.cpu().numpy().reshape(H, W, 3)
d = np.argwhere((got.view(np.uint32) != want.view(np.uint32)).any(axis=2))
print("diff pixels", len(d))
if not len(d):
    sys.exit(0)
j, i = [int(x) for x in d[0]]
print("pixel", i, j, "gpu", got[j, i], "ref", want[j, i])
os.environ["RT_TRACE_ITEM"] = str(j * W + i)
os.environ["RT_TRACE_OUT"] = "/tmp/trace.bin"
ctx.render(rt.make_args(W, H, spp, FB, 1, 50, 0, **kw), fb.data_ptr())
t = np.fromfile("/tmp/trace.bin", np.float32).reshape(256, 16)
n = int(t[0].view(np.uint32)[0])
g = t[1:1 + min(n, 255)]
import ctypes
RL = ref_cpu.lib()
RL.ref_capture_rays.restype = ctypes.c_longlong
RL.ref_capture_rays.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
cap = np.zeros((100000, 8), np.float32)
RL.ref_capture_rays(cap.ctypes.data, len(cap))
segs = np.zeros(W * H, np.int32)
_, _, sp = ref.render(W, H, spp, FB, 50, 0, rows=(j, H), threads=1, seg_per_pixel=True)
ncap = RL.ref_capture_rays(None, 0)
before = int(sp[j * W:j * W + i].sum())
r = cap[before:before + int(sp[j * W + i])]
print("gpu segments", n, "ref segments", len(r))
for k in range(max(len(g), len(r))):
    gl = g[k] if k < len(g) else None
    rl = r[k] if k < len(r) else None
    same = gl is not None and rl is not None and (gl[:7].view(np.uint32) == rl[:7].view(np.uint32)).all()
    gs = "" if gl is None else (f"s{gl[14:16].view(np.int32)} o{gl[0:3]} d{gl[3:6]} t{gl[7]:.6g} mat{gl[8:9].view(np.int32)[0]} "
                                f"p{gl[9:12]} rng{gl[12:14].view(np.uint32)}")
    rs = "" if rl is None else f"o{rl[0:3]} d{rl[3:6]}"
    print(k, "OK " if same else "DIFF", gs, "| ref", rs)
