"""Diagnostic: list the pixels where the GPU (default variant) differs from the oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import raytracing_gpu_amd as rt
from oracle import ref_cpu
scene = sys.argv[1]; W, H, spp, nfb = [int(x) for x in sys.argv[2:6]]
ctx = rt.Context(0); ctx.upload(rt.Scene.builtin(scene)); ctx.render_init(W, H, 1984)
ref = ref_cpu.RefScene(scene)
fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
ctx.render(rt.make_args(W, H, spp, 0, nfb, 50, 0), fb.data_ptr())
g = fb.cpu().numpy().reshape(nfb, H, W, 3)
print("kernel", ctx.last_render_kernel())
for f in range(nfb):
    want = ref.render(W, H, spp, f, 50, 0)[0].reshape(H, W, 3)
    d = (g[f].view(np.uint32) != want.view(np.uint32)).any(axis=2)
    for j, i in zip(*np.nonzero(d)):
        print(f"fb {f} j {j} i {i} gpu {g[f, j, i]} ref {want[j, i]}")
