"""Diagnostic: GPU vs oracle per variant for one scene; prints differing pixel counts."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import raytracing_gpu_amd as rt
from oracle import ref_cpu
scene = sys.argv[1]; W, H, spp, nfb = [int(x) for x in sys.argv[2:6]]
ctx = rt.Context(0); ctx.upload(rt.Scene.builtin(scene)); ctx.render_init(W, H, 1984)
ref = ref_cpu.RefScene(scene)
want = [ref.render(W, H, spp, f, 50, 0)[0].reshape(H, W, 3) for f in range(nfb)]
for name, kw in [("culled", {}), ("exact", {"exact": True}), ("nolds", {"lds": False}), ("stats", {"stats": True})]:
    fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
    c = ctx.render(rt.make_args(W, H, spp, 0, nfb, 50, 0, **kw), fb.data_ptr())
    g = fb.cpu().numpy().reshape(nfb, H, W, 3)
    d = sum(int((g[f].view(np.uint32) != want[f].view(np.uint32)).any(axis=2).sum()) for f in range(nfb))
    print(name, "diff pixels", d, "segments", c["segments"])
