"""Diagnostic: render one scene repeatedly with forced-widest variants; count differing pixels vs the oracle.

usage: diag_repeat.py scene W H spp nfb reps mode[,mode...]   (modes: culled exact stats exact_stats nolds audit)
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import raytracing_gpu_amd as rt
from oracle import ref_cpu

MODES = {"culled": {}, "nolds": {"lds": False}, "exact": {"exact": True}, "stats": {"stats": True},
         "exact_stats": {"exact": True, "stats": True}, "audit": {"audit": True}}
scene = sys.argv[1]; W, H, spp, nfb, reps = [int(x) for x in sys.argv[2:7]]
modes = sys.argv[7].split(",")
ctx = rt.Context(0); ctx.upload(rt.Scene.builtin(scene)); ctx.render_init(W, H, 1984)
ref = ref_cpu.RefScene(scene)
want = np.stack([ref.render(W, H, spp, f, 50, 0)[0].reshape(H, W, 3) for f in range(nfb)])
for m in modes:
    res = []
    for _ in range(reps):
        fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
        ctx.render(rt.make_args(W, H, spp, 0, nfb, 50, 0, widest=True, **MODES[m]), fb.data_ptr())
        got = fb.cpu().numpy().reshape(nfb, H, W, 3)
        res.append(int((got.view(np.uint32) != want.view(np.uint32)).any(axis=3).sum()))
    print(os.environ.get("RT_HIP_LIB", "default"), m, "diff pixels per run:", res, flush=True)
