"""Diagnostic: what C4's texel misses cost.  The door scene with its image texture at several sizes
(the synthetic image of bench.py, resized): scatter directions do not depend on the albedo, so the
paths and segment counts are the same and only the texels' footprint in L2 changes.

usage: diag_texsize.py [W H spp nfb]   (default C4: 1920 1079 16 16)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import raytracing_gpu_amd as rt
from raytracing_gpu_amd import assets

W, H, spp, nfb = [int(x) for x in sys.argv[1:5]] if len(sys.argv) > 4 else (1920, 1079, 16, 16)
m = assets.door_mesh_from_fixture(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "tests", "golden", "door_assimp.npz"))
ctx = rt.Context(0)
fb = torch.empty(nfb * H * W * 3, dtype=torch.float32, device="cuda")
for side in (2048, 1024, 512, 64):
    ctx.upload(rt.Scene.builtin("door", images=[assets.synthetic_image(side, side)], meshes=[m]))
    ctx.render_init(W, H, 1984)
    args = rt.make_args(W, H, spp, 0, nfb, 50, 0)
    ms = []
    for _ in range(5):
        c = ctx.render(args, fb.data_ptr())
        ms.append(ctx.last_render_ms())
    print(f"texture {side}x{side} ({3 * side * side / 1e6:.1f} MB): warm {min(ms[2:]):.2f} ms, "
          f"{c['segments']} segments, {ctx.last_render_kernel()}", flush=True)
