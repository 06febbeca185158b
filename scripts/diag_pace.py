"""Diagnostic: per-segment pace of a lane when its wave has (almost) the GPU to itself.  Tiny images
(W x 1 pixels, one wave or less) with many samples: launch time / the longest item's segment count
is the serial time per segment of that item's lane.

usage: diag_pace.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import raytracing_gpu_amd as rt

out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
os.makedirs(out, exist_ok=True)
ctx = rt.Context(0)
ctx.upload(rt.Scene.builtin("big1"))
for W, H, spp, env in ((64, 1, 100, {}), (8, 1, 100, {}), (1, 1, 400, {}), (64, 1, 100, {"RT_SHADE_MIN": "1"}),
                       (8, 1, 100, {"RT_SHADE_MIN": "1"}), (1, 1, 400, {"RT_NO_LDS": "1"}), (640, 1, 100, {}),
                       (4096, 1, 100, {})):
    ctx.render_init(W, H, 1984)
    os.environ.update({k: v for k, v in env.items() if k.startswith("RT_SHADE")})
    args = rt.make_args(W, H, spp, 0, 1, 50, 0, lds="RT_NO_LDS" not in env)
    fb = torch.empty(W * H * 3, dtype=torch.float32, device="cuda")
    p = f"{out}/pace_cost.bin"
    ms = []
    for k in range(3):
        if k == 1:
            os.environ["RT_ITEM_COST_OUT"] = p
        c = ctx.render(args, fb.data_ptr())
        ms.append(ctx.last_render_ms())
        os.environ.pop("RT_ITEM_COST_OUT", None)
    for k in env:
        os.environ.pop(k, None)
    ic = np.fromfile(p, dtype=np.uint16).astype(np.int64)
    print(f"{W}x{H} x{spp} {env}: cold {ms[0]:.3f} ms, segments {c['segments']}, longest item {ic.max()}, "
          f"mean {ic.mean():.0f}: {ms[0] * 1e3 / ic.max():.2f} us per segment of the longest item "
          f"({ctx.last_render_kernel()})", flush=True)
