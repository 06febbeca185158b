"""Diagnostic: per-segment pace of a lane when its wave has (almost) the GPU to itself.  Tiny images
(W x 1 pixels, one wave or less) with many samples: launch time / the longest item's segment count
is the serial time per segment of that item's lane.  Needs a diagnostic build with the item-cost
dump (scripts/build_ab.sh pace raytracing_gpu_amd/csrc/rt_kernels.hip -DRT_DIAG=8; RT_HIP_LIB=...).

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
for W, H, spp, env in ((64, 1, 100, {}), (8, 1, 100, {}), (1, 1, 400, {}), (64, 1, 100, {"shade_min": 1}),
                       (8, 1, 100, {"shade_min": 1}), (1, 1, 400, {"no_lds": 1}), (640, 1, 100, {}),
                       (4096, 1, 100, {})):
    ctx.render_init(W, H, 1984)
    ctx.set_options(shade_min=env.get("shade_min", 0))
    args = rt.make_args(W, H, spp, 0, 1, 50, 0, lds="no_lds" not in env)
    fb = torch.empty(W * H * 3, dtype=torch.float32, device="cuda")
    p = f"{out}/pace_cost.bin"
    ms = []
    for k in range(3):
        if k == 1:
            os.environ["RT_ITEM_COST_OUT"] = p
        c = ctx.render(args, fb.data_ptr())
        ms.append(ctx.last_render_ms())
        os.environ.pop("RT_ITEM_COST_OUT", None)
    ic = np.fromfile(p, dtype=np.uint16).astype(np.int64)
    print(f"{W}x{H} x{spp} {env}: cold {ms[0]:.3f} ms, segments {c['segments']}, longest item {ic.max()}, "
          f"mean {ic.mean():.0f}: {ms[0] * 1e3 / ic.max():.2f} us per segment of the longest item "
          f"({ctx.last_render_kernel()})", flush=True)
