"""Diagnostic: data for offline studies of first-launch item orders (scripts/sim_order.py).

Needs a diagnostic build with the item-cost and probe dumps (scripts/build_ab.sh diag
raytracing_gpu_amd/csrc/rt_kernels.hip -DRT_DIAG=8; RT_HIP_LIB=build/ab/libdiag.so).  For each
workload and share (rank r of N, 4-row bands) it runs a first launch probed at every pixel with the
full depth (options.probe_schedule = 1, probe_depth = 0: the raw probe count of every pixel, written
to $RT_PROBE_OUT) and a second launch, whose schedule build writes the first launch's real per-item
segment counts ($RT_ITEM_COST_OUT).  Also times the product's own first launch (default options) of
the share.  Output: gpurun_out/order/<tag>.npz (probe, cost) + <tag>.json.

usage: diag_order.py scene W H spp nfb N rank [N rank ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import raytracing_gpu_amd as rt
from bench import scene_assets  # noqa: E402

scene, W, H, spp, nfb = sys.argv[1], *[int(x) for x in sys.argv[2:6]]
shares = [(int(sys.argv[k]), int(sys.argv[k + 1])) for k in range(6, len(sys.argv), 2)] or [(1, 0)]
out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "order")
os.makedirs(out, exist_ok=True)
ctx = rt.Context(0)
ctx.upload(rt.Scene.builtin(scene, **scene_assets(scene)[0]))
ctx.render_init(64, 36, 1984)
_t = torch.empty(64 * 36 * 3, dtype=torch.float32, device="cuda")
ctx.render(rt.make_args(64, 36, 1, 0, 1, 50, 0), _t.data_ptr())
ctx.render_init(W, H, 1984)
for n, r in shares:
    tag = f"{scene}_{W}x{H}_{nfb}x{spp}_N{n}r{r}"
    args = rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=4, band_first=r, band_stride=n)
    fresh = rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=4, band_first=r, band_stride=n, fresh=True)
    rows = rt.owned_rows(args)
    fb = torch.empty(nfb * len(rows) * W * 3, dtype=torch.float32, device="cuda")
    ctx.set_options(reset=True)
    prod = []
    for _ in range(3):  # the product's first launch (default options)
        ctx.render(fresh, fb.data_ptr())
        prod.append((ctx.last_render_ms(), ctx.last_kernel_ms()))
    natural = []
    for _ in range(3):  # natural order
        ctx.render(rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=4, band_first=r, band_stride=n,
                                schedule=False), fb.data_ptr())
        natural.append((ctx.last_render_ms(), ctx.last_kernel_ms()))
    ctx.set_options(probe_schedule=1, probe_depth=0)
    os.environ["RT_PROBE_OUT"] = f"{out}/{tag}_probe.bin"
    c = ctx.render(fresh, fb.data_ptr())
    os.environ.pop("RT_PROBE_OUT")
    os.environ["RT_ITEM_COST_OUT"] = f"{out}/{tag}_cost.bin"
    ctx.render(args, fb.data_ptr())
    os.environ.pop("RT_ITEM_COST_OUT")
    warm = []
    for _ in range(3):
        ctx.render(args, fb.data_ptr())
        warm.append((ctx.last_render_ms(), ctx.last_kernel_ms(), ctx.last_render_schedule()))
    import numpy as np

    pr = np.fromfile(f"{out}/{tag}_probe.bin", dtype=np.uint16)
    co = np.fromfile(f"{out}/{tag}_cost.bin", dtype=np.uint16)
    np.savez_compressed(f"{out}/{tag}.npz", probe=pr, cost=co)
    os.remove(f"{out}/{tag}_probe.bin")
    os.remove(f"{out}/{tag}_cost.bin")
    meta = dict(scene=scene, W=W, H=H, spp=spp, nfb=nfb, N=n, rank=r, rows=[int(x) for x in rows],
                segments=c["segments"], product_cold=sorted(prod), natural=sorted(natural), warm=warm)
    json.dump(meta, open(f"{out}/{tag}.json", "w"))
    print(tag, "product cold (call, kernel) ms", sorted(prod)[1], "natural", sorted(natural)[1],
          "warm", sorted(warm)[0][:2], flush=True)
    del fb
