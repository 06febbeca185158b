"""Diagnostic: per-item segment counts of C2 (RT_ITEM_COST_OUT, written by the measuring launch).

usage: diag_items.py [stride]   rank 0 of `stride` ranks (4-row bands)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import raytracing_gpu_amd as rt

stride = int(sys.argv[1]) if len(sys.argv) > 1 else 1
W, H, spp, nfb = 1200, 800, 10, 10
out = "/tmp/item_cost.bin"
os.environ["RT_ITEM_COST_OUT"] = out
ctx = rt.Context(0)
ctx.upload(rt.Scene.builtin("big1"))
ctx.render_init(W, H, 1984)
args = rt.make_args(W, H, spp, 0, nfb, 50, 0, band_rows=4, band_first=0, band_stride=stride)
rows = rt.owned_rows(args)
fb = torch.empty(nfb * len(rows) * W * 3, dtype=torch.float32, device="cuda")
ctx.render(args, fb.data_ptr())
c = np.fromfile(out, np.uint16).astype(np.int64)
print(f"stride {stride}: {len(c)} items, {c.sum()} segments, mean {c.mean():.2f}")
for q in (50, 90, 99, 99.9, 99.99, 100):
    print(f"  p{q}: {np.percentile(c, q):.0f} segments")
srt = np.sort(c)[::-1]
print("  top 20:", srt[:20].tolist())
lanes = 256 * 1024
print(f"  segments per lane (full grid of {lanes} lanes): {c.sum() / lanes:.1f}")
