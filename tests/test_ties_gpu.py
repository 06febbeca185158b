"""GPU parity of the tie rules between and inside list entries, on the test scenes "coincident" and
"coincident_step" (rt_scene.cpp scene_coincident, restated in the oracle): xy_rects in one plane as a
list primitive, as members of a reference BVH and as a translate(rotate_y(.., 0)) instance, so world
queries meet exact ties across entries -- hittable_list.h:23-39 passes the closest hit so far as t_max
(inclusive), so the later entry wins -- and inside a BVH (bvh.h:348-436: the first visited wins).

The merged list-world search (world_search) collects every entry's candidates into one (winner,
second) pair; an exact candidate of another entry must bound `second` whichever of the two arrives
first, or a tie is taken as certain (take_candidate<true>).  Its visiting order is an upload option,
so both arrival orders run here, with the entry loop, the forced exact fallback, the world tree and
the stepwise kernel's trailing primitives.
"""
import functools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REF, PIX = 0, 1


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@functools.lru_cache(maxsize=None)
def _want(scene, W, H, spp, nfb, cam):
    from oracle import ref_cpu

    ref = ref_cpu.RefScene(scene)
    out = [ref.render(W, H, spp, f, 50, cam) for f in range(nfb)]
    return [o[0].reshape(H, W, 3) for o in out], sum(int(o[1]["segments"]) for o in out)


MODES = {  # name: (context options, make_args kwargs, kernel name prefix)
    "merged_distance": (dict(merged_search=0, merge_order=0), {}, "render_kernel<"),
    "merged_list": (dict(merged_search=0, merge_order=1), {}, "render_kernel<"),
    "merged_reversed": (dict(merged_search=0, merge_order=2), {}, "render_kernel<"),
    "fallback": (dict(merged_search=2), {}, "render_kernel<"),
    "entry_loop": (dict(merged_search=1), {}, "render_kernel<"),
    "world_tree": (dict(world_tree=1), {}, "render_step_kernel<"),
    "widest": ({}, dict(widest=True, lds=False), "render_kernel<"),
    "exact": ({}, dict(exact=True), "render_kernel<"),
}


@pytest.mark.parametrize("cam", [REF, PIX], ids=["ref", "per_pixel"])
@pytest.mark.parametrize("mode", list(MODES))
def test_coincident_list_entries_bit_exact(rtlib, gpu_ctx, ctx_opts, oracle, mode, cam):
    """List world (primitive, BVH, instance, ground sphere) with exact ties across the entries: every
    search mode and visiting order, full frame and a share, cold and scheduled launches."""
    import torch

    W, H, spp, nfb = 96, 54, 4, 2
    want, segs = _want("coincident", W, H, spp, nfb, cam)
    opts, kw, prefix = MODES[mode]
    ctx_opts(**opts)
    gpu_ctx.upload(rtlib.Scene.builtin("coincident"))  # the upload-time options apply here
    for band in ((H, 0, 1), (4, 1, 3)):
        args = rtlib.make_args(W, H, spp, 0, nfb, 50, cam, band_rows=band[0], band_first=band[1],
                               band_stride=band[2], **kw)
        rows = rtlib.owned_rows(args)
        for launch in range(3):
            gpu_ctx.render_init(W, H, 1984)
            fb = torch.full((nfb * len(rows) * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
            cnt = gpu_ctx.render(args, fb.data_ptr())
            assert gpu_ctx.last_render_kernel().startswith(prefix), gpu_ctx.last_render_kernel()
            got = fb.cpu().numpy().reshape(nfb, len(rows), W, 3)
            for f in range(nfb):
                diff = (_bits(got[f]) != _bits(want[f][rows])).any(axis=2)
                assert not diff.any(), f"{mode} band {band} launch {launch} fb {f}: {int(diff.sum())} px"
            if band[2] == 1:
                assert cnt["segments"] == segs


@pytest.mark.parametrize("cam", [REF, PIX], ids=["ref", "per_pixel"])
@pytest.mark.parametrize("mode", ["product", "global", "no_step", "exact"])
def test_coincident_step_world_bit_exact(rtlib, gpu_ctx, oracle, mode, cam):
    """The stepwise kernel's world shape (a BVH, then primitives tested after its settle with t_max =
    the closest hit so far): exact ties between the BVH's rects and the trailing rect, in LDS and
    global-memory variants, against the segment loop and the exact visit set."""
    import torch

    W, H, spp, nfb = 96, 54, 4, 2
    want, segs = _want("coincident_step", W, H, spp, nfb, cam)
    kw = {"product": {}, "global": dict(lds=False), "no_step": dict(step=False), "exact": dict(exact=True)}[mode]
    gpu_ctx.upload(rtlib.Scene.builtin("coincident_step"))
    args = rtlib.make_args(W, H, spp, 0, nfb, 50, cam, **kw)
    for launch in range(3):
        gpu_ctx.render_init(W, H, 1984)
        fb = torch.full((nfb * H * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
        cnt = gpu_ctx.render(args, fb.data_ptr())
        if mode in ("product", "global"):
            assert gpu_ctx.last_render_kernel().startswith("render_step_kernel<"), gpu_ctx.last_render_kernel()
        got = fb.cpu().numpy().reshape(nfb, H, W, 3)
        for f in range(nfb):
            diff = (_bits(got[f]) != _bits(want[f])).any(axis=2)
            assert not diff.any(), f"{mode} launch {launch} fb {f}: {int(diff.sum())} px"
        assert cnt["segments"] == segs
