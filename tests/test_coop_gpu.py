"""GPU parity of the cooperative tail search (render_step_kernel<..|F_COOP>, the variant of cold
launches when the context option coop_max > 0): once the work counter is exhausted, a wave with at
most coop_max traversing lanes answers their queries with all 64 lanes, each testing every 64th leaf
of the world BVH's traversal tree, and combines the candidates across the wave.  The query's answer
must still be bvh.h:348-436's (the closest hit of the reference visit set, first visited on ties), so
every pixel and segment count equals the oracle's.  coop_max = 64 sends every tail query of the
launch through it.
"""
import functools
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REF, PIX = 0, 1
F_COOP = 1 << 18
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@functools.lru_cache(maxsize=None)
def _scene_kw(scene):
    from raytracing_gpu_amd import assets

    if scene != "door":
        return (), ()
    m = assets.door_mesh_from_fixture(os.path.join(GOLD, "door_assimp.npz"))
    img = assets.synthetic_image(1024, 1024)
    return (("images", (img,)), ("meshes", (m,))), (("images", (img,)), ("meshes", ((m.tris, True, 0),)))


@functools.lru_cache(maxsize=None)
def _want(scene, W, H, spp, nfb, cam):
    from oracle import ref_cpu

    oa = {k: list(v) for k, v in _scene_kw(scene)[1]}
    ref = ref_cpu.RefScene(scene, **oa)
    out = [ref.render(W, H, spp, f, 50, cam) for f in range(nfb)]
    return [o[0].reshape(H, W, 3) for o in out], sum(int(o[1]["segments"]) for o in out)


@pytest.mark.parametrize("coop_max", [8, 64])
@pytest.mark.parametrize("cam", [REF, PIX], ids=["ref", "per_pixel"])
@pytest.mark.parametrize("band", [(54, 0, 1), (4, 1, 3)], ids=["full", "share"])
@pytest.mark.parametrize("scene", ["big1", "coincident_step", "door", "triangles"])
def test_coop_cold_launch_bit_exact(rtlib, gpu_ctx, ctx_opts, oracle, scene, band, cam, coop_max):
    """Cold launches (no schedule) of the sphere (LDS), coincident-triangle and door (quantized LDS tree)
    worlds with the cooperative tail search, full frame and a share, against the oracle; then a warm
    launch of the same configuration (the plain variant) for the same bits."""
    import torch

    W, H, spp, nfb = 96, 54, 4, 2
    want, segs = _want(scene, W, H, spp, nfb, cam)
    ctx_opts(coop_max=coop_max)
    pa = {k: list(v) for k, v in _scene_kw(scene)[0]}
    gpu_ctx.upload(rtlib.Scene.builtin(scene, **pa))
    args = rtlib.make_args(W, H, spp, 0, nfb, 50, cam, band_rows=band[0], band_first=band[1], band_stride=band[2])
    rows = rtlib.owned_rows(args)
    for launch in range(3):
        gpu_ctx.render_init(W, H, 1984)
        fb = torch.full((nfb * len(rows) * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
        cnt = gpu_ctx.render(args, fb.data_ptr())
        name = gpu_ctx.last_render_kernel()
        mask = int(name.split("<")[1].rstrip(">"))
        assert name.startswith("render_step_kernel<") and bool(mask & F_COOP) == (launch == 0), (launch, name)
        got = fb.cpu().numpy().reshape(nfb, len(rows), W, 3)
        for f in range(nfb):
            diff = (_bits(got[f]) != _bits(want[f][rows])).any(axis=2)
            assert not diff.any(), f"{scene} launch {launch} fb {f}: {int(diff.sum())} pixels differ"
        if band[2] == 1:
            assert cnt["segments"] == segs
        assert cnt["samples"] == nfb * len(rows) * W * spp


@pytest.mark.parametrize("n,rank", [(8, 0), (8, 7), (1, 0)])
def test_coop_c2_share_equals_exact(rtlib, gpu_ctx, ctx_opts, n, rank):
    """C2's bench workload (1200x800, 10 fb x 10 spp) as rank `rank` of `n`, cold with the cooperative
    tail search at the product's bound and at 64: every float equals the reference visit set (exact
    traversal) over the whole share, same segment count."""
    import torch

    W, H, spp, nfb = 1200, 800, 10, 10
    gpu_ctx.upload(rtlib.Scene.builtin("big1"))
    kw = dict(band_rows=4, band_first=rank, band_stride=n)
    ex_args = rtlib.make_args(W, H, spp, 0, nfb, 50, REF, exact=True, **kw)
    rows = rtlib.owned_rows(ex_args)
    gpu_ctx.render_init(W, H, 1984)
    ex = torch.zeros(nfb * len(rows) * W * 3, dtype=torch.float32, device="cuda")
    ce = gpu_ctx.render(ex_args, ex.data_ptr())
    ex = ex.cpu().numpy()
    for cm in (8, 64):
        ctx_opts(coop_max=cm)
        args = rtlib.make_args(W, H, spp, 0, nfb, 50, REF, schedule=False, **kw)
        fb = torch.zeros(nfb * len(rows) * W * 3, dtype=torch.float32, device="cuda")
        cf = gpu_ctx.render(args, fb.data_ptr())
        assert int(gpu_ctx.last_render_kernel().split("<")[1].rstrip(">")) & F_COOP
        assert cf["segments"] == ce["segments"], cm
        assert np.array_equal(_bits(fb.cpu().numpy()), _bits(ex)), cm
