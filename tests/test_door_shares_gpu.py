"""GPU parity of C4's product shape: the door mesh on the quantized-LDS-tree stepwise kernel
(render_step_kernel<F_MESH|F_STEP|F_QLDS>) in the launches the C4 bench and its 4-GPU tiling run --
cold, scheduled (longest first) and split-sample launches, as rank r of N.

Pixel results depend only on global indices -- the RNG slot ((id+1) p + id+1) mod W*H and
curand_init(1984, slot, 0), render.h:91,101 -- so every owned row must equal the oracle's full-frame
row bit for bit on every launch.  The traversal being checked is bvh.h:348-436 over the triangles of
triangle.h:120-178 (the reference's H16 duplicates included), with the ground sphere after the mesh in
the world list (hittable_list.h:23-39).
"""
import functools
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REF, PIX = 0, 1
GOLD = os.path.join(os.path.dirname(__file__), "golden")
F_QLDS = 1 << 16


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@functools.lru_cache(maxsize=None)
def _door_assets(tex_w, tex_h):
    from raytracing_gpu_amd import assets

    m = assets.door_mesh_from_fixture(os.path.join(GOLD, "door_assimp.npz"))
    img = assets.synthetic_image(tex_w, tex_h)
    return m, img


@functools.lru_cache(maxsize=None)
def _oracle_frames(W, H, spp, nfb, cam, tex):
    """The oracle's full frames of the door scene (cached across the tests of this module)."""
    from oracle import ref_cpu

    m, img = _door_assets(*tex)
    ref = ref_cpu.RefScene("door", images=[img], meshes=[(m.tris, True, 0)])
    return [ref.render(W, H, spp, f, 50, cam)[0].reshape(H, W, 3) for f in range(nfb)]


def _upload_door(rtlib, ctx, tex):
    m, img = _door_assets(*tex)
    ctx.upload(rtlib.Scene.builtin("door", images=[img], meshes=[m]))  # a new scene generation: cold schedule


def _launches(rtlib, ctx, W, H, spp, nfb, cam, band, n):
    """n launches of one configuration (the first cold; n may be a list of flags: True = an
    RT_FLAG_FRESH launch, one that forgets the schedule first); yields (frame buffer [nfb, rows, W, 3], rows,
    counters, schedule bits) per launch, after checking the product kernel ran."""
    import torch

    args = rtlib.make_args(W, H, spp, 0, nfb, 50, cam, band_rows=band[0], band_first=band[1], band_stride=band[2])
    fresh = rtlib.make_args(W, H, spp, 0, nfb, 50, cam, band_rows=band[0], band_first=band[1], band_stride=band[2],
                            fresh=True)
    rows = rtlib.owned_rows(args)
    for k in range(n if isinstance(n, int) else len(n)):
        a = args if isinstance(n, int) or not n[k] else fresh
        ctx.render_init(W, H, 1984)
        fb = torch.full((nfb * len(rows) * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
        cnt = ctx.render(a, fb.data_ptr())
        name = ctx.last_render_kernel()
        assert name.startswith("render_step_kernel<") and int(name.split("<")[1].rstrip(">")) & F_QLDS, name
        yield fb.cpu().numpy().reshape(nfb, len(rows), W, 3), rows, cnt, ctx.last_render_schedule()


@pytest.mark.parametrize("n,rank", [(4, 0), (4, 3), (2, 1)])
def test_door_share_every_row(rtlib, gpu_ctx, oracle, n, rank):
    """C4's scene at 640x360, 4 fb x 4 spp, as rank `rank` of `n` (4-row bands): cold, scheduled and
    split launches against the oracle's full frame on every owned row, with equal segment counts."""
    W, H, spp, nfb, tex = 640, 360, 4, 4, (2048, 2048)
    want = _oracle_frames(W, H, spp, nfb, REF, tex)
    _upload_door(rtlib, gpu_ctx, tex)
    seen, segs = [], set()
    for k, (got, rows, cnt, sched) in enumerate(_launches(rtlib, gpu_ctx, W, H, spp, nfb, REF, (4, rank, n), 4)):
        seen.append(sched)
        segs.add(cnt["segments"])
        for f in range(nfb):
            diff = (_bits(got[f]) != _bits(want[f][rows])).any(axis=2)
            assert not diff.any(), f"door rank {rank}/{n} launch {k} fb {f}: {int(diff.sum())} pixels differ"
        assert cnt["samples"] == nfb * len(rows) * W * spp
    assert seen[0] == rtlib.RT_SCHED_PROBE and all(s & rtlib.RT_SCHED_PREVIOUS for s in seen[1:]), seen
    assert len(segs) == 1


@pytest.mark.parametrize("probe", [4, 1, 0], ids=["probe_grid4", "probe_every_pixel", "no_probe"])
@pytest.mark.parametrize("cam", [REF, PIX], ids=["ref", "per_pixel"])
def test_door_fresh_launches(rtlib, gpu_ctx, ctx_opts, oracle, cam, probe):
    """One-shot draws (RT_FLAG_FRESH) between scheduled ones, rank 3 of 4: a fresh launch runs as the
    configuration's first (probe launch on every probe-th row and pixel into the first fb slice,
    items longest first by its estimate; options.probe_schedule = 0: natural order) and the launch
    after it builds the schedule from the fresh launch's real counts.  Every launch equals the oracle
    bit for bit."""
    W, H, spp, nfb, tex = 320, 180, 4, 2, (1024, 1024)
    want = _oracle_frames(W, H, spp, nfb, cam, tex)
    ctx_opts(probe_schedule=probe)
    _upload_door(rtlib, gpu_ctx, tex)
    pattern = [True, False, False, True, False, True]
    seen, segs = [], set()
    for k, (got, rows, cnt, sched) in enumerate(_launches(rtlib, gpu_ctx, W, H, spp, nfb, cam, (4, 3, 4), pattern)):
        seen.append(sched)
        segs.add(cnt["segments"])
        for f in range(nfb):
            assert np.array_equal(_bits(got[f]), _bits(want[f][rows])), f"launch {k} fb {f}"
        assert cnt["samples"] == nfb * len(rows) * W * spp
    first = rtlib.RT_SCHED_PROBE if probe else 0
    assert [s == first for s in seen] == pattern, seen
    assert seen[1] & rtlib.RT_SCHED_PREVIOUS and seen[4] & rtlib.RT_SCHED_PREVIOUS, seen
    assert len(segs) == 1


@pytest.mark.parametrize("cam", [REF, PIX], ids=["ref", "per_pixel"])
@pytest.mark.parametrize("min_segs", [0.0, 1.0], ids=["default", "every_item"])
@pytest.mark.parametrize("band", [(54, 0, 1), (4, 1, 3), (4, 3, 4)], ids=["full", "share3", "share4"])
def test_door_split_samples_bit_exact(rtlib, gpu_ctx, ctx_opts, oracle, band, min_segs, cam):
    """Split samples on the quantized-tree kernel: launch 1 measures, launch 2 records the sample-start
    RNG states, launches 3+ run the split samples as separate work items and merge them in sample
    order.  Every launch equals the oracle bit for bit, in both camera modes, full frame and shares,
    at the product's threshold and with every item split."""
    W, H, spp, nfb, tex = 96, 54, 4, 2, (1024, 1024)
    want = _oracle_frames(W, H, spp, nfb, cam, tex)
    ctx_opts(split_min_segments=min_segs)
    _upload_door(rtlib, gpu_ctx, tex)
    seen = set()
    for k, (got, rows, cnt, sched) in enumerate(_launches(rtlib, gpu_ctx, W, H, spp, nfb, cam, band, 4)):
        seen.add(sched)
        for f in range(nfb):
            assert np.array_equal(_bits(got[f]), _bits(want[f][rows])), f"launch {k} fb {f}"
        assert cnt["samples"] == nfb * len(rows) * W * spp
    if min_segs:
        assert rtlib.RT_SCHED_PREVIOUS | rtlib.RT_SCHED_SPLIT_REPLAY in seen, seen


def test_door_full_size_share_rows(rtlib, gpu_ctx, oracle):
    """C4 at its image size as rank 3 of its 4 GPUs: 1920x1079, 2 fb x 2 spp, every launch of the share
    (cold, scheduled, split) against the oracle on a subset of the owned rows."""
    W, H, spp, nfb, tex = 1920, 1079, 2, 2, (2048, 2048)
    n, rank = 4, 3
    sub = (4 * rank + 1, 4 * n * 9)  # rows 13, 157, ...: all in band 3 mod 4
    js = list(range(sub[0], H, sub[1]))
    from oracle import ref_cpu

    m, img = _door_assets(*tex)
    ref = ref_cpu.RefScene("door", images=[img], meshes=[(m.tris, True, 0)])
    want = [ref.render(W, H, spp, f, 50, REF, rows=sub)[0].reshape(H, W, 3) for f in range(nfb)]
    _upload_door(rtlib, gpu_ctx, tex)
    for k, (got, rows, _, _) in enumerate(_launches(rtlib, gpu_ctx, W, H, spp, nfb, REF, (4, rank, n), 4)):
        pos = {int(j): q for q, j in enumerate(rows)}
        q = [pos[j] for j in js]
        for f in range(nfb):
            assert np.array_equal(_bits(got[f][q]), _bits(want[f][js])), f"launch {k} fb {f}"


def test_door_bench_share_equals_exact(rtlib, gpu_ctx):
    """C4's bench configuration as rank 3 of 4 (1920x1079, 16 fb x 16 spp: 31.7 items per resident lane,
    the split rule's 48-segment band): every launch -- cold, scheduled, split -- equals the reference
    visit set (exact traversal) over the whole share, every float, same segment count."""
    import torch

    W, H, spp, nfb, tex = 1920, 1079, 16, 16, (2048, 2048)
    band = (4, 3, 4)
    _upload_door(rtlib, gpu_ctx, tex)
    ex_args = rtlib.make_args(W, H, spp, 0, nfb, 50, REF, band_rows=4, band_first=3, band_stride=4, exact=True)
    rows = rtlib.owned_rows(ex_args)
    gpu_ctx.render_init(W, H, 1984)
    ex = torch.zeros(nfb * len(rows) * W * 3, dtype=torch.float32, device="cuda")
    ce = gpu_ctx.render(ex_args, ex.data_ptr())
    ex = ex.cpu().numpy().reshape(nfb, len(rows), W, 3)
    seen = []
    for k, (got, _, cnt, sched) in enumerate(_launches(rtlib, gpu_ctx, W, H, spp, nfb, REF, band, 4)):
        seen.append(sched)
        assert cnt["segments"] == ce["segments"], f"launch {k}"
        assert np.array_equal(_bits(got), _bits(ex)), f"launch {k}"
    assert seen[-1] == rtlib.RT_SCHED_PREVIOUS | rtlib.RT_SCHED_SPLIT_REPLAY, seen
