"""GPU parity of multi-GPU shares on the list-world kernel (render_kernel): the shapes C3 and C5 run
in as ranks of a multi-GPU draw.

A rank owns the 4-row bands b with b % N == rank (rt_owned_rows; band_first = rank, band_stride =
N).  Pixel results depend only on global indices -- the RNG slot ((id+1) p + id+1) mod W*H and
curand_init(1984, slot, 0), render.h:91,101 -- so every owned row must equal the oracle's full-frame
row bit for bit, on the cold launch and on the scheduled (longest-first) launches that follow it.
Share-size dependent paths exercised here: the camera-ray entry masks of list worlds
(bin_masks_kernel), the item schedule of a small share, and the step kernel's camera-list threshold
(options.bins_min_items_per_lane) on both sides of its switch.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REF = 0
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _assets(scene, tex_shape):
    """(product scene kwargs, oracle scene kwargs): the door mesh fixture and a synthetic texture of
    the real file's shape (the reference's files are not on a GPU box)."""
    from raytracing_gpu_amd import assets

    if scene not in ("final", "door"):
        return {}, {}
    m = assets.door_mesh_from_fixture(os.path.join(GOLD, "door_assimp.npz"))
    img = assets.synthetic_image(*tex_shape)
    return dict(images=[img], meshes=[m]), dict(images=[img], meshes=[(m.tris, True, 0)])


def _share(rtlib, ctx, W, H, spp, nfb, band, launches, kernel_prefix, cam=REF):
    """Render one rank's share `launches` times (cold, then scheduled); returns the last frame buffer
    as [nfb, owned rows, W, 3], the owned rows, and every launch's counters and schedule bits."""
    import torch

    args = rtlib.make_args(W, H, spp, 0, nfb, 50, cam, band_rows=band[0], band_first=band[1], band_stride=band[2])
    rows = rtlib.owned_rows(args)
    got, log = None, []
    for _ in range(launches):
        ctx.render_init(W, H, 1984)
        fb = torch.full((nfb * len(rows) * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
        cnt = ctx.render(args, fb.data_ptr())
        assert ctx.last_render_kernel().startswith(kernel_prefix), ctx.last_render_kernel()
        log.append((cnt, ctx.last_render_schedule()))
        g = fb.cpu().numpy().reshape(nfb, len(rows), W, 3)
        if got is not None:  # every launch of the share gives the same bits
            assert np.array_equal(_bits(g), _bits(got))
        got = g
    assert not np.isnan(got).any()
    return got, rows, log


@pytest.mark.parametrize("scene", ["cornell_smoke", "final"])
@pytest.mark.parametrize("n,rank", [(2, 0), (2, 1), (8, 0), (8, 7)])
def test_list_world_share_every_row(rtlib, gpu_ctx, oracle, scene, n, rank):
    """640x360 (final) / 200x200 (cornell_smoke), 2 fbs: rank `rank` of `n` against the oracle's full
    frame on every owned row, on the cold launch and on the two scheduled launches after it."""
    pa, oa = _assets(scene, (341, 152))
    W, H, spp, nfb = (640, 360, 1, 2) if scene == "final" else (200, 200, 2, 2)
    gpu_ctx.upload(rtlib.Scene.builtin(scene, **pa))
    got, rows, log = _share(rtlib, gpu_ctx, W, H, spp, nfb, (4, rank, n), 3, "render_kernel<")
    # (first launches in natural order: final's 1 x 2 samples per pixel are too few for a probe,
    # cornell_smoke has no BVH)
    assert log[0][1] == 0 and all(s & rtlib.RT_SCHED_PREVIOUS for _, s in log[2:])
    ref = oracle.RefScene(scene, **oa)
    segs = 0
    for f in range(nfb):
        want, _, per_px = ref.render(W, H, spp, f, 50, REF, seg_per_pixel=True)
        want = want.reshape(H, W, 3)[rows]
        segs += int(per_px.reshape(H, W)[rows].sum())
        diff = (_bits(got[f]) != _bits(want)).any(axis=2)
        assert not diff.any(), f"{scene} rank {rank}/{n} fb {f}: {int(diff.sum())} pixels differ"
    for cnt, _ in log:
        assert cnt["segments"] == segs
        assert cnt["samples"] == nfb * len(rows) * W * spp


@pytest.mark.parametrize("n,rank", [(8, 0), (8, 7), (2, 1)])
def test_c5_share_full_size(rtlib, gpu_ctx, oracle, n, rank):
    """C5 as one rank of its 8-GPU tiling: final at 3840x2159, 1 spp, 2 fbs; the share rendered whole
    on the GPU (cold, then scheduled), an owned-row subset against the oracle."""
    pa, oa = _assets("final", (3410, 1518))
    W, H, spp, nfb = 3840, 2159, 1, 2
    gpu_ctx.upload(rtlib.Scene.builtin("final", **pa))
    got, rows, _ = _share(rtlib, gpu_ctx, W, H, spp, nfb, (4, rank, n), 2, "render_kernel<")
    # owned rows 4 b + k with b = rank + N m: the oracle's progression row0 = 4 rank + 1, step 4 N * 9
    sub = (4 * rank + 1, 4 * n * 9)
    js = list(range(sub[0], H, sub[1]))
    pos = {int(j): q for q, j in enumerate(rows)}
    assert all(j in pos for j in js)
    ref = oracle.RefScene("final", **oa)
    for f in range(nfb):
        want = ref.render(W, H, spp, f, 50, REF, rows=sub)[0].reshape(H, W, 3)
        q = [pos[j] for j in js]
        assert np.array_equal(_bits(got[f][q]), _bits(want[js])), f"C5 rank {rank}/{n} fb {f}"


@pytest.mark.parametrize("threshold", [None, "0", "1e9"], ids=["default", "lists", "traverse"])
@pytest.mark.parametrize("n", [4, 8])
def test_step_share_across_camera_list_switch(rtlib, gpu_ctx, oracle, ctx_opts, n, threshold):
    """C2's 10-fb workload as rank N-1 of N = 4 (9.2 items per resident lane: camera lists on at the
    product's threshold of 6) and N = 8 (4.6: off), 1 spp per fb; also forced on and off.  Cold and
    scheduled launches against the oracle on an owned-row subset."""
    ctx_opts(bins_min_items_per_lane=6.0 if threshold is None else float(threshold))
    W, H, spp, nfb = 1200, 800, 1, 10
    rank = n - 1
    gpu_ctx.upload(rtlib.Scene.builtin("big1"))
    got, rows, _ = _share(rtlib, gpu_ctx, W, H, spp, nfb, (4, rank, n), 3, "render_step_kernel<")
    sub = (4 * rank + 2, 4 * n * 7)
    js = list(range(sub[0], H, sub[1]))
    pos = {int(j): q for q, j in enumerate(rows)}
    ref = oracle.RefScene("big1")
    for f in range(nfb):
        want = ref.render(W, H, spp, f, 50, REF, rows=sub)[0].reshape(H, W, 3)
        q = [pos[j] for j in js]
        assert np.array_equal(_bits(got[f][q]), _bits(want[js])), f"big1 rank {rank}/{n} fb {f}"


@pytest.mark.parametrize("scene", ["cornell", "cornell_smoke", "earth", "two_perlin", "final"])
def test_world_tree_bit_exact(rtlib, gpu_ctx, oracle, ctx_opts, scene):
    """The opt-in world tree (options.world_tree = 1 at upload: a list world flattened into one traversal tree
    for render_step_kernel, media after it in list order, inert sphere-bounded media skipped for sane
    rays): bit-exact against the oracle, full frame and a share, cold and scheduled launches."""
    ctx_opts(world_tree=1)
    pa, oa = _assets(scene, (341, 152))
    if scene == "earth":
        from raytracing_gpu_amd import assets

        img = assets.synthetic_image(341, 152)
        pa, oa = dict(images=[img]), dict(images=[img])
    W, H, spp, nfb = (96, 54, 2, 2) if scene not in ("cornell", "cornell_smoke") else (48, 48, 4, 2)
    gpu_ctx.upload(rtlib.Scene.builtin(scene, **pa))
    ref = oracle.RefScene(scene, **oa)
    want = [ref.render(W, H, spp, f, 50, REF) for f in range(nfb)]
    for band in ((H, 0, 1), (4, 1, 3)):
        got, rows, log = _share(rtlib, gpu_ctx, W, H, spp, nfb, band, 3, "render_step_kernel<")
        for f in range(nfb):
            diff = (_bits(got[f]) != _bits(want[f][0].reshape(H, W, 3)[rows])).any(axis=2)
            assert not diff.any(), f"{scene} band {band} fb {f}: {int(diff.sum())} pixels differ"
        if band[2] == 1:
            assert all(c["segments"] == sum(int(w[1]["segments"]) for w in want) for c, _ in log)


@pytest.mark.parametrize("ranks", [2, 8])
def test_multi_draw_final_matches_draw(rtlib, ranks):
    """rt_multi_draw (include/rt_multi.h) of C5's scene over `ranks` ranks sharing the box's GPU
    (host gather): the assembled image is byte-identical to the single-context rt_draw, on the cold
    draw and on the warm draws after it."""
    from raytracing_gpu_amd import multi

    pa, _ = _assets("final", (341, 152))
    sc = rtlib.Scene.builtin("final", **pa)
    W, H, spp, nfb = 320, 180, 2, 2
    args = rtlib.make_args(W, H, spp, 0, nfb, 50, REF, band_rows=4)
    ctx = rtlib.Context(0)
    try:
        ctx.upload(sc)
        want, cw = ctx.draw_args(args)
    finally:
        ctx.close()
    m = multi.Multi([0] * ranks, multi.RT_GATHER_HOST)
    try:
        m.upload(sc)
        for k in range(3):
            img, cnt, tm = m.draw(args)
            assert np.array_equal(img, want), f"draw {k}"
            assert cnt["segments"] == cw["segments"]
            assert tm["warm"] == (0 if k == 0 else 1)
    finally:
        m.close()


def test_multi_rccl_one_rank_matches_draw(rtlib):
    """The RCCL gather path of rt_multi (ncclCommInitAll, ncclGather inside a group, stream drain)
    with one rank on the box's device: the image equals rt_draw byte for byte, the gather moved the
    padded rows, and `warm` is 0 on the first draw of a configuration and 1 on its repeats."""
    from raytracing_gpu_amd import multi

    sc = rtlib.Scene.builtin("big1")
    W, H, spp, nfb = 160, 90, 2, 3
    args = rtlib.make_args(W, H, spp, 0, nfb, 50, REF, band_rows=4)
    ctx = rtlib.Context(0)
    try:
        ctx.upload(sc)
        want, cw = ctx.draw_args(args)
    finally:
        ctx.close()
    m = multi.Multi([0], multi.RT_GATHER_RCCL)
    try:
        m.upload(sc)
        for k in range(3):
            img, cnt, tm = m.draw(args)
            assert np.array_equal(img, want), f"draw {k}"
            assert cnt["segments"] == cw["segments"]
            assert tm["gather_bytes"] == H * W * 3
            assert tm["warm"] == (0 if k == 0 else 1)
    finally:
        m.close()


@pytest.mark.parametrize("cam", [0, 1], ids=["ref", "per_pixel"])
@pytest.mark.parametrize("min_segs", [None, "1"], ids=["default", "every_item"])
@pytest.mark.parametrize("band", [None, (4, 1, 3)], ids=["full", "share"])
@pytest.mark.parametrize("scene", ["cornell_smoke", "final"])
def test_list_world_split_samples_bit_exact(rtlib, gpu_ctx, oracle, ctx_opts, scene, band, min_segs, cam):
    """Split samples in render_kernel's parking variants (C5's F_FINAL; cornell_smoke through the
    widest global-memory variant F_ALL, as C3's own narrow variant does not split): launch 1 measures, launch 2
    records the sample-start RNG states of the longest items, launches 3+ run their samples as separate
    work items and merge them in sample order.  Every launch equals the oracle bit for bit, in both
    camera modes, full frame and share, at the product's threshold and with every item split."""
    if min_segs:
        ctx_opts(split_min_segments=float(min_segs))
    pa, oa = _assets(scene, (341, 152))
    W, H, spp, nfb = (96, 54, 4, 2) if scene == "final" else (48, 48, 4, 2)
    gpu_ctx.upload(rtlib.Scene.builtin(scene, **pa))  # a new scene generation: a fresh schedule
    ref = oracle.RefScene(scene, **oa)
    want = [ref.render(W, H, spp, f, 50, cam)[0].reshape(H, W, 3) for f in range(nfb)]
    band = band or (H, 0, 1)
    import torch

    args = rtlib.make_args(W, H, spp, 0, nfb, 50, cam, band_rows=band[0], band_first=band[1], band_stride=band[2],
                           widest=scene == "cornell_smoke", lds=scene != "cornell_smoke")
    rows = rtlib.owned_rows(args)
    seen = set()
    for launch in range(4):
        gpu_ctx.render_init(W, H, 1984)
        fb = torch.full((nfb * len(rows) * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
        cnt = gpu_ctx.render(args, fb.data_ptr())
        assert gpu_ctx.last_render_kernel().startswith("render_kernel<")
        seen.add(gpu_ctx.last_render_schedule())
        got = fb.cpu().numpy().reshape(nfb, len(rows), W, 3)
        for f in range(nfb):
            assert np.array_equal(_bits(got[f]), _bits(want[f][rows])), f"launch {launch} fb {f}"
        assert cnt["samples"] == nfb * len(rows) * W * spp
    if min_segs:
        assert rtlib.RT_SCHED_PREVIOUS | rtlib.RT_SCHED_SPLIT_REPLAY in seen


@pytest.mark.parametrize("mode", ["merged", "fallback", "entry_loop"])
@pytest.mark.parametrize("scene", ["final", "first", "two_perlin", "cornell"])
def test_merged_list_search_bit_exact(rtlib, gpu_ctx, oracle, ctx_opts, scene, mode):
    """render_kernel's merged list-world search (world_search: every entry's candidates in one
    winner/second pair with list tie keys, one settle per query; scenes of primitives, BVHs, instances
    and inert media): C5's own variant on final, the widest global-memory variant F_ALL on the
    primitive-only lists.  "fallback" (RT_MERGE_FALLBACK_ALL) runs the search and then answers every
    query through the exact entry loop, "entry_loop" (RT_MERGE_OFF) is the per-entry world_hit.  Full frame and
    a share, cold and scheduled launches, against the oracle bit for bit."""
    ctx_opts(merged_search={"merged": rtlib.RT_MERGE_ON, "fallback": rtlib.RT_MERGE_FALLBACK_ALL,
                            "entry_loop": rtlib.RT_MERGE_OFF}[mode])
    pa, oa = _assets(scene, (341, 152))
    W, H, spp, nfb = (96, 54, 2, 2) if scene != "cornell" else (48, 48, 4, 2)
    gpu_ctx.upload(rtlib.Scene.builtin(scene, **pa))  # merge_ok is decided at upload
    ref = oracle.RefScene(scene, **oa)
    want = [ref.render(W, H, spp, f, 50, REF) for f in range(nfb)]
    import torch

    for band in ((H, 0, 1), (4, 1, 3)):
        args = rtlib.make_args(W, H, spp, 0, nfb, 50, REF, band_rows=band[0], band_first=band[1],
                               band_stride=band[2], widest=scene != "final", lds=scene == "final")
        rows = rtlib.owned_rows(args)
        for launch in range(3):
            gpu_ctx.render_init(W, H, 1984)
            fb = torch.full((nfb * len(rows) * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
            cnt = gpu_ctx.render(args, fb.data_ptr())
            assert gpu_ctx.last_render_kernel().startswith("render_kernel<"), gpu_ctx.last_render_kernel()
            got = fb.cpu().numpy().reshape(nfb, len(rows), W, 3)
            for f in range(nfb):
                diff = (_bits(got[f]) != _bits(want[f][0].reshape(H, W, 3)[rows])).any(axis=2)
                assert not diff.any(), f"{scene} {mode} band {band} launch {launch} fb {f}: {int(diff.sum())} px"
            if band[2] == 1:
                assert cnt["segments"] == sum(int(w[1]["segments"]) for w in want)


@pytest.mark.parametrize("cam", [REF, 1], ids=["ref", "per_pixel"])
def test_final_share_probe_launch(rtlib, gpu_ctx, oracle, cam):
    """C5's scene as rank 1 of 4 at 320x180, 2 fb x 2 spp: the first launch of the share is
    probe-scheduled on render_kernel's merged-search variant (probe launch into the first fb slice,
    items longest first by its estimate), the next one scheduled by its real counts; both equal the
    oracle bit for bit on every owned row, in both camera modes."""
    pa, oa = _assets("final", (341, 152))
    W, H, spp, nfb = 320, 180, 2, 2
    gpu_ctx.upload(rtlib.Scene.builtin("final", **pa))
    got, rows, log = _share(rtlib, gpu_ctx, W, H, spp, nfb, (4, 1, 4), 2, "render_kernel<", cam=cam)
    assert log[0][1] == rtlib.RT_SCHED_PROBE and log[1][1] & rtlib.RT_SCHED_PREVIOUS, log
    ref = oracle.RefScene("final", **oa)
    for f in range(nfb):
        want = ref.render(W, H, spp, f, 50, cam)[0].reshape(H, W, 3)[rows]
        diff = (_bits(got[f]) != _bits(want)).any(axis=2)
        assert not diff.any(), f"final share fb {f}: {int(diff.sum())} pixels differ"
