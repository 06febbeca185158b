"""GPU parity of the item schedule across configurations and at the configured draw's scale.

The schedule (items claimed longest first, the split samples of the longest items) is a cache of one
configuration's earlier launches inside the context; the pixels must not depend on it.  Every frame
buffer here is compared with the oracle (or with the natural-order launch, RT_FLAG_NO_SCHEDULE, where
the image is too large for the oracle) bit for bit.  Pixel results depend only on global indices: the
RNG slot ((id+1) p + id+1) mod W*H and curand_init(1984, slot, 0) (render.h:91,101), render.h:152-162's
one launch per fb id.
"""
import functools
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REF, PIX = 0, 1
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@functools.lru_cache(maxsize=None)
def _big1_frames(W, H, spp, nfb, cam):
    from oracle import ref_cpu

    ref = ref_cpu.RefScene("big1")
    return [ref.render(W, H, spp, f, 50, cam)[0].reshape(H, W, 3) for f in range(nfb)]


def _launch(rtlib, ctx, W, H, spp, nfb, cam, **kw):
    import torch

    args = rtlib.make_args(W, H, spp, 0, nfb, 50, cam, **kw)
    rows = rtlib.owned_rows(args)
    ctx.render_init(W, H, 1984)
    fb = torch.full((nfb * len(rows) * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
    cnt = ctx.render(args, fb.data_ptr())
    return fb.cpu().numpy().reshape(nfb, len(rows), W, 3), rows, cnt, ctx.last_render_schedule()


@pytest.mark.parametrize("b_shape", [(64, 36), (128, 72)], ids=["b_smaller", "b_larger"])
@pytest.mark.parametrize("cam", [REF, PIX], ids=["ref", "per_pixel"])
def test_probe_launch_of_another_configuration_drops_the_schedule(rtlib, gpu_ctx, ctx_opts, oracle, b_shape, cam):
    """Round-5 advisor: a probe launch builds its schedule into the context's shared perm / split
    state.  Sequence: a large configuration first (it sizes the item buffers, so B fits them whether it
    is smaller or larger than A), A three times (scheduled, then split samples replayed), B's first
    launch (probe-scheduled), A again.  The last A must not claim its items through B's perm (items
    never claimed or claimed twice, or row reads past A's rows): every launch equals the oracle bit for
    bit with the oracle's segment count, and A after B runs as a first launch again."""
    ctx_opts(split_min_segments=1.0)  # every item of A split: the replayed state is what B would clobber
    A, B, BIG = (96, 54), b_shape, (160, 90)
    spp, nfb = 2, 2  # spp * fb_count >= 4: probe-eligible
    gpu_ctx.upload(rtlib.Scene.builtin("big1"))
    want_a = _big1_frames(*A, spp, nfb, cam)
    want_b = _big1_frames(*B, spp, nfb, cam)
    _launch(rtlib, gpu_ctx, *BIG, spp, nfb, cam)
    seq = ["A", "A", "A", "B", "A", "A"]
    seen = []
    for k, which in enumerate(seq):
        W, H = A if which == "A" else B
        got, rows, cnt, sched = _launch(rtlib, gpu_ctx, W, H, spp, nfb, cam)
        seen.append(sched)
        want = want_a if which == "A" else want_b
        for f in range(nfb):
            diff = (_bits(got[f]) != _bits(want[f][rows])).any(axis=2)
            assert not diff.any(), f"launch {k} ({which}) fb {f}: {int(diff.sum())} pixels differ"
        assert cnt["samples"] == nfb * H * W * spp
    assert seen[0] == rtlib.RT_SCHED_PROBE and seen[1] & rtlib.RT_SCHED_PREVIOUS, seen
    assert seen[2] == rtlib.RT_SCHED_PREVIOUS | rtlib.RT_SCHED_SPLIT_REPLAY, seen
    assert seen[3] == rtlib.RT_SCHED_PROBE, seen  # B's first launch
    assert seen[4] == rtlib.RT_SCHED_PROBE, seen  # A's schedule went with B's probe: cold again
    assert seen[5] & rtlib.RT_SCHED_PREVIOUS, seen


def test_bad_options_are_rejected(rtlib, gpu_ctx):
    """rt_ctx_set_options fails loudly (RT_ERR_ARG) on values include/rt_hip.h does not define, and
    keeps the previous options."""
    before = gpu_ctx.options()
    for bad in (dict(cost_shift=-2), dict(cost_shift=13), dict(world_tree=2), dict(quantized_tree=-1),
                dict(dedup_triangles=3), dict(split_order=2), dict(shade_min=65), dict(probe_schedule=-2),
                dict(probe_depth=-2), dict(spread_first=-2), dict(spread_first=65)):
        with pytest.raises(rtlib.RtError):
            gpu_ctx.set_options(**bad)
        assert gpu_ctx.options() == before, bad


def test_scheduled_launch_beyond_64m_items(rtlib, gpu_ctx, ctx_opts):
    """Round-5 verdict item 4a: a launch of more than 64 M items through its item schedule (32-bit perm
    positions; the limit is 2^31 items): big1 at 1200x800 as 70 fb x 2 spp (67.2 M items, fb ids up to
    69, slot products up to 70 * 960 000).  The probe-scheduled first launch, the scheduled second
    (it records split samples) and the split-replaying third each equal the natural-order launch
    (RT_FLAG_NO_SCHEDULE) bit for bit with the same segment count; two fbs checked against the oracle on
    a row subset."""
    import torch

    W, H, spp, nfb = 1200, 800, 2, 70
    assert nfb * W * H > 64 * 2**20
    # at 256 items per lane the share rule splits nothing: split the items of >= 16 segments (millions of
    # split samples, 32-bit claim positions past 64 M)
    ctx_opts(split_min_segments=16.0)
    gpu_ctx.upload(rtlib.Scene.builtin("big1"))
    n = nfb * H * W * 3

    def run(**kw):
        args = rtlib.make_args(W, H, spp, 0, nfb, 50, REF, **kw)
        gpu_ctx.render_init(W, H, 1984)
        fb = torch.full((n,), float("nan"), dtype=torch.float32, device="cuda")
        cnt = gpu_ctx.render(args, fb.data_ptr())
        return fb, cnt, gpu_ctx.last_render_schedule()

    ref_fb, ref_cnt, s0 = run(schedule=False)
    assert s0 == 0
    ref_bits = ref_fb.view(torch.int32)
    seen = []
    for _ in range(3):
        fb, cnt, sched = run()
        seen.append(sched)
        assert cnt["segments"] == ref_cnt["segments"] and cnt["samples"] == nfb * W * H * spp
        assert torch.equal(fb.view(torch.int32), ref_bits), f"launch {len(seen)} (schedule {sched})"
        del fb
    assert seen[0] == rtlib.RT_SCHED_PROBE, seen
    assert seen[1] & rtlib.RT_SCHED_PREVIOUS and seen[2] & rtlib.RT_SCHED_SPLIT_REPLAY, seen
    from oracle import ref_cpu

    ref = ref_cpu.RefScene("big1")
    sub = (3, 97)
    js = list(range(sub[0], H, sub[1]))
    got = ref_fb.view(nfb, H, W, 3)
    for f in (0, nfb - 1):
        want = ref.render(W, H, spp, f, 50, REF, rows=sub)[0].reshape(H, W, 3)
        assert np.array_equal(_bits(got[f, js].cpu().numpy()), _bits(want[js])), f"fb {f}"


@pytest.mark.parametrize("cam", [REF, PIX], ids=["ref", "per_pixel"])
def test_final_high_fb_ids_at_full_size(rtlib, gpu_ctx, oracle, cam):
    """Round-5 verdict item 4b: C5's configured draw renders fb ids up to 99 at 3840x2159, where the
    slot ((id+1) p + id+1) mod N (render.h:101) reaches 8.3e8.  fb_first 98, 2 fbs, 1 spp, as rank 5 of
    8 (4-row bands); cold and scheduled launches against the oracle on an owned-row subset."""
    from raytracing_gpu_amd import assets

    m = assets.door_mesh_from_fixture(os.path.join(GOLD, "door_assimp.npz"))
    img = assets.synthetic_image(3410, 1518)
    import torch

    W, H, spp, nfb, first = 3840, 2159, 1, 2, 98
    n, rank = 8, 5
    gpu_ctx.upload(rtlib.Scene.builtin("final", images=[img], meshes=[m]))
    args = rtlib.make_args(W, H, spp, first, nfb, 50, cam, band_rows=4, band_first=rank, band_stride=n)
    rows = rtlib.owned_rows(args)
    sub = (4 * rank + 2, 4 * n * 11)
    js = list(range(sub[0], H, sub[1]))
    pos = {int(j): q for q, j in enumerate(rows)}
    assert all(j in pos for j in js)
    ref = oracle.RefScene("final", images=[img], meshes=[(m.tris, True, 0)])
    want = [ref.render(W, H, spp, first + f, 50, cam, rows=sub)[0].reshape(H, W, 3) for f in range(nfb)]
    for launch in range(2):
        gpu_ctx.render_init(W, H, 1984)
        fb = torch.full((nfb * len(rows) * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
        gpu_ctx.render(args, fb.data_ptr())
        got = fb.cpu().numpy().reshape(nfb, len(rows), W, 3)
        q = [pos[j] for j in js]
        for f in range(nfb):
            assert np.array_equal(_bits(got[f][q]), _bits(want[f][js])), f"launch {launch} fb id {first + f}"


@pytest.mark.parametrize("depth", [0, 3, -1], ids=["full", "3", "auto"])
@pytest.mark.parametrize("scene", ["big1", "door", "final"])
def test_probe_depth_bit_exact(rtlib, gpu_ctx, ctx_opts, oracle, scene, depth):
    """options.probe_depth cuts a probe sample's path (the probe launch's output is discarded, its counts
    only order the items): the first launch equals the oracle bit for bit at every cap, on the stepwise
    kernel (big1, door) and on render_kernel's merged variant (final); the probe runs under the F_PROBE
    twin's symbol, and rt_last_kernel_ms times the render kernel alone (inside rt_last_render_ms)."""
    W, H, spp, nfb = 96, 54, 4, 2
    pa, oa = {}, {}
    if scene != "big1":
        from raytracing_gpu_amd import assets

        m = assets.door_mesh_from_fixture(os.path.join(GOLD, "door_assimp.npz"))
        img = assets.synthetic_image(341, 152)
        pa, oa = dict(images=[img], meshes=[m]), dict(images=[img], meshes=[(m.tris, True, 0)])
    ctx_opts(probe_depth=depth)
    gpu_ctx.upload(rtlib.Scene.builtin(scene, **pa))
    want = _big1_frames(W, H, spp, nfb, REF) if scene == "big1" else [
        oracle.RefScene(scene, **oa).render(W, H, spp, f, 50, REF)[0].reshape(H, W, 3) for f in range(nfb)]
    got, rows, cnt, sched = _launch(rtlib, gpu_ctx, W, H, spp, nfb, REF, fresh=True)
    assert sched == rtlib.RT_SCHED_PROBE
    name = gpu_ctx.last_render_kernel()
    assert not int(name.split("<")[1].rstrip(">")) & (1 << 18), name  # the render kernel, not its probe twin
    assert 0 < gpu_ctx.last_kernel_ms() <= gpu_ctx.last_render_ms()
    for f in range(nfb):
        assert np.array_equal(_bits(got[f]), _bits(want[f])), f"{scene} depth {depth} fb {f}"


def test_stats_twin_of_the_stepwise_variant(rtlib, gpu_ctx, oracle):
    """bench.py's counting pass runs the F_STATS twin of C2's stepwise LDS variant (the traversal that is
    timed, camera tile lists included): same frame buffers and segment count as the product launch, the
    oracle's pixels, and fewer node tests than the reference's exact visit set."""
    import torch

    W, H, spp, nfb = 160, 90, 2, 2
    gpu_ctx.upload(rtlib.Scene.builtin("big1"))
    out = {}
    for mode in ("product", "stats", "exact"):
        gpu_ctx.render_init(W, H, 1984)
        fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
        args = rtlib.make_args(W, H, spp, 0, nfb, 50, REF, stats=mode != "product", exact=mode == "exact",
                               schedule=False)
        cnt = gpu_ctx.render(args, fb.data_ptr())
        out[mode] = (fb.cpu().numpy(), cnt, gpu_ctx.last_render_kernel())
    assert out["product"][2] == "render_step_kernel<25730>", out["product"][2]
    assert out["stats"][2] == "render_step_kernel<25731>", out["stats"][2]
    assert out["stats"][1]["segments"] == out["product"][1]["segments"] == out["exact"][1]["segments"]
    assert np.array_equal(_bits(out["stats"][0]), _bits(out["product"][0]))
    assert 0 < out["stats"][1]["node_tests"] < out["exact"][1]["node_tests"]
    want = _big1_frames(W, H, spp, nfb, REF)
    got = out["stats"][0].reshape(nfb, H, W, 3)
    for f in range(nfb):
        assert np.array_equal(_bits(got[f]), _bits(want[f]))


@pytest.mark.parametrize("spread", [1, 7, 64])
@pytest.mark.parametrize("scene", ["big1", "door"])
def test_spread_head_bit_exact(rtlib, gpu_ctx, ctx_opts, oracle, scene, spread):
    """options.spread_first: a probe-ordered first launch hands its first 64 x waves positions out strided
    (spread_head_kernel).  Large enough that it applies (items >= 64 x the launch's waves: 16 waves per
    workgroup, one workgroup per CU), the launch equals the natural-order launch (RT_FLAG_NO_SCHEDULE)
    bit for bit with the same segment count, every item claimed once; a row subset against the oracle."""
    import torch

    W, H, spp, nfb = 640, 360, 2, 2
    assert nfb * W * H >= 64 * 16 * torch.cuda.get_device_properties(0).multi_processor_count
    pa, oa = {}, {}
    if scene != "big1":
        from raytracing_gpu_amd import assets

        m = assets.door_mesh_from_fixture(os.path.join(GOLD, "door_assimp.npz"))
        img = assets.synthetic_image(341, 152)
        pa, oa = dict(images=[img], meshes=[m]), dict(images=[img], meshes=[(m.tris, True, 0)])
    ctx_opts(spread_first=spread)
    gpu_ctx.upload(rtlib.Scene.builtin(scene, **pa))
    base, _, bcnt, s0 = _launch(rtlib, gpu_ctx, W, H, spp, nfb, REF, schedule=False)
    assert s0 == 0
    got, rows, cnt, sched = _launch(rtlib, gpu_ctx, W, H, spp, nfb, REF, fresh=True)
    assert sched == rtlib.RT_SCHED_PROBE
    assert cnt["segments"] == bcnt["segments"] and cnt["samples"] == nfb * W * H * spp
    assert np.array_equal(_bits(got), _bits(base)), f"{scene} spread {spread}"
    sub = (5, 41)
    js = list(range(sub[0], H, sub[1]))
    ref = oracle.RefScene(scene, **oa)
    for f in range(nfb):
        want = ref.render(W, H, spp, f, 50, REF, rows=sub)[0].reshape(H, W, 3)
        assert np.array_equal(_bits(got[f][js]), _bits(want[js])), f"{scene} spread {spread} fb {f}"
