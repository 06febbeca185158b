"""GPU parity: the gfx950 render kernel against the CPU oracle, through the C ABI.

Bar: bit-exact float frame buffers (compared as uint32 bit patterns) and identical segment
counts on the same seeded inputs; identical 8-bit output of the resolve (average_images).
Full-size configs are checked on row subsets the oracle finishes in seconds.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REF = 0
PIX = 1

SMALL = [
    # scene, W, H, spp, fb_first, fb_count, cam_mode
    ("basic", 64, 36, 2, 0, 2, REF),
    ("first", 64, 36, 3, 0, 2, REF),
    ("big1", 96, 54, 2, 0, 3, REF),
    ("big1", 80, 45, 2, 4, 2, PIX),
    ("two_spheres", 64, 36, 2, 0, 2, REF),
    ("two_perlin", 64, 36, 2, 0, 2, REF),
    ("cornell", 48, 48, 4, 0, 2, REF),
    ("cornell_smoke", 48, 48, 4, 0, 2, REF),
    ("triangle", 64, 36, 2, 0, 2, REF),
    ("triangles", 64, 36, 2, 0, 2, REF),
    ("backpack", 64, 36, 2, 0, 2, REF),
]


def _gpu_render(rt, ctx, scene, W, H, spp, fb_first, fb_count, cam, depth=50, band=None, exact=False, step=True):
    import torch

    sc = rt.Scene.builtin(scene)
    ctx.upload(sc)
    ctx.render_init(W, H, 1984)
    if band is None:
        args = rt.make_args(W, H, spp, fb_first, fb_count, depth, cam, exact=exact, step=step)
    else:
        args = rt.make_args(W, H, spp, fb_first, fb_count, depth, cam, band_rows=band[0], band_first=band[1],
                            band_stride=band[2], exact=exact, step=step)
    rows = rt.owned_rows(args)
    fb = torch.zeros(fb_count * len(rows) * W * 3, dtype=torch.float32, device="cuda")
    cnt = ctx.render(args, fb.data_ptr())
    torch.cuda.synchronize()
    return fb.cpu().numpy().reshape(fb_count, len(rows), W, 3), rows, cnt, args, fb


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("exact", [False, True], ids=["culled", "exact"])
@pytest.mark.parametrize("scene,W,H,spp,fb_first,fb_count,cam", SMALL)
def test_small_bit_exact(rtlib, gpu_ctx, oracle, scene, W, H, spp, fb_first, fb_count, cam, exact):
    gpu, rows, cnt, _, _ = _gpu_render(rtlib, gpu_ctx, scene, W, H, spp, fb_first, fb_count, cam, exact=exact)
    ref = oracle.RefScene(scene)
    segs = 0
    for f in range(fb_count):
        fb, c, _ = ref.render(W, H, spp, fb_first + f, 50, cam)
        segs += c["segments"]
        want = fb.reshape(H, W, 3)
        diff = _bits(gpu[f]) != _bits(want)
        assert not diff.any(), f"{scene} fb {fb_first + f}: {int(diff.any(axis=2).sum())} pixels differ"
    assert cnt["segments"] == segs
    assert cnt["samples"] == W * H * spp * fb_count


VARIANT_MODES = [  # every compiled kernel family, forced to its widest variant (RT_FLAG_WIDEST)
    ("culled", {}), ("culled_global", {"lds": False}), ("exact", {"exact": True}),
    ("stats", {"stats": True}), ("exact_stats", {"exact": True, "stats": True}), ("audit", {"audit": True}),
]


@pytest.mark.parametrize("scene,W,H,spp,fb_first,fb_count,cam", SMALL + [
    ("cornell_smoke", 200, 200, 4, 0, 1, REF),  # the round-2 ray-copy fault's scene, larger
])
def test_widest_variants_bit_exact(rtlib, gpu_ctx, oracle, scene, W, H, spp, fb_first, fb_count, cam):
    """The catch-all kernel variants must give the same pixels as the narrow ones a scene gets."""
    import torch

    ref = oracle.RefScene(scene)
    want = [ref.render(W, H, spp, fb_first + f, 50, cam)[0].reshape(H, W, 3) for f in range(fb_count)]
    gpu_ctx.upload(rtlib.Scene.builtin(scene))
    gpu_ctx.render_init(W, H, 1984)
    bad = []
    for name, kw in VARIANT_MODES:
        fb = torch.zeros(fb_count * H * W * 3, dtype=torch.float32, device="cuda")
        gpu_ctx.render(rtlib.make_args(W, H, spp, fb_first, fb_count, 50, cam, widest=True, **kw), fb.data_ptr())
        got = fb.cpu().numpy().reshape(fb_count, H, W, 3)
        n = sum(int((_bits(got[f]) != _bits(want[f])).any(axis=2).sum()) for f in range(fb_count))
        if n:
            bad.append(f"{name}: {n} pixels")
    assert not bad, f"{scene}: " + ", ".join(bad)


def _asset_scene(name):
    """(product images/meshes, oracle images/meshes) for scenes that read files in the reference:
    synthetic texture/mesh of the real assets' kind (the reference's files are not on a GPU box)."""
    from raytracing_gpu_amd import assets

    img = assets.synthetic_image(341, 152)
    if name == "earth":
        return dict(images=[img]), dict(images=[img])
    m = assets.synthetic_mesh(24, 32, image=0)
    return dict(images=[img], meshes=[m]), dict(images=[img], meshes=[(m.tris, m.vertex_normals, m.image)])


@pytest.mark.parametrize("exact", [False, True], ids=["culled", "exact"])
@pytest.mark.parametrize("scene", ["earth", "door"])
def test_asset_scene_bit_exact(rtlib, gpu_ctx, oracle, scene, exact):
    import torch

    W, H, spp, nfb = 64, 36, 3, 2
    pa, oa = _asset_scene(scene)
    gpu_ctx.upload(rtlib.Scene.builtin(scene, **pa))
    gpu_ctx.render_init(W, H, 1984)
    fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
    cnt = gpu_ctx.render(rtlib.make_args(W, H, spp, 0, nfb, 50, REF, exact=exact), fb.data_ptr())
    got = fb.cpu().numpy().reshape(nfb, H, W, 3)
    ref = oracle.RefScene(scene, **oa)
    segs = 0
    for f in range(nfb):
        want, c, _ = ref.render(W, H, spp, f, 50, REF)
        segs += c["segments"]
        diff = _bits(got[f]) != _bits(want.reshape(H, W, 3))
        assert not diff.any(), f"{scene} fb {f}: {int(diff.any(axis=2).sum())} pixels differ"
    assert cnt["segments"] == segs


@pytest.mark.parametrize("exact", [False, True], ids=["culled", "exact"])
def test_door_mesh_bit_exact(rtlib, gpu_ctx, oracle, exact):
    """C4 geometry: the reference's door.obj as assimp imports it (golden fixture), with the
    reference's create_meshes_d indexing (H16), synthetic texture of Door_C.jpg's shape."""
    import os

    import torch
    from raytracing_gpu_amd import assets

    m = assets.door_mesh_from_fixture(os.path.join(os.path.dirname(__file__), "golden", "door_assimp.npz"))
    img = assets.synthetic_image(1024, 1024)
    W, H, spp, nfb = 96, 54, 2, 2
    gpu_ctx.upload(rtlib.Scene.builtin("door", images=[img], meshes=[m]))
    gpu_ctx.render_init(W, H, 1984)
    fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
    cnt = gpu_ctx.render(rtlib.make_args(W, H, spp, 0, nfb, 50, REF, exact=exact), fb.data_ptr())
    got = fb.cpu().numpy().reshape(nfb, H, W, 3)
    ref = oracle.RefScene("door", images=[img], meshes=[(m.tris, True, 0)])
    segs = 0
    for f in range(nfb):
        want, c, _ = ref.render(W, H, spp, f, 50, REF)
        segs += c["segments"]
        diff = _bits(got[f]) != _bits(want.reshape(H, W, 3))
        assert not diff.any(), f"door fb {f}: {int(diff.any(axis=2).sum())} pixels differ"
    assert cnt["segments"] == segs


@pytest.mark.parametrize("exact", [False, True], ids=["culled", "exact"])
def test_final_scene_bit_exact(rtlib, gpu_ctx, oracle, exact):
    """C5 composition (boxes under a BVH, media, textures, xformed BVHs, the door mesh)."""
    import os

    import torch
    from raytracing_gpu_amd import assets

    m = assets.door_mesh_from_fixture(os.path.join(os.path.dirname(__file__), "golden", "door_assimp.npz"))
    img = assets.synthetic_image(341, 152)
    W, H, spp, nfb = 80, 45, 2, 2
    gpu_ctx.upload(rtlib.Scene.builtin("final", images=[img], meshes=[m]))
    gpu_ctx.render_init(W, H, 1984)
    fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
    cnt = gpu_ctx.render(rtlib.make_args(W, H, spp, 0, nfb, 50, REF, exact=exact), fb.data_ptr())
    got = fb.cpu().numpy().reshape(nfb, H, W, 3)
    ref = oracle.RefScene("final", images=[img], meshes=[(m.tris, True, 0)])
    segs = 0
    for f in range(nfb):
        want, c, _ = ref.render(W, H, spp, f, 50, REF)
        segs += c["segments"]
        diff = _bits(got[f]) != _bits(want.reshape(H, W, 3))
        assert not diff.any(), f"final fb {f}: {int(diff.any(axis=2).sum())} pixels differ"
    assert cnt["segments"] == segs


def test_resolve_matches_average_images(rtlib, gpu_ctx, oracle):
    import torch

    W, H, spp, nfb = 64, 36, 2, 3
    gpu, rows, _, args, fb = _gpu_render(rtlib, gpu_ctx, "big1", W, H, spp, 0, nfb, REF)
    out = torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda")
    gpu_ctx.resolve(args, fb.data_ptr(), out.data_ptr())
    got = out.cpu().numpy().reshape(H, W, 3)[::-1]  # bottom-up rows -> PNG order
    want, _, _ = oracle.draw("big1", W, H, spp, nfb)
    assert np.array_equal(got, want)


def test_draw_entry_point(rtlib, gpu_ctx, oracle):
    s = rtlib.render_settings(image_width=80, samples_per_pixel_per_fb=2, no_fb=2, max_depth=50)
    img, cnt = rtlib.draw(rtlib.Scene.builtin("basic"), s, ctx=gpu_ctx)
    # int(80 / double(16.0f/9.0f)) = int(44.9999993) = 44 (H18)
    assert img.shape == (s.image_height, 80, 3) and s.image_height == 44
    want, _, tot = oracle.draw("basic", 80, 44, 2, 2)
    assert np.array_equal(img, want)
    assert cnt["segments"] == tot["segments"]


def test_band_tiles_stitch_to_full_frame(rtlib, gpu_ctx):
    W, H, spp = 72, 41, 2
    full, _, cfull, _, _ = _gpu_render(rtlib, gpu_ctx, "big1", W, H, spp, 0, 2, REF)
    seen = np.zeros(H, bool)
    segs = 0
    for rank in range(3):
        part, rows, c, _, _ = _gpu_render(rtlib, gpu_ctx, "big1", W, H, spp, 0, 2, REF, band=(8, rank, 3))
        assert np.array_equal(_bits(part), _bits(full[:, rows]))
        seen[rows] = True
        segs += c["segments"]
    assert seen.all()
    assert segs == cfull["segments"]


@pytest.mark.parametrize("scene,W,H,spp,rows", [
    ("big1", 1200, 800, 2, (3, 97)),        # C2 size (1200x800), 9 rows
    ("big1", 1200, 800, 4, (1, 40)),        # C2 size, 20 rows at 4 spp
    ("cornell_smoke", 800, 800, 2, (5, 131)),  # C3 size, 7 rows
    ("cornell_smoke", 800, 800, 4, (2, 25)),   # C3 size, 32 rows at 4 spp
])
def test_full_size_row_subset(rtlib, gpu_ctx, oracle, scene, W, H, spp, rows):
    gpu, _, _, _, _ = _gpu_render(rtlib, gpu_ctx, scene, W, H, spp, 0, 1, REF)
    fb, _, _ = oracle.RefScene(scene).render(W, H, spp, 0, 50, REF, rows=rows)
    want = fb.reshape(H, W, 3)
    js = list(range(rows[0], H, rows[1]))
    assert np.array_equal(_bits(gpu[0][js]), _bits(want[js]))


def test_stats_counters_match_oracle(rtlib, gpu_ctx, oracle):
    """Node/primitive test counts of the exact-traversal stats variant equal the oracle's (the
    reference's visit set); the culled traversal visits strictly fewer."""
    W, H, spp = 48, 27, 2
    import torch

    sc = rtlib.Scene.builtin("big1")
    gpu_ctx.upload(sc)
    gpu_ctx.render_init(W, H, 1984)
    args = rtlib.make_args(W, H, spp, 0, 1, 50, REF, stats=True, exact=True)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    cnt = gpu_ctx.render(args, fb.data_ptr())
    _, c, _ = oracle.RefScene("big1").render(W, H, spp, 0, 50, REF)
    assert cnt["segments"] == c["segments"]
    assert cnt["node_tests"] == c["node_tests"]
    assert cnt["prim_tests"] == c["prim_tests"]
    fast = gpu_ctx.render(rtlib.make_args(W, H, spp, 0, 1, 50, REF, stats=True), fb.data_ptr())
    assert fast["segments"] == c["segments"] and fast["node_tests"] < c["node_tests"]


@pytest.mark.parametrize("scene,W,H,spp,nfb", [
    ("big1", 1200, 800, 10, 10),          # the whole C2 bench workload (100 rays/pixel)
    ("cornell_smoke", 800, 800, 10, 2),   # C3 geometry, 20 rays/pixel
])
def test_culled_equals_exact_full_workload(rtlib, gpu_ctx, scene, W, H, spp, nfb):
    """Over an entire benchmark workload the culled traversal reproduces the reference-visit-set
    traversal bit for bit (every float of every fb) and with the same segment count."""
    fast, _, cf, _, _ = _gpu_render(rtlib, gpu_ctx, scene, W, H, spp, 0, nfb, REF)
    ex, _, ce, _, _ = _gpu_render(rtlib, gpu_ctx, scene, W, H, spp, 0, nfb, REF, exact=True)
    assert cf["segments"] == ce["segments"]
    assert np.array_equal(_bits(fast), _bits(ex))


@pytest.mark.parametrize("scene,W,H,spp,nfb", [
    ("final", 640, 360, 4, 2),            # C5 composition: ground boxes, xformed BVHs, media, door mesh
    ("door", 480, 270, 4, 2),             # C4 geometry (the real door mesh)
    ("door", 1920, 1079, 2, 1),           # C4 at its full image size
    ("final", 1280, 720, 2, 1),           # C5's bench size
])
def test_culled_equals_exact_asset_scenes(rtlib, gpu_ctx, scene, W, H, spp, nfb):
    """Mesh / texture scenes at sizes past the oracle's reach: culled traversal (candidate ranges,
    the sphere validation shortcut) equals the reference visit set, every float."""
    import os

    import torch
    from raytracing_gpu_amd import assets

    m = assets.door_mesh_from_fixture(os.path.join(os.path.dirname(__file__), "golden", "door_assimp.npz"))
    img = assets.synthetic_image(341, 152) if scene == "final" else assets.synthetic_image(1024, 1024)
    gpu_ctx.upload(rtlib.Scene.builtin(scene, images=[img], meshes=[m]))
    gpu_ctx.render_init(W, H, 1984)
    out = []
    for exact in (False, True):
        fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
        cnt = gpu_ctx.render(rtlib.make_args(W, H, spp, 0, nfb, 50, REF, exact=exact), fb.data_ptr())
        out.append((fb.cpu().numpy(), cnt["segments"]))
    assert out[0][1] == out[1][1]
    diff = _bits(out[0][0]) != _bits(out[1][0])
    assert not diff.any(), f"{scene}: {int(diff.sum())} floats differ"


@pytest.mark.parametrize("scene", ["door", "final"])
def test_coincident_triangles_leave_the_traversal_tree(rtlib, gpu_ctx, ctx_opts, scene):
    """The door's H16 duplicates (triangles repeating an earlier one's v0, e0, e1 bit for bit) keep
    one leaf per group in the traversal trees: every float and the segment count equal the build with
    every member (options.dedup_triangles = 0, read at upload) and the exact visit set, with fewer
    primitive tests."""
    import os

    import torch
    from raytracing_gpu_amd import assets

    m = assets.door_mesh_from_fixture(os.path.join(os.path.dirname(__file__), "golden", "door_assimp.npz"))
    img = assets.synthetic_image(341, 152)
    W, H, spp, nfb = 320, 180, 4, 2
    out = {}
    for mode in ("dedup", "all", "exact"):
        ctx_opts(dedup_triangles=0 if mode == "all" else 1)
        gpu_ctx.upload(rtlib.Scene.builtin(scene, images=[img], meshes=[m]))
        gpu_ctx.render_init(W, H, 1984)
        fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
        cnt = gpu_ctx.render(rtlib.make_args(W, H, spp, 0, nfb, 50, REF, stats=True, exact=mode == "exact"),
                             fb.data_ptr())
        out[mode] = (fb.cpu().numpy(), cnt)
    for mode in ("all", "exact"):
        assert out[mode][1]["segments"] == out["dedup"][1]["segments"]
        assert np.array_equal(_bits(out[mode][0]), _bits(out["dedup"][0])), mode
    assert out["dedup"][1]["prim_tests"] < out["all"][1]["prim_tests"]
    if scene == "door":  # the product variant keeps the (smaller) tree quantized in LDS (F_QLDS = 1 << 16)
        fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
        cnt = gpu_ctx.render(rtlib.make_args(W, H, spp, 0, nfb, 50, REF), fb.data_ptr())
        name = gpu_ctx.last_render_kernel()
        assert name.startswith("render_step_kernel<") and int(name.split("<")[1].split(">")[0]) & (1 << 16), name
        assert cnt["segments"] == out["dedup"][1]["segments"]
        assert np.array_equal(_bits(fb.cpu().numpy()), _bits(out["dedup"][0]))


@pytest.mark.parametrize("scene,W,H,spp,nfb,cam", [
    ("big1", 1200, 800, 10, 10, REF),     # the whole C2 bench workload
    ("big1", 333, 187, 3, 2, PIX),
    ("basic", 200, 100, 4, 2, REF),
    ("first", 160, 90, 4, 2, REF),
])
def test_step_kernel_equals_segment_loop(rtlib, gpu_ctx, oracle, scene, W, H, spp, nfb, cam):
    """render_step_kernel (one traversal step per loop trip, batched shading; the default for
    worlds that are one BVH) gives every float of the segment-per-trip kernel, same segments."""
    a, _, ca, _, _ = _gpu_render(rtlib, gpu_ctx, scene, W, H, spp, 0, nfb, cam)
    b, _, cb, _, _ = _gpu_render(rtlib, gpu_ctx, scene, W, H, spp, 0, nfb, cam, step=False)
    assert ca["segments"] == cb["segments"] and ca["samples"] == cb["samples"]
    assert np.array_equal(_bits(a), _bits(b))
    if W * H * spp <= 20000:
        ref = oracle.RefScene(scene)
        for f in range(nfb):
            want, _, _ = ref.render(W, H, spp, f, 50, cam)
            assert np.array_equal(_bits(a[f]), _bits(want.reshape(H, W, 3)))


@pytest.mark.parametrize("key,scene,W,H,spp,fbs,depth", [
    ("c1_basic", "basic", 200, 100, 1, [0], 1),
    ("c2_big1", "big1", 120, 68, 4, [0, 1], 50),
    ("c3_cornell_smoke", "cornell_smoke", 64, 64, 4, [0, 1], 50),
])
def test_against_committed_golden(rtlib, gpu_ctx, key, scene, W, H, spp, fbs, depth):
    """GPU output vs the committed oracle fixtures (tests/golden/renders.npz), without the live oracle."""
    import os

    import torch

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "renders.npz"))
    gpu, _, cnt, args, fb = _gpu_render(rtlib, gpu_ctx, scene, W, H, spp, fbs[0], len(fbs), REF, depth=depth)
    for k, f in enumerate(fbs):
        assert np.array_equal(_bits(gpu[k]), _bits(g[f"{key}_fb{f}"]))
    assert cnt["segments"] == sum(int(g[f"{key}_fb{f}_segments"][0]) for f in fbs)
    out = torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda")
    gpu_ctx.resolve(args, fb.data_ptr(), out.data_ptr())
    assert np.array_equal(out.cpu().numpy().reshape(H, W, 3)[::-1], g[f"{key}_png"])


def test_render_init_states_match_curand_init(rtlib, gpu_ctx, oracle):
    """rt_render_init == curand_init(1984, slot, 0) for every slot class: chunk starts, chunk
    interiors, the last slot, and the golden subsequences of tests/golden/xorwow_uniforms.json."""
    import json
    import os

    W, H = 1200, 800
    gpu_ctx.render_init(W, H, 1984)
    rng = np.random.default_rng(7)
    slots = sorted(set([0, 1, 2, 15, 16, 17, 1023, 959999, W * H - 1] + list(rng.integers(0, W * H, 200))))
    for s in slots:
        got = gpu_ctx.read_states(int(s), 1)[0]
        assert np.array_equal(got, oracle.xorwow_init(1984, int(s), 0)), s
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "xorwow_uniforms.json")))
    for s, words in gold["states"].items():
        assert np.array_equal(gpu_ctx.read_states(int(s), 1)[0], np.array(words, np.uint32))


EDGE = [
    # scene, W, H, spp, fb_first, fb_count, cam, depth
    ("basic", 1, 1, 3, 0, 2, REF, 50),          # N = 1: every slot is 0
    ("basic", 200, 100, 1, 0, 1, REF, 1),       # config C1: depth 1, explicit height
    ("big1", 7, 3, 5, 37, 2, REF, 50),          # odd sizes, a large fb id
    ("cornell_smoke", 17, 13, 3, 0, 3, PIX, 2),  # per-pixel camera, depth 2 through the media
    ("two_perlin", 33, 9, 1, 5, 1, REF, 3),
]


@pytest.mark.parametrize("scene,W,H,spp,fb_first,fb_count,cam,depth", EDGE)
def test_edge_configs_bit_exact(rtlib, gpu_ctx, oracle, scene, W, H, spp, fb_first, fb_count, cam, depth):
    gpu, rows, cnt, _, _ = _gpu_render(rtlib, gpu_ctx, scene, W, H, spp, fb_first, fb_count, cam, depth=depth)
    ref = oracle.RefScene(scene)
    segs = 0
    for f in range(fb_count):
        fb, c, _ = ref.render(W, H, spp, fb_first + f, depth, cam)
        segs += c["segments"]
        assert np.array_equal(_bits(gpu[f]), _bits(fb.reshape(H, W, 3))), f"{scene} fb {fb_first + f}"
    assert cnt["segments"] == segs


def test_abi_error_contract(rtlib):
    """Every call reports failure through its status and rt_last_error; nothing aborts."""
    import torch

    ctx = rtlib.Context(0)
    fb = torch.zeros(64 * 36 * 3, dtype=torch.float32, device="cuda")
    args = rtlib.make_args(64, 36, 1)
    with pytest.raises(rtlib.RtError, match="no scene"):
        ctx.render(args, fb.data_ptr())
    ctx.upload(rtlib.Scene.builtin("basic"))
    with pytest.raises(rtlib.RtError, match="render_init"):
        ctx.render(args, fb.data_ptr())
    ctx.render_init(64, 36, 1984)
    with pytest.raises(rtlib.RtError, match="render_init"):
        ctx.render(rtlib.make_args(65, 36, 1), fb.data_ptr())
    with pytest.raises(rtlib.RtError):
        ctx.render(args, 0)
    with pytest.raises(rtlib.RtError, match="band"):
        ctx.render(rtlib.make_args(64, 36, 1, band_rows=8, band_first=3, band_stride=2), fb.data_ptr())
    with pytest.raises(rtlib.RtError):
        ctx.render(rtlib.make_args(64, 36, 0), fb.data_ptr())
    ctx.render(args, fb.data_ptr())  # still usable after the failures
    ctx.close()


def test_bench_two_ranks_match_one(tmp_path):
    """bench.py's N>1 path (bands, resolve, all-gather, assembly) as the driver launches it
    (torch.distributed.run), rehearsed with two ranks on one GPU over gloo: the assembled image
    is byte-identical to the single-rank run."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["bench.py", "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-stats",
              "--width", "200", "--height", "112", "--spp", "2", "--nfb", "2"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    one = subprocess.run([sys.executable, *common, "--png", str(tmp_path / "n1.png")], cwd=root, env=env,
                         capture_output=True, text=True, timeout=600)
    assert one.returncode == 0, one.stderr[-2000:]
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", "29533", *common, "--gpus", "2",
                          "--backend", "gloo", "--png", str(tmp_path / "n2.png")], cwd=root, env=env,
                         capture_output=True, text=True, timeout=600)
    assert two.returncode == 0, two.stderr[-2000:]
    assert '"n_gpus": 2' in two.stdout
    assert (tmp_path / "n1.png").read_bytes() == (tmp_path / "n2.png").read_bytes()


def test_bench_inprocess_two_ranks_match_one(tmp_path):
    """`python bench.py --gpus 2` exactly as the driver invokes BENCH (no launcher): the C++
    multi-GPU driver (librt_multi.so) in one process, two ranks sharing the box's GPU with host
    gathers.  The JSON line says n_gpus 2 and the assembled image is byte-identical to N = 1."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["bench.py", "--steps", "1", "--warmup", "1", "--warm-steps", "1", "--no-cpu-baseline",
              "--no-stats", "--width", "200", "--height", "112", "--spp", "2", "--nfb", "2"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    one = subprocess.run([sys.executable, *common, "--png", str(tmp_path / "n1.png")], cwd=root, env=env,
                         capture_output=True, text=True, timeout=600)
    assert one.returncode == 0, one.stderr[-2000:]
    two = subprocess.run([sys.executable, *common, "--gpus", "2", "--gather", "host",
                          "--png", str(tmp_path / "n2.png")], cwd=root, env=env,
                         capture_output=True, text=True, timeout=600)
    assert two.returncode == 0, two.stderr[-2000:]
    line = json.loads([x for x in two.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and "librt_multi.so" in line["driver"]
    assert line["value"] > 0 and line["warm_ms_per_step"] > 0
    assert (tmp_path / "n1.png").read_bytes() == (tmp_path / "n2.png").read_bytes()


def test_host_buffers_match_device(rtlib, gpu_ctx, oracle):
    """rt_render / rt_resolve also take host pointers (host or device frame buffer):
    the kernels write a staged device buffer that is copied back; bits equal the device path's
    and the oracle's."""
    import torch

    W, H, spp, nfb = 64, 36, 2, 2
    dev, rows, cnt, args, fb = _gpu_render(rtlib, gpu_ctx, "big1", W, H, spp, 0, nfb, REF, band=(4, 1, 3))
    host = np.zeros(nfb * len(rows) * W * 3, np.float32)
    cnt_h = gpu_ctx.render(args, host.ctypes.data)
    assert cnt_h["segments"] == cnt["segments"]
    assert np.array_equal(_bits(host.reshape(dev.shape)), _bits(dev))
    ref = oracle.RefScene("big1")
    for f in range(nfb):
        want = ref.render(W, H, spp, f, 50, REF)[0].reshape(H, W, 3)[rows]
        assert np.array_equal(_bits(dev[f]), _bits(want))
    out_dev = torch.zeros(len(rows) * W * 3, dtype=torch.uint8, device="cuda")
    gpu_ctx.resolve(args, fb.data_ptr(), out_dev.data_ptr())
    out_host = np.zeros(len(rows) * W * 3, np.uint8)
    gpu_ctx.resolve(args, host.ctypes.data, out_host.ctypes.data)  # host in, host out
    assert np.array_equal(out_host, out_dev.cpu().numpy())


@pytest.mark.parametrize("threshold", ["0", "6", "1e9"], ids=["lists", "default", "traverse"])
def test_camera_lists_on_and_off(rtlib, gpu_ctx, oracle, threshold, ctx_opts):
    """Camera rays through the 8x8-tile candidate lists (threshold 0), the product's default
    threshold (6 items per resident lane: off for this size) and never: same bits as the oracle."""
    ctx_opts(bins_min_items_per_lane=float(threshold))
    W, H, spp, nfb = 96, 54, 2, 2
    gpu, rows, cnt, _, _ = _gpu_render(rtlib, gpu_ctx, "big1", W, H, spp, 0, nfb, REF)
    ref = oracle.RefScene("big1")
    segs = 0
    for f in range(nfb):
        want, c, _ = ref.render(W, H, spp, f, 50, REF)
        segs += c["segments"]
        assert np.array_equal(_bits(gpu[f]), _bits(want.reshape(H, W, 3)))
    assert cnt["segments"] == segs


@pytest.mark.parametrize("order", [None, "0"], ids=["longest_first", "item_order"])
@pytest.mark.parametrize("min_segs", [None, "1"], ids=["default", "every_item"])
@pytest.mark.parametrize("band", [None, (4, 1, 3)], ids=["full", "share"])
def test_split_samples_bit_exact(rtlib, gpu_ctx, oracle, ctx_opts, min_segs, band, order):
    """Warm launches split the samples of the longest items over work items (launch 1 measures,
    launch 2 records the sample-start RNG states and segment counts, launches 3+ claim the split
    samples and the other items longest first -- or, options.split_order = 0, samples in item order -- and
    merge): every launch's frame buffer equals the oracle's bit for bit, with the same segment and
    sample counts."""
    import torch

    if min_segs:
        ctx_opts(split_min_segments=float(min_segs))
    if order is not None:
        ctx_opts(split_order=int(order))
    W, H, spp, nfb = 96, 54, 4, 2
    sc = rtlib.Scene.builtin("big1")
    gpu_ctx.upload(sc)  # new scene generation: a fresh schedule
    ref = oracle.RefScene("big1")
    want = [ref.render(W, H, spp, f, 50, REF) for f in range(nfb)]
    kw = {} if band is None else dict(band_rows=band[0], band_first=band[1], band_stride=band[2])
    args = rtlib.make_args(W, H, spp, 0, nfb, 50, REF, **kw)
    rows = rtlib.owned_rows(args)
    segs = sum(int(w[1]["segments"]) for w in want) if band is None else None
    for launch in range(4):
        gpu_ctx.render_init(W, H, 1984)
        fb = torch.full((nfb * len(rows) * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
        cnt = gpu_ctx.render(args, fb.data_ptr())
        got = fb.cpu().numpy().reshape(nfb, len(rows), W, 3)
        for f in range(nfb):
            assert np.array_equal(_bits(got[f]), _bits(want[f][0].reshape(H, W, 3)[rows])), f"launch {launch} fb {f}"
        assert cnt["samples"] == nfb * len(rows) * W * spp
        if segs is not None:
            assert cnt["segments"] == segs


@pytest.mark.parametrize("scene,W,H,spp,rows", [
    ("door", 1920, 1079, 2, (7, 120)),    # C4 size (1920x1079), 9 rows
    ("final", 3840, 2159, 1, (11, 270)),  # C5 size (3840x2159), 8 rows
])
def test_full_size_mesh_rows(rtlib, gpu_ctx, oracle, scene, W, H, spp, rows):
    """C4 / C5 at their full image sizes (bench.py's assets: the door mesh fixture, synthetic
    textures of the real files' shapes), a row subset against the oracle, two fbs."""
    import os

    import torch
    from raytracing_gpu_amd import assets

    m = assets.door_mesh_from_fixture(os.path.join(os.path.dirname(__file__), "golden", "door_assimp.npz"))
    img = assets.synthetic_image(2048, 2048) if scene == "door" else assets.synthetic_image(3410, 1518)
    nfb = 2
    gpu_ctx.upload(rtlib.Scene.builtin(scene, images=[img], meshes=[m]))
    gpu_ctx.render_init(W, H, 1984)
    fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
    gpu_ctx.render(rtlib.make_args(W, H, spp, 0, nfb, 50, REF), fb.data_ptr())
    got = fb.cpu().numpy().reshape(nfb, H, W, 3)
    ref = oracle.RefScene(scene, images=[img], meshes=[(m.tris, True, 0)])
    js = list(range(rows[0], H, rows[1]))
    for f in range(nfb):
        want = ref.render(W, H, spp, f, 50, REF, rows=rows)[0].reshape(H, W, 3)
        assert np.array_equal(_bits(got[f][js]), _bits(want[js])), f"{scene} fb {f}"


def test_split_samples_switch_cam_mode_and_seed(rtlib, gpu_ctx, oracle):
    """One context, one configuration drawn warm in REF mode (measure, record, split), then with
    the other camera mode and another seed in between: the split items must never start from RNG
    states recorded under another camera mode or seed.  Every launch equals the oracle (seed 1984)
    or the cold render of the same seed (seed 7), bit for bit."""
    import torch

    W, H, spp, nfb = 96, 54, 4, 2
    gpu_ctx.upload(rtlib.Scene.builtin("big1"))
    ref = oracle.RefScene("big1")
    want = {cam: [ref.render(W, H, spp, f, 50, cam)[0].reshape(H, W, 3) for f in range(nfb)] for cam in (REF, PIX)}

    def launch(cam, seed=1984, **kw):
        gpu_ctx.render_init(W, H, seed)
        fb = torch.full((nfb * H * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
        cnt = gpu_ctx.render(rtlib.make_args(W, H, spp, 0, nfb, 50, cam, seed=seed, **kw), fb.data_ptr())
        return fb.cpu().numpy().reshape(nfb, H, W, 3), cnt, gpu_ctx.last_render_schedule()

    cold7 = {cam: launch(cam, 7, schedule=False)[0] for cam in (REF, PIX)}
    seen = set()
    for k, (cam, seed) in enumerate([(REF, 1984)] * 4 + [(PIX, 1984), (REF, 1984), (PIX, 1984), (PIX, 1984),
                                     (PIX, 1984), (REF, 7), (REF, 1984), (PIX, 7), (PIX, 1984)]):
        got, cnt, sched = launch(cam, seed)
        seen.add(sched)
        exp = want[cam] if seed == 1984 else cold7[cam]
        for f in range(nfb):
            assert np.array_equal(_bits(got[f]), _bits(exp[f])), f"launch {k} cam {cam} seed {seed} fb {f}"
        assert cnt["samples"] == nfb * H * W * spp
    assert rtlib.RT_SCHED_PREVIOUS | rtlib.RT_SCHED_SPLIT_REPLAY in seen  # the split replay did run


@pytest.mark.parametrize("launches", [4])
def test_c2_primary_split_rows(rtlib, gpu_ctx, oracle, launches):
    """C2 as SURVEY.md 8d names it first: no_fb = 1 x samples_per_pixel_per_fb = 100 (render.h:24's
    default), 1200x800, depth 50.  Every launch of the whole image (cold, schedule, split-recording,
    split-replay) against the oracle on a row subset."""
    import torch

    W, H, spp = 1200, 800, 100
    rows = (3, 101)  # 8 rows
    js = list(range(rows[0], H, rows[1]))
    want = oracle.RefScene("big1").render(W, H, spp, 0, 50, REF, rows=rows)[0].reshape(H, W, 3)
    gpu_ctx.upload(rtlib.Scene.builtin("big1"))
    args = rtlib.make_args(W, H, spp, 0, 1, 50, REF)
    for launch in range(launches):
        gpu_ctx.render_init(W, H, 1984)
        fb = torch.full((H * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
        cnt = gpu_ctx.render(args, fb.data_ptr())
        got = fb.cpu().numpy().reshape(H, W, 3)
        assert np.array_equal(_bits(got[js]), _bits(want[js])), f"launch {launch}"
        assert not np.isnan(got).any()
        assert cnt["samples"] == W * H * spp


def test_c2_primary_split_culled_equals_exact(rtlib, gpu_ctx):
    """The whole 1 x 100 C2 workload: culled (and, from the third launch, split-sample) rendering
    equals the reference visit set, every float, same segment count."""
    ex, _, ce, _, _ = _gpu_render(rtlib, gpu_ctx, "big1", 1200, 800, 100, 0, 1, REF, exact=True)
    import torch

    args = rtlib.make_args(1200, 800, 100, 0, 1, 50, REF)
    for launch in range(3):
        gpu_ctx.render_init(1200, 800, 1984)
        fb = torch.zeros(1200 * 800 * 3, dtype=torch.float32, device="cuda")
        cf = gpu_ctx.render(args, fb.data_ptr())
        assert cf["segments"] == ce["segments"], f"launch {launch}"
        assert np.array_equal(_bits(fb.cpu().numpy().reshape(ex.shape)), _bits(ex)), f"launch {launch}"



@pytest.mark.parametrize("grid", [3, 7])
@pytest.mark.parametrize("band", [None, (3, 1, 2)], ids=["full", "share"])
@pytest.mark.parametrize("cam", [REF, PIX], ids=["ref", "per_pixel"])
def test_probe_grid_edges(rtlib, gpu_ctx, oracle, ctx_opts, grid, band, cam):
    """Probe-scheduled first launches on grids that do not divide the image (101x57, every 3rd /
    7th row position and pixel), fb ids 2..3 of a call, full frame and a 3-row-band share: the probe
    writes into the first fb slice of the call, which the launch overwrites; every pixel equals the
    oracle and the launch reports RT_SCHED_PROBE."""
    ctx_opts(probe_schedule=grid)
    W, H, spp, fb_first, fb_count = 101, 57, 2, 2, 2
    gpu, rows, cnt, _, _ = _gpu_render(rtlib, gpu_ctx, "big1", W, H, spp, fb_first, fb_count, cam, band=band)
    assert gpu_ctx.last_render_schedule() == rtlib.RT_SCHED_PROBE
    ref = oracle.RefScene("big1")
    for f in range(fb_count):
        want = ref.render(W, H, spp, fb_first + f, 50, cam)[0].reshape(H, W, 3)[rows]
        diff = (_bits(gpu[f]) != _bits(want)).any(axis=2)
        assert not diff.any(), f"grid {grid} fb {fb_first + f}: {int(diff.sum())} pixels differ"
    assert cnt["samples"] == len(rows) * W * spp * fb_count
