"""The C++ callers of the boundary: examples/rt_main (the reference's main.cu rewritten against
include/rt_hip.h) and librt_multi.so (include/rt_multi.h: draw() tiled over
several GPUs with one RCCL gather).

CPU: librt_multi.so loads and exports every symbol rt_multi.h declares; argument checks that
return before touching a GPU; rt_main's usage exit.
GPU (`-m gpu`): rt_main's images are byte-identical to the CPU oracle's draw(); rt_multi's band
tiling + gather + assembly is byte-identical to the single-GPU draw for 1..4 ranks (ranks sharing
the box's one GPU with the host gather; the RCCL gather with one rank per device), and the
product ingestion path (rt_obj_load + rt_image_load -> rt_scene_build_ex -> render) matches the
oracle on committed OBJ / JPEG fixtures.
"""
import ctypes
import json
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
RT_MAIN = os.path.join(ROOT, "examples", "bin", "rt_main")
MULTI = os.path.join(ROOT, "raytracing_gpu_amd", "librt_multi.so")


def _multi_lib(rtlib):
    rtlib.lib()  # torch's HIP runtime first, then librt_hip.so (librt_multi links both)
    return ctypes.CDLL(MULTI)


def test_multi_exports_every_declared_symbol(rtlib):
    hdr = open(os.path.join(ROOT, "include", "rt_multi.h")).read()
    declared = set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rt_multi_\w+)\s*\(", hdr, re.M))
    assert {"rt_multi_create", "rt_multi_draw", "rt_multi_upload", "rt_multi_destroy"} <= declared
    L = _multi_lib(rtlib)
    assert not [n for n in sorted(declared) if not hasattr(L, n)]


def test_multi_argument_checks(rtlib):
    """Errors a caller gets before any device is touched: status codes, no abort."""
    L = _multi_lib(rtlib)
    L.rt_multi_create.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]
    h = ctypes.c_void_p()
    devs = (ctypes.c_int32 * 2)(0, 0)
    RT_ERR_ARG = 1
    assert L.rt_multi_create(0, devs, 0, ctypes.byref(h)) == RT_ERR_ARG          # no ranks
    assert L.rt_multi_create(17, devs, 0, ctypes.byref(h)) == RT_ERR_ARG         # > RT_MULTI_MAX_RANKS
    assert L.rt_multi_create(2, devs, 7, ctypes.byref(h)) == RT_ERR_ARG          # unknown gather
    assert L.rt_multi_create(2, devs, 0, ctypes.byref(h)) == RT_ERR_ARG          # RCCL: one rank per device
    assert not h.value


def test_rt_main_usage():
    assert os.path.exists(RT_MAIN), "examples/bin/rt_main not built (python -m raytracing_gpu_amd._build)"
    p = subprocess.run([RT_MAIN], capture_output=True, text=True)
    assert p.returncode == 2 and "usage" in p.stderr


def _read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    m = re.match(rb"P6\n(\d+) (\d+)\n255\n", data)
    W, H = int(m.group(1)), int(m.group(2))
    return np.frombuffer(data[m.end():], np.uint8).reshape(H, W, 3)


def _rt_main(tmp_path, *args):
    out = str(tmp_path / "out.ppm")
    p = subprocess.run([RT_MAIN, *map(str, args[:4]), out, *map(str, args[4:])], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return _read_ppm(out), lines


@pytest.mark.gpu
@pytest.mark.parametrize("scene,W,spp,nfb", [("basic", 64, 2, 2), ("big1", 96, 2, 3), ("cornell_smoke", 48, 3, 2)])
def test_rt_main_matches_oracle(oracle, tmp_path, scene, W, spp, nfb):
    img, lines = _rt_main(tmp_path, scene, W, spp, nfb)
    want, _, tot = oracle.draw(scene, W, img.shape[0], spp, nfb)
    assert img.shape == want.shape and np.array_equal(img, want)
    assert lines[-1]["segments"] == tot["segments"]


@pytest.mark.gpu
@pytest.mark.parametrize("ranks,band", [(1, 4), (2, 4), (3, 4), (4, 3), (3, 1)])
def test_multi_host_gather_matches_draw(tmp_path, ranks, band):
    """Band tiling + gather + assembly: byte-identical to rt_draw for any rank count / band size
    (ranks share the GPU; the host gather stands in for RCCL, which needs distinct devices).  Four
    draws: the cold one, the one that builds the schedule and records the split items' states, and
    two with split samples; the image is the last draw's."""
    one, l1 = _rt_main(tmp_path, "big1", 120, 2, 3)
    got, lm = _rt_main(tmp_path, "big1", 120, 2, 3, "--devices", ",".join(["0"] * ranks), "--gather", "host",
                       "--band-rows", band, "--repeat", 4)
    assert np.array_equal(got, one)
    assert all(x["segments"] == l1[0]["segments"] for x in lm)
    assert lm[0]["warm"] == 0 and all(x["warm"] == 1 for x in lm[1:])


@pytest.mark.gpu
def test_multi_rccl_gather_matches_draw(tmp_path):
    """The RCCL path (ncclCommInitAll + ncclGather) with one rank per visible device."""
    import torch

    n = torch.cuda.device_count()
    one, _ = _rt_main(tmp_path, "big1", 120, 2, 3)
    got, lm = _rt_main(tmp_path, "big1", 120, 2, 3, "--devices", ",".join(str(d) for d in range(n)), "--gather",
                       "rccl", "--repeat", 2)
    assert np.array_equal(got, one)
    assert lm[-1]["gather_bytes"] > 0


@pytest.mark.gpu
def test_ingestion_path_matches_oracle(oracle, tmp_path):
    """Product ingestion end to end from C++: rt_obj_load (committed OBJ) + rt_image_load (committed
    JPEG) -> rt_scene_build_ex("door") -> draw, against the oracle on the same decoded assets
    (rt_obj_load is pinned to assimp in test_obj_cpu.py, rt_image_decode to stb_image in
    test_image_cpu.py)."""
    from raytracing_gpu_amd import assets

    obj = os.path.join(GOLD, "obj", "case1.obj")
    tex = os.path.join(GOLD, "jpeg", "rgb444.jpg")
    img, lines = _rt_main(tmp_path, "door", 96, 2, 2, "--obj", obj, "--tex", tex)
    m = assets.load_obj(obj)
    t = assets.load_image(tex)
    s = oracle.RefScene("door", images=[t], meshes=[(m.tris, True, 0)])
    H = img.shape[0]
    qs, segs = [], 0
    for f in range(2):
        fb, c, _ = s.render(96, H, 2, f, 50, oracle.REF_CAM_REF_SLOT0)
        qs.append(oracle.quantize_fb(fb, 96, H))
        segs += c["segments"]
    want = oracle.average(qs, 96, H)
    assert np.array_equal(img, want)
    assert lines[-1]["segments"] == segs
    # the mesh is in view: a third of the pixels are not background
    assert (np.abs(img.astype(int) - img[0, 0].astype(int)).sum(-1) > 12).mean() > 0.2
