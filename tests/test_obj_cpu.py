"""OBJ ingestion (csrc/rt_obj.cpp) against assimp's own import of the same files.

Golden vectors: tests/golden/make_obj_golden.py (assimp v3.3 embedded in this container's Qt3D
plugin; the reference used assimp 5.x).  Bit-exact positions, normals, uvs and triangle order.
"""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
DOOR = "/root/reference/assets/door/door.obj"


def _golden_triangles(npz, global_index):
    """Triangles as create_meshes_d builds them from processMesh's concatenated arrays."""
    d = np.load(npz)
    n = int(d["n_meshes"][0])
    V = np.concatenate([d[f"v{k}"] for k in range(n)])
    N = np.concatenate([d[f"n{k}"] for k in range(n)])
    UV = np.concatenate([d[f"uv{k}"] for k in range(n)])
    rows, off = [], 0
    for k in range(n):
        for f in d[f"f{k}"]:
            ids = [int(i) + (off if global_index else 0) for i in f if i >= 0]
            rows.append(np.concatenate([V[ids].ravel(), N[ids].ravel(), UV[ids].ravel()]))
        off += len(d[f"v{k}"])
    return np.asarray(rows, np.float32).reshape(-1, 24), n


@pytest.mark.parametrize("case", ["case1", "case2"])
@pytest.mark.parametrize("mode", [0, 1], ids=["reference_index", "global_index"])
def test_obj_cases_match_assimp(rtlib, case, mode):
    from raytracing_gpu_amd import assets

    m = assets.load_obj(os.path.join(GOLD, "obj", case + ".obj"), mode)
    want, nmesh = _golden_triangles(os.path.join(GOLD, "obj", case + ".npz"), mode == 1)
    assert m.n_meshes == nmesh
    assert m.tris.shape == want.shape
    assert np.array_equal(m.tris.view(np.uint32), want.view(np.uint32))


def test_obj_case1_texture(rtlib):
    from raytracing_gpu_amd import assets

    m = assets.load_obj(os.path.join(GOLD, "obj", "case1.obj"))
    assert m.n_textures == 2 and m.texture_path.endswith("obj/red.png")


@pytest.mark.skipif(not os.path.exists(DOOR), reason="reference assets not present")
@pytest.mark.parametrize("mode", [0, 1], ids=["reference_index", "global_index"])
def test_door_obj_matches_assimp(rtlib, mode):
    from raytracing_gpu_amd import assets

    m = assets.load_obj(DOOR, mode)
    want, nmesh = _golden_triangles(os.path.join(GOLD, "door_assimp.npz"), mode == 1)
    assert (m.n_meshes, len(m)) == (nmesh, 4330) == (6, want.shape[0])
    assert np.array_equal(m.tris.view(np.uint32), want.view(np.uint32))
    assert m.n_textures == 1 and m.texture_path.endswith("door/Door_C.jpg")


def test_mesh_from_arrays_matches_loader(rtlib):
    from raytracing_gpu_amd import assets

    path = os.path.join(GOLD, "door_assimp.npz")
    for mode in (0, 1):
        want, _ = _golden_triangles(path, mode == 1)
        got = assets.door_mesh_from_fixture(path, mode)
        assert np.array_equal(got.tris.view(np.uint32), want.view(np.uint32))
