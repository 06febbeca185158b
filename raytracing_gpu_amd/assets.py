"""Scene assets: decoded images and triangle meshes handed to rt_scene_build_ex.

The reference reads these files while it builds a scene: stbi_load for textures
(texture.h:166-203, make_image) and assimp for OBJ meshes (triangle_mesh.h:129-352,
create_meshes).  Here the host decodes them and passes plain arrays through the C ABI:

- `load_image(path)` decodes JPEGs with the native decoder restating stb_image v2.26 (the
  reference's vendored loader) bit-exactly, and lossless formats with Pillow.
- `synthetic_image(w, h)` is a deterministic texture of any shape (tests and benchmarks on a GPU
  box, where the reference's files do not exist).
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, Structure, c_float, c_int32, c_uint8, c_void_p

import numpy as np

TRI_FLOATS = 24  # v0 v1 v2 (9), n0 n1 n2 (9), u0 v0 u1 v1 u2 v2 (6)


class rt_image_asset(Structure):
    _fields_ = [("width", c_int32), ("height", c_int32), ("bytes_per_pixel", c_int32), ("pad", c_int32),
                ("data", POINTER(c_uint8))]


class rt_mesh_asset(Structure):
    _fields_ = [("n_triangles", c_int32), ("vertex_normals", c_int32), ("image", c_int32), ("pad", c_int32),
                ("data", POINTER(c_float))]


class rt_scene_assets(Structure):
    _fields_ = [("n_images", c_int32), ("n_meshes", c_int32), ("images", POINTER(rt_image_asset)),
                ("meshes", POINTER(rt_mesh_asset))]


class Mesh:
    """Triangle soup of one mesh as create_meshes_d builds it: (n, 24) float32 rows."""

    def __init__(self, tris: np.ndarray, vertex_normals: bool = True, image: int = 0, texture_path: str = ""):
        self.tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, TRI_FLOATS)
        self.vertex_normals = bool(vertex_normals)
        self.image = int(image)
        self.texture_path = texture_path

    def __len__(self) -> int:
        return self.tris.shape[0]


def decode_jpeg(data: bytes) -> np.ndarray:
    """Baseline JPEG -> HxWxC uint8 with stb_image v2.26's arithmetic (rt_image_decode): the texel
    bytes the reference's make_image() uploads."""
    from . import RtError, lib

    h = c_void_p()
    buf = np.frombuffer(data, np.uint8)
    rc = lib().rt_image_decode(buf.ctypes.data, len(buf), ctypes.byref(h))
    if rc != 0:
        raise RtError(f"rt_image_decode failed with status {rc} (not a baseline grey/YCbCr JPEG?)")
    try:
        v = ctypes.cast(lib().rt_image_view(h), POINTER(rt_image_asset)).contents
        n = v.width * v.height * v.bytes_per_pixel
        return np.ctypeslib.as_array(v.data, shape=(n,)).copy().reshape(v.height, v.width, v.bytes_per_pixel)
    finally:
        lib().rt_image_free(h)


def load_image(path: str) -> np.ndarray:
    """Decode an image file to HxWxC uint8 like stbi_load(path, .., 0).  JPEGs go through the native
    stb-exact decoder; lossless formats (PNG, ...) through Pillow, whose bytes are the file's."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:2] == b"\xff\xd8":
        return decode_jpeg(data)
    from PIL import Image

    im = Image.open(path)
    if im.mode not in ("L", "LA", "RGB", "RGBA"):
        im = im.convert("RGB")
    a = np.asarray(im, dtype=np.uint8)
    return a[:, :, None] if a.ndim == 2 else a


def synthetic_image(width: int, height: int, channels: int = 3, seed: int = 1984) -> np.ndarray:
    """Deterministic test texture: smooth gradients plus a hashed high-frequency component."""
    y, x = np.mgrid[0:height, 0:width].astype(np.uint32)
    h = (x * np.uint32(73856093)) ^ (y * np.uint32(19349663)) ^ np.uint32(seed * 83492791 & 0xFFFFFFFF)
    out = np.empty((height, width, channels), np.uint8)
    for c in range(channels):
        g = ((x * (c + 1) * 255) // max(width - 1, 1) + (y * (3 - c) * 255) // max(height - 1, 1)) & 255
        out[:, :, c] = ((g + ((h >> (8 * c)) & 31)) & 255).astype(np.uint8)
    return out


def pack_assets(images, meshes):
    """ctypes view of images/meshes; returns (objects to keep alive, pointer to rt_scene_assets)."""
    imgs = [np.ascontiguousarray(i, dtype=np.uint8) for i in images]
    imgs = [i[:, :, None] if i.ndim == 2 else i for i in imgs]
    ia = (rt_image_asset * max(len(imgs), 1))()
    for k, im in enumerate(imgs):
        ia[k] = rt_image_asset(im.shape[1], im.shape[0], im.shape[2], 0, im.ctypes.data_as(POINTER(c_uint8)))
    ma = (rt_mesh_asset * max(len(meshes), 1))()
    for k, m in enumerate(meshes):
        ma[k] = rt_mesh_asset(len(m), 1 if m.vertex_normals else 0, m.image, 0, m.tris.ctypes.data_as(POINTER(c_float)))
    a = rt_scene_assets(len(imgs), len(meshes), ia, ma)
    keep = (imgs, meshes, ia, ma, a)
    return keep, ctypes.cast(ctypes.pointer(a), c_void_p)


def synthetic_mesh(nu: int = 24, nv: int = 32, image: int = 0) -> Mesh:
    """Deterministic test mesh near the door scene's look-at point: a wavy sheet of nu x nv quads
    (two triangles each) with analytic vertex normals and uvs in [0, 1]."""
    u = np.linspace(0.0, 1.0, nu + 1, dtype=np.float64)
    v = np.linspace(0.0, 1.0, nv + 1, dtype=np.float64)
    U, Vv = np.meshgrid(u, v, indexing="ij")
    X = U - 0.5
    Y = 2.0 * Vv
    Z = 0.15 * np.sin(6.0 * U) * np.cos(4.0 * Vv)
    dzdu = 0.9 * np.cos(6.0 * U) * np.cos(4.0 * Vv)
    dzdv = -0.6 * np.sin(6.0 * U) * np.sin(4.0 * Vv)
    # normal = (1, 0, dzdu) x (0, 2, dzdv) normalised
    N = np.stack([-2.0 * dzdu, -dzdv, 2.0 * np.ones_like(U)], axis=-1)
    N /= np.linalg.norm(N, axis=-1, keepdims=True)
    P = np.stack([X, Y, Z], axis=-1)
    rows = []
    for i in range(nu):
        for j in range(nv):
            q = [(i, j), (i + 1, j), (i + 1, j + 1), (i, j + 1)]
            for a, b, c in ((0, 1, 2), (0, 2, 3)):
                ids = (q[a], q[b], q[c])
                row = [*P[ids[0]], *P[ids[1]], *P[ids[2]], *N[ids[0]], *N[ids[1]], *N[ids[2]]]
                for k in ids:
                    row += [U[k], Vv[k]]
                rows.append(row)
    return Mesh(np.asarray(rows, np.float32), vertex_normals=True, image=image)


class rt_obj_info(Structure):
    _fields_ = [("n_triangles", c_int32), ("n_meshes", c_int32), ("n_vertices", c_int32), ("n_textures", c_int32),
                ("triangles", POINTER(c_float)), ("texture", ctypes.c_char_p)]


OBJ_INDEX_REFERENCE = 0  # create_meshes_d: per-mesh local indices into the concatenated arrays (H16)
OBJ_INDEX_GLOBAL = 1     # each mesh's indices offset by its first vertex


def load_obj(path: str, index_mode: int = OBJ_INDEX_REFERENCE) -> Mesh:
    """Import an OBJ the way the reference's create_meshes() does (assimp Triangulate|GenNormals,
    processNode order), through rt_obj_load.  Returns a Mesh (vertex normals, image 0) whose
    texture_path is the first diffuse texture of its materials."""
    from . import RtError, lib

    h = c_void_p()
    rc = lib().rt_obj_load(path.encode(), int(index_mode), ctypes.byref(h))
    if rc != 0:
        raise RtError(f"rt_obj_load({path!r}) failed with status {rc}")
    try:
        info = ctypes.cast(lib().rt_obj_view(h), POINTER(rt_obj_info)).contents
        n = info.n_triangles
        tris = np.ctypeslib.as_array(info.triangles, shape=(n * TRI_FLOATS,)).copy() if n else np.zeros(0, np.float32)
        m = Mesh(tris, vertex_normals=True, image=0, texture_path=(info.texture or b"").decode())
        m.n_meshes = info.n_meshes
        m.n_textures = info.n_textures
        return m
    finally:
        lib().rt_obj_free(h)


def mesh_from_arrays(vertices, normals, uvs, faces, index_mode: int = OBJ_INDEX_REFERENCE, image: int = 0) -> Mesh:
    """create_meshes_d (triangle_mesh.h:147-204) over per-mesh arrays in processNode order, for
    callers that import meshes themselves: vertices/normals (n_k, 3), uvs (n_k, 2), faces (m_k, 3)
    per mesh.  OBJ_INDEX_REFERENCE indexes the concatenated arrays with local indices (H16)."""
    V = np.concatenate([np.asarray(v, np.float32).reshape(-1, 3) for v in vertices])
    N = np.concatenate([np.asarray(n, np.float32).reshape(-1, 3) for n in normals])
    UV = np.concatenate([np.asarray(u, np.float32).reshape(-1, 2) for u in uvs])
    idx, off = [], 0
    for v, f in zip(vertices, faces):
        f = np.asarray(f, np.int64).reshape(-1, 3)
        idx.append(f + (off if index_mode == OBJ_INDEX_GLOBAL else 0))
        off += len(v)
    I = np.concatenate(idx)
    tris = np.concatenate([V[I].reshape(-1, 9), N[I].reshape(-1, 9), UV[I].reshape(-1, 6)], axis=1)
    return Mesh(tris, vertex_normals=True, image=image)


def door_mesh_from_fixture(path: str, index_mode: int = OBJ_INDEX_REFERENCE) -> Mesh:
    """The C4 door mesh from tests/golden/door_assimp.npz (assimp's import of the reference's
    assets/door/door.obj, see tests/golden/make_obj_golden.py), for runs where the reference's
    files are absent (GPU boxes)."""
    d = np.load(path)
    n = int(d["n_meshes"][0])
    return mesh_from_arrays([d[f"v{k}"] for k in range(n)], [d[f"n{k}"] for k in range(n)],
                            [d[f"uv{k}"] for k in range(n)], [d[f"f{k}"][:, :3] for k in range(n)], index_mode)
