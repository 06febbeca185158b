"""ctypes wrapper of the CPU oracle (oracle/_build/libref_cpu.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker or the CPU baseline — never as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libref_cpu.so")

REF_CAM_REF_SLOT0 = 0
REF_CAM_PER_PIXEL = 1


class ref_counters(ctypes.Structure):
    _fields_ = [("segments", ctypes.c_longlong), ("node_tests", ctypes.c_longlong),
                ("prim_tests", ctypes.c_longlong), ("samples", ctypes.c_longlong)]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        L.ref_scene_create.argtypes = [ctypes.c_char_p, c_int, POINTER(c_void_p)]
        L.ref_scene_create_ex.argtypes = [ctypes.c_char_p, c_int, c_void_p, POINTER(c_void_p)]
        L.ref_scene_destroy.argtypes = [c_void_p]
        L.ref_scene_aspect.argtypes = [c_void_p]
        L.ref_scene_aspect.restype = c_float
        L.ref_scene_h20.argtypes = [c_void_p]
        L.ref_scene_table.argtypes = [c_void_p, c_void_p, c_int]
        L.ref_scene_bvh_axes.argtypes = [c_void_p, c_void_p, c_int]
        L.ref_scene_set_camera.argtypes = [c_void_p, POINTER(c_float), POINTER(c_float), c_float, c_float, c_float]
        L.ref_render.argtypes = [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                 c_void_p, c_void_p, POINTER(ref_counters)]
        L.ref_quantize_fb.argtypes = [c_void_p, c_int, c_int, c_void_p]
        L.ref_average.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p]
        L.ref_xorwow_init.argtypes = [c_uint64, c_uint64, c_uint64, POINTER(c_uint32)]
        L.ref_xorwow_next.argtypes = [POINTER(c_uint32)]
        L.ref_xorwow_next.restype = c_uint32
        L.ref_xorwow_uniform.argtypes = [POINTER(c_uint32)]
        L.ref_xorwow_uniform.restype = c_float
        L.ref_xorwow_jump_matrix.argtypes = [c_int, c_int, POINTER(c_uint32)]
        _lib = L
    return _lib


class _Image(ctypes.Structure):
    _fields_ = [("width", c_int), ("height", c_int), ("bytes_per_pixel", c_int), ("pad", c_int),
                ("data", c_void_p)]


class _Mesh(ctypes.Structure):
    _fields_ = [("n_triangles", c_int), ("vertex_normals", c_int), ("image", c_int), ("pad", c_int),
                ("data", c_void_p)]


class _Assets(ctypes.Structure):
    _fields_ = [("n_images", c_int), ("n_meshes", c_int), ("images", POINTER(_Image)), ("meshes", POINTER(_Mesh))]


class RefScene:
    def __init__(self, name: str, rtl: bool = False, images=None, meshes=None):
        """images: HxWxC uint8 arrays; meshes: (tris (n, 24) float32, vertex_normals, image index)."""
        self.name = name
        self._h = c_void_p()
        if images is None and meshes is None:
            rc = lib().ref_scene_create(name.encode(), 1 if rtl else 0, ctypes.byref(self._h))
        else:
            imgs = [np.ascontiguousarray(i, np.uint8) for i in (images or [])]
            imgs = [i[:, :, None] if i.ndim == 2 else i for i in imgs]
            ms = [(np.ascontiguousarray(t, np.float32).reshape(-1, 24), vn, im) for t, vn, im in (meshes or [])]
            ia = (_Image * max(len(imgs), 1))()
            for k, im in enumerate(imgs):
                ia[k] = _Image(im.shape[1], im.shape[0], im.shape[2], 0, im.ctypes.data)
            ma = (_Mesh * max(len(ms), 1))()
            for k, (t, vn, im) in enumerate(ms):
                ma[k] = _Mesh(t.shape[0], 1 if vn else 0, im, 0, t.ctypes.data)
            a = _Assets(len(imgs), len(ms), ia, ma)
            rc = lib().ref_scene_create_ex(name.encode(), 1 if rtl else 0, ctypes.byref(a), ctypes.byref(self._h))
        if rc != 0:
            raise ValueError(f"unknown oracle scene {name!r} (or missing assets)")

    @property
    def aspect(self) -> float:
        return float(lib().ref_scene_aspect(self._h))

    @property
    def h20(self) -> bool:
        return bool(lib().ref_scene_h20(self._h))

    def table(self) -> np.ndarray:
        t = np.zeros((4096, 13), np.float32)
        n = lib().ref_scene_table(self._h, t.ctypes.data, 4096)
        return t[:n].copy()

    def bvh_axes(self) -> np.ndarray:
        a = np.zeros(1 << 16, np.int32)
        n = lib().ref_scene_bvh_axes(self._h, a.ctypes.data, a.size)
        return a[:n].copy()

    def set_camera(self, frm, at, vfov, aperture, focus) -> None:
        f = (c_float * 3)(*frm)
        a = (c_float * 3)(*at)
        lib().ref_scene_set_camera(self._h, f, a, vfov, aperture, focus)

    def render(self, W: int, H: int, spp: int, fb_id: int = 0, max_depth: int = 50,
               cam_mode: int = REF_CAM_REF_SLOT0, rows=None, threads: int = 0,
               fb: np.ndarray | None = None, seg_per_pixel: bool = False):
        """Render one fb.  rows = (row0, row_step) subset; returns (fb[H*W*3] float32, counters, segs)."""
        if fb is None:
            fb = np.zeros(W * H * 3, np.float32)
        segs = np.zeros(W * H, np.int32) if seg_per_pixel else None
        row0, step = rows if rows is not None else (0, 1)
        c = ref_counters()
        rc = lib().ref_render(self._h, W, H, spp, fb_id, max_depth, cam_mode, row0, step, threads,
                              fb.ctypes.data, segs.ctypes.data if segs is not None else None, ctypes.byref(c))
        if rc != 0:
            raise RuntimeError("ref_render failed")
        return fb, c.as_dict(), segs

    def __del__(self):
        try:
            if self._h:
                lib().ref_scene_destroy(self._h)
        except Exception:
            pass


def quantize_fb(fb: np.ndarray, W: int, H: int) -> np.ndarray:
    out = np.zeros(W * H * 3, np.uint8)
    lib().ref_quantize_fb(np.ascontiguousarray(fb, np.float32).ctypes.data, W, H, out.ctypes.data)
    return out


def average(ppms: list, W: int, H: int) -> np.ndarray:
    """average_images over quantised fbs (each in PPM/PNG row order); returns HxWx3 uint8."""
    arrs = [np.ascontiguousarray(p, np.uint8) for p in ppms]
    ptrs = (c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    out = np.zeros(W * H * 3, np.uint8)
    lib().ref_average(ptrs, len(arrs), W, H, out.ctypes.data)
    return out.reshape(H, W, 3)


def draw(name: str, W: int, H: int, spp: int, no_fb: int, max_depth: int = 50,
         cam_mode: int = REF_CAM_REF_SLOT0, threads: int = 0):
    """Oracle draw(): returns (PNG-order image, list of per-fb float fbs, total counters)."""
    s = RefScene(name)
    fbs, qs = [], []
    tot = {"segments": 0, "node_tests": 0, "prim_tests": 0, "samples": 0}
    for f in range(no_fb):
        fb, c, _ = s.render(W, H, spp, f, max_depth, cam_mode, threads=threads)
        fbs.append(fb)
        qs.append(quantize_fb(fb, W, H))
        for k in tot:
            tot[k] += c[k]
    return average(qs, W, H), fbs, tot


def xorwow_init(seed: int, subsequence: int, offset: int = 0) -> np.ndarray:
    st = (c_uint32 * 6)()
    lib().ref_xorwow_init(seed, subsequence, offset, st)
    return np.frombuffer(st, np.uint32).copy()


def xorwow_uniforms(seed: int, subsequence: int, n: int, offset: int = 0) -> np.ndarray:
    st = (c_uint32 * 6)()
    lib().ref_xorwow_init(seed, subsequence, offset, st)
    return np.array([lib().ref_xorwow_uniform(st) for _ in range(n)], np.float32)


def jump_matrix(which: int, i: int) -> np.ndarray:
    m = (c_uint32 * 800)()
    lib().ref_xorwow_jump_matrix(which, i, m)
    return np.frombuffer(m, np.uint32).copy()
