"""Golden vectors for the stb_image-exact JPEG decoder (raytracing_gpu_amd/csrc/rt_image.cpp).

Writes small synthetic JPEGs (this project's own images, encoded by Pillow with the sampling
layouts, restart intervals and odd sizes a decoder must handle) into jpeg/, decodes each with the
reference's vendored stb_image v2.26 (compiled in place: `make -C oracle ref` ->
oracle/_ref/libref_stbi.so, stbi_load(path, .., 0) as texture.h:173 calls it) and stores the
bytes in jpeg/expected.npz.  Run in this container only: python tests/golden/make_jpeg_golden.py
"""
import ctypes
import io
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

CASES = [  # name, height, width, mode, Pillow save options
    ("rgb444", 40, 56, "RGB", dict(quality=90, subsampling=0)),
    ("rgb422_odd", 37, 53, "RGB", dict(quality=75, subsampling=1)),
    ("rgb420_odd", 45, 61, "RGB", dict(quality=85, subsampling=2)),
    ("rgb420_restart", 64, 80, "RGB", dict(quality=60, subsampling=2, restart_marker_blocks=5)),
    ("grey_odd", 29, 35, "L", dict(quality=80)),
    ("rgb420_q100", 33, 33, "RGB", dict(quality=100, subsampling=2)),
]


def image(h, w, mode, seed):
    from raytracing_gpu_amd import assets

    a = assets.synthetic_image(w, h, 3, seed)
    rs = np.random.RandomState(seed)
    a = np.clip(a.astype(np.int32) + rs.randint(-40, 40, a.shape), 0, 255).astype(np.uint8)
    return Image.fromarray(a).convert(mode)


def main():
    lib = os.path.join(ROOT, "oracle", "_ref", "libref_stbi.so")
    if not os.path.exists(lib):
        raise SystemExit("build the reference stb_image first: make -C oracle ref")
    L = ctypes.CDLL(lib)
    L.ref_stbi_load.restype = ctypes.c_void_p
    L.ref_stbi_load.argtypes = [ctypes.c_char_p] + [ctypes.POINTER(ctypes.c_int)] * 3
    L.ref_stbi_free.argtypes = [ctypes.c_void_p]
    out = {}
    os.makedirs(os.path.join(HERE, "jpeg"), exist_ok=True)
    for k, (name, h, w, mode, opts) in enumerate(CASES):
        b = io.BytesIO()
        image(h, w, mode, 100 + k).save(b, "JPEG", **opts)
        path = os.path.join(HERE, "jpeg", name + ".jpg")
        with open(path, "wb") as f:
            f.write(b.getvalue())
        W, H, C = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        p = L.ref_stbi_load(path.encode(), ctypes.byref(W), ctypes.byref(H), ctypes.byref(C))
        a = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(H.value, W.value, C.value))
        out[name] = a.copy()
        L.ref_stbi_free(p)
        print(name, out[name].shape)
    np.savez_compressed(os.path.join(HERE, "jpeg", "expected.npz"), **out)


if __name__ == "__main__":
    main()
