"""Texture decoding (csrc/rt_image.cpp) against the reference's own stb_image v2.26.

Golden vectors: tests/golden/make_jpeg_golden.py (stb_image compiled in place from the
reference, oracle/_ref).  Bit-exact texel bytes.
"""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
JPEG = os.path.join(HERE, "golden", "jpeg")
REF_TEXTURES = ["/root/reference/textures/earthmap.jpg", "/root/reference/textures/earthmap_old.jpg",
                "/root/reference/assets/door/Door_C.jpg", "/root/reference/assets/door/Reflexion.jpg"]
STBI = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libref_stbi.so")


@pytest.mark.parametrize("name", ["rgb444", "rgb422_odd", "rgb420_odd", "rgb420_restart", "grey_odd", "rgb420_q100"])
def test_jpeg_cases_match_stb_image(rtlib, name):
    from raytracing_gpu_amd import assets

    want = np.load(os.path.join(JPEG, "expected.npz"))[name]
    got = assets.load_image(os.path.join(JPEG, name + ".jpg"))
    assert got.shape == want.shape and np.array_equal(got, want)


def _stbi(path):
    import ctypes

    L = ctypes.CDLL(STBI)
    L.ref_stbi_load.restype = ctypes.c_void_p
    L.ref_stbi_load.argtypes = [ctypes.c_char_p] + [ctypes.POINTER(ctypes.c_int)] * 3
    L.ref_stbi_free.argtypes = [ctypes.c_void_p]
    W, H, C = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    p = L.ref_stbi_load(path.encode(), ctypes.byref(W), ctypes.byref(H), ctypes.byref(C))
    a = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(H.value, W.value, C.value)).copy()
    L.ref_stbi_free(p)
    return a


@pytest.mark.skipif(not (os.path.exists(STBI) and os.path.exists(REF_TEXTURES[0])), reason="reference not present")
@pytest.mark.parametrize("path", REF_TEXTURES, ids=lambda p: os.path.basename(p))
def test_reference_textures_match_stb_image(rtlib, path):
    from raytracing_gpu_amd import assets

    want = _stbi(path)
    got = assets.load_image(path)
    assert got.shape == want.shape and np.array_equal(got, want)


def test_rejects_non_jpeg(rtlib):
    from raytracing_gpu_amd import assets

    with pytest.raises(Exception):
        assets.decode_jpeg(b"\x89PNG\r\n\x1a\n" + b"\0" * 64)


def _with_sos_selector(data: bytes, tt: int) -> bytes:
    """The file with the first scan component's Huffman table selector byte replaced."""
    k = data.index(b"\xff\xda")
    # FFDA, Ls (2), Ns (1), then (Cs, Td<<4|Ta) pairs
    b = bytearray(data)
    b[k + 6] = tt
    return bytes(b)


@pytest.mark.parametrize("tt", [0x50, 0x05, 0xF0, 0x22], ids=["dc5", "ac5", "dc15", "undefined2"])
def test_rejects_bad_huffman_selectors(rtlib, tt):
    """SOS table selectors past the 4 tables, or naming a table no DHT defined, are rejected (stb_image
    v2.26: 'bad DC huff' / 'bad AC huff') instead of indexing out of bounds / uninitialised tables."""
    from raytracing_gpu_amd import assets

    with open(os.path.join(JPEG, "rgb444.jpg"), "rb") as f:
        data = f.read()
    assets.decode_jpeg(_with_sos_selector(data, 0x00))  # table 0/0 is defined: still decodes
    with pytest.raises(Exception):
        assets.decode_jpeg(_with_sos_selector(data, tt))
