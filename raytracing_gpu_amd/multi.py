"""ctypes mirror of include/rt_multi.h: the C++ multi-GPU draw() (librt_multi.so).

One process drives every rank: one rt_ctx per device, one host thread per rank (render_init +
render + resolve of its row bands), ONE ncclGather of the 8-bit rows to rank 0 over xGMI, host
assembly in PNG order (csrc/rt_multi.cpp).  This is the product's multi-GPU driver; bench.py
uses it for `--gpus N` when no torch.distributed launcher started it.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_uint8, c_void_p

import numpy as np

from . import lib as _rt_lib
from . import rt_counters, rt_render_args, rt_scene_soa, RtError

MULTI_PATH = os.environ.get("RT_MULTI_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt_multi.so")  # override: experiments
RT_GATHER_RCCL = 0
RT_GATHER_HOST = 1
MAX_RANKS = 16


class rt_multi_timing(ctypes.Structure):
    _fields_ = [("total_ms", c_float), ("render_ms_max", c_float), ("gather_ms", c_float),
                ("gather_bytes", c_float), ("render_ms", c_float * MAX_RANKS), ("kernel_ms", c_float * MAX_RANKS),
                ("warm", c_int32), ("pad", c_int32)]


ABI = {
    "rt_multi_create": (c_int, [c_int32, POINTER(c_int32), c_int32, POINTER(c_void_p)]),
    "rt_multi_destroy": (c_int, [c_void_p]),
    "rt_multi_last_error": (c_char_p, [c_void_p]),
    "rt_multi_upload": (c_int, [c_void_p, POINTER(rt_scene_soa)]),
    "rt_multi_draw": (c_int, [c_void_p, POINTER(rt_render_args), POINTER(c_uint8), POINTER(rt_counters),
                              POINTER(rt_multi_timing)]),
}

_mlib = None


def lib() -> ctypes.CDLL:
    global _mlib
    if _mlib is None:
        if not os.path.exists(MULTI_PATH):
            raise RuntimeError(f"{MULTI_PATH} missing: run `python -m raytracing_gpu_amd._build`")
        _rt_lib()  # torch's HIP runtime, then librt_hip.so (librt_multi.so links both)
        L = ctypes.CDLL(MULTI_PATH)
        for name, (res, args) in ABI.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _mlib = L
    return _mlib


class Multi:
    """rt_multi over `devices` (one rank each; RT_GATHER_HOST lets ranks share a device)."""

    def __init__(self, devices, gather: int = RT_GATHER_RCCL):
        self.n = len(devices)
        devs = (c_int32 * self.n)(*devices)
        self._m = c_void_p()
        rc = lib().rt_multi_create(self.n, devs, gather, ctypes.byref(self._m))
        if rc != 0:
            raise RtError(f"rt_multi_create({list(devices)}, gather={gather}) failed with status {rc}")

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            msg = lib().rt_multi_last_error(self._m)
            raise RtError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def upload(self, scene) -> None:
        self._check(lib().rt_multi_upload(self._m, ctypes.byref(scene.soa)), "rt_multi_upload")

    def draw(self, args: rt_render_args) -> tuple[np.ndarray, dict, dict]:
        """(PNG-order HxWx3 image, counters summed over ranks, timing)."""
        img = np.zeros((args.height, args.width, 3), np.uint8)
        cnt = rt_counters()
        tm = rt_multi_timing()
        self._check(lib().rt_multi_draw(self._m, ctypes.byref(args), img.ctypes.data_as(POINTER(c_uint8)),
                                        ctypes.byref(cnt), ctypes.byref(tm)), "rt_multi_draw")
        timing = {"total_ms": tm.total_ms, "render_ms_max": tm.render_ms_max, "gather_ms": tm.gather_ms,
                  "gather_bytes": int(tm.gather_bytes), "render_ms": list(tm.render_ms[: self.n]),
                  "kernel_ms": list(tm.kernel_ms[: self.n]), "warm": int(tm.warm)}
        return img, cnt.as_dict(), timing

    def close(self) -> None:
        if getattr(self, "_m", None):
            lib().rt_multi_destroy(self._m)
            self._m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
