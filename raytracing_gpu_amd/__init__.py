"""raytracing_gpu_amd — MI355X (gfx950) drop-in for the per-pixel render path of
daRoyalCacti/Raytracing_GPU.

Host mirror of the reference's interface for that path (names and argument meaning kept):

  * ``render_settings``  — render.h:21-50 (image_width, samples_per_pixel_per_fb, no_fb, ...)
  * ``scene`` / ``Scene.builtin(name)`` — struct scene and its subclasses, scenes.h:36-621
  * ``draw(scene, settings)`` — render.h:118-174 (render_init, no_fb render launches, per-fb
    quantise + square-average); returns the PNG raster instead of writing ./image.png
  * ``Context.render_init / render / resolve`` — the kernels render_init (render.h:84-92) and
    render (render.h:94-113) behind the C ABI of include/rt_hip.h

Everything is computed by librt_hip.so (hand-written HIP for gfx950).  There is no CPU fallback:
if the library is missing or the device call fails, the call raises.
"""
from __future__ import annotations

import ctypes
import sys
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_int64, c_uint8, c_uint64, c_void_p
from dataclasses import dataclass

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RT_HIP_LIB") or os.path.join(_PKG, "librt_hip.so")  # override: experiments

RT_CAM_REF_SLOT0 = 0
RT_CAM_PER_PIXEL = 1
RT_FLAG_EXACT_TRAVERSAL = 1
RT_FLAG_AUDIT = 2
RT_FLAG_NO_LDS = 4
RT_FLAG_WIDEST = 8
RT_FLAG_NO_STEP = 16
RT_FLAG_NO_SCHEDULE = 32
RT_FLAG_NO_CAMERA_BINS = 64
RT_FLAG_NO_SPLIT = 128
RT_FLAG_FRESH = 256
RT_SCHED_PREVIOUS = 1
RT_SCHED_SPLIT_REPLAY = 2
RT_SCHED_PROBE = 4

PRIM_SPHERE, PRIM_MOVING_SPHERE, PRIM_RECT_XY, PRIM_RECT_XZ, PRIM_RECT_YZ, PRIM_TRIANGLE = range(6)
OBJ_PRIM, OBJ_LIST, OBJ_BVH, OBJ_XFORM, OBJ_MEDIUM = range(5)
MAT_LAMBERTIAN, MAT_METAL, MAT_DIELECTRIC, MAT_DIFFUSE_LIGHT, MAT_ISOTROPIC = range(5)

BUILTIN_SCENES = ("basic", "first", "big1", "two_spheres", "two_perlin", "cornell", "cornell_smoke")


# ---------------------------------------------------------------- C structs (include/rt_hip.h)
class rt_camera(ctypes.Structure):
    _fields_ = [("origin", c_float * 3), ("lower_left", c_float * 3), ("horizontal", c_float * 3),
                ("vertical", c_float * 3), ("u", c_float * 3), ("v", c_float * 3), ("w", c_float * 3),
                ("lens_radius", c_float), ("time0", c_float), ("time1", c_float)]


class rt_prim(ctypes.Structure):
    _fields_ = [("p", c_float * 10), ("type", c_int32), ("material", c_int32)]


class rt_bvh_node(ctypes.Structure):
    _fields_ = [("lo", c_float * 3), ("leaf_a", c_int32), ("hi", c_float * 3), ("leaf_b", c_int32)]


class rt_object(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("a", c_int32), ("b", c_int32), ("c", c_int32), ("f", c_float * 8)]


class rt_material(ctypes.Structure):
    _fields_ = [("type", c_int32), ("texture", c_int32), ("param", c_float), ("pad", c_int32)]


class rt_texture(ctypes.Structure):
    _fields_ = [("type", c_int32), ("a", c_int32), ("b", c_int32), ("pad", c_int32),
                ("color", c_float * 3), ("scale", c_float)]


class rt_scene_soa(ctypes.Structure):
    _fields_ = [("camera", rt_camera), ("background", c_float * 3), ("aspect", c_float),
                ("world", POINTER(c_int32)), ("n_world", c_int32),
                ("objects", POINTER(rt_object)), ("n_objects", c_int32),
                ("prims", POINTER(rt_prim)), ("n_prims", c_int32),
                ("triangles", c_void_p), ("n_triangles", c_int32),
                ("nodes", POINTER(rt_bvh_node)), ("n_nodes", c_int32),
                ("materials", POINTER(rt_material)), ("n_materials", c_int32),
                ("textures", POINTER(rt_texture)), ("n_textures", c_int32),
                ("perlins", c_void_p), ("n_perlins", c_int32),
                ("images", c_void_p), ("n_images", c_int32),
                ("texels", c_void_p), ("n_texels", c_int64)]


class rt_render_args(ctypes.Structure):
    _fields_ = [("width", c_int32), ("height", c_int32), ("spp", c_int32), ("fb_first", c_int32),
                ("fb_count", c_int32), ("max_depth", c_int32), ("cam_mode", c_int32),
                ("band_rows", c_int32), ("band_first", c_int32), ("band_stride", c_int32),
                ("stats", c_int32), ("flags", c_int32), ("seed", c_uint64)]


class rt_ctx_options(ctypes.Structure):
    """include/rt_hip.h rt_ctx_options: implementation choices that change no pixel (defaults from
    rt_ctx_options_default, the measured product configuration)."""
    _fields_ = [("world_tree", c_int32), ("quantized_tree", c_int32), ("merged_search", c_int32),
                ("merge_order", c_int32), ("dedup_triangles", c_int32), ("shade_min", c_int32),
                ("bins_min_items_per_lane", c_float), ("split_min_segments", c_float), ("split_order", c_int32),
                ("cost_shift", c_int32), ("long_pct", c_float), ("probe_schedule", c_int32),
                ("probe_max_items_per_lane", c_float), ("probe_depth", c_int32),
                ("spread_first", c_int32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


RT_MERGE_ON, RT_MERGE_OFF, RT_MERGE_FALLBACK_ALL = range(3)
RT_ORDER_DISTANCE, RT_ORDER_LIST, RT_ORDER_REVERSED = range(3)
# Options every new Context starts from, on top of the library defaults (tests force the camera-ray
# tile lists on through this; the product leaves it empty).
DEFAULT_OPTIONS: dict = {}


class rt_counters(ctypes.Structure):
    _fields_ = [("segments", c_uint64), ("node_tests", c_uint64), ("prim_tests", c_uint64),
                ("samples", c_uint64), ("fallbacks", c_uint64)]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


# Every entry point of include/rt_hip.h: name -> (restype, argtypes)
ABI = {
    "rt_ctx_create": (c_int, [c_int, POINTER(c_void_p)]),
    "rt_ctx_destroy": (c_int, [c_void_p]),
    "rt_last_error": (c_char_p, [c_void_p]),
    "rt_ctx_options_default": (None, [POINTER(rt_ctx_options)]),
    "rt_ctx_set_options": (c_int, [c_void_p, POINTER(rt_ctx_options)]),
    "rt_ctx_get_options": (c_int, [c_void_p, POINTER(rt_ctx_options)]),
    "rt_owned_rows": (c_int32, [POINTER(rt_render_args), POINTER(c_int32)]),
    "rt_scene_upload": (c_int, [c_void_p, POINTER(rt_scene_soa)]),
    "rt_render_init": (c_int, [c_void_p, c_int32, c_int32, c_uint64]),
    "rt_read_states": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
    "rt_render": (c_int, [c_void_p, POINTER(rt_render_args), c_void_p, POINTER(rt_counters)]),
    "rt_last_render_ms": (c_float, [c_void_p]),
    "rt_last_kernel_ms": (c_float, [c_void_p]),
    "rt_last_render_kernel": (ctypes.c_char_p, [c_void_p]),
    "rt_last_render_schedule": (c_int32, [c_void_p]),
    "rt_audit_log": (c_int, [c_void_p, POINTER(c_float), c_int32]),
    "rt_resolve": (c_int, [c_void_p, POINTER(rt_render_args), c_void_p, c_void_p]),
    "rt_draw": (c_int, [c_void_p, POINTER(rt_render_args), POINTER(c_uint8), POINTER(rt_counters)]),
    "rt_scene_build": (c_int, [c_char_p, POINTER(c_void_p)]),
    "rt_scene_build_ex": (c_int, [c_char_p, c_void_p, POINTER(c_void_p)]),
    "rt_obj_load": (c_int, [c_char_p, c_int, POINTER(c_void_p)]),
    "rt_obj_view": (c_void_p, [c_void_p]),
    "rt_obj_free": (None, [c_void_p]),
    "rt_image_decode": (c_int, [c_void_p, ctypes.c_int64, POINTER(c_void_p)]),
    "rt_image_load": (c_int, [c_char_p, POINTER(c_void_p)]),
    "rt_image_view": (c_void_p, [c_void_p]),
    "rt_image_free": (None, [c_void_p]),
    "rt_scene_view": (POINTER(rt_scene_soa), [c_void_p]),
    "rt_scene_free": (None, [c_void_p]),
}

_lib = None


def lib() -> ctypes.CDLL:
    """Load librt_hip.so (raises if it has not been built: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `python -m raytracing_gpu_amd._build` "
                               "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        # torch (device memory, streams, RCCL) bundles its own libamdhip64.so.7: load it first so
        # this library binds to the same HIP runtime instance instead of a second copy.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in ABI.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class RtError(RuntimeError):
    pass


# ---------------------------------------------------------------- render_settings (render.h:21-50)
@dataclass
class render_settings:
    aspect_ratio: float = 16.0 / 9.0
    image_width: int = 1200
    image_height: int = 0
    samples_per_pixel_per_fb: int = 100
    no_fb: int = 10
    threads_x: int = 8  # kept for interface parity; the gfx950 kernel sizes its own launch
    threads_y: int = 8
    max_depth: int = 50
    rays_per_pixel: int = 0
    num_pixels: int = 0

    def calc_height(self) -> None:
        # static_cast<int>(image_width / aspect_ratio) with a double aspect (H18)
        self.image_height = int(self.image_width / float(np.float32(self.aspect_ratio)))

    def calc_rays_per_pixel(self) -> None:
        self.rays_per_pixel = self.samples_per_pixel_per_fb * self.no_fb

    def calc_num_pixels(self) -> None:
        self.num_pixels = self.image_width * self.image_height

    def calc_all(self) -> None:
        self.calc_height()
        self.calc_rays_per_pixel()
        self.calc_num_pixels()


# ---------------------------------------------------------------- scenes (scenes.h)
class Scene:
    """A flattened host scene built by the C++ scene library (rt_scene_build)."""

    def __init__(self, handle: c_void_p, name: str):
        self._h = handle
        self.name = name
        self.soa = lib().rt_scene_view(self._h).contents

    @classmethod
    def builtin(cls, name: str, images=None, meshes=None) -> "Scene":
        """Build a reference scene.  images: HxWxC uint8 arrays (decoded textures, stbi_load layout);
        meshes: raytracing_gpu_amd.assets.Mesh objects (24 floats per triangle).  Scenes that read
        files in the reference ("earth", "door", "cup", "final") need them; see assets.py."""
        h = c_void_p()
        if images is None and meshes is None:
            rc = lib().rt_scene_build(name.encode(), ctypes.byref(h))
        else:
            from .assets import pack_assets

            keep, ptr = pack_assets(images or [], meshes or [])
            rc = lib().rt_scene_build_ex(name.encode(), ptr, ctypes.byref(h))
            del keep
        if rc != 0:
            raise RtError(f"rt_scene_build({name!r}) failed with status {rc}")
        return cls(h, name)

    @property
    def aspect(self) -> float:
        return float(self.soa.aspect)

    @property
    def background(self) -> tuple:
        return tuple(self.soa.background)

    def prims(self) -> np.ndarray:
        """(n, 12) float32 view of the primitive records (type/material as raw int bits)."""
        n = self.soa.n_prims
        buf = ctypes.cast(self.soa.prims, POINTER(c_float * (12 * n))).contents
        return np.frombuffer(buf, dtype=np.float32).reshape(n, 12).copy()

    def close(self) -> None:
        if self._h:
            lib().rt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def scene(name: str) -> Scene:
    return Scene.builtin(name)


# ---------------------------------------------------------------- context (C ABI wrapper)
def make_args(width: int, height: int, spp: int, fb_first: int = 0, fb_count: int = 1, max_depth: int = 50,
              cam_mode: int = RT_CAM_REF_SLOT0, band_rows: int = 0, band_first: int = 0, band_stride: int = 1,
              stats: bool = False, seed: int = 1984, exact: bool = False, audit: bool = False,
              lds: bool = True, widest: bool = False, step: bool = True, schedule: bool = True,
              bins: bool = True, split: bool = True, fresh: bool = False) -> rt_render_args:
    flags = (RT_FLAG_EXACT_TRAVERSAL if exact else 0) | (RT_FLAG_AUDIT if audit else 0) | (0 if lds else RT_FLAG_NO_LDS)
    flags |= RT_FLAG_WIDEST if widest else 0
    flags |= 0 if step else RT_FLAG_NO_STEP
    flags |= 0 if schedule else RT_FLAG_NO_SCHEDULE
    flags |= 0 if bins else RT_FLAG_NO_CAMERA_BINS
    flags |= 0 if split else RT_FLAG_NO_SPLIT
    flags |= RT_FLAG_FRESH if fresh else 0
    return rt_render_args(width, height, spp, fb_first, fb_count, max_depth, cam_mode,
                          band_rows if band_rows > 0 else height, band_first, band_stride,
                          1 if stats else 0, flags, seed)


def owned_rows(args: rt_render_args) -> np.ndarray:
    n = lib().rt_owned_rows(ctypes.byref(args), None)
    rows = (c_int32 * max(n, 1))()
    lib().rt_owned_rows(ctypes.byref(args), rows)
    return np.frombuffer(rows, dtype=np.int32)[:n].copy()


class Context:
    """One HIP device: owns the device copy of a scene, the RNG states and a stream."""

    def __init__(self, device: int = 0):
        L = lib()
        self._c = c_void_p()
        rc = L.rt_ctx_create(device, ctypes.byref(self._c))
        if rc != 0:
            raise RtError(f"rt_ctx_create(device={device}) failed with status {rc}")
        self.device = device
        if DEFAULT_OPTIONS:
            self.set_options(**DEFAULT_OPTIONS)

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            msg = lib().rt_last_error(self._c)
            raise RtError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def options(self) -> dict:
        o = rt_ctx_options()
        self._check(lib().rt_ctx_get_options(self._c, ctypes.byref(o)), "rt_ctx_get_options")
        return o.as_dict()

    def set_options(self, reset: bool = False, **kw) -> dict:
        """Change context options (include/rt_hip.h rt_ctx_options); reset=True starts from the
        library defaults.  Upload-time options apply from the next upload.  Returns the options before."""
        before = self.options()
        o = rt_ctx_options()
        if reset:
            lib().rt_ctx_options_default(ctypes.byref(o))
        else:
            self._check(lib().rt_ctx_get_options(self._c, ctypes.byref(o)), "rt_ctx_get_options")
        for k, v in kw.items():
            if k not in before:
                raise KeyError(f"unknown context option {k!r}")
            setattr(o, k, v)
        self._check(lib().rt_ctx_set_options(self._c, ctypes.byref(o)), "rt_ctx_set_options")
        return before

    def upload(self, scene: Scene) -> None:
        self._check(lib().rt_scene_upload(self._c, ctypes.byref(scene.soa)), "rt_scene_upload")

    def render_init(self, width: int, height: int, seed: int = 1984) -> None:
        self._check(lib().rt_render_init(self._c, width, height, seed), "rt_render_init")

    def read_states(self, first: int, count: int) -> np.ndarray:
        out = np.zeros((count, 6), np.uint32)
        self._check(lib().rt_read_states(self._c, first, count, out.ctypes.data), "rt_read_states")
        return out

    def _after_torch(self) -> None:
        """The C ABI runs on the context's own HIP stream and expects device buffers that are ready:
        wait for work torch has queued on its current stream (e.g. the fill of a torch.zeros output)."""
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            torch.cuda.current_stream(self.device).synchronize()

    def render(self, args: rt_render_args, fb_dev_ptr: int) -> dict:
        self._after_torch()
        cnt = rt_counters()
        self._check(lib().rt_render(self._c, ctypes.byref(args), c_void_p(fb_dev_ptr), ctypes.byref(cnt)),
                    "rt_render")
        return cnt.as_dict()

    def resolve(self, args: rt_render_args, fb_dev_ptr: int, out_dev_ptr: int) -> None:
        self._after_torch()
        self._check(lib().rt_resolve(self._c, ctypes.byref(args), c_void_p(fb_dev_ptr), c_void_p(out_dev_ptr)),
                    "rt_resolve")

    def last_render_ms(self) -> float:
        """Device time of the last render call (a first launch's probe and schedule included)."""
        return float(lib().rt_last_render_ms(self._c))

    def last_kernel_ms(self) -> float:
        """Device time of the last render call's render kernel alone (rocprof's duration of it)."""
        return float(lib().rt_last_kernel_ms(self._c))

    def last_render_kernel(self) -> str:
        """rocprof name stem of the kernel the last render launched."""
        return lib().rt_last_render_kernel(self._c).decode()

    def last_render_schedule(self) -> int:
        """RT_SCHED_* bits of the last render launch (0: cold, nothing reused from an earlier launch)."""
        return int(lib().rt_last_render_schedule(self._c))

    def audit_log(self, cap: int = 4096) -> tuple[int, np.ndarray]:
        """(number of disagreements, [min(n, cap), 16] float32 entries) of the last audit render."""
        buf = np.zeros((cap, 16), np.float32)
        n = lib().rt_audit_log(self._c, buf.ctypes.data_as(POINTER(c_float)), cap)
        if n < 0:
            raise RtError("rt_audit_log failed")
        return n, buf[: min(n, cap)].copy()

    def draw_args(self, args: rt_render_args) -> tuple[np.ndarray, dict]:
        img = np.zeros((args.height, args.width, 3), dtype=np.uint8)
        cnt = rt_counters()
        self._check(lib().rt_draw(self._c, ctypes.byref(args), img.ctypes.data_as(POINTER(c_uint8)),
                                  ctypes.byref(cnt)), "rt_draw")
        return img, cnt.as_dict()

    def close(self) -> None:
        if getattr(self, "_c", None):
            lib().rt_ctx_destroy(self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def draw(curr_scene: Scene, settings: render_settings, ctx: Context | None = None,
         cam_mode: int = RT_CAM_REF_SLOT0, seed: int = 1984) -> tuple[np.ndarray, dict]:
    """draw() of render.h:118-174: returns (PNG-order HxWx3 uint8 image, counters)."""
    if settings.image_height <= 0:
        settings.aspect_ratio = curr_scene.aspect
        settings.calc_all()
    own = ctx is None
    ctx = ctx or Context(0)
    try:
        ctx.upload(curr_scene)
        args = make_args(settings.image_width, settings.image_height, settings.samples_per_pixel_per_fb,
                         0, settings.no_fb, settings.max_depth, cam_mode, seed=seed)
        return ctx.draw_args(args)
    finally:
        if own:
            ctx.close()


def write_png(path: str, img: np.ndarray) -> None:
    from PIL import Image

    Image.fromarray(np.ascontiguousarray(img, dtype=np.uint8), "RGB").save(path)
