"""Pixel pins: the reference's own renders (/root/reference/images/*.png) as small fixtures.

The reference holds no tests and no golden data for its render path; the only pixel-level
evidence it carries are the PNGs its author rendered with it (images/, 1200 px wide).  This
script turns them into 150-wide block means (8x8 pixel boxes of the 8-bit PNG values, rows
cropped from the top to a multiple of 8) so that tests/test_image_pin.py can compare oracle
renders (CPU) and librt_hip.so renders (GPU) with them statistically (correlation + PSNR).

Which image is which scene (scenes.h structs; found by rendering every scene with the oracle and
correlating):

- 674-row images come from the current code (H18: int(1200 / (double)(16.0f/9.0f)) = 674):
  image10.75 earth, image13 triangle, image14 triangles, image15/16 door.
  They match as rendered.
- 675-row images come from an older revision of the code (a different height formula) whose
  frames are mirrored left-right against the current camera: image5.75 basic (symmetric, so
  the mirror is moot), image6.5 first, image7 big_scene1,
  image8 two_spheres, image9 two_perlin.  They match mirrored (the same sphere placements,
  colours and materials; unmirrored correlation is 0.46 for image7 against 0.995 mirrored).
- 1200x1200: image11 cornell_box, image12 cornell_smoke_box.

The fixture also carries 1/16-size box-downsampled copies of the two textures the matching
scenes read (textures/earthmap.jpg, assets/door/Door_C.jpg, decoded with the stb_image-exact
rt_image_decode), so the tests run where /root/reference is absent (the GPU box).  At 150-wide
block resolution the downsampled texture moves correlation by < 1e-3 (measured at 1/1 .. 1/32).

Run from the repo root (needs /root/reference and the built librt_hip.so):
    python tests/golden/make_image_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

REF = "/root/reference"
BLOCK = 8  # 1200 -> 150 wide

# image -> (scene, mirrored, note)
PINS = {
    "image5.75": ("basic", True, "basic_scene, older code (675 rows, mirrored frame; the scene is left-right symmetric)"),
    "image6.5": ("first", True, "first_scene, older code (675 rows, mirrored frame)"),
    "image7": ("big1", True, "big_scene1 (C2), older code (675 rows, mirrored frame)"),
    "image8": ("two_spheres", True, "two_spheres_scene, older code (675 rows, mirrored frame)"),
    "image9": ("two_perlin", True, "two_perlin_spheres_scene, older code (675 rows, mirrored frame)"),
    "image10.75": ("earth", False, "earth_scene, current code (674 rows)"),
    "image11": ("cornell", False, "cornell_box_scene (1200x1200)"),
    "image12": ("cornell_smoke", False, "cornell_smoke_box_scene (C3, 1200x1200)"),
    "image13": ("triangle", False, "triangle_scene, current code (674 rows)"),
    "image14": ("triangles", False, "triangles_scene, current code (674 rows)"),
    "image15": ("door", False, "door_scene (C4 mesh), current code (674 rows), earlier spp"),
    "image16": ("door", False, "door_scene (C4 mesh), current code (674 rows)"),
}
TEXTURES = {"tex_earth": "textures/earthmap.jpg", "tex_door": "assets/door/Door_C.jpg"}
TEX_DOWN = 16


def block_means(img: np.ndarray, b: int) -> np.ndarray:
    h = (img.shape[0] // b) * b
    w = (img.shape[1] // b) * b
    a = img[:h, :w].astype(np.float64)
    return a.reshape(h // b, b, w // b, b, a.shape[2]).mean(axis=(1, 3))


def main() -> None:
    from PIL import Image

    from raytracing_gpu_amd import assets

    out, meta = {}, {"block": BLOCK, "width": 1200, "tex_down": TEX_DOWN, "images": {}}
    for name, (scene, mirror, note) in PINS.items():
        a = np.asarray(Image.open(os.path.join(REF, "images", name + ".png")).convert("RGB"), np.uint8)
        if mirror:
            a = a[:, ::-1]
        bm = block_means(a, BLOCK)
        out[name] = np.round(bm).astype(np.uint8)
        meta["images"][name] = {"scene": scene, "mirrored": mirror, "rows": int(a.shape[0]),
                                "cols": int(a.shape[1]), "note": note}
    for key, rel in TEXTURES.items():
        t = assets.load_image(os.path.join(REF, rel))
        out[key] = np.round(block_means(t, TEX_DOWN)).astype(np.uint8)
        meta[key] = {"source": rel, "decoded_shape": list(t.shape), "stored_shape": list(out[key].shape)}
    np.savez_compressed(os.path.join(HERE, "ref_images.npz"), **out)
    with open(os.path.join(HERE, "ref_images.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", ", ".join(sorted(out)))


if __name__ == "__main__":
    main()
