"""Multi-GPU tiling of the frame buffer (one process per GPU, torch.distributed over RCCL).

Rows are dealt in bands of `band_rows` round-robin over ranks (cheap sky rows and costly ground
rows interleave, so ranks stay balanced).  Every rank renders its rows for every fb and resolves
them to 8-bit (the per-fb quantise + square-average of color.h:19-170 is per pixel, hence
rank-local); one all-gather of the 8-bit rows (padded to the largest rank) assembles the image.
"""
from __future__ import annotations

import numpy as np


def band_rows(height: int, band: int, rank: int, world: int) -> np.ndarray:
    """Rows owned by `rank` (ascending; j = 0 is the bottom row) — same rule as rt_owned_rows."""
    rows = []
    b = rank
    while b * band < height:
        rows.extend(range(b * band, min((b + 1) * band, height)))
        b += world
    return np.array(rows, dtype=np.int32)


def plan(height: int, band: int, world: int) -> list:
    return [band_rows(height, band, r, world) for r in range(world)]


def pad_rows(img_rows: np.ndarray, max_rows: int) -> np.ndarray:
    out = np.zeros((max_rows,) + img_rows.shape[1:], img_rows.dtype)
    out[: len(img_rows)] = img_rows
    return out


def assemble(gathered: np.ndarray, rows_per_rank: list, height: int) -> np.ndarray:
    """gathered: [world][max_rows][W][3] uint8 in owned-row order -> PNG-order image [H][W][3]."""
    world, _, W, _ = gathered.shape
    pic = np.zeros((height, W, 3), np.uint8)
    for r in range(world):
        rows = rows_per_rank[r]
        pic[height - 1 - rows] = gathered[r, : len(rows)]
    return pic
