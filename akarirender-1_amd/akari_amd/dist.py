"""Multi-GPU frame partition: tile-split across ranks + one frame-end gather (RCCL over xGMI).

The reference renders on one device (core/device.cpp:154-173 only lists devices) with its
framebuffer split in tiles (kernel/integrators/cpu/integrator.cpp:92-115,
gpu/cuda/integrator.cpp:152-168).  Pixels are independent — the sampler is seeded per pixel with
x + y*W (cpu/integrator.cpp:124) — so interleaving tiles over ranks gives the same image for any
rank count, bit for bit.  The only exchange is the gather of each rank's packed film to rank 0.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

Rect = Tuple[int, int, int, int]


def tile_grid(width: int, height: int, tile: int) -> List[Rect]:
    out = []
    for y in range(0, height, tile):
        for x in range(0, width, tile):
            out.append((x, y, min(width, x + tile), min(height, y + tile)))
    return out


def tiles_for_rank(width: int, height: int, tile: int, rank: int, world: int) -> List[Rect]:
    """Interleaved assignment: tile k of the row-major tile grid -> rank k % world (load balance:
    every rank samples every region of the frame)."""
    return [t for k, t in enumerate(tile_grid(width, height, tile)) if k % world == rank]


def n_pixels(tiles: Sequence[Rect]) -> int:
    return sum((x1 - x0) * (y1 - y0) for x0, y0, x1, y1 in tiles)


def max_pixels_per_rank(width, height, tile, world) -> int:
    return max(n_pixels(tiles_for_rank(width, height, tile, r, world)) for r in range(world))


def unpack_to_frame(packed: np.ndarray, tiles: Sequence[Rect], width: int, height: int,
                    radiance: np.ndarray, weight: np.ndarray):
    """Scatter one rank's packed film ([rgb * P | w * P] with P >= its pixel count, tiles in order,
    row-major inside a tile) into full-frame buffers (Film::merge_tile, core/film.h:85-95)."""
    cap = packed.size // 4
    rgb = packed[:3 * cap].reshape(cap, 3)
    w = packed[3 * cap:]
    k = 0
    for x0, y0, x1, y1 in tiles:
        n = (x1 - x0) * (y1 - y0)
        radiance[y0:y1, x0:x1] += rgb[k:k + n].reshape(y1 - y0, x1 - x0, 3)
        weight[y0:y1, x0:x1] += w[k:k + n].reshape(y1 - y0, x1 - x0)
        k += n
    return radiance, weight


def gather_frame(film, width: int, height: int, tile: int, group=None):
    """all-gather every rank's packed film tensor (equal capacity) and assemble the full frame on
    every rank (rank 0 uses it).  `film` is a 1-D tensor laid out [rgb * cap | w * cap]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    gathered = torch.empty(world * film.numel(), dtype=film.dtype, device=film.device)
    dist.all_gather_into_tensor(gathered, film, group=group)
    parts = gathered.cpu().numpy().reshape(world, -1)
    rad = np.zeros((height, width, 3), np.float32)
    wt = np.zeros((height, width), np.float32)
    for r in range(world):
        unpack_to_frame(parts[r], tiles_for_rank(width, height, tile, r, world), width, height, rad, wt)
    return rad, wt
