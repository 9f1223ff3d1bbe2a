"""Image-tile sharding used by the multi-GPU path.

Tiles are 8x8 pixels (one wave of the render kernel), numbered scanline over the tile grid;
tile t belongs to shard t % shard_count.  This module mirrors the kernel's assignment
(csrc/hip/pt_render.hip, render_tiles) so host code can reason about which pixels a shard
writes -- e.g. to check that shards partition the image, or to pick a CPU-baseline subset.
Every pixel's result depends only on its own RNG subsequence (Morton index), so a sharded
render summed over shards is bit-identical to the 1-shard render (x + 0 = x).
"""
from __future__ import annotations

import numpy as np

TILE = 8


def tiles_shape(width: int, height: int):
    return (width + TILE - 1) // TILE, (height + TILE - 1) // TILE


def shard_tiles(width: int, height: int, shard_index: int, shard_count: int) -> np.ndarray:
    tx, ty = tiles_shape(width, height)
    return np.arange(shard_index, tx * ty, shard_count, dtype=np.int64)


def tile_pixels(width: int, height: int, tiles: np.ndarray) -> np.ndarray:
    """Scanline pixel ids (y*W + x) of the given tiles, clipped to the image."""
    tx, _ = tiles_shape(width, height)
    lane = np.arange(64)
    mx = (lane & 1) | ((lane >> 1) & 2) | ((lane >> 2) & 4)
    my = ((lane >> 1) & 1) | ((lane >> 2) & 2) | ((lane >> 3) & 4)
    x = (tiles[:, None] % tx) * TILE + mx[None, :]
    y = (tiles[:, None] // tx) * TILE + my[None, :]
    ok = (x < width) & (y < height)
    return (y * width + x)[ok].astype(np.uint32)


def shard_pixels(width: int, height: int, shard_index: int, shard_count: int) -> np.ndarray:
    return tile_pixels(width, height, shard_tiles(width, height, shard_index, shard_count))
