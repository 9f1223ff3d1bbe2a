"""Image-tile sharding used by the multi-GPU path.

Tiles are tile_w x tile_h pixels (default 8x8, multiples of 8: pt_params.tile_w/tile_h), numbered
scanline over the tile grid; tile t belongs to shard t % shard_count.  Inside a tile the pixels come
in 8x8 blocks (row-major over the tile), Morton order within a block -- 64 consecutive work slots,
one wave.  This module mirrors the kernels' assignment (csrc/hip/pt_render.hip, unit_pixel) so
host code can reason about which pixels a shard writes -- e.g. to check that shards partition the
image, or to pick a CPU-baseline subset.  Every pixel's result depends only on its own RNG
subsequence (Morton index), so a sharded render summed over shards is bit-identical to the 1-shard
render (x + 0 = x).
"""
from __future__ import annotations

import numpy as np

TILE = 8


def _dims(tile_w, tile_h):
    tw = TILE if not tile_w else int(tile_w)
    th = TILE if not tile_h else int(tile_h)
    if tw % 8 or th % 8 or not (8 <= tw <= 256) or not (8 <= th <= 256):
        raise ValueError("tile size %dx%d: multiples of 8 up to 256" % (tw, th))
    return tw, th


def tiles_shape(width: int, height: int, tile_w: int = 0, tile_h: int = 0):
    tw, th = _dims(tile_w, tile_h)
    return (width + tw - 1) // tw, (height + th - 1) // th


def shard_tiles(width: int, height: int, shard_index: int, shard_count: int, tile_w: int = 0, tile_h: int = 0):
    tx, ty = tiles_shape(width, height, tile_w, tile_h)
    return np.arange(shard_index, tx * ty, shard_count, dtype=np.int64)


def tile_pixels(width: int, height: int, tiles: np.ndarray, tile_w: int = 0, tile_h: int = 0) -> np.ndarray:
    """Scanline pixel ids (y*W + x) of the given tiles in work-slot order, clipped to the image."""
    tw, th = _dims(tile_w, tile_h)
    tx, _ = tiles_shape(width, height, tw, th)
    lane = np.arange(64)
    mx = (lane & 1) | ((lane >> 1) & 2) | ((lane >> 2) & 4)
    my = ((lane >> 1) & 1) | ((lane >> 2) & 2) | ((lane >> 3) & 4)
    bx = tw // 8
    blk = np.arange((tw // 8) * (th // 8))
    ox = (blk % bx) * 8
    oy = (blk // bx) * 8
    tiles = np.asarray(tiles, dtype=np.int64)
    x = (tiles[:, None, None] % tx) * tw + ox[None, :, None] + mx[None, None, :]
    y = (tiles[:, None, None] // tx) * th + oy[None, :, None] + my[None, None, :]
    x, y = x.reshape(len(tiles), len(blk) * 64), y.reshape(len(tiles), len(blk) * 64)
    ok = (x < width) & (y < height)
    return (y * width + x)[ok].astype(np.uint32)


def shard_pixels(width: int, height: int, shard_index: int, shard_count: int, tile_w: int = 0,
                 tile_h: int = 0) -> np.ndarray:
    return tile_pixels(width, height, shard_tiles(width, height, shard_index, shard_count, tile_w, tile_h),
                       tile_w, tile_h)


def morton_index(x, y):
    """camera.h:66-75 mortonPxltoI, vectorised (the reference's imgBuff index of pixel (x, y))."""
    x = np.asarray(x, dtype=np.uint64)
    y = np.asarray(y, dtype=np.uint64)
    r = np.zeros(np.broadcast(x, y).shape, dtype=np.uint64)
    for b in range(16):
        r |= ((x >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b)
        r |= ((y >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b + 1)
    return r


def to_scanline(buf: np.ndarray, width: int, height: int) -> np.ndarray:
    """A Morton-ordered (reference imgBuff) W*H*3 buffer as a scanline (H, W, 3) image."""
    yy, xx = np.mgrid[0:height, 0:width]
    idx = morton_index(xx, yy).astype(np.int64)
    return np.asarray(buf).reshape(-1, 3)[idx.reshape(-1)].reshape(height, width, 3)


def shard_pixels_lib(width: int, height: int, shard_index: int, shard_count: int, tile_w: int = 0,
                     tile_h: int = 0) -> np.ndarray:
    """The same list from libptamd (pt_shard_pixels: the kernels' own mapping function, run on the host)."""
    import ctypes as C
    from . import _lib as L
    n = C.c_uint32(0)
    L.check(L.lib().pt_shard_pixels(width, height, shard_index, shard_count, tile_w, tile_h, None, 0, C.byref(n)))
    out = np.zeros(max(1, n.value), dtype=np.uint32)
    L.check(L.lib().pt_shard_pixels(width, height, shard_index, shard_count, tile_w, tile_h, out.ctypes.data,
                                    len(out), C.byref(n)))
    return out[:n.value]
