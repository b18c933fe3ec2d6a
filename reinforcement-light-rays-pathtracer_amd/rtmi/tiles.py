"""Image-tile partitioning for multi-GPU rendering.

Tiles of `tile` x `tile` pixels in row-major order; tile k belongs to rank
k mod P (round-robin for load balance: light-path cost varies strongly over
the image).  Every rank renders the same number of tiles (short ranks repeat
their first tile; the copy is dropped at assembly) so the per-rank buffers
are equal-sized for one all-gather.  The RNG is keyed on the global pixel,
so the assembled image is bit-identical for any P.
"""
from __future__ import annotations

import numpy as np


def tile_origins(width: int, height: int, tile: int) -> np.ndarray:
    ys, xs = np.meshgrid(np.arange(0, height, tile), np.arange(0, width, tile), indexing="ij")
    return np.stack([xs.ravel(), ys.ravel()], axis=1).astype(np.int32)


def tiles_per_rank(n_tiles: int, world: int) -> int:
    return (n_tiles + world - 1) // world


def rank_tiles(width: int, height: int, tile: int, rank: int, world: int) -> np.ndarray:
    """Origins of the tiles rank `rank` renders, padded to tiles_per_rank."""
    allt = tile_origins(width, height, tile)
    mine = allt[rank::world]
    k = tiles_per_rank(len(allt), world)
    if len(mine) == 0:
        mine = allt[:1]
    if len(mine) < k:
        mine = np.concatenate([mine, np.repeat(mine[:1], k - len(mine), axis=0)], axis=0)
    return np.ascontiguousarray(mine, np.int32)


def rank_tile_count(width: int, height: int, tile: int, rank: int, world: int) -> int:
    """Number of real (non-padding) tiles among rank_tiles(...): padding repeats a tile,
    which is harmless for a pure render but must not be rendered twice by a learning
    renderer (Expected SARSA would count its TD targets twice)."""
    return len(tile_origins(width, height, tile)[rank::world])


def assemble(gathered: np.ndarray, width: int, height: int, tile: int, world: int) -> np.ndarray:
    """gathered: (world, k, tile, tile, 3) per-rank tile buffers -> (height, width, 3)."""
    allt = tile_origins(width, height, tile)
    img = np.zeros((height, width, 3), np.float32)
    for idx, (x, y) in enumerate(allt):
        r, j = idx % world, idx // world
        h = min(tile, height - y)
        w = min(tile, width - x)
        img[y:y + h, x:x + w] = gathered[r, j, :h, :w]
    return img
