"""Image-tile partitioning for multi-GPU rendering.

Tiles of `tile` x `tile` pixels in row-major order; tile (tx, ty) belongs to rank
(tx + ty) mod P: diagonals dealt round-robin, so every rank's tiles are spread
over the whole image (light-path cost varies strongly over it; plain row-major
round-robin gives each rank full-height column stripes when the tile row length
is a multiple of P -- 5% imbalance at P = 2 on the Cornell box, tools/scale_probe.py).
Every rank renders the same number of tiles (short ranks repeat their first tile;
the copy is dropped at assembly) so the per-rank buffers are equal-sized for one
all-gather.  The RNG is keyed on the global pixel, so the assembled image is
bit-identical for any P.
"""
from __future__ import annotations

import numpy as np


def tile_origins(width: int, height: int, tile: int) -> np.ndarray:
    ys, xs = np.meshgrid(np.arange(0, height, tile), np.arange(0, width, tile), indexing="ij")
    return np.stack([xs.ravel(), ys.ravel()], axis=1).astype(np.int32)


def tile_owners(width: int, height: int, tile: int, world: int) -> np.ndarray:
    """Rank of every tile of tile_origins(...) (row-major): (tx + ty) mod world."""
    ntx = (width + tile - 1) // tile
    nty = (height + tile - 1) // tile
    ty, tx = np.meshgrid(np.arange(nty), np.arange(ntx), indexing="ij")
    return ((tx + ty) % world).ravel().astype(np.int64)


def rank_tile_indices(width: int, height: int, tile: int, rank: int, world: int) -> np.ndarray:
    """Row-major indices (into tile_origins) of the real tiles of `rank`, ascending."""
    return np.nonzero(tile_owners(width, height, tile, world) == rank)[0]


def tiles_per_rank(width: int, height: int, tile: int, world: int) -> int:
    """Tile slots per rank: the largest rank's real tile count."""
    return int(np.bincount(tile_owners(width, height, tile, world), minlength=world).max())


def rank_tiles(width: int, height: int, tile: int, rank: int, world: int) -> np.ndarray:
    """Origins of the tiles rank `rank` renders, padded to tiles_per_rank."""
    allt = tile_origins(width, height, tile)
    mine = allt[rank_tile_indices(width, height, tile, rank, world)]
    k = tiles_per_rank(width, height, tile, world)
    if len(mine) == 0:
        mine = allt[:1]
    if len(mine) < k:
        mine = np.concatenate([mine, np.repeat(mine[:1], k - len(mine), axis=0)], axis=0)
    return np.ascontiguousarray(mine, np.int32)


def rank_tile_count(width: int, height: int, tile: int, rank: int, world: int) -> int:
    """Number of real (non-padding) tiles among rank_tiles(...): padding repeats a tile,
    which is harmless for a pure render but must not be rendered twice by a learning
    renderer (Expected SARSA would count its TD targets twice)."""
    return len(rank_tile_indices(width, height, tile, rank, world))


def assemble(gathered: np.ndarray, width: int, height: int, tile: int, world: int) -> np.ndarray:
    """gathered: (world, k, tile, tile, 3) per-rank tile buffers -> (height, width, 3)."""
    allt = tile_origins(width, height, tile)
    owners = tile_owners(width, height, tile, world)
    slot = np.zeros(world, np.int64)
    img = np.zeros((height, width, 3), np.float32)
    for idx, (x, y) in enumerate(allt):
        r = owners[idx]
        j = slot[r]
        slot[r] += 1
        h = min(tile, height - y)
        w = min(tile, width - x)
        img[y:y + h, x:x + w] = gathered[r, j, :h, :w]
    return img
