"""Tile-row sharding of the film across GPUs (one process per GPU) and reassembly of the
all-gathered bands.

The reference splits the film into 32x32 tiles in linear order (src/render/imagesplitter.cc:30-49)
and hands them to CPU threads from an atomic counter (imagefilm.cc:447-487).  Across GPUs the unit
is a whole tile row: rank r renders tile rows r, r + N, r + 2N, ... (round-robin, which balances
the Cornell box's cheap open-front rows against its expensive interior), plus the one-pixel halo
row above each of its tile rows so that the forward splat footprint is complete and
every owned pixel is bit-identical to a single-GPU render.  The finished rows travel in one RCCL
all-gather per frame.
"""
from __future__ import annotations

import numpy as np


def tile_rows(height: int, tile: int) -> int:
    return (height + tile - 1) // tile


def owned_tile_rows(height: int, tile: int, rank: int, world: int):
    return [r for r in range(tile_rows(height, tile)) if r % world == rank]


def band_rows(height: int, tile: int, world: int) -> int:
    """Pixel rows of the (padded) band every rank contributes to the all-gather."""
    return ((tile_rows(height, tile) + world - 1) // world) * tile


def pack_band(image, height: int, tile: int, rank: int, world: int, xp=np):
    """Rows owned by `rank` from a (H, W, C) image, packed into a (band_rows, W, C) band."""
    out = xp.zeros((band_rows(height, tile, world),) + tuple(image.shape[1:]), dtype=image.dtype)
    for k, r in enumerate(owned_tile_rows(height, tile, rank, world)):
        y0, y1 = r * tile, min(height, r * tile + tile)
        out[k * tile:k * tile + (y1 - y0)] = image[y0:y1]
    return out


def assemble(gathered, height: int, tile: int, world: int, xp=np):
    """(world * band_rows, W, C) all-gather result -> (H, W, C) image."""
    br = band_rows(height, tile, world)
    out = xp.zeros((height,) + tuple(gathered.shape[1:]), dtype=gathered.dtype)
    for rank in range(world):
        band = gathered[rank * br:(rank + 1) * br]
        for k, r in enumerate(owned_tile_rows(height, tile, rank, world)):
            y0, y1 = r * tile, min(height, r * tile + tile)
            out[y0:y1] = band[k * tile:k * tile + (y1 - y0)]
    return out
