"""Sharding of the film across GPUs (one process per GPU) and reassembly of the all-gathered bands.

Default (yafaray_amd_setRowBandShard): rank r renders the contiguous pixel rows
[H r / N, H (r + 1) / N) plus the halo row(s) above (and below) whose splats reach into them.  The
Cornell box's per-row cost varies by under +-7 %, so equal bands balance the GPUs; only one halo row
per rank is rendered twice.  Alternative (yafaray_amd_setTileRowShard), described below:

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


def band_range(height: int, rank: int, world: int):
    """Pixel rows [y0, y1) of `rank` under the contiguous row-band split (render.cc shard_mode 1)."""
    return height * rank // world, height * (rank + 1) // world


def band_rows_max(height: int, world: int) -> int:
    return max(band_range(height, r, world)[1] - band_range(height, r, world)[0] for r in range(world))


def pack_row_band(image, rank: int, world: int, xp=np):
    """The rows of `rank`'s band from a (H, W, C) image, zero-padded to band_rows_max rows."""
    H = image.shape[0]
    y0, y1 = band_range(H, rank, world)
    out = xp.zeros((band_rows_max(H, world),) + tuple(image.shape[1:]), dtype=image.dtype)
    out[:y1 - y0] = image[y0:y1]
    return out


def assemble_row_bands(gathered, height: int, world: int, xp=np):
    """(world * band_rows_max, W, C) all-gather result -> (H, W, C) image."""
    br = band_rows_max(height, world)
    out = xp.zeros((height,) + tuple(gathered.shape[1:]), dtype=gathered.dtype)
    for rank in range(world):
        y0, y1 = band_range(height, rank, world)
        out[y0:y1] = gathered[rank * br:rank * br + (y1 - y0)]
    return out


def rebalance_bands(bounds, times, cap_rows=None, damping=0.5):
    """Host-side load balancing of the row bands (bench.py, between frames).  `bounds` = world + 1
    band boundaries, `times` = each rank's last render time.  Each band's time is spread evenly over
    its rows (a piecewise-constant cost density), the boundaries move towards equal cost (damped),
    every band keeps >= 1 row and <= cap_rows rows.  Pure and deterministic: every rank computes the
    same result from the same all-gathered times."""
    world = len(bounds) - 1
    H = int(bounds[-1])
    if world <= 1 or H < world:
        return list(bounds)
    dens = np.zeros(H)
    for r in range(world):
        rows = bounds[r + 1] - bounds[r]
        if rows > 0:
            dens[bounds[r]:bounds[r + 1]] = max(float(times[r]), 1e-9) / rows
    cum = np.concatenate([[0.0], np.cumsum(dens)])
    new = [0]
    for r in range(1, world):
        target = cum[-1] * r / world
        y = int(np.searchsorted(cum, target))
        # interpolate inside the row for the closer boundary
        if 0 < y <= H and (cum[y] - target) > (target - cum[y - 1]):
            y -= 1
        y = int(round(damping * bounds[r] + (1.0 - damping) * y))
        new.append(y)
    new.append(H)
    for r in range(1, world):
        new[r] = min(max(new[r], new[r - 1] + 1), H - (world - r))
    if cap_rows is not None and max(new[r + 1] - new[r] for r in range(world)) > cap_rows:
        return list(bounds)
    return new
