"""Test infrastructure (never imported by the product): paired statistics of a GPU image against the
oracle's image of the same frame, for integrator paths whose random draws differ by construction
(Russian roulette: the reference seeds one generator per tile from rand(), integrator_tiled.cc:272;
the GPU one per sample — DESIGN.md §3).

Both images share every Halton / Faure draw, so their per-pixel difference isolates the RR noise.
The difference image (mean over RGB) is cut into 8x8 blocks; the block means are independent, so
  * block z   = block mean / (block sd / 8)                        (local bias, e.g. one surface)
  * global z  = mean of the block means / (their sd / sqrt(blocks)) (a frame-wide bias)
An unbiased GPU path gives |global z| < 4 with probability > 0.9999.
"""
import numpy as np


def paired_z(gpu, ref, block=8):
    g = np.asarray(gpu, np.float64)[..., :3]
    o = np.asarray(ref, np.float64)[..., :3]
    d = (g - o).mean(-1)
    hb, wb = d.shape[0] // block, d.shape[1] // block
    blocks = d[:hb * block, :wb * block].reshape(hb, block, wb, block).transpose(0, 2, 1, 3).reshape(hb * wb, block * block)
    m = blocks.mean(1)
    sd = blocks.std(1, ddof=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        z = np.where(sd > 0, m / (sd / block), 0.0)
    se = m.std(ddof=1) / np.sqrt(len(m)) if len(m) > 1 else 0.0
    mean_z = float(m.mean() / se) if se > 0 else 0.0
    return {"blocks": int(len(m)), "max_abs_block_z": float(np.abs(z).max()), "frac_abs_block_z_gt_4": float((np.abs(z) > 4).mean()),
            "mean_diff": float(m.mean()), "mean_diff_se": float(se), "mean_z": mean_z,
            "mean_rel_diff": float((g.mean() - o.mean()) / max(1e-12, o.mean()))}
