"""Record golden vectors of the reference's own texturing building blocks.

Run here (needs oracle/_ref/libyafref_prims.so, built from /root/reference by oracle/Makefile):
    python tests/golden/make_golden_tex.py
Writes tests/golden/tex_prims.npz: the image buffer pixel types' storage round trip
(include/image/image_buffers.h: Rgba1010108, Rgb101010, Rgba7773, Rgb565, Gray8, Gray, GrayAlpha,
RgbAlpha), colour-space conversions and HSV adjustment (include/color/color.h), the bicubic
weights (include/math/interpolation.h) and FAST_MATH pow (include/math/math.h), each computed by
the reference code itself.  The oracle's texturing (oracle/yaftex.h) is pinned against them
(tests/test_oracle_golden.py).
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tex_prims.npz")


def inputs(seed=20261016):
    rng = np.random.default_rng(seed)
    n = 4096
    rgba = rng.random((n, 4)).astype(np.float32) * 1.25 - 0.1
    rgba[:256] = rng.integers(0, 256, (256, 4)) / np.float32(255.0)        # 8-bit texel values
    rgba[256:512] = rng.integers(0, 1024, (256, 4)) / np.float32(1023.0)   # 10-bit values
    rgb = rng.random((n, 3)).astype(np.float32) * 1.1
    rgb[:64] = rng.integers(0, 256, (64, 3)) / np.float32(255.0)
    sat_hue = np.stack([rng.random(n) * 2.0, rng.random(n) * 12.0 - 6.0], 1).astype(np.float32)
    cub = rng.random((n, 17)).astype(np.float32) * 2.0 - 0.5
    ab = np.stack([rng.random(n) * 1.5, rng.random(n) * 3.0], 1).astype(np.float32)
    return rgba, rgb, sat_hue, cub, ab


def run(lib, prefix, rgba, rgb, sat_hue, cub, ab):
    f = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    g = {}
    n = len(rgba)
    for kind in range(8):
        out = np.empty_like(rgba)
        getattr(lib, prefix + "tex_quantize")(kind, f(rgba), f(out), n)
        g[f"quant{kind}"] = out
    for d in (0, 1):
        for cs, gam in ((1, 2.2), (2, 1.0), (3, 1.0), (4, 1.0)):
            out = np.empty_like(rgb)
            getattr(lib, prefix + "color_space")(d, cs, C.c_float(gam), f(rgb), f(out), len(rgb))
            g[f"cs{d}_{cs}"] = out
    out = np.empty_like(rgb)
    getattr(lib, prefix + "hsv_adjust")(f(rgb), f(sat_hue), f(out), len(rgb))
    g["hsv"] = out
    out = np.empty((len(cub), 4), np.float32)
    getattr(lib, prefix + "cubic")(f(cub), f(out), len(cub))
    g["cubic"] = out
    out = np.empty(len(ab), np.float32)
    getattr(lib, prefix + "pow")(f(ab), f(out), len(ab))
    g["pow"] = out
    return g


def main():
    if O.ref_lib() is None:
        sys.exit("oracle/_ref not built (needs /root/reference): the committed tex_prims.npz is used as is")
    rgba, rgb, sat_hue, cub, ab = inputs()
    g = run(O.ref_lib(), "ref_", rgba, rgb, sat_hue, cub, ab)
    np.savez_compressed(OUT, rgba=rgba, rgb=rgb, sat_hue=sat_hue, cub=cub, ab=ab, **g)
    print("wrote", OUT, len(g), "arrays")


if __name__ == "__main__":
    main()
