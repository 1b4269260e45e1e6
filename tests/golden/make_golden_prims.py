"""Record golden input/output vectors of the reference's own numeric building blocks.

Run here (needs oracle/_ref/libyafref_prims.so, built from /root/reference by oracle/Makefile):
    python tests/golden/make_golden_prims.py
Writes tests/golden/prims.npz: for every primitive an input array and the reference's output,
computed by the reference code itself (include/sampler/sample.h, src/sampler/halton.cc,
include/math/math.h FAST_MATH/FAST_TRIG, include/math/random.h, include/geometry/vector.h,
include/geometry/bound.h, include/math/filter.h, include/color/color.h).
The CPU oracle and the device numerics are pinned against this file (tests/test_oracle_golden.py).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "prims.npz")


def main():
    r = O.ref_prims()
    if r is None:
        sys.exit("oracle/_ref not built (needs /root/reference): the committed prims.npz is used as is")
    rng = np.random.default_rng(20240515)
    n = 4096
    g = {}
    bits = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    bits[:64] = np.arange(64)
    rr = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    rr[:128] = 0
    g["ri_bits"], g["ri_r"] = bits, rr
    for w in ("riVdC", "riS", "riLp"):
        g[w] = r.ri(w, bits, rr)
    g["fnv_in"] = bits
    g["fnv"] = r.fnv32(bits)
    dims = np.repeat(np.arange(1, 50, dtype=np.int32), 96)
    idx = rng.integers(0, 2**32, len(dims), dtype=np.uint64).astype(np.uint32)
    idx[::3] = rng.integers(0, 100000, len(idx[::3]))
    g["lds_dim"], g["lds_idx"] = dims, idx
    g["lds"] = r.lds(dims, idx)
    hal = []
    starts = [0, 1, 2, 7, 12345, 2**31 + 5, 2**32 - 1, 4294967295 - 4567, 987654]
    for base in (2, 3, 5):
        for st in starts:
            hal.append(r.halton_seq(base, st, 16))
    g["halton_bases"] = np.array([b for b in (2, 3, 5) for _ in starts], np.int32)
    g["halton_starts"] = np.array(starts * 3, np.uint32)
    g["halton_seq"] = np.stack(hal)
    x = np.concatenate([rng.uniform(-40, 40, n), rng.uniform(-7, 7, n), np.linspace(-2 * np.pi, 2 * np.pi, 257)]).astype(np.float32)
    g["trig_x"] = x
    g["sin"] = r.unary("sin", x)
    g["cos"] = r.unary("cos", x)
    ex = rng.uniform(-20, 5, n).astype(np.float32)
    g["exp_x"], g["exp"] = ex, r.unary("exp", ex)
    nv = rng.normal(size=(n, 3)).astype(np.float32)
    nv /= np.linalg.norm(nv, axis=1, keepdims=True)
    nv = nv.astype(np.float32)
    nv[:4] = [[0, 0, 1], [0, 0, -1], [1, 0, 0], [0, 1, 0]]
    cs = r.unary("coords_system", nv.reshape(-1), width_out=6, width_in=3)
    g["coords_in"], g["coords"] = nv, cs.reshape(n, 6)
    s = rng.random((n, 2)).astype(np.float32)
    s[:8, 0] = 1.0
    nrv = np.concatenate([nv, cs.reshape(n, 6)], 1)
    g["hemi_nrv"], g["hemi_s"], g["hemi"] = nrv, s, r.cos_hemisphere(nrv, s)
    v = (rng.normal(size=(n, 3)) * rng.uniform(1e-3, 1e3, (n, 1))).astype(np.float32)
    g["norm_in"], g["norm"] = v, r.unary("normalize", v.reshape(-1), 3, 3).reshape(n, 3)
    lo = rng.uniform(-2, 0, (n, 3))
    box = np.concatenate([lo, lo + rng.uniform(0, 3, (n, 3))], 1).astype(np.float32)
    ray = np.concatenate([rng.uniform(-4, 4, (n, 3)), rng.normal(size=(n, 3)), rng.uniform(0, 10, (n, 1))], 1).astype(np.float32)
    ray[:64, 3] = 0
    ray[64:128, 4] = 0
    g["bound_box"], g["bound_ray"], g["bound"] = box, ray, r.bound_cross(box, ray)
    seeds = np.array([0, 1, 123, 2**31, 4000000000, 30903], np.uint32)
    g["mwc_seeds"] = seeds
    g["mwc"] = np.stack([r.mwc(int(sd), 256) for sd in seeds])
    d = rng.uniform(-1.5, 1.5, (n, 2)).astype(np.float32)
    g["gauss_in"], g["gauss"] = d, r.unary("filter_gauss", d.reshape(-1), 1, 2)
    dv = np.concatenate([rng.uniform(-5, 5, n), np.arange(-20, 20) * 0.5, np.arange(-20, 20) * 0.5 + 1e-12,
                         np.arange(-20, 20) * 0.5 - 1e-12]).astype(np.float64)
    g["int_in"] = dv
    g["round_to_int"] = r.int_of_double("round_to_int", dv)
    g["floor_to_int"] = r.int_of_double("floor_to_int", dv)
    c = rng.uniform(0, 5, (n, 3)).astype(np.float32)
    g["clamp_in"], g["clamp_1_5"], g["clamp_0"] = c, r.clamp_proportional(c, 1.5), r.clamp_proportional(c, 0.0)
    np.savez_compressed(OUT, **g)
    print("wrote", OUT, os.path.getsize(OUT), "bytes,", len(g), "arrays")
    # round 2: src/geometry/vector.cc, src/color/color.cc, src/render/imagesplitter.cc
    g2 = {}
    r12 = rng.random((n, 2)).astype(np.float32)
    r12[:9] = [[0.5, 0.5], [0, 0], [1, 1], [0, 1], [1, 0], [0.5, 0], [0, 0.5], [0.25, 0.75], [0.75, 0.25]]
    g2["shirley_in"], g2["shirley"] = r12, r.shirley(r12)
    rgbe = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    rgbe[:16, 3] = 0
    rgbe[16:32, 3] = [1, 2, 100, 127, 128, 129, 130, 135, 136, 137, 150, 200, 250, 254, 255, 255]
    g2["rgbe_in"], g2["rgbe"] = rgbe, r.rgbe(rgbe)
    sizes = [(1920, 1080, 32), (64, 48, 16), (50, 38, 8), (33, 7, 4), (256, 256, 64), (100, 1, 32)]
    g2["tiles_sizes"] = np.array(sizes, np.int32)
    for k, (w, h, bs) in enumerate(sizes):
        g2[f"tiles_linear_{k}"] = r.tiles(w, h, bs, "linear")
        g2[f"tiles_centre_{k}"] = r.tiles(w, h, bs, "centre")      # ties broken by std::random_device
        g2[f"tiles_linear_t8_{k}"] = r.tiles(w, h, bs, "linear", nthreads=8)
    OUT2 = os.path.join(os.path.dirname(OUT), "prims_r02.npz")
    np.savez_compressed(OUT2, **g2)
    print("wrote", OUT2, os.path.getsize(OUT2), "bytes,", len(g2), "arrays")


if __name__ == "__main__":
    main()
