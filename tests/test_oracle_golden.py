"""Pin the CPU oracle (oracle/yafcpu.cc) against the reference's own code:
(1) the committed golden vectors of tests/golden/prims.npz (made by make_golden_prims.py from
    oracle/_ref, i.e. the reference sources compiled here), always;
(2) the live reference building blocks on fresh random inputs, when oracle/_ref is built."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "prims.npz"))


@pytest.fixture(scope="module")
def o(oracle_built):
    return oracle_built.oracle_prims()


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.kind == "f":
        return np.array_equal(a.view(np.uint32 if a.dtype == np.float32 else np.uint64),
                              b.astype(a.dtype).view(np.uint32 if a.dtype == np.float32 else np.uint64))
    return np.array_equal(a, b)


@pytest.mark.parametrize("w", ["riVdC", "riS", "riLp"])
def test_radical_inverse(o, w):
    assert same(o.ri(w, G["ri_bits"], G["ri_r"]), G[w])


def test_fnv(o):
    assert same(o.fnv32(G["fnv_in"]), G["fnv"])


def test_low_discrepancy_faure(o):
    assert same(o.lds(G["lds_dim"], G["lds_idx"]), G["lds"])


def test_halton_incremental(o):
    for base, start, seq in zip(G["halton_bases"], G["halton_starts"], G["halton_seq"]):
        assert same(o.halton_seq(int(base), int(start), len(seq)), seq), (base, start)


def test_fast_trig_and_exp(o):
    assert same(o.unary("sin", G["trig_x"]), G["sin"])
    assert same(o.unary("cos", G["trig_x"]), G["cos"])
    assert same(o.unary("exp", G["exp_x"]), G["exp"])


def test_vectors_and_hemisphere(o):
    assert same(o.unary("coords_system", G["coords_in"].reshape(-1), 6, 3).reshape(-1, 6), G["coords"])
    assert same(o.unary("normalize", G["norm_in"].reshape(-1), 3, 3).reshape(-1, 3), G["norm"])
    assert same(o.cos_hemisphere(G["hemi_nrv"], G["hemi_s"]), G["hemi"])


def test_bound_cross(o):
    assert same(o.bound_cross(G["bound_box"], G["bound_ray"]), G["bound"])


def test_mwc(o):
    for seed, ref in zip(G["mwc_seeds"], G["mwc"]):
        assert same(o.mwc(int(seed), len(ref)), ref)


def test_film_filter_and_rounding(o):
    assert same(o.unary("filter_gauss", G["gauss_in"].reshape(-1), 1, 2), G["gauss"])
    assert same(o.int_of_double("round_to_int", G["int_in"]), G["round_to_int"])
    assert same(o.int_of_double("floor_to_int", G["int_in"]), G["floor_to_int"])
    assert same(o.clamp_proportional(G["clamp_in"], 1.5), G["clamp_1_5"])
    assert same(o.clamp_proportional(G["clamp_in"], 0.0), G["clamp_0"])


def test_live_reference_random_inputs(o, oracle_built):
    r = oracle_built.ref_prims()
    if r is None:
        pytest.skip("oracle/_ref not built (reference tree absent): golden vectors above still pin the oracle")
    rng = np.random.default_rng(99)
    n = 100000
    b = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    rr = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for w in ("riVdC", "riS", "riLp"):
        assert same(o.ri(w, b, rr), r.ri(w, b, rr))
    dims = rng.integers(1, 50, n).astype(np.int32)
    assert same(o.lds(dims, b), r.lds(dims, b))
    x = rng.uniform(-50, 50, n).astype(np.float32)
    assert same(o.unary("sin", x), r.unary("sin", x))
    assert same(o.unary("cos", x), r.unary("cos", x))


# ---- round 2 (tests/golden/prims_r02.npz): src/geometry/vector.cc shirleyDisk, src/color/color.cc +
# color.h Rgbe, src/render/imagesplitter.cc tile lists ----
G2 = np.load(os.path.join(HERE, "golden", "prims_r02.npz"))


def test_shirley_disk(o):
    assert same(o.shirley(G2["shirley_in"]), G2["shirley"])


def test_rgbe_decode(o):
    assert same(o.rgbe(G2["rgbe_in"]), G2["rgbe"])


def _centre_key(t, w, h):
    return (t[:, 0] - w // 2) ** 2 + (t[:, 1] - h // 2) ** 2


@pytest.mark.parametrize("k", range(6))
def test_tile_lists(o, k):
    w, h, bs = (int(v) for v in G2["tiles_sizes"][k])
    lin = G2[f"tiles_linear_{k}"]
    assert np.array_equal(o.tiles(w, h, bs, "linear"), lin)
    # centre: the reference shuffles with std::random_device before its (unstable) sort, so only the
    # key sequence is determined; the oracle / GPU keep linear order among ties (one of its outcomes)
    ref_c, ours = G2[f"tiles_centre_{k}"], o.tiles(w, h, bs, "centre")
    assert np.array_equal(np.sort(ref_c.view([("", ref_c.dtype)] * 4), axis=0), np.sort(ours.view([("", ours.dtype)] * 4), axis=0))
    assert np.array_equal(_centre_key(ref_c, w, h), _centre_key(ours, w, h))
    kk = _centre_key(ours, w, h)
    assert np.all(np.diff(kk) >= 0)
    # the reference with 8 render threads subdivides its last 16 tiles; the GPU and the oracle
    # render the one-thread list (documented): the lists agree up to there
    t8 = G2[f"tiles_linear_t8_{k}"]
    m = max(0, len(lin) - 16)
    assert np.array_equal(t8[:m], lin[:m])


def test_live_reference_round2_random_inputs(o, oracle_built):
    r = oracle_built.ref_prims()
    if r is None:
        pytest.skip("oracle/_ref not built (reference tree absent): golden vectors above still pin the oracle")
    rng = np.random.default_rng(7)
    r12 = rng.random((50000, 2)).astype(np.float32)
    assert same(o.shirley(r12), r.shirley(r12))
    b = rng.integers(0, 256, (50000, 4), dtype=np.uint8)
    assert same(o.rgbe(b), r.rgbe(b))
    for w, h, bs in [(37, 29, 5), (640, 480, 32), (1, 1, 16)]:
        assert np.array_equal(o.tiles(w, h, bs, "linear"), r.tiles(w, h, bs, "linear"))


# ---- texturing building blocks (tests/golden/tex_prims.npz, made by make_golden_tex.py from the
# reference's own image_buffers.h / color.h / interpolation.h / math.h) ----
TEX_KINDS = {0: "Rgba1010108", 1: "Rgb101010", 2: "Rgba7773", 3: "Rgb565", 4: "Gray8", 5: "Gray", 6: "GrayAlpha", 7: "RgbAlpha"}


@pytest.fixture(scope="module")
def tex_golden():
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tex_prims.npz"))


def test_oracle_texturing_primitives_bitexact(oracle_built, tex_golden):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden_tex as M
    g = tex_golden
    got = M.run(oracle_built.oracle_lib(), "yc_", g["rgba"], g["rgb"], g["sat_hue"], g["cub"], g["ab"])
    for k, v in got.items():
        assert np.array_equal(v.view(np.uint32), g[k].view(np.uint32)), f"{k}: {(v.view(np.uint32) != g[k].view(np.uint32)).sum()} mismatches"


def test_product_image_buffers_quantise_like_the_reference(product, tex_golden):
    """yafaray_createImage + setImageColor / getImageColor through every buffer type (host code of
    the drop-in library: no GPU involved) against the reference's own buffer classes."""
    kinds = {0: ("ColorAlpha", "optimized"), 1: ("Color", "optimized"), 2: ("ColorAlpha", "compressed"),
             3: ("Color", "compressed"), 4: ("Gray", "optimized"), 5: ("Gray", "none"), 6: ("GrayAlpha", "none"),
             7: ("ColorAlpha", "none")}
    rgba = tex_golden["rgba"][:1024]
    yi = product.Interface()
    yi.createScene()
    for kind, (typ, opt) in kinds.items():
        yi.paramsClearAll()
        yi.paramsSetString("type", typ)
        yi.paramsSetString("image_optimization", opt)
        yi.paramsSetInt("width", 32)
        yi.paramsSetInt("height", 32)
        h = yi.createImage(f"img{kind}")
        assert h, typ + "/" + opt
        out = np.empty_like(rgba)
        for i, c in enumerate(rgba):
            yi.setImageColor(h, i % 32, i // 32, *map(float, c))
            out[i] = yi.getImageColor(h, i % 32, i // 32)
        ref = tex_golden[f"quant{kind}"][:1024]
        assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), f"{TEX_KINDS[kind]}: {(out != ref).sum()} mismatches"
    yi.close()


@pytest.mark.parametrize("seed", [1, 2, 7920, 0x7fffffff, 0])
def test_glibc_rand_restatement(oracle_built, seed):
    """The oracle seeds each tile's Russian-roulette generator from a restatement of glibc's rand()
    (integrator_tiled.cc:272, the reference's scene setup reseeds with srand); pinned here against
    the real libc: srand(seed) then 2000 rand() calls (seed 0 behaves as seed 1 in glibc)."""
    import ctypes as C
    libc = C.CDLL("libc.so.6")
    libc.srand.argtypes = [C.c_uint]
    libc.rand.restype = C.c_int
    n = 2000
    libc.srand(seed)
    want = np.array([libc.rand() for _ in range(n)], np.uint32)
    got = oracle_built.glibc_rand(seed, n)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:5]
