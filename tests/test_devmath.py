"""The exact code the kernels run (libyafaray_amd/csrc/devmath.h), built for the host, against
(a) the reference's golden vectors and (b) real x87 long double arithmetic."""
import ctypes as C
import os
import subprocess
import tempfile

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "prims.npz"))


@pytest.fixture(scope="module")
def dm():
    out = os.path.join(tempfile.gettempdir(), "yaf_devmath_host.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", "-o", out,
                    os.path.join(HERE, "devmath_host.cc")], check=True)
    return C.CDLL(out)


def P(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def test_x87_emulation_vs_long_double():
    exe = os.path.join(tempfile.gettempdir(), "yaf_devmath_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe, os.path.join(HERE, "devmath_check.cc")],
                   check=True)
    r = subprocess.run([exe, "400000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("which,name", [(0, "riVdC"), (1, "riS"), (2, "riLp")])
def test_radical_inverses(dm, which, name):
    b, r = GOLD["ri_bits"], GOLD["ri_r"]
    o = np.empty(len(b), np.float32)
    dm.dm_ri(which, P(b, C.c_uint32), P(r, C.c_uint32), P(o, C.c_float), len(b))
    assert np.array_equal(o.view(np.uint32), GOLD[name].view(np.uint32))


def test_fnv(dm):
    b = GOLD["fnv_in"]
    o = np.empty(len(b), np.uint32)
    dm.dm_fnv(P(b, C.c_uint32), P(o, C.c_uint32), len(b))
    assert np.array_equal(o, GOLD["fnv"])


def test_trig_and_hemisphere(dm):
    x = GOLD["trig_x"]
    for fn, key in (("dm_sin", "sin"), ("dm_cos", "cos")):
        o = np.empty(len(x), np.float32)
        getattr(dm, fn)(P(x, C.c_float), P(o, C.c_float), len(x))
        assert np.array_equal(o.view(np.uint32), GOLD[key].view(np.uint32)), key
    nrv, s = np.ascontiguousarray(GOLD["hemi_nrv"]), np.ascontiguousarray(GOLD["hemi_s"])
    o = np.empty((len(s), 3), np.float32)
    dm.dm_hemi(P(nrv, C.c_float), P(s, C.c_float), P(o, C.c_float), len(s))
    assert np.array_equal(o.view(np.uint32), GOLD["hemi"].view(np.uint32))


def test_vectors(dm):
    cin = np.ascontiguousarray(GOLD["coords_in"])
    o = np.empty((len(cin), 6), np.float32)
    dm.dm_coords(P(cin, C.c_float), P(o, C.c_float), len(cin))
    assert np.array_equal(o.view(np.uint32), GOLD["coords"].view(np.uint32))
    v = np.ascontiguousarray(GOLD["norm_in"])
    o = np.empty_like(v)
    dm.dm_normalize(P(v, C.c_float), P(o, C.c_float), len(v))
    assert np.array_equal(o.view(np.uint32), GOLD["norm"].view(np.uint32))


def test_mwc(dm):
    for seed, ref in zip(GOLD["mwc_seeds"], GOLD["mwc"]):
        o = np.empty(len(ref), np.float64)
        dm.dm_mwc(C.c_uint32(int(seed)), len(ref), P(o, C.c_double))
        assert np.array_equal(o, ref)


def test_halton_first_matches_sequence_start(dm):
    # Halton(base, start).getNext() == first element of the reference sequence from `start`
    for base, start, seq in zip(GOLD["halton_bases"], GOLD["halton_starts"], GOLD["halton_seq"]):
        st = np.array([start], np.uint32)
        o = np.empty(1, np.float32)
        dm.dm_halton_first(C.c_uint32(int(base)), P(st, C.c_uint32), P(o, C.c_float), 1)
        assert o[0] == seq[0]


def test_low_discrepancy_faure(dm):
    # the device uses the Faure tables the host uploads (render.cc faurePerm); rebuild them here
    def perm(b):
        if b <= 2:
            return [0, 1]
        if b % 2 == 0:
            h = perm(b // 2)
            return [2 * v for v in h] + [2 * v + 1 for v in h]
        p, c = perm(b - 1), (b - 1) // 2
        out = []
        for i, v in enumerate(p):
            if i == c:
                out.append(c)
            out.append(v + (v >= c))
        return out
    primes = [1]
    c = 2
    while len(primes) < 50:
        if all(c % q for q in range(2, int(c ** 0.5) + 1)):
            primes.append(c)
        c += 1
    dims, idx, ref = GOLD["lds_dim"], GOLD["lds_idx"], GOLD["lds"]
    for d in np.unique(dims):
        m = dims == d
        pt = np.array(perm(3 if d <= 2 else primes[d]), np.uint8)
        ii = np.ascontiguousarray(idx[m])
        o = np.empty(len(ii), np.float64)
        dm.dm_lds(P(pt, C.c_uint8), C.c_uint32(primes[d]), C.c_double(round(1e9 / primes[d]) / 1e9), P(ii, C.c_uint32),
                  P(o, C.c_double), len(ii))
        assert np.array_equal(o, ref[m]), d


def test_magic_division_exact(dm):
    """udiv() (the digit loops' division by a run-time prime) equals n / d for every prime base the
    samplers use, on edge values and random 32-bit numerators."""
    rng = np.random.default_rng(7)
    n = np.concatenate([np.arange(0, 5000), 2**32 - 1 - np.arange(0, 5000), rng.integers(0, 2**32, 200000)]).astype(np.uint32)
    primes = [p for p in range(2, 260) if all(p % q for q in range(2, int(p**0.5) + 1))]
    for d in primes + [2**31, 2**31 - 1, 1000003]:
        nn = np.concatenate([n, (np.arange(1, 4000, dtype=np.uint64) * d % 2**32).astype(np.uint32)])
        nn = np.concatenate([nn, nn - 1, nn + 1]).astype(np.uint32)
        bad = dm.dm_udiv_check(d, P(nn, C.c_uint32), len(nn))
        assert bad == -1, (d, int(nn[bad]))


def test_libm_restatements_match_host_libm(dm):
    """TextureMapperNode's tube / sphere projections call libm's float atan2 / acos
    (shader_node_basic.cc:67, 77-78); devmath.h restates glibc's fdlibm algorithms so the device
    matches the reference build bit for bit.  2.4 M inputs: uniform in [-1, 1]^2, random exponents, and
    raw bit patterns (NaN, inf, zero, subnormal included)."""
    rng = np.random.default_rng(11)
    n = 800_000
    parts_y = [rng.uniform(-1, 1, n).astype(np.float32),
               (rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-30, 30, n)).astype(np.float32),
               rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)]
    parts_x = [rng.uniform(-1, 1, n).astype(np.float32),
               (rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-30, 30, n)).astype(np.float32),
               rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)]
    y = np.ascontiguousarray(np.concatenate(parts_y))
    x = np.ascontiguousarray(np.concatenate(parts_x))
    m = len(y)
    outs = [np.empty(m, np.float32) for _ in range(4)]
    dm.dm_libm(P(y, C.c_float), P(x, C.c_float), m, *[P(o, C.c_float) for o in outs])
    for dev, ref, name in ((outs[0], outs[1], "atan2f"), (outs[2], outs[3], "acosf")):
        both_nan = np.isnan(dev) & np.isnan(ref)
        same = (dev.view(np.uint32) == ref.view(np.uint32)) | both_nan
        assert same.all(), f"{name}: {(~same).sum()} of {m} differ, e.g. {y[~same][:3]} {x[~same][:3]}"


def test_sphere_v_long_double(dm):
    """1.f - 2.f * (acos * div_1_by_pi) with the long double product and difference: every acos value
    in [0, pi] on a fine grid plus random floats, against real x87 long double."""
    rng = np.random.default_rng(12)
    a = np.concatenate([np.linspace(0, np.pi, 1_000_001, dtype=np.float32), rng.uniform(0, np.pi, 1_000_000).astype(np.float32),
                        np.float32([0.0, np.float32(np.pi), np.float32(np.pi / 2)])])
    a = np.ascontiguousarray(a)
    dev, ref = np.empty_like(a), np.empty_like(a)
    dm.dm_sphere_v(P(a, C.c_float), len(a), P(dev, C.c_float), P(ref, C.c_float))
    bad = dev.view(np.uint32) != ref.view(np.uint32)
    assert not bad.any(), f"{bad.sum()} differ, e.g. {a[bad][:3]}"
