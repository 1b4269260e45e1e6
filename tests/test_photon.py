"""Photon mapping (BASELINE C5) on CPU: the oracle's photon map and point kd-tree against brute
force, and the device heap replica against libstdc++ (the reference's heap)."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from libyafaray_amd import scenes

HERE = os.path.dirname(os.path.abspath(__file__))


def test_heap_replica_matches_libstdcxx():
    exe = os.path.join(tempfile.gettempdir(), "yaf_photon_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(HERE, "photon_check.cc")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def kd_lookup(nodes, pos, p, r2):
    """All photons within squared radius r2 of p by walking the oracle's kd-tree layout
    (pkdtree.h:41-64: flags & 3 == 3 leaf, else axis; right child = flags >> 2, left = i + 1)."""
    out, stack = [], [0]
    while stack:
        i = stack.pop()
        data, flags = int(nodes[i, 0]), int(nodes[i, 1])
        if flags & 3 == 3:
            if ((pos[data] - p) ** 2).sum() < r2:
                out.append(data)
            continue
        axis, split = flags & 3, np.uint32(data).view(np.float32)
        right = flags >> 2
        d = p[axis] - split
        if d <= 0 or d * d < r2:
            stack.append(i + 1)
        if d > 0 or d * d < r2:
            stack.append(right)
    return sorted(out)


def test_photon_map_and_kdtree(oracle_built):
    spec = scenes.cornell_photon(16, 16, spp=1, photons=4000)
    osc = oracle_built.OracleScene(spec, threads=2)
    pos, d, col, nodes, n_paths = osc.photon_map()
    assert n_paths == 4000
    assert 1.5 * 4000 < len(pos) < 2.6 * 4000          # ~2 stored photons per path in the Cornell box
    assert np.all(np.isfinite(pos)) and np.all(col >= 0)
    assert np.allclose(np.linalg.norm(d, axis=1), 1.0, atol=5e-3)   # FAST_TRIG cosHemisphere is not exactly unit
    # every photon is a leaf exactly once; every interior node splits its subtree
    leaves = nodes[(nodes[:, 1] & 3) == 3, 0]
    assert sorted(leaves.tolist()) == list(range(len(pos)))
    rng = np.random.default_rng(3)
    for q in rng.uniform([-1, -1, 0], [1, 1, 2], (40, 3)).astype(np.float32):
        brute = sorted(np.nonzero(((pos - q) ** 2).sum(1) < 0.05)[0].tolist())
        assert kd_lookup(nodes, pos, q, 0.05) == brute


def test_photon_render_deterministic_and_thread_free(oracle_built):
    spec = scenes.cornell_photon(24, 16, spp=2, photons=3000)
    a, wa, _ = oracle_built.OracleScene(spec, threads=1).render()
    b, wb, _ = oracle_built.OracleScene(spec, threads=6).render()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    # the photon estimate adds light on top of direct lighting everywhere the camera sees a wall
    dl, _, _ = oracle_built.OracleScene(scenes.cornell(24, 16, spp=2, integrator="directlighting"), threads=4).render()
    assert (a[..., :3] >= dl[..., :3] - 1e-6).all() and a[..., :3].mean() > 1.5 * dl[..., :3].mean()
