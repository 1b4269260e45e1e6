"""The GPU point kd-tree build (pkd.hip) node for node against a numpy restatement of the
reference's build (include/photon/pkdtree.h:115-222: median element (start + end) / 2 of the largest
bound axis, order coordinate then element index), through yafaray_amd_buildPhotonTree.  Sizes on
both sides of the subtree phase (256 photons) and several top levels of the fused look-back
partition (k_level_partition: tiles of 2048 entries); the level-wise scan + partition passes
(YAFARAY_AMD_PKD_PARTITION=scan) must give the identical tree at photon-map scale."""
import numpy as np
import pytest

import libyafaray_amd as Y


def okey(f):
    f = np.where(f == 0, np.float32(0), f).astype(np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xffffffff, u | 0x80000000)


def largest(lo, hi):
    dx, dy, dz = (np.float32(hi[k]) - np.float32(lo[k]) for k in range(3))
    return (0 if dx > dz else 2) if dx > dy else (1 if dy > dz else 2)


def ref_tree(pos):
    """pkdtree.h:115-222 restated (nodes without the parent-plane words .y / .z of interior nodes)."""
    n = len(pos)
    keys = [okey(pos[:, a]) for a in range(3)]
    bits = pos.view(np.uint32)
    nodes = np.zeros((2 * n - 1, 4), np.uint32)
    depth = 0
    stack = [(0, np.arange(n), pos.min(0).copy(), pos.max(0).copy(), 0)]
    while stack:
        node, idx, lo, hi, d = stack.pop()
        depth = max(depth, d)
        if len(idx) == 1:
            i = int(idx[0])
            nodes[node] = (bits[i, 0], bits[i, 1], bits[i, 2], 3 | (i << 2))
            continue
        ax = largest(lo, hi)
        o = idx[np.lexsort((idx, keys[ax][idx]))]
        h = len(idx) // 2
        sp = pos[o[h], ax]
        right = node + 2 * h
        nodes[node] = (bits[o[h], ax], 0, 0, ax | (right << 2))
        lhi = hi.copy(); lhi[ax] = sp
        rlo = lo.copy(); rlo[ax] = sp
        stack.append((node + 1, o[:h], lo, lhi, d + 1))
        stack.append((right, o[h:], rlo, hi, d + 1))
    return nodes, depth


def positions(n, seed):
    rng = np.random.default_rng(seed)
    p = rng.random((n, 3), dtype=np.float32) * np.float32(4) - np.float32(2)
    if n > 10:
        p[::7, 1] = 0.5          # ties on one axis
        p[::11, 0] = -0.0        # -0 == +0 in the comparator
        p[::13] = p[0]           # coincident photons
    return p


def interior_core(nodes):
    """Interior nodes without the parent-plane words (pkd.hip adds them for k_gather_walk)."""
    out = nodes.copy()
    inner = (out[:, 3] & 3) != 3
    out[inner, 1] = 0
    out[inner, 2] = 0
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 256, 257, 3000, 9000, 40000])
def test_photon_tree_matches_reference_build(product, n):
    pos = positions(n, 100 + n)
    got, depth = Y.build_photon_tree(pos)
    want, wdepth = ref_tree(pos)
    bad = np.flatnonzero((interior_core(got) != want).any(axis=1))
    assert bad.size == 0, f"{bad.size} nodes differ, first {bad[0]}: {got[bad[0]]} vs {want[bad[0]]}"
    assert depth == wdepth


@pytest.mark.gpu
def test_photon_tree_fused_partition_equals_scan_passes(product, monkeypatch):
    """1.5 M photons (10 top levels, 733 tiles per list): the fused look-back partition and the
    separate scan + partition passes build the same tree."""
    pos = positions(1_500_000, 5)
    fused, d1 = Y.build_photon_tree(pos)
    monkeypatch.setenv("YAFARAY_AMD_PKD_PARTITION", "scan")
    scan, d2 = Y.build_photon_tree(pos)
    assert d1 == d2
    assert np.array_equal(fused, scan)
