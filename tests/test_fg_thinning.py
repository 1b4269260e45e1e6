"""Final gathering's radiance-point thinning (integrator_photon_mapping.cc:560-572): the serial
greedy walk of the reference (a point still in use is kept and marks its related points unused)
and the round formulation the GPU runs (libyafaray_amd/csrc/fgthin.hip: keep / kill rounds over
the undecided points) give the same kept set — the lexicographically-first maximal independent
set of the relation "squared distance < maxrad and normals on the same side".  Checked here on
random point sets with numpy restatements of both (the kernels themselves are checked on the GPU
by tests/test_final_gather.py, whose images depend on the kept set)."""
import numpy as np
import pytest


def related(pos, nrm, i, maxrad):
    v = pos - pos[i]
    d2 = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    nd = (nrm[:, 0] * nrm[i, 0] + nrm[:, 1] * nrm[i, 1]) + nrm[:, 2] * nrm[i, 2]
    return (d2 < maxrad) & (nd > 0)


def greedy(pos, nrm, maxrad):
    use = np.ones(len(pos), bool)
    kept = []
    for i in range(len(pos)):
        if use[i]:
            kept.append(i)
            use[related(pos, nrm, i, maxrad)] = False
    return kept


def rounds(pos, nrm, maxrad):
    n = len(pos)
    UND, KEPT, DEAD = 0, 1, 2
    state = np.zeros(n, np.int8)
    rel = [np.nonzero(related(pos, nrm, i, maxrad))[0] for i in range(n)]
    U = np.arange(n)
    r = 0
    while len(U):
        # keep: no undecided lower related point in the snapshot
        newk = [i for i in U if not np.any((rel[i] < i) & (state[rel[i]] == UND))]
        # kill: newly kept points mark their higher related points dead
        for i in newk:
            state[i] = KEPT
            hi = rel[i][rel[i] > i]
            state[hi] = DEAD
        U = np.array([i for i in U if state[i] == UND], dtype=np.int64)
        r += 1
        assert r <= n
    return list(np.nonzero(state == KEPT)[0]), r


@pytest.mark.parametrize("seed", range(6))
def test_rounds_equal_greedy(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(50, 400))
    pos = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    if seed % 2:
        pos[:, 2] = np.float32(0.25)          # points on a plane (as on the Cornell walls)
    nrm = rng.normal(size=(n, 3)).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    maxrad = np.float32(rng.uniform(0.01, 0.2))
    kept, r = rounds(pos, nrm, maxrad)
    assert kept == greedy(pos, nrm, maxrad)
    assert r >= 1
