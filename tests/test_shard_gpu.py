"""Film sharding across GPUs, rehearsed on one GPU: every rank's share (contiguous row band — the
default — or round-robin tile rows) is rendered by its own render call and the owned rows are
composed; the result must equal the one-GPU film bit for bit, Russian roulette on (its per-sample
seed is pixel-major, so it does not depend on the split), for filters whose splat footprint reaches
into neighbouring rows (halo rows)."""
import numpy as np
import pytest

from libyafaray_amd import scenes


def _compose(product, spec, world, mode):
    H, W = spec.render.height, spec.render.width
    rgba = np.full((H, W, 4), np.nan, np.float32)
    wt = np.full((H, W), np.nan, np.float32)
    covered = np.zeros(H, int)
    for r in range(world):
        a, w, st = product.render_spec(spec, shard=(r, world, mode))
        for y0, y1 in st["owned_rows"]:
            rgba[y0:y1] = a[y0:y1]
            wt[y0:y1] = w[y0:y1]
            covered[y0:y1] += 1
    assert (covered == 1).all(), "owned rows must partition the film"
    return rgba, wt


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode", [(2, "band"), (3, "band"), (8, "band"), (3, "tile"), (8, "tile")])
@pytest.mark.parametrize("filt", [("box", 1.0), ("gauss", 1.5)])
def test_sharded_film_equals_one_gpu(product, world, mode, filt):
    spec = scenes.cornell(128, 90, spp=4, bounces=4, rr=True, filter_type=filt[0], pixelwidth=filt[1])
    full, fw, _ = product.render_spec(spec)
    rgba, wt = _compose(product, spec, world, mode)
    assert np.array_equal(wt.view(np.uint32), fw.view(np.uint32))
    assert np.array_equal(rgba.view(np.uint32), full.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 5])
def test_render_group_bands_rebalanced(product, world):
    """The in-library render group's split (yafaray_amd_setRenderGroup): each member renders the
    band [b_r, b_r+1) the library's balancer assigns — here after two rounds of uneven times, so the
    bands are unequal — and groupCombine copies those rows from member r.  Rehearsed on one GPU with
    the same bands through setRowBandRange; the composition equals the one-GPU film bit for bit."""
    spec = scenes.cornell(96, 70, spp=4, bounces=4, rr=True, filter_type="gauss", pixelwidth=1.5)
    H = spec.render.height
    full, fw, _ = product.render_spec(spec)
    bounds = [H * r // world for r in range(world + 1)]
    for times in ([1.0 + 0.7 * r for r in range(world)], [3.0 - 0.4 * r for r in range(world)]):
        bounds = product.rebalance_bands(bounds, times)
    assert len(set(b - a for a, b in zip(bounds, bounds[1:]))) > 1, bounds
    rgba = np.full_like(full, np.nan)
    wt = np.full_like(fw, np.nan)
    for r in range(world):
        yi = product.Interface()
        scenes.apply(spec, yi)
        yi.L.yafaray_amd_setRowBandRange(yi.h, bounds[r], bounds[r + 1], world)
        yi.render()
        a, w = yi.film()
        assert yi.owned_rows() == [(bounds[r], bounds[r + 1])]
        rgba[bounds[r]:bounds[r + 1]] = a[bounds[r]:bounds[r + 1]]
        wt[bounds[r]:bounds[r + 1]] = w[bounds[r]:bounds[r + 1]]
        yi.close()
    assert np.array_equal(wt.view(np.uint32), fw.view(np.uint32))
    assert np.array_equal(rgba.view(np.uint32), full.view(np.uint32))


@pytest.mark.gpu
def test_render_group_of_one_and_id(product):
    """The group id is an RCCL unique id; a group of one renders exactly the plain film."""
    gid = product.render_group_id()
    assert len(gid) == 128
    spec = scenes.cornell(48, 32, spp=2, bounces=3)
    full, fw, _ = product.render_spec(spec)
    yi = product.Interface()
    scenes.apply(spec, yi)
    assert yi.L.yafaray_amd_setRenderGroup(yi.h, 0, 1, gid, len(gid))
    yi.render()
    a, w = yi.film()
    yi.close()
    assert np.array_equal(a.view(np.uint32), full.view(np.uint32))
