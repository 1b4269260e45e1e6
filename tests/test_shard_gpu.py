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
