"""Canceled renders (yafaray_cancelRendering between wavefront chunks).

Reference semantics (integrator_tiled.cc:292): a canceled worker stops before its next pixel, so
every pixel is either fully sampled or carries no sample and no weight.  The GPU renders the
pixel enumeration in chunks; after a cancel only the completed chunks' whole pixels may splat.

Checked against the uncanceled render of the same scene (itself oracle-checked bit for bit in
test_gpu_parity.py): a pixel whose footprint sources were all rendered equals the full render
bit for bit, a pixel none of whose sources were rendered has weight 0 and colour 0.
"""
import numpy as np
import pytest

from libyafaray_amd import scenes

pytestmark = pytest.mark.gpu


def sample_rank(W, H, ts):
    """Rank of every pixel in the GPU's sample enumeration of a one-band render (render.cc jobs,
    kernels.hip sampleCoord): strips of `ts` columns over the band's rows, left to right, pixels
    row-major inside a strip.  Chunks complete in this order."""
    y, x = np.mgrid[0:H, 0:W]
    tx = x // ts
    tw = np.minimum(ts, W - tx * ts)
    return tx * ts * H + y * tw + (x - tx * ts)


def render(product, spec, chunk, cancel_after=None):
    yi = product.Interface()
    scenes.apply(spec, yi)
    yi.L.yafaray_amd_setChunkSlots(yi.h, chunk)
    calls = []

    def progress(total, done):
        calls.append((total, done))
        if cancel_after is not None and done > 0 and len([c for c in calls if c[1] > 0]) >= cancel_after:
            yi.cancelRendering()

    yi.render(progress=progress)
    rgba, w = yi.film()
    st = yi.stats()
    yi.close()
    return rgba, w, st, calls


@pytest.mark.parametrize("cancel_after", [1, 3])
def test_cancel_between_chunks(product, cancel_after):
    W, H, spp, ts = 64, 48, 8, 16
    spec = scenes.cornell(W, H, spp=spp, bounces=4, rr=False)
    spec.render.tile_size = ts
    chunk = 4096   # 512 pixels per chunk: the frame in 6 chunks
    full, wfull, stf, _ = render(product, spec, chunk)
    part, wpart, stp, calls = render(product, spec, chunk, cancel_after)
    done_samples = stp["samples"]
    assert 0 < done_samples < stf["samples"], (done_samples, stf["samples"], calls)
    assert done_samples % spp == 0
    done_pix = done_samples // spp
    # progress reports are monotone and end before the whole frame
    dones = [c[1] for c in calls]
    assert dones == sorted(dones) and max(dones) < W * H
    rank = sample_rank(W, H, ts)
    rendered = rank < done_pix
    # box-1 footprint: a pixel collects samples from itself, its left, upper and upper-left neighbours
    src = np.zeros((H + 1, W + 1, 4), bool)
    for k, (dy, dx) in enumerate([(0, 0), (1, 0), (0, 1), (1, 1)]):
        src[dy:dy + H, dx:dx + W, k] = rendered
    src[0, :, 1] = src[0, :, 3] = True       # no upper neighbour: counts as "rendered" for "all"
    src[:, 0, 2] = src[:, 0, 3] = True
    all_src = src[:H, :W].all(-1)
    none_src = ~np.stack([rendered,
                          np.pad(rendered, ((1, 0), (0, 0)))[:H],
                          np.pad(rendered, ((0, 0), (1, 0)))[:, :W],
                          np.pad(rendered, ((1, 0), (1, 0)))[:H, :W]], -1).any(-1)
    assert all_src.sum() > 0 and none_src.sum() > 0
    assert np.array_equal(part[all_src].view(np.uint32), full[all_src].view(np.uint32))
    assert np.array_equal(wpart[all_src].view(np.uint32), wfull[all_src].view(np.uint32))
    assert np.all(wpart[none_src] == 0.0) and np.all(part[none_src] == 0.0)
    # mixed pixels carry part of the full weight
    assert np.all(wpart <= wfull)


def test_cancel_before_first_chunk(product):
    """A cancel issued from the opening progress call: nothing is rendered, the film is black."""
    spec = scenes.cornell(32, 24, spp=4, bounces=3, rr=False)
    yi = product.Interface()
    scenes.apply(spec, yi)
    yi.render(progress=lambda total, done: yi.cancelRendering())
    rgba, w = yi.film()
    assert yi.stats()["samples"] == 0
    yi.close()
    assert np.all(w == 0) and np.all(rgba == 0)
