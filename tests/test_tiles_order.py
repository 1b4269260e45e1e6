"""Tile order (ImageSplitter, imagesplitter.cc:30-107) and the per-tile callbacks
(ImageFilm::nextArea / finishArea, imagefilm.cc:447-568).

The tile order decides the film's splat order (a pixel sums the samples of its footprint sources in
the order their tiles finish) and the order of the highlightArea / putPixel / flushArea callbacks.
"centre" is the reference's default (ImageSpliterCentreSorter: squared distance of the tile corner
to the image centre; the reference breaks ties by a random shuffle, here ties keep linear order);
"random" uses a fixed seed here (the reference seeds from std::random_device).  Both sides render
as one reference thread does (no subdivision of the last tiles).

Parity: the film equals the oracle's film of the same order (<= 4 ULP, gauss filter so that every
sample splats across tile borders).  Callbacks: one highlightArea + the tile's putPixels + one
flushArea per tile in the order, area ids 0..n-1; a putPixel shows the pixel as the one-thread render
does when its tile finishes — equal to the final value wherever every footprint source's tile
finished no later; the final flush shows the film.
"""
import dataclasses

import numpy as np
import pytest

from libyafaray_amd import scenes


def tile_order(W, H, ts, order):
    """The tile list in render order, as (x0, y0, x1, y1) — the restatement of imagesplitter.cc."""
    ntx, nty = (W + ts - 1) // ts, (H + ts - 1) // ts
    ids = list(range(ntx * nty))
    if order == "centre":
        key = lambda i: ((i % ntx) * ts - W // 2) ** 2 + ((i // ntx) * ts - H // 2) ** 2
        ids = sorted(ids, key=key)   # Python's sort is stable: ties keep linear order
    elif order != "linear":
        raise ValueError(order)
    return [((i % ntx) * ts, (i // ntx) * ts, min(W, (i % ntx) * ts + ts), min(H, (i // ntx) * ts + ts)) for i in ids]


def ulp_diff(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7fffffff), a)
    b = np.where(b < 0, -(b & 0x7fffffff), b)
    return np.abs(a - b)


def spec(order, W=50, H=38, ts=8, spp=2, filt="gauss"):
    s = scenes.cornell(W, H, spp=spp, bounces=3, rr=False, integrator="directlighting")
    return s.with_render(tiles_order=order, tile_size=ts, filter_type=filt, aa_pixelwidth=1.0)   # gauss: 2x2 forward footprint


def test_centre_order_restatement():
    t = tile_order(64, 48, 16, "centre")
    assert len(t) == 12 and t[0] == (32, 16, 48, 32)    # the tile whose corner is the centre
    keys = [(x - 32) ** 2 + (y - 24) ** 2 for x, y, _, _ in t]
    assert keys == sorted(keys)


@pytest.mark.parametrize("order", ["linear", "centre"])
def test_restatement_matches_oracle_tile_lists(oracle_built, order):
    """tile_order() (used by the callback test) = the oracle's list, itself pinned against the
    reference's ImageSplitter (tests/test_oracle_golden.py::test_tile_lists)."""
    o = oracle_built.oracle_prims()
    for W, H, ts in [(50, 38, 8), (64, 48, 16), (1920, 1080, 32)]:
        t = o.tiles(W, H, ts, order)
        assert [(x, y, x + w, y + h) for x, y, w, h in t.tolist()] == tile_order(W, H, ts, order)


def test_oracle_orders_differ_only_by_summation_order(oracle_built):
    a, wa, _ = oracle_built.OracleScene(spec("linear"), threads=4).render()
    b, wb, _ = oracle_built.OracleScene(spec("centre"), threads=4).render()
    assert np.all(ulp_diff(wa, wb) <= 4) and np.all(ulp_diff(a, b) <= 8)


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["linear", "centre", "random"])
def test_tile_order_film_matches_oracle(product, oracle_built, order):
    s = spec(order)
    rgba, w, _ = product.render_spec(s)
    orgba, ow, _ = oracle_built.OracleScene(s, threads=8).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    d = ulp_diff(rgba, orgba)
    assert d.max() <= 4, f"{(d > 4).sum()} values > 4 ULP"


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["linear", "centre"])
def test_per_tile_callbacks(product, order):
    s = spec(order)
    W, H, ts = s.render.width, s.render.height, s.render.tile_size
    yi = product.Interface()
    scenes.apply(s, yi)
    events = []
    tile_px = {}
    final = np.zeros((H, W, 4), np.float32)
    state = {"flushed": False, "cur": None}

    def highlight(aid, x0, y0, x1, y1):
        events.append(("h", aid, (x0, y0, x1, y1)))
        state["cur"] = aid

    def put(x, y, r, g, b, a):
        if state["flushed"] or state["cur"] is None:
            final[y, x] = (r, g, b, a)   # the final flush (after the last tile)
        else:
            tile_px[(x, y)] = (r, g, b, a)

    def flush_area(aid, x0, y0, x1, y1):
        events.append(("f", aid, (x0, y0, x1, y1)))
        state["cur"] = None

    def flush():
        state["flushed"] = True

    # the final putPixels come after every tile's flushArea (cur is None then)
    yi.render(put_pixel=put, flush_area=flush_area, flush=flush, highlight_area=highlight)
    film, wts = yi.film()
    yi.close()
    expect = tile_order(W, H, ts, order)
    assert [e for e in events if e[0] == "h"] == [("h", k, t) for k, t in enumerate(expect)]
    assert [e for e in events if e[0] == "f"] == [("f", k, t) for k, t in enumerate(expect)]
    assert all(events[2 * k][0] == "h" and events[2 * k + 1][0] == "f" for k in range(len(expect)))
    assert len(tile_px) == W * H
    assert np.array_equal(final.view(np.uint32), film.view(np.uint32))
    part = np.zeros_like(final)
    for (x, y), v in tile_px.items():
        part[y, x] = v
    # rank of every pixel's tile; gauss sources of (x, y): (x-1..x, y-1..y)
    rank = np.zeros((H, W), np.int64)
    for k, (x0, y0, x1, y1) in enumerate(expect):
        rank[y0:y1, x0:x1] = k
    pad = np.pad(rank, ((1, 0), (1, 0)), constant_values=-1)
    src_max = np.maximum.reduce([pad[1:, 1:], pad[:-1, 1:], pad[1:, :-1], pad[:-1, :-1]])
    settled = src_max <= rank
    assert np.array_equal(part[settled].view(np.uint32), film[settled].view(np.uint32))
    if order == "linear":
        assert settled.all()
    else:
        assert (~settled).any() and not np.array_equal(part[~settled], film[~settled])
