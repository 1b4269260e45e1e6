"""Multi-GPU path on CPU: tile-row sharding + all-gather reassembly over torch.distributed (gloo,
world size 2 and 3), checked against the single-process film bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import tiles


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, image, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    H, W, _ = image.shape
    ts = 32
    band = torch.from_numpy(tiles.pack_band(image, H, ts, rank, world))
    parts = [torch.zeros_like(band) for _ in range(world)]
    dist.all_gather(parts, band)
    full = tiles.assemble(torch.cat(parts).numpy(), H, ts, world)
    if rank == 0:
        q.put(full)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_reassembles_the_film(world, oracle_built):
    from libyafaray_amd import scenes
    spec = scenes.cornell(96, 70, spp=2, bounces=3, rr=False)
    image, _, _ = oracle_built.OracleScene(spec, threads=4).render()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, image, q)) for r in range(world)]
    for p in procs:
        p.start()
    full = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(full.view(np.uint32), image.view(np.uint32))


def test_sharding_covers_every_row_once():
    for H, ts, world in [(1080, 32, 8), (1080, 32, 3), (70, 32, 4), (31, 32, 2)]:
        seen = np.zeros(H, int)
        for r in range(world):
            for t in tiles.owned_tile_rows(H, ts, r, world):
                seen[t * ts:min(H, t * ts + ts)] += 1
        assert (seen == 1).all()


def _band_worker(rank, world, port, image, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    H = image.shape[0]
    band = torch.from_numpy(tiles.pack_row_band(image, rank, world))
    parts = [torch.zeros_like(band) for _ in range(world)]
    dist.all_gather(parts, band)
    full = tiles.assemble_row_bands(torch.cat(parts).numpy(), H, world)
    if rank == 0:
        q.put(full)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_reassembles_row_bands(world, oracle_built):
    """The default split (contiguous row bands, bench.py) through gloo all-gather."""
    from libyafaray_amd import scenes
    spec = scenes.cornell(96, 70, spp=2, bounces=3, rr=False)
    image, _, _ = oracle_built.OracleScene(spec, threads=4).render()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_band_worker, args=(r, world, port, image, q)) for r in range(world)]
    for p in procs:
        p.start()
    full = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(full.view(np.uint32), image.view(np.uint32))


def test_row_bands_cover_every_row_once():
    for H, world in [(1080, 8), (1080, 3), (70, 4), (5, 8), (1, 2)]:
        seen = np.zeros(H, int)
        for r in range(world):
            y0, y1 = tiles.band_range(H, r, world)
            seen[y0:y1] += 1
        assert (seen == 1).all()
        assert tiles.band_rows_max(H, world) <= -(-H // world)


def test_rebalance_bands_moves_towards_equal_cost():
    """bench.py's band load balancing (tiles.rebalance_bands): boundaries stay ordered, every band keeps
    >= 1 row, the cap is honoured, equal times keep equal bands, and a slow band shrinks."""
    H, world = 1080, 8
    bounds = [tiles.band_range(H, r, world)[0] for r in range(world)] + [H]
    assert tiles.rebalance_bands(bounds, [1.0] * world) == bounds
    times = [1.0] * world
    times[3] = 2.0
    new = tiles.rebalance_bands(bounds, times)
    assert new[0] == 0 and new[-1] == H and all(new[r] < new[r + 1] for r in range(world))
    assert new[4] - new[3] < bounds[4] - bounds[3]
    # iterating with a fixed per-row cost density converges to equal cost per band
    dens = np.linspace(1.0, 3.0, H)
    b = list(bounds)
    for _ in range(30):
        cost = [dens[b[r]:b[r + 1]].sum() for r in range(world)]
        b = tiles.rebalance_bands(b, cost)
    cost = [dens[b[r]:b[r + 1]].sum() for r in range(world)]
    assert max(cost) / min(cost) < 1.03
    # a cap that the new split would exceed keeps the old bounds; degenerate sizes are left alone
    cap = max(bounds[r + 1] - bounds[r] for r in range(world))
    assert tiles.rebalance_bands(bounds, times, cap_rows=cap) in (bounds, new)
    assert tiles.rebalance_bands([0, 3], [1.0]) == [0, 3]
    tiny = tiles.rebalance_bands([0, 1, 2, 3], [5.0, 1.0, 1.0])
    assert tiny == [0, 1, 2, 3]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_library_band_balancer_matches_python(product, world):
    """yafaray_amd_rebalanceBands (the in-library group's balancer, C++) == tiles.rebalance_bands."""
    rng = np.random.default_rng(world)
    for H in (70, 1080):
        bounds = tiles_bounds = [H * r // world for r in range(world + 1)]
        for _ in range(6):
            times = list(rng.uniform(0.5, 2.0, world))
            lib = product.rebalance_bands(bounds, times)
            py = tiles.rebalance_bands(tiles_bounds, times)
            assert lib == [int(v) for v in py], (lib, py)
            assert lib[0] == 0 and lib[-1] == H and all(b > a for a, b in zip(lib, lib[1:]))
            bounds = tiles_bounds = lib


def _lib_band_worker(rank, world, port, image, weights, bounds, q):
    """One render-group member on gloo running the LIBRARY's band plan (yafaray_amd_packBand /
    unpackBands, the host twins of GpuRenderer::exchangeRows): it holds the film only in its own band
    (NaN elsewhere), packs its slot, all-gathers, unpacks the other members' rows."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import libyafaray_amd as Y
    film = np.full_like(image, np.nan)
    wt = np.full_like(weights, np.nan)
    y0, y1 = bounds[rank], bounds[rank + 1]
    film[y0:y1] = image[y0:y1]
    wt[y0:y1] = weights[y0:y1]
    out = []
    for arr in (film, wt):
        send = torch.from_numpy(Y.pack_band(arr, bounds, rank))
        parts = [torch.zeros_like(send) for _ in range(world)]
        dist.all_gather(parts, send)
        out.append(Y.unpack_bands(torch.cat(parts).numpy(), bounds, rank, arr))
    q.put((rank, out[0], out[1]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_library_band_plan_over_gloo(product, oracle_built, world):
    """The in-library render group's combine plan on CPU ranks: uneven (rebalanced) bands packed and
    unpacked by libyafaray4.so around a gloo all-gather give every member the whole film, bit for bit."""
    from libyafaray_amd import scenes
    spec = scenes.cornell(96, 70, spp=2, bounces=3, rr=False)
    image, weights, _ = oracle_built.OracleScene(spec, threads=4).render()
    H = image.shape[0]
    bounds = [H * r // world for r in range(world + 1)]
    bounds = product.rebalance_bands(bounds, [1.0 + 0.8 * r for r in range(world)])
    assert len(set(b - a for a, b in zip(bounds, bounds[1:]))) > 1, bounds
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lib_band_worker, args=(r, world, port, image, weights, bounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, film, wt in got:
        assert np.array_equal(film.view(np.uint32), image.view(np.uint32)), rank
        assert np.array_equal(wt.view(np.uint32), weights.view(np.uint32)), rank


def test_library_band_plan_rejects_bad_bounds(product):
    film = np.zeros((10, 4, 4), np.float32)
    with pytest.raises(RuntimeError):
        product.pack_band(film, [0, 5, 9], 0)       # does not end at the film height
    with pytest.raises(RuntimeError):
        product.pack_band(film, [0, 6, 5, 10], 1)   # bounds out of order
