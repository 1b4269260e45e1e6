"""Device group: one process renders one film on several GPUs (yafaray_amd_setDeviceGroup, the
render parameter "gpus").  Each member renders a row band (+ halo rows) on its own host thread and
HIP stream; between adaptive passes the members agree on their status and exchange the accumulated
rows (nextPass reads neighbouring pixels); at the end member 0 pulls every band (hipMemcpyPeer).

The rehearsal maps N logical members onto the one GPU of the test box — the members, threads,
barriers, band plan and copies are exactly those of N GPUs (a peer copy between two members of one
device is a device copy).  The reference's counterpart is its render threads sharing the film's
tiles (integrator_tiled.cc:246-264, imagesplitter.cc:30-107): the film must not depend on how many
workers render it, so every case is compared bit for bit with the one-member render (itself
oracle-checked in test_gpu_parity.py / test_film_io.py / test_final_gather.py).
"""
import dataclasses

import numpy as np
import pytest

import filmfile
from libyafaray_amd import scenes

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _same(a, b):
    return np.array_equal(_bits(a), _bits(b))


@pytest.mark.parametrize("members", [2, 3, 8])
@pytest.mark.parametrize("filt", [("box", 1.0), ("gauss", 1.5), ("mitchell", 1.5)])
def test_device_group_film_equals_one_member(product, members, filt):
    """Path tracing with Russian roulette (pixel-major RR seeds: split-independent), filters whose
    footprint reaches one or more rows into the neighbouring bands."""
    spec = scenes.cornell(96, 70, spp=4, bounces=4, rr=True, filter_type=filt[0], pixelwidth=filt[1])
    full, fw, st1 = product.render_spec(spec, members=1)
    rgba, w, st = product.render_spec(spec, members=members)
    assert _same(w, fw)
    assert _same(rgba, full)
    assert st["samples"] >= st1["samples"]   # halo rows are rendered by two members
    assert st["owned_rows"] == [(0, spec.render.height)]


def test_device_group_size_and_default(product):
    """setDeviceGroup decides the member count; without it the "gpus" parameter (-1: every visible
    device) does — on the one-GPU test box that is one member."""
    spec = scenes.cornell(32, 24, spp=1, bounces=2)
    yi = product.Interface()
    scenes.apply(spec, yi)
    assert yi.device_group_size() >= 1
    yi.set_device_group(5)
    assert yi.device_group_size() == 5
    yi.set_device_group(0)
    assert yi.device_group_size() >= 1
    yi.close()


@pytest.mark.parametrize("members", [2, 4])
def test_device_group_repeated_frames_rebalance(product, members):
    """Frames after the first use bands moved by the members' measured times (rebalanceBands); the
    film stays bit-identical frame after frame."""
    spec = scenes.cornell(64, 48, spp=2, bounces=3, rr=True, filter_type="gauss", pixelwidth=1.5)
    full, fw, _ = product.render_spec(spec, members=1)
    yi = product.Interface()
    scenes.apply(spec, yi)
    yi.set_device_group(members)
    for _ in range(3):
        yi.render_quiet()
        a, w = yi.film()
        assert _same(a, full) and _same(w, fw)
    yi.close()


ADAPTIVE = {
    "dl-3pass": lambda: scenes.test01(64, 64, spp=2).with_render(aa_passes=3, aa_inc_samples=2, aa_threshold=0.02),
    "pt-all-options": lambda: scenes.cornell(48, 40, spp=2, bounces=4, rr=False).with_render(
        aa_passes=4, aa_inc_samples=1, aa_threshold=0.01, aa_dark_detection_type="curve", aa_detect_color_noise=True,
        aa_variance_pixels=3, aa_variance_edge_size=6, aa_resampled_floor=60.0, aa_sample_multiplier_factor=1.5),
    "pt-gauss-rr": lambda: scenes.cornell(56, 44, spp=2, bounces=3, rr=True, filter_type="gauss", pixelwidth=1.5).with_render(
        aa_passes=3, aa_inc_samples=2, aa_threshold=0.02),
}


@pytest.mark.parametrize("members", [2, 3])
@pytest.mark.parametrize("case", list(ADAPTIVE))
def test_device_group_adaptive_passes(product, case, members):
    """Adaptive anti-aliasing across bands: nextPass over the exchanged whole film, each member
    resamples the flagged pixels of its band + halo rows, its film rows accumulate them."""
    spec = ADAPTIVE[case]()
    full, fw, st1 = product.render_spec(spec, members=1, chunk_slots=4096)
    rgba, w, st = product.render_spec(spec, members=members, chunk_slots=4096)
    assert st1["samples"] > spec.render.width * spec.render.height * spec.render.aa_samples   # passes ran
    assert _same(w, fw), f"{(w != fw).sum()} weights differ"
    assert _same(rgba, full)


def test_device_group_film_save_and_resume(product, tmp_path):
    """Film files (imagefilm.cc:817-1130) with a device group: the saved accumulators are the whole
    film's (combined from every band), and a resumed 3-pass render equals the uninterrupted one."""
    def spec(**kw):
        return scenes.test01(64, 64, spp=2).with_render(aa_inc_samples=2, aa_threshold=0.02, **kw)
    full, fw, _ = product.render_spec(spec(aa_passes=3), members=1)
    p1, p3 = str(tmp_path / "one"), str(tmp_path / "three")
    a1, w1, _ = product.render_spec(spec(aa_passes=3, film_load_save_mode="save", film_load_save_path=p1).with_render(
        aa_threshold=1e30), members=1)
    a3, w3, _ = product.render_spec(spec(aa_passes=3, film_load_save_mode="save", film_load_save_path=p3).with_render(
        aa_threshold=1e30), members=3)
    f1, f3 = filmfile.read(filmfile.film_path(p1)), filmfile.read(filmfile.film_path(p3))
    assert _same(f3.weights, f1.weights) and _same(f3.layers[0], f1.layers[0])
    assert f3.sampling_offset == f1.sampling_offset
    assert _same(a3, a1) and _same(w3, w1)
    a, w, _ = product.render_spec(spec(aa_passes=3, film_load_save_mode="load-save", film_load_save_path=p3,
                                       film_autosave_interval_type="pass-interval"), members=3)
    assert _same(w, fw) and _same(a, full)


def test_device_group_tile_callbacks(product):
    """A group render reports every tile (highlightArea + flushArea in render order) after the bands
    are combined, then the final putPixel flush of the whole film."""
    spec = scenes.cornell(80, 56, spp=1, bounces=2)
    spec.render.tile_size = 16
    spec.render.tiles_order = "linear"
    yi = product.Interface()
    scenes.apply(spec, yi)
    yi.set_device_group(3)
    ev, px, prog = [], {}, []
    yi.render(progress=lambda t, d: prog.append((t, d)),
              highlight_area=lambda aid, x0, y0, x1, y1: ev.append(("h", aid, (x0, y0, x1, y1))),
              flush_area=lambda aid, x0, y0, x1, y1: ev.append(("f", aid, (x0, y0, x1, y1))),
              put_pixel=lambda x, y, r, g, b, a: px.__setitem__((x, y), (r, g, b, a)))
    film, _ = yi.film()
    yi.close()
    W, H, ts = 80, 56, 16
    tiles = [(tx, ty, min(W, tx + ts), min(H, ty + ts)) for ty in range(0, H, ts) for tx in range(0, W, ts)]
    assert [e for e in ev if e[0] == "f"] == [("f", k, t) for k, t in enumerate(tiles)]
    assert [e for e in ev if e[0] == "h"] == [("h", k, t) for k, t in enumerate(tiles)]
    assert len(px) == W * H
    got = np.zeros_like(film)
    for (x, y), v in px.items():
        got[y, x] = v
    assert _same(got, film)
    assert prog and prog[-1] == (W * H, W * H)


def test_device_group_photon_map(product):
    """PhotonIntegrator (diffuse map, k-NN gather) with a device group."""
    spec = scenes.cornell_photon(48, 36, spp=1, photons=20000, search=50, radius=0.1)
    full, fw, _ = product.render_spec(spec, members=1)
    rgba, w, _ = product.render_spec(spec, members=3)
    assert _same(w, fw) and _same(rgba, full)


def test_device_group_final_gather(product):
    spec = scenes.cornell_photon(40, 30, spp=1, photons=20000, search=50, radius=0.1)
    spec = dataclasses.replace(spec, render=dataclasses.replace(spec.render, pm_final_gather=True, fg_samples=4))
    full, fw, _ = product.render_spec(spec, members=1)
    rgba, w, _ = product.render_spec(spec, members=2)
    assert _same(w, fw) and _same(rgba, full)


@pytest.mark.parametrize("fault", ["1", "0", "2:1", "0:2"])
def test_device_group_member_failure_ends_every_member(product, monkeypatch, fault):
    """A member that fails (injected: before rendering, or at the start of an adaptive pass) makes
    every member stop at the next status agreement: the render reports the error, nobody waits
    forever, and the next render (no fault) is complete again."""
    spec = scenes.cornell(48, 40, spp=2, bounces=3, rr=False).with_render(aa_passes=3, aa_inc_samples=1, aa_threshold=0.01)
    yi = product.Interface()
    scenes.apply(spec, yi)
    yi.set_device_group(3)
    monkeypatch.setenv("YAFARAY_AMD_FAULT_MEMBER", fault)
    with pytest.raises(RuntimeError, match="failure|failed"):
        yi.render_quiet()
    monkeypatch.delenv("YAFARAY_AMD_FAULT_MEMBER")
    yi.render_quiet()
    a, w = yi.film()
    yi.close()
    full, fw, _ = product.render_spec(spec, members=1)
    assert _same(a, full) and _same(w, fw)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("fault", ["1:concat", "0:concat", "2:concat"])
def test_device_group_photon_concat_failure_ends_every_member(product, monkeypatch, fault):
    """a member that fails after the photon-map counts were exchanged and before the maps
    are concatenated (injected: as if the concatenated map's allocation failed) stops the group at
    the agreement in front of the copies — no member is left waiting inside the concatenation — and
    the next render (no fault) is complete again."""
    spec = scenes.cornell_photon(40, 30, spp=1, photons=20000, search=50, radius=0.1).with_render(pm_final_gather=True, fg_samples=4)
    yi = product.Interface()
    scenes.apply(spec, yi)
    yi.set_device_group(3)
    monkeypatch.setenv("YAFARAY_AMD_FAULT_MEMBER", fault)
    with pytest.raises(RuntimeError, match="failure|failed"):
        yi.render_quiet()
    monkeypatch.delenv("YAFARAY_AMD_FAULT_MEMBER")
    yi.render_quiet()
    a, w = yi.film()
    yi.close()
    full, fw, _ = product.render_spec(spec, members=1)
    assert _same(a, full) and _same(w, fw)


def test_device_group_cancel(product):
    """yafaray_cancelRendering during a group render: every member stops at its next chunk, the
    members still combine, and every pixel is either complete or empty (as a canceled one-GPU
    render, test_cancel.py)."""
    W, H, spp = 64, 48, 8
    spec = scenes.cornell(W, H, spp=spp, bounces=3, rr=False)
    full, fw, _ = product.render_spec(spec, members=1)
    yi = product.Interface()
    scenes.apply(spec, yi)
    yi.set_device_group(2)
    yi.L.yafaray_amd_setChunkSlots(yi.h, 2048)
    calls = []

    def progress(total, done):
        calls.append(done)
        if done > 0:
            yi.cancelRendering()
    yi.render(progress=progress)
    a, w = yi.film()
    st = yi.stats()
    yi.close()
    assert 0 < st["samples"] < W * H * spp
    # box filter: positive weights, so a pixel has the full weight exactly when all its splat sources
    # were rendered — then it equals the uncanceled film; a pixel without any source is empty
    complete = w == fw
    assert complete.any() and not complete.all()
    assert (w <= fw).all()
    assert _same(a[complete], full[complete])
    assert (a[w == 0] == 0).all()


def _ulp(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7fffffff), a)
    b = np.where(b < 0, -(b & 0x7fffffff), b)
    return np.abs(a - b)


def _specular_photon_spec(integrator, **kw):
    s = scenes.cornell_specular(48, 36, spp=1, integrator=integrator, raydepth=3)
    r = dataclasses.replace(s.render, pm_caustic_photons=20000, caustic_radius=kw.pop("radius", 0.1), **kw)
    if integrator == "photonmapping":
        r = dataclasses.replace(r, pm_photons=20000, pm_search=50, pm_diffuse_radius=0.1, pm_bounces=5)
    return dataclasses.replace(s, render=r)


SHARDED_PHOTONS = {
    "dl-caustics": lambda: _specular_photon_spec("directlighting", pm_caustics=True, caustic_search=40),
    "pm-caustics": lambda: _specular_photon_spec("photonmapping", pm_caustics=True, radius=0.05),
    "pm-final-gather": lambda: dataclasses.replace(
        scenes.cornell_photon(40, 30, spp=1, photons=20000, search=50, radius=0.1),
        render=dataclasses.replace(scenes.cornell_photon(40, 30, spp=1, photons=20000, search=50, radius=0.1).render,
                                   pm_final_gather=True, fg_samples=4)),
}


@pytest.mark.parametrize("members", [2, 3, 8])
@pytest.mark.parametrize("case", list(SHARDED_PHOTONS))
def test_device_group_sharded_photon_maps_match_oracle(product, oracle_built, case, members):
    """Photon shooting split across the members (contiguous photon-id ranges, the reference threads'
    split, integrator_photon_mapping.cc:118-127, 437-441), the maps concatenated in member order and
    their point kd-trees built distributed (r06): the same maps (counts) and film as the oracle's
    one-thread shooting."""
    spec = SHARDED_PHOTONS[case]()
    rgba, w, st = product.render_spec(spec, members=members)
    o = oracle_built.OracleScene(spec, threads=8)
    orgba, ow, _ = o.render()
    assert np.array_equal(w, ow)
    u = _ulp(rgba, orgba)
    assert u.max() <= 4, f"{(u > 4).sum()} values > 4 ULP"
    if spec.render.pm_caustics:
        assert st["caustic_photons"] == len(o.photon_map("caustic")[0]) > 0
    if spec.render.integrator == "photonmapping":
        assert st["photons"] == len(o.photon_map("diffuse")[0])
    # the maps' point kd-trees were built distributed: each member its own subtrees below level
    # ceil(log2 members), exchanged (pkd.hip yafamd_build_pkd_kd_member, render.cc exchangeTree)
    def split_level(n):
        d = int(np.ceil(np.log2(members)))
        for _ in range(d):
            if n <= 256:
                return 0
            n = (n + 1) // 2
        return d
    assert st["pkd_split_level"] == max(split_level(st["photons"]), split_level(st["caustic_photons"]))
    if st["photons"] > 2048:
        assert st["pkd_split_level"] > 0
