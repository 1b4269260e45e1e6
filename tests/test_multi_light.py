"""Scenes with several lights (the configs have one; the reference takes any number).

* DirectLightIntegrator and the first vertex of PathIntegrator sum every light
  (estimateAllDirectLight, integrator_montecarlo.cc:54-68, lights in name order): bit-exact against
  the oracle (<= 4 ULP, 0 observed).
* Later path vertices call estimateOneDirectLight (:70-78): ONE light, picked by
  Halton(2, base_sampling_offset + n - 1) with n a running counter of the calls
  (integrator_tiled.cc:48, reset at render start :169-171).  The reference keeps one counter per
  render thread, so n depends on the thread schedule; with one thread it is the number of calls of
  every sample rendered before.  The GPU reproduces the one-thread counter exactly: a count run
  follows every path (closest rays and shading only), an exclusive scan in tile order gives each
  sample its first counter value (render.cc lpcBases), and the render proper takes consecutive values
  — so Russian roulette off, the image is bit-identical to the one-thread oracle, on one GPU, with
  adaptive passes and in a device group.  With RR on (RR streams are statistical by design) the
  image is compared with the 16-thread oracle (per-thread counters) by the paired z test.
* Final gathering (integrator_photon_mapping.cc:703) and specular recursion trees keep a pick
  that mixes the pixel and sample into the counter (kernels.hip pickLight): matched statistically.
"""
import dataclasses

import numpy as np
import pytest

from libyafaray_amd import scenes

pytestmark = pytest.mark.gpu


def _ulp(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7fffffff), a)
    b = np.where(b < 0, -(b & 0x7fffffff), b)
    return np.abs(a - b)


def with_lights(spec, n):
    """The Cornell box with n lights (scenes.with_extra_lights: its area light, a warm point bulb and a
    second, smaller, bluish area light off-centre under the ceiling)."""
    return scenes.with_extra_lights(spec, n)


@pytest.mark.parametrize("n", [2, 3])
def test_direct_light_all_lights_bitexact(product, oracle_built, n):
    spec = with_lights(scenes.cornell(96, 72, spp=4, integrator="directlighting"), n)
    rgba, w, _ = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w, ow)
    u = _ulp(rgba, orgba)
    assert u.max() <= 4, f"{(u > 4).sum()} values > 4 ULP"


EXACT = {
    "2-lights": lambda: with_lights(scenes.cornell(96, 72, spp=4, bounces=5, rr=False), 2),
    "3-lights-paths2": lambda: with_lights(scenes.cornell(80, 64, spp=2, bounces=4, rr=False), 3).with_render(path_samples=2),
    "3-lights-adaptive": lambda: with_lights(scenes.cornell(64, 48, spp=2, bounces=4, rr=False), 3).with_render(
        aa_passes=3, aa_inc_samples=2, aa_threshold=0.01),
    "2-lights-centre-order": lambda: with_lights(scenes.cornell(96, 72, spp=2, bounces=4, rr=False, tile_size=16), 2).with_render(
        tiles_order="centre"),
}


@pytest.mark.parametrize("case", list(EXACT))
@pytest.mark.parametrize("members", [1, 3])
def test_path_multi_light_one_thread_order_bitexact(product, oracle_built, case, members):
    spec = EXACT[case]()
    rgba, w, st = product.render_spec(spec, members=members, chunk_slots=4096)
    orgba, ow, octr = oracle_built.OracleScene(spec, threads=1).render()
    assert np.array_equal(w, ow)
    u = _ulp(rgba, orgba)
    assert u.max() <= 4, f"{(u > 4).sum()} values > 4 ULP"


def test_path_multi_light_hash_pick_is_not_the_reference_order(product, oracle_built, monkeypatch):
    """YAFARAY_AMD_LIGHT_PICK=hash (pickLight) renders a different image (the counter matters)."""
    spec = EXACT["2-lights"]()
    monkeypatch.setenv("YAFARAY_AMD_LIGHT_PICK", "hash")
    rgba, _, _ = product.render_spec(spec)
    monkeypatch.delenv("YAFARAY_AMD_LIGHT_PICK")
    orgba, _, _ = oracle_built.OracleScene(spec, threads=1).render()
    assert _ulp(rgba, orgba).max() > 4


@pytest.mark.parametrize("pick", ["counter", "hash"])
@pytest.mark.parametrize("n", [2, 3])
@pytest.mark.parametrize("seed", [0, 7919])
def test_path_multi_light_statistical(product, oracle_built, n, seed, pick, monkeypatch):
    """pick "hash": the fallback pick (recursion trees, final gathering) must be unbiased too."""
    from oracle.stats import paired_z
    spec = with_lights(scenes.cornell(256, 256, spp=64, bounces=8, rr=True), n).with_render(rr_seed=seed)
    if pick == "hash":
        monkeypatch.setenv("YAFARAY_AMD_LIGHT_PICK", "hash")
    rgba, w, _ = product.render_spec(spec)
    monkeypatch.delenv("YAFARAY_AMD_LIGHT_PICK", raising=False)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=16, rr_seed=seed).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    z = paired_z(rgba, orgba)
    assert abs(z["mean_z"]) < 4.0, z
    assert z["max_abs_block_z"] < 6.0, z
    assert abs(z["mean_rel_diff"]) < 0.01, z


def test_final_gather_two_lights_statistical(product, oracle_built):
    """PhotonIntegrator with final gathering: the gather paths' estimateOneDirectLight
    (integrator_photon_mapping.cc:703) picks between two lights; photons are emitted from both
    (Pdf1D over the lights' power)."""
    from oracle.stats import paired_z
    spec = scenes.cornell_photon(128, 96, spp=4, photons=200000, search=50, radius=0.1)
    spec = with_lights(spec, 2).with_render(pm_final_gather=True, fg_samples=16)
    rgba, w, st = product.render_spec(spec)
    o = oracle_built.OracleScene(spec, threads=16)
    orgba, ow, _ = o.render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    assert st["photons"] == len(o.photon_map("diffuse")[0])
    z = paired_z(rgba, orgba)
    assert abs(z["mean_z"]) < 4.0, z
    assert z["max_abs_block_z"] < 6.0, z


@pytest.mark.parametrize("members", [1, 3])
def test_light_pick_counters_over_budget_fall_back_to_hash(product, members, monkeypatch):
    """the one-thread pick's per-sample counters (4 B per camera sample of a pass) that do
    not fit the memory budget make the pass fall back to the hashed pick instead of failing the render
    (YAFARAY_AMD_LPC_MAX_MB forces it here): the image equals the YAFARAY_AMD_LIGHT_PICK=hash render bit
    for bit, on one GPU and in a device group (whose members agree on the fallback)."""
    spec = EXACT["2-lights"]()
    monkeypatch.setenv("YAFARAY_AMD_LPC_MAX_MB", "0")
    a, wa, _ = product.render_spec(spec, members=members)
    monkeypatch.delenv("YAFARAY_AMD_LPC_MAX_MB")
    monkeypatch.setenv("YAFARAY_AMD_LIGHT_PICK", "hash")
    b, wb, _ = product.render_spec(spec, members=members)
    assert np.array_equal(wa, wb)
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


@pytest.mark.parametrize("case", ["3-lights-adaptive", "dl-3-lights", "dl-specular-tree"])
def test_nee_request_word_packing(product, oracle_built, case, monkeypatch):
    """k_shade packs each NEE request's (pixel offset, sample index, mode, light) word into 8 B
    (kernels.hip neePmStore: the sample index relative to the pass's first one); the 16-B form
    (YAFARAY_AMD_NEE_PM16=1, used when a pass has >= 2^20 samples per pixel or > 2^11 lights)
    must render the same image bit for bit, and both equal the one-thread oracle."""
    if case == "3-lights-adaptive":
        spec = EXACT["3-lights-adaptive"]()
    elif case == "dl-3-lights":
        spec = with_lights(scenes.cornell(64, 48, spp=4, integrator="directlighting"), 3)
    else:
        # a specular recursion tree: the spawned nodes' NEE requests carry their sample's index
        spec = with_lights(scenes.cornell_specular(48, 36, spp=2, integrator="directlighting", raydepth=3), 2)
    a, wa, _ = product.render_spec(spec)
    monkeypatch.setenv("YAFARAY_AMD_NEE_PM16", "1")
    b, wb, _ = product.render_spec(spec)
    assert np.array_equal(wa, wb)
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))
    o, wo, _ = oracle_built.OracleScene(spec, threads=1).render()
    assert np.array_equal(wa, wo)
    assert _ulp(a, o).max() <= 4


@pytest.mark.parametrize("case", ["2-lights", "3-lights-paths2", "3-lights-adaptive", "rr-on", "overflow"])
def test_deferred_light_pick_equals_count_run(product, oracle_built, case, monkeypatch):
    """r06: the one-thread light pick without a count run (lpc_mode 3: every addition to a path colour kept
    as a record, the lights picked from the counter bases after the pass, the records folded in order) renders
    the count run's image bit for bit (YAFARAY_AMD_LIGHT_PICK=count), RR on and off, several chunks; a pass
    whose records overflow their budget (YAFARAY_AMD_DFR_CAP) renders again with the count run."""
    if case == "rr-on":
        spec = with_lights(scenes.cornell(96, 72, spp=8, bounces=8, rr=True), 3)
    elif case == "overflow":
        spec = EXACT["2-lights"]()
        monkeypatch.setenv("YAFARAY_AMD_DFR_CAP", "5000")
    else:
        spec = EXACT[case]()
    a, wa, sa = product.render_spec(spec, chunk_slots=4096)
    monkeypatch.delenv("YAFARAY_AMD_DFR_CAP", raising=False)
    monkeypatch.setenv("YAFARAY_AMD_LIGHT_PICK", "count")
    b, wb, sb = product.render_spec(spec, chunk_slots=4096)
    assert np.array_equal(wa, wb)
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32)), int(_ulp(a, b).max())
    if case != "rr-on":
        o, wo, _ = oracle_built.OracleScene(spec, threads=1).render()
        assert _ulp(a, o).max() <= 4
