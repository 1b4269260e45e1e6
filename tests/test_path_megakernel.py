"""k_path (the megakernel form of the integrator for LDS-resident scenes, kernels.hip) against the
wavefront pipeline (k_camera -> [k_trace -> k_shade -> k_nee] x iterations) on the same scenes: the
films must be bit-identical — both run the same per-sample functions in the same order, only the
place the path state lives differs (registers vs HBM queues).  k_path is opt-in
(YAFARAY_AMD_PATH=mega; slower than the wavefront on C2), the wavefront the default.
The wavefront itself is pinned to the oracle by the other GPU tests; one case here also checks
k_path against the oracle directly."""
import dataclasses
import os

import numpy as np
import pytest

from libyafaray_amd import scenes


@pytest.fixture(autouse=True)
def _needs_experiments(experiments):
    """k_path and k_nee<TR> are compiled only into -DYAF_EXPERIMENTS builds (measured slower)."""


def _render(product, spec, wavefront, chunk=None):
    old = os.environ.get("YAFARAY_AMD_PATH")
    try:
        os.environ["YAFARAY_AMD_PATH"] = "wavefront" if wavefront else "mega"
        return product.render_spec(spec, chunk_slots=chunk, profile=True)
    finally:
        if old is None:
            os.environ.pop("YAFARAY_AMD_PATH", None)
        else:
            os.environ["YAFARAY_AMD_PATH"] = old


def _with_render(spec, **kw):
    return dataclasses.replace(spec, render=dataclasses.replace(spec.render, **kw))


def _cases():
    base = scenes.cornell(96, 64, spp=4, bounces=5, rr=True)
    two_lights = dataclasses.replace(
        base, lights=base.lights + [scenes.Light("bulb", type="pointlight", color=(1.0, 0.9, 0.8), power=1.5, from_=(0.3, -0.2, 1.6))])
    emissive = dataclasses.replace(base, materials=base.materials[:1] + [dataclasses.replace(base.materials[1], emit=0.4)] + base.materials[2:])
    dof = dataclasses.replace(base, camera=dataclasses.replace(base.camera, aperture=0.05, dof_distance=3.5, bokeh_type="hexagon"))
    return {
        "pt_rr_box": (base, None),
        "pt_rr_gauss_chunks": (scenes.cornell(96, 64, spp=4, bounces=5, rr=True, filter_type="gauss", pixelwidth=1.5), 5000),
        "pt_norr_paths2_lsamples2": (_with_render(scenes.cornell(64, 48, spp=2, bounces=4, light_samples=2), path_samples=2), None),
        "direct_light": (scenes.cornell(96, 64, spp=4, integrator="directlighting"), None),
        "direct_light_two_lights": (_with_render(two_lights, integrator="directlighting"), None),
        "pt_two_lights": (two_lights, None),
        "pt_emissive_background": (dataclasses.replace(emissive, background=scenes.Background((0.2, 0.3, 0.4), 1.0)), None),
        "pt_bg_transparent": (_with_render(base, bg_transp=True), None),
        "pt_adaptive_passes": (_with_render(base, aa_passes=3, aa_inc_samples=2, aa_threshold=0.02, aa_detect_color_noise=True), None),
        "pt_dof": (dof, None),
        "pt_crop": (_with_render(base, xstart=16, ystart=8), None),
    }


CASES = _cases()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_path_megakernel_equals_wavefront(product, name):
    spec, chunk = CASES[name]
    a, w, st = _render(product, spec, wavefront=False, chunk=chunk)
    b, wb, stb = _render(product, spec, wavefront=True, chunk=chunk)
    if name == "pt_two_lights":
        # several lights under path tracing pick their light from the one-thread counter, whose count
        # run the wavefront provides (render.cc lpcBases): the megakernel steps aside
        assert st["kernel_times"].get("k_path", {}).get("launches", 0) == 0
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
        return
    assert "k_path" in st["kernel_times"] and st["kernel_times"]["k_path"]["launches"] > 0, st["kernel_times"].keys()
    assert stb["kernel_times"].get("k_path", {}).get("launches", 0) == 0
    assert "k_shade" not in st["kernel_times"] or st["kernel_times"]["k_shade"]["launches"] == 0
    assert np.array_equal(w.view(np.uint32), wb.view(np.uint32))
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), np.argwhere(a.view(np.uint32) != b.view(np.uint32))[:5]
    # the same rays were traced (closest + shadow counted in-kernel)
    assert st["closest_rays"] == stb["closest_rays"] and st["shadow_rays"] == stb["shadow_rays"]


@pytest.mark.gpu
def test_path_megakernel_matches_oracle(product, oracle_built):
    """RR off: every pixel within 4 ULP of the CPU restatement (0 observed for the wavefront)."""
    spec = scenes.cornell(80, 60, spp=8, bounces=5, rr=False, filter_type="gauss", pixelwidth=1.5)
    a, w, st = _render(product, spec, wavefront=False)
    assert st["kernel_times"]["k_path"]["launches"] > 0
    ref, wref, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w, wref)
    ulp = np.abs(a.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulp.max() <= 4, ulp.max()


@pytest.mark.gpu
def test_path_megakernel_not_used_where_ineligible(product):
    """Transparent shadows and photon maps keep the wavefront even when k_path is asked for (their
    stages have no k_path form); without the opt-in every scene renders through the wavefront."""
    spec = scenes.cornell_transparent_shadows(48, 32, spp=2)
    _, _, st = _render(product, spec, wavefront=False)
    assert st["kernel_times"].get("k_path", {}).get("launches", 0) == 0
    assert st["kernel_times"]["k_shade"]["launches"] > 0
    os.environ.pop("YAFARAY_AMD_PATH", None)
    _, _, st = product.render_spec(scenes.cornell(32, 24, spp=2, bounces=3), profile=True)
    assert st["kernel_times"].get("k_path", {}).get("launches", 0) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["pt_rr_gauss_chunks", "pt_norr_paths2_lsamples2", "direct_light_two_lights", "pt_two_lights"])
def test_nee_inplace_shadow_rays_equal_queued(product, name):
    """k_nee<.., TR> (opt-in YAFARAY_AMD_NEE_TRACE=1): the lane that sampled a light traces its shadow
    rays in place instead of queueing them for k_trace — same occlusion, same film bits, same ray
    counts."""
    spec, chunk = CASES[name]
    old = os.environ.get("YAFARAY_AMD_NEE_TRACE")
    try:
        os.environ["YAFARAY_AMD_NEE_TRACE"] = "1"
        a, w, st = product.render_spec(spec, chunk_slots=chunk, profile=True)
        os.environ["YAFARAY_AMD_NEE_TRACE"] = "0"
        b, wb, stb = product.render_spec(spec, chunk_slots=chunk, profile=True)
    finally:
        if old is None:
            os.environ.pop("YAFARAY_AMD_NEE_TRACE", None)
        else:
            os.environ["YAFARAY_AMD_NEE_TRACE"] = old
    assert np.array_equal(w.view(np.uint32), wb.view(np.uint32))
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert st["closest_rays"] == stb["closest_rays"] and st["shadow_rays"] == stb["shadow_rays"]
