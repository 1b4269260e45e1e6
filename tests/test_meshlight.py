"""meshlight / objectlight (src/light/light_object_light.cc, factory src/light/light.cc:48): a light
whose shape is a mesh object.  Its faces are sampled by area (sampleSurface :89-107: Pdf1D over the
face areas, TrianglePrimitive::sample), illumSample (:111-146) gives the pdf with the reference's
1e-8 guard, the MIS material sample hits the light's own faces (intersect :183-201 — which never
stores the hit distance, so the pdf uses the caller's t = -1 and the shadow ray is unbounded, both
reproduced), photons leave from sampled faces (emitPhoton :148-163), and the photon light pick
weighs it by color * area (x 2 double-sided, :109).

Checked against the oracle's restatement (oracle/yafcpu.cc meshSampleSurface / meshIllumSample /
meshIntersect): DirectLight and PathIntegrator (Russian roulette off) within 4 ULP (0 expected), a
single-sided panel and a double-sided 72-face sphere, alone and next to the box's area light (two
lights: the one-thread light-pick counter); the PhotonIntegrator's photon map (counts) and image,
with and without final gathering; a 10082-face double-sided sphere through the light's BVH2.  Parity is pinned by the restatement only (no
reference golden images)."""
import dataclasses

import numpy as np
import pytest

from libyafaray_amd import scenes


def _ulp(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7fffffff), a)
    b = np.where(b < 0, -(b & 0x7fffffff), b)
    return np.abs(a - b)


def test_oracle_meshlight_energy_scales_with_power(oracle_built):
    """CPU: the restatement's image is linear in the meshlight's power (DirectLight, RR-free)."""
    a, _, _ = oracle_built.OracleScene(scenes.cornell_meshlight(32, 24, spp=1, integrator="directlighting", power=2.0), threads=4).render()
    b, _, _ = oracle_built.OracleScene(scenes.cornell_meshlight(32, 24, spp=1, integrator="directlighting", power=4.0), threads=4).render()
    assert np.isfinite(a).all() and a[..., :3].mean() > 0.0
    np.testing.assert_allclose(b[..., :3], 2.0 * a[..., :3], rtol=1e-5, atol=1e-6)


CASES = {
    "dl-panel": dict(integrator="directlighting", shape="panel"),
    "dl-sphere-2sided": dict(integrator="directlighting", shape="sphere", double_sided=True),
    "pt-panel": dict(integrator="pathtracing", shape="panel"),
    "pt-sphere-2sided": dict(integrator="pathtracing", shape="sphere", double_sided=True, samples=3),
    "pt-sphere-and-area": dict(integrator="pathtracing", shape="sphere", keep_area=True),
    "dl-panel-and-area": dict(integrator="directlighting", shape="panel", keep_area=True),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(CASES))
def test_meshlight_matches_oracle(product, oracle_built, case):
    spec = scenes.cornell_meshlight(80, 60, spp=4, bounces=4, rr=False, **CASES[case])
    rgba, w, st = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=1).render()
    assert np.array_equal(w, ow)
    u = _ulp(rgba, orgba)
    assert u.max() <= 4, f"{(u > 4).sum()} values > 4 ULP"
    assert rgba[..., :3].mean() > 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("fg", [False, True])
def test_meshlight_photon_mapping_matches_oracle(product, oracle_built, fg):
    spec = scenes.cornell_meshlight(48, 36, spp=1, integrator="photonmapping", shape="sphere", double_sided=True)
    spec = spec.with_render(pm_photons=20000, pm_search=50, pm_diffuse_radius=0.1, pm_bounces=5, pm_final_gather=fg, fg_samples=4)
    rgba, w, st = product.render_spec(spec)
    o = oracle_built.OracleScene(spec, threads=8)
    orgba, ow, _ = o.render()
    assert st["photons"] == len(o.photon_map("diffuse")[0]) > 0
    assert np.array_equal(w, ow)
    u = _ulp(rgba, orgba)
    assert u.max() <= 4, f"{(u > 4).sum()} values > 4 ULP"


BIG = {
    "dl-bigsphere-2sided": dict(integrator="directlighting", double_sided=True),
    "pt-bigsphere-2sided-and-area": dict(integrator="pathtracing", double_sided=True, keep_area=True),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(BIG))
def test_meshlight_bvh_10k_faces_matches_oracle(product, oracle_built, monkeypatch, case):
    """A 10082-face double-sided meshlight: the material-sampled rays find the closest face through the
    light's BVH2 (the oracle tests every face, as the reference's kd-tree answers); within 4 ULP of the
    oracle, and bit-identical to the per-face loop (YAFARAY_AMD_MESHLIGHT_BVH=0)."""
    spec = scenes.cornell_meshlight(48, 36, spp=2, bounces=3, rr=False, shape="bigsphere", **BIG[case])
    assert spec.objects[-1].nt > 10000
    rgba, w, st = product.render_spec(spec)
    # one oracle thread: with two lights the path tracer's light pick is the one-thread counter
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=1).render()
    assert np.array_equal(w, ow)
    u = _ulp(rgba, orgba)
    assert u.max() <= 4, f"{(u > 4).sum()} values > 4 ULP"
    assert rgba[..., :3].mean() > 0.0
    monkeypatch.setenv("YAFARAY_AMD_MESHLIGHT_BVH", "0")
    lin, lw, _ = product.render_spec(spec)
    assert np.array_equal(lin.view(np.uint32), rgba.view(np.uint32)) and np.array_equal(lw, w)


@pytest.mark.gpu
def test_meshlight_missing_object_fails_loudly(product):
    spec = scenes.cornell_meshlight(32, 24, spp=1, integrator="directlighting")
    spec = dataclasses.replace(spec, lights=[dataclasses.replace(spec.lights[0], object_name="no_such_object")])
    with pytest.raises(RuntimeError, match="not found"):
        product.render_spec(spec)
