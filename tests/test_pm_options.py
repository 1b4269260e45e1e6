"""PhotonIntegrator options beyond the estimates (integrator_photon_mapping.cc factory :765-850):

* show_map (:876-881 with final gathering, :924-929 without): a camera hit shows the colour of the
  nearest photon facing its shading normal — the radiance map within lookup_rad_ (4 r^4), or the
  diffuse map within ds_radius_ — after its emission, plus the caustics and the specular recursion;
* do_AO: only the ambient-occlusion render layers read it (generateOcclusionLayers, :991-995); the
  combined image is unchanged (integrate never calls sampleAmbientOcclusion).

GPU (k_gather's G_SHOWMAP requests, pkNearest) against the oracle's restatement, <= 4 ULP."""
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


def _spec(fg=False, show=True, specular=False, caustics=False, **kw):
    if specular:
        s = scenes.cornell_specular(48, 36, spp=1, integrator="photonmapping", raydepth=3)
        s = dataclasses.replace(s, render=dataclasses.replace(s.render, pm_photons=20000, pm_search=50, pm_diffuse_radius=0.1,
                                                              pm_bounces=5, pm_caustics=caustics, pm_caustic_photons=20000,
                                                              caustic_radius=0.05))
    else:
        s = scenes.cornell_photon(48, 36, spp=1, photons=20000, search=50, radius=0.1)
    r = dataclasses.replace(s.render, pm_final_gather=fg, fg_samples=4, pm_show_map=show, **kw)
    return dataclasses.replace(s, render=r)


def test_oracle_show_map_differs_and_is_deterministic(oracle_built):
    a, wa, _ = oracle_built.OracleScene(_spec(), threads=4).render()
    b, _, _ = oracle_built.OracleScene(_spec(), threads=2).render()
    c, _, _ = oracle_built.OracleScene(_spec(show=False), threads=4).render()
    assert np.array_equal(a, b) and (wa > 0).all()
    assert np.isfinite(a).all() and (a[..., :3] > 0).mean() > 0.5
    assert not np.array_equal(a, c)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(), dict(fg=True), dict(specular=True, caustics=True), dict(specular=True, fg=True)],
                         ids=["diffuse-map", "radiance-map", "caustics-specular", "fg-specular"])
def test_show_map_matches_oracle(product, oracle_built, kw):
    spec = _spec(**kw)
    rgba, w, _ = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w, ow)
    d = _ulp(rgba, orgba)
    assert d.max() <= 4, f"{(d > 4).sum()} values > 4 ULP"


@pytest.mark.gpu
def test_show_map_device_group(product):
    spec = _spec(fg=True)
    a, w, _ = product.render_spec(spec, members=1)
    b, wb, _ = product.render_spec(spec, members=3)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(w, wb)


@pytest.mark.gpu
def test_photon_do_ao_leaves_the_combined_image(product):
    base = _spec(show=False)
    a, _, _ = product.render_spec(base)
    b, _, _ = product.render_spec(dataclasses.replace(base, render=dataclasses.replace(base.render, pm_do_ao=True)))
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
