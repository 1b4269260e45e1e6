"""photon_only lights (Light::photonOnly): render_view.cc:83-91 leaves such a light out of the
integrators' light list (getLightsVisible: no next-event estimation, not counted by
estimateOneDirectLight's pick) while getLightsEmittingDiffusePhotons / ...CausticPhotons (:93-111) keep
it, so it still shoots diffuse and caustic photons; its illumSample refuses anyway (light_area.cc:68,
light_point.cc:40, light_object_light.cc:110).

The photon-only light here is named to sort BEFORE the visible one ("a_bulb" < "area"), so the photon
lists (name order over every light) and the integrators' list (name order over the visible lights)
differ in order as well as in length.  GPU cases: PhotonIntegrator with and without final gathering,
DirectLight with caustic photons, PathIntegrator caustic_type = photon — each within 4 ULP of the
oracle's restatement with equal photon counts (the same bar as the other photon-map tests).
"""
import dataclasses

import numpy as np
import pytest

from libyafaray_amd import scenes

ULP_TOL = 4


def ulp_diff(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7fffffff), a)
    b = np.where(b < 0, -(b & 0x7fffffff), b)
    return np.abs(a - b)


def bulb(photon_only=True, **kw):
    return scenes.Light("a_bulb", type="pointlight", color=(1.0, 0.85, 0.6), power=3.0, from_=(0.3, -0.2, 1.5),
                        photon_only=photon_only, **kw)


def with_bulb(spec, photon_only=True, **kw):
    return dataclasses.replace(spec, lights=list(spec.lights) + [bulb(photon_only, **kw)])


def pm_spec(fg=False, W=48, H=36, photons=20000):
    s = scenes.cornell_photon(W, H, spp=1, photons=photons, search=50, radius=0.1)
    if fg:
        s = s.with_render(pm_final_gather=True, fg_samples=8, fg_bounces=2)
    return with_bulb(s)


def specular_spec(integrator, **kw):
    s = scenes.cornell_specular(48, 36, spp=1, integrator=integrator, raydepth=3)
    r = dataclasses.replace(s.render, pm_caustic_photons=20000, caustic_radius=0.15, **kw)
    return with_bulb(dataclasses.replace(s, render=r))


# ---------------------------------------------------------------------------------------------
# CPU: the oracle restatement
# ---------------------------------------------------------------------------------------------
def test_oracle_photon_only_light_is_invisible_to_the_integrator(oracle_built):
    """DirectLight without photon maps: the photon-only light adds nothing (bit-identical to the scene
    without it); as a normal light it does."""
    base = scenes.cornell(32, 24, spp=2, integrator="directlighting")
    a, wa, _ = oracle_built.OracleScene(base, threads=4).render()
    b, wb, _ = oracle_built.OracleScene(with_bulb(base), threads=4).render()
    c, _, _ = oracle_built.OracleScene(with_bulb(base, photon_only=False), threads=4).render()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(wa, wb)
    assert (c[..., :3] - a[..., :3]).max() > 1e-3


def test_oracle_photon_only_light_shoots_photons(oracle_built):
    """The photon map changes with the photon-only light (the same paths are now shared between two
    lights by energy), and with_diffuse = false on it restores the one-light map."""
    base = scenes.cornell_photon(24, 16, spp=1, photons=4000)
    p0, *_ = oracle_built.OracleScene(base, threads=2).photon_map()
    p1, *_ = oracle_built.OracleScene(with_bulb(base), threads=2).photon_map()
    p2, *_ = oracle_built.OracleScene(with_bulb(base, with_diffuse=False), threads=2).photon_map()
    assert len(p0) != len(p1) or not np.array_equal(p0, p1)
    assert np.array_equal(p0, p2)


# ---------------------------------------------------------------------------------------------
# GPU parity
# ---------------------------------------------------------------------------------------------
def compare(product, oracle_built, spec):
    rgba, w, st = product.render_spec(spec)
    o = oracle_built.OracleScene(spec, threads=8)
    orgba, ow, _ = o.render()
    assert np.array_equal(w, ow), "film weights differ"
    u = ulp_diff(rgba, orgba)
    assert u.max() <= ULP_TOL, (f"{(u > ULP_TOL).sum()} values > {ULP_TOL} ULP, max {u.max()} at "
                                f"{np.unravel_index(u.argmax(), u.shape)}")
    return st, o


@pytest.mark.gpu
@pytest.mark.parametrize("fg", [False, True])
def test_photon_mapping_photon_only_light_matches_oracle(product, oracle_built, fg):
    st, o = compare(product, oracle_built, pm_spec(fg=fg))
    dpos, *_ = o.photon_map("diffuse")
    assert st["photons"] == len(dpos) > 0


@pytest.mark.gpu
def test_directlight_caustics_photon_only_light_matches_oracle(product, oracle_built):
    st, o = compare(product, oracle_built, specular_spec("directlighting", pm_caustics=True))
    cpos, *_ = o.photon_map("caustic")
    assert st["caustic_photons"] == len(cpos) > 0


@pytest.mark.gpu
def test_pathtracing_photon_caustics_photon_only_light_matches_oracle(product, oracle_built):
    st, o = compare(product, oracle_built, specular_spec("pathtracing", caustic_type="photon", bounces=3, rr_min_bounces=3))
    cpos, *_ = o.photon_map("caustic")
    assert st["caustic_photons"] == len(cpos) > 0
