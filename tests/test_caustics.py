"""Caustic photon map: MonteCarloIntegrator::createCausticMap / causticWorker
(integrator_montecarlo.cc:421-625) shot on the GPU and estimated by k_gather
(estimateCausticPhotons :627-648 via causticPhotons :410-419), for the three integrators that use it:

  * PhotonIntegrator "caustics" (default on; cPhotons, causticRadius, caustic_mix, caus_depth = bounces)
    — integrate() adds it at diffuse hits (integrator_photon_mapping.cc:980-984), and specular
    materials recurse through recursiveRaytrace (:986), at whose nodes the diffuse map and the
    caustic map are gathered again;
  * DirectLight "caustics" (photons, caustic_mix, caustic_depth, caustic_radius), between the direct
    light and the AO (integrator_direct_light.cc:120-124);
  * PathIntegrator caustic_type photon | both (integrator_path_tracer.cc:149-152).

Scene: the C2 Cornell box with a mirror-and-diffuse tall box, a transparent short box and a mirror
back wall (scenes.cornell_specular), so caustic paths exist.  Tolerance as the other photon-map
tests: per value <= 4 ULP of the oracle (no Russian roulette); weights equal; the caustic map's
photon count equal to the oracle's.
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


def spec_for(integrator, photons=20000, radius=0.1, search=None, depth=None, raydepth=3, W=48, H=36, spp=1, **kw):
    s = scenes.cornell_specular(W, H, spp=spp, integrator=integrator, raydepth=raydepth)
    r = dataclasses.replace(s.render, pm_caustic_photons=photons, caustic_radius=radius, caustic_search=search,
                            caustic_depth=depth, **kw)
    if integrator == "photonmapping":
        r = dataclasses.replace(r, pm_photons=kw.get("pm_photons", 20000), pm_search=50, pm_diffuse_radius=0.1, pm_bounces=5)
    return dataclasses.replace(s, render=r)


def compare(product, oracle_built, spec, chunk_slots=None):
    rgba, w, st = product.render_spec(spec, chunk_slots=chunk_slots)
    o = oracle_built.OracleScene(spec, threads=8)
    orgba, ow, _ = o.render()
    assert np.array_equal(w, ow), "film weights differ"
    u = ulp_diff(rgba, orgba)
    assert u.max() <= ULP_TOL, (f"{(u > ULP_TOL).sum()} values > {ULP_TOL} ULP, max {u.max()} at "
                                f"{np.unravel_index(u.argmax(), u.shape)}: {rgba.reshape(-1)[u.argmax()]} vs {orgba.reshape(-1)[u.argmax()]}")
    return rgba, st, o


# ---------------------------------------------------------------------------------------------
# CPU: the oracle restatement
# ---------------------------------------------------------------------------------------------
def test_oracle_caustic_map_contents(oracle_built):
    o = oracle_built.OracleScene(spec_for("directlighting", pm_caustics=True), threads=4)
    pos, d, col, nodes, n_paths = o.photon_map("caustic")
    assert n_paths == 20000
    assert 0 < len(pos) < n_paths
    assert np.isfinite(pos).all() and (col >= 0).all() and np.isfinite(col).all()
    assert np.allclose(np.linalg.norm(d, axis=1), 1.0, atol=1e-3)   # fast-math normalisations
    assert len(nodes) == 2 * len(pos) - 1
    # a plain Cornell box has no specular paths: the map stays empty
    plain = scenes.cornell(32, 24, spp=1, integrator="directlighting")
    plain = dataclasses.replace(plain, render=dataclasses.replace(plain.render, pm_caustics=True, pm_caustic_photons=5000))
    pos0, *_ = oracle_built.OracleScene(plain, threads=4).photon_map("caustic")
    assert len(pos0) == 0


def test_oracle_caustic_lights_flag(oracle_built):
    s = spec_for("directlighting", pm_caustics=True)
    s = dataclasses.replace(s, lights=[dataclasses.replace(l, with_caustic=False) for l in s.lights])
    pos, *_ = oracle_built.OracleScene(s, threads=4).photon_map("caustic")
    assert len(pos) == 0


@pytest.mark.parametrize("integrator,kw", [("directlighting", dict(pm_caustics=True)),
                                           ("pathtracing", dict(caustic_type="photon", bounces=3, rr_min_bounces=3)),
                                           ("photonmapping", dict(pm_caustics=True))])
def test_oracle_caustics_add_light(oracle_built, integrator, kw):
    on = spec_for(integrator, **kw)
    off_kw = dict(kw, pm_caustics=False) if "pm_caustics" in kw else dict(kw, caustic_type="none")
    off = spec_for(integrator, **off_kw)
    a, wa, _ = oracle_built.OracleScene(on, threads=4).render()
    b, wb, _ = oracle_built.OracleScene(off, threads=4).render()
    assert np.isfinite(a).all() and np.array_equal(wa, wb)
    assert (a[..., :3] >= b[..., :3] - 1e-6).all() and (a - b).max() > 1e-3


# ---------------------------------------------------------------------------------------------
# GPU parity
# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("ao", [False, True])
def test_directlight_caustics_match_oracle(product, oracle_built, ao):
    s = spec_for("directlighting", pm_caustics=True, search=40)
    if ao:
        s = s.with_render(do_ao=True, ao_samples=4, ao_distance=0.8)
    _, st, o = compare(product, oracle_built, s)
    pos, *_ = o.photon_map("caustic")
    assert st["caustic_photons"] == len(pos) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("ctype", ["photon", "both"])
def test_pathtracing_photon_caustics_match_oracle(product, oracle_built, ctype):
    s = spec_for("pathtracing", caustic_type=ctype, bounces=3, rr_min_bounces=3, path_samples=2, radius=0.15)
    _, st, o = compare(product, oracle_built, s)
    pos, *_ = o.photon_map("caustic")
    assert st["caustic_photons"] == len(pos)


@pytest.mark.gpu
@pytest.mark.parametrize("caustics", [False, True])
def test_photon_mapping_specular_matches_oracle(product, oracle_built, caustics):
    """PhotonIntegrator with specular materials: recursiveRaytrace nodes gather the diffuse map (and
    the caustic map) again — the refusal of round 1 is lifted."""
    s = spec_for("photonmapping", pm_caustics=caustics, radius=0.05)
    _, st, o = compare(product, oracle_built, s)
    pos, *_ = o.photon_map("caustic")
    assert st["caustic_photons"] == (len(pos) if caustics else 0)
    dpos, *_ = o.photon_map("diffuse")
    assert st["photons"] == len(dpos)


@pytest.mark.gpu
def test_caustics_depth_and_several_chunks(product, oracle_built):
    """caustic_depth 1 (a single specular bounce), k = 12, a small chunk so that gathers run for
    several wavefront chunks."""
    s = spec_for("directlighting", pm_caustics=True, depth=1, search=12, radius=0.2, W=40, H=30, spp=2)
    compare(product, oracle_built, s, chunk_slots=1200)
