"""Scenes with several lights (the configs have one; the reference takes any number).

* DirectLightIntegrator and the first vertex of PathIntegrator sum every light
  (estimateAllDirectLight, integrator_montecarlo.cc:54-68, lights in name order): bit-exact against
  the oracle (<= 4 ULP, 0 observed).
* Later path vertices and final gathering call estimateOneDirectLight (:70-78): ONE light, picked by
  Halton(2, base_sampling_offset + n - 1) with n a per-thread running counter
  (integrator_tiled.cc:48, :169-171) — schedule-dependent in the reference itself.  The GPU's pick
  (kernels.hip pickLight: the pixel's sampling offset and sample number mixed into an odd stride, so
  every light takes its 1 / num_lights share at every depth) is matched statistically against the
  oracle's per-thread counter: the paired global z of the difference image within 4 and no 8x8
  block beyond 6 (oracle/stats.py), for two seeds, area + point lights.  A counter that is the same
  for every sample (the r03 GPU pick) fails this test: it picks one light per depth for the whole
  film."""
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
    """The Cornell box with n lights: its area light, a warm point bulb and a second (smaller,
    bluish) area light off-centre under the ceiling."""
    extra = [scenes.Light("bulb", type="pointlight", color=(1.0, 0.85, 0.7), power=1.2, from_=(0.45, -0.3, 1.5)),
             scenes.Light("panel", type="arealight", color=(0.6, 0.7, 1.0), power=2.5, corner=(-0.8, 0.5, 1.9),
                          point1=(-0.8, 0.8, 1.9), point2=(-0.5, 0.5, 1.9), samples=1)]
    return dataclasses.replace(spec, lights=spec.lights + extra[:n - 1])


@pytest.mark.parametrize("n", [2, 3])
def test_direct_light_all_lights_bitexact(product, oracle_built, n):
    spec = with_lights(scenes.cornell(96, 72, spp=4, integrator="directlighting"), n)
    rgba, w, _ = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w, ow)
    u = _ulp(rgba, orgba)
    assert u.max() <= 4, f"{(u > 4).sum()} values > 4 ULP"


@pytest.mark.parametrize("n", [2, 3])
@pytest.mark.parametrize("seed", [0, 7919])
def test_path_multi_light_statistical(product, oracle_built, n, seed):
    from oracle.stats import paired_z
    spec = with_lights(scenes.cornell(256, 256, spp=64, bounces=8, rr=True), n).with_render(rr_seed=seed)
    rgba, w, _ = product.render_spec(spec)
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
