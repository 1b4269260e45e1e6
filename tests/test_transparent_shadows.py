"""Transparent shadows (integrator "transpShad" / "shadowDepth"; MonteCarloIntegrator tr_shad_,
Accelerator::isShadowed with max_depth (accelerator.cc:80-93), AcceleratorKdTree::intersectTs
(accelerator_kdtree.cc:916-1061), ShinyDiffuseMaterial::getTransparency
(material_shiny_diffuse.cc:441-465), `lcol *= scol` in integrator_montecarlo.cc:122, 212, 335).

GPU (k_trace<TS> hit lists + k_tshadow filter colours) against the CPU oracle, per pixel <= 4 ULP
(in practice bit-identical).  Parity note: the reference multiplies the filter colours in its
kd-tree cell order; GPU and oracle both use ascending (t, primitive) order, which gives the same
value as any order for up to two transparent surfaces per shadow ray (a product of two rounded
factors is order-free); with three or more the kd-tree order is a build artefact ("parity
unpinned" beyond the ULP-level order effect).
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


def test_oracle_transparent_shadows_let_light_through(oracle_built):
    """CPU: with transpShad the panes and glass boxes tint the shadows instead of blocking them."""
    spec = scenes.cornell_transparent_shadows(40, 30, spp=1)
    a, w, _ = oracle_built.OracleScene(spec, threads=4).render()
    b, _, _ = oracle_built.OracleScene(spec.with_render(transp_shad=False), threads=4).render()
    assert np.isfinite(a).all() and (w > 0).all()
    assert a[..., :3].mean() > b[..., :3].mean() * 1.1
    assert (a[..., :3] >= b[..., :3] - 1e-6).mean() > 0.99   # light only added, never removed (bar 2 tmin)


def test_oracle_shadow_depth_limits(oracle_built):
    """CPU: shadowDepth 0 shadows at any transparent surface, i.e. the opaque image up to the
    [2 tmin, tmax - tmin) range of intersectTs; a larger depth lets more light through."""
    spec = scenes.cornell_transparent_shadows(40, 30, spp=1)
    d0, _, _ = oracle_built.OracleScene(spec.with_render(shadow_depth=0), threads=4).render()
    d1, _, _ = oracle_built.OracleScene(spec.with_render(shadow_depth=1), threads=4).render()
    d5, _, _ = oracle_built.OracleScene(spec, threads=4).render()
    opq, _, _ = oracle_built.OracleScene(spec.with_render(transp_shad=False), threads=4).render()
    assert (np.abs(d0 - opq).max(-1) > 1e-6).mean() < 0.01
    assert d0[..., :3].mean() < d1[..., :3].mean() < d5[..., :3].mean()


def _compare(product, oracle_built, spec):
    rgba, w, st = product.render_spec(spec)
    orgba, ow, ctr = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w, ow), "film weights differ"
    u = ulp_diff(rgba, orgba)
    assert u.max() <= ULP_TOL, (f"max {u.max()} ULP at {np.unravel_index(u.argmax(), u.shape)}: "
                                f"{rgba.reshape(-1)[u.argmax()]} vs {orgba.reshape(-1)[u.argmax()]}")
    assert st["closest_rays"] == ctr[0], f"closest rays {st['closest_rays']} vs oracle {ctr[0]}"
    assert st["shadow_rays"] == ctr[1], f"shadow rays {st['shadow_rays']} vs oracle {ctr[1]}"
    return rgba


def _smooth_tall_box(spec):
    objs = [dataclasses.replace(o, smooth_angle=80.0) if o.name == "tall_box" else o for o in spec.objects]
    return dataclasses.replace(spec, objects=objs)


CASES = {
    "dl_area_2panes": dict(),
    "dl_area_4panes": dict(panes=4),
    "dl_point": dict(point_light=True),
    "dl_depth0": dict(shadow_depth=0),
    "dl_depth1": dict(shadow_depth=1),
    "dl_depth2_light_samples4": dict(shadow_depth=2, light_samples=4),
    "pt_3panes": dict(panes=3, integrator="pathtracing", bounces=3),
    "pt_point": dict(point_light=True, integrator="pathtracing", bounces=4),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(CASES))
def test_transparent_shadows_match_oracle(product, oracle_built, case):
    _compare(product, oracle_built, scenes.cornell_transparent_shadows(64, 48, spp=2, **CASES[case]))


@pytest.mark.gpu
def test_transparent_shadows_smooth_normals_match_oracle(product, oracle_built):
    """Surface attributes at the shadow hits (interpolated normals drive faceForward / Fresnel in
    getTransparency): k_tshadow runs surfAttr like k_surface."""
    spec = _smooth_tall_box(scenes.cornell_transparent_shadows(64, 48, spp=2, panes=1))
    _compare(product, oracle_built, spec)


@pytest.mark.gpu
def test_transparent_shadows_off_is_unchanged(product, oracle_built):
    """transpShad false keeps the opaque any-hit path (same scene, same oracle)."""
    spec = scenes.cornell_transparent_shadows(64, 48, spp=2).with_render(transp_shad=False)
    _compare(product, oracle_built, spec)


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [70, 100])
def test_deep_shadow_depth_matches_oracle(product, oracle_built, depth):
    """shadowDepth beyond 64 (the reference's intersectTs takes any depth, accelerator_kdtree.cc:916-1061):
    a stack of 72 equally transparent panes under the light, so shadow rays cross up to 72 transparent
    surfaces — with shadowDepth 70 the ones crossing more are shadowed, with 100 all are filtered."""
    spec = scenes.cornell_transparent_shadows(32, 24, spp=1, panes=72, pane_step=0.015, pane_shrink=0.0, pane_alpha=0.97,
                                              shadow_depth=depth)
    _compare(product, oracle_built, spec)


def _pm_fg_spec(**kw):
    """PhotonIntegrator with final gathering over the transparent-shadow Cornell box: close gather
    paths (fg_min_pathlen 0.8) run estimateOneDirectLight (integrator_photon_mapping.cc:703), whose
    shadow rays take the transparent-shadow test (integrator_montecarlo.cc:112, 206, 330)."""
    spec = scenes.cornell_transparent_shadows(48, 36, spp=1, integrator="photonmapping", **kw)
    return spec.with_render(pm_photons=20000, pm_search=50, pm_diffuse_radius=0.1, pm_bounces=5, pm_caustics=False,
                            pm_final_gather=True, fg_samples=4, fg_bounces=3, fg_min_pathlen=0.8)


def test_oracle_final_gather_transparent_shadows_add_light(oracle_built):
    a, w, _ = oracle_built.OracleScene(_pm_fg_spec(), threads=4).render()
    b, _, _ = oracle_built.OracleScene(_pm_fg_spec().with_render(transp_shad=False), threads=4).render()
    assert np.isfinite(a).all() and (w > 0).all()
    assert a[..., :3].mean() > b[..., :3].mean()


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(), dict(point_light=True), dict(shadow_depth=1, panes=3)], ids=["area", "point", "depth1"])
def test_final_gather_transparent_shadows_match_oracle(product, oracle_built, kw):
    """k_fg<TSH>: the gather paths' inline shadow rays collect the transparent surfaces in a per-lane
    list and multiply their filter colour into the light colour (tsFilterColor, as k_tshadow)."""
    spec = _pm_fg_spec(**kw)
    rgba, w, _ = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w, ow)
    u = ulp_diff(rgba, orgba)
    assert u.max() <= ULP_TOL, f"{(u > ULP_TOL).sum()} values > {ULP_TOL} ULP, max {u.max()}"
