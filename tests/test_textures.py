"""Image textures, shader nodes and surface attributes: the GPU path (k_surface
+ the ATTR instantiations of k_shade / k_nee, through the C ABI) against the CPU oracle
(oracle/yaftex.h) on the same scenes.

Tolerance: per pixel <= 4 ULP (the texture arithmetic is restated operation for operation, so in
practice the images are bit-identical).  The tube / sphere projections call libm's float atan2 / acos
(shader_node_basic.cc:67, 77-78): the device restates glibc's fdlibm algorithms (devmath.h
libmAtan2f / libmAcosf, pinned against the host libm by tests/test_devmath.py), so they are held to
the same bar since round 5 (round 4 used the device math library and a statistical tolerance).
"""
import dataclasses

import numpy as np
import pytest

from libyafaray_amd import scenes
import texscenes as T

ULP_TOL = 4


def ulp_diff(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7fffffff), a)
    b = np.where(b < 0, -(b & 0x7fffffff), b)
    return np.abs(a - b)


def build_case(name, **kw):
    mats, imgs, texs = T.CASES[name]()
    return T.grid_scene(mats, imgs, texs, **kw)


# ---------------------------------------------------------------------------------------------
# CPU: the oracle's texturing path runs and actually textures
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("case", list(T.CASES))
def test_oracle_textured_cases_render(oracle_built, case):
    spec = build_case(case, width=24, height=18, spp=1)
    rgba, w, _ = oracle_built.OracleScene(spec, threads=4).render()
    assert np.isfinite(rgba).all() and (w > 0).all()
    # the same geometry with every material's nodes dropped must look different
    plain = dataclasses.replace(spec, materials=[dataclasses.replace(m, params=None, nodes=[]) for m in spec.materials])
    rgba2, _, _ = oracle_built.OracleScene(plain, threads=4).render()
    assert np.abs(rgba - rgba2).max() > 0.01


def test_oracle_test01_textured_differs_only_on_loadable_textures(oracle_built):
    """Only the TGA and HDR cubes change: the PNG / JPG / TIFF / EXR images cannot be loaded by the
    reference as built without those libraries, which drops their textures (plain colour)."""
    a, _, _ = oracle_built.OracleScene(scenes.test01_textured(64, 64, spp=1), threads=4).render()
    b, _, _ = oracle_built.OracleScene(scenes.test01(64, 64, spp=1), threads=4).render()
    diff = np.abs(a - b).max(axis=2) > 0
    assert 50 < diff.sum() < 64 * 64 // 3


# ---------------------------------------------------------------------------------------------
# GPU vs oracle
# ---------------------------------------------------------------------------------------------
def _compare(product, oracle_built, spec, tol_ulp=ULP_TOL):
    rgba, w, st = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w, ow), "film weights differ"
    u = ulp_diff(rgba, orgba)
    assert u.max() <= tol_ulp, f"max {u.max()} ULP at {np.unravel_index(u.argmax(), u.shape)}: {rgba.reshape(-1)[u.argmax()]} vs {orgba.reshape(-1)[u.argmax()]}"
    return rgba, st


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(T.CASES))
def test_textures_direct_light_match_oracle(product, oracle_built, case):
    _compare(product, oracle_built, build_case(case))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["images", "layers"])
def test_textures_path_tracer_match_oracle(product, oracle_built, case):
    """PathIntegrator without RR: textured BSDF sampling, emission and NEE through k_shade/k_nee<ATTR>."""
    _compare(product, oracle_built, build_case(case, integrator="pathtracing", width=64, height=48, spp=2))


@pytest.mark.gpu
def test_textures_path_samples_carry_first_hit_attributes(product, oracle_built):
    """path_samples > 1: later subpaths restart from the first hit, whose shader colour and shading
    normal travel with the path state (DevPaths::v0attr)."""
    spec = build_case("layers", integrator="pathtracing", width=48, height=36, spp=1, sphere_smooth=40.0)
    spec = spec.with_render(path_samples=3)
    _compare(product, oracle_built, spec)


@pytest.mark.gpu
@pytest.mark.parametrize("angle,normals", [(180.0, False), (30.0, False), (0.05, False), (None, True)])
def test_smooth_normals_match_oracle(product, oracle_built, angle, normals):
    """MeshObject::smoothNormals (all-faces and angle-limited) and exported vertex normals."""
    spec = build_case("images", sphere_smooth=angle if angle is not None else 180.0, normals=normals)
    _compare(product, oracle_built, spec)
    _compare(product, oracle_built, spec.with_render(integrator="pathtracing", bounces=3, aa_samples=1))


@pytest.mark.gpu
def test_test01_textured_matches_oracle(product, oracle_built):
    """BASELINE C1 with the reference's own texturing (test01.c: TGA + HDR cubes, gauss 1.5)."""
    rgba, st = _compare(product, oracle_built, scenes.test01_textured(128, 128, spp=4))
    plain, _, _ = product.render_spec(scenes.test01(128, 128, spp=4))
    assert np.abs(rgba - plain).max() > 0.1


@pytest.mark.gpu
def test_textures_photon_mapping_match_oracle(product, oracle_built):
    """PhotonIntegrator over textured / smooth materials: photon scattering uses the hit's shader
    colour (k_photon_bounce<ATTR>), the density estimate the camera hit's (k_gather<ATTR>)."""
    spec = build_case("layers", width=48, height=36, spp=1, sphere_smooth=60.0)
    spec = spec.with_render(integrator="photonmapping", pm_photons=20000, pm_search=30, pm_diffuse_radius=0.4)
    rgba, w, st = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    opos, _, _, _, _ = oracle_built.OracleScene(spec, threads=8).photon_map()
    assert st["photons"] == len(opos)
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    u = ulp_diff(rgba, orgba)
    assert u.max() <= ULP_TOL, f"max {u.max()} ULP"
