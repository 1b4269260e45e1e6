"""Oren-Nayar diffuse BRDF, DirectLight ambient occlusion, material additionaldepth, the AA light
sample multiplier and multi-sample area lights: the HIP path (through the C ABI) against the CPU
oracle on the same scenes.

References:
  * Oren-Nayar: ShinyDiffuseMaterial::initOrenNayar / orenNayar (material_shiny_diffuse.cc:146-188),
    applied in eval (:228-233) and in the diffuse branch of sample (:320-325); the texture sigma
    path ("sigma_oren_shader") computes A / B in double per hit.
  * Ambient occlusion: TiledIntegrator::sampleAmbientOcclusion (integrator_tiled.cc:644-691) called
    by DirectLightIntegrator::integrate (integrator_direct_light.cc:124) for diffuse hits.
  * additionaldepth: integrator_direct_light.cc:107 / integrator_montecarlo.cc:923.
  * AA_light_sample_multiplier_factor: integrator_tiled.cc:190, integrator_montecarlo.cc:396.

Tolerance: per pixel <= 4 ULP of the oracle (no Russian roulette); weights equal.
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


def compare(product, oracle_built, spec, chunk_slots=None):
    rgba, w, st = product.render_spec(spec, chunk_slots=chunk_slots)
    orgba, ow, ctr = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w, ow), "film weights differ"
    u = ulp_diff(rgba, orgba)
    assert u.max() <= ULP_TOL, (f"max {u.max()} ULP at {np.unravel_index(u.argmax(), u.shape)}: "
                                f"{rgba.reshape(-1)[u.argmax()]} vs {orgba.reshape(-1)[u.argmax()]}")
    return rgba, st, ctr


def oren_cornell(integrator="directlighting", sigma=0.5, **kw):
    s = scenes.cornell(64, 48, spp=2, bounces=4, rr=False, integrator=integrator, **kw)
    mats = [dataclasses.replace(m, diffuse_brdf="oren_nayar", sigma=sigma * (1 + 0.5 * k)) for k, m in enumerate(s.materials)]
    return dataclasses.replace(s, materials=mats)


def ao_spec(base="cornell", samples=6, dist=0.8, color=(0.9, 0.8, 0.7), **kw):
    if base == "cornell":
        s = scenes.cornell(64, 48, spp=2, bounces=3, rr=False, integrator="directlighting", **kw)
    elif base == "test01":
        s = scenes.test01(64, 64, spp=2)
    else:
        s = scenes.cornell_transparent_shadows(64, 48, spp=2, panes=2, **kw)
    return s.with_render(do_ao=True, ao_samples=samples, ao_distance=dist, ao_color=color)


# ---------------------------------------------------------------------------------------------
# CPU: the oracle restatement behaves (no GPU)
# ---------------------------------------------------------------------------------------------
def test_oracle_oren_nayar_darkens_and_stays_finite(oracle_built):
    lam = scenes.cornell(32, 24, spp=1, integrator="directlighting")
    on = oren_cornell(sigma=0.8).with_render(width=32, height=24, aa_samples=1).with_camera(resx=32, resy=24)
    a, wa, _ = oracle_built.OracleScene(lam, threads=4).render()
    b, wb, _ = oracle_built.OracleScene(on, threads=4).render()
    assert np.isfinite(b).all() and np.array_equal(wa, wb)
    assert np.abs(a - b).max() > 1e-3
    # Oren-Nayar with sigma -> 0 is Lambert (A = 1, B = 0)
    z = dataclasses.replace(on, materials=[dataclasses.replace(m, sigma=0.0) for m in on.materials])
    c, _, _ = oracle_built.OracleScene(z, threads=4).render()
    assert np.array_equal(a.view(np.uint32), c.view(np.uint32))


def test_oracle_ao_adds_light(oracle_built):
    s = scenes.cornell(32, 24, spp=1, integrator="directlighting")
    a, _, _ = oracle_built.OracleScene(s, threads=4).render()
    b, _, (ncl, nsh) = oracle_built.OracleScene(s.with_render(do_ao=True, ao_samples=4), threads=4).render()
    assert np.isfinite(b).all()
    assert (b[..., :3] >= a[..., :3] - 1e-6).all() and (b - a).max() > 0.01
    assert nsh > 4 * 32 * 24 * 0.5


# ---------------------------------------------------------------------------------------------
# GPU parity
# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("integrator", ["directlighting", "pathtracing"])
@pytest.mark.parametrize("sigma", [0.25, 0.9])
def test_oren_nayar_matches_oracle(product, oracle_built, integrator, sigma):
    compare(product, oracle_built, oren_cornell(integrator, sigma))


@pytest.mark.gpu
def test_oren_nayar_test01_matches_oracle(product, oracle_built):
    s = scenes.test01(64, 64, spp=2)
    s = dataclasses.replace(s, materials=[dataclasses.replace(m, diffuse_brdf="oren_nayar", sigma=0.6) for m in s.materials])
    compare(product, oracle_built, s)


@pytest.mark.gpu
def test_oren_nayar_texture_sigma(product, oracle_built):
    """sigma_oren_shader: a scalar layer node drives sigma per hit (double A / B), with a mirror
    component on one material so the tree path runs too."""
    import texscenes as T
    imgs = [T.procedural_image("p", opt="none", seed=41)]
    tx = [T.texture("q", "p")]
    mats = []
    for k in range(3):
        nodes = [T.layer("root", "map"), T.mapper("map", "q", texco="uv", mapping="plain"),
                 T.layer("sig", "map", do_color=T.B(False), do_scalar=T.B(True), use_alpha=T.B(True), def_val=T.F(0.3 + 0.2 * k),
                         valfac=T.F(0.9), upper_value=T.F(0.5))]
        extra = {"diffuse_brdf": T.S("oren_nayar"), "sigma": T.F(0.4), "sigma_oren_shader": T.S("sig")}
        if k == 2:
            extra["specular_reflect"] = T.F(0.3)
        m = T.material(f"on{k}", nodes, **extra)
        mats.append(dataclasses.replace(m, diffuse_brdf="oren_nayar", sigma=0.4, specular_reflect=0.3 if k == 2 else 0.0))
    spec = T.grid_scene(mats, imgs, tx, width=64, height=48, spp=1)
    compare(product, oracle_built, spec)


@pytest.mark.gpu
@pytest.mark.parametrize("base", ["cornell", "test01"])
def test_ambient_occlusion_matches_oracle(product, oracle_built, base):
    _, st, ctr = compare(product, oracle_built, ao_spec(base))
    assert st["closest_rays"] == ctr[0]


@pytest.mark.gpu
def test_ambient_occlusion_transparent_shadows(product, oracle_built):
    compare(product, oracle_built, ao_spec("transparent", samples=4, dist=1.5))


@pytest.mark.gpu
def test_ambient_occlusion_emitting_and_specular(product, oracle_built):
    """An emitting diffuse material adds emit * pdf per AO sample; the specular tree runs AO at
    every integrate() node; several chunks."""
    s = scenes.cornell_specular(48, 36, spp=2, raydepth=2)
    mats = [dataclasses.replace(m, emit=0.3) if m.name == "red" else m for m in s.materials]
    s = dataclasses.replace(s, materials=mats).with_render(do_ao=True, ao_samples=5, ao_distance=0.6)
    compare(product, oracle_built, s, chunk_slots=1500)


@pytest.mark.gpu
@pytest.mark.parametrize("raydepth,add", [(0, 2), (1, 1), (1, 3)])
def test_additional_depth(product, oracle_built, raydepth, add):
    """A mirror material's additionaldepth extends the recursion below raydepth."""
    s = scenes.cornell_specular(48, 36, spp=1, raydepth=raydepth)
    mats = [dataclasses.replace(m, additionaldepth=add) if m.name == "tall_mirror" else m for m in s.materials]
    s = dataclasses.replace(s, materials=mats)
    rgba, _, _ = compare(product, oracle_built, s)
    base, _, _ = product.render_spec(dataclasses.replace(s, materials=[dataclasses.replace(m, additionaldepth=0) for m in mats]))
    assert np.abs(rgba - base).max() > 0, "additionaldepth changed nothing"


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", ["directlighting", "pathtracing"])
def test_area_light_several_samples(product, oracle_built, integrator):
    """Area light with 5 samples: consecutive Halton draws of one sequence (halton.h getNext)."""
    compare(product, oracle_built, scenes.cornell(48, 36, spp=2, bounces=3, integrator=integrator, light_samples=5))


@pytest.mark.gpu
@pytest.mark.parametrize("factor", [2.0, 0.5])
def test_light_sample_multiplier(product, oracle_built, factor):
    s = scenes.cornell(48, 36, spp=2, bounces=3, integrator="directlighting", light_samples=3).with_render(
        aa_passes=3, aa_inc_samples=2, aa_threshold=0.0, aa_light_sample_multiplier_factor=factor)
    _, st, ctr = compare(product, oracle_built, s)
    assert st["shadow_rays"] == ctr[1]


# ---------------------------------------------------------------------------------------------
# features the GPU core refuses (the reference would render them; no silent divergence)
# ---------------------------------------------------------------------------------------------
def _interface(product):
    yi = product.Interface()
    yi.createScene()
    return yi


def test_refused_features_fail_loudly(product):
    yi = _interface(product)
    yi.paramsClearAll()
    yi.paramsSetString("type", "shinydiffusemat")
    yi.paramsSetFloat("wireframe_amount", 0.5)
    assert not yi.createMaterial("wire")
    yi.paramsClearAll()
    yi.paramsSetString("type", "constant")
    yi.paramsSetBool("ibl", True)
    assert not yi.createBackground("bg")
    yi.paramsClearAll()
    yi.paramsSetString("type", "mesh")
    yi.paramsSetString("visibility", "shadow_only")
    assert not yi.createObject("obj")
    yi.paramsClearAll()
    yi.paramsSetString("type", "shinydiffusemat")
    yi.paramsSetString("diffuse_brdf", "oren_nayar")
    yi.paramsSetFloat("sigma", 0.3)
    assert yi.createMaterial("on")   # supported now
    yi.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["bounces12"])
def test_refused_render_settings(product, case):
    """(photon caustics — PT caustic_type photon | both, DirectLight caustics — are supported since
    round 2: tests/test_caustics.py)"""
    s = scenes.cornell(16, 16, spp=1, bounces=4)
    if case == "bounces12":
        s = s.with_render(bounces=12)
    with pytest.raises(RuntimeError):
        product.render_spec(s)
