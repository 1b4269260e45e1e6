"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same inputs.

Tolerances (BASELINE.json north_star: "radiance matches the reference CPU integrator within a
stated float tolerance"):
  * ray level — closest-hit t and primitive bit-exact, shadow occlusion exact (exact-t ties
    between different primitives resolve to the lower index in both; none occur here);
  * DirectLight and PathTracer without Russian roulette — per pixel |d| <= 4 ULP of the oracle
    value (the device emulates the reference's x87 products exactly, so in
    practice the images are bit-identical);
  * PathTracer with Russian roulette — the reference draws RR numbers from a per-tile glibc
    rand() seed, so the comparison is statistical: 8x8-pixel block means within 4 sigma.
"""
import numpy as np
import pytest

from libyafaray_amd import scenes

pytestmark = pytest.mark.gpu


def ulp_diff(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7fffffff), a)
    b = np.where(b < 0, -(b & 0x7fffffff), b)
    return np.abs(a - b)


def random_rays(spec, n, seed):
    rng = np.random.default_rng(seed)
    lo, hi = spec.verts.min(0), spec.verts.max(0)
    c = (lo + hi) / 2
    ext = (hi - lo).max()
    o = c + (rng.random((n, 3)) - 0.5) * ext * 1.6
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tmin = np.zeros((n, 1))
    tmax = np.where(rng.random((n, 1)) < 0.3, rng.random((n, 1)) * ext, -1.0)
    return np.concatenate([o, d, tmin, tmax], 1).astype(np.float32)


def product_scene(product, spec):
    yi = product.Interface()
    scenes.apply(spec, yi)
    return yi


# BVH layouts under test: BVH4 (default), BVH4 with a 4-level LDS stack (exercises the HBM spill
# levels of k_trace / k_photon_bounce), and the binary BVH2
# and the device-built BVH4 (bvhgpu.hip: PLOC + collapse; the default for >= 64 K triangles)
# "brute": scenes of <= 64 triangles (the Cornell box) through k_trace_brute (opt-in; the other
# variants pin the BVH traversal explicitly); "ray-sort": k_trace<SORT> (LDS-resident scenes)
BVH_VARIANTS = {"bvh4": {"YAFARAY_AMD_BVH_BUILD": "host", "YAFARAY_AMD_TRACE": "bvh"},
                "bvh4-spill": {"YAFARAY_AMD_LDS_STACK": "4", "YAFARAY_AMD_TRACE": "bvh"},
                "bvh2": {"YAFARAY_AMD_BVH_WIDTH": "2", "YAFARAY_AMD_TRACE": "bvh"},
                "gpu-build": {"YAFARAY_AMD_BVH_BUILD": "gpu", "YAFARAY_AMD_TRACE": "bvh"},
                "bvh4-global": {"YAFARAY_AMD_SCENE_LDS": "0", "YAFARAY_AMD_TRACE": "bvh"},
                # r05: the device-built tree in global memory traced through its BVH8 (opt-in, k_trace's refill loop)
                "bvh8-global": {"YAFARAY_AMD_BVH_BUILD": "gpu", "YAFARAY_AMD_SCENE_LDS": "0", "YAFARAY_AMD_TRACE": "bvh",
                                "YAFARAY_AMD_BVH8": "1"},
                "brute": {"YAFARAY_AMD_TRACE": "brute"},
                # ray-stream sorting (opt-in): each wave's window of queue entries in key order
                "ray-sort": {"YAFARAY_AMD_RAY_SORT": "1", "YAFARAY_AMD_TRACE": "bvh"}}


def use_bvh(monkeypatch, variant):
    if variant in ("brute", "ray-sort"):
        from conftest import experiments_built
        if not experiments_built():
            pytest.skip("k_trace_brute / ray sorting live in -DYAF_EXPERIMENTS builds only")
    for k, v in BVH_VARIANTS[variant].items():
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("bvh", ["bvh4", "bvh2", "gpu-build"])
@pytest.mark.parametrize("which", ["cornell", "test01", "sphere"])
def test_trace_closest_and_shadow_bitexact(product, oracle_built, which, bvh, monkeypatch):
    """Ray level on all three scenes; "sphere" is BASELINE C4 (1M triangles, BVH in HBM/L2)."""
    use_bvh(monkeypatch, bvh)
    spec = {"cornell": lambda: scenes.cornell(32, 32, spp=1), "test01": lambda: scenes.test01(32, 32, spp=1),
            "sphere": lambda: scenes.cornell_sphere(width=32, height=32, spp=1)}[which]()
    rays = random_rays(spec, 20000, 7)
    yi = product_scene(product, spec)
    t, prim = yi.trace_closest(rays)
    osc = oracle_built.OracleScene(spec)
    ohit, oprim = osc.trace_closest(rays)
    assert np.array_equal(prim, oprim), f"{(prim != oprim).sum()} primitive mismatches"
    hit = oprim >= 0
    assert np.array_equal(t[hit].view(np.uint32), ohit[hit, 0].view(np.uint32))
    occ = yi.trace_shadow(rays)
    assert np.array_equal(occ, osc.trace_shadow(rays))
    yi.close()


def _subset(spec, n_tris):
    """The first n_tris triangles of a scene as one object (edge cases of the BVH builders)."""
    import dataclasses
    tris = spec.tris[:n_tris]
    used = np.unique(tris)
    remap = np.full(len(spec.verts), -1, np.int32)
    remap[used] = np.arange(len(used), dtype=np.int32)
    return dataclasses.replace(spec, verts=spec.verts[used], tris=remap[tris], tri_mat=spec.tri_mat[:n_tris],
                               objects=[scenes.Object("subset", 0, len(used), 0, n_tris)])


@pytest.mark.parametrize("n_tris", [1, 2, 3, 5, 34, 3200])
def test_gpu_bvh_build_small_and_ragged(product, oracle_built, n_tris, monkeypatch):
    """Device BVH build on 1, 2, 3, 5 triangles, the Cornell box and a 3,200-triangle sphere: rays
    bit-exact with the oracle (a wrong box or a lost triangle changes hits)."""
    use_bvh(monkeypatch, "gpu-build")
    if n_tris == 3200:
        spec = scenes.cornell_sphere(n=40, width=32, height=32, spp=1)
    else:
        spec = _subset(scenes.cornell(32, 32, spp=1), n_tris)
    rays = random_rays(spec, 8000, 11)
    yi = product_scene(product, spec)
    t, prim = yi.trace_closest(rays)
    osc = oracle_built.OracleScene(spec)
    ohit, oprim = osc.trace_closest(rays)
    assert np.array_equal(prim, oprim), f"{(prim != oprim).sum()} primitive mismatches"
    hit = oprim >= 0
    assert hit.any() or n_tris < 3
    assert np.array_equal(t[hit].view(np.uint32), ohit[hit, 0].view(np.uint32))
    assert np.array_equal(yi.trace_shadow(rays), osc.trace_shadow(rays))
    yi.close()


@pytest.mark.parametrize("n_tris", [1, 2, 3, 5, 34, 3200])
def test_bvh8_refill_equals_bvh4(product, n_tris, monkeypatch):
    """r05: k_trace's refill loop over the device build's BVH8 (opt-in YAFARAY_AMD_BVH8=1, scenes in global
    memory) against the same tree's BVH4 (the default) on 1, 2, 3, 5 triangles, the Cornell box and a 3,200-triangle
    sphere, a 4-level LDS stack (the HBM spill levels): bit-identical path-traced films."""
    use_bvh(monkeypatch, "bvh8-global")
    monkeypatch.setenv("YAFARAY_AMD_LDS_STACK", "4")
    if n_tris == 3200:
        spec = scenes.cornell_sphere(n=40, width=40, height=30, spp=4, bounces=6, rr=True)
    else:
        import dataclasses
        base = scenes.cornell(40, 30, spp=4, bounces=6, rr=True)
        spec = dataclasses.replace(_subset(base, n_tris), lights=base.lights, materials=base.materials) if n_tris < 34 else base
    a, wa, sa = product.render_spec(spec)
    assert sa["scene_in_lds"] == 0
    monkeypatch.setenv("YAFARAY_AMD_BVH8", "0")
    b, wb, sb = product.render_spec(spec)
    assert np.array_equal(wa, wb)
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))
    assert sa["closest_rays"] == sb["closest_rays"] and sa["shadow_rays"] == sb["shadow_rays"]


@pytest.mark.gpu
def test_ray_binning_equals_unbinned(product, monkeypatch):
    """r06: ray binning (YAFARAY_AMD_RAY_BIN=1: each queue segment's bounce rays traced in (octant, origin Morton)
    order through a permutation, hits written back to the rays' own queue addresses) gives the unbinned film
    bit for bit on the BVH8 refill path (device build, scene in global memory, several chunks)."""
    use_bvh(monkeypatch, "bvh8-global")
    spec = scenes.cornell_sphere(n=40, width=48, height=36, spp=4, bounces=6, rr=True)
    a, wa, sa = product.render_spec(spec, chunk_slots=1500)
    monkeypatch.setenv("YAFARAY_AMD_RAY_BIN", "1")
    b, wb, sb = product.render_spec(spec, chunk_slots=1500)
    assert sa["scene_in_lds"] == 0 and sa["bvh_width"] == 8
    assert np.array_equal(wa, wb)
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))
    assert sa["closest_rays"] == sb["closest_rays"] and sa["shadow_rays"] == sb["shadow_rays"]


@pytest.mark.parametrize("offset", [(1000.0, -500.0, 250.0), (0.0, 0.0, 0.0)])
def test_bvh8_far_from_origin_and_thin_geometry(product, monkeypatch, offset):
    """r05: the quantised BVH8's byte planes are rounded outwards over the node origin; geometry far from
    the origin (large coordinates, small quanta relative to them) and a sliver of near-degenerate triangles
    must still give the BVH4's hits: bit-identical films (device build, scene in global memory)."""
    import dataclasses
    spec = scenes.cornell_sphere(n=40, width=40, height=30, spp=2, bounces=5, rr=True)
    # a fan of thin triangles (1e-4 wide) across the box
    base = len(spec.verts)
    sl = []
    for k in range(16):
        x = -0.8 + 0.1 * k
        sl += [(x, -0.5, 0.2), (x + 1e-4, 0.5, 0.2), (x + 2e-4, 0.0, 1.6)]
    verts = np.concatenate([spec.verts, np.asarray(sl, np.float32)]) + np.asarray(offset, np.float32)
    tris = np.concatenate([spec.tris, np.arange(base, base + len(sl), dtype=np.int32).reshape(-1, 3)])
    tri_mat = np.concatenate([spec.tri_mat, np.zeros(len(sl) // 3, np.int32)])
    objs = list(spec.objects) + [scenes.Object("slivers", base, len(sl), len(spec.tris), len(sl) // 3)]
    sh = lambda p: tuple(float(a) + float(b) for a, b in zip(p, offset))
    cam = dataclasses.replace(spec.camera, from_=sh(spec.camera.from_), to=sh(spec.camera.to), up=sh(spec.camera.up))
    lights = [dataclasses.replace(l, from_=sh(l.from_), corner=sh(l.corner), point1=sh(l.point1), point2=sh(l.point2)) for l in spec.lights]
    spec = dataclasses.replace(spec, verts=verts, tris=tris, tri_mat=tri_mat, objects=objs, camera=cam, lights=lights)
    use_bvh(monkeypatch, "bvh8-global")
    a, wa, sa = product.render_spec(spec)
    assert sa["scene_in_lds"] == 0 and sa["bvh_width"] == 8
    monkeypatch.setenv("YAFARAY_AMD_BVH8", "0")
    b, wb, sb = product.render_spec(spec)
    assert sb["bvh_width"] == 4
    assert np.array_equal(wa, wb)
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))
    assert a[..., :3].mean() > 0.0


def test_direct_light_test01_matches_oracle(product, oracle_built):
    spec = scenes.test01(96, 96, spp=4)
    rgba, w, st = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    d = ulp_diff(rgba, orgba)
    assert d.max() <= 4, f"max ULP {d.max()} at {np.unravel_index(d.argmax(), d.shape)}"
    assert st["samples"] == 96 * 96 * 4


@pytest.mark.parametrize("bvh", list(BVH_VARIANTS))
def test_path_noRR_cornell_matches_oracle(product, oracle_built, bvh, monkeypatch):
    use_bvh(monkeypatch, bvh)
    spec = scenes.cornell(80, 60, spp=8, bounces=8, rr=False)
    rgba, w, st = product.render_spec(spec, chunk_slots=8192)
    orgba, ow, octr = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    d = ulp_diff(rgba, orgba)
    bad = (d > 4).sum()
    assert d.max() <= 4, f"{bad} values > 4 ULP, max {d.max()} at {np.unravel_index(d.argmax(), d.shape)}"
    # ray accounting: same queries as the reference loop (no RR)
    assert st["closest_rays"] == octr[0]
    assert st["shadow_rays"] <= octr[1]


_sphere_oracle = {}


@pytest.mark.parametrize("bvh", list(BVH_VARIANTS))
def test_path_noRR_sphere_matches_oracle(product, oracle_built, bvh, monkeypatch):
    """BASELINE C4 scene (Cornell box + 999,698-triangle sphere): the BVH does not fit LDS, so this
    exercises the global-memory traversal (k_trace<false, *>) end to end."""
    use_bvh(monkeypatch, bvh)
    spec = scenes.cornell_sphere(width=64, height=48, spp=4, bounces=8, rr=False)
    rgba, w, st = product.render_spec(spec)
    assert st["scene_in_lds"] == 0
    if "ref" not in _sphere_oracle:
        _sphere_oracle["ref"] = oracle_built.OracleScene(spec, threads=8).render()
    orgba, ow, octr = _sphere_oracle["ref"]
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    d = ulp_diff(rgba, orgba)
    assert d.max() <= 4, f"{(d > 4).sum()} values > 4 ULP, max {d.max()} at {np.unravel_index(d.argmax(), d.shape)}"
    assert st["closest_rays"] == octr[0]


ADAPTIVE_AA = {
    # DirectLight on test01, 3 passes of 2 extra samples
    "dl-3pass": lambda: scenes.test01(64, 64, spp=2).with_render(aa_passes=3, aa_inc_samples=2, aa_threshold=0.02),
    # every nextPass option: dark-curve thresholds, colour-noise detection, variance windows, the
    # resampled-floor threshold decay and a growing sample multiplier
    "pt-all-options": lambda: scenes.cornell(48, 40, spp=2, bounces=4, rr=False).with_render(
        aa_passes=4, aa_inc_samples=1, aa_threshold=0.01, aa_dark_detection_type="curve", aa_detect_color_noise=True,
        aa_variance_pixels=3, aa_variance_edge_size=6, aa_resampled_floor=60.0, aa_sample_multiplier_factor=1.5),
    "pt-linear-dark": lambda: scenes.cornell(40, 32, spp=1, bounces=3, rr=False).with_render(
        aa_passes=3, aa_inc_samples=3, aa_threshold=0.03, aa_dark_detection_type="linear", aa_dark_threshold_factor=0.7),
    # threshold 0: every pixel is resampled in every pass (doMoreSamples)
    "threshold-0": lambda: scenes.test01(40, 40, spp=1).with_render(aa_passes=2, aa_inc_samples=2, aa_threshold=0.0),
}


@pytest.mark.parametrize("case", list(ADAPTIVE_AA))
def test_adaptive_aa_matches_oracle(product, oracle_built, case):
    """Adaptive anti-aliasing passes (integrator_tiled.cc:172-231, imagefilm.cc:259-420): the GPU's
    nextPass flags, resampled pixel lists and accumulated film against the oracle's restatement."""
    spec = ADAPTIVE_AA[case]()
    rgba, w, st = product.render_spec(spec, chunk_slots=4096)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32)), f"{(w != ow).sum()} weight mismatches"
    d = ulp_diff(rgba, orgba)
    assert d.max() <= 4, f"{(d > 4).sum()} values > 4 ULP, max {d.max()} at {np.unravel_index(d.argmax(), d.shape)}"
    assert st["samples"] > spec.render.width * spec.render.height * spec.render.aa_samples   # later passes ran


DOF_CASES = {
    "disk1": dict(aperture=0.15, dof_distance=3.5),
    "disk2-center": dict(aperture=0.2, dof_distance=3.0, bokeh_type="disk2", bokeh_bias="center"),
    "triangle-edge-rot": dict(aperture=0.1, dof_distance=4.0, bokeh_type="triangle", bokeh_bias="edge", bokeh_rotation=30.0),
    "square": dict(aperture=0.12, dof_distance=3.8, bokeh_type="square"),
    "pentagon": dict(aperture=0.12, dof_distance=3.8, bokeh_type="pentagon", bokeh_rotation=7.0),
    "hexagon-rot": dict(aperture=0.1, dof_distance=4.0, bokeh_type="hexagon", bokeh_rotation=-12.5),
    "ring": dict(aperture=0.1, dof_distance=4.0, bokeh_type="ring"),
}


@pytest.mark.parametrize("case", list(DOF_CASES))
def test_depth_of_field_matches_oracle(product, oracle_built, case):
    """Perspective camera with aperture (camera_perspective.cc:71-146): Halton(3)/(5) lens streams,
    every bokeh shape and bias, against the oracle — PT without RR, <= 4 ULP."""
    spec = scenes.cornell(48, 36, spp=4, bounces=3, rr=False).with_camera(**DOF_CASES[case])
    rgba, w, _ = product.render_spec(spec, chunk_slots=2048)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    d = ulp_diff(rgba, orgba)
    assert d.max() <= 4, f"{(d > 4).sum()} values > 4 ULP, max {d.max()} at {np.unravel_index(d.argmax(), d.shape)}"


@pytest.mark.parametrize("clip", [(3.4, -1.0), (0.0, 4.6), (3.4, 4.6)])
def test_camera_clip_planes_match_oracle(product, oracle_built, clip):
    """nearClip / farClip (camera.cc:51-71, camera_perspective.cc:128-146): every camera ray carries
    its own (tmin, tmax) — the queue's side array of a pass's first iteration (the bounce rays'
    12-B records carry neither) — PT without RR against the oracle, <= 4 ULP."""
    spec = scenes.cornell(48, 36, spp=2, bounces=3, rr=False).with_camera(near_clip=clip[0], far_clip=clip[1])
    rgba, w, _ = product.render_spec(spec, chunk_slots=2048)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    assert ulp_diff(rgba, orgba).max() <= 4


def test_depth_of_field_with_adaptive_passes(product, oracle_built):
    """DOF lens streams restart at every pass's offset (integrator_tiled.cc:314-316)."""
    spec = scenes.test01(40, 40, spp=2).with_camera(aperture=0.3, dof_distance=8.0, bokeh_type="pentagon").with_render(
        aa_passes=3, aa_inc_samples=2, aa_threshold=0.02)
    rgba, w, _ = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    assert ulp_diff(rgba, orgba).max() <= 4


def test_path_gauss_filter_and_multichunk(product, oracle_built):
    spec = scenes.cornell(72, 40, spp=3, bounces=4, rr=False, filter_type="gauss", pixelwidth=1.5, tile_size=16)
    rgba, w, _ = product.render_spec(spec, chunk_slots=1024)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    assert ulp_diff(rgba, orgba).max() <= 4


@pytest.mark.parametrize("seed", [0, 7919])
def test_path_RR_statistical(product, oracle_built, seed):
    """Russian roulette on (the reference default): the GPU's per-sample RR streams against the
    oracle's per-tile ones (integrator_path_tracer.cc:249-255, integrator_tiled.cc:272) — unbiased
    means a paired global z of the difference image within 4 (oracle/stats.py), for two independent
    seeds on both sides; no 8x8 block may stand out either."""
    from oracle.stats import paired_z
    spec = scenes.cornell(256, 256, spp=64, bounces=8, rr=True).with_render(rr_seed=seed)
    rgba, w, _ = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=16, rr_seed=seed).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    z = paired_z(rgba, orgba)
    assert abs(z["mean_z"]) < 4.0, z
    assert z["max_abs_block_z"] < 6.0, z
    assert abs(z["mean_rel_diff"]) < 0.01, z


def test_reference_client_test01_renders(tmp_path):
    """The reference's tests/test01/test01.c client (built by `make -C oracle clients`) renders its
    scene on the GPU through the drop-in library.  Its TGA and HDR textures load (the reference's
    own test data, next to the executable's working directory as the client expects); the TIFF /
    PNG / JPG / EXR ones fail with the same errors the reference built without those libraries logs
    (src/format/format.cc:40-66), and nothing else is an error."""
    import os
    import shutil
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "clients", "test01")
    if not os.path.exists(exe):
        pytest.skip("reference clients not built")
    for ext in ("tga", "hdr"):
        shutil.copyfile(os.path.join(scenes.TEX01_DIR, "tex." + ext), os.path.join(tmp_path, "tex." + ext))
    r = subprocess.run([exe], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-2000:]
    assert "loaded from file 'tex.tga'" in out and "loaded from file 'tex.hdr'" in out, out[-2000:]
    expected = ("image file format", "Couldn't load from file 'tex.", "could not be created", "no valid image type",
                "dropping texture", "TextureMapper: texture")
    errors = [ln for ln in out.splitlines() if "ERROR" in ln and not any(e in ln for e in expected)]
    assert not errors, errors[:5]
    for ext in ("tif", "png", "jpg", "exr"):
        assert f"format '{ext}'" in out


@pytest.mark.parametrize("bvh", list(BVH_VARIANTS))
def test_photon_mapping_matches_oracle(product, oracle_built, bvh, monkeypatch):
    """BASELINE C5 pipeline at a small size: photon shooting (GPU wavefront), point kd-tree,
    k-NN gather with the reference's heap order, PM integrate (emission twice, direct light,
    density estimate) — per pixel <= 4 ULP of the oracle."""
    use_bvh(monkeypatch, bvh)
    spec = scenes.cornell_photon(64, 48, spp=2, photons=30000, search=50, radius=0.1)
    rgba, w, st = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    opos, _, _, _, npaths = oracle_built.OracleScene(spec, threads=8).photon_map()
    assert st["photons"] == len(opos)
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    d = ulp_diff(rgba, orgba)
    assert d.max() <= 4, f"{(d > 4).sum()} values > 4 ULP, max {d.max()} at {np.unravel_index(d.argmax(), d.shape)}"


@pytest.mark.parametrize("photons", [120, 400000])
def test_photon_map_sizes_match_oracle(product, oracle_built, photons):
    """Photon-map sizes on both sides of the GPU kd-tree build's phase switch (pkd.hip: subtrees of
    <= 256 photons are finished in LDS, larger nodes are split level by level across the chip):
    ~240 photons (LDS phase only) and ~800 K photons (11 top levels)."""
    spec = scenes.cornell_photon(48, 36, spp=1, photons=photons, search=50, radius=0.1)
    rgba, w, st = product.render_spec(spec)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    d = ulp_diff(rgba, orgba)
    assert d.max() <= 4, f"{(d > 4).sum()} values > 4 ULP, max {d.max()} at {np.unravel_index(d.argmax(), d.shape)}"
    assert st["gather_visits"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("rr", [False, True])
def test_throughput_record_without_w_equals_full_record(product, monkeypatch, rr):
    """r05: scenes whose every sample() sets the weight w before it is read keep the throughput as a
    12-B record (DevScene::w_live = 0, host.cc); YAFARAY_AMD_W_LIVE=1 forces the 16-B record that carries
    w — the two renders must be bit-identical (RR off and on: the stateless RR draw is the same)."""
    spec = scenes.cornell(80, 60, spp=8, bounces=6, rr=rr)
    a, wa, _ = product.render_spec(spec)
    monkeypatch.setenv("YAFARAY_AMD_W_LIVE", "1")
    b, wb, _ = product.render_spec(spec)
    assert np.array_equal(wa, wb)
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))
