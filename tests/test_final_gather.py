"""PhotonIntegrator final gathering (finalGather = true, the reference's default):
integrator_photon_mapping.cc:183-193 (radiance points while shooting the diffuse map), :540-591
(thinning with EliminatePhoton over a point kd-tree, pre-gathering, the radiance map's tree),
:39-88 (preGatherWorker), :640-763 (finalGathering), :874-917 (integrate with final gathering);
photon.cc:136-142 (findNearest).

GPU: radiance points in k_photon_bounce, compaction, thinning in rounds (fgthin.hip), k_pregather, the radiance map's
point kd-tree (pkd.hip), k_fg (gather paths traced in place, estimateOneDirectLight with in-place
shadow rays, radiance-map lookups) before k_gather.  Compared with the oracle restatement
(oracle/yafcpu.cc finalGathering / buildRadianceMap): per value <= 4 ULP, weights equal.

The radiance-point subset is drawn by the reference from the global FastRandom shared by the photon
threads (:186, schedule-dependent); both sides here keep the deposits whose slot hash selects one
in eight (fgRadSelect), so the radiance map is matched to the reference statistically, like RR.
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


def fg_spec(W=48, H=36, spp=1, photons=20000, specular=False, **kw):
    if specular:
        s = scenes.cornell_specular(W, H, spp=spp, integrator="photonmapping", raydepth=3)
        r = dataclasses.replace(s.render, pm_photons=photons, pm_search=50, pm_diffuse_radius=0.1, pm_bounces=5,
                                pm_caustics=False)
        s = dataclasses.replace(s, render=r)
    else:
        s = scenes.cornell_photon(W, H, spp=spp, photons=photons, search=50, radius=0.1)
    fg = dict(pm_final_gather=True, fg_samples=8)
    fg.update(kw)
    return dataclasses.replace(s, render=dataclasses.replace(s.render, **fg))


# ---------------------------------------------------------------------------------------------
# CPU: the oracle restatement
# ---------------------------------------------------------------------------------------------
def test_oracle_radiance_map(oracle_built):
    spec = fg_spec(16, 12, photons=20000)
    o = oracle_built.OracleScene(spec, threads=4)
    dpos, _, _, _, n_paths = o.photon_map("diffuse")
    rpos, rn, rcol, nodes, rpaths = o.photon_map("radiance")
    assert rpaths == n_paths
    # one deposit in eight becomes a radiance point, and thinning removes some of them
    assert 0 < len(rpos) < len(dpos) / 8 * 1.2
    assert np.allclose(np.linalg.norm(rn, axis=1), 1.0, atol=1e-3)
    assert np.all(np.isfinite(rcol)) and np.all(rcol >= 0) and rcol.max() > 0
    # the kept points are pairwise "far" in the EliminatePhoton sense: no later kept point lies within
    # the squared distance 0.01 * diffuseRadius of an earlier one with a normal on the same side
    maxrad = np.float32(0.01) * np.float32(0.1)
    for i in range(len(rpos)):
        d2 = ((rpos[i + 1:] - rpos[i]) ** 2).sum(1)
        same = (rn[i + 1:] * rn[i]).sum(1) > 0
        assert not np.any((d2 < maxrad) & same)
    # every point is a leaf of the radiance map's tree exactly once
    leaves = nodes[(nodes[:, 1] & 3) == 3, 0]
    assert sorted(leaves.tolist()) == list(range(len(rpos)))


def test_oracle_final_gather_deterministic_and_indirect(oracle_built):
    spec = fg_spec(20, 14, spp=1, photons=8000, fg_samples=4)
    a, wa, _ = oracle_built.OracleScene(spec, threads=1).render()
    b, wb, _ = oracle_built.OracleScene(spec, threads=6).render()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    # final gathering adds indirect light on top of the direct light everywhere on the walls
    dl_spec = dataclasses.replace(spec, render=dataclasses.replace(spec.render, integrator="directlighting", pm_final_gather=False))
    dl, _, _ = oracle_built.OracleScene(dl_spec, threads=4).render()
    assert (a[..., :3] >= dl[..., :3] - 1e-6).all() and a[..., :3].mean() > 1.1 * dl[..., :3].mean()


# ---------------------------------------------------------------------------------------------
# GPU: the HIP path against the oracle
# ---------------------------------------------------------------------------------------------
def compare(product, oracle_built, spec, chunk_slots=None):
    rgba, w, st = product.render_spec(spec, chunk_slots=chunk_slots)
    o = oracle_built.OracleScene(spec, threads=8)
    orgba, ow, _ = o.render()
    dpos, *_ = o.photon_map("diffuse")
    assert st["photons"] == len(dpos)
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32)), "film weights differ"
    u = ulp_diff(rgba, orgba)
    assert u.max() <= ULP_TOL, (f"{(u > ULP_TOL).sum()} values > {ULP_TOL} ULP, max {u.max()} at "
                                f"{np.unravel_index(u.argmax(), u.shape)}: {rgba.reshape(-1)[u.argmax()]} vs {orgba.reshape(-1)[u.argmax()]}")
    return rgba


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(), dict(fg_bounces=0), dict(fg_min_pathlen=0.8, fg_bounces=3), dict(fg_samples=3, spp=2)],
                         ids=["default", "bounces0", "close-paths", "spp2"])
def test_final_gather_matches_oracle(product, oracle_built, kw):
    compare(product, oracle_built, fg_spec(**kw))


@pytest.mark.gpu
def test_final_gather_specular_matches_oracle(product, oracle_built):
    """Mirror and transparent surfaces: gather paths that bounce specularly (caustic gather paths
    look the radiance map up inside the loop) and recursiveRaytrace nodes that final-gather again."""
    compare(product, oracle_built, fg_spec(specular=True, fg_min_pathlen=0.3))


@pytest.mark.gpu
def test_final_gather_host_thinning_matches_oracle(product, oracle_built, monkeypatch):
    """The host twin of the radiance-point thinning (render.cc eliminateRadPoints, used when the
    dense GPU grid would be too large) gives the same radiance map as the GPU rounds (fgthin.hip)."""
    monkeypatch.setenv("YAFARAY_AMD_FG_THIN", "host")
    compare(product, oracle_built, fg_spec(photons=30000))


@pytest.mark.gpu
def test_final_gather_off_is_unchanged(product, oracle_built):
    spec = fg_spec(pm_final_gather=False)
    compare(product, oracle_built, spec)


@pytest.mark.gpu
def test_final_gather_textured_point_light_matches_oracle(product, oracle_built):
    """Textured / smooth materials and a point light: gather hits evaluate the shader-node colour
    (k_fg<EXT> with surface attributes), radiance points the reflectivity of the textured hit, and
    estimateOneDirectLight takes the point-light branch (shadow ray traced in place)."""
    import texscenes as T
    mats, imgs, texs = T.CASES["layers"]()
    spec = T.grid_scene(mats, imgs, texs, width=40, height=30, spp=1, sphere_smooth=60.0)
    spec = spec.with_render(integrator="photonmapping", pm_photons=20000, pm_search=30, pm_diffuse_radius=0.4,
                            pm_final_gather=True, fg_samples=4, fg_min_pathlen=1.5)
    compare(product, oracle_built, spec)


@pytest.mark.gpu
def test_launch_sequence_per_integrator(product):
    """k_gather / k_fg run only where the integrator has photon-map estimates to finish (a path
    tracer without photon caustics launches neither; final gathering launches k_fg once per chunk,
    in the iteration the direct-light pipeline finishes)."""
    pt = scenes.cornell(32, 24, spp=1, bounces=3, rr=False)
    _, _, st = product.render_spec(pt, profile=True)
    kt = st["kernel_times"]
    assert kt.get("k_gather", {}).get("launches", 0) == 0 and kt.get("k_fg", {}).get("launches", 0) == 0
    _, _, st = product.render_spec(fg_spec(24, 18, fg_samples=2), profile=True)
    kt = st["kernel_times"]
    assert kt["k_fg"]["launches"] == 1 and kt["k_gather"]["launches"] == 1


@pytest.mark.gpu
def test_final_gather_several_chunks_and_aa_passes(product, oracle_built):
    """Final gathering over several wavefront chunks (the gather queue of each chunk) and with
    adaptive AA passes (PixelSamplingData of the resampled pixels' later passes)."""
    compare(product, oracle_built, fg_spec(32, 24, spp=2, fg_samples=3), chunk_slots=300)
    spec = fg_spec(32, 24, spp=1, fg_samples=2, aa_passes=2, aa_inc_samples=1, aa_threshold=0.02)
    compare(product, oracle_built, spec)


@pytest.mark.gpu
@pytest.mark.parametrize("factor", [1.5, 0.6])
def test_final_gather_indirect_sample_multiplier(product, oracle_built, factor):
    """AA_indirect_sample_multiplier_factor with adaptive passes: pass p final-gathers
    ceilf(fg_samples * factor^p) paths per hit (integrator_photon_mapping.cc:648, integrator_tiled.cc:191),
    the PixelSamplingData offsets still stride by fg_samples."""
    spec = fg_spec(32, 24, spp=1, fg_samples=3, aa_passes=3, aa_inc_samples=1, aa_threshold=0.01,
                   aa_indirect_sample_multiplier_factor=factor)
    compare(product, oracle_built, spec)


@pytest.mark.gpu
def test_final_gather_nearest_lds_stack_equals_private(product, monkeypatch):
    """k_fg's radiance-map nearest searches with the far-child stack in an LDS column (pkNearestLds,
    the parent plane recomputing the stacked distance) visit what the private-array stack visits:
    the film is bit-identical."""
    spec = fg_spec(48, 36, fg_samples=8)
    a, w, _ = product.render_spec(spec)
    monkeypatch.setenv("YAFARAY_AMD_FG_NEAREST", "private")
    b, wb, _ = product.render_spec(spec)
    assert np.array_equal(w.view(np.uint32), wb.view(np.uint32))
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["default", "close-paths", "specular", "textured", "batches"])
def test_final_gather_per_path_lanes_equal_lane_per_request(product, monkeypatch, case):
    """r06: final gathering with one lane per gather path (k_fg_first / k_fg_long / k_fg_sum: the bouncing
    paths compacted into their own launch, each path's additions kept as terms and summed per request in
    path order) gives the film of k_fg's one lane per request (YAFARAY_AMD_FG=lane) bit for bit — the
    reference's addition order (integrator_photon_mapping.cc:707-755) is unchanged."""
    if case == "textured":
        import texscenes as T
        mats, imgs, texs = T.CASES["layers"]()
        spec = T.grid_scene(mats, imgs, texs, width=40, height=30, spp=1, sphere_smooth=60.0)
        spec = spec.with_render(integrator="photonmapping", pm_photons=20000, pm_search=30, pm_diffuse_radius=0.4,
                                pm_final_gather=True, fg_samples=4, fg_min_pathlen=1.5)
    elif case == "specular":
        spec = fg_spec(specular=True, fg_min_pathlen=0.3)
    elif case == "close-paths":
        spec = fg_spec(fg_min_pathlen=0.8, fg_bounces=3, fg_samples=6)
    else:
        spec = fg_spec(W=64, H=48, fg_samples=8)
    if case == "batches":
        monkeypatch.setenv("YAFARAY_AMD_FG_BATCH", "7")   # request positions per segment and batch: several batches
    a, w, st = product.render_spec(spec, profile=True)
    monkeypatch.delenv("YAFARAY_AMD_FG_BATCH", raising=False)
    monkeypatch.setenv("YAFARAY_AMD_FG", "lane")
    b, wb, st_b = product.render_spec(spec, profile=True)
    assert np.array_equal(w.view(np.uint32), wb.view(np.uint32))
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), int(ulp_diff(a, b).max())
    # the same paths and radiance-map lookups were counted by both kernels
    for k in ("fg_paths", "fg_lookups"):
        assert st[k] == st_b[k] and st[k] > 0, (k, st[k], st_b[k])


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["default", "close-paths", "specular", "textured"])
def test_final_gather_grid_nearest_equals_kd_search(product, monkeypatch, case):
    """r06: the radiance map's nearest searches over its uniform grid (gridNearest; a tie of the smallest
    facing distance asks the kd search) return the kd search's photon (YAFARAY_AMD_FG_GRID=0): bit-identical
    films, the same lookups."""
    if case == "textured":
        import texscenes as T
        mats, imgs, texs = T.CASES["layers"]()
        spec = T.grid_scene(mats, imgs, texs, width=40, height=30, spp=1, sphere_smooth=60.0)
        spec = spec.with_render(integrator="photonmapping", pm_photons=20000, pm_search=30, pm_diffuse_radius=0.4,
                                pm_final_gather=True, fg_samples=4, fg_min_pathlen=1.5)
    elif case == "specular":
        spec = fg_spec(specular=True, fg_min_pathlen=0.3)
    elif case == "close-paths":
        spec = fg_spec(fg_min_pathlen=0.8, fg_bounces=3, fg_samples=6)
    else:
        spec = fg_spec(W=64, H=48, fg_samples=8, photons=60000)
    a, w, st = product.render_spec(spec)
    monkeypatch.setenv("YAFARAY_AMD_FG_GRID", "0")
    b, wb, st_b = product.render_spec(spec)
    assert np.array_equal(w.view(np.uint32), wb.view(np.uint32))
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), int(ulp_diff(a, b).max())
    assert st["fg_lookups"] == st_b["fg_lookups"] > 0


@pytest.mark.gpu
def test_final_gather_lds_scene_near_cap_with_deep_radiance_map(product, oracle_built, monkeypatch):
    """an LDS-resident scene near the 48 KB cap with a deep radiance map.  k_fg stages its
    primitive / material tables only while stack + scene + nearest-search column + tables fit 64 KB
    (fgStageTables, the same decision in the kernel and the launch), so the render runs and matches the
    oracle — with one lane per gather path and with one lane per request alike."""
    # a 426-triangle sphere in the box: 37 KB of BVH4 nodes + triangles, 24 stack levels (n = 15 leaves LDS)
    s = scenes.cornell_sphere(n=14, width=40, height=30, spp=1, integrator="photonmapping")
    spec = dataclasses.replace(s, render=dataclasses.replace(
        s.render, pm_photons=3_000_000, pm_search=50, pm_diffuse_radius=0.035, pm_bounces=5, pm_caustics=False,
        pm_final_gather=True, fg_samples=4))
    a, w, st = product.render_spec(spec)
    assert st["scene_in_lds"] == 1
    assert (8 * st["bvh_nodes"] + 3 * len(spec.tris)) * 16 >= 36 * 1024, st["bvh_nodes"]   # near the 48 KB cap
    assert st["radiance_photons"] > 1 << 15, st["radiance_photons"]   # kd depth >= 16: a 17-level nearest-search column
    o = oracle_built.OracleScene(spec, threads=8)
    orgba, ow, _ = o.render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    u = ulp_diff(a, orgba)
    assert u.max() <= ULP_TOL, f"{(u > ULP_TOL).sum()} values > {ULP_TOL} ULP"
    monkeypatch.setenv("YAFARAY_AMD_FG", "lane")
    b, wb, _ = product.render_spec(spec)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
