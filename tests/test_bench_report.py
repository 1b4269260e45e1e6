"""bench.py's reporting arithmetic on synthetic inputs (no GPU): the per-kernel table and the contract's
roofline object must never report rates from mismatched frames (a PMC pass that spans two frames
is per launch, scaled to the launches of one frame), and the dominant kernel's object carries both
the algorithmic and the measured HBM rate."""
import types

import bench


def _args(scene="cornell"):
    return types.SimpleNamespace(width=1920, height=1080, spp=64, scene=scene, fg=0)


def _stats():
    return {"closest_rays": 460_000_000, "shadow_rays": 290_000_000, "node_visits": 2_500_000_000, "tri_tests": 2_450_000_000,
            "bvh_width": 4, "scene_in_lds": 1, "photons": 0}


def _kt():
    # ms per frame, launches per frame, items per frame
    return {"k_shade": {"ms": 27.0, "launches": 24, "items": 460_000_000},
            "k_trace": {"ms": 26.5, "launches": 24, "items": 750_000_000},
            "k_nee": {"ms": 13.7, "launches": 24, "items": 328_000_000},
            "k_camera": {"ms": 1.0, "launches": 2, "items": 132_710_400},
            "k_film": {"ms": 1.1, "launches": 1, "items": 132_710_400}}


def _pmc():
    # a PMC pass over two frames: 48 dispatches of the per-iteration kernels, totals twice one frame's
    per = {"k_shade": 4.66e9, "k_trace": 1.58e9, "k_nee": 1.70e9, "k_camera": 3.18e9, "k_film": 5.5e9}
    disp = {"k_shade": 48, "k_trace": 48, "k_nee": 48, "k_camera": 4, "k_film": 2}
    return {"kernels": {k: {"dispatches": disp[k], "hbm_bytes_per_launch": v, "hbm_bytes_total": v * disp[k], "valu_lane_util": 0.5,
                            "sq_insts_valu_per_launch": 4e8} for k, v in per.items()}}


def test_traffic_is_per_frame_even_when_the_pmc_pass_spans_two_frames():
    a, s, kt = _args(), _stats(), _kt()
    kernels, frame_ms = bench.kernel_table(a, s, kt, _pmc())
    assert abs(frame_ms - sum(v["ms"] for v in kt.values())) < 1e-9
    for k, e in kernels.items():
        # bytes per frame = per launch x this frame's launches, so the rate is physical (< HBM peak)
        assert e["traffic_bytes"] == int(_pmc()["kernels"][k]["hbm_bytes_per_launch"] * kt[k]["launches"])
        assert e["traffic_frac"] < 1.0, (k, e)
    assert kernels["k_shade"]["algo_bytes_per_item"] == 64.0          # SURVEY §8d path-state model


def test_dominant_roofline_reports_algorithmic_and_measured_rates():
    a, s, kt = _args(), _stats(), _kt()
    kernels, _ = bench.kernel_table(a, s, kt, _pmc())
    roof = bench.dominant_roofline(s, kt, kernels, _pmc(), scene="cornell")
    assert roof["kernel"] == "k_shade" and roof["bound"] == "hbm"
    assert roof["peak"] == bench.HBM_PEAK_GBS
    assert abs(roof["frac"] - roof["achieved"] / bench.HBM_PEAK_GBS) < 1e-3
    assert roof["traffic"] == _pmc()["kernels"]["k_shade"]["hbm_bytes_per_launch"]
    assert 0.0 < roof["traffic_frac"] < 1.0
    # measured bytes per vertex in the limiter: 4.66e9 B per launch over 460 M / 24 entries
    assert "243 B per vertex" in roof["limiter"]


def test_dominant_roofline_for_trace_carries_the_survey_model_and_valu_limiter():
    a, s, kt = _args(), _stats(), _kt()
    kt["k_trace"]["ms"] = 40.0   # make k_trace the largest kernel
    kernels, _ = bench.kernel_table(a, s, kt, _pmc())
    roof = bench.dominant_roofline(s, kt, kernels, _pmc(), scene="cornell")
    assert roof["kernel"] == "k_trace"
    assert roof["survey_per_ray_model"]["closest_B"] == 273.0
    assert roof["traversal"]["served_from"] == "LDS"
    assert roof["limiter"].startswith("VALU")


def test_pkd_build_has_an_algorithmic_model():
    """C5's dominant kernel record (the kd-tree build) reports a roofline, not 0 GB/s: the model counts
    the top levels of the exact-median build (nodes of more than 256 photons)."""
    n = 19_646_342
    levels, m = 0, n
    while m > 256:
        m = (m + 1) // 2
        levels += 1
    assert levels == 17
    assert bench.pkd_build_bytes(0) == 0.0
    assert abs(bench.pkd_build_bytes(n) - n * (28 + 48 + 108 + 17 * 108 + 48 + 32 + 36)) < 1.0
    a, s = _args("photon"), dict(_stats(), photons=n)
    kt = {"pkd_build": {"ms": 20.0, "launches": 1, "items": n}, "k_gather": {"ms": 7.0, "launches": 1, "items": 2_000_000}}
    kernels, _ = bench.kernel_table(a, s, kt, None)
    roof = bench.dominant_roofline(s, kt, kernels, None, "photon")
    assert roof["kernel"] == "pkd_build" and roof["achieved"] > 1000.0 and 0.0 < roof["frac"] < 1.0


def test_multi_kernel_kind_traffic_is_per_frame():
    """pkd_build is ~160 dispatches per PMC pass (levels, sorts, subtrees) but one launch record per frame:
    its traffic is the pass's total over the frames the pass rendered (k_film dispatches), not one
    dispatch's average."""
    n = 19_646_342
    a, s = _args("photon"), dict(_stats(), photons=n)
    kt = {"pkd_build": {"ms": 19.3, "launches": 1, "items": n}, "k_film": {"ms": 0.07, "launches": 1, "items": 2_073_600}}
    pmc = {"kernels": {"pkd_build": {"dispatches": 162, "hbm_bytes_per_launch": 0.74e9, "hbm_bytes_total": 162 * 0.74e9},
                       "k_film": {"dispatches": 2, "hbm_bytes_per_launch": 0.33e9, "hbm_bytes_total": 0.66e9}}}
    kernels, _ = bench.kernel_table(a, s, kt, pmc)
    assert abs(kernels["pkd_build"]["traffic_bytes"] - 162 * 0.74e9 / 2) < 1e3
    roof = bench.dominant_roofline(s, kt, kernels, pmc, "photon")
    assert roof["kernel"] == "pkd_build" and abs(roof["traffic"] - 162 * 0.74e9 / 2) < 1e3


# --------------------------------------------------------------------------------------------------
# physical-possibility checks: no kernel may report an algorithmic rate above the
# HBM spec, nor a PMC-measured rate above the guide's measured achievable HBM bandwidth
# --------------------------------------------------------------------------------------------------
ACHIEVABLE_GBS = 6290.0   # MI355X_MICROARCH.md: measured achievable HBM read+write rate


def _physical(line):
    bad = []
    for k, e in (line.get("kernels") or {}).items():
        if e.get("frac") is not None and e["frac"] > 1.0:
            bad.append((k, "frac", e["frac"]))
        # the guide's 6.29 TB/s is a float4 copy (reads + writes); a kernel whose PMC traffic is >= 99 %
        # writes (k_camera: 32 B per sample streamed out, 6.2-6.4 TB/s) is bounded by the 8 TB/s peak only
        limit = bench.HBM_PEAK_GBS if (e.get("traffic_write_frac") or 0) >= 0.99 else ACHIEVABLE_GBS
        if e.get("traffic_gbs") is not None and e["traffic_gbs"] > limit:
            bad.append((k, "traffic_gbs", e["traffic_gbs"]))
    roof = line.get("roofline") or {}
    if roof.get("frac") is not None and roof["frac"] > 1.0:
        bad.append(("roofline", "frac", roof["frac"]))
    return bad


def test_k_camera_model_matches_its_32_byte_writes():
    """r05's line printed k_camera frac 1.026 with a stale 40-B model; the kernel writes 32 B per sample
    (24-B ray records + 8-B compact record; PMC WRITE_SIZE = 32.0 B x samples)."""
    a, s = _args(), _stats()
    kt = {"k_camera": {"ms": 0.647, "launches": 1, "items": 132_710_400}}   # r05: 0.647 ms per frame
    kernels, _ = bench.kernel_table(a, s, kt, None)
    assert kernels["k_camera"]["algo_bytes_per_item"] == 32.0
    assert kernels["k_camera"]["frac"] < 1.0
    assert not _physical({"kernels": kernels})


def test_pkd_build_charges_each_tree_its_own_points_and_pmc_is_per_frame():
    """C5 + FG builds two trees per frame (the 19.6 M-photon diffuse map and the 16 K-point radiance map):
    each is charged its own item count, and the PMC total of a frame is not multiplied by the two launch
    records (r05 printed 7.36 TB/s)."""
    n, nk = 19_646_342, 16_409
    s = dict(_stats(), photons=n, radiance_photons=nk)
    assert bench.pkd_trees(s, 2) == [n, nk]
    a = _args("photon")
    kt = {"pkd_build": {"ms": 16.2, "launches": 2, "items": n}, "k_film": {"ms": 0.07, "launches": 1, "items": 2_073_600}}
    # profiles/pmc_photon-...-fg32.json (r05): 556 pkd dispatches, 238.3 GB over the pass's 4 frames
    pmc = {"kernels": {"pkd_build": {"dispatches": 556, "hbm_bytes_per_launch": 0.4286e9, "hbm_bytes_total": 238.3e9},
                       "k_film": {"dispatches": 4, "hbm_bytes_per_launch": 0.334e9, "hbm_bytes_total": 1.336e9}}}
    kernels, _ = bench.kernel_table(a, s, kt, pmc)
    e = kernels["pkd_build"]
    assert abs(e["algo_bytes_per_item"] * n - (bench.pkd_build_bytes(n) + bench.pkd_build_bytes(nk))) < n
    assert abs(e["traffic_bytes"] - 238.3e9 / 4) < 1e3   # one frame's bytes, not x 2 launch records
    assert not _physical({"kernels": kernels}), _physical({"kernels": kernels})


def test_fg_and_pregather_models_count_their_lookups():
    a = _args("photon")
    s = dict(_stats(), fg_paths=60_000_000, fg_lookups=55_000_000, fg_nearest_visits=1_600_000_000,
             pregather_visits=20_000_000, pregather_photons=800_000)
    kt = {"k_fg": {"ms": 27.2, "launches": 1, "items": 2_000_000}, "k_pregather": {"ms": 2.7, "launches": 2, "items": 16_409}}
    kernels, _ = bench.kernel_table(a, s, kt, None)
    fg = kernels["k_fg"]["algo_bytes_per_item"] * 2_000_000
    assert abs(fg - (80 * 2e6 + 16 * 1.6e9 + 12 * 55e6 + 16 * 60e6)) < 2e6
    assert kernels["k_pregather"]["algo_bytes_per_item"] > 140.0
    assert kernels["k_fg"]["frac"] > 0.01   # r05's model excluded all of k_fg's work (frac 0.0007)
    assert not _physical({"kernels": kernels})


def test_committed_round6_lines_are_physically_possible():
    """Every committed bench line of this round (profiles/r06_*.json, BENCH_r06.json when present)."""
    import glob
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = sorted(glob.glob(os.path.join(root, "profiles", "r06_*.json"))) + [p for p in [os.path.join(root, "BENCH_r06.json")]
                                                                              if os.path.exists(p)]
    for p in paths:
        with open(p) as f:
            txt = f.read()
        lines = []
        for raw in txt.splitlines():
            raw = raw.strip()
            if raw.startswith("{") and '"kernels"' in raw:
                try:
                    lines.append(json.loads(raw))
                except ValueError:
                    pass
        if not lines:
            try:
                obj = json.loads(txt)
            except ValueError:
                continue
            obj = obj.get("parsed", obj) if isinstance(obj, dict) else None
            if isinstance(obj, dict) and "kernels" in obj:
                lines.append(obj)
        for line in lines:
            assert not _physical(line), (os.path.basename(p), _physical(line))
