"""photon_maps_processing (integrator_photon_mapping.cc:279-385, 599-624, factory :844-847;
integrator_montecarlo.cc:546-637 for the PathIntegrator's caustic map, factory
integrator_path_tracer.cc:360-363):

* "generate-save" writes <film_load_save_path>_diffuse / _caustic / _fg_radiance.photonmap in the
  reference's PhotonMap::save format (photon.cc:89-110) — header, name, paths, search radius,
  kd-tree threads, count, position + colour per photon — followed by this library's direction
  block (photonfile.h), which the reference's loader never reads;
* "load" reads them (PhotonMap::load, photon.cc:54-87); any missing / invalid file turns the
  integrator into "generate-save" for good (:323);
* "reuse-previous" keeps the maps of this integrator's previous render; an empty map falls back to
  "generate" (:328-358);
* any other value generates.

Checked: the GPU's saved maps equal the oracle's maps (count, paths, positions and colours within
4 ULP) and carry the reference header; loading them back (a fresh scene) or reusing them renders
bit-identically to generating; a reference-format file (no directions, e.g. written by the
reference itself) loads with zero directions on the GPU exactly as in the oracle's restatement of
PhotonMap::load (<= 4 ULP); fallbacks as above; a device group writes the files once."""
import dataclasses
import os
import struct

import numpy as np
import pytest

from libyafaray_amd import scenes

HEADER = b"YAF_PHOTONMAPv1\0"
DIR_TAG = b"YAFAMD_PHOTON_DIRSv1\0"
MODES = {"generate": 0, "generate-save": 1, "load": 2, "reuse-previous": 3}


def read_map(path):
    """(name, paths, search_radius, threads, pos[n,3], col[n,3], dirs[n,3] or None)."""
    b = open(path, "rb").read()
    assert b.startswith(HEADER)
    o = len(HEADER)
    e = b.index(b"\0", o)
    name = b[o:e].decode()
    o = e + 1
    paths, radius, threads, n = struct.unpack_from("<ifiI", b, o)
    o += 16
    rec = np.frombuffer(b, np.float32, 6 * n, o).reshape(n, 6)
    o += 24 * n
    dirs = None
    if b[o:o + len(DIR_TAG)] == DIR_TAG:
        o += len(DIR_TAG)
        (nd,) = struct.unpack_from("<I", b, o)
        assert nd == n
        dirs = np.frombuffer(b, np.float32, 3 * n, o + 4).reshape(n, 3)
        o += 4 + 12 * n
    assert o == len(b), "trailing bytes"
    return name, paths, radius, threads, rec[:, :3], rec[:, 3:], dirs


def write_ref_map(path, name, paths, pos, col, threads=1):
    """A reference-format file (PhotonMap::save, no direction block)."""
    pos = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
    col = np.ascontiguousarray(col, np.float32).reshape(-1, 3)
    with open(path, "wb") as f:
        f.write(HEADER + name.encode() + b"\0")
        f.write(struct.pack("<ifiI", int(paths), 1.0, int(threads), len(pos)))
        f.write(np.concatenate([pos, col], axis=1).astype(np.float32).tobytes())


def _ulp(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7fffffff), a)
    b = np.where(b < 0, -(b & 0x7fffffff), b)
    return np.abs(a - b)


def pm_spec(base, mode="generate", fg=False, caustics=False, specular=False):
    if specular:
        s = scenes.cornell_specular(48, 36, spp=1, integrator="photonmapping", raydepth=3)
        s = s.with_render(pm_photons=20000, pm_search=50, pm_diffuse_radius=0.1, pm_bounces=5, pm_caustics=caustics,
                          pm_caustic_photons=20000, caustic_radius=0.05)
    else:
        s = scenes.cornell_photon(48, 36, spp=1, photons=20000, search=50, radius=0.1)
        s = s.with_render(pm_caustics=caustics)
    return s.with_render(pm_final_gather=fg, fg_samples=4, pm_maps_processing=mode, film_load_save_path=str(base))


def pt_spec(base, mode="generate"):
    s = scenes.cornell_specular(48, 36, spp=1, integrator="pathtracing", raydepth=3)
    s = s.with_render(caustic_type="photon", bounces=3, rr_min_bounces=3, path_samples=2, pm_caustic_photons=20000,
                      caustic_radius=0.15)
    return s.with_render(pm_maps_processing=mode, film_load_save_path=str(base))


def files(base):
    return {k: f"{base}_{k}.photonmap" for k in ("diffuse", "caustic", "fg_radiance")}


# ---------------------------------------------------------------------------------------------
# CPU: the oracle's restatement of PhotonMap::load
# ---------------------------------------------------------------------------------------------
def test_oracle_load_reference_files(oracle_built, tmp_path):
    base = tmp_path / "scene"
    gen = oracle_built.OracleScene(pm_spec(base), threads=4)
    a, wa, _ = gen.render()
    pos, d, col, nodes, paths = gen.photon_map("diffuse")
    write_ref_map(files(base)["diffuse"], "Diffuse Photon Map", paths, pos, col)
    # a missing caustic file would fail the load: the scene has caustics off
    ld = oracle_built.OracleScene(pm_spec(base, "load"), threads=4)
    b, wb, _ = ld.render()
    lpos, ld_dir, lcol, lnodes, lpaths = ld.photon_map("diffuse")
    assert np.array_equal(lpos, pos) and np.array_equal(lcol, col) and lpaths == paths
    assert np.array_equal(lnodes, nodes) and not ld_dir.any()
    assert np.array_equal(wa, wb) and np.isfinite(b).all()
    # zero directions only change the estimates' side test (integrator_photon_mapping.cc:966-970)
    assert np.abs(a - b).mean() < 0.05 * np.abs(a).mean()


def test_oracle_load_missing_file_generates(oracle_built, tmp_path):
    a, _, _ = oracle_built.OracleScene(pm_spec(tmp_path / "x"), threads=4).render()
    b, _, _ = oracle_built.OracleScene(pm_spec(tmp_path / "x", "load"), threads=4).render()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_map_file_helpers_round_trip(tmp_path):
    p = tmp_path / "m.photonmap"
    pos = np.random.default_rng(1).random((7, 3), np.float32)
    col = np.random.default_rng(2).random((7, 3), np.float32)
    write_ref_map(p, "Caustic Photon Map", 123, pos, col, threads=4)
    name, paths, radius, threads, p2, c2, dirs = read_map(p)
    assert (name, paths, radius, threads) == ("Caustic Photon Map", 123, 1.0, 4) and dirs is None
    assert np.array_equal(p2, pos) and np.array_equal(c2, col)


# ---------------------------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(), dict(fg=True), dict(specular=True, caustics=True, fg=True)],
                         ids=["diffuse", "fg", "caustics-fg"])
def test_generate_save_then_load_is_bit_identical(product, oracle_built, tmp_path, kw):
    base = tmp_path / "scene"
    ref, wref, st0 = product.render_spec(pm_spec(base, **kw))
    assert st0["photon_maps_mode"] == 0 and not os.path.exists(files(base)["diffuse"])
    a, wa, st1 = product.render_spec(pm_spec(base, "generate-save", **kw))
    assert st1["photon_maps_mode"] == 1
    assert np.array_equal(a.view(np.uint32), ref.view(np.uint32)) and np.array_equal(wa, wref)
    # the files: reference header and fields, the oracle's maps, the direction block
    o = oracle_built.OracleScene(pm_spec(base, **kw), threads=8)
    want = [("diffuse", "Diffuse Photon Map", "diffuse")]
    if kw.get("caustics"):
        want.append(("caustic", "Caustic Photon Map", "caustic"))
    if kw.get("fg"):
        want.append(("fg_radiance", "FG Radiance Photon Map", "radiance"))
    for key, name, which in want:
        fname, paths, radius, threads, pos, col, dirs = read_map(files(base)[key])
        opos, odir, ocol, _, opaths = o.photon_map(which)
        assert fname == name and radius == 1.0 and threads >= 1
        assert paths == (0 if which == "radiance" else opaths)
        assert len(pos) == len(opos) > 0 and dirs is not None
        assert _ulp(pos, opos).max() <= 4 and _ulp(col, ocol).max() <= 4
    for key in ("diffuse", "caustic", "fg_radiance"):
        assert os.path.exists(files(base)[key]) == any(w[0] == key for w in want)
    # load them back in a fresh scene: the generated render, bit for bit, without shooting
    b, wb, st2 = product.render_spec(pm_spec(base, "load", **kw), profile=True)
    assert st2["photon_maps_mode"] == 2
    assert np.array_equal(b.view(np.uint32), ref.view(np.uint32)) and np.array_equal(wb, wref)
    assert st2["photons"] == st1["photons"] and st2["kernel_times"].get("k_photon_emit", {}).get("launches", 0) == 0


@pytest.mark.gpu
def test_pathtracer_caustic_map_files(product, tmp_path):
    base = tmp_path / "pt"
    ref, _, st0 = product.render_spec(pt_spec(base, "generate-save"))
    assert st0["photon_maps_mode"] == 1 and st0["caustic_photons"] > 0
    assert os.path.exists(files(base)["caustic"]) and not os.path.exists(files(base)["diffuse"])
    b, _, st1 = product.render_spec(pt_spec(base, "load"))
    assert st1["photon_maps_mode"] == 2 and st1["caustic_photons"] == st0["caustic_photons"]
    assert np.array_equal(b.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("fg", [False, True])
def test_reference_format_files_match_oracle(product, oracle_built, tmp_path, fg):
    """Files without directions (the reference's own): the GPU loads zero directions like the
    oracle's restatement of PhotonMap::load; with final gathering the radiance map's normals are
    zero too, so findNearest (photon.cc:136-164, n * dir > 0) never accepts a radiance photon."""
    base = tmp_path / "ref"
    o = oracle_built.OracleScene(pm_spec(base, fg=fg), threads=8)
    pos, _, col, _, paths = o.photon_map("diffuse")
    write_ref_map(files(base)["diffuse"], "Diffuse Photon Map", paths, pos, col)
    if fg:
        rpos, _, rcol, _, _ = o.photon_map("radiance")
        write_ref_map(files(base)["fg_radiance"], "FG Radiance Photon Map", 0, rpos, rcol)
    spec = pm_spec(base, "load", fg=fg)
    rgba, w, st = product.render_spec(spec)
    assert st["photon_maps_mode"] == 2
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w, ow)
    d = _ulp(rgba, orgba)
    assert d.max() <= 4, f"{(d > 4).sum()} values > 4 ULP"


@pytest.mark.gpu
def test_load_fallbacks(product, tmp_path):
    base = tmp_path / "missing"
    ref, _, _ = product.render_spec(pm_spec(base, fg=True))
    # a missing file: generate and save, and the integrator stays in generate-save
    yi = product.Interface()
    scenes.apply(pm_spec(base, "load", fg=True), yi)
    yi.render()
    a, _ = yi.film()
    assert yi.stats()["photon_maps_mode"] == 1
    assert os.path.exists(files(base)["diffuse"]) and os.path.exists(files(base)["fg_radiance"])
    assert np.array_equal(a.view(np.uint32), ref.view(np.uint32))
    os.remove(files(base)["diffuse"])
    yi.render()
    assert yi.stats()["photon_maps_mode"] == 1 and os.path.exists(files(base)["diffuse"])
    yi.close()
    # an invalid header fails the load as a missing file does
    with open(files(base)["diffuse"], "r+b") as f:
        f.write(b"NOT_A_MAP")
    b, _, st = product.render_spec(pm_spec(base, "load", fg=True))
    assert st["photon_maps_mode"] == 1 and np.array_equal(b.view(np.uint32), ref.view(np.uint32))
    # a corrupt photon count (2^32 - 1 records announced, none present) is a truncated file: the
    # loader checks the file length before it allocates, and the integrator generates and saves
    write_ref_map(files(base)["diffuse"], "Diffuse Photon Map", 1, np.zeros((0, 3)), np.zeros((0, 3)))
    with open(files(base)["diffuse"], "r+b") as f:
        f.seek(len(HEADER) + len(b"Diffuse Photon Map\0") + 12)
        f.write(struct.pack("<I", 0xFFFFFFFF))
    b, _, st = product.render_spec(pm_spec(base, "load", fg=True))
    assert st["photon_maps_mode"] == 1 and np.array_equal(b.view(np.uint32), ref.view(np.uint32))
    # an unknown value generates (factory :847)
    c, _, st = product.render_spec(pm_spec(base, "bogus", fg=True))
    assert st["photon_maps_mode"] == 0 and np.array_equal(c.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
def test_reuse_previous(product, tmp_path):
    """Deliberate extension: the reference turns a reuse-previous integrator whose
    maps are empty into PhotonsGenerateOnly for good (integrator_photon_mapping.cc:328-358), so a
    fresh integrator there never reuses anything; here the fallback holds for that render only and
    the second render reuses the maps the first one generated (the feature's documented intent)."""
    spec = pm_spec(tmp_path / "r", "reuse-previous", fg=True)
    ref, _, _ = product.render_spec(pm_spec(tmp_path / "r", fg=True))
    yi = product.Interface()
    yi.L.yafaray_amd_setProfileKernels(yi.h, 1)
    scenes.apply(spec, yi)
    yi.render()
    a, _ = yi.film()
    assert yi.stats()["photon_maps_mode"] == 0   # nothing to reuse yet: generate
    yi.render()
    b, _ = yi.film()
    st = yi.stats()
    assert st["photon_maps_mode"] == 3 and yi.kernel_times().get("k_photon_emit", {}).get("launches", 0) == 0
    assert st["photons"] > 0 and st["radiance_photons"] > 0
    yi.close()
    assert np.array_equal(a.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(b.view(np.uint32), ref.view(np.uint32))
    assert not any(os.path.exists(f) for f in files(tmp_path / "r").values())


@pytest.mark.gpu
def test_device_group_save_and_load(product, tmp_path):
    base = tmp_path / "grp"
    ref, _, _ = product.render_spec(pm_spec(base, fg=True))
    a, _, st = product.render_spec(pm_spec(base, "generate-save", fg=True), members=3)
    assert st["photon_maps_mode"] == 1 and np.array_equal(a.view(np.uint32), ref.view(np.uint32))
    one, _, _ = product.render_spec(pm_spec(tmp_path / "one", "generate-save", fg=True))
    for k in ("diffuse", "fg_radiance"):
        assert open(files(base)[k], "rb").read() == open(files(tmp_path / "one")[k], "rb").read()
    b, _, st = product.render_spec(pm_spec(base, "load", fg=True), members=3)
    assert st["photon_maps_mode"] == 2 and np.array_equal(b.view(np.uint32), ref.view(np.uint32))
    # reuse in a group: every member keeps the whole maps
    yi = product.Interface()
    scenes.apply(pm_spec(base, "reuse-previous", fg=True), yi)
    yi.set_device_group(3, None)
    yi.render()
    yi.render()
    c, _ = yi.film()
    assert yi.stats()["photon_maps_mode"] == 3
    yi.close()
    assert np.array_equal(c.view(np.uint32), ref.view(np.uint32))
