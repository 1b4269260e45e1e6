"""The drop-in boundary on CPU: libyafaray4.so loads, exports every symbol the headers declare
under the reference's version node, stages a whole scene through the C API, and fails loudly
(no CPU fallback) when there is no GPU."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    return set(re.findall(r"YAFARAY_C_API_EXPORT[^;]*?\b(yafaray_\w+)\s*\(", src))


def exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    syms = {}
    for line in out.splitlines():
        parts = line.split()
        if len(parts) == 3 and parts[1] == "T":
            name, _, ver = parts[2].partition("@")
            syms[name] = ver.strip("@")
    return syms


def test_every_declared_symbol_is_exported(product):
    syms = exported(product.LIB_PATH)
    api = declared("yafaray_c_api.h")
    ext = declared("yafaray_amd.h")
    assert len(api) >= 77, len(api)
    missing = sorted((api | ext) - set(syms))
    assert not missing, missing
    # the reference's names carry the reference's version node
    assert all(syms[s] == "LIBYAFARAY_4.0.0" for s in api), {s: syms[s] for s in api if syms[s] != "LIBYAFARAY_4.0.0"}
    assert all(syms[s].startswith("LIBYAFARAY_AMD_1.") for s in ext), {s: syms[s] for s in ext}
    # nothing else leaks out (reference: CXX_VISIBILITY_PRESET hidden, src/CMakeLists.txt:22)
    assert set(syms) == api | ext, sorted(set(syms) - api - ext)[:10]


def test_reference_api_names_cover_the_reference_header():
    ref = "/root/reference/include/public_api/yafaray_c_api.h"
    if not os.path.exists(ref):
        pytest.skip("reference tree absent")
    src = open(ref).read()
    ref_names = set(re.findall(r"YAFARAY_C_API_EXPORT[^;]*?\b(yafaray_\w+)\s*\(", src))
    assert ref_names == declared("yafaray_c_api.h")


def test_scene_staging_and_loud_failure_without_gpu(product):
    import torch
    from libyafaray_amd import scenes
    yi = product.Interface()
    spec = scenes.cornell(32, 24, spp=2)
    scenes.apply(spec, yi)
    assert yi.getSceneFilmWidth() == 32 and yi.getSceneFilmHeight() == 24
    if torch.cuda.is_available() or os.path.exists("/dev/kfd"):
        pytest.skip("GPU present: the render path is covered by the gpu tests")
    with pytest.raises(RuntimeError, match="no HIP device"):
        yi.render()
    yi.close()


def test_unsupported_plugins_rejected_reference_style(product):
    yi = product.Interface()
    yi.createScene()
    yi.paramsClearAll()
    yi.paramsSetString("type", "glass")
    assert yi.createMaterial("g") == 0           # material.cc:52-61: unknown/unsupported -> null
    yi.paramsClearAll()
    yi.paramsSetString("type", "photonmapping")
    yi.paramsSetBool("show_map", True)              # served (k_gather's nearest-photon requests)
    assert yi.createIntegrator("pm") == 1
    yi.paramsClearAll()
    yi.paramsSetString("type", "photonmapping")
    yi.paramsSetString("photon_maps_processing", "bogus")   # unknown mode: generate (factory :847)
    assert yi.createIntegrator("pm_bad") == 1
    yi.paramsClearAll()
    yi.paramsSetString("type", "photonmapping")     # reference defaults (final gathering on)
    assert yi.createIntegrator("pm2") == 1
    yi.paramsClearAll()
    yi.paramsSetString("type", "pathtracing")
    assert yi.createIntegrator("pm2") == 0          # duplicate name (scene.cc:419-422)
    yi.paramsClearAll()
    yi.paramsSetString("type", "photonmapping")
    yi.paramsSetBool("transpShad", True)            # final gathering with transparent shadows (k_fg<TSH>)
    assert yi.createIntegrator("pm3") == 1
    yi.paramsClearAll()
    yi.paramsSetString("type", "shinydiffusemat")
    assert yi.createMaterial("d") == 1
    yi.paramsClearAll()
    assert yi.createMaterial("d") == 0           # duplicate name
    yi.paramsClearAll()
    yi.paramsSetString("integrator_name", "missing")
    yi.setupRender()
    assert "existing" in yi.last_error()         # scene.cc:552-556
    yi.close()


def test_params_are_strictly_typed(product):
    # include/common/param.h getVal: a Float param does not satisfy an int request (and v.v.)
    yi = product.Interface()
    yi.createScene()
    yi.paramsClearAll()
    yi.paramsSetString("type", "arealight")
    yi.paramsSetFloat("samples", 3.0)            # wrong type: the default (4) is kept
    yi.paramsSetVector("corner", 0, 0, 0)
    yi.paramsSetVector("point1", 1, 0, 0)
    yi.paramsSetVector("point2", 0, 1, 0)
    assert yi.createLight("l") == 1
    yi.close()


CLIENTS = os.path.join(ROOT, "oracle", "_ref", "clients")


@pytest.mark.skipif(not os.path.isdir(CLIENTS), reason="reference clients not built (needs /root/reference at build time)")
@pytest.mark.parametrize("t", ["00", "01", "02", "03", "04"])
def test_reference_clients_link_and_run(product, tmp_path, t):
    """The reference's own C clients (tests/test0N/test0N.c), compiled against include/ and linked
    against libyafaray4.so.4, resolve every symbol and run to completion.  Without a GPU the render
    step logs the no-fallback error; unsupported plugin types are logged, never fatal."""
    exe = os.path.join(CLIENTS, f"test{t}")
    r = subprocess.run([exe], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-2000:]
    assert "symbol lookup error" not in out and "error while loading" not in out


def _versioned(product, name, version):
    """dlvsym: the given version of a versioned symbol (ctypes' getattr binds the default @@ one)."""
    import ctypes as C
    libc = C.CDLL(None)
    dlvsym = libc.dlvsym
    dlvsym.restype = C.c_void_p
    dlvsym.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p]
    addr = dlvsym(product.lib()._handle, name.encode(), version.encode())
    assert addr, f"{name}@{version} not found"
    return C.CFUNCTYPE(None, C.c_void_p, C.c_void_p)(addr)


def test_get_stats_versions_keep_their_struct_sizes(product):
    """yafaray_amd_getStats@LIBYAFARAY_AMD_1.0 writes only the 1.0 struct's bytes (a client linked
    against it allocates no more); the default @@LIBYAFARAY_AMD_1.4 writes every field through
    fg_thin_rounds (the header carried those before getStatsEx existed); getStatsEx copies
    min(size, sizeof) bytes."""
    import ctypes as C
    yi = product.Interface()
    yi.createScene()
    v10 = product.Stats.gather_visits.offset
    v14 = product.Stats.gather_queries.offset
    assert v14 > v10
    buf = (C.c_ubyte * (C.sizeof(product.Stats) + 64))()
    for fn, size in ((_versioned(product, "yafaray_amd_getStats", "LIBYAFARAY_AMD_1.0"), v10),
                     (_versioned(product, "yafaray_amd_getStats", "LIBYAFARAY_AMD_1.4"), v14),
                     (lambda h, p: yi.L.yafaray_amd_getStats(h, C.cast(p, C.POINTER(product.Stats))), v14)):
        C.memset(buf, 0xA5, C.sizeof(buf))
        fn(yi.h, C.addressof(buf))
        assert all(b == 0xA5 for b in bytes(buf)[size:]), "getStats wrote past its struct"
        assert any(b != 0xA5 for b in bytes(buf)[:v10])
    C.memset(buf, 0xA5, C.sizeof(buf))
    n = yi.L.yafaray_amd_getStatsEx(yi.h, C.cast(buf, C.POINTER(product.Stats)), 24)
    assert n == 24 and all(b == 0xA5 for b in bytes(buf)[24:])
    assert yi.L.yafaray_amd_getStatsEx(yi.h, C.cast(buf, C.POINTER(product.Stats)), 1 << 20) == C.sizeof(product.Stats)
    yi.close()


def test_build_info_and_group_report(product):
    """yafaray_amd_buildInfo names the device objects' flags (no variant flags in the product build);
    getGroupReport is valid JSON before any render (one GPU, no bounds)."""
    import json
    info = product.build_info()
    assert "arch=gfx950" in info and "extra=[]" in info, info
    yi = product.Interface()
    yi.createScene()
    r = yi.group_report()
    assert r["mode"] == "one GPU" and r["bounds"] == [] and r["member_ms"] == []
    yi.close()
