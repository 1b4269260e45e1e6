"""libyafaray_amd — Python host mirror of libYafaRay's C API over the MI355X core (libyafaray4.so).

The shared library is the product: every call below is a thin ctypes forward to an extern "C"
symbol of include/yafaray_c_api.h (reference include/public_api/yafaray_c_api.h:53-130) or of the
MI355X extensions in include/yafaray_amd.h.  There is no Python or CPU fallback: importing works
without a GPU (so the C ABI can be inspected), but rendering / tracing raise if the HIP path
fails.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("YAFARAY_AMD_LIB") or os.path.join(HERE, "libyafaray4.so")

# enums (yafaray_c_api.h)
LOG_MUTE, LOG_ERROR, LOG_WARNING, LOG_PARAMS, LOG_INFO, LOG_VERBOSE, LOG_DEBUG = range(7)
CONSOLE_HIDDEN, CONSOLE_NORMAL = 0, 1

PutPixelCb = C.CFUNCTYPE(None, C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float,
                         C.c_void_p)
FlushAreaCb = C.CFUNCTYPE(None, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p)
FlushCb = C.CFUNCTYPE(None, C.c_char_p, C.c_void_p)
NotifyViewCb = C.CFUNCTYPE(None, C.c_char_p, C.c_void_p)
NotifyLayerCb = C.CFUNCTYPE(None, C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_void_p)
ProgressCb = C.CFUNCTYPE(None, C.c_int, C.c_int, C.c_char_p, C.c_void_p)
LoggerCb = C.CFUNCTYPE(None, C.c_int, C.c_long, C.c_char_p, C.c_char_p, C.c_void_p)


class Stats(C.Structure):
    _fields_ = [("closest_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("node_visits", C.c_uint64),
                ("tri_tests", C.c_uint64), ("samples", C.c_uint64), ("build_seconds", C.c_double),
                ("render_seconds", C.c_double), ("trace_kernel_ms", C.c_double), ("trace_launches", C.c_uint64),
                ("bvh_nodes", C.c_uint32), ("bvh_depth", C.c_uint32), ("scene_in_lds", C.c_uint32),
                ("bvh_width", C.c_uint32), ("trace_grid", C.c_uint32), ("shade_grid", C.c_uint32),
                ("trace_block", C.c_uint32), ("stack_depth", C.c_uint32), ("shade_kernel_ms", C.c_double),
                ("nee_kernel_ms", C.c_double), ("photons", C.c_uint64), ("photon_seconds", C.c_double),
                ("photon_shoot_seconds", C.c_double), ("photon_tree_seconds", C.c_double), ("gather_visits", C.c_uint64),
                ("caustic_photons", C.c_uint64), ("radiance_points", C.c_uint64), ("radiance_photons", C.c_uint64),
                ("fg_thin_seconds", C.c_double), ("fg_radiance_seconds", C.c_double), ("fg_thin_rounds", C.c_int64),
                ("gather_queries", C.c_uint64), ("gather_photons", C.c_uint64),
                ("photon_maps_mode", C.c_int32), ("reserved0", C.c_int32),
                ("gather_accepts", C.c_uint64), ("gather_overflows", C.c_uint64),
                ("photon_paths_traced", C.c_uint64), ("photon_slots", C.c_uint64),
                ("fg_paths", C.c_uint64), ("fg_lookups", C.c_uint64), ("fg_nearest_visits", C.c_uint64),
                ("pregather_visits", C.c_uint64), ("pregather_photons", C.c_uint64), ("pkd_split_level", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def build(quiet: bool = True) -> str:
    """Compile libyafaray4.so for gfx950 in-tree (libyafaray_amd/csrc/Makefile)."""
    import subprocess
    out = subprocess.run(["make", "-C", os.path.join(HERE, "csrc"), "-j8"], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("libyafaray4.so build failed:\n" + out.stdout[-4000:] + out.stderr[-4000:])
    if not quiet:
        print(out.stdout)
    return LIB_PATH


def lib():
    """Load libyafaray4.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run libyafaray_amd.build() (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        vp, cp, i, d, f, b = C.c_void_p, C.c_char_p, C.c_int, C.c_double, C.c_float, C.c_int
        sig = {
            "yafaray_createInterface": (vp, [i, cp, C.c_void_p, vp, i]),
            "yafaray_destroyInterface": (None, [vp]),
            "yafaray_createScene": (None, [vp]),
            "yafaray_getSceneFilmWidth": (i, [vp]),
            "yafaray_getSceneFilmHeight": (i, [vp]),
            "yafaray_startGeometry": (b, [vp]),
            "yafaray_endGeometry": (b, [vp]),
            "yafaray_endObject": (b, [vp]),
            "yafaray_addVertex": (i, [vp, d, d, d]),
            "yafaray_addVertexWithOrco": (i, [vp, d, d, d, d, d, d]),
            "yafaray_addTriangle": (b, [vp, i, i, i]),
            "yafaray_addTriangleWithUv": (b, [vp, i, i, i, i, i, i]),
            "yafaray_addUv": (i, [vp, f, f]),
            "yafaray_addNormal": (None, [vp, d, d, d]),
            "yafaray_smoothMesh": (b, [vp, cp, d]),
            "yafaray_createImage": (vp, [vp, cp]),
            "yafaray_setImageColor": (b, [vp, i, i, f, f, f, f]),
            "yafaray_getImageColor": (b, [vp, i, i, C.POINTER(f), C.POINTER(f), C.POINTER(f), C.POINTER(f)]),
            "yafaray_paramsSetMatrix": (None, [vp, cp] + [f] * 16 + [b]),
            "yafaray_paramsSetVector": (None, [vp, cp, d, d, d]),
            "yafaray_paramsSetString": (None, [vp, cp, cp]),
            "yafaray_paramsSetBool": (None, [vp, cp, b]),
            "yafaray_paramsSetInt": (None, [vp, cp, i]),
            "yafaray_paramsSetFloat": (None, [vp, cp, d]),
            "yafaray_paramsSetColor": (None, [vp, cp, f, f, f, f]),
            "yafaray_paramsClearAll": (None, [vp]),
            "yafaray_paramsPushList": (None, [vp]),
            "yafaray_paramsEndList": (None, [vp]),
            "yafaray_setCurrentMaterial": (None, [vp, cp]),
            "yafaray_createObject": (b, [vp, cp]),
            "yafaray_createLight": (b, [vp, cp]),
            "yafaray_createTexture": (b, [vp, cp]),
            "yafaray_createMaterial": (b, [vp, cp]),
            "yafaray_createCamera": (b, [vp, cp]),
            "yafaray_createBackground": (b, [vp, cp]),
            "yafaray_createIntegrator": (b, [vp, cp]),
            "yafaray_createRenderView": (b, [vp, cp]),
            "yafaray_createOutput": (b, [vp, cp]),
            "yafaray_setRenderPutPixelCallback": (None, [vp, PutPixelCb, vp]),
            "yafaray_setRenderFlushAreaCallback": (None, [vp, FlushAreaCb, vp]),
            "yafaray_setRenderHighlightAreaCallback": (None, [vp, FlushAreaCb, vp]),
            "yafaray_setRenderFlushCallback": (None, [vp, FlushCb, vp]),
            "yafaray_setRenderNotifyViewCallback": (None, [vp, NotifyViewCb, vp]),
            "yafaray_setRenderNotifyLayerCallback": (None, [vp, NotifyLayerCb, vp]),
            "yafaray_setupRender": (None, [vp]),
            "yafaray_render": (None, [vp, ProgressCb, vp, i]),
            "yafaray_defineLayer": (None, [vp]),
            "yafaray_setConsoleVerbosityLevel": (None, [vp, i]),
            "yafaray_setLogVerbosityLevel": (None, [vp, i]),
            "yafaray_cancelRendering": (None, [vp]),
            "yafaray_setInputColorSpace": (None, [vp, cp, f]),
            "yafaray_getVersionString": (vp, []),
            "yafaray_deallocateCharPointer": (None, [vp]),
            "yafaray_amd_addVertices": (i, [vp, C.POINTER(C.c_double), i]),
            "yafaray_amd_addTriangles": (b, [vp, C.POINTER(C.c_int), i]),
            "yafaray_amd_buildAccelerator": (b, [vp]),
            "yafaray_amd_traceClosest": (b, [vp, C.POINTER(C.c_float), i, C.POINTER(C.c_float), C.POINTER(C.c_int)]),
            "yafaray_amd_traceShadow": (b, [vp, C.POINTER(C.c_float), i, C.POINTER(C.c_int)]),
            "yafaray_amd_getFilm": (b, [vp, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
            "yafaray_amd_getFilmDevice": (b, [vp, vp, i, i]),
            "yafaray_amd_setTileRowShard": (None, [vp, i, i]),
            "yafaray_amd_setRowBandShard": (None, [vp, i, i]),
            "yafaray_amd_setRowBandRange": (None, [vp, i, i, i]),
            "yafaray_amd_getOwnedRows": (i, [vp, C.POINTER(C.c_int), i]),
            "yafaray_amd_renderQuiet": (b, [vp]),
            "yafaray_amd_getStats": (None, [vp, C.POINTER(Stats)]),
            "yafaray_amd_buildInfo": (cp, []),
            "yafaray_amd_getGroupReport": (C.c_size_t, [vp, C.c_char_p, C.c_size_t]),
            "yafaray_amd_getStatsEx": (C.c_size_t, [vp, C.POINTER(Stats), C.c_size_t]),
            "yafaray_amd_setDeviceGroup": (b, [vp, i, C.POINTER(C.c_int)]),
            "yafaray_amd_getDeviceGroupSize": (i, [vp]),
            "yafaray_amd_packBand": (i, [C.POINTER(C.c_float), i, i, i, C.POINTER(C.c_int), i, i, C.POINTER(C.c_float)]),
            "yafaray_amd_unpackBands": (i, [C.POINTER(C.c_float), i, i, i, C.POINTER(C.c_int), i, i, C.POINTER(C.c_float)]),
            "yafaray_amd_buildPhotonTree": (b, [C.POINTER(C.c_float), i, C.POINTER(C.c_uint32), C.POINTER(C.c_int)]),
            "yafaray_amd_buildPhotonTreeMember": (b, [C.POINTER(C.c_float), i, i, i, C.POINTER(C.c_uint32), C.POINTER(C.c_float),
                                                      C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double)]),
            "yafaray_amd_photonTreeSegments": (None, [C.c_uint, i, i, i, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                                      C.POINTER(C.c_uint32)]),
            "yafaray_amd_setChunkSlots": (None, [vp, i]),
            "yafaray_amd_setProfileKernels": (None, [vp, b]),
            "yafaray_amd_setTraceStats": (None, [vp, b]),
            "yafaray_amd_lastError": (cp, [vp]),
            "yafaray_amd_getRenderGroupId": (i, [vp, i]),
            "yafaray_amd_setRenderGroup": (b, [vp, i, i, vp, i]),
            "yafaray_amd_rebalanceBands": (i, [C.POINTER(C.c_int), i, C.POINTER(C.c_double), i, C.POINTER(C.c_int)]),
            "yafaray_amd_getKernelTimes": (i, [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                               C.POINTER(C.c_uint64), i]),
        }
        optional = {"yafaray_amd_buildInfo", "yafaray_amd_getGroupReport"}   # LIBYAFARAY_AMD_1.4 (variant builds of older sources lack them)
        for name, (res, args) in sig.items():
            if name in optional and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def build_info() -> str:
    """The library's build flags (yafaray_amd_buildInfo): device arch + extra flags, host compiler."""
    L = lib()
    return L.yafaray_amd_buildInfo().decode() if hasattr(L, "yafaray_amd_buildInfo") else "unknown (library before LIBYAFARAY_AMD_1.4)"


def lib_sha256() -> str:
    """sha256 of the loaded libyafaray4.so (bench.py prints it with build_info)."""
    import hashlib
    with open(LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def version() -> str:
    L = lib()
    p = L.yafaray_getVersionString()
    s = C.cast(p, C.c_char_p).value.decode()
    L.yafaray_deallocateCharPointer(p)
    return s


def _b(s):
    return s.encode() if isinstance(s, str) else s


class Interface:
    """One yafaray_Interface_t.  Method names are the C API's without the `yafaray_` prefix."""

    def __init__(self, console=CONSOLE_HIDDEN, verbosity=LOG_WARNING):
        self.L = lib()
        self.h = self.L.yafaray_createInterface(0, None, None, None, console)
        self.L.yafaray_setConsoleVerbosityLevel(self.h, verbosity)
        self._keep = []

    def close(self):
        if self.h:
            self.L.yafaray_destroyInterface(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- generic forwarding for simple calls ---
    def __getattr__(self, name):
        fn = getattr(lib(), "yafaray_" + name, None)
        if fn is None:
            raise AttributeError(name)

        def call(*args):
            return fn(self.h, *[_b(a) for a in args])
        return call

    # --- images (the handle is the first argument, not the interface) ---
    def setImageColor(self, image, x, y, r, g, b, a):
        return self.L.yafaray_setImageColor(image, x, y, r, g, b, a)

    def getImageColor(self, image, x, y):
        c = [C.c_float() for _ in range(4)]
        ok = self.L.yafaray_getImageColor(image, x, y, *[C.byref(v) for v in c])
        return tuple(v.value for v in c) if ok else None

    # --- bulk geometry (extensions) ---
    def addVertices(self, xyz):
        a = np.ascontiguousarray(xyz, np.float64).reshape(-1)
        return self.L.yafaray_amd_addVertices(self.h, a.ctypes.data_as(C.POINTER(C.c_double)), len(a) // 3)

    def addTriangles(self, abc):
        a = np.ascontiguousarray(abc, np.int32).reshape(-1)
        if not self.L.yafaray_amd_addTriangles(self.h, a.ctypes.data_as(C.POINTER(C.c_int)), len(a) // 3):
            raise RuntimeError(self.last_error())

    def last_error(self) -> str:
        e = self.L.yafaray_amd_lastError(self.h)
        return e.decode() if e else ""

    # --- render ---
    def render(self, progress=None, put_pixel=None, flush_area=None, flush=None, highlight_area=None):
        # every callback is (re)registered, a missing one as NULL (an empty CFUNCTYPE instance): the library
        # keeps the pointers between renders, and the previous render's ctypes thunks are released below
        # (self._keep) — a render without a callback after one with it called a freed thunk
        cbs = []
        cb = FlushAreaCb(lambda v, aid, x0, y0, x1, y1, d: highlight_area(aid, x0, y0, x1, y1)) if highlight_area is not None else FlushAreaCb()
        self.L.yafaray_setRenderHighlightAreaCallback(self.h, cb, None)
        cbs.append(cb)
        cb = PutPixelCb(lambda v, l, x, y, r, g, b, a, d: put_pixel(x, y, r, g, b, a)) if put_pixel is not None else PutPixelCb()
        self.L.yafaray_setRenderPutPixelCallback(self.h, cb, None)
        cbs.append(cb)
        cb = FlushAreaCb(lambda v, aid, x0, y0, x1, y1, d: flush_area(aid, x0, y0, x1, y1)) if flush_area is not None else FlushAreaCb()
        self.L.yafaray_setRenderFlushAreaCallback(self.h, cb, None)
        cbs.append(cb)
        cb = FlushCb(lambda v, d: flush()) if flush is not None else FlushCb()
        self.L.yafaray_setRenderFlushCallback(self.h, cb, None)
        cbs.append(cb)
        pcb = ProgressCb(lambda t, dn, tag, d: progress(t, dn) if progress else None)
        cbs.append(pcb)
        self._keep = cbs
        before = self.last_error()
        self.L.yafaray_render(self.h, pcb, None, CONSOLE_HIDDEN)
        err = self.last_error()
        if err and err != before:
            raise RuntimeError("yafaray_render failed: " + err)

    def render_quiet(self):
        if not self.L.yafaray_amd_renderQuiet(self.h):
            raise RuntimeError("render failed: " + self.last_error())

    def film(self):
        w, h = self.L.yafaray_getSceneFilmWidth(self.h), self.L.yafaray_getSceneFilmHeight(self.h)
        rgba = np.empty((h, w, 4), np.float32)
        wt = np.empty((h, w), np.float32)
        if not self.L.yafaray_amd_getFilm(self.h, rgba.ctypes.data_as(C.POINTER(C.c_float)),
                                          wt.ctypes.data_as(C.POINTER(C.c_float))):
            raise RuntimeError("no film: " + self.last_error())
        return rgba, wt

    def stats(self) -> dict:
        s = Stats()
        self.L.yafaray_amd_getStatsEx(self.h, C.byref(s), C.sizeof(s))
        return s.as_dict()

    def set_device_group(self, members, devices=None):
        """yafaray_amd_setDeviceGroup: `members` renderers of this process share the film (row bands);
        devices[m] = member m's HIP device (None: current device + m modulo the visible devices, so
        several logical members can share one GPU).  members <= 0: back to the "gpus" parameter."""
        arr = None
        if devices is not None:
            arr = (C.c_int * len(devices))(*[int(d) for d in devices])
        if not self.L.yafaray_amd_setDeviceGroup(self.h, int(members), arr):
            raise RuntimeError("setDeviceGroup failed: " + self.last_error())

    def device_group_size(self) -> int:
        return int(self.L.yafaray_amd_getDeviceGroupSize(self.h))

    def group_report(self) -> dict:
        """How the last render was split across GPUs (yafaray_amd_getGroupReport): mode, devices, the
        peer-access matrix, the band copy path, band bounds and each member's render time."""
        import json
        n = int(self.L.yafaray_amd_getGroupReport(self.h, None, 0))
        if n <= 0:
            raise RuntimeError("getGroupReport failed: " + self.last_error())
        buf = C.create_string_buffer(n)
        self.L.yafaray_amd_getGroupReport(self.h, buf, n)
        return json.loads(buf.value.decode())

    def kernel_times(self) -> dict:
        """{kernel: {"ms", "launches", "items"}} of the last render with profiling on (yafaray_amd_getKernelTimes)."""
        n = 32
        names = (C.c_char_p * n)()
        ms = (C.c_double * n)()
        la = (C.c_uint64 * n)()
        it = (C.c_uint64 * n)()
        k = self.L.yafaray_amd_getKernelTimes(self.h, names, ms, la, it, n)
        return {names[j].decode(): {"ms": ms[j], "launches": la[j], "items": it[j]} for j in range(min(k, n)) if la[j]}

    def owned_rows(self):
        """[(y0, y1), ...] pixel rows this rank's last render owns (yafaray_amd_getOwnedRows)."""
        n = self.L.yafaray_amd_getOwnedRows(self.h, None, 0)
        buf = (C.c_int * max(2, 2 * n))()
        self.L.yafaray_amd_getOwnedRows(self.h, buf, n)
        return [(buf[2 * k], buf[2 * k + 1]) for k in range(n)]

    def trace_closest(self, rays):
        r = np.ascontiguousarray(rays, np.float32).reshape(-1)
        n = len(r) // 8
        t = np.empty(n, np.float32)
        p = np.empty(n, np.int32)
        if not self.L.yafaray_amd_traceClosest(self.h, r.ctypes.data_as(C.POINTER(C.c_float)), n,
                                               t.ctypes.data_as(C.POINTER(C.c_float)),
                                               p.ctypes.data_as(C.POINTER(C.c_int))):
            raise RuntimeError("traceClosest failed: " + self.last_error())
        return t, p

    def trace_shadow(self, rays):
        r = np.ascontiguousarray(rays, np.float32).reshape(-1)
        n = len(r) // 8
        o = np.empty(n, np.int32)
        if not self.L.yafaray_amd_traceShadow(self.h, r.ctypes.data_as(C.POINTER(C.c_float)), n,
                                              o.ctypes.data_as(C.POINTER(C.c_int))):
            raise RuntimeError("traceShadow failed: " + self.last_error())
        return o


def render_group_id() -> bytes:
    """A fresh render-group id (RCCL unique id) for yafaray_amd_setRenderGroup."""
    buf = C.create_string_buffer(128)
    n = lib().yafaray_amd_getRenderGroupId(buf, 128)
    if n <= 0:
        raise RuntimeError("yafaray_amd_getRenderGroupId failed")
    return buf.raw[:n]


def join_render_group(yi, rank, world, dist):
    """Make `yi` member `rank` of a `world`-GPU render group (one process per GPU): rank 0 creates
    the id, torch.distributed broadcasts it, every member joins on its current HIP device.  The
    library then splits every render into row bands and all-gathers them over RCCL itself."""
    obj = [render_group_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(obj, src=0)
    gid = obj[0]
    if not yi.L.yafaray_amd_setRenderGroup(yi.h, int(rank), int(world), gid, len(gid)):
        raise RuntimeError("setRenderGroup failed: " + yi.last_error())


def build_photon_tree(xyz):
    """The GPU point kd-tree of n positions ((n, 3) float32): ((2n - 1, 4) uint32 nodes, depth) in
    the reference's depth-first layout (yafaray_amd_buildPhotonTree)."""
    import numpy as np
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    n = int(xyz.shape[0])
    nodes = np.zeros((2 * n - 1, 4), np.uint32)
    depth = C.c_int(0)
    ok = lib().yafaray_amd_buildPhotonTree(xyz.ctypes.data_as(C.POINTER(C.c_float)), n,
                                           nodes.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(depth))
    if not ok:
        raise RuntimeError("yafaray_amd_buildPhotonTree failed")
    return nodes, depth.value


def build_photon_tree_member(xyz, member, members):
    """A group member's share of the distributed point kd-tree build (yafaray_amd_buildPhotonTreeMember):
    (nodes (2n - 1, 4) uint32, kd-order positions (n, 4) float32, depth, split level, device ms)."""
    import numpy as np
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    n = int(xyz.shape[0])
    nodes = np.zeros((2 * n - 1, 4), np.uint32)
    kd = np.zeros((n, 4), np.float32)
    depth, level, ms = C.c_int(0), C.c_int(0), C.c_double(0)
    ok = lib().yafaray_amd_buildPhotonTreeMember(xyz.ctypes.data_as(C.POINTER(C.c_float)), n, member, members,
                                                 nodes.ctypes.data_as(C.POINTER(C.c_uint32)), kd.ctypes.data_as(C.POINTER(C.c_float)),
                                                 C.byref(depth), C.byref(level), C.byref(ms))
    if not ok:
        raise RuntimeError("yafaray_amd_buildPhotonTreeMember failed")
    return nodes, kd, depth.value, level.value, ms.value


def photon_tree_segments(n, level, member=0, members=1):
    """The level-`level` subtrees of a tree over n photons ((2^level, 3) uint32: node, start, end) and the
    owned range [s0, s1) of member `member` (yafaray_amd_photonTreeSegments)."""
    import numpy as np
    seg = np.zeros((1 << level, 3), np.uint32)
    s0, s1 = C.c_uint32(0), C.c_uint32(0)
    lib().yafaray_amd_photonTreeSegments(n, level, member, members, seg.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(s0), C.byref(s1))
    return seg, (s0.value, s1.value)


def rebalance_bands(bounds, times, cap_rows=0):
    """The library's band balancer (yafaray_amd_rebalanceBands)."""
    world = len(bounds) - 1
    b = (C.c_int * (world + 1))(*bounds)
    t = (C.c_double * world)(*times)
    out = (C.c_int * (world + 1))()
    lib().yafaray_amd_rebalanceBands(b, world, t, int(cap_rows), out)
    return list(out)


def pack_band(film, bounds, rank):
    """The library's band plan (yafaray_amd_packBand): `rank`'s rows of a (H, W, C) float32 film in a
    zero-padded (max band rows, W, C) buffer, as the render group sends it."""
    film = np.ascontiguousarray(film, np.float32)
    H, W = film.shape[:2]
    ch = 1 if film.ndim == 2 else film.shape[2]
    world = len(bounds) - 1
    rows = max(bounds[r + 1] - bounds[r] for r in range(world))
    out = np.zeros((rows, W) + film.shape[2:], np.float32)
    b = (C.c_int * (world + 1))(*bounds)
    fp = C.POINTER(C.c_float)
    if not lib().yafaray_amd_packBand(film.ctypes.data_as(fp), W, H, ch, b, world, int(rank), out.ctypes.data_as(fp)):
        raise RuntimeError("packBand failed")
    return out


def unpack_bands(gathered, bounds, rank, film):
    """The library's band plan (yafaray_amd_unpackBands): every other member's rows of an all-gather
    result (world * max band rows, W, C) into `film` (H, W, C), in place; `rank`'s own rows stay."""
    gathered = np.ascontiguousarray(gathered, np.float32)
    assert film.dtype == np.float32 and film.flags["C_CONTIGUOUS"]
    H, W = film.shape[:2]
    ch = 1 if film.ndim == 2 else film.shape[2]
    world = len(bounds) - 1
    b = (C.c_int * (world + 1))(*bounds)
    fp = C.POINTER(C.c_float)
    if not lib().yafaray_amd_unpackBands(gathered.ctypes.data_as(fp), W, H, ch, b, world, int(rank), film.ctypes.data_as(fp)):
        raise RuntimeError("unpackBands failed")
    return film


def render_spec(spec, chunk_slots=None, profile=False, shard=None, members=None, devices=None):
    """Replay a scenes.SceneSpec through the C API and render it; returns (rgba, weights, stats).
    members: a device group of this many members (set_device_group)."""
    from . import scenes
    yi = Interface()
    scenes.apply(spec, yi)
    if members is not None:
        yi.set_device_group(members, devices)
    if chunk_slots:
        yi.L.yafaray_amd_setChunkSlots(yi.h, int(chunk_slots))
    if profile:
        yi.L.yafaray_amd_setProfileKernels(yi.h, 1)
    if shard is not None:
        # (rank, world[, mode]): mode "band" (default, contiguous row band) or "tile" (tile rows r % world)
        fn = yi.L.yafaray_amd_setTileRowShard if (len(shard) > 2 and shard[2] == "tile") else yi.L.yafaray_amd_setRowBandShard
        fn(yi.h, int(shard[0]), int(shard[1]))
    yi.render()
    rgba, w = yi.film()
    st = yi.stats()
    st["owned_rows"] = yi.owned_rows()
    if profile:
        st["kernel_times"] = yi.kernel_times()
    yi.close()
    return rgba, w, st
