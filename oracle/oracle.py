"""TEST INFRASTRUCTURE ONLY — ctypes bindings for the CPU oracle (liboracle.so) and for the
reference's own numeric building blocks (oracle/_ref/libyafref_prims.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.  The
product path (libyafaray_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libyafref_prims.so")

YC_MAT_SHINYDIFFUSE, YC_MAT_LIGHT = 0, 1
YC_LIGHT_POINT, YC_LIGHT_AREA = 0, 1
YC_INT_DIRECT, YC_INT_PATH, YC_INT_PHOTON = 0, 1, 2
FILTERS = {"box": 0, "gauss": 1, "mitchell": 2, "lanczos": 3}


class yc_material(C.Structure):
    _fields_ = [("type", C.c_int), ("color", C.c_float * 3), ("diffuse_strength", C.c_float),
                ("emit_strength", C.c_float), ("double_sided", C.c_int), ("receive_shadows", C.c_int),
                ("flat_material", C.c_int)]


class yc_light(C.Structure):
    _fields_ = [("type", C.c_int), ("color", C.c_float * 3), ("power", C.c_float), ("from_", C.c_float * 3),
                ("point1", C.c_float * 3), ("point2", C.c_float * 3), ("samples", C.c_int),
                ("cast_shadows", C.c_int)]


class yc_camera(C.Structure):
    _fields_ = [("from_", C.c_float * 3), ("to", C.c_float * 3), ("up", C.c_float * 3), ("resx", C.c_int),
                ("resy", C.c_int), ("focal", C.c_float), ("aspect", C.c_float), ("near_clip", C.c_float),
                ("far_clip", C.c_float), ("aperture", C.c_float), ("dof_distance", C.c_float),
                ("bokeh_rotation", C.c_float), ("bokeh_type", C.c_int), ("bokeh_bias", C.c_int)]


class yc_render(C.Structure):
    _fields_ = [("integrator", C.c_int), ("width", C.c_int), ("height", C.c_int), ("aa_samples", C.c_int),
                ("filter", C.c_int), ("filter_size", C.c_float), ("tile_size", C.c_int), ("bounces", C.c_int),
                ("path_samples", C.c_int), ("rr_min_bounces", C.c_int), ("caustic_path", C.c_int),
                ("has_background", C.c_int), ("bg_color", C.c_float * 3), ("bg_transp", C.c_int),
                ("shadow_bias_auto", C.c_int), ("shadow_bias", C.c_float), ("ray_min_dist_auto", C.c_int),
                ("ray_min_dist", C.c_float), ("base_sampling_offset", C.c_int), ("clamp_samples", C.c_float),
                ("threads", C.c_int), ("rr_seed", C.c_uint32), ("pm_photons", C.c_int), ("pm_search", C.c_int),
                ("pm_diffuse_radius", C.c_float), ("pm_bounces", C.c_int), ("pm_caustics", C.c_int),
                ("pm_threads", C.c_int), ("aa_passes", C.c_int), ("aa_inc_samples", C.c_int), ("aa_threshold", C.c_float),
                ("aa_resampled_floor", C.c_float), ("aa_sample_multiplier_factor", C.c_float),
                ("aa_detect_color_noise", C.c_int), ("aa_dark_detection_type", C.c_int),
                ("aa_dark_threshold_factor", C.c_float), ("aa_variance_edge_size", C.c_int), ("aa_variance_pixels", C.c_int)]


class yc_scene(C.Structure):
    _fields_ = [("n_verts", C.c_int), ("verts", C.POINTER(C.c_float)), ("n_tris", C.c_int),
                ("tris", C.POINTER(C.c_int)), ("tri_mat", C.POINTER(C.c_int)), ("n_mats", C.c_int),
                ("mats", C.POINTER(yc_material)), ("n_lights", C.c_int), ("lights", C.POINTER(yc_light)),
                ("cam", yc_camera), ("rp", yc_render)]


class yc_counters(C.Structure):
    _fields_ = [("closest_rays", C.c_uint64), ("shadow_rays", C.c_uint64)]


def build(quiet: bool = True) -> None:
    """Build liboracle.so (and oracle/_ref when the reference tree is present)."""
    out = subprocess.run(["make", "-C", HERE, "all"], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


_oracle = None
_ref = None


def oracle_lib():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            build()
        _oracle = C.CDLL(ORACLE_SO)
    return _oracle


def ref_lib():
    """The reference's own building blocks, or None when oracle/_ref was not built."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        _ref = C.CDLL(REF_SO)
    return _ref


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


# ---- numeric building blocks (same call shape on both libs: prefix 'yc_' or 'ref_') ----------

def prim_call(lib, prefix: str, name: str, *arrays_and_n):
    return getattr(lib, prefix + name)(*arrays_and_n)


class Prims:
    """Uniform numpy wrappers over either liboracle ('yc_') or the reference harness ('ref_')."""

    def __init__(self, lib, prefix):
        self.lib, self.px = lib, prefix

    def f(self, name):
        return getattr(self.lib, self.px + name)

    def ri(self, which, bits, r):
        bits = np.ascontiguousarray(bits, np.uint32)
        r = np.ascontiguousarray(r, np.uint32)
        out = np.empty(len(bits), np.float32)
        self.f(which)(_p(bits, C.c_uint32), _p(r, C.c_uint32), _p(out, C.c_float), C.c_int(len(bits)))
        return out

    def fnv32(self, v):
        v = np.ascontiguousarray(v, np.uint32)
        out = np.empty(len(v), np.uint32)
        self.f("fnv32")(_p(v, C.c_uint32), _p(out, C.c_uint32), C.c_int(len(v)))
        return out

    def lds(self, dim, idx):
        dim = np.ascontiguousarray(dim, np.int32)
        idx = np.ascontiguousarray(idx, np.uint32)
        out = np.empty(len(idx), np.float64)
        self.f("lds")(_p(dim, C.c_int), _p(idx, C.c_uint32), _p(out, C.c_double), C.c_int(len(idx)))
        return out

    def halton_seq(self, base, start, steps):
        out = np.empty(steps, np.float32)
        self.f("halton_seq")(C.c_int(base), C.c_uint32(start), C.c_int(steps), _p(out, C.c_float))
        return out

    def unary(self, name, x, width_out=1, width_in=1, ctype=C.c_float, otype=C.c_float, odt=np.float32,
              idt=np.float32):
        x = np.ascontiguousarray(x, idt)
        n = len(x) // width_in if x.ndim == 1 else x.shape[0]
        out = np.empty(n * width_out, odt)
        self.f(name)(_p(x, ctype), _p(out, otype), C.c_int(n))
        return out

    def cos_hemisphere(self, nrv, s):
        nrv = np.ascontiguousarray(nrv, np.float32).reshape(-1)
        s = np.ascontiguousarray(s, np.float32).reshape(-1)
        n = len(s) // 2
        out = np.empty(3 * n, np.float32)
        self.f("cos_hemisphere")(_p(nrv, C.c_float), _p(s, C.c_float), _p(out, C.c_float), C.c_int(n))
        return out.reshape(n, 3)

    def bound_cross(self, box, ray):
        box = np.ascontiguousarray(box, np.float32).reshape(-1)
        ray = np.ascontiguousarray(ray, np.float32).reshape(-1)
        n = len(box) // 6
        out = np.empty(3 * n, np.float32)
        self.f("bound_cross")(_p(box, C.c_float), _p(ray, C.c_float), _p(out, C.c_float), C.c_int(n))
        return out.reshape(n, 3)

    def mwc(self, seed, steps):
        out = np.empty(steps, np.float64)
        self.f("mwc")(C.c_uint32(seed), C.c_int(steps), _p(out, C.c_double))
        return out

    def clamp_proportional(self, rgb, mx):
        rgb = np.ascontiguousarray(rgb, np.float32).reshape(-1)
        out = np.empty_like(rgb)
        self.f("clamp_proportional")(_p(rgb, C.c_float), C.c_float(mx), _p(out, C.c_float), C.c_int(len(rgb) // 3))
        return out.reshape(-1, 3)

    def int_of_double(self, name, v):
        v = np.ascontiguousarray(v, np.float64)
        out = np.empty(len(v), np.int32)
        self.f(name)(_p(v, C.c_double), _p(out, C.c_int), C.c_int(len(v)))
        return out


def oracle_prims() -> Prims:
    return Prims(oracle_lib(), "yc_")


def ref_prims():
    lib = ref_lib()
    return Prims(lib, "ref_") if lib is not None else None


def film_table(filter_name: str, filter_size: float):
    lib = oracle_lib()
    tab = np.empty(256, np.float32)
    fw, ts = C.c_float(), C.c_float()
    lib.yc_film_table(C.c_int(FILTERS[filter_name]), C.c_float(filter_size), _p(tab, C.c_float), C.byref(fw),
                      C.byref(ts))
    return tab, fw.value, ts.value


# ---- scene-level oracle ------------------------------------------------------------------------

class OracleScene:
    """Owns the numpy buffers referenced by a yc_scene struct built from a SceneSpec."""

    def __init__(self, spec, threads: int = 1, rr_seed: int = 0):
        s = spec
        self.verts = np.ascontiguousarray(s.verts, np.float32).reshape(-1)
        self.tris = np.ascontiguousarray(s.tris, np.int32).reshape(-1)
        self.tri_mat = np.ascontiguousarray(s.tri_mat, np.int32).reshape(-1)
        mats = (yc_material * max(1, len(s.materials)))()
        for i, m in enumerate(s.materials):
            mats[i].type = YC_MAT_LIGHT if m.type == "light_mat" else YC_MAT_SHINYDIFFUSE
            if m.type == "light_mat":
                mats[i].color[:] = [np.float32(c) * np.float32(m.power) for c in m.color]
            else:
                mats[i].color[:] = list(m.color)
            mats[i].diffuse_strength = m.diffuse_reflect
            mats[i].emit_strength = m.emit
            mats[i].double_sided = int(m.double_sided)
            mats[i].receive_shadows = int(m.receive_shadows)
            mats[i].flat_material = int(m.flat_material)
        lights = (yc_light * max(1, len(s.lights)))()
        for i, l in enumerate(s.render_lights()):
            lights[i].type = YC_LIGHT_POINT if l.type == "pointlight" else YC_LIGHT_AREA
            lights[i].color[:] = list(l.color)
            lights[i].power = l.power
            lights[i].from_[:] = list(l.from_ if l.type == "pointlight" else l.corner)
            lights[i].point1[:] = list(l.point1)
            lights[i].point2[:] = list(l.point2)
            lights[i].samples = l.samples
            lights[i].cast_shadows = int(l.cast_shadows)
        self.mats, self.lights = mats, lights
        sc = yc_scene()
        sc.n_verts = len(self.verts) // 3
        sc.verts = _p(self.verts, C.c_float)
        sc.n_tris = len(self.tris) // 3
        sc.tris = _p(self.tris, C.c_int)
        sc.tri_mat = _p(self.tri_mat, C.c_int)
        sc.n_mats = len(s.materials)
        sc.mats = C.cast(mats, C.POINTER(yc_material))
        sc.n_lights = len(s.lights)
        sc.lights = C.cast(lights, C.POINTER(yc_light))
        cam = s.camera
        sc.cam.from_[:] = list(cam.from_)
        sc.cam.to[:] = list(cam.to)
        sc.cam.up[:] = list(cam.up)
        sc.cam.resx, sc.cam.resy = cam.resx, cam.resy
        sc.cam.focal, sc.cam.aspect = cam.focal, cam.aspect_ratio
        sc.cam.near_clip, sc.cam.far_clip = cam.near_clip, cam.far_clip
        sc.cam.aperture, sc.cam.dof_distance, sc.cam.bokeh_rotation = cam.aperture, cam.dof_distance, cam.bokeh_rotation
        sc.cam.bokeh_type = {"disk2": 1, "triangle": 3, "square": 4, "pentagon": 5, "hexagon": 6, "ring": 7}.get(cam.bokeh_type, 0)
        sc.cam.bokeh_bias = {"center": 1, "edge": 2}.get(cam.bokeh_bias, 0)
        r = s.render
        rp = sc.rp
        rp.integrator = {"pathtracing": YC_INT_PATH, "photonmapping": YC_INT_PHOTON}.get(r.integrator, YC_INT_DIRECT)
        rp.width, rp.height = r.width, r.height
        rp.aa_samples = r.aa_samples
        rp.filter = FILTERS[r.filter_type]
        rp.filter_size = r.aa_pixelwidth
        rp.tile_size = r.tile_size
        rp.bounces, rp.path_samples, rp.rr_min_bounces = r.bounces, r.path_samples, r.rr_min_bounces
        rp.caustic_path = int(r.caustic_type in ("path", "both"))
        rp.has_background = int(s.background is not None)
        if s.background is not None:
            rp.bg_color[:] = [np.float32(c) * np.float32(s.background.power) for c in s.background.color]
        rp.bg_transp = int(r.bg_transp)
        rp.shadow_bias_auto, rp.shadow_bias = int(r.shadow_bias_auto), r.shadow_bias
        rp.ray_min_dist_auto, rp.ray_min_dist = int(r.ray_min_dist_auto), r.ray_min_dist
        rp.base_sampling_offset = r.base_sampling_offset
        rp.clamp_samples = r.clamp_samples
        rp.threads = threads
        rp.rr_seed = rr_seed
        rp.pm_photons, rp.pm_search, rp.pm_diffuse_radius = r.pm_photons, r.pm_search, r.pm_diffuse_radius
        rp.pm_bounces, rp.pm_caustics, rp.pm_threads = r.pm_bounces, int(r.pm_caustics), r.threads_photons
        rp.aa_passes = max(1, r.aa_passes)
        rp.aa_inc_samples = r.aa_inc_samples if r.aa_inc_samples > 0 else r.aa_samples
        rp.aa_threshold, rp.aa_resampled_floor = r.aa_threshold, r.aa_resampled_floor
        rp.aa_sample_multiplier_factor = r.aa_sample_multiplier_factor
        rp.aa_detect_color_noise = int(r.aa_detect_color_noise)
        rp.aa_dark_detection_type = {"linear": 1, "curve": 2}.get(r.aa_dark_detection_type, 0)
        rp.aa_dark_threshold_factor = r.aa_dark_threshold_factor
        rp.aa_variance_edge_size, rp.aa_variance_pixels = r.aa_variance_edge_size, r.aa_variance_pixels
        self.sc = sc
        self.spec = spec

    def render(self, y0: int = 0, y1: int = 0):
        r = self.spec.render
        rgba = np.zeros(r.width * r.height * 4, np.float32)
        w = np.zeros(r.width * r.height, np.float32)
        ctr = yc_counters()
        oracle_lib().yc_render_image(C.byref(self.sc), C.c_int(y0), C.c_int(y1), _p(rgba, C.c_float),
                                     _p(w, C.c_float), C.byref(ctr))
        return rgba.reshape(r.height, r.width, 4), w.reshape(r.height, r.width), (ctr.closest_rays, ctr.shadow_rays)

    def photon_map(self):
        """(pos, dir, col [n x 3 each], kd nodes [m x 2 uint32], n_paths) of the diffuse photon map."""
        L = oracle_lib()
        n_paths = C.c_int(0)
        n = L.yc_photon_map(C.byref(self.sc), None, None, None, None, C.byref(n_paths))
        if n < 0:
            raise RuntimeError("photon map failed (too few photons)")
        pos, d, col = (np.empty(3 * n, np.float32) for _ in range(3))
        nodes = np.empty(2 * max(1, 2 * n - 1), np.uint32)
        L.yc_photon_map(C.byref(self.sc), _p(pos, C.c_float), _p(d, C.c_float), _p(col, C.c_float),
                        _p(nodes, C.c_uint32), C.byref(n_paths))
        return pos.reshape(n, 3), d.reshape(n, 3), col.reshape(n, 3), nodes.reshape(-1, 2)[:max(0, 2 * n - 1)], n_paths.value

    def render_samples(self, xys):
        xys = np.ascontiguousarray(xys, np.int32).reshape(-1)
        n = len(xys) // 3
        out = np.empty(4 * n, np.float32)
        oracle_lib().yc_render_samples(C.byref(self.sc), C.c_int(n), _p(xys, C.c_int), _p(out, C.c_float))
        return out.reshape(n, 4)

    def trace_closest(self, rays):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1)
        n = len(rays) // 8
        hit = np.empty(4 * n, np.float32)
        prim = np.empty(n, np.int32)
        oracle_lib().yc_trace_closest(C.byref(self.sc), C.c_int(n), _p(rays, C.c_float), _p(hit, C.c_float),
                                      _p(prim, C.c_int))
        return hit.reshape(n, 4), prim

    def trace_shadow(self, rays):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1)
        n = len(rays) // 8
        occ = np.empty(n, np.int32)
        oracle_lib().yc_trace_shadow(C.byref(self.sc), C.c_int(n), _p(rays, C.c_float), _p(occ, C.c_int))
        return occ
