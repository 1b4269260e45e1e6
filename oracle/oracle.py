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
YC_LIGHT_POINT, YC_LIGHT_AREA, YC_LIGHT_MESH = 0, 1, 2
YC_INT_DIRECT, YC_INT_PATH, YC_INT_PHOTON = 0, 1, 2
FILTERS = {"box": 0, "gauss": 1, "mitchell": 2, "lanczos": 3}


class yc_material(C.Structure):
    _fields_ = [("type", C.c_int), ("color", C.c_float * 3), ("diffuse_strength", C.c_float),
                ("emit_strength", C.c_float), ("double_sided", C.c_int), ("receive_shadows", C.c_int),
                ("flat_material", C.c_int), ("diffuse_shader", C.c_int), ("diffuse_refl_shader", C.c_int),
                ("specular_reflect", C.c_float), ("transparency", C.c_float), ("translucency", C.c_float),
                ("transmit_filter", C.c_float), ("ior", C.c_float), ("fresnel_effect", C.c_int), ("mirror_color", C.c_float * 3),
                ("transparentbias_factor", C.c_float), ("transparentbias_multiply_raydepth", C.c_int), ("reflect", C.c_float),
                ("additional_depth", C.c_int), ("oren_nayar", C.c_int), ("sigma", C.c_double), ("sigma_shader", C.c_int)]


class yc_image(C.Structure):
    _fields_ = [("format", C.c_int), ("data", C.POINTER(C.c_uint8)), ("size", C.c_int), ("type", C.c_int),
                ("optimization", C.c_int), ("color_space", C.c_int), ("gamma", C.c_float), ("width", C.c_int),
                ("height", C.c_int), ("n_set", C.c_int), ("set_xy", C.POINTER(C.c_int)), ("set_rgba", C.POINTER(C.c_float))]


class yc_texture(C.Structure):
    _fields_ = [("image", C.c_int), ("interpolation", C.c_int), ("clip", C.c_int), ("xrepeat", C.c_int),
                ("yrepeat", C.c_int), ("mirror_x", C.c_int), ("mirror_y", C.c_int), ("rot90", C.c_int),
                ("even_tiles", C.c_int), ("odd_tiles", C.c_int), ("cropmin_x", C.c_float), ("cropmin_y", C.c_float),
                ("cropmax_x", C.c_float), ("cropmax_y", C.c_float), ("checker_dist", C.c_float), ("intensity", C.c_float),
                ("contrast", C.c_float), ("saturation", C.c_float), ("hue", C.c_float), ("factor_red", C.c_float),
                ("factor_green", C.c_float), ("factor_blue", C.c_float), ("clamp", C.c_int)]


class yc_node(C.Structure):
    _fields_ = [("type", C.c_int), ("blend", C.c_int), ("input", C.c_int * 3), ("no_rgb", C.c_int), ("stencil", C.c_int),
                ("negative", C.c_int), ("do_color", C.c_int), ("do_scalar", C.c_int), ("color_input", C.c_int),
                ("use_alpha", C.c_int), ("texture", C.c_int), ("coords", C.c_int), ("projection", C.c_int),
                ("map", C.c_int * 3), ("col1", C.c_float * 4), ("col2", C.c_float * 4), ("val", C.c_float * 4),
                ("scale", C.c_float * 3), ("offset", C.c_float * 3), ("mtx", C.c_float * 16)]


class yc_object(C.Structure):
    _fields_ = [("v0", C.c_int), ("nv", C.c_int), ("t0", C.c_int), ("nt", C.c_int), ("has_orco", C.c_int),
                ("has_uv", C.c_int), ("normals_exported", C.c_int), ("smooth", C.c_int), ("smooth_angle", C.c_float)]


class yc_light(C.Structure):
    _fields_ = [("type", C.c_int), ("color", C.c_float * 3), ("power", C.c_float), ("from_", C.c_float * 3),
                ("point1", C.c_float * 3), ("point2", C.c_float * 3), ("samples", C.c_int),
                ("cast_shadows", C.c_int), ("shoot_caustic", C.c_int), ("shoot_diffuse", C.c_int),
                ("object", C.c_int), ("double_sided", C.c_int), ("photon_only", C.c_int)]


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
                ("aa_dark_threshold_factor", C.c_float), ("aa_variance_edge_size", C.c_int), ("aa_variance_pixels", C.c_int),
                ("raydepth", C.c_int), ("bg_transp_refract", C.c_int),
                ("transp_shad", C.c_int), ("shadow_depth", C.c_int), ("do_ao", C.c_int), ("ao_samples", C.c_int),
                ("ao_dist", C.c_float), ("ao_col", C.c_float * 3), ("aa_light_sample_multiplier_factor", C.c_float),
                ("caus_map", C.c_int), ("caus_photons", C.c_int), ("caus_search", C.c_int), ("caus_depth", C.c_int),
                ("caus_radius", C.c_float), ("tiles_order", C.c_int),
                ("pm_fg", C.c_int), ("fg_samples", C.c_int), ("fg_bounces", C.c_int), ("fg_min_pathlen", C.c_float),
                ("crop_x0", C.c_int), ("crop_y0", C.c_int), ("pm_show_map", C.c_int),
                ("pm_load_path", C.c_char_p), ("aa_indirect_sample_multiplier_factor", C.c_float)]


class yc_scene(C.Structure):
    _fields_ = [("n_verts", C.c_int), ("verts", C.POINTER(C.c_float)), ("n_tris", C.c_int),
                ("tris", C.POINTER(C.c_int)), ("tri_mat", C.POINTER(C.c_int)), ("n_mats", C.c_int),
                ("mats", C.POINTER(yc_material)), ("n_lights", C.c_int), ("lights", C.POINTER(yc_light)),
                ("cam", yc_camera), ("rp", yc_render), ("n_objects", C.c_int), ("objects", C.POINTER(yc_object)),
                ("orco", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)), ("uvs", C.POINTER(C.c_float)),
                ("tri_uv", C.POINTER(C.c_int)), ("n_images", C.c_int), ("images", C.POINTER(yc_image)),
                ("n_textures", C.c_int), ("textures", C.POINTER(yc_texture)), ("n_nodes", C.c_int),
                ("nodes", C.POINTER(yc_node))]


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


def glibc_rand(seed: int, n: int) -> np.ndarray:
    """The oracle's restatement of glibc rand() after srand(seed): the first n values (uint32)."""
    out = np.empty(max(1, n), np.uint32)
    oracle_lib().yc_glibc_rand(C.c_uint32(seed), C.c_int(n), _p(out, C.c_uint32))
    return out[:n]


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


def _shirley(self, r12):
    r12 = np.ascontiguousarray(r12, np.float32).reshape(-1)
    out = np.empty_like(r12)
    self.f("shirley_disk")(_p(r12, C.c_float), _p(out, C.c_float), C.c_int(len(r12) // 2))
    return out.reshape(-1, 2)


def _rgbe(self, b):
    b = np.ascontiguousarray(b, np.uint8).reshape(-1)
    out = np.empty(3 * (len(b) // 4), np.float32)
    self.f("rgbe_decode")(_p(b, C.c_uint8), _p(out, C.c_float), C.c_int(len(b) // 4))
    return out.reshape(-1, 3)


def _tiles(self, w, h, bs, order, nthreads=1):
    """order: "linear" | "centre" | "random"; (x, y, w, h) per region in render order."""
    cap = ((w + bs - 1) // bs) * ((h + bs - 1) // bs) * 16 + 16
    out = np.empty(4 * cap, np.int32)
    if self.px == "ref_":
        code = {"linear": 0, "random": 1, "centre": 2}[order]
        n = self.f("tiles")(C.c_int(w), C.c_int(h), C.c_int(bs), C.c_int(code), C.c_int(nthreads), _p(out, C.c_int), C.c_int(cap))
    else:
        code = {"linear": 0, "centre": 1, "random": 2}[order]
        n = self.f("tiles")(C.c_int(w), C.c_int(h), C.c_int(bs), C.c_int(code), _p(out, C.c_int), C.c_int(cap))
    return out[:4 * n].reshape(-1, 4)


Prims.shirley, Prims.rgbe, Prims.tiles = _shirley, _rgbe, _tiles


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

# ---- texturing: the reference's host-side setup, restated (scene.cc createMapItem, image.cc:38-100,
# format.cc:40-66, texture_image.cc:477-596, material_node.cc:102-187, shader node factories) ----
_IMG_TYPES = {"ColorAlpha": 4, "Color": 3, "GrayAlpha": 2, "Gray": 1}
_CS = {"Raw_Manual_Gamma": 1, "LinearRGB": 2, "sRGB": 3, "XYZ": 4}
_CLIP = {"extend": 0, "clip": 1, "clipcube": 2, "checker": 4}
_BLEND = {"add": 1, "multiply": 2, "subtract": 3, "screen": 4, "divide": 5, "difference": 6, "darken": 7,
          "lighten": 8, "overlay": 9}
_ROOTS = ("diffuse_shader", "mirror_color_shader", "bump_shader", "mirror_shader", "transparency_shader",
          "translucency_shader", "sigma_oren_shader", "diffuse_refl_shader", "IOR_shader", "wireframe_shader")


def _get(pm, key, kind, default=None):
    """ParamMap::getParam: strictly typed (a value of another kind reads as absent)."""
    tv = pm.get(key)
    if tv is None or tv[0] != kind:
        return default
    return tv[1]


def _texturing(self, spec, mats):
    """Fill the texturing part of self.sc from spec (images, textures, node programs, surface attributes)."""
    keep = []
    sc = self.sc
    # images (Image::factory)
    img_index, imgs = {}, []
    for im in spec.images:
        pm = im.params
        if im.name in img_index or _get(pm, "type", "s") is None:
            continue
        y = yc_image()
        itype = _IMG_TYPES.get(_get(pm, "type", "s", "ColorAlpha"), 0)
        opt = {"none": 0, "compressed": 2}.get(_get(pm, "image_optimization", "s", "optimized"), 1)
        cs = _CS.get(_get(pm, "color_space", "s", "Raw_Manual_Gamma"), 1)
        y.type, y.optimization, y.color_space = itype, opt, cs
        y.gamma = float(_get(pm, "gamma", "f", 1.0))
        y.width, y.height = int(_get(pm, "width", "i", 100)), int(_get(pm, "height", "i", 100))
        fn = _get(pm, "filename", "s", "")
        loaded = False
        if fn:
            path = fn if os.path.isabs(fn) or not im.base_dir else os.path.join(im.base_dir, fn)
            ext = os.path.splitext(fn)[1][1:].lower()
            fmt = 1 if ext in ("tga", "tpic") else 2 if ext in ("hdr", "pic") else 0
            if fmt and os.path.exists(path):
                data = np.frombuffer(open(path, "rb").read(), np.uint8).copy()
                keep.append(data)
                y.format, y.data, y.size = fmt, _p(data, C.c_uint8), len(data)
                if fmt == 2:
                    y.optimization = 0
                loaded = True   # the oracle decides decode failures itself (falls back to an empty image)
        if not loaded and itype == 0:
            continue            # Image::factory(w, h, Type::None) -> nullptr: the image does not exist
        if im.set_pixels:
            xy = np.asarray([(x, yy) for (x, yy, _) in im.set_pixels], np.int32).reshape(-1)
            rgba = np.asarray([c for (_, _, c) in im.set_pixels], np.float32).reshape(-1)
            keep += [xy, rgba]
            y.n_set, y.set_xy, y.set_rgba = len(im.set_pixels), _p(xy, C.c_int), _p(rgba, C.c_float)
        img_index[im.name] = len(imgs)
        imgs.append(y)
    # textures (ImageTexture::factory)
    tex_index, texs = {}, []
    for t in spec.textures:
        pm = t.params
        if t.name in tex_index or _get(pm, "type", "s") != "image":
            continue
        iname = _get(pm, "image_name", "s", "")
        if iname not in img_index:
            continue
        x = yc_texture()
        x.image = img_index[iname]
        interp = _get(pm, "interpolate", "s", "")
        x.interpolation = {"none": 0, "bicubic": 2}.get(interp, 1)
        x.clip = _CLIP.get(_get(pm, "clipping", "s", ""), 3)
        x.xrepeat, x.yrepeat = int(_get(pm, "xrepeat", "i", 1)), int(_get(pm, "yrepeat", "i", 1))
        x.mirror_x, x.mirror_y = int(_get(pm, "mirror_x", "b", False)), int(_get(pm, "mirror_y", "b", False))
        x.rot90 = int(_get(pm, "rot90", "b", False))
        x.even_tiles, x.odd_tiles = int(_get(pm, "even_tiles", "b", False)), int(_get(pm, "odd_tiles", "b", True))
        x.cropmin_x, x.cropmin_y = _get(pm, "cropmin_x", "f", 0.0), _get(pm, "cropmin_y", "f", 0.0)
        x.cropmax_x, x.cropmax_y = _get(pm, "cropmax_x", "f", 1.0), _get(pm, "cropmax_y", "f", 1.0)
        x.checker_dist = _get(pm, "checker_dist", "f", 0.0)
        x.intensity, x.contrast = _get(pm, "adj_intensity", "f", 1.0), _get(pm, "adj_contrast", "f", 1.0)
        x.saturation, x.hue = _get(pm, "adj_saturation", "f", 1.0), _get(pm, "adj_hue", "f", 0.0)
        x.factor_red = _get(pm, "adj_mult_factor_red", "f", 1.0)
        x.factor_green = _get(pm, "adj_mult_factor_green", "f", 1.0)
        x.factor_blue = _get(pm, "adj_mult_factor_blue", "f", 1.0)
        x.clamp = int(_get(pm, "adj_clamp", "b", False))
        tex_index[t.name] = len(texs)
        texs.append(x)
    # shader nodes per material (loadNodes / configInputs / parseNodes); nodes are global in yc_scene
    nodes = []
    for mi, m in enumerate(spec.materials):
        if m.params is None or not m.nodes:
            continue
        table, order, ok = {}, [], True
        for nd in m.nodes:
            el = _get(nd, "element", "s")
            if el is not None and el != "shader_node":
                continue
            name, typ = _get(nd, "name", "s"), _get(nd, "type", "s")
            if name is None or typ is None or name in table:
                ok = False
                break
            y = yc_node()
            y.input[:] = [-1, -1, -1]
            if typ == "texture_mapper":
                tname = _get(nd, "texture", "s")
                if tname not in tex_index:
                    ok = False
                    break
                y.type, y.texture = 3, tex_index[tname]
                y.coords = {"uv": 0, "orco": 2, "transformed": 3}.get(_get(nd, "texco", "s", "global"), 1)
                y.projection = {"cube": 1, "tube": 2, "sphere": 3}.get(_get(nd, "mapping", "s", "plain"), 0)
                y.map[:] = [min(3, max(0, int(_get(nd, k, "i", dflt)))) for k, dflt in (("proj_x", 1), ("proj_y", 2), ("proj_z", 3))]
                y.scale[:] = list(_get(nd, "scale", "v", (1.0, 1.0, 1.0)))
                y.offset[:] = list(_get(nd, "offset", "v", (0.0, 0.0, 0.0)))
                y.mtx[:] = list(_get(nd, "transform", "m", (1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1)))
                y.do_scalar = int(_get(nd, "do_scalar", "b", True))
            elif typ == "value":
                y.type = 0
                c = _get(nd, "color", "c", (1.0, 1.0, 1.0, 1.0))
                y.col1[:] = [c[0], c[1], c[2], _get(nd, "alpha", "f", 1.0)]
                y.val[0] = _get(nd, "scalar", "f", 1.0)
            elif typ == "mix":
                y.type = 1
                b = _BLEND.get(_get(nd, "blend_mode", "s", ""), 0)
                y.blend = 0 if b == 5 else b
                y.val[0] = _get(nd, "cfactor", "f", 0.5) if y.blend == 0 else 0.0
            elif typ == "layer":
                y.type = 2
                b = _BLEND.get(_get(nd, "blend_mode", "s", ""), 0)
                y.blend = 0 if b == 9 else b
                c = _get(nd, "def_col", "c", (1.0, 1.0, 1.0, 1.0))
                y.col1[:] = [c[0], c[1], c[2], 1.0]
                y.val[0], y.val[1], y.val[2] = _get(nd, "colfac", "f", 1.0), _get(nd, "valfac", "f", 1.0), _get(nd, "def_val", "f", 1.0)
                for fld, key, dflt in (("no_rgb", "noRGB", False), ("stencil", "stencil", False), ("negative", "negative", False),
                                       ("do_color", "do_color", True), ("do_scalar", "do_scalar", False),
                                       ("color_input", "color_input", True), ("use_alpha", "use_alpha", False)):
                    setattr(y, fld, int(_get(nd, key, "b", dflt)))
            else:
                ok = False
                break
            table[name] = (y, nd)
            order.append(name)
        if ok:
            for name in order:
                y, nd = table[name]
                if y.type == 2:
                    inp = _get(nd, "input", "s")
                    if inp not in table:
                        ok = False
                        break
                    up = _get(nd, "upper_layer", "s")
                    if up is not None:
                        if up not in table:
                            ok = False
                            break
                    else:
                        y.col2[:] = list(_get(nd, "upper_color", "c", (0.0, 0.0, 0.0, 0.0)))
                        y.val[3] = _get(nd, "upper_value", "f", 0.0)
                elif y.type == 1:
                    for k, (ik, ck) in enumerate((("input1", "color1"), ("input2", "color2"))):
                        inp = _get(nd, ik, "s")
                        if inp is not None:
                            if inp not in table:
                                ok = False
                        elif _get(nd, ck, "c") is not None:
                            (y.col1 if k == 0 else y.col2)[:] = list(_get(nd, ck, "c"))
                        else:
                            ok = False
                    if _get(nd, "factor", "s") is not None:
                        ok = ok and _get(nd, "factor", "s") in table
                    elif _get(nd, "value", "f") is not None:
                        y.val[0] = _get(nd, "value", "f")
                    else:
                        ok = False
                    if not ok:
                        break
        if not ok:
            continue   # loadNodes cleared the table: plain colours
        base = len(nodes)
        gidx = {name: base + k for k, name in enumerate(order)}
        for name in order:
            y, nd = table[name]
            if y.type == 2:
                y.input[0] = gidx[_get(nd, "input", "s")]
                if _get(nd, "upper_layer", "s") is not None:
                    y.input[1] = gidx[_get(nd, "upper_layer", "s")]
            elif y.type == 1:
                for k, key in enumerate(("input1", "input2", "factor")):
                    if _get(nd, key, "s") is not None:
                        y.input[k] = gidx[_get(nd, key, "s")]
            nodes.append(y)
        for root, fld in (("diffuse_shader", "diffuse_shader"), ("diffuse_refl_shader", "diffuse_refl_shader"),
                          ("sigma_oren_shader", "sigma_shader")):
            nm = _get(m.params, root, "s")
            if nm is not None and nm in gidx:
                setattr(mats[mi], fld, gidx[nm])
    # surface attributes per object
    objs = (yc_object * max(1, len(spec.objects)))()
    for k, o in enumerate(spec.objects):
        objs[k].v0, objs[k].nv, objs[k].t0, objs[k].nt = o.v0, o.nv, o.t0, o.nt
        objs[k].has_orco = int(spec.orco is not None and o.has_orco)
        objs[k].has_uv = int(o.nuv > 0)
        objs[k].normals_exported = int(spec.normals is not None)
        objs[k].smooth = int(o.smooth_angle is not None)
        objs[k].smooth_angle = o.smooth_angle if o.smooth_angle is not None else 0.0
    sc.n_objects, sc.objects = len(spec.objects), C.cast(objs, C.POINTER(yc_object))
    keep.append(objs)
    for fld, arr, ct, dt in (("orco", spec.orco, C.c_float, np.float32), ("normals", spec.normals, C.c_float, np.float32),
                             ("uvs", spec.uvs, C.c_float, np.float32), ("tri_uv", spec.tri_uv, C.c_int, np.int32)):
        if arr is not None:
            a = np.ascontiguousarray(arr, dt).reshape(-1)
            keep.append(a)
            setattr(sc, fld, _p(a, ct))
    if imgs:
        ia = (yc_image * len(imgs))(*imgs)
        keep.append(ia)
        sc.n_images, sc.images = len(imgs), C.cast(ia, C.POINTER(yc_image))
    if texs:
        ta = (yc_texture * len(texs))(*texs)
        keep.append(ta)
        sc.n_textures, sc.textures = len(texs), C.cast(ta, C.POINTER(yc_texture))
    if nodes:
        na = (yc_node * len(nodes))(*nodes)
        keep.append(na)
        sc.n_nodes, sc.nodes = len(nodes), C.cast(na, C.POINTER(yc_node))
    self._tex_keep = keep


class OracleScene:
    """Owns the numpy buffers referenced by a yc_scene struct built from a SceneSpec."""

    def __init__(self, spec, threads: int = 1, rr_seed: int = 0):
        s = spec
        self.verts = np.ascontiguousarray(s.verts, np.float32).reshape(-1)
        self.tris = np.ascontiguousarray(s.tris, np.int32).reshape(-1)
        self.tri_mat = np.ascontiguousarray(s.tri_mat, np.int32).reshape(-1)
        mats = (yc_material * max(1, len(s.materials)))()
        for i, m in enumerate(s.materials):
            mats[i].type = {"light_mat": YC_MAT_LIGHT, "mirror": 2, "null": 3}.get(m.type, YC_MAT_SHINYDIFFUSE)
            if m.type == "light_mat":
                mats[i].color[:] = [np.float32(c) * np.float32(m.power) for c in m.color]
            else:
                mats[i].color[:] = list(m.color)
            mats[i].diffuse_strength = m.diffuse_reflect
            mats[i].emit_strength = m.emit
            mats[i].double_sided = int(m.double_sided)
            mats[i].receive_shadows = int(m.receive_shadows)
            mats[i].flat_material = int(m.flat_material)
            mats[i].diffuse_shader = mats[i].diffuse_refl_shader = -1
            mats[i].specular_reflect, mats[i].transparency = m.specular_reflect, m.transparency
            mats[i].translucency, mats[i].transmit_filter = m.translucency, m.transmit_filter
            mats[i].ior, mats[i].fresnel_effect = m.ior, int(m.fresnel)
            mats[i].mirror_color[:] = list(m.mirror_color)
            mats[i].transparentbias_factor = m.transparentbias_factor
            mats[i].transparentbias_multiply_raydepth = int(m.transparentbias_multiply_raydepth)
            mats[i].reflect = m.reflect
            mats[i].additional_depth = m.additionaldepth
            mats[i].oren_nayar = int(m.diffuse_brdf == "oren_nayar")
            mats[i].sigma = m.sigma
            mats[i].sigma_shader = -1
        lights = (yc_light * max(1, len(s.lights)))()
        for i, l in enumerate(s.render_lights()):
            lights[i].type = {"pointlight": YC_LIGHT_POINT, "meshlight": YC_LIGHT_MESH, "objectlight": YC_LIGHT_MESH}.get(l.type, YC_LIGHT_AREA)
            if lights[i].type == YC_LIGHT_MESH:
                lights[i].object = [o.name for o in s.objects].index(l.object_name)
                lights[i].double_sided = int(l.double_sided)
            lights[i].color[:] = list(l.color)
            lights[i].power = l.power
            lights[i].from_[:] = list(l.from_ if l.type == "pointlight" else l.corner)
            lights[i].point1[:] = list(l.point1)
            lights[i].point2[:] = list(l.point2)
            lights[i].samples = l.samples
            lights[i].shoot_caustic = int(getattr(l, "with_caustic", True))
            lights[i].shoot_diffuse = int(getattr(l, "with_diffuse", True))
            lights[i].cast_shadows = int(l.cast_shadows)
            lights[i].photon_only = int(getattr(l, "photon_only", False))
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
        rp.crop_x0, rp.crop_y0 = getattr(r, "xstart", 0), getattr(r, "ystart", 0)
        rp.pm_show_map = int(bool(getattr(r, "pm_show_map", False)))
        # photon_maps_processing "load": the maps from <film_load_save_path>_*.photonmap
        self._load_path = None
        if getattr(r, "pm_maps_processing", "generate") == "load":
            self._load_path = getattr(r, "film_load_save_path", "./").encode()
        rp.pm_load_path = self._load_path
        rp.clamp_samples = r.clamp_samples
        rp.threads = threads
        rp.rr_seed = rr_seed
        rp.pm_photons, rp.pm_search, rp.pm_diffuse_radius = r.pm_photons, r.pm_search, r.pm_diffuse_radius
        rp.pm_bounces, rp.pm_caustics, rp.pm_threads = r.pm_bounces, int(r.pm_caustics), r.threads_photons
        from libyafaray_amd.scenes import caustic_params
        cm = caustic_params(r)
        rp.caus_map, rp.caus_photons, rp.caus_search = int(cm.enabled), cm.photons, cm.search
        rp.caus_depth, rp.caus_radius = cm.depth, cm.radius
        rp.tiles_order = {"linear": 0, "random": 2}.get(getattr(r, "tiles_order", "linear"), 1)
        rp.pm_fg = int(r.integrator == "photonmapping" and r.pm_final_gather)
        rp.fg_samples, rp.fg_bounces = r.fg_samples, r.fg_bounces
        rp.fg_min_pathlen = r.fg_min_pathlen if r.fg_min_pathlen is not None else r.pm_diffuse_radius
        rp.aa_passes = max(1, r.aa_passes)
        rp.aa_inc_samples = r.aa_inc_samples if r.aa_inc_samples > 0 else r.aa_samples
        rp.aa_threshold, rp.aa_resampled_floor = r.aa_threshold, r.aa_resampled_floor
        rp.aa_sample_multiplier_factor = r.aa_sample_multiplier_factor
        rp.aa_detect_color_noise = int(r.aa_detect_color_noise)
        rp.aa_dark_detection_type = {"linear": 1, "curve": 2}.get(r.aa_dark_detection_type, 0)
        rp.aa_dark_threshold_factor = r.aa_dark_threshold_factor
        rp.aa_variance_edge_size, rp.aa_variance_pixels = r.aa_variance_edge_size, r.aa_variance_pixels
        rp.raydepth, rp.bg_transp_refract = r.raydepth, int(r.bg_transp_refract)
        rp.transp_shad, rp.shadow_depth = int(r.transp_shad), r.shadow_depth
        rp.do_ao, rp.ao_samples, rp.ao_dist = int(r.do_ao), r.ao_samples, r.ao_distance
        rp.ao_col[:] = list(r.ao_color)
        rp.aa_light_sample_multiplier_factor = r.aa_light_sample_multiplier_factor
        rp.aa_indirect_sample_multiplier_factor = r.aa_indirect_sample_multiplier_factor
        self.sc = sc
        self.spec = spec
        _texturing(self, spec, mats)

    def render(self, y0: int = 0, y1: int = 0):
        r = self.spec.render
        rgba = np.zeros(r.width * r.height * 4, np.float32)
        w = np.zeros(r.width * r.height, np.float32)
        ctr = yc_counters()
        oracle_lib().yc_render_image(C.byref(self.sc), C.c_int(y0), C.c_int(y1), _p(rgba, C.c_float),
                                     _p(w, C.c_float), C.byref(ctr))
        return rgba.reshape(r.height, r.width, 4), w.reshape(r.height, r.width), (ctr.closest_rays, ctr.shadow_rays)

    def photon_map(self, which="diffuse"):
        """(pos, dir, col [n x 3 each], kd nodes [m x 2 uint32], n_paths) of the diffuse, caustic or
        final-gather radiance map (dir = the radiance point's normal)."""
        L = oracle_lib()
        w = {"caustic": 1, "radiance": 2}.get(which, 0)
        n_paths = C.c_int(0)
        n = L.yc_photon_map_ex(C.byref(self.sc), w, None, None, None, None, C.byref(n_paths))
        if n < 0:
            raise RuntimeError("photon map failed (too few photons)")
        pos, d, col = (np.empty(3 * max(1, n), np.float32) for _ in range(3))
        nodes = np.empty(2 * max(1, 2 * n - 1), np.uint32)
        L.yc_photon_map_ex(C.byref(self.sc), w, _p(pos, C.c_float), _p(d, C.c_float), _p(col, C.c_float),
                           _p(nodes, C.c_uint32), C.byref(n_paths))
        return (pos[:3 * n].reshape(n, 3), d[:3 * n].reshape(n, 3), col[:3 * n].reshape(n, 3),
                nodes.reshape(-1, 2)[:max(0, 2 * n - 1)], n_paths.value)

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
