"""Texturing test scenes: a grid of cubes, one material per cube, each material a shader-node
tree over image textures (tests/test_textures.py).

Every cube carries orco coordinates (object-local -1..1), per-face UVs that overshoot [0, 1] (so
the clip modes matter) and, optionally, smoothMesh normals.  The images are the reference's own
tests/test01 TGA / HDR files plus small procedural images written through yafaray_setImageColor
(every image buffer type and optimisation).  Parameter maps are typed exactly as a reference
client passes them (s f i b v c m).
"""
import math
import os

import numpy as np

from libyafaray_amd import scenes

TEX01 = scenes.TEX01_DIR


def S(v):
    return ("s", v)


def F(v):
    return ("f", float(v))


def I(v):
    return ("i", int(v))


def B(v):
    return ("b", bool(v))


def V(*v):
    return ("v", tuple(float(x) for x in v))


def Col(*v):
    return ("c", tuple(float(x) for x in (v + (1.0,) * (4 - len(v)))))


def procedural_image(name, w=13, h=9, type_="ColorAlpha", opt="none", seed=0, color_space=None, gamma=None):
    """An empty image filled with a deterministic pattern via setImageColor (values in [0, 1.2])."""
    rng = np.random.default_rng(seed)
    px = []
    for y in range(h):
        for x in range(w):
            r = 0.5 + 0.5 * math.sin(0.9 * x + 0.3 * y)
            g = (x * 7 + y * 3) % 11 / 10.0
            b = rng.random() * 1.2
            a = 0.25 + 0.75 * ((x + 2 * y) % 5) / 4.0
            px.append((x, y, (r, g, b, a)))
    params = {"type": S(type_), "image_optimization": S(opt), "width": I(w), "height": I(h)}
    if color_space:
        params["color_space"] = S(color_space)
    if gamma is not None:
        params["gamma"] = F(gamma)
    return scenes.ImageSpec(name, params, set_pixels=px)


def file_image(name, fname, opt="optimized", color_space="sRGB", type_="image"):
    return scenes.ImageSpec(name, {"type": S(type_), "filename": S(fname), "image_optimization": S(opt),
                                   "color_space": S(color_space), "gamma": F(1.0)}, TEX01)


def texture(name, image, **kw):
    p = {"type": S("image"), "image_name": S(image)}
    for k, v in kw.items():
        p[k] = v
    return scenes.TextureSpec(name, p)


def mapper(name, tex, texco="orco", mapping="cube", proj=(1, 2, 3), scale=(1, 1, 1), offset=(0, 0, 0), **kw):
    n = {"element": S("shader_node"), "type": S("texture_mapper"), "name": S(name), "texture": S(tex),
         "texco": S(texco), "mapping": S(mapping), "proj_x": I(proj[0]), "proj_y": I(proj[1]), "proj_z": I(proj[2]),
         "scale": V(*scale), "offset": V(*offset)}
    n.update(kw)
    return n


def layer(name, input_, blend="mix", colfac=1.0, upper_color=(0.8, 0.8, 0.8, 1.0), **kw):
    n = {"element": S("shader_node"), "type": S("layer"), "name": S(name), "input": S(input_), "blend_mode": S(blend),
         "colfac": F(colfac), "upper_color": Col(*upper_color), "def_col": Col(1, 0, 1), "do_color": B(True),
         "do_scalar": B(False), "color_input": B(True), "use_alpha": B(False), "noRGB": B(False), "stencil": B(False),
         "negative": B(False)}
    n.update(kw)
    return n


def value(name, color=(1, 1, 1), alpha=1.0, scalar=1.0):
    return {"element": S("shader_node"), "type": S("value"), "name": S(name), "color": Col(*color), "alpha": F(alpha),
            "scalar": F(scalar)}


def mix(name, blend="mix", **kw):
    n = {"element": S("shader_node"), "type": S("mix"), "name": S(name), "blend_mode": S(blend)}
    n.update(kw)
    return n


def material(name, nodes, diffuse_shader="root", color=(0.8, 0.8, 0.8), diffuse=1.0, emit=0.0, **kw):
    p = {"type": S("shinydiffusemat"), "color": Col(*color), "diffuse_reflect": F(diffuse), "emit": F(emit)}
    if diffuse_shader:
        p["diffuse_shader"] = S(diffuse_shader)
    p.update(kw)
    return scenes.Material(name, color=tuple(color), diffuse_reflect=diffuse, emit=emit, params=p, nodes=list(nodes))


def _cube(c, s):
    """8 vertices (orco = the local corner) and 12 triangles + per-face uv indices."""
    corners = [(x, y, z) for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)]
    verts = [(c[0] + s * x, c[1] + s * y, c[2] + s * z) for (x, y, z) in corners]
    faces = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    tris, tuv = [], []
    for (a, b, cc, d) in faces:
        tris += [(a, b, cc), (a, cc, d)]
        tuv += [(0, 1, 2), (0, 2, 3)]
    return verts, [tuple(map(float, k)) for k in corners], tris, tuv


def _sphere(c, r, n=10):
    verts, orco = [], []
    for i in range(n + 1):
        th = math.pi * i / n
        for j in range(n):
            ph = 2 * math.pi * j / n
            p = (math.sin(th) * math.cos(ph), math.sin(th) * math.sin(ph), math.cos(th))
            verts.append(tuple(c[k] + r * p[k] for k in range(3)))
            orco.append(p)
    tris = []
    for i in range(n):
        for j in range(n):
            a, b = i * n + j, i * n + (j + 1) % n
            cc, d = (i + 1) * n + j, (i + 1) * n + (j + 1) % n
            tris += [(a, cc, b), (b, cc, d)]
    return verts, orco, tris


def grid_scene(mats, images, textures, integrator="directlighting", width=96, height=72, spp=2, sphere_smooth=None,
               normals=False, bounces=3, cols=4):
    """One cube per material on a grid (plus an untextured floor); camera from the front-top corner
    so three faces of every cube are seen.  sphere_smooth: add a smoothed UV sphere (angle) using
    the first material."""
    verts, orco, tris, tri_mat, uvs, tri_uv, objects = [], [], [], [], [], [], []
    uv_face = [(-0.25, -0.25), (1.25, -0.25), (1.25, 1.25), (-0.25, 1.25)]
    floor = scenes.Material("floor", color=(0.6, 0.6, 0.6))
    all_mats = list(mats) + [floor]
    for k, m in enumerate(mats):
        cx, cy = (k % cols) * 2.6, (k // cols) * 2.6
        v, o, t, tu = _cube((cx, cy, 1.0), 0.9)
        v0, t0, u0 = len(verts), len(tris), len(uvs)
        verts += v
        orco += o
        tris += [(a + v0, b + v0, c + v0) for (a, b, c) in t]
        tri_mat += [k] * len(t)
        uvs += uv_face
        tri_uv += [(a + u0, b + u0, c + u0) for (a, b, c) in tu]
        objects.append(scenes.Object(f"cube{k}", v0, len(v), t0, len(t), uv0=u0, nuv=4))
    if sphere_smooth is not None:
        v, o, t = _sphere((-2.6, 1.3, 1.0), 1.0)
        v0, t0 = len(verts), len(tris)
        verts += v
        orco += o
        tris += [(a + v0, b + v0, c + v0) for (a, b, c) in t]
        tri_mat += [0] * len(t)
        tri_uv += [(-1, -1, -1)] * len(t)
        objects.append(scenes.Object("sphere", v0, len(v), t0, len(t), smooth_angle=sphere_smooth))
    # floor
    ext = 2.6 * cols
    fv = [(-4.0, -3.0, 0.0), (ext + 1.0, -3.0, 0.0), (ext + 1.0, ext, 0.0), (-4.0, ext, 0.0)]
    v0, t0 = len(verts), len(tris)
    verts += fv
    orco += [(0.0, 0.0, 0.0)] * 4
    tris += [(v0, v0 + 1, v0 + 2), (v0, v0 + 2, v0 + 3)]
    tri_mat += [len(mats)] * 2
    tri_uv += [(-1, -1, -1)] * 2
    objects.append(scenes.Object("floor", v0, 4, t0, 2, has_orco=False))
    verts = np.asarray(verts, np.float32)
    nrm = None
    if normals:
        nrm = verts - verts.mean(0)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    light = scenes.Light("pt", type="pointlight", color=(1.0, 1.0, 1.0), power=90.0, from_=(ext * 0.3, -2.0, 9.0))
    cam = scenes.Camera(from_=(ext * 0.45, -9.0, 8.0), to=(ext * 0.42, 2.0, 0.5), up=(ext * 0.45, -9.0, 9.0),
                        resx=width, resy=height, focal=1.1)
    rend = scenes.Render(integrator=integrator, width=width, height=height, aa_samples=spp, filter_type="box",
                         aa_pixelwidth=1.0, bounces=bounces, rr_min_bounces=bounces, caustic_type="none", raydepth=2)
    return scenes.SceneSpec(verts, np.asarray(tris, np.int32), np.asarray(tri_mat, np.int32), all_mats, [light], cam,
                            rend, scenes.Background((0.05, 0.06, 0.08), 1.0), objects,
                            orco=np.asarray(orco, np.float32), normals=nrm, uvs=np.asarray(uvs, np.float32).reshape(-1, 2),
                            tri_uv=np.asarray(tri_uv, np.int32), images=list(images), textures=list(textures))


# ---------------------------------------------------------------------------------------------
# cases
# ---------------------------------------------------------------------------------------------
def case_images():
    """Image buffer types / optimisations / colour spaces, and the two reference texture files."""
    imgs = [file_image("tga", "tex.tga"), file_image("hdr", "tex.hdr"),
            file_image("tga_c", "tex.tga", opt="compressed", color_space="LinearRGB"),
            file_image("tga_g", "tex.tga", opt="optimized", type_="Gray", color_space="XYZ"),
            procedural_image("ca_none", opt="none", seed=1), procedural_image("ca_opt", opt="optimized", seed=2),
            procedural_image("ca_comp", opt="compressed", seed=3), procedural_image("c_opt", type_="Color", opt="optimized", seed=4),
            procedural_image("c_comp", type_="Color", opt="compressed", seed=5), procedural_image("g_opt", type_="Gray", seed=6, opt="optimized"),
            procedural_image("ga", type_="GrayAlpha", seed=7), procedural_image("c_none", type_="Color", opt="none", seed=8)]
    texs = [texture("t_" + im.name, im.name) for im in imgs]
    mats = []
    for k, im in enumerate(imgs):
        mats.append(material(f"m{k}", [layer("root", "map"), mapper("map", "t_" + im.name)]))
    return mats, imgs, texs


def case_clip_interp():
    """Clip modes, interpolation, repeat / mirror / crop / rot90 / checker on uv coordinates."""
    imgs = [procedural_image("p", opt="none", seed=11), file_image("tga", "tex.tga")]
    tx = [
        texture("rep_bil", "p", clipping=S("repeat"), interpolate=S("bilinear"), xrepeat=I(3), yrepeat=I(2)),
        texture("rep_mir", "p", clipping=S("repeat"), interpolate=S("bicubic"), mirror_x=B(True), mirror_y=B(True), xrepeat=I(2)),
        texture("clip_none", "p", clipping=S("clip"), interpolate=S("none")),
        texture("extend_cub", "p", clipping=S("extend"), interpolate=S("bicubic")),
        texture("clipcube", "tga", clipping=S("clipcube")),
        texture("checker", "p", clipping=S("checker"), even_tiles=B(True), odd_tiles=B(False), checker_dist=F(0.2)),
        texture("crop_rot", "tga", cropmin_x=F(0.2), cropmax_x=F(0.7), cropmin_y=F(0.1), cropmax_y=F(0.9), rot90=B(True)),
        texture("mirror_none", "p", interpolate=S("none"), mirror_x=B(True)),
    ]
    mats = []
    for k, t in enumerate(tx):
        texco = "orco" if t.name == "clipcube" else "uv"
        mats.append(material(f"m{k}", [layer("root", "map"), mapper("map", t.name, texco=texco, mapping="plain" if texco == "uv" else "cube")]))
    return mats, imgs, tx


def case_adjust_mapping():
    """Texture adjustments and mapper coordinates / projections / axis maps / scale / offset."""
    imgs = [file_image("tga", "tex.tga"), procedural_image("p", opt="optimized", seed=21, color_space="sRGB")]
    tx = [texture("adj", "tga", adj_intensity=F(1.2), adj_contrast=F(0.8), adj_saturation=F(0.5), adj_hue=F(40.0),
                  adj_mult_factor_red=F(1.3), adj_mult_factor_green=F(0.9), adj_mult_factor_blue=F(0.7), adj_clamp=B(True)),
          texture("adj2", "p", adj_hue=F(-100.0), adj_saturation=F(1.5)),
          texture("plain", "tga")]
    mtx = ("m", (0.5, 0.1, 0.0, 0.2, -0.1, 0.5, 0.0, 0.1, 0.0, 0.0, 0.5, 0.0, 0.0, 0.0, 0.0, 1.0))
    mats = [
        material("m0", [layer("root", "map"), mapper("map", "adj")]),
        material("m1", [layer("root", "map"), mapper("map", "adj2", texco="uv", mapping="plain")]),
        material("m2", [layer("root", "map"), mapper("map", "plain", texco="global", mapping="cube", scale=(0.6, 0.6, 0.6),
                                                       offset=(0.1, -0.2, 0.0))]),
        material("m3", [layer("root", "map"), mapper("map", "plain", texco="transformed", mapping="plain", transform=mtx)]),
        material("m4", [layer("root", "map"), mapper("map", "plain", texco="orco", mapping="plain", proj=(2, 3, 1))]),
        material("m5", [layer("root", "map"), mapper("map", "plain", texco="orco", mapping="cube", proj=(0, 3, 2),
                                                       scale=(1.5, 0.5, 1.0))]),
        material("m6", [layer("root", "map"), mapper("map", "adj2", texco="uv", mapping="plain", proj=(2, 1, 3))]),
        material("m7", [layer("root", "map"), mapper("map", "plain", texco="reflect", mapping="cube")]),   # reflect -> global
    ]
    return mats, imgs, tx


def case_tube_sphere():
    """Tube / sphere projections (atan2 / acos: libm vs device, compared with a tolerance)."""
    imgs = [file_image("tga", "tex.tga")]
    tx = [texture("t", "tga")]
    mats = [material("m0", [layer("root", "map"), mapper("map", "t", mapping="tube")]),
            material("m1", [layer("root", "map"), mapper("map", "t", mapping="sphere")])]
    return mats, imgs, tx


def case_layers():
    """LayerNode blend modes and flags, stacked layers, value / mix nodes, diffuse_refl_shader, emit."""
    imgs = [file_image("tga", "tex.tga"), procedural_image("p", opt="none", seed=31)]
    tx = [texture("t", "tga"), texture("q", "p", interpolate=S("bicubic"))]
    mats = []
    for k, bl in enumerate(["mix", "add", "multiply", "subtract", "screen", "divide", "difference", "darken", "lighten"]):
        mats.append(material(f"b{k}", [layer("root", "map", blend=bl, colfac=0.7, upper_color=(0.3, 0.5, 0.7, 0.9)),
                                        mapper("map", "q", texco="uv", mapping="plain")]))
    mats.append(material("stack", [layer("root", "map2", blend="multiply", upper_layer=S("l1")),
                                   layer("l1", "map", blend="mix", stencil=B(True), colfac=0.8),
                                   mapper("map", "t"), mapper("map2", "q", texco="uv", mapping="plain")]))
    mats.append(material("flags", [layer("root", "map", blend="add", negative=B(True), noRGB=B(True), def_col=Col(0.2, 0.9, 0.4)),
                                   mapper("map", "q", texco="uv", mapping="plain")]))
    mats.append(material("scalar", [layer("root", "map"), mapper("map", "t"),
                                    layer("refl", "map2", blend="screen", do_color=B(False), do_scalar=B(True), use_alpha=B(True),
                                          def_val=F(0.6), valfac=F(0.9), upper_value=F(0.3)),
                                    mapper("map2", "q", texco="uv", mapping="plain")],
                         diffuse_refl_shader=S("refl")))
    mats.append(material("value_mix", [mix("root", blend="mix", input1=S("v1"), input2=S("map"), factor=S("v2")),
                                       value("v1", color=(0.9, 0.2, 0.1), alpha=0.5, scalar=0.25),
                                       value("v2", scalar=0.4), mapper("map", "t")]))
    for k, bl in enumerate(["add", "multiply", "subtract", "screen", "difference", "darken", "lighten", "overlay"]):
        mats.append(material(f"x{k}", [mix("root", blend=bl, input1=S("map"), color2=Col(0.3, 0.6, 0.9, 0.7), value=F(0.6)),
                                        mapper("map", "q", texco="uv", mapping="plain")]))
    mats.append(material("emit", [layer("root", "map"), mapper("map", "t")], emit=0.4))
    # node list failures clear every node: plain colours (material_node.cc:151-167)
    mats.append(material("broken", [layer("root", "nosuch"), mapper("map", "t")], color=(0.2, 0.7, 0.3)))
    mats.append(material("notex", [layer("root", "map"), mapper("map", "missing_texture")], color=(0.7, 0.3, 0.2)))
    return mats, imgs, tx


CASES = {"images": case_images, "clip_interp": case_clip_interp, "adjust_mapping": case_adjust_mapping,
         "tube_sphere": case_tube_sphere, "layers": case_layers}
