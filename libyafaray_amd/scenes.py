"""Scene descriptions used by the tests, the bench and the smoke check.

A `SceneSpec` is plain data (numpy geometry + small dataclasses).  `apply(spec, yi)` replays it
through the C API exactly the way the reference's C clients do (tests/test01/test01.c:27-1018:
paramsSet* -> create* -> addVertex/addTriangle -> setupRender -> render), so every product
render in this repository goes through the drop-in boundary.

Builders:
  * `cornell(...)`       — BASELINE config C2/C3: 5 walls + 2 boxes (34 triangles), 0.5 x 0.5 area
                           light at z = 1.98, camera from (0, -3.9, 1), focal 1.4.
  * `cornell_sphere(...)`— config C4: C2 + a UV sphere of 707 x 707 x 2 = 999,698 triangles.
  * `test01(...)`        — config C1: the reference's tests/test01 scene (six cubes + plane, point
                           light, direct lighting, gauss 1.5) with textures stripped; its geometry is
                           read from tests/golden/test01_scene.json (made by make_test01_scene.py).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np


@dataclass
class Material:
    name: str
    type: str = "shinydiffusemat"          # or "light_mat"
    color: tuple = (0.8, 0.8, 0.8)
    diffuse_reflect: float = 1.0
    emit: float = 0.0
    power: float = 1.0                     # light_mat
    double_sided: bool = False             # light_mat
    receive_shadows: bool = True
    flat_material: bool = False
    # shinydiffuse specular / transparent / translucent components (material_shiny_diffuse.cc:490-566)
    specular_reflect: float = 0.0
    transparency: float = 0.0
    translucency: float = 0.0
    transmit_filter: float = 1.0
    ior: float = 1.33
    fresnel: bool = False
    mirror_color: tuple = (1.0, 1.0, 1.0)
    transparentbias_factor: float = 0.0
    transparentbias_multiply_raydepth: bool = False
    reflect: float = 1.0                   # type "mirror": colour * reflect
    diffuse_brdf: str = "lambert"          # "oren_nayar" (material_shiny_diffuse.cc:561-571)
    sigma: float = 0.1                     # Oren-Nayar roughness
    additionaldepth: int = 0               # extra recursiveRaytrace depth (integrator_montecarlo.cc:923)
    # full typed parameter map {key: (kind, value)} (kinds s f i b v c m) and the pushed shader-node
    # lists, as a reference client passes them (tests/test01/test01.c:268-650); when set, apply()
    # issues exactly these instead of the fields above
    params: Optional[dict] = None
    nodes: List[dict] = field(default_factory=list)


@dataclass
class ImageSpec:
    """yafaray_createImage: typed params; a relative "filename" is resolved against base_dir.
    set_pixels: yafaray_setImageColor calls [(x, y, (r, g, b, a))] issued after creation."""
    name: str
    params: dict
    base_dir: str = ""
    set_pixels: List[tuple] = field(default_factory=list)


@dataclass
class TextureSpec:
    name: str
    params: dict


@dataclass
class Light:
    name: str
    type: str = "pointlight"               # or "arealight"
    color: tuple = (1.0, 1.0, 1.0)
    power: float = 1.0
    from_: tuple = (0.0, 0.0, 0.0)         # pointlight
    corner: tuple = (0.0, 0.0, 0.0)        # arealight
    point1: tuple = (0.0, 0.0, 0.0)
    point2: tuple = (0.0, 0.0, 0.0)
    samples: int = 1
    cast_shadows: bool = True
    with_caustic: bool = True              # shoots caustic photons (light_area.cc / light_point.cc params)
    with_diffuse: bool = True              # shoots diffuse photons
    object_name: str = ""                  # meshlight / objectlight: the emitting object
    double_sided: bool = False             # meshlight
    photon_only: bool = False              # shoots photons only (Light::photonOnly, render_view.cc:83-111)


@dataclass
class Camera:
    from_: tuple
    to: tuple
    up: tuple
    resx: int
    resy: int
    focal: float = 1.0
    aspect_ratio: float = 1.0
    near_clip: float = 0.0
    far_clip: float = -1.0
    # depth of field (camera_perspective.cc:190-224)
    aperture: float = 0.0
    dof_distance: float = 0.0
    bokeh_type: str = "disk1"       # disk1 disk2 triangle square pentagon hexagon ring
    bokeh_bias: str = "uniform"     # uniform center edge
    bokeh_rotation: float = 0.0


@dataclass
class Background:
    color: tuple = (0.0, 0.0, 0.0)
    power: float = 1.0


@dataclass
class Render:
    integrator: str = "pathtracing"        # or "directlighting"
    width: int = 64
    height: int = 64
    aa_samples: int = 1
    filter_type: str = "box"
    aa_pixelwidth: float = 1.0
    tile_size: int = 32
    tiles_order: str = "linear"             # linear | centre (the reference default) | random
    bounces: int = 8
    path_samples: int = 1
    rr_min_bounces: int = 0
    caustic_type: str = "path"
    raydepth: int = 5
    bg_transp: bool = False
    bg_transp_refract: bool = False
    transp_shad: bool = False               # transparent shadows (MonteCarloIntegrator tr_shad_)
    shadow_depth: int = 5                   # "shadowDepth" (integrator_path_tracer.cc:295)
    shadow_bias_auto: bool = True
    shadow_bias: float = 0.0005
    ray_min_dist_auto: bool = True
    ray_min_dist: float = 0.00005
    base_sampling_offset: int = 0
    xstart: int = 0                         # cropped film: its origin in camera pixels (imagefilm.cc:66)
    ystart: int = 0
    rr_seed: int = 0                        # GPU-core "adv_rr_seed" (the oracle's OracleScene rr_seed)
    computer_node: int = 0
    # film load/save (imagefilm.cc:55-118)
    film_load_save_mode: str = "none"       # "save" | "load-save"
    film_load_save_path: str = "./"
    film_autosave_interval_type: str = "none"   # "pass-interval" | "time-interval"
    film_autosave_interval_passes: int = 1
    clamp_samples: float = 0.0
    accelerator: str = "yafaray-kdtree-original"
    # adaptive anti-aliasing (scene.cc:582-595; defaults of aa_noise_params.h:27-46)
    aa_passes: int = 1
    aa_inc_samples: int = 0                 # 0: AA_minsamples (scene.cc:584)
    aa_threshold: float = 0.05
    aa_resampled_floor: float = 0.0
    aa_sample_multiplier_factor: float = 1.0
    aa_detect_color_noise: bool = False
    aa_dark_detection_type: str = "none"    # none | linear | curve
    aa_dark_threshold_factor: float = 0.0
    aa_variance_edge_size: int = 10
    aa_variance_pixels: int = 0
    # photonmapping (integrator_photon_mapping.cc:765-850)
    pm_photons: int = 100000
    pm_search: int = 50
    pm_diffuse_radius: float = 0.1
    pm_bounces: int = 5
    pm_caustics: bool = False               # PhotonIntegrator / DirectLight "caustics"
    pm_caustic_photons: int = 500000        # PM "cPhotons"; DirectLight / PathIntegrator "photons"
    caustic_search: int = None              # "caustic_mix" (PM default: search; DL / PT: 100)
    caustic_radius: float = None            # PM "causticRadius" (0.01); DL / PT "caustic_radius" (0.25)
    caustic_depth: int = None               # DL / PT "caustic_depth" (10); PM uses "bounces"
    threads_photons: int = 1
    # PhotonIntegrator final gathering (factory :777-810; the reference default is on)
    pm_final_gather: bool = False
    fg_samples: int = 32
    pm_show_map: bool = False               # PhotonIntegrator "show_map" (integrator_photon_mapping.cc:876-881, 924-929)
    pm_do_ao: bool = False                  # PhotonIntegrator "do_AO" (affects only the AO render layers)
    # photon_maps_processing (PhotonIntegrator / PathIntegrator): generate, generate-save, load, reuse-previous;
    # the files are <film_load_save_path>_diffuse / _caustic / _fg_radiance.photonmap
    pm_maps_processing: str = "generate"
    fg_bounces: int = 2
    fg_min_pathlen: float = None            # default: diffuseRadius
    # DirectLight ambient occlusion (integrator_direct_light.cc:161-186)
    do_ao: bool = False
    ao_samples: int = 32
    ao_distance: float = 1.0
    ao_color: tuple = (1.0, 1.0, 1.0)
    aa_light_sample_multiplier_factor: float = 1.0
    aa_indirect_sample_multiplier_factor: float = 1.0


@dataclass
class Object:
    name: str
    v0: int            # first vertex (global index)
    nv: int
    t0: int            # first triangle (global index)
    nt: int
    uv0: int = 0       # first uv value (global index into SceneSpec.uvs)
    nuv: int = 0
    smooth_angle: Optional[float] = None   # yafaray_smoothMesh(name, angle) after endObject
    has_orco: bool = True                  # with SceneSpec.orco: addVertexWithOrco (else addVertex)


@dataclass
class SceneSpec:
    verts: np.ndarray                       # (N, 3) float32
    tris: np.ndarray                        # (M, 3) int32 — global vertex indices
    tri_mat: np.ndarray                     # (M,) int32 — index into materials
    materials: List[Material]
    lights: List[Light]
    camera: Camera
    render: Render
    background: Optional[Background] = None
    objects: List[Object] = field(default_factory=list)
    # surface attributes and textures (optional)
    orco: Optional[np.ndarray] = None       # (N, 3) per vertex: addVertexWithOrco
    normals: Optional[np.ndarray] = None    # (N, 3) per vertex: addNormal after the vertices
    uvs: Optional[np.ndarray] = None        # (U, 2) addUv values
    tri_uv: Optional[np.ndarray] = None     # (M, 3) global uv indices (-1: addTriangle)
    images: List[ImageSpec] = field(default_factory=list)
    textures: List[TextureSpec] = field(default_factory=list)

    def render_lights(self):
        """Lights in the order the integrators see them: by name (render_view.cc:61, std::map)."""
        return sorted(self.lights, key=lambda l: l.name)

    def with_render(self, **kw):
        import dataclasses
        return dataclasses.replace(self, render=dataclasses.replace(self.render, **kw))

    def with_camera(self, **kw):
        import dataclasses
        return dataclasses.replace(self, camera=dataclasses.replace(self.camera, **kw))


# ---------------------------------------------------------------------------------------------
# geometry helpers
# ---------------------------------------------------------------------------------------------

class _Builder:
    def __init__(self):
        self.verts, self.tris, self.tri_mat, self.objects = [], [], [], []

    def add_object(self, name, verts, tris, mat):
        v0, t0 = len(self.verts), len(self.tris)
        self.verts.extend([tuple(map(float, v)) for v in verts])
        self.tris.extend([(a + v0, b + v0, c + v0) for (a, b, c) in tris])
        self.tri_mat.extend([mat] * len(tris))
        self.objects.append(Object(name, v0, len(verts), t0, len(tris)))

    def arrays(self):
        return (np.asarray(self.verts, np.float32).reshape(-1, 3), np.asarray(self.tris, np.int32).reshape(-1, 3),
                np.asarray(self.tri_mat, np.int32))


def _quad(p0, p1, p2, p3):
    return [p0, p1, p2, p3], [(0, 1, 2), (0, 2, 3)]


def _box(cx, cy, sx, sy, h, angle_deg):
    a = math.radians(angle_deg)
    ca, sa = math.cos(a), math.sin(a)
    corners = []
    for dz in (0.0, h):
        for (ux, uy) in ((-sx, -sy), (sx, -sy), (sx, sy), (-sx, sy)):
            corners.append((cx + ux * ca - uy * sa, cy + ux * sa + uy * ca, dz))
    tris = [(0, 2, 1), (0, 3, 2),            # bottom
            (4, 5, 6), (4, 6, 7),            # top
            (0, 1, 5), (0, 5, 4), (1, 2, 6), (1, 6, 5), (2, 3, 7), (2, 7, 6), (3, 0, 4), (3, 4, 7)]
    return corners, tris


def cornell(width=1920, height=1080, spp=64, bounces=8, rr=False, integrator="pathtracing",
            filter_type="box", pixelwidth=1.0, light_samples=1, tile_size=32) -> SceneSpec:
    """BASELINE C2: Cornell box, area light 0.5 x 0.5 at z = 1.98 facing down, power 6."""
    b = _Builder()
    mats = [Material("white", color=(0.75, 0.75, 0.75)), Material("red", color=(0.75, 0.1, 0.1)),
            Material("green", color=(0.1, 0.75, 0.1))]
    W, R, G = 0, 1, 2
    b.add_object("floor", *_quad((-1, -1, 0), (1, -1, 0), (1, 1, 0), (-1, 1, 0)), W)
    b.add_object("ceiling", *_quad((-1, -1, 2), (-1, 1, 2), (1, 1, 2), (1, -1, 2)), W)
    b.add_object("back", *_quad((-1, 1, 0), (1, 1, 0), (1, 1, 2), (-1, 1, 2)), W)
    b.add_object("left", *_quad((-1, -1, 0), (-1, 1, 0), (-1, 1, 2), (-1, -1, 2)), R)
    b.add_object("right", *_quad((1, -1, 0), (1, -1, 2), (1, 1, 2), (1, 1, 0)), G)
    b.add_object("short_box", *_box(0.35, -0.25, 0.3, 0.3, 0.6, -17.0), W)
    b.add_object("tall_box", *_box(-0.35, 0.35, 0.3, 0.3, 1.2, 17.0), W)
    verts, tris, tri_mat = b.arrays()
    light = Light("area", type="arealight", color=(1.0, 1.0, 1.0), power=6.0, corner=(-0.25, -0.25, 1.98),
                  point1=(-0.25, 0.25, 1.98), point2=(0.25, -0.25, 1.98), samples=light_samples)
    cam = Camera(from_=(0.0, -3.9, 1.0), to=(0.0, 0.0, 1.0), up=(0.0, -3.9, 2.0), resx=width, resy=height,
                 focal=1.4)
    rend = Render(integrator=integrator, width=width, height=height, aa_samples=spp, filter_type=filter_type,
                  aa_pixelwidth=pixelwidth, tile_size=tile_size, bounces=bounces, path_samples=1,
                  rr_min_bounces=(0 if rr else bounces), caustic_type="none")
    return SceneSpec(verts, tris, tri_mat, mats, [light], cam, rend, Background((0.0, 0.0, 0.0), 1.0), b.objects)


def with_extra_lights(spec, n):
    """The scene with n lights: its own light, then a warm point bulb and a second (smaller, bluish) area
    light off-centre under the ceiling (multi-light tests; bench.py --lights)."""
    import dataclasses
    extra = [Light("bulb", type="pointlight", color=(1.0, 0.85, 0.7), power=1.2, from_=(0.45, -0.3, 1.5)),
             Light("panel", type="arealight", color=(0.6, 0.7, 1.0), power=2.5, corner=(-0.8, 0.5, 1.9),
                   point1=(-0.8, 0.8, 1.9), point2=(-0.5, 0.5, 1.9), samples=1)]
    return dataclasses.replace(spec, lights=list(spec.lights) + extra[:max(0, n - 1)])


def cornell_meshlight(width=96, height=72, spp=4, bounces=4, rr=False, integrator="pathtracing", shape="panel",
                      double_sided=False, samples=2, keep_area=False, power=3.0, **kw) -> SceneSpec:
    """The Cornell box lit by a meshlight (light_object_light.cc): an emitting object with a light_mat
    material whose faces the light samples.  shape "panel": a 0.6 x 0.6 quad (2 faces) under the
    ceiling facing down; "sphere": a low-poly UV sphere (72 faces of different areas) hanging in the
    box; "bigsphere": the same sphere with 71 x 71 x 2 = 10082 faces (the meshlight BVH case).
    keep_area: the box's area light stays as a second light."""
    s = cornell(width, height, spp=spp, bounces=bounces, rr=rr, integrator=integrator, **kw)
    if shape == "panel":
        lv, lt = _quad((-0.3, -0.3, 1.9), (-0.3, 0.3, 1.9), (0.3, 0.3, 1.9), (0.3, -0.3, 1.9))
        lv = np.asarray(lv, np.float32)
        lt = np.asarray(lt, np.int32)
    else:
        lv, lt = uv_sphere(71 if shape == "bigsphere" else 6, center=(0.35, -0.3, 1.45), r=0.18)
    mats = list(s.materials) + [Material("lamp", type="light_mat", color=(1.0, 0.9, 0.75), power=power, double_sided=double_sided)]
    v0 = len(s.verts)
    verts = np.concatenate([s.verts, np.asarray(lv, np.float32)])
    tris = np.concatenate([s.tris, np.asarray(lt, np.int32) + v0])
    tri_mat = np.concatenate([s.tri_mat, np.full(len(lt), len(mats) - 1, np.int32)])
    objs = list(s.objects) + [Object("lamp_mesh", v0, len(lv), len(s.tris), len(lt))]
    ml = Light("lamp", type="meshlight", color=(1.0, 0.9, 0.75), power=power, object_name="lamp_mesh", double_sided=double_sided,
               samples=samples)
    lights = (list(s.lights) if keep_area else []) + [ml]
    import dataclasses
    return dataclasses.replace(s, verts=verts, tris=tris, tri_mat=tri_mat, materials=mats, lights=lights, objects=objs)


def cornell_photon(width=1920, height=1080, spp=1, photons=10_000_000, search=50, radius=0.1, bounces=5,
                   caustics=False, **kw) -> SceneSpec:
    """BASELINE C5: the C2 Cornell box rendered by the PhotonIntegrator (diffuse photon map,
    k-NN density estimate, finalGather off — SURVEY.md §8d)."""
    import dataclasses
    s = cornell(width, height, spp=spp, integrator="photonmapping", **kw)
    r = dataclasses.replace(s.render, pm_photons=photons, pm_search=search, pm_diffuse_radius=radius,
                            pm_bounces=bounces, pm_caustics=caustics)
    return dataclasses.replace(s, render=r)


def uv_sphere(n=707, center=(0.0, 0.0, 1.0), r=0.5):
    """SURVEY.md §8d C4 generator: vertex (i, j) = r(sin t cos p, sin t sin p, cos t) + c,
    t = pi i / n, p = 2 pi j / n; faces (a, c, b), (b, c, d) per quad -> n * n * 2 triangles."""
    i = np.arange(n + 1, dtype=np.float64)[:, None]
    j = np.arange(n, dtype=np.float64)[None, :]
    th, ph = math.pi * i / n, 2.0 * math.pi * j / n
    x = r * np.sin(th) * np.cos(ph) + center[0]
    y = r * np.sin(th) * np.sin(ph) + center[1]
    z = r * np.cos(th) * np.ones_like(ph) + center[2]
    verts = np.stack([x, y, z], -1).reshape(-1, 3).astype(np.float32)
    ii, jj = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    a = ii * n + jj
    bb = ii * n + (jj + 1) % n
    c = (ii + 1) * n + jj
    d = (ii + 1) * n + (jj + 1) % n
    tris = np.stack([np.stack([a, c, bb], -1), np.stack([bb, c, d], -1)], 2).reshape(-1, 3).astype(np.int32)
    return verts, tris


def cornell_sphere(n=707, **kw) -> SceneSpec:
    """BASELINE C4: the C2 Cornell box plus a UV sphere (centre (0,0,1), r 0.5, white)."""
    s = cornell(**kw)
    sv, st = uv_sphere(n)
    v0 = len(s.verts)
    verts = np.concatenate([s.verts, sv])
    tris = np.concatenate([s.tris, st + v0])
    tri_mat = np.concatenate([s.tri_mat, np.zeros(len(st), np.int32)])
    objs = list(s.objects) + [Object("sphere", v0, len(sv), len(s.tris), len(st))]
    import dataclasses
    return dataclasses.replace(s, verts=verts, tris=tris, tri_mat=tri_mat, objects=objs)


GOLDEN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def test01(width=256, height=256, spp=4, filter_type="gauss", pixelwidth=1.5, tile_size=32) -> SceneSpec:
    """BASELINE C1: the reference's test01 scene, textures stripped (diffuse colour only)."""
    with open(os.path.join(GOLDEN_DIR, "test01_scene.json")) as f:
        d = json.load(f)
    b = _Builder()
    mat_names = [m["name"] for m in d["materials"]]
    mats = [Material(m["name"], color=tuple(m["color"]), diffuse_reflect=m["diffuse_reflect"], emit=m["emit"])
            for m in d["materials"]]
    for o in d["objects"]:
        b.add_object(o["name"], o["verts"], o["tris"], mat_names.index(o["material"]))
    verts, tris, tri_mat = b.arrays()
    lights = [Light(l["name"], type="pointlight", color=tuple(l["color"]), power=l["power"], from_=tuple(l["from"]))
              for l in d["lights"]]
    c = d["camera"]
    cam = Camera(from_=tuple(c["from"]), to=tuple(c["to"]), up=tuple(c["up"]), resx=width, resy=height,
                 focal=c["focal"])
    bg = Background(tuple(d["background"]["color"]), d["background"]["power"])
    rend = Render(integrator="directlighting", width=width, height=height, aa_samples=spp,
                  filter_type=filter_type, aa_pixelwidth=pixelwidth, tile_size=tile_size, raydepth=2)
    return SceneSpec(verts, tris, tri_mat, mats, lights, cam, rend, bg, b.objects)


TEX01_DIR = os.path.join(GOLDEN_DIR, "tex01")


def test01_textured(width=256, height=256, spp=4, filter_type="gauss", pixelwidth=1.5, tile_size=32) -> SceneSpec:
    """BASELINE C1 with the reference's own texturing: every createImage / createTexture /
    createMaterial call of tests/test01/test01.c (typed parameter maps + shader-node lists) and the
    cubes' orco coordinates.  Images resolve against tests/golden/tex01 (tex.tga, tex.hdr); the
    PNG / JPG / TIFF / EXR images fail to load exactly as in the reference built without those
    libraries (src/format/format.cc:40-66), which drops their textures and nodes."""
    import dataclasses
    s = test01(width, height, spp, filter_type, pixelwidth, tile_size)
    with open(os.path.join(GOLDEN_DIR, "test01_scene.json")) as f:
        d = json.load(f)
    mats = []
    for m, mf in zip(s.materials, d["materials_full"]):
        assert m.name == mf["name"]
        mats.append(dataclasses.replace(m, params={k: tuple(v) for k, v in mf["params"].items()},
                                        nodes=[{k: tuple(v) for k, v in nd.items()} for nd in mf["nodes"]]))
    images = [ImageSpec(im["name"], {k: tuple(v) for k, v in im["params"].items()}, TEX01_DIR) for im in d["images"]]
    textures = [TextureSpec(t["name"], {k: tuple(v) for k, v in t["params"].items()}) for t in d["textures"]]
    orco = np.asarray([oc for o in d["objects"] for oc in (o["orco"] if o["orco"] else o["verts"])], np.float32)
    has_orco = all(len(o["orco"]) == len(o["verts"]) for o in d["objects"] if o["orco"])
    assert has_orco
    # objects without orco (the plane) replay addVertex: their orco rows are placeholders
    objs = [dataclasses.replace(o, has_orco=bool(od["orco"])) for o, od in zip(s.objects, d["objects"])]
    return dataclasses.replace(s, materials=mats, images=images, textures=textures, orco=orco, objects=objs)


# ---------------------------------------------------------------------------------------------
# replay through the C API (the drop-in boundary)
# ---------------------------------------------------------------------------------------------

def set_typed(api, k, tv):
    """paramsSet* for one typed value (kind, value): s f i b v c m."""
    kind, v = tv
    if kind == "s":
        api.paramsSetString(k, v)
    elif kind == "f":
        api.paramsSetFloat(k, float(v))
    elif kind == "i":
        api.paramsSetInt(k, int(v))
    elif kind == "b":
        api.paramsSetBool(k, bool(v))
    elif kind == "v":
        api.paramsSetVector(k, *map(float, v))
    elif kind == "c":
        api.paramsSetColor(k, *map(float, v))
    elif kind == "m":
        api.paramsSetMatrix(k, *map(float, v), False)
    else:
        raise ValueError(f"unknown parameter kind {kind!r}")


@dataclass
class CausticParams:
    enabled: bool
    photons: int
    search: int
    radius: float
    depth: int


def caustic_params(r) -> CausticParams:
    """The caustic photon map settings of render spec `r` with each integrator's defaults
    (PhotonIntegrator::factory integrator_photon_mapping.cc:765-850, DirectLightIntegrator::factory
    integrator_direct_light.cc:147-190, PathIntegrator::factory integrator_path_tracer.cc:325-342)."""
    if r.integrator == "photonmapping":
        return CausticParams(bool(r.pm_caustics), r.pm_caustic_photons,
                             r.caustic_search if r.caustic_search is not None else r.pm_search,
                             r.caustic_radius if r.caustic_radius is not None else 0.01, r.pm_bounces)
    enabled = bool(r.pm_caustics) if r.integrator == "directlighting" else r.caustic_type in ("photon", "both")
    return CausticParams(enabled, r.pm_caustic_photons, r.caustic_search if r.caustic_search is not None else 100,
                         r.caustic_radius if r.caustic_radius is not None else 0.25,
                         r.caustic_depth if r.caustic_depth is not None else 10)


def apply(spec: SceneSpec, api) -> None:
    """Issue the reference C-API call sequence for `spec` on `api` (a libyafaray_amd.Interface)."""
    api.createScene()
    for im in spec.images:
        api.paramsClearAll()
        for k, tv in im.params.items():
            if k == "filename" and tv[1] and not os.path.isabs(tv[1]) and im.base_dir:
                tv = ("s", os.path.join(im.base_dir, tv[1]))
            set_typed(api, k, tv)
        h = api.createImage(im.name)
        for (x, y, c) in im.set_pixels:
            if h:
                api.setImageColor(h, x, y, *c)
    for t in spec.textures:
        api.paramsClearAll()
        for k, tv in t.params.items():
            set_typed(api, k, tv)
        api.createTexture(t.name)
    for m in spec.materials:
        api.paramsClearAll()
        if m.params is not None:
            for k, tv in m.params.items():
                set_typed(api, k, tv)
            for nd in m.nodes:
                api.paramsPushList()
                for k, tv in nd.items():
                    set_typed(api, k, tv)
            api.paramsEndList()
            api.createMaterial(m.name)
            continue
        api.paramsSetString("type", m.type)
        api.paramsSetColor("color", *m.color, 1.0)
        if m.type == "light_mat":
            api.paramsSetFloat("power", m.power)
            api.paramsSetBool("double_sided", m.double_sided)
        elif m.type == "mirror":
            api.paramsSetFloat("reflect", m.reflect)
        elif m.type == "null":
            pass
        else:
            api.paramsSetFloat("specular_reflect", m.specular_reflect)
            api.paramsSetFloat("transparency", m.transparency)
            api.paramsSetFloat("translucency", m.translucency)
            api.paramsSetFloat("transmit_filter", m.transmit_filter)
            api.paramsSetFloat("IOR", m.ior)
            api.paramsSetBool("fresnel_effect", m.fresnel)
            api.paramsSetColor("mirror_color", *m.mirror_color, 1.0)
            api.paramsSetFloat("transparentbias_factor", m.transparentbias_factor)
            api.paramsSetBool("transparentbias_multiply_raydepth", m.transparentbias_multiply_raydepth)
            api.paramsSetFloat("diffuse_reflect", m.diffuse_reflect)
            api.paramsSetFloat("emit", m.emit)
            api.paramsSetBool("receive_shadows", m.receive_shadows)
            api.paramsSetBool("flat_material", m.flat_material)
            if m.diffuse_brdf != "lambert":
                api.paramsSetString("diffuse_brdf", m.diffuse_brdf)
                api.paramsSetFloat("sigma", m.sigma)
            if m.additionaldepth:
                api.paramsSetInt("additionaldepth", m.additionaldepth)
        api.createMaterial(m.name)
    api.paramsClearAll()
    for l in spec.lights:
        api.paramsClearAll()
        api.paramsSetString("type", l.type)
        api.paramsSetColor("color", *l.color, 1.0)
        api.paramsSetFloat("power", l.power)
        api.paramsSetBool("cast_shadows", l.cast_shadows)
        if not l.with_caustic:
            api.paramsSetBool("with_caustic", False)
        if not l.with_diffuse:
            api.paramsSetBool("with_diffuse", False)
        if l.photon_only:
            api.paramsSetBool("photon_only", True)
        if l.type == "pointlight":
            api.paramsSetVector("from", *l.from_)
        elif l.type in ("meshlight", "objectlight"):
            api.paramsSetString("object_name", l.object_name)
            api.paramsSetBool("double_sided", l.double_sided)
            api.paramsSetInt("samples", l.samples)
        else:
            api.paramsSetVector("corner", *l.corner)
            api.paramsSetVector("point1", *l.point1)
            api.paramsSetVector("point2", *l.point2)
            api.paramsSetInt("samples", l.samples)
        api.createLight(l.name)
    for o in spec.objects:
        api.paramsClearAll()
        api.paramsSetString("type", "mesh")
        api.paramsSetInt("num_vertices", o.nv)
        api.paramsSetInt("num_faces", o.nt)
        use_orco = spec.orco is not None and o.has_orco
        api.paramsSetBool("has_orco", use_orco)
        api.paramsSetBool("has_uv", o.nuv > 0)
        api.createObject(o.name)
        if use_orco:
            for v, oc in zip(spec.verts[o.v0:o.v0 + o.nv], spec.orco[o.v0:o.v0 + o.nv]):
                api.addVertexWithOrco(*map(float, v), *map(float, oc))
        else:
            api.addVertices(spec.verts[o.v0:o.v0 + o.nv])
        if spec.normals is not None:
            for n in spec.normals[o.v0:o.v0 + o.nv]:
                api.addNormal(*map(float, n))
        for k in range(o.nuv):
            api.addUv(*map(float, spec.uvs[o.uv0 + k]))
        tri = spec.tris[o.t0:o.t0 + o.nt] - o.v0
        mats = spec.tri_mat[o.t0:o.t0 + o.nt]
        if spec.tri_uv is not None and o.nuv > 0:
            tuv = spec.tri_uv[o.t0:o.t0 + o.nt]
            cur = None
            for k in range(o.nt):
                if mats[k] != cur:
                    cur = mats[k]
                    api.setCurrentMaterial(spec.materials[int(cur)].name)
                a, b, c = map(int, tri[k])
                if tuv[k][0] >= 0:
                    api.addTriangleWithUv(a, b, c, *(int(u) - o.uv0 for u in tuv[k]))
                else:
                    api.addTriangle(a, b, c)
            api.endObject()
            if o.smooth_angle is not None:
                api.smoothMesh(o.name, float(o.smooth_angle))
            continue
        # setCurrentMaterial + addTriangle runs (object_mesh.cc:78-86)
        start = 0
        while start < len(tri):
            end = start
            while end < len(tri) and mats[end] == mats[start]:
                end += 1
            api.setCurrentMaterial(spec.materials[int(mats[start])].name)
            api.addTriangles(tri[start:end])
            start = end
        api.endObject()
        if o.smooth_angle is not None:
            api.smoothMesh(o.name, float(o.smooth_angle))
    cam = spec.camera
    api.paramsClearAll()
    api.paramsSetString("type", "perspective")
    api.paramsSetVector("from", *cam.from_)
    api.paramsSetVector("to", *cam.to)
    api.paramsSetVector("up", *cam.up)
    api.paramsSetInt("resx", cam.resx)
    api.paramsSetInt("resy", cam.resy)
    api.paramsSetFloat("focal", cam.focal)
    api.paramsSetFloat("aspect_ratio", cam.aspect_ratio)
    api.paramsSetFloat("nearClip", cam.near_clip)
    api.paramsSetFloat("farClip", cam.far_clip)
    if cam.aperture != 0.0:
        api.paramsSetFloat("aperture", cam.aperture)
        api.paramsSetFloat("dof_distance", cam.dof_distance)
        api.paramsSetString("bokeh_type", cam.bokeh_type)
        api.paramsSetString("bokeh_bias", cam.bokeh_bias)
        api.paramsSetFloat("bokeh_rotation", cam.bokeh_rotation)
    api.createCamera("cam")
    api.paramsClearAll()
    api.paramsSetString("camera_name", "cam")
    api.createRenderView("")
    if spec.background is not None:
        api.paramsClearAll()
        api.paramsSetString("type", "constant")
        api.paramsSetColor("color", *spec.background.color, 1.0)
        api.paramsSetFloat("power", spec.background.power)
        api.createBackground("world_background")
    r = spec.render
    cm = caustic_params(r)
    api.paramsClearAll()
    api.paramsSetString("type", r.integrator)
    api.paramsSetInt("raydepth", r.raydepth)
    api.paramsSetBool("bg_transp", r.bg_transp)
    api.paramsSetBool("bg_transp_refract", r.bg_transp_refract)
    api.paramsSetBool("transpShad", r.transp_shad)
    api.paramsSetInt("shadowDepth", r.shadow_depth)
    if r.integrator == "pathtracing":
        api.paramsSetInt("bounces", r.bounces)
        api.paramsSetInt("path_samples", r.path_samples)
        api.paramsSetInt("russian_roulette_min_bounces", r.rr_min_bounces)
        api.paramsSetString("caustic_type", r.caustic_type)
    if r.integrator in ("pathtracing", "directlighting") and cm.enabled:
        api.paramsSetInt("photons", cm.photons)
        api.paramsSetInt("caustic_mix", cm.search)
        api.paramsSetInt("caustic_depth", cm.depth)
        api.paramsSetFloat("caustic_radius", cm.radius)
    if r.integrator == "photonmapping":
        api.paramsSetInt("photons", r.pm_photons)
        api.paramsSetInt("cPhotons", r.pm_caustic_photons)
        api.paramsSetInt("search", r.pm_search)
        api.paramsSetFloat("diffuseRadius", r.pm_diffuse_radius)
        api.paramsSetInt("bounces", r.pm_bounces)
        api.paramsSetBool("caustics", r.pm_caustics)
        api.paramsSetInt("caustic_mix", cm.search)
        api.paramsSetFloat("causticRadius", cm.radius)
        api.paramsSetBool("finalGather", bool(r.pm_final_gather))
        if r.pm_show_map:
            api.paramsSetBool("show_map", True)
        if r.pm_do_ao:
            api.paramsSetBool("do_AO", True)
        if r.pm_final_gather:
            api.paramsSetInt("fg_samples", r.fg_samples)
            api.paramsSetInt("fg_bounces", r.fg_bounces)
            if r.fg_min_pathlen is not None:
                api.paramsSetFloat("fg_min_pathlen", r.fg_min_pathlen)
    if r.integrator == "directlighting" and r.pm_caustics:
        api.paramsSetBool("caustics", True)
    if r.integrator == "directlighting" and r.do_ao:
        api.paramsSetBool("do_AO", True)
        api.paramsSetInt("AO_samples", r.ao_samples)
        api.paramsSetFloat("AO_distance", r.ao_distance)
        api.paramsSetColor("AO_color", *r.ao_color, 1.0)
    if r.integrator in ("pathtracing", "photonmapping") and r.pm_maps_processing != "generate":
        api.paramsSetString("photon_maps_processing", r.pm_maps_processing)
    api.createIntegrator("default")
    api.paramsClearAll()
    api.paramsSetString("type", "combined")
    api.paramsSetString("image_type", "ColorAlpha")
    api.defineLayer()
    api.paramsClearAll()
    api.paramsSetString("integrator_name", "default")
    if spec.background is not None:
        api.paramsSetString("background_name", "world_background")
    api.paramsSetInt("width", r.width)
    api.paramsSetInt("height", r.height)
    if r.xstart or r.ystart:
        api.paramsSetInt("xstart", r.xstart)
        api.paramsSetInt("ystart", r.ystart)
    api.paramsSetInt("AA_minsamples", r.aa_samples)
    api.paramsSetInt("AA_passes", r.aa_passes)
    if r.aa_inc_samples > 0:
        api.paramsSetInt("AA_inc_samples", r.aa_inc_samples)
    api.paramsSetFloat("AA_threshold", r.aa_threshold)
    api.paramsSetFloat("AA_resampled_floor", r.aa_resampled_floor)
    api.paramsSetFloat("AA_sample_multiplier_factor", r.aa_sample_multiplier_factor)
    api.paramsSetFloat("AA_light_sample_multiplier_factor", r.aa_light_sample_multiplier_factor)
    api.paramsSetFloat("AA_indirect_sample_multiplier_factor", r.aa_indirect_sample_multiplier_factor)
    api.paramsSetBool("AA_detect_color_noise", r.aa_detect_color_noise)
    api.paramsSetString("AA_dark_detection_type", r.aa_dark_detection_type)
    api.paramsSetFloat("AA_dark_threshold_factor", r.aa_dark_threshold_factor)
    api.paramsSetInt("AA_variance_edge_size", r.aa_variance_edge_size)
    api.paramsSetInt("AA_variance_pixels", r.aa_variance_pixels)
    api.paramsSetString("filter_type", r.filter_type)
    api.paramsSetFloat("AA_pixelwidth", r.aa_pixelwidth)
    api.paramsSetFloat("AA_clamp_samples", r.clamp_samples)
    api.paramsSetInt("tile_size", r.tile_size)
    api.paramsSetString("tiles_order", r.tiles_order)
    api.paramsSetBool("adv_auto_shadow_bias_enabled", r.shadow_bias_auto)
    api.paramsSetFloat("adv_shadow_bias_value", r.shadow_bias)
    api.paramsSetBool("adv_auto_min_raydist_enabled", r.ray_min_dist_auto)
    api.paramsSetFloat("adv_min_raydist_value", r.ray_min_dist)
    api.paramsSetInt("adv_base_sampling_offset", r.base_sampling_offset)
    if r.rr_seed:
        api.paramsSetInt("adv_rr_seed", r.rr_seed)
    api.paramsSetInt("adv_computer_node", r.computer_node)
    api.paramsSetString("film_load_save_mode", r.film_load_save_mode)
    api.paramsSetString("film_load_save_path", r.film_load_save_path)
    api.paramsSetString("film_autosave_interval_type", r.film_autosave_interval_type)
    api.paramsSetInt("film_autosave_interval_passes", r.film_autosave_interval_passes)
    api.paramsSetString("scene_accelerator", r.accelerator)
    api.paramsSetInt("threads", -1)
    api.paramsSetInt("threads_photons", r.threads_photons)
    api.setupRender()
    api.paramsClearAll()


def cornell_specular(width=64, height=48, spp=2, integrator="directlighting", bounces=4, raydepth=5, fresnel=True,
                     rr=False, **kw) -> SceneSpec:
    """The C2 Cornell box with the shinydiffuse components the configs leave at zero and the mirror
    material: tall box mirror + diffuse (Fresnel), short box transparent with a transmit filter
    and translucency, back wall a `mirror` material (MonteCarloIntegrator::recursiveRaytrace,
    material_shiny_diffuse.cc:249-433, material_glass.cc:435-460)."""
    import dataclasses
    s = cornell(width, height, spp=spp, bounces=bounces, rr=rr, integrator=integrator, **kw)
    mats = list(s.materials) + [
        Material("tall_mirror", color=(0.7, 0.7, 0.75), specular_reflect=0.7, fresnel=fresnel, ior=1.6,
                 mirror_color=(0.9, 0.85, 0.8)),
        Material("short_glassy", color=(0.3, 0.8, 0.4), transparency=0.7, transmit_filter=0.6, translucency=0.2,
                 diffuse_reflect=0.5, specular_reflect=0.1, transparentbias_factor=0.001),
        Material("back_mirror", type="mirror", color=(0.8, 0.9, 1.0), reflect=0.75)]
    tri_mat = s.tri_mat.copy()
    names = [o.name for o in s.objects]
    for o in s.objects:
        if o.name == "tall_box":
            tri_mat[o.t0:o.t0 + o.nt] = len(s.materials)
        elif o.name == "short_box":
            tri_mat[o.t0:o.t0 + o.nt] = len(s.materials) + 1
        elif o.name == "back":
            tri_mat[o.t0:o.t0 + o.nt] = len(s.materials) + 2
    r = dataclasses.replace(s.render, raydepth=raydepth)
    return dataclasses.replace(s, materials=mats, tri_mat=tri_mat, render=r)


def cornell_transparent_shadows(width=64, height=48, spp=2, integrator="directlighting", panes=2, shadow_depth=5,
                                point_light=False, bounces=3, pane_step=0.15, pane_shrink=0.05, pane_alpha=None,
                                **kw) -> SceneSpec:
    """Transparent shadows (MonteCarloIntegrator tr_shad_, accelerator_kdtree.cc:916-1061): the C2
    Cornell box with `panes` stacked transparent shinydiffuse panes under the light (tinted, with
    transmit filters), a transparent Fresnel + mirror tall box and a transparent + translucent short
    box, so that shadow rays cross 0 .. panes + 2 transparent surfaces; `shadow_depth` is the
    integrator's shadowDepth.  With point_light a point light replaces the area light (diracLight)."""
    import dataclasses
    s = cornell(width, height, spp=spp, bounces=bounces, rr=False, integrator=integrator, **kw)
    b = _Builder()
    b.verts = [tuple(v) for v in s.verts.tolist()]
    b.tris = [tuple(t) for t in s.tris.tolist()]
    b.tri_mat = [int(m) for m in s.tri_mat]
    b.objects = list(s.objects)
    tints = [(0.9, 0.3, 0.3), (0.3, 0.9, 0.4), (0.35, 0.45, 0.95), (0.9, 0.9, 0.3)]
    mats = list(s.materials)
    for k in range(panes):
        z = 1.6 - pane_step * k
        h = 0.45 - pane_shrink * k
        # pane_alpha: every pane equally transparent (deep stacks: shadowDepth tests)
        mats.append(Material(f"pane{k}", color=tints[k % len(tints)], transparency=(0.8 - 0.1 * k) if pane_alpha is None else pane_alpha,
                             transmit_filter=(0.9 - 0.2 * k) if pane_alpha is None else 0.5, diffuse_reflect=0.6))
        b.add_object(f"pane{k}", *_quad((-h, -h, z), (h, -h, z), (h, h, z), (-h, h, z)), len(mats) - 1)
    verts, tris, tri_mat = b.arrays()
    mats.append(Material("tall_glass", color=(0.6, 0.7, 0.9), transparency=0.6, transmit_filter=0.5,
                         specular_reflect=0.3, fresnel=True, ior=1.5, diffuse_reflect=0.4))
    mats.append(Material("short_transl", color=(0.8, 0.6, 0.3), transparency=0.4, translucency=0.3,
                         transmit_filter=0.7, diffuse_reflect=0.5))
    for o in b.objects:
        if o.name == "tall_box":
            tri_mat[o.t0:o.t0 + o.nt] = len(mats) - 2
        elif o.name == "short_box":
            tri_mat[o.t0:o.t0 + o.nt] = len(mats) - 1
    lights = s.lights
    if point_light:
        lights = [Light("point", type="pointlight", color=(1.0, 1.0, 1.0), power=3.0, from_=(0.1, -0.1, 1.9))]
    r = dataclasses.replace(s.render, transp_shad=True, shadow_depth=shadow_depth, raydepth=2)
    return dataclasses.replace(s, verts=verts, tris=tris, tri_mat=tri_mat, materials=mats, lights=lights,
                               objects=b.objects, render=r)
