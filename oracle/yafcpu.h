// TEST INFRASTRUCTURE ONLY — the CPU oracle for the path-tracing hot path.
//
// A plain C++ restatement of libYafaRay's per-sample Monte Carlo loop (tiled sample loop,
// DirectLight and Path integrators, MC light estimation, shinydiffuse/light_mat materials,
// point/area lights, perspective camera, film splatting) written scalar and close to the
// reference's own code structure, with `long double` wherever the reference's expressions
// promote to x87 80-bit.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
// may load it; the product path (libyafaray_amd) never does.
//
// Parity status: the numeric building blocks (samplers, Halton/Faure, FAST_TRIG sin/cos,
// cosHemisphere, Vec3, Bound::cross, MWC, gauss filter, rounding helpers) are PINNED against the
// reference's own code compiled in oracle/_ref (tests/golden/prims.npz).  The integrator
// composition is a restatement (reference library unbuildable here).

#pragma once
#include <cstdint>

extern "C" {

enum { YC_MAT_SHINYDIFFUSE = 0, YC_MAT_LIGHT = 1, YC_MAT_MIRROR = 2, YC_MAT_NULL = 3 };
enum { YC_LIGHT_POINT = 0, YC_LIGHT_AREA = 1, YC_LIGHT_MESH = 2 };
enum { YC_INT_DIRECT = 0, YC_INT_PATH = 1, YC_INT_PHOTON = 2 };
enum { YC_FILTER_BOX = 0, YC_FILTER_GAUSS = 1, YC_FILTER_MITCHELL = 2, YC_FILTER_LANCZOS = 3 };

typedef struct {
	int type;                 // YC_MAT_*
	float color[3];           // shinydiffuse diffuse colour / light_mat colour (already * power)
	float diffuse_strength;   // shinydiffuse "diffuse_reflect"
	float emit_strength;      // shinydiffuse "emit"
	int double_sided;         // light_mat
	int receive_shadows;
	int flat_material;
	int diffuse_shader;       // shader-node roots (indices into yc_scene.nodes, -1: none)
	int diffuse_refl_shader;
	// shinydiffuse specular / transparent / translucent components (material_shiny_diffuse.cc:490-566);
	// mirror material: color * reflect (material_glass.cc:453-460)
	float specular_reflect, transparency, translucency, transmit_filter, ior;
	int fresnel_effect;
	float mirror_color[3];
	float transparentbias_factor;
	int transparentbias_multiply_raydepth;
	float reflect;            // mirror material
	// ShinyDiffuseMaterial::factory (material_shiny_diffuse.cc:507, 561-571): additionaldepth,
	// diffuse_brdf = "oren_nayar" with "sigma" (double), root "sigma_oren_shader" (yc_scene.nodes, -1: none)
	int additional_depth;
	int oren_nayar;
	double sigma;
	int sigma_shader;
} yc_material;

// ---- texturing (material_node.cc, texture_image.cc, shader_node_*.cc; see yaftex.h) ----
typedef struct {
	int format;               // 0: no file (empty image of width x height), 1: TGA bytes, 2: Radiance HDR bytes
	const uint8_t *data; int size;
	int type;                 // Image::Type: 0 none, 1 gray, 2 gray+alpha, 3 color, 4 color+alpha
	int optimization;         // 0 none, 1 optimized, 2 compressed
	int color_space;          // ColorSpace (color.h:36): 1 raw/gamma, 2 linear, 3 sRGB, 4 XYZ
	float gamma;
	int width, height;
	int n_set; const int *set_xy; const float *set_rgba;   // yafaray_setImageColor calls, in order
} yc_image;

typedef struct {
	int image;
	int interpolation;        // 0 none, 1 bilinear, 2 bicubic
	int clip;                 // ImageTexture::ClipMode: 0 extend, 1 clip, 2 clipcube, 3 repeat, 4 checker
	int xrepeat, yrepeat;
	int mirror_x, mirror_y, rot90, even_tiles, odd_tiles;
	float cropmin_x, cropmin_y, cropmax_x, cropmax_y, checker_dist;
	float intensity, contrast, saturation, hue, factor_red, factor_green, factor_blue;   // hue in degrees
	int clamp;
} yc_texture;

typedef struct {
	int type;                 // 0 value, 1 mix, 2 layer, 3 texture_mapper
	int blend;                // 0 mix 1 add 2 multiply 3 subtract 4 screen 5 divide 6 difference 7 darken 8 lighten 9 overlay
	int input[3];             // mix: input1, input2, factor; layer: input, upper_layer (node indices, -1 none)
	int no_rgb, stencil, negative, do_color, do_scalar, color_input, use_alpha;   // layer (do_scalar: also mapper)
	int texture, coords, projection, map[3];      // mapper: coords 0 uv 1 global 2 orco 3 transformed; proj 0 plain 1 cube 2 tube 3 sphere
	float col1[4], col2[4];   // value colour+alpha / mix color1, color2 / layer def_col, upper_color
	float val[4];             // value scalar / mix cfactor, val1, val2 / layer colfac, valfac, def_val, upper_value
	float scale[3], offset[3];
	float mtx[16];
} yc_node;

typedef struct {
	int v0, nv, t0, nt;       // vertex / triangle ranges of the object
	int has_orco;             // orco given per vertex (yc_scene.orco rows of this object)
	int has_uv;               // addUv values exist for this object
	int normals_exported;     // addNormal per vertex before the faces (yc_scene.normals rows)
	int smooth;               // smoothMesh called after endObject
	float smooth_angle;
} yc_object;

typedef struct {
	int type;                 // YC_LIGHT_*
	float color[3];           // raw colour param
	float power;
	float from[3];            // point light position / area light corner
	float point1[3];          // area light
	float point2[3];          // area light
	int samples;              // area light
	int cast_shadows;
	int shoot_caustic;        // "with_caustic" (getLightsEmittingCausticPhotons)
	int shoot_diffuse;        // "with_diffuse" (getLightsEmittingDiffusePhotons)
	int object;               // meshlight: index into yc_scene::objects
	int double_sided;         // meshlight
	int photon_only;          // shoots photons only: not in the integrators' light list (render_view.cc:83-91)
} yc_light;

typedef struct {
	float from[3], to[3], up[3];
	int resx, resy;
	float focal, aspect;
	float near_clip, far_clip;
	float aperture, dof_distance, bokeh_rotation;   // depth of field (camera_perspective.cc:28-52)
	int bokeh_type;                                 // BokehType: 0 disk1, 1 disk2, 3..6 polygons, 7 ring
	int bokeh_bias;                                 // 0 uniform, 1 center, 2 edge
} yc_camera;

typedef struct {
	int integrator;           // YC_INT_*
	int width, height;        // film
	int aa_samples;           // AA_minsamples (single pass)
	int filter;               // YC_FILTER_*
	float filter_size;        // AA_pixelwidth
	int tile_size;
	int bounces, path_samples, rr_min_bounces;
	int caustic_path;         // PathIntegrator caustic_type != none && != photon
	int has_background;
	float bg_color[3];        // constant background colour * power
	int bg_transp;
	int shadow_bias_auto; float shadow_bias;
	int ray_min_dist_auto; float ray_min_dist;
	int base_sampling_offset;
	float clamp_samples;
	int threads;              // oracle worker threads for the sample loop (film order is fixed)
	uint32_t rr_seed;         // stand-in for the reference's glibc rand() per-tile seed term
	// photon mapping (integrator_photon_mapping.cc factory :765-850; finalGather = false only)
	int pm_photons;           // "photons" (diffuse map)
	int pm_search;            // "search" (k of the k-NN gather)
	float pm_diffuse_radius;  // "diffuseRadius" — used as the SQUARED gather radius (:954)
	int pm_bounces;           // "bounces"
	int pm_caustics;          // unused (kept for layout); the caustic map is caus_map below
	int pm_threads;           // threads_photons: the photon count is rounded to a multiple (:437)
	// adaptive anti-aliasing (scene.cc:582-595, aa_noise_params.h:27-46; integrator_tiled.cc:172-231)
	int aa_passes;
	int aa_inc_samples;
	float aa_threshold;
	float aa_resampled_floor;            // % of the pixels
	float aa_sample_multiplier_factor;
	int aa_detect_color_noise;
	int aa_dark_detection_type;          // 0 none, 1 linear, 2 curve
	float aa_dark_threshold_factor;
	int aa_variance_edge_size;
	int aa_variance_pixels;
	int raydepth;             // recursiveRaytrace depth (DirectLight / PathIntegrator "raydepth")
	int bg_transp_refract;
	// transparent shadows (integrator "transpShad" / "shadowDepth", MonteCarloIntegrator tr_shad_ / s_depth_)
	int transp_shad, shadow_depth;
	// DirectLight ambient occlusion (integrator_direct_light.cc:161-163, 183-186): do_AO, AO_samples,
	// AO_distance, AO_color; AA_light_sample_multiplier_factor (scene.cc:589, integrator_tiled.cc:190)
	int do_ao, ao_samples;
	float ao_dist;
	float ao_col[3];
	float aa_light_sample_multiplier_factor;
	// caustic photon map (MonteCarloIntegrator::createCausticMap / causticWorker, integrator_montecarlo.cc
	// :410-640): PhotonIntegrator "caustics" (cPhotons, causticRadius, caustic_mix, bounces),
	// DirectLight "caustics" and PathIntegrator caustic_type photon|both (photons, caustic_radius,
	// caustic_mix, caustic_depth)
	int caus_map;
	int caus_photons, caus_search, caus_depth;
	float caus_radius;
	int tiles_order;          // 0 linear, 1 centre (the reference default), 2 random (fixed seed)
	// PhotonIntegrator final gathering (integrator_photon_mapping.cc:39-88, 183-193, 540-591, 640-763,
	// 874-917; factory :777-810): finalGather, fg_samples, fg_bounces, fg_min_pathlen
	int pm_fg;
	int fg_samples, fg_bounces;
	float fg_min_pathlen;
	// cropped film (imagefilm.cc:66, 129-132): the film covers camera pixels [crop_x0, crop_x0 + width)
	// x [crop_y0, crop_y0 + height); pixel sampling and camera rays use the camera's coordinates
	int crop_x0, crop_y0;
	// PhotonIntegrator "show_map" (integrator_photon_mapping.cc:876-881, 924-929): the nearest photon's
	// colour (radiance map with final gathering, else the diffuse map) instead of the estimates
	int pm_show_map;
	// photon_maps_processing "load" (integrator_photon_mapping.cc:279-326, montecarlo.cc:548-563): the
	// maps come from <pm_load_path>_caustic / _diffuse / _fg_radiance.photonmap (PhotonMap::load,
	// photon.cc:54-87); a failed load generates them.  NULL: generate.
	const char *pm_load_path;
	// AA_indirect_sample_multiplier_factor (integrator_tiled.cc:191): final gathering's paths per pass
	float aa_indirect_sample_multiplier_factor;
} yc_render;

typedef struct {
	int n_verts; const float *verts;
	int n_tris; const int *tris; const int *tri_mat;
	int n_mats; const yc_material *mats;
	int n_lights; const yc_light *lights;   // already in render order (alphabetical by name)
	yc_camera cam;
	yc_render rp;
	// optional texturing / surface attributes (all NULL / 0 for untextured flat scenes)
	int n_objects; const yc_object *objects;
	const float *orco;        // n_verts x 3
	const float *normals;     // n_verts x 3 (exported normals)
	const float *uvs;         // uv values, 2 per entry
	const int *tri_uv;        // n_tris x 3 global uv indices (-1: none)
	int n_images; const yc_image *images;
	int n_textures; const yc_texture *textures;
	int n_nodes; const yc_node *nodes;
} yc_scene;

typedef struct {
	uint64_t closest_rays, shadow_rays;
} yc_counters;

// Renders rows [y0, y1) of the film (all rows if y1 <= y0).  rgba: width*height*4 floats
// (normalized, the put-pixel/flush values), weights: width*height (may be NULL).  The film pass
// walks the reference's linear tile order, so results do not depend on `threads`.
int yc_render_image(const yc_scene *scene, int y0, int y1, float *rgba, float *weights, yc_counters *counters);

// Photon map of a PhotonIntegrator scene (shot in photon-id order, the reference's one-thread
// order): positions/directions/colours (3 floats each) and the point kd-tree (2 uint32 per node:
// split-position bits or photon index, flags).  Returns the photon count (n_paths in *n_paths),
// or -1.  Pass NULL buffers to query the count.
int yc_photon_map(const yc_scene *scene, float *pos, float *dir, float *col, uint32_t *nodes, int *n_paths);
void yc_shirley_disk(const float *r12, float *uv, int n);
int yc_tiles(int w, int h, int bs, int order, int *out, int cap);
void yc_glibc_rand(uint32_t seed, int n, uint32_t *out);
void yc_rgbe_decode(const uint8_t *rgbe, float *rgb, int n);
int yc_photon_map_ex(const yc_scene *scene, int which, float *pos, float *dir, float *col, uint32_t *nodes, int *n_paths);

// Per-sample radiance for a list of (x, y, s) camera samples (RGBA per sample).
int yc_render_samples(const yc_scene *scene, int n, const int *xys, float *rgba);

// Ray-level oracle: closest hit / any hit against the scene triangles.
// rays: 8 floats each (from xyz, dir xyz, tmin, tmax(<0 = inf)).
// hit out: 4 floats (t, bary_u, bary_v, bary_w) + prim index (-1 = miss).
int yc_trace_closest(const yc_scene *scene, int n, const float *rays, float *hit, int *prim);
int yc_trace_shadow(const yc_scene *scene, int n, const float *rays, int *occluded);

// Numeric building blocks (pinned against oracle/_ref).
void yc_riVdC(const uint32_t *bits, const uint32_t *r, float *out, int n);
void yc_riS(const uint32_t *bits, const uint32_t *r, float *out, int n);
void yc_riLp(const uint32_t *bits, const uint32_t *r, float *out, int n);
void yc_fnv32(const uint32_t *in, uint32_t *out, int n);
void yc_lds(const int *dim, const uint32_t *idx, double *out, int n);
void yc_halton_seq(int base, uint32_t start, int steps, float *out);
void yc_sin(const float *x, float *out, int n);
void yc_cos(const float *x, float *out, int n);
void yc_exp(const float *x, float *out, int n);
void yc_cos_hemisphere(const float *n_ru_rv, const float *s, float *out, int n);
void yc_coords_system(const float *in, float *out, int n);
void yc_normalize(const float *in, float *out, int n);
void yc_bound_cross(const float *box, const float *ray, float *out, int n);
void yc_mwc(uint32_t seed, int steps, double *out);
void yc_filter_gauss(const float *dxdy, float *out, int n);
void yc_round_to_int(const double *v, int *out, int n);
void yc_floor_to_int(const double *v, int *out, int n);
void yc_clamp_proportional(const float *rgb, float max_value, float *out, int n);
void yc_film_table(int filter, float filter_size, float *table16x16, float *filterw, float *table_scale);

}
