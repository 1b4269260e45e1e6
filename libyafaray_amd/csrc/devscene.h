// Plain-old-data layout shared by the host driver (render.cc) and the HIP kernels
// (kernels.hip).  Everything the hot path reads per sample lives in HBM in these layouts:
//
//   nodes   : BVH2 with both child boxes stored in the parent, 4 x float4 = 64 B per node
//             n0 = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)   n1 = (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
//             n2 = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)   n3 = (child0, child1, count0, count1)
//             child >= 0: inner node index; child < 0: leaf, triangles [~child, ~child + count)
//   tris    : triangles in leaf order, 3 x float4 = 48 B: (v0, eps) (e1, prim) (e2, 0) — the
//             Moller-Trumbore operands of primitive_triangle.cc:47-49 precomputed on the host with
//             the same float operations, so the device test is bit-identical to the reference's.
//   prim_ng : per original primitive (ng.xyz, material index) — TrianglePrimitive::getSurface.
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

namespace yafamd
{
struct DevStats;

// Final gathering's radiance map as a dense uniform grid (fgthin.hip yafamd_rad_grid, r06), next to its point
// kd-tree: cells of `cell` >= half the lookup radius, the photons in cell order (pos: position + the photon's
// index in the map's arrays as bits; dir: its normal), start[c] .. start[c + 1] the photons of cell c (cells
// x-fastest).  findNearest over it (kernels.hip gridNearest) returns the kd search's photon whenever the nearest
// facing distance is unique; a tie falls back to the kd search (the reference's visit order decides it).
struct RadGrid
{
	const uint32_t *start;   // null: no grid
	const float4 *pos;
	const float4 *dir;
	float lo[3];
	float cell, inv_cell;
	int nx, ny, nz;
};

enum : uint32_t
{
	B_NONE = 0, B_SPECULAR = 1u << 0, B_GLOSSY = 1u << 1, B_DIFFUSE = 1u << 2, B_DISPERSIVE = 1u << 3,
	B_REFLECT = 1u << 4, B_TRANSMIT = 1u << 5, B_FILTER = 1u << 6, B_EMIT = 1u << 7, B_VOLUMETRIC = 1u << 8,
	B_ALL = B_SPECULAR | B_GLOSSY | B_DIFFUSE | B_DISPERSIVE | B_REFLECT | B_TRANSMIT | B_FILTER
};

enum : uint32_t { MAT_SHINYDIFFUSE = 0, MAT_LIGHT = 1, MAT_MIRROR = 2, MAT_NULL = 3 };
// ShinyDiffuseMaterial components and options (material_shiny_diffuse.cc:38-87, 548-566)
enum : uint32_t { SD_MIRROR = 1u, SD_TRANSPARENT = 2u, SD_TRANSLUCENT = 4u, SD_DIFFUSE = 8u, SD_FRESNEL = 16u, SD_TBIAS_MULT = 32u,
                  SD_OREN_NAYAR = 64u };
enum : uint32_t { LIGHT_POINT = 0, LIGHT_AREA = 1, LIGHT_MESH = 2 };
constexpr int kMeshTriF4 = 7;   // float4 per meshlight face (DevScene::mesh_tris)
enum : int { INT_DIRECT = 0, INT_PATH = 1, INT_PHOTON = 2 };

struct DevMaterial
{
	uint32_t type, bsdf_flags, n_bsdf, double_sided;
	uint32_t receive_shadows, flat;
	int add_depth;          // additionaldepth (Material::additional_depth_, integrator_montecarlo.cc:923)
	int sigma_root;         // sigma_oren_shader root (program-local, -1: none)
	float diffuse[4];       // shinydiffuse diffuse colour
	float emit[4];          // shinydiffuse emit colour / light_mat colour * power
	float comp[4];          // getComponents() (no shader nodes)
	uint32_t c_flags[4];
	uint32_t c_index[4];
	// shader-node program (material_node.cc:60-100: the nodes the roots depend on, in evaluation
	// order): nodes [node0, node0 + n_nodes) of DevScene::shader_nodes; roots are program-local
	// indices (-1: none).  emit_strength multiplies the diffuse shader's colour in emit()
	// (material_shiny_diffuse.cc:242-247).
	int node0, n_nodes, diffuse_root, drefl_root;
	float emit_strength;
	float tfilter;          // transmit_filter
	float ior_sq;           // IOR^2 (Fresnel)
	float tbias;            // transparentbias_factor (specularRefract, integrator_montecarlo.cc:890-898)
	uint32_t sd_flags;      // SD_*
	float on_a, on_b;       // Oren-Nayar A / B (initOrenNayar, material_shiny_diffuse.cc:146-152), SD_OREN_NAYAR
	uint32_t pad4;
	float mirror_col[4];    // shinydiffuse mirror_color; mirror material: colour * reflect
};

// ---- textures and shader nodes (src/texture/texture_image.cc, src/shader/shader_node_*.cc) ----
enum : int { INTERP_NONE = 0, INTERP_BILINEAR = 1, INTERP_BICUBIC = 2 };
// ImageTexture::ClipMode (include/texture/texture_image.h:62), same numbering
enum : int { CLIP_EXTEND = 0, CLIP_CLIP = 1, CLIP_CLIPCUBE = 2, CLIP_REPEAT = 3, CLIP_CHECKER = 4 };
enum : uint32_t
{
	TEXF_MIRROR_X = 1u, TEXF_MIRROR_Y = 2u, TEXF_ROT90 = 4u, TEXF_CROPX = 8u, TEXF_CROPY = 16u,
	TEXF_CHECK_ODD = 32u, TEXF_CHECK_EVEN = 64u, TEXF_ADJ = 128u, TEXF_CLAMP = 256u
};
// ColorSpace (include/color/color.h:36)
enum : int { CS_RAW_MANUAL_GAMMA = 1, CS_LINEAR_RGB = 2, CS_SRGB = 3, CS_XYZ_D65 = 4 };

// An image texture: its texels are the image buffer's getColor() values (already quantised the
// way the reference's optimized/compressed buffers store them), row-major in DevScene::texels.
struct DevTexture
{
	uint32_t texel0;
	int w, h, interp;
	int clip, xrep, yrep;
	uint32_t flags;
	float cropminx, cropmaxx, cropminy, cropmaxy;
	float checker_dist, intensity, contrast, saturation;
	float hue, fr, fg, fb;      // hue already / 60 (texture.cc:139)
	int raw_cs;                 // original colour space of the image file (getRawColor)
	float raw_gamma;
	int pad0, pad1;
};

enum : int { NODE_VALUE = 0, NODE_MIX = 1, NODE_LAYER = 2, NODE_TEXMAP = 3 };
// MixNode variants (shader_node_basic.cc:656-672) and LayerNode blend modes (shader_node_layer.cc:320-330)
enum : int { BLEND_MIX = 0, BLEND_ADD, BLEND_MULT, BLEND_SUB, BLEND_SCREEN, BLEND_DIV, BLEND_DIFF, BLEND_DARK, BLEND_LIGHT, BLEND_OVERLAY };
// LayerNode flags (shader_node_layer.h) + the booleans of the node
enum : uint32_t
{
	LAYER_RGB_TO_INT = 1u, LAYER_STENCIL = 2u, LAYER_NEGATIVE = 4u, LAYER_DO_COLOR = 8u, LAYER_DO_SCALAR = 16u,
	LAYER_COLOR_INPUT = 32u, LAYER_USE_ALPHA = 64u
};
// TextureMapperNode::Coords / Projection (shader_node_basic.h)
enum : int { TC_UV = 0, TC_GLOBAL, TC_ORCO, TC_TRANSFORMED, TC_NORMAL, TC_WINDOW };
enum : int { PROJ_PLAIN = 0, PROJ_CUBE, PROJ_TUBE, PROJ_SPHERE };

struct DevNode
{
	int type, mode;            // NODE_*, BLEND_* (mix / layer)
	int in[3];                 // program-local inputs (-1: constant).  mix: input1, input2, factor;
	                           // layer: input, upper_layer
	uint32_t flags;            // layer: LAYER_*; mapper: bit 0 = do_scalar
	int tex;                   // mapper: texture index
	int coords, proj, map_x, map_y, map_z;
	int pad0, pad1, pad2, pad3;
	float c0[4], c1[4];        // value: colour+alpha; mix: color1, color2; layer: def_col, upper_col
	float f[4];                // value: scalar; mix: cfactor, val1, val2; layer: colfac, valfac, def_val, upper_val
	float scale[4], offset[4]; // mapper (offset already doubled, shader_node_basic.cc:372)
	float mtx[16];             // mapper "transform" (row-major Matrix4)
};

// Per-primitive surface attributes (primitive_triangle.cc:97-176), kAttrF4 float4 per primitive:
//   [0] v0 (.w = flags ATTR_*)  [1] e1  [2] e2          Moller-Trumbore operands (barycentrics)
//   [3..5] orco vertices        [6] (u0, v0, u1, v1)  [7] (u2, v2, -, -)
//   [8..10] vertex normals (smooth / exported normals; face normal where a vertex has none)
constexpr int kAttrF4 = 11;
constexpr int kMaxNodes = 16;   // shader nodes per material program
enum : uint32_t { ATTR_ORCO = 1u, ATTR_UV = 2u, ATTR_SMOOTH = 4u };

struct DevLight
{
	uint32_t type, cast_shadows;
	int32_t samples;        // area: ceilf(samples * light sample multiplier)
	float inv_samples;
	float color[4];
	float pos[4];           // point position / area corner
	float to_x[4], to_y[4], fnormal[4];
	float c2[4], c3[4], c4[4];
	float du[4], dv[4];     // area: emission frame (light_area.cc:47-51), photon emission
	float area;
	uint32_t nee_base;      // first NEE entry of this light in the estimateAllDirectLight layout
	uint32_t nee_count;     // point: 1, area: 2 * samples
	uint32_t shoot;         // bit 0: diffuse photons, bit 1: caustic photons
	// meshlight / objectlight (light_object_light.cc): triangles [mesh0, mesh0 + mesh_n) of
	// DevScene::mesh_tris / mesh_cdf (the mesh's faces in creation order), double-sided emission
	uint32_t mesh0, mesh_n, double_sided;
	// photon_only (Light::photonOnly): the light shoots photons but the integrators do not see it
	// (render_view.cc:83-91) — it sits after the DevScene::n_lights visible lights and has no NEE entries
	uint32_t photon_only;
	// meshlight: its faces' own BVH2 (the reference's per-light kd-tree, light_object_light.cc:62-70) for the
	// material-sampled rays — nodes [bvh_node0, ...) of DevScene::mesh_nodes, triangle records from
	// bvh_tri0 of DevScene::mesh_btris (leaf order, the face index in e1.w); bvh_depth 0: test every face
	uint32_t bvh_node0, bvh_tri0, bvh_depth, pad1;
};

struct DevCamera
{
	float pos[4], vright[4], vup[4], vto[4], cam_z[4], near_p[4], far_p[4];
	int resx, resy;
	int ray_tt;                    // the camera rays need their own (tmin, tmax): a near plane off the camera
	                               // position or a far plane in front of it (else every ray has (0, unbounded))
	int pad1;
	// depth of field (camera_perspective.cc:28-52, 71-146): aperture * camera axes, bokeh polygon
	float dof_rt[4], dof_up[4];
	float aperture, dof_distance;
	int bokeh_type, bokeh_bias;    // BokehType (0 disk1, 1 disk2, 3..6 polygon, 7 ring), BkhBiasType
	float ls[16];                  // polygon vertices (cos, sin) pairs
};

// A band of pixel rows rendered as a run of tiles (imagesplitter.cc:30-49 linear order):
// tiles of width `tile` left to right, pixels row-major inside each tile.
struct DevJob
{
	int y0, y1;             // pixel rows [y0, y1)
	uint64_t sample_base;   // first sample id of the job in the frame-local enumeration
};

struct DevScene
{
	const float4 *nodes;
	const float4 *tris;
	const float4 *prim_ng;
	const DevMaterial *mats;
	const DevLight *lights;
	const uint8_t *faure;          // concatenated Faure digit permutations, dims 0..49
	const uint4 *faure_dim;        // per dimension: (base, table offset, division magic m, shift)
	const double *faure_inv;       // inv_prims (halton.cc:413)
	int n_nodes, n_tris, n_mats, n_lights;
	int node_f4;                   // float4 per BVH node: 4 (BVH2) or 8 (BVH4)
	int scene_in_lds;              // nodes+tris copied to LDS by each trace workgroup
	int brute;                     // YAFARAY_AMD_TRACE=brute: k_trace_brute tests every triangle of a tiny scene
	int ray_sort;                  // k_trace orders each wave's window of queue entries by ray kind + direction (LDS counting sort)
	int lds_nodes, lds_tris;
	int lds_top;                   // BVH4 in global memory: k_trace stages nodes [0, lds_top) in LDS (the top treelet)
	const float4 *nodes8;          // quantised BVH8 of a device-built tree (8 float4 per node) for k_trace's refill loop, or null
	const float4 *tris8;           // its triangle records (leaves in node order)
	int lds_top8;                  // its nodes k_trace stages in LDS
	// meshlight triangles (DevLight::mesh0 / mesh_n): kMeshTriF4 float4 each — the exact-test record
	// (v0 + eps, e1 + index, e2), the vertices v0, v1, v2 and the geometric normal — and the area
	// distribution's normalised cdf (sample_pdf1d.h)
	const float4 *mesh_tris;
	const float *mesh_cdf;
	const float4 *mesh_nodes;      // meshlight BVH2 nodes (4 float4 each, DevLight::bvh_node0)
	const float4 *mesh_btris;      // meshlight BVH2 triangle records (3 float4 each, leaf order)

	DevCamera cam;

	int integrator, width, height, spp;
	int tile, bounces, path_samples, rr_min_bounces;
	int caustic_path, has_bg, bg_transp, nee_k;
	uint32_t n_seg, cap_a, cap_s;   // queue segments; capacities: active list / NEE requests, shadow rays (= nee_k * cap_a)
	float bg[4];
	int shadow_bias_auto, ray_min_dist_auto;
	float shadow_bias, ray_min_dist;
	uint32_t base_offset, rr_seed;
	float clamp_samples;
	// adaptive anti-aliasing (integrator_tiled.cc:172-231): passes > 1 switch the sub-pixel
	// positions to riVdC / riS of the global sample index; pass_offset = samples of earlier passes;
	// plist = the pixels this pass resamples, in the reference's visiting order (null: every pixel,
	// enumerated by the jobs)
	int aa_multipass;
	uint32_t pass_offset;
	const uint32_t *plist;
	int nee_all_count;             // entries of the estimateAllDirectLight layout
	int faure_bytes;               // size of the permutation table (padded to 16 B)
	int small_tables;              // materials + per-primitive normals fit k_shade / k_nee LDS

	// photon mapping (integrator_photon_mapping.cc): diffuse photon map + point kd-tree
	const float4 *ph_pos;          // (position, colour.r) per photon, kd-tree order of the map
	const float4 *ph_dir;          // (direction, colour.g)
	const float *ph_colb;          // colour.b
	const uint4 *pk_nodes;         // point kd-tree (pkdtree.h:41-64): .w flags (axis / leaf, right child or photon << 2),
	                               // interior .x split position, leaf .xyz the photon's position
	uint2 *pk_stack;               // k_gather lookup stacks: pm_stack levels x gather lanes (HBM)
	int n_photons, pm_paths, pm_search, pm_stack;
	float pm_radius2;              // "diffuseRadius", used as the squared gather radius (:954)
	// light selection for photon emission (sample_pdf1d.h: Pdf1D over the total energy of the
	// lights that shoot diffuse photons, render_view.cc:103-110)
	const int *ph_lights;          // photon light k -> index into lights
	const float *light_cdf;
	const float *light_func;
	float light_inv_integral;
	int n_ph_lights;
	// caustic photon map (MonteCarloIntegrator::createCausticMap / causticWorker,
	// integrator_montecarlo.cc:410-640): same layout as the diffuse map; caus_map = the integrator
	// adds causticPhotons() at diffuse hits (PhotonIntegrator / DirectLight "caustics",
	// PathIntegrator caustic_type photon | both) and the map holds photons
	const float4 *cph_pos;
	const float4 *cph_dir;
	const float *cph_colb;
	const uint4 *cpk_nodes;
	int caus_map, c_photons, c_paths, c_search;
	float c_radius2;               // caustic_radius^2 (float product, :629)
	int gather_on;                 // k_shade queues k_gather requests (diffuse and / or caustic estimates)
	// PhotonIntegrator final gathering (integrator_photon_mapping.cc:39-88, 183-193, 540-591, 640-763):
	// radiance points picked while shooting the diffuse map, thinned and pre-gathered into the
	// radiance map (same layout as the photon maps, .xyz of rph_dir = the point's normal); k_fg
	// traces the gather paths of every diffuse camera hit and looks the radiance map up
	int fg_on, fg_samples, fg_bounces;
	int fg_pass_samples;           // gather paths of this pass: ceilf(fg_samples * AA indirect multiplier) (:648); 0: fg_samples
	float fg_min_pathlen;          // gather_dist_
	float fg_lookup_rad;           // lookup_rad_ = 4 diffuseRadius^2 (:245)
	float fg_i_scale;              // preGatherWorker i_scale = 1 / (nPaths pi), long double on the host (:53)
	const float4 *rph_pos;
	const float4 *rph_dir;
	const float *rph_colb;
	const uint4 *rpk_nodes;
	int n_rphotons;
	int rpk_lds;                   // k_fg: levels of the radiance-map nearest search held in an LDS column (tree depth + 1;
	                               // 0: the private-array stack)
	RadGrid rgrid;                 // the radiance map's uniform grid (k_fg_first / k_fg_long; start null: the kd search)

	// surface attributes and shader nodes: only when some material has nodes or some mesh has
	// orco / uv / smooth normals (has_attr); k_surface then fills DevQueues::sattr per hit
	int has_attr, n_textures;
	const float4 *prim_attr;       // kAttrF4 per primitive
	const float4 *texels;
	const DevTexture *textures;
	const DevNode *shader_nodes;

	// EXT kernels: materials beyond diffuse shinydiffuse / light_mat, shader nodes, or the specular
	// recursion tree (MonteCarloIntegrator::recursiveRaytrace, integrator_montecarlo.cc:664-968):
	// every integrate() call is a node; nodes of ray level L + 1 are spawned by the level-L pass
	// and traced by the next pass; k_combine folds the tree bottom-up in the reference's order.
	int ext, tree, raydepth, cur_level;
	int max_add_depth;             // largest material additionaldepth (sizes the recursion tree)
	int bg_transp_refract;
	// transparent shadows (MonteCarloIntegrator tr_shad_ / s_depth_, accelerator_kdtree.cc:916-1061):
	// shadow rays keep tmin in sh_o.w, k_trace<TS> lists the transparent surfaces each one crosses
	// (DevQueues::ts_hit, s_depth per ray), k_tshadow multiplies their filter colours into the
	// NEE contributions whose factors k_nee kept in DevPaths::ts
	int tr_shad, s_depth;
	// DirectLight ambient occlusion (TiledIntegrator::sampleAmbientOcclusion, integrator_tiled.cc:644-691):
	// ao_samples NEE entries per diffuse camera vertex after the lights' (nee_all_count) entries
	int do_ao, ao_samples;
	float ao_dist;
	float ao_col[3];
	struct DevStats *stats;        // per-workgroup counters (null: not counted)
	int trace_stats;               // k_trace counts node visits / triangle tests (0: rays only)
	int crop_x0, crop_y0;          // cropped film (xstart / ystart): film pixel (x, y) = camera pixel (x + crop_x0, y + crop_y0)
	int show_map;                  // PhotonIntegrator show_map: camera hits show the nearest photon (k_gather, G_SHOWMAP)
	uint32_t node_base;            // node id of spawn slot 0 (= level-0 capacity of the chunk)
	uint32_t spawn_cap;
	float4 *node_own;              // per node: colour before recursiveRaytrace's result, alpha
	int2 *node_child;              // per node: reflect / refract child node ids (-1: none)
	float4 *node_w;                // per node: the colour the parent multiplies this node's total by
	float4 *spawn_o, *spawn_d;     // spawned rays (origin, tmin) (direction, tmax)
	uint4 *spawn_pr;               // (pixel offset, sample index, MWC x, MWC c)
	uint32_t *spawn_count;         // [0] spawned records, [1] overflow flag
	// estimateOneDirectLight's light pick in the reference's one-thread order (integrator_montecarlo.cc:70-78,
	// the counter integrator_tiled.cc:48 / :169-171): lpc holds one counter per camera sample of the pass,
	// pixel-major ((y * width + x) * spp + s).  lpc_mode 1 (count run): each call adds one to its sample's
	// counter and estimates nothing; 2: the counter starts at the calls of every sample the one-thread
	// render visits before it (render.cc lpcBases: an exclusive scan in tile order) and each call takes
	// the next value; 0: pickLight
	uint32_t *lpc;
	int lpc_mode;          // 3: deferred pick (r06) — every addition to a path colour becomes a record (below), resolved after the pass
	// deferred light pick (lpc_mode 3, kernels.hip k_dfr_*): one 80-B record per active entry slot of every
	// iteration (dfr_seg_off: this iteration's first slot of every segment; a record = hit point + primitive,
	// wo + the sample's previous record, throughput or term + kind, emission + the call's ordinal, the pixel's
	// sampling offset + sample index + counter index + light), dfr_last: per camera sample of the pass its last
	// record (+1, bit 31: diffuse first hit; all ones: not finalized)
	uint32_t *dfr_kind;    // per slot: 0 none, 1 light estimate, 2 known term | has emission << 2 | the call's ordinal << 3 (k_dfr_part replaces it with the picked light)
	float4 *dfr_pp;        // hit point, primitive (kind 1)
	float4 *dfr_wo;        // wo, the picked light (k_dfr_nee)
	float4 *dfr_a;         // the vertex throughput (kind 1) or the term (kind 2), the camera sample's counter index
	float4 *dfr_emit;      // emission added to the estimate (kind 1 with has emission)
	uint2 *dfr_pix;        // the pixel's sampling offset, sample index (kind 1)
	uint32_t *dfr_last;
	const uint32_t *dfr_seg_off;
	uint32_t dfr_cap;
	int nee_pm16;          // 1: NEE requests keep the 16-B pixel / mode word (YAFARAY_AMD_NEE_PM16=1; else 8 B where it fits)
	int w_live;            // 1: the integrator's sample weight w must persist across vertices (DevPaths::thr.w); 0: thr is a 12-B record
	int no_lean;           // 1: the general k_shade / k_nee instantiations even where a lean one applies (YAFARAY_AMD_SHADE_LEAN=0: tests, A/B)
	int has_mesh_light;    // some light is a meshlight (k_nee's lean instantiation has no meshlight code)
	int fg_probe;          // diagnostic (YAFARAY_AMD_FG_PROBE, wrong images): 1 = k_fg_first skips its radiance-map lookups
};

struct DevFilm
{
	float table[256];
	float filterw, table_scale;
	int reach_fwd, reach_back;     // footprint reach: sources in [x - reach_fwd, x + reach_back]
	int width, height, spp, tile;
	int multipass;                 // AA_passes > 1: riVdC / riS sub-pixel positions
	uint32_t sample_offset;        // base sampling offset + this pass's offset
	// tile order of the splats (ImageSplitter, imagesplitter.cc:30-107): rank of tile ty * ntx + tx
	// in the one-thread render order; null = linear (rank = tile id)
	const uint32_t *tile_rank;
	int ntx;
	// partial film: each pixel as ImageFilm::finishArea shows it when its tile finishes in a one-thread
	// render (imagefilm.cc:489-520): only sources of tiles ranked <= its own; accum / weights untouched
	int partial;
	int crop_x0, crop_y0;          // cropped film: the sample positions hash the camera pixel (x + crop_x0, y + crop_y0)
};

// Per-chunk wavefront state (structure of arrays, capacity = chunk slots).
struct DevPaths
{
	float4 *thr;           // throughput, .w = the integrator's persistent sample weight `w`
	float4 *col;           // col (first-vertex estimate), .w = stage | subpath << 8 | depth << 20 (bits)
	float4 *pcol;          // path_col, .w = flags: mat_bsd_fs (v1 flags) | bits below (bits)
	float4 *pwo;           // pwo (outgoing direction at the current path vertex): ST_FIRST entries only
	float4 *pend_thr;      // throughput at the pending vertex (after Russian roulette), 12 B per entry (kernels.hip F3)
	float4 *pend_emit;     // emission pending at that vertex
	float4 *v0p;           // first hit p .w = prim (bits)   — only used when path_samples > 1
	float4 *v0wo;          // first hit wo
	uint4 *pr;             // compact record (no specular recursion tree): (sample id, stage, MWC x, MWC c) —
	                       // the pixel, PixelSamplingData offset_ / sample_ derive from the sample id;
	                       // tree renders: (PixelSamplingData::offset_, sample_, MWC x, MWC c) with the
	                       // sample / node id in DevQueues::slot and the stage in col.w
	float4 *csmp;          // compact record: the first-vertex estimate `col` per chunk sample (indexed by
	                       // sample id), written when it changes, read where it is used (F_COLS)
	float *nee;            // [slots * nee_k] contributions as 12-B records (3 floats); an entry without a valid
	                       // sample has its occlusion byte set (k_trace writes only the bytes of emitted rays)
	float *nee_aw;         // [slots * nee_k] the AO entries' material-sample pdf (sampleAmbientOcclusion)
	uint8_t *occ;          // [slots * nee_k] shadow results
	float4 *ts;            // [3 * slots * nee_k] transparent shadows: the contribution's factors
	                       // (surf colour, a) (light colour, b) (c, c divides) — contrib = ((surf * (L * scol)) * a) * b  (* or /) c
	float4 *v0attr;        // [2 * slots] first-hit surface attributes (has_attr && path_samples > 1)
};

struct DevQueues
{
	// active list (parallel to the closest-ray queue)
	int *slot;
	// closest rays as 12-B records (3 floats per entry): origin, direction (x = NaN: no ray this
	// iteration).  The queue of a pass's first iteration (camera / spawned rays) carries each ray's
	// (tmin, tmax) in ray_tt (tmax < 0: infinite; a spawned node's additional depth in it); every later
	// iteration's rays (k_shade's bounces) have (ray_min_dist, infinite) and ray_tt == nullptr
	float *ray_o;
	float *ray_d;
	float2 *ray_tt;
	float tmin_dflt;       // tmin of the rays without ray_tt (camera rays with the default clip planes: 0;
	                       // bounce rays: ray_min_dist); tmax unbounded
	float *hit_t;
	int *hit_prim;
	// shadow rays
	float4 *sh_o;          // origin, .w = tmin of the light ray (read by transparent shadows only)
	float4 *sh_d;          // direction, .w = t_max (already tmax - 2 tmin, or inf)
	int *sh_idx;           // slot * nee_k + entry
	float2 *ts_hit;        // [s_depth * shadow rays] transparent shadows: (t, prim bits) of each transparent surface crossed
	int *ts_n;             // [shadow rays] number of entries in ts_hit (0 when occluded or clear)
	float4 *sattr;         // [2 * entries] k_surface output for the hit: (N, diffuse_refl), (diffuse colour, -)
	const uint32_t *perm;  // ray binning (r06, BVH8 refill loop): closest entry a0 + j traces the ray of entry perm[a0 + j]
	                       // (its segment's rays ordered by direction octant + origin Morton code); null: identity
};

// Next-event-estimation requests written by k_shade, consumed by k_nee in the same iteration, and
// k_gather's requests.  NEE (r04): one slot per entry k of the next active list (request of entry k
// at k, so the index is implicit): wo_k = (outgoing direction, primitive bits), x = NaN for an entry
// without a request; the hit point is the next queue's ray origin at k (the vertex's continuation
// ray starts there, a pending-only entry stores it), p_prim unused.
struct DevNeeQueue
{
	float4 *p_prim;        // gather: hit point, .w = primitive (bits)
	float4 *wo_k;          // gather: outgoing direction, .w = sample id (bits); NEE: (wo, primitive bits)
	uint4 *pix_mode;       // NEE: (PixelSamplingData offset, sample index, mode | light << 8, 0), packed to 8 B
	                       // per request while neePm8 (kernels.hip); gather: the first-vertex colour + alpha
	float4 *attr;          // [2 * requests] surface attributes of the vertex (has_attr only)
	float4 *extra;         // gather requests only: colour added after the estimates, .w = G_* mode bits
};

// k_gather request modes (DevNeeQueue::extra.w)
enum : uint32_t
{
	G_DIFFUSE = 1u,   // diffuse-map density estimate (PhotonIntegrator)
	G_CAUSTIC = 2u,   // causticPhotons()
	G_EXTRA = 4u,     // then add extra.xyz
	G_FG = 8u,        // finalGathering() (k_fg, before k_gather): extra.xy = (pixel offset, sample index) bits
	G_SHOWMAP = 16u,  // show_map: the nearest photon's colour (radiance map with final gathering, else the diffuse map)
};

// Queues are segmented: segment b (capacity cap_a entries / cap_s shadow rays) belongs to workgroup
// b of k_shade and k_nee, whose grids are the n_seg segments.  A workgroup consumes its segment and
// appends its outputs to the same segment of the next queue through an LDS counter (one LDS atomic
// per wave, no global atomics, no workgroup barriers), then publishes the count with a plain store.
// An entry yields at most one next entry (and at most nee_k shadow rays), so a segment never
// outgrows the camera's share.  k_trace runs n_seg * m workgroups, m per segment.
// Photon paths in flight while the photon map is shot (render.cc / k_photon_*).
struct PhotonState
{
	float4 *ray_o;       // origin, tmin
	float4 *ray_d;       // direction
	float4 *pcol;        // photon colour, .w = flags (bit 0 caustic, bit 1 direct)
	uint32_t *alive[2];  // photon ids of the current / next bounce, segmented: segment s (= k_photon_bounce
	                     // workgroup s) holds seg_cap entries at s * seg_cap; kDeadPhoton marks a hole.  Bounce 0:
	                     // local id i at position i (segment s = the contiguous ids [s seg_cap, (s + 1) seg_cap)),
	                     // so a wave's lanes read consecutive path records
	uint32_t *n_alive;   // [(bounces + 2) * n_segs] entries per segment and bounce (bounce 0: derived from the id
	                     // layout); the host sums them for the paths traced (the bounce kernel's work items)
	uint32_t seg_cap, n_segs;
	// deposit slots, bounce-major: slot (i, b) = b * n_local + i, so a bounce's lanes (consecutive local ids)
	// store consecutive records; the compaction (k_photon_count / k_photon_scatter) emits them in photon-id
	// order, bounces in order — the reference's one-thread order
	uint32_t n_local, n_slot_rows;   // local ids, bounces + 1
	float4 *dep_a;       // deposit slots: (position, colour.r)
	float4 *dep_b;       // (direction, colour.g)
	float *dep_c;        // colour.b
	uint8_t *dep_flag;   // 1 = a photon was stored in this slot
	// final gathering (diffuse map only): radiance point per deposit slot (:184-193)
	float4 *rad_a;       // (position, refl.r)
	float4 *rad_b;       // (normal facing the photon, refl.g)
	float4 *rad_c;       // (refl.b, transm.rgb)
	uint8_t *rad_flag;   // 1 = this deposit is a radiance point (null: final gathering off)
};

// the lights one photon map is shot from (render_view.cc:103-110: lights emitting diffuse / caustic
// photons) with their Pdf1D over the total energies (sample_pdf1d.h:52-66), and the map kind
struct PhotonSet
{
	const int *lights;   // k -> index into DevScene::lights
	const float *cdf;
	const float *func;
	float inv_integral;
	int n_lights;
	int caustic;         // 0: diffuseWorker rules, 1: causticWorker rules
};

// ImageFilm::nextPass inputs (imagefilm.cc:259-420; aa_noise_params.h:27-46)
struct DevAaParams
{
	int detect_color_noise;        // colorDifference over r, g, b, a as well as brightness
	int dark_type;                 // 0 none, 1 linear, 2 curve
	float dark_factor;             // AA_dark_threshold_factor
	int variance_edge;             // AA_variance_edge_size
	int variance_pixels;           // AA_variance_pixels (0: off)
};

struct DevCounters
{
	uint32_t *n_active;   // [n_seg] active-list entries (closest rays + paths) per segment
	uint32_t *n_shadow;   // [n_seg] shadow rays per segment
	uint32_t *n_nee;      // [n_seg] NEE requests per segment
	uint32_t *n_gather;   // [n_seg] photon-map estimate requests per segment (k_gather)
};

// Per-workgroup counters (record b belongs to workgroup b of every launch on the stream: plain
// read-modify-writes, no atomics; summed on the host after the render)
struct DevStats
{
	unsigned long long closest_rays, shadow_rays, node_visits, tri_tests;
	unsigned long long shade_entries;    // active-list entries k_shade processed
	unsigned long long nee_requests;     // NEE requests k_nee served
	unsigned long long gather_queries;   // photon density estimates k_gather computed
	unsigned long long gather_visits;    // point kd-tree nodes k_gather fetched
	unsigned long long gather_photons;   // photons the density estimates read (heap entries summed)
	unsigned long long gather_accepts;   // two-pass gather: photons the walk accepted (log entries)
	unsigned long long gather_overflows; // two-pass gather: requests whose log overflowed (walked again)
	unsigned long long fg_paths;         // final gathering: gather paths k_fg traced
	unsigned long long fg_lookups;       // final gathering: radiance-map nearest searches
	unsigned long long fg_nearest_visits;// final gathering: radiance-map kd nodes those searches fetched
	unsigned long long pre_visits;       // k_pregather: diffuse-map kd nodes fetched
	unsigned long long pre_photons;      // k_pregather: photons summed into the radiance estimates
};

// the two-pass diffuse gather's accepted-photon log for one batch of the gather queue (kernels.hip
// GatherLog): cap entries of 8 bytes per request, seg_cap queue positions per segment from j0
struct GatherLogDesc
{
	void *e;
	uint32_t *n;
	uint32_t cap, seg_cap, j0;
	uint32_t split;   // k_gather<REPLAY>: the 6-byte split heap where eligible (YAFARAY_AMD_GATHER_HEAP=packed: 0)
	uint32_t exact;   // k_gather_walk: the exact-radius walk (k <= 64; YAFARAY_AMD_GATHER_WALK=exact), else the bounded walk
	uint32_t *spill;  // k_gather_walk: far-child stack levels beyond the LDS ones (-DYAF_WALK_LDS_LEVELS), per walk thread
};

// one batch of final gathering with one lane per gather path (kernels.hip k_fg_first / k_fg_long / k_fg_sum)
struct FgBatch
{
	uint32_t j0, seg_cap;   // request positions of this batch in every segment
	int n_sampl;            // gather paths per request of this pass
	int n_terms;            // terms a bouncing path can add: fg_bounces + 1
	float4 *terms;          // [seg][pos - j0][path]: (term, tag): tag 0 no term, 1 one term, 2 + i: bouncing path i of the segment
	float4 *longs;          // [seg][i][3]: (origin, t) (direction, prim) (throughput, path id in the segment's batch)
	float4 *long_terms;     // [seg][i][n_terms]: (term, 1) or (0, 0)
	uint32_t *long_count;   // [seg]
	uint32_t long_cap;      // bouncing paths per segment (= seg_cap * n_sampl: every path may bounce)
};

} // namespace yafamd
