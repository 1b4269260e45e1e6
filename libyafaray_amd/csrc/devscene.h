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

enum : uint32_t
{
	B_NONE = 0, B_SPECULAR = 1u << 0, B_GLOSSY = 1u << 1, B_DIFFUSE = 1u << 2, B_DISPERSIVE = 1u << 3,
	B_REFLECT = 1u << 4, B_TRANSMIT = 1u << 5, B_FILTER = 1u << 6, B_EMIT = 1u << 7, B_VOLUMETRIC = 1u << 8,
	B_ALL = B_SPECULAR | B_GLOSSY | B_DIFFUSE | B_DISPERSIVE | B_REFLECT | B_TRANSMIT | B_FILTER
};

enum : uint32_t { MAT_SHINYDIFFUSE = 0, MAT_LIGHT = 1 };
enum : uint32_t { LIGHT_POINT = 0, LIGHT_AREA = 1 };
enum : int { INT_DIRECT = 0, INT_PATH = 1, INT_PHOTON = 2 };

struct DevMaterial
{
	uint32_t type, bsdf_flags, n_bsdf, double_sided;
	uint32_t receive_shadows, flat, pad0, pad1;
	float diffuse[4];       // shinydiffuse diffuse colour
	float emit[4];          // shinydiffuse emit colour / light_mat colour * power
	float comp[4];          // getComponents() (no shader nodes)
	uint32_t c_flags[4];
	uint32_t c_index[4];
};

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
};

struct DevCamera
{
	float pos[4], vright[4], vup[4], vto[4], cam_z[4], near_p[4], far_p[4];
	int resx, resy, pad0, pad1;
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
	int lds_nodes, lds_tris;

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
	const uint2 *pk_nodes;         // point kd-tree (pkdtree.h:41-64): (split bits | photon, flags)
	int n_photons, pm_paths, pm_search, pm_stack;
	float pm_radius2;              // "diffuseRadius", used as the squared gather radius (:954)
	// light selection for photon emission (sample_pdf1d.h: Pdf1D over the total energy of the
	// lights that shoot diffuse photons, render_view.cc:103-110)
	const int *ph_lights;          // photon light k -> index into lights
	const float *light_cdf;
	const float *light_func;
	float light_inv_integral;
	int n_ph_lights;
};

struct DevFilm
{
	float table[256];
	float filterw, table_scale;
	int reach_fwd, reach_back;     // footprint reach: sources in [x - reach_fwd, x + reach_back]
	int width, height, spp, tile;
	int multipass;                 // AA_passes > 1: riVdC / riS sub-pixel positions
	uint32_t sample_offset;        // base sampling offset + this pass's offset
};

// Per-chunk wavefront state (structure of arrays, capacity = chunk slots).
struct DevPaths
{
	float4 *thr;           // throughput, .w = the integrator's persistent sample weight `w`
	float4 *col;           // col (first-vertex estimate), .w = stage | subpath << 8 | depth << 20 (bits)
	float4 *pcol;          // path_col, .w = flags: mat_bsd_fs (v1 flags) | bits below (bits)
	float4 *pwo;           // pwo (outgoing direction at the current path vertex): ST_FIRST entries only
	float4 *pend_thr;      // throughput at the pending vertex (after Russian roulette)
	float4 *pend_emit;     // emission pending at that vertex
	float4 *v0p;           // first hit p .w = prim (bits)   — only used when path_samples > 1
	float4 *v0wo;          // first hit wo
	uint4 *pr;             // (PixelSamplingData::offset_, PixelSamplingData::sample_, MWC x, MWC c)
	float4 *nee;           // [slots * nee_k] contributions .w = valid
	uint8_t *occ;          // [slots * nee_k] shadow results
};

struct DevQueues
{
	// active list (parallel to the closest-ray queue)
	int *slot;
	float4 *ray_o;         // origin, .w = tmin
	float4 *ray_d;         // direction, .w = tmax (< 0: infinite); NaN: no ray this iteration
	float *hit_t;
	int *hit_prim;
	// shadow rays
	float4 *sh_o;          // origin, .w unused
	float4 *sh_d;          // direction, .w = t_max (already tmax - 2 tmin, or inf)
	int *sh_idx;           // slot * nee_k + entry
};

// Next-event-estimation requests written by k_shade, consumed by k_nee in the same iteration.
struct DevNeeQueue
{
	float4 *p_prim;        // hit point, .w = primitive (bits)
	float4 *wo_k;          // outgoing direction, .w = index k of the path in the next active list (bits)
	uint4 *pix_mode;       // (PixelSamplingData offset, sample index, mode | light << 8, 0)
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
	uint32_t *alive[2];  // photon ids of the current / next bounce
	uint32_t *n_alive;   // [2]
	float4 *dep_a;       // deposit slots: (position, colour.r)
	float4 *dep_b;       // (direction, colour.g)
	float *dep_c;        // colour.b
	uint8_t *dep_flag;   // 1 = a photon was stored in this slot
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
};

struct DevStats
{
	unsigned long long closest_rays, shadow_rays, node_visits, tri_tests;
};

} // namespace yafamd
