// GPU driver (see render.h).  Plain C++ against the HIP runtime API; kernels are launched
// through the extern "C" wrappers at the end of kernels.hip.
#include "render.h"
#include "devmath.h"
#include "photonfile.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <future>
#include <mutex>
#include <sstream>
#include <unordered_map>

using namespace yafamd;

extern "C" {
hipError_t yafamd_launch_camera(const DevScene *S, const DevPaths *P, const DevQueues *Q, const DevCounters *cnt,
                                const DevJob *jobs, int n_jobs, uint64_t chunk_base, int n, hipStream_t st);
hipError_t yafamd_launch_surface(const DevScene *S, const DevQueues *Q, const DevCounters *cnt, hipStream_t st);
hipError_t yafamd_launch_tshadow(const DevScene *S, const DevQueues *Q, const DevCounters *cnt, const DevPaths *P, hipStream_t st);
hipError_t yafamd_launch_spawn(const DevScene *S, const DevPaths *P, const DevQueues *Q, const DevCounters *cnt, uint32_t s0, int n,
                               hipStream_t st);
hipError_t yafamd_launch_combine(const DevScene *S, uint32_t lo, uint32_t hi, int final_level, float4 *samples, const DevJob *jobs,
                                 int n_jobs, uint64_t chunk_base, hipStream_t st);
hipError_t yafamd_launch_trace(const DevScene *S, const DevQueues *Q, const DevCounters *cnt, const DevPaths *P,
                               DevStats *stats, int stack_depth, int *spill, int grid, hipStream_t st);
int yafamd_trace_block();
int yafamd_shade_fused();
int yafamd_walk_lds_levels(int pm_stack);
int yafamd_walk_threads(const DevScene *S);
int yafamd_shade_fused_for(const DevScene *S);
int yafamd_experiments();
int yafamd_trace_blocks_per_cu(int lds_scene, int wide, size_t dyn_lds);
int yafamd_shade_blocks_per_cu();
hipError_t yafamd_launch_shade(const DevScene *S, const DevPaths *Pc, const DevPaths *Pn, const DevQueues *Q,
                               const DevQueues *Qn, const DevNeeQueue *N, const DevNeeQueue *G, const DevCounters *cnt,
                               const DevCounters *cnt_next, float4 *samples, const DevJob *jobs, int n_jobs, uint64_t chunk_base,
                               hipStream_t st);
int yafamd_path_eligible(const DevScene *S, int stack_depth, int spill);
int yafamd_path_blocks_per_cu(const DevScene *S, int stack_depth);
hipError_t yafamd_launch_path(const DevScene *S, float4 *samples, const DevJob *jobs, int n_jobs, uint64_t chunk_base, uint32_t n,
                              uint32_t *next, int stack_depth, int grid, hipStream_t st);
hipError_t yafamd_launch_nee(const DevScene *S, const DevNeeQueue *N, const DevPaths *Pn, const DevQueues *Qn,
                             const DevCounters *cnt_next, int stack_depth, hipStream_t st);
int yafamd_nee_blocks_per_cu();
hipError_t yafamd_photon_emit(const DevScene *S, const PhotonState *P, const PhotonSet *L, uint32_t n_photons, uint32_t h0, uint32_t n_local,
                              int max_bounces, hipStream_t st);
hipError_t yafamd_photon_bounce(const DevScene *S, const PhotonState *P, const PhotonSet *L, uint32_t n_photons, uint32_t h0,
                                uint32_t n_local, int max_bounces, int bounce, int cur, int stack_depth, int *spill, int grid, hipStream_t st);
hipError_t yafamd_photon_compact(const PhotonState *P, uint32_t *scratch_counts, uint32_t *total_dev, float4 *pos, float4 *dir, float *colb,
                                 hipStream_t st);
hipError_t yafamd_launch_gather(const DevScene *S, const DevNeeQueue *G, const DevCounters *cnt_next, float4 *samples,
                                const DevJob *jobs, int n_jobs, uint64_t chunk_base, const GatherLogDesc *log, hipStream_t st);
hipError_t yafamd_launch_gather_walk(const DevScene *S, const DevNeeQueue *G, const DevCounters *cnt_next, const GatherLogDesc *log,
                                     hipStream_t st);
int yafamd_gather_walk_k();
size_t yafamd_gather_lds_bytes(const DevScene *S);
hipError_t yafamd_rad_compact(const PhotonState *P, uint32_t *scratch_counts, uint32_t *total_dev, float4 *a, float4 *b, float4 *c, hipStream_t st);
hipError_t yafamd_rad_refl(const DevScene *S, float4 *a, float4 *b, float4 *c, const uint32_t *kept, uint32_t n, hipStream_t st);
hipError_t yafamd_pregather(const DevScene *S, const float4 *a, const float4 *b, const float4 *c, const uint32_t *kept, uint32_t n,
                            float4 *out_pos, float4 *out_dir, float *out_colb, DevStats *stats, hipStream_t st);
int yafamd_fg_paths_eligible(const DevScene *S);
hipError_t yafamd_launch_fg_paths(const DevScene *S, const DevNeeQueue *G, const DevCounters *cnt_next, int stack_depth, int *spill, int grid,
                                  const FgBatch *B, hipStream_t st);
hipError_t yafamd_thin_rad_points(const float4 *pos, const float4 *nrm, uint32_t n, float maxrad, uint32_t *kept_out, uint32_t *n_kept,
                                  int *rounds_out, hipStream_t st, void **scratch);
void yafamd_thin_scratch_free(void *scratch);
hipError_t yafamd_rad_grid(const float4 *pos, const float4 *dir, uint32_t n, float lookup_rad, RadGrid *out, hipStream_t st, void **scratch);
void yafamd_rad_grid_free(void *scratch);
int yafamd_dfr_eligible(const DevScene *S);
hipError_t yafamd_dfr_segoff(const DevCounters *cnt, uint32_t n_seg, uint32_t *seg_off, uint32_t *dfr_total, uint32_t cap, uint32_t *overflow,
                             uint32_t *it_start, hipStream_t st);
hipError_t yafamd_dfr_accum(const DevScene *S, const DevPaths *P, uint32_t r0, uint32_t r1, uint32_t batch0, float4 *pcol, hipStream_t st);
hipError_t yafamd_dfr_nee(const DevScene *S, const DevPaths *P, const DevQueues *Q, const DevCounters *cnt, uint32_t r0, uint32_t total, uint32_t *idx,
                         uint32_t *n_rec, hipStream_t st);
hipError_t yafamd_dfr_fold(const DevScene *S, float4 *samples, uint32_t n_ctr, const float4 *pcol, hipStream_t st);
hipError_t yafamd_ray_bin(const DevQueues *Q, const DevCounters *cnt, uint32_t n_seg, uint32_t cap_a, const float *lo, const float *hi,
                          uint32_t *keys_in, uint32_t *keys_out, uint32_t *iota, uint32_t *perm, void *tmp, size_t *tmp_bytes, hipStream_t st);
hipError_t yafamd_launch_fg(const DevScene *S, const DevNeeQueue *G, const DevCounters *cnt_next, int stack_depth, int *spill, int grid, float2 *ts_scratch,
                            hipStream_t st);
size_t yafamd_gather_lanes(const DevScene *S);
hipError_t yafamd_build_bvh_gpu(const float *verts_dev, const int *tris_dev, int n, void **nodes_out, void **tris_out,
                                int *n_nodes, int *depth, int *stack_need, int *ploc_iters, YafBvh8 *w8, hipStream_t st);
hipError_t yafamd_build_pkd(const float4 *pos_dev, uint32_t n, uint4 *nodes_dev, int *depth_out, hipStream_t st, void **scratch);
hipError_t yafamd_build_pkd_kd(const float4 *pos_dev, const float4 *dir_dev, const float *colb_dev, uint32_t n, uint4 *nodes_dev, float4 *kpos,
                               float4 *kdir, float *kcolb, int *depth_out, hipStream_t st, void **scratch);
void yafamd_pkd_scratch_free(void *scratch);
hipError_t yafamd_build_pkd_kd_member(const float4 *pos_dev, const float4 *dir_dev, const float *colb_dev, uint32_t n, uint4 *nodes_dev, float4 *kpos,
                                      float4 *kdir, float *kcolb, int *depth_out, hipStream_t st, void **scratch, int member, int members,
                                      int *split_level);
void yafamd_pkd_top_segments(uint32_t n, int level, uint32_t *out);
void yafamd_pkd_owned_segments(int level, int member, int members, uint32_t *s0, uint32_t *s1);
hipError_t yafamd_pkd_parent_planes(uint4 *nodes_dev, uint32_t n, hipStream_t st);
hipError_t yafamd_launch_done_flags(const DevScene *S, const DevJob *jobs, int n_jobs, uint32_t n_pix, uint32_t done_pix, uint8_t *flags,
                                    hipStream_t st);
hipError_t yafamd_lpc_seg(const uint32_t *lpc, int W, int spp, int ts, int y0, int y1, uint32_t *seg, hipStream_t st);
hipError_t yafamd_lpc_prefix(uint32_t *lpc, int W, int spp, int ts, int y0, int y1, const uint32_t *segbase, hipStream_t st);
hipError_t yafamd_launch_film(const DevFilm *F, const float4 *samples, const uint8_t *flags, float4 *accum, float4 *out,
                              float *weights, int y0, int y1, float clamp_samples, int accumulate, hipStream_t st);
hipError_t yafamd_aa_next_pass(const float4 *accum, const float *weights, int W, int H, int tile, const DevAaParams *prm,
                               float threshold, uint8_t *flags, uint32_t *plist, uint32_t *count, int ry0, int ry1, uint32_t *local_count,
                               hipStream_t st);
hipError_t yafamd_launch_trace_rays(const DevScene *S, int any, const float4 *ro, const float4 *rd, int n, float *t_out,
                                    int *prim_out, int stack_depth, hipStream_t st);
}

namespace
{

// The renderer's device made current for the duration of a call; the caller's device is restored
// (several renderers of one process, on different devices, may be driven from one thread).
struct DeviceGuard
{
	int prev = -1;
	bool set = false;
	explicit DeviceGuard(int dev)
	{
		if(dev >= 0 && hipGetDevice(&prev) == hipSuccess && prev != dev) set = hipSetDevice(dev) == hipSuccess;
	}
	~DeviceGuard()
	{
		if(set) (void)hipSetDevice(prev);
	}
};

struct Buf
{
	void *p = nullptr;
	size_t bytes = 0;
	void release()
	{
		if(p) (void)hipFree(p);
		p = nullptr;
		bytes = 0;
	}
};

// Faure digit permutations (Faure 1992 construction; the reference holds them as literal tables,
// src/sampler/halton.cc:26-401) and the 9-decimal inverse primes of halton.cc:413.
std::vector<int> faurePerm(int b)
{
	if(b <= 2) return {0, 1};
	if((b & 1) == 0)
	{
		const std::vector<int> h = faurePerm(b / 2);
		std::vector<int> out;
		for(int v : h) out.push_back(2 * v);
		for(int v : h) out.push_back(2 * v + 1);
		return out;
	}
	const std::vector<int> p = faurePerm(b - 1);
	const int c = (b - 1) / 2;
	std::vector<int> out;
	for(int i = 0; i < (int)p.size(); ++i)
	{
		if(i == c) out.push_back(c);
		out.push_back(p[i] + (p[i] >= c ? 1 : 0));
	}
	return out;
}

// Final gathering's radiance-point thinning (integrator_photon_mapping.cc:560-572): in shooting
// order, a point still in use is kept and marks every point within the squared distance `maxrad`
// (strictly less, the pkd lookup's test, pkdtree.h:263-268) whose normal faces the same side
// (EliminatePhoton, photon.h:172-180) as unused.  The reference answers the range queries with a
// point kd-tree; the kept set does not depend on how they are answered, so a uniform grid of cell
// sqrt(maxrad) serves them here.  pos / nrm: 4 floats per point (xyz used).
std::vector<uint32_t> eliminateRadPoints(const std::vector<float4> &pos, const std::vector<float4> &nrm, float maxrad)
{
	std::vector<uint32_t> kept;
	const size_t n = pos.size();
	if(!n) return kept;
	const double cell = std::sqrt((double)maxrad) * 1.0001 + 1e-30;
	// dense grid over the points' bound (counting sort, O(n)) when it has at most 2^24 cells
	double lo[3] = {pos[0].x, pos[0].y, pos[0].z}, hi[3] = {lo[0], lo[1], lo[2]};
	for(size_t i = 1; i < n; ++i)
	{
		const double v[3] = {pos[i].x, pos[i].y, pos[i].z};
		for(int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], v[a]); hi[a] = std::max(hi[a], v[a]); }
	}
	double dims[3];
	double ncell_d = 1.0;
	for(int a = 0; a < 3; ++a) { dims[a] = std::floor((hi[a] - lo[a]) / cell) + 1.0; ncell_d *= dims[a]; }
	if(ncell_d <= (double)(1 << 24))
	{
		const int64_t nx = (int64_t)dims[0], ny = (int64_t)dims[1], nz = (int64_t)dims[2];
		auto axisCell = [&](double v, int a, int64_t na) {
			int64_t c = (int64_t)std::floor((v - lo[a]) / cell);
			return c < 0 ? 0 : (c >= na ? na - 1 : c);
		};
		std::vector<uint32_t> cid(n), start((size_t)(nx * ny * nz) + 1, 0), order(n);
		for(size_t i = 0; i < n; ++i)
		{
			const int64_t cx = axisCell(pos[i].x, 0, nx), cy = axisCell(pos[i].y, 1, ny), cz = axisCell(pos[i].z, 2, nz);
			cid[i] = (uint32_t)((cz * ny + cy) * nx + cx);
			++start[cid[i] + 1];
		}
		for(size_t c = 1; c < start.size(); ++c) start[c] += start[c - 1];
		{
			std::vector<uint32_t> fill(start.begin(), start.end() - 1);
			for(uint32_t i = 0; i < n; ++i) order[fill[cid[i]]++] = i;
		}
		std::vector<uint8_t> use(n, 1);
		for(uint32_t i = 0; i < n; ++i)
		{
			if(!use[i]) continue;
			kept.push_back(i);
			const float4 q = pos[i], qn = nrm[i];
			const int64_t cx = axisCell(q.x, 0, nx), cy = axisCell(q.y, 1, ny), cz = axisCell(q.z, 2, nz);
			for(int64_t z = std::max<int64_t>(0, cz - 1); z <= std::min(nz - 1, cz + 1); ++z)
				for(int64_t y = std::max<int64_t>(0, cy - 1); y <= std::min(ny - 1, cy + 1); ++y)
					for(int64_t x = std::max<int64_t>(0, cx - 1); x <= std::min(nx - 1, cx + 1); ++x)
					{
						const size_t c = (size_t)((z * ny + y) * nx + x);
						for(uint32_t k = start[c]; k < start[c + 1]; ++k)
						{
							const uint32_t j = order[k];
							if(!use[j]) continue;
							const float vx = pos[j].x - q.x, vy = pos[j].y - q.y, vz = pos[j].z - q.z;
							const float d2 = vx * vx + vy * vy + vz * vz;
							const float nd = nrm[j].x * qn.x + nrm[j].y * qn.y + nrm[j].z * qn.z;
							if(d2 < maxrad && nd > 0.f) use[j] = 0;
						}
					}
		}
		return kept;
	}
	// sparse fallback: hashed cells
	auto cellOf = [&](const float4 &p, int dx, int dy, int dz) {
		const int64_t x = (int64_t)std::floor(p.x / cell) + dx, y = (int64_t)std::floor(p.y / cell) + dy, z = (int64_t)std::floor(p.z / cell) + dz;
		return (uint64_t)(x * 73856093) ^ (uint64_t)(y * 19349663) ^ (uint64_t)(z * 83492791);
	};
	std::unordered_map<uint64_t, std::vector<uint32_t>> grid;
	grid.reserve(n);
	for(uint32_t i = 0; i < n; ++i) grid[cellOf(pos[i], 0, 0, 0)].push_back(i);
	std::vector<uint8_t> use(n, 1);
	for(uint32_t i = 0; i < n; ++i)
	{
		if(!use[i]) continue;
		kept.push_back(i);
		const float4 q = pos[i], qn = nrm[i];
		for(int dx = -1; dx <= 1; ++dx)
			for(int dy = -1; dy <= 1; ++dy)
				for(int dz = -1; dz <= 1; ++dz)
				{
					const auto it = grid.find(cellOf(q, dx, dy, dz));
					if(it == grid.end()) continue;
					for(uint32_t j : it->second)
					{
						const float vx = pos[j].x - q.x, vy = pos[j].y - q.y, vz = pos[j].z - q.z;
						const float d2 = vx * vx + vy * vy + vz * vz;
						const float nd = nrm[j].x * qn.x + nrm[j].y * qn.y + nrm[j].z * qn.z;
						if(d2 < maxrad && nd > 0.f) use[j] = 0;
					}
				}
	}
	return kept;
}

} // namespace

struct GpuRenderer::Impl
{
	bool ok = false, init_done = false;
	hipStream_t stream = nullptr;
	Buf nodes, tris, prim_ng, mats, lights, faure, faure_dim, faure_inv;
	Buf nodes8, tris8;          // quantised BVH8 of the device-built tree and its triangles (k_trace's refill loop), or empty
	int n_nodes8 = 0, need8 = 0, lds_top8 = 0, depth8 = 0;
	int trace_grid_bvh4 = 0;   // the grid of the BVH4 k_trace when a BVH8 exists (transparent shadows)
	Buf pre_stats;             // k_pregather's counters (one DevStats)
	Buf fg_terms, fg_longs, fg_long_terms, fg_long_count;   // the per-path final gathering's batch buffers (FgBatch)
	Buf bin_keys, bin_keys2, bin_iota, bin_perm, bin_tmp;   // ray binning (YAFARAY_AMD_RAY_BIN)
	Buf dfr_kind, dfr_pp, dfr_wo, dfr_a, dfr_emit, dfr_pix;   // deferred light pick (lpc_mode 3): the records (DevScene dfr_*)
	Buf dfr_last, dfr_segoff, dfr_misc, dfr_its, dfr_pcol;     // per-sample flags, slots, iteration starts, per-sample path colours
	Buf dfr_idx, dfr_nrec;                                     // a batch's records grouped by light (k_dfr_part)
	float scene_lo[3] = {0.f, 0.f, 0.f}, scene_hi[3] = {0.f, 0.f, 0.f};
	bool pre_stats_valid = false;
	// surface attributes, textures and shader-node programs (texeval.h)
	Buf prim_attr, shader_nodes, textures, texels;
	// specular recursion tree (k_spawn / k_combine): spawned rays and per-node records
	Buf spawn_o, spawn_d, spawn_pr, node_own, node_child, node_w, spawn_count;
	bool has_attr = false, attr_alloc = false;
	int ts_alloc = 0;   // shadowDepth the transparent-shadow buffers were sized for (0: none)
	int n_textures = 0;
	// photon mapping: light selection Pdf1D, photon paths in flight, the map and its kd-tree
	Buf ph_lights, light_cdf, light_func;
	float light_inv_integral = 0.f;
	int n_ph_lights = 0;
	Buf cph_lights, clight_cdf, clight_func;   // lights shooting caustic photons
	float clight_inv_integral = 0.f;
	int n_cph_lights = 0;
	Buf cph_pos, cph_dir, cph_colb, cpk_nodes;   // caustic photon map + kd-tree
	Buf tile_rank, pfilm;                        // tile order ranks; partial film of the per-tile callbacks
	Buf mesh_tris, mesh_cdf;                     // meshlight faces and area distributions
	Buf mesh_nodes, mesh_btris;                  // meshlight BVH2s (nodes, triangle records)
	int c_photons = 0, c_paths = 0, c_depth = 0;
	Buf ph_ray_o, ph_ray_d, ph_pcol, ph_alive0, ph_alive1, ph_n_alive, dep_a, dep_b, dep_c, dep_flag, ph_scan, ph_total;
	Buf ph_pos, ph_dir, ph_colb, pk_nodes, pk_stack;
	// final gathering: radiance points per deposit slot, compacted, kept (indices), the radiance map
	Buf rad_a, rad_b, rad_c, rad_flag, radc_a, radc_b, radc_c, rad_kept, rph_pos, rph_dir, rph_colb, rpk_nodes;
	// a group member's own segment of a photon map / of the radiance points before the concatenation
	Buf seg_pos, seg_dir, seg_colb, seg_ra, seg_rb, seg_rc;
	Buf fg_ts;   // k_fg's transparent-shadow hit lists (s_depth per lane of the trace grid)
	Buf g_log, g_log_n;   // the two-pass diffuse gather's accepted-photon log (one batch of the gather queue)
	Buf walk_spill;       // k_gather_walk's stack levels beyond the LDS ones (tuning builds)
	// the maps' records in kd (leaf) order, written by the tree build (diffuse, caustic, radiance): the
	// kernels read these; the arrays above stay in photon order (saveMap, the group concatenation)
	Buf kd_pos[3], kd_dir[3], kd_colb[3];
	bool kd_on[3] = {false, false, false};
	int n_rphotons = 0;
	uint32_t n_rad_points = 0;
	int d_depth = 0, r_depth = 0;           // kd-tree depths of the diffuse / radiance maps
	uint64_t map_owner[3] = {0, 0, 0};      // integrator instance that built / loaded each map (diffuse, caustic, radiance)
	// render group (RCCL communicator over the group's GPUs) and its exchange buffers
	ncclComm_t comm = nullptr;
	Buf g_send, g_recv, g_wsend, g_wrecv, g_times, g_status;
	// scratch of the photon kd-tree build (pkd.hip) and of the radiance-point thinning (fgthin.hip)
	void *pkd_scratch = nullptr, *thin_scratch = nullptr, *rgrid_scratch = nullptr;
	std::vector<DevLight> host_lights;   // as uploaded (light sample multiplier passes rewrite the device copy)
	std::vector<DevLight> pass_lights;   // staging of the current pass's copy (alive until the stream syncs)
	int n_photons = 0, pm_paths = 0, pm_stack = 0;
	uint32_t pm_local = 0;   // diffuse photon paths this member shot (its share in a group render)
	int n_nodes = 0, n_tris = 0, n_mats = 0, n_lights = 0, depth = 0, stack_depth = 32, node_f4 = 4;
	int lds_stack = 32;    // k_trace stack levels held in LDS; levels [lds_stack, stack_depth) spill to `spill`
	Buf spill;
	bool scene_in_lds = false;
	int lds_top = 0;   // BVH4 in global memory: nodes k_trace stages in LDS (the top treelet)
	int faure_bytes = 0;
	// frame buffers
	Buf samples, film, weights, jobs;
	Buf accum, aa_flags, aa_plist;   // unnormalised film (adaptive passes add to it), nextPass flags, resampled pixels
	int film_w = 0, film_h = 0;
	// chunk buffers
	size_t slots_cap = 0;
	bool v0_alloc = false, tree_alloc = false, ao_alloc = false;
	int nee_cap = 0;
	std::vector<Buf> chunk_bufs;
	DevPaths P[2]{};       // path state, parallel to Q[q] (indexed by queue position)
	DevQueues Q[2]{};
	Buf counters, stats;
	Buf path_next;         // k_path: the chunk's sample counter
	// estimateOneDirectLight's one-thread light-pick counters (lpcBases): one per sample of the pass,
	// the row segments' sums and bases, and the count run's own statistics (not the frame's)
	Buf lpc, lpc_seg, lpc_stats;
	std::vector<hipEvent_t> ev_pool;   // [0], [1]: the render's start / end; then the profile events
	// profile mode: HIP events before / after every launch on the render stream
	bool prof_on = false;
	size_t ev_n = 2;
	struct ProfRec { int kind, e0, e1; };
	std::vector<ProfRec> prof_recs;
	hipEvent_t event(size_t i)
	{
		while(ev_pool.size() <= i)
		{
			hipEvent_t e = nullptr;
			if(hipEventCreate(&e) != hipSuccess) return nullptr;
			ev_pool.push_back(e);
		}
		return ev_pool[i];
	}
	int profBegin()
	{
		if(!prof_on) return -1;
		hipEvent_t e = event(ev_n);
		if(!e || hipEventRecord(e, stream) != hipSuccess) return -1;
		return (int)ev_n++;
	}
	void profEnd(int kind, int e0)
	{
		if(e0 < 0) return;
		hipEvent_t e = event(ev_n);
		if(!e || hipEventRecord(e, stream) != hipSuccess) return;
		prof_recs.push_back({kind, e0, (int)ev_n});
		++ev_n;
	}
	int trace_grid = 2048, shade_grid = 1024, nee_grid = 1024, n_cu = 256;
	DevNeeQueue N{};
	DevNeeQueue G{};   // k_gather requests (photon-map estimates)
	bool g_alloc = false;

	~Impl()
	{
		for(Buf *b : {&ph_lights, &light_cdf, &light_func, &ph_ray_o, &ph_ray_d, &ph_pcol, &ph_alive0, &ph_alive1, &ph_n_alive,
		              &dep_a, &dep_b, &dep_c, &dep_flag, &ph_scan, &ph_total, &ph_pos, &ph_dir, &ph_colb, &pk_nodes, &pk_stack, &cph_lights,
		              &clight_cdf, &clight_func, &cph_pos, &cph_dir, &cph_colb, &cpk_nodes, &tile_rank, &pfilm})
			b->release();
		for(Buf *b : {&prim_attr, &shader_nodes, &textures, &texels, &spawn_o, &spawn_d, &spawn_pr, &node_own, &node_child, &node_w,
		              &spawn_count})
			b->release();
		for(Buf *b : {&spill, &nodes, &tris, &prim_ng, &mats, &lights, &faure, &faure_dim, &faure_inv, &samples, &film,
		              &weights, &jobs, &counters, &stats, &accum, &aa_flags, &aa_plist})
			b->release();
		for(Buf &b : chunk_bufs) b.release();
		for(Buf *b : {&g_send, &g_recv, &g_wsend, &g_wrecv, &g_times, &g_status}) b->release();
		for(Buf *b : {&fg_ts, &g_log, &g_log_n, &walk_spill, &path_next, &lpc, &lpc_seg, &lpc_stats, &mesh_tris, &mesh_cdf, &mesh_nodes, &mesh_btris, &pre_stats, &fg_terms, &fg_longs,
		              &fg_long_terms, &fg_long_count, &bin_keys, &bin_keys2, &bin_iota, &bin_perm, &bin_tmp, &dfr_kind, &dfr_pp,
		              &dfr_wo, &dfr_a, &dfr_emit, &dfr_pix, &dfr_last, &dfr_segoff, &dfr_misc, &dfr_its, &dfr_pcol,
		              &dfr_idx, &dfr_nrec}) b->release();
		for(int m = 0; m < 3; ++m)
			for(Buf *b : {&kd_pos[m], &kd_dir[m], &kd_colb[m]}) b->release();
		for(Buf *b : {&rad_a, &rad_b, &rad_c, &rad_flag, &radc_a, &radc_b, &radc_c, &rad_kept, &rph_pos, &rph_dir, &rph_colb, &rpk_nodes, &seg_pos,
		              &seg_dir, &seg_colb, &seg_ra, &seg_rb, &seg_rc})
			b->release();
		yafamd_pkd_scratch_free(pkd_scratch);
		yafamd_thin_scratch_free(thin_scratch);
		yafamd_rad_grid_free(rgrid_scratch);
		if(comm) (void)ncclCommDestroy(comm);
		for(hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
		if(stream) (void)hipStreamDestroy(stream);
	}
};

#define HIPCHECK(expr)                                                                                         \
	do                                                                                                         \
	{                                                                                                          \
		const hipError_t e_ = (expr);                                                                          \
		if(e_ != hipSuccess)                                                                                   \
		{                                                                                                      \
			std::ostringstream os_;                                                                            \
			os_ << "GPU: " << #expr << " failed: " << hipGetErrorString(e_) << " (" << __FILE__ << ":" << __LINE__ << ")"; \
			log_.error(os_.str());                                                                             \
			return false;                                                                                      \
		}                                                                                                      \
	} while(0)

#define NCCLCHECK(expr)                                                                                        \
	do                                                                                                         \
	{                                                                                                          \
		const ncclResult_t r_ = (expr);                                                                        \
		if(r_ != ncclSuccess)                                                                                  \
		{                                                                                                      \
			log_.error(std::string("GPU group: ") + #expr + " failed: " + ncclGetErrorString(r_));            \
			return false;                                                                                      \
		}                                                                                                      \
	} while(0)

// a launch timed in profile mode (kernel kind `kind`)
#define PROF(kind, expr)                                                                                       \
	do                                                                                                         \
	{                                                                                                          \
		const int e0_ = d_->profBegin();                                                                       \
		HIPCHECK(expr);                                                                                        \
		d_->profEnd(kind, e0_);                                                                                \
	} while(0)

GpuRenderer::GpuRenderer(Logger &log, int device) : d_(new Impl), log_(log), device_(device) {}
GpuRenderer::~GpuRenderer()
{
	DeviceGuard g(device_);
	delete d_;
}

void *GpuRenderer::d_comm() const { return (void *)d_->comm; }

int GpuRenderer::deviceCount()
{
	int n = 0;
	return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int GpuRenderer::currentDevice()
{
	int d = 0;
	return hipGetDevice(&d) == hipSuccess ? d : 0;
}

void GpuRenderer::enablePeerAccess(const std::vector<int> &devices)
{
	// direct loads / copies between the group's GPUs over xGMI (hipMemcpyPeer works without it, staged)
	for(int a : devices)
		for(int b : devices)
		{
			if(a == b) continue;
			int can = 0;
			if(hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
			DeviceGuard g(a);
			if(hipDeviceEnablePeerAccess(b, 0) != hipSuccess) (void)hipGetLastError();   // already enabled
		}
}

bool GpuRenderer::ready()
{
	if(d_->init_done) return d_->ok;
	d_->init_done = true;
	int n = 0;
	if(hipGetDeviceCount(&n) != hipSuccess || n == 0)
	{
		log_.error("GPU: no HIP device available — the MI355X core has no CPU fallback");
		return false;
	}
	if(device_ >= n)
	{
		log_.error("GPU: device " + std::to_string(device_) + " requested, " + std::to_string(n) + " visible");
		return false;
	}
	if(device_ < 0) HIPCHECK(hipGetDevice(&device_));
	DeviceGuard guard(device_);
	HIPCHECK(hipStreamCreateWithFlags(&d_->stream, hipStreamNonBlocking));
	int dev = device_;
	hipDeviceProp_t prop;
	HIPCHECK(hipGetDeviceProperties(&prop, dev));
	d_->n_cu = prop.multiProcessorCount;
	d_->shade_grid = d_->n_cu * std::max(1, yafamd_shade_blocks_per_cu());
	if(const char *e = getenv("YAFARAY_AMD_SHADE_GRID")) d_->shade_grid = std::max(1, atoi(e));   // tuning sweeps
	d_->nee_grid = d_->n_cu * std::max(1, yafamd_nee_blocks_per_cu());
	if(const char *e = getenv("YAFARAY_AMD_NEE_GRID")) d_->nee_grid = std::max(1, atoi(e));
	// queue segments = k_shade / k_nee workgroups (devscene.h DevCounters)
	d_->nee_grid = d_->shade_grid;
	std::ostringstream os;
	os << "GPU: device " << dev << " " << prop.name << " (" << prop.gcnArchName << ", " << prop.multiProcessorCount << " CUs, "
	   << (prop.totalGlobalMem >> 30) << " GiB)";
	log_.info(os.str());
	d_->ok = true;
	return true;
}

template<class T>
static bool allocCopy(Logger &log_, Buf &b, const T *src, size_t count)
{
	b.release();
	const size_t bytes = std::max<size_t>(16, count * sizeof(T));
	HIPCHECK(hipMalloc(&b.p, bytes));
	b.bytes = bytes;
	if(count) HIPCHECK(hipMemcpy(b.p, src, count * sizeof(T), hipMemcpyHostToDevice));
	return true;
}

static bool ensure(Logger &log_, Buf &b, size_t bytes)
{
	if(b.bytes >= bytes && b.p) return true;
	b.release();
	HIPCHECK(hipMalloc(&b.p, std::max<size_t>(bytes, 16)));
	b.bytes = std::max<size_t>(bytes, 16);
	return true;
}

bool GpuRenderer::upload(HostScene &hs)
{
	if(!ready()) return false;
	DeviceGuard guard(device_);
	Impl &d = *d_;
	if(hs.gpu_build)
	{
		// device build: PLOC + BVH4 collapse (bvhgpu.hip); only the mesh crosses PCIe
		// (the scene bounds: ray binning quantises ray origins in them)
		for(int a = 0; a < 3; ++a) { d.scene_lo[a] = 3.4e38f; d.scene_hi[a] = -3.4e38f; }
		for(size_t k = 0; k + 2 < hs.verts.size(); k += 3)
			for(int a = 0; a < 3; ++a)
			{
				d.scene_lo[a] = std::min(d.scene_lo[a], hs.verts[k + (size_t)a]);
				d.scene_hi[a] = std::max(d.scene_hi[a], hs.verts[k + (size_t)a]);
			}
		Buf v, t;
		if(!allocCopy(log_, v, hs.verts.data(), hs.verts.size())) return false;
		if(!allocCopy(log_, t, hs.tris.data(), hs.tris.size())) return false;
		d.nodes.release();
		d.tris.release();
		d.nodes8.release();
		d.tris8.release();
		void *np = nullptr, *tp = nullptr;
		int nn = 0, depth = 0, need = 0, iters = 0;
		// the 8-wide collapse too, quantised (bvhgpu.hip k_q8_write), traversed by k_trace's refill loop for
		// scenes in global memory: C4 k_trace 140 -> 125 ms per frame (the float BVH8 was slower:
		// 106 VGPRs); YAFARAY_AMD_BVH8=0 keeps the BVH4 there
		const char *b8 = std::getenv("YAFARAY_AMD_BVH8");
		YafBvh8 w8;
		const hipError_t e = yafamd_build_bvh_gpu((const float *)v.p, (const int *)t.p, hs.n_prims, &np, &tp, &nn, &depth, &need, &iters,
		                                          (b8 && *b8 == '0') ? nullptr : &w8, d.stream);
		v.release();
		t.release();
		if(w8.nodes)
		{
			d.nodes8.p = w8.nodes;
			d.nodes8.bytes = (size_t)std::max(1, w8.n_nodes) * 128;
			d.tris8.p = w8.tris;
			d.tris8.bytes = (size_t)std::max(1, hs.n_prims) * 48;
			d.n_nodes8 = w8.n_nodes;
			d.need8 = w8.stack_need;
			d.depth8 = w8.depth;
		}
		HIPCHECK(e);
		d.nodes.p = np;
		d.nodes.bytes = (size_t)std::max(1, nn) * 128;
		d.tris.p = tp;
		d.tris.bytes = (size_t)std::max(1, hs.n_prims) * 48;
		hs.bvh.width = 4;
		hs.bvh.n_nodes = nn;
		hs.bvh.depth = depth;
		hs.bvh.stack_need = need;
		hs.bvh.max_leaf = hs.n_prims > 0 ? 1 : 0;
		hs.ploc_iters = iters;
	}
	else
	{
		d.nodes8.release();
		d.tris8.release();
		d.n_nodes8 = 0;
		if(!allocCopy(log_, d.nodes, hs.bvh.nodes.data(), hs.bvh.nodes.size())) return false;
		if(!allocCopy(log_, d.tris, hs.bvh.tris.data(), hs.bvh.tris.size())) return false;
	}
	if(!allocCopy(log_, d.prim_ng, hs.prim_ng.data(), hs.prim_ng.size())) return false;
	if(!allocCopy(log_, d.mats, hs.mats.data(), hs.mats.size())) return false;
	if(!allocCopy(log_, d.lights, hs.lights.data(), hs.lights.size())) return false;
	d.host_lights = hs.lights;
	if(!hs.mesh_cdf.empty())
	{
		if(!allocCopy(log_, d.mesh_tris, hs.mesh_tris.data(), hs.mesh_tris.size()) || !allocCopy(log_, d.mesh_cdf, hs.mesh_cdf.data(), hs.mesh_cdf.size()) ||
		   !allocCopy(log_, d.mesh_nodes, hs.mesh_nodes.data(), hs.mesh_nodes.size()) || !allocCopy(log_, d.mesh_btris, hs.mesh_btris.data(), hs.mesh_btris.size()))
			return false;
	}
	else for(Buf *b : {&d.mesh_tris, &d.mesh_cdf, &d.mesh_nodes, &d.mesh_btris}) b->release();
	d.has_attr = hs.has_attr;
	d.n_textures = (int)hs.textures.size();
	if(hs.has_attr)
	{
		if(!allocCopy(log_, d.prim_attr, hs.prim_attr.data(), hs.prim_attr.size())) return false;
		if(!allocCopy(log_, d.shader_nodes, hs.shader_nodes.data(), hs.shader_nodes.size())) return false;
		if(!allocCopy(log_, d.textures, hs.textures.data(), hs.textures.size())) return false;
		if(!allocCopy(log_, d.texels, hs.texels.data(), hs.texels.size())) return false;
	}
	else for(Buf *b : {&d.prim_attr, &d.shader_nodes, &d.textures, &d.texels}) b->release();
	d.n_nodes = hs.bvh.n_nodes;
	d.n_tris = hs.n_prims;
	d.n_mats = (int)hs.mats.size();
	// the visible lights come first (Scene::buildAccelerator); photon-only ones follow and only the photon
	// sets below refer to them
	d.n_lights = 0;
	for(const DevLight &L : hs.lights) d.n_lights += L.photon_only ? 0 : 1;
	{
		// sample_pdf1d.h:52-66 over the lights shooting diffuse (bit 0) / caustic (bit 1) photons
		// (render_view.cc:103-110), energies = totalEnergy().energy() (light_area.cc:64,
		// light_point.h:41, color.h:59)
		for(int set = 0; set < 2; ++set)
		{
			std::vector<int> idx;
			std::vector<float> func;
			for(int i : hs.light_name_order)
			{
				const DevLight &L = hs.lights[i];
				if(!(L.shoot & (1u << set))) continue;
				float e[3];
				// point: 4 pi color; area: color * area; mesh (light_object_light.cc:109): double-sided ? 2 color area : color area
				for(int k = 0; k < 3; ++k)
					e[k] = (L.type == LIGHT_POINT)   ? static_cast<float>(3.14159265358979323846264338327950288L) * (4.0f * L.color[k])
					       : (L.type == LIGHT_MESH) ? (L.double_sided ? (2.f * L.color[k]) * L.area : L.color[k] * L.area)
					                                : L.area * L.color[k];
				func.push_back((e[0] + e[1] + e[2]) * 0.333333f);
				idx.push_back(i);
			}
			(set ? d.n_cph_lights : d.n_ph_lights) = (int)idx.size();
			if(idx.empty()) continue;
			std::vector<float> cdf(func.size());
			const double delta = 1.0 / static_cast<double>(func.size());
			double c = 0.0;
			for(size_t i = 0; i < func.size(); ++i)
			{
				c += static_cast<double>(func[i]) * delta;
				cdf[i] = static_cast<float>(c);
			}
			const float integral = static_cast<float>(c);
			for(float &e : cdf) e /= integral;
			(set ? d.clight_inv_integral : d.light_inv_integral) = 1.f / integral;
			if(!allocCopy(log_, set ? d.cph_lights : d.ph_lights, idx.data(), idx.size())) return false;
			if(!allocCopy(log_, set ? d.clight_cdf : d.light_cdf, cdf.data(), cdf.size())) return false;
			if(!allocCopy(log_, set ? d.clight_func : d.light_func, func.data(), func.size())) return false;
		}
	}
	d.depth = hs.bvh.depth;
	d.node_f4 = hs.bvh.width == 4 ? 8 : 4;
	int need = hs.bvh.width == 4 ? hs.bvh.stack_need : hs.bvh.depth;
	if(d.nodes8.p) need = std::max(need, d.need8);   // one stack serves both trees
	d.stack_depth = std::max(8, ((need + 2 + 7) / 8) * 8);
	// BVH4's worst-case bound (3 deferred siblings per level) is far above what rays use: k_trace
	// keeps the first levels in LDS (occupancy) and spills deeper ones to HBM
	d.lds_stack = d.stack_depth;
	if(d.node_f4 == 8) d.lds_stack = std::min(d.stack_depth, 16);
	if(const char *e = getenv("YAFARAY_AMD_LDS_STACK"); e && *e) d.lds_stack = std::min(d.stack_depth, std::max(4, atoi(e)));
	const size_t scene_bytes = (size_t)(d.node_f4 * d.n_nodes + 3 * d.n_tris) * 16;
	d.scene_in_lds = scene_bytes + (size_t)d.lds_stack * yafamd_trace_block() * 4 <= 48 * 1024;
	// (k_trace's packed child keys carry a node index in 9 bits: 48 KB holds at most 384 BVH4 nodes)
	if(d.node_f4 == 8 && d.n_nodes >= 512) d.scene_in_lds = false;
	if(const char *e = getenv("YAFARAY_AMD_SCENE_LDS"); e && *e == '0') d.scene_in_lds = false;   // tests: global-memory traversal on small scenes
	// a BVH4 in global memory: k_trace's refill loop reads the top treelet (the first levels, which
	// every ray visits) from LDS — 21 nodes = the root and two full levels below it, 2.7 KB per
	// workgroup; YAFARAY_AMD_LDS_TOP=n stages n nodes (0: none)
	d.lds_top = 0;
	if(d.node_f4 == 8 && !d.scene_in_lds)
	{
		int top = 21;
		if(const char *e = getenv("YAFARAY_AMD_LDS_TOP"); e && *e) top = std::max(0, atoi(e));
		d.lds_top = std::min(top, d.n_nodes);
		// the treelet and the stack share the workgroup's LDS: clamp the treelet so that k_trace still
		// launches — 64 KB per workgroup, the launch limit
		const size_t stack_b = (size_t)d.lds_stack * yafamd_trace_block() * 4, lds_max = 64 * 1024;
		const int fit = stack_b >= lds_max ? 0 : (int)((lds_max - stack_b) / 144);   // 144 B per staged node (kernels.hip kTopStride)
		if(d.lds_top > fit)
		{
			log_.warning("GPU: YAFARAY_AMD_LDS_TOP=" + std::to_string(d.lds_top) + " does not fit the trace workgroup's LDS; using " +
			             std::to_string(fit) + " nodes");
			d.lds_top = fit;
		}
	}
	// the BVH8's top treelet: the root and its eight children (80 B per node, kernels.hip kTop8Stride)
	d.lds_top8 = 0;
	if(d.nodes8.p && !d.scene_in_lds)
	{
		int top = 9;
		if(const char *e = getenv("YAFARAY_AMD_LDS_TOP8"); e && *e) top = std::max(0, atoi(e));
		const size_t stack_b = (size_t)d.lds_stack * yafamd_trace_block() * 4, lds_max = 64 * 1024;
		const int fit = stack_b >= lds_max ? 0 : (int)((lds_max - stack_b) / 80);
		d.lds_top8 = std::min(std::min(top, d.n_nodes8), fit);
	}
	{
		// persistent trace grid = every resident workgroup once (LDS: per-lane stack (+ scene copy or top treelet))
		const bool w8 = d.nodes8.p && !d.scene_in_lds;
		const size_t dyn = (size_t)d.lds_stack * yafamd_trace_block() * 4 +
		                   (d.scene_in_lds ? scene_bytes : w8 ? (size_t)d.lds_top8 * 80 : (size_t)d.lds_top * 144);
		d.trace_grid = d.n_cu * std::max(1, yafamd_trace_blocks_per_cu(d.scene_in_lds ? 1 : 0, w8 ? 8 : (d.node_f4 == 8 ? 1 : 0), dyn));
		if(const char *e = getenv("YAFARAY_AMD_TRACE_GRID")) d.trace_grid = std::max(1, atoi(e));
		// a whole number of workgroups per queue segment
		d.trace_grid = std::max(1, d.trace_grid / d.shade_grid) * d.shade_grid;
		// transparent shadows launch the BVH4 kernels even when a BVH8 exists (launch_trace): their own
		// resident grid, never above trace_grid (the spill column and statistics are sized for that)
		d.trace_grid_bvh4 = d.trace_grid;
		if(w8 && !getenv("YAFARAY_AMD_TRACE_GRID"))
		{
			const size_t dyn4 = (size_t)d.lds_stack * yafamd_trace_block() * 4 + (size_t)d.lds_top * 144;
			int g4 = d.n_cu * std::max(1, yafamd_trace_blocks_per_cu(0, d.node_f4 == 8 ? 1 : 0, dyn4));
			g4 = std::max(1, g4 / d.shade_grid) * d.shade_grid;
			d.trace_grid_bvh4 = std::min(g4, d.trace_grid);
		}
	}
	d.spill.release();
	if(d.lds_stack < d.stack_depth &&
	   !ensure(log_, d.spill, (size_t)(d.stack_depth - d.lds_stack) * d.trace_grid * yafamd_trace_block() * sizeof(int)))
		return false;
	// Faure tables, dims 0..49 (halton.cc:403-414: dims 0-2 share the base-3 table)
	std::vector<uint8_t> perm;
	std::vector<uint32_t> off(50), base(50);
	std::vector<double> inv(50);
	int primes[50];
	primes[0] = 1;
	for(int k = 1, c = 2; k < 50; ++c)
	{
		bool pr = true;
		for(int q = 2; q * q <= c; ++q) if(c % q == 0) { pr = false; break; }
		if(pr) primes[k++] = c;
	}
	for(int dim = 0; dim < 50; ++dim)
	{
		const std::vector<int> p = faurePerm(dim <= 2 ? 3 : primes[dim]);
		off[dim] = (uint32_t)perm.size();
		for(int v : p) perm.push_back((uint8_t)v);
		base[dim] = (uint32_t)primes[dim];
		inv[dim] = (double)std::llround(1e9 / primes[dim]) / 1e9;
	}
	while(perm.size() % 16) perm.push_back(0);   // staged to LDS as 16-B words
	d.faure_bytes = (int)perm.size();
	if(!allocCopy(log_, d.faure, perm.data(), perm.size())) return false;
	std::vector<uint4> fdim(50);
	for(int dim = 0; dim < 50; ++dim)
	{
		const UDiv dv = udivMake(base[dim]);
		fdim[dim] = make_uint4(base[dim], off[dim], dv.m, dv.sh);
	}
	if(!allocCopy(log_, d.faure_dim, fdim.data(), fdim.size())) return false;
	if(!allocCopy(log_, d.faure_inv, inv.data(), inv.size())) return false;
	stats_.bvh_nodes = (uint32_t)((d.nodes8.p && !d.scene_in_lds) ? d.n_nodes8 : d.n_nodes);
	stats_.bvh_depth = (uint32_t)((d.nodes8.p && !d.scene_in_lds) ? d.depth8 : d.depth);   // of the tree k_trace traverses
	stats_.bvh_width = (d.nodes8.p && !d.scene_in_lds) ? 8u : d.node_f4 == 8 ? 4u : 2u;   // the tree k_trace traverses
	stats_.scene_in_lds = d.scene_in_lds ? 1u : 0u;
	stats_.trace_grid = (uint32_t)d.trace_grid;
	stats_.shade_grid = (uint32_t)d.shade_grid;
	stats_.trace_block = (uint32_t)yafamd_trace_block();
	stats_.stack_depth = (uint32_t)d.stack_depth;
	return true;
}

static void fillScenePointers(GpuRenderer::Impl &d, DevScene &S)
{
	S.nodes = (const float4 *)d.nodes.p;
	S.tris = (const float4 *)d.tris.p;
	S.nodes8 = (d.nodes8.p && !d.scene_in_lds) ? (const float4 *)d.nodes8.p : nullptr;
	S.lds_top8 = d.lds_top8;
	S.tris8 = (const float4 *)d.tris8.p;
	S.prim_ng = (const float4 *)d.prim_ng.p;
	S.mats = (const DevMaterial *)d.mats.p;
	S.lights = (const DevLight *)d.lights.p;
	S.has_mesh_light = 0;
	for(const DevLight &L : d.host_lights) S.has_mesh_light |= L.type == LIGHT_MESH ? 1 : 0;
	S.mesh_tris = (const float4 *)d.mesh_tris.p;
	S.mesh_nodes = (const float4 *)d.mesh_nodes.p;
	S.mesh_btris = (const float4 *)d.mesh_btris.p;
	S.mesh_cdf = (const float *)d.mesh_cdf.p;
	S.faure = (const uint8_t *)d.faure.p;
	S.faure_bytes = d.faure_bytes;
	// materials + per-primitive normals staged in LDS by k_shade / k_nee when they are small
	S.small_tables = ((size_t)d.n_mats * sizeof(DevMaterial) + (size_t)d.n_tris * 16 <= 24 * 1024) ? 1 : 0;
	S.faure_dim = (const uint4 *)d.faure_dim.p;
	S.faure_inv = (const double *)d.faure_inv.p;
	S.n_nodes = d.n_nodes;
	S.node_f4 = d.node_f4;
	S.n_tris = d.n_tris;
	S.n_mats = d.n_mats;
	S.n_lights = d.n_lights;
	S.scene_in_lds = d.scene_in_lds ? 1 : 0;
	S.lds_top = d.lds_top;
	// YAFARAY_AMD_TRACE=brute: scenes of at most 64 triangles test every triangle (k_trace_brute).
	// Measured slower than the BVH on C2 (k_trace 39.0 vs 34.7 ms per frame: 34 exact triangle
	// tests per ray at full lane occupancy cost more than ~3.4 node + 3.3 triangle visits at 0.35),
	// so the BVH stays the default
	// (the measured-and-dropped pipelines — k_trace_brute, ray sorting, the megakernel, in-place NEE
	// shadow rays, the bounded gather walk, the fused shade — exist only in a -DYAF_EXPERIMENTS build)
	{
		const char *e = getenv("YAFARAY_AMD_TRACE");
		S.brute = (yafamd_experiments() && e && std::string(e) == "brute") ? 1 : 0;
	}
	// ray-stream sorting in k_trace (opt-in, YAFARAY_AMD_RAY_SORT=1): measured on C2 it lifts the
	// VALU lane utilisation 0.44 -> 0.50 but costs more than it saves (k_trace 27.6 -> 28.9 ms per
	// frame: the key pass reads every direction twice and the sort's registers spill), DESIGN.md §5
	{
		const char *e = getenv("YAFARAY_AMD_RAY_SORT");
		S.ray_sort = (yafamd_experiments() && e && *e == '1') ? 1 : 0;
	}
	S.ph_lights = (const int *)d.ph_lights.p;
	S.light_cdf = (const float *)d.light_cdf.p;
	S.light_func = (const float *)d.light_func.p;
	S.light_inv_integral = d.light_inv_integral;
	S.n_ph_lights = d.n_ph_lights;
	S.has_attr = d.has_attr ? 1 : 0;
	S.n_textures = d.n_textures;
	S.prim_attr = (const float4 *)d.prim_attr.p;
	S.shader_nodes = (const DevNode *)d.shader_nodes.p;
	S.textures = (const DevTexture *)d.textures.p;
	S.texels = (const float4 *)d.texels.p;
	if(S.has_attr) { S.ext = 1; S.w_live = 1; }
}

// One photon map on the GPU: shoot N paths from the light set L (diffuseWorker /
// causticWorker rules by L.caustic), compact the deposits in photon-id order (one reference
// thread's append order) and build the point kd-tree node for node like the reference (pkd.hip).
// which = 0: the diffuse map buffers, 1: the caustic map buffers.
bool GpuRenderer::shootMap(RenderParams &rp, const PhotonSet &L, uint32_t N, int bounces, int which, uint32_t &n_out, int &depth_out)
{
	Impl &d = *d_;
	DevScene &S = rp.scene;
	n_out = 0;
	depth_out = 0;
	const auto t0 = std::chrono::steady_clock::now();
	const uint32_t slots = (uint32_t)bounces + 1u;
	if((uint64_t)N * slots > 0xffffffffull) { log_.error("PhotonIntegrator: photons x (bounces + 1) exceeds 2^32 deposit slots"); return false; }
	// A group render splits the photon paths: member r shoots the contiguous photon ids
	// [N r / world, N (r + 1) / world) — the reference's threads shoot contiguous id ranges too
	// (integrator_photon_mapping.cc:118-127, 437-441) — and the members concatenate their maps in
	// member order, which is photon-id order: every member then holds the one-GPU map.
	const bool group_render = !rp.band_bounds.empty() && grouped();
	const int world = group_render ? rp.shard_world : 1, me = group_render ? rp.shard_rank : 0;
	const uint32_t h0 = (uint32_t)((uint64_t)N * me / world), h1 = (uint32_t)((uint64_t)N * (me + 1) / world);
	const uint32_t NL = h1 - h0;
	if(which == 0) d.pm_local = NL;
	const size_t n_slots = (size_t)NL * slots;
	// segmented alive lists: one segment per k_photon_bounce workgroup (the trace grid)
	const uint32_t ph_segs = (uint32_t)std::max(1, d.trace_grid), ph_cap = (NL + ph_segs - 1) / ph_segs;
	if(!ensure(log_, d.ph_ray_o, (size_t)NL * 16) || !ensure(log_, d.ph_ray_d, (size_t)NL * 16) || !ensure(log_, d.ph_pcol, (size_t)NL * 16) ||
	   !ensure(log_, d.ph_alive0, (size_t)ph_segs * ph_cap * 4 + 4) || !ensure(log_, d.ph_alive1, (size_t)ph_segs * ph_cap * 4 + 4) ||
	   !ensure(log_, d.ph_n_alive, (size_t)(slots + 1) * ph_segs * 4) ||
	   !ensure(log_, d.dep_a, n_slots * 16) || !ensure(log_, d.dep_b, n_slots * 16) || !ensure(log_, d.dep_c, n_slots * 4) ||
	   !ensure(log_, d.dep_flag, n_slots) || !ensure(log_, d.ph_scan, (((size_t)NL + 1023) / 1024) * 4 + 16) || !ensure(log_, d.ph_total, 16))
		return false;
	PhotonState P{};
	P.ray_o = (float4 *)d.ph_ray_o.p;
	P.ray_d = (float4 *)d.ph_ray_d.p;
	P.pcol = (float4 *)d.ph_pcol.p;
	P.alive[0] = (uint32_t *)d.ph_alive0.p;
	P.alive[1] = (uint32_t *)d.ph_alive1.p;
	P.n_alive = (uint32_t *)d.ph_n_alive.p;
	P.seg_cap = ph_cap;
	P.n_segs = ph_segs;
	P.n_local = NL;
	P.n_slot_rows = slots;
	P.dep_a = (float4 *)d.dep_a.p;
	P.dep_b = (float4 *)d.dep_b.p;
	P.dep_c = (float *)d.dep_c.p;
	P.dep_flag = (uint8_t *)d.dep_flag.p;
	if(n_slots) HIPCHECK(hipMemsetAsync(d.dep_flag.p, 0, n_slots, d.stream));
	// final gathering: radiance points of the diffuse map's deposits (:184-193)
	const bool want_rad = which == 0 && rp.pm.final_gather;
	P.rad_a = P.rad_b = P.rad_c = nullptr;
	P.rad_flag = nullptr;
	if(want_rad)
	{
		if(!ensure(log_, d.rad_a, n_slots * 16) || !ensure(log_, d.rad_b, n_slots * 16) || !ensure(log_, d.rad_c, n_slots * 16) ||
		   !ensure(log_, d.rad_flag, n_slots))
			return false;
		P.rad_a = (float4 *)d.rad_a.p;
		P.rad_b = (float4 *)d.rad_b.p;
		P.rad_c = (float4 *)d.rad_c.p;
		P.rad_flag = (uint8_t *)d.rad_flag.p;
		if(n_slots) HIPCHECK(hipMemsetAsync(d.rad_flag.p, 0, n_slots, d.stream));
	}
	PROF(KK_PHOTON_EMIT, yafamd_photon_emit(&S, &P, &L, N, h0, NL, bounces, d.stream));
	int cur = 0;
	for(int b = 0; b <= bounces; ++b)
	{
		PROF(KK_PHOTON_BOUNCE, yafamd_photon_bounce(&S, &P, &L, N, h0, NL, bounces, b, cur, d.lds_stack, (int *)d.spill.p, d.trace_grid, d.stream));
		cur ^= 1;
	}
	// the member's map in photon-id order (outputs sized for the worst case: every slot stored); a group
	// member compacts into its segment buffers, the concatenation fills the map buffers below
	Buf &pos = which ? d.cph_pos : d.ph_pos, &dir = which ? d.cph_dir : d.ph_dir, &colb = which ? d.cph_colb : d.ph_colb;
	Buf &nodes = which ? d.cpk_nodes : d.pk_nodes;
	Buf &cpos = group_render ? d.seg_pos : pos, &cdir = group_render ? d.seg_dir : dir, &ccolb = group_render ? d.seg_colb : colb;
	uint32_t n = 0;
	if(!ensure(log_, cpos, n_slots * 16) || !ensure(log_, cdir, n_slots * 16) || !ensure(log_, ccolb, n_slots * 4)) return false;
	PROF(KK_PHOTON_COMPACT, yafamd_photon_compact(&P, (uint32_t *)d.ph_scan.p, (uint32_t *)d.ph_total.p, (float4 *)cpos.p, (float4 *)cdir.p,
	                                              (float *)ccolb.p, d.stream));
	HIPCHECK(hipMemcpyAsync(&n, d.ph_total.p, 4, hipMemcpyDeviceToHost, d.stream));
	{
		// the bounce launches' work: every slot of bounce 0's list, then the paths each bounce kept
		std::vector<uint32_t> alive((size_t)(slots + 1) * ph_segs);
		HIPCHECK(hipMemcpyAsync(alive.data(), d.ph_n_alive.p, alive.size() * 4, hipMemcpyDeviceToHost, d.stream));
		HIPCHECK(hipStreamSynchronize(d.stream));
		uint64_t traced = NL;
		for(size_t k = ph_segs; k < (size_t)slots * ph_segs; ++k) traced += alive[k];
		stats_.photon_paths_traced += traced;
		stats_.photon_slots += n_slots;
	}
	uint32_t nr = 0;
	if(want_rad)
	{
		Buf &ra = group_render ? d.seg_ra : d.radc_a, &rb = group_render ? d.seg_rb : d.radc_b, &rc = group_render ? d.seg_rc : d.radc_c;
		if(!ensure(log_, ra, n_slots * 16) || !ensure(log_, rb, n_slots * 16) || !ensure(log_, rc, n_slots * 16)) return false;
		PROF(KK_PHOTON_COMPACT, yafamd_rad_compact(&P, (uint32_t *)d.ph_scan.p, (uint32_t *)d.ph_total.p, (float4 *)ra.p, (float4 *)rb.p,
		                                           (float4 *)rc.p, d.stream));
		HIPCHECK(hipMemcpyAsync(&nr, d.ph_total.p, 4, hipMemcpyDeviceToHost, d.stream));
		HIPCHECK(hipStreamSynchronize(d.stream));
	}
	if(group_render)
	{
		// agree, exchange the members' counts, then concatenate the segments in member order
		const int st = groupStatus(0);
		if(st >= 2)
		{
			log_.error("GPU group: a member failed; render abandoned");
			return false;
		}
		std::vector<uint32_t> counts, rcounts;
		if(!groupCounts(n, counts) || (want_rad && !groupCounts(nr, rcounts))) return false;
		uint64_t tot = 0, rtot = 0;
		for(uint32_t c : counts) tot += c;
		for(uint32_t c : rcounts) rtot += c;
		bool ok = true;
		if(tot > 0xffffffffull || rtot > 0xffffffffull)
		{
			log_.error("PhotonIntegrator: photon map exceeds 2^32 photons");
			ok = false;
		}
		ok = ok && ensure(log_, pos, std::max<uint64_t>(tot, 1) * 16) && ensure(log_, dir, std::max<uint64_t>(tot, 1) * 16) &&
		     ensure(log_, colb, std::max<uint64_t>(tot, 1) * 4);
		ok = ok && (!want_rad || (ensure(log_, d.radc_a, std::max<uint64_t>(rtot, 1) * 16) && ensure(log_, d.radc_b, std::max<uint64_t>(rtot, 1) * 16) &&
		                          ensure(log_, d.radc_c, std::max<uint64_t>(rtot, 1) * 16)));
		if(fault_concat_)
		{
			log_.error("GPU group: injected failure of member " + std::to_string(me) + " between the photon counts and the concatenation");
			ok = false;
		}
		// every member allocates the concatenated map before anyone copies: agree on the outcome, so a
		// member that could not allocate stops the group here instead of leaving the others waiting
		// inside groupConcat (its groupAbort would pair with their first arrival there)
		if(groupStatus(ok ? 0 : 2) >= 2)
		{
			if(ok) log_.error("GPU group: a member failed; render abandoned");
			return false;
		}
		if(!groupConcat(which ? 1 : 0, counts) || (want_rad && !groupConcat(2, rcounts))) return false;
		n = (uint32_t)tot;
		nr = (uint32_t)rtot;
	}
	n_out = n;
	if(want_rad) d.n_rad_points = nr;
	const auto t1 = std::chrono::steady_clock::now();
	stats_.photon_shoot_seconds += std::chrono::duration<double>(t1 - t0).count();
	d.kd_on[which] = false;
	if(n == 0) return true;
	// point kd-tree of the map, built on the GPU node for node like the reference's (pkd.hip)
	if(!ensure(log_, nodes, (2 * (size_t)n - 1) * sizeof(uint4))) return false;
	int depth = 0;
	if(!buildMapTree(which, pos.p, dir.p, colb.p, n, nodes.p, depth, group_render)) return false;
	depth_out = depth;
	stats_.photon_tree_seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
	return true;
}

// estimateOneDirectLight's light pick in the reference's one-thread order (integrator_montecarlo.cc:70-78
// with the counter of integrator_tiled.cc:48, reset at render start, :169-171).  The count run left
// each sample's number of calls in d.lpc (pixel-major, `spp` per pixel).  The one-thread render visits
// the tiles in rank order and inside a tile the rows, pixels and samples in order, so a sample's
// counter starts at: the calls of the render's earlier passes + those of every row segment (one tile
// row) visited before its segment + those of the samples before it in the segment.  The segment sums
// come from the rows each member owns (a group sums the members' tables: every row has one owner),
// the bases are laid out on the host in tile order, and k_lpc_prefix writes every counter of the rows
// [jy0, jy1) this member renders (its band + halo rows).  cut: the count run was canceled (in a group:
// any member's was): the pass renders nothing.
bool GpuRenderer::lpcBases(RenderParams &rp, int spp, int jy0, int jy1, bool group_render, bool &cut)
{
	Impl &d = *d_;
	const DevScene &S = rp.scene;
	const int W = S.width, H = S.height, ts = S.tile, ntx = (W + ts - 1) / ts, nty = (H + ts - 1) / ts;
	const size_t n_seg = (size_t)H * ntx;
	if(!ensure(log_, d.lpc_seg, n_seg * 4)) return false;
	HIPCHECK(hipMemsetAsync(d.lpc_seg.p, 0, n_seg * 4, d.stream));
	// the rows this member owns: its band in a group (owned_rows_ covers the whole film once the
	// accumulators were exchanged before an adaptive pass; the halo rows belong to the neighbours)
	std::vector<std::pair<int, int>> own = owned_rows_;
	if(group_render) own.assign(1, {std::max(0, rp.shard_y0), std::min(H, rp.shard_y1)});
	for(const auto &o : own)
		HIPCHECK(yafamd_lpc_seg((const uint32_t *)d.lpc.p, W, spp, ts, o.first, o.second, (uint32_t *)d.lpc_seg.p, d.stream));
	lpc_seg_host_.assign(n_seg, 0u);
	HIPCHECK(hipMemcpyAsync(lpc_seg_host_.data(), d.lpc_seg.p, n_seg * 4, hipMemcpyDeviceToHost, d.stream));
	HIPCHECK(hipStreamSynchronize(d.stream));
	std::vector<uint32_t> seg = lpc_seg_host_;
	if(group_render)
	{
		// every member's table is complete when all have arrived; sum them, and nobody overwrites its
		// table before everyone summed (the second arrival)
		const int st = groupStatus(cut ? 1 : 0);
		if(st >= 2)
		{
			log_.error("GPU group: a member failed; render abandoned");
			return false;
		}
		if(peers_ && peers_->size() > 1)
		{
			for(int r = 0; r < peers_->size(); ++r)
			{
				if(r == peer_rank_) continue;
				const std::vector<uint32_t> &o = peers_->member(r)->lpc_seg_host_;
				for(size_t k = 0; k < n_seg && k < o.size(); ++k) seg[k] += o[k];
			}
			peers_->arrive(0);
		}
		else if(d.comm)
		{
			NCCLCHECK(ncclAllReduce(d.lpc_seg.p, d.lpc_seg.p, n_seg, ncclUint32, ncclSum, d.comm, d.stream));
			HIPCHECK(hipMemcpyAsync(seg.data(), d.lpc_seg.p, n_seg * 4, hipMemcpyDeviceToHost, d.stream));
			HIPCHECK(hipStreamSynchronize(d.stream));
		}
		if(st == 1) cut = true;
	}
	if(cut) return true;
	// bases in the one-thread visiting order: tiles by rank, rows inside a tile
	std::vector<int> by_rank((size_t)ntx * nty);
	for(int t = 0; t < ntx * nty; ++t) by_rank[t] = t;
	if(rp.tile_rank.size() == by_rank.size())
		for(int t = 0; t < ntx * nty; ++t) by_rank[rp.tile_rank[(size_t)t]] = t;
	std::vector<uint32_t> base(n_seg, 0u);
	uint32_t carry = lpc_carry_;
	for(int t : by_rank)
	{
		const int tx = t % ntx, ty = t / ntx;
		for(int y = ty * ts; y < std::min(H, ty * ts + ts); ++y)
		{
			base[(size_t)y * ntx + tx] = carry;
			carry += seg[(size_t)y * ntx + tx];
		}
	}
	lpc_carry_ = carry;
	HIPCHECK(hipMemcpyAsync(d.lpc_seg.p, base.data(), n_seg * 4, hipMemcpyHostToDevice, d.stream));
	HIPCHECK(yafamd_lpc_prefix((uint32_t *)d.lpc.p, W, spp, ts, jy0, jy1, (const uint32_t *)d.lpc_seg.p, d.stream));
	HIPCHECK(hipStreamSynchronize(d.stream));   // `base` is consumed
	return true;
}

// The members' counts of a photon-map segment, in member order (a status agreement precedes).
bool GpuRenderer::groupCounts(uint32_t mine, std::vector<uint32_t> &all)
{
	Impl &d = *d_;
	if(peers_ && peers_->size() > 1)
	{
		seg_count_ = mine;
		peers_->arrive(0);
		all.assign((size_t)peers_->size(), 0u);
		for(int r = 0; r < peers_->size(); ++r) all[(size_t)r] = peers_->member(r)->seg_count_;
		peers_->arrive(0);   // nobody overwrites its count before everyone read it
		return true;
	}
	const int world = group_world_;
	all.assign((size_t)world, 0u);
	if(!ensure(log_, d.g_status, 16 + 4 * (size_t)world)) return false;
	uint32_t *dev = (uint32_t *)d.g_status.p + 4;
	HIPCHECK(hipMemcpyAsync(dev, &mine, 4, hipMemcpyHostToDevice, d.stream));
	NCCLCHECK(ncclAllGather(dev, dev + 1, 1, ncclUint32, d.comm, d.stream));
	HIPCHECK(hipMemcpyAsync(all.data(), dev + 1, 4 * (size_t)world, hipMemcpyDeviceToHost, d.stream));
	HIPCHECK(hipStreamSynchronize(d.stream));
	return true;
}

// Concatenate every member's segment (counts[r] entries) in member order into this member's arrays:
// kind 0 the diffuse photon map, 1 the caustic map, 2 the radiance points (final gathering).
bool GpuRenderer::groupConcat(int kind, const std::vector<uint32_t> &counts)
{
	Impl &d = *d_;
	struct Arr { Buf Impl::*src, Impl::*dst; size_t elem; };
	std::vector<Arr> arrs;
	if(kind == 2) arrs = {{&Impl::seg_ra, &Impl::radc_a, 16}, {&Impl::seg_rb, &Impl::radc_b, 16}, {&Impl::seg_rc, &Impl::radc_c, 16}};
	else if(kind == 1) arrs = {{&Impl::seg_pos, &Impl::cph_pos, 16}, {&Impl::seg_dir, &Impl::cph_dir, 16}, {&Impl::seg_colb, &Impl::cph_colb, 4}};
	else arrs = {{&Impl::seg_pos, &Impl::ph_pos, 16}, {&Impl::seg_dir, &Impl::ph_dir, 16}, {&Impl::seg_colb, &Impl::ph_colb, 4}};
	std::vector<uint64_t> off(counts.size() + 1, 0);
	for(size_t r = 0; r < counts.size(); ++r) off[r + 1] = off[r] + counts[r];
	if(peers_ && peers_->size() > 1)
	{
		peers_->arrive(0);
		bool ok = true;
		for(int r = 0; r < peers_->size() && ok; ++r)
		{
			if(!counts[(size_t)r]) continue;
			GpuRenderer *src = peers_->member(r);
			for(const Arr &a : arrs)
				ok = ok && hipMemcpyPeerAsync((char *)(d.*(a.dst)).p + off[(size_t)r] * a.elem, device_, (*src->d_.*(a.src)).p, src->device_,
				                              counts[(size_t)r] * a.elem, d.stream) == hipSuccess;
		}
		ok = ok && hipStreamSynchronize(d.stream) == hipSuccess;
		if(!ok) log_.error("GPU group: photon map copy between members failed");
		peers_->arrive(0);
		return ok;
	}
	NCCLCHECK(ncclGroupStart());
	for(int r = 0; r < group_world_; ++r)
	{
		if(!counts[(size_t)r]) continue;
		for(const Arr &a : arrs)
		{
			char *dst = (char *)(d.*(a.dst)).p + off[(size_t)r] * a.elem;
			const void *src = r == group_rank_ ? (d.*(a.src)).p : dst;
			NCCLCHECK(ncclBroadcast(src, dst, counts[(size_t)r] * a.elem, ncclChar, r, d.comm, d.stream));
		}
	}
	NCCLCHECK(ncclGroupEnd());
	HIPCHECK(hipStreamSynchronize(d.stream));
	return true;
}

// The point kd-tree of map `which` (0 diffuse, 1 caustic, 2 radiance) over its n records, built on the
// GPU node for node like the reference's (pkd.hip).  The subtree pass also copies the records into kd
// (leaf) order (kd_pos / kd_dir / kd_colb) and the leaves index those copies, so a k-NN lookup's
// photons are read from neighbouring lines; YAFARAY_AMD_PKD_ORDER=photon keeps photon-order leaves
// (measurement switch; the estimates are identical either way).
//
// group_split (a device / render group's photon maps, every member holding the whole map): the build is
// distributed — member r sorts and runs the top levels above level D = ceil(log2 members) like everyone,
// then only its own level-D subtrees (pkd.hip yafamd_build_pkd_kd_member), and the members exchange those
// subtrees' node and record ranges (exchangeTree).  YAFARAY_AMD_PKD_SPLIT=0: every member builds the tree.
bool GpuRenderer::buildMapTree(int which, const void *pos, const void *dir, const void *colb, uint32_t n, void *nodes, int &depth, bool group_split)
{
	Impl &d = *d_;
	const char *oe = std::getenv("YAFARAY_AMD_PKD_ORDER");
	const bool kd = !(oe && std::string(oe) == "photon");
	d.kd_on[which] = false;
	int members = 1, me = 0;
	if(group_split && peers_ && peers_->size() > 1)
	{
		members = peers_->size();
		me = peer_rank_;
	}
	else if(group_split && d.comm && group_world_ > 1)
	{
		members = group_world_;
		me = group_rank_;
	}
	if(const char *se = std::getenv("YAFARAY_AMD_PKD_SPLIT"); se && *se == '0') members = 1;
	if(kd && n && members > 1)
	{
		// every member reaches the status agreement below, whatever failed before it
		bool ok = ensure(log_, d.kd_pos[which], (size_t)n * 16) && ensure(log_, d.kd_dir[which], (size_t)n * 16) &&
		          ensure(log_, d.kd_colb[which], (size_t)n * 4);
		int D = 0;
		if(ok)
		{
			const int e0 = d.profBegin();
			const hipError_t e = yafamd_build_pkd_kd_member((const float4 *)pos, (const float4 *)dir, (const float *)colb, n, (uint4 *)nodes,
			                                                (float4 *)d.kd_pos[which].p, (float4 *)d.kd_dir[which].p, (float *)d.kd_colb[which].p,
			                                                &depth, d.stream, &d.pkd_scratch, me, members, &D);
			d.profEnd(KK_PHOTON_TREE, e0);
			ok = e == hipSuccess && hipStreamSynchronize(d.stream) == hipSuccess;
			if(!ok) log_.error(std::string("GPU: point kd-tree build failed (") + hipGetErrorString(e) + ")");
		}
		if(groupStatus(ok ? 0 : 2) >= 2)
		{
			if(ok) log_.error("GPU group: a member failed; render abandoned");
			return false;
		}
		d.kd_on[which] = true;
		stats_.pkd_split_level = std::max<uint64_t>(stats_.pkd_split_level, (uint64_t)D);
		return D == 0 || exchangeTree(which, n, nodes, D, members);
	}
	if(kd && n)
	{
		if(!ensure(log_, d.kd_pos[which], (size_t)n * 16) || !ensure(log_, d.kd_dir[which], (size_t)n * 16) ||
		   !ensure(log_, d.kd_colb[which], (size_t)n * 4))
			return false;
		PROF(KK_PHOTON_TREE, yafamd_build_pkd_kd((const float4 *)pos, (const float4 *)dir, (const float *)colb, n, (uint4 *)nodes,
		                                         (float4 *)d.kd_pos[which].p, (float4 *)d.kd_dir[which].p, (float *)d.kd_colb[which].p, &depth,
		                                         d.stream, &d.pkd_scratch));
		d.kd_on[which] = true;
	}
	else if(n) PROF(KK_PHOTON_TREE, yafamd_build_pkd((const float4 *)pos, n, (uint4 *)nodes, &depth, d.stream, &d.pkd_scratch));
	HIPCHECK(hipStreamSynchronize(d.stream));
	return true;
}

// The distributed build's exchange: every member receives the node range [node, node + 2m - 1) and the
// kd-order record range [start, end) of every level-D subtree another member built (the ancestors above
// level D every member built itself), then writes the parent planes over the whole tree.
bool GpuRenderer::exchangeTree(int which, uint32_t n, void *nodes, int D, int members)
{
	Impl &d = *d_;
	std::vector<uint32_t> top((size_t)3 << D);
	yafamd_pkd_top_segments(n, D, top.data());
	std::vector<int> owner((size_t)1 << D, 0);
	for(int r = 0; r < members; ++r)
	{
		uint32_t s0 = 0, s1 = 0;
		yafamd_pkd_owned_segments(D, r, members, &s0, &s1);
		for(uint32_t s = s0; s < s1; ++s) owner[s] = r;
	}
	auto nodesOf = [which](Impl &m) -> Buf & { return which == 0 ? m.pk_nodes : which == 1 ? m.cpk_nodes : m.rpk_nodes; };
	struct Range { size_t off, bytes; };
	auto ranges = [&](uint32_t s) {
		const uint32_t node = top[3 * (size_t)s], a = top[3 * (size_t)s + 1], b = top[3 * (size_t)s + 2];
		return std::array<Range, 4>{Range{(size_t)node * 16, (2 * (size_t)(b - a) - 1) * 16}, Range{(size_t)a * 16, (size_t)(b - a) * 16},
		                            Range{(size_t)a * 16, (size_t)(b - a) * 16}, Range{(size_t)a * 4, (size_t)(b - a) * 4}};
	};
	const int e0 = d.profBegin();
	if(peers_ && peers_->size() > 1)
	{
		peers_->arrive(0);   // every member's subtrees are built (each synchronised its stream)
		bool ok = true;
		for(uint32_t s = 0; s < owner.size() && ok; ++s)
		{
			if(owner[s] == peer_rank_) continue;
			GpuRenderer *src = peers_->member(owner[s]);
			Impl &sd = *src->d_;
			void *dst_p[4] = {nodes, d.kd_pos[which].p, d.kd_dir[which].p, d.kd_colb[which].p};
			const void *src_p[4] = {nodesOf(sd).p, sd.kd_pos[which].p, sd.kd_dir[which].p, sd.kd_colb[which].p};
			const auto rg = ranges(s);
			for(int k = 0; k < 4 && ok; ++k)
				ok = hipMemcpyPeerAsync((char *)dst_p[k] + rg[k].off, device_, (const char *)src_p[k] + rg[k].off, src->device_, rg[k].bytes, d.stream) ==
				     hipSuccess;
		}
		ok = ok && hipStreamSynchronize(d.stream) == hipSuccess;
		if(!ok) log_.error("GPU group: point kd-tree copy between members failed");
		peers_->arrive(0);   // nobody rebuilds before everyone copied
		if(!ok) return false;
	}
	else
	{
		void *bufs[4] = {nodes, d.kd_pos[which].p, d.kd_dir[which].p, d.kd_colb[which].p};
		NCCLCHECK(ncclGroupStart());
		for(uint32_t s = 0; s < owner.size(); ++s)
		{
			const auto rg = ranges(s);
			for(int k = 0; k < 4; ++k)
			{
				char *p = (char *)bufs[k] + rg[k].off;
				NCCLCHECK(ncclBroadcast(p, p, rg[k].bytes, ncclChar, owner[s], d.comm, d.stream));
			}
		}
		NCCLCHECK(ncclGroupEnd());
	}
	HIPCHECK(yafamd_pkd_parent_planes((uint4 *)nodes, n, d.stream));
	d.profEnd(KK_PHOTON_TREE, e0);
	HIPCHECK(hipStreamSynchronize(d.stream));
	return true;
}

// the records the kernels read for map `which`, field f (0 pos, 1 dir, 2 colb): the kd-order copies
// when its tree indexes them
const void *GpuRenderer::mapView(int which, int f, const void *photon_order) const
{
	if(!d_->kd_on[which]) return photon_order;
	return f == 0 ? d_->kd_pos[which].p : f == 1 ? d_->kd_dir[which].p : d_->kd_colb[which].p;
}

// Final gathering's radiance map (integrator_photon_mapping.cc:540-591): the radiance points shootMap
// compacted are thinned on the host (eliminateRadPoints), pre-gathered on the GPU (k_pregather) and
// the point kd-tree of the radiance map is built like the photon maps'.
bool GpuRenderer::buildRadianceMap(RenderParams &rp)
{
	Impl &d = *d_;
	DevScene &S = rp.scene;
	const PhotonParams &pm = rp.pm;
	const uint32_t nr = d.n_rad_points;
	const auto tr0 = std::chrono::steady_clock::now();
	const float maxrad = 0.01f * pm.radius2;   // :568 (used as a squared distance)
	if(!ensure(log_, d.rad_kept, (size_t)std::max(1u, nr) * 4)) return false;
	// thinning on the GPU (fgthin.hip); the host twin serves grids too large for a dense cell table
	uint32_t nk = 0;
	int rounds = 0;
	// YAFARAY_AMD_FG_THIN=host forces the host twin (tests compare both)
	const char *thin_env = std::getenv("YAFARAY_AMD_FG_THIN");
	const bool host_thin = thin_env && std::string(thin_env) == "host";
	const hipError_t te = host_thin ? hipErrorNotSupported
	                                : yafamd_thin_rad_points((const float4 *)d.radc_a.p, (const float4 *)d.radc_b.p, nr, maxrad,
	                                                         (uint32_t *)d.rad_kept.p, &nk, &rounds, d.stream, &d.thin_scratch);
	if(te == hipErrorNotSupported)
	{
		std::vector<float4> pos(nr), nrm(nr);
		HIPCHECK(hipMemcpyAsync(pos.data(), d.radc_a.p, (size_t)nr * 16, hipMemcpyDeviceToHost, d.stream));
		HIPCHECK(hipMemcpyAsync(nrm.data(), d.radc_b.p, (size_t)nr * 16, hipMemcpyDeviceToHost, d.stream));
		HIPCHECK(hipStreamSynchronize(d.stream));
		const std::vector<uint32_t> kept = eliminateRadPoints(pos, nrm, maxrad);
		nk = (uint32_t)kept.size();
		if(nk) HIPCHECK(hipMemcpyAsync(d.rad_kept.p, kept.data(), (size_t)nk * 4, hipMemcpyHostToDevice, d.stream));
		HIPCHECK(hipStreamSynchronize(d.stream));
		rounds = -1;
	}
	else HIPCHECK(te);
	stats_.radiance_points = nr;
	stats_.radiance_photons = nk;
	stats_.fg_thin_rounds = rounds;
	stats_.fg_thin_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - tr0).count();
	d.n_rphotons = 0;
	d.r_depth = 0;
	publishRadianceMap(S, pm, 0);
	std::ostringstream os;
	os << "PhotonIntegrator: " << nr << " radiance points, " << nk << " kept for the radiance map ("
	   << (rounds >= 0 ? "GPU thinning, " + std::to_string(rounds) + " rounds" : std::string("host thinning")) << ", "
	   << stats_.fg_thin_seconds * 1e3 << " ms)";
	log_.info(os.str());
	if(nk == 0) return true;
	if(!ensure(log_, d.rph_pos, (size_t)nk * 16) || !ensure(log_, d.rph_dir, (size_t)nk * 16) || !ensure(log_, d.rph_colb, (size_t)nk * 4) ||
	   !ensure(log_, d.rpk_nodes, (2 * (size_t)nk - 1) * sizeof(uint4)))
		return false;
	// the kept points' reflectivities (deferred by k_photon_bounce in scenes without EXT materials)
	PROF(KK_PREGATHER, yafamd_rad_refl(&S, (float4 *)d.radc_a.p, (float4 *)d.radc_b.p, (float4 *)d.radc_c.p, (const uint32_t *)d.rad_kept.p, nk,
	                                   d.stream));
	DevScene probe = S;
	probe.n_seg = (uint32_t)d.shade_grid;   // the gather grid k_pregather shares pk_stack with
	// its node visits and summed photons (statistics; read with the render's)
	if(!ensure(log_, d.pre_stats, sizeof(DevStats))) return false;
	HIPCHECK(hipMemsetAsync(d.pre_stats.p, 0, sizeof(DevStats), d.stream));
	d.pre_stats_valid = true;
	PROF(KK_PREGATHER, yafamd_pregather(&probe, (const float4 *)d.radc_a.p, (const float4 *)d.radc_b.p, (const float4 *)d.radc_c.p,
	                                    (const uint32_t *)d.rad_kept.p, nk, (float4 *)d.rph_pos.p, (float4 *)d.rph_dir.p, (float *)d.rph_colb.p,
	                                    (DevStats *)d.pre_stats.p, d.stream));
	int depth = 0;
	if(!buildMapTree(2, d.rph_pos.p, d.rph_dir.p, d.rph_colb.p, nk, d.rpk_nodes.p, depth)) return false;
	d.n_rphotons = (int)nk;
	d.r_depth = depth;
	stats_.fg_radiance_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - tr0).count();
	publishRadianceMap(S, pm, nk);
	return true;
}

// The scene fields of final gathering over a radiance map of nk photons (built, loaded or kept).
void GpuRenderer::publishRadianceMap(DevScene &S, const PhotonParams &pm, uint32_t nk)
{
	Impl &d = *d_;
	S.fg_on = 1;
	S.fg_samples = pm.fg_samples;
	S.fg_bounces = pm.fg_bounces;
	S.fg_min_pathlen = pm.fg_min_pathlen;
	S.fg_lookup_rad = 4 * pm.radius2 * pm.radius2;                                   // :245
	S.fg_i_scale = static_cast<float>(1.f / ((float)S.pm_paths * 3.1415926535897932384626433832795L));   // :53 (math::num_pi)
	S.n_rphotons = (int)nk;
	S.rph_pos = nk ? (const float4 *)mapView(2, 0, d.rph_pos.p) : nullptr;
	S.rph_dir = nk ? (const float4 *)mapView(2, 1, d.rph_dir.p) : nullptr;
	S.rph_colb = nk ? (const float *)mapView(2, 2, d.rph_colb.p) : nullptr;
	S.rpk_nodes = nk ? (const uint4 *)d.rpk_nodes.p : nullptr;
	// k_fg's nearest searches keep their far-child stack in LDS when the tree is shallow enough
	S.rpk_lds = (nk && d.r_depth + 1 <= 32) ? d.r_depth + 1 : 0;
	if(const char *e = getenv("YAFARAY_AMD_FG_NEAREST"); e && std::string(e) == "private") S.rpk_lds = 0;
	// the per-path final gathering's nearest searches over a uniform grid of the map (RadGrid; a tie of the
	// nearest distance asks the kd search); YAFARAY_AMD_FG_GRID=0 keeps the kd search for every lookup
	S.rgrid = RadGrid{};
	const char *ge = getenv("YAFARAY_AMD_FG_GRID");
	if(nk && !(ge && *ge == '0'))
	{
		const hipError_t e = yafamd_rad_grid(S.rph_pos, S.rph_dir, nk, S.fg_lookup_rad, &S.rgrid, d.stream, &d.rgrid_scratch);
		if(e != hipSuccess)
		{
			if(e != hipErrorNotSupported) log_.warning("PhotonIntegrator: radiance-map grid not built (" + std::string(hipGetErrorString(e)) + "); kd searches");
			(void)hipGetLastError();
			S.rgrid = RadGrid{};
		}
	}
}

namespace
{
const char *const kMapNames[3] = {"Diffuse Photon Map", "Caustic Photon Map", "FG Radiance Photon Map"};   // :105-107, montecarlo.cc:49
}

// PhotonMap::load (photon.cc:54-87) into the device map `which` (0 diffuse, 1 caustic, 2 radiance)
// and its kd-tree (updateTree).
bool GpuRenderer::loadMap(RenderParams &rp, int which, const std::string &file)
{
	Impl &d = *d_;
	log_.info(std::string("Integrator: Loading ") + kMapNames[which] + " from: " + file +
	          ". If it does not match the scene you could have crashes and/or incorrect renders, USE WITH CARE!");
	photonfile::Map m;
	if(!photonfile::load(log_, file, m)) return false;
	if(!m.has_dir)
		log_.warning(std::string("Integrator: ") + file + " holds no photon directions (a reference-format file): they load as zero, "
		             "as the reference's PhotonMap::load leaves them");
	const uint32_t n = m.size();
	d.kd_on[which] = false;
	Buf &pos = which == 0 ? d.ph_pos : which == 1 ? d.cph_pos : d.rph_pos;
	Buf &dir = which == 0 ? d.ph_dir : which == 1 ? d.cph_dir : d.rph_dir;
	Buf &colb = which == 0 ? d.ph_colb : which == 1 ? d.cph_colb : d.rph_colb;
	Buf &nodes = which == 0 ? d.pk_nodes : which == 1 ? d.cpk_nodes : d.rpk_nodes;
	std::vector<float4> hp(n), hd(n);
	std::vector<float> hb(n);
	for(size_t i = 0; i < n; ++i)
	{
		hp[i] = make_float4(m.pos[i * 3], m.pos[i * 3 + 1], m.pos[i * 3 + 2], m.col[i * 3]);
		hd[i] = make_float4(m.dir[i * 3], m.dir[i * 3 + 1], m.dir[i * 3 + 2], m.col[i * 3 + 1]);
		hb[i] = m.col[i * 3 + 2];
	}
	const size_t cap = std::max<size_t>(n, 1);
	if(!ensure(log_, pos, cap * 16) || !ensure(log_, dir, cap * 16) || !ensure(log_, colb, cap * 4) || !ensure(log_, nodes, (2 * cap - 1) * sizeof(uint4)))
		return false;
	int depth = 0;
	if(n)
	{
		HIPCHECK(hipMemcpyAsync(pos.p, hp.data(), (size_t)n * 16, hipMemcpyHostToDevice, d.stream));
		HIPCHECK(hipMemcpyAsync(dir.p, hd.data(), (size_t)n * 16, hipMemcpyHostToDevice, d.stream));
		HIPCHECK(hipMemcpyAsync(colb.p, hb.data(), (size_t)n * 4, hipMemcpyHostToDevice, d.stream));
		if(!buildMapTree(which, pos.p, dir.p, colb.p, n, nodes.p, depth)) return false;
	}
	HIPCHECK(hipStreamSynchronize(d.stream));
	if(which == 0) { d.n_photons = (int)n; d.pm_paths = m.paths; d.d_depth = depth; }
	else if(which == 1) { d.c_photons = (int)n; d.c_paths = m.paths; d.c_depth = depth; }
	else { d.n_rphotons = (int)n; d.r_depth = depth; }
	d.map_owner[which] = rp.pm.owner;
	std::ostringstream os;
	os << "Integrator: " << kMapNames[which] << " loaded: " << n << " photons, " << m.paths << " paths (kd-tree depth " << depth << ")";
	log_.info(os.str());
	return true;
}

// PhotonMap::save (photon.cc:89-110) of the device map `which`, plus the direction block (photonfile.h).
bool GpuRenderer::saveMap(RenderParams &rp, int which, const std::string &file)
{
	Impl &d = *d_;
	const uint32_t n = (uint32_t)(which == 0 ? d.n_photons : which == 1 ? d.c_photons : d.n_rphotons);
	const Buf &pos = which == 0 ? d.ph_pos : which == 1 ? d.cph_pos : d.rph_pos;
	const Buf &dir = which == 0 ? d.ph_dir : which == 1 ? d.cph_dir : d.rph_dir;
	const Buf &colb = which == 0 ? d.ph_colb : which == 1 ? d.cph_colb : d.rph_colb;
	std::vector<float4> hp(n), hd(n);
	std::vector<float> hb(n);
	if(n)
	{
		HIPCHECK(hipMemcpyAsync(hp.data(), pos.p, (size_t)n * 16, hipMemcpyDeviceToHost, d.stream));
		HIPCHECK(hipMemcpyAsync(hd.data(), dir.p, (size_t)n * 16, hipMemcpyDeviceToHost, d.stream));
		HIPCHECK(hipMemcpyAsync(hb.data(), colb.p, (size_t)n * 4, hipMemcpyDeviceToHost, d.stream));
		HIPCHECK(hipStreamSynchronize(d.stream));
	}
	photonfile::Map m;
	m.name = kMapNames[which];
	m.paths = which == 0 ? d.pm_paths : which == 1 ? d.c_paths : 0;   // the radiance map's paths stay 0 (:398, 585)
	m.threads_pkd_tree = std::max(1, rp.pm.threads);
	m.pos.resize((size_t)n * 3);
	m.col.resize((size_t)n * 3);
	m.dir.resize((size_t)n * 3);
	for(size_t i = 0; i < n; ++i)
	{
		const float p[3] = {hp[i].x, hp[i].y, hp[i].z}, c[3] = {hp[i].w, hd[i].w, hb[i]}, w[3] = {hd[i].x, hd[i].y, hd[i].z};
		for(int k = 0; k < 3; ++k)
		{
			m.pos[i * 3 + k] = p[k];
			m.col[i * 3 + k] = c[k];
			m.dir[i * 3 + k] = w[k];
		}
	}
	log_.info(std::string("Integrator: Saving ") + kMapNames[which] + " to: " + file);
	return photonfile::save(log_, file, m);
}

bool GpuRenderer::buildPhotonMap(RenderParams &rp)
{
	Impl &d = *d_;
	DevScene &S = rp.scene;
	PhotonParams &pm = rp.pm;
	S.n_photons = 0;
	S.pm_paths = 0;
	S.pm_search = pm.search;
	S.pm_radius2 = pm.radius2;
	S.pm_stack = 8;
	S.caus_map = 0;
	S.c_photons = 0;
	S.c_paths = 0;
	S.c_search = std::max(1, pm.caustic_search);
	S.c_radius2 = pm.caustic_radius * pm.caustic_radius;   // integrator_montecarlo.cc:629
	S.gather_on = 0;
	stats_.photon_shoot_seconds = stats_.photon_tree_seconds = 0.0;
	stats_.pkd_split_level = 0;
	const auto t0 = std::chrono::steady_clock::now();
	// integrator_photon_mapping.cc:437 / integrator_montecarlo.cc:604 (threads_photons <= 0 counts as one)
	const uint32_t T = (uint32_t)std::max(1, pm.threads);
	const bool want_diffuse = S.integrator == INT_PHOTON && pm.diffuse_map;
	const bool want_fg = want_diffuse && pm.final_gather;
	const bool want_caustic = pm.caustic_map;
	d.pm_local = 0;
	// ---- photon_maps_processing (integrator_photon_mapping.cc:279-385, integrator_montecarlo.cc:546-573) ----
	int mode = pm.processing;
	if(mode == PhotonParams::PM_LOAD)
	{
		// every enabled map is read (caustic, diffuse, radiance); one failure regenerates all and saves them
		bool failed = false;
		if(want_caustic && !loadMap(rp, 1, pm.map_path + "_caustic.photonmap")) failed = true;
		if(want_diffuse && !loadMap(rp, 0, pm.map_path + "_diffuse.photonmap")) failed = true;
		if(want_fg && !loadMap(rp, 2, pm.map_path + "_fg_radiance.photonmap")) failed = true;
		if(failed)
		{
			log_.warning("Integrator: photon maps loading failed, changing to Generate and Save mode.");
			mode = PhotonParams::PM_GENERATE_SAVE;
		}
	}
	if(mode == PhotonParams::PM_REUSE)
	{
		// the maps of the previous render of this integrator, if it left them (an empty one cannot be reused)
		auto keep = [&](bool want, int which, int count, const char *what) {
			if(!want) return;
			log_.info(std::string("Integrator: Reusing ") + what + " photon map from memory. If it does not match the scene you could have "
			          "crashes and/or incorrect renders, USE WITH CARE!");
			if(d.map_owner[which] != pm.owner || count == 0)
			{
				log_.warning(std::string("Integrator: ") + what + " photon map enabled but empty, cannot be reused: changing to Generate mode.");
				mode = PhotonParams::PM_GENERATE;
			}
		};
		keep(want_caustic, 1, d.c_photons, "caustics");
		keep(want_diffuse, 0, d.n_photons, "diffuse");
		keep(want_fg, 2, d.n_rphotons, "FG radiance");
	}
	// a group render: every member generates (the shooting is sharded) if any member has to
	if(!rp.band_bounds.empty() && grouped())
	{
		const bool mine = mode == PhotonParams::PM_GENERATE || mode == PhotonParams::PM_GENERATE_SAVE;
		const int st = groupStatus(mine ? 1 : 0);
		if(st >= 2)
		{
			log_.error("GPU group: a member failed; render abandoned");
			return false;
		}
		if(st == 1 && !mine)
		{
			log_.warning("GPU group: another member has to generate its photon maps; generating them here too");
			mode = pm.processing == PhotonParams::PM_LOAD ? PhotonParams::PM_GENERATE_SAVE : PhotonParams::PM_GENERATE;
		}
	}
	pm.processing = mode;
	stats_.photon_maps_mode = mode;
	const bool generate = mode == PhotonParams::PM_GENERATE || mode == PhotonParams::PM_GENERATE_SAVE;
	if(generate)
	{
		int depth_c = 0, depth_d = 0;
		d.c_photons = d.c_paths = d.c_depth = 0;
		d.n_photons = d.pm_paths = d.d_depth = 0;
		d.n_rphotons = d.r_depth = 0;
		d.map_owner[0] = d.map_owner[1] = d.map_owner[2] = 0;
		// ---- caustic map (createCausticMap, integrator_montecarlo.cc:565-625) ----
		if(want_caustic)
		{
			if(d.n_cph_lights == 0) log_.warning("Integrator: no lights shoot caustic photons; caustic photon map empty");
			else if(pm.caustic_photons > 0)
			{
				const uint32_t N = std::max(T, ((uint32_t)pm.caustic_photons / T) * T);
				PhotonSet L{(const int *)d.cph_lights.p, (const float *)d.clight_cdf.p, (const float *)d.clight_func.p, d.clight_inv_integral,
				            d.n_cph_lights, 1};
				uint32_t n = 0;
				if(!shootMap(rp, L, N, std::max(0, pm.caustic_depth), 1, n, depth_c)) return false;
				d.c_photons = (int)n;
				d.c_paths = (int)N;
				d.c_depth = depth_c;
				std::ostringstream os;
				os << "Integrator: shot " << N << " caustic photons, stored " << n << " (kd-tree depth " << depth_c << ")";
				log_.info(os.str());
			}
			d.map_owner[1] = pm.owner;
		}
		// ---- diffuse map (PhotonIntegrator::preprocess, integrator_photon_mapping.cc:242-638) ----
		uint32_t n = 0;
		uint32_t N = 0;
		if(S.integrator == INT_PHOTON && pm.photons > 0)
		{
			if(d.n_ph_lights == 0) log_.warning("PhotonIntegrator: no lights shoot diffuse photons; diffuse photon map disabled");
			else
			{
				N = std::max(T, ((uint32_t)pm.photons / T) * T);
				PhotonSet L{(const int *)d.ph_lights.p, (const float *)d.light_cdf.p, (const float *)d.light_func.p, d.light_inv_integral,
				            d.n_ph_lights, 0};
				if(!shootMap(rp, L, N, pm.bounces, 0, n, depth_d)) return false;
				if(n < 50) { log_.error("PhotonIntegrator: Too few diffuse photons, stopping now."); return false; }   // :448-452
			}
		}
		d.n_photons = (int)n;
		d.pm_paths = (int)N;
		d.d_depth = depth_d;
		if(want_diffuse) d.map_owner[0] = pm.owner;
		std::ostringstream os;
		if(S.integrator == INT_PHOTON)
		{
			os << "PhotonIntegrator: shot " << N << " photons, stored " << n << " (kd-tree depth " << depth_d << ")";
			log_.info(os.str());
		}
	}
	// ---- the maps the render reads (generated, loaded or kept) ----
	if(want_caustic && d.c_photons > 0)
	{
		S.caus_map = 1;
		S.c_photons = d.c_photons;
		S.c_paths = d.c_paths;
		S.cph_pos = (const float4 *)mapView(1, 0, d.cph_pos.p);
		S.cph_dir = (const float4 *)mapView(1, 1, d.cph_dir.p);
		S.cph_colb = (const float *)mapView(1, 2, d.cph_colb.p);
		S.cpk_nodes = (const uint4 *)d.cpk_nodes.p;
	}
	const int n_diffuse = S.integrator == INT_PHOTON ? d.n_photons : 0;
	// the radiance map of a generating render is at most as deep as the diffuse map it came from
	d.pm_stack = std::max({d.d_depth, d.c_depth, generate ? 0 : d.r_depth}) + 1;
	S.ph_pos = (const float4 *)mapView(0, 0, d.ph_pos.p);
	S.ph_dir = (const float4 *)mapView(0, 1, d.ph_dir.p);
	S.ph_colb = (const float *)mapView(0, 2, d.ph_colb.p);
	S.pk_nodes = (const uint4 *)d.pk_nodes.p;
	S.n_photons = n_diffuse;
	S.pm_paths = S.integrator == INT_PHOTON ? d.pm_paths : 0;
	S.pm_stack = d.pm_stack;
	S.gather_on = (S.n_photons > 0 || S.caus_map) ? 1 : 0;
	if(S.gather_on)
	{
		// k_gather's lookup stacks (pm_stack levels per gather lane, in HBM)
		DevScene seg_probe = S;
		seg_probe.n_seg = (uint32_t)d.shade_grid;   // the queue segments of the render that follows
		if(!ensure(log_, d.pk_stack, (size_t)d.pm_stack * yafamd_gather_lanes(&seg_probe) * sizeof(uint2))) return false;
		S.pk_stack = (uint2 *)d.pk_stack.p;
	}
	S.fg_on = 0;
	S.fg_pass_samples = 0;
	S.n_rphotons = 0;
	S.rpk_lds = 0;
	if(want_fg && n_diffuse > 0)
	{
		if(generate)
		{
			if(!buildRadianceMap(rp)) return false;
			d.map_owner[2] = pm.owner;
		}
		else
			publishRadianceMap(S, pm, (uint32_t)d.n_rphotons);
	}
	stats_.photons = (uint64_t)n_diffuse;
	stats_.caustic_photons = S.caus_map ? (uint64_t)d.c_photons : 0;
	if(S.fg_on) stats_.radiance_photons = (uint64_t)d.n_rphotons;
	// ---- generate-save: the maps to files (integrator_photon_mapping.cc:599-624, montecarlo.cc:630-636) ----
	if(mode == PhotonParams::PM_GENERATE_SAVE && pm.write_files)
	{
		bool ok = true;
		if(want_diffuse) ok = saveMap(rp, 0, pm.map_path + "_diffuse.photonmap") && ok;
		if(want_caustic) ok = saveMap(rp, 1, pm.map_path + "_caustic.photonmap") && ok;
		if(want_fg && S.fg_on) ok = saveMap(rp, 2, pm.map_path + "_fg_radiance.photonmap") && ok;
		if(!ok) log_.warning("Integrator: saving the photon maps failed; the render goes on");
	}
	const auto t2 = std::chrono::steady_clock::now();
	stats_.photon_seconds = std::chrono::duration<double>(t2 - t0).count();
	if(S.integrator == INT_PHOTON)
	{
		std::ostringstream os;
		os << "PhotonIntegrator: photon maps ready in " << stats_.photon_seconds << " s";
		log_.info(os.str());
	}
	return true;
}

bool GpuRenderer::render(RenderParams &rp, volatile bool *canceled)
{
	if(!ready()) return false;
	DeviceGuard guard(device_);
	Impl &d = *d_;
	// a group render: the members meet between adaptive passes (status + accumulator exchange)
	const bool group_render = !rp.band_bounds.empty() && grouped();
	if(group_render && ((int)rp.band_bounds.size() != rp.shard_world + 1 || rp.shard_mode != 2))
	{
		log_.error("GPU group: band bounds do not match the group");
		return false;
	}
	DevScene &S = rp.scene;
	fillScenePointers(d, S);
	stats_.photons = 0;
	stats_.photon_paths_traced = stats_.photon_slots = 0;
	stats_.caustic_photons = 0;
	stats_.radiance_points = stats_.radiance_photons = 0;
	stats_.fg_thin_seconds = stats_.fg_radiance_seconds = 0.0;
	stats_.fg_thin_rounds = 0;
	stats_.photon_seconds = 0.0;
	d.prof_on = rp.profile;
	d.ev_n = 2;
	d.prof_recs.clear();
	ktimes_ = KernelTimes{};
	S.caus_map = 0;
	S.gather_on = 0;
	S.n_photons = 0;
	S.fg_on = 0;
	S.n_rphotons = 0;
	S.rpk_lds = 0;
	if(S.integrator == INT_PHOTON || rp.pm.caustic_map)
	{
		// PhotonIntegrator::preprocess (integrator_photon_mapping.cc:242-638) / createCausticMap
		// (integrator_montecarlo.cc:565-625): the photon maps are rebuilt for every render, as the
		// reference's "generate" mode does
		if(!buildPhotonMap(rp)) return false;
		if(S.fg_on && S.tr_shad &&
		   !ensure(log_, d.fg_ts, (size_t)d.trace_grid * yafamd_trace_block() * (size_t)std::max(1, S.s_depth) * sizeof(float2)))
			return false;
		if(yafamd_gather_lds_bytes(&S) > 64 * 1024)
		{
			log_.error("Integrator: photon search " + std::to_string(std::max(S.pm_search, S.c_search)) + " needs more LDS than the gather kernel has");
			return false;
		}
	}
	const int W = S.width, H = S.height, spp = S.spp, ts = S.tile;
	// ---- jobs: owned rows (+ halo rows for the film gather when sharded) ----
	// shard_mode 1: one contiguous band of H / world pixel rows per rank (per-row cost is nearly
	// uniform, so equal bands balance the GPUs and only one halo row is rendered twice);
	// shard_mode 0: whole tile rows r % world == rank.  Either way every owned pixel gets exactly the
	// samples, and the film order, of a one-GPU render.
	const int tile_rows = (H + ts - 1) / ts;
	std::vector<DevJob> jobs;
	owned_rows_.clear();
	uint64_t total = 0;
	if(rp.shard_world <= 1) owned_rows_.push_back({0, H});
	else if(rp.shard_mode == 2)
	{
		const int y0 = std::max(0, rp.shard_y0), y1 = std::min(H, rp.shard_y1);
		if(y1 > y0) owned_rows_.push_back({y0, y1});
	}
	else if(rp.shard_mode == 1)
	{
		const int y0 = (int)((int64_t)H * rp.shard_rank / rp.shard_world), y1 = (int)((int64_t)H * (rp.shard_rank + 1) / rp.shard_world);
		if(y1 > y0) owned_rows_.push_back({y0, y1});
	}
	else
		for(int r = 0; r < tile_rows; ++r)
		{
			if(r % rp.shard_world != rp.shard_rank) continue;
			const int y0 = r * ts, y1 = std::min(H, y0 + ts);
			if(!owned_rows_.empty() && owned_rows_.back().second == y0) owned_rows_.back().second = y1;
			else owned_rows_.push_back({y0, y1});
		}
	for(const auto &o : owned_rows_)
	{
		const int y0 = o.first, y1 = o.second;
		if(rp.shard_world > 1 && rp.film.reach_fwd > 0 && y0 > 0)
		{
			const int hy0 = std::max(0, y0 - rp.film.reach_fwd);
			jobs.push_back({hy0, y0, total});
			total += (uint64_t)W * (y0 - hy0) * spp;
		}
		jobs.push_back({y0, y1, total});
		total += (uint64_t)W * (y1 - y0) * spp;
		if(rp.shard_world > 1 && rp.film.reach_back > 0 && y1 < H)
		{
			const int hy1 = std::min(H, y1 + rp.film.reach_back);
			jobs.push_back({y1, hy1, total});
			total += (uint64_t)W * (hy1 - y1) * spp;
		}
	}
	if(!allocCopy(log_, d.jobs, jobs.data(), jobs.size())) return false;
	const int n_jobs = (int)jobs.size();
	// ---- frame buffers ----
	if(!ensure(log_, d.samples, (size_t)W * H * spp * sizeof(float4))) return false;
	if(!ensure(log_, d.film, (size_t)W * H * sizeof(float4))) return false;
	if(!ensure(log_, d.accum, (size_t)W * H * sizeof(float4))) return false;
	if(!ensure(log_, d.weights, (size_t)W * H * sizeof(float))) return false;
	d.film_w = W;
	d.film_h = H;
	HIPCHECK(hipMemsetAsync(d.film.p, 0, (size_t)W * H * sizeof(float4), d.stream));
	HIPCHECK(hipMemsetAsync(d.weights.p, 0, (size_t)W * H * sizeof(float), d.stream));
	HIPCHECK(hipMemsetAsync(d.accum.p, 0, (size_t)W * H * sizeof(float4), d.stream));
	if(rp.load_rgba && rp.load_weights)
	{
		// film files loaded and summed on the host (imageFilmLoadAllInFolder) become the accumulators
		HIPCHECK(hipMemcpyAsync(d.accum.p, rp.load_rgba, (size_t)W * H * sizeof(float4), hipMemcpyHostToDevice, d.stream));
		HIPCHECK(hipMemcpyAsync(d.weights.p, rp.load_weights, (size_t)W * H * sizeof(float), hipMemcpyHostToDevice, d.stream));
		HIPCHECK(hipStreamSynchronize(d.stream));
	}
	// ---- chunk buffers ----
	size_t M = (size_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)rp.chunk_slots, std::max<uint64_t>(total, 1)));
	// a group member's band moves from frame to frame (rebalanceBands): the chunk buffers hold twice an equal
	// share, so a band that grows does not re-allocate them (GBs, hipFree + hipMalloc) between timed frames
	if(rp.shard_world > 1)
	{
		const uint64_t share2 = 2 * (((uint64_t)W * H * spp + rp.shard_world - 1) / rp.shard_world);
		M = std::max<size_t>(M, (size_t)std::min<uint64_t>((uint64_t)rp.chunk_slots, share2));
	}
	if(S.tree)
	{
		// the recursion tree of a chunk holds up to 2^(raydepth + 1) - 2 spawned nodes per sample
		// (88 B each): cap the level-0 chunk at 2 M samples and the spawn records at 64 per sample
		M = std::min<size_t>(M, (size_t)1 << 21);
		const int depth = std::max(0, std::min(S.raydepth + S.max_add_depth, 5));
		const size_t per = std::max<size_t>(2, ((size_t)1 << (depth + 1)) - 2);
		const size_t cap = M * per;
		if(!ensure(log_, d.spawn_o, cap * 16) || !ensure(log_, d.spawn_d, cap * 16) || !ensure(log_, d.spawn_pr, cap * 16) ||
		   !ensure(log_, d.node_own, (M + cap) * 16) || !ensure(log_, d.node_child, (M + cap) * 8) || !ensure(log_, d.node_w, (M + cap) * 16) ||
		   !ensure(log_, d.spawn_count, 16))
			return false;
		S.node_base = (uint32_t)M;
		S.spawn_cap = (uint32_t)cap;
		S.spawn_o = (float4 *)d.spawn_o.p;
		S.spawn_d = (float4 *)d.spawn_d.p;
		S.spawn_pr = (uint4 *)d.spawn_pr.p;
		S.node_own = (float4 *)d.node_own.p;
		S.node_child = (int2 *)d.node_child.p;
		S.node_w = (float4 *)d.node_w.p;
		S.spawn_count = (uint32_t *)d.spawn_count.p;
	}
	S.cur_level = 0;
	// AA_light_sample_multiplier_factor: pass p draws ceilf(samples * factor^p) samples per area light
	// (integrator_montecarlo.cc:396), so the NEE layout changes per pass; size it for the largest
	const bool light_mult = rp.aa.passes > 1 && rp.aa.light_sample_multiplier_factor != 1.f;
	auto lightLayout = [&](float mult, std::vector<DevLight> &ls) -> int {
		ls = d.host_lights;
		uint32_t base = 0, max_one = 1;
		for(DevLight &L : ls)
		{
			if(L.photon_only) continue;   // no NEE entries (after the visible lights)
			if(L.type == LIGHT_AREA || L.type == LIGHT_MESH)
			{
				L.samples = (int)ceilf((float)L.samples * mult);
				L.inv_samples = 1.f / (float)L.samples;
				L.nee_count = 2u * (uint32_t)std::max(0, L.samples);
			}
			L.nee_base = base;
			base += L.nee_count;
			max_one = std::max(max_one, L.nee_count);
		}
		S.nee_all_count = (int)base;
		return (int)std::max(base + (S.do_ao ? (uint32_t)S.ao_samples : 0u), max_one);
	};
	if(light_mult)
	{
		float mult = 1.f;
		std::vector<DevLight> tmp;
		for(int p = 1; p < rp.aa.passes; ++p)
		{
			mult *= rp.aa.light_sample_multiplier_factor;
			S.nee_k = std::max(S.nee_k, lightLayout(mult, tmp));
		}
		lightLayout(1.f, tmp);
	}
	const int K = std::max(1, S.nee_k);
	const bool need_v0 = S.path_samples > 1 || S.integrator == INT_PHOTON || S.caus_map;
	const bool need_g = S.gather_on != 0;
	// segment capacity: the camera deals groups of 256 samples round-robin over the segments
	const size_t R = (size_t)d.shade_grid;
	auto shardCap = [R](size_t m) { return (((m + 255) / 256 + R - 1) / R) * 256; };
	const bool need_attr = S.has_attr != 0;
	const int need_ts = S.tr_shad ? std::max(1, S.s_depth) : 0;
	const bool need_tree = S.tree != 0;   // the full record (slot + col.w stage) only with a specular recursion tree
	// transparent shadows keep shadowDepth (t, primitive) pairs per shadow ray: deep lists shrink the chunk
	// so that the lists stay within 16 GB
	if(need_ts > 0) M = std::min(M, std::max<size_t>(65536, ((size_t)16 << 30) / ((size_t)K * 8 * (size_t)need_ts)));
	if(M > d.slots_cap || K > d.nee_cap || need_v0 != d.v0_alloc || need_attr != d.attr_alloc || need_ts != d.ts_alloc || need_g != d.g_alloc || (S.do_ao != 0) != d.ao_alloc ||
	   need_tree != d.tree_alloc)
	{
		// Wavefront buffers for M samples in flight (~0.7 KB each: 288 GB of HBM holds tens of millions,
		// and big chunks amortise the per-launch cost).  On allocation failure the chunk is halved.
		for(;;)
		{
			const size_t MA = R * shardCap(M);   // addresses of the segmented arrays
			for(Buf &b : d.chunk_bufs) b.release();
			d.chunk_bufs.clear();
			auto A = [&](size_t bytes) -> void * {
				d.chunk_bufs.emplace_back();
				Buf &b = d.chunk_bufs.back();
				if(hipMalloc(&b.p, std::max<size_t>(bytes, 16)) != hipSuccess)
				{
					b.p = nullptr;
					(void)hipGetLastError();
					return nullptr;
				}
				b.bytes = bytes;
				return b.p;
			};
			for(int q = 0; q < 2; ++q)
			{
				DevPaths &P = d.P[q];
				P.thr = (float4 *)A(MA * 16);
				P.col = (float4 *)A(need_tree ? MA * 16 : 16);
				P.pcol = (float4 *)A(MA * 16);
				P.pwo = (float4 *)A(MA * 16);
				P.pend_thr = (float4 *)A(MA * 16);
				P.pend_emit = (float4 *)A(MA * 16);
				P.v0p = (float4 *)A(need_v0 ? MA * 16 : 16);      // first-hit data: path_samples > 1 only
				P.v0wo = (float4 *)A(need_v0 ? MA * 16 : 16);
				P.pr = (uint4 *)A(MA * 16);
				P.nee = (float *)A(MA * K * 12);
				P.nee_aw = (float *)A(S.do_ao ? MA * K * 4 : 16);
				P.occ = (uint8_t *)A(MA * K);
				P.v0attr = (float4 *)A(need_v0 && need_attr ? MA * 32 : 16);
				P.ts = (float4 *)A(need_ts ? MA * K * 48 : 16);
			}
			for(int q = 0; q < 2; ++q)
			{
				DevQueues &Q = d.Q[q];
				Q.slot = (int *)A(need_tree ? MA * 4 : 16);
				Q.ray_o = (float *)A(MA * 12);
				Q.ray_d = (float *)A(MA * 12);
				// (tmin, tmax) of the camera / spawned rays: a pass's first iteration, always queue 0
				Q.ray_tt = q == 0 ? (float2 *)A(MA * 8) : nullptr;
				Q.hit_t = (float *)A(MA * 4);
				Q.hit_prim = (int *)A(MA * 4);
				Q.sh_o = (float4 *)A(MA * K * 16);
				Q.sh_d = (float4 *)A(MA * K * 16);
				Q.sh_idx = (int *)A(MA * K * 4);
				Q.sattr = (float4 *)A(need_attr ? MA * 32 : 16);
				Q.ts_hit = (float2 *)A(need_ts ? MA * K * 8 * (size_t)need_ts : 16);
				Q.ts_n = (int *)A(need_ts ? MA * K * 4 : 16);
			}
			// the compact record's first-vertex estimates, by chunk sample id (shared by both state sets)
			d.P[0].csmp = d.P[1].csmp = (float4 *)A(need_tree ? 16 : MA * 16);
			d.N.p_prim = (float4 *)A(16);   // (NEE: the hit point is the next queue's ray origin)
			d.N.wo_k = (float4 *)A(MA * 16);
			d.N.pix_mode = (uint4 *)A(MA * 16);
			d.N.attr = (float4 *)A(need_attr ? MA * 32 : 16);
			d.N.extra = nullptr;
			d.G.p_prim = (float4 *)A(need_g ? MA * 16 : 16);
			d.G.wo_k = (float4 *)A(need_g ? MA * 16 : 16);
			d.G.pix_mode = (uint4 *)A(need_g ? MA * 16 : 16);
			d.G.extra = (float4 *)A(need_g ? MA * 16 : 16);
			d.G.attr = (float4 *)A(need_g && need_attr ? MA * 32 : 16);
			bool ok = true;
			for(const Buf &b : d.chunk_bufs) ok = ok && b.p;
			if(ok) break;
			if(M <= 65536) { log_.error("GPU: out of device memory for the wavefront buffers"); return false; }
			M /= 2;
			log_.warning("GPU: wavefront buffers do not fit, retrying with " + std::to_string(M) + " samples in flight");
		}
		d.v0_alloc = need_v0;
		d.attr_alloc = need_attr;
		d.ts_alloc = need_ts;
		d.g_alloc = need_g;
		d.tree_alloc = need_tree;
		d.ao_alloc = S.do_ao != 0;
		d.slots_cap = M;
		d.nee_cap = K;
	}
	S.n_seg = (uint32_t)R;
	S.cap_a = (uint32_t)shardCap(d.slots_cap);
	S.cap_s = S.cap_a * (uint32_t)K;
	// The two-pass diffuse gather (k_gather_walk + k_gather<REPLAY>, kernels.hip): its log holds `cap`
	// logged photons per request for a batch of
	// seg_cap queue positions per segment (within 16 GB); YAFARAY_AMD_GATHER=single keeps one pass.
	GatherLogDesc glog{nullptr, nullptr, 0u, 0u, 0u, 0u, 0u};
	bool walk_gather = false;
	{
		const char *ge = std::getenv("YAFARAY_AMD_GATHER");
		const bool single = ge && std::string(ge) == "single";
		if(S.gather_on && S.n_photons > 0 && S.pm_search <= yafamd_gather_walk_k() && !single)
		{
			const char *ce = std::getenv("YAFARAY_AMD_GATHER_LOG");
			const uint32_t cap = ((uint32_t)std::max(S.pm_search, ce ? atoi(ce) : 512) + 1u) & ~1u;   // even: pairs
			size_t seg_cap = S.cap_a;
			while((size_t)R * seg_cap * cap * 8 > (16ull << 30) && seg_cap > 64) seg_cap = ((seg_cap / 2 + 63) / 64) * 64;
			if(!ensure(log_, d.g_log, (size_t)R * seg_cap * cap * 8) || !ensure(log_, d.g_log_n, (size_t)R * seg_cap * 4)) return false;
			const char *he = std::getenv("YAFARAY_AMD_GATHER_HEAP");
			const uint32_t split = (he && std::string(he) == "packed") ? 0u : 1u;
			const char *we = std::getenv("YAFARAY_AMD_GATHER_WALK");
			// the walk with the k smallest distances in registers (k <= 64): the bounded walk
			// (YAFARAY_AMD_GATHER_WALK=bound, experiments builds; there also any k > 64) measured slower on C5
			// (walk 13.9 -> 16.3 ms, replay 7.4 -> 12.1 ms per frame: its superset log); without it a larger
			// k takes the one-pass gather (yafamd_gather_walk_k)
			const uint32_t exact = (yafamd_experiments() && we && std::string(we) == "bound") ? 0u : 1u;
			glog = GatherLogDesc{d.g_log.p, (uint32_t *)d.g_log_n.p, cap, (uint32_t)seg_cap, 0u, split, exact, nullptr};
			// the walk's far-child stack levels beyond the LDS ones (tuning builds: -DYAF_WALK_LDS_LEVELS)
			const int lv = yafamd_walk_lds_levels(d.pm_stack), deep = std::max(1, d.pm_stack) - lv;
			if(deep > 0)
			{
				if(!ensure(log_, d.walk_spill, (size_t)deep * yafamd_walk_threads(&S) * 4)) return false;
				glog.spill = (uint32_t *)d.walk_spill.p;
			}
			walk_gather = true;
		}
	}
	// final gathering with one lane per gather path (kernels.hip k_fg_first / k_fg_long / k_fg_sum): its batch
	// buffers, sized for the pass's path count (AA_indirect_sample_multiplier_factor changes it per pass) with
	// room for every path to bounce (no overflow); a batch is seg_cap request positions of every segment,
	// within 6 GB
	const bool fg_paths = yafamd_fg_paths_eligible(&S) != 0;
	// ray binning for the BVH8 refill loop (opt-in experiment, YAFARAY_AMD_RAY_BIN=1): sort keys and the permutation
	bool ray_bin = false;
	if(const char *e = std::getenv("YAFARAY_AMD_RAY_BIN"); e && *e == '1' && S.nodes8 && !S.scene_in_lds && !S.tr_shad && R <= 1024)
	{
		const size_t n = (size_t)R * S.cap_a;
		size_t tb = 0;
		HIPCHECK(yafamd_ray_bin(nullptr, nullptr, (uint32_t)R, S.cap_a, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &tb, d.stream));
		if(!ensure(log_, d.bin_keys, n * 4) || !ensure(log_, d.bin_keys2, n * 4) || !ensure(log_, d.bin_iota, n * 4) || !ensure(log_, d.bin_perm, n * 4) ||
		   !ensure(log_, d.bin_tmp, tb))
			return false;
		ray_bin = true;
	}
	FgBatch fgb{};
	auto fgPrepare = [&]() -> bool {
		const int ns = S.fg_pass_samples > 0 ? S.fg_pass_samples : std::max(1, S.fg_samples);
		const int nt = std::max(0, S.fg_bounces) + 1;
		const size_t per_pos = (size_t)R * (size_t)ns * (16 + 48 + 16 * (size_t)nt);
		size_t cap_max = std::max<size_t>(1, ((size_t)6 << 30) / per_pos);
		if(const char *e = getenv("YAFARAY_AMD_FG_BATCH"); e && atoi(e) > 0) cap_max = std::min(cap_max, (size_t)atoi(e));   // tests: several batches
		const size_t nb = ((size_t)S.cap_a + cap_max - 1) / cap_max;
		const size_t seg_cap = std::max<size_t>(1, ((size_t)S.cap_a + nb - 1) / std::max<size_t>(1, nb));
		const size_t paths = (size_t)R * seg_cap * (size_t)ns;
		if(!ensure(log_, d.fg_terms, paths * 16) || !ensure(log_, d.fg_longs, paths * 48) || !ensure(log_, d.fg_long_terms, paths * 16 * (size_t)nt) ||
		   !ensure(log_, d.fg_long_count, (size_t)R * 4))
			return false;
		fgb = FgBatch{0u, (uint32_t)seg_cap, ns, nt, (float4 *)d.fg_terms.p, (float4 *)d.fg_longs.p, (float4 *)d.fg_long_terms.p,
		              (uint32_t *)d.fg_long_count.p, (uint32_t)(seg_cap * (size_t)ns)};
		return true;
	};
	if(!ensure(log_, d.counters, 2 * 4 * R * sizeof(uint32_t))) return false;
	if(!ensure(log_, d.stats, sizeof(DevStats) * (size_t)d.trace_grid)) return false;
	HIPCHECK(hipMemsetAsync(d.counters.p, 0, 2 * 4 * R * sizeof(uint32_t), d.stream));
	HIPCHECK(hipMemsetAsync(d.stats.p, 0, sizeof(DevStats) * (size_t)d.trace_grid, d.stream));
	DevCounters cnt[2];
	for(int q = 0; q < 2; ++q)
	{
		uint32_t *base_q = (uint32_t *)d.counters.p + (size_t)q * 4 * R;
		cnt[q].n_active = base_q;
		cnt[q].n_shadow = base_q + R;
		cnt[q].n_nee = base_q + 2 * R;
		cnt[q].n_gather = base_q + 3 * R;
	}
	DevStats *dstats = (DevStats *)d.stats.p;
	S.stats = dstats;
	// Opt-in YAFARAY_AMD_NEE_TRACE=1: k_nee traces its shadow rays in place for LDS-resident scenes
	// (kernels.hip k_nee<.., TR>) when the whole stack bound fits LDS.  Measured on C2: k_trace
	// 26.9 -> 18.2 ms per frame but k_nee 15.1 -> 29.4 ms (the traversal at k_nee's 4 waves / SIMD
	// instead of k_trace's 8), frame 72.6 -> 79.0 ms — so the shadow rays stay queued for k_trace.
	int nee_trace_stack = 0;
	{
		const char *ne = std::getenv("YAFARAY_AMD_NEE_TRACE");
		if(yafamd_experiments() && ne && std::string(ne) == "1" && d.lds_stack >= d.stack_depth) nee_trace_stack = d.lds_stack;
	}
	// The megakernel (k_path, kernels.hip; opt-in YAFARAY_AMD_PATH=mega) for scenes whose BVH, stack
	// and tables live in LDS and need none of the wavefront-only stages (EXT shading, transparent
	// shadows, photon maps, AO): one lane per sample, the same functions in the same order, the film
	// bit-identical.  Measured on C2: 124 ms per frame at its best occupancy vs 73 ms for the wavefront
	//  — so the wavefront stays the default.
	// estimateOneDirectLight with several lights (path tracing) picks its light from the one-thread
	// render's running counter: every pass runs a count run first (lpcBases).  A specular recursion tree
	// (several integrate() nodes per sample) and caller-side shards (no exchange of the other rows'
	// counts) keep pickLight; YAFARAY_AMD_LIGHT_PICK=hash forces it.
	bool lpc_on = S.integrator == INT_PATH && S.n_lights > 1 && !S.tree && (rp.shard_world <= 1 || group_render);
	if(const char *lp = std::getenv("YAFARAY_AMD_LIGHT_PICK"); lp && std::string(lp) == "hash") lpc_on = false;
	lpc_carry_ = 0;
	S.lpc = nullptr;
	S.lpc_mode = 0;
	S.nee_pm16 = 0;
	if(const char *e = std::getenv("YAFARAY_AMD_NEE_PM16"); e && *e == '1') S.nee_pm16 = 1;   // tests: the 16-B request word
	if(const char *e = std::getenv("YAFARAY_AMD_W_LIVE"); e && *e == '1') S.w_live = 1;        // tests: the 16-B throughput record
	S.no_lean = 0;
	S.fg_probe = 0;
	if(const char *e = std::getenv("YAFARAY_AMD_FG_PROBE"); e && *e) S.fg_probe = atoi(e);   // timing attribution only
	if(const char *e = std::getenv("YAFARAY_AMD_SHADE_LEAN"); e && *e == '0') S.no_lean = 1;   // tests: the general k_shade
	int path_grid = 0;
	if(!lpc_on)
	{
		const char *pe = std::getenv("YAFARAY_AMD_PATH");
		const bool on = yafamd_experiments() && pe && std::string(pe) == "mega";
		if(on && yafamd_path_eligible(&S, d.lds_stack, d.lds_stack < d.stack_depth ? 1 : 0))
		{
			path_grid = std::min(d.trace_grid, d.n_cu * std::max(1, yafamd_path_blocks_per_cu(&S, d.lds_stack)));
			if(const char *e = getenv("YAFARAY_AMD_PATH_GRID")) path_grid = std::min(d.trace_grid, std::max(1, atoi(e)));
			if(!ensure(log_, d.path_next, 16)) return false;
		}
	}
	const int n_paths = std::max(1, S.path_samples);
	const int iters = (S.integrator == INT_PATH) ? 2 + n_paths * (S.bounces + 2) : 3;

	// ---- events ----
	auto ensureEvents = [&](size_t need) -> bool {
		while(d.ev_pool.size() < need)
		{
			hipEvent_t e;
			HIPCHECK(hipEventCreate(&e));
			d.ev_pool.push_back(e);
		}
		return true;
	};
	if(!ensureEvents(2)) return false;
	HIPCHECK(hipEventRecord(d.ev_pool[0], d.stream));
	// one pass: `n_total` camera samples (the jobs' enumeration, or S.plist x S.spp) through the wavefront
	// one wavefront pass over the active list started by k_camera / k_spawn
	DevStats *run_stats = dstats;   // the light-pick count runs count into their own statistics
	auto iterate = [&](uint64_t base) -> bool {
		int cur = 0;
		// a light-pick count run (S.lpc_mode 1) follows the paths only: no estimates, no shadow rays
		const bool count_run = S.lpc_mode == 1;
		for(int it = 0; it < iters; ++it)
		{
			// the first iteration's closest rays (camera / spawned, queue 0) carry their own (tmin, tmax);
			// k_shade's bounce rays all have (ray_min_dist, infinite)
			DevQueues qc = d.Q[cur];
			// (camera rays with the default clip planes all have (0, unbounded): k_camera writes no ray_tt)
			if(it != 0 || (S.cur_level == 0 && !S.cam.ray_tt)) qc.ray_tt = nullptr;
			qc.tmin_dflt = it == 0 ? 0.f : S.ray_min_dist;
			qc.perm = nullptr;
			if(ray_bin && it >= 1 && !count_run)
			{
				// the bounce rays ordered by direction octant + origin (camera rays are coherent already)
				size_t tb = d.bin_tmp.bytes;
				HIPCHECK(yafamd_ray_bin(&qc, &cnt[cur], S.n_seg, S.cap_a, d.scene_lo, d.scene_hi, (uint32_t *)d.bin_keys.p, (uint32_t *)d.bin_keys2.p,
				                        (uint32_t *)d.bin_iota.p, (uint32_t *)d.bin_perm.p, d.bin_tmp.p, &tb, d.stream));
				qc.perm = (const uint32_t *)d.bin_perm.p;
			}
			PROF(KK_TRACE, yafamd_launch_trace(&S, &qc, &cnt[cur], &d.P[cur], run_stats, d.lds_stack, (int *)d.spill.p,
			                                    S.tr_shad ? d.trace_grid_bvh4 : d.trace_grid, d.stream));
			// material-shade dispatch for textured / smooth scenes: surface attributes + shader nodes
			// of every hit, before k_shade reads them
			// transparent shadows: filter colours of the transparent surfaces the shadow rays crossed
			if(S.tr_shad && !count_run) PROF(KK_TSHADOW, yafamd_launch_tshadow(&S, &qc, &cnt[cur], &d.P[cur], d.stream));
			if(S.has_attr) PROF(KK_SURFACE, yafamd_launch_surface(&S, &qc, &cnt[cur], d.stream));
			// the deferred light pick's record slots of this iteration (one per active entry)
			if(S.lpc_mode == 3)
				HIPCHECK(yafamd_dfr_segoff(&cnt[cur], S.n_seg, (uint32_t *)d.dfr_segoff.p, (uint32_t *)d.dfr_misc.p, S.dfr_cap,
				                           (uint32_t *)d.dfr_misc.p + 1, (uint32_t *)d.dfr_its.p, d.stream));
			PROF(KK_SHADE, yafamd_launch_shade(&S, &d.P[cur], &d.P[cur ^ 1], &qc, &d.Q[cur ^ 1], &d.N, &d.G, &cnt[cur], &cnt[cur ^ 1],
			                             (float4 *)d.samples.p, (const DevJob *)d.jobs.p, n_jobs, base, d.stream));

			// photon-map estimates of the finished diffuse first hits: the direct-lighting pipeline
			// (photon mapping, DirectLight) connects its NEE in iteration 1 and finishes there; path
			// tracing finishes paths in any iteration
			const bool dl_pipeline = S.integrator != INT_PATH;
			// (show_map: the camera hits finish in iteration 0, with their nearest-photon requests)
			if(S.gather_on && !count_run && (!dl_pipeline || it == 1 || (S.show_map && it == 0)))
			{
				// final gathering adds its estimate to the requests' colour before k_gather ends them
				if(S.fg_on && fg_paths)
				{
					if(!fgPrepare()) return false;
					// one lane per gather path, in batches of request positions (every segment's [j0, j0 + seg_cap))
					for(uint32_t j0 = 0; j0 < S.cap_a; j0 += fgb.seg_cap)
					{
						FgBatch B = fgb;
						B.j0 = j0;
						HIPCHECK(hipMemsetAsync(fgb.long_count, 0, (size_t)S.n_seg * 4, d.stream));
						PROF(KK_FG, yafamd_launch_fg_paths(&S, &d.G, &cnt[cur ^ 1], d.lds_stack, (int *)d.spill.p, d.trace_grid, &B, d.stream));
					}
				}
				else if(S.fg_on)
					PROF(KK_FG, yafamd_launch_fg(&S, &d.G, &cnt[cur ^ 1], d.lds_stack, (int *)d.spill.p, d.trace_grid, (float2 *)d.fg_ts.p, d.stream));
				if(walk_gather)
					for(uint32_t j0 = 0; j0 < S.cap_a; j0 += glog.seg_cap)
					{
						GatherLogDesc L = glog;
						L.j0 = j0;
						PROF(KK_GATHER_WALK, yafamd_launch_gather_walk(&S, &d.G, &cnt[cur ^ 1], &L, d.stream));
						PROF(KK_GATHER, yafamd_launch_gather(&S, &d.G, &cnt[cur ^ 1], (float4 *)d.samples.p, (const DevJob *)d.jobs.p, n_jobs, base,
						                                     &L, d.stream));
					}
				else
					PROF(KK_GATHER, yafamd_launch_gather(&S, &d.G, &cnt[cur ^ 1], (float4 *)d.samples.p, (const DevJob *)d.jobs.p, n_jobs, base,
					                                     nullptr, d.stream));
			}
			// NEE requests (none in iteration 1 of photon mapping, whose entries all finish there)
			if(!yafamd_shade_fused_for(&S) && !(S.integrator == INT_PHOTON && it == 1) && !count_run)
				PROF(KK_NEE, yafamd_launch_nee(&S, &d.N, &d.P[cur ^ 1], &d.Q[cur ^ 1], &cnt[cur ^ 1], nee_trace_stack, d.stream));
			// (non-EXT k_shade runs the NEE itself: FUSED)
			cur ^= 1;
		}
		return true;
	};
	bool tree_overflow_logged = false;
	// one pass: `n_total` camera samples (the jobs' enumeration, or S.plist x S.spp) through the wavefront;
	// `done` = samples of the chunks that ran (< n_total only when the render was canceled)
	uint64_t done = 0;
	auto runSamples = [&](uint64_t n_total) -> bool {
	done = 0;
	for(uint64_t base = 0; base < n_total; base += M, done = std::min(base, n_total))
	{
		if(canceled && *canceled) break;
		const int n = (int)std::min<uint64_t>(M, n_total - base);
		if(rp.on_chunk && base > 0)
		{
			HIPCHECK(hipStreamSynchronize(d.stream));
			rp.on_chunk(base, n_total);
			if(canceled && *canceled) break;
		}
		if(path_grid > 0)
		{
			HIPCHECK(hipMemsetAsync(d.path_next.p, 0, 4, d.stream));
			PROF(KK_PATH, yafamd_launch_path(&S, (float4 *)d.samples.p, (const DevJob *)d.jobs.p, n_jobs, base, (uint32_t)n, (uint32_t *)d.path_next.p,
			                                 d.lds_stack, path_grid, d.stream));
			continue;
		}
		if(S.tree) HIPCHECK(hipMemsetAsync(d.spawn_count.p, 0, 16, d.stream));
		S.cur_level = 0;
		PROF(KK_CAMERA, yafamd_launch_camera(&S, &d.P[0], &d.Q[0], &cnt[0], (const DevJob *)d.jobs.p, n_jobs, base, n, d.stream));
		if(!iterate(base)) return false;
		if(!S.tree) continue;
		// recursiveRaytrace levels: the nodes the last pass spawned are the next pass's active list
		std::vector<std::pair<uint32_t, uint32_t>> levels;
		uint32_t done = 0;
		for(int level = 1;; ++level)
		{
			uint32_t hc[2] = {0, 0};
			HIPCHECK(hipMemcpyAsync(hc, d.spawn_count.p, 8, hipMemcpyDeviceToHost, d.stream));
			HIPCHECK(hipStreamSynchronize(d.stream));
			if(hc[1] && !tree_overflow_logged)
			{
				log_.error("Integrator: the specular recursion tree exceeded its " + std::to_string(S.spawn_cap) + " node records; deeper rays dropped");
				tree_overflow_logged = true;
			}
			const uint32_t total_spawned = std::min(hc[0], S.spawn_cap);
			if(total_spawned <= done) break;
			S.cur_level = level;
			for(uint32_t sub = done; sub < total_spawned; sub += (uint32_t)M)
			{
				const int nn = (int)std::min<uint64_t>(M, total_spawned - sub);
				PROF(KK_SPAWN, yafamd_launch_spawn(&S, &d.P[0], &d.Q[0], &cnt[0], sub, nn, d.stream));
				if(!iterate(base)) return false;
			}
			levels.push_back({done, total_spawned});
			done = total_spawned;
		}
		for(size_t k = levels.size(); k-- > 0;)
			PROF(KK_COMBINE, yafamd_launch_combine(&S, S.node_base + levels[k].first, S.node_base + levels[k].second, 0, nullptr, nullptr, 0, 0, d.stream));
		PROF(KK_COMBINE, yafamd_launch_combine(&S, 0, (uint32_t)n, 1, (float4 *)d.samples.p, (const DevJob *)d.jobs.p, n_jobs, base, d.stream));
		S.cur_level = 0;
	}
	return true;
	};
	// one pass's samples; with the one-thread light pick a count run first (the paths only: closest
	// rays and shading, no estimates), then the counters' bases (lpcBases), then the render proper
	int jy0 = H, jy1 = 0;
	for(const DevJob &j : jobs)
	{
		jy0 = std::min(jy0, j.y0);
		jy1 = std::max(jy1, j.y1);
	}
	auto runPass = [&](uint64_t n_total, int pass_spp) -> bool {
		if(!lpc_on) return runSamples(n_total);
		const size_t n_ctr = (size_t)W * H * (size_t)pass_spp;
		// one 4-B counter per camera sample of the pass (8.5 GB at 1080p x 1024 spp): above a budget of a
		// quarter of the device's free memory, or when the allocation fails, the pass falls back to the
		// hashed pick (matched statistically) instead of failing the render
		{
			size_t free_b = 0, total_b = 0;
			const bool have = hipMemGetInfo(&free_b, &total_b) == hipSuccess;
			bool fits = d.lpc.bytes >= n_ctr * 4 || (have && n_ctr * 4 <= (free_b + d.lpc.bytes) / 4);
			if(const char *e = std::getenv("YAFARAY_AMD_LPC_MAX_MB"); e && *e) fits = fits && (n_ctr * 4 >> 20) < (size_t)std::max(0, atoi(e));
			auto tryEnsure = [](Buf &b, size_t bytes) {
				if(b.p && b.bytes >= bytes) return true;
				b.release();
				if(hipMalloc(&b.p, std::max<size_t>(bytes, 16)) != hipSuccess)
				{
					b.p = nullptr;
					(void)hipGetLastError();
					return false;
				}
				b.bytes = std::max<size_t>(bytes, 16);
				return true;
			};
			bool can = fits && tryEnsure(d.lpc, n_ctr * 4) && tryEnsure(d.lpc_stats, sizeof(DevStats) * (size_t)d.trace_grid);
			if(group_render)
			{
				// every member takes the same pick (the count run's bases are exchanged): fall back together
				const int st = groupStatus(can ? 0 : 1);
				if(st >= 2)
				{
					log_.error("GPU group: a member failed; render abandoned");
					return false;
				}
				can = st == 0;
			}
			if(!can)
			{
				log_.warning("Integrator: the one-thread light-pick counters (" + std::to_string(n_ctr * 4 >> 20) +
				             " MB) exceed the memory budget; this pass picks lights by sample hash");
				return runSamples(n_total);
			}
		}
		// the deferred pick (r06): the pass once with every addition to a path colour kept as a record, the
		// lights picked from the counters' bases afterwards, the records folded in order — no count run.  A
		// group render (collective bases) and scenes it does not serve keep the count run; so does a pass whose
		// records overflow their budget (a third of the free memory), rendered again below
		if(!group_render && yafamd_dfr_eligible(&S))
		{
			size_t free_b = 0, total_b = 0;
			(void)hipMemGetInfo(&free_b, &total_b);
			const size_t want = n_ctr * (size_t)(S.bounces + 2) * (size_t)std::max(1, S.path_samples);
			size_t cap = std::min<size_t>(want, (free_b / 3) / 76);
			cap = std::min<size_t>(cap, 0x7ffffff0u);
			if(const char *e = std::getenv("YAFARAY_AMD_DFR_CAP"); e && atoi(e) > 0) cap = std::min<size_t>(cap, (size_t)atoi(e));   // tests: the overflow
			bool ok_mem = cap > 0 && ensure(log_, d.dfr_kind, cap * 4) && ensure(log_, d.dfr_pp, cap * 16) && ensure(log_, d.dfr_wo, cap * 16) &&
			              ensure(log_, d.dfr_a, cap * 16) && ensure(log_, d.dfr_emit, cap * 16) && ensure(log_, d.dfr_pix, cap * 8) &&
			              ensure(log_, d.dfr_last, n_ctr * 4) &&
			              ensure(log_, d.dfr_segoff, (size_t)S.n_seg * 4) && ensure(log_, d.dfr_misc, 16) && ensure(log_, d.dfr_its, 4096 * 4) &&
			              ensure(log_, d.dfr_pcol, n_ctr * 16) && ensure(log_, d.dfr_idx, (size_t)S.n_seg * S.cap_a * 4) &&
			              ensure(log_, d.dfr_nrec, (size_t)S.n_seg * 4);
			if(ok_mem)
			{
				HIPCHECK(hipMemsetAsync(d.lpc.p, 0, n_ctr * 4, d.stream));
				HIPCHECK(hipMemsetAsync(d.dfr_last.p, 0xff, n_ctr * 4, d.stream));
				HIPCHECK(hipMemsetAsync(d.dfr_misc.p, 0, 16, d.stream));
				HIPCHECK(hipMemsetAsync(d.dfr_its.p, 0, 4, d.stream));
				HIPCHECK(hipMemsetAsync(d.dfr_pcol.p, 0, n_ctr * 16, d.stream));
				S.lpc = (uint32_t *)d.lpc.p;
				S.dfr_kind = (uint32_t *)d.dfr_kind.p;
				S.dfr_pp = (float4 *)d.dfr_pp.p;
				S.dfr_wo = (float4 *)d.dfr_wo.p;
				S.dfr_a = (float4 *)d.dfr_a.p;
				S.dfr_emit = (float4 *)d.dfr_emit.p;
				S.dfr_pix = (uint2 *)d.dfr_pix.p;
				S.dfr_last = (uint32_t *)d.dfr_last.p;
				S.dfr_seg_off = (const uint32_t *)d.dfr_segoff.p;
				S.dfr_cap = (uint32_t)cap;
				S.lpc_mode = 3;
				const bool ok = runSamples(n_total);
				S.lpc_mode = 0;
				if(!ok) return false;
				uint32_t misc[2] = {0u, 0u};
				std::vector<uint32_t> its(4096, 0u);
				HIPCHECK(hipMemcpyAsync(misc, d.dfr_misc.p, 8, hipMemcpyDeviceToHost, d.stream));
				HIPCHECK(hipMemcpyAsync(its.data(), d.dfr_its.p, its.size() * 4, hipMemcpyDeviceToHost, d.stream));
				HIPCHECK(hipStreamSynchronize(d.stream));
				if(its[0] > 4095u) misc[1] = 1u;   // more iterations than recorded starts: the count run serves
				if(!misc[1])
				{
					bool cut = done < n_total;
					if(!lpcBases(rp, pass_spp, jy0, jy1, group_render, cut)) return false;
					if(cut)
					{
						done = 0;   // canceled before the pass rendered anything
						return true;
					}
					const uint32_t total_slots = misc[0];
					const uint32_t batch = S.n_seg * S.cap_a;
					for(uint32_t r0 = 0; r0 < total_slots; r0 += batch)
					{
						PROF(KK_DFR, yafamd_dfr_nee(&S, &d.P[0], &d.Q[0], &cnt[0], r0, total_slots, (uint32_t *)d.dfr_idx.p, (uint32_t *)d.dfr_nrec.p,
						                            d.stream));
						DevQueues qs = d.Q[0];
						qs.ray_tt = nullptr;
						qs.perm = nullptr;
						qs.tmin_dflt = S.ray_min_dist;
						PROF(KK_TRACE, yafamd_launch_trace(&S, &qs, &cnt[0], &d.P[0], run_stats, d.lds_stack, (int *)d.spill.p, d.trace_grid, d.stream));
						// every sample's terms of this batch, iteration range by iteration range (one record per sample and
						// iteration; the ranges increase with the slots, so the additions keep the one-pass order)
						const uint32_t r1 = std::min<uint64_t>((uint64_t)r0 + batch, total_slots);
						for(uint32_t k = 0; k < its[0]; ++k)
						{
							const uint32_t a = std::max(its[1 + k], r0), b = std::min((k + 1 < its[0]) ? its[2 + k] : total_slots, r1);
							if(b > a) PROF(KK_DFR, yafamd_dfr_accum(&S, &d.P[0], a, b, r0, (float4 *)d.dfr_pcol.p, d.stream));
						}
					}
					PROF(KK_DFR, yafamd_dfr_fold(&S, (float4 *)d.samples.p, (uint32_t)n_ctr, (const float4 *)d.dfr_pcol.p, d.stream));
					return true;
				}
				log_.info("Integrator: the deferred light pick's records exceed their budget (" + std::to_string(cap) +
				          " slots); the pass renders again with a count run");
			}
		}
		HIPCHECK(hipMemsetAsync(d.lpc.p, 0, n_ctr * 4, d.stream));
		HIPCHECK(hipMemsetAsync(d.lpc_stats.p, 0, sizeof(DevStats) * (size_t)d.trace_grid, d.stream));
		S.lpc = (uint32_t *)d.lpc.p;
		S.lpc_mode = 1;
		S.stats = (DevStats *)d.lpc_stats.p;
		run_stats = S.stats;
		auto on_chunk = rp.on_chunk;
		rp.on_chunk = nullptr;   // progress is reported by the render proper
		const bool ok = runSamples(n_total);
		rp.on_chunk = on_chunk;
		S.stats = dstats;
		run_stats = dstats;
		S.lpc_mode = 0;
		if(!ok) return false;
		bool cut = done < n_total;
		if(!lpcBases(rp, pass_spp, jy0, jy1, group_render, cut)) return false;
		if(cut)
		{
			done = 0;   // canceled before the pass rendered anything
			return true;
		}
		S.lpc_mode = 2;
		const bool ok2 = runSamples(n_total);
		S.lpc_mode = 0;
		return ok2;
	};

	// ---- pass 0 (every pixel), then the adaptive passes (TiledIntegrator::render, integrator_tiled.cc:172-231) ----
	const int passes = std::max(1, rp.aa.passes);
	S.aa_multipass = passes > 1 ? 1 : 0;
	S.pass_offset = 0;
	S.plist = nullptr;
	rp.film.multipass = S.aa_multipass;
	rp.film.sample_offset = S.base_offset;
	rp.film.ntx = (W + ts - 1) / ts;
	rp.film.tile_rank = nullptr;
	rp.film.partial = 0;
	if(!rp.tile_rank.empty())
	{
		if(!allocCopy(log_, d.tile_rank, rp.tile_rank.data(), rp.tile_rank.size())) return false;
		rp.film.tile_rank = (const uint32_t *)d.tile_rank.p;
	}
	// per-tile callbacks: the partial film of a pass (before its film launch adds to the accumulators)
	const bool tiles_cb = (bool)rp.on_tiles && rp.shard_world == 1 && groupWorld() <= 1;
	auto emitTiles = [&](int pass, const uint8_t *flags, int accumulate) -> bool {
		if(!tiles_cb) return true;
		if(!ensure(log_, d.pfilm, (size_t)W * H * sizeof(float4))) return false;
		DevFilm Fp = rp.film;
		Fp.partial = 1;
		PROF(KK_FILM, yafamd_launch_film(&Fp, (const float4 *)d.samples.p, flags, (float4 *)d.accum.p, (float4 *)d.pfilm.p, (float *)d.weights.p, 0, H,
		                            S.clamp_samples, accumulate, d.stream));
		std::vector<float> host((size_t)W * H * 4);
		HIPCHECK(hipMemcpyAsync(host.data(), d.pfilm.p, host.size() * sizeof(float), hipMemcpyDeviceToHost, d.stream));
		HIPCHECK(hipStreamSynchronize(d.stream));
		rp.on_tiles(pass, host);
		return true;
	};
	uint64_t samples_total = total;
	if(rp.resumed)
	{
		// renderPass(0, sampling_offset): no samples; the loaded film is only normalised
		DevFilm F0 = rp.film;
		F0.spp = 0;
		for(const auto &r : owned_rows_)
			PROF(KK_FILM, yafamd_launch_film(&F0, (const float4 *)d.samples.p, nullptr, (float4 *)d.accum.p, (float4 *)d.film.p,
			                            (float *)d.weights.p, r.first, r.second, S.clamp_samples, 1, d.stream));
		samples_total = 0;
		sampling_offset_ = rp.resume_sampling_offset;
	}
	else
	{
		if(!runPass(total, spp)) return false;
		const uint8_t *done_flags = nullptr;
		if(done < total)
		{
			// canceled: only the pixels of the completed chunks splat (the others were never rendered)
			if(!ensure(log_, d.aa_flags, (size_t)W * H)) return false;
			HIPCHECK(hipMemsetAsync(d.aa_flags.p, 0, (size_t)W * H, d.stream));
			HIPCHECK(yafamd_launch_done_flags(&S, (const DevJob *)d.jobs.p, n_jobs, (uint32_t)(total / (uint64_t)spp), (uint32_t)(done / (uint64_t)spp),
			                                  (uint8_t *)d.aa_flags.p, d.stream));
			done_flags = (const uint8_t *)d.aa_flags.p;
			samples_total = done / (uint64_t)spp * (uint64_t)spp;
		}
		if(done == total && !emitTiles(0, nullptr, 0)) return false;
		for(const auto &r : owned_rows_)
			PROF(KK_FILM, yafamd_launch_film(&rp.film, (const float4 *)d.samples.p, done_flags, (float4 *)d.accum.p, (float4 *)d.film.p,
			                            (float *)d.weights.p, r.first, r.second, S.clamp_samples, 0, d.stream));
		// renderPass sets the sampling offset before its workers start (integrator_tiled.cc:244), so a
		// canceled pass advances it too
		sampling_offset_ = (uint32_t)spp;
	}
	passes_done_ = 1;
	if(passes > 1)
	{
		if(!ensure(log_, d.aa_flags, (size_t)W * H) || !ensure(log_, d.aa_plist, (size_t)W * H * 4)) return false;
		float threshold = rp.aa.threshold, sample_multiplier = 1.f, light_multiplier = 1.f, indirect_multiplier = 1.f;
		bool threshold_changed = true;
		int acum = spp, resampled = 0;
		int resampled_local = 0;   // of them in this member's rows (+ halo rows): the pixels it renders
		const int floor_pixels = (int)floorf(rp.aa.resampled_floor * (float)(W * H) / 100.f);
		for(int pass = 1; pass < passes; ++pass)
		{
			if(group_render && fault_pass_ == pass)
			{
				log_.error("GPU group: injected failure of member " + std::to_string(rp.shard_rank) + " at pass " + std::to_string(pass + 1));
				return false;
			}
			if(group_render)
			{
				// every member's film of the last pass is complete: agree on going on (a member that was
				// canceled or failed stops everyone here), then every member assembles the whole accumulated
				// film — nextPass compares pixels with their neighbours across band boundaries
				HIPCHECK(hipStreamSynchronize(d.stream));
				const int st = groupStatus((canceled && *canceled) ? 1 : 0);
				if(st >= 2)
				{
					log_.error("GPU group: a member failed; render abandoned");
					return false;
				}
				if(st == 1) break;
				if(!exchangeRows(rp.band_bounds, XR_ACCUM, true)) return false;
			}
			else if(canceled && *canceled) break;
			sample_multiplier *= rp.aa.sample_multiplier_factor;
			light_multiplier *= rp.aa.light_sample_multiplier_factor;
			indirect_multiplier *= rp.aa.indirect_sample_multiplier_factor;
			S.fg_pass_samples = (int)ceilf((float)std::max(1, S.fg_samples) * indirect_multiplier);
			if(light_mult)
			{
				HIPCHECK(hipStreamSynchronize(d.stream));   // the previous pass's staging copy is consumed
				lightLayout(light_multiplier, d.pass_lights);
				HIPCHECK(hipMemcpyAsync(d.lights.p, d.pass_lights.data(), d.pass_lights.size() * sizeof(DevLight), hipMemcpyHostToDevice,
				                        d.stream));
			}
			const bool skip = resampled <= 0.f && !threshold_changed;
			if(rp.on_next_pass)
			{
				HIPCHECK(hipStreamSynchronize(d.stream));
				rp.on_next_pass(skip);
			}
			if(skip) {}   // nextPass(..., skipNextPass = true)
			else
			{
				// the flags of the whole film; the pixel list restricted to the rows whose samples this
				// member's film rows gather (its band + halo rows)
				uint32_t count = 0, local = 0;
				int ry0 = 0, ry1 = H;
				if(group_render)
				{
					ry0 = std::max(0, rp.shard_y0 - rp.film.reach_fwd);
					ry1 = std::min(H, rp.shard_y1 + rp.film.reach_back);
				}
				PROF(KK_AA, yafamd_aa_next_pass((const float4 *)d.accum.p, (const float *)d.weights.p, W, H, ts, &rp.aa.dev, threshold,
				                             (uint8_t *)d.aa_flags.p, (uint32_t *)d.aa_plist.p, &count, ry0, ry1, &local, d.stream));
				resampled = (int)count;
				resampled_local = (int)local;
				threshold_changed = false;
				if(const char *dump = getenv("YAFARAY_AMD_AA_DUMP"); dump && *dump)
				{
					// diagnostics: the pass's flags as W*H bytes
					std::vector<uint8_t> hf((size_t)W * H);
					HIPCHECK(hipMemcpy(hf.data(), d.aa_flags.p, hf.size(), hipMemcpyDeviceToHost));
					if(FILE *f = fopen((std::string(dump) + "_pass" + std::to_string(pass) + ".bin").c_str(), "wb"))
					{
						fwrite(hf.data(), 1, hf.size(), f);
						fclose(f);
					}
				}
			}
			const int n_pass = (int)ceilf(rp.aa.inc_samples * sample_multiplier);
			{
				std::ostringstream os;
				os << "Rendering pass " << pass + 1 << " of " << passes << ", resampling " << resampled << " pixels x " << n_pass << " samples.";
				log_.info(os.str());
			}
			if(resampled > 0 && n_pass > 0)
			{
				if(!ensure(log_, d.samples, (size_t)W * H * n_pass * sizeof(float4))) return false;
				S.spp = n_pass;
				S.pass_offset = (uint32_t)acum;
				S.plist = (const uint32_t *)d.aa_plist.p;
				rp.film.spp = n_pass;
				rp.film.sample_offset = S.base_offset + (uint32_t)acum;
				const uint64_t n_total = (uint64_t)resampled_local * (uint64_t)n_pass;
				if(!runPass(n_total, n_pass)) return false;
				if(done < n_total)
					HIPCHECK(yafamd_launch_done_flags(&S, (const DevJob *)d.jobs.p, n_jobs, (uint32_t)resampled_local, (uint32_t)(done / (uint64_t)n_pass),
					                                  (uint8_t *)d.aa_flags.p, d.stream));
				if(done == n_total && !emitTiles(passes_done_, (const uint8_t *)d.aa_flags.p, 1)) return false;
				for(const auto &r : owned_rows_)
					PROF(KK_FILM, yafamd_launch_film(&rp.film, (const float4 *)d.samples.p, (const uint8_t *)d.aa_flags.p, (float4 *)d.accum.p,
					                            (float4 *)d.film.p, (float *)d.weights.p, r.first, r.second, S.clamp_samples, 1, d.stream));
				samples_total += done / (uint64_t)n_pass * (uint64_t)n_pass;
				sampling_offset_ = (uint32_t)(acum + n_pass);   // renderPass: setSamplingOffset(offset + samples), :244
				if(done < n_total)
				{
					// canceled mid-pass; a group member stops at the next status agreement, with the others
					if(group_render)
					{
						acum += n_pass;
						continue;
					}
					break;
				}
				++passes_done_;
			}
			acum += n_pass;
			if(resampled < floor_pixels)
			{
				const float ratio = std::min(8.f, ((float)floor_pixels / resampled));
				threshold *= (1.f - 0.1f * ratio);
				if(threshold > 0.f) threshold_changed = true;
			}
		}
		S.spp = spp;
		S.pass_offset = 0;
		S.plist = nullptr;
		S.fg_pass_samples = 0;
		rp.film.spp = spp;
		if(light_mult)
		{
			HIPCHECK(hipStreamSynchronize(d.stream));
			lightLayout(1.f, d.pass_lights);
			HIPCHECK(hipMemcpy(d.lights.p, d.pass_lights.data(), d.pass_lights.size() * sizeof(DevLight), hipMemcpyHostToDevice));
		}
	}
	HIPCHECK(hipEventRecord(d.ev_pool[1], d.stream));
	HIPCHECK(hipStreamSynchronize(d.stream));
	float ms = 0.f;
	HIPCHECK(hipEventElapsedTime(&ms, d.ev_pool[0], d.ev_pool[1]));
	DevStats hs{};
	{
		std::vector<DevStats> per_block((size_t)d.trace_grid);
		HIPCHECK(hipMemcpy(per_block.data(), d.stats.p, sizeof(DevStats) * per_block.size(), hipMemcpyDeviceToHost));
		for(const DevStats &b : per_block)
		{
			hs.closest_rays += b.closest_rays;
			hs.shadow_rays += b.shadow_rays;
			hs.node_visits += b.node_visits;
			hs.tri_tests += b.tri_tests;
			hs.shade_entries += b.shade_entries;
			hs.nee_requests += b.nee_requests;
			hs.gather_queries += b.gather_queries;
			hs.gather_visits += b.gather_visits;
			hs.gather_photons += b.gather_photons;
			hs.gather_accepts += b.gather_accepts;
			hs.gather_overflows += b.gather_overflows;
			hs.fg_paths += b.fg_paths;
			hs.fg_lookups += b.fg_lookups;
			hs.fg_nearest_visits += b.fg_nearest_visits;
		}
		if(d.pre_stats_valid)
		{
			DevStats pre{};
			HIPCHECK(hipMemcpy(&pre, d.pre_stats.p, sizeof(DevStats), hipMemcpyDeviceToHost));
			hs.pre_visits = pre.pre_visits;
			hs.pre_photons = pre.pre_photons;
			d.pre_stats_valid = false;   // counted once: a reused radiance map is not pre-gathered again
		}
	}
	stats_.closest_rays = hs.closest_rays;
	stats_.shadow_rays = hs.shadow_rays;
	stats_.node_visits = hs.node_visits;
	stats_.tri_tests = hs.tri_tests;
	stats_.samples = samples_total;
	stats_.render_seconds = ms * 1e-3;
	stats_.trace_kernel_ms = 0.0;
	stats_.shade_kernel_ms = 0.0;
	stats_.nee_kernel_ms = 0.0;
	stats_.trace_launches = 0;
	if(rp.profile)
	{
		for(const Impl::ProfRec &pr : d.prof_recs)
		{
			float t = 0.f;
			HIPCHECK(hipEventElapsedTime(&t, d.ev_pool[pr.e0], d.ev_pool[pr.e1]));
			ktimes_.ms[pr.kind] += t;
			++ktimes_.launches[pr.kind];
		}
		ktimes_.items[KK_CAMERA] = samples_total;
		ktimes_.items[KK_FILM] = samples_total;
		ktimes_.items[KK_TRACE] = hs.closest_rays + hs.shadow_rays;
		ktimes_.items[KK_PATH] = ktimes_.launches[KK_PATH] ? samples_total : 0;
		ktimes_.items[KK_SHADE] = hs.shade_entries;
		ktimes_.items[KK_NEE] = hs.nee_requests;
		ktimes_.items[KK_GATHER] = hs.gather_queries;
		ktimes_.items[KK_GATHER_WALK] = ktimes_.launches[KK_GATHER_WALK] ? hs.gather_queries : 0;
		ktimes_.items[KK_FG] = S.fg_on ? hs.gather_queries : 0;   // every diffuse-map request runs its final gathering first
		ktimes_.items[KK_PREGATHER] = (uint64_t)d.n_rphotons;
		ktimes_.items[KK_PHOTON_EMIT] = (uint64_t)d.pm_local;
		ktimes_.items[KK_PHOTON_BOUNCE] = stats_.photon_paths_traced;
		ktimes_.items[KK_PHOTON_COMPACT] = ktimes_.items[KK_PHOTON_TREE] = stats_.photons;
		stats_.trace_kernel_ms = ktimes_.ms[KK_TRACE];
		stats_.shade_kernel_ms = ktimes_.ms[KK_SHADE];
		stats_.nee_kernel_ms = ktimes_.ms[KK_NEE] + ktimes_.ms[KK_GATHER] + ktimes_.ms[KK_GATHER_WALK];
		stats_.trace_launches = ktimes_.launches[KK_TRACE];
	}
	stats_.gather_visits = hs.gather_visits;
	stats_.gather_photons = hs.gather_photons;
	stats_.gather_queries = hs.gather_queries;
	stats_.gather_accepts = hs.gather_accepts;
	stats_.gather_overflows = hs.gather_overflows;
	stats_.fg_paths = hs.fg_paths;
	stats_.fg_lookups = hs.fg_lookups;
	stats_.fg_nearest_visits = hs.fg_nearest_visits;
	stats_.pregather_visits = hs.pre_visits;
	stats_.pregather_photons = hs.pre_photons;
	d.prof_on = false;
	return true;
}

// a 64-B header records how the block was obtained (1: hipHostMalloc, 0: malloc when pinning failed,
// e.g. without a device), so that pinnedFree releases it the same way
void *yafamd::pinnedAlloc(size_t bytes)
{
	const size_t n = bytes + 64;
	void *p = nullptr;
	uint32_t tag = 1;
	if(hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess || !p)
	{
		(void)hipGetLastError();
		p = std::malloc(n);
		tag = 0;
		if(!p) return nullptr;
	}
	std::memcpy(p, &tag, sizeof(tag));
	return static_cast<char *>(p) + 64;
}

void yafamd::pinnedFree(void *q)
{
	if(!q) return;
	void *p = static_cast<char *>(q) - 64;
	uint32_t tag = 0;
	std::memcpy(&tag, p, sizeof(tag));
	if(tag == 1) (void)hipHostFree(p);
	else std::free(p);
}

bool GpuRenderer::download(PinnedFloats &rgba, PinnedFloats &weights, int w, int h, bool with_rgba, bool with_weights)
{
	DeviceGuard guard(device_);
	Impl &d = *d_;
	if(!d.film.p || w != d.film_w || h != d.film_h) { log_.error("GPU: no film to download"); return false; }
	// the buffers keep their size across frames (no re-allocation, no re-pinning after the first)
	if(rgba.size() != (size_t)w * h * 4) rgba.resize((size_t)w * h * 4);
	if(weights.size() != (size_t)w * h) weights.resize((size_t)w * h);
	if(with_rgba) HIPCHECK(hipMemcpyAsync(rgba.data(), d.film.p, rgba.size() * 4, hipMemcpyDeviceToHost, d.stream));
	if(with_weights) HIPCHECK(hipMemcpyAsync(weights.data(), d.weights.p, weights.size() * 4, hipMemcpyDeviceToHost, d.stream));
	HIPCHECK(hipStreamSynchronize(d.stream));
	return true;
}

bool GpuRenderer::downloadAccum(std::vector<float> &rgba, std::vector<float> &weights)
{
	DeviceGuard guard(device_);
	Impl &d = *d_;
	if(!d.accum.p || !d.weights.p) { log_.error("GPU: no film to download"); return false; }
	rgba.resize((size_t)d.film_w * d.film_h * 4);
	weights.resize((size_t)d.film_w * d.film_h);
	HIPCHECK(hipStreamSynchronize(d.stream));
	HIPCHECK(hipMemcpy(rgba.data(), d.accum.p, rgba.size() * 4, hipMemcpyDeviceToHost));
	HIPCHECK(hipMemcpy(weights.data(), d.weights.p, weights.size() * 4, hipMemcpyDeviceToHost));
	return true;
}

bool GpuRenderer::filmToDevice(void *dst, int y0, int y1)
{
	DeviceGuard guard(device_);
	Impl &d = *d_;
	if(!d.film.p || y0 < 0 || y1 > d.film_h || y1 < y0) { log_.error("GPU: bad film row range"); return false; }
	const size_t row = (size_t)d.film_w * sizeof(float4);
	HIPCHECK(hipMemcpy(dst, (char *)d.film.p + row * y0, row * (y1 - y0), hipMemcpyDeviceToDevice));
	return true;
}

bool GpuRenderer::traceRays(bool any, const float *rays, int n, float *t, int *prim)
{
	if(!ready()) return false;
	DeviceGuard guard(device_);
	Impl &d = *d_;
	if(!d.nodes.p) { log_.error("GPU: no acceleration structure built"); return false; }
	std::vector<float> o((size_t)n * 4), dd((size_t)n * 4);
	for(int i = 0; i < n; ++i)
	{
		const float *r = rays + 8 * (size_t)i;
		o[4 * i] = r[0]; o[4 * i + 1] = r[1]; o[4 * i + 2] = r[2]; o[4 * i + 3] = r[6];
		dd[4 * i] = r[3]; dd[4 * i + 1] = r[4]; dd[4 * i + 2] = r[5]; dd[4 * i + 3] = r[7];
	}
	Buf bo, bd, bt, bp;
	bool ok = allocCopy(log_, bo, o.data(), o.size()) && allocCopy(log_, bd, dd.data(), dd.size()) &&
	          ensure(log_, bt, (size_t)n * 4) && ensure(log_, bp, (size_t)n * 4);
	if(ok)
	{
		DevScene S{};
		fillScenePointers(d, S);
		ok = yafamd_launch_trace_rays(&S, any ? 1 : 0, (const float4 *)bo.p, (const float4 *)bd.p, n, (float *)bt.p, (int *)bp.p,
		                              d.stack_depth, d.stream) == hipSuccess &&
		     hipStreamSynchronize(d.stream) == hipSuccess;
		if(!ok) log_.error("GPU: trace launch failed");
		if(ok && t) ok = hipMemcpy(t, bt.p, (size_t)n * 4, hipMemcpyDeviceToHost) == hipSuccess;
		if(ok && prim) ok = hipMemcpy(prim, bp.p, (size_t)n * 4, hipMemcpyDeviceToHost) == hipSuccess;
	}
	bo.release();
	bd.release();
	bt.release();
	bp.release();
	return ok;
}

// ---------------------------------------------------------------------------------------------
// render group
// ---------------------------------------------------------------------------------------------

bool GpuRenderer::joinGroup(int rank, int world, const void *rccl_id, size_t id_bytes)
{
	if(!ready()) return false;
	DeviceGuard guard(device_);
	Impl &d = *d_;
	if(d.comm)
	{
		(void)ncclCommDestroy(d.comm);
		d.comm = nullptr;
	}
	group_rank_ = 0;
	group_world_ = 1;
	if(world <= 1) return true;
	if(rank < 0 || rank >= world || !rccl_id || id_bytes < sizeof(ncclUniqueId))
	{
		log_.error("GPU group: bad rank / world / id");
		return false;
	}
	ncclUniqueId id;
	std::memcpy(&id, rccl_id, sizeof(id));
	NCCLCHECK(ncclCommInitRank(&d.comm, world, id, rank));
	group_rank_ = rank;
	group_world_ = world;
	std::ostringstream os;
	os << "GPU group: member " << rank << " of " << world << " (RCCL)";
	log_.info(os.str());
	return true;
}

int PeerGroup::arrive(int status)
{
	std::unique_lock<std::mutex> lk(mtx_);
	cur_max_ = std::max(cur_max_, status);
	if(++count_ == (int)members_.size())
	{
		last_max_ = cur_max_;
		cur_max_ = 0;
		count_ = 0;
		++gen_;
		cv_.notify_all();
		return last_max_;
	}
	const int g = gen_;
	cv_.wait(lk, [&] { return gen_ != g; });
	// last_max_ stays valid: the next generation cannot complete before this member arrives again
	return last_max_;
}

int GpuRenderer::groupStatus(int mine)
{
	Impl &d = *d_;
	int st = mine;
	if(peers_ && peers_->size() > 1) st = peers_->arrive(mine);
	else if(d.comm)
	{
		DeviceGuard guard(device_);
		// the maximum over the members (RCCL all-reduce of one int)
		if(!ensure(log_, d.g_status, 16)) st = 2;
		else
		{
			int out = 2;
			const bool ok = hipMemcpyAsync(d.g_status.p, &mine, sizeof(int), hipMemcpyHostToDevice, d.stream) == hipSuccess &&
			                ncclAllReduce(d.g_status.p, (char *)d.g_status.p + 4, 1, ncclInt32, ncclMax, d.comm, d.stream) == ncclSuccess &&
			                hipMemcpyAsync(&out, (char *)d.g_status.p + 4, sizeof(int), hipMemcpyDeviceToHost, d.stream) == hipSuccess &&
			                hipStreamSynchronize(d.stream) == hipSuccess;
			st = ok ? out : 2;
			if(!ok) log_.error("GPU group: status all-reduce failed");
		}
	}
	if(st >= 2) failure_seen_ = true;
	return st;
}

void GpuRenderer::groupAbort()
{
	if(!failure_seen_ && grouped()) (void)groupStatus(2);
	failure_seen_ = true;
}

bool GpuRenderer::exchangeRows(const std::vector<int> &bounds, int what, bool to_all)
{
	Impl &d = *d_;
	DeviceGuard guard(device_);
	const int W = d.film_w, H = d.film_h;
	const bool peer_mode = peers_ && peers_->size() > 1;
	const int world = peer_mode ? peers_->size() : group_world_;
	const int me = peer_mode ? peer_rank_ : group_rank_;
	if(world <= 1) return true;
	if((int)bounds.size() != world + 1 || bounds.front() != 0 || bounds.back() != H)
	{
		log_.error("GPU group: band bounds do not cover the film");
		return false;
	}
	const size_t row4 = (size_t)W * sizeof(float4), row1 = (size_t)W * sizeof(float);
	HIPCHECK(hipStreamSynchronize(d.stream));
	if(peer_mode)
	{
		// every member's buffers are final when all have arrived; the receivers pull the other bands
		// (hipMemcpyPeer: xGMI between GPUs, a device copy between logical members of one GPU), and
		// nobody touches its buffers again before the second arrival
		peers_->arrive(0);
		bool ok = true;
		if(to_all || me == 0)
			for(int r = 0; r < world && ok; ++r)
			{
				const int a = bounds[r], b = bounds[r + 1];
				if(r == me || b <= a) continue;
				GpuRenderer *src = peers_->member(r);
				Impl &o = *src->d_;
				auto pull = [&](void *dst, const void *sp, size_t row) {
					return hipMemcpyPeerAsync((char *)dst + row * a, device_, (const char *)sp + row * a, src->device_, row * (b - a), d.stream) == hipSuccess;
				};
				if(what & XR_FILM) ok = ok && pull(d.film.p, o.film.p, row4);
				if(what & XR_ACCUM) ok = ok && pull(d.accum.p, o.accum.p, row4);
				if(what & (XR_FILM | XR_ACCUM)) ok = ok && pull(d.weights.p, o.weights.p, row1);
			}
		ok = ok && hipStreamSynchronize(d.stream) == hipSuccess;
		if(!ok) log_.error("GPU group: band copy between members failed");
		if(what & XR_TIMES)
		{
			member_ms_.assign((size_t)world, 0.0);
			for(int r = 0; r < world; ++r) member_ms_[r] = peers_->member(r)->stats_.render_seconds * 1e3;
		}
		peers_->arrive(0);
		if(ok && (to_all || me == 0)) owned_rows_.assign(1, {0, H});
		return ok;
	}
	// RCCL: all-gather fixed-size band slots (bandPack / bandUnpack's plan) and scatter them into the film
	const size_t band_px = (size_t)bandSlotRows(bounds) * W;
	if(!ensure(log_, d.g_send, band_px * sizeof(float4)) || !ensure(log_, d.g_recv, band_px * world * sizeof(float4)) ||
	   !ensure(log_, d.g_wsend, band_px * sizeof(float)) || !ensure(log_, d.g_wrecv, band_px * world * sizeof(float)) ||
	   !ensure(log_, d.g_times, 2 * (size_t)world * sizeof(double)))
		return false;
	const int y0 = bounds[me], y1 = bounds[me + 1];
	const int kinds[2] = {XR_FILM, XR_ACCUM};
	for(int kind : kinds)
	{
		if(!(what & kind)) continue;
		void *src4 = kind == XR_FILM ? d.film.p : d.accum.p;
		if(y1 > y0)
		{
			HIPCHECK(hipMemcpyAsync(d.g_send.p, (char *)src4 + row4 * y0, row4 * (y1 - y0), hipMemcpyDeviceToDevice, d.stream));
			HIPCHECK(hipMemcpyAsync(d.g_wsend.p, (char *)d.weights.p + row1 * y0, row1 * (y1 - y0), hipMemcpyDeviceToDevice, d.stream));
		}
		NCCLCHECK(ncclGroupStart());
		NCCLCHECK(ncclAllGather(d.g_send.p, d.g_recv.p, band_px * 4, ncclFloat32, d.comm, d.stream));
		NCCLCHECK(ncclAllGather(d.g_wsend.p, d.g_wrecv.p, band_px, ncclFloat32, d.comm, d.stream));
		NCCLCHECK(ncclGroupEnd());
		for(int r = 0; r < world; ++r)
		{
			const int a = bounds[r], b = bounds[r + 1];
			if(b <= a || r == me) continue;
			HIPCHECK(hipMemcpyAsync((char *)src4 + row4 * a, (char *)d.g_recv.p + (size_t)r * band_px * sizeof(float4), row4 * (b - a),
			                        hipMemcpyDeviceToDevice, d.stream));
			HIPCHECK(hipMemcpyAsync((char *)d.weights.p + row1 * a, (char *)d.g_wrecv.p + (size_t)r * band_px * sizeof(float), row1 * (b - a),
			                        hipMemcpyDeviceToDevice, d.stream));
		}
	}
	if(what & XR_TIMES)
	{
		double *times = (double *)d.g_times.p;
		const double mine = stats_.render_seconds * 1e3;
		HIPCHECK(hipMemcpyAsync(times, &mine, sizeof(double), hipMemcpyHostToDevice, d.stream));
		NCCLCHECK(ncclAllGather(times, times + world, 1, ncclFloat64, d.comm, d.stream));
		member_ms_.assign((size_t)world, 0.0);
		HIPCHECK(hipMemcpyAsync(member_ms_.data(), times + world, sizeof(double) * world, hipMemcpyDeviceToHost, d.stream));
	}
	HIPCHECK(hipStreamSynchronize(d.stream));
	owned_rows_.assign(1, {0, H});
	return true;
}

bool GpuRenderer::renderMember(RenderParams &rp, volatile bool *canceled)
{
	failure_seen_ = false;
	member_ms_.clear();
	// YAFARAY_AMD_FAULT_MEMBER=m[:p] (tests of the failure protocol): member m fails before rendering
	// (p = 0, default), at the start of adaptive pass p + 1, or (p = "concat") after the members
	// exchanged their photon-map counts, before the maps are concatenated
	fault_pass_ = -1;
	fault_concat_ = false;
	if(const char *e = getenv("YAFARAY_AMD_FAULT_MEMBER"); e && *e && atoi(e) == rp.shard_rank)
	{
		const char *c = std::strchr(e, ':');
		fault_concat_ = c && std::strcmp(c + 1, "concat") == 0;
		fault_pass_ = fault_concat_ ? -1 : c ? atoi(c + 1) : 0;
		if(fault_pass_ == 0)
		{
			log_.error("GPU group: injected failure of member " + std::to_string(rp.shard_rank) + " before rendering");
			groupAbort();
			return false;
		}
	}
	if(!render(rp, canceled))
	{
		groupAbort();
		return false;
	}
	// the final status agreement: a failed member stops everyone, a canceled one still combines (the
	// partial film, as a canceled one-GPU render)
	const int st = groupStatus(0);
	if(st >= 2)
	{
		log_.error("GPU group: a member failed; render abandoned");
		return false;
	}
	const int what = XR_FILM | XR_TIMES | (rp.combine_accum ? XR_ACCUM : 0);
	if(!exchangeRows(rp.band_bounds, what, rp.combine_all))
	{
		failure_seen_ = true;   // the exchange itself failed: no further agreement can be trusted
		return false;
	}
	return true;
}

namespace yafamd
{

int bandSlotRows(const std::vector<int> &bounds)
{
	int rows = 1;
	for(size_t r = 0; r + 1 < bounds.size(); ++r) rows = std::max(rows, bounds[r + 1] - bounds[r]);
	return rows;
}

static bool bandsValid(const std::vector<int> &bounds, int H, int rank)
{
	const int world = (int)bounds.size() - 1;
	if(world < 1 || rank < 0 || rank >= world || bounds.front() != 0 || bounds.back() != H) return false;
	for(int r = 0; r < world; ++r)
		if(bounds[r + 1] < bounds[r]) return false;
	return true;
}

bool bandPack(const float *film, int W, int H, int ch, const std::vector<int> &bounds, int rank, float *send)
{
	if(!film || !send || W < 1 || ch < 1 || !bandsValid(bounds, H, rank)) return false;
	const size_t row = (size_t)W * ch;
	const int y0 = bounds[rank], y1 = bounds[rank + 1];
	std::memset(send, 0, (size_t)bandSlotRows(bounds) * row * sizeof(float));
	std::memcpy(send, film + row * y0, (size_t)(y1 - y0) * row * sizeof(float));
	return true;
}

bool bandUnpack(const float *recv, int W, int H, int ch, const std::vector<int> &bounds, int rank, float *film)
{
	if(!film || !recv || W < 1 || ch < 1 || !bandsValid(bounds, H, rank)) return false;
	const size_t row = (size_t)W * ch, slot = (size_t)bandSlotRows(bounds) * row;
	for(int r = 0; r + 1 < (int)bounds.size(); ++r)
	{
		const int a = bounds[r], b = bounds[r + 1];
		if(r == rank || b <= a) continue;
		std::memcpy(film + row * a, recv + slot * r, (size_t)(b - a) * row * sizeof(float));
	}
	return true;
}

std::vector<int> equalBands(int height, int world)
{
	std::vector<int> b((size_t)world + 1);
	for(int r = 0; r <= world; ++r) b[r] = (int)((int64_t)height * r / world);
	return b;
}

std::vector<int> rebalanceBands(const std::vector<int> &bounds, const std::vector<double> &times, int cap_rows, double damping)
{
	const int world = (int)bounds.size() - 1;
	const int H = bounds.back();
	if(world <= 1 || H < world || (int)times.size() < world) return bounds;
	std::vector<double> cum((size_t)H + 1, 0.0);
	{
		std::vector<double> dens((size_t)H, 0.0);
		for(int r = 0; r < world; ++r)
		{
			const int rows = bounds[r + 1] - bounds[r];
			if(rows > 0)
				for(int y = bounds[r]; y < bounds[r + 1]; ++y) dens[y] = std::max(times[r], 1e-9) / rows;
		}
		for(int y = 0; y < H; ++y) cum[y + 1] = cum[y] + dens[y];
	}
	std::vector<int> nb(1, 0);
	for(int r = 1; r < world; ++r)
	{
		const double target = cum[H] * r / world;
		int y = (int)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
		if(y > 0 && y <= H && (cum[y] - target) > (target - cum[y - 1])) --y;
		y = (int)std::nearbyint(damping * bounds[r] + (1.0 - damping) * y);   // round half to even, as Python's round()
		nb.push_back(y);
	}
	nb.push_back(H);
	for(int r = 1; r < world; ++r) nb[r] = std::min(std::max(nb[r], nb[r - 1] + 1), H - (world - r));
	if(cap_rows > 0)
		for(int r = 0; r < world; ++r)
			if(nb[r + 1] - nb[r] > cap_rows) return bounds;
	return nb;
}

} // namespace yafamd
