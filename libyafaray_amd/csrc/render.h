// GPU driver of the hot path: uploads the scene in the devscene.h layouts, runs the wavefront
// pipeline of kernels.hip chunk by chunk on one HIP stream, and gathers the film.
//
// Replaces TiledIntegrator::render / renderPass / renderWorker / renderTile
// (src/integrator/surface/integrator_tiled.cc:50-408): instead of `threads` CPU workers pulling
// 32x32 tiles from an atomic counter, the whole tile list is one enumeration of camera samples
// (tile order preserved) processed `chunk_slots` samples at a time by the GPU.
#pragma once

#include "bvh.h"
#include "devscene.h"
#include "host.h"

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace yafamd
{


struct HostScene
{
	BvhOutput bvh;                       // host build (nodes + triangle records), or metadata of the GPU build
	bool gpu_build = false;              // build the BVH4 on the device from verts / tris (bvhgpu.hip)
	std::vector<float> verts;            // xyz per vertex   (gpu_build only)
	std::vector<int> tris;               // 3 indices per triangle (gpu_build only)
	int ploc_iters = 0;                  // PLOC iterations of the GPU build
	std::vector<float> prim_ng;          // 4 floats per primitive
	std::vector<DevMaterial> mats;
	std::vector<DevLight> lights;        // the visible lights by name (the integrators' order), then the photon-only ones
	std::vector<int> light_name_order;   // every light by name (the photon maps' light lists, render_view.cc:93-111)
	std::vector<float> mesh_tris;        // meshlight faces: kMeshTriF4 float4 each (DevScene::mesh_tris)
	std::vector<float> mesh_cdf;         // their area distributions' normalised cdf, per light
	std::vector<float> mesh_nodes;       // each meshlight's BVH2 over its faces (16 floats per node)
	std::vector<float> mesh_btris;       // ... and its triangle records in leaf order (12 floats each)
	int n_prims = 0;
	// surface attributes / textures / shader nodes (texeval.h), only when has_attr
	bool has_attr = false;
	std::vector<float> prim_attr;        // kAttrF4 float4 per primitive
	std::vector<DevNode> shader_nodes;
	std::vector<DevTexture> textures;
	std::vector<float> texels;           // RGBA per texel
};

struct PhotonParams
{
	int photons = 0;           // diffuse photons to shoot (0: no diffuse map)
	int caustic_photons = 0;   // caustic photons to shoot
	bool caustic_map = false;  // build the caustic map and add causticPhotons() at diffuse hits
	int caustic_search = 50;   // "caustic_mix"
	float caustic_radius = 0.25f;
	int caustic_depth = 10;
	int search = 50;           // k of the k-NN gather
	float radius2 = 0.1f;      // "diffuseRadius" (squared radius of the gather)
	int bounces = 5;
	int threads = -1;          // threads_photons: photon count rounded to a multiple (:437); <= 0 -> 1
	// final gathering (integrator_photon_mapping.cc factory :777-810)
	bool final_gather = false;
	int fg_samples = 32;
	int fg_bounces = 2;
	float fg_min_pathlen = 0.1f;   // gather_dist_ (default diffuseRadius)
	// photon_maps_processing (integrator_photon_mapping.cc:844-847, integrator_path_tracer.cc:360-363)
	int processing = PM_GENERATE;  // in: the integrator's mode; out: the mode the render used after fallbacks
	bool diffuse_map = false;      // PhotonIntegrator "diffuse" (use_photon_diffuse_)
	std::string map_path;          // film_load_save_path: <path>_diffuse / _caustic / _fg_radiance.photonmap
	uint64_t owner = 0;            // the integrator instance the maps belong to ("reuse-previous")
	bool write_files = true;       // this member writes the files (member 0 of a group)
	enum : int { PM_GENERATE = 0, PM_GENERATE_SAVE = 1, PM_LOAD = 2, PM_REUSE = 3 };
};

// adaptive anti-aliasing (scene.cc:582-595, aa_noise_params.h:27-46; TiledIntegrator::render,
// integrator_tiled.cc:172-231)
struct AaParams
{
	int passes = 1;
	int inc_samples = 1;               // AA_inc_samples (defaults to AA_minsamples)
	float light_sample_multiplier_factor = 1.f;   // AA_light_sample_multiplier_factor (integrator_tiled.cc:190)
	float indirect_sample_multiplier_factor = 1.f;   // AA_indirect_sample_multiplier_factor (:191; final gathering's path count)
	float threshold = 0.05f;
	float resampled_floor = 0.f;       // % of the pixels
	float sample_multiplier_factor = 1.f;
	DevAaParams dev{0, 0, 0.f, 10, 0};
};

// Kernel kinds timed by the profile mode (HIP events around every launch on the render stream)
enum KernelKind : int
{
	KK_CAMERA = 0, KK_TRACE, KK_SURFACE, KK_TSHADOW, KK_SHADE, KK_NEE, KK_GATHER, KK_SPAWN, KK_COMBINE, KK_FILM, KK_AA,
	KK_PHOTON_EMIT, KK_PHOTON_BOUNCE, KK_PHOTON_COMPACT, KK_PHOTON_TREE, KK_FG, KK_PREGATHER, KK_GATHER_WALK, KK_PATH, KK_DFR, KK_COUNT
};
inline const char *kernelKindName(int k)
{
	static const char *n[KK_COUNT] = {"k_camera", "k_trace", "k_surface", "k_tshadow", "k_shade", "k_nee", "k_gather", "k_spawn",
	                                  "k_combine", "k_film", "aa_next_pass", "k_photon_emit", "k_photon_bounce", "photon_compact",
	                                  "pkd_build", "k_fg", "k_pregather", "k_gather_walk", "k_path", "k_dfr"};
	return (k >= 0 && k < KK_COUNT) ? n[k] : "";
}
struct KernelTimes
{
	double ms[KK_COUNT] = {};
	uint64_t launches[KK_COUNT] = {};
	uint64_t items[KK_COUNT] = {};   // work units: samples (camera, film), rays (trace), entries (shade),
	                                 // requests (nee), queries (gather), photon paths (emit, bounce), photons (tree)
};

struct RenderParams
{
	DevScene scene;                      // pointers filled by the renderer
	PhotonParams pm;
	AaParams aa;
	DevFilm film;
	int shard_rank = 0, shard_world = 1;
	int shard_mode = 1;   // 0: tile rows r % world == rank, 1: contiguous row band [H rank / world, H (rank + 1) / world),
	                      // 2: the explicit band [shard_y0, shard_y1) (host-side load balancing)
	int shard_y0 = 0, shard_y1 = 0;
	int chunk_slots = 1 << 27;   // samples in flight per wavefront chunk (134 M: the C2 frame in one chunk)
	bool profile = false;
	// film load/save (filmio.h): accumulators loaded from film files, uploaded before the first pass;
	// resumed = the first pass renders no samples (integrator_tiled.cc:174-177)
	const float *load_rgba = nullptr, *load_weights = nullptr;
	bool resumed = false;
	uint32_t resume_sampling_offset = 0;   // the loaded films' sampling offset (max over the files)
	// ImageFilm::nextPass hook (imagefilm.cc:259-287), called before every adaptive pass with
	// skipped = the pass's nextPass was skipped; the film autosave lives there
	std::function<void(bool skipped)> on_next_pass;
	// progress hook after every completed chunk (the reference's per-tile progress updates,
	// integrator_tiled.cc:258-262): samples done / samples of the pass.  Set -> one stream sync per chunk.
	std::function<void(uint64_t done, uint64_t total)> on_chunk;
	// tile order (ImageSplitter): rank of every tile id ty * ntx + tx; empty = linear
	std::vector<uint32_t> tile_rank;
	// per-pass hook for the per-tile callbacks (ImageFilm::finishArea, imagefilm.cc:489-568): the
	// pass's partial film (RGBA, W x H) — each pixel as the one-thread render shows it when its tile
	// finishes.  Single GPU, uncanceled passes.
	std::function<void(int pass, const std::vector<float> &partial)> on_tiles;
	// Group render (the film split into contiguous row bands over the members of a device group or
	// a render group, GpuRenderer::renderMember): the members' band boundaries (world + 1 rows; this
	// member is shard_rank).  Empty: not a group render.  Between adaptive passes the members agree
	// on their status and exchange the accumulated film rows (nextPass reads neighbouring pixels).
	std::vector<int> band_bounds;
	// final combine: every member receives the whole film (render group: each process owns a film)
	// or only member 0 (device group: the scene's film lives on member 0)
	bool combine_all = true;
	// final combine also carries the unnormalised accumulators (film files are saved from them)
	bool combine_accum = false;
};

class GpuRenderer;

// Device group: the member renderers of ONE process (one per GPU, or several logical members on one
// GPU for rehearsals) rendering one film.  Each member runs on its own host thread; they meet at
// arrive(), a barrier that also agrees on a status (0 ok, 1 canceled, 2 failed: the maximum over the
// members), and copy band rows from each other's device buffers (hipMemcpyPeer over xGMI) while
// every member waits inside the exchange.
class PeerGroup
{
	public:
		explicit PeerGroup(std::vector<GpuRenderer *> members) : members_(std::move(members)) {}
		int size() const { return (int)members_.size(); }
		GpuRenderer *member(int m) const { return members_[(size_t)m]; }
		int arrive(int status);

	private:
		std::vector<GpuRenderer *> members_;
		std::mutex mtx_;
		std::condition_variable cv_;
		int count_ = 0, gen_ = 0, cur_max_ = 0, last_max_ = 0;
};

class GpuRenderer
{
	public:
		// device: the HIP device of this renderer (-1: the calling thread's current device at first use).
		// Every public method makes it current for its duration (and restores the caller's device).
		explicit GpuRenderer(Logger &log, int device = -1);
		~GpuRenderer();
		bool ready();
		int device() const { return device_; }
		static int deviceCount();
		static int currentDevice();
		static void enablePeerAccess(const std::vector<int> &devices);
		bool upload(HostScene &hs);   // fills hs.bvh's metadata when the BVH is built on the device
		bool render(RenderParams &rp, volatile bool *canceled);
		int lastPassCount() const { return passes_done_; }
		uint32_t samplingOffset() const { return sampling_offset_; }   // ImageFilm::sampling_offset_ after the last pass
		bool downloadAccum(std::vector<float> &rgba, std::vector<float> &weights);   // unnormalised film (film files)   // AA passes rendered by the last render()
		// one stream sync, DMA into pinned memory; either part can be skipped
		bool download(PinnedFloats &rgba, PinnedFloats &weights, int w, int h, bool with_rgba = true, bool with_weights = true);
		bool filmToDevice(void *dst, int y0, int y1);
		bool traceRays(bool any, const float *rays, int n, float *t, int *prim);
		bool buildPhotonMap(RenderParams &rp);
		bool buildRadianceMap(RenderParams &rp);
		bool shootMap(RenderParams &rp, const PhotonSet &L, uint32_t N, int bounces, int which, uint32_t &n_out, int &depth_out);
		// photon map files / maps kept from the previous render (photon_maps_processing); which: 0
		// diffuse, 1 caustic, 2 radiance map
		bool loadMap(RenderParams &rp, int which, const std::string &file);
		bool saveMap(RenderParams &rp, int which, const std::string &file);
		bool buildMapTree(int which, const void *pos, const void *dir, const void *colb, uint32_t n, void *nodes, int &depth, bool group_split = false);
		bool exchangeTree(int which, uint32_t n, void *nodes, int D, int members);
		const void *mapView(int which, int field, const void *photon_order) const;
		void publishRadianceMap(DevScene &S, const PhotonParams &pm, uint32_t nk);

		// ---- render group: the film split into contiguous row bands over several GPUs ----
		// One member per GPU (one process per GPU, each calling joinGroup with the same RCCL id).
		// After a member rendered its band (RenderParams shard_mode 2), groupCombine all-gathers every
		// member's band rows (normalised RGBA + weights) and render time over RCCL into this member's
		// film, so every member ends with the whole frame; the band boundaries for the next frame
		// come from rebalanceBands over the gathered times.  imagesplitter.cc:30-107 partitions the
		// reference's film into tiles for threads; imagefilm.cc:997-1008 sums film files of nodes.
		bool joinGroup(int rank, int world, const void *rccl_id, size_t id_bytes);
		int groupRank() const { return group_rank_; }
		int groupWorld() const { return group_world_; }
		// device group membership (one process): member `m` of `g` (null: none)
		void setPeers(std::shared_ptr<PeerGroup> g, int m) { peers_ = std::move(g); peer_rank_ = m; }
		bool grouped() const { return (d_comm() != nullptr) || (peers_ && peers_->size() > 1); }
		// Render this member's band (rp.band_bounds, rp.shard_rank) and combine the bands: render() +
		// the final status agreement + the band exchange; on failure the member still takes part in
		// the next status agreement (with "failed") so that no member waits for it forever.
		bool renderMember(RenderParams &rp, volatile bool *canceled);
		// the members' render times (ms) of the last group render, in member order
		const std::vector<double> &memberMs() const { return member_ms_; }
		// Status agreement (every member calls it at the same point): the maximum of the members'
		// statuses (0 ok, 1 canceled, 2 failed); a transport error counts as failed.
		int groupStatus(int mine);
		// Tell the others this member failed, unless a failure was already agreed on.
		void groupAbort();
		enum : int { XR_FILM = 1, XR_ACCUM = 2, XR_TIMES = 4 };
		// Copy every other member's band rows of the chosen buffers into this member (to_all: every
		// member receives; else member 0 only).  XR_FILM: normalised film + weights, XR_ACCUM:
		// accumulators + weights, XR_TIMES: the members' render times (memberMs).
		bool exchangeRows(const std::vector<int> &bounds, int what, bool to_all);
		const yafaray_amd_stats_t &stats() const { return stats_; }
		const KernelTimes &kernelTimes() const { return ktimes_; }
		std::vector<std::pair<int, int>> ownedRows() const { return owned_rows_; }

		struct Impl;

	private:
		void *d_comm() const;
		bool groupCounts(uint32_t mine, std::vector<uint32_t> &all);
		bool groupConcat(int kind, const std::vector<uint32_t> &counts);
		uint32_t seg_count_ = 0;   // this member's photon-map segment count (read by the peers)
		// estimateOneDirectLight's one-thread counter: bases of a pass's samples from its count run
		bool lpcBases(RenderParams &rp, int spp, int jy0, int jy1, bool group_render, bool &cut);
		std::vector<uint32_t> lpc_seg_host_;   // this member's row-segment call counts (read by the peers)
		uint32_t lpc_carry_ = 0;               // calls of the render's earlier passes
		Impl *d_;
		Logger &log_;
		int device_ = -1;
		std::shared_ptr<PeerGroup> peers_;
		int peer_rank_ = 0;
		bool failure_seen_ = false;   // a group status agreement of this render returned "failed"
		int fault_pass_ = -1;         // failure injection (tests of the group protocol): fail at this pass
		bool fault_concat_ = false;   // ... or between the photon-map counts and their concatenation
		std::vector<double> member_ms_;
		yafaray_amd_stats_t stats_{};
		KernelTimes ktimes_{};
		std::vector<std::pair<int, int>> owned_rows_;
		int passes_done_ = 0;
		int group_rank_ = 0, group_world_ = 1;
		uint32_t sampling_offset_ = 0;
};

// Band boundaries (world + 1 rows) moved towards equal cost from each band's last render time:
// each band's time is spread evenly over its rows (piecewise-constant cost density), boundaries
// move towards the equal-cost split (damping: the fraction of the old boundary kept; 0.5 half way, 0 all
// the way), every band keeps >= 1 row; a result with a band above cap_rows rows (0: no cap) keeps the old
// bounds.  Pure and deterministic, so every group member computes the same bounds from the same gathered
// times (tests/tiles.py mirrors it).
std::vector<int> rebalanceBands(const std::vector<int> &bounds, const std::vector<double> &times, int cap_rows, double damping = 0.5);
std::vector<int> equalBands(int height, int world);

// The render group's band exchange plan (GpuRenderer::exchangeRows does it with device copies and an
// RCCL all-gather; the host twins below let tests run the same plan over gloo): member r sends its
// rows [bounds[r], bounds[r + 1]) in a slot of bandSlotRows() rows (zero-padded), the all-gather
// concatenates the slots in member order, every member copies the other members' rows back into
// its film.  ch = floats per pixel (4: RGBA, 1: weights).
int bandSlotRows(const std::vector<int> &bounds);
bool bandPack(const float *film, int W, int H, int ch, const std::vector<int> &bounds, int rank, float *send);
bool bandUnpack(const float *recv, int W, int H, int ch, const std::vector<int> &bounds, int rank, float *film);

} // namespace yafamd
