/*
 * yafaray_amd.h — MI355X extensions next to the drop-in ABI (yafaray_c_api.h).
 *
 * These entry points are additive (version node LIBYAFARAY_AMD_1.0): a reference client never
 * needs them.  They expose what a GPU host wants beyond the reference's per-pixel callbacks:
 *
 *  - bulk geometry upload (one call per object instead of one per vertex / triangle);
 *  - the batched ray-level seam that replaces the reference's per-ray const virtuals
 *    Accelerator::intersect / Accelerator::isShadowed (reference include/accelerator/accelerator.h:53-69,
 *    src/accelerator/accelerator.cc:55-78): SoA rays in, hits out, on the GPU BVH;
 *  - the rendered film (normalised RGBA + weights) as arrays, the in-kernel ray / node / triangle
 *    counters and per-phase timings the bench reports;
 *  - multi-GPU: render only a subset of tile rows (one process per GPU; the tile results are then
 *    all-gathered over RCCL by the caller).
 *
 * All pointers are plain host pointers unless a name says `_dev` (HIP device pointers, e.g. from
 * torch tensors on the same device).  Errors are reported the reference's way (logger + return 0).
 */
#ifndef YAFARAY_AMD_H
#define YAFARAY_AMD_H

#include "yafaray_c_api.h"
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct
{
	uint64_t closest_rays;      /* closest-hit queries issued to the BVH */
	uint64_t shadow_rays;       /* any-hit (shadow) queries */
	uint64_t node_visits;       /* BVH nodes fetched (64 B each) */
	uint64_t tri_tests;         /* triangles tested (48 B each) */
	uint64_t samples;           /* camera samples rendered */
	double build_seconds;       /* BVH build + upload (host) */
	double render_seconds;      /* GPU wall time of the sample loop + film (hipEvent) */
	double trace_kernel_ms;     /* summed k_trace time (hipEvent pairs), 0 if not profiled */
	uint64_t trace_launches;
	uint32_t bvh_nodes, bvh_depth, scene_in_lds, bvh_width;   /* bvh_width: children per node of the tree k_trace traverses (2, 4, or 8: the quantised BVH8) */
	uint32_t trace_grid, shade_grid;   /* persistent grids (workgroups) of k_trace / k_shade */
	uint32_t trace_block, stack_depth;
	double shade_kernel_ms;     /* summed k_shade time (hipEvent pairs), 0 if not profiled */
	double nee_kernel_ms;       /* summed k_nee time */
	uint64_t photons;           /* photons stored in the diffuse photon map (photon mapping) */
	double photon_seconds;      /* photon shooting + kd-tree build + upload */
	double photon_shoot_seconds, photon_tree_seconds;
	uint64_t gather_visits;     /* point kd-tree nodes fetched by the photon density estimates */
	uint64_t caustic_photons;   /* photons stored in the caustic photon map (0: none / disabled) */
	uint64_t radiance_points;   /* final gathering: radiance points picked while shooting */
	uint64_t radiance_photons;  /* final gathering: points kept (thinned) in the radiance map */
	double fg_thin_seconds;     /* final gathering: radiance-point thinning (host) incl. their download */
	double fg_radiance_seconds; /* final gathering: radiance map total (thinning, pre-gather, kd-tree) */
	int64_t fg_thin_rounds;     /* final gathering: GPU thinning rounds (-1: thinned on the host) */
	uint64_t gather_queries;    /* photon-map estimate requests k_gather served (1.2) */
	uint64_t gather_photons;    /* photon records the density estimates read (1.2) */
	int32_t photon_maps_mode;   /* photon_maps_processing the last render used after its fallbacks: 0 generate,
	                               1 generate-save, 2 load, 3 reuse-previous (1.2) */
	int32_t reserved0;
	uint64_t gather_accepts;    /* two-pass gather: photons the k_gather_walk logged (1.2) */
	uint64_t gather_overflows;  /* two-pass gather: requests whose log overflowed and were walked again (1.2) */
	uint64_t photon_paths_traced; /* photon shooting: path records the bounce launches traced, summed over bounces and maps (1.5) */
	uint64_t photon_slots;      /* photon shooting: deposit slots scanned by the compactions (paths x (bounces + 1)) (1.5) */
	uint64_t fg_paths;          /* final gathering: gather paths traced by k_fg (1.6) */
	uint64_t fg_lookups;        /* final gathering: radiance-map nearest searches (1.6) */
	uint64_t fg_nearest_visits; /* final gathering: radiance-map kd nodes those searches fetched (1.6) */
	uint64_t pregather_visits;  /* final gathering: diffuse-map kd nodes the radiance-map pre-gather fetched (1.6) */
	uint64_t pregather_photons; /* final gathering: photons summed by the pre-gather (1.6) */
	uint64_t pkd_split_level;   /* device / render group: the level at which the members split the last point kd-tree
	                               build (each built the subtrees below it it owns; 0 = every member built the whole tree) (1.6) */
} yafaray_amd_stats_t;

/* Bytes of the LIBYAFARAY_AMD_1.0 struct (its fields end at photon_tree_seconds): yafaray_amd_getStats
 * writes exactly these, so clients built against the 1.0 header keep working; newer clients call
 * yafaray_amd_getStatsEx with sizeof(yafaray_amd_stats_t). */
#define YAFARAY_AMD_STATS_V1_0_SIZE (offsetof(yafaray_amd_stats_t, gather_visits))
/* Bytes yafaray_amd_getStats@@LIBYAFARAY_AMD_1.4 (the default a client links against now) writes: every
 * field through fg_thin_rounds, which the header carried before getStatsEx existed.  Clients linked
 * against the 1.0 symbol keep receiving YAFARAY_AMD_STATS_V1_0_SIZE bytes. */
#define YAFARAY_AMD_STATS_V1_4_SIZE (offsetof(yafaray_amd_stats_t, gather_queries))

/* Bulk geometry: n vertices (xyz doubles, as addVertex) / n triangles (abc ints, as addTriangle). */
YAFARAY_C_API_EXPORT int yafaray_amd_addVertices(yafaray_Interface_t *interface, const double *xyz, int n);
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_addTriangles(yafaray_Interface_t *interface, const int *abc, int n);

/* Build (or rebuild) the GPU acceleration structure for the current scene. */
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_buildAccelerator(yafaray_Interface_t *interface);

/* Batched ray queries.  rays: n x 8 floats (from xyz, dir xyz, tmin, tmax; tmax < 0 = infinite).
 * closest: hits n x 1 float t (-1 = miss), prims n ints (global triangle index in creation order).
 * shadow : occluded n ints (Accelerator::isShadowed semantics: origin moved by tmin, t_max = tmax - 2 tmin). */
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_traceClosest(yafaray_Interface_t *interface, const float *rays, int n, float *t, int *prims);
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_traceShadow(yafaray_Interface_t *interface, const float *rays, int n, int *occluded);

/* Film of the last render: rgba width*height*4 floats (normalised, = put-pixel values), weights width*height. */
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_getFilm(const yafaray_Interface_t *interface, float *rgba, float *weights);
/* Film straight into device memory (rows [y0, y1) of a width*height*4 float buffer on the render device). */
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_getFilmDevice(const yafaray_Interface_t *interface, void *rgba_dev, int y0, int y1);

/* Restrict the next render to tile rows r with r % world == rank (one process per GPU).  world = 1 renders all. */
YAFARAY_C_API_EXPORT void yafaray_amd_setTileRowShard(yafaray_Interface_t *interface, int rank, int world);
/* Restrict the next render to the contiguous pixel-row band [height*rank/world, height*(rank+1)/world)
   (the default split across GPUs: per-row cost is nearly uniform; one halo row is rendered twice). */
YAFARAY_C_API_EXPORT void yafaray_amd_setRowBandShard(yafaray_Interface_t *interface, int rank, int world);
/* Restrict the next render to the explicit pixel-row band [y0, y1) of a film split over `world` GPUs
   (host-side load balancing moves the band boundaries between frames; halo rows are added here). */
YAFARAY_C_API_EXPORT void yafaray_amd_setRowBandRange(yafaray_Interface_t *interface, int y0, int y1, int world);
/* Pixel-row ranges [rows[2k], rows[2k+1]) owned by this rank in the last render; returns their count
   (at most max_ranges are written). */
YAFARAY_C_API_EXPORT int yafaray_amd_getOwnedRows(const yafaray_Interface_t *interface, int *rows, int max_ranges);

/* Render without callbacks / console output (bench loop); same work as yafaray_render. */
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_renderQuiet(yafaray_Interface_t *interface);

/* Counters and timings of the last render: YAFARAY_AMD_STATS_V1_4_SIZE bytes (a client linked against the
 * LIBYAFARAY_AMD_1.0 version of this symbol: YAFARAY_AMD_STATS_V1_0_SIZE bytes). */
YAFARAY_C_API_EXPORT void yafaray_amd_getStats(const yafaray_Interface_t *interface, yafaray_amd_stats_t *stats);
/* (LIBYAFARAY_AMD_1.2) All counters: copies min(bytes, sizeof(yafaray_amd_stats_t)) bytes, returns how many. */
YAFARAY_C_API_EXPORT size_t yafaray_amd_getStatsEx(const yafaray_Interface_t *interface, yafaray_amd_stats_t *stats, size_t bytes);

/* Per-kernel timing of the last render with setProfileKernels on (HIP events before / after every
 * launch on the render stream): for each kernel kind k < return value (and < max): its name, summed
 * launch time in ms, launch count and work items (samples for k_camera / k_film, rays for k_trace,
 * active entries for k_shade, requests for k_nee, queries for k_gather, photon paths for the photon
 * shoot, stored photons for the photon map).  Any output pointer may be NULL.  (LIBYAFARAY_AMD_1.1) */
YAFARAY_C_API_EXPORT int yafaray_amd_getKernelTimes(const yafaray_Interface_t *interface, const char **names, double *ms, uint64_t *launches,
                                                    uint64_t *items, int max);

/* Render group (LIBYAFARAY_AMD_1.1): several GPUs render one film, one member per GPU (e.g. one
 * process per GPU).  Member 0 creates the group id (an RCCL unique id, <= 128 bytes) and hands it to
 * the others by any host means; every member then calls setRenderGroup with its rank on its own
 * current HIP device.  From then on yafaray_render / renderQuiet on each member renders a contiguous
 * band of pixel rows (+ the halo rows its splats need) and all-gathers every band over RCCL (xGMI)
 * into the member's film: each member ends with the whole frame, bit-identical to a one-GPU render.
 * The bands follow the members' measured render times from frame to frame (rebalanceBands).
 * world = 1 leaves the group.  getRenderGroupId returns the id size (0 on failure). */
YAFARAY_C_API_EXPORT int yafaray_amd_getRenderGroupId(void *id, int bytes);
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_setRenderGroup(yafaray_Interface_t *interface, int rank, int world, const void *id, int bytes);
/* Device group (LIBYAFARAY_AMD_1.2): ONE process renders one film on several GPUs — one member per
 * GPU, each on its own host thread and HIP stream, rendering a contiguous row band (+ halo rows);
 * the members exchange the accumulated film between adaptive passes and member 0 pulls every band
 * over xGMI at the end, so the film is bit-identical to a one-GPU render.  By default the group is
 * every visible device (render parameter "gpus": -1 = all, n = the first n devices starting at the
 * current one; env YAFARAY_AMD_GPUS overrides), so an unmodified reference client's yafaray_render
 * uses the whole node.  setDeviceGroup fixes the members explicitly: devices[m] is member m's HIP
 * device (devices NULL: the current device + m, modulo the visible devices — several logical members
 * may share one GPU, which rehearses the group on one device); members <= 0 returns to "gpus".
 * A render group (setRenderGroup) always renders with one member per process. */
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_setDeviceGroup(yafaray_Interface_t *interface, int members, const int *devices);
/* Members the next render uses (0 on failure, e.g. no GPU). */
YAFARAY_C_API_EXPORT int yafaray_amd_getDeviceGroupSize(yafaray_Interface_t *interface);

/* The group's band balancer: world + 1 boundaries and each band's render time -> new boundaries
 * (out, world + 1 ints); cap_rows > 0 rejects a split with a larger band.  Returns 1. */
YAFARAY_C_API_EXPORT int yafaray_amd_rebalanceBands(const int *bounds, int world, const double *times, int cap_rows, int *out);

/* (LIBYAFARAY_AMD_1.2) The render group's band exchange plan on host arrays, as the group runs it on
 * device buffers: packBand writes member `rank`'s rows [bounds[rank], bounds[rank+1]) of a
 * width x height x channels film into a zero-padded slot of the largest band's rows; after an
 * all-gather of the slots (member order), unpackBands copies every other member's rows into the
 * film.  Return 1 (0: bad arguments). */
YAFARAY_C_API_EXPORT int yafaray_amd_packBand(const float *film, int width, int height, int channels, const int *bounds, int world, int rank,
                                              float *send);
YAFARAY_C_API_EXPORT int yafaray_amd_unpackBands(const float *recv, int width, int height, int channels, const int *bounds, int world,
                                                 int rank, float *film);

/* Tuning: samples in flight per wavefront chunk (default 1 << 25, halved automatically if it does not fit) and whether to time k_trace with events. */
/* (LIBYAFARAY_AMD_1.3) The photon map's point kd-tree on its own (batched seam for
 * PointKdTree<T>::PointKdTree, reference include/photon/pkdtree.h:115-222): n positions (x, y, z) in,
 * 2n - 1 nodes of 4 uint32 out in the reference's depth-first layout (.w: bits 0-1 axis or 3 = leaf,
 * interior: right child << 2 and .x the split position bits, .y / .z the parent's plane; leaf:
 * photon index << 2 and .xyz its position bits), *depth = deepest level (root 0).  Current device. */
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_buildPhotonTree(const float *xyz, int n, unsigned int *nodes, int *depth);
/* (LIBYAFARAY_AMD_1.6) The distributed build of a device / render group (what a group render runs for its
 * photon maps): member `member` of `members` builds the levels above *split_level = ceil(log2 members)
 * (0: too few photons to split — the whole tree) and the level-D subtrees it owns, with the map's records
 * in kd order (leaves index kd_pos, n x 4 floats); the other members' subtrees and the parent planes
 * (.y / .z of interior nodes) are left zero — a group exchanges the ranges yafaray_amd_photonTreeSegments
 * gives and writes the planes.  *ms = the build's device time (second of two builds).  Current device. */
YAFARAY_C_API_EXPORT yafaray_bool_t yafaray_amd_buildPhotonTreeMember(const float *xyz, int n, int member, int members, unsigned int *nodes,
                                                                      float *kd_pos, int *depth, int *split_level, double *ms);
/* (LIBYAFARAY_AMD_1.6) The level-`level` subtrees of a tree over n photons, (node, start, end) each in
 * segments[3 << level] (nodes [node, node + 2 (end - start) - 1), kd-order records [start, end)), and the
 * consecutive ones member `member` of `members` owns: [*s0, *s1). */
YAFARAY_C_API_EXPORT void yafaray_amd_photonTreeSegments(unsigned int n, int level, int member, int members, unsigned int *segments,
                                                         unsigned int *s0, unsigned int *s1);
YAFARAY_C_API_EXPORT void yafaray_amd_setChunkSlots(yafaray_Interface_t *interface, int slots);
YAFARAY_C_API_EXPORT void yafaray_amd_setProfileKernels(yafaray_Interface_t *interface, yafaray_bool_t enable);
/* (LIBYAFARAY_AMD_1.2) Per-visit BVH node / triangle counters in the traversal kernels (default on).
 * Off: the stats report rays only (node_visits / tri_tests stay 0) and k_trace runs ~1-2% faster. */
YAFARAY_C_API_EXPORT void yafaray_amd_setTraceStats(yafaray_Interface_t *interface, yafaray_bool_t enable);

/* Diagnostic: summed wave cycles of the k_shade phases (load, connect, hit, next segment, compaction,
 * NEE) since the last reset; returns the number of counters, 0 unless the library was built with
 * -DYAF_PHASE_TIMING (never in the product build). */
YAFARAY_C_API_EXPORT int yafaray_amd_getPhaseCycles(unsigned long long *cycles, int n, yafaray_bool_t reset);

/* (LIBYAFARAY_AMD_1.4) The library's build: the device objects' architecture and extra compile flags
 * (a variant build, e.g. -DYAF_PHASE_TIMING, shows here) and the host compiler.  Static storage. */
YAFARAY_C_API_EXPORT const char *yafaray_amd_buildInfo(void);
/* (LIBYAFARAY_AMD_1.4) How the last render was split across GPUs, as one JSON object: "mode" ("one GPU",
 * "device group", "render group"), "members", "devices", the hipDeviceCanAccessPeer matrix over this
 * process's distinct member devices ("peer_devices", "peer_access"), "copy_path" (how the bands
 * travel), "bounds" (the row-band boundaries the render used), "member_ms" (each member's render time)
 * and "next_bounds" (the rebalanced boundaries of the next frame).  Writes at most bytes - 1 characters
 * + NUL into buf (may be NULL) and returns the length the whole report needs, NUL included (0: no scene). */
YAFARAY_C_API_EXPORT size_t yafaray_amd_getGroupReport(yafaray_Interface_t *interface, char *buf, size_t bytes);

/* Last error message (empty if none); owned by the interface. */
YAFARAY_C_API_EXPORT const char *yafaray_amd_lastError(const yafaray_Interface_t *interface);

#ifdef __cplusplus
}
#endif

#endif /* YAFARAY_AMD_H */
