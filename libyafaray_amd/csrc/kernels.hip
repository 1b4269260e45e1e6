// HIP kernels of the MI355X path-tracing core (gfx950, wave64).
//
// Wavefront pipeline for one chunk of camera samples (render.cc drives it):
//
//   k_camera  -> [ k_trace -> k_shade ] x iterations -> (all chunks) -> k_film
//
//   k_camera : one camera sample per slot — TiledIntegrator::renderTile sample loop
//              (integrator_tiled.cc:288-361) + PerspectiveCamera::shootRay
//              (camera_perspective.cc:128-146).
//   k_trace  : closest-hit rays of the active list + any-hit shadow rays in one launch —
//              Accelerator::intersect / isShadowed (accelerator.cc:55-78) over a BVH2;
//              AcceleratorKdTree::intersect / intersectS semantics (accelerator_kdtree.cc:726-746,
//              851-873) and TrianglePrimitive::intersect (primitive_triangle.cc:44-71).
//              Small scenes are staged into LDS per workgroup; the per-lane traversal stack
//              lives in LDS ([level][lane] layout: conflict-free).
//   k_shade  : connects the previous vertex's next-event estimate with the shadow results, then
//              shades the new hit: emission, MC light estimation (integrator_montecarlo.cc:54-408),
//              BSDF sampling (material_shiny_diffuse.cc:244-327), Russian roulette, and appends
//              the next extension ray / shadow rays with wave-ballot compaction
//              (PathIntegrator::integrate integrator_path_tracer.cc:120-290,
//               DirectLightIntegrator::integrate integrator_direct_light.cc:97-144).
//   k_film   : ImageFilm::addSample (imagefilm.cc:680-733) as a per-destination-pixel gather
//              that replays the reference's single-thread linear-tile splat order, so every film
//              sum is bit-identical without a mutex or atomics; then flush normalisation
//              (imagefilm.cc:590-617, color.h:554-558).
//
// Compiled with -ffp-contract=off: every float expression keeps the reference's order.

#include <hip/hip_runtime.h>
#include <cstdlib>
#include <string>
#include "devmath.h"
#include "photonheap.h"
#include "devscene.h"
#include "texeval.h"

namespace yafamd
{

#ifndef YAF_TRACE_BLOCK
#define YAF_TRACE_BLOCK 128
#endif
// k_shade / k_nee (non-EXT instantiations): at least 4 waves per SIMD (<= 128 VGPRs; the unconstrained allocation took
// 132 / 143 and 3 waves).  Measured on C2: 1400 -> 1500 Msamples/s (shade 0.70 -> 0.62 ms per
// launch, NEE 17.7 -> 15.6 ms per frame), -DYAF_*_MIN_WAVES=n overrides for tuning
#ifndef YAF_SHADE_MIN_WAVES
#define YAF_SHADE_MIN_WAVES 4
#endif
#ifndef YAF_SHADE_LEAN_WAVES
#define YAF_SHADE_LEAN_WAVES 4
#endif
#ifndef YAF_SHADE_PREFETCH
#define YAF_SHADE_PREFETCH 1
#endif
constexpr int kTraceBlock = YAF_TRACE_BLOCK;
// -DYAF_EXPERIMENTS: the pipelines measured and dropped stay buildable for re-measurement but out of
// the product library (kExperiments; yafaray_amd_buildInfo records the flag): k_trace_brute, ray-stream
// sorting in k_trace, the megakernel k_path, k_nee tracing its shadow rays in place, the bounded-radius
// gather walk and the fused shade (-DYAF_FUSE on top).
#ifdef YAF_EXPERIMENTS
constexpr bool kExperiments = true;
#else
constexpr bool kExperiments = false;
#endif
// -DYAF_EXPERIMENTS -DYAF_FUSE: the non-EXT k_shade runs the NEE itself (no k_nee launch).  Measured on C2 (r02):
// 1591 Msamples/s split vs 1455 fused at 3 waves/SIMD (1347 at 4 with 240 B/lane of scratch, 1154
// at 2) — the HBM-bound shade loses more occupancy than the request round trip costs.
#if defined(YAF_FUSE) && defined(YAF_EXPERIMENTS)
constexpr bool kShadeFused = true;
#else
constexpr bool kShadeFused = false;
#endif
// -DYAF_FUSE_LEAN=1 (tuning build): the lean k_shade of the plain path tracer runs the NEE itself
#ifndef YAF_FUSE_LEAN
#define YAF_FUSE_LEAN 0
#endif
constexpr int kShadeBlock = 256;

enum : uint32_t
{
	ST_CAMERA = 0,       // closest ray = camera ray; hit is v0
	ST_FIRST = 1,        // ray = first path segment of the current subpath; hit is v1
	ST_BOUNCE = 2,       // ray = bounce `depth`; hit is v_{depth+1}
	ST_NORAY = 3         // no ray this iteration (only a pending connect, then an action)
};
// flags word
enum : uint32_t
{
	F_MATFLAGS = 0xffffu,        // mat_bsd_fs captured at the first path vertex
	F_SAMPLED = 1u << 16,        // s.sampled_flags_ != None at the first segment
	F_CAUSTIC = 1u << 17,
	F_PEND_V0 = 1u << 18,        // pending: estimateAllDirectLight at v0
	F_PEND_ONE = 1u << 19,       // pending: estimateOneDirectLight at v_k
	F_PEND_EMIT = 1u << 20,      // pending emission add
	F_V0_DIFFUSE = 1u << 21,     // v0 had the Diffuse flag (NEE estimated there)
	F_COLS = 1u << 22,           // compact record: a nonzero first-vertex estimate is stored in csmp[sample id]
	F_SHOWMAP = 1u << 16,        // PhotonIntegrator show_map camera hit (shares bit 16 with F_SAMPLED: path tracing only)
	F_AO_EMIT = 1u << 23,        // ambient occlusion at an emitting v0: pend_emit holds emit(wo)
	F_LNUM_SHIFT = 24            // light picked by estimateOneDirectLight (8 bits)
};

__device__ __forceinline__ float u2f(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t f2u(float f) { return __float_as_uint(f); }
__device__ __forceinline__ V3 xyz(const float4 &a) { return v3(a.x, a.y, a.z); }
__device__ __forceinline__ C3 rgb(const float4 &a) { return C3{a.x, a.y, a.z}; }
__device__ __forceinline__ float4 f4(V3 v, float w) { return make_float4(v.x, v.y, v.z, w); }
__device__ __forceinline__ float4 f4(C3 c, float w) { return make_float4(c.r, c.g, c.b, w); }

__device__ __forceinline__ int laneId() { return __lane_id(); }

// Wave-level append: returns this lane's index in the queue (valid only where `want`).
__device__ __forceinline__ uint32_t waveAppend(bool want, uint32_t *counter)
{
	const uint64_t mask = __ballot(want);
	if(mask == 0) return 0;
	const int leader = __ffsll((unsigned long long)mask) - 1;
	uint32_t base = 0;
	if(laneId() == leader) base = atomicAdd(counter, (uint32_t)__popcll(mask));
	base = __shfl(base, leader);
	const uint64_t below = mask & ((1ull << laneId()) - 1ull);
	return base + (uint32_t)__popcll(below);
}

// Path-state stores of k_shade: the next state is read back only after k_trace / k_nee ran over
// GBs of other data, so caching it buys nothing: they are non-temporal (YAF_NT_STORE), and so are
// the queues, NEE requests and shadow rays (YAF_NT_STORE2).  C2, same box: 1697 / 1707 (plain),
// 1702 / 1723 (state only), 1720 / 1733 Msamples/s (both).  -DYAF_NT_STORE=0 / -DYAF_NT_STORE2=0
// restore plain stores.
#ifndef YAF_NT_STORE
#define YAF_NT_STORE 1
#endif
#ifndef YAF_NT_STORE2
#define YAF_NT_STORE2 1
#endif
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
template<class T>
__device__ __forceinline__ void stStore(T *p, const T &v)
{
	static_assert(sizeof(T) == 16, "16-byte path-state records");
#if YAF_NT_STORE
	u32x4_t w;
	__builtin_memcpy(&w, &v, 16);
	__builtin_nontemporal_store(w, reinterpret_cast<u32x4_t *>(p));
#else
	*p = v;
#endif
}
// the compact path record (sample id, stage): 8 B, non-temporal as the 16-B records
__device__ __forceinline__ void stStoreU2(uint2 *p, uint2 v)
{
	typedef uint32_t u2_t __attribute__((ext_vector_type(2)));
	u2_t w;
	w.x = v.x;
	w.y = v.y;
#if YAF_NT_STORE
	__builtin_nontemporal_store(w, reinterpret_cast<u2_t *>(p));
#else
	*reinterpret_cast<u2_t *>(p) = w;
#endif
}
// wider use (queues, NEE requests and contributions, shadow rays): -DYAF_NT_STORE2
template<class T>
__device__ __forceinline__ void stStore2(T *p, const T &v)
{
#if YAF_NT_STORE2
	if constexpr(sizeof(T) == 16)
	{
		u32x4_t w;
		__builtin_memcpy(&w, &v, 16);
		__builtin_nontemporal_store(w, reinterpret_cast<u32x4_t *>(p));
	}
	else __builtin_nontemporal_store(v, p);
#else
	*p = v;
#endif
}

// 12-byte records (one dwordx3 per lane, 4-byte aligned): the pending throughput, whose fourth
// component was never read
struct F3
{
	float x, y, z;
};

// Closest-ray queue entry i (DevQueues::ray_o / ray_d: 12-B records, 24 B per ray instead of 32):
// false when the entry carries no ray this iteration (NaN direction x).  tmin / tmax (< 0:
// infinite) come from ray_tt in a pass's first iteration when its rays carry their own (spawned rays;
// camera rays with clip planes), else (Q.tmin_dflt, infinite): camera rays 0, k_shade's bounces
// ray_min_dist.
// -DYAF_NT_RAYLOAD=1: the ray streams of k_trace are loaded / stored non-temporally (streaming
// lines evicted first: the node working set of a BVH in global memory keeps more of the L2)
#ifndef YAF_NT_RAYLOAD
#define YAF_NT_RAYLOAD 0
#endif
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ F3 rayLd3(const float *p, uint32_t i)
{
#if YAF_NT_RAYLOAD
	const float *q = p + 3 * (size_t)i;
	return F3{__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1), __builtin_nontemporal_load(q + 2)};
#else
	return reinterpret_cast<const F3 *>(p)[i];
#endif
}
__device__ __forceinline__ float4 rayLd4(const float4 *p)
{
#if YAF_NT_RAYLOAD
	const f32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t *>(p));
	return make_float4(v.x, v.y, v.z, v.w);
#else
	return *p;
#endif
}
template<class T>
__device__ __forceinline__ void raySt(T *p, T v)
{
#if YAF_NT_RAYLOAD
	__builtin_nontemporal_store(v, p);
#else
	*p = v;
#endif
}

__device__ __forceinline__ bool loadQRay(const DevQueues &Q, uint32_t i, V3 &o, V3 &d, float &tmin, float &tmax_w)
{
	// (both records loaded before the test: one memory round trip, not two dependent ones)
	const F3 dd = rayLd3(Q.ray_d, i);
	const F3 oo = rayLd3(Q.ray_o, i);
	d = v3(dd.x, dd.y, dd.z);
	o = v3(oo.x, oo.y, oo.z);
	if(dd.x != dd.x) return false;
	if(Q.ray_tt)
	{
		const float2 tt = Q.ray_tt[i];
		tmin = tt.x;
		tmax_w = tt.y;
	}
	else
	{
		tmin = Q.tmin_dflt;
		tmax_w = -1.f;
	}
	return true;
}
typedef float f32x3a4_t __attribute__((ext_vector_type(3))) __attribute__((aligned(4)));
__device__ __forceinline__ void storeQRay(const DevQueues &Q, uint32_t i, V3 o, V3 d)
{
#if YAF_NT_STORE2
	f32x3a4_t vo, vd;
	vo.x = o.x; vo.y = o.y; vo.z = o.z;
	vd.x = d.x; vd.y = d.y; vd.z = d.z;
	__builtin_nontemporal_store(vo, reinterpret_cast<f32x3a4_t *>(Q.ray_o + 3 * (size_t)i));
	__builtin_nontemporal_store(vd, reinterpret_cast<f32x3a4_t *>(Q.ray_d + 3 * (size_t)i));
#else
	reinterpret_cast<F3 *>(Q.ray_o)[i] = F3{o.x, o.y, o.z};
	reinterpret_cast<F3 *>(Q.ray_d)[i] = F3{d.x, d.y, d.z};
#endif
}
// a 12-B path-state record (the throughput without w), non-temporal as the 16-B ones
__device__ __forceinline__ void stStoreF3(float4 *base, uint32_t k, C3 c)
{
#if YAF_NT_STORE
	f32x3a4_t v;
	v.x = c.r; v.y = c.g; v.z = c.b;
	__builtin_nontemporal_store(v, reinterpret_cast<f32x3a4_t *>(reinterpret_cast<float *>(base) + 3 * (size_t)k));
#else
	reinterpret_cast<F3 *>(base)[k] = F3{c.r, c.g, c.b};
#endif
}
__device__ __forceinline__ void storeQNoRay(const DevQueues &Q, uint32_t i)
{
	Q.ray_d[3 * (size_t)i] = __builtin_nanf("");
}

// NEE request's third word pair, 8 B instead of 16 (k_shade writes it, k_nee reads it): (PixelSamplingData
// offset, s | mode << 20 | light << 21) with s = the sample index minus the pass's first index
// (base_offset + pass_offset, the same for every sample of a launch).  Used while the pass has fewer
// than 2^20 samples per pixel and the scene at most 2^11 lights (neePm8); else the 16-B form.
constexpr uint32_t kPmSBits = 20, kPmLBits = 11;
__device__ __forceinline__ bool neePm8(const DevScene &S)
{
	return !S.nee_pm16 && (uint32_t)S.spp < (1u << kPmSBits) && S.n_lights <= (1 << kPmLBits);
}
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
#ifdef YAF_CHECKED
// checked builds (-DYAF_CHECKED, as pkd's PK_GUARD): a request whose sample index lies outside the pass's
// [base + pass_offset, + spp) window would alias another sample's NEE sequence in the 8-B word; the
// first offending source line is recorded here (yafaray_amd_buildInfo reports the flag, tests read it)
__device__ uint32_t g_nee_pm_err = 0;
#define NEE_PM_GUARD(cond) do { if(!(cond)) atomicCAS(&g_nee_pm_err, 0u, (uint32_t)__LINE__); } while(0)
#else
#define NEE_PM_GUARD(cond) do {} while(0)
#endif
__device__ __forceinline__ void neePmStore(const DevScene &S, uint4 *pm, uint32_t j, uint32_t offset, uint32_t sample_idx, uint32_t mode_l)
{
	if(neePm8(S))
	{
		NEE_PM_GUARD(sample_idx - S.base_offset - S.pass_offset < (uint32_t)S.spp);
		u32x2_t w;
		w.x = offset;
		w.y = (sample_idx - S.base_offset - S.pass_offset) | ((mode_l & 1u) << kPmSBits) | ((mode_l >> 8) << (kPmSBits + 1));
#if YAF_NT_STORE2
		__builtin_nontemporal_store(w, reinterpret_cast<u32x2_t *>(pm) + j);
#else
		reinterpret_cast<u32x2_t *>(pm)[j] = w;
#endif
	}
	else stStore2(&pm[j], make_uint4(offset, sample_idx, mode_l, 0u));
}
// (offset, sample index, mode | light << 8, 0) as k_shade queued it
__device__ __forceinline__ uint4 neePmLoad(const DevScene &S, const uint4 *pm, uint32_t j)
{
	if(neePm8(S))
	{
		const uint2 w = reinterpret_cast<const uint2 *>(pm)[j];
		const uint32_t rel = w.y & ((1u << kPmSBits) - 1u);
		return make_uint4(w.x, S.base_offset + S.pass_offset + rel, ((w.y >> kPmSBits) & 1u) | ((w.y >> (kPmSBits + 1)) << 8), 0u);
	}
	return pm[j];
}

// Segment worked on by this k_trace workgroup, its rank among the segment's workgroups and their
// number (the trace grid is a multiple of n_seg).
struct SegLoop
{
	uint32_t s, r, nb;
};
__device__ __forceinline__ SegLoop segLoop(uint32_t n_seg)
{
	SegLoop L;
	L.s = blockIdx.x % n_seg;
	L.r = blockIdx.x / n_seg;
	L.nb = (gridDim.x - L.s + n_seg - 1) / n_seg;
	return L;
}

// Diagnostic build (-DYAF_PHASE_TIMING): per-phase wave cycles of k_shade (clock64 deltas summed
// by lane 0 of each wave), read with yafaray_amd_getPhaseCycles.  Off in the product build.
#ifdef YAF_PHASE_TIMING
__device__ unsigned long long g_phase[16];
#define PHASE_DECL uint64_t ph_t = clock64(); uint64_t ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PHASE(k) do { const uint64_t t_ = clock64(); ph_acc[k] += t_ - ph_t; ph_t = t_; } while(0)
#define PHASE_FLUSH do { if(laneId() == 0) for(int k_ = 0; k_ < 8; ++k_) atomicAdd(&g_phase[k_], (unsigned long long)ph_acc[k_]); } while(0)
#else
#define PHASE_DECL
#define PHASE(k)
#define PHASE_FLUSH
#endif

// ---------------------------------------------------------------------------------------------
// k_camera
// ---------------------------------------------------------------------------------------------
struct SampleCoord { int x, y, s; };

// sample id (frame-local enumeration over jobs) -> pixel + sample index
__device__ SampleCoord sampleCoord(const DevJob *jobs, int n_jobs, int width, int tile, int spp, uint64_t sid)
{
	// last job whose first sample is <= sid (jobs are in ascending sample_base order)
	int j = 0, hi = n_jobs - 1;
	while(j < hi)
	{
		const int mid = (j + hi + 1) >> 1;
		if(jobs[mid].sample_base <= sid) j = mid;
		else hi = mid - 1;
	}
	const DevJob job = jobs[j];
	const uint64_t local = sid - job.sample_base;
	const uint32_t pix = (uint32_t)(local / (uint64_t)spp);
	const int s = (int)(local % (uint64_t)spp);
	const int bh = job.y1 - job.y0;
	const uint32_t per_tile = (uint32_t)(tile * bh);
	const int tx = (int)(pix / per_tile);
	const int tw = min(tile, width - tx * tile);
	const uint32_t l = pix - (uint32_t)tx * per_tile;
	SampleCoord c;
	c.x = tx * tile + (int)(l % (uint32_t)tw);
	c.y = job.y0 + (int)(l / (uint32_t)tw);
	c.s = s;
	return c;
}

// camera_perspective.cc:71-85
__device__ __forceinline__ float biasDist(int bias, float r)
{
	if(bias == 1) return sqrtf(sqrtf(r) * r);           // BbCenter
	if(bias == 2) return sqrtf(1.f - r * r);            // BbEdge
	return sqrtf(r);                                    // BbNone
}

// vector.cc:128-163 (the long double pi/4 products round like x87)
__device__ __forceinline__ void shirleyDisk(float r_1, float r_2, float &u, float &v)
{
	float phi = 0.f, r = 0.f;
	const float a = 2.f * r_1 - 1.f, b = 2.f * r_2 - 1.f;
	if(a > -b)
	{
		if(a > b) { r = a; phi = x87mul(kDivPiBy4, b / a); }
		else { r = b; phi = x87mul(kDivPiBy4, 2.f - a / b); }
	}
	else
	{
		if(a < b) { r = -a; phi = x87mul(kDivPiBy4, 4.f + b / a); }
		else
		{
			r = -b;
			phi = (b != 0) ? x87mul(kDivPiBy4, 6.f - a / b) : 0.f;
		}
	}
	u = r * fcos(phi);
	v = r * fsin(phi);
}

// camera_perspective.cc:87-124 getLensUv (sampleTsd for the polygon bokehs)
__device__ void lensUv(const DevCamera &c, float r_1, float r_2, float &u, float &v)
{
	const int t = c.bokeh_type;
	if(t >= 3 && t <= 6)
	{
		const float fn = static_cast<float>(t);
		int idx = int(r_1 * fn);
		r_1 = (r_1 - ((float)idx) / fn) * fn;
		r_1 = biasDist(c.bokeh_bias, r_1);
		const float b_1 = r_1 * r_2;
		const float b_0 = r_1 - b_1;
		idx <<= 1;
		u = c.ls[idx] * b_0 + c.ls[idx + 2] * b_1;
		v = c.ls[idx + 1] * b_0 + c.ls[idx + 3] * b_1;
	}
	else if(t == 1 || t == 7)
	{
		const float w = 6.28318548f * r_2;   // (float)math::mult_pi_by_2 * r_2
		if(t == 7) r_1 = sqrtf((float)0.707106781 + (float)0.292893218);
		else r_1 = biasDist(c.bokeh_bias, r_1);
		u = r_1 * fcos(w);
		v = r_1 * fsin(w);
	}
	else shirleyDisk(r_1, r_2, u, v);
}

// sample id -> pixel + sample index: the jobs' enumeration, or an adaptive pass's pixel list
__device__ __forceinline__ SampleCoord sampleAt(const DevScene &S, const DevJob *jobs, int n_jobs, uint64_t sid)
{
	if(S.plist)
	{
		const uint32_t pix = S.plist[sid / (uint64_t)S.spp];
		SampleCoord c;
		c.x = (int)(pix % (uint32_t)S.width);
		c.y = (int)(pix / (uint32_t)S.width);
		c.s = (int)(sid % (uint64_t)S.spp);
		return c;
	}
	return sampleCoord(jobs, n_jobs, S.width, S.tile, S.spp, sid);
}

// One camera sample: TiledIntegrator::renderTile's sample position (integrator_tiled.cc:313-340) and
// PerspectiveCamera::shootRay (camera_perspective.cc:128-146), plus the sample's Russian-roulette seed.
// k_camera (wavefront) and k_path (megakernel) both start their samples here.
__device__ __forceinline__ void cameraRay(const DevScene &S, const SampleCoord &sc, V3 &from, V3 &dir, float &tmin, float &tmax, uint32_t &seed)
{
	// integrator_tiled.cc:313-335 (camera pixel coordinates: a cropped film starts at crop_x0 / crop_y0)
	const int cx = sc.x + S.crop_x0, cy = sc.y + S.crop_y0;
	const uint32_t offset = fnv32((uint32_t)cy * fnv32((uint32_t)cx));
	const uint32_t sample_idx = S.base_offset + S.pass_offset + (uint32_t)sc.s;   // PixelSamplingData::sample_
	float dx = 0.5f, dy = 0.5f;
	if(S.aa_multipass)
	{
		dx = riVdC(sample_idx, offset);
		dy = riS(sample_idx, offset);
	}
	else if(S.spp > 1)
	{
		const float d_1 = 1.f / (float)S.spp;
		dx = (0.5f + (float)sc.s) * d_1;
		dy = riLp((uint32_t)sc.s + offset);
	}
	const float px = (float)cx + dx, py = (float)cy + dy;
	// camera_perspective.cc:128-146, plane.h:37-40
	const DevCamera &c = S.cam;
	const V3 pos = v3(c.pos[0], c.pos[1], c.pos[2]);
	dir = v3(c.vright[0], c.vright[1], c.vright[2]) * px + v3(c.vup[0], c.vup[1], c.vup[2]) * py + v3(c.vto[0], c.vto[1], c.vto[2]);
	dir = normalize(dir);
	const V3 cz = v3(c.cam_z[0], c.cam_z[1], c.cam_z[2]);
	tmin = dot(cz, v3(c.near_p[0], c.near_p[1], c.near_p[2]) - pos) / dot(dir, cz);
	tmax = dot(cz, v3(c.far_p[0], c.far_p[1], c.far_p[2]) - pos) / dot(dir, cz);
	from = pos;
	if(c.aperture != 0.f)
	{
		// integrator_tiled.cc:314-316, 336-340: Halton(3) / Halton(5) lens streams started at the
		// pass offset + pixel offset, one getNext() per sample; camera_perspective.cc:137-144
		const uint32_t hstart = S.base_offset + S.pass_offset + offset;
		const float lu = haltonNext(3u, hstart, sc.s + 1), lv = haltonNext(5u, hstart, sc.s + 1);
		float u, v;
		lensUv(c, lu, lv, u, v);
		const V3 li = v3(c.dof_rt[0], c.dof_rt[1], c.dof_rt[2]) * u + v3(c.dof_up[0], c.dof_up[1], c.dof_up[2]) * v;
		from = from + li;
		dir = normalize(dir * c.dof_distance - li);
	}
	// RR generator: per-sample MWC (the reference seeds one per tile from rand(), so RR
	// output is matched statistically — integrator_tiled.cc:272), seeded from the pixel-major sample
	// id so that the image does not depend on how the film is split over GPUs or chunks
	// (64-bit id: W * H * spp passes 2^32 at 4K x 1024 spp; both halves are hashed)
	const uint64_t gid = ((uint64_t)sc.y * (uint64_t)S.width + (uint64_t)sc.x) * (uint64_t)S.spp + (uint64_t)sc.s;
	const uint32_t gid32 = (uint32_t)gid ^ fnv32((uint32_t)(gid >> 32));
	seed = fnv32(gid32 ^ S.rr_seed ^ (S.pass_offset * 0x9e3779b9u)) + 123u;
}

__global__ void __launch_bounds__(256) k_camera(DevScene S, DevPaths P, DevQueues Q, DevCounters cnt,
                                                 const DevJob *jobs, int n_jobs, uint64_t chunk_base, int n)
{
	// sample i of the chunk -> segment (i / 256) % n_seg, groups of 256 dense within the segment (r05: dealing
	// the groups in eight contiguous runs, one per XCD's segments, was measured 18 % / 50 % slower on C2 / C4 —
	// the regions' different path lengths leave whole XCDs idle at the end of each launch)
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if((uint32_t)i < S.n_seg)
	{
		const uint32_t groups = (uint32_t)n / 256u, rem = (uint32_t)n % 256u, sg = (uint32_t)i, R = S.n_seg;
		cnt.n_active[sg] = (groups / R) * 256u + (sg < groups % R ? 256u : 0u) + (sg == groups % R ? rem : 0u);
		cnt.n_shadow[sg] = 0;
	}
	if(i >= n) return;
	const uint32_t g = (uint32_t)i / 256u;
	const uint32_t a = (g % S.n_seg) * S.cap_a + (g / S.n_seg) * 256u + (uint32_t)i % 256u;
	const SampleCoord sc = sampleAt(S, jobs, n_jobs, chunk_base + (uint64_t)i);
	V3 from, dir;
	float tmin, tmax;
	uint32_t seed;
	cameraRay(S, sc, from, dir, tmin, tmax, seed);
	// the compact record carries the sample id and the stage in pr (offset / sample index derive
	// from the sample id); a specular recursion tree keeps them in the queue's slot and col.w
	// (compact record: the zero throughput, path colour, w and flags of a camera entry are implied by
	// its stage — k_shade does not read them — so they are not written: 32 B per sample each way)
	storeQRay(Q, a, from, dir);
	if(S.cam.ray_tt) Q.ray_tt[a] = make_float2(tmin, tmax);
	if(!S.tree) reinterpret_cast<uint2 *>(P.pr)[a] = make_uint2((uint32_t)i, ST_CAMERA);   // (RR: rrRandom)
	else
	{
		const int cx = sc.x + S.crop_x0, cy = sc.y + S.crop_y0;
		const uint32_t offset = fnv32((uint32_t)cy * fnv32((uint32_t)cx));
		const uint32_t sample_idx = S.base_offset + S.pass_offset + (uint32_t)sc.s;
		Q.slot[a] = i;          // sample id within the chunk travels with the queue entry
		P.thr[a] = make_float4(0.f, 0.f, 0.f, 0.f);                        // w = 0
		P.col[a] = make_float4(0.f, 0.f, 0.f, __uint_as_float(ST_CAMERA));   // stage
		P.pcol[a] = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));         // flags
		P.pr[a] = make_uint4(offset, sample_idx, 30903u, seed);
	}
}

// ---------------------------------------------------------------------------------------------
// k_trace: BVH2 / BVH4 traversal
// ---------------------------------------------------------------------------------------------
#ifndef YAF_TOP_STRIDE
#define YAF_TOP_STRIDE 9
#endif
constexpr int kTopStride = YAF_TOP_STRIDE;
#ifndef YAF_LANE_REMAT
#define YAF_LANE_REMAT 1
#endif   // float4 per node of the LDS top treelet (8 used + 1 pad)
struct TraceCtx
{
	const float4 *nodes;
	const float4 *tris;
	int *stack;     // LDS, [level * kTraceBlock + lane], levels [0, lds_depth)
	int lds_depth;
	int *spill;     // HBM, [(level - lds_depth) * spill_stride + global lane] (BVH4 deep levels)
	uint32_t spill_stride;
	// the top treelet of a BVH4 in global memory staged in LDS: nodes [0, n_top) at kTopStride float4 each
	// (144 B: a 128-B stride put every node's plane p on the same 4 of the 64 banks, so the 16 lanes of a
	// ds_read_b128 group at different nodes conflicted up to 8-way; 36-dword strides spread 16 nodes
	// over 16 distinct bank quads) (both builders number
	// the wide nodes level by level, so these are the levels every ray starts with)
	const float4 *top = nullptr;
	int n_top = 0;
	uint32_t wave_base = 0;   // threadIdx.x of the wave's lane 0 (scalar; set with the context: waveBase())
};
// threadIdx.x of the wave's first lane, and this lane's threadIdx.x re-derived from it (v_mbcnt, opaque so
// that it is recomputed where used instead of keeping threadIdx.x live — or spilled — across the loops)
__device__ __forceinline__ uint32_t waveBase() { return __builtin_amdgcn_readfirstlane((uint32_t)threadIdx.x) & ~63u; }
__device__ __forceinline__ uint32_t tidFrom(uint32_t wave_base)
{
	uint32_t l;
	asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
	return wave_base + l;
}

// Transparent-shadow hit list of one shadow ray (accelerator_kdtree.cc:1001-1023): an opaque
// surface shadows; each transparent one is recorded until `cap` (= shadowDepth) are recorded, the
// next one shadows.  A BVH holds every triangle once, so the reference's `filtered` set (one
// factor per primitive) needs no lookup.
struct TsList
{
	float2 *hit;
	int n, cap;
	const float4 *prim_ng;
	const DevMaterial *mats;
};

__device__ __forceinline__ bool tsShadows(TsList &L, float t, int prim)
{
	const int mat = __float_as_int(L.prim_ng[prim].w);
	if(!(L.mats[mat].sd_flags & SD_TRANSPARENT)) return true;
	if(L.n >= L.cap) return true;
	L.hit[L.n] = make_float2(t, __int_as_float(prim));
	++L.n;
	return false;
}

__device__ __forceinline__ void boxPair(const float4 &n0, const float4 &n1, const float4 &n2, V3 o, V3 id,
                                        float t0, float t1, bool &h0, bool &h1, float &tn0, float &tn1)
{
	// child 0
	float ax = (n0.x - o.x) * id.x, bx = (n0.y - o.x) * id.x;
	float ay = (n0.z - o.y) * id.y, by = (n0.w - o.y) * id.y;
	float az = (n2.x - o.z) * id.z, bz = (n2.y - o.z) * id.z;
	float lo = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), t0));
	float hi = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), t1));
	h0 = lo <= hi;
	tn0 = lo;
	ax = (n1.x - o.x) * id.x; bx = (n1.y - o.x) * id.x;
	ay = (n1.z - o.y) * id.y; by = (n1.w - o.y) * id.y;
	az = (n2.z - o.z) * id.z; bz = (n2.w - o.z) * id.z;
	lo = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), t0));
	hi = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), t1));
	h1 = lo <= hi;
	tn1 = lo;
}

// primitive_triangle.cc:44-71.  Returns t or -1.  The reference's arithmetic (correctly rounded
// 1/det, then products) evaluated branch-free: every lane computes the same instruction stream
// and the reference's early returns become one combined predicate (NaN comparisons keep their
// reference outcome).  `t_cut` is unused by the exact test.  (The short-circuit form is kept on
// purpose: the compiler turns it into det -> u -> (v, t) early outs; a bitwise predicate that
// computes every term measured k_trace 27.6 -> 35.4 ms per C2 frame.)
// Correctly rounded 1/x: v_rcp_f32 + one FMA Newton step, which tools/rcp_check.hip
// verified exhaustively on gfx950 to equal the IEEE quotient for every float with
// 2^-125 <= |x| <= 2^125 (other magnitudes, zero, inf and NaN take the IEEE division).
__device__ __forceinline__ float rcpExact(float x)
{
	const float ax = fabsf(x);
	if(ax >= 0x1p-125f && ax <= 0x1p125f)
	{
		const float y = __builtin_amdgcn_rcpf(x);
		return __builtin_fmaf(y, __builtin_fmaf(-x, y, 1.f), y);
	}
	return 1.f / x;
}

__device__ __forceinline__ float triTest(const float4 &a, const float4 &b, const float4 &c, V3 o, V3 d, float t_cut)
{
	(void)t_cut;
	const V3 v0 = xyz(a), e1 = xyz(b), e2 = xyz(c);
	const float eps = a.w;
	const V3 pvec = cross(d, e2);
	const float det = dot(e1, pvec);
	const float inv_det = rcpExact(det);
	const V3 tvec = o - v0;
	const float u = dot(tvec, pvec) * inv_det;
	const V3 qvec = cross(tvec, e1);
	const float v = dot(d, qvec) * inv_det;
	const float t = dot(e2, qvec) * inv_det;
	const bool miss = (det > -eps && det < eps) || (u < 0.f || u > 1.f) || (v < 0.f) || ((u + v) > 1.f) || (t < eps);
	return miss ? -1.f : t;
}

// per-visit statistics of the traversal (node visits, triangle tests); -DYAF_TRACE_NOSTATS drops them
#ifdef YAF_TRACE_NOSTATS
#define TRACE_STAT(x) do {} while(0)
#else
#define TRACE_STAT(x) x
#endif

// Closest hit with t in [tmin, tmax) (ties -> lower primitive index), or any hit with t in
// [0, tmax).  Box tests are conservative (boxes padded at build time + a relative slack), so
// culling never drops a hit the exhaustive reference semantics would return.
template<bool ANY, bool TS = false, bool STATS = true>
__device__ bool traverse2(const TraceCtx &C, V3 o, V3 d, float tmin, float tmax, float &t_best, int &prim_best,
                          uint32_t &visits, uint32_t &tests, TsList *ts = nullptr)
{
	const int lane = threadIdx.x;
	V3 dd = d;
	if(fabsf(dd.x) < 1e-20f) dd.x = copysignf(1e-20f, dd.x);
	if(fabsf(dd.y) < 1e-20f) dd.y = copysignf(1e-20f, dd.y);
	if(fabsf(dd.z) < 1e-20f) dd.z = copysignf(1e-20f, dd.z);
	const V3 id = v3(rcpExact(dd.x), rcpExact(dd.y), rcpExact(dd.z));
	const float box_t0 = ANY ? -1e-3f : (tmin - 1e-3f * (1.f + fabsf(tmin)));
	t_best = tmax;
	prim_best = -1;
	int sp = 0;
	int node = 0;
	for(;;)
	{
		if(STATS) TRACE_STAT(++visits);
		const float4 *np = C.nodes + 4 * node;
		const float4 n0 = np[0], n1 = np[1], n2 = np[2], n3 = np[3];
		const float slack_t = (t_best < 3.0e38f) ? t_best * 1.0000005f + 1e-6f : 3.4e38f;
		bool h0, h1;
		float tn0, tn1;
		boxPair(n0, n1, n2, o, id, box_t0, slack_t, h0, h1, tn0, tn1);
		const int c0 = __float_as_int(n3.x), c1 = __float_as_int(n3.y);
		const int k0 = __float_as_int(n3.z), k1 = __float_as_int(n3.w);
		int next = -1;
		// leaves are tested right away; inner children are descended nearest-first
#pragma unroll
		for(int side = 0; side < 2; ++side)
		{
			const bool h = side ? h1 : h0;
			const int c = side ? c1 : c0;
			const int k = side ? k1 : k0;
			if(!h || c >= 0 || k == 0) continue;
			const int start = ~c;
			for(int q = start; q < start + k; ++q)
			{
				if(STATS) TRACE_STAT(++tests);
				const float4 *tp = C.tris + 3 * q;
				const float4 ta = tp[0], tb = tp[1], tc = tp[2];
				const float t = triTest(ta, tb, tc, o, d, ANY ? tmax : t_best);
				if(t == -1.f) continue;
				const int prim = __float_as_int(tb.w);
				if(ANY && TS)
				{
					// intersectTs: t in [tmin, t_max) of the moved ray (tmin kept, accelerator.cc:82-85)
					if(t < tmax && t >= tmin && tsShadows(*ts, t, prim)) { t_best = t; prim_best = prim; return true; }
				}
				else if(ANY)
				{
					if(t < tmax && t >= 0.f) { t_best = t; prim_best = prim; return true; }
				}
				else if(t >= tmin && (t < t_best || (t == t_best && prim_best >= 0 && prim < prim_best)))
				{
					t_best = t;
					prim_best = prim;
				}
			}
		}
		const bool i0 = h0 && c0 >= 0, i1 = h1 && c1 >= 0;
		if(i0 && i1)
		{
			const bool first0 = tn0 <= tn1;
			next = first0 ? c0 : c1;
			C.stack[sp * kTraceBlock + lane] = first0 ? c1 : c0;
			++sp;
		}
		else if(i0) next = c0;
		else if(i1) next = c1;
		if(next < 0)
		{
			if(sp == 0) break;
			--sp;
			next = C.stack[sp * kTraceBlock + lane];
		}
		node = next;
	}
	return prim_best >= 0;
}

__device__ __forceinline__ float lane4(const float4 &v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

__device__ __forceinline__ void cswap(float &ka, int &va, float &kb, int &vb)
{
	const bool sw = kb < ka;
	const float k = sw ? kb : ka;
	kb = sw ? ka : kb;
	ka = k;
	const int v = sw ? vb : va;
	vb = sw ? va : vb;
	va = v;
}

// Near / far planes of a BVH4 node's boxes for one ray.  By the sign of the inverse direction the
// slab's entry plane is the low bound (1/d >= 0) or the high one for every box, and fma(b, 1/d, -o/d)
// is monotone in b, so max(near distances) / min(far distances) are exactly the values of the
// per-child min / max over both planes — 4 x 6 fewer min / max per visit for six per-lane addresses.
struct SlabSel { int nx, ny, nz; };   // float4 index in the node of the near plane per axis (far: ^ 1)
__device__ __forceinline__ SlabSel slabSel(V3 id) { return SlabSel{id.x >= 0.f ? 0 : 1, id.y >= 0.f ? 2 : 3, id.z >= 0.f ? 4 : 5}; }

// Child order after a BVH4 visit (results never depend on it: closest hits tie-break on the primitive
// index, any hits answer occluded / not): closest rays sort the hit inner children by entry distance
// (YAF_CLOSEST_SORT, the culling order); any-hit rays skip the network (YAF_ANY_SORT=1 restores it)
#ifndef YAF_ANY_SORT
#define YAF_ANY_SORT 0
#endif
#ifndef YAF_CLOSEST_SORT
#define YAF_CLOSEST_SORT 1
#endif
// BVH4 (bvh.cc: collapsed binary SAH tree, 128 B nodes with the four child boxes in SoA form).
// Same hit semantics as traverse2: leaf children are tested as soon as their box is hit, inner
// children are sorted by entry distance (5-exchange network) and descended nearest-first.
// PACK (LDS-resident trees, < 512 nodes): the closest rays' child order from packed integer keys (below);
// -DYAF_PACKED_SORT=1 also packs the BVH8 refill loop's 19-exchange network.  Measured and off (r06, same
// box A/B): C2 k_trace 25.9 -> 27.2 ms per frame (fewer VALU per exchange, but the key packing and the
// child masks cost more than the selects they replace at the 64-VGPR budget), C4 unchanged (126.4 ms)
#ifndef YAF_PACKED_SORT
#define YAF_PACKED_SORT 0
#endif
constexpr uint32_t kPackNodeBits = 9;   // node index bits of a packed key: LDS-resident BVH4s have <= 384 nodes (48 KB)
template<bool ANY, bool SPILL, bool TS = false, bool STATS = true, bool PACK = false>
__device__ bool traverse4(const TraceCtx &C, V3 o, V3 d, float tmin, float tmax, float &t_best, int &prim_best,
                          uint32_t &visits, uint32_t &tests, TsList *ts = nullptr)
{
#if YAF_LANE_REMAT
	// the lane's stack column from the wave's first thread (scalar) and the lane id (v_mbcnt, re-derived at
	// every push / pop — opaque, so not hoisted): at the 64-VGPR budget a loop-invariant column address
	// was spilled and reloaded from scratch at every push (a vector-memory wait per push)
#define YAF_LANE ((int)tidFrom(C.wave_base))
#else
	const int lane = threadIdx.x;
#define YAF_LANE lane
#endif
	V3 dd = d;
	if(fabsf(dd.x) < 1e-20f) dd.x = copysignf(1e-20f, dd.x);
	if(fabsf(dd.y) < 1e-20f) dd.y = copysignf(1e-20f, dd.y);
	if(fabsf(dd.z) < 1e-20f) dd.z = copysignf(1e-20f, dd.z);
	const V3 id = v3(rcpExact(dd.x), rcpExact(dd.y), rcpExact(dd.z));
	// slab distances as fma(bound, 1/d, -o/d): the rounding of o/d is covered by the boxes' build-time
	// padding (mag * 1e-5, bvh.cc padBox) as the rounding of (bound - o) is
	const V3 oid = v3(o.x * id.x, o.y * id.y, o.z * id.z);
	const SlabSel sel = slabSel(id);
	const float box_t0 = ANY ? -1e-3f : (tmin - 1e-3f * (1.f + fabsf(tmin)));
	const float inf = __builtin_huge_valf();
	const uint32_t glane = blockIdx.x * blockDim.x + threadIdx.x;
	t_best = tmax;
	prim_best = -1;
	int sp = 0;
	int node = 0;
	// the first lds_depth levels live in LDS; deeper ones (rare) spill to this lane's HBM column
	auto push = [&](int v) {
		if(!SPILL || sp < C.lds_depth) C.stack[sp * kTraceBlock + YAF_LANE] = v;   // (!SPILL: the bound fits the LDS levels)
		else if(SPILL) C.spill[(uint32_t)(sp - C.lds_depth) * C.spill_stride + glane] = v;
	};
	// the box culling distance: recomputed only where t_best changes (a closest hit), not per visit
	auto slackOf = [](float t) { return (t < 3.0e38f) ? t * 1.0000005f + 1e-6f : 3.4e38f; };
	float slack_t = slackOf(t_best);
	for(;;)
	{
		if(STATS) TRACE_STAT(++visits);
		const float4 *np = C.nodes + 8 * node;
		const float4 nx = np[sel.nx], fx = np[sel.nx ^ 1], ny = np[sel.ny], fy = np[sel.ny ^ 1], nz = np[sel.nz], fz = np[sel.nz ^ 1], cf = np[6], kf = np[7];
		float key[4];
		int child[4], count[4];
		uint32_t leaves = 0;
		// the four slab tests first, so the node's registers are free before any triangle test
#pragma unroll
		for(int k = 0; k < 4; ++k)
		{
			const float lo = fmaxf(fmaxf(__builtin_fmaf(lane4(nx, k), id.x, -oid.x), __builtin_fmaf(lane4(ny, k), id.y, -oid.y)),
			                       fmaxf(__builtin_fmaf(lane4(nz, k), id.z, -oid.z), box_t0));
			const float hi = fminf(fminf(__builtin_fmaf(lane4(fx, k), id.x, -oid.x), __builtin_fmaf(lane4(fy, k), id.y, -oid.y)),
			                       fminf(__builtin_fmaf(lane4(fz, k), id.z, -oid.z), slack_t));
			// selects, not branches: a lane-varying `if` here costs an exec-mask save / restore per child
			const uint32_t h = lo <= hi ? 1u : 0u;
			child[k] = __float_as_int(lane4(cf, k));
			count[k] = __float_as_int(lane4(kf, k));
			const uint32_t inner = child[k] >= 0 ? 1u : 0u;
			key[k] = (h & inner) ? lo : inf;
			leaves |= (h & (inner ^ 1u) & (count[k] > 0 ? 1u : 0u)) << k;
		}
		// the hit leaves' triangles as one per-lane list (leaf order, then triangle order), so that a
		// wave runs max-over-lanes tests per node instead of one pass per leaf slot any lane hit
		int e[4], s4[4];
		{
			int acc = 0;
#pragma unroll
			for(int k = 0; k < 4; ++k)
			{
				const bool l = leaves & (1u << k);
				s4[k] = ~child[k] - acc;
				acc += l ? count[k] : 0;
				e[k] = acc;
			}
		}
		for(int i = 0; i < e[3]; ++i)
		{
			const int q = i + (i < e[0] ? s4[0] : i < e[1] ? s4[1] : i < e[2] ? s4[2] : s4[3]);
			{
				if(STATS) TRACE_STAT(++tests);
				const float4 *tp = C.tris + 3 * q;
				const float4 ta = tp[0], tb = tp[1], tc = tp[2];
				const float t = triTest(ta, tb, tc, o, d, ANY ? tmax : t_best);
				if(t == -1.f) continue;
				const int prim = __float_as_int(tb.w);
				if(ANY && TS)
				{
					// intersectTs: t in [tmin, t_max) of the moved ray (tmin kept, accelerator.cc:82-85)
					if(t < tmax && t >= tmin && tsShadows(*ts, t, prim)) { t_best = t; prim_best = prim; return true; }
				}
				else if(ANY)
				{
					if(t < tmax && t >= 0.f) { t_best = t; prim_best = prim; return true; }
				}
				else if(t >= tmin && (t < t_best || (t == t_best && prim_best >= 0 && prim < prim_best)))
				{
					t_best = t;
					prim_best = prim;
					slack_t = slackOf(t_best);
				}
			}
		}
		int next;
		if constexpr(ANY && !YAF_ANY_SORT)
		{
			// any hit: the answer does not depend on the order the hit children are visited in (there is
			// no distance to cull against), so no sorting network — the first hit inner child is descended,
			// the others pushed in node order
			next = -1;
#pragma unroll
			for(int k = 0; k < 4; ++k)
			{
				if(!(key[k] < inf)) continue;
				if(next < 0) next = child[k];
				else { push(child[k]); ++sp; }
			}
		}
		else if constexpr(PACK && YAF_PACKED_SORT && YAF_CLOSEST_SORT)
		{
			// one 32-bit key per hit inner child: the entry distance clamped at 0 with the child's node index in
			// the low kPackNodeBits bits (the order is a culling heuristic only — closest hits tie-break on the
			// primitive index, so neither the clamp nor the dropped mantissa bits change a result), sorted as
			// unsigned integers: a compare-exchange is one v_min_u32 + v_max_u32 instead of a compare and four
			// selects, and the child comes back with a mask; a missed child is all ones
			constexpr uint32_t nm = (1u << kPackNodeBits) - 1u;
			uint32_t pk[4];
#pragma unroll
			for(int k = 0; k < 4; ++k)
				pk[k] = key[k] < inf ? ((__float_as_uint(fmaxf(key[k], 0.f)) & ~nm) | (uint32_t)child[k]) : 0xffffffffu;
			auto cx = [](uint32_t &a, uint32_t &b) {
				const uint32_t lo = min(a, b);
				b = max(a, b);
				a = lo;
			};
			cx(pk[0], pk[1]);
			cx(pk[2], pk[3]);
			cx(pk[0], pk[2]);
			cx(pk[1], pk[3]);
			cx(pk[1], pk[2]);
			if(pk[3] != 0xffffffffu) { push((int)(pk[3] & nm)); ++sp; }
			if(pk[2] != 0xffffffffu) { push((int)(pk[2] & nm)); ++sp; }
			if(pk[1] != 0xffffffffu) { push((int)(pk[1] & nm)); ++sp; }
			next = pk[0] != 0xffffffffu ? (int)(pk[0] & nm) : -1;
		}
		else if constexpr(!YAF_CLOSEST_SORT)
		{
			// (tuning variant) the nearest hit child descended, the others pushed in node order
			int kmin = 0;
#pragma unroll
			for(int k = 1; k < 4; ++k) kmin = key[k] < key[kmin] ? k : kmin;
			next = key[kmin] < inf ? child[kmin] : -1;
#pragma unroll
			for(int k = 3; k >= 0; --k)
				if(k != kmin && key[k] < inf) { push(child[k]); ++sp; }
		}
		else
		{
			cswap(key[0], child[0], key[1], child[1]);
			cswap(key[2], child[2], key[3], child[3]);
			cswap(key[0], child[0], key[2], child[2]);
			cswap(key[1], child[1], key[3], child[3]);
			cswap(key[1], child[1], key[2], child[2]);
			if(key[3] < inf) { push(child[3]); ++sp; }
			if(key[2] < inf) { push(child[2]); ++sp; }
			if(key[1] < inf) { push(child[1]); ++sp; }
			next = key[0] < inf ? child[0] : -1;
		}
		if(next < 0)
		{
			if(sp == 0) break;
			--sp;
			next = (!SPILL || sp < C.lds_depth) ? C.stack[sp * kTraceBlock + YAF_LANE]
			                                    : C.spill[(uint32_t)(sp - C.lds_depth) * C.spill_stride + glane];
		}
		node = next;
	}
	return prim_best >= 0;
}

// k_trace's BVH4 loop with per-lane ray refill: a lane works through its own sequence of queue
// entries (j, j + stride, ...), closest rays then shadow rays, and starts its next ray as soon as
// its traversal ends, so a wave runs as long as its longest lane's sum of rays instead of the sum
// over rays of the longest lane.  Every ray runs the sequence of traverse4 (same visits, culling,
// leaf order and early exits), so hits are identical.
#undef YAF_LANE

template<bool SPILL, bool STATS = true>
__device__ void traceRefill4(const TraceCtx &C, const DevQueues &Q, const DevPaths &P, uint32_t n_a, uint32_t total,
                             uint32_t a0, uint32_t s0, uint32_t j, uint32_t stride, uint32_t &visits, uint32_t &tests,
                             uint32_t &n_closest, uint32_t &n_shadow)
{
	const int lane = threadIdx.x;
	const uint32_t glane = blockIdx.x * blockDim.x + threadIdx.x;
	const float inf = __builtin_huge_valf();
	V3 o = v3(0.f, 0.f, 0.f), d = o, id = o, oid = o;
	SlabSel sel{0, 2, 4};
	float tmin = 0.f, tmax = 0.f, box_t0 = 0.f, t_best = 0.f;
	int prim_best = -1, sp = 0, node = -1;
	bool any = false;
	uint32_t cur = 0;
	auto push = [&](int v) {
		if(sp < C.lds_depth) C.stack[sp * kTraceBlock + lane] = v;
		else if(SPILL) C.spill[(uint32_t)(sp - C.lds_depth) * C.spill_stride + glane] = v;
	};
	for(;;)
	{
		if(node < 0)
		{
			// next ray of this lane (closest entries with a NaN direction carry no ray)
			bool got = false;
			for(;;)
			{
				if(j >= total) break;
				cur = j;
				j += stride;
				if(cur < n_a)
				{
					float tw;
					if(!loadQRay(Q, a0 + cur, o, d, tmin, tw)) continue;
					tmax = (tw >= 0.f) ? tw : inf;
					any = false;
					++n_closest;
				}
				else
				{
					const float4 od = rayLd4(&Q.sh_o[s0 + (cur - n_a)]);
					const float4 dd = rayLd4(&Q.sh_d[s0 + (cur - n_a)]);
					o = xyz(od);
					d = xyz(dd);
					tmin = 0.f;
					tmax = dd.w;
					any = true;
					++n_shadow;
				}
				got = true;
				break;
			}
			if(!got) break;
			V3 dq = d;
			if(fabsf(dq.x) < 1e-20f) dq.x = copysignf(1e-20f, dq.x);
			if(fabsf(dq.y) < 1e-20f) dq.y = copysignf(1e-20f, dq.y);
			if(fabsf(dq.z) < 1e-20f) dq.z = copysignf(1e-20f, dq.z);
			id = v3(rcpExact(dq.x), rcpExact(dq.y), rcpExact(dq.z));
			oid = v3(o.x * id.x, o.y * id.y, o.z * id.z);
			sel = slabSel(id);
			box_t0 = any ? -1e-3f : (tmin - 1e-3f * (1.f + fabsf(tmin)));
			t_best = tmax;
			prim_best = -1;
			sp = 0;
			node = 0;
		}
		if(STATS) TRACE_STAT(++visits);
		float4 nx, fx, ny, fy, nz, fz, cf, kf;
		if(node < C.n_top)
		{
			// the top treelet from LDS (an explicit LDS pointer: ds_read, not flat loads)
			typedef float V4 __attribute__((ext_vector_type(4)));
			typedef const __attribute__((address_space(3))) V4 *LdsV4;
			const LdsV4 tp = (LdsV4)(C.top + kTopStride * node);
			auto ld = [&](int k) {
				const V4 v = tp[k];
				return make_float4(v.x, v.y, v.z, v.w);
			};
			nx = ld(sel.nx); fx = ld(sel.nx ^ 1); ny = ld(sel.ny); fy = ld(sel.ny ^ 1); nz = ld(sel.nz); fz = ld(sel.nz ^ 1); cf = ld(6); kf = ld(7);
		}
		else
		{
			const float4 *np = C.nodes + 8 * node;
			nx = np[sel.nx]; fx = np[sel.nx ^ 1]; ny = np[sel.ny]; fy = np[sel.ny ^ 1]; nz = np[sel.nz]; fz = np[sel.nz ^ 1]; cf = np[6]; kf = np[7];
		}
		const float slack_t = (t_best < 3.0e38f) ? t_best * 1.0000005f + 1e-6f : 3.4e38f;
		float key[4];
		int child[4], e[4], s4[4];
		int acc = 0;
#pragma unroll
		for(int k = 0; k < 4; ++k)
		{
			const float lo = fmaxf(fmaxf(__builtin_fmaf(lane4(nx, k), id.x, -oid.x), __builtin_fmaf(lane4(ny, k), id.y, -oid.y)),
			                       fmaxf(__builtin_fmaf(lane4(nz, k), id.z, -oid.z), box_t0));
			const float hi = fminf(fminf(__builtin_fmaf(lane4(fx, k), id.x, -oid.x), __builtin_fmaf(lane4(fy, k), id.y, -oid.y)),
			                       fminf(__builtin_fmaf(lane4(fz, k), id.z, -oid.z), slack_t));
			const uint32_t h = lo <= hi ? 1u : 0u;
			child[k] = __float_as_int(lane4(cf, k));
			const int count = __float_as_int(lane4(kf, k));
			const uint32_t inner = child[k] >= 0 ? 1u : 0u;
			key[k] = (h & inner) ? lo : inf;
			s4[k] = ~child[k] - acc;
			acc += (h & (inner ^ 1u)) ? count : 0;
			e[k] = acc;
		}
		bool done = false;
		for(int i = 0; i < e[3]; ++i)
		{
			const int q = i + (i < e[0] ? s4[0] : i < e[1] ? s4[1] : i < e[2] ? s4[2] : s4[3]);
			if(STATS) TRACE_STAT(++tests);
			const float4 *tp = C.tris + 3 * q;
			const float4 ta = tp[0], tb = tp[1], tc = tp[2];
			const float t = triTest(ta, tb, tc, o, d, t_best);
			if(t == -1.f) continue;
			const int prim = __float_as_int(tb.w);
			if(any)
			{
				if(t < tmax && t >= 0.f) { t_best = t; prim_best = prim; done = true; break; }
			}
			else if(t >= tmin && (t < t_best || (t == t_best && prim_best >= 0 && prim < prim_best)))
			{
				t_best = t;
				prim_best = prim;
			}
		}
		if(!done)
		{
			cswap(key[0], child[0], key[1], child[1]);
			cswap(key[2], child[2], key[3], child[3]);
			cswap(key[0], child[0], key[2], child[2]);
			cswap(key[1], child[1], key[3], child[3]);
			cswap(key[1], child[1], key[2], child[2]);
			if(key[3] < inf) { push(child[3]); ++sp; }
			if(key[2] < inf) { push(child[2]); ++sp; }
			if(key[1] < inf) { push(child[1]); ++sp; }
			int next = key[0] < inf ? child[0] : -1;
			if(next < 0 && sp > 0)
			{
				--sp;
				next = (!SPILL || sp < C.lds_depth) ? C.stack[sp * kTraceBlock + lane]
				                                    : C.spill[(uint32_t)(sp - C.lds_depth) * C.spill_stride + glane];
			}
			node = next;
			done = next < 0;
		}
		if(done)
		{
			// (the NEE entry of an opaque shadow ray rides in sh_o.w: re-read at the end rather than held
			// in a register through the traversal, which spilled at this kernel's 6-wave budget)
			if(any) P.occ[__float_as_int(Q.sh_o[s0 + (cur - n_a)].w)] = prim_best >= 0 ? 1 : 0;   // P = state set of the consumer shade
			else
			{
				raySt(&Q.hit_t[a0 + cur], t_best);
				raySt(&Q.hit_prim[a0 + cur], prim_best);
			}
			node = -1;
		}
	}
}

// ---- quantised BVH8 (bvhgpu.hip k_q8_write: the device-built tree collapsed to eight children, child
// boxes as bytes over a per-node origin and power-of-two quanta, rounded outwards; opt-in for scenes in
// global memory).  A visit reads 80 B (one line): origin, quanta, child masks, the first inner child, the
// first leaf triangle (the BVH8's own triangle array, leaves in node order) and the six byte planes;
// the slab test decodes t = q · (2^e / d) + (origin − o) / d.  The decoded boxes contain the float boxes
// (which carry the BVH4's padding), the triangle test and the tie rule are the BVH4's: the same hits.
#ifndef YAF_W8_SORT
#define YAF_W8_SORT 1
#endif
constexpr int kTop8Stride = 5;   // float4 per staged node in LDS (the 80 B a visit reads: 20 dwords, so 16
                                 // consecutive nodes start on 16 distinct bank quads)
__device__ __forceinline__ float q8Byte(uint32_t lo4, uint32_t hi4, int k)
{
	const uint32_t w = k < 4 ? lo4 : hi4;
	return (float)((w >> (8 * (k & 3))) & 0xffu);   // (v_cvt_f32_ubyteN)
}

template<bool SPILL, bool STATS = true>
__device__ void traceRefill8(const TraceCtx &C, const DevQueues &Q, const DevPaths &P, uint32_t n_a, uint32_t total,
                             uint32_t a0, uint32_t s0, uint32_t j, uint32_t stride, uint32_t &visits, uint32_t &tests,
                             uint32_t &n_closest, uint32_t &n_shadow)
{
	const uint32_t glane = blockIdx.x * blockDim.x + threadIdx.x;
	const float inf = __builtin_huge_valf();
	V3 o = v3(0.f, 0.f, 0.f), d = o, id = o;
	float tmin = 0.f, tmax = 0.f, box_t0 = 0.f, t_best = 0.f;
	int prim_best = -1, sp = 0, node = -1;
	bool any = false;
	uint32_t cur = 0;
	auto push = [&](int v) {
		if(sp < C.lds_depth) C.stack[sp * kTraceBlock + (int)tidFrom(C.wave_base)] = v;
		else if(SPILL) C.spill[(uint32_t)(sp - C.lds_depth) * C.spill_stride + glane] = v;
	};
	for(;;)
	{
		if(node < 0)
		{
			bool got = false;
			for(;;)
			{
				if(j >= total) break;
				cur = j;
				j += stride;
				if(cur < n_a)
				{
					float tw;
					// (ray binning: the entry's ray and hit live at the permuted queue address)
					if(Q.perm) cur = Q.perm[a0 + cur] - a0;
					if(!loadQRay(Q, a0 + cur, o, d, tmin, tw)) continue;
					tmax = (tw >= 0.f) ? tw : inf;
					any = false;
					++n_closest;
				}
				else
				{
					const float4 od = rayLd4(&Q.sh_o[s0 + (cur - n_a)]);
					const float4 dd = rayLd4(&Q.sh_d[s0 + (cur - n_a)]);
					o = xyz(od);
					d = xyz(dd);
					tmin = 0.f;
					tmax = dd.w;
					any = true;
					++n_shadow;
				}
				got = true;
				break;
			}
			if(!got) break;
			V3 dq = d;
			if(fabsf(dq.x) < 1e-20f) dq.x = copysignf(1e-20f, dq.x);
			if(fabsf(dq.y) < 1e-20f) dq.y = copysignf(1e-20f, dq.y);
			if(fabsf(dq.z) < 1e-20f) dq.z = copysignf(1e-20f, dq.z);
			id = v3(rcpExact(dq.x), rcpExact(dq.y), rcpExact(dq.z));
			box_t0 = any ? -1e-3f : (tmin - 1e-3f * (1.f + fabsf(tmin)));
			t_best = tmax;
			prim_best = -1;
			sp = 0;
			node = 0;
		}
		if(STATS) TRACE_STAT(++visits);
		float4 n0, n1, n2, n3, n4;
		if(node < C.n_top)
		{
			typedef float V4 __attribute__((ext_vector_type(4)));
			typedef const __attribute__((address_space(3))) V4 *LdsV4;
			const LdsV4 tp = (LdsV4)(C.top + kTop8Stride * node);
			auto ld = [&](int k) {
				const V4 v = tp[k];
				return make_float4(v.x, v.y, v.z, v.w);
			};
			n0 = ld(0); n1 = ld(1); n2 = ld(2); n3 = ld(3); n4 = ld(4);
		}
		else
		{
			const float4 *np = C.nodes + 8 * node;
			n0 = np[0]; n1 = np[1]; n2 = np[2]; n3 = np[3]; n4 = np[4];
		}
		const uint32_t meta = __float_as_uint(n0.w);
		const uint32_t inner = meta >> 24, leaf = __float_as_uint(n1.x) & 0xffu;
		const int inner_base = __float_as_int(n1.y), tri_base = __float_as_int(n1.z);
		// per axis: t of plane q = q * A + B (A = 2^e / d, B = (origin - o) / d), near / far byte rows by the sign of 1/d
		const float ax = __uint_as_float((meta & 0xffu) << 23) * id.x, ay = __uint_as_float(((meta >> 8) & 0xffu) << 23) * id.y,
		            az = __uint_as_float(((meta >> 16) & 0xffu) << 23) * id.z;
		const float bx = (n0.x - o.x) * id.x, by = (n0.y - o.y) * id.y, bz = (n0.z - o.z) * id.z;
		const bool px = id.x >= 0.f, py = id.y >= 0.f, pz = id.z >= 0.f;
		const uint32_t nx0 = __float_as_uint(px ? n2.x : n2.z), nx1 = __float_as_uint(px ? n2.y : n2.w);
		const uint32_t fx0 = __float_as_uint(px ? n2.z : n2.x), fx1 = __float_as_uint(px ? n2.w : n2.y);
		const uint32_t ny0 = __float_as_uint(py ? n3.x : n3.z), ny1 = __float_as_uint(py ? n3.y : n3.w);
		const uint32_t fy0 = __float_as_uint(py ? n3.z : n3.x), fy1 = __float_as_uint(py ? n3.w : n3.y);
		const uint32_t nz0 = __float_as_uint(pz ? n4.x : n4.z), nz1 = __float_as_uint(pz ? n4.y : n4.w);
		const uint32_t fz0 = __float_as_uint(pz ? n4.z : n4.x), fz1 = __float_as_uint(pz ? n4.w : n4.y);
		const float slack_t = (t_best < 3.0e38f) ? t_best * 1.0000005f + 1e-6f : 3.4e38f;
		float key[8];
		int child[8];
		uint32_t leaves = 0;
#pragma unroll
		for(int k = 0; k < 8; ++k)
		{
			const float lo = fmaxf(fmaxf(__builtin_fmaf(q8Byte(nx0, nx1, k), ax, bx), __builtin_fmaf(q8Byte(ny0, ny1, k), ay, by)),
			                       fmaxf(__builtin_fmaf(q8Byte(nz0, nz1, k), az, bz), box_t0));
			const float hi = fminf(fminf(__builtin_fmaf(q8Byte(fx0, fx1, k), ax, bx), __builtin_fmaf(q8Byte(fy0, fy1, k), ay, by)),
			                       fminf(__builtin_fmaf(q8Byte(fz0, fz1, k), az, bz), slack_t));
			const uint32_t h = lo <= hi ? 1u : 0u;
			const uint32_t isi = (inner >> k) & 1u;
			key[k] = (h & isi) ? lo : inf;
			child[k] = inner_base + __builtin_popcount(inner & ((1u << k) - 1u));
			leaves |= (h & (leaf >> k) & 1u) << k;
		}
		bool done = false;
		for(uint32_t m = leaves; m; m &= m - 1u)
		{
			const int k = __builtin_ctz(m);
			const int q = tri_base + __builtin_popcount(leaf & ((1u << k) - 1u));
			if(STATS) TRACE_STAT(++tests);
			const float4 *tp = C.tris + 3 * q;
			const float4 ta = tp[0], tb = tp[1], tc = tp[2];
			const float t = triTest(ta, tb, tc, o, d, t_best);
			if(t == -1.f) continue;
			const int prim = __float_as_int(tb.w);
			if(any)
			{
				if(t < tmax && t >= 0.f) { t_best = t; prim_best = prim; done = true; break; }
			}
			else if(t >= tmin && (t < t_best || (t == t_best && prim_best >= 0 && prim < prim_best)))
			{
				t_best = t;
				prim_best = prim;
			}
		}
		if(!done && YAF_W8_SORT && YAF_PACKED_SORT)
		{
			// the same network over packed 32-bit keys: the entry distance clamped at 0 with the child's rank
			// among the node's inner children (consecutive from inner_base) in the low 3 bits, compared as
			// unsigned integers (v_min_u32 + v_max_u32 per exchange instead of a compare and four selects; no
			// child array).  The order is a culling heuristic only: closest hits tie-break on the primitive
			// index and any-hit rays answer occluded or not, so the clamp and the 3 dropped mantissa bits
			// change no result.  A missed child is all ones.
			uint32_t pk[8];
#pragma unroll
			for(int k = 0; k < 8; ++k)
				pk[k] = key[k] < inf ? ((__float_as_uint(fmaxf(key[k], 0.f)) & ~7u) | (uint32_t)__builtin_popcount(inner & ((1u << k) - 1u)))
				                     : 0xffffffffu;
			auto cx = [](uint32_t &a, uint32_t &b) {
				const uint32_t lo = min(a, b);
				b = max(a, b);
				a = lo;
			};
			cx(pk[0], pk[1]); cx(pk[2], pk[3]); cx(pk[4], pk[5]); cx(pk[6], pk[7]);
			cx(pk[0], pk[2]); cx(pk[1], pk[3]); cx(pk[4], pk[6]); cx(pk[5], pk[7]);
			cx(pk[1], pk[2]); cx(pk[5], pk[6]);
			cx(pk[0], pk[4]); cx(pk[1], pk[5]); cx(pk[2], pk[6]); cx(pk[3], pk[7]);
			cx(pk[2], pk[4]); cx(pk[3], pk[5]);
			cx(pk[1], pk[2]); cx(pk[3], pk[4]); cx(pk[5], pk[6]);
#pragma unroll
			for(int k = 7; k >= 1; --k)
				if(pk[k] != 0xffffffffu) { push(inner_base + (int)(pk[k] & 7u)); ++sp; }
			int next = pk[0] != 0xffffffffu ? inner_base + (int)(pk[0] & 7u) : -1;
			if(next < 0 && sp > 0)
			{
				--sp;
				next = (!SPILL || sp < C.lds_depth) ? C.stack[sp * kTraceBlock + (int)tidFrom(C.wave_base)]
				                                    : C.spill[(uint32_t)(sp - C.lds_depth) * C.spill_stride + glane];
			}
			node = next;
			done = next < 0;
		}
		else if(!done)
		{
			if(YAF_W8_SORT)
			{
				// Batcher's odd-even merge network (19 compare-exchanges): nearest child descended first, the
				// others pushed farthest first
				cswap(key[0], child[0], key[1], child[1]); cswap(key[2], child[2], key[3], child[3]);
				cswap(key[4], child[4], key[5], child[5]); cswap(key[6], child[6], key[7], child[7]);
				cswap(key[0], child[0], key[2], child[2]); cswap(key[1], child[1], key[3], child[3]);
				cswap(key[4], child[4], key[6], child[6]); cswap(key[5], child[5], key[7], child[7]);
				cswap(key[1], child[1], key[2], child[2]); cswap(key[5], child[5], key[6], child[6]);
				cswap(key[0], child[0], key[4], child[4]); cswap(key[1], child[1], key[5], child[5]);
				cswap(key[2], child[2], key[6], child[6]); cswap(key[3], child[3], key[7], child[7]);
				cswap(key[2], child[2], key[4], child[4]); cswap(key[3], child[3], key[5], child[5]);
				cswap(key[1], child[1], key[2], child[2]); cswap(key[3], child[3], key[4], child[4]);
				cswap(key[5], child[5], key[6], child[6]);
			}
			else
			{
				int kmin = 0;
#pragma unroll
				for(int k = 1; k < 8; ++k) kmin = key[k] < key[kmin] ? k : kmin;
#pragma unroll
				for(int k = 1; k < 8; ++k)
					if(k == kmin) { cswap(key[0], child[0], key[k], child[k]); }
			}
#pragma unroll
			for(int k = 7; k >= 1; --k)
				if(key[k] < inf) { push(child[k]); ++sp; }
			int next = key[0] < inf ? child[0] : -1;
			if(next < 0 && sp > 0)
			{
				--sp;
				next = (!SPILL || sp < C.lds_depth) ? C.stack[sp * kTraceBlock + (int)tidFrom(C.wave_base)]
				                                    : C.spill[(uint32_t)(sp - C.lds_depth) * C.spill_stride + glane];
			}
			node = next;
			done = next < 0;
		}
		if(done)
		{
			if(any) P.occ[__float_as_int(Q.sh_o[s0 + (cur - n_a)].w)] = prim_best >= 0 ? 1 : 0;
			else
			{
				raySt(&Q.hit_t[a0 + cur], t_best);
				raySt(&Q.hit_prim[a0 + cur], prim_best);
			}
			node = -1;
		}
	}
}

template<bool ANY, bool WIDE, bool SPILL = true, bool TS = false, bool STATS = true, bool PACK = false>
__device__ __forceinline__ bool traverse(const TraceCtx &C, V3 o, V3 d, float tmin, float tmax, float &t_best,
                                         int &prim_best, uint32_t &visits, uint32_t &tests, TsList *ts = nullptr)
{
	if(WIDE) return traverse4<ANY, SPILL, TS, STATS, PACK>(C, o, d, tmin, tmax, t_best, prim_best, visits, tests, ts);
	return traverse2<ANY, TS, STATS>(C, o, d, tmin, tmax, t_best, prim_best, visits, tests, ts);
}

// k_trace asks the register allocator for 8 waves per SIMD for LDS-resident scenes (<= 64 VGPRs;
// measured +3% on C2 over the unconstrained 68) and 6 for scenes in global memory, whose refill
// loop (traceRefill4) needs the registers (C4: 226 -> 189 ms of k_trace per frame at 6, spills at 8);
// -DYAF_TRACE_WAVES=n overrides both for tuning
#ifdef YAF_TRACE_WAVES
#define YAF_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(YAF_TRACE_WAVES)))
#else
#ifndef YAF_TRACE8_WAVES
#define YAF_TRACE8_WAVES 6
#endif
#define YAF_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(LDS_SCENE ? 8 : (W8 ? YAF_TRACE8_WAVES : 6))))
#endif

// ---------------------------------------------------------------------------------------------
// Ray-stream sorting.  The queues hold rays in sample order (neighbouring pixels, 64 samples each),
// so the rays of one window of a segment start close together but leave in every direction: lanes
// of one wave then visit different BVH nodes in different orders (C2: 0.42 of the VALU lanes do
// useful work).  Each wave takes a window of kSortWin consecutive queue entries, orders them by a
// key (closest / shadow, direction octant, major axis) with a counting sort in its own LDS slice —
// ranks from ballot-matched key groups, no LDS atomics — and traces them in that order, so a wave
// holds one kind of ray of one octant.  Every ray's query is unchanged (its hit goes back to its
// own queue address), so results are identical to the unsorted loop.
// ---------------------------------------------------------------------------------------------
#ifndef YAF_SORT_PER
#define YAF_SORT_PER 4
#endif
constexpr int kSortPer = YAF_SORT_PER;        // entries per lane and window
constexpr int kSortWin = 64 * kSortPer;
constexpr int kSortBins = 64;                 // = wave width: one bin per lane in the scan

struct WaveSort
{
	uint16_t perm[kSortWin];
	uint32_t base[kSortBins];
};

// kind bit (shadow), octant (3 bits), major axis (0..2); 63 = no ray
__device__ __forceinline__ uint32_t rayKey(const float4 &d, bool shadow)
{
	const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
	const uint32_t major = (ax >= ay && ax >= az) ? 0u : (ay >= az ? 1u : 2u);
	const uint32_t oct = (d.x < 0.f ? 1u : 0u) | (d.y < 0.f ? 2u : 0u) | (d.z < 0.f ? 4u : 0u);
	return (shadow ? 32u : 0u) | (oct << 2) | major;
}

// W.perm = the window's entry indices (0 .. kSortWin-1, entry r * 64 + lane has key[r]) in key order
__device__ __forceinline__ void waveSortWindow(WaveSort &W, const uint32_t (&key)[kSortPer])
{
	const int lane = laneId();
	const uint64_t lt = (1ull << lane) - 1ull;
	W.base[lane] = 0;
	__builtin_amdgcn_wave_barrier();
	uint32_t off[kSortPer];
#pragma unroll
	for(int r = 0; r < kSortPer; ++r)
	{
		const uint32_t k = key[r];
		uint64_t m = ~0ull;
#pragma unroll
		for(int b = 0; b < 6; ++b)
		{
			const bool bit = (k >> b) & 1u;
			const uint64_t bal = __ballot(bit);
			m &= bit ? bal : ~bal;
		}
		const uint32_t below = (uint32_t)__popcll(m & lt);
		const uint32_t old = W.base[k];
		off[r] = old + below;
		__builtin_amdgcn_wave_barrier();
		if(below == 0) W.base[k] = old + (uint32_t)__popcll(m);   // one lane per key group
		__builtin_amdgcn_wave_barrier();
	}
	// exclusive scan of the 64 bin counts, one bin per lane
	const uint32_t c = W.base[lane];
	uint32_t inc = c;
#pragma unroll
	for(int o = 1; o < 64; o <<= 1)
	{
		const uint32_t v = __shfl_up(inc, o);
		if(lane >= o) inc += v;
	}
	__builtin_amdgcn_wave_barrier();
	W.base[lane] = inc - c;
	__builtin_amdgcn_wave_barrier();
#pragma unroll
	for(int r = 0; r < kSortPer; ++r) W.perm[W.base[key[r]] + off[r]] = (uint16_t)(r * 64 + lane);
	__builtin_amdgcn_wave_barrier();
}

// SPILL = false: the whole stack bound fits the LDS levels (no spill column): pushes and pops are
// plain LDS accesses (with a possible spill the compiler merges both address spaces into flat
// accesses, whose pops wait for every outstanding vector-memory operation)
// STATS = false: no per-visit node / triangle counters (timed frames; the counts come from a frame
// rendered with them — the frame is deterministic, so they are the same)
// SORT: ray-stream sorting of each wave's window (above)
// W8: the refill loop over the BVH8 (S.nodes8; global-memory scenes without transparent shadows)
template<bool LDS_SCENE, bool WIDE, bool TS, bool SPILL = true, bool STATS = true, bool SORT = false, bool W8 = false>
__global__ void __launch_bounds__(kTraceBlock) YAF_TRACE_ATTR k_trace(DevScene S, DevQueues Q, DevCounters cnt, DevPaths P,
                                                      DevStats *stats, int stack_depth, int *spill)
{
	extern __shared__ float4 smem[];
	int *stack = reinterpret_cast<int *>(smem);
	TraceCtx C;
	C.wave_base = waveBase();
	C.stack = stack;
	C.lds_depth = stack_depth;
	C.spill = spill;
	C.spill_stride = gridDim.x * blockDim.x;
	if(LDS_SCENE)
	{
		float4 *lds_nodes = smem + (stack_depth * kTraceBlock) / 4;
		float4 *lds_tris = lds_nodes + S.node_f4 * S.n_nodes;
		for(int k = threadIdx.x; k < S.node_f4 * S.n_nodes; k += blockDim.x) lds_nodes[k] = S.nodes[k];
		for(int k = threadIdx.x; k < 3 * S.n_tris; k += blockDim.x) lds_tris[k] = S.tris[k];
		__syncthreads();
		C.nodes = lds_nodes;
		C.tris = lds_tris;
	}
	else
	{
		C.nodes = S.nodes;
		C.tris = S.tris;
		if constexpr(W8)
		{
			C.nodes = S.nodes8;
			C.tris = S.tris8;
			if(S.lds_top8 > 0)
			{
				float4 *top = smem + (stack_depth * kTraceBlock) / 4;
				for(int k = threadIdx.x; k < 5 * S.lds_top8; k += blockDim.x) top[(k / 5) * kTop8Stride + (k % 5)] = S.nodes8[8 * (k / 5) + (k % 5)];
				__syncthreads();
				C.top = top;
				C.n_top = S.lds_top8;
			}
		}
		else if(WIDE && S.lds_top > 0)
		{
			// the top treelet (refill loop only): nodes [0, lds_top) after the stack
			float4 *top = smem + (stack_depth * kTraceBlock) / 4;
			for(int k = threadIdx.x; k < 8 * S.lds_top; k += blockDim.x) top[(k >> 3) * kTopStride + (k & 7)] = S.nodes[k];
			__syncthreads();
			C.top = top;
			C.n_top = S.lds_top;
		}
	}
	const SegLoop L = segLoop(S.n_seg);
	const uint32_t n_a = cnt.n_active[L.s], n_s = cnt.n_shadow[L.s];
	const uint32_t total = n_a + n_s;
	const uint32_t a0 = L.s * S.cap_a, s0 = L.s * S.cap_s;
	uint32_t visits = 0, tests = 0, n_closest = 0, n_shadow = 0;
	// rays traced by traceEntry, counted per wave (ballots into scalar registers): per-lane counters
	// bumped on the two branches were merged into one address-selected increment of a private array,
	// a scratch load + store per ray, or spilled at the 64-VGPR budget
	uint32_t w_closest = 0, w_shadow = 0;
	auto countWave = [&](int kind) {
		w_closest += (uint32_t)__popcll(__ballot(kind == 1));
		w_shadow += (uint32_t)__popcll(__ballot(kind == 2));
	};
	const uint32_t stride = L.nb * blockDim.x;
	// one queue entry: closest ray (j < n_a) or shadow ray (n_a <= j < total)
	auto traceEntry = [&](uint32_t j) -> int {
		if(j < n_a)
		{
			const uint32_t i = a0 + j;
			V3 o, d;
			float tmin, tw;
			if(loadQRay(Q, i, o, d, tmin, tw))   // (a NaN direction marks "no ray this iteration")
			{
				float t;
				int prim;
				const float tmax = (tw >= 0.f) ? tw : __builtin_huge_valf();
				traverse<false, WIDE, SPILL, false, STATS, LDS_SCENE>(C, o, d, tmin, tmax, t, prim, visits, tests);
				raySt(&Q.hit_t[i], t);
				raySt(&Q.hit_prim[i], prim);
				return 1;
			}
		}
		else if(j < total)
		{
			const uint32_t k = s0 + (j - n_a);
			const float4 od = rayLd4(&Q.sh_o[k]), dd = rayLd4(&Q.sh_d[k]);
			float t;
			int prim;
			bool occ;
			if(TS)
			{
				TsList L;
				L.hit = Q.ts_hit + (size_t)k * (uint32_t)S.s_depth;
				L.n = 0;
				L.cap = S.s_depth;
				L.prim_ng = S.prim_ng;
				L.mats = S.mats;
				occ = traverse<true, WIDE, SPILL, true>(C, xyz(od), xyz(dd), od.w, dd.w, t, prim, visits, tests, &L);
				Q.ts_n[k] = occ ? 0 : L.n;
			}
			else occ = traverse<true, WIDE, SPILL, false, STATS>(C, xyz(od), xyz(dd), 0.f, dd.w, t, prim, visits, tests);
			// (opaque shadows: the NEE entry index rides in sh_o.w)
			P.occ[TS ? Q.sh_idx[k] : __float_as_int(od.w)] = occ ? 1 : 0;   // P = state set of the consumer shade
			return 2;
		}
		return 0;
	};
	if constexpr(SORT)
	{
		// wave-private windows of kSortWin entries, dealt round-robin over the segment's waves
		__shared__ WaveSort wsort[kTraceBlock / 64];
		WaveSort &W = wsort[threadIdx.x >> 6];
		const uint32_t nwv = blockDim.x >> 6;
		const uint32_t gw = L.r * nwv + (threadIdx.x >> 6), nw = L.nb * nwv;
		for(uint32_t w0 = gw * kSortWin; w0 < total; w0 += nw * kSortWin)
		{
			uint32_t key[kSortPer];
#pragma unroll
			for(int r = 0; r < kSortPer; ++r)
			{
				const uint32_t j = w0 + (uint32_t)(r * 64) + laneId();
				uint32_t k = kSortBins - 1;
				if(j < n_a)
				{
					const F3 dd = reinterpret_cast<const F3 *>(Q.ray_d)[a0 + j];
					if(!(dd.x != dd.x)) k = rayKey(make_float4(dd.x, dd.y, dd.z, 0.f), false);
				}
				else if(j < total) k = rayKey(Q.sh_d[s0 + (j - n_a)], true);
				key[r] = k;
			}
			waveSortWindow(W, key);
#pragma unroll 1
			for(int r = 0; r < kSortPer; ++r) countWave(traceEntry(w0 + W.perm[r * 64 + laneId()]));
		}
	}
	else
	{
#ifdef YAF_TRACE_NOREFILL
	// the BVH8 (quantised 80-B nodes, its own triangle order) is only walked by traceRefill8; traceEntry
	// reads C.nodes as a BVH4
	static_assert(!W8, "YAF_TRACE_NOREFILL builds cannot traverse the quantised BVH8: set YAFARAY_AMD_BVH8=0 and drop the W8 instantiations");
#else
	// refill pays where traversals are long (meshes in global memory: C4 -16%); on the short
	// LDS-resident traversals of small scenes its per-visit bookkeeping costs more (C2 +35%)
	if(W8)
		traceRefill8<true, STATS>(C, Q, P, n_a, total, a0, s0, L.r * blockDim.x + threadIdx.x, stride, visits, tests, n_closest, n_shadow);
	else if(!LDS_SCENE && WIDE && !TS)
		traceRefill4<true, STATS>(C, Q, P, n_a, total, a0, s0, L.r * blockDim.x + threadIdx.x, stride, visits, tests, n_closest, n_shadow);
	else
#endif
	// one uniform trip count per workgroup so every lane reaches the same exits (the lane's thread index
	// re-derived per entry: threadIdx.x kept live across the traversal was spilled and reloaded per visit)
	for(uint32_t base = L.r * blockDim.x; base < total; base += stride) countWave(traceEntry(base + (YAF_LANE_REMAT ? tidFrom(C.wave_base) : threadIdx.x)));
	}
	if(laneId() == 0)
	{
		n_closest += w_closest;
		n_shadow += w_shadow;
	}
	// statistics (rays issued, nodes visited, triangles tested): wave reduce, then one plain
	// read-modify-write per workgroup into its own record (no atomics: the same block index owns
	// the same record in every launch of the stream; summed on the host after the render)
	for(int off = 32; off > 0; off >>= 1)
	{
		visits += __shfl_down(visits, off);
		tests += __shfl_down(tests, off);
		n_closest += __shfl_down(n_closest, off);
		n_shadow += __shfl_down(n_shadow, off);
	}
	__shared__ uint32_t red[kTraceBlock / 64][4];
	const int wid = threadIdx.x >> 6;
	if(laneId() == 0) { red[wid][0] = visits; red[wid][1] = tests; red[wid][2] = n_closest; red[wid][3] = n_shadow; }
	__syncthreads();
	if(threadIdx.x < 4)
	{
		unsigned long long v = 0;
		for(int w = 0; w < kTraceBlock / 64; ++w) v += red[w][threadIdx.x];
		unsigned long long *rec = &stats[blockIdx.x].closest_rays;
		const int slot = (threadIdx.x == 0) ? 2 : (threadIdx.x == 1) ? 3 : (threadIdx.x == 2) ? 0 : 1;
		if(v) rec[slot] += v;
	}
}

// ---------------------------------------------------------------------------------------------
// k_trace_brute (opt-in, YAFARAY_AMD_TRACE=brute; measured slower than the BVH on C2, see
// render.cc): the same queries for scenes of at most kBruteTris triangles by testing every triangle — the reference's own AcceleratorSimpleTest semantics
// (accelerator_simple_test.cc:61-139; closest = the lowest (t, primitive) in [tmin, tmax), any =
// a hit in [0, tmax)), which equal the BVH's by construction.  The triangle loop is wave-uniform:
// the vertices come through scalar loads shared by the 64 lanes, every lane does the same
// arithmetic (no divergence, no stack), and a shadow wave stops when all its lanes are occluded.
// ---------------------------------------------------------------------------------------------
constexpr int kBruteTris = 64;
#ifdef YAF_EXPERIMENTS

template<bool ANY>
__device__ __forceinline__ bool bruteTrace(const float4 *__restrict__ tris, int n_tris, V3 o, V3 d, float tmin, float tmax, float &t_best,
                                           int &prim_best, uint32_t &tests, bool active)
{
	t_best = tmax;
	prim_best = -1;
	bool hit = false;
	for(int q = 0; q < n_tris; ++q)
	{
		// wave-uniform index through the constant address space -> scalar loads (the K$ holds the
		// whole scene)
#ifdef __HIP_DEVICE_COMPILE__
		typedef const float4 __attribute__((address_space(4))) *ConstF4;
		const ConstF4 ct = (ConstF4)tris;
		const int qs = __builtin_amdgcn_readfirstlane(q);
		const float4 ta = ct[3 * qs], tb = ct[3 * qs + 1], tc = ct[3 * qs + 2];
#else   // (host pass of the single-source compile: never executed)
		const float4 ta = tris[3 * q], tb = tris[3 * q + 1], tc = tris[3 * q + 2];
#endif
		const float t = triTest(ta, tb, tc, o, d, t_best);
		const int prim = __float_as_int(tb.w);
		if(ANY)
		{
			if(!hit && t != -1.f && t < tmax && t >= 0.f) { hit = true; t_best = t; prim_best = prim; }
			if((q & 3) == 3 && __all(hit || !active)) break;
		}
		else if(t != -1.f && t >= tmin && (t < t_best || (t == t_best && prim_best >= 0 && prim < prim_best)))
		{
			t_best = t;
			prim_best = prim;
		}
	}
	if(active) tests += (uint32_t)n_tris;
	return prim_best >= 0;
}

__global__ void __launch_bounds__(kTraceBlock) k_trace_brute(DevScene S, DevQueues Q, DevCounters cnt, DevPaths P, DevStats *stats)
{
	const float4 *__restrict__ tris = S.tris;
	const int n_tris = S.n_tris;
	const SegLoop L = segLoop(S.n_seg);
	const uint32_t n_a = cnt.n_active[L.s], n_s = cnt.n_shadow[L.s];
	const uint32_t total = n_a + n_s;
	const uint32_t a0 = L.s * S.cap_a, s0 = L.s * S.cap_s;
	uint32_t tests = 0, n_closest = 0, n_shadow = 0;
	const uint32_t stride = L.nb * blockDim.x;
	// closest rays fill the first n_a positions, shadow rays the rest: a wave is (almost always)
	// all closest or all shadow, and runs one of the two uniform loops
	for(uint32_t base = L.r * blockDim.x; base < total; base += stride)
	{
		const uint32_t j = base + threadIdx.x;
		const bool closest = j < n_a, shadow = !closest && j < total;
		if(__any(closest))
		{
			V3 o = v3(0.f, 0.f, 0.f), d = v3(0.f, 0.f, 1.f);
			float tmin = 0.f, tw = -1.f;
			const bool ray = closest && loadQRay(Q, a0 + j, o, d, tmin, tw);   // NaN direction: no ray this iteration
			if(!ray) { o = v3(0.f, 0.f, 0.f); d = v3(0.f, 0.f, 1.f); }
			float t;
			int prim;
			const float tmax = (tw >= 0.f) ? tw : __builtin_huge_valf();
			bruteTrace<false>(tris, n_tris, o, d, tmin, tmax, t, prim, tests, ray);
			if(ray)
			{
				Q.hit_t[a0 + j] = t;
				Q.hit_prim[a0 + j] = prim;
				++n_closest;
			}
		}
		if(__any(shadow))
		{
			float4 od = make_float4(0.f, 0.f, 0.f, 0.f), dd = make_float4(0.f, 0.f, 1.f, 0.f);
			const uint32_t k = s0 + (j - n_a);
			if(shadow) { od = Q.sh_o[k]; dd = Q.sh_d[k]; }
			float t;
			int prim;
			const bool occ = bruteTrace<true>(tris, n_tris, xyz(od), xyz(dd), 0.f, dd.w, t, prim, tests, shadow);
			if(shadow)
			{
				P.occ[__float_as_int(od.w)] = occ ? 1 : 0;   // P = state set of the consumer shade (index in sh_o.w)
				++n_shadow;
			}
		}
	}
	for(int off = 32; off > 0; off >>= 1)
	{
		tests += __shfl_down(tests, off);
		n_closest += __shfl_down(n_closest, off);
		n_shadow += __shfl_down(n_shadow, off);
	}
	__shared__ uint32_t red[kTraceBlock / 64][3];
	const int wid = threadIdx.x >> 6;
	if(laneId() == 0) { red[wid][0] = tests; red[wid][1] = n_closest; red[wid][2] = n_shadow; }
	__syncthreads();
	if(threadIdx.x < 3)
	{
		unsigned long long v = 0;
		for(int w = 0; w < kTraceBlock / 64; ++w) v += red[w][threadIdx.x];
		unsigned long long *rec = &stats[blockIdx.x].closest_rays;
		const int slot = (threadIdx.x == 0) ? 3 : (threadIdx.x == 1) ? 0 : 1;   // tri_tests, closest, shadow
		if(v) rec[slot] += v;
	}
}
#endif   // YAF_EXPERIMENTS (k_trace_brute)

// ---------------------------------------------------------------------------------------------
// k_shade
// ---------------------------------------------------------------------------------------------
struct Surf
{
	V3 p, n, ng, nu, nv;
	int mat;
	uint32_t flags;
	C3 dcol;          // diffuse shader colour (read by EXT kernels only)
	float drefl;      // diffuse_refl_shader scalar
	float sigma;      // sigma_oren_shader scalar (Oren-Nayar with a texture sigma)
};

// Surface attributes computed by k_surface for the hit (texeval.h): shading normal + frame,
// diffuse shader colour and diffuse_refl scalar
__device__ __forceinline__ void applyAttr(Surf &s, const float4 &a0, const float4 &a1)
{
	s.n = v3(a0.x, a0.y, a0.z);
	coordsSystem(s.n, s.nu, s.nv);
	s.drefl = a0.w;
	s.dcol = C3{a1.x, a1.y, a1.z};
	s.sigma = a1.w;
}

__device__ __forceinline__ Surf makeSurf(const DevScene &S, V3 o, V3 d, float t, int prim)
{
	// accelerator.cc:61 hit point + primitive_triangle.cc:97-176 (flat shading: N = Ng)
	Surf s;
	s.p = o + t * d;
	const float4 g = S.prim_ng[prim];
	s.ng = xyz(g);
	s.n = s.ng;
	coordsSystem(s.n, s.nu, s.nv);
	s.mat = __float_as_int(g.w);
	s.flags = S.mats[s.mat].bsdf_flags;
	const DevMaterial &m = S.mats[s.mat];
	s.dcol = C3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};   // read only by EXT kernels
	s.drefl = 1.f;
	s.sigma = 0.f;
	return s;
}

__device__ __forceinline__ V3 faceForward(V3 ng, V3 n, V3 wo) { return (dot(ng, wo) < 0) ? -n : n; }

// ---- materials ----
// Non-EXT kernels only see diffuse shinydiffuse / light_mat (the configs' materials) and keep the
// lean arithmetic; EXT kernels run the whole ShinyDiffuseMaterial (mirror / transparent /
// translucent / diffuse components with Fresnel, shader-node colours) and the mirror / null
// materials (material_glass.cc:435-475).

// material_shiny_diffuse.cc:102-114
__device__ __forceinline__ float fresnelKr(const DevMaterial &m, V3 wo, V3 n)
{
	if(!(m.sd_flags & SD_FRESNEL)) return 1.f;
	const V3 N = (dot(wo, n) < 0.f) ? -n : n;
	const float c = dot(wo, N);
	float g = m.ior_sq + c * c - 1.f;
	if(g < 0.f) g = 0.f;
	else g = sqrtf(g);
	const float aux = c * (g + c);
	return ((0.5f * (g - c) * (g - c)) / ((g + c) * (g + c))) * (1.f + ((aux - 1) * (aux - 1)) / ((aux + 1) * (aux + 1)));
}

// vector.h:255-260
__device__ __forceinline__ V3 reflectDir(V3 normal, V3 v)
{
	const float vn = dot(v, normal);
	if(vn < 0.f) return -v;
	return 2.f * vn * normal - v;
}

// material_shiny_diffuse.cc:154-188 ShinyDiffuseMaterial::orenNayar(wi, wo, n, use_texture_sigma,
// texture_sigma): float arithmetic with the A / B members, or double arithmetic with a texture sigma
__device__ float orenNayar(V3 wi, V3 wo, V3 n, const DevMaterial &m, const Surf &sp)
{
	const float cos_ti = fmaxf(-1.f, fminf(1.f, dot(n, wi)));
	const float cos_to = fmaxf(-1.f, fminf(1.f, dot(n, wo)));
	float maxcos_f = 0.f;
	if(cos_ti < 0.9999f && cos_to < 0.9999f)
	{
		const V3 v_1 = normalize(wi - n * cos_ti);
		const V3 v_2 = normalize(wo - n * cos_to);
		maxcos_f = fmaxf(0.f, dot(v_1, v_2));
	}
	float sin_alpha, tan_beta;
	if(cos_to >= cos_ti)
	{
		sin_alpha = sqrtf(1.f - cos_ti * cos_ti);
		tan_beta = sqrtf(1.f - cos_to * cos_to) / ((cos_to == 0.f) ? 1e-8f : cos_to);
	}
	else
	{
		sin_alpha = sqrtf(1.f - cos_to * cos_to);
		tan_beta = sqrtf(1.f - cos_ti * cos_ti) / ((cos_ti == 0.f) ? 1e-8f : cos_ti);
	}
	if(m.sigma_root >= 0)
	{
		const double texture_sigma = (double)sp.sigma;
		const double sigma_squared = texture_sigma * texture_sigma;
		const double a = 1.0 - 0.5 * (sigma_squared / (sigma_squared + 0.33));
		const double b = 0.45 * sigma_squared / (sigma_squared + 0.09);
		return fminf(1.f, fmaxf(0.f, (float)(a + b * (double)maxcos_f * (double)sin_alpha * (double)tan_beta)));
	}
	return fminf(1.f, fmaxf(0.f, m.on_a + m.on_b * maxcos_f * sin_alpha * tan_beta));
}

// material_shiny_diffuse.cc:190-238 (eval), material_simple.cc / material_glass.cc (black)
template<bool EXT = false>
__device__ C3 matEval(const DevMaterial &m, const Surf &sp, V3 wo, V3 wl, uint32_t bsdfs)
{
	if(m.type != MAT_SHINYDIFFUSE) return c3(0.f);
	const V3 n = faceForward(sp.ng, sp.n, wo);
	if(!(bsdfs & (m.bsdf_flags & B_DIFFUSE))) return c3(0.f);
	const C3 dcol = EXT ? sp.dcol : C3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
	if(!EXT)
	{
		const float m_t = (1.f - 1.f * m.comp[0]) * (1.f - m.comp[1]);
		if((double)dot(n, wl) < 0.0 && !m.flat) return c3(0.f);
		const float m_d = m_t * (1.f - m.comp[2]) * m.comp[3];
		return m_d * dcol;
	}
	const float cos_ng_wo = dot(sp.ng, wo);
	const float cos_ng_wl = dot(sp.ng, wl);
	const float kr = fresnelKr(m, wo, n);
	const float m_t = (1.f - kr * m.comp[0]) * (1.f - m.comp[1]);
	const bool transmit = (cos_ng_wo * cos_ng_wl) < 0.f;
	if(transmit && (m.sd_flags & SD_TRANSLUCENT)) return m.comp[2] * m_t * dcol;
	if((double)dot(n, wl) < 0.0 && !m.flat) return c3(0.f);
	float m_d = m_t * (1.f - m.comp[2]) * m.comp[3];
	if(m.sd_flags & SD_OREN_NAYAR) m_d *= orenNayar(wo, wl, n, m, sp);   // :228-233
	if(m.drefl_root >= 0) m_d *= sp.drefl;   // :235
	return m_d * dcol;
}

// material_shiny_diffuse.cc:242-247, material_simple.cc:50-55
template<bool EXT = false>
__device__ C3 matEmit(const DevMaterial &m, const Surf &sp, V3 wo)
{
	if(m.type == MAT_LIGHT)
	{
		if(m.double_sided) return C3{m.emit[0], m.emit[1], m.emit[2]};
		return dot(wo, sp.n) > 0 ? C3{m.emit[0], m.emit[1], m.emit[2]} : c3(0.f);
	}
	if(EXT && m.type != MAT_SHINYDIFFUSE) return c3(0.f);
	if(EXT && m.diffuse_root >= 0) return sp.dcol * m.emit_strength;
	return C3{m.emit[0], m.emit[1], m.emit[2]};
}

// material_shiny_diffuse.cc:107-119 (accumulate with the Fresnel factor kr)
__device__ __forceinline__ void accumulateComp(const float *c, float kr, float *a)
{
	a[0] = c[0] * kr;
	float acc = 1.f - a[0];
	a[1] = c[1] * acc;
	acc *= 1.f - c[1];
	a[2] = c[2] * acc;
	acc *= 1.f - c[2];
	a[3] = c[3] * acc;
}

// material_shiny_diffuse.cc:457-475 getAlpha
__device__ __forceinline__ float matAlpha(const DevMaterial &m, const Surf &sp, V3 wo)
{
	if(!(m.sd_flags & SD_TRANSPARENT)) return 1.f;
	const V3 n = faceForward(sp.ng, sp.n, wo);
	const float kr = fresnelKr(m, wo, n);
	const float refl = (1.f - m.comp[0] * kr) * m.comp[1];
	return 1.f - refl;
}

struct BsdfSample
{
	float s_1, s_2, pdf;
	uint32_t flags, sampled;
};

// material_shiny_diffuse.cc:249-337, material_simple.cc:42-48, material_glass.cc:435-468
template<bool EXT = false>
__device__ C3 matSample(const DevMaterial &m, const Surf &sp, V3 wo, V3 &wi, BsdfSample &s, float &w)
{
	if(m.type == MAT_LIGHT || (EXT && m.type == MAT_NULL))
	{
		s.pdf = 0.f;
		w = 0.f;
		return c3(0.f);
	}
	if(EXT && m.type == MAT_MIRROR)
	{
		wi = reflectDir(sp.n, wo);
		s.sampled = B_SPECULAR | B_REFLECT;
		w = 1.f;
		return C3{m.mirror_col[0], m.mirror_col[1], m.mirror_col[2]} * rcpExact(fabsf(dot(sp.n, wi)));
	}
	const float cos_ng_wo = dot(sp.ng, wo);
	const V3 n = faceForward(sp.ng, sp.n, wo);
	float accum_c[4];
	accumulateComp(m.comp, EXT ? fresnelKr(m, wo, n) : 1.f, accum_c);
	float sum = 0.f, val[4], width[4];
	uint32_t choice[4];
	int n_match = 0, pick = -1;
	for(int i = 0; i < (int)m.n_bsdf; ++i)
	{
		if((s.flags & m.c_flags[i]) == m.c_flags[i])
		{
			width[n_match] = accum_c[m.c_index[i]];
			sum += width[n_match];
			choice[n_match] = m.c_flags[i];
			val[n_match] = sum;
			++n_match;
		}
	}
	if(!n_match || (double)sum < 0.00001) { s.sampled = B_NONE; s.pdf = 0.f; return c3(1.f); }
	const float inv_sum = 1.f / sum;
	for(int i = 0; i < n_match; ++i)
	{
		val[i] *= inv_sum;
		width[i] *= inv_sum;
		if((s.s_1 <= val[i]) && (pick < 0)) pick = i;
	}
	if(pick < 0) pick = n_match - 1;
	float s_1;
	if(pick > 0) s_1 = (s.s_1 - val[pick - 1]) / width[pick];
	else s_1 = s.s_1 / width[pick];
	const C3 dcol = EXT ? sp.dcol : C3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
	C3 scolor = c3(0.f);
	const uint32_t ch = choice[pick];
	if(EXT && ch == (B_SPECULAR | B_REFLECT))
	{
		wi = reflectDir(n, wo);
		s.pdf = width[pick];
		scolor = C3{m.mirror_col[0], m.mirror_col[1], m.mirror_col[2]} * (accum_c[0]);
		scolor = scolor * rcpExact(fmaxf(fabsf(dot(sp.n, wi)), 1.0e-6f));
	}
	else if(EXT && ch == (B_TRANSMIT | B_FILTER))
	{
		wi = -wo;
		scolor = accum_c[1] * (m.tfilter * dcol + c3(1.f - m.tfilter));
		if((double)fabsf(dot(wi, n)) < 1e-6) s.pdf = 0.f;
		else s.pdf = width[pick];
	}
	else if(EXT && ch == (B_DIFFUSE | B_TRANSMIT))
	{
		wi = cosHemisphere(-n, sp.nu, sp.nv, s_1, s.s_2);
		if(cos_ng_wo * dot(sp.ng, wi) < 0) scolor = accum_c[2] * dcol;
		s.pdf = fabsf(dot(wi, n)) * width[pick];
	}
	else
	{
		wi = cosHemisphere(n, sp.nu, sp.nv, s_1, s.s_2);
		if(cos_ng_wo * dot(sp.ng, wi) > 0) scolor = accum_c[3] * dcol;
		if(EXT && (m.sd_flags & SD_OREN_NAYAR)) scolor = scolor * orenNayar(wo, wi, n, m, sp);   // :320-325
		s.pdf = fabsf(dot(wi, n)) * width[pick];
	}
	s.sampled = ch;
	w = fabsf(dot(wi, sp.n)) / (s.pdf * 0.99f + 0.01f);
	const float alpha = EXT ? matAlpha(m, sp, wo) : 1.f;
	w = w * (alpha) + 1.f * (1.f - alpha);
	return scolor;
}

// material_shiny_diffuse.cc:339-377
template<bool EXT = false>
__device__ float matPdf(const DevMaterial &m, const Surf &sp, V3 wo, V3 wi, uint32_t bsdfs)
{
	if(m.type != MAT_SHINYDIFFUSE) return 0.f;
	if(!(bsdfs & B_DIFFUSE)) return 0.f;
	float pdf = 0.f;
	const float cos_ng_wo = dot(sp.ng, wo);
	const V3 n = faceForward(sp.ng, sp.n, wo);
	float accum_c[4];
	accumulateComp(m.comp, EXT ? fresnelKr(m, wo, n) : 1.f, accum_c);
	float sum = 0.f;
	int n_match = 0;
	for(int i = 0; i < (int)m.n_bsdf; ++i)
	{
		if(bsdfs & m.c_flags[i])
		{
			const float width = accum_c[m.c_index[i]];
			sum += width;
			if(m.c_flags[i] == (B_DIFFUSE | B_REFLECT)) pdf += fabsf(dot(wi, n)) * width;
			else if(EXT && m.c_flags[i] == (B_DIFFUSE | B_TRANSMIT) && cos_ng_wo * dot(sp.ng, wi) < 0) pdf += fabsf(dot(wi, n)) * width;
			++n_match;
		}
	}
	if(!n_match || (double)sum < 0.00001) return 0.f;
	return pdf / sum;
}

// getSpecular: material_shiny_diffuse.cc:390-433, material_glass.cc:443-451 (mirror)
struct SpecOut
{
	bool refl, refr;
	V3 rdir, tdir;
	C3 rcol, tcol;
};
__device__ SpecOut matSpecular(const DevMaterial &m, const Surf &sp, V3 wo)
{
	SpecOut o;
	o.refl = o.refr = false;
	o.rdir = o.tdir = v3(0.f, 0.f, 0.f);
	o.rcol = o.tcol = c3(0.f);
	if(m.type == MAT_MIRROR)
	{
		o.refl = true;
		o.rcol = C3{m.mirror_col[0], m.mirror_col[1], m.mirror_col[2]};
		o.rdir = reflectDir(faceForward(sp.ng, sp.n, wo), wo);
		return o;
	}
	if(m.type != MAT_SHINYDIFFUSE) return o;
	const bool backface = dot(wo, sp.ng) < 0.f;
	const V3 n = backface ? -sp.n : sp.n;
	const V3 ng = backface ? -sp.ng : sp.ng;
	const float kr = fresnelKr(m, wo, n);
	if(m.sd_flags & SD_TRANSPARENT)
	{
		o.refr = true;
		o.tdir = -wo;
		const C3 tcol = m.tfilter * sp.dcol + c3(1.f - m.tfilter);
		o.tcol = (1.f - m.comp[0] * kr) * m.comp[1] * tcol;
	}
	if(m.sd_flags & SD_MIRROR)
	{
		o.refl = true;
		const float vn = 2.f * (wo.x * n.x + wo.y * n.y + wo.z * n.z);   // Vec3::reflect (vector.h:227-232)
		V3 d = v3(vn * n.x - wo.x, vn * n.y - wo.y, vn * n.z - wo.z);
		const float cos_wi_ng = dot(d, ng);
		if((double)cos_wi_ng < 0.01)
		{
			const float f = (float)(0.01 - (double)cos_wi_ng);
			d = v3(d.x + f * ng.x, d.y + f * ng.y, d.z + f * ng.z);
			d = normalize(d);
		}
		o.rdir = d;
		o.rcol = C3{m.mirror_col[0], m.mirror_col[1], m.mirror_col[2]} * (m.comp[0] * kr);
	}
	return o;
}

__device__ __forceinline__ V3 lv(const float *a) { return v3(a[0], a[1], a[2]); }

// light_area.cc:116-135
__device__ __forceinline__ bool areaTri(V3 a, V3 b, V3 c, V3 o, V3 d, float &t)
{
	const V3 edge_1 = b - a;
	const V3 edge_2 = c - a;
	const V3 pvec = cross(d, edge_2);
	const float det = dot(edge_1, pvec);
	if(det == 0.f) return false;
	const float inv_det = rcpExact(det);
	const V3 tvec = o - a;
	const float u = dot(tvec, pvec) * inv_det;
	if(u < 0.f || u > 1.f) return false;
	const V3 qvec = cross(tvec, edge_1);
	const float v = dot(d, qvec) * inv_det;
	if((v < 0.f) || ((u + v) > 1.f)) return false;
	t = dot(edge_2, qvec) * inv_det;
	return true;
}

struct ShadeOut;
__device__ __forceinline__ void emitShadow(bool want, V3 o, V3 d, float t_max, float tmin, int idx, const ShadeOut &out);

// where neeLight's shadow rays go: ShadeOut appends them to the next queue (k_trace traces them);
// k_path's emitter keeps them per lane and traces them in place
struct ShadeOut
{
	uint32_t *sh_count;    // shadow-ray counter of the shard
	uint32_t sh_base;      // first address of the shard's shadow queue
	DevQueues Qn;
	bool idx_in_o;         // opaque shadows: the NEE entry index rides in sh_o.w (no sh_idx array traffic);
	                       // transparent shadows keep tmin there (k_tshadow) and the index in sh_idx
	__device__ __forceinline__ void emit(bool want, V3 o, V3 d, float t_max, float tmin, int idx) const
	{
		emitShadow(want, o, d, t_max, tmin, idx, *this);
	}
};

// estimateOneDirectLight's light pick (integrator_montecarlo.cc:70-78): lnum = the light that
// Halton(2, base_sampling_offset + n - 1).getNext() selects, where the reference's n is a per-thread
// running counter of the calls (integrator_tiled.cc:48, reset at render start, :169-171) — its value
// depends on which samples the thread rendered before, i.e. on the thread schedule.  Here n of a call
// is u * stride + local: u hashes the pixel's sampling offset and the sample number (PixelSamplingData,
// so the pick does not depend on how the film is split across GPUs or chunks), local counts the
// calls of the sample's path (depth + subpath * bounces), and the stride is odd, so the low bits of
// n — which decide the leading digits of the radical inverse, hence the light — run through every
// residue as u varies: every light is picked with its 1 / num_lights share at every depth.  (A
// counter that is the same for every sample — local alone — picks the same light at a given depth
// for the whole film: a biased image once there are >= 2 lights.)  Path tracing uses the reference's
// one-thread counter instead (DevScene::lpc); this pick serves final gathering and recursion trees.
// The light of the call whose running counter is n: Halton(2, base_sampling_offset + n - 1).getNext()
// (integrator_montecarlo.cc:74-75).
__device__ __forceinline__ uint32_t lightOfCounter(const DevScene &S, uint32_t n)
{
	const float hv = haltonFirst(2u, 0.5, S.base_offset + n - 1u);
	return (uint32_t)min((int)(hv * (float)S.n_lights), S.n_lights - 1);
}

__device__ __forceinline__ uint32_t mix32(uint32_t h)
{
	h ^= h >> 16;
	h *= 0x7feb352du;
	h ^= h >> 15;
	h *= 0x846ca68bu;
	h ^= h >> 16;
	return h;
}

// Russian roulette draw (path_tracer.cc:249-251: random_generator(), the reference's per-tile
// generator seeded from rand() — schedule-dependent, so RR is matched statistically): a
// hash of the sample's pixel-major global id (as k_camera's seed), the RR seed, the pass, the subpath
// and the bounce.  Stateless: the compact path record carries no generator state (8 B instead of 16
// per vertex each way), and the image does not depend on how the film is split over GPUs or chunks.
__device__ __forceinline__ float rrRandom(const DevScene &S, const SampleCoord &sc, uint32_t subpath, int depth)
{
	const uint64_t gid = ((uint64_t)sc.y * (uint64_t)S.width + (uint64_t)sc.x) * (uint64_t)S.spp + (uint64_t)sc.s;
	uint32_t h = mix32((uint32_t)gid ^ mix32((uint32_t)(gid >> 32) ^ S.rr_seed ^ (S.pass_offset * 0x9e3779b9u)));
	h = mix32(h ^ (subpath * 0x85ebca6bu + (uint32_t)depth * 0xc2b2ae35u));
	return (float)((double)h * kSampleMultRatio);
}

__device__ __forceinline__ uint32_t pickLight(const DevScene &S, uint32_t offset, uint32_t sample_idx, uint32_t local, uint32_t stride)
{
	if(S.n_lights <= 1) return 0u;
	// hashed, not linear in the sample number: the sample's low-discrepancy dimensions (sub-pixel
	// position, BSDF directions) are functions of the same number, and a pick that follows its low
	// bits would select one light for one stratum of directions — a biased image
	const uint32_t u = mix32(offset ^ mix32(sample_idx + 0x9E3779B9u));
	const float hv = haltonFirst(2u, 0.5, S.base_offset + (u * (stride | 1u) + local) - 1u);
	return (uint32_t)min((int)(hv * (float)S.n_lights), S.n_lights - 1);
}

// Appends (or not) one shadow ray per lane — every lane of the wave must call.
__device__ __forceinline__ void emitShadow(bool want, V3 o, V3 d, float t_max, float tmin, int idx, const ShadeOut &out)
{
	const uint32_t k = out.sh_base + waveAppend(want, out.sh_count);
	if(want)
	{
		stStore2(&out.Qn.sh_o[k], f4(o, out.idx_in_o ? __int_as_float(idx) : tmin));
		stStore2(&out.Qn.sh_d[k], f4(d, t_max));
		if(!out.idx_in_o) stStore2(&out.Qn.sh_idx[k], idx);
	}
}

// accelerator.cc:69-78: origin moved by tmin, t_max = tmax - 2 tmin (tmax >= 0) else inf
__device__ __forceinline__ void shadowRayOf(V3 from, V3 dir, float tmin, float tmax, V3 &o, float &t_max)
{
	o = from + dir * tmin;
	t_max = (tmax >= 0.f) ? tmax - 2 * tmin : __builtin_huge_valf();
}

// Transparent shadows: the factors of an NEE contribution whose light colour k_tshadow still has
// to filter (integrator_montecarlo.cc:122, 212, 335: `lcol *= scol` comes before the products)
__device__ __forceinline__ void tsFactors(float4 *ts, int e, C3 surf, float a, C3 lcol, float b, float c, bool div)
{
	ts[3 * (size_t)e] = f4(surf, a);
	ts[3 * (size_t)e + 1] = f4(lcol, b);
	ts[3 * (size_t)e + 2] = make_float4(c, div ? 1.f : 0.f, 0.f, 0.f);
}

// Next-event estimation for one light: writes the contributions of every sample into
// nee[base ...] and emits the shadow rays.  integrator_montecarlo.cc:80-408.
// Wave-uniform structure: `active` lanes do the work, every lane of the wave walks the same loop
// bounds (the shadow-ray appends are wave-level).
// ---- meshlight / objectlight (light_object_light.cc) ----
// ObjectLight::sampleSurface (:89-107): a face by the area distribution (Pdf1D::dSample, a
// lower_bound over the cdf), s_1 rescaled inside its cdf step, then TrianglePrimitive::sample
// (primitive_triangle.cc:220-234) and the face's geometric normal
__device__ __forceinline__ void meshSampleSurface(const DevScene &S, const DevLight &L, float s_1, float s_2, V3 &p, V3 &n)
{
	const float *cdf = S.mesh_cdf + L.mesh0;
	const int nt = (int)L.mesh_n;
	int k;
	if(s_1 <= 0.f) k = 0;
	else if(s_1 >= 1.f) k = nt - 1;
	else
	{
		int lo = 0, hi = nt;   // first index with cdf >= s_1 (std::lower_bound)
		while(lo < hi)
		{
			const int mid = (lo + hi) >> 1;
			if(cdf[mid] < s_1) lo = mid + 1;
			else hi = mid;
		}
		k = lo;
	}
	if(k >= nt)
	{
		// the reference's "Sampling error" branch: default point and normal
		p = v3(0.f, 0.f, 0.f);
		n = p;
		return;
	}
	float delta = cdf[k], ss_1;
	if(k > 0)
	{
		delta -= cdf[k - 1];
		ss_1 = (s_1 - cdf[k - 1]) / delta;
	}
	else ss_1 = s_1 / delta;
	const float4 *t = S.mesh_tris + (size_t)kMeshTriF4 * (L.mesh0 + (uint32_t)k);
	const V3 v0 = xyz(t[3]), v1 = xyz(t[4]), v2 = xyz(t[5]);
	n = xyz(t[6]);
	const float su_1 = sqrtf(ss_1);
	const float u = 1.f - su_1;
	const float v = s_2 * su_1;
	p = (u * v0 + v * v1) + (1.f - u - v) * v2;
}

// The light-sample half of areaLightSampleLight for an area light (light_area.cc:66-96) or a mesh
// light (light_object_light.cc:111-146): direction and distance to the sampled point and the pdf.
template<bool NOMESH = false>
__device__ __forceinline__ bool lightIllumSample(const DevScene &S, const DevLight &L, V3 sp_p, float s_1, float s_2, V3 &ldir, float &dist, float &pdf)
{
	V3 p, fn;
	if(!NOMESH && L.type == LIGHT_MESH) meshSampleSurface(S, L, s_1, s_2, p, fn);
	else
	{
		p = lv(L.pos) + s_1 * lv(L.to_x) + s_2 * lv(L.to_y);
		fn = lv(L.fnormal);
	}
	ldir = p - sp_p;
	const float dist_sqr = lengthSqr(ldir);
	dist = sqrtf(dist_sqr);
	if((double)dist <= 0.0) return false;
	ldir = ldir * rcpExact(dist);
	if(!NOMESH && L.type == LIGHT_MESH)
	{
		float cos_angle = -dot(ldir, fn);
		if(cos_angle <= 0)
		{
			if(L.double_sided) cos_angle = -cos_angle;
			else return false;
		}
		const float amc = L.area * cos_angle;
		pdf = x87mulDiv(kPi, dist_sqr, (amc == 0.f) ? 1e-8f : amc);
		return true;
	}
	const float cos_angle = dot(ldir, fn);
	if(cos_angle <= 0) return false;
	pdf = x87mulDiv(kPi, dist_sqr, L.area * cos_angle);
	return true;
}

// The closest face of a meshlight along (p, dir) with t >= tmin through the light's BVH2 (its faces'
// own tree, as the reference's per-light kd-tree, light_object_light.cc:62-70, 186-204): the same exact
// triangle test and the same answer as testing every face in creation order — the smallest t, equal t
// resolved to the lowest face index; boxes are culled conservatively (padded at build time, relative
// slack on t).  Returns the face index or -1.  A private per-lane stack (the tree is <= 60 levels deep).
__device__ int meshLightClosest(const DevScene &S, const DevLight &L, V3 o, V3 d, float tmin)
{
	const float4 *nodes = S.mesh_nodes + 4 * (size_t)L.bvh_node0;
	const float4 *tris = S.mesh_btris + 3 * (size_t)L.bvh_tri0;
	V3 dd = d;
	if(fabsf(dd.x) < 1e-20f) dd.x = copysignf(1e-20f, dd.x);
	if(fabsf(dd.y) < 1e-20f) dd.y = copysignf(1e-20f, dd.y);
	if(fabsf(dd.z) < 1e-20f) dd.z = copysignf(1e-20f, dd.z);
	const V3 id = v3(rcpExact(dd.x), rcpExact(dd.y), rcpExact(dd.z));
	const float box_t0 = tmin - 1e-3f * (1.f + fabsf(tmin));
	float t_best = __builtin_huge_valf();
	int best = -1;
	int stk[64];
	int sp = 0, node = 0;
	for(;;)
	{
		const float4 *np = nodes + 4 * node;
		const float4 n0 = np[0], n1 = np[1], n2 = np[2], n3 = np[3];
		const float slack_t = (t_best < 3.0e38f) ? t_best * 1.0000005f + 1e-6f : 3.4e38f;
		bool h0, h1;
		float tn0, tn1;
		boxPair(n0, n1, n2, o, id, box_t0, slack_t, h0, h1, tn0, tn1);
		const int c0 = __float_as_int(n3.x), c1 = __float_as_int(n3.y), k0 = __float_as_int(n3.z), k1 = __float_as_int(n3.w);
#pragma unroll
		for(int side = 0; side < 2; ++side)
		{
			const bool h = side ? h1 : h0;
			const int c = side ? c1 : c0, k = side ? k1 : k0;
			if(!h || c >= 0 || k == 0) continue;
			for(int q = ~c; q < ~c + k; ++q)
			{
				const float4 ta = tris[3 * q], tb = tris[3 * q + 1], tc = tris[3 * q + 2];
				const float t = triTest(ta, tb, tc, o, d, t_best);
				const int face = __float_as_int(tb.w);
				if(t != -1.f && t >= tmin && (t < t_best || (t == t_best && face < best)))
				{
					t_best = t;
					best = face;
				}
			}
		}
		const bool i0 = h0 && c0 >= 0, i1 = h1 && c1 >= 0;
		int next = -1;
		if(i0 && i1)
		{
			const bool first0 = tn0 <= tn1;
			next = first0 ? c0 : c1;
			stk[sp++] = first0 ? c1 : c0;
		}
		else if(i0) next = c0;
		else if(i1) next = c1;
		if(next < 0)
		{
			if(sp == 0) break;
			next = stk[--sp];
		}
		node = next;
	}
	return best;
}

// Light::intersect of areaLightSampleMaterial's material-sampled ray (origin p, direction dir, tmin
// b_tmin): the light's pdf and the shadow ray's t (< 0: unbounded).  Area light: light_area.cc:137-151.
// Mesh light: light_object_light.cc:183-201 — the closest face (the light's own kd-tree, faces with
// t >= tmin) gives the normal; the reference never stores the hit distance in `t` (the caller's ray
// tmax, -1), so 1 / (t * t) is 1 and the shadow ray is unbounded: both reproduced.
template<bool NOMESH = false>
__device__ __forceinline__ bool lightMatHit(const DevScene &S, const DevLight &L, V3 p, V3 dir, float b_tmin, float &t, float &light_pdf)
{
	if(!NOMESH && L.type == LIGHT_MESH)
	{
		float t_best = __builtin_huge_valf();
		int best = -1;
		const float4 *tr = S.mesh_tris + (size_t)kMeshTriF4 * L.mesh0;
		if(L.bvh_depth > 0) best = meshLightClosest(S, L, p, dir, b_tmin);
		else
			for(int k = 0; k < (int)L.mesh_n; ++k)
			{
				const float th = triTest(tr[kMeshTriF4 * k], tr[kMeshTriF4 * k + 1], tr[kMeshTriF4 * k + 2], p, dir, t_best);
				if(th != -1.f && th >= b_tmin && th < t_best)
				{
					t_best = th;
					best = k;
				}
			}
		if(best < 0) return false;
		const V3 n = xyz(tr[kMeshTriF4 * best + 6]);
		float cos_angle = -dot(dir, n);
		if(cos_angle <= 0.f)
		{
			if(L.double_sided) cos_angle = fabsf(cos_angle);
			else return false;
		}
		t = -1.f;
		light_pdf = x87mul(kDiv1ByPi, 1.f * L.area * cos_angle);
		return true;
	}
	const V3 fn = lv(L.fnormal);
	const float cos_angle = dot(dir, fn);
	if(cos_angle <= 0) return false;
	if(!areaTri(lv(L.pos), lv(L.c2), lv(L.c3), p, dir, t))
	{
		if(!areaTri(lv(L.pos), lv(L.c3), lv(L.c4), p, dir, t)) return false;
	}
	if(!(t > 1.0e-10f)) return false;
	light_pdf = x87mul(kDiv1ByPi, rcpExact(t * t) * L.area * cos_angle);
	return true;
}

// NEE contribution slots.  In HBM (DevPaths::nee) a 12-B colour record per entry: an entry without a
// valid sample gets its occlusion byte set (k_trace writes the bytes of emitted shadow rays only), so
// the connection's `valid && !occluded` test is the occlusion byte alone; the AO entries' pdf goes to
// nee_aw.  The megakernel's LDS slots keep float4 (contribution, valid) — and the byte, too.
struct NeeHbm
{
	float *c;
	float *aw;
};
__device__ __forceinline__ NeeHbm neeHbm(const DevPaths &P) { return NeeHbm{P.nee, P.nee_aw}; }
__device__ __forceinline__ void neePut(float4 *nee, uint8_t *occ, int e, C3 c, bool ok)
{
	nee[e] = f4(c, ok ? 1.f : 0.f);
	occ[e] = ok ? 0 : 1;
}
#ifndef YAF_NEE_SKIP_INVALID
#define YAF_NEE_SKIP_INVALID 1
#endif
__device__ __forceinline__ void neePut(const NeeHbm &nee, uint8_t *occ, int e, C3 c, bool ok)
{
	// an entry without a sample (most material-sampled entries: the direction misses the light) writes its
	// occlusion byte only — every reader tests the byte before it uses the record (neeSumT, aoSum)
	if(!YAF_NEE_SKIP_INVALID || ok) reinterpret_cast<F3 *>(nee.c)[e] = F3{c.r, c.g, c.b};
	occ[e] = ok ? 0 : 1;
}
__device__ __forceinline__ C3 neeGet(const NeeHbm &nee, int e)
{
	const F3 c = reinterpret_cast<const F3 *>(nee.c)[e];
	return C3{c.x, c.y, c.z};
}

// NOMESH: the scene has no meshlight (k_nee's lean instantiation drops that code)
template<bool EXT, class Out, class NeeT, bool NOMESH = false>
__device__ void neeLight(const DevScene &S, const DevLight &L, const DevMaterial &m, const Surf &sp, V3 wo,
                         uint32_t loffs, uint32_t sample_idx, uint32_t offset, bool active, int e0,
                         NeeT nee, uint8_t *occ, const Out &out, float4 *ts = nullptr)
{
	const bool cast_shadows = L.cast_shadows && m.receive_shadows;
	const float p_len = length(sp.p);
	const float sh_tmin = S.shadow_bias_auto ? S.shadow_bias * fmaxf(1.f, p_len) : S.shadow_bias;
	if(L.type == LIGHT_POINT)
	{
		// light_point.cc:38-57 + montecarlo.cc:80-154
		bool ok = active;
		C3 contrib = c3(0.f);
		V3 ldir = lv(L.pos) - sp.p;
		const float dist_sqr = ldir.x * ldir.x + ldir.y * ldir.y + ldir.z * ldir.z;
		const float dist = sqrtf(dist_sqr);
		if((double)dist == 0.0) ok = false;
		V3 so = sp.p;
		float st = 0.f;
		if(ok)
		{
			const float idist_sqr = rcpExact(dist_sqr);
			ldir = ldir * rcpExact(dist);
			const C3 lcol = C3{L.color[0], L.color[1], L.color[2]} * idist_sqr;
			const float angle = m.flat ? 1.f : fabsf(dot(sp.n, ldir));
			const C3 surf_col = matEval<EXT>(m, sp, wo, ldir, B_ALL);
			const C3 transmit = c3(1.f);
			contrib = surf_col * lcol * angle * transmit;
			shadowRayOf(sp.p, ldir, sh_tmin, dist, so, st);
			if(ts && cast_shadows) tsFactors(ts, e0, surf_col, angle, lcol, 1.f, 1.f, false);
		}
		if(active) neePut(nee, occ, e0, contrib, ok);
		out.emit(ok && cast_shadows, so, ldir, st, sh_tmin, e0);
		return;
	}
	// area light: montecarlo.cc:393-405
	const uint32_t l_offs = loffs * 4567u;
	const int num_samples = L.samples;
	const uint32_t offs = (uint32_t)num_samples * sample_idx + offset + l_offs;
	const C3 lcolor = C3{L.color[0], L.color[1], L.color[2]};
	// areaLightSampleLight (montecarlo.cc:156-282) and areaLightSampleMaterial (:284-383) draw the
	// same Halton(2/3) sequences from setStart(offs - 1) (:399-403): computed once for both
	HaltonInc<2> hal_2;
	HaltonInc<3> hal_3;
	hal_2.value = hal_3.value = 0.0;
	if(active)
	{
		hal_2.start(offs - 1u);
		hal_3.start(offs - 1u);
	}
	for(int i = 0; i < num_samples; ++i)
	{
		float s_1 = 0.f, s_2 = 0.f;
		if(active)
		{
			s_1 = hal_2.next();
			s_2 = hal_3.next();
		}
		bool ok = active;
		C3 contrib = c3(0.f);
		V3 so = sp.p, ldir = v3(0.f, 0.f, 1.f);
		float st = 0.f;
		if(ok)
		{
			// light_area.cc:66-96 / light_object_light.cc:111-146
			float dist = 0.f, pdf = 0.f;
			ok = lightIllumSample<NOMESH>(S, L, sp.p, s_1, s_2, ldir, dist, pdf);
			if(ok)
			{
				if(pdf > 1e-6f)
				{
					const C3 surf_col = matEval<EXT>(m, sp, wo, ldir, B_ALL);
					const float angle = m.flat ? 1.f : fabsf(dot(sp.n, ldir));
					float w = 1.f;
					const float m_pdf = matPdf<EXT>(m, sp, wo, ldir, B_GLOSSY | B_DIFFUSE | B_DISPERSIVE | B_REFLECT | B_TRANSMIT);
					if(m_pdf > 1e-6f)
					{
						const float l_2 = pdf * pdf;
						const float m_2 = m_pdf * m_pdf;
						w = l_2 / (l_2 + m_2);
					}
					contrib = surf_col * lcolor * angle * w / pdf;
					shadowRayOf(sp.p, ldir, sh_tmin, dist, so, st);
					if(ts && cast_shadows) tsFactors(ts, e0 + i, surf_col, angle, lcolor, w, pdf, true);
				}
				else ok = false;
			}
		}
		if(active) neePut(nee, occ, e0 + i, contrib, ok);
		out.emit(ok && cast_shadows, so, ldir, st, sh_tmin, e0 + i);

		// areaLightSampleMaterial (montecarlo.cc:284-383)
		ok = active;
		contrib = c3(0.f);
		so = sp.p;
		V3 dir = v3(0.f, 0.f, 1.f);
		st = 0.f;
		const float b_tmin = S.ray_min_dist_auto ? S.ray_min_dist * fmaxf(1.f, p_len) : S.ray_min_dist;
		if(ok)
		{
			BsdfSample s;
			s.s_1 = s_1;
			s.s_2 = s_2;
			s.flags = B_GLOSSY | B_DIFFUSE | B_DISPERSIVE | B_REFLECT | B_TRANSMIT;
			s.pdf = 0.f;
			s.sampled = B_NONE;
			float W = 0.f;
			const C3 surf_col = matSample<EXT>(m, sp, wo, dir, s, W);
			ok = s.pdf > 1e-6f;
			float t = 0.f, lpdf = 0.f;
			if(ok)
			{
				// light_area.cc:137-151
				// light_area.cc:137-151 / light_object_light.cc:183-201
				ok = lightMatHit<NOMESH>(S, L, sp.p, dir, b_tmin, t, lpdf);
			}
			if(ok)
			{
				const float light_pdf = lpdf;
				if(light_pdf > 1e-6f)
				{
					const float l_pdf = rcpExact(light_pdf);
					const float l_2 = l_pdf * l_pdf;
					const float m_2 = s.pdf * s.pdf;
					const float w = m_2 / (l_2 + m_2);
					contrib = surf_col * lcolor * w * W;
					shadowRayOf(sp.p, dir, b_tmin, t, so, st);
					if(ts && cast_shadows) tsFactors(ts, e0 + num_samples + i, surf_col, w, lcolor, W, 1.f, false);
				}
				else ok = false;
			}
		}
		if(active) neePut(nee, occ, e0 + num_samples + i, contrib, ok);
		out.emit(ok && cast_shadows, so, dir, st, b_tmin, e0 + num_samples + i);
	}
}

// TiledIntegrator::sampleAmbientOcclusion (integrator_tiled.cc:644-691; clay = false, one ray
// division): one entry per AO sample after the lights' entries — (ao_col * surf_col * cos * w, pdf)
// — and its shadow ray (tmin = shadow bias, tmax = AO_distance).  The material sample keeps the
// previous direction when it draws none (light_ray.dir_ persists, :647); such samples weigh 0.
template<bool EXT>
__device__ void aoSamples(const DevScene &S, const DevMaterial &m, const Surf &sp, V3 wo, uint32_t sample_idx, uint32_t offset,
                          bool active, int e0, const NeeHbm &nee, uint8_t *occ, const ShadeOut &out, float4 *ts)
{
	const int n = S.ao_samples;
	const uint32_t offs = (uint32_t)n * sample_idx + offset;
	HaltonInc<2> hal_2;
	HaltonInc<3> hal_3;
	hal_2.value = hal_3.value = 0.0;
	if(active)
	{
		hal_2.start(offs - 1u);
		hal_3.start(offs - 1u);
	}
	const float sh_tmin = S.shadow_bias_auto ? S.shadow_bias * fmaxf(1.f, length(sp.p)) : S.shadow_bias;
	const C3 ao_col = C3{S.ao_col[0], S.ao_col[1], S.ao_col[2]};
	V3 dir = v3(0.f, 0.f, 0.f);
	for(int i = 0; i < n; ++i)
	{
		bool want = false;
		V3 so = sp.p;
		float st = 0.f;
		if(active)
		{
			BsdfSample s;
			s.s_1 = hal_2.next();
			s.s_2 = hal_3.next();
			s.flags = B_GLOSSY | B_DIFFUSE | B_REFLECT;
			s.pdf = 0.f;
			s.sampled = B_NONE;
			float w = 0.f;
			const C3 surf_col = matSample<EXT>(m, sp, wo, dir, s, w);
			const float cos = fabsf(dot(sp.n, dir));
			const C3 contrib = ao_col * surf_col * cos * w;
			// a zero contribution does not depend on the occlusion: no ray
			want = !(contrib.r == 0.f && contrib.g == 0.f && contrib.b == 0.f);
			shadowRayOf(sp.p, dir, sh_tmin, S.ao_dist, so, st);
			if(ts && want) tsFactors(ts, e0 + i, surf_col, cos, ao_col, w, 1.f, false);
			reinterpret_cast<F3 *>(nee.c)[e0 + i] = F3{contrib.r, contrib.g, contrib.b};
			nee.aw[e0 + i] = s.pdf;
			occ[e0 + i] = 0;
		}
		emitShadow(want, so, dir, st, sh_tmin, e0 + i, out);
	}
}

// AO result of a vertex: sum in sample order of emit * pdf (emitting materials) and the unoccluded
// contributions, divided by the sample count (integrator_tiled.cc:672-690)
__device__ C3 aoSum(const DevScene &S, const NeeHbm &nee, const uint8_t *occ, int k0, bool emitting, C3 emit)
{
	C3 col = c3(0.f);
	for(int i = 0; i < S.ao_samples; ++i)
	{
		if(emitting) col = col + emit * nee.aw[k0 + i];
		if(!occ[k0 + i]) col = col + neeGet(nee, k0 + i);
	}
	return col / (float)S.ao_samples;
}

// Sum of one light's entries with the reference's addition order (montecarlo.cc:385-408).
// ge(k) / go(k): NEE entry k and its occlusion byte (from memory, or from values loaded earlier)
template<class GetE, class GetO>
__device__ __forceinline__ C3 neeSumT(const DevLight &L, int k0, GetE ge, GetO go)
{
	if(L.type == LIGHT_POINT)
	{
		const float4 e = ge(k0);
		C3 c = c3(0.f);
		if(e.w != 0.f && !go(k0)) c = c + rgb(e);
		return c3(0.f) + c;
	}
	C3 acc_l = c3(0.f), acc_m = c3(0.f);
	for(int i = 0; i < L.samples; ++i)
	{
		const float4 e = ge(k0 + i);
		if(e.w != 0.f && !go(k0 + i)) acc_l = acc_l + rgb(e);
	}
	for(int i = 0; i < L.samples; ++i)
	{
		const float4 e = ge(k0 + L.samples + i);
		if(e.w != 0.f && !go(k0 + L.samples + i)) acc_m = acc_m + rgb(e);
	}
	const C3 col_l = acc_l * L.inv_samples;
	const C3 col_m = acc_m * L.inv_samples;
	return (c3(0.f) + col_l) + col_m;
}

__device__ C3 neeSum(const DevScene &S, const DevLight &L, const float4 *nee, const uint8_t *occ, int k0)
{
	return neeSumT(L, k0, [&](int k) { return nee[k]; }, [&](int k) { return occ[k] != 0; });
}

__device__ __forceinline__ float ldsDim(const DevScene &S, int dim, uint32_t n)
{
	const uint4 fd = S.faure_dim[dim];
	UDiv dv;
	dv.m = fd.z;
	dv.sh = fd.w;
	return (float)lowDiscrepancy(S.faure + fd.y, fd.x, dv, S.faure_inv[dim], n);
}

// k_shade / k_nee stage their per-sample lookup tables in LDS once per workgroup: the Faure
// permutations and dimension descriptors (every Halton draw of the path sampler), and for small
// scenes the materials and per-primitive normals (every hit).  The returned scene copy points at
// the LDS copies, so the shading code reads them at LDS latency instead of L2 latency.
__device__ __forceinline__ void copy16(uint4 *dst, const void *src, int n)
{
	const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
	for(int k = threadIdx.x; k < n; k += blockDim.x) dst[k] = s4[k];
}

// scenes whose primitive records do not fit (C4) still get their materials in LDS when those are small:
// the material read after each hit's primitive record is then an LDS access, not a second L2 round trip
#ifndef YAF_STAGE_MATS
#define YAF_STAGE_MATS 1
#endif
constexpr size_t kStageMatsMax = 8192;
__host__ __device__ inline bool stageMatsOnly(const DevScene &S, bool small)
{
	return YAF_STAGE_MATS && !small && (size_t)S.n_mats * sizeof(DevMaterial) <= kStageMatsMax;
}
__host__ __device__ inline size_t shadeLdsBytes(const DevScene &S, bool small)
{
	size_t b = 50 * 16 + 25 * 16 + (size_t)S.faure_bytes;
	if(small) b += (size_t)S.n_mats * sizeof(DevMaterial) + (size_t)S.n_tris * 16;
	else if(stageMatsOnly(S, small)) b += (size_t)S.n_mats * sizeof(DevMaterial);
	return b;
}

template<bool SMALL>
__device__ __forceinline__ DevScene stageTables(const DevScene &G, uint4 *smem)
{
	DevScene S = G;
	uint4 *p = smem;
	copy16(p, G.faure_dim, 50);
	S.faure_dim = p;
	p += 50;
	copy16(p, G.faure_inv, 25);
	S.faure_inv = reinterpret_cast<const double *>(p);
	p += 25;
	if(SMALL)
	{
		const int nm = G.n_mats * (int)(sizeof(DevMaterial) / 16);
		copy16(p, G.mats, nm);
		S.mats = reinterpret_cast<const DevMaterial *>(p);
		p += nm;
		copy16(p, G.prim_ng, G.n_tris);
		S.prim_ng = reinterpret_cast<const float4 *>(p);
		p += G.n_tris;
	}
	else if(stageMatsOnly(G, false))
	{
		const int nm = G.n_mats * (int)(sizeof(DevMaterial) / 16);
		copy16(p, G.mats, nm);
		S.mats = reinterpret_cast<const DevMaterial *>(p);
		p += nm;
	}
	copy16(p, G.faure, G.faure_bytes / 16);
	S.faure = reinterpret_cast<const uint8_t *>(p);
	__syncthreads();
	return S;
}

struct ShadeArgs
{
	DevScene S;
	DevPaths Pc;         // state of the current active list (indexed by queue position)
	DevPaths Pn;         // state of the next active list (written at the compacted position)
	DevQueues Q;         // current (active list + hits)
	DevQueues Qn;        // next
	DevNeeQueue N;       // NEE requests for k_nee
	DevNeeQueue G;       // photon-map estimate requests for k_gather (gather_on)
	DevCounters cnt;     // counts of the current queue
	DevCounters cnt_next;
	float4 *samples;     // frame sample buffer [(y * W + x) * spp + s]
	const DevJob *jobs;
	int n_jobs;
	uint64_t chunk_base;
};

__device__ __forceinline__ void writeSampleAt(const ShadeArgs &A, const SampleCoord &sc, C3 col, float alpha)
{
	if(alpha > 1.f) alpha = 1.f;   // integrator_tiled.cc:399
	A.samples[((size_t)sc.y * A.S.width + sc.x) * A.S.spp + sc.s] = f4(col, alpha);
}

__device__ __forceinline__ void writeSample(const ShadeArgs &A, uint32_t sid, C3 col, float alpha)
{
	writeSampleAt(A, sampleAt(A.S, A.jobs, A.n_jobs, A.chunk_base + (uint64_t)sid), col, alpha);
}

// First hit v0 of a later subpath, rebuilt from the primitive stored with the camera hit.
__device__ __forceinline__ Surf surfFromPrim(const DevScene &S, V3 p, int prim)
{
	Surf s;
	s.p = p;
	const float4 g = S.prim_ng[prim];
	s.ng = xyz(g);
	s.n = s.ng;
	coordsSystem(s.n, s.nu, s.nv);
	s.mat = __float_as_int(g.w);
	s.flags = S.mats[s.mat].bsdf_flags;
	const DevMaterial &m = S.mats[s.mat];
	s.dcol = C3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
	s.drefl = 1.f;
	s.sigma = 0.f;
	return s;
}

// MonteCarloIntegrator::recursiveRaytrace (integrator_montecarlo.cc:925-968) for the integrate()
// node `node` hit at ray level S.cur_level: the specular reflect / refract children of ray level
// cur_level + 1 are appended to the spawn list (traced by the next pass) and linked to the node;
// k_combine later adds their totals times the specular colours, reflect first.
// additional_depth: the value integrate() received (max over the ancestors' materials, carried in the
// spawned ray's tmax as -1 - depth); the node's own material raises it (direct_light.cc:107,
// path_tracer.cc:133) and the children inherit it.
__device__ void spawnSpecular(const DevScene &S, const DevMaterial &m, const Surf &sp, V3 wo, uint32_t node, uint2 pix, uint2 rng,
                              int additional_depth)
{
	int2 child = make_int2(-1, -1);
	const int level = S.cur_level + 1;
	additional_depth = max(additional_depth, m.add_depth);
	if((sp.flags & (B_SPECULAR | B_FILTER)) && level <= S.raydepth + additional_depth && level < 20)
	{
		const SpecOut so = matSpecular(m, sp, wo);
		for(int k = 0; k < 2; ++k)
		{
			const bool want = k == 0 ? so.refl : so.refr;
			if(!want) continue;
			const uint32_t idx = atomicAdd(&S.spawn_count[0], 1u);
			if(idx >= S.spawn_cap) { atomicOr(&S.spawn_count[1], 1u); continue; }
			V3 from = sp.p;
			const V3 dir = k == 0 ? so.rdir : so.tdir;
			if(k == 1 && m.tbias > 0.f)
			{
				// specularRefract (:890-898): origin pushed along the refracted direction
				float f = m.tbias;
				if(m.sd_flags & SD_TBIAS_MULT) f *= (float)level;
				from = sp.p + dir * f;
			}
			S.spawn_o[idx] = f4(from, S.ray_min_dist);
			S.spawn_d[idx] = f4(dir, -1.f - (float)additional_depth);   // tmax < 0: unbounded ray
			// the child's own Russian-roulette stream (statistical parity, as the camera's)
			S.spawn_pr[idx] = make_uint4(pix.x, pix.y, rng.x ^ (0x9e3779b9u * (uint32_t)(2 * level + k + 1)), rng.y + 1u + (uint32_t)k);
			S.node_w[S.node_base + idx] = f4(k == 0 ? so.rcol : so.tcol, 0.f);
			if(k == 0) child.x = (int)(S.node_base + idx);
			else child.y = (int)(S.node_base + idx);
		}
	}
	S.node_child[node] = child;
}

// One path vertex per active queue entry.  Control flow restates PathIntegrator::integrate
// (integrator_path_tracer.cc:120-290) / DirectLightIntegrator::integrate (:97-144) as a state
// machine whose vertices are processed one iteration at a time:
//   1. connect the estimate left pending by the previous vertex (its shadow rays were traced
//      by this iteration's k_trace) — additions happen in the reference's order;
//   2. shade the new hit (camera hit v0, first segment hit v1, or bounce hit);
//   3. sample the next segment, or end the subpath (next subpath / finalize);
//   4. wave-ballot compaction: the entry's state moves to its position in the next queue
//      (coalesced SoA reads and writes, no indirection);
//   5. next-event estimation into the next state: contributions + shadow rays.
// FUSED (the non-EXT instantiations): step 5 runs the next-event estimation in place instead of
// queueing requests for k_nee — the NEE request round trip through HBM (48 B written + read per
// vertex) and one launch per iteration disappear; the shade loop is HBM-bound, so the light
// sampling arithmetic overlaps its memory traffic.
// LEAN: the plain path tracer (PathIntegrator, one path per sample, no AO / photon maps / caustic map /
// gather queue) with those scene switches fixed at compile time, so the other integrators' state
// (first-hit records, gather requests, AO sums) costs no registers (launch_shade picks it)
// DEFER (lpc_mode 3, r06): estimateOneDirectLight's light pick in the one-thread order without a count run —
// every addition to the path colour (the pending light estimate with its throughput and emission, or a term known
// at once) is written as a record chained per sample instead of being added; k_dfr_* pick the lights once the
// pass's counter bases are known, estimate them, and fold the records in order (the same additions)
template<bool SMALL, bool EXT, bool FUSED = false, bool LEAN = false, bool DEFER = false>
__global__ void __launch_bounds__(kShadeBlock, EXT ? 1 : (LEAN ? YAF_SHADE_LEAN_WAVES : YAF_SHADE_MIN_WAVES)) k_shade(ShadeArgs A)
{
	extern __shared__ uint4 shade_smem[];
	DevScene S_ = stageTables<SMALL>(A.S, shade_smem);
	if constexpr(LEAN)
	{
		S_.integrator = INT_PATH;
		S_.path_samples = 1;
		S_.do_ao = 0;
		S_.caus_map = 0;
		S_.show_map = 0;
		S_.gather_on = 0;
		S_.n_photons = 0;
		S_.fg_on = 0;
		S_.tree = 0;
		S_.has_attr = 0;
	}
	const DevScene S = S_;
	const bool ATTR = EXT && S.has_attr != 0;   // k_surface output present
	const DevPaths &Pc = A.Pc;
	const DevPaths &Pn = A.Pn;
	// workgroup b works on segment b and appends to segment b of the next queue
	const uint32_t seg = blockIdx.x;
	const uint32_t n_a = A.cnt.n_active[seg];
	const uint32_t a0 = seg * S.cap_a;
	__shared__ uint32_t s_count[4];   // next active entries, NEE requests, shadow rays (FUSED), gather requests
	if(threadIdx.x < 4) s_count[threadIdx.x] = 0;
	__syncthreads();
	ShadeOut out;
	out.sh_count = &s_count[2];
	out.sh_base = seg * S.cap_s;
	out.Qn = A.Qn;
	out.idx_in_o = !S.tr_shad;
	const bool is_path = S.integrator == INT_PATH;
	const bool is_photon = S.integrator == INT_PHOTON;
	// first-hit data carried to the end (the photon-map estimates of k_gather read it)
	const bool keep_v0 = S.path_samples > 1 || is_photon || S.caus_map;
	// DirectLight with a caustic map: causticPhotons() comes between the direct light and the AO
	// (integrator_direct_light.cc:120-124), so the AO sum rides with the gather request
	const bool ao_after_caustic = S.caus_map && S.integrator == INT_DIRECT;
	const uint32_t n_paths = (uint32_t)max(1, S.path_samples);
	const int K = S.nee_k;
	const uint32_t stride = blockDim.x;
	// compact record (every render without a specular recursion tree): pr = (sample id, stage, MWC);
	// the pixel and its sampling offsets are recomputed from the sample id, the first-vertex estimate
	// lives in csmp[sample id] (written when it changes, read where it is used) instead of travelling
	// with every vertex
	const bool compact = !(EXT && S.tree);
	PHASE_DECL
#if YAF_SHADE_PREFETCH
	// the next iteration's compact record (the head of the entry's dependent load chain) is loaded while
	// this one is shaded
	uint2 pr_n = make_uint2(0u, ST_NORAY);
	if(compact && threadIdx.x < n_a) pr_n = reinterpret_cast<const uint2 *>(Pc.pr)[a0 + threadIdx.x];
#endif
	for(uint32_t base_j = 0; base_j < n_a; base_j += stride)
	{
		const bool live = base_j + threadIdx.x < n_a;
		const uint32_t i = a0 + base_j + threadIdx.x;   // address of the entry (shard base + position)
#if YAF_SHADE_PREFETCH
		const uint2 pr_cur = pr_n;
		if(compact && base_j + stride + threadIdx.x < n_a) pr_n = reinterpret_cast<const uint2 *>(Pc.pr)[i + stride];
#endif
		// ---- 0. load the entry (coalesced loads; stage, flags and w ride in the .w lanes) ----
		uint32_t sid = 0, stage = ST_NORAY, flags = 0;
		uint2 pix = make_uint2(0u, 0u), rng = make_uint2(0u, 0u);
		float w = 0.f;
		float4 thr4 = make_float4(0.f, 0.f, 0.f, 0.f), col4 = thr4, pcol4 = thr4, pwo4 = thr4, pthr4 = thr4, pem4 = thr4;
		float4 v0p4 = thr4, v0wo4 = thr4;
		float4 v0a0 = thr4, v0a1 = thr4;   // first-hit surface attributes (ATTR && keep_v0)
		SampleCoord sc{0, 0, 0};
		if(live)
		{
			if(compact)
			{
				// compact record: (sample id, stage), 8 B — the RR draw is a hash (rrRandom)
#if YAF_SHADE_PREFETCH
				const uint2 pr = pr_cur;
#else
				const uint2 pr = reinterpret_cast<const uint2 *>(Pc.pr)[i];
#endif
				sid = pr.x;
				stage = pr.y;
				sc = sampleAt(S, A.jobs, A.n_jobs, A.chunk_base + (uint64_t)sid);
				pix = make_uint2(fnv32((uint32_t)(sc.y + S.crop_y0) * fnv32((uint32_t)(sc.x + S.crop_x0))),
				                 S.base_offset + S.pass_offset + (uint32_t)sc.s);
			}
			else
			{
				const uint4 pr = Pc.pr[i];
				rng = make_uint2(pr.z, pr.w);
				sid = (uint32_t)A.Q.slot[i];
				pix = make_uint2(pr.x, pr.y);
				col4 = Pc.col[i];
				stage = __float_as_uint(col4.w);
			}
			// a compact camera entry starts from zero throughput, colour, w and flags (k_camera does not
			// write them) and has no first-hit data yet
			if(!compact || (stage & 0xffu) != ST_CAMERA)
			{
				if(S.w_live) thr4 = Pc.thr[i];
				else
				{
					// w is set by every sample() of this scene before it is read: a 12-B throughput record
					const F3 t = reinterpret_cast<const F3 *>(Pc.thr)[i];
					thr4 = make_float4(t.x, t.y, t.z, 0.f);
				}
				pcol4 = Pc.pcol[i];
				if(keep_v0) { v0p4 = Pc.v0p[i]; v0wo4 = Pc.v0wo[i]; }
				if(ATTR && keep_v0) { v0a0 = Pc.v0attr[2 * (size_t)i]; v0a1 = Pc.v0attr[2 * (size_t)i + 1]; }
			}
			w = thr4.w;
			flags = __float_as_uint(pcol4.w);
			// only the first segment of a subpath reads the previous wo (path_tracer.cc:193-197)
			if((stage & 0xffu) == ST_FIRST) pwo4 = Pc.pwo[i];
			if(flags & F_PEND_ONE)
			{
				const F3 t = reinterpret_cast<const F3 *>(Pc.pend_thr)[i];
				pthr4 = make_float4(t.x, t.y, t.z, 0.f);
			}
			if(flags & (F_PEND_EMIT | F_AO_EMIT)) pem4 = Pc.pend_emit[i];
		}
		C3 thr = rgb(thr4), col = rgb(col4), pcol = rgb(pcol4);
		const float alpha = 1.f;   // live entries are opaque (transparent background is written at ST_CAMERA)
		V3 pwo = xyz(pwo4);
		const uint32_t st = stage & 0xffu;
		uint32_t subpath = (stage >> 8) & 0xfffu;
		int depth = (int)(stage >> 20);
		const uint32_t offset = pix.x, sample_idx = pix.y;
		C3 ao_extra = c3(0.f);
		// compact record: col comes from csmp on first use; col_dirty = changed this iteration
		bool col_ld = !compact, col_dirty = false;
		auto loadCol = [&]() {
			if(!col_ld)
			{
				col = (flags & F_COLS) ? rgb(Pc.csmp[sid]) : c3(0.f);
				col_ld = true;
			}
		};

		PHASE(0);
		// ---- 1. connect the pending next-event estimate ----
		const int kb = (int)i * K;
		// (HBM slots: validity is in the occlusion byte)
		auto ge = [&](int k) { return f4(neeGet(neeHbm(Pc), k), 1.f); };
		auto go = [&](int k) { return Pc.occ[k] != 0; };
		if(live && (flags & F_PEND_V0))
		{
			loadCol();
			col_dirty = true;
			// estimateAllDirectLight (montecarlo.cc:54-68): col += sum over lights in name order
			C3 total = c3(0.f);
			for(int l = 0; l < S.n_lights; ++l) total = total + neeSumT(S.lights[l], kb + (int)S.lights[l].nee_base, ge, go);
			col = col + total;
			// DirectLight: col += sampleAmbientOcclusion (integrator_direct_light.cc:124)
			if(S.do_ao)
			{
				const C3 ao = aoSum(S, neeHbm(Pc), Pc.occ, (int)i * K + S.nee_all_count, (flags & F_AO_EMIT) != 0, rgb(pem4));
				if(ao_after_caustic) ao_extra = ao;
				else col = col + ao;
			}
		}
		if(live && (flags & F_PEND_ONE))
		{
			// path_tracer.cc:201-207 / :244-266: lcol = estimateOne * nlights (+ emit); path_col += lcol * thr
			const int lnum = (int)(flags >> F_LNUM_SHIFT);
			C3 lcol = neeSumT(S.lights[lnum], kb, ge, go) * (float)S.n_lights;
			if(flags & F_PEND_EMIT) lcol = lcol + rgb(pem4);
			pcol = pcol + lcol * rgb(pthr4);
		}
		flags &= ~(F_PEND_V0 | F_PEND_ONE | F_PEND_EMIT | F_AO_EMIT);

		PHASE(1);
		// ---- 2. the new hit ----
		Surf sp;
		sp.p = v3(0.f, 0.f, 0.f); sp.n = sp.ng = sp.nu = sp.nv = sp.p; sp.mat = 0; sp.flags = 0;
		sp.dcol = c3(0.f); sp.drefl = 1.f; sp.sigma = 0.f;
		float4 sa0 = make_float4(0.f, 0.f, 0.f, 0.f), sa1 = sa0;
		V3 wo = v3(0.f, 0.f, 1.f);
		bool have_hit = false;
		int hit_prim = -1;
		int add_depth_in = 0;   // additional_depth of a spawned specular node (spawnSpecular)
		if(live && st != ST_NORAY)
		{
			hit_prim = A.Q.hit_prim[i];
			if(hit_prim >= 0)
			{
				V3 ro, rd;
				float tmin_unused, tw;
				loadQRay(A.Q, i, ro, rd, tmin_unused, tw);
				if(EXT && S.cur_level > 0) add_depth_in = (int)(-tw) - 1;
				have_hit = true;
				sp = makeSurf(S, ro, rd, A.Q.hit_t[i], hit_prim);
				if(ATTR)
				{
					sa0 = A.Q.sattr[2 * (size_t)i];
					sa1 = A.Q.sattr[2 * (size_t)i + 1];
					applyAttr(sp, sa0, sa1);
				}
				wo = -rd;
			}
		}
		bool nee_v0 = false, nee_one = false, sample_next = false, end_sub = false, finalize = false, start_sub = false;
		// DEFER: this vertex's record — 1: a light estimate to pick and estimate later (dfr_a = its throughput),
		// 2: a term known now (dfr_a)
		int dfr_kind = 0;
		C3 dfr_a = c3(0.f), dfr_emit = c3(0.f);
		uint32_t dfr_n = 0, dfr_has_emit = 0;
		C3 emit_pend = c3(0.f);
		C3 pend_thr = c3(0.f);
		if(live)
		{
			if(st == ST_NORAY) end_sub = true;   // a finished subpath whose estimate just got connected
			else if(st == ST_CAMERA)
			{
				if(!have_hit)
				{
					// integrator_tiled.cc:707-720 background
					C3 bg = c3(0.f);
					float a = 1.f;
					if(S.bg_transp && (!EXT || S.cur_level == 0 || S.bg_transp_refract)) a = 0.f;
					else if(S.has_bg) bg = C3{S.bg[0], S.bg[1], S.bg[2]};
					if(EXT && S.tree)
					{
						S.node_own[sid] = f4(bg, a);
						S.node_child[sid] = make_int2(-1, -1);
					}
					else if(compact) writeSampleAt(A, sc, bg, a);
					else writeSample(A, sid, bg, a);
				}
				else
				{
					const DevMaterial &m = S.mats[sp.mat];
					if(EXT && S.tree) spawnSpecular(S, m, sp, wo, sid, make_uint2(offset, sample_idx), rng, add_depth_in);
					col = c3(0.f);
					col_ld = true;
					col_dirty = true;
					// photon_mapping.cc:868-869 adds emit(wo) unconditionally and :938-946 adds it again
					// for emitting materials; the other integrators add it once (direct_light.cc:120);
					// show_map (:876-881, 924-929): the first emit, then the nearest photon (k_gather)
					const bool show = is_photon && S.show_map;
					if(is_photon) col = col + matEmit<EXT>(m, sp, wo);
					if((sp.flags & B_EMIT) && !show) col = col + matEmit<EXT>(m, sp, wo);
					if(sp.flags & B_DIFFUSE) { nee_v0 = !show; flags |= F_V0_DIFFUSE; }
					if(show) flags |= F_SHOWMAP;
					if(S.do_ao && (sp.flags & B_DIFFUSE) && (sp.flags & B_EMIT))
					{
						emit_pend = matEmit<EXT>(m, sp, wo);   // sampleAmbientOcclusion adds sp.emit(wo) * pdf per sample
						flags |= F_AO_EMIT;
					}
					if(is_photon || (S.caus_map && (sp.flags & B_DIFFUSE)))
					{
						v0p4 = f4(sp.p, __int_as_float(hit_prim));
						v0wo4 = f4(wo, 0.f);
						if(ATTR) { v0a0 = sa0; v0a1 = sa1; }
					}
					if(is_path && (sp.flags & B_DIFFUSE))
					{
						v0p4 = f4(sp.p, __int_as_float(hit_prim));
						v0wo4 = f4(wo, 0.f);
						if(ATTR) { v0a0 = sa0; v0a1 = sa1; }
						start_sub = true;
						subpath = 0;
					}
					else end_sub = true;
				}
			}
			else if(st == ST_FIRST)
			{
				if(!have_hit) end_sub = true;     // path_tracer.cc:192 `continue`
				else
				{
					// path_tracer.cc:193-207
					if(flags & F_SAMPLED) pwo = wo;
					else wo = pwo;
					nee_one = true;
					flags = (flags & ~F_MATFLAGS) | (sp.flags & F_MATFLAGS);
					if(sp.flags & B_EMIT) { emit_pend = matEmit<EXT>(S.mats[sp.mat], sp, wo); flags |= F_PEND_EMIT; }
					pend_thr = thr;
					depth = 1;
					sample_next = true;
				}
			}
			else   // ST_BOUNCE, ray of loop iteration `depth`
			{
				if(!have_hit) end_sub = true;     // path_tracer.cc:235
				else
				{
					const uint32_t mfl = flags & F_MATFLAGS;
					pwo = wo;
					bool killed = false;
					if(depth > S.rr_min_bounces)
					{
						// path_tracer.cc:249-255 (the draw does not depend on the light estimate); the
						// specular recursion tree's nodes keep a per-node MWC stream in their full record
						float random_value;
						if(compact) random_value = rrRandom(S, sc, subpath, depth);
						else
						{
							Mwc g{rng.x, rng.y};
							random_value = (float)g.next();
							rng = make_uint2(g.x, g.c);
						}
						const float probability = maxComp(thr);
						if(probability <= 0.f || probability < random_value) killed = true;
						else thr = thr * rcpExact(probability);
					}
					if(killed) end_sub = true;
					else
					{
						if((mfl & B_EMIT) && (flags & F_CAUSTIC)) { emit_pend = matEmit<EXT>(S.mats[sp.mat], sp, wo); flags |= F_PEND_EMIT; }
						if(mfl & B_DIFFUSE) { nee_one = true; pend_thr = thr; }
						else
						{
							// lcol = 0 (+ emission): nothing to trace, connect now
							C3 lcol = c3(0.f);
							if(flags & F_PEND_EMIT) lcol = lcol + emit_pend;
							if(DEFER) { dfr_kind = 2; dfr_a = lcol * thr; }
							else pcol = pcol + lcol * thr;
							flags &= ~F_PEND_EMIT;
						}
						++depth;
						sample_next = true;
					}
				}
			}
		}
		uint32_t lnum = 0;
		if(nee_one && S.lpc_mode != 0 && compact)
		{
			// integrator_montecarlo.cc:70-78 light pick with the one-thread render's running counter:
			// the sample's calls are sequential (one entry per sample), so the counter is read and
			// advanced in place
			uint32_t *c = &S.lpc[((size_t)sc.y * (size_t)S.width + (size_t)sc.x) * (size_t)S.spp + (size_t)sc.s];
			const uint32_t n = *c;
			*c = n + 1u;
			if(S.lpc_mode == 1) nee_one = false;   // count run: the call is counted, nothing is estimated
			else if(DEFER && S.lpc_mode == 3)
			{
				// the call's ordinal in its sample; the estimate, its emission and throughput go to the record
				dfr_kind = 1;
				dfr_n = n;
				dfr_a = pend_thr;
				dfr_has_emit = (flags & F_PEND_EMIT) ? 1u : 0u;
				if(dfr_has_emit) dfr_emit = emit_pend;
				flags &= ~F_PEND_EMIT;
				nee_one = false;
			}
			else lnum = lightOfCounter(S, n);
		}
		else if(nee_one)
		{
			// integrator_montecarlo.cc:70-78 light pick (pickLight: multi-light PT is matched
			// statistically, one light exactly)
			lnum = pickLight(S, offset, sample_idx, (uint32_t)depth + subpath * (uint32_t)S.bounces, n_paths * (uint32_t)(S.bounces + 1));
		}
		if(S.lpc_mode == 1) nee_v0 = false;   // count run: no estimateAllDirectLight either
		if(DEFER && live && dfr_kind == 0)
		{
			// no addition at this vertex: the slot stays empty (its kind word)
			const uint32_t slot = A.S.dfr_seg_off[seg] + (i - a0);
			if(slot < S.dfr_cap) S.dfr_kind[slot] = 0u;
		}
		if(DEFER && dfr_kind != 0)
		{
			// the record at this entry's slot of the iteration, chained to the sample's previous one (whose
			// index + 1 rides in the path colour's red bits: the colour itself is only summed at the end)
			const uint32_t slot = A.S.dfr_seg_off[seg] + (i - a0);
			if(slot < S.dfr_cap)
			{
				const uint32_t q = (uint32_t)(((size_t)sc.y * (size_t)S.width + (size_t)sc.x) * (size_t)S.spp + (size_t)sc.s);
				S.dfr_kind[slot] = (uint32_t)dfr_kind | (dfr_has_emit << 2) | (dfr_n << 3);
				S.dfr_a[slot] = f4(dfr_a, __uint_as_float(q));
				if(dfr_kind == 1)
				{
					S.dfr_pp[slot] = f4(sp.p, __int_as_float(hit_prim));
					S.dfr_wo[slot] = f4(wo, 0.f);
					S.dfr_pix[slot] = make_uint2(offset, sample_idx);
					if(dfr_has_emit) S.dfr_emit[slot] = f4(dfr_emit, 0.f);
				}
			}
		}
		if(nee_one) flags = (flags & ((1u << F_LNUM_SHIFT) - 1u)) | (lnum << F_LNUM_SHIFT) | F_PEND_ONE;
		if(nee_v0) flags |= F_PEND_V0;
		const bool pending = (flags & (F_PEND_V0 | F_PEND_ONE)) != 0;

		PHASE(2);
		// ---- 3. next segment ----
		V3 ray_o = v3(0.f, 0.f, 0.f), ray_d = v3(0.f, 0.f, 1.f);
		bool want_ray = false;
		if(live && sample_next)
		{
			if(depth < S.bounces)
			{
				// path_tracer.cc:211-234, loop iteration `depth`
				const uint32_t offs = n_paths * sample_idx + offset + subpath;
				const int d_4 = 4 * depth;
				BsdfSample s;
				s.s_1 = ldsDim(S, d_4 + 3, offs);
				s.s_2 = ldsDim(S, d_4 + 4, offs);
				s.flags = B_ALL;
				s.pdf = 0.f;
				s.sampled = B_NONE;
				V3 dir = v3(0.f, 0.f, 0.f);
				C3 scol = matSample<EXT>(S.mats[sp.mat], sp, wo, dir, s, w);
				scol = scol * w;
				if(isBlack(scol)) end_sub = true;
				else
				{
					thr = thr * scol;
					if(S.caustic_path && (s.sampled & (B_SPECULAR | B_GLOSSY | B_FILTER))) flags |= F_CAUSTIC;
					else flags &= ~F_CAUSTIC;
					ray_o = sp.p;
					ray_d = dir;
					want_ray = true;
					stage = ST_BOUNCE | (subpath << 8) | ((uint32_t)depth << 20);
				}
			}
			else end_sub = true;
		}
		if(live && end_sub && !pending)
		{
			// end of the subpath: next subpath (path_tracer.cc:166) or the end of integrate()
			if(is_path && (flags & F_V0_DIFFUSE) && subpath + 1 < n_paths) { start_sub = true; ++subpath; }
			else finalize = true;
		}
		if(live && start_sub)
		{
			// path_tracer.cc:168-191: first segment of subpath `subpath` from v0
			Surf s0 = (st == ST_CAMERA) ? sp : surfFromPrim(S, xyz(v0p4), __float_as_int(v0p4.w));
			if(ATTR && st != ST_CAMERA) applyAttr(s0, v0a0, v0a1);
			const V3 wo0 = (st == ST_CAMERA) ? wo : xyz(v0wo4);
			const uint32_t offs = n_paths * sample_idx + offset + subpath;
			BsdfSample s;
			s.s_1 = riVdC(offs);
			s.s_2 = ldsDim(S, 2, offs);
			s.flags = B_DIFFUSE | B_REFLECT | B_TRANSMIT;
			s.pdf = 0.f;
			s.sampled = B_NONE;
			V3 dir = v3(0.f, 0.f, 0.f);
			C3 scol = matSample<EXT>(S.mats[s0.mat], s0, wo0, dir, s, w);
			thr = scol * w;
			pwo = wo0;
			if(s.sampled != B_NONE) flags |= F_SAMPLED;
			else flags &= ~F_SAMPLED;
			flags &= ~F_CAUSTIC;
			ray_o = s0.p;
			ray_d = dir;
			want_ray = true;
			stage = ST_FIRST | (subpath << 8);
		}
		// a diffuse first hit still owes its photon-map estimates (k_gather): the diffuse map's
		// density estimate (photon mapping) and / or causticPhotons(); whatever the integrator adds
		// after them rides along as `extra` (DirectLight: the AO sum; path tracing: the paths)
		// show_map: every camera hit asks for its nearest photon (and the caustics at diffuse hits)
		const bool want_show = live && finalize && is_photon && (flags & F_SHOWMAP);
		const bool want_gather = want_show || (live && finalize && (flags & F_V0_DIFFUSE) && ((is_photon && S.n_photons > 0) || S.caus_map));
		C3 g_extra = c3(0.f);
		uint32_t g_mode = 0;
		if(want_gather)
		{
			loadCol();
			g_mode = ((is_photon && S.n_photons > 0) ? (S.fg_on ? G_FG : G_DIFFUSE) : 0u) | (S.caus_map ? G_CAUSTIC : 0u);
			if(want_show) g_mode = G_SHOWMAP | ((S.caus_map && (flags & F_V0_DIFFUSE)) ? G_CAUSTIC : 0u);
			// final gathering (k_fg) needs the PixelSamplingData of the sample
			if(g_mode & G_FG) g_extra = C3{__uint_as_float(offset), __uint_as_float(sample_idx), 0.f};
			if(ao_after_caustic && S.do_ao) { g_extra = ao_extra; g_mode |= G_EXTRA; }
			if(is_path) { g_extra = pcol / (float)n_paths; g_mode |= G_EXTRA; }   // path_tracer.cc:274-278
		}
		if(DEFER && live && finalize && !want_gather)
		{
			// the first-vertex estimate alone; k_dfr_fold adds the paths' colour (col + pcol / n, + 0)
			loadCol();
			writeSampleAt(A, sc, col, alpha);
			S.dfr_last[((size_t)sc.y * (size_t)S.width + (size_t)sc.x) * (size_t)S.spp + (size_t)sc.s] = (is_path && (flags & F_V0_DIFFUSE)) ? 1u : 0u;
		}
		else if(live && finalize && !want_gather)
		{
			loadCol();
			// path_tracer.cc:274-278 / direct_light.cc:129-131
			if(is_path && (flags & F_V0_DIFFUSE)) col = col + pcol / (float)n_paths;
			col = col + c3(0.f);   // recursiveRaytrace: no specular/glossy component
			if(EXT && S.tree) S.node_own[sid] = f4(col, alpha);   // recursiveRaytrace's part: k_combine
			else if(compact) writeSampleAt(A, sc, col, alpha);
			else writeSample(A, sid, col, alpha);
		}

		PHASE(3);
		// ---- 4. compaction: the entry moves to position k of the next queue ----
		const bool keep = live && (want_ray || pending);   // pending => never finalized this iteration
		const bool want_nee = live && (nee_v0 || nee_one);
		// the entry stays in its shard: at most one next entry per entry, so the shard never overflows
		const uint32_t k = a0 + waveAppend(keep, &s_count[0]);
		if(keep && compact && col_dirty)
		{
			// the first-vertex estimate changed: store it by sample id (zero is implied by a clear F_COLS)
			if((__float_as_uint(col.r) | __float_as_uint(col.g) | __float_as_uint(col.b)) != 0u)
			{
				Pc.csmp[sid] = f4(col, 0.f);
				flags |= F_COLS;
			}
			else flags &= ~F_COLS;
		}
		if(keep)
		{
			if(!compact) stStore2(&A.Qn.slot[k], (int)sid);
			if(want_ray) storeQRay(A.Qn, k, ray_o, ray_d);   // (tmin = ray_min_dist, tmax infinite: loadQRay)
			else
			{
				storeQNoRay(A.Qn, k);
				// a pending-only entry keeps its hit point here for its NEE request (k_nee reads the
				// vertex from the ray origin; a continuing entry's ray starts at the vertex)
				if(!FUSED && want_nee) reinterpret_cast<F3 *>(A.Qn.ray_o)[k] = F3{sp.p.x, sp.p.y, sp.p.z};
				stage = ST_NORAY | (subpath << 8) | ((uint32_t)depth << 20);
			}
			if(compact) stStoreU2(reinterpret_cast<uint2 *>(Pn.pr) + k, make_uint2(sid, stage));
			else
			{
				stStore(&Pn.pr[k], make_uint4(pix.x, pix.y, rng.x, rng.y));
				stStore(&Pn.col[k], f4(col, __uint_as_float(stage)));
			}
			if(S.w_live) stStore(&Pn.thr[k], f4(thr, w));
			else stStoreF3(Pn.thr, k, thr);
			stStore(&Pn.pcol[k], f4(pcol, __uint_as_float(flags)));
			if((stage & 0xffu) == ST_FIRST) Pn.pwo[k] = f4(pwo, 0.f);
			if(nee_one) reinterpret_cast<F3 *>(Pn.pend_thr)[k] = F3{pend_thr.r, pend_thr.g, pend_thr.b};
			if(flags & (F_PEND_EMIT | F_AO_EMIT)) Pn.pend_emit[k] = f4(emit_pend, 0.f);
			if(keep_v0) { Pn.v0p[k] = v0p4; Pn.v0wo[k] = v0wo4; }
			if(ATTR && keep_v0) { Pn.v0attr[2 * (size_t)k] = v0a0; Pn.v0attr[2 * (size_t)k + 1] = v0a1; }
		}

		PHASE(4);
		// ---- 5. next-event estimation request (served by k_nee; wants -> keep, so k is valid) ----
		// (photon mapping: the gather requests of the last iteration use the same queue — a path
		// never asks for NEE and a gather in the same iteration, and the DL-style pipeline of the
		// photon integrator serves NEE in iteration 0 and gathers in iteration 1)
		if(FUSED)
		{
			// k_nee's work in place (integrator_montecarlo.cc:54-408): contributions into the next
			// state at k * nee_k, shadow rays appended to segment `seg` of the next queue
			const int e0 = (int)k * K;
			const bool all = live && nee_v0, one = live && nee_one;
			const DevMaterial &m = S.mats[sp.mat];
			float4 *ts = S.tr_shad ? Pn.ts : nullptr;
			if(__any(all))
			{
				for(int l = 0; l < S.n_lights; ++l)
					neeLight<EXT, ShadeOut, NeeHbm, LEAN>(S, S.lights[l], m, sp, wo, (uint32_t)l, sample_idx, offset, all, e0 + (int)S.lights[l].nee_base,
					                                    neeHbm(Pn), Pn.occ, out, ts);
				if(S.do_ao) aoSamples<EXT>(S, m, sp, wo, sample_idx, offset, all, e0 + S.nee_all_count, neeHbm(Pn), Pn.occ, out, ts);
			}
			if(__any(one))
			{
				for(int l = 0; l < S.n_lights; ++l)
				{
					const bool mine = one && lnum == (uint32_t)l;
					if(!__any(mine)) continue;
					neeLight<EXT, ShadeOut, NeeHbm, LEAN>(S, S.lights[l], m, sp, wo, (uint32_t)l, sample_idx, offset, mine, e0, neeHbm(Pn), Pn.occ, out, ts);
				}
			}
		}
		// NEE requests sit at the entry's own next-queue position k (DevNeeQueue): no index and no hit
		// point travel with them (k_nee reads the vertex from the next queue's ray origin at k); the
		// append only counts them (statistics)
		(void)waveAppend(!FUSED && want_nee, &s_count[1]);
		const uint32_t jg = waveAppend(want_gather, &s_count[3]);
		if(!FUSED && keep)
		{
			if(want_nee)
			{
				stStore2(&A.N.wo_k[k], f4(wo, __int_as_float(hit_prim)));
				neePmStore(S, A.N.pix_mode, k, offset, sample_idx, (nee_v0 ? 1u : 0u) | (lnum << 8));
				if(ATTR)
				{
					A.N.attr[2 * (size_t)k] = f4(sp.n, sp.drefl);
					A.N.attr[2 * (size_t)k + 1] = f4(sp.dcol, sp.sigma);
				}
			}
			else reinterpret_cast<float *>(A.N.wo_k)[4 * (size_t)k] = __builtin_nanf("");   // no request
		}
		if(want_gather)
		{
			const uint32_t j = a0 + jg;
			A.G.p_prim[j] = v0p4;
			A.G.wo_k[j] = f4(xyz(v0wo4), __uint_as_float(sid));
			A.G.pix_mode[j] = make_uint4(__float_as_uint(col.r), __float_as_uint(col.g), __float_as_uint(col.b), __float_as_uint(alpha));
			A.G.extra[j] = f4(g_extra, __uint_as_float(g_mode));
			if(ATTR)
			{
				A.G.attr[2 * (size_t)j] = v0a0;
				A.G.attr[2 * (size_t)j + 1] = v0a1;
			}
		}
		PHASE(5);
	}
	PHASE_FLUSH;
	__syncthreads();
	if(threadIdx.x == 0)
	{
		A.cnt_next.n_active[seg] = s_count[0];
		A.cnt_next.n_nee[seg] = s_count[1];
		if(FUSED) A.cnt_next.n_shadow[seg] = s_count[2];
		if(S.gather_on) A.cnt_next.n_gather[seg] = s_count[3];
		if(S.stats) S.stats[seg].shade_entries += n_a;
	}
}

// ---------------------------------------------------------------------------------------------
// k_nee: next-event estimation for the vertices k_shade queued (integrator_montecarlo.cc:54-408).
// Dense (every lane has a request), so the light-sampling arithmetic runs at full SIMD width and
// k_shade keeps fewer registers live.  Contributions go to the next state set at k * nee_k,
// shadow rays to the next queue (workgroup-level appends).
// ---------------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------------
// specular recursion tree: k_spawn starts the traced nodes of one ray level (the camera's role for
// them), k_combine folds totals bottom-up (integrator_montecarlo.cc:866-968):
//   total(node) = own + ((0 + total(reflect) * reflect colour) + total(refract) * refract colour)
//   alpha(node) = children ? (sum of their alphas) / count : own alpha
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_spawn(DevScene S, DevPaths P, DevQueues Q, DevCounters cnt, uint32_t s0, int n)
{
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if((uint32_t)i < S.n_seg)
	{
		const uint32_t groups = (uint32_t)n / 256u, rem = (uint32_t)n % 256u, sg = (uint32_t)i, R = S.n_seg;
		cnt.n_active[sg] = (groups / R) * 256u + (sg < groups % R ? 256u : 0u) + (sg == groups % R ? rem : 0u);
		cnt.n_shadow[sg] = 0;
	}
	if(i >= n) return;
	const uint32_t g = (uint32_t)i / 256u;
	const uint32_t a = (g % S.n_seg) * S.cap_a + (g / S.n_seg) * 256u + (uint32_t)i % 256u;
	const uint32_t idx = s0 + (uint32_t)i;
	Q.slot[a] = (int)(S.node_base + idx);
	const float4 so = S.spawn_o[idx], sd = S.spawn_d[idx];
	storeQRay(Q, a, xyz(so), xyz(sd));
	Q.ray_tt[a] = make_float2(so.w, sd.w);
	P.thr[a] = make_float4(0.f, 0.f, 0.f, 0.f);
	P.col[a] = make_float4(0.f, 0.f, 0.f, __uint_as_float(ST_CAMERA));
	P.pcol[a] = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
	P.pr[a] = S.spawn_pr[idx];
}

// nodes [lo, hi) of one level; final: level 0, write the camera samples (integrator_tiled.cc:399)
__global__ void __launch_bounds__(256) k_combine(DevScene S, uint32_t lo, uint32_t hi, int final_level, float4 *samples,
                                                 const DevJob *jobs, int n_jobs, uint64_t chunk_base)
{
	const uint32_t n = lo + blockIdx.x * blockDim.x + threadIdx.x;
	if(n >= hi) return;
	const float4 own = S.node_own[n];
	const int2 ch = S.node_child[n];
	C3 rt = c3(0.f);
	float asum = 0.f;
	int count = 0;
	if(ch.x >= 0)
	{
		const float4 t = S.node_own[ch.x], w = S.node_w[ch.x];
		rt = rt + C3{t.x, t.y, t.z} * C3{w.x, w.y, w.z};
		asum += t.w;
		++count;
	}
	if(ch.y >= 0)
	{
		const float4 t = S.node_own[ch.y], w = S.node_w[ch.y];
		rt = rt + C3{t.x, t.y, t.z} * C3{w.x, w.y, w.z};
		asum += t.w;
		++count;
	}
	const C3 col = C3{own.x, own.y, own.z} + rt;
	float alpha = count > 0 ? asum / (float)count : own.w;
	if(final_level)
	{
		const SampleCoord sc = sampleAt(S, jobs, n_jobs, chunk_base + (uint64_t)n);
		if(alpha > 1.f) alpha = 1.f;
		samples[((size_t)sc.y * S.width + sc.x) * S.spp + sc.s] = f4(col, alpha);
	}
	else S.node_own[n] = f4(col, alpha);
}

// ---------------------------------------------------------------------------------------------
// k_surface: material-shade dispatch for scenes with textures / shader nodes / smooth normals.
// For every hit of the active queue: barycentrics -> shading normal, orco, uv
// (TrianglePrimitive::getSurface, primitive_triangle.cc:97-176), then the material's shader-node
// program (Material::initBsdf, material_shiny_diffuse.cc:133-141) -> diffuse colour + diffuse_refl.
// Written per queue entry for k_shade (and from there into the NEE requests for k_nee).  Kept out
// of k_shade so the untextured hot path carries none of its registers.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kShadeBlock) k_surface(DevScene S, DevQueues Q, DevCounters cnt)
{
	const uint32_t seg = blockIdx.x;
	const uint32_t n_a = cnt.n_active[seg];
	const uint32_t a0 = seg * S.cap_a;
	for(uint32_t j = threadIdx.x; j < n_a; j += blockDim.x)
	{
		const uint32_t i = a0 + j;
		V3 o, d;
		float tmin_unused, tw_unused;
		if(!loadQRay(Q, i, o, d, tmin_unused, tw_unused)) continue;   // no ray this iteration (NaN marker)
		const int prim = Q.hit_prim[i];
		if(prim < 0) continue;
		const V3 p = o + Q.hit_t[i] * d;   // accelerator.cc:61
		const SurfAttr sa = surfAttr(S.prim_attr, S.prim_ng, prim, o, d, p);
		const DevMaterial &m = S.mats[__float_as_int(S.prim_ng[prim].w)];
		C3 dcol = C3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
		float drefl = 1.f, sigma = 0.f;
		if(m.n_nodes > 0) evalNodes(m, S.shader_nodes, S.textures, S.texels, sa, dcol, drefl, sigma);
		Q.sattr[2 * (size_t)i] = f4(sa.n, drefl);
		Q.sattr[2 * (size_t)i + 1] = f4(dcol, sigma);
	}
}

// Transparent shadows, second half (accelerator_kdtree.cc:1011-1018 + accelerator.cc:80-93): for
// every shadow ray k_trace<TS> left unoccluded with transparent surfaces on it, the filter colour
// is the product of their ShinyDiffuseMaterial::getTransparency (material_shiny_diffuse.cc:441-465,
// wo = the ray direction) at the surface point getSurface builds from the moved ray; then the NEE
// contribution is rebuilt with `lcol *= scol` where the reference applies it.  Factors multiply in
// ascending (t, primitive) order (the kd-tree's cell order: the same value for up to two surfaces).
// tsFilterColor: that product for one ray (h: its n (t, prim) pairs; o, d: the moved shadow ray).
__device__ C3 tsFilterColor(const DevScene &S, float2 *h, int n, V3 o, V3 d)
{
	// insertion sort by (t, prim)
	for(int a = 1; a < n; ++a)
	{
		const float2 x = h[a];
		int b = a - 1;
		while(b >= 0 && (h[b].x > x.x || (h[b].x == x.x && __float_as_int(h[b].y) > __float_as_int(x.y))))
		{
			h[b + 1] = h[b];
			--b;
		}
		h[b + 1] = x;
	}
	C3 scol = c3(1.f);
	for(int a = 0; a < n; ++a)
	{
		const float t = h[a].x;
		const int prim = __float_as_int(h[a].y);
		const V3 p = o + t * d;
		const float4 g = S.prim_ng[prim];
		const V3 ng = xyz(g);
		const DevMaterial &m = S.mats[__float_as_int(g.w)];
		V3 nrm = ng;
		C3 dcol = C3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
		if(S.has_attr)
		{
			const SurfAttr sa = surfAttr(S.prim_attr, S.prim_ng, prim, o, d, p);
			nrm = sa.n;
			float drefl = 1.f, sigma = 0.f;
			if(m.n_nodes > 0) evalNodes(m, S.shader_nodes, S.textures, S.texels, sa, dcol, drefl, sigma);
		}
		const V3 nf = faceForward(ng, nrm, d);
		const float kr = fresnelKr(m, d, nf);
		float accum = 1.f;
		if(m.sd_flags & SD_MIRROR) accum = 1.f - kr * m.comp[0];
		accum *= m.comp[1] * accum;
		const C3 tcol = m.tfilter * dcol + c3(1.f - m.tfilter);
		scol = scol * (accum * tcol);
	}
	return scol;
}

// k_tshadow: the filter colour of each such ray times the NEE factors tsFactors stored
__global__ void __launch_bounds__(kShadeBlock) k_tshadow(DevScene S, DevQueues Q, DevCounters cnt, DevPaths P)
{
	const uint32_t seg = blockIdx.x;
	const uint32_t n_s = cnt.n_shadow[seg];
	const uint32_t s0 = seg * S.cap_s;
	const uint32_t cap = (uint32_t)S.s_depth;
	for(uint32_t j = threadIdx.x; j < n_s; j += blockDim.x)
	{
		const uint32_t k = s0 + j;
		const int n = Q.ts_n[k];
		if(n <= 0) continue;
		const C3 scol = tsFilterColor(S, Q.ts_hit + (size_t)k * cap, n, xyz(Q.sh_o[k]), xyz(Q.sh_d[k]));
		const uint32_t e = (uint32_t)Q.sh_idx[k];
		const float4 f0 = P.ts[3 * (size_t)e], f1 = P.ts[3 * (size_t)e + 1], f2 = P.ts[3 * (size_t)e + 2];
		C3 x = rgb(f0) * (rgb(f1) * scol);
		x = x * f0.w;
		x = x * f1.w;
		x = (f2.y != 0.f) ? x / f2.x : x * f2.x;
		reinterpret_cast<F3 *>(P.nee)[e] = F3{x.r, x.g, x.b};
	}
}

// Shadow-ray emitter of k_path and of k_nee's in-place variant: neeLight's rays are recorded per lane
// (origin + t_max, direction + want; entry idx - base) and traced after the light sampling; lanes
// that emit nothing leave their cleared records
struct PathShadows
{
	float4 *rec;
	int base;
	__device__ __forceinline__ void emit(bool want, V3 o, V3 d, float t_max, float tmin, int idx) const
	{
		(void)tmin;   // the origin is already moved (shadowRayOf); the any-hit test starts at 0
		if(want)
		{
			rec[2 * (idx - base)] = f4(o, t_max);
			rec[2 * (idx - base) + 1] = f4(d, 1.f);
		}
	}
};

// The rays one k_path lane owes before its next vertex: the shadow rays its last NEE recorded
// (rec entries with `want`, when `shadows`) and its closest ray (when `closest`).  traceRefill4's
// scheme: one BVH4 visit per loop trip and a lane starts its next ray as soon as one ends, so the
// wave runs for its busiest lane's sum of traversals (not one full traversal per ray slot, most of
// whose lanes would idle: the MIS material-sample shadow ray exists for a few lanes only).  Every ray
// runs traverse4's exact sequence of visits, culling, leaf order and exits: hits are identical.
template<bool STATS, int STRIDE = kTraceBlock>
__device__ __forceinline__ void traceLaneRays(const TraceCtx &C, const float4 *rec, uint8_t *occ, int K, bool shadows, bool closest, V3 co,
                                              V3 cd, float ctmin, float ctmax, float &hit_t, int &hit_prim, uint32_t &visits,
                                              uint32_t &tests, uint32_t &n_closest, uint32_t &n_shadow)
{
	const int lane = threadIdx.x;
	const float inf = __builtin_huge_valf();
	V3 o = v3(0.f, 0.f, 0.f), d = o, id = o, oid = o;
	SlabSel sel{0, 2, 4};
	float tmax = 0.f, tmin = 0.f, box_t0 = 0.f, t_best = 0.f;
	int prim_best = -1, sp = 0, node = -1, cur = 0;
	int e = shadows ? 0 : K;
	bool any = false, cl = closest;
	for(;;)
	{
		if(node < 0)
		{
			// this lane's next ray: the recorded shadow rays in entry order, then the closest ray
			bool got = false;
			while(e < K)
			{
				const int ee = e++;
				const float4 dd = rec[2 * ee + 1];
				if(dd.w == 0.f) continue;
				const float4 od = rec[2 * ee];
				o = xyz(od);
				d = xyz(dd);
				tmin = 0.f;
				tmax = od.w;
				any = true;
				cur = ee;
				++n_shadow;
				got = true;
				break;
			}
			if(!got && cl)
			{
				cl = false;
				o = co;
				d = cd;
				tmin = ctmin;
				tmax = ctmax;
				any = false;
				++n_closest;
				got = true;
			}
			if(!got) break;
			V3 dq = d;
			if(fabsf(dq.x) < 1e-20f) dq.x = copysignf(1e-20f, dq.x);
			if(fabsf(dq.y) < 1e-20f) dq.y = copysignf(1e-20f, dq.y);
			if(fabsf(dq.z) < 1e-20f) dq.z = copysignf(1e-20f, dq.z);
			id = v3(rcpExact(dq.x), rcpExact(dq.y), rcpExact(dq.z));
			oid = v3(o.x * id.x, o.y * id.y, o.z * id.z);
			sel = slabSel(id);
			box_t0 = any ? -1e-3f : (tmin - 1e-3f * (1.f + fabsf(tmin)));
			t_best = tmax;
			prim_best = -1;
			sp = 0;
			node = 0;
		}
		if(STATS) TRACE_STAT(++visits);
		const float4 *np = C.nodes + 8 * node;
		const float4 nx = np[sel.nx], fx = np[sel.nx ^ 1], ny = np[sel.ny], fy = np[sel.ny ^ 1], nz = np[sel.nz], fz = np[sel.nz ^ 1], cf = np[6], kf = np[7];
		const float slack_t = (t_best < 3.0e38f) ? t_best * 1.0000005f + 1e-6f : 3.4e38f;
		float key[4];
		int child[4], e4[4], s4[4];
		int acc = 0;
#pragma unroll
		for(int k = 0; k < 4; ++k)
		{
			const float lo = fmaxf(fmaxf(__builtin_fmaf(lane4(nx, k), id.x, -oid.x), __builtin_fmaf(lane4(ny, k), id.y, -oid.y)),
			                       fmaxf(__builtin_fmaf(lane4(nz, k), id.z, -oid.z), box_t0));
			const float hi = fminf(fminf(__builtin_fmaf(lane4(fx, k), id.x, -oid.x), __builtin_fmaf(lane4(fy, k), id.y, -oid.y)),
			                       fminf(__builtin_fmaf(lane4(fz, k), id.z, -oid.z), slack_t));
			const uint32_t h = lo <= hi ? 1u : 0u;
			child[k] = __float_as_int(lane4(cf, k));
			const int count = __float_as_int(lane4(kf, k));
			const uint32_t inner = child[k] >= 0 ? 1u : 0u;
			key[k] = (h & inner) ? lo : inf;
			s4[k] = ~child[k] - acc;
			acc += (h & (inner ^ 1u)) ? count : 0;
			e4[k] = acc;
		}
		bool done = false;
		for(int i = 0; i < e4[3]; ++i)
		{
			const int q = i + (i < e4[0] ? s4[0] : i < e4[1] ? s4[1] : i < e4[2] ? s4[2] : s4[3]);
			if(STATS) TRACE_STAT(++tests);
			const float4 *tp = C.tris + 3 * q;
			const float4 ta = tp[0], tb = tp[1], tc = tp[2];
			const float t = triTest(ta, tb, tc, o, d, t_best);
			if(t == -1.f) continue;
			const int prim = __float_as_int(tb.w);
			if(any)
			{
				if(t < tmax && t >= 0.f) { t_best = t; prim_best = prim; done = true; break; }
			}
			else if(t >= tmin && (t < t_best || (t == t_best && prim_best >= 0 && prim < prim_best)))
			{
				t_best = t;
				prim_best = prim;
			}
		}
		if(!done)
		{
			cswap(key[0], child[0], key[1], child[1]);
			cswap(key[2], child[2], key[3], child[3]);
			cswap(key[0], child[0], key[2], child[2]);
			cswap(key[1], child[1], key[3], child[3]);
			cswap(key[1], child[1], key[2], child[2]);
			if(key[3] < inf) { C.stack[sp * STRIDE + lane] = child[3]; ++sp; }
			if(key[2] < inf) { C.stack[sp * STRIDE + lane] = child[2]; ++sp; }
			if(key[1] < inf) { C.stack[sp * STRIDE + lane] = child[1]; ++sp; }
			int next = key[0] < inf ? child[0] : -1;
			if(next < 0 && sp > 0)
			{
				--sp;
				next = C.stack[sp * STRIDE + lane];
			}
			node = next;
			done = next < 0;
		}
		if(done)
		{
			if(any) occ[cur] = prim_best >= 0 ? 1 : 0;
			else
			{
				hit_t = t_best;
				hit_prim = prim_best;
			}
			node = -1;
		}
	}
}

struct NeeArgs
{
	DevScene S;
	DevNeeQueue N;
	DevPaths Pn;
	DevQueues Qn;
	DevCounters cnt_next;
	int stack_depth;     // TR: traversal stack levels (all in LDS)
};

// k_nee<.., TR = true> (LDS-resident BVH4 scenes without transparent shadows): the shadow rays are
// traced by the lane that sampled them, right after the light sampling (traceLaneRays over the
// scene staged in LDS), and the occlusion bytes written in place — the shadow rays never go through
// HBM (36 B written by k_nee and read back by k_trace per ray) and k_trace traces closest rays only.
__host__ __device__ inline size_t neeTraceLdsBytes(const DevScene &S, int stack_depth)
{
	return shadeLdsBytes(S, true) + (size_t)(S.node_f4 * S.n_nodes + 3 * S.n_tris) * 16 + (size_t)stack_depth * kShadeBlock * 4 +
	       (size_t)kShadeBlock * S.nee_k * 32;
}

#ifndef YAF_NEE_MIN_WAVES
#define YAF_NEE_MIN_WAVES 4
#endif
#ifndef YAF_NEE_LEAN_WAVES
#define YAF_NEE_LEAN_WAVES 4
#endif
#ifndef YAF_NEE_PREFETCH
#define YAF_NEE_PREFETCH 0
#endif
// LEAN: no ambient occlusion, transparent shadows or meshlights (launch_nee picks it), so their code and
// registers drop out
template<bool SMALL, bool EXT, bool TR = false, bool TSTATS = false, bool LEAN = false>
__global__ void __launch_bounds__(kShadeBlock, EXT ? 1 : (LEAN ? YAF_NEE_LEAN_WAVES : YAF_NEE_MIN_WAVES)) k_nee(NeeArgs A)
{
	extern __shared__ uint4 shade_smem[];
	DevScene S_ = stageTables<SMALL>(A.S, shade_smem);
	if constexpr(LEAN)
	{
		S_.do_ao = 0;
		S_.tr_shad = 0;
		S_.has_attr = 0;
	}
	const DevScene S = S_;
	const bool ATTR = EXT && S.has_attr != 0;
	TraceCtx C;
	C.wave_base = waveBase();
	float4 *rec = nullptr;
	if(TR)
	{
		float4 *lds_nodes = reinterpret_cast<float4 *>(shade_smem) + shadeLdsBytes(S, SMALL) / 16;
		float4 *lds_tris = lds_nodes + S.node_f4 * S.n_nodes;
		int *stack = reinterpret_cast<int *>(lds_tris + 3 * S.n_tris);
		rec = reinterpret_cast<float4 *>(stack + A.stack_depth * kShadeBlock) + 2 * threadIdx.x * S.nee_k;
		for(int k = threadIdx.x; k < S.node_f4 * S.n_nodes; k += blockDim.x) lds_nodes[k] = A.S.nodes[k];
		for(int k = threadIdx.x; k < 3 * S.n_tris; k += blockDim.x) lds_tris[k] = A.S.tris[k];
		__syncthreads();
		C.nodes = lds_nodes;
		C.tris = lds_tris;
		C.stack = stack;
		C.lds_depth = A.stack_depth;
		C.spill = nullptr;
		C.spill_stride = 0;
	}
	uint32_t n_shadow = 0, n_dummy = 0, visits = 0, tests = 0;
	// workgroup b serves the NEE requests of segment b, shadow rays go to segment b
	const uint32_t seg = blockIdx.x;
	__shared__ uint32_t s_count;
	if(threadIdx.x == 0) s_count = 0;
	__syncthreads();
	ShadeOut out;
	out.sh_count = &s_count;
	out.sh_base = seg * S.cap_s;
	out.Qn = A.Qn;
	out.idx_in_o = !S.tr_shad;
	// one request slot per entry of the next active list (k_shade writes entry k's request at k; a
	// NaN direction marks an entry without one)
	const uint32_t n_req = A.cnt_next.n_nee[seg];
	const uint32_t n_slots = A.cnt_next.n_active[seg];
	const uint32_t a0 = seg * S.cap_a;
	const int K = S.nee_k;
	const uint32_t stride = blockDim.x;
#if YAF_NEE_PREFETCH
	// the next iteration's request is loaded while this one is computed (software pipelining: k_nee
	// waits on these loads, SQ_WAIT_ANY 0.52 at VALU issue 0.19)
	float4 wk_n = make_float4(0.f, 0.f, 0.f, 0.f);
	F3 o_n{0.f, 0.f, 0.f};
	uint4 pm_n = make_uint4(0u, 0u, 0u, 0u);
	if(threadIdx.x < n_slots)
	{
		wk_n = A.N.wo_k[a0 + threadIdx.x];
		o_n = reinterpret_cast<const F3 *>(A.Qn.ray_o)[a0 + threadIdx.x];
		pm_n = neePmLoad(S, A.N.pix_mode, a0 + threadIdx.x);
	}
#endif
	for(uint32_t base_j = 0; base_j < n_slots; base_j += stride)
	{
		const uint32_t j = a0 + base_j + threadIdx.x;
		float4 wk = make_float4(0.f, 0.f, 0.f, 0.f);
		V3 p = v3(0.f, 0.f, 0.f);
		uint4 pm = make_uint4(0u, 0u, 0u, 0u);
		bool live = base_j + threadIdx.x < n_slots;
#if YAF_NEE_PREFETCH
		if(live)
		{
			wk = wk_n;
			p = v3(o_n.x, o_n.y, o_n.z);
			pm = pm_n;
			live = !(wk.x != wk.x);
		}
		if(base_j + stride + threadIdx.x < n_slots)
		{
			wk_n = A.N.wo_k[j + stride];
			o_n = reinterpret_cast<const F3 *>(A.Qn.ray_o)[j + stride];
			pm_n = neePmLoad(S, A.N.pix_mode, j + stride);
		}
#else
		if(live)
		{
			// every load issued before the request test (one memory round trip)
			wk = A.N.wo_k[j];
			const F3 o = reinterpret_cast<const F3 *>(A.Qn.ray_o)[j];
			p = v3(o.x, o.y, o.z);
			pm = neePmLoad(S, A.N.pix_mode, j);
			live = !(wk.x != wk.x);
		}
#endif
		Surf sp;
		sp.p = v3(0.f, 0.f, 0.f); sp.n = sp.ng = sp.nu = sp.nv = sp.p; sp.mat = 0; sp.flags = 0;
		sp.dcol = c3(0.f); sp.drefl = 1.f; sp.sigma = 0.f;
		if(live) sp = surfFromPrim(S, p, __float_as_int(wk.w));
		if(ATTR && live) applyAttr(sp, A.N.attr[2 * (size_t)j], A.N.attr[2 * (size_t)j + 1]);
		const V3 wo = xyz(wk);
		const int e0 = (int)j * K;
		const bool all = live && (pm.z & 1u);
		const bool one = live && !(pm.z & 1u);
		const uint32_t lnum = pm.z >> 8;
		if constexpr(TR)
		{
			// the same light sampling with the shadow rays recorded in LDS, then traced by this lane
			// (estimateAllDirectLight at every light's nee_base, estimateOneDirectLight at 0)
			if(live)
				for(int e = 0; e < K; ++e) rec[2 * e + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
			const PathShadows rs{rec, e0};
			for(int l = 0; l < S.n_lights; ++l)
			{
				const bool mine = all || (one && lnum == (uint32_t)l);
				if(!__any(mine)) continue;
				neeLight<EXT>(S, S.lights[l], S.mats[sp.mat], sp, wo, (uint32_t)l, pm.y, pm.x, mine, e0 + (all ? (int)S.lights[l].nee_base : 0),
				              neeHbm(A.Pn), A.Pn.occ, rs);
			}
			float t_dummy;
			int p_dummy;
			if(__any(live))
				traceLaneRays<TSTATS, kShadeBlock>(C, rec, A.Pn.occ + e0, K, live, false, v3(0.f, 0.f, 0.f), v3(0.f, 0.f, 1.f), 0.f, 0.f, t_dummy,
				                                  p_dummy, visits, tests, n_dummy, n_shadow);
			continue;
		}
		if(__any(all))
		{
			// estimateAllDirectLight (montecarlo.cc:54-68)
			for(int l = 0; l < S.n_lights; ++l)
				neeLight<EXT, ShadeOut, NeeHbm, LEAN>(S, S.lights[l], S.mats[sp.mat], sp, wo, (uint32_t)l, pm.y, pm.x, all,
				         e0 + (int)S.lights[l].nee_base, neeHbm(A.Pn), A.Pn.occ, out, S.tr_shad ? A.Pn.ts : nullptr);
			if(S.do_ao)
				aoSamples<EXT>(S, S.mats[sp.mat], sp, wo, pm.y, pm.x, all, e0 + S.nee_all_count, neeHbm(A.Pn), A.Pn.occ, out,
				               S.tr_shad ? A.Pn.ts : nullptr);
		}
		if(__any(one))
		{
			// estimateOneDirectLight (montecarlo.cc:70-78), light `lnum`
			for(int l = 0; l < S.n_lights; ++l)
			{
				const bool mine = one && lnum == (uint32_t)l;
				if(!__any(mine)) continue;
				neeLight<EXT, ShadeOut, NeeHbm, LEAN>(S, S.lights[l], S.mats[sp.mat], sp, wo, (uint32_t)l, pm.y, pm.x, mine, e0, neeHbm(A.Pn), A.Pn.occ, out,
				              S.tr_shad ? A.Pn.ts : nullptr);
			}
		}
	}
	if(TR)
	{
		// the in-place shadow rays join the frame's ray count (k_trace counts the queued ones)
		for(int off = 32; off > 0; off >>= 1) n_shadow += __shfl_down(n_shadow, off);
		if(laneId() == 0 && n_shadow) atomicAdd(&s_count, n_shadow);
	}
	__syncthreads();
	if(threadIdx.x == 0)
	{
		A.cnt_next.n_shadow[seg] = TR ? 0u : s_count;
		if(S.stats)
		{
			S.stats[seg].nee_requests += n_req;
			if(TR) S.stats[seg].shadow_rays += s_count;
		}
	}
	if(TR && TSTATS && S.stats)
	{
		// per-visit counters of the in-place shadow rays (the statistics frame only)
		for(int off = 32; off > 0; off >>= 1)
		{
			visits += __shfl_down(visits, off);
			tests += __shfl_down(tests, off);
		}
		if(laneId() == 0)
		{
			atomicAdd(&S.stats[seg].node_visits, (unsigned long long)visits);
			atomicAdd(&S.stats[seg].tri_tests, (unsigned long long)tests);
		}
	}
}

// ---------------------------------------------------------------------------------------------
// Deferred light pick (lpc_mode 3, r06; integrator_montecarlo.cc:70-78 with the one-thread counter
// integrator_tiled.cc:48): the path pass (k_shade<.., DEFER>) counts every sample's estimateOneDirectLight
// calls and writes one record per addition to a path colour; once the counter bases are known (lpcBases),
//   k_dfr_segoff   (before every k_shade of the path pass) this iteration's first record slot per segment;
//   k_dfr_nee      a batch of records: the light of call n of a sample is lightOfCounter(base + n), sampled as
//                  k_nee samples it (contributions at slot * K, shadow rays to the segment's queue);
//   k_trace        the batch's shadow rays;
//   k_dfr_accum    per iteration range of the batch: lcol = estimate * n_lights (+ emission), term = lcol *
//                  throughput (k_shade's connection), pcol = pcol + term per sample — iteration by iteration, so
//                  every sample's additions in the one-pass render's order;
//   k_dfr_fold     per sample: the first-vertex estimate + pcol / n (k_shade's finalize): the film is bit for bit
//                  the count-run render's.
// ---------------------------------------------------------------------------------------------
struct DfrArgs
{
	DevScene S;
	uint32_t *idx;         // per batch segment: its light-estimate records grouped by light (k_dfr_part), cap_a slots each
	uint32_t *n_rec;       // per batch segment: their count
	DevPaths P;            // contributions / occlusion bytes of the batch (slot - r0) * K
	DevQueues Q;           // the batch's shadow rays (segment s: slots r0 + s * cap_a ..)
	DevCounters cnt;       // n_active = 0, n_shadow per segment
	uint32_t r0, total;    // batch start, records of the pass
	uint32_t *dfr_total;   // running slot count of the path pass (k_dfr_segoff)
	uint32_t *overflow;
	uint32_t n_ctr;        // camera samples of the pass (k_dfr_fold)
	float4 *samples;
};

// this iteration's record slots: one per active entry, segments in order, after the earlier iterations'
__global__ void __launch_bounds__(1024) k_dfr_segoff(const uint32_t *n_active, uint32_t n_seg, uint32_t *seg_off, uint32_t *dfr_total, uint32_t cap,
                                                   uint32_t *overflow, uint32_t *it_start)
{
	__shared__ uint32_t part[1024];
	const uint32_t t = threadIdx.x;
	const uint32_t per = (n_seg + 1023u) / 1024u;
	uint32_t sum = 0;
	for(uint32_t k = 0; k < per; ++k)
	{
		const uint32_t s = t * per + k;
		if(s < n_seg) sum += n_active[s];
	}
	part[t] = sum;
	__syncthreads();
	for(uint32_t off = 1; off < 1024u; off <<= 1)
	{
		const uint32_t v = t >= off ? part[t - off] : 0u;
		__syncthreads();
		part[t] += v;
		__syncthreads();
	}
	const uint32_t base = *dfr_total;
	uint32_t run = base + part[t] - sum;
	for(uint32_t k = 0; k < per; ++k)
	{
		const uint32_t s = t * per + k;
		if(s < n_seg)
		{
			seg_off[s] = run;
			run += n_active[s];
		}
	}
	__syncthreads();
	if(t == 1023u)
	{
		// the iteration's first slot (k_dfr_accum runs the iterations in order); it_start[0] counts them
		const uint32_t k = it_start[0];
		if(k < 4095u) it_start[1u + k] = base;
		it_start[0] = k + 1u;
		const uint64_t end = (uint64_t)base + part[1023];
		*dfr_total = end > 0xffffffffull ? 0xffffffffu : (uint32_t)end;
		if(end > cap) *overflow = 1u;
	}
}

// one batch segment's light-estimate records grouped by their light (a counting sort in LDS; the order inside a
// light is irrelevant — every record is estimated on its own): k_dfr_nee's waves then sample one light with all
// lanes instead of one pass per light over a mixed wave (lane utilisation 0.37 unsorted)
constexpr int kDfrMaxLights = 16;
// Wave-aggregated LDS counters: one atomic per distinct light in the wave (per-lane atomics on two or three
// addresses serialise); returns this lane's position within its light (valid where `rec`).
__device__ __forceinline__ uint32_t waveAppendKeyed(bool rec, uint32_t key, uint32_t *ctr)
{
	uint64_t pending = __ballot(rec);
	uint32_t pos = 0;
	while(pending)
	{
		const int leader = __ffsll((unsigned long long)pending) - 1;
		const uint32_t k = (uint32_t)__shfl((int)key, leader);
		const bool mine = rec && key == k;
		const uint64_t m = __ballot(mine);
		uint32_t base = 0;
		if(laneId() == leader) base = atomicAdd(&ctr[k], (uint32_t)__popcll(m));
		base = (uint32_t)__shfl((int)base, leader);
		if(mine) pos = base + (uint32_t)__popcll(m & ((1ull << laneId()) - 1ull));
		pending &= ~m;
	}
	return pos;
}

__global__ void __launch_bounds__(1024) k_dfr_part(DfrArgs A)
{
	const DevScene &S = A.S;
	const uint32_t seg = blockIdx.x;
	const uint32_t first = A.r0 + seg * S.cap_a;
	const uint32_t n = first < A.total ? min(S.cap_a, A.total - first) : 0u;
	__shared__ uint32_t cnt[kDfrMaxLights];
	if(threadIdx.x < kDfrMaxLights) cnt[threadIdx.x] = 0u;
	__syncthreads();
	// pass 1: each record's light (its sample's counter base + the call's ordinal) replaces the spent ordinal in
	// the kind word (k_dfr_nee / k_dfr_accum read it there); counts per light
	for(uint32_t base_j = 0; base_j < n; base_j += blockDim.x)
	{
		const uint32_t jj = base_j + threadIdx.x;
		bool rec = false;
		uint32_t l = 0;
		if(jj < n)
		{
			const uint32_t slot = first + jj;
			const uint32_t kind = S.dfr_kind[slot];
			const uint32_t q = __float_as_uint(S.dfr_a[slot].w);   // (loaded with the kind; a hole's is not used)
			rec = (kind & 3u) == 1u;
			if(rec)
			{
				l = lightOfCounter(S, S.lpc[q] + (kind >> 3));
				S.dfr_kind[slot] = (kind & 7u) | (l << 3);
			}
		}
		waveAppendKeyed(rec, l, cnt);
	}
	__syncthreads();
	if(threadIdx.x == 0)
	{
		uint32_t run = 0;
		for(int l = 0; l < kDfrMaxLights; ++l)
		{
			const uint32_t c = cnt[l];
			cnt[l] = run;
			run += c;
		}
		A.n_rec[seg] = run;
	}
	__syncthreads();
	// pass 2: the slots grouped by light (the order inside a light is irrelevant)
	for(uint32_t base_j = 0; base_j < n; base_j += blockDim.x)
	{
		const uint32_t jj = base_j + threadIdx.x;
		const uint32_t kind = jj < n ? S.dfr_kind[first + jj] : 0u;
		const bool rec = (kind & 3u) == 1u;
		const uint32_t pos = waveAppendKeyed(rec, kind >> 3, cnt);
		if(rec) A.idx[(size_t)seg * S.cap_a + pos] = first + jj;
	}
}

// LEAN: no meshlight in the scene (neeLight's NOMESH: no private arrays), k_nee's occupancy
template<bool SMALL, bool LEAN>
__global__ void __launch_bounds__(kShadeBlock, LEAN ? YAF_NEE_LEAN_WAVES : YAF_NEE_MIN_WAVES) k_dfr_nee(DfrArgs A)
{
	extern __shared__ uint4 shade_smem[];
	const DevScene S_ = stageTables<SMALL>(A.S, shade_smem);
	const DevScene &S = S_;
	const uint32_t seg = blockIdx.x;
	__shared__ uint32_t s_count;
	if(threadIdx.x == 0) s_count = 0;
	__syncthreads();
	ShadeOut out;
	out.sh_count = &s_count;
	out.sh_base = seg * S.cap_s;
	out.Qn = A.Q;
	out.idx_in_o = true;
	// the segment's light-estimate records, grouped by light (k_dfr_part; every listed slot is a light estimate).
	// The loop is latency bound (4 waves per SIMD, one record per lane and trip): the next trip's slot is
	// fetched before this trip's estimate, and a record's arrays are loaded together
	const uint32_t n = A.n_rec[seg];
	const int K = S.nee_k;
	const uint32_t *list = A.idx + (size_t)seg * S.cap_a;
	uint32_t slot_next = threadIdx.x < n ? list[threadIdx.x] : A.r0;
	for(uint32_t base_j = 0; base_j < n; base_j += blockDim.x)
	{
		const uint32_t jj = base_j + threadIdx.x;
		const bool live = jj < n;
		const uint32_t slot = slot_next;
		const uint32_t kind = S.dfr_kind[slot];
		const float4 r0 = S.dfr_pp[slot], r1 = S.dfr_wo[slot], r2 = S.dfr_a[slot];
		const uint2 pix = S.dfr_pix[slot];
		slot_next = jj + blockDim.x < n ? list[jj + blockDim.x] : A.r0;
		Surf sp;
		sp.p = v3(0.f, 0.f, 0.f); sp.n = sp.ng = sp.nu = sp.nv = sp.p; sp.mat = 0; sp.flags = 0;
		sp.dcol = c3(0.f); sp.drefl = 1.f; sp.sigma = 0.f;
		uint32_t lnum = 0;
		if(live)
		{
			lnum = kind >> 3;   // k_dfr_part's pick
			sp = surfFromPrim(S, xyz(r0), __float_as_int(r0.w));
		}
		const V3 wo = xyz(r1);
		const int e0 = (int)(slot - A.r0) * K;   // (k_dfr_accum reads them by slot)
		for(int l = 0; l < S.n_lights; ++l)
		{
			const bool mine = live && lnum == (uint32_t)l;
			if(!__any(mine)) continue;
			neeLight<false, ShadeOut, NeeHbm, LEAN>(S, S.lights[l], S.mats[sp.mat], sp, wo, (uint32_t)l, pix.y, pix.x, mine,
			                                  e0, neeHbm(A.P), A.P.occ, out, nullptr);
		}
	}
	__syncthreads();
	if(threadIdx.x == 0)
	{
		A.cnt.n_shadow[seg] = s_count;
		A.cnt.n_active[seg] = 0u;
	}
}

// the terms of slots [r0, total) of one iteration (a sample has at most one record per iteration, and the
// iterations' ranges are processed in order): a light estimate becomes lcol = estimate * n_lights (+ emission),
// term = lcol * throughput (k_shade's connection, its contributions at (slot - batch) * K of this batch), a known
// term is taken as it is, and pcol = pcol + term per sample (the additions of the one-pass render, in order)
__global__ void __launch_bounds__(256) k_dfr_accum(DfrArgs A, float4 *pcol, uint32_t batch0)
{
	const DevScene &S = A.S;
	const uint32_t slot = A.r0 + blockIdx.x * blockDim.x + threadIdx.x;
	if(slot >= A.total) return;
	const uint32_t kind = S.dfr_kind[slot];
	if((kind & 3u) == 0u) return;
	const float4 a = S.dfr_a[slot];
	C3 term = rgb(a);
	if((kind & 3u) == 1u)
	{
		const uint32_t lnum = kind >> 3;   // k_dfr_part's pick
		const int kb = (int)(slot - batch0) * S.nee_k;
		auto ge = [&](int k) { return f4(neeGet(neeHbm(A.P), k), 1.f); };
		auto go = [&](int k) { return A.P.occ[k] != 0; };
		// path_tracer.cc:201-207 / :244-266 as k_shade connects it
		C3 lcol = neeSumT(S.lights[lnum], kb, ge, go) * (float)S.n_lights;
		if(kind & 4u) lcol = lcol + rgb(S.dfr_emit[slot]);
		term = lcol * term;
	}
	// the sample's colour as one aligned 16-B record: one load and one store (three 4-B read-modify-writes
	// of a 12-B record before)
	const uint32_t q = __float_as_uint(a.w);
	const float4 pc = pcol[q];
	pcol[q] = make_float4(pc.x + term.r, pc.y + term.g, pc.z + term.b, 0.f);
}

// per camera sample of the pass: the first-vertex estimate + the paths' colour (k_shade's finalize)
__global__ void __launch_bounds__(256) k_dfr_fold(DfrArgs A, const float4 *pcol)
{
	const DevScene &S = A.S;
	const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
	if(q >= A.n_ctr) return;
	const uint32_t v = S.dfr_last[q];
	if(v == 0xffffffffu) return;   // not finalized in this pass
	const float4 c4 = A.samples[q];
	C3 col = rgb(c4);
	if(v & 1u) col = col + rgb(pcol[q]) / (float)max(1, S.path_samples);
	col = col + c3(0.f);   // recursiveRaytrace: no specular / glossy component (k_shade's finalize)
	A.samples[q] = f4(col, c4.w);
}

// ---------------------------------------------------------------------------------------------
// k_path: the megakernel form of the same integrator for scenes that live in LDS.  One lane carries
// one camera sample through its whole integrate() — k_camera's ray, then per vertex k_trace's
// closest hit, k_shade's state machine (the compact record's stages, flags and deferred
// connection) and k_nee's light sampling, whose shadow rays the lane traces in place — and takes the
// next sample of its wave's pool when the sample is written.  The path state stays in registers and
// the NEE contributions in LDS, so none of the wavefront's per-vertex HBM traffic (~270 B of state
// and queues per vertex, ~125 B per NEE request) exists; HBM sees the camera samples' film records
// only.  Every function on the way is the wavefront's own (cameraRay, traverse4, makeSurf,
// matSample / matEmit, neeLight, neeSum), called in the same order per sample, so the film is
// bit-identical to the wavefront's.  Eligible: non-EXT materials, BVH4 scene + stack bound in LDS,
// PathIntegrator / DirectLight without AO, photon or caustic maps, transparent shadows (render.cc
// pathEligible).
// ---------------------------------------------------------------------------------------------
constexpr int kPathMaxK = 8;        // NEE entries per vertex kept per lane in LDS
constexpr int kPathBatch = 256;     // samples a wave takes from the chunk counter at a time

struct PathArgs
{
	DevScene S;
	float4 *samples;       // frame sample buffer [(y * W + x) * spp + s]
	const DevJob *jobs;
	int n_jobs;
	uint64_t chunk_base;
	uint32_t n;            // samples of the chunk
	uint32_t *next;        // the chunk's sample counter (zero at launch)
	int stack_depth;       // traversal stack levels (all in LDS)
};

__host__ __device__ inline size_t pathLdsBytes(const DevScene &S, int stack_depth)
{
	return shadeLdsBytes(S, true) + (size_t)(S.node_f4 * S.n_nodes + 3 * S.n_tris) * 16 + (size_t)stack_depth * kTraceBlock * 4 +
	       (size_t)kTraceBlock * S.nee_k * (16 + 32) + (((size_t)kTraceBlock * S.nee_k + 15) & ~(size_t)15);
}

// k_path's register budget: 2 waves per SIMD (<= 256 VGPRs incl. AGPRs; the unconstrained
// allocation took 260 -> 1 wave); -DYAF_PATH_WAVES=n for tuning
#ifndef YAF_PATH_WAVES
#define YAF_PATH_WAVES 2
#endif
template<bool STATS>
__global__ void __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(YAF_PATH_WAVES))) k_path(PathArgs A)
{
	extern __shared__ uint4 path_smem[];
	const DevScene S = stageTables<true>(A.S, path_smem);
	const int K = S.nee_k;
	const int lane = threadIdx.x;
	float4 *lds_nodes = reinterpret_cast<float4 *>(path_smem) + shadeLdsBytes(S, true) / 16;
	float4 *lds_tris = lds_nodes + S.node_f4 * S.n_nodes;
	int *stack = reinterpret_cast<int *>(lds_tris + 3 * S.n_tris);
	float4 *nee_all = reinterpret_cast<float4 *>(stack + A.stack_depth * kTraceBlock);
	float4 *rec_all = nee_all + kTraceBlock * K;
	uint8_t *occ_all = reinterpret_cast<uint8_t *>(rec_all + 2 * kTraceBlock * K);
	for(int k = threadIdx.x; k < S.node_f4 * S.n_nodes; k += blockDim.x) lds_nodes[k] = A.S.nodes[k];
	for(int k = threadIdx.x; k < 3 * S.n_tris; k += blockDim.x) lds_tris[k] = A.S.tris[k];
	__syncthreads();
	TraceCtx C;
	C.wave_base = waveBase();
	C.nodes = lds_nodes;
	C.tris = lds_tris;
	C.stack = stack;
	C.lds_depth = A.stack_depth;
	C.spill = nullptr;
	C.spill_stride = 0;
	float4 *nee = nee_all + lane * K;
	float4 *rec = rec_all + 2 * lane * K;
	uint8_t *occ = occ_all + lane * K;
	const PathShadows out{rec, 0};
	const bool is_path = S.integrator == INT_PATH;
	const uint32_t n_paths = (uint32_t)max(1, S.path_samples);
	const float inf = __builtin_huge_valf();

	// the lane's sample: record of k_shade's compact form, in registers
	bool active = false;
	uint32_t sid = 0, stage = ST_NORAY, flags = 0, offset = 0, sample_idx = 0;
	uint2 rng = make_uint2(0u, 0u);
	float w = 0.f;
	C3 thr = c3(0.f), col = c3(0.f), pcol = c3(0.f), pthr = c3(0.f), pem = c3(0.f);
	V3 pwo = v3(0.f, 0.f, 0.f), ray_o = pwo, ray_d = pwo;
	float ray_tmin = 0.f, ray_tmax = 0.f;
	float4 v0p4 = make_float4(0.f, 0.f, 0.f, 0.f), v0wo4 = v0p4;
	SampleCoord sc{0, 0, 0};
	// the wave's pool of chunk samples [pool, pool_end) (wave-uniform)
	uint32_t pool = 0, pool_end = 0;
	bool exhausted = false;
	uint32_t n_closest = 0, n_shadow = 0, n_vert = 0, n_nee = 0, visits = 0, tests = 0;
	PHASE_DECL
	for(;;)
	{
		// ---- samples for the idle lanes (k_camera) ----
		const uint64_t need = __ballot(!active);
		if(need && !exhausted)
		{
			if(pool == pool_end)
			{
				uint32_t b = 0;
				if(laneId() == 0) b = atomicAdd(A.next, (uint32_t)kPathBatch);
				b = __shfl(b, 0);
				pool = min(b, A.n);
				pool_end = (uint32_t)min((uint64_t)b + kPathBatch, (uint64_t)A.n);
				if(pool == pool_end) exhausted = true;
			}
			const uint32_t avail = pool_end - pool;
			const uint32_t rank = (uint32_t)__popcll(need & ((1ull << laneId()) - 1ull));
			if(!active && rank < avail)
			{
				sid = pool + rank;
				sc = sampleAt(S, A.jobs, A.n_jobs, A.chunk_base + (uint64_t)sid);
				uint32_t seed;
				cameraRay(S, sc, ray_o, ray_d, ray_tmin, ray_tmax, seed);
				offset = fnv32((uint32_t)(sc.y + S.crop_y0) * fnv32((uint32_t)(sc.x + S.crop_x0)));
				sample_idx = S.base_offset + S.pass_offset + (uint32_t)sc.s;
				rng = make_uint2(30903u, seed);
				stage = ST_CAMERA;
				flags = 0;
				w = 0.f;
				thr = col = pcol = c3(0.f);
				active = true;
			}
			pool += min(avail, (uint32_t)__popcll(need));
		}
		if(!__any(active))
		{
			if(exhausted) break;
			continue;
		}
		PHASE(0);
		const bool live = active;
		const uint32_t st = stage & 0xffu;
		uint32_t subpath = (stage >> 8) & 0xfffu;
		int depth = (int)(stage >> 20);

		// ---- the rays this sample owes: the last NEE's shadow rays + the closest ray (k_trace) ----
		float hit_t = 0.f;
		int hit_prim = -1;
		{
			const bool sh = live && (flags & (F_PEND_V0 | F_PEND_ONE)) != 0;
			const bool cl = live && st != ST_NORAY;
			if(__any(sh || cl))
				traceLaneRays<STATS>(C, rec, occ, K, sh, cl, ray_o, ray_d, ray_tmin, ray_tmax >= 0.f ? ray_tmax : inf, hit_t, hit_prim, visits, tests,
				                     n_closest, n_shadow);
		}
		if(live) ++n_vert;
		PHASE(1);

		// ---- 1. connect the pending next-event estimate (k_shade step 1) ----
		if(live && (flags & F_PEND_V0))
		{
			C3 total = c3(0.f);
			for(int l = 0; l < S.n_lights; ++l) total = total + neeSum(S, S.lights[l], nee, occ, (int)S.lights[l].nee_base);
			col = col + total;
		}
		if(live && (flags & F_PEND_ONE))
		{
			const int lnum = (int)(flags >> F_LNUM_SHIFT);
			C3 lcol = neeSum(S, S.lights[lnum], nee, occ, 0) * (float)S.n_lights;
			if(flags & F_PEND_EMIT) lcol = lcol + pem;
			pcol = pcol + lcol * pthr;
		}
		flags &= ~(F_PEND_V0 | F_PEND_ONE | F_PEND_EMIT | F_AO_EMIT);

		// ---- 2. the new hit ----
		Surf sp;
		sp.p = v3(0.f, 0.f, 0.f); sp.n = sp.ng = sp.nu = sp.nv = sp.p; sp.mat = 0; sp.flags = 0;
		sp.dcol = c3(0.f); sp.drefl = 1.f; sp.sigma = 0.f;
		V3 wo = v3(0.f, 0.f, 1.f);
		bool have_hit = false;
		if(live && st != ST_NORAY && hit_prim >= 0)
		{
			have_hit = true;
			sp = makeSurf(S, ray_o, ray_d, hit_t, hit_prim);
			wo = -ray_d;
		}
		bool nee_v0 = false, nee_one = false, sample_next = false, end_sub = false, finalize = false, start_sub = false;
		C3 emit_pend = c3(0.f), pend_thr = c3(0.f);
		if(live)
		{
			if(st == ST_NORAY) end_sub = true;
			else if(st == ST_CAMERA)
			{
				if(!have_hit)
				{
					// integrator_tiled.cc:707-720 background
					C3 bg = c3(0.f);
					float a = 1.f;
					if(S.bg_transp) a = 0.f;
					else if(S.has_bg) bg = C3{S.bg[0], S.bg[1], S.bg[2]};
					A.samples[((size_t)sc.y * S.width + sc.x) * S.spp + sc.s] = f4(bg, a);
				}
				else
				{
					const DevMaterial &m = S.mats[sp.mat];
					col = c3(0.f);
					if(sp.flags & B_EMIT) col = col + matEmit<false>(m, sp, wo);
					if(sp.flags & B_DIFFUSE) { nee_v0 = true; flags |= F_V0_DIFFUSE; }
					if(is_path && (sp.flags & B_DIFFUSE))
					{
						v0p4 = f4(sp.p, __int_as_float(hit_prim));
						v0wo4 = f4(wo, 0.f);
						start_sub = true;
						subpath = 0;
					}
					else end_sub = true;
				}
			}
			else if(st == ST_FIRST)
			{
				if(!have_hit) end_sub = true;     // path_tracer.cc:192 `continue`
				else
				{
					// path_tracer.cc:193-207
					if(flags & F_SAMPLED) pwo = wo;
					else wo = pwo;
					nee_one = true;
					flags = (flags & ~F_MATFLAGS) | (sp.flags & F_MATFLAGS);
					if(sp.flags & B_EMIT) { emit_pend = matEmit<false>(S.mats[sp.mat], sp, wo); flags |= F_PEND_EMIT; }
					pend_thr = thr;
					depth = 1;
					sample_next = true;
				}
			}
			else   // ST_BOUNCE
			{
				if(!have_hit) end_sub = true;     // path_tracer.cc:235
				else
				{
					const uint32_t mfl = flags & F_MATFLAGS;
					pwo = wo;
					bool killed = false;
					if(depth > S.rr_min_bounces)
					{
						// path_tracer.cc:249-255 (the wavefront's stateless draw)
						const float random_value = rrRandom(S, sc, subpath, depth);
						const float probability = maxComp(thr);
						if(probability <= 0.f || probability < random_value) killed = true;
						else thr = thr * rcpExact(probability);
					}
					if(killed) end_sub = true;
					else
					{
						if((mfl & B_EMIT) && (flags & F_CAUSTIC)) { emit_pend = matEmit<false>(S.mats[sp.mat], sp, wo); flags |= F_PEND_EMIT; }
						if(mfl & B_DIFFUSE) { nee_one = true; pend_thr = thr; }
						else
						{
							C3 lcol = c3(0.f);
							if(flags & F_PEND_EMIT) lcol = lcol + emit_pend;
							pcol = pcol + lcol * thr;
							flags &= ~F_PEND_EMIT;
						}
						++depth;
						sample_next = true;
					}
				}
			}
		}
		uint32_t lnum = 0;
		if(nee_one)
		{
			// integrator_montecarlo.cc:70-78 light pick (as k_shade)
			lnum = pickLight(S, offset, sample_idx, (uint32_t)depth + subpath * (uint32_t)S.bounces, n_paths * (uint32_t)(S.bounces + 1));
			flags = (flags & ((1u << F_LNUM_SHIFT) - 1u)) | (lnum << F_LNUM_SHIFT) | F_PEND_ONE;
		}
		if(nee_v0) flags |= F_PEND_V0;
		const bool pending = (flags & (F_PEND_V0 | F_PEND_ONE)) != 0;

		PHASE(2);
		// ---- 3. next segment: one material sample per lane (k_shade's two sampling sites merged) ----
		bool want_ray = false;
		V3 nray_o = v3(0.f, 0.f, 0.f), nray_d = v3(0.f, 0.f, 1.f);
		const bool try_next = live && sample_next && depth < S.bounces;
		if(live && sample_next && !try_next) end_sub = true;
		// the end of a subpath known before sampling: next subpath (path_tracer.cc:166) or the end
		if(live && !try_next && end_sub && !pending)
		{
			if(is_path && (flags & F_V0_DIFFUSE) && subpath + 1 < n_paths) { start_sub = true; ++subpath; }
			else finalize = true;
		}
		for(int pass = 0; pass < 2; ++pass)
		{
			// pass 0: the continuing lanes (path_tracer.cc:211-234, loop iteration `depth`) and the lanes
			// starting a subpath (:168-191); pass 1: the lanes whose continuation drew nothing and start
			// their next subpath (path_samples > 1)
			const bool smp = pass == 0 ? (try_next || (live && start_sub)) : (live && start_sub);
			if(!__any(smp)) continue;
			const bool cont = pass == 0 && try_next;
			Surf ss = sp;
			V3 wos = wo;
			const uint32_t offs = n_paths * sample_idx + offset + subpath;
			BsdfSample s;
			s.pdf = 0.f;
			s.sampled = B_NONE;
			if(cont)
			{
				const int d_4 = 4 * depth;
				s.s_1 = ldsDim(S, d_4 + 3, offs);
				s.s_2 = ldsDim(S, d_4 + 4, offs);
				s.flags = B_ALL;
			}
			else
			{
				if(st != ST_CAMERA && smp) ss = surfFromPrim(S, xyz(v0p4), __float_as_int(v0p4.w));
				if(st != ST_CAMERA) wos = xyz(v0wo4);
				s.s_1 = riVdC(offs);
				s.s_2 = ldsDim(S, 2, offs);
				s.flags = B_DIFFUSE | B_REFLECT | B_TRANSMIT;
			}
			V3 dir = v3(0.f, 0.f, 0.f);
			float wnew = w;
			C3 scol = c3(0.f);
			if(smp) scol = matSample<false>(S.mats[ss.mat], ss, wos, dir, s, wnew);
			if(smp) w = wnew;
			if(cont)
			{
				scol = scol * w;
				if(isBlack(scol)) end_sub = true;
				else
				{
					thr = thr * scol;
					if(S.caustic_path && (s.sampled & (B_SPECULAR | B_GLOSSY | B_FILTER))) flags |= F_CAUSTIC;
					else flags &= ~F_CAUSTIC;
					nray_o = sp.p;
					nray_d = dir;
					want_ray = true;
					stage = ST_BOUNCE | (subpath << 8) | ((uint32_t)depth << 20);
				}
			}
			else if(smp)
			{
				thr = scol * w;
				pwo = wos;
				if(s.sampled != B_NONE) flags |= F_SAMPLED;
				else flags &= ~F_SAMPLED;
				flags &= ~F_CAUSTIC;
				nray_o = ss.p;
				nray_d = dir;
				want_ray = true;
				stage = ST_FIRST | (subpath << 8);
			}
			if(pass == 0)
			{
				start_sub = false;
				if(cont && end_sub && !pending)
				{
					if(is_path && (flags & F_V0_DIFFUSE) && subpath + 1 < n_paths) { start_sub = true; ++subpath; }
					else finalize = true;
				}
			}
		}
		PHASE(3);
		if(live && finalize)
		{
			// path_tracer.cc:274-278 / direct_light.cc:129-131
			if(is_path && (flags & F_V0_DIFFUSE)) col = col + pcol / (float)n_paths;
			col = col + c3(0.f);   // recursiveRaytrace: no specular/glossy component
			A.samples[((size_t)sc.y * S.width + sc.x) * S.spp + sc.s] = f4(col, 1.f);
		}
		// ---- 4. the sample goes on (k_shade's compaction) ----
		active = live && (want_ray || pending);
		if(active)
		{
			if(want_ray)
			{
				ray_o = nray_o;
				ray_d = nray_d;
				ray_tmin = S.ray_min_dist;
				ray_tmax = -1.f;
			}
			else stage = ST_NORAY | (subpath << 8) | ((uint32_t)depth << 20);
			if(nee_one) pthr = pend_thr;
			if(flags & F_PEND_EMIT) pem = emit_pend;
		}

		PHASE(4);
		// ---- 5. next-event estimation (k_nee): contributions into LDS, shadow rays recorded for the
		// next trip's trace ----
		const bool all = live && nee_v0, one = live && nee_one;
		if(__any(all || one))
		{
			if(all || one)
				for(int e = 0; e < K; ++e) rec[2 * e + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
			const DevMaterial &m = S.mats[sp.mat];
			// estimateAllDirectLight (montecarlo.cc:54-68: every light, at its nee_base) and
			// estimateOneDirectLight (:70-78: light `lnum`, at 0) in one pass over the lights
			for(int l = 0; l < S.n_lights; ++l)
			{
				const bool mine = all || (one && lnum == (uint32_t)l);
				if(!__any(mine)) continue;
				neeLight<false>(S, S.lights[l], m, sp, wo, (uint32_t)l, sample_idx, offset, mine, all ? (int)S.lights[l].nee_base : 0, nee, occ, out);
			}
			if(all || one) ++n_nee;
		}
		PHASE(5);
	}
	PHASE_FLUSH;
	// statistics: the wave sums, one read-modify-write per workgroup into its own record
	for(int off = 32; off > 0; off >>= 1)
	{
		n_closest += __shfl_down(n_closest, off);
		n_shadow += __shfl_down(n_shadow, off);
		n_vert += __shfl_down(n_vert, off);
		n_nee += __shfl_down(n_nee, off);
		visits += __shfl_down(visits, off);
		tests += __shfl_down(tests, off);
	}
	__shared__ uint32_t red[kTraceBlock / 64][6];
	const int wid = threadIdx.x >> 6;
	if(laneId() == 0)
	{
		red[wid][0] = n_closest; red[wid][1] = n_shadow; red[wid][2] = visits;
		red[wid][3] = tests; red[wid][4] = n_vert; red[wid][5] = n_nee;
	}
	__syncthreads();
	if(threadIdx.x < 6 && S.stats)
	{
		unsigned long long v = 0;
		for(int k = 0; k < kTraceBlock / 64; ++k) v += red[k][threadIdx.x];
		unsigned long long *r = &S.stats[blockIdx.x].closest_rays;   // closest, shadow, visits, tests, shade entries, NEE requests
		if(v) r[threadIdx.x] += v;
	}
}

// ---------------------------------------------------------------------------------------------
// k_film: deterministic gather splat + flush normalisation
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int roundToInt(double v) { return (int)(v + (.5 - 1.4e-11)); }
__device__ __forceinline__ int floorToInt(double v) { return (int)floor(v); }

// rank of a pixel in the single-thread tile order (imagesplitter.cc:30-107): tiles by their rank
// (linear when F.tile_rank is null), pixels row-major inside a tile (integrator_tiled.cc:288-290)
__device__ __forceinline__ uint32_t tileRankOf(const DevFilm &F, int x, int y)
{
	const int ty = y / F.tile, tx = x / F.tile;
	return F.tile_rank ? F.tile_rank[ty * F.ntx + tx] : (uint32_t)(ty * F.ntx + tx);
}
__device__ __forceinline__ uint64_t pixelRank(const DevFilm &F, int x, int y, int W, int H, int ts)
{
	const int ty = y / ts, tx = x / ts;
	const int tw = min(ts, W - tx * ts);
	return (uint64_t)tileRankOf(F, x, y) * (uint64_t)ts * ts + (uint64_t)(y - ty * ts) * tw + (x - tx * ts);
}

// RF / RB: compile-time footprint reach (box and gauss filters: RF = 1, RB = 0 -> a 2x2 window
// kept in registers); RF = RB = -1 selects the generic runtime window (<= 9x9).
template<int RF, int RB>
__global__ void __launch_bounds__(256) k_film(DevFilm F, const float4 *samples, const uint8_t *flags, float4 *accum,
                                              float4 *out, float *weights, int y0, int y1, float clamp_samples, int accumulate)
{
	constexpr bool kStatic = RF >= 0;
	constexpr int kWin = kStatic ? (RF + RB + 1) * (RF + RB + 1) : 81;
	const int x = blockIdx.x * blockDim.x + threadIdx.x;
	const int y = y0 + blockIdx.y;
	if(x >= F.width || y >= y1) return;
	const int W = F.width, H = F.height, spp = F.spp;
	const int rf = kStatic ? RF : F.reach_fwd, rb = kStatic ? RB : F.reach_back;
	// candidate sources, sorted by their rank in the reference's splat order
	int sx[kWin], sy[kWin];
	uint64_t rk[kWin];
	int n = 0;
	const uint32_t own_tile = F.partial ? tileRankOf(F, x, y) : 0u;
#pragma unroll
	for(int dyy = 0; dyy < (kStatic ? RF + RB + 1 : 9); ++dyy)
	{
#pragma unroll
		for(int dxx = 0; dxx < (kStatic ? RF + RB + 1 : 9); ++dxx)
		{
			if(!kStatic && (dyy > rf + rb || dxx > rf + rb)) continue;
			const int yy = y - rf + dyy, xx = x - rf + dxx;
			if(yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
			if(F.partial && tileRankOf(F, xx, yy) > own_tile) continue;   // tile not finished yet
			const uint64_t r = pixelRank(F, xx, yy, W, H, F.tile);
			int p = n++;
			while(p > 0 && rk[p - 1] > r) { rk[p] = rk[p - 1]; sx[p] = sx[p - 1]; sy[p] = sy[p - 1]; --p; }
			rk[p] = r; sx[p] = xx; sy[p] = yy;
		}
	}
	const size_t p = (size_t)y * W + x;
	// adaptive passes add to the film of the earlier passes (imagefilm.cc addSample: += per sample)
	float wsum = accumulate ? weights[p] : 0.f;
	float4 acc = accumulate ? accum[p] : make_float4(0.f, 0.f, 0.f, 0.f);
	const float d_1 = 1.f / (float)spp;
	for(int c = 0; c < n; ++c)
	{
		const int px = sx[c], py = sy[c];
		const uint32_t offset = fnv32((uint32_t)(py + F.crop_y0) * fnv32((uint32_t)(px + F.crop_x0)));
		const int ox = x - px, oy = y - py;
		// adaptive pass: only resampled pixels splat.  (Skipping them while building the candidate list
		// instead lost diagonal candidates in the unrolled k_film<1, 0> — tools/film_probe.hip.)
		const int ns = (flags && !flags[(size_t)py * W + px]) ? 0 : spp;
		for(int s = 0; s < ns; ++s)
		{
			float dx = 0.5f, dy = 0.5f;
			if(F.multipass)
			{
				dx = riVdC(F.sample_offset + (uint32_t)s, offset);
				dy = riS(F.sample_offset + (uint32_t)s, offset);
			}
			else if(spp > 1)
			{
				dx = (0.5f + (float)s) * d_1;
				dy = riLp((uint32_t)s + offset);
			}
			// imagefilm.cc:684-707 footprint of this sample, then the table weight at (x, y)
			const int dx_0 = max(0 - px, roundToInt((double)dx - F.filterw));
			const int dx_1 = min(W - px - 1, roundToInt((double)dx + F.filterw - 1.0));
			const int dy_0 = max(0 - py, roundToInt((double)dy - F.filterw));
			const int dy_1 = min(H - py - 1, roundToInt((double)dy + F.filterw - 1.0));
			if(ox < dx_0 || ox > dx_1 || oy < dy_0 || oy > dy_1) continue;
			const int xi = floorToInt(fabs(((double)ox - (dx - 0.5)) * F.table_scale));
			const int yi = floorToInt(fabs(((double)oy - (dy - 0.5)) * F.table_scale));
			const float wt = F.table[yi * 16 + xi];
			wsum = wsum + wt;
			const float4 col = samples[((size_t)py * W + px) * spp + s];
			float r = col.x, g = col.y, b = col.z;
			if(clamp_samples > 0.f)
			{
				// color.h:415-440 clampProportionalRgb
				const float max_rgb = fmaxf(r, fmaxf(g, b));
				const float adj = clamp_samples / max_rgb;
				if(max_rgb > clamp_samples)
				{
					if(r >= max_rgb) { r = clamp_samples; g *= adj; b *= adj; }
					else if(g >= max_rgb) { g = clamp_samples; r *= adj; b *= adj; }
					else { b = clamp_samples; r *= adj; g *= adj; }
				}
			}
			acc.x = acc.x + r * wt;
			acc.y = acc.y + g * wt;
			acc.z = acc.z + b * wt;
			acc.w = acc.w + col.w * wt;
		}
	}
	if(!F.partial)
	{
		weights[p] = wsum;
		accum[p] = acc;
	}
	// Rgba::normalized (color.h:554-558): colour * (1 / weight) — operator/ takes the reciprocal first
	if(wsum != 0.f)
	{
		const float inv = 1.f / wsum;
		out[p] = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
	}
	else out[p] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Canceled render (integrator_tiled.cc:292: a canceled worker stops before its next pixel, so a
// pixel is either fully sampled or not at all): flags the pixels whose samples the completed
// chunks rendered, for k_film's `flags` argument.  Pass 0 enumerates the jobs (pixel ranks
// [0, n_pix)); an adaptive pass (plist) clears the flags of its pixels beyond `done_pix`.
__global__ void __launch_bounds__(256) k_done_flags(DevScene S, const DevJob *jobs, int n_jobs, uint32_t n_pix, uint32_t done_pix,
                                                    uint8_t *flags)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n_pix) return;
	if(S.plist)
	{
		if(p >= done_pix) flags[S.plist[p]] = 0;
		return;
	}
	const SampleCoord c = sampleCoord(jobs, n_jobs, S.width, S.tile, S.spp, (uint64_t)p * (uint64_t)S.spp);
	flags[(size_t)c.y * S.width + c.x] = p < done_pix ? 1 : 0;
}

// ---------------------------------------------------------------------------------------------
// light-pick counters (DevScene::lpc, render.cc lpcBases).  A row segment = one row of one tile: its
// pixels' counters (spp each) are contiguous in the pixel-major layout, and the one-thread render
// visits them in that order (renderTile, integrator_tiled.cc:281-345: rows, then pixels, then
// samples).  k_lpc_seg sums each segment of rows [y0, y1); k_lpc_prefix turns each segment's
// counts into the counter values its samples start from: the segment's base (the calls of every
// sample visited before the segment, from the host) + the exclusive prefix sum inside it.
// One wave per segment.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_lpc_seg(const uint32_t *lpc, int W, int spp, int ts, int y0, int y1, uint32_t *seg)
{
	const int ntx = (W + ts - 1) / ts;
	const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) / 64u), lane = (int)(threadIdx.x & 63u);
	if(wave >= (y1 - y0) * ntx) return;
	const int y = y0 + wave / ntx, tx = wave % ntx;
	const int x0 = tx * ts, x1 = min(W, x0 + ts);
	const size_t b = ((size_t)y * W + x0) * spp, n = (size_t)(x1 - x0) * spp;
	uint32_t acc = 0;
	for(size_t k = lane; k < n; k += 64) acc += lpc[b + k];
	for(int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off);
	if(lane == 0) seg[(size_t)y * ntx + tx] = acc;
}

__global__ void __launch_bounds__(256) k_lpc_prefix(uint32_t *lpc, int W, int spp, int ts, int y0, int y1, const uint32_t *segbase)
{
	const int ntx = (W + ts - 1) / ts;
	const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) / 64u), lane = (int)(threadIdx.x & 63u);
	if(wave >= (y1 - y0) * ntx) return;
	const int y = y0 + wave / ntx, tx = wave % ntx;
	const int x0 = tx * ts, x1 = min(W, x0 + ts);
	const size_t b = ((size_t)y * W + x0) * spp, n = (size_t)(x1 - x0) * spp;
	uint32_t carry = segbase[(size_t)y * ntx + tx];
	for(size_t k0 = 0; k0 < n; k0 += 64)
	{
		const size_t k = k0 + (size_t)lane;
		const uint32_t v = k < n ? lpc[b + k] : 0u;
		uint32_t x = v;
		for(int off = 1; off < 64; off <<= 1)
		{
			const uint32_t t = __shfl_up(x, off);
			if(lane >= off) x += t;
		}
		if(k < n) lpc[b + k] = carry + (x - v);
		carry += __shfl(x, 63);
	}
}

// ---------------------------------------------------------------------------------------------
// ray-level entry (batched Accelerator::intersect / isShadowed for parity tests and hosts)
// ---------------------------------------------------------------------------------------------
template<bool ANY, bool WIDE>
__global__ void __launch_bounds__(kTraceBlock) k_trace_rays(DevScene S, const float4 *ro, const float4 *rd, int n,
                                                           float *t_out, int *prim_out, int stack_depth)
{
	extern __shared__ float4 smem[];
	TraceCtx C;
	C.wave_base = waveBase();
	C.stack = reinterpret_cast<int *>(smem);
	C.lds_depth = stack_depth;   // the full bound: no spill (traverse<..., SPILL = false>)
	C.spill = nullptr;
	C.spill_stride = 0;
	C.nodes = S.nodes;
	C.tris = S.tris;
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= n) return;
	const float4 o = ro[i], d = rd[i];
	uint32_t v = 0, t = 0;
	float tb;
	int pb;
	if(ANY)
	{
		// accelerator.cc:69-78
		V3 so;
		float tm;
		shadowRayOf(xyz(o), xyz(d), o.w, d.w, so, tm);
		const bool occ = traverse<true, WIDE, false>(C, so, xyz(d), 0.f, tm, tb, pb, v, t);
		t_out[i] = occ ? 1.f : 0.f;
		prim_out[i] = occ ? pb : -1;
	}
	else
	{
		const float tmax = (d.w >= 0.f) ? d.w : __builtin_huge_valf();
		const bool hit = traverse<false, WIDE, false>(C, xyz(o), xyz(d), o.w, tmax, tb, pb, v, t);
		t_out[i] = hit ? tb : -1.f;
		prim_out[i] = hit ? pb : -1;
	}
}

// =============================================================================================
// Photon mapping (integrator_photon_mapping.cc, BASELINE C5)
// =============================================================================================
// Photon paths are shot as a wavefront of their own: k_photon_emit starts every photon id h
// (integrator_photon_mapping.cc:127-156), then one k_photon_bounce launch per bounce traces the
// rays, deposits on diffuse hits and scatters (:162-219).  Deposits land in slot
// h * (bounces + 1) + bounce, so a stable compaction of the slots yields the photon map in
// exactly the order one reference thread would append it (photon id, then bounce).

// sample.h:58-75 (uniform sphere; the angle is a long double product)
__device__ __forceinline__ V3 sphereDir(float s_1, float s_2)
{
	V3 dir;
	dir.z = 1.0f - 2.0f * s_1;
	float r = 1.0f - dir.z * dir.z;
	if(r > 0.0f)
	{
		r = sqrtf(r);
		const float a = x87mul(kMultPiBy2, s_2);
		dir.x = fcos(a) * r;
		dir.y = fsin(a) * r;
	}
	else
	{
		dir.x = 0.0f;
		dir.y = 0.0f;
	}
	return dir;
}


constexpr uint32_t kDeadPhoton = 0xffffffffu;   // a hole in the segmented alive list (k_photon_emit)

struct PhotonArgs
{
	DevScene S;
	PhotonState P;
	PhotonSet L;         // the shooting lights and the map kind (diffuse / caustic)
	uint32_t n_photons;  // photon paths of the whole map (rounded like the reference, :437)
	uint32_t h0, n_local;   // this launch's photon ids [h0, h0 + n_local) (a group member's share); the
	                        // path buffers and deposit slots are indexed by the local id h - h0
	int max_bounces;
	int bounce;          // k_photon_bounce: the bounce this launch traces
	int cur;             // alive list read by this launch
	int stack_depth;   // LDS stack levels (deeper levels spill, BVH4)
	int *spill;
};

// :127-156 — photon id h: light pick by Pdf1D::dSample over the lights' energies, emitPhoton
__global__ void __launch_bounds__(256) k_photon_emit(PhotonArgs A)
{
	const DevScene &S = A.S;
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;   // local id
	const uint32_t h = A.h0 + i;                                 // photon id
	bool ok = i < A.n_local;
	V3 o = v3(0.f, 0.f, 0.f), d = o;
	C3 pcol = c3(0.f);
	if(ok)
	{
		const float s_1 = riVdC(h);
		const float s_2 = ldsDim(S, 2, h);
		const float s_3 = ldsDim(S, 3, h);
		const float s_4 = ldsDim(S, 4, h);
		// diffuseWorker: h * (1 / n) (:133); causticWorker: h / n (integrator_montecarlo.cc:444)
		const float s_l = A.L.caustic ? float(h) / static_cast<float>(A.n_photons) : float(h) * (1.f / static_cast<float>(A.n_photons));
		// sample_pdf1d.h:77-93 dSample (lower_bound over the cdf)
		const int nl = A.L.n_lights;
		int light_num;
		if(s_l <= 0.f) light_num = 0;
		else if(s_l >= 1.f) light_num = nl - 1;
		else
		{
			light_num = 0;
			while(light_num < nl && A.L.cdf[light_num] < s_l) ++light_num;
			if(light_num >= nl) light_num = nl - 1;
		}
		const float light_num_pdf = A.L.func[light_num] * A.L.inv_integral;
		const DevLight &L = S.lights[A.L.lights[light_num]];
		float light_pdf;
		// light_area.cc:98-104, light_point.cc:79-85
		if(L.type == LIGHT_POINT)
		{
			o = lv(L.pos);
			d = sphereDir(s_1, s_2);
			light_pdf = x87mul(kPi, 4.0f);
		}
		else if(L.type == LIGHT_MESH)
		{
			// light_object_light.cc:148-163
			light_pdf = L.area;
			V3 n;
			meshSampleSurface(S, L, s_3, s_4, o, n);
			V3 cu, cv;
			coordsSystem(n, cu, cv);
			if(L.double_sided)
			{
				light_pdf *= 2.f;
				if(s_1 > 0.5f) d = cosHemisphere(-n, cu, cv, (s_1 - 0.5f) * 2.f, s_2);
				else d = cosHemisphere(n, cu, cv, s_1 * 2.f, s_2);
			}
			else d = cosHemisphere(n, cu, cv, s_1, s_2);
		}
		else
		{
			light_pdf = L.area;
			o = lv(L.pos) + s_3 * lv(L.to_x) + s_4 * lv(L.to_y);
			d = cosHemisphere(-lv(L.fnormal), lv(L.du), lv(L.dv), s_1, s_2);
		}
		const float f_num_lights = static_cast<float>(nl);
		pcol = C3{L.color[0], L.color[1], L.color[2]} * (f_num_lights * light_pdf / light_num_pdf);
		ok = !isBlack(pcol);
	}
	// the path's place in the alive list: position i, i.e. segment i / seg_cap (the bounce workgroup that
	// traces it) — no counter (a global per-wave atomic here serialised 156 K appends on one address: 1.8 ms
	// for 10 M photons), and a wave of the bounce kernel reads consecutive path records (r04 dealt ids
	// round-robin over the segments: every lane's 16-B loads touched its own 128-B line, 7.9x the model's
	// bytes); a photon that carries no energy leaves a hole
	if(i < A.n_local) A.P.alive[0][i] = ok ? i : kDeadPhoton;
	if(ok)
	{
		A.P.ray_o[i] = f4(o, S.ray_min_dist);
		A.P.ray_d[i] = f4(d, -1.f);
		A.P.pcol[i] = f4(pcol, __uint_as_float(2u));   // caustic = false, direct = true
	}
}

// Final gathering: :186 keeps a deposit as a radiance point when the global FastRandom draws
// < 0.125 (shared by the photon threads, so schedule-dependent); a hash of the deposit slot (photon
// id, bounce) keeps one in eight here — the oracle uses the same hash
__device__ __forceinline__ bool fgRadSelect(uint32_t slot) { return (fnv32(slot ^ 0x6a09e667u) & 7u) == 0u; }

// material.cc:156-174 Material::getReflectivity: the mean of 16 weighted material samples
template<bool EXT>
__device__ C3 getReflectivity(const DevScene &S, const DevMaterial &m, const Surf &sp, uint32_t flags)
{
	if(!(flags & (B_TRANSMIT | B_REFLECT) & sp.flags)) return c3(0.f);
	C3 total = c3(0.f);
	for(int i = 0; i < 16; ++i)
	{
		const float s_1 = 0.03125f + 0.0625f * static_cast<float>(i);
		const float s_2 = riVdC((uint32_t)i);
		BsdfSample s;
		s.s_1 = ldsDim(S, 2, (uint32_t)i);
		s.s_2 = ldsDim(S, 3, (uint32_t)i);
		s.flags = flags;
		s.pdf = 0.f;
		s.sampled = B_NONE;
		const V3 wo = cosHemisphere(sp.n, sp.nu, sp.nv, s_1, s_2);
		V3 wi = v3(0.f, 0.f, 0.f);
		float w = 0.f;
		const C3 col = matSample<EXT>(m, sp, wo, wi, s, w);
		total = total + col * w;
	}
	return total * 0.0625f;
}

// :162-219 — one bounce of every live photon path: intersect, deposit, scatter (material.cc:137-153)
template<bool LDS_SCENE, bool WIDE, bool EXT, bool SPILL = true>
__global__ void __launch_bounds__(kTraceBlock) k_photon_bounce(PhotonArgs A)
{
	const DevScene &S = A.S;
	extern __shared__ float4 smem[];
	TraceCtx C;
	C.wave_base = waveBase();
	C.stack = reinterpret_cast<int *>(smem);
	C.lds_depth = A.stack_depth;
	C.spill = A.spill;
	C.spill_stride = gridDim.x * blockDim.x;
	if(LDS_SCENE)
	{
		float4 *lds_nodes = smem + (A.stack_depth * kTraceBlock) / 4;
		float4 *lds_tris = lds_nodes + S.node_f4 * S.n_nodes;
		for(int k = threadIdx.x; k < S.node_f4 * S.n_nodes; k += blockDim.x) lds_nodes[k] = S.nodes[k];
		for(int k = threadIdx.x; k < 3 * S.n_tris; k += blockDim.x) lds_tris[k] = S.tris[k];
		__syncthreads();
		C.nodes = lds_nodes;
		C.tris = lds_tris;
	}
	else
	{
		C.nodes = S.nodes;
		C.tris = S.tris;
	}
	// workgroup `seg` traces segment `seg` of the alive list and appends the paths that continue to
	// segment `seg` of the next list through an LDS counter (an entry yields at most one next entry, so
	// a segment never outgrows its share; no global atomics — the main wavefront's queue scheme)
	__shared__ uint32_t s_next;
	if(threadIdx.x == 0) s_next = 0;
	__syncthreads();
	const uint32_t seg = blockIdx.x, G = A.P.n_segs, cap = A.P.seg_cap;
	const uint32_t n = A.bounce == 0 ? (A.n_local > seg * cap ? min(cap, A.n_local - seg * cap) : 0u) : A.P.n_alive[(uint32_t)A.bounce * G + seg];
	const uint32_t *alive_cur = A.P.alive[A.cur] + (size_t)seg * cap;
	const int nxt = A.cur ^ 1;
	uint32_t *alive_nxt = A.P.alive[nxt] + (size_t)seg * cap;
	const uint32_t slots = (uint32_t)A.max_bounces + 1u;
	const size_t row = (size_t)A.bounce * A.P.n_local;   // this bounce's deposit slots: row + local id
	uint32_t visits = 0, tests = 0;
	for(uint32_t base = 0; base < n; base += blockDim.x)
	{
		const uint32_t j = base + threadIdx.x;
		bool cont = false;
		uint32_t i = 0, h = 0;   // local id, photon id
		V3 new_o = v3(0.f, 0.f, 0.f), new_d = new_o;
		C3 new_col = c3(0.f);
		uint32_t new_flags = 0;
		if(j < n) i = alive_cur[j];
		if(j < n && i != kDeadPhoton)
		{
			h = A.h0 + i;
			const float4 ro = A.P.ray_o[i], rd = A.P.ray_d[i], pc = A.P.pcol[i];
			float t;
			int prim;
			if(traverse<false, WIDE, SPILL>(C, xyz(ro), xyz(rd), ro.w, __builtin_huge_valf(), t, prim, visits, tests))
			{
				Surf sp = makeSurf(S, xyz(ro), xyz(rd), t, prim);
				if(EXT && S.has_attr)
				{
					// the photon hit's textured colour / shading normal (initBsdf in diffuseWorker)
					const SurfAttr sa = surfAttr(S.prim_attr, S.prim_ng, prim, xyz(ro), xyz(rd), sp.p);
					const DevMaterial &m = S.mats[sp.mat];
					C3 dcol = C3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
					float drefl = 1.f, sigma = 0.f;
					if(m.n_nodes > 0) evalNodes(m, S.shader_nodes, S.textures, S.texels, sa, dcol, drefl, sigma);
					applyAttr(sp, f4(sa.n, drefl), f4(dcol, sigma));
				}
				const V3 wi = -xyz(rd);
				const C3 lcol = rgb(pc);
				uint32_t flags = __float_as_uint(pc.w);
				const bool caustic = flags & 1u, direct = flags & 2u;
				// diffuse map: non-caustic photons on diffuse surfaces (:173-180); caustic map: caustic
				// photons on diffuse / glossy surfaces (integrator_montecarlo.cc:480-488)
				const bool store = A.L.caustic ? ((sp.flags & (B_DIFFUSE | B_GLOSSY)) && caustic) : ((sp.flags & B_DIFFUSE) && !caustic);
				if(store)
				{
					const size_t slot = row + i;
					A.P.dep_a[slot] = f4(sp.p, lcol.r);
					A.P.dep_b[slot] = f4(wi, lcol.g);
					A.P.dep_c[slot] = lcol.b;
					A.P.dep_flag[slot] = 1;
					// :184-193 radiance point (final gathering): normal faced to the photon, reflectivities
					if(A.P.rad_flag && !A.L.caustic && fgRadSelect(h * slots + (uint32_t)A.bounce))
					{
						if constexpr(EXT)
						{
							const DevMaterial &m = S.mats[sp.mat];
							const C3 refl = getReflectivity<EXT>(S, m, sp, B_DIFFUSE | B_GLOSSY | B_REFLECT);
							const C3 transm = getReflectivity<EXT>(S, m, sp, B_DIFFUSE | B_GLOSSY | B_TRANSMIT);
							A.P.rad_a[slot] = f4(sp.p, refl.r);
							A.P.rad_b[slot] = f4(faceForward(sp.ng, sp.n, wi), refl.g);
							A.P.rad_c[slot] = make_float4(refl.b, transm.r, transm.g, transm.b);
						}
						else
						{
							// the reflectivities (32 material samples, for one deposit in eight: the other lanes of
							// the wave waited) are computed by k_rad_refl for the points the thinning keeps, one
							// lane each; the point carries its primitive (flat shading: surfFromPrim rebuilds sp)
							A.P.rad_a[slot] = f4(sp.p, __int_as_float(prim));
							A.P.rad_b[slot] = f4(faceForward(sp.ng, sp.n, wi), 0.f);
						}
						A.P.rad_flag[slot] = 1;
					}
				}
				if(A.bounce < A.max_bounces)
				{
					const int d_5 = 3 * A.bounce + 5;
					BsdfSample s;
					s.s_1 = ldsDim(S, d_5, h);
					s.s_2 = ldsDim(S, d_5 + 1, h);
					const float s_3 = ldsDim(S, d_5 + 2, h);
					// PSample flags: All (diffuse map), AllSpecular | Glossy | Filter | Dispersive (caustic
					// map, integrator_montecarlo.cc:497)
					s.flags = A.L.caustic ? (B_SPECULAR | B_REFLECT | B_TRANSMIT | B_GLOSSY | B_FILTER | B_DISPERSIVE) : B_ALL;
					s.pdf = 0.f;
					s.sampled = B_NONE;
					float w = 0.f;
					V3 wo = v3(0.f, 0.f, 0.f);
					const C3 scol = matSample<EXT>(S.mats[sp.mat], sp, wi, wo, s, w);
					if(s.pdf > 1.0e-6f)
					{
						const C3 cnew = lcol * c3(1.f) * scol * w;
						const float new_max = fmaxf(cnew.r, fmaxf(cnew.g, cnew.b));
						const float old_max = fmaxf(lcol.r, fmaxf(lcol.g, lcol.b));
						const float prob = fminf(1.f, new_max / old_max);
						if(s_3 <= prob && prob > 1e-4f)
						{
							new_col = cnew / prob;
							const uint32_t sf = s.sampled;
							const bool nc = ((sf & (B_GLOSSY | B_SPECULAR | B_DISPERSIVE)) && direct) ||
							                ((sf & (B_GLOSSY | B_SPECULAR | B_FILTER | B_DISPERSIVE)) && caustic);
							const bool nd = (sf & B_FILTER) && direct;
							new_flags = (nc ? 1u : 0u) | (nd ? 2u : 0u);
							new_o = sp.p;
							new_d = wo;
							// caustic-only shooting stops once the path is neither (:520-521)
							cont = !A.L.caustic || nc || nd;
						}
					}
				}
			}
		}
		const uint32_t k = waveAppend(cont, &s_next);
		if(cont)
		{
			alive_nxt[k] = i;
			A.P.ray_o[i] = f4(new_o, S.ray_min_dist);
			A.P.ray_d[i] = f4(new_d, -1.f);
			A.P.pcol[i] = f4(new_col, __uint_as_float(new_flags));
		}
	}
	__syncthreads();
	if(threadIdx.x == 0) A.P.n_alive[(uint32_t)(A.bounce + 1) * G + seg] = s_next;
}

// Stable compaction of the bounce-major deposit slots into photon-id order (bounces in order per
// photon): per block of 1024 local ids the stored deposits are counted, the counts scanned in one
// workgroup, then each thread writes its photon's deposits at its place in the block.
__global__ void __launch_bounds__(256) k_photon_count(const uint8_t *flag, uint32_t n_local, uint32_t rows, uint32_t *counts)
{
	const uint32_t b0 = blockIdx.x * 1024u;
	uint32_t c = 0;
	for(uint32_t k = threadIdx.x; k < 1024u; k += 256u)
		if(b0 + k < n_local)
			for(uint32_t b = 0; b < rows; ++b) c += flag[(size_t)b * n_local + b0 + k];
	for(int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off);
	__shared__ uint32_t red[4];
	if(laneId() == 0) red[threadIdx.x >> 6] = c;
	__syncthreads();
	if(threadIdx.x == 0) counts[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(1024) k_photon_scan(uint32_t *counts, uint32_t n, uint32_t *total)
{
	// exclusive scan of n counts by one workgroup: each thread scans a contiguous run
	__shared__ uint32_t part[1024];
	const uint32_t per = (n + 1023u) / 1024u;
	const uint32_t a = threadIdx.x * per, b = min(n, a + per);
	uint32_t sum = 0;
	for(uint32_t k = a; k < b; ++k) sum += counts[k];
	part[threadIdx.x] = sum;
	__syncthreads();
	if(threadIdx.x == 0)
	{
		uint32_t run = 0;
		for(int k = 0; k < 1024; ++k) { const uint32_t v = part[k]; part[k] = run; run += v; }
		*total = run;
	}
	__syncthreads();
	uint32_t run = part[threadIdx.x];
	for(uint32_t k = a; k < b; ++k) { const uint32_t v = counts[k]; counts[k] = run; run += v; }
}

// The first output position of local id (blockIdx.x * 1024 + threadIdx.x)'s deposits: the block's
// offset + the deposits of the block's earlier ids (flags of `rows` bounce rows; c = this id's count).
__device__ __forceinline__ uint32_t depositBase(const uint8_t *flag, uint32_t n_local, uint32_t rows, const uint32_t *offsets, uint32_t &c)
{
	__shared__ uint32_t wsum[16];
	const uint32_t i = blockIdx.x * 1024u + threadIdx.x;
	c = 0;
	if(i < n_local)
		for(uint32_t b = 0; b < rows; ++b) c += flag[(size_t)b * n_local + i];
	// inclusive scan over the wave, then the earlier waves' totals
	uint32_t s = c;
	for(int off = 1; off < 64; off <<= 1)
	{
		const uint32_t v = __shfl_up(s, off);
		if(laneId() >= off) s += v;
	}
	const int wid = threadIdx.x >> 6;
	if(laneId() == 63) wsum[wid] = s;
	__syncthreads();
	uint32_t base = offsets[blockIdx.x];
	for(int w = 0; w < wid; ++w) base += wsum[w];
	return base + s - c;
}

__global__ void __launch_bounds__(1024) k_photon_scatter(PhotonState P, const uint32_t *offsets, float4 *pos, float4 *dir, float *colb)
{
	uint32_t c;
	uint32_t o = depositBase(P.dep_flag, P.n_local, P.n_slot_rows, offsets, c);
	const uint32_t i = blockIdx.x * 1024u + threadIdx.x;
	for(uint32_t b = 0; c > 0 && b < P.n_slot_rows; ++b)
	{
		const size_t k = (size_t)b * P.n_local + i;
		if(!P.dep_flag[k]) continue;
		pos[o] = P.dep_a[k];
		dir[o] = P.dep_b[k];
		colb[o] = P.dep_c[k];
		++o;
		--c;
	}
}

// ---------------------------------------------------------------------------------------------
// k_gather: the photon density estimate of PhotonIntegrator::integrate (:953-976) for every
// diffuse camera hit, after its direct light has been connected: k-NN lookup in the point
// kd-tree (pkdtree.h:225-292) with PhotonGather's heap (photon.cc:31-52, photonheap.h), then the
// contributions are added to the sample's colour in heap-array order and the sample is written.
// ---------------------------------------------------------------------------------------------
constexpr int kGatherBlock = 64;
#ifndef YAF_GATHER_PER_SEG
#define YAF_GATHER_PER_SEG 4
#endif
constexpr int kGatherPerSeg = YAF_GATHER_PER_SEG;   // workgroups per queue segment (fills the chip: 4 x 1024 x 64 lanes)
#ifndef YAF_GATHER_STACK_LDS
#define YAF_GATHER_STACK_LDS 0     // 1: lookup stack in LDS (8 B x depth per lane) instead of HBM
#endif
#ifndef YAF_GATHER_XCD
#define YAF_GATHER_XCD 1           // 1: each XCD gathers a contiguous eighth of the segments (L2 locality)
#endif
//
// The walk is latency-bound (a chain of dependent loads, 64 lanes on 64 neighbouring pixels), so
// the levers are occupancy, coherence and L2 locality (C5 measurements):
//   * the only per-lane LDS is the k-entry heap; one 8-byte slot = index + distance, so a sift step
//     moves a slot with one 64-bit access.  The lookup stack is a per-lane HBM column (pushes are
//     fire-and-forget stores, pops hit L2): an LDS stack costs occupancy and measured slower;
//   * a far child whose plane distance already exceeds the current radius is never pushed (the
//     reference pushes it and discards it when popped; the radius never grows, so the visit order
//     and the heap are unchanged) — 53 -> 42 ms;
//   * workgroups are renumbered so that each XCD walks the photons of a contiguous eighth of the
//     image (56 -> 53 ms);
//   * tried and dropped: one node per loop trip (if-if, 67 ms), lanes refilling independently with
//     the estimate in a second kernel (lanes drift apart and stop sharing cache lines, 59-70 ms).
// The accepted-photon log of the two-pass diffuse gather (k_gather_walk -> k_gather<REPLAY>), for
// the queue positions [j0, j0 + seg_cap) of every segment (one batch): batch query q = seg * seg_cap
// + (position - j0); its entries at e[q * cap ..) (written in 16-byte pairs, so a request fills its
// own cache lines); n[q] = entries (> cap: overflowed, not replayable).
struct GatherLog
{
	uint2 *e;          // (photon index, squared distance bits)
	uint32_t *n;
	uint32_t cap;      // entries per query
	uint32_t seg_cap;  // queue positions per segment in this batch (a multiple of 64)
	uint32_t j0;       // first queue position of the batch
	uint32_t *spill = nullptr;   // the walk's stack levels beyond YAF_WALK_LDS_LEVELS ([level][walk thread])
};

struct GatherArgs
{
	DevScene S;
	DevNeeQueue G;           // gather requests: (p, prim), (wo, sample id), (colour, alpha) bits, (extra, mode)
	DevCounters cnt_next;    // n_gather = requests per segment
	float4 *samples;
	const DevJob *jobs;
	int n_jobs;
	uint64_t chunk_base;
	GatherLog log;           // REPLAY: the walk's log of this batch
};

__host__ __device__ inline size_t gatherTableBytes(const DevScene &S, bool small)
{
	return small ? (size_t)S.n_mats * sizeof(DevMaterial) + (size_t)S.n_tris * 16 : 0;
}

// heap slots: the larger k of the maps in use
__host__ __device__ inline int gatherHeapSlots(const DevScene &S)
{
	const int kd = S.n_photons > 0 ? S.pm_search : 1;
	const int kc = S.caus_map ? S.c_search : 1;
	return kd > kc ? kd : kc;
}

__host__ __device__ inline size_t gatherLdsBytes(const DevScene &S)
{
	return (size_t)kGatherBlock * 8u * (size_t)gatherHeapSlots(S) +
	       (YAF_GATHER_STACK_LDS ? (size_t)kGatherBlock * 8u * (size_t)S.pm_stack : 0u);
}

// workgroups are dealt to the 8 XCDs round-robin: renumber them so that XCD x gets the contiguous
// run of segments [x, x + 1) * n_seg / 8 (neighbouring pixels -> one L2)
__device__ __forceinline__ void gatherSegPart(uint32_t n_seg, uint32_t &seg, uint32_t &part, uint32_t &parts)
{
	const uint32_t nb = gridDim.x;
	parts = nb / n_seg;
	if(YAF_GATHER_XCD && (nb & 7u) == 0)
	{
		const uint32_t v = (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
		seg = v / parts;
		part = v % parts;
	}
	else
	{
		seg = blockIdx.x % n_seg;
		part = blockIdx.x / n_seg;
	}
}

// PhotonMap::gather (photon.cc:55-64): k-NN lookup in a point kd-tree (pkdtree.h:225-292,
// NON_REC_LOOKUP) with PhotonGather's heap (photon.cc:31-52); returns the photons found, leaves
// the heap in `heap` and the final squared radius in max_d2
__device__ __forceinline__ int pkLookup(const uint4 *nodes, V3 p, int k, float &max_d2, const HeapRefPacked &heap, uint2 *stk, uint32_t gstride,
                                        uint32_t &visits)
{
	// nodes: .w = flags (bits 0-1 axis, 3 = leaf; interior: right child << 2, leaf: photon << 2),
	// interior .x = split position; leaf .xyz = the photon's position
	int found = 0;
	uint32_t curr = 0;
	int sp_top = 0;   // entries above the reference's "nowhere" sentinel
	for(;;)
	{
		uint4 nd = nodes[curr];
		++visits;
		while((nd.w & 3u) != 3u)
		{
			const int axis = (int)(nd.w & 3u);
			const float split_val = __uint_as_float(nd.x);
			const float pa = axis == 0 ? p.x : (axis == 1 ? p.y : p.z);
			uint32_t far_child;
			if(pa <= split_val) { far_child = nd.w >> 2; curr = curr + 1; }
			else { far_child = curr + 1; curr = nd.w >> 2; }
			// the reference pushes every far child and discards it at pop time when (p - split)^2 >
			// max_d2; max_d2 never grows, so one that already fails now is never visited
			float d2 = pa - split_val;
			d2 *= d2;
			if(d2 <= max_d2)
			{
				stk[(size_t)sp_top * gstride] = make_uint2(far_child, __float_as_uint(d2));
				++sp_top;
			}
			nd = nodes[curr];
			++visits;
		}
		const uint32_t ph = nd.w >> 2;
		const V3 v = v3(__uint_as_float(nd.x), __uint_as_float(nd.y), __uint_as_float(nd.z)) - p;
		const float dist_2 = v.x * v.x + v.y * v.y + v.z * v.z;
		if(dist_2 < max_d2)
		{
			// photon.cc:31-52
			if(found < k)
			{
				heap.i(found) = ph;
				heap.d(found) = dist_2;
				++found;
				if(found == k)
				{
					heapMake(heap, k);
					max_d2 = heap.d(0);
				}
			}
			else
			{
				heapReplaceTop(heap, k, ph, dist_2);
				max_d2 = heap.d(0);
			}
		}
		if(sp_top == 0) break;
		uint2 top = stk[(size_t)(sp_top - 1) * gstride];
		bool done = false;
		while(__uint_as_float(top.y) > max_d2)
		{
			--sp_top;
			if(sp_top == 0) { done = true; break; }
			top = stk[(size_t)(sp_top - 1) * gstride];
		}
		if(done) break;
		curr = top.x;
		--sp_top;
	}
	return found;
}

// ---- two-pass diffuse gather ----
// The walk of pkLookup depends on the heap only through max_d2, the largest of the k smallest
// distances accepted so far — a function of the accepted multiset, not of the heap's layout.
// Pass 1 (k_gather_walk) keeps those k distances in registers (unrolled over kWalkK; no LDS, so
// several times the resident waves of k_gather for the latency-bound walk) and logs every accepted
// photon (index, distance) in visit order.  Pass 2 (k_gather<REPLAY>) feeds the log through
// PhotonGather's heap in LDS — the reference's element moves exactly — and computes the estimate.
#ifndef YAF_WALK_K
#define YAF_WALK_K 64
#endif
constexpr int kWalkK = YAF_WALK_K;
// The exact walk keeps YAF_WALK_LDS_LEVELS far-child stack levels in LDS and the deeper ones in an HBM
// column per walk thread (0: every level in LDS): with the 16-bit key slots (68 VGPRs) the 26-level LDS
// column capped residency at 6 waves per SIMD; 20 levels: C5 walk 14.0 -> 13.3-13.7 ms (16 levels: 14.8,
// the deeper pushes go to HBM; 22: 13.4-14.1)
#ifndef YAF_WALK_LDS_LEVELS
#define YAF_WALK_LDS_LEVELS 20
#endif
constexpr int kWalkLdsLevels = YAF_WALK_LDS_LEVELS;   // register slots of the walk (>= the search's k)
#ifndef YAF_WALK_PER_SEG
#define YAF_WALK_PER_SEG 16
#endif
constexpr int kWalkPerSeg = YAF_WALK_PER_SEG;   // walk workgroups per queue segment

// pkLookup's walk with the k smallest distances in registers: kd[] ascending, its first kWalkK - k
// slots pinned at -1 (below every distance) and the rest +inf, so after any number of insertions
// kd[kWalkK - 1] is the largest of the k smallest accepted distances (+inf while fewer than k were
// accepted) and the reference's max_d2 is min(radius, kd[kWalkK - 1]).  One insertion is one v_med3
// per slot with no "heap full" branch, so the compiler keeps one copy of the array (the two-case
// form held two: 153 VGPRs, 3 waves / SIMD).  The stack is an LDS column of
// far-child indices (4 B; stk[level * kGatherBlock]): a popped interior node carries its parent's
// plane (pkd.hip), from which the plane distance the reference stacked is recomputed; a popped leaf
// is tested directly (its photon lies beyond that plane, so the reference's pop-time rejection and
// the distance test agree).  The accepted photons go to this request's log lg[0 ..) in pairs
// (16-byte stores; the first `cap`); returns how many were accepted.
#ifndef YAF_WALK_PACK
#define YAF_WALK_PACK 1
#endif
#if YAF_WALK_PACK
// The walk's slots as 16-bit keys, two per VGPR: the bfloat16 bits of each distance rounded UP (for
// non-negative floats the bits are monotone, so the k-th smallest key bounds the k-th smallest
// distance from above).  The walk then prunes and logs with a bound >= the reference's max_d2 — a
// superset log in the same visit order, which the replay filters with the exact test (as the
// bounded walk's, pkWalkBound) — in 32 VGPRs instead of 64.  Insertion of key x into the ascending
// slots: slot i <- max(slot i-1, min(slot i, x)) for every pair at once (alignbit + packed min / max).
typedef unsigned short walk_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t walkKey(float d2) { return (__float_as_uint(d2) + 0xffffu) >> 16; }
__device__ __forceinline__ uint32_t pkMaxU16(uint32_t a, uint32_t b)
{
	return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(walk_u16x2, a), __builtin_bit_cast(walk_u16x2, b)));
}
__device__ __forceinline__ uint32_t pkMinU16(uint32_t a, uint32_t b)
{
	return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(walk_u16x2, a), __builtin_bit_cast(walk_u16x2, b)));
}
#endif
__device__ __forceinline__ uint32_t pkWalk(const uint4 *nodes, V3 p, int k, float max_d2, uint2 *lg, uint32_t cap, uint32_t *stk,
                                           uint32_t &visits, int lds_lv = 1 << 30, uint32_t *spill = nullptr, uint32_t spill_stride = 0)
{
	auto spush = [&](int lv, uint32_t v) {
		if(kWalkLdsLevels == 0 || lv < lds_lv) stk[lv * kGatherBlock] = v;
		else spill[(size_t)(lv - lds_lv) * spill_stride] = v;
	};
	auto spop = [&](int lv) -> uint32_t {
		return (kWalkLdsLevels == 0 || lv < lds_lv) ? stk[lv * kGatherBlock] : spill[(size_t)(lv - lds_lv) * spill_stride];
	};
	const float radius2 = max_d2;
	// (an opaque bound: otherwise the 64 initial values are hoisted out of the request loop and
	// stay live across every walk — 64 more VGPRs)
	int pinned = kWalkK - k;
	asm volatile("" : "+s"(pinned));
#if YAF_WALK_PACK
	constexpr uint32_t kEmpty = 0x7f80u;   // +inf
	uint32_t kp[kWalkK / 2];
#pragma unroll
	for(int i = 0; i < kWalkK / 2; ++i)
		kp[i] = ((2 * i < pinned) ? 0u : kEmpty) | (((2 * i + 1 < pinned) ? 0u : kEmpty) << 16);
#else
	float kd[kWalkK];
#pragma unroll
	for(int i = 0; i < kWalkK; ++i) kd[i] = (i < pinned) ? -1.f : __builtin_huge_valf();
#endif
	uint32_t n_acc = 0;
	uint2 pend = make_uint2(0u, 0u);
	uint32_t curr = 0;
	int sp_top = 0;
	uint4 nd = nodes[0];
	++visits;
	for(;;)
	{
		while((nd.w & 3u) != 3u)
		{
			const int axis = (int)(nd.w & 3u);
			const float split_val = __uint_as_float(nd.x);
			const float pa = axis == 0 ? p.x : (axis == 1 ? p.y : p.z);
			uint32_t far_child;
			if(pa <= split_val) { far_child = nd.w >> 2; curr = curr + 1; }
			else { far_child = curr + 1; curr = nd.w >> 2; }
			float d2 = pa - split_val;
			d2 *= d2;
			if(d2 <= max_d2)
			{
				spush(sp_top, far_child);
				++sp_top;
			}
			nd = nodes[curr];
			++visits;
		}
		const uint32_t ph = nd.w >> 2;
		const V3 v = v3(__uint_as_float(nd.x), __uint_as_float(nd.y), __uint_as_float(nd.z)) - p;
		const float dist_2 = v.x * v.x + v.y * v.y + v.z * v.z;
		if(dist_2 < max_d2)
		{
			const uint2 e = make_uint2(ph, __float_as_uint(dist_2));
			if(n_acc & 1u)
			{
				if(n_acc < cap) *reinterpret_cast<uint4 *>(lg + (n_acc - 1u)) = make_uint4(pend.x, pend.y, e.x, e.y);
			}
			else pend = e;
			++n_acc;
			// insert (the largest slot drops out): below k accepted this fills a +inf slot (the heap
			// grows); from then on it removes the top and adds dist_2 (pop_heap + push_heap)
#if YAF_WALK_PACK
			const uint32_t x = walkKey(dist_2), xx = x | (x << 16);
#pragma unroll
			for(int i = kWalkK / 2 - 1; i > 0; --i)
				kp[i] = pkMaxU16(__builtin_amdgcn_alignbit(kp[i], kp[i - 1], 16u), pkMinU16(kp[i], xx));
			kp[0] = pkMaxU16(kp[0] << 16, pkMinU16(kp[0], xx));
			max_d2 = fminf(radius2, __uint_as_float(kp[kWalkK / 2 - 1] & 0xffff0000u));
#else
#pragma unroll
			for(int i = kWalkK - 1; i > 0; --i) kd[i] = __builtin_amdgcn_fmed3f(kd[i - 1], kd[i], dist_2);
			kd[0] = fminf(kd[0], dist_2);
			max_d2 = fminf(radius2, kd[kWalkK - 1]);
#endif
		}
		// pop the next far child the current radius still reaches
		bool more = false;
		while(sp_top > 0)
		{
			--sp_top;
			curr = spop(sp_top);
			nd = nodes[curr];
			++visits;
			if((nd.w & 3u) != 3u)
			{
				const uint32_t pax = nd.z;
				const float pa = pax == 0u ? p.x : (pax == 1u ? p.y : p.z);
				float d2 = pa - __uint_as_float(nd.y);
				d2 *= d2;
				if(d2 > max_d2) continue;
			}
			more = true;
			break;
		}
		if(!more) break;
	}
	if((n_acc & 1u) && n_acc <= cap) lg[n_acc - 1u] = pend;
	return n_acc;
}

// pkLookup's walk with a conservative radius (the default walk).  The walk may prune and log with any
// bound T(t) >= the reference's max_d2(t): every photon the reference accepts is then logged in visit
// order (pruning never drops one: a photon beyond a split plane is at least the plane distance away,
// in float as in reals, since rounding is monotonic), and the replay (replayLog) re-applies the exact
// test d < max_d2, which rejects the extra entries — photons of subtrees the reference pruned, or
// farther than its radius at the time.  The k-th smallest logged distance equals the k-th smallest
// accepted one (an extra entry is never below the radius of its time, which only shrinks), so a
// histogram of the logged distances bounds max_d2 from above: bin j holds distances with
// (bits(radius2) - bits(d)) >> kWalkBinShift = j (the last bin open below; 2 bins per octave), and
// T = the upper edge of the deepest bin B with >= k logged entries at or below it.  One insertion is
// a byte increment in the lane's own LDS column and, rarely, a step of B — no k-slot array
// (k_gather_walk's exact form keeps k sorted distances in 64 VGPRs and pays 64 v_med3 per insertion),
// so any k is served.  Byte counters saturate at 255: counts are then lower bounds, T stays
// conservative.  tools/walk_sim.cc models the visits and log entries per request of both bounds.
#ifndef YAF_WALK_BINS
#define YAF_WALK_BINS 32
#endif
#ifndef YAF_WALK_BIN_SHIFT
#define YAF_WALK_BIN_SHIFT 22
#endif
constexpr int kWalkBins = YAF_WALK_BINS;   // multiple of 4 (four byte counters per LDS word)
constexpr int kWalkBinShift = YAF_WALK_BIN_SHIFT;
static_assert(kWalkBins % 4 == 0, "byte counters in words");

__host__ __device__ inline int walkLdsLevels(int pm_stack)
{
	const int all = pm_stack > 1 ? pm_stack : 1;
	return (kWalkLdsLevels > 0 && kWalkLdsLevels < all) ? kWalkLdsLevels : all;
}
__host__ __device__ inline size_t walkLdsBytes(int pm_stack, bool hist)
{
	// (the bounded walk keeps its whole stack in LDS)
	return (size_t)(hist ? (pm_stack > 1 ? pm_stack : 1) : walkLdsLevels(pm_stack)) * kGatherBlock * 4u + (hist ? (size_t)kWalkBins * kGatherBlock : 0u);
}

__device__ __forceinline__ uint32_t pkWalkBound(const uint4 *nodes, V3 p, int k, float radius2, uint2 *lg, uint32_t cap, uint32_t *stk,
                                                uint32_t *hist, uint32_t &visits)
{
	const uint32_t rb = __float_as_uint(radius2);
	// deepest usable bin: its edge bits(radius2) - (B << shift) + 1 stays a positive float
	const int top_bin = min(kWalkBins - 1, (int)(rb >> kWalkBinShift) - 1);
#pragma unroll
	for(int w = 0; w < kWalkBins / 4; ++w) hist[w * kGatherBlock] = 0u;
	float T = radius2;
	int B = 0;              // T = edge(B): radius2 for B = 0
	uint32_t below = 0;     // counted entries in bins > B
	uint32_t n_acc = 0;
	uint2 pend = make_uint2(0u, 0u);
	uint32_t curr = 0;
	int sp_top = 0;
	uint4 nd = nodes[0];
	++visits;
	for(;;)
	{
		while((nd.w & 3u) != 3u)
		{
			const int axis = (int)(nd.w & 3u);
			const float split_val = __uint_as_float(nd.x);
			const float pa = axis == 0 ? p.x : (axis == 1 ? p.y : p.z);
			uint32_t far_child;
			if(pa <= split_val) { far_child = nd.w >> 2; curr = curr + 1; }
			else { far_child = curr + 1; curr = nd.w >> 2; }
			float d2 = pa - split_val;
			d2 *= d2;
			if(d2 <= T)
			{
				stk[sp_top * kGatherBlock] = far_child;
				++sp_top;
			}
			nd = nodes[curr];
			++visits;
		}
		const uint32_t ph = nd.w >> 2;
		const V3 v = v3(__uint_as_float(nd.x), __uint_as_float(nd.y), __uint_as_float(nd.z)) - p;
		const float dist_2 = v.x * v.x + v.y * v.y + v.z * v.z;
		if(dist_2 < T)
		{
			const uint2 e = make_uint2(ph, __float_as_uint(dist_2));
			if(n_acc & 1u)
			{
				if(n_acc < cap) *reinterpret_cast<uint4 *>(lg + (n_acc - 1u)) = make_uint4(pend.x, pend.y, e.x, e.y);
			}
			else pend = e;
			++n_acc;
			if(top_bin > 0)
			{
				const int j = (int)min((rb - __float_as_uint(dist_2)) >> kWalkBinShift, (uint32_t)top_bin);
				uint32_t *w = hist + (j >> 2) * kGatherBlock;
				const uint32_t sh = (uint32_t)(j & 3) * 8u, word = *w;
				if(((word >> sh) & 255u) != 255u)
				{
					*w = word + (1u << sh);
					if(j > B) ++below;
				}
				if(below >= (uint32_t)k)
				{
					do
					{
						++B;
						below -= (hist[(B >> 2) * kGatherBlock] >> ((uint32_t)(B & 3) * 8u)) & 255u;
					} while(B < top_bin && below >= (uint32_t)k);
					T = __uint_as_float(rb - ((uint32_t)B << kWalkBinShift) + 1u);
				}
			}
		}
		bool more = false;
		while(sp_top > 0)
		{
			--sp_top;
			curr = stk[sp_top * kGatherBlock];
			nd = nodes[curr];
			++visits;
			if((nd.w & 3u) != 3u)
			{
				const uint32_t pax = nd.z;
				const float pa = pax == 0u ? p.x : (pax == 1u ? p.y : p.z);
				float d2 = pa - __uint_as_float(nd.y);
				d2 *= d2;
				if(d2 > T) continue;
			}
			more = true;
			break;
		}
		if(!more) break;
	}
	if((n_acc & 1u) && n_acc <= cap) lg[n_acc - 1u] = pend;
	return n_acc;
}

__device__ __forceinline__ uint2 *gatherLogAt(const GatherLog &L, uint32_t q)
{
	return L.e + (size_t)q * L.cap;
}

// pass 1 over one batch of the gather queue (diffuse-map requests; the others log nothing)
#ifndef YAF_WALK_WAVES
#define YAF_WALK_WAVES 6
#endif
template<bool BOUND>
__global__ void __launch_bounds__(kGatherBlock) __attribute__((amdgpu_waves_per_eu(YAF_WALK_WAVES))) k_gather_walk(GatherArgs A)
{
	extern __shared__ uint32_t walk_stack[];
	const DevScene &S = A.S;
	uint32_t *stk = walk_stack + threadIdx.x;
	uint32_t *hist = walk_stack + (size_t)max(1, S.pm_stack) * kGatherBlock + threadIdx.x;
	uint32_t seg, part, parts;
	gatherSegPart(S.n_seg, seg, part, parts);
	const uint32_t j1 = min(A.cnt_next.n_gather[seg], A.log.j0 + A.log.seg_cap);
	const uint32_t a0 = seg * S.cap_a;
	uint32_t visits = 0, accepts = 0;
	for(uint32_t jj = A.log.j0 + part * kGatherBlock + threadIdx.x; jj < j1; jj += parts * kGatherBlock)
	{
		const uint32_t j = a0 + jj;
		const uint32_t q = seg * A.log.seg_cap + (jj - A.log.j0);
		uint32_t n_acc = 0;
		if(__float_as_uint(A.G.extra[j].w) & G_DIFFUSE)
		{
			if(BOUND) n_acc = pkWalkBound(S.pk_nodes, xyz(A.G.p_prim[j]), S.pm_search, S.pm_radius2, gatherLogAt(A.log, q), A.log.cap, stk, hist, visits);
			else n_acc = pkWalk(S.pk_nodes, xyz(A.G.p_prim[j]), S.pm_search, S.pm_radius2, gatherLogAt(A.log, q), A.log.cap, stk, visits,
			                    walkLdsLevels(S.pm_stack), A.log.spill + (blockIdx.x * blockDim.x + threadIdx.x), gridDim.x * blockDim.x);
		}
		A.log.n[q] = n_acc;
		accepts += n_acc;
	}
	for(int off = 32; off > 0; off >>= 1)
	{
		visits += __shfl_down(visits, off);
		accepts += __shfl_down(accepts, off);
	}
	if(threadIdx.x == 0 && S.stats)
	{
		atomicAdd(&S.stats[seg].gather_visits, (unsigned long long)visits);
		atomicAdd(&S.stats[seg].gather_accepts, (unsigned long long)accepts);
	}
}

__device__ int pkNearest(const uint4 *nodes, const float4 *dirs, V3 p, V3 n, float max_d2, uint32_t *visits = nullptr);

// PhotonGather (photon.cc:31-52) over one request's logged photons, in the walk's visit order, with
// the reference's acceptance test d < max_d2 (pkdtree.h:270; the bounded walk logs a superset).
// POS: the heap keeps the entry's log position (HeapRefSplit), else the photon index.
template<bool POS, class H>
__device__ __forceinline__ void replayLog(const H &heap, const uint2 *lg, uint32_t n_acc, int k, int &found, float &max_d2)
{
	uint4 pair = make_uint4(0u, 0u, 0u, 0u);
	for(uint32_t a = 0; a < n_acc; ++a)
	{
		if(!(a & 1u)) pair = (a + 1u < n_acc) ? *reinterpret_cast<const uint4 *>(lg + a) : make_uint4(lg[a].x, lg[a].y, 0u, 0u);
		const uint2 e = (a & 1u) ? make_uint2(pair.z, pair.w) : make_uint2(pair.x, pair.y);
		const float d = __uint_as_float(e.y);
		const uint32_t v = POS ? a : e.x;
		if(found < k)
		{
			heap.i(found) = v;
			heap.d(found) = d;
			++found;
			if(found == k)
			{
				heapMake(heap, k);
				max_d2 = heap.d(0);
			}
		}
		else if(d < max_d2)
		{
			heapReplaceTop(heap, k, v, d);
			max_d2 = heap.d(0);
		}
	}
}

// HS (REPLAY without a caustic map): the split 6-byte heap (HeapRefSplit) — 1.5 -> 2 waves / SIMD at
// k = 50; a request whose log overflowed walks again with the heap in its own log (8 B slots in HBM).
template<bool SMALL, bool EXT, bool REPLAY = false, bool HS = false>
__global__ void __launch_bounds__(kGatherBlock) k_gather(GatherArgs A)
{
	extern __shared__ uint4 gather_smem[];
	DevScene S = A.S;
	if(SMALL)
	{
		uint4 *p = gather_smem;
		const int nm = S.n_mats * (int)(sizeof(DevMaterial) / 16);
		copy16(p, S.mats, nm);
		S.mats = reinterpret_cast<const DevMaterial *>(p);
		p += nm;
		copy16(p, S.prim_ng, S.n_tris);
		S.prim_ng = reinterpret_cast<const float4 *>(p);
		__syncthreads();
	}
	const bool ATTR = EXT && S.has_attr != 0;
	// per-lane heap, lane-interleaved after the staged tables
	uint32_t *lds_words = reinterpret_cast<uint32_t *>(gather_smem) + gatherTableBytes(A.S, SMALL) / 4;
	const int lane = threadIdx.x;
	HeapRefPacked heap;
	heap.e = lds_words + 2 * lane;
	heap.stride = kGatherBlock;
	HeapRefSplit hsplit;
	hsplit.dw = lds_words + lane;
	hsplit.iw = reinterpret_cast<uint16_t *>(lds_words + (size_t)gatherHeapSlots(S) * kGatherBlock) + lane;
	hsplit.stride = kGatherBlock;
	// lookup stack: this lane's column, [level][lane] (LDS after the heap, or the HBM stack buffer)
#if YAF_GATHER_STACK_LDS
	const uint32_t gstride = kGatherBlock;
	uint2 *stk = reinterpret_cast<uint2 *>(lds_words + (size_t)2 * gatherHeapSlots(S) * kGatherBlock) + threadIdx.x;
#else
	const uint32_t gstride = gridDim.x * kGatherBlock;
	uint2 *stk = S.pk_stack + blockIdx.x * kGatherBlock + threadIdx.x;
#endif
	uint32_t seg, part, parts;
	gatherSegPart(S.n_seg, seg, part, parts);
	const uint32_t n_all = A.cnt_next.n_gather[seg];
	// REPLAY: this batch's queue positions [j0, j0 + seg_cap) only
	const uint32_t jb = REPLAY ? A.log.j0 : 0u;
	const uint32_t n_req = REPLAY ? min(n_all, A.log.j0 + A.log.seg_cap) : n_all;
	const uint32_t a0 = seg * S.cap_a;
	uint32_t visits = 0, photons = 0, overflows = 0;
	for(uint32_t base_j = jb + part * kGatherBlock; base_j < n_req; base_j += parts * kGatherBlock)
	{
		if(base_j + threadIdx.x >= n_req) continue;
		const uint32_t j = a0 + base_j + threadIdx.x;
		const float4 pp = A.G.p_prim[j];
		const float4 ex = A.G.extra[j];
		const uint32_t mode = __float_as_uint(ex.w);
		const V3 p = xyz(pp);
		float max_d2 = S.pm_radius2;
		int found = 0;
		const uint2 *lg = nullptr;   // HS: the request's log (heap slots hold positions in it)
		bool from_log = false;       // HS: true after a replay, false when the heap is the log itself
		if(mode & G_DIFFUSE)
		{
			const uint32_t q = seg * A.log.seg_cap + (base_j + threadIdx.x - jb);
			const uint32_t n_acc = REPLAY ? A.log.n[q] : 0u;
			if(REPLAY) lg = gatherLogAt(A.log, q);
			if(REPLAY && n_acc <= A.log.cap)
			{
				if(HS)
				{
					replayLog<true>(hsplit, lg, n_acc, S.pm_search, found, max_d2);
					from_log = true;
				}
				else replayLog<false>(heap, lg, n_acc, S.pm_search, found, max_d2);
			}
			else
			{
				if(REPLAY) ++overflows;   // the log overflowed: walk again with the heap
				if(HS)
				{
					HeapRefPacked gh;
					gh.e = reinterpret_cast<uint32_t *>(const_cast<uint2 *>(lg));
					gh.stride = 1;
					found = pkLookup(S.pk_nodes, p, S.pm_search, max_d2, gh, stk, gstride, visits);
				}
				else found = pkLookup(S.pk_nodes, p, S.pm_search, max_d2, heap, stk, gstride, visits);
			}
		}
		photons += (uint32_t)found;
		const float4 wk = A.G.wo_k[j];
		const uint4 cb = A.G.pix_mode[j];
		Surf sp = surfFromPrim(S, p, __float_as_int(pp.w));
		if(ATTR) applyAttr(sp, A.G.attr[2 * (size_t)j], A.G.attr[2 * (size_t)j + 1]);
		const V3 wo = xyz(wk);
		const uint32_t sid = __float_as_uint(wk.w);
		C3 col = C3{__uint_as_float(cb.x), __uint_as_float(cb.y), __uint_as_float(cb.z)};
		const float alpha = __uint_as_float(cb.w);
		const DevMaterial &m = S.mats[sp.mat];
		// ---- diffuse-map density estimate (integrator_photon_mapping.cc:953-976), heap-array order ----
		if(found > 0)
		{
			const float scale = x87recipMul(kPi, (float)S.pm_paths * max_d2);
			for(int i = 0; i < found; ++i)
			{
				const uint32_t ph = HS ? lg[from_log ? (uint32_t)hsplit.i(i) : (uint32_t)i].x : heap.i(i);
				const float4 a = S.ph_pos[ph], b = S.ph_dir[ph];
				const C3 pc = C3{a.w, b.w, S.ph_colb[ph]};
				const C3 surf_col = matEval<EXT>(m, sp, wo, xyz(b), B_DIFFUSE);
				const C3 col_tmp = surf_col * scale * pc;
				col = col + col_tmp;
			}
		}
		// ---- show_map (integrator_photon_mapping.cc:876-881 final gathering: the radiance map within
		// lookup_rad_; :924-929: the diffuse map within ds_radius_): the nearest photon facing the shading normal
		if(mode & G_SHOWMAP)
		{
			const V3 n = faceForward(sp.ng, sp.n, wo);
			if(S.fg_on)
			{
				const int nn = S.n_rphotons > 0 ? pkNearest(S.rpk_nodes, S.rph_dir, p, n, S.fg_lookup_rad) : -1;
				if(nn >= 0) col = col + C3{S.rph_pos[nn].w, S.rph_dir[nn].w, S.rph_colb[nn]};
			}
			else
			{
				const int nn = S.n_photons > 0 ? pkNearest(S.pk_nodes, S.ph_dir, p, n, S.pm_radius2) : -1;
				if(nn >= 0) col = col + C3{S.ph_pos[nn].w, S.ph_dir[nn].w, S.ph_colb[nn]};
			}
		}
		// ---- causticPhotons / estimateCausticPhotons (integrator_montecarlo.cc:410-419, 627-648) ----
		if(!HS && (mode & G_CAUSTIC))   // HS is only launched without a caustic map
		{
			float r2 = S.c_radius2;
			const int nc = pkLookup(S.cpk_nodes, p, S.c_search, r2, heap, stk, gstride, visits);
			photons += (uint32_t)nc;
			const float ir2 = 1.f / r2;
			C3 sum = c3(0.f);
			if(nc > 0)
			{
				for(int i = 0; i < nc; ++i)
				{
					const uint32_t ph = heap.i(i);
					const float4 a = S.cph_pos[ph], b = S.cph_dir[ph];
					const C3 pc = C3{a.w, b.w, S.cph_colb[ph]};
					const C3 surf_col = matEval<EXT>(m, sp, wo, xyz(b), B_ALL);
					// sample.h:31-35 kernel(d^2, 1 / r^2) = 3 ir2 / pi (1 - d^2 ir2)^2 in long double
					const float sk = 1.f - heap.d(i) * ir2;
					const float kern = x87mul3(kDiv1ByPi, 3.f * ir2, sk, sk);
					sum = sum + surf_col * kern * pc;
				}
				sum = sum * (1.f / static_cast<float>(S.c_paths));
			}
			col = col + sum;
		}
		if(mode & G_EXTRA) col = col + C3{ex.x, ex.y, ex.z};   // DirectLight AO / the path tracer's paths
		col = col + c3(0.f);   // recursiveRaytrace: the specular tree's part is folded in by k_combine
		if(EXT && S.tree) S.node_own[sid] = f4(col, alpha);
		else
		{
			const SampleCoord sc = sampleAt(S, A.jobs, A.n_jobs, A.chunk_base + (uint64_t)sid);
			A.samples[((size_t)sc.y * S.width + sc.x) * S.spp + sc.s] = f4(col, alpha > 1.f ? 1.f : alpha);
		}
	}
	// counters: wave sums, then one atomic per workgroup (several workgroups share a segment)
	for(int off = 32; off > 0; off >>= 1)
	{
		visits += __shfl_down(visits, off);
		photons += __shfl_down(photons, off);
		overflows += __shfl_down(overflows, off);
	}
	if(threadIdx.x == 0 && S.stats)
	{
		atomicAdd(&S.stats[seg].gather_visits, (unsigned long long)visits);
		atomicAdd(&S.stats[seg].gather_photons, (unsigned long long)photons);
		if(REPLAY && overflows) atomicAdd(&S.stats[seg].gather_overflows, (unsigned long long)overflows);
		if(part == 0) atomicAdd(&S.stats[seg].gather_queries, (unsigned long long)(n_req > jb ? n_req - jb : 0u));
	}
}

// ---------------------------------------------------------------------------------------------
// Final gathering (PhotonIntegrator, finalGather = true)
// ---------------------------------------------------------------------------------------------
// Stable compaction of the radiance points (deposit-slot order = one reference thread's order),
// after k_photon_count / k_photon_scan over rad_flag
__global__ void __launch_bounds__(1024) k_rad_scatter(PhotonState P, const uint32_t *offsets, float4 *out_a, float4 *out_b, float4 *out_c)
{
	uint32_t c;
	uint32_t o = depositBase(P.rad_flag, P.n_local, P.n_slot_rows, offsets, c);
	const uint32_t i = blockIdx.x * 1024u + threadIdx.x;
	for(uint32_t b = 0; c > 0 && b < P.n_slot_rows; ++b)
	{
		const size_t k = (size_t)b * P.n_local + i;
		if(!P.rad_flag[k]) continue;
		out_a[o] = P.rad_a[k];
		out_b[o] = P.rad_b[k];
		out_c[o] = P.rad_c[k];
		++o;
		--c;
	}
}

// The radiance points' getReflectivity means (integrator_photon_mapping.cc:188-190, material.cc:156-174)
// for the kept points of a scene without EXT materials (k_photon_bounce deferred them: .w of a holds
// the primitive): a = (p, refl.r), b = (normal, refl.g), c = (refl.b, transm) as the bounce writes
// them for EXT scenes
__global__ void __launch_bounds__(256) k_rad_refl(DevScene S, float4 *a, float4 *b, float4 *c, const uint32_t *kept, uint32_t n)
{
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if(t >= n) return;
	const uint32_t q = kept[t];
	const float4 pa = a[q];
	const Surf sp = surfFromPrim(S, xyz(pa), __float_as_int(pa.w));
	const DevMaterial &m = S.mats[sp.mat];
	const C3 refl = getReflectivity<false>(S, m, sp, B_DIFFUSE | B_GLOSSY | B_REFLECT);
	const C3 transm = getReflectivity<false>(S, m, sp, B_DIFFUSE | B_GLOSSY | B_TRANSMIT);
	a[q].w = refl.r;
	b[q].w = refl.g;
	c[q] = make_float4(refl.b, transm.r, transm.g, transm.b);
}

// preGatherWorker (integrator_photon_mapping.cc:39-88) for every kept radiance point: k-NN gather of
// the diffuse map within diffuseRadius^2, sum in heap-array order (refl for photons arriving on the
// normal's side, transm otherwise), stored as Photon(normal, pos, sum) of the radiance map
struct PreGatherArgs
{
	DevScene S;
	const float4 *rad_a, *rad_b, *rad_c;
	const uint32_t *kept;
	uint32_t n;
	float4 *out_pos, *out_dir;
	float *out_colb;
	DevStats *stats;   // [0]: pre_visits / pre_photons of the launch (bench.py's byte model), or null
};

__global__ void __launch_bounds__(kGatherBlock) k_pregather(PreGatherArgs A)
{
	extern __shared__ uint4 gather_smem[];
	const DevScene &S = A.S;
	uint32_t *lds_words = reinterpret_cast<uint32_t *>(gather_smem);
	HeapRefPacked heap;
	heap.e = lds_words + 2 * threadIdx.x;
	heap.stride = kGatherBlock;
	const uint32_t gstride = gridDim.x * kGatherBlock;
	uint2 *stk = S.pk_stack + blockIdx.x * kGatherBlock + threadIdx.x;
	const float ds_radius_2 = S.pm_radius2 * S.pm_radius2;   // :42 ds_rad * ds_rad (pm_radius2 holds ds_rad)
	uint32_t visits = 0, found_sum = 0;
	for(uint32_t j = blockIdx.x * kGatherBlock + threadIdx.x; j < A.n; j += gstride)
	{
		const uint32_t r = A.kept[j];
		const float4 a = A.rad_a[r], b = A.rad_b[r], c = A.rad_c[r];
		const V3 pos = xyz(a), rnorm = xyz(b);
		const C3 refl = C3{a.w, b.w, c.x}, transm = C3{c.y, c.z, c.w};
		float radius = ds_radius_2;
		const int found = pkLookup(S.pk_nodes, pos, S.pm_search, radius, heap, stk, gstride, visits);
		C3 sum = c3(0.f);
		if(found > 0)
		{
			found_sum += (uint32_t)found;
			const float scale = S.fg_i_scale / radius;
			for(int i = 0; i < found; ++i)
			{
				const uint32_t ph = heap.i(i);
				const float4 pa = S.ph_pos[ph], pb = S.ph_dir[ph];
				const C3 pc = C3{pa.w, pb.w, S.ph_colb[ph]};
				if(dot(rnorm, xyz(pb)) > 0.f) sum = sum + refl * scale * pc;
				else sum = sum + transm * scale * pc;
			}
		}
		A.out_pos[j] = f4(pos, sum.r);
		A.out_dir[j] = f4(rnorm, sum.g);
		A.out_colb[j] = sum.b;
	}
	if(A.stats)
	{
		for(int off = 32; off > 0; off >>= 1)
		{
			visits += __shfl_down(visits, off);
			found_sum += __shfl_down(found_sum, off);
		}
		if(laneId() == 0)
		{
			atomicAdd(&A.stats->pre_visits, (unsigned long long)visits);
			atomicAdd(&A.stats->pre_photons, (unsigned long long)found_sum);
		}
	}
}

// PhotonMap::findNearest (photon.cc:136-142): NearestPhoton (photon.h:159-169) over the
// non-recursive lookup (pkdtree.h:225-292) — the last photon accepted (facing n, strictly closer
// than the shrinking radius); far children that already fail the radius are not pushed (the radius
// never grows, so the reference discards them at pop time).  -1: none.
__device__ int pkNearest(const uint4 *nodes, const float4 *dirs, V3 p, V3 n, float max_d2, uint32_t *visits)
{
	uint2 stk[64];
	int nearest = -1;
	uint32_t curr = 0;
	int sp_top = 0;
	uint32_t nv = 1;
	for(;;)
	{
		uint4 nd = nodes[curr];
		while((nd.w & 3u) != 3u)
		{
			const int axis = (int)(nd.w & 3u);
			const float split_val = __uint_as_float(nd.x);
			const float pa = axis == 0 ? p.x : (axis == 1 ? p.y : p.z);
			uint32_t far_child;
			if(pa <= split_val) { far_child = nd.w >> 2; curr = curr + 1; }
			else { far_child = curr + 1; curr = nd.w >> 2; }
			float d2 = pa - split_val;
			d2 *= d2;
			if(d2 <= max_d2 && sp_top < 64)
			{
				stk[sp_top] = make_uint2(far_child, __float_as_uint(d2));
				++sp_top;
			}
			nd = nodes[curr];
			++nv;
		}
		const uint32_t ph = nd.w >> 2;
		const V3 v = v3(__uint_as_float(nd.x), __uint_as_float(nd.y), __uint_as_float(nd.z)) - p;
		const float dist_2 = v.x * v.x + v.y * v.y + v.z * v.z;
		if(dist_2 < max_d2)
		{
			if(dot(xyz(dirs[ph]), n) > 0.f) { nearest = (int)ph; max_d2 = dist_2; }
		}
		if(sp_top == 0) break;
		uint2 top = stk[sp_top - 1];
		bool done = false;
		while(__uint_as_float(top.y) > max_d2)
		{
			--sp_top;
			if(sp_top == 0) { done = true; break; }
			top = stk[sp_top - 1];
		}
		if(done) break;
		curr = top.x;
		--sp_top;
		++nv;
	}
	if(visits) *visits += nv;
	return nearest;
}

// PhotonMap::findNearest over the radiance map's uniform grid (RadGrid, fgthin.hip yafamd_rad_grid): the
// facing photon of smallest distance below max_d2 — the photon the kd search (pkNearest) returns, whose only
// dependence on its visit order is which of several facing photons at exactly the same smallest distance it
// keeps (its test is strict: the first one visited).  Such a tie returns -2 and the caller asks the kd search.
// The search grows a block of cells around the point's cell: R = 1 (3 x 3 x 3 cells) first, and a larger block
// only while the best distance so far is not below the block's reach (R cells: every photon outside the block
// is at least that far); rows of 2R + 1 cells along x are contiguous in cell order, and a row farther than the
// best distance (its box, with a margin for the cell rounding) is skipped.  A photon tested again in a larger
// block changes nothing (not below the best, and the tie test skips the kept photon).  The distance and facing
// tests are pkNearest's expressions, so an accepted photon is one it accepts.
__device__ int gridNearest(const RadGrid &g, V3 p, V3 n, float max_d2, uint32_t &visits)
{
	auto cellOf = [](float v, float lo, float inv, int na) {
		const int c = (int)floorf((v - lo) * inv);
		return c < 0 ? 0 : (c >= na ? na - 1 : c);
	};
	const int cx = cellOf(p.x, g.lo[0], g.inv_cell, g.nx), cy = cellOf(p.y, g.lo[1], g.inv_cell, g.ny), cz = cellOf(p.z, g.lo[2], g.inv_cell, g.nz);
	const float margin = 1e-3f * g.cell;
	// squared distance from p to the slab [a, b] of one axis (0 inside)
	auto axisD = [](float v, float a, float b) {
		const float d = v < a ? a - v : (v > b ? v - b : 0.f);
		return d * d;
	};
	// cells per axis that cover the lookup radius (RadGrid: cell >= half of it)
	const int r_max = (int)ceilf(sqrtf(max_d2) * g.inv_cell * 1.001f) + 1;
	float best = max_d2;
	int res = -1;
	bool tie = false;
#pragma unroll 1
	for(int R = 1;; ++R)
	{
		const int x0 = max(cx - R, 0), x1 = min(cx + R, g.nx - 1);
		const float dxx = axisD(p.x, g.lo[0] + (float)x0 * g.cell - margin, g.lo[0] + (float)(x1 + 1) * g.cell + margin);
#pragma unroll 1
		for(int z = max(cz - R, 0); z <= min(cz + R, g.nz - 1); ++z)
		{
			const float dz = axisD(p.z, g.lo[2] + (float)z * g.cell - margin, g.lo[2] + (float)(z + 1) * g.cell + margin);
#pragma unroll 1
			for(int y = max(cy - R, 0); y <= min(cy + R, g.ny - 1); ++y)
			{
				const float dy = axisD(p.y, g.lo[1] + (float)y * g.cell - margin, g.lo[1] + (float)(y + 1) * g.cell + margin);
				if(dxx + dy + dz > best) continue;   // no photon of this row is as close as the best
				const uint32_t base = (uint32_t)((z * g.ny + y) * g.nx);
				const uint32_t k0 = g.start[base + (uint32_t)x0], k1 = g.start[base + (uint32_t)x1 + 1u];
				visits += 1u + (k1 - k0);   // (statistics: the row's start words and its photon records, 16 B each)
				for(uint32_t k = k0; k < k1; ++k)
				{
					const float4 q = g.pos[k];
					const V3 v = v3(q.x, q.y, q.z) - p;
					const float dist_2 = v.x * v.x + v.y * v.y + v.z * v.z;
					if(dist_2 <= best)
					{
						const int idx = (int)__float_as_uint(q.w);
						if(dot(xyz(g.dir[k]), n) > 0.f)
						{
							if(dist_2 < best) { best = dist_2; res = idx; tie = false; }
							else if(res >= 0 && idx != res) tie = true;   // same smallest distance as the photon kept
						}
					}
				}
			}
		}
		// every photon outside this block is at least R cells (less the margin) from p, whose cell is its centre
		const float reach = fmaxf((float)R * g.cell - 2.f * margin, 0.f);
		if(R >= r_max || best < reach * reach) break;
	}
	return tie ? -2 : res;
}

// pkNearest with its far-child stack in an LDS column (4 B per level, stk[level * STRIDE]; cap >= the
// tree depth, so nothing is dropped): a popped interior node carries its parent's plane (pkd.hip), from
// which the distance pkNearest stacked is recomputed for its pop-time test; a popped leaf goes to the
// distance test directly (its photon lies beyond that plane: the two tests agree, as in pkWalk).  Same
// visits in the same order as pkNearest, so the same nearest photon.
template<int STRIDE>
__device__ __forceinline__ int pkNearestLds(const uint4 *nodes, const float4 *dirs, V3 p, V3 n, float max_d2, uint32_t *stk, int cap,
                                            uint32_t &visits)
{
	int nearest = -1;
	uint32_t curr = 0;
	int sp_top = 0;
	uint4 nd = nodes[0];
	++visits;
	for(;;)
	{
		while((nd.w & 3u) != 3u)
		{
			const int axis = (int)(nd.w & 3u);
			const float split_val = __uint_as_float(nd.x);
			const float pa = axis == 0 ? p.x : (axis == 1 ? p.y : p.z);
			uint32_t far_child;
			if(pa <= split_val) { far_child = nd.w >> 2; curr = curr + 1; }
			else { far_child = curr + 1; curr = nd.w >> 2; }
			float d2 = pa - split_val;
			d2 *= d2;
			if(d2 <= max_d2 && sp_top < cap)
			{
				stk[sp_top * STRIDE] = far_child;
				++sp_top;
			}
			nd = nodes[curr];
			++visits;
		}
		const uint32_t ph = nd.w >> 2;
		const V3 v = v3(__uint_as_float(nd.x), __uint_as_float(nd.y), __uint_as_float(nd.z)) - p;
		const float dist_2 = v.x * v.x + v.y * v.y + v.z * v.z;
		if(dist_2 < max_d2)
		{
			if(dot(xyz(dirs[ph]), n) > 0.f) { nearest = (int)ph; max_d2 = dist_2; }
		}
		bool more = false;
		while(sp_top > 0)
		{
			--sp_top;
			curr = stk[sp_top * STRIDE];
			nd = nodes[curr];
			++visits;
			if((nd.w & 3u) != 3u)
			{
				const uint32_t pax = nd.z;
				const float pa = pax == 0u ? p.x : (pax == 1u ? p.y : p.z);
				float d2 = pa - __uint_as_float(nd.y);
				d2 *= d2;
				if(d2 > max_d2) continue;
			}
			more = true;
			break;
		}
		if(!more) break;
	}
	return nearest;
}

// MonteCarloIntegrator::doLightEstimation for one light (integrator_montecarlo.cc:80-408) with the
// shadow rays traced in place: neeLight's arithmetic, neeSum's addition order.  TSH: transparent
// shadows (tr_shad_, :112, 206, 330): the surfaces a shadow ray crosses are collected in ts_buf
// (s_depth entries of this lane) and their filter colour scol multiplies the light colour
// (:122, 212, 335) as k_tshadow does for the wavefront path.
template<bool EXT, bool WIDE, bool SPILL = true, bool TSH = false>
__device__ C3 lightEstimateInline(const DevScene &S, const TraceCtx &C, const DevLight &L, const DevMaterial &m, const Surf &sp, V3 wo,
                                  uint32_t loffs, uint32_t sample_idx, uint32_t offset, uint32_t &visits, uint32_t &tests,
                                  float2 *ts_buf = nullptr)
{
	const bool cast_shadows = L.cast_shadows && m.receive_shadows;
	const float p_len = length(sp.p);
	const float sh_tmin = S.shadow_bias_auto ? S.shadow_bias * fmaxf(1.f, p_len) : S.shadow_bias;
	float t_hit;
	int p_hit;
	// the shadow test of a moved shadow ray (origin so, [tmin, st)); scol = its filter colour
	auto shadowed = [&](V3 so, V3 dir, float tmin, float st, C3 &scol) -> bool {
		scol = c3(1.f);
		if(!cast_shadows) return false;
		if(TSH)
		{
			TsList Lt;
			Lt.hit = ts_buf;
			Lt.n = 0;
			Lt.cap = S.s_depth;
			Lt.prim_ng = S.prim_ng;
			Lt.mats = S.mats;
			if(traverse<true, WIDE, SPILL, true>(C, so, dir, tmin, st, t_hit, p_hit, visits, tests, &Lt)) return true;
			if(Lt.n > 0) scol = tsFilterColor(S, ts_buf, Lt.n, so, dir);
			return false;
		}
		return traverse<true, WIDE, SPILL>(C, so, dir, 0.f, st, t_hit, p_hit, visits, tests);
	};
	if(L.type == LIGHT_POINT)
	{
		C3 c = c3(0.f);
		V3 ldir = lv(L.pos) - sp.p;
		const float dist_sqr = ldir.x * ldir.x + ldir.y * ldir.y + ldir.z * ldir.z;
		const float dist = sqrtf(dist_sqr);
		if(!((double)dist == 0.0))
		{
			const float idist_sqr = rcpExact(dist_sqr);
			ldir = ldir * rcpExact(dist);
			const C3 lcol = C3{L.color[0], L.color[1], L.color[2]} * idist_sqr;
			const float angle = m.flat ? 1.f : fabsf(dot(sp.n, ldir));
			const C3 surf_col = matEval<EXT>(m, sp, wo, ldir, B_ALL);
			V3 so;
			float st;
			shadowRayOf(sp.p, ldir, sh_tmin, dist, so, st);
			C3 scol;
			if(!shadowed(so, ldir, sh_tmin, st, scol)) c = c + surf_col * (TSH && cast_shadows ? lcol * scol : lcol) * angle * c3(1.f);
		}
		return c3(0.f) + c;
	}
	const uint32_t l_offs = loffs * 4567u;
	const int num_samples = L.samples;
	const uint32_t offs = (uint32_t)num_samples * sample_idx + offset + l_offs;
	const C3 lcolor = C3{L.color[0], L.color[1], L.color[2]};
	HaltonInc<2> hal_2;
	HaltonInc<3> hal_3;
	hal_2.value = hal_3.value = 0.0;
	hal_2.start(offs - 1u);
	hal_3.start(offs - 1u);
	C3 acc_l = c3(0.f), acc_m = c3(0.f);
	const float b_tmin = S.ray_min_dist_auto ? S.ray_min_dist * fmaxf(1.f, p_len) : S.ray_min_dist;
	for(int i = 0; i < num_samples; ++i)
	{
		const float s_1 = hal_2.next();
		const float s_2 = hal_3.next();
		// areaLightSampleLight (montecarlo.cc:156-282), light_area.cc:66-96 / light_object_light.cc:111-146
		{
			V3 ldir = v3(0.f, 0.f, 1.f);
			float dist = 0.f, pdf = 0.f;
			const bool ok = lightIllumSample(S, L, sp.p, s_1, s_2, ldir, dist, pdf);
			if(ok)
			{
				if(pdf > 1e-6f)
				{
					const C3 surf_col = matEval<EXT>(m, sp, wo, ldir, B_ALL);
					const float angle = m.flat ? 1.f : fabsf(dot(sp.n, ldir));
					float w = 1.f;
					const float m_pdf = matPdf<EXT>(m, sp, wo, ldir, B_GLOSSY | B_DIFFUSE | B_DISPERSIVE | B_REFLECT | B_TRANSMIT);
					if(m_pdf > 1e-6f)
					{
						const float l_2 = pdf * pdf;
						const float m_2 = m_pdf * m_pdf;
						w = l_2 / (l_2 + m_2);
					}
					V3 so;
					float st;
					shadowRayOf(sp.p, ldir, sh_tmin, dist, so, st);
					C3 scol;
					if(!shadowed(so, ldir, sh_tmin, st, scol))
						acc_l = acc_l + surf_col * (TSH && cast_shadows ? lcolor * scol : lcolor) * angle * w / pdf;
				}
			}
		}
		// areaLightSampleMaterial (montecarlo.cc:284-383), light_area.cc:137-151
		{
			BsdfSample s;
			s.s_1 = s_1;
			s.s_2 = s_2;
			s.flags = B_GLOSSY | B_DIFFUSE | B_DISPERSIVE | B_REFLECT | B_TRANSMIT;
			s.pdf = 0.f;
			s.sampled = B_NONE;
			float W = 0.f;
			V3 dir = v3(0.f, 0.f, 1.f);
			const C3 surf_col = matSample<EXT>(m, sp, wo, dir, s, W);
			bool ok = s.pdf > 1e-6f;
			float t = 0.f, lpdf = 0.f;
			if(ok)
			{
				// light_area.cc:137-151 / light_object_light.cc:183-201
				ok = lightMatHit(S, L, sp.p, dir, b_tmin, t, lpdf);
			}
			if(ok)
			{
				const float light_pdf = lpdf;
				if(light_pdf > 1e-6f)
				{
					const float l_pdf = rcpExact(light_pdf);
					const float l_2 = l_pdf * l_pdf;
					const float m_2 = s.pdf * s.pdf;
					const float w = m_2 / (l_2 + m_2);
					V3 so;
					float st;
					shadowRayOf(sp.p, dir, b_tmin, t, so, st);
					C3 scol;
					if(!shadowed(so, dir, b_tmin, st, scol))
						acc_m = acc_m + surf_col * (TSH && cast_shadows ? lcolor * scol : lcolor) * w * W;
				}
			}
		}
	}
	const C3 col_l = acc_l * L.inv_samples;
	const C3 col_m = acc_m * L.inv_samples;
	return (c3(0.f) + col_l) + col_m;
}

// the hit of a gather ray: surface + (textured scenes) the shader-node colour at the hit, as
// k_photon_bounce evaluates it
template<bool EXT>
__device__ __forceinline__ Surf fgSurf(const DevScene &S, V3 o, V3 d, float t, int prim)
{
	Surf sp = makeSurf(S, o, d, t, prim);
	if(EXT && S.has_attr)
	{
		const SurfAttr sa = surfAttr(S.prim_attr, S.prim_ng, prim, o, d, sp.p);
		const DevMaterial &m = S.mats[sp.mat];
		C3 dcol = C3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
		float drefl = 1.f, sigma = 0.f;
		if(m.n_nodes > 0) evalNodes(m, S.shader_nodes, S.textures, S.texels, sa, dcol, drefl, sigma);
		applyAttr(sp, f4(sa.n, drefl), f4(dcol, sigma));
	}
	return sp;
}

// k_fg: PhotonIntegrator::finalGathering (integrator_photon_mapping.cc:640-763) for every gather
// request with G_FG, one lane per request: fg_samples paths from the camera hit, each traced in
// place (closest rays and the shadow rays of estimateOneDirectLight), ended by a radiance-map
// lookup; the result is added to the request's colour (:908-910, clamp_indirect = 0) for k_gather.
// `mat_bsd_fs` of the reference (:682) is a reference into the first gather hit's MaterialData,
// which the next intersect() frees (:741): here the current hit's flags are read (YafaRay's intent).
struct FgArgs
{
	DevScene S;
	DevNeeQueue G;
	DevCounters cnt_next;
	int stack_depth;
	int *spill;
	float2 *ts_scratch;   // transparent shadows: s_depth (t, prim) entries per lane of the grid
};

// k_fg: the gather-path megakernel wants ~230 VGPRs unconstrained (2 waves / SIMD); capped for 4
// waves / SIMD it spills a little and runs faster (C5 + FG 32: 42.2 -> 31.0 ms; 3 waves: 34.8 ms)
#ifndef YAF_FG_WAVES
#define YAF_FG_WAVES 4
#endif
#define YAF_FG_ATTR __attribute__((amdgpu_waves_per_eu(YAF_FG_WAVES)))
// YAF_FG_REMAT: each gather path rebuilds the request's surface (fewer registers live through the traversals)
#ifndef YAF_FG_REMAT
#define YAF_FG_REMAT 1
#endif
// YAF_FG_STAGE: an LDS-resident scene's primitive records and materials are staged after the stacks as
// well (the gather paths' surface lookups from LDS instead of L2)
#ifndef YAF_FG_STAGE
#define YAF_FG_STAGE 1
#endif
// Staging only when the whole dynamic LDS of the launch stays within 64 KB: the trace stack, the scene,
// the nearest-search column rounded to 16 B, then the materials and primitive records.  The kernel and
// yafamd_launch_fg take the same decision from the same (uniform) arguments.
__host__ __device__ inline bool fgStageTables(const DevScene &S, bool lds_scene, bool ext, int stack_depth)
{
	if(!(YAF_FG_STAGE && lds_scene && !ext && S.small_tables)) return false;
	const size_t stack_b = (size_t)stack_depth * kTraceBlock * sizeof(int);
	const size_t scene_b = (size_t)(S.node_f4 * S.n_nodes + 3 * S.n_tris) * 16u;
	const size_t nstk_b = (((size_t)S.rpk_lds * kTraceBlock * sizeof(uint32_t)) + 15u) & ~(size_t)15u;
	const size_t tab_b = (size_t)S.n_mats * sizeof(DevMaterial) + (size_t)S.n_tris * 16u;
	return stack_b + scene_b + nstk_b + tab_b <= (size_t)64 * 1024;
}
template<bool LDS_SCENE, bool WIDE, bool EXT, bool SPILL = true, bool TSH = false>
__global__ void __launch_bounds__(kTraceBlock) YAF_FG_ATTR k_fg(FgArgs A)
{
	DevScene S_ = A.S;
	const DevScene &S = S_;
	extern __shared__ float4 smem[];
	TraceCtx C;
	C.wave_base = waveBase();
	C.stack = reinterpret_cast<int *>(smem);
	C.lds_depth = A.stack_depth;
	C.spill = A.spill;
	C.spill_stride = gridDim.x * blockDim.x;
	if(LDS_SCENE)
	{
		float4 *lds_nodes = smem + (A.stack_depth * kTraceBlock) / 4;
		float4 *lds_tris = lds_nodes + S.node_f4 * S.n_nodes;
		for(int k = threadIdx.x; k < S.node_f4 * S.n_nodes; k += blockDim.x) lds_nodes[k] = S.nodes[k];
		for(int k = threadIdx.x; k < 3 * S.n_tris; k += blockDim.x) lds_tris[k] = S.tris[k];
		__syncthreads();
		C.nodes = lds_nodes;
		C.tris = lds_tris;
	}
	else
	{
		C.nodes = S.nodes;
		C.tris = S.tris;
	}
	// the radiance-map nearest searches' LDS stack column (S.rpk_lds levels), after the stack and scene
	uint32_t *nstk = reinterpret_cast<uint32_t *>(smem + (A.stack_depth * kTraceBlock) / 4 +
	                                              (LDS_SCENE ? S.node_f4 * S.n_nodes + 3 * S.n_tris : 0)) + threadIdx.x;
	if(fgStageTables(A.S, LDS_SCENE, EXT, A.stack_depth))
	{
		// after the nearest-search column (S.rpk_lds levels of one word per lane)
		uint4 *tp = reinterpret_cast<uint4 *>(smem + (A.stack_depth * kTraceBlock) / 4 + (S.node_f4 * S.n_nodes + 3 * S.n_tris) +
		                                      ((size_t)S.rpk_lds * kTraceBlock + 3) / 4);
		const int nm = A.S.n_mats * (int)(sizeof(DevMaterial) / 16);
		copy16(tp, A.S.mats, nm);
		copy16(tp + nm, A.S.prim_ng, A.S.n_tris);
		__syncthreads();
		S_.mats = reinterpret_cast<const DevMaterial *>(tp);
		S_.prim_ng = reinterpret_cast<const float4 *>(tp + nm);
	}
	// statistics of the frame (bench.py's k_fg byte model): gather paths traced, radiance-map lookups and
	// the radiance-map kd nodes they fetched
	uint32_t n_paths = 0, n_lookups = 0, n_nvisits = 0;
	auto nearestRad = [&](V3 hp, V3 sf) -> int {
		++n_lookups;
		return S.rpk_lds > 0 ? pkNearestLds<kTraceBlock>(S.rpk_nodes, S.rph_dir, hp, sf, S.fg_lookup_rad, nstk, S.rpk_lds, n_nvisits)
		                     : pkNearest(S.rpk_nodes, S.rph_dir, hp, sf, S.fg_lookup_rad, &n_nvisits);
	};
	const bool ATTR = EXT && S.has_attr != 0;
	const SegLoop L = segLoop(S.n_seg);
	const uint32_t n_req = A.cnt_next.n_gather[L.s];
	const uint32_t a0 = L.s * S.cap_a;
	uint32_t visits = 0, tests = 0;
	// finalGathering (integrator_photon_mapping.cc:648): ceilf(max(1, n_paths) * aa_indirect_sample_multiplier_)
	const int n_sampl = S.fg_pass_samples > 0 ? S.fg_pass_samples : max(1, S.fg_samples);
	float2 *ts_buf = TSH ? A.ts_scratch + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * (size_t)S.s_depth : nullptr;
	for(uint32_t jj = L.r * blockDim.x + threadIdx.x; jj < n_req; jj += L.nb * blockDim.x)
	{
		const uint32_t j = a0 + jj;
		const float4 ex = A.G.extra[j];
		if(!(__float_as_uint(ex.w) & G_FG)) continue;
		const uint32_t offset = __float_as_uint(ex.x), sample_idx = __float_as_uint(ex.y);
		const float4 pp = A.G.p_prim[j];
#if !YAF_FG_REMAT
		Surf sp0 = surfFromPrim(S, xyz(pp), __float_as_int(pp.w));
		if(ATTR) applyAttr(sp0, A.G.attr[2 * (size_t)j], A.G.attr[2 * (size_t)j + 1]);
		const DevMaterial &m0 = S.mats[sp0.mat];
#endif
		const V3 wo0 = xyz(A.G.wo_k[j]);
		C3 path_col = c3(0.f);
		for(int i = 0; i < n_sampl; ++i)
		{
#if YAF_FG_REMAT
			// the request's surface is rebuilt for every gather path (bit for bit the same) instead of being
			// kept in registers through the traversals: the opaque copy keeps it inside the loop
			float4 ppi = pp;
			asm volatile("" : "+v"(ppi.x), "+v"(ppi.y), "+v"(ppi.z), "+v"(ppi.w));
			Surf sp0 = surfFromPrim(S, xyz(ppi), __float_as_int(ppi.w));
			if(ATTR) applyAttr(sp0, A.G.attr[2 * (size_t)j], A.G.attr[2 * (size_t)j + 1]);
			const DevMaterial &m0 = S.mats[sp0.mat];
#endif
			const uint32_t offs = (uint32_t)S.fg_samples * sample_idx + offset + (uint32_t)i;
			BsdfSample s;
			s.s_1 = riVdC(offs);
			s.s_2 = ldsDim(S, 2, offs);
			s.flags = B_DIFFUSE | B_REFLECT | B_TRANSMIT;
			s.pdf = 0.f;
			s.sampled = B_NONE;
			float w = 0.f;
			V3 dir = v3(0.f, 0.f, 0.f);
			C3 scol = matSample<EXT>(m0, sp0, wo0, dir, s, w);
			scol = scol * w;
			if(isBlack(scol)) continue;
			C3 throughput = scol;
			float t;
			int prim;
			V3 from = sp0.p;
			++n_paths;
			if(!traverse<false, WIDE, SPILL>(C, from, dir, S.ray_min_dist, __builtin_huge_valf(), t, prim, visits, tests)) continue;
			Surf hit = fgSurf<EXT>(S, from, dir, t, prim);
			float length = t;
			uint32_t mat_bsd_fs = hit.flags;
			bool did_hit = true;
			bool caustic = false;
			bool close = length < S.fg_min_pathlen;
			bool do_bounce = close || (mat_bsd_fs & B_SPECULAR);
			C3 lcol = c3(0.f);
			for(int depth = 0; depth < S.fg_bounces && do_bounce; ++depth)
			{
				const int d_4 = 4 * depth;
				const V3 pwo = -dir;
				const DevMaterial &mh = S.mats[hit.mat];
				if(mat_bsd_fs & B_DIFFUSE)
				{
					if(close)
					{
						// estimateOneDirectLight (integrator_montecarlo.cc:70-78); the light pick as pickLight
						// describes (the reference's counter runs per thread; one light is exact)
						const uint32_t lnum = pickLight(S, offset, sample_idx, (uint32_t)i * (uint32_t)max(1, S.fg_bounces) + (uint32_t)depth,
						                                (uint32_t)n_sampl * (uint32_t)(max(1, S.fg_bounces) + 1));
						lcol = (S.n_lights > 0)
						           ? lightEstimateInline<EXT, WIDE, SPILL, TSH>(S, C, S.lights[lnum], mh, hit, pwo, lnum, sample_idx, offset, visits, tests,
						                                                        ts_buf) *
						                 (float)S.n_lights
						           : c3(0.f);
					}
					else if(caustic)
					{
						const V3 sf = faceForward(hit.ng, hit.n, pwo);
						const int nearest = nearestRad(hit.p, sf);
						if(nearest >= 0) lcol = C3{S.rph_pos[nearest].w, S.rph_dir[nearest].w, S.rph_colb[nearest]};
					}
					if(close || caustic)
					{
						if(mat_bsd_fs & B_EMIT) lcol = lcol + matEmit<EXT>(mh, hit, pwo);
						path_col = path_col + lcol * throughput;
					}
				}
				BsdfSample sb;
				sb.s_1 = ldsDim(S, d_4 + 3, offs);
				sb.s_2 = ldsDim(S, d_4 + 4, offs);
				sb.flags = close ? B_ALL : (B_SPECULAR | B_REFLECT | B_TRANSMIT | B_FILTER);
				sb.pdf = 0.f;
				sb.sampled = B_NONE;
				V3 ndir = v3(0.f, 0.f, 0.f);
				scol = matSample<EXT>(mh, hit, pwo, ndir, sb, w);
				if(sb.pdf <= 1.0e-6f) { did_hit = false; break; }
				scol = scol * w;
				throughput = throughput * scol;
				from = hit.p;
				dir = ndir;
				if(!traverse<false, WIDE, SPILL>(C, from, dir, S.ray_min_dist, __builtin_huge_valf(), t, prim, visits, tests)) { did_hit = false; break; }
				hit = fgSurf<EXT>(S, from, dir, t, prim);
				mat_bsd_fs = hit.flags;
				length += t;
				caustic = (caustic || !depth) && (sb.sampled & (B_SPECULAR | B_FILTER));
				close = length < S.fg_min_pathlen;
				do_bounce = caustic || close;
			}
			if(did_hit && (mat_bsd_fs & (B_DIFFUSE | B_GLOSSY)))
			{
				const V3 sf = faceForward(hit.ng, hit.n, -dir);
				const int nearest = nearestRad(hit.p, sf);
				if(nearest >= 0) lcol = C3{S.rph_pos[nearest].w, S.rph_dir[nearest].w, S.rph_colb[nearest]};
				if(mat_bsd_fs & B_EMIT)
				{
#if YAF_FG_REMAT
					// the hit rebuilt (bit for bit) rather than kept live through the nearest search
					float tt = t;
					asm volatile("" : "+v"(tt));
					hit = fgSurf<EXT>(S, from, dir, tt, prim);
#endif
					lcol = lcol + matEmit<EXT>(S.mats[hit.mat], hit, -dir);
				}
				path_col = path_col + lcol * throughput;
			}
		}
		const C3 fg = path_col / (float)n_sampl;
		const uint4 cb = A.G.pix_mode[j];
		const C3 col = C3{__uint_as_float(cb.x), __uint_as_float(cb.y), __uint_as_float(cb.z)} + fg;
		A.G.pix_mode[j] = make_uint4(__float_as_uint(col.r), __float_as_uint(col.g), __float_as_uint(col.b), cb.w);
	}
	if(S.stats)
	{
		for(int off = 32; off > 0; off >>= 1)
		{
			n_paths += __shfl_down(n_paths, off);
			n_lookups += __shfl_down(n_lookups, off);
			n_nvisits += __shfl_down(n_nvisits, off);
		}
		if(laneId() == 0)
		{
			atomicAdd(&S.stats[L.s].fg_paths, (unsigned long long)n_paths);
			atomicAdd(&S.stats[L.s].fg_lookups, (unsigned long long)n_lookups);
			atomicAdd(&S.stats[L.s].fg_nearest_visits, (unsigned long long)n_nvisits);
		}
	}
}

// ---------------------------------------------------------------------------------------------
// Final gathering with one lane per gather path (r06; k_fg kept for transparent shadows and scenes in
// global memory).  k_fg ran one lane per request through its fg_samples paths: the rare paths that bounce
// (a close or specular first hit: the light estimate with its shadow rays, further traversals) kept
// ~230 registers live for every lane (89 spilled at 4 waves per SIMD, 4.8 GB of scratch traffic per
// launch) and held their wave at VALU lane utilisation 0.28.  Here a batch of requests runs as
//   k_fg_first  one lane per (request, path): the path's first segment (matSample, closest ray), the
//               radiance-map lookup of the paths that end at their first hit — their one term — and the
//               paths that bounce appended to a per-segment list with the state after their first hit;
//   k_fg_long   one lane per bouncing path: finalGathering's bounce loop and last lookup (k_fg's code),
//               every addition to the path colour kept as a term;
//   k_fg_sum    one lane per request: the terms summed path by path, in the order k_fg added them
//               (path_col = path_col + term, integrator_photon_mapping.cc:707-755), bit for bit k_fg's.
// A batch is the request positions [j0, j0 + seg_cap) of every segment of the gather queue.
// ---------------------------------------------------------------------------------------------

constexpr uint32_t kFgDone = 0xffffffffu;   // terms tag of a request's first path: k_fg_first already added its paths

struct FgPathArgs
{
	FgArgs A;
	FgBatch B;
};

// k_fg's prologue: the trace context (stack, LDS scene), the nearest-search column, the staged tables
template<bool LDS_SCENE, bool EXT>
__device__ __forceinline__ uint32_t *fgPrologue(const FgArgs &A, DevScene &S_, TraceCtx &C, float4 *smem)
{
	const DevScene &S = S_;
	C.wave_base = waveBase();
	C.stack = reinterpret_cast<int *>(smem);
	C.lds_depth = A.stack_depth;
	C.spill = A.spill;
	C.spill_stride = gridDim.x * blockDim.x;
	if(LDS_SCENE)
	{
		float4 *lds_nodes = smem + (A.stack_depth * kTraceBlock) / 4;
		float4 *lds_tris = lds_nodes + S.node_f4 * S.n_nodes;
		for(int k = threadIdx.x; k < S.node_f4 * S.n_nodes; k += blockDim.x) lds_nodes[k] = S.nodes[k];
		for(int k = threadIdx.x; k < 3 * S.n_tris; k += blockDim.x) lds_tris[k] = S.tris[k];
		__syncthreads();
		C.nodes = lds_nodes;
		C.tris = lds_tris;
	}
	else
	{
		C.nodes = S.nodes;
		C.tris = S.tris;
	}
	uint32_t *nstk = reinterpret_cast<uint32_t *>(smem + (A.stack_depth * kTraceBlock) / 4 +
	                                              (LDS_SCENE ? S.node_f4 * S.n_nodes + 3 * S.n_tris : 0)) + threadIdx.x;
	if(fgStageTables(A.S, LDS_SCENE, EXT, A.stack_depth))
	{
		uint4 *tp = reinterpret_cast<uint4 *>(smem + (A.stack_depth * kTraceBlock) / 4 + (S.node_f4 * S.n_nodes + 3 * S.n_tris) +
		                                      ((size_t)S.rpk_lds * kTraceBlock + 3) / 4);
		const int nm = A.S.n_mats * (int)(sizeof(DevMaterial) / 16);
		copy16(tp, A.S.mats, nm);
		copy16(tp + nm, A.S.prim_ng, A.S.n_tris);
		__syncthreads();
		S_.mats = reinterpret_cast<const DevMaterial *>(tp);
		S_.prim_ng = reinterpret_cast<const float4 *>(tp + nm);
	}
	return nstk;
}

__device__ __forceinline__ void fgStats(const DevScene &S, uint32_t seg, uint32_t n_paths, uint32_t n_lookups, uint32_t n_nvisits)
{
	if(!S.stats) return;
	for(int off = 32; off > 0; off >>= 1)
	{
		n_paths += __shfl_down(n_paths, off);
		n_lookups += __shfl_down(n_lookups, off);
		n_nvisits += __shfl_down(n_nvisits, off);
	}
	if(laneId() == 0)
	{
		atomicAdd(&S.stats[seg].fg_paths, (unsigned long long)n_paths);
		atomicAdd(&S.stats[seg].fg_lookups, (unsigned long long)n_lookups);
		atomicAdd(&S.stats[seg].fg_nearest_visits, (unsigned long long)n_nvisits);
	}
}

// requests of segment `s` in this batch
__device__ __forceinline__ uint32_t fgBatchRequests(const FgArgs &A, const FgBatch &B, uint32_t s)
{
	const uint32_t n_req = A.cnt_next.n_gather[s];
	return n_req > B.j0 ? min(n_req - B.j0, B.seg_cap) : 0u;
}

template<bool LDS_SCENE, bool WIDE, bool EXT, bool SPILL>
__global__ void __launch_bounds__(kTraceBlock) k_fg_first(FgPathArgs PA)
{
	const FgArgs &A = PA.A;
	const FgBatch &B = PA.B;
	DevScene S_ = A.S;
	const DevScene &S = S_;
	extern __shared__ float4 smem[];
	TraceCtx C;
	uint32_t *nstk = fgPrologue<LDS_SCENE, EXT>(A, S_, C, smem);
	uint32_t n_paths = 0, n_lookups = 0, n_nvisits = 0, visits = 0, tests = 0;
	const bool ATTR = EXT && S.has_attr != 0;
	const SegLoop L = segLoop(S.n_seg);
	const uint32_t n_b = fgBatchRequests(A, B, L.s);
	const uint32_t ns = (uint32_t)B.n_sampl;
	const uint32_t n_p = n_b * ns;
	const uint32_t a0 = L.s * S.cap_a;
	float4 *terms = B.terms + (size_t)L.s * B.seg_cap * ns;
	// a request's paths are one aligned group of ns lanes when ns divides the wave: a group without a bouncing
	// path folds its terms in path order right here (k_fg_sum then skips the request)
	const bool fold = (64u % ns) == 0u;
	for(uint32_t p = L.r * blockDim.x + threadIdx.x; p < n_p; p += L.nb * blockDim.x)
	{
		const uint32_t jj = p / ns, i = p - jj * ns;
		const uint32_t j = a0 + B.j0 + jj;
		const float4 ex = A.G.extra[j];
		const bool req_fg = (__float_as_uint(ex.w) & G_FG) != 0u;   // (k_fg_sum skips the others as well)
		float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
		if(req_fg)
		{
		const uint32_t offset = __float_as_uint(ex.x), sample_idx = __float_as_uint(ex.y);
		const float4 pp = A.G.p_prim[j];
		Surf sp0 = surfFromPrim(S, xyz(pp), __float_as_int(pp.w));
		if(ATTR) applyAttr(sp0, A.G.attr[2 * (size_t)j], A.G.attr[2 * (size_t)j + 1]);
		const DevMaterial &m0 = S.mats[sp0.mat];
		const V3 wo0 = xyz(A.G.wo_k[j]);
		const uint32_t offs = (uint32_t)S.fg_samples * sample_idx + offset + i;
		BsdfSample s;
		s.s_1 = riVdC(offs);
		s.s_2 = ldsDim(S, 2, offs);
		s.flags = B_DIFFUSE | B_REFLECT | B_TRANSMIT;
		s.pdf = 0.f;
		s.sampled = B_NONE;
		float w = 0.f;
		V3 dir = v3(0.f, 0.f, 0.f);
		C3 scol = matSample<EXT>(m0, sp0, wo0, dir, s, w);
		scol = scol * w;
		if(!isBlack(scol))
		{
			const C3 throughput = scol;
			const V3 from = sp0.p;
			float t;
			int prim;
			++n_paths;
			if(traverse<false, WIDE, SPILL, false, false, LDS_SCENE>(C, from, dir, S.ray_min_dist, __builtin_huge_valf(), t, prim, visits, tests))
			{
				const Surf hit = fgSurf<EXT>(S, from, dir, t, prim);
				const uint32_t mat_bsd_fs = hit.flags;
				const bool close = t < S.fg_min_pathlen;
				const bool do_bounce = close || (mat_bsd_fs & B_SPECULAR);
				if(do_bounce && S.fg_bounces > 0)
				{
					// the bounce loop runs in k_fg_long (compacted: a wave of bouncing paths)
					const uint32_t q = atomicAdd(&B.long_count[L.s], 1u);
					float4 *rec = B.longs + ((size_t)L.s * B.long_cap + q) * 3;
					rec[0] = f4(from, t);
					rec[1] = f4(dir, __int_as_float(prim));
					rec[2] = f4(throughput, __uint_as_float(p));
					out.w = __uint_as_float(2u + q);
				}
				else if(mat_bsd_fs & (B_DIFFUSE | B_GLOSSY))
				{
					// the path ends at its first hit: k_fg's last lookup (lcol is still zero here)
					C3 lcol = c3(0.f);
					const V3 sf = faceForward(hit.ng, hit.n, -dir);
					++n_lookups;
					int nearest = S.fg_probe == 1 ? -1 : S.rgrid.start ? gridNearest(S.rgrid, hit.p, sf, S.fg_lookup_rad, n_nvisits) : -2;
					if(nearest == -2)
						nearest = S.rpk_lds > 0 ? pkNearestLds<kTraceBlock>(S.rpk_nodes, S.rph_dir, hit.p, sf, S.fg_lookup_rad, nstk, S.rpk_lds, n_nvisits)
						                        : pkNearest(S.rpk_nodes, S.rph_dir, hit.p, sf, S.fg_lookup_rad, &n_nvisits);
					if(nearest >= 0) lcol = C3{S.rph_pos[nearest].w, S.rph_dir[nearest].w, S.rph_colb[nearest]};
					if(mat_bsd_fs & B_EMIT) lcol = lcol + matEmit<EXT>(S.mats[hit.mat], hit, -dir);
					out = f4(lcol * throughput, __uint_as_float(1u));
				}
			}
		}
		}
		if(fold)
		{
			// ns | 64: p = 64 w + lane, so path i of the request sits in lane (lane - i) + i of this wave
			const uint32_t lane = laneId(), g0 = lane - i;
			const bool longp = __float_as_uint(out.w) >= 2u;
			const uint64_t lm = __ballot(longp);
			const uint64_t gm = (ns == 64u ? ~0ull : ((1ull << ns) - 1ull)) << g0;
			if((lm & gm) == 0ull)
			{
				// path_col = path_col + term, path by path (k_fg's order), the sum in every lane of the group
				C3 path_col = c3(0.f);
				for(uint32_t q = 0; q < ns; ++q)
				{
					const int src = (int)(g0 + q);
					const float tr = __shfl(out.x, src), tg = __shfl(out.y, src), tb = __shfl(out.z, src);
					const uint32_t tt = __shfl(__float_as_uint(out.w), src);
					if(tt == 1u) path_col = path_col + C3{tr, tg, tb};
				}
				if(i == 0u && req_fg)
				{
					const C3 fg = path_col / (float)B.n_sampl;
					const uint4 cb = A.G.pix_mode[j];
					const C3 col = C3{__uint_as_float(cb.x), __uint_as_float(cb.y), __uint_as_float(cb.z)} + fg;
					A.G.pix_mode[j] = make_uint4(__float_as_uint(col.r), __float_as_uint(col.g), __float_as_uint(col.b), cb.w);
					terms[p] = make_float4(0.f, 0.f, 0.f, __uint_as_float(kFgDone));
				}
			}
			else terms[p] = out;
		}
		else terms[p] = out;
	}
	fgStats(S, L.s, n_paths, n_lookups, n_nvisits);
}

template<bool LDS_SCENE, bool WIDE, bool EXT, bool SPILL, bool TSH>
__global__ void __launch_bounds__(kTraceBlock) YAF_FG_ATTR k_fg_long(FgPathArgs PA)
{
	const FgArgs &A = PA.A;
	const FgBatch &B = PA.B;
	DevScene S_ = A.S;
	const DevScene &S = S_;
	extern __shared__ float4 smem[];
	TraceCtx C;
	uint32_t *nstk = fgPrologue<LDS_SCENE, EXT>(A, S_, C, smem);
	uint32_t n_lookups = 0, n_nvisits = 0, visits = 0, tests = 0;
	auto nearestRad = [&](V3 hp, V3 sf) -> int {
		++n_lookups;
		const int g = S.rgrid.start ? gridNearest(S.rgrid, hp, sf, S.fg_lookup_rad, n_nvisits) : -2;
		if(g != -2) return g;
		return S.rpk_lds > 0 ? pkNearestLds<kTraceBlock>(S.rpk_nodes, S.rph_dir, hp, sf, S.fg_lookup_rad, nstk, S.rpk_lds, n_nvisits)
		                     : pkNearest(S.rpk_nodes, S.rph_dir, hp, sf, S.fg_lookup_rad, &n_nvisits);
	};
	const SegLoop L = segLoop(S.n_seg);
	const uint32_t n_long = B.long_count[L.s];
	const uint32_t ns = (uint32_t)B.n_sampl;
	const uint32_t a0 = L.s * S.cap_a;
	const int n_sampl = B.n_sampl;
	float2 *ts_buf = TSH ? A.ts_scratch + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * (size_t)S.s_depth : nullptr;
	for(uint32_t q = L.r * blockDim.x + threadIdx.x; q < n_long; q += L.nb * blockDim.x)
	{
		const float4 *rec = B.longs + ((size_t)L.s * B.long_cap + q) * 3;
		const float4 r0 = rec[0], r1 = rec[1], r2 = rec[2];
		const uint32_t p = __float_as_uint(r2.w);
		const uint32_t jj = p / ns, i = p - jj * ns;
		const uint32_t j = a0 + B.j0 + jj;
		const float4 ex = A.G.extra[j];
		const uint32_t offset = __float_as_uint(ex.x), sample_idx = __float_as_uint(ex.y);
		const uint32_t offs = (uint32_t)S.fg_samples * sample_idx + offset + i;
		float4 *out = B.long_terms + ((size_t)L.s * B.long_cap + q) * (size_t)B.n_terms;
		int nt = 0;
		C3 throughput = rgb(r2);
		V3 from = xyz(r0), dir = xyz(r1);
		float t = r0.w;
		int prim = __float_as_int(r1.w);
		float w = 0.f;
		C3 scol;
		// k_fg from the first hit on (the same statements; path_col additions become terms)
		Surf hit = fgSurf<EXT>(S, from, dir, t, prim);
		float length = t;
		uint32_t mat_bsd_fs = hit.flags;
		bool did_hit = true;
		bool caustic = false;
		bool close = length < S.fg_min_pathlen;
		bool do_bounce = close || (mat_bsd_fs & B_SPECULAR);
		C3 lcol = c3(0.f);
		for(int depth = 0; depth < S.fg_bounces && do_bounce; ++depth)
		{
			const int d_4 = 4 * depth;
			const V3 pwo = -dir;
			const DevMaterial &mh = S.mats[hit.mat];
			if(mat_bsd_fs & B_DIFFUSE)
			{
				if(close)
				{
					const uint32_t lnum = pickLight(S, offset, sample_idx, (uint32_t)i * (uint32_t)max(1, S.fg_bounces) + (uint32_t)depth,
					                                (uint32_t)n_sampl * (uint32_t)(max(1, S.fg_bounces) + 1));
					lcol = (S.n_lights > 0)
					           ? lightEstimateInline<EXT, WIDE, SPILL, TSH>(S, C, S.lights[lnum], mh, hit, pwo, lnum, sample_idx, offset, visits, tests,
					                                                        ts_buf) *
					                 (float)S.n_lights
					           : c3(0.f);
				}
				else if(caustic)
				{
					const V3 sf = faceForward(hit.ng, hit.n, pwo);
					const int nearest = nearestRad(hit.p, sf);
					if(nearest >= 0) lcol = C3{S.rph_pos[nearest].w, S.rph_dir[nearest].w, S.rph_colb[nearest]};
				}
				if(close || caustic)
				{
					if(mat_bsd_fs & B_EMIT) lcol = lcol + matEmit<EXT>(mh, hit, pwo);
					if(nt < B.n_terms) out[nt++] = f4(lcol * throughput, 1.f);
				}
			}
			BsdfSample sb;
			sb.s_1 = ldsDim(S, d_4 + 3, offs);
			sb.s_2 = ldsDim(S, d_4 + 4, offs);
			sb.flags = close ? B_ALL : (B_SPECULAR | B_REFLECT | B_TRANSMIT | B_FILTER);
			sb.pdf = 0.f;
			sb.sampled = B_NONE;
			V3 ndir = v3(0.f, 0.f, 0.f);
			scol = matSample<EXT>(mh, hit, pwo, ndir, sb, w);
			if(sb.pdf <= 1.0e-6f) { did_hit = false; break; }
			scol = scol * w;
			throughput = throughput * scol;
			from = hit.p;
			dir = ndir;
			if(!traverse<false, WIDE, SPILL>(C, from, dir, S.ray_min_dist, __builtin_huge_valf(), t, prim, visits, tests)) { did_hit = false; break; }
			hit = fgSurf<EXT>(S, from, dir, t, prim);
			mat_bsd_fs = hit.flags;
			length += t;
			caustic = (caustic || !depth) && (sb.sampled & (B_SPECULAR | B_FILTER));
			close = length < S.fg_min_pathlen;
			do_bounce = caustic || close;
		}
		if(did_hit && (mat_bsd_fs & (B_DIFFUSE | B_GLOSSY)))
		{
			const V3 sf = faceForward(hit.ng, hit.n, -dir);
			const int nearest = nearestRad(hit.p, sf);
			if(nearest >= 0) lcol = C3{S.rph_pos[nearest].w, S.rph_dir[nearest].w, S.rph_colb[nearest]};
			if(mat_bsd_fs & B_EMIT) lcol = lcol + matEmit<EXT>(S.mats[hit.mat], hit, -dir);
			if(nt < B.n_terms) out[nt++] = f4(lcol * throughput, 1.f);
		}
		for(int k = nt; k < B.n_terms; ++k) out[k] = make_float4(0.f, 0.f, 0.f, 0.f);
	}
	fgStats(S, L.s, 0u, n_lookups, n_nvisits);
}

__global__ void __launch_bounds__(256) k_fg_sum(FgPathArgs PA)
{
	const FgArgs &A = PA.A;
	const FgBatch &B = PA.B;
	const DevScene &S = A.S;
	const uint32_t s = blockIdx.y;
	const uint32_t n_b = fgBatchRequests(A, B, s);
	const uint32_t ns = (uint32_t)B.n_sampl;
	const uint32_t a0 = s * S.cap_a;
	for(uint32_t jj = blockIdx.x * blockDim.x + threadIdx.x; jj < n_b; jj += gridDim.x * blockDim.x)
	{
		const uint32_t j = a0 + B.j0 + jj;
		if(!(__float_as_uint(A.G.extra[j].w) & G_FG)) continue;
		const float4 *tp = B.terms + ((size_t)s * B.seg_cap + jj) * ns;
		if(__float_as_uint(tp[0].w) == kFgDone) continue;   // folded by k_fg_first (no bouncing path)
		C3 path_col = c3(0.f);
		for(uint32_t i = 0; i < ns; ++i)
		{
			const float4 tv = tp[i];
			const uint32_t tag = __float_as_uint(tv.w);
			if(tag == 1u) path_col = path_col + rgb(tv);
			else if(tag >= 2u)
			{
				const float4 *lt = B.long_terms + ((size_t)s * B.long_cap + (tag - 2u)) * (size_t)B.n_terms;
				for(int k = 0; k < B.n_terms; ++k)
				{
					const float4 v = lt[k];
					if(v.w != 0.f) path_col = path_col + rgb(v);
				}
			}
		}
		const C3 fg = path_col / (float)B.n_sampl;
		const uint4 cb = A.G.pix_mode[j];
		const C3 col = C3{__uint_as_float(cb.x), __uint_as_float(cb.y), __uint_as_float(cb.z)} + fg;
		A.G.pix_mode[j] = make_uint4(__float_as_uint(col.r), __float_as_uint(col.g), __float_as_uint(col.b), cb.w);
	}
}

} // namespace yafamd

// ---------------------------------------------------------------------------------------------
// launch wrappers used by render.cc (C++ host code, no HIP language there)
// ---------------------------------------------------------------------------------------------
using namespace yafamd;

extern "C" {

int yafamd_trace_block() { return kTraceBlock; }

// Whether the non-EXT k_shade runs the next-event estimation itself (then render.cc launches no
// k_nee for those scenes); -DYAF_FUSE builds that variant (measured slower, see kShadeFused).
int yafamd_shade_fused() { return kShadeFused ? 1 : 0; }
// the k_shade this scene launches runs the NEE itself (kShadeFused, or the lean fused tuning build)
int yafamd_shade_fused_for(const DevScene *S)
{
	if(S->ext) return 0;
	if(kShadeFused) return 1;
	return (YAF_FUSE_LEAN && S->integrator == INT_PATH && S->path_samples <= 1 && !S->do_ao && !S->caus_map && !S->gather_on && !S->show_map &&
	        S->n_photons == 0 && !S->tree && !S->has_attr && !S->no_lean && !S->tr_shad && !S->has_mesh_light) ? 1 : 0;
}

// Whether the measured-and-dropped pipelines are compiled in (-DYAF_EXPERIMENTS)
int yafamd_experiments() { return kExperiments ? 1 : 0; }

// The flags this device object was compiled with (Makefile DEVINFO): yafaray_amd_buildInfo.
#ifndef YAF_DEVICE_BUILD
#define YAF_DEVICE_BUILD "arch=? extra=[?] (built outside csrc/Makefile)"
#endif
const char *yafamd_device_build() { return YAF_DEVICE_BUILD
#ifdef YAF_PHASE_TIMING
	" phase-timing"
#endif
	; }

// Diagnostic: k_shade phase cycles (only a -DYAF_PHASE_TIMING build records them).
int yafamd_phase_cycles(unsigned long long *out, int n, int reset)
{
#ifdef YAF_PHASE_TIMING
	unsigned long long h[16];
	if(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_phase), sizeof(h)) != hipSuccess) return 0;
	for(int k = 0; k < n && k < 16; ++k) out[k] = h[k];
	if(reset)
	{
		const unsigned long long z[16] = {};
		if(hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)) != hipSuccess) return 0;
	}
	return 16;
#else
	(void)out; (void)n; (void)reset;
	return 0;
#endif
}

// Resident workgroups per CU of the persistent kernels (their grids fill the chip exactly once).
int yafamd_trace_blocks_per_cu(int lds_scene, int wide, size_t dyn_lds)
{
	int nb = 0;
	hipError_t e;
	if(wide == 8) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_trace<false, true, false, true, false, false, true>, kTraceBlock, dyn_lds);
	else if(lds_scene) e = wide ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_trace<true, true, false>, kTraceBlock, dyn_lds)
	                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_trace<true, false, false>, kTraceBlock, dyn_lds);
	else e = wide ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_trace<false, true, false>, kTraceBlock, dyn_lds)
	              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_trace<false, false, false>, kTraceBlock, dyn_lds);
	return e == hipSuccess ? nb : 0;
}

int yafamd_path_blocks_per_cu(const DevScene *S, int stack_depth)
{
	int nb = 0;
#ifdef YAF_EXPERIMENTS
	if(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_path<false>, kTraceBlock, pathLdsBytes(*S, stack_depth)) != hipSuccess) nb = 0;
#else
	(void)S; (void)stack_depth;
#endif
	return nb;
}

int yafamd_nee_blocks_per_cu()
{
	int nb = 0;
	if(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_nee<true, false>), kShadeBlock, 8192) != hipSuccess) nb = 0;
	return nb;
}

int yafamd_shade_blocks_per_cu()
{
	int nb = 0;
	if(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_shade<true, false>), kShadeBlock, 8192) != hipSuccess) nb = 0;
	return nb;
}

hipError_t yafamd_launch_camera(const DevScene *S, const DevPaths *P, const DevQueues *Q, const DevCounters *cnt,
                                const DevJob *jobs, int n_jobs, uint64_t chunk_base, int n, hipStream_t st)
{
	if(n <= 0) return hipSuccess;
	const int threads = max(n, (int)S->n_seg);   // the first n_seg threads also write the segment counts
	hipLaunchKernelGGL(k_camera, dim3((threads + 255) / 256), dim3(256), 0, st, *S, *P, *Q, *cnt, jobs, n_jobs, chunk_base, n);
	return hipGetLastError();
}

hipError_t yafamd_launch_trace(const DevScene *S, const DevQueues *Q, const DevCounters *cnt, const DevPaths *P,
                               DevStats *stats, int stack_depth, int *spill, int grid, hipStream_t st)
{
	const size_t stack_bytes = (size_t)stack_depth * kTraceBlock * sizeof(int);
	const bool wide = S->node_f4 == 8;
	const size_t lds_scene = S->scene_in_lds ? (size_t)(S->node_f4 * S->n_nodes + 3 * S->n_tris) * sizeof(float4)
	                                         : (wide ? (size_t)S->lds_top * kTopStride * sizeof(float4) : 0);
	const size_t bytes = stack_bytes + lds_scene;
	if(S->nodes8 && !S->scene_in_lds && !S->tr_shad)
	{
		// the BVH8 refill loop (global-memory scenes; its top treelet instead of the BVH4's)
		const size_t bytes8 = stack_bytes + (size_t)S->lds_top8 * kTop8Stride * sizeof(float4);
		if(S->trace_stats)
			hipLaunchKernelGGL((k_trace<false, true, false, true, true, false, true>), dim3(grid), dim3(kTraceBlock), bytes8, st, *S, *Q, *cnt, *P, stats,
			                   stack_depth, spill);
		else
			hipLaunchKernelGGL((k_trace<false, true, false, true, false, false, true>), dim3(grid), dim3(kTraceBlock), bytes8, st, *S, *Q, *cnt, *P, stats,
			                   stack_depth, spill);
		return hipGetLastError();
	}
#ifdef YAF_EXPERIMENTS
	if(S->brute && !S->tr_shad && S->n_tris <= kBruteTris)
	{
		hipLaunchKernelGGL(k_trace_brute, dim3(grid), dim3(kTraceBlock), 0, st, *S, *Q, *cnt, *P, stats);
		return hipGetLastError();
	}
#endif
#define YAF_TRACE_LAUNCH(L, W, T, SP) hipLaunchKernelGGL((k_trace<L, W, T, SP>), dim3(grid), dim3(kTraceBlock), bytes, st, *S, *Q, *cnt, *P, stats, stack_depth, spill)
	// no spill column: the LDS levels hold the whole stack bound (LDS-resident scenes)
	const bool nospill = spill == nullptr;
	if(S->tr_shad)
	{
		if(S->scene_in_lds)
		{
			if(nospill) { if(wide) YAF_TRACE_LAUNCH(true, true, true, false); else YAF_TRACE_LAUNCH(true, false, true, false); }
			else if(wide) YAF_TRACE_LAUNCH(true, true, true, true);
			else YAF_TRACE_LAUNCH(true, false, true, true);
		}
		else if(wide) YAF_TRACE_LAUNCH(false, true, true, true);
		else YAF_TRACE_LAUNCH(false, false, true, true);
	}
	else if(S->scene_in_lds)
	{
#ifdef YAF_EXPERIMENTS
		if(nospill && wide && S->ray_sort)
		{
			if(S->trace_stats)
				hipLaunchKernelGGL((k_trace<true, true, false, false, true, true>), dim3(grid), dim3(kTraceBlock), bytes, st, *S, *Q, *cnt, *P, stats,
				                   stack_depth, spill);
			else
				hipLaunchKernelGGL((k_trace<true, true, false, false, false, true>), dim3(grid), dim3(kTraceBlock), bytes, st, *S, *Q, *cnt, *P, stats,
				                   stack_depth, spill);
		}
		else
#endif
		if(nospill && wide && !S->trace_stats)
			hipLaunchKernelGGL((k_trace<true, true, false, false, false>), dim3(grid), dim3(kTraceBlock), bytes, st, *S, *Q, *cnt, *P, stats,
			                   stack_depth, spill);
		else if(nospill) { if(wide) YAF_TRACE_LAUNCH(true, true, false, false); else YAF_TRACE_LAUNCH(true, false, false, false); }
		else if(wide) YAF_TRACE_LAUNCH(true, true, false, true);
		else YAF_TRACE_LAUNCH(true, false, false, true);
	}
#ifdef YAF_EXPERIMENTS
	else if(wide && S->ray_sort)
	{
		if(S->trace_stats)
			hipLaunchKernelGGL((k_trace<false, true, false, true, true, true>), dim3(grid), dim3(kTraceBlock), bytes, st, *S, *Q, *cnt, *P, stats,
			                   stack_depth, spill);
		else
			hipLaunchKernelGGL((k_trace<false, true, false, true, false, true>), dim3(grid), dim3(kTraceBlock), bytes, st, *S, *Q, *cnt, *P, stats,
			                   stack_depth, spill);
	}
#endif
	else if(wide && !S->trace_stats)
		hipLaunchKernelGGL((k_trace<false, true, false, true, false>), dim3(grid), dim3(kTraceBlock), bytes, st, *S, *Q, *cnt, *P, stats,
		                   stack_depth, spill);
	else if(wide) YAF_TRACE_LAUNCH(false, true, false, true);
	else YAF_TRACE_LAUNCH(false, false, false, true);
#undef YAF_TRACE_LAUNCH
	return hipGetLastError();
}

hipError_t yafamd_launch_shade(const DevScene *S, const DevPaths *Pc, const DevPaths *Pn, const DevQueues *Q,
                               const DevQueues *Qn, const DevNeeQueue *N, const DevNeeQueue *G, const DevCounters *cnt,
                               const DevCounters *cnt_next, float4 *samples, const DevJob *jobs, int n_jobs, uint64_t chunk_base,
                               hipStream_t st)
{
	ShadeArgs A;
	A.S = *S;
	A.Pc = *Pc;
	A.Pn = *Pn;
	A.Q = *Q;
	A.Qn = *Qn;
	A.N = *N;
	A.G = *G;
	A.cnt = *cnt;
	A.cnt_next = *cnt_next;
	A.samples = samples;
	A.jobs = jobs;
	A.n_jobs = n_jobs;
	A.chunk_base = chunk_base;
	const size_t lds = shadeLdsBytes(*S, S->small_tables != 0);
	if(S->lpc_mode == 3)
	{
		// the deferred light pick's path pass (yafamd_dfr_eligible scenes only)
		if(S->ext || S->tree || S->gather_on) return hipErrorInvalidValue;
		const bool lean = S->integrator == INT_PATH && S->path_samples <= 1 && !S->do_ao && !S->caus_map && !S->show_map && S->n_photons == 0 &&
		                  !S->has_attr && !S->no_lean;
		if(lean) { if(S->small_tables) hipLaunchKernelGGL((k_shade<true, false, false, true, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
		           else hipLaunchKernelGGL((k_shade<false, false, false, true, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A); }
		else if(S->small_tables) hipLaunchKernelGGL((k_shade<true, false, false, false, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
		else hipLaunchKernelGGL((k_shade<false, false, false, false, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
		return hipGetLastError();
	}
	if(S->ext)
	{
		if(S->small_tables) hipLaunchKernelGGL((k_shade<true, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
		else hipLaunchKernelGGL((k_shade<false, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	}
	else if(!kShadeFused && S->integrator == INT_PATH && S->path_samples <= 1 && !S->do_ao && !S->caus_map && !S->gather_on && !S->show_map &&
	        S->n_photons == 0 && !S->tree && !S->has_attr && !S->no_lean)
	{
		if(yafamd_shade_fused_for(S))
		{
			if(S->small_tables) hipLaunchKernelGGL((k_shade<true, false, true, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
			else hipLaunchKernelGGL((k_shade<false, false, true, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
		}
		else if(S->small_tables) hipLaunchKernelGGL((k_shade<true, false, false, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
		else hipLaunchKernelGGL((k_shade<false, false, false, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	}
	else if(S->small_tables) hipLaunchKernelGGL((k_shade<true, false, kShadeFused>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	else hipLaunchKernelGGL((k_shade<false, false, kShadeFused>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	return hipGetLastError();
}

// the deferred light pick serves this scene: the plain path tracer (compact records, no recursion tree, photon
// estimates, surface attributes or transparent shadows); YAFARAY_AMD_LIGHT_PICK=count keeps the count run
int yafamd_dfr_eligible(const DevScene *S)
{
	if(S->n_lights > kDfrMaxLights) return 0;
	if(S->integrator != INT_PATH || S->ext || S->tree || S->gather_on || S->tr_shad || S->has_attr || S->caus_map || S->do_ao) return 0;
	const char *e = getenv("YAFARAY_AMD_LIGHT_PICK");
	return (e && std::string(e) == "count") ? 0 : 1;
}

hipError_t yafamd_dfr_segoff(const DevCounters *cnt, uint32_t n_seg, uint32_t *seg_off, uint32_t *dfr_total, uint32_t cap, uint32_t *overflow,
                             uint32_t *it_start, hipStream_t st)
{
	hipLaunchKernelGGL(k_dfr_segoff, dim3(1), dim3(1024), 0, st, cnt->n_active, n_seg, seg_off, dfr_total, cap, overflow, it_start);
	return hipGetLastError();
}

// one batch of records [r0, r0 + n_seg * cap_a): light pick + estimate (shadow rays to Q), the caller traces them, then connect
hipError_t yafamd_dfr_nee(const DevScene *S, const DevPaths *P, const DevQueues *Q, const DevCounters *cnt, uint32_t r0, uint32_t total, uint32_t *idx,
                         uint32_t *n_rec, hipStream_t st)
{
	if(S->n_lights > kDfrMaxLights) return hipErrorInvalidValue;
	DfrArgs A{};
	A.S = *S;
	A.P = *P;
	A.Q = *Q;
	A.cnt = *cnt;
	A.r0 = r0;
	A.total = total;
	A.idx = idx;
	A.n_rec = n_rec;
	hipLaunchKernelGGL(k_dfr_part, dim3(S->n_seg), dim3(1024), 0, st, A);
	const size_t lds = shadeLdsBytes(*S, S->small_tables != 0);
	const bool lean = !S->has_mesh_light;
	if(S->small_tables) { if(lean) hipLaunchKernelGGL((k_dfr_nee<true, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	                      else hipLaunchKernelGGL((k_dfr_nee<true, false>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A); }
	else if(lean) hipLaunchKernelGGL((k_dfr_nee<false, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	else hipLaunchKernelGGL((k_dfr_nee<false, false>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	return hipGetLastError();
}

hipError_t yafamd_dfr_accum(const DevScene *S, const DevPaths *P, uint32_t r0, uint32_t r1, uint32_t batch0, float4 *pcol, hipStream_t st)
{
	if(r1 <= r0) return hipSuccess;
	DfrArgs A{};
	A.S = *S;
	A.P = *P;
	A.r0 = r0;
	A.total = r1;
	hipLaunchKernelGGL(k_dfr_accum, dim3((r1 - r0 + 255) / 256), dim3(256), 0, st, A, pcol, batch0);
	return hipGetLastError();
}

hipError_t yafamd_dfr_fold(const DevScene *S, float4 *samples, uint32_t n_ctr, const float4 *pcol, hipStream_t st)
{
	if(n_ctr == 0) return hipSuccess;
	DfrArgs A{};
	A.S = *S;
	A.samples = samples;
	A.n_ctr = n_ctr;
	hipLaunchKernelGGL(k_dfr_fold, dim3((n_ctr + 255) / 256), dim3(256), 0, st, A, pcol);
	return hipGetLastError();
}

hipError_t yafamd_launch_spawn(const DevScene *S, const DevPaths *P, const DevQueues *Q, const DevCounters *cnt, uint32_t s0, int n,
                               hipStream_t st)
{
	const int grid = ((n > (int)S->n_seg ? n : (int)S->n_seg) + 255) / 256;
	hipLaunchKernelGGL(k_spawn, dim3(grid), dim3(256), 0, st, *S, *P, *Q, *cnt, s0, n);
	return hipGetLastError();
}

hipError_t yafamd_launch_combine(const DevScene *S, uint32_t lo, uint32_t hi, int final_level, float4 *samples, const DevJob *jobs,
                                 int n_jobs, uint64_t chunk_base, hipStream_t st)
{
	if(hi <= lo) return hipSuccess;
	hipLaunchKernelGGL(k_combine, dim3((hi - lo + 255) / 256), dim3(256), 0, st, *S, lo, hi, final_level, samples, jobs, n_jobs, chunk_base);
	return hipGetLastError();
}

hipError_t yafamd_launch_surface(const DevScene *S, const DevQueues *Q, const DevCounters *cnt, hipStream_t st)
{
	hipLaunchKernelGGL(k_surface, dim3(S->n_seg), dim3(kShadeBlock), 0, st, *S, *Q, *cnt);
	return hipGetLastError();
}

hipError_t yafamd_launch_tshadow(const DevScene *S, const DevQueues *Q, const DevCounters *cnt, const DevPaths *P, hipStream_t st)
{
	hipLaunchKernelGGL(k_tshadow, dim3(S->n_seg), dim3(kShadeBlock), 0, st, *S, *Q, *cnt, *P);
	return hipGetLastError();
}

// k_path (megakernel) for one chunk of n samples; `next` = a zeroed device counter.  Returns
// hipErrorInvalidValue when the scene is not eligible (yafamd_path_eligible).
int yafamd_path_eligible(const DevScene *S, int stack_depth, int spill)
{
	return (kExperiments && !S->ext && !S->tree && !S->tr_shad && !S->has_attr && !S->do_ao && !S->gather_on && !S->caus_map && S->integrator != INT_PHOTON &&
	        S->scene_in_lds && S->node_f4 == 8 && !spill && S->small_tables && S->nee_k >= 1 && S->nee_k <= kPathMaxK && !S->brute &&
	        pathLdsBytes(*S, stack_depth) <= 64 * 1024)
	           ? 1
	           : 0;
}

hipError_t yafamd_launch_path(const DevScene *S, float4 *samples, const DevJob *jobs, int n_jobs, uint64_t chunk_base, uint32_t n,
                              uint32_t *next, int stack_depth, int grid, hipStream_t st)
{
	if(!yafamd_path_eligible(S, stack_depth, 0)) return hipErrorInvalidValue;
	if(n == 0) return hipSuccess;
	PathArgs A;
	A.S = *S;
	A.samples = samples;
	A.jobs = jobs;
	A.n_jobs = n_jobs;
	A.chunk_base = chunk_base;
	A.n = n;
	A.next = next;
	A.stack_depth = stack_depth;
#ifdef YAF_EXPERIMENTS
	const size_t lds = pathLdsBytes(*S, stack_depth);
	if(S->trace_stats) hipLaunchKernelGGL(k_path<true>, dim3(grid), dim3(kTraceBlock), lds, st, A);
	else hipLaunchKernelGGL(k_path<false>, dim3(grid), dim3(kTraceBlock), lds, st, A);
	return hipGetLastError();
#else
	(void)grid; (void)st;
	return hipErrorInvalidValue;
#endif
}

// k_nee traces its shadow rays in place (TR) for non-EXT LDS-resident BVH4 scenes whose stack bound
// fits LDS, without transparent shadows (their filter colours need k_tshadow's lists)
int yafamd_nee_trace_eligible(const DevScene *S, int stack_depth)
{
	return (kExperiments && !S->ext && !S->tr_shad && !S->has_attr && S->scene_in_lds && S->node_f4 == 8 && S->small_tables && S->nee_k >= 1 &&
	        S->nee_k <= kPathMaxK && !S->brute && neeTraceLdsBytes(*S, stack_depth) <= 64 * 1024)
	           ? 1
	           : 0;
}

hipError_t yafamd_launch_nee(const DevScene *S, const DevNeeQueue *N, const DevPaths *Pn, const DevQueues *Qn,
                             const DevCounters *cnt_next, int stack_depth, hipStream_t st)
{
	NeeArgs A;
	A.S = *S;
	A.N = *N;
	A.Pn = *Pn;
	A.Qn = *Qn;
	A.cnt_next = *cnt_next;
	const size_t lds = shadeLdsBytes(*S, S->small_tables != 0);
	A.stack_depth = stack_depth;
#ifdef YAF_EXPERIMENTS
	if(stack_depth > 0 && yafamd_nee_trace_eligible(S, stack_depth))
	{
		if(S->trace_stats) hipLaunchKernelGGL((k_nee<true, false, true, true>), dim3(S->n_seg), dim3(kShadeBlock), neeTraceLdsBytes(*S, stack_depth), st, A);
		else hipLaunchKernelGGL((k_nee<true, false, true>), dim3(S->n_seg), dim3(kShadeBlock), neeTraceLdsBytes(*S, stack_depth), st, A);
		return hipGetLastError();
	}
#endif
	if(S->ext)
	{
		if(S->small_tables) hipLaunchKernelGGL((k_nee<true, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
		else hipLaunchKernelGGL((k_nee<false, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	}
	else if(!S->do_ao && !S->tr_shad && !S->has_mesh_light && !S->no_lean)
	{
		if(S->small_tables) hipLaunchKernelGGL((k_nee<true, false, false, false, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
		else hipLaunchKernelGGL((k_nee<false, false, false, false, true>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	}
	else if(S->small_tables) hipLaunchKernelGGL((k_nee<true, false>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	else hipLaunchKernelGGL((k_nee<false, false>), dim3(S->n_seg), dim3(kShadeBlock), lds, st, A);
	return hipGetLastError();
}

// photon ids [h0, h0 + n_local) of a map of n_photons paths
hipError_t yafamd_photon_emit(const DevScene *S, const PhotonState *P, const PhotonSet *L, uint32_t n_photons, uint32_t h0, uint32_t n_local,
                              int max_bounces, hipStream_t st)
{
	PhotonArgs A;
	A.S = *S;
	A.P = *P;
	A.L = *L;
	A.n_photons = n_photons;
	A.h0 = h0;
	A.n_local = n_local;
	A.max_bounces = max_bounces;
	A.bounce = 0;
	A.cur = 0;
	A.stack_depth = 0;
	A.spill = nullptr;
	if(n_local == 0) return hipSuccess;
	hipLaunchKernelGGL(k_photon_emit, dim3((n_local + 255) / 256), dim3(256), 0, st, A);
	return hipGetLastError();
}

hipError_t yafamd_photon_bounce(const DevScene *S, const PhotonState *P, const PhotonSet *L, uint32_t n_photons, uint32_t h0,
                                uint32_t n_local, int max_bounces, int bounce, int cur, int stack_depth, int *spill, int grid, hipStream_t st)
{
	PhotonArgs A;
	A.S = *S;
	A.P = *P;
	A.L = *L;
	A.n_photons = n_photons;
	A.h0 = h0;
	A.n_local = n_local;
	A.max_bounces = max_bounces;
	A.bounce = bounce;
	A.cur = cur;
	A.stack_depth = stack_depth;
	A.spill = spill;
	if((uint32_t)grid != P->n_segs) return hipErrorInvalidValue;   // one workgroup per alive-list segment
	const size_t stack_bytes = (size_t)stack_depth * kTraceBlock * sizeof(int);
	if(S->scene_in_lds)
	{
		const size_t bytes = stack_bytes + (size_t)(S->node_f4 * S->n_nodes + 3 * S->n_tris) * sizeof(float4);
		const bool ns = spill == nullptr;   // no spill column: plain LDS stack
		if(S->ext)
		{
			if(S->node_f4 == 8)
			{
				if(ns) hipLaunchKernelGGL((k_photon_bounce<true, true, true, false>), dim3(grid), dim3(kTraceBlock), bytes, st, A);
				else hipLaunchKernelGGL((k_photon_bounce<true, true, true>), dim3(grid), dim3(kTraceBlock), bytes, st, A);
			}
			else hipLaunchKernelGGL((k_photon_bounce<true, false, true>), dim3(grid), dim3(kTraceBlock), bytes, st, A);
		}
		else if(S->node_f4 == 8)
		{
			if(ns) hipLaunchKernelGGL((k_photon_bounce<true, true, false, false>), dim3(grid), dim3(kTraceBlock), bytes, st, A);
			else hipLaunchKernelGGL((k_photon_bounce<true, true, false>), dim3(grid), dim3(kTraceBlock), bytes, st, A);
		}
		else hipLaunchKernelGGL((k_photon_bounce<true, false, false>), dim3(grid), dim3(kTraceBlock), bytes, st, A);
	}
	else if(S->ext)
	{
		if(S->node_f4 == 8) hipLaunchKernelGGL((k_photon_bounce<false, true, true>), dim3(grid), dim3(kTraceBlock), stack_bytes, st, A);
		else hipLaunchKernelGGL((k_photon_bounce<false, false, true>), dim3(grid), dim3(kTraceBlock), stack_bytes, st, A);
	}
	else if(S->node_f4 == 8) hipLaunchKernelGGL((k_photon_bounce<false, true, false>), dim3(grid), dim3(kTraceBlock), stack_bytes, st, A);
	else hipLaunchKernelGGL((k_photon_bounce<false, false, false>), dim3(grid), dim3(kTraceBlock), stack_bytes, st, A);
	return hipGetLastError();
}

// Stable compaction of the deposit slots into the photon map; *total_dev receives the count.
// (scratch_counts: one count per 1024 local ids)
hipError_t yafamd_photon_compact(const PhotonState *P, uint32_t *scratch_counts, uint32_t *total_dev, float4 *pos, float4 *dir, float *colb,
                                 hipStream_t st)
{
	const uint32_t nb = (P->n_local + 1023u) / 1024u;
	if(nb == 0) return hipSuccess;
	hipLaunchKernelGGL(k_photon_count, dim3(nb), dim3(256), 0, st, P->dep_flag, P->n_local, P->n_slot_rows, scratch_counts);
	hipLaunchKernelGGL(k_photon_scan, dim3(1), dim3(1024), 0, st, scratch_counts, nb, total_dev);
	hipLaunchKernelGGL(k_photon_scatter, dim3(nb), dim3(1024), 0, st, *P, (const uint32_t *)scratch_counts, pos, dir, colb);
	return hipGetLastError();
}

hipError_t yafamd_launch_gather(const DevScene *S, const DevNeeQueue *G, const DevCounters *cnt_next, float4 *samples,
                                const DevJob *jobs, int n_jobs, uint64_t chunk_base, const GatherLogDesc *log, hipStream_t st)
{
	GatherArgs A;
	A.S = *S;
	A.G = *G;
	A.cnt_next = *cnt_next;
	A.samples = samples;
	A.jobs = jobs;
	A.n_jobs = n_jobs;
	A.chunk_base = chunk_base;
	A.log = GatherLog{nullptr, nullptr, 0u, 0u, 0u};
	const bool replay = log != nullptr;
	if(replay) A.log = GatherLog{(uint2 *)log->e, log->n, log->cap, log->seg_cap, log->j0};
	const dim3 grid(S->n_seg * kGatherPerSeg);
#ifdef YAF_GATHER_NO_SMALL
	const bool small = false;
#else
	const bool small = S->small_tables != 0;
#endif
	// the split heap: a replay without a caustic map (its lookups need photon indices in the heap)
	const bool split = replay && log->split && !S->caus_map && log->cap <= 65536u && !YAF_GATHER_STACK_LDS;
	const size_t lds = gatherTableBytes(*S, small) +
	                   (split ? (size_t)kGatherBlock * 6u * (size_t)gatherHeapSlots(*S) : gatherLdsBytes(*S));
#define YAF_GATHER_LAUNCH(SM, E) \
	do { if(split) hipLaunchKernelGGL((k_gather<SM, E, true, true>), grid, dim3(kGatherBlock), lds, st, A); \
	     else if(replay) hipLaunchKernelGGL((k_gather<SM, E, true>), grid, dim3(kGatherBlock), lds, st, A); \
	     else hipLaunchKernelGGL((k_gather<SM, E, false>), grid, dim3(kGatherBlock), lds, st, A); } while(0)
	if(S->ext)
	{
		if(small) YAF_GATHER_LAUNCH(true, true);
		else YAF_GATHER_LAUNCH(false, true);
	}
	else if(small) YAF_GATHER_LAUNCH(true, false);
	else YAF_GATHER_LAUNCH(false, false);
#undef YAF_GATHER_LAUNCH
	return hipGetLastError();
}

// pass 1 of the two-pass diffuse gather over one batch (see k_gather_walk)
hipError_t yafamd_launch_gather_walk(const DevScene *S, const DevNeeQueue *G, const DevCounters *cnt_next, const GatherLogDesc *log,
                                     hipStream_t st)
{
	// the walk with the k smallest distances in registers (k <= kWalkK), else the bounded walk
	const bool exact = log->exact && S->pm_search <= kWalkK;
	if((log->seg_cap & 63u) || (log->cap & 1u) || S->pm_search < 1) return hipErrorInvalidValue;
	GatherArgs A;
	A.S = *S;
	A.G = *G;
	A.cnt_next = *cnt_next;
	A.samples = nullptr;
	A.jobs = nullptr;
	A.n_jobs = 0;
	A.chunk_base = 0;
	A.log = GatherLog{(uint2 *)log->e, log->n, log->cap, log->seg_cap, log->j0, log->spill};
	if(exact && walkLdsLevels(S->pm_stack) < max(1, S->pm_stack) && !log->spill) return hipErrorInvalidValue;
	const size_t lds = walkLdsBytes(S->pm_stack, !exact);
	if(exact) hipLaunchKernelGGL(k_gather_walk<false>, dim3(S->n_seg * kWalkPerSeg), dim3(kGatherBlock), lds, st, A);
#ifdef YAF_EXPERIMENTS
	else hipLaunchKernelGGL(k_gather_walk<true>, dim3(S->n_seg * kWalkPerSeg), dim3(kGatherBlock), lds, st, A);
#else
	else return hipErrorInvalidValue;
#endif
	return hipGetLastError();
}

// k_gather_walk's stack column: levels kept in LDS and the walk grid's threads (render.cc sizes the spill)
int yafamd_walk_lds_levels(int pm_stack) { return walkLdsLevels(pm_stack); }
int yafamd_walk_threads(const DevScene *S) { return (int)(S->n_seg * kWalkPerSeg * kGatherBlock); }

// the largest k the two-pass gather serves: the register walk's k; experiments builds also the bounded
// walk (the split replay heap's 16-bit log positions bound it)
int yafamd_gather_walk_k() { return kExperiments ? 65535 : kWalkK; }

// Final gathering: compaction of the radiance points (reuses the photon count / scan kernels on
// rad_flag); *total_dev receives the count
hipError_t yafamd_rad_compact(const PhotonState *P, uint32_t *scratch_counts, uint32_t *total_dev, float4 *a, float4 *b, float4 *c, hipStream_t st)
{
	const uint32_t nb = (P->n_local + 1023u) / 1024u;
	if(nb == 0) return hipSuccess;
	hipLaunchKernelGGL(k_photon_count, dim3(nb), dim3(256), 0, st, P->rad_flag, P->n_local, P->n_slot_rows, scratch_counts);
	hipLaunchKernelGGL(k_photon_scan, dim3(1), dim3(1024), 0, st, scratch_counts, nb, total_dev);
	hipLaunchKernelGGL(k_rad_scatter, dim3(nb), dim3(1024), 0, st, *P, (const uint32_t *)scratch_counts, a, b, c);
	return hipGetLastError();
}

// k_rad_refl over the kept radiance points (scenes without EXT materials)
hipError_t yafamd_rad_refl(const DevScene *S, float4 *a, float4 *b, float4 *c, const uint32_t *kept, uint32_t n, hipStream_t st)
{
	if(n == 0 || S->ext) return hipSuccess;
	hipLaunchKernelGGL(k_rad_refl, dim3((n + 255) / 256), dim3(256), 0, st, *S, a, b, c, kept, n);
	return hipGetLastError();
}

// preGatherWorker over the kept radiance points (n of them, indices `kept` into the compacted
// arrays); the grid is the gather grid, whose lanes the HBM lookup stack (S->pk_stack) is sized for
hipError_t yafamd_pregather(const DevScene *S, const float4 *a, const float4 *b, const float4 *c, const uint32_t *kept, uint32_t n,
                            float4 *out_pos, float4 *out_dir, float *out_colb, DevStats *stats, hipStream_t st)
{
	if(n == 0) return hipSuccess;
	PreGatherArgs A;
	A.S = *S;
	A.rad_a = a;
	A.rad_b = b;
	A.rad_c = c;
	A.kept = kept;
	A.n = n;
	A.out_pos = out_pos;
	A.out_dir = out_dir;
	A.out_colb = out_colb;
	A.stats = stats;
	const size_t lds = (size_t)kGatherBlock * 8u * (size_t)max(1, S->pm_search);
	hipLaunchKernelGGL(k_pregather, dim3(S->n_seg * kGatherPerSeg), dim3(kGatherBlock), lds, st, A);
	return hipGetLastError();
}

// k_fg over the gather queue of one iteration (before k_gather), on the trace grid
hipError_t yafamd_launch_fg(const DevScene *S, const DevNeeQueue *G, const DevCounters *cnt_next, int stack_depth, int *spill, int grid,
                            float2 *ts_scratch, hipStream_t st)
{
	FgArgs A;
	A.S = *S;
	A.G = *G;
	A.cnt_next = *cnt_next;
	A.stack_depth = stack_depth;
	A.spill = spill;
	A.ts_scratch = ts_scratch;
	// (+ the nearest-search column: S->rpk_lds levels of 4 B per lane, after the stack and scene)
	const size_t stack_bytes = (size_t)stack_depth * kTraceBlock * sizeof(int);
	const size_t nstk_bytes = (size_t)S->rpk_lds * kTraceBlock * sizeof(uint32_t);
	const bool wide = S->node_f4 == 8;
	// an LDS-resident scene: the column rounded to 16 B, then the staged tables (fgStageTables)
	const size_t stage_bytes = fgStageTables(*S, S->scene_in_lds != 0, S->ext != 0, stack_depth)
	                               ? ((nstk_bytes + 15) & ~(size_t)15) + (size_t)S->n_mats * sizeof(DevMaterial) + (size_t)S->n_tris * 16
	                               : nstk_bytes;
	if(S->tr_shad)
	{
		// transparent shadows (the spilling variants: without a spill column they never spill)
		if(!ts_scratch) return hipErrorInvalidValue;
		const size_t bytes = (S->scene_in_lds ? stack_bytes + (size_t)(S->node_f4 * S->n_nodes + 3 * S->n_tris) * sizeof(float4) : stack_bytes) +
		                     (S->scene_in_lds ? stage_bytes : nstk_bytes);
#define YAF_FG_LAUNCH_TS(L, W, E) hipLaunchKernelGGL((k_fg<L, W, E, true, true>), dim3(grid), dim3(kTraceBlock), bytes, st, A)
		if(S->scene_in_lds)
		{
			if(S->ext) { if(wide) YAF_FG_LAUNCH_TS(true, true, true); else YAF_FG_LAUNCH_TS(true, false, true); }
			else if(wide) YAF_FG_LAUNCH_TS(true, true, false);
			else YAF_FG_LAUNCH_TS(true, false, false);
		}
		else if(S->ext) { if(wide) YAF_FG_LAUNCH_TS(false, true, true); else YAF_FG_LAUNCH_TS(false, false, true); }
		else if(wide) YAF_FG_LAUNCH_TS(false, true, false);
		else YAF_FG_LAUNCH_TS(false, false, false);
#undef YAF_FG_LAUNCH_TS
		return hipGetLastError();
	}
#define YAF_FG_LAUNCH(L, W, E, B) hipLaunchKernelGGL((k_fg<L, W, E>), dim3(grid), dim3(kTraceBlock), B, st, A)
#define YAF_FG_LAUNCH_NS(W, E, B) hipLaunchKernelGGL((k_fg<true, W, E, false>), dim3(grid), dim3(kTraceBlock), B, st, A)
	if(S->scene_in_lds)
	{
		const size_t bytes = stack_bytes + (size_t)(S->node_f4 * S->n_nodes + 3 * S->n_tris) * sizeof(float4) + stage_bytes;
		if(spill == nullptr)   // the LDS levels hold the whole stack bound: plain LDS pushes / pops
		{
			if(S->ext) { if(wide) YAF_FG_LAUNCH_NS(true, true, bytes); else YAF_FG_LAUNCH_NS(false, true, bytes); }
			else if(wide) YAF_FG_LAUNCH_NS(true, false, bytes);
			else YAF_FG_LAUNCH_NS(false, false, bytes);
		}
		else if(S->ext) { if(wide) YAF_FG_LAUNCH(true, true, true, bytes); else YAF_FG_LAUNCH(true, false, true, bytes); }
		else if(wide) YAF_FG_LAUNCH(true, true, false, bytes);
		else YAF_FG_LAUNCH(true, false, false, bytes);
	}
	else if(S->ext) { if(wide) YAF_FG_LAUNCH(false, true, true, stack_bytes + nstk_bytes); else YAF_FG_LAUNCH(false, false, true, stack_bytes + nstk_bytes); }
	else if(wide) YAF_FG_LAUNCH(false, true, false, stack_bytes + nstk_bytes);
	else YAF_FG_LAUNCH(false, false, false, stack_bytes + nstk_bytes);
#undef YAF_FG_LAUNCH
#undef YAF_FG_LAUNCH_NS
	return hipGetLastError();
}

// the per-path final gathering (k_fg_first / k_fg_long / k_fg_sum) serves this scene: LDS-resident scenes
// without transparent shadows (k_fg keeps the others); YAFARAY_AMD_FG=lane forces k_fg (tests, A/B)
int yafamd_fg_paths_eligible(const DevScene *S)
{
	if(!S->scene_in_lds || S->tr_shad) return 0;
	const char *e = getenv("YAFARAY_AMD_FG");
	return (e && std::string(e) == "lane") ? 0 : 1;
}

// one batch of the per-path final gathering: the caller zeroed B->long_count (n_seg words)
hipError_t yafamd_launch_fg_paths(const DevScene *S, const DevNeeQueue *G, const DevCounters *cnt_next, int stack_depth, int *spill, int grid,
                                  const FgBatch *B, hipStream_t st)
{
	if(!yafamd_fg_paths_eligible(S)) return hipErrorInvalidValue;
	FgPathArgs PA;
	PA.A.S = *S;
	PA.A.G = *G;
	PA.A.cnt_next = *cnt_next;
	PA.A.stack_depth = stack_depth;
	PA.A.spill = spill;
	PA.A.ts_scratch = nullptr;
	PA.B = *B;
	// with the radiance-map grid the kd search only settles ties (rare): its private-array stack, no LDS
	// column (more resident workgroups)
	if(S->rgrid.start) PA.A.S.rpk_lds = 0;
	const size_t stack_bytes = (size_t)stack_depth * kTraceBlock * sizeof(int);
	const size_t nstk_bytes = (size_t)PA.A.S.rpk_lds * kTraceBlock * sizeof(uint32_t);
	const size_t stage_bytes = fgStageTables(PA.A.S, true, S->ext != 0, stack_depth)
	                               ? ((nstk_bytes + 15) & ~(size_t)15) + (size_t)S->n_mats * sizeof(DevMaterial) + (size_t)S->n_tris * 16
	                               : nstk_bytes;
	const size_t bytes = stack_bytes + (size_t)(S->node_f4 * S->n_nodes + 3 * S->n_tris) * sizeof(float4) + stage_bytes;
	const bool wide = S->node_f4 == 8, ext = S->ext != 0, sp = spill != nullptr;
#define YAF_FGP(W, E, SP)                                                                                                      \
	do                                                                                                                         \
	{                                                                                                                          \
		hipLaunchKernelGGL((k_fg_first<true, W, E, SP>), dim3(grid), dim3(kTraceBlock), bytes, st, PA);                       \
		hipLaunchKernelGGL((k_fg_long<true, W, E, SP, false>), dim3(grid), dim3(kTraceBlock), bytes, st, PA);                 \
	} while(0)
	if(wide) { if(ext) { if(sp) YAF_FGP(true, true, true); else YAF_FGP(true, true, false); } else { if(sp) YAF_FGP(true, false, true); else YAF_FGP(true, false, false); } }
	else { if(ext) { if(sp) YAF_FGP(false, true, true); else YAF_FGP(false, true, false); } else { if(sp) YAF_FGP(false, false, true); else YAF_FGP(false, false, false); } }
#undef YAF_FGP
	const uint32_t gx = min((B->seg_cap + 255u) / 256u, 64u);
	hipLaunchKernelGGL(k_fg_sum, dim3(gx, S->n_seg), dim3(256), 0, st, PA);
	return hipGetLastError();
}

// lanes of one gather launch (the HBM lookup stack holds pm_stack levels per lane)
size_t yafamd_gather_lanes(const DevScene *S) { return (size_t)S->n_seg * (kWalkPerSeg > kGatherPerSeg ? kWalkPerSeg : kGatherPerSeg) * kGatherBlock; }

size_t yafamd_gather_lds_bytes(const DevScene *S) { return gatherTableBytes(*S, S->small_tables != 0) + gatherLdsBytes(*S); }

hipError_t yafamd_launch_done_flags(const DevScene *S, const DevJob *jobs, int n_jobs, uint32_t n_pix, uint32_t done_pix, uint8_t *flags,
                                    hipStream_t st)
{
	if(n_pix == 0) return hipSuccess;
	hipLaunchKernelGGL(k_done_flags, dim3((n_pix + 255) / 256), dim3(256), 0, st, *S, jobs, n_jobs, n_pix, done_pix, flags);
	return hipGetLastError();
}

hipError_t yafamd_lpc_seg(const uint32_t *lpc, int W, int spp, int ts, int y0, int y1, uint32_t *seg, hipStream_t st)
{
	const int n = (y1 - y0) * ((W + ts - 1) / ts);
	if(n <= 0) return hipSuccess;
	hipLaunchKernelGGL(k_lpc_seg, dim3((n + 3) / 4), dim3(256), 0, st, lpc, W, spp, ts, y0, y1, seg);
	return hipGetLastError();
}

hipError_t yafamd_lpc_prefix(uint32_t *lpc, int W, int spp, int ts, int y0, int y1, const uint32_t *segbase, hipStream_t st)
{
	const int n = (y1 - y0) * ((W + ts - 1) / ts);
	if(n <= 0) return hipSuccess;
	hipLaunchKernelGGL(k_lpc_prefix, dim3((n + 3) / 4), dim3(256), 0, st, lpc, W, spp, ts, y0, y1, segbase);
	return hipGetLastError();
}

hipError_t yafamd_launch_film(const DevFilm *F, const float4 *samples, const uint8_t *flags, float4 *accum, float4 *out,
                              float *weights, int y0, int y1, float clamp_samples, int accumulate, hipStream_t st)
{
	if(y1 <= y0) return hipSuccess;
	const dim3 grid((F->width + 255) / 256, y1 - y0);
	if(F->reach_fwd == 1 && F->reach_back == 0)
		hipLaunchKernelGGL((k_film<1, 0>), grid, dim3(256), 0, st, *F, samples, flags, accum, out, weights, y0, y1, clamp_samples, accumulate);
	else
		hipLaunchKernelGGL((k_film<-1, -1>), grid, dim3(256), 0, st, *F, samples, flags, accum, out, weights, y0, y1, clamp_samples,
		                   accumulate);
	return hipGetLastError();
}

hipError_t yafamd_launch_trace_rays(const DevScene *S, int any, const float4 *ro, const float4 *rd, int n, float *t_out,
                                    int *prim_out, int stack_depth, hipStream_t st)
{
	if(n <= 0) return hipSuccess;
	const size_t stack_bytes = (size_t)stack_depth * kTraceBlock * sizeof(int);
	const dim3 grid((n + kTraceBlock - 1) / kTraceBlock);
	const bool wide = S->node_f4 == 8;
	if(any && wide) hipLaunchKernelGGL((k_trace_rays<true, true>), grid, dim3(kTraceBlock), stack_bytes, st, *S, ro, rd, n, t_out, prim_out, stack_depth);
	else if(any) hipLaunchKernelGGL((k_trace_rays<true, false>), grid, dim3(kTraceBlock), stack_bytes, st, *S, ro, rd, n, t_out, prim_out, stack_depth);
	else if(wide) hipLaunchKernelGGL((k_trace_rays<false, true>), grid, dim3(kTraceBlock), stack_bytes, st, *S, ro, rd, n, t_out, prim_out, stack_depth);
	else hipLaunchKernelGGL((k_trace_rays<false, false>), grid, dim3(kTraceBlock), stack_bytes, st, *S, ro, rd, n, t_out, prim_out, stack_depth);
	return hipGetLastError();
}

}
