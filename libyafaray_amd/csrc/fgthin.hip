// Final gathering's radiance-point thinning on the GPU (reference integrator_photon_mapping.cc:560-572).
//
// The reference walks the radiance points in shooting order; a point still in use is kept and, by a
// range lookup in a point kd-tree (EliminatePhoton, photon.h:172-180), marks every point within the
// squared distance maxrad (strictly less) whose normal faces the same side as unused — itself
// included.  The kept set is the lexicographically-first maximal independent set of the graph
// "within maxrad and normals on the same side" (the relation is symmetric bit for bit: (a - b)^2 =
// (b - a)^2 and the dot products commute), so it can be decided in rounds without the serial walk:
//
//   round r: an undecided point none of whose lower-index neighbours is undecided is kept (snapshot
//            of the states, two buffers); then every point kept in this round marks its higher-index
//            neighbours dead, as the reference's lookup from a kept point does
//
// The lowest undecided point is always kept, so the rounds end; in practice ~15 rounds decide
// millions of points (C5: 2.46 M points, 16 K kept).  Neighbours come from a dense uniform grid of cell > sqrt(maxrad) (counting sort by
// cell); the rounds work in cell order (positions, normals and states copied into the counting sort's
// order, so a cell's entries are read contiguously), and the kept indices are compacted in shooting
// order at the end.  Host twin: render.cc eliminateRadPoints.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "devscene.h"

namespace
{

struct ThinBuf
{
	void *p = nullptr;
	size_t bytes = 0;
	template<class T> T *as() { return reinterpret_cast<T *>(p); }
	hipError_t ensure(size_t b)
	{
		if(b < 16) b = 16;
		if(p && bytes >= b) return hipSuccess;
		if(p) (void)hipFree(p);
		p = nullptr;
		bytes = 0;
		const hipError_t e = hipMalloc(&p, b);
		if(e == hipSuccess) bytes = b;
		return e;
	}
};

// scratch kept between renders (the radiance map is rebuilt every frame); one per renderer
struct ThinScratch
{
	ThinBuf part, cid, count, start, order, st0, st1, counter, tmp, n_sel, klist, spos, snrm;
	~ThinScratch()
	{
		for(ThinBuf *b : {&part, &cid, &count, &start, &order, &st0, &st1, &counter, &tmp, &n_sel, &klist, &spos, &snrm})
			if(b->p) (void)hipFree(b->p);
	}
};

constexpr int kBoundBlocks = 256;
constexpr uint8_t kUndecided = 0, kKept = 1, kDead = 2;

struct ThinGrid
{
	double lo[3];
	double inv_cell;
	int nx, ny, nz;
};

__device__ __forceinline__ int axisCell(float v, double lo, double inv_cell, int na)
{
	const int c = (int)floor(((double)v - lo) * inv_cell);
	return c < 0 ? 0 : (c >= na ? na - 1 : c);
}

__global__ void __launch_bounds__(256) k_thin_bound(const float4 *pos, uint32_t n, float4 *part)
{
	float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
	for(uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
	{
		const float4 p = pos[i];
		lo[0] = fminf(lo[0], p.x); lo[1] = fminf(lo[1], p.y); lo[2] = fminf(lo[2], p.z);
		hi[0] = fmaxf(hi[0], p.x); hi[1] = fmaxf(hi[1], p.y); hi[2] = fmaxf(hi[2], p.z);
	}
	__shared__ float s[6][256];
	for(int a = 0; a < 3; ++a) { s[a][threadIdx.x] = lo[a]; s[3 + a][threadIdx.x] = hi[a]; }
	__syncthreads();
	for(int off = 128; off > 0; off >>= 1)
	{
		if((int)threadIdx.x < off)
			for(int a = 0; a < 3; ++a)
			{
				s[a][threadIdx.x] = fminf(s[a][threadIdx.x], s[a][threadIdx.x + off]);
				s[3 + a][threadIdx.x] = fmaxf(s[3 + a][threadIdx.x], s[3 + a][threadIdx.x + off]);
			}
		__syncthreads();
	}
	if(threadIdx.x == 0)
	{
		part[2 * blockIdx.x] = make_float4(s[0][0], s[1][0], s[2][0], 0.f);
		part[2 * blockIdx.x + 1] = make_float4(s[3][0], s[4][0], s[5][0], 0.f);
	}
}

__global__ void __launch_bounds__(256) k_thin_cells(const float4 *pos, uint32_t n, ThinGrid g, uint32_t *cid, uint32_t *count)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= n) return;
	const float4 p = pos[i];
	const int cx = axisCell(p.x, g.lo[0], g.inv_cell, g.nx), cy = axisCell(p.y, g.lo[1], g.inv_cell, g.ny),
	          cz = axisCell(p.z, g.lo[2], g.inv_cell, g.nz);
	const uint32_t c = (uint32_t)((cz * g.ny + cy) * g.nx + cx);
	cid[i] = c;
	atomicAdd(&count[c], 1u);
}

__global__ void __launch_bounds__(256) k_thin_fill(const uint32_t *cid, uint32_t n, const uint32_t *start, uint32_t *fill, uint32_t *order)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= n) return;
	const uint32_t c = cid[i];
	order[start[c] + atomicAdd(&fill[c], 1u)] = i;   // order inside a cell is irrelevant (marking is idempotent)
}

// the points in cell order: spos[k] / snrm[k] of point order[k]
__global__ void __launch_bounds__(256) k_thin_sort(const float4 *pos, const float4 *nrm, const uint32_t *order, uint32_t n, float4 *spos,
                                                  float4 *snrm)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if(k >= n) return;
	const uint32_t j = order[k];
	spos[k] = pos[j];
	snrm[k] = nrm[j];
}

// the final states back in shooting order
__global__ void __launch_bounds__(256) k_thin_unsort(const uint8_t *sst, const uint32_t *order, uint32_t n, uint8_t *st)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if(k < n) st[order[k]] = sst[k];
}

// neighbour cells of a point (clamped 3x3x3 block) — the relation's reach is < one cell per axis.  The
// point's own cell comes first (most likely to hold a related point, which ends the keep scan), then
// the other 26 in z, y, x order
#define THIN_FOR_CELLS(q)                                                                                      \
	const int cx_ = axisCell(q.x, g.lo[0], g.inv_cell, g.nx), cy_ = axisCell(q.y, g.lo[1], g.inv_cell, g.ny),   \
	          cz_ = axisCell(q.z, g.lo[2], g.inv_cell, g.nz);                                                    \
	for(int t_ = 0, u_ = 13; t_ < 27 && !stop; u_ = t_ < 13 ? t_ : t_ + 1, ++t_)                                 \
		if(const int z = cz_ + u_ / 9 - 1, y = cy_ + (u_ / 3) % 3 - 1, x = cx_ + u_ % 3 - 1;                      \
		   z >= 0 && z < g.nz && y >= 0 && y < g.ny && x >= 0 && x < g.nx)

// EliminatePhoton's test (pkdtree.h:263-268 strict distance, photon.h:177 normals on one side),
// symmetric bit for bit in the two points
__device__ __forceinline__ bool thinRelated(const float4 &p, const float4 &pn, const float4 &q, const float4 &qn, float maxrad)
{
	const float vx = p.x - q.x, vy = p.y - q.y, vz = p.z - q.z;
	const float d2 = vx * vx + vy * vy + vz * vz;
	const float nd = pn.x * qn.x + pn.y * qn.y + pn.z * qn.z;
	return d2 < maxrad && nd > 0.f;
}

// round, part 1: an undecided point none of whose lower-index related points is undecided (in the
// snapshot `sin`) is kept; the kept points of earlier rounds have already killed their related
// higher points (part 2), so the dead ones are skipped and the scan stops at the first undecided
// one.  kKeepLanes lanes per point split the entries of each cell (uniform trip counts inside a
// group, so every lane of the group sees its vote); one lane per point measured 2.7 ms per round.
// Everything is indexed by cell-order position p (the point's shooting index is order[p]; states,
// positions and normals are in cell order, so a group reads a cell's entries contiguously).
constexpr uint32_t kKeepLanes = 8;
__global__ void __launch_bounds__(256) k_thin_keep(const float4 *pos, const float4 *nrm, const uint32_t *order, const uint32_t *start,
                                                  ThinGrid g, const uint8_t *sin, uint8_t *sout, uint32_t n, float maxrad, uint32_t *klist,
                                                  uint32_t *n_klist)
{
	const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t p = tid / kKeepLanes, sub = tid % kKeepLanes;
	const uint64_t gmask = ((1ull << kKeepLanes) - 1ull) << (__lane_id() & ~(kKeepLanes - 1u));
	if(p >= n) return;   // whole groups leave together (n * kKeepLanes threads, groups aligned)
	const uint8_t s0 = sin[p];
	if(s0 != kUndecided)
	{
		if(sub == 0) sout[p] = s0;
		return;
	}
	const uint32_t i = order[p];
	const float4 q = pos[p], qn = nrm[p];
	bool stop = false;
	THIN_FOR_CELLS(q)
	{
		const uint32_t c = (uint32_t)((z * g.ny + y) * g.nx + x);
		const uint32_t k0 = start[c], k1 = start[c + 1];
		for(uint32_t base = k0; base < k1; base += kKeepLanes)
		{
			const uint32_t k = base + sub;
			bool hit = false;
			if(k < k1)
			{
				hit = sin[k] == kUndecided && order[k] < i && thinRelated(pos[k], nrm[k], q, qn, maxrad);
			}
			if(__ballot(hit) & gmask) { stop = true; break; }
		}
	}
	if(sub == 0)
	{
		sout[p] = stop ? kUndecided : kKept;
		// part 2 works on this list (its order is irrelevant: the kills are idempotent); one atomic per
		// wave on the list's single counter instead of one per kept point
		const uint64_t want = __ballot(!stop);
		if(want)
		{
			const uint32_t leader = (uint32_t)__ffsll((unsigned long long)want) - 1u;
			uint32_t base = 0;
			if(__lane_id() == leader) base = atomicAdd(n_klist, (uint32_t)__popcll(want));
			base = __shfl(base, (int)leader);
			if(!stop) klist[base + (uint32_t)__popcll(want & ((1ull << __lane_id()) - 1ull))] = p;
		}
	}
}

// round, part 2: every point kept in this round marks its related higher points dead (the
// reference's EliminatePhoton lookup from a kept point); none of them can have been kept in part 1
// (it saw this point undecided below it).  One wave per kept point: the lanes split the entries of
// its 27 cells (a lane per point measured 2.5 ms per round — a few thousand long serial scans)
__global__ void __launch_bounds__(256) k_thin_kill(const float4 *pos, const float4 *nrm, const uint32_t *order, const uint32_t *start,
                                                  ThinGrid g, uint8_t *sout, const uint32_t *klist, const uint32_t *n_klist, float maxrad)
{
	const uint32_t lane = __lane_id();
	const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_waves = (gridDim.x * blockDim.x) >> 6;
	const uint32_t nk = *n_klist;
	for(uint32_t t = wave; t < nk; t += n_waves)
	{
		const uint32_t p = klist[t], i = order[p];
		const float4 q = pos[p], qn = nrm[p];
		const int cx = axisCell(q.x, g.lo[0], g.inv_cell, g.nx), cy = axisCell(q.y, g.lo[1], g.inv_cell, g.ny),
		          cz = axisCell(q.z, g.lo[2], g.inv_cell, g.nz);
		for(int z = max(0, cz - 1); z <= min(g.nz - 1, cz + 1); ++z)
			for(int y = max(0, cy - 1); y <= min(g.ny - 1, cy + 1); ++y)
				for(int x = max(0, cx - 1); x <= min(g.nx - 1, cx + 1); ++x)
				{
					const uint32_t c = (uint32_t)((z * g.ny + y) * g.nx + x);
					const uint32_t k1 = start[c + 1];
					for(uint32_t k = start[c] + lane; k < k1; k += 64)
					{
						if(order[k] > i && thinRelated(pos[k], nrm[k], q, qn, maxrad)) sout[k] = kDead;
					}
				}
	}
}

// whether any point is still undecided (the round loop only tests for zero): a plain store of 1 by
// every wave that has one — identical values, no atomic (a per-wave atomicAdd on one counter took
// 150 us per round for 2.5 M points)
__global__ void __launch_bounds__(256) k_thin_count(const uint8_t *st, uint32_t n, uint32_t *any_undecided)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	const bool u = i < n && st[i] == kUndecided;
	const uint64_t m = __ballot(u);
	if(m && __lane_id() == 0) *any_undecided = 1u;
}

struct IsKept
{
	const uint8_t *st;
	__host__ __device__ bool operator()(uint32_t i) const { return st[i] == kKept; }
};

} // namespace

#define THCHECK(x)                                                                                             \
	do                                                                                                         \
	{                                                                                                          \
		const hipError_t e_ = (x);                                                                             \
		if(e_ != hipSuccess) return e_;                                                                        \
	} while(0)

extern "C" void yafamd_thin_scratch_free(void *scratch) { delete static_cast<ThinScratch *>(scratch); }

// ---- final gathering's radiance-map grid (findNearest over cells, kernels.hip gridNearest) ----
struct RadGridScratch
{
	ThinBuf part, cid, count, start, order, tmp, gpos, gdir;
	~RadGridScratch()
	{
		for(ThinBuf *b : {&part, &cid, &count, &start, &order, &tmp, &gpos, &gdir})
			if(b->p) (void)hipFree(b->p);
	}
};

__device__ __forceinline__ int radCell(float v, float lo, float inv_cell, int na)
{
	const int c = (int)floorf((v - lo) * inv_cell);
	return c < 0 ? 0 : (c >= na ? na - 1 : c);
}

__global__ void __launch_bounds__(256) k_rg_cells(const float4 *pos, uint32_t n, yafamd::RadGrid g, uint32_t *cid, uint32_t *count)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= n) return;
	const float4 p = pos[i];
	const uint32_t c = (uint32_t)((radCell(p.z, g.lo[2], g.inv_cell, g.nz) * g.ny + radCell(p.y, g.lo[1], g.inv_cell, g.ny)) * g.nx +
	                              radCell(p.x, g.lo[0], g.inv_cell, g.nx));
	cid[i] = c;
	atomicAdd(&count[c], 1u);
}

// cell order: the photon's position + its index (bits) and its normal
__global__ void __launch_bounds__(256) k_rg_fill(const float4 *pos, const float4 *dir, const uint32_t *cid, uint32_t n, const uint32_t *start,
                                                uint32_t *fill, float4 *gpos, float4 *gdir)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= n) return;
	const uint32_t c = cid[i];
	const uint32_t k = start[c] + atomicAdd(&fill[c], 1u);   // order inside a cell is irrelevant (minimum + tie test)
	const float4 p = pos[i];
	gpos[k] = make_float4(p.x, p.y, p.z, __uint_as_float(i));
	gdir[k] = dir[i];
}

extern "C" void yafamd_rad_grid_free(void *scratch) { delete static_cast<RadGridScratch *>(scratch); }

// The grid over the radiance map's n photons (pos / dir: the arrays the lookups index, kd order), cell =
// sqrt(lookup_rad) / 3: the nearest radiance photon is mostly within the 3 x 3 x 3 cells around a point
// (gridNearest grows its block only when it is not).  hipErrorNotSupported above 2^22 cells (the kd search serves then).  The grid lives in *scratch
// until the next build.
extern "C" hipError_t yafamd_rad_grid(const float4 *pos, const float4 *dir, uint32_t n, float lookup_rad, yafamd::RadGrid *out, hipStream_t st,
                                      void **scratch)
{
	*out = yafamd::RadGrid{};
	if(n == 0 || !(lookup_rad > 0.f)) return hipErrorNotSupported;
	if(!scratch) return hipErrorInvalidValue;
	if(!*scratch) *scratch = new RadGridScratch;
	RadGridScratch &S = *static_cast<RadGridScratch *>(*scratch);
	THCHECK(S.part.ensure(2 * kBoundBlocks * sizeof(float4)));
	hipLaunchKernelGGL(k_thin_bound, dim3(kBoundBlocks), dim3(256), 0, st, pos, n, S.part.as<float4>());
	std::vector<float4> part(2 * kBoundBlocks);
	THCHECK(hipMemcpyAsync(part.data(), S.part.p, part.size() * sizeof(float4), hipMemcpyDeviceToHost, st));
	THCHECK(hipStreamSynchronize(st));
	float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
	for(int b = 0; b < kBoundBlocks; ++b)
	{
		const float4 l = part[2 * b], h = part[2 * b + 1];
		lo[0] = std::min(lo[0], l.x); lo[1] = std::min(lo[1], l.y); lo[2] = std::min(lo[2], l.z);
		hi[0] = std::max(hi[0], h.x); hi[1] = std::max(hi[1], h.y); hi[2] = std::max(hi[2], h.z);
	}
	const double cell = std::sqrt((double)lookup_rad) / 3.0;
	double dims[3], ncell = 1.0;
	for(int a = 0; a < 3; ++a)
	{
		if(!std::isfinite(lo[a]) || !std::isfinite(hi[a])) return hipErrorNotSupported;
		dims[a] = std::floor(((double)hi[a] - (double)lo[a]) / cell) + 1.0;
		ncell *= dims[a];
	}
	if(!(ncell <= (double)(1 << 22))) return hipErrorNotSupported;
	yafamd::RadGrid g{};
	for(int a = 0; a < 3; ++a) g.lo[a] = lo[a];
	g.cell = (float)cell;
	g.inv_cell = (float)(1.0 / cell);
	g.nx = (int)dims[0];
	g.ny = (int)dims[1];
	g.nz = (int)dims[2];
	const uint32_t nc = (uint32_t)ncell;
	THCHECK(S.cid.ensure((size_t)n * 4));
	THCHECK(S.count.ensure(((size_t)nc + 1) * 4));
	THCHECK(S.start.ensure(((size_t)nc + 1) * 4));
	THCHECK(S.gpos.ensure((size_t)n * sizeof(float4)));
	THCHECK(S.gdir.ensure((size_t)n * sizeof(float4)));
	THCHECK(hipMemsetAsync(S.count.p, 0, ((size_t)nc + 1) * 4, st));
	const dim3 blocks((n + 255) / 256);
	hipLaunchKernelGGL(k_rg_cells, blocks, dim3(256), 0, st, pos, n, g, S.cid.as<uint32_t>(), S.count.as<uint32_t>());
	size_t scan_bytes = 0;
	THCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, S.count.as<uint32_t>(), S.start.as<uint32_t>(), (int)nc + 1, st));
	THCHECK(S.tmp.ensure(scan_bytes));
	THCHECK(hipcub::DeviceScan::ExclusiveSum(S.tmp.p, scan_bytes, S.count.as<uint32_t>(), S.start.as<uint32_t>(), (int)nc + 1, st));
	THCHECK(hipMemsetAsync(S.count.p, 0, ((size_t)nc + 1) * 4, st));
	hipLaunchKernelGGL(k_rg_fill, blocks, dim3(256), 0, st, pos, dir, S.cid.as<uint32_t>(), n, S.start.as<uint32_t>(), S.count.as<uint32_t>(),
	                   S.gpos.as<float4>(), S.gdir.as<float4>());
	THCHECK(hipGetLastError());
	g.start = S.start.as<uint32_t>();
	g.pos = S.gpos.as<float4>();
	g.dir = S.gdir.as<float4>();
	*out = g;
	return hipSuccess;
}

// pos / nrm: the compacted radiance points (xyz used); kept_out: device, n entries of capacity.
// Returns hipErrorNotSupported when the dense grid would exceed 2^26 cells (the caller thins on the
// host then).  *scratch: the caller's scratch (created on first use, yafamd_thin_scratch_free).
extern "C" hipError_t yafamd_thin_rad_points(const float4 *pos, const float4 *nrm, uint32_t n, float maxrad, uint32_t *kept_out,
                                             uint32_t *n_kept, int *rounds_out, hipStream_t st, void **scratch)
{
	*n_kept = 0;
	*rounds_out = 0;
	if(n == 0) return hipSuccess;
	if(!scratch) return hipErrorInvalidValue;
	if(!*scratch) *scratch = new ThinScratch;
	ThinScratch &S = *static_cast<ThinScratch *>(*scratch);
	THCHECK(S.part.ensure(2 * kBoundBlocks * sizeof(float4)));
	hipLaunchKernelGGL(k_thin_bound, dim3(kBoundBlocks), dim3(256), 0, st, pos, n, S.part.as<float4>());
	std::vector<float4> part(2 * kBoundBlocks);
	THCHECK(hipMemcpyAsync(part.data(), S.part.p, part.size() * sizeof(float4), hipMemcpyDeviceToHost, st));
	THCHECK(hipStreamSynchronize(st));
	double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
	for(int b = 0; b < kBoundBlocks; ++b)
	{
		const float4 l = part[2 * b], h = part[2 * b + 1];
		lo[0] = std::min(lo[0], (double)l.x); lo[1] = std::min(lo[1], (double)l.y); lo[2] = std::min(lo[2], (double)l.z);
		hi[0] = std::max(hi[0], (double)h.x); hi[1] = std::max(hi[1], (double)h.y); hi[2] = std::max(hi[2], (double)h.z);
	}
	// cell a little larger than sqrt(maxrad): two points closer than that differ by <= 1 cell per axis
	const double cell = std::sqrt((double)maxrad) * 1.001 + 1e-30;
	double dims[3], ncell = 1.0;
	for(int a = 0; a < 3; ++a) { dims[a] = std::floor((hi[a] - lo[a]) / cell) + 1.0; ncell *= dims[a]; }
	if(!(ncell <= (double)(1 << 26))) return hipErrorNotSupported;
	ThinGrid g;
	for(int a = 0; a < 3; ++a) g.lo[a] = lo[a];
	g.inv_cell = 1.0 / cell;
	g.nx = (int)dims[0];
	g.ny = (int)dims[1];
	g.nz = (int)dims[2];
	const uint32_t nc = (uint32_t)ncell;
	THCHECK(S.cid.ensure((size_t)n * 4));
	THCHECK(S.order.ensure((size_t)n * 4));
	THCHECK(S.count.ensure(((size_t)nc + 1) * 4));
	THCHECK(S.start.ensure(((size_t)nc + 1) * 4));
	THCHECK(S.st0.ensure(n));
	THCHECK(S.st1.ensure(n));
	THCHECK(S.counter.ensure(16));
	THCHECK(S.klist.ensure((size_t)n * 4));
	THCHECK(S.n_sel.ensure(16));
	THCHECK(S.spos.ensure((size_t)n * sizeof(float4)));
	THCHECK(S.snrm.ensure((size_t)n * sizeof(float4)));
	THCHECK(hipMemsetAsync(S.count.p, 0, ((size_t)nc + 1) * 4, st));
	const dim3 blocks((n + 255) / 256);
	hipLaunchKernelGGL(k_thin_cells, blocks, dim3(256), 0, st, pos, n, g, S.cid.as<uint32_t>(), S.count.as<uint32_t>());
	size_t scan_bytes = 0;
	THCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, S.count.as<uint32_t>(), S.start.as<uint32_t>(), (int)nc + 1, st));
	size_t sel_bytes = 0;
	hipcub::CountingInputIterator<uint32_t> iota(0);
	hipcub::TransformInputIterator<bool, IsKept, hipcub::CountingInputIterator<uint32_t>> flags(iota, IsKept{S.st0.as<uint8_t>()});
	THCHECK(hipcub::DeviceSelect::Flagged(nullptr, sel_bytes, iota, flags, kept_out, S.n_sel.as<uint32_t>(), (int)n, st));
	THCHECK(S.tmp.ensure(std::max(scan_bytes, sel_bytes)));
	THCHECK(hipcub::DeviceScan::ExclusiveSum(S.tmp.p, scan_bytes, S.count.as<uint32_t>(), S.start.as<uint32_t>(), (int)nc + 1, st));
	THCHECK(hipMemsetAsync(S.count.p, 0, ((size_t)nc + 1) * 4, st));
	hipLaunchKernelGGL(k_thin_fill, blocks, dim3(256), 0, st, S.cid.as<uint32_t>(), n, S.start.as<uint32_t>(), S.count.as<uint32_t>(),
	                   S.order.as<uint32_t>());
	hipLaunchKernelGGL(k_thin_sort, blocks, dim3(256), 0, st, pos, nrm, S.order.as<uint32_t>(), n, S.spos.as<float4>(), S.snrm.as<float4>());
	const float4 *spos = S.spos.as<float4>(), *snrm = S.snrm.as<float4>();
	THCHECK(hipMemsetAsync(S.st0.p, kUndecided, n, st));
	uint8_t *sin = S.st0.as<uint8_t>(), *sout = S.st1.as<uint8_t>();
	uint32_t undecided = n;
	int rounds = 0;
	while(undecided > 0)
	{
		THCHECK(hipMemsetAsync(S.counter.p, 0, 8, st));   // [0] any point undecided (0 / 1), [1] kept-list length
		uint32_t *n_klist = S.counter.as<uint32_t>() + 1;
		hipLaunchKernelGGL(k_thin_keep, dim3((uint32_t)(((uint64_t)n * kKeepLanes + 255) / 256)), dim3(256), 0, st, spos, snrm, S.order.as<uint32_t>(), S.start.as<uint32_t>(), g, sin, sout, n, maxrad,
		                   S.klist.as<uint32_t>(), n_klist);
		hipLaunchKernelGGL(k_thin_kill, dim3(1024), dim3(256), 0, st, spos, snrm, S.order.as<uint32_t>(), S.start.as<uint32_t>(), g, sout,
		                   S.klist.as<uint32_t>(), n_klist, maxrad);
		hipLaunchKernelGGL(k_thin_count, blocks, dim3(256), 0, st, sout, n, S.counter.as<uint32_t>());
		THCHECK(hipGetLastError());
		THCHECK(hipMemcpyAsync(&undecided, S.counter.p, 4, hipMemcpyDeviceToHost, st));
		THCHECK(hipStreamSynchronize(st));
		std::swap(sin, sout);
		++rounds;
		if(rounds > 1000000) return hipErrorUnknown;   // cannot happen: every round decides the lowest undecided point
	}
	// the final states are in `sin` (cell order): back to shooting order in `sout`, then the kept indices
	hipLaunchKernelGGL(k_thin_unsort, blocks, dim3(256), 0, st, sin, S.order.as<uint32_t>(), n, sout);
	hipcub::TransformInputIterator<bool, IsKept, hipcub::CountingInputIterator<uint32_t>> kflags(iota, IsKept{sout});
	THCHECK(hipcub::DeviceSelect::Flagged(S.tmp.p, sel_bytes, iota, kflags, kept_out, S.n_sel.as<uint32_t>(), (int)n, st));
	THCHECK(hipMemcpyAsync(n_kept, S.n_sel.p, 4, hipMemcpyDeviceToHost, st));
	THCHECK(hipStreamSynchronize(st));
	*rounds_out = rounds;
	return hipSuccess;
}
