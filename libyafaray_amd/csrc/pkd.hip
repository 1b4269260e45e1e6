// GPU build of the photon map's point kd-tree (reference include/photon/pkdtree.h:115-222).
//
// The reference builds it recursively with std::nth_element: every node splits its photons at the
// median (element (start + end) / 2) along the largest axis of the node bound, under the total
// order "coordinate, then element address".  The resulting tree depends only on the photon set and
// that order — not on how nth_element arranges elements inside each half — so any exact median
// split reproduces it node for node.
//
// Layout of the work (all of it data-parallel, no host round trip per level):
//   records  three lists of the photons sorted by (coord_a, index), a = x, y, z (radix sorts); an
//            entry carries all three orderable coordinate keys + the index (16 B), so any list can
//            be split by any axis without gathers.  Every node's photons occupy the same index range
//            [start, end) in all three lists.
//   top      level-synchronous while nodes hold more than kSub photons: per node the largest axis of
//            its bound picks the list whose element (start + end) / 2 is the median; each list is
//            stably partitioned around it ((key, index) < median goes left: one exclusive scan per
//            list whose input is that comparison).  A node of m > 1 photons always has two children,
//            so level d holds exactly 2^d nodes of floor / ceil(n / 2^d) photons and all nodes of a
//            level leave the top phase together.
//   bottom   one workgroup per remaining subtree (<= kSub photons) finishes it in LDS, level by
//            level with the same rule.
// Node layout is the reference's depth-first one: a subtree of m photons has 2m - 1 nodes, node i's
// left child is i + 1 and its right child i + 2 nl.  Node record (uint4): .w = flags (bits 0-1 axis,
// 3 = leaf; interior: right child << 2, leaf: photon index << 2), interior .x = split position bits,
// leaf .xyz = the photon's position bits (k_gather reads them without a second load).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdint>
#include <vector>

namespace
{

constexpr int kSub = 256;           // subtree size finished by one workgroup in LDS (~51 KB of LDS)
constexpr int kSubThreads = 256;

struct Seg
{
	uint32_t node, start, end;   // tree node and its photon range in the lists
	float lo[3], hi[3];          // node bound (pkdtree.h:152-160)
};

// per node of the current top level: split axis and median element
struct Split
{
	uint32_t axis, split_el, med_key, med_idx;
};

__device__ __forceinline__ float coordOf(const float4 &p, int a) { return a == 0 ? p.x : (a == 1 ? p.y : p.z); }
__device__ __forceinline__ uint32_t keyOf(const uint4 &r, int a) { return a == 0 ? r.x : (a == 1 ? r.y : r.z); }

// orderable key of a float coordinate; -0 and +0 compare equal in the reference's comparator
__device__ __forceinline__ uint32_t orderKey(float f)
{
	if(f == 0.f) f = 0.f;
	const uint32_t u = __float_as_uint(f);
	return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// "left of the median" in the (coordinate, index) order of `axis`
__device__ __forceinline__ bool leftOf(const uint4 &r, uint32_t axis, uint32_t med_key, uint32_t med_idx)
{
	const uint32_t k = keyOf(r, (int)axis);
	return k < med_key || (k == med_key && r.w < med_idx);
}

// bound.h:111-115 largestAxis
__device__ __forceinline__ int largestAxis(const float *lo, const float *hi)
{
	const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
	return (dx > dy) ? ((dx > dz) ? 0 : 2) : ((dy > dz) ? 1 : 2);
}

__global__ void k_keys(const float4 *pos, uint32_t n, uint32_t *kx, uint32_t *ky, uint32_t *kz, uint32_t *iota)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= n) return;
	const float4 p = pos[i];
	kx[i] = orderKey(p.x);
	ky[i] = orderKey(p.y);
	kz[i] = orderKey(p.z);
	iota[i] = i;
}

__global__ void k_records(const uint32_t *sorted_idx, uint32_t n, const uint32_t *kx, const uint32_t *ky, const uint32_t *kz, uint4 *rec)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	const uint32_t i = sorted_idx[p];
	rec[p] = make_uint4(kx[i], ky[i], kz[i], i);
}

// root bound (pkdtree.h:98-101): per-workgroup min/max, then one workgroup folds the partials
__global__ void k_bound(const float4 *pos, uint32_t n, float *partial /* gridDim.x * 6 */)
{
	float v[6] = {3.4e38f, 3.4e38f, 3.4e38f, -3.4e38f, -3.4e38f, -3.4e38f};
	for(uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
	{
		const float4 p = pos[i];
		v[0] = fminf(v[0], p.x); v[1] = fminf(v[1], p.y); v[2] = fminf(v[2], p.z);
		v[3] = fmaxf(v[3], p.x); v[4] = fmaxf(v[4], p.y); v[5] = fmaxf(v[5], p.z);
	}
	__shared__ float red[6][256];
	for(int k = 0; k < 6; ++k) red[k][threadIdx.x] = v[k];
	__syncthreads();
	for(int w = blockDim.x / 2; w > 0; w >>= 1)
	{
		if((int)threadIdx.x < w)
		{
			for(int k = 0; k < 3; ++k) red[k][threadIdx.x] = fminf(red[k][threadIdx.x], red[k][threadIdx.x + w]);
			for(int k = 3; k < 6; ++k) red[k][threadIdx.x] = fmaxf(red[k][threadIdx.x], red[k][threadIdx.x + w]);
		}
		__syncthreads();
	}
	if(threadIdx.x < 6) partial[blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

// fold the partials (256 threads) and create the root segment
__global__ void k_root(const float *partial, uint32_t n_part, uint32_t n, Seg *segs)
{
	__shared__ float red[6][256];
	float v[6] = {3.4e38f, 3.4e38f, 3.4e38f, -3.4e38f, -3.4e38f, -3.4e38f};
	for(uint32_t b = threadIdx.x; b < n_part; b += blockDim.x)
	{
		for(int k = 0; k < 3; ++k) v[k] = fminf(v[k], partial[b * 6 + k]);
		for(int k = 3; k < 6; ++k) v[k] = fmaxf(v[k], partial[b * 6 + k]);
	}
	for(int k = 0; k < 6; ++k) red[k][threadIdx.x] = v[k];
	__syncthreads();
	for(int w = blockDim.x / 2; w > 0; w >>= 1)
	{
		if((int)threadIdx.x < w)
		{
			for(int k = 0; k < 3; ++k) red[k][threadIdx.x] = fminf(red[k][threadIdx.x], red[k][threadIdx.x + w]);
			for(int k = 3; k < 6; ++k) red[k][threadIdx.x] = fmaxf(red[k][threadIdx.x], red[k][threadIdx.x + w]);
		}
		__syncthreads();
	}
	if(threadIdx.x == 0)
	{
		Seg g;
		g.node = 0;
		g.start = 0;
		g.end = n;
		for(int k = 0; k < 3; ++k)
		{
			g.lo[k] = red[k][0];
			g.hi[k] = red[3 + k][0];
		}
		segs[0] = g;
	}
}

// ---- top phase (one level: every node splits in two) ----
__global__ void k_level_split(const Seg *segs, uint32_t n_seg, const uint4 *rx, const uint4 *ry, const uint4 *rz, const float4 *pos,
                              uint4 *nodes, Split *splits, Seg *next)
{
	const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
	if(s >= n_seg) return;
	const Seg g = segs[s];
	const int axis = largestAxis(g.lo, g.hi);
	const uint32_t se = (g.start + g.end) / 2;
	const uint4 med = (axis == 0 ? rx : (axis == 1 ? ry : rz))[se];
	const float split_pos = coordOf(pos[med.w], axis);
	const uint32_t nl = se - g.start;
	const uint32_t right = g.node + 2u * nl;
	nodes[g.node] = make_uint4(__float_as_uint(split_pos), 0u, 0u, (uint32_t)axis | (right << 2));
	splits[s] = {(uint32_t)axis, se, keyOf(med, axis), med.w};
	Seg l = g, r = g;
	l.node = g.node + 1;
	l.end = se;
	l.hi[axis] = split_pos;
	r.node = right;
	r.start = se;
	r.lo[axis] = split_pos;
	next[2 * s] = l;
	next[2 * s + 1] = r;
}

// the scan input of the stable partitions: 1 for entries left of their node's median
struct LeftFlag
{
	const uint4 *rec;
	const uint32_t *seg_of;
	const Split *splits;
	__host__ __device__ uint32_t operator()(const uint32_t &p) const
	{
		const Split sp = splits[seg_of[p]];
		return leftOf(rec[p], sp.axis, sp.med_key, sp.med_idx) ? 1u : 0u;
	}
};

__global__ void k_partition(const uint4 *rec, uint32_t n, const uint32_t *scan, const uint32_t *seg_of, const Seg *segs, const Split *splits,
                            uint4 *out)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	const uint32_t s = seg_of[p];
	const Split sp = splits[s];
	const uint4 r = rec[p];
	const uint32_t start = segs[s].start;
	const uint32_t left_before = scan[p] - scan[start];
	const uint32_t np = leftOf(r, sp.axis, sp.med_key, sp.med_idx) ? start + left_before : sp.split_el + ((p - start) - left_before);
	out[np] = r;
}

__global__ void k_seg_of(uint32_t *seg_of, uint32_t n, const Split *splits)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	const uint32_t s = seg_of[p];
	seg_of[p] = 2u * s + (p < splits[s].split_el ? 0u : 1u);
}

// ---- bottom phase: one workgroup per subtree of <= kSub photons ----
// LDS: the three lists of the subtree (in / out buffers), per-entry flags + scan, the level's
// segments.  The same split rule as the top phase, restricted to the workgroup's range.
struct LSeg
{
	uint32_t node, start, end;   // start / end relative to the subtree's first element
	float lo[3], hi[3];
};

__global__ void __launch_bounds__(kSubThreads) k_subtrees(const Seg *segs, const uint4 *gx, const uint4 *gy, const uint4 *gz, const float4 *pos,
                                                        uint4 *nodes, int base_level, int *max_level)
{
	constexpr uint16_t kNone = 0xffffu;
	constexpr int kPer = kSub / kSubThreads;   // entries per thread
	__shared__ uint4 buf[2][3][kSub];
	__shared__ uint32_t scan[3][kSub + 1];
	__shared__ LSeg lsegs[2][kSub];
	__shared__ Split lsplit[kSub];
	__shared__ uint32_t cb[kSub + 1];          // child segment base (2 x splitting segments before s)
	__shared__ uint16_t seg_of[kSub];
	const Seg g = segs[blockIdx.x];
	const uint32_t m = g.end - g.start;
	const int t = threadIdx.x;
	for(uint32_t e = t; e < m; e += kSubThreads)
	{
		buf[0][0][e] = gx[g.start + e];
		buf[0][1][e] = gy[g.start + e];
		buf[0][2][e] = gz[g.start + e];
		seg_of[e] = 0;
	}
	if(t == 0)
	{
		LSeg l;
		l.node = g.node;
		l.start = 0;
		l.end = m;
		for(int k = 0; k < 3; ++k) { l.lo[k] = g.lo[k]; l.hi[k] = g.hi[k]; }
		lsegs[0][0] = l;
	}
	__syncthreads();
	int cur = 0, cs = 0, level = base_level;
	uint32_t ns = 1;
	bool any_leaf_seen = false;
	while(ns > 0)
	{
		// per segment: a leaf (one photon) or a split at the median of its largest axis
		bool leaf_here = false;
		for(uint32_t s = t; s < ns; s += kSubThreads)
		{
			const LSeg l = lsegs[cs][s];
			if(l.end - l.start == 1)
			{
				// pkdtree.h:29-33 createLeaf: the photon (and, for k_gather, its position)
				const uint32_t idx = buf[cur][0][l.start].w;
				const float4 ph = pos[idx];
				nodes[l.node] = make_uint4(__float_as_uint(ph.x), __float_as_uint(ph.y), __float_as_uint(ph.z), 3u | (idx << 2));
				lsplit[s] = {3u, 0u, 0u, 0u};
				cb[s + 1] = 0;
				leaf_here = true;
				continue;
			}
			const int axis = largestAxis(l.lo, l.hi);
			const uint32_t se = (l.start + l.end) / 2;
			const uint4 med = buf[cur][axis][se];
			const float split_pos = coordOf(pos[med.w], axis);
			const uint32_t right = l.node + 2u * (se - l.start);
			nodes[l.node] = make_uint4(__float_as_uint(split_pos), 0u, 0u, (uint32_t)axis | (right << 2));
			lsplit[s] = {(uint32_t)axis, se, keyOf(med, axis), med.w};
			cb[s + 1] = 2;
		}
		if(t == 0) cb[0] = 0;
		if(__syncthreads_or(leaf_here ? 1 : 0)) any_leaf_seen = true;
		if(any_leaf_seen && t == 0) atomicMax(max_level, level);   // deepest level holding a node so far
		// inclusive scan of the child counts -> cb[s] = children of segments [0, s)
		for(uint32_t off = 1; off <= ns; off <<= 1)
		{
			uint32_t v[kPer + 1];
			int q = 0;
			for(uint32_t s = t + 1; s <= ns; s += kSubThreads, ++q) v[q] = cb[s] + (s > off ? cb[s - off] : 0u);
			__syncthreads();
			q = 0;
			for(uint32_t s = t + 1; s <= ns; s += kSubThreads, ++q) cb[s] = v[q];
			__syncthreads();
		}
		const uint32_t n_next = cb[ns];
		if(n_next == 0) break;
		// stable partition of each list inside every splitting segment (entries of leaves stay put)
		for(int a = 0; a < 3; ++a)
			for(uint32_t e = t; e < m; e += kSubThreads)
			{
				const uint16_t s = seg_of[e];
				uint32_t f = 0;
				if(s != kNone)
				{
					const Split sp = lsplit[s];
					if(sp.axis != 3u) f = leftOf(buf[cur][a][e], sp.axis, sp.med_key, sp.med_idx) ? 1u : 0u;
				}
				scan[a][e + 1] = f;
			}
		if(t < 3) scan[t][0] = 0;
		__syncthreads();
		for(uint32_t off = 1; off < m; off <<= 1)
		{
			uint32_t v[3][kPer + 1];
			int q = 0;
			for(uint32_t e = t + 1; e <= m; e += kSubThreads, ++q)
				for(int a = 0; a < 3; ++a) v[a][q] = scan[a][e] + (e > off ? scan[a][e - off] : 0u);
			__syncthreads();
			q = 0;
			for(uint32_t e = t + 1; e <= m; e += kSubThreads, ++q)
				for(int a = 0; a < 3; ++a) scan[a][e] = v[a][q];
			__syncthreads();
		}
		for(int a = 0; a < 3; ++a)
			for(uint32_t e = t; e < m; e += kSubThreads)
			{
				const uint4 r = buf[cur][a][e];
				const uint16_t s = seg_of[e];
				if(s == kNone || lsplit[s].axis == 3u) { buf[cur ^ 1][a][e] = r; continue; }
				const Split sp = lsplit[s];
				const uint32_t start = lsegs[cs][s].start;
				const uint32_t left_before = scan[a][e] - scan[a][start];
				const uint32_t np = leftOf(r, sp.axis, sp.med_key, sp.med_idx) ? start + left_before : sp.split_el + ((e - start) - left_before);
				buf[cur ^ 1][a][np] = r;
			}
		// the next level's segments
		for(uint32_t s = t; s < ns; s += kSubThreads)
		{
			const Split sp = lsplit[s];
			if(sp.axis == 3u) continue;
			const LSeg l = lsegs[cs][s];
			const float split_pos = coordOf(pos[sp.med_idx], (int)sp.axis);
			LSeg lo = l, hi = l;
			lo.node = l.node + 1;
			lo.end = sp.split_el;
			lo.hi[sp.axis] = split_pos;
			hi.node = l.node + 2u * (sp.split_el - l.start);
			hi.start = sp.split_el;
			hi.lo[sp.axis] = split_pos;
			lsegs[cs ^ 1][cb[s]] = lo;
			lsegs[cs ^ 1][cb[s] + 1] = hi;
		}
		__syncthreads();
		for(uint32_t e = t; e < m; e += kSubThreads)
		{
			const uint16_t s = seg_of[e];
			if(s == kNone) continue;
			const Split sp = lsplit[s];
			seg_of[e] = (sp.axis == 3u) ? kNone : (uint16_t)(cb[s] + (e < sp.split_el ? 0u : 1u));
		}
		ns = n_next;
		cur ^= 1;
		cs ^= 1;
		++level;
		__syncthreads();
	}
}

struct DevBuf
{
	void *p = nullptr;
	size_t bytes = 0;
	void release()
	{
		if(p) (void)hipFree(p);
		p = nullptr;
		bytes = 0;
	}
	template<class T> T *as() { return reinterpret_cast<T *>(p); }
	hipError_t ensure(size_t b)
	{
		if(b < 16) b = 16;
		if(p && bytes >= b) return hipSuccess;
		release();
		const hipError_t e = hipMalloc(&p, b);
		if(e == hipSuccess) bytes = b;
		return e;
	}
};

// scratch of the build, kept between builds (the photon map is rebuilt every frame)
struct PkdScratch
{
	DevBuf kx, ky, kz, iota, sorted_keys, sorted_idx, sort_tmp, rec[3], rec_out, segs[2], seg_of, scan, scan_tmp, splits, partial, max_level;
	~PkdScratch()
	{
		for(DevBuf *b : {&kx, &ky, &kz, &iota, &sorted_keys, &sorted_idx, &sort_tmp, &rec[0], &rec[1], &rec[2], &rec_out, &segs[0], &segs[1],
		                 &seg_of, &scan, &scan_tmp, &splits, &partial, &max_level})
			b->release();
	}
};
PkdScratch g_pkd;

#define PKCHECK(x) do { hipError_t e_ = (x); if(e_ != hipSuccess) return e_; } while(0)

} // namespace

// pos_dev: n photons (position in .xyz); nodes_dev: 2n - 1 nodes (uint4, see the header comment).
// *depth_out: deepest level (root = 0) — the lookup stack needs depth + 1 entries.
extern "C" hipError_t yafamd_build_pkd(const float4 *pos_dev, uint32_t n, uint4 *nodes_dev, int *depth_out, hipStream_t st)
{
	if(n == 0) return hipSuccess;
	PkdScratch &S = g_pkd;
	const uint32_t B = 256, G = (n + B - 1) / B;
	for(DevBuf *b : {&S.kx, &S.ky, &S.kz, &S.iota, &S.sorted_keys, &S.sorted_idx, &S.seg_of}) PKCHECK(b->ensure((size_t)n * 4));
	PKCHECK(S.scan.ensure(((size_t)n + 1) * 4));
	for(DevBuf *b : {&S.rec[0], &S.rec[1], &S.rec[2], &S.rec_out}) PKCHECK(b->ensure((size_t)n * 16));
	// lists sorted by (coordinate, index): stable radix sorts of the keys over index order
	hipLaunchKernelGGL(k_keys, dim3(G), dim3(B), 0, st, pos_dev, n, S.kx.as<uint32_t>(), S.ky.as<uint32_t>(), S.kz.as<uint32_t>(),
	                   S.iota.as<uint32_t>());
	size_t sort_bytes = 0;
	PKCHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, S.kx.as<uint32_t>(), S.sorted_keys.as<uint32_t>(), S.iota.as<uint32_t>(),
	                                           S.sorted_idx.as<uint32_t>(), (int)n, 0, 32, st));
	PKCHECK(S.sort_tmp.ensure(sort_bytes));
	const uint32_t *keys[3] = {S.kx.as<uint32_t>(), S.ky.as<uint32_t>(), S.kz.as<uint32_t>()};
	for(int a = 0; a < 3; ++a)
	{
		PKCHECK(hipcub::DeviceRadixSort::SortPairs(S.sort_tmp.p, sort_bytes, keys[a], S.sorted_keys.as<uint32_t>(), S.iota.as<uint32_t>(),
		                                           S.sorted_idx.as<uint32_t>(), (int)n, 0, 32, st));
		hipLaunchKernelGGL(k_records, dim3(G), dim3(B), 0, st, S.sorted_idx.as<uint32_t>(), n, keys[0], keys[1], keys[2], S.rec[a].as<uint4>());
	}
	// root bound (pkdtree.h:98-101) and the root segment
	const uint32_t n_part = std::min<uint32_t>(G, 1024);
	PKCHECK(S.partial.ensure((size_t)n_part * 6 * 4));
	PKCHECK(S.segs[0].ensure((size_t)n * sizeof(Seg)));
	PKCHECK(S.segs[1].ensure((size_t)n * sizeof(Seg)));
	PKCHECK(S.splits.ensure((size_t)n * sizeof(Split)));
	PKCHECK(S.max_level.ensure(16));
	hipLaunchKernelGGL(k_bound, dim3(n_part), dim3(256), 0, st, pos_dev, n, S.partial.as<float>());
	hipLaunchKernelGGL(k_root, dim3(1), dim3(256), 0, st, S.partial.as<float>(), n_part, n, S.segs[0].as<Seg>());
	PKCHECK(hipMemsetAsync(S.seg_of.p, 0, (size_t)n * 4, st));
	PKCHECK(hipMemsetAsync(S.max_level.p, 0, 4, st));
	size_t scan_bytes = 0;
	{
		hipcub::CountingInputIterator<uint32_t> it(0);
		hipcub::TransformInputIterator<uint32_t, LeftFlag, hipcub::CountingInputIterator<uint32_t>> in(it, LeftFlag{});
		PKCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, in, S.scan.as<uint32_t>(), (int)n, st));
	}
	PKCHECK(S.scan_tmp.ensure(scan_bytes));
	// top phase: level d has 2^d nodes of floor / ceil(n / 2^d) photons
	uint32_t n_seg = 1;
	int cur = 0, level = 0;
	uint32_t max_m = n;
	while(max_m > (uint32_t)kSub)
	{
		const uint32_t Gs = (n_seg + B - 1) / B;
		hipLaunchKernelGGL(k_level_split, dim3(Gs), dim3(B), 0, st, S.segs[cur].as<Seg>(), n_seg, S.rec[0].as<uint4>(), S.rec[1].as<uint4>(),
		                   S.rec[2].as<uint4>(), pos_dev, nodes_dev, S.splits.as<Split>(), S.segs[cur ^ 1].as<Seg>());
		for(int a = 0; a < 3; ++a)
		{
			hipcub::CountingInputIterator<uint32_t> it(0);
			hipcub::TransformInputIterator<uint32_t, LeftFlag, hipcub::CountingInputIterator<uint32_t>> in(
			    it, LeftFlag{S.rec[a].as<uint4>(), S.seg_of.as<uint32_t>(), S.splits.as<Split>()});
			PKCHECK(hipcub::DeviceScan::ExclusiveSum(S.scan_tmp.p, scan_bytes, in, S.scan.as<uint32_t>(), (int)n, st));
			hipLaunchKernelGGL(k_partition, dim3(G), dim3(B), 0, st, S.rec[a].as<uint4>(), n, S.scan.as<uint32_t>(), S.seg_of.as<uint32_t>(),
			                   S.segs[cur].as<Seg>(), S.splits.as<Split>(), S.rec_out.as<uint4>());
			std::swap(S.rec[a].p, S.rec_out.p);
			std::swap(S.rec[a].bytes, S.rec_out.bytes);
		}
		hipLaunchKernelGGL(k_seg_of, dim3(G), dim3(B), 0, st, S.seg_of.as<uint32_t>(), n, S.splits.as<Split>());
		n_seg *= 2;
		max_m = (max_m + 1) / 2;
		cur ^= 1;
		++level;
	}
	// bottom phase: one workgroup per subtree
	hipLaunchKernelGGL(k_subtrees, dim3(n_seg), dim3(kSubThreads), 0, st, S.segs[cur].as<Seg>(), S.rec[0].as<uint4>(), S.rec[1].as<uint4>(),
	                   S.rec[2].as<uint4>(), pos_dev, nodes_dev, level, S.max_level.as<int>());
	int depth = 0;
	PKCHECK(hipMemcpyAsync(&depth, S.max_level.p, 4, hipMemcpyDeviceToHost, st));
	PKCHECK(hipStreamSynchronize(st));
	*depth_out = depth;
	return hipGetLastError();
}
