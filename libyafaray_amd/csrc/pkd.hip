// GPU build of the photon map's point kd-tree (reference include/photon/pkdtree.h:115-222).
//
// The reference builds it recursively with std::nth_element: every node splits its photons at the
// median (element (start + end) / 2) along the largest axis of the node bound, under the total
// order "coordinate, then element address".  The resulting tree depends only on the photon set and
// that order — not on how nth_element arranges elements inside each half — so any exact median
// split reproduces it node for node.  Here all nodes of a level are split at once from three
// presorted index lists (one per axis, kept sorted inside every node range by stable partitions):
//
//   sort:   S_a = photon indices sorted by (coord_a, index) for a = x, y, z   (radix sorts)
//   level:  per node: axis = largest axis of its bound, median = S_axis[split_el];
//           flag the nl photons left of the median, stable-partition S_x, S_y, S_z by the flag
//           (one exclusive scan each), children get the split bound.
//
// Node layout is the reference's depth-first one: a subtree of m photons has 2m - 1 nodes, so node
// i's left child is i + 1 and its right child i + 2 nl.  Work O(n log n), all of it data-parallel.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdint>
#include <vector>

namespace
{

struct Seg
{
	uint32_t node, start, end;   // tree node and its photon range in the sorted lists
	float lo[3], hi[3];          // node bound (pkdtree.h:152-160)
};

__device__ __forceinline__ float coordOf(const float4 &p, int a) { return a == 0 ? p.x : (a == 1 ? p.y : p.z); }

// orderable key of a float coordinate; -0 and +0 compare equal in the reference's comparator
__global__ void k_keys(const float4 *pos, uint32_t n, int axis, uint32_t *keys, uint32_t *vals)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= n) return;
	float f = coordOf(pos[i], axis);
	if(f == 0.f) f = 0.f;
	uint32_t u = __float_as_uint(f);
	u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
	keys[i] = u;
	vals[i] = i;
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

__global__ void k_bound_final(float *partial, uint32_t n_part)
{
	if(threadIdx.x != 0) return;
	for(uint32_t b = 1; b < n_part; ++b)
	{
		for(int k = 0; k < 3; ++k) partial[k] = fminf(partial[k], partial[b * 6 + k]);
		for(int k = 3; k < 6; ++k) partial[k] = fmaxf(partial[k], partial[b * 6 + k]);
	}
}

// per node of the level: axis, median, the node itself (or a leaf), and whether it has children
__global__ void k_level_nodes(const Seg *segs, uint32_t n_seg, const uint32_t *sx, const uint32_t *sy, const uint32_t *sz,
                              const float4 *pos, uint2 *nodes, uint32_t *split_el, int8_t *axis_of, uint32_t *n_children)
{
	const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
	if(s >= n_seg) return;
	const Seg g = segs[s];
	if(g.end - g.start == 1)
	{
		nodes[g.node] = make_uint2(sx[g.start], 3u);   // pkdtree.h:29-33 createLeaf
		axis_of[s] = -1;
		n_children[s] = 0;
		return;
	}
	// bound.h:111-115 largestAxis
	const float dx = g.hi[0] - g.lo[0], dy = g.hi[1] - g.lo[1], dz = g.hi[2] - g.lo[2];
	const int axis = (dx > dy) ? ((dx > dz) ? 0 : 2) : ((dy > dz) ? 1 : 2);
	const uint32_t se = (g.start + g.end) / 2;
	const uint32_t *sa = axis == 0 ? sx : (axis == 1 ? sy : sz);
	const float split_pos = coordOf(pos[sa[se]], axis);
	const uint32_t nl = se - g.start;
	nodes[g.node] = make_uint2(__float_as_uint(split_pos), (uint32_t)axis | ((g.node + 2u * nl) << 2));
	split_el[s] = se;
	axis_of[s] = (int8_t)axis;
	n_children[s] = 2;
}

// flag[e] = 1 for the photons left of their node's median (by the node's split axis order)
__global__ void k_flags(const uint32_t *seg_of, uint32_t n, const uint32_t *sx, const uint32_t *sy, const uint32_t *sz,
                        const int8_t *axis_of, const uint32_t *split_el, uint8_t *flag)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	const uint32_t s = seg_of[p];
	if(s == 0xffffffffu) return;
	const int axis = axis_of[s];
	if(axis < 0) return;
	const uint32_t *sa = axis == 0 ? sx : (axis == 1 ? sy : sz);
	flag[sa[p]] = p < split_el[s] ? 1 : 0;
}

__global__ void k_gather_flags(const uint32_t *sa, uint32_t n, const uint8_t *flag, const uint32_t *seg_of, const int8_t *axis_of,
                               uint32_t *fl)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	const uint32_t s = seg_of[p];
	fl[p] = (s != 0xffffffffu && axis_of[s] >= 0) ? flag[sa[p]] : 0u;
}

// stable partition of one sorted list inside every splitting node
__global__ void k_partition(const uint32_t *sa, uint32_t n, const uint32_t *fl, const uint32_t *scan, const uint32_t *seg_of,
                            const Seg *segs, const int8_t *axis_of, const uint32_t *split_el, uint32_t *out)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	const uint32_t s = seg_of[p];
	if(s == 0xffffffffu || axis_of[s] < 0) { out[p] = sa[p]; return; }
	const uint32_t start = segs[s].start;
	const uint32_t left_before = scan[p] - scan[start];
	const uint32_t np = fl[p] ? start + left_before : split_el[s] + ((p - start) - left_before);
	out[np] = sa[p];
}

// children of the level's splitting nodes (child_base = exclusive scan of n_children)
__global__ void k_children(const Seg *segs, uint32_t n_seg, const int8_t *axis_of, const uint32_t *split_el,
                           const uint32_t *child_base, const uint2 *nodes, Seg *next)
{
	const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
	if(s >= n_seg || axis_of[s] < 0) return;
	const Seg g = segs[s];
	const int axis = axis_of[s];
	const float split_pos = __uint_as_float(nodes[g.node].x);
	const uint32_t se = split_el[s];
	Seg l = g, r = g;
	l.node = g.node + 1;
	l.end = se;
	l.hi[axis] = split_pos;
	r.node = g.node + 2u * (se - g.start);
	r.start = se;
	r.lo[axis] = split_pos;
	next[child_base[s]] = l;
	next[child_base[s] + 1] = r;
}

// positions of the next level: the left child keeps [start, split_el), the right [split_el, end)
__global__ void k_seg_of(uint32_t *seg_of, uint32_t n, const int8_t *axis_of, const uint32_t *split_el,
                         const uint32_t *child_base)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	const uint32_t s = seg_of[p];
	if(s == 0xffffffffu) return;
	if(axis_of[s] < 0) { seg_of[p] = 0xffffffffu; return; }
	seg_of[p] = child_base[s] + (p < split_el[s] ? 0u : 1u);
}

__global__ void k_init_seg(Seg *segs, uint32_t n, const float *lohi, uint32_t *seg_of)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p < n) seg_of[p] = 0;
	if(p == 0)
	{
		Seg g;
		g.node = 0;
		g.start = 0;
		g.end = n;
		for(int k = 0; k < 3; ++k)
		{
			g.lo[k] = lohi[k];
			g.hi[k] = lohi[3 + k];
		}
		segs[0] = g;
	}
}

struct DevBuf
{
	void *p = nullptr;
	~DevBuf() { if(p) (void)hipFree(p); }
	template<class T> T *as() { return reinterpret_cast<T *>(p); }
	hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes < 16 ? 16 : bytes); }
};

#define PKCHECK(x) do { hipError_t e_ = (x); if(e_ != hipSuccess) return e_; } while(0)

} // namespace

// pos_dev: n photons (position in .xyz); nodes_dev: 2n - 1 nodes (split/photon, flags).
// *depth_out: deepest level (root = 0) — the lookup stack needs depth + 1 entries.
extern "C" hipError_t yafamd_build_pkd(const float4 *pos_dev, uint32_t n, uint2 *nodes_dev, int *depth_out, hipStream_t st)
{
	if(n == 0) return hipSuccess;
	const uint32_t B = 256, G = (n + B - 1) / B;
	DevBuf keys, keys_out, s[3], tmp_vals, tmp_sort, segs[2], seg_of, flag, fl, scan, split_el, axis_of, n_child, child_base,
	    lohi, tmp_scan, counts;
	PKCHECK(keys.alloc((size_t)n * 4));
	PKCHECK(keys_out.alloc((size_t)n * 4));
	PKCHECK(tmp_vals.alloc((size_t)n * 4));
	for(auto &b : s) PKCHECK(b.alloc((size_t)n * 4));
	// S_a: photon indices sorted by (coordinate, index) — radix sort is stable, indices start ascending
	size_t sort_bytes = 0;
	PKCHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, keys.as<uint32_t>(), keys_out.as<uint32_t>(),
	                                           tmp_vals.as<uint32_t>(), s[0].as<uint32_t>(), (int)n, 0, 32, st));
	PKCHECK(tmp_sort.alloc(sort_bytes));
	for(int a = 0; a < 3; ++a)
	{
		hipLaunchKernelGGL(k_keys, dim3(G), dim3(B), 0, st, pos_dev, n, a, keys.as<uint32_t>(), tmp_vals.as<uint32_t>());
		PKCHECK(hipcub::DeviceRadixSort::SortPairs(tmp_sort.p, sort_bytes, keys.as<uint32_t>(), keys_out.as<uint32_t>(),
		                                           tmp_vals.as<uint32_t>(), s[a].as<uint32_t>(), (int)n, 0, 32, st));
	}
	// root bound (pkdtree.h:98-101)
	const uint32_t n_part = std::min<uint32_t>(G, 1024);
	PKCHECK(lohi.alloc((size_t)n_part * 6 * 4));
	hipLaunchKernelGGL(k_bound, dim3(n_part), dim3(256), 0, st, pos_dev, n, lohi.as<float>());
	hipLaunchKernelGGL(k_bound_final, dim3(1), dim3(64), 0, st, lohi.as<float>(), n_part);
	PKCHECK(segs[0].alloc((size_t)n * sizeof(Seg)));
	PKCHECK(segs[1].alloc((size_t)n * sizeof(Seg)));
	PKCHECK(seg_of.alloc((size_t)n * 4));
	PKCHECK(flag.alloc(n));
	PKCHECK(fl.alloc((size_t)n * 4));
	PKCHECK(scan.alloc((size_t)n * 4));
	PKCHECK(split_el.alloc((size_t)n * 4));
	PKCHECK(axis_of.alloc(n));
	PKCHECK(n_child.alloc((size_t)n * 4 + 4));
	PKCHECK(child_base.alloc((size_t)n * 4 + 4));
	hipLaunchKernelGGL(k_init_seg, dim3(G), dim3(B), 0, st, segs[0].as<Seg>(), n, lohi.as<float>(), seg_of.as<uint32_t>());
	size_t scan_bytes = 0;
	PKCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, fl.as<uint32_t>(), scan.as<uint32_t>(), (int)n + 1, st));
	PKCHECK(tmp_scan.alloc(scan_bytes));
	DevBuf s_out;
	PKCHECK(s_out.alloc((size_t)n * 4));
	uint32_t n_seg = 1;
	int cur = 0, level = 0;
	while(n_seg > 0)
	{
		const uint32_t Gs = (n_seg + B - 1) / B;
		hipLaunchKernelGGL(k_level_nodes, dim3(Gs), dim3(B), 0, st, segs[cur].as<Seg>(), n_seg, s[0].as<uint32_t>(), s[1].as<uint32_t>(),
		                   s[2].as<uint32_t>(), pos_dev, nodes_dev, split_el.as<uint32_t>(), axis_of.as<int8_t>(), n_child.as<uint32_t>());
		// children: exclusive scan of the per-node child counts (one extra slot = total)
		PKCHECK(hipMemsetAsync(n_child.as<uint32_t>() + n_seg, 0, 4, st));
		PKCHECK(hipcub::DeviceScan::ExclusiveSum(tmp_scan.p, scan_bytes, n_child.as<uint32_t>(), child_base.as<uint32_t>(), (int)n_seg + 1, st));
		uint32_t n_next = 0;
		PKCHECK(hipMemcpyAsync(&n_next, child_base.as<uint32_t>() + n_seg, 4, hipMemcpyDeviceToHost, st));
		if(level > 0 || n_next > 0)
		{
			hipLaunchKernelGGL(k_flags, dim3(G), dim3(B), 0, st, seg_of.as<uint32_t>(), n, s[0].as<uint32_t>(), s[1].as<uint32_t>(),
			                   s[2].as<uint32_t>(), axis_of.as<int8_t>(), split_el.as<uint32_t>(), flag.as<uint8_t>());
			for(int a = 0; a < 3; ++a)
			{
				hipLaunchKernelGGL(k_gather_flags, dim3(G), dim3(B), 0, st, s[a].as<uint32_t>(), n, flag.as<uint8_t>(), seg_of.as<uint32_t>(),
				                   axis_of.as<int8_t>(), fl.as<uint32_t>());
				PKCHECK(hipcub::DeviceScan::ExclusiveSum(tmp_scan.p, scan_bytes, fl.as<uint32_t>(), scan.as<uint32_t>(), (int)n, st));
				hipLaunchKernelGGL(k_partition, dim3(G), dim3(B), 0, st, s[a].as<uint32_t>(), n, fl.as<uint32_t>(), scan.as<uint32_t>(),
				                   seg_of.as<uint32_t>(), segs[cur].as<Seg>(), axis_of.as<int8_t>(), split_el.as<uint32_t>(),
				                   s_out.as<uint32_t>());
				std::swap(s[a].p, s_out.p);
			}
			hipLaunchKernelGGL(k_children, dim3(Gs), dim3(B), 0, st, segs[cur].as<Seg>(), n_seg, axis_of.as<int8_t>(), split_el.as<uint32_t>(),
			                   child_base.as<uint32_t>(), (const uint2 *)nodes_dev, segs[cur ^ 1].as<Seg>());
			hipLaunchKernelGGL(k_seg_of, dim3(G), dim3(B), 0, st, seg_of.as<uint32_t>(), n, axis_of.as<int8_t>(), split_el.as<uint32_t>(),
			                   child_base.as<uint32_t>());
		}
		PKCHECK(hipStreamSynchronize(st));
		if(n_next == 0) break;
		n_seg = n_next;
		cur ^= 1;
		++level;
	}
	*depth_out = level;
	return hipGetLastError();
}
