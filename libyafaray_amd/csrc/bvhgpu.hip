// GPU build of the BVH4 the traversal kernels consume (devscene.h layout), replacing the host
// build for large meshes.  Reference: the accelerator is built inside render()
// (scene.cc:218, 1032-1060; AcceleratorKdTree::buildTree, accelerator_kdtree.cc:420-628).  Closest
// hits do not depend on the acceleration structure (ties resolve to the lower
// primitive index in the traversal), so a different tree is a legal drop-in; what must match the
// host build is the triangle record (packTriangle, same float operations) and conservativeness.
//
//   1. primitive boxes, centroid bound, 63-bit Morton codes, radix sort (hipcub)
//   2. PLOC (Meister & Bittner 2018): clusters in Morton order; every iteration each cluster finds
//      the neighbour within +-16 positions whose merged box has the smallest surface area (ties ->
//      lower index, which makes the globally best pair mutual, so every iteration merges), mutual
//      pairs merge into a new binary node, one exclusive scan compacts — until one cluster is left
//   3. collapse to BVH4 level by level exactly like the host (open the inner child of largest
//      area until four children), wide nodes numbered level by level (children after parents)
//   4. worst-case stack need bottom-up (levels in reverse), triangle records in Morton order
//
// Everything is deterministic (stable sort, scans, no float atomics).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <climits>
#include <cstdint>
#include <type_traits>
#include <vector>

#include "bvh.h"

namespace
{

constexpr int kB = 256;
#ifndef YAF_PLOC_RADIUS
#define YAF_PLOC_RADIUS 16
#endif
constexpr int kRadius = YAF_PLOC_RADIUS;   // PLOC search window (+-positions in Morton order)
constexpr int kEmpty = INT_MIN;   // empty child slot in the collapse lists (~p for leaves, p >= 0 never hits it)

struct DevBuf
{
	void *p = nullptr;
	~DevBuf() { if(p) (void)hipFree(p); }
	template<class T> T *as() { return reinterpret_cast<T *>(p); }
	hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes < 16 ? 16 : bytes); }
	void *release()
	{
		void *q = p;
		p = nullptr;
		return q;
	}
};

#define BVCHECK(x) do { hipError_t e_ = (x); if(e_ != hipSuccess) return e_; } while(0)

__device__ __forceinline__ float3 ld3(const float *v, int k) { return make_float3(v[3 * k], v[3 * k + 1], v[3 * k + 2]); }

// per-primitive box + per-workgroup partial bound of the centroids
__global__ void __launch_bounds__(kB) k_prims(const float *verts, const int *tris, int n, float4 *blo, float4 *bhi, float *partial)
{
	const int i = blockIdx.x * kB + threadIdx.x;
	float c[3] = {3.4e38f, 3.4e38f, 3.4e38f}, d[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
	if(i < n)
	{
		const float3 a = ld3(verts, tris[3 * i]), b = ld3(verts, tris[3 * i + 1]), e = ld3(verts, tris[3 * i + 2]);
		const float3 lo = make_float3(fminf(fminf(a.x, b.x), e.x), fminf(fminf(a.y, b.y), e.y), fminf(fminf(a.z, b.z), e.z));
		const float3 hi = make_float3(fmaxf(fmaxf(a.x, b.x), e.x), fmaxf(fmaxf(a.y, b.y), e.y), fmaxf(fmaxf(a.z, b.z), e.z));
		blo[i] = make_float4(lo.x, lo.y, lo.z, 0.f);
		bhi[i] = make_float4(hi.x, hi.y, hi.z, 0.f);
		c[0] = d[0] = 0.5f * (lo.x + hi.x);
		c[1] = d[1] = 0.5f * (lo.y + hi.y);
		c[2] = d[2] = 0.5f * (lo.z + hi.z);
	}
	__shared__ float red[6][kB];
	for(int k = 0; k < 3; ++k) { red[k][threadIdx.x] = c[k]; red[3 + k][threadIdx.x] = d[k]; }
	__syncthreads();
	for(int w = kB / 2; w > 0; w >>= 1)
	{
		if(threadIdx.x < w)
			for(int k = 0; k < 3; ++k)
			{
				red[k][threadIdx.x] = fminf(red[k][threadIdx.x], red[k][threadIdx.x + w]);
				red[3 + k][threadIdx.x] = fmaxf(red[3 + k][threadIdx.x], red[3 + k][threadIdx.x + w]);
			}
		__syncthreads();
	}
	if(threadIdx.x < 6) partial[6 * blockIdx.x + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void __launch_bounds__(kB) k_fold(const float *partial, int g, float *cb)
{
	float v[6] = {3.4e38f, 3.4e38f, 3.4e38f, -3.4e38f, -3.4e38f, -3.4e38f};
	for(int b = threadIdx.x; b < g; b += kB)
		for(int k = 0; k < 3; ++k)
		{
			v[k] = fminf(v[k], partial[6 * b + k]);
			v[3 + k] = fmaxf(v[3 + k], partial[6 * b + 3 + k]);
		}
	__shared__ float red[6][kB];
	for(int k = 0; k < 6; ++k) red[k][threadIdx.x] = v[k];
	__syncthreads();
	for(int w = kB / 2; w > 0; w >>= 1)
	{
		if(threadIdx.x < w)
			for(int k = 0; k < 3; ++k)
			{
				red[k][threadIdx.x] = fminf(red[k][threadIdx.x], red[k][threadIdx.x + w]);
				red[3 + k][threadIdx.x] = fmaxf(red[3 + k][threadIdx.x], red[3 + k][threadIdx.x + w]);
			}
		__syncthreads();
	}
	if(threadIdx.x < 6) cb[threadIdx.x] = red[threadIdx.x][0];
}

__device__ __forceinline__ uint64_t spread21(uint64_t x)
{
	x &= 0x1fffffull;
	x = (x | x << 32) & 0x1f00000000ffffull;
	x = (x | x << 16) & 0x1f0000ff0000ffull;
	x = (x | x << 8) & 0x100f00f00f00f00full;
	x = (x | x << 4) & 0x10c30c30c30c30c3ull;
	x = (x | x << 2) & 0x1249249249249249ull;
	return x;
}

__global__ void __launch_bounds__(kB) k_morton(const float4 *blo, const float4 *bhi, int n, const float *cb, uint64_t *keys, int *vals)
{
	const int i = blockIdx.x * kB + threadIdx.x;
	if(i >= n) return;
	const float4 lo = blo[i], hi = bhi[i];
	const float c[3] = {0.5f * (lo.x + hi.x), 0.5f * (lo.y + hi.y), 0.5f * (lo.z + hi.z)};
	uint64_t q[3];
	for(int k = 0; k < 3; ++k)
	{
		const float ext = cb[3 + k] - cb[k];
		float f = ext > 0.f ? (c[k] - cb[k]) / ext * 2097151.f : 0.f;
		f = fminf(fmaxf(f, 0.f), 2097151.f);
		q[k] = (uint64_t)f;
	}
	keys[i] = (spread21(q[0]) << 2) | (spread21(q[1]) << 1) | spread21(q[2]);
	vals[i] = i;
}

// clusters start as the leaves in Morton order; .w of the low corner = node code (~position: leaf)
__global__ void __launch_bounds__(kB) k_leaves(const int *order, int n, const float4 *blo, const float4 *bhi, float4 *lbox_lo,
                                               float4 *lbox_hi, float4 *clo, float4 *chi)
{
	const int p = blockIdx.x * kB + threadIdx.x;
	if(p >= n) return;
	const int t = order[p];
	const float4 lo = blo[t], hi = bhi[t];
	lbox_lo[p] = lo;
	lbox_hi[p] = hi;
	clo[p] = make_float4(lo.x, lo.y, lo.z, __int_as_float(~p));
	chi[p] = hi;
}

__device__ __forceinline__ float halfArea(const float4 &lo, const float4 &hi)
{
	const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
	return dx * dy + dy * dz + dz * dx;
}

// nearest neighbour of every cluster within +-kRadius positions (LDS window)
__global__ void __launch_bounds__(kB) k_nn(const float4 *clo, const float4 *chi, int m, int *nn)
{
	__shared__ float4 slo[kB + 2 * kRadius], shi[kB + 2 * kRadius];
	const int base = blockIdx.x * kB - kRadius;
	for(int k = threadIdx.x; k < kB + 2 * kRadius; k += kB)
	{
		const int j = base + k;
		if(j >= 0 && j < m) { slo[k] = clo[j]; shi[k] = chi[j]; }
	}
	__syncthreads();
	const int i = blockIdx.x * kB + threadIdx.x;
	if(i >= m) return;
	const float4 lo = slo[threadIdx.x + kRadius], hi = shi[threadIdx.x + kRadius];
	float best = __builtin_huge_valf();
	int bj = -1;
	for(int o = -kRadius; o <= kRadius; ++o)
	{
		const int j = i + o;
		if(o == 0 || j < 0 || j >= m) continue;
		const float4 l2 = slo[threadIdx.x + kRadius + o], h2 = shi[threadIdx.x + kRadius + o];
		const float4 ulo = make_float4(fminf(lo.x, l2.x), fminf(lo.y, l2.y), fminf(lo.z, l2.z), 0.f);
		const float4 uhi = make_float4(fmaxf(hi.x, h2.x), fmaxf(hi.y, h2.y), fmaxf(hi.z, h2.z), 0.f);
		const float a = halfArea(ulo, uhi);
		if(a < best) { best = a; bj = j; }   // ascending j, strict: ties keep the lower index
	}
	nn[i] = bj;
}

// flags[i] = (merges here << 32) | (cluster survives); flags[m] = 0 so the scan's last entry is the total
__global__ void __launch_bounds__(kB) k_mflags(const int *nn, int m, uint64_t *flags)
{
	const int i = blockIdx.x * kB + threadIdx.x;
	if(i > m) return;
	if(i == m) { flags[m] = 0; return; }
	const int j = nn[i];
	const bool mutual = nn[j] == i;
	const uint64_t merge = (mutual && i < j) ? 1u : 0u;
	const uint64_t valid = (mutual && i > j) ? 0u : 1u;
	flags[i] = (merge << 32) | valid;
}

__global__ void __launch_bounds__(kB) k_merge(const float4 *clo, const float4 *chi, const int *nn, const uint64_t *scan, int m,
                                              int node_base, float4 *clo2, float4 *chi2, float4 *bn_lo, float4 *bn_hi, int2 *bn_child)
{
	const int i = blockIdx.x * kB + threadIdx.x;
	if(i >= m) return;
	const int j = nn[i];
	const bool mutual = nn[j] == i;
	if(mutual && i > j) return;   // absorbed by its partner
	const uint64_t s = scan[i];
	const int pos = (int)(s & 0xffffffffu);
	float4 lo = clo[i], hi = chi[i];
	if(mutual)
	{
		const int id = node_base + (int)(s >> 32);
		const float4 l2 = clo[j], h2 = chi[j];
		bn_child[id] = make_int2(__float_as_int(lo.w), __float_as_int(l2.w));
		lo = make_float4(fminf(lo.x, l2.x), fminf(lo.y, l2.y), fminf(lo.z, l2.z), __int_as_float(id));
		hi = make_float4(fmaxf(hi.x, h2.x), fmaxf(hi.y, h2.y), fmaxf(hi.z, h2.z), 0.f);
		bn_lo[id] = lo;
		bn_hi[id] = hi;
	}
	clo2[pos] = lo;
	chi2[pos] = hi;
}

// bvh.cc padBox, same float operations
__device__ __forceinline__ void padAxis(float lo, float hi, float &plo, float &phi)
{
	const float mag = fabsf(lo) + fabsf(hi) + (hi - lo);
	const float pad = mag * 1e-5f + 1e-7f;
	plo = lo - pad;
	phi = hi + pad;
}

// collapse step 1: the (up to) W binary children of each wide node of this level (W = 4: the BVH4 every
// traversal reads; W = 8: the BVH8 k_trace's refill loop reads for scenes in global memory)
template<int W>
__global__ void __launch_bounds__(kB) k_collapse_list(const int *wl, int L, const float4 *bn_lo, const float4 *bn_hi,
                                                      const int2 *bn_child, int4 *lists, uint32_t *n_inner)
{
	const int k = blockIdx.x * kB + threadIdx.x;
	if(k > L) return;
	if(k == L) { n_inner[L] = 0; return; }
	const int code = wl[k];
	int list[W];
#pragma unroll
	for(int s = 0; s < W; ++s) list[s] = kEmpty;
	int cnt;
	if(code < 0) { list[0] = code; cnt = 1; }   // a leaf root (one triangle)
	else
	{
		const int2 ch = bn_child[code];
		list[0] = ch.x;
		list[1] = ch.y;
		cnt = 2;
		while(cnt < W)
		{
			int best = -1;
			float best_area = -1.f;
			for(int s = 0; s < cnt; ++s)
				if(list[s] >= 0)
				{
					const float4 lo = bn_lo[list[s]], hi = bn_hi[list[s]];
					const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
					const float a = 2.f * (dx * dy + dy * dz + dz * dx);
					if(a > best_area) { best_area = a; best = s; }
				}
			if(best < 0) break;
			const int2 c = bn_child[list[best]];
			for(int s = cnt; s > best + 1; --s) list[s] = list[s - 1];
			list[best] = c.x;
			list[best + 1] = c.y;
			++cnt;
		}
	}
	uint32_t inner = 0;
#pragma unroll
	for(int s = 0; s < W; ++s) inner += (list[s] != kEmpty && list[s] >= 0) ? 1u : 0u;
#pragma unroll
	for(int q = 0; q < W / 4; ++q) lists[(size_t)k * (W / 4) + q] = make_int4(list[4 * q], list[4 * q + 1], list[4 * q + 2], list[4 * q + 3]);
	n_inner[k] = inner;
}

// collapse step 2: write the wide nodes of this level, queue their inner children as the next level.
// W = 4: 8 float4 (lo.x, hi.x, lo.y, hi.y, lo.z, hi.z, child, count — four lanes each); W = 8: 16 float4,
// the same eight arrays with eight lanes (two float4 each)
template<int W>
__global__ void __launch_bounds__(kB) k_collapse_write(const int4 *lists, int L, const uint32_t *off, int ls, int le,
                                                       const float4 *bn_lo, const float4 *bn_hi, const float4 *lbox_lo,
                                                       const float4 *lbox_hi, float4 *nodes, int *wl_next)
{
	const int k = blockIdx.x * kB + threadIdx.x;
	if(k >= L) return;
	int list[W];
#pragma unroll
	for(int q = 0; q < W / 4; ++q)
	{
		const int4 l4 = lists[(size_t)k * (W / 4) + q];
		list[4 * q] = l4.x; list[4 * q + 1] = l4.y; list[4 * q + 2] = l4.z; list[4 * q + 3] = l4.w;
	}
	float o[8 * W];
	int r = 0;
	for(int s = 0; s < W; ++s)
	{
		const int c = list[s];
		float lo[3] = {1.f, 1.f, 1.f}, hi[3] = {-1.f, -1.f, -1.f};
		int child = -1, count = 0;
		if(c != kEmpty)
		{
			float4 blo, bhi;
			if(c < 0) { blo = lbox_lo[~c]; bhi = lbox_hi[~c]; child = c; count = 1; }
			else
			{
				blo = bn_lo[c];
				bhi = bn_hi[c];
				const int slot = (int)off[k] + r;
				child = le + slot;
				wl_next[slot] = c;
				++r;
			}
			padAxis(blo.x, bhi.x, lo[0], hi[0]);
			padAxis(blo.y, bhi.y, lo[1], hi[1]);
			padAxis(blo.z, bhi.z, lo[2], hi[2]);
		}
		o[0 * W + s] = lo[0]; o[1 * W + s] = hi[0];
		o[2 * W + s] = lo[1]; o[3 * W + s] = hi[1];
		o[4 * W + s] = lo[2]; o[5 * W + s] = hi[2];
		o[6 * W + s] = __int_as_float(child);
		o[7 * W + s] = __int_as_float(count);
	}
	float4 *dst = nodes + 2 * W * (size_t)(ls + k);
	for(int q = 0; q < 2 * W; ++q) dst[q] = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
}

// worst-case traversal stack entries below each wide node (bvh.cc: deferred siblings along a path)
template<int W>
__global__ void __launch_bounds__(kB) k_need(const float4 *nodes, int ls, int le, int *need)
{
	const int w = ls + blockIdx.x * kB + threadIdx.x;
	if(w >= le) return;
	const float *nd = reinterpret_cast<const float *>(nodes + 2 * W * (size_t)w);
	int inner = 0, deep = 0;
	for(int s = 0; s < W; ++s)
	{
		const int c = __float_as_int(nd[6 * W + s]), k = __float_as_int(nd[7 * W + s]);
		if(c >= 0 && k == 0) { ++inner; deep = max(deep, need[c]); }
	}
	need[w] = max(0, inner - 1) + deep;
}

// ---- quantised BVH8 (k_trace's refill loop over global-memory scenes, opt-in) ----
// Node (128 B, the first 80 B read per visit): origin (the children's padded lower corner), per axis a
// power-of-two quantum (biased exponent byte), inner / leaf child masks, the first inner child's node
// index (inner children are consecutive) and the first of the node's leaf triangles (copied
// consecutively into the BVH8's own triangle array), then per axis the children's lower / upper planes
// as bytes: plane = origin + q · 2^e with q rounded outwards (one quantum of margin) — every decoded box
// contains the float box, which contains the padded triangle box.
//   dw0-2 origin, dw3 exps x/y/z | inner mask << 24, dw4 leaf mask, dw5 inner base, dw6 tri base, dw7 0,
//   dw8-9 lo.x[8], dw10-11 hi.x[8], dw12-13 lo.y, dw14-15 hi.y, dw16-17 lo.z, dw18-19 hi.z
__global__ void __launch_bounds__(kB) k_q8_count(const float4 *nodes8, int n, uint32_t *leaves)
{
	const int w = blockIdx.x * kB + threadIdx.x;
	if(w > n) return;
	if(w == n) { leaves[n] = 0; return; }
	const float *nd = reinterpret_cast<const float *>(nodes8 + 16 * (size_t)w);
	uint32_t c = 0;
	for(int s = 0; s < 8; ++s) c += (__float_as_int(nd[6 * 8 + s]) < 0 && __float_as_int(nd[7 * 8 + s]) == 1) ? 1u : 0u;
	leaves[w] = c;
}

__device__ __forceinline__ int q8Exp(float extent)
{
	// the smallest power of two s with extent <= 254 s (so that ceil + one quantum of margin stays <= 255)
	const float need = extent / 254.f;
	int e = -126;
	if(need > 0.f)
	{
		int ex;
		const float m = frexpf(need, &ex);   // need = m 2^ex, m in [0.5, 1)
		e = (m == 0.5f) ? ex - 1 : ex;
		// float division rounding: make sure extent <= 254 * 2^e holds
		while(ldexpf(254.f, e) < extent) ++e;
	}
	return max(-126, min(127, e));
}

__global__ void __launch_bounds__(kB) k_q8_write(const float4 *nodes8, int n, const uint32_t *tri_base, const float4 *tris_in,
                                                 float4 *qnodes, float4 *tris8)
{
	const int w = blockIdx.x * kB + threadIdx.x;
	if(w >= n) return;
	const float *nd = reinterpret_cast<const float *>(nodes8 + 16 * (size_t)w);
	float lo[3] = {3.4e38f, 3.4e38f, 3.4e38f}, hi[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
	uint32_t inner = 0, leaf = 0;
	int inner_base = -1;
	for(int s = 0; s < 8; ++s)
	{
		const int c = __float_as_int(nd[6 * 8 + s]), k = __float_as_int(nd[7 * 8 + s]);
		const bool isl = c < 0 && k == 1, isi = c >= 0;
		if(!isl && !isi) continue;
		if(isi) { inner |= 1u << s; if(inner_base < 0) inner_base = c; }
		else leaf |= 1u << s;
		for(int a = 0; a < 3; ++a)
		{
			lo[a] = fminf(lo[a], nd[(2 * a) * 8 + s]);
			hi[a] = fmaxf(hi[a], nd[(2 * a + 1) * 8 + s]);
		}
	}
	uint32_t q[6][2] = {{0u, 0u}, {0u, 0u}, {0u, 0u}, {0u, 0u}, {0u, 0u}, {0u, 0u}};
	int ex[3] = {0, 0, 0};
	for(int a = 0; a < 3; ++a)
	{
		if(!(lo[a] <= hi[a])) { lo[a] = 0.f; hi[a] = 0.f; }
		ex[a] = q8Exp(hi[a] - lo[a]);
	}
	uint32_t rank = 0;
	for(int s = 0; s < 8; ++s)
	{
		const int c = __float_as_int(nd[6 * 8 + s]);
		uint32_t bl[3] = {255u, 255u, 255u}, bh[3] = {0u, 0u, 0u};   // empty slot: inverted box
		if((inner | leaf) & (1u << s))
			for(int a = 0; a < 3; ++a)
			{
				const float sc = ldexpf(1.f, ex[a]);
				const float fl = floorf((nd[(2 * a) * 8 + s] - lo[a]) / sc) - 1.f;
				const float fh = ceilf((nd[(2 * a + 1) * 8 + s] - lo[a]) / sc) + 1.f;
				bl[a] = (uint32_t)fminf(fmaxf(fl, 0.f), 255.f);
				bh[a] = (uint32_t)fminf(fmaxf(fh, 0.f), 255.f);
			}
		for(int a = 0; a < 3; ++a)
		{
			q[2 * a][s >> 2] |= bl[a] << (8 * (s & 3));
			q[2 * a + 1][s >> 2] |= bh[a] << (8 * (s & 3));
		}
		if(leaf & (1u << s))
		{
			const size_t dst = (size_t)tri_base[w] + rank++;
			for(int r = 0; r < 3; ++r) tris8[3 * dst + r] = tris_in[3 * (size_t)(~c) + r];
		}
	}
	uint32_t o[32];
	o[0] = __float_as_uint(lo[0]); o[1] = __float_as_uint(lo[1]); o[2] = __float_as_uint(lo[2]);
	o[3] = (uint32_t)(ex[0] + 127) | ((uint32_t)(ex[1] + 127) << 8) | ((uint32_t)(ex[2] + 127) << 16) | (inner << 24);
	o[4] = leaf;
	o[5] = (uint32_t)max(inner_base, 0);
	o[6] = tri_base[w];
	o[7] = 0u;
	for(int p = 0; p < 6; ++p) { o[8 + 2 * p] = q[p][0]; o[9 + 2 * p] = q[p][1]; }
	for(int k = 20; k < 32; ++k) o[k] = 0u;
	float4 *dst = qnodes + 8 * (size_t)w;
	for(int k = 0; k < 8; ++k) dst[k] = make_float4(__uint_as_float(o[4 * k]), __uint_as_float(o[4 * k + 1]), __uint_as_float(o[4 * k + 2]), __uint_as_float(o[4 * k + 3]));
}

// bvh.cc packTriangle, same float operations (the eps of the exact test must match the oracle's)
__global__ void __launch_bounds__(kB) k_pack(const int *order, int n, const float *verts, const int *tris, float4 *out)
{
	const int p = blockIdx.x * kB + threadIdx.x;
	if(p >= n) return;
	const int t = order[p];
	const float3 v0 = ld3(verts, tris[3 * t]), v1 = ld3(verts, tris[3 * t + 1]), v2 = ld3(verts, tris[3 * t + 2]);
	const float e1[3] = {v1.x - v0.x, v1.y - v0.y, v1.z - v0.z};
	const float e2[3] = {v2.x - v0.x, v2.y - v0.y, v2.z - v0.z};
	const float l1 = sqrtf(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
	const float l2 = sqrtf(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
	const float eps = 0.1f * 0.00005f * ((l1 < l2) ? l2 : l1);
	out[3 * (size_t)p] = make_float4(v0.x, v0.y, v0.z, eps);
	out[3 * (size_t)p + 1] = make_float4(e1[0], e1[1], e1[2], __int_as_float(t));
	out[3 * (size_t)p + 2] = make_float4(e2[0], e2[1], e2[2], 0.f);
}

__global__ void k_empty_root(float4 *nodes)
{
	const int q = threadIdx.x;
	if(q >= 8) return;
	float4 v;
	if(q < 6) v = (q & 1) ? make_float4(-1.f, -1.f, -1.f, -1.f) : make_float4(1.f, 1.f, 1.f, 1.f);
	else if(q == 6) v = make_float4(__int_as_float(-1), __int_as_float(-1), __int_as_float(-1), __int_as_float(-1));
	else v = make_float4(0.f, 0.f, 0.f, 0.f);
	nodes[q] = v;
}

inline int blocks(long n) { return (int)((n + kB - 1) / kB); }

} // namespace

// verts_dev: xyz floats, tris_dev: 3 vertex indices per triangle (both on the device).
// Allocates *nodes_out (8 float4 per wide node) and *tris_out (3 float4 per triangle, Morton
// order); the caller owns them (hipFree).  *n_nodes, *depth (wide levels), *stack_need as bvh.h.
// w8 (optional): the same binary tree collapsed to a BVH8 as well (16 float4 per node, the same triangle
// records); the caller owns w8->nodes.
extern "C" hipError_t yafamd_build_bvh_gpu(const float *verts_dev, const int *tris_dev, int n, void **nodes_out, void **tris_out,
                                           int *n_nodes, int *depth, int *stack_need, int *ploc_iters, yafamd::YafBvh8 *w8, hipStream_t st)
{
	*nodes_out = *tris_out = nullptr;
	if(w8) *w8 = yafamd::YafBvh8{};
	DevBuf nodes, trisb;
	const int cap_nodes = n > 1 ? n - 1 : 1;
	BVCHECK(nodes.alloc((size_t)cap_nodes * 8 * sizeof(float4)));
	BVCHECK(trisb.alloc((size_t)(n > 0 ? n : 1) * 3 * sizeof(float4)));
	*ploc_iters = 0;
	if(n == 0)
	{
		hipLaunchKernelGGL(k_empty_root, dim3(1), dim3(64), 0, st, nodes.as<float4>());
		BVCHECK(hipGetLastError());
		BVCHECK(hipStreamSynchronize(st));
		*n_nodes = 1;
		*depth = 1;
		*stack_need = 0;
		*nodes_out = nodes.release();
		*tris_out = trisb.release();
		return hipSuccess;
	}
	const int G = blocks(n);
	DevBuf blo, bhi, partial, cb, keys, keys2, vals, order, lbox_lo, lbox_hi, c[4], nn, flags, scan, bn_lo, bn_hi, bn_child, tmp;
	BVCHECK(blo.alloc((size_t)n * 16));
	BVCHECK(bhi.alloc((size_t)n * 16));
	BVCHECK(partial.alloc((size_t)G * 6 * 4));
	BVCHECK(cb.alloc(6 * 4));
	BVCHECK(keys.alloc((size_t)n * 8));
	BVCHECK(keys2.alloc((size_t)n * 8));
	BVCHECK(vals.alloc((size_t)n * 4));
	BVCHECK(order.alloc((size_t)n * 4));
	BVCHECK(lbox_lo.alloc((size_t)n * 16));
	BVCHECK(lbox_hi.alloc((size_t)n * 16));
	for(DevBuf &b : c) BVCHECK(b.alloc((size_t)n * 16));
	BVCHECK(nn.alloc((size_t)n * 4));
	BVCHECK(flags.alloc((size_t)(n + 1) * 8));
	BVCHECK(scan.alloc((size_t)(n + 1) * 8));
	BVCHECK(bn_lo.alloc((size_t)cap_nodes * 16));
	BVCHECK(bn_hi.alloc((size_t)cap_nodes * 16));
	BVCHECK(bn_child.alloc((size_t)cap_nodes * 8));

	hipLaunchKernelGGL(k_prims, dim3(G), dim3(kB), 0, st, verts_dev, tris_dev, n, blo.as<float4>(), bhi.as<float4>(), partial.as<float>());
	hipLaunchKernelGGL(k_fold, dim3(1), dim3(kB), 0, st, partial.as<float>(), G, cb.as<float>());
	hipLaunchKernelGGL(k_morton, dim3(G), dim3(kB), 0, st, blo.as<float4>(), bhi.as<float4>(), n, cb.as<float>(), keys.as<uint64_t>(), vals.as<int>());
	BVCHECK(hipGetLastError());
	size_t sort_bytes = 0, scan_bytes = 0;
	BVCHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, keys.as<uint64_t>(), keys2.as<uint64_t>(), vals.as<int>(),
	                                           order.as<int>(), n, 0, 63, st));
	BVCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, flags.as<uint64_t>(), scan.as<uint64_t>(), n + 1, st));
	size_t scan32_bytes = 0;
	BVCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan32_bytes, (uint32_t *)nullptr, (uint32_t *)nullptr, n + 1, st));
	BVCHECK(tmp.alloc(std::max(sort_bytes, std::max(scan_bytes, scan32_bytes))));
	BVCHECK(hipcub::DeviceRadixSort::SortPairs(tmp.p, sort_bytes, keys.as<uint64_t>(), keys2.as<uint64_t>(), vals.as<int>(),
	                                           order.as<int>(), n, 0, 63, st));
	hipLaunchKernelGGL(k_leaves, dim3(G), dim3(kB), 0, st, order.as<int>(), n, blo.as<float4>(), bhi.as<float4>(), lbox_lo.as<float4>(),
	                   lbox_hi.as<float4>(), c[0].as<float4>(), c[1].as<float4>());
	hipLaunchKernelGGL(k_pack, dim3(G), dim3(kB), 0, st, order.as<int>(), n, verts_dev, tris_dev, trisb.as<float4>());
	BVCHECK(hipGetLastError());

	// PLOC
	int m = n, node_base = 0, cur = 0;
	uint64_t *tot = nullptr;
	BVCHECK(hipHostMalloc((void **)&tot, sizeof(uint64_t)));
	struct HostFree { uint64_t *p; ~HostFree() { if(p) (void)hipHostFree(p); } } tot_guard{tot};
	while(m > 1)
	{
		float4 *clo = c[2 * cur].as<float4>(), *chi = c[2 * cur + 1].as<float4>();
		float4 *clo2 = c[2 * (cur ^ 1)].as<float4>(), *chi2 = c[2 * (cur ^ 1) + 1].as<float4>();
		hipLaunchKernelGGL(k_nn, dim3(blocks(m)), dim3(kB), 0, st, clo, chi, m, nn.as<int>());
		hipLaunchKernelGGL(k_mflags, dim3(blocks(m + 1)), dim3(kB), 0, st, nn.as<int>(), m, flags.as<uint64_t>());
		BVCHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, scan_bytes, flags.as<uint64_t>(), scan.as<uint64_t>(), m + 1, st));
		hipLaunchKernelGGL(k_merge, dim3(blocks(m)), dim3(kB), 0, st, clo, chi, nn.as<int>(), scan.as<uint64_t>(), m, node_base, clo2, chi2,
		                   bn_lo.as<float4>(), bn_hi.as<float4>(), bn_child.as<int2>());
		BVCHECK(hipGetLastError());
		BVCHECK(hipMemcpyAsync(tot, scan.as<uint64_t>() + m, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
		BVCHECK(hipStreamSynchronize(st));
		const int merges = (int)(*tot >> 32), valid = (int)(*tot & 0xffffffffu);
		if(merges == 0 || merges + valid != m) return hipErrorUnknown;   // cannot happen (the best pair is mutual)
		node_base += merges;
		m = valid;
		cur ^= 1;
		++*ploc_iters;
	}
	if(n > 1 && node_base != n - 1) return hipErrorUnknown;

	// collapse to BVH4 (and BVH8), level by level
	DevBuf wl[2], lists, n_inner, off, need;
	BVCHECK(wl[0].alloc((size_t)cap_nodes * 4));
	BVCHECK(wl[1].alloc((size_t)cap_nodes * 4));
	// W / 4 int4 per wide node of a level (k_collapse_list): at most 2 x 16 B for the BVH8, and a level never
	// holds more wide nodes than the binary tree has inner nodes (cap_nodes)
	BVCHECK(lists.alloc((size_t)cap_nodes * 2 * sizeof(int4)));
	BVCHECK(n_inner.alloc((size_t)(cap_nodes + 1) * 4));
	BVCHECK(off.alloc((size_t)(cap_nodes + 1) * 4));
	BVCHECK(need.alloc((size_t)cap_nodes * 4));
	const int root = n == 1 ? ~0 : n - 2;   // the last merge made the root
	uint32_t *tot32 = reinterpret_cast<uint32_t *>(tot);
	auto collapse = [&](auto width, float4 *dst, int *n_out, int *depth_out, int *need_out) -> hipError_t {
		constexpr int W = decltype(width)::value;
		BVCHECK(hipMemcpyAsync(wl[0].p, &root, sizeof(int), hipMemcpyHostToDevice, st));
		std::vector<std::pair<int, int>> levels;
		int ls = 0, L = 1, w = 0;
		while(L > 0)
		{
			const int le = ls + L;
			levels.push_back({ls, le});
			hipLaunchKernelGGL(k_collapse_list<W>, dim3(blocks(L + 1)), dim3(kB), 0, st, wl[w].as<int>(), L, bn_lo.as<float4>(), bn_hi.as<float4>(),
			                   bn_child.as<int2>(), lists.as<int4>(), n_inner.as<uint32_t>());
			BVCHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, scan32_bytes, n_inner.as<uint32_t>(), off.as<uint32_t>(), L + 1, st));
			hipLaunchKernelGGL(k_collapse_write<W>, dim3(blocks(L)), dim3(kB), 0, st, lists.as<int4>(), L, off.as<uint32_t>(), ls, le,
			                   bn_lo.as<float4>(), bn_hi.as<float4>(), lbox_lo.as<float4>(), lbox_hi.as<float4>(), dst, wl[w ^ 1].as<int>());
			BVCHECK(hipGetLastError());
			BVCHECK(hipMemcpyAsync(tot32, off.as<uint32_t>() + L, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
			BVCHECK(hipStreamSynchronize(st));
			const int next = (int)*tot32;
			if(le + next > cap_nodes) return hipErrorUnknown;
			ls = le;
			L = next;
			w ^= 1;
		}
		*n_out = ls;
		*depth_out = (int)levels.size();
		for(int l = (int)levels.size() - 1; l >= 0; --l)
			hipLaunchKernelGGL(k_need<W>, dim3(blocks(levels[l].second - levels[l].first)), dim3(kB), 0, st, dst, levels[l].first, levels[l].second,
			                   need.as<int>());
		BVCHECK(hipGetLastError());
		BVCHECK(hipMemcpyAsync(tot32, need.p, sizeof(int), hipMemcpyDeviceToHost, st));
		BVCHECK(hipStreamSynchronize(st));
		*need_out = (int)*tot32;
		return hipSuccess;
	};
	BVCHECK(collapse(std::integral_constant<int, 4>{}, nodes.as<float4>(), n_nodes, depth, stack_need));
	if(w8)
	{
		// the 8-wide collapse in float, then quantised (k_q8_*) with the leaves' triangles in node order
		DevBuf nodes8, qnodes, tris8, leaves, base;
		BVCHECK(nodes8.alloc((size_t)cap_nodes * 16 * sizeof(float4)));
		BVCHECK(collapse(std::integral_constant<int, 8>{}, nodes8.as<float4>(), &w8->n_nodes, &w8->depth, &w8->stack_need));
		const int n8 = w8->n_nodes;
		BVCHECK(leaves.alloc((size_t)(n8 + 1) * 4));
		BVCHECK(base.alloc((size_t)(n8 + 1) * 4));
		hipLaunchKernelGGL(k_q8_count, dim3(blocks(n8 + 1)), dim3(kB), 0, st, nodes8.as<float4>(), n8, leaves.as<uint32_t>());
		size_t qb = 0;
		BVCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, qb, leaves.as<uint32_t>(), base.as<uint32_t>(), n8 + 1, st));
		DevBuf qtmp;
		BVCHECK(qtmp.alloc(qb));
		BVCHECK(hipcub::DeviceScan::ExclusiveSum(qtmp.p, qb, leaves.as<uint32_t>(), base.as<uint32_t>(), n8 + 1, st));
		BVCHECK(qnodes.alloc((size_t)std::max(1, n8) * 8 * sizeof(float4)));
		BVCHECK(tris8.alloc((size_t)n * 3 * sizeof(float4)));
		hipLaunchKernelGGL(k_q8_write, dim3(blocks(n8)), dim3(kB), 0, st, nodes8.as<float4>(), n8, base.as<uint32_t>(), trisb.as<float4>(),
		                   qnodes.as<float4>(), tris8.as<float4>());
		BVCHECK(hipGetLastError());
		BVCHECK(hipStreamSynchronize(st));
		w8->nodes = qnodes.release();
		w8->tris = tris8.release();
	}
	*nodes_out = nodes.release();
	*tris_out = trisb.release();
	return hipSuccess;
}

// ---------------------------------------------------------------------------------------------
// Ray binning for the BVH8 refill loop (r06, YAFARAY_AMD_RAY_BIN=1): the closest rays of
// every queue segment ordered by (direction octant, Morton code of the origin in the scene bounds), so that the
// waves traversing at the same time read the same part of the tree.  One 32-bit key per queue slot: the
// segment in the high 10 bits (the sort then keeps each segment's slots inside the segment), octant (3 bits),
// a 19-bit Morton code (6 / 6 / 7 bits of x / y / z); empty slots after the segment's rays and "no ray" entries
// sort to the segment's end.  k_trace's refill loop traces entry a0 + j's ray at perm[a0 + j] and writes the hit
// there: every ray's query is unchanged, so hits are identical.
// ---------------------------------------------------------------------------------------------
#include "devscene.h"

namespace
{
__device__ __forceinline__ uint32_t spreadBits(uint32_t v)   // bit i -> bit 3 i (v < 2^7)
{
	uint32_t r = 0;
#pragma unroll
	for(int i = 0; i < 7; ++i) r |= ((v >> i) & 1u) << (3 * i);
	return r;
}

__global__ void __launch_bounds__(256) k_ray_keys(yafamd::DevQueues Q, const uint32_t *n_active, uint32_t n_seg, uint32_t cap_a, float3 lo,
                                                  float3 inv_ext, uint32_t *keys, uint32_t *iota)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if(i >= n_seg * cap_a) return;
	const uint32_t s = i / cap_a, j = i - s * cap_a;
	uint32_t k = 0x3fffffu;   // empty slot: the segment's end
	if(j < n_active[s])
	{
		const float dx = Q.ray_d[3 * (size_t)i], dy = Q.ray_d[3 * (size_t)i + 1], dz = Q.ray_d[3 * (size_t)i + 2];
		if(dx != dx) k = 0x3ffffeu;   // no ray this iteration
		else
		{
			const float ox = Q.ray_o[3 * (size_t)i], oy = Q.ray_o[3 * (size_t)i + 1], oz = Q.ray_o[3 * (size_t)i + 2];
			const uint32_t oct = (dx < 0.f ? 1u : 0u) | (dy < 0.f ? 2u : 0u) | (dz < 0.f ? 4u : 0u);
			auto q = [](float v, float l, float inv, uint32_t m) {
				const float t = (v - l) * inv;
				const int c = (int)(t * (float)(m + 1u));
				return (uint32_t)(c < 0 ? 0 : (c > (int)m ? (int)m : c));
			};
			const uint32_t mx = q(ox, lo.x, inv_ext.x, 63u), my = q(oy, lo.y, inv_ext.y, 63u), mz = q(oz, lo.z, inv_ext.z, 127u);
			const uint32_t morton = (spreadBits(mx) | (spreadBits(my) << 1) | (spreadBits(mz) << 2)) & 0x7ffffu;
			k = (oct << 19) | morton;
		}
	}
	keys[i] = (s << 22) | k;
	iota[i] = i;
}
} // namespace

// scratch: keys_in / keys_out / iota / perm (n_seg * cap_a words each) + the sort's temporary storage
extern "C" hipError_t yafamd_ray_bin(const yafamd::DevQueues *Q, const yafamd::DevCounters *cnt, uint32_t n_seg, uint32_t cap_a, const float *lo,
                                     const float *hi, uint32_t *keys_in, uint32_t *keys_out, uint32_t *iota, uint32_t *perm, void *tmp,
                                     size_t *tmp_bytes, hipStream_t st)
{
	const size_t n = (size_t)n_seg * cap_a;
	if(n_seg > 1024u || n > 0x7fffffffu) return hipErrorInvalidValue;
	if(!tmp) return hipcub::DeviceRadixSort::SortPairs(nullptr, *tmp_bytes, keys_in, keys_out, iota, perm, (int)n, 0, 32, st);
	const float3 l = make_float3(lo[0], lo[1], lo[2]);
	const float3 ie = make_float3(1.f / fmaxf(hi[0] - lo[0], 1e-20f), 1.f / fmaxf(hi[1] - lo[1], 1e-20f), 1.f / fmaxf(hi[2] - lo[2], 1e-20f));
	hipLaunchKernelGGL(k_ray_keys, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, *Q, cnt->n_active, n_seg, cap_a, l, ie, keys_in, iota);
	return hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, keys_in, keys_out, iota, perm, (int)n, 0, 32, st);
}
