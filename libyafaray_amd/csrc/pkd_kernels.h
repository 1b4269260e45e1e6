// Device code of the photon kd-tree build (pkd.hip): node splitting, partitions and the LDS
// subtree kernel.  Kept apart from the host driver so tools/pkd_emu.cc can run the same kernels
// on CPU threads (one std::thread per lane, barriers for __syncthreads) under ThreadSanitizer.
#pragma once

// Checked build (-DPKD_CHECK, tools/pkd_check.py): every computed index is range-checked before
// use; a failure records the first offending source line and the index is clamped, so a broken
// invariant shows up as a line number instead of a memory fault.
#ifdef PKD_CHECK
__device__ uint32_t g_pkd_err;
#define PK_GUARD(cond, idx) do { if(!(cond)) { atomicCAS(&g_pkd_err, 0u, (uint32_t)__LINE__); (idx) = 0; } } while(0)
#else
#define PK_GUARD(cond, idx) do {} while(0)
#endif

// status words of the decoupled look-back (k_level_partition): device atomics at agent scope, or
// the emulator's host atomics
#ifdef PKD_EMU
inline uint64_t pkLoadStatus(const uint64_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void pkStoreStatus(uint64_t *p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
inline void pkBackoff() {}
#else
// relaxed: a status word carries its tag and its count together, so no other data has to be
// ordered with it (acquire loads invalidate the CU's vector cache on every poll: measured 2.4x slower)
__device__ __forceinline__ uint64_t pkLoadStatus(const uint64_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void pkStoreStatus(uint64_t *p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void pkBackoff() { __builtin_amdgcn_s_sleep(2); }
#endif

namespace yafamd_pkd
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

// Component selects on values already in registers.  Taking the record by reference let the
// compiler turn the select into a branchy address computation whose lowering dropped the axis-2
// case in one unrolled copy of the flag loop (the key was then read from LDS address 0); loading
// the whole record first keeps the selects as v_cndmask.
__device__ __forceinline__ float coordOf(const float4 p, int a)
{
	float c = p.x;
	c = (a == 1) ? p.y : c;
	c = (a == 2) ? p.z : c;
	return c;
}
__device__ __forceinline__ uint32_t keyOf(const uint4 r, int a)
{
	uint32_t k = r.x;
	k = (a == 1) ? r.y : k;
	k = (a == 2) ? r.z : k;
	return k;
}

// orderable key of a float coordinate; -0 and +0 compare equal in the reference's comparator
__device__ __forceinline__ uint32_t orderKey(float f)
{
	if(f == 0.f) f = 0.f;
	const uint32_t u = __float_as_uint(f);
	return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// the coordinate back from its orderable key (exact: the key keeps every bit of the float, except that
// -0 became +0 — callers load the coordinate itself for a zero key)
__device__ __forceinline__ float keyCoord(uint32_t k)
{
	return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
constexpr uint32_t kZeroKey = 0x80000000u;

// "left of the median" in the (coordinate, index) order of `axis`
__device__ __forceinline__ bool leftOf(const uint4 r, uint32_t axis, uint32_t med_key, uint32_t med_idx)
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

// the three sort keys (one array per axis for the radix sorts) and the same keys interleaved with
// the index (the record every list entry carries)
__global__ void k_keys(const float4 *pos, uint32_t n, uint32_t *kx, uint32_t *ky, uint32_t *kz, uint32_t *iota, uint4 *kxyz)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= n) return;
	const float4 p = pos[i];
	const uint4 r = make_uint4(orderKey(p.x), orderKey(p.y), orderKey(p.z), i);
	kx[i] = r.x;
	ky[i] = r.y;
	kz[i] = r.z;
	iota[i] = i;
	kxyz[i] = r;
}

// list entry p = the record of the p-th photon in sorted order: one 16-byte gather (three 4-byte
// gathers from the per-axis arrays touched three cache lines per entry: 0.93 -> 0.4 ms per list at
// 19.6 M photons)
__global__ void k_records(const uint32_t *sorted_idx, uint32_t n, const uint4 *kxyz, uint4 *rec)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	rec[p] = kxyz[sorted_idx[p]];
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
__global__ void k_level_split(const Seg *segs, uint32_t n_seg, uint32_t n, const uint4 *rx, const uint4 *ry, const uint4 *rz, const float4 *pos,
                              uint4 *nodes, Split *splits, Seg *next, uint32_t *seg_nl)
{
	uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
	if(s >= n_seg) return;
	const Seg g = segs[s];
	const int axis = largestAxis(g.lo, g.hi);
	uint32_t se = (g.start + g.end) / 2;
	PK_GUARD(g.start < se && g.end <= n, se);
	uint4 med = (axis == 0 ? rx : (axis == 1 ? ry : rz))[se];
	PK_GUARD(med.w < n, med.w);
	const float split_pos = coordOf(pos[med.w], axis);
	const uint32_t nl = se - g.start;
	uint32_t right = g.node + 2u * nl;
	uint32_t nd = g.node;
	PK_GUARD(right < 2 * n - 1 && nd < right, nd);
	PK_GUARD(2 * s + 1 < n, s);
	nodes[nd] = make_uint4(__float_as_uint(split_pos), 0u, 0u, (uint32_t)axis | (right << 2));
	splits[s] = {(uint32_t)axis, se, keyOf(med, axis), med.w};
	if(seg_nl) seg_nl[s] = nl;   // entries going left (k_level_partition: their exclusive sum over segments)
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
	uint32_t n;
	__host__ __device__ uint32_t operator()(const uint32_t &p_in) const
	{
		uint32_t p = p_in;
		PK_GUARD(p < n, p);
		uint32_t so = seg_of[p];
		PK_GUARD(so < n, so);
		const Split sp = splits[so];
		const uint4 r = rec[p];
		return leftOf(r, sp.axis, sp.med_key, sp.med_idx) ? 1u : 0u;
	}
};

__global__ void k_partition(const uint4 *rec, uint32_t n, const uint32_t *scan, const uint32_t *seg_of, const Seg *segs, const Split *splits,
                            uint4 *out)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	uint32_t s = seg_of[p];
	PK_GUARD(s < n, s);
	const Split sp = splits[s];
	const uint4 r = rec[p];
	const uint32_t start = segs[s].start;
	const uint32_t left_before = scan[p] - scan[start];
	uint32_t np = leftOf(r, sp.axis, sp.med_key, sp.med_idx) ? start + left_before : sp.split_el + ((p - start) - left_before);
	PK_GUARD(np < n, np);
	out[np] = r;
}

__global__ void k_seg_of(uint32_t *seg_of, uint32_t n, const Split *splits)
{
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	uint32_t s = seg_of[p];
	PK_GUARD(s < n, s);
	seg_of[p] = 2u * s + (p < splits[s].split_el ? 0u : 1u);
}

// ---- one top level of all three lists in one pass (decoupled look-back) ----
// Replaces LeftFlag scan + k_partition per list + k_seg_of: every entry's list position after the
// stable partition needs the number of left-going entries before it in its segment = (left flags
// before it in the whole list) - (left entries of the earlier segments).  The second term is known
// in advance (segment j sends exactly split_el - start left in every list: seg_left, an exclusive
// sum over the segments); the first is a single-pass scan: each tile of kPartTile entries counts
// its flags, publishes the count, and looks back over its predecessors' published counts / prefixes
// (Merrill & Garland's decoupled look-back).  Tiles are numbered by a ticket taken at start, so every
// tile a workgroup waits on has already started.  Per entry: the record (16 B) read once and written
// once; its segment follows from its position (segOfPos: r04, replacing a per-entry segment array
// read per list and rewritten per level).  Measured on
// C5 (19.6 M photons, 17 top levels): 0.76 ms per level for the three lists, kd build 22.2 -> 20.3 ms
// per frame against the scan + partition passes (tiles of 4 / 16 items per thread: 20.8 / 24.6 ms).
#ifndef YAF_PART_ITEMS
#define YAF_PART_ITEMS 8
#endif
#ifndef YAF_PART_NT
#define YAF_PART_NT 1
#endif
#ifndef YAF_PART_PRELOAD
#define YAF_PART_PRELOAD 1
#endif
#ifndef YAF_SUB_FAST
#define YAF_SUB_FAST 1
#endif
#ifndef YAF_SUB_2BUF
#define YAF_SUB_2BUF 0
#endif
constexpr int kPartItems = YAF_PART_ITEMS;
constexpr uint32_t kPartThreads = 256;
constexpr uint32_t kPartTile = kPartThreads * kPartItems;
constexpr uint32_t kPartSpinLimit = 1u << 22;

struct PartArgs
{
	const uint4 *in[3];
	uint4 *out[3];
	uint32_t level;      // top level d: 2^d segments, segment s = the path bits of the recursive halving
	const Seg *segs;
	const Split *splits;
	const uint32_t *seg_left;
	uint32_t n, n_tiles, epoch;
	// the entries [lo, hi) partitioned: the whole list, or the owned subtrees of a group member's build
	// (consecutive level-D segments); segs / splits / seg_left hold n_seg segments, the first being global
	// segment seg_base of this level
	uint32_t lo, hi, seg_base, n_seg;
	uint32_t *ticket;
	uint64_t *status;    // 3 x n_tiles: (tag << 32) | count; tag 2 epoch = tile count, 2 epoch + 1 = inclusive prefix
	uint32_t *err;       // set when a look-back gave up (spin limit): the build reports an error
};

// Segment of list position e at top level d: level d's segments are the recursive halving of [0, n)
// at (start + end) / 2 (every node of the top phase splits, k_level_split), segment s = the path bits.
__device__ __forceinline__ uint32_t segOfPos(uint32_t e, uint32_t n, uint32_t level)
{
	uint32_t s = 0, lo = 0, hi = n;
	for(uint32_t l = 0; l < level; ++l)
	{
		const uint32_t mid = (lo + hi) / 2u;
		const bool right = e >= mid;
		s = 2u * s + (right ? 1u : 0u);
		lo = right ? mid : lo;
		hi = right ? hi : mid;
	}
	return s;
}

// segments a tile can touch: top-phase segments hold >= kSub entries (the phase runs while a node
// holds more than kSub, and sizes differ by at most one), so a tile spans at most
// kPartTile / kSub + 1 of them
constexpr uint32_t kPartSegs = kPartTile / (uint32_t)kSub + 2u;

#if defined(YAF_PART_WAVES) && !defined(PKD_EMU)
__global__ void __launch_bounds__(kPartThreads) __attribute__((amdgpu_waves_per_eu(YAF_PART_WAVES))) k_level_partition(PartArgs A)
#else
__global__ void __launch_bounds__(kPartThreads) k_level_partition(PartArgs A)
#endif
{
	__shared__ uint32_t s_id, s_first, s_acc, s_seg0;
	__shared__ uint32_t s_wsum[kPartItems][kPartThreads / 64];
	__shared__ uint32_t s_start[kPartSegs];
	const uint32_t t = threadIdx.x, wv = t >> 6;
	if(t == 0) s_id = atomicAdd(A.ticket, 1u);
	__syncthreads();
	const uint32_t id = s_id;
	const uint32_t list = id % 3u, tile = id / 3u;
	const uint4 *in = A.in[list];
	uint4 *out = A.out[list];
	uint64_t *st = A.status + (size_t)list * A.n_tiles;
	const uint32_t base = A.lo + tile * kPartTile;
	// the tile's segments: the first by descent, the starts of it and its successors from the segment
	// list (no per-entry segment array: 16 B per photon and level less traffic)
	if(t == 0) s_seg0 = segOfPos(base, A.n, A.level) - A.seg_base;
	__syncthreads();
	const uint32_t seg0 = s_seg0, n_seg = A.n_seg;
#if YAF_PART_PRELOAD
	// the tile's splits staged with the segment starts, and every record loaded before the first flag is
	// computed: the eight 16-B loads of a thread are in flight together (computing each flag right after
	// its load kept one HBM round trip per item in the dependence chain)
	__shared__ Split s_split[kPartSegs];
	if(t < kPartSegs)
	{
		const bool ok = seg0 + t < n_seg;
		s_start[t] = ok ? A.segs[seg0 + t].start : 0xffffffffu;
		if(ok) s_split[t] = A.splits[seg0 + t];
	}
	uint4 r[kPartItems];
#pragma unroll
	for(int i = 0; i < kPartItems; ++i)
	{
		const uint32_t e = base + (uint32_t)i * kPartThreads + t;
		r[i] = e < A.hi ? in[e] : make_uint4(0u, 0u, 0u, 0u);
	}
	__syncthreads();
#else
	if(t < kPartSegs) s_start[t] = seg0 + t < n_seg ? A.segs[seg0 + t].start : 0xffffffffu;
	__syncthreads();
	uint4 r[kPartItems];
#endif
	uint32_t so[kPartItems], pre[kPartItems];
	bool f[kPartItems];
	for(int i = 0; i < kPartItems; ++i)
	{
		const uint32_t e = base + (uint32_t)i * kPartThreads + t;
		f[i] = false;
		so[i] = 0;
#if !YAF_PART_PRELOAD
		r[i] = make_uint4(0u, 0u, 0u, 0u);
#endif
		if(e < A.hi)
		{
#if !YAF_PART_PRELOAD
			r[i] = in[e];
#endif
			uint32_t j = 0;
			while(j + 1u < kPartSegs && s_start[j + 1u] <= e) ++j;
			so[i] = seg0 + j;
			PK_GUARD(so[i] < n_seg && A.segs[so[i]].start <= e && e < A.segs[so[i]].end, so[i]);
#if YAF_PART_PRELOAD
			const Split sp = s_split[j];
#else
			const Split sp = A.splits[so[i]];
#endif
			f[i] = leftOf(r[i], sp.axis, sp.med_key, sp.med_idx);
		}
		const uint64_t b = __ballot(f[i]);
		pre[i] = (uint32_t)__popcll(b & __lanemask_lt());
		if((t & 63u) == 0) s_wsum[i][wv] = (uint32_t)__popcll(b);
	}
	__syncthreads();
	// entry order within the tile: row i (= item i of every thread), then thread
	uint32_t agg = 0;
	for(int i = 0; i < kPartItems; ++i)
	{
		uint32_t before = 0, row = 0;
		for(uint32_t w = 0; w < kPartThreads / 64; ++w)
		{
			const uint32_t c = s_wsum[i][w];
			before += (w < wv) ? c : 0u;
			row += c;
		}
		pre[i] += agg + before;
		agg += row;
	}
	const uint64_t tag_agg = (uint64_t)(2u * A.epoch) << 32, tag_inc = (uint64_t)(2u * A.epoch + 1u) << 32;
	uint32_t excl = 0;
	if(tile > 0)
	{
		if(t == 0)
		{
			pkStoreStatus(&st[tile], tag_agg | agg);
			// one lane polls the predecessor (with back-off) until it has published something; the
			// window read below then rarely finds a tile that has not
			for(uint32_t spins = 0; (uint32_t)(pkLoadStatus(&st[tile - 1]) >> 32) < 2u * A.epoch; ++spins)
			{
				if(spins >= kPartSpinLimit) { atomicMax(reinterpret_cast<int *>(A.err), 1); break; }
				pkBackoff();
			}
		}
		__syncthreads();
		// look back over windows of 64 predecessors: thread t < 64 reads tile (top - t); the window
		// ends at the nearest tile that published its inclusive prefix (tiles < 0 count as an
		// inclusive 0)
		int top = (int)tile - 1;
		for(;;)
		{
			const int j = top - (int)t;
			const bool reader = t < 64u;
			bool ready = true, inc = reader;
			uint32_t val = 0;
			for(uint32_t spins = 0;; ++spins)
			{
				if(reader && j >= 0)
				{
					const uint64_t v = pkLoadStatus(&st[j]);
					const uint32_t tag = (uint32_t)(v >> 32);
					ready = tag >= 2u * A.epoch;
					inc = tag == 2u * A.epoch + 1u;
					val = (uint32_t)v;
				}
				if(!__syncthreads_or(!ready)) break;
				if(spins >= kPartSpinLimit)
				{
					if(t == 0) atomicMax(reinterpret_cast<int *>(A.err), 1);
					inc = reader;
					break;
				}
				pkBackoff();
			}
			if(t == 0) { s_first = 0xffffffffu; s_acc = 0; }
			__syncthreads();
			if(inc) atomicMin(&s_first, t);
			__syncthreads();
			const uint32_t first = s_first;
			if(j >= 0 && t <= first && val) atomicAdd(&s_acc, val);
			__syncthreads();
			excl += s_acc;
			if(first != 0xffffffffu) break;
			top -= 64;
			__syncthreads();
		}
	}
	if(t == 0) pkStoreStatus(&st[tile], tag_inc | (excl + agg));
	for(int i = 0; i < kPartItems; ++i)
	{
		const uint32_t e = base + (uint32_t)i * kPartThreads + t;
		if(e >= A.hi) continue;
		const uint32_t s = so[i];
#if YAF_PART_PRELOAD
		const uint32_t start = s_start[s - seg0], split_el = s_split[s - seg0].split_el;
#else
		const uint32_t start = s_start[s - seg0], split_el = A.splits[s].split_el;
#endif
		const uint32_t left_before = excl + pre[i] - A.seg_left[s];
		uint32_t np = f[i] ? start + left_before : split_el + ((e - start) - left_before);
		PK_GUARD(np < A.n, np);
#if YAF_PART_NT && defined(__HIP_DEVICE_COMPILE__)
		// written once, read by the next level's launch (2.2 GB per level: nothing to keep in L2)
		typedef uint32_t pk_u32x4 __attribute__((ext_vector_type(4)));
		pk_u32x4 w;
		__builtin_memcpy(&w, &r[i], 16);
		__builtin_nontemporal_store(w, reinterpret_cast<pk_u32x4 *>(&out[np]));
#else
		out[np] = r[i];
#endif
	}
}

// ---- bottom phase: one workgroup per subtree of <= kSub photons ----
// One lane per list entry and per segment (kSub == kSubThreads): the three lists of the subtree
// sit in LDS (in / out buffers); per level every segment either becomes a leaf or splits at the
// median of its largest bound axis; the stable partitions take their offsets from wave ballots
// (prefix popcounts + four per-wave totals) instead of a shared-memory scan.  Three barriers per
// level.  The rule and node numbering are the top phase's, restricted to the workgroup's range.
struct LSeg
{
	uint32_t node, start, end;   // start / end relative to the subtree's first element
	float lo[3], hi[3];
};

// Optional output of the subtree pass: the map's photons in kd (leaf) order.  Leaf i of the
// depth-first layout holds list position s (the photon's rank in the tree's in-order leaf
// sequence); with a payload, the leaf's index field is s instead of the photon index and the
// photon's three records are copied to kpos / kdir / kcolb[s].  The k nearest photons of a lookup
// then sit in a few neighbouring cache lines instead of one line per photon and field (k_gather,
// k_pregather, k_fg).  Search order and results are unchanged: the index only rides along in the
// heaps, no comparison reads it.
struct KdPayload
{
	const float4 *dir = nullptr;
	const float *colb = nullptr;
	float4 *kpos = nullptr, *kdir = nullptr;
	float *kcolb = nullptr;
};

constexpr int kSubWaves = kSubThreads / 64;
static_assert(kSub == kSubThreads && kSubWaves == 4, "one lane per entry, four waves");

__device__ __forceinline__ uint32_t lanePrefix(uint64_t ballot)
{
	return (uint32_t)__popcll(ballot & __lanemask_lt());
}

__global__ void __launch_bounds__(kSubThreads) k_subtrees(const Seg *segs, const uint4 *gx, const uint4 *gy, const uint4 *gz, const float4 *pos,
                                                        uint4 *nodes, uint32_t n, int base_level, int *max_level, KdPayload kp = KdPayload{})
{
	constexpr uint16_t kNone = 0xffffu;
	// one copy of the three lists: an entry is read into registers (phase 2) before any entry is scattered
	// (phase 3, after two barriers), and the next level reads after the closing barrier — 40 KB of LDS instead
	// of 52 KB, four workgroups per CU instead of three (YAF_SUB_2BUF=1: the double buffer)
#if YAF_SUB_2BUF
	__shared__ uint4 buf2[2][3][kSub];
#define PK_BUF(c) buf2[(c)]
#else
	__shared__ uint4 buf1[3][kSub];
#define PK_BUF(c) buf1
#endif
	__shared__ uint32_t scan[3][kSub];         // exclusive count of left-going entries before e, per list
	// the level's segments: read by their threads in phase 1 (kept in registers to phase 3) and written as the
	// next level's in phase 3, so one copy (+ the starts the entries read in phase 3) suffices
	__shared__ LSeg lsegs[kSub];
	__shared__ uint32_t lseg_start[kSub];
	__shared__ Split lsplit[kSub];
	__shared__ uint32_t cb[kSub];              // first child segment of splitting segment s
	__shared__ uint16_t seg_of[kSub];          // segment of entry position e (kNone once a leaf)
	__shared__ uint32_t wsum[4][kSubWaves];    // per-wave ballot totals: lists 0-2, splitting segments
#if YAF_SUB_FAST
	__shared__ uint32_t leaf_node[kSub];       // node of the leaf at entry position e
#endif
	const Seg g = segs[blockIdx.x];
	uint32_t m = g.end - g.start;
	PK_GUARD(m >= 1 && m <= blockDim.x && blockDim.x <= (uint32_t)kSub && g.end <= n, m);
	// one lane per entry: the launch takes the largest subtree rounded up to whole waves (<= kSub), so a
	// level of 150-photon subtrees runs three waves per workgroup instead of four
	const uint32_t t = threadIdx.x, wv = t >> 6, nw = blockDim.x >> 6;
	const bool act = t < m;
	if(act)
	{
		PK_BUF(0)[0][t] = gx[g.start + t];
		PK_BUF(0)[1][t] = gy[g.start + t];
		PK_BUF(0)[2][t] = gz[g.start + t];
	}
	seg_of[t] = act ? 0 : kNone;
	if(t == 0)
	{
		LSeg l;
		l.node = g.node;
		l.start = 0;
		l.end = m;
		for(int k = 0; k < 3; ++k) { l.lo[k] = g.lo[k]; l.hi[k] = g.hi[k]; }
		lsegs[0] = l;
	}
	__syncthreads();
	int cur = 0, level = base_level;
	uint32_t ns = 1;
	for(;;)
	{
		// (1) segment t: a leaf (one photon, pkdtree.h:29-33) or a split at the median of its largest axis
		bool split = false;
		LSeg myseg;
		if(t < ns)
		{
			const LSeg l = lsegs[t];
			myseg = l;
			lseg_start[t] = l.start;
			if(l.end - l.start == 1)
			{
#if YAF_SUB_FAST
				// the leaf's node record and payload are written after the last level (leaf_node, below): its
				// gathers then overlap with every other leaf's instead of stalling the level they finish in
				leaf_node[l.start] = l.node;
#else
				uint32_t idx = PK_BUF(cur)[0][l.start].w;
				PK_GUARD(idx < n, idx);
				const float4 ph = pos[idx];
				uint32_t nd = l.node;
				PK_GUARD(nd < 2 * n - 1, nd);
				uint32_t tag = idx;
				if(kp.kpos)
				{
					tag = g.start + l.start;
					PK_GUARD(tag < n, tag);
					kp.kpos[tag] = ph;
					kp.kdir[tag] = kp.dir[idx];
					kp.kcolb[tag] = kp.colb[idx];
				}
				nodes[nd] = make_uint4(__float_as_uint(ph.x), __float_as_uint(ph.y), __float_as_uint(ph.z), 3u | (tag << 2));
#endif
				lsplit[t] = {3u, 0u, 0u, 0u};
			}
			else
			{
				const int axis = largestAxis(l.lo, l.hi);
				uint32_t se = (l.start + l.end) / 2;
				PK_GUARD(se > l.start && l.end <= m, se);
				uint4 med = PK_BUF(cur)[axis][se];
				PK_GUARD(med.w < n, med.w);
#if YAF_SUB_FAST
				// the split position from the median's key (no dependent load per level; a zero key may be -0)
				const uint32_t mk = keyOf(med, axis);
				const float split_pos = mk != kZeroKey ? keyCoord(mk) : coordOf(pos[med.w], axis);
#else
				const float split_pos = coordOf(pos[med.w], axis);
#endif
				const uint32_t right = l.node + 2u * (se - l.start);
				uint32_t nd = l.node;
				PK_GUARD(right < 2 * n - 1, nd);
				nodes[nd] = make_uint4(__float_as_uint(split_pos), 0u, 0u, (uint32_t)axis | (right << 2));
				lsplit[t] = {(uint32_t)axis, se, keyOf(med, axis), med.w};
				split = true;
			}
		}
		const uint64_t bs = __ballot(split);
		if((t & 63) == 0) wsum[3][wv] = (uint32_t)__popcll(bs);
		__syncthreads();
		uint32_t n_split = 0, split_before = 0;
		for(uint32_t w = 0; w < nw; ++w)
		{
			const uint32_t c = wsum[3][w];
			split_before += (w < wv) ? c : 0u;
			n_split += c;
		}
		if(n_split == 0)
		{
			// every segment of this level was a leaf: the deepest level of this subtree (the device build
			// passes no max_level: one atomic per subtree on a single address serialised 131 K workgroups;
			// the depth follows from the largest subtree, pkd.hip)
			if(t == 0 && max_level) atomicMax(max_level, level);
			break;
		}
		if(split) cb[t] = 2u * (split_before + lanePrefix(bs));
		// (2) left-of-median flags of the three lists, prefix counts from ballots
		uint16_t so = seg_of[t];
		Split sp = {3u, 0u, 0u, 0u};
		if(so != kNone)
		{
			PK_GUARD(so < ns, so);
			sp = lsplit[so];
		}
		const bool part = sp.axis != 3u;
		uint4 r[3];
		uint32_t pre[3];
		bool f[3];
		for(int a = 0; a < 3; ++a)
		{
			r[a] = act ? PK_BUF(cur)[a][t] : make_uint4(0u, 0u, 0u, 0u);
			f[a] = part && leftOf(r[a], sp.axis, sp.med_key, sp.med_idx);
			const uint64_t b = __ballot(f[a]);
			pre[a] = lanePrefix(b);
			if((t & 63) == 0) wsum[a][wv] = (uint32_t)__popcll(b);
		}
		__syncthreads();
		for(int a = 0; a < 3; ++a)
		{
			uint32_t off = 0;
			for(uint32_t w = 0; w < wv; ++w) off += wsum[a][w];
			pre[a] += off;
			scan[a][t] = pre[a];
		}
		__syncthreads();
		// (3) scatter (entries of leaves stay put), the next level's segments and entry segments
		if(act)
		{
			uint16_t nso = kNone;
			if(part)
			{
				const uint32_t start = lseg_start[so];
				for(int a = 0; a < 3; ++a)
				{
					const uint32_t left_before = pre[a] - scan[a][start];
					uint32_t np = f[a] ? start + left_before : sp.split_el + ((t - start) - left_before);
					PK_GUARD(np < m, np);
					PK_BUF(cur ^ 1)[a][np] = r[a];
				}
				nso = (uint16_t)(cb[so] + (t < sp.split_el ? 0u : 1u));
			}
			else
				for(int a = 0; a < 3; ++a) PK_BUF(cur ^ 1)[a][t] = r[a];
			seg_of[t] = nso;
		}
		if(split)
		{
			const LSeg l = myseg;
			const Split ls = lsplit[t];
#if YAF_SUB_FAST
			const float split_pos = ls.med_key != kZeroKey ? keyCoord(ls.med_key) : coordOf(pos[ls.med_idx], (int)ls.axis);
#else
			const float split_pos = coordOf(pos[ls.med_idx], (int)ls.axis);
#endif
			uint32_t c0 = cb[t];
			PK_GUARD(c0 + 1 < 2 * n_split, c0);
			LSeg lo = l, hi = l;
			lo.node = l.node + 1;
			lo.end = ls.split_el;
			hi.node = l.node + 2u * (ls.split_el - l.start);
			hi.start = ls.split_el;
			// lo.hi[axis] = hi.lo[axis] = split position, written without a dynamic array index
			for(int k = 0; k < 3; ++k)
			{
				lo.hi[k] = (k == (int)ls.axis) ? split_pos : l.hi[k];
				hi.lo[k] = (k == (int)ls.axis) ? split_pos : l.lo[k];
			}
			lsegs[c0] = lo;
			lsegs[c0 + 1] = hi;
		}
		ns = 2u * n_split;
		cur ^= 1;
		++level;
		__syncthreads();
	}
#if YAF_SUB_FAST
	// every entry position is one leaf (a subtree of m photons has m leaves): its record sits at that
	// position of the lists, which leaves never move
	if(act)
	{
		uint32_t idx = PK_BUF(cur)[0][t].w;
		PK_GUARD(idx < n, idx);
		const float4 ph = pos[idx];
		uint32_t nd = leaf_node[t];
		PK_GUARD(nd < 2 * n - 1, nd);
		uint32_t tag = idx;
		if(kp.kpos)
		{
			tag = g.start + t;
			PK_GUARD(tag < n, tag);
			kp.kpos[tag] = ph;
			kp.kdir[tag] = kp.dir[idx];
			kp.kcolb[tag] = kp.colb[idx];
		}
		nodes[nd] = make_uint4(__float_as_uint(ph.x), __float_as_uint(ph.y), __float_as_uint(ph.z), 3u | (tag << 2));
	}
#endif
}
#undef PK_BUF

} // namespace yafamd_pkd
