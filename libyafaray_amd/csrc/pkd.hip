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
//            stably partitioned around it ((key, index) < median goes left): the three lists in one
//            single-pass launch with a decoupled look-back (k_level_partition; the level-wise
//            exclusive scan + partition per list remains as YAFARAY_AMD_PKD_PARTITION=scan).  A node of m > 1 photons always has two children,
//            so level d holds exactly 2^d nodes of floor / ceil(n / 2^d) photons and all nodes of a
//            level leave the top phase together.
//   bottom   one workgroup per remaining subtree (<= kSub photons) finishes it in LDS, level by
//            level with the same rule.
// Node layout is the reference's depth-first one: a subtree of m photons has 2m - 1 nodes, node i's
// left child is i + 1 and its right child i + 2 nl.  Node record (uint4): .w = flags (bits 0-1 axis,
// 3 = leaf; interior: right child << 2, leaf: photon index << 2), interior .x = split position bits,
// leaf .xyz = the photon's position bits (k_gather reads them without a second load).  Interior
// nodes also carry their parent's splitting plane (.y = split bits, .z = axis; the root: 0, 3), so a
// walk that stacks only far-child indices can re-derive the plane distance when it pops one
// (k_gather_walk); the reference's tree is unaffected.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#include "pkd_kernels.h"

namespace
{

using namespace yafamd_pkd;

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
	DevBuf kx, ky, kz, kxyz, iota, sorted_keys, sorted_idx, sort_tmp, rec[3], rec_out, segs[2], seg_of, scan, scan_tmp, splits, partial, max_level;
	// fused level partition (k_level_partition)
	DevBuf rec_out2[2], seg_of2, seg_nl, seg_left, status, part_misc;
	~PkdScratch()
	{
		for(DevBuf *b : {&kx, &ky, &kz, &kxyz, &iota, &sorted_keys, &sorted_idx, &sort_tmp, &rec[0], &rec[1], &rec[2], &rec_out, &segs[0], &segs[1],
		                 &seg_of, &scan, &scan_tmp, &splits, &partial, &max_level, &rec_out2[0], &rec_out2[1], &seg_of2, &seg_nl, &seg_left,
		                 &status, &part_misc})
			b->release();
	}
};

#define PKCHECK(x) do { hipError_t e_ = (x); if(e_ != hipSuccess) return e_; } while(0)

} // namespace

// The build scratch belongs to the caller (one per renderer, so per device): *scratch is created on
// the first build and reused; yafamd_pkd_scratch_free releases it.
extern "C" void yafamd_pkd_scratch_free(void *scratch) { delete static_cast<PkdScratch *>(scratch); }

// pos_dev: n photons (position in .xyz); nodes_dev: 2n - 1 nodes (uint4, see the header comment).
// *depth_out: deepest level (root = 0) — the lookup stack needs depth + 1 entries.
// every interior node's children: the interior ones get its splitting plane (.y split, .z axis)
__global__ void __launch_bounds__(256) k_parent_planes(uint4 *nodes, uint32_t n_nodes)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if(i >= n_nodes) return;
	const uint4 nd = nodes[i];
	if((nd.w & 3u) == 3u) return;
	const uint32_t kids[2] = {i + 1u, nd.w >> 2};
	for(uint32_t c : kids)
		if(c < n_nodes && (nodes[c].w & 3u) != 3u)
		{
			nodes[c].y = nd.x;
			nodes[c].z = nd.w & 3u;
		}
	if(i == 0u) { nodes[0].y = 0u; nodes[0].z = 3u; }
}

static hipError_t buildPkd(const float4 *pos_dev, uint32_t n, uint4 *nodes_dev, int *depth_out, hipStream_t st, void **scratch, const KdPayload &kp,
                           int member = 0, int members = 1, int *split_level = nullptr);

extern "C" hipError_t yafamd_build_pkd(const float4 *pos_dev, uint32_t n, uint4 *nodes_dev, int *depth_out, hipStream_t st, void **scratch)
{
	return buildPkd(pos_dev, n, nodes_dev, depth_out, st, scratch, KdPayload{});
}

// The level at which a group of `members` splits the build: D = ceil(log2 members), when the top phase runs
// at least D levels (every node of the levels < D holds more than kSub photons); 0 = not split.
extern "C" int yafamd_pkd_split_level(uint32_t n, int members)
{
	if(members <= 1) return 0;
	int D = 0;
	while((1 << D) < members) ++D;
	uint32_t max_m = n;
	for(int l = 0; l < D; ++l)
	{
		if(max_m <= (uint32_t)kSub) return 0;
		max_m = (max_m + 1) / 2;
	}
	return D;
}

// The level-D segments of a tree over n photons, in order (node, start, end each): level d's nodes are the
// recursive halving of [0, n) at (start + end) / 2, a node's left child is node + 1 and its right child
// node + 2 (mid - start) (the depth-first layout).  A subtree of m photons occupies nodes [node, node + 2m - 1)
// and list (kd-order record) positions [start, end).
extern "C" void yafamd_pkd_top_segments(uint32_t n, int level, uint32_t *out /* 3 << level */)
{
	std::vector<uint32_t> cur{0u, 0u, n}, nxt;
	for(int l = 0; l < level; ++l)
	{
		nxt.clear();
		for(size_t k = 0; k < cur.size(); k += 3)
		{
			const uint32_t node = cur[k], a = cur[k + 1], b = cur[k + 2], mid = (a + b) / 2;
			nxt.insert(nxt.end(), {node + 1u, a, mid, node + 2u * (mid - a), mid, b});
		}
		cur.swap(nxt);
	}
	std::copy(cur.begin(), cur.end(), out);
}

// the level-D segments member r of `members` finishes: [s0, s1), consecutive
extern "C" void yafamd_pkd_owned_segments(int level, int member, int members, uint32_t *s0, uint32_t *s1)
{
	*s0 = (uint32_t)(((uint64_t)member << level) / (uint64_t)members);
	*s1 = (uint32_t)(((uint64_t)(member + 1) << level) / (uint64_t)members);
}

// the interior nodes' parent planes (k_parent_planes) — after a group's member builds were exchanged
extern "C" hipError_t yafamd_pkd_parent_planes(uint4 *nodes_dev, uint32_t n, hipStream_t st)
{
	if(n == 0) return hipSuccess;
	hipLaunchKernelGGL(k_parent_planes, dim3((2 * n - 1 + 255) / 256), dim3(256), 0, st, nodes_dev, 2 * n - 1);
	return hipGetLastError();
}

// A group member's share of the build (the distributed point kd-tree): the same sorts and top
// levels < D as the whole build (every member writes the same ancestor nodes), then only the level-D
// subtrees this member owns (yafamd_pkd_owned_segments) — their nodes and kd-order records; the other
// members' subtrees are left unwritten and the parent planes are not written (the caller exchanges the
// ranges yafamd_pkd_top_segments gives, then runs yafamd_pkd_parent_planes).  *split_level = D, or 0 when
// the tree is too small to split (then this was the whole build, parent planes included).
extern "C" hipError_t yafamd_build_pkd_kd_member(const float4 *pos_dev, const float4 *dir_dev, const float *colb_dev, uint32_t n, uint4 *nodes_dev,
                                                 float4 *kpos, float4 *kdir, float *kcolb, int *depth_out, hipStream_t st, void **scratch, int member,
                                                 int members, int *split_level)
{
	if(n && (!dir_dev || !colb_dev || !kpos || !kdir || !kcolb)) return hipErrorInvalidValue;
	if(members < 1 || member < 0 || member >= members || !split_level) return hipErrorInvalidValue;
	KdPayload kp;
	kp.dir = dir_dev;
	kp.colb = colb_dev;
	kp.kpos = kpos;
	kp.kdir = kdir;
	kp.kcolb = kcolb;
	return buildPkd(pos_dev, n, nodes_dev, depth_out, st, scratch, kp, member, members, split_level);
}

// The same build, and the map's records copied into kd (leaf) order by the subtree pass: leaves
// then carry kd positions (KdPayload, pkd_kernels.h); kpos / kdir / kcolb hold n records each.
extern "C" hipError_t yafamd_build_pkd_kd(const float4 *pos_dev, const float4 *dir_dev, const float *colb_dev, uint32_t n, uint4 *nodes_dev,
                                          float4 *kpos, float4 *kdir, float *kcolb, int *depth_out, hipStream_t st, void **scratch)
{
	if(n && (!dir_dev || !colb_dev || !kpos || !kdir || !kcolb)) return hipErrorInvalidValue;
	KdPayload kp;
	kp.dir = dir_dev;
	kp.colb = colb_dev;
	kp.kpos = kpos;
	kp.kdir = kdir;
	kp.kcolb = kcolb;
	return buildPkd(pos_dev, n, nodes_dev, depth_out, st, scratch, kp);
}

static hipError_t buildPkd(const float4 *pos_dev, uint32_t n, uint4 *nodes_dev, int *depth_out, hipStream_t st, void **scratch, const KdPayload &kp,
                           int member, int members, int *split_level)
{
	if(split_level) *split_level = 0;
	if(n == 0) return hipSuccess;
	// fused partitions (default) or the scan + partition passes per list (YAFARAY_AMD_PKD_PARTITION=scan;
	// a member build then builds the whole tree)
	const char *pe = getenv("YAFARAY_AMD_PKD_PARTITION");
	const bool fused = !(pe && std::string(pe) == "scan");
	const int D = fused ? yafamd_pkd_split_level(n, members) : 0;
	if(split_level) *split_level = D;
	if(!scratch) return hipErrorInvalidValue;
	if(!*scratch) *scratch = new PkdScratch;
	PkdScratch &S = *static_cast<PkdScratch *>(*scratch);
	const uint32_t B = 256, G = (n + B - 1) / B;
	for(DevBuf *b : {&S.kx, &S.ky, &S.kz, &S.iota, &S.sorted_keys, &S.sorted_idx, &S.seg_of}) PKCHECK(b->ensure((size_t)n * 4));
	PKCHECK(S.scan.ensure(((size_t)n + 1) * 4));
	for(DevBuf *b : {&S.rec[0], &S.rec[1], &S.rec[2], &S.rec_out, &S.kxyz}) PKCHECK(b->ensure((size_t)n * 16));
	// lists sorted by (coordinate, index): stable radix sorts of the keys over index order
	hipLaunchKernelGGL(k_keys, dim3(G), dim3(B), 0, st, pos_dev, n, S.kx.as<uint32_t>(), S.ky.as<uint32_t>(), S.kz.as<uint32_t>(),
	                   S.iota.as<uint32_t>(), S.kxyz.as<uint4>());
	size_t sort_bytes = 0;
	PKCHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, S.kx.as<uint32_t>(), S.sorted_keys.as<uint32_t>(), S.iota.as<uint32_t>(),
	                                           S.sorted_idx.as<uint32_t>(), (int)n, 0, 32, st));
	PKCHECK(S.sort_tmp.ensure(sort_bytes));
	const uint32_t *keys[3] = {S.kx.as<uint32_t>(), S.ky.as<uint32_t>(), S.kz.as<uint32_t>()};
	for(int a = 0; a < 3; ++a)
	{
		PKCHECK(hipcub::DeviceRadixSort::SortPairs(S.sort_tmp.p, sort_bytes, keys[a], S.sorted_keys.as<uint32_t>(), S.iota.as<uint32_t>(),
		                                           S.sorted_idx.as<uint32_t>(), (int)n, 0, 32, st));
		hipLaunchKernelGGL(k_records, dim3(G), dim3(B), 0, st, S.sorted_idx.as<uint32_t>(), n, S.kxyz.as<uint4>(), S.rec[a].as<uint4>());
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
	PKCHECK(hipMemsetAsync(S.max_level.p, 0, 4, st));
	size_t scan_bytes = 0;
	{
		hipcub::CountingInputIterator<uint32_t> it(0);
		hipcub::TransformInputIterator<uint32_t, LeftFlag, hipcub::CountingInputIterator<uint32_t>> in(it, LeftFlag{});
		PKCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, in, S.scan.as<uint32_t>(), (int)n, st));
	}
	PKCHECK(S.scan_tmp.ensure(scan_bytes));
	if(!fused) PKCHECK(hipMemsetAsync(S.seg_of.p, 0, (size_t)n * 4, st));   // the scan passes' per-entry segments
	const uint32_t n_tiles = (n + kPartTile - 1) / kPartTile;
	size_t left_scan_bytes = 0;
	if(fused)
	{
		for(DevBuf *b : {&S.rec_out2[0], &S.rec_out2[1]}) PKCHECK(b->ensure((size_t)n * 16));
		for(DevBuf *b : {&S.seg_nl, &S.seg_left}) PKCHECK(b->ensure((size_t)n * 4));
		PKCHECK(S.status.ensure((size_t)3 * n_tiles * 8));
		PKCHECK(S.part_misc.ensure(64));   // [0] ticket, [1] error
		PKCHECK(hipMemsetAsync(S.status.p, 0, (size_t)3 * n_tiles * 8, st));
		PKCHECK(hipMemsetAsync(S.part_misc.p, 0, 64, st));
		PKCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, left_scan_bytes, S.seg_nl.as<uint32_t>(), S.seg_left.as<uint32_t>(), (int)n, st));
		PKCHECK(S.scan_tmp.ensure(std::max(scan_bytes, left_scan_bytes)));
	}
	// top phase: level d has 2^d nodes of floor / ceil(n / 2^d) photons.  A member build (D > 0) narrows
	// to its consecutive level-D segments [s0, s1) once level D is reached: their entries [lo, hi) are
	// partitioned, and seg_base maps a level's global segment number to the local list
	uint32_t n_seg = 1;
	int cur = 0, level = 0;
	uint32_t max_m = n;
	uint32_t lo = 0, hi = n, s0 = 0;
	bool narrowed = false;
	auto narrow = [&]() -> hipError_t {
		uint32_t s1 = 0;
		yafamd_pkd_owned_segments(D, member, members, &s0, &s1);
		std::vector<uint32_t> top((size_t)3 << D);
		yafamd_pkd_top_segments(n, D, top.data());
		lo = top[3 * (size_t)s0 + 1];
		hi = top[3 * (size_t)(s1 - 1) + 2];
		// the owned segments at the front of the other list (their bounds came from the levels above)
		PKCHECK(hipMemcpyAsync(S.segs[cur ^ 1].p, S.segs[cur].as<Seg>() + s0, (size_t)(s1 - s0) * sizeof(Seg), hipMemcpyDeviceToDevice, st));
		cur ^= 1;
		n_seg = s1 - s0;
		narrowed = true;
		return hipSuccess;
	};
	while(max_m > (uint32_t)kSub)
	{
		if(D > 0 && level == D) PKCHECK(narrow());
		const uint32_t seg_base = D > 0 && level >= D ? s0 << (level - D) : 0u;
		const uint32_t Gs = (n_seg + B - 1) / B;
		hipLaunchKernelGGL(k_level_split, dim3(Gs), dim3(B), 0, st, S.segs[cur].as<Seg>(), n_seg, n, S.rec[0].as<uint4>(), S.rec[1].as<uint4>(),
		                   S.rec[2].as<uint4>(), pos_dev, nodes_dev, S.splits.as<Split>(), S.segs[cur ^ 1].as<Seg>(),
		                   fused ? S.seg_nl.as<uint32_t>() : nullptr);
		if(fused)
		{
			PKCHECK(hipcub::DeviceScan::ExclusiveSum(S.scan_tmp.p, left_scan_bytes, S.seg_nl.as<uint32_t>(), S.seg_left.as<uint32_t>(), (int)n_seg, st));
			PKCHECK(hipMemsetAsync(S.part_misc.p, 0, 4, st));   // ticket
			PartArgs P;
			DevBuf *outs[3] = {&S.rec_out, &S.rec_out2[0], &S.rec_out2[1]};
			for(int a = 0; a < 3; ++a)
			{
				P.in[a] = S.rec[a].as<uint4>();
				P.out[a] = outs[a]->as<uint4>();
			}
			P.level = (uint32_t)level;
			P.segs = S.segs[cur].as<Seg>();
			P.splits = S.splits.as<Split>();
			P.seg_left = S.seg_left.as<uint32_t>();
			P.n = n;
			P.n_tiles = (hi - lo + kPartTile - 1) / kPartTile;
			P.lo = lo;
			P.hi = hi;
			P.seg_base = seg_base;
			P.n_seg = n_seg;
			P.epoch = (uint32_t)level + 1u;
			P.ticket = S.part_misc.as<uint32_t>();
			P.err = S.part_misc.as<uint32_t>() + 1;
			P.status = S.status.as<uint64_t>();
			hipLaunchKernelGGL(k_level_partition, dim3(3 * P.n_tiles), dim3(kPartThreads), 0, st, P);
			for(int a = 0; a < 3; ++a)
			{
				std::swap(S.rec[a].p, outs[a]->p);
				std::swap(S.rec[a].bytes, outs[a]->bytes);
			}
			n_seg *= 2;
			max_m = (max_m + 1) / 2;
			cur ^= 1;
			++level;
			continue;
		}
		for(int a = 0; a < 3; ++a)
		{
			hipcub::CountingInputIterator<uint32_t> it(0);
			hipcub::TransformInputIterator<uint32_t, LeftFlag, hipcub::CountingInputIterator<uint32_t>> in(
			    it, LeftFlag{S.rec[a].as<uint4>(), S.seg_of.as<uint32_t>(), S.splits.as<Split>(), n});
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
	if(D > 0 && !narrowed) PKCHECK(narrow());   // the top phase ended at level D
	// bottom phase: one workgroup per subtree
	// the deepest level: the largest subtree (ceil(n / 2^level) photons) halves (its larger half
	// rounding up) until single photons — the device build computes it here instead of one atomicMax per
	// subtree on a single address; the checked build still takes the atomic and compares
#ifdef PKD_CHECK
	int *dev_max_level = S.max_level.as<int>();
#else
	int *dev_max_level = nullptr;
#endif
	const uint32_t sub_threads = std::min<uint32_t>((uint32_t)kSubThreads, (std::max<uint32_t>(max_m, 1u) + 63u) & ~63u);
	hipLaunchKernelGGL(k_subtrees, dim3(n_seg), dim3(sub_threads), 0, st, S.segs[cur].as<Seg>(), S.rec[0].as<uint4>(), S.rec[1].as<uint4>(),
	                   S.rec[2].as<uint4>(), pos_dev, nodes_dev, n, level, dev_max_level, kp);
	if(D == 0) hipLaunchKernelGGL(k_parent_planes, dim3((2 * n - 1 + 255) / 256), dim3(256), 0, st, nodes_dev, 2 * n - 1);
	int depth = level;
	for(uint32_t m = max_m; m > 1u; m = (m + 1u) / 2u) ++depth;
	uint32_t part_err = 0;
#ifdef PKD_CHECK
	int dev_depth = 0;
	PKCHECK(hipMemcpyAsync(&dev_depth, S.max_level.p, 4, hipMemcpyDeviceToHost, st));
#endif
	if(fused && level > 0) PKCHECK(hipMemcpyAsync(&part_err, S.part_misc.as<uint32_t>() + 1, 4, hipMemcpyDeviceToHost, st));
	PKCHECK(hipStreamSynchronize(st));
	if(part_err) return hipErrorLaunchFailure;   // a look-back gave up: the tree is not trustworthy
#ifdef PKD_CHECK
	if(dev_depth != depth) return hipErrorLaunchFailure;
#endif
	*depth_out = depth;
	return hipGetLastError();
}

#ifdef PKD_CHECK
// checked build only: the first failed range check (source line), 0 = none; clears it
extern "C" uint32_t yafamd_pkd_check_error()
{
	uint32_t e = 0, z = 0;
	if(hipMemcpyFromSymbol(&e, HIP_SYMBOL(g_pkd_err), 4) != hipSuccess) return 0xffffffffu;
	(void)hipMemcpyToSymbol(HIP_SYMBOL(g_pkd_err), &z, 4);
	return e;
}
// checked build only: the three record lists as the subtree phase saw them (3 x n uint4)
extern "C" hipError_t yafamd_pkd_check_lists(void *scratch, uint4 *host, uint32_t n)
{
	if(!scratch) return hipErrorInvalidValue;
	PkdScratch &S = *static_cast<PkdScratch *>(scratch);
	for(int a = 0; a < 3; ++a)
		PKCHECK(hipMemcpy(host + (size_t)a * n, S.rec[a].p, (size_t)n * 16, hipMemcpyDeviceToHost));
	return hipSuccess;
}
#endif
