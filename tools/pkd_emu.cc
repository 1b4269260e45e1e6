// CPU emulation of the photon kd-tree build kernels (libyafaray_amd/csrc/pkd_kernels.h): every
// workgroup runs as blockDim std::threads with a std::barrier for __syncthreads, LDS arrays become
// function statics shared by those threads, and the host driver's steps (radix sorts, scans) are
// restated serially.  Built with -fsanitize=thread it reports LDS races; either way the tree is
// checked against a direct restatement of the reference build (pkdtree.h:115-222).
//
//   g++ -std=c++20 -O1 -g -fsanitize=thread -pthread tools/pkd_emu.cc -o /tmp/pkd_emu && /tmp/pkd_emu 3 300 5000
#include <algorithm>
#include <atomic>
#include <barrier>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <numeric>
#include <random>
#include <thread>
#include <vector>

struct uint4 { uint32_t x, y, z, w; };
struct float4 { float x, y, z, w; };
struct uint2 { uint32_t x, y; };
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return {x, y, z, w}; }
inline uint32_t __float_as_uint(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float __uint_as_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
struct Dim3 { uint32_t x = 0, y = 0, z = 0; };
thread_local Dim3 threadIdx, blockIdx;
Dim3 blockDim, gridDim;
std::barrier<> *g_bar = nullptr;
inline void __syncthreads() { g_bar->arrive_and_wait(); }
std::atomic<int> g_or[2];
thread_local int g_or_phase = 0;
inline int __syncthreads_or(int p)
{
	const int ph = g_or_phase;
	g_or_phase ^= 1;
	if(p) g_or[ph].fetch_or(1);
	g_bar->arrive_and_wait();
	const int r = g_or[ph].load();
	g_bar->arrive_and_wait();
	if(threadIdx.x == 0) g_or[ph].store(0);
	return r;
}
// wave ops: every lane of the block calls them in uniform control flow (as the kernels do)
std::atomic<uint64_t> g_ballot[2][16];
thread_local int g_ballot_phase = 0;
inline uint64_t __ballot(int p)
{
	const int ph = g_ballot_phase;
	g_ballot_phase ^= 1;
	const uint32_t w = threadIdx.x / 64, lane = threadIdx.x % 64;
	if(p) g_ballot[ph][w].fetch_or(1ull << lane);
	g_bar->arrive_and_wait();
	const uint64_t r = g_ballot[ph][w].load();
	g_bar->arrive_and_wait();
	if(lane == 0) g_ballot[ph][w].store(0);
	return r;
}
inline uint64_t __lanemask_lt() { return (1ull << (threadIdx.x % 64)) - 1ull; }
inline int __popcll(uint64_t v) { return __builtin_popcountll(v); }
template<class T> T atomicCAS(T *a, T c, T v) { __atomic_compare_exchange_n(a, &c, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST); return c; }
inline int atomicMax(int *a, int v)
{
	int o = __atomic_load_n(a, __ATOMIC_SEQ_CST);
	while(o < v && !__atomic_compare_exchange_n(a, &o, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {}
	return o;
}
#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __shared__ static
#define __launch_bounds__(x)
#define PKD_CHECK 1
#define PKD_EMU 1
inline uint32_t atomicAdd(uint32_t *a, uint32_t v) { return __atomic_fetch_add(a, v, __ATOMIC_SEQ_CST); }
inline uint32_t atomicMin(uint32_t *a, uint32_t v)
{
	uint32_t o = __atomic_load_n(a, __ATOMIC_SEQ_CST);
	while(v < o && !__atomic_compare_exchange_n(a, &o, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {}
	return o;
}

#include "../libyafaray_amd/csrc/pkd_kernels.h"

using namespace yafamd_pkd;

// one workgroup at a time, blockDim threads each
static void launch(uint32_t grid, uint32_t block, const std::function<void()> &body)
{
	gridDim.x = grid;
	blockDim.x = block;
	for(uint32_t b = 0; b < grid; ++b)
	{
		std::barrier<> bar((std::ptrdiff_t)block);
		g_bar = &bar;
		std::vector<std::thread> th;
		for(uint32_t t = 0; t < block; ++t)
			th.emplace_back([&, b, t] {
				blockIdx.x = b;
				threadIdx.x = t;
				body();
			});
		for(auto &x : th) x.join();
	}
}

// element-wise kernels with no barriers: one CPU thread walks the grid
static void launchFlat(uint32_t grid, uint32_t block, const std::function<void()> &body)
{
	gridDim.x = grid;
	blockDim.x = block;
	for(uint32_t b = 0; b < grid; ++b)
		for(uint32_t t = 0; t < block; ++t)
		{
			blockIdx.x = b;
			threadIdx.x = t;
			body();
		}
}

static uint32_t okey(float f)
{
	if(f == 0.f) f = 0.f;
	const uint32_t u = __float_as_uint(f);
	return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// pkdtree.h:115-222 restated directly: recursive median split of the largest bound axis
static int refBuild(const std::vector<float4> &pos, std::vector<uint32_t> idx, uint32_t node, float lo[3], float hi[3], std::vector<uint4> &nodes, int d)
{
	if(idx.size() == 1)
	{
		const float4 p = pos[idx[0]];
		nodes[node] = make_uint4(__float_as_uint(p.x), __float_as_uint(p.y), __float_as_uint(p.z), 3u | (idx[0] << 2));
		return d;
	}
	const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
	const int ax = (dx > dy) ? ((dx > dz) ? 0 : 2) : ((dy > dz) ? 1 : 2);
	auto c = [&](uint32_t i) { const float4 &p = pos[i]; return ax == 0 ? p.x : (ax == 1 ? p.y : p.z); };
	std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return okey(c(a)) != okey(c(b)) ? okey(c(a)) < okey(c(b)) : a < b; });
	const size_t h = idx.size() / 2;
	const float sp = c(idx[h]);
	const uint32_t right = node + 2u * (uint32_t)h;
	nodes[node] = make_uint4(__float_as_uint(sp), 0u, 0u, (uint32_t)ax | (right << 2));
	float lhi[3] = {hi[0], hi[1], hi[2]}, rlo[3] = {lo[0], lo[1], lo[2]};
	lhi[ax] = sp;
	rlo[ax] = sp;
	const int a = refBuild(pos, std::vector<uint32_t>(idx.begin(), idx.begin() + h), node + 1, lo, lhi, nodes, d + 1);
	const int b = refBuild(pos, std::vector<uint32_t>(idx.begin() + h, idx.end()), right, rlo, hi, nodes, d + 1);
	return std::max(a, b);
}

// pkd.hip yafamd_pkd_split_level / yafamd_pkd_top_segments, restated for the member builds
static int splitLevel(uint32_t n, int members)
{
	if(members <= 1) return 0;
	int D = 0;
	while((1 << D) < members) ++D;
	uint32_t m = n;
	for(int l = 0; l < D; ++l)
	{
		if(m <= (uint32_t)kSub) return 0;
		m = (m + 1) / 2;
	}
	return D;
}
static std::vector<uint32_t> topSegments(uint32_t n, int level)
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
	return cur;
}

// pkd.hip's build driver over the emulated kernels: the whole tree (members 1) or member `member`'s share;
// returns the number of top levels (-1: a look-back gave up)
static int build(const std::vector<float4> &pos, uint32_t n, bool fused, int member, int members, std::vector<uint4> &nodes, int &max_level,
                 uint32_t &max_m_out)
{
	max_level = 0;
	const uint32_t B = 256, G = (n + B - 1) / B;
	std::vector<uint32_t> kx(n), ky(n), kz(n), iota(n);
	std::vector<uint4> kxyz(n);
	launchFlat(G, B, [&] { k_keys(pos.data(), n, kx.data(), ky.data(), kz.data(), iota.data(), kxyz.data()); });
	std::vector<uint4> rec[3], rec_out(n);
	const std::vector<uint32_t> *keys[3] = {&kx, &ky, &kz};
	for(int a = 0; a < 3; ++a)
	{
		std::vector<uint32_t> si(iota);
		std::stable_sort(si.begin(), si.end(), [&](uint32_t i, uint32_t j) { return (*keys[a])[i] < (*keys[a])[j]; });
		rec[a].resize(n);
		launchFlat(G, B, [&] { k_records(si.data(), n, kxyz.data(), rec[a].data()); });
	}
	const uint32_t n_part = std::min<uint32_t>(G, 1024);
	std::vector<float> partial(n_part * 6);
	std::vector<Seg> segs[2] = {std::vector<Seg>(n), std::vector<Seg>(n)};
	std::vector<Split> splits(n);
	std::vector<uint32_t> seg_of(n, 0), scan(n + 1), seg_nl(n), seg_left(n);
	nodes.assign(2 * n - 1, make_uint4(0xdead, 0xdead, 0xdead, 0xdead));
	launch(n_part, 256, [&] { k_bound(pos.data(), n, partial.data()); });
	launch(1, 256, [&] { k_root(partial.data(), n_part, n, segs[0].data()); });
	uint32_t n_seg = 1, max_m = n;
	int cur = 0, level = 0;
	// a member build (pkd.hip yafamd_build_pkd_kd_member): the levels < D whole, then only the owned level-D
	// segments [s0, s1), whose entries are [lo, hi)
	const int D = splitLevel(n, members);
	uint32_t lo = 0, hi = n, s0 = 0;
	bool narrowed = false;
	auto narrow = [&] {
		const uint32_t s1 = (uint32_t)(((uint64_t)(member + 1) << D) / (uint64_t)members);
		s0 = (uint32_t)(((uint64_t)member << D) / (uint64_t)members);
		const std::vector<uint32_t> top = topSegments(n, D);
		lo = top[3 * (size_t)s0 + 1];
		hi = top[3 * (size_t)(s1 - 1) + 2];
		std::copy(segs[cur].begin() + s0, segs[cur].begin() + s1, segs[cur ^ 1].begin());
		cur ^= 1;
		n_seg = s1 - s0;
		narrowed = true;
	};
	while(max_m > (uint32_t)kSub)
	{
		if(D > 0 && level == D) narrow();
		const uint32_t seg_base = D > 0 && level >= D ? s0 << (level - D) : 0u;
		launchFlat((n_seg + B - 1) / B, B, [&] {
			k_level_split(segs[cur].data(), n_seg, n, rec[0].data(), rec[1].data(), rec[2].data(), pos.data(), nodes.data(), splits.data(),
			              segs[cur ^ 1].data(), seg_nl.data());
		});
		if(fused)
		{
			// pkd.hip's fused level: seg_left = exclusive sum of the left counts, one k_level_partition
			// launch over the three lists (workgroups run one after another here, so every look-back
			// finds its predecessor's inclusive prefix)
			uint32_t acc = 0;
			for(uint32_t k = 0; k < n_seg; ++k) { seg_left[k] = acc; acc += seg_nl[k]; }
			const uint32_t n_tiles = (hi - lo + kPartTile - 1) / kPartTile;
			std::vector<uint64_t> status(3 * n_tiles, 0);
			uint32_t misc[2] = {0, 0};
			std::vector<uint4> outs[3] = {std::vector<uint4>(n), std::vector<uint4>(n), std::vector<uint4>(n)};
			PartArgs P;
			for(int a = 0; a < 3; ++a) { P.in[a] = rec[a].data(); P.out[a] = outs[a].data(); }
			P.level = (uint32_t)level;
			P.segs = segs[cur].data();
			P.splits = splits.data();
			P.seg_left = seg_left.data();
			P.n = n;
			P.n_tiles = n_tiles;
			P.lo = lo;
			P.hi = hi;
			P.seg_base = seg_base;
			P.n_seg = n_seg;
			P.epoch = (uint32_t)level + 1u;
			P.ticket = &misc[0];
			P.err = &misc[1];
			P.status = status.data();
			launch(3 * n_tiles, kPartThreads, [&] { k_level_partition(P); });
			if(misc[1]) { std::printf("look-back gave up\n"); return -1; }
			for(int a = 0; a < 3; ++a) std::swap(rec[a], outs[a]);
			n_seg *= 2;
			max_m = (max_m + 1) / 2;
			cur ^= 1;
			++level;
			continue;
		}
		for(int a = 0; a < 3; ++a)
		{
			LeftFlag f{rec[a].data(), seg_of.data(), splits.data(), n};
			uint32_t acc = 0;
			for(uint32_t p = 0; p < n; ++p) { scan[p] = acc; acc += f(p); }
			launchFlat(G, B, [&] { k_partition(rec[a].data(), n, scan.data(), seg_of.data(), segs[cur].data(), splits.data(), rec_out.data()); });
			std::swap(rec[a], rec_out);
		}
		launchFlat(G, B, [&] { k_seg_of(seg_of.data(), n, splits.data()); });
		n_seg *= 2;
		max_m = (max_m + 1) / 2;
		cur ^= 1;
		++level;
	}
	if(D > 0 && !narrowed) narrow();
	launch(n_seg, std::min<uint32_t>((uint32_t)kSubThreads, (std::max<uint32_t>(max_m, 1u) + 63u) & ~63u), [&] {
		k_subtrees(segs[cur].data(), rec[0].data(), rec[1].data(), rec[2].data(), pos.data(), nodes.data(), n, level, &max_level);
	});
	max_m_out = max_m;
	return level;
}

static bool run(uint32_t n, uint32_t seed, bool fused)
{
	std::mt19937 rng(seed);
	std::uniform_real_distribution<float> U(-2.f, 2.f);
	std::vector<float4> pos(n);
	for(uint32_t i = 0; i < n; ++i)
	{
		pos[i] = {U(rng), U(rng), U(rng), 0.f};
		if(n > 10 && i % 7 == 0) pos[i].y = 0.5f;
		if(n > 10 && i % 11 == 0) pos[i].x = -0.f;
		if(n > 10 && i % 13 == 0) pos[i] = pos[0];
	}
	std::vector<uint4> nodes;
	int max_level = 0;
	uint32_t max_m = 0;
	const int level = build(pos, n, fused, 0, 1, nodes, max_level, max_m);
	if(level < 0) return false;
	std::vector<uint4> want(2 * n - 1);
	float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
	for(const float4 &p : pos)
	{
		lo[0] = std::min(lo[0], p.x); lo[1] = std::min(lo[1], p.y); lo[2] = std::min(lo[2], p.z);
		hi[0] = std::max(hi[0], p.x); hi[1] = std::max(hi[1], p.y); hi[2] = std::max(hi[2], p.z);
	}
	std::vector<uint32_t> all(n);
	std::iota(all.begin(), all.end(), 0u);
	const int depth = refBuild(pos, all, 0, lo, hi, want, 0);
	size_t bad = 0, first = 0;
	for(size_t i = 0; i < want.size(); ++i)
		if(std::memcmp(&want[i], &nodes[i], 16) != 0 && bad++ == 0) first = i;
	std::printf("%s n=%u top_levels=%d check_line=%u depth=%d ref_depth=%d mismatching_nodes=%zu", fused ? "fused" : "scan", n, level, g_pkd_err, max_level, depth, bad);
	if(bad) std::printf(" first=%zu got=(%x %x %x %x) want=(%x %x %x %x)", first, nodes[first].x, nodes[first].y, nodes[first].z, nodes[first].w,
	                    want[first].x, want[first].y, want[first].z, want[first].w);
	std::printf("\n");
	// pkd.hip's arithmetic depth (the largest subtree halved down to single photons)
	int calc = level;
	for(uint32_t m = max_m; m > 1u; m = (m + 1u) / 2u) ++calc;
	if(calc != max_level) std::printf("arithmetic depth %d != %d\n", calc, max_level);
	bool ok = bad == 0 && g_pkd_err == 0 && depth == max_level && calc == max_level;
	g_pkd_err = 0;
	// the distributed build: every member's share, its owned level-D subtrees' node ranges merged over member
	// 0's array (the ancestors every member writes), node for node the whole build
	for(int members : {2, 3, 5, 8})
	{
		if(!fused) break;
		const int D = splitLevel(n, members);
		if(D == 0) continue;
		const std::vector<uint32_t> top = topSegments(n, D);
		std::vector<uint4> merged;
		for(int r = 0; r < members && ok; ++r)
		{
			std::vector<uint4> part;
			int ml = 0;
			uint32_t mm = 0;
			ok = build(pos, n, true, r, members, part, ml, mm) == level && g_pkd_err == 0;
			if(r == 0) merged = part;
			const uint32_t s0 = (uint32_t)(((uint64_t)r << D) / (uint64_t)members), s1 = (uint32_t)(((uint64_t)(r + 1) << D) / (uint64_t)members);
			for(uint32_t sg = s0; sg < s1; ++sg)
			{
				const uint32_t node = top[3 * sg], m = top[3 * sg + 2] - top[3 * sg + 1];
				std::copy(part.begin() + node, part.begin() + node + 2 * m - 1, merged.begin() + node);
			}
		}
		size_t mb = 0;
		for(size_t i = 0; i < want.size() && ok; ++i) mb += std::memcmp(&want[i], &merged[i], 16) != 0;
		std::printf("  members=%d split_level=%d mismatching_nodes=%zu\n", members, D, mb);
		ok = ok && mb == 0;
	}
	return ok;
}

int main(int argc, char **argv)
{
	bool ok = true;
	for(int i = 1; i < argc; ++i)
		for(bool fused : {false, true}) ok = run((uint32_t)std::atoi(argv[i]), 7u + (uint32_t)i, fused) && ok;
	std::printf(ok ? "OK\n" : "FAILED\n");
	return ok ? 0 : 1;
}
