// CPU model of k_gather_walk's pruning threshold (design probe, not product code).
//
// The walk may prune and log with any threshold T(t) >= the reference's max_d2(t) as long as the
// replay re-applies the exact acceptance test: the log then holds a superset of the accepted
// photons in visit order and the replay recovers the reference's sequence.  This probe compares,
// on a synthetic Cornell-like photon set, the visits and log entries per query of
//   exact   T = max_d2 (the k smallest distances kept, as k_gather_walk does in registers)
//   ladder  M counters of logged entries below T / r^m (m = 1..M, lower bounds): T drops one rung
//           when the first counter reaches k; the counters shift and the deepest restarts at 0.
// Build: g++ -O2 -std=c++17 -o /tmp/walk_sim tools/walk_sim.cc
// Run:   /tmp/walk_sim [photons] [queries] [k] [radius]
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <queue>
#include <random>
#include <vector>

struct Node { float split; int axis; uint32_t right; int leaf; uint32_t ph; };

static std::vector<float> P;   // xyz
static std::vector<Node> N;

static void build(std::vector<uint32_t> &idx, size_t s, size_t e, uint32_t node, float lo[3], float hi[3])
{
	if(e - s == 1) { N[node] = {0, 3, 0, 1, idx[s]}; return; }
	const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
	const int a = (dx > dy) ? ((dx > dz) ? 0 : 2) : ((dy > dz) ? 1 : 2);
	const size_t m = (s + e) / 2;
	std::nth_element(idx.begin() + s, idx.begin() + m, idx.begin() + e, [a](uint32_t x, uint32_t y) {
		const float cx = P[3 * x + a], cy = P[3 * y + a];
		return cx < cy || (cx == cy && x < y);
	});
	const float sp = P[3 * idx[m] + a];
	const uint32_t right = node + 2 * (uint32_t)(m - s);
	N[node] = {sp, a, right, 0, 0};
	float lh[3] = {hi[0], hi[1], hi[2]}, rl[3] = {lo[0], lo[1], lo[2]};
	lh[a] = sp;
	rl[a] = sp;
	build(idx, s, m, node + 1, lo, lh);
	build(idx, m, e, right, rl, hi);
}

struct Res { uint64_t visits = 0, logged = 0, accepted = 0; };

// mode 0: exact; mode 1: ladder (M rungs of ratio r)
static void walk(const float *p, int k, float radius2, int mode, int M, float r, Res &res)
{
	std::priority_queue<float> heap;   // exact k smallest (mode 0), and the replay's check
	std::vector<float> logd;
	float T = radius2;
	std::vector<uint32_t> cnt(M, 0);
	std::vector<uint32_t> stk;
	auto maxd2 = [&]() { return (int)heap.size() < k ? radius2 : heap.top(); };
	uint32_t curr = 0;
	for(;;)
	{
		for(;;)
		{
			const Node &nd = N[curr];
			++res.visits;
			if(nd.leaf) break;
			const float pa = p[nd.axis];
			uint32_t far;
			if(pa <= nd.split) { far = nd.right; curr = curr + 1; }
			else { far = curr + 1; curr = nd.right; }
			float d2 = pa - nd.split;
			d2 *= d2;
			const float thr = mode == 0 ? maxd2() : T;
			if(d2 <= thr) { stk.push_back(far); stk.push_back(*(uint32_t *)&d2); }
		}
		const Node &lf = N[curr];
		const float vx = P[3 * lf.ph] - p[0], vy = P[3 * lf.ph + 1] - p[1], vz = P[3 * lf.ph + 2] - p[2];
		const float d = vx * vx + vy * vy + vz * vz;
		const float thr = mode == 0 ? maxd2() : T;
		if(d < thr)
		{
			++res.logged;
			// the replay's exact test
			if(d < maxd2())
			{
				++res.accepted;
				heap.push(d);
				if((int)heap.size() > k) heap.pop();
			}
			if(mode == 2)
			{
				// absolute histogram: bin j = [radius2 r^-(j+1), radius2 r^-j), the last bin open below
				int j = (int)std::floor(std::log(radius2 / d) / std::log(r));
				j = std::max(0, std::min(j, M - 1));
				++cnt[j];
				// T = edge(B) with B the deepest rung such that >= k entries lie below edge(B)
				uint32_t below = 0;
				int B = 0;
				for(int m = M - 1; m >= 0; --m)
				{
					below += cnt[m];   // entries in bins >= m: below edge(m)
					if(below >= (uint32_t)k) { B = m; break; }
				}
				if(below >= (uint32_t)k) T = std::min(T, radius2 * std::pow(r, -(float)B));
			}
			if(mode == 1)
			{
				float e = T;
				for(int m = 0; m < M; ++m) { e /= r; cnt[m] += d < e; }
				while(cnt[0] >= (uint32_t)k)
				{
					T /= r;
					for(int m = 0; m + 1 < M; ++m) cnt[m] = cnt[m + 1];
					cnt[M - 1] = 0;
				}
			}
		}
		bool more = false;
		while(!stk.empty())
		{
			uint32_t d2b = stk.back(); stk.pop_back();
			uint32_t far = stk.back(); stk.pop_back();
			const float d2 = *(float *)&d2b;
			const float thr2 = mode == 0 ? maxd2() : T;
			if(d2 > thr2) continue;
			curr = far;
			more = true;
			break;
		}
		if(!more) break;
	}
}

int main(int argc, char **argv)
{
	const size_t n = argc > 1 ? atol(argv[1]) : 2000000;
	const int nq = argc > 2 ? atoi(argv[2]) : 20000;
	const int k = argc > 3 ? atoi(argv[3]) : 50;
	const float radius = argc > 4 ? (float)atof(argv[4]) : 0.1f;
	std::mt19937 rng(7);
	std::uniform_real_distribution<float> u(-1.f, 1.f);
	auto wallPoint = [&](float *q) {
		// five walls of [-1,1]^3 (no front), denser near the ceiling light: a Cornell-like photon set
		const int w = rng() % 5;
		float a = u(rng), b = u(rng);
		if(rng() % 3 == 0) { a *= 0.5f; b *= 0.5f; }
		switch(w)
		{
		case 0: q[0] = a; q[1] = b; q[2] = -1.f; break;
		case 1: q[0] = a; q[1] = b; q[2] = 1.f; break;
		case 2: q[0] = -1.f; q[1] = a; q[2] = b; break;
		case 3: q[0] = 1.f; q[1] = a; q[2] = b; break;
		default: q[0] = a; q[1] = 1.f; q[2] = b; break;
		}
	};
	P.resize(3 * n);
	for(size_t i = 0; i < n; ++i) wallPoint(&P[3 * i]);
	std::vector<uint32_t> idx(n);
	for(size_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
	N.resize(2 * n - 1);
	float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
	for(size_t i = 0; i < n; ++i)
		for(int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], P[3 * i + a]); hi[a] = std::max(hi[a], P[3 * i + a]); }
	build(idx, 0, n, 0, lo, hi);
	std::vector<float> qs(3 * nq);
	for(int i = 0; i < nq; ++i) wallPoint(&qs[3 * i]);
	struct Cfg { int mode, M; float r; };
	const Cfg cfgs[] = {{0, 0, 1.f}, {1, 4, std::pow(2.f, 0.25f)}, {1, 8, std::pow(2.f, 0.25f)}, {1, 8, std::pow(2.f, 0.125f)},
	                    {1, 16, std::pow(2.f, 0.125f)}, {1, 4, std::pow(2.f, 0.5f)}, {1, 2, 2.f},
	                    {2, 64, std::pow(2.f, 0.25f)}, {2, 32, std::pow(2.f, 0.5f)}, {2, 128, std::pow(2.f, 0.125f)}, {2, 16, 2.f}};
	for(const Cfg &c : cfgs)
	{
		Res r;
		for(int i = 0; i < nq; ++i) walk(&qs[3 * i], k, radius * radius, c.mode, c.M, c.r, r);
		std::printf("%s M=%2d r=%.3f  visits/q %.1f  logged/q %.1f  accepted/q %.1f\n", c.mode == 2 ? "hist  " : c.mode ? "ladder" : "exact ", c.M, c.r,
		            (double)r.visits / nq, (double)r.logged / nq, (double)r.accepted / nq);
	}
	return 0;
}
