// Host check of the GPU BVH layouts (libyafaray_amd/csrc/bvh.cc): for BVH2 and BVH4, every
// triangle sits in exactly one leaf, every child box encloses its subtree, and a host replica of
// the device traversal order (nearest-first, leaves tested on box hit) returns the same closest
// hit (t, lowest primitive on ties) and the same any-hit verdict as an exhaustive loop, while
// never using more stack than the builder's bound.  Build: g++ -O2 -std=c++17 bvh_check.cc
// ../libyafaray_amd/csrc/bvh.cc
#include "../libyafaray_amd/csrc/bvh.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

using namespace yafamd;

static int asInt(float f) { int i; std::memcpy(&i, &f, 4); return i; }

static int fails = 0;
#define CHECK(c, ...) do { if(!(c)) { ++fails; if(fails < 20) { std::printf(__VA_ARGS__); std::printf("\n"); } } } while(0)

struct Ray { float o[3], d[3]; };

// primitive_triangle.cc:44-71 in the packed record form (v0, e1, e2, eps)
static float triTest(const float *r, const Ray &ray)
{
	const float *v0 = r, *e1 = r + 4, *e2 = r + 8;
	const float eps = r[3];
	const float p[3] = {ray.d[1] * e2[2] - ray.d[2] * e2[1], ray.d[2] * e2[0] - ray.d[0] * e2[2], ray.d[0] * e2[1] - ray.d[1] * e2[0]};
	const float det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
	if(det > -eps && det < eps) return -1.f;
	const float inv = 1.f / det;
	const float tv[3] = {ray.o[0] - v0[0], ray.o[1] - v0[1], ray.o[2] - v0[2]};
	const float u = (tv[0] * p[0] + tv[1] * p[1] + tv[2] * p[2]) * inv;
	if(u < 0.f || u > 1.f) return -1.f;
	const float q[3] = {tv[1] * e1[2] - tv[2] * e1[1], tv[2] * e1[0] - tv[0] * e1[2], tv[0] * e1[1] - tv[1] * e1[0]};
	const float v = (ray.d[0] * q[0] + ray.d[1] * q[1] + ray.d[2] * q[2]) * inv;
	if(v < 0.f || u + v > 1.f) return -1.f;
	const float t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
	return t < eps ? -1.f : t;
}

struct Child { float lo[3], hi[3]; int c, k; };

static Child childOf(const BvhOutput &b, int node, int k)
{
	Child ch;
	if(b.width == 4)
	{
		const float *o = &b.nodes[32 * (size_t)node];
		for(int a = 0; a < 3; ++a) { ch.lo[a] = o[8 * a + k]; ch.hi[a] = o[8 * a + 4 + k]; }
		ch.c = asInt(o[24 + k]);
		ch.k = asInt(o[28 + k]);
	}
	else
	{
		const float *o = &b.nodes[16 * (size_t)node];
		const int base = k ? 4 : 0;
		ch.lo[0] = o[base + 0]; ch.hi[0] = o[base + 1]; ch.lo[1] = o[base + 2]; ch.hi[1] = o[base + 3];
		ch.lo[2] = o[8 + 2 * k]; ch.hi[2] = o[9 + 2 * k];
		ch.c = asInt(o[12 + k]);
		ch.k = asInt(o[14 + k]);
	}
	return ch;
}

static bool boxHit(const Child &ch, const Ray &r, float t1, float &tn)
{
	float lo = 0.f, hi = t1;
	for(int a = 0; a < 3; ++a)
	{
		const float d = std::fabs(r.d[a]) < 1e-20f ? std::copysign(1e-20f, r.d[a]) : r.d[a];
		const float ta = (ch.lo[a] - r.o[a]) / d, tb = (ch.hi[a] - r.o[a]) / d;
		lo = std::max(lo, std::min(ta, tb));
		hi = std::min(hi, std::max(ta, tb));
	}
	tn = lo;
	return lo <= hi;
}

// the device traversal order; returns closest (any = false) or first (any = true) hit
static bool traverse(const BvhOutput &b, const Ray &r, bool any, float &t_best, int &prim_best, int &max_sp)
{
	const int W = b.width;
	std::vector<int> stack;
	t_best = 3.4e38f;
	prim_best = -1;
	int node = 0;
	for(;;)
	{
		std::vector<std::pair<float, int>> inner;
		for(int k = 0; k < W; ++k)
		{
			const Child ch = childOf(b, node, k);
			float tn;
			const float slack = t_best < 3.0e38f ? t_best * 1.0000005f + 1e-6f : 3.4e38f;
			if(!boxHit(ch, r, slack, tn)) continue;
			if(ch.c >= 0) { inner.push_back({tn, ch.c}); continue; }
			if(ch.k == 0) continue;
			for(int q = ~ch.c; q < ~ch.c + ch.k; ++q)
			{
				const float *rec = &b.tris[12 * (size_t)q];
				const float t = triTest(rec, r);
				if(t < 0.f) continue;
				const int prim = asInt(rec[7]);
				if(any) { t_best = t; prim_best = prim; return true; }
				if(t < t_best || (t == t_best && prim < prim_best)) { t_best = t; prim_best = prim; }
			}
		}
		std::stable_sort(inner.begin(), inner.end(), [](auto &x, auto &y) { return x.first < y.first; });
		for(int k = (int)inner.size() - 1; k >= 1; --k) stack.push_back(inner[k].second);
		max_sp = std::max(max_sp, (int)stack.size());
		if(!inner.empty()) { node = inner[0].second; continue; }
		if(stack.empty()) break;
		node = stack.back();
		stack.pop_back();
	}
	return prim_best >= 0;
}

static void checkStructure(const BvhOutput &b, int n_tris, const std::vector<float> &verts, const std::vector<int> &tris)
{
	std::vector<int> seen(n_tris, 0);
	std::vector<std::pair<int, int>> todo{{0, 1}};
	int depth = 0;
	while(!todo.empty())
	{
		auto [node, dep] = todo.back();
		todo.pop_back();
		depth = std::max(depth, dep);
		for(int k = 0; k < b.width; ++k)
		{
			const Child ch = childOf(b, node, k);
			std::vector<int> sub;   // triangles under this child
			if(ch.c >= 0)
			{
				CHECK(ch.c > node && ch.c < b.n_nodes, "bad child index %d of node %d", ch.c, node);
				todo.push_back({ch.c, dep + 1});
				std::vector<int> st{ch.c};
				while(!st.empty())
				{
					const int n = st.back();
					st.pop_back();
					for(int j = 0; j < b.width; ++j)
					{
						const Child g = childOf(b, n, j);
						if(g.c >= 0) st.push_back(g.c);
						else for(int q = ~g.c; q < ~g.c + g.k; ++q) sub.push_back(q);
					}
				}
			}
			else
				for(int q = ~ch.c; q < ~ch.c + ch.k; ++q)
				{
					sub.push_back(q);
					const int prim = asInt(b.tris[12 * (size_t)q + 7]);
					CHECK(prim >= 0 && prim < n_tris, "bad prim %d", prim);
					if(prim >= 0 && prim < n_tris) ++seen[prim];
				}
			for(int q : sub)
			{
				const int prim = asInt(b.tris[12 * (size_t)q + 7]);
				for(int v = 0; v < 3; ++v)
					for(int a = 0; a < 3; ++a)
					{
						const float x = verts[3 * (size_t)tris[3 * prim + v] + a];
						CHECK(x >= ch.lo[a] && x <= ch.hi[a], "node %d child %d does not enclose prim %d", node, k, prim);
					}
			}
		}
	}
	for(int t = 0; t < n_tris; ++t) CHECK(seen[t] == 1, "prim %d in %d leaves", t, seen[t]);
	CHECK(depth == b.depth, "depth %d vs reported %d", depth, b.depth);
}

static void run(const char *name, const std::vector<float> &verts, const std::vector<int> &tris, int width, int leaf, std::mt19937 &rng)
{
	const int n = (int)tris.size() / 3;
	BvhInput in{verts.data(), tris.data(), n};
	in.width = width;
	const BvhOutput b = buildBvh(in, leaf, 4);
	CHECK(b.width == width, "%s: width %d", name, b.width);
	checkStructure(b, n, verts, tris);
	std::uniform_real_distribution<float> U(-1.f, 1.f);
	int max_sp = 0, hits = 0;
	for(int i = 0; i < 4000; ++i)
	{
		Ray r;
		for(int a = 0; a < 3; ++a) { r.o[a] = 1.5f * U(rng); r.d[a] = U(rng); }
		if(i % 7 == 0) r.d[i % 3] = 0.f;   // axis-parallel components
		float tb, te = 3.4e38f;
		int pb, pe = -1;
		const bool hit = traverse(b, r, false, tb, pb, max_sp);
		for(int q = 0; q < n; ++q)
		{
			const float t = triTest(&b.tris[12 * (size_t)q], r);
			const int prim = asInt(b.tris[12 * (size_t)q + 7]);
			if(t >= 0.f && (t < te || (t == te && prim < pe))) { te = t; pe = prim; }
		}
		CHECK(hit == (pe >= 0) && (!hit || (tb == te && pb == pe)), "%s w%d leaf%d ray %d: tree (%d %g %d) brute (%g %d)",
		      name, width, leaf, i, hit, tb, pb, te, pe);
		float ta;
		int pa;
		CHECK(traverse(b, r, true, ta, pa, max_sp) == (pe >= 0), "%s w%d any-hit verdict ray %d", name, width, i);
		hits += hit;
	}
	const int bound = width == 4 ? b.stack_need : b.depth;
	CHECK(max_sp <= bound, "%s w%d: stack use %d above bound %d", name, width, max_sp, bound);
	std::printf("%s w%d leaf%d: %d tris, %d nodes, depth %d, stack bound %d (used %d), %d hits\n", name, width, leaf, n,
	            b.n_nodes, b.depth, bound, max_sp, hits);
}

int main()
{
	std::mt19937 rng(7);
	std::uniform_real_distribution<float> U(-1.f, 1.f);
	for(int n : {1, 2, 3, 5, 37, 2000})
	{
		std::vector<float> verts;
		std::vector<int> tris;
		for(int t = 0; t < n; ++t)
		{
			const float c[3] = {U(rng), U(rng), U(rng)};
			for(int v = 0; v < 3; ++v)
			{
				for(int a = 0; a < 3; ++a) verts.push_back(c[a] + 0.2f * U(rng));
				tris.push_back(3 * t + v);
			}
		}
		char name[32];
		std::snprintf(name, sizeof name, "soup%d", n);
		for(int w : {2, 4})
			for(int leaf : {1, 4}) run(name, verts, tris, w, leaf, rng);
	}
	if(fails) { std::printf("%d failures\n", fails); return 1; }
	return 0;
}
