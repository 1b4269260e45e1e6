// Binned-SAH BVH2 builder (see bvh.h).
#include "bvh.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstring>
#include <future>
#include <limits>
#include <mutex>

namespace yafamd
{

namespace
{

struct Box
{
	float lo[3] = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), std::numeric_limits<float>::max()};
	float hi[3] = {-std::numeric_limits<float>::max(), -std::numeric_limits<float>::max(), -std::numeric_limits<float>::max()};
	void grow(const float *p)
	{
		for(int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
	}
	void grow(const Box &b)
	{
		for(int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
	}
	bool valid() const { return lo[0] <= hi[0]; }
	float area() const
	{
		if(!valid()) return 0.f;
		const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
		return 2.f * (dx * dy + dy * dz + dz * dx);
	}
};

struct BuildNode
{
	Box box;
	int left = -1, right = -1;   // children (BuildNode indices) for inner nodes
	int start = 0, count = 0;    // leaf range in `order`
};

struct Builder
{
	const BvhInput &in;
	int leaf_size;
	std::vector<Box> tri_box;
	std::vector<float> cent;     // 3 per triangle
	std::vector<int> order;
	std::vector<BuildNode> nodes;
	std::mutex mtx;

	float node_cost = 0.5f;   // SAH: cost of one node visit (two box tests) relative to one triangle test
	explicit Builder(const BvhInput &i, int ls) : in(i), leaf_size(ls) {}

	int newNode()
	{
		std::lock_guard<std::mutex> g(mtx);
		nodes.emplace_back();
		return (int)nodes.size() - 1;
	}

	// returns node index; recursion builds children (optionally in parallel near the top)
	int build(int start, int end, int par_depth)
	{
		Box box, cbox;
		for(int i = start; i < end; ++i)
		{
			box.grow(tri_box[order[i]]);
			cbox.grow(&cent[3 * order[i]]);
		}
		const int id = newNode();
		const int n = end - start;
		auto makeLeaf = [&]() {
			std::lock_guard<std::mutex> g(mtx);
			nodes[id].box = box;
			nodes[id].start = start;
			nodes[id].count = n;
			return id;
		};
		if(n <= leaf_size) return makeLeaf();
		// binned SAH over all three axes
		constexpr int kBins = 32;
		int best_axis = -1, best_split = -1;
		float best_cost = std::numeric_limits<float>::max();
		const float leaf_cost = (float)n;
		for(int axis = 0; axis < 3; ++axis)
		{
			const float cmin = cbox.lo[axis], cext = cbox.hi[axis] - cbox.lo[axis];
			if(!(cext > 0.f)) continue;
			Box bb[kBins];
			int bc[kBins] = {0};
			const float scale = kBins / cext;
			for(int i = start; i < end; ++i)
			{
				int b = (int)((cent[3 * order[i] + axis] - cmin) * scale);
				b = std::min(std::max(b, 0), kBins - 1);
				bb[b].grow(tri_box[order[i]]);
				++bc[b];
			}
			float ra[kBins];
			int rc[kBins];
			Box acc;
			int cnt = 0;
			for(int b = kBins - 1; b > 0; --b)
			{
				acc.grow(bb[b]);
				cnt += bc[b];
				ra[b] = acc.area();
				rc[b] = cnt;
			}
			acc = Box();
			cnt = 0;
			const float inv_area = 1.f / std::max(box.area(), 1e-30f);
			for(int b = 0; b < kBins - 1; ++b)
			{
				acc.grow(bb[b]);
				cnt += bc[b];
				if(cnt == 0 || rc[b + 1] == 0) continue;
				const float cost = node_cost + (acc.area() * cnt + ra[b + 1] * rc[b + 1]) * inv_area;
				if(cost < best_cost) { best_cost = cost; best_axis = axis; best_split = b; }
			}
		}
		int mid;
		if(best_axis < 0)
		{
			if(n <= 2 * leaf_size) return makeLeaf();
			mid = (start + end) / 2;   // all centroids coincide: split by index
		}
		else
		{
			if(best_cost >= leaf_cost && n <= 2 * leaf_size) return makeLeaf();
			const float cmin = cbox.lo[best_axis], scale = kBins / (cbox.hi[best_axis] - cbox.lo[best_axis]);
			auto it = std::partition(order.begin() + start, order.begin() + end, [&](int t) {
				int b = (int)((cent[3 * t + best_axis] - cmin) * scale);
				b = std::min(std::max(b, 0), kBins - 1);
				return b <= best_split;
			});
			mid = (int)(it - order.begin());
			if(mid == start || mid == end) mid = (start + end) / 2;
		}
		int l, r;
		if(par_depth > 0 && n > 4096)
		{
			auto fl = std::async(std::launch::async, [&]() { return build(start, mid, par_depth - 1); });
			r = build(mid, end, par_depth - 1);
			l = fl.get();
		}
		else
		{
			l = build(start, mid, 0);
			r = build(mid, end, 0);
		}
		std::lock_guard<std::mutex> g(mtx);
		nodes[id].box = box;
		nodes[id].left = l;
		nodes[id].right = r;
		return id;
	}
};

// Conservative padding so that the float slab test never culls a box the exact triangle test
// would hit inside (traversal culling is a performance decision only).
void padBox(const Box &b, float *lo, float *hi)
{
	for(int k = 0; k < 3; ++k)
	{
		const float mag = std::fabs(b.lo[k]) + std::fabs(b.hi[k]) + (b.hi[k] - b.lo[k]);
		const float pad = mag * 1e-5f + 1e-7f;
		lo[k] = b.lo[k] - pad;
		hi[k] = b.hi[k] + pad;
	}
}

int intAsFloatBits(int v, float &f)
{
	std::memcpy(&f, &v, 4);
	return v;
}

} // namespace

void packTriangle(const float *v0, const float *v1, const float *v2, int prim, float *o)
{
	const float e1[3] = {v1[0] - v0[0], v1[1] - v0[1], v1[2] - v0[2]};
	const float e2[3] = {v2[0] - v0[0], v2[1] - v0[1], v2[2] - v0[2]};
	const float l1 = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
	const float l2 = std::sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
	const float eps = 0.1f * 0.00005f * std::max(l1, l2);
	o[0] = v0[0]; o[1] = v0[1]; o[2] = v0[2]; o[3] = eps;
	o[4] = e1[0]; o[5] = e1[1]; o[6] = e1[2];
	intAsFloatBits(prim, o[7]);
	o[8] = e2[0]; o[9] = e2[1]; o[10] = e2[2]; o[11] = 0.f;
}

BvhOutput buildBvh(const BvhInput &in, int leaf_size, int threads)
{
	BvhOutput out;
	Builder b(in, leaf_size);
	if(in.node_cost > 0.f) b.node_cost = in.node_cost;
	const int n = in.n_tris;
	b.tri_box.resize(n);
	b.cent.resize(3 * (size_t)n);
	b.order.resize(n);
	for(int t = 0; t < n; ++t)
	{
		const float *p0 = in.verts + 3 * in.tris[3 * t], *p1 = in.verts + 3 * in.tris[3 * t + 1], *p2 = in.verts + 3 * in.tris[3 * t + 2];
		Box bx;
		bx.grow(p0);
		bx.grow(p1);
		bx.grow(p2);
		b.tri_box[t] = bx;
		for(int k = 0; k < 3; ++k) b.cent[3 * t + k] = 0.5f * (bx.lo[k] + bx.hi[k]);
		b.order[t] = t;
	}
	b.nodes.reserve(2 * (size_t)std::max(1, n / std::max(1, leaf_size)) + 16);
	int par = 0;
	for(int t = threads; t > 1; t >>= 1) ++par;
	const int root = (n > 0) ? b.build(0, n, par) : -1;

	// flatten: inner nodes get device indices in DFS order; leaves are folded into their parent
	std::vector<int> dev_index(b.nodes.size(), -1);
	std::vector<int> stack;
	std::vector<int> inner_order;
	std::vector<int> depth_of(b.nodes.size(), 0);
	if(root >= 0 && b.nodes[root].left >= 0) stack.push_back(root);
	while(!stack.empty())
	{
		const int id = stack.back();
		stack.pop_back();
		dev_index[id] = (int)inner_order.size();
		inner_order.push_back(id);
		out.depth = std::max(out.depth, depth_of[id] + 1);
		const BuildNode &nd = b.nodes[id];
		for(int c : {nd.right, nd.left})
			if(b.nodes[c].left >= 0) { depth_of[c] = depth_of[id] + 1; stack.push_back(c); }
	}
	// triangles in leaf order
	out.tris.resize(12 * (size_t)n);
	for(int i = 0; i < n; ++i)
	{
		const int t = b.order[i];
		packTriangle(in.verts + 3 * in.tris[3 * t], in.verts + 3 * in.tris[3 * t + 1], in.verts + 3 * in.tris[3 * t + 2], t,
		             &out.tris[12 * (size_t)i]);
	}
	auto writeChild = [&](const BuildNode &c, int ci, float *lo, float *hi, int &child, int &count) {
		if(ci < 0 || (c.count == 0 && c.left < 0))
		{
			lo[0] = lo[1] = lo[2] = 1.f;
			hi[0] = hi[1] = hi[2] = -1.f;
			child = -1;
			count = 0;
			return;
		}
		padBox(c.box, lo, hi);
		if(c.left >= 0) { child = dev_index[ci]; count = 0; }
		else
		{
			child = ~c.start;
			count = c.count;
			out.max_leaf = std::max(out.max_leaf, c.count);
		}
	};
	if(in.width == 4)
	{
		// BVH4: collapse the binary tree — each wide node takes the two children of a binary node
		// and keeps opening its inner child of largest surface area until it holds four children.
		// Layout per node (8 float4): lo.x[4], hi.x[4], lo.y[4], hi.y[4], lo.z[4], hi.z[4],
		// child[4] (inner: node index >= 0; leaf: ~first triangle; empty: -1), count[4] (0 inner/empty, n leaf).
		out.width = 4;
		std::vector<int> wide_of;   // BuildNode index of each wide node's binary source
		std::vector<std::array<int, 4>> kids;
		std::vector<int> wdepth;
		std::vector<int> index_of(b.nodes.size(), -1);
		wide_of.push_back(root);
		kids.push_back({-1, -1, -1, -1});
		wdepth.push_back(1);
		for(size_t w = 0; w < wide_of.size(); ++w)
		{
			// a leaf (or empty) root becomes the single child of a synthetic wide root
			std::vector<int> list;
			if(wide_of[w] < 0) {}
			else if(b.nodes[wide_of[w]].left < 0) list.push_back(wide_of[w]);
			else list = {b.nodes[wide_of[w]].left, b.nodes[wide_of[w]].right};
			while(list.size() < 4)
			{
				int best = -1;
				float best_area = -1.f;
				for(size_t k = 0; k < list.size(); ++k)
				{
					const BuildNode &c = b.nodes[list[k]];
					if(c.left >= 0 && c.box.area() > best_area) { best_area = c.box.area(); best = (int)k; }
				}
				if(best < 0) break;
				const BuildNode &c = b.nodes[list[best]];
				list[best] = c.left;
				list.insert(list.begin() + best + 1, c.right);
			}
			for(size_t k = 0; k < list.size(); ++k)
			{
				kids[w][k] = list[k];
				if(b.nodes[list[k]].left >= 0)
				{
					index_of[list[k]] = (int)wide_of.size();
					wide_of.push_back(list[k]);
					kids.push_back({-1, -1, -1, -1});
					wdepth.push_back(wdepth[w] + 1);
				}
			}
		}
		out.n_nodes = (int)wide_of.size();
		out.depth = 0;
		for(int dd : wdepth) out.depth = std::max(out.depth, dd);
		out.nodes.assign(32 * (size_t)out.n_nodes, 0.f);
		for(int w = 0; w < out.n_nodes; ++w)
		{
			float *o = &out.nodes[32 * (size_t)w];
			for(int k = 0; k < 4; ++k)
			{
				const int ci = kids[w][k];
				float lo[3] = {1.f, 1.f, 1.f}, hi[3] = {-1.f, -1.f, -1.f};
				int child = -1, count = 0;
				if(ci >= 0)
				{
					const BuildNode &c = b.nodes[ci];
					if(c.left >= 0 || c.count > 0)
					{
						padBox(c.box, lo, hi);
						if(c.left >= 0) { child = index_of[ci]; count = 0; }
						else
						{
							child = ~c.start;
							count = c.count;
							out.max_leaf = std::max(out.max_leaf, c.count);
						}
					}
				}
				o[0 + k] = lo[0]; o[4 + k] = hi[0];
				o[8 + k] = lo[1]; o[12 + k] = hi[1];
				o[16 + k] = lo[2]; o[20 + k] = hi[2];
				intAsFloatBits(child, o[24 + k]);
				intAsFloatBits(count, o[28 + k]);
			}
		}
		// children are numbered after their parent, so one reverse sweep sees every subtree first
		std::vector<int> need(out.n_nodes, 0);
		for(int w = out.n_nodes - 1; w >= 0; --w)
		{
			int inner = 0, deepest = 0;
			for(int k = 0; k < 4; ++k)
				if(kids[w][k] >= 0 && b.nodes[kids[w][k]].left >= 0)
				{
					++inner;
					deepest = std::max(deepest, need[index_of[kids[w][k]]]);
				}
			need[w] = std::max(0, inner - 1) + deepest;
		}
		out.stack_need = need[0];
		return out;
	}
	if(inner_order.empty())
	{
		// a single leaf (or an empty scene): synthesise an inner root with one leaf child
		out.nodes.assign(16, 0.f);
		float lo0[3], hi0[3], lo1[3], hi1[3];
		int c0, k0, c1, k1;
		BuildNode empty;
		if(root >= 0) writeChild(b.nodes[root], root, lo0, hi0, c0, k0);
		else writeChild(empty, -1, lo0, hi0, c0, k0);
		writeChild(empty, -1, lo1, hi1, c1, k1);
		float *o = out.nodes.data();
		o[0] = lo0[0]; o[1] = hi0[0]; o[2] = lo0[1]; o[3] = hi0[1];
		o[4] = lo1[0]; o[5] = hi1[0]; o[6] = lo1[1]; o[7] = hi1[1];
		o[8] = lo0[2]; o[9] = hi0[2]; o[10] = lo1[2]; o[11] = hi1[2];
		intAsFloatBits(c0, o[12]); intAsFloatBits(c1, o[13]); intAsFloatBits(k0, o[14]); intAsFloatBits(k1, o[15]);
		out.n_nodes = 1;
		out.depth = 1;
		return out;
	}
	out.n_nodes = (int)inner_order.size();
	out.nodes.assign(16 * (size_t)out.n_nodes, 0.f);
	for(int d = 0; d < out.n_nodes; ++d)
	{
		const BuildNode &nd = b.nodes[inner_order[d]];
		float lo0[3], hi0[3], lo1[3], hi1[3];
		int c0, k0, c1, k1;
		writeChild(b.nodes[nd.left], nd.left, lo0, hi0, c0, k0);
		writeChild(b.nodes[nd.right], nd.right, lo1, hi1, c1, k1);
		float *o = &out.nodes[16 * (size_t)d];
		o[0] = lo0[0]; o[1] = hi0[0]; o[2] = lo0[1]; o[3] = hi0[1];
		o[4] = lo1[0]; o[5] = hi1[0]; o[6] = lo1[1]; o[7] = hi1[1];
		o[8] = lo0[2]; o[9] = hi0[2]; o[10] = lo1[2]; o[11] = hi1[2];
		intAsFloatBits(c0, o[12]); intAsFloatBits(c1, o[13]); intAsFloatBits(k0, o[14]); intAsFloatBits(k1, o[15]);
	}
	return out;
}

} // namespace yafamd
