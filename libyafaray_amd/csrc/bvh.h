// Host-side BVH builder for the GPU traversal kernels.
//
// Replaces the reference's accelerator build (AcceleratorKdTree::buildTree,
// src/accelerator/accelerator_kdtree.cc:420-628, SAH kd-tree with clipping).  The closest /
// any hit a traversal returns does not depend on the acceleration structure, so
// a binned-SAH BVH2 whose inner nodes store both child boxes (one 64 B fetch per step, two slab
// tests) is a legal drop-in that maps far better onto wave64 SIMD than pointer-chasing kd nodes.
#pragma once

#include <cstdint>
#include <vector>

namespace yafamd
{

struct BvhInput
{
	const float *verts;     // xyz per vertex
	const int *tris;        // 3 vertex indices per triangle
	int n_tris;
	float node_cost = 0.f;   // SAH node cost (<= 0: default 0.5)
	int width = 4;           // 2: BVH2 (4 float4 per node), 4: BVH4 (8 float4 per node)
};

// The device build's optional 8-wide collapse of the same binary tree, quantised (bvhgpu.hip k_q8_write:
// 8 float4 per node) with its own copy of the triangle records in node order; k_trace's refill loop
// traverses it for scenes in global memory (opt-in YAFARAY_AMD_BVH8=1).
struct YafBvh8
{
	void *nodes = nullptr;   // device memory, owned by the caller
	void *tris = nullptr;    // device memory (3 float4 per triangle), owned by the caller
	int n_nodes = 0, depth = 0, stack_need = 0;
};

struct BvhOutput
{
	std::vector<float> nodes;   // 16 (BVH2) or 32 (BVH4) floats per node (devscene.h layout)
	int width = 2;
	std::vector<float> tris;    // 12 floats per triangle, leaf order (devscene.h layout)
	int n_nodes = 0;
	int depth = 0;              // inner-node depth (bounds the traversal stack)
	int max_leaf = 0;
	int stack_need = 0;         // worst-case traversal stack entries (BVH4: sum of deferred siblings along a path)
};

// Builds the tree.  `threads` > 1 builds independent subtrees concurrently.
BvhOutput buildBvh(const BvhInput &in, int leaf_size = 4, int threads = 1);

// The triangle record exactly as the device test consumes it (primitive_triangle.cc:47-49):
// v0, e1 = v1 - v0, e2 = v2 - v0, eps = 0.1f * min_raydist * max(|e1|, |e2|).
void packTriangle(const float *v0, const float *v1, const float *v2, int prim, float *out12);

} // namespace yafamd
