// k-nearest-photon max-heap with exactly the element moves of libstdc++'s std::make_heap /
// std::pop_heap / std::push_heap (bits/stl_heap.h: __adjust_heap, __push_heap), which the
// reference's PhotonGather uses on FoundPhoton (operator< on the squared distance;
// src/photon/photon.cc:31-52).  The density estimate sums the found photons in heap-array order
// (integrator_photon_mapping.cc:964-975), so reproducing the array order bit for bit requires the
// same algorithm, not just any heap.  Compiled for the device (kernels.hip) and for the host
// (tests/photon_check.cc pins it against std:: on random inputs with ties).
#pragma once

#include <cstdint>
#include <type_traits>

#if defined(__HIPCC__)
#define YPH __host__ __device__ __forceinline__
#else
#define YPH inline
#endif

namespace yafamd
{

// Heap storage accessor: entries are (photon index, squared distance), possibly strided in LDS.
struct HeapRef
{
	uint32_t *idx;
	float *dist;
	int stride;   // distance in elements between consecutive heap slots (lanes interleaved in LDS)
	YPH uint32_t &i(int k) const { return idx[k * stride]; }
	YPH float &d(int k) const { return dist[k * stride]; }
};

// Packed storage: slot k = (index, distance bits) in one 8-byte word, so a slot moves with one
// 64-bit LDS read / write (k_gather: lanes interleaved, stride = workgroup lanes).
struct HeapRefPacked
{
	uint32_t *e;   // e[2 * k * stride] = index, e[2 * k * stride + 1] = distance bits
	int stride;
	YPH uint32_t &i(int k) const { return e[2 * k * stride]; }
	YPH float &d(int k) const { return reinterpret_cast<float *>(e)[2 * k * stride + 1]; }
};

// Split storage for a replayed gather (k_gather<REPLAY>): slot k = distance (32-bit column) + the
// entry's position in the request's accepted-photon log (16-bit column), 6 B per slot instead of 8,
// so more waves fit the CU's LDS; the photon index is read from the log when the estimate is summed.
struct HeapRefSplit
{
	uint32_t *dw;   // dw[k * stride] = distance bits
	uint16_t *iw;   // iw[k * stride] = log position
	int stride;
	YPH uint16_t &i(int k) const { return iw[k * stride]; }
	YPH float &d(int k) const { return reinterpret_cast<float *>(dw)[k * stride]; }
};

// __push_heap(first, holeIndex, topIndex, value)
template<class H> YPH void heapPushUp(const H &h, int hole, int top, uint32_t vi, float vd)
{
	int parent = (hole - 1) / 2;
	while(hole > top && h.d(parent) < vd)
	{
		h.i(hole) = h.i(parent);
		h.d(hole) = h.d(parent);
		hole = parent;
		parent = (hole - 1) / 2;
	}
	h.i(hole) = static_cast<typename std::remove_reference<decltype(h.i(0))>::type>(vi);
	h.d(hole) = vd;
}

// __adjust_heap(first, holeIndex, len, value)
template<class H> YPH void heapAdjust(const H &h, int hole, int len, uint32_t vi, float vd)
{
	const int top = hole;
	int second = hole;
	while(second < (len - 1) / 2)
	{
		second = 2 * (second + 1);
		if(h.d(second) < h.d(second - 1)) --second;
		h.i(hole) = h.i(second);
		h.d(hole) = h.d(second);
		hole = second;
	}
	if((len & 1) == 0 && second == (len - 2) / 2)
	{
		second = 2 * (second + 1);
		h.i(hole) = h.i(second - 1);
		h.d(hole) = h.d(second - 1);
		hole = second - 1;
	}
	heapPushUp(h, hole, top, vi, vd);
}

// std::make_heap(first, first + len)
template<class H> YPH void heapMake(const H &h, int len)
{
	if(len < 2) return;
	for(int parent = (len - 2) / 2;; --parent)
	{
		const uint32_t vi = h.i(parent);
		const float vd = h.d(parent);
		heapAdjust(h, parent, len, vi, vd);
		if(parent == 0) return;
	}
}

// std::pop_heap(first, first + len) followed by first[len - 1] = new value and
// std::push_heap(first, first + len): PhotonGather's "replace the farthest" step.
template<class H> YPH void heapReplaceTop(const H &h, int len, uint32_t ni, float nd)
{
	if(len > 1)
	{
		// __pop_heap: value = *(last - 1); *(last - 1) = *first; __adjust_heap(first, 0, len - 1, value)
		const uint32_t vi = h.i(len - 1);
		const float vd = h.d(len - 1);
		h.i(len - 1) = h.i(0);
		h.d(len - 1) = h.d(0);
		heapAdjust(h, 0, len - 1, vi, vd);
	}
	h.i(len - 1) = static_cast<typename std::remove_reference<decltype(h.i(0))>::type>(ni);
	h.d(len - 1) = nd;
	// __push_heap(first, len - 1, 0, value)
	heapPushUp(h, len - 1, 0, ni, nd);
}

} // namespace yafamd
