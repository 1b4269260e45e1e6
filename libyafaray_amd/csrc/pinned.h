// Page-locked host allocations (render.cc pinnedAlloc / pinnedFree) for host buffers the GPU fills
// every frame.
#pragma once

#include <cstddef>
#include <new>
#include <vector>

namespace yafamd
{

// Page-locked host memory (hipHostMalloc) for the film the flush downloads every frame: the copy runs at
// PCIe DMA speed instead of through a pageable bounce buffer (imagefilm.cc:570-670's flush is part of the
// reference's render()).  Falls back to malloc when pinning fails.
void *pinnedAlloc(size_t bytes);
void pinnedFree(void *p);
template<class T>
struct PinnedAlloc
{
	using value_type = T;
	PinnedAlloc() = default;
	template<class U> PinnedAlloc(const PinnedAlloc<U> &) {}
	T *allocate(size_t n)
	{
		void *p = pinnedAlloc(n * sizeof(T));
		if(!p) throw std::bad_alloc();
		return static_cast<T *>(p);
	}
	void deallocate(T *p, size_t) { pinnedFree(p); }
	template<class U> bool operator==(const PinnedAlloc<U> &) const { return true; }
	template<class U> bool operator!=(const PinnedAlloc<U> &) const { return false; }
};
using PinnedFloats = std::vector<float, PinnedAlloc<float>>;

} // namespace yafamd
