// Host check: libyafaray_amd/csrc/photonheap.h reproduces std::make_heap / pop_heap / push_heap
// element for element on PhotonGather's access pattern (src/photon/photon.cc:31-52), including
// equal distances.  Built and run by tests/test_photon.py.
#include "../libyafaray_amd/csrc/photonheap.h"
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

using namespace yafamd;

struct Found
{
	uint32_t i;
	float d;
	bool operator<(const Found &o) const { return d < o.d; }
};

int main()
{
	std::mt19937 rng(2024);
	long bad = 0, runs = 0;
	for(int k : {1, 2, 3, 4, 5, 7, 8, 16, 49, 50, 51, 64})
		for(int trial = 0; trial < 300; ++trial)
		{
			const int n = 1 + (int)(rng() % 400);
			const int levels = (trial % 3 == 0) ? 5 : 100000;   // many ties in a third of the runs
			std::vector<Found> ref(k);
			std::vector<uint32_t> hi(k);
			std::vector<float> hd(k);
			HeapRef h{hi.data(), hd.data(), 1};
			uint32_t found = 0;
			float max_ref = 1e30f, max_mine = 1e30f;
			for(int c = 0; c < n; ++c)
			{
				const float d = (float)(rng() % levels) * 0.25f;
				if(d >= max_ref) continue;
				if(found < (uint32_t)k)
				{
					ref[found] = {(uint32_t)c, d};
					hi[found] = (uint32_t)c;
					hd[found] = d;
					++found;
					if(found == (uint32_t)k)
					{
						std::make_heap(ref.begin(), ref.end());
						heapMake(h, k);
						max_ref = ref[0].d;
						max_mine = hd[0];
					}
				}
				else
				{
					std::pop_heap(ref.begin(), ref.end());
					ref[k - 1] = {(uint32_t)c, d};
					std::push_heap(ref.begin(), ref.end());
					heapReplaceTop(h, k, (uint32_t)c, d);
					max_ref = ref[0].d;
					max_mine = hd[0];
				}
				if(max_ref != max_mine) ++bad;
			}
			for(uint32_t q = 0; q < found; ++q)
				if(ref[q].i != hi[q] || ref[q].d != hd[q]) { ++bad; break; }
			++runs;
		}
	printf("runs=%ld bad=%ld\n", runs, bad);
	return bad ? 1 : 0;
}
