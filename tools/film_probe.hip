// Probe: k_film weights for one adaptive pass with synthetic inputs (diagnostics only).
#include "../libyafaray_amd/csrc/kernels.hip"
#include <cstdio>
#include <vector>

int main(int argc, char **argv)
{
	const int W = 48, H = 40, spp = 2;
	const int accumulate = argc > 1 ? atoi(argv[1]) : 1;
	const int use_flags = argc > 2 ? atoi(argv[2]) : 1;
	DevFilm F{};
	for(int i = 0; i < 256; ++i) F.table[i] = 1.f;
	F.filterw = 0.501f;
	F.table_scale = (float)(0.9999 * 16 / F.filterw);
	F.reach_fwd = 1;
	F.reach_back = 0;
	F.width = W; F.height = H; F.spp = spp; F.tile = 32;
	F.multipass = 1;
	F.sample_offset = 5;
	float4 *samples, *accum, *out;
	float *weights;
	uint8_t *flags;
	hipMalloc(&samples, (size_t)W * H * spp * 16);
	hipMalloc(&accum, (size_t)W * H * 16);
	hipMalloc(&out, (size_t)W * H * 16);
	hipMalloc(&weights, (size_t)W * H * 4);
	hipMalloc(&flags, (size_t)W * H);
	hipMemset(samples, 0, (size_t)W * H * spp * 16);
	hipMemset(accum, 0, (size_t)W * H * 16);
	hipMemset(weights, 0, (size_t)W * H * 4);
	hipMemset(flags, 1, (size_t)W * H);
	yafamd_launch_film(&F, samples, use_flags ? flags : nullptr, accum, out, weights, 0, H, 0.f, accumulate, 0);
	hipDeviceSynchronize();
	std::vector<float> w((size_t)W * H);
	hipMemcpy(w.data(), weights, w.size() * 4, hipMemcpyDeviceToHost);
	printf("accumulate %d flags %d: w(3,40)=%g w(8,29)=%g w(2,39)=%g w(0,0)=%g\n", accumulate, use_flags, w[3 * W + 40], w[8 * W + 29],
	       w[2 * W + 39], w[0]);
	return 0;
}
