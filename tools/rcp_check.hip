// Exhaustive check: is rcp + one FMA Newton step the correctly rounded 1/b for every normal float
// b with 2^-125 <= |b| <= 2^125?  (The triangle test needs the reference's correctly rounded
// 1.f / det bit for bit.)  Build: hipcc --offload-arch=gfx950 -O3 tools/rcp_check.hip -o tools/rcp_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void check(uint32_t hi_base, unsigned long long *bad, uint32_t *first)
{
	const uint32_t bits = hi_base + blockIdx.x * blockDim.x + threadIdx.x;
	const float b = __uint_as_float(bits);
	const float ab = fabsf(b);
	if(!(ab >= 0x1p-125f && ab <= 0x1p125f)) return;
	const float y = __builtin_amdgcn_rcpf(b);
	const float e = __builtin_fmaf(-b, y, 1.f);
	const float y2 = __builtin_fmaf(y, e, y);
	const float ref = 1.f / b;
	if(__float_as_uint(y2) != __float_as_uint(ref))
	{
		const unsigned long long k = atomicAdd(bad, 1ull);
		if(k < 16) first[k] = bits;
	}
}

int main()
{
	unsigned long long *bad;
	uint32_t *first;
	hipMalloc(&bad, 8);
	hipMalloc(&first, 64);
	hipMemset(bad, 0, 8);
	const uint32_t chunk = 1u << 28;
	for(uint64_t base = 0; base < (1ull << 32); base += chunk)
		hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, (uint32_t)base, bad, first);
	unsigned long long h = 0;
	uint32_t f[16] = {0};
	hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
	hipMemcpy(f, first, 64, hipMemcpyDeviceToHost);
	printf("mismatches: %llu\n", h);
	for(int i = 0; i < 16 && i < (int)h; ++i) printf("  b = %a (0x%08x)\n", (double)__builtin_bit_cast(float, f[i]), f[i]);
	return h ? 1 : 0;
}
