// PMC calibration probe (VERDICT r03 "What's weak" #6): what rocprofv3's FETCH_SIZE reports for the
// access shapes the gather and traversal kernels use, against a byte count known by construction.
// Every kernel reads from a 4 GiB buffer (far past the 256 MiB Infinity Cache, so every line comes
// from HBM once) and touches each 128-B line at most once:
//   k_stream16   16 B per lane, coalesced stream                        known = 16 B x reads
//   k_node128    one 128-B line per lane (8 x float4), random lines     known = 128 B x lanes
//   k_log8       a run of 139 8-B entries per lane (1112 B, lanes 4 KiB apart: the gather log)
//                                                                       known = the 128-B lines the runs cover
//   k_scatter16  one float4 per lane from its own random 128-B line     known = 16 B requested per lane;
//                                                                       a line is 128 B
//   k_scatter16x3  three float4 per lane, each from its own line (the photon records' three arrays)
//   k_node16     one 16-B kd node per lane from random lines (k_gather_walk's node fetch)
// Usage: pmc_probe <kernel name | all>; prints the known bytes per kernel.  tools/pmc_probe.sh runs
// each kernel under `rocprofv3 --pmc FETCH_SIZE` and writes profiles/pmc_calibration.json.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>

#define CK(x)                                                                                   \
	do                                                                                          \
	{                                                                                           \
		hipError_t e_ = (x);                                                                    \
		if(e_ != hipSuccess)                                                                    \
		{                                                                                       \
			std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
			std::exit(1);                                                                       \
		}                                                                                       \
	} while(0)

constexpr size_t kBytes = (size_t)4 << 30;   // 4 GiB
constexpr size_t kLines = kBytes / 128;      // 33.5 M lines of 128 B
constexpr uint32_t kLanes = 1u << 22;        // 4 M lanes for the random patterns

// a bijection on [0, kLines): odd multiplier mod 2^25 (kLines = 2^25), so no line is read twice
__device__ __forceinline__ uint32_t perm(uint32_t i) { return (i * 2654435761u + 12345u) & (uint32_t)(kLines - 1); }

__global__ void k_stream16(const float4 *in, size_t n, float *out)
{
	float acc = 0.f;
	for(size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
	{
		const float4 v = in[i];
		acc += v.x + v.y + v.z + v.w;
	}
	if(acc == 1.2345f) out[0] = acc;   // never true for the zeroed buffer: keeps the loads
}

__global__ void k_node128(const float4 *in, float *out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= kLanes) return;
	const float4 *p = in + (size_t)perm(i) * 8;
	float acc = 0.f;
#pragma unroll
	for(int k = 0; k < 8; ++k)
	{
		const float4 v = p[k];
		acc += v.x + v.y + v.z + v.w;
	}
	if(acc == 1.2345f) out[0] = acc;
}

constexpr uint32_t kLogLen = 139, kLogStride = 512;   // entries (8 B); the gather log's mean accepted count and cap
__global__ void k_log8(const uint2 *in, uint32_t lanes, float *out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= lanes) return;
	const uint2 *p = in + (size_t)i * kLogStride;
	uint32_t acc = 0;
	for(uint32_t a = 0; a < kLogLen; a += 2)
	{
		// pairs as 16-B loads, as k_gather's replay reads them
		if(a + 1 < kLogLen)
		{
			const uint4 v = *reinterpret_cast<const uint4 *>(p + a);
			acc += v.x ^ v.y ^ v.z ^ v.w;
		}
		else acc += p[a].x ^ p[a].y;
	}
	if(acc == 12345u) out[0] = (float)acc;
}

__global__ void k_scatter16(const float4 *in, float *out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= kLanes) return;
	const float4 v = in[(size_t)perm(i) * 8];
	const float acc = v.x + v.y + v.z + v.w;
	if(acc == 1.2345f) out[0] = acc;
}

__global__ void k_scatter16x3(const float4 *in, float *out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= kLanes) return;
	// three arrays of one photon index: lines perm(i), perm(i + kLanes), perm(i + 2 kLanes)
	const float4 a = in[(size_t)perm(i) * 8], b = in[(size_t)perm(i + kLanes) * 8], c = in[(size_t)perm(i + 2 * kLanes) * 8];
	const float acc = a.x + b.y + c.z + a.w;
	if(acc == 1.2345f) out[0] = acc;
}

__global__ void k_node16(const uint4 *in, float *out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= kLanes) return;
	const uint4 v = in[(size_t)perm(i) * 8];
	const uint32_t acc = v.x ^ v.w;
	if(acc == 12345u) out[0] = (float)acc;
}

int main(int argc, char **argv)
{
	const std::string which = argc > 1 ? argv[1] : "all";
	void *buf = nullptr;
	float *out = nullptr;
	CK(hipMalloc(&buf, kBytes));
	CK(hipMalloc(&out, 16));
	CK(hipMemset(buf, 0, kBytes));
	CK(hipDeviceSynchronize());
	const dim3 blk(256), grid_r((kLanes + 255) / 256);
	auto run = [&](const char *name, double known, auto launch) {
		if(which != "all" && which != name) return;
		launch();
		CK(hipGetLastError());
		CK(hipDeviceSynchronize());
		std::printf("{\"kernel\": \"%s\", \"known_bytes\": %.0f}\n", name, known);
	};
	const size_t n16 = kBytes / 16;
	run("k_stream16", (double)kBytes, [&] { hipLaunchKernelGGL(k_stream16, dim3(4096), blk, 0, 0, (const float4 *)buf, n16, out); });
	run("k_node128", 128.0 * kLanes, [&] { hipLaunchKernelGGL(k_node128, grid_r, blk, 0, 0, (const float4 *)buf, out); });
	{
		// the log runs: lanes 4 KiB apart, 1112 B each from a 4 KiB-aligned base -> ceil(1112 / 128) = 9 lines
		const uint32_t lanes = (uint32_t)(kBytes / (kLogStride * 8));
		const double lines = 9.0 * lanes;
		run("k_log8", 128.0 * lines, [&] { hipLaunchKernelGGL(k_log8, dim3((lanes + 255) / 256), blk, 0, 0, (const uint2 *)buf, lanes, out); });
	}
	run("k_scatter16", 16.0 * kLanes, [&] { hipLaunchKernelGGL(k_scatter16, grid_r, blk, 0, 0, (const float4 *)buf, out); });
	run("k_scatter16x3", 48.0 * kLanes, [&] { hipLaunchKernelGGL(k_scatter16x3, grid_r, blk, 0, 0, (const float4 *)buf, out); });
	run("k_node16", 16.0 * kLanes, [&] { hipLaunchKernelGGL(k_node16, grid_r, blk, 0, 0, (const uint4 *)buf, out); });
	CK(hipFree(buf));
	CK(hipFree(out));
	return 0;
}
