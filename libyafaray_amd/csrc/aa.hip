// Adaptive anti-aliasing on the GPU: ImageFilm::nextPass (reference src/render/imagefilm.cc:259-420)
// as data-parallel kernels over the accumulated film, plus the list of pixels the next pass
// resamples in the reference's visiting order (tiles of the linear order, rows inside a tile:
// integrator_tiled.cc:269-290, imagesplitter.cc:30-107).
//
// The reference walks source pixels (x, y) < (W - 1, H - 1) and, when the colour difference to a
// neighbour reaches the source's threshold, flags both pixels.  Flags are only ever set, so the
// result is order-free: here every pixel gathers the comparisons that would flag it — as a source
// (right, down, down-right, down-left) and as the neighbour of the sources left, up, up-left and
// up-right of it — each against that source's threshold.  Variance windows (AA_variance_pixels)
// are a first pass per source and a window gather per pixel.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdint>

#include "devscene.h"

namespace
{

using yafamd::DevAaParams;

constexpr int kB = 256;

struct Film
{
	const float4 *acc;
	const float *w;
	int W, H;
	// Rgba::normalized (color.h:554-558; operator/ multiplies by the reciprocal, :312-316)
	__device__ float4 color(int x, int y) const
	{
		const size_t p = (size_t)y * W + x;
		const float wt = w[p];
		if(wt == 0.f) return make_float4(0.f, 0.f, 0.f, 0.f);
		const float f = 1.f / wt;
		const float4 c = acc[p];
		return make_float4(c.x * f, c.y * f, c.z * f, c.w * f);
	}
};

// imagefilm.cc:799-815
__device__ float darkCurve(float b)
{
	if(b <= 0.10f) return 0.0001f;
	else if(b <= 0.20f) return (0.0001f + (b - 0.10f) * (0.0010f - 0.0001f) / 0.10f);
	else if(b <= 0.30f) return (0.0010f + (b - 0.20f) * (0.0020f - 0.0010f) / 0.10f);
	else if(b <= 0.40f) return (0.0020f + (b - 0.30f) * (0.0035f - 0.0020f) / 0.10f);
	else if(b <= 0.50f) return (0.0035f + (b - 0.40f) * (0.0055f - 0.0035f) / 0.10f);
	else if(b <= 0.60f) return (0.0055f + (b - 0.50f) * (0.0075f - 0.0055f) / 0.10f);
	else if(b <= 0.70f) return (0.0075f + (b - 0.60f) * (0.0100f - 0.0075f) / 0.10f);
	else if(b <= 0.80f) return (0.0100f + (b - 0.70f) * (0.0150f - 0.0100f) / 0.10f);
	else if(b <= 0.90f) return (0.0150f + (b - 0.80f) * (0.0250f - 0.0150f) / 0.10f);
	else if(b <= 1.00f) return (0.0250f + (b - 0.90f) * (0.0400f - 0.0250f) / 0.10f);
	else if(b <= 1.20f) return (0.0400f + (b - 1.00f) * (0.0800f - 0.0400f) / 0.20f);
	else if(b <= 1.40f) return (0.0800f + (b - 1.20f) * (0.0950f - 0.0800f) / 0.20f);
	else if(b <= 1.80f) return (0.0950f + (b - 1.40f) * (0.1000f - 0.0950f) / 0.40f);
	else return 0.1000f;
}

// the threshold a source pixel compares with (imagefilm.cc:325-335, abscol2Bri color.h:62)
__device__ float sourceThreshold(const float4 &c, const DevAaParams &a, float threshold)
{
	const float bri = 0.2126f * fabsf(c.x) + 0.7152f * fabsf(c.y) + 0.0722f * fabsf(c.z);
	if(a.dark_type == 1 && a.dark_factor > 0.f) return threshold * ((1.f - a.dark_factor) + (bri * a.dark_factor));
	if(a.dark_type == 2) return darkCurve(bri);
	return threshold;
}

// Rgba::colorDifference (color.h:450-467), col2Bri (color.h:61)
__device__ float colorDifference(const float4 &a, const float4 &b, bool rgb)
{
	const float bri_a = 0.2126f * a.x + 0.7152f * a.y + 0.0722f * a.z;
	const float bri_b = 0.2126f * b.x + 0.7152f * b.y + 0.0722f * b.z;
	float d = fabsf(bri_b - bri_a);
	if(rgb)
	{
		const float rd = fabsf(b.x - a.x), gd = fabsf(b.y - a.y), bd = fabsf(b.z - a.z), ad = fabsf(b.w - a.w);
		if(d < rd) d = rd;
		if(d < gd) d = gd;
		if(d < bd) d = bd;
		if(d < ad) d = ad;
	}
	return d;
}

// source (x, y) -> does a neighbour comparison in direction (ox, oy) reach its threshold?
__device__ bool edge(const Film &F, const DevAaParams &a, float threshold, int x, int y, int ox, int oy)
{
	const float4 c = F.color(x, y);
	return colorDifference(c, F.color(x + ox, y + oy), a.detect_color_noise != 0) >= sourceThreshold(c, a, threshold);
}

// imagefilm.cc:354-385: the variance count of source (x, y)
__global__ void __launch_bounds__(kB) k_aa_variance(Film F, DevAaParams a, float threshold, uint8_t *var)
{
	const int x = blockIdx.x * kB + threadIdx.x, y = blockIdx.y;
	if(x >= F.W) return;
	const int W = F.W, H = F.H;
	uint8_t v = 0;
	if(x < W - 1 && y < H - 1)
	{
		const float th = sourceThreshold(F.color(x, y), a, threshold);
		const bool rgb = a.detect_color_noise != 0;
		const int half = a.variance_edge / 2;
		int vx = 0, vy = 0;
		for(int xd = -half; xd < half - 1; ++xd)
		{
			int xi = x + xd;
			if(xi < 0) xi = 0;
			else if(xi >= W - 1) xi = W - 2;
			if(colorDifference(F.color(xi, y), F.color(xi + 1, y), rgb) >= th) ++vx;
		}
		for(int yd = -half; yd < half - 1; ++yd)
		{
			int yi = y + yd;
			if(yi < 0) yi = 0;
			else if(yi >= H - 1) yi = H - 2;
			if(colorDifference(F.color(x, yi), F.color(x, yi + 1), rgb) >= th) ++vy;
		}
		v = (vx + vy >= a.variance_pixels) ? 1 : 0;
	}
	var[(size_t)y * W + x] = v;
}

// is `p` among the clamped window coordinates {clamp(s + d, 0, n - 1) : d in [-half, half)}?
__device__ __forceinline__ bool inWindow(int p, int s, int half, int n)
{
	if(p > 0 && p < n - 1) return p >= s - half && p <= s + half - 1;
	if(p == 0) return s - half <= 0;
	return s + half - 1 >= n - 1;   // p == n - 1
}

__global__ void __launch_bounds__(kB) k_aa_flags(Film F, DevAaParams a, float threshold, const uint8_t *var, uint8_t *flags)
{
	const int x = blockIdx.x * kB + threadIdx.x, y = blockIdx.y;
	const int W = F.W, H = F.H;
	if(x >= W) return;
	bool f = !(F.w[(size_t)y * W + x] > 0.f);   // :302-309: unrendered (or zero-weight) pixels
	const bool src = x < W - 1 && y < H - 1;
	// as the source of the comparison
	if(!f && src)
		f = edge(F, a, threshold, x, y, 1, 0) || edge(F, a, threshold, x, y, 0, 1) || edge(F, a, threshold, x, y, 1, 1) ||
		    (x > 0 && edge(F, a, threshold, x, y, -1, 1));
	// as the neighbour of the sources left, up, up-left, up-right of it
	if(!f && x > 0 && y < H - 1) f = edge(F, a, threshold, x - 1, y, 1, 0);
	if(!f && y > 0 && x < W - 1) f = edge(F, a, threshold, x, y - 1, 0, 1);
	if(!f && x > 0 && y > 0) f = edge(F, a, threshold, x - 1, y - 1, 1, 1);
	if(!f && y > 0 && x + 1 < W - 1) f = edge(F, a, threshold, x + 1, y - 1, -1, 1);
	if(!f && a.variance_pixels > 0)
	{
		// sources whose flag window covers this pixel (imagefilm.cc:387-400)
		const int half = a.variance_edge / 2;
		const int sx0 = (x == 0) ? 0 : x - half + 1, sx1 = (x == W - 1) ? W - 2 : min(W - 2, x + half);
		const int sy0 = (y == 0) ? 0 : y - half + 1, sy1 = (y == H - 1) ? H - 2 : min(H - 2, y + half);
		for(int sy = max(0, sy0); sy <= sy1 && !f; ++sy)
			for(int sx = max(0, sx0); sx <= sx1 && !f; ++sx)
				if(var[(size_t)sy * W + sx] && inWindow(x, sx, half, W) && inWindow(y, sy, half, H)) f = true;
	}
	flags[(size_t)y * W + x] = f ? 1 : 0;
}

// visiting position q -> pixel (tile rows top to bottom, tiles left to right, rows in a tile)
__device__ __forceinline__ void visitPixel(uint32_t q, int W, int H, int ts, int &x, int &y)
{
	const uint32_t band_px = (uint32_t)W * (uint32_t)ts;
	const int r = (int)(q / band_px);
	const int y0 = r * ts, bh = min(ts, H - y0);
	const uint32_t l = q - (uint32_t)r * band_px;
	const uint32_t per_tile = (uint32_t)ts * (uint32_t)bh;
	const int tx = (int)(l / per_tile);
	const int tw = min(ts, W - tx * ts);
	const uint32_t k = l - (uint32_t)tx * per_tile;
	x = tx * ts + (int)(k % (uint32_t)tw);
	y = y0 + (int)(k / (uint32_t)tw);
}

// fq[q] = pixel q of the visiting order is resampled and lies in rows [ry0, ry1)
__global__ void __launch_bounds__(kB) k_aa_order(const uint8_t *flags, int W, int H, int ts, int ry0, int ry1, uint32_t *fq)
{
	const uint32_t q = blockIdx.x * kB + threadIdx.x, n = (uint32_t)W * (uint32_t)H;
	if(q > n) return;
	if(q == n) { fq[n] = 0; return; }
	int x, y;
	visitPixel(q, W, H, ts, x, y);
	fq[q] = (y >= ry0 && y < ry1) ? flags[(size_t)y * W + x] : 0u;
}

__global__ void __launch_bounds__(kB) k_aa_scatter(const uint32_t *fq, const uint32_t *pos, int W, int H, int ts, uint32_t *plist)
{
	const uint32_t q = blockIdx.x * kB + threadIdx.x, n = (uint32_t)W * (uint32_t)H;
	if(q >= n || !fq[q]) return;
	int x, y;
	visitPixel(q, W, H, ts, x, y);
	plist[pos[q]] = (uint32_t)y * (uint32_t)W + (uint32_t)x;
}

struct DevBuf
{
	void *p = nullptr;
	~DevBuf() { if(p) (void)hipFree(p); }
	hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes < 16 ? 16 : bytes); }
};

#define AACHECK(x) do { hipError_t e_ = (x); if(e_ != hipSuccess) return e_; } while(0)

} // namespace

// nextPass: flags (W*H bytes) and the resampled pixels in visiting order (plist, W*H entries);
// *count = how many.  threshold <= 0 resamples every pixel (doMoreSamples, imagefilm.cc:672-675).
// Rows [ry0, ry1) (a group member's band + halo rows): plist holds only the resampled pixels of those
// rows, *local_count of them; *count stays the whole film's.
extern "C" hipError_t yafamd_aa_next_pass(const float4 *accum, const float *weights, int W, int H, int tile, const DevAaParams *prm,
                                          float threshold, uint8_t *flags, uint32_t *plist, uint32_t *count, int ry0, int ry1,
                                          uint32_t *local_count, hipStream_t st)
{
	const uint32_t n = (uint32_t)W * (uint32_t)H;
	Film F{accum, weights, W, H};
	const dim3 grid((W + kB - 1) / kB, H);
	if(!(threshold > 0.f)) AACHECK(hipMemsetAsync(flags, 1, n, st));
	else
	{
		DevBuf var;
		if(prm->variance_pixels > 0)
		{
			AACHECK(var.alloc(n));
			hipLaunchKernelGGL(k_aa_variance, grid, dim3(kB), 0, st, F, *prm, threshold, (uint8_t *)var.p);
		}
		hipLaunchKernelGGL(k_aa_flags, grid, dim3(kB), 0, st, F, *prm, threshold, (const uint8_t *)var.p, flags);
		AACHECK(hipGetLastError());
	}
	DevBuf fq, pos, tmp;
	AACHECK(fq.alloc((size_t)(n + 1) * 4));
	AACHECK(pos.alloc((size_t)(n + 1) * 4));
	const bool part = ry0 > 0 || ry1 < H;
	size_t bytes = 0;
	AACHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (uint32_t *)fq.p, (uint32_t *)pos.p, (int)n + 1, st));
	AACHECK(tmp.alloc(bytes));
	if(part)
	{
		// the whole film's count first (the pass loop's threshold decay uses it)
		hipLaunchKernelGGL(k_aa_order, dim3((n + 1 + kB - 1) / kB), dim3(kB), 0, st, flags, W, H, tile, 0, H, (uint32_t *)fq.p);
		AACHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, bytes, (uint32_t *)fq.p, (uint32_t *)pos.p, (int)n + 1, st));
		AACHECK(hipMemcpyAsync(count, (uint32_t *)pos.p + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
		AACHECK(hipStreamSynchronize(st));
	}
	hipLaunchKernelGGL(k_aa_order, dim3((n + 1 + kB - 1) / kB), dim3(kB), 0, st, flags, W, H, tile, part ? ry0 : 0, part ? ry1 : H, (uint32_t *)fq.p);
	AACHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, bytes, (uint32_t *)fq.p, (uint32_t *)pos.p, (int)n + 1, st));
	hipLaunchKernelGGL(k_aa_scatter, dim3((n + kB - 1) / kB), dim3(kB), 0, st, (const uint32_t *)fq.p, (const uint32_t *)pos.p, W, H, tile, plist);
	AACHECK(hipGetLastError());
	AACHECK(hipMemcpyAsync(local_count, (uint32_t *)pos.p + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
	AACHECK(hipStreamSynchronize(st));
	if(!part) *count = *local_count;
	return hipSuccess;
}
