// Host-side (x86-64) numerics for the scene-setup values the GPU consumes: film filter table,
// camera frame, light frames, colour-space conversion.  Compiled by the host compiler, so the
// reference's `long double` expressions are evaluated in x87 80-bit exactly as the reference's
// own build does (include/math/math.h:46-250, include/math/filter.h:34-90).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstring>

namespace yafamd
{
namespace hm
{
using LD = long double;
constexpr LD num_pi = 3.1415926535897932384626433832795L;
constexpr LD div_pi_by_2 = 1.5707963267948966192313216916398L;
constexpr LD mult_pi_by_2 = 6.283185307179586476925286766559L;
constexpr LD div_pi_by_180 = 0.01745329251994329576923690768489L;
constexpr LD div_1_by_2pi = 0.15915494309189533576888376337251L;
constexpr LD div_4_by_pi = 1.2732395447351626861510701069801L;
constexpr LD div_4_by_squared_pi = 0.40528473456935108577551785283891L;
constexpr LD log2e = 1.4426950408889634073599246810019L;

inline float polyexp(float x)
{
	return x * (x * (x * (x * (x * 1.8775767e-3f + 8.9893397e-3f) + 5.5826318e-2f) + 2.4015361e-1f) + 6.9315308e-1f) + 9.9999994e-1f;
}
inline float exp2f_fast(float x)
{
	x = std::min(x, 129.00000f);
	x = std::max(x, -126.99999f);
	const int ip = static_cast<int>(x - 0.5f);
	const float fp = x - static_cast<float>(ip);
	const int ep = (ip + 127) << 23;
	float e;
	std::memcpy(&e, &ep, 4);
	return e * polyexp(fp);
}
inline float polylog(float x)
{
	return x * (x * (x * (x * (x * -3.4436006e-2f + 3.1821337e-1f) + -1.2315303f) + 2.5988452f) + -3.3241990f) + 3.1157899f;
}
inline float log2f_fast(float x)
{
	int i;
	std::memcpy(&i, &x, 4);
	const float e = static_cast<float>(((i & 0x7F800000) >> 23) - 127);
	const int mi = (i & 0x7FFFFF) | 0x3f800000;
	float m;
	std::memcpy(&m, &mi, 4);
	return polylog(m) * (m - 1.0f) + e;
}
inline float powf_fast(float a, float b) { return exp2f_fast(static_cast<float>(log2f_fast(a) * b)); }
inline float expf_fast(float a) { return exp2f_fast(static_cast<float>(log2e * a)); }
inline float sinf_fast(float x)
{
	if(x > mult_pi_by_2 || x < -mult_pi_by_2) x -= ((int)(x * static_cast<float>(div_1_by_2pi))) * static_cast<float>(mult_pi_by_2);
	if(x < -num_pi) x += static_cast<float>(mult_pi_by_2);
	else if(x > num_pi) x -= static_cast<float>(mult_pi_by_2);
	x = (static_cast<float>(div_4_by_pi * x)) - (static_cast<float>(div_4_by_squared_pi * x * std::abs(x)));
	const float result = 0.225f * (x * std::abs(x) - x) + x;
	if(result <= -1.f) return -1.f;
	else if(result >= 1.f) return 1.f;
	return result;
}
inline float cosf_fast(float x) { return sinf_fast(x + static_cast<float>(div_pi_by_2)); }   // math.h:247-254

// include/math/filter.h:34-90
inline float filterBox(float, float) { return 1.f; }
inline float filterGauss(float dx, float dy)
{
	const float r_2 = dx * dx + dy * dy;
	return std::max(0.f, expf_fast(-6 * r_2) - 0.00247875f);
}
inline float filterMitchell(float dx, float dy)
{
	const float x = 2.f * std::sqrt(dx * dx + dy * dy);
	if(x >= 2.f) return 0.f;
	if(x >= 1.f) return x * (x * (x * -0.38888889f + 2.0f) - 3.33333333f) + 1.77777778f;
	return x * x * (1.16666666f * x - 2.0f) + 0.88888889f;
}
inline float filterLanczos(float dx, float dy)
{
	const float x = std::sqrt(dx * dx + dy * dy);
	if(x == 0.f) return 1.f;
	if(-2 < x && x < 2)
	{
		const float a = static_cast<float>(num_pi * x);
		const float b = static_cast<float>(div_pi_by_2 * x);
		return (sinf_fast(a) * sinf_fast(b)) / (a * b);
	}
	return 0.f;
}

// include/color/color.h:338-343 (sRGB -> linear, FAST_MATH pow)
inline float linearFromSrgb(float v)
{
	if(v <= 0.04045f) return v / 12.92f;
	return powf_fast(((v + 0.055f) / 1.055f), 2.4f);
}

} // namespace hm
} // namespace yafamd
