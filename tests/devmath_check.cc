// Host-side check of libyafaray_amd/csrc/devmath.h (the exact x87 double-rounding emulation the
// GPU kernels use) against real x86 long double arithmetic — the semantics of the reference
// expressions (include/math/math.h:218-250, include/sampler/sample.h:45-54,
// src/light/light_area.cc:88, :149).  Built and run by tests/test_devmath.py.
#include "../libyafaray_amd/csrc/devmath.h"
#include <cstdio>
#include <cstring>
#include <random>

using namespace yafamd;
using LD = long double;

static const LD pi = 3.1415926535897932384626433832795L;
static const LD div_1_by_pi = 0.31830988618379067153776752674503L;
static const LD mult_pi_by_2 = 6.283185307179586476925286766559L;
static const LD div_1_by_2pi = 0.15915494309189533576888376337251L;
static const LD div_4_by_pi = 1.2732395447351626861510701069801L;
static const LD div_4_by_squared_pi = 0.40528473456935108577551785283891L;
static const LD div_pi_by_2 = 1.5707963267948966192313216916398L;

static float refSin(float x)
{
	if(x > mult_pi_by_2 || x < -mult_pi_by_2) x -= ((int)(x * static_cast<float>(div_1_by_2pi))) * static_cast<float>(mult_pi_by_2);
	if(x < -pi) x += static_cast<float>(mult_pi_by_2);
	else if(x > pi) x -= static_cast<float>(mult_pi_by_2);
	x = (static_cast<float>(div_4_by_pi * x)) - (static_cast<float>(div_4_by_squared_pi * x * std::abs(x)));
	const float result = 0.225f * (x * std::abs(x) - x) + x;
	if(result <= -1.f) return -1.f;
	else if(result >= 1.f) return 1.f;
	return result;
}

static bool same(float a, float b) { uint32_t x, y; memcpy(&x, &a, 4); memcpy(&y, &b, 4); return x == y; }

int main(int argc, char **argv)
{
	const long n = argc > 1 ? atol(argv[1]) : 2000000;
	std::mt19937_64 rng(12345);
	std::uniform_real_distribution<float> u(-30.f, 30.f), s(0.f, 1.f), pos(1e-4f, 50.f);
	long bad_mul = 0, bad_mul2 = 0, bad_div = 0, bad_sin = 0, bad_cos = 0, bad_hemi = 0;
	// the constants themselves
	const X87Const cs[] = {kPi, kDivPiBy2, kDiv1ByPi, kMultPiBy2, kDiv1By2Pi, kDiv4ByPi, kDiv4BySquaredPi};
	const LD ls[] = {pi, div_pi_by_2, div_1_by_pi, mult_pi_by_2, div_1_by_2pi, div_4_by_pi, div_4_by_squared_pi};
	int bad_const = 0;
	for(int k = 0; k < 7; ++k) if((LD)cs[k].hi + (LD)cs[k].lo != ls[k]) ++bad_const;
	for(long i = 0; i < n; ++i)
	{
		float x = u(rng);
		if(i % 7 == 0) x = s(rng) * 7.f;
		if(i % 11 == 0) { uint32_t b = (uint32_t)rng(); b = (b & 0x807fffffu) | (((b >> 23) % 40 + 100) << 23); memcpy(&x, &b, 4); }
		if(!same(x87mul(kDiv4ByPi, x), (float)(div_4_by_pi * x))) ++bad_mul;
		if(!same(x87mul(kMultPiBy2, x), (float)(x * mult_pi_by_2))) ++bad_mul;
		if(!same(x87mul(kDiv1ByPi, x), (float)(x * div_1_by_pi))) ++bad_mul;
		if(!same(x87mul2(kDiv4BySquaredPi, x, std::abs(x)), (float)(div_4_by_squared_pi * x * std::abs(x)))) ++bad_mul2;
		const float a = pos(rng), b = pos(rng);
		if(!same(x87mulDiv(kPi, a, b), (float)(a * pi / b))) ++bad_div;
		{
			// integrator_photon_mapping.cc:963 — 1.f / ((float)paths * radius * num_pi)
			const float pr = (float)(1 + (rng() % 20000000)) * (a * 1e-3f);
			if(!same(x87recipMul(kPi, pr), (float)(1.f / (pr * pi)))) ++bad_div;
			// the exact (slow) paths on every input, not only near rounding midpoints
			if(!same(x87recipMulExact(kPi.hi, kPi.lo, pr), (float)(1.f / (pr * pi)))) ++bad_div;
			if(!same(x87mulDivExact(kPi.hi, kPi.lo, a, b), (float)(a * pi / b))) ++bad_div;
			if(x != 0.f && !same(x87mulExact(kDiv4ByPi.hi, kDiv4ByPi.lo, x), (float)(div_4_by_pi * x))) ++bad_mul;
			if(x != 0.f && !same(x87mul2Exact(kDiv4BySquaredPi.hi, kDiv4BySquaredPi.lo, x, std::abs(x)), (float)(div_4_by_squared_pi * x * std::abs(x)))) ++bad_mul2;
		}
		if(!same(fsin(x), refSin(x))) ++bad_sin;
		if(!same(fcos(x), refSin(x + static_cast<float>(div_pi_by_2)))) ++bad_cos;
		const float s2 = s(rng);
		if(!same(x87mul(kMultPiBy2, s2), (float)(s2 * mult_pi_by_2))) ++bad_hemi;
	}
	printf("n=%ld const=%d mul=%ld mul2=%ld div=%ld sin=%ld cos=%ld hemi=%ld\n", n, bad_const, bad_mul, bad_mul2, bad_div, bad_sin, bad_cos, bad_hemi);
	return (bad_const + bad_mul + bad_mul2 + bad_div + bad_sin + bad_cos + bad_hemi) ? 1 : 0;
}
