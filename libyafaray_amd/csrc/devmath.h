// Device numerics of the hot path: libYafaRay's float expressions restated for gfx950 so that
// every sample reproduces the reference CPU build bit for bit.
//
// Three hazards from SURVEY.md Appendix A are handled here:
//  * no FMA contraction: the whole library is compiled with -ffp-contract=off, and every
//    expression below keeps the reference's left-to-right evaluation order;
//  * x87 promotions: the reference multiplies floats by `long double` constants
//    (include/math/math.h:46-65), so on x86-64 the product is rounded to a 64-bit significand and
//    then to float.  gfx950 has no 80-bit type, so x87mul*() reproduce that double rounding
//    exactly from an exact double-double product (two-product via fma + exact error terms);
//  * FAST_TRIG parabolic sin/cos (math.h:218-250) and the Faure-scrambled Halton sequences
//    (src/sampler/halton.cc:421-441) in double precision, which is IEEE on gfx950.
//
// The header is also compiled for the host (tests/test_devmath.py builds a tiny g++ harness
// that checks x87mul*() against real long double on millions of inputs).
#pragma once

#include <cstdint>
#include <cmath>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define YD __host__ __device__ __forceinline__
#ifdef YAF_INLINE_COLD
#define YD_COLD YD
#else
#define YD_COLD inline __host__ __device__ __attribute__((noinline, cold))
#endif
#else
#define YD inline
#define YD_COLD inline __attribute__((noinline, cold))
#endif

namespace yafamd
{

// ---------------------------------------------------------------------------------------------
// long double constants as exact (hi, lo) double pairs: hi = (double)C, lo = (double)(C - hi).
// Values from include/math/math.h:46-88 (verified exact by tests/test_devmath.py).
// ---------------------------------------------------------------------------------------------
struct X87Const { double hi, lo; };
constexpr X87Const kPi = {0x1.921fb54442d18p+1, 0x1.1a8p-53};
constexpr X87Const kDivPiBy2 = {0x1.921fb54442d18p+0, 0x1.1a8p-54};
constexpr X87Const kDivPiBy4 = {0x1.921fb54442d18p-1, 0x1.1a8p-55};
constexpr X87Const kDiv1ByPi = {0x1.45f306dc9c883p-2, -0x1.6bp-56};
constexpr X87Const kMultPiBy2 = {0x1.921fb54442d18p+2, 0x1.1a8p-52};
constexpr X87Const kDiv1By2Pi = {0x1.45f306dc9c883p-3, -0x1.6bp-57};
constexpr X87Const kDiv4ByPi = {0x1.45f306dc9c883p+0, -0x1.6bp-54};
constexpr X87Const kDiv4BySquaredPi = {0x1.9f02f6222c72p-2, -0x1.248p-56};
// (float) casts of the same constants, as the reference writes static_cast<float>(math::...)
constexpr float kPiF = 0x1.921fb6p+1f;
constexpr float kDivPiBy2F = 0x1.921fb6p+0f;
constexpr float kMultPiBy2F = 0x1.921fb6p+2f;
constexpr float kDiv1By2PiF = 0x1.45f306p-3f;
constexpr double kSampleMultRatio = 0x1p-32;            // math.h:88 (exact power of two)
constexpr float kMinRaydistGlobal = 0.00005f;           // include/common/yafaray_common.h:28

// ---------------------------------------------------------------------------------------------
// exact x87 double rounding emulation
// ---------------------------------------------------------------------------------------------
struct DD { double hi, lo; };

YD DD fastTwoSum(double a, double b)
{
	const double s = a + b;
	return {s, b - (s - a)};
}

// ilogb for finite non-zero doubles via the exponent bits (normal range only)
YD int expOf(double x)
{
	uint64_t u;
	__builtin_memcpy(&u, &x, 8);
	return (int)((u >> 52) & 0x7ff) - 1023;
}

YD bool isPow2(double x)
{
	uint64_t u;
	__builtin_memcpy(&u, &x, 8);
	return (u & 0xfffffffffffffull) == 0;
}

// Round |v| (non-negative, normalized |lo| <= ulp(hi)/2 + small) to a 64-bit significand, RNE.
// Result exact as (hi, r*q64).
YD DD round64(DD v)
{
	const int eh = expOf(v.hi);
	const int ev = (isPow2(v.hi) && v.lo < 0.0) ? eh - 1 : eh;
	const double q64 = ldexp(1.0, ev - 63);
	const double r = rint(v.lo / q64);   // parity of the full significand == parity of r
	return {v.hi, r * q64};
}

// Round a non-negative exact value (hi, lo) to float, RNE (normal float range).
YD float round24(DD v)
{
	if(v.hi == 0.0) return (float)v.lo;
	const int eh = expOf(v.hi);
	const int e2 = (isPow2(v.hi) && v.lo < 0.0) ? eh - 1 : eh;
	const double qf = ldexp(1.0, e2 - 23);
	const double t = v.hi / qf;
	const double I = floor(t);
	const double f = t - I;
	const double d = v.lo / qf;
	double k = I;
	if(f > 0.5) k = I + 1.0;
	else if(f == 0.5)
	{
		if(d > 0.0) k = I + 1.0;
		else if(d == 0.0) k = (fmod(I, 2.0) != 0.0) ? I + 1.0 : I;
	}
	else if(f == 0.0 && d < 0.0 && e2 == eh)
	{
		// value slightly below an integer multiple: RNE keeps I (|d| < 1/2)
		k = I;
	}
	return (float)(k * qf);
}

// exact product C * x (C a long double constant, x a float) as a normalized DD
YD DD exactMul(const X87Const &c, double xd)
{
	const double p = c.hi * xd;
	const double e = fma(c.hi, xd, -p);
	const double q = c.lo * xd;
	return fastTwoSum(p, e + q);
}

// Fast path of the emulation: a double-precision approximation D of the exact value E is within
// 2^-50 |E| of it.  When D is farther than 1e-6 float-ulp from every float rounding midpoint, E
// and its x87 64-bit rounding lie on the same side of that midpoint as D, so (float)D is the
// reference's result; only the ~1e-6 of cases near a midpoint take the exact path.
YD bool safeToRound(double d, float &f)
{
	f = (float)d;
	uint32_t b;
	__builtin_memcpy(&b, &f, 4);
	const int ef = (int)((b >> 23) & 0xffu);
	if(ef == 0 || ef >= 254) return false;      // zero / subnormal / huge: take the exact path
	const double df = (double)f;
	// |d - df| in units of the float ulp 2^(ef - 150): an exact power-of-two scaling (no double division)
	const double t = ldexp(fabs(d - df), 150 - ef);   // in [0, 0.5]
	const bool low_binade = ((b & 0x7fffffu) == 0) && (fabs(d) < fabs(df));
	return (low_binade ? 0.25 : 0.5) - t > 1e-6;
}

// Exact (slow) paths, taken only within 1e-6 float-ulp of a rounding midpoint: kept out of line so
// their code and registers do not weigh on the callers.
YD_COLD float x87mulExact(double chi, double clo, float x)
{
	const X87Const c = {chi, clo};
	const double ax = fabs((double)x);
	const float r = round24(round64(exactMul(c, ax)));
	return x < 0.f ? -r : r;
}

YD_COLD float x87mul2Exact(double chi, double clo, float x, float y)
{
	const X87Const c = {chi, clo};
	const double ax = fabs((double)x), ay = fabs((double)y);
	const DD t = round64(exactMul(c, ax));
	const double p = t.hi * ay;
	const double e = fma(t.hi, ay, -p);
	const double q = t.lo * ay;
	const float r = round24(round64(fastTwoSum(p, e + q)));
	return ((x < 0.f) != (y < 0.f)) ? -r : r;
}

YD_COLD float x87mulDivExact(double chi, double clo, float a, float b)
{
	const X87Const c = {chi, clo};
	const DD n = round64(exactMul(c, (double)a));
	const double bd = (double)b;
	const double q1 = n.hi / bd;
	const double r1 = fma(-q1, bd, n.hi);
	const double q2 = (r1 + n.lo) / bd;
	return round24(round64(fastTwoSum(q1, q2)));
}

// (float)(1.0L / ((long double)C * a)) with a > 0 (photon density scale,
// integrator_photon_mapping.cc:963: 1.f / ((float)paths * radius * num_pi)): the product is
// rounded to 64 bits, the quotient formed to ~104 bits, then rounded to 64 bits and to float.
YD_COLD float x87recipMulExact(double chi, double clo, float a)
{
	const X87Const c = {chi, clo};
	const DD t = round64(exactMul(c, (double)a));
	const double q1 = 1.0 / t.hi;
	const double r1 = fma(-q1, t.hi, 1.0) - q1 * t.lo;   // 1 - q1 * (t.hi + t.lo), exact to ~2^-104
	const double q2 = r1 / t.hi;
	return round24(round64(fastTwoSum(q1, q2)));
}

YD float x87recipMul(const X87Const &c, float a)
{
	float f;
	if(safeToRound(1.0 / (c.hi * (double)a), f)) return f;
	return x87recipMulExact(c.hi, c.lo, a);
}

// (float)((long double)C * x)
YD float x87mul(const X87Const &c, float x)
{
	if(x == 0.f || !(fabsf(x) < 3.0e38f)) return (float)(c.hi * (double)x);
	float f;
	if(safeToRound(c.hi * (double)x, f)) return f;
	return x87mulExact(c.hi, c.lo, x);
}

// (float)((long double)C * x * y) — two x87 roundings then the float one
YD float x87mul2(const X87Const &c, float x, float y)
{
	if(x == 0.f || y == 0.f) return (float)(c.hi * (double)x * (double)y);
	float f;
	if(safeToRound(c.hi * (double)x * (double)y, f)) return f;
	return x87mul2Exact(c.hi, c.lo, x, y);
}

YD_COLD float x87mul3Exact(double chi, double clo, float x, float y, float z)
{
	const X87Const c = {chi, clo};
	DD t = round64(exactMul(c, (double)x));
	const double f2[2] = {(double)y, (double)z};
	for(int k = 0; k < 2; ++k)
	{
		const double p = t.hi * f2[k];
		const double e = fma(t.hi, f2[k], -p);
		const double q = t.lo * f2[k];
		t = round64(fastTwoSum(p, e + q));
	}
	return round24(t);
}

// (float)((long double)C * x * y * z) for x, y, z >= 0: three x87 roundings then the float one
// (the photon kernel 3 ir / pi (1 - d^2 ir)^2, sample.h:31-35)
YD float x87mul3(const X87Const &c, float x, float y, float z)
{
	if(x == 0.f || y == 0.f || z == 0.f) return 0.f;
	float f;
	if(safeToRound(c.hi * (double)x * (double)y * (double)z, f)) return f;
	return x87mul3Exact(c.hi, c.lo, x, y, z);
}

// (float)(((long double)C * a) / (long double)b) with a, b > 0 floats (light pdfs,
// src/light/light_area.cc:88).  The quotient is formed to ~104 bits (double-double) before the
// two roundings.
YD float x87mulDiv(const X87Const &c, float a, float b)
{
	if(a == 0.f) return 0.f;
	float f;
	if(safeToRound(c.hi * (double)a / (double)b, f)) return f;
	return x87mulDivExact(c.hi, c.lo, a, b);
}

// (float)(1.f - 2.f * ((long double)x * C)) for x >= 0 (TextureMapperNode::sphereMap's v coordinate,
// shader_node_basic.cc:78: the acos times div_1_by_pi is rounded to 64 bits, doubled (exact), subtracted
// from one and rounded to 64 bits, then to float).  Textured scenes only: always the exact path.
YD_COLD float x87oneMinus2Mul(const X87Const &c, float x)
{
	if(x == 0.f) return 1.f;
	const DD t = round64(exactMul(c, (double)x));
	// 1 - 2 t as an exact double-double: two-sum of 1 and -2 t.hi, then the -2 t.lo tail
	const double b = -2.0 * t.hi;
	const double s = 1.0 + b;
	const double bb = s - 1.0;
	const double err = (1.0 - (s - bb)) + (b - bb);
	DD v = fastTwoSum(s, err - 2.0 * t.lo);
	if(v.hi == 0.0) return (float)v.lo;
	const bool neg = v.hi < 0.0;
	if(neg) v = DD{-v.hi, -v.lo};
	const float r = round24(round64(v));
	return neg ? -r : r;
}

// ---------------------------------------------------------------------------------------------
// libm's float atan2f / atanf / acosf as the reference's x86-64 build calls them (std::atan2 /
// std::acos on floats, shader_node_basic.cc:67, 77-78 via math.h:252-258).  glibc 2.35 implements them
// as the fdlibm float algorithms (sysdeps/ieee754/flt-32 e_atan2f.c, s_atanf.c, e_acosf.c — not
// correctly rounded: 15 % of atan2f and 8 % of acosf results differ from the double-rounded value), so
// the device restates those algorithms operation for operation; tests/test_devmath.py checks this host
// build against the host's libm bit for bit on millions of inputs.
// ---------------------------------------------------------------------------------------------
YD uint32_t fbits(float f)
{
	uint32_t u;
	__builtin_memcpy(&u, &f, 4);
	return u;
}
YD float bitsf(uint32_t u)
{
	float f;
	__builtin_memcpy(&f, &u, 4);
	return f;
}

YD float libmAtanf(float x)
{
	// atan(0.5), atan(1), atan(1.5), atan(inf) split in (hi, lo); the odd / even polynomial of atan
	constexpr float hi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
	constexpr float lo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
	constexpr float a0 = 3.3333334327e-01f, a1 = -2.0000000298e-01f, a2 = 1.4285714924e-01f, a3 = -1.1111110449e-01f,
	                a4 = 9.0908870101e-02f, a5 = -7.6918758452e-02f, a6 = 6.6610731184e-02f, a7 = -5.8335702866e-02f,
	                a8 = 4.9768779427e-02f, a9 = -3.6531571299e-02f, a10 = 1.6285819933e-02f;
	const int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
	int id;
	if(ix >= 0x4c000000)   // |x| >= 2^25
	{
		if(ix > 0x7f800000) return x + x;
		return hx > 0 ? hi[3] + lo[3] : -hi[3] - lo[3];
	}
	if(ix < 0x3ee00000)    // |x| < 0.4375
	{
		if(ix < 0x31000000) return x;
		id = -1;
	}
	else
	{
		x = fabsf(x);
		if(ix < 0x3f980000)
		{
			if(ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
			else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
		}
		else if(ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
		else { id = 3; x = -1.0f / x; }
	}
	const float z = x * x, w = z * z;
	const float s1 = z * (a0 + w * (a2 + w * (a4 + w * (a6 + w * (a8 + w * a10)))));
	const float s2 = w * (a1 + w * (a3 + w * (a5 + w * (a7 + w * a9))));
	if(id < 0) return x - x * (s1 + s2);
	const float r = hi[id] - ((x * (s1 + s2) - lo[id]) - x);
	return hx < 0 ? -r : r;
}

YD float libmAtan2f(float y, float x)
{
	constexpr float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
	                pi_lo = -8.7422776573e-08f;
	const int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff, hy = (int32_t)fbits(y), iy = hy & 0x7fffffff;
	if(ix > 0x7f800000 || iy > 0x7f800000) return x + y;
	if(hx == 0x3f800000) return libmAtanf(y);
	const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
	if(iy == 0) return m <= 1 ? y : (m == 2 ? pi + tiny : -pi - tiny);
	if(ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
	if(ix == 0x7f800000)
	{
		if(iy == 0x7f800000)
			return m == 0 ? pi_o_4 + tiny : m == 1 ? -pi_o_4 - tiny : m == 2 ? 3.0f * pi_o_4 + tiny : -3.0f * pi_o_4 - tiny;
		return m == 0 ? 0.0f : m == 1 ? -0.0f : m == 2 ? pi + tiny : -pi - tiny;
	}
	if(iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
	const int k = (iy - ix) >> 23;
	float z;
	if(k > 60) z = pi_o_2 + 0.5f * pi_lo;
	else if(hx < 0 && k < -60) z = 0.0f;
	else z = libmAtanf(fabsf(y / x));
	switch(m)
	{
		case 0: return z;
		case 1: return bitsf(fbits(z) ^ 0x80000000u);
		case 2: return pi - (z - pi_lo);
		default: return (z - pi_lo) - pi;
	}
}

YD float libmAcosf(float x)
{
	constexpr float pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
	constexpr float pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f, pS3 = -4.0055535734e-02f,
	                pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f, qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f,
	                qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
	const int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
	if(ix == 0x3f800000) return hx > 0 ? 0.0f : pi + 2.0f * pio2_lo;
	if(ix > 0x3f800000) return (x - x) / (x - x);
	if(ix < 0x3f000000)   // |x| < 0.5
	{
		if(ix <= 0x23000000) return pio2_hi + pio2_lo;
		const float z = x * x;
		const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
		const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
		const float r = p / q;
		return pio2_hi - (x - (pio2_lo - x * r));
	}
	if(hx < 0)            // x < -0.5
	{
		const float z = (1.0f + x) * 0.5f;
		const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
		const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
		const float s = sqrtf(z);
		const float r = p / q;
		const float w = r * s - pio2_lo;
		return pi - 2.0f * (s + w);
	}
	const float z = (1.0f - x) * 0.5f;   // x > 0.5
	const float s = sqrtf(z);
	const float df = bitsf(fbits(s) & 0xfffff000u);
	const float c = (z - df * df) / (s + df);
	const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
	const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
	const float r = p / q;
	const float w = r * s + c;
	return 2.0f * (df + w);
}

// x > C / x < -C with C long double (exact for float x, see DESIGN.md numerics note)
YD bool gtC(float x, const X87Const &c) { return (double)x > c.hi || ((double)x == c.hi && c.lo < 0.0); }
YD bool ltNegC(float x, const X87Const &c) { return (double)x < -c.hi || ((double)x == -c.hi && c.lo < 0.0); }

// ---------------------------------------------------------------------------------------------
// math.h FAST_TRIG sin / cos
// ---------------------------------------------------------------------------------------------
YD float fsin(float x)
{
	if(gtC(x, kMultPiBy2) || ltNegC(x, kMultPiBy2)) x -= ((int)(x * kDiv1By2PiF)) * kMultPiBy2F;
	if(ltNegC(x, kPi)) x += kMultPiBy2F;
	else if(gtC(x, kPi)) x -= kMultPiBy2F;
	x = x87mul(kDiv4ByPi, x) - x87mul2(kDiv4BySquaredPi, x, fabsf(x));
	const float result = 0.225f * (x * fabsf(x) - x) + x;
	if(result <= -1.f) return -1.f;
	else if(result >= 1.f) return 1.f;
	return result;
}

YD float fcos(float x) { return fsin(x + kDivPiBy2F); }

// ---------------------------------------------------------------------------------------------
// vectors / colours with the reference's operation order (include/geometry/vector.h:108-276,
// include/color/color.h:258-296)
// ---------------------------------------------------------------------------------------------
struct V3 { float x, y, z; };
YD V3 v3(float a, float b, float c) { return {a, b, c}; }
YD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
YD V3 operator*(float f, V3 v) { return {f * v.x, f * v.y, f * v.z}; }
YD V3 operator*(V3 v, float f) { return {f * v.x, f * v.y, f * v.z}; }
YD V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
YD V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
YD V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
YD V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
YD float lengthSqr(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
YD float length(V3 a) { return sqrtf(lengthSqr(a)); }
YD V3 normalize(V3 v)
{
	float len = lengthSqr(v);
	if(len != 0.f)
	{
		len = 1.f / sqrtf(len);
		v.x *= len; v.y *= len; v.z *= len;
	}
	return v;
}
YD void coordsSystem(V3 n, V3 &u, V3 &v)
{
	if((n.x == 0.f) && (n.y == 0.f))
	{
		u = (n.z < 0.f) ? v3(-1.f, 0.f, 0.f) : v3(1.f, 0.f, 0.f);
		v = v3(0.f, 1.f, 0.f);
	}
	else
	{
		const float d = 1.f / sqrtf(n.y * n.y + n.x * n.x);
		u = v3(n.y * d, -n.x * d, 0.f);
		v = cross(n, u);
	}
}

struct C3 { float r, g, b; };
YD C3 c3(float f) { return {f, f, f}; }
YD C3 operator*(C3 a, C3 b) { return {a.r * b.r, a.g * b.g, a.b * b.b}; }
YD C3 operator*(float f, C3 c) { return {f * c.r, f * c.g, f * c.b}; }
YD C3 operator*(C3 c, float f) { return {f * c.r, f * c.g, f * c.b}; }
YD C3 operator/(C3 c, float f) { return {c.r / f, c.g / f, c.b / f}; }
YD C3 operator+(C3 a, C3 b) { return {a.r + b.r, a.g + b.g, a.b + b.b}; }
YD bool isBlack(C3 c) { return c.r == 0 && c.g == 0 && c.b == 0; }
YD float maxComp(C3 c) { return fmaxf(c.r, fmaxf(c.g, c.b)); }

// ---------------------------------------------------------------------------------------------
// samplers: include/sampler/sample.h:45-151, include/sampler/halton.h:41-81, halton.cc:421-441,
// include/math/random.h:56-104
// ---------------------------------------------------------------------------------------------
YD float clamp01(float v) { return fmaxf(0.f, fminf(1.f, v)); }

// Halton(base) of the camera lens (halton.h:47-81): setStart(start), then k getNext() calls; the
// value after the k-th call (incremental radical inverse in double, as the reference)
YD float haltonNext(uint32_t base, uint32_t start, int k)
{
	const double inv_base = 1.0 / static_cast<double>(base);
	double factor = inv_base, value = 0.0;
	while(start > 0)
	{
		value += static_cast<double>(start % base) * factor;
		start /= base;
		factor *= inv_base;
	}
	for(int i = 0; i < k; ++i)
	{
		const double r = 0.9999999999 - value;
		if(inv_base < r) value += inv_base;
		else
		{
			double hh = 0.0, h = inv_base;
			while(h >= r)
			{
				hh = h;
				h *= inv_base;
			}
			value += hh + h - 1.0;
		}
	}
	return clamp01(static_cast<float>(value));
}

YD uint32_t bitReverse32(uint32_t v)
{
#if defined(__HIP_DEVICE_COMPILE__)
	return __builtin_bitreverse32(v);
#else
	v = (v << 16) | (v >> 16);
	v = ((v & 0x00ff00ffu) << 8) | ((v & 0xff00ff00u) >> 8);
	v = ((v & 0x0f0f0f0fu) << 4) | ((v & 0xf0f0f0f0u) >> 4);
	v = ((v & 0x33333333u) << 2) | ((v & 0xccccccccu) >> 2);
	return ((v & 0x55555555u) << 1) | ((v & 0xaaaaaaaau) >> 1);
#endif
}

YD float riVdC(uint32_t bits, uint32_t r = 0)
{
	bits = (bits << 16) | (bits >> 16);
	bits = ((bits & 0x00ff00ffu) << 8) | ((bits & 0xff00ff00u) >> 8);
	bits = ((bits & 0x0f0f0f0fu) << 4) | ((bits & 0xf0f0f0f0u) >> 4);
	bits = ((bits & 0x33333333u) << 2) | ((bits & 0xccccccccu) >> 2);
	bits = ((bits & 0x55555555u) << 1) | ((bits & 0xaaaaaaaau) >> 1);
	return clamp01((float)((double)(bits ^ r) * kSampleMultRatio));
}

YD float riS(uint32_t i, uint32_t r = 0)
{
	for(uint32_t v = 1u << 31; i; i >>= 1, v ^= v >> 1)
		if(i & 1) r ^= v;
	return clamp01((float)((double)r * kSampleMultRatio));
}

// Larcher-Pillichshammer: bit k of i toggles bits [31-k, 31] of r, so bit (31-t) of r is the
// parity of i >> t — a suffix-XOR scan plus a bit reversal instead of the 32-step loop.
YD float riLp(uint32_t i, uint32_t r = 0)
{
	uint32_t y = i;
	y ^= y >> 1;
	y ^= y >> 2;
	y ^= y >> 4;
	y ^= y >> 8;
	y ^= y >> 16;
	r ^= bitReverse32(y);
	return clamp01((float)((double)r * kSampleMultRatio));
}

YD uint32_t fnv32(uint32_t value)
{
	uint32_t hash = 0x811c9dc5u;
	for(int k = 0; k < 4; ++k)
	{
		hash ^= (value >> (8 * k)) & 0xffu;
		hash *= 0x01000193u;
	}
	return hash;
}

// The digit weights of halton.h:53-63's loop (factor = 1/B, then factor *= 1/B per digit) as
// compile-time constants: the same sequence of double roundings, evaluated by the compiler
template<uint32_t B>
struct HaltonFactors
{
	static constexpr int n = 34;
	static constexpr int digits = B == 3 ? 21 : B == 5 ? 14 : 32;   // base-B digits of a 32-bit start
	double f[n];
	constexpr HaltonFactors() : f()
	{
		const double inv = 1.0 / static_cast<double>(B);
		double x = inv;
		for(int k = 0; k < n; ++k)
		{
			f[k] = x;
			x *= inv;
		}
	}
};

// Halton(base, start) as a running generator (halton.h:41-81: setStart, then getNext per draw) —
// for loops that draw consecutive numbers of one sequence (area-light samples, AO samples)
template<uint32_t B>
struct HaltonInc
{
	double value;
	static constexpr double inv_base = 1.0 / static_cast<double>(B);
	YD void start(uint32_t s)
	{
		if(B == 2)
		{
			// distinct powers of two: the digit sum is exactly bitreverse(s) * 2^-32
			value = static_cast<double>(bitReverse32(s)) * 2.3283064365386962890625e-10;
			return;
		}
		// the digit loop unrolled over the constant weights (no running factor product) and run for
		// every digit position a 32-bit start can have: past the last digit the terms are +0, which
		// leaves the (non-negative) sum unchanged, so the value is the loop's bit for bit
		constexpr HaltonFactors<B> F;
		constexpr int nd = HaltonFactors<B>::digits;
		value = 0.0;
#pragma unroll
		for(int k = 0; k < nd; ++k)
		{
			value += static_cast<double>(s % B) * F.f[k];
			s /= B;
		}
	}
	YD float next()
	{
		const double r = 0.9999999999 - value;
		if(inv_base < r) value += inv_base;
		else
		{
			double hh = 0.0, h = inv_base;
			while(h >= r)
			{
				hh = h;
				h *= inv_base;
			}
			value += hh + h - 1.0;
		}
		return clamp01(static_cast<float>(value));
	}
};

// Halton(base, start).getNext() — one fresh generator per call site (integrator_montecarlo.cc:399)
YD float haltonFirst(uint32_t base, double inv_base, uint32_t start)
{
	double value = 0.0;
	if(base == 2)
	{
		// halton.h:53-63 in base 2 sums distinct powers of two: exactly bitreverse(start) * 2^-32
		value = (double)bitReverse32(start) * kSampleMultRatio;
	}
	else
	{
		double factor = inv_base;
		while(start > 0)
		{
			value += (double)(start % base) * factor;
			start /= base;
			factor *= inv_base;
		}
	}
	const double r = 0.9999999999 - value;
	if(inv_base < r) value += inv_base;
	else
	{
		double hh = 0.0, h = inv_base;
		while(h >= r)
		{
			hh = h;
			h *= inv_base;
		}
		value += hh + h - 1.0;
	}
	return clamp01((float)value);
}

// Exact unsigned division by a divisor d in [2, 2^31] known only at run time, from a
// precomputed magic number (Granlund–Montgomery "round-up" form): q = (t + ((n - t) >> 1)) >> sh
// with t = mulhi(n, m).  Replaces the ~20-instruction generic u32 division in the digit loops.
struct UDiv { uint32_t m, sh; };
YD UDiv udivMake(uint32_t d)
{
	uint32_t l = 0;
	while((1ull << l) < (uint64_t)d) ++l;                       // ceil(log2 d)
	UDiv q;
	q.m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
	q.sh = l - 1;
	return q;
}
YD uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
YD uint32_t udiv(uint32_t n, UDiv q)
{
	const uint32_t t = mulhi32(n, q.m);
	return (t + ((n - t) >> 1)) >> q.sh;
}

// Faure-scrambled radical inverse (halton.cc:421-441).  `perm` points at the digit permutation
// of the dimension, `base` its prime, `dv` the magic of `base`, `f` the reference's inv_prims
// entry (llround(1e9 / p) / 1e9, NOT 1/p: the digit sequence comes from truncating dn * f, exactly
// as the reference does).
YD double lowDiscrepancy(const uint8_t *perm, uint32_t base, UDiv dv, double f, uint32_t n)
{
	double value = 0.0, dn = (double)n, factor = f;
	while(n > 0)
	{
		const uint32_t digit = n - udiv(n, dv) * base;   // n % base
		value += (double)perm[digit] * factor;
		dn *= f;
		n = (uint32_t)dn;
		factor *= f;
	}
	return value;
}

struct Mwc
{
	uint32_t x, c;
	YD double next()
	{
		const uint32_t a = 1791398085u, ah = a >> 16, al = a & 65535u;
		const uint32_t xh = x >> 16, xl = x & 65535u;
		x = x * a + c;
		c = xh * ah + ((xh * al) >> 16) + ((xl * ah) >> 16);
		if(xl * al >= ~c + 1) c++;
		return (double)x * kSampleMultRatio;
	}
};

// sample.h:45-54
YD V3 cosHemisphere(V3 n, V3 ru, V3 rv, float s_1, float s_2)
{
	if(s_1 >= 1.0f) return n;
	const float z_1 = s_1;
	const float z_2 = x87mul(kMultPiBy2, s_2);
	const V3 a = ru * fcos(z_2);
	const V3 b = rv * fsin(z_2);
	return (a + b) * sqrtf(1.f - z_1) + n * sqrtf(z_1);
}

} // namespace yafamd
