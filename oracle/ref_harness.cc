// TEST INFRASTRUCTURE ONLY — never linked into, loaded by or called from the product path.
//
// Thin extern "C" harness around the *reference's own* header-only / self-contained numeric
// building blocks of the hot path.  The reference library as a whole is unbuildable under this
// round's rules (logger.h -> yafaray_c_api.h -> the CMake-generated yafaray_c_api_export.h), but
// the pieces below compile from their own few source files with plain g++:
//
//   include/math/math.h            FAST_MATH/FAST_TRIG sin/cos/exp/log/pow, roundToInt, floorToInt
//   include/sampler/sample.h       riVdC / riS / riLp / fnv32ABuf / cosHemisphere / sphere
//   include/sampler/halton.h       Halton::setStart/getNext
//   src/sampler/halton.cc          Halton::lowDiscrepancySampling (Faure-scrambled radical inverse)
//   include/math/random.h          RandomGenerator (MWC)
//   src/math/random.cc             FastRandom::myseed_
//   include/geometry/vector.h      Vec3 normalize / createCoordsSystem / reflectDir
//   include/geometry/bound.h       Bound::cross (Smits slab test)
//   include/math/filter.h          box / gauss filter kernels (film table entries)
//   include/color/color.h          Rgb::clampProportionalRgb
//
// oracle/Makefile compiles this file together with the two .cc files above, straight from
// /root/reference, with the reference's Release flags (-O3 -DNDEBUG -DFAST_MATH -DFAST_TRIG,
// C++11), into oracle/_ref/libyafref_prims.so.  tests/golden/make_golden_prims.py then records
// input/output vectors from it, and the CPU oracle (oracle/yafcpu.cc) is pinned against them.

#include "common/yafaray_common.h"
#include "math/math.h"
#include "sampler/sample.h"
#include "sampler/halton.h"
#include "math/random.h"
#include "geometry/vector.h"
#include "geometry/bound.h"
#include "math/filter.h"
#include "color/color.h"

#include <cstdint>

using namespace yafaray;

extern "C" {

void ref_riVdC(const uint32_t *bits, const uint32_t *r, float *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = sample::riVdC(bits[i], r[i]);
}

void ref_riS(const uint32_t *bits, const uint32_t *r, float *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = sample::riS(bits[i], r[i]);
}

void ref_riLp(const uint32_t *bits, const uint32_t *r, float *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = sample::riLp(bits[i], r[i]);
}

void ref_fnv32(const uint32_t *in, uint32_t *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = sample::fnv32ABuf(in[i]);
}

void ref_lds(const int *dim, const uint32_t *idx, double *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = Halton::lowDiscrepancySampling(dim[i], idx[i]);
}

// Halton(base, start) followed by `steps` calls of getNext(); writes every value.
void ref_halton_seq(int base, uint32_t start, int steps, float *out)
{
	Halton h(base, start);
	for(int i = 0; i < steps; ++i) out[i] = h.getNext();
}

// One fresh Halton(base, start[i]).getNext() per element (how the integrators use it).
void ref_halton_first(int base, const uint32_t *start, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		Halton h(base, start[i]);
		out[i] = h.getNext();
	}
}

void ref_sin(const float *x, float *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = math::sin(x[i]);
}

void ref_cos(const float *x, float *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = math::cos(x[i]);
}

void ref_exp(const float *x, float *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = math::exp(x[i]);
}

void ref_sqrt(const float *x, float *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = math::sqrt(x[i]);
}

// n_ru_rv: 9 floats per element (n, ru, rv), s: 2 floats per element, out: 3 floats
void ref_cos_hemisphere(const float *n_ru_rv, const float *s, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const float *p = n_ru_rv + 9 * i;
		const Vec3 nn{p[0], p[1], p[2]}, ru{p[3], p[4], p[5]}, rv{p[6], p[7], p[8]};
		const Vec3 r = sample::cosHemisphere(nn, ru, rv, s[2 * i], s[2 * i + 1]);
		out[3 * i] = r[0]; out[3 * i + 1] = r[1]; out[3 * i + 2] = r[2];
	}
}

// in: 3 floats (a normal); out: 6 floats (nu, nv)
void ref_coords_system(const float *in, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const Vec3 nn{in[3 * i], in[3 * i + 1], in[3 * i + 2]};
		const auto uv = Vec3::createCoordsSystem(nn);
		for(int k = 0; k < 3; ++k) { out[6 * i + k] = uv.first[k]; out[6 * i + 3 + k] = uv.second[k]; }
	}
}

void ref_normalize(const float *in, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		Vec3 v{in[3 * i], in[3 * i + 1], in[3 * i + 2]};
		v.normalize();
		out[3 * i] = v[0]; out[3 * i + 1] = v[1]; out[3 * i + 2] = v[2];
	}
}

// box: 6 floats (a, g); ray: 7 floats (from, dir, tmax); out: 3 floats (crossed, enter, leave)
void ref_bound_cross(const float *box, const float *ray, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const float *b = box + 6 * i, *r = ray + 7 * i;
		const Bound bound{Point3{b[0], b[1], b[2]}, Point3{b[3], b[4], b[5]}};
		const Ray rr{Point3{r[0], r[1], r[2]}, Vec3{r[3], r[4], r[5]}};
		const Bound::Cross c = bound.cross(rr, r[6]);
		out[3 * i] = c.crossed_ ? 1.f : 0.f;
		out[3 * i + 1] = c.crossed_ ? c.enter_ : 0.f;
		out[3 * i + 2] = c.crossed_ ? c.leave_ : 0.f;
	}
}

void ref_mwc(uint32_t seed, int steps, double *out)
{
	RandomGenerator rg(seed);
	for(int i = 0; i < steps; ++i) out[i] = rg();
}

void ref_filter_gauss(const float *dxdy, float *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = math::filter::gauss(dxdy[2 * i], dxdy[2 * i + 1]);
}

void ref_round_to_int(const double *v, int *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = math::roundToInt(v[i]);
}

void ref_floor_to_int(const double *v, int *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = math::floorToInt(v[i]);
}

// rgb in/out: 3 floats per element
void ref_clamp_proportional(const float *rgb, float max_value, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		Rgb c{rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]};
		c.clampProportionalRgb(max_value);
		out[3 * i] = c.r_; out[3 * i + 1] = c.g_; out[3 * i + 2] = c.b_;
	}
}

}
