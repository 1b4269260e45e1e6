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
//   include/color/color.h          Rgb::clampProportionalRgb, colour-space conversions, HSV
//   include/image/image_buffers.h  the image buffer pixel types (texture storage quantisation)
//   include/math/interpolation.h   cubicInterpolate (bicubic texture lookups)
//   src/geometry/vector.cc         Vec3::shirleyDisk (depth-of-field lens samples)
//   src/render/imagesplitter.cc    ImageSplitter tile lists (linear / centre / random orders)
//   src/color/color.cc             Rgbe (the HDR texture pixels; decoding is inline in color.h)
//
// oracle/Makefile compiles this file together with the .cc files above, straight from
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
#include "image/image_buffers.h"
#include "math/interpolation.h"
#include "render/imagesplitter.h"
#include "render/render_data.h"

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


// ---- texturing building blocks (image_buffers.h, color.h, interpolation.h) ----
}
template<class T> static Rgba roundTrip(const Rgba &c) { T px; px.setColor(c); return px.getColor(); }
extern "C" {

// kind: 0 Rgba1010108, 1 Rgb101010, 2 Rgba7773, 3 Rgb565, 4 Gray8, 5 Gray, 6 GrayAlpha, 7 RgbAlpha
void ref_tex_quantize(int kind, const float *in, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const Rgba c{in[4 * i], in[4 * i + 1], in[4 * i + 2], in[4 * i + 3]};
		Rgba r;
		switch(kind)
		{
			case 0: r = roundTrip<Rgba1010108>(c); break;
			case 1: r = roundTrip<Rgb101010>(c); break;
			case 2: r = roundTrip<Rgba7773>(c); break;
			case 3: r = roundTrip<Rgb565>(c); break;
			case 4: r = roundTrip<Gray8>(c); break;
			case 5: r = roundTrip<Gray>(c); break;
			case 6: r = roundTrip<GrayAlpha>(c); break;
			default: r = roundTrip<RgbAlpha>(c); break;
		}
		out[4 * i] = r.r_; out[4 * i + 1] = r.g_; out[4 * i + 2] = r.b_; out[4 * i + 3] = r.a_;
	}
}

// dir 0: linearRgbFromColorSpace, 1: colorSpaceFromLinearRgb (rgb in/out, 3 floats)
void ref_color_space(int dir, int cs, float gamma, const float *in, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		Rgb c{in[3 * i], in[3 * i + 1], in[3 * i + 2]};
		if(dir == 0) c.linearRgbFromColorSpace((ColorSpace)cs, gamma);
		else c.colorSpaceFromLinearRgb((ColorSpace)cs, gamma);
		out[3 * i] = c.r_; out[3 * i + 1] = c.g_; out[3 * i + 2] = c.b_;
	}
}

// rgbToHsv, s *= sat, h += hue (wrapped as texture.cc:230-240), hsvToRgb; sat_hue: 2 floats
void ref_hsv_adjust(const float *in, const float *sat_hue, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		Rgb c{in[3 * i], in[3 * i + 1], in[3 * i + 2]};
		float h = 0.f, s = 0.f, v = 0.f;
		c.rgbToHsv(h, s, v);
		s *= sat_hue[2 * i];
		h += sat_hue[2 * i + 1];
		if(h < 0.f) h += 6.f;
		else if(h > 6.f) h -= 6.f;
		c.hsvToRgb(h, s, v);
		out[3 * i] = c.r_; out[3 * i + 1] = c.g_; out[3 * i + 2] = c.b_;
	}
}

// cubicInterpolate over Rgba: in = 4 colours (16 floats) + x per element
void ref_cubic(const float *in, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const float *p = in + 17 * i;
		const Rgba y0{p[0], p[1], p[2], p[3]}, y1{p[4], p[5], p[6], p[7]}, y2{p[8], p[9], p[10], p[11]}, y3{p[12], p[13], p[14], p[15]};
		const Rgba r = math::cubicInterpolate(y0, y1, y2, y3, p[16]);
		out[4 * i] = r.r_; out[4 * i + 1] = r.g_; out[4 * i + 2] = r.b_; out[4 * i + 3] = r.a_;
	}
}

void ref_pow(const float *ab, float *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = math::pow(ab[2 * i], ab[2 * i + 1]);
}

}

extern "C" {

// Vec3::shirleyDisk (vector.cc:127-160): (r1, r2) -> (u, v)
void ref_shirley_disk(const float *r12, float *uv, int n)
{
	for(int i = 0; i < n; ++i) Vec3::shirleyDisk(r12[2 * i], r12[2 * i + 1], uv[2 * i], uv[2 * i + 1]);
}

// Rgbe -> Rgb (color.h:204-213): RGBE bytes -> linear RGB
void ref_rgbe_decode(const uint8_t *rgbe, float *rgb, int n)
{
	for(int i = 0; i < n; ++i)
	{
		Rgbe p;
		for(int k = 0; k < 4; ++k) p.rgbe_[k] = rgbe[4 * i + k];
		const Rgb c = static_cast<Rgb>(p);
		rgb[3 * i] = c.r_;
		rgb[3 * i + 1] = c.g_;
		rgb[3 * i + 2] = c.b_;
	}
}

// ImageSplitter (imagesplitter.cc:30-107): the region list of an image, order 0 linear, 1 random,
// 2 centre (TilesOrderType), for `nthreads` render threads; out = (x, y, w, h) per region, returns
// the region count (<= cap)
int ref_tiles(int w, int h, int bs, int order, int nthreads, int *out, int cap)
{
	const ImageSplitter::TilesOrderType t = order == 0 ? ImageSplitter::Linear : order == 1 ? ImageSplitter::Random : ImageSplitter::CentreRandom;
	ImageSplitter sp(w, h, 0, 0, bs, t, nthreads);
	int n = 0;
	RenderArea a;
	while(n < cap && sp.getArea(n, a))
	{
		out[4 * n] = a.x_;
		out[4 * n + 1] = a.y_;
		out[4 * n + 2] = a.w_;
		out[4 * n + 3] = a.h_;
		++n;
	}
	return n;
}

}
