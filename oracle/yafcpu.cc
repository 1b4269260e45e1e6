// TEST INFRASTRUCTURE ONLY — CPU oracle (restatement) of libYafaRay's path-tracing hot path.
// See yafcpu.h for scope and parity status.  Every function cites the reference file:line it
// restates (paths relative to the reference repository root).  Built by oracle/Makefile with
// -ffp-contract=off so that no FMA contraction happens (the reference Release build is plain
// x86-64 SSE2, Appendix A.1 of SURVEY.md).

#include "yafcpu.h"

#include <algorithm>
#include <random>
#include <array>
#include <cstdlib>
#include <sstream>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <string>
#include <cstring>
#include <limits>
#include <memory>
#include <thread>
#include <vector>

namespace yc
{
using LD = long double;

// include/math/math.h:46-88 — x87 long double constants (the promotions matter for parity).
constexpr LD num_pi = 3.1415926535897932384626433832795L;
constexpr LD div_pi_by_2 = 1.5707963267948966192313216916398L;
constexpr LD div_1_by_pi = 0.31830988618379067153776752674503L;
constexpr LD mult_pi_by_2 = 6.283185307179586476925286766559L;
constexpr LD div_1_by_2pi = 0.15915494309189533576888376337251L;
constexpr LD div_4_by_pi = 1.2732395447351626861510701069801L;
constexpr LD div_4_by_squared_pi = 0.40528473456935108577551785283891L;
constexpr LD log2e = 1.4426950408889634073599246810019L;
constexpr LD ln2 = 0.69314718055994530941723212145818L;
constexpr LD sample_mult_ratio = 0.00000000023283064365386962890625L;
constexpr LD div_pi_by_4 = 0.78539816339744830961566084581988L;
constexpr LD div_pi_by_180 = 0.01745329251994329576923690768489L;
constexpr float min_raydist_global = 0.00005f;   // include/common/yafaray_common.h:28

// ---------------------------------------------------------------------------------------------
// math (include/math/math.h)
// ---------------------------------------------------------------------------------------------

// math.h:218-245 (FAST_TRIG parabolic sine)
static inline float fsin(float x)
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

// math.h:247-254
static inline float fcos(float x) { return fsin(x + static_cast<float>(div_pi_by_2)); }

// math.h:144-169 + 199-206: FAST_MATH sqrt is std::sqrt on x86-64.
static inline float fsqrt(float x) { return std::sqrt(x); }

union BitTw { int i; float f; };

// math.h:96-125
static inline float polyexp(float x)
{
	return x * (x * (x * (x * (x * 1.8775767e-3f + 8.9893397e-3f) + 5.5826318e-2f) + 2.4015361e-1f) + 6.9315308e-1f) + 9.9999994e-1f;
}
static inline float fexp2(float x)
{
	BitTw ip, fp, ep;
	x = std::min(x, 129.00000f);
	x = std::max(x, -126.99999f);
	ip.i = static_cast<int>(x - 0.5f);
	fp.f = (x - static_cast<float>(ip.i));
	ep.i = ((ip.i + 127) << 23);
	return ep.f * polyexp(fp.f);
}
// math.h:183-188 (FAST_MATH exp)
static inline float fexp(float a) { return fexp2(static_cast<float>(log2e * a)); }

// math.h:268-296 (FAST_INT disabled)
static inline int roundToInt(double v) { return static_cast<int>(v + (.5 - 1.4e-11)); }
static inline int floorToInt(double v) { return static_cast<int>(std::floor(v)); }

// ---------------------------------------------------------------------------------------------
// geometry (include/geometry/vector.h)
// ---------------------------------------------------------------------------------------------
struct V3
{
	float x = 0.f, y = 0.f, z = 0.f;
	V3() = default;
	V3(float a, float b, float c) : x(a), y(b), z(c) {}
	float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
	float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
	float lengthSqr() const { return x * x + y * y + z * z; }
	float length() const { return fsqrt(lengthSqr()); }
	// vector.h:201-210
	V3 &normalize()
	{
		float len = lengthSqr();
		if(len != 0.f)
		{
			len = 1.f / fsqrt(len);
			x *= len; y *= len; z *= len;
		}
		return *this;
	}
	// vector.h:234-243
	float normLen()
	{
		float vl = lengthSqr();
		if(vl != 0.f)
		{
			vl = fsqrt(vl);
			const float d = 1.f / vl;
			x *= d; y *= d; z *= d;
		}
		return vl;
	}
	V3 &operator+=(const V3 &s) { x += s.x; y += s.y; z += s.z; return *this; }
	V3 &operator*=(float s) { x *= s; y *= s; z *= s; return *this; }
};
// vector.h:108-186
static inline float dot(const V3 &a, const V3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 operator*(float f, const V3 &v) { return {f * v.x, f * v.y, f * v.z}; }
static inline V3 operator*(const V3 &v, float f) { return {f * v.x, f * v.y, f * v.z}; }
static inline V3 operator^(const V3 &a, const V3 &b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static inline V3 operator-(const V3 &a, const V3 &b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 operator+(const V3 &a, const V3 &b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 operator-(const V3 &v) { return {-v.x, -v.y, -v.z}; }

// vector.h:262-276
static inline void createCoordsSystem(const V3 &n, V3 &u, V3 &v)
{
	if((n.x == 0.f) && (n.y == 0.f))
	{
		u = (n.z < 0.f ? V3{-1.f, 0.f, 0.f} : V3{1.f, 0.f, 0.f});
		v = V3{0.f, 1.f, 0.f};
	}
	else
	{
		const float d = 1.f / fsqrt(n.y * n.y + n.x * n.x);
		u = V3{n.y * d, -n.x * d, 0.f};
		v = n ^ u;
	}
}

// ---------------------------------------------------------------------------------------------
// colour (include/color/color.h)
// ---------------------------------------------------------------------------------------------
struct C3
{
	float r = 0.f, g = 0.f, b = 0.f;
	C3() = default;
	explicit C3(float f) : r(f), g(f), b(f) {}
	C3(float a, float bb, float c) : r(a), g(bb), b(c) {}
	bool isBlack() const { return r == 0 && g == 0 && b == 0; }
	float maximum() const { return std::max(r, std::max(g, b)); }
	C3 &operator+=(const C3 &c) { r += c.r; g += c.g; b += c.b; return *this; }
	C3 &operator*=(const C3 &c) { r *= c.r; g *= c.g; b *= c.b; return *this; }
	C3 &operator*=(float f) { r *= f; g *= f; b *= f; return *this; }
	// color.h:415-440
	void clampProportional(float max_value)
	{
		if(max_value > 0.f)
		{
			const float max_rgb = std::max(r, std::max(g, b));
			const float adj = max_value / max_rgb;
			if(max_rgb > max_value)
			{
				if(r >= max_rgb) { r = max_value; g *= adj; b *= adj; }
				else if(g >= max_rgb) { g = max_value; r *= adj; b *= adj; }
				else { b = max_value; r *= adj; g *= adj; }
			}
		}
	}
};
static inline C3 operator*(const C3 &a, const C3 &b) { return {a.r * b.r, a.g * b.g, a.b * b.b}; }
static inline C3 operator*(float f, const C3 &c) { return {f * c.r, f * c.g, f * c.b}; }
static inline C3 operator*(const C3 &c, float f) { return {f * c.r, f * c.g, f * c.b}; }
static inline C3 operator/(const C3 &c, float f) { return {c.r / f, c.g / f, c.b / f}; }
static inline C3 operator+(const C3 &a, const C3 &b) { return {a.r + b.r, a.g + b.g, a.b + b.b}; }

// ---------------------------------------------------------------------------------------------
// samplers (include/sampler/sample.h, include/sampler/halton.h, src/sampler/halton.cc,
// include/math/random.h)
// ---------------------------------------------------------------------------------------------
// sample.h:102-110
static inline float riVdC(uint32_t bits, uint32_t r = 0)
{
	bits = (bits << 16) | (bits >> 16);
	bits = ((bits & 0x00ff00ff) << 8) | ((bits & 0xff00ff00) >> 8);
	bits = ((bits & 0x0f0f0f0f) << 4) | ((bits & 0xf0f0f0f0) >> 4);
	bits = ((bits & 0x33333333) << 2) | ((bits & 0xcccccccc) >> 2);
	bits = ((bits & 0x55555555) << 1) | ((bits & 0xaaaaaaaa) >> 1);
	return std::max(0.f, std::min(1.f, static_cast<float>(static_cast<double>(bits ^ r) * sample_mult_ratio)));
}
// sample.h:112-117 (Sobol generator matrix: v ^= v >> 1)
static inline float riS(uint32_t i, uint32_t r = 0)
{
	for(uint32_t v = 1u << 31; i; i >>= 1, v ^= v >> 1)
		if(i & 1) r ^= v;
	return std::max(0.f, std::min(1.f, static_cast<float>(static_cast<double>(r) * sample_mult_ratio)));
}
// sample.h:119-124 (Larcher-Pillichshammer: v |= v >> 1)
static inline float riLp(uint32_t i, uint32_t r = 0)
{
	for(uint32_t v = 1u << 31; i; i >>= 1, v |= v >> 1)
		if(i & 1) r ^= v;
	return std::max(0.f, std::min(1.f, static_cast<float>(static_cast<double>(r) * sample_mult_ratio)));
}

// integrator_tiled.cc:319-335: sub-pixel position of sample `sample` (sample_idx = pass offset + sample)
static inline void sampleOffsets(int passes, int n_samples, int sample, uint32_t sample_idx, uint32_t offset, float &dx, float &dy)
{
	dx = 0.5f;
	dy = 0.5f;
	if(passes > 1)
	{
		dx = riVdC(sample_idx, offset);
		dy = riS(sample_idx, offset);
	}
	else if(n_samples > 1)
	{
		dx = (0.5f + static_cast<float>(sample)) * (1.f / static_cast<float>(n_samples));
		dy = riLp(sample + offset);
	}
}

// sample.h:132-149 (FNV-1a over the 4 little-endian bytes)
static inline uint32_t fnv32(uint32_t value)
{
	uint32_t hash = 0x811c9dc5u;
	for(int k = 0; k < 4; ++k)
	{
		hash ^= (value >> (8 * k)) & 0xffu;
		hash *= 0x01000193u;
	}
	return hash;
}

// sample.h:45-54 — note the long double product s_2 * 2pi before the float conversion.
static inline V3 cosHemisphere(const V3 &n, const V3 &ru, const V3 &rv, float s_1, float s_2)
{
	if(s_1 >= 1.0f) return n;
	const float z_1 = s_1;
	const float z_2 = static_cast<float>(s_2 * mult_pi_by_2);
	const V3 a = ru * fcos(z_2);
	const V3 b = rv * fsin(z_2);
	return (a + b) * fsqrt(1.f - z_1) + n * fsqrt(z_1);
}

// halton.h:41-81
struct Halton
{
	uint32_t base;
	double inv_base, value;
	explicit Halton(int b) : base(b), inv_base(1.0 / static_cast<double>(b)), value(0.0) {}
	Halton(int b, uint32_t start) : Halton(b) { setStart(start); }
	void setStart(uint32_t start)
	{
		double factor = inv_base;
		value = 0.0;
		while(start > 0)
		{
			value += static_cast<double>(start % base) * factor;
			start /= base;
			factor *= inv_base;
		}
	}
	float getNext()
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
		return std::max(0.f, std::min(1.f, static_cast<float>(value)));
	}
};

// Faure digit permutations (halton.cc:26-401 holds them as literal tables; here they are
// generated by Faure's recursive construction and checked against the reference tables
// through oracle/_ref).  sigma_2 = identity; sigma_2b = (2*sigma_b, 2*sigma_b + 1);
// sigma_{2b+1} = sigma_2b with entries >= b shifted up by one and b inserted in the middle.
static std::vector<int> faurePerm(int b)
{
	if(b <= 2) return {0, 1};
	if((b & 1) == 0)
	{
		const std::vector<int> h = faurePerm(b / 2);
		std::vector<int> out;
		for(int v : h) out.push_back(2 * v);
		for(int v : h) out.push_back(2 * v + 1);
		return out;
	}
	const std::vector<int> p = faurePerm(b - 1);
	const int c = (b - 1) / 2;
	std::vector<int> out;
	for(int i = 0; i < static_cast<int>(p.size()); ++i)
	{
		if(i == c) out.push_back(c);
		out.push_back(p[i] + (p[i] >= c ? 1 : 0));
	}
	return out;
}

struct FaureTables
{
	int prims[50];
	double inv_prims[50];
	std::vector<int> sigma[50];
	FaureTables()
	{
		// halton.cc:409-414: prims[0] = 1, then the first 49 primes; inv_prims are 1/p rounded to
		// 9 decimals (literal decimal constants in the reference, reproduced exactly as n / 1e9).
		int p = 1, k = 0;
		prims[k++] = 1;
		for(int c = 2; k < 50; ++c)
		{
			bool pr = true;
			for(int d = 2; d * d <= c; ++d) if(c % d == 0) { pr = false; break; }
			if(pr) prims[k++] = c;
		}
		(void)p;
		for(int i = 0; i < 50; ++i)
		{
			inv_prims[i] = static_cast<double>(std::llround(1e9 / prims[i])) / 1e9;
			// halton.cc:403-407: dims 0..2 share the base-3 table
			sigma[i] = faurePerm(i <= 2 ? 3 : prims[i]);
		}
	}
};
static const FaureTables &faure()
{
	static const FaureTables t;
	return t;
}

// halton.cc:421-441
static double lowDiscrepancySampling(int dim, uint32_t n)
{
	double value = 0.0;
	if(dim == 0) return 0.0;  // base 1: the reference loops forever for n > 0; never used
	if(dim < 50)
	{
		const FaureTables &t = faure();
		const std::vector<int> &sigma = t.sigma[dim];
		const uint32_t base = t.prims[dim];
		const double f = t.inv_prims[dim];
		double dn = static_cast<double>(n);
		double factor = f;
		while(n > 0)
		{
			value += static_cast<double>(sigma[n % base]) * factor;
			dn *= f;
			n = static_cast<uint32_t>(dn);
			factor *= f;
		}
	}
	return value;
}

// random.h:56-104 (MWC)
struct Mwc
{
	uint32_t x = 30903, c = 0;
	explicit Mwc(uint32_t seed) : c(seed) {}
	double operator()()
	{
		const uint32_t a = 1791398085u, ah = a >> 16, al = a & 65535u;
		const uint32_t xh = x >> 16, xl = x & 65535u;
		x = x * a + c;
		c = xh * ah + ((xh * al) >> 16) + ((xl * ah) >> 16);
		if(xl * al >= ~c + 1) c++;
		return static_cast<double>(static_cast<LD>(x) * sample_mult_ratio);
	}
};

// ---------------------------------------------------------------------------------------------
// film filter (include/math/filter.h:34-90, src/render/imagefilm.cc:129-162)
// ---------------------------------------------------------------------------------------------
static float filterBox(float, float) { return 1.f; }
static float filterGauss(float dx, float dy)
{
	const float r_2 = dx * dx + dy * dy;
	return std::max(0.f, fexp(-6 * r_2) - 0.00247875f);
}
static float filterMitchell(float dx, float dy)
{
	const float x = 2.f * fsqrt(dx * dx + dy * dy);
	if(x >= 2.f) return 0.f;
	if(x >= 1.f) return x * (x * (x * -0.38888889f + 2.0f) - 3.33333333f) + 1.77777778f;
	return x * x * (1.16666666f * x - 2.0f) + 0.88888889f;
}
static float filterLanczos(float dx, float dy)
{
	const float x = fsqrt(dx * dx + dy * dy);
	if(x == 0.f) return 1.f;
	if(-2 < x && x < 2)
	{
		const float a = static_cast<float>(num_pi * x);
		const float b = static_cast<float>(div_pi_by_2 * x);
		return (fsin(a) * fsin(b)) / (a * b);
	}
	return 0.f;
}

struct FilmTable
{
	float table[256];
	float filterw, table_scale;
	FilmTable(int filter, float filter_size)
	{
		// imagefilm.cc:129 filterw_(filter_size * 0.5), 144-151, 153-162
		filterw = static_cast<float>(filter_size * 0.5);
		float (*ff)(float, float) = filterBox;
		switch(filter)
		{
			case YC_FILTER_MITCHELL: ff = filterMitchell; filterw *= 2.6f; break;
			case YC_FILTER_LANCZOS: ff = filterLanczos; break;
			case YC_FILTER_GAUSS: ff = filterGauss; filterw *= 2.f; break;
			default: ff = filterBox; break;
		}
		filterw = std::min(std::max(0.501f, filterw), 0.5f * 8);
		const float scale = 1.f / 16.f;
		for(int y = 0; y < 16; ++y)
			for(int x = 0; x < 16; ++x) table[y * 16 + x] = ff((x + .5f) * scale, (y + .5f) * scale);
		table_scale = static_cast<float>(0.9999 * 16 / filterw);
	}
};

#include "yaftex.h"

// ---------------------------------------------------------------------------------------------
// scene restatement
// ---------------------------------------------------------------------------------------------
enum BsdfFlags : unsigned
{
	BNone = 0, BSpecular = 1 << 0, BGlossy = 1 << 1, BDiffuse = 1 << 2, BDispersive = 1 << 3,
	BReflect = 1 << 4, BTransmit = 1 << 5, BFilter = 1 << 6, BEmit = 1 << 7, BVolumetric = 1 << 8,
	BAll = BSpecular | BGlossy | BDiffuse | BDispersive | BReflect | BTransmit | BFilter
};

struct Material
{
	int type = YC_MAT_SHINYDIFFUSE;
	unsigned bsdf_flags = BNone;
	C3 diffuse_color, emit_color, light_col;
	float components[4] = {0.f, 0.f, 0.f, 0.f};
	float emit_strength = 0.f;
	int diffuse_shader = -1, diffuse_refl_shader = -1;   // shader-node roots (yc_scene.nodes)
	bool is_mirror = false, is_transparent = false, is_translucent = false, fresnel = false, tbias_mult = false;
	float ior_squared = 1.f, transmit_filter = 1.f, tbias = 0.f;
	C3 mirror_color;          // shinydiffuse mirror colour / mirror material ref_col_
	bool is_diffuse = false, double_sided = false, receive_shadows = true, flat = false;
	int additional_depth = 0;   // Material::additional_depth_ (material_shiny_diffuse.cc:548)
	// Oren-Nayar (material_shiny_diffuse.cc:146-152): coefficients as the float members the
	// reference stores them in; sigma_shader: root of sigma_oren_shader (-1: none)
	bool oren_nayar = false;
	float on_a = 0.f, on_b = 0.f;
	int sigma_shader = -1;
	int n_bsdf = 0;
	unsigned c_flags[4];
	int c_index[4];
};

struct Light
{
	int type = YC_LIGHT_POINT;
	bool cast_shadows = true;
	C3 color;
	V3 position;
	// area light (light_area.cc:33-53)
	V3 corner, to_x, to_y, fnormal, normal, du, dv, c2, c3, c4;
	float area = 0.f, inv_area = 0.f;
	int samples = 1;
	bool shoot_caustic = true, shoot_diffuse = true;   // "with_caustic" / "with_diffuse"
	bool photon_only = false;   // "photon_only": in the photon lists only (render_view.cc:83-111)
	// meshlight (light_object_light.cc:46-73): the object's faces, their area cdf (sample_pdf1d.h)
	std::vector<V3> mv0, mv1, mv2, mng;
	std::vector<float> mcdf;
	bool double_sided = false;
};

struct Tri
{
	V3 v0, v1, v2, ng;
	int mat;
};

// per-triangle surface attributes (FacePrimitive + MeshObject data read by getSurface)
struct TriAttr
{
	bool has_orco = false, has_uv = false, smooth = false;
	V3 orco[3];
	float u[3] = {0.f, 0.f, 0.f}, v[3] = {0.f, 0.f, 0.f};
	V3 vn[3];
	int nidx[3] = {-1, -1, -1};
};

struct Camera
{
	V3 position, vright, vup, vto, cam_z;
	V3 near_p, far_p;
	int resx, resy;
	// camera_perspective.cc:28-52, 59-62: depth of field
	float aperture = 0.f, dof_distance = 0.f;
	V3 dof_rt, dof_up;
	int bokeh_type = 0, bokeh_bias = 0;
	std::vector<float> ls;
};

// halton.h:30-81 (the camera's lens streams)
struct HaltonSeq
{
	unsigned int base;
	double inv_base, value = 0.0;
	explicit HaltonSeq(int b) : base(b), inv_base(1.0 / static_cast<double>(b)) {}
	void setStart(unsigned int start)
	{
		double factor = inv_base;
		value = 0.0;
		while(start > 0)
		{
			value += static_cast<double>(start % base) * factor;
			start /= base;
			factor *= inv_base;
		}
	}
	float getNext()
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
		return std::max(0.f, std::min(1.f, static_cast<float>(value)));
	}
};

// camera_perspective.cc:71-85
static float biasDist(int bias, float r)
{
	switch(bias)
	{
		case 1: return std::sqrt(std::sqrt(r) * r);
		case 2: return std::sqrt(1.f - r * r);
		default: return std::sqrt(r);
	}
}

// vector.cc:128-163
static void shirleyDisk(float r_1, float r_2, float &u, float &v)
{
	float phi = 0.f, r = 0.f;
	const float a = 2.f * r_1 - 1.f;
	const float b = 2.f * r_2 - 1.f;
	if(a > -b)
	{
		if(a > b) { r = a; phi = div_pi_by_4 * (b / a); }
		else { r = b; phi = div_pi_by_4 * (2.f - a / b); }
	}
	else
	{
		if(a < b) { r = -a; phi = div_pi_by_4 * (4.f + b / a); }
		else
		{
			r = -b;
			if(b != 0) phi = div_pi_by_4 * (6.f - a / b);
			else phi = 0.f;
		}
	}
	u = r * fcos(phi);
	v = r * fsin(phi);
}

// camera_perspective.cc:87-124
static void lensUv(const Camera &c, float r_1, float r_2, float &u, float &v)
{
	switch(c.bokeh_type)
	{
		case 3: case 4: case 5: case 6:
		{
			const auto fn = static_cast<float>(c.bokeh_type);
			int idx = int(r_1 * fn);
			r_1 = (r_1 - ((float)idx) / fn) * fn;
			r_1 = biasDist(c.bokeh_bias, r_1);
			const float b_1 = r_1 * r_2;
			const float b_0 = r_1 - b_1;
			idx <<= 1;
			u = c.ls[idx] * b_0 + c.ls[idx + 2] * b_1;
			v = c.ls[idx + 1] * b_0 + c.ls[idx + 3] * b_1;
			break;
		}
		case 1: case 7:
		{
			const float w = (float)mult_pi_by_2 * r_2;
			if(c.bokeh_type == 7) r_1 = std::sqrt((float)0.707106781 + (float)0.292893218);
			else r_1 = biasDist(c.bokeh_bias, r_1);
			u = r_1 * fcos(w);
			v = r_1 * fsin(w);
			break;
		}
		default: shirleyDisk(r_1, r_2, u, v);
	}
}

struct Ray
{
	V3 from, dir;
	float tmin = 0.f, tmax = -1.f;
};

struct SurfacePoint
{
	V3 p, n, ng, nu, nv;
	const Material *mat = nullptr;
	int prim = -1;
	unsigned bsdf_flags = 0;
	C3 dcol;            // getShaderColor(diffuse_shader_, ..., diffuse_color_)
	float drefl = 1.f;  // diffuse_refl_shader_ scalar
	float sigma = 0.f;  // sigma_oren_shader_ scalar (getShaderScalar(..., 0.f))
};

struct IsectData
{
	bool hit = false;
	float t = 0.f, bu = 0.f, bv = 0.f, bw = 0.f;
	int prim = -1;
};

// primitive_triangle.cc:44-71 (Moller-Trumbore with the reference's edge-scaled epsilon)
static inline IsectData triIntersect(const Tri &tr, const Ray &ray)
{
	IsectData d;
	const V3 edge_1 = tr.v1 - tr.v0;
	const V3 edge_2 = tr.v2 - tr.v0;
	const float epsilon = 0.1f * min_raydist_global * std::max(edge_1.length(), edge_2.length());
	const V3 pvec = ray.dir ^ edge_2;
	const float det = dot(edge_1, pvec);
	if(det > -epsilon && det < epsilon) return d;
	const float inv_det = 1.f / det;
	const V3 tvec = ray.from - tr.v0;
	const float u = dot(tvec, pvec) * inv_det;
	if(u < 0.f || u > 1.f) return d;
	const V3 qvec = tvec ^ edge_1;
	const float v = dot(ray.dir, qvec) * inv_det;
	if((v < 0.f) || ((u + v) > 1.f)) return d;
	const float t = dot(edge_2, qvec) * inv_det;
	if(t < epsilon) return d;
	d.hit = true;
	d.t = t;
	d.bu = 1.f - u - v;
	d.bv = u;
	d.bw = v;
	return d;
}

// Plain binary BVH used only to make the oracle fast enough on big meshes.  Boxes are padded
// so that culling is conservative: the closest / any hit returned is the one the reference's
// exhaustive semantics define (accelerator_kdtree.cc:726-746, 851-873); only exact-t ties
// between different primitives may resolve differently.
struct BvhNode
{
	double lo[3], hi[3];
	int left = -1, right = -1, start = 0, count = 0;
};

class Scene
{
	public:
		std::vector<Tri> tris;
		std::vector<Material> mats;
		std::vector<Light> lights;
		std::vector<const Light *> visible;   // RenderView::getLightsVisible (render_view.cc:83-91): the integrators' lights
		Camera cam;
		yc_render rp;
		std::unique_ptr<FilmTable> film;
		std::vector<BvhNode> nodes;
		std::vector<int> order;
		// texturing
		bool has_attr = false;
		std::vector<TriAttr> tattr;
		std::vector<std::unique_ptr<OImageBase>> images;
		std::vector<OTexture> texs;
		std::vector<yc_node> shader_nodes;

		explicit Scene(const yc_scene &s);
		void setupTexturing(const yc_scene &s);
		void surface(const IsectData &d, SurfacePoint &sp) const;
		IsectData intersect(const Ray &ray, float t_max, bool any, uint64_t *ctr) const;
		void allHits(const Ray &ray, float t_max, std::vector<IsectData> &out) const;
		void buildBvh();
		int buildRec(int start, int end, std::vector<V3> &cent);
};

Scene::Scene(const yc_scene &s)
{
	rp = s.rp;
	// materials: material_shiny_diffuse.cc:28-87 (ctor + config), material_simple.cc:36-70
	for(int i = 0; i < s.n_mats; ++i)
	{
		const yc_material &m = s.mats[i];
		Material mm;
		mm.type = m.type;
		mm.receive_shadows = m.receive_shadows != 0;
		mm.flat = m.flat_material != 0;
		if(m.type == YC_MAT_LIGHT)
		{
			mm.bsdf_flags = BEmit;
			mm.light_col = C3(m.color[0], m.color[1], m.color[2]);
			mm.double_sided = m.double_sided != 0;
		}
		else if(m.type == YC_MAT_MIRROR)
		{
			// MirrorMaterial ctor (material_glass.h:86-91): ref_col_ = r_col * ref_val, flags Specular
			mm.mirror_color = C3(m.color[0], m.color[1], m.color[2]) * m.reflect;
			mm.bsdf_flags = BSpecular;
		}
		else if(m.type == YC_MAT_NULL) mm.bsdf_flags = BNone;
		else
		{
			mm.diffuse_color = C3(m.color[0], m.color[1], m.color[2]);
			mm.emit_color = m.emit_strength * mm.diffuse_color;
			mm.emit_strength = m.emit_strength;
			mm.diffuse_shader = m.diffuse_shader;
			mm.diffuse_refl_shader = m.diffuse_refl_shader;
			mm.mirror_color = C3(m.mirror_color[0], m.mirror_color[1], m.mirror_color[2]);
			mm.transmit_filter = m.transmit_filter;
			mm.tbias = m.transparentbias_factor;
			mm.tbias_mult = m.transparentbias_multiply_raydepth != 0;
			if(m.fresnel_effect) { mm.fresnel = true; mm.ior_squared = m.ior * m.ior; }
			if(m.emit_strength > 0.f) mm.bsdf_flags |= BEmit;
			// ShinyDiffuseMaterial::config (material_shiny_diffuse.cc:41-87)
			float acc = 1.f;
			if(m.specular_reflect > 0.00001f)
			{
				mm.is_mirror = true;
				if(!mm.fresnel) acc = 1.f - m.specular_reflect;
				mm.bsdf_flags |= BSpecular | BReflect;
				mm.c_flags[mm.n_bsdf] = BSpecular | BReflect;
				mm.c_index[mm.n_bsdf] = 0;
				++mm.n_bsdf;
			}
			if(m.transparency * acc > 0.00001f)
			{
				mm.is_transparent = true;
				acc *= 1.f - m.transparency;
				mm.bsdf_flags |= BTransmit | BFilter;
				mm.c_flags[mm.n_bsdf] = BTransmit | BFilter;
				mm.c_index[mm.n_bsdf] = 1;
				++mm.n_bsdf;
			}
			if(m.translucency * acc > 0.00001f)
			{
				mm.is_translucent = true;
				acc *= 1.f - m.transparency;
				mm.bsdf_flags |= BDiffuse | BTransmit;
				mm.c_flags[mm.n_bsdf] = BDiffuse | BTransmit;
				mm.c_index[mm.n_bsdf] = 2;
				++mm.n_bsdf;
			}
			if(m.diffuse_strength * acc > 0.00001f)
			{
				mm.is_diffuse = true;
				mm.bsdf_flags |= BDiffuse | BReflect;
				mm.c_flags[mm.n_bsdf] = BDiffuse | BReflect;
				mm.c_index[mm.n_bsdf] = 3;
				++mm.n_bsdf;
			}
			// material_shiny_diffuse.cc:88-100 getComponents (no component shader nodes)
			mm.components[0] = mm.is_mirror ? m.specular_reflect : 0.f;
			mm.components[1] = mm.is_transparent ? m.transparency : 0.f;
			mm.components[2] = mm.is_translucent ? m.translucency : 0.f;
			mm.components[3] = mm.is_diffuse ? m.diffuse_strength : 0.f;
			mm.additional_depth = m.additional_depth;
			if(m.oren_nayar)
			{
				// initOrenNayar(double sigma) (:146-152): double arithmetic stored to float members
				const double sigma_squared = m.sigma * m.sigma;
				mm.on_a = static_cast<float>(1.0 - 0.5 * (sigma_squared / (sigma_squared + 0.33)));
				mm.on_b = static_cast<float>(0.45 * sigma_squared / (sigma_squared + 0.09));
				mm.oren_nayar = true;
				mm.sigma_shader = m.sigma_shader;
			}
		}
		mats.push_back(mm);
	}
	// lights: light_point.cc:28-35, light_area.cc:33-53
	for(int i = 0; i < s.n_lights; ++i)
	{
		const yc_light &l = s.lights[i];
		Light L;
		L.type = l.type;
		L.cast_shadows = l.cast_shadows != 0;
		L.shoot_caustic = l.shoot_caustic != 0;
		L.shoot_diffuse = l.shoot_diffuse != 0;
		L.photon_only = l.photon_only != 0;
		const C3 col(l.color[0], l.color[1], l.color[2]);
		if(l.type == YC_LIGHT_POINT)
		{
			L.position = V3(l.from[0], l.from[1], l.from[2]);
			L.color = col * l.power;
		}
		else if(l.type == YC_LIGHT_MESH)
		{
			// ObjectLight::factory (:221-254) + initIs (:46-73); faces resolved after the geometry below
			L.color = col * l.power * static_cast<float>(num_pi);
			L.samples = l.samples;
			L.double_sided = l.double_sided != 0;
		}
		else
		{
			L.corner = V3(l.from[0], l.from[1], l.from[2]);
			const V3 p1(l.point1[0], l.point1[1], l.point1[2]), p2(l.point2[0], l.point2[1], l.point2[2]);
			L.to_x = p1 - L.corner;
			L.to_y = p2 - L.corner;
			L.samples = l.samples;
			L.fnormal = L.to_y ^ L.to_x;
			L.color = col * l.power * static_cast<float>(num_pi);
			L.area = L.fnormal.normLen();
			L.inv_area = static_cast<float>(1.0 / L.area);
			L.normal = -L.fnormal;
			L.du = L.to_x;
			L.du.normalize();
			L.dv = L.normal ^ L.du;
			L.c2 = L.corner + L.to_x;
			L.c3 = L.corner + (L.to_x + L.to_y);
			L.c4 = L.corner + L.to_y;
		}
		lights.push_back(L);
	}
	// geometry: primitive_triangle.cc:34-37 + 87-95 (geometric normal), object_mesh.cc:78-86
	for(int i = 0; i < s.n_tris; ++i)
	{
		Tri t;
		const int *idx = s.tris + 3 * i;
		t.v0 = V3(s.verts[3 * idx[0]], s.verts[3 * idx[0] + 1], s.verts[3 * idx[0] + 2]);
		t.v1 = V3(s.verts[3 * idx[1]], s.verts[3 * idx[1] + 1], s.verts[3 * idx[1] + 2]);
		t.v2 = V3(s.verts[3 * idx[2]], s.verts[3 * idx[2] + 1], s.verts[3 * idx[2] + 2]);
		t.ng = ((t.v1 - t.v0) ^ (t.v2 - t.v0)).normalize();
		t.mat = s.tri_mat[i];
		tris.push_back(t);
	}
	// meshlights: ObjectLight::initIs (light_object_light.cc:46-73) over the object's faces in creation
	// order — areas (primitive_triangle.cc:208-213), cdf (sample_pdf1d.h:52-66), total area in double
	for(int i = 0; i < s.n_lights; ++i)
	{
		if(s.lights[i].type != YC_LIGHT_MESH) continue;
		Light &L = lights[(size_t)i];
		const yc_object &o = s.objects[s.lights[i].object];
		std::vector<float> areas;
		double total = 0.0;
		for(int k = o.t0; k < o.t0 + o.nt; ++k)
		{
			const Tri &t = tris[(size_t)k];
			L.mv0.push_back(t.v0);
			L.mv1.push_back(t.v1);
			L.mv2.push_back(t.v2);
			L.mng.push_back(t.ng);
			const V3 e01 = t.v1 - t.v0, e02 = t.v2 - t.v0;
			areas.push_back(0.5f * (e01 ^ e02).length());
			total += areas.back();
		}
		const double delta = 1.0 / static_cast<double>(areas.size());
		double c = 0.0;
		for(float a : areas)
		{
			c += static_cast<double>(a) * delta;
			L.mcdf.push_back(static_cast<float>(c));
		}
		const float integral = static_cast<float>(c);
		for(float &e : L.mcdf) e /= integral;
		L.area = static_cast<float>(total);
		L.inv_area = static_cast<float>(1.f / total);
	}
	for(const Light &L : lights)
		if(!L.photon_only) visible.push_back(&L);
	// camera: camera.cc:51-71, camera_perspective.cc:28-69 (no depth of field)
	const yc_camera &c = s.cam;
	const V3 pos(c.from[0], c.from[1], c.from[2]), look(c.to[0], c.to[1], c.to[2]), up(c.up[0], c.up[1], c.up[2]);
	cam.resx = c.resx;
	cam.resy = c.resy;
	const float aspect_ratio = c.aspect * (float)c.resy / (float)c.resx;
	V3 cam_y = up - pos;
	V3 cam_z = look - pos;
	V3 cam_x = cam_z ^ cam_y;
	cam_y = cam_z ^ cam_x;
	cam_x.normalize();
	cam_y.normalize();
	cam_z.normalize();
	cam.position = pos;
	cam.cam_z = cam_z;
	cam.near_p = pos + cam_z * c.near_clip;
	cam.far_p = pos + cam_z * c.far_clip;
	cam.vright = cam_x;
	cam.vup = aspect_ratio * cam_y;
	cam.vto = (cam_z * c.focal) - V3(static_cast<float>(0.5) * (cam.vup + cam.vright));
	cam.vup = V3(cam.vup.x / (float)c.resy, cam.vup.y / (float)c.resy, cam.vup.z / (float)c.resy);
	cam.vright = V3(cam.vright.x / (float)c.resx, cam.vright.y / (float)c.resx, cam.vright.z / (float)c.resx);
	cam.aperture = c.aperture;
	cam.dof_distance = c.dof_distance;
	cam.dof_rt = c.aperture * cam_x;
	cam.dof_up = c.aperture * cam_y;
	cam.bokeh_type = c.bokeh_type;
	cam.bokeh_bias = c.bokeh_bias;
	if(c.bokeh_type >= 3 && c.bokeh_type <= 6)
	{
		float w = c.bokeh_rotation * div_pi_by_180, wi = mult_pi_by_2 / (float)c.bokeh_type;   // degToRad
		const int ns = (c.bokeh_type + 2) * 2;
		cam.ls.resize(ns);
		for(int i = 0; i < ns; i += 2)
		{
			cam.ls[i] = fcos(w);
			cam.ls[i + 1] = fsin(w);
			w += wi;
		}
	}
	film.reset(new FilmTable(rp.filter, rp.filter_size));
	buildBvh();
	setupTexturing(s);
}

// Images (image.cc:38-137 with the TGA / HDR loaders), image textures (texture_image.cc:477-596),
// shader nodes, and per-triangle surface attributes incl. MeshObject::smoothNormals
// (object_mesh.cc:125-240).
void Scene::setupTexturing(const yc_scene &s)
{
	for(int i = 0; i < s.n_images; ++i)
	{
		const yc_image &im = s.images[i];
		std::unique_ptr<OImageBase> img;
		const bool gray = im.type == ImgGray || im.type == ImgGrayAlpha;
		int cs = im.color_space;
		if(im.format == 1) img = loadTga(im.data, (size_t)im.size, im.optimization, cs, im.gamma, gray);
		else if(im.format == 2) { img = loadHdr(im.data, (size_t)im.size, gray); cs = CsLinearRgb; }
		if(!img) img = makeImage(im.width, im.height, im.type, im.optimization);
		if(img)
		{
			img->color_space = cs;
			img->gamma = im.gamma;
			for(int k = 0; k < im.n_set; ++k)
			{
				const int x = im.set_xy[2 * k], y = im.set_xy[2 * k + 1];
				const float *c = im.set_rgba + 4 * k;
				if(x >= 0 && y >= 0 && x < img->w && y < img->h) img->setColor(x, y, Rgba(c[0], c[1], c[2], c[3]));
			}
		}
		images.push_back(std::move(img));
	}
	for(int i = 0; i < s.n_textures; ++i)
	{
		const yc_texture &t = s.textures[i];
		OTexture o;
		o.img = images[t.image].get();
		o.interp = t.interpolation;
		o.clip = t.clip;
		o.xrepeat = t.xrepeat;
		o.yrepeat = t.yrepeat;
		o.mirror_x = t.mirror_x != 0;
		o.mirror_y = t.mirror_y != 0;
		o.rot90 = t.rot90 != 0;
		o.checker_even = t.even_tiles != 0;
		o.checker_odd = t.odd_tiles != 0;
		o.checker_dist = t.checker_dist;
		o.cropminx = t.cropmin_x; o.cropminy = t.cropmin_y; o.cropmaxx = t.cropmax_x; o.cropmaxy = t.cropmax_y;
		o.cropx = (o.cropminx != 0.0) || (o.cropmaxx != 1.0);
		o.cropy = (o.cropminy != 0.0) || (o.cropmaxy != 1.0);
		o.adj_intensity = t.intensity; o.adj_contrast = t.contrast; o.adj_saturation = t.saturation;
		o.adj_hue = t.hue / 60.f;
		o.adj_r = t.factor_red; o.adj_g = t.factor_green; o.adj_b = t.factor_blue;
		o.adj_clamp = t.clamp != 0;
		o.adjustments_set = t.intensity != 1.f || t.contrast != 1.f || t.saturation != 1.f || t.hue != 0.f || t.factor_red != 1.f ||
		                    t.factor_green != 1.f || t.factor_blue != 1.f || t.clamp;
		o.orig_cs = o.img->color_space;
		o.orig_gamma = o.img->gamma;
		texs.push_back(o);
	}
	shader_nodes.assign(s.nodes, s.nodes + s.n_nodes);
	for(const Material &m : mats) if(m.diffuse_shader >= 0 || m.diffuse_refl_shader >= 0 || m.sigma_shader >= 0) has_attr = true;
	tattr.resize(tris.size());
	for(int oi = 0; oi < s.n_objects; ++oi)
	{
		const yc_object &ob = s.objects[oi];
		auto P = [&](int v) { return V3(s.verts[3 * v], s.verts[3 * v + 1], s.verts[3 * v + 2]); };
		std::vector<V3> normals;   // MeshObject::normals_
		if(ob.normals_exported) for(int v = 0; v < ob.nv; ++v) normals.push_back(V3(s.normals[3 * (ob.v0 + v)], s.normals[3 * (ob.v0 + v) + 1], s.normals[3 * (ob.v0 + v) + 2]));
		std::vector<std::array<int, 3>> fn(ob.nt, std::array<int, 3>{-1, -1, -1});   // FacePrimitive::vertex_normals_
		for(int t = 0; t < ob.nt; ++t)
			if(ob.normals_exported) for(int r = 0; r < 3; ++r) fn[t][r] = s.tris[3 * (ob.t0 + t) + r] - ob.v0;   // object_mesh.cc:84
		bool smooth = false;
		if(ob.smooth)
		{
			smooth = true;
			if(!(ob.normals_exported && (int)normals.size() == ob.nv))
			{
				// object_mesh.cc:125-240 over object-local vertex indices
				auto vi = [&](int t, int r) { return s.tris[3 * (ob.t0 + t) + r] - ob.v0; };
				auto lp = [&](int v) { return P(ob.v0 + v); };
				auto sine = [&](int a, int b, int c) {
					const V3 e1 = lp(b) - lp(a), e2 = lp(c) - lp(a);
					const float div = (e1.length() * e2.length()) * 0.99999f + 0.00001f;
					float arg = ((e1 ^ e2).length() / div) * 0.99999f;
					if(arg > 1.f) arg = 1.f;
					return fasin(arg);
				};
				normals.resize(ob.nv, V3(0.f, 0.f, 0.f));
				if(ob.smooth_angle >= 180)
				{
					for(int t = 0; t < ob.nt; ++t)
					{
						const V3 n = tris[ob.t0 + t].ng;
						for(int r = 0; r < 3; ++r) normals[vi(t, r)] += n * sine(vi(t, r), vi(t, (r + 1) % 3), vi(t, (r + 2) % 3));
						for(int r = 0; r < 3; ++r) fn[t][r] = vi(t, r);
					}
					for(V3 &n : normals) n.normalize();
				}
				else if(ob.smooth_angle > 0.1f)
				{
					const float threshold = fcos(static_cast<float>(ob.smooth_angle * div_pi_by_180));
					std::vector<std::vector<int>> pf(ob.nv);
					std::vector<std::vector<float>> ps(ob.nv);
					for(int t = 0; t < ob.nt; ++t)
						for(int r = 0; r < 3; ++r)
						{
							ps[vi(t, r)].push_back(sine(vi(t, r), vi(t, (r + 1) % 3), vi(t, (r + 2) % 3)));
							pf[vi(t, r)].push_back(t);
						}
					for(int pid = 0; pid < ob.nv; ++pid)
					{
						std::vector<V3> vns;
						std::vector<int> vns_idx;
						for(size_t j = 0; j < pf[pid].size(); ++j)
						{
							const int f = pf[pid][j];
							const V3 face_n = tris[ob.t0 + f].ng;
							V3 vn = face_n * ps[pid][j];
							bool sm = false;
							for(size_t k = 0; k < pf[pid].size(); ++k)
							{
								if(pf[pid][k] == f) continue;
								const V3 n2 = tris[ob.t0 + pf[pid][k]].ng;
								if(dot(face_n, n2) > threshold) { sm = true; vn += n2 * ps[pid][k]; }
							}
							int idx = -1;
							if(sm)
							{
								vn.normalize();
								for(size_t q = 0; q < vns.size(); ++q)
									if(dot(vn, vns[q]) > 0.999f) { idx = vns_idx[q]; break; }
								if(idx == -1)
								{
									idx = (int)normals.size();
									vns.push_back(vn);
									vns_idx.push_back(idx);
									normals.push_back(vn);
								}
							}
							for(int r = 0; r < 3; ++r) if(vi(f, r) == pid) { fn[f][r] = idx; break; }
						}
					}
				}
			}
		}
		const bool use_normals = smooth || ob.normals_exported;
		if(use_normals) has_attr = true;
		for(int t = 0; t < ob.nt; ++t)
		{
			TriAttr &ta = tattr[ob.t0 + t];
			const int *idx = s.tris + 3 * (ob.t0 + t);
			if(ob.has_orco)
			{
				ta.has_orco = true;
				for(int r = 0; r < 3; ++r) ta.orco[r] = V3(s.orco[3 * idx[r]], s.orco[3 * idx[r] + 1], s.orco[3 * idx[r] + 2]);
			}
			if(ob.has_uv && s.tri_uv && s.tri_uv[3 * (ob.t0 + t)] >= 0)
			{
				ta.has_uv = true;
				for(int r = 0; r < 3; ++r)
				{
					const int ui = s.tri_uv[3 * (ob.t0 + t) + r];
					ta.u[r] = s.uvs[2 * ui];
					ta.v[r] = s.uvs[2 * ui + 1];
				}
			}
			if(use_normals)
			{
				ta.smooth = true;
				for(int r = 0; r < 3; ++r)
				{
					ta.nidx[r] = fn[t][r];
					if(fn[t][r] >= 0 && fn[t][r] < (int)normals.size()) ta.vn[r] = normals[fn[t][r]];
				}
			}
		}
	}
}

// TrianglePrimitive::getSurface (primitive_triangle.cc:97-176) + ShinyDiffuse::initBsdf's node
// evaluation (material_shiny_diffuse.cc:133-141) for the surface point of hit `d`
void Scene::surface(const IsectData &d, SurfacePoint &sp) const
{
	const Tri &tr = tris[d.prim];
	const Material &m = mats[tr.mat];
	sp.dcol = m.diffuse_color;
	sp.drefl = 1.f;
	if(!has_attr) return;
	const TriAttr &ta = tattr[d.prim];
	const float bu = d.bu, bv = d.bv, bw = d.bw;
	if(ta.smooth)
	{
		V3 v[3];
		for(int r = 0; r < 3; ++r) v[r] = ta.nidx[r] >= 0 ? ta.vn[r] : sp.ng;   // getVertexNormal
		sp.n = bu * v[0] + bv * v[1] + bw * v[2];
		sp.n.normalize();
		createCoordsSystem(sp.n, sp.nu, sp.nv);
	}
	if(m.diffuse_shader < 0 && m.diffuse_refl_shader < 0 && m.sigma_shader < 0) return;
	TexPoint tp;
	tp.p = sp.p;
	tp.ng = sp.ng;
	if(ta.has_orco)
	{
		tp.orco_p = bu * ta.orco[0] + bv * ta.orco[1] + bw * ta.orco[2];
		tp.orco_ng = ((ta.orco[1] - ta.orco[0]) ^ (ta.orco[2] - ta.orco[0])).normalize();
	}
	else
	{
		tp.orco_p = sp.p;
		tp.orco_ng = sp.ng;
	}
	bool implicit_uv = true;
	if(ta.has_uv)
	{
		tp.u = bu * ta.u[0] + bv * ta.u[1] + bw * ta.u[2];
		tp.v = bu * ta.v[0] + bv * ta.v[1] + bw * ta.v[2];
		const float du_1 = ta.u[1] - ta.u[0], du_2 = ta.u[2] - ta.u[0];
		const float dv_1 = ta.v[1] - ta.v[0], dv_2 = ta.v[2] - ta.v[0];
		const float det = du_1 * dv_2 - dv_1 * du_2;
		if(std::abs(det) > 1e-30f) implicit_uv = false;
	}
	if(implicit_uv)
	{
		tp.u = bu;
		tp.v = bv;
	}
	NodeEval ev(shader_nodes, texs, tp);
	if(m.diffuse_shader >= 0)
	{
		const Rgba c = ev.get(m.diffuse_shader).col;
		sp.dcol = C3(c.r, c.g, c.b);
	}
	if(m.diffuse_refl_shader >= 0) sp.drefl = ev.get(m.diffuse_refl_shader).val;
	if(m.sigma_shader >= 0) sp.sigma = ev.get(m.sigma_shader).val;
}

int Scene::buildRec(int start, int end, std::vector<V3> &cent)
{
	BvhNode n;
	for(int k = 0; k < 3; ++k) { n.lo[k] = 1e300; n.hi[k] = -1e300; }
	for(int i = start; i < end; ++i)
	{
		const Tri &t = tris[order[i]];
		for(int k = 0; k < 3; ++k)
		{
			n.lo[k] = std::min(n.lo[k], (double)std::min(t.v0[k], std::min(t.v1[k], t.v2[k])));
			n.hi[k] = std::max(n.hi[k], (double)std::max(t.v0[k], std::max(t.v1[k], t.v2[k])));
		}
	}
	for(int k = 0; k < 3; ++k)
	{
		const double pad = 1e-5 * (std::fabs(n.lo[k]) + std::fabs(n.hi[k]) + (n.hi[k] - n.lo[k])) + 1e-9;
		n.lo[k] -= pad;
		n.hi[k] += pad;
	}
	const int id = (int)nodes.size();
	nodes.push_back(n);
	if(end - start <= 4)
	{
		nodes[id].start = start;
		nodes[id].count = end - start;
		return id;
	}
	int axis = 0;
	double ext = -1;
	for(int k = 0; k < 3; ++k)
		if(nodes[id].hi[k] - nodes[id].lo[k] > ext) { ext = nodes[id].hi[k] - nodes[id].lo[k]; axis = k; }
	const int mid = (start + end) / 2;
	std::nth_element(order.begin() + start, order.begin() + mid, order.begin() + end,
					 [&](int a, int b) { return cent[a][axis] < cent[b][axis] || (cent[a][axis] == cent[b][axis] && a < b); });
	const int l = buildRec(start, mid, cent);
	const int r = buildRec(mid, end, cent);
	nodes[id].left = l;
	nodes[id].right = r;
	return id;
}

void Scene::buildBvh()
{
	order.resize(tris.size());
	std::vector<V3> cent(tris.size());
	for(size_t i = 0; i < tris.size(); ++i)
	{
		order[i] = (int)i;
		for(int k = 0; k < 3; ++k) cent[i][k] = (tris[i].v0[k] + tris[i].v1[k] + tris[i].v2[k]) / 3.f;
	}
	nodes.clear();
	if(!tris.empty()) buildRec(0, (int)tris.size(), cent);
}

static inline bool boxHit(const BvhNode &n, const Ray &ray, double t0, double t1)
{
	double tn = t0, tf = t1;
	for(int k = 0; k < 3; ++k)
	{
		const double o = ray.from[k], d = ray.dir[k];
		if(d == 0.0)
		{
			if(o < n.lo[k] || o > n.hi[k]) return false;
			continue;
		}
		double a = (n.lo[k] - o) / d, b = (n.hi[k] - o) / d;
		if(a > b) std::swap(a, b);
		tn = std::max(tn, a);
		tf = std::min(tf, b);
		if(tn > tf) return false;
	}
	return true;
}

// closest: accelerator_kdtree.cc:726-746 (t < t_max && t >= ray.tmin); any: :851-873
// (t < t_max && t >= 0).  All primitives are "normal" visibility here.
IsectData Scene::intersect(const Ray &ray, float t_max, bool any, uint64_t *ctr) const
{
	if(ctr) ++*ctr;
	IsectData best;
	float best_t = t_max;
	if(nodes.empty()) return best;
	int stack[128];
	int sp = 0;
	stack[sp++] = 0;
	const double lo_t = -1e-3 * (1.0 + std::fabs(ray.tmin));
	while(sp)
	{
		const BvhNode &n = nodes[stack[--sp]];
		const double hi_t = std::isinf(best_t) ? 1e300 : (double)best_t * (1.0 + 1e-5) + 1e-6;
		if(!boxHit(n, ray, lo_t, hi_t)) continue;
		if(n.count)
		{
			for(int i = n.start; i < n.start + n.count; ++i)
			{
				const int pi = order[i];
				IsectData d = triIntersect(tris[pi], ray);
				if(!d.hit) continue;
				if(any)
				{
					if(d.t < t_max && d.t >= 0.f) { d.prim = pi; return d; }
				}
				else if(d.t < best_t && d.t >= ray.tmin)
				{
					// keep the lower primitive index on exact ties so the result is order-free
					d.prim = pi;
					best = d;
					best_t = d.t;
				}
				else if(d.t == best_t && best.hit && pi < best.prim && d.t >= ray.tmin)
				{
					d.prim = pi;
					best = d;
				}
			}
		}
		else
		{
			stack[sp++] = n.left;
			stack[sp++] = n.right;
		}
	}
	return best;
}

// Every primitive hit with t in [ray.tmin, t_max) — the candidate set of intersectTs
// (accelerator_kdtree.cc:1001-1023: '<' t_max, '>=' ray.tmin_, material visibility only).
void Scene::allHits(const Ray &ray, float t_max, std::vector<IsectData> &out) const
{
	out.clear();
	if(nodes.empty()) return;
	int stack[128];
	int sp = 0;
	stack[sp++] = 0;
	const double lo_t = -1e-3 * (1.0 + std::fabs(ray.tmin));
	const double hi_t = std::isinf(t_max) ? 1e300 : (double)t_max * (1.0 + 1e-5) + 1e-6;
	while(sp)
	{
		const BvhNode &n = nodes[stack[--sp]];
		if(!boxHit(n, ray, lo_t, hi_t)) continue;
		if(n.count)
		{
			for(int i = n.start; i < n.start + n.count; ++i)
			{
				const int pi = order[i];
				IsectData d = triIntersect(tris[pi], ray);
				if(!d.hit || !(d.t < t_max && d.t >= ray.tmin)) continue;
				d.prim = pi;
				out.push_back(d);
			}
		}
		else
		{
			stack[sp++] = n.left;
			stack[sp++] = n.right;
		}
	}
}

// ---------------------------------------------------------------------------------------------
// render-side restatement
// ---------------------------------------------------------------------------------------------
struct Sample
{
	float s_1, s_2, pdf = 0.f;
	unsigned flags, sampled_flags = BNone;
	Sample(float a, float b, unsigned f) : s_1(a), s_2(b), flags(f) {}
};

struct LSample
{
	float s_1, s_2;
	C3 col;
	float pdf;
};

class Renderer
{
	public:
		Renderer(const Scene &s) : sc_(s) {}
		const Scene &sc_;
		std::atomic<uint64_t> n_closest{0}, n_shadow{0};
		float light_mult = 1.f;   // TiledIntegrator::aa_light_sample_multiplier_ of the current pass
		float indirect_mult = 1.f;   // TiledIntegrator::aa_indirect_sample_multiplier_ of the current pass

		// per-thread state
		struct Thread
		{
			uint64_t closest = 0, shadow = 0;
			uint32_t correlative = 0;
		};

		// accelerator.cc:55-67 + primitive_triangle.cc:97-176 (flat-shaded, no UV/orco use)
		bool intersect(Thread &th, Ray &ray, SurfacePoint &sp) const
		{
			const float t_max = (ray.tmax >= 0.f) ? ray.tmax : std::numeric_limits<float>::infinity();
			const IsectData d = sc_.intersect(ray, t_max, false, &th.closest);
			if(!d.hit) return false;
			const Tri &tr = sc_.tris[d.prim];
			sp.p = ray.from + d.t * ray.dir;
			sp.ng = tr.ng;
			sp.n = tr.ng;
			createCoordsSystem(sp.n, sp.nu, sp.nv);
			sp.mat = &sc_.mats[tr.mat];
			sp.bsdf_flags = sp.mat->bsdf_flags;
			sp.prim = d.prim;
			sc_.surface(d, sp);
			ray.tmax = d.t;
			return true;
		}
		// accelerator.cc:69-78
		bool isShadowed(Thread &th, const Ray &ray) const
		{
			Ray sray = ray;
			sray.from += sray.dir * sray.tmin;
			const float t_max = (ray.tmax >= 0.f) ? sray.tmax - 2 * sray.tmin : std::numeric_limits<float>::infinity();
			return sc_.intersect(sray, t_max, true, &th.shadow).hit;
		}
		// accelerator.cc:80-93 + accelerator_kdtree.cc:916-1061 (transparent shadows).  The origin
		// moves by tmin but tmin is kept, so hits count from 2 tmin along the original ray.  An opaque
		// hit, or more than `shadow_depth` distinct transparent ones, shadows; otherwise the filter
		// colour is the product of the transparent surfaces' getTransparency(ray.dir).  The kd-tree
		// multiplies in its cell-visiting order; here (and on the GPU) the order is ascending
		// (t, primitive), identical in value for up to two transparent surfaces (a product of two
		// rounded factors does not depend on the order).
		bool isShadowedTs(Thread &th, const Ray &ray, C3 &scol) const
		{
			++th.shadow;
			Ray sray = ray;
			sray.from += sray.dir * sray.tmin;
			const float t_max = (ray.tmax >= 0.f) ? sray.tmax - 2 * sray.tmin : std::numeric_limits<float>::infinity();
			scol = C3(1.f);
			std::vector<IsectData> hits;
			sc_.allHits(sray, t_max, hits);
			int n_transp = 0;
			for(const IsectData &d : hits)
			{
				const Material &m = sc_.mats[sc_.tris[d.prim].mat];
				if(!m.is_transparent) return true;
				++n_transp;
			}
			if(n_transp > sc_.rp.shadow_depth) return true;
			std::sort(hits.begin(), hits.end(), [](const IsectData &a, const IsectData &b) {
				return a.t < b.t || (a.t == b.t && a.prim < b.prim);
			});
			for(const IsectData &d : hits)
			{
				// getSurface (primitive_triangle.cc:97-176) at the hit of the moved ray, then
				// ShinyDiffuseMaterial::getTransparency (material_shiny_diffuse.cc:441-465), wo = ray dir
				SurfacePoint sp;
				const Tri &tr = sc_.tris[d.prim];
				sp.p = sray.from + d.t * sray.dir;
				sp.ng = tr.ng;
				sp.n = tr.ng;
				createCoordsSystem(sp.n, sp.nu, sp.nv);
				sp.mat = &sc_.mats[tr.mat];
				sp.prim = d.prim;
				sc_.surface(d, sp);
				scol = scol * getTransparency(sp, sray.dir);
			}
			return false;
		}
		static C3 getTransparency(const SurfacePoint &sp, const V3 &wo)
		{
			const Material &m = *sp.mat;
			const V3 n = faceForward(sp.ng, sp.n, wo);
			const float kr = fresnelKr(m, wo, n);
			float accum = 1.f;
			if(m.is_mirror) accum = 1.f - kr * m.components[0];
			accum *= m.components[1] * accum;
			const C3 tcol = m.transmit_filter * sp.dcol + C3(1.f - m.transmit_filter);
			return accum * tcol;
		}

		// surface.h:62-65
		static V3 faceForward(const V3 &ng, const V3 &n, const V3 &wo) { return (dot(ng, wo) < 0) ? -n : n; }

		// material_shiny_diffuse.cc:107-119 accumulate (Kr = 1: no Fresnel)
		static void accumulate(const float *c, float kr, float *a)
		{
			a[0] = c[0] * kr;
			float acc = 1.f - a[0];
			a[1] = c[1] * acc;
			acc *= 1.f - c[1];
			a[2] = c[2] * acc;
			acc *= 1.f - c[2];
			a[3] = c[3] * acc;
		}

		// material_shiny_diffuse.cc:102-114
		static float fresnelKr(const Material &m, const V3 &wo, const V3 &n)
		{
			if(!m.fresnel) return 1.f;
			const V3 N = (dot(wo, n) < 0.f) ? -n : n;
			const float c = dot(wo, N);
			float g = m.ior_squared + c * c - 1.f;
			if(g < 0.f) g = 0.f;
			else g = fsqrt(g);
			const float aux = c * (g + c);
			return ((0.5f * (g - c) * (g - c)) / ((g + c) * (g + c))) * (1.f + ((aux - 1) * (aux - 1)) / ((aux + 1) * (aux + 1)));
		}
		// vector.h:255-260
		static V3 reflectDir(const V3 &normal, const V3 &v)
		{
			const float vn = dot(v, normal);
			if(vn < 0.f) return -v;
			return 2.f * vn * normal - v;
		}

		// material_shiny_diffuse.cc:154-188 ShinyDiffuseMaterial::orenNayar(wi, wo, n, use_texture_sigma,
		// texture_sigma); math::sqrt is std::sqrt under FAST_MATH
		static float orenNayar(const V3 &wi, const V3 &wo, const V3 &n, const Material &m, const SurfacePoint &sp)
		{
			const float cos_ti = std::max(-1.f, std::min(1.f, dot(n, wi)));
			const float cos_to = std::max(-1.f, std::min(1.f, dot(n, wo)));
			float maxcos_f = 0.f;
			if(cos_ti < 0.9999f && cos_to < 0.9999f)
			{
				V3 v_1 = wi - n * cos_ti;
				v_1.normalize();
				V3 v_2 = wo - n * cos_to;
				v_2.normalize();
				maxcos_f = std::max(0.f, dot(v_1, v_2));
			}
			float sin_alpha, tan_beta;
			if(cos_to >= cos_ti)
			{
				sin_alpha = fsqrt(1.f - cos_ti * cos_ti);
				tan_beta = fsqrt(1.f - cos_to * cos_to) / ((cos_to == 0.f) ? 1e-8f : cos_to);
			}
			else
			{
				sin_alpha = fsqrt(1.f - cos_to * cos_to);
				tan_beta = fsqrt(1.f - cos_ti * cos_ti) / ((cos_ti == 0.f) ? 1e-8f : cos_ti);
			}
			if(m.sigma_shader >= 0)
			{
				const double texture_sigma = sp.sigma;
				const double sigma_squared = texture_sigma * texture_sigma;
				const double a = 1.0 - 0.5 * (sigma_squared / (sigma_squared + 0.33));
				const double b = 0.45 * sigma_squared / (sigma_squared + 0.09);
				return std::min(1.f, std::max(0.f, (float)(a + b * maxcos_f * sin_alpha * tan_beta)));
			}
			return std::min(1.f, std::max(0.f, m.on_a + m.on_b * maxcos_f * sin_alpha * tan_beta));
		}

		// material_shiny_diffuse.cc:196-238 (mirror / null / light materials evaluate to black)
		C3 eval(const SurfacePoint &sp, const V3 &wo, const V3 &wl, unsigned bsdfs) const
		{
			const Material &m = *sp.mat;
			if(m.type != YC_MAT_SHINYDIFFUSE) return C3(0.f);
			const float cos_ng_wo = dot(sp.ng, wo);
			const float cos_ng_wl = dot(sp.ng, wl);
			const V3 n = faceForward(sp.ng, sp.n, wo);
			if(!(bsdfs & (m.bsdf_flags & BDiffuse))) return C3(0.f);
			const float kr = fresnelKr(m, wo, n);
			const float m_t = (1.f - kr * m.components[0]) * (1.f - m.components[1]);
			const bool transmit = (cos_ng_wo * cos_ng_wl) < 0.f;
			if(transmit && m.is_translucent) return m.components[2] * m_t * sp.dcol;
			if(dot(n, wl) < 0.0 && !m.flat) return C3(0.f);
			float m_d = m_t * (1.f - m.components[2]) * m.components[3];
			if(m.oren_nayar) m_d *= orenNayar(wo, wl, n, m, sp);   // :228-233
			if(m.diffuse_refl_shader >= 0) m_d *= sp.drefl;   // :235
			return m_d * sp.dcol;
		}

		// material_shiny_diffuse.cc:242-247, material_simple.cc:50-55
		C3 emit(const SurfacePoint &sp, const V3 &wo) const
		{
			const Material &m = *sp.mat;
			if(m.type == YC_MAT_LIGHT)
			{
				if(m.double_sided) return m.light_col;
				const float angle = dot(wo, sp.n);
				return angle > 0 ? m.light_col : C3(0.f);
			}
			if(m.type != YC_MAT_SHINYDIFFUSE) return C3(0.f);
			if(m.diffuse_shader >= 0) return sp.dcol * m.emit_strength;   // :242-247
			return m.emit_color;
		}

		// material_shiny_diffuse.cc:457-475
		static float getAlpha(const SurfacePoint &sp, const V3 &wo)
		{
			const Material &m = *sp.mat;
			if(!m.is_transparent) return 1.f;
			const V3 n = faceForward(sp.ng, sp.n, wo);
			const float kr = fresnelKr(m, wo, n);
			const float refl = (1.f - m.components[0] * kr) * m.components[1];
			return 1.f - refl;
		}

		// material_shiny_diffuse.cc:249-337, material_simple.cc:42-48, material_glass.cc:435-468
		C3 sample(const SurfacePoint &sp, const V3 &wo, V3 &wi, Sample &s, float &w) const
		{
			const Material &m = *sp.mat;
			if(m.type == YC_MAT_LIGHT || m.type == YC_MAT_NULL)
			{
				s.pdf = 0.f;
				w = 0.f;
				return C3(0.f);
			}
			if(m.type == YC_MAT_MIRROR)
			{
				wi = reflectDir(sp.n, wo);
				s.sampled_flags = BSpecular | BReflect;
				w = 1.f;
				return m.mirror_color * (1.f / std::abs(dot(sp.n, wi)));
			}
			const float cos_ng_wo = dot(sp.ng, wo);
			const V3 n = faceForward(sp.ng, sp.n, wo);
			const float kr = fresnelKr(m, wo, n);
			float accum_c[4];
			accumulate(m.components, kr, accum_c);
			float sum = 0.f, val[4], width[4];
			unsigned choice[4];
			int n_match = 0, pick = -1;
			for(int i = 0; i < m.n_bsdf; ++i)
			{
				if((s.flags & m.c_flags[i]) == m.c_flags[i])
				{
					width[n_match] = accum_c[m.c_index[i]];
					sum += width[n_match];
					choice[n_match] = m.c_flags[i];
					val[n_match] = sum;
					++n_match;
				}
			}
			if(!n_match || sum < 0.00001) { s.sampled_flags = BNone; s.pdf = 0.f; return C3(1.f); }
			const float inv_sum = 1.f / sum;
			for(int i = 0; i < n_match; ++i)
			{
				val[i] *= inv_sum;
				width[i] *= inv_sum;
				if((s.s_1 <= val[i]) && (pick < 0)) pick = i;
			}
			if(pick < 0) pick = n_match - 1;
			float s_1;
			if(pick > 0) s_1 = (s.s_1 - val[pick - 1]) / width[pick];
			else s_1 = s.s_1 / width[pick];
			C3 scolor(0.f);
			switch(choice[pick])
			{
				case(BSpecular | BReflect):
					wi = reflectDir(n, wo);
					s.pdf = width[pick];
					scolor = m.mirror_color * (accum_c[0]);
					scolor *= 1.f / std::max(std::abs(dot(sp.n, wi)), 1.0e-6f);
					break;
				case(BTransmit | BFilter):
					wi = -wo;
					scolor = accum_c[1] * (m.transmit_filter * sp.dcol + C3(1.f - m.transmit_filter));
					if(std::abs(dot(wi, n)) < 1e-6) s.pdf = 0.f;
					else s.pdf = width[pick];
					break;
				case(BDiffuse | BTransmit):
					wi = cosHemisphere(-n, sp.nu, sp.nv, s_1, s.s_2);
					if(cos_ng_wo * dot(sp.ng, wi) < 0) scolor = accum_c[2] * sp.dcol;
					s.pdf = std::abs(dot(wi, n)) * width[pick];
					break;
				default:
					wi = cosHemisphere(n, sp.nu, sp.nv, s_1, s.s_2);
					if(cos_ng_wo * dot(sp.ng, wi) > 0) scolor = accum_c[3] * sp.dcol;
					if(m.oren_nayar) scolor *= orenNayar(wo, wi, n, m, sp);   // :320-325
					s.pdf = std::abs(dot(wi, n)) * width[pick];
					break;
			}
			s.sampled_flags = choice[pick];
			w = std::abs(dot(wi, sp.n)) / (s.pdf * 0.99f + 0.01f);
			const float alpha = getAlpha(sp, wo);
			w = w * (alpha) + 1.f * (1.f - alpha);
			return scolor;
		}

		// material_shiny_diffuse.cc:339-377
		float pdf(const SurfacePoint &sp, const V3 &wo, const V3 &wi, unsigned bsdfs) const
		{
			const Material &m = *sp.mat;
			if(m.type != YC_MAT_SHINYDIFFUSE) return 0.f;
			if(!(bsdfs & BDiffuse)) return 0.f;
			float pdf = 0.f;
			const float cos_ng_wo = dot(sp.ng, wo);
			const V3 n = faceForward(sp.ng, sp.n, wo);
			float accum_c[4];
			accumulate(m.components, fresnelKr(m, wo, n), accum_c);
			float sum = 0.f, width;
			int n_match = 0;
			for(int i = 0; i < m.n_bsdf; ++i)
			{
				if(bsdfs & m.c_flags[i])
				{
					width = accum_c[m.c_index[i]];
					sum += width;
					if(m.c_flags[i] == (BDiffuse | BTransmit)) { if(cos_ng_wo * dot(sp.ng, wi) < 0) pdf += std::abs(dot(wi, n)) * width; }
					else if(m.c_flags[i] == (BDiffuse | BReflect)) pdf += std::abs(dot(wi, n)) * width;
					++n_match;
				}
			}
			if(!n_match || sum < 0.00001) return 0.f;
			return pdf / sum;
		}

		// getSpecular: material_shiny_diffuse.cc:390-433, material_glass.cc:443-451 (mirror)
		struct Specular { bool refl = false, refr = false; V3 rdir, tdir; C3 rcol, tcol; };
		Specular getSpecular(const SurfacePoint &sp, const V3 &wo) const
		{
			Specular r;
			const Material &m = *sp.mat;
			if(m.type == YC_MAT_MIRROR)
			{
				r.refl = true;
				r.rcol = m.mirror_color;
				r.rdir = reflectDir(faceForward(sp.ng, sp.n, wo), wo);
				return r;
			}
			if(m.type != YC_MAT_SHINYDIFFUSE) return r;
			const bool backface = dot(wo, sp.ng) < 0.f;
			const V3 n = backface ? -sp.n : sp.n;
			const V3 ng = backface ? -sp.ng : sp.ng;
			const float kr = fresnelKr(m, wo, n);
			if(m.is_transparent)
			{
				r.refr = true;
				r.tdir = -wo;
				const C3 tcol = m.transmit_filter * sp.dcol + C3(1.f - m.transmit_filter);
				r.tcol = (1.f - m.components[0] * kr) * m.components[1] * tcol;
			}
			if(m.is_mirror)
			{
				r.refl = true;
				V3 d = wo;
				const float vn = 2.f * (d.x * n.x + d.y * n.y + d.z * n.z);   // Vec3::reflect
				d = V3(vn * n.x - d.x, vn * n.y - d.y, vn * n.z - d.z);
				const float cos_wi_ng = dot(d, ng);
				if(cos_wi_ng < 0.01)
				{
					d += static_cast<float>(0.01 - cos_wi_ng) * ng;
					d.normalize();
				}
				r.rdir = d;
				r.rcol = m.mirror_color * (m.components[0] * kr);
			}
			return r;
		}

		// MonteCarloIntegrator::recursiveRaytrace (integrator_montecarlo.cc:925-968) with the
		// specular reflect / refract branches (:866-923); `ray_level` is the recursion's (caller + 1)
		void recursiveRaytrace(Thread &th, Mwc &rng, int ray_level, unsigned bsdfs, const SurfacePoint &sp, const V3 &wo,
		                       uint32_t sample_idx, uint32_t offset, C3 &col, float &alpha, int additional_depth) const
		{
			col = C3(0.f);
			float asum = 0.f;
			int count = 0;
			if(ray_level <= sc_.rp.raydepth + additional_depth && ray_level < 20 && (bsdfs & (BGlossy | BSpecular | BFilter)) && (bsdfs & (BSpecular | BFilter)))
			{
				const Specular spec = getSpecular(sp, wo);
				const Material &m = *sp.mat;
				for(int k = 0; k < 2; ++k)
				{
					if(!(k == 0 ? spec.refl : spec.refr)) continue;
					Ray ref_ray;
					ref_ray.dir = k == 0 ? spec.rdir : spec.tdir;
					ref_ray.from = sp.p;
					if(k == 1 && m.tbias > 0.f)
					{
						float f = m.tbias;
						if(m.tbias_mult) f *= ray_level;
						ref_ray.from = sp.p + ref_ray.dir * f;
					}
					ref_ray.tmin = sc_.rp.ray_min_dist;
					ref_ray.tmax = -1.f;
					C3 c;
					float a;
					integrate(th, ref_ray, rng, sample_idx, offset, c, a, ray_level, additional_depth);
					c *= (k == 0 ? spec.rcol : spec.tcol);
					col += c;
					asum += a;
					++count;
				}
			}
			alpha = count > 0 ? asum / count : 1.f;
		}

		void integrate(Thread &th, Ray &ray, Mwc &rng, uint32_t sample_idx, uint32_t offset, C3 &col, float &alpha, int ray_level,
		               int additional_depth = 0) const
		{
			if(sc_.rp.integrator == YC_INT_PATH) integratePath(th, ray, rng, sample_idx, offset, col, alpha, ray_level, additional_depth);
			else if(sc_.rp.integrator == YC_INT_PHOTON) integratePhoton(th, ray, rng, sample_idx, offset, col, alpha, ray_level, additional_depth);
			else integrateDirect(th, ray, rng, sample_idx, offset, col, alpha, ray_level, additional_depth);
		}

		float shadowTmin(const SurfacePoint &sp) const
		{
			return sc_.rp.shadow_bias_auto ? sc_.rp.shadow_bias * std::max(1.f, sp.p.length()) : sc_.rp.shadow_bias;
		}

		// light_area.cc:66-96
		// ObjectLight::sampleSurface (light_object_light.cc:89-107) + TrianglePrimitive::sample
		// (primitive_triangle.cc:220-234): (point, geometric normal); zeros on the "Sampling error" branch
		static std::pair<V3, V3> meshSampleSurface(const Light &L, float s_1, float s_2)
		{
			const size_t n = L.mcdf.size();
			size_t k;
			if(s_1 <= 0.f) k = 0;
			else if(s_1 >= 1.f) k = n - 1;
			else k = (size_t)(std::lower_bound(L.mcdf.begin(), L.mcdf.end(), s_1) - L.mcdf.begin());
			if(k >= n) return {V3(0.f, 0.f, 0.f), V3(0.f, 0.f, 0.f)};
			float ss_1, delta = L.mcdf[k];
			if(k > 0)
			{
				delta -= L.mcdf[k - 1];
				ss_1 = (s_1 - L.mcdf[k - 1]) / delta;
			}
			else ss_1 = s_1 / delta;
			const float su_1 = fsqrt(ss_1);
			const float u = 1.f - su_1;
			const float v = s_2 * su_1;
			return {u * L.mv0[k] + v * L.mv1[k] + (1.f - u - v) * L.mv2[k], L.mng[k]};
		}
		// light_object_light.cc:111-146
		static bool meshIllumSample(const Light &L, const SurfacePoint &sp, LSample &s, Ray &wi)
		{
			const auto sampled = meshSampleSurface(L, s.s_1, s.s_2);
			const V3 &p = sampled.first, &n = sampled.second;
			V3 ldir = p - sp.p;
			const float dist_sqr = ldir.lengthSqr();
			const float dist = fsqrt(dist_sqr);
			if(dist <= 0.0) return false;
			ldir *= 1.f / dist;
			float cos_angle = -dot(ldir, n);
			if(cos_angle <= 0)
			{
				if(L.double_sided) cos_angle = -cos_angle;
				else return false;
			}
			wi.tmax = dist;
			wi.dir = ldir;
			s.col = L.color;
			const float area_mul_cosangle = L.area * cos_angle;
			s.pdf = static_cast<float>(dist_sqr * num_pi / ((area_mul_cosangle == 0.f) ? 1e-8f : area_mul_cosangle));
			return true;
		}
		// light_object_light.cc:183-201: the closest face of the light's own tree (faces with
		// t >= ray.tmin, accelerator_kdtree.cc:731) gives the normal; `t` is never written there, so the
		// caller's value stays (areaLightSampleMaterial passes its ray's tmax, -1: 1 / (t * t) = 1)
		static bool meshIntersect(const Light &L, const Ray &ray, float &t, C3 &col, float &ipdf)
		{
			float t_hit = std::numeric_limits<float>::infinity();
			int best = -1;
			for(size_t k = 0; k < L.mv0.size(); ++k)
			{
				Tri tr;
				tr.v0 = L.mv0[k];
				tr.v1 = L.mv1[k];
				tr.v2 = L.mv2[k];
				const IsectData d = triIntersect(tr, ray);
				if(d.hit && d.t < t_hit && d.t >= ray.tmin)
				{
					t_hit = d.t;
					best = (int)k;
				}
			}
			if(best < 0) return false;
			const V3 n = L.mng[(size_t)best];
			float cos_angle = dot(ray.dir, -n);
			if(cos_angle <= 0.f)
			{
				if(L.double_sided) cos_angle = std::abs(cos_angle);
				else return false;
			}
			const float idist_sqr = 1.f / (t * t);
			ipdf = static_cast<float>(idist_sqr * L.area * cos_angle * div_1_by_pi);
			col = L.color;
			return true;
		}
		static bool areaIllumSample(const Light &L, const SurfacePoint &sp, LSample &s, Ray &wi)
		{
			if(L.type == YC_LIGHT_MESH) return meshIllumSample(L, sp, s, wi);
			const V3 p = L.corner + s.s_1 * L.to_x + s.s_2 * L.to_y;
			V3 ldir = p - sp.p;
			const float dist_sqr = ldir.lengthSqr();
			const float dist = fsqrt(dist_sqr);
			if(dist <= 0.0) return false;
			ldir *= 1.f / dist;
			const float cos_angle = dot(ldir, L.fnormal);
			if(cos_angle <= 0) return false;
			wi.tmax = dist;
			wi.dir = ldir;
			s.col = L.color;
			s.pdf = static_cast<float>(dist_sqr * num_pi / (L.area * cos_angle));
			return true;
		}
		// light_area.cc:116-135
		static bool areaTri(const V3 &a, const V3 &b, const V3 &c, const Ray &ray, float &t)
		{
			const V3 edge_1 = b - a;
			const V3 edge_2 = c - a;
			const V3 pvec = ray.dir ^ edge_2;
			const float det = dot(edge_1, pvec);
			if(det == 0.f) return false;
			const float inv_det = 1.f / det;
			const V3 tvec = ray.from - a;
			const float u = dot(tvec, pvec) * inv_det;
			if(u < 0.f || u > 1.f) return false;
			const V3 qvec = tvec ^ edge_1;
			const float v = dot(ray.dir, qvec) * inv_det;
			if((v < 0.f) || ((u + v) > 1.f)) return false;
			t = dot(edge_2, qvec) * inv_det;
			return true;
		}
		// light_area.cc:137-151
		static bool areaIntersect(const Light &L, const Ray &ray, float &t, C3 &col, float &ipdf)
		{
			if(L.type == YC_LIGHT_MESH) return meshIntersect(L, ray, t, col, ipdf);
			const float cos_angle = dot(ray.dir, L.fnormal);
			if(cos_angle <= 0) return false;
			if(!areaTri(L.corner, L.c2, L.c3, ray, t))
			{
				if(!areaTri(L.corner, L.c3, L.c4, ray, t)) return false;
			}
			if(!(t > 1.0e-10f)) return false;
			col = L.color;
			ipdf = static_cast<float>(1.f / (t * t) * L.area * cos_angle * div_1_by_pi);
			return true;
		}

		// integrator_montecarlo.cc:80-154 (point light)
		C3 diracLight(Thread &th, const Light &L, const V3 &wo, const SurfacePoint &sp, bool cast_shadows) const
		{
			// light_point.cc:38-57
			V3 ldir = L.position - sp.p;
			const float dist_sqr = ldir.x * ldir.x + ldir.y * ldir.y + ldir.z * ldir.z;
			const float dist = fsqrt(dist_sqr);
			if(dist == 0.0) return C3(0.f);
			const float idist_sqr = 1.f / (dist_sqr);
			ldir *= 1.f / dist;
			Ray light_ray;
			light_ray.tmax = dist;
			light_ray.dir = ldir;
			const C3 lcol = L.color * idist_sqr;
			C3 col(0.f);
			light_ray.from = sp.p;
			light_ray.tmin = shadowTmin(sp);
			bool shadowed = false;
			C3 scol(0.f);
			if(cast_shadows) shadowed = sc_.rp.transp_shad ? isShadowedTs(th, light_ray, scol) : isShadowed(th, light_ray);
			const float angle_light_normal = sp.mat->flat ? 1.f : std::abs(dot(sp.n, light_ray.dir));
			if(!shadowed)
			{
				const C3 surf_col = eval(sp, wo, light_ray.dir, BAll);
				const C3 transmit_col(1.f);
				const C3 lcol_s = (sc_.rp.transp_shad && cast_shadows) ? lcol * scol : lcol;
				col += surf_col * lcol_s * angle_light_normal * transmit_col;
			}
			return col;
		}

		// integrator_montecarlo.cc:156-282
		C3 areaLightSampleLight(Thread &th, Halton &hal_2, Halton &hal_3, const Light &L, const V3 &wo, const SurfacePoint &sp, bool cast_shadows, unsigned num_samples, float inv_num_samples) const
		{
			Ray light_ray;
			light_ray.from = sp.p;
			C3 col(0.f);
			LSample ls;
			for(unsigned i = 0; i < num_samples; ++i)
			{
				ls.s_1 = hal_2.getNext();
				ls.s_2 = hal_3.getNext();
				if(areaIllumSample(L, sp, ls, light_ray))
				{
					light_ray.tmin = shadowTmin(sp);
					bool shadowed = false;
					C3 scol(0.f);
					if(cast_shadows) shadowed = sc_.rp.transp_shad ? isShadowedTs(th, light_ray, scol) : isShadowed(th, light_ray);
					if(!shadowed && ls.pdf > 1e-6f)
					{
						if(sc_.rp.transp_shad && cast_shadows) ls.col = ls.col * scol;
						const C3 surf_col = eval(sp, wo, light_ray.dir, BAll);
						const float angle_light_normal = sp.mat->flat ? 1.f : std::abs(dot(sp.n, light_ray.dir));
						float w = 1.f;
						const float m_pdf = pdf(sp, wo, light_ray.dir, BGlossy | BDiffuse | BDispersive | BReflect | BTransmit);
						if(m_pdf > 1e-6f)
						{
							const float l_2 = ls.pdf * ls.pdf;
							const float m_2 = m_pdf * m_pdf;
							w = l_2 / (l_2 + m_2);
						}
						col += surf_col * ls.col * angle_light_normal * w / ls.pdf;
					}
				}
			}
			return col * inv_num_samples;
		}

		// integrator_montecarlo.cc:284-383
		C3 areaLightSampleMaterial(Thread &th, Halton &hal_2, Halton &hal_3, const Light &L, const V3 &wo, const SurfacePoint &sp, bool cast_shadows, unsigned num_samples, float inv_num_samples) const
		{
			Ray b_ray;
			C3 col(0.f), lcol;
			for(unsigned i = 0; i < num_samples; ++i)
			{
				if(sc_.rp.ray_min_dist_auto) b_ray.tmin = sc_.rp.ray_min_dist * std::max(1.f, sp.p.length());
				else b_ray.tmin = sc_.rp.ray_min_dist;
				b_ray.from = sp.p;
				const float s_1 = hal_2.getNext();
				const float s_2 = hal_3.getNext();
				float W = 0.f;
				Sample s(s_1, s_2, BGlossy | BDiffuse | BDispersive | BReflect | BTransmit);
				const C3 surf_col = sample(sp, wo, b_ray.dir, s, W);
				float light_pdf;
				if(s.pdf > 1e-6f && areaIntersect(L, b_ray, b_ray.tmax, lcol, light_pdf))
				{
					bool shadowed = false;
					C3 scol(0.f);
					if(cast_shadows) shadowed = sc_.rp.transp_shad ? isShadowedTs(th, b_ray, scol) : isShadowed(th, b_ray);
					if(!shadowed && light_pdf > 1e-6f)
					{
						if(sc_.rp.transp_shad && cast_shadows) lcol = lcol * scol;
						const float l_pdf = 1.f / light_pdf;
						const float l_2 = l_pdf * l_pdf;
						const float m_2 = s.pdf * s.pdf;
						const float w = m_2 / (l_2 + m_2);
						col += surf_col * lcol * w * W;
					}
				}
			}
			return col * inv_num_samples;
		}

		// integrator_montecarlo.cc:385-408
		C3 doLightEstimation(Thread &th, const Light &L, const SurfacePoint &sp, const V3 &wo, unsigned loffs, uint32_t sample_idx, uint32_t offset) const
		{
			C3 col(0.f);
			const bool cast_shadows = L.cast_shadows && sp.mat->receive_shadows;
			if(L.type == YC_LIGHT_POINT) col += diracLight(th, L, wo, sp, cast_shadows);
			else
			{
				const unsigned l_offs = loffs * 4567;
				// integrator_montecarlo.cc:396: ceilf(nSamples() * aa_light_sample_multiplier_)
				const int num_samples = static_cast<int>(ceilf(static_cast<float>(L.samples) * light_mult));
				const float inv_num_samples = 1.f / static_cast<float>(num_samples);
				const unsigned offs = num_samples * sample_idx + offset + l_offs;
				Halton hal_2(2, offs - 1);
				Halton hal_3(3, offs - 1);
				col += areaLightSampleLight(th, hal_2, hal_3, L, wo, sp, cast_shadows, num_samples, inv_num_samples);
				hal_2.setStart(offs - 1);
				hal_3.setStart(offs - 1);
				col += areaLightSampleMaterial(th, hal_2, hal_3, L, wo, sp, cast_shadows, num_samples, inv_num_samples);
			}
			return col;
		}

		// integrator_montecarlo.cc:54-68
		C3 estimateAllDirectLight(Thread &th, const SurfacePoint &sp, const V3 &wo, uint32_t sample_idx, uint32_t offset) const
		{
			C3 col(0.f);
			unsigned loffs = 0;
			for(const Light *L : sc_.visible)
			{
				col += doLightEstimation(th, *L, sp, wo, loffs, sample_idx, offset);
				++loffs;
			}
			return col;
		}

		// integrator_montecarlo.cc:70-78 (the light pick uses a per-thread running counter)
		C3 estimateOneDirectLight(Thread &th, const SurfacePoint &sp, const V3 &wo, uint32_t sample_idx, uint32_t offset) const
		{
			const int num_lights = (int)sc_.visible.size();
			if(num_lights == 0) return C3(0.f);
			Halton hal_2(2, sc_.rp.base_sampling_offset + th.correlative - 1);
			const int lnum = std::min(static_cast<int>(hal_2.getNext() * static_cast<float>(num_lights)), num_lights - 1);
			++th.correlative;
			return doLightEstimation(th, *sc_.visible[lnum], sp, wo, lnum, sample_idx, offset) * static_cast<float>(num_lights);
		}

		// integrator_tiled.cc:707-720
		void background(const Ray &, C3 &col, float &alpha, int ray_level = 0) const
		{
			if(sc_.rp.bg_transp && (ray_level == 0 || sc_.rp.bg_transp_refract)) { col = C3(0.f); alpha = 0.f; }
			else if(sc_.rp.has_background) { col = C3(sc_.rp.bg_color[0], sc_.rp.bg_color[1], sc_.rp.bg_color[2]); alpha = 1.f; }
			else { col = C3(0.f); alpha = 1.f; }
		}

		// integrator_direct_light.cc:97-144
		// TiledIntegrator::sampleAmbientOcclusion (integrator_tiled.cc:644-691), clay = false, one ray division
		C3 sampleAmbientOcclusion(Thread &th, const SurfacePoint &sp, const V3 &wo, uint32_t sample_idx, uint32_t offset) const
		{
			const yc_render &rp = sc_.rp;
			C3 col(0.f);
			const unsigned mat_bsdfs = sp.bsdf_flags;
			Ray light_ray;
			light_ray.from = sp.p;
			light_ray.dir = V3(0.f, 0.f, 0.f);
			const int n = rp.ao_samples;
			const unsigned offs = n * sample_idx + offset;
			Halton hal_2(2, offs - 1);
			Halton hal_3(3, offs - 1);
			const C3 ao_col(rp.ao_col[0], rp.ao_col[1], rp.ao_col[2]);
			for(int i = 0; i < n; ++i)
			{
				const float s_1 = hal_2.getNext();
				const float s_2 = hal_3.getNext();
				light_ray.tmin = shadowTmin(sp);
				light_ray.tmax = rp.ao_dist;
				float w = 0.f;
				Sample s(s_1, s_2, BGlossy | BDiffuse | BReflect);
				const C3 surf_col = sample(sp, wo, light_ray.dir, s, w);
				if(mat_bsdfs & BEmit) col += emit(sp, wo) * s.pdf;
				bool shadowed;
				C3 scol(0.f);
				if(rp.transp_shad) shadowed = isShadowedTs(th, light_ray, scol);
				else shadowed = isShadowed(th, light_ray);
				if(!shadowed)
				{
					const float cos = std::abs(dot(sp.n, light_ray.dir));
					if(rp.transp_shad) col += ao_col * scol * surf_col * cos * w;
					else col += ao_col * surf_col * cos * w;
				}
			}
			return col / static_cast<float>(n);
		}

		void integrateDirect(Thread &th, Ray &ray, Mwc &rng, uint32_t sample_idx, uint32_t offset, C3 &col, float &alpha, int ray_level = 0,
		                     int additional_depth = 0) const
		{
			col = C3(0.f);
			alpha = 1.f;
			SurfacePoint sp;
			if(intersect(th, ray, sp))
			{
				const unsigned mat_bsdfs = sp.bsdf_flags;
				const V3 wo = -ray.dir;
				additional_depth = std::max(additional_depth, sp.mat->additional_depth);   // :107
				if(mat_bsdfs & BEmit) col += emit(sp, wo);
				if(mat_bsdfs & BDiffuse)
				{
					col += estimateAllDirectLight(th, sp, wo, sample_idx, offset);
					if(sc_.rp.caus_map) col += causticPhotons(sp, wo);                                  // :120-123
					if(sc_.rp.do_ao) col += sampleAmbientOcclusion(th, sp, wo, sample_idx, offset);   // :124
				}
				C3 rcol;
				recursiveRaytrace(th, rng, ray_level + 1, mat_bsdfs, sp, wo, sample_idx, offset, rcol, alpha, additional_depth);
				col += rcol;
			}
			else background(ray, col, alpha, ray_level);
		}

		// integrator_path_tracer.cc:120-290
		void integratePath(Thread &th, Ray &ray, Mwc &rng, uint32_t sample_idx, uint32_t offset, C3 &col, float &alpha, int ray_level = 0,
		                   int additional_depth = 0) const
		{
			const yc_render &rp = sc_.rp;
			col = C3(0.f);
			alpha = 1.f;
			float w = 0.f;
			SurfacePoint sp;
			if(!intersect(th, ray, sp)) { background(ray, col, alpha, ray_level); return; }
			const unsigned mat_bsdfs = sp.bsdf_flags;
			const V3 wo = -ray.dir;
			additional_depth = std::max(additional_depth, sp.mat->additional_depth);   // path_tracer.cc:133
			if(mat_bsdfs & BEmit) col += emit(sp, wo);
			if(mat_bsdfs & BDiffuse)
			{
				col += estimateAllDirectLight(th, sp, wo, sample_idx, offset);
				if(sc_.rp.caus_map) col += causticPhotons(sp, wo);   // path_tracer.cc:149-152 (caustic_type photon | both)
			}
			unsigned path_flags = BDiffuse;
			if(mat_bsdfs & path_flags)
			{
				C3 path_col(0.f);
				path_flags |= (BDiffuse | BReflect | BTransmit);
				const int n_samples = std::max(1, rp.path_samples);
				for(int i = 0; i < n_samples; ++i)
				{
					const unsigned offs = rp.path_samples * sample_idx + offset + i;
					C3 throughput(1.f), lcol, scol;
					SurfacePoint hit = sp;
					V3 pwo = wo;
					Ray p_ray;
					const float s_1 = riVdC(offs);
					const float s_2 = static_cast<float>(lowDiscrepancySampling(2, offs));
					Sample s(s_1, s_2, path_flags);
					scol = sample(sp, pwo, p_ray.dir, s, w);
					scol *= w;
					throughput = scol;
					p_ray.tmin = rp.ray_min_dist;
					p_ray.tmax = -1.f;
					p_ray.from = sp.p;
					SurfacePoint nh;
					if(!intersect(th, p_ray, nh)) continue;
					hit = nh;
					if(s.sampled_flags != BNone) pwo = -p_ray.dir;
					lcol = estimateOneDirectLight(th, hit, pwo, sample_idx, offset);
					const unsigned mat_bsd_fs = hit.bsdf_flags;
					if(mat_bsd_fs & BEmit) lcol += emit(hit, pwo);
					path_col += lcol * throughput;
					bool caustic = false;
					for(int depth = 1; depth < rp.bounces; ++depth)
					{
						const int d_4 = 4 * depth;
						s.s_1 = static_cast<float>(lowDiscrepancySampling(d_4 + 3, offs));
						s.s_2 = static_cast<float>(lowDiscrepancySampling(d_4 + 4, offs));
						s.flags = BAll;
						scol = sample(hit, pwo, p_ray.dir, s, w);
						scol *= w;
						if(scol.isBlack()) break;
						throughput *= scol;
						caustic = rp.caustic_path && (s.sampled_flags & (BSpecular | BGlossy | BFilter));
						p_ray.tmin = rp.ray_min_dist;
						p_ray.tmax = -1.f;
						p_ray.from = hit.p;
						SurfacePoint nh2;
						if(!intersect(th, p_ray, nh2)) break;
						hit = nh2;
						pwo = -p_ray.dir;
						if(mat_bsd_fs & BDiffuse) lcol = estimateOneDirectLight(th, hit, pwo, sample_idx, offset);
						else lcol = C3(0.f);
						if(depth > rp.rr_min_bounces)
						{
							const float random_value = static_cast<float>(rng());
							const float probability = throughput.maximum();
							if(probability <= 0.f || probability < random_value) break;
							throughput *= 1.f / probability;
						}
						if((mat_bsd_fs & BEmit) && caustic) lcol += emit(hit, pwo);
						path_col += lcol * throughput;
					}
				}
				col += path_col / static_cast<float>(n_samples);
			}
			C3 rcol;
			recursiveRaytrace(th, rng, ray_level + 1, mat_bsdfs, sp, wo, sample_idx, offset, rcol, alpha, additional_depth);
			col += rcol;
		}

		// ------------------------------------------------------------------------------------
		// Photon mapping (integrator_photon_mapping.cc, finalGather = false)
		// ------------------------------------------------------------------------------------
		// include/photon/photon.h:30-78 (no SMALL_PHOTONS)
		struct Photon { V3 pos, dir; C3 col; };
		// include/photon/pkdtree.h:41-64: leaf -> photon index, interior -> split + right child
		struct PkNode
		{
			uint32_t data = 0;    // split position bits (interior) or photon index (leaf)
			uint32_t flags = 0;   // bits 0-1 axis (3 = leaf), bits 2.. right child
			bool isLeaf() const { return (flags & 3u) == 3u; }
			int axis() const { return (int)(flags & 3u); }
			float split() const { float f; std::memcpy(&f, &data, 4); return f; }
			uint32_t right() const { return flags >> 2; }
		};
		// photon.h:103-140 PhotonMap: photons in append order (photon-id order: one reference
		// thread's order), the kd-tree over them, and the number of shot paths
		struct PhotonMapData
		{
			std::vector<Photon> photons;
			std::vector<PkNode> nodes;
			int n_paths = 0;
			bool ready() const { return !nodes.empty(); }   // updateTree ran on a non-empty map
		};
		PhotonMapData dmap;   // diffuse map (PhotonIntegrator)
		PhotonMapData cmap;   // caustic map (MonteCarloIntegrator::createCausticMap)
		// final gathering: photon.h:91-99 RadData, and the radiance map of Photon(normal, pos,
		// pre-gathered radiance) (integrator_photon_mapping.cc:80, 585-589)
		struct RadData { V3 pos, normal; C3 refl, transm; };
		std::vector<RadData> rad_points;
		PhotonMapData rmap;

		// :186 draws the global FastRandom (shared by the photon threads, so schedule-dependent)
		// against 0.125; here a hash of the deposit slot (photon id, bounce) keeps one in eight, and
		// the GPU uses the same hash (the radiance-point subset is matched statistically, like RR)
		static bool fgRadSelect(uint32_t slot) { return (fnv32(slot ^ 0x6a09e667u) & 7u) == 0u; }

		// material.cc:156-174 Material::getReflectivity
		C3 getReflectivity(const SurfacePoint &sp, unsigned flags) const
		{
			if(!(flags & (BTransmit | BReflect) & sp.bsdf_flags)) return C3(0.f);
			C3 total(0.f);
			for(int i = 0; i < 16; ++i)
			{
				const float s_1 = 0.03125f + 0.0625f * static_cast<float>(i);
				const float s_2 = riVdC((uint32_t)i);
				const float s_3 = static_cast<float>(lowDiscrepancySampling(2, (uint32_t)i));
				const float s_4 = static_cast<float>(lowDiscrepancySampling(3, (uint32_t)i));
				const V3 wo = cosHemisphere(sp.n, sp.nu, sp.nv, s_1, s_2);
				V3 wi;
				Sample s(s_3, s_4, flags);
				float w = 0.f;
				const C3 col = sample(sp, wo, wi, s, w);
				total += col * w;
			}
			return total * 0.0625f;
		}

		// include/sampler/sample_pdf1d.h:52-93 (cumulateStep1DDf + dSample)
		struct Pdf1D
		{
			std::vector<float> func, cdf;
			float integral = 0.f, inv_integral = 0.f;
			explicit Pdf1D(const std::vector<float> &f) : func(f), cdf(f.size())
			{
				const double delta = 1.0 / static_cast<double>(f.size());
				double c = 0.0;
				for(size_t i = 0; i < f.size(); ++i)
				{
					c += static_cast<double>(f[i]) * delta;
					cdf[i] = static_cast<float>(c);
				}
				integral = static_cast<float>(c);
				for(float &e : cdf) e /= integral;
				inv_integral = 1.f / integral;
			}
			int dSample(float u, float &pdf) const
			{
				int index;
				if(u <= 0.f) index = 0;
				else if(u >= 1.f) index = (int)cdf.size() - 1;
				else index = (int)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
				pdf = func[index] * inv_integral;
				return index;
			}
		};

		// sample.h:58-75
		static V3 sphereDir(float s_1, float s_2)
		{
			V3 dir;
			dir.z = 1.0f - 2.0f * s_1;
			float r = 1.0f - dir.z * dir.z;
			if(r > 0.0f)
			{
				r = fsqrt(r);
				const float a = static_cast<float>(mult_pi_by_2 * s_2);
				dir.x = fcos(a) * r;
				dir.y = fsin(a) * r;
			}
			else { dir.x = 0.0f; dir.y = 0.0f; }
			return dir;
		}

		// light_area.cc:98-104, light_point.cc:79-85
		static C3 emitPhoton(const Light &L, float s_1, float s_2, float s_3, float s_4, Ray &ray, float &ipdf)
		{
			if(L.type == YC_LIGHT_POINT)
			{
				ray.from = L.position;
				ray.dir = sphereDir(s_1, s_2);
				ipdf = static_cast<float>(4.0f * num_pi);
				return L.color;
			}
			if(L.type == YC_LIGHT_MESH)
			{
				// light_object_light.cc:148-163
				ipdf = L.area;
				const auto sampled = meshSampleSurface(L, s_3, s_4);
				ray.from = sampled.first;
				const V3 normal = sampled.second;
				V3 cu, cv;
				createCoordsSystem(normal, cu, cv);
				if(L.double_sided)
				{
					ipdf *= 2.f;
					if(s_1 > 0.5f) ray.dir = cosHemisphere(-normal, cu, cv, (s_1 - 0.5f) * 2.f, s_2);
					else ray.dir = cosHemisphere(normal, cu, cv, s_1 * 2.f, s_2);
				}
				else ray.dir = cosHemisphere(normal, cu, cv, s_1, s_2);
				return L.color;
			}
			ipdf = L.area;
			ray.from = L.corner + s_3 * L.to_x + s_4 * L.to_y;
			ray.dir = cosHemisphere(L.normal, L.du, L.dv, s_1, s_2);
			return L.color;
		}

		// light_area.cc:64, light_point.h:41 (Rgb::energy, color.h:59)
		static float lightEnergy(const Light &L)
		{
			// light_object_light.cc:109: double-sided ? 2 color area : color area
			const C3 e = (L.type == YC_LIGHT_POINT)  ? (L.color * 4.0f) * static_cast<float>(num_pi)
			             : (L.type == YC_LIGHT_MESH) ? (L.double_sided ? (2.f * L.color) * L.area : L.color * L.area)
			                                         : L.color * L.area;
			return (e.r + e.g + e.b) * 0.333333f;
		}

		// material.cc:137-153 (Material::scatterPhoton) with PSample (material.h:260-268); `flags` is
		// PSample's flag set: All for the diffuse map, AllSpecular | Glossy | Filter | Dispersive for
		// the caustic map (integrator_montecarlo.cc:497)
		bool scatterPhoton(const SurfacePoint &sp, const V3 &wi, V3 &wo, float s_1, float s_2, float s_3, const C3 &lcol,
		                   C3 &color_out, unsigned &sampled, unsigned flags = BAll) const
		{
			float w = 0.f;
			Sample s(s_1, s_2, flags);
			const C3 scol = sample(sp, wi, wo, s, w);
			sampled = s.sampled_flags;
			if(s.pdf > 1.0e-6f)
			{
				const C3 alpha(1.f);
				const C3 cnew = lcol * alpha * scol * w;
				const float new_max = std::max(cnew.r, std::max(cnew.g, cnew.b));
				const float old_max = std::max(lcol.r, std::max(lcol.g, lcol.b));
				const float prob = std::min(1.f, new_max / old_max);
				if(s_3 <= prob && prob > 1e-4f)
				{
					color_out = cnew / prob;
					return true;
				}
			}
			return false;
		}

		// render_view.cc:103-110 getLightsEmittingDiffusePhotons / getLightsEmittingCausticPhotons
		std::vector<const Light *> photonLights(bool caustic) const
		{
			std::vector<const Light *> v;
			for(const Light &L : sc_.lights)
				if(caustic ? L.shoot_caustic : L.shoot_diffuse) v.push_back(&L);
			return v;
		}

		// integrator_photon_mapping.cc:110-235 (diffuseWorker), photons in photon-id order
		void shootDiffusePhotons(Thread &th)
		{
			const yc_render &rp = sc_.rp;
			PhotonMapData &M = dmap;
			M.photons.clear();
			rad_points.clear();
			const std::vector<const Light *> lights = photonLights(false);
			const int num_lights = (int)lights.size();
			if(num_lights == 0 || rp.pm_photons <= 0) { M.n_paths = 0; return; }
			std::vector<float> energies(num_lights);
			for(int i = 0; i < num_lights; ++i) energies[i] = lightEnergy(*lights[i]);
			const Pdf1D light_power(energies);
			const int T = std::max(1, rp.pm_threads);
			const unsigned n_photons = std::max((unsigned)T, ((unsigned)rp.pm_photons / T) * T);   // :437
			const float f_num_lights = static_cast<float>(num_lights);
			const float inv_diff_photons = 1.f / static_cast<float>(n_photons);
			for(unsigned h = 0; h < n_photons; ++h)
			{
				const float s_1 = riVdC(h);
				const float s_2 = static_cast<float>(lowDiscrepancySampling(2, h));
				const float s_3 = static_cast<float>(lowDiscrepancySampling(3, h));
				const float s_4 = static_cast<float>(lowDiscrepancySampling(4, h));
				const float s_l = float(h) * inv_diff_photons;
				float light_num_pdf;
				const int light_num = light_power.dSample(s_l, light_num_pdf);
				Ray ray;
				float light_pdf;
				C3 pcol = emitPhoton(*lights[light_num], s_1, s_2, s_3, s_4, ray, light_pdf);
				ray.tmin = rp.ray_min_dist;
				ray.tmax = -1.f;
				pcol = pcol * (f_num_lights * light_pdf / light_num_pdf);
				if(pcol.r == 0.f && pcol.g == 0.f && pcol.b == 0.f) continue;
				int n_bounces = 0;
				bool caustic_photon = false, direct_photon = true;
				for(;;)
				{
					SurfacePoint sp;
					if(!intersect(th, ray, sp)) break;
					const V3 wi = -ray.dir;
					if(sp.bsdf_flags & BDiffuse)
					{
						if(!caustic_photon) M.photons.push_back({sp.p, wi, pcol});
						// :184-193 radiance point for final gathering (one deposit in eight)
						if(rp.pm_fg && !caustic_photon && fgRadSelect(h * (uint32_t)(rp.pm_bounces + 1) + (uint32_t)n_bounces))
						{
							RadData rd;
							rd.pos = sp.p;
							rd.normal = faceForward(sp.ng, sp.n, wi);
							rd.refl = getReflectivity(sp, BDiffuse | BGlossy | BReflect);
							rd.transm = getReflectivity(sp, BDiffuse | BGlossy | BTransmit);
							rad_points.push_back(rd);
						}
					}
					if(n_bounces == rp.pm_bounces) break;
					const int d_5 = 3 * n_bounces + 5;
					const float s_5 = static_cast<float>(lowDiscrepancySampling(d_5, h));
					const float s_6 = static_cast<float>(lowDiscrepancySampling(d_5 + 1, h));
					const float s_7 = static_cast<float>(lowDiscrepancySampling(d_5 + 2, h));
					V3 wo;
					C3 ncol;
					unsigned sampled = BNone;
					if(!scatterPhoton(sp, wi, wo, s_5, s_6, s_7, pcol, ncol, sampled)) break;
					pcol = ncol;
					caustic_photon = ((sampled & (BGlossy | BSpecular | BDispersive)) && direct_photon) ||
					                 ((sampled & (BGlossy | BSpecular | BFilter | BDispersive)) && caustic_photon);
					direct_photon = (sampled & BFilter) && direct_photon;
					ray.from = sp.p;
					ray.dir = wo;
					ray.tmin = rp.ray_min_dist;
					ray.tmax = -1.f;
					++n_bounces;
				}
			}
			M.n_paths = (int)n_photons;
		}

		// integrator_montecarlo.cc:421-544 (causticWorker) with createCausticMap's photon count
		// (:588-604), photons in photon-id order: a photon is stored on a diffuse / glossy surface
		// only after a specular / glossy (/ filter) bounce, and paths scatter only specularly
		void shootCausticPhotons(Thread &th)
		{
			const yc_render &rp = sc_.rp;
			PhotonMapData &M = cmap;
			M.photons.clear();
			M.nodes.clear();
			M.n_paths = 0;
			const std::vector<const Light *> lights = photonLights(true);
			const int num_lights = (int)lights.size();
			if(num_lights == 0 || !rp.caus_map) return;
			std::vector<float> energies(num_lights);
			for(int i = 0; i < num_lights; ++i) energies[i] = lightEnergy(*lights[i]);
			const Pdf1D light_power(energies);
			const int T = std::max(1, rp.pm_threads);
			const unsigned n_photons = std::max((unsigned)T, ((unsigned)std::max(0, rp.caus_photons) / T) * T);   // :604
			const float f_num_lights = static_cast<float>(num_lights);
			const unsigned flags = BSpecular | BReflect | BTransmit | BGlossy | BFilter | BDispersive;   // :497
			for(unsigned h = 0; h < n_photons; ++h)
			{
				const float s_1 = riVdC(h);
				const float s_2 = static_cast<float>(lowDiscrepancySampling(2, h));
				const float s_3 = static_cast<float>(lowDiscrepancySampling(3, h));
				const float s_4 = static_cast<float>(lowDiscrepancySampling(4, h));
				const float s_l = static_cast<float>(h) / static_cast<float>(n_photons);   // :444
				float light_num_pdf;
				const int light_num = light_power.dSample(s_l, light_num_pdf);
				Ray ray;
				float light_pdf;
				C3 pcol = emitPhoton(*lights[light_num], s_1, s_2, s_3, s_4, ray, light_pdf);
				ray.tmin = rp.ray_min_dist;
				ray.tmax = -1.f;
				pcol = pcol * (f_num_lights * light_pdf / light_num_pdf);
				if(pcol.r == 0.f && pcol.g == 0.f && pcol.b == 0.f) continue;
				int n_bounces = 0;
				bool caustic_photon = false, direct_photon = true;
				for(;;)
				{
					SurfacePoint sp;
					if(!intersect(th, ray, sp)) break;
					const V3 wi = -ray.dir;
					if(sp.bsdf_flags & (BDiffuse | BGlossy))
					{
						if(caustic_photon) M.photons.push_back({sp.p, wi, pcol});
					}
					if(n_bounces == rp.caus_depth) break;
					const int d_5 = 3 * n_bounces + 5;
					const float s_5 = static_cast<float>(lowDiscrepancySampling(d_5, h));
					const float s_6 = static_cast<float>(lowDiscrepancySampling(d_5 + 1, h));
					const float s_7 = static_cast<float>(lowDiscrepancySampling(d_5 + 2, h));
					V3 wo;
					C3 ncol;
					unsigned sampled = BNone;
					if(!scatterPhoton(sp, wi, wo, s_5, s_6, s_7, pcol, ncol, sampled, flags)) break;
					pcol = ncol;
					caustic_photon = ((sampled & (BGlossy | BSpecular | BDispersive)) && direct_photon) ||
					                 ((sampled & (BGlossy | BSpecular | BFilter | BDispersive)) && caustic_photon);
					direct_photon = (sampled & BFilter) && direct_photon;
					if(!(caustic_photon || direct_photon)) break;   // :520-521
					ray.from = sp.p;
					ray.dir = wo;
					ray.tmin = rp.ray_min_dist;
					ray.tmax = -1.f;
					++n_bounces;
				}
			}
			M.n_paths = (int)n_photons;
		}

		// pkdtree.h:115-222 (the threaded and sequential builds produce the same DFS layout)
		static void buildPhotonTree(PhotonMapData &M)
		{
			const uint32_t n = (uint32_t)M.photons.size();
			M.nodes.assign(n ? 2 * (size_t)n - 1 : 0, PkNode());
			if(!n) return;
			std::vector<uint32_t> el(n);
			for(uint32_t i = 0; i < n; ++i) el[i] = i;
			V3 lo = M.photons[0].pos, hi = M.photons[0].pos;
			for(uint32_t i = 1; i < n; ++i)
				for(int a = 0; a < 3; ++a)
				{
					lo[a] = std::min(lo[a], M.photons[i].pos[a]);
					hi[a] = std::max(hi[a], M.photons[i].pos[a]);
				}
			uint32_t next = 0;
			buildRec(M, 0, n, lo, hi, el.data(), next);
		}
		static void buildRec(PhotonMapData &M, uint32_t start, uint32_t end, V3 lo, V3 hi, uint32_t *el, uint32_t &next)
		{
			if(end - start == 1)
			{
				M.nodes[next].flags = 3;
				M.nodes[next].data = el[start];
				++next;
				return;
			}
			// bound.h:111-115 largestAxis
			const V3 d = hi - lo;
			const int axis = (d.x > d.y) ? ((d.x > d.z) ? 0 : 2) : ((d.y > d.z) ? 1 : 2);
			const uint32_t split_el = (start + end) / 2;
			// pkdtree.h:66-74 CompareNode: by coordinate, ties by element address (= index)
			std::nth_element(el + start, el + split_el, el + end, [&](uint32_t a, uint32_t b) {
				const float pa = M.photons[a].pos[axis], pb = M.photons[b].pos[axis];
				return pa == pb ? (a < b) : pa < pb;
			});
			const uint32_t cur = next;
			const float split_pos = M.photons[el[split_el]].pos[axis];
			std::memcpy(&M.nodes[cur].data, &split_pos, 4);
			M.nodes[cur].flags = (uint32_t)axis;
			++next;
			V3 hi_l = hi, lo_r = lo;
			hi_l[axis] = split_pos;
			lo_r[axis] = split_pos;
			buildRec(M, start, split_el, lo, hi_l, el, next);
			M.nodes[cur].flags = (M.nodes[cur].flags & 3u) | (next << 2);
			buildRec(M, split_el, end, lo_r, hi, el, next);
		}

		// photon.h:93-100 FoundPhoton (operator< on the squared distance)
		struct Found
		{
			uint32_t photon;
			float dist_square;
			bool operator<(const Found &o) const { return dist_square < o.dist_square; }
		};

		// pkdtree.h:225-292 (non-recursive lookup) + photon.cc:31-52 (PhotonGather heap management)
		static int gather(const PhotonMapData &M, const V3 &p, Found *found, uint32_t k, float &max_dist_squared)
		{
			struct Stack { int node; float s; int axis; };
			Stack stack[64];
			uint32_t n_found = 0;
			int curr = 0;
			int sp = 1;
			stack[sp].node = -1;
			for(;;)
			{
				while(!M.nodes[curr].isLeaf())
				{
					const int axis = M.nodes[curr].axis();
					const float split_val = M.nodes[curr].split();
					int far_child;
					if(p[axis] <= split_val) { far_child = (int)M.nodes[curr].right(); curr = curr + 1; }
					else { far_child = curr + 1; curr = (int)M.nodes[curr].right(); }
					++sp;
					stack[sp].node = far_child;
					stack[sp].axis = axis;
					stack[sp].s = split_val;
				}
				const Photon &ph = M.photons[M.nodes[curr].data];
				const V3 v = ph.pos - p;
				float dist_2 = v.lengthSqr();
				if(dist_2 < max_dist_squared)
				{
					if(n_found < k)
					{
						found[n_found++] = {M.nodes[curr].data, dist_2};
						if(n_found == k)
						{
							std::make_heap(found, found + k);
							max_dist_squared = found[0].dist_square;
						}
					}
					else
					{
						std::pop_heap(found, found + k);
						found[k - 1] = {M.nodes[curr].data, dist_2};
						std::push_heap(found, found + k);
						max_dist_squared = found[0].dist_square;
					}
				}
				if(stack[sp].node < 0) return (int)n_found;
				int axis = stack[sp].axis;
				dist_2 = p[axis] - stack[sp].s;
				dist_2 *= dist_2;
				while(dist_2 > max_dist_squared)
				{
					--sp;
					if(stack[sp].node < 0) return (int)n_found;
					axis = stack[sp].axis;
					dist_2 = p[axis] - stack[sp].s;
					dist_2 *= dist_2;
				}
				curr = stack[sp].node;
				--sp;
			}
		}

		// sample.h:31-35 kernel: 3 / (pi r^2) (1 - d^2 / r^2)^2, the product formed in long double
		static float photonKernel(float r_photon_2, float ir_gather_2)
		{
			const float s = (1.f - r_photon_2 * ir_gather_2);
			return static_cast<float>(3.f * ir_gather_2 * div_1_by_pi * s * s);
		}

		// MonteCarloIntegrator::estimateCausticPhotons (integrator_montecarlo.cc:627-648) via
		// causticPhotons (:410-419; clamp_indirect = 0)
		C3 causticPhotons(const SurfacePoint &sp, const V3 &wo) const
		{
			const yc_render &rp = sc_.rp;
			if(!cmap.ready()) return C3(0.f);
			std::vector<Found> gathered((size_t)std::max(1, rp.caus_search));
			const float caus_radius = rp.caus_radius;
			float g_radius_square = caus_radius * caus_radius;
			const int n_gathered = gather(cmap, sp.p, gathered.data(), (uint32_t)rp.caus_search, g_radius_square);
			g_radius_square = 1.f / g_radius_square;
			C3 sum(0.f);
			if(n_gathered > 0)
			{
				for(int i = 0; i < n_gathered; ++i)
				{
					const Photon &ph = cmap.photons[gathered[i].photon];
					const C3 surf_col = eval(sp, wo, ph.dir, BAll);
					const float k = photonKernel(gathered[i].dist_square, g_radius_square);
					sum += surf_col * k * ph.col;
				}
				sum *= 1.f / static_cast<float>(cmap.n_paths);
			}
			return sum;
		}

		// :560-572: radiance points in shooting order; each kept point marks every point within the
		// squared distance `maxrad` (strictly less, pkdtree.h:263-268) whose normal faces the same side
		// (EliminatePhoton, photon.h:172-180) as unused, itself included — the kept set is the greedy
		// one in index order whatever the lookup's visiting order.  A uniform grid of cell sqrt(maxrad)
		// finds the candidates (the r_tree of the reference only serves this range query).
		static std::vector<uint32_t> eliminateRadPoints(const std::vector<RadData> &pts, float maxrad)
		{
			std::vector<uint32_t> kept;
			const size_t n = pts.size();
			if(!n) return kept;
			const double cell = std::sqrt((double)maxrad) * 1.0001 + 1e-30;
			auto key = [&](const V3 &p, int dx, int dy, int dz) {
				const int64_t x = (int64_t)std::floor(p.x / cell) + dx, y = (int64_t)std::floor(p.y / cell) + dy,
				              z = (int64_t)std::floor(p.z / cell) + dz;
				return (uint64_t)(x * 73856093) ^ (uint64_t)(y * 19349663) ^ (uint64_t)(z * 83492791);
			};
			std::unordered_map<uint64_t, std::vector<uint32_t>> grid;
			for(uint32_t i = 0; i < n; ++i) grid[key(pts[i].pos, 0, 0, 0)].push_back(i);
			std::vector<uint8_t> use(n, 1);
			for(uint32_t i = 0; i < n; ++i)
			{
				if(!use[i]) continue;
				kept.push_back(i);
				const RadData &q = pts[i];
				for(int dx = -1; dx <= 1; ++dx)
					for(int dy = -1; dy <= 1; ++dy)
						for(int dz = -1; dz <= 1; ++dz)
						{
							auto it = grid.find(key(q.pos, dx, dy, dz));
							if(it == grid.end()) continue;
							for(uint32_t j : it->second)
							{
								const V3 v = pts[j].pos - q.pos;
								if(v.lengthSqr() < maxrad && dot(pts[j].normal, q.normal) > 0.f) use[j] = 0;
							}
						}
			}
			return kept;
		}

		// :540-591 + preGatherWorker (:39-88): the kept radiance points gather the diffuse map within
		// diffuseRadius^2 (here the radius IS squared, unlike integrate()'s :954) and store
		// Photon(normal, pos, sum) in the radiance map, whose tree updateTree builds (:589)
		void buildRadianceMap()
		{
			const yc_render &rp = sc_.rp;
			const std::vector<uint32_t> kept = eliminateRadPoints(rad_points, 0.01f * rp.pm_diffuse_radius);
			const float ds_radius_2 = rp.pm_diffuse_radius * rp.pm_diffuse_radius;
			const float i_scale = static_cast<float>(1.f / ((float)dmap.n_paths * num_pi));
			rmap.photons.clear();
			rmap.nodes.clear();
			std::vector<Found> gathered((size_t)std::max(1, rp.pm_search));
			for(uint32_t idx : kept)
			{
				const RadData &r = rad_points[idx];
				float radius = ds_radius_2;
				const int n_gathered = gather(dmap, r.pos, gathered.data(), (uint32_t)rp.pm_search, radius);
				C3 sum(0.f);
				if(n_gathered > 0)
				{
					const float scale = i_scale / radius;
					for(int i = 0; i < n_gathered; ++i)
					{
						const Photon &ph = dmap.photons[gathered[i].photon];
						if(dot(r.normal, ph.dir) > 0.f) sum += r.refl * scale * ph.col;
						else sum += r.transm * scale * ph.col;
					}
				}
				rmap.photons.push_back({r.pos, r.normal, sum});
			}
			rmap.n_paths = dmap.n_paths;
			if(!rmap.photons.empty()) buildPhotonTree(rmap);
		}

		// photon.cc:136-142 findNearest: NearestPhoton (photon.h:159-169) over the non-recursive
		// lookup — the last photon accepted (facing n, strictly closer than the shrinking radius)
		static int findNearest(const PhotonMapData &M, const V3 &p, const V3 &n, float max_dist_squared)
		{
			if(!M.ready()) return -1;   // an empty radiance map has no tree (the reference would crash)
			struct Stack { int node; float s; int axis; };
			Stack stack[64];
			int nearest = -1;
			int curr = 0;
			int sp = 1;
			stack[sp].node = -1;
			for(;;)
			{
				while(!M.nodes[curr].isLeaf())
				{
					const int axis = M.nodes[curr].axis();
					const float split_val = M.nodes[curr].split();
					int far_child;
					if(p[axis] <= split_val) { far_child = (int)M.nodes[curr].right(); curr = curr + 1; }
					else { far_child = curr + 1; curr = (int)M.nodes[curr].right(); }
					++sp;
					stack[sp].node = far_child;
					stack[sp].axis = axis;
					stack[sp].s = split_val;
				}
				const Photon &ph = M.photons[M.nodes[curr].data];
				const V3 v = ph.pos - p;
				float dist_2 = v.lengthSqr();
				if(dist_2 < max_dist_squared)
				{
					if(dot(ph.dir, n) > 0.f) { nearest = (int)M.nodes[curr].data; max_dist_squared = dist_2; }
				}
				if(stack[sp].node < 0) return nearest;
				int axis = stack[sp].axis;
				dist_2 = p[axis] - stack[sp].s;
				dist_2 *= dist_2;
				while(dist_2 > max_dist_squared)
				{
					--sp;
					if(stack[sp].node < 0) return nearest;
					axis = stack[sp].axis;
					dist_2 = p[axis] - stack[sp].s;
					dist_2 *= dist_2;
				}
				curr = stack[sp].node;
				--sp;
			}
		}

		// :640-763 finalGathering, one ray division (no decorrelation) and indirect sample multiplier 1
		// (AA_indirect_sample_multiplier_factor is refused with AA passes).  `mat_bsd_fs` (:682) is a
		// reference into the first gather hit's MaterialData, which the next intersect() frees (:741):
		// undefined from the second hit on; here it reads the current hit's flags (YafaRay's intent).
		C3 finalGathering(Thread &th, const SurfacePoint &sp, const V3 &wo, uint32_t sample_idx, uint32_t offset) const
		{
			const yc_render &rp = sc_.rp;
			const float lookup_rad = 4 * rp.pm_diffuse_radius * rp.pm_diffuse_radius;   // :245
			C3 path_col(0.f);
			float w = 0.f;
			// integrator_photon_mapping.cc:648
			const int n_sampl = (int)ceilf(std::max(1, rp.fg_samples) * indirect_mult);
			for(int i = 0; i < n_sampl; ++i)
			{
				C3 throughput(1.f);
				float length = 0;
				SurfacePoint hit = sp;
				V3 pwo = wo;
				Ray p_ray;
				const unsigned offs = (unsigned)rp.fg_samples * sample_idx + offset + (unsigned)i;
				C3 lcol(0.f), scol;
				const float s_1 = riVdC(offs);
				const float s_2 = static_cast<float>(lowDiscrepancySampling(2, offs));
				Sample s(s_1, s_2, BDiffuse | BReflect | BTransmit);
				scol = sample(hit, pwo, p_ray.dir, s, w);
				scol *= w;
				if(scol.isBlack()) continue;
				p_ray.tmin = rp.ray_min_dist;
				p_ray.tmax = -1.f;
				p_ray.from = hit.p;
				throughput = scol;
				{
					SurfacePoint nh;
					if(!intersect(th, p_ray, nh)) continue;
					hit = nh;
				}
				bool did_hit = true;
				length = p_ray.tmax;
				unsigned mat_bsd_fs = hit.bsdf_flags;
				const bool has_spec = mat_bsd_fs & BSpecular;
				bool caustic = false;
				bool close = length < rp.fg_min_pathlen;
				bool do_bounce = close || has_spec;
				for(int depth = 0; depth < rp.fg_bounces && do_bounce; ++depth)
				{
					const int d_4 = 4 * depth;
					pwo = -p_ray.dir;
					if(mat_bsd_fs & BDiffuse)
					{
						if(close) lcol = estimateOneDirectLight(th, hit, pwo, sample_idx, offset);
						else if(caustic)
						{
							const V3 sf = faceForward(hit.ng, hit.n, pwo);
							const int nearest = findNearest(rmap, hit.p, sf, lookup_rad);
							if(nearest >= 0) lcol = rmap.photons[nearest].col;
						}
						if(close || caustic)
						{
							if(mat_bsd_fs & BEmit) lcol += emit(hit, pwo);
							path_col += lcol * throughput;
						}
					}
					Sample sb(static_cast<float>(lowDiscrepancySampling(d_4 + 3, offs)), static_cast<float>(lowDiscrepancySampling(d_4 + 4, offs)),
					          close ? BAll : (BSpecular | BReflect | BTransmit | BFilter));
					scol = sample(hit, pwo, p_ray.dir, sb, w);
					if(sb.pdf <= 1.0e-6f) { did_hit = false; break; }
					scol *= w;
					p_ray.tmin = rp.ray_min_dist;
					p_ray.tmax = -1.f;
					p_ray.from = hit.p;
					throughput *= scol;
					SurfacePoint nh;
					if(!intersect(th, p_ray, nh)) { did_hit = false; break; }
					hit = nh;
					mat_bsd_fs = hit.bsdf_flags;
					length += p_ray.tmax;
					caustic = (caustic || !depth) && (sb.sampled_flags & (BSpecular | BFilter));
					close = length < rp.fg_min_pathlen;
					do_bounce = caustic || close;
				}
				if(did_hit && (mat_bsd_fs & (BDiffuse | BGlossy)))
				{
					const V3 sf = faceForward(hit.ng, hit.n, -p_ray.dir);
					const int nearest = findNearest(rmap, hit.p, sf, lookup_rad);
					if(nearest >= 0) lcol = rmap.photons[nearest].col;
					if(mat_bsd_fs & BEmit) lcol += emit(hit, -p_ray.dir);
					path_col += lcol * throughput;
				}
			}
			return path_col / (float)n_sampl;
		}

		// integrator_photon_mapping.cc:852-1004 (show_map = false)
		void integratePhoton(Thread &th, Ray &ray, Mwc &rng, uint32_t sample_idx, uint32_t offset, C3 &col, float &alpha, int ray_level = 0,
		                     int additional_depth = 0) const
		{
			const yc_render &rp = sc_.rp;
			col = C3(0.f);
			alpha = 1.f;
			SurfacePoint sp;
			if(intersect(th, ray, sp))
			{
				const V3 wo = -ray.dir;
				const unsigned mat_bsdfs = sp.bsdf_flags;
				additional_depth = std::max(additional_depth, sp.mat->additional_depth);   // :863
				col += emit(sp, wo);                                   // :868-869
				if(rp.pm_show_map && !dmap.photons.empty())
				{
					// :876-881 (final gathering: the radiance map within lookup_rad_) / :924-929 (the
					// diffuse map within ds_radius_): the nearest photon facing the shading normal
					const V3 n = faceForward(sp.ng, sp.n, wo);
					const PhotonMapData &M = rp.pm_fg ? rmap : dmap;
					const float r2 = rp.pm_fg ? 4 * rp.pm_diffuse_radius * rp.pm_diffuse_radius : rp.pm_diffuse_radius;   // :245
					const int nearest = M.photons.empty() ? -1 : findNearest(M, sp.p, n, r2);
					if(nearest >= 0) col += M.photons[nearest].col;
				}
				else if(rp.pm_fg)
				{
					// :874-917 (use_photon_diffuse_ && final_gather_), clamp_indirect = 0
					if(mat_bsdfs & BEmit) col += emit(sp, wo);         // :895-903
					if(mat_bsdfs & BDiffuse)
					{
						col += estimateAllDirectLight(th, sp, wo, sample_idx, offset);
						col += finalGathering(th, sp, wo, sample_idx, offset);
					}
				}
				else
				{
				if(mat_bsdfs & BEmit) col += emit(sp, wo);             // :938-946 (added a second time)
				if(mat_bsdfs & BDiffuse) col += estimateAllDirectLight(th, sp, wo, sample_idx, offset);
				std::vector<Found> gathered((size_t)std::max(1, rp.pm_search));
				float radius = rp.pm_diffuse_radius;                   // "actually the square radius"
				int n_gathered = 0;
				if(!dmap.photons.empty()) n_gathered = gather(dmap, sp.p, gathered.data(), (uint32_t)rp.pm_search, radius);
				if(n_gathered > 0)
				{
					const float scale = 1.f / ((float)dmap.n_paths * radius * num_pi);
					for(int i = 0; i < n_gathered; ++i)
					{
						const Photon &ph = dmap.photons[gathered[i].photon];
						const C3 surf_col = eval(sp, wo, ph.dir, BDiffuse);
						const C3 col_tmp = surf_col * scale * ph.col;
						col += col_tmp;
					}
				}
				}
				if(rp.caus_map && (mat_bsdfs & BDiffuse)) col += causticPhotons(sp, wo);   // :981-984
				C3 rcol;
				recursiveRaytrace(th, rng, ray_level + 1, mat_bsdfs, sp, wo, sample_idx, offset, rcol, alpha, additional_depth);   // :986
				col += rcol;
			}
			else background(ray, col, alpha, ray_level);
		}

		// PhotonMap::load (photon.cc:54-87): "YAF_PHOTONMAPv1\0", name, paths, search radius, kd-tree
		// threads, count, then position + colour per photon, and updateTree.  The file holds no
		// directions and Photon() leaves dir_ uninitialised (photon.h:33): zero here, as fresh memory.
		static bool loadPhotonMap(const std::string &file, PhotonMapData &M)
		{
			M = PhotonMapData{};
			FILE *fp = std::fopen(file.c_str(), "rb");
			if(!fp) return false;
			auto readStr = [&](std::string &str) {
				str.clear();
				int c;
				while((c = std::fgetc(fp)) != EOF && c != 0) str += (char)c;
				return c == 0;
			};
			std::string header, name;
			int32_t paths = 0, threads = 0;
			float radius = 0.f;
			uint32_t n = 0;
			bool ok = readStr(header) && header == "YAF_PHOTONMAPv1" && readStr(name) && std::fread(&paths, 4, 1, fp) == 1 &&
			          std::fread(&radius, 4, 1, fp) == 1 && std::fread(&threads, 4, 1, fp) == 1 && std::fread(&n, 4, 1, fp) == 1;
			if(ok)
			{
				M.photons.resize(n);
				for(Photon &p : M.photons)
				{
					float v[6];
					if(std::fread(v, 4, 6, fp) != 6) { ok = false; break; }
					p.pos = V3(v[0], v[1], v[2]);
					p.dir = V3();
					p.col.r = v[3];
					p.col.g = v[4];
					p.col.b = v[5];
				}
			}
			std::fclose(fp);
			if(!ok) { M = PhotonMapData{}; return false; }
			M.n_paths = paths;
			if(!M.photons.empty()) buildPhotonTree(M);
			return true;
		}

		// preprocess: the caustic map (PathIntegrator / DirectLight / PhotonIntegrator, when enabled),
		// then the diffuse map (PhotonIntegrator)
		bool preprocessPhotons()
		{
			Thread th;
			if(sc_.rp.pm_load_path)
			{
				const std::string base = sc_.rp.pm_load_path;
				bool ok = true;
				if(sc_.rp.caus_map) ok = loadPhotonMap(base + "_caustic.photonmap", cmap) && ok;
				if(sc_.rp.integrator == YC_INT_PHOTON)
				{
					ok = loadPhotonMap(base + "_diffuse.photonmap", dmap) && ok;
					if(sc_.rp.pm_fg) ok = loadPhotonMap(base + "_fg_radiance.photonmap", rmap) && ok;
				}
				if(ok) return true;
				cmap = PhotonMapData{};   // a failed load generates every map (and would save them)
				dmap = PhotonMapData{};
				rmap = PhotonMapData{};
			}
			if(sc_.rp.caus_map)
			{
				shootCausticPhotons(th);
				if(!cmap.photons.empty()) buildPhotonTree(cmap);
			}
			if(sc_.rp.integrator != YC_INT_PHOTON) return true;
			shootDiffusePhotons(th);
			if(dmap.photons.size() < 50) return false;   // :448-452 "Too few diffuse photons"
			buildPhotonTree(dmap);
			if(sc_.rp.pm_fg) buildRadianceMap();
			return true;
		}

		// camera_perspective.cc:128-146 + plane.h:37-40
		// camera_perspective.cc:128-146
		Ray shootRay(float px, float py, float lu = 0.5f, float lv = 0.5f) const
		{
			const Camera &c = sc_.cam;
			Ray ray;
			ray.from = c.position;
			ray.dir = c.vright * px + c.vup * py + c.vto;
			ray.dir.normalize();
			ray.tmin = dot(c.cam_z, (c.near_p - ray.from)) / dot(ray.dir, c.cam_z);
			ray.tmax = dot(c.cam_z, (c.far_p - ray.from)) / dot(ray.dir, c.cam_z);
			if(c.aperture != 0.f)
			{
				float u, v;
				lensUv(c, lu, lv, u, v);
				const V3 li = c.dof_rt * u + c.dof_up * v;
				ray.from = ray.from + li;
				ray.dir = (ray.dir * c.dof_distance) - li;
				ray.dir.normalize();
			}
			return ray;
		}

		// integrator_tiled.cc:288-405 for one pixel: writes n_samples RGBA
		// integrator_tiled.cc:303-345: n_samples camera samples of pixel (j, i); pass_offs = the
		// pass offset plus the film's base sampling offset (renderPass, :240-250)
		void renderPixel(Thread &th, Mwc &rng, int i, int j, float *out, int n_samples, int pass_offs) const
		{
			const yc_render &rp = sc_.rp;
			// film pixel (j, i) is camera pixel (j + crop_x0, i + crop_y0): renderTile's loops run over
			// the splitter's areas in camera coordinates (imagesplitter.cc:43-46, integrator_tiled.cc:288-342)
			i += rp.crop_y0;
			j += rp.crop_x0;
			const uint32_t offset = fnv32(static_cast<uint32_t>(i) * fnv32(static_cast<uint32_t>(j)));
			// :284-285, 315-316: lens streams Halton(3) / Halton(5) started at pass offset + pixel offset
			HaltonSeq hal_u(3), hal_v(5);
			hal_u.setStart(pass_offs + offset);
			hal_v.setStart(pass_offs + offset);
			for(int sample = 0; sample < n_samples; ++sample)
			{
				const uint32_t sample_idx = pass_offs + sample;
				float dx, dy;
				sampleOffsets(rp.aa_passes, n_samples, sample, sample_idx, offset, dx, dy);
				float lens_u = 0.5f, lens_v = 0.5f;
				if(sc_.cam.aperture != 0.f)
				{
					lens_u = hal_u.getNext();
					lens_v = hal_v.getNext();
				}
				Ray ray = shootRay(j + dx, i + dy, lens_u, lens_v);
				C3 col;
				float alpha;
				if(rp.integrator == YC_INT_PATH) integratePath(th, ray, rng, sample_idx, offset, col, alpha);
				else if(rp.integrator == YC_INT_PHOTON) integratePhoton(th, ray, rng, sample_idx, offset, col, alpha);
				else integrateDirect(th, ray, rng, sample_idx, offset, col, alpha);
				if(alpha > 1.f) alpha = 1.f;
				out[4 * sample] = col.r;
				out[4 * sample + 1] = col.g;
				out[4 * sample + 2] = col.b;
				out[4 * sample + 3] = alpha;
			}
		}
};

// integrator_tiled.cc:56-67 + imagefilm.cc:447-487 + imagesplitter.cc:30-107 (linear order,
// one thread: no tail subdivision)
struct Tile { int x, y, w, h, rank = 0; };

// glibc rand() (random_r TYPE_3: r[i] = r[i-3] + r[i-31], output r >> 1, seeded by srand's
// 16807-LCG fill and 310 discarded outputs): the reference seeds each tile's Russian-roulette
// generator with the next rand() (integrator_tiled.cc:272), one call per tile in render order.
static std::vector<uint32_t> glibcRandSequence(uint32_t seed, size_t n)
{
	std::vector<int32_t> r(344 + n);
	r[0] = (int32_t)(seed == 0 ? 1 : seed);
	for(int i = 1; i < 31; ++i)
	{
		const int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
		int64_t word = 16807 * lo - 2836 * hi;
		if(word < 0) word += 2147483647;
		r[i] = (int32_t)word;
	}
	for(int i = 31; i < 34; ++i) r[i] = r[i - 31];
	for(size_t i = 34; i < r.size(); ++i) r[i] = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
	std::vector<uint32_t> out(n);
	for(size_t k = 0; k < n; ++k) out[k] = ((uint32_t)r[k + 344]) >> 1;
	return out;
}

static std::vector<Tile> tilesLinear(int w, int h, int bs)
{
	std::vector<Tile> t;
	const int nx = (w + bs - 1) / bs, ny = (h + bs - 1) / bs;
	for(int j = 0; j < ny; ++j)
		for(int i = 0; i < nx; ++i)
		{
			Tile r{i * bs, j * bs, 0, 0};
			r.w = std::min(bs, w - r.x);
			r.h = std::min(bs, h - r.y);
			t.push_back(r);
		}
	return t;
}

struct Film
{
	int w, h;
	std::vector<float> rgba, weight;
	const FilmTable &tab;
	float clamp_samples;
	Film(int ww, int hh, const FilmTable &t, float cs) : w(ww), h(hh), rgba(4 * (size_t)ww * hh, 0.f), weight((size_t)ww * hh, 0.f), tab(t), clamp_samples(cs) {}
	// imagefilm.cc:680-733
	void addSample(int x, int y, float dx, float dy, const float *col_in)
	{
		const int dx_0 = std::max(0 - x, roundToInt(static_cast<double>(dx) - tab.filterw));
		const int dx_1 = std::min(w - x - 1, roundToInt(static_cast<double>(dx) + tab.filterw - 1.0));
		const int dy_0 = std::max(0 - y, roundToInt(static_cast<double>(dy) - tab.filterw));
		const int dy_1 = std::min(h - y - 1, roundToInt(static_cast<double>(dy) + tab.filterw - 1.0));
		int x_index[9], y_index[9];
		const double x_offs = dx - 0.5;
		for(int i = dx_0, n = 0; i <= dx_1; ++i, ++n) x_index[n] = floorToInt(std::abs((static_cast<double>(i) - x_offs) * tab.table_scale));
		const double y_offs = dy - 0.5;
		for(int i = dy_0, n = 0; i <= dy_1; ++i, ++n) y_index[n] = floorToInt(std::abs((static_cast<double>(i) - y_offs) * tab.table_scale));
		const int x_0 = x + dx_0, x_1 = x + dx_1, y_0 = y + dy_0, y_1 = y + dy_1;
		for(int j = y_0; j <= y_1; ++j)
			for(int i = x_0; i <= x_1; ++i)
			{
				const float wt = tab.table[y_index[j - y_0] * 16 + x_index[i - x_0]];
				const size_t p = (size_t)j * w + i;
				weight[p] = weight[p] + wt;
				C3 c(col_in[0], col_in[1], col_in[2]);
				c.clampProportional(clamp_samples);
				rgba[4 * p] = rgba[4 * p] + c.r * wt;
				rgba[4 * p + 1] = rgba[4 * p + 1] + c.g * wt;
				rgba[4 * p + 2] = rgba[4 * p + 2] + c.b * wt;
				rgba[4 * p + 3] = rgba[4 * p + 3] + col_in[3] * wt;
			}
	}
};

// imagefilm.cc:799-815
static float darkThresholdCurve(float b)
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

struct Rgba4 { float r, g, b, a; };

// Rgba::normalized (color.h:554-558, operator/ :312-316)
static Rgba4 filmColor(const Film &film, int W, int x, int y)
{
	const size_t p = (size_t)y * W + x;
	const float w = film.weight[p];
	if(w == 0.f) return {0.f, 0.f, 0.f, 0.f};
	const float f = 1.f / w;
	return {film.rgba[4 * p] * f, film.rgba[4 * p + 1] * f, film.rgba[4 * p + 2] * f, film.rgba[4 * p + 3] * f};
}

// Rgba::colorDifference (color.h:450-467), col2Bri (color.h:61)
static float colorDifference(const Rgba4 &a, const Rgba4 &c2, bool rgb)
{
	const float bri_a = 0.2126f * a.r + 0.7152f * a.g + 0.0722f * a.b;
	const float bri_c = 0.2126f * c2.r + 0.7152f * c2.g + 0.0722f * c2.b;
	float d = std::abs(bri_c - bri_a);
	if(rgb)
	{
		const float rd = std::abs(c2.r - a.r), gd = std::abs(c2.g - a.g), bd = std::abs(c2.b - a.b), ad = std::abs(c2.a - a.a);
		if(d < rd) d = rd;
		if(d < gd) d = gd;
		if(d < bd) d = bd;
		if(d < ad) d = ad;
	}
	return d;
}

// ImageFilm::nextPass (imagefilm.cc:259-420) with adaptive_aa = true and no DebugSamplingFactor
// layer: flags the pixels the next pass resamples; returns their count.  doMoreSamples
// (:672-675) resamples every pixel when the threshold is <= 0.
static int aaNextPass(const Film &film, int W, int H, const yc_render &rp, float threshold, std::vector<uint8_t> &flags)
{
	flags.assign((size_t)W * H, 0);
	if(!(threshold > 0.f))
	{
		flags.assign((size_t)W * H, 1);
		return W * H;
	}
	const bool rgb = rp.aa_detect_color_noise != 0;
	const int half = rp.aa_variance_edge_size / 2;
	auto set = [&](int x, int y) { flags[(size_t)y * W + x] = 1; };
	for(int y = 0; y < H; ++y)
		for(int x = 0; x < W; ++x) flags[(size_t)y * W + x] = (film.weight[(size_t)y * W + x] > 0.f) ? 0 : 1;
	float th = threshold;
	for(int y = 0; y < H - 1; ++y)
		for(int x = 0; x < W - 1; ++x)
		{
			const Rgba4 pc = filmColor(film, W, x, y);
			const float bri = 0.2126f * std::abs(pc.r) + 0.7152f * std::abs(pc.g) + 0.0722f * std::abs(pc.b);   // abscol2Bri
			if(rp.aa_dark_detection_type == 1 && rp.aa_dark_threshold_factor > 0.f)
				th = threshold * ((1.f - rp.aa_dark_threshold_factor) + (bri * rp.aa_dark_threshold_factor));
			else if(rp.aa_dark_detection_type == 2) th = darkThresholdCurve(bri);
			if(colorDifference(pc, filmColor(film, W, x + 1, y), rgb) >= th) { set(x, y); set(x + 1, y); }
			if(colorDifference(pc, filmColor(film, W, x, y + 1), rgb) >= th) { set(x, y); set(x, y + 1); }
			if(colorDifference(pc, filmColor(film, W, x + 1, y + 1), rgb) >= th) { set(x, y); set(x + 1, y + 1); }
			if(x > 0 && colorDifference(pc, filmColor(film, W, x - 1, y + 1), rgb) >= th) { set(x, y); set(x - 1, y + 1); }
			if(rp.aa_variance_pixels > 0)
			{
				int vx = 0, vy = 0;
				for(int xd = -half; xd < half - 1; ++xd)
				{
					int xi = x + xd;
					if(xi < 0) xi = 0;
					else if(xi >= W - 1) xi = W - 2;
					if(colorDifference(filmColor(film, W, xi, y), filmColor(film, W, xi + 1, y), rgb) >= th) ++vx;
				}
				for(int yd = -half; yd < half - 1; ++yd)
				{
					int yi = y + yd;
					if(yi < 0) yi = 0;
					else if(yi >= H - 1) yi = H - 2;
					if(colorDifference(filmColor(film, W, x, yi), filmColor(film, W, x, yi + 1), rgb) >= th) ++vy;
				}
				if(vx + vy >= rp.aa_variance_pixels)
					for(int xd = -half; xd < half; ++xd)
						for(int yd = -half; yd < half; ++yd)
						{
							const int xi = std::min(std::max(x + xd, 0), W - 1), yi = std::min(std::max(y + yd, 0), H - 1);
							set(xi, yi);
						}
			}
		}
	int n = 0;
	for(uint8_t f : flags) n += f;
	return n;
}

static int renderImage(const yc_scene *s, int y0, int y1, float *out_rgba, float *out_w, yc_counters *ctr)
{
	Scene sc(*s);
	Renderer R(sc);
	if(!R.preprocessPhotons()) return -1;
	const yc_render &rp = sc.rp;
	const int W = rp.width, H = rp.height;
	if(y1 <= y0) { y0 = 0; y1 = H; }
	Film film(W, H, *sc.film, rp.clamp_samples);
	const int passes = std::max(1, rp.aa_passes);
	if(passes > 1 && (y0 != 0 || y1 != H)) return -2;   // adaptive passes need the whole film
	std::vector<Tile> all = tilesLinear(W, H, rp.tile_size);
	// imagesplitter.cc:30-107 tile order for one render thread: random (the reference seeds from
	// std::random_device; a fixed seed here and in the GPU host), centre (ImageSpliterCentreSorter,
	// imagesplitter.h:97-109: squared distance of the tile corner to the image centre; ties in
	// linear order, the reference breaks them randomly)
	if(rp.tiles_order == 2) std::shuffle(all.begin(), all.end(), std::mt19937(0x59414641u));
	else if(rp.tiles_order == 1)
		std::stable_sort(all.begin(), all.end(), [W, H](const Tile &a, const Tile &b) {
			return (a.x - W / 2) * (a.x - W / 2) + (a.y - H / 2) * (a.y - H / 2) < (b.x - W / 2) * (b.x - W / 2) + (b.y - H / 2) * (b.y - H / 2);
		});
	std::vector<Tile> tiles;
	for(size_t k = 0; k < all.size(); ++k)
	{
		const Tile &t = all[k];
		const int ya = std::max(t.y, y0), yb = std::min(t.y + t.h, y1);
		if(ya < yb) tiles.push_back({t.x, ya, t.w, yb - ya, (int)k});
	}
	// each tile's rand() in the one-thread render order (srand(1 + rr_seed))
	const std::vector<uint32_t> tile_rand = glibcRandSequence(1u + rp.rr_seed, all.size());
	const int nthreads = std::max(1, rp.threads);
	std::vector<Renderer::Thread> th(nthreads);
	std::vector<uint8_t> flags;   // imagefilm flags_ (adaptive passes)
	// renderPass (integrator_tiled.cc:236-267 / renderTile :269-345): tiles in parallel, each tile
	// sequential (reference renderWorker), then the film pass in linear tile order (reference
	// single-thread order), so the output is thread-count free.  `adaptive`: only flagged pixels.
	auto renderPass = [&](int n_samples, int pass_offs, bool adaptive) {
		const size_t band = 256;
		for(size_t t0 = 0; t0 < tiles.size(); t0 += band)
		{
			const size_t t1 = std::min(tiles.size(), t0 + band);
			std::vector<std::vector<float>> buf(t1 - t0);
			std::atomic<size_t> next{t0};
			auto worker = [&](int tid) {
				for(;;)
				{
					const size_t k = next++;
					if(k >= t1) break;
					const Tile &a = tiles[k];
					std::vector<float> &b = buf[k - t0];
					b.resize((size_t)a.w * a.h * n_samples * 4);
					// integrator_tiled.cc:272 — RandomGenerator(rand() + offset*(resx*y0+x0) + 123)
					Mwc rng(tile_rand[(size_t)a.rank] + pass_offs * (sc.cam.resx * a.y + a.x) + 123);
					for(int i = a.y; i < a.y + a.h; ++i)
						for(int j = a.x; j < a.x + a.w; ++j)
						{
							if(adaptive && !flags[(size_t)i * W + j]) continue;   // doMoreSamples (:290)
							R.renderPixel(th[tid], rng, i, j, &b[(((size_t)(i - a.y) * a.w + (j - a.x)) * n_samples) * 4], n_samples,
							              pass_offs);
						}
				}
			};
			if(nthreads == 1) worker(0);
			else
			{
				std::vector<std::thread> pool;
				for(int tt = 0; tt < nthreads; ++tt) pool.emplace_back(worker, tt);
				for(auto &p : pool) p.join();
			}
			for(size_t k = t0; k < t1; ++k)
			{
				const Tile &a = tiles[k];
				const std::vector<float> &b = buf[k - t0];
				for(int i = a.y; i < a.y + a.h; ++i)
					for(int j = a.x; j < a.x + a.w; ++j)
					{
						if(adaptive && !flags[(size_t)i * W + j]) continue;
						const uint32_t offset = fnv32(static_cast<uint32_t>(i + rp.crop_y0) * fnv32(static_cast<uint32_t>(j + rp.crop_x0)));
						for(int sample = 0; sample < n_samples; ++sample)
						{
							float dx, dy;
							sampleOffsets(passes, n_samples, sample, pass_offs + sample, offset, dx, dy);
							film.addSample(j, i, dx, dy, &b[((((size_t)(i - a.y) * a.w + (j - a.x)) * n_samples) + sample) * 4]);
						}
					}
			}
		}
	};
	// TiledIntegrator::render (integrator_tiled.cc:172-231)
	const int base = rp.base_sampling_offset;
	renderPass(rp.aa_samples, base, false);
	float threshold = rp.aa_threshold;
	float sample_multiplier = 1.f;
	bool threshold_changed = true;
	int acum = rp.aa_samples, resampled = 0;
	const int floor_pixels = (int)floorf(rp.aa_resampled_floor * (float)(W * H) / 100.f);
	for(int pass = 1; pass < passes; ++pass)
	{
		sample_multiplier *= rp.aa_sample_multiplier_factor;
		R.light_mult *= rp.aa_light_sample_multiplier_factor;   // integrator_tiled.cc:190
		R.indirect_mult *= rp.aa_indirect_sample_multiplier_factor;   // :191
		if(resampled <= 0.f && !threshold_changed) {}   // nextPass(..., skipNextPass = true): flags untouched
		else
		{
			resampled = aaNextPass(film, W, H, rp, threshold, flags);
			threshold_changed = false;
			if(const char *dump = getenv("YC_AA_DUMP"); dump && *dump)
				if(FILE *f = fopen((std::string(dump) + "_pass" + std::to_string(pass) + ".bin").c_str(), "wb"))
				{
					fwrite(flags.data(), 1, flags.size(), f);
					fclose(f);
				}
		}
		const int n_pass = (int)ceilf(rp.aa_inc_samples * sample_multiplier);
		if(resampled > 0) renderPass(n_pass, base + acum, true);
		acum += n_pass;
		if(resampled < floor_pixels)
		{
			const float ratio = std::min(8.f, ((float)floor_pixels / resampled));
			threshold *= (1.f - 0.1f * ratio);
			if(threshold > 0.f) threshold_changed = true;
		}
	}
	// imagefilm.cc:590-617 flush: Rgba::normalized (color.h:554-558) = colour * (1 / weight)
	// (operator/ takes the reciprocal first, color.h:312-316)
	for(size_t p = 0; p < (size_t)W * H; ++p)
	{
		const float wt = film.weight[p];
		const float inv = (wt != 0.f) ? 1.f / wt : 0.f;
		for(int k = 0; k < 4; ++k) out_rgba[4 * p + k] = (wt != 0.f) ? film.rgba[4 * p + k] * inv : 0.f;
		if(out_w) out_w[p] = wt;
	}
	if(ctr)
	{
		ctr->closest_rays = 0;
		ctr->shadow_rays = 0;
		for(const auto &t : th) { ctr->closest_rays += t.closest; ctr->shadow_rays += t.shadow; }
	}
	return 0;
}

} // namespace yc

using namespace yc;

extern "C" {

int yc_render_image(const yc_scene *scene, int y0, int y1, float *rgba, float *weights, yc_counters *counters)
{
	return renderImage(scene, y0, y1, rgba, weights, counters);
}

int yc_render_samples(const yc_scene *s, int n, const int *xys, float *rgba)
{
	Scene sc(*s);
	Renderer R(sc);
	if(!R.preprocessPhotons()) return -1;
	Renderer::Thread th;
	const yc_render &rp = sc.rp;
	const int spp = rp.aa_samples;
	const float d_1 = 1.f / static_cast<float>(spp);
	for(int k = 0; k < n; ++k)
	{
		const int j = xys[3 * k] + rp.crop_x0, i = xys[3 * k + 1] + rp.crop_y0, sample = xys[3 * k + 2];
		const uint32_t offset = fnv32(static_cast<uint32_t>(i) * fnv32(static_cast<uint32_t>(j)));
		float dx = 0.5f, dy = 0.5f;
		if(spp > 1)
		{
			dx = (0.5f + static_cast<float>(sample)) * d_1;
			dy = riLp(sample + offset);
		}
		Ray ray = R.shootRay(j + dx, i + dy);
		Mwc rng(rp.rr_seed + 123);
		C3 col;
		float alpha;
		const uint32_t sample_idx = rp.base_sampling_offset + sample;
		if(rp.integrator == YC_INT_PATH) R.integratePath(th, ray, rng, sample_idx, offset, col, alpha);
		else if(rp.integrator == YC_INT_PHOTON) R.integratePhoton(th, ray, rng, sample_idx, offset, col, alpha);
		else R.integrateDirect(th, ray, rng, sample_idx, offset, col, alpha);
		rgba[4 * k] = col.r; rgba[4 * k + 1] = col.g; rgba[4 * k + 2] = col.b; rgba[4 * k + 3] = std::min(alpha, 1.f);
	}
	return 0;
}

int yc_trace_closest(const yc_scene *s, int n, const float *rays, float *hit, int *prim)
{
	Scene sc(*s);
	for(int k = 0; k < n; ++k)
	{
		const float *r = rays + 8 * k;
		Ray ray;
		ray.from = V3(r[0], r[1], r[2]);
		ray.dir = V3(r[3], r[4], r[5]);
		ray.tmin = r[6];
		ray.tmax = r[7];
		const float t_max = (ray.tmax >= 0.f) ? ray.tmax : std::numeric_limits<float>::infinity();
		const IsectData d = sc.intersect(ray, t_max, false, nullptr);
		hit[4 * k] = d.hit ? d.t : -1.f;
		hit[4 * k + 1] = d.bu;
		hit[4 * k + 2] = d.bv;
		hit[4 * k + 3] = d.bw;
		prim[k] = d.hit ? d.prim : -1;
	}
	return 0;
}

int yc_trace_shadow(const yc_scene *s, int n, const float *rays, int *occluded)
{
	Scene sc(*s);
	for(int k = 0; k < n; ++k)
	{
		const float *r = rays + 8 * k;
		Ray ray;
		ray.from = V3(r[0], r[1], r[2]);
		ray.dir = V3(r[3], r[4], r[5]);
		ray.tmin = r[6];
		ray.tmax = r[7];
		const float t_max = (ray.tmax >= 0.f) ? ray.tmax : std::numeric_limits<float>::infinity();
		occluded[k] = sc.intersect(ray, t_max, true, nullptr).hit ? 1 : 0;
	}
	return 0;
}

void yc_riVdC(const uint32_t *bits, const uint32_t *r, float *out, int n) { for(int i = 0; i < n; ++i) out[i] = riVdC(bits[i], r[i]); }
void yc_riS(const uint32_t *bits, const uint32_t *r, float *out, int n) { for(int i = 0; i < n; ++i) out[i] = riS(bits[i], r[i]); }
void yc_riLp(const uint32_t *bits, const uint32_t *r, float *out, int n) { for(int i = 0; i < n; ++i) out[i] = riLp(bits[i], r[i]); }
void yc_fnv32(const uint32_t *in, uint32_t *out, int n) { for(int i = 0; i < n; ++i) out[i] = fnv32(in[i]); }
void yc_lds(const int *dim, const uint32_t *idx, double *out, int n) { for(int i = 0; i < n; ++i) out[i] = lowDiscrepancySampling(dim[i], idx[i]); }
void yc_halton_seq(int base, uint32_t start, int steps, float *out)
{
	Halton h(base, start);
	for(int i = 0; i < steps; ++i) out[i] = h.getNext();
}
void yc_sin(const float *x, float *out, int n) { for(int i = 0; i < n; ++i) out[i] = fsin(x[i]); }
void yc_cos(const float *x, float *out, int n) { for(int i = 0; i < n; ++i) out[i] = fcos(x[i]); }
void yc_exp(const float *x, float *out, int n) { for(int i = 0; i < n; ++i) out[i] = fexp(x[i]); }
void yc_cos_hemisphere(const float *p9, const float *s, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const float *p = p9 + 9 * i;
		const V3 r = cosHemisphere(V3(p[0], p[1], p[2]), V3(p[3], p[4], p[5]), V3(p[6], p[7], p[8]), s[2 * i], s[2 * i + 1]);
		out[3 * i] = r.x; out[3 * i + 1] = r.y; out[3 * i + 2] = r.z;
	}
}
void yc_coords_system(const float *in, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		V3 u, v;
		createCoordsSystem(V3(in[3 * i], in[3 * i + 1], in[3 * i + 2]), u, v);
		out[6 * i] = u.x; out[6 * i + 1] = u.y; out[6 * i + 2] = u.z;
		out[6 * i + 3] = v.x; out[6 * i + 4] = v.y; out[6 * i + 5] = v.z;
	}
}
void yc_normalize(const float *in, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		V3 v(in[3 * i], in[3 * i + 1], in[3 * i + 2]);
		v.normalize();
		out[3 * i] = v.x; out[3 * i + 1] = v.y; out[3 * i + 2] = v.z;
	}
}
// bound.h:141-211 (Smits)
void yc_bound_cross(const float *box, const float *ray, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const float *b = box + 6 * i, *r = ray + 7 * i;
		const V3 a0(b[0], b[1], b[2]), a1(b[3], b[4], b[5]);
		const V3 from(r[0], r[1], r[2]), dir(r[3], r[4], r[5]);
		const float t_max = r[6];
		const V3 p = from - a0;
		float lmin = -1e38f, lmax = 1e38f, ltmin, ltmax;
		bool ok = true;
		for(int k = 0; k < 3 && ok; ++k)
		{
			if(dir[k] != 0)
			{
				const float inv = 1.f / dir[k];
				if(inv > 0) { ltmin = -p[k] * inv; ltmax = ((a1[k] - a0[k]) - p[k]) * inv; }
				else { ltmin = ((a1[k] - a0[k]) - p[k]) * inv; ltmax = -p[k] * inv; }
				if(k == 0) { lmin = ltmin; lmax = ltmax; }
				else { lmin = std::max(ltmin, lmin); lmax = std::min(ltmax, lmax); }
				if((lmax < 0) || (lmin > t_max)) ok = false;
			}
		}
		if(ok && (lmin <= lmax) && (lmax >= 0) && (lmin <= t_max)) { out[3 * i] = 1.f; out[3 * i + 1] = lmin; out[3 * i + 2] = lmax; }
		else { out[3 * i] = 0.f; out[3 * i + 1] = 0.f; out[3 * i + 2] = 0.f; }
	}
}
void yc_mwc(uint32_t seed, int steps, double *out)
{
	Mwc m(seed);
	for(int i = 0; i < steps; ++i) out[i] = m();
}
void yc_filter_gauss(const float *dxdy, float *out, int n) { for(int i = 0; i < n; ++i) out[i] = filterGauss(dxdy[2 * i], dxdy[2 * i + 1]); }
void yc_round_to_int(const double *v, int *out, int n) { for(int i = 0; i < n; ++i) out[i] = roundToInt(v[i]); }
void yc_floor_to_int(const double *v, int *out, int n) { for(int i = 0; i < n; ++i) out[i] = floorToInt(v[i]); }
void yc_clamp_proportional(const float *rgb, float max_value, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		C3 c(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]);
		c.clampProportional(max_value);
		out[3 * i] = c.r; out[3 * i + 1] = c.g; out[3 * i + 2] = c.b;
	}
}
void yc_film_table(int filter, float filter_size, float *table, float *filterw, float *table_scale)
{
	FilmTable t(filter, filter_size);
	std::memcpy(table, t.table, sizeof(t.table));
	*filterw = t.filterw;
	*table_scale = t.table_scale;
}


// pinned against oracle/_ref ref_shirley_disk (vector.cc:127-160)
void yc_shirley_disk(const float *r12, float *uv, int n)
{
	for(int i = 0; i < n; ++i) shirleyDisk(r12[2 * i], r12[2 * i + 1], uv[2 * i], uv[2 * i + 1]);
}

// the RR tile seeds' generator on its own: the first n values glibc's rand() returns after
// srand(seed) (pinned against libc by tests/test_oracle_golden.py::test_glibc_rand_restatement)
void yc_glibc_rand(uint32_t seed, int n, uint32_t *out)
{
	const std::vector<uint32_t> v = glibcRandSequence(seed, n > 0 ? (size_t)n : 0);
	for(int i = 0; i < n; ++i) out[i] = v[(size_t)i];
}

// tile lists of renderImage (one render thread): order 0 linear, 1 centre, 2 random (fixed seed);
// out = (x, y, w, h) per tile, pinned against ref_tiles (imagesplitter.cc:30-107)
int yc_tiles(int w, int h, int bs, int order, int *out, int cap)
{
	std::vector<Tile> all = tilesLinear(w, h, bs);
	if(order == 2) std::shuffle(all.begin(), all.end(), std::mt19937(0x59414641u));
	else if(order == 1)
		std::stable_sort(all.begin(), all.end(), [w, h](const Tile &a, const Tile &b) {
			return (a.x - w / 2) * (a.x - w / 2) + (a.y - h / 2) * (a.y - h / 2) < (b.x - w / 2) * (b.x - w / 2) + (b.y - h / 2) * (b.y - h / 2);
		});
	int n = 0;
	for(const Tile &t : all)
	{
		if(n >= cap) break;
		out[4 * n] = t.x; out[4 * n + 1] = t.y; out[4 * n + 2] = t.w; out[4 * n + 3] = t.h;
		++n;
	}
	return n;
}

// which: 0 the diffuse map (PhotonIntegrator), 1 the caustic map, 2 the final-gather radiance map
int yc_photon_map_ex(const yc_scene *s, int which, float *pos, float *dir, float *col, uint32_t *nodes, int *n_paths)
{
	Scene sc(*s);
	Renderer R(sc);
	if(!R.preprocessPhotons()) return -1;
	const auto &M = which == 1 ? R.cmap : which == 2 ? R.rmap : R.dmap;
	const size_t n = M.photons.size();
	if(n_paths) *n_paths = M.n_paths;
	for(size_t i = 0; i < n; ++i)
	{
		const auto &p = M.photons[i];
		if(pos) { pos[3 * i] = p.pos.x; pos[3 * i + 1] = p.pos.y; pos[3 * i + 2] = p.pos.z; }
		if(dir) { dir[3 * i] = p.dir.x; dir[3 * i + 1] = p.dir.y; dir[3 * i + 2] = p.dir.z; }
		if(col) { col[3 * i] = p.col.r; col[3 * i + 1] = p.col.g; col[3 * i + 2] = p.col.b; }
	}
	if(nodes)
		for(size_t i = 0; i < M.nodes.size(); ++i) { nodes[2 * i] = M.nodes[i].data; nodes[2 * i + 1] = M.nodes[i].flags; }
	return (int)n;
}

int yc_photon_map(const yc_scene *s, float *pos, float *dir, float *col, uint32_t *nodes, int *n_paths)
{
	return yc_photon_map_ex(s, 0, pos, dir, col, nodes, n_paths);
}

// ---- texturing building blocks (yaftex.h), pinned against oracle/_ref ref_tex_* ----
// HDR pixels (format_hdr.cc via color.h:204-213), pinned against ref_rgbe_decode
void yc_rgbe_decode(const uint8_t *rgbe, float *rgb, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const yc::Rgba c = yc::rgbeToRgba(rgbe + 4 * i);
		rgb[3 * i] = c.r;
		rgb[3 * i + 1] = c.g;
		rgb[3 * i + 2] = c.b;
	}
}

void yc_tex_quantize(int kind, const float *in, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const yc::Rgba c(in[4 * i], in[4 * i + 1], in[4 * i + 2], in[4 * i + 3]);
		yc::Rgba r;
		switch(kind)
		{
			case 0: { yc::PxRgba1010108 p; p.set(c); r = p.get(); break; }
			case 1: { yc::PxRgb101010 p; p.set(c); r = p.get(); break; }
			case 2: { yc::PxRgba7773 p; p.set(c); r = p.get(); break; }
			case 3: { yc::PxRgb565 p; p.set(c); r = p.get(); break; }
			case 4: { yc::PxGray8 p; p.set(c); r = p.get(); break; }
			case 5: { yc::PxGray p; p.set(c); r = p.get(); break; }
			case 6: { yc::PxGrayAlpha p; p.set(c); r = p.get(); break; }
			default: { yc::PxRgbAlpha p; p.set(c); r = p.get(); break; }
		}
		out[4 * i] = r.r; out[4 * i + 1] = r.g; out[4 * i + 2] = r.b; out[4 * i + 3] = r.a;
	}
}

void yc_color_space(int dir, int cs, float gamma, const float *in, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		yc::Rgba c(in[3 * i], in[3 * i + 1], in[3 * i + 2], 1.f);
		if(dir == 0) yc::linearRgbFromColorSpace(c, cs, gamma);
		else yc::colorSpaceFromLinearRgb(c, cs, gamma);
		out[3 * i] = c.r; out[3 * i + 1] = c.g; out[3 * i + 2] = c.b;
	}
}

void yc_hsv_adjust(const float *in, const float *sat_hue, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		yc::Rgba c(in[3 * i], in[3 * i + 1], in[3 * i + 2], 1.f);
		float h = 0.f, s = 0.f, v = 0.f;
		yc::rgbToHsv(c, h, s, v);
		s *= sat_hue[2 * i];
		h += sat_hue[2 * i + 1];
		if(h < 0.f) h += 6.f;
		else if(h > 6.f) h -= 6.f;
		yc::hsvToRgb(c, h, s, v);
		out[3 * i] = c.r; out[3 * i + 1] = c.g; out[3 * i + 2] = c.b;
	}
}

void yc_cubic(const float *in, float *out, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const float *p = in + 17 * i;
		const yc::Rgba r = yc::OTexture::cubic(yc::Rgba(p[0], p[1], p[2], p[3]), yc::Rgba(p[4], p[5], p[6], p[7]),
		                                       yc::Rgba(p[8], p[9], p[10], p[11]), yc::Rgba(p[12], p[13], p[14], p[15]), p[16]);
		out[4 * i] = r.r; out[4 * i + 1] = r.g; out[4 * i + 2] = r.b; out[4 * i + 3] = r.a;
	}
}

void yc_pow(const float *ab, float *out, int n)
{
	for(int i = 0; i < n; ++i) out[i] = yc::fpow(ab[2 * i], ab[2 * i + 1]);
}

}
