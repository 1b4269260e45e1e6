// Surface attributes, image textures and shader-node programs for the GPU hot path.
//
// Restates, per hit point:
//   * TrianglePrimitive::getSurface (src/geometry/primitive/primitive_triangle.cc:97-176): the
//     barycentrics of the hit (recomputed from the ray exactly as intersect() did, :44-71),
//     orco point / normal, UV and the interpolated smooth normal;
//   * ImageTexture::getColor / getRawColor / getFloat (src/texture/texture_image.cc:46-235,
//     include/texture/texture.h:57) with Texture::applyAdjustments (src/texture/texture.cc:194-262);
//   * TextureMapperNode / ValueNode / MixNode (src/shader/shader_node_basic.cc:56-676) and
//     LayerNode (src/shader/shader_node_layer.cc:29-332), evaluated in dependency order.
// The image buffers' quantisation (image_buffers.h) happened on the host: texels hold getColor().
// Compiled -ffp-contract=off; every expression keeps the reference's operation order.
#pragma once

#include "devmath.h"
#include "devscene.h"

namespace yafamd
{

struct C4 { float r, g, b, a; };
YD V3 xyz4(const float4 &a) { return v3(a.x, a.y, a.z); }
YD C4 c4(float r, float g, float b, float a) { return {r, g, b, a}; }
YD C4 c4(float f) { return {f, f, f, f}; }   // explicit Rgba(float g): alpha = g too (color.h:149)
YD C4 operator+(C4 a, C4 b) { return {a.r + b.r, a.g + b.g, a.b + b.b, a.a + b.a}; }
YD C4 operator-(C4 a, C4 b) { return {a.r - b.r, a.g - b.g, a.b - b.b, a.a - b.a}; }
YD C4 operator*(float f, C4 c) { return {f * c.r, f * c.g, f * c.b, f * c.a}; }
YD C4 operator*(C4 a, C4 b) { return {a.r * b.r, a.g * b.g, a.b * b.b, a.a * b.a}; }
YD C4 ld4(const float *p) { return {p[0], p[1], p[2], p[3]}; }
YD C4 f4c(const float4 &v) { return {v.x, v.y, v.z, v.w}; }
YD float col2Bri(C4 c) { return (0.2126f * c.r + 0.7152f * c.g + 0.0722f * c.b); }   // color.h:61

// ---- FAST_MATH pow (include/math/math.h:96-178) ----
YD float fmPolyexp(float x)
{
	return x * (x * (x * (x * (x * 1.8775767e-3f + 8.9893397e-3f) + 5.5826318e-2f) + 2.4015361e-1f) + 6.9315308e-1f) + 9.9999994e-1f;
}
YD float fmExp2(float x)
{
	x = fminf(x, 129.00000f);
	x = fmaxf(x, -126.99999f);
	const int ipart = (int)(x - 0.5f);
	const float fpart = x - (float)ipart;
	const int ei = (ipart + 127) << 23;
	float e;
	__builtin_memcpy(&e, &ei, 4);
	return e * fmPolyexp(fpart);
}
YD float fmPolylog(float x)
{
	return x * (x * (x * (x * (x * -3.4436006e-2f + 3.1821337e-1f) + -1.2315303f) + 2.5988452f) + -3.3241990f) + 3.1157899f;
}
YD float fmLog2(float x)
{
	int i;
	__builtin_memcpy(&i, &x, 4);
	const float e = (float)(((i & 0x7F800000) >> 23) - 127);
	const int mi = (i & 0x7FFFFF) | 0x3f800000;
	float m;
	__builtin_memcpy(&m, &mi, 4);
	return fmPolylog(m) * (m - 1.0f) + e;
}
YD float fmPow(float a, float b) { return fmExp2((float)(fmLog2(a) * b)); }

// color.h:336-348, 379-405 (getRawColor re-encodes into the image's original colour space)
YD float sRgbFromLinear(float v)
{
	if(v <= 0.0031308f) return v * 12.92f;
	return (1.055f * fmPow(v, 0.416667f)) - 0.055f;
}
YD C4 colorSpaceFromLinear(C4 c, int cs, float gamma)
{
	if(cs == CS_SRGB)
	{
		c.r = sRgbFromLinear(c.r); c.g = sRgbFromLinear(c.g); c.b = sRgbFromLinear(c.b);
	}
	else if(cs == CS_XYZ_D65)
	{
		const float r = c.r, g = c.g, b = c.b;
		c.r = 0.412400f * r + 0.357600f * g + 0.180500f * b;
		c.g = 0.212600f * r + 0.715200f * g + 0.072200f * b;
		c.b = 0.019300f * r + 0.119200f * g + 0.950500f * b;
	}
	else if(cs == CS_RAW_MANUAL_GAMMA && gamma != 1.f)
	{
		if(gamma <= 0.f) gamma = 1.0e-2f;
		const float ig = 1.f / gamma;
		c.r = fmPow(c.r, ig); c.g = fmPow(c.g, ig); c.b = fmPow(c.b, ig);
	}
	return c;
}

YD void clampRgb0(C4 &c)
{
	if(c.r < 0.0) c.r = 0.0f;
	if(c.g < 0.0) c.g = 0.0f;
	if(c.b < 0.0) c.b = 0.0f;
}

// color.h:470-512
YD void rgbToHsv(C4 c, float &h, float &s, float &v)
{
	const float r_1 = fmaxf(c.r, 0.f), g_1 = fmaxf(c.g, 0.f), b_1 = fmaxf(c.b, 0.f);
	const float max_component = fmaxf(fmaxf(r_1, g_1), b_1);
	const float min_component = fminf(fminf(r_1, g_1), b_1);
	const float range = max_component - min_component;
	v = max_component;
	if(fabsf(range) < 1.0e-6f) { h = 0.f; s = 0.f; }
	else if(max_component == r_1) { h = fmodf((g_1 - b_1) / range, 6.f); s = range / fmaxf(v, 1.0e-6f); }
	else if(max_component == g_1) { h = ((b_1 - r_1) / range) + 2.f; s = range / fmaxf(v, 1.0e-6f); }
	else if(max_component == b_1) { h = ((r_1 - g_1) / range) + 4.f; s = range / fmaxf(v, 1.0e-6f); }
	else { h = 0.f; s = 0.f; v = 0.f; }
	if(h < 0.f) h += 6.f;
}
YD void hsvToRgb(C4 &c, float h, float s, float v)
{
	const float cc = v * s;
	const float x = cc * (1.f - fabsf(fmodf(h, 2.f) - 1.f));
	const float m = v - cc;
	float r_1 = 0.f, g_1 = 0.f, b_1 = 0.f;
	if(h >= 0.f && h < 1.f) { r_1 = cc; g_1 = x; b_1 = 0.f; }
	else if(h >= 1.f && h < 2.f) { r_1 = x; g_1 = cc; b_1 = 0.f; }
	else if(h >= 2.f && h < 3.f) { r_1 = 0.f; g_1 = cc; b_1 = x; }
	else if(h >= 3.f && h < 4.f) { r_1 = 0.f; g_1 = x; b_1 = cc; }
	else if(h >= 4.f && h < 5.f) { r_1 = x; g_1 = 0.f; b_1 = cc; }
	else if(h >= 5.f && h < 6.f) { r_1 = cc; g_1 = 0.f; b_1 = x; }
	c.r = r_1 + m;
	c.g = g_1 + m;
	c.b = b_1 + m;
}

// texture.cc:194-262
YD C4 applyIntensityContrast(const DevTexture &t, C4 c)
{
	if(!(t.flags & TEXF_ADJ)) return c;
	C4 ret = c;
	if(t.intensity != 1.f || t.contrast != 1.f)
	{
		ret.r = (c.r - 0.5f) * t.contrast + t.intensity - 0.5f;
		ret.g = (c.g - 0.5f) * t.contrast + t.intensity - 0.5f;
		ret.b = (c.b - 0.5f) * t.contrast + t.intensity - 0.5f;
	}
	if(t.flags & TEXF_CLAMP) clampRgb0(ret);
	return ret;
}
YD C4 applyColorAdjust(const DevTexture &t, C4 c)
{
	if(!(t.flags & TEXF_ADJ)) return c;
	C4 ret = c;
	if(t.fr != 1.f) ret.r *= t.fr;
	if(t.fg != 1.f) ret.g *= t.fg;
	if(t.fb != 1.f) ret.b *= t.fb;
	if(t.flags & TEXF_CLAMP) clampRgb0(ret);
	if(t.saturation != 1.f || t.hue != 0.f)
	{
		float h = 0.f, s = 0.f, v = 0.f;
		rgbToHsv(ret, h, s, v);
		s *= t.saturation;
		h += t.hue;
		if(h < 0.f) h += 6.f;
		else if(h > 6.f) h -= 6.f;
		hsvToRgb(ret, h, s, v);
		if(t.flags & TEXF_CLAMP) clampRgb0(ret);
	}
	return ret;
}
YD float applyIntensityContrastF(const DevTexture &t, float f)
{
	if(!(t.flags & TEXF_ADJ)) return f;
	float ret = f;
	if(t.intensity != 1.f || t.contrast != 1.f) ret = (f - 0.5f) * t.contrast + t.intensity - 0.5f;
	if(t.flags & TEXF_CLAMP)
	{
		if(ret < 0.f) ret = 0.f;
		else if(ret > 1.f) ret = 1.f;
	}
	return ret;
}

// texture_image.cc:99-171 (returns `outside`)
YD bool texDoMapping(const DevTexture &t, V3 &p)
{
	bool outside = false;
	p = v3(0.5f * p.x + 0.5f, 0.5f * p.y + 0.5f, 0.5f * p.z + 0.5f);
	if(t.clip == CLIP_REPEAT)
	{
		if(t.xrep > 1) p.x *= (float)t.xrep;
		if(t.yrep > 1) p.y *= (float)t.yrep;
		if((t.flags & TEXF_MIRROR_X) && (int)ceilf(p.x) % 2 == 0) p.x = -p.x;
		if((t.flags & TEXF_MIRROR_Y) && (int)ceilf(p.y) % 2 == 0) p.y = -p.y;
		if(p.x > 1.f) p.x -= (float)(int)p.x;
		else if(p.x < 0.f) p.x += (float)(1 - (int)p.x);
		if(p.y > 1.f) p.y -= (float)(int)p.y;
		else if(p.y < 0.f) p.y += (float)(1 - (int)p.y);
	}
	if(t.flags & TEXF_CROPX) p.x = t.cropminx + p.x * (t.cropmaxx - t.cropminx);
	if(t.flags & TEXF_CROPY) p.y = t.cropminy + p.y * (t.cropmaxy - t.cropminy);
	if(t.flags & TEXF_ROT90) { const float tmp = p.x; p.x = p.y; p.y = tmp; }
	switch(t.clip)
	{
		case CLIP_CLIPCUBE:
			if((p.x < 0) || (p.x > 1) || (p.y < 0) || (p.y > 1) || (p.z < -1) || (p.z > 1)) outside = true;
			break;
		case CLIP_CHECKER:
		{
			const int xs = (int)floorf(p.x), ys = (int)floorf(p.y);
			p.x -= (float)xs;
			p.y -= (float)ys;
			if(!(t.flags & TEXF_CHECK_ODD) && !((xs + ys) & 1)) { outside = true; break; }
			if(!(t.flags & TEXF_CHECK_EVEN) && ((xs + ys) & 1)) { outside = true; break; }
			if(t.checker_dist < 1.0)
			{
				p.x = (p.x - 0.5f) / (1.f - t.checker_dist) + 0.5f;
				p.y = (p.y - 0.5f) / (1.f - t.checker_dist) + 0.5f;
			}
		}
		// fall through (texture_image.cc:152 "continue to TCL_CLIP")
		case CLIP_CLIP:
			if((p.x < 0) || (p.x > 1) || (p.y < 0) || (p.y > 1)) outside = true;
			break;
		case CLIP_EXTEND:
			if(p.x > 0.99999f) p.x = 0.99999f; else if(p.x < 0) p.x = 0;
			if(p.y > 0.99999f) p.y = 0.99999f; else if(p.y < 0) p.y = 0;
			// fall through
		default:
			outside = false;
			break;
	}
	return outside;
}

// texture_image.cc:181-235
YD void interpCoords(int &c_0, int &c_1, int &c_2, int &c_3, float &dec, float cf, int res, bool repeat, bool mirror)
{
	if(repeat)
	{
		c_1 = ((int)cf) % res;
		if(mirror)
		{
			if(cf < 0.f)
			{
				c_0 = 1 % res;
				c_2 = c_1;
				c_3 = c_0;
				dec = -cf;
			}
			else if(cf >= (float)(res - 1))
			{
				c_0 = (2 * res - 1) % res;
				c_2 = c_1;
				c_3 = c_0;
				dec = cf - (float)((int)cf);
			}
			else
			{
				c_0 = (res + c_1 - 1) % res;
				c_2 = c_1 + 1;
				if(c_2 >= res) c_2 = (2 * res - c_2) % res;
				c_3 = c_1 + 2;
				if(c_3 >= res) c_3 = (2 * res - c_3) % res;
				dec = cf - (float)((int)cf);
			}
		}
		else
		{
			if(cf > 0.f)
			{
				c_0 = (res + c_1 - 1) % res;
				c_2 = (c_1 + 1) % res;
				c_3 = (c_1 + 2) % res;
				dec = cf - (float)((int)cf);
			}
			else
			{
				c_0 = 1 % res;
				c_2 = (res - 1) % res;
				c_3 = (res - 2) % res;
				dec = -cf;
			}
		}
	}
	else
	{
		c_1 = max(0, min(res - 1, (int)cf));
		if(cf > 0.f) c_2 = min(res - 1, c_1 + 1);
		else c_2 = 0;
		c_0 = max(0, c_1 - 1);
		c_3 = min(res - 1, c_2 + 1);
		dec = cf - floorf(cf);
	}
}

YD C4 texel(const float4 *px, const DevTexture &t, int x, int y) { return f4c(px[t.texel0 + (uint32_t)y * (uint32_t)t.w + (uint32_t)x]); }

// math/interpolation.h:69-80
YD C4 cubicInterp(C4 y_0, C4 y_1, C4 y_2, C4 y_3, float x)
{
	const float x_squared = x * x;
	const float x_cubed = x * x_squared;
	const C4 a_0 = y_3 - y_2 - y_0 + y_1;
	const C4 a_1 = y_0 - y_1 - a_0;
	const C4 a_2 = y_2 - y_0;
	const C4 a_3 = y_1;
	return x_cubed * a_0 + x_squared * a_1 + x * a_2 + a_3;
}

// texture_image.cc:237-343
YD C4 texInterpolate(const float4 *px, const DevTexture &t, V3 p)
{
	const int resx = t.w, resy = t.h;
	const float half = t.interp == INTERP_NONE ? 0.f : 0.5f;
	const float xf = ((float)resx * (p.x - floorf(p.x))) - half;
	const float yf = ((float)resy * (p.y - floorf(p.y))) - half;
	int x_0, x_1, x_2, x_3, y_0, y_1, y_2, y_3;
	float dx, dy;
	const bool rep = t.clip == CLIP_REPEAT;
	interpCoords(x_0, x_1, x_2, x_3, dx, xf, resx, rep, (t.flags & TEXF_MIRROR_X) != 0);
	interpCoords(y_0, y_1, y_2, y_3, dy, yf, resy, rep, (t.flags & TEXF_MIRROR_Y) != 0);
	if(t.interp == INTERP_NONE) return texel(px, t, x_1, y_1);
	if(t.interp == INTERP_BILINEAR)
	{
		const C4 c_11 = texel(px, t, x_1, y_1);
		const C4 c_21 = texel(px, t, x_2, y_1);
		const C4 c_12 = texel(px, t, x_1, y_2);
		const C4 c_22 = texel(px, t, x_2, y_2);
		const float w_11 = (1 - dx) * (1 - dy);
		const float w_12 = (1 - dx) * dy;
		const float w_21 = dx * (1 - dy);
		const float w_22 = dx * dy;
		return (w_11 * c_11) + (w_12 * c_12) + (w_21 * c_21) + (w_22 * c_22);
	}
	const int xs[4] = {x_0, x_1, x_2, x_3};
	C4 cy[4];
	for(int j = 0; j < 4; ++j)
	{
		const int yy = j == 0 ? y_0 : j == 1 ? y_1 : j == 2 ? y_2 : y_3;
		cy[j] = cubicInterp(texel(px, t, xs[0], yy), texel(px, t, xs[1], yy), texel(px, t, xs[2], yy), texel(px, t, xs[3], yy), dx);
	}
	return cubicInterp(cy[0], cy[1], cy[2], cy[3], dy);
}

// texture_image.cc:72-80 (ImageTexture::getColor)
YD C4 texGetColor(const float4 *px, const DevTexture &t, V3 p)
{
	V3 p_1 = v3(p.x, -p.y, p.z);
	if(texDoMapping(t, p_1)) return c4(0.f);
	const C4 ret = texInterpolate(px, t, p_1);
	return applyColorAdjust(t, applyIntensityContrast(t, ret));
}

// texture.h:57: applyIntensityContrastAdjustments(getRawColor(p).col2Bri())
YD float texGetFloat(const float4 *px, const DevTexture &t, V3 p)
{
	const C4 raw = colorSpaceFromLinear(texGetColor(px, t, p), t.raw_cs, t.raw_gamma);
	return applyIntensityContrastF(t, col2Bri(raw));
}

// ---- TextureMapperNode (shader_node_basic.cc:56-137) ----
YD V3 mapTube(V3 p)
{
	V3 res;
	res.y = p.z;
	const float d = p.x * p.x + p.y * p.y;
	if(d > 0.f)
	{
		res.z = 1.f / sqrtf(d);
		res.x = x87mul(kDiv1ByPi, -libmAtan2f(p.x, p.y));
	}
	else res.x = res.z = 0.f;
	return res;
}
YD V3 mapSphere(V3 p)
{
	V3 res = v3(0.f, 0.f, 0.f);
	const float d = p.x * p.x + p.y * p.y + p.z * p.z;
	if(d > 0.f)
	{
		res.z = sqrtf(d);
		if((p.x != 0.f) && (p.y != 0.f)) res.x = x87mul(kDiv1ByPi, -libmAtan2f(p.x, p.y));
		// math.h:252-258 acos with the domain clamp (libm's acosf, restated in devmath.h), then
		// 1.f - 2.f * (acos * div_1_by_pi) with the long double product and difference (x87oneMinus2Mul)
		const float q = p.z / res.z;
		const float ac = (q <= -1.f) ? kPiF : (q >= 1.f) ? 0.f : libmAcosf(q);
		res.y = x87oneMinus2Mul(kDiv1ByPi, ac);
	}
	return res;
}
YD V3 mapCube(V3 p, V3 n)
{
	int axis;
	if(fabsf(n.z) >= fabsf(n.x) && fabsf(n.z) >= fabsf(n.y)) axis = 2;
	else if(fabsf(n.y) >= fabsf(n.x) && fabsf(n.y) >= fabsf(n.z)) axis = 1;
	else axis = 0;
	if(axis == 0) return v3(p.y, p.z, p.x);
	if(axis == 1) return v3(p.x, p.z, p.y);
	return p;
}
YD float comp(V3 p, int k) { return k == 0 ? p.x : k == 1 ? p.y : p.z; }
YD V3 texMapping(const DevNode &nd, V3 p, V3 n)
{
	V3 tp = p;
	if(nd.coords == TC_UV) tp = v3(2.f * tp.x - 1.f, 2.f * tp.y - 1.f, tp.z);
	const float tm[4] = {0.f, tp.x, tp.y, tp.z};
	tp = v3(tm[nd.map_x], tm[nd.map_y], tm[nd.map_z]);
	if(nd.proj == PROJ_TUBE) tp = mapTube(tp);
	else if(nd.proj == PROJ_SPHERE) tp = mapSphere(tp);
	else if(nd.proj == PROJ_CUBE) tp = mapCube(tp, n);
	// Point3::mult(texpt, scale_) + offset_
	return v3(tp.x * nd.scale[0] + nd.offset[0], tp.y * nd.scale[1] + nd.offset[1], tp.z * nd.scale[2] + nd.offset[2]);
}

// The surface values the node tree and the materials read (SurfacePoint subset)
struct SurfAttr
{
	V3 p, ng, n;           // hit point, geometric normal, shading normal
	V3 orco_p, orco_ng;
	float u, v;
};

// Matrix4 * Point3 / Matrix4 * Vec3 (include/geometry/matrix.h)
YD V3 mtxPoint(const float *m, V3 p)
{
	return v3(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3], m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7],
	          m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11]);
}
YD V3 mtxVec(const float *m, V3 v)
{
	return v3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z, m[8] * v.x + m[9] * v.y + m[10] * v.z);
}

// ---- LayerNode blends (shader_node_layer.cc:187-285) on Rgb ----
YD C3 blendRgb(C3 tex, C3 out, float fact, float facg, int mode)
{
	switch(mode)
	{
		case BLEND_MULT:
			fact *= facg;
			return (c3(1.f - facg) + fact * tex) * out;
		case BLEND_SCREEN:
		{
			const C3 white = c3(1.0f);
			fact *= facg;
			const C3 wt = C3{white.r - tex.r, white.g - tex.g, white.b - tex.b};
			const C3 wo = C3{white.r - out.r, white.g - out.g, white.b - out.b};
			const C3 k = (c3(1.f - facg) + fact * wt) * wo;
			return C3{white.r - k.r, white.g - k.g, white.b - k.b};
		}
		case BLEND_SUB:
			fact = -fact;
			// fall through
		case BLEND_ADD:
			fact *= facg;
			return fact * tex + out;
		case BLEND_DIV:
		{
			fact *= facg;
			C3 itex = tex;
			if(itex.r != 0.f) itex.r = 1.f / itex.r;
			if(itex.g != 0.f) itex.g = 1.f / itex.g;
			if(itex.b != 0.f) itex.b = 1.f / itex.b;
			return (1.f - fact) * out + fact * out * itex;
		}
		case BLEND_DIFF:
		{
			fact *= facg;
			const C3 tmo = C3{fabsf(tex.r - out.r), fabsf(tex.g - out.g), fabsf(tex.b - out.b)};
			return (1.f - fact) * out + fact * tmo;
		}
		case BLEND_DARK:
		{
			fact *= facg;
			C3 col = fact * tex;
			if(col.r > out.r) col.r = out.r;
			if(col.g > out.g) col.g = out.g;
			if(col.b > out.b) col.b = out.b;
			return col;
		}
		case BLEND_LIGHT:
		{
			fact *= facg;
			C3 col = fact * tex;
			if(col.r < out.r) col.r = out.r;
			if(col.g < out.g) col.g = out.g;
			if(col.b < out.b) col.b = out.b;
			return col;
		}
		default:
			fact *= facg;
			return fact * tex + (1.f - fact) * out;
	}
}
YD float blendValue(float tex, float out, float fact, float facg, int mode)
{
	fact *= facg;
	float facm = 1.f - fact;
	switch(mode)
	{
		case BLEND_MULT:
			facm = 1.f - facg;
			return (facm + fact * tex) * out;
		case BLEND_SCREEN:
			facm = 1.f - facg;
			return 1.f - (facm + fact * (1.f - tex)) * (1.f - out);
		case BLEND_SUB:
			fact = -fact;
			// fall through
		case BLEND_ADD:
			return fact * tex + out;
		case BLEND_DIV:
			if(tex == 0.f) return 0.f;
			return facm * out + fact * out / tex;
		case BLEND_DIFF:
			return facm * out + fact * fabsf(tex - out);
		case BLEND_DARK:
		{
			const float col = fact * tex;
			if(col < out) return col;
			return out;
		}
		case BLEND_LIGHT:
		{
			const float col = fact * tex;
			if(col > out) return col;
			return out;
		}
		default:
			return fact * tex + facm * out;
	}
}

// Evaluates the material's node program at the surface point; returns the diffuse shader colour
// (Rgb of its getColor) and the diffuse_refl_shader scalar (1 when absent).
YD void evalNodes(const DevMaterial &m, const DevNode *nodes, const DevTexture *texs, const float4 *px,
                  const SurfAttr &sa, C3 &dcol, float &drefl, float &sigma)
{
	C4 rc[kMaxNodes];
	float rv[kMaxNodes];
	const int n = min(m.n_nodes, kMaxNodes);
	for(int k = 0; k < n; ++k)
	{
		const DevNode &nd = nodes[m.node0 + k];
		C4 col = c4(0.f);
		float val = 0.f;
		if(nd.type == NODE_VALUE)
		{
			col = ld4(nd.c0);
			val = nd.f[0];
		}
		else if(nd.type == NODE_TEXMAP)
		{
			// getCoords (:138-163) + doMapping (:106-133); no ray differentials (bilinear/bicubic/none)
			V3 tp, ng;
			if(nd.coords == TC_UV) { tp = v3(sa.u, sa.v, 0.f); ng = sa.ng; }
			else if(nd.coords == TC_ORCO) { tp = sa.orco_p; ng = sa.orco_ng; }
			else if(nd.coords == TC_TRANSFORMED) { tp = mtxPoint(nd.mtx, sa.p); ng = mtxVec(nd.mtx, sa.ng); }
			else { tp = sa.p; ng = sa.ng; }
			tp = texMapping(nd, tp, ng);
			const DevTexture &t = texs[nd.tex];
			col = texGetColor(px, t, tp);
			val = (nd.flags & 1u) ? texGetFloat(px, t, tp) : 0.f;
		}
		else if(nd.type == NODE_MIX)
		{
			// shader_node_basic.cc:406-430 getInputs + the variant's eval
			const float f_2 = nd.in[2] >= 0 ? rv[nd.in[2]] : nd.f[0];
			C4 cin_1 = nd.in[0] >= 0 ? rc[nd.in[0]] : ld4(nd.c0);
			float fin_1 = nd.in[0] >= 0 ? rv[nd.in[0]] : nd.f[1];
			C4 cin_2 = nd.in[1] >= 0 ? rc[nd.in[1]] : ld4(nd.c1);
			float fin_2 = nd.in[1] >= 0 ? rv[nd.in[1]] : nd.f[2];
			const float f_1 = 1.f - f_2;
			switch(nd.mode)
			{
				case BLEND_ADD: col = cin_1 + f_2 * cin_2; val = fin_1 + f_2 * fin_2; break;
				case BLEND_MULT:
					// MultNode (:472-484) multiplies fin_2, not fin_1, and returns fin_1
					col = cin_1 * (c4(f_1) + f_2 * cin_2);
					val = fin_1;
					break;
				case BLEND_SUB: col = cin_1 - f_2 * cin_2; val = fin_1 - f_2 * fin_2; break;
				case BLEND_SCREEN:
					col = c4(1.f) - (c4(f_1) + f_2 * (c4(1.f) - cin_2)) * (c4(1.f) - cin_1);
					val = 1.f - (f_1 + f_2 * (1.f - fin_2)) * (1.f - fin_1);
					break;
				case BLEND_DIFF:
					col = c4(f_1 * cin_1.r + f_2 * fabsf(cin_1.r - cin_2.r), f_1 * cin_1.g + f_2 * fabsf(cin_1.g - cin_2.g),
					         f_1 * cin_1.b + f_2 * fabsf(cin_1.b - cin_2.b), f_1 * cin_1.a + f_2 * fabsf(cin_1.a - cin_2.a));
					val = f_1 * fin_1 + f_2 * fabsf(fin_1 - fin_2);
					break;
				case BLEND_DARK:
				case BLEND_LIGHT:
				{
					const bool dark = nd.mode == BLEND_DARK;
					cin_2 = f_2 * cin_2;
					if(dark ? cin_2.r < cin_1.r : cin_2.r > cin_1.r) cin_1.r = cin_2.r;
					if(dark ? cin_2.g < cin_1.g : cin_2.g > cin_1.g) cin_1.g = cin_2.g;
					if(dark ? cin_2.b < cin_1.b : cin_2.b > cin_1.b) cin_1.b = cin_2.b;
					if(dark ? cin_2.a < cin_1.a : cin_2.a > cin_1.a) cin_1.a = cin_2.a;
					fin_2 *= f_2;
					if(dark ? fin_2 < fin_1 : fin_2 > fin_1) fin_1 = fin_2;
					col = cin_1;
					val = fin_1;
					break;
				}
				case BLEND_OVERLAY:
				{
					auto ov = [&](float a, float b) { return (a < 0.5f) ? a * (f_1 + 2.f * f_2 * b) : 1.f - (f_1 + 2.f * f_2 * (1.f - b)) * (1.f - a); };
					col = c4(ov(cin_1.r, cin_2.r), ov(cin_1.g, cin_2.g), ov(cin_1.b, cin_2.b), ov(cin_1.a, cin_2.a));
					val = ov(fin_1, fin_2);
					break;
				}
				default:
					col = f_1 * cin_1 + f_2 * cin_2;
					val = f_1 * fin_1 + f_2 * fin_2;
					break;
			}
		}
		else if(nd.type == NODE_LAYER)
		{
			// shader_node_layer.cc:29-112
			const uint32_t fl = nd.flags;
			C4 texcolor = c4(0.f, 0.f, 0.f, 1.f);
			float tin = 0.f, ta = 1.f;
			C4 rcol = nd.in[1] >= 0 ? rc[nd.in[1]] : ld4(nd.c1);
			float rval = nd.in[1] >= 0 ? rv[nd.in[1]] : nd.f[3];
			float stencil_tin = rcol.a;
			bool tex_rgb = (fl & LAYER_COLOR_INPUT) != 0;
			if(fl & LAYER_COLOR_INPUT)
			{
				texcolor = rc[nd.in[0]];
				ta = texcolor.a;
			}
			else tin = rv[nd.in[0]];
			if(fl & LAYER_RGB_TO_INT)
			{
				tin = col2Bri(texcolor);
				tex_rgb = false;
			}
			if(fl & LAYER_NEGATIVE)
			{
				if(tex_rgb) texcolor = c4(1.f) - texcolor;
				tin = 1.f - tin;
			}
			if(fl & LAYER_STENCIL)
			{
				if(tex_rgb)
				{
					const float fact = ta;
					ta *= stencil_tin;
					stencil_tin *= fact;
				}
				else
				{
					const float fact = tin;
					tin *= stencil_tin;
					stencil_tin *= fact;
				}
			}
			if(fl & LAYER_DO_COLOR)
			{
				if(!tex_rgb) texcolor = ld4(nd.c0);
				else tin = ta;
				float tin_tr;
				if(tin > 1.f) tin_tr = 1.f;
				else if(tin < 0.f) tin_tr = 0.f;
				else tin_tr = tin;
				const C3 b = blendRgb(C3{texcolor.r, texcolor.g, texcolor.b}, C3{rcol.r, rcol.g, rcol.b}, tin_tr, stencil_tin * nd.f[0], nd.mode);
				rcol = c4(b.r, b.g, b.b, 1.f);
				clampRgb0(rcol);
			}
			if(fl & LAYER_DO_SCALAR)
			{
				if(tex_rgb)
				{
					if(fl & LAYER_USE_ALPHA)
					{
						tin = ta;
						if(fl & LAYER_NEGATIVE) tin = 1.f - tin;
					}
					else tin = col2Bri(texcolor);
				}
				rval = blendValue(nd.f[2], rval, tin, stencil_tin * nd.f[1], nd.mode);
				if(rval < 0.f) rval = 0.f;
			}
			rcol.a = stencil_tin;
			col = rcol;
			val = rval;
		}
		rc[k] = col;
		rv[k] = val;
	}
	if(m.diffuse_root >= 0) { const C4 c = rc[m.diffuse_root]; dcol = C3{c.r, c.g, c.b}; }
	else dcol = C3{m.diffuse[0], m.diffuse[1], m.diffuse[2]};
	drefl = m.drefl_root >= 0 ? rv[m.drefl_root] : 1.f;
	sigma = m.sigma_root >= 0 ? rv[m.sigma_root] : 0.f;   // getShaderScalar(sigma_oren_shader_, ..., 0.f)
}

// primitive_triangle.cc:44-71 barycentrics of the (already found) hit + getSurface :97-176
YD SurfAttr surfAttr(const float4 *attr, const float4 *prim_ng, int prim, V3 o, V3 d, V3 p)
{
	const float4 *a = attr + (size_t)prim * kAttrF4;
	const float4 a0 = a[0];
	const uint32_t fl = __float_as_uint(a0.w);
	const V3 v0 = v3(a0.x, a0.y, a0.z), e1 = xyz4(a[1]), e2 = xyz4(a[2]);
	const V3 pvec = cross(d, e2);
	const float det = dot(e1, pvec);
	const float inv_det = 1.f / det;
	const V3 tvec = o - v0;
	const float u = dot(tvec, pvec) * inv_det;
	const V3 qvec = cross(tvec, e1);
	const float v = dot(d, qvec) * inv_det;
	const float bu = 1.f - u - v, bv = u, bw = v;
	SurfAttr s;
	s.p = p;
	s.ng = xyz4(prim_ng[prim]);
	if(fl & ATTR_SMOOTH)
	{
		const V3 n0 = xyz4(a[8]), n1 = xyz4(a[9]), n2 = xyz4(a[10]);
		s.n = normalize(bu * n0 + bv * n1 + bw * n2);
	}
	else s.n = s.ng;
	if(fl & ATTR_ORCO)
	{
		const V3 o0 = xyz4(a[3]), o1 = xyz4(a[4]), o2 = xyz4(a[5]);
		s.orco_p = bu * o0 + bv * o1 + bw * o2;
		s.orco_ng = normalize(cross(o1 - o0, o2 - o0));
	}
	else
	{
		s.orco_p = p;
		s.orco_ng = s.ng;
	}
	if(fl & ATTR_UV)
	{
		const float4 uv01 = a[6], uv2 = a[7];
		s.u = bu * uv01.x + bv * uv01.z + bw * uv2.x;
		s.v = bu * uv01.y + bv * uv01.w + bw * uv2.y;
	}
	else
	{
		s.u = bu;
		s.v = bv;
	}
	return s;
}

} // namespace yafamd
