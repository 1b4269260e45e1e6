// TEST INFRASTRUCTURE ONLY — oracle restatement of libYafaRay's texturing path: image loading
// (TGA, Radiance HDR), the image buffer types' storage, ImageTexture lookups, the shader nodes
// (texture_mapper / value / mix / layer), TrianglePrimitive::getSurface's surface attributes
// (orco, uv, smooth normals) and MeshObject::smoothNormals.  Included by yafcpu.cc after its math /
// V3 / C3 section; written scalar and close to the reference's own class structure.
//
// Reference files (paths relative to the reference root): src/format/format_tga.cc,
// include/format/format_tga_util.h, src/format/format_hdr.cc, include/format/format_hdr_util.h,
// src/image/image.cc, include/image/image_buffers.h, include/image/image_*.h,
// include/color/color.h, include/math/interpolation.h, src/texture/texture.cc,
// src/texture/texture_image.cc, src/shader/shader_node_basic.cc, src/shader/shader_node_layer.cc,
// src/geometry/primitive/primitive_triangle.cc, src/geometry/object/object_mesh.cc.

// ---------------------------------------------------------------------------------------------
// FAST_MATH log2 / pow (include/math/math.h:127-178)
// ---------------------------------------------------------------------------------------------
static inline float polylog(float x)
{
	return x * (x * (x * (x * (x * -3.4436006e-2f + 3.1821337e-1f) + -1.2315303f) + 2.5988452f) + -3.3241990f) + 3.1157899f;
}
static inline float flog2(float x)
{
	BitTw one, i, m, e;
	one.f = 1.0f;
	i.f = x;
	e.f = static_cast<float>(((i.i & 0x7F800000) >> 23) - 127);
	m.i = (i.i & 0x7FFFFF) | one.i;
	return polylog(m.f) * (m.f - one.f) + e.f;
}
static inline float fpow(float a, float b) { return fexp2(static_cast<float>(flog2(a) * b)); }

// math.h:252-266 (domain-clamped acos / asin)
static inline float facos(float x)
{
	if(x <= -1.f) return static_cast<float>(num_pi);
	else if(x >= 1.f) return 0.f;
	return std::acos(x);
}
static inline float fasin(float x)
{
	if(x <= -1.f) return static_cast<float>(-div_pi_by_2);
	else if(x >= 1.f) return static_cast<float>(div_pi_by_2);
	return std::asin(x);
}

// ---------------------------------------------------------------------------------------------
// Rgba (include/color/color.h:142-330)
// ---------------------------------------------------------------------------------------------
struct Rgba
{
	float r = 0.f, g = 0.f, b = 0.f, a = 1.f;
	Rgba() = default;
	Rgba(float r_, float g_, float b_, float a_ = 1.f) : r(r_), g(g_), b(b_), a(a_) {}
	explicit Rgba(float v) : r(v), g(v), b(v), a(v) {}
	float col2Bri() const { return (0.2126f * r + 0.7152f * g + 0.0722f * b); }
	void clampRgb0()
	{
		if(r < 0.0) r = 0.0;
		if(g < 0.0) g = 0.0;
		if(b < 0.0) b = 0.0;
	}
};
static inline Rgba operator+(const Rgba &x, const Rgba &y) { return {x.r + y.r, x.g + y.g, x.b + y.b, x.a + y.a}; }
static inline Rgba operator-(const Rgba &x, const Rgba &y) { return {x.r - y.r, x.g - y.g, x.b - y.b, x.a - y.a}; }
static inline Rgba operator*(const Rgba &x, const Rgba &y) { return {x.r * y.r, x.g * y.g, x.b * y.b, x.a * y.a}; }
static inline Rgba operator*(float f, const Rgba &c) { return {f * c.r, f * c.g, f * c.b, f * c.a}; }
static inline Rgba operator*(const Rgba &c, float f) { return {f * c.r, f * c.g, f * c.b, f * c.a}; }

// color.h:336-380 linearRgbFromColorSpace / colorSpaceFromLinearRgb (ColorSpace numbering :36)
enum { CsRawManualGamma = 1, CsLinearRgb = 2, CsSrgb = 3, CsXyzD65 = 4 };
static inline float linearRgbFromSRgb(float v)
{
	if(v <= 0.04045f) return (v / 12.92f);
	return fpow(((v + 0.055f) / 1.055f), 2.4f);
}
static inline float sRgbFromLinearRgb(float v)
{
	if(v <= 0.0031308f) return (v * 12.92f);
	return ((1.055f * fpow(v, 0.416667f)) - 0.055f);
}
static inline void linearRgbFromColorSpace(Rgba &c, int cs, float gamma)
{
	if(cs == CsSrgb)
	{
		c.r = linearRgbFromSRgb(c.r);
		c.g = linearRgbFromSRgb(c.g);
		c.b = linearRgbFromSRgb(c.b);
	}
	else if(cs == CsXyzD65)
	{
		static const float m[3][3] = {{3.2406255f, -1.537208f, -0.4986286f}, {-0.9689307f, 1.8757561f, 0.0415175f}, {0.0557101f, -0.2040211f, 1.0569959f}};
		const float o[3] = {c.r, c.g, c.b};
		c.r = m[0][0] * o[0] + m[0][1] * o[1] + m[0][2] * o[2];
		c.g = m[1][0] * o[0] + m[1][1] * o[1] + m[1][2] * o[2];
		c.b = m[2][0] * o[0] + m[2][1] * o[1] + m[2][2] * o[2];
	}
	else if(cs == CsRawManualGamma && gamma != 1.f)
	{
		c.r = fpow(c.r, gamma);
		c.g = fpow(c.g, gamma);
		c.b = fpow(c.b, gamma);
	}
}
static inline void colorSpaceFromLinearRgb(Rgba &c, int cs, float gamma)
{
	if(cs == CsSrgb)
	{
		c.r = sRgbFromLinearRgb(c.r);
		c.g = sRgbFromLinearRgb(c.g);
		c.b = sRgbFromLinearRgb(c.b);
	}
	else if(cs == CsXyzD65)
	{
		static const float m[3][3] = {{0.412400f, 0.357600f, 0.180500f}, {0.212600f, 0.715200f, 0.072200f}, {0.019300f, 0.119200f, 0.950500f}};
		const float o[3] = {c.r, c.g, c.b};
		c.r = m[0][0] * o[0] + m[0][1] * o[1] + m[0][2] * o[2];
		c.g = m[1][0] * o[0] + m[1][1] * o[1] + m[1][2] * o[2];
		c.b = m[2][0] * o[0] + m[2][1] * o[1] + m[2][2] * o[2];
	}
	else if(cs == CsRawManualGamma && gamma != 1.f)
	{
		if(gamma <= 0.f) gamma = 1.0e-2f;
		const float inv_gamma = 1.f / gamma;
		c.r = fpow(c.r, inv_gamma);
		c.g = fpow(c.g, inv_gamma);
		c.b = fpow(c.b, inv_gamma);
	}
}

// color.h:470-512
static inline void rgbToHsv(const Rgba &c, float &h, float &s, float &v)
{
	const float r_1 = std::max(c.r, 0.f), g_1 = std::max(c.g, 0.f), b_1 = std::max(c.b, 0.f);
	const float max_component = std::max(std::max(r_1, g_1), b_1);
	const float min_component = std::min(std::min(r_1, g_1), b_1);
	const float range = max_component - min_component;
	v = max_component;
	if(std::abs(range) < 1.0e-6f) { h = 0.f; s = 0.f; }
	else if(max_component == r_1) { h = std::fmod((g_1 - b_1) / range, 6.f); s = range / std::max(v, 1.0e-6f); }
	else if(max_component == g_1) { h = ((b_1 - r_1) / range) + 2.f; s = range / std::max(v, 1.0e-6f); }
	else if(max_component == b_1) { h = ((r_1 - g_1) / range) + 4.f; s = range / std::max(v, 1.0e-6f); }
	else { h = 0.f; s = 0.f; v = 0.f; }
	if(h < 0.f) h += 6.f;
}
static inline void hsvToRgb(Rgba &c, float h, float s, float v)
{
	const float cc = v * s;
	const float x = cc * (1.f - std::abs(std::fmod(h, 2.f) - 1.f));
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

// ---------------------------------------------------------------------------------------------
// image buffer pixel types (include/image/image_buffers.h), stored bit for bit as there
// ---------------------------------------------------------------------------------------------
// (uint8_t)roundf(x) / (uint16_t)roundf(x) as an x86-64 build evaluates them
static inline uint8_t toU8(float v) { const float r = std::roundf(v); return (uint8_t)(int32_t)((r > -2147483904.f && r < 2147483648.f) ? (int32_t)r : INT32_MIN); }
static inline uint16_t toU16(float v) { const float r = std::roundf(v); return (uint16_t)(int32_t)((r > -2147483904.f && r < 2147483648.f) ? (int32_t)r : INT32_MIN); }

struct PxRgba1010108   // :265-296
{
	uint8_t extra = 0, r = 0, g = 0, b = 0, a = 0;
	void set(const Rgba &c)
	{
		const uint16_t r10 = toU16(c.r * 1023.f), g10 = toU16(c.g * 1023.f), b10 = toU16(c.b * 1023.f);
		r = r10 & 0xFF; extra = (extra & 0x0F) | ((r10 & 0x0300) >> 4);
		g = g10 & 0xFF; extra = (extra & 0x33) | ((g10 & 0x0300) >> 6);
		b = b10 & 0xFF; extra = (extra & 0x3C) | ((b10 & 0x0300) >> 8);
		a = toU8(c.a * 255.f);
	}
	Rgba get() const
	{
		return {(float)(uint16_t)(r + ((uint16_t)(extra & 0x30) << 4)) / 1023.f, (float)(uint16_t)(g + ((uint16_t)(extra & 0x0C) << 6)) / 1023.f,
		        (float)(uint16_t)(b + ((uint16_t)(extra & 0x03) << 8)) / 1023.f, (float)a / 255.f};
	}
};
struct PxRgb101010   // :236-263
{
	uint8_t extra = 0, r = 0, g = 0, b = 0;
	void set(const Rgba &c)
	{
		const uint16_t r10 = toU16(c.r * 1023.f), g10 = toU16(c.g * 1023.f), b10 = toU16(c.b * 1023.f);
		r = r10 & 0xFF; extra = (extra & 0x0F) | ((r10 & 0x0300) >> 4);
		g = g10 & 0xFF; extra = (extra & 0x33) | ((g10 & 0x0300) >> 6);
		b = b10 & 0xFF; extra = (extra & 0x3C) | ((b10 & 0x0300) >> 8);
	}
	Rgba get() const
	{
		return {(float)(uint16_t)(r + ((uint16_t)(extra & 0x30) << 4)) / 1023.f, (float)(uint16_t)(g + ((uint16_t)(extra & 0x0C) << 6)) / 1023.f,
		        (float)(uint16_t)(b + ((uint16_t)(extra & 0x03) << 8)) / 1023.f, 1.f};
	}
};
struct PxRgba7773   // :141-170
{
	uint8_t ra = 0, ga = 0, ba = 0;
	void set(const Rgba &c)
	{
		ra = (ra & 0x01) | (toU8(c.r * 255.f) & 0xFE);
		ga = (ga & 0x01) | (toU8(c.g * 255.f) & 0xFE);
		ba = (ba & 0x01) | (toU8(c.b * 255.f) & 0xFE);
		const uint8_t a8 = toU8(c.a * 255.f);
		ra = (ra & 0xFE) | ((a8 & 0x80) >> 7);
		ga = (ga & 0xFE) | ((a8 & 0x40) >> 6);
		ba = (ba & 0xFE) | ((a8 & 0x20) >> 5);
	}
	Rgba get() const
	{
		const uint8_t a8 = ((ra & 0x01) << 7) | ((ga & 0x01) << 6) | ((ba & 0x01) << 5);
		return {(float)(ra & 0xFE) / 254.f, (float)(ga & 0xFE) / 254.f, (float)(ba & 0xFE) / 254.f, (float)a8 / 224.f};
	}
};
struct PxRgb565   // :216-234
{
	uint16_t v = 0;
	void set(const Rgba &c)
	{
		v = (v & 0x07FF) | ((toU8(c.r * 255.f) & 0xF8) << 8);
		v = (v & 0xF81F) | ((toU8(c.g * 255.f) & 0xFC) << 3);
		v = (v & 0xFFE0) | ((toU8(c.b * 255.f) & 0xF8) >> 3);
	}
	Rgba get() const
	{
		return {(float)(uint8_t)((v & 0xF800) >> 8) / 248.f, (float)(uint8_t)((v & 0x07E0) >> 3) / 252.f, (float)(uint8_t)((v & 0x001F) << 3) / 248.f, 1.f};
	}
};
struct PxGray8   // :193-214
{
	uint8_t v = 0;
	void set(const Rgba &c) { v = toU8(((c.r + c.g + c.b) / 3.f) * 255.f); }
	Rgba get() const { const float f = (float)v / 255.f; return {f, f, f, 1.f}; }
};
struct PxGray   // :52-62
{
	float v = 0.f;
	void set(const Rgba &c) { v = (c.r + c.g + c.b) / 3.f; }
	Rgba get() const { return {v, v, v, 1.f}; }
};
struct PxGrayAlpha   // :64-72
{
	float v = 0.f, a = 0.f;
	void set(const Rgba &c) { v = (c.r + c.g + c.b) / 3.f; a = c.a; }
	Rgba get() const { return {v, v, v, a}; }
};
struct PxRgb   // image_color.h (ImageBuffer2D<Rgb>)
{
	float r = 0.f, g = 0.f, b = 0.f;
	void set(const Rgba &c) { r = c.r; g = c.g; b = c.b; }
	Rgba get() const { return {r, g, b, 1.f}; }
};
struct PxRgbAlpha   // :106-115 (rgba_{0.f}: explicit Rgba(float) -> alpha 0)
{
	Rgba c{0.f};
	void set(const Rgba &x) { c = x; }
	Rgba get() const { return c; }
};

enum { ImgNone = 0, ImgGray = 1, ImgGrayAlpha = 2, ImgColor = 3, ImgColorAlpha = 4 };   // image.h:47
enum { OptNone = 0, OptOptimized = 1, OptCompressed = 2 };                              // image.h:48

struct OImageBase
{
	int w = 0, h = 0, color_space = CsRawManualGamma;
	float gamma = 1.f;
	virtual ~OImageBase() = default;
	virtual Rgba getColor(int x, int y) const = 0;
	virtual void setColor(int x, int y, const Rgba &c) = 0;
};
template<class Px>
struct OImage : OImageBase
{
	std::vector<Px> buf;
	OImage(int width, int height) { w = width; h = height; buf.resize((size_t)std::max(0, w) * std::max(0, h)); }
	Rgba getColor(int x, int y) const override { return buf[(size_t)x * h + y].get(); }   // Buffer<T,2>: x * height + y
	void setColor(int x, int y, const Rgba &c) override { buf[(size_t)x * h + y].set(c); }
};

// Image::factory(logger, width, height, type, optimization) (image.cc:102-137)
static std::unique_ptr<OImageBase> makeImage(int w, int h, int type, int opt)
{
	switch(type)
	{
		case ImgColorAlpha:
			if(opt == OptOptimized) return std::unique_ptr<OImageBase>(new OImage<PxRgba1010108>(w, h));
			if(opt == OptCompressed) return std::unique_ptr<OImageBase>(new OImage<PxRgba7773>(w, h));
			return std::unique_ptr<OImageBase>(new OImage<PxRgbAlpha>(w, h));
		case ImgColor:
			if(opt == OptOptimized) return std::unique_ptr<OImageBase>(new OImage<PxRgb101010>(w, h));
			if(opt == OptCompressed) return std::unique_ptr<OImageBase>(new OImage<PxRgb565>(w, h));
			return std::unique_ptr<OImageBase>(new OImage<PxRgb>(w, h));
		case ImgGrayAlpha: return std::unique_ptr<OImageBase>(new OImage<PxGrayAlpha>(w, h));
		case ImgGray:
			if(opt == OptOptimized || opt == OptCompressed) return std::unique_ptr<OImageBase>(new OImage<PxGray8>(w, h));
			return std::unique_ptr<OImageBase>(new OImage<PxGray>(w, h));
		default: return nullptr;
	}
}

// ---------------------------------------------------------------------------------------------
// TGA loading (format_tga.cc:199-396)
// ---------------------------------------------------------------------------------------------
struct ByteFile
{
	const uint8_t *d;
	size_t n, pos = 0;
	bool eof = false;
	size_t read(void *dst, size_t k)
	{
		size_t got = 0;
		uint8_t *o = (uint8_t *)dst;
		while(got < k && pos < n) o[got++] = d[pos++];
		if(got < k) { std::memset(o + got, 0, k - got); eof = true; }
		return got;
	}
	uint8_t u8() { uint8_t v = 0; read(&v, 1); return v; }
	uint16_t u16() { uint8_t b[2]; read(b, 2); return (uint16_t)(b[0] | (b[1] << 8)); }
};

static constexpr double inv_31 = 1.0 / 31.0;                              // format.h:60
static constexpr double inv_max_8_bit = 1.0 / static_cast<double>(255);   // format.h:61

static Rgba tgaProcess(int depth, bool gray, const uint8_t *px, const std::vector<Rgba> &cmap)
{
	switch(depth)
	{
		case 8:
			if(gray) return Rgba((float)(px[0] * inv_max_8_bit));               // processGray8 (:129-132)
			return px[0] < cmap.size() ? cmap[px[0]] : Rgba();                   // processColor8 (:139-143)
		case 15:
		case 16:
		{
			const uint16_t c = (uint16_t)(px[0] | (px[1] << 8));
			if(depth == 16 && gray)   // processGray16 (:133-137)
			{
				const float v = (float)((c & 0x00FF) * inv_max_8_bit);
				return {v, v, v, static_cast<float>(((c & 0xFF00) >> 8) * inv_max_8_bit)};
			}
			// processColor15 / processColor16 (:145-162) with the masks as named in format_tga_util.h
			Rgba out {static_cast<float>(((c & 0x003E) >> 11) * inv_31), static_cast<float>(((c & 0x07C0) >> 6) * inv_31),
			          static_cast<float>(((c & 0xF800) >> 1) * inv_31), 1.f};
			if(depth == 16) out.a = static_cast<float>(c & 0x0001);
			return out;
		}
		case 24:   // processColor24: TgaPixelRgb {b, g, r}
			return {static_cast<float>(px[2] * inv_max_8_bit), static_cast<float>(px[1] * inv_max_8_bit), static_cast<float>(px[0] * inv_max_8_bit), 1.f};
		default:   // processColor32: TgaPixelRgba {b, g, r, a}
			return {static_cast<float>(px[2] * inv_max_8_bit), static_cast<float>(px[1] * inv_max_8_bit), static_cast<float>(px[0] * inv_max_8_bit),
			        static_cast<float>(px[3] * inv_max_8_bit)};
	}
}

static std::unique_ptr<OImageBase> loadTga(const uint8_t *data, size_t size, int opt, int cs, float gamma, bool grayscale)
{
	ByteFile f{data, size};
	const uint8_t id_length = f.u8(), cmap_type = f.u8(), image_type = f.u8();
	f.u16();   // first colour map entry (unused, as in the reference)
	const uint16_t cm_entries = f.u16();
	const uint8_t cm_depth = f.u8();
	f.u16(); f.u16();
	const uint16_t width = f.u16(), height = f.u16();
	const uint8_t depth = f.u8(), desc = f.u8();
	const uint8_t alpha_bits = desc & 0x0F;
	bool is_rle = false, has_cmap = false, is_gray = false;
	switch(image_type)
	{
		case 0: return nullptr;
		case 1: if(!cmap_type) return nullptr; has_cmap = true; break;
		case 3: is_gray = true; break;
		case 9: if(!cmap_type) return nullptr; has_cmap = true; is_rle = true; break;
		case 11: is_gray = true; is_rle = true; break;
		case 10: is_rle = true; break;
		default: break;
	}
	if(has_cmap && cm_depth != 15 && cm_depth != 16 && cm_depth != 24 && cm_depth != 32) return nullptr;
	if(is_gray) { if((depth != 8 && depth != 16) || (alpha_bits != 8 && depth == 16)) return nullptr; }
	else if(has_cmap) { if(depth > 16) return nullptr; }
	else if((depth != 15 && depth != 16 && depth != 24 && depth != 32) || (alpha_bits != 1 && depth == 16) || (alpha_bits != 8 && depth == 32)) return nullptr;
	f.pos += id_length;
	const bool has_alpha = (alpha_bits != 0 || cm_depth == 32);
	int type = grayscale ? ImgGray : ImgColor;
	if(has_alpha) type = grayscale ? ImgGrayAlpha : ImgColorAlpha;
	if(!has_alpha && !grayscale && (cm_depth == 16 || cm_depth == 32 || depth == 16 || depth == 32)) type = ImgColorAlpha;
	auto img = makeImage(width, height, type, opt);
	std::vector<Rgba> cmap;
	if(has_cmap)
	{
		const int eb = cm_depth <= 16 ? 2 : cm_depth / 8;
		for(int k = 0; k < cm_entries; ++k)
		{
			uint8_t b[4] = {0, 0, 0, 0};
			f.read(b, eb);
			cmap.push_back(tgaProcess(cm_depth == 15 ? 15 : cm_depth, false, b, cmap));
		}
	}
	int min_x = 0, max_x = width, step_x = 1, min_y = 0, max_y = height, step_y = 1;
	if(!(desc & 0x20)) { min_y = height - 1; max_y = -1; step_y = -1; }
	if(desc & 0x10) { min_x = width - 1; max_x = -1; step_x = -1; }
	const int bpp = depth == 8 ? 1 : depth <= 16 ? 2 : depth / 8;
	auto store = [&](int x, int y, const uint8_t *px) {
		Rgba c = tgaProcess(depth, is_gray, px, cmap);
		linearRgbFromColorSpace(c, cs, gamma);
		img->setColor(x, y, c);
	};
	if(is_rle)
	{
		int x = min_x, y = min_y;
		while(!f.eof && y != max_y)
		{
			const uint8_t pack = f.u8();
			if(f.eof) break;
			const bool run = (pack & 0x80) != 0;
			const int rep = (pack & 0x7F) + 1;
			uint8_t px[4] = {0, 0, 0, 0};
			if(run) f.read(px, bpp);
			for(int k = 0; k < rep && y != max_y; ++k)
			{
				if(!run) f.read(px, bpp);
				store(x, y, px);
				x += step_x;
				if(x == max_x) { x = min_x; y += step_y; }
			}
		}
	}
	else
	{
		std::vector<uint8_t> raw((size_t)width * height * bpp);
		f.read(raw.data(), raw.size());
		size_t i = 0;
		for(int y = min_y; y != max_y; y += step_y)
			for(int x = min_x; x != max_x; x += step_x, ++i) store(x, y, &raw[i * bpp]);
	}
	return img;
}

// ---------------------------------------------------------------------------------------------
// Radiance HDR loading (format_hdr.cc:36-309, format_hdr_util.h:53-107)
// ---------------------------------------------------------------------------------------------
static Rgba rgbeToRgba(const uint8_t p[4])
{
	if(p[3])
	{
		const float f = std::ldexp(1.f, p[3] - (128 + 8));
		return {f * p[0], f * p[1], f * p[2], 1.f};
	}
	return {0.f, 0.f, 0.f, 1.0f};
}

static std::unique_ptr<OImageBase> loadHdr(const uint8_t *data, size_t size, bool grayscale)
{
	ByteFile f{data, size};
	auto line = [&]() {
		std::string s;
		while(f.pos < f.n && s.size() < 999)
		{
			const char ch = (char)f.d[f.pos++];
			s.push_back(ch);
			if(ch == '\n') break;
		}
		return s;
	};
	std::string l = line();
	if(l.find("#?") == std::string::npos) return nullptr;
	for(;;)
	{
		l = line();
		if(l.empty() || l == "\n") break;
		const size_t fp = l.find("FORMAT=");
		if(fp != std::string::npos && l.substr(fp + 7).find("32-bit_rle_rgbe") == std::string::npos) return nullptr;
	}
	std::vector<std::string> tok;
	{
		std::istringstream is(line());
		std::string t;
		while(is >> t) tok.push_back(t);
	}
	if(tok.size() < 4) return nullptr;
	const bool y_first = tok[0].find('Y') != std::string::npos;
	const int wi = y_first ? 3 : 1, hi = y_first ? 1 : 3, xi = y_first ? 2 : 0, yi = y_first ? 0 : 2;
	const int fi = y_first ? 0 : 1, si = y_first ? 1 : 0;
	const int width = std::atoi(tok[wi].c_str()), height = std::atoi(tok[hi].c_str());
	if(width <= 0 || height <= 0) return nullptr;
	int mn[2], mx[2], st[2];
	mn[fi] = 0; mx[fi] = height; st[fi] = 1;
	mn[si] = 0; mx[si] = width; st[si] = 1;
	if(tok[xi].find('+') == std::string::npos) { mn[si] = width - 1; mx[si] = -1; st[si] = -1; }
	if(tok[yi].find('-') == std::string::npos) { mn[fi] = height - 1; mx[fi] = -1; st[fi] = -1; }
	auto img = makeImage(width, height, grayscale ? ImgGrayAlpha : ImgColorAlpha, OptNone);
	const int scan_width = y_first ? width : height;
	auto put = [&](int a, int b, const uint8_t *p) {
		const Rgba c = rgbeToRgba(p);   // linear RGB: no conversion
		if(y_first) img->setColor(a, b, c);
		else img->setColor(b, a, c);
	};
	// readOrle: its store loop steps by max_[1] (first pixel only for a left-to-right scan)
	auto orle = [&](int y, int sw) -> bool {
		std::vector<std::array<uint8_t, 4>> scan((size_t)std::max(1, sw), std::array<uint8_t, 4>{0, 0, 0, 0});
		int rshift = 0;
		for(int x = mn[1]; x < sw;)
		{
			uint8_t px[4];
			if(f.read(px, 4) != 4) return false;
			if(px[0] == 1 && px[1] == 1 && px[2] == 1)
			{
				int count = (int)px[3] << rshift;
				if(count > sw - x) return false;
				const std::array<uint8_t, 4> prev = x >= 1 ? scan[x - 1] : std::array<uint8_t, 4>{0, 0, 0, 0};
				while(count--) scan[x++] = prev;
				rshift += 8;
			}
			else
			{
				if(x >= 0) scan[x] = {px[0], px[1], px[2], px[3]};
				++x;
				rshift = 0;
			}
		}
		int j = 0;
		for(int x = mn[1]; x != mx[1]; x += mx[1])
		{
			put(x, y, scan[j].data());
			++j;
			if(mx[1] == 0) break;
		}
		return true;
	};
	auto arle = [&](int y, int sw) -> bool {
		std::vector<std::array<uint8_t, 4>> scan((size_t)std::max(1, sw), std::array<uint8_t, 4>{0, 0, 0, 0});
		for(int chan = 0; chan < 4; ++chan)
		{
			int j = 0;
			while(j < sw)
			{
				uint8_t count = 0;
				if(f.read(&count, 1) != 1) return false;
				if(count > 128)
				{
					count &= 0x7F;
					if(count + j > sw) return false;
					uint8_t col = 0;
					if(f.read(&col, 1) != 1) return false;
					while(count--) scan[j++][chan] = col;
				}
				else
				{
					if(count + j > sw) return false;
					while(count--)
					{
						uint8_t col = 0;
						if(f.read(&col, 1) != 1) return false;
						scan[j++][chan] = col;
					}
				}
			}
		}
		int j = 0;
		for(int x = mn[1]; x != mx[1]; x += st[1], ++j)
		{
			static const uint8_t zero[4] = {0, 0, 0, 0};
			put(x, y, j < sw ? scan[j].data() : zero);
		}
		return true;
	};
	if(scan_width < 8 || scan_width > 0x7fff)
	{
		for(int y = mn[0]; y != mx[0]; y += st[0])
			if(!orle(y, scan_width)) return nullptr;
		return img;
	}
	for(int y = mn[0]; y != mx[0]; y += st[0])
	{
		uint8_t px[4];
		if(f.read(px, 4) != 4) return nullptr;
		const int count = (int)(px[2] << 8 | px[3]);
		if(px[0] == 2 && px[1] == 2 && count < 0x8000)
		{
			if(count > scan_width) return nullptr;
			if(!arle(y, count)) return nullptr;
		}
		else
		{
			f.pos -= 4;
			f.eof = false;
			if(!orle(y, scan_width)) return nullptr;
		}
	}
	return img;
}

// ---------------------------------------------------------------------------------------------
// ImageTexture (texture_image.cc:46-235) + Texture adjustments (texture.cc:134-262)
// ---------------------------------------------------------------------------------------------
enum { ClipExtend = 0, ClipClip = 1, ClipClipCube = 2, ClipRepeat = 3, ClipChecker = 4 };   // texture_image.h:62
enum { InterpNone = 0, InterpBilinear = 1, InterpBicubic = 2 };

struct OTexture
{
	const OImageBase *img = nullptr;
	int interp = InterpBilinear, clip = ClipRepeat, xrepeat = 1, yrepeat = 1;
	bool mirror_x = false, mirror_y = false, rot90 = false, checker_even = false, checker_odd = true, cropx = false, cropy = false;
	float cropminx = 0.f, cropmaxx = 1.f, cropminy = 0.f, cropmaxy = 1.f, checker_dist = 0.f;
	float adj_intensity = 1.f, adj_contrast = 1.f, adj_saturation = 1.f, adj_hue = 0.f;
	float adj_r = 1.f, adj_g = 1.f, adj_b = 1.f;
	bool adj_clamp = false, adjustments_set = false;
	int orig_cs = CsRawManualGamma;
	float orig_gamma = 1.f;

	bool doMapping(V3 &t) const
	{
		bool outside = false;
		t = 0.5f * t + V3(0.5f, 0.5f, 0.5f);
		if(clip == ClipRepeat)
		{
			if(xrepeat > 1) t.x *= static_cast<float>(xrepeat);
			if(yrepeat > 1) t.y *= static_cast<float>(yrepeat);
			if(mirror_x && static_cast<int>(ceilf(t.x)) % 2 == 0) t.x = -t.x;
			if(mirror_y && static_cast<int>(ceilf(t.y)) % 2 == 0) t.y = -t.y;
			if(t.x > 1.f) t.x -= static_cast<int>(t.x);
			else if(t.x < 0.f) t.x += 1 - static_cast<int>(t.x);
			if(t.y > 1.f) t.y -= static_cast<int>(t.y);
			else if(t.y < 0.f) t.y += 1 - static_cast<int>(t.y);
		}
		if(cropx) t.x = cropminx + t.x * (cropmaxx - cropminx);
		if(cropy) t.y = cropminy + t.y * (cropmaxy - cropminy);
		if(rot90) std::swap(t.x, t.y);
		if(clip == ClipClipCube)
		{
			if((t.x < 0) || (t.x > 1) || (t.y < 0) || (t.y > 1) || (t.z < -1) || (t.z > 1)) outside = true;
		}
		else if(clip == ClipChecker || clip == ClipClip)
		{
			bool checked_out = false;
			if(clip == ClipChecker)
			{
				const int xs = static_cast<int>(std::floor(t.x)), ys = static_cast<int>(std::floor(t.y));
				t.x -= xs;
				t.y -= ys;
				if(!checker_odd && !((xs + ys) & 1)) checked_out = true;
				else if(!checker_even && ((xs + ys) & 1)) checked_out = true;
				else if(checker_dist < 1.0)
				{
					t.x = (t.x - 0.5f) / (1.f - checker_dist) + 0.5f;
					t.y = (t.y - 0.5f) / (1.f - checker_dist) + 0.5f;
				}
			}
			if(checked_out) outside = true;
			else if((t.x < 0) || (t.x > 1) || (t.y < 0) || (t.y > 1)) outside = true;
		}
		else if(clip == ClipExtend)
		{
			if(t.x > 0.99999f) t.x = 0.99999f; else if(t.x < 0) t.x = 0;
			if(t.y > 0.99999f) t.y = 0.99999f; else if(t.y < 0) t.y = 0;
		}
		return outside;
	}

	static void coords(int &c0, int &c1, int &c2, int &c3, float &dec, float cf, int res, bool repeat, bool mirror)
	{
		if(repeat)
		{
			c1 = (static_cast<int>(cf)) % res;
			if(mirror)
			{
				if(cf < 0.f) { c0 = 1 % res; c2 = c1; c3 = c0; dec = -cf; }
				else if(cf >= (res - 1)) { c0 = (2 * res - 1) % res; c2 = c1; c3 = c0; dec = cf - (static_cast<int>(cf)); }
				else
				{
					c0 = (res + c1 - 1) % res;
					c2 = c1 + 1;
					if(c2 >= res) c2 = (2 * res - c2) % res;
					c3 = c1 + 2;
					if(c3 >= res) c3 = (2 * res - c3) % res;
					dec = cf - (static_cast<int>(cf));
				}
			}
			else if(cf > 0.f)
			{
				c0 = (res + c1 - 1) % res;
				c2 = (c1 + 1) % res;
				c3 = (c1 + 2) % res;
				dec = cf - (static_cast<int>(cf));
			}
			else
			{
				c0 = 1 % res;
				c2 = (res - 1) % res;
				c3 = (res - 2) % res;
				dec = -cf;
			}
		}
		else
		{
			c1 = std::max(0, std::min(res - 1, (static_cast<int>(cf))));
			c2 = (cf > 0.f) ? std::min(res - 1, c1 + 1) : 0;
			c0 = std::max(0, c1 - 1);
			c3 = std::min(res - 1, c2 + 1);
			dec = cf - std::floor(cf);
		}
	}

	static Rgba cubic(const Rgba &y0, const Rgba &y1, const Rgba &y2, const Rgba &y3, float x)   // interpolation.h:69-80
	{
		const float x2 = x * x;
		const float x3 = x * x2;
		const Rgba a0 = y3 - y2 - y0 + y1;
		const Rgba a1 = y0 - y1 - a0;
		const Rgba a2 = y2 - y0;
		const Rgba a3 = y1;
		return (a0 * x3 + a1 * x2 + a2 * x + a3);
	}

	Rgba interpolate(const V3 &p) const
	{
		const int resx = img->w, resy = img->h;
		const float sub = interp == InterpNone ? 0.f : 0.5f;
		const float xf = (static_cast<float>(resx) * (p.x - std::floor(p.x))) - sub;
		const float yf = (static_cast<float>(resy) * (p.y - std::floor(p.y))) - sub;
		int x0, x1, x2, x3, y0, y1, y2, y3;
		float dx, dy;
		coords(x0, x1, x2, x3, dx, xf, resx, clip == ClipRepeat, mirror_x);
		coords(y0, y1, y2, y3, dy, yf, resy, clip == ClipRepeat, mirror_y);
		if(interp == InterpNone) return img->getColor(x1, y1);
		if(interp == InterpBilinear)
		{
			const Rgba c11 = img->getColor(x1, y1), c21 = img->getColor(x2, y1), c12 = img->getColor(x1, y2), c22 = img->getColor(x2, y2);
			const float w11 = (1 - dx) * (1 - dy), w12 = (1 - dx) * dy, w21 = dx * (1 - dy), w22 = dx * dy;
			return (w11 * c11) + (w12 * c12) + (w21 * c21) + (w22 * c22);
		}
		const int xs[4] = {x0, x1, x2, x3}, ys[4] = {y0, y1, y2, y3};
		Rgba cy[4];
		for(int j = 0; j < 4; ++j)
			cy[j] = cubic(img->getColor(xs[0], ys[j]), img->getColor(xs[1], ys[j]), img->getColor(xs[2], ys[j]), img->getColor(xs[3], ys[j]), dx);
		return cubic(cy[0], cy[1], cy[2], cy[3], dy);
	}

	Rgba adjustIntensityContrast(const Rgba &c) const
	{
		if(!adjustments_set) return c;
		Rgba ret = c;
		if(adj_intensity != 1.f || adj_contrast != 1.f)
		{
			ret.r = (c.r - 0.5f) * adj_contrast + adj_intensity - 0.5f;
			ret.g = (c.g - 0.5f) * adj_contrast + adj_intensity - 0.5f;
			ret.b = (c.b - 0.5f) * adj_contrast + adj_intensity - 0.5f;
		}
		if(adj_clamp) ret.clampRgb0();
		return ret;
	}
	Rgba adjustColor(const Rgba &c) const
	{
		if(!adjustments_set) return c;
		Rgba ret = c;
		if(adj_r != 1.f) ret.r *= adj_r;
		if(adj_g != 1.f) ret.g *= adj_g;
		if(adj_b != 1.f) ret.b *= adj_b;
		if(adj_clamp) ret.clampRgb0();
		if(adj_saturation != 1.f || adj_hue != 0.f)
		{
			float h = 0.f, s = 0.f, v = 0.f;
			rgbToHsv(ret, h, s, v);
			s *= adj_saturation;
			h += adj_hue;
			if(h < 0.f) h += 6.f;
			else if(h > 6.f) h -= 6.f;
			hsvToRgb(ret, h, s, v);
			if(adj_clamp) ret.clampRgb0();
		}
		return ret;
	}
	Rgba getColor(const V3 &p) const
	{
		V3 p1(p.x, -p.y, p.z);
		if(doMapping(p1)) return Rgba(0.f);
		return adjustColor(adjustIntensityContrast(interpolate(p1)));
	}
	float getFloat(const V3 &p) const
	{
		Rgba raw = getColor(p);
		colorSpaceFromLinearRgb(raw, orig_cs, orig_gamma);
		float f = raw.col2Bri();
		if(!adjustments_set) return f;
		if(adj_intensity != 1.f || adj_contrast != 1.f) f = (f - 0.5f) * adj_contrast + adj_intensity - 0.5f;
		if(adj_clamp) f = f < 0.f ? 0.f : (f > 1.f ? 1.f : f);
		return f;
	}
};

// ---------------------------------------------------------------------------------------------
// shader nodes (shader_node_basic.cc, shader_node_layer.cc)
// ---------------------------------------------------------------------------------------------
enum { NodeValue = 0, NodeMix = 1, NodeLayer = 2, NodeMapper = 3 };
enum { BlMix = 0, BlAdd, BlMult, BlSub, BlScreen, BlDiv, BlDiff, BlDark, BlLight, BlOverlay };
enum { TcUv = 0, TcGlobal, TcOrco, TcTransformed };
enum { PrPlain = 0, PrCube, PrTube, PrSphere };

// the SurfacePoint values the nodes read
struct TexPoint
{
	V3 p, ng, orco_p, orco_ng;
	float u = 0.f, v = 0.f;
};

struct NodeOut { Rgba col; float val = 0.f; };

// TextureMapperNode::doMapping (:106-133) + the maps (:56-100)
static V3 mapperDoMapping(const yc_node &nd, const V3 &p, const V3 &n)
{
	V3 t = p;
	if(nd.coords == TcUv) t = V3(2.f * t.x - 1.f, 2.f * t.y - 1.f, t.z);
	const float tm[4] = {0.f, t.x, t.y, t.z};
	t = V3(tm[nd.map[0]], tm[nd.map[1]], tm[nd.map[2]]);
	if(nd.projection == PrTube)
	{
		V3 r;
		r.y = t.z;
		const float d = t.x * t.x + t.y * t.y;
		if(d > 0.f)
		{
			r.z = 1.f / fsqrt(d);
			r.x = static_cast<float>(-std::atan2(t.x, t.y) * div_1_by_pi);
		}
		else r.x = r.z = 0.f;
		t = r;
	}
	else if(nd.projection == PrSphere)
	{
		V3 r(0.f, 0.f, 0.f);
		const float d = t.x * t.x + t.y * t.y + t.z * t.z;
		if(d > 0.f)
		{
			r.z = fsqrt(d);
			if((t.x != 0.f) && (t.y != 0.f)) r.x = static_cast<float>(-std::atan2(t.x, t.y) * div_1_by_pi);
			r.y = static_cast<float>(1.f - 2.f * (facos(t.z / r.z) * div_1_by_pi));
		}
		t = r;
	}
	else if(nd.projection == PrCube)
	{
		static const int ma[3][3] = {{1, 2, 0}, {0, 2, 1}, {0, 1, 2}};
		int axis;
		if(std::abs(n.z) >= std::abs(n.x) && std::abs(n.z) >= std::abs(n.y)) axis = 2;
		else if(std::abs(n.y) >= std::abs(n.x) && std::abs(n.y) >= std::abs(n.z)) axis = 1;
		else axis = 0;
		t = V3(t[ma[axis][0]], t[ma[axis][1]], t[ma[axis][2]]);
	}
	// Point3::mult(texpt, scale_) + offset_ (offset_ = 2 * offset, :372)
	return V3(t.x * nd.scale[0] + 2 * nd.offset[0], t.y * nd.scale[1] + 2 * nd.offset[1], t.z * nd.scale[2] + 2 * nd.offset[2]);
}

// Rgb blends of LayerNode::textureRgbBlend (shader_node_layer.cc:187-253); alpha unused
static Rgba layerRgbBlend(const Rgba &tex, const Rgba &out, float fact, float facg, int mode)
{
	auto rgb = [](float r, float g, float b) { return Rgba(r, g, b, 1.f); };
	switch(mode)
	{
		case BlMult:
			fact *= facg;
			return rgb(((1.f - facg) + fact * tex.r) * out.r, ((1.f - facg) + fact * tex.g) * out.g, ((1.f - facg) + fact * tex.b) * out.b);
		case BlScreen:
			fact *= facg;
			return rgb(1.f - ((1.f - facg) + fact * (1.f - tex.r)) * (1.f - out.r), 1.f - ((1.f - facg) + fact * (1.f - tex.g)) * (1.f - out.g),
			           1.f - ((1.f - facg) + fact * (1.f - tex.b)) * (1.f - out.b));
		case BlSub:
		case BlAdd:
			if(mode == BlSub) fact = -fact;
			fact *= facg;
			return rgb(fact * tex.r + out.r, fact * tex.g + out.g, fact * tex.b + out.b);
		case BlDiv:
		{
			fact *= facg;
			const float ir = tex.r != 0.f ? 1.f / tex.r : tex.r, ig = tex.g != 0.f ? 1.f / tex.g : tex.g, ib = tex.b != 0.f ? 1.f / tex.b : tex.b;
			return rgb((1.f - fact) * out.r + (fact * out.r) * ir, (1.f - fact) * out.g + (fact * out.g) * ig, (1.f - fact) * out.b + (fact * out.b) * ib);
		}
		case BlDiff:
			fact *= facg;
			return rgb((1.f - fact) * out.r + fact * std::abs(tex.r - out.r), (1.f - fact) * out.g + fact * std::abs(tex.g - out.g),
			           (1.f - fact) * out.b + fact * std::abs(tex.b - out.b));
		case BlDark:
		case BlLight:
		{
			fact *= facg;
			float c[3] = {fact * tex.r, fact * tex.g, fact * tex.b};
			const float o[3] = {out.r, out.g, out.b};
			for(int k = 0; k < 3; ++k)
				if(mode == BlDark ? c[k] > o[k] : c[k] < o[k]) c[k] = o[k];
			return rgb(c[0], c[1], c[2]);
		}
		default:
			fact *= facg;
			return rgb(fact * tex.r + (1.f - fact) * out.r, fact * tex.g + (1.f - fact) * out.g, fact * tex.b + (1.f - fact) * out.b);
	}
}
// LayerNode::textureValueBlend (:255-285), flip = false
static float layerValueBlend(float tex, float out, float fact, float facg, int mode)
{
	fact *= facg;
	float facm = 1.f - fact;
	switch(mode)
	{
		case BlMult: facm = 1.f - facg; return (facm + fact * tex) * out;
		case BlScreen: facm = 1.f - facg; return 1.f - (facm + fact * (1.f - tex)) * (1.f - out);
		case BlSub: fact = -fact; return fact * tex + out;
		case BlAdd: return fact * tex + out;
		case BlDiv: if(tex == 0.f) return 0.f; return facm * out + fact * out / tex;
		case BlDiff: return facm * out + fact * std::abs(tex - out);
		case BlDark: { const float col = fact * tex; return col < out ? col : out; }
		case BlLight: { const float col = fact * tex; return col > out ? col : out; }
		default: return fact * tex + facm * out;
	}
}

// Evaluates node `k` (and, recursively, its inputs) at the surface point, memoised per point
struct NodeEval
{
	const std::vector<yc_node> &nodes;
	const std::vector<OTexture> &texs;
	const TexPoint &tp;
	std::vector<NodeOut> out;
	std::vector<char> done;
	NodeEval(const std::vector<yc_node> &n, const std::vector<OTexture> &t, const TexPoint &p)
		: nodes(n), texs(t), tp(p), out(n.size()), done(n.size(), 0) {}

	const NodeOut &get(int k)
	{
		if(done[k]) return out[k];
		const yc_node &nd = nodes[k];
		NodeOut r;
		if(nd.type == NodeValue)
		{
			r.col = Rgba(nd.col1[0], nd.col1[1], nd.col1[2], nd.col1[3]);
			r.val = nd.val[0];
		}
		else if(nd.type == NodeMapper)
		{
			V3 p, n;
			switch(nd.coords)
			{
				case TcUv: p = V3(tp.u, tp.v, 0.f); n = tp.ng; break;
				case TcOrco: p = tp.orco_p; n = tp.orco_ng; break;
				case TcTransformed:
				{
					const float *m = nd.mtx;
					p = V3(m[0] * tp.p.x + m[1] * tp.p.y + m[2] * tp.p.z + m[3], m[4] * tp.p.x + m[5] * tp.p.y + m[6] * tp.p.z + m[7],
					       m[8] * tp.p.x + m[9] * tp.p.y + m[10] * tp.p.z + m[11]);
					n = V3(m[0] * tp.ng.x + m[1] * tp.ng.y + m[2] * tp.ng.z, m[4] * tp.ng.x + m[5] * tp.ng.y + m[6] * tp.ng.z,
					       m[8] * tp.ng.x + m[9] * tp.ng.y + m[10] * tp.ng.z);
					break;
				}
				default: p = tp.p; n = tp.ng; break;
			}
			const V3 t = mapperDoMapping(nd, p, n);
			const OTexture &tex = texs[nd.texture];
			r.col = tex.getColor(t);
			r.val = nd.do_scalar ? tex.getFloat(t) : 0.f;
		}
		else if(nd.type == NodeMix)
		{
			const float f2 = nd.input[2] >= 0 ? get(nd.input[2]).val : nd.val[0];
			Rgba c1, c2;
			float v1, v2;
			if(nd.input[0] >= 0) { c1 = get(nd.input[0]).col; v1 = get(nd.input[0]).val; }
			else { c1 = Rgba(nd.col1[0], nd.col1[1], nd.col1[2], nd.col1[3]); v1 = nd.val[1]; }
			if(nd.input[1] >= 0) { c2 = get(nd.input[1]).col; v2 = get(nd.input[1]).val; }
			else { c2 = Rgba(nd.col2[0], nd.col2[1], nd.col2[2], nd.col2[3]); v2 = nd.val[2]; }
			const float f1 = 1.f - f2;
			switch(nd.blend)
			{
				case BlAdd: r.col = c1 + f2 * c2; r.val = v1 + f2 * v2; break;
				case BlMult: r.col = c1 * (Rgba(f1) + f2 * c2); r.val = v1; break;   // MultNode returns fin_1
				case BlSub: r.col = c1 - f2 * c2; r.val = v1 - f2 * v2; break;
				case BlScreen:
					r.col = Rgba(1.f) - (Rgba(f1) + f2 * (Rgba(1.f) - c2)) * (Rgba(1.f) - c1);
					r.val = 1.f - (f1 + f2 * (1.f - v2)) * (1.f - v1);
					break;
				case BlDiff:
					r.col = Rgba(f1 * c1.r + f2 * std::abs(c1.r - c2.r), f1 * c1.g + f2 * std::abs(c1.g - c2.g), f1 * c1.b + f2 * std::abs(c1.b - c2.b),
					             f1 * c1.a + f2 * std::abs(c1.a - c2.a));
					r.val = f1 * v1 + f2 * std::abs(v1 - v2);
					break;
				case BlDark:
				case BlLight:
				{
					const bool dark = nd.blend == BlDark;
					c2 = c2 * f2;
					float *a[4] = {&c1.r, &c1.g, &c1.b, &c1.a};
					const float b[4] = {c2.r, c2.g, c2.b, c2.a};
					for(int q = 0; q < 4; ++q)
						if(dark ? b[q] < *a[q] : b[q] > *a[q]) *a[q] = b[q];
					v2 *= f2;
					if(dark ? v2 < v1 : v2 > v1) v1 = v2;
					r.col = c1;
					r.val = v1;
					break;
				}
				case BlOverlay:
				{
					auto ov = [&](float x, float y) { return (x < 0.5f) ? x * (f1 + 2.f * f2 * y) : 1.f - (f1 + 2.f * f2 * (1.f - y)) * (1.f - x); };
					r.col = Rgba(ov(c1.r, c2.r), ov(c1.g, c2.g), ov(c1.b, c2.b), ov(c1.a, c2.a));
					r.val = ov(v1, v2);
					break;
				}
				default: r.col = f1 * c1 + f2 * c2; r.val = f1 * v1 + f2 * v2; break;
			}
		}
		else if(nd.type == NodeLayer)
		{
			Rgba texcolor;
			float tin = 0.f, ta = 1.f;
			Rgba rcol = nd.input[1] >= 0 ? get(nd.input[1]).col : Rgba(nd.col2[0], nd.col2[1], nd.col2[2], nd.col2[3]);
			float rval = nd.input[1] >= 0 ? get(nd.input[1]).val : nd.val[3];
			float stencil_tin = rcol.a;
			bool tex_rgb = nd.color_input != 0;
			if(nd.color_input) { texcolor = get(nd.input[0]).col; ta = texcolor.a; }
			else tin = get(nd.input[0]).val;
			if(nd.no_rgb) { tin = texcolor.col2Bri(); tex_rgb = false; }
			if(nd.negative)
			{
				if(tex_rgb) texcolor = Rgba(1.f) - texcolor;
				tin = 1.f - tin;
			}
			if(nd.stencil)
			{
				if(tex_rgb) { const float fact = ta; ta *= stencil_tin; stencil_tin *= fact; }
				else { const float fact = tin; tin *= stencil_tin; stencil_tin *= fact; }
			}
			if(nd.do_color)
			{
				if(!tex_rgb) texcolor = Rgba(nd.col1[0], nd.col1[1], nd.col1[2], nd.col1[3]);
				else tin = ta;
				const float tin_tr = tin > 1.f ? 1.f : (tin < 0.f ? 0.f : tin);
				rcol = layerRgbBlend(texcolor, rcol, tin_tr, stencil_tin * nd.val[0], nd.blend);
				rcol.clampRgb0();
			}
			if(nd.do_scalar)
			{
				if(tex_rgb)
				{
					if(nd.use_alpha) { tin = ta; if(nd.negative) tin = 1.f - tin; }
					else tin = texcolor.col2Bri();
				}
				rval = layerValueBlend(nd.val[2], rval, tin, stencil_tin * nd.val[1], nd.blend);
				if(rval < 0.f) rval = 0.f;
			}
			rcol.a = stencil_tin;
			r.col = rcol;
			r.val = rval;
		}
		out[k] = r;
		done[k] = 1;
		return out[k];
	}
};
