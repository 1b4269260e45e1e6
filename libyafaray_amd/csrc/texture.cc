// Host side of image textures and shader nodes (see texture.h for the reference map).
#include "texture.h"
#include "hostmath.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <sstream>

namespace yafamd
{

// ---------------------------------------------------------------------------------------------
// image buffers (include/image/image_buffers.h)
// ---------------------------------------------------------------------------------------------
namespace
{
// (uintN_t)roundf(v) as compiled for x86-64: cvttss2si to int32 (out of range -> INT_MIN), then
// truncation to N bits
inline uint32_t castRound(float v)
{
	const float r = std::roundf(v);
	int32_t i;
	if(!(r > -2147483904.f && r < 2147483648.f)) i = INT32_MIN;
	else i = (int32_t)r;
	return (uint32_t)i;
}
inline uint8_t u8r(float v) { return (uint8_t)castRound(v); }
inline uint16_t u16r(float v) { return (uint16_t)castRound(v); }
} // namespace

HostImage::HostImage(int width, int height, int t, int o) : w(width), h(height), type(t), opt(o)
{
	px.assign((size_t)std::max(0, w) * std::max(0, h) * 4, 0.f);
	// Buffers zero-initialise their storage; getColor() of zero storage:
	//   Rgba1010108 / Rgba7773: (0,0,0,0); Rgb101010 / Rgb565 / Gray8 / Rgb / Gray: (0,0,0,1);
	//   RgbAlpha: Rgba{0.f} = (0,0,0,0); GrayAlpha: (0, 0) -> (0,0,0,0)
	const bool alpha0 = (type == IMG_COLOR_ALPHA) || (type == IMG_GRAY_ALPHA);
	for(size_t i = 0; i < px.size(); i += 4) { px[i] = px[i + 1] = px[i + 2] = 0.f; px[i + 3] = alpha0 ? 0.f : 1.f; }
}

void HostImage::setColor(int x, int y, const float c[4])
{
	if(x < 0 || y < 0 || x >= w || y >= h) return;
	float *p = &px[4 * ((size_t)y * w + x)];
	const float r = c[0], g = c[1], b = c[2], a = c[3];
	if(type == IMG_COLOR_ALPHA)
	{
		if(opt == OPT_OPTIMIZED)
		{
			// Rgba1010108 (image_buffers.h:265-296)
			p[0] = (float)(u16r(r * 1023.f) & 0x3FF) / 1023.f;
			p[1] = (float)(u16r(g * 1023.f) & 0x3FF) / 1023.f;
			p[2] = (float)(u16r(b * 1023.f) & 0x3FF) / 1023.f;
			p[3] = (float)u8r(a * 255.f) / 255.f;
		}
		else if(opt == OPT_COMPRESSED)
		{
			// Rgba7773 (:141-170)
			p[0] = (float)(u8r(r * 255.f) & 0xFE) / 254.f;
			p[1] = (float)(u8r(g * 255.f) & 0xFE) / 254.f;
			p[2] = (float)(u8r(b * 255.f) & 0xFE) / 254.f;
			p[3] = (float)(u8r(a * 255.f) & 0xE0) / 224.f;
		}
		else { p[0] = r; p[1] = g; p[2] = b; p[3] = a; }   // RgbAlpha
	}
	else if(type == IMG_COLOR)
	{
		if(opt == OPT_OPTIMIZED)
		{
			// Rgb101010 (:236-263)
			p[0] = (float)(u16r(r * 1023.f) & 0x3FF) / 1023.f;
			p[1] = (float)(u16r(g * 1023.f) & 0x3FF) / 1023.f;
			p[2] = (float)(u16r(b * 1023.f) & 0x3FF) / 1023.f;
		}
		else if(opt == OPT_COMPRESSED)
		{
			// Rgb565 (:216-234)
			p[0] = (float)(u8r(r * 255.f) & 0xF8) / 248.f;
			p[1] = (float)(u8r(g * 255.f) & 0xFC) / 252.f;
			p[2] = (float)(u8r(b * 255.f) & 0xF8) / 248.f;
		}
		else { p[0] = r; p[1] = g; p[2] = b; }   // Rgb
		p[3] = 1.f;
	}
	else if(type == IMG_GRAY)
	{
		float v;
		if(opt == OPT_NONE) v = (r + g + b) / 3.f;                       // Gray
		else v = (float)u8r(((r + g + b) / 3.f) * 255.f) / 255.f;       // Gray8 (:193-214)
		p[0] = p[1] = p[2] = v;
		p[3] = 1.f;
	}
	else if(type == IMG_GRAY_ALPHA)
	{
		const float v = (r + g + b) / 3.f;                               // GrayAlpha (:64-72)
		p[0] = p[1] = p[2] = v;
		p[3] = a;
	}
}

void HostImage::getColor(int x, int y, float c[4]) const
{
	if(x < 0 || y < 0 || x >= w || y >= h) { c[0] = c[1] = c[2] = c[3] = 0.f; return; }
	const float *p = &px[4 * ((size_t)y * w + x)];
	for(int k = 0; k < 4; ++k) c[k] = p[k];
}

// ---------------------------------------------------------------------------------------------
// colour spaces (include/color/color.h:336-380)
// ---------------------------------------------------------------------------------------------
static void linearRgbFromColorSpace(float c[4], int cs, float gamma)
{
	if(cs == CS_SRGB)
		for(int k = 0; k < 3; ++k) c[k] = hm::linearFromSrgb(c[k]);
	else if(cs == CS_XYZ_D65)
	{
		const float r = c[0], g = c[1], b = c[2];
		c[0] = 3.2406255f * r + -1.537208f * g + -0.4986286f * b;
		c[1] = -0.9689307f * r + 1.8757561f * g + 0.0415175f * b;
		c[2] = 0.0557101f * r + -0.2040211f * g + 1.0569959f * b;
	}
	else if(cs == CS_RAW_MANUAL_GAMMA && gamma != 1.f)
		for(int k = 0; k < 3; ++k) c[k] = hm::powf_fast(c[k], gamma);
}

static int colorSpaceFromName(const std::string &n, int def)
{
	if(n == "Raw_Manual_Gamma") return CS_RAW_MANUAL_GAMMA;
	if(n == "LinearRGB") return CS_LINEAR_RGB;
	if(n == "sRGB") return CS_SRGB;
	if(n == "XYZ") return CS_XYZ_D65;
	return def;
}

// ---------------------------------------------------------------------------------------------
// TGA (src/format/format_tga.cc, include/format/format_tga_util.h)
// ---------------------------------------------------------------------------------------------
namespace
{
#pragma pack(push, 1)
struct TgaHeader
{
	uint8_t id_length, color_map_type, image_type;
	uint16_t cm_first, cm_count;
	uint8_t cm_depth;
	uint16_t x_origin, y_origin, width, height;
	uint8_t bit_depth, desc;
};
#pragma pack(pop)
static_assert(sizeof(TgaHeader) == 18, "TGA header is 18 bytes");

constexpr double kInv31 = 1.0 / 31.0;            // format.h:60-61
constexpr double kInv255 = 1.0 / 255.0;

struct Rgba4 { float c[4]; };

// format_tga.cc:139-196 (the 15/16-bit masks are applied as the reference names them)
Rgba4 tgaColor15(uint16_t c)
{
	return {{(float)(((c & 0x003E) >> 11) * kInv31), (float)(((c & 0x07C0) >> 6) * kInv31), (float)(((c & 0xF800) >> 1) * kInv31), 1.f}};
}
Rgba4 tgaColor16(uint16_t c)
{
	return {{(float)(((c & 0x003E) >> 11) * kInv31), (float)(((c & 0x07C0) >> 6) * kInv31), (float)(((c & 0xF800) >> 1) * kInv31),
	         (float)(c & 0x0001)}};
}
Rgba4 tgaColor24(const uint8_t *p) { return {{(float)(p[2] * kInv255), (float)(p[1] * kInv255), (float)(p[0] * kInv255), 1.f}}; }
Rgba4 tgaColor32(const uint8_t *p) { return {{(float)(p[2] * kInv255), (float)(p[1] * kInv255), (float)(p[0] * kInv255), (float)(p[3] * kInv255)}}; }
Rgba4 tgaGray8(uint8_t v) { const float g = (float)(v * kInv255); return {{g, g, g, g}}; }   // Rgba(float): alpha = g
Rgba4 tgaGray16(uint16_t c)
{
	const float g = (float)((c & 0x00FF) * kInv255);
	return {{g, g, g, (float)(((c & 0xFF00) >> 8) * kInv255)}};
}

struct Reader
{
	const std::vector<uint8_t> &d;
	size_t pos = 0;
	bool eof = false;
	explicit Reader(const std::vector<uint8_t> &data) : d(data) {}
	// fread semantics: copies what is left, zero-fills the rest, sets eof on a short read
	size_t read(void *dst, size_t n)
	{
		const size_t k = std::min(n, d.size() - std::min(pos, d.size()));
		if(k) std::memcpy(dst, d.data() + pos, k);
		if(k < n) { std::memset((uint8_t *)dst + k, 0, n - k); eof = true; }
		pos += k;
		return k;
	}
};
} // namespace

static std::shared_ptr<HostImage> loadTga(Logger &log, const std::string &name, const std::vector<uint8_t> &data, int opt, int cs,
                                          float gamma, bool grayscale)
{
	Reader rd(data);
	TgaHeader hd;
	rd.read(&hd, sizeof(hd));
	const uint8_t alpha_depth = hd.desc & 0x0F;
	bool is_rle = false, has_cmap = false, is_gray = false;
	// precheckFile (format_tga.cc:198-283)
	switch(hd.image_type)
	{
		case 0: log.error("TGA: TGA file \"" + name + "\" has no image data!"); return nullptr;
		case 1: if(!hd.color_map_type) { log.error("TGA: ColorMap type and no color map embedded"); return nullptr; } has_cmap = true; break;
		case 3: is_gray = true; break;
		case 9: if(!hd.color_map_type) { log.error("TGA: ColorMap type and no color map embedded"); return nullptr; } has_cmap = true; is_rle = true; break;
		case 11: is_gray = true; is_rle = true; break;
		case 10: is_rle = true; break;
		case 2: break;
		default: break;
	}
	if(has_cmap && hd.cm_depth != 15 && hd.cm_depth != 16 && hd.cm_depth != 24 && hd.cm_depth != 32) { log.error("TGA: ColorMap bit depth not supported"); return nullptr; }
	if(is_gray)
	{
		if(hd.bit_depth != 8 && hd.bit_depth != 16) { log.error("TGA: invalid gray bit depth"); return nullptr; }
		if(alpha_depth != 8 && hd.bit_depth == 16) { log.error("TGA: invalid alpha bit depth for 16 bit gray image"); return nullptr; }
	}
	else if(has_cmap)
	{
		if(hd.bit_depth > 16) { log.error("TGA: invalid indexed bit depth"); return nullptr; }
	}
	else
	{
		if(hd.bit_depth != 15 && hd.bit_depth != 16 && hd.bit_depth != 24 && hd.bit_depth != 32) { log.error("TGA: invalid bit depth"); return nullptr; }
		if(alpha_depth != 1 && hd.bit_depth == 16) { log.error("TGA: invalid alpha bit depth for 16 bit color image"); return nullptr; }
		if(alpha_depth != 8 && hd.bit_depth == 32) { log.error("TGA: invalid alpha bit depth for 32 bit color image"); return nullptr; }
	}
	rd.pos += hd.id_length;   // fseek over the image id
	const bool has_alpha = (alpha_depth != 0 || hd.cm_depth == 32);
	int type = grayscale ? IMG_GRAY : IMG_COLOR;
	if(has_alpha) type = grayscale ? IMG_GRAY_ALPHA : IMG_COLOR_ALPHA;
	if(!has_alpha && !grayscale && (hd.cm_depth == 16 || hd.cm_depth == 32 || hd.bit_depth == 16 || hd.bit_depth == 32)) type = IMG_COLOR_ALPHA;
	int iopt = opt;
	if(type == IMG_GRAY && iopt == OPT_COMPRESSED) iopt = OPT_OPTIMIZED;
	auto img = std::make_shared<HostImage>(hd.width, hd.height, type, iopt);
	std::vector<Rgba4> cmap;
	if(has_cmap)
	{
		cmap.resize(hd.cm_count);
		for(int i = 0; i < hd.cm_count; ++i)
		{
			uint8_t b[4] = {0, 0, 0, 0};
			if(hd.cm_depth == 15 || hd.cm_depth == 16)
			{
				rd.read(b, 2);
				const uint16_t v = (uint16_t)(b[0] | (b[1] << 8));
				cmap[i] = hd.cm_depth == 15 ? tgaColor15(v) : tgaColor16(v);
			}
			else if(hd.cm_depth == 24) { rd.read(b, 3); cmap[i] = tgaColor24(b); }
			else { rd.read(b, 4); cmap[i] = tgaColor32(b); }
		}
	}
	const int W = hd.width, H = hd.height;
	int min_x = 0, max_x = W, step_x = 1, min_y = 0, max_y = H, step_y = 1;
	if(!((hd.desc & 0x20) >> 5)) { min_y = H - 1; max_y = -1; step_y = -1; }
	if((hd.desc & 0x10) >> 4) { min_x = W - 1; max_x = -1; step_x = -1; }
	const int bpp = hd.bit_depth == 8 ? 1 : hd.bit_depth <= 16 ? 2 : hd.bit_depth == 24 ? 3 : 4;
	auto decode = [&](const uint8_t *b) -> Rgba4 {
		switch(hd.bit_depth)
		{
			case 8:
				if(is_gray) return tgaGray8(b[0]);
				return b[0] < cmap.size() ? cmap[b[0]] : Rgba4{{0.f, 0.f, 0.f, 1.f}};
			case 15: return tgaColor15((uint16_t)(b[0] | (b[1] << 8)));
			case 16: return is_gray ? tgaGray16((uint16_t)(b[0] | (b[1] << 8))) : tgaColor16((uint16_t)(b[0] | (b[1] << 8)));
			case 24: return tgaColor24(b);
			default: return tgaColor32(b);
		}
	};
	auto put = [&](int x, int y, Rgba4 c) {
		linearRgbFromColorSpace(c.c, cs, gamma);
		img->setColor(x, y, c.c);
	};
	if(is_rle)
	{
		// readRleImage (:86-110)
		int x = min_x, y = min_y;
		while(!rd.eof && y != max_y)
		{
			uint8_t pack = 0;
			rd.read(&pack, 1);
			if(rd.eof) break;
			const bool rle_pack = (pack & 0x80) != 0;
			const int rep = (int)(pack & 0x7F) + 1;
			uint8_t b[4] = {0, 0, 0, 0};
			if(rle_pack) rd.read(b, bpp);
			for(int i = 0; i < rep && y != max_y; ++i)
			{
				if(!rle_pack) rd.read(b, bpp);
				put(x, y, decode(b));
				x += step_x;
				if(x == max_x) { x = min_x; y += step_y; }
			}
		}
	}
	else
	{
		// readDirectImage (:112-127)
		std::vector<uint8_t> raw((size_t)W * H * bpp);
		rd.read(raw.data(), raw.size());
		size_t i = 0;
		for(int y = min_y; y != max_y; y += step_y)
			for(int x = min_x; x != max_x; x += step_x)
			{
				put(x, y, decode(&raw[i * bpp]));
				++i;
			}
	}
	return img;
}

// ---------------------------------------------------------------------------------------------
// Radiance HDR (src/format/format_hdr.cc, include/format/format_hdr_util.h)
// ---------------------------------------------------------------------------------------------
namespace
{
struct Rgbe { uint8_t r, g, b, e; };
// RgbePixel::getRgba (format_hdr_util.h:98-107)
Rgba4 rgbeColor(const Rgbe &p)
{
	if(p.e)
	{
		const float f = std::ldexp(1.f, (int)p.e - (128 + 8));
		return {{f * p.r, f * p.g, f * p.b, 1.f}};
	}
	return {{0.f, 0.f, 0.f, 1.f}};
}
bool fgetsLine(Reader &rd, std::string &line)
{
	line.clear();
	if(rd.pos >= rd.d.size()) return false;
	while(rd.pos < rd.d.size() && line.size() < 999)
	{
		const char ch = (char)rd.d[rd.pos++];
		line.push_back(ch);
		if(ch == '\n') break;
	}
	return true;
}
} // namespace

static std::shared_ptr<HostImage> loadHdr(Logger &log, const std::string &name, const std::vector<uint8_t> &data, int cs, float gamma,
                                          bool grayscale)
{
	Reader rd(data);
	std::string line;
	// readHeader (:118-184)
	fgetsLine(rd, line);
	if(line.find("#?") == std::string::npos) { log.error("HDR: File is not a valid Radiance RBGE image..."); return nullptr; }
	for(;;)
	{
		if(!fgetsLine(rd, line)) line.clear();
		if(line == "" || line == "\n") break;
		size_t fp;
		if((fp = line.find("FORMAT=")) != std::string::npos)
		{
			if(line.substr(fp + 7).find("32-bit_rle_rgbe") == std::string::npos) { log.error("HDR: only RGBE images are supported"); return nullptr; }
		}
	}
	fgetsLine(rd, line);
	std::vector<std::string> tok;
	{
		std::istringstream is(line);
		std::string t;
		while(is >> t) tok.push_back(t);
	}
	if(tok.size() < 4) { log.error("HDR: bad size line in \"" + name + "\""); return nullptr; }
	const bool y_first = tok[0].find('Y') != std::string::npos;
	int wi = 3, hi = 1, xi = 2, yi = 0, f = 0, s = 1;
	if(!y_first) { wi = 1; hi = 3; xi = 0; yi = 2; f = 1; s = 0; }
	const int width = std::atoi(tok[wi].c_str()), height = std::atoi(tok[hi].c_str());
	const bool from_left = tok[xi].find('+') != std::string::npos;
	const bool from_top = tok[yi].find('-') != std::string::npos;
	int mn[2], mx[2], st[2];
	mn[f] = 0; mx[f] = height; st[f] = 1;
	mn[s] = 0; mx[s] = width; st[s] = 1;
	if(!from_left) { mn[s] = width - 1; mx[s] = -1; st[s] = -1; }
	if(!from_top) { mn[f] = height - 1; mx[f] = -1; st[f] = -1; }
	if(width <= 0 || height <= 0) { log.error("HDR: bad image size"); return nullptr; }
	// HDR: linear RGB, no optimisation (image.cc:72-79); type from getTypeFromSettings(true, grayscale)
	(void)cs; (void)gamma;
	auto img = std::make_shared<HostImage>(width, height, grayscale ? IMG_GRAY_ALPHA : IMG_COLOR_ALPHA, OPT_NONE);
	const int scan_width = y_first ? width : height;
	auto put = [&](int x, int y, const Rgbe &p) {
		Rgba4 c = rgbeColor(p);
		if(y_first) img->setColor(x, y, c.c);
		else img->setColor(y, x, c.c);
	};
	// readOrle (:186-229), including its put-loop, which advances by max_[1] and so stores only the
	// first pixel of the scanline
	auto readOrle = [&](int y, int sw) -> bool {
		std::vector<Rgbe> scan((size_t)std::max(1, sw), Rgbe{0, 0, 0, 0});
		int rshift = 0;
		for(int x = mn[1]; x < sw;)
		{
			Rgbe px;
			if(rd.read(&px, 4) != 4) { log.error("HDR: An error has occurred while reading RLE scanline header..."); return false; }
			if(px.r == 1 && px.g == 1 && px.b == 1)
			{
				int count = (int)px.e << rshift;
				if(count > sw - x) { log.error("HDR: Scanline width greater than image width..."); return false; }
				const Rgbe prev = x >= 1 ? scan[x - 1] : Rgbe{0, 0, 0, 0};
				while(count--) scan[x++] = prev;
				rshift += 8;
			}
			else
			{
				if(x >= 0) scan[x] = px;
				++x;
				rshift = 0;
			}
		}
		int j = 0;
		for(int x = mn[1]; x != mx[1]; x += mx[1])
		{
			put(x, y, scan[j]);
			++j;
			if(mx[1] == 0) break;
		}
		return true;
	};
	// readArle (:231-309)
	auto readArle = [&](int y, int sw) -> bool {
		std::vector<Rgbe> scan((size_t)std::max(1, sw), Rgbe{0, 0, 0, 0});
		for(int chan = 0; chan < 4; ++chan)
		{
			int j = 0;
			while(j < sw)
			{
				uint8_t count = 0;
				if(rd.read(&count, 1) != 1) { log.error("HDR: An error has occurred while reading ARLE scanline..."); return false; }
				if(count > 128)
				{
					count &= 0x7F;
					if(count + j > sw) { log.error("HDR: Run width greater than image width..."); return false; }
					uint8_t col = 0;
					if(rd.read(&col, 1) != 1) { log.error("HDR: An error has occurred while reading ARLE scanline..."); return false; }
					while(count--) (&scan[j++].r)[chan] = col;
				}
				else
				{
					if(count + j > sw) { log.error("HDR: Non-run width greater than image width or equal to zero..."); return false; }
					while(count--)
					{
						uint8_t col = 0;
						if(rd.read(&col, 1) != 1) { log.error("HDR: An error has occurred while reading ARLE scanline..."); return false; }
						(&scan[j++].r)[chan] = col;
					}
				}
			}
		}
		int j = 0;
		for(int x = mn[1]; x != mx[1]; x += st[1])
		{
			put(x, y, j < sw ? scan[j] : Rgbe{0, 0, 0, 0});
			++j;
		}
		return true;
	};
	if(scan_width < 8 || scan_width > 0x7fff)
	{
		for(int y = mn[0]; y != mx[0]; y += st[0])
			if(!readOrle(y, scan_width)) { log.error("HDR: An error has occurred while reading uncompressed scanline..."); return nullptr; }
		return img;
	}
	for(int y = mn[0]; y != mx[0]; y += st[0])
	{
		Rgbe px;
		if(rd.read(&px, 4) != 4) { log.error("HDR: An error has occurred while reading scanline start..."); return nullptr; }
		const int arle = (int)(px.b << 8 | px.e);
		if(px.r == 2 && px.g == 2 && arle < 0x8000)
		{
			if(arle > scan_width) { log.error("HDR: Error reading, invalid ARLE scanline width..."); return nullptr; }
			if(!readArle(y, arle)) return nullptr;
		}
		else
		{
			rd.pos -= 4;
			rd.eof = false;
			if(!readOrle(y, scan_width)) return nullptr;
		}
	}
	return img;
}

static bool readFile(const std::string &path, std::vector<uint8_t> &out)
{
	std::FILE *fp = std::fopen(path.c_str(), "rb");
	if(!fp) return false;
	std::fseek(fp, 0, SEEK_END);
	const long n = std::ftell(fp);
	std::fseek(fp, 0, SEEK_SET);
	out.resize(n > 0 ? (size_t)n : 0);
	const size_t got = out.empty() ? 0 : std::fread(out.data(), 1, out.size(), fp);
	std::fclose(fp);
	out.resize(got);
	return true;
}

// image.cc:38-100
std::shared_ptr<HostImage> createImage(Logger &log, const std::string &name, const ParamMap &p)
{
	int width = 100, height = 100;
	std::string type_str = "ColorAlpha", opt_str = "optimized", cs_str = "Raw_Manual_Gamma", filename;
	double gamma = 1.0;
	p.get("type", type_str);
	p.get("image_optimization", opt_str);
	p.get("filename", filename);
	p.get("width", width);
	p.get("height", height);
	p.get("color_space", cs_str);
	p.get("gamma", gamma);
	int opt = OPT_OPTIMIZED;
	if(opt_str == "none") opt = OPT_NONE;
	else if(opt_str == "compressed") opt = OPT_COMPRESSED;
	int type = IMG_NONE;
	if(type_str == "ColorAlpha") type = IMG_COLOR_ALPHA;
	else if(type_str == "Color") type = IMG_COLOR;
	else if(type_str == "GrayAlpha") type = IMG_GRAY_ALPHA;
	else if(type_str == "Gray") type = IMG_GRAY;
	int cs = colorSpaceFromName(cs_str, CS_RAW_MANUAL_GAMMA);
	std::shared_ptr<HostImage> img;
	if(filename.empty()) log.verbose("Image '" + name + "': creating empty image with width=" + std::to_string(width) + " height=" + std::to_string(height));
	else
	{
		// format.cc:40-66: the reference as built without optional libraries reads TGA and HDR
		std::string ext;
		const size_t dot = filename.find_last_of('.');
		if(dot != std::string::npos) ext = filename.substr(dot + 1);
		for(char &c : ext) c = (char)std::tolower((unsigned char)c);
		const bool grayscale = type == IMG_GRAY || type == IMG_GRAY_ALPHA;
		if(ext == "tga" || ext == "tpic" || ext == "hdr" || ext == "pic")
		{
			std::vector<uint8_t> data;
			const bool hdr = ext == "hdr" || ext == "pic";
			if(hdr)
			{
				cs = CS_LINEAR_RGB;   // image.cc:72-79: HDR forces linear RGB and no optimisation
				opt = OPT_NONE;
			}
			if(!readFile(filename, data)) log.error("Image '" + name + "': cannot open file " + filename);
			else img = hdr ? loadHdr(log, filename, data, cs, (float)gamma, grayscale) : loadTga(log, filename, data, opt, cs, (float)gamma, grayscale);
		}
		else log.error("Cannot process file, libYafaRay has not been built with support for image file format '" + ext + "'");
		if(img) log.info("Image '" + name + "': loaded from file '" + filename + "'");
		else log.error("Image '" + name + "': Couldn't load from file '" + filename + "', creating empty image with width=" + std::to_string(width) + " height=" + std::to_string(height));
	}
	if(!img)
	{
		// Image::factory(width, height, type, optimization) (image.cc:102-137)
		if(type == IMG_NONE) { log.error("Image '" + name + "': no valid image type, image not created"); return nullptr; }
		int o = opt;
		if(type == IMG_GRAY_ALPHA) o = OPT_NONE;
		if(type == IMG_GRAY && o == OPT_COMPRESSED) o = OPT_OPTIMIZED;
		img = std::make_shared<HostImage>(std::max(0, width), std::max(0, height), type, o);
	}
	img->color_space = cs;
	img->gamma = (float)gamma;
	return img;
}

// ---------------------------------------------------------------------------------------------
// ImageTexture::factory (texture_image.cc:477-596)
// ---------------------------------------------------------------------------------------------
bool createTexture(Logger &log, const std::map<std::string, std::shared_ptr<HostImage>> &images, const std::string &name,
                   const ParamMap &p, HostTexture &out)
{
	std::string type;
	if(!p.get("type", type)) { log.error("Texture '" + name + "': no type given"); return false; }
	if(type != "image")
	{
		log.error("Texture '" + name + "': texture type '" + type + "' is not evaluated by the GPU core (image textures only)");
		return false;
	}
	std::string image_name, interp_str, clip;
	bool normalmap = false;
	p.get("interpolate", interp_str);
	p.get("normalmap", normalmap);
	p.get("image_name", image_name);
	if(image_name.empty()) { log.error("ImageTexture: Required argument image_name not found for image texture"); return false; }
	auto it = images.find(image_name);
	if(it == images.end() || !it->second) { log.error("ImageTexture: Couldn't load image file, dropping texture."); return false; }
	HostTexture ht;
	ht.img = it->second;
	DevTexture &t = ht.t;
	t.w = ht.img->w;
	t.h = ht.img->h;
	if(interp_str == "none") t.interp = INTERP_NONE;
	else if(interp_str == "bicubic") t.interp = INTERP_BICUBIC;
	else t.interp = INTERP_BILINEAR;   // bilinear, and the mipmap modes without mipmap parameters
	ht.mipmap = interp_str == "mipmap_trilinear" || interp_str == "mipmap_ewa";
	bool rot90 = false, even = false, odd = true, mirror_x = false, mirror_y = false, clamp = false;
	int xrep = 1, yrep = 1;
	double minx = 0.0, miny = 0.0, maxx = 1.0, maxy = 1.0, cdist = 0.0;
	float intensity = 1.f, contrast = 1.f, saturation = 1.f, hue = 0.f, fr = 1.f, fg = 1.f, fb = 1.f;
	p.get("xrepeat", xrep);
	p.get("yrepeat", yrep);
	p.get("cropmin_x", minx);
	p.get("cropmin_y", miny);
	p.get("cropmax_x", maxx);
	p.get("cropmax_y", maxy);
	p.get("rot90", rot90);
	p.get("clipping", clip);
	p.get("even_tiles", even);
	p.get("odd_tiles", odd);
	p.get("checker_dist", cdist);
	p.get("mirror_x", mirror_x);
	p.get("mirror_y", mirror_y);
	p.get("adj_mult_factor_red", fr);
	p.get("adj_mult_factor_green", fg);
	p.get("adj_mult_factor_blue", fb);
	p.get("adj_intensity", intensity);
	p.get("adj_contrast", contrast);
	p.get("adj_saturation", saturation);
	p.get("adj_hue", hue);
	p.get("adj_clamp", clamp);
	t.xrep = xrep;
	t.yrep = yrep;
	// setCrop (:173-179)
	t.cropminx = (float)minx; t.cropmaxx = (float)maxx; t.cropminy = (float)miny; t.cropmaxy = (float)maxy;
	if((t.cropminx != 0.0) || (t.cropmaxx != 1.0)) t.flags |= TEXF_CROPX;
	if((t.cropminy != 0.0) || (t.cropmaxy != 1.0)) t.flags |= TEXF_CROPY;
	if(rot90) t.flags |= TEXF_ROT90;
	// string2Cliptype (:584-595)
	t.clip = CLIP_REPEAT;
	if(clip == "extend") t.clip = CLIP_EXTEND;
	else if(clip == "clip") t.clip = CLIP_CLIP;
	else if(clip == "clipcube") t.clip = CLIP_CLIPCUBE;
	else if(clip == "checker") t.clip = CLIP_CHECKER;
	if(even) t.flags |= TEXF_CHECK_EVEN;
	if(odd) t.flags |= TEXF_CHECK_ODD;
	t.checker_dist = (float)cdist;
	if(mirror_x) t.flags |= TEXF_MIRROR_X;
	if(mirror_y) t.flags |= TEXF_MIRROR_Y;
	// Texture::setAdjustments (texture.cc:134-192)
	t.intensity = intensity;
	t.contrast = contrast;
	t.saturation = saturation;
	t.hue = hue / 60.f;
	t.fr = fr; t.fg = fg; t.fb = fb;
	if(clamp) t.flags |= TEXF_CLAMP;
	if(intensity != 1.f || contrast != 1.f || saturation != 1.f || hue != 0.f || fr != 1.f || fg != 1.f || fb != 1.f || clamp) t.flags |= TEXF_ADJ;
	t.raw_cs = ht.img->color_space;
	t.raw_gamma = ht.img->gamma;
	if(normalmap) log.warning("Texture '" + name + "': normal maps only feed bump mapping, which the GPU core does not evaluate");
	out = ht;
	return true;
}

// ---------------------------------------------------------------------------------------------
// shader-node programs
// ---------------------------------------------------------------------------------------------
namespace
{
struct NodeDesc
{
	std::string name, type;
	DevNode d{};
	std::vector<std::string> deps;      // dependency names (getDependencies order)
	int slot[3] = {-1, -1, -1};         // which DevNode::in[] each dependency fills
	bool uses_uv_mipmap = false;
};

int blendFromName(const std::string &s, bool layer)
{
	if(s == "add") return BLEND_ADD;
	if(s == "multiply") return BLEND_MULT;
	if(s == "subtract") return BLEND_SUB;
	if(s == "screen") return BLEND_SCREEN;
	if(s == "divide") return layer ? BLEND_DIV : BLEND_MIX;   // MixNode has no divide variant (:663)
	if(s == "difference") return BLEND_DIFF;
	if(s == "darken") return BLEND_DARK;
	if(s == "lighten") return BLEND_LIGHT;
	if(s == "overlay") return layer ? BLEND_MIX : BLEND_OVERLAY;   // LayerNode: overlay commented out
	return BLEND_MIX;
}
} // namespace

bool buildNodeProgram(Logger &log, const std::map<std::string, int> &texture_index, const std::vector<HostTexture> &textures,
                      const std::string &mat, const ParamMap &mp, const std::list<ParamMap> &nodes, std::vector<DevNode> &prog,
                      int &diffuse_root, int &drefl_root, int &sigma_root)
{
	prog.clear();
	diffuse_root = drefl_root = sigma_root = -1;
	// ---- loadNodes (material_node.cc:102-169) ----
	std::map<std::string, NodeDesc> table;
	bool error = false;
	std::vector<const ParamMap *> node_params;
	for(const ParamMap &pm : nodes)
	{
		std::string element;
		if(pm.get("element", element)) { if(element != "shader_node") continue; }
		else log.warning("NodeMaterial: No element type given; assuming shader node");
		node_params.push_back(&pm);
		NodeDesc nd;
		if(!pm.get("name", nd.name)) { log.error("NodeMaterial: Name of shader node not specified!"); error = true; break; }
		if(table.count(nd.name)) { log.error("NodeMaterial: Multiple nodes with identically names!"); error = true; break; }
		if(!pm.get("type", nd.type)) { log.error("NodeMaterial: Type of shader node not specified!"); error = true; break; }
		DevNode &d = nd.d;
		for(int k = 0; k < 3; ++k) d.in[k] = -1;
		d.tex = -1;
		bool ok = true;
		if(nd.type == "texture_mapper")
		{
			// TextureMapperNode::factory (shader_node_basic.cc:305-375)
			std::string texname, option;
			if(!pm.get("texture", texname)) { log.error("TextureMapper: No texture given for texture mapper!"); ok = false; }
			else
			{
				auto ti = texture_index.find(texname);
				if(ti == texture_index.end()) { log.error("TextureMapper: texture '" + texname + "' does not exist!"); ok = false; }
				else
				{
					const HostTexture &ht = textures[ti->second];
					d.type = NODE_TEXMAP;
					d.tex = ti->second;
					d.coords = TC_GLOBAL;
					d.proj = PROJ_PLAIN;
					bool coords_unsupported = false;
					if(pm.get("texco", option))
					{
						if(option == "uv") d.coords = TC_UV;
						else if(option == "global") d.coords = TC_GLOBAL;
						else if(option == "orco") d.coords = TC_ORCO;
						else if(option == "transformed") d.coords = TC_TRANSFORMED;
						else if(option == "window" || option == "normal") coords_unsupported = true;
						// reflect / stick / stress / tangent: mapped as global (:156-161)
					}
					if(coords_unsupported)
					{
						log.error("Material '" + mat + "': texture coordinates '" + option + "' (camera-dependent) are not evaluated by the GPU core");
						return false;
					}
					if(pm.get("mapping", option))   // image textures are discrete (texture_image.h:67)
					{
						if(option == "plain") d.proj = PROJ_PLAIN;
						else if(option == "cube") d.proj = PROJ_CUBE;
						else if(option == "tube") d.proj = PROJ_TUBE;
						else if(option == "sphere") d.proj = PROJ_SPHERE;
					}
					float mtx[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
					auto pit = pm.items().find("transform");
					if(pit != pm.items().end() && pit->second.type == Param::Matrix && pit->second.vval.size() == 16)
						for(int k = 0; k < 16; ++k) mtx[k] = pit->second.vval[k];
					for(int k = 0; k < 16; ++k) d.mtx[k] = mtx[k];
					float scale[3] = {1.f, 1.f, 1.f}, offset[3] = {0.f, 0.f, 0.f};
					pm.getVec("scale", scale);
					pm.getVec("offset", offset);
					bool scalar = true;
					pm.get("do_scalar", scalar);
					int map[3] = {1, 2, 3};
					pm.get("proj_x", map[0]);
					pm.get("proj_y", map[1]);
					pm.get("proj_z", map[2]);
					for(int &m : map) m = std::min(3, std::max(0, m));
					d.map_x = map[0]; d.map_y = map[1]; d.map_z = map[2];
					for(int k = 0; k < 3; ++k) { d.scale[k] = scale[k]; d.offset[k] = 2 * offset[k]; }
					d.flags = scalar ? 1u : 0u;
					nd.uses_uv_mipmap = ht.mipmap && d.coords == TC_UV;
				}
			}
		}
		else if(nd.type == "value")
		{
			// ValueNode::factory (:389-398)
			float col[4] = {1.f, 1.f, 1.f, 1.f};
			float alpha = 1.f, val = 1.f;
			pm.getColor("color", col);
			pm.get("alpha", alpha);
			pm.get("scalar", val);
			d.type = NODE_VALUE;
			d.c0[0] = col[0]; d.c0[1] = col[1]; d.c0[2] = col[2]; d.c0[3] = alpha;
			d.f[0] = val;
		}
		else if(nd.type == "mix")
		{
			// MixNode::factory (:652-673) + configInputs (:432-470)
			float cfactor = 0.5f;
			std::string blend;
			pm.get("cfactor", cfactor);
			pm.get("blend_mode", blend);
			d.type = NODE_MIX;
			d.mode = blendFromName(blend, false);
			d.f[0] = d.mode == BLEND_MIX ? cfactor : 0.f;   // MixNode(cfactor); the variants keep cfactor_ = 0
			d.f[1] = d.f[2] = 0.f;                                            // val_1_ / val_2_ (left unset)
		}
		else if(nd.type == "layer")
		{
			// LayerNode::factory (:291-331)
			float def_col[4] = {1.f, 1.f, 1.f, 1.f};
			bool do_color = true, do_scalar = false, color_input = true, use_alpha = false, stencil = false, no_rgb = false, negative = false;
			double def_val = 1.0, colfac = 1.0, valfac = 1.0;
			std::string blend;
			pm.getColor("def_col", def_col);
			pm.get("colfac", colfac);
			pm.get("def_val", def_val);
			pm.get("valfac", valfac);
			pm.get("do_color", do_color);
			pm.get("do_scalar", do_scalar);
			pm.get("color_input", color_input);
			pm.get("use_alpha", use_alpha);
			pm.get("noRGB", no_rgb);
			pm.get("stencil", stencil);
			pm.get("negative", negative);
			pm.get("blend_mode", blend);
			d.type = NODE_LAYER;
			d.mode = blendFromName(blend, true);
			uint32_t fl = 0;
			if(no_rgb) fl |= LAYER_RGB_TO_INT;
			if(stencil) fl |= LAYER_STENCIL;
			if(negative) fl |= LAYER_NEGATIVE;
			if(do_color) fl |= LAYER_DO_COLOR;
			if(do_scalar) fl |= LAYER_DO_SCALAR;
			if(color_input) fl |= LAYER_COLOR_INPUT;
			if(use_alpha) fl |= LAYER_USE_ALPHA;
			d.flags = fl;
			d.c0[0] = def_col[0]; d.c0[1] = def_col[1]; d.c0[2] = def_col[2]; d.c0[3] = 1.f;   // Rgba{Rgb}
			d.f[0] = (float)colfac;
			d.f[1] = (float)valfac;
			d.f[2] = (float)def_val;
		}
		else
		{
			log.error("NodeMaterial: No shader node could be constructed.'" + nd.type + "'!");
			ok = false;
		}
		if(!ok) { error = true; break; }
		table[nd.name] = nd;
	}
	if(!error)
	{
		// configInputs (layer: shader_node_layer.cc:136-177; mix: shader_node_basic.cc:432-470)
		for(const ParamMap *pmp : node_params)
		{
			const ParamMap &pm = *pmp;
			std::string name;
			pm.get("name", name);
			NodeDesc &nd = table[name];
			std::string in;
			bool ok = true;
			if(nd.type == "layer")
			{
				if(pm.get("input", in)) { if(!table.count(in)) { log.warning("LayerNode: Couldn't get input " + in); ok = false; } else { nd.deps.push_back(in); nd.slot[nd.deps.size() - 1] = 0; } }
				else { log.warning("LayerNode: input not set"); ok = false; }
				if(ok && pm.get("upper_layer", in))
				{
					if(!table.count(in)) ok = false;
					else { nd.deps.push_back(in); nd.slot[nd.deps.size() - 1] = 1; }
				}
				else if(ok)
				{
					float uc[4] = {0.f, 0.f, 0.f, 0.f};
					if(!pm.getColor("upper_color", uc)) uc[0] = uc[1] = uc[2] = uc[3] = 0.f;
					for(int k = 0; k < 4; ++k) nd.d.c1[k] = uc[k];
					float uv = 0.f;
					if(!pm.get("upper_value", uv)) uv = 0.f;
					nd.d.f[3] = uv;
				}
			}
			else if(nd.type == "mix")
			{
				float c[4];
				if(pm.get("input1", in)) { if(!table.count(in)) { log.error("MixNode: Couldn't get input1 " + in); ok = false; } else { nd.deps.push_back(in); nd.slot[nd.deps.size() - 1] = 0; } }
				else if(pm.getColor("color1", c)) for(int k = 0; k < 4; ++k) nd.d.c0[k] = c[k];
				else { log.error("MixNode: Color1 not set"); ok = false; }
				if(ok)
				{
					if(pm.get("input2", in)) { if(!table.count(in)) { log.error("MixNode: Couldn't get input2 " + in); ok = false; } else { nd.deps.push_back(in); nd.slot[nd.deps.size() - 1] = 1; } }
					else if(pm.getColor("color2", c)) for(int k = 0; k < 4; ++k) nd.d.c1[k] = c[k];
					else { log.error("MixNode: Color2 not set"); ok = false; }
				}
				if(ok)
				{
					float v;
					if(pm.get("factor", in)) { if(!table.count(in)) { log.error("MixNode: Couldn't get factor " + in); ok = false; } else { nd.deps.push_back(in); nd.slot[nd.deps.size() - 1] = 2; } }
					else if(pm.get("value", v)) nd.d.f[0] = v;
					else { log.error("MixNode: Value not set"); ok = false; }
				}
			}
			if(!ok) { log.error("NodeMaterial: Shader node configuration failed! (name='" + name + "')"); error = true; break; }
		}
	}
	if(error) table.clear();
	// ---- parseNodes (material_node.cc:171-187) over the shinydiffuse roots (:579-605) ----
	static const char *roots[] = {"diffuse_shader", "mirror_color_shader", "bump_shader", "mirror_shader", "transparency_shader",
	                              "translucency_shader", "sigma_oren_shader", "diffuse_refl_shader", "IOR_shader", "wireframe_shader"};
	std::string root_node[10];
	for(int r = 0; r < 10; ++r)
	{
		std::string name;
		if(!mp.get(roots[r], name)) continue;
		if(table.count(name)) root_node[r] = name;
		else log.warning(std::string("Shader node ") + roots[r] + " '" + name + "' does not exist!");
	}
	for(int r = 0; r < 10; ++r)
		if(!root_node[r].empty() && r != 0 && r != 6 && r != 7)
		{
			log.error("Material '" + mat + "': shader node root '" + roots[r] +
			          "' is not evaluated by the GPU core (diffuse_shader / sigma_oren_shader / diffuse_refl_shader only)");
			return false;
		}
	// ---- the nodes the roots depend on, dependencies first (solveNodesOrder :60-100) ----
	std::map<std::string, int> placed;
	std::set<std::string> visiting;
	std::vector<std::string> order;
	std::function<bool(const std::string &)> place = [&](const std::string &n) -> bool {
		if(placed.count(n)) return true;
		if(visiting.count(n)) { log.error("NodeMaterial: cyclic shader node dependency at '" + n + "'"); return false; }
		visiting.insert(n);
		for(const std::string &dep : table[n].deps)
			if(!place(dep)) return false;
		visiting.erase(n);
		placed[n] = (int)order.size();
		order.push_back(n);
		return true;
	};
	for(int r : {0, 6, 7})
		if(!root_node[r].empty() && !place(root_node[r])) return false;
	if((int)order.size() > kMaxNodes) { log.error("Material '" + mat + "': more than " + std::to_string(kMaxNodes) + " shader nodes"); return false; }
	for(const std::string &n : order)
	{
		const NodeDesc &nd = table[n];
		if(nd.uses_uv_mipmap)
		{
			log.error("Material '" + mat + "': mipmap interpolation on uv coordinates (ray differentials) is not evaluated by the GPU core");
			return false;
		}
		DevNode d = nd.d;
		for(size_t k = 0; k < nd.deps.size(); ++k) d.in[nd.slot[k]] = placed[nd.deps[k]];
		prog.push_back(d);
	}
	if(!root_node[0].empty()) diffuse_root = placed[root_node[0]];
	if(!root_node[7].empty()) drefl_root = placed[root_node[7]];
	if(!root_node[6].empty()) sigma_root = placed[root_node[6]];
	return true;
}

} // namespace yafamd
