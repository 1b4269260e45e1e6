// Host side of image textures and shader nodes: image loading (TGA, Radiance HDR) into the
// reference's image buffer types, ImageTexture parameters, and per-material shader-node programs
// (the node tree flattened in dependency order for texeval.h on the device).
//
// Reference: src/image/image.cc:38-137 (Image::factory), include/image/image_buffers.h (buffer
// quantisation), src/format/format_tga.cc, src/format/format_hdr.cc, src/format/format.cc:40-66,
// src/texture/texture_image.cc:477-596 (ImageTexture::factory), src/material/material_node.cc
// (loadNodes / parseNodes / solveNodesOrder), src/shader/shader_node_basic.cc and
// src/shader/shader_node_layer.cc (node factories and configInputs).
#pragma once

#include "host.h"

#include <list>
#include <memory>
#include <string>
#include <vector>

namespace yafamd
{

// Image::Type / Image::Optimization (include/image/image.h:47-48), same numbering
enum : int { IMG_NONE = 0, IMG_GRAY = 1, IMG_GRAY_ALPHA = 2, IMG_COLOR = 3, IMG_COLOR_ALPHA = 4 };
enum : int { OPT_NONE = 0, OPT_OPTIMIZED = 1, OPT_COMPRESSED = 2 };

struct HostImage
{
	int w = 0, h = 0;
	int type = IMG_COLOR_ALPHA, opt = OPT_OPTIMIZED;
	int color_space = CS_RAW_MANUAL_GAMMA;
	float gamma = 1.f;
	std::vector<float> px;     // getColor() per texel (RGBA), row-major y * w + x

	HostImage(int width, int height, int t, int o);
	// Image::setColor through the buffer class of (type, optimization) — the stored value is what
	// that buffer's getColor() returns afterwards
	void setColor(int x, int y, const float c[4]);
	void getColor(int x, int y, float c[4]) const;
};

// Image::factory(logger, scene, name, params) (image.cc:38-100); nullptr on failure (logged)
std::shared_ptr<HostImage> createImage(Logger &log, const std::string &name, const ParamMap &p);

struct HostTexture
{
	DevTexture t{};
	std::shared_ptr<HostImage> img;
	bool mipmap = false;       // mipmap_trilinear / mipmap_ewa requested
};

// Texture::factory for type "image" (texture_image.cc:477-596); false on failure (logged)
bool createTexture(Logger &log, const std::map<std::string, std::shared_ptr<HostImage>> &images, const std::string &name,
                   const ParamMap &p, HostTexture &out);

// ShinyDiffuseMaterial node setup (material_shiny_diffuse.cc:579-660 + material_node.cc:60-170):
// loads the node list, resolves the roots named in `mp`, and flattens the nodes the supported
// roots depend on into `prog` (evaluation order).  A node-list failure clears every node, as the
// reference does (the material then uses its plain colours).  Returns false (logged) only for
// features the GPU core does not evaluate (roots other than diffuse_shader / diffuse_refl_shader,
// unsupported coordinates, mipmap interpolation on uv coordinates).
bool buildNodeProgram(Logger &log, const std::map<std::string, int> &texture_index, const std::vector<HostTexture> &textures,
                      const std::string &mat, const ParamMap &mp, const std::list<ParamMap> &nodes, std::vector<DevNode> &prog,
                      int &diffuse_root, int &drefl_root, int &sigma_root);

} // namespace yafamd
