// Film load / save ("resume" films): the reference's binary ImageFilm file
// (src/render/imagefilm.cc:817-1130) — header "YAF_FILMv4_0_0\0", computer node, base sampling
// offset, sampling offset, width, height, cx0, cx1, cy0, cy1, layer count, then the weights
// (float per pixel, row-major) and each layer's unnormalised RGBA (4 floats per pixel).
// The GPU film keeps exactly these accumulators (GpuRenderer accum / weights), so a film written
// here and loaded back continues the render where it stopped.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace yafamd
{

class Logger;

namespace filmio
{

struct Film
{
	uint32_t computer_node = 0, base_sampling_offset = 0, sampling_offset = 0;
	int width = 0, height = 0, cx0 = 0, cx1 = 0, cy0 = 0, cy1 = 0;
	std::vector<float> weights;   // [height * width]
	std::vector<float> rgba;      // [height * width * 4], the "combined" layer
};

// film_load_save_mode (imagefilm.cc:89-91)
enum Mode { None = 0, Save = 1, LoadAndSave = 2 };
Mode parseMode(const std::string &s);

// ImageFilm::getFilmPath (imagefilm.cc:817-825): path + " - node NNNN.film"
std::string filmPath(const std::string &path, int computer_node);
// ImageFilm::imageFilmSave (imagefilm.cc:1020-1102)
bool save(Logger &log, const std::string &file, const Film &f);
// ImageFilm::imageFilmLoad (imagefilm.cc:827-938): false (warning logged) on a missing file, a bad
// header or a film whose size / borders / layer count differ from `expect`
bool load(Logger &log, const std::string &file, const Film &expect, Film &out);
// ImageFilm::imageFilmLoadAllInFolder (imagefilm.cc:940-1018): every "<base>*.film" next to `path`,
// in sorted order, summed into `acc` (weights, colours; offsets = max).  Returns true if any loaded.
bool loadAllInFolder(Logger &log, const std::string &path, Film &acc);
// ImageFilm::imageFilmFileBackup (imagefilm.cc:1104-1130): rename an existing film to "-previous.bak"
void backup(Logger &log, const std::string &file);

}   // namespace filmio
}   // namespace yafamd
