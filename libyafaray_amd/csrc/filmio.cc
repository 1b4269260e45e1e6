// Film load / save — see filmio.h.  Host-only file I/O; the GPU side is an upload of the loaded
// accumulators before the first pass and a download at pass boundaries / the end of the render.
#include "filmio.h"
#include "host.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <dirent.h>
#include <sys/stat.h>

namespace yafamd
{
namespace filmio
{

static const char kHeader[] = "YAF_FILMv4_0_0";

Mode parseMode(const std::string &s)
{
	if(s == "load-save") return LoadAndSave;
	if(s == "save") return Save;
	return None;
}

std::string filmPath(const std::string &path, int computer_node)
{
	char node[32];
	snprintf(node, sizeof(node), "%04d", computer_node);   // std::setfill('0') << std::setw(4)
	return path + " - node " + node + ".film";
}

bool save(Logger &log, const std::string &file, const Film &f)
{
	log.info("Saving internal ImageFilm file");
	FILE *fp = fopen(file.c_str(), "wb");
	if(!fp)
	{
		log.warning("imageFilm: could not open '" + file + "' for writing");
		return false;
	}
	const int32_t hdr[7] = {f.width, f.height, f.cx0, f.cx1, f.cy0, f.cy1, 1};
	const uint32_t offs[3] = {f.computer_node, f.base_sampling_offset, f.sampling_offset};
	bool ok = fwrite(kHeader, 1, sizeof(kHeader), fp) == sizeof(kHeader);   // string + its '\0' (file.cc:190-194)
	ok = ok && fwrite(offs, sizeof(uint32_t), 3, fp) == 3;
	ok = ok && fwrite(hdr, sizeof(int32_t), 7, fp) == 7;
	ok = ok && fwrite(f.weights.data(), sizeof(float), f.weights.size(), fp) == f.weights.size();
	ok = ok && fwrite(f.rgba.data(), sizeof(float), f.rgba.size(), fp) == f.rgba.size();
	fclose(fp);
	if(!ok) log.warning("imageFilm: error while writing '" + file + "'");
	return ok;
}

bool load(Logger &log, const std::string &file, const Film &expect, Film &out)
{
	log.info("imageFilm: Loading film from: \"" + file);
	FILE *fp = fopen(file.c_str(), "rb");
	if(!fp)
	{
		log.warning("imageFilm file '" + file + "' not found, canceling load operation");
		return false;
	}
	// File::read(std::string): characters up to the first '\0'
	std::string header;
	for(int c; (c = fgetc(fp)) != EOF && c != 0;) header += (char)c;
	if(header != kHeader)
	{
		log.warning("imageFilm file '" + file + "' does not contain a valid YafaRay image file");
		fclose(fp);
		return false;
	}
	uint32_t offs[3] = {0, 0, 0};
	int32_t dims[7] = {0, 0, 0, 0, 0, 0, 0};
	bool ok = fread(offs, sizeof(uint32_t), 3, fp) == 3;
	static const char *names[6] = {"Image width", "Image height", "Border cx0", "Border cx1", "Border cy0", "Border cy1"};
	const int want[7] = {expect.width, expect.height, expect.cx0, expect.cx1, expect.cy0, expect.cy1, 1};
	for(int k = 0; ok && k < 7; ++k)
	{
		ok = fread(&dims[k], sizeof(int32_t), 1, fp) == 1;
		if(ok && dims[k] != want[k])
		{
			log.warning(std::string("imageFilm: loading/reusing film check failed. ") + (k < 6 ? names[k] : "Number of image layers") +
			            ", expected=" + std::to_string(want[k]) + ", in reused/loaded film=" + std::to_string(dims[k]));
			fclose(fp);
			return false;
		}
	}
	out = expect;
	out.computer_node = offs[0];
	out.base_sampling_offset = offs[1];
	out.sampling_offset = offs[2];
	const size_t n = (size_t)expect.width * expect.height;
	out.weights.assign(n, 0.f);
	out.rgba.assign(4 * n, 0.f);
	// a short file leaves the rest of the film at zero, as the reference's unchecked reads do
	ok = ok && fread(out.weights.data(), sizeof(float), n, fp) == n;
	ok = ok && fread(out.rgba.data(), sizeof(float), 4 * n, fp) == 4 * n;
	fclose(fp);
	if(!ok) log.warning("imageFilm: film file '" + file + "' is truncated");
	return true;
}

static bool isRegularFile(const std::string &p)
{
	struct stat st;
	return ::lstat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

// Path(full_path) (file.cc:45-73): directory before the last separator, base name before the last dot
static void splitPath(const std::string &full, std::string &dir, std::string &base, std::string &ext)
{
	std::string name = full;
	const size_t sep = full.find_last_of("\\/");
	dir = sep != std::string::npos ? full.substr(0, sep) : std::string();
	if(sep != std::string::npos) name = full.substr(sep + 1);
	const size_t dot = name.find_last_of('.');
	base = dot != std::string::npos ? name.substr(0, dot) : name;
	ext = dot != std::string::npos ? name.substr(dot + 1) : std::string();
}

bool loadAllInFolder(Logger &log, const std::string &path, Film &acc)
{
	log.info("Loading ImageFilm files");
	std::string dir, base_image, ext;
	splitPath(path, dir, base_image, ext);
	if(dir.empty()) dir = ".";
	std::vector<std::string> films;
	if(DIR *d = opendir(dir.c_str()))
	{
		while(const dirent *e = readdir(d))
		{
			const std::string name = e->d_name;
			if(name == "." || name == "..") continue;
			const std::string full = dir + "//" + name;
			if(!isRegularFile(full)) continue;
			std::string fd, fb, fe;
			splitPath(name, fd, fb, fe);
			if(fe == "film" && fb.rfind(base_image, 0) == 0) films.push_back(full);
		}
		closedir(d);
	}
	std::sort(films.begin(), films.end());
	bool any = false;
	for(const auto &file : films)
	{
		Film f;
		if(!load(log, file, acc, f))
		{
			log.warning("ImageFilm: Could not load film file '" + file + "'");
			continue;
		}
		any = true;
		for(size_t i = 0; i < acc.weights.size(); ++i) acc.weights[i] = acc.weights[i] + f.weights[i];
		for(size_t i = 0; i < acc.rgba.size(); ++i) acc.rgba[i] = acc.rgba[i] + f.rgba[i];
		acc.sampling_offset = std::max(acc.sampling_offset, f.sampling_offset);
		acc.base_sampling_offset = std::max(acc.base_sampling_offset, f.base_sampling_offset);
	}
	return any;
}

void backup(Logger &log, const std::string &file)
{
	log.info("Creating backup of the previous ImageFilm file...");
	if(!isRegularFile(file)) return;
	const std::string bak = file + "-previous.bak";
	::remove(bak.c_str());
	if(::rename(file.c_str(), bak.c_str()) != 0) log.warning("imageFilm: error during imageFilm file backup");
}

}   // namespace filmio
}   // namespace yafamd
