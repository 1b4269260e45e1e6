// Photon map files: see photonfile.h (reference src/photon/photon.cc:54-110, common/file.cc:169-200).
#include "photonfile.h"
#include "host.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>

namespace yafamd
{
namespace photonfile
{

namespace
{

const char kHeader[] = "YAF_PHOTONMAPv1";
const char kDirBlock[] = "YAFAMD_PHOTON_DIRSv1";

struct FileCloser { void operator()(FILE *f) const { if(f) fclose(f); } };
using FilePtr = std::unique_ptr<FILE, FileCloser>;

// File::read(std::string) (file.cc:169-181): characters up to the NUL; false at the end of the file
bool readString(FILE *fp, std::string &s, size_t max_len = 4096)
{
	s.clear();
	for(;;)
	{
		const int c = fgetc(fp);
		if(c == EOF) return false;
		if(c == 0) return true;
		if(s.size() >= max_len) return false;
		s += (char)c;
	}
}

template<typename T> bool readPod(FILE *fp, T &v) { return fread(&v, sizeof(T), 1, fp) == 1; }
template<typename T> bool writePod(FILE *fp, const T &v) { return fwrite(&v, sizeof(T), 1, fp) == 1; }
// File::append(std::string) (file.cc:190-194): the characters and a NUL
bool writeString(FILE *fp, const std::string &s) { return fwrite(s.c_str(), 1, s.size() + 1, fp) == s.size() + 1; }

}   // namespace

bool load(Logger &log, const std::string &file, Map &out)
{
	out = Map{};
	FilePtr fp(fopen(file.c_str(), "rb"));
	if(!fp)
	{
		log.warning("PhotonMap file '" + file + "' not found, canceling load operation");
		return false;
	}
	std::string header;
	if(!readString(fp.get(), header) || header != kHeader)
	{
		log.warning("PhotonMap file '" + file + "' does not contain a valid YafaRay photon map");
		return false;
	}
	uint32_t n = 0;
	if(!readString(fp.get(), out.name) || !readPod(fp.get(), out.paths) || !readPod(fp.get(), out.search_radius) ||
	   !readPod(fp.get(), out.threads_pkd_tree) || !readPod(fp.get(), n))
	{
		log.warning("PhotonMap file '" + file + "' is truncated");
		return false;
	}
	// the reference reads position xyz then colour rgb per photon (photon.cc:78-85).  The count comes
	// from the file: check that the file holds that many records before allocating for them (a corrupt
	// count would otherwise ask for up to 96 GB and throw)
	const long here = std::ftell(fp.get());
	if(here < 0 || std::fseek(fp.get(), 0, SEEK_END) != 0)
	{
		log.warning("PhotonMap file '" + file + "' is truncated");
		return false;
	}
	const long end = std::ftell(fp.get());
	if(end < here || (uint64_t)(end - here) < (uint64_t)n * 24u || std::fseek(fp.get(), here, SEEK_SET) != 0)
	{
		log.warning("PhotonMap file '" + file + "' is truncated");
		out = Map{};
		return false;
	}
	std::vector<float> rec((size_t)n * 6);
	if(n && fread(rec.data(), sizeof(float) * 6, n, fp.get()) != n)
	{
		log.warning("PhotonMap file '" + file + "' is truncated");
		out = Map{};
		return false;
	}
	out.pos.resize((size_t)n * 3);
	out.col.resize((size_t)n * 3);
	out.dir.assign((size_t)n * 3, 0.f);
	for(size_t i = 0; i < n; ++i)
		for(int c = 0; c < 3; ++c)
		{
			out.pos[i * 3 + c] = rec[i * 6 + c];
			out.col[i * 3 + c] = rec[i * 6 + 3 + c];
		}
	// the direction block of this library's files (absent from the reference's)
	std::string tag;
	uint32_t nd = 0;
	if(readString(fp.get(), tag, sizeof(kDirBlock)) && tag == kDirBlock && readPod(fp.get(), nd) && nd == n &&
	   (n == 0 || fread(out.dir.data(), sizeof(float) * 3, n, fp.get()) == n))
		out.has_dir = true;
	else
		std::fill(out.dir.begin(), out.dir.end(), 0.f);
	return true;
}

bool save(Logger &log, const std::string &file, const Map &m)
{
	FilePtr fp(fopen(file.c_str(), "wb"));
	if(!fp)
	{
		log.error("PhotonMap: cannot write '" + file + "'");
		return false;
	}
	const uint32_t n = m.size();
	bool ok = writeString(fp.get(), kHeader) && writeString(fp.get(), m.name) && writePod(fp.get(), m.paths) &&
	          writePod(fp.get(), m.search_radius) && writePod(fp.get(), m.threads_pkd_tree) && writePod(fp.get(), n);
	std::vector<float> rec((size_t)n * 6);
	for(size_t i = 0; i < n; ++i)
		for(int c = 0; c < 3; ++c)
		{
			rec[i * 6 + c] = m.pos[i * 3 + c];
			rec[i * 6 + 3 + c] = m.col[i * 3 + c];
		}
	ok = ok && (n == 0 || fwrite(rec.data(), sizeof(float) * 6, n, fp.get()) == n);
	if(m.dir.size() == m.pos.size())
		ok = ok && writeString(fp.get(), kDirBlock) && writePod(fp.get(), n) && (n == 0 || fwrite(m.dir.data(), sizeof(float) * 3, n, fp.get()) == n);
	ok = fflush(fp.get()) == 0 && ok;
	if(!ok) log.error("PhotonMap: writing '" + file + "' failed");
	return ok;
}

}   // namespace photonfile
}   // namespace yafamd
