// Photon map files (photon_maps_processing "generate-save" / "load"): the reference's binary
// PhotonMap file (src/photon/photon.cc:54-110) — "YAF_PHOTONMAPv1\0", the map name (NUL
// terminated), paths (int32), search radius (float), kd-tree threads (int32), photon count
// (uint32), then per photon position xyz and colour rgb (6 floats, append order).
//
// The reference format carries no photon directions: PhotonMap::load resizes the photon vector
// with Photon(), which leaves dir_ uninitialised (photon.h:33, 87), so a loaded map's diffuse
// estimates see whatever that memory held — zero in practice (fresh pages), which is what a file
// without directions gives here.  Files written by this library append a direction block after
// the reference payload ("YAFAMD_PHOTON_DIRSv1\0", count, 3 floats per photon): the reference's
// loader stops before it (it reads exactly the v1 payload), and the loader here restores the
// directions, so a saved and re-loaded map renders bit-identically to the generated one.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace yafamd
{

class Logger;

namespace photonfile
{

struct Map
{
	std::string name;
	int32_t paths = 0;              // PhotonMap::paths_ (shot paths the estimates divide by)
	float search_radius = 1.f;      // PhotonMap::search_radius_ (never set by the integrators: 1)
	int32_t threads_pkd_tree = 1;   // PhotonMap::threads_pkd_tree_ (threads_photons)
	std::vector<float> pos;         // 3 per photon
	std::vector<float> col;         // 3 per photon
	std::vector<float> dir;         // 3 per photon; all zero when the file has no direction block
	bool has_dir = false;
	uint32_t size() const { return (uint32_t)(pos.size() / 3); }
};

// PhotonMap::load (photon.cc:54-87): false with a warning on a missing file or a bad header
bool load(Logger &log, const std::string &file, Map &out);
// PhotonMap::save (photon.cc:89-110) + the direction block
bool save(Logger &log, const std::string &file, const Map &m);

}   // namespace photonfile
}   // namespace yafamd
