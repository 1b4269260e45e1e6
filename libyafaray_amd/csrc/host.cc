// Host side: logger, scene assembly and render orchestration (see host.h).
#include "host.h"
#include "filmio.h"
#include "hostmath.h"
#include "render.h"
#include "texture.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <random>
#include <set>
#include <sstream>
#include <thread>

namespace yafamd
{

// ---------------------------------------------------------------------------------------------
// Logger (include/common/logger.h:62-166)
// ---------------------------------------------------------------------------------------------
void Logger::log(int level, const std::string &msg, bool set_error)
{
	std::lock_guard<std::mutex> g(mtx_);
	if(set_error) last_error_ = msg;
	const std::time_t now = std::time(nullptr);
	char tod[16];
	std::strftime(tod, sizeof(tod), "%H:%M:%S", std::localtime(&now));
	if(cb_ && level <= log_level_) cb_((yafaray_LogLevel_t)level, (long)now, tod, msg.c_str(), data_);
	if(console_ == YAFARAY_DISPLAY_CONSOLE_NORMAL && level <= console_level_)
	{
		static const char *names[] = {"", "ERROR", "WARNING", "PARAMS", "INFO", "VERB", "DEBUG"};
		std::fprintf(level <= YAFARAY_LOG_LEVEL_WARNING ? stderr : stdout, "[%s] %s: %s\n", print_datetime_ ? tod : "",
		             names[std::min(std::max(level, 0), 6)], msg.c_str());
	}
}

std::string ParamMap::print() const
{
	std::ostringstream os;
	for(const auto &kv : map_)
	{
		os << kv.first << "=";
		const Param &p = kv.second;
		switch(p.type)
		{
			case Param::Int: os << p.ival; break;
			case Param::Bool: os << (p.bval ? "true" : "false"); break;
			case Param::Float: os << p.fval; break;
			case Param::String: os << p.sval; break;
			default:
				os << "(";
				for(size_t i = 0; i < p.vval.size(); ++i) os << (i ? "," : "") << p.vval[i];
				os << ")";
		}
		os << " ";
	}
	return os.str();
}

// ---------------------------------------------------------------------------------------------
// small float vector helpers with the reference's operation order (vector.h:108-276)
// ---------------------------------------------------------------------------------------------
namespace
{
struct F3 { float x, y, z; };
inline F3 sub(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline F3 add(F3 a, F3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline F3 mul(F3 v, float f) { return {f * v.x, f * v.y, f * v.z}; }
inline F3 crs(F3 a, F3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float lsq(F3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
inline F3 nrm(F3 v)
{
	float len = lsq(v);
	if(len != 0.f)
	{
		len = 1.f / std::sqrt(len);
		v.x *= len; v.y *= len; v.z *= len;
	}
	return v;
}
inline float normLen(F3 &v)
{
	float vl = lsq(v);
	if(vl != 0.f)
	{
		vl = std::sqrt(vl);
		const float d = 1.f / vl;
		v.x *= d; v.y *= d; v.z *= d;
	}
	return vl;
}
inline F3 f3(const float *p) { return {p[0], p[1], p[2]}; }
inline void put(float *dst, F3 v, float w = 0.f) { dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = w; }
} // namespace

// ---------------------------------------------------------------------------------------------
// Scene
// ---------------------------------------------------------------------------------------------
Scene::Scene(Logger &l) : log(l) {}
Scene::~Scene() = default;

GpuRenderer *Scene::gpu()
{
	if(!gpu_) gpu_.reset(new GpuRenderer(log));
	return gpu_.get();
}

GpuRenderer *Scene::member(int m) { return m == 0 ? gpu() : extra_[(size_t)m - 1].get(); }

const KernelTimes &Scene::kernelTimes()
{
	if(kt_sum_) return *kt_sum_;
	return gpu()->kernelTimes();
}

// The device group of this process (the analogue of the reference's render threads, scene.cc:547-610
// and integrator_tiled.cc:246-264: there `threads` workers share the film's tiles; here one member per
// GPU renders a row band of it).  Member 0 is the renderer on the caller's current device; a render
// group over RCCL (one process per GPU) has exactly one member per process.
bool Scene::syncMembers()
{
	if(!gpu()->ready()) return false;
	const int count = GpuRenderer::deviceCount();
	const int d0 = gpu()->device();
	std::vector<int> devs;
	if(gpu()->groupWorld() > 1) devs = {d0};
	else if(!device_group.empty())
	{
		for(size_t m = 0; m < device_group.size(); ++m)
		{
			const int d = device_group[m] >= 0 ? device_group[m] : (int)((d0 + (int)m) % std::max(1, count));
			if(d >= count)
			{
				log.error("Device group: device " + std::to_string(d) + " requested, " + std::to_string(count) + " visible");
				return false;
			}
			devs.push_back(d);
		}
	}
	else
	{
		int n = setup.gpus;
		if(const char *e = getenv("YAFARAY_AMD_GPUS"); e && *e) n = atoi(e);
		if(n <= 0 || n > count) n = count;
		devs.push_back(d0);
		for(int d = 0; d < count && (int)devs.size() < n; ++d)
			if(d != d0) devs.push_back(d);
	}
	if(devs == member_devs_) return true;
	extra_.clear();
	if(devs[0] != d0)
	{
		if(gpu()->groupWorld() > 1)
		{
			log.error("Device group: a render-group member renders on its own device only");
			return false;
		}
		gpu_.reset(new GpuRenderer(log, devs[0]));
		if(!gpu_->ready()) return false;
	}
	for(size_t m = 1; m < devs.size(); ++m) extra_.emplace_back(new GpuRenderer(log, devs[m]));
	{
		const std::set<int> uniq(devs.begin(), devs.end());
		GpuRenderer::enablePeerAccess(std::vector<int>(uniq.begin(), uniq.end()));
	}
	member_devs_ = devs;
	geometry_dirty = true;   // every member holds its own copy of the scene
	group_bounds.clear();
	kt_sum_.reset();
	if(devs.size() > 1)
	{
		std::ostringstream os;
		os << "Device group: " << devs.size() << " members on devices";
		for(int d : devs) os << " " << d;
		log.info(os.str());
	}
	return true;
}

// What the last render's split looked like, for a caller that wants to check or log it (bench.py's
// multi-GPU line): the group kind, the members' devices, which device pairs can access each other
// directly (hipDeviceCanAccessPeer: the band copies then run over xGMI without staging), how the bands
// travel, the band boundaries the render used and each member's render time.
std::string Scene::groupReport()
{
	std::ostringstream os;
	auto list = [&os](const auto &v) {
		os << "[";
		for(size_t k = 0; k < v.size(); ++k) os << (k ? ", " : "") << v[k];
		os << "]";
	};
	const int gw = gpu_ ? gpu_->groupWorld() : 1;
	const int n = gw > 1 ? gw : memberCount();
	const char *mode = gw > 1 ? "render group" : n > 1 ? "device group" : "one GPU";
	os << "{\"mode\": \"" << mode << "\", \"members\": " << n;
	if(gw > 1) os << ", \"rank\": " << gpu_->groupRank() << ", \"device\": " << gpu_->device();
	std::vector<int> devs = member_devs_;
	if(gw > 1 && gpu_) devs = {gpu_->device()};
	os << ", \"devices\": ";
	list(devs);
	// peer-access matrix over the distinct devices of this process's members
	const std::set<int> uniq(devs.begin(), devs.end());
	const std::vector<int> ud(uniq.begin(), uniq.end());
	bool all_peer = true;
	os << ", \"peer_devices\": ";
	list(ud);
	os << ", \"peer_access\": [";
	for(size_t a = 0; a < ud.size(); ++a)
	{
		os << (a ? ", " : "") << "[";
		for(size_t b = 0; b < ud.size(); ++b)
		{
			int can = a == b ? 1 : 0;
			if(a != b && hipDeviceCanAccessPeer(&can, ud[a], ud[b]) != hipSuccess) can = 0;
			if(a != b && !can) all_peer = false;
			os << (b ? ", " : "") << can;
		}
		os << "]";
	}
	os << "]";
	const char *path = "none (one member)";
	if(gw > 1) path = "RCCL all-gather of band slots (xGMI between GPUs)";
	else if(n > 1 && ud.size() == 1) path = "hipMemcpyPeerAsync between logical members of one device (device-to-device copy)";
	else if(n > 1) path = all_peer ? "hipMemcpyPeerAsync with peer access enabled (direct xGMI)" : "hipMemcpyPeerAsync, staged (no peer access on some pair)";
	os << ", \"copy_path\": \"" << path << "\", \"bounds\": ";
	list(last_bounds_);
	os << ", \"member_ms\": ";
	list(last_member_ms_);
	os << ", \"next_bounds\": ";
	list(group_bounds);
	os << "}";
	return os.str();
}

// One film rendered by every member of the device group, each on its own host thread (member 0 on
// the caller's): row bands + halo rows; the members meet between adaptive passes and at the end,
// where member 0 pulls every band over xGMI (GpuRenderer::renderMember / exchangeRows).
bool Scene::renderDeviceGroup(RenderParams &rp)
{
	const int n = memberCount();
	std::vector<GpuRenderer *> ms;
	for(int m = 0; m < n; ++m) ms.push_back(member(m));
	auto group = std::make_shared<PeerGroup>(ms);
	std::vector<RenderParams> rps((size_t)n, rp);
	std::vector<char> ok((size_t)n, 0);
	for(int m = 0; m < n; ++m)
	{
		RenderParams &r = rps[(size_t)m];
		r.shard_rank = m;
		r.shard_y0 = rp.band_bounds[(size_t)m];
		r.shard_y1 = rp.band_bounds[(size_t)m + 1];
		r.pm.write_files = m == 0;
		if(m > 0)
		{
			// the client's callbacks run on the caller's thread only (member 0)
			r.on_chunk = nullptr;
			r.on_next_pass = nullptr;
			r.on_tiles = nullptr;
		}
		ms[(size_t)m]->setPeers(group, m);
	}
	std::vector<std::thread> th;
	for(int m = 1; m < n; ++m) th.emplace_back([&, m] { ok[(size_t)m] = ms[(size_t)m]->renderMember(rps[(size_t)m], &canceled) ? 1 : 0; });
	ok[0] = ms[0]->renderMember(rps[0], &canceled) ? 1 : 0;
	for(std::thread &t : th) t.join();
	for(GpuRenderer *g : ms) g->setPeers(nullptr, 0);
	rp.pm.processing = rps[0].pm.processing;
	// counters and per-kernel times summed over the members (GPU time), wall time of the slowest
	yafaray_amd_stats_t st = ms[0]->stats();
	if(!kt_sum_) kt_sum_.reset(new KernelTimes);
	*kt_sum_ = ms[0]->kernelTimes();
	for(int m = 1; m < n; ++m)
	{
		const yafaray_amd_stats_t &o = ms[(size_t)m]->stats();
		st.closest_rays += o.closest_rays;
		st.shadow_rays += o.shadow_rays;
		st.node_visits += o.node_visits;
		st.tri_tests += o.tri_tests;
		st.samples += o.samples;
		st.gather_visits += o.gather_visits;
		st.gather_queries += o.gather_queries;
		st.gather_photons += o.gather_photons;
		st.gather_accepts += o.gather_accepts;
		st.gather_overflows += o.gather_overflows;
		st.photon_paths_traced += o.photon_paths_traced;
		st.photon_slots += o.photon_slots;
		st.fg_paths += o.fg_paths;
		st.fg_lookups += o.fg_lookups;
		st.fg_nearest_visits += o.fg_nearest_visits;
		st.pregather_visits += o.pregather_visits;
		st.pregather_photons += o.pregather_photons;
		st.pkd_split_level = std::max(st.pkd_split_level, o.pkd_split_level);
		st.trace_kernel_ms += o.trace_kernel_ms;
		st.shade_kernel_ms += o.shade_kernel_ms;
		st.nee_kernel_ms += o.nee_kernel_ms;
		st.trace_launches += o.trace_launches;
		st.render_seconds = std::max(st.render_seconds, o.render_seconds);
		const KernelTimes &k = ms[(size_t)m]->kernelTimes();
		for(int q = 0; q < KK_COUNT; ++q)
		{
			kt_sum_->ms[q] += k.ms[q];
			kt_sum_->launches[q] += k.launches[q];
			kt_sum_->items[q] += k.items[q];
		}
	}
	group_stats_ = st;
	for(char c : ok)
		if(!c) return false;
	return true;
}

// scene.cc:977-1004, object_mesh.cc:35-86
bool Scene::createObject(const std::string &name, const ParamMap &p)
{
	if(objects.count(name)) { log.error("Scene: object '" + name + "' already exists"); return false; }
	std::string type = "mesh";
	p.get("type", type);
	if(type != "mesh") { log.error("Scene: object type '" + type + "' is not supported by the GPU core (meshes only)"); return false; }
	MeshObject &o = objects[name];
	o.name = name;
	p.get("is_base_object", o.is_base);
	p.get("visibility", o.visibility);
	// visibility::fromString (include/common/visibility.h:36-43): unknown strings are "normal"
	if(o.visibility == "shadow_only" || o.visibility == "no_shadows")
	{
		log.error("Scene: object '" + name + "' visibility '" + o.visibility + "' is not supported by the GPU core (normal / invisible)");
		objects.erase(name);
		return false;
	}
	int nv = 0, nf = 0;
	if(p.get("num_vertices", nv) && nv > 0) o.verts.reserve(3 * (size_t)nv);
	if(p.get("num_faces", nf) && nf > 0) { o.tris.reserve(3 * (size_t)nf); o.tri_mat.reserve(nf); }
	object_order.push_back(name);
	current_object = &o;
	geometry_dirty = true;
	return true;
}

bool Scene::endObject()
{
	if(!current_object) { log.error("Scene: endObject() without an object"); return false; }
	current_object->ended = true;
	current_object = nullptr;
	return true;
}

int Scene::addVertex(float x, float y, float z)
{
	if(!current_object) { log.error("Scene: addVertex() outside of an object"); return -1; }
	auto &v = current_object->verts;
	v.push_back(x);
	v.push_back(y);
	v.push_back(z);
	return (int)(v.size() / 3) - 1;
}

int Scene::addVertexWithOrco(float x, float y, float z, float ox, float oy, float oz)
{
	const int id = addVertex(x, y, z);
	if(id < 0) return id;
	// scene.cc:948-956: addPoint + addOrcoPoint (hasOrco() = orco list non-empty)
	auto &o = current_object->orco;
	o.push_back(ox);
	o.push_back(oy);
	o.push_back(oz);
	return id;
}

void Scene::addNormal(float x, float y, float z)
{
	// object_mesh.cc:111-116 (normals exported: faces added afterwards index them by vertex)
	if(!current_object) { log.error("Scene: addNormal() outside of an object"); return; }
	auto &n = current_object->normals;
	n.push_back(x);
	n.push_back(y);
	n.push_back(z);
}

int Scene::addUv(float u, float v)
{
	if(!current_object) { log.error("Scene: addUv() outside of an object"); return 0; }
	auto &uv = current_object->uvs;
	uv.push_back(u);
	uv.push_back(v);
	return (int)(uv.size() / 2) - 1;
}

bool Scene::addTriangle(int a, int b, int c, int uv_a, int uv_b, int uv_c)
{
	if(!current_object) { log.error("Scene: addTriangle() outside of an object"); return false; }
	const int nv = (int)(current_object->verts.size() / 3);
	if(a < 0 || b < 0 || c < 0 || a >= nv || b >= nv || c >= nv)
	{
		log.error("Scene: addTriangle() vertex index out of range in object '" + current_object->name + "'");
		return false;
	}
	auto it = material_index.find(current_material);
	if(it == material_index.end())
	{
		log.error("Scene: addTriangle() with no valid current material ('" + current_material + "')");
		return false;
	}
	const int nuv = (int)(current_object->uvs.size() / 2);
	if(uv_a >= nuv || uv_b >= nuv || uv_c >= nuv)
	{
		log.error("Scene: addTriangleWithUv() uv index out of range in object '" + current_object->name + "'");
		return false;
	}
	current_object->tris.push_back(a);
	current_object->tris.push_back(b);
	current_object->tris.push_back(c);
	current_object->tri_mat.push_back(it->second);
	current_object->tri_uv.push_back(uv_a);
	current_object->tri_uv.push_back(uv_b);
	current_object->tri_uv.push_back(uv_c);
	// object_mesh.cc:84: faces added after normals were exported use the vertex normals
	const bool exported = !current_object->normals.empty();
	current_object->tri_nidx.push_back(exported ? a : -1);
	current_object->tri_nidx.push_back(exported ? b : -1);
	current_object->tri_nidx.push_back(exported ? c : -1);
	return true;
}

HostImage *Scene::createImage(const std::string &name, const ParamMap &p)
{
	// scene.cc:518-521 createMapItem: an existing name is a warning, a missing type an error
	if(images.count(name)) { log.warning("Scene: Image '" + name + "' already exists!"); return nullptr; }
	std::string type;
	if(!p.get("type", type)) { log.error("Scene: Image '" + name + "': type not specified"); return nullptr; }
	std::shared_ptr<HostImage> img = yafamd::createImage(log, name, p);
	if(!img) { log.error("Scene: Image '" + name + "' could not be created"); return nullptr; }
	images[name] = img;
	return img.get();
}

bool Scene::createTexture(const std::string &name, const ParamMap &p)
{
	if(texture_index.count(name)) { log.warning("Scene: Texture '" + name + "' already exists!"); return false; }
	HostTexture t;
	if(!yafamd::createTexture(log, images, name, p, t)) return false;
	texture_index[name] = (int)textures.size();
	textures.push_back(t);
	return true;
}

// scene.cc:909-932 + object_mesh.cc:118-240 (MeshObject::smoothNormals)
bool Scene::smoothMesh(const std::string &name, float angle)
{
	MeshObject *o = nullptr;
	if(!name.empty())
	{
		auto it = objects.find(name);
		if(it == objects.end()) { log.error("Scene: smoothMesh(): object '" + name + "' not found"); return false; }
		o = &it->second;
	}
	else o = current_object;
	if(!o) return false;
	const size_t nv = o->verts.size() / 3, nt = o->tri_mat.size();
	if(!o->normals.empty() && o->normals.size() / 3 == nv) { o->smooth = true; return true; }
	struct V { float x, y, z; };
	auto P = [&](int i) { return V{o->verts[3 * (size_t)i], o->verts[3 * (size_t)i + 1], o->verts[3 * (size_t)i + 2]}; };
	auto sub3 = [](V a, V b) { return V{a.x - b.x, a.y - b.y, a.z - b.z}; };
	auto crs3 = [](V a, V b) { return V{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; };
	auto len3 = [](V a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); };
	auto nrm3 = [](V v) {
		float l = v.x * v.x + v.y * v.y + v.z * v.z;
		if(l != 0.f) { l = 1.f / std::sqrt(l); v.x *= l; v.y *= l; v.z *= l; }
		return v;
	};
	auto dot3 = [](V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; };
	// Vec3::sinFromVectors (vector.h:212-219) with math::asin's domain clamp (math.h:260-266)
	auto angleSine = [&](int a, int b, int c) {
		const V e1 = sub3(P(b), P(a)), e2 = sub3(P(c), P(a));
		const float div = (len3(e1) * len3(e2)) * 0.99999f + 0.00001f;
		float arg = (len3(crs3(e1, e2)) / div) * 0.99999f;
		if(arg > 1.f) arg = 1.f;
		if(arg <= -1.f) return static_cast<float>(-hm::div_pi_by_2);
		if(arg >= 1.f) return static_cast<float>(hm::div_pi_by_2);
		return std::asin(arg);
	};
	auto faceN = [&](size_t t) { return nrm3(crs3(sub3(P(o->tris[3 * t + 1]), P(o->tris[3 * t])), sub3(P(o->tris[3 * t + 2]), P(o->tris[3 * t])))); };
	std::vector<V> normals(nv, V{0.f, 0.f, 0.f});
	for(size_t i = 0; i < std::min(nv, o->normals.size() / 3); ++i) normals[i] = V{o->normals[3 * i], o->normals[3 * i + 1], o->normals[3 * i + 2]};
	if(o->tri_nidx.size() < 3 * nt) o->tri_nidx.resize(3 * nt, -1);
	if(angle >= 180)
	{
		for(size_t t = 0; t < nt; ++t)
		{
			const V n = faceN(t);
			const int *vi = &o->tris[3 * t];
			for(int r = 0; r < 3; ++r)
			{
				const float sn = angleSine(vi[r], vi[(r + 1) % 3], vi[(r + 2) % 3]);
				V &acc = normals[vi[r]];
				acc.x += n.x * sn; acc.y += n.y * sn; acc.z += n.z * sn;
				o->tri_nidx[3 * t + r] = vi[r];
			}
		}
		for(V &n : normals) n = nrm3(n);
	}
	else if(angle > 0.1f)
	{
		const float threshold = hm::cosf_fast(static_cast<float>(angle * hm::div_pi_by_180));
		std::vector<std::vector<size_t>> pfaces(nv);
		std::vector<std::vector<float>> psines(nv);
		for(size_t t = 0; t < nt; ++t)
		{
			const int *vi = &o->tris[3 * t];
			for(int r = 0; r < 3; ++r)
			{
				psines[vi[r]].push_back(angleSine(vi[r], vi[(r + 1) % 3], vi[(r + 2) % 3]));
				pfaces[vi[r]].push_back(t);
			}
		}
		for(size_t pid = 0; pid < nv; ++pid)
		{
			int j = 0;
			std::vector<V> vn;
			std::vector<int> vn_idx;
			for(size_t f : pfaces[pid])
			{
				bool smooth = false;
				const V fn = faceN(f);
				V vnorm{fn.x * psines[pid][j], fn.y * psines[pid][j], fn.z * psines[pid][j]};
				int k = 0;
				for(size_t f2 : pfaces[pid])
				{
					if(f == f2) { k++; continue; }
					const V fn2 = faceN(f2);
					if(dot3(fn, fn2) > threshold)
					{
						smooth = true;
						vnorm.x += fn2.x * psines[pid][k]; vnorm.y += fn2.y * psines[pid][k]; vnorm.z += fn2.z * psines[pid][k];
					}
					k++;
				}
				int nidx = -1;
				if(smooth)
				{
					vnorm = nrm3(vnorm);
					for(size_t q = 0; q < vn.size(); ++q)
						if(dot3(vnorm, vn[q]) > 0.999f) { nidx = vn_idx[q]; break; }
					if(nidx == -1)
					{
						nidx = (int)normals.size();
						vn.push_back(vnorm);
						vn_idx.push_back(nidx);
						normals.push_back(vnorm);
					}
				}
				for(int r = 0; r < 3; ++r)
					if(o->tris[3 * f + r] == (int)pid) { o->tri_nidx[3 * f + r] = nidx; break; }
				j++;
			}
		}
	}
	o->normals.clear();
	for(const V &n : normals) { o->normals.push_back(n.x); o->normals.push_back(n.y); o->normals.push_back(n.z); }
	o->smooth = true;
	geometry_dirty = true;
	return true;
}

// material_shiny_diffuse.cc:28-87 + 495-640, material_simple.cc:36-70
bool Scene::createMaterial(const std::string &name, const ParamMap &p, const std::list<ParamMap> &nodes)
{
	if(materials.count(name)) { log.error("Scene: material '" + name + "' already exists"); return false; }
	std::string type;
	p.get("type", type);
	DevMaterial m{};
	m.receive_shadows = 1;
	m.diffuse_root = m.drefl_root = m.sigma_root = -1;
	bool b;
	if(type == "shinydiffusemat")
	{
		float col[4] = {1.f, 1.f, 1.f, 1.f};
		p.getColor("color", col);
		float diffuse = 1.f, transparency = 0.f, translucency = 0.f, mirror = 0.f, emit = 0.f, ior = 1.33f, tfilter = 1.f;
		float tbias = 0.f, wire = 0.f;
		float mcol[4] = {1.f, 1.f, 1.f, 1.f};
		int add_depth = 0;
		bool fresnel = false, tbias_mult = false;
		p.get("diffuse_reflect", diffuse);
		p.get("transparency", transparency);
		p.get("translucency", translucency);
		p.get("specular_reflect", mirror);
		p.get("emit", emit);
		p.get("IOR", ior);
		p.get("transmit_filter", tfilter);
		p.get("fresnel_effect", fresnel);
		p.getColor("mirror_color", mcol);
		p.get("transparentbias_factor", tbias);
		p.get("transparentbias_multiply_raydepth", tbias_mult);
		p.get("wireframe_amount", wire);
		p.get("additionaldepth", add_depth);
		// material_shiny_diffuse.cc:561-571: diffuse_brdf "oren_nayar" -> initOrenNayar(sigma) (:146-152),
		// double arithmetic stored to the float A / B members
		std::string brdf;
		if(p.get("diffuse_brdf", brdf) && brdf == "oren_nayar")
		{
			double sigma = 0.1;
			p.get("sigma", sigma);
			const double sigma_squared = sigma * sigma;
			m.on_a = static_cast<float>(1.0 - 0.5 * (sigma_squared / (sigma_squared + 0.33)));
			m.on_b = static_cast<float>(0.45 * sigma_squared / (sigma_squared + 0.09));
			m.sd_flags |= SD_OREN_NAYAR;
		}
		m.add_depth = add_depth;
		if(wire > 0.f)
		{
			log.error("Material '" + name + "': wireframe shading (wireframe_amount > 0) is not supported by the GPU core");
			return false;
		}
		// shader nodes (material_shiny_diffuse.cc:579-660)
		std::vector<DevNode> prog;
		int droot = -1, rroot = -1, sroot = -1;
		if(!buildNodeProgram(log, texture_index, textures, name, p, nodes, prog, droot, rroot, sroot)) return false;
		m.n_nodes = (int)prog.size();
		m.diffuse_root = droot;
		m.drefl_root = rroot;
		m.sigma_root = (m.sd_flags & SD_OREN_NAYAR) ? sroot : -1;   // sigma_oren_shader_ is read by orenNayar only
		m.emit_strength = emit;
		if(!prog.empty()) mat_nodes[name] = prog;
		m.type = MAT_SHINYDIFFUSE;
		for(int k = 0; k < 3; ++k) m.diffuse[k] = col[k];
		for(int k = 0; k < 3; ++k) m.emit[k] = emit * col[k];     // emit_color_(emit_strength * diffuse_color)
		for(int k = 0; k < 3; ++k) m.mirror_col[k] = mcol[k];
		if(emit > 0.f) m.bsdf_flags |= B_EMIT;
		m.tfilter = tfilter;
		m.tbias = tbias;
		if(tbias_mult) m.sd_flags |= SD_TBIAS_MULT;
		if(fresnel) { m.sd_flags |= SD_FRESNEL; m.ior_sq = ior * ior; }   // :560-565
		// ShinyDiffuseMaterial::config (material_shiny_diffuse.cc:41-87): component order, flags
		float acc = 1.f;
		if(mirror > 0.00001f)
		{
			m.sd_flags |= SD_MIRROR;
			if(!fresnel) acc = 1.f - mirror;
			m.bsdf_flags |= B_SPECULAR | B_REFLECT;
			m.c_flags[m.n_bsdf] = B_SPECULAR | B_REFLECT;
			m.c_index[m.n_bsdf] = 0;
			++m.n_bsdf;
			m.comp[0] = mirror;
		}
		if(transparency * acc > 0.00001f)
		{
			m.sd_flags |= SD_TRANSPARENT;
			acc *= 1.f - transparency;
			m.bsdf_flags |= B_TRANSMIT | B_FILTER;
			m.c_flags[m.n_bsdf] = B_TRANSMIT | B_FILTER;
			m.c_index[m.n_bsdf] = 1;
			++m.n_bsdf;
			m.comp[1] = transparency;
		}
		if(translucency * acc > 0.00001f)
		{
			m.sd_flags |= SD_TRANSLUCENT;
			acc *= 1.f - transparency;   // sic (:68): the transparency strength
			m.bsdf_flags |= B_DIFFUSE | B_TRANSMIT;
			m.c_flags[m.n_bsdf] = B_DIFFUSE | B_TRANSMIT;
			m.c_index[m.n_bsdf] = 2;
			++m.n_bsdf;
			m.comp[2] = translucency;
		}
		if(diffuse * acc > 0.00001f)
		{
			m.sd_flags |= SD_DIFFUSE;
			m.bsdf_flags |= B_DIFFUSE | B_REFLECT;
			m.c_flags[m.n_bsdf] = B_DIFFUSE | B_REFLECT;
			m.c_index[m.n_bsdf] = 3;
			++m.n_bsdf;
			m.comp[3] = diffuse;
		}
		if(p.get("receive_shadows", b)) m.receive_shadows = b ? 1 : 0;
		if(p.get("flat_material", b)) m.flat = b ? 1 : 0;
	}
	else if(type == "light_mat")
	{
		float col[4] = {1.f, 1.f, 1.f, 1.f};
		double power = 1.0;
		bool ds = false;
		p.getColor("color", col);
		p.get("power", power);
		p.get("double_sided", ds);
		m.type = MAT_LIGHT;
		m.bsdf_flags = B_EMIT;
		for(int k = 0; k < 3; ++k) m.emit[k] = static_cast<float>(power) * col[k];
		m.double_sided = ds ? 1 : 0;
	}
	else if(type == "mirror")
	{
		// MirrorMaterial (material_glass.cc:453-460, material_glass.h:86-91): ref_col_ = color * reflect
		float col[4] = {1.f, 1.f, 1.f, 1.f};
		float refl = 1.f;
		p.getColor("color", col);
		p.get("reflect", refl);
		m.type = MAT_MIRROR;
		m.bsdf_flags = B_SPECULAR;
		for(int k = 0; k < 3; ++k) m.mirror_col[k] = col[k] * refl;
	}
	else if(type == "null")
	{
		m.type = MAT_NULL;   // NullMaterial: no BSDF components (material_glass.cc:463-473)
		m.bsdf_flags = B_NONE;
	}
	else
	{
		log.error("Scene: material type '" + type + "' is not supported by the GPU core");
		return false;
	}
	materials[name] = m;
	material_index[name] = (int)material_order.size();
	material_order.push_back(name);
	return true;
}

// light_point.cc:28-35 + 104-132, light_area.cc:33-53 + 168-204
bool Scene::createLight(const std::string &name, const ParamMap &p)
{
	std::string type;
	p.get("type", type);
	DevLight L{};
	float col[4] = {1.f, 1.f, 1.f, 1.f};
	float power = 1.f;
	bool enabled = true, cast = true, photon_only = false;
	p.getColor("color", col);
	p.get("power", power);
	p.get("light_enabled", enabled);
	p.get("cast_shadows", cast);
	p.get("photon_only", photon_only);
	L.cast_shadows = cast ? 1 : 0;
	bool shoot_d = true, shoot_c = true;   // light_area.cc:179-200, light_point.cc:111-128
	p.get("with_diffuse", shoot_d);
	p.get("with_caustic", shoot_c);
	L.shoot = (shoot_d ? 1u : 0u) | (shoot_c ? 2u : 0u);
	if(type == "pointlight")
	{
		float from[3] = {0.f, 0.f, 0.f};
		p.getVec("from", from);
		L.type = LIGHT_POINT;
		for(int k = 0; k < 3; ++k) { L.pos[k] = from[k]; L.color[k] = power * col[k]; }
		L.samples = 1;
		L.inv_samples = 1.f;
		L.nee_count = 1;
	}
	else if(type == "arealight")
	{
		float corner[3] = {0, 0, 0}, p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
		int samples = 4;
		p.getVec("corner", corner);
		p.getVec("point1", p1);
		p.getVec("point2", p2);
		p.get("samples", samples);
		std::string object_name;
		if(p.get("object_name", object_name) && !object_name.empty())
			object_name.clear();   // AreaLight::init -> Object::setLight: read only by the bidirectional integrator (primitive_triangle.cc:166)
		L.type = LIGHT_AREA;
		const F3 c = f3(corner), tx = sub(f3(p1), c), ty = sub(f3(p2), c);
		F3 fn = crs(ty, tx);
		const float pi_f = static_cast<float>(hm::num_pi);
		for(int k = 0; k < 3; ++k) L.color[k] = pi_f * (power * col[k]);
		L.area = normLen(fn);
		const F3 c2 = add(c, tx), c3 = add(c, add(tx, ty)), c4 = add(c, ty);
		put(L.pos, c);
		put(L.to_x, tx);
		put(L.to_y, ty);
		put(L.fnormal, fn);
		put(L.c2, c2);
		put(L.c3, c3);
		put(L.c4, c4);
		// light_area.cc:47-51: normal = -fnormal, du = normalize(to_x), dv = normal ^ du
		const F3 nrml = {-fn.x, -fn.y, -fn.z};
		F3 du = tx;
		{
			float len = du.x * du.x + du.y * du.y + du.z * du.z;
			if(len != 0.f)
			{
				len = 1.f / std::sqrt(len);
				du = {du.x * len, du.y * len, du.z * len};
			}
		}
		put(L.du, du);
		put(L.dv, crs(nrml, du));
		// integrator_montecarlo.cc:396: ceilf(nSamples * aa_light_sample_multiplier(1))
		L.samples = (int)std::ceil((float)samples * 1.f);
		if(L.samples < 1) L.samples = 1;
		L.inv_samples = 1.f / (float)L.samples;
		L.nee_count = 2 * (uint32_t)L.samples;
	}
	else if(type == "meshlight" || type == "objectlight")
	{
		// ObjectLight::factory (light_object_light.cc:221-254): color * power * pi, samples 4, the faces
		// of `object_name` (resolved when the scene is built: ObjectLight::init, :75-87)
		std::string object_name;
		int samples = 4;
		bool dbl = false;
		p.get("object_name", object_name);
		p.get("samples", samples);
		p.get("double_sided", dbl);
		L.type = LIGHT_MESH;
		const float pi_f = static_cast<float>(hm::num_pi);
		for(int k = 0; k < 3; ++k) L.color[k] = (col[k] * power) * pi_f;
		L.double_sided = dbl ? 1u : 0u;
		L.samples = std::max(1, (int)std::ceil((float)samples * 1.f));
		L.inv_samples = 1.f / (float)L.samples;
		L.nee_count = 2 * (uint32_t)L.samples;   // light samples + material samples (canIntersect)
		if(enabled) light_objects[name] = object_name;
	}
	else
	{
		log.error("Scene: light type '" + type + "' is not supported by the GPU core");
		return false;
	}
	if(!enabled) { log.verbose("Light '" + name + "' disabled: not used"); return true; }
	if(photon_only)
	{
		// render_view.cc:83-111: left out of the integrators' light list (getLightsVisible) but still in
		// the lists of lights shooting diffuse / caustic photons; its illumSample refuses anyway
		// (light_area.cc:68, light_point.cc:40, light_object_light.cc:110)
		L.photon_only = 1;
		L.nee_count = 0;
		log.verbose("Light '" + name + "' is photon-only: it shoots photons, the integrators do not sample it");
	}
	lights[name] = L;
	return true;
}

bool Scene::createCamera(const std::string &name, const ParamMap &p)
{
	std::string type;
	p.get("type", type);
	if(type != "perspective") { log.error("Scene: camera type '" + type + "' is not supported by the GPU core"); return false; }
	CameraDesc c;
	p.getVec("from", c.from);
	p.getVec("to", c.to);
	p.getVec("up", c.up);
	p.get("resx", c.resx);
	p.get("resy", c.resy);
	p.get("focal", c.focal);
	p.get("aperture", c.aperture);
	p.get("aspect_ratio", c.aspect);
	p.get("nearClip", c.near_clip);
	p.get("farClip", c.far_clip);
	p.get("dof_distance", c.dof_distance);
	p.get("bokeh_type", c.bokeh_type);
	p.get("bokeh_bias", c.bokeh_bias);
	p.get("bokeh_rotation", c.bokeh_rotation);
	cameras[name] = c;
	return true;
}

bool Scene::createBackground(const std::string &name, const ParamMap &p)
{
	std::string type;
	p.get("type", type);
	if(type != "constant") { log.error("Scene: background type '" + type + "' is not supported by the GPU core"); return false; }
	float col[4] = {0.f, 0.f, 0.f, 1.f};
	float power = 1.f;
	bool ibl = false;
	p.getColor("color", col);
	p.get("power", power);
	p.get("ibl", ibl);
	if(ibl)
	{
		// background_constant.cc:58-69 would add a "bglight" (BackgroundLight) to the scene
		log.error("Background '" + name + "': image-based lighting (ibl = true) is not supported by the GPU core");
		return false;
	}
	backgrounds[name] = {power * col[0], power * col[1], power * col[2]};   // background_constant.cc:56
	return true;
}

bool Scene::createIntegrator(const std::string &name, const ParamMap &p)
{
	std::string type;
	p.get("type", type);
	if(type != "directlighting" && type != "pathtracing" && type != "photonmapping")
	{
		log.error("Scene: integrator type '" + type + "' is not supported by the GPU core (directlighting, pathtracing, photonmapping)");
		return false;
	}
	if(integrators.count(name))
	{
		log.warning("Scene: Integrator '" + name + "' already exists!");   // scene.cc:419-422 (createMapItem)
		return false;
	}
	if(type == "photonmapping")
	{
		// integrator_photon_mapping.cc:765-850.  The GPU core serves the diffuse photon map with the
		// k-NN density estimate (finalGather = false) or final gathering (the default, with opaque or
		// transparent shadows), the map display (show_map) and the photon map files / reuse
		// (photon_maps_processing); the options are read at render time.
		bool ao = false;
		p.get("do_AO", ao);
		// do_AO only feeds the ambient-occlusion render layers (generateOcclusionLayers,
		// integrator_photon_mapping.cc:991-995); the combined image the GPU core produces does not use it
		// (PhotonIntegrator::integrate never calls sampleAmbientOcclusion)
		if(ao) log.info("PhotonIntegrator: do_AO only affects the AO render layers; the combined layer is unchanged");
	}
	integrators[name] = p;
	// photon_maps_processing (integrator_photon_mapping.cc:844-847, integrator_path_tracer.cc:360-363;
	// other integrators keep MonteCarloIntegrator's PhotonsGenerateOnly): an unknown value generates
	IntegratorState &st = integrator_state[name];
	st.id = ++integrator_ids_;
	st.processing = PhotonParams::PM_GENERATE;
	std::string processing = "generate";
	if((type == "photonmapping" || type == "pathtracing") && p.get("photon_maps_processing", processing))
	{
		if(processing == "generate-save") st.processing = PhotonParams::PM_GENERATE_SAVE;
		else if(processing == "load") st.processing = PhotonParams::PM_LOAD;
		else if(processing == "reuse-previous") st.processing = PhotonParams::PM_REUSE;
	}
	return true;
}

bool Scene::createRenderView(const std::string &name, const ParamMap &p)
{
	std::string cam;
	p.get("camera_name", cam);
	views[name] = cam;
	return true;
}

// scene.cc:528-644 + imagefilm.cc:48-127
bool Scene::setupRender(const ParamMap &p)
{
	RenderSetup s;
	if(!p.get("integrator_name", s.integrator_name)) { log.error("Scene: Specify an Integrator!!"); return false; }
	if(!integrators.count(s.integrator_name)) { log.error("Scene: Specify an _existing_ Integrator!!"); return false; }
	std::string vol;
	// scene.cc:564-572: a named integrator that is not a volume integrator is an error; an unknown name
	// means no volume integrator.  Volume integrator types are not created by the GPU core, so every
	// existing integrator is a surface one.
	if(p.get("volintegrator_name", vol) && integrators.count(vol))
	{
		log.error("Scene: Integrator '" + vol + "' is not a volume integrator!");
		return false;
	}
	if(p.get("background_name", s.background_name) && !backgrounds.count(s.background_name))
		log.error("Scene: please specify an _existing_ Background!!");
	p.get("AA_passes", s.aa_passes);
	p.get("AA_minsamples", s.aa_samples);
	s.aa_inc_samples = s.aa_samples;   // scene.cc:584
	p.get("AA_inc_samples", s.aa_inc_samples);
	p.get("AA_threshold", s.aa_threshold);
	p.get("AA_resampled_floor", s.aa_resampled_floor);
	p.get("AA_sample_multiplier_factor", s.aa_sample_multiplier_factor);
	p.get("AA_light_sample_multiplier_factor", s.aa_light_sample_multiplier_factor);
	p.get("AA_indirect_sample_multiplier_factor", s.aa_indirect_sample_multiplier_factor);
	p.get("AA_detect_color_noise", s.aa_detect_color_noise);
	p.get("AA_dark_detection_type", s.aa_dark_detection_type);
	p.get("AA_dark_threshold_factor", s.aa_dark_threshold_factor);
	p.get("AA_variance_edge_size", s.aa_variance_edge_size);
	p.get("AA_variance_pixels", s.aa_variance_pixels);
	p.get("AA_clamp_samples", s.clamp_samples);
	p.get("threads", s.threads);
	p.get("gpus", s.gpus);
	p.get("threads_photons", s.threads_photons);
	p.get("adv_auto_shadow_bias_enabled", s.shadow_bias_auto);
	p.get("adv_shadow_bias_value", s.shadow_bias);
	p.get("adv_auto_min_raydist_enabled", s.ray_min_dist_auto);
	p.get("adv_min_raydist_value", s.ray_min_dist);
	p.get("adv_base_sampling_offset", s.base_sampling_offset);
	p.get("adv_rr_seed", s.rr_seed);
	p.get("adv_computer_node", s.computer_node);
	p.get("film_load_save_mode", s.film_load_save_mode);
	p.get("film_load_save_path", s.film_load_save_path);
	p.get("film_autosave_interval_type", s.film_autosave_interval_type);
	p.get("film_autosave_interval_passes", s.film_autosave_interval_passes);
	p.get("film_autosave_interval_seconds", s.film_autosave_interval_seconds);
	p.get("scene_accelerator", s.accelerator);
	p.get("AA_pixelwidth", s.aa_pixelwidth);
	p.get("width", s.width);
	p.get("height", s.height);
	p.get("xstart", s.xstart);
	p.get("ystart", s.ystart);
	p.get("filter_type", s.filter);
	p.get("tile_size", s.tile_size);
	p.get("tiles_order", s.tiles_order);
	if(s.accelerator != "yafaray-kdtree-original" && s.accelerator != "yafaray-kdtree-multi-thread" && s.accelerator != "yafaray-simpletest")
		log.warning("Accelerator type '" + s.accelerator + "' could not be created, using the GPU BVH instead.");  // accelerator.cc:47-51
	if(s.filter != "box" && s.filter != "gauss" && s.filter != "mitchell" && s.filter != "lanczos")
	{
		log.warning("ImageFilm: No AA filter defined defaulting to Box!");
		s.filter = "box";
	}
	if(s.tile_size < 1) s.tile_size = 32;
	s.aa_samples = std::max(1, s.aa_samples);
	s.valid = true;
	setup = s;
	return true;
}

// ObjectLight::initIs (light_object_light.cc:46-73): the faces of the light's object in creation
// order, their areas (TrianglePrimitive::surfaceArea, primitive_triangle.cc:208-213), the area
// distribution (sample_pdf1d.h:52-66, the cdf accumulated in double) and the total area (summed in
// double, stored as float); per face the exact-test record, the vertices and the geometric normal.
bool Scene::meshLightFaces(const std::string &name, DevLight &L, HostScene &hs)
{
	auto lo = light_objects.find(name);
	auto it = lo == light_objects.end() ? objects.end() : objects.find(lo->second);
	if(it == objects.end() || it->second.tri_mat.empty())
	{
		log.error("Light '" + name + "': object '" + (lo == light_objects.end() ? std::string() : lo->second) + "' not found or empty");
		return false;
	}
	const MeshObject &o = it->second;
	const size_t nt = o.tri_mat.size();
	L.mesh0 = (uint32_t)(hs.mesh_cdf.size());
	L.mesh_n = (uint32_t)nt;
	std::vector<float> areas(nt);
	double total = 0.0;
	for(size_t t = 0; t < nt; ++t)
	{
		const F3 a = f3(&o.verts[3 * (size_t)o.tris[3 * t]]), b = f3(&o.verts[3 * (size_t)o.tris[3 * t + 1]]),
		         c = f3(&o.verts[3 * (size_t)o.tris[3 * t + 2]]);
		areas[t] = 0.5f * std::sqrt(lsq(crs(sub(b, a), sub(c, a))));
		total += areas[t];
		float rec[kMeshTriF4 * 4];
		packTriangle(&o.verts[3 * (size_t)o.tris[3 * t]], &o.verts[3 * (size_t)o.tris[3 * t + 1]], &o.verts[3 * (size_t)o.tris[3 * t + 2]], (int)t, rec);
		put(rec + 12, a);
		put(rec + 16, b);
		put(rec + 20, c);
		put(rec + 24, nrm(crs(sub(b, a), sub(c, a))));
		hs.mesh_tris.insert(hs.mesh_tris.end(), rec, rec + kMeshTriF4 * 4);
	}
	const double delta = 1.0 / static_cast<double>(nt);
	double cum = 0.0;
	std::vector<float> cdf(nt);
	for(size_t t = 0; t < nt; ++t)
	{
		cum += static_cast<double>(areas[t]) * delta;
		cdf[t] = static_cast<float>(cum);
	}
	const float integral = static_cast<float>(cum);
	for(float &e : cdf) e /= integral;
	hs.mesh_cdf.insert(hs.mesh_cdf.end(), cdf.begin(), cdf.end());
	L.area = static_cast<float>(total);
	// the light's own BVH2 over its faces (the reference's per-light kd-tree, light_object_light.cc:62-70):
	// the material-sampled rays find the closest face through it instead of testing every face
	L.bvh_depth = 0;
	const char *mb = std::getenv("YAFARAY_AMD_MESHLIGHT_BVH");   // "0": test every face (A/B, tests)
	if(nt > 8 && !(mb && *mb == '0'))
	{
		BvhInput bi;
		bi.verts = o.verts.data();
		bi.tris = o.tris.data();
		bi.n_tris = (int)nt;
		bi.width = 2;
		const BvhOutput bo = buildBvh(bi, 4, 1);
		if(bo.depth > 0 && bo.depth <= 60)
		{
			L.bvh_node0 = (uint32_t)(hs.mesh_nodes.size() / 16);
			L.bvh_tri0 = (uint32_t)(hs.mesh_btris.size() / 12);
			L.bvh_depth = (uint32_t)bo.depth;
			hs.mesh_nodes.insert(hs.mesh_nodes.end(), bo.nodes.begin(), bo.nodes.end());
			hs.mesh_btris.insert(hs.mesh_btris.end(), bo.tris.begin(), bo.tris.end());
		}
		else log.warning("Light '" + name + "': the BVH over its " + std::to_string(nt) + " faces is too deep; every face is tested");
	}
	return true;
}

bool Scene::buildAccelerator()
{
	if(!syncMembers()) return false;
	// scene.cc:1032-1060 updateObjects: gather visible, non-base mesh primitives
	std::vector<float> verts;
	std::vector<int> tris, tri_mat;
	for(const std::string &name : object_order)
	{
		const MeshObject &o = objects[name];
		if(o.is_base || o.visibility == "invisible") continue;
		const int v0 = (int)(verts.size() / 3);
		verts.insert(verts.end(), o.verts.begin(), o.verts.end());
		for(size_t t = 0; t < o.tri_mat.size(); ++t)
		{
			tris.push_back(o.tris[3 * t] + v0);
			tris.push_back(o.tris[3 * t + 1] + v0);
			tris.push_back(o.tris[3 * t + 2] + v0);
			tri_mat.push_back(o.tri_mat[t]);
		}
	}
	const auto t0 = std::chrono::steady_clock::now();
	HostScene hs;
	hs.n_prims = (int)tri_mat.size();
	BvhInput in{verts.data(), tris.data(), hs.n_prims};
	int leaf = 1;   // pure SAH leaves (measured best on the Cornell box)
	if(const char *e = getenv("YAFARAY_AMD_BVH_LEAF")) leaf = std::max(1, atoi(e));          // tuning sweeps
	if(const char *e = getenv("YAFARAY_AMD_BVH_NODE_COST")) in.node_cost = (float)atof(e);
	if(const char *e = getenv("YAFARAY_AMD_BVH_WIDTH")) in.width = atoi(e) == 2 ? 2 : 4;
	// large meshes are built on the device (bvhgpu.hip), small ones (LDS-resident scenes, where the
	// binned-SAH tree's quality matters most) on the host; YAFARAY_AMD_BVH_BUILD=gpu|host overrides
	hs.gpu_build = in.width == 4 && hs.n_prims >= 65536;
	if(const char *e = getenv("YAFARAY_AMD_BVH_BUILD"); e && *e) hs.gpu_build = in.width == 4 && std::string(e) == "gpu";
	if(hs.gpu_build)
	{
		hs.verts = verts;
		hs.tris = tris;
	}
	else hs.bvh = buildBvh(in, leaf, 8);
	// primitive_triangle.cc:87-95 geometric normal; material index per primitive
	hs.prim_ng.resize(4 * (size_t)hs.n_prims);
	for(int t = 0; t < hs.n_prims; ++t)
	{
		const F3 a = f3(&verts[3 * (size_t)tris[3 * t]]), b = f3(&verts[3 * (size_t)tris[3 * t + 1]]), c = f3(&verts[3 * (size_t)tris[3 * t + 2]]);
		const F3 n = nrm(crs(sub(b, a), sub(c, a)));
		float matf;
		std::memcpy(&matf, &tri_mat[t], 4);
		put(&hs.prim_ng[4 * (size_t)t], n, matf);
	}
	for(const std::string &mn : material_order)
	{
		DevMaterial m = materials[mn];
		auto nit = mat_nodes.find(mn);
		m.node0 = (int)hs.shader_nodes.size();
		if(nit != mat_nodes.end()) hs.shader_nodes.insert(hs.shader_nodes.end(), nit->second.begin(), nit->second.end());
		else m.n_nodes = 0;
		if(m.n_nodes > 0) hs.has_attr = true;
		hs.mats.push_back(m);
	}
	if(hs.mats.empty()) hs.mats.push_back(DevMaterial{});
	// image textures: texels = the image buffers' getColor() values (one copy per image)
	{
		std::map<const HostImage *, uint32_t> placed;
		for(const HostTexture &ht : textures)
		{
			DevTexture t = ht.t;
			auto pit = placed.find(ht.img.get());
			if(pit == placed.end())
			{
				const uint32_t off = (uint32_t)(hs.texels.size() / 4);
				hs.texels.insert(hs.texels.end(), ht.img->px.begin(), ht.img->px.end());
				pit = placed.emplace(ht.img.get(), off).first;
			}
			t.texel0 = pit->second;
			hs.textures.push_back(t);
		}
	}
	for(const std::string &name : object_order)
	{
		const MeshObject &o = objects[name];
		if(o.is_base || o.visibility == "invisible") continue;
		if(o.smooth || !o.normals.empty()) hs.has_attr = true;
	}
	if(hs.has_attr)
	{
		// per-primitive surface attributes (texeval.h surfAttr; primitive_triangle.cc:97-176)
		hs.prim_attr.assign((size_t)hs.n_prims * kAttrF4 * 4, 0.f);
		int t = 0;
		for(const std::string &name : object_order)
		{
			const MeshObject &o = objects[name];
			if(o.is_base || o.visibility == "invisible") continue;
			const bool has_orco = !o.orco.empty(), has_uv = !o.uvs.empty(), smooth = o.smooth || !o.normals.empty();
			const size_t nn = o.normals.size() / 3;
			for(size_t k = 0; k < o.tri_mat.size(); ++k, ++t)
			{
				float *a = &hs.prim_attr[(size_t)t * kAttrF4 * 4];
				const int *vi = &o.tris[3 * k];
				const F3 p0 = f3(&o.verts[3 * (size_t)vi[0]]), p1 = f3(&o.verts[3 * (size_t)vi[1]]), p2 = f3(&o.verts[3 * (size_t)vi[2]]);
				uint32_t fl = 0;
				put(a + 4, sub(p1, p0));
				put(a + 8, sub(p2, p0));
				if(has_orco && o.orco.size() >= 3 * (o.verts.size() / 3))
				{
					fl |= ATTR_ORCO;
					for(int r = 0; r < 3; ++r) put(a + 12 + 4 * r, f3(&o.orco[3 * (size_t)vi[r]]));
				}
				const int *ui = o.tri_uv.size() >= 3 * (k + 1) ? &o.tri_uv[3 * k] : nullptr;
				if(has_uv && ui && ui[0] >= 0 && ui[1] >= 0 && ui[2] >= 0)
				{
					const float *u0 = &o.uvs[2 * (size_t)ui[0]], *u1 = &o.uvs[2 * (size_t)ui[1]], *u2 = &o.uvs[2 * (size_t)ui[2]];
					const float du_1 = u1[0] - u0[0], du_2 = u2[0] - u0[0], dv_1 = u1[1] - u0[1], dv_2 = u2[1] - u0[1];
					const float det = du_1 * dv_2 - dv_1 * du_2;
					if(std::abs(det) > 1e-30f) fl |= ATTR_UV;   // else implicit uv (:144-152)
					a[24] = u0[0]; a[25] = u0[1]; a[26] = u1[0]; a[27] = u1[1];
					a[28] = u2[0]; a[29] = u2[1];
				}
				if(smooth)
				{
					fl |= ATTR_SMOOTH;
					const float *ng = &hs.prim_ng[4 * (size_t)t];
					for(int r = 0; r < 3; ++r)
					{
						const int ni = o.tri_nidx.size() >= 3 * (k + 1) ? o.tri_nidx[3 * k + r] : -1;
						if(ni >= 0 && (size_t)ni < nn) put(a + 32 + 4 * r, f3(&o.normals[3 * (size_t)ni]));
						else put(a + 32 + 4 * r, F3{ng[0], ng[1], ng[2]});   // getVertexNormal: face normal
					}
				}
				float flf;
				std::memcpy(&flf, &fl, 4);
				put(a, p0, flf);
			}
		}
	}
	// the visible lights in name order (render_view.cc:83-91: the integrators' list), then the photon-only
	// ones (only the photon maps' light sets refer to them)
	{
		std::map<std::string, int> at;
		for(int pass = 0; pass < 2; ++pass)
			for(auto &kv : lights)
			{
				DevLight L = kv.second;
				if((L.photon_only != 0) != (pass == 1)) continue;
				if(L.type == LIGHT_MESH && !meshLightFaces(kv.first, L, hs)) return false;
				at[kv.first] = (int)hs.lights.size();
				hs.lights.push_back(L);
			}
		for(const auto &kv : at) hs.light_name_order.push_back(kv.second);
	}
	uint32_t base = 0;
	for(DevLight &L : hs.lights) { L.nee_base = base; base += L.nee_count; }
	for(int m = 0; m < memberCount(); ++m)
		if(!member(m)->upload(hs)) return false;
	const auto t1 = std::chrono::steady_clock::now();
	stats.build_seconds = std::chrono::duration<double>(t1 - t0).count();
	std::ostringstream os;
	os << "Accelerator: BVH" << hs.bvh.width << (hs.gpu_build ? " (built on the GPU: PLOC + collapse)" : " (binned SAH on the host)") << " over " << hs.n_prims << " triangles: " << hs.bvh.n_nodes << " nodes, depth " << hs.bvh.depth
	   << ", max leaf " << hs.bvh.max_leaf << " (" << stats.build_seconds << " s)";
	log.info(os.str());
	geometry_dirty = false;
	return true;
}

// scene.cc:203-263 Scene::render + integrator_tiled.cc:97-233 (single AA pass)
// ImageSplitter (imagesplitter.cc:30-107) for one render thread (no subdivision of the last tiles):
// the tile ids ty * ntx + tx in render order.  "linear": row-major; "random": a fixed-seed shuffle
// (the reference seeds from std::random_device); anything else, the reference's default "centre":
// by squared distance of the tile corner to the image centre (ImageSpliterCentreSorter,
// imagesplitter.h:97-109, integer arithmetic), ties in linear order (the reference breaks them by
// a random shuffle before its unstable sort).
static std::vector<int> tileOrder(int W, int H, int ts, const std::string &order)
{
	const int ntx = (W + ts - 1) / ts, nty = (H + ts - 1) / ts;
	std::vector<int> ids((size_t)ntx * nty);
	for(size_t i = 0; i < ids.size(); ++i) ids[i] = (int)i;
	if(order == "linear") return ids;
	if(order == "random")
	{
		std::shuffle(ids.begin(), ids.end(), std::mt19937(0x59414641u));
		return ids;
	}
	auto key = [&](int id) {
		const int x = (id % ntx) * ts, y = (id / ntx) * ts;
		return (x - W / 2) * (x - W / 2) + (y - H / 2) * (y - H / 2);
	};
	std::stable_sort(ids.begin(), ids.end(), [&](int a, int b) { return key(a) < key(b); });
	return ids;
}

bool Scene::render(const Callbacks &cb, yafaray_ProgressBarCallback_t progress, void *progress_data, bool quiet)
{
	if(!setup.valid) { log.error("Scene: No ImageFilm present, bailing out..."); return false; }
	if(views.empty()) { log.error("Scene: no render view defined"); return false; }
	canceled = false;
	if(!syncMembers()) return false;
	if(geometry_dirty && !buildAccelerator()) return false;
	const RenderSetup &s = setup;
	const ParamMap &ip = integrators[s.integrator_name];
	std::string itype;
	ip.get("type", itype);
	for(const auto &view : views)
	{
		auto cit = cameras.find(view.second);
		if(cit == cameras.end()) { log.error("RenderView '" + view.first + "': Camera not found in the scene."); return false; }
		const CameraDesc &c = cit->second;
		RenderParams rp{};
		DevScene &S = rp.scene;
		// camera.cc:51-71 + camera_perspective.cc:28-69
		const F3 pos = f3(c.from), look = f3(c.to), up = f3(c.up);
		const float aspect_ratio = c.aspect * (float)c.resy / (float)c.resx;
		F3 cam_y = sub(up, pos), cam_z = sub(look, pos);
		F3 cam_x = crs(cam_z, cam_y);
		cam_y = crs(cam_z, cam_x);
		cam_x = nrm(cam_x);
		cam_y = nrm(cam_y);
		cam_z = nrm(cam_z);
		F3 vright = cam_x, vup = mul(cam_y, aspect_ratio);
		const F3 vto = sub(mul(cam_z, c.focal), mul(add(vup, vright), static_cast<float>(0.5)));
		vup = {vup.x / (float)c.resy, vup.y / (float)c.resy, vup.z / (float)c.resy};
		vright = {vright.x / (float)c.resx, vright.y / (float)c.resx, vright.z / (float)c.resx};
		put(S.cam.pos, pos);
		put(S.cam.vright, vright);
		put(S.cam.vup, vup);
		put(S.cam.vto, vto);
		put(S.cam.cam_z, cam_z);
		put(S.cam.near_p, add(pos, mul(cam_z, c.near_clip)));
		put(S.cam.far_p, add(pos, mul(cam_z, c.far_clip)));
		{
			// cameraRay's numerators (dot(cam_z, plane point - pos), the device's float operations): a near
			// plane through the position gives tmin = 0 and a far numerator < 0 a negative (unbounded) tmax
			// for every ray — then k_camera writes no per-ray (tmin, tmax) and k_trace takes (0, unbounded)
			const F3 dn = sub(add(pos, mul(cam_z, c.near_clip)), pos), df = sub(add(pos, mul(cam_z, c.far_clip)), pos);
			const bool near0 = dn.x == 0.f && dn.y == 0.f && dn.z == 0.f;
			const float far_num = cam_z.x * df.x + cam_z.y * df.y + cam_z.z * df.z;
			S.cam.ray_tt = (near0 && far_num < -1e-20f) ? 0 : 1;
		}
		S.cam.resx = c.resx;
		S.cam.resy = c.resy;
		// depth of field (camera_perspective.cc:28-52, 59-62, 212-224)
		S.cam.aperture = c.aperture;
		S.cam.dof_distance = c.dof_distance;
		put(S.cam.dof_rt, mul(cam_x, c.aperture));
		put(S.cam.dof_up, mul(cam_y, c.aperture));
		{
			int bt = 0;
			if(c.bokeh_type == "disk2") bt = 1;
			else if(c.bokeh_type == "triangle") bt = 3;
			else if(c.bokeh_type == "square") bt = 4;
			else if(c.bokeh_type == "pentagon") bt = 5;
			else if(c.bokeh_type == "hexagon") bt = 6;
			else if(c.bokeh_type == "ring") bt = 7;
			S.cam.bokeh_type = bt;
			S.cam.bokeh_bias = c.bokeh_bias == "center" ? 1 : (c.bokeh_bias == "edge" ? 2 : 0);
			for(float &v : S.cam.ls) v = 0.f;
			if(bt >= 3 && bt <= 6)
			{
				// math::degToRad and mult_pi_by_2 / ns are long double expressions rounded to float
				float w = static_cast<float>(c.bokeh_rotation * hm::div_pi_by_180);
				const float wi = static_cast<float>(hm::mult_pi_by_2 / static_cast<float>(bt));
				for(int i = 0; i < (bt + 2) * 2; i += 2)
				{
					S.cam.ls[i] = hm::sinf_fast(w + static_cast<float>(hm::div_pi_by_2));   // math::cos (FAST_TRIG)
					S.cam.ls[i + 1] = hm::sinf_fast(w);
					w += wi;
				}
			}
		}
		// integrator + render parameters
		S.integrator = (itype == "pathtracing") ? INT_PATH : (itype == "photonmapping") ? INT_PHOTON : INT_DIRECT;
		if(S.integrator == INT_PHOTON)
		{
			// integrator_photon_mapping.cc:765-850 defaults
			int photons = 100000, cphotons = 500000, search = 50, pbounces = 5;
			float ds_rad = 0.1f, c_rad = 0.01f;
			bool caustics = true, diffuse = true;
			ip.get("photons", photons);
			ip.get("cPhotons", cphotons);
			ip.get("search", search);
			int caustic_mix = search;
			ip.get("caustic_mix", caustic_mix);
			ip.get("diffuseRadius", ds_rad);
			ip.get("causticRadius", c_rad);
			ip.get("bounces", pbounces);
			ip.get("caustics", caustics);
			ip.get("diffuse", diffuse);
			rp.pm.photons = diffuse ? std::max(0, photons) : 0;
			rp.pm.diffuse_map = diffuse;
			// the caustic map: MonteCarloIntegrator::createCausticMap with caus_depth = bounces
			rp.pm.caustic_map = caustics;
			rp.pm.caustic_photons = std::max(0, cphotons);
			rp.pm.caustic_search = std::max(1, caustic_mix);
			rp.pm.caustic_radius = c_rad;
			rp.pm.caustic_depth = std::max(0, pbounces);
			rp.pm.search = std::max(1, search);
			rp.pm.radius2 = ds_rad;
			rp.pm.bounces = std::max(0, pbounces);
			rp.pm.threads = s.threads_photons;
			// final gathering (:777-810): fg_samples, fg_bounces, fg_min_pathlen (default diffuseRadius)
			bool fg = true;
			int fg_samples = 32, fg_bounces = 2;
			float gather_dist = ds_rad;
			ip.get("finalGather", fg);
			ip.get("fg_samples", fg_samples);
			ip.get("fg_bounces", fg_bounces);
			ip.get("fg_min_pathlen", gather_dist);
			rp.pm.final_gather = fg && diffuse;
			bool show_map = false;
			ip.get("show_map", show_map);
			S.show_map = (show_map && diffuse && rp.pm.photons > 0) ? 1 : 0;
			rp.pm.fg_samples = fg_samples;
			rp.pm.fg_bounces = fg_bounces;
			rp.pm.fg_min_pathlen = gather_dist;
		}
		S.width = s.width;
		S.height = s.height;
		S.spp = s.aa_samples;
		S.tile = s.tile_size;
		int bounces = 3, path_samples = 32, rr_min = 0;
		std::string caustic_type;
		ip.get("bounces", bounces);
		ip.get("path_samples", path_samples);
		ip.get("russian_roulette_min_bounces", rr_min);
		S.caustic_path = 1;   // PathIntegrator ctor: CausticType::Path (integrator_path_tracer.cc:43)
		// DirectLight "caustics" / PathIntegrator caustic_type photon | both: the caustic photon map
		// (integrator_direct_light.cc:147-190, integrator_path_tracer.cc:325-342; defaults photons
		// 500000, caustic_mix 100, caustic_depth 10, caustic_radius 0.25 as double)
		auto causticParams = [&]() {
			int c_photons = 500000, c_search = 100, c_depth = 10;
			double c_rad = 0.25;
			ip.get("photons", c_photons);
			ip.get("caustic_mix", c_search);
			ip.get("caustic_depth", c_depth);
			ip.get("caustic_radius", c_rad);
			rp.pm.caustic_map = true;
			rp.pm.caustic_photons = std::max(0, c_photons);
			rp.pm.caustic_search = std::max(1, c_search);
			rp.pm.caustic_depth = std::max(0, c_depth);
			rp.pm.caustic_radius = static_cast<float>(c_rad);
			rp.pm.threads = s.threads_photons;
		};
		if(S.integrator == INT_PATH && ip.get("caustic_type", caustic_type))
		{
			if(caustic_type == "none") S.caustic_path = 0;
			else if(caustic_type == "photon") { S.caustic_path = 0; causticParams(); }
			else if(caustic_type == "both") causticParams();
		}
		if(S.integrator == INT_DIRECT)
		{
			bool caus = false, ao = false;
			ip.get("caustics", caus);
			ip.get("do_AO", ao);
			if(caus) causticParams();
			// integrator_direct_light.cc:161-186: do_AO, AO_samples (32), AO_distance (1.0, double), AO_color (1)
			if(ao)
			{
				int ao_samples = 32;
				double ao_dist = 1.0;
				float ao_col[4] = {1.f, 1.f, 1.f, 1.f};
				ip.get("AO_samples", ao_samples);
				ip.get("AO_distance", ao_dist);
				ip.getColor("AO_color", ao_col);
				if(ao_samples < 1)
				{
					log.error("DirectLight: AO_samples must be >= 1");   // the reference divides by it (integrator_tiled.cc:690)
					return false;
				}
				S.do_ao = 1;
				S.ao_samples = ao_samples;
				S.ao_dist = static_cast<float>(ao_dist);
				for(int k = 0; k < 3; ++k) S.ao_col[k] = ao_col[k];
			}
		}
		S.bounces = bounces;
		S.path_samples = (S.integrator == INT_PATH) ? std::max(1, path_samples) : 1;
		S.rr_min_bounces = rr_min;
		bool bg_transp = false, bg_transp_refract = false;
		ip.get("bg_transp", bg_transp);
		ip.get("bg_transp_refract", bg_transp_refract);
		S.bg_transp = bg_transp ? 1 : 0;
		S.bg_transp_refract = bg_transp_refract ? 1 : 0;
		// specular recursion (integrator_direct_light.cc:152-192, integrator_path_tracer.cc:299-306)
		int raydepth = 5;
		ip.get("raydepth", raydepth);
		S.raydepth = raydepth;
		// transparent shadows (integrator_path_tracer.cc:294-311, integrator_direct_light.cc:148-164,
		// integrator_photon_mapping.cc:767-796): "transpShad", "shadowDepth" (default 5)
		bool transp_shad = false;
		int shadow_depth = 5;
		ip.get("transpShad", transp_shad);
		ip.get("shadowDepth", shadow_depth);
		S.tr_shad = transp_shad ? 1 : 0;
		S.s_depth = std::max(0, shadow_depth);
		S.tree = 0;
		S.ext = 0;
		S.w_live = 0;
		S.max_add_depth = 0;
		for(const auto &kv : materials)
		{
			const DevMaterial &m = kv.second;
			S.max_add_depth = std::max(S.max_add_depth, m.add_depth);
			if(m.bsdf_flags & (B_SPECULAR | B_FILTER)) S.tree = 1;
			if(m.type == MAT_MIRROR || m.type == MAT_NULL || m.n_nodes > 0 ||
			   (m.sd_flags & (SD_MIRROR | SD_TRANSPARENT | SD_TRANSLUCENT | SD_FRESNEL | SD_OREN_NAYAR)))
				S.ext = 1;
			// a shinydiffuse sample() that matches no component returns before it sets w
			// (material_shiny_diffuse.cc:259-262), and the path tracer multiplies by the previous w
			if(m.type == MAT_SHINYDIFFUSE && (m.n_bsdf == 0 || (double)m.comp[3] < 0.00001)) S.w_live = 1;
		}
		// the sample weight w persists across vertices only when some sample() can leave it unset: the
		// EXT materials (Fresnel / transparency can shrink the diffuse share) or a non-diffuse shinydiffuse;
		// else k_shade keeps the throughput as a 12-B record
		if(S.ext) S.w_live = 1;

		S.has_bg = 0;
		if(!s.background_name.empty() && backgrounds.count(s.background_name))
		{
			const auto &bgc = backgrounds[s.background_name];
			S.has_bg = 1;
			for(int k = 0; k < 3; ++k) S.bg[k] = bgc[k];
		}
		S.shadow_bias_auto = s.shadow_bias_auto ? 1 : 0;
		S.shadow_bias = s.shadow_bias;
		S.ray_min_dist_auto = s.ray_min_dist_auto ? 1 : 0;
		S.ray_min_dist = s.ray_min_dist;
		S.base_offset = (uint32_t)s.base_sampling_offset;
		// cropped film (imagefilm.cc:66, 129-132): film pixel (x, y) is camera pixel (x + xstart, y + ystart)
		S.crop_x0 = s.xstart;
		S.crop_y0 = s.ystart;
		S.clamp_samples = s.clamp_samples;
		S.rr_seed = (uint32_t)s.rr_seed;
		uint32_t nee_all = 0, nee_max_one = 1;
		for(auto &kv : lights)
		{
			nee_all += kv.second.nee_count;
			nee_max_one = std::max(nee_max_one, kv.second.nee_count);
		}
		S.nee_all_count = (int)nee_all;
		// NEE entries per vertex: estimateAllDirectLight's (+ the AO samples), or one light's
		S.nee_k = (int)std::max(nee_all + (S.do_ao ? (uint32_t)S.ao_samples : 0u), nee_max_one);
		if(S.integrator == INT_PATH && S.path_samples > 4095) { log.error("PathIntegrator: path_samples > 4095 unsupported"); return false; }
		if(S.integrator == INT_PATH && 4 * S.bounces + 4 >= 50)
		{
			// halton.cc:439: dimensions >= 50 draw from the racy global FastRandom (not reproducible)
			log.error("PathIntegrator: bounces > 11 use Halton dimensions >= 50, which the reference draws from a racy "
			          "global FastRandom; not supported by the GPU core");
			return false;
		}
		// film (imagefilm.cc:129-173)
		DevFilm &F = rp.film;
		float filterw = static_cast<float>(s.aa_pixelwidth * 0.5);
		float (*ff)(float, float) = hm::filterBox;
		if(s.filter == "mitchell") { ff = hm::filterMitchell; filterw *= 2.6f; }
		else if(s.filter == "lanczos") ff = hm::filterLanczos;
		else if(s.filter == "gauss") { ff = hm::filterGauss; filterw *= 2.f; }
		filterw = std::min(std::max(0.501f, filterw), 0.5f * 8);
		const float scale = 1.f / 16.f;
		for(int y = 0; y < 16; ++y)
			for(int x = 0; x < 16; ++x) F.table[y * 16 + x] = ff((x + .5f) * scale, (y + .5f) * scale);
		F.filterw = filterw;
		F.table_scale = static_cast<float>(0.9999 * 16 / filterw);
		F.reach_fwd = std::max(0, (int)((double)filterw + (.5 - 1.4e-11)));
		F.reach_back = std::max(0, -(int)(-(double)filterw + (.5 - 1.4e-11)));
		F.width = s.width;
		F.height = s.height;
		F.crop_x0 = s.xstart;
		F.crop_y0 = s.ystart;
		F.spp = s.aa_samples;
		F.tile = s.tile_size;
		rp.shard_rank = shard_rank;
		rp.shard_world = std::max(1, shard_world);
		rp.shard_mode = shard_mode;
		rp.shard_y0 = shard_y0;
		rp.shard_y1 = shard_y1;
		// Several GPUs render this film: the render group (one process per GPU, RCCL) or the device
		// group of this process (one host thread per GPU).  Each member renders its row band (+ halo
		// rows); the members exchange the accumulated film between adaptive passes and combine the
		// bands at the end (GpuRenderer::renderMember).
		const int group_world = gpu()->groupWorld();
		const int n_members = memberCount();
		const int world = group_world > 1 ? group_world : n_members;
		const bool grouped = world > 1;
		last_bounds_.clear();
		last_member_ms_.clear();
		if(grouped)
		{
			if((int)group_bounds.size() != world + 1 || group_bounds.back() != s.height) group_bounds = equalBands(s.height, world);
			if(s.height < world)
			{
				log.error("Scene: the film has fewer rows than GPUs rendering it");
				return false;
			}
			rp.shard_world = world;
			rp.shard_rank = group_world > 1 ? gpu()->groupRank() : 0;
			rp.shard_mode = 2;
			rp.band_bounds = group_bounds;
			rp.shard_y0 = group_bounds[rp.shard_rank];
			rp.shard_y1 = group_bounds[rp.shard_rank + 1];
			rp.combine_all = group_world > 1;
		}
		rp.aa.passes = std::max(1, s.aa_passes);
		if(rp.aa.passes > 1 && rp.shard_world > 1 && !grouped)
		{
			// nextPass compares neighbouring pixels across the whole film; a caller-side shard
			// (setTileRowShard / setRowBandShard) only holds its own rows and has no exchange
			log.error("Scene: AA_passes > 1 with a caller-sharded film is not supported (use a render or device group)");
			return false;
		}
		rp.aa.inc_samples = s.aa_inc_samples;
		rp.aa.light_sample_multiplier_factor = s.aa_light_sample_multiplier_factor;
		rp.aa.indirect_sample_multiplier_factor = s.aa_indirect_sample_multiplier_factor;
		rp.aa.threshold = s.aa_threshold;
		rp.aa.resampled_floor = s.aa_resampled_floor;
		rp.aa.sample_multiplier_factor = s.aa_sample_multiplier_factor;
		rp.aa.dev.detect_color_noise = s.aa_detect_color_noise ? 1 : 0;
		rp.aa.dev.dark_type = s.aa_dark_detection_type == "linear" ? 1 : (s.aa_dark_detection_type == "curve" ? 2 : 0);   // scene.cc:624-626
		rp.aa.dev.dark_factor = s.aa_dark_threshold_factor;
		rp.aa.dev.variance_edge = s.aa_variance_edge_size;
		rp.aa.dev.variance_pixels = s.aa_variance_pixels;
		rp.chunk_slots = chunk_slots;
		rp.profile = profile_kernels;
		S.trace_stats = trace_stats ? 1 : 0;
		film_w = s.width;
		film_h = s.height;
		if(!quiet)
		{
			std::ostringstream os;
			os << itype << ": " << s.width << "x" << s.height << " x " << s.aa_samples << " spp, filter " << s.filter << " " << s.aa_pixelwidth
			   << ", tile " << s.tile_size;
			if(S.integrator == INT_PATH) os << ", bounces " << S.bounces << ", path_samples " << S.path_samples << ", rr_min " << S.rr_min_bounces;
			log.params(os.str());
			if(cb.notify_view) cb.notify_view(view.first.c_str(), cb.notify_view_data);
			if(cb.notify_layer) cb.notify_layer("combined", "Combined", s.width, s.height, 4, cb.notify_layer_data);
			if(progress) progress(s.width * s.height, 0, "Rendering...", progress_data);
		}
		// ---- film load / save (ImageFilm::init imagefilm.cc:225-241, flush :657-662, nextPass :282-286) ----
		const filmio::Mode fmode = filmio::parseMode(s.film_load_save_mode);
		filmio::Film film_io;
		film_io.computer_node = (uint32_t)s.computer_node;
		film_io.base_sampling_offset = (uint32_t)s.base_sampling_offset;
		film_io.width = s.width;
		film_io.height = s.height;
		film_io.cx0 = s.xstart;
		film_io.cx1 = s.xstart + s.width;
		film_io.cy0 = s.ystart;
		film_io.cy1 = s.ystart + s.height;
		const std::string film_file = filmio::filmPath(s.film_load_save_path, s.computer_node);
		if(fmode != filmio::None && rp.shard_world > 1 && !grouped)
		{
			log.error("Scene: film load/save with a caller-sharded film is not supported (use a render or device group)");
			return false;
		}
		// a group render combines the accumulators too (the film file is saved from them); in a render
		// group only member 0 writes the files, every member reads them
		rp.combine_accum = fmode != filmio::None;
		const bool io_member = group_world <= 1 || gpu()->groupRank() == 0;
		if(fmode == filmio::LoadAndSave)
		{
			film_io.weights.assign((size_t)s.width * s.height, 0.f);
			film_io.rgba.assign((size_t)s.width * s.height * 4, 0.f);
			if(filmio::loadAllInFolder(log, s.film_load_save_path, film_io))
			{
				rp.resumed = true;
				rp.load_rgba = film_io.rgba.data();
				rp.load_weights = film_io.weights.data();
				rp.resume_sampling_offset = film_io.sampling_offset;
				S.base_offset = film_io.base_sampling_offset;
				rp.film.sample_offset = S.base_offset;
				log.info(itype + ": Combining ImageFilm files, skipping pass 1...");
			}
		}
		if(fmode != filmio::None && io_member) filmio::backup(log, film_file);
		auto saveFilm = [&]() {
			filmio::Film out = film_io;
			out.sampling_offset = gpu()->samplingOffset();
			if(gpu()->downloadAccum(out.rgba, out.weights)) filmio::save(log, film_file, out);
		};
		int autosave_passes = 0;
		const auto autosave_t0 = std::chrono::steady_clock::now();
		auto autosave_last = autosave_t0;
		if(fmode != filmio::None && io_member && s.film_autosave_interval_type != "none")
			rp.on_next_pass = [&](bool skipped) {
				++autosave_passes;
				if(skipped) return;
				if(s.film_autosave_interval_type == "pass-interval" && autosave_passes >= s.film_autosave_interval_passes)
				{
					saveFilm();
					autosave_passes = 0;
				}
				// time-interval autosave: checked at pass boundaries (the reference checks per finished tile)
				const auto now = std::chrono::steady_clock::now();
				if(s.film_autosave_interval_type == "time-interval" &&
				   std::chrono::duration<double>(now - autosave_last).count() > s.film_autosave_interval_seconds)
				{
					saveFilm();
					autosave_last = now;
				}
			};
		// tile order of the film splats and of the per-tile callbacks
		const std::vector<int> order = tileOrder(s.width, s.height, s.tile_size, s.tiles_order);
		rp.tile_rank.assign(order.size(), 0u);
		for(size_t k = 0; k < order.size(); ++k) rp.tile_rank[(size_t)order[k]] = (uint32_t)k;
		const bool tile_cbs = !quiet && (cb.put_pixel || cb.flush_area || cb.highlight_area);
		// per-tile callbacks with the one-thread partial film inside the render (one GPU); a group or
		// caller-sharded render reports the tiles after the film is complete (below)
		const bool tiles_in_render = tile_cbs && rp.shard_world == 1;
		if(tiles_in_render)
		{
			// ImageFilm::nextArea / finishArea per tile in render order (imagefilm.cc:447-568):
			// highlightArea, putPixel over the tile (rows, then columns) with the values the one-thread
			// render shows when the tile finishes, flushArea, progress by the tile's area
			const int ntx = (s.width + s.tile_size - 1) / s.tile_size;
			const std::string vname = view.first;
			rp.on_tiles = [&, ntx, vname, order](int pass, const std::vector<float> &part) {
				(void)pass;
				const int n_pix = s.width * s.height;
				int done_px = 0;
				for(size_t k = 0; k < order.size(); ++k)
				{
					const int tx = (order[k] % ntx) * s.tile_size, ty = (order[k] / ntx) * s.tile_size;
					const int x1 = std::min(s.width, tx + s.tile_size), y1 = std::min(s.height, ty + s.tile_size);
					// areas in camera coordinates (imagefilm.cc:462-467, 533), pixels in film coordinates (:527)
					if(cb.highlight_area)
						cb.highlight_area(vname.c_str(), (int)k, tx + s.xstart, ty + s.ystart, x1 + s.xstart, y1 + s.ystart, cb.highlight_area_data);
					if(cb.put_pixel)
						for(int y = ty; y < y1; ++y)
							for(int x = tx; x < x1; ++x)
							{
								const float *px = &part[4 * ((size_t)y * s.width + x)];
								cb.put_pixel(vname.c_str(), "combined", x, y, px[0], px[1], px[2], px[3], cb.put_pixel_data);
							}
					if(cb.flush_area) cb.flush_area(vname.c_str(), (int)k, tx + s.xstart, ty + s.ystart, x1 + s.xstart, y1 + s.ystart, cb.flush_area_data);
					done_px += (x1 - tx) * (y1 - ty);
					if(progress) progress(n_pix, done_px, "Rendering...", progress_data);
				}
			};
		}
		else if(progress && !quiet)
		{
			const int n_pix = s.width * s.height;
			rp.on_chunk = [&, n_pix](uint64_t done, uint64_t total) {
				progress(n_pix, (int)((double)n_pix * (double)done / (double)std::max<uint64_t>(1, total)), "Rendering...", progress_data);
			};
		}
		// photon_maps_processing: files next to the film's load / save path (getFilmSavePath), written by
		// one member of a group
		IntegratorState &ist = integrator_state[s.integrator_name];
		rp.pm.processing = ist.processing;
		rp.pm.owner = ist.id;
		rp.pm.map_path = s.film_load_save_path;
		rp.pm.write_files = io_member;
		bool ok;
		if(!grouped)
		{
			kt_sum_.reset();
			ok = gpu()->render(rp, &canceled);
		}
		else if(group_world > 1)
		{
			kt_sum_.reset();
			ok = gpu()->renderMember(rp, &canceled);
		}
		else ok = renderDeviceGroup(rp);
		if(ist.processing == PhotonParams::PM_LOAD && rp.pm.processing == PhotonParams::PM_GENERATE_SAVE)
			ist.processing = PhotonParams::PM_GENERATE_SAVE;   // integrator_photon_mapping.cc:323, montecarlo.cc:560
		if(!ok) return false;
		if(grouped)
		{
			const std::vector<double> &ms = gpu()->memberMs();
			last_bounds_ = group_bounds;
			last_member_ms_ = ms;
			// the first frame on the initial equal split moves the boundaries all the way to the measured
			// equal-cost split (the second frame is balanced); later frames move half way
			// (damped against frame-to-frame noise).  Every member sees the same bounds and times: same result
			if((int)ms.size() == world)
			{
				const bool initial = group_bounds == equalBands(s.height, world);
				group_bounds = rebalanceBands(group_bounds, ms, 0, initial ? 0.0 : 0.5);
			}
		}
		if(fmode != filmio::None && io_member) saveFilm();
		const double build = stats.build_seconds;
		stats = (grouped && group_world <= 1) ? group_stats_ : gpu()->stats();
		stats.build_seconds = build;
		film_on_gpu_only = quiet;
		if(quiet) continue;
		// the flush needs the colours (putPixel); the weights stay on the GPU until getFilm asks for them
		if(!gpu()->download(film_rgba, film_weights, s.width, s.height, true, false)) return false;
		film_weights_stale = true;
		{
			std::ostringstream os;
			os << "Render: " << stats.samples << " samples, " << stats.closest_rays << " closest + " << stats.shadow_rays
			   << " shadow rays in " << stats.render_seconds << " s";
			log.info(os.str());
		}
		// imagefilm.cc:570-670 flush: every owned pixel, then the flush callback (the per-tile
		// finishArea callbacks ran inside the render, rp.on_tiles)
		const auto owned = gpu()->ownedRows();
		auto ownedRow = [&](int y) {
			for(const auto &r : owned) if(y >= r.first && y < r.second) return true;
			return false;
		};
		if(tile_cbs && !tiles_in_render)
		{
			// ImageFilm::nextArea / finishArea of every tile this process owns, in render order, after the
			// group combined the film (the put-pixel values follow in the flush below)
			const int ntx = (s.width + s.tile_size - 1) / s.tile_size, n_pix = s.width * s.height;
			int done_px = 0;
			for(size_t k = 0; k < order.size(); ++k)
			{
				const int tx = (order[k] % ntx) * s.tile_size, ty = (order[k] / ntx) * s.tile_size;
				const int x1 = std::min(s.width, tx + s.tile_size), y1 = std::min(s.height, ty + s.tile_size);
				int oy0 = y1, oy1 = ty;
				for(int y = ty; y < y1; ++y)
					if(ownedRow(y)) { oy0 = std::min(oy0, y); oy1 = std::max(oy1, y + 1); }
				if(oy1 <= oy0) continue;
				if(cb.highlight_area)
					cb.highlight_area(view.first.c_str(), (int)k, tx + s.xstart, oy0 + s.ystart, x1 + s.xstart, oy1 + s.ystart, cb.highlight_area_data);
				if(cb.flush_area)
					cb.flush_area(view.first.c_str(), (int)k, tx + s.xstart, oy0 + s.ystart, x1 + s.xstart, oy1 + s.ystart, cb.flush_area_data);
				done_px += (x1 - tx) * (oy1 - oy0);
				if(progress) progress(n_pix, done_px, "Rendering...", progress_data);
			}
		}
		if(cb.put_pixel)
			for(int y = 0; y < s.height; ++y)
			{
				if(!ownedRow(y)) continue;
				for(int x = 0; x < s.width; ++x)
				{
					const float *px = &film_rgba[4 * ((size_t)y * s.width + x)];
					cb.put_pixel(view.first.c_str(), "combined", x, y, px[0], px[1], px[2], px[3], cb.put_pixel_data);
				}
			}
		if(cb.flush) cb.flush(view.first.c_str(), cb.flush_data);
		if(progress)
		{
			// a canceled render reports the pixels it completed
			const int done_pix = canceled ? (int)std::min<uint64_t>((uint64_t)s.width * s.height, stats.samples / (uint64_t)std::max(1, s.aa_samples))
			                              : s.width * s.height;
			progress(s.width * s.height, done_pix, canceled ? "Rendering canceled" : "Rendering finished", progress_data);
		}
	}
	return true;
}

} // namespace yafamd
