// Host side of the drop-in library: parameter staging, logging, scene assembly and the render
// entry, mirroring the reference's Interface / Scene / ParamMap / Logger
// (src/interface/interface.cc:34-357, src/scene/scene.cc:203-1060, include/common/param.h:38-112,
// include/common/logger.h:62-166).  Only the GPU renderer (render.h) touches HIP.
#pragma once

#include "pinned.h"
#include "../../include/yafaray_c_api.h"
#include "../../include/yafaray_amd.h"
#include "devscene.h"

#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace yafamd
{
struct HostScene;


// ---- ParamMap (include/common/param.h:38-112: strictly typed getVal) ----
struct Param
{
	enum Type : int { None = -1, Int = 1, Bool, Float, String, Vector, Color, Matrix };
	Type type = None;
	int ival = 0;
	bool bval = false;
	double fval = 0.0;
	std::string sval;
	std::vector<float> vval;
};

class ParamMap
{
	public:
		bool get(const std::string &k, std::string &v) const { auto p = find(k, Param::String); if(p) v = p->sval; return p; }
		bool get(const std::string &k, int &v) const { auto p = find(k, Param::Int); if(p) v = p->ival; return p; }
		bool get(const std::string &k, bool &v) const { auto p = find(k, Param::Bool); if(p) v = p->bval; return p; }
		bool get(const std::string &k, float &v) const { auto p = find(k, Param::Float); if(p) v = (float)p->fval; return p; }
		bool get(const std::string &k, double &v) const { auto p = find(k, Param::Float); if(p) v = p->fval; return p; }
		bool getVec(const std::string &k, float *v3) const
		{
			auto p = find(k, Param::Vector);
			if(p) { v3[0] = p->vval[0]; v3[1] = p->vval[1]; v3[2] = p->vval[2]; }
			return p;
		}
		bool getColor(const std::string &k, float *c4) const
		{
			auto p = find(k, Param::Color);
			if(p) { c4[0] = p->vval[0]; c4[1] = p->vval[1]; c4[2] = p->vval[2]; c4[3] = p->vval[3]; }
			return p;
		}
		Param &operator[](const std::string &k) { return map_[k]; }
		void clear() { map_.clear(); }
		std::string print() const;
		const std::map<std::string, Param> &items() const { return map_; }

	private:
		const Param *find(const std::string &k, Param::Type t) const
		{
			auto it = map_.find(k);
			if(it == map_.end() || it->second.type != t) return nullptr;
			return &it->second;
		}
		std::map<std::string, Param> map_;
};

// ---- Logger (include/common/logger.h:62-166) ----
class Logger
{
	public:
		Logger(yafaray_LoggerCallback_t cb, void *data, yafaray_DisplayConsole_t console) : cb_(cb), data_(data), console_(console) {}
		void setCallback(yafaray_LoggerCallback_t cb, void *data) { cb_ = cb; data_ = data; }
		void setConsoleLevel(int l) { console_level_ = l; }
		void setLogLevel(int l) { log_level_ = l; }
		void setPrintDateTime(bool b) { print_datetime_ = b; }
		void setColors(bool b) { colors_ = b; }
		void log(int level, const std::string &msg, bool set_error = false);
		// thread-safe: the members of a device group log from their own threads
		void error(const std::string &m) { log(YAFARAY_LOG_LEVEL_ERROR, m, true); }
		void warning(const std::string &m) { log(YAFARAY_LOG_LEVEL_WARNING, m); }
		void params(const std::string &m) { log(YAFARAY_LOG_LEVEL_PARAMS, m); }
		void info(const std::string &m) { log(YAFARAY_LOG_LEVEL_INFO, m); }
		void verbose(const std::string &m) { log(YAFARAY_LOG_LEVEL_VERBOSE, m); }
		void debug(const std::string &m) { log(YAFARAY_LOG_LEVEL_DEBUG, m); }
		bool isDebug() const { return console_level_ >= YAFARAY_LOG_LEVEL_DEBUG || log_level_ >= YAFARAY_LOG_LEVEL_DEBUG; }
		const std::string &lastError() const { return last_error_; }
		void clearError()
		{
			std::lock_guard<std::mutex> g(mtx_);
			last_error_.clear();
		}

	private:
		yafaray_LoggerCallback_t cb_;
		void *data_;
		yafaray_DisplayConsole_t console_;
		int console_level_ = YAFARAY_LOG_LEVEL_INFO, log_level_ = YAFARAY_LOG_LEVEL_VERBOSE;
		bool print_datetime_ = true, colors_ = false;
		std::string last_error_;
		std::mutex mtx_;
};

// ---- scene objects ----
struct MeshObject
{
	std::string name;
	std::vector<float> verts;            // xyz (addVertex casts the doubles to float, interface.cc:88)
	std::vector<int> tris;               // abc (object-local vertex indices)
	std::vector<int> tri_mat;            // material index per triangle
	// surface attributes (object_mesh.h:48-76): orco per vertex, uv values + per-triangle uv
	// indices, exported / smoothed vertex normals
	std::vector<float> orco;             // xyz per vertex (addVertexWithOrco)
	std::vector<float> uvs;              // (u, v) per addUv
	std::vector<int> tri_uv;             // 3 per triangle (-1: addTriangle without uv)
	std::vector<float> normals;          // xyz per addNormal / smoothMesh
	std::vector<int> tri_nidx;           // 3 normal indices per triangle (-1: face normal)
	bool smooth = false;
	bool is_base = false;
	std::string visibility = "normal";
	bool ended = false;
};

struct CameraDesc
{
	float from[3] = {0.f, 1.f, 0.f}, to[3] = {0.f, 0.f, 0.f}, up[3] = {0.f, 1.f, 1.f};
	int resx = 320, resy = 200;
	float aspect = 1.f, focal = 1.f, aperture = 0.f;
	float near_clip = 0.f, far_clip = -1.f;
	float dof_distance = 0.f, bokeh_rotation = 0.f;
	std::string bokeh_type = "disk1", bokeh_bias = "uniform";
};

struct RenderSetup
{
	std::string integrator_name, background_name;
	int width = 320, height = 240, xstart = 0, ystart = 0;
	int aa_passes = 1, aa_samples = 1;
	// adaptive AA (scene.cc:582-595; defaults of aa_noise_params.h:27-46)
	int aa_inc_samples = 1;
	float aa_threshold = 0.05f, aa_resampled_floor = 0.f, aa_sample_multiplier_factor = 1.f;
	float aa_light_sample_multiplier_factor = 1.f, aa_indirect_sample_multiplier_factor = 1.f;
	bool aa_detect_color_noise = false;
	std::string aa_dark_detection_type = "none";
	float aa_dark_threshold_factor = 0.f;
	int aa_variance_edge_size = 10, aa_variance_pixels = 0;
	float aa_pixelwidth = 1.5f, clamp_samples = 0.f;
	std::string filter = "box";
	int tile_size = 32;
	std::string tiles_order = "centre";
	int threads = -1, threads_photons = -1;
	// GPUs of this process that render the film together (the device group, one host thread and
	// HIP stream per GPU, row bands combined over xGMI): -1 = every visible device, as the
	// reference's threads = -1 uses every core (scene.cc:547-610); YAFARAY_AMD_GPUS overrides
	int gpus = -1;
	bool shadow_bias_auto = true, ray_min_dist_auto = true;
	float shadow_bias = 0.0005f, ray_min_dist = 0.00005f;
	int base_sampling_offset = 0, computer_node = 0;
	// GPU-core extension: seed of the per-sample Russian-roulette generators (the reference seeds one
	// per tile from rand(), integrator_tiled.cc:272 — matched statistically; the seed lets the parity
	// checks draw independent RR streams)
	int rr_seed = 0;
	// film load/save (imagefilm.cc:55-118)
	std::string film_load_save_mode = "none", film_load_save_path = "./", film_autosave_interval_type = "none";
	int film_autosave_interval_passes = 1;
	double film_autosave_interval_seconds = 300.0;
	std::string accelerator = "yafaray-kdtree-original";
	bool valid = false;
};

struct Callbacks
{
	yafaray_RenderNotifyViewCallback_t notify_view = nullptr; void *notify_view_data = nullptr;
	yafaray_RenderNotifyLayerCallback_t notify_layer = nullptr; void *notify_layer_data = nullptr;
	yafaray_RenderPutPixelCallback_t put_pixel = nullptr; void *put_pixel_data = nullptr;
	yafaray_RenderHighlightPixelCallback_t highlight_pixel = nullptr; void *highlight_pixel_data = nullptr;
	yafaray_RenderFlushAreaCallback_t flush_area = nullptr; void *flush_area_data = nullptr;
	yafaray_RenderFlushCallback_t flush = nullptr; void *flush_data = nullptr;
	yafaray_RenderHighlightAreaCallback_t highlight_area = nullptr; void *highlight_area_data = nullptr;
};

class GpuRenderer;
struct KernelTimes;
struct RenderParams;
struct HostImage;
struct HostTexture;

class Scene
{
	public:
		explicit Scene(Logger &l);
		~Scene();
		Logger &log;
		std::map<std::string, DevMaterial> materials;
		std::map<std::string, int> material_index;    // creation order index
		std::vector<std::string> material_order;
		std::map<std::string, DevLight> lights;        // std::map: name order (render_view.cc:61)
		std::map<std::string, std::string> light_objects;   // meshlight / objectlight -> its object (resolved when the scene is built)
		std::map<std::string, MeshObject> objects;
		std::vector<std::string> object_order;
		std::map<std::string, CameraDesc> cameras;
		std::map<std::string, std::string> views;     // view name -> camera name
		std::map<std::string, std::vector<float>> backgrounds;   // colour * power
		std::map<std::string, ParamMap> integrators;
		// per integrator: its instance id (the photon maps a render keeps belong to it) and its
		// photon_maps_processing mode (a failed "load" turns into "generate-save" for good, as the
		// reference's PhotonIntegrator rewrites its photon_map_processing_)
		struct IntegratorState { uint64_t id = 0; int processing = 0; };
		std::map<std::string, IntegratorState> integrator_state;
		uint64_t integrator_ids_ = 0;
		std::vector<std::string> layers;
		std::map<std::string, ParamMap> outputs;
		std::map<std::string, std::shared_ptr<HostImage>> images;
		std::map<std::string, int> texture_index;                 // name -> textures[]
		std::vector<HostTexture> textures;
		std::map<std::string, std::vector<DevNode>> mat_nodes;    // material -> node program
		RenderSetup setup;
		MeshObject *current_object = nullptr;
		std::string current_material;
		bool geometry_dirty = true;
		int shard_rank = 0, shard_world = 1, shard_mode = 1;
		int shard_y0 = 0, shard_y1 = 0;   // shard_mode 2: explicit row band
		std::vector<int> group_bounds;    // render / device group: row-band boundaries of the members (rebalanced per frame)
		// explicit device group (yafaray_amd_setDeviceGroup): the device of each member (-1: device of
		// member 0 + m, modulo the visible devices); empty: the "gpus" render parameter decides
		std::vector<int> device_group;
		int chunk_slots = 1 << 27;   // samples in flight per wavefront chunk (134 M: the C2 frame in one chunk)
		bool profile_kernels = false;
		bool trace_stats = true;   // per-visit node / triangle counters in k_trace (yafaray_amd_setTraceStats)
		volatile bool canceled = false;

		bool createObject(const std::string &name, const ParamMap &p);
		bool endObject();
		int addVertex(float x, float y, float z);
		int addVertexWithOrco(float x, float y, float z, float ox, float oy, float oz);
		void addNormal(float x, float y, float z);
		int addUv(float u, float v);
		bool addTriangle(int a, int b, int c, int uv_a = -1, int uv_b = -1, int uv_c = -1);
		bool smoothMesh(const std::string &name, float angle);
		bool createMaterial(const std::string &name, const ParamMap &p, const std::list<ParamMap> &nodes);
		HostImage *createImage(const std::string &name, const ParamMap &p);
		bool createTexture(const std::string &name, const ParamMap &p);
		bool createLight(const std::string &name, const ParamMap &p);
		bool createCamera(const std::string &name, const ParamMap &p);
		bool createBackground(const std::string &name, const ParamMap &p);
		bool createIntegrator(const std::string &name, const ParamMap &p);
		bool createRenderView(const std::string &name, const ParamMap &p);
		bool setupRender(const ParamMap &p);
		bool render(const Callbacks &cb, yafaray_ProgressBarCallback_t progress, void *progress_data, bool quiet);
		bool buildAccelerator();
		GpuRenderer *gpu();                 // member 0 (holds the film, serves the ray seam)
		int memberCount() const { return 1 + (int)extra_.size(); }
		GpuRenderer *member(int m);
		bool syncMembers();                 // (re)create the device group's members for the current settings
		const KernelTimes &kernelTimes();   // per-kernel timing of the last profiled render (summed over members)
		std::string groupReport();          // JSON: how the last render was split (yafaray_amd_getGroupReport)

		// film of the last render
		PinnedFloats film_rgba, film_weights;   // page-locked: the per-frame download is a DMA
		int film_w = 0, film_h = 0;
		bool film_on_gpu_only = false;   // the last render was quiet: film_rgba / film_weights are stale
		bool film_weights_stale = false; // the last flush downloaded film_rgba only (getFilm fetches the weights)
		yafaray_amd_stats_t stats{};

	private:
		bool renderDeviceGroup(RenderParams &rp);
		bool meshLightFaces(const std::string &name, DevLight &L, HostScene &hs);
		std::unique_ptr<GpuRenderer> gpu_;
		std::vector<std::unique_ptr<GpuRenderer>> extra_;   // device group members 1..
		std::vector<int> member_devs_;                      // devices of the current members
		std::unique_ptr<KernelTimes> kt_sum_;
		yafaray_amd_stats_t group_stats_{};                 // counters of the last device-group render
		std::vector<int> last_bounds_;                      // band boundaries the last group render used
		std::vector<double> last_member_ms_;                // and each member's render time
};

class Interface
{
	public:
		Interface(yafaray_LoggerCallback_t cb, void *data, yafaray_DisplayConsole_t console) : logger(cb, data, console), cparams(&params) {}
		Logger logger;
		ParamMap params;
		std::list<ParamMap> nodes_params;
		ParamMap *cparams;
		std::unique_ptr<Scene> scene;
		Callbacks callbacks;
		float input_gamma = 1.f;
		int input_color_space = 1;   // RawManualGamma (interface.h:133-134)

		Scene *sc()
		{
			if(!scene) { logger.error("Interface: no scene created (call yafaray_createScene first)"); }
			return scene.get();
		}
};

} // namespace yafamd
