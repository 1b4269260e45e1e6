// extern "C" entry points of libyafaray4.so — the drop-in boundary (include/yafaray_c_api.h) and
// the MI355X extensions (include/yafaray_amd.h).  Reference counterpart:
// src/public_api/yafaray_c_api.cc:32-433 + src/interface/interface.cc:34-357.
#include "../../include/yafaray_amd.h"
#include "../../include/yafaray_c_api.h"
#include "host.h"
#include "texture.h"
#include "hostmath.h"
#include "render.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace yafamd;

static Interface *I(yafaray_Interface_t *p) { return reinterpret_cast<Interface *>(p); }
static const Interface *I(const yafaray_Interface_t *p) { return reinterpret_cast<const Interface *>(p); }

static char *dupString(const std::string &s)
{
	char *c = static_cast<char *>(std::malloc(s.size() + 1));
	std::memcpy(c, s.c_str(), s.size() + 1);
	return c;
}

extern "C" int yafamd_phase_cycles(unsigned long long *out, int n, int reset);
extern "C" const char *yafamd_device_build();
#define YAF_HOST_BUILD "hipcc/clang " __VERSION__ " -O3 -ffp-contract=off"

extern "C" {

yafaray_Interface_t *yafaray_createInterface(yafaray_Interface_Type_t interface_type, const char *exported_file_path, yafaray_LoggerCallback_t logger_callback, void *callback_data, yafaray_DisplayConsole_t display_console)
{
	auto *it = new Interface(logger_callback, callback_data, display_console);
	if(interface_type != YAFARAY_INTERFACE_FOR_RENDERING)
		it->logger.warning("Interface: scene exporters (XML/C/Python) are not part of the GPU core; creating a rendering interface");
	(void)exported_file_path;
	return reinterpret_cast<yafaray_Interface_t *>(it);
}

void yafaray_destroyInterface(yafaray_Interface_t *interface) { delete I(interface); }

void yafaray_setLoggingCallback(yafaray_Interface_t *interface, yafaray_LoggerCallback_t cb, void *data) { I(interface)->logger.setCallback(cb, data); }

void yafaray_createScene(yafaray_Interface_t *interface)
{
	Interface *it = I(interface);
	it->scene.reset(new Scene(it->logger));
	it->params.clear();
}

int yafaray_getSceneFilmWidth(const yafaray_Interface_t *interface)
{
	const Interface *it = I(interface);
	return it->scene ? it->scene->setup.width : 0;
}

int yafaray_getSceneFilmHeight(const yafaray_Interface_t *interface)
{
	const Interface *it = I(interface);
	return it->scene ? it->scene->setup.height : 0;
}

yafaray_bool_t yafaray_startGeometry(yafaray_Interface_t *interface) { return I(interface)->sc() ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE; }
yafaray_bool_t yafaray_endGeometry(yafaray_Interface_t *interface) { return I(interface)->sc() ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE; }

unsigned int yafaray_getNextFreeId(yafaray_Interface_t *interface)
{
	Scene *s = I(interface)->sc();
	return s ? (unsigned int)s->objects.size() + 1 : 0;
}

yafaray_bool_t yafaray_endObject(yafaray_Interface_t *interface)
{
	Scene *s = I(interface)->sc();
	return (s && s->endObject()) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

int yafaray_addVertex(yafaray_Interface_t *interface, double x, double y, double z)
{
	Scene *s = I(interface)->sc();
	return s ? s->addVertex((float)x, (float)y, (float)z) : -1;
}

int yafaray_addVertexWithOrco(yafaray_Interface_t *interface, double x, double y, double z, double ox, double oy, double oz)
{
	Scene *s = I(interface)->sc();
	return s ? s->addVertexWithOrco((float)x, (float)y, (float)z, (float)ox, (float)oy, (float)oz) : -1;
}

void yafaray_addNormal(yafaray_Interface_t *interface, double nx, double ny, double nz)
{
	Scene *s = I(interface)->sc();
	if(s) s->addNormal((float)nx, (float)ny, (float)nz);
}

yafaray_bool_t yafaray_addTriangle(yafaray_Interface_t *interface, int a, int b, int c)
{
	Scene *s = I(interface)->sc();
	return (s && s->addTriangle(a, b, c)) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

yafaray_bool_t yafaray_addTriangleWithUv(yafaray_Interface_t *interface, int a, int b, int c, int uv_a, int uv_b, int uv_c)
{
	Scene *s = I(interface)->sc();
	return (s && s->addTriangle(a, b, c, uv_a, uv_b, uv_c)) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

int yafaray_addUv(yafaray_Interface_t *interface, float u, float v)
{
	Scene *s = I(interface)->sc();
	return s ? s->addUv(u, v) : 0;
}

yafaray_bool_t yafaray_smoothMesh(yafaray_Interface_t *interface, const char *name, double angle)
{
	Scene *s = I(interface)->sc();
	return (s && s->smoothMesh(name ? name : "", (float)angle)) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

yafaray_bool_t yafaray_addInstance(yafaray_Interface_t *interface, const char *base_object_name, float, float, float, float, float, float, float, float, float, float, float, float, float, float, float, float)
{
	I(interface)->logger.error(std::string("Scene: instances ('") + (base_object_name ? base_object_name : "") + "') are not supported by the GPU core yet");
	return YAFARAY_BOOL_FALSE;
}

yafaray_bool_t yafaray_addInstanceArray(yafaray_Interface_t *interface, const char *base_object_name, const float obj_to_world[4][4])
{
	(void)obj_to_world;
	return yafaray_addInstance(interface, base_object_name, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0);
}

// ---- params (interface.cc:118-172) ----
void yafaray_paramsSetVector(yafaray_Interface_t *interface, const char *name, double x, double y, double z)
{
	Param &p = (*I(interface)->cparams)[name];
	p = Param();
	p.type = Param::Vector;
	p.vval = {(float)x, (float)y, (float)z};
}

void yafaray_paramsSetString(yafaray_Interface_t *interface, const char *name, const char *s)
{
	Param &p = (*I(interface)->cparams)[name];
	p = Param();
	p.type = Param::String;
	p.sval = s ? s : "";
}

void yafaray_paramsSetBool(yafaray_Interface_t *interface, const char *name, yafaray_bool_t b)
{
	Param &p = (*I(interface)->cparams)[name];
	p = Param();
	p.type = Param::Bool;
	p.bval = b != YAFARAY_BOOL_FALSE;
}

void yafaray_paramsSetInt(yafaray_Interface_t *interface, const char *name, int i)
{
	Param &p = (*I(interface)->cparams)[name];
	p = Param();
	p.type = Param::Int;
	p.ival = i;
}

void yafaray_paramsSetFloat(yafaray_Interface_t *interface, const char *name, double f)
{
	Param &p = (*I(interface)->cparams)[name];
	p = Param();
	p.type = Param::Float;
	p.fval = f;
}

void yafaray_paramsSetColor(yafaray_Interface_t *interface, const char *name, float r, float g, float b, float a)
{
	Interface *it = I(interface);
	float c[3] = {r, g, b};
	// Rgb::linearRgbFromColorSpace (color.h:352-380) with the interface's input colour space
	if(it->input_color_space == 3)
		for(float &v : c) v = hm::linearFromSrgb(v);
	else if(it->input_color_space == 4)
	{
		const float m[3][3] = {{3.2406255f, -1.537208f, -0.4986286f}, {-0.9689307f, 1.8757561f, 0.0415175f}, {0.0557101f, -0.2040211f, 1.0569959f}};
		const float o[3] = {c[0], c[1], c[2]};
		for(int k = 0; k < 3; ++k) c[k] = m[k][0] * o[0] + m[k][1] * o[1] + m[k][2] * o[2];
	}
	else if(it->input_color_space == 1 && it->input_gamma != 1.f)
		for(float &v : c) v = hm::powf_fast(v, it->input_gamma);
	Param &p = (*it->cparams)[name];
	p = Param();
	p.type = Param::Color;
	p.vval = {c[0], c[1], c[2], a};
}

void yafaray_paramsSetMatrix(yafaray_Interface_t *interface, const char *name, float m_00, float m_01, float m_02, float m_03, float m_10, float m_11, float m_12, float m_13, float m_20, float m_21, float m_22, float m_23, float m_30, float m_31, float m_32, float m_33, yafaray_bool_t transpose)
{
	Param &p = (*I(interface)->cparams)[name];
	p = Param();
	p.type = Param::Matrix;
	p.vval = {m_00, m_01, m_02, m_03, m_10, m_11, m_12, m_13, m_20, m_21, m_22, m_23, m_30, m_31, m_32, m_33};
	if(transpose)
		for(int i = 0; i < 4; ++i)
			for(int j = i + 1; j < 4; ++j) std::swap(p.vval[i * 4 + j], p.vval[j * 4 + i]);
}

void yafaray_paramsSetMatrixArray(yafaray_Interface_t *interface, const char *name, const float m[4][4], yafaray_bool_t transpose)
{
	yafaray_paramsSetMatrix(interface, name, m[0][0], m[0][1], m[0][2], m[0][3], m[1][0], m[1][1], m[1][2], m[1][3], m[2][0], m[2][1], m[2][2], m[2][3], m[3][0], m[3][1], m[3][2], m[3][3], transpose);
}

void yafaray_paramsClearAll(yafaray_Interface_t *interface)
{
	Interface *it = I(interface);
	it->params.clear();
	it->nodes_params.clear();
	it->cparams = &it->params;
}

void yafaray_paramsPushList(yafaray_Interface_t *interface)
{
	Interface *it = I(interface);
	it->nodes_params.emplace_back();
	it->cparams = &it->nodes_params.back();
}

void yafaray_paramsEndList(yafaray_Interface_t *interface)
{
	Interface *it = I(interface);
	it->cparams = &it->params;
}

// ---- create* (interface.cc:183-197) ----
void yafaray_setCurrentMaterial(yafaray_Interface_t *interface, const char *name)
{
	Scene *s = I(interface)->sc();
	if(!s) return;
	if(!s->materials.count(name ? name : "")) s->log.warning(std::string("Scene: material '") + (name ? name : "") + "' not found");
	s->current_material = name ? name : "";
}

#define CREATE(fn, method)                                                                     \
	yafaray_bool_t fn(yafaray_Interface_t *interface, const char *name)                        \
	{                                                                                          \
		Interface *it = I(interface);                                                          \
		Scene *s = it->sc();                                                                   \
		return (s && s->method(name ? name : "", it->params)) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE; \
	}

CREATE(yafaray_createObject, createObject)
CREATE(yafaray_createLight, createLight)
yafaray_bool_t yafaray_createMaterial(yafaray_Interface_t *interface, const char *name)
{
	// interface.cc:183-186: the material factory also receives the pushed node lists
	Interface *it = I(interface);
	Scene *s = it->sc();
	return (s && s->createMaterial(name ? name : "", it->params, it->nodes_params)) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}
CREATE(yafaray_createCamera, createCamera)
CREATE(yafaray_createBackground, createBackground)
CREATE(yafaray_createIntegrator, createIntegrator)
CREATE(yafaray_createRenderView, createRenderView)

yafaray_bool_t yafaray_createTexture(yafaray_Interface_t *interface, const char *name)
{
	Interface *it = I(interface);
	Scene *s = it->sc();
	return (s && s->createTexture(name ? name : "", it->params)) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

yafaray_bool_t yafaray_createVolumeRegion(yafaray_Interface_t *interface, const char *name)
{
	I(interface)->logger.error(std::string("Scene: volume region '") + (name ? name : "") + "': participating media are not supported by the GPU core");
	return YAFARAY_BOOL_FALSE;
}

yafaray_bool_t yafaray_createOutput(yafaray_Interface_t *interface, const char *name)
{
	Interface *it = I(interface);
	Scene *s = it->sc();
	if(!s) return YAFARAY_BOOL_FALSE;
	s->outputs[name ? name : ""] = it->params;
	it->logger.warning(std::string("Scene: image output '") + (name ? name : "") + "' registered; image files are not written by the GPU core (use the put-pixel callbacks / yafaray_amd_getFilm)");
	return YAFARAY_BOOL_TRUE;
}

yafaray_bool_t yafaray_removeOutput(yafaray_Interface_t *interface, const char *name)
{
	Scene *s = I(interface)->sc();
	return (s && s->outputs.erase(name ? name : "")) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

void yafaray_clearOutputs(yafaray_Interface_t *interface)
{
	Scene *s = I(interface)->sc();
	if(s) s->outputs.clear();
}

void yafaray_clearAll(yafaray_Interface_t *interface)
{
	Interface *it = I(interface);
	if(it->scene) it->scene.reset(new Scene(it->logger));
	it->params.clear();
	it->nodes_params.clear();
	it->cparams = &it->params;
}

// ---- callbacks ----
#define SETCB(fn, type, field)                                                                 \
	void fn(yafaray_Interface_t *interface, type cb, void *data)                               \
	{                                                                                          \
		I(interface)->callbacks.field = cb;                                                    \
		I(interface)->callbacks.field##_data = data;                                           \
	}
SETCB(yafaray_setRenderNotifyViewCallback, yafaray_RenderNotifyViewCallback_t, notify_view)
SETCB(yafaray_setRenderNotifyLayerCallback, yafaray_RenderNotifyLayerCallback_t, notify_layer)
SETCB(yafaray_setRenderPutPixelCallback, yafaray_RenderPutPixelCallback_t, put_pixel)
SETCB(yafaray_setRenderHighlightPixelCallback, yafaray_RenderHighlightPixelCallback_t, highlight_pixel)
SETCB(yafaray_setRenderFlushAreaCallback, yafaray_RenderFlushAreaCallback_t, flush_area)
SETCB(yafaray_setRenderFlushCallback, yafaray_RenderFlushCallback_t, flush)
SETCB(yafaray_setRenderHighlightAreaCallback, yafaray_RenderHighlightAreaCallback_t, highlight_area)

// ---- render ----
void yafaray_setupRender(yafaray_Interface_t *interface)
{
	Interface *it = I(interface);
	Scene *s = it->sc();
	if(s) s->setupRender(it->params);
}

void yafaray_render(yafaray_Interface_t *interface, yafaray_ProgressBarCallback_t monitor_callback, void *callback_data, yafaray_DisplayConsole_t progress_bar_display_console)
{
	(void)progress_bar_display_console;
	Interface *it = I(interface);
	Scene *s = it->sc();
	if(s) s->render(it->callbacks, monitor_callback, callback_data, false);
}

void yafaray_defineLayer(yafaray_Interface_t *interface)
{
	Interface *it = I(interface);
	Scene *s = it->sc();
	if(!s) return;
	std::string type;
	it->params.get("type", type);
	if(type != "combined") it->logger.warning("Layers: layer '" + type + "' is not produced by the GPU core (combined only)");
	s->layers.push_back(type);
}

// ---- logging ----
void yafaray_enablePrintDateTime(yafaray_Interface_t *interface, yafaray_bool_t value) { I(interface)->logger.setPrintDateTime(value != YAFARAY_BOOL_FALSE); }
void yafaray_setConsoleVerbosityLevel(yafaray_Interface_t *interface, yafaray_LogLevel_t l) { I(interface)->logger.setConsoleLevel((int)l); }
void yafaray_setLogVerbosityLevel(yafaray_Interface_t *interface, yafaray_LogLevel_t l) { I(interface)->logger.setLogLevel((int)l); }

yafaray_LogLevel_t yafaray_logLevelFromString(const char *s)
{
	const std::string v = s ? s : "";
	if(v == "mute") return YAFARAY_LOG_LEVEL_MUTE;
	if(v == "error") return YAFARAY_LOG_LEVEL_ERROR;
	if(v == "warning") return YAFARAY_LOG_LEVEL_WARNING;
	if(v == "params") return YAFARAY_LOG_LEVEL_PARAMS;
	if(v == "info") return YAFARAY_LOG_LEVEL_INFO;
	if(v == "verbose") return YAFARAY_LOG_LEVEL_VERBOSE;
	if(v == "debug") return YAFARAY_LOG_LEVEL_DEBUG;
	return YAFARAY_LOG_LEVEL_VERBOSE;
}

void yafaray_printDebug(yafaray_Interface_t *interface, const char *msg) { I(interface)->logger.debug(msg ? msg : ""); }
void yafaray_printVerbose(yafaray_Interface_t *interface, const char *msg) { I(interface)->logger.verbose(msg ? msg : ""); }
void yafaray_printInfo(yafaray_Interface_t *interface, const char *msg) { I(interface)->logger.info(msg ? msg : ""); }
void yafaray_printParams(yafaray_Interface_t *interface, const char *msg) { I(interface)->logger.params(msg ? msg : ""); }
void yafaray_printWarning(yafaray_Interface_t *interface, const char *msg) { I(interface)->logger.warning(msg ? msg : ""); }
void yafaray_printError(yafaray_Interface_t *interface, const char *msg) { I(interface)->logger.error(msg ? msg : ""); }

void yafaray_cancelRendering(yafaray_Interface_t *interface)
{
	Interface *it = I(interface);
	if(it->scene) it->scene->canceled = true;   // polled between wavefront chunks
}

void yafaray_setInputColorSpace(yafaray_Interface_t *interface, const char *color_space_string, float gamma_val)
{
	Interface *it = I(interface);
	const std::string n = color_space_string ? color_space_string : "";
	// Rgb::colorSpaceFromName (color.cc:123-130)
	if(n == "LinearRGB") it->input_color_space = 2;
	else if(n == "sRGB") it->input_color_space = 3;
	else if(n == "XYZ") it->input_color_space = 4;
	else it->input_color_space = 1;
	it->input_gamma = gamma_val;
}

// ---- images (scene.cc:518-521, image.cc:38-137): owned by the scene, as in the reference (scene.h:214) ----
yafaray_Image_t *yafaray_createImage(yafaray_Interface_t *interface, const char *name)
{
	Interface *it = I(interface);
	Scene *s = it->sc();
	return s ? reinterpret_cast<yafaray_Image_t *>(s->createImage(name ? name : "", it->params)) : nullptr;
}

// Image::setColor through the image's buffer type (quantised as the reference stores it)
yafaray_bool_t yafaray_setImageColor(yafaray_Image_t *image, int x, int y, float r, float g, float b, float a)
{
	auto *img = reinterpret_cast<HostImage *>(image);
	if(!img || x < 0 || y < 0 || x >= img->w || y >= img->h) return YAFARAY_BOOL_FALSE;
	const float c[4] = {r, g, b, a};
	img->setColor(x, y, c);
	return YAFARAY_BOOL_TRUE;
}

yafaray_bool_t yafaray_getImageColor(const yafaray_Image_t *image, int x, int y, float *r, float *g, float *b, float *a)
{
	auto *img = reinterpret_cast<const HostImage *>(image);
	if(!img || x < 0 || y < 0 || x >= img->w || y >= img->h) return YAFARAY_BOOL_FALSE;
	float c[4];
	img->getColor(x, y, c);
	*r = c[0]; *g = c[1]; *b = c[2]; *a = c[3];
	return YAFARAY_BOOL_TRUE;
}

void yafaray_setConsoleLogColorsEnabled(yafaray_Interface_t *interface, yafaray_bool_t colors_enabled) { I(interface)->logger.setColors(colors_enabled != YAFARAY_BOOL_FALSE); }

int yafaray_getVersionMajor() { return 4; }
int yafaray_getVersionMinor() { return 0; }
int yafaray_getVersionPatch() { return 0; }
char *yafaray_getVersionString() { return dupString("4.0.0-mi355x (libYafaRay C API on HIP/gfx950)"); }

char *yafaray_getLayersTable(const yafaray_Interface_t *interface)
{
	(void)interface;
	return dupString("combined\tCombined\tColorAlpha\n");
}

char *yafaray_getViewsTable(const yafaray_Interface_t *interface)
{
	const Interface *it = I(interface);
	std::string s;
	if(it->scene)
		for(const auto &v : it->scene->views) s += v.first + "\t" + v.second + "\n";
	return dupString(s);
}

void yafaray_deallocateCharPointer(char *p) { std::free(p); }

// ---------------------------------------------------------------------------------------------
// extensions (include/yafaray_amd.h)
// ---------------------------------------------------------------------------------------------
int yafaray_amd_addVertices(yafaray_Interface_t *interface, const double *xyz, int n)
{
	Scene *s = I(interface)->sc();
	if(!s || !s->current_object) { I(interface)->logger.error("Scene: addVertices() outside of an object"); return -1; }
	int last = -1;
	for(int i = 0; i < n; ++i) last = s->addVertex((float)xyz[3 * i], (float)xyz[3 * i + 1], (float)xyz[3 * i + 2]);
	return last;
}

yafaray_bool_t yafaray_amd_addTriangles(yafaray_Interface_t *interface, const int *abc, int n)
{
	Scene *s = I(interface)->sc();
	if(!s) return YAFARAY_BOOL_FALSE;
	for(int i = 0; i < n; ++i)
		if(!s->addTriangle(abc[3 * i], abc[3 * i + 1], abc[3 * i + 2])) return YAFARAY_BOOL_FALSE;
	return YAFARAY_BOOL_TRUE;
}

yafaray_bool_t yafaray_amd_buildAccelerator(yafaray_Interface_t *interface)
{
	Scene *s = I(interface)->sc();
	return (s && s->buildAccelerator()) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

yafaray_bool_t yafaray_amd_traceClosest(yafaray_Interface_t *interface, const float *rays, int n, float *t, int *prims)
{
	Scene *s = I(interface)->sc();
	if(!s) return YAFARAY_BOOL_FALSE;
	if(s->geometry_dirty && !s->buildAccelerator()) return YAFARAY_BOOL_FALSE;
	return s->gpu()->traceRays(false, rays, n, t, prims) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

yafaray_bool_t yafaray_amd_traceShadow(yafaray_Interface_t *interface, const float *rays, int n, int *occluded)
{
	Scene *s = I(interface)->sc();
	if(!s) return YAFARAY_BOOL_FALSE;
	if(s->geometry_dirty && !s->buildAccelerator()) return YAFARAY_BOOL_FALSE;
	std::vector<float> t((size_t)std::max(n, 1));
	if(!s->gpu()->traceRays(true, rays, n, t.data(), nullptr)) return YAFARAY_BOOL_FALSE;
	for(int i = 0; i < n; ++i) occluded[i] = t[i] != 0.f ? 1 : 0;
	return YAFARAY_BOOL_TRUE;
}

yafaray_bool_t yafaray_amd_getFilm(const yafaray_Interface_t *interface, float *rgba, float *weights)
{
	const Interface *it = I(interface);
	if(!it->scene) return YAFARAY_BOOL_FALSE;
	Scene *s = it->scene.get();
	// a quiet render (renderQuiet) leaves the film on the GPU: fetch it now
	if(s->film_on_gpu_only)
	{
		if(!s->gpu()->download(s->film_rgba, s->film_weights, s->film_w, s->film_h)) return YAFARAY_BOOL_FALSE;
		s->film_weights_stale = false;
	}
	else if(s->film_weights_stale && weights)
	{
		// a flushed render downloaded the colours only (the put-pixel values): the weights on demand
		if(!s->gpu()->download(s->film_rgba, s->film_weights, s->film_w, s->film_h, false)) return YAFARAY_BOOL_FALSE;
		s->film_weights_stale = false;
	}
	s->film_on_gpu_only = false;
	if(s->film_rgba.empty()) return YAFARAY_BOOL_FALSE;
	if(rgba) std::memcpy(rgba, it->scene->film_rgba.data(), it->scene->film_rgba.size() * 4);
	if(weights) std::memcpy(weights, it->scene->film_weights.data(), it->scene->film_weights.size() * 4);
	return YAFARAY_BOOL_TRUE;
}

yafaray_bool_t yafaray_amd_getFilmDevice(const yafaray_Interface_t *interface, void *rgba_dev, int y0, int y1)
{
	const Interface *it = I(interface);
	if(!it->scene) return YAFARAY_BOOL_FALSE;
	return it->scene->gpu()->filmToDevice(rgba_dev, y0, y1) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

void yafaray_amd_setTileRowShard(yafaray_Interface_t *interface, int rank, int world)
{
	Scene *s = I(interface)->sc();
	if(!s) return;
	s->shard_world = world < 1 ? 1 : world;
	s->shard_rank = (rank < 0 || rank >= s->shard_world) ? 0 : rank;
	s->shard_mode = 0;
}

void yafaray_amd_setRowBandShard(yafaray_Interface_t *interface, int rank, int world)
{
	Scene *s = I(interface)->sc();
	if(!s) return;
	s->shard_world = world < 1 ? 1 : world;
	s->shard_rank = (rank < 0 || rank >= s->shard_world) ? 0 : rank;
	s->shard_mode = 1;
}

void yafaray_amd_setRowBandRange(yafaray_Interface_t *interface, int y0, int y1, int world)
{
	Scene *s = I(interface)->sc();
	if(!s) return;
	s->shard_world = world < 1 ? 1 : world;
	s->shard_rank = 0;
	s->shard_mode = 2;
	s->shard_y0 = y0;
	s->shard_y1 = y1;
}

int yafaray_amd_getOwnedRows(const yafaray_Interface_t *interface, int *rows, int max_ranges)
{
	const Interface *it = I(interface);
	if(!it->scene) return 0;
	const auto owned = it->scene->gpu()->ownedRows();
	const int n = (int)owned.size();
	for(int k = 0; k < n && k < max_ranges && rows; ++k)
	{
		rows[2 * k] = owned[k].first;
		rows[2 * k + 1] = owned[k].second;
	}
	return n;
}

yafaray_bool_t yafaray_amd_renderQuiet(yafaray_Interface_t *interface)
{
	Interface *it = I(interface);
	Scene *s = it->sc();
	Callbacks none;
	return (s && s->render(none, nullptr, nullptr, true)) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

// yafaray_amd_getStats has two versions.  @LIBYAFARAY_AMD_1.0 (what clients linked before 1.4
// bound to) copies the 1.0 struct's fields only: the oldest clients allocate no more.  The default
// @@LIBYAFARAY_AMD_1.4 (what a client linking now binds to) copies every field the header carried
// while getStats was the only accessor — through fg_thin_rounds — so a client built against that header
// reads them all; getStatsEx copies any length.
void yafamd_getStats_v1_0(const yafaray_Interface_t *interface, yafaray_amd_stats_t *stats)
{
	const Interface *it = I(interface);
	if(it->scene && stats) std::memcpy((void *)stats, &it->scene->stats, YAFARAY_AMD_STATS_V1_0_SIZE);
}

void yafamd_getStats_v1_4(const yafaray_Interface_t *interface, yafaray_amd_stats_t *stats)
{
	const Interface *it = I(interface);
	if(it->scene && stats) std::memcpy((void *)stats, &it->scene->stats, YAFARAY_AMD_STATS_V1_4_SIZE);
}
__asm__(".symver yafamd_getStats_v1_0, yafaray_amd_getStats@LIBYAFARAY_AMD_1.0");
__asm__(".symver yafamd_getStats_v1_4, yafaray_amd_getStats@@LIBYAFARAY_AMD_1.4");

const char *yafaray_amd_buildInfo()
{
	static const std::string info = std::string("device: ") + yafamd_device_build() + "; host: " + YAF_HOST_BUILD;
	return info.c_str();
}

size_t yafaray_amd_getGroupReport(yafaray_Interface_t *interface, char *buf, size_t bytes)
{
	Scene *s = I(interface)->sc();
	if(!s) return 0;
	const std::string r = s->groupReport();
	if(buf && bytes)
	{
		const size_t n = std::min(bytes - 1, r.size());
		std::memcpy(buf, r.data(), n);
		buf[n] = 0;
	}
	return r.size() + 1;
}

size_t yafaray_amd_getStatsEx(const yafaray_Interface_t *interface, yafaray_amd_stats_t *stats, size_t bytes)
{
	const Interface *it = I(interface);
	if(!it->scene || !stats) return 0;
	const size_t n = std::min(bytes, sizeof(yafaray_amd_stats_t));
	std::memcpy((void *)stats, &it->scene->stats, n);
	return n;
}

yafaray_bool_t yafaray_amd_setDeviceGroup(yafaray_Interface_t *interface, int members, const int *devices)
{
	Scene *s = I(interface)->sc();
	if(!s) return YAFARAY_BOOL_FALSE;
	s->device_group.clear();
	for(int m = 0; m < members; ++m) s->device_group.push_back(devices ? devices[m] : -1);
	if(members > 64)
	{
		I(interface)->logger.error("Device group: at most 64 members");
		s->device_group.clear();
		return YAFARAY_BOOL_FALSE;
	}
	return YAFARAY_BOOL_TRUE;
}

int yafaray_amd_getDeviceGroupSize(yafaray_Interface_t *interface)
{
	Scene *s = I(interface)->sc();
	if(!s || !s->syncMembers()) return 0;
	return s->memberCount();
}

void yafaray_amd_setChunkSlots(yafaray_Interface_t *interface, int slots)
{
	Scene *s = I(interface)->sc();
	if(s) s->chunk_slots = slots < 1024 ? 1024 : slots;
}

void yafaray_amd_setTraceStats(yafaray_Interface_t *interface, yafaray_bool_t enable)
{
	Scene *s = I(interface)->sc();
	if(s) s->trace_stats = enable != YAFARAY_BOOL_FALSE;
}

void yafaray_amd_setProfileKernels(yafaray_Interface_t *interface, yafaray_bool_t enable)
{
	Scene *s = I(interface)->sc();
	if(s) s->profile_kernels = enable != YAFARAY_BOOL_FALSE;
}

const char *yafaray_amd_lastError(const yafaray_Interface_t *interface) { return I(interface)->logger.lastError().c_str(); }

int yafaray_amd_getRenderGroupId(void *id, int bytes)
{
	ncclUniqueId uid;
	if(!id || bytes < (int)sizeof(uid) || ncclGetUniqueId(&uid) != ncclSuccess) return 0;
	std::memcpy(id, &uid, sizeof(uid));
	return (int)sizeof(uid);
}

yafaray_bool_t yafaray_amd_setRenderGroup(yafaray_Interface_t *interface, int rank, int world, const void *id, int bytes)
{
	Scene *s = I(interface)->sc();
	if(!s) return YAFARAY_BOOL_FALSE;
	s->group_bounds.clear();
	return s->gpu()->joinGroup(rank, world, id, bytes < 0 ? 0 : (size_t)bytes) ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

int yafaray_amd_rebalanceBands(const int *bounds, int world, const double *times, int cap_rows, int *out)
{
	if(!bounds || !times || !out || world < 1) return 0;
	const std::vector<int> b(bounds, bounds + world + 1);
	const std::vector<double> t(times, times + world);
	const std::vector<int> nb = rebalanceBands(b, t, cap_rows);
	for(int r = 0; r <= world; ++r) out[r] = nb[r];
	return 1;
}

// the point kd-tree build on its own (a batched seam for PointKdTree<T>::PointKdTree,
// include/photon/pkdtree.h:115-222): n positions (xyz) in, 2n - 1 nodes (4 x uint32 each, the
// layout of pkd.hip) and the deepest level out; runs on the current HIP device with its own stream
extern "C" hipError_t yafamd_build_pkd(const float4 *pos_dev, uint32_t n, uint4 *nodes_dev, int *depth_out, hipStream_t st, void **scratch);
extern "C" void yafamd_pkd_scratch_free(void *scratch);
yafaray_bool_t yafaray_amd_buildPhotonTree(const float *xyz, int n, unsigned int *nodes, int *depth)
{
	if(!xyz || !nodes || !depth || n < 1) return YAFARAY_BOOL_FALSE;
	std::vector<float4> pos((size_t)n);
	for(int i = 0; i < n; ++i) pos[(size_t)i] = make_float4(xyz[3 * (size_t)i], xyz[3 * (size_t)i + 1], xyz[3 * (size_t)i + 2], 0.f);
	float4 *pos_dev = nullptr;
	uint4 *nodes_dev = nullptr;
	hipStream_t st = nullptr;
	void *scratch = nullptr;
	bool ok = hipStreamCreate(&st) == hipSuccess && hipMalloc(&pos_dev, pos.size() * sizeof(float4)) == hipSuccess &&
	          hipMalloc(&nodes_dev, (2 * (size_t)n - 1) * sizeof(uint4)) == hipSuccess &&
	          hipMemcpyAsync(pos_dev, pos.data(), pos.size() * sizeof(float4), hipMemcpyHostToDevice, st) == hipSuccess &&
	          yafamd_build_pkd(pos_dev, (uint32_t)n, nodes_dev, depth, st, &scratch) == hipSuccess &&
	          hipMemcpyAsync(nodes, nodes_dev, (2 * (size_t)n - 1) * sizeof(uint4), hipMemcpyDeviceToHost, st) == hipSuccess &&
	          hipStreamSynchronize(st) == hipSuccess;
	if(scratch) yafamd_pkd_scratch_free(scratch);
	if(pos_dev) (void)hipFree(pos_dev);
	if(nodes_dev) (void)hipFree(nodes_dev);
	if(st) (void)hipStreamDestroy(st);
	return ok ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

// (1.6) a device / render group member's share of the distributed build (pkd.hip yafamd_build_pkd_kd_member):
// the whole top above the split level and the member's own subtrees, nodes and kd-order positions out
// (the other members' ranges zero); built twice, *ms = the second build's device time
extern "C" hipError_t yafamd_build_pkd_kd_member(const float4 *pos_dev, const float4 *dir_dev, const float *colb_dev, uint32_t n, uint4 *nodes_dev,
                                                 float4 *kpos, float4 *kdir, float *kcolb, int *depth_out, hipStream_t st, void **scratch, int member,
                                                 int members, int *split_level);
extern "C" void yafamd_pkd_top_segments(uint32_t n, int level, uint32_t *out);
extern "C" void yafamd_pkd_owned_segments(int level, int member, int members, uint32_t *s0, uint32_t *s1);
yafaray_bool_t yafaray_amd_buildPhotonTreeMember(const float *xyz, int n, int member, int members, unsigned int *nodes, float *kd_pos, int *depth,
                                                 int *split_level, double *ms)
{
	if(!xyz || !nodes || !kd_pos || !depth || !split_level || n < 1 || members < 1 || member < 0 || member >= members) return YAFARAY_BOOL_FALSE;
	std::vector<float4> pos((size_t)n);
	for(int i = 0; i < n; ++i) pos[(size_t)i] = make_float4(xyz[3 * (size_t)i], xyz[3 * (size_t)i + 1], xyz[3 * (size_t)i + 2], 0.f);
	const size_t nn = 2 * (size_t)n - 1;
	float4 *pos_dev = nullptr, *dir_dev = nullptr, *kpos = nullptr, *kdir = nullptr;
	float *colb = nullptr, *kcolb = nullptr;
	uint4 *nodes_dev = nullptr;
	hipStream_t st = nullptr;
	hipEvent_t e0 = nullptr, e1 = nullptr;
	void *scratch = nullptr;
	bool ok = hipStreamCreate(&st) == hipSuccess && hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess &&
	          hipMalloc(&pos_dev, (size_t)n * 16) == hipSuccess && hipMalloc(&dir_dev, (size_t)n * 16) == hipSuccess &&
	          hipMalloc(&colb, (size_t)n * 4) == hipSuccess && hipMalloc(&kpos, (size_t)n * 16) == hipSuccess &&
	          hipMalloc(&kdir, (size_t)n * 16) == hipSuccess && hipMalloc(&kcolb, (size_t)n * 4) == hipSuccess &&
	          hipMalloc(&nodes_dev, nn * 16) == hipSuccess && hipMemcpyAsync(pos_dev, pos.data(), (size_t)n * 16, hipMemcpyHostToDevice, st) == hipSuccess &&
	          hipMemsetAsync(dir_dev, 0, (size_t)n * 16, st) == hipSuccess && hipMemsetAsync(colb, 0, (size_t)n * 4, st) == hipSuccess;
	for(int pass = 0; pass < 2 && ok; ++pass)
	{
		ok = hipMemsetAsync(nodes_dev, 0, nn * 16, st) == hipSuccess && hipMemsetAsync(kpos, 0, (size_t)n * 16, st) == hipSuccess &&
		     hipEventRecord(e0, st) == hipSuccess &&
		     yafamd_build_pkd_kd_member(pos_dev, dir_dev, colb, (uint32_t)n, nodes_dev, kpos, kdir, kcolb, depth, st, &scratch, member, members,
		                                split_level) == hipSuccess &&
		     hipEventRecord(e1, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
	}
	float t = 0.f;
	ok = ok && hipEventElapsedTime(&t, e0, e1) == hipSuccess && hipMemcpy(nodes, nodes_dev, nn * 16, hipMemcpyDeviceToHost) == hipSuccess &&
	     hipMemcpy(kd_pos, kpos, (size_t)n * 16, hipMemcpyDeviceToHost) == hipSuccess;
	if(ms) *ms = t;
	if(scratch) yafamd_pkd_scratch_free(scratch);
	for(void *p : {(void *)pos_dev, (void *)dir_dev, (void *)colb, (void *)kpos, (void *)kdir, (void *)kcolb, (void *)nodes_dev})
		if(p) (void)hipFree(p);
	if(e0) (void)hipEventDestroy(e0);
	if(e1) (void)hipEventDestroy(e1);
	if(st) (void)hipStreamDestroy(st);
	return ok ? YAFARAY_BOOL_TRUE : YAFARAY_BOOL_FALSE;
}

// (1.6) the level-D subtrees of a tree over n photons (node, start, end each: 3 << level values) and the
// ones member r of `members` owns ([s0, s1))
void yafaray_amd_photonTreeSegments(unsigned int n, int level, int member, int members, unsigned int *segments, unsigned int *s0, unsigned int *s1)
{
	if(segments) yafamd_pkd_top_segments(n, level, segments);
	if(s0 && s1 && members >= 1) yafamd_pkd_owned_segments(level, member, members, s0, s1);
}

int yafaray_amd_packBand(const float *film, int width, int height, int channels, const int *bounds, int world, int rank, float *send)
{
	if(!bounds || world < 1) return 0;
	return bandPack(film, width, height, channels, std::vector<int>(bounds, bounds + world + 1), rank, send) ? 1 : 0;
}

int yafaray_amd_unpackBands(const float *recv, int width, int height, int channels, const int *bounds, int world, int rank, float *film)
{
	if(!bounds || world < 1) return 0;
	return bandUnpack(recv, width, height, channels, std::vector<int>(bounds, bounds + world + 1), rank, film) ? 1 : 0;
}

int yafaray_amd_getKernelTimes(const yafaray_Interface_t *interface, const char **names, double *ms, uint64_t *launches, uint64_t *items,
                               int max)
{
	const Interface *it = I(interface);
	if(!it->scene) return 0;
	const KernelTimes &kt = it->scene->kernelTimes();
	for(int k = 0; k < KK_COUNT && k < max; ++k)
	{
		if(names) names[k] = kernelKindName(k);
		if(ms) ms[k] = kt.ms[k];
		if(launches) launches[k] = kt.launches[k];
		if(items) items[k] = kt.items[k];
	}
	return KK_COUNT;
}

int yafaray_amd_getPhaseCycles(unsigned long long *cycles, int n, yafaray_bool_t reset)
{
	return yafamd_phase_cycles(cycles, n, reset != YAFARAY_BOOL_FALSE ? 1 : 0);
}

}
