// IG::Device over the igx_* C-ABI (include/igx.h, include/igx_scene.h).
//
// Same class, nested settings structs and member functions as the reference
// plugin surface `IG::Device` (src/runtime/device/Device.h:14-74), so a runtime
// written against it compiles against this header:
//   * assignScene takes the reference's SceneSettings with a SceneDatabase*
//     (table types in scene_database.h, same members as table/*.h); the tables
//     reach the device through igx_scene_from_database;
//   * render takes the TechniqueVariantShaderSet.  In the reference that is the
//     technique variant's compiled shader code; igx has no shader JIT, so here
//     the "shader set" is the shading tables the shaders were generated from
//     (materials, lights, camera, technique: igx_shading_view).  The scene is
//     uploaded on the first render after assignScene and whenever the shading
//     tables' contents change (materials, lights, technique, film; a copy of
//     the last uploaded ones is compared, so a set edited in place or a new
//     set at a freed one's address is seen), as the reference compiles and
//     loads its shaders lazily.  A camera change alone does not re-upload: it
//     reaches the device through igx_set_camera;
//   * render's ParameterSet (RuntimeStructs.h:56-70) carries the runtime's
//     camera orientation (__camera_eye / __camera_dir / __camera_up,
//     Runtime::setCameraOrientationParameter, Runtime.cpp:700-705), which
//     overrides the shading view's camera; its other parameters drive the
//     reference's shading networks, which igx does not have, and are ignored;
//   * capture_shading builds the shader set of an in-memory scene
//     (igx_objscene_*, the `const Scene*` of Runtime::loadFromScene) without a
//     file;
//   * the framebuffer, statistics, resize and release calls map one to one.
// tonemap / evaluateGlare / imageinfo / bake (Device.h:66-69) are outside the
// hot path ("stub or CPU fallback"): tonemap and imageinfo run
// on the host over getFramebufferForHost (restating entrypoints/tonemap.art and
// entrypoints/imageinfo.art with core/color.art); evaluateGlare and bake have
// no igx counterpart (the glare shader needs the camera's solid-angle model,
// bake a compiled shading-tree shader) and log and return an empty result.
// Errors from the C-ABI become std::runtime_error, which a Runtime turns into
// its bool / IG_LOG path (Runtime.cpp:159-162); an unknown AOV name alone gives
// the reference's empty accessor {nullptr, 0}.
#pragma once

#include "film_tools.h"
#include "igx.h"
#include "scene_database.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace IG {

// Target.h:19-68 reduced to what the device uses: a HIP ordinal
class Target {
public:
    static Target makeGPU(int device = 0) { return Target(device); }
    int device() const { return mDevice; }
    bool isGPU() const { return true; }

private:
    explicit Target(int d) : mDevice(d) {}
    int mDevice = 0;
};

struct Ray { // RuntimeStructs.h: org, dir, range (tmin, tmax)
    float org[3];
    float dir[3];
    float range[2];
};
static_assert(sizeof(Ray) == 8 * sizeof(float), "ray-list layout of igx_render_params::rays");

struct TechniqueVariantShaderSet {
    igx_shading_view shading{};
};
struct TechniqueVariantInfo {};
using Vector3f = std::array<float, 3>;
using Vector4f = std::array<float, 4>;
struct ParameterSet { // RuntimeStructs.h:56-70
    std::unordered_map<std::string, int> IntParameters;
    std::unordered_map<std::string, float> FloatParameters;
    std::unordered_map<std::string, Vector3f> VectorParameters;
    std::unordered_map<std::string, Vector4f> ColorParameters;
    bool empty() const { return IntParameters.empty() && FloatParameters.empty() && VectorParameters.empty() && ColorParameters.empty(); }
};

// RuntimeStructs.h:6-54 (the reference's utility-shader settings and outputs)
struct TonemapSettings {
    const char* AOV;
    size_t Method;
    bool UseGamma;
    float Scale;
    float ExposureFactor;
    float ExposureOffset;
};
struct GlareSettings {
    const char* AOV;
    float Scale;
    float LuminanceMax;
    float LuminanceAverage;
    float LuminanceMultiplier;
    float VerticalIlluminance;
};
struct GlareOutput {
    float DGP;
    float VerticalIlluminance;
    int NumPixels;
    float AvgLum;
    float AvgOmega;
};
struct ImageInfoSettings {
    const char* AOV;
    float Scale;
    size_t Bins;
    int* HistogramR;
    int* HistogramG;
    int* HistogramB;
    int* HistogramL;
    bool AcquireErrorStats;
    bool AcquireHistogram;
};
struct ImageInfoOutput {
    float Min;
    float Max;
    float Average;
    float SoftMin;
    float SoftMax;
    float Median;
    int InfCount;
    int NaNCount;
    int NegCount;
};
// shader/ShaderUtils.h: a compiled shader and its local registry; igx has no
// shader JIT, so a bake request carries nothing it could run
template <typename T>
struct ShaderOutput {
    T Exec = nullptr;
};


// The shader set of a scene igx loaded itself (igx_scene_load_* or, for the
// reference's in-memory scenes, igx_scene_from_objects): its film, camera,
// technique, materials and lights.  The views point into `scene`, which must
// outlive the shader set.
inline TechniqueVariantShaderSet capture_shading(const igx_scene* scene) {
    const igx_scene_desc* d = igx_scene_get_desc(scene);
    if (!d) throw std::runtime_error("igx: capture_shading without a scene");
    TechniqueVariantShaderSet s;
    s.shading.film_width = d->film_width;
    s.shading.film_height = d->film_height;
    s.shading.camera = d->camera;
    s.shading.technique = d->technique;
    s.shading.num_materials = d->num_materials;
    s.shading.materials = d->materials;
    s.shading.num_lights = d->num_lights;
    s.shading.lights = d->lights;
    return s;
}

// Statistics.h quantities the device fills (CameraRayCount, BounceRayCount,
// ShadowRayCount; shadow rays counted when valid)
class Statistics {
public:
    uint64_t cameraRayCount() const { return mStats.camera_rays; }
    uint64_t bounceRayCount() const { return mStats.bounce_rays; }
    uint64_t shadowRayCount() const { return mStats.shadow_rays; }
    const igx_stats& raw() const { return mStats; }
    // Statistics::dump (Statistics.cpp:151-290): kernel times (with the
    // device's "timing" option, SetupSettings::AcquireStats) in place of the
    // reference's per-shader timers, then the ray quantities; PrimaryRays =
    // camera + bounce, TotalRays = camera + bounce + shadow (:286-290)
    std::string dump(size_t totalMS, size_t iter) const {
        std::string out = "Statistics:\n  Kernels (summed HIP-event time, ms):\n";
        auto row = [&](const char* name, double ms, uint64_t launches) {
            char b[160];
            std::snprintf(b, sizeof(b), "  |-%-14s %10.3f [%llu]%s", name, ms, (unsigned long long)launches,
                          iter ? "" : "\n");
            out += b;
            if (iter) {
                std::snprintf(b, sizeof(b), "  %10.3f per Iteration\n", ms / (double)iter);
                out += b;
            }
        };
        row("Extend", mStats.ms_extend, mStats.launches_extend);
        row("Trace", mStats.ms_trace, mStats.launches_trace);
        row("Shadow", mStats.ms_shadow, mStats.launches_shadow);
        row("Finish", mStats.ms_finish, mStats.launches_finish);
        row("Generate", mStats.ms_generate, 0);
        row("Resolve", mStats.ms_resolve, 0);
        out += "  Quantities:\n";
        auto qty = [&](const char* name, uint64_t count) {
            char b[160];
            std::snprintf(b, sizeof(b), "  |-%-12s %llu per ms [%llu]\n", name,
                          (unsigned long long)(count / (totalMS ? totalMS : 1)), (unsigned long long)count);
            out += b;
        };
        qty("CameraRays", mStats.camera_rays);
        qty("ShadowRays", mStats.shadow_rays);
        qty("BounceRays", mStats.bounce_rays);
        qty("PrimaryRays", mStats.camera_rays + mStats.bounce_rays);
        qty("TotalRays", mStats.camera_rays + mStats.bounce_rays + mStats.shadow_rays);
        return out;
    }
    igx_stats mStats{};
};

class Device {
public:
    struct SetupSettings { // Device.h:18-23
        Target target = Target::makeGPU(0);
        bool AcquireStats = false;
        bool DebugTrace = false;
        bool IsInteractive = false;
    };

    struct SceneSettings { // Device.h:25-30
        SceneDatabase* database = nullptr;
        const std::vector<std::string>* aov_map = nullptr;
        const std::vector<std::string>* resource_map = nullptr;
        const std::vector<int32_t>* entity_per_material = nullptr;
    };

    struct RenderSettings { // Device.h:32-42
        const Ray* rays = nullptr; // non-null: width = number of rays, height = 1
        size_t spi = 8;
        size_t width = 0;
        size_t height = 0;
        size_t iteration = 0;
        size_t frame = 0;
        size_t user_seed = 0;
        TechniqueVariantInfo info;
        bool denoise = false;
        // igx: tile sharding over ranks; 0 = whole film
        int tile_size = 0, tile_offset = 0, tile_stride = 1;
    };

    struct AOVAccessor { // Device.h:44-47
        float* Data;
        size_t IterationCount;
    };

    explicit Device(const SetupSettings& settings) : mSettings(settings) {
        if (igx_create(settings.target.device(), &mDev) != IGX_OK || !mDev)
            throw std::runtime_error("igx_create failed for HIP device " + std::to_string(settings.target.device()));
        if (settings.AcquireStats) check(igx_set_option(mDev, "timing", 1));
    }
    ~Device() {
        releaseAll();
        if (mDev) igx_destroy(mDev);
    }
    Device(const Device&) = delete;
    Device& operator=(const Device&) = delete;

    void assignScene(const SceneSettings& settings) {
        if (!settings.database) throw std::runtime_error("igx: assignScene without a SceneDatabase");
        mScene = settings;
        releaseAll(); // upload at the next render
    }

    void render(const TechniqueVariantShaderSet& shader_set, const RenderSettings& s, const ParameterSet* params = nullptr) {
        if (!mScene.database) throw std::runtime_error("igx: render before assignScene");
        if (!mUploaded || !mLast.same(shader_set.shading)) upload(shader_set);
        igx_camera cam = shader_set.shading.camera;
        if (params) { // the runtime's camera orientation (Runtime.cpp:700-705)
            auto put = [&](const char* key, float* dst) {
                auto it = params->VectorParameters.find(key);
                if (it != params->VectorParameters.end()) std::memcpy(dst, it->second.data(), 3 * sizeof(float));
            };
            put("__camera_eye", cam.eye);
            put("__camera_dir", cam.dir);
            put("__camera_up", cam.up);
        }
        if (std::memcmp(&cam, &mCamera, sizeof(cam)) != 0) {
            check(igx_set_camera(mDev, &cam));
            mCamera = cam;
        }
        igx_render_params p{};
        p.spi = (int)s.spi;
        p.iteration = (int)s.iteration;
        p.frame = (int)s.frame;
        p.seed = (int)s.user_seed;
        if (s.rays) { // ray-list mode (Runtime::trace, Runtime.cpp:385-407)
            p.num_rays = (int)s.width;
            p.rays = reinterpret_cast<const float*>(s.rays);
        } else {
            p.width = (int)s.width;
            p.height = (int)s.height;
            p.tile_size = s.tile_size;
            p.tile_offset = s.tile_offset;
            p.tile_stride = s.tile_stride;
        }
        check(igx_render(mDev, &p));
        mWidth = s.width;
        mHeight = s.rays ? 1 : s.height;
    }

    void resize(size_t width, size_t height) {
        mWidth = width;
        mHeight = height;
        check(igx_clear(mDev));
    }

    void releaseAll() {
        if (mUploaded) igx_scene_free(mUploaded);
        mUploaded = nullptr;
        mLast = ShadingCopy{};
    }

    Target target() const { return mSettings.target; }
    size_t framebufferWidth() const { return mWidth; }
    size_t framebufferHeight() const { return mHeight; }
    bool isInteractive() const { return mSettings.IsInteractive; }

    // the film ("" / "Color") or a named AOV of the technique ("Direct Weights",
    // "NEE Weights" with aov_mis); an unknown name gives {nullptr, 0}, as the
    // reference's getAOVImageForHost / ForDevice (Device.cpp:1330-1388).  Every
    // other failure (a HIP error, a failed asynchronous render) throws: the
    // name is resolved first (igx_aov_device_ptr needs no GPU work), so only
    // IGX_ERR_INVALID_ARGUMENT on an unknown name maps to the empty accessor
    AOVAccessor getFramebufferForHost(const std::string& name = "") {
        if (!knownAOV(name)) return AOVAccessor{nullptr, 0};
        std::vector<float>& buf = mHostFB[name.empty() ? "Color" : name];
        buf.resize(mWidth * mHeight * 3);
        uint64_t iters = 0;
        check(igx_get_aov(mDev, name.c_str(), buf.data(), buf.size(), &iters));
        return AOVAccessor{buf.data(), (size_t)iters};
    }
    AOVAccessor getFramebufferForDevice(const std::string& name = "") {
        if (!knownAOV(name)) return AOVAccessor{nullptr, 0};
        float* ptr = nullptr;
        size_t n = 0;
        uint64_t iters = 0;
        check(igx_synchronize(mDev));
        check(igx_aov_device_ptr(mDev, name.c_str(), &ptr, &n));
        check(igx_get_framebuffer(mDev, nullptr, 0, &iters));
        return AOVAccessor{ptr, (size_t)iters};
    }
    void clearFramebuffer(const std::string& = "") { check(igx_clear(mDev)); }
    void clearAllFramebuffer() { check(igx_clear(mDev)); }

    const Statistics* getStatistics() {
        check(igx_get_stats(mDev, &mStats.mStats));
        return &mStats;
    }

    // entrypoints/tonemap.art on the host over the AOV's host copy (film_tools.h)
    void tonemap(uint32_t* out_pixels, const TonemapSettings& ts) {
        const AOVAccessor acc = getFramebufferForHost(ts.AOV ? ts.AOV : "");
        if (!acc.Data || !out_pixels) return;
        const float inv_iter = acc.IterationCount > 0 ? 1.0f / (float)acc.IterationCount : 0.0f;
        igx::tonemap_film(acc.Data, mWidth * mHeight, ts.Scale * inv_iter, (int)ts.Method, ts.UseGamma, ts.ExposureFactor,
                          ts.ExposureOffset, out_pixels);
    }
    // The glare shader (Device.cpp:1689-1723) evaluates the daylight glare
    // probability over the camera's solid-angle model; igx has none: logged, empty
    GlareOutput evaluateGlare(uint32_t*, const GlareSettings&) {
        std::fprintf(stderr, "igx: evaluateGlare is not provided by the igx device (outside the traced path)\n");
        return GlareOutput{0, 0, 0, 0, 0};
    }
    // entrypoints/imageinfo.art on the host over the AOV's host copy (film_tools.h)
    ImageInfoOutput imageinfo(const ImageInfoSettings& is) {
        const AOVAccessor acc = getFramebufferForHost(is.AOV ? is.AOV : "");
        if (!acc.Data) return ImageInfoOutput{0, 0, 0, 0, 0, 0, 0, 0, 0};
        const float inv_iter = acc.IterationCount > 0 ? 1.0f / (float)acc.IterationCount : 0.0f;
        const igx::FilmInfo f = igx::imageinfo_film(acc.Data, mWidth, mHeight, is.Scale * inv_iter, is.Bins, is.HistogramR, is.HistogramG,
                                                    is.HistogramB, is.HistogramL, is.AcquireErrorStats, is.AcquireHistogram);
        return ImageInfoOutput{f.min, f.max, f.avg, f.soft_min, f.soft_max, f.median, f.inf_count, f.nan_count, f.neg_count};
    }
    // Device::bake (Device.cpp:1761-1774) runs a shading-tree shader compiled
    // by the reference's JIT (ShadingTree.cpp:527); igx compiles none: logged,
    // `output` left untouched
    void bake(const ShaderOutput<void*>&, const std::vector<std::string>*, float*) {
        std::fprintf(stderr, "igx: bake is not provided by the igx device (no shading-tree shaders)\n");
    }

    // igx extras: render() only queues work; wait for it (timing, host reads)
    void synchronize() { check(igx_synchronize(mDev)); }
    igx_device* handle() { return mDev; }

private:
    // "" / "Color", and the MIS AOVs when the uploaded technique has them
    bool knownAOV(const std::string& name) const {
        if (name.empty() || name == "Color") return true;
        return mLast.valid && mLast.technique.aov_mis && (name == "Direct Weights" || name == "NEE Weights");
    }
    void check(igx_status s) {
        if (s != IGX_OK) throw std::runtime_error(std::string("igx: ") + igx_last_error(mDev));
    }
    void upload(const TechniqueVariantShaderSet& shader_set) {
        DatabaseViewStorage view(*mScene.database);
        char err[1024] = {0};
        igx_scene* sc = igx_scene_from_database(&view.view, &shader_set.shading, err, sizeof(err));
        if (!sc) throw std::runtime_error(std::string("igx: scene database: ") + err);
        igx_status st = igx_upload_scene(mDev, igx_scene_get_desc(sc));
        releaseAll();
        mUploaded = sc;
        check(st);
        mLast.take(shader_set.shading);
        mCamera = shader_set.shading.camera; // igx_upload_scene set it
    }

    // a copy of the shading tables last uploaded (the camera aside: it does
    // not need an upload), to see in-place edits and reused addresses
    struct ShadingCopy {
        bool valid = false;
        int32_t film_width = 0, film_height = 0;
        igx_technique technique{};
        std::vector<igx_material> materials;
        std::vector<igx_light> lights;
        void take(const igx_shading_view& v) {
            valid = true;
            film_width = v.film_width;
            film_height = v.film_height;
            technique = v.technique;
            materials.assign(v.materials, v.materials + v.num_materials);
            lights.assign(v.lights, v.lights + v.num_lights);
        }
        bool same(const igx_shading_view& v) const {
            return valid && film_width == v.film_width && film_height == v.film_height &&
                   std::memcmp(&technique, &v.technique, sizeof(technique)) == 0 && materials.size() == v.num_materials &&
                   lights.size() == v.num_lights &&
                   (materials.empty() || std::memcmp(materials.data(), v.materials, materials.size() * sizeof(igx_material)) == 0) &&
                   (lights.empty() || std::memcmp(lights.data(), v.lights, lights.size() * sizeof(igx_light)) == 0);
        }
    };

    SetupSettings mSettings;
    SceneSettings mScene;
    igx_device* mDev = nullptr;
    igx_scene* mUploaded = nullptr;
    ShadingCopy mLast;
    igx_camera mCamera{};
    size_t mWidth = 0, mHeight = 0;
    std::unordered_map<std::string, std::vector<float>> mHostFB; // per AOV name
    Statistics mStats;
};

} // namespace IG
