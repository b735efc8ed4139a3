// IG::Device facade over the igx_* C-ABI (include/igx.h).
//
// Mirrors the reference plugin surface `IG::Device` (src/runtime/device/Device.h:14-74)
// for the path this build covers: construction from SetupSettings, assignScene,
// render one iteration, framebuffer access, clear, resize, statistics.  The
// reference's tonemap/glare/imageinfo/bake entry points (Device.h:52-62) are
// outside the hot path and are not provided.  Errors from the C-ABI become
// std::runtime_error, which a Runtime turns into its bool/IG_LOG path
// (Runtime.cpp:159-162).
#pragma once

#include "igx.h"

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace IG {

struct SetupSettings {      // Device.h:18-23 (Target reduced to a HIP ordinal)
    int Device = 0;
    bool AcquireStats = false;
    bool DebugTrace = false;
    bool IsInteractive = false;
};

struct SceneSettings {      // Device.h:25-30 (SceneDatabase -> igx_scene_desc)
    const igx_scene_desc* Database = nullptr;
};

struct RenderSettings {     // Device.h:32-42
    const float* rays = nullptr;   // ray-list mode (igtrace), 8 floats per ray
    size_t ray_count = 0;
    size_t spi = 8;
    size_t width = 0, height = 0;
    size_t iteration = 0;
    size_t frame = 0;
    int user_seed = 0;
    int tile_size = 0, tile_offset = 0, tile_stride = 1;
};

struct AOVAccessor {        // Device.h:44-47
    const float* Data;
    size_t IterationCount;
};

class Device {
public:
    explicit Device(const SetupSettings& settings) : mSettings(settings) {
        if (igx_create(settings.Device, &mDev) != IGX_OK || !mDev)
            throw std::runtime_error("igx_create failed for HIP device " + std::to_string(settings.Device));
        if (settings.AcquireStats) check(igx_set_option(mDev, "timing", 1));
    }
    ~Device() {
        if (mDev) igx_destroy(mDev);
    }
    Device(const Device&) = delete;
    Device& operator=(const Device&) = delete;

    void assignScene(const SceneSettings& settings) { check(igx_upload_scene(mDev, settings.Database)); }

    void render(const RenderSettings& s) {
        igx_render_params p{};
        p.width = (int)s.width;
        p.height = (int)s.height;
        p.spi = (int)s.spi;
        p.iteration = (int)s.iteration;
        p.frame = (int)s.frame;
        p.seed = s.user_seed;
        p.tile_size = s.tile_size;
        p.tile_offset = s.tile_offset;
        p.tile_stride = s.tile_stride;
        p.num_rays = (int)s.ray_count;
        p.rays = s.rays;
        check(igx_render(mDev, &p));
        mWidth = s.ray_count ? s.ray_count : s.width;
        mHeight = s.ray_count ? 1 : s.height;
    }

    AOVAccessor getFramebufferForHost(const std::string& name = "") {
        if (!name.empty()) return AOVAccessor{nullptr, 0}; // only the colour framebuffer exists (Device.cpp:1303-1305)
        mHostFB.resize(mWidth * mHeight * 3);
        uint64_t iters = 0;
        check(igx_get_framebuffer(mDev, mHostFB.data(), mHostFB.size(), &iters));
        return AOVAccessor{mHostFB.data(), (size_t)iters};
    }

    void clearFramebuffer() { check(igx_clear(mDev)); }

    // render() only queues work; wait for it (timing, device-side reads)
    void synchronize() { check(igx_synchronize(mDev)); }

    igx_stats getStatistics() {
        igx_stats s{};
        check(igx_get_stats(mDev, &s));
        return s;
    }

    igx_device* handle() { return mDev; }

private:
    void check(igx_status s) {
        if (s != IGX_OK) throw std::runtime_error(std::string("igx: ") + igx_last_error(mDev));
    }
    SetupSettings mSettings;
    igx_device* mDev = nullptr;
    size_t mWidth = 0, mHeight = 0;
    std::vector<float> mHostFB;
};

} // namespace IG
