// Every member of the reference's IG::Device (src/runtime/device/Device.h:49-73)
// called through the header-only facade host/Device.h (tests/test_inmem.py
// compiles it with g++ against libigx.so and runs it on the GPU):
//   * the accessors target / framebufferWidth / framebufferHeight / isInteractive;
//   * tonemap and imageinfo (host restatements of entrypoints/tonemap.art and
//     entrypoints/imageinfo.art over getFramebufferForHost), checked against a
//     direct computation from the film;
//   * evaluateGlare and bake: explicit stubs (empty result, output untouched);
//   * getFramebufferForHost / ForDevice: an unknown AOV name gives {nullptr, 0}
//     (Device.cpp:1330-1388), any other failure throws -- here a failed
//     asynchronous render (option fail_chunk), which must not come back as a
//     null pointer;
//   * a failed shading capture throws std::runtime_error, which the reference's
//     Runtime::loadFromFile turns into `false` (Runtime.cpp:159-162), where the
//     round-5 binding aborted.
// Prints "ok" when every check passed.
#include "Device.h"
#include "igx_scene.h"
#include "scene_database.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

static int bad = 0;
#define CHECK(c, ...)                         \
    do {                                      \
        if (!(c)) {                           \
            std::printf("FAIL: " __VA_ARGS__); \
            std::printf("\n");                \
            ++bad;                            \
        }                                     \
    } while (0)

template <typename F>
static bool throws(F f) {
    try {
        f();
    } catch (const std::runtime_error&) {
        return true;
    }
    return false;
}

// a lit plane: diffuse ground, point light (create_flat_scene + "point")
static igx_objscene* lit_plane() {
    igx_objscene* s = igx_objscene_create(nullptr);
    auto num = [&](int o, const char* k, float v) { igx_objscene_set_property(s, o, k, IGX_PROP_NUMBER, &v, 1); };
    auto vec3 = [&](int o, const char* k, float x, float y, float z) {
        const float v[3] = {x, y, z};
        igx_objscene_set_property(s, o, k, IGX_PROP_VECTOR3, v, 3);
    };
    auto str = [&](int o, const char* k, const char* v) { igx_objscene_set_property(s, o, k, IGX_PROP_STRING, v, 1); };
    int t = igx_objscene_add(s, IGX_OBJ_TECHNIQUE, "path", nullptr, nullptr);
    const int32_t depth = 3;
    igx_objscene_set_property(s, t, "max_depth", IGX_PROP_INTEGER, &depth, 1);
    int c = igx_objscene_add(s, IGX_OBJ_CAMERA, "perspective", nullptr, nullptr);
    num(c, "fov", 90);
    const float xf[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, -1, 0, 0, 0, 1};
    igx_objscene_set_property(s, c, "transform", IGX_PROP_TRANSFORM, xf, 16);
    int f = igx_objscene_add(s, IGX_OBJ_FILM, "image", nullptr, nullptr);
    const float size[2] = {96, 64};
    igx_objscene_set_property(s, f, "size", IGX_PROP_VECTOR2, size, 2);
    int b = igx_objscene_add(s, IGX_OBJ_BSDF, "diffuse", "ground", nullptr);
    vec3(b, "reflectance", 0.8f, 0.5f, 0.3f);
    int sh = igx_objscene_add(s, IGX_OBJ_SHAPE, "rectangle", "Bottom", nullptr);
    num(sh, "width", 2);
    num(sh, "height", 2);
    const int32_t yes = 1;
    igx_objscene_set_property(s, sh, "flip_normals", IGX_PROP_BOOL, &yes, 1);
    int e = igx_objscene_add(s, IGX_OBJ_ENTITY, "", "Bottom", nullptr);
    str(e, "shape", "Bottom");
    str(e, "bsdf", "ground");
    int l = igx_objscene_add(s, IGX_OBJ_LIGHT, "point", "_light", nullptr);
    vec3(l, "position", 0, 0, -2);
    vec3(l, "intensity", 3, 3, 3);
    return s;
}

int main() {
    // ---- a failed capture throws (no abort) --------------------------------
    CHECK(throws([] { (void)IG::capture_shading(nullptr); }), "capture_shading(nullptr) did not throw");
    {
        igx_objscene* os = igx_objscene_create(nullptr);
        int e = igx_objscene_add(os, IGX_OBJ_ENTITY, "", "orphan", nullptr);
        igx_objscene_set_property(os, e, "shape", IGX_PROP_STRING, "missing", 1);
        char err[256] = {0};
        igx_scene* sc = igx_scene_from_objects(os, err, sizeof(err));
        igx_objscene_free(os);
        // the binding's capture throws this message
        CHECK(!sc && err[0], "a scene with an unknown shape was accepted");
        if (sc) igx_scene_free(sc);
    }

    IG::Device::SetupSettings setup;
    setup.IsInteractive = true;
    IG::Device dev(setup);
    CHECK(dev.target().device() == 0 && dev.target().isGPU(), "target");
    CHECK(dev.isInteractive(), "isInteractive");
    CHECK(dev.framebufferWidth() == 0 && dev.framebufferHeight() == 0, "framebuffer size before a render");

    igx_objscene* os = lit_plane();
    char err[512] = {0};
    igx_scene* sc = igx_scene_from_objects(os, err, sizeof(err));
    igx_objscene_free(os);
    if (!sc) {
        std::printf("FAIL: scene: %s\n", err);
        return 1;
    }
    IG::TechniqueVariantShaderSet shaders = IG::capture_shading(sc);
    IG::SceneDatabase db;
    igx_shading_view unused{};
    IG::serialize_scene(*igx_scene_get_desc(sc), db, unused);
    IG::Device::SceneSettings ss;
    ss.database = &db;
    dev.assignScene(ss);
    IG::Device::RenderSettings rs;
    rs.spi = 4;
    rs.width = 96;
    rs.height = 64;
    dev.render(shaders, rs);
    dev.render(shaders, rs);
    CHECK(dev.framebufferWidth() == 96 && dev.framebufferHeight() == 64, "framebuffer size");

    // ---- AOV accessors ------------------------------------------------------
    IG::Device::AOVAccessor fb = dev.getFramebufferForHost("");
    CHECK(fb.Data && fb.IterationCount == 2, "film: %p %zu", (void*)fb.Data, fb.IterationCount);
    std::vector<float> film(fb.Data, fb.Data + 96 * 64 * 3);
    IG::Device::AOVAccessor unk = dev.getFramebufferForHost("Normals");
    CHECK(!unk.Data && unk.IterationCount == 0, "unknown AOV on the host");
    IG::Device::AOVAccessor unkd = dev.getFramebufferForDevice("Normals");
    CHECK(!unkd.Data && unkd.IterationCount == 0, "unknown AOV on the device");
    IG::Device::AOVAccessor mis = dev.getFramebufferForHost("NEE Weights"); // no aov_mis in this technique
    CHECK(!mis.Data, "MIS AOV without aov_mis");
    IG::Device::AOVAccessor dfb = dev.getFramebufferForDevice("Color");
    CHECK(dfb.Data && dfb.IterationCount == 2, "device film");

    // ---- tonemap: method 0 (identity curve), no gamma, against the film ----
    std::vector<uint32_t> px(96 * 64, 0xdeadbeefu);
    IG::TonemapSettings ts{"", 0, false, 1.0f, 1.0f, 0.0f};
    dev.tonemap(px.data(), ts);
    int tm_bad = 0, lit = 0;
    for (size_t i = 0; i < px.size(); ++i) {
        float c[3];
        for (int k = 0; k < 3; ++k) c[k] = film[3 * i + k] / 2.0f;
        // xyY round trip returns the colour up to float rounding: compare bytes within 1
        for (int k = 0; k < 3; ++k) {
            const int want = (int)(std::fmin(std::fmax(c[k], 0.0f), 1.0f) * 255);
            const int got = (int)((px[i] >> (16 - 8 * k)) & 255u);
            if (std::abs(got - want) > 1) ++tm_bad;
        }
        lit += (px[i] & 0xffffffu) != 0;
        if ((px[i] >> 24) != 255u) ++tm_bad;
    }
    CHECK(tm_bad == 0 && lit > 100, "tonemap: %d bad channels, %d lit pixels", tm_bad, lit);
    // Reinhard with gamma: luminance L / (1 + L) < 1 then gamma, so no pixel
    // is flagged (cyan NaN, pink inf, orange negative) and each is opaque
    IG::TonemapSettings tr{"Color", 1, true, 1.0f, 1.0f, 0.0f};
    dev.tonemap(px.data(), tr);
    int flagged = 0;
    for (uint32_t p : px) flagged += (p >> 24) != 255u || p == 0xff00ffffu || p == 0xffff0096u || p == 0xffffff00u;
    CHECK(flagged == 0, "reinhard flagged %d pixels", flagged);

    // ---- imageinfo: min / max / average luminance against the film ---------
    std::vector<int> hr(16), hg(16), hb(16), hl(16);
    IG::ImageInfoSettings is{"", 1.0f, 16, hr.data(), hg.data(), hb.data(), hl.data(), true, true};
    IG::ImageInfoOutput io = dev.imageinfo(is);
    double mn = 1e30, mx = -1e30, sum = 0;
    for (size_t i = 0; i < px.size(); ++i) {
        const double r = film[3 * i] / 2.0, g = film[3 * i + 1] / 2.0, b = film[3 * i + 2] / 2.0;
        const double Y = 0.2126729 * r + 0.7151522 * g + 0.0721750 * b;
        mn = std::fmin(mn, Y);
        mx = std::fmax(mx, Y);
        sum += Y;
    }
    const double avg = sum / (double)px.size();
    CHECK(std::fabs(io.Min - mn) <= 1e-5 * (1 + mx) && std::fabs(io.Max - mx) <= 1e-5 * mx && std::fabs(io.Average - avg) <= 1e-4 * avg,
          "imageinfo min/max/avg %g %g %g vs %g %g %g", io.Min, io.Max, io.Average, mn, mx, avg);
    CHECK(io.SoftMin >= io.Min && io.SoftMax <= io.Max && io.Median >= 0 && io.Median <= io.Max, "imageinfo soft stats");
    CHECK(io.InfCount == 0 && io.NaNCount == 0, "imageinfo error counts");
    long hs = 0;
    for (int v : hl) hs += v;
    CHECK(hs == (long)px.size(), "luminance histogram holds %ld of %zu pixels", hs, px.size());

    // ---- the stubs ----------------------------------------------------------
    IG::GlareOutput go = dev.evaluateGlare(px.data(), IG::GlareSettings{"", 1, 0, 0, 0, 0});
    CHECK(go.DGP == 0 && go.NumPixels == 0, "glare stub");
    float baked[4] = {1, 2, 3, 4};
    dev.bake(IG::ShaderOutput<void*>{}, nullptr, baked);
    CHECK(baked[0] == 1 && baked[3] == 4, "bake stub wrote its output");

    // ---- statistics, resize, clear ------------------------------------------
    const IG::Statistics* st = dev.getStatistics();
    CHECK(st && st->cameraRayCount() == 2ull * 96 * 64 * 4, "camera rays %llu", (unsigned long long)(st ? st->cameraRayCount() : 0));

    // ---- a failed asynchronous render throws from the accessors -------------
    igx_set_option(dev.handle(), "capacity", 4096);
    igx_set_option(dev.handle(), "fail_chunk", 2);
    bool render_threw = throws([&] { dev.render(shaders, rs); });
    bool host_threw = throws([&] { (void)dev.getFramebufferForHost(""); });
    bool dev_threw = throws([&] { (void)dev.getFramebufferForDevice(""); });
    CHECK(!render_threw || host_threw, "render threw but the host accessor did not");
    CHECK(host_threw, "getFramebufferForHost returned after a failed render");
    CHECK(dev_threw, "getFramebufferForDevice returned after a failed render");
    dev.clearAllFramebuffer(); // lifts the failure (igx_clear)
    igx_set_option(dev.handle(), "capacity", 0);
    dev.render(shaders, rs);
    IG::Device::AOVAccessor again = dev.getFramebufferForHost("");
    CHECK(again.Data && again.IterationCount == 1, "render after the failure");

    dev.resize(48, 32);
    CHECK(dev.framebufferWidth() == 48 && dev.framebufferHeight() == 32, "resize");
    dev.releaseAll();
    igx_scene_free(sc);
    std::printf(bad ? "failed\n" : "ok\n");
    return bad ? 1 : 0;
}
