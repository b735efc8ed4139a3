// GPU check of the in-memory scene path through the reference's binding seam
// (tests/test_inmem.py compiles it with g++ against libigx.so): the
// reference's create_flat_scene (src/tests/integrator/common/__init__.py:37-66)
// plus one light is built object by object with igx_objscene_* -- as a binding
// forwards the `const Scene*` of Runtime::loadFromScene, no file, no JSON --
// captured with IG::capture_shading, written into the reference's tables
// (serialize_scene stands in for the reference loader), handed to the IG::Device
// facade through assignScene, and rendered at 1000^2, spi 8.  Prints one line
// per case: "<case> <mean> <standard error>"; the test compares them with
// tests/golden/analytic_kats.json.  Then checks the facade's upload rules: an
// in-place edit of the shader set's materials re-uploads (the image halves), and
// the ParameterSet camera moves the camera without one.
#include "Device.h"
#include "igx_scene.h"
#include "scene_database.h"

#include <cmath>
#include <cstdio>
#include <cstring>
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

static void num(igx_objscene* s, int o, const char* k, float v) { igx_objscene_set_property(s, o, k, IGX_PROP_NUMBER, &v, 1); }
static void integer(igx_objscene* s, int o, const char* k, int32_t v) { igx_objscene_set_property(s, o, k, IGX_PROP_INTEGER, &v, 1); }
static void vec3(igx_objscene* s, int o, const char* k, float x, float y, float z) {
    const float v[3] = {x, y, z};
    igx_objscene_set_property(s, o, k, IGX_PROP_VECTOR3, v, 3);
}
static void str(igx_objscene* s, int o, const char* k, const char* v) { igx_objscene_set_property(s, o, k, IGX_PROP_STRING, v, 1); }

// create_flat_scene + `light` ("point" at (0, 0, -2) or a constant "env")
static igx_objscene* flat_scene(const std::string& light) {
    igx_objscene* s = igx_objscene_create(nullptr);
    int t = igx_objscene_add(s, IGX_OBJ_TECHNIQUE, "path", nullptr, nullptr);
    integer(s, t, "max_depth", 2);
    int c = igx_objscene_add(s, IGX_OBJ_CAMERA, "perspective", nullptr, nullptr);
    num(s, c, "fov", 90);
    num(s, c, "near_clip", 0.01f);
    num(s, c, "far_clip", 100);
    // the parser's Transformf of [1,0,0,0, 0,1,0,0, 0,0,1,-1], row-major 4x4
    const float xf[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, -1, 0, 0, 0, 1};
    igx_objscene_set_property(s, c, "transform", IGX_PROP_TRANSFORM, xf, 16);
    int f = igx_objscene_add(s, IGX_OBJ_FILM, "image", nullptr, nullptr);
    const float size[2] = {1000, 1000};
    igx_objscene_set_property(s, f, "size", IGX_PROP_VECTOR2, size, 2);
    int b = igx_objscene_add(s, IGX_OBJ_BSDF, "diffuse", "ground", nullptr);
    vec3(s, b, "reflectance", 1, 1, 1);
    int sh = igx_objscene_add(s, IGX_OBJ_SHAPE, "rectangle", "Bottom", nullptr);
    num(s, sh, "width", 2);
    num(s, sh, "height", 2);
    const int32_t yes = 1;
    igx_objscene_set_property(s, sh, "flip_normals", IGX_PROP_BOOL, &yes, 1);
    int e = igx_objscene_add(s, IGX_OBJ_ENTITY, "", "Bottom", nullptr);
    str(s, e, "shape", "Bottom");
    str(s, e, "bsdf", "ground");
    if (light == "point") {
        int l = igx_objscene_add(s, IGX_OBJ_LIGHT, "point", "_light", nullptr);
        vec3(s, l, "position", 0, 0, -2);
        vec3(s, l, "intensity", 1, 1, 1);
    } else if (light == "env") {
        int l = igx_objscene_add(s, IGX_OBJ_LIGHT, "env", "_light", nullptr);
        vec3(s, l, "radiance", 1, 1, 1);
    }
    return s;
}

static void mean_se(IG::Device& dev, double& mean, double& se) {
    auto fb = dev.getFramebufferForHost();
    const size_t n = dev.framebufferWidth() * dev.framebufferHeight();
    double s = 0, s2 = 0;
    for (size_t i = 0; i < n; ++i) {
        const double v = (fb.Data[3 * i] + fb.Data[3 * i + 1] + fb.Data[3 * i + 2]) / 3.0 / (double)fb.IterationCount;
        s += v;
        s2 += v * v;
    }
    mean = s / (double)n;
    se = std::sqrt(std::max(0.0, s2 / (double)n - mean * mean) / (double)n);
}

int main() {
    IG::Device::SetupSettings setup;
    IG::Device dev(setup);
    IG::Device::RenderSettings rs;
    rs.spi = 8;
    rs.width = rs.height = 1000;
    for (const char* light : {"point", "env"}) {
        igx_objscene* os = flat_scene(light);
        char err[1024] = {0};
        igx_scene* sc = igx_scene_from_objects(os, err, sizeof(err));
        igx_objscene_free(os);
        if (!sc) {
            std::printf("FAIL: %s: %s\n", light, err);
            return 1;
        }
        IG::TechniqueVariantShaderSet shaders = IG::capture_shading(sc);
        IG::SceneDatabase db;
        igx_shading_view unused{};
        IG::serialize_scene(*igx_scene_get_desc(sc), db, unused);
        IG::Device::SceneSettings ss;
        ss.database = &db;
        dev.assignScene(ss);
        dev.clearAllFramebuffer();
        dev.render(shaders, rs);
        double m, se;
        mean_se(dev, m, se);
        std::printf("%s %.9g %.9g\n", light, m, se);

        if (std::string(light) == "point") {
            // in-place edit of the shader set's material (same address): must re-upload
            std::vector<igx_material> mats(shaders.shading.materials, shaders.shading.materials + shaders.shading.num_materials);
            shaders.shading.materials = mats.data();
            dev.clearAllFramebuffer();
            dev.render(shaders, rs);
            double m1, se1;
            mean_se(dev, m1, se1);
            for (auto& mt : mats)
                for (float& k : mt.kd) k *= 0.5f;
            dev.clearAllFramebuffer();
            dev.render(shaders, rs);
            double m2, se2;
            mean_se(dev, m2, se2);
            CHECK(std::fabs(m1 - m) <= 1e-7 * std::max(1.0, m), "same contents rendered differently: %g vs %g", m1, m);
            CHECK(std::fabs(m2 - 0.5 * m1) <= 1e-3 * m1, "edited material not uploaded: %g vs %g", m2, 0.5 * m1);
            // the runtime's camera orientation: from z = -1 to z = -3 the 2x2 plane
            // covers a ninth of the 90-degree film, so the mean drops
            IG::ParameterSet ps;
            ps.VectorParameters["__camera_eye"] = {0, 0, -3};
            dev.clearAllFramebuffer();
            dev.render(shaders, rs, &ps);
            double m3, se3;
            mean_se(dev, m3, se3);
            CHECK(m3 < 0.3 * m2 && m3 > 0, "camera parameter not applied: %g vs %g", m3, m2);
            dev.clearAllFramebuffer();
            dev.render(shaders, rs);
            double m4, se4;
            mean_se(dev, m4, se4);
            CHECK(std::fabs(m4 - m2) <= 1e-7 * std::max(1.0, m2), "camera not restored without parameters: %g vs %g", m4, m2);
        }
        dev.releaseAll();
        igx_scene_free(sc);
    }
    std::printf(bad ? "failed\n" : "ok\n");
    return bad ? 1 : 0;
}
