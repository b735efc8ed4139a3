// igtrace-style frontend over the HIP device (src/frontend/trace/main.cpp:16-170):
// reads rays "ox oy oz dx dy dz [tmin [tmax]]" one per line (from a file given
// with --input, else stdin), traces every ray with the scene's path tracer at
// spi 1 for --spp iterations in ray-list mode, and writes the mean radiance
// "r\tg\tb" per ray in scientific notation (to --output or stdout).  As in the
// reference, a missing tmin is 0 and tmax <= tmin means unbounded.
#include "Device.h"
#include "igx_scene.h"

#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <iterator>
#include <sstream>
#include <string>
#include <vector>

static void usage() {
    std::fprintf(stderr, "usage: igtrace SCENE.json [--input RAYS.txt] [--spp N] [--seed N] [--gpu-device N] [-o OUT.txt]\n");
}

static std::vector<float> read_rays(std::istream& is) {
    std::vector<float> rays;
    std::string line;
    while (std::getline(is, line)) {
        if (line.empty()) break;
        std::stringstream ss(line);
        std::vector<float> d{std::istream_iterator<float>(ss), std::istream_iterator<float>()};
        if (d.size() < 6) continue; // ignored, as the reference does
        float tmin = d.size() > 6 ? d[6] : 0.0f;
        float tmax = d.size() > 7 ? d[7] : 0.0f;
        if (tmax <= tmin) tmax = FLT_MAX;
        rays.insert(rays.end(), {d[0], d[1], d[2], d[3], d[4], d[5], tmin, tmax});
    }
    return rays;
}

int main(int argc, char** argv) {
    std::string scene_path, in_path, out_path;
    int spp = 1, seed = 0, device = 0;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { usage(); std::exit(2); }
            return argv[++i];
        };
        if (a == "--spp") spp = std::atoi(next());
        else if (a == "--seed") seed = std::atoi(next());
        else if (a == "--gpu-device") device = std::atoi(next());
        else if (a == "--input") in_path = next();
        else if (a == "-o" || a == "--output") out_path = next();
        else if (a == "-h" || a == "--help") { usage(); return 0; }
        else if (!a.empty() && a[0] == '-') { usage(); return 2; }
        else scene_path = a;
    }
    if (scene_path.empty()) { usage(); return 2; }
    std::vector<float> rays;
    if (in_path.empty()) rays = read_rays(std::cin);
    else {
        std::ifstream f(in_path);
        rays = read_rays(f);
    }
    const size_t n = rays.size() / 8;
    if (n == 0) { std::fprintf(stderr, "No rays given\n"); return 1; }
    char err[1024] = {0};
    igx_scene* scene = igx_scene_load_file(scene_path.c_str(), err, sizeof(err));
    if (!scene) { std::fprintf(stderr, "failed to load scene: %s\n", err); return 1; }
    int rc = 0;
    try {
        IG::SceneDatabase db; // the loader's tables, as Runtime hands them over (Runtime.cpp:477-485)
        IG::TechniqueVariantShaderSet shaders;
        IG::serialize_scene(*igx_scene_get_desc(scene), db, shaders.shading);
        IG::Device::SetupSettings ss;
        ss.target = IG::Target::makeGPU(device);
        IG::Device dev(ss);
        IG::Device::SceneSettings sc;
        sc.database = &db;
        dev.assignScene(sc);
        const int iters = spp < 1 ? 1 : spp; // SPI fixed to 1 (trace/main.cpp:80)
        for (int it = 0; it < iters; ++it) {
            IG::Device::RenderSettings rs; // Runtime::trace (Runtime.cpp:385-407): width = ray count
            rs.rays = reinterpret_cast<const IG::Ray*>(rays.data());
            rs.width = n;
            rs.height = 1;
            rs.spi = 1;
            rs.iteration = it;
            rs.user_seed = seed;
            dev.render(shaders, rs, nullptr);
        }
        IG::Device::AOVAccessor acc = dev.getFramebufferForHost("");
        std::FILE* f = out_path.empty() ? stdout : std::fopen(out_path.c_str(), "w");
        if (!f) throw std::runtime_error("cannot write " + out_path);
        const float inv = acc.IterationCount ? 1.0f / (float)acc.IterationCount : 0.0f;
        for (size_t i = 0; i < n; ++i)
            std::fprintf(f, "%e\t%e\t%e\n", acc.Data[3 * i] * inv, acc.Data[3 * i + 1] * inv, acc.Data[3 * i + 2] * inv);
        if (f != stdout) std::fclose(f);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        rc = 1;
    }
    igx_scene_free(scene);
    return rc;
}
