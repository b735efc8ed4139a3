// igcli-style frontend over the HIP device (src/frontend/cli/main.cpp:54-179):
// loads a scene, renders spp samples in iterations of spi on one GPU, prints
// Msamples/s like the reference (cli/main.cpp:135, 172-178) plus Mrays/s, and
// writes the averaged image as EXR (Image::save, Image.h:92-101), or PFM when
// the output name ends in .pfm.  The scene reaches the device as the
// reference's does: the loader's tables (SceneDatabase, serialize_scene) go
// through IG::Device::assignScene, the shading tables through render's shader
// set (Runtime.cpp:477-485, 343).
#include "Device.h"
#include "igx_scene.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static void usage() {
    std::fprintf(stderr,
                 "usage: igcli SCENE.json [--spp N] [--spi N] [--seed N] [--gpu-device N] [-o out.exr|out.pfm]\n");
}

int main(int argc, char** argv) {
    std::string scene_path, out_path;
    int spp = 0, spi = 8, seed = 0, device = 0;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { usage(); std::exit(2); }
            return argv[++i];
        };
        if (a == "--spp") spp = std::atoi(next());
        else if (a == "--spi") spi = std::atoi(next());
        else if (a == "--seed") seed = std::atoi(next());
        else if (a == "--gpu-device") device = std::atoi(next());
        else if (a == "-o" || a == "--output") out_path = next();
        else if (a == "--gpu") {}
        else if (a == "-h" || a == "--help") { usage(); return 0; }
        else if (!a.empty() && a[0] == '-') { usage(); return 2; }
        else scene_path = a;
    }
    if (scene_path.empty()) { usage(); return 2; }
    char err[1024] = {0};
    igx_scene* scene = igx_scene_load_file(scene_path.c_str(), err, sizeof(err));
    if (!scene) { std::fprintf(stderr, "failed to load scene: %s\n", err); return 1; }
    const igx_scene_desc* desc = igx_scene_get_desc(scene);
    if (spp <= 0) spp = spi;
    int iters = (spp + spi - 1) / spi; // igcli rounds spp up to a multiple of spi (cli/main.cpp:110-113)
    try {
        IG::SceneDatabase db;
        IG::TechniqueVariantShaderSet shaders;
        IG::serialize_scene(*desc, db, shaders.shading);
        IG::Device::SetupSettings ss;
        ss.target = IG::Target::makeGPU(device);
        IG::Device dev(ss);
        IG::Device::SceneSettings sc;
        sc.database = &db;
        dev.assignScene(sc);
        std::vector<double> rates;
        double total_s = 0; // wall time of the render loop (cli/main.cpp:127-135)
        for (int it = 0; it < iters; ++it) {
            IG::Device::RenderSettings rs;
            rs.spi = spi;
            rs.width = desc->film_width;
            rs.height = desc->film_height;
            rs.iteration = it;
            rs.user_seed = seed;
            auto t0 = std::chrono::steady_clock::now();
            dev.render(shaders, rs, nullptr);
            dev.synchronize(); // render() only queues the iteration
            double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            rates.push_back((double)spi * desc->film_width * desc->film_height / s / 1e6);
            total_s += s;
        }
        const igx_stats& st = dev.getStatistics()->raw();
        std::sort(rates.begin(), rates.end());
        double rays = (double)(st.camera_rays + st.bounce_rays + st.shadow_rays);
        std::printf("# %f %f %f Msamples/s\n", rates.front(), rates[rates.size() / 2], rates.back());
        std::printf("# %.3f Mrays/s (camera %llu, bounce %llu, shadow %llu) over %.3f ms\n", rays / total_s / 1e6,
                    (unsigned long long)st.camera_rays, (unsigned long long)st.bounce_rays, (unsigned long long)st.shadow_rays,
                    total_s * 1e3);
        if (!out_path.empty()) {
            IG::Device::AOVAccessor acc = dev.getFramebufferForHost("");
            float inv = acc.IterationCount ? 1.0f / acc.IterationCount : 0.0f;
            const bool pfm = out_path.size() >= 4 && out_path.compare(out_path.size() - 4, 4, ".pfm") == 0;
            if (!pfm) {
                if (igx_write_exr(out_path.c_str(), acc.Data, desc->film_width, desc->film_height, 3, inv) != 0) {
                    std::fprintf(stderr, "cannot write %s\n", out_path.c_str());
                    return 1;
                }
            } else {
                FILE* f = std::fopen(out_path.c_str(), "wb");
                if (!f) { std::fprintf(stderr, "cannot write %s\n", out_path.c_str()); return 1; }
                std::fprintf(f, "PF\n%d %d\n-1.0\n", desc->film_width, desc->film_height);
                for (int y = desc->film_height - 1; y >= 0; --y) { // PFM rows go bottom-up
                    std::vector<float> row(3 * desc->film_width);
                    for (int x = 0; x < 3 * desc->film_width; ++x) row[x] = acc.Data[(size_t)y * 3 * desc->film_width + x] * inv;
                    std::fwrite(row.data(), sizeof(float), row.size(), f);
                }
                std::fclose(f);
            }
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        igx_scene_free(scene);
        return 1;
    }
    igx_scene_free(scene);
    return 0;
}
