// igcli-style frontend over the HIP device (src/frontend/cli/main.cpp:54-179):
// loads a scene, renders spp samples in iterations of spi on one GPU (or
// iterations until --time seconds of rendering, main.cpp:138), prints
// Msamples/s like the reference (cli/main.cpp:135, 172-178) plus Mrays/s, and
// writes the averaged image as EXR (Image::save, Image.h:92-101), or PFM when
// the output name ends in .pfm.  The scene reaches the device as the
// reference's does: the loader's tables (SceneDatabase, serialize_scene) go
// through IG::Device::assignScene, the shading tables through render's shader
// set (Runtime.cpp:477-485, 343).  --eye / --dir / --up override the scene
// camera's orientation the way Runtime::setCameraOrientationParameter does
// (main.cpp:103-107, Runtime.cpp:703-708): as the __camera_* vector
// parameters of render's ParameterSet.  --width / --height override the film
// (ProgramOptions.cpp:135-139).  --stats prints Statistics::dump's quantities
// (main.cpp:155-166).  Options of the reference's other targets and of its
// shader compiler are refused with a message.
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
                 "usage: igcli SCENE.json [--spp N | --time SECONDS] [--spi N] [--seed N] [--gpu] [--gpu-device N]\n"
                 "             [--width W --height H] [--eye X Y Z] [--dir X Y Z] [--up X Y Z] [--stats]\n"
                 "             [-o out.exr|out.pfm]\n");
}

int main(int argc, char** argv) {
    std::string scene_path, out_path;
    int spp = 0, spi = 8, seed = 0, device = 0, width = 0, height = 0;
    double render_time = 0; // --time: seconds of rendering instead of a sample count
    bool stats = false;
    IG::ParameterSet params; // the camera orientation overrides (__camera_eye / _dir / _up)
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { usage(); std::exit(2); }
            return argv[++i];
        };
        auto vec3 = [&](const char* key) {
            IG::Vector3f v;
            for (int k = 0; k < 3; ++k) {
                const char* t = next();
                char* end = nullptr;
                v[k] = std::strtof(t, &end);
                if (end == t || *end) { std::fprintf(stderr, "igcli: %s needs three numbers\n", a.c_str()); std::exit(2); }
            }
            params.VectorParameters[key] = v;
        };
        if (a == "--spp") spp = std::atoi(next());
        else if (a == "--spi") spi = std::atoi(next());
        else if (a == "--seed") seed = std::atoi(next());
        else if (a == "--gpu-device") device = std::atoi(next());
        else if (a == "--time") render_time = std::atof(next());
        else if (a == "--width") width = std::atoi(next());
        else if (a == "--height") height = std::atoi(next());
        else if (a == "--eye") vec3("__camera_eye");
        else if (a == "--dir") vec3("__camera_dir");
        else if (a == "--up") vec3("__camera_up");
        else if (a == "--stats" || a == "--stats-full") stats = true;
        else if (a == "-o" || a == "--output") out_path = next();
        else if (a == "--gpu" || a == "--no-progress" || a == "--no-color" || a == "-q" || a == "--quiet") {}
        else if (a == "--cpu" || a == "--cpu-arch" || a == "--cpu-threads" || a == "--cpu-vectorwidth") {
            std::fprintf(stderr, "igcli: %s: this build's device is GPU-only (igx, HIP on gfx950); the reference's CPU "
                                 "device is not part of it\n", a.c_str());
            return 2;
        }
        else if (a == "-h" || a == "--help") { usage(); return 0; }
        else if (!a.empty() && a[0] == '-') {
            std::fprintf(stderr, "igcli: unknown option %s\n", a.c_str());
            usage();
            return 2;
        }
        else scene_path = a;
    }
    if (spp > 0 && render_time > 0) { std::fprintf(stderr, "igcli: --time excludes --spp\n"); return 2; }
    if ((width > 0) != (height > 0)) { std::fprintf(stderr, "igcli: --width needs --height and vice versa\n"); return 2; }
    if (spi < 1) { std::fprintf(stderr, "igcli: --spi must be positive\n"); return 2; }
    if (scene_path.empty()) { usage(); return 2; }
    char err[1024] = {0};
    igx_scene* scene = igx_scene_load_file(scene_path.c_str(), err, sizeof(err));
    if (!scene) { std::fprintf(stderr, "failed to load scene: %s\n", err); return 1; }
    const igx_scene_desc* desc = igx_scene_get_desc(scene);
    if (spp <= 0) spp = spi;
    // igcli rounds spp up to a multiple of spi (cli/main.cpp:110-113); with
    // --time the loop runs until that much rendering time has passed
    const int iters = render_time > 0 ? 0 : (spp + spi - 1) / spi;
    const int W = width > 0 ? width : desc->film_width, H = height > 0 ? height : desc->film_height;
    try {
        IG::SceneDatabase db;
        IG::TechniqueVariantShaderSet shaders;
        IG::serialize_scene(*desc, db, shaders.shading);
        IG::Device::SetupSettings ss;
        ss.target = IG::Target::makeGPU(device);
        ss.AcquireStats = stats;
        IG::Device dev(ss);
        IG::Device::SceneSettings sc;
        sc.database = &db;
        dev.assignScene(sc);
        std::vector<double> rates;
        double total_s = 0; // wall time of the render loop (cli/main.cpp:127-135)
        const auto t_all = std::chrono::steady_clock::now();
        for (int it = 0; render_time > 0 ? total_s < render_time : it < iters; ++it) {
            IG::Device::RenderSettings rs;
            rs.spi = spi;
            rs.width = W;
            rs.height = H;
            rs.iteration = it;
            rs.user_seed = seed;
            auto t0 = std::chrono::steady_clock::now();
            dev.render(shaders, rs, params.empty() ? nullptr : &params);
            dev.synchronize(); // render() only queues the iteration
            double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            rates.push_back((double)spi * W * H / s / 1e6);
            total_s += s;
        }
        const igx_stats& st = dev.getStatistics()->raw();
        std::sort(rates.begin(), rates.end());
        double rays = (double)(st.camera_rays + st.bounce_rays + st.shadow_rays);
        std::printf("# %f %f %f Msamples/s\n", rates.front(), rates[rates.size() / 2], rates.back());
        std::printf("# %.3f Mrays/s (camera %llu, bounce %llu, shadow %llu) over %.3f ms\n", rays / total_s / 1e6,
                    (unsigned long long)st.camera_rays, (unsigned long long)st.bounce_rays, (unsigned long long)st.shadow_rays,
                    total_s * 1e3);
        if (stats) {
            const size_t all_ms = (size_t)(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_all).count());
            std::printf("%s  Iterations: %zu\n  SPP: %zu\n  SPI: %d\n", dev.getStatistics()->dump(all_ms, rates.size()).c_str(),
                        rates.size(), rates.size() * (size_t)spi, spi);
        }
        if (!out_path.empty()) {
            IG::Device::AOVAccessor acc = dev.getFramebufferForHost("");
            float inv = acc.IterationCount ? 1.0f / acc.IterationCount : 0.0f;
            const bool pfm = out_path.size() >= 4 && out_path.compare(out_path.size() - 4, 4, ".pfm") == 0;
            if (!pfm) {
                if (igx_write_exr(out_path.c_str(), acc.Data, W, H, 3, inv) != 0) {
                    std::fprintf(stderr, "cannot write %s\n", out_path.c_str());
                    return 1;
                }
            } else {
                FILE* f = std::fopen(out_path.c_str(), "wb");
                if (!f) { std::fprintf(stderr, "cannot write %s\n", out_path.c_str()); return 1; }
                std::fprintf(f, "PF\n%d %d\n-1.0\n", W, H);
                for (int y = H - 1; y >= 0; --y) { // PFM rows go bottom-up
                    std::vector<float> row(3 * W);
                    for (int x = 0; x < 3 * W; ++x) row[x] = acc.Data[(size_t)y * 3 * W + x] * inv;
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
