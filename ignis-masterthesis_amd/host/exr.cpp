// Minimal OpenEXR (single part, scanline, NO_COMPRESSION) writer and reader
// for linear RGB(A) float images.  Stands in for Image::save / Image::load
// (src/runtime/Image.h:92-101, tinyexr in the reference) on the output side of
// the render path: igcli and the C-ABI write the averaged framebuffer as EXR.
//
// File layout (OpenEXR 2 file format): magic 20000630, version 2 (flags 0),
// header attributes (name\0 type\0 int32 size, value) terminated by a null
// byte, a line-offset table (one uint64 per scanline), then per scanline:
// int32 y, int32 byte count, and the line's samples channel by channel in
// alphabetical channel order (A, B, G, R), each as width float32 values.
#include "igx_scene.h"

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

void put_bytes(std::vector<uint8_t>& b, const void* p, size_t n) {
    const uint8_t* c = static_cast<const uint8_t*>(p);
    b.insert(b.end(), c, c + n);
}
template <typename T>
void put(std::vector<uint8_t>& b, T v) { put_bytes(b, &v, sizeof(T)); }
void put_str(std::vector<uint8_t>& b, const char* s) { put_bytes(b, s, std::strlen(s) + 1); }

void attr(std::vector<uint8_t>& b, const char* name, const char* type, const std::vector<uint8_t>& value) {
    put_str(b, name);
    put_str(b, type);
    put<int32_t>(b, (int32_t)value.size());
    b.insert(b.end(), value.begin(), value.end());
}

} // namespace

extern "C" int igx_write_exr(const char* path, const float* rgb, int32_t width, int32_t height, int32_t channels, float scale) {
    if (!path || !rgb || width <= 0 || height <= 0 || (channels != 3 && channels != 4)) return -1;
    static const char* names4[] = {"A", "B", "G", "R"};
    static const char* names3[] = {"B", "G", "R"};
    const char** names = channels == 4 ? names4 : names3;
    auto src_channel = [&](int k) { // alphabetical position -> interleaved RGB(A) index
        const char* n = names[k];
        return n[0] == 'R' ? 0 : n[0] == 'G' ? 1 : n[0] == 'B' ? 2 : 3;
    };
    std::vector<uint8_t> hdr;
    put<uint32_t>(hdr, 20000630u);
    put<uint32_t>(hdr, 2u);
    {
        std::vector<uint8_t> v;
        for (int k = 0; k < channels; ++k) {
            put_str(v, names[k]);
            put<int32_t>(v, 2); // FLOAT
            put<uint8_t>(v, 0); // pLinear
            put<uint8_t>(v, 0);
            put<uint8_t>(v, 0);
            put<uint8_t>(v, 0);
            put<int32_t>(v, 1); // xSampling
            put<int32_t>(v, 1); // ySampling
        }
        put<uint8_t>(v, 0);
        attr(hdr, "channels", "chlist", v);
    }
    attr(hdr, "compression", "compression", {0});
    {
        std::vector<uint8_t> v;
        put<int32_t>(v, 0);
        put<int32_t>(v, 0);
        put<int32_t>(v, width - 1);
        put<int32_t>(v, height - 1);
        attr(hdr, "dataWindow", "box2i", v);
        attr(hdr, "displayWindow", "box2i", v);
    }
    attr(hdr, "lineOrder", "lineOrder", {0});
    {
        std::vector<uint8_t> v;
        put<float>(v, 1.0f);
        attr(hdr, "pixelAspectRatio", "float", v);
    }
    {
        std::vector<uint8_t> v;
        put<float>(v, 0.0f);
        put<float>(v, 0.0f);
        attr(hdr, "screenWindowCenter", "v2f", v);
    }
    {
        std::vector<uint8_t> v;
        put<float>(v, 1.0f);
        attr(hdr, "screenWindowWidth", "float", v);
    }
    put<uint8_t>(hdr, 0);

    const size_t line_bytes = (size_t)width * channels * sizeof(float);
    const uint64_t table_end = hdr.size() + (uint64_t)height * 8;
    std::FILE* f = std::fopen(path, "wb");
    if (!f) return -2;
    bool ok = std::fwrite(hdr.data(), 1, hdr.size(), f) == hdr.size();
    for (int32_t y = 0; y < height && ok; ++y) {
        uint64_t off = table_end + (uint64_t)y * (8 + line_bytes);
        ok = std::fwrite(&off, 8, 1, f) == 1;
    }
    std::vector<float> line((size_t)width * channels);
    for (int32_t y = 0; y < height && ok; ++y) {
        for (int k = 0; k < channels; ++k) {
            const int c = src_channel(k);
            for (int32_t x = 0; x < width; ++x) {
                float v = c < 3 ? rgb[((size_t)y * width + x) * 3 + c] * scale : 1.0f;
                line[(size_t)k * width + x] = v;
            }
        }
        int32_t yy = y, nb = (int32_t)line_bytes;
        ok = std::fwrite(&yy, 4, 1, f) == 1 && std::fwrite(&nb, 4, 1, f) == 1 &&
             std::fwrite(line.data(), 1, line_bytes, f) == line_bytes;
    }
    ok = (std::fclose(f) == 0) && ok;
    return ok ? 0 : -3;
}
