// Host restatements of the reference's film utility shaders, used by the
// IG::Device facade (host/Device.h) and the reference-side binding
//  for Device::tonemap / Device::imageinfo, which are
// outside the traced path ("stub or CPU fallback"):
//   * tonemap_film   -- entrypoints/tonemap.art (ig_tonemap_pipeline)
//   * imageinfo_film -- entrypoints/imageinfo.art (ig_imageinfo_pipeline)
// with the colour conversions and tone curves of core/color.art:77-142.
// Plain types only, so a translation unit that defines the reference's own
// IG::Device can include it.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace igx {

struct FilmColor { float r, g, b; };

// core/color.art:84-100: sRGB -> CIE xyY (Y is the luminance) and back
inline FilmColor srgb_to_xyY(FilmColor c) {
    const float X = 0.4124564f * c.r + 0.3575761f * c.g + 0.1804375f * c.b;
    const float Y = 0.2126729f * c.r + 0.7151522f * c.g + 0.0721750f * c.b;
    const float Z = 0.0193339f * c.r + 0.1191920f * c.g + 0.9503041f * c.b;
    const float n = X + Y + Z;
    if (n <= 1.1920929e-7f) return FilmColor{0, 0, 0};
    return FilmColor{X / n, Y / n, Y};
}
inline FilmColor xyY_to_srgb(FilmColor c) {
    if (c.g <= 1.1920929e-7f) return FilmColor{0, 0, 0};
    const float X = c.r * c.b / c.g, Y = c.b, Z = (1 - c.r - c.g) * c.b / c.g;
    return FilmColor{3.2404542f * X - 1.5371385f * Y - 0.4985314f * Z, -0.9692660f * X + 1.8760108f * Y + 0.0415560f * Z,
                     0.0556434f * X - 0.2040259f * Y + 1.0572252f * Z};
}
inline float film_safe_div(float a, float b) { return b == 0 ? 0.0f : a / b; }
// mod tonemapping (core/color.art:101-134): 0 none, 1 Reinhard, 2 modified
// Reinhard (white point 4), 3 ACES (Narkowicz 2015), else Uncharted 2
inline float tonemap_curve(int method, float L) {
    switch (method) {
    case 0: return L;
    case 1: return film_safe_div(L, 1.0f + L);
    case 2: return film_safe_div(L * (1.0f + L / 16.0f), 1.0f + L);
    case 3: return film_safe_div(L * (2.51f * L + 0.03f), L * (2.43f * L + 0.59f) + 0.14f);
    default: {
        auto f = [](float x) {
            return ((x * (0.15f * x + 0.10f * 0.50f) + 0.20f * 0.02f) / (x * (0.15f * x + 0.50f) + 0.20f * 0.30f)) - 0.02f / 0.30f;
        };
        return f(L) / f(11.2f);
    }
    }
}
inline float srgb_gamma(float x) { return x <= 0.0031308f ? 12.92f * x : 1.055f * std::pow(x, 0.416666667f) - 0.055f; }
inline uint32_t packed_color(uint32_t r, uint32_t g, uint32_t b, uint32_t a) { return (a << 24) | (r << 16) | (g << 8) | b; }
inline uint32_t color_byte(float v) { return (uint32_t)(uint8_t)(std::min(std::max(v, 0.0f), 1.0f) * 255); }

// ig_tonemap_pipeline: each pixel scaled by `scale` (the caller's Scale /
// IterationCount), to xyY; NaN luminance cyan, inf pink, a negative
// component orange; else the tone curve on exposure_factor * Y +
// exposure_offset, back to sRGB, optional sRGB gamma, packed ARGB bytes
inline void tonemap_film(const float* rgb, size_t pixels, float scale, int method, bool use_gamma, float exposure_factor,
                         float exposure_offset, uint32_t* out) {
    for (size_t i = 0; i < pixels; ++i) {
        const FilmColor c = srgb_to_xyY(FilmColor{rgb[3 * i] * scale, rgb[3 * i + 1] * scale, rgb[3 * i + 2] * scale});
        if (std::isnan(c.b)) { out[i] = packed_color(0, 255, 255, 255); continue; }
        if (!std::isfinite(c.b)) { out[i] = packed_color(255, 0, 150, 255); continue; }
        if (c.r < 0 || c.g < 0 || c.b < 0) { out[i] = packed_color(255, 255, 0, 255); continue; }
        FilmColor o = xyY_to_srgb(FilmColor{c.r, c.g, tonemap_curve(method, exposure_factor * c.b + exposure_offset)});
        if (use_gamma) o = FilmColor{srgb_gamma(o.r), srgb_gamma(o.g), srgb_gamma(o.b)};
        out[i] = packed_color(color_byte(o.r), color_byte(o.g), color_byte(o.b), 255);
    }
}

struct FilmInfo {
    float min, max, avg, soft_min, soft_max, median;
    int inf_count, nan_count, neg_count;
};
// ig_imageinfo_pipeline: luminance min / max / average of the scaled film
// (non-finite components read as 0); on films larger than 10 x 10 the soft
// min / max / median from the 3x3 windows of the interior pixels (2nd, 8th
// and 5th of each sorted window; min of the non-negative soft minima, max of
// the soft maxima, mean of the medians), else min / max / average; inf / NaN /
// negative component counts; histograms of R, G, B and luminance over
// [min, soft max] in `bins` bins
inline FilmInfo imageinfo_film(const float* rgb, size_t w, size_t h, float scale, size_t bins, int* hr, int* hg, int* hb, int* hl,
                               bool error_stats, bool histogram) {
    FilmInfo out{0, 0, 0, 0, 0, 0, 0, 0, 0};
    const size_t n = w * h;
    auto fin = [&](size_t k) { const float a = rgb[k]; return std::isfinite(a) ? a : 0.0f; };
    std::vector<float> L(n);
    float mn = INFINITY, mx = -INFINITY, sum = 0;
    for (size_t i = 0; i < n; ++i) {
        L[i] = srgb_to_xyY(FilmColor{fin(3 * i) * scale, fin(3 * i + 1) * scale, fin(3 * i + 2) * scale}).b;
        mn = std::fmin(mn, L[i]);
        mx = std::fmax(mx, L[i]);
        sum += L[i];
    }
    out.min = mn;
    out.max = mx;
    out.avg = n ? sum / (float)n : 0.0f;
    if (w > 10 && h > 10) {
        float smin = 3.40282347e38f, smax = 0, med = 0;
        const float mf = film_safe_div(1, (float)((w - 2) * (h - 2)));
        for (size_t y = 1; y + 1 < h; ++y)
            for (size_t x = 1; x + 1 < w; ++x) {
                float win[9];
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j) win[3 * i + j] = L[(y + i - 1) * w + (x + j - 1)];
                std::sort(win, win + 9);
                if (win[1] >= 0) smin = std::min(smin, win[1]);
                if (win[7] >= 0) smax = std::max(smax, win[7]);
                if (win[4] >= 0) med += win[4] * mf;
            }
        out.soft_min = smin;
        out.soft_max = smax;
        out.median = med;
    } else {
        out.soft_min = out.min;
        out.soft_max = out.max;
        out.median = out.avg;
    }
    if (error_stats)
        for (size_t k = 0; k < 3 * n; ++k) {
            const float c = rgb[k];
            out.inf_count += std::isinf(c) ? 1 : 0;
            out.nan_count += std::isnan(c) ? 1 : 0;
            out.neg_count += std::signbit(c) ? 1 : 0;
        }
    if (histogram && bins > 0 && hr && hg && hb && hl) {
        const float start = out.min < out.max ? out.min : 0.0f;
        const float end = out.min < out.soft_max ? out.soft_max : (out.min < out.max ? out.max : start + 1);
        const float factor = film_safe_div((float)bins, std::fmax(0.0f, end - start));
        auto bin = [&](float v) { return std::min(std::max((int)((v - start) * factor), 0), (int)bins - 1); };
        int* hist[4] = {hr, hg, hb, hl};
        for (int c = 0; c < 4; ++c) std::fill(hist[c], hist[c] + bins, 0);
        for (size_t i = 0; i < n; ++i) {
            const float r = fin(3 * i) * scale, g = fin(3 * i + 1) * scale, b = fin(3 * i + 2) * scale;
            ++hr[bin(r)];
            ++hg[bin(g)];
            ++hb[bin(b)];
            ++hl[bin(srgb_to_xyY(FilmColor{r, g, b}).b)];
        }
    }
    return out;
}

} // namespace igx
