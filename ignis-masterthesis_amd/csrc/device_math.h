// Device math, RNG and sampling helpers for the gfx950 kernels.
// Each helper restates the Artic stdlib function named in its comment
// (paths relative to /root/reference/src/artic).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace igxd {

constexpr float FLT_EPS_ = 1.1920928955e-07f;    // core/common.art:3
constexpr float FLT_MAX_ = 3.4028234664e+38f;    // core/common.art:4
constexpr float PI_ = 3.14159265359f;            // core/common.art:7
constexpr float INV_PI_ = 0.31830988618379067154f; // core/common.art:8

struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ f3 mulf(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// vec3_cross (core/vector.art:106-109)
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float len(f3 a) { return sqrtf(dot(a, a)); }
// vec3_normalize (core/vector.art:140): v * (1 / |v|)
__device__ __forceinline__ f3 normalize(f3 a) { return mulf(a, 1.0f / len(a)); }
__device__ __forceinline__ f3 f3of(float4 v) { return mk(v.x, v.y, v.z); }

// safe_rcp (core/common.art:95-98)
__device__ __forceinline__ float safe_rcp(float x) {
    const float min_rcp = 1e-8f;
    float ax = x > 0 ? x : -x;
    if (ax < min_rcp) return copysignf(FLT_MAX_, x); // prodsign(flt_max, x)
    return 1.0f / x;
}
// safe_div / safe_sqrt / clampf (core/common.art:167-171)
__device__ __forceinline__ float safe_div(float a, float b) { return fabsf(b) <= FLT_EPS_ ? 0.0f : a / b; }
// clamp (core/common.art, integer form)
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ float safe_sqrt(float a) { return sqrtf(fmaxf(0.0f, a)); }
__device__ __forceinline__ float safe_div_one(float a, float b) { return fabsf(b) <= FLT_EPS_ ? 1.0f : a / b; }
__device__ __forceinline__ float clampf(float v, float l, float u) { return fminf(u, fmaxf(l, v)); }
// sum_of_prod (core/common.art:148-153)
__device__ __forceinline__ float sum_of_prod(float a, float b, float c, float d) {
    float cd = c * d;
    float s = fmaf(a, b, cd);
    float err = fmaf(c, d, -cd);
    return s + err;
}
// lerp2 (core/common.art:124-126)
__device__ __forceinline__ float lerp2(float a, float b, float c, float k1, float k2) {
    return (1 - k1 - k2) * a + k1 * b + k2 * c;
}
__device__ __forceinline__ f3 lerp2(f3 a, f3 b, f3 c, float k1, float k2) {
    return mk(lerp2(a.x, b.x, c.x, k1, k2), lerp2(a.y, b.y, c.y, k1, k2), lerp2(a.z, b.z, c.z, k1, k2));
}
// vec3_reflect / vec3_refract (core/vector.art:126,129)
__device__ __forceinline__ f3 reflect(f3 v, f3 n) { return sub(mulf(n, 2 * dot(n, v)), v); }
__device__ __forceinline__ f3 refract(f3 v, f3 n, float eta, float cos_i, float cos_t) {
    return sub(mulf(n, eta * cos_i - cos_t), mulf(v, eta));
}

// make_orthonormal_mat3x3 (core/matrix.art:20-28); columns t, b, n
struct Frame {
    f3 t, b, n;
};
__device__ __forceinline__ Frame make_frame(f3 n) {
    float sign = copysignf(1.0f, n.z);
    float a = -1.0f / (sign + n.z);
    float b = n.x * n.y * a;
    Frame f;
    f.t = mk(1 + sign * n.x * n.x * a, sign * b, -sign * n.x);
    f.b = mk(b, sign + n.y * n.y * a, -n.y);
    f.n = n;
    return f;
}
// mat3x3_mul(local, v) = t*v.x + b*v.y + n*v.z (core/matrix.art:79-82)
__device__ __forceinline__ f3 frame_to_world(const Frame& f, f3 v) {
    return mk(f.t.x * v.x + f.b.x * v.y + f.n.x * v.z, f.t.y * v.x + f.b.y * v.y + f.n.y * v.z,
              f.t.z * v.x + f.b.z * v.y + f.n.z * v.z);
}

// ---- RNG: FNV seed + TEA counter generator (core/random.art:1-92) ----------
__device__ __forceinline__ uint32_t hash_combine(uint32_t h, uint32_t d) {
    h = (h * 16777619u) ^ (d & 0xFFu);
    h = (h * 16777619u) ^ ((d >> 8) & 0xFFu);
    h = (h * 16777619u) ^ ((d >> 16) & 0xFFu);
    h = (h * 16777619u) ^ ((d >> 24) & 0xFFu);
    return h;
}
__device__ __forceinline__ uint32_t create_random_seed(int sample, int iter, int frame, int x, int y, int user) {
    uint32_t h = 0x811C9DC5u;
    h = hash_combine(h, (uint32_t)sample);
    h = hash_combine(h, (uint32_t)iter);
    h = hash_combine(h, (uint32_t)frame);
    h = hash_combine(h, (uint32_t)x);
    h = hash_combine(h, (uint32_t)y);
    h = hash_combine(h, (uint32_t)user);
    return h;
}
__device__ __forceinline__ uint32_t sample_tea_u32(uint32_t v0, uint32_t v1) {
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        sum += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v1;
}
struct Rng {
    uint32_t seed, counter;
    __device__ __forceinline__ uint32_t next_u32() { return sample_tea_u32(seed, counter++); }
    // next_f32: [1,2) mantissa trick minus 1 (core/random.art:65-70)
    __device__ __forceinline__ float next_f32() {
        uint32_t x = next_u32();
        return __uint_as_float((x & 0x7FFFFFu) | 0x3F800000u) - 1.0f;
    }
    // next_i32(s, e), e inclusive, rejection sampling (core/random.art:46-63)
    __device__ __forceinline__ int next_i32(int s, int e) {
        uint32_t range = (uint32_t)(e - s);
        if (range == 0xFFFFFFFFu) return (int)next_u32() + s;
        uint32_t erange = range + 1;
        uint32_t scaling = 0xFFFFFFFFu / erange;
        uint32_t past = erange * scaling;
        uint32_t ret = next_u32();
        while (ret >= past) ret = next_u32();
        return (int)(ret / scaling) + s;
    }
};

// ---- sampling (core/sampling.art, core/warp.art) ---------------------------
// sample_cosine_hemisphere (core/sampling.art:65-76) + make_dir_sample_from_thetaphi (:12-19)
__device__ __forceinline__ f3 sample_cosine_hemisphere(float u, float v, float* pdf) {
    float c = safe_sqrt(v);
    float s = safe_sqrt(1 - v);
    float phi = 2 * PI_ * u;
    *pdf = c / PI_;
    return mk(s * cosf(phi), s * sinf(phi), c);
}
// equal_area_square_to_sphere (core/warp.art:63-91)
__device__ __forceinline__ f3 equal_area_square_to_sphere(float px, float py) {
    float u = 2 * px - 1;
    float v = 2 * py - 1;
    float au = fabsf(u), av = fabsf(v);
    float sd = 1 - (au + av);
    float d = fabsf(sd);
    float r = 1 - d;
    float phi = (r == 0 ? 1.0f : (av - au) / r + 1) * PI_ / 4;
    float cos_theta = copysignf(1 - r * r, sd);
    float sin_theta = safe_sqrt(2 - r * r) * r;
    float cos_phi = copysignf(cosf(phi), u);
    float sin_phi = copysignf(sinf(phi), v);
    return mk(cos_phi * sin_theta, sin_phi * sin_theta, cos_theta);
}

} // namespace igxd
