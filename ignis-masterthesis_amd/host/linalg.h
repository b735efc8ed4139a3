// Small float linear-algebra helpers for the host-side loader and BVH builder.
// Affine transforms follow Eigen's Transformf semantics the reference loader
// relies on (src/runtime/loader/Parser.cpp:164-237): translate/scale/rotate
// right-multiply onto the current transform.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>

namespace igx {

struct V3 {
    float x = 0, y = 0, z = 0;
    V3() = default;
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator*(float s, V3 a) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float norm(V3 a) { return std::sqrt(dot(a, a)); }
inline float norm2(V3 a) { return dot(a, a); }
inline V3 normalized(V3 a) {
    float n = norm(a);
    return n > 0 ? a / n : a;
}
inline V3 vmin(V3 a, V3 b) { return {std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z)}; }
inline V3 vmax(V3 a, V3 b) { return {std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z)}; }
inline bool approx(V3 a, V3 b, float eps) {
    // Eigen isApprox: ||a-b|| <= eps * min(||a||, ||b||)
    return norm(a - b) <= eps * std::min(norm(a), norm(b));
}

struct BBox {
    V3 min{std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), std::numeric_limits<float>::max()};
    V3 max{-std::numeric_limits<float>::max(), -std::numeric_limits<float>::max(), -std::numeric_limits<float>::max()};
    void extend(V3 p) { min = vmin(min, p); max = vmax(max, p); }
    void extend(const BBox& b) { min = vmin(min, b.min); max = vmax(max, b.max); }
    bool empty() const { return min.x > max.x || min.y > max.y || min.z > max.z; }
    V3 diameter() const { return empty() ? V3() : max - min; }
    V3 center() const { return (max + min) / 2.0f; }
    float half_area() const {
        V3 d = max - min;
        float kx = std::max(d.x, 0.f), ky = std::max(d.y, 0.f), kz = std::max(d.z, 0.f);
        return kx * (ky + kz) + ky * kz;
    }
    // BoundingBox::inflate (src/runtime/math/BoundingBox.h:56-64)
    void inflate(float eps) {
        V3 d = max - min;
        for (int i = 0; i < 3; ++i)
            if (d[i] < eps) { max[i] += eps / 2; min[i] -= eps / 2; }
    }
};

// 4x4 row-major affine matrix
struct M4 {
    float m[16];
    M4() { for (int i = 0; i < 16; ++i) m[i] = (i % 5 == 0) ? 1.f : 0.f; }
    float& at(int r, int c) { return m[r * 4 + c]; }
    float at(int r, int c) const { return m[r * 4 + c]; }
    static M4 identity() { return M4(); }
    bool is_identity() const {
        for (int i = 0; i < 16; ++i)
            if (m[i] != ((i % 5 == 0) ? 1.f : 0.f)) return false;
        return true;
    }
};
inline M4 operator*(const M4& a, const M4& b) {
    M4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float s = 0;
            for (int k = 0; k < 4; ++k) s += a.at(i, k) * b.at(k, j);
            r.at(i, j) = s;
        }
    return r;
}
inline V3 xform_point(const M4& t, V3 p) {
    float x = t.at(0, 0) * p.x + t.at(0, 1) * p.y + t.at(0, 2) * p.z + t.at(0, 3);
    float y = t.at(1, 0) * p.x + t.at(1, 1) * p.y + t.at(1, 2) * p.z + t.at(1, 3);
    float z = t.at(2, 0) * p.x + t.at(2, 1) * p.y + t.at(2, 2) * p.z + t.at(2, 3);
    float w = t.at(3, 0) * p.x + t.at(3, 1) * p.y + t.at(3, 2) * p.z + t.at(3, 3);
    return {x / w, y / w, z / w};
}
inline V3 xform_dir(const M4& t, V3 d) {
    return {t.at(0, 0) * d.x + t.at(0, 1) * d.y + t.at(0, 2) * d.z,
            t.at(1, 0) * d.x + t.at(1, 1) * d.y + t.at(1, 2) * d.z,
            t.at(2, 0) * d.x + t.at(2, 1) * d.y + t.at(2, 2) * d.z};
}
inline M4 translation(V3 v) { M4 r; r.at(0, 3) = v.x; r.at(1, 3) = v.y; r.at(2, 3) = v.z; return r; }
inline M4 scaling(V3 s) { M4 r; r.at(0, 0) = s.x; r.at(1, 1) = s.y; r.at(2, 2) = s.z; return r; }
inline M4 axis_rotation(int axis, float rad) {
    M4 r;
    float c = std::cos(rad), s = std::sin(rad);
    int a = (axis + 1) % 3, b = (axis + 2) % 3;
    r.at(a, a) = c; r.at(a, b) = -s; r.at(b, a) = s; r.at(b, b) = c;
    return r;
}

// 3x3 helpers (row-major) -------------------------------------------------------
struct M3 {
    float m[9];
};
inline M3 linear_of(const M4& t) {
    M3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i * 3 + j] = t.at(i, j);
    return r;
}
inline float det3(const M3& a) {
    const float* m = a.m;
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}
inline M3 inverse3(const M3& a) {
    const float* m = a.m;
    float d = det3(a);
    float id = 1.0f / d;
    M3 r;
    r.m[0] = (m[4] * m[8] - m[5] * m[7]) * id;
    r.m[1] = (m[2] * m[7] - m[1] * m[8]) * id;
    r.m[2] = (m[1] * m[5] - m[2] * m[4]) * id;
    r.m[3] = (m[5] * m[6] - m[3] * m[8]) * id;
    r.m[4] = (m[0] * m[8] - m[2] * m[6]) * id;
    r.m[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    r.m[6] = (m[3] * m[7] - m[4] * m[6]) * id;
    r.m[7] = (m[1] * m[6] - m[0] * m[7]) * id;
    r.m[8] = (m[0] * m[4] - m[1] * m[3]) * id;
    return r;
}
inline M3 transpose3(const M3& a) {
    M3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i * 3 + j] = a.m[j * 3 + i];
    return r;
}
inline V3 mul3(const M3& a, V3 v) {
    return {a.m[0] * v.x + a.m[1] * v.y + a.m[2] * v.z, a.m[3] * v.x + a.m[4] * v.y + a.m[5] * v.z,
            a.m[6] * v.x + a.m[7] * v.y + a.m[8] * v.z};
}
// Affine inverse (linear part inverted, translation -L^-1 t)
inline M4 affine_inverse(const M4& t) {
    M3 li = inverse3(linear_of(t));
    V3 tr{t.at(0, 3), t.at(1, 3), t.at(2, 3)};
    V3 nt = -mul3(li, tr);
    M4 r;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) r.at(i, j) = li.m[i * 3 + j];
        r.at(i, 3) = nt[i];
    }
    return r;
}

} // namespace igx
