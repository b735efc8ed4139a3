// CPU check of the quantised 4-wide nodes (host/bvh_build.cpp quantize_bvh4,
// device node_step4q): for random child boxes at many magnitudes and extents,
// (1) the decoded box o + q * s contains the child box with at least half a
// quantum to spare, and (2) every random ray whose slab test accepts the exact
// box (node_step4's float formula) is accepted by the quantised slab test
// (node_step4q's formula), with the same tmin / tmax clamps.
#include "bvh_build.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>

static float safe_rcp(float x) {
    const float e = 1.0e-9f; // device_math.h's cutoff does not matter for this check
    return std::fabs(x) < e ? std::copysign(1.0f / e, x) : 1.0f / x;
}

int main() {
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> u(0.f, 1.f);
    long bad_box = 0, bad_ray = 0, rays = 0, accepted = 0;
    for (int it = 0; it < 20000; ++it) {
        const float mag = std::pow(10.f, -3.f + 6.f * u(rng));     // coordinates 1e-3 .. 1e3
        const float ext = mag * std::pow(10.f, -7.f + 7.f * u(rng)); // node extent down to 1e-7 of them
        const float c[3] = {mag * (2 * u(rng) - 1), mag * (2 * u(rng) - 1), mag * (2 * u(rng) - 1)};
        igx::Bvh4Node n{};
        for (int k = 0; k < 4; ++k) {
            float* lo[3] = {n.lo_x, n.lo_y, n.lo_z};
            float* hi[3] = {n.hi_x, n.hi_y, n.hi_z};
            const bool absent = k == 3 && (it % 5) == 0;
            n.ref[k] = absent ? igx::kEmptyRef : k;
            for (int a = 0; a < 3; ++a) {
                if (absent) { lo[a][k] = hi[a][k] = INFINITY; continue; }
                const float p = c[a] + ext * (u(rng) - 0.5f), q = c[a] + ext * (u(rng) - 0.5f);
                lo[a][k] = std::fmin(p, q);
                hi[a][k] = std::fmax(p, q) + (u(rng) < 0.1f ? 0.f : 0.f);
            }
        }
        const igx::Bvh4QNode qn = igx::quantize_bvh4(n);
        const float org[3] = {qn.origin[0], qn.origin[1], qn.origin[2]};
        const float sc[3] = {qn.sx, qn.sy, qn.sz};
        const uint32_t ql[3] = {qn.qlo_x, qn.qlo_y, qn.qlo_z}, qh[3] = {qn.qhi_x, qn.qhi_y, qn.qhi_z};
        for (int k = 0; k < 4; ++k) {
            if (n.ref[k] == igx::kEmptyRef) continue;
            const float* lo[3] = {n.lo_x, n.lo_y, n.lo_z};
            const float* hi[3] = {n.hi_x, n.hi_y, n.hi_z};
            for (int a = 0; a < 3; ++a) {
                const double dl = (double)org[a] + ((ql[a] >> (8 * k)) & 255u) * (double)sc[a];
                const double dh = (double)org[a] + ((qh[a] >> (8 * k)) & 255u) * (double)sc[a];
                if (!(dl <= lo[a][k] - 0.5 * sc[a] && dh >= hi[a][k] + 0.5 * sc[a])) ++bad_box;
            }
        }
        // rays: from around the node towards it, the device formulas
        for (int r = 0; r < 20; ++r) {
            float o[3], d[3];
            const float far = ext * std::pow(10.f, 3.f * u(rng));
            float dn = 0;
            for (int a = 0; a < 3; ++a) {
                o[a] = c[a] + far * (2 * u(rng) - 1);
                d[a] = c[a] + ext * (u(rng) - 0.5f) - o[a];
                dn += d[a] * d[a];
            }
            dn = std::sqrt(dn);
            for (float& x : d) x /= dn;
            float idir[3], iorg[3];
            for (int a = 0; a < 3; ++a) {
                idir[a] = safe_rcp(d[a]);
                iorg[a] = -(o[a] * idir[a]);
            }
            const float tmin = 0, tmax = 3.4e38f;
            float S[3], O[3];
            for (int a = 0; a < 3; ++a) {
                S[a] = sc[a] * idir[a];
                O[a] = std::fmaf(org[a], idir[a], iorg[a]);
            }
            for (int k = 0; k < 4; ++k) {
                if (n.ref[k] == igx::kEmptyRef) continue;
                const float* lo[3] = {n.lo_x, n.lo_y, n.lo_z};
                const float* hi[3] = {n.hi_x, n.hi_y, n.hi_z};
                float en = tmin, ex = tmax, qe = tmin, qx = tmax;
                for (int a = 0; a < 3; ++a) {
                    const float t0 = std::fmaf(lo[a][k], idir[a], iorg[a]), t1 = std::fmaf(hi[a][k], idir[a], iorg[a]);
                    en = std::fmax(en, std::fmin(t0, t1));
                    ex = std::fmin(ex, std::fmax(t0, t1));
                    const float q0 = std::fmaf((float)((ql[a] >> (8 * k)) & 255u), S[a], O[a]);
                    const float q1 = std::fmaf((float)((qh[a] >> (8 * k)) & 255u), S[a], O[a]);
                    qe = std::fmax(qe, std::fmin(q0, q1));
                    qx = std::fmin(qx, std::fmax(q0, q1));
                }
                ++rays;
                if (en <= ex) {
                    ++accepted;
                    if (!(qe <= qx)) ++bad_ray;
                }
            }
        }
    }
    std::printf("boxes with < half a quantum of slack: %ld; rays accepted by the exact box %ld of %ld, rejected by the quantised one: %ld\n",
                bad_box, accepted, rays, bad_ray);
    std::printf(bad_box || bad_ray ? "failed\n" : "ok\n");
    return bad_box || bad_ray ? 1 : 0;
}
