// CPU check of the quantised 4-wide nodes (host/bvh_build.cpp quantize_bvh4,
// device node_step4q): for random child boxes at many magnitudes and extents,
// (1) the decoded box o + q * s contains the child box with at least half a
// quantum to spare, and (2) every random ray whose slab test accepts the exact
// box (node_step4's float formula) is accepted by the quantised slab test
// (node_step4q's formula, both the octant-ordered form the device uses and the
// min / max form, each with the exit widening QSLAB_EXIT_WIDEN), with the same
// tmin / tmax clamps, for ray origins up to 1e6 node extents away and rays
// aimed at points on the child boxes' faces; and (3) the ordered and min / max
// forms give the same entry and exit distances.  Without the widening, rays
// from far away are rejected now and then (counted and printed, not failed).
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
    const float widen = 1.0f + 0x1p-20f; // igx_kernels.h QSLAB_EXIT_WIDEN
    long bad_box = 0, bad_ray = 0, bad_ordered = 0, unwidened_rejects = 0, rays = 0, accepted = 0;
    for (int it = 0; it < 100000; ++it) {
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
            const float far = ext * std::pow(10.f, 6.f * u(rng));
            // half the rays aim at a point on a face of a present child's box
            float aim[3];
            const int kc = (int)(u(rng) * 3.999f), fa = (int)(u(rng) * 2.999f);
            const bool on_face = (r & 1) && n.ref[kc] != igx::kEmptyRef;
            for (int a = 0; a < 3; ++a) {
                const float* lo = a == 0 ? n.lo_x : a == 1 ? n.lo_y : n.lo_z;
                const float* hi = a == 0 ? n.hi_x : a == 1 ? n.hi_y : n.hi_z;
                if (!on_face) aim[a] = c[a] + ext * (u(rng) - 0.5f);
                else if (a == fa) aim[a] = u(rng) < 0.5f ? lo[kc] : hi[kc];
                else aim[a] = lo[kc] + (hi[kc] - lo[kc]) * u(rng);
            }
            float dn = 0;
            for (int a = 0; a < 3; ++a) {
                o[a] = c[a] + far * (2 * u(rng) - 1);
                d[a] = aim[a] - o[a];
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
                float en = tmin, ex = tmax, qe = tmin, qx = INFINITY, oe = tmin, ox = INFINITY;
                for (int a = 0; a < 3; ++a) {
                    const float t0 = std::fmaf(lo[a][k], idir[a], iorg[a]), t1 = std::fmaf(hi[a][k], idir[a], iorg[a]);
                    en = std::fmax(en, std::fmin(t0, t1));
                    ex = std::fmin(ex, std::fmax(t0, t1));
                    const uint32_t bl = (ql[a] >> (8 * k)) & 255u, bh = (qh[a] >> (8 * k)) & 255u;
                    const float q0 = std::fmaf((float)bl, S[a], O[a]);
                    const float q1 = std::fmaf((float)bh, S[a], O[a]);
                    qe = std::fmax(qe, std::fmin(q0, q1));
                    qx = std::fmin(qx, std::fmax(q0, q1));
                    // octant-ordered: near / far byte by the sign of idir
                    const bool neg = std::signbit(idir[a]);
                    oe = std::fmax(oe, std::fmaf((float)(neg ? bh : bl), S[a], O[a]));
                    ox = std::fmin(ox, std::fmaf((float)(neg ? bl : bh), S[a], O[a]));
                }
                if (oe != qe || ox != qx) ++bad_ordered;
                const float qx_raw = std::fmin(qx, tmax);
                qx = std::fmin(qx * widen, tmax);
                ++rays;
                if (en <= ex) {
                    ++accepted;
                    if (!(qe <= qx)) ++bad_ray;
                    if (!(qe <= qx_raw)) ++unwidened_rejects;
                }
            }
        }
    }
    std::printf("boxes with < half a quantum of slack: %ld; rays accepted by the exact box %ld of %ld, rejected by the quantised one: %ld "
                "(without the exit widening: %ld); ordered != min/max distances: %ld\n",
                bad_box, accepted, rays, bad_ray, unwidened_rejects, bad_ordered);
    const bool fail = bad_box || bad_ray || bad_ordered;
    std::printf(fail ? "failed\n" : "ok\n");
    return fail ? 1 : 0;
}
