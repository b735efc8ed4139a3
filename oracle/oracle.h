/*
 * oracle.h — CPU restatement of the reference path for parity checks.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so, and only as the checker
 * or the timed CPU baseline.  The product path (libigx.so) never links or
 * calls it.
 *
 * What it restates (paths relative to /root/reference/src/artic):
 *   driver/mapping_cpu.art:694-836   cpu_trace: 16x16 tiles over all cores
 *   traversal/mapping_cpu.art:398-495 cpu_traverse_helper (scalar: per-entry tmin
 *                                    culling, nearer-first, entity leaf box test)
 *   traversal/intersection.art       MT triangle test, slab test
 *   shapes/trimesh.art, sphere.art   surface elements, analytic sphere
 *   technique/pathtracer.art         on_hit / on_miss / on_shadow / on_bounce
 *   bsdf/diffuse.art, dielectric.art Lambert, pure dielectric
 *   light/area.art (plane), env.art (spherical), point.art, spot.art
 *   core/random.art                  FNV seed + TEA counter RNG
 * Each path is a pure function of (pixel, sample, iteration, frame, seed), so
 * the wavefront order of the reference (sort by entity, compaction) does not
 * change any per-path value; the oracle therefore walks each path to its end.
 * Per-path radiance is accumulated hit-emission/miss first, then the NEE
 * contribution of the same bounce, and pixels sum samples in sample order,
 * matching the GPU resolve.
 *
 * Parity status: restatement pinned by the reference's own known answers
 * (src/tests/artic/test_intersection.art; analytic integrator values re-derived
 * in tests/golden/README.md).  The reference itself cannot be built or run here
 * (AnyDSL/Artic JIT, TBB and CPM dependencies are absent).
 */
#ifndef IGX_ORACLE_H
#define IGX_ORACLE_H

#include <stdint.h>

#include "../include/igx_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_params {
    int32_t width, height;
    int32_t spi;
    int32_t iteration, frame, seed;
    int32_t threads;          /* 0: all cores */
    /* optional pixel window [x0, x1) x [y0, y1); x1 == 0 means full film */
    int32_t x0, y0, x1, y1;
    /* ray-list mode: num_rays > 0 (8 floats per ray), film = num_rays x 1 */
    int32_t num_rays;
    const float* rays;
    /* 1: the reference CPU device's wavefront per 16x16 tile (cpu_trace,
     * driver/mapping_cpu.art:694-836: a stream of spi * 256 rays, closest
     * hits, sort by entity, shading in entity order, compaction, any-hit
     * shadow stream, splats into the film); 0: each path to its end.  Per
     * path both compute the same radiance; the film sums in another order. */
    int32_t stream;
    /* per-path probes (tests): 0 = every sample; s + 1 = only sample s of
     * each pixel enters the film (scaled by 1 / spi as usual; per-path mode) */
    int32_t probe_sample;
    /* the path tracer's MIS AOVs (technique aov_mis, PathTechnique.cpp:16-25):
     * non-null = "Direct Weights" (emission hits and misses, pathtracer.art:128,158)
     * and "NEE Weights" (unoccluded shadow rays, :206) splat here like the film */
    float* aov_direct;
    float* aov_nee;
} oracle_params;

typedef struct oracle_stats {
    uint64_t camera_rays, bounce_rays, shadow_rays;
    uint64_t node_visits, leaf_visits, tri_tests;
    double seconds;
    int32_t threads;
} oracle_stats;

typedef struct oracle_scene oracle_scene;

oracle_scene* oracle_scene_create(const igx_scene_desc* desc);
void oracle_scene_free(oracle_scene* s);

/* Adds one iteration to fb (width*height*3, row-major RGB): fb += sum_s L_s / spi. */
int oracle_render(const oracle_scene* s, const oracle_params* p, float* fb, oracle_stats* stats);

/* Closest hit for n rays (8 floats: org, dir, tmin, tmax); flags = ray flags. */
void oracle_trace_hits(const oracle_scene* s, const float* rays, int32_t n, uint32_t flags, int32_t* ent_prim, float* tuv);
void oracle_trace_occlusion(const oracle_scene* s, const float* rays, int32_t n, uint32_t flags, int32_t* occluded);

/* Primitive tests (for the reference's Artic KATs, test_intersection.art).
 * tri: v0, e1 = v0 - v1, e2 = v2 - v0, n = cross(e1, e2) (12 floats); ray: org, dir, tmin, tmax.
 * Returns 1 on hit and writes t, u, v. */
int oracle_intersect_tri(const float* tri12, const float* ray8, float* tuv);
/* Slab test intersect_ray_box_single: returns 1 on hit and writes t. */
int oracle_intersect_box(const float* bmin3, const float* bmax3, const float* ray8, float* t);

/* RNG helpers exposed for tests (core/random.art). */
uint32_t oracle_random_seed(int32_t sample, int32_t iter, int32_t frame, int32_t x, int32_t y, int32_t user);
float oracle_next_f32(uint32_t seed, uint32_t* counter);
/* principled BSDF * cos(wi) in a front-facing local frame (normal +z), n pairs,
 * diffuse lobe `model` (0 the reference's, 1 Disney 2015 split on the
 * roughness input, 2 Burley 2012; tests/golden/cycles_box_model.py) */
/* tie rule at equal distance: 0 larger (entity, primitive) wins (the
 * device's), 1 the later-visited hit wins (the reference's); process-wide */
void oracle_set_tie_rule(int reference);
void oracle_principled_eval(const igx_material* m, int n, const float* wo, const float* wi, int model, float* out);

#ifdef __cplusplus
}
#endif
#endif
