// Kernel-side building blocks: traversal, surface elements, BSDFs, lights and
// the path-tracer technique.  Restates (per function comment) the Artic code
// the reference JIT-specialises into its GPU kernels:
//   traversal/mapping_gpu.art, traversal/intersection.art, shapes/trimesh.art,
//   shapes/sphere.art, bsdf/diffuse.art, bsdf/dielectric.art, light/*.art,
//   technique/pathtracer.art.
#pragma once

#include "device_math.h"
#include "device_scene.h"

namespace igxd {

struct SceneView {
    const float4* nodes;   // unified BVH2 node array: every BLAS, then the TLAS
    const float4* tris;    // 3 x float4 per triangle slot: (v0, prim id), (e1 = v0-v1), (e2 = v2-v0)
    const float4* inst;    // 4 x float4 per TLAS leaf slot (see device_scene.h)
    const float4* spheres; // origin.xyz, radius
    const float4* ent;     // ENT_STRIDE x float4 per entity
    const float4* vtx;     // mesh vertices (object space)
    const float4* nrm;     // mesh vertex normals (object space)
    const int4* idx;       // faces: local vertex indices
    const DevMaterial* mats;
    const DevLight* lights;
    int tlas_root;         // root node of the TLAS, or its only leaf (one entity)
    int num_lights;        // infinite lights first (light/light_selector.art:26-44)
    int num_infinite;
    float scene_radius;    // bbox_radius(scene_bbox) * 1.01 (light/env.art:75)
    DevCamera cam;
    int max_depth, min_depth, nee;
    float clamp;
    int num_nodes, num_inst, num_tris; // table sizes (for staging the traversal tables in LDS)
    // treelet: nodes [0, tree_n) of `nodes` (the hottest, igx_upload_scene's
    // hot order) staged in LDS at `tree` by stage_treelet (variant_tree kernels)
    const float4* tree;
    int tree_n;
    int* spill;            // traversal-stack overflow area of the launching stream (see TStack)
    int node_f4;           // float4s per BVH node (4: BVH2, 8: 4-wide)
    const int* ent_enc;    // per entity: its index among the enclosing entities (trace_enclosed), else -1
    const int2* enc;       // per enclosing entity: entity id, TLAS leaf slot
    const float4* enc_box; // per enclosing entity: world box lo.xyz, hi.xyz (path classes, option path_classes 3)
    int num_enc;
    int selector;          // NEE light selector in effect (IGX_SELECT_*; host/light_select.h)
    const float* sel_cdf;  // simple: CDF over the finite lights ([c_1 .. c_{n-1}, 1])
    const uint32_t* sel_tree; // hierarchy: codes (padded to 4), then 8 words per entry
    // world-space unit face normals per (entity, face), precomputed at upload
    // for scenes with few face instances (nullptr otherwise): fn_tab[ent_fn[e] + prim]
    const int* ent_fn;
    const float4* fn_tab;
    // per mesh face (shape level, at idx_off + prim): the three object-space
    // vertex normals with the vertex indices in .w (int bits), uploaded for
    // scenes with few faces (nullptr otherwise): one record per hit instead
    // of the face's index record and three scattered normal loads behind it;
    // with it, row 3 .w of the entity record holds ent_fn (int bits)
    const float4* fsh;
    // per mesh vertex: texture coordinates (as vtx), uploaded only when a
    // material carries a texture (DevMaterial::pad, textured_material)
    const float2* uv;
};

// Copy the traversal tables (nodes, instances, triangles) of a small scene
// into LDS, laid out back to back, and point a block-local view at them: the
// node loop then reads LDS (~50-cycle ds_read) instead of the vector-memory
// path, which the divergent node fetches otherwise keep busy.
// The enclosing entities' world boxes (path / shadow-ray classes, read by
// every lane at every append): a small LDS copy, so the class test does not
// wait on dependent global loads (they cost k_extend ~10 % of its wave time).
constexpr int MAX_ENC_BOXES = 32;
template <int BLOCK_>
__device__ __forceinline__ const float4* stage_enc_boxes(const SceneView& sv) {
    __shared__ float4 enc_box_lds[2 * MAX_ENC_BOXES];
    for (int k = threadIdx.x; k < 2 * sv.num_enc; k += BLOCK_) enc_box_lds[k] = sv.enc_box[k];
    return enc_box_lds;
}

template <int BLOCK_>
__device__ __forceinline__ SceneView stage_scene_lds(const SceneView& sv, float4* lds) {
    const int nf = sv.node_f4, sh = nf == 8 ? 3 : 2, ns = nf; // node stride in LDS (float4)
    const int n4 = sv.num_nodes * ns, i4 = sv.num_inst * 4, t3 = sv.num_tris * 3;
    for (int k = threadIdx.x; k < sv.num_nodes * nf; k += BLOCK_) lds[(k >> sh) * ns + (k & (nf - 1))] = sv.nodes[k];
    for (int k = threadIdx.x; k < i4; k += BLOCK_) lds[n4 + k] = sv.inst[k];
    for (int k = threadIdx.x; k < t3; k += BLOCK_) lds[n4 + i4 + k] = sv.tris[k];
    const float4* eb = stage_enc_boxes<BLOCK_>(sv);
    __syncthreads();
    SceneView l = sv;
    l.enc_box = eb;
    l.nodes = lds;
    l.inst = lds + n4;
    l.tris = lds + n4 + i4;
    return l;
}

// Stage the treelet (the scene's first tree_n nodes, the ones rays visit
// most: the top of the TLAS and of the busiest BLAS) in LDS for a kernel
// whose tables stay in global memory; node steps below tree_n then read LDS
// instead of waiting on an L2 / Infinity-Cache round trip.  Block-uniform:
// every thread of the block calls it before any divergent code.
template <int BLOCK_>
__device__ __forceinline__ SceneView stage_treelet(const SceneView& sv, float4* lds) {
    SceneView l = sv;
    l.tree = lds;
    if (sv.tree_n > 0 || sv.num_enc > 0) {
        const int n4 = sv.tree_n * sv.node_f4;
        for (int k = threadIdx.x; k < n4; k += BLOCK_) lds[k] = sv.nodes[k];
        l.enc_box = stage_enc_boxes<BLOCK_>(sv);
        __syncthreads();
    }
    return l;
}

struct TraceStats {
    uint32_t nodes, leaves, tris, blas, hits;
    uint32_t wnodes, wleaves; // wave-level iterations of the node loop / leaf phase (SIMD efficiency)
    // node visits in the TLAS, and at nodes of hot-order rank < 256 / 512 /
    // 1280 (order_hot_nodes: the prefixes a treelet can stage)
    uint32_t tlas_nodes = 0, hot[3] = {0, 0, 0};
    // k_extend phase clocks (wave-level, s_memtime): load, trace, shade, store
    unsigned long long cyc[4] = {0, 0, 0, 0};
    // k_extend by the class of the wave's group (camera, A, B, C): trace
    // cycles 0-3, shade cycles 4-7, groups 8-11, wave-level node iterations
    // 12-15, lane node visits 16-19 -- the wave's 20 counters in LDS (lane 0
    // updates them), so the instrumentation holds no registers
    unsigned long long* cls = nullptr;
    // shading sub-phase clocks of the instrumented k_extend (shade_step<.., true>):
    // class bucket of the wave's group and the last mark
    int bucket = 0;
    unsigned long long t_sub = 0;
};

// true on the lowest active lane of the wave (counts one event per wave)
__device__ __forceinline__ bool first_active_lane() {
    return (int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1;
}

// one node visit of the instrumented traversal
__device__ __forceinline__ void count_node(TraceStats& st, bool in_blas, int node) {
    st.nodes++;
    if (first_active_lane()) st.wnodes++;
    st.tlas_nodes += in_blas ? 0 : 1;
    st.hot[0] += node < 256 ? 1 : 0;
    st.hot[1] += node < 512 ? 1 : 0;
    st.hot[2] += node < 1280 ? 1 : 0;
}

// Ray flags (traversal/ray.art:19-23)
constexpr uint32_t RAY_CAMERA = 0x1, RAY_LIGHT = 0x2, RAY_BOUNCE = 0x4, RAY_SHADOW = 0x8, RAY_TYPE_MASK = 0xF;
#ifndef IGX_IDENTITY_INSTANCES
#define IGX_IDENTITY_INSTANCES 1
#endif
// instance record flag (info.w, next to the visibility bits): the trimesh
// instance's to_local is the identity, so its entity-space ray is the world
// ray (instance_test skips the transform; set by igx_upload_scene)
constexpr uint32_t INST_IDENTITY = 1u << 30;
// ... or a pure translation (rows (1 0 0 tx), (0 1 0 ty), (0 0 1 tz)): the
// entity-space ray is (o + t, d), so its reciprocal direction is the world
// ray's (IGX_TRANSLATE_INSTANCES)
#ifndef IGX_TRANSLATE_INSTANCES
#define IGX_TRANSLATE_INSTANCES 1
#endif
constexpr uint32_t INST_TRANSLATE = 1u << 29;
// the identity / translation shortcuts give transform_ray's direction bit for
// bit when no component is zero (with x != 0: 1*x + 0*y + 0*z == x)
__device__ __forceinline__ bool shortcut_dir_ok(f3 d) { return d.x != 0.0f && d.y != 0.0f && d.z != 0.0f; }

// ---------------------------------------------------------------------------
// Two-level traversal: TLAS (entities) -> BLAS (triangles) or analytic sphere.
// One loop for both levels with a per-lane stack in LDS (column layout: entry
// k of lane l at stk[k * stride], conflict-free).  Follows gpu_traverse_scene /
// gpu_traverse_helper / gpu_traverse_prim (traversal/mapping_gpu.art:73-226):
// slab test intersect_ray_box with ray.tmin folded in (intersection.art:170-181),
// nearer child first, tmax shrinks on every accepted hit, entity-local rays are
// NOT renormalised so t stays global (ray.art:53-59), entity visibility flags
// (ray.art:51), Moeller-Trumbore with -eps barycentric tolerance and u,v clamp
// (intersection.art:71-101), analytic sphere (shapes/sphere.art:104-130).
// ---------------------------------------------------------------------------
// Traversal state of one ray; trav_step advances it to the next leaf (or the
// end).  (Persistent lane-refill and if-if single-step variants built on this
// were measured slower on gfx950 than the plain grid-stride while-while loop:
// DESIGN.md §3.)
struct Trav {
    f3 o, d;          // world ray
    f3 lo, ld;        // ray of the current level (world at the TLAS, entity space in a BLAS)
    f3 idir, iorg;    // slab-test form of the current-level ray
    float tmin, tmax; // tmax shrinks on every accepted hit
    int node, sp;
    int cur_ent;
    int hit_ent, hit_prim;
    float hu, hv;
    uint32_t rflags;
    bool in_blas, found;
};

__device__ __forceinline__ bool is_leaf_ref(int r) { return r < 0 && r > REF_EXIT; }

// Per-lane traversal stack: the first `cap` entries live in an LDS column
// (entry e at lds[e * stride]); deeper entries, which only rays in the
// deepest parts of a wide or deep BVH reach, spill to a global column
// (entry e at spill[(e - cap) * sstride], one column per grid thread).  A
// small LDS stack thus serves every scene: LDS per block, and so occupancy,
// no longer scales with the worst-case stack depth.
// The LDS column stride is the block size, a compile-time constant: a push or
// pop is then one shift-add, not a quarter-rate v_mul_lo_u32.
constexpr int TSTACK_STRIDE = 256; // threads per block of every traversal kernel
struct TStack {
    int* lds;
    int* spill;
    int cap;
    int sstride;
};
// LDS entries through an LDS pointer, spill entries through a global one: the
// compiler then emits ds_* and global_* instructions instead of merging the
// two sources into flat ones (IGX_STACK_SPLIT 0: the plain generic form)
#ifndef IGX_STACK_SPLIT
#define IGX_STACK_SPLIT 1
#endif
typedef __attribute__((address_space(3))) int lds_int;
typedef __attribute__((address_space(1))) int global_int;
template <bool SPILL>
__device__ __forceinline__ void tpush(const TStack& s, int& sp, int v) {
    if constexpr (IGX_STACK_SPLIT && SPILL) {
        if (sp < s.cap) ((lds_int*)s.lds)[sp * TSTACK_STRIDE] = v;
        else ((global_int*)s.spill)[(sp - s.cap) * s.sstride] = v;
    } else {
        if (!SPILL || sp < s.cap) s.lds[sp * TSTACK_STRIDE] = v;
        else s.spill[(sp - s.cap) * s.sstride] = v;
    }
    ++sp;
}
template <bool SPILL>
__device__ __forceinline__ int tpop(const TStack& s, int& sp) {
    --sp;
    if constexpr (IGX_STACK_SPLIT && SPILL) {
        int v;
        if (sp < s.cap) v = ((lds_int*)s.lds)[sp * TSTACK_STRIDE];
        else v = ((global_int*)s.spill)[(sp - s.cap) * s.sstride];
        return v;
    } else {
        return (!SPILL || sp < s.cap) ? s.lds[sp * TSTACK_STRIDE] : s.spill[(sp - s.cap) * s.sstride];
    }
}
// The entry a pop would return (entry sp - 1; sp >= 1 inside a walk, entry 0
// holds the exit sentinel), read at the start of a node step or leaf together
// with the node's own loads: a step that ends in a pop then takes the entry
// from a register instead of waiting on a second, dependent LDS read
// (IGX_PEEK_POP; 0: the pop reads the entry when it happens).
#ifndef IGX_PEEK_POP
#define IGX_PEEK_POP 1
#endif
template <bool SPILL>
__device__ __forceinline__ int tpeek(const TStack& s, int sp) {
    const int e = sp > 0 ? sp - 1 : 0;
    if constexpr (SPILL) {
        if (e >= s.cap) return ((global_int*)s.spill)[(e - s.cap) * s.sstride];
    }
    return ((lds_int*)s.lds)[e * TSTACK_STRIDE];
}
// the pop of a step that peeked (top = tpeek(ts, sp) at its start)
template <bool SPILL, bool PEEK>
__device__ __forceinline__ int tpop_peeked(const TStack& s, int& sp, int top) {
    if constexpr (PEEK) {
        --sp;
        return top;
    } else {
        return tpop<SPILL>(s, sp);
    }
}
template <bool SPILL, bool PEEK>
__device__ __forceinline__ int tpeek_opt(const TStack& s, int sp) {
    if constexpr (PEEK) return tpeek<SPILL>(s, sp);
    else return 0;
}

// Push the farther hit children of a 4-wide node: r1 .. r(n-1) of the
// children sorted nearest first (n hit children, r(n-1) the deepest entry,
// r1 on top).  When all of them fit the LDS column with a slot to spare, the
// three stores are unconditional: an entry that is not pushed (n < 4, n < 3)
// is written to the dead slot just above the new top, so the step has no
// per-push branch (IGX_PUSH_SELECT; otherwise one guarded push each).
#ifndef IGX_PUSH_SELECT
#define IGX_PUSH_SELECT 1
#endif
template <bool SPILL>
__device__ __forceinline__ void tpush_hits3(const TStack& s, int& sp, int n, int r1, int r2, int r3) {
    if constexpr (IGX_PUSH_SELECT) {
        if (n < 2) return;
        const int top = sp + n - 2;
        if (top + 1 < s.cap) {
            const int dead = top + 1;
            lds_int* col = (lds_int*)s.lds;
            col[top * TSTACK_STRIDE] = r1;
            col[(n > 2 ? top - 1 : dead) * TSTACK_STRIDE] = r2;
            col[(n > 3 ? top - 2 : dead) * TSTACK_STRIDE] = r3;
            sp = top + 1;
            return;
        }
    }
    if (n > 3) tpush<SPILL>(s, sp, r3);
    if (n > 2) tpush<SPILL>(s, sp, r2);
    if (n > 1) tpush<SPILL>(s, sp, r1);
}
__device__ __forceinline__ TStack make_tstack(int* lds_base, int cap, int* spill) {
    const int g = blockIdx.x * TSTACK_STRIDE + threadIdx.x;
    return TStack{lds_base + threadIdx.x, spill + g, cap, (int)(gridDim.x * TSTACK_STRIDE)};
}

// Closest-hit acceptance with an order-independent tie rule: among hits at the
// same distance the larger (entity, primitive) wins.  The reference keeps the
// later-visited one (t <= tmax, intersection.art:97), which depends on BVH
// topology and traversal order; this rule makes the result independent of
// both (tile sharding, tail vs wavefront kernel, persistent-lane refill).
__device__ __forceinline__ bool accept_hit(const Trav& t, float th, int ent, int prim) {
    return th >= t.tmin && (th < t.tmax || (th == t.tmax && (ent > t.hit_ent || (ent == t.hit_ent && prim > t.hit_prim))));
}

__device__ __forceinline__ void trav_init(const SceneView& sv, Trav& t, f3 o, f3 d, float tmin, float tmax, uint32_t rflags,
                                          const TStack& ts) {
    t.o = o;
    t.d = d;
    t.lo = o;
    t.ld = d;
    t.idir = mk(safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z));
    t.iorg = mk(-(o.x * t.idir.x), -(o.y * t.idir.y), -(o.z * t.idir.z));
    t.tmin = tmin;
    t.tmax = fminf(tmax, FLT_MAX_); // finite: +inf bounds (absent children) then fail every slab test
    t.rflags = rflags;
    t.cur_ent = -1;
    t.hit_ent = -1;
    t.hit_prim = -1;
    t.hu = 0;
    t.hv = 0;
    t.in_blas = false;
    t.found = false;
    ts.lds[0] = REF_EXIT;
    t.sp = 1;
    t.node = sv.num_inst > 0 ? sv.tlas_root : REF_EXIT; // the root may be a leaf (one entity)
}

// The N float4s of node `node` (NS float4s apart): treelet nodes (TREE, node
// < tree_n) from LDS, the others from global memory: a branch per source
// with LDS and global loads (ds_read_b128 / global_load_dwordx4).  Round 3:
// primitives frame 33.1 / 33.1 -> 31.2 / 31.3 ms, S-deep 177.4 / 173.7 ->
// 161.8 / 162.1 ms against one generic (flat) load sequence serving both
// address spaces (IGX_TREE_SPLIT_LOADS 0; profiles/r03_ab_split_loads.log).
#ifndef IGX_TREE_SPLIT_LOADS
#define IGX_TREE_SPLIT_LOADS 1
#endif
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const f4v lds_f4v;
typedef __attribute__((address_space(1))) const f4v global_f4v;
template <int N, int NS, bool TREE>
__device__ __forceinline__ void load_node(const SceneView& sv, int node, float4 (&f)[N]) {
    if constexpr (IGX_TREE_SPLIT_LOADS && TREE) {
        if (node < sv.tree_n) {
            lds_f4v* np = (lds_f4v*)(sv.tree + NS * node);
#pragma unroll
            for (int k = 0; k < N; ++k) {
                const f4v v = np[k];
                f[k] = make_float4(v.x, v.y, v.z, v.w);
            }
        } else {
            global_f4v* np = (global_f4v*)(sv.nodes + NS * node);
#pragma unroll
            for (int k = 0; k < N; ++k) {
                const f4v v = np[k];
                f[k] = make_float4(v.x, v.y, v.z, v.w);
            }
        }
    } else {
        const float4* np = (TREE && node < sv.tree_n ? sv.tree : sv.nodes) + NS * node;
#pragma unroll
        for (int k = 0; k < N; ++k) f[k] = np[k];
    }
}
__device__ __forceinline__ int4 as_int4(float4 v) {
    return make_int4(__float_as_int(v.x), __float_as_int(v.y), __float_as_int(v.z), __float_as_int(v.w));
}

// Octant-ordered slab tests (the reference CPU traversal's `ordered` box test,
// intersection.art:174-176 with mapping_cpu.art:20-31, 181): per axis the
// bound the ray meets first is chosen by the sign of its inverse direction,
// so the entry distance is a max over three near planes and the exit a min
// over three far planes, without a min / max pair per axis and child.  For a
// positive inverse direction fma(lo, idir, iorg) <= fma(hi, idir, iorg)
// (rounding is monotone), so the ordered and the unordered test give the same
// entry and exit bit for bit; they differ only when a slab distance is NaN
// (a direction component below 1e-8 with |origin| > 1: inf - inf), where the
// reference's CPU and GPU tests differ in the same way.
// Quantised 4-wide nodes (IGX_ORDERED_SLAB_Q, default on): one select per
// axis and node picks the near and far byte words.  Round 4, same box,
// identical images: soup-1M 8-iteration frame 290.5 / 287.4 -> 268.8 / 270.8
// ms (trace 178.0 / 172.9 -> 160.0 / 163.2, shadow 228.7 / 227.1 -> 213.2 /
// 213.8), S-soup-16M 1-iteration frame 66.3 / 66.7 -> 63.2 / 62.8 ms
// (profiles/r04_ab_ordered_slab.log).
// (4-wide float nodes keep min / max: the same ordering by load address
// measured S-deep -1 % but primitives +4 %, round 4.)
#ifndef IGX_ORDERED_SLAB_Q
#define IGX_ORDERED_SLAB_Q 1
#endif
// Quantised exit widening: the quantised slab distance fma(q, S, O) carries
// the rounding of O = fma(origin, idir, iorg) on top of its own, up to about
// 2^-23 of the distance to the node, which the half quantum of slack only
// covers out to ~1.7e4 node extents.  The exit distance is
// scaled by 1 + 2^-20 (the exit plane's own distance bounds both roundings,
// entry <= exit), so the test stays a superset of the exact box test for
// rays from any distance (tests/native/quantize_check.cpp: origins up to
// 1e6 node extents away).  Only |exit| matters: a box with exit < tmin is
// rejected either way.
constexpr float QSLAB_EXIT_WIDEN = 1.0f + 0x1p-20f;
// Slab test of both children of BVH2 node `node` (intersect_ray_box,
// intersection.art:170-181, with ray.tmin folded in).  Returns the next node
// (nearer child first; the other is pushed) or the popped entry.
template <bool STATS, bool SPILL, int NS, bool TREE, bool PEEK>
__device__ __forceinline__ int node_step2(const SceneView& sv, const Trav& t, int node, const TStack& ts, int& sp,
                                         TraceStats& st) {
    if (STATS) count_node(st, t.in_blas, node);
    // treelet nodes (TREE, node < tree_n) from LDS, the others from global
    // memory (load_node: a branch per address space)
    float4 f[4];
    load_node<4, NS, TREE>(sv, node, f);
    const int top = tpeek_opt<SPILL, PEEK>(ts, sp);
    const float4 a = f[0], b = f[1], c = f[2];
    const int4 r = as_int4(f[3]);
    // child 0 box: lo (a.x, a.z, b.x) hi (a.y, a.w, b.y)
    // slab distances with explicit FMAs (the only contracted arithmetic
    // in the device code, built with -ffp-contract=off)
    float t0x = fmaf(a.x, t.idir.x, t.iorg.x), t1x = fmaf(a.y, t.idir.x, t.iorg.x);
    float t0y = fmaf(a.z, t.idir.y, t.iorg.y), t1y = fmaf(a.w, t.idir.y, t.iorg.y);
    float t0z = fmaf(b.x, t.idir.z, t.iorg.z), t1z = fmaf(b.y, t.idir.z, t.iorg.z);
    float en0 = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), t.tmin));
    float ex0 = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), t.tmax));
    // child 1 box: lo (b.z, c.x, c.z) hi (b.w, c.y, c.w)
    float s0x = fmaf(b.z, t.idir.x, t.iorg.x), s1x = fmaf(b.w, t.idir.x, t.iorg.x);
    float s0y = fmaf(c.x, t.idir.y, t.iorg.y), s1y = fmaf(c.y, t.idir.y, t.iorg.y);
    float s0z = fmaf(c.z, t.idir.z, t.iorg.z), s1z = fmaf(c.w, t.idir.z, t.iorg.z);
    float en1 = fmaxf(fmaxf(fminf(s0x, s1x), fminf(s0y, s1y)), fmaxf(fminf(s0z, s1z), t.tmin));
    float ex1 = fminf(fminf(fmaxf(s0x, s1x), fmaxf(s0y, s1y)), fminf(fmaxf(s0z, s1z), t.tmax));
    bool h0 = en0 <= ex0, h1 = en1 <= ex1;
    if (h0 && h1) {
        bool first0 = en0 < en1;
        tpush<SPILL>(ts, sp, first0 ? r.y : r.x);
        return first0 ? r.x : r.y;
    }
    if (h0) return r.x;
    if (h1) return r.y;
    return tpop_peeked<SPILL, PEEK>(ts, sp, top);
}

// Slab test of the four children of a 4-wide node (SoA bounds: one float4 per
// bound, child k in component k).  Hit children are ordered by entry distance
// with a 5-exchange sorting network; the nearest is returned and the others
// pushed farthest-first, or the stack is popped when none is hit.  Absent
// children have +inf bounds, which no slab test accepts.
__device__ __forceinline__ void slab4(float lo, float hi, float idir, float iorg, float& tn, float& tf) {
    float a = fmaf(lo, idir, iorg), b = fmaf(hi, idir, iorg);
    tn = fminf(a, b);
    tf = fmaxf(a, b);
}
__device__ __forceinline__ void cswap(float& da, int& ra, float& db, int& rb) {
    bool sw = db < da;
    float td = sw ? db : da;
    int tr = sw ? rb : ra;
    db = sw ? da : db;
    rb = sw ? ra : rb;
    da = td;
    ra = tr;
}
template <bool STATS, bool SPILL, int NS, bool TREE, bool PEEK>
__device__ __forceinline__ int node_step4(const SceneView& sv, const Trav& t, int node, const TStack& ts, int& sp,
                                          TraceStats& st) {
    if (STATS) count_node(st, t.in_blas, node);
    float4 f[7];
    load_node<7, NS, TREE>(sv, node, f); // see node_step2
    const int top = tpeek_opt<SPILL, PEEK>(ts, sp);
    const float4 lx = f[0], hx = f[1], ly = f[2], hy = f[3], lz = f[4], hz = f[5];
    const int4 r = as_int4(f[6]);
    float d[4];
    int ref[4] = {r.x, r.y, r.z, r.w};
    const float LX[4] = {lx.x, lx.y, lx.z, lx.w}, HX[4] = {hx.x, hx.y, hx.z, hx.w};
    const float LY[4] = {ly.x, ly.y, ly.z, ly.w}, HY[4] = {hy.x, hy.y, hy.z, hy.w};
    const float LZ[4] = {lz.x, lz.y, lz.z, lz.w}, HZ[4] = {hz.x, hz.y, hz.z, hz.w};
    int n = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float nx, fx, ny, fy, nz, fz;
        slab4(LX[k], HX[k], t.idir.x, t.iorg.x, nx, fx);
        slab4(LY[k], HY[k], t.idir.y, t.iorg.y, ny, fy);
        slab4(LZ[k], HZ[k], t.idir.z, t.iorg.z, nz, fz);
        float en = fmaxf(fmaxf(nx, ny), fmaxf(nz, t.tmin));
        float ex = fminf(fminf(fx, fy), fminf(fz, t.tmax));
        bool h = en <= ex;
        d[k] = h ? en : INFINITY;
        n += h ? 1 : 0;
    }
    if (n == 0) return tpop_peeked<SPILL, PEEK>(ts, sp, top);
    cswap(d[0], ref[0], d[1], ref[1]);
    cswap(d[2], ref[2], d[3], ref[3]);
    cswap(d[0], ref[0], d[2], ref[2]);
    cswap(d[1], ref[1], d[3], ref[3]);
    cswap(d[1], ref[1], d[2], ref[2]);
    tpush_hits3<SPILL>(ts, sp, n, ref[1], ref[2], ref[3]);
    return ref[0];
}

// Quantised 4-wide node (64 B, host Bvh4QNode): per axis an origin and a
// power-of-two scale, child bounds as bytes.  The slab distance of code q on
// axis a is fma(q, s_a * idir_a, fma(o_a, idir_a, iorg_a)); the boxes carry at
// least half a quantum of slack (quantize_bvh4) and the exit distance is
// widened by QSLAB_EXIT_WIDEN, so every ray the exact box accepts is accepted
// here.  Absent children (kEmptyRef) are masked by ref.
template <bool STATS, bool SPILL, bool TREE, bool PEEK>
__device__ __forceinline__ int node_step4q(const SceneView& sv, const Trav& t, int node, const TStack& ts, int& sp,
                                           TraceStats& st) {
    if (STATS) count_node(st, t.in_blas, node);
    float4 f[4];
    load_node<4, 4, TREE>(sv, node, f); // see node_step2
    const int top = tpeek_opt<SPILL, PEEK>(ts, sp);
    const float4 A = f[0], B = f[1], C = f[2];
    const int4 r = as_int4(f[3]);
    const float SX = A.w * t.idir.x, SY = B.x * t.idir.y, SZ = B.y * t.idir.z;
    const float OX = fmaf(A.x, t.idir.x, t.iorg.x), OY = fmaf(A.y, t.idir.y, t.iorg.y), OZ = fmaf(A.z, t.idir.z, t.iorg.z);
    uint32_t qlx = __float_as_uint(B.z), qhx = __float_as_uint(B.w);
    uint32_t qly = __float_as_uint(C.x), qhy = __float_as_uint(C.y);
    uint32_t qlz = __float_as_uint(C.z), qhz = __float_as_uint(C.w);
    if constexpr (IGX_ORDERED_SLAB_Q) { // near / far byte words by the sign of idir (= the sign of S*)
        const bool sx = __float_as_int(t.idir.x) < 0, sy = __float_as_int(t.idir.y) < 0, sz = __float_as_int(t.idir.z) < 0;
        const uint32_t nx = sx ? qhx : qlx, fx = sx ? qlx : qhx;
        const uint32_t ny = sy ? qhy : qly, fy = sy ? qly : qhy;
        const uint32_t nz = sz ? qhz : qlz, fz = sz ? qlz : qhz;
        qlx = nx, qhx = fx, qly = ny, qhy = fy, qlz = nz, qhz = fz;
    }
    float d[4];
    int ref[4] = {r.x, r.y, r.z, r.w};
    int n = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float ax = fmaf((float)((qlx >> (8 * k)) & 255u), SX, OX), bx = fmaf((float)((qhx >> (8 * k)) & 255u), SX, OX);
        const float ay = fmaf((float)((qly >> (8 * k)) & 255u), SY, OY), by = fmaf((float)((qhy >> (8 * k)) & 255u), SY, OY);
        const float az = fmaf((float)((qlz >> (8 * k)) & 255u), SZ, OZ), bz = fmaf((float)((qhz >> (8 * k)) & 255u), SZ, OZ);
        float en, ex;
        if constexpr (IGX_ORDERED_SLAB_Q) { // a* near, b* far
            en = fmaxf(fmaxf(ax, ay), fmaxf(az, t.tmin));
            ex = fminf(fminf(fminf(bx, by), bz) * QSLAB_EXIT_WIDEN, t.tmax);
        } else {
            en = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), t.tmin));
            ex = fminf(fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz)) * QSLAB_EXIT_WIDEN, t.tmax);
        }
        const bool h = en <= ex && ref[k] != REF_EMPTY;
        d[k] = h ? en : INFINITY;
        n += h ? 1 : 0;
    }
    if (n == 0) return tpop_peeked<SPILL, PEEK>(ts, sp, top);
    cswap(d[0], ref[0], d[1], ref[1]);
    cswap(d[2], ref[2], d[3], ref[3]);
    cswap(d[0], ref[0], d[2], ref[2]);
    cswap(d[1], ref[1], d[3], ref[3]);
    cswap(d[1], ref[1], d[2], ref[2]);
    tpush_hits3<SPILL>(ts, sp, n, ref[1], ref[2], ref[3]);
    return ref[0];
}

// stack-top peek (tpeek) in the node steps and leaves of kernels whose nodes
// come from global memory (the peek's LDS read overlaps the node fetch);
// with LDS-staged nodes it is one more LDS read per step for no latency saved.
// Round 6: soup-16M frame 55.4 -> 54.5 ms, S-deep 146.6 -> 145.9 ms, diamond
// (LDS-staged) 90.2 -> 90.9 ms with it, so it is off there.
template <int V>
constexpr bool variant_peek() { return IGX_PEEK_POP && !variant_lds_nodes(V); }
template <bool STATS, int V>
__device__ __forceinline__ int node_step(const SceneView& sv, const Trav& t, int node, const TStack& ts, int& sp,
                                         TraceStats& st) {
    constexpr bool PK = variant_peek<V>();
    if constexpr (variant_q4(V)) return node_step4q<STATS, variant_spill(V), variant_tree(V), PK>(sv, t, node, ts, sp, st);
    else if constexpr (variant_width(V) == 4) return node_step4<STATS, variant_spill(V), 8, variant_tree(V), PK>(sv, t, node, ts, sp, st);
    else return node_step2<STATS, variant_spill(V), 4, variant_tree(V), PK>(sv, t, node, ts, sp, st);
}

// Back from a BLAS: restore the world ray (recomputed: cheaper than keeping
// six more registers live through the whole traversal).
__device__ __forceinline__ void leave_blas(Trav& t) {
    t.lo = t.o;
    t.ld = t.d;
    t.idir = mk(safe_rcp(t.d.x), safe_rcp(t.d.y), safe_rcp(t.d.z));
    t.iorg = mk(-(t.o.x * t.idir.x), -(t.o.y * t.idir.y), -(t.o.z * t.idir.z));
    t.in_blas = false;
}

// Test TLAS leaf slot `slot`: analytic sphere hit, or entry into the entity's
// BLAS (returns true and sets `blas_root`; the ray moves to entity space).
template <bool STATS>
__device__ __forceinline__ bool instance_test(const SceneView& sv, Trav& t, int slot, int& blas_root, TraceStats& st) {
    if (STATS) st.leaves++;
    const float4* ip = sv.inst + 4 * slot;
    int4 info = *reinterpret_cast<const int4*>(ip + 3);
    uint32_t ef = (uint32_t)info.w;
    if ((t.rflags & RAY_TYPE_MASK) != ((t.rflags & ef) & RAY_TYPE_MASK)) return false; // check_ray_visibility
    // the shortcuts take the world direction as the entity-space one; a zero
    // component keeps its sign there, while transform_ray's 1*d + 0*d' + 0*d''
    // may turn -0 into +0 (and safe_rcp then gives +FLT_MAX, not -FLT_MAX):
    // such rays take the general transform
    const bool exact_dir = shortcut_dir_ok(t.d);
    if (IGX_IDENTITY_INSTANCES && (ef & INST_IDENTITY) && exact_dir) {
        // identity to_local: t.lo / t.ld / t.idir / t.iorg already hold the
        // world ray of the TLAS walk
        if (STATS) st.blas++;
        t.cur_ent = info.x;
        t.in_blas = true;
        blas_root = info.z;
        return true;
    }
    if (IGX_TRANSLATE_INSTANCES && (ef & INST_TRANSLATE) && exact_dir) {
        // transform_ray with a translation: ((1*o.x + 0*o.y) + 0*o.z) + tx is o.x + tx
        if (STATS) st.blas++;
        t.lo = mk(t.o.x + ip[0].w, t.o.y + ip[1].w, t.o.z + ip[2].w);
        t.iorg = mk(-(t.lo.x * t.idir.x), -(t.lo.y * t.idir.y), -(t.lo.z * t.idir.z));
        t.cur_ent = info.x;
        t.in_blas = true;
        blas_root = info.z;
        return true;
    }
    float4 m0 = ip[0], m1 = ip[1], m2 = ip[2];
    const f3 o = t.o, d = t.d;
    // transform_ray (ray.art:53-59): point and direction, no renormalisation
    f3 lo2 = mk(m0.x * o.x + m0.y * o.y + m0.z * o.z + m0.w,
                m1.x * o.x + m1.y * o.y + m1.z * o.z + m1.w,
                m2.x * o.x + m2.y * o.y + m2.z * o.z + m2.w);
    f3 ld2 = mk(m0.x * d.x + m0.y * d.y + m0.z * d.z,
                m1.x * d.x + m1.y * d.y + m1.z * d.z,
                m2.x * d.x + m2.y * d.y + m2.z * d.z);
    if (info.y == 1) {
        // analytic sphere in entity space (intersect_sphere, shapes/sphere.art:104-130)
        float4 sph = sv.spheres[info.z];
        f3 L = sub(lo2, f3of(sph));
        float S = -dot(L, ld2);
        float D2 = dot(ld2, ld2);
        float L2 = dot(L, L);
        float R2 = sph.w * sph.w * D2;
        float M2 = L2 * D2 - S * S;
        if (!(S < 0 || M2 > R2)) {
            float Q = sqrtf(R2 - M2);
            float ta = (S - Q) / D2, tb = (S + Q) / D2;
            float t0 = ta > tb ? tb : ta, t1 = ta > tb ? ta : tb;
            float th = t0 < t.tmin ? t1 : t0;
            if (accept_hit(t, th, info.x, 0)) {
                t.tmax = th;
                t.hit_ent = info.x;
                t.hit_prim = 0;
                // prim coords are only texture coordinates for spheres; not needed downstream
                t.hu = 0;
                t.hv = 0;
                t.found = true;
            }
        }
        return false;
    }
    if (STATS) st.blas++;
    t.lo = lo2;
    t.ld = ld2;
    t.idir = mk(safe_rcp(ld2.x), safe_rcp(ld2.y), safe_rcp(ld2.z));
    t.iorg = mk(-(lo2.x * t.idir.x), -(lo2.y * t.idir.y), -(lo2.z * t.idir.z));
    t.cur_ent = info.x;
    t.in_blas = true;
    blas_root = info.z;
    return true;
}

// Moeller-Trumbore against triangle slot `slot` in the current BLAS
// (make_gpu_tri_prim, shapes/trimesh.art:124-160; intersection.art:71-101).
template <bool STATS>
__device__ __forceinline__ void tri_test(const SceneView& sv, Trav& t, int slot, TraceStats& st) {
    if (STATS) st.tris++;
    const float4* tp = sv.tris + 3 * slot;
    float4 q0 = tp[0], q1 = tp[1], q2 = tp[2];
    f3 v0 = f3of(q0), e1 = f3of(q1), e2 = f3of(q2);
    f3 n = cross(e1, e2);
    f3 cc = sub(v0, t.lo);
    f3 rr = cross(t.ld, cc);
    float det = dot(n, t.ld);
    float inv_det = 1.0f / det;
    float u = dot(rr, e2) * inv_det;
    float v = dot(rr, e1) * inv_det;
    float w = 1 - u - v;
    bool ok = u >= -FLT_EPS_ && v >= -FLT_EPS_ && w >= -FLT_EPS_;
    if (ok) {
        float th = dot(cc, n) * inv_det;
        int prim = __float_as_int(q0.w);
        if (accept_hit(t, th, t.cur_ent, prim)) {
            t.tmax = th;
            t.hit_ent = t.cur_ent;
            t.hit_prim = prim;
            t.hu = u > 0 ? u : 0;
            t.hv = v > 0 ? v : 0;
            t.found = true;
        }
    }
}

// One traversal step (while-while): inner nodes down to a leaf, then that
// leaf or the BLAS return marker.  Returns true once the ray is finished
// (stack exhausted, or the first hit for any-hit rays).  ANYM: 0 closest
// hit, 1 any hit, 2 per lane (`any_rt`), so that closest-hit and any-hit rays
// of one wave step through the same instructions (k_finish_pairs).
template <int ANYM, bool STATS, int V>
__device__ __forceinline__ bool trav_step_core(const SceneView& sv, Trav& t, const TStack& ts, TraceStats& st, bool any_rt) {
    const bool ANY = ANYM == 2 ? any_rt : ANYM == 1;
    int node = t.node;
    int sp = t.sp;
    constexpr bool SPILL = variant_spill(V);
    if constexpr (variant_ifif(V)) {
        // if-if: one inner node per call, so a lane that reached a leaf does
        // not idle until every lane of the wave has reached one
        if (node >= 0) {
            t.node = node_step<STATS, V>(sv, t, node, ts, sp, st);
            t.sp = sp;
            return false;
        }
    } else {
        while (node >= 0) node = node_step<STATS, V>(sv, t, node, ts, sp, st);
    }
    if (node == REF_EXIT) {
        t.node = node;
        t.sp = sp;
        return true;
    }
    if (STATS && first_active_lane()) st.wleaves++;
    // every leaf and marker ends in a pop (or an instance's BLAS entry): its
    // entry is read with the leaf's first loads (tpeek)
    constexpr bool PK = variant_peek<V>();
    const int top = tpeek_opt<SPILL, PK>(ts, sp);
    if (node == REF_MARKER) {
        leave_blas(t);
        t.node = tpop_peeked<SPILL, PK>(ts, sp, top);
        t.sp = sp;
        return false;
    }
    int code = ~node;
    int first = code >> LEAF_COUNT_BITS;
    int count = (code & ((1 << LEAF_COUNT_BITS) - 1)) + 1;
    if (!t.in_blas) {
        // TLAS leaf: entity instances (one per leaf as built here)
        int root = 0;
        bool entered = false;
#pragma unroll 1
        for (int k = 0; k < count && !entered; ++k) {
            entered = instance_test<STATS>(sv, t, first + k, root, st);
            if (ANY && t.found) {
                t.node = REF_EXIT;
                t.sp = sp;
                return true;
            }
        }
        if (entered) {
            tpush<SPILL>(ts, sp, REF_MARKER);
            t.node = root;
        } else {
            t.node = tpop_peeked<SPILL, PK>(ts, sp, top);
        }
    } else {
#pragma unroll 1
        for (int k = 0; k < count; ++k) {
            tri_test<STATS>(sv, t, first + k, st);
            if (ANY && t.found) {
                t.node = REF_EXIT;
                t.sp = sp;
                return true;
            }
        }
        t.node = tpop_peeked<SPILL, PK>(ts, sp, top);
    }
    t.sp = sp;
    return false;
}

template <bool ANY, bool STATS, int V>
__device__ __forceinline__ bool trav_step(const SceneView& sv, Trav& t, const TStack& ts, TraceStats& st) {
    return trav_step_core<ANY ? 1 : 0, STATS, V>(sv, t, ts, st, false);
}

// Whole-ray traversal (used by the tail kernel and the hit-level harness).
template <bool ANY, bool STATS, int V>
__device__ __forceinline__ bool trace_ray(const SceneView& sv, f3 o, f3 d, float tmin, float& tmax, uint32_t rflags,
                                          const TStack& ts, int& hit_ent, int& hit_prim, float& hu, float& hv,
                                          TraceStats& st) {
    Trav t;
    trav_init(sv, t, o, d, tmin, tmax, rflags, ts);
    while (!trav_step<ANY, STATS, V>(sv, t, ts, st)) {
    }
    tmax = t.tmax;
    hit_ent = t.hit_ent;
    hit_prim = t.hit_prim;
    hu = t.hu;
    hv = t.hv;
    return t.found;
}

// Closest hit of a ray that travels inside enclosing entity number `enc` (a closed,
// non-thin dielectric mesh whose world box keeps a margin from every other
// entity's box, igx_upload_scene).  The ray starts on the entity's surface,
// i.e. in its box; along the ray the box is one interval from the start, every
// hit on the entity lies in it and every other entity lies beyond it.  So a
// hit the entity's BLAS finds is the closest hit of the whole scene -- the
// same (t, u, v) the full traversal computes, from the same entity-space ray
// (instance_test's transform).  Returns false (nothing written) when the
// entity is not visible to the ray or its BLAS yields no hit; the caller then
// traces the ray from the TLAS root.
// Traversal state of trace_enclosed's BLAS-only walk; false when the entity
// is not visible to the ray (nothing to walk).
template <bool STATS>
__device__ __forceinline__ bool trav_init_enclosed(const SceneView& sv, Trav& t, int enc, f3 o, f3 d, float tmin, float tmax,
                                                   uint32_t rflags, const TStack& ts, TraceStats& st) {
    const int slot = sv.enc[enc].y;
    const float4* ip = sv.inst + 4 * slot;
    const int4 info = *reinterpret_cast<const int4*>(ip + 3);
    if ((rflags & RAY_TYPE_MASK) != ((rflags & (uint32_t)info.w) & RAY_TYPE_MASK)) return false;
    t.o = o;
    t.d = d;
    const bool exact_dir = shortcut_dir_ok(d); // see instance_test
    if (IGX_IDENTITY_INSTANCES && ((uint32_t)info.w & INST_IDENTITY) && exact_dir) { // as instance_test
        t.lo = o;
        t.ld = d;
    } else if (IGX_TRANSLATE_INSTANCES && ((uint32_t)info.w & INST_TRANSLATE) && exact_dir) {
        t.lo = mk(o.x + ip[0].w, o.y + ip[1].w, o.z + ip[2].w);
        t.ld = d;
    } else {
        const float4 m0 = ip[0], m1 = ip[1], m2 = ip[2];
        t.lo = mk(m0.x * o.x + m0.y * o.y + m0.z * o.z + m0.w, m1.x * o.x + m1.y * o.y + m1.z * o.z + m1.w,
                  m2.x * o.x + m2.y * o.y + m2.z * o.z + m2.w);
        t.ld = mk(m0.x * d.x + m0.y * d.y + m0.z * d.z, m1.x * d.x + m1.y * d.y + m1.z * d.z, m2.x * d.x + m2.y * d.y + m2.z * d.z);
    }
    t.idir = mk(safe_rcp(t.ld.x), safe_rcp(t.ld.y), safe_rcp(t.ld.z));
    t.iorg = mk(-(t.lo.x * t.idir.x), -(t.lo.y * t.idir.y), -(t.lo.z * t.idir.z));
    t.tmin = tmin;
    t.tmax = fminf(tmax, FLT_MAX_); // see trav_init
    t.rflags = rflags;
    t.cur_ent = info.x;
    t.hit_ent = -1;
    t.hit_prim = -1;
    t.hu = 0;
    t.hv = 0;
    t.in_blas = true;
    t.found = false;
    ts.lds[0] = REF_EXIT;
    t.sp = 1;
    t.node = info.z; // BLAS root (or its only leaf)
    if (STATS) { st.leaves++; st.blas++; }
    return true;
}
template <bool STATS, int V>
__device__ __forceinline__ bool trace_enclosed(const SceneView& sv, int enc, f3 o, f3 d, float tmin, float& tmax,
                                               uint32_t rflags, const TStack& ts, int& hit_ent, int& hit_prim, float& hu,
                                               float& hv, TraceStats& st) {
    Trav t;
    if (!trav_init_enclosed<STATS>(sv, t, enc, o, d, tmin, tmax, rflags, ts, st)) return false;
    while (!trav_step<false, STATS, V>(sv, t, ts, st)) {
    }
    if (!t.found) return false;
    tmax = t.tmax;
    hit_ent = t.hit_ent;
    hit_prim = t.hit_prim;
    hu = t.hu;
    hv = t.hv;
    return true;
}

// Closest hit of a path's ray: rays inside enclosing entity `inside` (>= 0)
// walk that entity's BLAS first (trace_enclosed), the rest from the TLAS
// root -- in ONE loop, so that a wave holding both kinds steps them together
// (two loops one after the other ran the wave's enclosed lanes and then its
// other lanes, each half idle).  An enclosed walk that finds nothing falls back
// to the full traversal (rare: a ray grazing out through a crack).
template <bool STATS, int V>
__device__ __forceinline__ void trace_path_ray(const SceneView& sv, int inside, f3 o, f3 d, float tmin, float& tmax,
                                               uint32_t rflags, const TStack& ts, int& hit_ent, int& hit_prim, float& hu,
                                               float& hv, TraceStats& st) {
    Trav t;
    bool enclosed = inside >= 0 && trav_init_enclosed<STATS>(sv, t, inside, o, d, tmin, tmax, rflags, ts, st);
    if (!enclosed) trav_init(sv, t, o, d, tmin, tmax, rflags, ts);
    for (;;) {
        while (!trav_step<false, STATS, V>(sv, t, ts, st)) {
        }
        if (!enclosed || t.found) break;
        trav_init(sv, t, o, d, tmin, tmax, rflags, ts);
        enclosed = false;
    }
    tmax = t.tmax;
    hit_ent = t.hit_ent;
    hit_prim = t.hit_prim;
    hu = t.hu;
    hv = t.hv;
}

// Persistent lanes with ray refill (Aila & Laine, "Understanding the
// efficiency of ray traversal on GPUs", 2009): a wave walks a sequence of C
// ray positions; a lane whose ray is finished goes idle, and once at least
// `refill_min` lanes are idle (or all are) the idle lanes take the next rays
// of the sequence, so waves stop running long stretches with a handful of
// active lanes.  seq.reserve(cursor, m) (wave-uniform) readies the next m
// positions and is false once the sequence is exhausted; seq.at(c, i) maps
// position c to a stream index (false: nothing there).
// fetch(i, t) -> bool loads ray i into t (false: nothing to trace);
// finish(i, t) consumes a finished ray.
template <bool ANY, bool STATS, int V, typename Seq, typename Fetch, typename Finish>
__device__ __forceinline__ void refill_loop(const SceneView& sv, const TStack& ts, Seq& seq, int refill_min, Fetch fetch,
                                            Finish finish, TraceStats& st) {
    const int lane = (int)__lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    int cursor = 0; // wave-uniform
    bool more = true; // wave-uniform: the sequence is not yet exhausted
    bool busy = false;
    int pos = 0;
    Trav t;
    for (;;) {
        const uint64_t idle = __ballot(!busy);
        const int nidle = __popcll(idle);
        if (more && (nidle >= refill_min || nidle == 64)) more = seq.reserve(cursor, nidle);
        if (more && (nidle >= refill_min || nidle == 64)) {
            if (!busy) {
                const int c = cursor + __popcll(idle & below);
                if (seq.at(c, pos)) busy = fetch(pos, t);
            }
            cursor += nidle;
        } else if (nidle == 64) {
            break; // sequence exhausted, nothing in flight
        }
        if (busy && trav_step<ANY, STATS, V>(sv, t, ts, st)) {
            finish(pos, t);
            busy = false;
        }
    }
}

// ---------------------------------------------------------------------------
// Surface element (shapes/trimesh.art:14-39, shapes/sphere.art:50-64)
// ---------------------------------------------------------------------------
struct Surface {
    f3 point;
    f3 face_normal;
    Frame local;
    bool entering;
};

__device__ __forceinline__ f3 xform_point_rows(float4 r0, float4 r1, float4 r2, f3 p) {
    return mk(r0.x * p.x + r0.y * p.y + r0.z * p.z + r0.w, r1.x * p.x + r1.y * p.y + r1.z * p.z + r1.w,
              r2.x * p.x + r2.y * p.y + r2.z * p.z + r2.w);
}
__device__ __forceinline__ f3 xform_dir_rows(float4 r0, float4 r1, float4 r2, f3 p) {
    return mk(r0.x * p.x + r0.y * p.y + r0.z * p.z, r1.x * p.x + r1.y * p.y + r1.z * p.z,
              r2.x * p.x + r2.y * p.y + r2.z * p.z);
}

__device__ __forceinline__ Surface surface_element(const SceneView& sv, int ent_id, int prim, float t, float hu, float hv,
                                                   f3 ro, f3 rd, int& material) {
    const float4* ep = sv.ent + ENT_STRIDE * ent_id;
    float4 g0 = ep[0], g1 = ep[1], g2 = ep[2];
    float4 n0 = ep[3], n1 = ep[4], n2 = ep[5];
    int4 info = *reinterpret_cast<const int4*>(ep + 6); // shape type, material, vtx_off, idx_off|sphere
    material = info.y;
    Surface s;
    s.point = add(ro, mulf(rd, t));
    if (info.x == 1) {
        float4 sph = sv.spheres[info.w];
        f3 dir = sub(s.point, xform_point_rows(g0, g1, g2, f3of(sph)));
        float l = len(dir);
        f3 nrm = mulf(dir, 1 / l);
        s.entering = true;
        s.face_normal = nrm;
        s.local = make_frame(nrm);
        return s;
    }
    if (sv.fsh) {
        // the face's shading record: vertex normals and indices (fsh), the
        // entity's face-normal offset in row 3 .w; the same values as the
        // index / normal tables give, so the same bits
        const float4* fr = sv.fsh + 3 * (info.w + prim);
        const float4 r0 = fr[0], r1 = fr[1], r2 = fr[2];
        f3 fn;
        if (sv.fn_tab) {
            fn = f3of(sv.fn_tab[__float_as_int(n0.w) + prim]);
        } else {
            f3 v0 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + __float_as_int(r0.w)]));
            f3 v1 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + __float_as_int(r1.w)]));
            f3 v2 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + __float_as_int(r2.w)]));
            f3 e1 = sub(v1, v0), e2 = sub(v2, v0);
            f3 n = cross(e1, e2);
            float nn = len(n);
            fn = mulf(n, 1 / nn);
        }
        f3 ln = lerp2(f3of(r0), f3of(r1), f3of(r2), hu, hv);
        f3 normal = normalize(xform_dir_rows(n0, n1, n2, ln));
        s.entering = dot(rd, fn) <= 0;
        s.face_normal = s.entering ? fn : neg(fn);
        s.local = make_frame(s.entering ? normal : neg(normal));
        return s;
    }
    int4 f = sv.idx[info.w + prim];
    f3 fn;
    if (sv.fn_tab) {
        // the upload computed the same make_triangle normal on the host
        fn = f3of(sv.fn_tab[sv.ent_fn[ent_id] + prim]);
    } else {
        f3 v0 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + f.x]));
        f3 v1 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + f.y]));
        f3 v2 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + f.z]));
        // make_triangle (core/triangle.art:11-26)
        f3 e1 = sub(v1, v0), e2 = sub(v2, v0);
        f3 n = cross(e1, e2);
        float nn = len(n);
        fn = mulf(n, 1 / nn);
    }
    f3 ln = lerp2(f3of(sv.nrm[info.z + f.x]), f3of(sv.nrm[info.z + f.y]), f3of(sv.nrm[info.z + f.z]), hu, hv);
    f3 normal = normalize(xform_dir_rows(n0, n1, n2, ln));
    s.entering = dot(rd, fn) <= 0;
    s.face_normal = s.entering ? fn : neg(fn);
    s.local = make_frame(s.entering ? normal : neg(normal));
    return s;
}

// ---------------------------------------------------------------------------
// Lights
// ---------------------------------------------------------------------------
// compute_sq of make_plane_area_emitter (light/area.art:127-176)
struct SQ {
    f3 o, n;
    float x0, y0, z0, x1, y1, b0, b1, k, s;
};
__device__ __forceinline__ float safe_acos(float a) { return acosf(clampf(a, -1, 1)); }
__device__ __forceinline__ SQ compute_sq(const DevLight& L, f3 from) {
    f3 origin = mk(L.origin[0], L.origin[1], L.origin[2]);
    f3 ex = mk(L.ex[0], L.ex[1], L.ex[2]);
    f3 ey = mk(L.ey[0], L.ey[1], L.ey[2]);
    f3 normal = mk(L.normal[0], L.normal[1], L.normal[2]);
    float width = L.origin[3], height = L.ex[3];
    f3 dir = sub(origin, from);
    SQ q;
    q.x0 = dot(dir, ex);
    q.y0 = dot(dir, ey);
    float z0_ = dot(dir, normal);
    q.x1 = q.x0 + width;
    q.y1 = q.y0 + height;
    bool nsb = !signbit(z0_);
    q.z0 = nsb ? -z0_ : z0_;
    q.n = nsb ? neg(normal) : normal;
    // diff = (x0, y1, x1, y0) - (x1, y0, x0, y1); nz_ = (y0, x1, y1, x0) * diff
    float dx = q.x0 - q.x1, dy = q.y1 - q.y0, dz = q.x1 - q.x0, dw = q.y0 - q.y1;
    float zx = q.y0 * dx, zy = q.x1 * dy, zz = q.y1 * dz, zw = q.x0 * dw;
    float z02 = q.z0 * q.z0;
    float nzx = zx / sqrtf((dx * dx) * z02 + zx * zx);
    float nzy = zy / sqrtf((dy * dy) * z02 + zy * zy);
    float nzz = zz / sqrtf((dz * dz) * z02 + zz * zz);
    float nzw = zw / sqrtf((dw * dw) * z02 + zw * zw);
    float g0 = safe_acos(-nzx * nzy);
    float g1 = safe_acos(-nzy * nzz);
    float g2 = safe_acos(-nzz * nzw);
    float g3 = safe_acos(-nzw * nzx);
    q.b0 = nzx;
    q.b1 = nzz;
    q.k = 2 * PI_ - g2 - g3;
    q.s = g0 + g1 - q.k;
    q.o = from;
    return q;
}

// square_to_concentric_disk (core/warp.art:2-22)
__device__ __forceinline__ void concentric_disk(float u, float v, float& x, float& y) {
    float a = 2 * u - 1, b = 2 * v - 1;
    if (a == 0 && b == 0) {
        x = 0;
        y = 0;
    } else if (a * a > b * b) {
        float phi = (PI_ / 4) * safe_div(b, a);
        x = cosf(phi) * a;
        y = sinf(phi) * a;
    } else {
        float phi = (PI_ / 2) - (PI_ / 4) * safe_div(a, b);
        x = cosf(phi) * b;
        y = sinf(phi) * b;
    }
}
struct DirectSample {
    f3 pos, dir;
    f3 intensity;
    float pdf_value;
    bool pdf_solid; // measure of pdf_value: solid angle or area
    float cos, dist;
};

__device__ __forceinline__ float pdf_as_solid(float value, bool solid, float cos, float dist2) {
    return solid ? value : value * dist2 / cos; // driver/pdf.art:15-32
}

// Light::sample_direct for the light types on the hot path
template <bool FULL>
__device__ __forceinline__ DirectSample light_sample_direct(const SceneView& sv, const DevLight& L, Rng& rnd,
                                                            const Surface& from) {
    DirectSample ds;
    f3 rad = mk(L.radiance[0], L.radiance[1], L.radiance[2]);
    if (L.type == LIGHT_PLANE) {
        // make_area_light.sample_direct (light/area.art:10-27) + plane sampler (area.art:178-224)
        float ux = rnd.next_f32();
        float uy = rnd.next_f32();
        SQ q = compute_sq(L, from.point);
        f3 ex = mk(L.ex[0], L.ex[1], L.ex[2]);
        f3 ey = mk(L.ey[0], L.ey[1], L.ey[2]);
        float au = fmaf(ux, q.s, q.k);
        float fu = fmaf(cosf(au), q.b0, -q.b1) / sinf(au);
        float cu = clampf(copysignf(1.0f, fu) / sqrtf(sum_of_prod(fu, fu, q.b0, q.b0)), -1, 1);
        float xu = clampf(-(cu * q.z0) / sqrtf(fmaf(-cu, cu, 1.0f)), q.x0, q.x1);
        float dd = sqrtf(sum_of_prod(xu, xu, q.z0, q.z0));
        float h0 = q.y0 / sqrtf(sum_of_prod(dd, dd, q.y0, q.y0));
        float h1 = q.y1 / sqrtf(sum_of_prod(dd, dd, q.y1, q.y1));
        float hv = fmaf(uy, h1 - h0, h0);
        float hv2 = hv * hv;
        float yv = hv2 < 1 - 1e-6f ? (hv * dd) / sqrtf(1 - hv2) : q.y1;
        f3 p = add(q.o, add(mulf(ex, xu), add(mulf(ey, yv), mulf(q.n, q.z0))));
        float pdf_s = safe_div(1, q.s);
        f3 dir_ = sub(p, from.point);
        float dist = len(dir_);
        f3 dir = mulf(dir_, safe_div(1, dist));
        f3 normal = mk(L.normal[0], L.normal[1], L.normal[2]);
        ds.pos = p;
        ds.dir = dir;
        ds.intensity = mulf(rad, q.s);
        ds.pdf_value = pdf_s;
        ds.pdf_solid = true;
        ds.cos = dot(dir, normal) * (from.entering ? -1.0f : 1.0f);
        ds.dist = dist;
    } else if (L.type == LIGHT_ENV) {
        // make_environment_light_function_spherical.sample_direct (light/env.art:80-84)
        float ux = rnd.next_f32();
        float uy = rnd.next_f32();
        f3 dir = equal_area_square_to_sphere(ux, uy);
        float pdf = 1 / (4 * PI_);
        ds.intensity = mulf(rad, 1 / pdf);
        ds.pos = add(from.point, mulf(dir, sv.scene_radius));
        ds.dir = dir;
        ds.pdf_value = pdf;
        ds.pdf_solid = true;
        ds.cos = 1.0f;
        ds.dist = sv.scene_radius;
    } else if (L.type == LIGHT_DIRECTIONAL) {
        // make_directional_light.sample_direct (light/directional.art:6): delta pdf, cos 1
        f3 dir = mk(L.normal[0], L.normal[1], L.normal[2]);
        ds.pos = add(from.point, mulf(dir, -sv.scene_radius));
        ds.dir = neg(dir);
        ds.intensity = rad;
        ds.pdf_value = 1;
        ds.pdf_solid = true; // delta: as_solid = 1
        ds.cos = 1;
        ds.dist = sv.scene_radius;
    } else if (L.type == LIGHT_SUN) {
        // make_sun_light.sample_direct (light/sun.art:10-14) with sample_uniform_cone
        // (core/sampling.art:106-116) in make_orthonormal_mat3x3(dir)
        const float cos_angle = L.spot[0], sun_area = L.spot[1];
        float u = rnd.next_f32();
        float v = rnd.next_f32();
        float c1 = 1 - cos_angle;
        float px, py;
        concentric_disk(u, v, px, py);
        float n2 = px * px + py * py;
        float z = cos_angle + c1 * (1 - n2);
        float sc = safe_sqrt(c1 * (2 - c1 * n2));
        float pdf = safe_div_one(1, 2 * PI_ * (1 - cos_angle));
        f3 ndir = frame_to_world(make_frame(mk(L.normal[0], L.normal[1], L.normal[2])), mk(px * sc, py * sc, z));
        ds.pos = mk(0, 0, 0);
        ds.dir = neg(ndir);
        ds.intensity = mulf(rad, 1 / (sun_area * pdf));
        ds.pdf_value = 1;
        ds.pdf_solid = true;
        ds.cos = z;
        ds.dist = INFINITY;
    } else if (FULL && (L.type == LIGHT_SPHERE || L.type == LIGHT_MESH)) {
        // make_area_light.sample_direct (light/area.art:12-27) over the sphere emitter
        // (area.art:248-274) or the triangle-shape emitter (area.art:48-57)
        float ux = rnd.next_f32();
        float uy = rnd.next_f32();
        const float4* ep = sv.ent + ENT_STRIDE * L.entity;
        float4 g0 = ep[0], g1 = ep[1], g2 = ep[2];
        f3 p, fn;
        float pdf_a, weight;
        if (L.type == LIGHT_SPHERE) {
            float4 n0 = ep[3], n1 = ep[4], n2 = ep[5];
            f3 so = mk(L.origin[0], L.origin[1], L.origin[2]);
            float r = L.origin[3];
            float inv_area = 1 / L.spot[0];
            f3 glb_org = xform_point_rows(g0, g1, g2, so);
            f3 nrm = equal_area_square_to_sphere(ux, uy);
            p = xform_point_rows(g0, g1, g2, add(so, mulf(nrm, r)));
            fn = normalize(xform_dir_rows(n0, n1, n2, nrm));
            f3 os = sub(from.point, glb_org), pq = sub(from.point, p);
            if (!(dot(pq, pq) <= dot(os, os))) { // keep the point on the visible side
                f3 op = sub(p, glb_org);
                f3 np = sub(p, mulf(op, 2));
                f3 nn = normalize(sub(np, glb_org));
                p = xform_point_rows(g0, g1, g2, add(so, mulf(nn, r)));
                fn = normalize(xform_dir_rows(n0, n1, n2, nn));
            }
            pdf_a = 2 * inv_area;
            weight = 1 / (2 * inv_area);
        } else {
            int4 info = *reinterpret_cast<const int4*>(ep + 6);
            float cnt = L.spot[0];
            float uxc = ux * cnt;
            int f = min((int)uxc, (int)cnt - 1);
            float su = uxc - (float)f, sw = uy;
            if (su + sw > 1) { su = 1 - su; sw = 1 - sw; } // sample_triangle (core/sampling.art:34-36)
            int4 fi = sv.idx[info.w + f];
            f3 v0 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + fi.x]));
            f3 v1 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + fi.y]));
            f3 v2 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + fi.z]));
            f3 n = cross(sub(v1, v0), sub(v2, v0));
            float nn = len(n);
            fn = mulf(n, 1 / nn);
            float inv_area = 1 / (nn / 2);
            p = lerp2(v0, v1, v2, su, sw);
            pdf_a = inv_area / cnt;
            weight = cnt / inv_area;
        }
        f3 dir_ = sub(p, from.point);
        float dist = len(dir_);
        f3 dir = mulf(dir_, safe_div(1, dist));
        ds.pos = p;
        ds.dir = dir;
        ds.intensity = mulf(rad, weight);
        ds.pdf_value = pdf_a;
        ds.pdf_solid = false;
        ds.cos = dot(dir, fn) * (from.entering ? -1.0f : 1.0f);
        ds.dist = dist;
    } else if (L.type == LIGHT_POINT) {
        // make_point_light.sample_direct (light/point.art:3-8)
        f3 pos = mk(L.origin[0], L.origin[1], L.origin[2]);
        f3 dir_ = sub(pos, from.point);
        float dist = len(dir_);
        ds.dir = mulf(dir_, safe_div(1, dist));
        ds.pos = pos;
        ds.intensity = rad;
        ds.pdf_value = 1;
        ds.pdf_solid = false;
        ds.cos = 1;
        ds.dist = dist;
    } else {
        // make_spot_light.sample_direct (light/spot.art:27-36)
        f3 pos = mk(L.origin[0], L.origin[1], L.origin[2]);
        f3 sdir = mk(L.normal[0], L.normal[1], L.normal[2]);
        f3 od_ = sub(pos, from.point);
        float dist = len(od_);
        f3 od = mulf(od_, safe_div(1, dist));
        float cos_angle = dot(neg(od), sdir);
        float cos_cut = L.spot[0], blend = L.spot[2];
        float factor = blend <= FLT_EPS_ ? (cos_angle <= cos_cut ? 0.0f : 1.0f)
                                         : [&] { float x = clampf((cos_angle - cos_cut) / blend, 0, 1); return x * x * (3 - 2 * x); }();
        ds.intensity = mulf(rad, factor);
        ds.pos = pos;
        ds.dir = od;
        ds.cos = -dot(od, sdir);
        ds.pdf_value = dot(neg(od), sdir) > cos_cut ? 1.0f : 0.0f;
        ds.pdf_solid = false;
        ds.dist = dist;
    }
    return ds;
}

// Light::pdf_direct for lights that can be hit (area: plane, sphere, mesh; env),
// in solid-angle measure.  (hu, hv) are the hit's prim_coords, which the
// shape emitter reuses as its sample coordinates (light/area.art:41, 59-67).
template <bool FULL>
__device__ __forceinline__ float light_pdf_direct_solid(const SceneView& sv, const DevLight& L, f3 ray_org, float cos,
                                                        float dist2, float hu, float hv) {
    if (L.type == LIGHT_PLANE) {
        SQ q = compute_sq(L, ray_org);
        return safe_div(1, q.s); // solid measure
    }
    if (FULL && L.type == LIGHT_SPHERE) return pdf_as_solid(2 / L.spot[0], false, cos, dist2); // area.art:282-284
    if (FULL && L.type == LIGHT_MESH) {
        const float4* ep = sv.ent + ENT_STRIDE * L.entity;
        float4 g0 = ep[0], g1 = ep[1], g2 = ep[2];
        int4 info = *reinterpret_cast<const int4*>(ep + 6);
        float cnt = L.spot[0];
        int f = min((int)(hu * cnt), (int)cnt - 1);
        int4 fi = sv.idx[info.w + f];
        f3 v0 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + fi.x]));
        f3 v1 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + fi.y]));
        f3 v2 = xform_point_rows(g0, g1, g2, f3of(sv.vtx[info.z + fi.z]));
        float inv_area = 1 / (len(cross(sub(v1, v0), sub(v2, v0))) / 2);
        (void)hv;
        return pdf_as_solid(inv_area / cnt, false, cos, dist2);
    }
    (void)cos; (void)dist2; (void)hu; (void)hv;
    return 1 / (4 * PI_); // env spherical: equal_area_sphere_pdf
}

// ---------------------------------------------------------------------------
// NEE light selection (light/light_selector.art).  Lights are ordered infinite
// first; finite light f is sv.lights[num_infinite + f].  "uniform" picks any
// light with probability 1/n; "simple" samples the finite lights by a flux
// CDF (make_cdf_light_selector, core/cdf.art:40-70) and "hierarchy" by a
// light BVH walked from the shading point (make_hierarchy_light_selector,
// light/light_hierarchy.art); with infinite lights both spend half the
// probability on picking one of those uniformly.  Light counts are
// compile-time constants in the reference's generated code, so a single
// light costs no random draw (pick_light_id, make_light_hierarchy).
// ---------------------------------------------------------------------------
constexpr int SEL_UNIFORM = 0, SEL_SIMPLE = 1, SEL_HIERARCHY = 2;

// make_cdf_1d (core/cdf.art:40-45): get(0) = 0, get(i) = cdf[i - 1]
__device__ __forceinline__ float cdf_get(const float* cdf, int i) { return i == 0 ? 0.0f : cdf[i - 1]; }
__device__ __forceinline__ int cdf_sample_discrete(const float* cdf, int n, float u, float& pdf) {
    // interval::binary_search(n + 1, get(i) <= u) (core/interval.art:7-23)
    int first = 0, len = n + 1;
    while (len > 0) {
        const int half = len / 2, middle = first + half;
        if (cdf_get(cdf, middle) <= u) {
            first = middle + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    const int off = min(clampi(first - 1, 0, n), n - 1);
    pdf = cdf_get(cdf, off + 1) - cdf_get(cdf, off);
    return off;
}

// light hierarchy entry (light_hierarchy::load_entry, light/light_hierarchy.art:24-37)
struct LhEntry {
    f3 pos, dir;
    float flux;
    int id;
    bool has_dir, is_leaf;
};
__device__ __forceinline__ LhEntry lh_load(const uint32_t* entries, int id) {
    const float4 e1 = *reinterpret_cast<const float4*>(entries + 8 * id);
    const float4 e2 = *reinterpret_cast<const float4*>(entries + 8 * id + 4);
    const int index = __float_as_int(e2.w);
    return LhEntry{mk(e1.x, e1.y, e1.z), mk(e2.x, e2.y, e2.z), fabsf(e1.w), index < 0 ? -index - 1 : index,
                   !signbit(e1.w), index >= 0};
}
// get_entry_cost / get_left_prop (light/light_hierarchy.art:39-56)
__device__ __forceinline__ float lh_cost(const LhEntry& e, f3 pos) {
    const f3 cdir = sub(e.pos, pos);
    const float dist2 = dot(cdir, cdir);
    const float cos_d = e.has_dir ? fabsf(dot(e.dir, normalize(cdir))) : 1.0f;
    return safe_div(e.flux * cos_d, dist2);
}
__device__ __forceinline__ float lh_left_prop(const LhEntry& l, const LhEntry& r, f3 pos) {
    const float cl = lh_cost(l, pos), cr = lh_cost(r, pos);
    return 1 / (1 + cr / cl);
}

// sample one finite light (id in [0, nf)) and its selection pdf among the finite lights
__device__ __forceinline__ int finite_select(const SceneView& sv, int nf, Rng& rnd, f3 from, float& pdf) {
    if (sv.selector == SEL_SIMPLE) return cdf_sample_discrete(sv.sel_cdf, nf, rnd.next_f32(), pdf);
    if (nf == 1) { // make_light_hierarchy, single light (light_hierarchy.art:104-108)
        pdf = 1.0f;
        return 0;
    }
    const uint32_t* data = sv.sel_tree + ((nf + 3) & ~3); // sample_light_id (light_hierarchy.art:63-78)
    float p = 1.0f;
    LhEntry e = lh_load(data, 0);
    while (!e.is_leaf) {
        const LhEntry l = lh_load(data, e.id), r = lh_load(data, e.id + 1);
        const float prop = lh_left_prop(l, r, from);
        const bool is_left = rnd.next_f32() < prop;
        e = is_left ? l : r;
        p *= is_left ? prop : 1 - prop;
    }
    pdf = p;
    return e.id;
}
__device__ __forceinline__ float finite_select_pdf(const SceneView& sv, int nf, int f, f3 from) {
    if (sv.selector == SEL_SIMPLE) return cdf_get(sv.sel_cdf, f + 1) - cdf_get(sv.sel_cdf, f);
    if (nf == 1) return 1.0f;
    uint32_t code = sv.sel_tree[f]; // compute_pdf (light_hierarchy.art:80-97)
    const uint32_t* data = sv.sel_tree + ((nf + 3) & ~3);
    float p = 1.0f;
    LhEntry e = lh_load(data, 0);
    while (!e.is_leaf) {
        const LhEntry l = lh_load(data, e.id), r = lh_load(data, e.id + 1);
        const float prop = lh_left_prop(l, r, from);
        const bool is_left = (code & 0x1u) == 0;
        e = is_left ? l : r;
        p *= is_left ? prop : 1 - prop;
        code >>= 1;
    }
    return p;
}

// LightSelector::sample: light index and selection pdf
__device__ __forceinline__ int select_light(const SceneView& sv, Rng& rnd, f3 from, float& pdf) {
    const int n = sv.num_lights, ninf = sv.num_infinite, nf = n - ninf;
    if (sv.selector == SEL_UNIFORM) { // make_uniform_light_selector (light_selector.art:26-44)
        pdf = 1.0f / (float)n;
        return n <= 1 ? 0 : rnd.next_i32(0, n - 1);
    }
    if (ninf == 0) return finite_select(sv, nf, rnd, from, pdf);
    const float q = rnd.next_f32();
    if (q < 0.5f) { // infinite_ratio 0.5
        pdf = (1 / (float)ninf) * 0.5f;
        return ninf <= 1 ? 0 : rnd.next_i32(0, ninf - 1);
    }
    float p;
    const int f = finite_select(sv, nf, rnd, from, p);
    pdf = p * (1 - 0.5f);
    return ninf + f;
}
// LightSelector::pdf of light `lid` seen from `from`
__device__ __forceinline__ float select_pdf(const SceneView& sv, int lid, f3 from) {
    const int n = sv.num_lights, ninf = sv.num_infinite, nf = n - ninf;
    if (sv.selector == SEL_UNIFORM) return n == 0 ? 1.0f : 1.0f / (float)n;
    if (ninf == 0) return finite_select_pdf(sv, nf, lid, from);
    if (lid < ninf) return (1 / (float)ninf) * 0.5f;
    return finite_select_pdf(sv, nf, lid - ninf, from) * (1 - 0.5f);
}

// ---------------------------------------------------------------------------
// BSDFs (bsdf/diffuse.art:2-11, bsdf/dielectric.art:2-23) and fresnel
// (core/fresnel.art:7-28)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float fresnel_factor(float eta, float cos_i, float cos_t) {
    float rs = safe_div(eta * cos_i - cos_t, eta * cos_i + cos_t);
    float rp = safe_div(cos_i - eta * cos_t, cos_i + eta * cos_t);
    return clampf((rs * rs + rp * rp) * 0.5f, 0, 1);
}

struct BsdfSample {
    f3 in_dir;
    float pdf;
    f3 color; // already divided by the pdf, cosine applied (make_bsdf_sample)
    float eta;
    bool valid;
};

__device__ __forceinline__ BsdfSample reject_sample() {
    BsdfSample b;
    b.in_dir = mk(0, 0, 0);
    b.pdf = 0;
    b.color = mk(0, 0, 0);
    b.eta = 1;
    b.valid = false;
    return b;
}
__device__ __forceinline__ BsdfSample make_sample(f3 dir, float pdf, f3 color, float eta) {
    BsdfSample b;
    b.in_dir = dir;
    b.pdf = pdf;
    b.color = color;
    b.eta = eta;
    b.valid = true;
    return b;
}

__device__ __forceinline__ float positive_cos(f3 a, f3 b) {
    float c = dot(a, b);
    return c >= 0 ? c : 0;
}
__device__ __forceinline__ float absolute_cos(f3 a, f3 b) { return fabsf(dot(a, b)); }
__device__ __forceinline__ f3 lerp3(f3 a, f3 b, float t) { // color_lerp (core/color.art:18-22)
    return mk((1 - t) * a.x + t * b.x, (1 - t) * a.y + t * b.y, (1 - t) * a.z + t * b.z);
}
__device__ __forceinline__ float lerp1(float a, float b, float k) { return (1 - k) * a + k * b; } // common.art:120
__device__ __forceinline__ f3 to_local(const Frame& f, f3 v) { return mk(dot(f.t, v), dot(f.b, v), dot(f.n, v)); }

// fresnel(eta, cos_i).factor, or 1 on total internal reflection (math::fresnel_dielectric, core/math.art:120)
__device__ __forceinline__ float fresnel_dielectric(float eta, float cos_i) {
    float eta2 = cos_i < 0 ? 1 / eta : eta;
    float cos2_t = 1 - (1 - cos_i * cos_i) * eta2 * eta2; // snell (core/fresnel.art:13)
    if (cos2_t <= 0.0f) return 1.0f;
    return fresnel_factor(eta2, fabsf(cos_i), sqrtf(cos2_t));
}
// conductor_factor (core/fresnel.art:29-36)
__device__ __forceinline__ float conductor_factor(float n, float k, float cos_i) {
    float f = n * n + k * k;
    float d1 = f * cos_i * cos_i;
    float d2 = 2.0f * n * cos_i;
    float rs = safe_div(d1 - d2, d1 + d2);
    float rp = safe_div(f - d2 + cos_i * cos_i, f + d2 + cos_i * cos_i);
    return clampf((rs * rs + rp * rp) * 0.5f, 0, 1);
}
// fresnel_diffuse_factor (core/fresnel.art:42-64)
__device__ __forceinline__ float fresnel_diffuse_factor(float eta) {
    if (eta < 1) return -1.4399f * (eta * eta) + 0.7099f * eta + 0.6681f + 0.0636f / eta;
    float i1 = 1 / eta, i2 = i1 * i1, i3 = i2 * i1, i4 = i3 * i1, i5 = i4 * i1;
    return 0.919317f - 3.4793f * i1 + 6.75335f * i2 - 7.80989f * i3 + 4.98554f * i4 - 1.36881f * i5;
}
__device__ __forceinline__ float diff_of_prod(float a, float b, float c, float d) { // common.art:132-137
    float cd = c * d;
    float diff = fmaf(a, b, -cd);
    float err = fmaf(-c, d, cd);
    return diff + err;
}

// ---- microfacet distributions (core/microfacet.art) ----------------------
__device__ __forceinline__ float ndf_ggx(const Frame& l, f3 m, float au, float av) { // :187-197
    float cz = dot(l.n, m), cx = dot(l.t, m), cy = dot(l.b, m);
    float kx = cx / au, ky = cy / av;
    float k = kx * kx + ky * ky + cz * cz;
    return safe_div(1, PI_ * au * av * k * k);
}
__device__ __forceinline__ float ndf_beckmann(const Frame& l, f3 m, float au, float av) { // :175-185
    float cz = dot(l.n, m), cx = dot(l.t, m), cy = dot(l.b, m);
    float kx = cx / au, ky = cy / av;
    float k2 = safe_div(kx * kx + ky * ky, cz * cz);
    return safe_div(expf(-k2), PI_ * au * av * cz * cz * cz * cz);
}
__device__ __forceinline__ float g1_smith(const Frame& l, f3 w, float au, float av) { // :157-173
    float cz = dot(l.n, w);
    if (fabsf(cz) <= FLT_EPS_) return 0;
    float cx = dot(l.t, w), cy = dot(l.b, w);
    float kx = au * cx, ky = av * cy;
    float a2 = kx * kx + ky * ky;
    if (a2 <= FLT_EPS_) return 1;
    float k2 = a2 / (cz * cz);
    return 2 / (1 + sqrtf(1 + k2));
}
__device__ __forceinline__ float g1_walter(const Frame& l, f3 w, float au, float av) { // :136-155
    float cz = dot(l.n, w);
    if (fabsf(cz) <= FLT_EPS_) return 0;
    float cx = dot(l.t, w), cy = dot(l.b, w);
    float kx = au * cx, ky = av * cy;
    float k2 = (kx * kx + ky * ky) / (cz * cz);
    if (k2 <= FLT_EPS_) return 1;
    float a = 1 / sqrtf(k2), a2 = 1 / k2;
    return a >= 1.6f ? 1.0f : (3.535f * a + 2.181f * a2) / (1.0f + 2.276f * a + 2.577f * a2);
}
__device__ __forceinline__ float mf_D(const DevMaterial& m, const Frame& l, f3 h) {
    return m.dist == MF_BECKMANN ? ndf_beckmann(l, h, m.eta[3], m.kappa[3]) : ndf_ggx(l, h, m.eta[3], m.kappa[3]);
}
__device__ __forceinline__ float mf_G(const DevMaterial& m, const Frame& l, f3 wi, f3 wo) {
    if (m.dist == MF_BECKMANN) return g1_walter(l, wi, m.eta[3], m.kappa[3]) * g1_walter(l, wo, m.eta[3], m.kappa[3]);
    return g1_smith(l, wi, m.eta[3], m.kappa[3]) * g1_smith(l, wo, m.eta[3], m.kappa[3]);
}
// pdf_vndf_ggx (:337-340)
__device__ __forceinline__ float pdf_vndf_ggx(const Frame& l, f3 w, f3 h, float au, float av) {
    float cz = absolute_cos(l.n, w);
    return safe_div(g1_smith(l, w, au, av) * absolute_cos(w, h) * ndf_ggx(l, h, au, av), cz);
}
__device__ __forceinline__ float mf_pdf(const DevMaterial& m, const Frame& l, f3 wo, f3 h) {
    if (m.dist == MF_VNDF_GGX) return pdf_vndf_ggx(l, wo, h, m.eta[3], m.kappa[3]);
    return mf_D(m, l, h) * absolute_cos(l.n, h); // make_microfacet_distribution.pdf (:265)
}
// sample_vndf_ggx (:340-366) with sample_vndf_ggx_11 (:287-304) in frame l
__device__ __forceinline__ f3 vndf_ggx_sample(const Frame& l, Rng& rnd, f3 wo, float au, float av) {
    f3 vl = to_local(l, wo);
    f3 sl = normalize(mk(au * vl.x, av * vl.y, vl.z));
    float st = safe_sqrt(1 - sl.z * sl.z); // sin_cos_phi (core/shading.art:46-53)
    float sin_phi = 0, cos_phi = 1;
    if (fabsf(st) > FLT_EPS_) {
        sin_phi = sl.y / st;
        cos_phi = sl.x / st;
    }
    float ct = fabsf(sl.z);
    float u0 = rnd.next_f32();
    float u1 = rnd.next_f32();
    float px, py;
    concentric_disk(u0, u1, px, py);
    float sv = 0.5f * (1 + ct);
    float y = (1 - sv) * safe_sqrt(1 - px * px) + sv * py;
    float z = safe_sqrt(1 - y * y - px * px);
    float sin_t = safe_sqrt(1 - ct * ct);
    float nrm = safe_div(1, sum_of_prod(sin_t, y, ct, z));
    float slx = diff_of_prod(ct, y, sin_t, z) * nrm, sly = px * nrm;
    float s2x = (cos_phi * slx - sin_phi * sly) * au;
    float s2y = (sin_phi * slx + cos_phi * sly) * av;
    f3 nh = isfinite(s2x) ? normalize(mk(-s2x, -s2y, 1)) : mk(0, 0, 0);
    return frame_to_world(l, nh);
}
// Microfacet normal sample of the material's distribution for outgoing wo.
__device__ __forceinline__ f3 mf_sample(const DevMaterial& m, const Frame& l, Rng& rnd, f3 wo, float& pdf) {
    const float au = m.eta[3], av = m.kappa[3];
    if (m.dist == MF_VNDF_GGX) {
        f3 h = vndf_ggx_sample(l, rnd, wo, au, av);
        pdf = pdf_vndf_ggx(l, wo, h, au, av);
        return h;
    }
    float u0 = rnd.next_f32();
    float u1 = rnd.next_f32();
    const float ar = av / au;
    if (m.dist == MF_BECKMANN) {
        // make_beckmann_model.sample (:211-232)
        float phi = atanf(ar * tanf(2 * PI_ * u1));
        float cos_phi = cosf(phi);
        float sin_phi = sqrtf(1 - cos_phi * cos_phi);
        float kx = cos_phi / au, ky = sin_phi / av;
        float k2 = 1 / (kx * kx + ky * ky);
        float cos_t = 1 / sqrtf(1 - k2 * logf(1.0f - u0));
        float cos_t2 = cos_t * cos_t;
        float sin_t = sqrtf(1 - cos_t2);
        pdf = (1 - u0) / (PI_ * au * av * cos_t2 * cos_t);
        return frame_to_world(l, mk(sin_t * cos_phi, sin_t * sin_phi, cos_t));
    }
    // make_ggx_model.sample (:236-262); the isotropic case uses phi = 2 pi u1
    float phi = au == av ? 2 * PI_ * u1 : atanf(ar * tanf(2 * PI_ * u1));
    float cos_phi = cosf(phi);
    float sin_phi = sqrtf(1 - cos_phi * cos_phi);
    float kx = cos_phi / au, ky = sin_phi / av;
    float d2 = kx * kx + ky * ky;
    float a2 = safe_div(1, d2);
    float t2 = a2 * u0 / (1 - u0);
    float cos_t = 1 / sqrtf(1 + t2);
    float cos_t2 = cos_t * cos_t;
    float sin_t = sqrtf(1 - cos_t2);
    float k2 = d2 * (sin_t * sin_t) / cos_t2;
    pdf = safe_div(1, PI_ * au * av * cos_t2 * cos_t * (1 + k2) * (1 + k2));
    return frame_to_world(l, mk(sin_t * cos_phi, sin_t * sin_phi, cos_t));
}

// ---- BSDFs ------------------------------------------------------------------
// Fresnel term of a conductor lobe: per-channel conductor_factor; plastic's
// specular lobe is a conductor with eta 0, k 1 (PlasticBSDF.cpp:38-42).
__device__ __forceinline__ f3 conductor_fresnel(const DevMaterial& m, float c) {
    if (m.type == MAT_PLASTIC)
        return mk(conductor_factor(0, 1, c), conductor_factor(0, 1, c), conductor_factor(0, 1, c));
    return mk(conductor_factor(m.eta[0], m.kappa[0], c), conductor_factor(m.eta[1], m.kappa[1], c),
              conductor_factor(m.eta[2], m.kappa[2], c));
}
// make_rough_base_conductor_bsdf.eval with kd = black (bsdf/conductor.art:57-69)
__device__ __forceinline__ f3 rough_conductor_eval(const DevMaterial& m, const Surface& s, f3 in, f3 out) {
    const f3 N = s.local.n;
    float cos_o = absolute_cos(out, N), cos_i = absolute_cos(in, N);
    if (cos_o <= FLT_EPS_ || cos_i <= FLT_EPS_) return mk(0, 0, 0);
    f3 h = normalize(add(in, out));
    float D = mf_D(m, s.local, h);
    float G = mf_G(m, s.local, in, out);
    f3 F = conductor_fresnel(m, absolute_cos(out, h));
    f3 ks = mk(m.ks[0], m.ks[1], m.ks[2]);
    return mulf(mul(ks, F), D * G / (4 * cos_o));
}
__device__ __forceinline__ float rough_conductor_pdf(const DevMaterial& m, const Surface& s, f3 in, f3 out) {
    f3 h = normalize(add(in, out));
    float jacob = safe_div(1, 4 * absolute_cos(out, h));
    return mf_pdf(m, s.local, out, h) * jacob;
}
// conductor / plastic specular lobe sample (bsdf/conductor.art:1-27, 42-55, 71-100)
__device__ __forceinline__ BsdfSample specular_lobe_sample(const DevMaterial& m, const Surface& s, Rng& rnd, f3 out) {
    const f3 N = s.local.n;
    const f3 ks = mk(m.ks[0], m.ks[1], m.ks[2]);
    if (m.dist == MF_DELTA) {
        if (m.mirror || m.type == MAT_PLASTIC) return make_sample(reflect(out, N), 1, ks, 1); // make_mirror_bsdf
        float cos_i = dot(out, N);                                                          // make_pure_conductor_bsdf
        return make_sample(reflect(out, N), 1, mul(ks, conductor_fresnel(m, cos_i)), 1);
    }
    float cos_o = absolute_cos(out, N);
    if (cos_o <= FLT_EPS_) return reject_sample();
    float spdf;
    f3 sn = mf_sample(m, s.local, rnd, out, spdf);
    if (dot(sn, sn) <= FLT_EPS_) return reject_sample();
    f3 oh = normalize(sn);
    f3 h = signbit(dot(oh, out)) ? neg(oh) : oh;
    f3 in = reflect(out, h);
    if (absolute_cos(in, N) <= FLT_EPS_) return reject_sample();
    float jacob = 1 / (4 * absolute_cos(out, h));
    float pdf = spdf * jacob;
    return make_sample(in, pdf, mulf(rough_conductor_eval(m, s, in, out), safe_div(1, pdf)), 1);
}
__device__ __forceinline__ bool lobe_is_specular(const DevMaterial& m) { return m.dist == MF_DELTA; }

// Diffuse: Lambert, or Oren-Nayar when roughness > eps (bsdf/diffuse.art:2-46)
template <bool FULL = true>
__device__ __forceinline__ f3 diffuse_eval(const DevMaterial& m, const Surface& s, f3 in, f3 out) {
    const f3 N = s.local.n;
    const f3 kd = mk(m.kd[0], m.kd[1], m.kd[2]);
    const float alpha = m.kd[3];
    if (!FULL || alpha <= FLT_EPS_) return mulf(kd, absolute_cos(in, N) * INV_PI_);
    float a2 = alpha * alpha;
    float p1 = absolute_cos(in, N), p2 = absolute_cos(out, N);
    float sv = -p1 * p2 + positive_cos(out, in);
    float t = sv <= FLT_EPS_ ? 1.0f : fmaxf(FLT_EPS_, fmaxf(p1, p2));
    float A = 1 - 0.5f * a2 / (a2 + 0.33f);
    float B = 0.45f * a2 / (a2 + 0.09f);
    float C = 0.17f * a2 / (a2 + 0.13f);
    return mulf(add(mulf(kd, (A + (B * sv / t)) / PI_), mul(kd, mulf(kd, C / PI_))), p1);
}
template <bool FULL = true>
__device__ __forceinline__ BsdfSample diffuse_sample(const DevMaterial& m, const Surface& s, Rng& rnd, f3 out) {
    float u = rnd.next_f32();
    float v = rnd.next_f32();
    float pdf;
    f3 ld = sample_cosine_hemisphere(u, v, &pdf);
    f3 dir = frame_to_world(s.local, ld);
    if (!FULL || m.kd[3] <= FLT_EPS_) return make_sample(dir, pdf, mk(m.kd[0], m.kd[1], m.kd[2]), 1);
    return make_sample(dir, pdf, mulf(diffuse_eval(m, s, dir, out), 1 / pdf), 1);
}
__device__ __forceinline__ float diffuse_pdf(const Surface& s, f3 in) { return positive_cos(in, s.local.n) / PI_; }

// Plastic (bsdf/plastic.art): Fresnel-weighted variadic mix of a diffuse lobe
// with inner-scattering term and a conductor(eta 0, k 1) specular lobe.
__device__ __forceinline__ float plastic_scatter(const DevMaterial& m, float cos_i) {
    const float eta = m.ks[3] / m.kt[3];
    const float fdr = fresnel_diffuse_factor(eta);
    float fi = fresnel_dielectric(eta, cos_i);
    return (1 - fi) * eta * eta / (1 - fdr);
}
__device__ __forceinline__ f3 plastic_diffuse_eval(const DevMaterial& m, const Surface& s, f3 in) {
    const f3 kd = mk(m.kd[0], m.kd[1], m.kd[2]);
    return mulf(mulf(kd, absolute_cos(in, s.local.n) * INV_PI_), plastic_scatter(m, absolute_cos(in, s.local.n)));
}
__device__ __forceinline__ float plastic_mix(const DevMaterial& m, const Surface& s, f3 out) {
    return fresnel_dielectric(m.ks[3] / m.kt[3], absolute_cos(out, s.local.n));
}

// ---- principled BSDF (bsdf/principled.art) -----------------------------------
// Works in the shading frame: wo / wi / h are local, the microfacet lobes use
// the identity frame (make_vndf_ggx_distribution(face_normal, identity, ...)).
// DevMaterial packing: kd = base colour, ior | ks = diffuse_transmission,
// specular_transmission, specular_tint, roughness_u | kt = roughness_v,
// flatness, metallic, sheen | eta = sheen_tint, clearcoat, clearcoat_gloss,
// clearcoat_roughness | mirror bit 0 = thin, bit 1 = clearcoat_top_only.
struct Principled {
    f3 base;
    float ior, dtrans, strans, stint, ru, rv, flat, metal, sheen, sheen_tint, cc, cc_gloss, cc_rough, eta;
    bool thin, cc_top, entering;
};
__device__ __forceinline__ Principled principled_of(const DevMaterial& m, const Surface& s) {
    Principled p;
    p.base = mk(m.kd[0], m.kd[1], m.kd[2]);
    p.ior = m.kd[3];
    p.dtrans = m.ks[0];
    p.strans = m.ks[1];
    p.stint = m.ks[2];
    p.ru = fmaxf(1e-3f, m.ks[3]);
    p.rv = fmaxf(1e-3f, m.kt[0]);
    p.flat = m.kt[1];
    p.metal = m.kt[2];
    p.sheen = m.kt[3];
    p.sheen_tint = m.eta[0];
    p.cc = m.eta[1];
    p.cc_gloss = m.eta[2];
    p.cc_rough = m.eta[3];
    p.thin = (m.mirror & 1) != 0;
    p.cc_top = (m.mirror & 2) != 0;
    p.entering = s.entering;
    p.eta = (s.entering || p.thin) ? 1 / p.ior : p.ior;
    return p;
}
__device__ __forceinline__ Frame frame_identity() { return Frame{mk(1, 0, 0), mk(0, 1, 0), mk(0, 0, 1)}; }
__device__ __forceinline__ float luminance(f3 c) { return c.x * 0.2126f + c.y * 0.7152f + c.z * 0.0722f; } // color.art:28
__device__ __forceinline__ f3 tint_color(f3 c) {
    float lum = luminance(c);
    return lum <= FLT_EPS_ ? mk(1, 1, 1) : mk(c.x / lum, c.y / lum, c.z / lum);
}
__device__ __forceinline__ float schlick_approx(float f) { // fresnel.art:88-91
    float s = clampf(1 - f, 0, 1);
    return (s * s) * (s * s) * s;
}
__device__ __forceinline__ float schlick_r0(float eta) {
    float f = clampf((eta - 1) / (eta + 1), -1, 1);
    return f * f;
}
__device__ __forceinline__ bool same_hemi(f3 a, f3 b) { return (a.z >= 0) == (b.z >= 0); }
__device__ __forceinline__ f3 make_same_hemi(f3 a, f3 b) { return same_hemi(a, b) ? b : neg(b); }
__device__ __forceinline__ f3 make_positive_hemi(f3 v) { return v.z >= 0 ? v : neg(v); }
__device__ __forceinline__ float refr_jacobian(float eta, float ci, float co) { // shading.art:71-74
    float jd = ci + co * eta;
    return safe_div(eta * eta * ci, jd * jd);
}
__device__ __forceinline__ f3 principled_reflection(const Principled& p, f3 wo, f3 wi, f3 h) {
    const Frame I = frame_identity();
    // evalDisneyFresnelTerm
    float HdV = fabsf(dot(wo, h)), HdL = fabsf(dot(wi, h));
    f3 F = mk(0, 0, 0);
    if (!(HdV * HdL <= FLT_EPS_)) {
        float f1 = fresnel_dielectric(p.eta, HdV);
        f3 a = lerp3(mk(1, 1, 1), tint_color(p.base), p.stint);
        f3 r0 = lerp3(mulf(a, schlick_r0(p.eta)), p.base, p.metal);
        float sk = schlick_approx(HdL);
        f3 f2 = add(r0, mulf(sub(mk(1, 1, 1), r0), sk));
        F = lerp3(mk(f1, f1, f1), f2, p.metal);
    }
    float D = ndf_ggx(I, h, p.ru, p.rv);
    float G = g1_smith(I, wi, p.ru, p.rv) * g1_smith(I, wo, p.ru, p.rv);
    float jacob = safe_div(1, 4 * wo.z);
    return mulf(F, fabsf(D * G * jacob));
}
__device__ __forceinline__ f3 principled_eval_local(const Principled& p, f3 wo, f3 wi) {
    const Frame I = frame_identity();
    const bool is_trans = !same_hemi(wi, wo);
    f3 h = make_same_hemi(wo, is_trans ? normalize(add(wi, mulf(wo, p.eta))) : normalize(add(wi, wo)));
    const bool in_front = p.entering == (wi.z >= 0), out_front = p.entering == (wo.z >= 0);
    const float aNdL = fabsf(wi.z), aNdV = fabsf(wo.z);
    if (aNdL <= 1e-5f) return mk(0, 0, 0);
    f3 c = mk(0, 0, 0);
    const float diffuse_weight = (p.thin ? 1.0f : 1 - clampf(p.metal, 0, 1)) * (1 - clampf(p.strans, 0, 1));
    const float trans_weight = (1 - clampf(p.metal, 0, 1)) * clampf(p.strans, 0, 1);
    const float lk = schlick_approx(aNdL), vk = schlick_approx(aNdV);
    if (!is_trans) {
        if (diffuse_weight > 0) { // evalDiffuseTerm
            float diff = (1 - 0.5f * lk) * (1 - 0.5f * vk);
            float VdotL = fabsf(dot(wi, wo));
            float rr = (VdotL + 1) * (p.ru + p.rv) / 2;
            float retro = rr * (lk + vk + lk * vk * (rr - 1));
            float ss = 1;
            if (p.thin) { // evalSubsurfaceTerm
                float r2 = p.ru * p.rv;
                float HdotL = dot(wi, h);
                float fss90 = HdotL * HdotL * r2;
                float fss = (1 - lk + fss90 * lk) * (1 - vk + fss90 * vk);
                float sub_ = 1.25f * (fss * (1 / (aNdL + aNdV + 1e-5f) - 0.5f) + 0.5f);
                ss = 1 - p.flat + sub_ * p.flat;
            }
            float d = INV_PI_ * (diff + retro) * ss * aNdL * diffuse_weight;
            c = add(c, mulf(p.base, d));
        }
        if (p.sheen > 0) { // evalSheenTerm
            f3 st = lerp3(mk(1, 1, 1), tint_color(p.base), p.sheen_tint);
            c = add(c, mulf(mulf(st, p.sheen * lk * aNdL), diffuse_weight));
        }
        c = add(c, principled_reflection(p, wo, wi, h)); // spec_weight = 1
        if ((!p.cc_top || (in_front && out_front)) && p.cc > 0) { // evalClearcoatTerm
            const float F0 = 0.04f, R = 0.25f;
            float R2 = fmaxf(0.001f, p.cc_rough * (1 - p.cc_gloss) + 0.01f * p.cc_gloss);
            float aHdL = fabsf(dot(wi, h));
            float d = ndf_ggx(I, h, R2, R2);
            float f = F0 + (1 - F0) * schlick_approx(aHdL);
            float g = g1_smith(I, wi, R, R) * g1_smith(I, wo, R, R);
            float jacob = safe_div(1, 4 * wo.z);
            float v = fabsf(R * d * f * g * jacob * wi.z);
            c = add(c, mulf(mk(v, v, v), p.cc));
        }
    } else {
        if (p.thin && p.dtrans > 0) { // evalTranslucentTerm
            float diff = (1 - 0.5f * lk) * (1 - 0.5f * vk);
            c = add(c, mulf(p.base, INV_PI_ * diff * aNdL * p.dtrans));
        }
        if (p.strans > 0) { // evalRefractionTerm
            float term;
            if (p.thin) {
                float ft = fresnel_dielectric(p.eta, aNdV);
                float F = ft + (1 - ft) * ft / (ft + 1);
                term = 1 - F;
            } else {
                float HdI = dot(wi, h), HdO = dot(wo, h);
                float F = fresnel_dielectric(p.eta, fabsf(HdO));
                float D = ndf_ggx(I, h, p.ru, p.rv);
                float G = g1_smith(I, wi, p.ru, p.rv) * g1_smith(I, wo, p.ru, p.rv);
                float jacob = refr_jacobian(p.eta, HdI, HdO);
                float norm = fabsf(safe_div(HdO * jacob, wo.z));
                term = (1 - F) * D * G * norm;
            }
            f3 col = p.thin ? mk(sqrtf(p.base.x), sqrtf(p.base.y), sqrtf(p.base.z)) : p.base;
            c = add(c, mulf(mulf(col, term), trans_weight));
        }
    }
    return c;
}
struct Lobes { float diff_refl, diff_trans, spec_refl, spec_trans; };
__device__ __forceinline__ Lobes principled_lobes(const Principled& p, f3 wo) { // calcLobeDistribution
    float metal = clampf(p.metal, 0, 1), dt = clampf(p.dtrans, 0, 1), stn = clampf(p.strans, 0, 1);
    float abs_gen = luminance(p.base);
    float abs_spec = lerp1(1.0f, luminance(tint_color(p.base)), p.stint);
    float diff_refl = clampf(abs_gen * (1 - metal) * (1 - stn), 0, 1);
    float F = fresnel_dielectric(p.eta, fabsf(wo.z));
    float spec_refl = clampf(abs_spec * (1 - F) + F, 0, 1);
    if (!(dt > 0 || stn > 0)) {
        float norm = diff_refl + spec_refl;
        if (norm <= FLT_EPS_) return Lobes{1, 0, 0, 0};
        return Lobes{diff_refl / norm, 0, spec_refl / norm, 0};
    }
    float diff_trans = clampf(abs_gen * dt * diff_refl, 0, 1);
    float spec_trans = clampf((1 - F) * abs_gen * (1 - metal) * stn, 0, 1);
    float norm = diff_refl + spec_refl + diff_trans + spec_trans;
    if (norm <= FLT_EPS_) return Lobes{1, 0, 0, 0};
    return Lobes{diff_refl / norm, diff_trans / norm, spec_refl / norm, spec_trans / norm};
}
__device__ __forceinline__ float bound_spec_pdf(float v) { return v <= 1e-5f ? 0.0f : v; }
__device__ __forceinline__ float principled_spec_refl_pdf(const Principled& p, f3 wo, f3 wi) {
    f3 pwo = make_positive_hemi(wo), pwi = make_positive_hemi(wi);
    f3 H = normalize(add(pwo, pwi));
    float cho = dot(pwo, H);
    return fabsf(bound_spec_pdf(pdf_vndf_ggx(frame_identity(), pwo, H, p.ru, p.rv)) * safe_div(1, 4 * cho));
}
__device__ __forceinline__ float principled_spec_trans_pdf(const Principled& p, f3 wo, f3 wi) {
    f3 pwo = make_positive_hemi(wo), pwi = neg(make_positive_hemi(wi));
    f3 H = normalize(add(pwi, mulf(pwo, p.eta)));
    float chi = dot(pwi, H), cho = dot(pwo, H);
    return fabsf(bound_spec_pdf(pdf_vndf_ggx(frame_identity(), pwo, H, p.ru, p.rv)) * refr_jacobian(p.eta, chi, cho));
}
__device__ __forceinline__ float principled_pdf_local(const Principled& p, f3 wo, f3 wi) {
    if (fabsf(wo.z) <= 1e-5f || fabsf(wi.z) <= 1e-5f) return 0;
    Lobes l = principled_lobes(p, wo);
    float dp = fabsf(wi.z) / PI_;
    if (same_hemi(wo, wi)) return l.diff_refl * dp + l.spec_refl * principled_spec_refl_pdf(p, wo, wi);
    if (p.thin) return l.diff_trans * dp + l.spec_trans;
    return l.diff_trans * dp + l.spec_trans * principled_spec_trans_pdf(p, wo, wi);
}
__device__ __forceinline__ f3 principled_eval(const DevMaterial& m, const Surface& s, f3 in, f3 out) {
    Principled p = principled_of(m, s);
    return principled_eval_local(p, to_local(s.local, out), to_local(s.local, in));
}
__device__ __forceinline__ float principled_pdf(const DevMaterial& m, const Surface& s, f3 in, f3 out) {
    Principled p = principled_of(m, s);
    return principled_pdf_local(p, to_local(s.local, out), to_local(s.local, in));
}
__device__ __forceinline__ BsdfSample principled_sample(const DevMaterial& m, const Surface& s, Rng& rnd, f3 out) {
    const Principled p = principled_of(m, s);
    const Frame I = frame_identity();
    const f3 wo = to_local(s.local, out);
    if (fabsf(wo.z) <= 1e-5f) return reject_sample();
    const Lobes l = principled_lobes(p, wo);
    const float pick = rnd.next_f32();
    f3 wi;
    float pdf;
    if (pick < l.diff_refl) {
        float u = rnd.next_f32(), v = rnd.next_f32(), cp;
        wi = make_same_hemi(wo, sample_cosine_hemisphere(u, v, &cp));
        pdf = cp * l.diff_refl + principled_spec_refl_pdf(p, wo, wi) * l.spec_refl;
    } else if (pick < l.diff_refl + l.diff_trans) {
        float u = rnd.next_f32(), v = rnd.next_f32(), cp;
        wi = neg(make_same_hemi(wo, sample_cosine_hemisphere(u, v, &cp)));
        pdf = cp * l.diff_trans + principled_spec_trans_pdf(p, wo, wi) * l.spec_trans;
    } else if (pick < l.diff_refl + l.diff_trans + l.spec_trans) {
        if (p.thin) {
            wi = neg(wo);
            pdf = l.spec_trans;
        } else {
            f3 pwo = make_positive_hemi(wo);
            f3 sn = vndf_ggx_sample(I, rnd, pwo, p.ru, p.rv);
            float spdf = pdf_vndf_ggx(I, pwo, sn, p.ru, p.rv);
            if (spdf <= 1e-5f || dot(sn, sn) <= FLT_EPS_) return reject_sample();
            f3 oH = normalize(sn);
            f3 H = signbit(dot(oH, pwo)) ? neg(oH) : oH;
            float cho = dot(pwo, H);
            // fresnel(eta, cos_h_o) (core/fresnel.art:15-26)
            float eta2 = cho < 0 ? 1 / p.eta : p.eta;
            float cos2_t = 1 - (1 - cho * cho) * eta2 * eta2;
            if (!(cos2_t <= 0.0f)) {
                float ct = sqrtf(cos2_t);
                float cos_t = cho < 0 ? -ct : ct;
                f3 pwi = normalize(refract(pwo, H, p.eta, cho, cos_t));
                if (!(!same_hemi(pwo, pwi) && cho > FLT_EPS_ && -pwi.z > 1e-5f)) return reject_sample();
                wi = neg(make_same_hemi(wo, pwi));
                pdf = fabsf(spdf * refr_jacobian(p.eta, dot(pwi, H), cho)) * l.spec_trans + fabsf(wi.z) / PI_ * l.diff_trans;
            } else { // total reflection
                f3 pwi = normalize(reflect(pwo, H));
                if (!(same_hemi(pwo, pwi) && cho > FLT_EPS_ && pwi.z > 1e-5f)) return reject_sample();
                wi = make_same_hemi(wo, pwi);
                pdf = spdf * safe_div(1, 4 * cho) * l.spec_trans + fabsf(wi.z) / PI_ * l.diff_trans;
            }
        }
    } else {
        f3 pwo = make_positive_hemi(wo);
        f3 sn = vndf_ggx_sample(I, rnd, pwo, p.ru, p.rv);
        float spdf = pdf_vndf_ggx(I, pwo, sn, p.ru, p.rv);
        if (spdf <= 1e-5f || dot(sn, sn) <= FLT_EPS_) return reject_sample();
        f3 oH = normalize(sn);
        f3 H = signbit(dot(oH, pwo)) ? neg(oH) : oH;
        float cho = dot(pwo, H);
        f3 pwi = normalize(reflect(pwo, H));
        if (!(same_hemi(pwo, pwi) && cho > FLT_EPS_ && pwi.z > 1e-5f)) return reject_sample();
        wi = make_same_hemi(wo, pwi);
        pdf = fabsf(spdf * safe_div(1, 4 * cho)) * l.spec_refl + fabsf(wi.z) / PI_ * l.diff_refl;
    }
    if (pdf <= FLT_EPS_) return reject_sample();
    const float s_eta = (p.thin || same_hemi(wo, wi)) ? 1.0f : p.eta;
    const f3 in_dir = frame_to_world(s.local, wi);
    return make_sample(in_dir, pdf, mulf(principled_eval(m, s, in_dir, out), 1 / pdf), s_eta);
}

// FULL = false compiles only the materials and lights of the basic set
// (Lambert diffuse, dielectric; plane/env/point/spot/directional/sun lights):
// the upload picks that kernel variant when the scene needs nothing more, so
// scenes like the diamond do not pay the wider shading code's registers.
template <bool FULL>
__device__ __forceinline__ bool bsdf_is_specular(const DevMaterial& m) {
    return m.type == MAT_DIELECTRIC || (FULL && m.type == MAT_CONDUCTOR && m.dist == MF_DELTA);
}
template <bool FULL>
__device__ __forceinline__ f3 bsdf_eval(const DevMaterial& m, const Surface& s, f3 in, f3 out) {
    if (!FULL) return m.type == MAT_DIFFUSE ? diffuse_eval<false>(m, s, in, out) : mk(0, 0, 0);
    switch (m.type) {
    case MAT_DIFFUSE: return diffuse_eval(m, s, in, out);
    case MAT_PRINCIPLED: return principled_eval(m, s, in, out);
    case MAT_CONDUCTOR: return m.dist == MF_DELTA ? mk(0, 0, 0) : rough_conductor_eval(m, s, in, out);
    case MAT_PLASTIC: {
        float k = plastic_mix(m, s, out);
        f3 spec = m.dist == MF_DELTA ? mk(0, 0, 0) : rough_conductor_eval(m, s, in, out);
        return lerp3(plastic_diffuse_eval(m, s, in), spec, k);
    }
    default: return mk(0, 0, 0);
    }
}
template <bool FULL>
__device__ __forceinline__ float bsdf_pdf(const DevMaterial& m, const Surface& s, f3 in, f3 out) {
    if (!FULL) return m.type == MAT_DIFFUSE ? diffuse_pdf(s, in) : 0.0f;
    switch (m.type) {
    case MAT_DIFFUSE: return diffuse_pdf(s, in);
    case MAT_PRINCIPLED: return principled_pdf(m, s, in, out);
    case MAT_CONDUCTOR: return m.dist == MF_DELTA ? 0.0f : rough_conductor_pdf(m, s, in, out);
    case MAT_PLASTIC: {
        float k = plastic_mix(m, s, out);
        float sp = m.dist == MF_DELTA ? 0.0f : rough_conductor_pdf(m, s, in, out);
        return lerp1(diffuse_pdf(s, in), sp, k);
    }
    default: return 0;
    }
}

// make_pure_dielectric_bsdf.sample, adjoint = false (bsdf/dielectric.art)
__device__ __forceinline__ BsdfSample dielectric_sample(const DevMaterial& m, const Surface& s, Rng& rnd, f3 out_dir) {
    float n1 = m.ks[3], n2 = m.kt[3];
    if (m.mirror) {
        // thin interface (make_thin_dielectric_bsdf, bsdf/dielectric.art:26-47): always
        // outside -> inside, F sums the slab's inter-reflections, straight transmission
        float f = fresnel_dielectric(n1 / n2, absolute_cos(out_dir, s.local.n));
        float F = f + (1 - f) * f / (f + 1);
        if (rnd.next_f32() > F) return make_sample(mulf(out_dir, -1.0f), 1, mk(m.kt[0], m.kt[1], m.kt[2]), 1);
        return make_sample(normalize(reflect(out_dir, s.local.n)), 1, mk(m.ks[0], m.ks[1], m.ks[2]), 1);
    }
    float k = s.entering ? n1 / n2 : n2 / n1;
    f3 n = s.local.n;
    float cos_o = dot(out_dir, n);
    // fresnel(k, cos_o), FresnelTerm{cos_t=0, factor=1} when total internal reflection
    float ft_cos_t = 0, ft_factor = 1;
    {
        float eta2 = cos_o < 0 ? 1 / k : k;
        float cos2_t = 1 - (1 - cos_o * cos_o) * eta2 * eta2;
        if (!(cos2_t <= 0.0f)) {
            float ct = sqrtf(cos2_t);
            ft_cos_t = cos_o < 0 ? -ct : ct;
            ft_factor = fresnel_factor(eta2, fabsf(cos_o), ct);
        }
    }
    if (rnd.next_f32() > ft_factor)
        return make_sample(refract(out_dir, n, k, cos_o, ft_cos_t), 1, mk(m.kt[0], m.kt[1], m.kt[2]), k);
    return make_sample(reflect(out_dir, n), 1, mk(m.ks[0], m.ks[1], m.ks[2]), 1);
}

template <bool FULL>
__device__ __forceinline__ BsdfSample bsdf_sample(const DevMaterial& m, const Surface& s, Rng& rnd, f3 out) {
    if (!FULL) return m.type == MAT_DIELECTRIC ? dielectric_sample(m, s, rnd, out) : diffuse_sample<false>(m, s, rnd, out);
    switch (m.type) {
    case MAT_DIFFUSE: return diffuse_sample(m, s, rnd, out);
    case MAT_DIELECTRIC: return dielectric_sample(m, s, rnd, out);
    case MAT_CONDUCTOR: return specular_lobe_sample(m, s, rnd, out);
    case MAT_PRINCIPLED: return principled_sample(m, s, rnd, out);
    default: break;
    }
    // plastic: make_variadic_mix_bsdf(diffuse_extra, specular, mix_f).sample (bsdf/mix.art:29-62)
    const float k = plastic_mix(m, s, out);
    const bool spec_delta = lobe_is_specular(m);
    auto diffuse_extra = [&]() {
        BsdfSample b = diffuse_sample(m, s, rnd, out); // Lambert lobe (kd, cosine pdf)
        b.color = mulf(b.color, plastic_scatter(m, absolute_cos(b.in_dir, s.local.n)));
        return b;
    };
    if (k <= 0) return diffuse_extra();
    if (k >= 1) return specular_lobe_sample(m, s, rnd, out);
    if (rnd.next_f32() < 1 - k) {
        BsdfSample b = diffuse_extra(); // sample_mat(diffuse, specular, k)
        if (b.valid) {
            if (spec_delta) return b;
            float p = lerp1(b.pdf, rough_conductor_pdf(m, s, b.in_dir, out), k);
            f3 c = lerp3(mulf(b.color, b.pdf), rough_conductor_eval(m, s, b.in_dir, out), k);
            b.pdf = p;
            b.color = mk(c.x / p, c.y / p, c.z / p);
            return b;
        }
        return specular_lobe_sample(m, s, rnd, out);
    }
    BsdfSample b = specular_lobe_sample(m, s, rnd, out); // sample_mat(specular, diffuse, 1 - k)
    if (b.valid) {
        float p = lerp1(b.pdf, diffuse_pdf(s, b.in_dir), 1 - k);
        f3 c = lerp3(mulf(b.color, b.pdf), plastic_diffuse_eval(m, s, b.in_dir), 1 - k);
        b.pdf = p;
        b.color = mk(c.x / p, c.y / p, c.z / p);
        return b;
    }
    return diffuse_extra();
}

} // namespace igxd
