// MI355X (gfx950) wavefront path-tracing device: kernels + host driver + C-ABI.
//
// Hot path = the reference's per-iteration loop gpu_trace
// (src/artic/driver/mapping_gpu.art:728-870) re-designed for CDNA4:
//   * all paths of one or more iterations are resident in HBM as one wavefront
//     ("chunk", up to 128 M paths) instead of refilling a 1M-ray stream
//     (mapping_gpu.art:1125);
//   * one fused "extend" kernel per bounce does closest-hit traversal AND
//     shading (the reference launches traverse, 3 sort kernels with a host scan,
//     one hit-shade kernel per material, miss shade, then compaction with a D2H
//     sync: mapping_gpu.art:45-68, 403-498, 114-205, 229-266, 685-714); scenes
//     whose tables exceed one XCD's L2 split it into a persistent-lane trace
//     kernel and a shade kernel;
//   * surviving paths and shadow rays are compacted on the fly with a 64-lane
//     ballot and one atomic per wave on one of 64 shard counters (no sort, no
//     host round trip);
//   * shadow rays are traced by a separate any-hit kernel over the compacted
//     shadow stream (gpu_traverse_secondary, mapping_gpu.art:70-112);
//   * the last paths of a chunk run to their end in a tail kernel on a second
//     stream, overlapping the next chunk;
//   * radiance is accumulated per path slot with plain read-modify-writes (each
//     slot is owned by exactly one ray at a time), then a resolve kernel adds
//     sum(L_s)/spi to the framebuffer -- deterministic, no float atomics
//     (the reference splats with atomic adds, driver/accumulator.art:4-21).
#include "igx.h"

#include "device_math.h"
#include "device_scene.h"
#include "igx_kernels.h"
#include "../host/bvh_build.h"
#include "../host/light_select.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <map>
#include <cmath>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <type_traits>

using namespace igxd;

// The file is compiled once per part (Makefile: -DIGX_PART=n) so the many
// kernel instantiations build in parallel:
//   0 = host driver, C-ABI and the small kernels; 1 = k_extend variants;
//   2 = k_finish variants; 3 = k_trace / k_trace_refill / k_shade / k_shadow /
//   k_shadow_refill variants.  Types and device functions are shared; each
//   part instantiates only its own launch helpers (explicit instantiation),
//   the others see them as extern templates.
#ifndef IGX_PART
#define IGX_PART 0
#endif

namespace igxh {

constexpr int BLOCK = 256;
[[maybe_unused]] constexpr int MAX_BLOCKS_PER_CU = 8;  // 2048 threads per CU; grids never exceed num_cus * this
[[maybe_unused]] constexpr int MAX_STACK = 128;        // traversal stack entries (LDS + spill) per ray
constexpr int MAX_BOUNCES = 256;          // path depth is stored in 8 bits (p1.w, above the 24-bit RNG counter)
constexpr long long MAX_CHUNK_PATHS = 1ll << 27; // paths per chunk (one wavefront), ~25 GB of stream buffers per slot
// a path's slot in its chunk takes the low 27 bits of the slot word; the top
// 5 carry 1 + the index of the enclosing entity it is in (at most 31 entities)
constexpr int SLOT_BITS = 27;
constexpr uint32_t SLOT_MASK = (1u << SLOT_BITS) - 1;
[[maybe_unused]] constexpr int MAX_ENCLOSING = 31;
static_assert(MAX_CHUNK_PATHS <= (1ll << SLOT_BITS), "path slots must fit the slot bits");
// Occupancy target (waves per SIMD) of k_extend, with global and with
// LDS-staged traversal tables: 4 caps it at 128 VGPRs.  k_finish keeps the
// compiler's choice (it would spill).
#ifndef EXTEND_WAVES
#define EXTEND_WAVES 4
#endif
// the full shading variant on global tables: 3 waves per SIMD (no spills)
// instead of 4 (~150 spilled VGPRs): materials frame 55.3 -> 54.0 ms; the
// basic variant stays at 4 (S-deep 31.5 -> 36.1, primitives 22.0 -> 24.3 ms
// at 3), profiles/r02_ab_extend_waves.log
#ifndef EXTEND_WAVES_FULL
#define EXTEND_WAVES_FULL 3
#endif
#ifndef EXTEND_WAVES_LDS
#define EXTEND_WAVES_LDS 4
#endif


// ---------------------------------------------------------------------------
// Streams (SoA of 16-byte records)
// ---------------------------------------------------------------------------
// Every compacted stream is cut into NSH shards of `shard_cap` records
// (record (s, pos) at index s * shard_cap + pos), each with its own counter:
// a wave appends to the shard of its global wave index, so the append is one
// returning atomic per wave on a word shared by 1/NSH of the waves, and no
// block barrier holds a wave behind the slowest of its block.
constexpr int NSH = 64;             // shards per stream (one per lane of the counting wave)
constexpr int CSTRIDE = 16;         // ints between two shard counters: one 64-B atomic line each
constexpr int CROW = NSH * CSTRIDE; // ints per counter row (one row per stream and bounce)
constexpr int WAVES_PER_BLOCK = BLOCK / 64;
// k_trace_refill stages no treelet: its top nodes stay L2 hits anyway, and
// without one its node fetches are global loads instead of the flat loads
// that serve LDS and global addresses alike (soup-1M 8-iteration frame
// 315.8 / 313.5 -> 305.6 / 307.2 ms, soup-16M 118.2 -> 117.9 ms;
// profiles/r03_ab_trace_global.log).  k_finish_pairs stages none either
// (soup-16M k_finish_pairs 6.0 -> 8.5 ms with one, r05_ab_finish_treelet.log).
// k_extend and the shadow kernels on global-table scenes: LDS treelet (1)
// or none and global node loads (0)
#ifndef EXTEND_TREELET
#define EXTEND_TREELET 1
#endif
#ifndef SHADOW_TREELET
#define SHADOW_TREELET 1
#endif
// k_extend's dynamic groups: the append's atomic round trip also takes the
// wave's next group (1, wave_append_paths) or take_group issues its own (0)
#ifndef IGX_CLAIM_NEXT
#define IGX_CLAIM_NEXT 1
#endif
// bounce b >= 2 launches a grid sized to the paths entering bounce b - 1 (1)
// instead of the chunk's first-bounce grid (0)
#ifndef IGX_LIVE_GRID
#define IGX_LIVE_GRID 1
#endif
[[maybe_unused]] constexpr int GRID_QUANTUM = NSH / WAVES_PER_BLOCK; // grids are multiples of this: every shard gets the same waves

struct PathBuf {
    float4* p0; // org.xyz, slot (int bits; bits 27-31: 1 + the enclosing entity index the path is in, 0: none)
    float4* p1; // dir.xyz, rnd counter
    float4* p2; // contrib.rgb, inv_pdf
    float2* p3; // eta, RNG seed (uint bits): hashed once by k_generate, not per bounce
    int shard_cap;
    int c_base; // record index of the class-C region (FrameArgs::classify 4), 0: none
};
struct ShadowBuf {
    float4* s0; // org.xyz, slot
    float4* s1; // dir.xyz, tmax
    float4* s2; // colour.rgb, -
    int shard_cap;
    float4* aov_nee; // "NEE Weights" per path slot (technique aov_mis), nullptr: off
};
struct HitBuf {
    float4* h;  // t, u, v, entity (int bits; -1 = miss)
    int* prim;  // primitive id
};

#ifndef IGX_AOV
#define IGX_AOV 1 // 0: experiment builds without the AOV code (its cost on the default path)
#endif
struct FrameArgs {
    int width, height, spi, iter, frame, seed;
    int tile_size, tile_offset, tile_stride, tiles_x;
    int num_rays;
    const float* rays;   // device copy of the ray list (ray-list mode)
    int chunk_pixel0;    // first local pixel of this chunk
    int chunk_pixels;    // local pixels in this chunk
    int chunk_iters;     // consecutive iterations (iter, iter + 1, ...) the chunk covers
    float inv_spi;
    int gen_n;           // > 0: this k_extend launch is bounce 0 and generates its n camera paths itself
    int classify;        // surviving paths' stream class (see wave_append_paths): 0 all A, 1 B = inside a dielectric (eta != 1), 2 B = after a specular event
    int dynamic;         // k_extend: waves take 64-path groups from per-shard work counters (KernelCounters::work)
    int shadow_classes;  // shadow rays crossing an enclosing entity's box go to the back of their shard (shadow_class_b)
    int reverse;         // k_extend: a shard's positions are taken from its end (class C, then B, then A:
                         // the groups whose paths run longest start first, the short ones fill the launch's end)
    int probe_sample;    // test hook (option "probe_sample"): 0 = k_resolve adds every sample; s + 1 = sample s only
    // the path tracer's MIS AOVs (technique aov_mis, PathTechnique.cpp:16-25):
    // per path slot beside L, "Direct Weights" = emission hits and misses
    // (pathtracer.art:128,158), "NEE Weights" = unoccluded shadow rays (:206);
    // nullptr: off (the default path pays one scalar branch per add)
    float4* aov_di;
    float4* aov_nee;
};

// path slot -> (local pixel, sample, iteration): slots run over the chunk's
// pixels x spi samples, one such block per iteration of the chunk
__device__ __forceinline__ void slot_coords(const FrameArgs& fa, int slot, int& lp, int& sample, int& iter) {
    const int per_iter = fa.chunk_pixels * fa.spi;
    const int it = slot / per_iter;
    const int r = slot - it * per_iter;
    const int q = r / fa.spi;
    lp = fa.chunk_pixel0 + q;
    sample = r - q * fa.spi;
    iter = fa.iter + it;
}

// local pixel -> global (x, y); false if the slot lies outside the film
// Pixel order of the local pixel index: eight consecutive pixels (one wave's
// camera group at spi 8) form a 4 x 2 block instead of a 1 x 8 row run, when
// the width (tile side) is a multiple of 4 and the height even: the group's
// camera rays then diverge less in the traversal (IGX_PIXEL_BLOCKS).  Every
// user of the index (generation, resolve, tile packing) maps it here, and a
// path's arithmetic depends on its pixel only, so the film is the same.
#ifndef IGX_PIXEL_BLOCKS
#define IGX_PIXEL_BLOCKS 1
#endif
__device__ __forceinline__ void block_order(int r, int w, int& x, int& y) {
    const int pair = r / (2 * w), q = r - pair * 2 * w; // row pair, index in it
    x = (q >> 3) * 4 + (q & 3);
    y = 2 * pair + ((q >> 2) & 1);
}
// BLOCKED false: the row-major order (the packed tile layout of igx_pack_tiles)
template <bool BLOCKED = true>
__device__ __forceinline__ bool local_to_global(const FrameArgs& fa, int lp, int& x, int& y) {
    if (fa.num_rays > 0) { x = lp; y = 0; return lp < fa.num_rays; }
    if (fa.tile_size <= 0) {
        if (BLOCKED && IGX_PIXEL_BLOCKS && (fa.width & 3) == 0 && (fa.height & 1) == 0) block_order(lp, fa.width, x, y);
        else { y = lp / fa.width; x = lp - y * fa.width; }
        return true;
    }
    int T = fa.tile_size;
    int k = lp / (T * T);
    int r = lp - k * T * T;
    int ty, tx;
    if (BLOCKED && IGX_PIXEL_BLOCKS && (T & 3) == 0) block_order(r, T, tx, ty);
    else { ty = r / T; tx = r - ty * T; }
    int t = fa.tile_offset + k * fa.tile_stride;
    int tyy = t / fa.tiles_x, txx = t - tyy * fa.tiles_x;
    x = txx * T + tx;
    y = tyy * T + ty;
    return x < fa.width && y < fa.height;
}

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

template <typename T>
__device__ __forceinline__ T uniform_load(const T* p) {
    return __builtin_amdgcn_readfirstlane(*p);
}

// ---------------------------------------------------------------------------
// Sharded streams (see PathBuf)
// ---------------------------------------------------------------------------
static_assert(NSH == 64 && BLOCK % 64 == 0 && NSH % WAVES_PER_BLOCK == 0, "one shard counter per lane of a wave");
static_assert(BLOCK == TSTACK_STRIDE, "traversal stacks are laid out for BLOCK threads");

// Records of all shards of a counter row: lane l reads shard l; wave-uniform.
// A path-stream counter is two words (class A records from the front of the
// shard, class B from its back, wave_append_paths); other streams leave the
// second word 0.
__device__ __forceinline__ int row_total(const int* row) {
    const int* r = row + lane_id() * CSTRIDE;
    int v = r[0] + r[1] + r[2];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return __builtin_amdgcn_readfirstlane(v);
}

// Wave g of the grid's G waves serves shard s = g % NSH, as the k-th of the
// K = G / NSH waves of that shard (grids are multiples of GRID_QUANTUM blocks).
struct WaveWork {
    int s, k, K;
};
__device__ __forceinline__ WaveWork wave_work() {
    const int g = __builtin_amdgcn_readfirstlane((int)blockIdx.x * WAVES_PER_BLOCK + (int)(threadIdx.x >> 6));
    return WaveWork{g % NSH, g / NSH, (int)gridDim.x * WAVES_PER_BLOCK / NSH};
}

// Storage index of path i of a freshly generated chunk: consecutive groups of
// 64 paths go round-robin to the shards, so every wave of the first bounce
// reads 64 neighbouring paths (8 pixels x spi 8).
__device__ __forceinline__ int gen_index(int i, int shard_cap) {
    return ((i >> 6) & (NSH - 1)) * shard_cap + ((i >> 12) << 6) + (i & 63);
}
// Shard counts of a generated chunk of n paths (written by lanes 0..NSH-1).
__device__ __forceinline__ int gen_shard_count(int n, int s) {
    const int rem = (n & (64 * NSH - 1)) - s * 64;
    return (n >> 12) * 64 + (rem < 0 ? 0 : (rem > 64 ? 64 : rem));
}

// Records of path-stream shard s: `a` of class A at offsets [0, a) and ab - a
// of class B at offsets shard_cap - 1 down to shard_cap - (ab - a); with a
// class-C region (PathBuf::c_base, FrameArgs::classify 4) n - ab of class C
// at its offsets [0, n - ab).  Position pos in [0, n) of the shard maps to
// stream index path_index(...) (stream_index for two-class streams), so
// consecutive positions, and so the 64 paths of one wave, share a class.
struct ShardCount {
    int a, ab, n;
};
__device__ __forceinline__ ShardCount shard_count(const int* cnt, int s) {
    const int a = uniform_load(cnt + s * CSTRIDE), b = uniform_load(cnt + s * CSTRIDE + 1);
    const int c = uniform_load(cnt + s * CSTRIDE + 2);
    return ShardCount{a, a + b, a + b + c};
}
__device__ __forceinline__ int stream_index(int s, int pos, int a, int shard_cap) {
    return s * shard_cap + (pos < a ? pos : shard_cap - 1 - (pos - a));
}
__device__ __forceinline__ int path_index(const PathBuf& b, int s, int pos, const ShardCount& sc) {
    return pos < sc.ab ? stream_index(s, pos, sc.a, b.shard_cap) : b.c_base + s * b.shard_cap + (pos - sc.ab);
}

// Wave-level compaction of the surviving paths (class A appended from the
// front of the wave's shard, class B from its back, class C from the front
// of the shard's class-C region: the next bounce's waves then trace paths of
// one class, e.g. all inside a dielectric) and of the shadow rays (A front,
// B back): one returning 64-bit atomic per counter (a/b counts in its two
// words; the class-C count in word 2), lanes 0-2 issue them in one
// instruction; positions inside the wave by ballot prefix.  `dst` is the
// record offset from the start of the shard (c_base added for class C).
// Needs every lane of the wave active.
// `claim` (k_extend's dynamic groups): lane 3 also takes the wave's next group
// of its shard from that shard's work counter in the same round trip
// (`claimed`, wave-uniform; -1 without `claim`), so the next group's path
// loads follow the stores without a second returning atomic in between.
__device__ __forceinline__ void wave_append_paths(bool alive, int cls, bool shadow, bool sh_b, int* cp, int* cs,
                                                  int shard_cap, int c_base, int sh_cap, int& dst, int& sdst,
                                                  int* claim = nullptr, int* claimed = nullptr) {
    const int lane = lane_id();
    const uint64_t ma = __ballot(alive && cls == 0), mb = __ballot(alive && cls == 1), mc = __ballot(alive && cls == 2);
    const uint64_t sa = __ballot(shadow && !sh_b), sb = __ballot(shadow && sh_b);
    const uint64_t below = (1ull << lane) - 1ull;
    const unsigned long long want = lane == 0   ? ((unsigned long long)__popcll(ma) | ((unsigned long long)__popcll(mb) << 32))
                                    : lane == 1 ? ((unsigned long long)__popcll(sa) | ((unsigned long long)__popcll(sb) << 32))
                                                : (unsigned long long)__popcll(mc);
    unsigned long long r = 0;
    int nx = 0;
    if (lane < 3 && want != 0) r = atomicAdd(reinterpret_cast<unsigned long long*>(lane == 0 ? cp : lane == 1 ? cs : cp + 2), want);
    if (claim && lane == 3) nx = atomicAdd(claim, 1);
    if (claim) *claimed = __builtin_amdgcn_readfirstlane(__shfl(nx, 3));
    const int lo = (int)(uint32_t)r, hi = (int)(uint32_t)(r >> 32);
    const int a0 = __shfl(lo, 0), b0 = __shfl(hi, 0), s0 = __shfl(lo, 1), t0 = __shfl(hi, 1), c0 = __shfl(lo, 2);
    dst = cls == 1   ? shard_cap - 1 - (b0 + __popcll(mb & below))
          : cls == 2 ? c_base + c0 + __popcll(mc & below)
                     : a0 + __popcll(ma & below);
    sdst = sh_b ? sh_cap - 1 - (t0 + __popcll(sb & below)) : s0 + __popcll(sa & below);
}



// ---------------------------------------------------------------------------
// generate: camera rays (gpu_generate_rays, mapping_gpu.art:618-667;
// make_camera_emitter, driver/emitter.art:6-16; perspective camera,
// camera/perspective.art:29-42; uniform pixel sampler, sampler/pixel_sampler.art:4-10).
// Slot i of the chunk holds path i; no compaction (tile padding slots are
// written as dead paths with depth 0), so no atomics.
// ---------------------------------------------------------------------------
// Path i of the chunk at its camera vertex (k_generate, and k_extend's fused
// bounce 0).  Path state layout: see PathState below.
struct GenPath {
    f3 o, d;
    uint32_t counter, seed;
    int depth;
};
__device__ __forceinline__ GenPath gen_path(const FrameArgs& fa, const SceneView& sv, int i) {
    int lp, sample, iter;
    slot_coords(fa, i, lp, sample, iter);
    int x, y;
    GenPath g{mk(0, 0, 0), mk(0, 0, 1), 1, 0, 0}; // depth 0: dead (tile padding)
    if (local_to_global(fa, lp, x, y)) {
        g.depth = 1;
        g.seed = create_random_seed(sample, iter, fa.frame, x, y, fa.seed);
        Rng rnd{g.seed, 1};
        if (fa.num_rays > 0) {
            // make_list_emitter (driver/emitter.art:18-30): no random draws
            const float* r = fa.rays + 8 * x;
            g.o = mk(r[0], r[1], r[2]);
            g.d = mk(r[3], r[4], r[5]);
        } else {
            float rx = rnd.next_f32();
            float ry = rnd.next_f32();
            float nx = 2 * ((float)x + rx) / (float)fa.width - 1;
            float ny = 1 - 2 * ((float)y + ry) / (float)fa.height;
            const DevCamera& c = sv.cam;
            f3 v = mk(c.scale_x * nx, c.scale_y * ny, 1);
            f3 w = mk(c.right[0] * v.x + c.up[0] * v.y + c.dir[0] * v.z,
                      c.right[1] * v.x + c.up[1] * v.y + c.dir[1] * v.z,
                      c.right[2] * v.x + c.up[2] * v.y + c.dir[2] * v.z);
            g.o = mk(c.eye[0], c.eye[1], c.eye[2]);
            g.d = normalize(w);
        }
        g.counter = rnd.counter;
    }
    return g;
}

#if IGX_PART == 0
__global__ void __launch_bounds__(BLOCK) k_generate(FrameArgs fa, SceneView sv, PathBuf out, float4* L, int* cnt0) {
    const int n = fa.chunk_pixels * fa.spi * fa.chunk_iters;
    if (blockIdx.x == 0 && threadIdx.x < NSH) cnt0[threadIdx.x * CSTRIDE] = gen_shard_count(n, threadIdx.x);
    for (int i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        L[i] = make_float4(0, 0, 0, 0);
        if (IGX_AOV && fa.aov_di) fa.aov_di[i] = fa.aov_nee[i] = make_float4(0, 0, 0, 0);
        const GenPath g = gen_path(fa, sv, i);
        const int e = gen_index(i, out.shard_cap);
        out.p0[e] = make_float4(g.o.x, g.o.y, g.o.z, __int_as_float(i));
        out.p1[e] = make_float4(g.d.x, g.d.y, g.d.z, __uint_as_float(g.counter | ((uint32_t)g.depth << 24)));
        out.p2[e] = make_float4(1, 1, 1, 0); // init_pt_raypayload (technique/pathtracer.art:33-38)
        out.p3[e] = make_float2(1.0f, __uint_as_float(g.seed));
    }
}

#endif

// ---------------------------------------------------------------------------
// One bounce of one path: closest hit + technique (gpu_traverse_primary +
// gpu_hit_shade + gpu_miss_shade, restating technique/pathtracer.art:52-200
// on_hit / on_shadow / on_bounce / on_miss).  Shared by the wavefront extend
// kernel and the tail kernel, so both produce bit-identical paths.
// ---------------------------------------------------------------------------
struct KernelCounters {
    int* cnt_in;
    int* cnt_out;
    int* cnt_shadow;
    unsigned long long* stats; // instrumentation counters (igx_get_stats: visits 0-12, phase clocks 16-19)
    int* work;                 // per-shard group counters of this bounce (FrameArgs::dynamic)
};

struct PathState {
    f3 o, d;
    uint32_t counter, seed;
    f3 contrib;
    float inv_pdf, eta;
    int slot, depth;
    int inside; // index of the enclosing entity the path travels in (trace_enclosed), -1: none known
};

struct ShadowRec {
    f3 o, d, color;
    float tmax;
};

// stream class of a surviving path (FrameArgs::classify): 1 B = inside a
// dielectric (eta != 1); 2 B = after a specular event; 3 B = inside a
// dielectric or its next ray crosses the world box of an enclosing entity
// (the paths whose traversal enters a large BLAS and that will likely shade
// a dielectric), A = the rest (wall-to-wall paths: short walks, diffuse)
// (the class only orders the stream, so the slab test may use the hardware
// reciprocal, v_rcp_f32, instead of three IEEE divisions)
__device__ __forceinline__ f3 fast_rcp3(f3 d) {
    return mk(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z));
}
__device__ __forceinline__ bool crosses_enclosing_box(const SceneView& sv, f3 o, f3 d) {
    const f3 id = fast_rcp3(d);
    bool hit = false;
    for (int k = 0; k < sv.num_enc && !hit; ++k) {
        const float4 lo = sv.enc_box[2 * k], hi = sv.enc_box[2 * k + 1];
        const float ax = (lo.x - o.x) * id.x, bx = (hi.x - o.x) * id.x;
        const float ay = (lo.y - o.y) * id.y, by = (hi.y - o.y) * id.y;
        const float az = (lo.z - o.z) * id.z, bz = (hi.z - o.z) * id.z;
        const float en = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
        const float ex = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
        hit = en <= ex && ex >= 0.0f;
    }
    return hit;
}
// shadow-ray class (FrameArgs::classify 3): B = the segment [0, tmax] of the
// shadow ray crosses an enclosing entity's box (its any-hit walk enters that
// BLAS), A = the rest; stored like the path classes (shard front / back)
__device__ __forceinline__ bool shadow_class_b(int enabled, const SceneView& sv, f3 o, f3 d, float tmax) {
    if (!enabled) return false;
    const f3 id = fast_rcp3(d);
    bool hit = false;
    for (int k = 0; k < sv.num_enc && !hit; ++k) {
        const float4 lo = sv.enc_box[2 * k], hi = sv.enc_box[2 * k + 1];
        const float ax = (lo.x - o.x) * id.x, bx = (hi.x - o.x) * id.x;
        const float ay = (lo.y - o.y) * id.y, by = (hi.y - o.y) * id.y;
        const float az = (lo.z - o.z) * id.z, bz = (hi.z - o.z) * id.z;
        const float en = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
        const float ex = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
        hit = en <= ex && ex >= 0.0f && en <= tmax;
    }
    return hit;
}
// 4: three classes, C = inside a dielectric, B = its next ray crosses an
// enclosing entity's world box, A = the rest (the fused schedule only: the
// split schedule's hit records have no class-C region)
__device__ __forceinline__ int path_class(int classify, const SceneView& sv, const PathState& ps) {
    switch (classify) {
    case 1: return ps.eta != 1.0f;
    case 2: return ps.inv_pdf == 0.0f;
    case 3: return ps.eta != 1.0f || crosses_enclosing_box(sv, ps.o, ps.d);
    case 4: return ps.eta != 1.0f ? 2 : crosses_enclosing_box(sv, ps.o, ps.d);
    default: return 0;
    }
}

__device__ __forceinline__ PathState path_from_records(float4 p0, float4 p1, float4 p2, float2 p3) {
    PathState s;
    s.o = f3of(p0);
    s.d = f3of(p1);
    const uint32_t sw = __float_as_uint(p0.w);
    s.slot = (int)(sw & SLOT_MASK);
    s.inside = (int)(sw >> SLOT_BITS) - 1;
    const uint32_t cd = __float_as_uint(p1.w);
    s.depth = (int)(cd >> 24);
    s.counter = cd & 0xFFFFFFu;
    s.contrib = f3of(p2);
    s.inv_pdf = p2.w;
    s.eta = p3.x;
    s.seed = __float_as_uint(p3.y);
    return s;
}
__device__ __forceinline__ PathState load_path(const PathBuf& in, int i) {
    return path_from_records(in.p0[i], in.p1[i], in.p2[i], in.p3[i]);
}

__device__ __forceinline__ void store_path(const PathBuf& out, int i, const PathState& s) {
    out.p0[i] = make_float4(s.o.x, s.o.y, s.o.z, __uint_as_float((uint32_t)s.slot | ((uint32_t)(s.inside + 1) << SLOT_BITS)));
    out.p1[i] = make_float4(s.d.x, s.d.y, s.d.z, __uint_as_float(s.counter | ((uint32_t)s.depth << 24)));
    out.p2[i] = make_float4(s.contrib.x, s.contrib.y, s.contrib.z, s.inv_pdf);
    out.p3[i] = make_float2(s.eta, __uint_as_float(s.seed));
}

__device__ __forceinline__ f3 handle_color(const SceneView& sv, f3 c) {
    if (sv.clamp > 0) return mk(fminf(c.x, sv.clamp), fminf(c.y, sv.clamp), fminf(c.z, sv.clamp));
    return c;
}

// Ray interval and visibility flags of the ray a path traces at its current
// vertex (camera / list ray at depth 1, bounce ray with the 0.001 offset
// afterwards; pathtracer.art:41, ray.art:21).
__device__ __forceinline__ void ray_extent(const FrameArgs& fa, const SceneView& sv, int depth, int slot, float& tmin,
                                           float& tmax, uint32_t& rflags) {
    if (depth == 1) {
        if (fa.num_rays > 0) {
            int lp, sample, iter;
            slot_coords(fa, slot, lp, sample, iter);
            tmin = fa.rays[8 * lp + 6];
            tmax = fa.rays[8 * lp + 7];
            rflags = 0;
        } else {
            tmin = sv.cam.tmin;
            tmax = sv.cam.tmax;
            rflags = RAY_CAMERA;
        }
    } else {
        tmin = 0.001f; // offset (pathtracer.art:41)
        tmax = FLT_MAX_;
        rflags = RAY_BOUNCE;
    }
}

// Shades the closest hit (or miss, hit_ent < 0) of the path's current ray and
// advances `ps` by one bounce.  Returns whether the path continues (ps then
// holds the bounced ray); fills the radiance gathered at this vertex (Lacc,
// has_l) and the NEE shadow ray (has_shadow, sr).
// A textured diffuse reflectance at the hit (DevMaterial::pad): the checker
// select(checkerboard(uvw * scale) == 1, kd1, kd) of texture/checkerboard.art:2
// on the texture coordinates (u, v, 0), interpolated with the hit's
// barycentrics (vec2_lerp2, shapes/trimesh.art:25; core/vector.art:150-153);
// math::wrap(x, 0, 2) as i32 % 2 per axis (core/math.art:88-91)
__device__ __forceinline__ int checker_bit(float x) {
    const float w = x - 2.0f * floorf(x / 2.0f);
    return ((int)w) % 2;
}
__device__ __forceinline__ void apply_texture(const SceneView& sv, DevMaterial& m, int ent_id, int prim, float hu, float hv) {
    if (__float_as_int(m.pad[0]) != 1) return;
    const int4 info = *reinterpret_cast<const int4*>(sv.ent + ENT_STRIDE * ent_id + 6); // shape type, material, vtx_off, idx_off
    if (info.x == 1) return; // analytic sphere: refused at upload
    const int4 f = sv.idx[info.w + prim];
    const float2 t0 = sv.uv[info.z + f.x], t1 = sv.uv[info.z + f.y], t2 = sv.uv[info.z + f.z];
    const float u = lerp2(t0.x, t1.x, t2.x, hu, hv), v = lerp2(t0.y, t1.y, t2.y, hu, hv);
    const float sc = m.pad[1];
    // node_checkerboard3(uvw * sc): ((a == b) == (c == 1)) with c of the zero w
    const int a = checker_bit(u * sc), b = checker_bit(v * sc), c = checker_bit(0.0f * sc);
    if ((a == b) == (c == 1)) {
        m.kd[0] = m.pad[2];
        m.kd[1] = m.pad[3];
        m.kd[2] = m.pad[4];
    }
}

// Shading sub-phase clock of the instrumented k_extend (CLK): the wave's
// shader clock since the previous mark goes to sub-phase k of its group's
// class (cls[20 + 4 * bucket + k]); marks sit in the hit path, executed by
// the wave for its active lanes.
template <bool CLK>
__device__ __forceinline__ void sub_mark(TraceStats* st, int k) {
    if constexpr (CLK) {
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        if (first_active_lane()) st->cls[20 + 4 * st->bucket + k] += now - st->t_sub;
        st->t_sub = now;
    }
}

template <bool FULL, bool CLK = false>
__device__ __forceinline__ bool shade_step(const FrameArgs& fa, const SceneView& sv, PathState& ps, int hit_ent,
                                           int hit_prim, float tmax, float hu, float hv, f3& Lacc, bool& has_l,
                                           bool& has_shadow, ShadowRec& sr, TraceStats* clk = nullptr) {
    Lacc = mk(0, 0, 0);
    has_l = false;
    has_shadow = false;
    const f3 rd = ps.d;
    if (hit_ent < 0) {
        // on_miss (pathtracer.art:136-163): every infinite, non-delta light
        for (int li = 0; li < sv.num_infinite; ++li) {
            const DevLight& Lt = sv.lights[li];
            if (Lt.delta) continue;
            f3 emit = mk(Lt.radiance[0], Lt.radiance[1], Lt.radiance[2]);
            float pdf_s = 1 / (4 * PI_);
            const float sel = sv.selector == SEL_UNIFORM ? 1.0f / (float)sv.num_lights : select_pdf(sv, li, ps.o);
            float mis = sv.nee ? 1 / (1 + ps.inv_pdf * sel * pdf_s) : 1.0f;
            Lacc = add(Lacc, handle_color(sv, mulf(mul(ps.contrib, emit), mis)));
            has_l = true;
        }
        return false;
    }
    int mat_id;
    Surface s = surface_element(sv, hit_ent, hit_prim, tmax, hu, hv, ps.o, rd, mat_id);
    // the full variant shades a copy of the material, into which a texture
    // writes its value at the hit; the basic one reads the table in place
    std::conditional_t<FULL, DevMaterial, const DevMaterial&> m = sv.mats[mat_id];
    if constexpr (FULL)
        if (sv.uv) apply_texture(sv, m, hit_ent, hit_prim, hu, hv);
    sub_mark<CLK>(clk, 0); // surface element + material
    // on_hit (pathtracer.art:114-134)
    if (m.light >= 0 && s.entering) {
        float dt = -dot(rd, s.local.n);
        if (dt > FLT_EPS_) {
            const DevLight& Lt = sv.lights[m.light];
            f3 emit = mk(Lt.radiance[0], Lt.radiance[1], Lt.radiance[2]);
            float pdf_s = light_pdf_direct_solid<FULL>(sv, Lt, ps.o, dt, tmax * tmax, hu, hv);
            const float sel = sv.selector == SEL_UNIFORM ? 1.0f / (float)sv.num_lights : select_pdf(sv, m.light, ps.o);
            float mis = sv.nee ? 1 / (1 + ps.inv_pdf * sel * pdf_s) : 1.0f;
            Lacc = add(Lacc, handle_color(sv, mulf(mul(ps.contrib, emit), mis)));
            has_l = true;
        }
    }
    sub_mark<CLK>(clk, 1); // emission
    // seed of the path's (sample, iteration, frame, pixel, user seed),
    // create_random_seed (core/random.art:34-43), carried in the path state
    Rng rnd{ps.seed, ps.counter};
    f3 out_dir = neg(rd);
    const bool specular = bsdf_is_specular<FULL>(m);
    // on_shadow (pathtracer.art:52-112)
    if (sv.nee && !specular && sv.num_lights > 0 && ps.depth + 1 <= sv.max_depth) {
        float sel_pdf;
        const int lid = select_light(sv, rnd, s.point, sel_pdf);
        const DevLight& Lt = sv.lights[lid];
        DirectSample ls = light_sample_direct<FULL>(sv, Lt, rnd, s);
        float pdf_l_s = pdf_as_solid(ls.pdf_value, ls.pdf_solid, ls.cos, ls.dist * ls.dist) * sel_pdf;
        if (pdf_l_s > FLT_EPS_ && ls.cos > FLT_EPS_) {
            f3 in_dir = ls.dir;
            float mis;
            if (Lt.delta) {
                mis = 1.0f;
            } else {
                float pdf_e_s = bsdf_pdf<FULL>(m, s, in_dir, out_dir); // pdf to sample the light by the bsdf
                mis = 1 / (1 + pdf_e_s / pdf_l_s);
            }
            float factor = ls.pdf_value / pdf_l_s;
            f3 ev = bsdf_eval<FULL>(m, s, in_dir, out_dir);
            sr.color = handle_color(sv, mulf(mul(ls.intensity, mul(ps.contrib, ev)), mis * factor));
            sr.o = s.point;
            if (Lt.infinite) {
                sr.d = in_dir;
                sr.tmax = FLT_MAX_;
            } else {
                sr.d = sub(ls.pos, s.point);
                sr.tmax = 1 - 0.001f;
            }
            has_shadow = true;
        }
    }
    sub_mark<CLK>(clk, 2); // NEE (light sample, BSDF eval / pdf)
    // on_bounce (pathtracer.art:165-200)
    if (!(ps.depth + 1 <= sv.max_depth)) return false;
    BsdfSample bs = bsdf_sample<FULL>(m, s, rnd, out_dir);
    if (!bs.valid) return false;
    f3 c2 = mul(ps.contrib, bs.color);
    float rr = 1.0f;
    if (ps.depth + 1 > sv.min_depth) {
        f3 e = mulf(c2, ps.eta * ps.eta);
        rr = clampf(fmaxf(fmaxf(e.x, e.y), e.z), 0.05f, 0.95f); // russian_roulette_pbrt
    }
    if (rnd.next_f32() >= rr) return false;
    ps.inv_pdf = specular ? 0 : 1 / bs.pdf;
    ps.contrib = mulf(c2, 1 / rr);
    ps.eta = ps.eta * bs.eta;
    // the entity the bounced ray travels in: entering an enclosing entity by
    // transmission puts the path inside it, leaving by transmission or
    // hitting anything else outside; a reflection inside keeps it inside
    const int enc = sv.ent_enc[hit_ent];
    if (enc < 0) {
        ps.inside = -1;
    } else if (dot(bs.in_dir, s.face_normal) * dot(rd, s.face_normal) > 0) { // continued through the surface
        ps.inside = s.entering ? enc : -1;
    } else if (ps.inside != enc) {
        ps.inside = -1;
    }
    ps.o = s.point;
    ps.d = bs.in_dir;
    ps.counter = rnd.counter;
    ps.depth = ps.depth + 1;
    return true;
}

// One bounce of one path: closest hit + shading.  Used by the tail kernel; the
// wavefront runs the same two halves as k_trace + k_shade, so both produce
// bit-identical paths.
// Instrumentation of k_extend's phases: the wave's shader clock (s_memtime,
// a read of the counter) since the previous mark is added to phase k; marks
// sit at wave-uniform points.
__device__ __forceinline__ void phase_mark(TraceStats& st, unsigned long long& last, int k) {
    // the phase's memory operations completed, and no instruction moves across the mark
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    st.cyc[k] += now - last;
    last = now;
}
template <bool STATS, int V>
__device__ __forceinline__ bool extend_step(const FrameArgs& fa, const SceneView& sv, const TStack& ts, PathState& ps, f3& Lacc,
                                            bool& has_l, bool& has_shadow, ShadowRec& sr, TraceStats& st) {
    float tmin, tmax;
    uint32_t rflags;
    ray_extent(fa, sv, ps.depth, ps.slot, tmin, tmax, rflags);
    int hit_ent, hit_prim;
    float hu = 0, hv = 0;
    // a ray inside an enclosing entity hits it first: its BLAS alone decides
    // (the full traversal from the TLAS root only when that finds nothing)
    trace_path_ray<STATS, V>(sv, ps.inside, ps.o, ps.d, tmin, tmax, rflags, ts, hit_ent, hit_prim, hu, hv, st);
    if (STATS && hit_ent >= 0) st.hits++;
    return shade_step<variant_full(V)>(fa, sv, ps, hit_ent, hit_prim, tmax, hu, hv, Lacc, has_l, has_shadow, sr);
}

__device__ __forceinline__ void add_radiance(float4* L, int slot, f3 c) {
    float4 l = L[slot];
    L[slot] = make_float4(l.x + c.x, l.y + c.y, l.z + c.z, 0);
}
// an AOV's per-path slot (FrameArgs::aov_di / aov_nee; kernel-argument pointer: a scalar branch)
// ON: compiled in (the wavefront kernels carry it in their full-shading
// variant only, which an aov_mis scene selects; the shadow kernels always)
template <bool ON = true>
__device__ __forceinline__ void add_aov(float4* A, int slot, f3 c) {
    if (ON && IGX_AOV && A) add_radiance(A, slot, c);
}

// extend_step of the instrumented k_extend (STATS): the trace and shade halves
// with phase clocks between them (load -> 0, trace -> 1, shade -> 2), and the
// per-class counters of the wave's group (`bucket`: camera, A, B, C; lane 0
// adds the wave's trace / shade cycles, one group, its wave-level node-loop
// iterations and its lanes' node visits, both reduced over the wave).
template <int V>
__device__ __forceinline__ bool extend_step_instrumented(const FrameArgs& fa, const SceneView& sv, const TStack& ts, float4* L,
                                                      PathState& ps, bool act, int bucket, bool& has_shadow, ShadowRec& sr,
                                                      TraceStats& st, unsigned long long& t_last) {
    int hit_ent = -1, hit_prim = -1;
    float hu = 0, hv = 0, tmin = 0, tmax = 0;
    uint32_t rflags = 0;
    bool alive = false;
    phase_mark(st, t_last, 0);
    const unsigned long long wn0 = st.wnodes, ln0 = st.nodes;
    if (act) {
        ray_extent(fa, sv, ps.depth, ps.slot, tmin, tmax, rflags);
        trace_path_ray<true, V>(sv, ps.inside, ps.o, ps.d, tmin, tmax, rflags, ts, hit_ent, hit_prim, hu, hv, st);
        if (hit_ent >= 0) st.hits++;
    }
    const unsigned long long c_tr = st.cyc[1];
    phase_mark(st, t_last, 1);
    // wnodes counts on the first active lane of each iteration, so the wave's
    // iterations are the sum over its lanes (as flush_stats reduces them)
    uint32_t visits = (uint32_t)(st.nodes - ln0), witers = (uint32_t)(st.wnodes - wn0);
    for (int off = 32; off > 0; off >>= 1) {
        visits += __shfl_xor(visits, off);
        witers += __shfl_xor(witers, off);
    }
    if (lane_id() == 0) {
        st.cls[bucket] += st.cyc[1] - c_tr;
        st.cls[8 + bucket] += 1;
        st.cls[12 + bucket] += witers;
        st.cls[16 + bucket] += visits;
    }
    st.bucket = bucket;
    st.t_sub = t_last;
    unsigned long long sub0 = 0;
    for (int k = 0; k < 3; ++k) sub0 += st.cls[20 + 4 * bucket + k];
    if (act) {
        f3 Lacc;
        bool has_l;
        alive = shade_step<variant_full(V), true>(fa, sv, ps, hit_ent, hit_prim, tmax, hu, hv, Lacc, has_l, has_shadow, sr, &st);
        if (has_l) {
            add_radiance(L, ps.slot, Lacc);
            add_aov<variant_full(V)>(fa.aov_di, ps.slot, Lacc);
        }
    }
    const unsigned long long c_sh = st.cyc[2];
    phase_mark(st, t_last, 2);
    if (lane_id() == 0) {
        st.cls[4 + bucket] += st.cyc[2] - c_sh;
        // sub-phase 3: the rest of the shade phase (BSDF sample, roulette, misses)
        unsigned long long sub1 = 0;
        for (int k = 0; k < 3; ++k) sub1 += st.cls[20 + 4 * bucket + k];
        st.cls[20 + 4 * bucket + 3] += (st.cyc[2] - c_sh) - (sub1 - sub0);
    }
    return alive;
}

template <bool STATS>
__device__ __forceinline__ void flush_stats(const TraceStats& st, unsigned long long* stats, int base, bool with_hits) {
    // slots: base+0..3 nodes/leaves/tris/blas, 8 hits, 9+base/4*2 .. wave node / leaf iterations
    unsigned long long a = st.nodes, b = st.leaves, c = st.tris, e = st.blas, h = st.hits, wn = st.wnodes, wl = st.wleaves;
    unsigned long long tl = st.tlas_nodes, h0 = st.hot[0], h1 = st.hot[1], h2 = st.hot[2];
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_down(a, off);
        b += __shfl_down(b, off);
        c += __shfl_down(c, off);
        e += __shfl_down(e, off);
        h += __shfl_down(h, off);
        wn += __shfl_down(wn, off);
        wl += __shfl_down(wl, off);
        tl += __shfl_down(tl, off);
        h0 += __shfl_down(h0, off);
        h1 += __shfl_down(h1, off);
        h2 += __shfl_down(h2, off);
    }
    if (lane_id() == 0) {
        atomicAdd(&stats[base + 0], a);
        atomicAdd(&stats[base + 1], b);
        atomicAdd(&stats[base + 2], c);
        atomicAdd(&stats[base + 3], e);
        if (with_hits) atomicAdd(&stats[8], h);
        atomicAdd(&stats[9 + (base / 4) * 2], wn);
        atomicAdd(&stats[10 + (base / 4) * 2], wl);
        if (base == 0) { // closest-hit node visits: in the TLAS, at hot-order ranks < 256 / 512 / 1280
            atomicAdd(&stats[50], tl);
            atomicAdd(&stats[51], h0);
            atomicAdd(&stats[52], h1);
            atomicAdd(&stats[53], h2);
        }
        if (st.cyc[0] | st.cyc[1] | st.cyc[2] | st.cyc[3]) {
            for (int k = 0; k < 4; ++k) atomicAdd(&stats[16 + k], st.cyc[k]);
            if (st.cls)
                for (int k = 0; k < 20; ++k)
                    if (st.cls[k]) atomicAdd(&stats[20 + k], st.cls[k]);
            if (st.cls) // shading sub-phase clocks by class (surface, emission, NEE, rest)
                for (int k = 0; k < 16; ++k)
                    if (st.cls[20 + k]) atomicAdd(&stats[54 + k], st.cls[20 + k]);
        }
    }
}

// Dynamic distribution of a launch's groups of 64 stream positions: the
// wave takes the next group of shard s from that shard's counter (work +
// s * CSTRIDE, one returning atomic per group); once s is exhausted it marks
// s in the launch's mask of exhausted shards (work + CROW, 64 bits), reads the
// mask (a coherent load: the scalar cache would hold it stale for the whole
// launch) and moves on to the next shard still open.  Returns the group index
// in shard s (s and n updated), or -1 once every shard is exhausted.  Waves
// that drew short paths take more groups, so a launch no longer waits on the
// wave with the slowest fixed share.
// `claimed` >= 0: the wave already took group `claimed` of shard s (k_extend's
// append, wave_append_paths): no atomic for it.
template <class CountOf>
__device__ __forceinline__ int take_group(int* work, int& s, uint64_t& done, int n, CountOf count_of, int claimed = -1) {
    unsigned long long* const done_mask = reinterpret_cast<unsigned long long*>(work + CROW);
    for (;;) {
        if (!((done >> s) & 1ull)) {
            int v = claimed;
            claimed = -1;
            if (v < 0) {
                v = 0;
                if (lane_id() == 0) v = atomicAdd(work + s * CSTRIDE, 1);
                v = __builtin_amdgcn_readfirstlane(v);
            }
            if (v * 64 < n) return v;
            // one atomicOr per shard, not one per wave that finds it exhausted
            if (lane_id() == 0 && !((__hip_atomic_load(done_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> s) & 1ull))
                atomicOr(done_mask, 1ull << s);
            done |= 1ull << s;
        }
        unsigned long long m = 0;
        if (lane_id() == 0) m = __hip_atomic_load(done_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        done |= (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)m) |
                ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(m >> 32)) << 32);
        const uint64_t open = ~done;
        if (!open) return -1;
        const int r = (s + 1) & (NSH - 1);
        const uint64_t rot = (open >> r) | (r ? (open << (NSH - r)) : 0ull);
        s = (r + __ffsll((unsigned long long)rot) - 1) & (NSH - 1);
        n = count_of(s);
    }
}

// path i of a generated chunk at its camera vertex (k_extend's fused bounce 0)
__device__ __forceinline__ PathState camera_path(const FrameArgs& fa, const SceneView& sv, int i) {
    const GenPath g = gen_path(fa, sv, i);
    PathState ps;
    ps.o = g.o;
    ps.d = g.d;
    ps.counter = g.counter;
    ps.seed = g.seed;
    ps.depth = g.depth;
    ps.slot = i;
    ps.contrib = mk(1, 1, 1); // init_pt_raypayload (technique/pathtracer.art:33-38)
    ps.inv_pdf = 0;
    ps.eta = 1.0f;
    ps.inside = -1;
    return ps;
}

// ---------------------------------------------------------------------------
// extend kernel: one bounce for every live path, compacted outputs.  Each
// wave walks its shard of the input stream and appends survivors and shadow
// rays to the same shard of the output streams (wave_append_paths): no block
// barrier, so a wave whose rays finish early moves on to its next 64 paths.
// ---------------------------------------------------------------------------
template <int V0, bool STATS, bool LDS>
__global__ void __launch_bounds__(BLOCK, LDS ? EXTEND_WAVES_LDS : (variant_full(V0) ? EXTEND_WAVES_FULL : EXTEND_WAVES)) k_extend(FrameArgs fa, SceneView gsv, PathBuf in, PathBuf out, ShadowBuf sh,
                                                  float4* L, KernelCounters kc, int tail_threshold) {
    constexpr int V = LDS ? kernel_variant(V0, true) : (EXTEND_TREELET ? kernel_variant(V0, false) : V0); // LDS-staged nodes: padded stride; global tables: treelet (device_scene.h) or global node loads
    __shared__ int stack_mem[LDS_STACK * BLOCK];
    extern __shared__ float4 lds_scene[];
    const TStack ts = make_tstack(stack_mem, LDS_STACK, gsv.spill);
    // gen_n > 0 (bounce 0 with generation fused; the host launches it only
    // when n > tail): the paths are the chunk's camera paths in k_generate's
    // shard order, built here instead of being read from the input stream.
    const bool gen = fa.gen_n > 0;
    if (!gen && row_total(kc.cnt_in) <= tail_threshold) return; // k_finish takes the remaining paths (block-uniform)
    const SceneView sv = LDS ? stage_scene_lds<BLOCK>(gsv, lds_scene) : stage_treelet<BLOCK>(gsv, lds_scene);
    TraceStats st{0, 0, 0, 0, 0, 0, 0};
    __shared__ unsigned long long cls_mem[STATS ? WAVES_PER_BLOCK * 36 : 1]; // per-class counters (instrumented)
    if constexpr (STATS) {
        st.cls = cls_mem + 36 * (threadIdx.x >> 6);
        if (lane_id() < 36) st.cls[lane_id()] = 0;
    }
    const WaveWork w = wave_work();
    // Groups of 64 positions of shard s: statically every K-th group from
    // the wave's own (grid-stride), or (fa.dynamic) the next group a shard
    // counter hands out, moving on to the following shards once the own is
    // exhausted -- waves that drew fast paths take more groups, so a launch
    // does not wait on the wave with the slowest share.  Survivors always go
    // to the shard the group came from (its output never exceeds its input).
    int s = w.s;
    auto count_of = [&](int sh_) {
        if (gen) {
            const int g = gen_shard_count(fa.gen_n, sh_);
            return ShardCount{g, g, g};
        }
        return shard_count(kc.cnt_in, sh_);
    };
    ShardCount sc = count_of(s);
    uint64_t done = 0; // shards this wave knows to be exhausted (dynamic)
    int p0 = w.k * 64;
    int claimed = -1; // next group of shard s, taken by the previous group's append (IGX_CLAIM_NEXT)
    unsigned long long t_last = STATS ? __builtin_amdgcn_s_memtime() : 0; // phase clocks (instrumented builds)
    for (;;) {
        if (fa.dynamic) {
            const int g = take_group(kc.work, s, done, sc.n, [&](int sh_) {
                sc = count_of(sh_);
                return sc.n;
            }, claimed);
            if (g < 0) break;
            p0 = g * 64;
        } else if (p0 >= sc.n) {
            break;
        }
        if (STATS) phase_mark(st, t_last, 3); // group distribution
        const int ns = sc.n;
        int* const c_out = kc.cnt_out + s * CSTRIDE;
        int* const c_sh = kc.cnt_shadow + s * CSTRIDE;
        const int q = p0 + lane_id();
        const int pos = (fa.reverse && !gen) ? ns - 1 - q : q; // reverse: longest classes first
        bool alive = false, has_shadow = false;
        PathState ps;
        ShadowRec sr;
        ps.depth = 0;
        if (q < ns) {
            if (gen) { // inverse of gen_index
                const int i = ((pos >> 6) << 12) | (s << 6) | (pos & 63);
                ps = camera_path(fa, sv, i);
                L[i] = make_float4(0, 0, 0, 0);
                if (variant_full(V0) && IGX_AOV && fa.aov_di) fa.aov_di[i] = fa.aov_nee[i] = make_float4(0, 0, 0, 0);
            } else {
                ps = load_path(in, path_index(in, s, pos, sc));
            }
            if (!STATS && ps.depth > 0) {
                f3 Lacc;
                bool has_l;
                alive = extend_step<STATS, V>(fa, sv, ts, ps, Lacc, has_l, has_shadow, sr, st);
                if (has_l) {
                    add_radiance(L, ps.slot, Lacc);
                    add_aov<variant_full(V0)>(fa.aov_di, ps.slot, Lacc);
                }
            }
        }
        if constexpr (STATS) {
            // class of the wave's group (wave-uniform): camera, A, B, C
            const int pg = (fa.reverse && !gen) ? ns - 1 - p0 : p0;
            const int bucket = gen ? 0 : (pg < sc.a ? 1 : pg < sc.ab ? 2 : 3);
            alive = extend_step_instrumented<V>(fa, sv, ts, L, ps, q < ns && ps.depth > 0, bucket, has_shadow, sr, st, t_last);
        }
        int dst, sdst;
        // dynamic groups: the append's round trip also takes the next group of
        // shard s, unless s is known exhausted
        int* const claim = (IGX_CLAIM_NEXT && fa.dynamic && !((done >> s) & 1ull)) ? kc.work + s * CSTRIDE : nullptr;
        wave_append_paths(alive, path_class(fa.classify, sv, ps), has_shadow,
                          has_shadow && shadow_class_b(fa.shadow_classes, sv, sr.o, sr.d, sr.tmax), c_out, c_sh, out.shard_cap,
                          out.c_base, sh.shard_cap, dst, sdst, claim, &claimed);
        if (!claim) claimed = -1;
        if (alive) store_path(out, s * out.shard_cap + dst, ps);
        if (has_shadow) {
            const int e = s * sh.shard_cap + sdst;
            sh.s0[e] = make_float4(sr.o.x, sr.o.y, sr.o.z, __int_as_float(ps.slot));
            sh.s1[e] = make_float4(sr.d.x, sr.d.y, sr.d.z, sr.tmax);
            sh.s2[e] = make_float4(sr.color.x, sr.color.y, sr.color.z, 0);
        }
        if (!fa.dynamic) p0 += w.K * 64;
        if (STATS) phase_mark(st, t_last, 3);
    }
    if (STATS) flush_stats<STATS>(st, kc.stats, 0, true);
}

// ---------------------------------------------------------------------------
// trace: closest hit of every live path's current ray (gpu_traverse_primary,
// mapping_gpu.art:45-68).  Traversal only, so the kernel stays small enough
// for high occupancy (the latency of the dependent node loads is what bounds
// it); each lane writes its own hit record (same index as its path).
// ---------------------------------------------------------------------------
template <int V0, bool STATS, int WAVES, bool LDS>
__global__ void __launch_bounds__(BLOCK, WAVES) k_trace(FrameArgs fa, SceneView gsv, PathBuf in, HitBuf hits,
                                                      const int* cnt, int tail_threshold, unsigned long long* stats) {
    constexpr int V = LDS ? kernel_variant(V0, true) : V0; // LDS-staged nodes: padded stride; global tables: global node loads (no treelet)
    __shared__ int stack_mem[LDS_STACK * BLOCK];
    extern __shared__ float4 lds_scene[];
    const TStack ts = make_tstack(stack_mem, LDS_STACK, gsv.spill);
    if (row_total(cnt) <= tail_threshold) return; // k_finish takes the remaining paths
    const SceneView sv = LDS ? stage_scene_lds<BLOCK>(gsv, lds_scene) : stage_treelet<BLOCK>(gsv, lds_scene);
    TraceStats st{0, 0, 0, 0, 0, 0, 0};
    const WaveWork w = wave_work();
    const ShardCount sc = shard_count(cnt, w.s);
    const int ns = sc.n;
    for (int pos = w.k * 64 + lane_id(); pos < ns; pos += w.K * 64) {
        const int i = path_index(in, w.s, pos, sc);
        float4 p0 = in.p0[i], p1 = in.p1[i];
        int depth = (int)(__float_as_uint(p1.w) >> 24);
        int hit_ent = -1, hit_prim = -1;
        float hu = 0, hv = 0, tmax = 0;
        if (depth > 0) {
            float tmin;
            uint32_t rflags;
            ray_extent(fa, sv, depth, (int)(__float_as_uint(p0.w) & SLOT_MASK), tmin, tmax, rflags);
            trace_ray<false, STATS, V>(sv, f3of(p0), f3of(p1), tmin, tmax, rflags, ts, hit_ent, hit_prim, hu, hv, st);
            if (STATS && hit_ent >= 0) st.hits++;
        }
        hits.h[i] = make_float4(tmax, hu, hv, __int_as_float(hit_ent));
        hits.prim[i] = hit_prim;
    }
    if (STATS) flush_stats<STATS>(st, stats, 0, true);
}

// ---------------------------------------------------------------------------
// shade: the path-tracer step at every hit / miss (gpu_hit_shade +
// gpu_miss_shade, mapping_gpu.art:114-266) for all materials at once, with
// wave-level compaction of surviving paths and shadow rays.
// ---------------------------------------------------------------------------
template <bool FULL>
__global__ void __launch_bounds__(BLOCK) k_shade(FrameArgs fa, SceneView sv, PathBuf in, HitBuf hits, PathBuf out,
                                                 ShadowBuf sh, float4* L, KernelCounters kc, int tail_threshold) {
    if (row_total(kc.cnt_in) <= tail_threshold) return;
    const WaveWork w = wave_work();
    const ShardCount sc = shard_count(kc.cnt_in, w.s);
    const int ns = sc.n;
    int* const c_out = kc.cnt_out + w.s * CSTRIDE;
    int* const c_sh = kc.cnt_shadow + w.s * CSTRIDE;
    for (int p0 = w.k * 64; p0 < ns; p0 += w.K * 64) {
        const int pos = p0 + lane_id();
        const int i = path_index(in, w.s, pos, sc);
        bool alive = false, has_shadow = false;
        PathState ps;
        ShadowRec sr;
        ps.depth = 0;
        if (pos < ns) {
            ps = load_path(in, i);
            if (ps.depth > 0) {
                float4 h = hits.h[i];
                int prim = hits.prim[i];
                f3 Lacc;
                bool has_l;
                alive = shade_step<FULL>(fa, sv, ps, __float_as_int(h.w), prim, h.x, h.y, h.z, Lacc, has_l, has_shadow, sr);
                if (has_l) {
                    add_radiance(L, ps.slot, Lacc);
                    add_aov<FULL>(fa.aov_di, ps.slot, Lacc);
                }
            }
        }
        int dst, sdst;
        wave_append_paths(alive, path_class(fa.classify, sv, ps), has_shadow,
                          has_shadow && shadow_class_b(fa.shadow_classes, sv, sr.o, sr.d, sr.tmax), c_out, c_sh, out.shard_cap,
                          out.c_base, sh.shard_cap, dst, sdst);
        if (alive) store_path(out, w.s * out.shard_cap + dst, ps);
        if (has_shadow) {
            const int e = w.s * sh.shard_cap + sdst;
            sh.s0[e] = make_float4(sr.o.x, sr.o.y, sr.o.z, __int_as_float(ps.slot));
            sh.s1[e] = make_float4(sr.d.x, sr.d.y, sr.d.z, sr.tmax);
            sh.s2[e] = make_float4(sr.color.x, sr.color.y, sr.color.z, 0);
        }
    }
}

// ---------------------------------------------------------------------------
// tail kernel: once few paths remain, each lane runs its path to the end
// (extend + inline any-hit shadow ray per bounce), replacing dozens of nearly
// empty per-bounce launches.  Same per-path arithmetic and the same radiance
// accumulation order as the wavefront kernels.
// ---------------------------------------------------------------------------
template <int V0, bool STATS, bool LDS>
__global__ void __launch_bounds__(BLOCK) k_finish(FrameArgs fa, SceneView gsv, PathBuf in, float4* L, const int* cnt,
                                                  int tail_threshold, unsigned long long* stats,
                                                  unsigned long long* tail_counts) {
    constexpr int V = LDS ? kernel_variant(V0, true) : V0; // LDS-staged nodes: padded stride; global tables: global node loads (the tail kernel stages no treelet)
    __shared__ int stack_mem[LDS_STACK * BLOCK];
    extern __shared__ float4 lds_scene[];
    const TStack ts = make_tstack(stack_mem, LDS_STACK, gsv.spill);
    const int n = row_total(cnt);
    if (n > tail_threshold || n == 0) return; // the wavefront kernels own this bounce
    const SceneView sv = LDS ? stage_scene_lds<BLOCK>(gsv, lds_scene) : stage_treelet<BLOCK>(gsv, lds_scene);
    TraceStats st{0, 0, 0, 0, 0, 0, 0};
    TraceStats sst{0, 0, 0, 0, 0, 0, 0};
    unsigned long long bounces = 0, shadows = 0;
    const WaveWork w = wave_work();
    const ShardCount sc = shard_count(cnt, w.s);
    const int ns = sc.n;
    for (int pos = w.k * 64 + lane_id(); pos < ns; pos += w.K * 64) {
        PathState ps = load_path(in, path_index(in, w.s, pos, sc));
        if (ps.depth <= 0) continue;
        for (;;) {
            f3 Lacc;
            bool has_l, has_shadow;
            ShadowRec sr;
            bool alive = extend_step<STATS, V>(fa, sv, ts, ps, Lacc, has_l, has_shadow, sr, st);
            if (has_l) {
                add_radiance(L, ps.slot, Lacc);
                add_aov<variant_full(V0)>(fa.aov_di, ps.slot, Lacc);
            }
            if (has_shadow) {
                ++shadows;
                float tm = sr.tmax;
                int e, p;
                float u, v;
                if (!trace_ray<true, STATS, V>(sv, sr.o, sr.d, 0.001f, tm, RAY_SHADOW, ts, e, p, u, v, sst)) {
                    add_radiance(L, ps.slot, sr.color);
                    add_aov<variant_full(V0)>(fa.aov_nee, ps.slot, sr.color);
                }
            }
            if (!alive) break;
            ++bounces;
        }
    }
    // ray statistics of the tail (continuation rays, valid shadow rays): one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        bounces += __shfl_down(bounces, off);
        shadows += __shfl_down(shadows, off);
    }
    if (lane_id() == 0 && (bounces | shadows)) {
        atomicAdd(&tail_counts[0], bounces);
        atomicAdd(&tail_counts[1], shadows);
    }
    if (STATS) {
        flush_stats<STATS>(st, stats, 0, true);
        flush_stats<STATS>(sst, stats, 4, false);
    }
}

// ---------------------------------------------------------------------------
// tail kernel with lane pairs (global-table scenes): on the soups a tail
// path's bounce is two dependent walks through HBM-resident tables (closest
// hit, then the NEE shadow ray), and the longest path sets the tail's length.
// Both rays of a bounce start at the same shading point and do not depend on
// each other, so here the even lane of a pair carries the path and traces its
// closest hits while the odd lane traces the path's shadow rays: the two walks
// overlap, and both lanes step through the same instructions (per-lane any-hit
// flag, trav_step_core).  Radiance is added in the wavefront's order (emission
// of bounce k, shadow ray of bounce k, emission of bounce k + 1), so the image
// is bit-identical to k_finish.
// ---------------------------------------------------------------------------
// occupancy target of k_finish_pairs (waves per SIMD).  The compiler's own
// choice is 212-234 VGPRs = 2 waves; 3 waves (168 VGPRs, ~30 spilled) hides
// more of the long tail's latency: soup-16M frame 70.6 -> 69.4 ms, soup-1M
// 54.3 -> 53.2 ms (tools/exp_n.sh, round 3)
#ifndef FINISH_PAIRS_WAVES
#define FINISH_PAIRS_WAVES 3
#endif
// Pairs step independently (round 6): a wave keeps stepping its busy lanes
// until TAIL_READY pairs have finished both walks (or none is busy), then
// processes those pairs alone (shadow verdict, shading, hand-over, next
// walks), so a pair no longer waits each bounce for the slowest walk of the
// wave.  Soup-1M 2-iteration frame 72.4-72.8 -> 71.8 ms (tail 4.1 -> 3.6-3.7
// ms), soup-16M and S-deep within noise, identical images (4 / 8 / 16 ready
// pairs alike; profiles/r06_ab_tail_pairs_desync.log).  The soup-16M tail
// stays ~5.5 ms: its first 8 bounces (98 K paths) take 3.2 ms of it
// (profiles/r06_tail_vs_max_depth_soup16.log), each a chain of dependent
// node fetches at 3 waves per SIMD.
constexpr int TAIL_READY = 8;
template <int V0, bool STATS>
__global__ void __launch_bounds__(BLOCK, FINISH_PAIRS_WAVES) k_finish_pairs(FrameArgs fa, SceneView gsv, PathBuf in, float4* L, const int* cnt,
                                                        int tail_threshold, unsigned long long* stats,
                                                        unsigned long long* tail_counts) {
    constexpr int V = V0; // global node loads (no treelet)
    __shared__ int stack_mem[LDS_STACK * BLOCK];
    extern __shared__ float4 lds_scene[];
    const TStack ts = make_tstack(stack_mem, LDS_STACK, gsv.spill);
    const int n = row_total(cnt);
    if (n > tail_threshold || n == 0) return; // the wavefront kernels own this bounce
    const SceneView sv = stage_treelet<BLOCK>(gsv, lds_scene);
    TraceStats st{0, 0, 0, 0, 0, 0, 0};
    TraceStats sst{0, 0, 0, 0, 0, 0, 0};
    unsigned long long bounces = 0, shadows = 0;
    const WaveWork w = wave_work();
    const ShardCount sc = shard_count(cnt, w.s);
    const int ns = sc.n;
    const int lane = lane_id(), partner = lane ^ 1;
    const bool path_lane = (lane & 1) == 0;
    constexpr uint64_t EVEN = 0x5555555555555555ull;
    for (int pos0 = w.k * 32; pos0 < ns; pos0 += w.K * 32) { // 32 paths per wave and pass
        const int pos = pos0 + (lane >> 1);
        PathState ps;
        ps.depth = 0;
        if (path_lane && pos < ns) ps = load_path(in, path_index(in, w.s, pos, sc));
        bool tracing = path_lane && pos < ns && ps.depth > 0; // path lane: its current ray needs a closest hit
        bool sh_trace = false;                                  // odd lane: a shadow ray to trace
        bool had_shadow = false;                                // path lane: its last shadow ray is out
        ShadowRec sr;
        f3 so = mk(0, 0, 0), sd = mk(0, 0, 1);
        float stmax = 0;
        Trav t;
        bool busy = false, enclosed = false;
        bool fresh = false; // this lane's walk has run since its pair was last processed
        TraceStats& tst = path_lane ? st : sst;
        bool start = true;  // the pair is at a bounce boundary: start its walks
        for (;;) {
            // ---- start the walks of the pairs at a bounce boundary ----
            if (start) {
                if (tracing) {
                    float tmin, tmax;
                    uint32_t rflags;
                    ray_extent(fa, sv, ps.depth, ps.slot, tmin, tmax, rflags);
                    enclosed = ps.inside >= 0 && trav_init_enclosed<STATS>(sv, t, ps.inside, ps.o, ps.d, tmin, tmax, rflags, ts, tst);
                    if (!enclosed) trav_init(sv, t, ps.o, ps.d, tmin, tmax, rflags, ts);
                    busy = fresh = true;
                } else if (sh_trace) {
                    trav_init(sv, t, so, sd, 0.001f, stmax, RAY_SHADOW, ts);
                    busy = fresh = true;
                }
                start = false;
            }
            // ---- step the busy lanes until TAIL_READY pairs (or all) have finished
            // both walks: a pair does not wait for the slowest walk of the wave ----
            uint64_t ready;
            for (;;) {
                const uint64_t bm = __ballot(busy), fm = __ballot(fresh);
                ready = ((fm | (fm >> 1)) & EVEN) & ~((bm | (bm >> 1)) & EVEN);
                if (bm == 0 || __popcll(ready) >= TAIL_READY) break;
                if (busy && trav_step_core<2, STATS, V>(sv, t, ts, tst, !path_lane)) {
                    busy = false;
                    if (tracing && enclosed && !t.found) {
                        // an enclosed walk that found nothing: the full traversal from the TLAS root
                        float tmin, tmax;
                        uint32_t rflags;
                        ray_extent(fa, sv, ps.depth, ps.slot, tmin, tmax, rflags);
                        trav_init(sv, t, ps.o, ps.d, tmin, tmax, rflags, ts);
                        enclosed = false;
                        busy = true;
                    }
                }
            }
            if (ready == 0) break; // no walk running and none to process: every pair is done
            if (!((ready >> (lane & ~1)) & 1)) continue;
            // ---- a ready pair: its shadow verdict, then the shading of its hit ----
            fresh = false;
            const bool occluded = __shfl(sh_trace && t.found, partner) != 0;
            if (path_lane && had_shadow && !occluded) {
                add_radiance(L, ps.slot, sr.color);
                add_aov<variant_full(V0)>(fa.aov_nee, ps.slot, sr.color);
            }
            bool cont = false, has_shadow = false;
            if (tracing) {
                if (STATS && t.hit_ent >= 0) st.hits++;
                f3 Lacc;
                bool has_l;
                cont = shade_step<variant_full(V)>(fa, sv, ps, t.hit_ent, t.hit_prim, t.tmax, t.hu, t.hv, Lacc, has_l, has_shadow, sr);
                if (has_l) {
                    add_radiance(L, ps.slot, Lacc);
                    add_aov<variant_full(V0)>(fa.aov_di, ps.slot, Lacc);
                }
                if (has_shadow) ++shadows;
                if (cont) ++bounces;
            }
            tracing = cont;
            had_shadow = has_shadow;
            // ---- hand the shadow ray to the odd lane ----
            const float ox = __shfl(sr.o.x, partner), oy = __shfl(sr.o.y, partner), oz = __shfl(sr.o.z, partner);
            const float dx = __shfl(sr.d.x, partner), dy = __shfl(sr.d.y, partner), dz = __shfl(sr.d.z, partner);
            const float tm = __shfl(sr.tmax, partner);
            const bool ph = __shfl(has_shadow, partner) != 0;
            if (!path_lane) {
                sh_trace = ph;
                so = mk(ox, oy, oz);
                sd = mk(dx, dy, dz);
                stmax = tm;
            }
            start = true;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        bounces += __shfl_down(bounces, off);
        shadows += __shfl_down(shadows, off);
    }
    if (lane_id() == 0 && (bounces | shadows)) {
        atomicAdd(&tail_counts[0], bounces);
        atomicAdd(&tail_counts[1], shadows);
    }
    if (STATS) {
        flush_stats<STATS>(st, stats, 0, true);
        flush_stats<STATS>(sst, stats, 4, false);
    }
}

// ---------------------------------------------------------------------------
// shadow: any-hit traversal; on miss add the NEE contribution
// (gpu_traverse_secondary, mapping_gpu.art:70-112; on_shadow_miss, pathtracer.art:202-209)
// ---------------------------------------------------------------------------
// One shadow ray's any-hit walk; unoccluded, its colour goes to the radiance
// slot (l: the slot's value, loaded before the walk so that the scattered
// read's latency overlaps the walk: diamond shadow time 20.6 -> 20.3 ms per
// frame, round 5).  Returns whether the ray is occluded.
template <bool STATS, int V>
__device__ __forceinline__ bool shadow_walk(const SceneView& sv, const TStack& ts, float4 s0, float4 s1, float4 col, float4 l,
                                            float4* L, float4* aov_nee, TraceStats& st) {
    float tmax = s1.w;
    int e, p;
    float u, v;
    const bool occl = trace_ray<true, STATS, V>(sv, f3of(s0), f3of(s1), 0.001f, tmax, RAY_SHADOW, ts, e, p, u, v, st);
    if (!occl) {
        const int slot = __float_as_int(s0.w);
        L[slot] = make_float4(l.x + col.x, l.y + col.y, l.z + col.z, 0); // add_radiance
        add_aov(aov_nee, slot, f3of(col));
    }
    return occl;
}

template <int V0, bool STATS, bool LDS>
__global__ void __launch_bounds__(BLOCK) k_shadow(SceneView gsv, ShadowBuf sh, float4* L, const int* cnt,
                                                  unsigned long long* stats, int* work) {
    constexpr int V = LDS ? kernel_variant(V0, true) : (SHADOW_TREELET ? kernel_variant(V0, false) : V0); // LDS-staged nodes: padded stride; global tables: treelet or global node loads
    __shared__ int stack_mem[LDS_STACK * BLOCK];
    extern __shared__ float4 lds_scene[];
    const TStack ts = make_tstack(stack_mem, LDS_STACK, gsv.spill);
    if (row_total(cnt) == 0) return;
    const SceneView sv = LDS ? stage_scene_lds<BLOCK>(gsv, lds_scene) : stage_treelet<BLOCK>(gsv, lds_scene);
    TraceStats st{0, 0, 0, 0, 0, 0, 0};
    unsigned long long cls_acc[2][6] = {}; // instrumented: per shadow class groups, wave iterations, visits, cycles, occluded, rays
    const WaveWork w = wave_work();
    const int lane = lane_id();
    // groups of 64 shadow rays: grid-stride over the wave's own shard, or
    // (work != nullptr) handed out by take_group
    int s = w.s;
    ShardCount sc = shard_count(cnt, s); // two shadow classes (wave_append_paths)
    // instrumented: the class of the group (wave-uniform), its wave cycles and visits
    unsigned long long c0 = 0;
    uint32_t wn0 = 0, ln0 = 0;
    auto stats_begin = [&]() {
        if constexpr (STATS) {
            c0 = __builtin_amdgcn_s_memtime();
            wn0 = st.wnodes;
            ln0 = st.nodes;
        }
    };
    auto stats_end = [&](int p0, bool act, bool occl) {
        if constexpr (STATS) {
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long c1 = __builtin_amdgcn_s_memtime();
            uint32_t visits = st.nodes - ln0, witers = st.wnodes - wn0, occ = occl ? 1 : 0, nr = act ? 1 : 0;
            for (int off = 32; off > 0; off >>= 1) {
                visits += __shfl_xor(visits, off);
                witers += __shfl_xor(witers, off);
                occ += __shfl_xor(occ, off);
                nr += __shfl_xor(nr, off);
            }
            // accumulated per wave (lane 0), flushed once at the end: no atomics in the timed region
            const int cls = p0 < sc.a ? 0 : 1;
            if (lane == 0) {
                cls_acc[cls][0] += 1;
                cls_acc[cls][1] += witers;
                cls_acc[cls][2] += visits;
                cls_acc[cls][3] += c1 - c0;
                cls_acc[cls][4] += occ;
                cls_acc[cls][5] += nr;
            }
        }
    };
    {
        uint64_t done = 0;
        for (int p0 = w.k * 64;; p0 += w.K * 64) {
            if (work) {
                p0 = take_group(work, s, done, sc.n, [&](int sh_) {
                    sc = shard_count(cnt, sh_);
                    return sc.n;
                });
                if (p0 < 0) break;
                p0 *= 64;
            } else if (p0 >= sc.n) {
                break;
            }
            const int pos = p0 + lane;
            stats_begin();
            bool occl = false;
            if (pos < sc.n) {
                const int i = stream_index(s, pos, sc.a, sh.shard_cap);
                occl = shadow_walk<STATS, V>(sv, ts, sh.s0[i], sh.s1[i], sh.s2[i], L[__float_as_int(sh.s0[i].w)], L, sh.aov_nee, st);
            }
            stats_end(p0, pos < sc.n, occl);
        }
    }
    if constexpr (STATS) {
        if (lane == 0)
            for (int c = 0; c < 2; ++c)
                for (int k = 0; k < 6; ++k)
                    if (cls_acc[c][k]) atomicAdd(&stats[k < 5 ? 40 + 2 * k + c : 70 + c], cls_acc[c][k]);
    }
    if (STATS) flush_stats<STATS>(st, stats, 4, false);
}

// ---------------------------------------------------------------------------
// Persistent-lane variants of trace and shadow (refill_loop) for scenes whose
// traversal tables stay in global memory: there a node step waits on an
// Infinity-Cache / HBM round trip, and refilling idle lanes cuts the number
// of wave-level steps.  Each wave walks the positions k, k + K, ... (in
// groups of 64) of its shard, like the grid-stride kernels.
// ---------------------------------------------------------------------------
// occupancy target of the persistent-lane kernels (waves per SIMD): 6 caps
// them at 80 VGPRs (trace 4.8 -> 4.5 ms per S-deep iteration, soup-16M
// 45.6 -> 43.3); 7 and 8 spill and run slower
#ifndef REFILL_WAVES
#define REFILL_WAVES 6
#endif
// with quantised nodes a node step holds 16 VGPRs of node data instead of 32
#ifndef REFILL_WAVES_Q4
#define REFILL_WAVES_Q4 6
#endif
// the if-if shadow kernel (split-schedule scenes) needs fewer registers: with
// quantised nodes and global stack / node loads it fits 7 waves per SIMD (72
// VGPRs, 2 spilled): soup-1M shadow time per 8-iteration frame 102.0 -> 98.2 ms,
// soup-16M 42.6 -> 42.0 ms (profiles/r03_ab_waves7.log; the trace kernel at 7
// waves spills 23 registers and runs slower, so it stays at 6)
#ifndef SHADOW_IFIF_WAVES
#define SHADOW_IFIF_WAVES 7
#endif
// LDS-staged tables (<= 48 KB + the 16 KB stack per block) allow at most
// 4 blocks per CU: the 6-wave VGPR cap would only force spills
#ifndef REFILL_WAVES_LDS
#define REFILL_WAVES_LDS 4
#endif
// The sequence of stream positions a persistent-lane wave walks
// (refill_loop): virtual position c lies in virtual group c >> 6.  Static
// (work == nullptr): virtual group j is group k + j * K of the wave's own
// shard.  Dynamic: virtual groups come from take_group as the wave reaches
// them.  A window of two slots holds the groups one refill can touch (a
// refill takes at most 64 positions).  All members are wave-uniform.
// CLASSES: the stream holds two path classes (stream_index); otherwise
// position pos of shard s is stored at s * shard_cap + pos.
template <bool CLASSES>
struct GroupSeq {
    const int* cnt;
    int* work;
    int shard_cap;
    WaveWork w;
    int s;
    uint64_t done;
    bool exhausted;
    int j0;                          // virtual group of slot 0
    int gs[2], gg[2], ga[2], gn[2]; // shard, group (< 0: empty slot), class-A count, count

    __device__ __forceinline__ ShardCount count_of(int sh) const {
        if constexpr (CLASSES) return shard_count(cnt, sh);
        const int n = uniform_load(cnt + sh * CSTRIDE);
        return ShardCount{n, n, n};
    }
    __device__ __forceinline__ void init(const int* cnt_, int* work_, int cap, const WaveWork& w_) {
        cnt = cnt_;
        work = work_;
        shard_cap = cap;
        w = w_;
        s = w.s;
        done = 0;
        exhausted = false;
        j0 = 0;
        gg[0] = gg[1] = -1;
    }
    // load the next virtual group (j0 + k) into slot k
    __device__ __forceinline__ bool fill(int k) {
        if (exhausted) return false;
        ShardCount sc = count_of(s);
        int g;
        if (work) {
            g = take_group(work, s, done, sc.n, [&](int sh_) {
                sc = count_of(sh_);
                return sc.n;
            });
        } else {
            g = w.k + (j0 + k) * w.K;
            if (g * 64 >= sc.n) g = -1;
        }
        if (g < 0) {
            exhausted = true;
            return false;
        }
        gs[k] = s;
        gg[k] = g;
        ga[k] = sc.a;
        gn[k] = sc.n;
        return true;
    }
    // make positions [cursor, cursor + m) resolvable as far as groups remain;
    // false once the sequence has nothing at cursor
    __device__ __forceinline__ bool reserve(int cursor, int m) {
        if (cursor >= (j0 + 1) * 64) { // slide the window
            gs[0] = gs[1];
            gg[0] = gg[1];
            ga[0] = ga[1];
            gn[0] = gn[1];
            gg[1] = -1;
            ++j0;
        }
        if (gg[0] < 0 && !fill(0)) return false;
        if (cursor + m > (j0 + 1) * 64 && gg[1] < 0) fill(1);
        return true;
    }
    // stream index of virtual position c (per lane); false: nothing there
    __device__ __forceinline__ bool at(int c, int& i) const {
        const int k = (c >> 6) - j0;
        const int g = k ? gg[1] : gg[0];
        if (g < 0) return false;
        const int pos = g * 64 + (c & 63);
        if (pos >= (k ? gn[1] : gn[0])) return false;
        const int sh = k ? gs[1] : gs[0];
        i = CLASSES ? stream_index(sh, pos, k ? ga[1] : ga[0], shard_cap) : sh * shard_cap + pos;
        return true;
    }
};

template <int V0, bool STATS, bool LDS>
__global__ void __launch_bounds__(BLOCK, LDS ? REFILL_WAVES_LDS : (variant_q4(V0) ? REFILL_WAVES_Q4 : REFILL_WAVES)) k_trace_refill(FrameArgs fa, SceneView gsv, PathBuf in, HitBuf hits,
                                                                     const int* cnt, int tail_threshold,
                                                                     unsigned long long* stats, int refill_min, int* work) {
    // LDS-staged nodes: padded stride; global tables: global node loads (no treelet)
    constexpr int V = LDS ? kernel_variant(V0, true) : V0;
    __shared__ int stack_mem[LDS_STACK * BLOCK];
    extern __shared__ float4 lds_scene[];
    const TStack ts = make_tstack(stack_mem, LDS_STACK, gsv.spill);
    if (row_total(cnt) <= tail_threshold) return; // k_finish takes the remaining paths
    const SceneView sv = LDS ? stage_scene_lds<BLOCK>(gsv, lds_scene) : stage_treelet<BLOCK>(gsv, lds_scene);
    TraceStats st{0, 0, 0, 0, 0, 0, 0};
    GroupSeq<true> seq;
    seq.init(cnt, work, in.shard_cap, wave_work());
    refill_loop<false, STATS, V>(
        sv, ts, seq, refill_min,
        [&](int i, Trav& t) -> bool {
            const float4 p0 = in.p0[i], p1 = in.p1[i];
            const int depth = (int)(__float_as_uint(p1.w) >> 24);
            if (depth == 0) {
                hits.h[i] = make_float4(0, 0, 0, __int_as_float(-1));
                hits.prim[i] = -1;
                return false;
            }
            float tmin, tmax;
            uint32_t rflags;
            ray_extent(fa, sv, depth, (int)(__float_as_uint(p0.w) & SLOT_MASK), tmin, tmax, rflags);
            trav_init(sv, t, f3of(p0), f3of(p1), tmin, tmax, rflags, ts);
            return true;
        },
        [&](int i, const Trav& t) {
            if (STATS && t.hit_ent >= 0) st.hits++;
            hits.h[i] = make_float4(t.tmax, t.hu, t.hv, __int_as_float(t.hit_ent));
            hits.prim[i] = t.hit_prim;
        },
        st);
    if (STATS) flush_stats<STATS>(st, stats, 0, true);
}

template <int V0, bool STATS, bool LDS>
__global__ void __launch_bounds__(BLOCK, LDS ? REFILL_WAVES_LDS : (variant_ifif(V0) ? SHADOW_IFIF_WAVES : REFILL_WAVES)) k_shadow_refill(SceneView gsv, ShadowBuf sh, float4* L, const int* cnt,
                                                                      unsigned long long* stats, int refill_min, int* work) {
    // LDS-staged nodes: padded stride; global tables: treelet, except with if-if
    // stepping (the split schedule's scenes), where global node loads beat the
    // treelet's flat loads: soup-1M 32-iteration frame 1179.6 / 1188.1 ->
    // 1154.5 / 1153.5 ms (profiles/r03_ab_treelet_global.log)
    constexpr int V = LDS ? kernel_variant(V0, true) : ((SHADOW_TREELET && !variant_ifif(V0)) ? kernel_variant(V0, false) : V0);
    __shared__ int stack_mem[LDS_STACK * BLOCK];
    extern __shared__ float4 lds_scene[];
    const TStack ts = make_tstack(stack_mem, LDS_STACK, gsv.spill);
    if (row_total(cnt) == 0) return;
    const SceneView sv = LDS ? stage_scene_lds<BLOCK>(gsv, lds_scene) : stage_treelet<BLOCK>(gsv, lds_scene);
    TraceStats st{0, 0, 0, 0, 0, 0, 0};
    GroupSeq<true> seq; // two shadow classes (wave_append_paths)
    seq.init(cnt, work, sh.shard_cap, wave_work());
    refill_loop<true, STATS, V>(
        sv, ts, seq, refill_min,
        [&](int i, Trav& t) -> bool {
            const float4 s0 = sh.s0[i], s1 = sh.s1[i];
            trav_init(sv, t, f3of(s0), f3of(s1), 0.001f, s1.w, RAY_SHADOW, ts);
            return true;
        },
        [&](int i, const Trav& t) {
            if (t.found) return;
            const int slot = __float_as_int(sh.s0[i].w);
            const f3 col = f3of(sh.s2[i]);
            add_radiance(L, slot, col);
            add_aov(sh.aov_nee, slot, col);
        },
        st);
    if (STATS) flush_stats<STATS>(st, stats, 4, false);
}

#if IGX_PART == 0
// resolve: fb += sum_s L_s / spi (driver/accumulator.art:13-19, make_standard_accumulator)
// A block owns 64 pixels; its RES_G waves sum one iteration each (lanes =
// pixels, the sample loop in order) into LDS, and wave 0 adds the iterations
// into the framebuffer in iteration order, so the float sums are those of one
// accumulation per render call.  One pixel per lane with all iterations in one
// lane was latency-bound (2.1 ms per 128M-path chunk); this form takes 1.4 ms.
// Coalesced loads through a 55 KB LDS transpose tile measured slower (3.2 ms):
// the kernel overlaps the next chunk's k_extend, whose LDS-resident BVH leaves
// no room for blocks with a large LDS footprint.
constexpr int RES_G = 8;
__global__ void __launch_bounds__(64 * RES_G) k_resolve(FrameArgs fa, const float4* L, float* fb, int fb_width) {
    __shared__ float part[RES_G][3][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int p = blockIdx.x * 64 + lane;
    int x = 0, y = 0;
    const bool in = p < fa.chunk_pixels && local_to_global(fa, fa.chunk_pixel0 + p, x, y);
    const size_t o = 3 * ((size_t)y * fb_width + x);
    float fr = 0, fg = 0, fbb = 0;
    if (w == 0 && in) {
        fr = fb[o + 0];
        fg = fb[o + 1];
        fbb = fb[o + 2];
    }
    for (int it0 = 0; it0 < fa.chunk_iters; it0 += RES_G) { // block-uniform trip count
        const int it = it0 + w;
        if (in && it < fa.chunk_iters) {
            const float4* Li = L + ((size_t)it * fa.chunk_pixels + p) * fa.spi;
            float r = 0, g = 0, b = 0;
            if (fa.probe_sample) { // per-path probes (tests): sample probe_sample - 1 only
                const float4 l = Li[fa.probe_sample - 1];
                r = l.x * fa.inv_spi;
                g = l.y * fa.inv_spi;
                b = l.z * fa.inv_spi;
            } else {
#pragma unroll 8
                for (int s = 0; s < fa.spi; ++s) {
                    float4 l = Li[s];
                    r += l.x * fa.inv_spi;
                    g += l.y * fa.inv_spi;
                    b += l.z * fa.inv_spi;
                }
            }
            part[w][0][lane] = r;
            part[w][1][lane] = g;
            part[w][2][lane] = b;
        }
        __syncthreads();
        if (w == 0 && in) {
            const int m = min(RES_G, fa.chunk_iters - it0);
            for (int k = 0; k < m; ++k) { // one accumulation per iteration, in order
                fr += part[k][0][lane];
                fg += part[k][1][lane];
                fbb += part[k][2][lane];
            }
        }
        __syncthreads();
    }
    if (w == 0 && in) {
        fb[o + 0] = fr;
        fb[o + 1] = fg;
        fb[o + 2] = fbb;
    }
}

__global__ void k_pack_tiles(FrameArgs fa, const float* fb, float* dst, int num_tiles) {
    int T = fa.tile_size;
    long long total = (long long)num_tiles * T * T;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        int x, y;
        bool in = local_to_global<false>(fa, (int)i, x, y); // each packed tile row-major
        for (int c = 0; c < 3; ++c) dst[3 * i + c] = in ? fb[3 * ((size_t)y * fa.width + x) + c] : 0.0f;
    }
}

#endif

// hit-level test kernels (one ray per lane)
template <int V>
__global__ void __launch_bounds__(BLOCK) k_trace_hits(SceneView sv, const float* rays, int n, uint32_t flags, int* ent_prim,
                                                      float* tuv, int any) {
    __shared__ int stack_mem[LDS_STACK * BLOCK];
    const TStack ts = make_tstack(stack_mem, LDS_STACK, sv.spill);
    TraceStats st{0, 0, 0, 0, 0, 0, 0};
    for (int i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        const float* r = rays + 8 * i;
        float tmax = r[7];
        int e, p;
        float u = 0, v = 0;
        if (any) {
            bool occ = trace_ray<true, false, V>(sv, mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), r[6], tmax, flags, ts, e, p, u, v, st);
            ent_prim[i] = occ ? 1 : 0;
        } else {
            trace_ray<false, false, V>(sv, mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), r[6], tmax, flags, ts, e, p, u, v, st);
            ent_prim[2 * i] = e;
            ent_prim[2 * i + 1] = p;
            tuv[3 * i] = e >= 0 ? tmax : r[7];
            tuv[3 * i + 1] = u;
            tuv[3 * i + 2] = v;
        }
    }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
// Two stream "slots" (path double-buffer, shadow stream, radiance, counters)
// alternate between chunks (a chunk = one iteration, or a capacity-sized part
// of it).  The wavefront bounces of chunk k run on the main stream; when the
// live-path count falls to the tail threshold, k_finish and the resolve of
// chunk k are queued on the tail stream and the host moves on to chunk k+1 in
// the other slot, so the latency-bound tail of one chunk overlaps the next
// chunk's full bounces.
struct TimedLaunch {
    hipEvent_t a, b;
    int kind; // 0 extend/shade, 1 shadow, 2 generate, 3 resolve, 4 finish, 5 trace
    int bounce;
};

struct Slot {
    size_t cap = 0;            // paths per chunk
    int shard_cap = 0;         // records per stream shard (NSH * shard_cap >= cap)
    PathBuf pa{}, pb{};
    ShadowBuf sh{};
    HitBuf hb{};
    float4* L = nullptr;
    float4* aov_di = nullptr;  // MIS AOV slots beside L (technique aov_mis): "Direct Weights",
    float4* aov_nee = nullptr; // "NEE Weights" (FrameArgs::aov_di / aov_nee)
    int* ctr = nullptr;        // device shard counters: row 2b = paths entering bounce b, row 2b+1 = shadow rays of bounce b (CROW ints per row)
    int* pinned = nullptr;     // host mirror
    long long n0 = 0;          // paths generated for the chunk (row 0)
    hipEvent_t done = nullptr; // recorded on the tail stream after the resolve
    std::vector<hipEvent_t> bounce_ev;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_next = 0;
    std::vector<TimedLaunch> timed;
    // pending statistics of the chunk last run in this slot
    bool pending = false;
    int switch_bounce = 0;     // first bounce handled by k_finish
    int launched = 0;          // extend/shadow launch pairs queued (the last may find its count <= tail and exit at once)
    bool split = true;         // chunk ran k_trace + k_shade
    int tail = 0;
    long long camera = 0;
};

enum { DYN_EXTEND = 1, DYN_SHADOW = 2, DYN_REFILL_TRACE = 4, DYN_REFILL_SHADOW = 8 };
// rows WORK_ROW0 + 4b: k_extend (or k_trace_refill) group counters of bounce b (take_group),
// + 1: its mask of exhausted shards, + 2 / + 3: the same for k_shadow
constexpr int WORK_ROW0 = 2 * MAX_BOUNCES + 4;
// instrumentation counters (igx_get_stats): 0-12 visit counts, 16-19 k_extend
// phase clocks, 20-39 k_extend by group class, 40-49 k_shadow by class, 50-53
// closest-hit node visits in the TLAS and by hot-order rank, 54-69 k_extend
// shading sub-phase clocks by class, 70-71 k_shadow rays by class
[[maybe_unused]] constexpr int DSTATS = 80;
constexpr int CTR_ROWS = WORK_ROW0 + 4 * MAX_BOUNCES;
// BLAS with more triangles build without spatial splits (load time; their
// triangles are small next to the scene in the suite's soups)
[[maybe_unused]] constexpr uint32_t SPATIAL_SPLIT_MAX_FACES = 1u << 21;
// face instances (faces x entities using them) up to which the upload
// precomputes world-space face normals (16 B each: at most 64 MB)
[[maybe_unused]] constexpr size_t FACE_NORMAL_TABLE_MAX = 4u << 20;
// mesh faces (over all shapes) up to which the upload writes the per-face
// shading records SceneView::fsh (48 B each: at most 192 MB)
[[maybe_unused]] constexpr size_t FACE_SHADE_MAX = 4u << 20;
[[maybe_unused]] constexpr size_t CTR_INTS = (size_t)CTR_ROWS * CROW;
// nodes moved to the front of the node array in hot order at upload (the
// largest treelet a kernel may stage: 160 KB of LDS / 128-B nodes)
[[maybe_unused]] constexpr size_t TREELET_FRONT = 1280;

// records in counter row `row` of the slot's host mirror (row 0: generated paths)
inline long long row_total(const Slot& s, int row) {
    if (row == 0) return s.n0;
    long long t = 0;
    const int* r = s.pinned + (size_t)row * CROW;
    for (int k = 0; k < NSH; ++k) t += r[k * CSTRIDE] + r[k * CSTRIDE + 1] + r[k * CSTRIDE + 2]; // classes A, B, C (wave_append_paths)
    return t;
}

} // namespace igxh

using namespace igxh;

struct igx_device {
    int hip_device = 0;
    hipStream_t stream = nullptr;  // main (wavefront) stream
    hipStream_t stream2 = nullptr; // slot 1's wavefront stream under concurrent chunks
    hipStream_t tail_stream = nullptr;
    std::string last_error;
    int num_cus = 256;
    size_t mem_total = 0;     // device memory (bytes)
    // options
    bool timing = false;
    bool instrument = false;
    int64_t capacity_opt = 0;
    // option "slot_budget_mb": device memory the two stream slots of this
    // handle may take (0 = auto: a quarter of the device memory)
    int64_t slot_budget_mb = 0;
    // option "stream_slots": chunks alternate between two slots (chunk k + 1's
    // bounces overlap chunk k's tail), or use one (half the memory; chunk k + 1
    // waits for chunk k).  A rank of a multi-GPU render holds two handles that
    // alternate frames, and a rank's share of a frame is one chunk, so there
    // one slot per handle loses nothing: bench.py sets 1 at N > 1
    int stream_slots = 2;
    // option "concurrent_chunks" (0/1): the fused schedule's chunks run
    // through ChunkScheduler, the two slots' chunks concurrently, each on its
    // own stream (one slot: a chunk still waits for the slot's previous one)
    int concurrent_opt = 1;
    int concurrent_start_pct = 10; // option "concurrent_start_pct": a chunk starts once the running one is down to this share of its paths
    // LDS treelet (stage_treelet) on global-table scenes: nodes staged per
    // kernel (the largest prefix of the hot order that keeps the kernel's
    // register-bound occupancy), recomputed when the scene or option changes.
    // Option "treelet": -1 auto, 0 off, n > 0 at most n nodes
    int tail_pairs_opt = -1;  // k_finish_pairs on global-table scenes (-1 auto = on, 0 off, 1 on)
    // The treelet kernels are k_extend and k_shadow / k_shadow_refill (not the
    // if-if variant): primitives 8.89 -> 8.37, S-deep 48.2 -> 45.8, soup-1M
    // 187.9 -> 184.9 ms per frame
    int64_t treelet_opt = -1;
    bool tree_dirty = true;
    int tree_ext = 0, tree_shadow = 0;
    int64_t tail_opt = -1;   // paths at or below which k_finish takes over (-1 = auto)
    int64_t tail_last_opt = -1; // the same for the last chunk of a render call, whose tail overlaps nothing (-1 = tail_opt)
    bool fuse_generate = true; // bounce 0 of the fused k_extend builds its camera paths (no k_generate pass)
    int split_opt = -1;      // k_trace + k_shade per bounce instead of the fused k_extend (-1: auto = global-table scenes)
    int refill_opt = -1;     // persistent-lane trace / shadow, refilled once this many lanes idle (0: off, -1: auto = 16)
    int shadow_ifif_opt = -1; // if-if stepping in k_shadow_refill (-1: auto = split-schedule scenes)
    int64_t lds_scene_max = 48 * 1024; // stage traversal tables in LDS when they fit (0 = never)
    size_t lds_scene_bytes = 0;        // bytes staged per block for the current scene (0 = global tables)
    size_t table_bytes = 0;            // traversal tables (nodes, instances, triangles) of the current scene
    size_t shading_bytes = 0;          // shading tables (entities, vertices, normals, faces, materials, lights)
    int leaf_size = 4;
    // stream class of surviving paths (FrameArgs::classify; option "path_classes"):
    // paths inside a dielectric go to the back of their shard, so the next
    // bounce's waves are all-inside or all-outside (diamond frame 152-155 ->
    // 143-145 ms, S-deep 49.1 -> 47.5 ms per 8-iteration frame; bit-identical)
    // 3: also paths whose next ray crosses an enclosing entity's world box
    // (diamond frame 132.5 -> 119.3 ms, k_extend 1770 -> 1591 us per launch,
    // bit-identical)
    // 4: three classes, the paths inside a dielectric in their own region of
    // the path buffers (class C), apart from those heading for the box (B):
    // diamond frame 109.6 -> 106.4 ms, bit-identical; the split schedule
    // falls back to 3 (its hit records have no class-C region)
    int classify_opt = 4;
    // option "shadow_classes": shadow rays whose segment crosses an enclosing
    // entity's box apart from the rest (shadow_class_b), 0/1: diamond shadow
    // time 26.9 -> 21.7 ms per frame, frame 121.1 -> 118.4 ms, bit-identical
    int shadow_classes_opt = 1;
    // option "dynamic" (DYN_* bits): DYN_EXTEND = k_extend waves take their
    // groups of 64 paths from per-shard counters (take_group) instead of a
    // fixed grid stride: diamond frame 142.4 -> 134.3 ms, materials 66.5 ->
    // 54.6, primitives 36.8 -> 33.9, bit-identical images; DYN_SHADOW = the
    // same for k_shadow (measured neutral: shadow rays cost about the same);
    // DYN_REFILL_TRACE / DYN_REFILL_SHADOW: the persistent-lane kernels
    // draw their groups the same way (GroupSeq): soup-1M 8-iteration frame
    // 452 -> 382 ms (k_shadow_refill 220 -> 164, k_trace_refill 205 -> 193),
    // S-deep 52.7 -> 48.6 ms
    int dynamic_opt = DYN_EXTEND | DYN_REFILL_TRACE | DYN_REFILL_SHADOW;
    // option "group_order": 1 = k_extend takes a shard's groups from its end
    // (classes C, B, A: longest paths first), 0 = from its front, -1 = auto
    int group_order_opt = -1;
    // option "face_normals": precomputed world-space face normals for scenes
    // with at most FACE_NORMAL_TABLE_MAX face instances (next upload)
    int face_normals_opt = 1;
    // option "face_shade": per-face shading records (SceneView::fsh) for
    // scenes with at most FACE_SHADE_MAX faces (next upload)
    int face_shade_opt = 1;
    float sah_node_cost = 1.0f;    // option "sah_node_cost_pct" (percent of one triangle test)
    int bvh_bins = 32;             // option "bvh_bins": SAH bins per axis of the BLAS builds (next upload)
    int bvh_bins_tlas = 32;        // option "bvh_bins_tlas": the same for the TLAS
    // SBVH for BLAS up to SPATIAL_SPLIT_MAX_FACES triangles (option "spatial_splits"):
    // off by default -- measured slower on the diamond (196 -> 230 ms per frame)
    // and neutral on primitives, S-deep and soup-1M
    bool spatial_splits = false;
    // 1: build every BLAS here even when the scene carries the reference's own
    // (igx_shape::ref_bvh, from the SceneDatabase adapter)
    bool rebuild_bvh = false;
    // scene
    bool has_scene = false;
    std::vector<void*> scene_allocs;
    SceneView sv{};
    igx_camera cam_desc{};
    int variant = 0;       // traversal variant of the scene (device_scene.h: width, spill)
    int bvh_width = 2;     // node width of the uploaded tables
    bool quantized = false; // the 4-wide nodes are quantised (Bvh4QNode, 64 B; variant bit 7)
    int quantize_opt = -1;  // option "bvh_quantize": -1 auto (4-wide scenes whose tables stay in global memory), 0, 1
    int nf4 = 4;            // float4s per node of the uploaded tables
    int bvh_width_opt = 0; // option "bvh_width": 0 = auto, 2, 4 (applies at the next upload)
    bool full_shading = false;     // the scene needs materials / lights beyond the basic set
    bool full_shading_opt = false; // option "full_shading": 1 = always compile-in the whole set
    // option "enclosing": paths inside a closed, isolated dielectric trace
    // only its BLAS (trace_enclosed); applies at the next upload
    bool enclosing_opt = true;
    int scene_depth = 0;   // worst-case stack entries of the scene
    int* spill_main = nullptr; // spill columns of the main, tail and shadow streams (and of slot 1's stream)
    int* spill_tail = nullptr;
    int* spill_shadow = nullptr;
    int* spill_main2 = nullptr;
    hipStream_t shadow_stream = nullptr; // split schedule: shadow rays of bounce b overlap the trace of bounce b + 1
    int overlap_shadow_opt = 1;           // option "overlap_shadow" (0/1)
    // streams
    Slot slots[2];
    int next_slot = 0;
    unsigned long long* dstats = nullptr;      // instrumentation counters
    unsigned long long* tail_counts = nullptr; // [2]: tail continuation rays, tail shadow rays
    float* ray_list = nullptr;
    size_t ray_list_cap = 0;
    // framebuffer
    float* fb = nullptr;
    size_t fb_count = 0;
    // MIS AOV films ("Direct Weights", "NEE Weights"; technique aov_mis), fb_count floats each
    bool aov_on = false;
    float* aov_fb[2] = {nullptr, nullptr};
    int fb_w = 0, fb_h = 0;
    uint64_t iteration_count = 0;
    // stats
    igx_stats stats{};
    // asynchronous rendering (option "async_render"): the worker thread and
    // its queue (render_impl, igx_clear); nullptr until the first queued render
    int async_opt = 1;
    struct AsyncRender* async = nullptr;
    // option "host_wait_us": the chunk scheduler's host thread sleeps this long
    // between polls that found no progress (after a few yields); 0 = yield only
    int host_wait_us = 20;
    // option "fail_chunk" (test hook): the n-th chunk the chunk scheduler
    // starts from now on fails with IGX_ERR_HIP instead
    int64_t fail_chunk_opt = 0;
    // option "probe_sample" (test hook): s + 1 = the film receives sample s of
    // each pixel only (the other paths are traced as usual), 0 = every sample
    int64_t probe_sample_opt = 0;
};
// the worker has queued everything submitted; its first error (part 0)
igx_status wait_idle(igx_device* dev);
igx_status wait_ready(igx_device* dev);
bool reset_async_failure(igx_device* dev);
void stop_async(igx_device* dev);

namespace igxh {

#if IGX_PART == 0
// Set on a handle's async worker thread (async_worker): errors raised there
// go to the worker's own message, which the host thread copies into
// last_error (wait_idle / wait_ready); the host thread alone writes last_error.
thread_local std::string* t_error_sink = nullptr;
igx_status fail(igx_device* d, igx_status s, const std::string& msg) {
    if (t_error_sink) *t_error_sink = msg;
    else if (d) d->last_error = msg;
    return s;
}

#define HIPCHK(expr)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return fail(dev, e_ == hipErrorOutOfMemory ? IGX_ERR_OUT_OF_MEMORY : IGX_ERR_HIP,         \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                           \
    } while (0)

template <typename T>
igx_status upload(igx_device* dev, const std::vector<T>& v, const T** out) {
    size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, bytes));
    dev->scene_allocs.push_back(p);
    if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    *out = reinterpret_cast<const T*>(p);
    return IGX_OK;
}

void free_scene(igx_device* dev) {
    for (void* p : dev->scene_allocs) (void)hipFree(p);
    dev->scene_allocs.clear();
    dev->spill_main = dev->spill_tail = dev->spill_shadow = dev->spill_main2 = nullptr;
    dev->has_scene = false;
}

// Largest grid any stream kernel is launched with (grid_for).
int max_grid(const igx_device* dev) {
    return std::max(GRID_QUANTUM, dev->num_cus * MAX_BLOCKS_PER_CU / GRID_QUANTUM * GRID_QUANTUM);
}

// Traversal variant of the scene and the spill columns for the stack entries
// beyond the LDS_STACK in LDS: one per grid thread of the largest grid, per
// stream.
igx_status configure_stack(igx_device* dev) {
    const int need = dev->scene_depth;
    const int extra = std::max(0, need - LDS_STACK);
    dev->variant = (dev->bvh_width >= 4 ? 2 : 0) | (extra > 0 ? 1 : 0) | (dev->full_shading ? 4 : 0) | (dev->quantized ? VARIANT_Q4 : 0);
    const size_t threads = (size_t)max_grid(dev) * BLOCK;
    for (int k = 0; k < 4; ++k) {
        int*& old = k == 0 ? dev->spill_main : k == 1 ? dev->spill_tail : k == 2 ? dev->spill_shadow : dev->spill_main2;
        if (old) {
            auto it = std::find(dev->scene_allocs.begin(), dev->scene_allocs.end(), (void*)old);
            if (it != dev->scene_allocs.end()) dev->scene_allocs.erase(it);
            (void)hipFree(old);
            old = nullptr;
        }
        void* p = nullptr;
        HIPCHK(hipMalloc(&p, std::max<size_t>(16, (size_t)extra * threads * sizeof(int))));
        dev->scene_allocs.push_back(p);
        (k == 0 ? dev->spill_main : k == 1 ? dev->spill_tail : k == 2 ? dev->spill_shadow : dev->spill_main2) = static_cast<int*>(p);
    }
    dev->sv.spill = dev->spill_main;
    return IGX_OK;
}

void free_slot_buffers(Slot& s) {
    void* ptrs[] = {s.pa.p0, s.pa.p1, s.pa.p2, s.pa.p3, s.pb.p0, s.pb.p1, s.pb.p2, s.pb.p3, s.sh.s0, s.sh.s1, s.sh.s2, s.L, s.hb.h, s.hb.prim,
                    s.aov_di, s.aov_nee};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    s.pa = PathBuf{};
    s.pb = PathBuf{};
    s.sh = ShadowBuf{};
    s.hb = HitBuf{};
    s.L = nullptr;
    s.aov_di = s.aov_nee = nullptr;
    s.cap = 0;
    s.shard_cap = 0;
}

// `hits`: the chunk runs the split schedule, whose k_trace writes a hit
// record per path (20 B) for k_shade; the fused schedule needs none.
// `region_c`: three path classes (FrameArgs::classify 4), so each path buffer
// holds a second set of records for class C (PathBuf::c_base); `aov`: the
// MIS AOV slots (technique aov_mis)
igx_status ensure_slot(igx_device* dev, Slot& s, size_t cap, bool hits, bool region_c, bool aov) {
    if (!s.ctr) {
        HIPCHK(hipMalloc((void**)&s.ctr, CTR_INTS * sizeof(int)));
        HIPCHK(hipHostMalloc((void**)&s.pinned, CTR_INTS * sizeof(int), hipHostMallocDefault));
        HIPCHK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        std::memset(s.pinned, 0, CTR_INTS * sizeof(int));
    }
    if (s.cap >= cap && (!hits || s.hb.h) && (!region_c || s.pa.c_base) && (!aov || s.aov_di)) return IGX_OK;
    free_slot_buffers(s);
    // shard capacity: a generated chunk puts at most ceil(cap / (64 NSH)) groups
    // of 64 paths in one shard, and a shard's outputs never exceed its inputs
    const int shard_cap = (int)((cap + 64 * NSH - 1) / (64 * NSH)) * 64;
    const size_t recs = (size_t)shard_cap * NSH;
    auto alloc4 = [&](float4** p, size_t k) -> igx_status { HIPCHK(hipMalloc((void**)p, k * sizeof(float4))); return IGX_OK; };
    igx_status st;
    const size_t precs = region_c ? 2 * recs : recs;
    if ((st = alloc4(&s.pa.p0, precs)) || (st = alloc4(&s.pa.p1, precs)) || (st = alloc4(&s.pa.p2, precs))) return st;
    HIPCHK(hipMalloc((void**)&s.pa.p3, precs * sizeof(float2)));
    if ((st = alloc4(&s.pb.p0, precs)) || (st = alloc4(&s.pb.p1, precs)) || (st = alloc4(&s.pb.p2, precs))) return st;
    HIPCHK(hipMalloc((void**)&s.pb.p3, precs * sizeof(float2)));
    s.pa.c_base = s.pb.c_base = region_c ? (int)recs : 0;
    if ((st = alloc4(&s.sh.s0, recs)) || (st = alloc4(&s.sh.s1, recs)) || (st = alloc4(&s.sh.s2, recs))) return st;
    if ((st = alloc4(&s.L, cap))) return st; // radiance is indexed by path slot, not sharded
    if (aov && ((st = alloc4(&s.aov_di, cap)) || (st = alloc4(&s.aov_nee, cap)))) return st;
    if (hits) {
        if ((st = alloc4(&s.hb.h, recs))) return st;
        HIPCHK(hipMalloc((void**)&s.hb.prim, recs * sizeof(int)));
    }
    s.pa.shard_cap = s.pb.shard_cap = s.sh.shard_cap = shard_cap;
    s.cap = cap;
    s.shard_cap = shard_cap;
    return IGX_OK;
}

hipEvent_t slot_event(Slot& s) {
    if (s.ev_next >= s.ev_pool.size()) {
        hipEvent_t e;
        (void)hipEventCreate(&e);
        s.ev_pool.push_back(e);
    }
    return s.ev_pool[s.ev_next++];
}

// Grid of a stream kernel: enough blocks for `items`, at most the resident
// blocks, always a multiple of GRID_QUANTUM (every shard gets the same waves).
int grid_for(igx_device* dev, long long items, int blocks_per_cu) {
    const long long q = GRID_QUANTUM;
    long long need = (items + BLOCK - 1) / BLOCK;
    long long cap = (long long)dev->num_cus * std::min(blocks_per_cu, MAX_BLOCKS_PER_CU);
    long long g = std::min((need + q - 1) / q * q, std::max(q, cap / q * q));
    return (int)std::max(q, g);
}

#endif // IGX_PART == 0

// Kernel schedule per scene (measured per scene):
//  * traversal tables in LDS (<= 48 KB): fused k_extend, grid-stride k_shadow;
//  * tables in global memory: shadow rays with persistent lanes (k_shadow_refill,
//    a refill once refill_min lanes idle);
//  * tables beyond 64 MiB: also split the bounce into k_trace (persistent
//    lanes) + k_shade -- there most node steps wait on an Infinity-Cache /
//    HBM round trip, and a traversal-only kernel keeps more waves resident
//    and lets lanes refill.  Below, the fused kernel with dynamic groups is
//    faster (no hit records): S-deep (18 MB of tables) 49.4 -> 46.9 ms per
//    8-iteration frame fused, soup-1M (104 MB) 382 split vs 451 fused.
constexpr size_t SPLIT_TABLE_BYTES = 64u << 20;
// order in which k_extend's dynamic groups take a shard's positions (option "group_order" -1)
#ifndef GROUP_ORDER_AUTO
#define GROUP_ORDER_AUTO 0
#endif
// tail kernel with lane pairs (k_finish_pairs) on global-table scenes; option "tail_pairs" (-1 auto, 0, 1)
inline bool use_tail_pairs(const igx_device* dev) {
    return dev->lds_scene_bytes == 0 && (dev->tail_pairs_opt < 0 ? true : dev->tail_pairs_opt != 0);
}
// dynamic LDS of a global-table kernel that stages `nodes` treelet nodes
inline size_t tree_bytes(const igx_device* dev, int nodes) { return (size_t)nodes * dev->nf4 * 16; }
inline int refill_min(const igx_device* dev) { return dev->refill_opt >= 0 ? dev->refill_opt : 16; }
// auto: global-table scenes only; an explicit "refill" applies to LDS-staged scenes too
inline bool use_refill(const igx_device* dev) {
    return refill_min(dev) > 0 && (dev->lds_scene_bytes == 0 || dev->refill_opt > 0);
}
inline bool use_split(const igx_device* dev) {
    return dev->split_opt >= 0 ? dev->split_opt != 0 : (dev->lds_scene_bytes == 0 && dev->table_bytes > SPLIT_TABLE_BYTES);
}
// if-if stepping for the persistent-lane shadow kernel (variant bit 4): on the
// big-table scenes of the split schedule a lane at a leaf no longer waits for
// the wave's slowest inner-node walk (any-hit rays end at their first
// occluder, so their lengths vary most); on S-deep-sized tables the while-while
// loop is faster.  Option "shadow_ifif": -1 auto, 0 off, 1 on.
inline bool use_shadow_ifif(const igx_device* dev) {
    return dev->shadow_ifif_opt >= 0 ? dev->shadow_ifif_opt != 0 : use_split(dev);
}

// Launch helpers dispatching on the scene's traversal variant.
// (bit 7, VARIANT_Q4: quantised 4-wide nodes, only with bit 1)
#define IGX_DISPATCH_VARIANT(v, MACRO)        \
    do {                                      \
        switch ((v) & (3 | VARIANT_Q4)) {     \
        case 0: MACRO(0); break;              \
        case 1: MACRO(1); break;              \
        case 2: MACRO(2); break;              \
        case 3: MACRO(3); break;              \
        case 2 | VARIANT_Q4: MACRO(130); break; \
        default: MACRO(131); break;           \
        }                                     \
    } while (0)
// shading kernels also dispatch on the material/light feature bit
#define IGX_DISPATCH_VARIANT8(v, MACRO)       \
    do {                                      \
        switch ((v) & (7 | VARIANT_Q4)) {     \
        case 0: MACRO(0); break;              \
        case 1: MACRO(1); break;              \
        case 2: MACRO(2); break;              \
        case 3: MACRO(3); break;              \
        case 4: MACRO(4); break;              \
        case 5: MACRO(5); break;              \
        case 6: MACRO(6); break;              \
        case 7: MACRO(7); break;              \
        case 2 | VARIANT_Q4: MACRO(130); break; \
        case 3 | VARIANT_Q4: MACRO(131); break; \
        case 6 | VARIANT_Q4: MACRO(134); break; \
        default: MACRO(135); break;           \
        }                                     \
    } while (0)

template <bool STATS>
void launch_extend(igx_device* dev, Slot& s, int grid, const FrameArgs& fa, const PathBuf& in, const PathBuf& out,
                   const KernelCounters& kc, int tail) {
    if (dev->lds_scene_bytes) {
#define L_EXTL(S) hipLaunchKernelGGL((k_extend<S, STATS, true>), dim3(grid), dim3(BLOCK), dev->lds_scene_bytes, dev->stream, fa, dev->sv, in, out, s.sh, s.L, kc, tail)
        IGX_DISPATCH_VARIANT8(dev->variant, L_EXTL);
#undef L_EXTL
        return;
    }
    SceneView tsv = dev->sv;
    tsv.tree_n = dev->tree_ext;
#define L_EXT(S) hipLaunchKernelGGL((k_extend<S, STATS, false>), dim3(grid), dim3(BLOCK), tree_bytes(dev, tsv.tree_n), dev->stream, fa, tsv, in, out, s.sh, s.L, kc, tail)
    IGX_DISPATCH_VARIANT8(dev->variant, L_EXT);
#undef L_EXT
}
// k_trace (the split schedule without persistent lanes): 5 waves per SIMD on
// global tables; LDS-staged tables set occupancy themselves
template <bool STATS>
void launch_trace(igx_device* dev, Slot& s, int grid, const FrameArgs& fa, const PathBuf& in, const int* cnt, int tail,
                  int* work) {
    if (use_refill(dev)) {
#define L_TRR(S)                                                                                                        \
    if (dev->lds_scene_bytes)                                                                                            \
        hipLaunchKernelGGL((k_trace_refill<S, STATS, true>), dim3(grid), dim3(BLOCK), dev->lds_scene_bytes, dev->stream, fa, \
                           dev->sv, in, s.hb, cnt, tail, dev->dstats, refill_min(dev), work);                            \
    else                                                                                                                 \
        hipLaunchKernelGGL((k_trace_refill<S, STATS, false>), dim3(grid), dim3(BLOCK), 0, dev->stream, fa, dev->sv, in, s.hb, \
                           cnt, tail, dev->dstats, refill_min(dev), work)
        IGX_DISPATCH_VARIANT(dev->variant, L_TRR);
#undef L_TRR
        return;
    }
    if (dev->lds_scene_bytes) {
#define L_TRL(S) hipLaunchKernelGGL((k_trace<S, STATS, 1, true>), dim3(grid), dim3(BLOCK), dev->lds_scene_bytes, dev->stream, fa, dev->sv, in, s.hb, cnt, tail, dev->dstats)
        IGX_DISPATCH_VARIANT(dev->variant, L_TRL);
#undef L_TRL
        return;
    }
#define L_TR(S) hipLaunchKernelGGL((k_trace<S, STATS, 5, false>), dim3(grid), dim3(BLOCK), 0, dev->stream, fa, dev->sv, in, s.hb, cnt, tail, dev->dstats)
    IGX_DISPATCH_VARIANT(dev->variant, L_TR);
#undef L_TR
}
template <bool STATS>
void launch_shadow(igx_device* dev, Slot& s, int grid, const int* cnt, int* work, hipStream_t strm) {
    SceneView tsv = dev->sv;
    tsv.tree_n = dev->tree_shadow;
    if (strm != dev->stream) tsv.spill = dev->spill_shadow; // concurrent with the main stream's kernels
    if (use_refill(dev)) {
#define L_SHR(S)                                                                                                        \
    if (dev->lds_scene_bytes)                                                                                            \
        hipLaunchKernelGGL((k_shadow_refill<S, STATS, true>), dim3(grid), dim3(BLOCK), dev->lds_scene_bytes, strm,   \
                           tsv, s.sh, s.L, cnt, dev->dstats, refill_min(dev), work);                                 \
    else                                                                                                                 \
        hipLaunchKernelGGL((k_shadow_refill<S, STATS, false>), dim3(grid), dim3(BLOCK), tree_bytes(dev, tsv.tree_n), strm, \
                           tsv, s.sh, s.L, cnt, dev->dstats, refill_min(dev), work)
#define L_SHRI(S)                                                                                                       \
    hipLaunchKernelGGL((k_shadow_refill<S | 16, STATS, false>), dim3(grid), dim3(BLOCK), tree_bytes(dev, tsv.tree_n), strm, \
                       tsv, s.sh, s.L, cnt, dev->dstats, refill_min(dev), work)
        if (!dev->lds_scene_bytes && use_shadow_ifif(dev)) IGX_DISPATCH_VARIANT(dev->variant, L_SHRI);
        else IGX_DISPATCH_VARIANT(dev->variant, L_SHR);
#undef L_SHRI
#undef L_SHR
        return;
    }
    if (dev->lds_scene_bytes) {
#define L_SHL(S) hipLaunchKernelGGL((k_shadow<S, STATS, true>), dim3(grid), dim3(BLOCK), dev->lds_scene_bytes, strm, tsv, s.sh, s.L, cnt, dev->dstats, work)
        IGX_DISPATCH_VARIANT(dev->variant, L_SHL);
#undef L_SHL
        return;
    }
#define L_SH(S) hipLaunchKernelGGL((k_shadow<S, STATS, false>), dim3(grid), dim3(BLOCK), tree_bytes(dev, tsv.tree_n), strm, tsv, s.sh, s.L, cnt, dev->dstats, work)
    IGX_DISPATCH_VARIANT(dev->variant, L_SH);
#undef L_SH
}
template <bool STATS>
void launch_finish(igx_device* dev, Slot& s, int grid, const FrameArgs& fa, const PathBuf& in, const int* cnt, int tail) {
    SceneView tsv = dev->sv;
    tsv.spill = dev->spill_tail; // k_finish runs concurrently with the main stream's kernels
    tsv.tree_n = 0;              // the tail kernels stage no treelet
    if (dev->lds_scene_bytes) {
#define L_FINL(S) hipLaunchKernelGGL((k_finish<S, STATS, true>), dim3(grid), dim3(BLOCK), dev->lds_scene_bytes, dev->tail_stream, fa, tsv, in, s.L, cnt, tail, dev->dstats, dev->tail_counts)
        IGX_DISPATCH_VARIANT8(dev->variant, L_FINL);
#undef L_FINL
        return;
    }
    if (use_tail_pairs(dev)) {
#define L_FINP(S) hipLaunchKernelGGL((k_finish_pairs<S, STATS>), dim3(grid), dim3(BLOCK), tree_bytes(dev, tsv.tree_n), dev->tail_stream, fa, tsv, in, s.L, cnt, tail, dev->dstats, dev->tail_counts)
        IGX_DISPATCH_VARIANT8(dev->variant, L_FINP);
#undef L_FINP
        return;
    }
#define L_FIN(S) hipLaunchKernelGGL((k_finish<S, STATS, false>), dim3(grid), dim3(BLOCK), tree_bytes(dev, tsv.tree_n), dev->tail_stream, fa, tsv, in, s.L, cnt, tail, dev->dstats, dev->tail_counts)
    IGX_DISPATCH_VARIANT8(dev->variant, L_FIN);
#undef L_FIN
}

// resident blocks per CU of a kernel (persistent grid sizing)
template <typename K>
int resident_blocks(K kernel, size_t dyn_lds = 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, BLOCK, dyn_lds) != hipSuccess || nb < 1) nb = 1;
    return nb;
}
#define IGX_RES1(K, V, ...) return lds ? resident_blocks(K<V, __VA_ARGS__, true>, lds) : resident_blocks(K<V, __VA_ARGS__, false>, tree)
#define IGX_RESIDENT(K, ...)                                         \
    do {                                                             \
        switch (v & (3 | VARIANT_Q4)) {                              \
        case 0: IGX_RES1(K, 0, __VA_ARGS__);                         \
        case 1: IGX_RES1(K, 1, __VA_ARGS__);                         \
        case 2: IGX_RES1(K, 2, __VA_ARGS__);                         \
        case 3: IGX_RES1(K, 3, __VA_ARGS__);                         \
        case 2 | VARIANT_Q4: IGX_RES1(K, 130, __VA_ARGS__);          \
        default: IGX_RES1(K, 131, __VA_ARGS__);                      \
        }                                                            \
    } while (0)
#define IGX_RESIDENT8(K, ...)                                        \
    do {                                                             \
        switch (v & (7 | VARIANT_Q4)) {                              \
        case 0: IGX_RES1(K, 0, __VA_ARGS__);                         \
        case 1: IGX_RES1(K, 1, __VA_ARGS__);                         \
        case 2: IGX_RES1(K, 2, __VA_ARGS__);                         \
        case 3: IGX_RES1(K, 3, __VA_ARGS__);                         \
        case 4: IGX_RES1(K, 4, __VA_ARGS__);                         \
        case 5: IGX_RES1(K, 5, __VA_ARGS__);                         \
        case 6: IGX_RES1(K, 6, __VA_ARGS__);                         \
        case 7: IGX_RES1(K, 7, __VA_ARGS__);                         \
        case 2 | VARIANT_Q4: IGX_RES1(K, 130, __VA_ARGS__);          \
        case 3 | VARIANT_Q4: IGX_RES1(K, 131, __VA_ARGS__);          \
        case 6 | VARIANT_Q4: IGX_RES1(K, 134, __VA_ARGS__);          \
        default: IGX_RES1(K, 135, __VA_ARGS__);                      \
        }                                                            \
    } while (0)
#define IGX_RESIDENT_G(K) IGX_RESIDENT(K, STATS)
template <bool STATS>
int extend_blocks_per_cu(int v, size_t lds, size_t tree) { IGX_RESIDENT8(k_extend, STATS); }
template <bool STATS>
int shadow_blocks_per_cu(int v, size_t lds, bool refill, size_t tree) {
    if (refill) IGX_RESIDENT_G(k_shadow_refill);
    IGX_RESIDENT(k_shadow, STATS);
}
template <bool STATS>
int finish_blocks_per_cu(int v, size_t lds, size_t tree, bool pairs) {
    if (!lds && pairs) {
#define L_RP(S) return resident_blocks(k_finish_pairs<S, STATS>, tree)
        IGX_DISPATCH_VARIANT8(v, L_RP);
#undef L_RP
    }
    IGX_RESIDENT8(k_finish, STATS);
}
template <bool STATS>
int trace_blocks_per_cu(int v, size_t lds, bool refill) {
    const size_t tree = 0; // no treelet (IGX_RES1)
    if (refill) IGX_RESIDENT_G(k_trace_refill);
    if (lds) IGX_RESIDENT(k_trace, STATS, 1);
    IGX_RESIDENT(k_trace, STATS, 5);
}
#undef IGX_RESIDENT
#undef IGX_RESIDENT8
#undef IGX_RESIDENT_G

void launch_shade(igx_device* dev, bool full, int grid, const FrameArgs& fa, const PathBuf& in, const HitBuf& hb,
                  const PathBuf& out, const ShadowBuf& sh, float4* L, const KernelCounters& kc, int tail);
int shade_blocks_per_cu(bool full);
#if IGX_PART == 3
void launch_shade(igx_device* dev, bool full, int grid, const FrameArgs& fa, const PathBuf& in, const HitBuf& hb,
                  const PathBuf& out, const ShadowBuf& sh, float4* L, const KernelCounters& kc, int tail) {
    if (full) hipLaunchKernelGGL(k_shade<true>, dim3(grid), dim3(BLOCK), 0, dev->stream, fa, dev->sv, in, hb, out, sh, L, kc, tail);
    else hipLaunchKernelGGL(k_shade<false>, dim3(grid), dim3(BLOCK), 0, dev->stream, fa, dev->sv, in, hb, out, sh, L, kc, tail);
}
int shade_blocks_per_cu(bool full) { return full ? resident_blocks(k_shade<true>) : resident_blocks(k_shade<false>); }
#endif

// Launch helpers: defined (explicitly instantiated) in their part, extern elsewhere.
#define IGX_EXTEND_HELPERS(X, S)                                                                                     \
    X void launch_extend<S>(igx_device*, Slot&, int, const FrameArgs&, const PathBuf&, const PathBuf&,               \
                            const KernelCounters&, int);                                                             \
    X int extend_blocks_per_cu<S>(int, size_t, size_t);
#define IGX_FINISH_HELPERS(X, S)                                                                                     \
    X void launch_finish<S>(igx_device*, Slot&, int, const FrameArgs&, const PathBuf&, const int*, int);             \
    X int finish_blocks_per_cu<S>(int, size_t, size_t, bool);
#define IGX_TRACE_HELPERS(X, S)                                                                                      \
    X void launch_trace<S>(igx_device*, Slot&, int, const FrameArgs&, const PathBuf&, const int*, int, int*);              \
    X void launch_shadow<S>(igx_device*, Slot&, int, const int*, int*, hipStream_t);                                       \
    X int trace_blocks_per_cu<S>(int, size_t, bool);                                                                  \
    X int shadow_blocks_per_cu<S>(int, size_t, bool, size_t);
#if IGX_PART == 1
IGX_EXTEND_HELPERS(template, true)
IGX_EXTEND_HELPERS(template, false)
#else
IGX_EXTEND_HELPERS(extern template, true)
IGX_EXTEND_HELPERS(extern template, false)
#endif
#if IGX_PART == 2
IGX_FINISH_HELPERS(template, true)
IGX_FINISH_HELPERS(template, false)
#else
IGX_FINISH_HELPERS(extern template, true)
IGX_FINISH_HELPERS(extern template, false)
#endif
#if IGX_PART == 3
IGX_TRACE_HELPERS(template, true)
IGX_TRACE_HELPERS(template, false)
#else
IGX_TRACE_HELPERS(extern template, true)
IGX_TRACE_HELPERS(extern template, false)
#endif
#undef IGX_RES1

#if IGX_PART == 0
// Wait for the chunk last run in `s` and fold its statistics in.
igx_status harvest(igx_device* dev, Slot& s) {
    if (!s.pending) return IGX_OK;
    HIPCHK(hipEventSynchronize(s.done));
    auto c = [&](int r) { return (uint64_t)row_total(s, r); };
    dev->stats.camera_rays += (uint64_t)s.camera;
    for (int b = 1; b <= s.switch_bounce; ++b) dev->stats.bounce_rays += c(2 * b);
    for (int b = 0; b < s.switch_bounce; ++b) dev->stats.shadow_rays += c(2 * b + 1);
    for (int b = 0; b < s.switch_bounce; ++b) dev->stats.extend_rays += c(2 * b);
    for (int b = 1; b <= s.switch_bounce; ++b) dev->stats.extend_paths_out += c(2 * b);
    // every queued launch counts (as rocprofv3 sees them), including one that
    // found the live count at or below the tail threshold and exited at once
    dev->stats.launches_extend += (uint64_t)s.launched;
    dev->stats.launches_shadow += (uint64_t)s.launched;
    if (s.split) dev->stats.launches_trace += (uint64_t)s.launched;
    bool finished = s.switch_bounce < MAX_BOUNCES && c(2 * s.switch_bounce) > 0;
    dev->stats.launches_finish += finished ? 1 : 0;
    if (dev->timing) {
        for (auto& t : s.timed) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, t.a, t.b);
            if (t.kind == 0) dev->stats.ms_extend += ms;
            else if (t.kind == 1) dev->stats.ms_shadow += ms;
            else if (t.kind == 2) dev->stats.ms_generate += ms;
            else if (t.kind == 3) dev->stats.ms_resolve += ms;
            else if (t.kind == 4 && finished) dev->stats.ms_finish += ms;
            else if (t.kind == 5) dev->stats.ms_trace += ms;
        }
    }
    s.timed.clear();
    s.ev_next = 0;
    s.pending = false;
    return IGX_OK;
}

igx_status drain(igx_device* dev) {
    igx_status st;
    if ((st = ::wait_idle(dev)) || (st = harvest(dev, dev->slots[0])) || (st = harvest(dev, dev->slots[1]))) return st;
    HIPCHK(hipStreamSynchronize(dev->stream));
    HIPCHK(hipStreamSynchronize(dev->stream2));
    HIPCHK(hipStreamSynchronize(dev->shadow_stream));
    HIPCHK(hipStreamSynchronize(dev->tail_stream));
    unsigned long long tc[2] = {0, 0};
    HIPCHK(hipMemcpy(tc, dev->tail_counts, sizeof(tc), hipMemcpyDeviceToHost));
    HIPCHK(hipMemset(dev->tail_counts, 0, sizeof(tc)));
    dev->stats.bounce_rays += tc[0];
    dev->stats.shadow_rays += tc[1];
    dev->stats.tail_bounce_rays += tc[0];
    dev->stats.tail_shadow_rays += tc[1];
    return IGX_OK;
}

// Treelet size of every global-table kernel: the largest prefix of the hot
// node order (order_hot_nodes) whose LDS copy keeps the kernel's resident
// blocks per CU (set by its register budget) -- the treelet takes LDS that
// would otherwise stay unused.  Binary search over hipOccupancy answers.
void configure_treelet(igx_device* dev) {
    dev->tree_ext = dev->tree_shadow = 0;
    dev->tree_dirty = false;
    if (!dev->has_scene || dev->lds_scene_bytes || dev->treelet_opt == 0) return;
    int cap = (int)std::min<size_t>(TREELET_FRONT, (size_t)dev->sv.num_nodes);
    if (dev->treelet_opt > 0) cap = (int)std::min<int64_t>(cap, dev->treelet_opt);
    const int v = dev->variant;
    const bool refill = use_refill(dev);
    auto fit = [&](auto blocks) {
        const int nb0 = blocks((size_t)0);
        int lo = 0, hi = cap;
        while (lo < hi) {
            const int mid = (lo + hi + 1) / 2;
            if (blocks(tree_bytes(dev, mid)) >= nb0) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    if (EXTEND_TREELET) dev->tree_ext = fit([&](size_t t) { return extend_blocks_per_cu<false>(v, 0, t); });
    // the if-if shadow kernel of the split schedule: global node loads beat a
    // treelet's flat loads there (profiles/r03_ab_treelet_global.log)
    if (SHADOW_TREELET && !(refill && use_shadow_ifif(dev))) dev->tree_shadow = fit([&](size_t t) { return shadow_blocks_per_cu<false>(v, 0, refill, t); });
    // k_trace_refill and the tail kernels: none -- the tail kernel overlaps the
    // next chunk's kernels, and LDS it holds keeps their blocks off the CU
    // (soup-1M frame +4 % with one)
}

// Film pixels among the chunk's local pixels (tiles at the film's right and
// bottom edges hang over it): per tile in closed form, the valid pixels among
// a tile's first m row-major pixels being min(m / T, h) * w + (m / T < h ?
// min(m % T, w) : 0).  (A per-pixel loop cost 8 ms of host time per 67 M-path
// config-5 chunk, during which the GPU idled: profiles/r04_timeline_gaps.log.)
long long valid_pixels_in_chunk(const FrameArgs& fa) {
    if (fa.num_rays > 0 || fa.tile_size <= 0) return fa.chunk_pixels;
    long long v = 0;
    const long long T = fa.tile_size, TT = T * T;
    const long long c0 = fa.chunk_pixel0, c1 = c0 + fa.chunk_pixels;
    for (long long k = c0 / TT; k * TT < c1; ++k) {
        const long long t = fa.tile_offset + k * fa.tile_stride;
        const long long ty = t / fa.tiles_x, tx = t - ty * fa.tiles_x;
        const long long w = std::max(0ll, std::min(T, fa.width - tx * T)), h = std::max(0ll, std::min(T, fa.height - ty * T));
        auto valid_first = [&](long long m) { // valid pixels among the tile's first m
            if (IGX_PIXEL_BLOCKS && (T & 3) == 0) { // 4 x 2 blocks along row pairs (block_order)
                const long long pairs = m / (2 * T), q = m - pairs * 2 * T, nb = q / 8, rem = q - nb * 8;
                const long long y0 = 2 * pairs, c0 = 4 * nb + std::min(rem, 4ll), c1 = 4 * nb + std::max(0ll, rem - 4);
                return std::min(y0, h) * w + (y0 < h ? std::min(c0, w) : 0) + (y0 + 1 < h ? std::min(c1, w) : 0);
            }
            const long long rows = m / T;
            return std::min(rows, h) * w + (rows < h ? std::min(m % T, w) : 0);
        };
        v += valid_first(std::min(TT, c1 - k * TT)) - valid_first(std::max(0ll, c0 - k * TT));
    }
    return v;
}

DevCamera make_camera(const igx_device* dev, int width, int height) {
    // make_perspective_camera (camera/perspective.art:29-42), compute_scale_from_{h,v}fov (:2-14)
    const igx_camera& c = dev->cam_desc;
    DevCamera k{};
    float aspect = c.aspect > 0 ? c.aspect : (float)width / (float)height;
    if (c.vertical_fov) {
        k.scale_y = std::tan(c.fov / 2);
        k.scale_x = k.scale_y * aspect;
    } else {
        k.scale_x = std::tan(c.fov / 2);
        k.scale_y = k.scale_x / aspect;
    }
    float dir[3] = {c.dir[0], c.dir[1], c.dir[2]}, up[3] = {c.up[0], c.up[1], c.up[2]};
    float r[3] = {dir[1] * up[2] - dir[2] * up[1], dir[2] * up[0] - dir[0] * up[2], dir[0] * up[1] - dir[1] * up[0]};
    float rl = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    float irl = 1 / rl;
    for (int i = 0; i < 3; ++i) {
        k.eye[i] = c.eye[i];
        k.dir[i] = dir[i];
        k.up[i] = up[i];
        k.right[i] = r[i] * irl;
    }
    k.tmin = c.near_clip;
    k.tmax = c.far_clip;
    return k;
}

#endif // IGX_PART == 0

} // namespace

#if IGX_PART == 0
// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" const char* igx_version(void) { return "igx 0.2 (gfx950 wavefront path tracer)"; }

extern "C" igx_status igx_create(int hip_device, igx_device** out) {
    if (!out) return IGX_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    igx_device* dev = new igx_device();
    dev->hip_device = hip_device;
    hipError_t e = hipSetDevice(hip_device);
    if (e != hipSuccess) {
        delete dev;
        return IGX_ERR_HIP;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, hip_device) == hipSuccess) {
        dev->num_cus = prop.multiProcessorCount;
        dev->mem_total = prop.totalGlobalMem;
    }
    if (hipStreamCreateWithFlags(&dev->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&dev->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&dev->tail_stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&dev->shadow_stream, hipStreamNonBlocking) != hipSuccess) {
        delete dev;
        return IGX_ERR_HIP;
    }
    if (hipMalloc((void**)&dev->dstats, DSTATS * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc((void**)&dev->tail_counts, 2 * sizeof(unsigned long long)) != hipSuccess) {
        delete dev;
        return IGX_ERR_OUT_OF_MEMORY;
    }
    (void)hipMemset(dev->dstats, 0, DSTATS * sizeof(unsigned long long));
    (void)hipMemset(dev->tail_counts, 0, 2 * sizeof(unsigned long long));
    *out = dev;
    return IGX_OK;
}

extern "C" igx_status igx_destroy(igx_device* dev) {
    if (!dev) return IGX_ERR_INVALID_ARGUMENT;
    (void)hipSetDevice(dev->hip_device);
    (void)wait_idle(dev);
    stop_async(dev);
    if (dev->stream) (void)hipStreamSynchronize(dev->stream);
    if (dev->stream2) (void)hipStreamSynchronize(dev->stream2);
    if (dev->tail_stream) (void)hipStreamSynchronize(dev->tail_stream);
    if (dev->shadow_stream) (void)hipStreamSynchronize(dev->shadow_stream);
    free_scene(dev);
    for (auto& s : dev->slots) {
        free_slot_buffers(s);
        if (s.ctr) (void)hipFree(s.ctr);
        if (s.pinned) (void)hipHostFree(s.pinned);
        if (s.done) (void)hipEventDestroy(s.done);
        for (auto& e : s.ev_pool) (void)hipEventDestroy(e);
    }
    if (dev->fb) (void)hipFree(dev->fb);
    for (float* a : dev->aov_fb)
        if (a) (void)hipFree(a);
    if (dev->dstats) (void)hipFree(dev->dstats);
    if (dev->tail_counts) (void)hipFree(dev->tail_counts);
    if (dev->ray_list) (void)hipFree(dev->ray_list);
    if (dev->stream) (void)hipStreamDestroy(dev->stream);
    if (dev->stream2) (void)hipStreamDestroy(dev->stream2);
    if (dev->tail_stream) (void)hipStreamDestroy(dev->tail_stream);
    if (dev->shadow_stream) (void)hipStreamDestroy(dev->shadow_stream);
    delete dev;
    return IGX_OK;
}

extern "C" const char* igx_last_error(const igx_device* dev) { return dev ? dev->last_error.c_str() : "null device"; }

extern "C" igx_status igx_set_option(igx_device* dev, const char* key, int64_t value) {
    if (!dev || !key) return IGX_ERR_INVALID_ARGUMENT;
    // options change what queued work reads: let the worker drain first
    if (igx_status w = wait_idle(dev); w != IGX_OK) return w;
    std::string k(key);
    dev->tree_dirty = true; // schedule options change which kernels run, and so their treelets
    if (k == "timing") dev->timing = value != 0;
    else if (k == "instrument") dev->instrument = value != 0;
    else if (k == "capacity") dev->capacity_opt = value;
    else if (k == "treelet") {
        if (value < -1) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "treelet must be -1 (auto), 0 (off) or a node count");
        dev->treelet_opt = value;
        dev->tree_dirty = true;
    }
    else if (k == "shadow_classes") dev->shadow_classes_opt = value != 0;
    else if (k == "overlap_shadow") dev->overlap_shadow_opt = value != 0;
    else if (k == "bvh_quantize") {
        if (value < -1 || value > 1) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "bvh_quantize must be -1 (auto), 0 or 1");
        dev->quantize_opt = (int)value;
    }
    else if (k == "tail_pairs") {
        if (value < -1 || value > 1) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "tail_pairs must be -1 (auto), 0 or 1");
        dev->tail_pairs_opt = (int)value;
    }
    else if (k == "stream_slots") {
        if (value != 1 && value != 2) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "stream_slots must be 1 or 2");
        if (value == 1 && dev->slots[1].cap) { // give the second slot's memory back
            igx_status st = harvest(dev, dev->slots[1]);
            if (st != IGX_OK) return st;
            free_slot_buffers(dev->slots[1]);
        }
        dev->stream_slots = (int)value;
    }
    else if (k == "slot_budget_mb") {
        if (value < 0) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "slot_budget_mb must be >= 0 (0 = auto)");
        dev->slot_budget_mb = value;
    }
    else if (k == "concurrent_chunks") dev->concurrent_opt = value != 0 ? 1 : 0;
    else if (k == "async_render") dev->async_opt = value != 0 ? 1 : 0;
    else if (k == "probe_sample") dev->probe_sample_opt = std::max<int64_t>(0, value);
    else if (k == "fail_chunk") dev->fail_chunk_opt = std::max<int64_t>(0, value);
    else if (k == "face_shade") dev->face_shade_opt = value != 0 ? 1 : 0;
    else if (k == "host_wait_us") dev->host_wait_us = (int)std::max<int64_t>(0, std::min<int64_t>(value, 10000));
    else if (k == "concurrent_start_pct") {
        if (value < 0 || value > 100) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "concurrent_start_pct must be 0..100");
        dev->concurrent_start_pct = (int)value;
    }
    else if (k == "tail_threshold") dev->tail_opt = value;
    else if (k == "tail_threshold_last") dev->tail_last_opt = value;
    else if (k == "fuse_generate") dev->fuse_generate = value != 0;
    else if (k == "split") {
        if (value < -1 || value > 1) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "split must be -1 (auto), 0 or 1");
        dev->split_opt = (int)value;
    }
    else if (k == "shadow_ifif") {
        if (value < -1 || value > 1) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "shadow_ifif must be -1 (auto), 0 or 1");
        dev->shadow_ifif_opt = (int)value;
    }
    else if (k == "refill") {
        if (value < -1 || value > 64) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "refill must be -1 (auto) or in [0, 64]");
        dev->refill_opt = (int)value;
    }
    else if (k == "lds_scene_max") {
        dev->lds_scene_max = value;
        size_t b = ((size_t)dev->sv.num_nodes * dev->sv.node_f4 + (size_t)dev->sv.num_inst * 4 +
                    (size_t)dev->sv.num_tris * 3) * 16; // LDS layout (stage_scene_lds)
        dev->lds_scene_bytes = dev->has_scene && (int64_t)b <= value ? b : 0;
    }
    else if (k == "full_shading") dev->full_shading_opt = value != 0;
    else if (k == "enclosing") dev->enclosing_opt = value != 0;
    else if (k == "bvh_width") {
        if (value != 0 && value != 2 && value != 4) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "bvh_width must be 0 (auto), 2 or 4");
        dev->bvh_width_opt = (int)value;
    }
    else if (k == "spatial_splits") dev->spatial_splits = value != 0;
    else if (k == "rebuild_bvh") dev->rebuild_bvh = value != 0;
    else if (k == "dynamic") dev->dynamic_opt = (int)(value & 15);
    else if (k == "group_order") {
        if (value < -1 || value > 1) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "group_order must be -1 (auto), 0 (A, B, C) or 1 (C, B, A)");
        dev->group_order_opt = (int)value;
    }
    else if (k == "face_normals") dev->face_normals_opt = value != 0;
    else if (k == "bvh_bins") {
        if (value < 2 || value > 4096) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "bvh_bins must be in [2, 4096]");
        dev->bvh_bins = (int)value;
    }
    else if (k == "bvh_bins_tlas") {
        if (value < 2 || value > 4096) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "bvh_bins_tlas must be in [2, 4096]");
        dev->bvh_bins_tlas = (int)value;
    }
    else if (k == "path_classes") {
        if (value < 0 || value > 4) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "path_classes must be in [0, 4]");
        dev->classify_opt = (int)value;
    }
    else if (k == "sah_node_cost_pct") {
        if (value < 10 || value > 2000) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "sah_node_cost_pct must be in [10, 2000]");
        dev->sah_node_cost = (float)value / 100.0f;
    }
    else if (k == "bvh_leaf_size") {
        if (value < 1 || value > 16) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "bvh_leaf_size must be in [1, 16]");
        dev->leaf_size = (int)value;
    } else return fail(dev, IGX_ERR_INVALID_ARGUMENT, "unknown option '" + k + "'");
    return IGX_OK;
}

extern "C" igx_status igx_wait_ready(igx_device* dev) {
    if (!dev) return IGX_ERR_INVALID_ARGUMENT;
    return wait_ready(dev);
}

extern "C" igx_status igx_synchronize(igx_device* dev) {
    if (!dev) return IGX_ERR_INVALID_ARGUMENT;
    HIPCHK(hipSetDevice(dev->hip_device));
    return drain(dev);
}

// A closed triangle mesh: with vertices welded by position, every edge
// borders exactly two faces (paths that enter it by transmission then hit it
// again before leaving).  Checked up to 1 M faces.
// Hot order of the node array for the LDS treelet (stage_treelet): the
// `front` inner nodes a ray most likely visits move to indices [0, front), so
// a kernel stages any prefix of the array as its treelet.  Visit likelihood
// follows the surface-area heuristic: the TLAS root has 1; a child has its
// parent's times the child box's area over the union of the sibling boxes
// (the chance a ray through the parent also crosses the child); a BLAS root
// collects the likelihood of every TLAS leaf that instances it.  The other
// nodes keep their relative (depth-first) order.  Every inner-node reference
// (node children, instance BLAS roots, the TLAS root) is renumbered; the
// traversal result does not depend on node numbering.
// `format`: 2 (BVH2, 64 B), 4 (4-wide, 128 B) or 5 (quantised 4-wide, 64 B).
static void order_hot_nodes(std::vector<float4>& nodes, int format, std::vector<float4>& inst, int& tlas_root, size_t front) {
    const int nf4 = format == 4 ? 8 : 4;
    const size_t nn = nodes.size() / nf4;
    if (nn == 0 || front == 0) return;
    const int width = format == 2 ? 2 : 4;
    auto ref = [&](size_t n, int k) -> int32_t& {
        return reinterpret_cast<int32_t*>(&nodes[n * nf4])[format == 4 ? 24 + k : 12 + k];
    };
    auto box = [&](size_t n, int k, float lo[3], float hi[3]) {
        const float* f = reinterpret_cast<const float*>(&nodes[n * nf4]);
        if (format == 5) { // origin + code * scale (Bvh4QNode)
            const uint32_t* u = reinterpret_cast<const uint32_t*>(f);
            const float sc[3] = {f[3], f[4], f[5]};
            for (int a = 0; a < 3; ++a) {
                lo[a] = f[a] + (float)((u[6 + 2 * a] >> (8 * k)) & 255u) * sc[a];
                hi[a] = f[a] + (float)((u[7 + 2 * a] >> (8 * k)) & 255u) * sc[a];
            }
            if (ref(n, k) == igx::kEmptyRef) lo[0] = INFINITY;
            return;
        }
        for (int a = 0; a < 3; ++a) {
            lo[a] = width == 4 ? f[8 * a + k] : f[6 * k + 2 * a];
            hi[a] = width == 4 ? f[8 * a + 4 + k] : f[6 * k + 2 * a + 1];
        }
    };
    auto half_area = [](const float lo[3], const float hi[3]) -> double {
        for (int a = 0; a < 3; ++a)
            if (!std::isfinite(lo[a]) || !std::isfinite(hi[a]) || lo[a] > hi[a]) return 0.0;
        const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
        return dx * dy + dy * dz + dz * dx;
    };
    // children of node n with the node's likelihood pn: f(child ref, child likelihood)
    auto children = [&](size_t n, double pn, auto&& f) {
        float ulo[3] = {INFINITY, INFINITY, INFINITY}, uhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double ak[4] = {0, 0, 0, 0};
        for (int k = 0; k < width; ++k) {
            float lo[3], hi[3];
            box(n, k, lo, hi);
            ak[k] = half_area(lo, hi);
            if (ak[k] <= 0) continue;
            for (int a = 0; a < 3; ++a) {
                ulo[a] = std::min(ulo[a], lo[a]);
                uhi[a] = std::max(uhi[a], hi[a]);
            }
        }
        const double ua = half_area(ulo, uhi);
        for (int k = 0; k < width; ++k) {
            const int32_t r = ref(n, k);
            if (r == igx::kEmptyRef || ak[k] <= 0) continue;
            f(r, ua > 0 ? pn * std::min(1.0, ak[k] / ua) : pn);
        }
    };
    std::vector<double> p(nn, 0.0), pblas(nn, 0.0);
    auto instances = [&](int32_t leaf, double pl) { // TLAS leaf: its instances' BLAS roots
        const int code = ~leaf;
        const int first = code >> igx::kLeafCountBits, count = (code & ((1 << igx::kLeafCountBits) - 1)) + 1;
        for (int k = 0; k < count; ++k) {
            int4 info;
            std::memcpy(&info, &inst[4 * (size_t)(first + k) + 3], 16);
            if (info.y == 0 && info.z >= 0 && (size_t)info.z < nn) pblas[info.z] += pl;
        }
    };
    std::vector<std::pair<int32_t, double>> todo;
    if (tlas_root >= 0) todo.push_back({tlas_root, 1.0});
    else if (!inst.empty()) instances(tlas_root, 1.0); // one entity: the root is its leaf
    while (!todo.empty()) { // TLAS (a tree)
        const auto [n, pn] = todo.back();
        todo.pop_back();
        p[n] += pn;
        children((size_t)n, pn, [&](int32_t r, double pc) {
            if (r >= 0) todo.push_back({r, pc});
            else instances(r, pc);
        });
    }
    for (size_t r = 0; r < nn; ++r) { // every BLAS from its root (a BLAS is a tree; shared BLAS summed at the root)
        if (pblas[r] <= 0) continue;
        todo.push_back({(int32_t)r, pblas[r]});
        while (!todo.empty()) {
            const auto [n, pn] = todo.back();
            todo.pop_back();
            p[n] += pn;
            children((size_t)n, pn, [&](int32_t c, double pc) {
                if (c >= 0) todo.push_back({c, pc});
            });
        }
    }
    std::vector<int32_t> order(nn);
    for (size_t i = 0; i < nn; ++i) order[i] = (int32_t)i;
    front = std::min(front, nn);
    std::partial_sort(order.begin(), order.begin() + front, order.end(), [&](int32_t a, int32_t b) {
        return p[a] != p[b] ? p[a] > p[b] : a < b;
    });
    std::vector<int32_t> newidx(nn, -1);
    for (size_t i = 0; i < front; ++i) newidx[order[i]] = (int32_t)i;
    int32_t next = (int32_t)front;
    for (size_t i = 0; i < nn; ++i)
        if (newidx[i] < 0) newidx[i] = next++;
    std::vector<float4> out(nodes.size());
    for (size_t i = 0; i < nn; ++i) std::copy(&nodes[i * nf4], &nodes[i * nf4] + nf4, &out[(size_t)newidx[i] * nf4]);
    nodes.swap(out);
    for (size_t i = 0; i < nn; ++i)
        for (int k = 0; k < width; ++k)
            if (ref(i, k) >= 0) ref(i, k) = newidx[ref(i, k)];
    for (size_t slot = 0; slot < inst.size() / 4; ++slot) {
        int4 info;
        std::memcpy(&info, &inst[4 * slot + 3], 16);
        if (info.y == 0 && info.z >= 0) {
            info.z = newidx[info.z];
            std::memcpy(&inst[4 * slot + 3], &info, 16);
        }
    }
    if (tlas_root >= 0) tlas_root = newidx[tlas_root];
}

static bool closed_mesh(const igx_mesh& m) {
    if (m.num_faces < 4 || m.num_faces > (1u << 20)) return false;
    std::map<std::array<float, 3>, uint32_t> weld;
    std::vector<uint32_t> id(m.num_vertices);
    for (uint32_t v = 0; v < m.num_vertices; ++v)
        id[v] = weld.emplace(std::array<float, 3>{m.vertices[3 * v], m.vertices[3 * v + 1], m.vertices[3 * v + 2]}, (uint32_t)weld.size()).first->second;
    std::map<std::pair<uint32_t, uint32_t>, int> edges;
    for (uint32_t f = 0; f < m.num_faces; ++f)
        for (int k = 0; k < 3; ++k) {
            uint32_t a = id[m.indices[3 * f + k]], b = id[m.indices[3 * f + (k + 1) % 3]];
            if (a == b) return false;
            ++edges[{std::min(a, b), std::max(a, b)}];
        }
    for (const auto& e : edges)
        if (e.second != 2) return false;
    return true;
}

extern "C" igx_status igx_upload_scene(igx_device* dev, const igx_scene_desc* desc) {
    if (!dev || !desc) return IGX_ERR_INVALID_ARGUMENT;
    HIPCHK(hipSetDevice(dev->hip_device));
    reset_async_failure(dev); // a new scene starts the handle afresh
    igx_status dst = drain(dev);
    if (dst != IGX_OK) return dst;
    free_scene(dev);

    // ---- phase 1: BVH2 of every trimesh shape and of the entity TLAS ------
    std::vector<igx::BvhBuildResult> brs(desc->num_shapes);
    int blas_depth2 = 0;
    for (uint32_t s = 0; s < desc->num_shapes; ++s) {
        const igx_shape& sh = desc->shapes[s];
        if (sh.type == IGX_SHAPE_SPHERE) continue;
        if (sh.mesh < 0 || (uint32_t)sh.mesh >= desc->num_meshes)
            return fail(dev, IGX_ERR_INVALID_ARGUMENT, "shape references an invalid mesh");
        const igx_mesh& m = desc->meshes[sh.mesh];
        igx::BvhBuildInput bi;
        bi.bmin.resize(3 * m.num_faces);
        bi.bmax.resize(3 * m.num_faces);
        bi.centroid.resize(3 * m.num_faces);
        for (uint32_t f = 0; f < m.num_faces; ++f) {
            for (int a = 0; a < 3; ++a) {
                float lo = 3.4e38f, hi = -3.4e38f;
                for (int k = 0; k < 3; ++k) {
                    uint32_t vi = m.indices[3 * f + k];
                    if (vi >= m.num_vertices) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "mesh index out of range");
                    float v = m.vertices[3 * vi + a];
                    lo = std::min(lo, v);
                    hi = std::max(hi, v);
                }
                bi.bmin[3 * f + a] = lo;
                bi.bmax[3 * f + a] = hi;
                bi.centroid[3 * f + a] = 0.5f * (lo + hi);
            }
        }
        if (sh.ref_bvh && !dev->rebuild_bvh) {
            // the reference loader's BLAS (Node2 + Tri1, TriMeshProvider.cpp:553-554)
            std::string err;
            if (!igx::bvh2_from_reference(sh.ref_bvh, sh.ref_bvh_bytes, m.num_faces, brs[s], err))
                return fail(dev, IGX_ERR_INVALID_ARGUMENT, "shape " + std::to_string(s) + ": " + err);
            blas_depth2 = std::max(blas_depth2, brs[s].depth);
            continue;
        }
        try {
            if (dev->spatial_splits && m.num_faces <= SPATIAL_SPLIT_MAX_FACES) {
                std::vector<float> tv(9 * (size_t)m.num_faces);
                for (uint32_t f = 0; f < m.num_faces; ++f)
                    for (int k = 0; k < 3; ++k)
                        for (int a = 0; a < 3; ++a) tv[9 * (size_t)f + 3 * k + a] = m.vertices[3 * m.indices[3 * f + k] + a];
                brs[s] = igx::build_sbvh2(bi, tv, dev->leaf_size);
            } else {
                brs[s] = igx::build_bvh2(bi, dev->leaf_size, dev->bvh_bins, dev->sah_node_cost);
            }
        } catch (const std::exception& ex) {
            return fail(dev, IGX_ERR_INVALID_ARGUMENT, ex.what());
        }
        blas_depth2 = std::max(blas_depth2, brs[s].depth);
    }
    igx::BvhBuildResult tlas_br;
    if (desc->num_entities > 0) {
        igx::BvhBuildInput bi;
        for (uint32_t e = 0; e < desc->num_entities; ++e) {
            const igx_entity& en = desc->entities[e];
            if (en.shape < 0 || (uint32_t)en.shape >= desc->num_shapes)
                return fail(dev, IGX_ERR_INVALID_ARGUMENT, "entity references an invalid shape");
            if (en.material < 0 || (uint32_t)en.material >= desc->num_materials)
                return fail(dev, IGX_ERR_INVALID_ARGUMENT, "entity references an invalid material");
            for (int a = 0; a < 3; ++a) {
                bi.bmin.push_back(en.bbox_min[a]);
                bi.bmax.push_back(en.bbox_max[a]);
                bi.centroid.push_back(0.5f * (en.bbox_min[a] + en.bbox_max[a]));
            }
        }
        tlas_br = igx::build_bvh2(bi, 1, dev->bvh_bins_tlas);
    }
    // Node width: BVH2 while its whole stack fits the LDS column (fewer,
    // cheaper node steps on small scenes), else 4-wide nodes (half the node
    // iterations on deep trees; the deepest entries spill).  Option
    // "bvh_width" forces either.
    const int width = dev->bvh_width_opt == 2 || dev->bvh_width_opt == 4
                          ? dev->bvh_width_opt
                          : (tlas_br.depth + blas_depth2 + 3 <= LDS_STACK ? 2 : 4);
    // 4-wide nodes quantised to 64 B (Bvh4QNode) on the split schedule's
    // scenes, whose node fetches go to the Infinity Cache / HBM (soup-16M frame
    // 74.7 -> 70.0, soup-1M 98.2 -> 92.8 ms); where the tables stay on chip the
    // decode only costs instructions (primitives 8.6 -> 9.4, S-deep 46.7 -> 49.5)
    size_t est_tri = 0;
    for (const auto& b : brs) est_tri += b.prim_order.size();
    const size_t est_bytes = est_tri * 48 + (size_t)desc->num_entities * 64 + (est_tri / 2 + desc->num_entities) * 128;
    const bool quantize = width == 4 && (dev->quantize_opt == 1 || (dev->quantize_opt < 0 && est_bytes > SPLIT_TABLE_BYTES));
    const int nf4 = quantize ? 4 : node_f4(width);

    // ---- phase 2: node, triangle and instance tables ----------------------
    std::vector<float4> nodes; // nf4 float4s per node
    std::vector<float4> tris, vtx, nrm, spheres;
    std::vector<float2> uvs; // texture coordinates, only for scenes with a textured material
    bool textured = false;
    for (uint32_t i = 0; i < desc->num_materials; ++i) textured = textured || desc->materials[i].texture != IGX_TEXTURE_NONE;
    std::vector<int4> idx;
    // per face: vertex normals and indices in one record (SceneView::fsh),
    // for scenes with at most FACE_SHADE_MAX faces over all meshes (48 B each)
    std::vector<float4> fsh;
    size_t total_faces = 0;
    for (uint32_t i = 0; i < desc->num_shapes; ++i)
        if (desc->shapes[i].type != IGX_SHAPE_SPHERE && desc->shapes[i].mesh >= 0) total_faces += desc->meshes[desc->shapes[i].mesh].num_faces;
    const bool with_fsh = dev->face_shade_opt && total_faces <= FACE_SHADE_MAX;
    // Append a built BVH2 (as Node2, or collapsed to 4-wide nodes) to the
    // unified node array: inner refs move by the array offset, leaf codes by
    // `leaf_off` slots.  Returns the node offset; `need` = stack entries the
    // tree can occupy.
    auto append_nodes = [&](const igx::BvhBuildResult& br, int leaf_off, int& need) -> int {
        const int node_off = (int)(nodes.size() / nf4);
        auto move_leaf = [&](int32_t ref) {
            int code = ~ref;
            return igx::encode_leaf((code >> igx::kLeafCountBits) + leaf_off, (code & ((1 << igx::kLeafCountBits) - 1)) + 1);
        };
        if (width == 2) {
            for (auto nd : br.nodes) {
                for (int k = 0; k < 2; ++k) {
                    if (nd.ref[k] >= 0) nd.ref[k] += node_off;
                    else if (nd.ref[k] != igx::kEmptyRef && nd.b[k * 6] <= nd.b[k * 6 + 1])
                        nd.ref[k] = move_leaf(nd.ref[k]); // empty and absent children keep their code
                }
                float4 f[4];
                std::memcpy(f, &nd, 64);
                nodes.insert(nodes.end(), f, f + 4);
            }
            need = br.depth;
        } else {
            igx::Bvh4Result b4 = igx::collapse_bvh4(br);
            for (auto nd : b4.nodes) {
                for (int k = 0; k < 4; ++k) {
                    if (nd.ref[k] >= 0) nd.ref[k] += node_off;
                    else if (nd.ref[k] != igx::kEmptyRef) nd.ref[k] = move_leaf(nd.ref[k]);
                }
                if (quantize) {
                    const igx::Bvh4QNode qn = igx::quantize_bvh4(nd);
                    float4 f[4];
                    std::memcpy(f, &qn, 64);
                    nodes.insert(nodes.end(), f, f + 4);
                } else {
                    float4 f[8];
                    std::memcpy(f, &nd, 128);
                    nodes.insert(nodes.end(), f, f + 8);
                }
            }
            need = b4.stack_need;
        }
        return node_off;
    };
    struct ShapeDev { int type, root, vtx_off, idx_off_or_sphere; };
    std::vector<ShapeDev> sdev(desc->num_shapes);
    int blas_depth = 0;
    for (uint32_t s = 0; s < desc->num_shapes; ++s) {
        const igx_shape& sh = desc->shapes[s];
        if (sh.type == IGX_SHAPE_SPHERE) {
            sdev[s] = {1, -1, 0, (int)spheres.size()};
            spheres.push_back(make_float4(sh.sphere[0], sh.sphere[1], sh.sphere[2], sh.sphere[3]));
            continue;
        }
        const igx_mesh& m = desc->meshes[sh.mesh];
        const igx::BvhBuildResult& br = brs[s];
        int tri_off = (int)(tris.size() / 3);
        if (tri_off + br.prim_order.size() >= (size_t)(1 << 26))
            return fail(dev, IGX_ERR_UNSUPPORTED, "too many triangles for the leaf encoding");
        int need = 0;
        int node_off = append_nodes(br, tri_off, need);
        blas_depth = std::max(blas_depth, need);
        for (uint32_t slot = 0; slot < br.prim_order.size(); ++slot) {
            uint32_t f = br.prim_order[slot];
            const uint32_t* ix = m.indices + 3 * f;
            const float* v0 = m.vertices + 3 * ix[0];
            const float* v1 = m.vertices + 3 * ix[1];
            const float* v2 = m.vertices + 3 * ix[2];
            // Tri1 (shapes/trimesh.art:107-114; TriBVHAdapter.h:148-158): e1 = v0 - v1, e2 = v2 - v0
            float4 q0 = make_float4(v0[0], v0[1], v0[2], 0);
            int32_t pid = (int32_t)f;
            std::memcpy(&q0.w, &pid, 4);
            tris.push_back(q0);
            tris.push_back(make_float4(v0[0] - v1[0], v0[1] - v1[1], v0[2] - v1[2], 0));
            tris.push_back(make_float4(v2[0] - v0[0], v2[1] - v0[1], v2[2] - v0[2], 0));
        }
        // a BLAS that is a single leaf is entered at the leaf itself
        int root_ref = node_off;
        if (br.root_is_leaf) {
            int code = ~br.root_leaf_ref;
            root_ref = igx::encode_leaf((code >> igx::kLeafCountBits) + tri_off, (code & ((1 << igx::kLeafCountBits) - 1)) + 1);
        }
        sdev[s] = {0, root_ref, (int)vtx.size(), (int)idx.size()};
        for (uint32_t v = 0; v < m.num_vertices; ++v) {
            vtx.push_back(make_float4(m.vertices[3 * v], m.vertices[3 * v + 1], m.vertices[3 * v + 2], 0));
            nrm.push_back(make_float4(m.normals[3 * v], m.normals[3 * v + 1], m.normals[3 * v + 2], 0));
            if (textured) uvs.push_back(m.texcoords ? make_float2(m.texcoords[2 * v], m.texcoords[2 * v + 1]) : make_float2(0, 0));
        }
        for (uint32_t f = 0; f < m.num_faces; ++f)
            idx.push_back(make_int4((int)m.indices[3 * f], (int)m.indices[3 * f + 1], (int)m.indices[3 * f + 2], 0));
        if (with_fsh)
            for (uint32_t f = 0; f < m.num_faces; ++f)
                for (int k = 0; k < 3; ++k) {
                    const uint32_t v = m.indices[3 * f + k];
                    float4 r = make_float4(m.normals[3 * v], m.normals[3 * v + 1], m.normals[3 * v + 2], 0);
                    const int vi = (int)v;
                    std::memcpy(&r.w, &vi, 4);
                    fsh.push_back(r);
                }
        brs[s] = igx::BvhBuildResult{}; // release the host copy
    }

    // ---- TLAS over entities (leaf size 1), instance records ---------------
    std::vector<float4> inst, ent;
    std::vector<int> ent_fn;       // per entity: first face-normal entry, -1 without a table
    std::vector<float4> fn_tab;    // world-space unit face normals (surface_element)
    std::vector<int> ent_enc; // per entity: enclosing index or -1
    std::vector<int2> enc_tab; // per enclosing index: entity, TLAS leaf slot
    std::vector<float4> enc_box; // per enclosing index: world box lo, hi
    int tlas_root = -1;
    int tlas_depth = 0;
    if (desc->num_entities > 0) {
        const igx::BvhBuildResult& br = tlas_br;
        int node_off = append_nodes(br, 0, tlas_depth);
        tlas_root = br.root_is_leaf ? br.root_leaf_ref : node_off; // single entity: start at its leaf
        for (uint32_t slot = 0; slot < br.prim_order.size(); ++slot) {
            uint32_t e = br.prim_order[slot];
            const igx_entity& en = desc->entities[e];
            const ShapeDev& sd = sdev[en.shape];
            for (int r = 0; r < 3; ++r)
                inst.push_back(make_float4(en.to_local[r * 4 + 0], en.to_local[r * 4 + 1], en.to_local[r * 4 + 2], en.to_local[r * 4 + 3]));
            static const float kIdentity[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
            const float* m = en.to_local;
            const bool linear_identity = m[0] == 1 && m[1] == 0 && m[2] == 0 && m[4] == 0 && m[5] == 1 && m[6] == 0 &&
                                         m[8] == 0 && m[9] == 0 && m[10] == 1 && std::isfinite(m[3]) &&
                                         std::isfinite(m[7]) && std::isfinite(m[11]);
            const bool identity = sd.type == 0 && std::equal(m, m + 12, kIdentity);
            const bool translate = sd.type == 0 && !identity && linear_identity;
            const uint32_t iflags = (en.flags & ~(INST_IDENTITY | INST_TRANSLATE)) | (identity ? INST_IDENTITY : 0u) |
                                    (translate ? INST_TRANSLATE : 0u);
            int4 info = make_int4((int)e, sd.type, sd.type == 1 ? sd.idx_off_or_sphere : sd.root, (int)iflags);
            float4 fi;
            std::memcpy(&fi, &info, 16);
            inst.push_back(fi);
        }
        // enclosing entities (trace_enclosed): a closed mesh of a non-thin
        // dielectric whose world box keeps a margin from every other entity's
        // box, at most MAX_ENCLOSING of them (ent_enc: index, enc_tab: entity and TLAS leaf slot)
        ent_enc.assign(desc->num_entities, -1);
        if (dev->enclosing_opt && desc->num_entities <= 4096) {
            float slo[3], shi[3];
            for (int a = 0; a < 3; ++a) { slo[a] = desc->scene_bbox_min[a]; shi[a] = desc->scene_bbox_max[a]; }
            const float margin = 1e-4f * std::max({shi[0] - slo[0], shi[1] - slo[1], shi[2] - slo[2], 1e-6f});
            std::vector<int> closed(desc->num_shapes, -1);
            for (uint32_t slot = 0; slot < br.prim_order.size(); ++slot) {
                const uint32_t e = br.prim_order[slot];
                const igx_entity& en = desc->entities[e];
                const igx_shape& sh = desc->shapes[en.shape];
                const igx_material& mat = desc->materials[en.material];
                if (sh.type != IGX_SHAPE_TRIMESH || mat.bsdf_type != IGX_BSDF_DIELECTRIC || mat.thin) continue;
                if (closed[en.shape] < 0) closed[en.shape] = closed_mesh(desc->meshes[sh.mesh]) ? 1 : 0;
                if (!closed[en.shape]) continue;
                bool apart = true;
                for (uint32_t o = 0; o < desc->num_entities && apart; ++o) {
                    if (o == e) continue;
                    const igx_entity& q = desc->entities[o];
                    bool overlap = true;
                    for (int a = 0; a < 3; ++a)
                        overlap = overlap && q.bbox_min[a] <= en.bbox_max[a] + margin && en.bbox_min[a] <= q.bbox_max[a] + margin;
                    apart = !overlap;
                }
                static_assert(MAX_ENCLOSING <= MAX_ENC_BOXES, "enclosing boxes are staged in LDS (stage_enc_boxes)");
                if (apart && (int)enc_tab.size() < MAX_ENCLOSING) {
                    ent_enc[e] = (int)enc_tab.size();
                    enc_tab.push_back(make_int2((int)e, (int)slot));
                    enc_box.push_back(make_float4(en.bbox_min[0], en.bbox_min[1], en.bbox_min[2], 0));
                    enc_box.push_back(make_float4(en.bbox_max[0], en.bbox_max[1], en.bbox_max[2], 0));
                }
            }
        }
        for (uint32_t e = 0; e < desc->num_entities; ++e) {
            const igx_entity& en = desc->entities[e];
            const ShapeDev& sd = sdev[en.shape];
            for (int r = 0; r < 3; ++r)
                ent.push_back(make_float4(en.to_global[r * 4 + 0], en.to_global[r * 4 + 1], en.to_global[r * 4 + 2], en.to_global[r * 4 + 3]));
            for (int r = 0; r < 3; ++r) ent.push_back(make_float4(en.normal[r * 3 + 0], en.normal[r * 3 + 1], en.normal[r * 3 + 2], 0));
            int4 info = make_int4(sd.type, en.material, sd.vtx_off, sd.idx_off_or_sphere);
            float4 fi;
            std::memcpy(&fi, &info, 16);
            ent.push_back(fi);
        }
        // world-space unit face normals of every (mesh entity, face) when the
        // scene has few face instances: surface_element then skips three vertex
        // loads and transforms per hit.  make_triangle (core/triangle.art:11-26)
        // on the entity's to_global rows, in float, same operation order.
        size_t face_instances = 0;
        for (uint32_t e = 0; e < desc->num_entities; ++e) {
            const igx_shape& sh = desc->shapes[desc->entities[e].shape];
            if (sh.type == IGX_SHAPE_TRIMESH && sh.mesh >= 0) face_instances += desc->meshes[sh.mesh].num_faces;
        }
        if (dev->face_normals_opt && face_instances > 0 && face_instances <= FACE_NORMAL_TABLE_MAX) {
            ent_fn.assign(desc->num_entities, -1);
            fn_tab.reserve(face_instances);
            for (uint32_t e = 0; e < desc->num_entities; ++e) {
                const igx_entity& en = desc->entities[e];
                const igx_shape& sh = desc->shapes[en.shape];
                if (sh.type != IGX_SHAPE_TRIMESH || sh.mesh < 0) continue;
                const igx_mesh& m = desc->meshes[sh.mesh];
                ent_fn[e] = (int)fn_tab.size();
                const float* T = en.to_global;
                auto xf = [&](uint32_t v, float out[3]) {
                    const float* p = m.vertices + 3 * v;
                    for (int r = 0; r < 3; ++r) {
                        float acc = T[r * 4 + 0] * p[0];
                        acc = acc + T[r * 4 + 1] * p[1];
                        acc = acc + T[r * 4 + 2] * p[2];
                        out[r] = acc + T[r * 4 + 3];
                    }
                };
                for (uint32_t f = 0; f < m.num_faces; ++f) {
                    float v0[3], v1[3], v2[3];
                    xf(m.indices[3 * f], v0);
                    xf(m.indices[3 * f + 1], v1);
                    xf(m.indices[3 * f + 2], v2);
                    const float e1[3] = {v1[0] - v0[0], v1[1] - v0[1], v1[2] - v0[2]};
                    const float e2[3] = {v2[0] - v0[0], v2[1] - v0[1], v2[2] - v0[2]};
                    const float n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
                    float nn2 = n[0] * n[0];
                    nn2 = nn2 + n[1] * n[1];
                    nn2 = nn2 + n[2] * n[2];
                    const float inv = 1 / std::sqrt(nn2);
                    fn_tab.push_back(make_float4(n[0] * inv, n[1] * inv, n[2] * inv, 0));
                }
            }
        }
        // the entity's face-normal offset in row 3 .w of its record, read
        // with the normal matrix by surface_element's fsh path (-1: none)
        for (uint32_t e = 0; e < desc->num_entities; ++e) {
            const int off = ent_fn.empty() ? -1 : ent_fn[e];
            std::memcpy(&ent[ENT_STRIDE * e + 3].w, &off, 4);
        }
    }

    // ---- materials and lights (infinite lights first) --------------------
    std::vector<int> light_remap(desc->num_lights, -1);
    std::vector<DevLight> lights;
    for (int pass = 0; pass < 2; ++pass)
        for (uint32_t l = 0; l < desc->num_lights; ++l) {
            const igx_light& L = desc->lights[l];
            bool infinite = L.type == IGX_LIGHT_ENV || L.type == IGX_LIGHT_DIRECTIONAL || L.type == IGX_LIGHT_SUN;
            if ((pass == 0) != infinite) continue;
            DevLight d{};
            d.type = L.type;
            d.infinite = infinite ? 1 : 0;
            d.delta = (L.type == IGX_LIGHT_POINT || L.type == IGX_LIGHT_SPOT || L.type == IGX_LIGHT_DIRECTIONAL ||
                       L.type == IGX_LIGHT_SUN) ? 1 : 0;
            for (int i = 0; i < 3; ++i) d.radiance[i] = L.radiance[i];
            if (L.type == IGX_LIGHT_PLANE) {
                // make_plane_area_emitter constants (light/area.art:107-115)
                float xa[3] = {L.x_axis[0], L.x_axis[1], L.x_axis[2]};
                float ya[3] = {L.y_axis[0], L.y_axis[1], L.y_axis[2]};
                float width = std::sqrt(xa[0] * xa[0] + xa[1] * xa[1] + xa[2] * xa[2]);
                float height = std::sqrt(ya[0] * ya[0] + ya[1] * ya[1] + ya[2] * ya[2]);
                float iw = 1 / width, ih = 1 / height;
                for (int i = 0; i < 3; ++i) {
                    d.origin[i] = L.origin[i];
                    d.ex[i] = xa[i] * iw;
                    d.ey[i] = ya[i] * ih;
                    d.normal[i] = L.normal[i];
                }
                d.origin[3] = width;
                d.ex[3] = height;
                d.ey[3] = 1 / L.area;
                d.normal[3] = L.area;
            } else if (L.type == IGX_LIGHT_POINT) {
                for (int i = 0; i < 3; ++i) d.origin[i] = L.origin[i];
            } else if (L.type == IGX_LIGHT_SPOT) {
                for (int i = 0; i < 3; ++i) { d.origin[i] = L.origin[i]; d.normal[i] = L.normal[i]; }
                float cc = std::cos(L.cutoff), cf = std::cos(L.falloff);
                d.spot[0] = cc;
                d.spot[1] = cf;
                d.spot[2] = cf - cc;
            } else if (L.type == IGX_LIGHT_DIRECTIONAL) {
                for (int i = 0; i < 3; ++i) d.normal[i] = L.normal[i];
            } else if (L.type == IGX_LIGHT_SUN) {
                // make_sun_light constants (light/sun.art:4-8)
                for (int i = 0; i < 3; ++i) d.normal[i] = L.normal[i];
                float c = L.cutoff;
                float r = std::sqrt(1 - c * c) / c; // sun_radius_from_cos_angle
                d.spot[0] = c;
                d.spot[1] = 3.14159265359f * r * r;
            } else if (L.type == IGX_LIGHT_SPHERE || L.type == IGX_LIGHT_MESH) {
                if (L.entity < 0 || (uint32_t)L.entity >= desc->num_entities)
                    return fail(dev, IGX_ERR_INVALID_ARGUMENT, "area light references an invalid entity");
                d.entity = L.entity;
                if (L.type == IGX_LIGHT_SPHERE) {
                    if (!(L.area > 0) || !(L.radius > 0))
                        return fail(dev, IGX_ERR_INVALID_ARGUMENT, "sphere light needs a positive radius and area");
                    for (int i = 0; i < 3; ++i) d.origin[i] = L.origin[i];
                    d.origin[3] = L.radius;
                    d.spot[0] = L.area;
                } else {
                    const igx_shape& sh = desc->shapes[desc->entities[L.entity].shape];
                    if (sh.type != IGX_SHAPE_TRIMESH || sh.mesh < 0 || desc->meshes[sh.mesh].num_faces == 0)
                        return fail(dev, IGX_ERR_INVALID_ARGUMENT, "mesh light needs a non-empty triangle entity");
                    d.spot[0] = (float)desc->meshes[sh.mesh].num_faces;
                }
            } else if (L.type != IGX_LIGHT_ENV) {
                return fail(dev, IGX_ERR_UNSUPPORTED, "unsupported light type");
            }
            light_remap[l] = (int)lights.size();
            lights.push_back(d);
        }
    int num_infinite = 0;
    for (auto& l : lights) num_infinite += l.infinite;
    // NEE selector tables over the finite lights, in device order (host/light_select.h)
    std::vector<igx_light> finite_lights;
    for (uint32_t l = 0; l < desc->num_lights; ++l)
        if (light_remap[l] >= num_infinite) finite_lights.push_back(desc->lights[l]);
    // (pass 1 above numbers the finite lights in desc order, so this is device order)
    const igx::LightSelectTables lsel = igx::build_light_select(desc->technique.light_selector, (int)lights.size(), finite_lights);
    std::vector<DevMaterial> mats(desc->num_materials);
    for (uint32_t i = 0; i < desc->num_materials; ++i) {
        const igx_material& m = desc->materials[i];
        DevMaterial d{};
        switch (m.bsdf_type) {
        case IGX_BSDF_DIFFUSE: d.type = MAT_DIFFUSE; break;
        case IGX_BSDF_DIELECTRIC: d.type = MAT_DIELECTRIC; break;
        case IGX_BSDF_CONDUCTOR: d.type = MAT_CONDUCTOR; break;
        case IGX_BSDF_PLASTIC: d.type = MAT_PLASTIC; break;
        case IGX_BSDF_PRINCIPLED: d.type = MAT_PRINCIPLED; break;
        default: return fail(dev, IGX_ERR_UNSUPPORTED, "unsupported bsdf type " + std::to_string(m.bsdf_type));
        }
        if (m.distribution < IGX_MICROFACET_DELTA || m.distribution > IGX_MICROFACET_BECKMANN)
            return fail(dev, IGX_ERR_INVALID_ARGUMENT, "invalid microfacet distribution");
        d.light = m.light >= 0 && (uint32_t)m.light < desc->num_lights ? light_remap[m.light] : -1;
        // check_if_delta_distribution (core/microfacet.art:272): alpha <= 1e-4 is a delta lobe
        const bool rough = m.distribution != IGX_MICROFACET_DELTA && m.alpha_u > 1e-4f && m.alpha_v > 1e-4f;
        d.dist = rough ? m.distribution : MF_DELTA;
        bool mirror = true; // make_conductor_bsdf: eta ~ black and k ~ white (bsdf/conductor.art:111-121)
        for (int c = 0; c < 3; ++c) {
            d.kd[c] = m.kd[c];
            d.ks[c] = m.ks[c];
            d.kt[c] = m.kt[c];
            d.eta[c] = m.eta[c];
            d.kappa[c] = m.kappa[c];
            mirror = mirror && std::fabs(m.eta[c]) <= 1e-4f && std::fabs(m.kappa[c] - 1.0f) <= 1e-4f;
        }
        d.mirror = mirror ? 1 : 0;
        if (m.bsdf_type == IGX_BSDF_DIELECTRIC) d.mirror = m.thin ? 1 : 0; // dielectric: thin flag
        d.kd[3] = m.bsdf_type == IGX_BSDF_DIFFUSE ? m.diffuse_alpha : 0.0f;
        d.ks[3] = m.ext_ior;
        d.kt[3] = m.int_ior;
        d.eta[3] = m.alpha_u;
        d.kappa[3] = m.alpha_v;
        if (m.texture == IGX_TEXTURE_CHECKER && m.bsdf_type == IGX_BSDF_DIFFUSE) {
            const int32_t kind = IGX_TEXTURE_CHECKER;
            std::memcpy(&d.pad[0], &kind, 4);
            d.pad[1] = m.tex_scale;
            for (int c = 0; c < 3; ++c) d.pad[2 + c] = m.tex_kd1[c];
        } else if (m.texture != IGX_TEXTURE_NONE) {
            return fail(dev, IGX_ERR_UNSUPPORTED, "texture " + std::to_string(m.texture) + " on this bsdf type");
        }
        if (m.bsdf_type == IGX_BSDF_PRINCIPLED) {
            // packing of the principled closure (igx_kernels.h, principled_of)
            DevMaterial q{};
            q.type = MAT_PRINCIPLED;
            q.light = d.light;
            q.dist = MF_VNDF_GGX;
            q.mirror = (m.thin ? 1 : 0) | (m.clearcoat_top_only ? 2 : 0);
            for (int c = 0; c < 3; ++c) q.kd[c] = m.kd[c];
            q.kd[3] = m.ior;
            q.ks[0] = m.diffuse_transmission;
            q.ks[1] = m.specular_transmission;
            q.ks[2] = m.specular_tint;
            q.ks[3] = m.alpha_u;
            q.kt[0] = m.alpha_v;
            q.kt[1] = m.flatness;
            q.kt[2] = m.metallic;
            q.kt[3] = m.sheen;
            q.eta[0] = m.sheen_tint;
            q.eta[1] = m.clearcoat;
            q.eta[2] = m.clearcoat_gloss;
            q.eta[3] = m.clearcoat_roughness;
            d = q;
        }
        mats[i] = d;
    }

    // hot nodes first: any prefix of the node array is a treelet (stage_treelet)
    order_hot_nodes(nodes, quantize ? 5 : width, inst, tlas_root, TREELET_FRONT);

    // ---- upload ----------------------------------------------------------
    SceneView sv{};
    igx_status st;
    if ((st = upload(dev, nodes, &sv.nodes)) || (st = upload(dev, tris, &sv.tris)) || (st = upload(dev, inst, &sv.inst)) ||
        (st = upload(dev, spheres, &sv.spheres)) || (st = upload(dev, ent, &sv.ent)) || (st = upload(dev, vtx, &sv.vtx)) ||
        (st = upload(dev, nrm, &sv.nrm)) || (st = upload(dev, idx, &sv.idx)) || (st = upload(dev, mats, &sv.mats)) ||
        (st = upload(dev, lights, &sv.lights)) || (st = upload(dev, lsel.cdf, &sv.sel_cdf)) ||
        (st = upload(dev, lsel.hierarchy, &sv.sel_tree)) || (st = upload(dev, ent_enc, &sv.ent_enc)) ||
        (st = upload(dev, enc_tab, &sv.enc)) || (st = upload(dev, enc_box, &sv.enc_box)) || (st = upload(dev, ent_fn, &sv.ent_fn)) ||
        (st = upload(dev, fn_tab, &sv.fn_tab)) || (st = upload(dev, uvs, &sv.uv)) || (st = upload(dev, fsh, &sv.fsh))) {
        free_scene(dev);
        return st;
    }
    if (fn_tab.empty()) sv.fn_tab = nullptr; // surface_element computes the normals
    if (fsh.empty()) sv.fsh = nullptr;       // ... reads the index and normal tables
    if (uvs.empty()) sv.uv = nullptr;
    sv.tlas_root = tlas_root;
    sv.num_nodes = (int)(nodes.size() / nf4);
    sv.node_f4 = nf4;
    dev->bvh_width = width;
    dev->quantized = quantize;
    dev->nf4 = nf4;
    sv.num_inst = (int)(inst.size() / 4);
    sv.num_enc = (int)enc_tab.size();
    sv.num_tris = (int)(tris.size() / 3);
    {
        size_t b = ((size_t)sv.num_nodes * nf4 + (size_t)sv.num_inst * 4 + (size_t)sv.num_tris * 3) * 16;
        const size_t bl = b; // LDS layout (stage_scene_lds): the same tables back to back
        dev->lds_scene_bytes = (int64_t)bl <= dev->lds_scene_max ? bl : 0;
        dev->table_bytes = b;
        dev->shading_bytes = ent.size() * sizeof(ent[0]) + vtx.size() * sizeof(vtx[0]) + nrm.size() * sizeof(nrm[0]) +
                             idx.size() * sizeof(idx[0]) + mats.size() * sizeof(DevMaterial) + lights.size() * sizeof(lights[0]) +
                             fn_tab.size() * sizeof(fn_tab[0]) + fsh.size() * sizeof(fsh[0]);
    }
    sv.num_lights = (int)lights.size();
    sv.num_infinite = num_infinite;
    sv.selector = lsel.selector;
    // bbox_radius(scene_bbox) * 1.01 (light/env.art:75; core/bbox.art:24)
    float dx = desc->scene_bbox_max[0] - desc->scene_bbox_min[0];
    float dy = desc->scene_bbox_max[1] - desc->scene_bbox_min[1];
    float dz = desc->scene_bbox_max[2] - desc->scene_bbox_min[2];
    sv.scene_radius = std::sqrt(dx * dx + dy * dy + dz * dz) / 2 * 1.01f;
    if (desc->technique.max_depth > 255) {
        free_scene(dev);
        return fail(dev, IGX_ERR_UNSUPPORTED, "max_depth above 255 is not supported (8-bit path depth)");
    }
    sv.max_depth = desc->technique.max_depth;
    sv.min_depth = desc->technique.min_depth;
    sv.nee = desc->technique.nee;
    sv.clamp = desc->technique.clamp;
    dev->cam_desc = desc->camera;
    dev->aov_on = desc->technique.aov_mis != 0;
    dev->sv = sv;
    // stack: TLAS pushes + BLAS pushes (the depth for BVH2) + marker + resume entry + exit sentinel
#ifndef IGX_STACK_SLACK
#define IGX_STACK_SLACK 0
#endif
    dev->scene_depth = tlas_depth + blas_depth + 3 + IGX_STACK_SLACK;
    if (dev->scene_depth > MAX_STACK) {
        free_scene(dev);
        return fail(dev, IGX_ERR_UNSUPPORTED, "BVH too deep for the traversal stack (" + std::to_string(dev->scene_depth) + " entries)");
    }
    // shading feature set (variant bit 2): beyond Lambert + dielectric and the
    // plane/env/point/spot/directional/sun lights
    dev->full_shading = dev->full_shading_opt;
    for (uint32_t i = 0; i < desc->num_materials; ++i) {
        const igx_material& m = desc->materials[i];
        if (m.bsdf_type == IGX_BSDF_CONDUCTOR || m.bsdf_type == IGX_BSDF_PLASTIC || m.bsdf_type == IGX_BSDF_PRINCIPLED ||
            (m.bsdf_type == IGX_BSDF_DIFFUSE && m.diffuse_alpha > 1.1920929e-7f))
            dev->full_shading = true;
    }
    for (uint32_t l = 0; l < desc->num_lights; ++l)
        if (desc->lights[l].type == IGX_LIGHT_SPHERE || desc->lights[l].type == IGX_LIGHT_MESH) dev->full_shading = true;
    if (textured) dev->full_shading = true; // textures are looked up by the full shading variant only
    if (dev->aov_on) dev->full_shading = true; // so are the MIS AOVs (add_aov)
    for (uint32_t e = 0; textured && e < desc->num_entities; ++e) {
        const igx_entity& en = desc->entities[e];
        if (desc->materials[en.material].texture != IGX_TEXTURE_NONE && desc->shapes[en.shape].type == IGX_SHAPE_SPHERE) {
            free_scene(dev);
            return fail(dev, IGX_ERR_UNSUPPORTED, "textured material on an analytic sphere (texture coordinates of spheres are not supported)");
        }
    }
    if ((st = configure_stack(dev)) != IGX_OK) {
        free_scene(dev);
        return st;
    }
    dev->has_scene = true;
    dev->tree_dirty = true;
    return IGX_OK;
}

// Concurrent chunks (option "concurrent_chunks", fused schedule with two
// stream slots).  The sequential schedule runs every chunk's bounces on the
// one main stream: chunk k + 1 starts only when chunk k's bounce loop has
// reached its tail threshold, so each chunk's last bounces -- a few hundred K
// long paths, a few hundred microseconds each at low occupancy -- run alone.
// Here slot k's chunk runs on its own stream (dev->stream / dev->stream2,
// spill columns spill_main / spill_main2), and one host thread advances both
// chunks' bounce loops as their lagged counts arrive (hipEventQuery, no
// blocking wait).  The next chunk starts once the running one is down to
// concurrent_start_pct % of its paths, so one chunk's late bounces share the
// GPU with the other's early ones.  The tail kernel runs on the chunk's own
// stream after its bounces; resolves (and framebuffer clears) go to the tail
// stream strictly in submission order, so the framebuffer sums every pixel's
// iterations in the sequential order: bit-identical images.
//
// Asynchronous rendering (option "async_render", on top of concurrent
// chunks): render and clear calls only queue their work for a per-handle
// worker thread that runs the same scheduler over consecutive calls, so the
// last chunk of frame k overlaps the first of frame k + 1 too (one chunk per
// frame on an 8-rank diamond share).  Every other call waits until the queue
// has drained (wait_idle).
struct ChunkPlan { // one render call's chunking (render_impl)
    FrameArgs fa{};
    DevCamera cam{};
    int iteration = 0, spi = 1, count = 1, width = 1;
    long long local_pixels = 0, chunk_pixels_max = 0;
    int iters_per_chunk = 1;
    size_t slot_cap = 0;
    int max_bounces = 1, ext_bpc = 1, sh_bpc = 1, fin_bpc = 1;
    bool pairs = false;
};
struct SchedItem {
    bool clear = false;
    std::shared_ptr<const ChunkPlan> plan;
    int it0 = 0;
    long long px0 = 0;
    bool last_of_plan = false;
    bool started = false;
    int slot = 0;
    FrameArgs fa{};
    long long n = 0;
    int tail = 0, chunk_pixels = 0, ext_grid = 0, sh_grid = 0, fin_grid = 0;
    bool fuse_gen = false;
    int b = 0, switch_b = -1;
    long long live = 0; // paths entering the last bounce whose count arrived
    bool loop_done = false, tail_queued = false;
    hipEvent_t fin_ev = nullptr;
};
struct ChunkScheduler {
    std::deque<SchedItem> items; // submission order
    bool empty() const { return items.empty(); }
    void add(const std::shared_ptr<const ChunkPlan>& plan) {
        const ChunkPlan& pl = *plan;
        const size_t first = items.size();
        for (int it0 = 0; it0 < pl.count; it0 += pl.iters_per_chunk)
            for (long long px0 = 0; px0 < pl.local_pixels; px0 += pl.chunk_pixels_max) {
                SchedItem s;
                s.plan = plan;
                s.it0 = it0;
                s.px0 = px0;
                items.push_back(s);
            }
        if (items.size() > first) items.back().last_of_plan = true;
    }
    void add_clear() {
        SchedItem s;
        s.clear = true;
        items.push_back(s);
    }
    igx_status step(igx_device* dev, bool& progress);
    // every chunk has started and is down to concurrent_start_pct % of its paths (or done)
    bool all_late(int pct) const {
        for (const SchedItem& r : items) {
            if (r.clear) continue;
            if (!r.started) return false;
            if (!r.loop_done && r.live * 100 > (long long)pct * r.n) return false;
        }
        return true;
    }
};
struct AsyncRender {
    std::thread th;
    std::mutex m;
    std::condition_variable cv, cv_idle;
    std::deque<std::pair<bool, std::shared_ptr<const ChunkPlan>>> jobs; // (clear, plan)
    bool stop = false, idle = true;
    bool late = true; // every chunk submitted has started and is in its late bounces (igx_wait_ready)
    // a step failed on the worker: everything queued was dropped, so the film
    // and the iteration count no longer agree.  The handle stays failed --
    // every call that waits for the queue returns `err` with `msg` as its last
    // error -- until igx_clear or igx_upload_scene (reset_async_failure)
    igx_status err = IGX_OK;
    std::string msg;
    ChunkScheduler sched; // the worker's
};

igx_status ChunkScheduler::step(igx_device* dev, bool& progress) {
    hipStream_t const main0 = dev->stream, tail0 = dev->tail_stream;
    int* const spill0 = dev->spill_main;
    int* const spill_tail0 = dev->spill_tail;
    hipStream_t const slot_stream[2] = {dev->stream, dev->stream2};
    int* const slot_spill[2] = {dev->spill_main, dev->spill_main2};
    const bool inst = dev->instrument;
    // the launch helpers read dev->stream, dev->tail_stream, dev->sv (camera,
    // spill columns): point them at slot k and the item's camera while its
    // work is queued
    auto use_slot = [&](const SchedItem& r) {
        dev->stream = dev->tail_stream = slot_stream[r.slot];
        dev->sv.spill = dev->spill_tail = slot_spill[r.slot];
        dev->sv.cam = r.plan->cam;
    };
    auto restore = [&]() {
        dev->stream = main0;
        dev->tail_stream = tail0;
        dev->sv.spill = spill0;
        dev->spill_tail = spill_tail0;
    };
    auto begin_timed = [&](Slot& S, int kind, int bounce, hipStream_t strm) {
        if (!dev->timing) return;
        TimedLaunch t{slot_event(S), slot_event(S), kind, bounce};
        (void)hipEventRecord(t.a, strm);
        S.timed.push_back(t);
    };
    auto end_timed = [&](Slot& S, hipStream_t strm) {
        if (!dev->timing) return;
        (void)hipEventRecord(S.timed.back().b, strm);
    };
#define IGX_CC(expr)                                                                                   \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) {                                                                        \
            restore();                                                                                 \
            return fail(dev, IGX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));         \
        }                                                                                              \
    } while (0)
    // start the next chunk once its slot's previous chunk has resolved and
    // every running chunk is in its late bounces (live paths at most
    // concurrent_start_pct % of its own): two chunks started together only
    // contend for the chip in their heavy early bounces
    SchedItem* nx = nullptr;
    bool late = true;
    for (SchedItem& r : items) {
        if (r.clear) continue;
        if (!r.started) {
            nx = &r;
            break;
        }
        if (!r.loop_done && r.live * 100 > (long long)dev->concurrent_start_pct * r.n) late = false;
    }
    if (nx && late) {
        const int k = dev->stream_slots == 1 ? 0 : dev->next_slot;
        Slot& S = dev->slots[k];
        bool busy = false;
        for (const SchedItem& r : items) busy = busy || (!r.clear && r.started && r.slot == k);
        if (!busy && S.pending) {
            const hipError_t q = hipEventQuery(S.done);
            if (q == hipErrorNotReady) busy = true;
            else IGX_CC(q);
        }
        if (!busy) {
            SchedItem& r = *nx;
            const ChunkPlan& pl = *r.plan;
            if (dev->fail_chunk_opt > 0 && --dev->fail_chunk_opt == 0) { // test hook (option "fail_chunk")
                restore();
                return fail(dev, IGX_ERR_HIP, "injected failure (option fail_chunk)");
            }
            igx_status st;
            if ((st = harvest(dev, S)) != IGX_OK || (st = ensure_slot(dev, S, pl.slot_cap, false, pl.fa.classify >= 4, dev->aov_on)) != IGX_OK) {
                restore();
                return st;
            }
            if (dev->stream_slots == 2) dev->next_slot ^= 1;
            r.started = true;
            r.slot = k;
            r.fa = pl.fa;
            // the slot keeps AOV buffers from an earlier aov_mis scene: only
            // a scene with the AOVs (and their films) writes them
            r.fa.aov_di = dev->aov_on && dev->aov_fb[0] ? S.aov_di : nullptr;
            r.fa.aov_nee = dev->aov_on && dev->aov_fb[1] ? S.aov_nee : nullptr;
            S.sh.aov_nee = r.fa.aov_nee;
            r.fa.iter = pl.iteration + r.it0;
            r.fa.chunk_iters = std::min(pl.iters_per_chunk, pl.count - r.it0);
            r.chunk_pixels = (int)std::min<long long>(pl.chunk_pixels_max, pl.local_pixels - r.px0);
            r.fa.chunk_pixel0 = (int)r.px0;
            r.fa.chunk_pixels = r.chunk_pixels;
            r.n = (long long)r.chunk_pixels * pl.spi * r.fa.chunk_iters;
            r.live = r.n;
            // tail threshold: as the sequential schedule (render_impl)
            const long long fin_lanes = (long long)pl.fin_bpc * dev->num_cus * BLOCK / (pl.pairs ? 2 : 1);
            const int64_t topt = r.last_of_plan && dev->tail_last_opt >= 0 ? dev->tail_last_opt : dev->tail_opt;
            r.tail = topt >= 0 ? (int)std::min<int64_t>(topt, 1 << 30) : (int)std::max<long long>(32768, std::min(r.n / 64, fin_lanes));
            S.tail = r.tail;
            S.camera = valid_pixels_in_chunk(r.fa) * pl.spi * r.fa.chunk_iters;
            S.n0 = r.n;
            S.split = false;
            S.bounce_ev.clear();
            S.launched = 0;
            r.ext_grid = grid_for(dev, r.n, pl.ext_bpc);
            r.sh_grid = grid_for(dev, r.n, pl.sh_bpc);
            r.fin_grid = grid_for(dev, std::min<long long>(r.n, r.tail) * (pl.pairs ? 2 : 1), pl.fin_bpc);
            r.fuse_gen = dev->fuse_generate && r.n > r.tail;
            use_slot(r);
            IGX_CC(hipMemsetAsync(S.ctr, 0, (size_t)(2 * pl.max_bounces + 4) * CROW * sizeof(int), dev->stream));
            if (dev->dynamic_opt)
                IGX_CC(hipMemsetAsync(S.ctr + (size_t)WORK_ROW0 * CROW, 0, (size_t)4 * pl.max_bounces * CROW * sizeof(int), dev->stream));
            if (!r.fuse_gen) {
                begin_timed(S, 2, -1, dev->stream);
                hipLaunchKernelGGL(k_generate, dim3(grid_for(dev, r.n, 8)), dim3(BLOCK), 0, dev->stream, r.fa, dev->sv, S.pa, S.L, S.ctr);
                end_timed(S, dev->stream);
                IGX_CC(hipGetLastError());
            }
            restore();
            if (r.n <= r.tail) { // the whole chunk is one tail pass
                r.switch_b = 0;
                r.loop_done = true;
            }
            progress = true;
        }
    }
    // advance every chunk's bounce loop as far as its lagged counts allow
    for (SchedItem& r : items) {
        if (r.clear || !r.started || r.tail_queued) continue;
        Slot& S = dev->slots[r.slot];
        const ChunkPlan& pl = *r.plan;
        const int max_bounces = pl.max_bounces;
        int* const cnt = S.ctr;
        auto row = [&](int rr) { return cnt + (size_t)rr * CROW; };
        use_slot(r);
        while (!r.loop_done) {
            if (r.b < max_bounces) {
                if (r.b >= 2) {
                    const hipError_t q = hipEventQuery(S.bounce_ev[r.b - 2]);
                    if (q == hipErrorNotReady) break;
                    IGX_CC(q);
                    r.live = row_total(S, 2 * (r.b - 1));
                    if (r.live <= r.tail) {
                        r.switch_b = r.b - 1;
                        r.loop_done = true;
                        break;
                    }
                }
                const int b = r.b;
                PathBuf in = (b & 1) ? S.pb : S.pa, out = (b & 1) ? S.pa : S.pb;
                KernelCounters kc{row(2 * b), row(2 * (b + 1)), row(2 * b + 1), dev->dstats, row(WORK_ROW0 + 4 * b)};
                begin_timed(S, 0, b, dev->stream);
                FrameArgs fb = r.fa;
                fb.gen_n = r.fuse_gen && b == 0 ? (int)r.n : 0;
                // grids sized to the paths known to remain (r.live: the count
                // entering bounce b - 1, an upper bound for bounce b's paths and
                // shadow rays): late bounces launch few waves, not a full chip
                // of waves that find no group (IGX_LIVE_GRID)
                const long long bound = IGX_LIVE_GRID && b >= 2 ? r.live : r.n;
                const int ext_grid = IGX_LIVE_GRID ? grid_for(dev, bound, pl.ext_bpc) : r.ext_grid;
                const int sh_grid = IGX_LIVE_GRID ? grid_for(dev, bound, pl.sh_bpc) : r.sh_grid;
                if (inst) launch_extend<true>(dev, S, ext_grid, fb, in, out, kc, r.tail);
                else launch_extend<false>(dev, S, ext_grid, fb, in, out, kc, r.tail);
                end_timed(S, dev->stream);
                begin_timed(S, 1, b, dev->stream);
                int* const sh_work =
                    (dev->dynamic_opt & (use_refill(dev) ? DYN_REFILL_SHADOW : DYN_SHADOW)) ? row(WORK_ROW0 + 4 * b + 2) : nullptr;
                if (inst) launch_shadow<true>(dev, S, sh_grid, row(2 * b + 1), sh_work, dev->stream);
                else launch_shadow<false>(dev, S, sh_grid, row(2 * b + 1), sh_work, dev->stream);
                end_timed(S, dev->stream);
                IGX_CC(hipGetLastError());
                IGX_CC(hipMemcpyAsync(S.pinned + (size_t)(2 * b + 1) * CROW, row(2 * b + 1), 2 * CROW * sizeof(int),
                                      hipMemcpyDeviceToHost, dev->stream));
                hipEvent_t e = slot_event(S);
                IGX_CC(hipEventRecord(e, dev->stream));
                S.bounce_ev.push_back(e);
                ++S.launched;
                ++r.b;
                progress = true;
            } else {
                // every bounce queued: the counts are known once the last one completed
                const hipError_t q = hipEventQuery(S.bounce_ev.back());
                if (q == hipErrorNotReady) break;
                IGX_CC(q);
                r.switch_b = max_bounces;
                for (int b = 1; b <= max_bounces; ++b)
                    if (row_total(S, 2 * b) <= r.tail) {
                        r.switch_b = b;
                        break;
                    }
                r.loop_done = true;
            }
        }
        if (r.loop_done && !r.tail_queued) {
            S.switch_bounce = r.switch_b;
            if (r.switch_b < MAX_BOUNCES) {
                PathBuf in = (r.switch_b & 1) ? S.pb : S.pa;
                begin_timed(S, 4, r.switch_b, dev->stream);
                if (inst) launch_finish<true>(dev, S, r.fin_grid, r.fa, in, row(2 * r.switch_b), r.tail);
                else launch_finish<false>(dev, S, r.fin_grid, r.fa, in, row(2 * r.switch_b), r.tail);
                end_timed(S, dev->stream);
                IGX_CC(hipGetLastError());
            }
            r.fin_ev = slot_event(S);
            IGX_CC(hipEventRecord(r.fin_ev, dev->stream));
            r.tail_queued = true;
            progress = true;
        }
        restore();
    }
    // resolves and framebuffer clears strictly in submission order on the tail stream
    while (!items.empty() && (items.front().clear || items.front().tail_queued)) {
        SchedItem& r = items.front();
        if (r.clear) {
            IGX_CC(hipMemsetAsync(dev->fb, 0, dev->fb_count * sizeof(float), tail0));
            for (float* a : dev->aov_fb)
                if (a) IGX_CC(hipMemsetAsync(a, 0, dev->fb_count * sizeof(float), tail0));
        } else {
            Slot& S = dev->slots[r.slot];
            IGX_CC(hipStreamWaitEvent(tail0, r.fin_ev, 0));
            begin_timed(S, 3, -1, tail0);
            hipLaunchKernelGGL(k_resolve, dim3((r.chunk_pixels + 63) / 64), dim3(64 * RES_G), 0, tail0, r.fa, S.L, dev->fb, r.plan->width);
            if (r.fa.aov_di) // the MIS AOVs, resolved like the film
                for (int k = 0; k < 2; ++k)
                    hipLaunchKernelGGL(k_resolve, dim3((r.chunk_pixels + 63) / 64), dim3(64 * RES_G), 0, tail0, r.fa,
                                       k ? S.aov_nee : S.aov_di, dev->aov_fb[k], r.plan->width);
            end_timed(S, tail0);
            IGX_CC(hipGetLastError());
            IGX_CC(hipEventRecord(S.done, tail0));
            S.pending = true;
        }
        items.pop_front();
        progress = true;
    }
#undef IGX_CC
    restore();
    return IGX_OK;
}

// The scheduler's host thread between steps that made no progress (every
// chunk waits on a lagged count): a few yields, then sleeps of host_wait_us,
// so a busy handle does not hold a CPU core at 100 % polling events (ADVICE
// r4).  The lag of two bounces keeps the GPU fed across one sleep.
// host_wait_us 0: yield only (the round-4 behaviour).
struct Backoff {
    int idle = 0;
    void wait(const igx_device* dev) {
        if (dev->host_wait_us <= 0 || idle < 8) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(dev->host_wait_us));
        ++idle;
    }
    void reset() { idle = 0; }
};

// Runs the scheduler in the calling thread until everything queued is resolved.
static igx_status run_scheduler(igx_device* dev, ChunkScheduler& sched) {
    Backoff bo;
    while (!sched.empty()) {
        bool progress = false;
        igx_status st = sched.step(dev, progress);
        if (st != IGX_OK) {
            sched.items.clear();
            return st;
        }
        if (progress) bo.reset();
        else bo.wait(dev);
    }
    return IGX_OK;
}

static void async_worker(igx_device* dev) {
    AsyncRender& a = *dev->async;
    (void)hipSetDevice(dev->hip_device);
    std::string worker_msg;
    t_error_sink = &worker_msg; // fail() on this thread: the handle's last_error is the host thread's
    Backoff bo;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(a.m);
            while (!a.jobs.empty()) {
                if (a.jobs.front().first) a.sched.add_clear();
                else a.sched.add(a.jobs.front().second);
                a.jobs.pop_front();
            }
            if (a.sched.empty()) {
                a.idle = true;
                a.cv_idle.notify_all();
                if (a.stop) return;
                a.cv.wait(lk, [&] { return a.stop || !a.jobs.empty(); });
                if (a.jobs.empty() && a.stop) return;
                a.idle = false;
                continue;
            }
        }
        bool progress = false;
        igx_status st = a.sched.step(dev, progress);
        if (st != IGX_OK) {
            // drop everything queued (a chunk may be half rendered into the
            // film) and mark the handle failed until a clear or upload
            std::lock_guard<std::mutex> lk(a.m);
            a.sched.items.clear();
            a.jobs.clear();
            if (a.err == IGX_OK) {
                a.err = st;
                a.msg = "async render: " + worker_msg;
            }
            continue;
        }
        if (progress) {
            bo.reset();
            const bool late = a.sched.all_late(dev->concurrent_start_pct);
            std::lock_guard<std::mutex> lk(a.m);
            a.late = late && a.jobs.empty();
            if (a.late) a.cv_idle.notify_all();
        } else {
            bo.wait(dev);
        }
    }
}

// Waits until every chunk submitted has started and is in its late bounces
// (down to concurrent_start_pct % of its paths), the point from which work on
// another handle of the same GPU overlaps it without slowing its heavy
// bounces (bench.py: frame k + 1 on the other handle); or until the queue has
// drained.  No-op without a worker.
igx_status wait_ready(igx_device* dev) {
    if (!dev->async) return IGX_OK;
    AsyncRender& a = *dev->async;
    std::unique_lock<std::mutex> lk(a.m);
    a.cv_idle.wait(lk, [&] { return (a.idle && a.jobs.empty()) || (a.late && a.jobs.empty()); });
    if (a.err != IGX_OK) dev->last_error = a.msg;
    return a.err;
}

// Waits until the worker has queued (on the GPU) everything submitted and
// returns its error, if it failed: the failure stays until igx_clear or
// igx_upload_scene.  No-op without a worker.
igx_status wait_idle(igx_device* dev) {
    if (!dev->async) return IGX_OK;
    AsyncRender& a = *dev->async;
    std::unique_lock<std::mutex> lk(a.m);
    a.cv_idle.wait(lk, [&] { return a.idle && a.jobs.empty(); });
    if (a.err != IGX_OK) dev->last_error = a.msg;
    return a.err;
}

// igx_clear / igx_upload_scene on a failed handle: wait until the worker is
// idle and lift the failure (the caller then resets the film or the scene).
// Returns whether the handle had failed.
bool reset_async_failure(igx_device* dev) {
    if (!dev->async) return false;
    AsyncRender& a = *dev->async;
    std::unique_lock<std::mutex> lk(a.m);
    a.cv_idle.wait(lk, [&] { return a.idle && a.jobs.empty(); });
    const bool failed = a.err != IGX_OK;
    a.err = IGX_OK;
    a.msg.clear();
    return failed;
}

void stop_async(igx_device* dev) {
    if (!dev->async) return;
    {
        std::lock_guard<std::mutex> lk(dev->async->m);
        dev->async->stop = true;
    }
    dev->async->cv.notify_all();
    if (dev->async->th.joinable()) dev->async->th.join();
    delete dev->async;
    dev->async = nullptr;
}

static void submit_async(igx_device* dev, bool clear, std::shared_ptr<const ChunkPlan> plan) {
    if (!dev->async) {
        dev->async = new AsyncRender();
        dev->async->th = std::thread(async_worker, dev);
    }
    {
        std::lock_guard<std::mutex> lk(dev->async->m);
        dev->async->jobs.push_back({clear, std::move(plan)});
        dev->async->idle = false;
        dev->async->late = false;
    }
    dev->async->cv.notify_all();
}

// Render `count` consecutive iterations (p->iteration, p->iteration + 1, ...).
// Small iterations are batched: one chunk then holds several iterations'
// paths (up to the path capacity), so a shard with few pixels (multi-GPU
// tiles) still fills the device; the film is bit-identical to `count`
// single-iteration calls.
static igx_status render_impl(igx_device* dev, const igx_render_params* p, int count) {
    if (!dev || !p || count < 1) return IGX_ERR_INVALID_ARGUMENT;
    if (!dev->has_scene) return fail(dev, IGX_ERR_NO_SCENE, "no scene uploaded");
    if (p->spi < 1) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "spi must be >= 1");
    auto t_start = std::chrono::steady_clock::now();
    HIPCHK(hipSetDevice(dev->hip_device));
    const bool list_mode = p->num_rays > 0;
    int width = list_mode ? p->num_rays : p->width;
    int height = list_mode ? 1 : p->height;
    if (width < 1 || height < 1) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "film size must be positive");
    if (p->tile_size > 0 && (p->tile_stride < 1 || p->tile_offset < 0 || p->tile_offset >= p->tile_stride))
        return fail(dev, IGX_ERR_INVALID_ARGUMENT, "invalid tile sharding parameters");
    if (list_mode && p->tile_size > 0) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "ray-list mode cannot be tile-sharded");
    // schedule: concurrent chunks on the fused schedule with two slots, queued
    // for the handle's worker thread when async_render is on; anything else
    // runs here once the worker has drained
    const bool split = use_split(dev);
    const bool conc = !list_mode && !split && dev->concurrent_opt;
    const bool async = conc && dev->async_opt;
    if (!async) {
        igx_status w = wait_idle(dev);
        if (w != IGX_OK) return w;
    } else if (dev->async) { // a failed handle takes no more work until a clear or upload
        std::lock_guard<std::mutex> lk(dev->async->m);
        if (dev->async->err != IGX_OK) {
            dev->last_error = dev->async->msg;
            return dev->async->err;
        }
    }

    // framebuffer (resize clears, as Device::resize)
    size_t fbc = (size_t)width * height * 3;
    const bool want_aov = dev->aov_on && !list_mode;
    if (dev->fb_w != width || dev->fb_h != height || !dev->fb || want_aov != (dev->aov_fb[0] != nullptr)) {
        igx_status dst = drain(dev);
        if (dst != IGX_OK) return dst;
        if (dev->fb) HIPCHK(hipFree(dev->fb));
        dev->fb = nullptr;
        for (float*& a : dev->aov_fb) {
            if (a) HIPCHK(hipFree(a));
            a = nullptr;
        }
        HIPCHK(hipMalloc((void**)&dev->fb, fbc * sizeof(float)));
        HIPCHK(hipMemsetAsync(dev->fb, 0, fbc * sizeof(float), dev->tail_stream));
        if (want_aov)
            for (float*& a : dev->aov_fb) {
                HIPCHK(hipMalloc((void**)&a, fbc * sizeof(float)));
                HIPCHK(hipMemsetAsync(a, 0, fbc * sizeof(float), dev->tail_stream));
            }
        dev->fb_w = width;
        dev->fb_h = height;
        dev->fb_count = fbc;
        dev->iteration_count = 0;
    }
    const DevCamera cam = make_camera(dev, width, height);
    if (!async) dev->sv.cam = cam; // the worker sets each chunk's camera itself

    FrameArgs fa{};
    fa.width = width;
    fa.height = height;
    fa.spi = p->spi;
    fa.iter = p->iteration;
    fa.frame = p->frame;
    fa.seed = p->seed;
    fa.inv_spi = 1.0f / (float)p->spi;
    fa.classify = dev->classify_opt;
    fa.shadow_classes = dev->shadow_classes_opt;
    fa.dynamic = dev->dynamic_opt & DYN_EXTEND;
    fa.reverse = fa.dynamic ? (dev->group_order_opt < 0 ? GROUP_ORDER_AUTO : dev->group_order_opt) : 0;
    fa.probe_sample = dev->probe_sample_opt > 0 && dev->probe_sample_opt <= p->spi ? (int)dev->probe_sample_opt : 0;
    long long local_pixels;
    if (list_mode) {
        // the previous ray list may still be read by a queued tail kernel
        igx_status dst = drain(dev);
        if (dst != IGX_OK) return dst;
        size_t need = (size_t)p->num_rays * 8;
        if (dev->ray_list_cap < need) {
            if (dev->ray_list) HIPCHK(hipFree(dev->ray_list));
            HIPCHK(hipMalloc((void**)&dev->ray_list, need * sizeof(float)));
            dev->ray_list_cap = need;
        }
        HIPCHK(hipMemcpy(dev->ray_list, p->rays, need * sizeof(float), hipMemcpyHostToDevice));
        fa.num_rays = p->num_rays;
        fa.rays = dev->ray_list;
        local_pixels = p->num_rays;
    } else if (p->tile_size > 0) {
        fa.tile_size = p->tile_size;
        fa.tile_offset = p->tile_offset;
        fa.tile_stride = p->tile_stride;
        fa.tiles_x = (width + p->tile_size - 1) / p->tile_size;
        int tiles_y = (height + p->tile_size - 1) / p->tile_size;
        int tiles = fa.tiles_x * tiles_y;
        int mine = tiles > p->tile_offset ? (tiles - p->tile_offset + p->tile_stride - 1) / p->tile_stride : 0;
        local_pixels = (long long)mine * p->tile_size * p->tile_size;
    } else {
        local_pixels = (long long)width * height;
    }
    // capacity: whole iteration resident when it fits (<= 16M paths), pixel aligned
    long long total_paths = local_pixels * p->spi;
    if (total_paths == 0) {
        dev->iteration_count += count;
        return IGX_OK;
    }
    // default chunk of a multi-iteration render: the largest power of two
    // whose stream slots take at most 30 % of the device memory (MI355X: 128 M
    // paths; two slots of 22.5 GB, 36.9 GB with three path classes).  Fewer,
    // larger chunks leave fewer tails that overlap nothing: diamond frame 193
    // -> 179 ms, S-deep 4096^2 865 -> 823 ms from 32 M to 128 M paths
    // (tools/sweep_frame.py).  Per path and slot: two path buffers (56 B a
    // record; twice that with the class-C region), shadow ray 48 B, hit
    // record 20 B (split schedule), radiance 16 B, and the two MIS AOV slots
    // (32 B) of an aov_mis scene.
    if (split && fa.classify >= 4) fa.classify = 3; // hit records have no class-C region
    const long long path_slot_bytes =
        2 * 56 * (fa.classify >= 4 ? 2 : 1) + 48 + (split ? 20 : 0) + 16 + (dev->aov_on && !list_mode ? 32 : 0);
    const long long slot_budget =
        dev->slot_budget_mb > 0 ? dev->slot_budget_mb * (1ll << 20) : (long long)((double)dev->mem_total * 0.3);
    long long auto_chunk_paths = 1ll << 24;
    while (auto_chunk_paths < MAX_CHUNK_PATHS && dev->stream_slots * (2 * auto_chunk_paths) * path_slot_bytes <= slot_budget)
        auto_chunk_paths *= 2;
    if (dev->slot_budget_mb > 0) // an explicit budget also bounds the chunk below 16 M paths
        auto_chunk_paths = std::max<long long>(1ll << 20, std::min<long long>(auto_chunk_paths, slot_budget / (dev->stream_slots * path_slot_bytes)));
    long long cap = dev->capacity_opt > 0 ? dev->capacity_opt
                                          : (count > 1 ? auto_chunk_paths : std::min<long long>({total_paths, 1ll << 24, auto_chunk_paths}));
    cap = std::min<long long>(cap, MAX_CHUNK_PATHS);
    cap = std::max<long long>(p->spi, (cap / p->spi) * p->spi);
    const long long chunk_pixels_max = std::min<long long>(cap, total_paths) / p->spi;
    const int iters_per_chunk = total_paths <= cap ? (int)std::min<long long>(count, cap / total_paths) : 1;
    const size_t slot_cap = (size_t)(chunk_pixels_max * p->spi * iters_per_chunk);

    const int max_bounces = std::min(std::max(dev->sv.max_depth, 1), MAX_BOUNCES - 1);
    const bool inst = dev->instrument;
    const int sd = dev->variant;
    const size_t ldsb = dev->lds_scene_bytes;
    if (dev->tree_dirty) configure_treelet(dev);
    const int ext_bpc = inst ? extend_blocks_per_cu<true>(sd, ldsb, tree_bytes(dev, dev->tree_ext))
                             : extend_blocks_per_cu<false>(sd, ldsb, tree_bytes(dev, dev->tree_ext));
    const bool refill = use_refill(dev);
    const int tr_bpc = inst ? trace_blocks_per_cu<true>(sd, dev->lds_scene_bytes, refill)
                            : trace_blocks_per_cu<false>(sd, dev->lds_scene_bytes, refill);
    const bool full = variant_full(sd);
    const int shade_bpc = shade_blocks_per_cu(full);
    const int sh_bpc = inst ? shadow_blocks_per_cu<true>(sd, dev->lds_scene_bytes, refill, tree_bytes(dev, dev->tree_shadow))
                            : shadow_blocks_per_cu<false>(sd, dev->lds_scene_bytes, refill, tree_bytes(dev, dev->tree_shadow));
    const bool pairs = use_tail_pairs(dev);
    const int fin_bpc = inst ? finish_blocks_per_cu<true>(sd, ldsb, 0, pairs) : finish_blocks_per_cu<false>(sd, ldsb, 0, pairs);

    if (conc) {
        auto plan = std::make_shared<ChunkPlan>();
        plan->fa = fa;
        plan->cam = cam;
        plan->iteration = p->iteration;
        plan->spi = p->spi;
        plan->count = count;
        plan->width = width;
        plan->local_pixels = local_pixels;
        plan->chunk_pixels_max = chunk_pixels_max;
        plan->iters_per_chunk = iters_per_chunk;
        plan->slot_cap = slot_cap;
        plan->max_bounces = max_bounces;
        plan->ext_bpc = ext_bpc;
        plan->sh_bpc = sh_bpc;
        plan->fin_bpc = fin_bpc;
        plan->pairs = pairs;
        dev->iteration_count += count;
        dev->stats.iterations += count;
        if (async) {
            submit_async(dev, false, std::move(plan));
        } else {
            ChunkScheduler sched;
            sched.add(plan);
            igx_status st = run_scheduler(dev, sched);
            if (st != IGX_OK) return st;
        }
        dev->stats.ms_render += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
        return IGX_OK;
    }

    for (int it0 = 0; it0 < count; it0 += iters_per_chunk)
    for (long long px0 = 0; px0 < local_pixels; px0 += chunk_pixels_max) {
        fa.iter = p->iteration + it0;
        fa.chunk_iters = std::min(iters_per_chunk, count - it0);
        Slot& S = dev->slots[dev->stream_slots == 1 ? 0 : dev->next_slot];
        dev->next_slot ^= 1;
        igx_status st = harvest(dev, S); // waits for the chunk that used this slot two chunks ago (one, with one slot)
        if (st != IGX_OK) return st;
        if ((st = ensure_slot(dev, S, slot_cap, split, fa.classify >= 4, dev->aov_on && !list_mode)) != IGX_OK) return st;
        fa.aov_di = dev->aov_on && dev->aov_fb[0] && !list_mode ? S.aov_di : nullptr;
        fa.aov_nee = dev->aov_on && dev->aov_fb[1] && !list_mode ? S.aov_nee : nullptr;
        S.sh.aov_nee = fa.aov_nee;

        auto begin_timed = [&](int kind, int bounce, hipStream_t strm) {
            if (!dev->timing) return;
            TimedLaunch t{slot_event(S), slot_event(S), kind, bounce};
            (void)hipEventRecord(t.a, strm);
            S.timed.push_back(t);
        };
        auto end_timed = [&](hipStream_t strm) {
            if (!dev->timing) return;
            (void)hipEventRecord(S.timed.back().b, strm);
        };

        int chunk_pixels = (int)std::min<long long>(chunk_pixels_max, local_pixels - px0);
        fa.chunk_pixel0 = (int)px0;
        fa.chunk_pixels = chunk_pixels;
        long long n = (long long)chunk_pixels * p->spi * fa.chunk_iters;
        // tail threshold (auto): n / 64, but at most what one pass of k_finish
        // holds (one path per resident lane): beyond that the tail kernel's
        // lanes loop over several long paths each and it outlasts the
        // overlapping chunk (diamond 32M-path chunks: 500K -> 196K tail paths,
        // 204.6 -> 195.0 ms per frame, tools/sweep_frame.py)
        // paths one pass of the tail kernel holds (lane pairs: one path per two lanes)
        const long long fin_lanes = (long long)fin_bpc * dev->num_cus * BLOCK / (pairs ? 2 : 1);
        const bool last_chunk = it0 + iters_per_chunk >= count && px0 + chunk_pixels_max >= local_pixels;
        const int64_t topt = last_chunk && dev->tail_last_opt >= 0 ? dev->tail_last_opt : dev->tail_opt;
        int tail = topt >= 0 ? (int)std::min<int64_t>(topt, 1 << 30)
                                      : (int)std::max<long long>(32768, std::min(n / 64, fin_lanes));
        S.tail = tail;
        S.camera = valid_pixels_in_chunk(fa) * p->spi * fa.chunk_iters;
        int* cnt = S.ctr; // row 2b: paths entering bounce b, row 2b+1: shadow rays of bounce b
        auto row = [&](int r) { return cnt + (size_t)r * CROW; };
        HIPCHK(hipMemsetAsync(S.ctr, 0, (size_t)(2 * max_bounces + 4) * CROW * sizeof(int), dev->stream));
        if (dev->dynamic_opt)
            HIPCHK(hipMemsetAsync(S.ctr + (size_t)WORK_ROW0 * CROW, 0, (size_t)4 * max_bounces * CROW * sizeof(int), dev->stream));
        // camera paths: built by bounce 0 of the fused k_extend when the chunk
        // runs through it (saves the 72 B/path round trip of k_generate)
        const bool fuse_gen = dev->fuse_generate && !split && n > tail;
        if (!fuse_gen) {
            begin_timed(2, -1, dev->stream);
            hipLaunchKernelGGL(k_generate, dim3(grid_for(dev, n, 8)), dim3(BLOCK), 0, dev->stream, fa, dev->sv, S.pa, S.L, cnt);
            end_timed(dev->stream);
            HIPCHK(hipGetLastError());
        }
        S.n0 = n;
        S.split = split;
        const int fin_grid = grid_for(dev, std::min<long long>(n, tail) * (pairs ? 2 : 1), fin_bpc);
        // Wavefront bounces on the main stream.  The host learns counts two
        // bounces late (async copies, no per-bounce sync); the device gates
        // k_extend off once the count is <= tail, and the host then queues
        // k_finish for that bounce's buffer on the tail stream.
        S.bounce_ev.clear();
        int switch_b = -1;
        S.launched = 0;
        // split schedule: the shadow rays of bounce b run on the shadow stream,
        // overlapping the trace of bounce b + 1 (independent: both come from
        // shade(b)); shade(b + 1) waits for them, as both add to the radiance
        // slots, so the additions keep their order and the image is unchanged
        const bool overlap = split && dev->overlap_shadow_opt;
        hipStream_t sh_strm = overlap ? dev->shadow_stream : dev->stream;
        hipEvent_t sh_done = nullptr; // the last shadow launch on the shadow stream
        if (n <= tail) switch_b = 0;
        for (int b = 0; switch_b < 0 && b < max_bounces; ++b) {
            long long bound = n; // paths known to remain (see the concurrent schedule)
            if (b >= 2) {
                HIPCHK(hipEventSynchronize(S.bounce_ev[b - 2]));
                bound = row_total(S, 2 * (b - 1));
                if (bound <= tail) {
                    switch_b = b - 1;
                    break;
                }
            }
            if (!IGX_LIVE_GRID) bound = n;
            const int ext_grid = grid_for(dev, bound, ext_bpc), tr_grid = grid_for(dev, bound, tr_bpc);
            const int shade_grid = grid_for(dev, bound, shade_bpc), sh_grid = grid_for(dev, bound, sh_bpc);
            PathBuf in = (b & 1) ? S.pb : S.pa, out = (b & 1) ? S.pa : S.pb;
            KernelCounters kc{row(2 * b), row(2 * (b + 1)), row(2 * b + 1), dev->dstats, row(WORK_ROW0 + 4 * b)};
            if (split) {
                begin_timed(5, b, dev->stream);
                int* const tr_work = (dev->dynamic_opt & DYN_REFILL_TRACE) ? row(WORK_ROW0 + 4 * b) : nullptr;
                if (inst) launch_trace<true>(dev, S, tr_grid, fa, in, row(2 * b), tail, tr_work);
                else launch_trace<false>(dev, S, tr_grid, fa, in, row(2 * b), tail, tr_work);
                end_timed(dev->stream);
                if (sh_done) HIPCHK(hipStreamWaitEvent(dev->stream, sh_done, 0));
                begin_timed(0, b, dev->stream);
                launch_shade(dev, full, shade_grid, fa, in, S.hb, out, S.sh, S.L, kc, tail);
                end_timed(dev->stream);
            } else {
                begin_timed(0, b, dev->stream);
                FrameArgs fb = fa;
                fb.gen_n = fuse_gen && b == 0 ? (int)n : 0;
                if (inst) launch_extend<true>(dev, S, ext_grid, fb, in, out, kc, tail);
                else launch_extend<false>(dev, S, ext_grid, fb, in, out, kc, tail);
                end_timed(dev->stream);
            }
            if (overlap) {
                hipEvent_t shaded = slot_event(S);
                HIPCHK(hipEventRecord(shaded, dev->stream));
                HIPCHK(hipStreamWaitEvent(sh_strm, shaded, 0));
            }
            begin_timed(1, b, sh_strm);
            int* const sh_work =
                (dev->dynamic_opt & (use_refill(dev) ? DYN_REFILL_SHADOW : DYN_SHADOW)) ? row(WORK_ROW0 + 4 * b + 2) : nullptr;
            if (inst) launch_shadow<true>(dev, S, sh_grid, row(2 * b + 1), sh_work, sh_strm);
            else launch_shadow<false>(dev, S, sh_grid, row(2 * b + 1), sh_work, sh_strm);
            end_timed(sh_strm);
            if (overlap) {
                sh_done = slot_event(S);
                HIPCHK(hipEventRecord(sh_done, sh_strm));
            }
            HIPCHK(hipGetLastError());
            // shadow counts of bounce b and path counts entering bounce b+1 (adjacent rows)
            HIPCHK(hipMemcpyAsync(S.pinned + (size_t)(2 * b + 1) * CROW, row(2 * b + 1), 2 * CROW * sizeof(int), hipMemcpyDeviceToHost, dev->stream));
            hipEvent_t e = slot_event(S);
            (void)hipEventRecord(e, dev->stream);
            S.bounce_ev.push_back(e);
            ++S.launched;
        }
        if (switch_b < 0) {
            // max_bounces launched: drain the lagged counts and find the first bounce at/below tail
            HIPCHK(hipStreamSynchronize(dev->stream));
            switch_b = max_bounces;
            for (int b = 1; b <= max_bounces; ++b)
                if (row_total(S, 2 * b) <= tail) { switch_b = b; break; }
        }
        S.switch_bounce = switch_b;
        // tail + resolve on the tail stream, after the main stream (and the
        // shadow stream's last launch) reached this point
        if (sh_done) HIPCHK(hipStreamWaitEvent(dev->stream, sh_done, 0));
        hipEvent_t reach = slot_event(S);
        HIPCHK(hipEventRecord(reach, dev->stream));
        HIPCHK(hipStreamWaitEvent(dev->tail_stream, reach, 0));
        if (switch_b < MAX_BOUNCES) {
            PathBuf in = (switch_b & 1) ? S.pb : S.pa;
            begin_timed(4, switch_b, dev->tail_stream);
            if (inst) launch_finish<true>(dev, S, fin_grid, fa, in, row(2 * switch_b), tail);
            else launch_finish<false>(dev, S, fin_grid, fa, in, row(2 * switch_b), tail);
            end_timed(dev->tail_stream);
        }
        begin_timed(3, -1, dev->tail_stream);
        hipLaunchKernelGGL(k_resolve, dim3((chunk_pixels + 63) / 64), dim3(64 * RES_G), 0, dev->tail_stream, fa, S.L, dev->fb, width);
        if (fa.aov_di)
            for (int k = 0; k < 2; ++k)
                hipLaunchKernelGGL(k_resolve, dim3((chunk_pixels + 63) / 64), dim3(64 * RES_G), 0, dev->tail_stream, fa,
                                   k ? S.aov_nee : S.aov_di, dev->aov_fb[k], width);
        end_timed(dev->tail_stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(S.done, dev->tail_stream));
        S.pending = true;
    }
    dev->iteration_count += count;
    dev->stats.iterations += count;
    dev->stats.ms_render += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return IGX_OK;
}

extern "C" igx_status igx_set_camera(igx_device* dev, const igx_camera* camera) {
    if (!dev || !camera) return IGX_ERR_INVALID_ARGUMENT;
    // queued chunks read the camera from their kernel arguments: no drain needed
    dev->cam_desc = *camera;
    return IGX_OK;
}

extern "C" igx_status igx_render(igx_device* dev, const igx_render_params* p) { return render_impl(dev, p, 1); }

extern "C" igx_status igx_render_iterations(igx_device* dev, const igx_render_params* p, int32_t count) {
    if (count < 1) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "iteration count must be >= 1");
    return render_impl(dev, p, count);
}

extern "C" igx_status igx_get_framebuffer(igx_device* dev, float* host_rgb, size_t count, uint64_t* iteration_count) {
    if (!dev) return IGX_ERR_INVALID_ARGUMENT;
    if (iteration_count) *iteration_count = dev->iteration_count;
    if (!host_rgb) return IGX_OK;
    if (!dev->fb) {
        std::memset(host_rgb, 0, count * sizeof(float));
        return IGX_OK;
    }
    if (count != dev->fb_count) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "framebuffer size mismatch: expected " + std::to_string(dev->fb_count));
    HIPCHK(hipSetDevice(dev->hip_device));
    igx_status st = drain(dev);
    if (st != IGX_OK) return st;
    HIPCHK(hipMemcpy(host_rgb, dev->fb, count * sizeof(float), hipMemcpyDeviceToHost));
    return IGX_OK;
}

// the path tracer's AOVs (Device::getFramebufferForHost(name), Device.cpp:1330-1363):
// "Color" (or "" / NULL) is the film; "Direct Weights" and "NEE Weights" exist
// with the technique's aov_mis (PathTechnique.cpp:23-27); any other name is an
// unknown AOV (the reference logs it and returns no data)
static int aov_index(igx_device* dev, const char* name) {
    const std::string n = name ? name : "";
    if (n.empty() || n == "Color") return -1;
    if (dev->aov_on && n == "Direct Weights") return 0;
    if (dev->aov_on && n == "NEE Weights") return 1;
    return -2;
}

extern "C" igx_status igx_get_aov(igx_device* dev, const char* name, float* host_rgb, size_t count, uint64_t* iteration_count) {
    if (!dev) return IGX_ERR_INVALID_ARGUMENT;
    const int k = aov_index(dev, name);
    if (k == -1) return igx_get_framebuffer(dev, host_rgb, count, iteration_count);
    if (k == -2) return fail(dev, IGX_ERR_INVALID_ARGUMENT, std::string("unknown aov '") + (name ? name : "") + "'");
    if (iteration_count) *iteration_count = dev->iteration_count;
    if (!host_rgb) return IGX_OK;
    if (!dev->aov_fb[k]) {
        std::memset(host_rgb, 0, count * sizeof(float));
        return IGX_OK;
    }
    if (count != dev->fb_count) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "aov size mismatch: expected " + std::to_string(dev->fb_count));
    HIPCHK(hipSetDevice(dev->hip_device));
    igx_status st = drain(dev);
    if (st != IGX_OK) return st;
    HIPCHK(hipMemcpy(host_rgb, dev->aov_fb[k], count * sizeof(float), hipMemcpyDeviceToHost));
    return IGX_OK;
}

extern "C" igx_status igx_aov_device_ptr(igx_device* dev, const char* name, float** ptr, size_t* count) {
    if (!dev || !ptr) return IGX_ERR_INVALID_ARGUMENT;
    const int k = aov_index(dev, name);
    if (k == -1) return igx_framebuffer_device_ptr(dev, ptr, count);
    if (k == -2) return fail(dev, IGX_ERR_INVALID_ARGUMENT, std::string("unknown aov '") + (name ? name : "") + "'");
    *ptr = dev->aov_fb[k];
    if (count) *count = dev->aov_fb[k] ? dev->fb_count : 0;
    return IGX_OK;
}

extern "C" igx_status igx_framebuffer_device_ptr(igx_device* dev, float** ptr, size_t* count) {
    if (!dev || !ptr) return IGX_ERR_INVALID_ARGUMENT;
    *ptr = dev->fb;
    if (count) *count = dev->fb_count;
    return IGX_OK;
}

extern "C" igx_status igx_pack_tiles(igx_device* dev, const igx_render_params* p, float* dst, size_t count) {
    if (!dev || !p || !dst || p->tile_size <= 0) return IGX_ERR_INVALID_ARGUMENT;
    if (!dev->fb) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "no framebuffer");
    if (p->width != dev->fb_w || p->height != dev->fb_h || p->tile_stride <= 0 || p->tile_offset < 0)
        return fail(dev, IGX_ERR_INVALID_ARGUMENT,
                    "pack_tiles: film " + std::to_string(p->width) + "x" + std::to_string(p->height) +
                        " does not match the framebuffer " + std::to_string(dev->fb_w) + "x" + std::to_string(dev->fb_h) +
                        " (or invalid tile offset / stride)");
    FrameArgs fa{};
    fa.width = p->width;
    fa.height = p->height;
    fa.tile_size = p->tile_size;
    fa.tile_offset = p->tile_offset;
    fa.tile_stride = p->tile_stride;
    fa.tiles_x = (p->width + p->tile_size - 1) / p->tile_size;
    int tiles_y = (p->height + p->tile_size - 1) / p->tile_size;
    int tiles = fa.tiles_x * tiles_y;
    int mine = tiles > p->tile_offset ? (tiles - p->tile_offset + p->tile_stride - 1) / p->tile_stride : 0;
    size_t need = (size_t)mine * p->tile_size * p->tile_size * 3;
    if (count < need) return fail(dev, IGX_ERR_INVALID_ARGUMENT, "pack buffer too small, need " + std::to_string(need));
    HIPCHK(hipSetDevice(dev->hip_device));
    igx_status st = drain(dev);
    if (st != IGX_OK) return st;
    hipLaunchKernelGGL(k_pack_tiles, dim3(1024), dim3(256), 0, dev->stream, fa, dev->fb, dst, mine);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(dev->stream));
    return IGX_OK;
}

extern "C" igx_status igx_clear(igx_device* dev) {
    if (!dev) return IGX_ERR_INVALID_ARGUMENT;
    bool failed = false;
    if (dev->async) {
        {
            std::lock_guard<std::mutex> lk(dev->async->m);
            failed = dev->async->err != IGX_OK;
        }
        if (!failed) { // ordered behind the queued renders' resolves by the worker
            submit_async(dev, true, nullptr);
            dev->iteration_count = 0;
            return IGX_OK;
        }
        // a failed handle: the worker dropped its queue; clear here and lift the failure
        reset_async_failure(dev);
        igx_status st = drain(dev);
        if (st != IGX_OK) return st;
    }
    if (dev->fb) {
        HIPCHK(hipSetDevice(dev->hip_device));
        // resolves of queued chunks land on the tail stream; clear behind them
        HIPCHK(hipMemsetAsync(dev->fb, 0, dev->fb_count * sizeof(float), dev->tail_stream));
        for (float* a : dev->aov_fb)
            if (a) HIPCHK(hipMemsetAsync(a, 0, dev->fb_count * sizeof(float), dev->tail_stream));
    }
    dev->iteration_count = 0;
    return IGX_OK;
}

extern "C" igx_status igx_get_stats(igx_device* dev, igx_stats* out) {
    if (!dev || !out) return IGX_ERR_INVALID_ARGUMENT;
    HIPCHK(hipSetDevice(dev->hip_device));
    igx_status st = drain(dev);
    if (st != IGX_OK) return st;
    *out = dev->stats;
    out->bvh_depth = dev->scene_depth;
    out->stack_entries = LDS_STACK;
    unsigned long long h[DSTATS] = {0};
    HIPCHK(hipMemcpy(h, dev->dstats, sizeof(h), hipMemcpyDeviceToHost));
    for (int k = 0; k < 2; ++k) {
        out->shadow_class_groups[k] = h[40 + k];
        out->shadow_class_node_iters[k] = h[42 + k];
        out->shadow_class_node_visits[k] = h[44 + k];
        out->shadow_class_cycles[k] = h[46 + k];
        out->shadow_class_occluded[k] = h[48 + k];
        out->shadow_class_rays[k] = h[70 + k];
    }
    for (int k = 0; k < 16; ++k) out->extend_class_shade_cycles[k] = h[54 + k];
    out->tlas_node_visits = h[50];
    for (int k = 0; k < 3; ++k) out->hot_node_visits[k] = h[51 + k];
    for (int k = 0; k < 8; ++k) out->extend_class_cycles[k] = h[20 + k];
    for (int k = 0; k < 4; ++k) {
        out->extend_class_groups[k] = h[28 + k];
        out->extend_class_node_iters[k] = h[32 + k];
        out->extend_class_node_visits[k] = h[36 + k];
    }
    out->extend_cycles_load = h[16];
    out->extend_cycles_trace = h[17];
    out->extend_cycles_shade = h[18];
    out->extend_cycles_store = h[19];
    out->node_visits = h[0];
    out->leaf_visits = h[1];
    out->tri_tests = h[2];
    out->blas_enters = h[3];
    out->shadow_node_visits = h[4];
    out->shadow_leaf_visits = h[5];
    out->shadow_tri_tests = h[6];
    out->shadow_blas_enters = h[7];
    out->shaded_hits = h[8];
    out->wave_node_iters = h[9];
    out->wave_leaf_iters = h[10];
    out->shadow_wave_node_iters = h[11];
    out->shadow_wave_leaf_iters = h[12];
    out->bvh_width = dev->bvh_width;
    out->node_bytes = dev->nf4 * 16;
    out->lds_scene_bytes = (int32_t)dev->lds_scene_bytes;
    if (dev->has_scene && dev->tree_dirty) configure_treelet(dev);
    out->shadow_blocks_per_cu = dev->has_scene ? shadow_blocks_per_cu<false>(dev->variant, dev->lds_scene_bytes, use_refill(dev),
                                                                            tree_bytes(dev, dev->tree_shadow)) : 0;
    out->treelet_nodes[0] = dev->tree_ext;
    out->treelet_nodes[1] = 0; // k_trace_refill: no treelet
    out->treelet_nodes[2] = dev->tree_shadow;
    out->treelet_nodes[3] = 0; // tail kernels: no treelet
    out->table_bytes = dev->table_bytes;
    out->shading_bytes = dev->shading_bytes;
    out->slot_bytes = 0;
    for (const Slot& s : dev->slots)
        out->slot_bytes += (uint64_t)s.shard_cap * NSH * (2 * 56 * (s.pa.c_base ? 2 : 1) + 48 + (s.hb.h ? 20 : 0)) +
                           (uint64_t)s.cap * (16 + (s.aov_di ? 32 : 0));
    return IGX_OK;
}

extern "C" igx_status igx_reset_stats(igx_device* dev) {
    if (!dev) return IGX_ERR_INVALID_ARGUMENT;
    HIPCHK(hipSetDevice(dev->hip_device));
    igx_status st = drain(dev);
    if (st != IGX_OK) return st;
    dev->stats = igx_stats{};
    HIPCHK(hipMemset(dev->dstats, 0, DSTATS * sizeof(unsigned long long)));
    return IGX_OK;
}

static igx_status trace_batch(igx_device* dev, const float* rays, int32_t n, uint32_t flags, int32_t* ent_prim, float* tuv, int any) {
    if (!dev || (n > 0 && (!rays || !ent_prim))) return IGX_ERR_INVALID_ARGUMENT;
    if (!dev->has_scene) return fail(dev, IGX_ERR_NO_SCENE, "no scene uploaded");
    if (n <= 0) return IGX_OK;
    HIPCHK(hipSetDevice(dev->hip_device));
    igx_status st = drain(dev);
    if (st != IGX_OK) return st;
    float *d_rays = nullptr, *d_tuv = nullptr;
    int* d_ep = nullptr;
    HIPCHK(hipMalloc((void**)&d_rays, (size_t)n * 8 * sizeof(float)));
    HIPCHK(hipMalloc((void**)&d_ep, (size_t)n * 2 * sizeof(int)));
    HIPCHK(hipMalloc((void**)&d_tuv, (size_t)n * 3 * sizeof(float)));
    HIPCHK(hipMemcpy(d_rays, rays, (size_t)n * 8 * sizeof(float), hipMemcpyHostToDevice));
    int grid = grid_for(dev, n, MAX_BLOCKS_PER_CU);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (dev->timing) { // kernel time into ms_trace (traversal-only harness timing)
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        HIPCHK(hipEventRecord(e0, dev->stream));
    }
#define L_TH(S) hipLaunchKernelGGL(k_trace_hits<S>, dim3(grid), dim3(BLOCK), 0, dev->stream, dev->sv, d_rays, n, flags, d_ep, d_tuv, any)
    IGX_DISPATCH_VARIANT(dev->variant, L_TH);
#undef L_TH
    HIPCHK(hipGetLastError());
    if (e1) HIPCHK(hipEventRecord(e1, dev->stream));
    HIPCHK(hipStreamSynchronize(dev->stream));
    if (e1) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        dev->stats.ms_trace += ms;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    HIPCHK(hipMemcpy(ent_prim, d_ep, (size_t)n * (any ? 1 : 2) * sizeof(int), hipMemcpyDeviceToHost));
    if (!any && tuv) HIPCHK(hipMemcpy(tuv, d_tuv, (size_t)n * 3 * sizeof(float), hipMemcpyDeviceToHost));
    (void)hipFree(d_rays);
    (void)hipFree(d_ep);
    (void)hipFree(d_tuv);
    return IGX_OK;
}

extern "C" igx_status igx_trace_hits(igx_device* dev, const float* rays, int32_t n, uint32_t flags, int32_t* ent_prim, float* tuv) {
    return trace_batch(dev, rays, n, flags, ent_prim, tuv, 0);
}

extern "C" igx_status igx_trace_occlusion(igx_device* dev, const float* rays, int32_t n, uint32_t flags, int32_t* occluded) {
    return trace_batch(dev, rays, n, flags, occluded, nullptr, 1);
}

#endif // IGX_PART == 0
