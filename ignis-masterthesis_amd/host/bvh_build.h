// Host-side binned-SAH BVH2 builder.
//
// Replaces madmann91/bvh (GIT_TAG v1, not vendored and unavailable offline),
// which the reference calls from build_bvh (src/runtime/bvh/TriBVHAdapter.h:163-202)
// for per-shape BLAS and from build_scene_bvh (src/runtime/bvh/SceneBVHAdapter.h:109-135)
// for the entity TLAS.  Topology differs from the reference's SBVH (parity of
// BVH topology is unpinned); closest-hit results do not depend
// on it.
//
// Output node layout = the device's 64-byte BVH2 node (DESIGN.md "HBM layout"):
//   float lo_hi[12]: c0.lo.x c0.hi.x c0.lo.y c0.hi.y | c0.lo.z c0.hi.z c1.lo.x c1.hi.x |
//                    c1.lo.y c1.hi.y c1.lo.z c1.hi.z          (Node2 interleaving,
//                    traversal/mapping_gpu.art:3-7)
//   int32 ref[2]:    >= 0 inner node index; < 0 leaf, ~ref = (first << 4) | (count - 1)
//   int32 pad[2]
// An absent child has an inverted (empty) box so its slab test always fails.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace igx {

struct BvhNode {
    float b[12];
    int32_t ref[2];
    int32_t pad[2];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode must be 64 bytes");

constexpr int kLeafCountBits = 4;               // up to 16 primitives per leaf
constexpr int32_t kMaxLeafFirst = 1 << 26;      // keeps ~ref above the stack sentinels

inline int32_t encode_leaf(int32_t first, int32_t count) { return ~((first << kLeafCountBits) | (count - 1)); }

struct BvhBuildInput {
    // per primitive: bounds min/max and centroid
    std::vector<float> bmin, bmax, centroid; // 3 floats each
    size_t count() const { return bmin.size() / 3; }
};

struct BvhBuildResult {
    std::vector<BvhNode> nodes;         // nodes[0] is the root (always an inner node)
    std::vector<uint32_t> prim_order;   // leaf slot -> original primitive index
    int depth = 0;                      // maximum root-to-leaf depth (number of inner levels)
    int max_leaf = 0;
    // All primitives fit one leaf: nodes[0] then references that leaf from
    // both children (keeps the array layout uniform), but traversal should
    // start at the leaf itself (root_leaf_ref) so it is not visited twice.
    bool root_is_leaf = false;
    int32_t root_leaf_ref = 0;
};

// Build a BVH2 with binned SAH.  `max_leaf` caps primitives per leaf (<= 16);
// `node_cost` is the SAH cost of a node step relative to one primitive test
// (a split is kept when node_cost + SAH(children) < primitive count).
BvhBuildResult build_bvh2(const BvhBuildInput& in, int max_leaf, int bins = 32, float node_cost = 1.0f);

// Binned SAH with spatial splits (SBVH) over triangles: `tri9` holds the
// three vertices of primitive i at [9 i, 9 i + 9).  A triangle may be
// referenced by several leaves (prim_order then repeats it); at most
// ref_budget * count references are added.  Closest hits are unchanged:
// every reference box bounds its part of the triangle.
BvhBuildResult build_sbvh2(const BvhBuildInput& in, const std::vector<float>& tri9, int max_leaf,
                           float ref_budget = 0.3f, int bins = 32);

// 4-wide node (128 B, two 64-B halves): child boxes as SoA so one float4
// load gives one bound of all four children.
//   float4 lo_x, hi_x, lo_y, hi_y, lo_z, hi_z   (child k in lane k)
//   int32  ref[4]: >= 0 inner node index, < 0 leaf code (encode_leaf), or
//                  kEmptyRef for an absent child, whose box is +inf on every
//                  bound so the slab test can never accept it
//   int32  pad[4]
struct Bvh4Node {
    float lo_x[4], hi_x[4], lo_y[4], hi_y[4], lo_z[4], hi_z[4];
    int32_t ref[4];
    int32_t pad[4];
};
static_assert(sizeof(Bvh4Node) == 128, "Bvh4Node must be 128 bytes");
constexpr int32_t kEmptyRef = (int32_t)0x80000002;

struct Bvh4Result {
    std::vector<Bvh4Node> nodes; // nodes[0] is the root
    int stack_need = 0;          // worst-case traversal stack entries: max over paths of sum(children - 1)
    int depth = 0;               // 4-wide levels
};

// Collapse a BVH2 into a BVH4: every 4-wide node absorbs the largest-area
// inner grandchildren of its BVH2 node until it has four children (the
// surface-area collapse of wide-BVH builders).  Leaf codes are kept.
Bvh4Result collapse_bvh4(const BvhBuildResult& bvh2);

// 4-wide node with quantised child boxes (64 B, half a Bvh4Node; traversed by
// node_step4q).  Per axis a a node origin o_a and a power-of-two scale s_a;
// child k's bound on axis a is o_a + q * s_a with q the byte k of the qlo / qhi
// word of that axis.  Every quantised box contains the child's (padded) box
// with at least half a quantum to spare on each side, and a quantum is at
// least 2^-19 of the coordinates' magnitude (16 float ulps), so the slab test
// accepts every ray the exact box would: the tree visits a superset of the
// triangles, and closest hits (independent of topology, accept_hit) stay the
// same.  Absent children keep kEmptyRef and are masked by their ref.
//   float o_x, o_y, o_z, s_x | float s_y, s_z, u32 qlo_x, qhi_x |
//   u32 qlo_y, qhi_y, qlo_z, qhi_z | int32 ref[4]
struct Bvh4QNode {
    float origin[3];
    float sx, sy, sz;
    uint32_t qlo_x, qhi_x, qlo_y, qhi_y, qlo_z, qhi_z;
    int32_t ref[4];
};
static_assert(sizeof(Bvh4QNode) == 64, "Bvh4QNode must be 64 bytes");
Bvh4QNode quantize_bvh4(const Bvh4Node& n);

// N-wide node before quantisation (quantize_bvh4): bounds per axis, child k in
// column k; absent children as in Bvh4Node (kEmptyRef, +inf bounds).
template <int N>
struct WideNode {
    float lo[3][N], hi[3][N];
    int32_t ref[N];
};
// Read the reference's GPU BLAS (one FixTables["trimesh_primbvh"] entry:
// u32 node_count, tri_count, 0, 0; Node2[]; Tri1[], TriMeshProvider.cpp:307-326)
// into the device's BVH2 form: same boxes and topology, leaf codes over the
// Tri1 slots, prim_order = each slot's prim_id.  Leaves above 16 triangles
// become small subtrees.  false + err on a malformed blob.
bool bvh2_from_reference(const uint8_t* blob, size_t bytes, uint32_t num_faces, BvhBuildResult& out, std::string& err);

} // namespace igx
