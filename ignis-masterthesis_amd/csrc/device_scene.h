// Device-resident scene and stream layouts (shared by host upload code and kernels).
// See DESIGN.md "HBM layout".  All arrays are 16-byte element aligned so every
// record is fetched with global_load_dwordx4.
#pragma once

#include <stdint.h>

#ifndef __HIPCC__
struct float4_ { float x, y, z, w; };
#endif

namespace igxd {

// Traversal encodings (see host/bvh_build.h)
constexpr int32_t REF_MARKER = (int32_t)0x80000000; // return from a BLAS to the TLAS
constexpr int32_t REF_EXIT = (int32_t)0x80000001;   // bottom of the traversal stack
constexpr int LEAF_COUNT_BITS = 4;

// Kernel variant V (a template parameter): bit 1 = 4-wide nodes (128-B SoA
// node, host Bvh4Node) instead of BVH2 (64-B Node2, host BvhNode); bit 0 =
// the scene's stack need exceeds the LDS stack, so pushes and pops check for
// the spill area; bit 2 = the scene uses materials or lights beyond the basic
// set (igx_kernels.h, bsdf_eval), compiled into the shading kernels only then.
// The upload picks the variant per scene.
#ifndef IGX_LDS_STACK
#define IGX_LDS_STACK 16
#endif
constexpr int LDS_STACK = IGX_LDS_STACK; // LDS traversal-stack entries per lane
__host__ __device__ constexpr int variant_width(int v) { return (v & 2) ? 4 : 2; }
__host__ __device__ constexpr bool variant_spill(int v) { return (v & 1) != 0; }
__host__ __device__ constexpr bool variant_full(int v) { return (v & 4) != 0; }
__host__ __device__ constexpr int node_f4(int width) { return width == 4 ? 8 : 4; }
// Bit 3: the node tables are staged in LDS (stage_scene_lds; set by the
// kernels on their LDS-staged SceneView).  The node steps then skip the
// stack-top peek (IGX_PEEK_POP), whose extra LDS read costs there what it
// saves where the nodes come from global memory.  (One float4 of padding per
// LDS node, round 2, measured neutral and was removed.)
__host__ __device__ constexpr bool variant_lds_nodes(int v) { return (v & 8) != 0; }
// Bit 4: if-if stepping (trav_step advances one inner node or one leaf per
// call) -- set only on k_shadow_refill launches for scenes on the split
// schedule (igx_device.hip, use_shadow_ifif).
__host__ __device__ constexpr bool variant_ifif(int v) { return (v & 16) != 0; }
// Bit 5: the node tables stay in global memory, but the hottest nodes (the
// first SceneView::tree_n of the node array, igx_upload_scene's hot order)
// are staged in LDS (the treelet); node steps below that index read LDS.
// Set by every kernel instantiation that does not stage the whole table.
constexpr int VARIANT_TREE = 32;
// Bit 7: quantised 4-wide nodes (64 B, node_step4q; host Bvh4QNode) instead of
// the 128-B 4-wide nodes -- half the node bytes per visit on scenes whose
// tables stay in global memory.  Set by the upload with bit 1 (option
// "bvh_quantize").
constexpr int VARIANT_Q4 = 128;
__host__ __device__ constexpr bool variant_q4(int v) { return (v & VARIANT_Q4) != 0; }
constexpr int32_t REF_EMPTY = (int32_t)0x80000002; // absent child of a 4-wide node (host kEmptyRef)
__host__ __device__ constexpr bool variant_tree(int v) { return (v & VARIANT_TREE) != 0; }
__host__ __device__ constexpr int kernel_variant(int v, bool lds) { return lds ? (v | 8) : (v | VARIANT_TREE); }

// Instance record (one per TLAS leaf slot): 64 B
//   row0..row2: to_local 3x4 (row-major, xyz = linear row, w = translation)
//   info: x = entity id, y = shape type (0 trimesh, 1 sphere), z = BLAS root node
//         index (trimesh) or sphere index (sphere), w = visibility flags
// The reference's EntityLeaf1 (traversal/bvh.art:52-61) carries the same data
// plus the entity box, which here lives in the parent TLAS node.

// Per-entity shading record: 3 rows of to_global, 3 rows of normal matrix,
// info (shape, material, vtx_offset, idx_offset) -> 7 x 16 B.
constexpr int ENT_STRIDE = 7;

enum : int32_t { MAT_DIFFUSE = 0, MAT_DIELECTRIC = 1, MAT_CONDUCTOR = 2, MAT_PLASTIC = 3, MAT_PRINCIPLED = 4 };
// microfacet distribution of conductor / plastic specular lobes
// (BSDF::setupRoughness, src/runtime/bsdf/BSDF.cpp:53-99)
enum : int32_t { MF_DELTA = 0, MF_VNDF_GGX = 1, MF_GGX = 2, MF_BECKMANN = 3 };
struct DevMaterial {   // 128 B
    int32_t type, light, dist, mirror; // mirror: delta conductor with eta = 0, k = 1 (make_mirror_bsdf);
                                       // dielectric: thin interface; principled: flag bits
    float kd[4];        // diffuse reflectance; w = Oren-Nayar roughness (0: Lambert)
    float ks[4];        // specular reflectance; w = n1 (ext ior)
    float kt[4];        // specular transmittance; w = n2 (int ior)
    float eta[4];       // conductor eta; w = alpha_u
    float kappa[4];     // conductor k; w = alpha_v
    float pad[8];       // textured diffuse (igx_material::texture): pad[0] = texture (int bits),
                        // pad[1] = scale, pad[2..4] = the colour where the checker is 1 (kd elsewhere)
};

enum : int32_t { LIGHT_PLANE = 1, LIGHT_ENV = 2, LIGHT_POINT = 3, LIGHT_SPOT = 4, LIGHT_DIRECTIONAL = 5, LIGHT_SUN = 6,
                   LIGHT_SPHERE = 7, LIGHT_MESH = 8 };
struct DevLight {      // 128 B
    int32_t type, infinite, delta, entity; // entity: emitting entity of sphere / mesh area lights
    float radiance[4];
    float origin[4];   // plane origin / point/spot position; w = plane width; sphere: object-space centre, radius
    float ex[4];       // plane x axis normalised; w = plane height
    float ey[4];       // plane y axis normalised; w = inv_area
    float normal[4];   // plane normal / spot direction; w = area
    float spot[4];     // spot: cos_cutoff, cos_falloff, blend range; sun: cos_angle, sun_area;
                       // sphere: emitter area (compute_ellipsoid_area); mesh: face count
    float pad2[4];
};

struct DevCamera {
    float eye[3], dir[3], up[3], right[3];
    float scale_x, scale_y;
    float tmin, tmax;
};

} // namespace igxd
