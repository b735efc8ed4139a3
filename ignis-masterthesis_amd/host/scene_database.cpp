// igx_scene_desc -> the reference's scene tables (see scene_database.h).
#include "scene_database.h"

#include "bvh_build.h"

#include <cmath>
#include <cstring>
#include <limits>
#include <stdexcept>

namespace IG {

namespace {

template <typename T>
void put(std::vector<uint8>& d, const T& v) {
    const size_t o = d.size();
    d.resize(o + sizeof(T));
    std::memcpy(d.data() + o, &v, sizeof(T));
}

// BvhBuildResult -> Node2[] in the adapter's convention (BvhNAdapter.h:121-148):
// inner child = index + 1, leaf = ~leaf_index(first slot); a root that is a
// leaf is wrapped with a cut-out sibling (BvhNAdapter.h:94-98)
void put_node2(std::vector<uint8>& d, const igx::BvhBuildResult& br, std::vector<char>& leaf_end) {
    leaf_end.assign(br.prim_order.size(), 0);
    auto child = [&](int32_t ref) -> int32_t {
        if (ref >= 0) return ref + 1;
        const int32_t code = ~ref, first = code >> igx::kLeafCountBits, count = (code & ((1 << igx::kLeafCountBits) - 1)) + 1;
        leaf_end[first + count - 1] = 1;
        return ~first;
    };
    if (br.root_is_leaf) {
        float b[12];
        std::memcpy(b, br.nodes[0].b, 6 * sizeof(float));
        const float inf = std::numeric_limits<float>::infinity();
        for (int a = 0; a < 3; ++a) { b[6 + 2 * a] = inf; b[7 + 2 * a] = -inf; }
        put(d, b);
        put(d, child(br.root_leaf_ref));
        put(d, (int32_t)0);
        put(d, (int64_t)0);
        return;
    }
    for (const igx::BvhNode& n : br.nodes) {
        put(d, n.b);
        put(d, child(n.ref[0]));
        put(d, child(n.ref[1]));
        put(d, (int64_t)0);
    }
}

igx::BvhBuildInput face_bounds(const igx_mesh& m) {
    igx::BvhBuildInput bi;
    bi.bmin.resize(3 * (size_t)m.num_faces);
    bi.bmax.resize(3 * (size_t)m.num_faces);
    bi.centroid.resize(3 * (size_t)m.num_faces);
    for (uint32_t f = 0; f < m.num_faces; ++f)
        for (int a = 0; a < 3; ++a) {
            float lo = std::numeric_limits<float>::max(), hi = -lo;
            for (int k = 0; k < 3; ++k) {
                const float v = m.vertices[3 * m.indices[3 * f + k] + a];
                lo = std::min(lo, v);
                hi = std::max(hi, v);
            }
            bi.bmin[3 * f + a] = lo;
            bi.bmax[3 * f + a] = hi;
            bi.centroid[3 * f + a] = 0.5f * (lo + hi);
        }
    return bi;
}

void col_major(const float* rows, int r, int c, float* out) {
    for (int j = 0; j < c; ++j)
        for (int i = 0; i < r; ++i) *out++ = rows[i * c + j];
}

} // namespace

void serialize_scene(const igx_scene_desc& desc, SceneDatabase& db, igx_shading_view& shading) {
    constexpr size_t kAlign = 16; // DefaultAlignment (LoaderContext.h:40)
    DynTable& shapes = db.DynTables["shapes"];
    FixTable& primbvh = db.FixTables["trimesh_primbvh"];
    std::vector<uint64> blas_offset(desc.num_shapes, 0);
    for (uint32_t s = 0; s < desc.num_shapes; ++s) {
        const igx_shape& sh = desc.shapes[s];
        if (sh.type == IGX_SHAPE_SPHERE) { // SphereProvider.cpp:40-47
            auto& d = shapes.addLookup(kSphereProviderID, 0, kAlign);
            for (int i = 0; i < 4; ++i) put(d, sh.sphere[i]);
            continue;
        }
        const igx_mesh& m = desc.meshes[sh.mesh];
        // TriMeshProvider.cpp:583-598
        auto& d = shapes.addLookup(kTrimeshProviderID, 0, kAlign);
        put(d, m.num_faces);
        put(d, m.num_vertices);
        put(d, m.num_vertices);
        put(d, m.num_vertices);
        for (int i = 0; i < 3; ++i) put(d, sh.bbox_min[i]);
        put(d, 0.0f);
        for (int i = 0; i < 3; ++i) put(d, sh.bbox_max[i]);
        put(d, 0.0f);
        for (const float* arr : {m.vertices, m.normals}) // writeAligned(.., 16): 12 B + 4 B pad
            for (uint32_t v = 0; v < m.num_vertices; ++v) {
                for (int i = 0; i < 3; ++i) put(d, arr[3 * v + i]);
                put(d, 0u);
            }
        for (uint32_t f = 0; f < m.num_faces; ++f) {
            for (int k = 0; k < 3; ++k) put(d, m.indices[3 * f + k]);
            put(d, 0u);
        }
        for (uint32_t v = 0; v < m.num_vertices; ++v) {
            put(d, m.texcoords[2 * v]);
            put(d, m.texcoords[2 * v + 1]);
        }
        // GPU-target BLAS: Node2 + Tri1 (TriMeshProvider.cpp:307-326, 361-369)
        igx::BvhBuildResult br = igx::build_bvh2(face_bounds(m), 4);
        auto& b = primbvh.addEntry(kAlign);
        blas_offset[s] = primbvh.currentOffset() / sizeof(float);
        put(b, (uint32_t)(br.root_is_leaf ? 1 : br.nodes.size()));
        put(b, (uint32_t)br.prim_order.size());
        put(b, (uint64_t)0);
        std::vector<char> leaf_end;
        put_node2(b, br, leaf_end);
        for (size_t slot = 0; slot < br.prim_order.size(); ++slot) { // TriBVHAdapter.h:148-158
            const uint32_t f = br.prim_order[slot];
            const float* v0 = m.vertices + 3 * m.indices[3 * f];
            const float* v1 = m.vertices + 3 * m.indices[3 * f + 1];
            const float* v2 = m.vertices + 3 * m.indices[3 * f + 2];
            for (int i = 0; i < 3; ++i) put(b, v0[i]);
            put(b, 0.0f);
            for (int i = 0; i < 3; ++i) put(b, v0[i] - v1[i]);
            put(b, 0.0f);
            for (int i = 0; i < 3; ++i) put(b, v2[i] - v0[i]);
            put(b, f | (leaf_end[slot] ? 0x80000000u : 0u));
        }
    }

    // entities (LoaderEntity.cpp:155-162) and one TLAS per provider (SceneBVHAdapter.h:88-135)
    FixTable& ents = db.FixTables["entities"];
    igx::BvhBuildInput tl[2];
    std::vector<uint32_t> members[2];
    BoundingBox box;
    for (int i = 0; i < 3; ++i) { box.min[i] = std::numeric_limits<float>::max(); box.max[i] = -box.min[i]; }
    for (uint32_t e = 0; e < desc.num_entities; ++e) {
        const igx_entity& en = desc.entities[e];
        auto& d = ents.addEntry(0);
        float rec[36];
        col_major(en.to_local, 3, 4, rec);
        col_major(en.to_global, 3, 4, rec + 12);
        col_major(en.normal, 3, 3, rec + 24);
        const uint32_t ids[3] = {(uint32_t)en.shape, (uint32_t)en.material, 0};
        std::memcpy(rec + 33, ids, sizeof(ids));
        put(d, rec);
        const int p = desc.shapes[en.shape].type == IGX_SHAPE_SPHERE ? 1 : 0;
        members[p].push_back(e);
        for (int a = 0; a < 3; ++a) {
            tl[p].bmin.push_back(en.bbox_min[a]);
            tl[p].bmax.push_back(en.bbox_max[a]);
            tl[p].centroid.push_back(0.5f * (en.bbox_min[a] + en.bbox_max[a]));
            box.min[a] = std::min(box.min[a], en.bbox_min[a]);
            box.max[a] = std::max(box.max[a], en.bbox_max[a]);
        }
    }
    for (int p = 0; p < 2; ++p) {
        if (members[p].empty()) continue;
        SceneBVH& bvh = db.SceneBVHs[p == 0 ? "trimesh" : "sphere"];
        igx::BvhBuildResult br = igx::build_bvh2(tl[p], 1);
        std::vector<char> leaf_end;
        put_node2(bvh.Nodes, br, leaf_end);
        for (size_t slot = 0; slot < br.prim_order.size(); ++slot) { // EntityLeaf1 (bvh.art:52-61)
            const uint32_t e = members[p][br.prim_order[slot]];
            const igx_entity& en = desc.entities[e];
            const uint64 off = blas_offset[en.shape];
            float loc[12];
            col_major(en.to_local, 3, 4, loc);
            for (int i = 0; i < 3; ++i) put(bvh.Leaves, en.bbox_min[i]);
            put(bvh.Leaves, e | (leaf_end[slot] ? 0x80000000u : 0u));
            for (int i = 0; i < 3; ++i) put(bvh.Leaves, en.bbox_max[i]);
            put(bvh.Leaves, (uint32_t)en.shape);
            put(bvh.Leaves, loc);
            put(bvh.Leaves, en.flags);
            put(bvh.Leaves, (uint32_t)en.material);
            put(bvh.Leaves, (uint32_t)(off & 0xFFFFFFFFu));
            put(bvh.Leaves, (uint32_t)(off >> 32));
        }
    }
    for (int i = 0; i < 3; ++i) {
        db.SceneBBox.min[i] = desc.scene_bbox_min[i];
        db.SceneBBox.max[i] = desc.scene_bbox_max[i];
    }
    float dx = box.max[0] - box.min[0], dy = box.max[1] - box.min[1], dz = box.max[2] - box.min[2];
    db.SceneRadius = desc.num_entities ? 0.5f * std::sqrt(dx * dx + dy * dy + dz * dz) : 0.0f;
    db.MaterialCount = desc.num_materials;

    shading = igx_shading_view{};
    shading.film_width = desc.film_width;
    shading.film_height = desc.film_height;
    shading.camera = desc.camera;
    shading.technique = desc.technique;
    shading.num_materials = desc.num_materials;
    shading.materials = desc.materials;
    shading.num_lights = desc.num_lights;
    shading.lights = desc.lights;
}

} // namespace IG
