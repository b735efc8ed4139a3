// CPU check of the C++ SceneDatabase path (compiled by tests/test_db_adapter.py
// against libigx.so; no GPU call): scene JSON -> igx loader -> serialize_scene
// (the reference's tables) -> DatabaseViewStorage -> igx_scene_from_database
// must give back the loader's desc bit for bit, every trimesh shape must carry
// a BLAS blob that bvh2_from_reference reads over all of the mesh's faces, and
// the IG::Device facade types must keep the reference's layouts.
#include "Device.h"
#include "bvh_build.h"
#include "igx_scene.h"
#include "scene_database.h"

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

static int bad = 0;
#define CHECK(c, ...)                         \
    do {                                      \
        if (!(c)) {                           \
            std::printf("FAIL: " __VA_ARGS__); \
            std::printf("\n");                \
            ++bad;                            \
        }                                     \
    } while (0)

template <typename T>
static bool same(const T& a, const T& b) { return std::memcmp(&a, &b, sizeof(T)) == 0; }

int main(int argc, char** argv) {
    static_assert(sizeof(IG::LookupEntry) == 16, "LookupEntry");
    for (int a = 1; a < argc; ++a) {
        char err[1024] = {0};
        igx_scene* sc = igx_scene_load_file(argv[a], err, sizeof(err));
        if (!sc) { std::printf("FAIL: load %s: %s\n", argv[a], err); return 1; }
        const igx_scene_desc& d = *igx_scene_get_desc(sc);
        IG::SceneDatabase db;
        igx_shading_view sh{};
        IG::serialize_scene(d, db, sh);
        CHECK(db.FixTables["entities"].entryCount() == d.num_entities, "%s entity count", argv[a]);
        CHECK(db.FixTables["entities"].data().size() == 144ull * d.num_entities, "%s entity bytes", argv[a]);
        CHECK(db.DynTables["shapes"].entryCount() == d.num_shapes, "%s shape count", argv[a]);
        IG::DatabaseViewStorage view(db);
        igx_scene* back = igx_scene_from_database(&view.view, &sh, err, sizeof(err));
        if (!back) { std::printf("FAIL: adapt %s: %s\n", argv[a], err); return 1; }
        const igx_scene_desc& e = *igx_scene_get_desc(back);
        CHECK(same(d.camera, e.camera) && same(d.technique, e.technique), "%s camera/technique", argv[a]);
        CHECK(d.num_meshes == e.num_meshes && d.num_shapes == e.num_shapes && d.num_entities == e.num_entities &&
                  d.num_materials == e.num_materials && d.num_lights == e.num_lights,
              "%s counts", argv[a]);
        for (uint32_t i = 0; i < d.num_meshes && i < e.num_meshes; ++i) {
            const igx_mesh &m = d.meshes[i], &n = e.meshes[i];
            bool ok = m.num_vertices == n.num_vertices && m.num_faces == n.num_faces &&
                      !std::memcmp(m.vertices, n.vertices, 12ull * m.num_vertices) &&
                      !std::memcmp(m.normals, n.normals, 12ull * m.num_vertices) &&
                      !std::memcmp(m.texcoords, n.texcoords, 8ull * m.num_vertices) &&
                      !std::memcmp(m.indices, n.indices, 12ull * m.num_faces);
            CHECK(ok, "%s mesh %u", argv[a], i);
        }
        size_t blobs = 0;
        for (uint32_t i = 0; i < d.num_shapes && i < e.num_shapes; ++i) {
            igx_shape s = e.shapes[i];
            const uint8_t* blob = s.ref_bvh;
            const uint64_t bytes = s.ref_bvh_bytes;
            s.ref_bvh = nullptr;
            s.ref_bvh_bytes = 0;
            CHECK(same(d.shapes[i], s), "%s shape %u", argv[a], i);
            if (s.type != IGX_SHAPE_TRIMESH) continue;
            ++blobs;
            igx::BvhBuildResult br;
            std::string msg;
            const uint32_t nf = e.meshes[s.mesh].num_faces;
            CHECK(blob && igx::bvh2_from_reference(blob, bytes, nf, br, msg), "%s BLAS of shape %u: %s", argv[a], i, msg.c_str());
            std::vector<char> seen(nf, 0);
            for (uint32_t p : br.prim_order) seen[p] = 1;
            size_t cover = 0;
            for (char c : seen) cover += c;
            CHECK(cover == nf && br.prim_order.size() == nf, "%s BLAS of shape %u covers %zu of %u faces", argv[a], i, cover, nf);
        }
        for (uint32_t i = 0; i < d.num_entities && i < e.num_entities; ++i)
            CHECK(same(d.entities[i], e.entities[i]), "%s entity %u", argv[a], i);
        for (uint32_t i = 0; i < d.num_materials && i < e.num_materials; ++i)
            CHECK(same(d.materials[i], e.materials[i]), "%s material %u", argv[a], i);
        for (uint32_t i = 0; i < d.num_lights && i < e.num_lights; ++i)
            CHECK(same(d.lights[i], e.lights[i]), "%s light %u", argv[a], i);
        std::printf("%s: %u entities, %u shapes, %zu BLAS blobs (%zu B), %zu TLAS\n", argv[a], d.num_entities, d.num_shapes,
                    blobs, db.FixTables["trimesh_primbvh"].data().size(), db.SceneBVHs.size());
        igx_scene_free(back);
        igx_scene_free(sc);
    }
    std::printf(bad ? "FAIL\n" : "ok\n");
    return bad ? 1 : 0;
}
