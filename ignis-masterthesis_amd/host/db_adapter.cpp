// SceneDatabase tables -> igx_scene (the Device::assignScene seam).
//
// The reference runtime hands its device the loader's tables
// (Runtime.cpp:477-485 -> Device::assignScene, Device.h:25-30):
//   FixTables["entities"]        LoaderEntity.cpp:155-162
//   DynTables["shapes"]          TriMeshProvider.cpp:583-598, SphereProvider.cpp:40-47
//   FixTables["trimesh_primbvh"] TriMeshProvider.cpp:307-326, 361-369
//   SceneBVHs[*].Leaves          SceneBVHAdapter.h:88-104 (EntityLeaf1, bvh.art:52-61)
// This file reads those byte layouts back into an igx_scene_desc.  Materials,
// lights, camera and technique are not tables in the reference (they become
// JIT shader code); they arrive as igx_shading_view.
#include "igx_scene.h"

#include "linalg.h"
#include "mesh.h"
#include "scene_store.h"

#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

using igx::BBox;
using igx::SceneStore;
using igx::V3;

namespace {

[[noreturn]] void fail(const std::string& m) { throw std::runtime_error(m); }

// bounds-checked little-endian reads from one table
struct Reader {
    const uint8_t* p;
    uint64_t n;
    const char* what;
    void need(uint64_t off, uint64_t len) const {
        if (!p || off > n || len > n - off) fail(std::string(what) + ": record beyond the end of the table");
    }
    template <typename T>
    T at(uint64_t off) const {
        need(off, sizeof(T));
        T v;
        std::memcpy(&v, p + off, sizeof(T));
        return v;
    }
};

constexpr uint64_t kEntityBytes = 36 * 4; // LoaderEntity.cpp:155-162
constexpr uint64_t kLeafBytes = 96;       // EntityLeaf1
constexpr uint64_t kTrimeshHeader = 48;   // 4 x u32 + bbox min.xyz, 0, max.xyz, 0

} // namespace

static void build_from_tables(SceneStore& S, const igx_database_view& db, const igx_shading_view& sh) {
    // ---- shapes (DynTables["shapes"]) ----
    if (db.shapes.count && !db.shapes.lookups) fail("shapes: lookup entries missing");
    Reader shp{db.shapes.data, db.shapes.bytes, "shapes"};
    std::vector<igx::TriMesh> tri(db.shapes.count);
    for (uint64_t s = 0; s < db.shapes.count; ++s) {
        const igx_lookup_entry& L = db.shapes.lookups[s];
        const uint64_t o = L.offset;
        igx_shape out{};
        out.mesh = -1;
        if (L.type_id == db.sphere_type_id) {
            // SphereProvider.cpp:40-47: origin.xyz, radius; bbox as SphereProvider.cpp:29-36
            out.type = IGX_SHAPE_SPHERE;
            for (int i = 0; i < 4; ++i) out.sphere[i] = shp.at<float>(o + 4 * i);
            if (!(out.sphere[3] > 0)) fail("shapes: sphere record with a non-positive radius");
            V3 c(out.sphere[0], out.sphere[1], out.sphere[2]);
            const float r = out.sphere[3];
            BBox b;
            b.extend(c + V3(r, 0, 0)); b.extend(c - V3(r, 0, 0));
            b.extend(c + V3(0, r, 0)); b.extend(c - V3(0, r, 0));
            b.extend(c + V3(0, 0, r)); b.extend(c - V3(0, 0, r));
            b.inflate(1e-5f);
            for (int i = 0; i < 3; ++i) { out.bbox_min[i] = b.min[i]; out.bbox_max[i] = b.max[i]; }
        } else if (L.type_id == db.trimesh_type_id) {
            // TriMeshProvider.cpp:583-598 / trimesh.art:75-96 (v_start = 12 floats)
            out.type = IGX_SHAPE_TRIMESH;
            const uint32_t nf = shp.at<uint32_t>(o), nv = shp.at<uint32_t>(o + 4);
            const uint32_t nn = shp.at<uint32_t>(o + 8), nt = shp.at<uint32_t>(o + 12);
            if (nf == 0 || nv == 0) fail("shapes: trimesh record without faces or vertices");
            if (nn != nv || nt != nv) fail("shapes: trimesh record whose normal / texcoord count differs from its vertex count");
            for (int i = 0; i < 3; ++i) {
                out.bbox_min[i] = shp.at<float>(o + 16 + 4 * i);
                out.bbox_max[i] = shp.at<float>(o + 32 + 4 * i);
            }
            const uint64_t v0 = o + kTrimeshHeader, n0 = v0 + 16ull * nv, i0 = n0 + 16ull * nn, t0 = i0 + 16ull * nf;
            shp.need(v0, t0 + 8ull * nt - v0);
            igx::TriMesh& m = tri[s];
            m.vertices.resize(nv);
            m.normals.resize(nv);
            m.texcoords.resize(nv);
            m.faces.resize(nf);
            for (uint32_t i = 0; i < nv; ++i) {
                float v[3], n[3], t[2];
                std::memcpy(v, shp.p + v0 + 16ull * i, 12);
                std::memcpy(n, shp.p + n0 + 16ull * i, 12);
                std::memcpy(t, shp.p + t0 + 8ull * i, 8);
                m.vertices[i] = V3(v[0], v[1], v[2]);
                m.normals[i] = V3(n[0], n[1], n[2]);
                m.texcoords[i] = {t[0], t[1]};
            }
            for (uint32_t f = 0; f < nf; ++f) {
                uint32_t ix[4];
                std::memcpy(ix, shp.p + i0 + 16ull * f, 16);
                for (int k = 0; k < 3; ++k)
                    if (ix[k] >= nv) fail("shapes: trimesh index beyond its vertices");
                m.faces[f] = {ix[0], ix[1], ix[2]};
            }
            // plane detection on the loaded mesh, as TriMeshProvider.cpp:562 does
            if (auto pl = igx::get_as_plane(m)) {
                out.is_plane = 1;
                for (int i = 0; i < 3; ++i) {
                    out.plane_origin[i] = pl->origin[i];
                    out.plane_x[i] = pl->x_axis[i];
                    out.plane_y[i] = pl->y_axis[i];
                }
                for (int i = 0; i < 8; ++i) out.plane_tex[i] = pl->tex[i];
            }
        } else {
            fail("shapes: lookup " + std::to_string(s) + " has provider type " + std::to_string(L.type_id) +
                 ", neither the trimesh nor the sphere provider");
        }
        S.shapes.push_back(out);
    }

    // ---- entities (FixTables["entities"], column-major 3x4 / 3x3) ----
    Reader ent{db.entities.data, db.entities.bytes, "entities"};
    const uint64_t ne = db.entities.count;
    ent.need(0, ne * kEntityBytes);
    std::vector<uint32_t> flags(ne, 0xFu);
    std::vector<uint64_t> blas_off(ne, ~0ull);
    std::vector<char> have_leaf(ne, 0);
    for (uint32_t b = 0; b < db.num_scene_bvhs; ++b) {
        const igx_db_table& t = db.scene_bvh_leaves[b];
        if (t.bytes % kLeafBytes) fail("SceneBVH leaves: size is not a multiple of 96 bytes");
        Reader lr{t.data, t.bytes, "SceneBVH leaves"};
        for (uint64_t l = 0; l < t.bytes / kLeafBytes; ++l) {
            const uint64_t o = l * kLeafBytes;
            const uint32_t id = lr.at<uint32_t>(o + 12) & 0x7FFFFFFFu; // bit 31: last of its leaf
            if (id >= ne) fail("SceneBVH leaves: entity id beyond the entity table");
            flags[id] = lr.at<uint32_t>(o + 80);
            blas_off[id] = (uint64_t)lr.at<uint32_t>(o + 88) | ((uint64_t)lr.at<uint32_t>(o + 92) << 32);
            have_leaf[id] = 1;
        }
    }
    std::vector<uint64_t> shape_blas(S.shapes.size(), ~0ull);
    for (uint64_t e = 0; e < ne; ++e) {
        float f[36];
        std::memcpy(f, ent.p + e * kEntityBytes, sizeof(f));
        igx_entity out{};
        uint32_t sid, mid;
        std::memcpy(&sid, &f[33], 4);
        std::memcpy(&mid, &f[34], 4);
        if (sid >= S.shapes.size()) fail("entities: shape id beyond the shapes table");
        if (mid >= sh.num_materials) fail("entities: material id beyond the material table");
        out.shape = (int32_t)sid;
        out.material = (int32_t)mid;
        out.flags = flags[e];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) {
                out.to_local[r * 4 + c] = f[c * 3 + r];
                out.to_global[r * 4 + c] = f[12 + c * 3 + r];
            }
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) out.normal[r * 3 + c] = f[24 + c * 3 + r];
        // BoundingBox::transformed (LoaderEntity.cpp:141, math/BoundingBox.h:84-95)
        const igx_shape& s = S.shapes[sid];
        igx::M4 t;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) t.at(r, c) = out.to_global[r * 4 + c];
        BBox eb;
        for (int c = 0; c < 8; ++c) {
            V3 p((c & 1) ? s.bbox_max[0] : s.bbox_min[0], (c & 2) ? s.bbox_max[1] : s.bbox_min[1], (c & 4) ? s.bbox_max[2] : s.bbox_min[2]);
            eb.extend(igx::xform_point(t, p));
        }
        for (int i = 0; i < 3; ++i) { out.bbox_min[i] = eb.min[i]; out.bbox_max[i] = eb.max[i]; }
        if (have_leaf[e] && s.type == IGX_SHAPE_TRIMESH) {
            if (shape_blas[sid] != ~0ull && shape_blas[sid] != blas_off[e]) fail("SceneBVH leaves: one shape with two BLAS offsets");
            shape_blas[sid] = blas_off[e];
        }
        S.entities.push_back(out);
    }

    // ---- reference BLAS blobs (FixTables["trimesh_primbvh"], offsets in floats) ----
    if (db.trimesh_primbvh.bytes > 0) {
        Reader bv{db.trimesh_primbvh.data, db.trimesh_primbvh.bytes, "trimesh_primbvh"};
        for (size_t s = 0; s < S.shapes.size(); ++s) {
            if (S.shapes[s].type != IGX_SHAPE_TRIMESH || shape_blas[s] == ~0ull) continue;
            // offsets count floats: refuse one beyond the table before scaling it
            // (a huge user word would wrap and select the wrong bytes)
            if (shape_blas[s] > db.trimesh_primbvh.bytes / 4) fail("trimesh_primbvh: BLAS offset beyond the table");
            const uint64_t o = shape_blas[s] * 4;
            const uint64_t nn = bv.at<uint32_t>(o), nt = bv.at<uint32_t>(o + 4);
            const uint64_t len = 16 + 64 * nn + 48 * nt;
            bv.need(o, len);
            S.bvh.emplace_back(bv.p + o, bv.p + o + len);
        }
    }

    // ---- meshes into flat arrays ----
    size_t blob = 0;
    for (size_t s = 0; s < S.shapes.size(); ++s) {
        igx_shape& out = S.shapes[s];
        if (out.type != IGX_SHAPE_TRIMESH) continue;
        const igx::TriMesh& m = tri[s];
        out.mesh = (int32_t)S.vtx.size();
        std::vector<float> v, n, t;
        std::vector<uint32_t> ix;
        for (auto& p : m.vertices) { v.push_back(p.x); v.push_back(p.y); v.push_back(p.z); }
        for (auto& p : m.normals) { n.push_back(p.x); n.push_back(p.y); n.push_back(p.z); }
        for (auto& p : m.texcoords) { t.push_back(p[0]); t.push_back(p[1]); }
        for (auto& f : m.faces) { ix.push_back(f[0]); ix.push_back(f[1]); ix.push_back(f[2]); }
        S.vtx.push_back(std::move(v));
        S.nrm.push_back(std::move(n));
        S.tex.push_back(std::move(t));
        S.idx.push_back(std::move(ix));
        if (db.trimesh_primbvh.bytes > 0 && shape_blas[s] != ~0ull) {
            out.ref_bvh = S.bvh[blob].data();
            out.ref_bvh_bytes = S.bvh[blob].size();
            ++blob;
        }
    }
    for (size_t i = 0; i < S.vtx.size(); ++i) {
        igx_mesh m{};
        m.num_vertices = (uint32_t)(S.vtx[i].size() / 3);
        m.num_faces = (uint32_t)(S.idx[i].size() / 3);
        m.vertices = S.vtx[i].data();
        m.normals = S.nrm[i].data();
        m.texcoords = S.tex[i].data();
        m.indices = S.idx[i].data();
        S.meshes.push_back(m);
    }

    // ---- shading half ----
    S.materials.assign(sh.materials, sh.materials + sh.num_materials);
    S.lights.assign(sh.lights, sh.lights + sh.num_lights);
    for (const igx_light& L : S.lights)
        if (L.entity >= 0 && (uint64_t)L.entity >= ne) fail("lights: area light entity beyond the entity table");
    for (const igx_material& m : S.materials)
        if (m.light >= (int32_t)S.lights.size()) fail("materials: light index beyond the light table");
    S.desc.film_width = sh.film_width;
    S.desc.film_height = sh.film_height;
    S.desc.camera = sh.camera;
    S.desc.technique = sh.technique;
    for (int i = 0; i < 3; ++i) {
        S.desc.scene_bbox_min[i] = db.scene_bbox_min[i];
        S.desc.scene_bbox_max[i] = db.scene_bbox_max[i];
    }
    S.publish();
}

static void set_err(char* err, size_t len, const std::string& msg) {
    if (!err || len == 0) return;
    std::strncpy(err, msg.c_str(), len - 1);
    err[len - 1] = 0;
}

extern "C" igx_scene* igx_scene_from_database(const igx_database_view* db, const igx_shading_view* shading, char* err,
                                              size_t err_len) {
    if (!db || !shading) { set_err(err, err_len, "null database or shading view"); return nullptr; }
    if (shading->num_materials && !shading->materials) { set_err(err, err_len, "null material table"); return nullptr; }
    if (shading->num_lights && !shading->lights) { set_err(err, err_len, "null light table"); return nullptr; }
    if (db->num_scene_bvhs && !db->scene_bvh_leaves) { set_err(err, err_len, "null SceneBVH leaf tables"); return nullptr; }
    auto* s = new igx_scene();
    try {
        build_from_tables(s->store, *db, *shading);
    } catch (const std::exception& e) {
        delete s;
        set_err(err, err_len, e.what());
        return nullptr;
    }
    return s;
}
