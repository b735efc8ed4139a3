// Triangle mesh container, procedural shapes and file readers (host side).
// Restates the geometry the reference loader feeds to its BVH builder:
// src/runtime/mesh/TriMesh.{h,cpp}, PlyFile.cpp, ObjFile.cpp and the shape
// setup functions in src/runtime/shape/TriMeshProvider.cpp:19-131.
#pragma once

#include "linalg.h"

#include <array>
#include <optional>
#include <string>
#include <vector>

namespace igx {

struct TriMesh {
    std::vector<V3> vertices;
    std::vector<V3> normals;
    std::vector<std::array<float, 2>> texcoords;
    std::vector<std::array<uint32_t, 3>> faces;

    size_t face_count() const { return faces.size(); }
    BBox compute_bbox() const;
    void flip_normals();              // TriMesh::flipNormals (TriMesh.cpp:34-43)
    void compute_vertex_normals();    // TriMesh::computeVertexNormals (TriMesh.cpp:96-115)
    void fix_normals(bool* bad);      // TriMesh::fixNormals (TriMesh.cpp:17-32)
    void make_texcoords_normalized(); // TriMesh::makeTexCoordsNormalized (TriMesh.cpp:123-142)
    void setup_face_normals_as_vertex_normals(); // TriMesh.cpp:152-197
    void transform(const M4& t);      // TriMesh::transform (TriMesh.cpp:263-273)
    void append(const TriMesh& other);
};

struct PlaneShape {
    V3 origin, x_axis, y_axis;
    std::array<float, 8> tex;
};
// TriMesh::getAsPlane (TriMesh.cpp:520-634)
std::optional<PlaneShape> get_as_plane(const TriMesh& mesh);

struct SphereShape {
    V3 origin;
    float radius;
};
// TriMesh::getAsSphere (TriMesh.cpp:636-698): a closed mesh whose vertices all
// lie on one sphere around its bbox centre
std::optional<SphereShape> get_as_sphere(const TriMesh& mesh);
// TriMesh::computeArea (TriMesh.cpp:199-209)
float compute_area(const TriMesh& mesh);

// Procedural shapes (TriMesh.cpp:700-1058)
TriMesh make_plane(V3 origin, V3 x_axis, V3 y_axis);
TriMesh make_triangle(V3 p0, V3 p1, V3 p2);
TriMesh make_rectangle(V3 p0, V3 p1, V3 p2, V3 p3);
TriMesh make_box(V3 origin, V3 x_axis, V3 y_axis, V3 z_axis);
TriMesh make_ico_sphere(V3 center, float radius, uint32_t subdivisions);
TriMesh make_uv_sphere(V3 center, float radius, uint32_t stacks, uint32_t slices);
TriMesh make_disk(V3 center, V3 normal, float radius, uint32_t sections);
TriMesh make_cone(V3 base_center, float base_radius, V3 tip, uint32_t sections, bool fill_cap);
TriMesh make_cylinder(V3 base_center, float base_radius, V3 top_center, float top_radius, uint32_t sections, bool fill_cap);

// Synthetic benchmark geometry (not part of the reference's
// shape set, exposed to scene files as igx extensions):
// `count` independent triangles, centroids uniform in [-1,1]^3, vertices =
// centroid + uniform offsets in [-e,e]^3 with e = 0.01 * (1M / count)^(1/3).
TriMesh make_soup(uint32_t count, uint64_t seed);
// (n x n)-quad grid over [-size/2, size/2]^2 displaced along z by `amplitude`
// times bilinear value noise on an 8x8-cell lattice of seeded random heights.
TriMesh make_displaced_grid(uint32_t n, float size, float amplitude, uint64_t seed);

// Tangent::frame with the Duff et al. basis (src/runtime/math/Tangent.h:52-73)
void tangent_frame(V3 n, V3& nx, V3& ny);

// File readers; return false and fill err on failure.
bool load_ply(const std::string& path, TriMesh& out, std::string& err);
bool load_obj(const std::string& path, TriMesh& out, std::string& err);

} // namespace igx
