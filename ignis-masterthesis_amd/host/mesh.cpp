// Procedural meshes and mesh readers; see mesh.h for the reference citations.
//
// Provenance: the shapes, normal helpers and the plane-emitter test reproduce
// the geometry of the reference's src/runtime/mesh/TriMesh.cpp (Ignis, MIT
// licence) so that the hot path intersects the same triangles; the code is
// written from the geometric definitions, and tests/golden/procedural_shapes.npz
// pins its output bit for bit.
#include "mesh.h"

#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <tuple>
#include <unordered_map>

namespace igx {

static constexpr float kPi = 3.14159265358979323846f;
static constexpr float kFltEps = 1.1920928955e-07f;

static V3 triangle_normal(V3 v0, V3 v1, V3 v2) { return cross(v1 - v0, v2 - v0); }

BBox TriMesh::compute_bbox() const {
    BBox b;
    for (auto& v : vertices) b.extend(v);
    return b;
}

void TriMesh::flip_normals() {
    for (auto& f : faces) std::swap(f[1], f[2]);
    for (auto& n : normals) n = -n;
}

// Smooth vertex normals: every vertex gets the normalised sum of the unit
// normals of the faces around it (no area or angle weighting, as the
// reference's computeVertexNormals).  Contributions are added in face order.
void TriMesh::compute_vertex_normals() {
    std::vector<V3> acc(vertices.size(), V3());
    for (const auto& f : faces) {
        const V3 n = normalized(triangle_normal(vertices[f[0]], vertices[f[1]], vertices[f[2]]));
        for (uint32_t v : f) acc[v] = acc[v] + n;
    }
    for (auto& n : acc) n = normalized(n);
    normals = std::move(acc);
}

// Normals read from files may be zero or NaN: those become +y (and *bad is
// set), the others are brought to unit length.
void TriMesh::fix_normals(bool* bad) {
    bool any_bad = false;
    for (auto& n : normals) {
        const float len2 = norm2(n);
        const bool degenerate = !(len2 > kFltEps); // also catches NaN
        any_bad = any_bad || degenerate;
        n = degenerate ? V3(0, 1, 0) : n / std::sqrt(len2);
    }
    if (bad) *bad = any_bad;
}

// Planar (x, y) projection of each vertex into the unit square of the mesh's
// bounding box; a flat axis maps to 0.
void TriMesh::make_texcoords_normalized() {
    const BBox box = compute_bbox();
    const V3 extent = box.diameter();
    auto coord = [&](float p, float lo, float size) { return size > kFltEps ? (p - lo) / size : 0.0f; };
    texcoords.resize(vertices.size());
    for (size_t i = 0; i < vertices.size(); ++i)
        texcoords[i] = {coord(vertices[i].x, box.min.x, extent.x), coord(vertices[i].y, box.min.y, extent.y)};
}

// Flat shading: every face gets three vertices of its own carrying the face's
// unit normal (and the texture coordinates of its corners).
void TriMesh::setup_face_normals_as_vertex_normals() {
    const bool has_uv = !texcoords.empty();
    std::vector<V3> pos, nrm;
    std::vector<std::array<float, 2>> uv;
    pos.reserve(faces.size() * 3);
    nrm.reserve(faces.size() * 3);
    if (has_uv) uv.reserve(faces.size() * 3);
    for (auto& f : faces) {
        const V3 n = normalized(triangle_normal(vertices[f[0]], vertices[f[1]], vertices[f[2]]));
        const uint32_t first = (uint32_t)pos.size();
        for (uint32_t v : f) {
            pos.push_back(vertices[v]);
            nrm.push_back(n);
            if (has_uv) uv.push_back(texcoords[v]);
        }
        f = {first, first + 1, first + 2};
    }
    vertices = std::move(pos);
    normals = std::move(nrm);
    if (has_uv) texcoords = std::move(uv);
}

void TriMesh::transform(const M4& t) {
    if (t.is_identity()) return;
    M3 nm = transpose3(inverse3(linear_of(t))); // NormalMatrix = L^T^-1 (TriMesh.cpp:245-248)
    for (auto& v : vertices) v = xform_point(t, v);
    for (auto& n : normals) n = normalized(mul3(nm, n));
}

void TriMesh::append(const TriMesh& o) {
    uint32_t off = (uint32_t)vertices.size();
    vertices.insert(vertices.end(), o.vertices.begin(), o.vertices.end());
    normals.insert(normals.end(), o.normals.begin(), o.normals.end());
    texcoords.insert(texcoords.end(), o.texcoords.begin(), o.texcoords.end());
    for (auto f : o.faces) faces.push_back({f[0] + off, f[1] + off, f[2] + off});
}

// ---------------------------------------------------------------------------
std::optional<SphereShape> get_as_sphere(const TriMesh& mesh) {
    constexpr float kEps = 1e-5f;
    if (mesh.face_count() < 32 || mesh.vertices.empty()) return std::nullopt; // too coarse to stand for a sphere
    const BBox b = mesh.compute_bbox();
    const V3 c = b.center();
    const V3 d = b.diameter();
    if (d.x * d.y * d.z <= kEps) return std::nullopt; // flat
    if (std::fabs(d.x - d.y) > kEps || std::fabs(d.x - d.z) > kEps || std::fabs(d.y - d.z) > kEps) return std::nullopt;
    auto dist2 = [&](V3 v) { V3 t = c - v; return dot(t, t); };
    const float r2 = dist2(mesh.vertices[0]);
    if (r2 <= kEps) return std::nullopt;
    bool octant[8] = {};
    for (size_t i = 0; i < mesh.vertices.size(); ++i) {
        if (i > 0 && std::fabs(dist2(mesh.vertices[i]) - r2) > kEps) return std::nullopt;
        V3 t = c - mesh.vertices[i];
        octant[(t.x < 0 ? 1 : 0) | (t.y < 0 ? 2 : 0) | (t.z < 0 ? 4 : 0)] = true;
    }
    for (bool o : octant)
        if (!o) return std::nullopt;
    return SphereShape{c, std::sqrt(r2)};
}

float compute_area(const TriMesh& mesh) {
    float a = 0;
    for (auto& f : mesh.faces)
        a += 0.5f * norm(cross(mesh.vertices[f[1]] - mesh.vertices[f[0]], mesh.vertices[f[2]] - mesh.vertices[f[0]]));
    return a;
}

// Plane-emitter detection (the reference's TriMesh::getAsPlane decides which
// area lights use the spherical-rectangle sampler, so the decision and the
// axes it returns must be the same):
//  * two faces over exactly four vertices.  The reference also scans meshes of
//    five or six vertices for duplicates, but its scan can register at most
//    three distinct corners, so such meshes are never planes;
//  * both faces have the same unit normal (within 1e-5, relative);
//  * each edge of the second face has the squared length of some edge of the
//    first (within 1e-5, absolute);
//  * the axes start at vertex 0 and span the widest corner angle among the
//    vertex pairs (1,2), (2,3), (3,1) -- the first in that order on ties --
//    swapped if needed so that x_axis x y_axis points along the face normal;
//  * texture coordinates of the corners origin, +x, +y, +x+y in slots 0..3
//    (unit square when the mesh has none).
std::optional<PlaneShape> get_as_plane(const TriMesh& mesh) {
    constexpr float kTol = 1e-5f;
    if (mesh.face_count() != 2 || mesh.vertices.size() != 4) return std::nullopt;
    const auto& P = mesh.vertices;
    const auto& A = mesh.faces[0];
    const auto& B = mesh.faces[1];

    const V3 normal = normalized(triangle_normal(P[A[0]], P[A[1]], P[A[2]]));
    if (!approx(normal, normalized(triangle_normal(P[B[0]], P[B[1]], P[B[2]])), kTol)) return std::nullopt;

    auto edges = [&](const std::array<uint32_t, 3>& f) {
        return std::array<float, 3>{norm2(P[f[0]] - P[f[1]]), norm2(P[f[1]] - P[f[2]]), norm2(P[f[2]] - P[f[0]])};
    };
    const auto ea = edges(A), eb = edges(B);
    for (float b : eb) {
        bool matched = false;
        for (float a : ea) matched = matched || std::abs(a - b) <= kTol;
        if (!matched) return std::nullopt;
    }

    // corner pair k = (k % 3 + 1, (k + 1) % 3 + 1): (1,2), (2,3), (3,1)
    const V3 origin = P[0];
    auto first_of = [](int k) { return (uint32_t)(k % 3 + 1); };
    auto second_of = [](int k) { return (uint32_t)((k + 1) % 3 + 1); };
    int widest = 0;
    float widest_angle = -1;
    for (int k = 0; k < 3; ++k) {
        const float ang = std::abs(std::acos(dot(normalized(P[first_of(k)] - origin), normalized(P[second_of(k)] - origin))));
        if (ang > widest_angle) { widest_angle = ang; widest = k; }
    }
    uint32_t vx = first_of(widest), vy = second_of(widest);
    PlaneShape shape;
    shape.origin = origin;
    shape.x_axis = P[vx] - origin;
    shape.y_axis = P[vy] - origin;
    if (dot(normal, normalized(cross(shape.x_axis, shape.y_axis))) < 0) {
        std::swap(shape.x_axis, shape.y_axis);
        std::swap(vx, vy);
    }
    if (mesh.texcoords.empty()) {
        shape.tex = {0, 0, 1, 0, 0, 1, 1, 1};
        return shape;
    }
    // The reference fills texture slots 1..3, rotated by the widest pair's
    // index, from vertices 1, 2, 3 in file order (1 and 2 exchanged when the
    // axes were swapped) rather than from the pair's own corners; kept so the
    // emitter's texture coordinates are the same.
    const bool swapped = vx != first_of(widest);
    const uint32_t from[3] = {swapped ? 2u : 1u, swapped ? 1u : 2u, 3u};
    auto put = [&](int slot, uint32_t v) {
        shape.tex[slot * 2] = mesh.texcoords[v][0];
        shape.tex[slot * 2 + 1] = mesh.texcoords[v][1];
    };
    put(0, 0);
    for (int j = 0; j < 3; ++j) put((j + widest) % 3 + 1, from[j]);
    return shape;
}

// ---------------------------------------------------------------------------
static void add_triangle(TriMesh& m, V3 origin, V3 xa, V3 ya) {
    V3 n = normalized(cross(xa, ya));
    uint32_t off = (uint32_t)m.vertices.size();
    m.vertices.insert(m.vertices.end(), {origin, origin + xa, origin + ya});
    m.normals.insert(m.normals.end(), {n, n, n});
    m.texcoords.insert(m.texcoords.end(), {{0, 0}, {1, 0}, {0, 1}});
    m.faces.push_back({off, off + 1, off + 2});
}

static void add_grid(TriMesh& m, V3 origin, V3 xa, V3 ya, uint32_t cx, uint32_t cy) {
    V3 n = normalized(cross(xa, ya));
    uint32_t off = (uint32_t)m.vertices.size();
    for (uint32_t j = 0; j <= cy; ++j)
        for (uint32_t i = 0; i <= cx; ++i) {
            float u = i / (float)cx, v = j / (float)cy;
            m.vertices.push_back(origin + xa * u + ya * v);
            m.normals.push_back(n);
            m.texcoords.push_back({u, v});
        }
    for (uint32_t j = 0; j < cy; ++j)
        for (uint32_t i = 0; i < cx; ++i) {
            uint32_t i1 = j * (cx + 1) + i + off;
            uint32_t i2 = (j + 1) * (cx + 1) + i + off;
            m.faces.push_back({i1, i1 + 1, i2 + 1});
            m.faces.push_back({i1, i2 + 1, i2});
        }
}

static void add_disk(TriMesh& m, V3 origin, V3 n, V3 nx, V3 ny, float radius, uint32_t sections, bool fill, bool flip = false) {
    float step = 1.0f / sections;
    uint32_t off = (uint32_t)m.vertices.size();
    if (fill) {
        m.vertices.push_back(origin);
        m.normals.push_back(n);
        m.texcoords.push_back({0, 0});
    }
    for (uint32_t i = 0; i < sections; ++i) {
        float x = std::cos(2 * kPi * step * i);
        float y = std::sin(2 * kPi * step * i);
        m.vertices.push_back(nx * (radius * x) + ny * (radius * y) + origin);
        m.normals.push_back(n);
        m.texcoords.push_back({0.5f * (x + 1), 0.5f * (y + 1)});
    }
    if (!fill) return;
    for (uint32_t i = 0; i < sections; ++i) {
        uint32_t c = i + 1;
        uint32_t nc = (i + 1 < sections ? i + 1 : 0) + 1;
        if (flip) m.faces.push_back({off, nc + off, c + off});
        else m.faces.push_back({off, c + off, nc + off});
    }
}

void tangent_frame(V3 n, V3& nx, V3& ny) {
    float sign = std::copysign(1.0f, n.z);
    float a = -1.0f / (sign + n.z);
    float b = n.x * n.y * a;
    nx = V3(1.0f + sign * n.x * n.x * a, sign * b, -sign * n.x);
    ny = V3(b, sign + n.y * n.y * a, -n.y);
    nx = normalized(nx);
    ny = normalized(ny);
}

TriMesh make_plane(V3 origin, V3 xa, V3 ya) { TriMesh m; add_grid(m, origin, xa, ya, 1, 1); return m; }
TriMesh make_triangle(V3 p0, V3 p1, V3 p2) { TriMesh m; add_triangle(m, p0, p1 - p0, p2 - p0); return m; }
TriMesh make_rectangle(V3 p0, V3 p1, V3 p2, V3 p3) {
    TriMesh m;
    add_triangle(m, p0, p1 - p0, p3 - p0);
    add_triangle(m, p1, p2 - p1, p3 - p1);
    return m;
}
TriMesh make_box(V3 o, V3 xa, V3 ya, V3 za) {
    V3 hhh = o + xa + ya + za;
    TriMesh m;
    add_grid(m, o, ya, xa, 1, 1);
    add_grid(m, o, xa, za, 1, 1);
    add_grid(m, o, za, ya, 1, 1);
    add_grid(m, hhh, -xa, -ya, 1, 1);
    add_grid(m, hhh, -za, -xa, 1, 1);
    add_grid(m, hhh, -ya, -za, 1, 1);
    return m;
}

TriMesh make_uv_sphere(V3 center, float radius, uint32_t stacks, uint32_t slices) {
    TriMesh m;
    float drho = 3.141592f / (float)stacks;
    float dtheta = 2 * 3.141592f / (float)slices;
    for (uint32_t i = 0; i <= stacks; ++i) {
        float rho = (float)i * drho;
        float srho = std::sin(rho), crho = std::cos(rho);
        for (uint32_t j = 0; j < slices; ++j) {
            float theta = (j == slices) ? 0.0f : j * dtheta;
            float stheta = -std::sin(theta), ctheta = std::cos(theta);
            V3 n(stheta * srho, ctheta * srho, crho);
            m.vertices.push_back(n * radius + center);
            m.normals.push_back(n);
            m.texcoords.push_back({(float)(0.5 * theta / kPi), rho / kPi});
        }
    }
    for (uint32_t i = 0; i <= stacks; ++i) {
        uint32_t cur = i * slices;
        uint32_t nxt = ((i + 1) % (stacks + 1)) * slices;
        for (uint32_t j = 0; j < slices; ++j) {
            uint32_t nj = (j + 1) % slices;
            uint32_t id0 = cur + j, id1 = cur + nj, id2 = nxt + j, id3 = nxt + nj;
            m.faces.push_back({id2, id3, id1});
            m.faces.push_back({id2, id1, id0});
        }
    }
    return m;
}

namespace {
// splitmix64: a fixed, platform-independent generator for the synthetic scenes
struct SplitMix {
    uint64_t x;
    uint64_t next() {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    float uniform() { return (float)(next() >> 40) * (1.0f / 16777216.0f); } // [0, 1)
    float range(float a, float b) { return a + (b - a) * uniform(); }
};
} // namespace

TriMesh make_soup(uint32_t count, uint64_t seed) {
    TriMesh m;
    SplitMix rng{seed};
    const float e = 0.01f * std::cbrt(1.0e6f / (float)std::max<uint32_t>(count, 1));
    m.vertices.resize((size_t)count * 3);
    m.normals.resize((size_t)count * 3);
    m.faces.resize(count);
    for (uint32_t i = 0; i < count; ++i) {
        V3 c(rng.range(-1, 1), rng.range(-1, 1), rng.range(-1, 1));
        V3 v[3];
        for (int k = 0; k < 3; ++k) v[k] = c + V3(rng.range(-e, e), rng.range(-e, e), rng.range(-e, e));
        V3 n = normalized(cross(v[1] - v[0], v[2] - v[0]));
        for (int k = 0; k < 3; ++k) {
            m.vertices[3 * (size_t)i + k] = v[k];
            m.normals[3 * (size_t)i + k] = n;
        }
        m.faces[i] = {3 * i, 3 * i + 1, 3 * i + 2};
    }
    return m;
}

TriMesh make_displaced_grid(uint32_t n, float size, float amplitude, uint64_t seed) {
    TriMesh m;
    SplitMix rng{seed};
    constexpr int L = 8; // lattice cells per side
    float lat[L + 1][L + 1];
    for (int j = 0; j <= L; ++j)
        for (int i = 0; i <= L; ++i) lat[j][i] = rng.uniform();
    auto noise = [&](float u, float v) { // u, v in [0, 1]
        float x = u * L, y = v * L;
        int i = std::min((int)x, L - 1), j = std::min((int)y, L - 1);
        float fx = x - i, fy = y - j;
        fx = fx * fx * (3 - 2 * fx);
        fy = fy * fy * (3 - 2 * fy);
        float a = lat[j][i] + (lat[j][i + 1] - lat[j][i]) * fx;
        float b = lat[j + 1][i] + (lat[j + 1][i + 1] - lat[j + 1][i]) * fx;
        return a + (b - a) * fy;
    };
    for (uint32_t j = 0; j <= n; ++j)
        for (uint32_t i = 0; i <= n; ++i) {
            float u = (float)i / n, v = (float)j / n;
            m.vertices.push_back(V3((u - 0.5f) * size, (v - 0.5f) * size, amplitude * noise(u, v)));
        }
    for (uint32_t j = 0; j < n; ++j)
        for (uint32_t i = 0; i < n; ++i) {
            uint32_t a = j * (n + 1) + i, b = a + 1, c = a + (n + 1), d = c + 1;
            m.faces.push_back({a, b, d});
            m.faces.push_back({a, d, c});
        }
    m.compute_vertex_normals();
    return m;
}

// Icosphere: the regular icosahedron on the unit sphere, refined by splitting
// every triangle into four at its edge midpoints (pushed back onto the sphere),
// then scaled and moved.  Vertex and face order follow the reference's
// MakeIcoSphere exactly (they decide the BVH and so the order of equal-distance
// hits): the 12 corners are (0, +-G, +-1), (+-1, 0, +-G), (+-G, +-1, 0)
// normalised (G the golden ratio), and a new midpoint is appended when its edge
// is met in ascending vertex order while faces are scanned in order.
TriMesh make_ico_sphere(V3 center, float radius, uint32_t subdivisions) {
    constexpr float G = 1.618033989f;
    static const uint32_t kFaces[20][3] = {
        {0, 8, 4},  {0, 5, 10}, {1, 6, 8},  {1, 10, 7}, {2, 4, 9},  {2, 11, 5}, {3, 9, 6},
        {3, 7, 11}, {1, 8, 0},  {1, 0, 10}, {3, 2, 9},  {3, 11, 2}, {5, 0, 4},  {5, 4, 2},
        {7, 6, 1},  {7, 3, 6},  {9, 4, 8},  {9, 8, 6},  {11, 10, 5}, {11, 7, 10}};
    TriMesh m;
    for (int axis = 0; axis < 3; ++axis) // corners lie in the planes x = 0, y = 0, z = 0
        for (float a : {-G, G})
            for (float b : {-1.0f, 1.0f}) {
                V3 v;
                v[(axis + 1) % 3] = a;
                v[(axis + 2) % 3] = b;
                m.vertices.push_back(normalized(v));
            }
    for (auto& f : kFaces) m.faces.push_back({f[0], f[1], f[2]});

    for (uint32_t level = 0; level < subdivisions; ++level) {
        const uint64_t stride = m.vertices.size();
        std::unordered_map<uint64_t, uint32_t> midpoint; // key: lo * stride + hi
        auto key = [&](uint32_t a, uint32_t b) { return (uint64_t)std::min(a, b) * stride + std::max(a, b); };
        for (const auto& f : m.faces)
            for (int e = 0; e < 3; ++e) {
                const uint32_t a = f[e], b = f[(e + 1) % 3];
                if (a < b) {
                    midpoint[key(a, b)] = (uint32_t)m.vertices.size();
                    m.vertices.push_back(normalized(m.vertices[a] + m.vertices[b]));
                }
            }
        std::vector<std::array<uint32_t, 3>> finer;
        finer.reserve(4 * m.faces.size());
        for (const auto& f : m.faces) {
            const uint32_t mid[3] = {midpoint[key(f[0], f[1])], midpoint[key(f[1], f[2])], midpoint[key(f[2], f[0])]};
            finer.push_back({mid[0], mid[1], mid[2]});                  // centre triangle
            for (int c = 0; c < 3; ++c) finer.push_back({f[c], mid[c], mid[(c + 2) % 3]}); // corner triangles
        }
        m.faces = std::move(finer);
    }

    // unit normals and spherical texture coordinates (phi from +y toward -x)
    m.normals.resize(m.vertices.size());
    m.texcoords.resize(m.vertices.size());
    for (size_t i = 0; i < m.vertices.size(); ++i) {
        const V3 n = normalized(m.vertices[i]);
        float phi = std::atan2(-n.x, n.y);
        if (phi < 0) phi += 2 * kPi;
        m.normals[i] = n;
        m.texcoords[i] = {phi / (2 * kPi), std::acos(n.z) / kPi};
    }
    M4 place;
    if (!(center.x == 0 && center.y == 0 && center.z == 0)) place = place * translation(center);
    if (radius != 1) place = place * scaling(V3(radius, radius, radius));
    m.transform(place);
    return m;
}

TriMesh make_disk(V3 center, V3 normal, float radius, uint32_t sections) {
    sections = std::max<uint32_t>(3, sections);
    V3 nx, ny;
    tangent_frame(normal, nx, ny);
    TriMesh m;
    add_disk(m, center, normal, nx, ny, radius, sections, true);
    return m;
}

TriMesh make_cone(V3 base, float base_radius, V3 tip, uint32_t sections, bool fill) {
    sections = std::max<uint32_t>(3, sections);
    V3 h = normalized(base - tip);
    V3 nx, ny;
    tangent_frame(h, nx, ny);
    TriMesh m;
    add_disk(m, base, h, nx, ny, base_radius, sections, fill);
    m.vertices.push_back(tip);
    m.normals.push_back(h);
    m.texcoords.push_back({0, 0});
    uint32_t start = fill ? 1 : 0;
    uint32_t tp = (uint32_t)m.vertices.size() - 1;
    for (uint32_t i = 0; i < sections; ++i) {
        uint32_t c = i + start, nc = (i + 1 < sections ? i + 1 : 0) + start;
        m.faces.push_back({c, tp, nc});
    }
    m.compute_vertex_normals();
    return m;
}

TriMesh make_cylinder(V3 base, float base_radius, V3 top, float top_radius, uint32_t sections, bool fill) {
    sections = std::max<uint32_t>(3, sections);
    V3 h = normalized(base - top);
    V3 nx, ny;
    tangent_frame(h, nx, ny);
    TriMesh m;
    add_disk(m, base, h, nx, ny, base_radius, sections, fill);
    uint32_t off = (uint32_t)m.vertices.size();
    add_disk(m, top, h, nx, ny, top_radius, sections, fill, true);
    uint32_t start = fill ? 1 : 0;
    for (uint32_t i = 0; i < sections; ++i) {
        uint32_t c = i + start, nc = (i + 1 < sections ? i + 1 : 0) + start;
        m.faces.push_back({c, c + off, nc});
        m.faces.push_back({c + off, nc + off, nc});
    }
    m.compute_vertex_normals();
    return m;
}

// ---------------------------------------------------------------------------
// PLY reader (ascii / binary little+big endian), after src/runtime/mesh/PlyFile.cpp.
// Polygons with more than three corners are fan-triangulated (the reference
// ear-clips, Triangulation.cpp; identical for convex faces).
namespace {
struct PlyProp {
    std::string name, type, list_count_type, list_item_type;
    bool is_list = false;
};
size_t ply_type_size(const std::string& t) {
    if (t == "char" || t == "uchar" || t == "int8" || t == "uint8" || t == "uint8_t") return 1;
    if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
    if (t == "int" || t == "uint" || t == "float" || t == "int32" || t == "uint32" || t == "float32") return 4;
    if (t == "double" || t == "float64") return 8;
    return 0;
}
double ply_read_bin(std::istream& in, const std::string& t, bool swap) {
    unsigned char buf[8];
    size_t n = ply_type_size(t);
    in.read(reinterpret_cast<char*>(buf), (std::streamsize)n);
    if (swap) std::reverse(buf, buf + n);
    if (t == "char" || t == "int8") return (double)(int8_t)buf[0];
    if (t == "uchar" || t == "uint8" || t == "uint8_t") return (double)buf[0];
    if (t == "short" || t == "int16") { int16_t v; std::memcpy(&v, buf, 2); return v; }
    if (t == "ushort" || t == "uint16") { uint16_t v; std::memcpy(&v, buf, 2); return v; }
    if (t == "int" || t == "int32") { int32_t v; std::memcpy(&v, buf, 4); return v; }
    if (t == "uint" || t == "uint32") { uint32_t v; std::memcpy(&v, buf, 4); return v; }
    if (t == "float" || t == "float32") { float v; std::memcpy(&v, buf, 4); return v; }
    double v; std::memcpy(&v, buf, 8); return v;
}
} // namespace

bool load_ply(const std::string& path, TriMesh& out, std::string& err) {
    std::ifstream in(path, std::ios::binary);
    if (!in) { err = "cannot open " + path; return false; }
    std::string line;
    std::getline(in, line);
    if (line.rfind("ply", 0) != 0) { err = path + ": not a ply file"; return false; }
    std::string format;
    size_t nv = 0, nf = 0;
    std::vector<PlyProp> vprops, fprops;
    std::vector<std::pair<std::string, size_t>> elements;
    std::string cur;
    while (std::getline(in, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream ss(line);
        std::string tok;
        ss >> tok;
        if (tok == "format") ss >> format;
        else if (tok == "element") {
            size_t n; ss >> cur >> n;
            elements.push_back({cur, n});
            if (cur == "vertex") nv = n;
            else if (cur == "face") nf = n;
        } else if (tok == "property") {
            PlyProp p;
            std::string t; ss >> t;
            if (t == "list") { p.is_list = true; ss >> p.list_count_type >> p.list_item_type >> p.name; }
            else { p.type = t; ss >> p.name; }
            if (cur == "vertex") vprops.push_back(p);
            else if (cur == "face") fprops.push_back(p);
        } else if (tok == "end_header") break;
    }
    bool ascii = format == "ascii";
    bool swap = format == "binary_big_endian";
    if (!ascii && format != "binary_little_endian" && !swap) { err = path + ": unknown ply format " + format; return false; }

    int ix = -1, iy = -1, iz = -1, inx = -1, iny = -1, inz = -1, iu = -1, ivv = -1;
    for (size_t i = 0; i < vprops.size(); ++i) {
        const auto& n = vprops[i].name;
        if (n == "x") ix = (int)i; else if (n == "y") iy = (int)i; else if (n == "z") iz = (int)i;
        else if (n == "nx") inx = (int)i; else if (n == "ny") iny = (int)i; else if (n == "nz") inz = (int)i;
        else if (n == "u" || n == "s" || n == "texture_u" || n == "texture_s") iu = (int)i;
        else if (n == "v" || n == "t" || n == "texture_v" || n == "texture_t") ivv = (int)i;
    }
    bool has_n = inx >= 0 && iny >= 0 && inz >= 0;
    bool has_uv = iu >= 0 && ivv >= 0;

    TriMesh m;
    std::vector<double> vals(vprops.size());
    for (auto& el : elements) {
        if (el.first == "vertex") {
            for (size_t i = 0; i < nv; ++i) {
                if (ascii) {
                    for (auto& v : vals) in >> v;
                } else {
                    for (size_t k = 0; k < vprops.size(); ++k) vals[k] = ply_read_bin(in, vprops[k].type, swap);
                }
                m.vertices.push_back(V3((float)vals[ix], (float)vals[iy], (float)vals[iz]));
                if (has_n) {
                    float nx = (float)vals[inx], ny = (float)vals[iny], nz = (float)vals[inz];
                    float l = std::sqrt(nx * nx + ny * ny + nz * nz);
                    if (l == 0.0f) l = 1.0f;
                    m.normals.push_back(V3(nx / l, ny / l, nz / l));
                }
                if (has_uv) m.texcoords.push_back({(float)vals[iu], (float)vals[ivv]});
            }
        } else if (el.first == "face") {
            for (size_t i = 0; i < nf; ++i) {
                std::vector<uint32_t> poly;
                for (auto& p : fprops) {
                    if (p.is_list) {
                        size_t cnt;
                        if (ascii) { in >> cnt; } else { cnt = (size_t)ply_read_bin(in, p.list_count_type, swap); }
                        std::vector<uint32_t> items(cnt);
                        for (size_t k = 0; k < cnt; ++k) {
                            double v;
                            if (ascii) in >> v; else v = ply_read_bin(in, p.list_item_type, swap);
                            items[k] = (uint32_t)v;
                        }
                        if (p.name == "vertex_indices" || p.name == "vertex_index") poly = items;
                    } else {
                        double v;
                        if (ascii) in >> v; else v = ply_read_bin(in, p.type, swap);
                        (void)v;
                    }
                }
                for (size_t k = 1; k + 1 < poly.size(); ++k) m.faces.push_back({poly[0], poly[k], poly[k + 1]});
            }
        } else {
            err = path + ": unsupported ply element " + el.first;
            return false;
        }
        if (!in) { err = path + ": truncated ply"; return false; }
    }
    if (m.vertices.empty() || m.faces.empty()) { err = path + ": empty mesh"; return false; }
    for (auto& f : m.faces)
        for (auto i : f)
            if (i >= m.vertices.size()) { err = path + ": index out of range"; return false; }
    if (m.normals.empty()) m.compute_vertex_normals();
    else m.fix_normals(nullptr);
    if (m.texcoords.empty()) m.make_texcoords_normalized();
    out = std::move(m);
    return true;
}

// OBJ reader: positions/texcoords/normals with (v,vt,vn) de-duplication as the
// reference does over tinyobjloader output (src/runtime/mesh/ObjFile.cpp).
bool load_obj(const std::string& path, TriMesh& out, std::string& err) {
    std::ifstream in(path);
    if (!in) { err = "cannot open " + path; return false; }
    std::vector<V3> pos, nrm;
    std::vector<std::array<float, 2>> tex;
    std::map<std::tuple<int, int, int>, uint32_t> remap;
    TriMesh m;
    bool any_normal_missing = false;
    std::string line;
    auto fix_index = [](int i, size_t n) { return i < 0 ? (int)n + i : i - 1; };
    while (std::getline(in, line)) {
        std::istringstream ss(line);
        std::string tok;
        ss >> tok;
        if (tok == "v") { V3 p; ss >> p.x >> p.y >> p.z; pos.push_back(p); }
        else if (tok == "vn") { V3 p; ss >> p.x >> p.y >> p.z; nrm.push_back(p); }
        else if (tok == "vt") { std::array<float, 2> t{0, 0}; ss >> t[0] >> t[1]; tex.push_back(t); }
        else if (tok == "f") {
            std::vector<uint32_t> poly;
            std::string c;
            while (ss >> c) {
                int vi = 0, ti = 0, ni = 0;
                int parsed[3] = {0, 0, 0};
                int which = 0;
                std::string num;
                for (size_t k = 0; k <= c.size(); ++k) {
                    if (k == c.size() || c[k] == '/') {
                        if (!num.empty()) parsed[which] = std::stoi(num);
                        num.clear();
                        ++which;
                    } else {
                        num += c[k];
                    }
                }
                vi = fix_index(parsed[0], pos.size());
                ti = parsed[1] ? fix_index(parsed[1], tex.size()) : -1;
                ni = parsed[2] ? fix_index(parsed[2], nrm.size()) : -1;
                if (ni < 0) any_normal_missing = true;
                auto key = std::make_tuple(vi, ti, ni);
                auto it = remap.find(key);
                uint32_t id;
                if (it == remap.end()) {
                    id = (uint32_t)m.vertices.size();
                    remap[key] = id;
                    m.vertices.push_back(pos.at(vi));
                    m.normals.push_back(ni >= 0 ? nrm.at(ni) : V3());
                    m.texcoords.push_back(ti >= 0 ? tex.at(ti) : std::array<float, 2>{0, 0});
                } else {
                    id = it->second;
                }
                poly.push_back(id);
            }
            for (size_t k = 1; k + 1 < poly.size(); ++k) m.faces.push_back({poly[0], poly[k], poly[k + 1]});
        }
    }
    if (m.vertices.empty() || m.faces.empty()) { err = path + ": empty mesh"; return false; }
    if (any_normal_missing) m.compute_vertex_normals();
    else m.fix_normals(nullptr);
    out = std::move(m);
    return true;
}

} // namespace igx
