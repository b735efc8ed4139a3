// Scene JSON -> igx_scene_desc (Ignis schema subset used by the hot path).
//
// Stand-in for the reference loader chain, which cannot be built offline:
//   SceneParser (src/runtime/loader/Parser.cpp) -> LoaderShape/TriMeshProvider/
//   SphereProvider (src/runtime/shape/*.cpp) -> LoaderEntity
//   (src/runtime/loader/LoaderEntity.cpp:32-205) -> lights/BSDFs.
// Only the pieces the configs in BASELINE.json exercise are supported; anything
// else is rejected with a message instead of being silently approximated.
#include "igx_scene.h"

#include "json.h"
#include "linalg.h"
#include "mesh.h"
#include "scene_store.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <optional>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

using igx::BBox;
using igx::M4;
using igx::TriMesh;
using igx::V3;
using igx::json::Value;
using igx::SceneStore;

namespace {

constexpr float kPi = 3.14159265358979323846f;
constexpr float kDeg2Rad = kPi / 180.0f;

[[noreturn]] void fail(const std::string& m) { throw std::runtime_error(m); }

std::string read_file(const std::string& path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) fail("cannot open " + path);
    std::stringstream ss;
    ss << in.rdbuf();
    return ss.str();
}

std::string dir_of(const std::string& p) {
    auto pos = p.find_last_of('/');
    return pos == std::string::npos ? std::string(".") : p.substr(0, pos);
}

std::string join_path(const std::string& base, const std::string& rel) {
    if (rel.empty() || rel[0] == '/' || base.empty()) return rel;
    return base + "/" + rel;
}

// --- property access, after SceneProperty getters (Parser.cpp:281-312) ----
struct Props {
    const Value* v;
    const Value* get(const char* k) const { return v ? v->find(k) : nullptr; }
    bool has(const char* k) const { return get(k) != nullptr; }
    float number(const char* k, float def) const {
        const Value* p = get(k);
        if (!p) return def;
        if (p->is_number()) return (float)p->num;
        if (p->is_bool()) return p->b ? 1.f : 0.f;
        fail(std::string("property '") + k + "' is not a number");
    }
    int64_t integer(const char* k, int64_t def) const {
        const Value* p = get(k);
        if (!p) return def;
        if (p->is_number()) return (int64_t)p->num;
        if (p->is_bool()) return p->b ? 1 : 0;
        fail(std::string("property '") + k + "' is not an integer");
    }
    bool boolean(const char* k, bool def) const {
        const Value* p = get(k);
        if (!p) return def;
        if (p->is_bool()) return p->b;
        if (p->is_number()) return p->num != 0;
        fail(std::string("property '") + k + "' is not a bool");
    }
    std::string string(const char* k, const std::string& def = "") const {
        const Value* p = get(k);
        if (!p) return def;
        if (!p->is_string()) fail(std::string("property '") + k + "' is not a string");
        return p->str;
    }
    V3 vec3(const char* k, V3 def) const {
        const Value* p = get(k);
        if (!p) return def;
        if (p->is_number()) return V3((float)p->num, (float)p->num, (float)p->num);
        if (!p->is_array() || (p->arr.size() != 3 && p->arr.size() != 2)) fail(std::string("property '") + k + "' is not a vec3");
        V3 r;
        for (size_t i = 0; i < p->arr.size(); ++i) {
            if (!p->arr[i].is_number()) fail(std::string("property '") + k + "' has non-number entries");
            r[(int)i] = (float)p->arr[i].num;
        }
        return r;
    }
    // colour: a number is a grey value, an array an RGB triple; a string is a
    // shading expression (ShadingTree::computeColor, PExpr), accepted here in
    // its constant forms only -- a number, color(v), color(r, g, b) or
    // color(r, g, b, a) (alpha dropped) -- as Blender exports plain colours
    V3 color(const char* k, V3 def) const {
        const Value* p = get(k);
        if (!p || !p->is_string()) return vec3(k, def);
        V3 c;
        if (!constant_color(p->str, c))
            fail(std::string("property '") + k + "': shading expression '" + p->str +
                 "' is not a constant colour (shading networks are not supported)");
        return c;
    }
    static bool constant_color(const std::string& e, V3& out) {
        const char* s = e.c_str();
        auto ws = [&]() { while (*s == ' ' || *s == '\t') ++s; };
        auto num = [&](float& v) {
            ws();
            char* end = nullptr;
            v = std::strtof(s, &end);
            if (end == s) return false;
            s = end;
            return true;
        };
        ws();
        float v[4];
        int n = 0;
        if (std::strncmp(s, "color", 5) == 0) {
            s += 5;
            ws();
            if (*s++ != '(') return false;
            for (;;) {
                if (n == 4 || !num(v[n++])) return false;
                ws();
                if (*s == ',') { ++s; continue; }
                if (*s++ != ')') return false;
                break;
            }
            if (n == 2) return false;
        } else if (!num(v[n++])) {
            return false;
        }
        ws();
        if (*s) return false;
        out = n == 1 ? V3(v[0], v[0], v[0]) : V3(v[0], v[1], v[2]);
        return true;
    }
};

// select(checkerboard(uvw * S) == 1, A, B) with constant colours A and B (the
// form Blender's exporter writes for a checker texture; PExpr: Transpiler.cpp
// select / checkerboard / uvw, texture/checkerboard.art:1-2); false for any
// other expression
bool checker_expression(const std::string& expr, float& scale, V3& a, V3& b) {
    std::string e;
    for (char c : expr)
        if (c != ' ' && c != '\t' && c != '\n') e += c;
    const std::string head = "select(checkerboard(uvw*";
    if (e.compare(0, head.size(), head) != 0) return false;
    const char* s = e.c_str() + head.size();
    char* end = nullptr;
    scale = std::strtof(s, &end);
    if (end == s) return false;
    const std::string mid = ")==1,";
    if (std::strncmp(end, mid.c_str(), mid.size()) != 0) return false;
    const size_t p0 = (size_t)(end - e.c_str()) + mid.size();
    // A ends at the comma at parenthesis depth 0; B at the closing parenthesis of select
    int depth = 0;
    size_t comma = std::string::npos;
    for (size_t i = p0; i < e.size(); ++i) {
        if (e[i] == '(') ++depth;
        else if (e[i] == ')') {
            if (depth == 0) break;
            --depth;
        } else if (e[i] == ',' && depth == 0) {
            comma = i;
            break;
        }
    }
    if (comma == std::string::npos || e.back() != ')') return false;
    return Props::constant_color(e.substr(p0, comma - p0), a) &&
           Props::constant_color(e.substr(comma + 1, e.size() - comma - 2), b);
}

M4 matrix_from_array(const Value& a) {
    size_t n = a.arr.size();
    M4 m;
    if (n == 9) {
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) m.at(i, j) = (float)a.arr[i * 3 + j].num;
    } else if (n == 12 || n == 16) {
        int rows = n == 12 ? 3 : 4;
        for (int i = 0; i < rows; ++i)
            for (int j = 0; j < 4; ++j) m.at(i, j) = (float)a.arr[i * 4 + j].num;
    } else {
        fail("transform matrix must have 9, 12 or 16 entries");
    }
    return m;
}

// lookAt (Parser.cpp:137-162)
M4 look_at(V3 eye, V3 center, V3 up) {
    V3 f = igx::normalized(center - eye);
    if (igx::norm2(f) <= 1.1920928955e-07f) f = V3(0, 0, 1);
    V3 u = igx::normalized(up);
    V3 s = igx::normalized(igx::cross(f, u));
    u = igx::cross(s, f);
    if (igx::norm2(u) <= 1.1920928955e-07f) igx::tangent_frame(f, s, u);
    M4 m;
    for (int r = 0; r < 3; ++r) {
        m.at(r, 0) = s[r];
        m.at(r, 1) = u[r];
        m.at(r, 2) = f[r];
        m.at(r, 3) = eye[r];
    }
    return m;
}

// applyTransformProperty (Parser.cpp:164-226): ops right-multiply in order
void apply_ops(M4& t, const Value& obj) {
    for (auto& kv : obj.obj) {
        const std::string& k = kv.first;
        const Value& v = kv.second;
        auto vec = [&](const Value& a) {
            V3 r;
            if (!a.is_array() || (a.arr.size() != 3 && a.arr.size() != 2)) fail("transform op '" + k + "' expects a vector");
            for (size_t i = 0; i < a.arr.size(); ++i) r[(int)i] = (float)a.arr[i].num;
            return r;
        };
        if (k == "translate") {
            t = t * igx::translation(vec(v));
        } else if (k == "scale") {
            if (v.is_number()) t = t * igx::scaling(V3((float)v.num, (float)v.num, (float)v.num));
            else t = t * igx::scaling(vec(v));
        } else if (k == "rotate") {
            V3 a = vec(v);
            t = t * igx::axis_rotation(0, kDeg2Rad * a.x) * igx::axis_rotation(1, kDeg2Rad * a.y) * igx::axis_rotation(2, kDeg2Rad * a.z);
        } else if (k == "qrotate") {
            if (!v.is_array() || v.arr.size() != 4) fail("qrotate expects [w,x,y,z]");
            float w = (float)v.arr[0].num, x = (float)v.arr[1].num, y = (float)v.arr[2].num, z = (float)v.arr[3].num;
            float n = std::sqrt(w * w + x * x + y * y + z * z);
            w /= n; x /= n; y /= n; z /= n;
            M4 r;
            r.at(0, 0) = 1 - 2 * (y * y + z * z); r.at(0, 1) = 2 * (x * y - z * w); r.at(0, 2) = 2 * (x * z + y * w);
            r.at(1, 0) = 2 * (x * y + z * w); r.at(1, 1) = 1 - 2 * (x * x + z * z); r.at(1, 2) = 2 * (y * z - x * w);
            r.at(2, 0) = 2 * (x * z - y * w); r.at(2, 1) = 2 * (y * z + x * w); r.at(2, 2) = 1 - 2 * (x * x + y * y);
            t = t * r;
        } else if (k == "lookat") {
            V3 origin(0, 0, 0), target(0, 1, 0), up(0, 0, 1), dir;
            bool has_dir = false;
            for (auto& kv2 : v.obj) {
                if (kv2.first == "origin") origin = vec(kv2.second);
                else if (kv2.first == "target") target = vec(kv2.second);
                else if (kv2.first == "up") up = vec(kv2.second);
                else if (kv2.first == "direction") { dir = vec(kv2.second); has_dir = true; }
            }
            t = t * look_at(origin, has_dir ? dir + origin : target, up);
        } else if (k == "matrix") {
            t = t * matrix_from_array(v);
        } else {
            fail("unknown transform entry '" + k + "'");
        }
    }
}

M4 get_transform(const Props& p, const char* key = "transform") {
    const Value* v = p.get(key);
    M4 t;
    if (!v) return t;
    if (v->is_array()) {
        if (!v->arr.empty() && v->arr[0].is_object()) {
            for (auto& op : v->arr) apply_ops(t, op);
        } else {
            t = matrix_from_array(*v);
        }
    } else if (v->is_object()) {
        apply_ops(t, *v);
    } else {
        fail(std::string("invalid transform in '") + key + "'");
    }
    // Transformf::makeAffine: bottom row := 0 0 0 1 (LoaderEntity.cpp:134)
    t.at(3, 0) = t.at(3, 1) = t.at(3, 2) = 0;
    t.at(3, 3) = 1;
    return t;
}

// Scene-level merge of externals, as the reference parser does it:
// `InternalSceneParser::loadFromJSON` (Parser.cpp:450-459) loads every external
// first, each into its own Scene that `Scene::addFrom` (Scene.cpp:5-23) copies
// into the current one, replacing objects of the same name and taking the
// external's technique / camera / film (even an absent one); only then are the
// current file's own objects added (`handleNamedObject`, Parser.cpp:350-392),
// again replacing by name, and its camera / technique / film set.  Named
// objects keep the position of their first definition.  Each object remembers
// the directory of the file that defined it (`SceneObject::baseDir`), so mesh
// paths of an external resolve against the external's directory.
const char* const kNamedCategories[] = {"shapes", "textures", "bsdfs", "lights", "media", "entities"};
const char* const kAnonymous[] = {"camera", "technique", "film"};

void put_named(Value& list, const Value& obj) {
    const Value* nm = obj.find("name");
    if (!nm || !nm->is_string()) fail("named scene object without a string 'name'");
    for (auto& e : list.arr) {
        const Value* en = e.find("name");
        if (en && en->str == nm->str) {
            e = obj;
            return;
        }
    }
    list.arr.push_back(obj);
}

Value& category(Value& doc, const std::string& key) {
    for (auto& kv : doc.obj)
        if (kv.first == key) return kv.second;
    Value v;
    v.type = Value::Array;
    doc.obj.emplace_back(key, v);
    return doc.obj.back().second;
}

void set_key(Value& doc, const std::string& key, const Value* v) {
    for (auto it = doc.obj.begin(); it != doc.obj.end(); ++it)
        if (it->first == key) {
            doc.obj.erase(it);
            break;
        }
    if (v) doc.obj.emplace_back(key, *v);
}

// Scene::addFrom(other)
void add_from(Value& dst, const Value& src) {
    for (const char* cat : kNamedCategories)
        if (const Value* l = src.find(cat))
            for (auto& o : l->arr) put_named(category(dst, cat), o);
    for (const char* k : kAnonymous) set_key(dst, k, src.find(k));
}

Value load_document(const std::string& text, const std::string& base_dir, int depth = 0) {
    if (depth > 8) fail("externals nested too deep");
    Value doc = igx::json::parse(text);
    if (!doc.is_object()) fail("scene root must be an object");
    Value scene;
    scene.type = Value::Object;
    if (const Value* ext = doc.find("externals")) {
        if (!ext->is_array()) fail("externals must be an array");
        for (auto& e : ext->arr) {
            const Value* fn = e.find("filename");
            if (!fn || !fn->is_string()) fail("external without filename");
            std::string path = join_path(base_dir, fn->str);
            add_from(scene, load_document(read_file(path), dir_of(path), depth + 1));
        }
    }
    for (const char* k : kAnonymous)
        if (const Value* v = doc.find(k)) set_key(scene, k, v);
    for (const char* cat : kNamedCategories) {
        const Value* l = doc.find(cat);
        if (!l) continue;
        if (!l->is_array()) fail(std::string("'") + cat + "' must be an array");
        for (auto& o : l->arr) {
            if (!o.is_object()) fail(std::string("'") + cat + "' elements must be objects");
            Value obj = o;
            if (!obj.find("__base_dir")) {
                Value bd;
                bd.type = Value::String;
                bd.str = base_dir;
                obj.obj.emplace_back("__base_dir", bd);
            }
            put_named(category(scene, cat), obj);
        }
    }
    return scene;
}

const Value* array_of(const Value& doc, const char* key) {
    const Value* v = doc.find(key);
    if (v && !v->is_array()) fail(std::string("'") + key + "' must be an array");
    return v;
}

// --- bsdf parameter tables (src/runtime/bsdf/BSDF.cpp:7-51) ----------------
float dielectric_ior(const std::string& mat, const std::string& bsdf) {
    static const std::pair<const char*, float> table[] = {
        {"vacuum", 1.0f}, {"bk7", 1.5046f}, {"glass", 1.5046f}, {"helium", 1.00004f}, {"hydrogen", 1.00013f},
        {"air", 1.000277f}, {"water", 1.333f}, {"ethanol", 1.361f}, {"diamond", 2.419f}, {"polypropylene", 1.49f}};
    std::string l = mat;
    for (auto& c : l) c = (char)std::tolower(c);
    for (auto& e : table)
        if (l == e.first) return e.second;
    fail("bsdf '" + bsdf + "': unknown dielectric material '" + mat + "'");
}

void conductor_spec(const std::string& mat, const std::string& bsdf, V3& eta, V3& k) {
    struct Spec { const char* name; float eta[3], k[3]; };
    static const Spec table[] = {
        {"aluminum", {1.34560f, 0.96521f, 0.61722f}, {7.47460f, 6.39950f, 5.30310f}},
        {"brass", {0.44400f, 0.52700f, 1.09400f}, {3.69500f, 2.76500f, 1.82900f}},
        {"copper", {0.27105f, 0.67693f, 1.31640f}, {3.60920f, 2.62480f, 2.29210f}},
        {"gold", {0.18299f, 0.42108f, 1.37340f}, {3.4242f, 2.34590f, 1.77040f}},
        {"iron", {2.91140f, 2.94970f, 2.58450f}, {3.08930f, 2.93180f, 2.76700f}},
        {"lead", {1.91000f, 1.83000f, 1.44000f}, {3.51000f, 3.40000f, 3.18000f}},
        {"mercury", {2.07330f, 1.55230f, 1.06060f}, {5.33830f, 4.65100f, 3.86280f}},
        {"platinum", {2.37570f, 2.08470f, 1.84530f}, {4.26550f, 3.71530f, 3.13650f}},
        {"silver", {0.15943f, 0.14512f, 0.13547f}, {3.92910f, 3.19000f, 2.38080f}},
        {"titanium", {2.74070f, 2.54180f, 2.26700f}, {3.81430f, 3.43450f, 3.03850f}},
        {"none", {0.0f, 0.0f, 0.0f}, {1.0f, 1.0f, 1.0f}}};
    std::string l = mat;
    for (auto& c : l) c = (char)std::tolower(c);
    for (auto& e : table)
        if (l == e.name) {
            eta = V3(e.eta[0], e.eta[1], e.eta[2]);
            k = V3(e.k[0], e.k[1], e.k[2]);
            return;
        }
    fail("bsdf '" + bsdf + "': unknown conductor material '" + mat + "'");
}

// BSDF::setupRoughness (BSDF.cpp:53-99) and microfacet::compute_explicit
// (core/microfacet.art:395-402): no roughness property -> delta lobe.
void setup_roughness(const Props& bp, igx_material& m) {
    const bool old = bp.has("alpha") || bp.has("alpha_u") || bp.has("alpha_v");
    const std::string p = old ? "alpha" : "roughness";
    const std::string pu = p + "_u", pv = p + "_v";
    if (!bp.has(p.c_str()) && !bp.has(pu.c_str()) && !bp.has(pv.c_str())) {
        m.distribution = IGX_MICROFACET_DELTA;
        return;
    }
    std::string dist = bp.string("distribution", "");
    m.distribution = dist == "ggx" ? IGX_MICROFACET_GGX : dist == "beckmann" ? IGX_MICROFACET_BECKMANN : IGX_MICROFACET_VNDF_GGX;
    if (bp.has(pu.c_str()) || bp.has(pv.c_str())) {
        m.alpha_u = bp.number(pu.c_str(), 0.1f);
        m.alpha_v = bp.number(pv.c_str(), 0.1f);
    } else {
        float r = bp.number(p.c_str(), 0.1f), an = bp.number("anisotropic", 0.0f);
        float aspect = an == 0.0f ? 1.0f : std::sqrt(1 - std::min(std::max(an, 0.0f), 1.0f) * 0.99f);
        m.alpha_u = r / aspect;
        m.alpha_v = r * aspect;
    }
}

// --- shapes -------------------------------------------------------------
struct LoadedShape {
    igx_shape shape{};
    TriMesh mesh;
    bool is_mesh = false;
};

TriMesh setup_trimesh(const std::string& type, const Props& p, const std::string& base_dir, const std::string& name) {
    TriMesh m;
    std::string err;
    if (type == "triangle") {
        m = igx::make_triangle(p.vec3("p0", V3(0, 0, 0)), p.vec3("p1", V3(1, 0, 0)), p.vec3("p2", V3(0, 1, 0)));
    } else if (type == "rectangle") {
        if (!p.has("p0")) {
            float w = p.number("width", 2.0f), h = p.number("height", 2.0f);
            V3 o = p.vec3("origin", V3(-w / 2, -h / 2, 0));
            m = igx::make_plane(o, V3(w, 0, 0), V3(0, h, 0));
        } else {
            m = igx::make_rectangle(p.vec3("p0", V3(-1, -1, 0)), p.vec3("p1", V3(1, -1, 0)), p.vec3("p2", V3(1, 1, 0)), p.vec3("p3", V3(-1, 1, 0)));
        }
    } else if (type == "cube" || type == "box") {
        float w = p.number("width", 2.0f), h = p.number("height", 2.0f), d = p.number("depth", 2.0f);
        V3 o = p.vec3("origin", V3(-w / 2, -h / 2, -d / 2));
        m = igx::make_box(o, V3(w, 0, 0), V3(0, h, 0), V3(0, 0, d));
    } else if (type == "icosphere") {
        m = igx::make_ico_sphere(p.vec3("center", V3()), p.number("radius", 1.0f), (uint32_t)p.integer("subdivisions", 4));
    } else if (type == "uvsphere") {
        m = igx::make_uv_sphere(p.vec3("center", V3()), p.number("radius", 1.0f), (uint32_t)p.integer("stacks", 32), (uint32_t)p.integer("slices", 16));
    } else if (type == "cylinder") {
        float br, tr;
        if (p.has("radius")) { br = tr = p.number("radius", 1.0f); }
        else { br = p.number("bottom_radius", 1.0f); tr = p.number("top_radius", br); }
        m = igx::make_cylinder(p.vec3("p0", V3()), br, p.vec3("p1", V3(0, 0, 1)), tr, (uint32_t)p.integer("sections", 32), p.boolean("filled", true));
    } else if (type == "cone") {
        m = igx::make_cone(p.vec3("p0", V3()), p.number("radius", 1.0f), p.vec3("p1", V3(0, 0, 1)), (uint32_t)p.integer("sections", 32), p.boolean("filled", true));
    } else if (type == "disk") {
        m = igx::make_disk(p.vec3("origin", V3()), p.vec3("normal", V3(0, 0, 1)), p.number("radius", 1.0f), (uint32_t)p.integer("sections", 32));
    } else if (type == "soup") {
        // igx extension: synthetic triangle soup of the benchmark suite
        int64_t cnt = p.integer("count", 1000000);
        if (cnt < 1 || cnt >= (1ll << 26)) fail("shape '" + name + "': soup count must be in [1, 2^26)");
        m = igx::make_soup((uint32_t)cnt, (uint64_t)p.integer("seed", 42));
    } else if (type == "displaced_grid") {
        // igx extension: value-noise height field of the S-deep scene
        m = igx::make_displaced_grid((uint32_t)p.integer("quads", 256), p.number("size", 2.0f), p.number("amplitude", 0.25f),
                                     (uint64_t)p.integer("seed", 7));
    } else if (type == "ply" || type == "obj" || type == "external") {
        std::string fn = join_path(base_dir, p.string("filename"));
        std::string ext = fn.size() >= 4 ? fn.substr(fn.size() - 4) : "";
        for (auto& c : ext) c = (char)std::tolower(c);
        bool ok;
        if (type == "ply" || (type == "external" && ext == ".ply")) ok = igx::load_ply(fn, m, err);
        else if (type == "obj" || (type == "external" && ext == ".obj")) ok = igx::load_obj(fn, m, err);
        else fail("shape '" + name + "': cannot determine mesh type of " + fn);
        if (!ok) fail("shape '" + name + "': " + err);
    } else {
        fail("shape '" + name + "': unsupported shape type '" + type + "'");
    }
    if (m.vertices.empty() || m.faces.empty()) fail("shape '" + name + "': no geometry generated");

    // User options (TriMeshProvider.cpp:528-541)
    if (p.boolean("flip_normals", false)) m.flip_normals();
    if (p.boolean("face_normals", false)) m.setup_face_normals_as_vertex_normals();
    else if (p.boolean("smooth_normals", false)) m.compute_vertex_normals();
    if (p.boolean("generic_uv", false)) m.make_texcoords_normalized();
    M4 t = get_transform(p);
    if (!t.is_identity()) m.transform(t);
    if (m.texcoords.size() != m.vertices.size()) m.make_texcoords_normalized();
    return m;
}

} // namespace

static void build_scene(SceneStore& S, const Value& doc, const std::string& base_dir) {
    // ---- film (Runtime.cpp:28-44) ----
    S.desc.film_width = 800;
    S.desc.film_height = 600;
    if (const Value* film = doc.find("film")) {
        Props fp{film};
        if (const Value* sz = fp.get("size")) {
            if (!sz->is_array() || sz->arr.size() != 2) fail("film.size must be [w, h]");
            S.desc.film_width = std::max(1, (int)sz->arr[0].num);
            S.desc.film_height = std::max(1, (int)sz->arr[1].num);
        }
    }

    // ---- technique (PathTechnique.cpp:8-17) ----
    igx_technique tech{64, 2, 0.0f, 1, IGX_SELECT_UNIFORM, 0};
    if (const Value* t = doc.find("technique")) {
        Props tp{t};
        std::string type = tp.string("type", "path");
        if (type != "path") fail("unsupported technique '" + type + "' (only 'path' is on the hot path)");
        tech.max_depth = tp.integer("max_depth", 64);
        tech.min_depth = tp.integer("min_depth", 2);
        tech.clamp = tp.number("clamp", 0.0f);
        tech.nee = tp.boolean("nee", true) ? 1 : 0;
        tech.aov_mis = tp.boolean("aov_mis", false) ? 1 : 0; // "Direct Weights" / "NEE Weights" (PathTechnique.cpp:16-27)
        // PathTechnique.cpp (light_selector) -> LoaderLight::generateLightSelector (LoaderLight.cpp:423-453):
        // "hierarchy" and "simple" select their sampler, anything else is the uniform selector
        const std::string sel = tp.string("light_selector", "");
        tech.light_selector = sel == "hierarchy" ? IGX_SELECT_HIERARCHY : sel == "simple" ? IGX_SELECT_SIMPLE : IGX_SELECT_UNIFORM;
    }
    S.desc.technique = tech;

    // ---- bsdfs ----
    std::unordered_map<std::string, igx_material> bsdfs;
    if (const Value* arr = array_of(doc, "bsdfs")) {
        for (auto& b : arr->arr) {
            Props bp{&b};
            std::string name = bp.string("name");
            std::string type = bp.string("type");
            igx_material m{};
            m.light = -1;
            m.ext_ior = 1.0f;
            m.int_ior = 1.5046f;
            m.kd[0] = m.kd[1] = m.kd[2] = 0.8f;
            for (int i = 0; i < 3; ++i) m.ks[i] = m.kt[i] = 1.0f;
            if (type == "diffuse" || type == "roughdiffuse") {
                m.bsdf_type = IGX_BSDF_DIFFUSE;
                V3 kd, kd1;
                float scale = 0;
                const Value* refl = bp.get("reflectance");
                if (refl && refl->is_string() && checker_expression(refl->str, scale, kd1, kd)) {
                    // the Blender exporter's checker texture (igx_material::texture)
                    m.texture = IGX_TEXTURE_CHECKER;
                    m.tex_scale = scale;
                    m.tex_kd1[0] = kd1.x; m.tex_kd1[1] = kd1.y; m.tex_kd1[2] = kd1.z;
                } else {
                    kd = bp.color("reflectance", V3(0.8f, 0.8f, 0.8f)); // DiffuseBSDF.cpp:17
                }
                m.kd[0] = kd.x; m.kd[1] = kd.y; m.kd[2] = kd.z;
                m.diffuse_alpha = bp.number(bp.has("alpha") ? "alpha" : "roughness", 0.0f); // Oren-Nayar above flt_eps
            } else if (type == "dielectric" || type == "glass") {
                m.bsdf_type = IGX_BSDF_DIELECTRIC; // DielectricBSDF.cpp:12-38
                V3 ks = bp.color("specular_reflectance", V3(1, 1, 1));
                V3 kt = bp.color("specular_transmittance", V3(1, 1, 1));
                m.ks[0] = ks.x; m.ks[1] = ks.y; m.ks[2] = ks.z;
                m.kt[0] = kt.x; m.kt[1] = kt.y; m.kt[2] = kt.z;
                m.ext_ior = bp.number("ext_ior", dielectric_ior(bp.string("ext_ior_material", "vacuum"), name));
                m.int_ior = bp.number("int_ior", dielectric_ior(bp.string("int_ior_material", "bk7"), name));
                m.thin = bp.boolean("thin", false) ? 1 : 0;
                if (bp.number("roughness", 0.0f) > 0.0f || bp.number("roughness_u", 0.0f) > 0.0f || bp.number("roughness_v", 0.0f) > 0.0f)
                    fail("bsdf '" + name + "': rough dielectric is not supported");
            } else if (type == "conductor" || type == "roughconductor" || type == "mirror") {
                // ConductorBSDF.cpp:12-33; material table BSDF.cpp:30-51 (default "none": eta 0, k 1)
                m.bsdf_type = IGX_BSDF_CONDUCTOR;
                V3 ks = bp.color("specular_reflectance", V3(1, 1, 1));
                m.ks[0] = ks.x; m.ks[1] = ks.y; m.ks[2] = ks.z;
                V3 eta(0, 0, 0), k(1, 1, 1);
                conductor_spec(bp.string("material", "none"), name, eta, k);
                eta = bp.color("eta", eta);
                k = bp.color("k", k);
                for (int c = 0; c < 3; ++c) { m.eta[c] = eta[c]; m.kappa[c] = k[c]; }
                setup_roughness(bp, m);
            } else if (type == "plastic" || type == "roughplastic") {
                // PlasticBSDF.cpp:12-46
                m.bsdf_type = IGX_BSDF_PLASTIC;
                V3 ks = bp.color("specular_reflectance", V3(1, 1, 1));
                V3 kd = bp.color("diffuse_reflectance", V3(0.8f, 0.8f, 0.8f));
                m.ks[0] = ks.x; m.ks[1] = ks.y; m.ks[2] = ks.z;
                m.kd[0] = kd.x; m.kd[1] = kd.y; m.kd[2] = kd.z;
                m.ext_ior = bp.number("ext_ior", dielectric_ior(bp.string("ext_ior_material", "vacuum"), name));
                m.int_ior = bp.number("int_ior", dielectric_ior(bp.string("int_ior_material", "polypropylene"), name));
                for (int c = 0; c < 3; ++c) { m.eta[c] = 0; m.kappa[c] = 1; }
                setup_roughness(bp, m);
            } else if (type == "principled") {
                // PrincipledBSDF::serialize (PrincipledBSDF.cpp:11-60)
                m.bsdf_type = IGX_BSDF_PRINCIPLED;
                V3 base = bp.color("base_color", V3(0.8f, 0.8f, 0.8f));
                m.kd[0] = base.x; m.kd[1] = base.y; m.kd[2] = base.z;
                const std::string ior_mat = bp.string("ior_material", "");
                m.ior = bp.number("ior", dielectric_ior(ior_mat.empty() ? "bk7" : ior_mat, name));
                m.diffuse_transmission = bp.number("diffuse_transmission", 0.0f);
                m.specular_transmission = bp.number("specular_transmission", 0.0f);
                m.specular_tint = bp.number("specular_tint", 0.0f);
                if (bp.has("roughness_u") || bp.has("roughness_v")) {
                    m.alpha_u = bp.number("roughness_u", 0.5f);
                    m.alpha_v = bp.number("roughness_v", 0.5f);
                } else {
                    // principled::compute_roughness (bsdf/principled.art:57-62)
                    float r = bp.number("roughness", 0.5f), an = bp.number("anisotropic", 0.0f);
                    float aspect = an == 0.0f ? 1.0f : std::sqrt(1 - std::min(std::max(an, 0.0f), 1.0f) * 0.9f);
                    m.alpha_u = r * r / aspect;
                    m.alpha_v = r * r * aspect;
                }
                m.distribution = IGX_MICROFACET_VNDF_GGX;
                m.flatness = bp.number("flatness", 0.0f);
                m.metallic = bp.number("metallic", 0.0f);
                m.sheen = bp.number("sheen", 0.0f);
                m.sheen_tint = bp.number("sheen_tint", 0.0f);
                m.clearcoat = bp.number("clearcoat", 0.0f);
                m.clearcoat_gloss = bp.number("clearcoat_gloss", 0.0f);
                m.clearcoat_roughness = bp.number("clearcoat_roughness", 0.1f);
                m.thin = bp.boolean("thin", false) ? 1 : 0;
                m.clearcoat_top_only = bp.boolean("clearcoat_top_only", true) ? 1 : 0;
            } else {
                fail("bsdf '" + name + "': unsupported bsdf type '" + type + "'");
            }
            bsdfs[name] = m;
        }
    }

    // ---- shapes ----
    std::unordered_map<std::string, int> shape_ids;
    std::vector<LoadedShape> shapes;
    if (const Value* arr = array_of(doc, "shapes")) {
        for (auto& s : arr->arr) {
            Props sp{&s};
            std::string name = sp.string("name");
            std::string type = sp.string("type");
            LoadedShape ls;
            if (type == "sphere") {
                // SphereProvider::handle (SphereProvider.cpp:10-53)
                V3 o = sp.vec3("center", V3());
                float r = sp.number("radius", 1.0f);
                if (r <= 0) fail("shape '" + name + "': invalid sphere radius");
                ls.shape.type = IGX_SHAPE_SPHERE;
                ls.shape.mesh = -1;
                ls.shape.sphere[0] = o.x; ls.shape.sphere[1] = o.y; ls.shape.sphere[2] = o.z; ls.shape.sphere[3] = r;
                BBox b;
                b.extend(o + V3(r, 0, 0)); b.extend(o - V3(r, 0, 0));
                b.extend(o + V3(0, r, 0)); b.extend(o - V3(0, r, 0));
                b.extend(o + V3(0, 0, r)); b.extend(o - V3(0, 0, r));
                b.inflate(1e-5f);
                for (int i = 0; i < 3; ++i) { ls.shape.bbox_min[i] = b.min[i]; ls.shape.bbox_max[i] = b.max[i]; }
            } else {
                const Value* obj_dir = s.find("__base_dir");
                ls.mesh = setup_trimesh(type, sp, obj_dir && obj_dir->is_string() ? obj_dir->str : base_dir, name);
                ls.is_mesh = true;
                ls.shape.type = IGX_SHAPE_TRIMESH;
                BBox b = ls.mesh.compute_bbox();
                b.inflate(1e-5f); // TriMeshProvider.cpp:537-538
                for (int i = 0; i < 3; ++i) { ls.shape.bbox_min[i] = b.min[i]; ls.shape.bbox_max[i] = b.max[i]; }
                if (auto pl = igx::get_as_plane(ls.mesh)) {
                    ls.shape.is_plane = 1;
                    for (int i = 0; i < 3; ++i) {
                        ls.shape.plane_origin[i] = pl->origin[i];
                        ls.shape.plane_x[i] = pl->x_axis[i];
                        ls.shape.plane_y[i] = pl->y_axis[i];
                    }
                    for (int i = 0; i < 8; ++i) ls.shape.plane_tex[i] = pl->tex[i];
                }
            }
            if (shape_ids.count(name)) fail("duplicate shape name '" + name + "'");
            shape_ids[name] = (int)shapes.size();
            shapes.push_back(std::move(ls));
        }
    }
    // ---- lights: find area-light entities first (LoaderEntity.cpp:82-84) ----
    std::unordered_map<std::string, const Value*> area_light_of_entity;
    const Value* lights_arr = array_of(doc, "lights");
    if (lights_arr)
        for (auto& l : lights_arr->arr) {
            Props lp{&l};
            if (lp.string("type") == "area") area_light_of_entity[lp.string("entity")] = &l;
        }

    // ---- entities, grouped by material in first-appearance order (LoaderEntity.cpp:42-103) ----
    struct MatKey { std::string bsdf; std::string light_entity; };
    std::vector<MatKey> mat_keys;
    std::vector<std::vector<const Value*>> groups;
    if (const Value* arr = array_of(doc, "entities")) {
        for (auto& e : arr->arr) {
            Props ep{&e};
            std::string bsdf = ep.string("bsdf");
            std::string name = ep.string("name");
            if (bsdf.empty()) fail("entity '" + name + "' has no bsdf");
            if (!bsdfs.count(bsdf)) fail("entity '" + name + "' has unknown bsdf '" + bsdf + "'");
            if (area_light_of_entity.count(name)) {
                mat_keys.push_back({bsdf, name});
                groups.push_back({&e});
            } else {
                size_t k = 0;
                for (; k < mat_keys.size(); ++k)
                    if (mat_keys[k].bsdf == bsdf && mat_keys[k].light_entity.empty()) break;
                if (k == mat_keys.size()) { mat_keys.push_back({bsdf, ""}); groups.push_back({}); }
                groups[k].push_back(&e);
            }
        }
    }
    BBox scene_bbox;
    std::unordered_map<std::string, int> entity_ids;
    for (size_t mid = 0; mid < groups.size(); ++mid) {
        igx_material m = bsdfs[mat_keys[mid].bsdf];
        m.light = -1;
        S.materials.push_back(m);
        S.material_bsdf.push_back(mat_keys[mid].bsdf);
        S.material_entity.push_back(mat_keys[mid].light_entity);
        for (const Value* e : groups[mid]) {
            Props ep{e};
            std::string name = ep.string("name");
            std::string shape = ep.string("shape");
            if (!shape_ids.count(shape)) fail("entity '" + name + "' has unknown shape '" + shape + "'");
            int sid = shape_ids[shape];
            igx_entity ent{};
            ent.shape = sid;
            ent.material = (int)mid;
            uint32_t flags = 0;
            if (ep.boolean("camera_visible", true)) flags |= 0x1;
            if (ep.boolean("light_visible", true)) flags |= 0x2;
            if (ep.boolean("bounce_visible", true)) flags |= 0x4;
            if (ep.boolean("shadow_visible", true)) flags |= 0x8;
            ent.flags = flags;
            M4 t = get_transform(ep);
            M4 inv = igx::affine_inverse(t);
            igx::M3 nm = igx::transpose3(igx::inverse3(igx::linear_of(t)));
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 4; ++c) { ent.to_global[r * 4 + c] = t.at(r, c); ent.to_local[r * 4 + c] = inv.at(r, c); }
            for (int i = 0; i < 9; ++i) ent.normal[i] = nm.m[i];
            // BoundingBox::transformed (math/BoundingBox.h:84-95)
            const igx_shape& sh = shapes[sid].shape;
            BBox eb;
            for (int c = 0; c < 8; ++c) {
                V3 p((c & 1) ? sh.bbox_max[0] : sh.bbox_min[0], (c & 2) ? sh.bbox_max[1] : sh.bbox_min[1], (c & 4) ? sh.bbox_max[2] : sh.bbox_min[2]);
                eb.extend(igx::xform_point(t, p));
            }
            for (int i = 0; i < 3; ++i) { ent.bbox_min[i] = eb.min[i]; ent.bbox_max[i] = eb.max[i]; }
            scene_bbox.extend(eb);
            entity_ids[name] = (int)S.entities.size();
            S.entity_names.push_back(name);
            S.entities.push_back(ent);
        }
    }

    // ---- lights ----
    if (lights_arr) {
        for (auto& l : lights_arr->arr) {
            Props lp{&l};
            std::string type = lp.string("type");
            std::string name = lp.string("name");
            igx_light L{};
            L.entity = -1;
            if (type == "area") {
                std::string ename = lp.string("entity");
                if (!entity_ids.count(ename)) fail("area light '" + name + "': no entity named '" + ename + "'");
                int eid = entity_ids[ename];
                const igx_entity& ent = S.entities[eid];
                const igx_shape& sh = shapes[ent.shape].shape;
                M4 t;
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 4; ++c) t.at(r, c) = ent.to_global[r * 4 + c];
                // AreaLight::AreaLight (AreaLight.cpp:38-99): choose the emitter representation
                const bool is_tri = sh.type == IGX_SHAPE_TRIMESH;
                const bool opt = lp.boolean("optimize", true) || !is_tri;
                std::optional<igx::SphereShape> sphere;
                if (sh.type == IGX_SHAPE_SPHERE) sphere = igx::SphereShape{V3(sh.sphere[0], sh.sphere[1], sh.sphere[2]), sh.sphere[3]};
                else if (!sh.is_plane) sphere = igx::get_as_sphere(shapes[ent.shape].mesh); // TriMeshProvider.cpp:563, 604-611
                auto scaled_len = [&](V3 axis) { return igx::norm(igx::xform_dir(t, axis)); };
                float host_area; // AreaLight::mArea, used by 'power'
                L.entity = eid;
                if (opt && sh.is_plane) {
                    // AreaLight.cpp:59-70, 129-145: make_plane_area_emitter
                    V3 o = igx::xform_point(t, V3(sh.plane_origin[0], sh.plane_origin[1], sh.plane_origin[2]));
                    V3 xa = igx::xform_dir(t, V3(sh.plane_x[0], sh.plane_x[1], sh.plane_x[2]));
                    V3 ya = igx::xform_dir(t, V3(sh.plane_y[0], sh.plane_y[1], sh.plane_y[2]));
                    V3 n = igx::normalized(igx::cross(xa, ya));
                    L.type = IGX_LIGHT_PLANE;
                    for (int i = 0; i < 3; ++i) { L.origin[i] = o[i]; L.x_axis[i] = xa[i]; L.y_axis[i] = ya[i]; L.normal[i] = n[i]; }
                    L.area = igx::norm(igx::cross(xa, ya));
                    host_area = L.area;
                    // AreaLight.cpp:66-69: position at the plane's centre, direction its normal
                    const V3 c = o + xa * 0.5f + ya * 0.5f;
                    for (int i = 0; i < 3; ++i) { L.select_position[i] = c[i]; L.select_direction[i] = n[i]; }
                    L.select_has_direction = 1;
                } else if (opt && sphere) {
                    // AreaLight.cpp:71-79, 146-152: make_sphere_area_emitter; the emitter's own
                    // area is compute_ellipsoid_area (shapes/sphere.art:21-27, P = 1.6)
                    const float r = sphere->radius;
                    float l1 = scaled_len(V3(r, 0, 0)), l2 = scaled_len(V3(0, r, 0)), l3 = scaled_len(V3(0, 0, r));
                    auto ellipsoid = [&](float P) {
                        return 4 * 3.14159265358979f *
                               std::pow((std::pow(l1 * l2, P) + std::pow(l1 * l3, P) + std::pow(l2 * l3, P)) / 3, 1 / P);
                    };
                    L.type = IGX_LIGHT_SPHERE;
                    for (int i = 0; i < 3; ++i) L.origin[i] = sphere->origin[i];
                    L.radius = r;
                    L.area = ellipsoid(1.6f);
                    host_area = ellipsoid(1.6075f); // approximate_ellipsoid_area (AreaLight.cpp:24-33)
                    const V3 c = igx::xform_point(t, sphere->origin); // AreaLight.cpp:74-77
                    for (int i = 0; i < 3; ++i) L.select_position[i] = c[i];
                } else if (is_tri) {
                    // AreaLight.cpp:80-90, 153-168: make_shape_area_emitter over the mesh
                    const igx::TriMesh& mesh = shapes[ent.shape].mesh;
                    if (mesh.face_count() == 0) fail("area light '" + name + "': entity '" + ename + "' has no faces");
                    L.type = IGX_LIGHT_MESH;
                    // approximate_area_scale (AreaLight.cpp:11-22) over the shape's bbox
                    V3 ls(sh.bbox_max[0] - sh.bbox_min[0], sh.bbox_max[1] - sh.bbox_min[1], sh.bbox_max[2] - sh.bbox_min[2]);
                    float w = scaled_len(V3(ls.x, 0, 0)), h = scaled_len(V3(0, ls.y, 0)), d = scaled_len(V3(0, 0, ls.z));
                    float half_area = ls.x * (ls.y + ls.z) + ls.y * ls.z;
                    host_area = igx::compute_area(mesh) * ((w * h + w * d + h * d) / half_area);
                    // AreaLight.cpp:84-86: the transformed bbox centre
                    const V3 c = igx::xform_point(t, V3((sh.bbox_min[0] + sh.bbox_max[0]) / 2, (sh.bbox_min[1] + sh.bbox_max[1]) / 2,
                                                        (sh.bbox_min[2] + sh.bbox_max[2]) / 2));
                    for (int i = 0; i < 3; ++i) L.select_position[i] = c[i];
                } else {
                    fail("area light '" + name + "': entity '" + ename + "' is not triangular");
                }
                V3 rad;
                if (lp.has("power")) {
                    // AreaLight::serialize (AreaLight.cpp:176-179): power * (inv_pi / area), the area
                    // printed into the generated shader at default stream precision
                    char buf[64];
                    std::snprintf(buf, sizeof(buf), "%g", (double)host_area);
                    const float area_code = std::strtof(buf, nullptr);
                    rad = lp.color("power", V3(1, 1, 1)) * (0.318309886183791f / area_code);
                } else {
                    rad = lp.color("radiance", V3(1, 1, 1));
                }
                for (int i = 0; i < 3; ++i) L.radiance[i] = rad[i];
                // AreaLight::precompute / computeFlux (AreaLight.cpp:99-113): mean of the power colour
                const V3 pw = lp.has("power") ? lp.color("power", V3(1, 1, 1)) : lp.color("radiance", V3(1, 1, 1)) * (host_area * kPi);
                L.select_flux = (pw.x + pw.y + pw.z) / 3;
                S.materials[ent.material].light = (int)S.lights.size();
            } else if (type == "env" || type == "constant" || type == "uniform") {
                // EnvironmentLight.cpp:28-78: constant radiance bakes to a 1x1 texture -> make_environment_light
                // a constant colour expression is accepted (Props::color); an image or
                // a varying expression is a textured environment (not supported).
                // The light's transform only rotates the texture lookup: without
                // effect on a constant environment
                V3 rad = lp.color("radiance", V3(1, 1, 1));
                V3 scale = lp.color("scale", V3(1, 1, 1));
                L.type = IGX_LIGHT_ENV;
                for (int i = 0; i < 3; ++i) L.radiance[i] = rad[i] * scale[i];
            } else if (type == "point") {
                V3 pos = lp.vec3("position", V3());
                // PointLight.cpp:16-30, 61-69: with `power` the intensity is power / (4 pi)
                // (the embedded SimplePointLight's mColor_Cache / SR), the flux the power
                const bool power = lp.has("power");
                const V3 pw = power ? lp.color("power", V3(1, 1, 1)) : lp.color("intensity", V3(1, 1, 1)) * (4 * kPi);
                const V3 I = power ? pw / (4 * kPi) : lp.color("intensity", V3(1, 1, 1));
                L.type = IGX_LIGHT_POINT;
                for (int i = 0; i < 3; ++i) { L.origin[i] = pos[i]; L.radiance[i] = I[i]; L.select_position[i] = pos[i]; }
                L.select_flux = (pw.x + pw.y + pw.z) / 3;
            } else if (type == "spot") {
                if (lp.has("power")) fail("spot light '" + name + "': 'power' is not supported");
                V3 pos = lp.vec3("position", V3());
                V3 dir = igx::normalized(lp.vec3("direction", V3(0, 0, 1)));
                V3 I = lp.color("intensity", V3(1, 1, 1));
                L.type = IGX_LIGHT_SPOT;
                for (int i = 0; i < 3; ++i) { L.origin[i] = pos[i]; L.normal[i] = dir[i]; L.radiance[i] = I[i]; }
                L.cutoff = lp.number("cutoff", 30.0f) * kDeg2Rad;
                L.falloff = lp.number("falloff", 20.0f) * kDeg2Rad;
                // SpotLight.cpp:17-38: flux = mean(intensity) * 2 pi (1 - (cos cutoff + cos falloff) / 2)
                const V3 pw = I * (2 * kPi * (1 - 0.5f * (std::cos(L.cutoff) + std::cos(L.falloff))));
                L.select_flux = (pw.x + pw.y + pw.z) / 3;
                for (int i = 0; i < 3; ++i) { L.select_position[i] = pos[i]; L.select_direction[i] = dir[i]; }
                L.select_has_direction = 1;
            } else if (type == "directional" || type == "sun") {
                // DirectionalLight.cpp:20-32, SunLight.cpp:24-46; direction via
                // LoaderUtils::getEA(...).toDirectionYUp() (LoaderUtils.cpp:140-156)
                V3 dir;
                if (lp.has("direction") || lp.has("sun_direction")) {
                    V3 d = igx::normalized(lp.vec3(lp.has("direction") ? "direction" : "sun_direction", V3(0, 0, 1)));
                    float theta = std::acos(d.y), phi = std::atan2(d.x, -d.z); // ElevationAzimuth::fromDirectionYUp
                    float el = 1.57079632679f - theta, az = phi < 0 ? phi + 6.28318530718f : phi;
                    dir = V3(std::cos(el) * std::sin(az), std::sin(el), -std::cos(el) * std::cos(az));
                } else if (lp.has("elevation") || lp.has("azimuth")) {
                    float el = lp.number("elevation", 0.0f), az = lp.number("azimuth", 0.0f);
                    dir = V3(std::cos(el) * std::sin(az), std::sin(el), -std::cos(el) * std::cos(az));
                } else {
                    fail("light '" + name + "': give 'direction', 'sun_direction' or 'elevation'/'azimuth' (time/location sun positions are not supported)");
                }
                V3 E = lp.color("irradiance", V3(1, 1, 1));
                L.type = type == "sun" ? IGX_LIGHT_SUN : IGX_LIGHT_DIRECTIONAL;
                for (int i = 0; i < 3; ++i) { L.normal[i] = dir[i]; L.radiance[i] = E[i]; }
                if (type == "sun")
                    L.cutoff = lp.has("radius") ? 1 / std::sqrt(lp.number("radius", 1.0f) * lp.number("radius", 1.0f) + 1) // sun_cos_angle_from_radius
                                                : std::cos(lp.number("angle", 11.4f) * kDeg2Rad / 2);
            } else {
                fail("light '" + name + "': unsupported light type '" + type + "'");
            }
            S.lights.push_back(L);
        }
    }

    // ---- meshes into flat arrays ----
    for (auto& ls : shapes) {
        if (ls.is_mesh) {
            ls.shape.mesh = (int)S.vtx.size();
            std::vector<float> v, n, t;
            std::vector<uint32_t> ix;
            v.reserve(ls.mesh.vertices.size() * 3);
            for (auto& p : ls.mesh.vertices) { v.push_back(p.x); v.push_back(p.y); v.push_back(p.z); }
            for (auto& p : ls.mesh.normals) { n.push_back(p.x); n.push_back(p.y); n.push_back(p.z); }
            for (auto& p : ls.mesh.texcoords) { t.push_back(p[0]); t.push_back(p[1]); }
            for (auto& f : ls.mesh.faces) { ix.push_back(f[0]); ix.push_back(f[1]); ix.push_back(f[2]); }
            S.vtx.push_back(std::move(v));
            S.nrm.push_back(std::move(n));
            S.tex.push_back(std::move(t));
            S.idx.push_back(std::move(ix));
        }
        S.shapes.push_back(ls.shape);
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

    // ---- camera (PerspectiveCamera.cpp, Camera.cpp:5-15) ----
    igx_camera cam{};
    cam.fov = 60.0f * kDeg2Rad;
    cam.vertical_fov = 0;
    cam.aspect = -1.0f;
    cam.near_clip = 0.0f;
    cam.far_clip = 3.4028234664e+38f;
    const Value* camv = doc.find("camera");
    Props cp{camv};
    if (camv) {
        std::string type = cp.string("type", "perspective");
        if (type != "perspective") fail("unsupported camera type '" + type + "'");
        if (cp.has("vfov")) { cam.vertical_fov = 1; cam.fov = cp.number("vfov", 60) * kDeg2Rad; }
        else if (cp.has("hfov")) cam.fov = cp.number("hfov", 60) * kDeg2Rad;
        else cam.fov = cp.number("fov", 60) * kDeg2Rad;
        if (cp.has("aspect_ratio")) cam.aspect = cp.number("aspect_ratio", 1);
        cam.near_clip = cp.number("near_clip", 0.0f);
        cam.far_clip = cp.number("far_clip", 3.4028234664e+38f);
        if (cam.far_clip < cam.near_clip) std::swap(cam.near_clip, cam.far_clip);
        if (cp.number("aperture_radius", 0.0f) > 1.1920928955e-07f) fail("depth-of-field camera is not supported");
    }
    if (camv && cp.has("transform")) {
        M4 t = get_transform(cp);
        V3 eye = igx::xform_point(t, V3());
        for (int i = 0; i < 3; ++i) { cam.eye[i] = eye[i]; cam.dir[i] = t.at(i, 2); cam.up[i] = t.at(i, 1); }
    } else if (scene_bbox.empty()) {
        cam.dir[2] = -1; cam.up[1] = 1;
    } else {
        // PerspectiveCamera::getOrientation without a transform
        float ar = cam.aspect > 0 ? cam.aspect : S.desc.film_width / (float)S.desc.film_height;
        V3 d = scene_bbox.diameter();
        float a = d.x / (2 * (cam.vertical_fov ? ar : 1));
        float b = d.y / (2 * (!cam.vertical_fov ? ar : 1));
        float s = std::sin(cam.fov / 2);
        float dist = std::abs(s) <= 1.1920928955e-07f ? 0 : std::max(a, b) * std::sqrt(1 / (s * s) - 1);
        V3 c = scene_bbox.center();
        cam.dir[2] = -1; cam.up[1] = 1;
        cam.eye[0] = c.x; cam.eye[1] = c.y; cam.eye[2] = scene_bbox.max.z + dist;
    }
    S.desc.camera = cam;

    for (int i = 0; i < 3; ++i) {
        S.desc.scene_bbox_min[i] = scene_bbox.empty() ? 0 : scene_bbox.min[i];
        S.desc.scene_bbox_max[i] = scene_bbox.empty() ? 0 : scene_bbox.max[i];
    }
    S.publish();
}

static void set_err(char* err, size_t len, const std::string& msg) {
    if (!err || len == 0) return;
    std::strncpy(err, msg.c_str(), len - 1);
    err[len - 1] = 0;
}

extern "C" igx_scene* igx_scene_load_string(const char* json_text, const char* base_dir, char* err, size_t err_len) {
    if (!json_text) { set_err(err, err_len, "null json"); return nullptr; }
    try {
        std::string base = base_dir ? base_dir : ".";
        Value doc = load_document(json_text, base);
        auto* s = new igx_scene();
        try {
            build_scene(s->store, doc, base);
        } catch (...) {
            delete s;
            throw;
        }
        return s;
    } catch (const std::exception& e) {
        set_err(err, err_len, e.what());
        return nullptr;
    }
}

extern "C" igx_scene* igx_scene_load_file(const char* path, char* err, size_t err_len) {
    if (!path) { set_err(err, err_len, "null path"); return nullptr; }
    try {
        std::string text = read_file(path);
        return igx_scene_load_string(text.c_str(), dir_of(path).c_str(), err, err_len);
    } catch (const std::exception& e) {
        set_err(err, err_len, e.what());
        return nullptr;
    }
}

extern "C" const igx_scene_desc* igx_scene_get_desc(const igx_scene* s) { return s ? &s->store.desc : nullptr; }
extern "C" void igx_scene_free(igx_scene* s) { delete s; }

extern "C" int32_t igx_scene_find_material(const igx_scene* s, const char* bsdf, const char* emissive_entity) {
    if (!s || !bsdf) return -1;
    const std::string e = emissive_entity ? emissive_entity : "";
    for (size_t i = 0; i < s->store.material_bsdf.size(); ++i)
        if (s->store.material_bsdf[i] == bsdf && s->store.material_entity[i] == e) return (int32_t)i;
    return -1;
}

extern "C" const char* igx_scene_entity_name(const igx_scene* s, uint32_t entity) {
    if (!s || entity >= s->store.entity_names.size()) return nullptr;
    return s->store.entity_names[entity].c_str();
}

// ---------------------------------------------------------------------------
// In-memory scenes (IG::Scene object model, include/igx_scene.h): the objects
// become the same document load_document builds from JSON, so build_scene
// reads both with one set of semantics.
// ---------------------------------------------------------------------------
struct igx_objscene {
    Value doc;
    std::string base_dir;
    std::vector<std::pair<std::string, std::string>> objs; // handle -> (category, name); anonymous: name empty
};

namespace {

const char* object_category(int32_t t) {
    switch (t) {
    case IGX_OBJ_BSDF: return "bsdfs";
    case IGX_OBJ_CAMERA: return "camera";
    case IGX_OBJ_ENTITY: return "entities";
    case IGX_OBJ_FILM: return "film";
    case IGX_OBJ_LIGHT: return "lights";
    case IGX_OBJ_MEDIUM: return "media";
    case IGX_OBJ_SHAPE: return "shapes";
    case IGX_OBJ_TECHNIQUE: return "technique";
    case IGX_OBJ_TEXTURE: return "textures";
    case IGX_OBJ_PARAMETER: return "parameters";
    default: return nullptr;
    }
}

bool anonymous_category(const std::string& c) { return c == "camera" || c == "film" || c == "technique"; }

Value* find_object(igx_objscene* sc, int32_t h) {
    if (!sc || h < 0 || (size_t)h >= sc->objs.size()) return nullptr;
    const auto& [cat, name] = sc->objs[(size_t)h];
    for (auto& kv : sc->doc.obj) {
        if (kv.first != cat) continue;
        if (anonymous_category(cat)) return &kv.second;
        for (auto& o : kv.second.arr) {
            const Value* n = o.find("name");
            if (n && n->str == name) return &o;
        }
    }
    return nullptr;
}

Value number_value(double x) {
    Value v;
    v.type = Value::Number;
    v.num = x;
    return v;
}

} // namespace

extern "C" igx_objscene* igx_objscene_create(const char* base_dir) {
    auto* s = new igx_objscene();
    s->doc.type = Value::Object;
    s->base_dir = base_dir ? base_dir : ".";
    return s;
}

extern "C" void igx_objscene_free(igx_objscene* s) { delete s; }

extern "C" int32_t igx_objscene_add(igx_objscene* sc, int32_t type, const char* plugin_type, const char* name,
                                    const char* base_dir) {
    const char* cat = object_category(type);
    if (!sc || !cat) return -1;
    Value obj;
    obj.type = Value::Object;
    Value t;
    t.type = Value::String;
    t.str = plugin_type ? plugin_type : "";
    obj.obj.emplace_back("type", t);
    Value bd;
    bd.type = Value::String;
    bd.str = base_dir ? base_dir : sc->base_dir;
    obj.obj.emplace_back("__base_dir", bd);
    std::string nm;
    if (!anonymous_category(cat)) {
        if (!name || !*name) return -1; // named objects need a name (Scene::add*)
        nm = name;
        Value n;
        n.type = Value::String;
        n.str = nm;
        obj.obj.emplace_back("name", n);
        put_named(category(sc->doc, cat), obj);
    } else {
        set_key(sc->doc, cat, &obj);
    }
    sc->objs.emplace_back(cat, nm);
    return (int32_t)sc->objs.size() - 1;
}

extern "C" int32_t igx_objscene_set_property(igx_objscene* sc, int32_t h, const char* key, int32_t type, const void* data,
                                             uint64_t count) {
    Value* obj = find_object(sc, h);
    // an array property may be empty (count 0, data NULL); every other form reads data
    const bool array = type == IGX_PROP_INTEGER_ARRAY || type == IGX_PROP_NUMBER_ARRAY;
    if (!obj || !key || (!data && (!array || count > 0))) return -1;
    const std::string k = key;
    if (k == "type" || k == "name" || k == "__base_dir") return -1; // set by igx_objscene_add
    Value v;
    auto floats = [&](const float* f, size_t n) {
        v.type = Value::Array;
        for (size_t i = 0; i < n; ++i) v.arr.push_back(number_value(f[i]));
    };
    switch (type) {
    case IGX_PROP_BOOL:
        v.type = Value::Bool;
        v.b = *static_cast<const int32_t*>(data) != 0;
        break;
    case IGX_PROP_INTEGER: v = number_value(*static_cast<const int32_t*>(data)); break;
    case IGX_PROP_NUMBER: v = number_value(*static_cast<const float*>(data)); break;
    case IGX_PROP_STRING:
        v.type = Value::String;
        v.str = static_cast<const char*>(data);
        break;
    case IGX_PROP_TRANSFORM: floats(static_cast<const float*>(data), 16); break;
    case IGX_PROP_VECTOR2: floats(static_cast<const float*>(data), 2); break;
    case IGX_PROP_VECTOR3: floats(static_cast<const float*>(data), 3); break;
    case IGX_PROP_NUMBER_ARRAY: floats(static_cast<const float*>(data), (size_t)count); break;
    case IGX_PROP_INTEGER_ARRAY:
        v.type = Value::Array;
        for (uint64_t i = 0; i < count; ++i) v.arr.push_back(number_value(static_cast<const int32_t*>(data)[i]));
        break;
    default: return -1;
    }
    for (auto& kv : obj->obj)
        if (kv.first == k) {
            kv.second = v;
            return 0;
        }
    obj->obj.emplace_back(k, v);
    return 0;
}

extern "C" igx_scene* igx_scene_from_objects(const igx_objscene* sc, char* err, size_t err_len) {
    if (!sc) { set_err(err, err_len, "null object scene"); return nullptr; }
    try {
        auto* s = new igx_scene();
        try {
            build_scene(s->store, sc->doc, sc->base_dir);
        } catch (...) {
            delete s;
            throw;
        }
        return s;
    } catch (const std::exception& e) {
        set_err(err, err_len, e.what());
        return nullptr;
    }
}
