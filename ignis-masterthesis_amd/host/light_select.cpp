// Light selector tables; see light_select.h.
#include "light_select.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace igx {

namespace {

struct P3 {
    float v[3];
};

struct PBox {
    P3 lo, hi;
    void extend(const P3& p) {
        for (int i = 0; i < 3; ++i) {
            lo.v[i] = std::min(lo.v[i], p.v[i]);
            hi.v[i] = std::max(hi.v[i], p.v[i]);
        }
    }
    P3 center() const { return P3{{(hi.v[0] + lo.v[0]) / 2, (hi.v[1] + lo.v[1]) / 2, (hi.v[2] + lo.v[2]) / 2}}; }
};

// PointBvh node (container/PointBvh.h): a leaf holds the index of one light
struct PNode {
    size_t index;
    PBox box;
    int axis; // < 0: leaf
};

struct Entry {
    P3 pos, dir;
    float flux; // negative: the light has no direction
    int32_t id;
};

// PointBvh::store (container/PointBvh.inl): descend by the node's mid plane
// after growing its box, then split the reached leaf in two halves of its box
void store(std::vector<PNode>& nodes, size_t leaf_idx, const P3& p) {
    if (nodes.empty()) {
        nodes.push_back(PNode{0, PBox{p, p}, -1});
        return;
    }
    size_t n = 0;
    for (;;) {
        nodes[n].box.extend(p);
        if (nodes[n].axis < 0) break;
        const float mid = nodes[n].box.center().v[nodes[n].axis];
        n = p.v[nodes[n].axis] < mid ? nodes[n].index : nodes[n].index + 1;
    }
    const PBox box = nodes[n].box;
    const float d[3] = {box.hi.v[0] - box.lo.v[0], box.hi.v[1] - box.lo.v[1], box.hi.v[2] - box.lo.v[2]};
    int axis = 0; // first of the largest extents (Eigen maxCoeff)
    for (int i = 1; i < 3; ++i)
        if (d[i] > d[axis]) axis = i;
    const float mid = d[axis] / 2; // half the extent, compared with the coordinate as the reference does
    const size_t old_leaf = nodes[n].index;
    const size_t left = nodes.size();
    nodes[n].index = left;
    nodes[n].axis = axis;
    PBox lb = box, rb = box; // BoundingBox::computeSplit(.., 0.5)
    const float off = (box.hi.v[axis] - box.lo.v[axis]) * 0.5f;
    lb.hi.v[axis] -= off;
    rb.lo.v[axis] += off;
    const bool new_left = p.v[axis] < mid;
    nodes.push_back(PNode{new_left ? leaf_idx : old_leaf, lb, -1});
    nodes.push_back(PNode{new_left ? old_leaf : leaf_idx, rb, -1});
}

// populateInnerNodes (LightHierarchy.cpp:46-73)
Entry populate(size_t id, uint32_t code, uint32_t depth, const std::vector<PNode>& nodes, const std::vector<Entry>& leaves,
               std::vector<Entry>& entries, std::vector<uint32_t>& codes) {
    const PNode& node = nodes[id];
    Entry& out = entries[id];
    if (node.axis < 0) {
        const Entry leaf = leaves[node.index];
        out = leaf;
        codes[leaf.id] = code;
        return out;
    }
    const Entry l = populate(node.index, code, depth + 1, nodes, leaves, entries, codes);
    const Entry r = populate(node.index + 1, code | (1u << depth), depth + 1, nodes, leaves, entries, codes);
    Entry e;
    e.pos = node.box.center();
    e.id = -(int32_t)(node.index + 1);
    const P3 unit_z{{0, 0, 1}};
    if (l.flux < 0 && r.flux < 0) {
        e.dir = unit_z;
        e.flux = l.flux + r.flux;
    } else if (l.flux < 0) {
        e.dir = unit_z;
        e.flux = -(-l.flux + r.flux);
    } else if (r.flux < 0) {
        e.dir = unit_z;
        e.flux = -(l.flux - r.flux);
    } else {
        P3 s{{l.dir.v[0] + r.dir.v[0], l.dir.v[1] + r.dir.v[1], l.dir.v[2] + r.dir.v[2]}};
        const float n = std::sqrt(s.v[0] * s.v[0] + s.v[1] * s.v[1] + s.v[2] * s.v[2]);
        for (float& c : s.v) c /= n; // Eigen normalized()
        e.dir = s;
        e.flux = l.flux + r.flux;
    }
    out = e;
    return e;
}

} // namespace

LightSelectTables build_light_select(int selector, int light_count, const std::vector<igx_light>& finite) {
    LightSelectTables t;
    const size_t n = finite.size();
    if (light_count <= 1 || n == 0) return t; // uniform (LoaderLight.cpp:428-429, empty cdf / hierarchy)
    if (selector == IGX_SELECT_SIMPLE) {
        // CDF::computeForArray (CDF.cpp:11-40)
        constexpr float MinEps = 1e-5f;
        std::vector<float> cdf(n);
        cdf[0] = finite[0].select_flux;
        for (size_t x = 1; x < n; ++x) cdf[x] = cdf[x - 1] + finite[x].select_flux;
        const float sum = cdf.back();
        if (sum > MinEps) {
            const float inv = 1.0f / sum;
            for (float& v : cdf) v *= inv;
        } else {
            const float inv = 1.0f / (float)n;
            for (size_t x = 0; x < n; ++x) cdf[x] = (float)x * inv;
        }
        cdf.back() = 1;
        t.selector = IGX_SELECT_SIMPLE;
        t.cdf = std::move(cdf);
    } else if (selector == IGX_SELECT_HIERARCHY) {
        std::vector<PNode> nodes;
        std::vector<Entry> leaves;
        for (size_t i = 0; i < n; ++i) {
            const igx_light& L = finite[i];
            Entry e;
            std::memcpy(e.pos.v, L.select_position, sizeof(e.pos.v));
            if (L.select_has_direction) std::memcpy(e.dir.v, L.select_direction, sizeof(e.dir.v));
            else e.dir = P3{{0, 0, 1}};
            e.flux = L.select_has_direction ? L.select_flux : -L.select_flux;
            e.id = (int32_t)i;
            leaves.push_back(e);
            store(nodes, leaves.size() - 1, e.pos);
        }
        // a leaf's code keeps one bit per level (bit d: right at depth d), so
        // the walk (light/light_hierarchy.art) is defined for at most 32
        // levels; the insertion-built tree can get deeper with clustered or
        // geometrically spaced lights (the reference leaves this as a TODO and
        // shifts past the word).  Such a scene gets the flux CDF instead:
        // also unbiased, and the same lights weighted by the same flux.
        std::vector<std::pair<size_t, uint32_t>> todo{{0, 0}};
        uint32_t deepest = 0;
        while (!todo.empty()) {
            const auto [id, d] = todo.back();
            todo.pop_back();
            deepest = std::max(deepest, d);
            if (nodes[id].axis >= 0) {
                todo.push_back({(size_t)nodes[id].index, d + 1});
                todo.push_back({(size_t)nodes[id].index + 1, d + 1});
            }
        }
        if (deepest > 32) return build_light_select(IGX_SELECT_SIMPLE, light_count, finite);
        std::vector<Entry> entries(nodes.size());
        std::vector<uint32_t> codes(n, 0);
        populate(0, 0, 0, nodes, leaves, entries, codes);
        const size_t pad = (n + 3) / 4 * 4; // writeAlignmentPad(16) after the codes
        t.hierarchy.assign(pad + 8 * entries.size(), 0u);
        std::memcpy(t.hierarchy.data(), codes.data(), n * sizeof(uint32_t));
        for (size_t k = 0; k < entries.size(); ++k) {
            const Entry& e = entries[k];
            float rec[8] = {e.pos.v[0], e.pos.v[1], e.pos.v[2], e.flux, e.dir.v[0], e.dir.v[1], e.dir.v[2], 0};
            std::memcpy(&rec[7], &e.id, 4);
            std::memcpy(t.hierarchy.data() + pad + 8 * k, rec, sizeof(rec));
        }
        t.selector = IGX_SELECT_HIERARCHY;
    }
    return t;
}

} // namespace igx
