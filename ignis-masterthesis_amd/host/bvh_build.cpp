// Binned-SAH BVH2 builder; see bvh_build.h.
#include "bvh_build.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <stdexcept>
#include <thread>
#include <future>
#include <cstring>
#include <functional>
#include <string>

namespace igx {

namespace {

struct Box {
    float lo[3] = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), std::numeric_limits<float>::max()};
    float hi[3] = {-std::numeric_limits<float>::max(), -std::numeric_limits<float>::max(), -std::numeric_limits<float>::max()};
    void grow(const float* a, const float* b) {
        for (int i = 0; i < 3; ++i) { lo[i] = std::min(lo[i], a[i]); hi[i] = std::max(hi[i], b[i]); }
    }
    void grow(const Box& o) { grow(o.lo, o.hi); }
    void grow_point(const float* p) { grow(p, p); }
    float half_area() const {
        float dx = std::max(hi[0] - lo[0], 0.f), dy = std::max(hi[1] - lo[1], 0.f), dz = std::max(hi[2] - lo[2], 0.f);
        return dx * (dy + dz) + dy * dz;
    }
    bool valid() const { return lo[0] <= hi[0]; }
};

struct TmpNode {
    Box box;
    int32_t left = -1, right = -1; // children (tmp indices), -1 for leaf
    uint32_t first = 0, count = 0;
};

struct Builder {
    const BvhBuildInput& in;
    int max_leaf;
    int bins;
    float node_cost = 1.0f;     // SAH cost of a node step relative to one primitive test
    std::vector<uint32_t>& idx; // shared; each builder only touches its own ranges
    std::vector<TmpNode> nodes;
    int par_depth;              // subtrees above this depth are built on their own threads

    Builder(const BvhBuildInput& i, int ml, int b, std::vector<uint32_t>& ix, int pd)
        : in(i), max_leaf(ml), bins(b), idx(ix), par_depth(pd) {}

    // Bin idx[first, first+count) by centroid along `axis`.
    void bin_range(uint32_t first, uint32_t count, int axis, float lo, float scale, Box* bbox, uint32_t* bcnt) const {
        for (uint32_t i = first; i < first + count; ++i) {
            uint32_t p = idx[i];
            int b = std::min(bins - 1, (int)((in.centroid[3 * p + axis] - lo) * scale));
            bbox[b].grow(&in.bmin[3 * p], &in.bmax[3 * p]);
            bcnt[b]++;
        }
    }

    // Returns tmp node index of a subtree over idx[first, first+count).
    int32_t build(uint32_t first, uint32_t count, int depth) {
        int32_t me = (int32_t)nodes.size();
        nodes.emplace_back();
        Box box, cbox;
        for (uint32_t i = first; i < first + count; ++i) {
            uint32_t p = idx[i];
            box.grow(&in.bmin[3 * p], &in.bmax[3 * p]);
            cbox.grow_point(&in.centroid[3 * p]);
        }
        nodes[me].box = box;
        nodes[me].first = first;
        nodes[me].count = count;
        if (count == 1) return me;

        // best binned SAH split
        float best_cost = std::numeric_limits<float>::max();
        int best_axis = -1, best_bin = -1;
        std::vector<Box> bbox(bins);
        std::vector<uint32_t> bcnt(bins);
        std::vector<float> right_area(bins);
        std::vector<uint32_t> right_cnt(bins);
        for (int axis = 0; axis < 3; ++axis) {
            float ext = cbox.hi[axis] - cbox.lo[axis];
            if (!(ext > 0)) continue;
            float scale = bins / ext;
            for (int b = 0; b < bins; ++b) { bbox[b] = Box(); bcnt[b] = 0; }
            bin_range(first, count, axis, cbox.lo[axis], scale, bbox.data(), bcnt.data());
            Box acc;
            uint32_t c = 0;
            for (int b = bins - 1; b > 0; --b) {
                acc.grow(bbox[b]);
                c += bcnt[b];
                right_area[b] = acc.valid() ? acc.half_area() : 0.f;
                right_cnt[b] = c;
            }
            acc = Box();
            c = 0;
            for (int b = 0; b < bins - 1; ++b) {
                acc.grow(bbox[b]);
                c += bcnt[b];
                if (c == 0 || right_cnt[b + 1] == 0) continue;
                float cost = acc.half_area() * c + right_area[b + 1] * right_cnt[b + 1];
                if (cost < best_cost) { best_cost = cost; best_axis = axis; best_bin = b; }
            }
        }
        float parent_area = box.half_area();
        // leaf vs split: node cost `node_cost`, intersection cost 1 per primitive (relative)
        float leaf_cost = (float)count;
        float split_cost = best_axis >= 0 ? node_cost + best_cost / std::max(parent_area, 1e-30f) : std::numeric_limits<float>::max();
        if ((int)count <= max_leaf && leaf_cost <= split_cost) return me;

        uint32_t mid;
        if (best_axis < 0) {
            mid = first + count / 2; // all centroids coincide: split in the middle
        } else {
            float ext = cbox.hi[best_axis] - cbox.lo[best_axis];
            float scale = bins / ext;
            auto it = std::partition(idx.begin() + first, idx.begin() + first + count, [&](uint32_t p) {
                int b = std::min(bins - 1, (int)((in.centroid[3 * p + best_axis] - cbox.lo[best_axis]) * scale));
                return b <= best_bin;
            });
            mid = (uint32_t)(it - idx.begin());
            if (mid == first || mid == first + count) mid = first + count / 2;
        }
        int32_t l, r;
        if (depth < par_depth && count >= 65536) {
            // left subtree on its own thread with its own node pool, merged after
            Builder sub(in, max_leaf, bins, idx, par_depth);
            sub.node_cost = node_cost;
            auto fut = std::async(std::launch::async, [&sub, first, mid, depth] { return sub.build(first, mid - first, depth + 1); });
            r = build(mid, first + count - mid, depth + 1);
            int32_t sroot = fut.get();
            const int32_t off = (int32_t)nodes.size();
            for (TmpNode t : sub.nodes) {
                if (t.left >= 0) { t.left += off; t.right += off; }
                nodes.push_back(t);
            }
            l = sroot + off;
        } else {
            l = build(first, mid - first, depth + 1);
            r = build(mid, first + count - mid, depth + 1);
        }
        nodes[me].left = l;
        nodes[me].right = r;
        return me;
    }
};

// Child boxes are written slightly enlarged, so that which triangles a ray
// tests does not depend on how the builder grouped them.  Moeller-Trumbore
// accepts barycentrics down to -FLT_EPSILON (intersection.art:71-101), i.e.
// hits up to about 2 * FLT_EPSILON * (longest edge) outside the triangle and
// its bounds, and the slab test's t carries float rounding relative to the
// coordinates.  A box that misses such a hit by an ulp would make the closest
// hit depend on the topology (a grouping that puts the triangle in a wider box
// tests it, another does not).  Pad: 8 * FLT_EPSILON of the box's extent sum
// plus 4 * FLT_EPSILON of the coordinate's magnitude, per side.
Box pad_box(const Box& b) {
    if (!(b.lo[0] <= b.hi[0] && b.lo[1] <= b.hi[1] && b.lo[2] <= b.hi[2])) return b; // empty child
    const float eps = std::numeric_limits<float>::epsilon();
    const float ext = (b.hi[0] - b.lo[0]) + (b.hi[1] - b.lo[1]) + (b.hi[2] - b.lo[2]);
    Box r = b;
    for (int a = 0; a < 3; ++a) {
        const float mag = std::max(std::fabs(b.lo[a]), std::fabs(b.hi[a]));
        const float pad = 8 * eps * ext + 4 * eps * mag;
        r.lo[a] = b.lo[a] - pad;
        r.hi[a] = b.hi[a] + pad;
    }
    return r;
}

void set_child(BvhNode& n, int k, const Box& box, int32_t ref) {
    const Box b = pad_box(box);
    int o = k == 0 ? 0 : 6;
    // c0: [0]=lo.x [1]=hi.x [2]=lo.y [3]=hi.y [4]=lo.z [5]=hi.z ; c1 likewise at +6
    n.b[o + 0] = b.lo[0]; n.b[o + 1] = b.hi[0];
    n.b[o + 2] = b.lo[1]; n.b[o + 3] = b.hi[1];
    n.b[o + 4] = b.lo[2]; n.b[o + 5] = b.hi[2];
    n.ref[k] = ref;
}

void set_empty(BvhNode& n, int k) {
    Box e; // inverted box: lo = +max, hi = -max
    set_child(n, k, e, -1);
}

// Flatten a tmp-node tree into BvhNodes in DFS pre-order; each inner tmp node
// becomes one BvhNode (leaves become leaf codes in their parent).
void flatten(const std::vector<TmpNode>& tn, int32_t root, BvhBuildResult& res) {
    auto leaf_ref = [&](const TmpNode& t) { return encode_leaf((int32_t)t.first, (int32_t)t.count); };
    struct Item { int32_t tmp; int32_t out; int depth; };
    std::vector<Item> stack;
    res.nodes.emplace_back();
    if (tn[root].left < 0) {
        // root itself is a leaf: both children reference it (an empty child
        // box would pass the min/max slab test; a duplicate leaf is harmless
        // for closest and any hit)
        set_child(res.nodes[0], 0, tn[root].box, leaf_ref(tn[root]));
        set_child(res.nodes[0], 1, tn[root].box, leaf_ref(tn[root]));
        res.depth = 1;
        res.root_is_leaf = true;
        res.root_leaf_ref = leaf_ref(tn[root]);
        return;
    }
    stack.push_back({root, 0, 1});
    while (!stack.empty()) {
        Item it = stack.back();
        stack.pop_back();
        res.depth = std::max(res.depth, it.depth);
        const TmpNode& t = tn[it.tmp];
        int32_t kids[2] = {t.left, t.right};
        // push right first so the left subtree is laid out right after its parent
        int32_t out_idx[2] = {-1, -1};
        for (int k = 0; k < 2; ++k) {
            const TmpNode& c = tn[kids[k]];
            if (c.left < 0) {
                set_child(res.nodes[it.out], k, c.box, leaf_ref(c));
            } else {
                out_idx[k] = (int32_t)res.nodes.size();
                res.nodes.emplace_back();
                set_child(res.nodes[it.out], k, c.box, out_idx[k]);
            }
            res.nodes[it.out].pad[k] = 0;
        }
        for (int k = 1; k >= 0; --k)
            if (out_idx[k] >= 0) stack.push_back({kids[k], out_idx[k], it.depth + 1});
    }
}

} // namespace

BvhBuildResult build_bvh2(const BvhBuildInput& in, int max_leaf, int bins, float node_cost) {
    if (max_leaf < 1 || max_leaf > (1 << kLeafCountBits)) throw std::invalid_argument("max_leaf out of range");
    BvhBuildResult res;
    const size_t n = in.count();
    res.max_leaf = max_leaf;
    if (n == 0) {
        BvhNode root{};
        set_empty(root, 0);
        set_empty(root, 1);
        res.nodes.push_back(root);
        res.depth = 1;
        return res;
    }
    if (n >= (size_t)kMaxLeafFirst) throw std::invalid_argument("too many primitives for the leaf encoding");
    std::vector<uint32_t> idx(n);
    for (size_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
    // up to 2^4 concurrent subtree builders for large inputs
    const int par_depth = n >= 262144 ? 4 : 0;
    Builder b(in, max_leaf, bins, idx, par_depth);
    b.node_cost = node_cost;
    b.nodes.reserve(2 * n / std::max(1, max_leaf) + 4);
    int32_t root = b.build(0, (uint32_t)n, 0);
    res.prim_order = std::move(idx);

    flatten(b.nodes, root, res);
    return res;
}

// ---------------------------------------------------------------------------
// Split BVH (Stich, Friedrich and Dietrich, "Spatial Splits in Bounding Volume
// Hierarchies", HPG 2009).  At every node the binned object split competes
// with a binned spatial split whose bins hold the bounds of the triangles'
// parts clipped to the bin slabs; a triangle the chosen plane cuts is then
// referenced from both sides, each with the bounds of its part.  Spatial
// splits are tried only where the object split's children overlap by more
// than alpha of the root area, and the added references are capped.
// ---------------------------------------------------------------------------
namespace {

struct Ref {
    uint32_t prim;
    Box box;
};

bool nonempty(const Box& b) { return b.lo[0] <= b.hi[0] && b.lo[1] <= b.hi[1] && b.lo[2] <= b.hi[2]; }

Box overlap(const Box& a, const Box& b) {
    Box r;
    for (int k = 0; k < 3; ++k) {
        r.lo[k] = std::max(a.lo[k], b.lo[k]);
        r.hi[k] = std::min(a.hi[k], b.hi[k]);
    }
    return r;
}

// Bounds of the part of triangle v (9 floats) with lo <= x[axis] <= hi,
// widened by a few ulps of the triangle's extent (so rounding of the
// edge-plane points never shrinks it below the true part) and intersected
// with the reference's current bounds `cur`.  Empty box if nothing is left.
Box clip_part(const float* v, int axis, float lo, float hi, const Box& cur) {
    Box b;
    for (int i = 0; i < 3; ++i) {
        const float* a = v + 3 * i;
        const float* c = v + 3 * ((i + 1) % 3);
        const float pa = a[axis], pc = c[axis];
        if (pa >= lo && pa <= hi) b.grow_point(a);
        const float planes[2] = {lo, hi};
        for (float pl : planes) {
            if ((pa < pl && pc > pl) || (pa > pl && pc < pl)) {
                const double t = ((double)pl - pa) / ((double)pc - pa);
                float q[3];
                for (int k = 0; k < 3; ++k) q[k] = (float)((double)a[k] + t * ((double)c[k] - a[k]));
                q[axis] = pl;
                b.grow_point(q);
            }
        }
    }
    if (!nonempty(b)) return Box();
    for (int k = 0; k < 3; ++k) {
        const float tmin = std::min({v[k], v[3 + k], v[6 + k]}), tmax = std::max({v[k], v[3 + k], v[6 + k]});
        const float scale = std::max({std::fabs(tmin), std::fabs(tmax), tmax - tmin});
        const float e = 8 * std::numeric_limits<float>::epsilon() * scale;
        b.lo[k] -= e;
        b.hi[k] += e;
    }
    Box r = overlap(b, cur);
    return nonempty(r) ? r : Box();
}

struct SplitBuilder {
    const float* V; // 9 floats per primitive
    int max_leaf, bins;
    float min_overlap; // alpha * root half-area
    long long budget;  // references spatial splits may still add
    std::vector<TmpNode> nodes;
    std::vector<uint32_t> order;

    int32_t make_leaf(const std::vector<Ref>& refs, const Box& box) {
        int32_t me = (int32_t)nodes.size();
        nodes.emplace_back();
        nodes[me].box = box;
        nodes[me].first = (uint32_t)order.size();
        nodes[me].count = (uint32_t)refs.size();
        for (const Ref& r : refs) order.push_back(r.prim);
        return me;
    }

    static void center(const Box& b, float* c) {
        for (int k = 0; k < 3; ++k) c[k] = 0.5f * (b.lo[k] + b.hi[k]);
    }

    int32_t build(std::vector<Ref>& refs) {
        const uint32_t n = (uint32_t)refs.size();
        Box box, cbox;
        for (const Ref& r : refs) {
            box.grow(r.box);
            float c[3];
            center(r.box, c);
            cbox.grow_point(c);
        }
        if (n == 1) return make_leaf(refs, box);
        const float parent_area = std::max(box.half_area(), 1e-30f);
        const float inf = std::numeric_limits<float>::max();

        // object split: binned SAH over reference centroids
        float best_o = inf;
        int ax_o = -1, bin_o = -1;
        Box lb_o, rb_o;
        std::vector<Box> bb(bins), rbox(bins);
        std::vector<uint32_t> cnt(bins), rcnt(bins);
        for (int axis = 0; axis < 3; ++axis) {
            const float ext = cbox.hi[axis] - cbox.lo[axis];
            if (!(ext > 0)) continue;
            const float scale = bins / ext;
            for (int b = 0; b < bins; ++b) { bb[b] = Box(); cnt[b] = 0; }
            for (const Ref& r : refs) {
                float c[3];
                center(r.box, c);
                int b = std::min(bins - 1, (int)((c[axis] - cbox.lo[axis]) * scale));
                bb[b].grow(r.box);
                cnt[b]++;
            }
            Box acc;
            uint32_t c = 0;
            for (int b = bins - 1; b > 0; --b) {
                acc.grow(bb[b]);
                c += cnt[b];
                rbox[b] = acc;
                rcnt[b] = c;
            }
            acc = Box();
            c = 0;
            for (int b = 0; b < bins - 1; ++b) {
                acc.grow(bb[b]);
                c += cnt[b];
                if (c == 0 || rcnt[b + 1] == 0) continue;
                float cost = acc.half_area() * c + rbox[b + 1].half_area() * rcnt[b + 1];
                if (cost < best_o) { best_o = cost; ax_o = axis; bin_o = b; lb_o = acc; rb_o = rbox[b + 1]; }
            }
        }

        // spatial split: binned over the node box, triangles clipped to the bins
        float best_s = inf;
        int ax_s = -1;
        float pos_s = 0;
        bool try_spatial = budget > 0;
        if (ax_o >= 0) {
            Box ov = overlap(lb_o, rb_o);
            try_spatial = try_spatial && nonempty(ov) && ov.half_area() > min_overlap;
        }
        if (try_spatial) {
            std::vector<uint32_t> enter(bins), leave(bins);
            for (int axis = 0; axis < 3; ++axis) {
                const float lo0 = box.lo[axis], ext = box.hi[axis] - lo0;
                if (!(ext > 0)) continue;
                const float w = ext / bins;
                auto plane = [&](int b) { return b >= bins ? box.hi[axis] : lo0 + w * b; };
                for (int b = 0; b < bins; ++b) { bb[b] = Box(); enter[b] = leave[b] = 0; }
                for (const Ref& r : refs) {
                    int b0 = std::min(bins - 1, std::max(0, (int)((r.box.lo[axis] - lo0) / w)));
                    int b1 = std::min(bins - 1, std::max(b0, (int)((r.box.hi[axis] - lo0) / w)));
                    enter[b0]++;
                    leave[b1]++;
                    if (b0 == b1) {
                        bb[b0].grow(r.box);
                        continue;
                    }
                    for (int b = b0; b <= b1; ++b) {
                        Box part = clip_part(V + 9 * (size_t)r.prim, axis, plane(b), plane(b + 1), r.box);
                        if (nonempty(part)) bb[b].grow(part);
                    }
                }
                Box acc;
                uint32_t c = 0;
                for (int b = bins - 1; b > 0; --b) {
                    acc.grow(bb[b]);
                    c += leave[b];
                    rbox[b] = acc;
                    rcnt[b] = c;
                }
                acc = Box();
                c = 0;
                for (int b = 0; b < bins - 1; ++b) {
                    acc.grow(bb[b]);
                    c += enter[b];
                    if (c == 0 || rcnt[b + 1] == 0 || !nonempty(acc) || !nonempty(rbox[b + 1])) continue;
                    float cost = acc.half_area() * c + rbox[b + 1].half_area() * rcnt[b + 1];
                    if (cost < best_s) { best_s = cost; ax_s = axis; pos_s = plane(b + 1); }
                }
            }
        }

        const float best = std::min(best_o, best_s);
        const float split_cost = best < inf ? 1.0f + best / parent_area : inf;
        if ((int)n <= max_leaf && (float)n <= split_cost) return make_leaf(refs, box);

        std::vector<Ref> L, R;
        if (best_s < best_o) {
            for (const Ref& r : refs) {
                if (r.box.hi[ax_s] <= pos_s) { L.push_back(r); continue; }
                if (r.box.lo[ax_s] >= pos_s) { R.push_back(r); continue; }
                Box lbx = clip_part(V + 9 * (size_t)r.prim, ax_s, -inf, pos_s, r.box);
                Box rbx = clip_part(V + 9 * (size_t)r.prim, ax_s, pos_s, inf, r.box);
                if (nonempty(lbx) && nonempty(rbx)) {
                    L.push_back({r.prim, lbx});
                    R.push_back({r.prim, rbx});
                    --budget;
                } else if (nonempty(rbx)) {
                    R.push_back(r);
                } else {
                    L.push_back(r);
                }
            }
        } else if (ax_o >= 0) {
            const float scale = bins / (cbox.hi[ax_o] - cbox.lo[ax_o]);
            for (const Ref& r : refs) {
                float c[3];
                center(r.box, c);
                int b = std::min(bins - 1, (int)((c[ax_o] - cbox.lo[ax_o]) * scale));
                (b <= bin_o ? L : R).push_back(r);
            }
        }
        if (L.empty() || R.empty()) {
            // no useful plane (coincident centroids): halve the list
            L.assign(refs.begin(), refs.begin() + n / 2);
            R.assign(refs.begin() + n / 2, refs.end());
        }
        std::vector<Ref>().swap(refs);
        const int32_t me = (int32_t)nodes.size();
        nodes.emplace_back();
        nodes[me].box = box;
        const int32_t l = build(L);
        const int32_t r = build(R);
        nodes[me].left = l;
        nodes[me].right = r;
        return me;
    }
};

} // namespace

BvhBuildResult build_sbvh2(const BvhBuildInput& in, const std::vector<float>& tri9, int max_leaf, float ref_budget,
                           int bins) {
    const size_t n = in.count();
    if (n == 0 || tri9.size() != 9 * n) return build_bvh2(in, max_leaf, bins);
    if (max_leaf < 1 || max_leaf > (1 << kLeafCountBits)) throw std::invalid_argument("max_leaf out of range");
    std::vector<Ref> refs(n);
    Box root;
    for (size_t i = 0; i < n; ++i) {
        refs[i].prim = (uint32_t)i;
        refs[i].box.grow(&in.bmin[3 * i], &in.bmax[3 * i]);
        root.grow(refs[i].box);
    }
    SplitBuilder sb{tri9.data(), max_leaf, bins, 1e-5f * root.half_area(), (long long)(ref_budget * (double)n), {}, {}};
    sb.nodes.reserve(2 * n / std::max(1, max_leaf) + 4);
    const int32_t r = sb.build(refs);
    if (sb.order.size() >= (size_t)kMaxLeafFirst) throw std::invalid_argument("too many references for the leaf encoding");
    BvhBuildResult res;
    res.max_leaf = max_leaf;
    res.prim_order = std::move(sb.order);
    flatten(sb.nodes, r, res);
    return res;
}

namespace {

struct Child2 {
    float lo[3], hi[3];
    int32_t ref; // BVH2 ref: >= 0 inner node index, < 0 leaf code
};

Child2 child_of(const BvhNode& n, int k) {
    Child2 c;
    const float* b = n.b + 6 * k;
    c.lo[0] = b[0]; c.hi[0] = b[1];
    c.lo[1] = b[2]; c.hi[1] = b[3];
    c.lo[2] = b[4]; c.hi[2] = b[5];
    c.ref = n.ref[k];
    return c;
}

float half_area(const Child2& c) {
    float dx = c.hi[0] - c.lo[0], dy = c.hi[1] - c.lo[1], dz = c.hi[2] - c.lo[2];
    return dx * (dy + dz) + dy * dz;
}

} // namespace

namespace {

// Surface-area collapse of a BVH2 into N-wide nodes (N = 4 or 8): every wide
// node absorbs the largest-area inner grandchildren of its BVH2 node until it
// has N children; children are laid out after their parent in DFS order.
template <int N>
void collapse_wide(const BvhBuildResult& in, std::vector<WideNode<N>>& out, int& depth, int& stack_need) {
    const float inf = std::numeric_limits<float>::infinity();
    auto set = [&](WideNode<N>& n, int k, const Child2& c, int32_t ref) {
        for (int a = 0; a < 3; ++a) {
            n.lo[a][k] = c.lo[a];
            n.hi[a][k] = c.hi[a];
        }
        n.ref[k] = ref;
    };
    auto empty_node = [&]() {
        WideNode<N> n{};
        for (int k = 0; k < N; ++k) {
            for (int a = 0; a < 3; ++a) n.lo[a][k] = n.hi[a][k] = inf;
            n.ref[k] = kEmptyRef;
        }
        return n;
    };
    out.clear();
    depth = 0;
    stack_need = 0;
    if (in.nodes.empty()) return;
    out.push_back(empty_node());
    if (in.root_is_leaf || in.prim_order.empty()) {
        if (in.root_is_leaf) set(out[0], 0, child_of(in.nodes[0], 0), in.root_leaf_ref);
        depth = 1;
        return;
    }
    // iterative DFS: (BVH2 inner node, output node, depth)
    struct Item { int32_t src; int32_t out; int depth; };
    std::vector<Item> stack{{0, 0, 1}};
    std::vector<int> nchild(1, 0);
    while (!stack.empty()) {
        Item it = stack.back();
        stack.pop_back();
        depth = std::max(depth, it.depth);
        Child2 kids[N];
        int nk = 0;
        for (int k = 0; k < 2; ++k) // an absent BVH2 child (kEmptyRef, bvh2_from_reference) stays absent
            if (in.nodes[it.src].ref[k] != kEmptyRef) kids[nk++] = child_of(in.nodes[it.src], k);
        while (nk < N) {
            int best = -1;
            float best_area = -1;
            for (int k = 0; k < nk; ++k)
                if (kids[k].ref >= 0 && half_area(kids[k]) > best_area) { best = k; best_area = half_area(kids[k]); }
            if (best < 0) break;
            const BvhNode& e = in.nodes[kids[best].ref];
            kids[best] = child_of(e, 0);
            kids[nk++] = child_of(e, 1);
        }
        nchild[it.out] = nk;
        int32_t out_idx[N];
        for (int k = 0; k < N; ++k) out_idx[k] = -1;
        for (int k = 0; k < nk; ++k) {
            if (kids[k].ref >= 0) {
                out_idx[k] = (int32_t)out.size();
                out.push_back(empty_node());
                nchild.push_back(0);
                set(out[it.out], k, kids[k], out_idx[k]);
            } else {
                set(out[it.out], k, kids[k], kids[k].ref);
            }
        }
        for (int k = nk - 1; k >= 0; --k)
            if (out_idx[k] >= 0) stack.push_back({kids[k].ref, out_idx[k], it.depth + 1});
    }
    // stack need: pushes along a path = sum over its nodes of (children - 1);
    // children come after their parent, so one reverse sweep computes it
    std::vector<int> need(out.size(), 0);
    for (size_t i = out.size(); i-- > 0;) {
        int below = 0;
        for (int k = 0; k < N; ++k)
            if (out[i].ref[k] >= 0) below = std::max(below, need[out[i].ref[k]]);
        need[i] = (nchild[i] - 1) + below;
    }
    stack_need = need[0];
}

// Quantise axis a of an N-wide node: origin o, power-of-two scale s and the
// child bytes (packed four to a word, child k in byte k % 4 of word k / 4).
// Every quantised bound keeps at least half a quantum of slack outside the
// child's box (exact arithmetic), and a quantum is at least 2^-19 of the
// coordinates' magnitude.
template <int N>
void quantize_axis(const float* lo, const float* hi, const bool* valid, float& origin, float& scale, uint32_t* wlo,
                   uint32_t* whi) {
    double l = INFINITY, h = -INFINITY;
    for (int k = 0; k < N; ++k)
        if (valid[k]) {
            l = std::min(l, (double)lo[k]);
            h = std::max(h, (double)hi[k]);
        }
    if (!(l <= h)) l = h = 0; // no valid child (never built, kept total)
    const double mag = std::max(std::fabs(l), std::fabs(h));
    // a quantum: the extent over 249 codes (three spare on each side), and at
    // least 2^-19 of the magnitude so rounding in the slab test stays far below it
    double s = std::max({(h - l) / 249.0, mag * std::ldexp(1.0, -19), std::ldexp(1.0, -100)});
    s = std::ldexp(1.0, (int)std::ceil(std::log2(s)));
    for (;;) {
        const float o = std::nextafter((float)(l - 2 * s), -INFINITY);
        bool ok = true;
        uint32_t wl[N / 4] = {}, wh[N / 4] = {};
        for (int k = 0; k < N; ++k) {
            long ql = 0, qh = 0;
            if (valid[k]) {
                ql = (long)std::floor(((double)lo[k] - o) / s) - 1;
                qh = (long)std::ceil(((double)hi[k] - o) / s) + 1;
                // at least half a quantum of slack on both sides, in exact arithmetic
                ok = ok && ql >= 0 && qh <= 255 && (double)o + ql * s <= lo[k] - 0.5 * s && (double)o + qh * s >= hi[k] + 0.5 * s;
            }
            wl[k / 4] |= (uint32_t)std::clamp(ql, 0L, 255L) << (8 * (k % 4));
            wh[k / 4] |= (uint32_t)std::clamp(qh, 0L, 255L) << (8 * (k % 4));
        }
        if (ok) {
            origin = o;
            scale = (float)s;
            for (int w = 0; w < N / 4; ++w) {
                wlo[w] = wl[w];
                whi[w] = wh[w];
            }
            return;
        }
        s *= 2;
    }
}

template <int N>
void valid_children(const WideNode<N>& n, bool* valid) {
    for (int k = 0; k < N; ++k) {
        valid[k] = n.ref[k] != kEmptyRef;
        for (int a = 0; a < 3; ++a)
            valid[k] = valid[k] && std::isfinite(n.lo[a][k]) && std::isfinite(n.hi[a][k]) && n.lo[a][k] <= n.hi[a][k];
    }
}

} // namespace

Bvh4Result collapse_bvh4(const BvhBuildResult& in) {
    Bvh4Result res;
    std::vector<WideNode<4>> w;
    collapse_wide<4>(in, w, res.depth, res.stack_need);
    res.nodes.resize(w.size());
    for (size_t i = 0; i < w.size(); ++i) {
        Bvh4Node& n = res.nodes[i];
        std::memset(&n, 0, sizeof(n));
        for (int k = 0; k < 4; ++k) {
            n.lo_x[k] = w[i].lo[0][k]; n.hi_x[k] = w[i].hi[0][k];
            n.lo_y[k] = w[i].lo[1][k]; n.hi_y[k] = w[i].hi[1][k];
            n.lo_z[k] = w[i].lo[2][k]; n.hi_z[k] = w[i].hi[2][k];
            n.ref[k] = w[i].ref[k];
        }
    }
    return res;
}

// ---------------------------------------------------------------------------
// Quantised wide nodes (Bvh4QNode; bvh_build.h)
// ---------------------------------------------------------------------------
Bvh4QNode quantize_bvh4(const Bvh4Node& n) {
    WideNode<4> w;
    for (int k = 0; k < 4; ++k) {
        w.lo[0][k] = n.lo_x[k]; w.hi[0][k] = n.hi_x[k];
        w.lo[1][k] = n.lo_y[k]; w.hi[1][k] = n.hi_y[k];
        w.lo[2][k] = n.lo_z[k]; w.hi[2][k] = n.hi_z[k];
        w.ref[k] = n.ref[k];
    }
    bool valid[4];
    valid_children<4>(w, valid);
    Bvh4QNode q{};
    for (int k = 0; k < 4; ++k) q.ref[k] = n.ref[k];
    float* sc[3] = {&q.sx, &q.sy, &q.sz};
    uint32_t* qlo[3] = {&q.qlo_x, &q.qlo_y, &q.qlo_z};
    uint32_t* qhi[3] = {&q.qhi_x, &q.qhi_y, &q.qhi_z};
    for (int a = 0; a < 3; ++a) quantize_axis<4>(w.lo[a], w.hi[a], valid, q.origin[a], *sc[a], qlo[a], qhi[a]);
    return q;
}

// ---------------------------------------------------------------------------
// Reference GPU BLAS (Node2 + Tri1 blob) -> BvhBuildResult.
// Node2 (traversal/mapping_gpu.art:3-7) stores the child boxes in the same
// interleaving as BvhNode; children are inner index + 1 (> 0), ~first Tri1
// (< 0) or 0 for a child the adapter cut out (BvhNAdapter.h:121-148).  A leaf
// runs until the Tri1 whose prim_id has bit 31 set (TriBVHAdapter.h:148-158).
// ---------------------------------------------------------------------------
namespace {

struct RefNode2 {
    float b[12];
    int32_t child[2];
    int32_t pad[2];
};
static_assert(sizeof(RefNode2) == 64, "Node2 is 64 bytes");
constexpr size_t kRefTri1Bytes = 48;

} // namespace

bool bvh2_from_reference(const uint8_t* blob, size_t bytes, uint32_t num_faces, BvhBuildResult& out, std::string& err) {
    out = BvhBuildResult{};
    if (!blob || bytes < 16) { err = "BLAS blob shorter than its header"; return false; }
    uint32_t hdr[4];
    std::memcpy(hdr, blob, 16);
    const uint64_t nn = hdr[0], nt = hdr[1];
    if (nn == 0 || nt == 0) { err = "BLAS blob without nodes or triangles"; return false; }
    if (16 + nn * sizeof(RefNode2) + nt * kRefTri1Bytes > bytes) { err = "BLAS blob shorter than its node and triangle arrays"; return false; }
    if (nt >= (uint64_t)kMaxLeafFirst) { err = "too many triangles for the leaf encoding"; return false; }
    std::vector<RefNode2> rn(nn);
    std::memcpy(rn.data(), blob + 16, nn * sizeof(RefNode2));
    const uint8_t* tris = blob + 16 + nn * sizeof(RefNode2);
    // slot -> face, and the leaf each slot starts
    out.prim_order.resize(nt);
    std::vector<uint8_t> ends(nt);
    for (uint64_t s = 0; s < nt; ++s) {
        uint32_t pid;
        std::memcpy(&pid, tris + s * kRefTri1Bytes + 44, 4);
        ends[s] = (pid >> 31) != 0;
        pid &= 0x7FFFFFFFu;
        if (pid >= num_faces) { err = "Tri1 prim_id beyond the mesh's faces"; return false; }
        out.prim_order[s] = pid;
    }
    auto leaf_count = [&](uint64_t first, uint32_t& count) {
        uint64_t s = first;
        while (s < nt && !ends[s]) ++s;
        if (s >= nt) return false;
        count = (uint32_t)(s - first + 1);
        return true;
    };
    const int max_leaf = 1 << kLeafCountBits;
    // A reference leaf of more than max_leaf triangles becomes a balanced
    // subtree of inner nodes over slices of it; every node of that subtree
    // keeps the leaf's box (conservative: each slice lies inside it).
    std::vector<int> ndepth; // levels below each output node (for the stack bound)
    struct Item { int64_t src; int out; int depth; };
    std::vector<Item> stack;
    out.nodes.emplace_back();
    stack.push_back({0, 0, 1});
    std::vector<char> seen(nn, 0);
    int depth = 1;
    // child boxes get the same pad as igx's own builder (pad_box, set_child),
    // so closest hits through an imported tree do not depend on its grouping
    // either; Node2 keeps a child box as lo.x, hi.x, lo.y, hi.y, lo.z, hi.z
    auto put_box = [&](int o, int k, const float* box) {
        Box b;
        for (int a = 0; a < 3; ++a) {
            b.lo[a] = box[2 * a];
            b.hi[a] = box[2 * a + 1];
        }
        const Box p = pad_box(b);
        float* dst = out.nodes[o].b + 6 * k;
        for (int a = 0; a < 3; ++a) {
            dst[2 * a] = p.lo[a];
            dst[2 * a + 1] = p.hi[a];
        }
    };
    // child k of output node `o`: set box + ref, creating split-leaf nodes as needed
    std::function<void(int, int, const float*, uint64_t, uint32_t, int)> put_leaf =
        [&](int o, int k, const float* box, uint64_t first, uint32_t count, int d) {
            put_box(o, k, box);
            if (count <= (uint32_t)max_leaf) {
                out.nodes[o].ref[k] = encode_leaf((int32_t)first, (int32_t)count);
                return;
            }
            const int idx = (int)out.nodes.size();
            out.nodes.emplace_back();
            out.nodes[o].ref[k] = idx;
            depth = std::max(depth, d + 1);
            const uint32_t half = count / 2;
            put_leaf(idx, 0, box, first, half, d + 1);
            put_leaf(idx, 1, box, first + half, count - half, d + 1);
        };
    bool root_leaf = false;
    while (!stack.empty()) {
        Item it = stack.back();
        stack.pop_back();
        if (it.src < 0 || (uint64_t)it.src >= nn) { err = "Node2 child index out of range"; return false; }
        if (seen[it.src]++) { err = "Node2 graph is not a tree"; return false; }
        depth = std::max(depth, it.depth);
        RefNode2 n = rn[it.src];
        // a cut-out child (0) repeats its sibling: harmless for closest and any
        // hit -- except under the root wrapping a single leaf
        // (BvhNAdapter.h:94-98), where the copy would be expanded a second time
        // when the leaf splits into a subtree: that child becomes absent instead
        if (n.child[0] == 0 && n.child[1] == 0) { err = "Node2 without children"; return false; }
        int absent = -1;
        for (int k = 0; k < 2; ++k)
            if (n.child[k] == 0) {
                n.child[k] = n.child[1 - k];
                std::memcpy(n.b + 6 * k, n.b + 6 * (1 - k), 6 * sizeof(float));
                if (it.src == 0 && n.child[k] < 0) {
                    root_leaf = true;
                    absent = k;
                }
            }
        out.nodes[it.out].pad[0] = out.nodes[it.out].pad[1] = 0;
        for (int k = 0; k < 2; ++k) {
            const int32_t c = n.child[k];
            if (k == absent) continue;
            if (c > 0) {
                const int idx = (int)out.nodes.size();
                out.nodes.emplace_back();
                put_box(it.out, k, n.b + 6 * k);
                out.nodes[it.out].ref[k] = idx;
                stack.push_back({(int64_t)c - 1, idx, it.depth + 1});
            } else {
                const uint64_t first = (uint64_t)(~c);
                uint32_t count = 0;
                if (first >= nt || !leaf_count(first, count)) { err = "Tri1 leaf without its end marker"; return false; }
                put_leaf(it.out, k, n.b + 6 * k, first, count, it.depth);
            }
        }
        if (absent >= 0) {
            // +inf bounds: no slab test accepts the child (as absent 4-wide children)
            float* dst = out.nodes[it.out].b + 6 * absent;
            for (int a = 0; a < 6; ++a) dst[a] = INFINITY;
            out.nodes[it.out].ref[absent] = kEmptyRef;
        }
    }
    out.depth = depth;
    out.max_leaf = max_leaf;
    if (root_leaf && out.nodes.size() == 1 && out.nodes[0].ref[0] < 0) {
        out.root_is_leaf = true;
        out.root_leaf_ref = out.nodes[0].ref[0];
    }
    return true;
}

} // namespace igx
