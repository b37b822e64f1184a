// rt_bvh.cpp — SAH BVH2 builder over world-space triangles (see rt_bvh.h): 256-bin binned SAH
// over all three axes for ranges above 1,024 triangles, an exact sweep over the sorted centroids
// below (C3g: extend nodes per ray 4.40 at 32 bins -> 3.93, 6.04 -> 6.15 Grays/s).
#include "rt_bvh.h"

#include <algorithm>
#include <cstdlib>
#include <functional>
#include <stdexcept>
#include <cmath>
#include <cstring>

namespace rt {

namespace {

struct Box {
    float lo[3], hi[3];
    void reset() { for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; } }
    void grow(const Box& b) { for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); } }
    void grow(const float* p) { for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); } }
    float area() const {
        float d0 = hi[0] - lo[0], d1 = hi[1] - lo[1], d2 = hi[2] - lo[2];
        if (!(d0 >= 0.0f)) return 0.0f;
        return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
    }
};

struct TmpNode {
    Box box;
    int left = -1, right = -1;
    uint32_t start = 0, count = 0;
};

#ifndef RT_SAH_BINS
#define RT_SAH_BINS 256
#endif
constexpr int kBins = RT_SAH_BINS;   // binned-SAH buckets per axis
#ifndef RT_SAH_SWEEP
#define RT_SAH_SWEEP 1024
#endif
constexpr uint32_t kSweepMax = RT_SAH_SWEEP;   // ranges up to this size: exact SAH sweep over sorted centroids

struct Builder {
    const std::vector<Box>& tri_box;
    const std::vector<float>& cen;  // 3 per tri
    std::vector<uint32_t>& idx;
    std::vector<TmpNode> nodes;
    int max_leaf, depth_limit, max_depth = 0;

    Builder(const std::vector<Box>& tb, const std::vector<float>& c, std::vector<uint32_t>& i, int ml, int dl)
        : tri_box(tb), cen(c), idx(i), max_leaf(ml), depth_limit(dl) {}

    static int ceil_log2(uint32_t x) { int r = 0; while ((1u << r) < x) ++r; return r; }

    int make_leaf(uint32_t s, uint32_t e, const Box& b) {
        TmpNode n;
        n.box = b; n.start = s; n.count = e - s;
        nodes.push_back(n);
        return (int)nodes.size() - 1;
    }

    int build(uint32_t s, uint32_t e, int depth) {
        max_depth = std::max(max_depth, depth);
        Box b; b.reset();
        Box cb; cb.reset();
        for (uint32_t i = s; i < e; ++i) { b.grow(tri_box[idx[i]]); cb.grow(&cen[3 * idx[i]]); }
        uint32_t n = e - s;
        if (n <= 1) return make_leaf(s, e, b);
        // axis = largest centroid extent
        int axis = 0;
        float ext[3];
        for (int k = 0; k < 3; ++k) ext[k] = cb.hi[k] - cb.lo[k];
        if (ext[1] > ext[axis]) axis = 1;
        if (ext[2] > ext[axis]) axis = 2;
        uint32_t mid = s;
        bool median = depth + ceil_log2((n + max_leaf - 1) / max_leaf) >= depth_limit - 1;
        bool split_found = false;
        if (ext[axis] <= 0.0f) {
            // all centroids coincide: leaf if small, otherwise object-median
            if (n <= (uint32_t)max_leaf) return make_leaf(s, e, b);
            median = true;
        }
        if (!median && n <= kSweepMax) {
            // exact SAH: every split of the centroid order on each axis (ties by triangle index)
            std::vector<uint32_t> ord[3];
            std::vector<float> rarea(n);
            float best_cost = INFINITY;
            int best_axis = -1;
            uint32_t best_i = 0;
            for (int a = 0; a < 3; ++a) {
                ord[a].assign(idx.begin() + s, idx.begin() + e);
                std::sort(ord[a].begin(), ord[a].end(), [&](uint32_t x, uint32_t y) {
                    const float cx = cen[3 * x + a], cy = cen[3 * y + a];
                    return cx < cy || (cx == cy && x < y);
                });
                Box acc; acc.reset();
                for (uint32_t i = n; i-- > 1;) { acc.grow(tri_box[ord[a][i]]); rarea[i] = acc.area(); }
                acc.reset();
                for (uint32_t i = 1; i < n; ++i) {
                    acc.grow(tri_box[ord[a][i - 1]]);
                    const float cost = acc.area() * (float)i + rarea[i] * (float)(n - i);
                    if (cost < best_cost) { best_cost = cost; best_axis = a; best_i = i; }
                }
            }
            float pa = b.area();
            float split_cost = 1.0f + (pa > 0 ? best_cost / pa : INFINITY);   // C_trav = 1
            if (best_axis >= 0 && (split_cost < (float)n || n > (uint32_t)max_leaf)) {
                std::copy(ord[best_axis].begin(), ord[best_axis].end(), idx.begin() + s);
                mid = s + best_i;
                split_found = true;
            } else if (n <= (uint32_t)max_leaf) {
                return make_leaf(s, e, b);
            }
        } else if (!median) {
            // binned SAH over all three axes
            float best_cost = INFINITY;
            int best_axis = -1, best_bin = -1;
            for (int a = 0; a < 3; ++a) {
                if (ext[a] <= 0.0f) continue;
                Box bb[kBins];
                uint32_t bc[kBins] = {0};
                for (auto& x : bb) x.reset();
                float scale = kBins / ext[a];
                for (uint32_t i = s; i < e; ++i) {
                    int bi = (int)((cen[3 * idx[i] + a] - cb.lo[a]) * scale);
                    bi = std::min(std::max(bi, 0), kBins - 1);
                    bb[bi].grow(tri_box[idx[i]]);
                    bc[bi]++;
                }
                float rarea[kBins];
                uint32_t rcnt[kBins];
                Box acc; acc.reset();
                uint32_t c = 0;
                for (int i = kBins - 1; i > 0; --i) {
                    acc.grow(bb[i]); c += bc[i];
                    rarea[i] = acc.area(); rcnt[i] = c;
                }
                acc.reset(); c = 0;
                for (int i = 0; i < kBins - 1; ++i) {
                    acc.grow(bb[i]); c += bc[i];
                    if (c == 0 || rcnt[i + 1] == 0) continue;
                    float cost = acc.area() * c + rarea[i + 1] * rcnt[i + 1];
                    if (cost < best_cost) { best_cost = cost; best_axis = a; best_bin = i; }
                }
            }
            float pa = b.area();
            float leaf_cost = (float)n;                             // C_isect = 1
            float split_cost = 1.0f + (pa > 0 ? best_cost / pa : INFINITY);  // C_trav = 1
            if (best_axis >= 0 && (split_cost < leaf_cost || n > (uint32_t)max_leaf)) {
                float scale = kBins / ext[best_axis];
                auto it = std::partition(idx.begin() + s, idx.begin() + e, [&](uint32_t t) {
                    int bi = (int)((cen[3 * t + best_axis] - cb.lo[best_axis]) * scale);
                    bi = std::min(std::max(bi, 0), kBins - 1);
                    return bi <= best_bin;
                });
                mid = (uint32_t)(it - idx.begin());
                if (mid > s && mid < e) split_found = true;
            } else if (n <= (uint32_t)max_leaf) {
                return make_leaf(s, e, b);
            }
        }
        if (!split_found) {
            if (n <= (uint32_t)max_leaf && !median) return make_leaf(s, e, b);
            mid = s + n / 2;
            std::nth_element(idx.begin() + s, idx.begin() + mid, idx.begin() + e, [&](uint32_t x, uint32_t y) {
                float cx = cen[3 * x + axis], cy = cen[3 * y + axis];
                return cx < cy || (cx == cy && x < y);
            });
        }
        if (n <= (uint32_t)max_leaf && median) return make_leaf(s, e, b);
        int me = (int)nodes.size();
        nodes.emplace_back();
        nodes[me].box = b;
        int l = build(s, mid, depth + 1);
        int r = build(mid, e, depth + 1);
        nodes[me].left = l;
        nodes[me].right = r;
        return me;
    }
};

void set_child(Bvh2Node& n, int slot, const Box& b, float pad) {
    n.lx[2 * slot] = b.lo[0] - pad; n.lx[2 * slot + 1] = b.hi[0] + pad;
    n.ly[2 * slot] = b.lo[1] - pad; n.ly[2 * slot + 1] = b.hi[1] + pad;
    n.lz[2 * slot] = b.lo[2] - pad; n.lz[2 * slot + 1] = b.hi[2] + pad;
}

void set_empty(Bvh2Node& n, int slot) {
    n.lx[2 * slot] = INFINITY; n.lx[2 * slot + 1] = -INFINITY;
    n.ly[2 * slot] = INFINITY; n.ly[2 * slot + 1] = -INFINITY;
    n.lz[2 * slot] = INFINITY; n.lz[2 * slot + 1] = -INFINITY;
    n.child[slot] = -1;  // leaf at slot 0 with zero triangles
    n.count[slot] = 0;
}

}  // namespace

BvhResult build_bvh2(const float* v, uint32_t n, int max_leaf, int depth_limit) {
    BvhResult out;
    std::vector<Box> tb(n);
    std::vector<float> cen(3 * (size_t)n);
    float maxabs = 1.0f;
    for (uint32_t i = 0; i < n; ++i) {
        tb[i].reset();
        for (int k = 0; k < 3; ++k) tb[i].grow(v + 9 * (size_t)i + 3 * k);
        for (int a = 0; a < 3; ++a) {
            cen[3 * i + a] = 0.5f * (tb[i].lo[a] + tb[i].hi[a]);
            maxabs = std::max(maxabs, std::max(std::fabs(tb[i].lo[a]), std::fabs(tb[i].hi[a])));
        }
    }
    out.pad = 4e-6f * maxabs;
    std::vector<uint32_t> idx(n);
    for (uint32_t i = 0; i < n; ++i) idx[i] = i;
    Builder b(tb, cen, idx, max_leaf, depth_limit);
    b.nodes.reserve(2 * (size_t)n / std::max(1, max_leaf) + 16);
    if (n == 0) {
        Bvh2Node r;
        std::memset(&r, 0, sizeof r);
        set_empty(r, 0);
        set_empty(r, 1);
        out.nodes.push_back(r);
        out.parent.push_back(-1);
        return out;
    }
    int root = b.build(0, n, 0);
    out.max_depth = b.max_depth;
    out.tri_order = idx;
    // flatten: one Bvh2Node per inner TmpNode, DFS order
    std::vector<int> map(b.nodes.size(), -1);
    std::vector<int> stack;
    if (b.nodes[root].left < 0) {
        Bvh2Node r;
        std::memset(&r, 0, sizeof r);
        set_child(r, 0, b.nodes[root].box, out.pad);
        r.child[0] = ~(int32_t)b.nodes[root].start;
        r.count[0] = (int32_t)b.nodes[root].count;
        set_empty(r, 1);
        out.nodes.push_back(r);
        out.parent.push_back(-1);
        return out;
    }
    // assign indices in DFS (pre-order, left first)
    stack.push_back(root);
    std::vector<int> order;
    while (!stack.empty()) {
        int t = stack.back();
        stack.pop_back();
        map[t] = (int)order.size();
        order.push_back(t);
        const TmpNode& tn = b.nodes[t];
        if (b.nodes[tn.right].left >= 0) stack.push_back(tn.right);
        if (b.nodes[tn.left].left >= 0) stack.push_back(tn.left);
    }
    out.nodes.resize(order.size());
    out.parent.assign(order.size(), -1);
    for (size_t k = 0; k < order.size(); ++k) {
        const TmpNode& tn = b.nodes[order[k]];
        Bvh2Node& o = out.nodes[k];
        std::memset(&o, 0, sizeof o);
        int ch[2] = {tn.left, tn.right};
        for (int s = 0; s < 2; ++s) {
            const TmpNode& c = b.nodes[ch[s]];
            set_child(o, s, c.box, out.pad);
            if (c.left >= 0) {
                o.child[s] = map[ch[s]];
                o.count[s] = 0;
                out.parent[map[ch[s]]] = (int)k;
            } else {
                o.child[s] = ~(int32_t)c.start;
                o.count[s] = (int32_t)c.count;
            }
        }
    }
    return out;
}

void refit_bvh2(BvhResult& bvh, const float* v) {
    // children have larger indices than parents (pre-order) -> sweep backwards
    for (int k = (int)bvh.nodes.size() - 1; k >= 0; --k) {
        Bvh2Node& nd = bvh.nodes[k];
        for (int s = 0; s < 2; ++s) {
            Box b; b.reset();
            if (nd.child[s] >= 0) {
                const Bvh2Node& c = bvh.nodes[nd.child[s]];
                for (int cs = 0; cs < 2; ++cs) {
                    Box cb;
                    cb.lo[0] = c.lx[2 * cs] + bvh.pad; cb.hi[0] = c.lx[2 * cs + 1] - bvh.pad;
                    cb.lo[1] = c.ly[2 * cs] + bvh.pad; cb.hi[1] = c.ly[2 * cs + 1] - bvh.pad;
                    cb.lo[2] = c.lz[2 * cs] + bvh.pad; cb.hi[2] = c.lz[2 * cs + 1] - bvh.pad;
                    if (c.child[cs] < 0 && c.count[cs] == 0) continue;
                    b.grow(cb);
                }
            } else {
                if (nd.count[s] == 0) continue;
                uint32_t first = (uint32_t)~nd.child[s];
                for (int32_t t = 0; t < nd.count[s]; ++t) {
                    uint32_t tri = bvh.tri_order[first + t];
                    for (int q = 0; q < 3; ++q) b.grow(v + 9 * (size_t)tri + 3 * q);
                }
            }
            set_child(nd, s, b, bvh.pad);
        }
    }
}

}  // namespace rt

// ---- compressed 8-wide collapse ------------------------------------------------------------------
namespace rt {

namespace {
struct WItem {
    float lo[3], hi[3];
    bool leaf;
    int node;            // BVH2 node (internal)
    uint32_t start, count;  // leaf range in BVH2 triangle order
};

float item_area(const WItem& it) {
    float d0 = it.hi[0] - it.lo[0], d1 = it.hi[1] - it.lo[1], d2 = it.hi[2] - it.lo[2];
    return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
}

void bvh2_children(const BvhResult& b2, int k, std::vector<WItem>& out) {
    const Bvh2Node& n = b2.nodes[k];
    for (int s = 0; s < 2; ++s) {
        if (n.child[s] < 0 && n.count[s] == 0) continue;  // empty slot
        WItem it;
        it.lo[0] = n.lx[2 * s]; it.hi[0] = n.lx[2 * s + 1];
        it.lo[1] = n.ly[2 * s]; it.hi[1] = n.ly[2 * s + 1];
        it.lo[2] = n.lz[2 * s]; it.hi[2] = n.lz[2 * s + 1];
        it.leaf = n.child[s] < 0;
        it.node = it.leaf ? -1 : n.child[s];
        it.start = it.leaf ? (uint32_t)~n.child[s] : 0u;
        it.count = it.leaf ? (uint32_t)n.count[s] : 0u;
        out.push_back(it);
    }
}
}  // namespace

void quantize_bvh8_node(Bvh8Node& nd, const float clo[8][3], const float chi[8][3], const bool used[8]) {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int c = 0; c < 8; ++c)
        if (used[c])
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], (double)clo[c][a]); hi[a] = std::max(hi[a], (double)chi[c][a]); }
    for (int a = 0; a < 3; ++a) {
        if (!(lo[a] <= hi[a])) { lo[a] = 0.0; hi[a] = 0.0; }
        nd.p[a] = (float)lo[a];
        if ((double)nd.p[a] > lo[a]) nd.p[a] = std::nextafter(nd.p[a], -INFINITY);  // p <= every child lo
        double ext = hi[a] - (double)nd.p[a];
        int e = -100;
        if (ext > 0.0) {
            e = (int)std::ceil(std::log2(ext / 255.0));
            while (std::ldexp(255.0, e) < ext) ++e;
        }
        e = std::max(-126, std::min(127, e));
        nd.e[a] = (uint8_t)(e + 127);
        double inv = std::ldexp(1.0, -e);
        for (int c = 0; c < 8; ++c) {
            uint8_t ql = 255, qh = 0;
            if (used[c]) {
                double fl = std::floor(((double)clo[c][a] - (double)nd.p[a]) * inv);
                double fh = std::ceil(((double)chi[c][a] - (double)nd.p[a]) * inv);
                ql = (uint8_t)std::max(0.0, std::min(255.0, fl));
                qh = (uint8_t)std::max(0.0, std::min(255.0, fh));
            }
            nd.q[16 * a + c] = ql;
            nd.q[16 * a + 8 + c] = qh;
        }
    }
}

namespace {
struct Job { int b2node; uint32_t b8node; int depth; };

// One 8-wide node from its child items (internal children are queued as new jobs).
void emit_bvh8_node(const BvhResult& b2, const Job& job, std::vector<WItem>& items, std::vector<Job>& queue,
                    Bvh8Result& out);

// Subtree triangle range [start, start + count) of every BVH2 internal node: the builder
// partitions index ranges, so a subtree's triangles are contiguous in tri_order.
struct Range { uint32_t start, count; };
std::vector<Range> subtree_ranges(const BvhResult& b2) {
    std::vector<Range> r(b2.nodes.size(), Range{0xffffffffu, 0u});
    for (int k = (int)b2.nodes.size() - 1; k >= 0; --k) {   // children after parents (pre-order)
        const Bvh2Node& n = b2.nodes[k];
        for (int s = 0; s < 2; ++s) {
            if (n.child[s] < 0 && n.count[s] == 0) continue;
            const Range c = n.child[s] < 0 ? Range{(uint32_t)~n.child[s], (uint32_t)n.count[s]} : r[n.child[s]];
            r[k].start = std::min(r[k].start, c.start);
            r[k].count += c.count;
        }
    }
    return r;
}
}  // namespace

// SAH-optimal 8-wide collapse (after Ylitie, Karras, Laine, "Efficient Incoherent Ray Traversal
// on GPUs Through Compressed Wide BVHs", HPG 2017, §4): dynamic programming over the BVH2 for
// the cheapest way to represent every subtree with at most i (1..8) slots of its parent, a slot
// being a leaf (<= 4 triangles, the meta field's limit) or an 8-wide child node:
//   C(n, 1)  = min(A(n) * c_prim * tris(n)  [tris(n) <= 4],  A(n) * c_node + D(n, 8))
//   C(n, i)  = min(C(n, i - 1), D(n, i)),   D(n, j) = min_k C(l, k) + C(r, j - k)
// (Round 1's greedy collapse, opening the largest child until 8, left 47 % of the C3g tree's
// nodes with two used slots whose box tests were mostly spent on empty slots.)
Bvh8Result collapse_bvh8_dp(const BvhResult& b2, float c_node, float c_prim) {
    // DP nodes: BVH2 internal nodes keep their index; leaf slots are appended
    struct DN { float area; uint32_t start, count; int kid[2]; bool leaf; WItem item; };
    const size_t ni = b2.nodes.size();
    std::vector<DN> dn(ni);
    const std::vector<Range> ranges = subtree_ranges(b2);
    for (size_t k = 0; k < ni; ++k) {
        dn[k].leaf = false;
        dn[k].start = ranges[k].start;
        dn[k].count = ranges[k].count;
    }
    for (size_t k = 0; k < ni; ++k) {
        std::vector<WItem> kids;
        bvh2_children(b2, (int)k, kids);
        dn[k].kid[0] = dn[k].kid[1] = -1;
        for (size_t s = 0; s < kids.size(); ++s) {
            int id;
            if (kids[s].leaf) {
                DN l;
                l.leaf = true;
                l.start = kids[s].start;
                l.count = kids[s].count;
                l.kid[0] = l.kid[1] = -1;
                l.item = kids[s];
                l.area = item_area(kids[s]);
                dn.push_back(l);
                id = (int)dn.size() - 1;
            } else {
                id = kids[s].node;
                dn[id].item = kids[s];
                dn[id].area = item_area(kids[s]);
            }
            dn[k].kid[s] = id;
        }
    }
    {   // the root's box: the union of its slots
        WItem r;
        for (int a = 0; a < 3; ++a) { r.lo[a] = INFINITY; r.hi[a] = -INFINITY; }
        for (int s = 0; s < 2; ++s) {
            const int c = dn[0].kid[s];
            if (c < 0) continue;
            for (int a = 0; a < 3; ++a) { r.lo[a] = std::min(r.lo[a], dn[c].item.lo[a]); r.hi[a] = std::max(r.hi[a], dn[c].item.hi[a]); }
        }
        r.leaf = false;
        r.node = 0;
        dn[0].item = r;
        dn[0].area = item_area(r);
    }
    const size_t nd = dn.size();
    std::vector<float> C(nd * 9, INFINITY);           // C(n, i), i = 1..8
    std::vector<int8_t> choice(nd * 9, 0);            // i = 1: 1 leaf / 2 node; i >= 2: 0 = C(n, i-1), k = split
    std::vector<int8_t> split8(nd, 1);                // best k of D(n, 8) (the node's own slots)
    constexpr uint32_t kLeafMax = 4;
    auto cost_of = [&](int id) {
        DN& n = dn[id];
        const float leaf = n.count <= kLeafMax ? n.area * c_prim * (float)n.count : INFINITY;
        if (n.leaf) {
            for (int i = 1; i <= 8; ++i) { C[id * 9 + i] = leaf; choice[id * 9 + i] = 1; }
            return;
        }
        float D[9];
        int8_t K[9];
        for (int j = 2; j <= 8; ++j) {
            D[j] = INFINITY;
            K[j] = 1;
            const int l = n.kid[0], r = n.kid[1];
            if (l < 0 || r < 0) {   // one-child node: the child alone
                const int c = l >= 0 ? l : r;
                D[j] = C[c * 9 + j - 1];
                K[j] = (int8_t)(j - 1);
                continue;
            }
            for (int k = 1; k < j; ++k) {
                const float v = C[l * 9 + k] + C[r * 9 + j - k];
                if (v < D[j]) { D[j] = v; K[j] = (int8_t)k; }
            }
        }
        const float node = n.area * c_node + D[8];
        split8[id] = K[8];
        C[id * 9 + 1] = std::min(leaf, node);
        // a leaf slot holds at most kLeafMax triangles (the tri_valid nibble): with both costs
        // infinite (box areas overflowing) a larger subtree must stay a node
        choice[id * 9 + 1] = (n.count <= kLeafMax && leaf <= node) ? 1 : 2;
        for (int i = 2; i <= 8; ++i) {
            if (D[i] < C[id * 9 + i - 1]) { C[id * 9 + i] = D[i]; choice[id * 9 + i] = K[i]; }
            else { C[id * 9 + i] = C[id * 9 + i - 1]; choice[id * 9 + i] = 0; }
        }
    };
    for (size_t id = ni; id < nd; ++id) cost_of((int)id);          // leaves
    for (int id = (int)ni - 1; id >= 0; --id) cost_of(id);        // internal, children first
    // slots of subtree `id` with budget j
    std::function<void(int, int, std::vector<WItem>&)> expand = [&](int id, int j, std::vector<WItem>& items) {
        const DN& n = dn[id];
        while (j >= 2 && choice[id * 9 + j] == 0) --j;
        if (j >= 2 && !n.leaf) {
            const int k = choice[id * 9 + j];
            const int l = n.kid[0], r = n.kid[1];
            if (l < 0 || r < 0) { expand(l >= 0 ? l : r, j - 1 > 0 ? j - 1 : 1, items); return; }
            expand(l, k, items);
            expand(r, j - k, items);
            return;
        }
        WItem it = n.item;
        if (n.leaf || choice[id * 9 + 1] == 1) {   // a leaf slot over the subtree's triangles
            it.leaf = true;
            it.node = -1;
            it.start = n.start;
            it.count = n.count;
        } else {
            it.leaf = false;
            it.node = id;
        }
        items.push_back(it);
    };
    Bvh8Result out;
    out.pad = b2.pad;
    std::vector<Job> queue;
    out.nodes.emplace_back();
    out.parent.push_back(-1);
    queue.push_back({0, 0u, 0});
    for (size_t qi = 0; qi < queue.size(); ++qi) {
        const Job job = queue[qi];
        std::vector<WItem> items;
        const DN& n = dn[job.b2node];
        if (n.kid[0] >= 0 && n.kid[1] >= 0) {
            const int k = split8[job.b2node];
            expand(n.kid[0], k, items);
            expand(n.kid[1], 8 - k, items);
        } else {
            bvh2_children(b2, job.b2node, items);
        }
        emit_bvh8_node(b2, job, items, queue, out);
    }
    out.node_box.resize(6 * out.nodes.size());
    return out;
}

namespace {
void emit_bvh8_node(const BvhResult& b2, const Job& job, std::vector<WItem>& items, std::vector<Job>& queue,
                    Bvh8Result& out) {
        out.max_depth = std::max(out.max_depth, job.depth + 1);
        // slot order: centroid along the longest axis of the node box
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (auto& it : items)
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], it.lo[a]); hi[a] = std::max(hi[a], it.hi[a]); }
        int axis = 0;
        for (int a = 1; a < 3; ++a) if (hi[a] - lo[a] > hi[axis] - lo[axis]) axis = a;
        std::stable_sort(items.begin(), items.end(), [&](const WItem& x, const WItem& y) {
            return x.lo[axis] + x.hi[axis] < y.lo[axis] + y.hi[axis];
        });
        // internal children first (slot = rank), then the leaves, each kind in centroid order
        std::stable_partition(items.begin(), items.end(), [](const WItem& x) { return !x.leaf; });
        Bvh8Node nd;
        std::memset(&nd, 0, sizeof nd);
        uint32_t n_internal = 0, n_tris = 0;
        for (auto& it : items) { if (!it.leaf) ++n_internal; else n_tris += it.count; }
        nd.axis_k = (uint8_t)(axis | (n_internal << 4));
        nd.child_base = (uint32_t)out.nodes.size();
        nd.tri_base = (uint32_t)out.tri_order.size();
        float clo[8][3], chi[8][3];
        bool used[8] = {false, false, false, false, false, false, false, false};
        uint32_t rank = 0;
        for (size_t c = 0; c < items.size(); ++c) {
            const WItem& it = items[c];
            used[c] = true;
            for (int a = 0; a < 3; ++a) { clo[c][a] = it.lo[a]; chi[c][a] = it.hi[a]; }
            if (!it.leaf) {
                uint32_t child = nd.child_base + rank;
                ++rank;
                queue.push_back({it.node, child, job.depth + 1});
            } else {
                const uint32_t j = (uint32_t)c - n_internal;
                if (it.count > 4) throw std::runtime_error("bvh8: leaf slot with more than 4 triangles");
                nd.tri_valid |= ((1u << it.count) - 1u) << (4 * j);
                for (uint32_t t = 0; t < it.count; ++t) out.tri_order.push_back(b2.tri_order[it.start + t]);
            }
        }
        (void)n_tris;
        quantize_bvh8_node(nd, clo, chi, used);
        out.nodes[job.b8node] = nd;
        for (uint32_t r = 0; r < n_internal; ++r) {
            out.nodes.emplace_back();
            out.parent.push_back((int32_t)job.b8node);
        }
        // node box (for refit / diagnostics)
        if (out.node_box.size() < 6 * out.nodes.size()) out.node_box.resize(6 * out.nodes.size(), 0.0f);
        for (int a = 0; a < 3; ++a) {
            out.node_box[6 * job.b8node + a] = lo[a];
            out.node_box[6 * job.b8node + 3 + a] = hi[a];
        }
}
}  // namespace

}  // namespace rt
