// rt_bvh.h — host BVH builder (replaces the driver-internal Metal BLAS/TLAS build,
// Utilities.swift:101-290 / Renderer.swift:464-606).
//
// Layout in HBM: one flat BVH2 over world-space triangles. Each 64-byte node
// holds the AABBs of BOTH children, so one node fetch = three 16-byte loads answers the two
// slab tests of a traversal step:
//   lx = (c0.lo.x, c0.hi.x, c1.lo.x, c1.hi.x), ly, lz likewise,
//   child[i] >= 0: inner node index; child[i] < 0: leaf, first triangle = ~child[i],
//   count[i] triangles (count 0 + inverted box = empty slot).
// Boxes are padded outward so the slab test is conservative w.r.t. the watertight triangle
// test: traversal then finds exactly the brute-force closest hit (ties broken by the smaller
// original triangle id), independent of tree shape — which is what makes the GPU result equal
// to the oracle's (which builds its own, different tree).
#pragma once
#include <stdint.h>
#include <vector>

namespace rt {

struct alignas(16) Bvh2Node {
    float lx[4];
    float ly[4];
    float lz[4];
    int32_t child[2];
    int32_t count[2];
};
static_assert(sizeof(Bvh2Node) == 64, "node is 64 B");

struct BvhResult {
    std::vector<Bvh2Node> nodes;
    std::vector<uint32_t> tri_order;   // BVH slot -> original triangle id
    std::vector<int32_t> parent;       // node -> parent node (-1 root), for refit
    int max_depth = 0;
    float pad = 0.0f;                  // absolute box padding used
};

// Compressed 8-wide node (80 B = five 16-byte loads; after Ylitie, Karras, Laine, HPG 2017).
// Child boxes are quantized to 8 bits per plane against the node's origin p and per-axis
// power-of-two scale 2^e, rounded outward, so the dequantized box p + q * 2^e always encloses
// the (padded) BVH2 box it came from: traversal stays conservative and exact.
//   slots: the k internal children first (slot r = rank r, node index child_base + r), then the
//            leaves (leaf j in slot k + j), then unused slots with an empty box (qlo = 255 > qhi = 0)
//   k:       bits 4..7 of axis_k (bits 0..1: the sort axis)
//   tri_valid: one nibble per leaf, bit 4j + i set when leaf j has a triangle i (1..4 triangles);
//            the leaves' triangles are contiguous from tri_base in slot order, so triangle (j, i)
//            is tri_base + popcount(tri_valid & ((1 << (4j + i)) - 1)).  A node test turns its
//            hit slots into internal ranks (the low k bits) and a triangle mask in nibble space
//            (the leaf bits spread to nibbles, & tri_valid) without per-child branches.
//   axis: children of each kind are sorted by centroid along `axis`; rays with d[axis] < 0 visit
//   them in reverse slot order (approximate front-to-back order for closest-hit culling).
// Byte order of q: [qlo.x 0..7][qhi.x 0..7][qlo.y ..][qhi.y ..][qlo.z ..][qhi.z ..].
struct alignas(16) Bvh8Node {
    float p[3];
    uint8_t e[3];     // biased exponents (e + 127): scale = 2^(e - 127)
    uint8_t axis_k;   // sort axis | k << 4
    uint32_t child_base;
    uint32_t tri_base;
    uint32_t tri_valid;
    uint32_t reserved;
    uint8_t q[48];
};
static_assert(sizeof(Bvh8Node) == 80, "wide node is 80 B");

struct Bvh8Result {
    std::vector<Bvh8Node> nodes;
    std::vector<uint32_t> tri_order;   // BVH8 triangle slot -> original triangle id
    std::vector<int32_t> parent;       // node -> parent node (-1 root)
    std::vector<float> node_box;       // 6 floats per node: lo xyz, hi xyz (padded), for refit
    int max_depth = 0;
    float pad = 0.0f;
};

// SAH-optimal collapse by dynamic programming over the BVH2 (Ylitie et al. 2017): every node
// slot is a leaf of <= 4 triangles or a child node, chosen to minimise
// sum(A(node) * c_node) + sum(A(leaf) * c_prim * triangles).  Best on a BVH2 with 1-triangle leaves.
Bvh8Result collapse_bvh8_dp(const BvhResult& b2, float c_node, float c_prim);

#if defined(__HIPCC__)
#define RT_BVH_HD __host__ __device__
#else
#define RT_BVH_HD
#endif
// Leaf j of a node: its first triangle slot (relative to tri_base) and its triangle count.
RT_BVH_HD inline uint32_t bvh8_leaf_first(uint32_t tri_valid, int j) {
    return (uint32_t)__builtin_popcount(j ? tri_valid & ((1u << (4 * j)) - 1u) : 0u);
}
RT_BVH_HD inline uint32_t bvh8_leaf_count(uint32_t tri_valid, int j) { return (uint32_t)__builtin_popcount((tri_valid >> (4 * j)) & 15u); }

// Re-quantize node n from its children's boxes (children: node_box of internal children, leaf
// triangle bounds from tri_verts in BVH8 triangle order, padded).  Host mirror of the refit kernel.
void quantize_bvh8_node(Bvh8Node& node, const float child_lo[8][3], const float child_hi[8][3], const bool used[8]);

// tri_verts: 9 floats per triangle (v0, v1, v2 world space), n triangles.
// max_depth_limit: the traversal stack bound; the builder falls back to median splits near it.
BvhResult build_bvh2(const float* tri_verts, uint32_t n, int max_leaf, int max_depth_limit);

// Recompute the boxes of an existing topology from new triangle positions (host refit;
// the device refit kernel mirrors it).
void refit_bvh2(BvhResult& bvh, const float* tri_verts);

}  // namespace rt
