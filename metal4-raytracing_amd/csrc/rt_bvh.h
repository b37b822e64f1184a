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

// tri_verts: 9 floats per triangle (v0, v1, v2 world space), n triangles.
// max_depth_limit: the traversal stack bound; the builder falls back to median splits near it.
BvhResult build_bvh2(const float* tri_verts, uint32_t n, int max_leaf, int max_depth_limit);

// Recompute the boxes of an existing topology from new triangle positions (host refit;
// the device refit kernel mirrors it).
void refit_bvh2(BvhResult& bvh, const float* tri_verts);

}  // namespace rt
