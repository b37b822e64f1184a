// rt_device.h — device-side scene layout and traversal shared by the HIP kernels.
//
// Data layout in HBM:
//   tris[16*k + ..]    float   64 B per BVH slot k: world-space v0, v1, v2 as (x, y, z, x, y) each
//                              (15 floats: a ray's (kz, kx, ky) window of every vertex is contiguous,
//                              tri_window), then the original triangle id (bits) in float 15
//   nodes[n]           Bvh2Node (64 B: both children's boxes, see rt_bvh.h)
//   tri_info[id]       uint4   (i0, i1, i2, inst<<8 | submesh) global vertex indices, original order
//   pos/prev_pos/nrm   float4  object-space vertex streams, all meshes concatenated (16 B stride,
//                              Model.vertexDescriptor, Model.swift:304-341)
//   inst/prev_inst     float   12 per instance: MTLPackedFloat4x3 column-major
//   materials[slot]    Material, slot = inst * max_submeshes + submesh (Raytracing.metal:337-339)
//   lights[]           Light
#pragma once
#include <hip/hip_runtime.h>
#include "rt_math.h"
#include "../../include/rt_types.h"
#include "rt_bvh.h"

namespace rt {

constexpr int kStackSize = 16;   // per-thread traversal stack entries (LDS): node groups of the 8-wide BVH
constexpr int kBlock = 256;      // threads per block for the traversal kernels

struct DevScene {
    const float* tris;   // 16 floats per slot (kTriFloats)
    const Bvh8Node* nodes8;
    const uint4* tri_info;
    const float4* pos;
    const float4* prev_pos;
    const float4* nrm;
    // per original triangle, 64 B: the object-space normals of vertices (i1, i2, i0) -- the order
    // :391 weights them by (u, v, w) -- with tri_info's w word in the first record's w, and the
    // triangle's tri_info (as bits) in the fourth: one cache line per shaded hit instead of the
    // tri_info record and three vertex-normal gathers behind it (build_tri_nrm, rt_util.hip)
    const float4* tri_nrm;
    const float* inst;
    const float* prev_inst;
    const Material* materials;
    const Light* lights;
    const HaltonDim* halton;
    const uint16_t* tri_bin;   // per original triangle: its BVH leaf slot * kSortMaxBins / num_tris
    int max_submeshes;
    int num_materials;         // instances * max_submeshes
    int num_tris;
    int num_nodes8;
    // texture path, set for textured scenes only (textured != 0)
    const uchar4* tex_texels = nullptr;   // RGBA8 pool, each texture row-major from its top row
    const uint4* tex_info = nullptr;      // per texture: (first texel, width, height, 0)
    const int4* mat_tex = nullptr;        // per material slot: (flags, t0, t1, t2), (t3, t4, t5, t6)
    const float2* uv = nullptr;           // per vertex
    const float* tex_lut = nullptr;       // byte -> float: [0, 256) linear, [256, 512) sRGB
    int textured = 0;
};

struct Hit {
    float t;
    uint32_t id;   // original triangle id, 0xffffffff = miss
    float u, v;
};

__host__ __device__ __forceinline__ f3 ld3(const float4& v) { return mk3(v.x, v.y, v.z); }

// ---- triangle records (64 B per BVH slot) ---------------------------------------------------------
constexpr int kTriFloats = 16;
__host__ __device__ __forceinline__ const float* tri_rec(const float* tris, uint32_t slot) {
    return tris + (size_t)kTriFloats * slot;
}
// vertex v of a record as the ray's (kz, kx, ky) components: three consecutive floats (one 12-B load)
struct Win3 { float a, b, c; };
__host__ __device__ __forceinline__ f3 tri_window(const float* rec, int v, int kz) {
    const Win3 w = *reinterpret_cast<const Win3*>(rec + 5 * v + kz);
    return mk3(w.a, w.b, w.c);
}
__host__ __device__ __forceinline__ uint32_t tri_id_at(const float* tris, uint32_t fidx) {   // fidx = slot * 16
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tris) + fidx * 4u + 60u);
}
// the same from the array base and a 32-bit float index (slot * 16 + 5 v + kz): uniform base,
// one 32-bit offset per lane (triangle arrays stay below 2^26 slots)
__host__ __device__ __forceinline__ f3 tri_window_at(const float* tris, uint32_t fidx) {
    const Win3 w = *reinterpret_cast<const Win3*>(reinterpret_cast<const char*>(tris) + fidx * 4u);
    return mk3(w.a, w.b, w.c);
}
__host__ __device__ __forceinline__ uint32_t tri_id(const float* rec) { return __builtin_bit_cast(uint32_t, rec[15]); }
// world-space vertex v (refit, host tools)
__host__ __device__ __forceinline__ f3 tri_vertex(const float* rec, int v) { return mk3(rec[5 * v], rec[5 * v + 1], rec[5 * v + 2]); }
// writes the record of world-space vertices w[0..8] and triangle id
__host__ __device__ __forceinline__ void tri_store(float* rec, const float* w, uint32_t id) {
    for (int v = 0; v < 3; ++v) {
        rec[5 * v + 0] = w[3 * v + 0];
        rec[5 * v + 1] = w[3 * v + 1];
        rec[5 * v + 2] = w[3 * v + 2];
        rec[5 * v + 3] = w[3 * v + 0];
        rec[5 * v + 4] = w[3 * v + 1];
    }
    rec[15] = __builtin_bit_cast(float, id);
}

// Object->world with the instance's packed 4x3 (columns c0..c3): ((c0*x + c1*y) + c2*z) + c3*w
__host__ __device__ __forceinline__ f3 xform(const float* m, f3 p, float w) {
    f3 c0 = mk3(m[0], m[1], m[2]), c1 = mk3(m[3], m[4], m[5]), c2 = mk3(m[6], m[7], m[8]), c3 = mk3(m[9], m[10], m[11]);
    return ((c0 * p.x + c1 * p.y) + c2 * p.z) + c3 * w;
}

struct TraceCounters {
    uint32_t nodes;       // 8-wide nodes fetched from global memory
    uint32_t tris;        // triangles tested
    uint32_t lds_nodes;   // node tests served from the LDS copy of the top levels (no memory traffic)
};

// ---- compressed 8-wide BVH traversal (rt_bvh.h Bvh8Node) --------------------------------------
struct RaySetup {
    f3 o;      // the origin in the ray's (kz, kx, ky) order (the triangle test's frame)
    RayPre pre;
    float ix, iy, iz;   // 1 / d (safe)
    float ox, oy, oz;   // o * (1 / d)
    uint32_t dneg;      // bit a = (d[a] < 0)
};

__host__ __device__ __forceinline__ RaySetup ray_setup(f3 o, f3 d) {
    RaySetup R;
    R.pre = ray_precompute(d);
    R.o = rot3(o, R.pre.kz);
    // slab reciprocals only steer the (conservative, padded) box tests: the 1-ulp hardware
    // reciprocal is enough on the device; triangle tests use the exact RayPre divisions.
    auto safe_inv = [](float x) {
        x = fabsf(x) < 1e-30f ? copysignf(1e-30f, x) : x;
#if defined(__HIP_DEVICE_COMPILE__)
        return __builtin_amdgcn_rcpf(x);
#else
        return 1.0f / x;
#endif
    };
    R.ix = safe_inv(d.x);
    R.iy = safe_inv(d.y);
    R.iz = safe_inv(d.z);
    R.ox = o.x * R.ix;
    R.oy = o.y * R.iy;
    R.oz = o.z * R.iz;
    R.dneg = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    return R;
}

__host__ __device__ __forceinline__ float byte_f(uint32_t w, int b) { return (float)((w >> (8 * b)) & 0xffu); }

// Slab-test the 8 children of node `ni` (five 16-byte loads).  Returns the internal children hit
// (bit r = internal rank r), the triangles to test (bit k = triangle tri_base + k), and the
// traversal direction of the node's slot order.
// The five 16-byte words of a node (from global memory or an LDS copy).
struct NodeU3 { uint32_t x, y, z; };   // child_base, tri_base, tri_valid (the reserved word is not read)
struct NodeWords {
    float4 h0;
    NodeU3 h1;
    uint4 qx, qy, qz;
};
// (32-bit byte offsets from the array base: the loads take the uniform base in SGPRs and one
// 32-bit offset per lane, no 64-bit address arithmetic; node arrays stay below 2^23 nodes)
__host__ __device__ __forceinline__ NodeWords load_node8(const Bvh8Node* nodes, uint32_t ni) {
    const char* base = reinterpret_cast<const char*>(nodes);
    const uint32_t o = ni * (uint32_t)sizeof(Bvh8Node);
    NodeWords w;
    w.h0 = *reinterpret_cast<const float4*>(base + o);
    w.h1 = *reinterpret_cast<const NodeU3*>(base + (o + 16u));   // 12 B: 76 of the node's 80 B are read
    w.qx = *reinterpret_cast<const uint4*>(base + (o + 32u));
    w.qy = *reinterpret_cast<const uint4*>(base + (o + 48u));
    w.qz = *reinterpret_cast<const uint4*>(base + (o + 64u));
    return w;
}

// Leaf bits j (j < 8) -> nibbles 4j..4j+3 (the triangle space of Bvh8Node::tri_valid).
__host__ __device__ __forceinline__ uint32_t spread_nibbles(uint32_t x) {
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    x = (x | (x << 3)) & 0x11111111u;
    return x * 15u;
}
// Triangle slot of bit k of a node test's triangle mask (nibble space): tri_base + the valid bits below k.
__host__ __device__ __forceinline__ uint32_t tri_slot(uint32_t tri_base, uint32_t tri_valid, int k) {
    return tri_base + (uint32_t)__builtin_popcount(tri_valid & ((1u << k) - 1u));
}

// Slab-test the 8 children of a node.  Outputs: the internal children hit (bit r = internal rank r
// = slot r), the triangles to test (nibble space: bit 4j + i = triangle i of leaf j, see
// tri_slot), the node's tri_valid word, and the traversal direction of the slot order.
// Branch-free over the children: each child only sets its bit of the hit-slot mask; the
// internal / leaf split and the triangle mask follow from the node's k and tri_valid once per node.
__host__ __device__ __forceinline__ void test_node8_words(const NodeWords& W, const RaySetup& R, float tmin, float tmax,
                                                          uint32_t& ihits, uint32_t& tmask, uint32_t& tvalid,
                                                          uint32_t& child_base, uint32_t& tri_base, bool& flip) {
    const float4 h0 = W.h0;
    const NodeU3 h1 = W.h1;
    const uint4 qx = W.qx, qy = W.qy, qz = W.qz;
    const uint32_t ew = __builtin_bit_cast(uint32_t, h0.w);
    const float sx = __builtin_bit_cast(float, (ew & 0xffu) << 23);
    const float sy = __builtin_bit_cast(float, ((ew >> 8) & 0xffu) << 23);
    const float sz = __builtin_bit_cast(float, ((ew >> 16) & 0xffu) << 23);
    const int axis = (int)((ew >> 24) & 3u);
    const uint32_t k_int = ew >> 28;   // internal children: slots 0 .. k_int - 1
    const float ax = sx * R.ix, ay = sy * R.iy, az = sz * R.iz;
    const float bx = __builtin_fmaf(h0.x, R.ix, -R.ox);
    const float by = __builtin_fmaf(h0.y, R.iy, -R.oy);
    const float bz = __builtin_fmaf(h0.z, R.iz, -R.oz);
    // near / far planes by direction sign
    const uint32_t nx0 = R.ix >= 0.0f ? qx.x : qx.z, nx1 = R.ix >= 0.0f ? qx.y : qx.w;
    const uint32_t fx0 = R.ix >= 0.0f ? qx.z : qx.x, fx1 = R.ix >= 0.0f ? qx.w : qx.y;
    const uint32_t ny0 = R.iy >= 0.0f ? qy.x : qy.z, ny1 = R.iy >= 0.0f ? qy.y : qy.w;
    const uint32_t fy0 = R.iy >= 0.0f ? qy.z : qy.x, fy1 = R.iy >= 0.0f ? qy.w : qy.y;
    const uint32_t nz0 = R.iz >= 0.0f ? qz.x : qz.z, nz1 = R.iz >= 0.0f ? qz.y : qz.w;
    const uint32_t fz0 = R.iz >= 0.0f ? qz.z : qz.x, fz1 = R.iz >= 0.0f ? qz.w : qz.y;
    const float tf_max = tmax * 1.0000004f;
    uint32_t hm = 0;
    #pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int b = c & 3;
        const uint32_t wnx = c < 4 ? nx0 : nx1, wfx = c < 4 ? fx0 : fx1;
        const uint32_t wny = c < 4 ? ny0 : ny1, wfy = c < 4 ? fy0 : fy1;
        const uint32_t wnz = c < 4 ? nz0 : nz1, wfz = c < 4 ? fz0 : fz1;
        const float tnx = __builtin_fmaf(byte_f(wnx, b), ax, bx), tfx = __builtin_fmaf(byte_f(wfx, b), ax, bx);
        const float tny = __builtin_fmaf(byte_f(wny, b), ay, by), tfy = __builtin_fmaf(byte_f(wfy, b), ay, by);
        const float tnz = __builtin_fmaf(byte_f(wnz, b), az, bz), tfz = __builtin_fmaf(byte_f(wfz, b), az, bz);
        const float tn = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, tmin));
        const float tf = fminf(fminf(tfx, tfy), fminf(tfz, tf_max));
        const bool hit = tn <= tf;
        hm |= hit ? (1u << c) : 0u;
    }
    ihits = hm & ((1u << k_int) - 1u);
    tmask = spread_nibbles(hm >> k_int) & h1.z;
    tvalid = h1.z;
    child_base = h1.x;
    tri_base = h1.y;
    flip = (R.dneg >> axis) & 1u;   // bit select: a dynamic pick of R.d lowers to a scratch access
}

__host__ __device__ __forceinline__ void test_node8(const Bvh8Node* nodes, uint32_t ni, const RaySetup& R, float tmin,
                                                    float tmax, uint32_t& ihits, uint32_t& tmask, uint32_t& tvalid,
                                                    uint32_t& child_base, uint32_t& tri_base, bool& flip) {
    test_node8_words(load_node8(nodes, ni), R, tmin, tmax, ihits, tmask, tvalid, child_base, tri_base, flip);
}

__host__ __device__ __forceinline__ int lowest_bit(uint32_t m) { return __builtin_ctz(m); }
__host__ __device__ __forceinline__ int highest_bit(uint32_t m) { return 31 - __builtin_clz(m); }

// Stack entry of a node group: child_base << 9 | flip << 8 | remaining internal hits.
__host__ __device__ __forceinline__ uint32_t pack_group(uint32_t base, bool flip, uint32_t hits) {
    return (base << 9) | ((uint32_t)flip << 8) | hits;
}

// Closest-hit (ANY=false) / any-hit (ANY=true) traversal of the 8-wide BVH. Triangles found by a
// node test are intersected before the next node is fetched (they shrink `best` first).
template <bool ANY, bool COUNT>
__host__ __device__ __forceinline__ bool trace8(const DevScene& S, f3 o, f3 d, float tmin, float tmax, Hit& hit,
                                                int* stack, TraceCounters& cnt, bool& overflow) {
    const RaySetup R = ray_setup(o, d);
    float best = tmax, bu = 0.0f, bv = 0.0f;
    uint32_t best_id = 0xffffffffu;
    uint32_t g_base = 0, g_hits = 1, t_base = 0, t_mask = 0, t_valid = 0;  // virtual group holding the root
    bool g_flip = false;
    int sp = 0;
    while (true) {
        if (t_mask) {
            const int k = lowest_bit(t_mask);
            t_mask &= t_mask - 1u;
            const float* rec = tri_rec(S.tris, tri_slot(t_base, t_valid, k));
            const int kz = R.pre.kz;
            if (COUNT) cnt.tris++;
            float t, V, W, det;
            if (intersect_rot(R.pre, R.o, tri_window(rec, 0, kz), tri_window(rec, 1, kz), tri_window(rec, 2, kz), tmin, best,
                              &t, &V, &W, &det)) {
                const uint32_t id = tri_id(rec);
                const float u = V / det, v = W / det;
                if (ANY) {
                    hit.t = t; hit.id = id; hit.u = u; hit.v = v;
                    return true;
                }
                if (t < best || id < best_id) { best = t; best_id = id; bu = u; bv = v; }
            }
            continue;
        }
        if (!g_hits) {
            if (sp == 0) break;
            --sp;
            const uint32_t e = (uint32_t)stack[sp * kBlock];
            g_base = e >> 9;
            g_flip = (e >> 8) & 1u;
            g_hits = e & 0xffu;
        }
        const int r = g_flip ? highest_bit(g_hits) : lowest_bit(g_hits);
        g_hits &= ~(1u << r);
        if (g_hits) {
            if (sp < kStackSize) {
                stack[sp * kBlock] = (int)pack_group(g_base, g_flip, g_hits);
                ++sp;
            } else {
                overflow = true;
            }
        }
        if (COUNT) cnt.nodes++;
        test_node8(S.nodes8, g_base + (uint32_t)r, R, tmin, best, g_hits, t_mask, t_valid, g_base, t_base, g_flip);
    }
    hit.t = best; hit.id = best_id; hit.u = bu; hit.v = bv;
    return best_id != 0xffffffffu;
}

}  // namespace rt
