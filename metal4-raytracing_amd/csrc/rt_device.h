// rt_device.h — device-side scene layout and traversal shared by the HIP kernels.
//
// Data layout in HBM:
//   tris[3*k + 0..2]   float4  world-space v0, v1, v2 of BVH slot k; v0.w = original triangle id
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

constexpr int kStackSize = 32;   // per-thread traversal stack entries (LDS)
constexpr int kBlock = 256;      // threads per block for the traversal kernels

struct DevScene {
    const float4* tris;
    const Bvh2Node* nodes;
    const uint4* tri_info;
    const float4* pos;
    const float4* prev_pos;
    const float4* nrm;
    const float* inst;
    const float* prev_inst;
    const Material* materials;
    const Light* lights;
    const HaltonDim* halton;
    int max_submeshes;
    int num_tris;
};

struct Hit {
    float t;
    uint32_t id;   // original triangle id, 0xffffffff = miss
    float u, v;
};

__device__ __forceinline__ f3 ld3(const float4& v) { return mk3(v.x, v.y, v.z); }

// Object->world with the instance's packed 4x3 (columns c0..c3): ((c0*x + c1*y) + c2*z) + c3*w
__device__ __forceinline__ f3 xform(const float* m, f3 p, float w) {
    f3 c0 = mk3(m[0], m[1], m[2]), c1 = mk3(m[3], m[4], m[5]), c2 = mk3(m[6], m[7], m[8]), c3 = mk3(m[9], m[10], m[11]);
    return ((c0 * p.x + c1 * p.y) + c2 * p.z) + c3 * w;
}

struct TraceCounters {
    uint32_t nodes;
    uint32_t tris;
};

// Closest-hit (ANY=false) or any-hit (ANY=true) traversal with a per-thread LDS stack.
// stack: this thread's column of a [kStackSize][kBlock] LDS array (stride kBlock words).
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool trace(const DevScene& S, f3 o, f3 d, float tmin, float tmax, Hit& hit,
                                      int* stack, TraceCounters& cnt, bool& overflow) {
    RayPre pre = ray_precompute(d);
    // conservative slab test (boxes are padded at build time; see rt_bvh.h)
    auto safe_inv = [](float x) {
        float ax = fabsf(x);
        return 1.0f / (ax < 1e-30f ? copysignf(1e-30f, x) : x);
    };
    const float ix = safe_inv(d.x), iy = safe_inv(d.y), iz = safe_inv(d.z);
    const float ox = o.x * ix, oy = o.y * iy, oz = o.z * iz;
    float best = tmax;
    uint32_t best_id = 0xffffffffu;
    float bu = 0.0f, bv = 0.0f;
    int sp = 0;
    int node = 0;
    const float4* tris = S.tris;
    while (true) {
        const float4* np = reinterpret_cast<const float4*>(S.nodes + node);
        float4 nx = np[0], ny = np[1], nz = np[2];
        int4 meta = *reinterpret_cast<const int4*>(np + 3);
        if (COUNT) cnt.nodes++;
        float tf = best * 1.0000004f;
        float a0 = __builtin_fmaf(nx.x, ix, -ox), b0 = __builtin_fmaf(nx.y, ix, -ox);
        float a1 = __builtin_fmaf(ny.x, iy, -oy), b1 = __builtin_fmaf(ny.y, iy, -oy);
        float a2 = __builtin_fmaf(nz.x, iz, -oz), b2 = __builtin_fmaf(nz.y, iz, -oz);
        float n0 = fmaxf(fmaxf(fminf(a0, b0), fminf(a1, b1)), fmaxf(fminf(a2, b2), tmin));
        float f0 = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fminf(fmaxf(a2, b2), tf));
        float c0 = __builtin_fmaf(nx.z, ix, -ox), d0 = __builtin_fmaf(nx.w, ix, -ox);
        float c1 = __builtin_fmaf(ny.z, iy, -oy), d1 = __builtin_fmaf(ny.w, iy, -oy);
        float c2 = __builtin_fmaf(nz.z, iz, -oz), d2 = __builtin_fmaf(nz.w, iz, -oz);
        float n1 = fmaxf(fmaxf(fminf(c0, d0), fminf(c1, d1)), fmaxf(fminf(c2, d2), tmin));
        float f1 = fminf(fminf(fmaxf(c0, d0), fmaxf(c1, d1)), fminf(fmaxf(c2, d2), tf));
        bool h0 = n0 <= f0, h1 = n1 <= f1;
        // leaves are intersected in place
        #pragma unroll
        for (int s = 0; s < 2; ++s) {
            bool hs = s == 0 ? h0 : h1;
            int ch = s == 0 ? meta.x : meta.y;
            int cnt_s = s == 0 ? meta.z : meta.w;
            if (hs && ch < 0) {
                int first = ~ch;
                for (int k = 0; k < cnt_s; ++k) {
                    const float4* tp = tris + 3 * (first + k);
                    float4 v0 = tp[0], v1 = tp[1], v2 = tp[2];
                    if (COUNT) cnt.tris++;
                    float t, u, v;
                    if (intersect_triangle(pre, o, ld3(v0), ld3(v1), ld3(v2), tmin, best, &t, &u, &v)) {
                        uint32_t id = __float_as_uint(v0.w);
                        if (ANY) { hit.t = t; hit.id = id; hit.u = u; hit.v = v; return true; }
                        if (t < best || id < best_id) { best = t; best_id = id; bu = u; bv = v; }
                    }
                }
                if (s == 0) h0 = false; else h1 = false;
            }
        }
        if (h0 && h1) {
            int near = n0 <= n1 ? meta.x : meta.y;
            int far = n0 <= n1 ? meta.y : meta.x;
            if (sp < kStackSize) { stack[sp * kBlock] = far; ++sp; } else { overflow = true; }
            node = near;
        } else if (h0) {
            node = meta.x;
        } else if (h1) {
            node = meta.y;
        } else {
            if (sp == 0) break;
            --sp;
            node = stack[sp * kBlock];
        }
    }
    hit.t = best; hit.id = best_id; hit.u = bu; hit.v = bv;
    return best_id != 0xffffffffu;
}

}  // namespace rt
