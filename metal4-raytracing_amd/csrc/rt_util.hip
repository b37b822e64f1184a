// rt_util.hip — small data-movement kernels around the hot path:
//   tile pack/unpack for the multi-GPU gather,
//   linear-blend skinning (Skinning.metal:7-49),
//   world-space triangle flatten + level-synchronous BVH refit (refitMTL4AccelerationStructures,
//   Renderer.swift:1084-1202).
#include "rt_kernels.h"

namespace rt {

// ---- tiles ----------------------------------------------------------------------------------
__global__ void pack_tiles_k(const float4* __restrict__ src, float4* __restrict__ dst, int width, int height, int tile,
                             int rank, int nranks, int tiles_x, int own) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)tile * tile * own) return;
    int x, y;
    tile_pixel(i, tile, rank, nranks, tiles_x, x, y);
    dst[i] = (x < width && y < height) ? src[(size_t)y * width + x] : make_float4(0, 0, 0, 0);
}
__global__ void unpack_tiles_k(const float4* __restrict__ src, float4* __restrict__ dst, int width, int height, int tile,
                               int rank, int nranks, int tiles_x, int own) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)tile * tile * own) return;
    int x, y;
    tile_pixel(i, tile, rank, nranks, tiles_x, x, y);
    if (x < width && y < height) dst[(size_t)y * width + x] = src[i];
}
void launch_pack_tiles(const float4* src, float4* dst, int width, int height, int tile, int rank, int nranks,
                       int tiles_x, int own, hipStream_t s) {
    size_t n = (size_t)tile * tile * own;
    if (!n) return;
    hipLaunchKernelGGL(pack_tiles_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst, width, height, tile,
                       rank, nranks, tiles_x, own);
}
void launch_unpack_tiles(const float4* src, float4* dst, int width, int height, int tile, int rank, int nranks,
                         int tiles_x, int own, hipStream_t s) {
    size_t n = (size_t)tile * tile * own;
    if (!n) return;
    hipLaunchKernelGGL(unpack_tiles_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst, width, height,
                       tile, rank, nranks, tiles_x, own);
}

// ---- RGBA16F readback (the reference's accumulation format, Renderer.swift:685) ----------------
// fp32 -> fp16 round to nearest even (v_cvt_f16_f32 in the default rounding mode; fp16 denormals
// kept, overflow to infinity), 8 B per pixel out
__global__ void to_half_k(const float4* __restrict__ src, ushort4* __restrict__ dst, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 v = src[i];
    const _Float16 h[4] = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
    dst[i] = make_ushort4(__builtin_bit_cast(uint16_t, h[0]), __builtin_bit_cast(uint16_t, h[1]),
                          __builtin_bit_cast(uint16_t, h[2]), __builtin_bit_cast(uint16_t, h[3]));
}
void launch_to_half(const float4* src, ushort4* dst, size_t n, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(to_half_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst, n);
}

// ---- skinning (Skinning.metal:7-49) ---------------------------------------------------------
__device__ __forceinline__ float4 m4v(const float* m, float x, float y, float z, float w) {
    // float4x4 * float4, column-major: ((c0*x + c1*y) + c2*z) + c3*w
    float4 r;
    r.x = ((m[0] * x + m[4] * y) + m[8] * z) + m[12] * w;
    r.y = ((m[1] * x + m[5] * y) + m[9] * z) + m[13] * w;
    r.z = ((m[2] * x + m[6] * y) + m[10] * z) + m[14] * w;
    r.w = ((m[3] * x + m[7] * y) + m[11] * z) + m[15] * w;
    return r;
}
__global__ void skin_k(const float4* __restrict__ rest_pos, const float4* __restrict__ rest_nrm,
                       const ushort4* __restrict__ jidx, const float4* __restrict__ jw, const float* __restrict__ joints,
                       float4* __restrict__ out_pos, float4* __restrict__ out_nrm, uint32_t n) {
    uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    float4 p = rest_pos[v], q = rest_nrm[v];
    ushort4 ix = jidx[v];
    float4 w = jw[v];
    float ws = ((w.x + w.y) + w.z) + w.w;
    if (ws < 0.0001f) w = make_float4(1.0f, 0.0f, 0.0f, 0.0f);
    const unsigned short js[4] = {ix.x, ix.y, ix.z, ix.w};
    const float ww[4] = {w.x, w.y, w.z, w.w};
    float4 sp = make_float4(0, 0, 0, 0);
    float sn[3] = {0, 0, 0};
    #pragma unroll
    for (int k = 0; k < 4; ++k) {
        float4 a = m4v(joints + 16 * js[k], p.x, p.y, p.z, 1.0f);
        sp.x = sp.x + ww[k] * a.x; sp.y = sp.y + ww[k] * a.y; sp.z = sp.z + ww[k] * a.z; sp.w = sp.w + ww[k] * a.w;
    }
    #pragma unroll
    for (int k = 0; k < 4; ++k) {
        float4 a = m4v(joints + 16 * js[k], q.x, q.y, q.z, 0.0f);
        sn[0] = sn[0] + ww[k] * a.x; sn[1] = sn[1] + ww[k] * a.y; sn[2] = sn[2] + ww[k] * a.z;
    }
    out_pos[v] = make_float4(sp.x, sp.y, sp.z, 0.0f);
    out_nrm[v] = make_float4(sn[0], sn[1], sn[2], 0.0f);
}
void launch_skin(const float4* rest_pos, const float4* rest_nrm, const ushort4* jidx, const float4* jw,
                 const float* joints, float4* out_pos, float4* out_nrm, uint32_t n, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(skin_k, dim3((n + 255) / 256), dim3(256), 0, s, rest_pos, rest_nrm, jidx, jw, joints, out_pos,
                       out_nrm, n);
}

// ---- per-triangle shading records (DevScene::tri_nrm) ------------------------------------------
__global__ void tri_nrm_k(const uint4* __restrict__ tri_info, const float4* __restrict__ nrm, float4* __restrict__ out,
                          uint32_t t0, uint32_t n) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t t = t0 + k;
    const uint4 ti = tri_info[t];
    const float4 n0 = nrm[ti.x], n1 = nrm[ti.y], n2 = nrm[ti.z];
    float4* r = out + 4 * (size_t)t;
    r[0] = make_float4(n1.x, n1.y, n1.z, __uint_as_float(ti.w));
    r[1] = make_float4(n2.x, n2.y, n2.z, 0.0f);
    r[2] = make_float4(n0.x, n0.y, n0.z, 0.0f);
    r[3] = __builtin_bit_cast(float4, ti);
}
void launch_tri_nrm(const uint4* tri_info, const float4* nrm, float4* tri_nrm, uint32_t t0, uint32_t n, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(tri_nrm_k, dim3((n + 255) / 256), dim3(256), 0, s, tri_info, nrm, tri_nrm, t0, n);
}

// ---- flatten world-space triangles into BVH slot order ----------------------------------------
__global__ void flatten_k(const uint4* __restrict__ tri_info, const uint32_t* __restrict__ slot_to_tri,
                          const float4* __restrict__ pos, const float* __restrict__ inst, float* __restrict__ tris,
                          uint32_t n, unsigned* __restrict__ maxabs_bits) {
    __shared__ float red[4];
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    float m = 0.0f;
    if (k < n) {
        uint32_t id = slot_to_tri[k];
        uint4 ti = tri_info[id];
        const float* M = inst + 12 * (ti.w >> 8);
        uint32_t vi[3] = {ti.x, ti.y, ti.z};
        float w9[9];
        #pragma unroll
        for (int q = 0; q < 3; ++q) {
            f3 w = xform(M, ld3(pos[vi[q]]), 1.0f);
            w9[3 * q] = w.x;
            w9[3 * q + 1] = w.y;
            w9[3 * q + 2] = w.z;
            m = fmaxf(m, fmaxf(fabsf(w.x), fmaxf(fabsf(w.y), fabsf(w.z))));
        }
        // the 64-B record (rt_device.h tri_store), written as four 16-B stores
        float r[kTriFloats];
        tri_store(r, w9, id);
        float4* dst = reinterpret_cast<float4*>(tris + (size_t)kTriFloats * k);
        #pragma unroll
        for (int q = 0; q < 4; ++q) dst[q] = make_float4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
    }
    // block max of |coordinate| -> one atomic per block (non-negative floats order as their bits)
    #pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0 && maxabs_bits)
        atomicMax(maxabs_bits, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}
void launch_flatten(const uint4* tri_info, const uint32_t* slot_to_tri, const float4* pos, const float* inst,
                    float* tris, uint32_t n, unsigned* maxabs_bits, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(flatten_k, dim3((n + 255) / 256), dim3(256), 0, s, tri_info, slot_to_tri, pos, inst, tris, n,
                       maxabs_bits);
}

// ---- tree quality after a refit: the node-area sum ------------------------------------------------
// sum over the 8-wide nodes of area(node box): proportional to the expected node visits of the rays
// crossing the scene (the node term of the SAH cost, not normalised by the root box, which a moved
// instance also grows).  One block, a fixed reduction order (deterministic); ~10 us for the
// dragon's 71K nodes.  A refit keeps the topology and grows the boxes of moved geometry; rt_api.cpp
// compares this against the value at the last build and rebuilds on the device when it has grown
// past rt_tuning.refit_rebuild_pct.
__device__ __forceinline__ float box_area(const float* b) {
    const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
    return (dx >= 0.0f && dy >= 0.0f && dz >= 0.0f) ? 2.0f * ((dx * dy + dy * dz) + dz * dx) : 0.0f;
}
__global__ void __launch_bounds__(1024) bvh_cost_k(const float* __restrict__ node_box, uint32_t nn, float* __restrict__ out) {
    __shared__ double red[1024];
    double s = 0.0;
    for (uint32_t n = threadIdx.x; n < nn; n += 1024) s += (double)box_area(node_box + 6 * (size_t)n);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = (float)red[0];
}
void launch_bvh_cost(const float* node_box, uint32_t nn, float* out, hipStream_t s) {
    hipLaunchKernelGGL(bvh_cost_k, dim3(1), dim3(1024), 0, s, node_box, nn, out);
}

// ---- level-synchronous refit of the 8-wide BVH: one launch per level, deepest first -------------
// Each node recomputes its children's boxes (internal: the child's stored box; leaf: bounds of its
// triangles + pad), re-quantizes them exactly as quantize_bvh8_node does on the host (double
// precision, outward rounding), and stores its own box for its parent.
__global__ void refit8_level_k(Bvh8Node* __restrict__ nodes, float* __restrict__ node_box,
                               const float* __restrict__ tris, const uint32_t* __restrict__ level_nodes,
                               uint32_t count, float pad_min, const unsigned* __restrict__ maxabs_bits) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    // the builder's padding rule (4e-6 * max |coordinate|) on the refitted geometry
    const float pad = fmaxf(pad_min, 4e-6f * __uint_as_float(*maxabs_bits));
    const uint32_t ni = level_nodes[i];
    Bvh8Node nd = nodes[ni];
    float clo[8][3], chi[8][3];
    bool used[8];
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int c = 0; c < 8; ++c) {
        // unused slots carry an empty quantized box (qlo = 255 > qhi = 0 on x)
        used[c] = !(nd.q[c] == 255 && nd.q[8 + c] == 0);
        if (!used[c]) continue;
        const uint32_t k_int = (uint32_t)nd.axis_k >> 4;
        float l[3] = {INFINITY, INFINITY, INFINITY}, h[3] = {-INFINITY, -INFINITY, -INFINITY};
        if ((uint32_t)c < k_int) {
            const float* b = node_box + 6 * (size_t)(nd.child_base + (uint32_t)c);
            for (int a = 0; a < 3; ++a) { l[a] = b[a]; h[a] = b[3 + a]; }
        } else {
            const int j = c - (int)k_int;
            const uint32_t first = nd.tri_base + bvh8_leaf_first(nd.tri_valid, j), n = bvh8_leaf_count(nd.tri_valid, j);
            for (uint32_t t = 0; t < n; ++t)
                for (int q = 0; q < 3; ++q) {
                    const f3 v = tri_vertex(tri_rec(tris, first + t), q);
                    l[0] = fminf(l[0], v.x); h[0] = fmaxf(h[0], v.x);
                    l[1] = fminf(l[1], v.y); h[1] = fmaxf(h[1], v.y);
                    l[2] = fminf(l[2], v.z); h[2] = fmaxf(h[2], v.z);
                }
            for (int a = 0; a < 3; ++a) { l[a] -= pad; h[a] += pad; }
        }
        for (int a = 0; a < 3; ++a) {
            clo[c][a] = l[a];
            chi[c][a] = h[a];
            lo[a] = fmin(lo[a], (double)l[a]);
            hi[a] = fmax(hi[a], (double)h[a]);
        }
    }
    for (int a = 0; a < 3; ++a) {
        if (!(lo[a] <= hi[a])) { lo[a] = 0.0; hi[a] = 0.0; }
        float p = (float)lo[a];
        if ((double)p > lo[a]) p = nextafterf(p, -INFINITY);
        nd.p[a] = p;
        double ext = hi[a] - (double)p;
        int e = -100;
        if (ext > 0.0) {
            e = (int)ceil(log2(ext / 255.0));
            while (ldexp(255.0, e) < ext) ++e;
        }
        e = max(-126, min(127, e));
        nd.e[a] = (uint8_t)(e + 127);
        const double inv = ldexp(1.0, -e);
        for (int c = 0; c < 8; ++c) {
            uint8_t ql = 255, qh = 0;
            if (used[c]) {
                double fl = floor(((double)clo[c][a] - (double)p) * inv);
                double fh = ceil(((double)chi[c][a] - (double)p) * inv);
                ql = (uint8_t)fmax(0.0, fmin(255.0, fl));
                qh = (uint8_t)fmax(0.0, fmin(255.0, fh));
            }
            nd.q[16 * a + c] = ql;
            nd.q[16 * a + 8 + c] = qh;
        }
        node_box[6 * (size_t)ni + a] = (float)lo[a];
        node_box[6 * (size_t)ni + 3 + a] = (float)hi[a];
    }
    nodes[ni] = nd;
}
void launch_refit8_level(Bvh8Node* nodes, float* node_box, const float* tris, const uint32_t* level_nodes,
                         uint32_t count, float pad_min, const unsigned* maxabs_bits, hipStream_t s) {
    if (!count) return;
    hipLaunchKernelGGL(refit8_level_k, dim3((count + 127) / 128), dim3(128), 0, s, nodes, node_box, tris, level_nodes,
                       count, pad_min, maxabs_bits);
}

}  // namespace rt
