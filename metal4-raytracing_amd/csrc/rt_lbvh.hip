// rt_lbvh.hip — on-device BVH build.
//
// Replaces the driver-internal Metal acceleration-structure build (Utilities.swift:101-290,
// Renderer.swift:464-606) and the legacy full-rebuild path (Renderer.swift:1252-1277) with a
// build that never leaves the GPU:
//   1. world-space triangle boxes, centroid bounds, max |coordinate| (box padding)
//   2. 64-bit keys: Morton code of the centroid (as many bits per axis as fit, up to 21) << id bits
//      | triangle id (unique keys)
//   3. stable LSD radix sort of the keys (8-bit digits: per-tile histograms, one scan, a
//      scatter whose in-tile ranks come from wave ballots, so equal digits keep their order)
//   4. binary radix tree over the sorted keys (Karras, HPG 2012), one thread per inner node
//   5. bottom-up boxes (the second child to finish computes its parent)
//   6. top-down collapse into the compressed 8-wide node layout of rt_bvh.h, one launch per
//      level: a node opens its largest-area child until it has 8 children; subtrees of <= 4
//      triangles become leaves.  Nodes are allocated level by level, so every level is one
//      contiguous index range (the refit's level lists) and the first nodes are the top levels
//      (the part wf_trace stages in LDS).
// Boxes are padded exactly as the host builder pads them, so traversal stays conservative and
// returns the same closest hits as with the host SAH tree: the image does not
// depend on which builder made the tree.
#include <algorithm>

#include "rt_kernels.h"

#include <cstring>
#include <utility>
#include <vector>

namespace rt {

namespace {

constexpr int kThreads = 256;
constexpr int kSortItems = 16;                    // keys per thread per sort tile
constexpr int kSortTile = kThreads * kSortItems;  // 4096
constexpr uint32_t kLeafMax = 4;                  // triangles per 8-wide leaf item

__device__ __forceinline__ uint32_t f2o(float f) {  // order-preserving float -> uint
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

__device__ __forceinline__ unsigned long long expand_bits21(uint32_t v) {  // 21 bits -> every third bit
    unsigned long long x = v & 0x1fffffu;
    x = (x | x << 32) & 0x1f00000000ffffull;
    x = (x | x << 16) & 0x1f0000ff0000ffull;
    x = (x | x << 8) & 0x100f00f00f00f00full;
    x = (x | x << 4) & 0x10c30c30c30c30c3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}

// 1. triangle boxes (lo.xyz, hi.xyz) in original order, centroid bounds, max |coordinate|
__global__ void __launch_bounds__(kThreads) lbvh_boxes_k(LbvhInput in, float* tri_box, uint32_t* bounds,
                                                         uint32_t* maxabs_bits) {
    __shared__ uint32_t sb[7];
    if (threadIdx.x < 7) sb[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    __syncthreads();
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t < in.n) {
        const uint4 ti = in.tri_info[t];
        const float* M = in.inst + 12 * (ti.w >> 8);   // same arithmetic as rt::xform / the host
        const f3 a = xform(M, ld3(in.pos[ti.x]), 1.0f);
        const f3 b = xform(M, ld3(in.pos[ti.y]), 1.0f);
        const f3 c = xform(M, ld3(in.pos[ti.z]), 1.0f);
        const float lo[3] = {fminf(fminf(a.x, b.x), c.x), fminf(fminf(a.y, b.y), c.y), fminf(fminf(a.z, b.z), c.z)};
        const float hi[3] = {fmaxf(fmaxf(a.x, b.x), c.x), fmaxf(fmaxf(a.y, b.y), c.y), fmaxf(fmaxf(a.z, b.z), c.z)};
        float m = 0.0f;
        for (int k = 0; k < 3; ++k) {
            tri_box[6 * (size_t)t + k] = lo[k];
            tri_box[6 * (size_t)t + 3 + k] = hi[k];
            const float cen = 0.5f * (lo[k] + hi[k]);
            atomicMin(&sb[k], f2o(cen));
            atomicMax(&sb[3 + k], f2o(cen));
            m = fmaxf(m, fmaxf(fabsf(lo[k]), fabsf(hi[k])));
        }
        atomicMax(&sb[6], __float_as_uint(m));
    }
    __syncthreads();
    if (threadIdx.x < 3) atomicMin(&bounds[threadIdx.x], sb[threadIdx.x]);
    else if (threadIdx.x < 6) atomicMax(&bounds[threadIdx.x], sb[threadIdx.x]);
    else if (threadIdx.x == 6) atomicMax(maxabs_bits, sb[6]);
}

// 2. keys = Morton(centroid) << id_bits | id: `mb` bits per axis, as many as fit beside the id
// bits in 64 (14 per axis for 881k triangles; finer cells split dense regions by position
// instead of by triangle id)
__global__ void __launch_bounds__(kThreads) lbvh_keys_k(uint32_t n, const float* tri_box, const uint32_t* bounds,
                                                        unsigned long long* keys, int mb, int id_bits) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= n) return;
    unsigned long long code = 0;
    const float cells = (float)(1u << mb);
    for (int k = 0; k < 3; ++k) {
        const float lo = o2f(bounds[k]), hi = o2f(bounds[3 + k]);
        const float cen = 0.5f * (tri_box[6 * (size_t)t + k] + tri_box[6 * (size_t)t + 3 + k]);
        const float ext = hi - lo;
        float u = ext > 0.0f ? (cen - lo) / ext : 0.0f;
        u = fminf(fmaxf(u, 0.0f), 1.0f);
        const uint32_t q = min((uint32_t)(u * cells), (1u << mb) - 1u);
        code |= expand_bits21(q) << (2 - k);
    }
    keys[t] = (code << id_bits) | t;
}

// after the radix tree: keep only the triangle id in every key (the later stages read it from
// the low 32 bits)
__global__ void __launch_bounds__(kThreads) lbvh_key_ids_k(unsigned long long* keys, uint32_t n,
                                                           unsigned long long id_mask) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t < n) keys[t] &= id_mask;
}

// 3. radix sort pass: per-tile digit histograms -> table[digit * tiles + tile]
__global__ void __launch_bounds__(kThreads) lbvh_hist_k(const unsigned long long* keys, uint32_t n, int shift,
                                                        uint32_t tiles, uint32_t* table) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kSortTile;
    for (int i = 0; i < kSortItems; ++i) {
        const uint32_t k = base + (uint32_t)i * kThreads + threadIdx.x;
        if (k < n) atomicAdd(&h[(uint32_t)(keys[k] >> shift) & 255u], 1u);
    }
    __syncthreads();
    table[(size_t)threadIdx.x * tiles + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of the whole table in one block (digit-major: the output offsets)
__global__ void __launch_bounds__(1024) lbvh_scan_k(uint32_t* table, uint32_t len) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (len + 1023) / 1024;
    const uint32_t b = min(threadIdx.x * per, len), e = min(b + per, len);
    uint32_t s = 0;
    for (uint32_t i = b; i < e; ++i) s += table[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {   // inclusive scan of the parts
        const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (uint32_t i = b; i < e; ++i) {
        const uint32_t v = table[i];
        table[i] = run;
        run += v;
    }
}

// Stable scatter.  Tile order is (row i, thread) = key order; the rank among equal digits inside
// one wave of a row comes from 8 ballots, across the row's waves from LDS counts, across rows
// from a running per-digit offset.
__global__ void __launch_bounds__(kThreads) lbvh_scatter_k(const unsigned long long* keys_in,
                                                           unsigned long long* keys_out, uint32_t n, int shift,
                                                           uint32_t tiles, const uint32_t* table) {
    __shared__ uint32_t run[256];
    __shared__ uint32_t wcnt[kThreads / 64][256];
    run[threadIdx.x] = table[(size_t)threadIdx.x * tiles + blockIdx.x];
    const int wave = threadIdx.x >> 6;
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const unsigned long long lt = (1ull << lane) - 1ull;
    const uint32_t base = blockIdx.x * kSortTile;
    for (int i = 0; i < kSortItems; ++i) {
        for (int w = 0; w < kThreads / 64; ++w) wcnt[w][threadIdx.x] = 0;
        __syncthreads();
        const uint32_t k = base + (uint32_t)i * kThreads + threadIdx.x;
        const bool valid = k < n;
        const unsigned long long key = valid ? keys_in[k] : 0ull;
        const uint32_t d = (uint32_t)(key >> shift) & 255u;
        unsigned long long m = __ballot(valid);
        for (int bit = 0; bit < 8; ++bit) {
            const bool set = (d >> bit) & 1u;
            const unsigned long long bb = __ballot(set);
            m &= set ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(m & lt);
        if (valid && rank == 0) wcnt[wave][d] = (uint32_t)__popcll(m);
        __syncthreads();
        {   // thread = digit: offsets of this row's waves, then advance the digit's run
            uint32_t acc = run[threadIdx.x];
            for (int w = 0; w < kThreads / 64; ++w) {
                const uint32_t c = wcnt[w][threadIdx.x];
                wcnt[w][threadIdx.x] = acc;
                acc += c;
            }
            run[threadIdx.x] = acc;
        }
        __syncthreads();
        if (valid) keys_out[wcnt[wave][d] + rank] = key;
        __syncthreads();
    }
}

// 4. radix tree (Karras 2012): inner node i of n-1; a child < 0 is the leaf at sorted position ~c
__device__ __forceinline__ int delta(const unsigned long long* k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    return __clzll(k[i] ^ k[j]);
}

__global__ void __launch_bounds__(kThreads) lbvh_tree_k(const unsigned long long* keys, uint32_t nn, int* child,
                                                        int* parent, int* leaf_parent, uint32_t* first,
                                                        uint32_t* count) {
    const int n = (int)nn;
    const int i = (int)(blockIdx.x * kThreads + threadIdx.x);
    if (i >= n - 1) return;
    const int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(keys, n, i, i - d);
    int lmax = 2;
    while (delta(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(keys, n, i, j);
    int s = 0;
    for (int div = 2;; div *= 2) {
        const int t = (l + div - 1) / div;
        if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
        if (t <= 1) break;
    }
    const int g = i + s * d + min(d, 0);
    if (j < 0 || j >= n || g < 0 || g + 1 >= n) return;   // guard (cannot happen for unique keys)
    const int lo = min(i, j), hi = max(i, j);
    const int left = lo == g ? ~g : g;
    const int right = hi == g + 1 ? ~(g + 1) : g + 1;
    child[2 * i] = left;
    child[2 * i + 1] = right;
    if (left >= 0) parent[left] = i;
    else leaf_parent[~left] = i;
    if (right >= 0) parent[right] = i;
    else leaf_parent[~right] = i;
    first[i] = (uint32_t)lo;
    count[i] = (uint32_t)(hi - lo + 1);
    if (i == 0) parent[0] = -1;
}

// 5. bottom-up boxes of the inner nodes (6 floats each, unpadded); the loads of a sibling's
// box written by another thread are agent-scope (past the CU's L1)
__device__ __forceinline__ void child_box(int c, const unsigned long long* keys, const float* tri_box,
                                          const float* node_box, float* b) {
    if (c < 0) {
        const uint32_t t = (uint32_t)keys[~c];
        for (int k = 0; k < 6; ++k) b[k] = tri_box[6 * (size_t)t + k];
    } else {
        for (int k = 0; k < 6; ++k)
            b[k] = __uint_as_float(__hip_atomic_load((uint32_t*)&node_box[6 * (size_t)c + k], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT));
    }
}

__global__ void __launch_bounds__(kThreads) lbvh_boxes_up_k(const unsigned long long* keys, uint32_t n, const int* child,
                                                            const int* parent, const int* leaf_parent,
                                                            const float* tri_box, float* node_box, uint32_t* flag) {
    const uint32_t k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= n) return;
    int p = leaf_parent[k];
    while (p >= 0 && p < (int)n - 1) {
        __threadfence();
        if (atomicAdd(&flag[p], 1u) == 0u) return;   // the sibling subtree is not finished yet
        __threadfence();
        float a[6], b[6];
        child_box(child[2 * p], keys, tri_box, node_box, a);
        child_box(child[2 * p + 1], keys, tri_box, node_box, b);
        for (int q = 0; q < 3; ++q) {
            __hip_atomic_store((uint32_t*)&node_box[6 * (size_t)p + q], __float_as_uint(fminf(a[q], b[q])),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store((uint32_t*)&node_box[6 * (size_t)p + 3 + q], __float_as_uint(fmaxf(a[3 + q], b[3 + q])),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        p = parent[p];
    }
}

// ---- 4b. PLOC (Meister, Bittner, "Parallel Locally-Ordered Clustering for Bounding Volume
// Hierarchy Construction", TVCG 2018): clusters start as the Morton-sorted triangles; every round
// each cluster finds the neighbour within +-kPlocR (in the current order) whose merged box has the
// smallest surface area, mutual nearest neighbours merge into a new inner node (at the lower
// position), and the survivors are compacted in order.  The globally cheapest neighbour pair is
// always mutual (ties go to the smaller index), so every round makes progress.
constexpr int kPlocR = 16;

__device__ __forceinline__ float area6(const float* a, const float* b) {
    const float d0 = fmaxf(a[3], b[3]) - fminf(a[0], b[0]);
    const float d1 = fmaxf(a[4], b[4]) - fminf(a[1], b[1]);
    const float d2 = fmaxf(a[5], b[5]) - fminf(a[2], b[2]);
    return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
}

__global__ void __launch_bounds__(kThreads) ploc_init_k(const unsigned long long* keys, const float* tri_box, uint32_t n,
                                                        int* cref, float* cbox, uint32_t* m0) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i == 0) *m0 = n;   // the first round's cluster count
    if (i >= n) return;
    cref[i] = ~(int)i;   // leaf at sorted position i
    const uint32_t t = (uint32_t)keys[i];
    for (int k = 0; k < 6; ++k) cbox[6 * (size_t)i + k] = tri_box[6 * (size_t)t + k];
}

// The round's cluster count comes from device memory (the previous round's scan): the host
// launches rounds in batches with grids sized by its last known count and reads the count back
// once per batch.
__global__ void __launch_bounds__(kThreads) ploc_nn_k(const float* cbox, const uint32_t* mp, int* nn) {
    const uint32_t m = *mp;
    if (blockIdx.x * kThreads >= m) return;
    __shared__ float sb[(kThreads + 2 * kPlocR) * 6];
    const int base = (int)(blockIdx.x * kThreads) - kPlocR;
    for (int t = threadIdx.x; t < kThreads + 2 * kPlocR; t += kThreads) {
        const int g = base + t;
        for (int k = 0; k < 6; ++k) sb[t * 6 + k] = (g >= 0 && g < (int)m) ? cbox[6 * (size_t)g + k] : 0.0f;
    }
    __syncthreads();
    const int i = (int)(blockIdx.x * kThreads + threadIdx.x);
    if (i >= (int)m) return;
    const float* bi = &sb[(threadIdx.x + kPlocR) * 6];
    float best = INFINITY;
    int bj = -1;
    for (int d = -kPlocR; d <= kPlocR; ++d) {   // ascending index: ties keep the smaller one
        const int j = i + d;
        if (d == 0 || j < 0 || j >= (int)m) continue;
        const float a = area6(bi, &sb[(threadIdx.x + kPlocR + d) * 6]);
        if (a < best) {
            best = a;
            bj = j;
        }
    }
    nn[i] = bj;
}

// mutual pairs merge into a new inner node at the lower position; keep[i] = cluster i survives
struct PlocMerge {
    const int* nn;
    const int* cref;
    const float* cbox;
    int* tref;          // this round's clusters before compaction
    float* tbox;
    uint32_t* keep;
    int* child;
    int* parent;
    int* leaf_parent;
    uint32_t* count;    // triangles under each inner node
    float* node_box;
    uint32_t* node_ctr;
    uint32_t* err;
    const uint32_t* mp;   // this round's cluster count
    uint32_t n;
};

__global__ void __launch_bounds__(kThreads) ploc_merge_k(PlocMerge M) {
    const int i = (int)(blockIdx.x * kThreads + threadIdx.x);
    if (i >= (int)*M.mp) return;
    const int j = M.nn[i];
    const bool mutual = j >= 0 && M.nn[j] == i;
    const int ri = M.cref[i];
    if (mutual && i > j) {   // the partner at the lower position creates the node
        M.keep[i] = 0u;
        return;
    }
    M.keep[i] = 1u;
    if (!mutual) {
        M.tref[i] = ri;
        for (int k = 0; k < 6; ++k) M.tbox[6 * (size_t)i + k] = M.cbox[6 * (size_t)i + k];
        return;
    }
    const uint32_t id = atomicAdd(M.node_ctr, 1u);
    if (id + 1 >= M.n) {   // guard: n - 1 inner nodes at most
        atomicOr(M.err, 16u);
        M.tref[i] = ri;
        return;
    }
    const int rj = M.cref[j];
    M.child[2 * id] = ri;
    M.child[2 * id + 1] = rj;
    uint32_t cnt = 0;
    for (int s = 0; s < 2; ++s) {
        const int r = s ? rj : ri;
        if (r >= 0) {
            M.parent[r] = (int)id;
            cnt += M.count[r];
        } else {
            M.leaf_parent[~r] = (int)id;
            cnt += 1u;
        }
    }
    M.count[id] = cnt;
    for (int k = 0; k < 3; ++k) {
        const float lo = fminf(M.cbox[6 * (size_t)i + k], M.cbox[6 * (size_t)j + k]);
        const float hi = fmaxf(M.cbox[6 * (size_t)i + 3 + k], M.cbox[6 * (size_t)j + 3 + k]);
        M.node_box[6 * (size_t)id + k] = lo;
        M.node_box[6 * (size_t)id + 3 + k] = hi;
        M.tbox[6 * (size_t)i + k] = lo;
        M.tbox[6 * (size_t)i + 3 + k] = hi;
    }
    M.tref[i] = (int)id;
}

// order-preserving compaction: per-block counts, one scan of the block counts, scatter
__global__ void __launch_bounds__(kThreads) ploc_count_k(const uint32_t* keep, const uint32_t* mp, uint32_t* bsum) {
    const uint32_t m = *mp;
    __shared__ uint32_t w[kThreads / 64];
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    const unsigned long long b = __ballot(i < m && keep[i]);
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = (uint32_t)__popcll(b);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int k = 0; k < kThreads / 64; ++k) s += w[k];
        bsum[blockIdx.x] = s;
    }
}

__global__ void __launch_bounds__(1024) ploc_scan_k(uint32_t* bsum, uint32_t nb, uint32_t* total) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t b = min(threadIdx.x * per, nb), e = min(b + per, nb);
    uint32_t s = 0;
    for (uint32_t i = b; i < e; ++i) s += bsum[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (uint32_t i = b; i < e; ++i) {
        const uint32_t v = bsum[i];
        bsum[i] = run;
        run += v;
    }
    if (threadIdx.x == 1023) *total = part[1023];
}

__global__ void __launch_bounds__(kThreads) ploc_scatter_k(const uint32_t* keep, const uint32_t* mp, const uint32_t* bsum,
                                                           const int* tref, const float* tbox, int* cref, float* cbox) {
    const uint32_t m = *mp;
    if (blockIdx.x * kThreads >= m) return;
    __shared__ uint32_t w[kThreads / 64];
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    const bool k = i < m && keep[i];
    const unsigned long long b = __ballot(k);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) w[wave] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t off = bsum[blockIdx.x];
    for (int q = 0; q < wave; ++q) off += w[q];
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    if (k) {
        const uint32_t o = off + (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
        cref[o] = tref[i];
        for (int c = 0; c < 6; ++c) cbox[6 * (size_t)o + c] = tbox[6 * (size_t)i + c];
    }
}

// ---- 5b. SAH dynamic programming over the BVH2 (the host builder's collapse_bvh8_dp, rt_bvh.cpp):
// per inner node the cheapest cost with 1..8 slots and the choices that reach it, bottom-up (the
// second child to finish computes its parent, as lbvh_boxes_up_k).  choice[10 * p + i]:
// i = 1: 1 leaf / 2 node; i >= 2: 0 = as with i - 1 slots, k = k slots to the left child;
// [10 * p + 9] = the left child's share of the node's own eight slots.
struct DpArgs {
    const unsigned long long* keys;   // low 32 bits = triangle id
    const int* child;
    const int* parent;
    const int* leaf_parent;
    const uint32_t* count;
    const float* tri_box;
    const float* node_box;
    float* cost;        // 8 per inner node
    uint8_t* choice;    // 10 per inner node
    uint32_t* flag;
    uint32_t n;
    float c_node, c_prim;
};

__device__ __forceinline__ float box_area(const float* b) {
    const float d0 = b[3] - b[0], d1 = b[4] - b[1], d2 = b[5] - b[2];
    return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
}

__device__ __forceinline__ void dp_child_costs(const DpArgs& A, int r, float* c) {
    if (r < 0) {   // one triangle: a leaf whatever the budget
        const float a = box_area(A.tri_box + 6 * (size_t)(uint32_t)A.keys[~r]) * A.c_prim;
        for (int i = 0; i < 8; ++i) c[i] = a;
    } else {   // plain loads after the acquire fence (independent, so they overlap)
        const float4 a = *reinterpret_cast<const float4*>(A.cost + 8 * (size_t)r);
        const float4 b = *reinterpret_cast<const float4*>(A.cost + 8 * (size_t)r + 4);
        c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w;
        c[4] = b.x; c[5] = b.y; c[6] = b.z; c[7] = b.w;
    }
}

__global__ void __launch_bounds__(kThreads) lbvh_dp_up_k(DpArgs A) {
    const uint32_t k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= A.n) return;
    int p = A.leaf_parent[k];
    while (p >= 0 && p < (int)A.n - 1) {
        // release this thread's cost stores, count the arrival; the second arrival acquires (the
        // fence invalidates this CU's L1, so the sibling's costs are read from L2).  Per-word
        // agent-scope atomic loads here serialised into ~50 us per tree level (4.8 ms a build).
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (atomicAdd(&A.flag[p], 1u) == 0u) return;   // the sibling subtree is not finished yet
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        float cl[8], cr[8], D[9];
        uint8_t K[9];
        dp_child_costs(A, A.child[2 * p], cl);
        dp_child_costs(A, A.child[2 * p + 1], cr);
        for (int j = 2; j <= 8; ++j) {
            D[j] = INFINITY;
            K[j] = 1;
            for (int q = 1; q < j; ++q) {
                const float v = cl[q - 1] + cr[j - q - 1];
                if (v < D[j]) {
                    D[j] = v;
                    K[j] = (uint8_t)q;
                }
            }
        }
        const float area = box_area(A.node_box + 6 * (size_t)p);
        const uint32_t cnt = A.count[p];
        const float leaf = cnt <= kLeafMax ? area * A.c_prim * (float)cnt : INFINITY;
        const float node = area * A.c_node + D[8];
        float c = fminf(leaf, node);
        float C[8];
        uint8_t ch[10];
        ch[0] = 0;
        ch[1] = leaf <= node ? 1 : 2;
        ch[9] = K[8];
        C[0] = c;
        for (int i = 2; i <= 8; ++i) {
            if (D[i] < c) {
                c = D[i];
                ch[i] = K[i];
            } else {
                ch[i] = 0;
            }
            C[i - 1] = c;
        }
        *reinterpret_cast<float4*>(A.cost + 8 * (size_t)p) = make_float4(C[0], C[1], C[2], C[3]);
        *reinterpret_cast<float4*>(A.cost + 8 * (size_t)p + 4) = make_float4(C[4], C[5], C[6], C[7]);
        for (int i = 0; i < 10; ++i) A.choice[10 * (size_t)p + i] = ch[i];
        p = A.parent[p];
    }
}

// 6. top-down collapse of one level into 8-wide nodes
struct Item {
    float lo[3], hi[3];
    int ref;           // BVH2 reference: >= 0 inner node, < 0 leaf ~position
    uint32_t first, count;
    bool leaf;
};

__device__ __forceinline__ float item_area(const Item& it) {
    const float d0 = it.hi[0] - it.lo[0], d1 = it.hi[1] - it.lo[1], d2 = it.hi[2] - it.lo[2];
    return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
}

struct CollapseArgs {
    const unsigned long long* keys;   // sorted: low 32 bits = triangle id
    const int* child;
    const uint32_t* first;
    const uint32_t* count;
    const float* tri_box;
    const float* node_box;            // BVH2 inner boxes
    const uint32_t* maxabs_bits;
    const int2* jobs_in;              // (BVH2 reference, 8-wide node)
    uint32_t n_jobs;
    int2* jobs_out;
    const uint8_t* choice;            // DP choices (lbvh_dp_up_k)
    uint32_t* counters;               // [0] 8-wide nodes allocated, [1] triangle slots, [2] next jobs,
                                      // [4] error flag (a capacity guard tripped)
    uint32_t n;                       // triangles = capacity of nodes8, tri_order, the job queues
    Bvh8Node* nodes8;
    float* node8_box;
    uint32_t* tri_order;
};

__device__ Item make_item(const CollapseArgs& A, int ref, float pad) {
    Item it;
    if (ref >= (int)A.n - 1 || (ref < 0 && (uint32_t)~ref >= A.n)) {   // guard (a malformed tree)
        atomicOr(&A.counters[4], 8u);
        ref = ~0;
    }
    it.ref = ref;
    const float* b;
    if (ref < 0) {
        const uint32_t pos = (uint32_t)~ref;
        b = A.tri_box + 6 * (size_t)(uint32_t)A.keys[pos];
        it.first = pos;
        it.count = 1;
    } else {
        b = A.node_box + 6 * (size_t)ref;
        it.first = A.first[ref];
        it.count = A.count[ref];
    }
    for (int k = 0; k < 3; ++k) {   // padded like the host builder's child boxes
        it.lo[k] = b[k] - pad;
        it.hi[k] = b[3 + k] + pad;
    }
    it.leaf = it.count <= kLeafMax;
    return it;
}

// device mirror of quantize_bvh8_node (rt_bvh.cpp)
__device__ void quantize_node(Bvh8Node& nd, const Item* items, int n_items) {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int c = 0; c < n_items; ++c)
        for (int a = 0; a < 3; ++a) {
            lo[a] = fmin(lo[a], (double)items[c].lo[a]);
            hi[a] = fmax(hi[a], (double)items[c].hi[a]);
        }
    for (int a = 0; a < 3; ++a) {
        if (!(lo[a] <= hi[a])) {
            lo[a] = 0.0;
            hi[a] = 0.0;
        }
        nd.p[a] = (float)lo[a];
        if ((double)nd.p[a] > lo[a]) nd.p[a] = nextafterf(nd.p[a], -INFINITY);   // p <= every child lo
        const double ext = hi[a] - (double)nd.p[a];
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
            if (c < n_items) {
                const double fl = floor(((double)items[c].lo[a] - (double)nd.p[a]) * inv);
                const double fh = ceil(((double)items[c].hi[a] - (double)nd.p[a]) * inv);
                ql = (uint8_t)fmax(0.0, fmin(255.0, fl));
                qh = (uint8_t)fmax(0.0, fmin(255.0, fh));
            }
            nd.q[16 * a + c] = ql;
            nd.q[16 * a + 8 + c] = qh;
        }
    }
}

__global__ void __launch_bounds__(kThreads) lbvh_collapse_k(CollapseArgs A) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= A.n_jobs) return;
    const float pad = 4e-6f * __uint_as_float(*A.maxabs_bits);
    const int2 job = A.jobs_in[j];
    if (job.x < 0 || (uint32_t)job.x + 1 >= A.n || (uint32_t)job.y >= A.n) {   // guard: never index out of range
        atomicOr(&A.counters[4], 1u);
        return;
    }
    Item items[8];
    int n_items = 0;
    // DP: the node's eight slots split between its children as chosen bottom-up; a subtree
    // with budget j either splits again (choice k) or becomes one slot (leaf or node)
    int2 st[16];
    int sp = 0;
    const int k8 = A.choice[10 * (size_t)job.x + 9];
    st[sp++] = make_int2(A.child[2 * job.x + 1], 8 - k8);
    st[sp++] = make_int2(A.child[2 * job.x], k8);
    while (sp > 0) {
        const int2 e = st[--sp];
        const int r = e.x;
        int b = e.y;
        if (r >= 0 && (uint32_t)r + 1 < A.n) {
            while (b >= 2 && A.choice[10 * (size_t)r + b] == 0) --b;
            if (b >= 2 && sp + 2 <= 16) {
                const int k = A.choice[10 * (size_t)r + b];
                st[sp++] = make_int2(A.child[2 * r + 1], b - k);
                st[sp++] = make_int2(A.child[2 * r], k);
                continue;
            }
        }
        if (n_items >= 8) {   // guard: the budgets add up to 8
            atomicOr(&A.counters[4], 32u);
            return;
        }
        Item it = make_item(A, r, pad);
        if (r >= 0) it.leaf = A.choice[10 * (size_t)r + 1] == 1 && it.count <= kLeafMax;
        items[n_items++] = it;
    }
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < n_items; ++i)
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], items[i].lo[a]);
            hi[a] = fmaxf(hi[a], items[i].hi[a]);
        }
    int axis = 0;
    for (int a = 1; a < 3; ++a)
        if (hi[a] - lo[a] > hi[axis] - lo[axis]) axis = a;
    for (int i = 1; i < n_items; ++i) {   // stable insertion sort of the slots by centroid along axis
        const Item x = items[i];
        const float kx = x.lo[axis] + x.hi[axis];
        int q = i - 1;
        while (q >= 0 && items[q].lo[axis] + items[q].hi[axis] > kx) {
            items[q + 1] = items[q];
            --q;
        }
        items[q + 1] = x;
    }
    {   // internal children first (slot = rank), then the leaves, each kind in centroid order
        Item sorted[8];
        int m = 0;
        for (int i = 0; i < n_items; ++i)
            if (!items[i].leaf) sorted[m++] = items[i];
        for (int i = 0; i < n_items; ++i)
            if (items[i].leaf) sorted[m++] = items[i];
        for (int i = 0; i < n_items; ++i) items[i] = sorted[i];
    }
    uint32_t n_internal = 0, n_tris = 0;
    for (int i = 0; i < n_items; ++i) {
        if (items[i].leaf) n_tris += items[i].count;
        else ++n_internal;
    }
    Bvh8Node nd;
    nd.tri_valid = 0u;
    nd.reserved = 0u;
    nd.axis_k = (uint8_t)(axis | (n_internal << 4));
    nd.child_base = n_internal ? atomicAdd(&A.counters[0], n_internal) : 0u;
    nd.tri_base = n_tris ? atomicAdd(&A.counters[1], n_tris) : 0u;
    if (nd.child_base + n_internal > A.n || nd.tri_base + n_tris > A.n) {
        atomicOr(&A.counters[4], 2u);
        return;
    }
    uint32_t rank = 0, toff = 0;
    for (int i = 0; i < n_items; ++i) {
        const Item& it = items[i];
        if (!it.leaf) {
            const uint32_t slot = atomicAdd(&A.counters[2], 1u);
            if (slot < A.n) A.jobs_out[slot] = make_int2(it.ref, (int)(nd.child_base + rank));
            else atomicOr(&A.counters[4], 4u);
            ++rank;
        } else {
            nd.tri_valid |= ((1u << it.count) - 1u) << (4u * ((uint32_t)i - n_internal));
            // the subtree's triangles (<= 4), left to right (PLOC subtrees are not contiguous in
            // the sorted order)
            int st[8];
            int sp = 0;
            uint32_t t = 0;
            st[sp++] = it.ref;
            while (sp > 0 && t < it.count) {
                const int r = st[--sp];
                if (r < 0) {
                    A.tri_order[nd.tri_base + toff + t++] = (uint32_t)A.keys[~r];
                } else if (sp + 2 <= 8) {
                    st[sp++] = A.child[2 * r + 1];
                    st[sp++] = A.child[2 * r];
                }
            }
            if (t != it.count) atomicOr(&A.counters[4], 64u);
            toff += it.count;
        }
    }
    quantize_node(nd, items, n_items);
    A.nodes8[job.y] = nd;
    for (int a = 0; a < 3; ++a) {
        A.node8_box[6 * (size_t)job.y + a] = lo[a];
        A.node8_box[6 * (size_t)job.y + 3 + a] = hi[a];
    }
}

// hit-sort bins of every triangle from its leaf slot (DevScene::tri_bin)
__global__ void __launch_bounds__(kThreads) lbvh_tri_bin_k(const uint32_t* tri_order, uint32_t n, uint16_t* tri_bin) {
    const uint32_t k = blockIdx.x * kThreads + threadIdx.x;
    if (k < n) tri_bin[tri_order[k]] = (uint16_t)(((unsigned long long)k * kSortMaxBins) / n);
}

// the refit's level list: nodes are allocated level by level, so it is the identity
__global__ void __launch_bounds__(kThreads) lbvh_iota_k(uint32_t* v, uint32_t n) {
    const uint32_t k = blockIdx.x * kThreads + threadIdx.x;
    if (k < n) v[k] = k;
}

inline unsigned blocks(size_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }
inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

size_t lbvh_scratch_bytes(uint32_t n) {
    const size_t tiles = (n + kSortTile - 1) / kSortTile;
    return 2 * align256(8 * (size_t)n)      // keys, ping-pong
           + align256(24 * (size_t)n)       // triangle boxes
           + align256(4 * 256 * tiles)      // sort table
           + align256(8 * (size_t)n)        // inner children
           + 2 * align256(4 * (size_t)n)    // inner parents, leaf parents
           + 2 * align256(4 * (size_t)n)    // first, count
           + align256(24 * (size_t)n)       // inner boxes
           + align256(4 * (size_t)n)        // bottom-up flags
           + 2 * align256(8 * (size_t)n)    // job queues
           + align256(64 * 4)               // bounds, maxabs, counters
           + 2 * align256(4 * (size_t)n)    // PLOC cluster refs (current, merged)
           + 2 * align256(24 * (size_t)n)   // PLOC cluster boxes
           + 2 * align256(4 * (size_t)n)    // PLOC nearest neighbours, keep flags
           + align256(4 * ((size_t)n / kThreads + 2))   // PLOC block counts
           + align256(32 * (size_t)n)       // DP costs
           + align256(10 * (size_t)n);      // DP choices
}

bool lbvh_build(const LbvhInput& in, const LbvhOutput& out, void* scratch, hipStream_t s, LbvhResult* res,
                const char** err) {
    const uint32_t n = in.n;
    if (n < 2) {
        *err = "lbvh: fewer than 2 triangles";
        return false;
    }
    const uint32_t tiles = (n + kSortTile - 1) / kSortTile;
    char* p = (char*)scratch;
    auto carve = [&p](size_t bytes) {
        void* r = p;
        p += align256(bytes);
        return r;
    };
    auto* keys = (unsigned long long*)carve(8 * (size_t)n);
    auto* keys2 = (unsigned long long*)carve(8 * (size_t)n);
    auto* tri_box = (float*)carve(24 * (size_t)n);
    auto* table = (uint32_t*)carve(4 * 256 * (size_t)tiles);
    auto* child = (int*)carve(8 * (size_t)n);
    auto* parent = (int*)carve(4 * (size_t)n);
    auto* leaf_parent = (int*)carve(4 * (size_t)n);
    auto* first = (uint32_t*)carve(4 * (size_t)n);
    auto* count = (uint32_t*)carve(4 * (size_t)n);
    auto* node_box = (float*)carve(24 * (size_t)n);
    auto* flag = (uint32_t*)carve(4 * (size_t)n);
    auto* jobs_a = (int2*)carve(8 * (size_t)n);
    auto* jobs_b = (int2*)carve(8 * (size_t)n);
    auto* misc = (uint32_t*)carve(64 * 4);   // [0..5] centroid bounds, [6] max |coord|, [8..12] counters,
                                             // [14] PLOC inner nodes, [15] PLOC clusters left
    auto* cref = (int*)carve(4 * (size_t)n);
    auto* tref = (int*)carve(4 * (size_t)n);
    auto* cbox = (float*)carve(24 * (size_t)n);
    auto* tbox = (float*)carve(24 * (size_t)n);
    auto* nn = (int*)carve(4 * (size_t)n);
    auto* keep = (uint32_t*)carve(4 * (size_t)n);
    auto* bsum = (uint32_t*)carve(4 * ((size_t)n / kThreads + 2));
    auto* cost = (float*)carve(32 * (size_t)n);
    auto* choice = (uint8_t*)carve(10 * (size_t)n);
#define LB_CHECK(expr)                    \
    do {                                  \
        hipError_t e_ = (expr);           \
        if (e_ != hipSuccess) {           \
            *err = hipGetErrorString(e_); \
            return false;                 \
        }                                 \
    } while (0)
    // bounds start empty, max |coord| at 1.0 (as the host builder), node counter past the root
    static const uint32_t init[16] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0, 0, 0, 0x3f800000u, 0,
                                      1u, 0, 0, 0, 0, 0, 0, 0};   // [14] PLOC node counter = 0
    LB_CHECK(hipMemcpyAsync(misc, init, sizeof init, hipMemcpyHostToDevice, s));
    LB_CHECK(hipMemsetAsync(flag, 0, 4 * (size_t)n, s));
    LB_CHECK(hipMemsetAsync(parent, 0xff, 4 * (size_t)n, s));        // -1: unset
    LB_CHECK(hipMemsetAsync(leaf_parent, 0xff, 4 * (size_t)n, s));
    lbvh_boxes_k<<<blocks(n), kThreads, 0, s>>>(in, tri_box, misc, misc + 6);
    int id_bits = 1;
    while (id_bits < 32 && (1ull << id_bits) < n) ++id_bits;
    const int mb = std::min(21, (64 - id_bits) / 3);
    lbvh_keys_k<<<blocks(n), kThreads, 0, s>>>(n, tri_box, misc, keys, mb, id_bits);
    // 8-bit digits over the key bits in use (ids + 3 * mb Morton bits)
    unsigned long long* src = keys;
    unsigned long long* dst = keys2;
    for (int shift = 0; shift < id_bits + 3 * mb; shift += 8) {
        lbvh_hist_k<<<tiles, kThreads, 0, s>>>(src, n, shift, tiles, table);
        lbvh_scan_k<<<1, 1024, 0, s>>>(table, 256 * tiles);
        lbvh_scatter_k<<<tiles, kThreads, 0, s>>>(src, dst, n, shift, tiles, table);
        std::swap(src, dst);
    }
    uint32_t* h_next = out.h_scratch;   // pinned
    int2* jin = jobs_a;
    int2* jout = jobs_b;
    LB_CHECK(hipMemsetAsync(jobs_a, 0, sizeof(int2), s));   // the root job: (BVH2 root, 8-wide node 0)
    if (in.ploc) {
        lbvh_key_ids_k<<<blocks(n), kThreads, 0, s>>>(src, n, (1ull << id_bits) - 1ull);
        ploc_init_k<<<blocks(n), kThreads, 0, s>>>(src, tri_box, n, cref, cbox, misc + 15);
        PlocMerge M;
        M.nn = nn;
        M.cref = cref;
        M.cbox = cbox;
        M.tref = tref;
        M.tbox = tbox;
        M.keep = keep;
        M.child = child;
        M.parent = parent;
        M.leaf_parent = leaf_parent;
        M.count = count;
        M.node_box = node_box;
        M.node_ctr = misc + 14;
        M.err = misc + 12;
        M.n = n;
        // cluster counts ping-pong between misc[15] and misc[16]: round r reads misc[15 + (r & 1)]
        uint32_t m = n;
        int round = 0;
        while (m > 1) {
            if (round >= 2000) {
                *err = "ploc: no convergence";
                return false;
            }
            const unsigned nb = blocks(m);   // an upper bound for every round of the batch
            const int batch = m > 65536 ? 4 : 8;
            for (int b = 0; b < batch; ++b, ++round) {
                uint32_t* mc = misc + 15 + (round & 1);
                uint32_t* mn = misc + 15 + ((round + 1) & 1);
                M.mp = mc;
                ploc_nn_k<<<nb, kThreads, 0, s>>>(cbox, mc, nn);
                ploc_merge_k<<<nb, kThreads, 0, s>>>(M);
                ploc_count_k<<<nb, kThreads, 0, s>>>(keep, mc, bsum);
                ploc_scan_k<<<1, 1024, 0, s>>>(bsum, nb, mn);
                ploc_scatter_k<<<nb, kThreads, 0, s>>>(keep, mc, bsum, tref, tbox, cref, cbox);
            }
            LB_CHECK(hipGetLastError());
            LB_CHECK(hipMemcpyAsync(h_next, misc + 15 + (round & 1), 4, hipMemcpyDeviceToHost, s));
            LB_CHECK(hipStreamSynchronize(s));
            if (*h_next >= m || *h_next == 0) {
                *err = "ploc: a batch of rounds merged nothing";
                return false;
            }
            m = *h_next;
        }
        LB_CHECK(hipMemcpyAsync(jobs_a, cref, 4, hipMemcpyDeviceToDevice, s));   // root = the last cluster
    } else {
        lbvh_tree_k<<<blocks(n - 1), kThreads, 0, s>>>(src, n, child, parent, leaf_parent, first, count);
        lbvh_key_ids_k<<<blocks(n), kThreads, 0, s>>>(src, n, (1ull << id_bits) - 1ull);
        lbvh_boxes_up_k<<<blocks(n), kThreads, 0, s>>>(src, n, child, parent, leaf_parent, tri_box, node_box, flag);
    }
    LB_CHECK(hipGetLastError());
    {   // SAH-DP choices of every inner node, bottom-up
        LB_CHECK(hipMemsetAsync(flag, 0, 4 * (size_t)n, s));
        DpArgs D;
        D.keys = src;
        D.child = child;
        D.parent = parent;
        D.leaf_parent = leaf_parent;
        D.count = count;
        D.tri_box = tri_box;
        D.node_box = node_box;
        D.cost = cost;
        D.choice = choice;
        D.flag = flag;
        D.n = n;
        D.c_node = in.c_node;
        D.c_prim = in.c_prim;
        lbvh_dp_up_k<<<blocks(n), kThreads, 0, s>>>(D);
        LB_CHECK(hipGetLastError());
    }
    // collapse, one level per launch; the next level's job count comes back to the host
    CollapseArgs A;
    A.keys = src;
    A.child = child;
    A.first = first;
    A.count = count;
    A.tri_box = tri_box;
    A.node_box = node_box;
    A.maxabs_bits = misc + 6;
    A.counters = misc + 8;
    A.n = n;
    A.nodes8 = out.nodes8;
    A.node8_box = out.node_box;
    A.tri_order = out.tri_order;
    A.choice = choice;
    res->level_off.assign(1, 0u);
    uint32_t n_jobs = 1, total = 1;
    while (n_jobs > 0) {
        if ((int)res->level_off.size() > kStackSize) {
            *err = "lbvh: 8-wide tree deeper than the traversal stack";
            return false;
        }
        LB_CHECK(hipMemsetAsync(misc + 10, 0, 4, s));
        A.jobs_in = jin;
        A.jobs_out = jout;
        A.n_jobs = n_jobs;
        lbvh_collapse_k<<<blocks(n_jobs), kThreads, 0, s>>>(A);
        LB_CHECK(hipGetLastError());
        LB_CHECK(hipMemcpyAsync(h_next, misc + 10, 4, hipMemcpyDeviceToHost, s));
        LB_CHECK(hipStreamSynchronize(s));
        const uint32_t next = *h_next;
        if (next > n) {
            *err = "lbvh: job queue overflow";
            return false;
        }
        res->level_off.push_back(total);
        total += next;
        n_jobs = next;
        std::swap(jin, jout);
    }
    res->num_nodes = total;
    res->max_depth = (int)res->level_off.size() - 1;
    LB_CHECK(hipMemcpyAsync(h_next, misc + 12, 4, hipMemcpyDeviceToHost, s));
    LB_CHECK(hipStreamSynchronize(s));
    if (*h_next != 0u) {
        *err = "lbvh: collapse capacity guard tripped";
        return false;
    }
    LB_CHECK(hipMemcpyAsync(h_next, misc + 9, 4, hipMemcpyDeviceToHost, s));   // triangle slots filled
    LB_CHECK(hipStreamSynchronize(s));
    if (*h_next != n) {
        *err = "lbvh: leaves do not cover every triangle once";
        return false;
    }
    LB_CHECK(hipMemcpyAsync(h_next, misc + 6, 4, hipMemcpyDeviceToHost, s));
    lbvh_tri_bin_k<<<blocks(n), kThreads, 0, s>>>(out.tri_order, n, out.tri_bin);
    lbvh_iota_k<<<blocks(total), kThreads, 0, s>>>(out.levels, total);
    LB_CHECK(hipGetLastError());
    LB_CHECK(hipStreamSynchronize(s));
    float m;
    std::memcpy(&m, h_next, 4);
    res->pad = 4e-6f * m;
#undef LB_CHECK
    return true;
}

}  // namespace rt
