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
    items[n_items++] = make_item(A, A.child[2 * job.x], pad);
    items[n_items++] = make_item(A, A.child[2 * job.x + 1], pad);
    while (n_items < 8) {   // open the inner child with the largest surface area
        int best = -1;
        float ba = -1.0f;
        for (int i = 0; i < n_items; ++i)
            if (!items[i].leaf && item_area(items[i]) > ba) {
                ba = item_area(items[i]);
                best = i;
            }
        if (best < 0) break;
        const int r = items[best].ref;
        items[best] = make_item(A, A.child[2 * r], pad);
        items[n_items++] = make_item(A, A.child[2 * r + 1], pad);
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
    uint32_t n_internal = 0, n_tris = 0;
    for (int i = 0; i < n_items; ++i) {
        if (items[i].leaf) n_tris += items[i].count;
        else ++n_internal;
    }
    Bvh8Node nd;
    for (int c = 0; c < 8; ++c) nd.meta[c] = 0;
    nd.axis = (uint8_t)axis;
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
            nd.meta[i] = (uint8_t)(0x80u | rank);
            const uint32_t slot = atomicAdd(&A.counters[2], 1u);
            if (slot < A.n) A.jobs_out[slot] = make_int2(it.ref, (int)(nd.child_base + rank));
            else atomicOr(&A.counters[4], 4u);
            ++rank;
        } else {
            nd.meta[i] = (uint8_t)(((it.count - 1u) << 5) | toff);
            for (uint32_t t = 0; t < it.count; ++t) A.tri_order[nd.tri_base + toff + t] = (uint32_t)A.keys[it.first + t];
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
           + align256(64 * 4);              // bounds, maxabs, counters
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
    auto* misc = (uint32_t*)carve(64 * 4);   // [0..5] centroid bounds, [6] max |coord|, [8..10] counters
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
                                      1u, 0, 0, 0, 0, 0, 0, 0};
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
    lbvh_tree_k<<<blocks(n - 1), kThreads, 0, s>>>(src, n, child, parent, leaf_parent, first, count);
    lbvh_key_ids_k<<<blocks(n), kThreads, 0, s>>>(src, n, (1ull << id_bits) - 1ull);
    lbvh_boxes_up_k<<<blocks(n), kThreads, 0, s>>>(src, n, child, parent, leaf_parent, tri_box, node_box, flag);
    LB_CHECK(hipGetLastError());
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
    static const int2 root = make_int2(0, 0);
    LB_CHECK(hipMemcpyAsync(jobs_a, &root, sizeof root, hipMemcpyHostToDevice, s));
    res->level_off.assign(1, 0u);
    uint32_t n_jobs = 1, total = 1;
    int2* jin = jobs_a;
    int2* jout = jobs_b;
    uint32_t* h_next = out.h_scratch;   // pinned
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
