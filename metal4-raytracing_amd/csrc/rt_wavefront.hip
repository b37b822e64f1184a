// rt_wavefront.hip — wavefront path tracer for gfx950.
//
// The per-pixel loop of raytracingKernel (Raytracing.metal:269-790) is split into stages over
// SoA path state and compacted queues, so every wave64 works on live paths only:
//   generate  one thread per (own pixel, sample): primary ray (:270-292) -> ray queue
//   extend    closest-hit traversal of the ray queue (:314-322)          -> hit records
//   shade     shade_step per hit (:324-774): updates path state, appends the continuation
//             ray to the next queue and the NEE shadow ray to the shadow queue
//   connect   any-hit traversal of the shadow queue (:716-743); unoccluded -> accum += contrib
//   finish    once fewer than kTailRays paths are alive, one launch runs every remaining path
//             to completion (trace -> shade -> shadow per thread): the long glass-path tail
//             costs the longest remaining path instead of one launch per bounce
//   [extra]   motion-adaptive extra samples (:779-789) as a second generate/iterate pass
//   resolve   per pixel: sum samples in sample order, average, temporal EMA (:777, :792-819)
//
// Queues are split into kShards segments; a block appends to segment blockIdx % 8 with ONE
// returning atomic per 256 entries (wave ballot + LDS prefix), so no counter word sees more
// than ~1/2048 of the entries (one word serialises at ~88 atomics/us, MI355X_MICROARCH.md
// 'dequeue').  Grids are multiples of 8, so segment k only receives chunks c == k (mod 8) and
// a segment of n/8 + 4096 (+ 256 per extra sample) entries can never overflow.
//
// Results are bit-identical to the megakernel: per-path arithmetic is the same shade_step,
// the accumulation order per path is the reference's (emission of step s, then its shadow
// contribution, then step s+1), and samples are summed per pixel in sample order.
#include "rt_shade.h"

#include <atomic>
#include <cstdio>
#include <cstring>
#include <vector>

namespace rt {

namespace {

// frames of kTeamAutoMin .. kTeamAutoPaths base paths use the finish kernel's team drain by default
// (rt_tuning.team = 0): the C3g rank shares gain, the tiny C1 frame (65K paths) loses 7.5 %
constexpr uint32_t kTeamAutoPaths = 2500000u;
constexpr uint32_t kTeamAutoMin = 262144u;

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

struct BlockAlloc {
    uint32_t w[kBlock / 64];
};

// Block-aggregated slot allocation; every thread of the block calls it (converged loop).
__device__ __forceinline__ uint32_t block_alloc(bool pred, uint32_t* counter, BlockAlloc& sh) {
    const int wave = threadIdx.x >> 6;
    unsigned long long m = __ballot(pred);
    uint32_t prefix = mbcnt64(m);
    if (lane_id() == 0) sh.w[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t c0 = sh.w[0], c1 = sh.w[1], c2 = sh.w[2], c3 = sh.w[3];
        uint32_t tot = c0 + c1 + c2 + c3;
        uint32_t b = tot ? atomicAdd(counter, tot) : 0u;
        sh.w[0] = b;
        sh.w[1] = b + c0;
        sh.w[2] = b + c0 + c1;
        sh.w[3] = b + c0 + c1 + c2;
    }
    __syncthreads();
    uint32_t r = sh.w[wave] + prefix;
    __syncthreads();
    return r;
}

// Three block-aggregated allocations at once (wf_shade: pr[0] shadow ray, pr[1] front / pr[2] back
// continuation ray), one returning global atomic per part and block, with the continuation rays
// grouped by the direction octant `oct` (3 bits) inside each part's range: a per-block counting
// sort of the appends through LDS atomics (the rank inside an octant is arbitrary), no separate
// sort pass.
struct BlockAllocOct {
    uint32_t cnt[3][8];    // shadow uses [0][0]
    uint32_t base[3][8];
};
__device__ __forceinline__ void block_alloc3_oct(const bool (&pr)[3], uint32_t oct, uint32_t* const (&ctr)[3],
                                                 BlockAllocOct& sh, uint32_t (&out)[3]) {
    if (threadIdx.x < 24) (&sh.cnt[0][0])[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t rank[3] = {0u, 0u, 0u};
    #pragma unroll
    for (int i = 0; i < 3; ++i)
        if (pr[i]) rank[i] = atomicAdd(&sh.cnt[i][i ? oct : 0u], 1u);
    __syncthreads();
    if (threadIdx.x < 3) {
        const int i = threadIdx.x;
        uint32_t tot = 0, pre[8];
        #pragma unroll
        for (int o = 0; o < 8; ++o) { pre[o] = tot; tot += sh.cnt[i][o]; }
        const uint32_t b = tot ? atomicAdd(ctr[i], tot) : 0u;
        #pragma unroll
        for (int o = 0; o < 8; ++o) sh.base[i][o] = b + pre[o];
    }
    __syncthreads();
    #pragma unroll
    for (int i = 0; i < 3; ++i) out[i] = sh.base[i][i ? oct : 0u] + rank[i];
    __syncthreads();
}

// Block-aggregated allocation of v slots per thread (wave scan + LDS prefix, one atomic per block).
__device__ __forceinline__ uint32_t block_alloc_n(uint32_t v, uint32_t* counter, BlockAlloc& sh) {
    const int wave = threadIdx.x >> 6;
    const uint32_t lane = lane_id();
    uint32_t incl = v;
    #pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t t = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += t;
    }
    if (lane == 63) sh.w[wave] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t c0 = sh.w[0], c1 = sh.w[1], c2 = sh.w[2], c3 = sh.w[3];
        uint32_t tot = c0 + c1 + c2 + c3;
        uint32_t b = tot ? atomicAdd(counter, tot) : 0u;
        sh.w[0] = b;
        sh.w[1] = b + c0;
        sh.w[2] = b + c0 + c1;
        sh.w[3] = b + c0 + c1 + c2;
    }
    __syncthreads();
    uint32_t r = sh.w[wave] + incl - v;
    __syncthreads();
    return r;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const uint32_t lane = lane_id();
    #pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(v, off, 64);
        if (lane >= (uint32_t)off) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t compact1by1(uint32_t x) {
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0f0f0f0fu;
    x = (x | (x >> 4)) & 0x00ff00ffu;
    x = (x | (x >> 8)) & 0x0000ffffu;
    return x;
}


__device__ __forceinline__ uint32_t pack_state(int bounce, int tpass, int step) {
    return (uint32_t)bounce | ((uint32_t)tpass << 8) | ((uint32_t)step << 16);
}

// n / d for 32-bit n by a multiply-high and two shifts (Granlund, Montgomery, PLDI 1994, fig. 4.1):
// the path-id -> pixel mappings run per refill / per shaded hit, where an integer division by a
// run-time divisor costs ~30 VALU instructions
struct FastDiv {
    uint32_t d, m, s1, s2;
};
static FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) ++l;
    f.m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
    f.s1 = l < 1 ? l : 1;
    f.s2 = l > 1 ? l - 1 : 0;
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    const uint32_t t = __umulhi(f.m, n);
    return (t + ((n - t) >> f.s1)) >> f.s2;
}

struct WfParams {
    WavefrontBuffers W;
    uint32_t base_paths;   // own pixels * spp
    uint32_t own_pixels;
    uint32_t seg_cap;      // entries per queue segment
    int spp;
    int refill_min;        // wf_trace / wf_finish_step refill once at least this many lanes of a wave are idle
    int chunk;             // wf_trace: rays per chunk grab
    uint32_t tail;         // live paths below which wf_finish_step runs the rest
    uint32_t sort_bins;    // hit-sort bins (0 = shade reads the extend queue unsorted)
    int diag;              // wf_finish_step: record the diagnostics slots (RT_WF_LOG)
    int shade_min;         // wf_finish_step: shade once this many lanes wait (or none traverses)
    int shade_min_x;       // wf_finish_step: the same once the launch's queue is exhausted (< 0: percent of busy lanes)
    int team;              // wf_finish_step: lanes per query in the drain (0: no team drain)
    int fchunk;            // wf_finish_step: paths per chunk grab
    int finish_frac;       // percent of the resident grid the finish launch takes
    int trace_frac;        // percent of the resident grid the bulk wf_trace launches take
    unsigned shade_blocks; // wf_shade grid
    int spans;             // record device-clock launch spans (rt_set_device_spans)
    int dev_ctl;           // device-side control (enqueue_wavefront): kernels read their queue sizes from
                           // the counters and skip once the live count fell below `tail`
    int finish_q;          // dev_ctl: the finish queue when every enqueued bulk round ran (written by generate)
    const FrameParams* Pd; // this frame's FrameParams in device memory (W.d_params)
    // own pixel index -> image pixel (own_pixel): tiles tile_id % nranks == rank of tile x tile pixels
    FastDiv spp_div, tile_px_div, tiles_x_div;   // by spp, tile * tile, tiles per row
    int tile, rank, nranks;
};

// own pixel index -> image coordinates (tiles tile_id % nranks == rank, Morton order in a tile)
__device__ __forceinline__ void own_pixel(const WfParams& Q, uint32_t i, int& px, int& py) {
    const uint32_t T = (uint32_t)Q.tile;
    const uint32_t k = fdiv(i, Q.tile_px_div), r = i - k * Q.tile_px_div.d;
    const uint32_t tid = (uint32_t)Q.rank + k * (uint32_t)Q.nranks;
    const uint32_t ty = fdiv(tid, Q.tiles_x_div), tx = tid - ty * Q.tiles_x_div.d;
    uint32_t lx, ly;
    if ((T & (T - 1)) == 0) {
        lx = compact1by1(r);
        ly = compact1by1(r >> 1);
    } else {
        lx = r % T;
        ly = r / T;
    }
    px = (int)(tx * T + lx);
    py = (int)(ty * T + ly);
}

// counter slots (cslot): [q*8 + shard] ray queues q = 0, 1; [16 + shard] shadow queue; [24] extra allocator
constexpr int kCntShadowQ = 16;
constexpr int kCntExtra = 24;
// [66..73] per-XCD chunk counters of the finish launch: XCD k takes chunks k, k + 8, k + 16, ...
// of the finish queue (its long-first order kept chip-wide).  One counter for the whole chip
// serialised the grabs: 3.4M paths in chunks of 32 were ~105K returning atomics on one line.
constexpr int kCntChunkFinish = 66;
constexpr int kCntSorted = 26;                 // hits the sort kept (misses dropped) = shade's input size
constexpr uint32_t kNoKey = 0xffffffffu;       // sort key of a miss (dropped by the sort)
constexpr int kCntDiagSegs = 27, kCntDiagIters = 28, kCntDiagTime = 29;   // wf_finish diagnostics
// dev_ctl: [30] tail mode (set by the first extend launch that found fewer than `tail` live
// paths; later bulk launches of the pass return at once), [31] the queue the finish launch reads
constexpr int kCntTailMode = 30, kCntFinishQ = 31;

// Device-clock span of a launch (WfFrameStats::trace_dev_ms): block 0 records the start, the last
// wave of every block its end, as a max on its XCD's line (`done`: an LDS wave counter zeroed
// before the block's first barrier); ts < 0 (host-driven rounds, or spans off: rt_set_device_spans)
// records nothing.  C3g, four slots: one 64-bit atomic per wave on one line cost the frame 2.5 %
// (8.67-8.71 -> 8.47-8.50 Grays/s), per block on per-XCD lines still ~1 % (8.58-8.62), so the
// spans are off unless asked for.
__device__ __forceinline__ void ts_start(const WfParams& Q, int ts) {
    if (ts >= 0 && blockIdx.x == 0 && threadIdx.x == 0) Q.W.tstamp[ts * kTsStride] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void ts_end(const WfParams& Q, int ts, uint32_t* done) {
    if (ts < 0 || lane_id() != 0) return;
    if (atomicAdd(done, 1u) == (blockDim.x + 63u) / 64u - 1u)
        atomicMax(&Q.W.tstamp[ts * kTsStride + kTsLine * (1 + (int)(blockIdx.x % 8u))],
                  (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// dev_ctl statistics: rounds run, wf_trace launches run, rays they traced
__device__ __forceinline__ void stat_add(const WfParams& Q, int word, uint32_t v) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&Q.W.counts[kWfStat + word], v);
}
__device__ __forceinline__ bool tail_mode(const WfParams& Q) {
    return Q.dev_ctl && __builtin_amdgcn_readfirstlane(Q.W.counts[cslot(kCntTailMode)]) != 0u;
}
constexpr int kCntChunkExtend = 32;   // 8 per-XCD chunk counters each
constexpr int kCntChunkConnect = 40;

// Inclusive prefix of a sharded queue's segment counts, loaded once per kernel (uniform, so the
// loads are scalar and the lookups below stay in registers).
struct ShardPrefix {
    uint32_t end[kShards];
};
__device__ __forceinline__ ShardPrefix load_prefix(const uint32_t* cnt, uint32_t cap = 0xffffffffu) {
    ShardPrefix p;
    uint32_t acc = 0;
    #pragma unroll
    for (int k = 0; k < kShards; ++k) {
        acc += min(__builtin_amdgcn_readfirstlane(cnt[cslot(k)]), cap);   // a counter may run past a full segment
        p.end[k] = acc;
    }
    return p;
}
// A ray queue's shard k holds L[k] entries at the front of its segment (ascending) and S[k] at the
// back (descending from seg_cap - 1): wf_shade appends the continuation rays of paths that have
// refracted (likely_long) at the front and the rest at the back, so the finish kernel, which
// takes the queue front parts first, starts the long glass paths before the short ones (they
// would otherwise set the end of its launch).  Primary rays (generate, extra samples) go to the
// front.  Counters: L in [q * 8 + k], S in [kCntBack + q * 8 + k].
constexpr int kCntBack = 50;
struct QueueShards {
    uint32_t L[kShards], S[kShards];
};
__device__ __forceinline__ QueueShards load_queue(const uint32_t* counts, int q, uint32_t seg_cap) {
    QueueShards r;
    #pragma unroll
    for (int k = 0; k < kShards; ++k) {
        const uint32_t l = min(__builtin_amdgcn_readfirstlane(counts[cslot(q * kShards + k)]), seg_cap);
        r.L[k] = l;
        r.S[k] = min(__builtin_amdgcn_readfirstlane(counts[cslot(kCntBack + q * kShards + k)]), seg_cap - l);
    }
    return r;
}
__device__ __forceinline__ uint32_t queue_len(const QueueShards& qs) {
    uint32_t n = 0;
    #pragma unroll
    for (int k = 0; k < kShards; ++k) n += qs.L[k] + qs.S[k];
    return n;
}
// shard-local index g (< L + S) -> position in the shard's segment
__device__ __forceinline__ uint32_t seg_pos(uint32_t g, uint32_t l, uint32_t seg_cap) {
    return g < l ? g : seg_cap - 1u - (g - l);
}
// dense consumer index g (< queue_len) -> entry index: the front parts of all shards first, then the back parts
__device__ __forceinline__ uint32_t dense_entry(const QueueShards& qs, uint32_t g, uint32_t seg_cap) {
    uint32_t ltot = 0;
    #pragma unroll
    for (int k = 0; k < kShards; ++k) ltot += qs.L[k];
    const bool back = g >= ltot;
    if (back) g -= ltot;
    uint32_t k = 0, start = 0, acc = 0;
    #pragma unroll
    for (int j = 0; j < kShards - 1; ++j) {
        acc += back ? qs.S[j] : qs.L[j];
        const bool past = g >= acc;
        k = past ? (uint32_t)(j + 1) : k;
        start = past ? acc : start;
    }
    const uint32_t i = g - start;
    return k * seg_cap + (back ? seg_cap - 1u - i : i);
}
__device__ __forceinline__ bool likely_long(const PathRegs& p) {
    return p.tpass > 0 || p.bounce < p.step;
}

// A path's state between launches: its accumulator here (indexed by path id), its throughput
// colour and bounce / step counters in the queue entry of its next ray (qc, d.w), its pixel,
// sample and Halton index recomputed from the path id (path_meta); only the extra-sample paths,
// whose ids do not encode their pixel, keep them in p_meta.
__device__ __forceinline__ void init_path(const WfParams& Q, uint32_t pid, uint32_t pix, int sample, uint32_t hidx) {
    Q.W.p_accum[pid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (pid >= Q.base_paths) Q.W.p_meta[pid] = make_uint4(pix, (uint32_t)sample, 0u, hidx);
}


__device__ __forceinline__ void flush_counters(const FrameParams& P, uint32_t closest, uint32_t shadow, uint32_t paths,
                                               const TraceCounters& tc, bool count, bool overflow,
                                               bool trace_kernel = false) {
    block_flush_counters(P.counters, closest, shadow, count ? tc.nodes : 0u, count ? tc.tris : 0u, paths, overflow,
                         trace_kernel, count ? tc.lds_nodes : 0u);
}

// per-pixel outputs of a shade step (depth / motion / G-buffer, :342-389, :506-515)
// (depth and motion: the hit is recorded and wf_motion evaluates it after the pass)
__device__ __forceinline__ void write_pixel_outputs(const FrameParams& P, uint32_t pix, const StepResult& r, const Hit& h,
                                                    bool full) {
    if (r.primary) P.prim_hit[pix] = make_uint4(h.id, __float_as_uint(h.u), __float_as_uint(h.v), 0u);
    if (full && r.gbuf && P.gbuffer) {
        size_t plane = (size_t)P.U.width * P.U.height;
        P.gbuffer[pix] = r.g0;
        P.gbuffer[plane + pix] = r.g1;
        P.gbuffer[2 * plane + pix] = r.g2;
        P.gbuffer[3 * plane + pix] = r.g3;
    }
}

}  // namespace

// ---- one traversal step of the compressed 8-wide BVH, shared by wf_trace and wf_finish_step ------
// The state of one query in registers: ray setup, closest hit so far (u = bu / bdet, v = bv / bdet:
// the division happens once, when the query ends), the current node group (child base, flip,
// remaining internal hits), the pending triangles of the last node test, and the LDS stack.
struct Trav {
    RaySetup R;
    float best, bu, bv, bdet;
    uint32_t best_id, g_base, g_hits, t_base, t_mask, t_valid;
    bool g_flip, hit_any;
    int sp;
};

__device__ __forceinline__ void trav_start(Trav& T, f3 o, f3 d, float tmax) {
    T.R = ray_setup(o, d);
    T.best = tmax;
    T.best_id = 0xffffffffu;
    T.bu = T.bv = 0.0f;
    T.bdet = 1.0f;
    T.g_base = 0;
    T.g_hits = 1;   // virtual group holding the root
    T.g_flip = false;
    T.t_mask = 0;
    T.sp = 0;
    T.hit_any = false;
}

// One iteration of a query: up to two triangles of the last node test (both fetched before either
// is tested: one memory latency; tested in mask order, so closest-hit updates are those of the
// serial loop), then — for a lane whose triangles ran out in this step, and for every lane without
// triangles — one 8-wide node: the next hit child of the current group in slot order (the node's
// children sorted along its longest axis, reversed for rays going the other way), its five 16-B
// words fetched from global memory (an LDS copy of the top levels measured no faster, DESIGN.md
// §3.5).  Returns true once the query is finished (any-hit: an occluder was found).
// The next node's group / stack bookkeeping and index (the step after the triangles of the last
// node test, or a node step without triangles).
__device__ __forceinline__ uint32_t next_node(Trav& T, int* stack, bool& overflow) {
    if (!T.g_hits) {
        --T.sp;
        const uint32_t ent = (uint32_t)stack[T.sp * kBlock];
        T.g_base = ent >> 9;
        T.g_flip = (ent >> 8) & 1u;
        T.g_hits = ent & 0xffu;
    }
    const int r = T.g_flip ? highest_bit(T.g_hits) : lowest_bit(T.g_hits);
    T.g_hits &= ~(1u << r);
    if (T.g_hits) {
        if (T.sp < kStackSize) {
            stack[T.sp * kBlock] = (int)pack_group(T.g_base, T.g_flip, T.g_hits);
            ++T.sp;
        } else {
            overflow = true;
        }
    }
    return T.g_base + (uint32_t)r;
}

// The node half of a traversal step: the next node of the current group (or the stack), its five
// 16-B words from global memory, the 8-wide test.
template <bool COUNT>
__device__ __forceinline__ void node_step(const DevScene& S, Trav& T, int* stack, TraceCounters& tc, bool& overflow,
                                          float cull) {
    const uint32_t ni = next_node(T, stack, overflow);
    if (COUNT) tc.nodes++;
    const NodeWords w = load_node8(S.nodes8, ni);
    test_node8_words(w, T.R, 0.0f, fminf(cull, T.best), T.g_hits, T.t_mask, T.t_valid, T.g_base, T.t_base, T.g_flip);
}

// `cull`: the distance bound of the box and triangle tests together with T.best (the lower of the
// two); lower than T.best in the finish kernel's team drain (the closest hit any member of the team
// has found), where T.best stays this lane's own hit.
template <bool COUNT>
__device__ __forceinline__ bool trav_step(const DevScene& S, Trav& T, bool any, int* stack, TraceCounters& tc,
                                          bool& overflow, float cull) {
    bool tdone = false;
    if (T.t_mask != 0u) {
        const int k0 = lowest_bit(T.t_mask);
        T.t_mask &= T.t_mask - 1u;
        const bool two = T.t_mask != 0u;
        const int k1 = two ? lowest_bit(T.t_mask) : k0;
        if (two) T.t_mask &= T.t_mask - 1u;
        // the bound is re-read for every test: a triangle must not be accepted beyond a closer hit
        // found earlier in this step (the update below assumes t <= T.best)
#ifdef RT_XP_STALE_BOUND
        // round 3's bug, kept as a build-time switch to show the parity tests catch it
        // (tests/test_gpu_traversal_variants.py): both triangles against the bound from before the step
        const float stale_bound = fminf(cull, T.best);
#define RT_ISECT(a, b, c) intersect_rot(T.R.pre, T.R.o, a, b, c, 0.0f, stale_bound, &t, &u, &v, &dt)
#else
#define RT_ISECT(a, b, c) intersect_rot(T.R.pre, T.R.o, a, b, c, 0.0f, fminf(cull, T.best), &t, &u, &v, &dt)
#endif
        // each vertex as the ray's (kz, kx, ky) window of its record: three 12-B loads and the id
        // per triangle, all in the slot's 64-B line (rt_device.h); both triangles' loads issue
        // before either test
        const uint32_t kz = (uint32_t)T.R.pre.kz;
        const uint32_t f0 = tri_slot(T.t_base, T.t_valid, k0) * (uint32_t)kTriFloats + kz;
        const uint32_t f1 = tri_slot(T.t_base, T.t_valid, k1) * (uint32_t)kTriFloats + kz;
        const f3 a0 = tri_window_at(S.tris, f0), a1 = tri_window_at(S.tris, f0 + 5u), a2 = tri_window_at(S.tris, f0 + 10u);
        const uint32_t ida = tri_id_at(S.tris, f0 - kz);
        const f3 b0 = tri_window_at(S.tris, f1), b1 = tri_window_at(S.tris, f1 + 5u), b2 = tri_window_at(S.tris, f1 + 10u);   // = a for one triangle
        const uint32_t idb = tri_id_at(S.tris, f1 - kz);
        if (COUNT) tc.tris += two ? 2u : 1u;
        float t, u, v, dt;
        if (RT_ISECT(a0, a1, a2)) {
            const uint32_t id = ida;
            if (any) {
                T.hit_any = true;
                tdone = true;
            } else if (t < T.best || id < T.best_id) {
                T.best = t;
                T.best_id = id;
                T.bu = u;
                T.bdet = dt;
                T.bv = v;
            }
        }
        if (two && !tdone && RT_ISECT(b0, b1, b2)) {
            const uint32_t id = idb;
            if (any) {
                T.hit_any = true;
                tdone = true;
            } else if (t < T.best || id < T.best_id) {
                T.best = t;
                T.best_id = id;
                T.bu = u;
                T.bdet = dt;
                T.bv = v;
            }
        }
    }
    if (!tdone && T.t_mask == 0u && (T.g_hits != 0u || T.sp > 0)) node_step<COUNT>(S, T, stack, tc, overflow, cull);
    return tdone || (T.t_mask == 0u && T.g_hits == 0u && T.sp == 0);
#undef RT_ISECT
}

// ---- base paths ----------------------------------------------------------------------------------------
// Halton index of sample s of pixel pix in this frame (:263-270)
__device__ __forceinline__ uint32_t base_hidx(const FrameParams& P, int spp, uint32_t pix, int s) {
    const Uniforms& U = P.U;
    const int maxExtra = (U.enableMotionAdaptiveSampling != 0) ? max(U.motionSamplingMaxExtraSamples, 0) : 0;
    const int frameOffset = (int)U.frameIndex * (spp + maxExtra) + s;
    return (uint32_t)(int)(P.random[pix] + (unsigned)frameOffset);
}
// Path pid of the base pass (own pixel pid / spp, sample pid % spp): its pixel, sample, Halton index
// (:263-270) and primary ray (:270-292).  False for a path of a tile pixel outside the image.
__device__ __forceinline__ bool base_path(const FrameParams& P, const WfParams& Q, const ShadeTabs& halton, uint32_t pid,
                                          uint32_t& pix, int& s, uint32_t& hidx, f3& o, f3& d) {
    const Uniforms& U = P.U;
    const uint32_t i = fdiv(pid, Q.spp_div);
    s = (int)(pid - i * Q.spp_div.d);
    int px, py;
    own_pixel(Q, i, px, py);
    if (px >= U.width || py >= U.height) return false;
    pix = (uint32_t)py * (uint32_t)U.width + (uint32_t)px;
    hidx = base_hidx(P, Q.spp, pix, s);
    primary_ray(U, halton, px, py, (int)hidx, o, d);
    return true;
}
// (pixel, sample, Halton index) of path pid: a base path's from its id, as wf_generate made them;
// an extra-sample path's from p_meta (wf_extra)
__device__ __forceinline__ uint3 path_meta(const FrameParams& P, const WfParams& Q, uint32_t pid) {
    if (pid >= Q.base_paths) {
        const uint4 m = Q.W.p_meta[pid];
        return make_uint3(m.x, m.y, m.w);
    }
    const uint32_t i = fdiv(pid, Q.spp_div);
    const int s = (int)(pid - i * Q.spp_div.d);
    int px, py;
    own_pixel(Q, i, px, py);
    const uint32_t pix = (uint32_t)py * (uint32_t)P.U.width + (uint32_t)px;
    return make_uint3(pix, (uint32_t)s, base_hidx(P, Q.spp, pix, s));
}
// Per-pixel defaults, written by the pixel's sample-0 path (:252-261).
__device__ __forceinline__ void init_pixel(const FrameParams& P, uint32_t pix) {
    P.depth[pix] = 1.0e8f;
    P.motion[pix] = make_float2(0.0f, 0.0f);
    P.prim_hit[pix] = make_uint4(0xffffffffu, 0u, 0u, 0u);
    if (P.gbuffer) {
        const size_t plane = (size_t)P.U.width * P.U.height;
        const float4 z = make_float4(0, 0, 0, 0);
        P.gbuffer[pix] = z;
        P.gbuffer[plane + pix] = z;
        P.gbuffer[2 * plane + pix] = z;
        P.gbuffer[3 * plane + pix] = z;
    }
}
// ---- generate -------------------------------------------------------------------------------------
// (A first round fused with generate -- extend making the primary rays at refill, shade starting
// the path state -- was measured slower)
__global__ void __launch_bounds__(kBlock) wf_generate(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    __shared__ HaltonDim lds_halton[kHaltonLds];
    __shared__ BlockAlloc ba;
    const ShadeTabs halton = load_tabs(S, lds_halton, nullptr);   // no shading: Halton only
    const Uniforms& U = P.U;
    const int spp = Q.spp;
    const int shard = blockIdx.x & (kShards - 1);
    float4* qout = Q.W.q[0] + 2 * (size_t)shard * Q.seg_cap;
    uint32_t n_paths = 0;
    const uint32_t total = Q.base_paths;
    if (Q.dev_ctl && blockIdx.x == 0 && threadIdx.x == 0) Q.W.counts[cslot(kCntFinishQ)] = (uint32_t)Q.finish_q;
    for (uint32_t base = blockIdx.x * kBlock; base < total; base += gridDim.x * kBlock) {
        uint32_t pid = base + threadIdx.x;
        int s = 0;
        uint32_t pix = 0, hidx = 0;
        f3 o = mk3(0, 0, 0), d = mk3(0, 0, 0);
        const bool valid = pid < total && base_path(P, Q, halton, pid, pix, s, hidx, o, d);
        if (valid) {
            init_path(Q, pid, pix, s, hidx);
            if (s == 0) init_pixel(P, pix);
            n_paths++;
        }
        bool live = valid && U.maxBounces > 0;
        uint32_t slot = block_alloc(live, &Q.W.counts[cslot(shard)], ba);
        if (live) {
            qout[2 * slot] = make_float4(o.x, o.y, o.z, __uint_as_float(pid));
            qout[2 * slot + 1] = make_float4(d.x, d.y, d.z, 0.0f);
        }
    }
    TraceCounters tc{0, 0, 0};
    flush_counters(P, 0, 0, n_paths, tc, false, false);
}

// ---- shade -------------------------------------------------------------------------------------------
// SORTED: the input is the hit-sorted array (wf_sort_scatter; misses already dropped) and the
// blocks of XCD k (blockIdx % 8) shade the k-th eighth of it, so one XCD's L2 serves one scene
// region and the rays / shadow rays it appends to its queue shard stay grouped by region for
// the next extend / connect launches (which hand shard k's range to XCD k).
// a 16-B load of data read once (nontemporal: it does not displace the lines gathered beside it).
// wf_shade and the finish refill read their queue entries this way; wf_trace (extend) does not
// (wf_shade reads the same entries again: nontemporal extend loads slowed it, round 4)
__device__ __forceinline__ float4 ld_stream(const float4* p) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 ld_shade(const float4* p) { return ld_stream(p); }
template <bool FULL, bool SORTED>
__global__ void __launch_bounds__(kBlock) wf_shade(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q, int cur) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    __shared__ HaltonDim lds_halton[kHaltonLds];
    __shared__ MatRec lds_mat[kMatLds];
    __shared__ float4 lds_inst[3 * kInstLds];
    __shared__ Light lds_light[kLightLds];
    __shared__ BlockAllocOct bao;
    if (tail_mode(Q)) return;
    const ShadeTabs halton = load_tabs(S, lds_halton, lds_mat, lds_inst, lds_light, P.U.lightCount);
    const Uniforms& U = P.U;
    const int next = 1 - cur;
    const int shard = blockIdx.x & (kShards - 1);
    const QueueShards qs = load_queue(Q.W.counts, cur, Q.seg_cap);
    const float4* qin = Q.W.q[cur];
    float4* qout = Q.W.q[next] + 2 * (size_t)shard * Q.seg_cap;
    float4* qcout = Q.W.qc[next] + (size_t)shard * Q.seg_cap;
    float4* sqout = Q.W.sq + 3 * (size_t)shard * Q.seg_cap;
    f2 zero2;
    zero2.x = 0.0f;
    zero2.y = 0.0f;
    // the blocks of XCD k (blockIdx % 8, the grid is a multiple of 8: grid_for) take queue shard k,
    // which XCD k's extend launch traced (unsorted), or the k-th eighth of the sorted array
    uint32_t beg = (blockIdx.x >> 3) * kBlock, end = 0, ebase = 0, lk = 0;
    const uint32_t stride = (gridDim.x >> 3) * kBlock;
    if (SORTED) {
        const uint32_t n = __builtin_amdgcn_readfirstlane(Q.W.counts[cslot(kCntSorted)]);
        beg += (uint32_t)(((uint64_t)n * (uint32_t)shard) / kShards);
        end = (uint32_t)(((uint64_t)n * (uint32_t)(shard + 1)) / kShards);
    } else {
        #pragma unroll
        for (int j = 0; j < kShards; ++j)
            if (j == shard) {
                lk = qs.L[j];
                end = qs.L[j] + qs.S[j];
            }
        ebase = (uint32_t)shard * Q.seg_cap;
    }
    for (uint32_t base = beg; base < end; base += stride) {
        uint32_t g = base + threadIdx.x;
        StepResult r;
        r.next = false;
        r.shadow = false;
        uint32_t pid = 0, nstate = 0;   // nstate, ncol: the continuation's state bits and colour
        bool front = true;              // the continuation goes to the queue front (likely_long)
        f3 rayO = mk3(0, 0, 0), rayD = mk3(0, 0, 0);
        float4 ncol = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (g < end) {
            float4 o, d, hv;
            size_t ce = 0;   // the entry's colour: sorted[4g + 3] / qc[cur][e]
            if (SORTED) {
                o = Q.W.sorted[4 * (size_t)g];
                d = Q.W.sorted[4 * (size_t)g + 1];
                hv = Q.W.sorted[4 * (size_t)g + 2];
                ce = 4 * (size_t)g + 3;
            } else {
                const uint32_t e = ebase + seg_pos(g, lk, Q.seg_cap);
                o = ld_shade(&qin[2 * (size_t)e]);
                d = ld_shade(&qin[2 * (size_t)e + 1]);
                hv = ld_shade(&Q.W.hits[e]);
                ce = e;
            }
            pid = __float_as_uint(o.w);
            Hit h;
            h.t = hv.x;
            h.id = __float_as_uint(hv.y);
            h.u = hv.z;
            h.v = hv.w;
            if (h.id != 0xffffffffu) {                                           // miss -> path ends (:321-322)
                const uint32_t state = __float_as_uint(d.w);
                const float4 c = state == 0u ? make_float4(1.0f, 1.0f, 1.0f, 0.0f)
                                             : (SORTED ? Q.W.sorted[ce] : ld_shade(&Q.W.qc[cur][ce]));
                // a continuation ray past bounce 0 carries its Halton index in qc.w: the pixel and sample
                // (and the per-pixel random offset behind them) are read only at bounce 0 (:342-389)
                uint4 meta;
                if ((state & 0xffu) != 0u) {
                    meta = make_uint4(0u, 1u, state, __float_as_uint(c.w));
                } else {
                    const uint3 pm = path_meta(P, Q, pid);
                    meta = make_uint4(pm.x, pm.y, state, pm.z);
                }
                // FULL=false: shade_step only adds color * emission to accum (:585), so it runs on a
                // zero accumulator and the stored one is read and updated only when that term is
                // non-zero (accum is never -0, so a + (0 + x) == a + x bit for bit); FULL (debug
                // modes assign accum) reads it first
                float4 a = FULL ? Q.W.p_accum[pid] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                PathRegs p;
                p.color = mk3(c.x, c.y, c.z);
                p.accum = mk3(a.x, a.y, a.z);
                p.bounce = (int)(meta.z & 0xffu);
                p.tpass = (int)((meta.z >> 8) & 0xffu);
                p.step = (int)(meta.z >> 16);
                int sample = (int)meta.y;
                rayO = ld3(o);
                rayD = ld3(d);
                shade_step<FULL, false>(S, U, halton, (int)meta.w, sample, rayO, rayD, h, p, sample == 0 && p.step == 0,
                                 zero2, false, zero2, r);
                write_pixel_outputs(P, meta.x, r, h, FULL);
                nstate = pack_state(p.bounce, p.tpass, p.step);
                front = likely_long(p);
                ncol = make_float4(p.color.x, p.color.y, p.color.z, __uint_as_float(meta.w));   // w: Halton index
                // radiance only changes on emissive hits (:585-586): skip the store otherwise
                if (__float_as_uint(p.accum.x) != __float_as_uint(a.x) || __float_as_uint(p.accum.y) != __float_as_uint(a.y) ||
                    __float_as_uint(p.accum.z) != __float_as_uint(a.z)) {
                    if (!FULL) {
                        const float4 s = Q.W.p_accum[pid];
                        p.accum = mk3(s.x + p.accum.x, s.y + p.accum.y, s.z + p.accum.z);
                    }
                    Q.W.p_accum[pid] = make_float4(p.accum.x, p.accum.y, p.accum.z, 0.0f);
                }
            }
        }
        const bool pr[3] = {r.shadow, r.next && front, r.next && !front};
        uint32_t* const ctr[3] = {&Q.W.counts[cslot(kCntShadowQ + shard)], &Q.W.counts[cslot(next * kShards + shard)],
                                  &Q.W.counts[cslot(kCntBack + next * kShards + shard)]};
        uint32_t slots[3];
        // continuation rays grouped by direction octant inside the block's range (round 5: +-0, kept)
        const uint32_t oct = (rayD.x < 0.0f ? 1u : 0u) | (rayD.y < 0.0f ? 2u : 0u) | (rayD.z < 0.0f ? 4u : 0u);
        block_alloc3_oct(pr, oct, ctr, bao, slots);
        const uint32_t ns = slots[0], nr = front ? slots[1] : Q.seg_cap - 1u - slots[2];
        if (r.shadow) {
            sqout[3 * (size_t)ns] = make_float4(r.so.x, r.so.y, r.so.z, __uint_as_float(pid));
            sqout[3 * (size_t)ns + 1] = make_float4(r.sd.x, r.sd.y, r.sd.z, r.stmax);
            sqout[3 * (size_t)ns + 2] = make_float4(r.contrib.x, r.contrib.y, r.contrib.z, 0.0f);
        }
        if (r.next) {
            qout[2 * (size_t)nr] = make_float4(rayO.x, rayO.y, rayO.z, __uint_as_float(pid));
            qout[2 * (size_t)nr + 1] = make_float4(rayD.x, rayD.y, rayD.z, __uint_as_float(nstate));
            qcout[nr] = ncol;
        }
    }
}

// ---- hit sort (between extend and shade) -------------------------------------------------------------
// A counting sort of the extend queue's hits by key (the bin of the hit triangle's BVH leaf slot,
// S.tri_bin; leaf order is spatially coherent, so a bin is one scene region), in three launches: per-block histograms, a scan of each bin's row of block counts, and a
// scatter that writes {o, d, hit} of every hit to its bin's range.  Misses are dropped (their
// paths end, :321-322).  The order inside a bin is arbitrary; per-path results do not depend on
// the order paths are shaded in, so the output stays bit-identical.
// block b's share of the dense queue index range (the same in hist and scatter)
__device__ __forceinline__ void sort_range(uint32_t n, uint32_t& beg, uint32_t& end) {
    beg = (uint32_t)(((uint64_t)n * blockIdx.x) / kSortBlocks);
    end = (uint32_t)(((uint64_t)n * (blockIdx.x + 1)) / kSortBlocks);
}

// sort key of queue entry e: kNoKey for a miss, else the leaf bin at Q.sort_bins resolution
__device__ __forceinline__ uint32_t sort_key(const DevScene& S, const WfParams& Q, uint32_t e, uint32_t shift) {
    const uint32_t id = __float_as_uint(Q.W.hits[e].y);
    return id == 0xffffffffu ? kNoKey : ((uint32_t)S.tri_bin[id] >> shift);
}

__global__ void __launch_bounds__(kSortThreads) wf_sort_hist(DevScene S, WfParams Q, int cur) {
    __shared__ uint32_t h[kSortMaxBins];
    if (tail_mode(Q)) return;
    const uint32_t shift = __builtin_ctz(kSortMaxBins) - __builtin_ctz(Q.sort_bins);
    const uint32_t K = Q.sort_bins;
    const QueueShards qs = load_queue(Q.W.counts, cur, Q.seg_cap);
    for (uint32_t k = threadIdx.x; k < K; k += kSortThreads) h[k] = 0;
    __syncthreads();
    uint32_t beg, end;
    sort_range(queue_len(qs), beg, end);
    for (uint32_t g = beg + threadIdx.x; g < end; g += kSortThreads) {
        const uint32_t k = sort_key(S, Q, dense_entry(qs, g, Q.seg_cap), shift);
        if (k != kNoKey) atomicAdd(&h[k], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < K; k += kSortThreads) Q.W.sort_table[(size_t)k * kSortBlocks + blockIdx.x] = h[k];
}

// one block per bin: exclusive scan of the bin's kSortBlocks block counts (in place) + bin total
__global__ void __launch_bounds__(kSortBlocks) wf_sort_rowscan(WfParams Q) {
    __shared__ uint32_t w[kSortBlocks / 64];
    if (tail_mode(Q)) return;
    uint32_t* row = Q.W.sort_table + (size_t)blockIdx.x * kSortBlocks;
    const uint32_t v = row[threadIdx.x];
    const uint32_t incl = wave_incl_scan(v);
    const int wave = threadIdx.x >> 6;
    if (lane_id() == 63) w[wave] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int i = 0; i < wave; ++i) base += w[i];
    row[threadIdx.x] = base + incl - v;
    if (threadIdx.x == kSortBlocks - 1) Q.W.sort_total[blockIdx.x] = base + incl;
}

__global__ void __launch_bounds__(kSortThreads) wf_sort_scatter(DevScene S, WfParams Q, int cur) {
    __shared__ uint32_t off[kSortMaxBins];
    if (tail_mode(Q)) return;
    const uint32_t shift = __builtin_ctz(kSortMaxBins) - __builtin_ctz(Q.sort_bins);
    __shared__ uint32_t w[kSortThreads / 64];
    const uint32_t K = Q.sort_bins, per = K / kSortThreads;   // 1, 2 or 4 bins per thread
    const QueueShards qs = load_queue(Q.W.counts, cur, Q.seg_cap);
    // bin starts: exclusive scan of the bin totals, plus this block's offset inside each bin
    uint32_t loc[kSortMaxBins / kSortThreads];
    uint32_t s = 0;
    for (uint32_t i = 0; i < per; ++i) {
        loc[i] = s;
        s += Q.W.sort_total[threadIdx.x * per + i];
    }
    const uint32_t incl = wave_incl_scan(s);
    const int wave = threadIdx.x >> 6;
    if (lane_id() == 63) w[wave] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int i = 0; i < wave; ++i) base += w[i];
    const uint32_t excl = base + incl - s;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t k = threadIdx.x * per + i;
        off[k] = excl + loc[i] + Q.W.sort_table[(size_t)k * kSortBlocks + blockIdx.x];
    }
    if (blockIdx.x == 0 && threadIdx.x == kSortThreads - 1) Q.W.counts[cslot(kCntSorted)] = excl + s;
    __syncthreads();
    const float4* qin = Q.W.q[cur];
    uint32_t beg, end;
    sort_range(queue_len(qs), beg, end);
    for (uint32_t g = beg + threadIdx.x; g < end; g += kSortThreads) {
        const uint32_t e = dense_entry(qs, g, Q.seg_cap);
        const float4 hv = Q.W.hits[e];
        const uint32_t id = __float_as_uint(hv.y);
        if (id == 0xffffffffu) continue;
        const uint32_t pos = atomicAdd(&off[(uint32_t)S.tri_bin[id] >> shift], 1u);
        const float4 o = qin[2 * (size_t)e], d = qin[2 * (size_t)e + 1];
        Q.W.sorted[4 * (size_t)pos] = o;
        Q.W.sorted[4 * (size_t)pos + 1] = d;
        Q.W.sorted[4 * (size_t)pos + 2] = hv;
        if (__float_as_uint(d.w) != 0u) Q.W.sorted[4 * (size_t)pos + 3] = Q.W.qc[cur][e];   // state 0: colour 1
    }
}

// connect: the accumulation of the unoccluded shadow rays of a wave, batched (one lane per pending
// entry: its path id and contribution from the shadow queue, then accum += contribution, :741-743)
// so the wave waits for these dependent loads once per up to 64 rays, not once per finishing step.
// A path has one shadow ray per connect launch, so the order of the additions is unchanged.
__device__ __forceinline__ void connect_flush(const WfParams& Q, const float4* qin, uint32_t* pend, uint32_t& npend) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t lane = lane_id();
    if (lane < npend) {
        const uint32_t e = pend[lane];
        const float4 o4 = qin[3 * (size_t)e];
        const float4 c = qin[3 * (size_t)e + 2];
        const uint32_t pid = __float_as_uint(o4.w);
        const float4 a = Q.W.p_accum[pid];
        Q.W.p_accum[pid] = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, 0.0f);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    npend = 0;
}

// ---- persistent traversal with per-lane refill (extend: ANY = false, connect: ANY = true) -----------
// The grid is the resident capacity.  Each XCD (blockIdx % 8) owns queue shard k (what its own shade blocks appended) and hands
// it out in chunks of Q.chunk rays, one atomic per chunk.  Every iteration advances each lane of a
// wave by one traversal step (trav_step); a lane whose query ended takes the next ray of the
// wave's chunk once at least Q.refill_min lanes are idle.  A wave therefore runs ~(steps of its
// rays) / 64 iterations instead of (slowest ray) x (rays per lane).
template <bool ANY, bool COUNT>
#ifndef RT_EXTEND_WAVES
#define RT_EXTEND_WAVES 8
#endif
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(ANY ? 8 : RT_EXTEND_WAVES, ANY ? 8 : RT_EXTEND_WAVES)))
wf_trace(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q, int cur, int ts) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    __shared__ int lds_stack[kStackSize * kBlock];
    int* stack = &lds_stack[threadIdx.x];
    if (Q.dev_ctl) {
        // device-side round control: extend decides (uniformly, from the counters) whether this
        // round runs in bulk or the rest of the pass goes to the finish launch
        const bool tm = tail_mode(Q);
        if (ANY) {
            if (tm) return;
        } else {
            if (tm || queue_len(load_queue(Q.W.counts, cur, Q.seg_cap)) < Q.tail) {
                if (!tm && blockIdx.x == 0 && threadIdx.x == 0) {
                    Q.W.counts[cslot(kCntTailMode)] = 1u;
                    Q.W.counts[cslot(kCntFinishQ)] = (uint32_t)cur;
                }
                return;
            }
        }
    }
    __shared__ uint32_t ts_done;
    if (threadIdx.x == 0) ts_done = 0u;
    ts_start(Q, ts);
    __syncthreads();
    // the shadow queue is one-sided, a ray queue two-sided (front / back parts)
    const uint32_t n = ANY ? load_prefix(Q.W.counts + cslot(kCntShadowQ)).end[kShards - 1]
                           : queue_len(load_queue(Q.W.counts, cur, Q.seg_cap));
    if (Q.dev_ctl) {
        stat_add(Q, kStatTraceRays, n);
        stat_add(Q, kStatTraceLaunches, 1u);
        if (!ANY) {
            stat_add(Q, kStatRounds, 1u);
            stat_add(Q, kStatExtendRays, n);
        }
    }
    if (!ANY && blockIdx.x == 0 && threadIdx.x < 3 * kShards) {  // reset the queues shade / connect fill
        const int next = 1 - cur;
        const uint32_t k = threadIdx.x & (kShards - 1), part = threadIdx.x / kShards;
        Q.W.counts[cslot(part == 0 ? next * kShards + k : part == 1 ? kCntShadowQ + k : kCntBack + next * kShards + k)] = 0;
    }
    // chunk counters of the OTHER traversal kind are reset here for its next launch (extend and
    // connect alternate; the frame start zeroes both)
    if (blockIdx.x == 0 && threadIdx.x < kShards)
        Q.W.counts[cslot((ANY ? kCntChunkExtend : kCntChunkConnect) + threadIdx.x)] = 0;
    const float4* qin = ANY ? Q.W.sq : Q.W.q[cur];
    const int qstride = ANY ? 3 : 2;
    // chunks of this XCD's part of the queue, grabbed with one atomic per chunk
    const uint32_t xcd = blockIdx.x & 7u;
    uint32_t* const chunk_ctr = Q.W.counts + cslot((ANY ? kCntChunkConnect : kCntChunkExtend) + (int)xcd);
    // XCD k traverses queue shard k, the segment its own shade blocks (blockIdx % 8 == k) appended:
    // entry = k * seg_cap + g, no per-lane search of the shard prefix
    // shard xcd's entries and its front part (two scalar loads)
    uint32_t xl, xend;
    if (ANY) {
        xl = xend = min(__builtin_amdgcn_readfirstlane(Q.W.counts[cslot(kCntShadowQ + (int)xcd)]), Q.seg_cap);
    } else {
        xl = min(__builtin_amdgcn_readfirstlane(Q.W.counts[cslot(cur * kShards + (int)xcd)]), Q.seg_cap);
        xend = xl + min(__builtin_amdgcn_readfirstlane(Q.W.counts[cslot(kCntBack + cur * kShards + (int)xcd)]),
                        Q.seg_cap - xl);
    }
    // (round 3; before, XCD k took the k-th eighth of the dense queue and every refilling lane
    // searched the prefix for its entry: 7.49 -> 7.56 Grays/s)
    const uint32_t xbeg = 0, ebase = xcd * Q.seg_cap;
    uint32_t wnext = 0, wend = 0;
    bool exhausted = false;

    TraceCounters tc{0, 0, 0};
    bool overflow = false;
    uint32_t rays = 0;
    bool active = false;
    uint32_t e = 0;
    Trav T;
    trav_start(T, mk3(0, 0, 0), mk3(1, 0, 0), 0.0f);
    uint32_t steps = 0;   // COUNT: iterations the current ray has taken
    __shared__ uint32_t lds_pend_all[ANY ? kBlock : 1];
    uint32_t* const lds_pend = &lds_pend_all[ANY ? (threadIdx.x & ~63u) : 0u];   // the wave's 64 slots
    uint32_t npend = 0;   // wave-uniform

    while (true) {
        // refill idle lanes from the wave's chunk
        const unsigned long long idle = __ballot(!active);
        const bool refill = __popcll(idle) >= Q.refill_min || idle == ~0ull;
        if (wnext >= wend && !exhausted && refill) {
            uint32_t base = 0;
            if (lane_id() == 0) base = atomicAdd(chunk_ctr, (uint32_t)Q.chunk);
            base = xbeg + __builtin_amdgcn_readfirstlane(base);
            if (base >= xend) {
                exhausted = true;
            } else {
                wnext = base;
                wend = min(base + (uint32_t)Q.chunk, xend);
            }
        }
        if (idle != 0ull && wnext < wend && refill) {
            if (!active) {
                uint32_t g = wnext + mbcnt64(idle);
                if (g < wend) {
                    e = ebase + (ANY ? g : seg_pos(g, xl, Q.seg_cap));
                    float4 o4 = qin[(size_t)qstride * e];
                    float4 d4 = qin[(size_t)qstride * e + 1];
                    trav_start(T, ld3(o4), ld3(d4), ANY ? d4.w : INFINITY);
                    active = true;
                    rays++;
                    if (COUNT) steps = 0;
                }
            }
            wnext += (uint32_t)__popcll(idle);
        }
        if (__ballot(active) == 0ull) {
            if (ANY) connect_flush(Q, qin, lds_pend, npend);
            break;
        }
        bool acc = false;
        if (active) {
            if (COUNT) ++steps;
            if (trav_step<COUNT>(S, T, ANY, stack, tc, overflow, T.best)) {
                active = false;
                if (COUNT && Q.diag) {   // steps-per-ray histogram (log2 bins) of the counting frame
                    atomicAdd(&Q.W.counts[kWfDiagSteps + (ANY ? 32 : 0) + (31 - __builtin_clz(steps))], 1u);
                    atomicMax(&Q.W.counts[kWfDiagSteps + 64 + (ANY ? 1 : 0)], steps);
                }
                if (ANY) acc = !T.hit_any;
                else Q.W.hits[e] = make_float4(T.best, __uint_as_float(T.best_id), T.bu / T.bdet, T.bv / T.bdet);
            }
        }
        if (ANY) {   // unoccluded shadow rays: their entries wait in the wave's LDS list (connect_flush)
            const unsigned long long m = __ballot(acc);
            if (m != 0ull) {
                const uint32_t k = (uint32_t)__popcll(m);
                if (npend + k > 64u) connect_flush(Q, qin, lds_pend, npend);
                if (acc) lds_pend[npend + mbcnt64(m)] = e;
                npend += k;
            }
        }
    }
    ts_end(Q, ts, &ts_done);
    flush_counters(P, ANY ? 0 : rays, ANY ? rays : 0, 0, tc, COUNT, overflow, true);
}

// ---- finish: the remaining paths to completion, step-interleaved ---------------------------------------
// Below Q.tail live paths, one persistent launch runs every remaining path to completion.  Every
// lane advances by ONE traversal step per iteration (trav_step, closest-hit or shadow any-hit), as
// in wf_trace.  A lane whose closest-hit query ended waits in kReady; the wave shades all waiting
// lanes together once at least Q.shade_min of them wait (or no lane is traversing), then each
// continues with its shadow ray, its next ray, or the next path of the queue.  A wave therefore
// costs the sum of its own lanes' steps, not the sum over segments of its slowest lane's query:
// the glass paths left at the tail (up to ~23 segments) do not wait for their wave's worst ray
// every segment.  Four waves per SIMD: the shading code's register peak (119 VGPRs, no scratch);
// five were measured no faster.
template <bool COUNT, bool FULL, bool TEAM>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4, 4)))
wf_finish_step(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q, int cur, int ts) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    if (cur < 0) cur = (int)__builtin_amdgcn_readfirstlane(Q.W.counts[cslot(kCntFinishQ)]);   // dev_ctl
    __shared__ int lds_stack[kStackSize * kBlock];
    __shared__ HaltonDim lds_halton[kHaltonLds];
    __shared__ MatRec lds_mat[kMatLds];
    __shared__ float4 lds_inst[3 * kInstLds];
    __shared__ Light lds_light[kLightLds];
    __shared__ float lds_sray[6][kBlock];   // each lane's shadow ray (origin, direction)
    int* stack = &lds_stack[threadIdx.x];
    __shared__ uint32_t ts_done;
    if (threadIdx.x == 0) ts_done = 0u;
    ts_start(Q, ts);
    const ShadeTabs halton = load_tabs(S, lds_halton, lds_mat, lds_inst, lds_light, P.U.lightCount);   // ends with a block barrier
    const Uniforms& U = P.U;
    const QueueShards qs = load_queue(Q.W.counts, cur, Q.seg_cap);   // front parts first: the likely-long paths
    const uint32_t n = queue_len(qs);
    if (Q.dev_ctl) stat_add(Q, kStatFinish, 1u);
    if (Q.dev_ctl && n > 0) stat_add(Q, kStatRounds, 1u);
    const float4* qin = Q.W.q[cur];
    const uint32_t kChunk = (uint32_t)Q.fchunk;   // paths per grab
    constexpr int kIdle = 0, kClosest = 1, kShadow = 2, kReady = 3;
    TraceCounters tc{0, 0, 0};
    bool overflow = false;
    uint32_t n_closest = 0, n_shadow = 0;
    f2 zero2;
    zero2.x = 0.0f;
    zero2.y = 0.0f;
    uint32_t wnext = 0, wend = 0;
    bool exhausted = false;
    int mode = kIdle;
    // path
    uint32_t pid = 0;
    uint4 meta = make_uint4(0, 0, 0, 0);
    PathRegs p;
    p.color = p.accum = mk3(0, 0, 0);
    p.bounce = p.tpass = p.step = 0;
    f3 rayO = mk3(0, 0, 0), rayD = mk3(0, 0, 0), contrib = mk3(0, 0, 0);
    bool next = false;
    Trav T;
    trav_start(T, mk3(0, 0, 0), mk3(1, 0, 0), 0.0f);
    // diagnostics (Q.diag, RT_WF_LOG): segments of the longest path, loop iterations and wall
    // time (s_memrealtime, 100 MHz) of the slowest wave, time in shading passes
    uint32_t segs = 0, max_segs = 0, iters = 0;
    const uint64_t t_start = Q.diag ? __builtin_amdgcn_s_memrealtime() : 0;
    // per wave, in LDS (no registers outside RT_WF_LOG runs): iterations and ticks at its queue's
    // exhaustion, active lanes summed over the iterations after it
    __shared__ uint32_t diag_x[kBlock / 64][3];
#define RT_DX diag_x[__builtin_amdgcn_readfirstlane(threadIdx.x) / 64u]
    if (Q.diag && lane_id() == 0) RT_DX[0] = RT_DX[1] = RT_DX[2] = 0xffffffffu;
    uint64_t t_shade = 0;
    uint32_t n_pass = 0, n_shaded = 0;
    auto end_path = [&]() {
        Q.W.p_accum[pid] = make_float4(p.accum.x, p.accum.y, p.accum.z, 0.0f);
        if (Q.diag > 1) {   // RT_WF_LOG=2: segments by entry class: bounce at entry, refracting (tpass > 0) or not
            const uint32_t b0 = min(meta.z & 0xffu, 8u), tp0 = (meta.z >> 8) & 0xffu;
            atomicAdd(&Q.W.counts[kWfDiagLen + ((tp0 ? 9u : 0u) + b0) * 32u + min(segs, 31u)], 1u);
        }
        mode = kIdle;
        max_segs = max(max_segs, segs);
        segs = 0;
    };

    // shade this lane's closest hit (:324-774); rayO / rayD become the next ray
    auto shade_hit = [&](StepResult& r) {
        Hit h;
        h.t = T.best;
        h.id = T.best_id;
        h.u = T.bu / T.bdet;
        h.v = T.bv / T.bdet;
        const int sample = (int)meta.y;
        shade_step<FULL, false>(S, U, halton, (int)meta.w, sample, rayO, rayD, h, p, sample == 0 && p.step == 0, zero2,
                                false, zero2, r);
        write_pixel_outputs(P, meta.x, r, h, FULL);
        next = r.next;
    };

    while (true) {
        // ---- refill idle lanes with the next remaining paths (chunks of Q.fchunk from the XCD's counter)
        const unsigned long long idle = __ballot(mode == kIdle);
        const bool refill = __popcll(idle) >= Q.refill_min || idle == ~0ull;
        if (wnext >= wend && !exhausted && refill) {
            uint32_t base = 0;
            // this XCD's next chunk (the grid has >= 8 blocks: launch_finish)
            if (lane_id() == 0) base = atomicAdd(Q.W.counts + cslot(kCntChunkFinish + (int)(blockIdx.x & 7u)), 1u);
            base = ((__builtin_amdgcn_readfirstlane(base) << 3) | (blockIdx.x & 7u)) * kChunk;
            if (base >= n) {
                exhausted = true;
                if (Q.diag && lane_id() == 0) {
                    RT_DX[0] = iters;
                    RT_DX[1] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_start);
                    RT_DX[2] = 0;
                }
            } else {
                wnext = base;
                wend = min(base + kChunk, n);
            }
        }
        if (idle != 0ull && wnext < wend && refill) {
            if (mode == kIdle) {
                const uint32_t g = wnext + mbcnt64(idle);
                if (g < wend) {
                    const uint32_t e = dense_entry(qs, g, Q.seg_cap);
                    const float4* src = qin + 2 * (size_t)e;
                    const float4 o = ld_stream(&src[0]);
                    const float4 d = ld_stream(&src[1]);
                    pid = __float_as_uint(o.w);
                    const uint32_t state = __float_as_uint(d.w);
                    const float4 c = state == 0u ? make_float4(1.0f, 1.0f, 1.0f, 0.0f)
                                     : ld_stream(&Q.W.qc[cur][e]);
                    if ((state & 0xffu) != 0u) {   // past bounce 0: the Halton index from qc.w (wf_shade)
                        meta = make_uint4(0u, 1u, state, __float_as_uint(c.w));
                    } else {
                        const uint3 pm = path_meta(P, Q, pid);
                        meta = make_uint4(pm.x, pm.y, state, pm.z);
                    }
                    const float4 a = Q.W.p_accum[pid];
                    p.color = mk3(c.x, c.y, c.z);
                    p.accum = mk3(a.x, a.y, a.z);
                    p.bounce = (int)(meta.z & 0xffu);
                    p.tpass = (int)((meta.z >> 8) & 0xffu);
                    p.step = (int)(meta.z >> 16);
                    rayO = ld3(o);
                    rayD = ld3(d);
                    trav_start(T, rayO, rayD, INFINITY);
                    mode = kClosest;
                    n_closest++;
                    segs++;
                }
            }
            wnext += (uint32_t)__popcll(idle);
        }
        const unsigned long long active = __ballot(mode != kIdle);
        if (active == 0ull) break;   // idle everywhere => refill found nothing
        if (TEAM && exhausted && __popcll(active) * Q.team <= 64) break;   // the rest: team drain below
        ++iters;
        if (Q.diag && exhausted && lane_id() == 0) RT_DX[2] += (uint32_t)__popcll(active);

        // ---- one traversal step (closest hit or shadow any-hit)
        if (mode == kClosest || mode == kShadow) {
            const bool any = mode == kShadow;
            if (trav_step<COUNT>(S, T, any, stack, tc, overflow, T.best)) {
                if (any) {   // shadow ray done: unoccluded -> add its contribution (:741-743)
                    if (!T.hit_any) p.accum = p.accum + contrib;
                    if (next) {
                        trav_start(T, rayO, rayD, INFINITY);
                        mode = kClosest;
                        n_closest++;
                        segs++;
                    } else {
                        end_path();
                    }
                } else if (T.best_id == 0xffffffffu) {   // miss -> path ends (:321-322)
                    end_path();
                } else {
                    mode = kReady;
                }
            }
        }

        // ---- shade the waiting lanes together (:324-774)
        const unsigned long long ready = __ballot(mode == kReady);
        int shade_thr = exhausted ? Q.shade_min_x : Q.shade_min;
        if (shade_thr < 0) shade_thr = max(1, -shade_thr * __popcll(__ballot(mode != kIdle)) / 100);   // % of the busy lanes
        if (ready != 0ull && (__popcll(ready) >= shade_thr || __ballot(mode == kClosest || mode == kShadow) == 0ull)) {
            const uint64_t ts0 = Q.diag ? __builtin_amdgcn_s_memrealtime() : 0;
            if (Q.diag) {
                ++n_pass;
                n_shaded += (uint32_t)__popcll(ready);
            }
            if (mode == kReady) {
                StepResult r;
                shade_hit(r);
                if (r.shadow) {
                    contrib = r.contrib;
                    trav_start(T, r.so, r.sd, r.stmax);
                    lds_sray[0][threadIdx.x] = r.so.x;
                    lds_sray[1][threadIdx.x] = r.so.y;
                    lds_sray[2][threadIdx.x] = r.so.z;
                    lds_sray[3][threadIdx.x] = r.sd.x;
                    lds_sray[4][threadIdx.x] = r.sd.y;
                    lds_sray[5][threadIdx.x] = r.sd.z;
                    mode = kShadow;
                    n_shadow++;
                } else if (r.next) {
                    trav_start(T, rayO, rayD, INFINITY);
                    mode = kClosest;
                    n_closest++;
                    segs++;
                } else {
                    end_path();
                }
            }
            // Every lane's ray setup is rebuilt from its ray (a pure function of it, so bit for bit
            // the one trav_start made): the ~19 registers of the traversing lanes' setups are then
            // dead while the shading code runs, which sets the kernel's register peak.
            if (mode == kShadow) {
                T.R = ray_setup(mk3(lds_sray[0][threadIdx.x], lds_sray[1][threadIdx.x], lds_sray[2][threadIdx.x]),
                                mk3(lds_sray[3][threadIdx.x], lds_sray[4][threadIdx.x], lds_sray[5][threadIdx.x]));
            } else {
                T.R = ray_setup(rayO, rayD);
            }
            if (Q.diag) t_shade += __builtin_amdgcn_s_memrealtime() - ts0;
        }

    }

    // ---- team drain (Q.team lanes per query).  The queue has run out and this wave holds at most
    // 64 / team paths: each moves to a team leader (lane team * r) and the team's lanes traverse its
    // query together, splitting the node groups and stack entries among themselves (XOR-paired
    // hand-offs every iteration) and sharing the closest hit found so far as their cull bound; a
    // closest-hit query ends with the lexicographic minimum of the members' (t, id), the serial
    // traversal's result, so the same bits; an any-hit query ends at any member's occluder.  The
    // leader shades, then the team starts the path's next query.
    if (TEAM && __ballot(mode != kIdle) != 0ull) {
        const int TM = Q.team;
        if (mode == kReady) {   // waiting lanes first: every busy lane then holds a query
            StepResult r;
            shade_hit(r);
            if (r.shadow) {
                contrib = r.contrib;
                trav_start(T, r.so, r.sd, r.stmax);
                lds_sray[0][threadIdx.x] = r.so.x;
                lds_sray[1][threadIdx.x] = r.so.y;
                lds_sray[2][threadIdx.x] = r.so.z;
                lds_sray[3][threadIdx.x] = r.sd.x;
                lds_sray[4][threadIdx.x] = r.sd.y;
                lds_sray[5][threadIdx.x] = r.sd.z;
                mode = kShadow;
                n_shadow++;
            } else if (r.next) {
                mode = kClosest;
                n_closest++;
                segs++;
            } else {
                end_path();
            }
        }
        const unsigned long long busy = __ballot(mode != kIdle);
        const int lane = (int)lane_id(), j = lane & (TM - 1), lead = lane - j, rk = lane / TM;
        const int nb = __popcll(busy);
        int src = lane;   // team leader rk takes the rk-th busy lane's path
        {
            unsigned long long b = busy;
            for (int k = 0; b; ++k) {
                const int l = __builtin_ctzll(b);
                b &= b - 1ull;
                if (j == 0 && rk == k) src = l;
            }
        }
        const bool leader = j == 0 && rk < nb;
        auto mvu = [&](uint32_t v) { return (uint32_t)__shfl((int)v, src); };
        auto mvf = [&](float v) { return __shfl(v, src); };
        auto mv3 = [&](f3 v) { return mk3(mvf(v.x), mvf(v.y), mvf(v.z)); };
        const uint32_t sbase = threadIdx.x & ~63u;
        // the leaders' shadow rays stay in LDS (each leader's slot; the members read it when the
        // team starts the query): six registers fewer across the shading code
        {
            float sr[6];
            #pragma unroll
            for (int c = 0; c < 6; ++c) sr[c] = lds_sray[c][sbase + src];
            #pragma unroll
            for (int c = 0; c < 6; ++c) lds_sray[c][threadIdx.x] = sr[c];
        }
        // the leaders' shadow tmax and contribution stay in LDS as well (lds_tx)
        __shared__ float lds_tx[4][kBlock];
        {
            const float t_src = mvf(T.best);
            const f3 c_src = mv3(contrib);
            lds_tx[0][threadIdx.x] = t_src;
            lds_tx[1][threadIdx.x] = c_src.x;
            lds_tx[2][threadIdx.x] = c_src.y;
            lds_tx[3][threadIdx.x] = c_src.z;
        }
        pid = mvu(pid);
        meta = make_uint4(mvu(meta.x), mvu(meta.y), mvu(meta.z), mvu(meta.w));
        p.color = mv3(p.color);
        p.accum = mv3(p.accum);
        p.bounce = (int)mvu((uint32_t)p.bounce);
        p.step = (int)mvu((uint32_t)p.step);
        p.tpass = (int)mvu((uint32_t)p.tpass);
        rayO = mv3(rayO);
        rayD = mv3(rayD);
        next = mvu(next ? 1u : 0u) != 0u;
        segs = mvu(segs);
        // every lane takes part in the shuffle: a bpermute inside the leaders' branch would read the
        // (inactive) non-leader source lanes as zero
        const int src_mode = (int)mvu((uint32_t)mode);
        mode = leader ? src_mode : kIdle;
        bool fresh = leader;   // the team starts the leader's query
        float cull = INFINITY;
        while (true) {
            const int lmode = __shfl(mode, lead);
            if (__ballot(lmode != kIdle) == 0ull) break;
            const bool team_on = lmode == kClosest || lmode == kShadow, any = lmode == kShadow;
            if (__shfl((int)fresh, lead) != 0 && team_on) {   // start the team's query on every member
                f3 o, d;
                float tmax;
                if (any) {
                    const uint32_t ls = sbase + (uint32_t)lead;
                    o = mk3(lds_sray[0][ls], lds_sray[1][ls], lds_sray[2][ls]);
                    d = mk3(lds_sray[3][ls], lds_sray[4][ls], lds_sray[5][ls]);
                    tmax = lds_tx[0][ls];
                } else {
                    o = mk3(__shfl(rayO.x, lead), __shfl(rayO.y, lead), __shfl(rayO.z, lead));
                    d = mk3(__shfl(rayD.x, lead), __shfl(rayD.y, lead), __shfl(rayD.z, lead));
                    tmax = INFINITY;
                }
                trav_start(T, o, d, tmax);
                if (j != 0) T.g_hits = 0;   // members start without work; the leader hands it out below
                cull = tmax;
            }
            fresh = false;
            // one traversal step of every member with work
            if (team_on && !(T.t_mask == 0u && T.g_hits == 0u && T.sp == 0))
                (void)trav_step<COUNT>(S, T, any, stack, tc, overflow, cull);
            // occluder anywhere in the team; the team's closest hit so far (the cull bound)
            int hit = (any && T.hit_any) ? 1 : 0;
            float bt = T.best;
            for (int k = 1; k < TM; k <<= 1) {
                hit |= __shfl_xor(hit, k);
                bt = fminf(bt, __shfl_xor(bt, k));
            }
            if (team_on && !any) cull = bt;
            if (hit) {
                T.t_mask = 0u;
                T.g_hits = 0u;
                T.sp = 0;
            }
            // hand-offs: in round k lane l pairs with lane l ^ k; an idle member takes the later
            // half (in visiting order) of its partner's node group, or its partner's top stack entry
            for (int k = 1; k < TM; ++k) {
                const bool idle_m = team_on && T.t_mask == 0u && T.g_hits == 0u && T.sp == 0;
                const bool give = team_on && (__popc(T.g_hits) >= 2 || T.sp > 0);
                const bool p_idle = __shfl_xor((int)idle_m, k) != 0, p_give = __shfl_xor((int)give, k) != 0;
                uint32_t pay = 0u;
                if (give && p_idle) {
                    if (__popc(T.g_hits) >= 2) {
                        uint32_t keep = 0u, rest = T.g_hits;
                        for (int c = __popc(T.g_hits) - __popc(T.g_hits) / 2; c > 0; --c) {
                            const int b = T.g_flip ? highest_bit(rest) : lowest_bit(rest);
                            keep |= 1u << b;
                            rest &= ~(1u << b);
                        }
                        pay = pack_group(T.g_base, T.g_flip, rest);
                        T.g_hits = keep;
                    } else {
                        --T.sp;
                        pay = (uint32_t)stack[T.sp * kBlock];
                    }
                }
                const uint32_t got = (uint32_t)__shfl_xor((int)pay, k);
                if (idle_m && p_give) {
                    T.g_base = got >> 9;
                    T.g_flip = (got >> 8) & 1u;
                    T.g_hits = got & 0xffu;
                }
            }
            // the team's query has ended once no member holds work
            int work = (team_on && !(T.t_mask == 0u && T.g_hits == 0u && T.sp == 0)) ? 1 : 0;
            for (int k = 1; k < TM; k <<= 1) work |= __shfl_xor(work, k);
            if (team_on && !work) {
                if (!any) {   // lexicographic minimum of the members' (t, id), with its (V, W, det)
                    float t = T.best, bu = T.bu, bv = T.bv, bd = T.bdet;
                    uint32_t id = T.best_id;
                    for (int k = 1; k < TM; k <<= 1) {
                        const float t2 = __shfl_xor(t, k), u2 = __shfl_xor(bu, k), v2 = __shfl_xor(bv, k),
                                    d2 = __shfl_xor(bd, k);
                        const uint32_t id2 = (uint32_t)__shfl_xor((int)id, k);
                        if (t2 < t || (t2 == t && id2 < id)) {
                            t = t2;
                            id = id2;
                            bu = u2;
                            bv = v2;
                            bd = d2;
                        }
                    }
                    T.best = t;
                    T.best_id = id;
                    T.bu = bu;
                    T.bv = bv;
                    T.bdet = bd;
                }
                if (j == 0) {   // the leader: the path's next step (as in the loop above)
                    if (any) {
                        if (!hit)
                            p.accum = p.accum + mk3(lds_tx[1][threadIdx.x], lds_tx[2][threadIdx.x], lds_tx[3][threadIdx.x]);
                        if (next) {
                            mode = kClosest;
                            n_closest++;
                            segs++;
                            fresh = true;
                        } else {
                            end_path();
                        }
                    } else if (T.best_id == 0xffffffffu) {
                        end_path();
                    } else {
                        mode = kReady;
                    }
                }
            }
            if (mode == kReady) {   // leaders: shade at once (the drain is latency-bound)
                StepResult r;
                shade_hit(r);
                if (r.shadow) {
                    lds_tx[1][threadIdx.x] = r.contrib.x;
                    lds_tx[2][threadIdx.x] = r.contrib.y;
                    lds_tx[3][threadIdx.x] = r.contrib.z;
                    lds_sray[0][threadIdx.x] = r.so.x;
                    lds_sray[1][threadIdx.x] = r.so.y;
                    lds_sray[2][threadIdx.x] = r.so.z;
                    lds_sray[3][threadIdx.x] = r.sd.x;
                    lds_sray[4][threadIdx.x] = r.sd.y;
                    lds_sray[5][threadIdx.x] = r.sd.z;
                    lds_tx[0][threadIdx.x] = r.stmax;
                    mode = kShadow;
                    n_shadow++;
                    fresh = true;
                } else if (r.next) {
                    mode = kClosest;
                    n_closest++;
                    segs++;
                    fresh = true;
                } else {
                    end_path();
                }
            }
        }
    }

    if (Q.diag) {
        const uint32_t dt = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_start);
        if (lane_id() == 0) {
            const uint32_t* dx = RT_DX;
            const bool x = dx[0] != 0xffffffffu;   // else its last grab was in range: it never saw the end
            const uint32_t it_x = x ? dx[0] : iters, t_x = x ? dx[1] : dt;
            atomicAdd(&Q.W.counts[kWfStat + kStatDiagItPre], it_x);
            atomicAdd(&Q.W.counts[kWfStat + kStatDiagItPost], iters - it_x);
            atomicAdd(&Q.W.counts[kWfStat + kStatDiagTPre], t_x);
            atomicAdd(&Q.W.counts[kWfStat + kStatDiagTPost], dt - t_x);
            atomicAdd(&Q.W.counts[kWfStat + kStatDiagLanesPost], x ? dx[2] : 0u);
            atomicAdd(&Q.W.counts[kWfDiagExh + min(t_x / 5000u, 63u)], 1u);
            atomicAdd(&Q.W.counts[kWfStat + kStatDiagShadeT], (uint32_t)t_shade);
            atomicAdd(&Q.W.counts[kWfStat + kStatDiagTotalT], dt);
            atomicAdd(&Q.W.counts[kWfStat + kStatDiagPasses], n_pass);
            atomicAdd(&Q.W.counts[kWfStat + kStatDiagShaded], n_shaded);
        }
        for (int off = 32; off > 0; off >>= 1) max_segs = max(max_segs, (uint32_t)__shfl_xor((int)max_segs, off, 64));
        if (lane_id() == 0) {
            atomicMax(&Q.W.counts[cslot(kCntDiagSegs)], max_segs);
            atomicMax(&Q.W.counts[cslot(kCntDiagIters)], iters);
            atomicMax(&Q.W.counts[cslot(kCntDiagTime)], dt);
            atomicAdd(&Q.W.counts[kWfDiagHist + min(dt / 5000u, 63u)], 1u);
        }
    }
#undef RT_DX
    ts_end(Q, ts, &ts_done);
    flush_counters(P, n_closest, n_shadow, 0, tc, COUNT, overflow);
}

// ---- motion-adaptive extra samples (:779-789) -----------------------------------------------------------
__global__ void __launch_bounds__(kBlock) wf_extra(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q, int qidx) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    __shared__ HaltonDim lds_halton[kHaltonLds];
    const ShadeTabs halton = load_tabs(S, lds_halton, nullptr);   // no shading: Halton only
    const Uniforms& U = P.U;
    const int maxExtra = (U.enableMotionAdaptiveSampling != 0) ? max(U.motionSamplingMaxExtraSamples, 0) : 0;
    const int stride = Q.spp + maxExtra;
    const int shard = blockIdx.x & (kShards - 1);
    float4* qout = Q.W.q[qidx] + 2 * (size_t)shard * Q.seg_cap;
    __shared__ BlockAlloc ba;
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    int px = 0, py = 0, e = 0;
    uint32_t pix = 0;
    if (i < Q.own_pixels) {
        own_pixel(Q, i, px, py);
        if (px < U.width && py < U.height) {
            pix = (uint32_t)py * (uint32_t)U.width + (uint32_t)px;
            float2 mv2 = P.motion[pix], pm2 = P.motion_prev[pix];
            f2 mv, pm;
            mv.x = mv2.x;
            mv.y = mv2.y;
            pm.x = pm2.x;
            pm.y = pm2.y;
            e = extra_samples(U, maxExtra, mv, pm);
        }
    }
    const uint32_t start = block_alloc_n((uint32_t)e, &Q.W.counts[cslot(kCntExtra)], ba);
    const uint32_t slot0 =
        block_alloc_n(U.maxBounces > 0 ? (uint32_t)e : 0u, &Q.W.counts[cslot(qidx * kShards + shard)], ba);
    if (e > 0) {
        const uint32_t offset = P.random[pix];
        for (int j = 0; j < e; ++j) {
            int s = Q.spp + j;
            uint32_t pid = Q.base_paths + start + (uint32_t)j;
            int hidx = (int)(offset + (unsigned)((int)U.frameIndex * stride + s));
            init_path(Q, pid, pix, s, (uint32_t)hidx);
            f3 o, d;
            primary_ray(U, halton, px, py, hidx, o, d);
            if (U.maxBounces > 0) {
                const uint32_t slot = slot0 + (uint32_t)j;
                qout[2 * (size_t)slot] = make_float4(o.x, o.y, o.z, __uint_as_float(pid));
                qout[2 * (size_t)slot + 1] = make_float4(d.x, d.y, d.z, 0.0f);
            }
        }
    }
    if (i < Q.own_pixels) Q.W.px_extra[i] = make_uint2(start, (uint32_t)e);
    TraceCounters tc{0, 0, 0};
    flush_counters(P, 0, 0, (uint32_t)e, tc, false, false);
}

// ---- depth + motion (:342-389) ----------------------------------------------------------------------
// After the base pass: every own pixel whose sample 0 had a bounce-0 hit gets the depth and motion
// vector of the last such hit (the value the per-pixel kernel leaves, since each of those hits
// overwrites it), evaluated here once instead of inside every shading launch, where it would
// hold ~25 VGPRs of transforms and cameras.
__global__ void __launch_bounds__(kBlock) wf_motion(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q) {
    const FrameParams& P = *Pp;
    const Uniforms& U = P.U;
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= Q.own_pixels) return;
    int px, py;
    own_pixel(Q, i, px, py);
    if (px >= U.width || py >= U.height) return;
    const size_t pix = (size_t)py * U.width + px;
    const uint4 ph = P.prim_hit[pix];
    if (ph.x == 0xffffffffu) return;   // no bounce-0 hit: generate's defaults stay
    float depth;
    f2 mv;
    primary_outputs(S, U, ph.x, __uint_as_float(ph.y), __uint_as_float(ph.z), depth, mv);
    P.depth[pix] = depth;
    P.motion[pix] = make_float2(mv.x, mv.y);
}

// ---- resolve (:777, :792-819) -------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) wf_resolve(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q, int with_extra) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    const Uniforms& U = P.U;
    uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= Q.own_pixels) return;
    int px, py;
    own_pixel(Q, i, px, py);
    if (px >= U.width || py >= U.height) return;
    size_t pix = (size_t)py * U.width + px;
    f3 total = mk3(0.0f, 0.0f, 0.0f);
    for (int s = 0; s < Q.spp; ++s) {
        float4 a = Q.W.p_accum[(size_t)i * Q.spp + s];
        total = total + mk3(a.x, a.y, a.z);
    }
    int nsamp = Q.spp;
    if (with_extra) {
        uint2 ex = Q.W.px_extra[i];
        for (uint32_t j = 0; j < ex.y; ++j) {
            float4 a = Q.W.p_accum[Q.base_paths + ex.x + j];
            total = total + mk3(a.x, a.y, a.z);
        }
        nsamp += (int)ex.y;
    }
    float2 mv2 = P.motion[pix], pm2 = P.motion_prev[pix];
    f2 mv, pm;
    mv.x = mv2.x;
    mv.y = mv2.y;
    pm.x = pm2.x;
    pm.y = pm2.y;
    f3 c = resolve_pixel(U, total, nsamp, mv, pm, P.accum_in, pix);
    P.accum_out[pix] = make_float4(c.x, c.y, c.z, 1.0f);
}

// Segment k only receives entries from blocks b == k (mod 8): at most n/8 + 256 per pass over n
// inputs, and (own pixels/8 + 256) * maxExtra from the extra-sample pass.
size_t wavefront_queue_entries(size_t paths, int max_extra) {
    return (size_t)kShards * (paths / kShards + 4096 + 256 * (size_t)max_extra);
}

static unsigned grid_for(uint32_t n, unsigned cap) {
    unsigned g = (unsigned)(((uint64_t)n + kBlock - 1) / kBlock);
    if (g > cap) g = cap;
    g = (g + kShards - 1) / kShards * kShards;  // multiple of 8: segment bound (see header)
    return g == 0 ? kShards : g;
}

#define WF_CHECK(expr)                                                                  \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) {                                                         \
            static thread_local char msg_[192];                                         \
            snprintf(msg_, sizeof msg_, "%.120s: %s", #expr, hipGetErrorString(e_));  \
            *err = msg_;                                                                \
            return false;                                                               \
        }                                                                               \
    } while (0)

// resident blocks (CUs x blocks per CU) of a persistent kernel
template <typename K>
static unsigned resident_grid(K kernel, int fallback_per_cu) {
    int dev = 0, cus = 256, per = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, kBlock, 0) != hipSuccess || per < 1)
        per = fallback_per_cu;
    return (unsigned)(cus * per);
}

// resident blocks of the persistent traversal kernel, queried once
// the bulk traversal launches: Q.trace_frac percent of the resident grid, a multiple of 8 (XCDs)
static unsigned trace_grid_cap(const WfParams& Q) {
    static const unsigned cap = resident_grid(wf_trace<false, false>, 4);
    return std::max(8u, cap * (unsigned)std::max(Q.trace_frac, 1) / 100u / 8u * 8u);
}

// the finish launch: Q.finish_frac percent of the resident grid (frames in flight: the rest of the
// machine stays free for the other frames' kernels)
template <bool COUNT, bool FULL, bool TEAM>
static unsigned finish_full_cap() {   // resident blocks of the finish kernel instance, queried once
    static const unsigned c = resident_grid(wf_finish_step<COUNT, FULL, TEAM>, 2);
    return c;
}
template <bool COUNT, bool FULL>
static void launch_finish(const DevScene& S, const WfParams& Q, int cur, uint32_t n, hipStream_t stream, int ts) {
    // at least one block per XCD: each takes the chunks of its XCD's counter (wf_finish_step).
    // Q.team: the kernel with the team drain (a separate instance: its code would raise the plain
    // kernel's register pressure), sized by its own occupancy (its LDS and registers differ)
    if (Q.team) {
        const unsigned cap = std::max(8u, finish_full_cap<COUNT, FULL, true>() * (unsigned)Q.finish_frac / 100u);
        hipLaunchKernelGGL((wf_finish_step<COUNT, FULL, true>), dim3(std::max(8u, grid_for(n, cap))), dim3(kBlock), 0,
                           stream, S, Q.Pd, Q, cur, ts);
    } else {
        const unsigned cap = std::max(8u, finish_full_cap<COUNT, FULL, false>() * (unsigned)Q.finish_frac / 100u);
        hipLaunchKernelGGL((wf_finish_step<COUNT, FULL, false>), dim3(std::max(8u, grid_for(n, cap))), dim3(kBlock), 0,
                           stream, S, Q.Pd, Q, cur, ts);
    }
}

static void launch_finish_any(const DevScene& S, const WfParams& Q, bool count, bool full, int cur, uint32_t n,
                              hipStream_t stream, int ts = -1) {
    if (count) full ? launch_finish<true, true>(S, Q, cur, n, stream, ts) : launch_finish<true, false>(S, Q, cur, n, stream, ts);
    else full ? launch_finish<false, true>(S, Q, cur, n, stream, ts) : launch_finish<false, false>(S, Q, cur, n, stream, ts);
}

static uint32_t queue_total(const uint32_t* h, int q) {   // q = 0, 1: a ray queue (both ends); 2: the shadow queue
    uint32_t s = 0;
    for (int k = 0; k < kShards; ++k) s += h[cslot(q * kShards + k)] + (q < 2 ? h[cslot(kCntBack + q * kShards + k)] : 0u);
    return s;
}

// Host-driven rounds (RT_WF_HOST=1 / RT_WF_LOG=1, and the bulk-only test configuration tail <= 1):
// every round's queue size is read back before the next launch.
static bool iterate(const DevScene& S, const FrameParams& P, WfParams& Q, int& cur, uint32_t n, bool count, bool full,
                    hipStream_t stream, WfFrameStats* fs, const char** err) {
    float* stage_ms = fs->stage_ms;
    const int max_it = P.U.maxBounces * (P.U.maxBounces + 1) + 2;
    WavefrontBuffers& W = Q.W;
    for (int it = 0; it < max_it && n > 0; ++it) {
        if (n < Q.tail) {   // the rest of the pass in one persistent finish launch
            WF_CHECK(hipEventRecord(W.ev[0], stream));
            WF_CHECK(hipMemsetAsync(W.counts + cslot(kCntChunkFinish), 0, cslot(kShards) * sizeof(uint32_t), stream));
            if (Q.diag) {
                WF_CHECK(hipMemsetAsync(W.counts + kWfDiagHist, 0, 64 * sizeof(uint32_t), stream));
                WF_CHECK(hipMemsetAsync(W.counts + kWfDiagExh, 0, 64 * sizeof(uint32_t), stream));
                WF_CHECK(hipMemsetAsync(W.counts + kWfStat + kStatDiagShadeT, 0, (kWfStatWords - kStatDiagShadeT) * sizeof(uint32_t),
                                        stream));
            }
            launch_finish_any(S, Q, count, full, cur, n, stream);
            WF_CHECK(hipGetLastError());
            WF_CHECK(hipEventRecord(W.ev[1], stream));
            WF_CHECK(hipMemcpyAsync(W.h_counts, W.counts, kWfCountWords * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                    stream));
            WF_CHECK(hipStreamSynchronize(stream));
            float a = 0;
            WF_CHECK(hipEventElapsedTime(&a, W.ev[0], W.ev[1]));
            stage_ms[5] += a;
            ++fs->finish_launches;
            ++fs->iterations;
            if (Q.diag) {
                fprintf(stderr, "[wf] it %d finish paths %u  %.3f ms; longest path %u segments, "
                        "slowest wave %u iterations in %.3f ms\n", it, n, a, W.h_counts[cslot(kCntDiagSegs)],
                        W.h_counts[cslot(kCntDiagIters)], W.h_counts[cslot(kCntDiagTime)] * 1e-5);
                const double st = W.h_counts[kWfStat + kStatDiagShadeT], tt = W.h_counts[kWfStat + kStatDiagTotalT];
                const double np = W.h_counts[kWfStat + kStatDiagPasses], ns = W.h_counts[kWfStat + kStatDiagShaded];
                fprintf(stderr, "[wf] finish: %.1f %% of wave time in shading passes, %.0f passes, %.1f lanes per pass\n",
                        tt > 0 ? 100.0 * st / tt : 0.0, np, np > 0 ? ns / np : 0.0);
                for (int cl = 0; cl < 18; ++cl) {
                    uint32_t tot = 0;
                    double sum = 0;
                    for (int b = 0; b < 32; ++b) {
                        tot += W.h_counts[kWfDiagLen + cl * 32 + b];
                        sum += (double)b * W.h_counts[kWfDiagLen + cl * 32 + b];
                    }
                    if (!tot) continue;
                    fprintf(stderr, "[wf] finish paths entering at bounce %d%s: %u, segments mean %.2f:", cl % 9,
                            cl >= 9 ? " refracting" : "", tot, sum / tot);
                    for (int b = 0; b < 32; ++b)
                        if (W.h_counts[kWfDiagLen + cl * 32 + b]) fprintf(stderr, " %d:%u", b, W.h_counts[kWfDiagLen + cl * 32 + b]);
                    fprintf(stderr, "\n");
                }
                fprintf(stderr, "[wf] finish wave end times (50 us bins):");
                for (int b = 0; b < 64; ++b)
                    if (W.h_counts[kWfDiagHist + b]) fprintf(stderr, " %d:%u", b, W.h_counts[kWfDiagHist + b]);
                fprintf(stderr, "\n[wf] finish queue exhausted at (50 us bins):");
                for (int b = 0; b < 64; ++b)
                    if (W.h_counts[kWfDiagExh + b]) fprintf(stderr, " %d:%u", b, W.h_counts[kWfDiagExh + b]);
                const double ip = W.h_counts[kWfStat + kStatDiagItPre], ix = W.h_counts[kWfStat + kStatDiagItPost];
                const double tp = W.h_counts[kWfStat + kStatDiagTPre], tx = W.h_counts[kWfStat + kStatDiagTPost];
                const double lx = W.h_counts[kWfStat + kStatDiagLanesPost];
                double waves = 0;
                for (int b = 0; b < 64; ++b) waves += W.h_counts[kWfDiagHist + b];
                waves = waves > 0 ? waves : 1;
                fprintf(stderr, "\n[wf] finish per wave: %.0f iterations at %.2f us before its queue ran out, %.0f at %.2f us "
                        "after (%.1f active lanes)\n", ip / waves, ip > 0 ? tp * 0.01 / ip : 0.0, ix / waves,
                        ix > 0 ? tx * 0.01 / ix : 0.0, ix > 0 ? lx / ix : 0.0);
            }
            return true;
        }
        int next = 1 - cur;
        WF_CHECK(hipEventRecord(W.ev[0], stream));
        unsigned g = grid_for(n, Q.shade_blocks);
        unsigned gt = grid_for(n, trace_grid_cap(Q));
        if (count) hipLaunchKernelGGL((wf_trace<false, true>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur, -1);
        else hipLaunchKernelGGL((wf_trace<false, false>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur, -1);
        WF_CHECK(hipEventRecord(W.ev[1], stream));
        const bool sort = Q.sort_bins != 0;
        if (sort) {
            hipLaunchKernelGGL(wf_sort_hist, dim3(kSortBlocks), dim3(kSortThreads), 0, stream, S, Q, cur);
            hipLaunchKernelGGL(wf_sort_rowscan, dim3(Q.sort_bins), dim3(kSortBlocks), 0, stream, Q);
            hipLaunchKernelGGL(wf_sort_scatter, dim3(kSortBlocks), dim3(kSortThreads), 0, stream, S, Q, cur);
        }
        WF_CHECK(hipEventRecord(W.ev[4], stream));
        if (full) {
            if (sort) hipLaunchKernelGGL((wf_shade<true, true>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
            else hipLaunchKernelGGL((wf_shade<true, false>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        } else {
            if (sort) hipLaunchKernelGGL((wf_shade<false, true>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
            else hipLaunchKernelGGL((wf_shade<false, false>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        }
        WF_CHECK(hipEventRecord(W.ev[2], stream));
        if (count) hipLaunchKernelGGL((wf_trace<true, true>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur, -1);
        else hipLaunchKernelGGL((wf_trace<true, false>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur, -1);
        WF_CHECK(hipGetLastError());
        WF_CHECK(hipEventRecord(W.ev[3], stream));
        WF_CHECK(hipMemcpyAsync(W.h_counts, W.counts, kWfCountWords * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        WF_CHECK(hipStreamSynchronize(stream));
        float a = 0, b = 0, c = 0, srt = 0;
        WF_CHECK(hipEventElapsedTime(&a, W.ev[0], W.ev[1]));
        WF_CHECK(hipEventElapsedTime(&srt, W.ev[1], W.ev[4]));
        WF_CHECK(hipEventElapsedTime(&b, W.ev[4], W.ev[2]));
        WF_CHECK(hipEventElapsedTime(&c, W.ev[2], W.ev[3]));
        stage_ms[1] += a;
        stage_ms[6] += srt;
        stage_ms[2] += b;
        stage_ms[3] += c;
        fs->trace_rays += (unsigned long long)n + queue_total(W.h_counts, 2);  // extend + connect rays
        fs->trace_closest_rays += n;
        fs->trace_launches += 2;
        fs->trace_ms += a + c;
        if (Q.diag) {
            fprintf(stderr, "[wf] it %d rays %u shadow %u  extend %.3f sort %.3f shade %.3f connect %.3f ms\n", it, n,
                    queue_total(W.h_counts, 2), a, srt, b, c);
            if (count) {
                for (int any = 0; any < 2; ++any) {
                    fprintf(stderr, "[wf]   %s steps/ray log2 bins (max %u):", any ? "connect" : "extend",
                            W.h_counts[kWfDiagSteps + 64 + any]);
                    for (int b2 = 0; b2 < 32; ++b2)
                        if (W.h_counts[kWfDiagSteps + 32 * any + b2])
                            fprintf(stderr, " %d:%u", b2, W.h_counts[kWfDiagSteps + 32 * any + b2]);
                    fprintf(stderr, "\n");
                }
                WF_CHECK(hipMemsetAsync(W.counts + kWfDiagSteps, 0, 66 * sizeof(uint32_t), stream));
            }
        }
        n = queue_total(W.h_counts, next);
        cur = next;
        ++fs->iterations;
    }
    return true;
}

// ---- device-side control: the whole frame enqueued without host round trips ------------------------
// The host enqueues `rounds_for(paths)` bulk rounds per pass (enough for the live paths to fall
// below the finish threshold when about half of them end per round), then one finish launch;
// the extend launch of a round that finds fewer than `tail` live paths flags tail mode and
// names its queue as the finish input, and every later bulk launch of the pass returns at once.
// Per-stage times come from events between the launches, ray counts and rounds from device
// counters; both are collected by wavefront_collect once the frame has finished.
namespace {
// Whether the HIP runtime takes timeline events inside a captured frame (external event-record
// nodes).  The system ROCm 7.2 runtime the C host links does; the HIP runtime PyTorch bundles
// refuses them (hipEventRecordWithFlags(..., hipEventRecordExternal) during capture: invalid
// argument), so after the first refusal frames are captured without them: the graphs then hold
// the frame's launches, memsets and copies only, and the per-stage times of replayed frames are
// not recorded (rt_stats kernel_ms; the frame's own time, taken outside the graphs, is).
// Process-wide and one-way (true -> false) for g_graph_events; g_ext_refused is the refusal flag of a
// capture attempt.  Atomics: contexts on other threads may capture concurrently (ThreadLocal capture).
static std::atomic<bool> g_graph_events{true};
static thread_local bool g_ext_refused = false;   // set when this thread's capture had an external event record refused

struct Enqueue {
    WfTimeline& T;
    hipStream_t stream;
    bool capture;   // recording into a HIP graph: events and cross-stream waits are external nodes
    int last = -1;
    bool mark(const char** err) {
        if (capture && !g_graph_events) return true;   // untimed capture
        if (T.n_ev >= WfTimeline::kMaxEv) {
            *err = "wavefront timeline: too many events";
            return false;
        }
        const hipError_t e = hipEventRecordWithFlags(T.ev[T.n_ev], stream, capture ? hipEventRecordExternal : 0u);
        if (e != hipSuccess) {
            if (capture) g_ext_refused = true;
            static thread_local char msg[160];
            snprintf(msg, sizeof msg, "hipEventRecordWithFlags(%s): %s", capture ? "external" : "0", hipGetErrorString(e));
            *err = msg;
            return false;
        }
        last = T.n_ev++;
        return true;
    }
    // closes the span [previous mark, now) as `stage`; without a previous mark (part 0 was captured
    // untimed and this part is recorded eagerly) it only marks: there is no start event to time from
    bool span(int stage, const char** err) {
        if (capture && !g_graph_events) return true;
        const int a = last;
        if (!mark(err)) return false;
        if (a >= 0) T.spans[T.n_spans++] = WfTimeline::Span{stage, a, last};
        return true;
    }
};
}  // namespace

static int rounds_for(uint64_t paths, uint32_t tail) {
    if (paths < tail) return 0;
    int k = 2;
    while (k < 16 && (paths >> (k - 1)) >= tail) ++k;
    return k;
}

static bool enqueue_pass(const DevScene& S, const FrameParams& P, const WfParams& Q, int rounds, bool count, bool full,
                         int ts, Enqueue& E, const char** err) {
    hipStream_t stream = E.stream;
    if (!Q.spans) ts = -1;   // no device-clock spans: the kernels skip the stamps
    const unsigned gt = trace_grid_cap(Q), g = Q.shade_blocks;
    for (int k = 0; k < rounds; ++k) {
        const int cur = k & 1;
        const bool kHitSort = Q.sort_bins != 0;
        if (count) hipLaunchKernelGGL((wf_trace<false, true>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur, ts + 2 * k);
        else hipLaunchKernelGGL((wf_trace<false, false>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur, ts + 2 * k);
        if (!E.span(1, err)) return false;
        if (kHitSort) {
            hipLaunchKernelGGL(wf_sort_hist, dim3(kSortBlocks), dim3(kSortThreads), 0, stream, S, Q, cur);
            hipLaunchKernelGGL(wf_sort_rowscan, dim3(Q.sort_bins), dim3(kSortBlocks), 0, stream, Q);
            hipLaunchKernelGGL(wf_sort_scatter, dim3(kSortBlocks), dim3(kSortThreads), 0, stream, S, Q, cur);
            if (!E.span(6, err)) return false;
        }
        if (full) {
            if (kHitSort) hipLaunchKernelGGL((wf_shade<true, true>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
            else hipLaunchKernelGGL((wf_shade<true, false>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        } else {
            if (kHitSort) hipLaunchKernelGGL((wf_shade<false, true>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
            else hipLaunchKernelGGL((wf_shade<false, false>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        }
        if (!E.span(2, err)) return false;
        if (count) hipLaunchKernelGGL((wf_trace<true, true>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur, ts + 2 * k + 1);
        else hipLaunchKernelGGL((wf_trace<true, false>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur, ts + 2 * k + 1);
        if (!E.span(3, err)) return false;
    }
    // the finish chunk counter is zero here: the frame start clears every counter and the
    // extra-sample pass clears it again before its own finish launch
    launch_finish_any(S, Q, count, full, -1, 1u << 30, stream, ts + kTsFinish);   // resident grid; input queue from the counters
    WF_CHECK(hipGetLastError());
    return E.span(5, err);
}

// One frame on `stream` in two parts: record_base = the base pass and the motion vectors,
// record_rest = the extra-sample pass and the resolve, which read the previous frame's outputs
// (the caller enqueues the wait for it in between).  Launch arguments come from S, Q and the
// buffer pointers in P; the per-frame values of P are read by the kernels from Q.Pd.
static bool record_base(const DevScene& S, const FrameParams& P, WfParams& Q, bool count, bool full,
                        hipStream_t stream, WfTimeline& T, bool capture, const char** err) {
    WavefrontBuffers& W = Q.W;
    Enqueue E{T, stream, capture};
    T.n_ev = T.n_spans = 0;
    if (!E.mark(err)) return false;
    // counters, and the launch-span stamps when they are recorded
    T.dev_spans = Q.spans != 0;
    WF_CHECK(hipMemsetAsync(W.counts, 0, Q.spans ? kWfCountAllocBytes : kWfTsOffset, stream));
    const int rounds = rounds_for(Q.base_paths, Q.tail);
    Q.finish_q = rounds & 1;
    hipLaunchKernelGGL(wf_generate, dim3(grid_for(Q.base_paths, 16384)), dim3(kBlock), 0, stream, S, Q.Pd, Q);
    WF_CHECK(hipGetLastError());
    if (!E.span(0, err)) return false;
    if (!enqueue_pass(S, P, Q, rounds, count, full, 0, E, err)) return false;
    hipLaunchKernelGGL(wf_motion, dim3(grid_for(Q.own_pixels, 1u << 30)), dim3(kBlock), 0, stream, S, Q.Pd, Q);
    WF_CHECK(hipGetLastError());
    return E.span(4, err);
}

static bool record_rest(const DevScene& S, const FrameParams& P, WfParams& Q, bool count, bool full, int maxExtra,
                        bool with_extra, hipStream_t stream, WfTimeline& T, bool capture, const char** err) {
    WavefrontBuffers& W = Q.W;
    Enqueue E{T, stream, capture};
    E.last = T.n_ev - 1;   // spans continue from record_base's last event
    if (with_extra) {
        // second pass over the motion-adaptive extra samples (:779-789), appended to queue 0
        const int rounds2 = rounds_for((uint64_t)Q.own_pixels * (uint64_t)maxExtra, Q.tail);
        WF_CHECK(hipMemsetAsync(W.counts, 0, cslot(kShards) * sizeof(uint32_t), stream));
        WF_CHECK(hipMemsetAsync(W.counts + cslot(kCntBack), 0, cslot(kShards) * sizeof(uint32_t), stream));
        WF_CHECK(hipMemsetAsync(W.counts + cslot(kCntChunkExtend), 0, cslot(2 * kShards) * sizeof(uint32_t), stream));
        WF_CHECK(hipMemsetD32Async(W.counts + cslot(kCntTailMode), 0u, 1, stream));
        WF_CHECK(hipMemsetD32Async(W.counts + cslot(kCntFinishQ), (uint32_t)(rounds2 & 1), 1, stream));
        WF_CHECK(hipMemsetAsync(W.counts + cslot(kCntChunkFinish), 0, cslot(kShards) * sizeof(uint32_t), stream));
        hipLaunchKernelGGL(wf_extra, dim3(grid_for(Q.own_pixels, 1u << 30)), dim3(kBlock), 0, stream, S, Q.Pd, Q, 0);
        WF_CHECK(hipGetLastError());
        if (!E.span(4, err)) return false;
        if (!enqueue_pass(S, P, Q, rounds2, count, full, kTsPass, E, err)) return false;
    }
    hipLaunchKernelGGL(wf_resolve, dim3(grid_for(Q.own_pixels, 1u << 30)), dim3(kBlock), 0, stream, S, Q.Pd, Q,
                       with_extra ? 1 : 0);
    WF_CHECK(hipGetLastError());
    if (!E.span(4, err)) return false;
    WF_CHECK(hipMemcpyAsync(W.h_counts, W.counts, Q.spans ? kWfCountAllocBytes : kWfTsOffset, hipMemcpyDeviceToHost,
                            stream));
    return true;
}

static bool record_part(const DevScene& S, const FrameParams& P, WfParams& Q, bool count, bool full, int maxExtra,
                        bool with_extra, int part, hipStream_t stream, WfTimeline& T, bool capture, const char** err) {
    return part == 0 ? record_base(S, P, Q, count, full, stream, T, capture, err)
                     : record_rest(S, P, Q, count, full, maxExtra, with_extra, stream, T, capture, err);
}


// part `part` of the frame (record_part), eagerly or captured into T.exec[part] and launched
static bool capture_part(const DevScene& S, const FrameParams& P, WfParams& Q, bool count, bool full, int maxExtra,
                         bool with_extra, int part, hipStream_t stream, WfTimeline& T, bool rebuild, const char** err) {
    if (rebuild) {
        const char* rerr = nullptr;
        hipGraph_t g = nullptr;
        const int n_ev = T.n_ev, n_spans = T.n_spans;
        hipError_t be, ce, ie;
        bool ok;
        for (int attempt = 0;; ++attempt) {
            g_ext_refused = false;
            be = hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal);
            ok = be == hipSuccess && record_part(S, P, Q, count, full, maxExtra, with_extra, part, stream, T, true, &rerr);
            ce = be == hipSuccess ? hipStreamEndCapture(stream, &g) : be;
            ie = hipErrorUnknown;
            if (ok && ce == hipSuccess && g) ie = hipGraphInstantiateWithFlags(&T.exec[part], g, 0);
            if (g) (void)hipGraphDestroy(g);
            g = nullptr;
            if (!ok && g_ext_refused && g_graph_events && attempt == 0) {
                // this runtime takes no timeline events in a graph: capture untimed from now on
                (void)hipGetLastError();
                g_graph_events = false;
                T.n_ev = n_ev;
                T.n_spans = n_spans;
                continue;
            }
            break;
        }
        if (!ok || ce != hipSuccess || ie != hipSuccess) {
            // capture refused (an API the runtime cannot capture): this slot renders eagerly from now on
            // (rt_stats total_graph_fallbacks counts its frames; the first refusal is reported here)
            static bool reported = false;
            if (!reported) {
                reported = true;
                fprintf(stderr, "rt: frame graph capture (part %d) refused: begin %s, record %s, end %s, instantiate %s; "
                        "the slot renders eagerly\n", part, hipGetErrorString(be), ok ? "ok" : (rerr ? rerr : "?"),
                        hipGetErrorString(ce), hipGetErrorString(ie));
            }
            (void)hipGetLastError();
            T.exec[part] = nullptr;
            T.graph_failed = true;
            T.n_ev = n_ev;
            T.n_spans = n_spans;
            return record_part(S, P, Q, count, full, maxExtra, with_extra, part, stream, T, false, err);
        }
    }
    WF_CHECK(hipGraphLaunch(T.exec[part], stream));
    return true;
}

static bool enqueue_wavefront(const DevScene& S, const FrameParams& P, WfParams& Q, bool count, bool full,
                              int maxExtra, bool extra_pass, hipStream_t stream, hipEvent_t prev_done, WfTimeline& T,
                              const char** err, bool graphs) {
    Q.dev_ctl = 1;
    Q.finish_q = 0;   // set by record_base from the round count
    const bool with_extra = maxExtra > 0 && extra_pass;
    if (!graphs || T.graph_failed) {
        T.graph_mode = graphs ? kGraphFallback : kGraphEager;
        if (!record_base(S, P, Q, count, full, stream, T, false, err)) return false;
        if (prev_done) WF_CHECK(hipStreamWaitEvent(stream, prev_done, 0));
        if (!record_rest(S, P, Q, count, full, maxExtra, with_extra, stream, T, false, err)) return false;
        T.pending = true;
        return true;
    }
    // The frame's launches, memsets and copies only take S, Q (by value) and the slot's fixed
    // buffers and events; everything that changes per frame is in the device FrameParams, uploaded
    // before the launch.  So the graph is valid while these bytes are.
    std::vector<uint8_t> key(sizeof(DevScene) + sizeof(WfParams) + 4 * sizeof(int));
    {
        WfParams Qk = Q;
        Qk.W.param_slot = 0;   // the upload ring position is host bookkeeping
        uint8_t* k = key.data();
        std::memcpy(k, &S, sizeof S);
        std::memcpy(k + sizeof S, &Qk, sizeof Qk);
        const int flags[4] = {count ? 1 : 0, full ? 1 : 0, with_extra ? 1 : 0, maxExtra};
        std::memcpy(k + sizeof S + sizeof Qk, flags, sizeof flags);
    }
    const bool rebuild = !T.exec[0] || !T.exec[1] || T.key != key;
    if (rebuild) {
        // the slot's previous frame has finished (its slot was harvested): its graphs can go
        for (hipGraphExec_t& x : T.exec)
            if (x) {
                WF_CHECK(hipGraphExecDestroy(x));
                x = nullptr;
            }
        T.key.clear();
    }
    if (!capture_part(S, P, Q, count, full, maxExtra, with_extra, 0, stream, T, rebuild, err)) return false;
    if (prev_done) WF_CHECK(hipStreamWaitEvent(stream, prev_done, 0));
    if (T.graph_failed) {   // part 0 could not be captured
        if (!record_rest(S, P, Q, count, full, maxExtra, with_extra, stream, T, false, err)) return false;
    } else if (!capture_part(S, P, Q, count, full, maxExtra, with_extra, 1, stream, T, rebuild, err)) {
        return false;
    }
    if (rebuild && !T.graph_failed) T.key.swap(key);
    T.graph_mode = T.graph_failed ? kGraphFallback : rebuild ? kGraphCapture : kGraphReplay;
    T.pending = true;
    return true;
}

bool wavefront_collect(const WavefrontBuffers& W, WfTimeline& T, WfFrameStats* fs, const char** err) {
    if (!T.pending) return true;
    T.pending = false;
    *fs = WfFrameStats{};
    for (int i = 0; i < T.n_spans; ++i) {
        const WfTimeline::Span& sp = T.spans[i];
        float ms = 0.0f;
        WF_CHECK(hipEventElapsedTime(&ms, T.ev[sp.a], T.ev[sp.b]));
        fs->stage_ms[sp.stage] += ms;
        if (sp.stage == 1 || sp.stage == 3) fs->trace_ms += ms;
    }
    fs->iterations = (int)W.h_counts[kWfStat + kStatRounds];
    fs->trace_launches = (int)W.h_counts[kWfStat + kStatTraceLaunches];
    fs->trace_rays = W.h_counts[kWfStat + kStatTraceRays];
    fs->trace_closest_rays = W.h_counts[kWfStat + kStatExtendRays];
    fs->finish_launches = (int)W.h_counts[kWfStat + kStatFinish];
    fs->graph_mode = T.graph_mode;
    for (int pass = 0; pass < (T.dev_spans ? 2 : 0); ++pass)   // device-clock spans (10 ns ticks) of the launches that ran
        for (int k = 0; k <= kTsFinish; ++k) {
            const int slot = pass * kTsPass + k;
            const unsigned long long a = W.h_tstamp[slot * kTsStride];
            unsigned long long b = 0;
            for (int x = 1; x <= 8; ++x) b = std::max(b, W.h_tstamp[slot * kTsStride + kTsLine * x]);
            if (a == 0 || b <= a) continue;
            const float ms = (float)((double)(b - a) * 1e-5);
            if (k == kTsFinish) {
                fs->finish_dev_ms += ms;
                fs->finish_dev_launches++;
            } else if (k < 2 * 16) {
                fs->trace_dev_ms += ms;
                fs->trace_dev_launches++;
            }
        }
    return true;
}

bool run_wavefront(const DevScene& S, const FrameParams& P, WavefrontBuffers& W, const WfTuning& tu, int own_tiles,
                   bool count, bool spans, int tail_paths, int sort_bins, bool extra_pass, int in_flight,
                   hipStream_t stream, hipEvent_t prev_done, WfTimeline* tl, WfFrameStats* fs, const char** err,
                   bool graphs) {
    WfParams Q;
    std::memset(&Q, 0, sizeof Q);   // no stray padding bytes (frame-graph key)
    Q.W = W;
    Q.spp = max(P.U.samplesPerPixel, 1);
    Q.own_pixels = (uint32_t)own_tiles * (uint32_t)P.tile_size * (uint32_t)P.tile_size;
    Q.base_paths = Q.own_pixels * (uint32_t)Q.spp;
    Q.seg_cap = (uint32_t)(W.queue_entries / kShards);
    Q.refill_min = tu.refill_min;
    Q.chunk = tu.chunk;
    Q.tail = tail_paths > 0 ? (uint32_t)tail_paths : tu.tail;
    Q.sort_bins = (uint32_t)sort_bins;
    Q.diag = tu.log;
    Q.shade_min = tu.shade_min;
    Q.shade_min_x = tu.shade_min_x;
    // the team drain pays where the drain is a large part of the finish: small frames (C3g rank
    // shares, DESIGN.md §3.3: 8-way +2.3 %, 4-way +1.5 %, 2-way ±1 %, the whole 1080p frame four in
    // flight ±0), but not the smallest (C1 256x256x1: -7.5 %)
    Q.team = tu.team >= 0 ? tu.team : (Q.base_paths >= kTeamAutoMin && Q.base_paths <= kTeamAutoPaths ? 4 : 0);
    Q.fchunk = tu.fchunk;
    Q.shade_blocks = tu.shade_blocks;
    Q.spans = spans ? 1 : 0;
    Q.spp_div = make_fastdiv((uint32_t)Q.spp);
    Q.tile = P.tile_size;
    Q.rank = P.rank;
    Q.nranks = P.nranks;
    Q.tile_px_div = make_fastdiv((uint32_t)P.tile_size * (uint32_t)P.tile_size);
    Q.tiles_x_div = make_fastdiv((uint32_t)max(P.tiles_x, 1));
    // frames in flight: the finish tail takes part of the resident grid and leaves the rest to the
    // other frames' bulk rounds (C3g sweeps, DESIGN.md §3: two slots 40 %; four or more 20 %: C3g
    // with four slots 20 / 25 / 33 % 8.49-8.54 / 8.21-8.50 / 8.28-8.36 Grays/s, and a multi-GPU
    // rank's share; three 33 %); one frame at a time: all of it
    // four or more frames in flight: the bulk traversal launches take 60 % of the resident grid,
    // leaving CUs to the other frames' kernels (C3g 8.51-8.64 -> 8.61-8.72 Grays/s over five
    // alternating pairs, 75 % +0.5 %; the 8-way rank share at 75 % +0.9 %); fewer frames: all of it
    // eight frames in flight (round 6): the smaller the frame, the smaller the share, so that more
    // frames' bulk rounds run side by side -- 20 % up to 2.5M base paths (8-way C3g rank share 7.26 ->
    // 7.51-7.54 Grays/s, 4-way 8.59 -> 8.87-8.88; 15 % 7.46-7.49), 30 % up to 6M (2-way 9.29 ->
    // 9.47-9.55), 40 % above (the whole C3g frame 9.74-9.83 -> 9.82-9.91; 50 % 9.80-9.81)
    // (profiles/r06_experiments.txt)
    Q.trace_frac = tu.trace_frac > 0 ? tu.trace_frac
                 : in_flight >= 8 ? (Q.base_paths <= 2500000u ? 20 : Q.base_paths <= 6000000u ? 30 : 40)
                 : in_flight >= 4 ? 60 : 100;
    // eight frames in flight of at most 6M base paths (a multi-GPU rank's share): 12 % (round 5,
    // after the slots stopped serialising: 8-way rank share 6.76 -> 7.02, 4-way 8.14 -> 8.44, 2-way
    // (4.1M paths) 9.12 -> 9.35 Grays/s; 8 % +-0, 33 % -10 %; the whole C3g frame (8.3M) +-0 and
    // configs[3]'s 16.6M-path rank share -2 %, so larger frames keep 20 %)
    Q.finish_frac = tu.finish_frac > 0 ? tu.finish_frac
                  : (in_flight >= 8 && Q.base_paths <= 6000000u) ? 12
                  : in_flight >= 4 ? 20 : in_flight == 2 ? 40 : (in_flight > 1 ? 100 / in_flight : 100);
    if (sort_bins && (sort_bins < kSortMinBins || sort_bins > kSortMaxBins || (sort_bins & (sort_bins - 1)) ||
                      !S.tri_bin || !W.sorted)) {
        *err = "bad hit-sort configuration";
        return false;
    }
    *fs = WfFrameStats{};
    float* stage_ms = fs->stage_ms;
    // tail <= 1 (bulk rounds only, a test configuration) keeps the host loop: its round count is
    // only bounded by maxBounces * (maxBounces + 1)
    const bool dev = tl && !tu.host_ctl && !tu.log && Q.tail > 1;
    Q.Pd = W.d_params;
    {   // this frame's parameters -> device; the slot's previous upload has executed once its event has
        const int slot = W.param_slot;
        W.param_slot = (slot + 1) % WavefrontBuffers::kParamSlots;
        WF_CHECK(hipEventSynchronize(W.param_ev[slot]));
        W.h_params[slot] = P;
        WF_CHECK(hipMemcpyAsync(W.d_params, &W.h_params[slot], sizeof(FrameParams), hipMemcpyHostToDevice, stream));
        WF_CHECK(hipEventRecord(W.param_ev[slot], stream));
    }
    const bool full = needs_full(P.U, S);
    const int maxExtra = (P.U.enableMotionAdaptiveSampling != 0) ? max(P.U.motionSamplingMaxExtraSamples, 0) : 0;
    if (dev) {
        // the device queries behind the grid sizes run before a stream is capturing (a capture
        // must hold stream work only)
        (void)trace_grid_cap(Q);
        (void)finish_full_cap<false, false, false>();
        (void)finish_full_cap<false, true, false>();
        (void)finish_full_cap<true, false, false>();
        (void)finish_full_cap<true, true, false>();
        (void)finish_full_cap<false, false, true>();
        (void)finish_full_cap<false, true, true>();
        (void)finish_full_cap<true, false, true>();
        (void)finish_full_cap<true, true, true>();
        return enqueue_wavefront(S, P, Q, count, full, maxExtra, extra_pass, stream, prev_done, *tl, err, graphs);
    }
    Q.dev_ctl = 0;
    Q.finish_q = 0;

    WF_CHECK(hipEventRecord(W.ev[0], stream));
    WF_CHECK(hipMemsetAsync(W.counts, 0, kWfCountWords * sizeof(uint32_t), stream));
    hipLaunchKernelGGL(wf_generate, dim3(grid_for(Q.base_paths, 16384)), dim3(kBlock), 0, stream, S, Q.Pd, Q);
    WF_CHECK(hipGetLastError());
    WF_CHECK(hipEventRecord(W.ev[1], stream));
    WF_CHECK(hipMemcpyAsync(W.h_counts, W.counts, kWfCountWords * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    WF_CHECK(hipStreamSynchronize(stream));
    float ms = 0;
    WF_CHECK(hipEventElapsedTime(&ms, W.ev[0], W.ev[1]));
    stage_ms[0] += ms;
    int cur = 0;
    if (!iterate(S, P, Q, cur, queue_total(W.h_counts, 0), count, full, stream, fs, err)) return false;

    if (prev_done) WF_CHECK(hipStreamWaitEvent(stream, prev_done, 0));
    WF_CHECK(hipEventRecord(W.ev[0], stream));
    hipLaunchKernelGGL(wf_motion, dim3(grid_for(Q.own_pixels, 1u << 30)), dim3(kBlock), 0, stream, S, Q.Pd, Q);
    WF_CHECK(hipGetLastError());
    if (maxExtra > 0) {
        // the extra-sample pass appends primary rays to queue `cur` (reset here)
        WF_CHECK(hipMemsetAsync(W.counts + cslot(cur * kShards), 0, cslot(kShards) * sizeof(uint32_t), stream));
        WF_CHECK(hipMemsetAsync(W.counts + cslot(kCntBack + cur * kShards), 0, cslot(kShards) * sizeof(uint32_t), stream));
        hipLaunchKernelGGL(wf_extra, dim3(grid_for(Q.own_pixels, 1u << 30)), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        WF_CHECK(hipGetLastError());
        WF_CHECK(hipMemcpyAsync(W.h_counts, W.counts, kWfCountWords * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        WF_CHECK(hipStreamSynchronize(stream));
        uint32_t n_extra = queue_total(W.h_counts, cur);
        if (n_extra > 0) {
            if (!iterate(S, P, Q, cur, n_extra, count, full, stream, fs, err)) return false;
        }
    }
    hipLaunchKernelGGL(wf_resolve, dim3(grid_for(Q.own_pixels, 1u << 30)), dim3(kBlock), 0, stream, S, Q.Pd, Q,
                       maxExtra > 0 ? 1 : 0);
    WF_CHECK(hipGetLastError());
    WF_CHECK(hipEventRecord(W.ev[1], stream));
    WF_CHECK(hipStreamSynchronize(stream));
    WF_CHECK(hipEventElapsedTime(&ms, W.ev[0], W.ev[1]));
    stage_ms[4] += ms;
    return true;
}

}  // namespace rt
