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

#include <cstdio>
#include <cstring>
#include <vector>

namespace rt {

namespace {

constexpr uint32_t kTailRaysDefault = 4194304;
static uint32_t tail_rays() {  // RT_TAIL_RAYS overrides (tuning experiments)
    static uint32_t v = [] { const char* e = getenv("RT_TAIL_RAYS"); return e ? (uint32_t)atol(e) : kTailRaysDefault; }();
    return v;
}

static int refill_min() {  // RT_REFILL_MIN overrides (tuning experiments)
    static int v = [] { const char* e = getenv("RT_REFILL_MIN"); return e ? atoi(e) : 8; }();
    return v;
}

static int chunk_size() {  // RT_CHUNK overrides (tuning experiments)
    static int v = [] { const char* e = getenv("RT_CHUNK"); return e ? atoi(e) : 64; }();
    return v;
}

static int env_int(const char* name, int dflt) {  // tuning experiments
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}

static bool wf_log() {  // RT_WF_LOG=1: per-iteration queue sizes and stage times on stderr
    static const bool v = env_int("RT_WF_LOG", 0) != 0;
    return v;
}

static uint32_t drain_paths() {  // RT_DRAIN_PATHS: finish rounds with fewer paths never drain
    static const uint32_t v = (uint32_t)env_int("RT_DRAIN_PATHS", 65536);
    return v;
}

static int tri_vote() {  // RT_TRI_VOTE overrides (tuning experiments)
    static int v = [] { const char* e = getenv("RT_TRI_VOTE"); return e ? atoi(e) : 0; }();
    return v;
}

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

__device__ __forceinline__ uint32_t compact1by1(uint32_t x) {
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0f0f0f0fu;
    x = (x | (x >> 4)) & 0x00ff00ffu;
    x = (x | (x >> 8)) & 0x0000ffffu;
    return x;
}

// own pixel index -> image coordinates (tiles tile_id % nranks == rank, Morton order in a tile)
__device__ __forceinline__ void own_pixel(const FrameParams& P, uint32_t i, int& px, int& py) {
    const uint32_t T = (uint32_t)P.tile_size, per = T * T;
    uint32_t k = i / per, r = i % per;
    int tid = P.rank + (int)k * P.nranks;
    int tx = tid % P.tiles_x, ty = tid / P.tiles_x;
    uint32_t lx, ly;
    if ((T & (T - 1)) == 0) {
        lx = compact1by1(r);
        ly = compact1by1(r >> 1);
    } else {
        lx = r % T;
        ly = r / T;
    }
    px = tx * (int)T + (int)lx;
    py = ty * (int)T + (int)ly;
}

__device__ __forceinline__ uint32_t pack_state(int bounce, int tpass, int step) {
    return (uint32_t)bounce | ((uint32_t)tpass << 8) | ((uint32_t)step << 16);
}

struct WfParams {
    WavefrontBuffers W;
    uint32_t base_paths;   // own pixels * spp
    uint32_t own_pixels;
    uint32_t seg_cap;      // entries per queue segment
    int spp;
    int refill_min;        // wf_trace refills once at least this many lanes of a wave are idle
    int tri_vote;          // wf_trace phase vote threshold (lanes with triangle work), 0 = off
    int chunk;             // wf_trace dynamic chunk size (rays per grab), 0 = static wave ranges
    uint32_t tail;         // live paths below which wf_finish runs the rest
    uint32_t sort_bins;    // hit-sort bins (0 = shade reads the extend queue unsorted)
    int sort_xcd;          // sorted shade: XCD k shades the k-th eighth of the sorted hits
    int steal;             // wf_trace: a wave whose XCD's eighth ran dry takes chunks of the others
    int diag;              // wf_finish: record the diagnostics slots (RT_WF_LOG)
    int finish_step;       // tail: wf_finish_step (1) or the per-segment wf_finish (0)
    int shade_min;         // wf_finish_step: shade once this many lanes wait (or none traverses)
    int drain_min;         // wf_finish_step: hand paths back to the next round below this many busy lanes
    int prio;              // finish input reordered by wf_prio (likely-long paths first) into W.sorted
    int fchunk;            // wf_finish_step: paths per chunk grab
    int finish_frac;       // percent of the resident grid the finish launch takes
    int dev_ctl;           // device-side control (enqueue_wavefront): kernels read their queue sizes from
                           // the counters and skip once the live count fell below `tail`
    int finish_q;          // dev_ctl: the finish queue when every enqueued bulk round ran (written by generate)
    const FrameParams* Pd; // this frame's FrameParams in device memory (W.d_params)
};

// counter slots (cslot): [q*8 + shard] ray queues q = 0, 1; [16 + shard] shadow queue; [24] extra allocator
constexpr int kCntShadowQ = 16;
constexpr int kCntExtra = 24;
constexpr int kCntChunkFinish = 25;
constexpr int kCntSorted = 26;                 // hits the sort kept (misses dropped) = shade's input size
constexpr uint32_t kNoKey = 0xffffffffu;       // sort key of a miss (dropped by the sort)
constexpr int kCntDiagSegs = 27, kCntDiagIters = 28, kCntDiagTime = 29;   // wf_finish diagnostics
// dev_ctl: [30] tail mode (set by the first extend launch that found fewer than `tail` live
// paths; later bulk launches of the pass return at once), [31] the queue the finish launch reads
constexpr int kCntTailMode = 30, kCntFinishQ = 31;
constexpr int kCntPrioHi = 48, kCntPrioLo = 49;   // wf_prio allocation counters (reset per launch)

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
__device__ __forceinline__ ShardPrefix load_prefix(const uint32_t* cnt) {
    ShardPrefix p;
    uint32_t acc = 0;
    #pragma unroll
    for (int k = 0; k < kShards; ++k) {
        acc += __builtin_amdgcn_readfirstlane(cnt[cslot(k)]);
        p.end[k] = acc;
    }
    return p;
}
// dense consumer index g (< p.end[kShards - 1]) -> entry index of the sharded queue
__device__ __forceinline__ uint32_t entry_of(const ShardPrefix& p, uint32_t g, uint32_t seg_cap) {
    uint32_t k = 0, start = 0;
    #pragma unroll
    for (int j = 0; j < kShards - 1; ++j) {
        const bool past = g >= p.end[j];
        k = past ? (uint32_t)(j + 1) : k;
        start = past ? p.end[j] : start;
    }
    return k * seg_cap + (g - start);
}

__device__ __forceinline__ void init_path(const WfParams& Q, uint32_t pid, uint32_t pix, int sample, uint32_t hidx) {
    Q.W.p_color[pid] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    Q.W.p_accum[pid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    Q.W.p_meta[pid] = make_uint4(pix, (uint32_t)sample, 0u, hidx);
}


__device__ __forceinline__ void flush_counters(const FrameParams& P, uint32_t closest, uint32_t shadow, uint32_t paths,
                                               const TraceCounters& tc, bool count, bool overflow,
                                               bool trace_kernel = false) {
    block_flush_counters(P.counters, closest, shadow, count ? tc.nodes : 0u, count ? tc.tris : 0u, paths, overflow,
                         trace_kernel);
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

// Node order: a group's hit internal children in the node's slot order (centroids along its
// longest axis, reversed for rays going the other way).  RT_NEAREST_FIRST=1 visits the nearest hit
// internal child (smallest entry distance) first: 2.3 % fewer node visits, but with the
// branch-free node test its per-child key costs more than the visits it saves (final round-2
// kernels: 7.09 -> 7.17 Grays/s with it off, A/B three runs each).
#ifndef RT_TRI_THEN_NODE
#define RT_TRI_THEN_NODE 1   // a lane may run its last triangle step and its next node step in one iteration
#endif
#ifndef RT_TRAV_SCHED
#define RT_TRAV_SCHED 1   // wf_trace iteration: 1 = triangle step, node step; 2 = + a second node step; 3 = + a second triangle step
#endif
#ifndef RT_PRIO_LOADS
#define RT_PRIO_LOADS 0   // raise the wave priority (s_setprio) while a traversal step issues its loads
#endif
#ifndef RT_TRI_B_MASKED
#define RT_TRI_B_MASKED 0   // 1: branch around the second triangle's loads (measured 1-2 % slower: 7.07 -> 6.97 Grays/s)
#endif
#ifndef RT_NEAREST_ANY
#define RT_NEAREST_ANY 1   // nearest-child-first for the shadow (any-hit) queue too
#endif
#ifndef RT_NEAREST_FIRST
#define RT_NEAREST_FIRST 0
#endif

// ---- generate -------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) wf_generate(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    __shared__ HaltonDim lds_halton[kHaltonLds];
    __shared__ BlockAlloc ba;
    const ShadeTabs halton = load_tabs(S, lds_halton, nullptr);   // no shading: Halton only
    const Uniforms& U = P.U;
    const int spp = Q.spp;
    const int maxExtra = (U.enableMotionAdaptiveSampling != 0) ? max(U.motionSamplingMaxExtraSamples, 0) : 0;
    const int stride = spp + maxExtra;
    const int shard = blockIdx.x & (kShards - 1);
    float4* qout = Q.W.q[0] + 2 * (size_t)shard * Q.seg_cap;
    uint32_t n_paths = 0;
    const uint32_t total = Q.base_paths;
    if (Q.dev_ctl && blockIdx.x == 0 && threadIdx.x == 0) Q.W.counts[cslot(kCntFinishQ)] = (uint32_t)Q.finish_q;
    for (uint32_t base = blockIdx.x * kBlock; base < total; base += gridDim.x * kBlock) {
        uint32_t pid = base + threadIdx.x;
        bool valid = pid < total;
        int px = 0, py = 0, s = 0;
        uint32_t pix = 0;
        if (valid) {
            s = (int)(pid % (uint32_t)spp);
            own_pixel(P, pid / (uint32_t)spp, px, py);
            valid = px < U.width && py < U.height;
            pix = (uint32_t)py * (uint32_t)U.width + (uint32_t)px;
        }
        f3 o = mk3(0, 0, 0), d = mk3(0, 0, 0);
        if (valid) {
            uint32_t offset = P.random[pix];
            int frameOffset = (int)U.frameIndex * stride + s;
            int hidx = (int)(offset + (unsigned)frameOffset);
            init_path(Q, pid, pix, s, (uint32_t)hidx);
            primary_ray(U, halton, px, py, hidx, o, d);
            if (s == 0) {  // per-pixel defaults (:252-261)
                P.depth[pix] = 1.0e8f;
                P.motion[pix] = make_float2(0.0f, 0.0f);
                P.prim_hit[pix] = make_uint4(0xffffffffu, 0u, 0u, 0u);
                if (P.gbuffer) {
                    size_t plane = (size_t)U.width * U.height;
                    float4 z = make_float4(0, 0, 0, 0);
                    P.gbuffer[pix] = z;
                    P.gbuffer[plane + pix] = z;
                    P.gbuffer[2 * plane + pix] = z;
                    P.gbuffer[3 * plane + pix] = z;
                }
            }
            n_paths++;
        }
        bool live = valid && U.maxBounces > 0;
        uint32_t slot = block_alloc(live, &Q.W.counts[cslot(shard)], ba);
        if (live) {
            qout[2 * slot] = make_float4(o.x, o.y, o.z, __uint_as_float(pid));
            qout[2 * slot + 1] = make_float4(d.x, d.y, d.z, 0.0f);
        }
    }
    TraceCounters tc{0, 0};
    flush_counters(P, 0, 0, n_paths, tc, false, false);
}

// ---- shade -------------------------------------------------------------------------------------------
// SORTED: the input is the hit-sorted array (wf_sort_scatter; misses already dropped) and the
// blocks of XCD k (blockIdx % 8) shade the k-th eighth of it, so one XCD's L2 serves one scene
// region and the rays / shadow rays it appends to its queue shard stay grouped by region for
// the next extend / connect launches (which hand shard k's range to XCD k).
template <bool FULL, bool SORTED>
// RT_SHADE_WAVES (build-time): force an occupancy; 5 waves (96 VGPRs + 44 B/lane spills) measured
// 3 % slower than the compiler's 4 waves at 123 VGPRs
#if defined(RT_SHADE_WAVES) && RT_SHADE_WAVES > 0
#define RT_SHADE_ATTR __attribute__((amdgpu_waves_per_eu(RT_SHADE_WAVES, RT_SHADE_WAVES)))
#else
#define RT_SHADE_ATTR
#endif
__global__ void __launch_bounds__(kBlock) RT_SHADE_ATTR wf_shade(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q, int cur) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    __shared__ HaltonDim lds_halton[kHaltonLds];
    __shared__ MatRec lds_mat[kMatLds];
    __shared__ BlockAlloc ba_ray, ba_sh;
    if (tail_mode(Q)) return;
    const ShadeTabs halton = load_tabs(S, lds_halton, lds_mat);
    const Uniforms& U = P.U;
    const int next = 1 - cur;
    const int shard = blockIdx.x & (kShards - 1);
    const ShardPrefix cnt = load_prefix(Q.W.counts + cslot(cur * kShards));
    uint32_t n = cnt.end[kShards - 1];
    const float4* qin = Q.W.q[cur];
    float4* qout = Q.W.q[next] + 2 * (size_t)shard * Q.seg_cap;
    float4* sqout = Q.W.sq + 3 * (size_t)shard * Q.seg_cap;
    f2 zero2;
    zero2.x = 0.0f;
    zero2.y = 0.0f;
    uint32_t beg = blockIdx.x * kBlock, end = n, stride = gridDim.x * kBlock;
    if (SORTED) n = __builtin_amdgcn_readfirstlane(Q.W.counts[cslot(kCntSorted)]);
    end = n;
    if (SORTED && Q.sort_xcd) {   // grid is a multiple of 8 (grid_for)
        beg = (uint32_t)(((uint64_t)n * (uint32_t)shard) / kShards);
        end = (uint32_t)(((uint64_t)n * (uint32_t)(shard + 1)) / kShards);
        beg += (blockIdx.x >> 3) * kBlock;
        stride = (gridDim.x >> 3) * kBlock;
    }
    for (uint32_t base = beg; base < end; base += stride) {
        uint32_t g = base + threadIdx.x;
        StepResult r;
        r.next = false;
        r.shadow = false;
        uint32_t pid = 0;
        f3 rayO = mk3(0, 0, 0), rayD = mk3(0, 0, 0);
        if (g < end) {
            float4 o, d, hv;
            if (SORTED) {
                o = Q.W.sorted[3 * (size_t)g];
                d = Q.W.sorted[3 * (size_t)g + 1];
                hv = Q.W.sorted[3 * (size_t)g + 2];
            } else {
                uint32_t e = entry_of(cnt, g, Q.seg_cap);
                o = qin[2 * (size_t)e];
                d = qin[2 * (size_t)e + 1];
                hv = Q.W.hits[e];
            }
            pid = __float_as_uint(o.w);
            Hit h;
            h.t = hv.x;
            h.id = __float_as_uint(hv.y);
            h.u = hv.z;
            h.v = hv.w;
            if (h.id != 0xffffffffu) {                                           // miss -> path ends (:321-322)
                uint4 meta = Q.W.p_meta[pid];
                float4 c = Q.W.p_color[pid];
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
                if (r.next) Q.W.p_color[pid] = make_float4(p.color.x, p.color.y, p.color.z, 0.0f);
                // radiance only changes on emissive hits (:585-586): skip the store otherwise
                if (__float_as_uint(p.accum.x) != __float_as_uint(a.x) || __float_as_uint(p.accum.y) != __float_as_uint(a.y) ||
                    __float_as_uint(p.accum.z) != __float_as_uint(a.z)) {
                    if (!FULL) {
                        const float4 s = Q.W.p_accum[pid];
                        p.accum = mk3(s.x + p.accum.x, s.y + p.accum.y, s.z + p.accum.z);
                    }
                    Q.W.p_accum[pid] = make_float4(p.accum.x, p.accum.y, p.accum.z, 0.0f);
                }
                if (r.next) Q.W.p_meta[pid] = make_uint4(meta.x, meta.y, pack_state(p.bounce, p.tpass, p.step), meta.w);
            }
        }
        uint32_t ns = block_alloc(r.shadow, &Q.W.counts[cslot(kCntShadowQ + shard)], ba_sh);
        if (r.shadow) {
            sqout[3 * (size_t)ns] = make_float4(r.so.x, r.so.y, r.so.z, __uint_as_float(pid));
            sqout[3 * (size_t)ns + 1] = make_float4(r.sd.x, r.sd.y, r.sd.z, r.stmax);
            sqout[3 * (size_t)ns + 2] = make_float4(r.contrib.x, r.contrib.y, r.contrib.z, 0.0f);
        }
        uint32_t nr = block_alloc(r.next, &Q.W.counts[cslot(next * kShards + shard)], ba_ray);
        if (r.next) {
            qout[2 * (size_t)nr] = make_float4(rayO.x, rayO.y, rayO.z, __uint_as_float(pid));
            qout[2 * (size_t)nr + 1] = make_float4(rayD.x, rayD.y, rayD.z, 0.0f);
        }
    }
}

// ---- hit sort (between extend and shade) -------------------------------------------------------------
// A counting sort of the extend queue's hits by key (the bin of the hit triangle's BVH leaf slot,
// S.tri_bin; leaf order is spatially coherent, so a bin is one scene region), in three launches: per-block histograms, a scan of each bin's row of block counts, and a
// scatter that writes {o, d, hit} of every hit to its bin's range.  Misses are dropped (their
// paths end, :321-322).  The order inside a bin is arbitrary; per-path results do not depend on
// the order paths are shaded in, so the output stays bit-identical.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const uint32_t lane = lane_id();
    #pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(v, off, 64);
        if (lane >= (uint32_t)off) v += t;
    }
    return v;
}

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
    const ShardPrefix cnt = load_prefix(Q.W.counts + cslot(cur * kShards));
    for (uint32_t k = threadIdx.x; k < K; k += kSortThreads) h[k] = 0;
    __syncthreads();
    uint32_t beg, end;
    sort_range(cnt.end[kShards - 1], beg, end);
    for (uint32_t g = beg + threadIdx.x; g < end; g += kSortThreads) {
        const uint32_t k = sort_key(S, Q, entry_of(cnt, g, Q.seg_cap), shift);
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
    const ShardPrefix cnt = load_prefix(Q.W.counts + cslot(cur * kShards));
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
    sort_range(cnt.end[kShards - 1], beg, end);
    for (uint32_t g = beg + threadIdx.x; g < end; g += kSortThreads) {
        const uint32_t e = entry_of(cnt, g, Q.seg_cap);
        const float4 hv = Q.W.hits[e];
        const uint32_t id = __float_as_uint(hv.y);
        if (id == 0xffffffffu) continue;
        const uint32_t pos = atomicAdd(&off[(uint32_t)S.tri_bin[id] >> shift], 1u);
        const float4 o = qin[2 * (size_t)e], d = qin[2 * (size_t)e + 1];
        Q.W.sorted[3 * (size_t)pos] = o;
        Q.W.sorted[3 * (size_t)pos + 1] = d;
        Q.W.sorted[3 * (size_t)pos + 2] = hv;
    }
}

// ---- persistent traversal with per-lane refill (extend: ANY = false, connect: ANY = true) -----------
// Each wave owns a static contiguous range of the queue and keeps all 64 lanes busy: a lane whose
// ray is finished takes the next ray of the range at the top of the next iteration, and every
// iteration advances each lane by exactly one unit of work — one 8-wide node test or one
// triangle.  The wave therefore runs ~(total units of its rays)/64 iterations instead of
// (slowest ray) x (rays per lane).
template <bool ANY, bool COUNT>
#ifndef RT_EXTEND_WAVES
#define RT_EXTEND_WAVES 8   // 64 VGPRs, no scratch (final round-2 node test; at 70 VGPRs it took 7 waves)
#endif
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(ANY ? 8 : RT_EXTEND_WAVES, ANY ? 8 : RT_EXTEND_WAVES))) wf_trace(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q, int cur) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    __shared__ int lds_stack[kStackSize * kBlock];
    constexpr int kTop = ANY ? RT_TOP_CONNECT : RT_TOP_EXTEND;
    __shared__ uint4 lds_top[kTop * 5];   // BVH top levels (BFS order: root, its children, ...)
    int* stack = &lds_stack[threadIdx.x];
    if (Q.dev_ctl) {
        // device-side round control: extend decides (uniformly, from the counters) whether this
        // round runs in bulk or the rest of the pass goes to the finish launch
        const bool tm = tail_mode(Q);
        if (ANY) {
            if (tm) return;
        } else {
            const ShardPrefix c0 = load_prefix(Q.W.counts + cslot(cur * kShards));
            if (tm || c0.end[kShards - 1] < Q.tail) {
                if (!tm && blockIdx.x == 0 && threadIdx.x == 0) {
                    Q.W.counts[cslot(kCntTailMode)] = 1u;
                    Q.W.counts[cslot(kCntFinishQ)] = (uint32_t)cur;
                }
                return;
            }
        }
    }
    const uint32_t n_top = (uint32_t)min(S.num_nodes8, kTop);
    for (uint32_t i = threadIdx.x; i < n_top * 5; i += kBlock)
        lds_top[i] = reinterpret_cast<const uint4*>(S.nodes8)[i];
    __syncthreads();
    const ShardPrefix cnt = load_prefix(ANY ? Q.W.counts + cslot(kCntShadowQ) : Q.W.counts + cslot(cur * kShards));
    const uint32_t n = cnt.end[kShards - 1];
    if (Q.dev_ctl) {
        stat_add(Q, kStatTraceRays, n);
        stat_add(Q, kStatTraceLaunches, 1u);
        if (!ANY) {
            stat_add(Q, kStatRounds, 1u);
            stat_add(Q, kStatExtendRays, n);
        }
    }
    if (!ANY && blockIdx.x == 0 && threadIdx.x < 2 * kShards) {  // reset the queues shade / connect fill
        const int next = 1 - cur;
        uint32_t k = threadIdx.x & (kShards - 1);
        Q.W.counts[cslot(threadIdx.x < kShards ? next * kShards + k : kCntShadowQ + k)] = 0;
    }
    // chunk counters of the OTHER traversal kind are reset here for its next launch (extend and
    // connect alternate; the frame start zeroes both)
    if (blockIdx.x == 0 && threadIdx.x < kShards)
        Q.W.counts[cslot((ANY ? kCntChunkExtend : kCntChunkConnect) + threadIdx.x)] = 0;
    const float4* qin = ANY ? Q.W.sq : Q.W.q[cur];
    const int qstride = ANY ? 3 : 2;
    // static wave ranges, contiguous per XCD (blocks b and b+8 share an XCD)
    const uint32_t nb = gridDim.x, per = nb / 8;
    uint32_t b = blockIdx.x;
    if (b < per * 8) b = (b & 7) * per + (b >> 3);
    const uint32_t waves = nb * (kBlock / 64);
    const uint32_t wv = b * (kBlock / 64) + (threadIdx.x >> 6);
    // static: this wave's range; dynamic (Q.chunk > 0): chunks of this XCD's eighth of the queue,
    // grabbed with one atomic per chunk when the current one runs out
    uint32_t wnext, wend;
    const uint32_t xcd = blockIdx.x & 7u;
    uint32_t* const chunk_ctr0 = Q.W.counts + cslot(ANY ? kCntChunkConnect : kCntChunkExtend);
    // eighth the wave grabs from: its own XCD's, then (Q.steal) the following XCDs' once that one
    // ran dry, so one slow region cannot hold the launch; 8 = nothing left
    uint32_t stolen = 0;
    if (Q.chunk > 0) {
        wnext = wend = 0;
    } else {
        wnext = (uint32_t)(((uint64_t)n * wv) / waves);
        wend = (uint32_t)(((uint64_t)n * (wv + 1)) / waves);
    }

    TraceCounters tc{0, 0};
    bool overflow = false;
    uint32_t rays = 0;
    bool active = false, hit_any = false, g_flip = false;
    uint32_t e = 0;
    RaySetup R = ray_setup(mk3(0, 0, 0), mk3(1, 0, 0));
    float best = 0.0f, bu = 0.0f, bv = 0.0f, bdet = 1.0f;   // closest hit: u = bu / bdet, v = bv / bdet
    uint32_t best_id = 0xffffffffu, g_base = 0, g_hits = 0, t_base = 0, t_mask = 0, t_valid = 0;
    int sp = 0;
    uint32_t steps = 0;   // COUNT: iterations the current ray has taken
    [[maybe_unused]] int g_near = -1;   // RT_NEAREST_FIRST: rank of the nearest hit child of the last node test

    while (true) {
        // refill idle lanes from the wave's range
        unsigned long long idle = __ballot(!active);
        if (Q.chunk > 0 && wnext >= wend && stolen < 8 && (__popcll(idle) >= Q.refill_min || idle == ~0ull)) {
            const uint32_t xc = (xcd + stolen) & 7u;
            const uint32_t xbeg = (uint32_t)(((uint64_t)n * xc) / 8), xend = (uint32_t)(((uint64_t)n * (xc + 1)) / 8);
            uint32_t base = 0;
            if (lane_id() == 0) base = atomicAdd(chunk_ctr0 + cslot((int)xc), (uint32_t)Q.chunk);
            base = xbeg + __builtin_amdgcn_readfirstlane(base);
            if (base >= xend) {
                stolen = Q.steal ? stolen + 1 : 8;
            } else {
                wnext = base;
                wend = min(base + (uint32_t)Q.chunk, xend);
            }
        }
        if (idle != 0ull && wnext < wend && (__popcll(idle) >= Q.refill_min || idle == ~0ull)) {
            if (!active) {
                uint32_t g = wnext + mbcnt64(idle);
                if (g < wend) {
                    e = entry_of(cnt, g, Q.seg_cap);
                    float4 o4 = qin[(size_t)qstride * e], d4 = qin[(size_t)qstride * e + 1];
                    R = ray_setup(ld3(o4), ld3(d4));
                    best = ANY ? d4.w : INFINITY;
                    best_id = 0xffffffffu;
                    bu = bv = 0.0f;
                    bdet = 1.0f;
                    g_base = 0;
                    g_hits = 1;   // virtual group holding the root
                    g_flip = false;
                    g_near = -1;
                    t_mask = 0;
                    sp = 0;
                    hit_any = false;
                    active = true;
                    rays++;
                    if (COUNT) steps = 0;
                }
            }
            wnext += (uint32_t)__popcll(idle);
        }
        if (__ballot(active) == 0ull) break;
        if (!active) continue;
        if (RT_PRIO_LOADS) __builtin_amdgcn_s_setprio(2);   // the wave about to issue its triangle loads goes first
        if (COUNT) ++steps;

        bool done = false;
        // Phase vote: a wave runs EITHER a triangle step OR a node step per iteration, so the
        // two code paths are never both issued; triangles wait until at least tri_vote lanes
        // have some (or no lane has node work).  tri_vote == 0: per-lane choice (both issued).
        bool do_tri = t_mask != 0u, do_node = t_mask == 0u;
        if (Q.tri_vote > 0) {
            const unsigned long long bt = __ballot(do_tri), bn = __ballot(do_node);
            const bool tri_phase = __popcll(bt) >= Q.tri_vote || bn == 0ull;
            do_tri = do_tri && tri_phase;
            do_node = do_node && !tri_phase;
        }
        // ---- up to two triangles: both fetched before either is tested (one memory latency),
        // tested in mask order so closest-hit updates are those of the serial loop
        auto tri_step = [&]() {
            const int k0 = lowest_bit(t_mask);
            t_mask &= t_mask - 1u;
            const bool two = t_mask != 0u;
            const int k1 = two ? lowest_bit(t_mask) : k0;
            if (two) t_mask &= t_mask - 1u;
            const float4* tp0 = S.tris + 3 * (size_t)tri_slot(t_base, t_valid, k0);
            const float4* tp1 = S.tris + 3 * (size_t)tri_slot(t_base, t_valid, k1);
            const float4 a0 = tp0[0], a1 = tp0[1], a2 = tp0[2];
            float4 b0 = a0, b1 = a1, b2 = a2;   // the second triangle is fetched only by lanes that have one
#if RT_TRI_B_MASKED
            if (two) {
                b0 = tp1[0];
                b1 = tp1[1];
                b2 = tp1[2];
            }
#else
            b0 = tp1[0];
            b1 = tp1[1];
            b2 = tp1[2];
#endif
            if (RT_PRIO_LOADS) __builtin_amdgcn_s_setprio(0);
            if (COUNT) tc.tris += two ? 2u : 1u;
            float t, u, v, dt;
            if (intersect_triangle_vw(R.pre, R.o, ld3(a0), ld3(a1), ld3(a2), 0.0f, best, &t, &u, &v, &dt)) {
                const uint32_t id = __float_as_uint(a0.w);
                if (ANY) {
                    hit_any = true;
                    done = true;
                } else if (t < best || id < best_id) {
                    best = t;
                    best_id = id;
                    bu = u;
                    bdet = dt;
                    bv = v;
                }
            }
            if (two && !done && intersect_triangle_vw(R.pre, R.o, ld3(b0), ld3(b1), ld3(b2), 0.0f, best, &t, &u, &v, &dt)) {
                const uint32_t id = __float_as_uint(b0.w);
                if (ANY) {
                    hit_any = true;
                    done = true;
                } else if (t < best || id < best_id) {
                    best = t;
                    best_id = id;
                    bu = u;
                    bdet = dt;
                    bv = v;
                }
            }
        };
        // ---- one 8-wide node
        auto node_step = [&]() {
            if (RT_PRIO_LOADS) __builtin_amdgcn_s_setprio(2);   // the wave about to issue its node loads goes first
            if (!g_hits) {  // sp > 0 here (checked at the end of the previous iteration)
                --sp;
                const uint32_t ent = (uint32_t)stack[sp * kBlock];
                g_base = ent >> 9;
                g_flip = (ent >> 8) & 1u;
                g_hits = ent & 0xffu;
            }
#if RT_NEAREST_FIRST
            const int r = g_near >= 0 ? g_near : (g_flip ? highest_bit(g_hits) : lowest_bit(g_hits));
            g_near = -1;
#else
            const int r = g_flip ? highest_bit(g_hits) : lowest_bit(g_hits);
#endif
            g_hits &= ~(1u << r);
            if (g_hits) {
                if (sp < kStackSize) {
                    stack[sp * kBlock] = (int)pack_group(g_base, g_flip, g_hits);
                    ++sp;
                } else {
                    overflow = true;
                }
            }
            if (COUNT) tc.nodes++;
            const uint32_t ni = g_base + (uint32_t)r;
            NodeWords w;
            if (ni < n_top) {
                const uint4* l = lds_top + 5 * ni;
                w.h0 = __builtin_bit_cast(float4, l[0]);
                w.h1 = l[1];
                w.qx = l[2];
                w.qy = l[3];
                w.qz = l[4];
            } else {
                w = load_node8(S.nodes8, ni);
            }
            if (RT_PRIO_LOADS) __builtin_amdgcn_s_setprio(0);
#if RT_NEAREST_FIRST
            test_node8_words(w, R, 0.0f, best, g_hits, t_mask, t_valid, g_base, t_base, g_flip,
                             (ANY && !RT_NEAREST_ANY) ? nullptr : &g_near);
#else
            test_node8_words(w, R, 0.0f, best, g_hits, t_mask, t_valid, g_base, t_base, g_flip);
#endif
        };
        if (do_tri) tri_step();
#if RT_TRI_THEN_NODE
        // a lane whose triangles ran out in this step takes its next node in the same iteration
        // (the node block is issued anyway for the wave's other lanes)
        if (Q.tri_vote == 0) do_node = !done && t_mask == 0u && (g_hits != 0u || sp > 0);
#endif
        if (do_node && !(do_tri && !RT_TRI_THEN_NODE)) node_step();
#if RT_TRAV_SCHED == 2
        // a second node step for lanes whose node test found no triangles
        if (Q.tri_vote == 0 && !done && t_mask == 0u && (g_hits != 0u || sp > 0)) node_step();
#elif RT_TRAV_SCHED == 3
        // the first triangle step of the leaves the node test just found
        if (Q.tri_vote == 0 && !done && t_mask != 0u) tri_step();
#endif
        if (!done && !t_mask && !g_hits && sp == 0) done = true;
        if (done) {
            active = false;
            if (COUNT && Q.diag) {   // steps-per-ray histogram (log2 bins) of the counting frame
                atomicAdd(&Q.W.counts[kWfDiagSteps + (ANY ? 32 : 0) + (31 - __builtin_clz(steps))], 1u);
                atomicMax(&Q.W.counts[kWfDiagSteps + 64 + (ANY ? 1 : 0)], steps);
            }
            if (ANY) {
                if (!hit_any) {
                    float4 o4 = qin[(size_t)qstride * e];
                    uint32_t pid = __float_as_uint(o4.w);
                    float4 c = qin[(size_t)qstride * e + 2];
                    float4 a = Q.W.p_accum[pid];
                    Q.W.p_accum[pid] = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, 0.0f);
                }
            } else {
                Q.W.hits[e] = make_float4(best, __uint_as_float(best_id), bu / bdet, bv / bdet);
            }
        }
    }
    flush_counters(P, ANY ? 0 : rays, ANY ? rays : 0, 0, tc, COUNT, overflow, true);
}

// ---- finish: run the remaining paths to completion --------------------------------------------------
template <bool COUNT, bool FULL>
__global__ void __launch_bounds__(kBlock) wf_finish(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q, int cur) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    if (cur < 0) cur = (int)__builtin_amdgcn_readfirstlane(Q.W.counts[cslot(kCntFinishQ)]);   // dev_ctl
    // Persistent: every lane runs ONE path segment (closest hit, shade, shadow ray) per iteration
    // and picks up the next remaining path as soon as its own ends, so a wave waits for its
    // slowest segment, not for its slowest path.  Paths come in chunks of 64 from one counter.
    __shared__ int lds_stack[kStackSize * kBlock];
    __shared__ HaltonDim lds_halton[kHaltonLds];
    __shared__ MatRec lds_mat[kMatLds];
    const ShadeTabs halton = load_tabs(S, lds_halton, lds_mat);
    const Uniforms& U = P.U;
    const ShardPrefix cnt = load_prefix(Q.W.counts + cslot(cur * kShards));
    const uint32_t n = cnt.end[kShards - 1];
    if (Q.dev_ctl) stat_add(Q, kStatFinish, 1u);
    if (Q.dev_ctl && n > 0) stat_add(Q, kStatRounds, 1u);
    const float4* qin = Q.W.q[cur];
    int* stack = &lds_stack[threadIdx.x];
    uint32_t* chunk_ctr = Q.W.counts + cslot(kCntChunkFinish);
    constexpr uint32_t kChunk = 64;
    TraceCounters tc{0, 0};
    bool overflow = false;
    uint32_t n_closest = 0, n_shadow = 0;
    f2 zero2;
    zero2.x = 0.0f;
    zero2.y = 0.0f;
    uint32_t wnext = 0, wend = 0;
    bool exhausted = false, active = false;
    uint32_t pid = 0;
    uint4 meta = make_uint4(0, 0, 0, 0);
    PathRegs p;
    p.color = p.accum = mk3(0, 0, 0);
    p.bounce = p.tpass = p.step = 0;
    f3 rayO = mk3(0, 0, 0), rayD = mk3(0, 0, 0);
    // diagnostics (Q.diag, RT_WF_LOG): segments of the longest path, loop iterations and wall
    // time (s_memrealtime, 100 MHz) of the slowest wave
    uint32_t segs = 0, max_segs = 0, iters = 0;
    const uint64_t t_start = Q.diag ? __builtin_amdgcn_s_memrealtime() : 0;
    while (true) {
        unsigned long long idle = __ballot(!active);
        if (wnext >= wend && !exhausted && (__popcll(idle) >= 8 || idle == ~0ull)) {
            uint32_t base = 0;
            if (lane_id() == 0) base = atomicAdd(chunk_ctr, kChunk);
            base = __builtin_amdgcn_readfirstlane(base);
            if (base >= n) {
                exhausted = true;
            } else {
                wnext = base;
                wend = min(base + kChunk, n);
            }
        }
        if (idle != 0ull && wnext < wend) {
            if (!active) {
                const uint32_t g = wnext + mbcnt64(idle);
                if (g < wend) {
                    const uint32_t e = entry_of(cnt, g, Q.seg_cap);
                    const float4 o = qin[2 * (size_t)e], d = qin[2 * (size_t)e + 1];
                    pid = __float_as_uint(o.w);
                    meta = Q.W.p_meta[pid];
                    const float4 c = Q.W.p_color[pid], a = Q.W.p_accum[pid];
                    p.color = mk3(c.x, c.y, c.z);
                    p.accum = mk3(a.x, a.y, a.z);
                    p.bounce = (int)(meta.z & 0xffu);
                    p.tpass = (int)((meta.z >> 8) & 0xffu);
                    p.step = (int)(meta.z >> 16);
                    rayO = ld3(o);
                    rayD = ld3(d);
                    active = true;
                }
            }
            wnext += (uint32_t)__popcll(idle);
        }
        if (__ballot(active) == 0ull) break;
        ++iters;
        if (!active) continue;
        // one segment of the path (:311-774)
        bool ends = true;
        ++segs;
        Hit h;
        n_closest++;
        if (trace8<false, COUNT>(S, rayO, rayD, 0.0f, INFINITY, h, stack, tc, overflow)) {
            const int sample = (int)meta.y;
            StepResult r;
            shade_step<FULL, false>(S, U, halton, (int)meta.w, sample, rayO, rayD, h, p, sample == 0 && p.step == 0, zero2,
                             false, zero2, r);
            write_pixel_outputs(P, meta.x, r, h, FULL);
            if (r.shadow) {
                Hit sh;
                n_shadow++;
                if (!trace8<true, COUNT>(S, r.so, r.sd, 0.0f, r.stmax, sh, stack, tc, overflow))
                    p.accum = p.accum + r.contrib;
            }
            ends = !r.next;
        }
        if (ends) {
            Q.W.p_accum[pid] = make_float4(p.accum.x, p.accum.y, p.accum.z, 0.0f);
            active = false;
            max_segs = max(max_segs, segs);
            segs = 0;
        }
    }
    if (Q.diag) {
        const uint32_t dt = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_start);
        for (int off = 32; off > 0; off >>= 1) max_segs = max(max_segs, (uint32_t)__shfl_xor((int)max_segs, off, 64));
        if (lane_id() == 0) {
            atomicMax(&Q.W.counts[cslot(kCntDiagSegs)], max_segs);
            atomicMax(&Q.W.counts[cslot(kCntDiagIters)], iters);
            atomicMax(&Q.W.counts[cslot(kCntDiagTime)], dt);
            atomicAdd(&Q.W.counts[kWfDiagHist + min(dt / 5000u, 63u)], 1u);
        }
    }
    flush_counters(P, n_closest, n_shadow, 0, tc, COUNT, overflow);
}

// ---- finish, step-interleaved ------------------------------------------------------------------------
// Same work as wf_finish, but every lane advances by ONE traversal step per iteration (one 8-wide
// node or up to two triangles, closest-hit or shadow any-hit), as in wf_trace.  A lane whose
// closest-hit traversal ended waits in kReady; the wave shades all waiting lanes together once
// at least Q.shade_min of them wait (or no lane is traversing), then each continues with its
// shadow ray, its next ray, or the next path of the queue.  A wave therefore costs the sum of its
// own lanes' steps, not the sum over segments of the slowest lane's traversal: the glass paths
// left at the tail (up to ~20 segments) no longer wait for their wave's worst ray every segment.
#ifndef RT_FINISH_REBUILD
#define RT_FINISH_REBUILD 1
#endif
template <bool COUNT, bool FULL, int WAVES>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES)))
wf_finish_step(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q, int cur) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    if (cur < 0) cur = (int)__builtin_amdgcn_readfirstlane(Q.W.counts[cslot(kCntFinishQ)]);   // dev_ctl
    __shared__ int lds_stack[kStackSize * kBlock];
    __shared__ uint4 lds_top[RT_TOP_FINISH * 5];
    __shared__ HaltonDim lds_halton[kHaltonLds];
    __shared__ MatRec lds_mat[kMatLds];
#if RT_FINISH_REBUILD
    __shared__ float lds_sray[6][kBlock];   // each lane's shadow ray (origin, direction)
#endif
    int* stack = &lds_stack[threadIdx.x];
    const uint32_t n_top = (uint32_t)min(S.num_nodes8, RT_TOP_FINISH);
    for (uint32_t i = threadIdx.x; i < n_top * 5; i += kBlock) lds_top[i] = reinterpret_cast<const uint4*>(S.nodes8)[i];
    const ShadeTabs halton = load_tabs(S, lds_halton, lds_mat);   // ends with a block barrier
    const Uniforms& U = P.U;
    const ShardPrefix cnt = load_prefix(Q.W.counts + cslot(cur * kShards));
    const uint32_t n = cnt.end[kShards - 1];
    if (Q.dev_ctl) stat_add(Q, kStatFinish, 1u);
    if (Q.dev_ctl && n > 0) stat_add(Q, kStatRounds, 1u);
    const float4* qin = Q.W.q[cur];
    uint32_t* chunk_ctr = Q.W.counts + cslot(kCntChunkFinish);
    const uint32_t kChunk = (uint32_t)Q.fchunk;   // paths per grab
    constexpr int kIdle = 0, kClosest = 1, kShadow = 2, kReady = 3;
    TraceCounters tc{0, 0};
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
    bool next = false, hit_any = false, draining = false;
    float4* qout = Q.W.q[1 - cur] + 2 * (size_t)(blockIdx.x & (kShards - 1)) * Q.seg_cap;
    uint32_t* qout_cnt = Q.W.counts + cslot((1 - cur) * kShards + (int)(blockIdx.x & (kShards - 1)));
    // traversal
    RaySetup R = ray_setup(mk3(0, 0, 0), mk3(1, 0, 0));
    float best = 0.0f, bu = 0.0f, bv = 0.0f, bdet = 1.0f;   // closest hit: u = bu / bdet, v = bv / bdet
    uint32_t best_id = 0xffffffffu, g_base = 0, g_hits = 0, t_base = 0, t_mask = 0, t_valid = 0;
    bool g_flip = false;
    int sp = 0;
    [[maybe_unused]] int g_near = -1;   // RT_NEAREST_FIRST: rank of the nearest hit child of the last node test
    auto start_trace = [&](f3 o, f3 d, float tmax) {
        R = ray_setup(o, d);
        best = tmax;
        best_id = 0xffffffffu;
        bu = bv = 0.0f;
        bdet = 1.0f;
        g_base = 0;
        g_hits = 1;   // virtual group holding the root
        g_flip = false;
        g_near = -1;
        t_mask = 0;
        sp = 0;
        hit_any = false;
    };
    // diagnostics (Q.diag, RT_WF_LOG): segments of the longest path, loop iterations and wall
    // time (s_memrealtime, 100 MHz) of the slowest wave
    uint32_t segs = 0, max_segs = 0, iters = 0;
    const uint64_t t_start = Q.diag ? __builtin_amdgcn_s_memrealtime() : 0;
    uint64_t t_shade = 0;
    uint32_t n_pass = 0, n_shaded = 0;
    auto end_path = [&]() {
        Q.W.p_accum[pid] = make_float4(p.accum.x, p.accum.y, p.accum.z, 0.0f);
        mode = kIdle;
        max_segs = max(max_segs, segs);
        segs = 0;
    };

    while (true) {
        // ---- refill idle lanes with the next remaining paths (chunks of 64 from one counter)
        const unsigned long long idle = __ballot(mode == kIdle);
        const bool refill = __popcll(idle) >= Q.refill_min || idle == ~0ull;
        if (wnext >= wend && !exhausted && refill) {
            uint32_t base = 0;
            if (lane_id() == 0) base = atomicAdd(chunk_ctr, kChunk);
            base = __builtin_amdgcn_readfirstlane(base);
            if (base >= n) {
                exhausted = true;
            } else {
                wnext = base;
                wend = min(base + kChunk, n);
            }
        }
        if (idle != 0ull && wnext < wend && refill) {
            if (mode == kIdle) {
                const uint32_t g = wnext + mbcnt64(idle);
                if (g < wend) {
                    // Q.prio: the input was reordered (wf_prio: likely-long paths first) into a
                    // flat array of {o, d} pairs
                    const float4* src = Q.prio ? Q.W.sorted + 2 * (size_t)g : qin + 2 * (size_t)entry_of(cnt, g, Q.seg_cap);
                    const float4 o = src[0], d = src[1];
                    pid = __float_as_uint(o.w);
                    meta = Q.W.p_meta[pid];
                    const float4 c = Q.W.p_color[pid], a = Q.W.p_accum[pid];
                    p.color = mk3(c.x, c.y, c.z);
                    p.accum = mk3(a.x, a.y, a.z);
                    p.bounce = (int)(meta.z & 0xffu);
                    p.tpass = (int)((meta.z >> 8) & 0xffu);
                    p.step = (int)(meta.z >> 16);
                    rayO = ld3(o);
                    rayD = ld3(d);
                    start_trace(rayO, rayD, INFINITY);
                    mode = kClosest;
                    n_closest++;
                    segs++;
                }
            }
            wnext += (uint32_t)__popcll(idle);
        }
        if (__ballot(mode != kIdle) == 0ull) break;   // idle everywhere => refill found nothing
        ++iters;

        // ---- drain (Q.drain_min > 0): once the queue is exhausted and fewer than drain_min lanes
        // of this wave are busy, paths at a closest-hit query are handed back as rays of the next
        // round (queue 1 - cur; the query restarts there, so the result is unchanged), lanes in a
        // shadow query finish it first.  The next launch packs the survivors into dense waves
        // instead of this wave running its few long paths alone.
        if (!draining && Q.drain_min > 0 && exhausted && wnext >= wend &&
            __popcll(__ballot(mode != kIdle)) < Q.drain_min)
            draining = true;
        if (draining) {
            const bool spill = mode == kClosest || mode == kReady;
            const unsigned long long sm = __ballot(spill);
            if (sm != 0ull) {
                uint32_t base = 0;
                if (lane_id() == 0) base = atomicAdd(qout_cnt, (uint32_t)__popcll(sm));
                base = __builtin_amdgcn_readfirstlane(base);
                if (spill) {
                    const uint32_t slot = base + mbcnt64(sm);
                    qout[2 * (size_t)slot] = make_float4(rayO.x, rayO.y, rayO.z, __uint_as_float(pid));
                    qout[2 * (size_t)slot + 1] = make_float4(rayD.x, rayD.y, rayD.z, 0.0f);
                    Q.W.p_color[pid] = make_float4(p.color.x, p.color.y, p.color.z, 0.0f);
                    Q.W.p_accum[pid] = make_float4(p.accum.x, p.accum.y, p.accum.z, 0.0f);
                    Q.W.p_meta[pid] = make_uint4(meta.x, meta.y, pack_state(p.bounce, p.tpass, p.step), meta.w);
                    n_closest--;   // traced again (and counted) by the next round
                    mode = kIdle;
                }
            }
            if (__ballot(mode != kIdle) == 0ull) break;
        }

        // ---- one traversal step (closest hit or shadow any-hit)
        if (mode == kClosest || mode == kShadow) {
            const bool any = mode == kShadow;
            bool tdone = false;
            const bool tri_step = t_mask != 0u;
            if (tri_step) {
                // up to two triangles, both fetched before either is tested, tested in mask order
                const int k0 = lowest_bit(t_mask);
                t_mask &= t_mask - 1u;
                const bool two = t_mask != 0u;
                const int k1 = two ? lowest_bit(t_mask) : k0;
                if (two) t_mask &= t_mask - 1u;
                const float4* tp0 = S.tris + 3 * (size_t)tri_slot(t_base, t_valid, k0);
                const float4* tp1 = S.tris + 3 * (size_t)tri_slot(t_base, t_valid, k1);
                const float4 a0 = tp0[0], a1 = tp0[1], a2 = tp0[2];
                float4 b0 = a0, b1 = a1, b2 = a2;   // the second triangle is fetched only by lanes that have one
#if RT_TRI_B_MASKED
                if (two) {
                    b0 = tp1[0];
                    b1 = tp1[1];
                    b2 = tp1[2];
                }
#else
                b0 = tp1[0];
                b1 = tp1[1];
                b2 = tp1[2];
#endif
                if (COUNT) tc.tris += two ? 2u : 1u;
                float t, u, v, dt;
                if (intersect_triangle_vw(R.pre, R.o, ld3(a0), ld3(a1), ld3(a2), 0.0f, best, &t, &u, &v, &dt)) {
                    const uint32_t id = __float_as_uint(a0.w);
                    if (any) {
                        hit_any = true;
                        tdone = true;
                    } else if (t < best || id < best_id) {
                        best = t;
                        best_id = id;
                        bu = u;
                        bdet = dt;
                        bv = v;
                    }
                }
                if (two && !tdone && intersect_triangle_vw(R.pre, R.o, ld3(b0), ld3(b1), ld3(b2), 0.0f, best, &t, &u, &v, &dt)) {
                    const uint32_t id = __float_as_uint(b0.w);
                    if (any) {
                        hit_any = true;
                        tdone = true;
                    } else if (t < best || id < best_id) {
                        best = t;
                        best_id = id;
                        bu = u;
                        bdet = dt;
                        bv = v;
                    }
                }
            }
            // a lane whose triangles ran out in this step takes its next node in the same
            // iteration (RT_TRI_THEN_NODE; the node block is issued anyway for other lanes)
            if (RT_TRI_THEN_NODE ? (!tdone && t_mask == 0u && (g_hits != 0u || sp > 0)) : !tri_step) {
                if (!g_hits) {   // sp > 0 here (checked at the end of the previous step)
                    --sp;
                    const uint32_t ent = (uint32_t)stack[sp * kBlock];
                    g_base = ent >> 9;
                    g_flip = (ent >> 8) & 1u;
                    g_hits = ent & 0xffu;
                }
#if RT_NEAREST_FIRST
                const int r = g_near >= 0 ? g_near : (g_flip ? highest_bit(g_hits) : lowest_bit(g_hits));
                g_near = -1;
#else
                const int r = g_flip ? highest_bit(g_hits) : lowest_bit(g_hits);
#endif
                g_hits &= ~(1u << r);
                if (g_hits) {
                    if (sp < kStackSize) {
                        stack[sp * kBlock] = (int)pack_group(g_base, g_flip, g_hits);
                        ++sp;
                    } else {
                        overflow = true;
                    }
                }
                if (COUNT) tc.nodes++;
                const uint32_t ni = g_base + (uint32_t)r;
                NodeWords w;
                if (ni < n_top) {
                    const uint4* l = lds_top + 5 * ni;
                    w.h0 = __builtin_bit_cast(float4, l[0]);
                    w.h1 = l[1];
                    w.qx = l[2];
                    w.qy = l[3];
                    w.qz = l[4];
                } else {
                    w = load_node8(S.nodes8, ni);
                }
#if RT_NEAREST_FIRST
                test_node8_words(w, R, 0.0f, best, g_hits, t_mask, t_valid, g_base, t_base, g_flip, &g_near);
#else
                test_node8_words(w, R, 0.0f, best, g_hits, t_mask, t_valid, g_base, t_base, g_flip);
#endif
            }
            if (!tdone && !t_mask && !g_hits && sp == 0) tdone = true;
            if (tdone) {
                if (any) {   // shadow ray done: unoccluded -> add its contribution (:741-743)
                    if (!hit_any) p.accum = p.accum + contrib;
                    if (next) {
                        start_trace(rayO, rayD, INFINITY);
                        mode = kClosest;
                        n_closest++;
                        segs++;
                    } else {
                        end_path();
                    }
                } else if (best_id == 0xffffffffu) {   // miss -> path ends (:321-322)
                    end_path();
                } else {
                    mode = kReady;
                }
            }
        }

        // ---- shade the waiting lanes together (:324-774)
        const unsigned long long ready = __ballot(mode == kReady);
        if (ready != 0ull &&
            (__popcll(ready) >= Q.shade_min || __ballot(mode == kClosest || mode == kShadow) == 0ull)) {
            const uint64_t ts0 = Q.diag ? __builtin_amdgcn_s_memrealtime() : 0;
            if (Q.diag) {
                ++n_pass;
                n_shaded += (uint32_t)__popcll(ready);
            }
            if (mode == kReady) {
                Hit h;
                h.t = best;
                h.id = best_id;
                h.u = bu / bdet;
                h.v = bv / bdet;
                const int sample = (int)meta.y;
                StepResult r;
                shade_step<FULL, false>(S, U, halton, (int)meta.w, sample, rayO, rayD, h, p, sample == 0 && p.step == 0,
                                 zero2, false, zero2, r);
                write_pixel_outputs(P, meta.x, r, h, FULL);
                next = r.next;
                if (r.shadow) {
                    contrib = r.contrib;
                    start_trace(r.so, r.sd, r.stmax);
#if RT_FINISH_REBUILD
                    lds_sray[0][threadIdx.x] = r.so.x;
                    lds_sray[1][threadIdx.x] = r.so.y;
                    lds_sray[2][threadIdx.x] = r.so.z;
                    lds_sray[3][threadIdx.x] = r.sd.x;
                    lds_sray[4][threadIdx.x] = r.sd.y;
                    lds_sray[5][threadIdx.x] = r.sd.z;
#endif
                    mode = kShadow;
                    n_shadow++;
                } else if (r.next) {
                    start_trace(rayO, rayD, INFINITY);
                    mode = kClosest;
                    n_closest++;
                    segs++;
                } else {
                    end_path();
                }
            }
#if RT_FINISH_REBUILD
            // Every lane's ray setup is rebuilt from its ray (a pure function of it, so bit for bit
            // the one start_trace made): the ~19 registers of the traversing lanes' setups are
            // then dead while the shading code runs, which sets the kernel's register peak.
            if (mode == kShadow) {
                R = ray_setup(mk3(lds_sray[0][threadIdx.x], lds_sray[1][threadIdx.x], lds_sray[2][threadIdx.x]),
                              mk3(lds_sray[3][threadIdx.x], lds_sray[4][threadIdx.x], lds_sray[5][threadIdx.x]));
            } else {
                R = ray_setup(rayO, rayD);
            }
#endif
            if (Q.diag) t_shade += __builtin_amdgcn_s_memrealtime() - ts0;
        }
    }
    if (Q.diag) {
        const uint32_t dt = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_start);
        if (lane_id() == 0) {
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
    flush_counters(P, n_closest, n_shadow, 0, tc, COUNT, overflow);
}

// ---- finish input order: likely-long paths first ---------------------------------------------------
// The finish launch lasts as long as its longest remaining paths: ~20 segments of glass paths
// whose queries run inside the dragon.  Handing those out first lets their serial chains run
// while the rest of the work fills the machine around them.  A path that is inside (or passing
// through) glass has transparencyPasses > 0 (:561-572).  Two-way partition of the queue into a
// flat array: such paths from the front, the others from the back.
__global__ void __launch_bounds__(kBlock) wf_prio(WfParams Q, int cur) {
    __shared__ BlockAlloc ba_hi, ba_lo;
    if (cur < 0) cur = (int)__builtin_amdgcn_readfirstlane(Q.W.counts[cslot(kCntFinishQ)]);
    const ShardPrefix cnt = load_prefix(Q.W.counts + cslot(cur * kShards));
    const uint32_t n = cnt.end[kShards - 1];
    const float4* qin = Q.W.q[cur];
    for (uint32_t base = blockIdx.x * kBlock; base < n; base += gridDim.x * kBlock) {
        const uint32_t g = base + threadIdx.x;
        float4 o = make_float4(0, 0, 0, 0), d = o;
        bool hi = false, lo = false;
        if (g < n) {
            const uint32_t e = entry_of(cnt, g, Q.seg_cap);
            o = qin[2 * (size_t)e];
            d = qin[2 * (size_t)e + 1];
            const uint32_t pid = __float_as_uint(o.w);
            hi = ((Q.W.p_meta[pid].z >> 8) & 0xffu) != 0u;
            lo = !hi;
        }
        const uint32_t a = block_alloc(hi, &Q.W.counts[cslot(kCntPrioHi)], ba_hi);
        const uint32_t b = block_alloc(lo, &Q.W.counts[cslot(kCntPrioLo)], ba_lo);
        if (hi || lo) {
            const uint32_t slot = hi ? a : n - 1 - b;
            Q.W.sorted[2 * (size_t)slot] = o;
            Q.W.sorted[2 * (size_t)slot + 1] = d;
        }
    }
}

// ---- finish with wave-local queues -------------------------------------------------------------------
// The step-interleaved finish kernel shades ready lanes at partial masks while the others idle or
// traverse; its VALU lane utilisation is ~19 %.  Here a lane never waits to be shaded: a lane
// whose closest-hit query found a hit pushes (path id, hit) onto its wave's hit queue in LDS and
// takes new work at once.  Once 64 hits are queued (or nothing else is left to do) all 64 lanes
// shade one queued hit each at full width, whatever their own traversal state, and push the
// path's shadow ray or continuation onto the wave's ray queue (path id only; the ray itself goes
// to per-path global slots).  Idle lanes refill from the ray queue first, then from the global
// path queue.  Per-path order is the reference's: emission (shade), shadow contribution (its
// query), then the next segment, so the image is bit-identical.
struct TravState {
    RaySetup R;
    float best, bu, bv;
    uint32_t best_id, g_base, g_hits, t_base, t_mask, t_valid;
    bool g_flip, hit_any;
    int sp;
};

__device__ __forceinline__ void trav_start(TravState& T, f3 o, f3 d, float tmax) {
    T.R = ray_setup(o, d);
    T.best = tmax;
    T.best_id = 0xffffffffu;
    T.bu = T.bv = 0.0f;
    T.g_base = 0;
    T.g_hits = 1;   // virtual group holding the root
    T.g_flip = false;
    T.t_mask = 0;
    T.sp = 0;
    T.hit_any = false;
}

// one traversal step (one 8-wide node or up to two triangles); true once the query is finished
template <bool COUNT>
__device__ __forceinline__ bool trav_step(const DevScene& S, TravState& T, bool any, int* stack, const uint4* lds_top,
                                          uint32_t n_top, TraceCounters& tc, bool& overflow) {
    bool tdone = false;
    if (T.t_mask) {
        const int k0 = lowest_bit(T.t_mask);
        T.t_mask &= T.t_mask - 1u;
        const bool two = T.t_mask != 0u;
        const int k1 = two ? lowest_bit(T.t_mask) : k0;
        if (two) T.t_mask &= T.t_mask - 1u;
        const float4* tp0 = S.tris + 3 * (size_t)tri_slot(T.t_base, T.t_valid, k0);
        const float4* tp1 = S.tris + 3 * (size_t)tri_slot(T.t_base, T.t_valid, k1);
        const float4 a0 = tp0[0], a1 = tp0[1], a2 = tp0[2];
        float4 b0 = a0, b1 = a1, b2 = a2;   // the second triangle is fetched only by lanes that have one
#if RT_TRI_B_MASKED
        if (two) {
            b0 = tp1[0];
            b1 = tp1[1];
            b2 = tp1[2];
        }
#else
        b0 = tp1[0];
        b1 = tp1[1];
        b2 = tp1[2];
#endif
        if (COUNT) tc.tris += two ? 2u : 1u;
        float t, u, v;
        if (intersect_triangle(T.R.pre, T.R.o, ld3(a0), ld3(a1), ld3(a2), 0.0f, T.best, &t, &u, &v)) {
            const uint32_t id = __float_as_uint(a0.w);
            if (any) {
                T.hit_any = true;
                tdone = true;
            } else if (t < T.best || id < T.best_id) {
                T.best = t;
                T.best_id = id;
                T.bu = u;
                T.bv = v;
            }
        }
        if (two && !tdone && intersect_triangle(T.R.pre, T.R.o, ld3(b0), ld3(b1), ld3(b2), 0.0f, T.best, &t, &u, &v)) {
            const uint32_t id = __float_as_uint(b0.w);
            if (any) {
                T.hit_any = true;
                tdone = true;
            } else if (t < T.best || id < T.best_id) {
                T.best = t;
                T.best_id = id;
                T.bu = u;
                T.bv = v;
            }
        }
    } else {
        if (!T.g_hits) {   // sp > 0 here (checked at the end of the previous step)
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
        if (COUNT) tc.nodes++;
        const uint32_t ni = T.g_base + (uint32_t)r;
        NodeWords w;
        if (ni < n_top) {
            const uint4* l = lds_top + 5 * ni;
            w.h0 = __builtin_bit_cast(float4, l[0]);
            w.h1 = l[1];
            w.qx = l[2];
            w.qy = l[3];
            w.qz = l[4];
        } else {
            w = load_node8(S.nodes8, ni);
        }
        test_node8_words(w, T.R, 0.0f, T.best, T.g_hits, T.t_mask, T.t_valid, T.g_base, T.t_base, T.g_flip);
    }
    return tdone || (!T.t_mask && !T.g_hits && T.sp == 0);
}

constexpr int kWaveQ = 128;   // hit / ray queue entries per wave (LDS)

template <bool COUNT, bool FULL>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4, 4)))
wf_finish_q(DevScene S, const FrameParams* __restrict__ Pp, WfParams Q, int cur) {
    const FrameParams& P = *Pp;   // per-frame parameters in device memory
    if (cur < 0) cur = (int)__builtin_amdgcn_readfirstlane(Q.W.counts[cslot(kCntFinishQ)]);   // dev_ctl
    __shared__ int lds_stack[kStackSize * kBlock];
    __shared__ uint4 lds_top[kTopNodes * 5];
    __shared__ HaltonDim lds_halton[kHaltonLds];
    __shared__ MatRec lds_mat[kMatLds];
    __shared__ float4 lds_hq_hit[kBlock / 64][kWaveQ];   // (t, triangle id bits, u, v)
    __shared__ uint32_t lds_hq_pid[kBlock / 64][kWaveQ];
    __shared__ uint32_t lds_rq[kBlock / 64][kWaveQ];     // path id | 0x80000000 for a shadow query
    int* stack = &lds_stack[threadIdx.x];
    const int wave = threadIdx.x >> 6;
    const uint32_t lane = lane_id();
    const uint32_t n_top = (uint32_t)min(S.num_nodes8, kTopNodes);
    for (uint32_t i = threadIdx.x; i < n_top * 5; i += kBlock) lds_top[i] = reinterpret_cast<const uint4*>(S.nodes8)[i];
    const ShadeTabs halton = load_tabs(S, lds_halton, lds_mat);   // ends with a block barrier
    const Uniforms& U = P.U;
    const ShardPrefix cnt = load_prefix(Q.W.counts + cslot(cur * kShards));
    const uint32_t n = cnt.end[kShards - 1];
    if (Q.dev_ctl) stat_add(Q, kStatFinish, 1u);
    if (Q.dev_ctl && n > 0) stat_add(Q, kStatRounds, 1u);
    const float4* qin = Q.W.q[cur];
    float4* const p_ray = Q.W.p_ray;     // 2 per path: next closest ray (o, d)
    float4* const p_sray = Q.W.p_sray;   // 3 per path: shadow ray (o; d, tmax; contribution, next)
    uint32_t* chunk_ctr = Q.W.counts + cslot(kCntChunkFinish);
    constexpr uint32_t kChunk = 64;
    constexpr int kIdle = 0, kClosest = 1, kShadow = 2, kHit = 3;   // kHit: a hit waiting for queue space
    TraceCounters tc{0, 0};
    bool overflow = false;
    uint32_t n_closest = 0, n_shadow = 0;
    f2 zero2;
    zero2.x = 0.0f;
    zero2.y = 0.0f;
    uint32_t wnext = 0, wend = 0, hq_n = 0, rq_n = 0;   // wave-uniform
    bool exhausted = false;
    int mode = kIdle;
    uint32_t pid = 0;
    TravState T;
    trav_start(T, mk3(0, 0, 0), mk3(1, 0, 0), 0.0f);

    while (true) {
        // ---- refill idle lanes: queued shadow / continuation rays first, then new paths
        unsigned long long idle = __ballot(mode == kIdle);
        if (idle != 0ull && (__popcll(idle) >= Q.refill_min || idle == ~0ull || rq_n > 0)) {
            const uint32_t take = min((uint32_t)__popcll(idle), rq_n);
            if (take > 0) {
                if (mode == kIdle) {
                    const uint32_t k = mbcnt64(idle);
                    if (k < take) {
                        const uint32_t e = lds_rq[wave][rq_n - 1 - k];
                        pid = e & 0x7fffffffu;
                        if (e >> 31) {
                            const float4 so = p_sray[3 * (size_t)pid], sd = p_sray[3 * (size_t)pid + 1];
                            trav_start(T, ld3(so), ld3(sd), sd.w);
                            mode = kShadow;
                            n_shadow++;
                        } else {
                            const float4 o = p_ray[2 * (size_t)pid], d = p_ray[2 * (size_t)pid + 1];
                            trav_start(T, ld3(o), ld3(d), INFINITY);
                            mode = kClosest;
                            n_closest++;
                        }
                    }
                }
                rq_n -= take;
                idle = __ballot(mode == kIdle);
            }
            const bool refill = idle != 0ull && (__popcll(idle) >= Q.refill_min || idle == ~0ull);
            if (wnext >= wend && !exhausted && refill) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(chunk_ctr, kChunk);
                base = __builtin_amdgcn_readfirstlane(base);
                if (base >= n) {
                    exhausted = true;
                } else {
                    wnext = base;
                    wend = min(base + kChunk, n);
                }
            }
            if (refill && wnext < wend) {
                if (mode == kIdle) {
                    const uint32_t g = wnext + mbcnt64(idle);
                    if (g < wend) {
                        const uint32_t e = entry_of(cnt, g, Q.seg_cap);
                        const float4 o = qin[2 * (size_t)e], d = qin[2 * (size_t)e + 1];
                        pid = __float_as_uint(o.w);
                        p_ray[2 * (size_t)pid] = o;   // the shading reads the segment's ray from here
                        p_ray[2 * (size_t)pid + 1] = d;
                        trav_start(T, ld3(o), ld3(d), INFINITY);
                        mode = kClosest;
                        n_closest++;
                    }
                }
                wnext += (uint32_t)__popcll(idle);
            }
        }
        const unsigned long long busy = __ballot(mode == kClosest || mode == kShadow);
        if (busy == 0ull && hq_n == 0 && rq_n == 0 && __ballot(mode == kHit) == 0ull && exhausted && wnext >= wend)
            break;

        // ---- one traversal step
        if (mode == kClosest || mode == kShadow) {
            const bool any = mode == kShadow;
            if (trav_step<COUNT>(S, T, any, stack, lds_top, n_top, tc, overflow)) {
                if (any) {   // shadow query done: unoccluded -> add its contribution (:741-743)
                    const float4 c = p_sray[3 * (size_t)pid + 2];
                    if (!T.hit_any) {
                        const float4 a = Q.W.p_accum[pid];
                        Q.W.p_accum[pid] = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, 0.0f);
                    }
                    if (c.w != 0.0f) {   // the path continues: its next ray was stored by the shading
                        const float4 o = p_ray[2 * (size_t)pid], d = p_ray[2 * (size_t)pid + 1];
                        trav_start(T, ld3(o), ld3(d), INFINITY);
                        mode = kClosest;
                        n_closest++;
                    } else {
                        mode = kIdle;
                    }
                } else {
                    mode = T.best_id == 0xffffffffu ? kIdle : kHit;   // miss -> path ends (:321-322)
                }
            }
        }

        // ---- queue the hits (lanes that find no space keep theirs and retry)
        {
            const unsigned long long hm = __ballot(mode == kHit);
            if (hm != 0ull) {
                const uint32_t pos = hq_n + mbcnt64(hm);
                if (mode == kHit && pos < (uint32_t)kWaveQ) {
                    lds_hq_hit[wave][pos] = make_float4(T.best, __uint_as_float(T.best_id), T.bu, T.bv);
                    lds_hq_pid[wave][pos] = pid;
                    mode = kIdle;
                }
                hq_n = min(hq_n + (uint32_t)__popcll(hm), (uint32_t)kWaveQ);
            }
        }

        // ---- shade 64 queued hits at full width (fewer once nothing else is left)
        const bool starving = exhausted && wnext >= wend && rq_n == 0;
        const uint32_t m = min(hq_n, 64u);
        if (m > 0 && rq_n + m <= (uint32_t)kWaveQ &&
            (m == 64u || __ballot(mode == kClosest || mode == kShadow) == 0ull ||
             (starving && __popcll(__ballot(mode == kIdle)) >= Q.shade_min))) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // ray / path stores of this wave
            uint32_t push = 0;   // this lane's ray-queue entry + 1 (0: none)
            if (lane < m) {
                const uint32_t slot = hq_n - m + lane;
                const uint32_t spid = lds_hq_pid[wave][slot];
                const float4 hv = lds_hq_hit[wave][slot];
                Hit h;
                h.t = hv.x;
                h.id = __float_as_uint(hv.y);
                h.u = hv.z;
                h.v = hv.w;
                const uint4 meta = Q.W.p_meta[spid];
                const float4 pc = Q.W.p_color[spid], pa = Q.W.p_accum[spid];
                const float4 o = p_ray[2 * (size_t)spid], d = p_ray[2 * (size_t)spid + 1];
                PathRegs pr;
                pr.color = mk3(pc.x, pc.y, pc.z);
                pr.accum = mk3(pa.x, pa.y, pa.z);
                pr.bounce = (int)(meta.z & 0xffu);
                pr.tpass = (int)((meta.z >> 8) & 0xffu);
                pr.step = (int)(meta.z >> 16);
                f3 rayO = ld3(o), rayD = ld3(d);
                const int sample = (int)meta.y;
                StepResult r;
                shade_step<FULL, false>(S, U, halton, (int)meta.w, sample, rayO, rayD, h, pr, sample == 0 && pr.step == 0,
                                 zero2, false, zero2, r);
                write_pixel_outputs(P, meta.x, r, h, FULL);
                Q.W.p_accum[spid] = make_float4(pr.accum.x, pr.accum.y, pr.accum.z, 0.0f);
                if (r.next) {
                    Q.W.p_color[spid] = make_float4(pr.color.x, pr.color.y, pr.color.z, 0.0f);
                    Q.W.p_meta[spid] = make_uint4(meta.x, meta.y, pack_state(pr.bounce, pr.tpass, pr.step), meta.w);
                    p_ray[2 * (size_t)spid] = make_float4(rayO.x, rayO.y, rayO.z, 0.0f);
                    p_ray[2 * (size_t)spid + 1] = make_float4(rayD.x, rayD.y, rayD.z, 0.0f);
                }
                if (r.shadow) {
                    p_sray[3 * (size_t)spid] = make_float4(r.so.x, r.so.y, r.so.z, 0.0f);
                    p_sray[3 * (size_t)spid + 1] = make_float4(r.sd.x, r.sd.y, r.sd.z, r.stmax);
                    p_sray[3 * (size_t)spid + 2] = make_float4(r.contrib.x, r.contrib.y, r.contrib.z, r.next ? 1.0f : 0.0f);
                    push = (spid | 0x80000000u) + 1u;
                } else if (r.next) {
                    push = spid + 1u;
                }
            }
            hq_n -= m;
            const unsigned long long pm = __ballot(push != 0u);
            if (push != 0u) lds_rq[wave][rq_n + mbcnt64(pm)] = push - 1u;
            rq_n += (uint32_t)__popcll(pm);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // before another lane loads them
        }
    }
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
        own_pixel(P, i, px, py);
        if (px < U.width && py < U.height) {
            pix = (uint32_t)py * (uint32_t)U.width + (uint32_t)px;
            float2 mv2 = P.motion[pix], pm2 = Q.W.motion_prev[pix];
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
    TraceCounters tc{0, 0};
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
    own_pixel(P, i, px, py);
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
    own_pixel(P, i, px, py);
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
    float2 mv2 = P.motion[pix], pm2 = Q.W.motion_prev[pix];
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

#define WF_CHECK(expr)                    \
    do {                                  \
        hipError_t e_ = (expr);           \
        if (e_ != hipSuccess) {           \
            *err = hipGetErrorString(e_); \
            return false;                 \
        }                                 \
    } while (0)

// resident blocks of the persistent traversal kernel (CUs x blocks per CU), queried once
static unsigned trace_grid_cap() {
    static unsigned cap = 0;
    if (!cap) {
        int dev = 0, cus = 256, per = 0;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, wf_trace<false, false>, kBlock, 0) != hipSuccess || per < 1)
            per = 4;
        cap = (unsigned)(cus * per);
    }
    return cap;
}

// resident blocks (CUs x blocks per CU) of a persistent kernel
template <typename K>
static unsigned resident_grid(K kernel, int fallback_per_cu) {
    int dev = 0, cus = 256, per = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, kBlock, 0) != hipSuccess || per < 1)
        per = fallback_per_cu;
    return (unsigned)(cus * per);
}

// the finish launch: step-interleaved (STEP, default) or per-segment kernel, grid = resident blocks
template <bool STEP, bool COUNT, bool FULL>
static void launch_finish(const DevScene& S, const FrameParams& P, const WfParams& Q, int cur, uint32_t n,
                          hipStream_t stream) {
    static const int waves = env_int("RT_FINISH_WAVES", 4);
    // Q.finish_frac < 100: the finish kernel takes that share of the resident grid, the rest of
    // the machine stays free for the next frame's kernels (frames in flight)
    if (STEP && Q.finish_frac < 100 && waves == 5) {
        static const unsigned full_cap = resident_grid(wf_finish_step<COUNT, FULL, 5>, 2);
        const unsigned cap = std::max(1u, full_cap * (unsigned)Q.finish_frac / 100u);
        hipLaunchKernelGGL((wf_finish_step<COUNT, FULL, 5>), dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
    } else if (STEP && waves == 5) {
        static const unsigned cap = resident_grid(wf_finish_step<COUNT, FULL, 5>, 2);
        hipLaunchKernelGGL((wf_finish_step<COUNT, FULL, 5>), dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
    } else if (STEP && Q.finish_frac < 100 && waves == 3) {
        static const unsigned full_cap = resident_grid(wf_finish_step<COUNT, FULL, 3>, 2);
        const unsigned cap = std::max(1u, full_cap * (unsigned)Q.finish_frac / 100u);
        hipLaunchKernelGGL((wf_finish_step<COUNT, FULL, 3>), dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
    } else if (STEP && Q.finish_frac < 100) {
        static const unsigned full_cap = resident_grid(wf_finish_step<COUNT, FULL, 4>, 2);
        const unsigned cap = std::max(1u, full_cap * (unsigned)Q.finish_frac / 100u);
        hipLaunchKernelGGL((wf_finish_step<COUNT, FULL, 4>), dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
    } else if (STEP && waves == 3) {
        static const unsigned cap = resident_grid(wf_finish_step<COUNT, FULL, 3>, 2);
        hipLaunchKernelGGL((wf_finish_step<COUNT, FULL, 3>), dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
    } else if (STEP) {
        static const unsigned cap = resident_grid(wf_finish_step<COUNT, FULL, 4>, 2);
        hipLaunchKernelGGL((wf_finish_step<COUNT, FULL, 4>), dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
    } else {
        static const unsigned cap = resident_grid(wf_finish<COUNT, FULL>, 2);
        hipLaunchKernelGGL((wf_finish<COUNT, FULL>), dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
    }
}

template <bool COUNT, bool FULL>
static void launch_finish_q(const WfParams& Q, const DevScene& S, int cur, uint32_t n, hipStream_t stream) {
    static const unsigned cap = resident_grid(wf_finish_q<COUNT, FULL>, 2);
    hipLaunchKernelGGL((wf_finish_q<COUNT, FULL>), dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
}

static void launch_finish_any(const DevScene& S, const FrameParams& P, const WfParams& Q, bool count, bool full, int cur,
                              uint32_t n, hipStream_t stream) {
    if (Q.prio) {
        (void)hipMemsetAsync(Q.W.counts + cslot(kCntPrioHi), 0, cslot(2) * sizeof(uint32_t), stream);
        hipLaunchKernelGGL(wf_prio, dim3(grid_for(n, 4096)), dim3(kBlock), 0, stream, Q, cur);
    }
    if (Q.finish_step == 2) {
        if (count) full ? launch_finish_q<true, true>(Q, S, cur, n, stream) : launch_finish_q<true, false>(Q, S, cur, n, stream);
        else full ? launch_finish_q<false, true>(Q, S, cur, n, stream) : launch_finish_q<false, false>(Q, S, cur, n, stream);
    } else if (Q.finish_step) {
        if (count) full ? launch_finish<true, true, true>(S, P, Q, cur, n, stream)
                        : launch_finish<true, true, false>(S, P, Q, cur, n, stream);
        else full ? launch_finish<true, false, true>(S, P, Q, cur, n, stream)
                  : launch_finish<true, false, false>(S, P, Q, cur, n, stream);
    } else {
        if (count) full ? launch_finish<false, true, true>(S, P, Q, cur, n, stream)
                        : launch_finish<false, true, false>(S, P, Q, cur, n, stream);
        else full ? launch_finish<false, false, true>(S, P, Q, cur, n, stream)
                  : launch_finish<false, false, false>(S, P, Q, cur, n, stream);
    }
}

static uint32_t queue_total(const uint32_t* h, int q) {
    uint32_t s = 0;
    for (int k = 0; k < kShards; ++k) s += h[cslot(q * kShards + k)];
    return s;
}

// Diagnostics (RT_WF_DUMP=<prefix>): the ray queue of every extend round written to
// <prefix>_it<k>.bin as n x 8 floats (o.xyz, path id bits, d.xyz, 0), dense order.
static void dump_queue(const WfParams& Q, int cur, int it, hipStream_t stream) {
    static const char* prefix = getenv("RT_WF_DUMP");
    if (!prefix) return;
    char name[512];
    snprintf(name, sizeof name, "%s_it%02d.bin", prefix, it);
    FILE* f = fopen(name, "wb");
    if (!f) return;
    std::vector<float4> buf;
    for (int k = 0; k < kShards; ++k) {
        const uint32_t c = Q.W.h_counts[cslot(cur * kShards + k)];
        buf.resize(2 * (size_t)c);
        if (c && hipMemcpyAsync(buf.data(), Q.W.q[cur] + 2 * (size_t)k * Q.seg_cap, 32 * (size_t)c,
                                hipMemcpyDeviceToHost, stream) == hipSuccess &&
            hipStreamSynchronize(stream) == hipSuccess)
            fwrite(buf.data(), 32, c, f);
    }
    fclose(f);
}

static bool iterate(const DevScene& S, const FrameParams& P, WfParams& Q, int& cur, uint32_t n, bool count, bool full,
                    hipStream_t stream, WfFrameStats* fs, const char** err) {
    float* stage_ms = fs->stage_ms;
    const int max_it = P.U.maxBounces * (P.U.maxBounces + 1) + 2;
    WavefrontBuffers& W = Q.W;
    for (int it = 0; it < max_it && n > 0; ++it) {
        if (n < Q.tail) {
            // run the tail in persistent finish launches; with draining (wf_finish_step), each
            // round hands the paths still alive at its end to the next round in queue 1 - cur
            // Small rounds run to completion (no drain): a few paths in one wave would otherwise be
            // handed on round after round; the round count is capped as well.
            const int drain_min = Q.drain_min;
            for (int round = 0; n > 0; ++round) {
                Q.drain_min = (n >= drain_paths() && round < 32) ? drain_min : 0;
                WF_CHECK(hipEventRecord(W.ev[0], stream));
                WF_CHECK(hipMemsetAsync(W.counts + cslot(kCntChunkFinish), 0, sizeof(uint32_t), stream));
                for (int k = 0; k < kShards; ++k)
                    WF_CHECK(hipMemsetAsync(W.counts + cslot((1 - cur) * kShards + k), 0, sizeof(uint32_t), stream));
                if (wf_log()) WF_CHECK(hipMemsetAsync(W.counts + kWfDiagHist, 0, 64 * sizeof(uint32_t), stream));
                launch_finish_any(S, P, Q, count, full, cur, n, stream);
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
                const uint32_t n_next = Q.drain_min > 0 ? queue_total(W.h_counts, 1 - cur) : 0u;
                if (wf_log()) {
                    fprintf(stderr, "[wf] it %d finish paths %u -> %u handed on  %.3f ms; longest path %u segments, "
                            "slowest wave %u iterations in %.3f ms\n", it, n, n_next, a,
                            W.h_counts[cslot(kCntDiagSegs)], W.h_counts[cslot(kCntDiagIters)],
                            W.h_counts[cslot(kCntDiagTime)] * 1e-5);
                    {
                        const double st = W.h_counts[kWfStat + kStatDiagShadeT], tt = W.h_counts[kWfStat + kStatDiagTotalT];
                        const double np = W.h_counts[kWfStat + kStatDiagPasses], ns = W.h_counts[kWfStat + kStatDiagShaded];
                        fprintf(stderr, "[wf] finish: %.1f %% of wave time in shading passes, %.0f passes, %.1f lanes per pass\n",
                                tt > 0 ? 100.0 * st / tt : 0.0, np, np > 0 ? ns / np : 0.0);
                    }
                    fprintf(stderr, "[wf] finish wave end times (50 us bins):");
                    for (int b = 0; b < 64; ++b)
                        if (W.h_counts[kWfDiagHist + b]) fprintf(stderr, " %d:%u", b, W.h_counts[kWfDiagHist + b]);
                    fprintf(stderr, "\n");
                }
                n = n_next;
                cur = 1 - cur;
                ++it;
            }
            Q.drain_min = drain_min;
            return true;
        }
        int next = 1 - cur;
        dump_queue(Q, cur, fs->iterations, stream);
        WF_CHECK(hipEventRecord(W.ev[0], stream));
        unsigned g = grid_for(n, 8192);
        unsigned gt = grid_for(n, trace_grid_cap());
        if (count) hipLaunchKernelGGL((wf_trace<false, true>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        else hipLaunchKernelGGL((wf_trace<false, false>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
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
        if (count) hipLaunchKernelGGL((wf_trace<true, true>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        else hipLaunchKernelGGL((wf_trace<true, false>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
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
        if (wf_log()) {
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
struct Enqueue {
    WfTimeline& T;
    hipStream_t stream;
    int last = -1;
    bool mark(const char** err) {
        if (T.n_ev >= WfTimeline::kMaxEv) {
            *err = "wavefront timeline: too many events";
            return false;
        }
        const hipError_t e = hipEventRecord(T.ev[T.n_ev], stream);
        if (e != hipSuccess) {
            *err = hipGetErrorString(e);
            return false;
        }
        last = T.n_ev++;
        return true;
    }
    // closes the span [previous mark, now) as `stage`
    bool span(int stage, const char** err) {
        const int a = last;
        if (!mark(err)) return false;
        T.spans[T.n_spans++] = WfTimeline::Span{stage, a, last};
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
                         Enqueue& E, const char** err) {
    hipStream_t stream = E.stream;
    const unsigned gt = trace_grid_cap(), g = 8192;
    for (int k = 0; k < rounds; ++k) {
        const int cur = k & 1;
        if (count) hipLaunchKernelGGL((wf_trace<false, true>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        else hipLaunchKernelGGL((wf_trace<false, false>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        if (!E.span(1, err)) return false;
        if (Q.sort_bins) {
            hipLaunchKernelGGL(wf_sort_hist, dim3(kSortBlocks), dim3(kSortThreads), 0, stream, S, Q, cur);
            hipLaunchKernelGGL(wf_sort_rowscan, dim3(Q.sort_bins), dim3(kSortBlocks), 0, stream, Q);
            hipLaunchKernelGGL(wf_sort_scatter, dim3(kSortBlocks), dim3(kSortThreads), 0, stream, S, Q, cur);
            if (!E.span(6, err)) return false;
        }
        if (full) {
            if (Q.sort_bins) hipLaunchKernelGGL((wf_shade<true, true>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
            else hipLaunchKernelGGL((wf_shade<true, false>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        } else {
            if (Q.sort_bins) hipLaunchKernelGGL((wf_shade<false, true>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
            else hipLaunchKernelGGL((wf_shade<false, false>), dim3(g), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        }
        if (!E.span(2, err)) return false;
        if (count) hipLaunchKernelGGL((wf_trace<true, true>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        else hipLaunchKernelGGL((wf_trace<true, false>), dim3(gt), dim3(kBlock), 0, stream, S, Q.Pd, Q, cur);
        if (!E.span(3, err)) return false;
    }
    // the finish chunk counter is zero here: the frame start clears every counter and the
    // extra-sample pass clears it again before its own finish launch
    launch_finish_any(S, P, Q, count, full, -1, 1u << 30, stream);   // resident grid; input queue from the counters
    WF_CHECK(hipGetLastError());
    return E.span(5, err);
}

// Issues one frame on `stream`.  Launch arguments come from S, Q and the buffer pointers in P;
// the per-frame values of P are read by the kernels from Q.Pd.
static bool record_frame(const DevScene& S, const FrameParams& P, WfParams& Q, bool count, bool full, int maxExtra,
                         bool with_extra, hipStream_t stream, hipEvent_t prev_done, WfTimeline& T, const char** err) {
    WavefrontBuffers& W = Q.W;
    T.n_ev = T.n_spans = 0;
    Enqueue E{T, stream};
    if (!E.mark(err)) return false;
    WF_CHECK(hipMemsetAsync(W.counts, 0, kWfCountWords * sizeof(uint32_t), stream));
    const int rounds = rounds_for(Q.base_paths, Q.tail);
    Q.finish_q = rounds & 1;
    hipLaunchKernelGGL(wf_generate, dim3(grid_for(Q.base_paths, 16384)), dim3(kBlock), 0, stream, S, Q.Pd, Q);
    WF_CHECK(hipGetLastError());
    if (!E.span(0, err)) return false;
    if (!enqueue_pass(S, P, Q, rounds, count, full, E, err)) return false;
    hipLaunchKernelGGL(wf_motion, dim3(grid_for(Q.own_pixels, 1u << 30)), dim3(kBlock), 0, stream, S, Q.Pd, Q);
    WF_CHECK(hipGetLastError());
    if (!E.span(4, err)) return false;
    if (prev_done) WF_CHECK(hipStreamWaitEvent(stream, prev_done, 0));
    if (with_extra) {
        // second pass over the motion-adaptive extra samples (:779-789), appended to queue 0
        const int rounds2 = rounds_for((uint64_t)Q.own_pixels * (uint64_t)maxExtra, Q.tail);
        WF_CHECK(hipMemsetAsync(W.counts, 0, cslot(kShards) * sizeof(uint32_t), stream));
        WF_CHECK(hipMemsetAsync(W.counts + cslot(kCntChunkExtend), 0, cslot(2 * kShards) * sizeof(uint32_t), stream));
        WF_CHECK(hipMemsetD32Async(W.counts + cslot(kCntTailMode), 0u, 1, stream));
        WF_CHECK(hipMemsetD32Async(W.counts + cslot(kCntFinishQ), (uint32_t)(rounds2 & 1), 1, stream));
        WF_CHECK(hipMemsetD32Async(W.counts + cslot(kCntChunkFinish), 0u, 1, stream));
        hipLaunchKernelGGL(wf_extra, dim3(grid_for(Q.own_pixels, 1u << 30)), dim3(kBlock), 0, stream, S, Q.Pd, Q, 0);
        WF_CHECK(hipGetLastError());
        if (!E.span(4, err)) return false;
        if (!enqueue_pass(S, P, Q, rounds2, count, full, E, err)) return false;
    }
    hipLaunchKernelGGL(wf_resolve, dim3(grid_for(Q.own_pixels, 1u << 30)), dim3(kBlock), 0, stream, S, Q.Pd, Q,
                       with_extra ? 1 : 0);
    WF_CHECK(hipGetLastError());
    if (!E.span(4, err)) return false;
    WF_CHECK(hipMemcpyAsync(W.h_counts, W.counts, kWfCountWords * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    return true;
}

static bool enqueue_wavefront(const DevScene& S, const FrameParams& P, WfParams& Q, bool count, bool full,
                              int maxExtra, bool extra_pass, hipStream_t stream, hipEvent_t prev_done, WfTimeline& T,
                              const char** err) {
    Q.dev_ctl = 1;
    Q.drain_min = 0;
    Q.finish_q = 0;   // set by record_frame from the round count
    const bool with_extra = maxExtra > 0 && extra_pass;
    if (!record_frame(S, P, Q, count, full, maxExtra, with_extra, stream, prev_done, T, err)) return false;
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
    return true;
}

bool run_wavefront(const DevScene& S, const FrameParams& P, WavefrontBuffers& W, int own_tiles, bool count,
                   int tail_paths, int sort_bins, bool extra_pass, int in_flight, hipStream_t stream,
                   hipEvent_t prev_done, WfTimeline* tl, WfFrameStats* fs, const char** err) {
    WfParams Q;
    Q.W = W;
    Q.spp = max(P.U.samplesPerPixel, 1);
    Q.own_pixels = (uint32_t)own_tiles * (uint32_t)P.tile_size * (uint32_t)P.tile_size;
    Q.base_paths = Q.own_pixels * (uint32_t)Q.spp;
    Q.seg_cap = (uint32_t)(W.queue_entries / kShards);
    Q.refill_min = refill_min();
    Q.tri_vote = tri_vote();
    Q.chunk = chunk_size();
    Q.tail = tail_paths > 0 ? (uint32_t)tail_paths : tail_rays();
    Q.sort_bins = (uint32_t)sort_bins;
    static const int sort_xcd = env_int("RT_SORT_XCD", 1), steal = env_int("RT_STEAL", 0);
    Q.sort_xcd = sort_xcd;
    Q.steal = steal;
    Q.diag = wf_log() ? 1 : 0;
    // tail kernel: 0 per-segment wf_finish, 1 step-interleaved wf_finish_step, 2 wave-queue wf_finish_q
    static const int finish_step = env_int("RT_FINISH_STEP", 1), shade_min = env_int("RT_SHADE_MIN", 16);
    Q.finish_step = finish_step;
    Q.shade_min = shade_min;
    static const int drain_min = env_int("RT_DRAIN", 0);   // measured slower on C3g: off
    Q.drain_min = Q.finish_step == 1 ? drain_min : 0;
    static const int prio = env_int("RT_PRIO", 0), fchunk = env_int("RT_FCHUNK", 32);
    Q.fchunk = max(1, fchunk);
    // frames in flight: 1 / in_flight of the machine for the tail, the rest for the other frames'
    // bulk rounds (C3g, 2 in flight: 5.94 -> 5.72 ms per frame at 50 %; 3 in flight: 33 %); one
    // frame at a time: all of it.  Four frames of a small frame (below 6M base paths, a rank's
    // share): 20 %, per-rank 4-way split 4.48 -> 4.69 Grays/s against 25 %; a large frame forced
    // to four slots keeps 25 % (the 20 % sweep covered rank shares only)
    static const int finish_frac = env_int("RT_FINISH_FRAC", 0);
    // (round 2, two slots at the 1.25M threshold: 30 % 5.88 / 5.84, 35 % 5.97 / 6.00, 40 % 6.03 /
    // 6.01, 45 % 6.07 / 5.99, 50 % 5.93 / 5.90 Grays/s)
    Q.finish_frac = finish_frac > 0 ? min(finish_frac, 100)
                  : (in_flight >= 4 && Q.base_paths < (6u << 20)) ? 20
                  : in_flight == 2 ? 40 : (in_flight > 1 ? 100 / in_flight : 100);
    Q.prio = (prio && Q.finish_step == 1 && W.sorted) ? 1 : 0;
    if (Q.finish_step == 2 && (!W.p_ray || !W.p_sray)) {
        *err = "wave-queue finish kernel without its path ray slots";
        return false;
    }
    if (sort_bins && (sort_bins < kSortMinBins || sort_bins > kSortMaxBins || (sort_bins & (sort_bins - 1)) ||
                      !S.tri_bin || !W.sorted)) {
        *err = "bad hit-sort configuration";
        return false;
    }
    *fs = WfFrameStats{};
    float* stage_ms = fs->stage_ms;
    static const bool host_ctl = env_int("RT_WF_HOST", 0) != 0 || getenv("RT_WF_DUMP") != nullptr;
    // tail <= 1 (bulk rounds only, a test configuration) keeps the host loop: its round count is
    // only bounded by maxBounces * (maxBounces + 1)
    const bool dev = tl && !host_ctl && !wf_log() && Q.drain_min == 0 && Q.tail > 1;
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
    if (dev)
        return enqueue_wavefront(S, P, Q, count, full, maxExtra, extra_pass, stream, prev_done, *tl, err);
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
