// rt_kernels.h — kernel parameter blocks and launch entry points (device code lives in *.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "rt_device.h"

namespace rt {

constexpr int kHaltonLds = 64;   // first Halton dimensions staged in LDS per block

// kCntNodes: every node test.  Slots 8 and 9 are unused (formerly LDS-served node tests).
// kCntTrace*: the share of the visits made by wf_trace launches.
enum CounterSlot {
    kCntClosest = 0, kCntShadow = 1, kCntNodes = 2, kCntTris = 3, kCntPaths = 4, kCntOverflow = 5,
    kCntTraceNodes = 6, kCntTraceTris = 7, kCntSlots = 10
};

struct FrameParams {
    Uniforms U;
    const uint32_t* random;
    const float4* accum_in;    // history (TextureIndexAccumulation, read)
    float4* accum_out;         // new accumulation (TextureIndexPreviousAccumulation, write)
    float* depth;
    float2* motion;            // read (previous frame) + write, in place
    const float2* motion_prev; // wavefront: the previous frame's motion target (it writes a new one)
    float4* gbuffer;           // 4 planes or null
    uint4* prim_hit;           // wavefront: sample 0's last bounce-0 hit per pixel (wf_motion input)
    unsigned long long* counters;
    int tile_size, rank, nranks, tiles_x;
};

__device__ __forceinline__ unsigned long long wave_sum(uint32_t v) {
    unsigned long long s = v;
    #pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

// Statistics counters: every (slot, replica) word sits on a 128-B line of its own and a block adds
// to replica blockIdx % 8 once per slot, so no line sees more than ~1/8 of the blocks' atomics
// (device-scope atomics on one line serialise at ~88/us).  The host sums the replicas.
constexpr int kCntReplicas = 8;
constexpr int kCntLineU64 = 16;
constexpr int kCounterWords = kCntSlots * kCntReplicas * kCntLineU64;
__host__ __device__ constexpr uint32_t cnt_word(int slot, int rep) {
    return ((uint32_t)slot * kCntReplicas + (uint32_t)rep) * kCntLineU64;
}

// Block-wide flush of the per-thread statistics; every thread of the block must call it.
// nodes: global node fetches, lds_nodes: node tests served from LDS (both count as node visits).
// trace_kernel: the node / triangle visits are also added to the kCntTrace* slots.
__device__ __forceinline__ void block_flush_counters(unsigned long long* counters, uint32_t closest, uint32_t shadow,
                                                     uint32_t nodes, uint32_t tris, uint32_t paths, bool overflow,
                                                     bool trace_kernel = false, uint32_t lds_nodes = 0) {
    __shared__ unsigned long long red[kBlock / 64][kCntSlots];
    const unsigned long long l = wave_sum(lds_nodes), n = wave_sum(nodes) + l, t = wave_sum(tris);
    const unsigned long long v[kCntSlots] = {wave_sum(closest), wave_sum(shadow), n, t, wave_sum(paths),
                                             __ballot(overflow) != 0ull ? 1ull : 0ull,
                                             trace_kernel ? n : 0ull, trace_kernel ? t : 0ull, l,
                                             trace_kernel ? l : 0ull};
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        #pragma unroll
        for (int k = 0; k < kCntSlots; ++k) red[wave][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < kCntSlots) {
        unsigned long long s = 0;
        #pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) s += red[w][threadIdx.x];
        if (s) atomicAdd(&counters[cnt_word(threadIdx.x, blockIdx.x & (kCntReplicas - 1))], s);
    }
}

void launch_megakernel(const DevScene& S, const FrameParams& P, int nblocks, bool count, hipStream_t stream);

// Wavefront pipeline (rt_wavefront.hip): path state SoA indexed by path id
// (own pixel index * spp + sample; extra samples after base_paths), ray queues of
// {float4 o (w = path id), float4 d}, hit records {t, tri id, u, v}, shadow queue of
// {float4 o (w = path id), float4 d (w = tmax), float4 contribution}.
constexpr int kShards = 8;        // queue segments (one allocation counter each)
// Counter slots: [0..7] queue 0, [8..15] queue 1, [16..23] shadow, [24] extra allocator,
// [32..39] / [40..47] per-XCD chunk counters of the extend / connect launches; each slot on a
// 128-B line of its own (cslot), so the per-XCD shards never contend for one line's atomics.
constexpr int kCntStride = 32;
constexpr int kCntSlotsWf = 74;                       // counter slots (cslot) before the diagnostics words
constexpr int kWfDiagHist = kCntSlotsWf * kCntStride; // 64 words: wf_finish wave end-time histogram (50 us bins)
constexpr int kWfDiagSteps = kWfDiagHist + 64;        // 66 words: wf_trace steps-per-ray histograms + max
constexpr int kWfStat = kWfDiagSteps + 66;              // 3 words: rounds, wf_trace launches, their rays
constexpr int kStatRounds = 0, kStatTraceLaunches = 1, kStatTraceRays = 2, kStatExtendRays = 3, kStatFinish = 4;
// wf_finish_step diagnostics (RT_WF_LOG): summed over waves, s_memrealtime ticks (10 ns) spent in
// shading passes and in total, shading passes and lanes shaded
constexpr int kStatDiagShadeT = 5, kStatDiagTotalT = 6, kStatDiagPasses = 7, kStatDiagShaded = 8;
// ... and split at the wave's queue exhaustion: iterations and ticks before / after it, and the
// wave's active lanes summed over its iterations after it
constexpr int kStatDiagItPre = 9, kStatDiagItPost = 10, kStatDiagTPre = 11, kStatDiagTPost = 12, kStatDiagLanesPost = 13;
constexpr int kWfStatWords = 14;
// wf_finish_step diagnostics (RT_WF_LOG): paths by segments run in the finish (32 bins) per entry
// class (18: bounce 0..8 at entry, x refracting or not), then the waves' queue-exhaustion times
// (64 bins of 50 us)
constexpr int kWfDiagLen = kWfStat + kWfStatWords;
constexpr int kWfDiagExh = kWfDiagLen + 18 * 32;
constexpr int kWfCountWords = kCntSlotsWf * kCntStride + 64 + 66 + kWfStatWords + 18 * 32 + 64;
__host__ __device__ constexpr uint32_t cslot(int c) { return (uint32_t)c * kCntStride; }
struct WavefrontBuffers {
    size_t queue_entries = 0;     // kShards segments of queue_entries / kShards
    float4* p_accum = nullptr;
    uint4* p_meta = nullptr;      // extra-sample paths only: (pixel, sample, 0, halton index)
    // ray queues: entry e = {origin, w = path id}, {direction, w = path state bits: bounce | tpass << 8 |
    // step << 16}; qc[q][e] = the path's throughput colour (absent for state 0, the primary ray: 1)
    float4* q[2] = {nullptr, nullptr};
    float4* qc[2] = {nullptr, nullptr};
    float4* hits = nullptr;
    float4* sq = nullptr;
    uint32_t* counts = nullptr;   // device counter slots (see cslot)
    uint32_t* h_counts = nullptr; // pinned host mirror
    // device-clock launch spans (kTsSlots launch slots x kTsStride words, s_memrealtime) + pinned mirror
    unsigned long long* tstamp = nullptr;
    unsigned long long* h_tstamp = nullptr;
    uint2* px_extra = nullptr;    // per own pixel: (first extra path - base_paths, count)
    // per-bounce hit sort (wf_sort_*): the hits reordered by key as {o, d, hit, colour} float4 quads,
    // per-(bin, block) counts, per-bin totals
    float4* sorted = nullptr;
    uint32_t* sort_table = nullptr;
    uint32_t* sort_total = nullptr;
    size_t cap_paths = 0;         // base + extra paths
    size_t cap_pixels = 0;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    // FrameParams of the frame in flight: one device copy the kernels read, uploaded from a ring
    // of pinned host slots
    static constexpr int kParamSlots = 4;
    FrameParams* d_params = nullptr;
    FrameParams* h_params = nullptr;
    hipEvent_t param_ev[kParamSlots] = {nullptr, nullptr, nullptr, nullptr};
    int param_slot = 0;
};
// Hit sort: kSortBlocks blocks of kSortThreads share one partition of the queue in the histogram
// and scatter kernels; bins are a power of two in [kSortMinBins, kSortMaxBins].
constexpr int kSortBlocks = 256;
constexpr int kSortThreads = 1024;
constexpr int kSortMinBins = 1024;
constexpr int kSortMaxBins = 4096;
constexpr int kSortBinsDefault = 0;   // off: measured slower on C3g (DESIGN.md §3 'Hit sort')
// Per-frame measurements of the wavefront pipeline. stage_ms: [0] generate, [1] extend,
// [2] shade, [3] connect, [4] resolve (+extra-sample bookkeeping), [5] finish, [6] hit sort.
// Launch slots of the device-clock spans: per pass (base, extra samples) two per round (extend
// 2k, connect 2k + 1; rounds <= 16) and the finish launch (kTsFinish); the extra pass at kTsPass.
constexpr int kTsPass = 40, kTsFinish = 33, kTsSlots = 2 * kTsPass;
// a launch slot: its start, then one end word per XCD, each on a 128-B line of its own (the last
// wave of every block takes the max on its XCD's line; one line for all would serialise them)
constexpr int kTsLine = 16, kTsStride = 9 * kTsLine;
// the counter words and, 8-byte aligned after them, the launch spans share one allocation
constexpr size_t kWfTsOffset = ((size_t)kWfCountWords * 4 + 7) / 8 * 8;
constexpr size_t kWfCountAllocBytes = kWfTsOffset + (size_t)kTsSlots * kTsStride * 8;
struct WfFrameStats {
    float trace_dev_ms, finish_dev_ms;   // device-clock spans of the extend + connect / finish launches
    int trace_dev_launches, finish_dev_launches;
    float stage_ms[7];
    int iterations;
    unsigned long long trace_rays;  // rays traced by wf_trace launches (extend + connect)
    unsigned long long trace_closest_rays;   // the extend share
    int trace_launches;
    float trace_ms;                 // their summed device time
    int finish_launches;
    int graph_mode;                 // kGraph*: how the frame was submitted
};
// The wavefront kernels' scheduling parameters, resolved (rt_tuning in rt_api.h: 0 = default there;
// rt_api.cpp fills these in).  Per context: the library reads no environment variable for them.
struct WfTuning {
    uint32_t tail = 4194304;      // finish threshold one frame at a time (frames in flight: rt_api.cpp kTailInFlight)
    int refill_min = 8;           // a wave refills once this many of its lanes are idle
    int chunk = 64;               // rays per chunk grab of the traversal kernel
    int fchunk = 64;              // paths per chunk grab of the finish kernel
    int shade_min = 24;           // the finish kernel shades once this many lanes wait
    int shade_min_x = -50;        // the same once its queue ran out (< 0: that percentage of the wave's busy lanes)
    int team = -1;                // finish drain lanes per query (-1: 4 for frames of kTeamAutoMin .. kTeamAutoPaths
                                  // base paths, off otherwise; 0: off; 2 / 4 / 8)
    int finish_frac = 0;          // percent of the resident grid the finish launch takes (0 = by frames in flight)
    int trace_frac = 0;           // percent of the resident grid the bulk wf_trace launches take (0 = by frames in flight)
    int log = 0;                  // 1: per-round queue sizes, stage times and finish diagnostics on stderr;
                                  // 2: also the finish paths' segment counts (one atomic per path)
    bool host_ctl = false;        // host-driven rounds (queue sizes read back every round)
    unsigned shade_blocks = 2048; // wf_shade grid (grid-stride loop), a multiple of 8: 1.6 waves of the resident
                                  // grid leaves CUs to the other frames in flight
};

// Runs one frame; returns false on a HIP error (message in *err).
// tail_paths: finish-kernel threshold (0 = default / RT_TAIL_RAYS).
// Host-side record of a frame enqueued with device-side control: events between the launches and
// which stage each interval belongs to; collected once the frame is done (wavefront_collect).
struct WfTimeline {
    static constexpr int kMaxEv = 160;
    struct Span {
        int stage, a, b;
    };
    hipEvent_t ev[kMaxEv] = {};
    Span spans[kMaxEv];
    int n_ev = 0, n_spans = 0;
    bool pending = false;
    bool dev_spans = false;   // the frame recorded device-clock launch spans (tstamp copied back)
    // RT_GRAPH: the slot's frame captured as two HIP graphs (events recorded as external event
    // nodes, so the spans above keep timing it) and replayed while `key` (every launch argument and
    // enqueue decision of the frame) is unchanged: exec[0] up to the motion vectors, exec[1] the
    // rest, with the wait for the previous frame enqueued between them (a plain stream wait, not a
    // captured external-event wait node)
    hipGraphExec_t exec[2] = {nullptr, nullptr};
    std::vector<uint8_t> key;
    bool graph_failed = false;   // capture was refused once: this slot stays eager
    int graph_mode = 0;          // the pending frame: kGraph* (rt_stats total_graph_*)
};
constexpr int kGraphEager = 0, kGraphReplay = 1, kGraphCapture = 2, kGraphFallback = 3;
// Runs (host-driven: queue sizes read back every round; with RT_WF_LOG / RT_WF_HOST=1) or enqueues (device-driven, the default: `tl` receives the timeline, stats come
// from wavefront_collect after the stream finished) one frame; false on a HIP error (*err).
// sort_bins: hit-sort bins (0 = no sort).  extra_pass: the motion-adaptive extra samples can be
// non-zero this frame (something moved in this or the previous frame); the device-driven mode
// skips their pass otherwise.  in_flight: frames that can overlap this one (> 1: the finish
// kernel takes 1 / in_flight of the resident grid and leaves the rest to the other frames).  prev_done (may be null): the previous frame, in flight on another
// stream; the extra-sample pass and the resolve (which read its accumulation and motion outputs)
// are ordered after it, everything before them overlaps it.
bool run_wavefront(const DevScene& S, const FrameParams& P, WavefrontBuffers& W, const WfTuning& tu, int own_tiles,
                   bool count, bool spans, int tail_paths, int sort_bins, bool extra_pass, int in_flight,
                   hipStream_t stream, hipEvent_t prev_done, WfTimeline* tl, WfFrameStats* fs, const char** err,
                   bool graphs = true);
bool wavefront_collect(const WavefrontBuffers& W, WfTimeline& T, WfFrameStats* fs, const char** err);
size_t wavefront_queue_entries(size_t paths, int max_extra);

// Packed-tile layout of the multi-GPU gather: element i of a rank's packed buffer is pixel
// (i % T, (i / T) % T) of its (i / T^2)-th own tile; own tile k is tile id rank + k * nranks.
__host__ __device__ __forceinline__ void tile_pixel(size_t i, int tile, int rank, int nranks, int tiles_x, int& x,
                                                    int& y) {
    const size_t per = (size_t)tile * tile;
    const int k = (int)(i / per), r = (int)(i % per);
    const int tid = rank + k * nranks;
    x = (tid % tiles_x) * tile + r % tile;
    y = (tid / tiles_x) * tile + r / tile;
}

// On-device BVH build (rt_lbvh.hip): LBVH over Morton codes collapsed into the compressed 8-wide
// layout of rt_bvh.h.  Inputs are the uploaded scene streams; outputs are caller-allocated device
// arrays sized for n triangles (nodes8 / node_box / levels: n entries, tri_order n, tri_bin n).
struct LbvhInput {
    const float4* pos;
    const uint4* tri_info;
    const float* inst;
    uint32_t n;
    int ploc = 1;          // BVH2 topology: 1 = PLOC clustering, 0 = LBVH radix tree (8-wide: SAH-DP collapse)
    float c_node = 1.0f;   // DP costs (as the host builder's)
    float c_prim = 0.5f;
};
struct LbvhOutput {
    Bvh8Node* nodes8;
    float* node_box;        // 6 floats per node (padded lo, hi)
    uint32_t* tri_order;    // 8-wide triangle slot -> original triangle id
    uint16_t* tri_bin;      // hit-sort bin per original triangle
    uint32_t* levels;       // refit level list (the identity: nodes are allocated level by level)
    uint32_t* h_scratch;    // 1 pinned host word
};
struct LbvhResult {
    std::vector<uint32_t> level_off;   // level k = nodes [level_off[k], level_off[k + 1])
    uint32_t num_nodes = 0;
    int max_depth = 0;
    float pad = 0.0f;
};
size_t lbvh_scratch_bytes(uint32_t n);
bool lbvh_build(const LbvhInput& in, const LbvhOutput& out, void* scratch, hipStream_t s, LbvhResult* res,
                const char** err);

// Utility kernels (rt_util.hip)
// G-buffer-guided denoise for RT_SCALER_DENOISED (rt_present.hip); returns tmp0 or tmp1, whichever
// holds the result (passes = 0 returns the demodulated radiance unremodulated: callers pass >= 1)
const float4* launch_denoise(const float4* accum, const float* depth, const float4* gbuf, float4* tmp0, float4* tmp1,
                             float4* guide, float4* alb, int w, int h, int passes, hipStream_t stream);
void launch_present(const float4* accum, const float* depth, const float2* motion, const float4* hist_in,
                    const float* hdepth_in, float4* hist_out, float* hdepth_out, uchar4* out, const float* thr, int w,
                    int h, int ow, int oh, int scaler, int srgb, int use_hist, hipStream_t stream);
void launch_pack_tiles(const float4* src, float4* dst, int width, int height, int tile, int rank, int nranks,
                       int tiles_x, int own, hipStream_t s);
void launch_unpack_tiles(const float4* src, float4* dst, int width, int height, int tile, int rank, int nranks,
                         int tiles_x, int own, hipStream_t s);
void launch_to_half(const float4* src, ushort4* dst, size_t n, hipStream_t s);
// sum of the node boxes' areas (node_box: 6 floats per node), one float out
void launch_bvh_cost(const float* node_box, uint32_t nn, float* out, hipStream_t s);
void launch_skin(const float4* rest_pos, const float4* rest_nrm, const ushort4* jidx, const float4* jw,
                 const float* joints, float4* out_pos, float4* out_nrm, uint32_t n, hipStream_t s);
// flatten also reduces max |world coordinate| into *maxabs_bits (float bits; zero it first)
void launch_flatten(const uint4* tri_info, const uint32_t* slot_to_tri, const float4* pos, const float* inst,
                    float* tris, uint32_t n, unsigned* maxabs_bits, hipStream_t s);
// per-triangle shading records of triangles [t0, t0 + n) (DevScene::tri_nrm) from tri_info and the
// vertex normals; rebuilt whenever normals change (scene upload, skinning)
void launch_tri_nrm(const uint4* tri_info, const float4* nrm, float4* tri_nrm, uint32_t t0, uint32_t n, hipStream_t s);
// pad = max(pad_min, 4e-6 * max |coordinate|) as the builder pads (rt_bvh.cpp)
void launch_refit8_level(Bvh8Node* nodes, float* node_box, const float* tris, const uint32_t* level_nodes,
                         uint32_t count, float pad_min, const unsigned* maxabs_bits, hipStream_t s);

}  // namespace rt
