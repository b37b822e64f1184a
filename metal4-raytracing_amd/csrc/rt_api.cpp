// rt_api.cpp — C-ABI implementation (include/rt_api.h): device memory, scene upload, BVH,
// per-pixel targets, frame dispatch.  Mirrors the responsibilities of the reference's Renderer
// (MetalRaytracing/Renderer.swift) for the hot path; all device work is issued in order on one
// HIP stream per context (the reference's MTL4CommandQueue + events, Renderer.swift:1405-1503).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_bvh.h"
#include "rt_kernels.h"

using namespace rt;

namespace {
thread_local std::string g_err;

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct MeshInfo {
    uint32_t vbase = 0, vcount = 0, joint_count = 0;
    uint32_t tbase = 0, tcount = 0;   // the mesh's triangles (original ids are assigned mesh by mesh)
    bool skinned = false;
};

// One frame in flight (Renderer.swift:207, 1406-1409 keeps up to 3): its wavefront memory, its
// per-frame targets and statistics, and the stream it renders on.  Consecutive frames rotate over
// the slots and overlap except where frame f needs frame f-1's results (the history target and
// the previous motion vectors: the extra-sample pass and the resolve).
struct FrameSlot {
    DevBuf qc, accum, meta, q0, q1, hits, sq, counts, extra, sorted, sort_table, sort_total, params;
    DevBuf depth, gbuffer, counters;
    DevBuf prim_hit;   // wavefront: per pixel, sample 0's last bounce-0 hit (id, u, v) for wf_motion
    WavefrontBuffers wf;
    WfTimeline wft;
    WfFrameStats wfs{};
    unsigned long long* h_counters = nullptr;   // pinned copy of `counters` after the frame
    hipStream_t own_stream = nullptr;           // slots 1..; slot 0 renders on rt_ctx::stream
    hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;
    bool pending = false, wavefront = false, used = false;
    bool gbuf_written = false;                  // the slot's last frame wrote the G-buffer (enableDenoiseGBuffer)
    uint64_t seq = 0;                           // frame number (harvest order)
    uint64_t ctx_seen = 0;                      // rt_ctx::ctx_work the slot's stream last waited for
    int gen = 0;                                // geometry generation the frame reads
    DevBuf* bufs[17] = {&qc, &accum, &meta, &q0, &q1, &hits, &sq, &counts, &extra, &sorted,
                        &sort_table, &sort_total, &params, &depth, &gbuffer, &counters, &prim_hit};
};
// Per-frame geometry (what skinning, instance transforms and refit rewrite between frames), in
// generations used round robin: frames read generation `gcur`; the first update after a frame
// copies it into the next generation (once the frames still reading that one, ngens frames back,
// have finished) and every update until the next frame writes there, so frames in flight keep
// their geometry while the next frame's is built (Renderer.swift keeps per-frame position buffers
// for the same reason, :1290-1303).  ngens = max(2, frames in flight): with an update before every
// frame (skinning, refit), all frames in flight still overlap, and no more copies exist than
// frames can read.
struct Geo {
    DevBuf pos, prev_pos, nrm, inst, prev_inst, tris, nodes, node_box, tri_bin, tri_nrm;
    DevBuf* all[10] = {&pos, &prev_pos, &nrm, &inst, &prev_inst, &tris, &nodes, &node_box, &tri_bin, &tri_nrm};
    uint32_t num_nodes8 = 0;
};
#ifndef RT_MAX_SLOTS
#define RT_MAX_SLOTS 8
#endif
constexpr int kMaxSlots = RT_MAX_SLOTS;
constexpr int kGens = kMaxSlots;   // generations allocated at most (ngens of them in use)
// default finish threshold with 2 / 3 / 4 frames in flight (C3g sweeps: 1.25M, 1M and 512K paths;
// round 2, with the DP-collapsed tree and the lighter shading kernels, two slots: 2M 5.88 / 5.89,
// 1.57M 5.90 (C3g enters the finish one round earlier between 1.5M and 1.57M live paths),
// 1.5M 5.97 / 6.02, 1M 6.02 / 6.00 Grays/s; four slots serve the small frames of multi-GPU ranks:
// 8-way split 2.92 -> 3.46 Grays/s per rank at 512K against 1M in round 1, 256K-786K within noise
// in round 2, with the finish kernel on 20 % of the grid)
// Final round-2 kernels, 8-way share with four slots: 256K 4.14 / 4.13, 512K 4.25 / 4.26, 768K
// 4.32 / 4.30 Grays/s per rank -> 768K for four slots.
constexpr int kTailInFlightTab[9] = {0, 0, 1310720, 1048576, 786432, 524288, 524288, 524288, 524288};
constexpr int kTailInFlight(int nfl) { return kTailInFlightTab[nfl < 8 ? nfl : 8]; }
// Default frames in flight (render_frame): their buffers, ~300 B per allocated path (pixels x (spp +
// motion-adaptive extra samples)) and slot (128 B path state and ray slots + 176 B of queues), stay
// within kSlotBudget of the 288 GB (1080p x 4 + 2 extra: 3.7 GB a slot; configs[3]'s 3840x2160x16
// frame on one GPU: 40 GB a slot, two slots).
constexpr uint64_t kSlotBudget = 96ull << 30, kSlotBytesPerPath = 300;
constexpr int kMotionTargets = kMaxSlots + 1;
// Default slots: eight when the HIP runtime gives the process at least eight hardware
// queues (GPU_MAX_HW_QUEUES, read once; HIP's default is 4), so every slot's stream has a queue of
// its own; four otherwise (more streams than queues serialise unrelated frames: eight slots on
// four queues measured 2.85 against 3.54 Grays/s per rank).  8-way rank share of C3g, eight
// queues: 4 slots 3.54 / 3.52, 8 slots 3.71 / 3.69; 4-way 4.73 / 4.70 -> 4.76 / 4.86.
static int small_frame_slots() {
    static const int n = [] {
        const char* e = getenv("GPU_MAX_HW_QUEUES");
        return (e && atoi(e) >= 8) ? 8 : 4;
    }();
    return n;
}
// Frames below this many allocated paths keep at most four slots: a configs[0]-sized frame (65K
// paths, ~0.05 ms) on eight slots / eight queues ran bimodally, 2.04-2.10 or 0.55-0.62 Grays/s
// (3 of 6 runs slow), against 2.10-2.54 on four (round 5); the 8-way C3g share (1M paths) gains
// 9 % from eight slots and was steady.  Round 6 traced six such runs (profiles/r06_c1_bimodal.txt):
// the kernels take the same time in slow and fast runs, the slow ones overlap their frames less
// (0.94-1.10 kernels at once against 1.38) -- slot streams sharing hardware queues serialise a
// frame whose GPU work is ~0.12 ms; at four slots there is queue room to spare.
constexpr uint64_t kSmallFramePaths = 1ull << 19;
constexpr uint64_t kSmallShareBasePaths = 2500000;   // see rt_render_frame's tail
constexpr int kTailShare = 786432;
// rt_set_tuning bounds: a chunk grab past the end of a queue still adds the chunk size to its
// 32-bit counter, once per wave (at most ~16K waves resident); 4096 x 16K stays far below 2^32
// minus any queue the library allocates.  The shade grid is grid-stride, so more blocks than
// 64K buy nothing.
constexpr int kMaxTuneChunk = 4096;
constexpr int kMaxTuneShadeBlocks = 65536;
}  // namespace

struct rt_ctx {
    int device = 0;
    int pipeline = RT_PIPELINE_MEGAKERNEL;
    int tail_paths = 0;
    int sort_bins = kSortBinsDefault;   // 0 = no hit sort
    hipStream_t own_stream = nullptr, stream = nullptr;
    std::string err;
    bool counting = false;
    bool spans = false;              // rt_set_device_spans
    bool graphs = true;              // rt_set_graphs
    rt_tuning tuning_req{};          // rt_set_tuning as given (0 = default)
    WfTuning tuning;                 // ... resolved

    // host scene copies
    std::vector<float4> h_pos, h_nrm;
    std::vector<uint4> h_tri_info;
    std::vector<float> h_inst;
    std::vector<Material> h_mat;
    std::vector<Light> h_lights;
    std::vector<MeshInfo> meshes;
    std::vector<float> h_world;   // 9 floats per triangle
    int max_sub = 1;
    uint32_t num_tris = 0, num_verts = 0, num_inst = 0;
    bool scene_ready = false, bvh_ready = false;
    bool world_dirty = false;  // device positions/transforms changed since h_world was computed

    // BVH
    BvhResult bvh;
    Bvh8Result bvh8;
    std::vector<uint32_t> level_nodes;
    std::vector<uint32_t> level_off;

    // device buffers
    Geo geo[kGens];
    int gcur = 0;            // generation new frames read
    int ngens = 2;           // generations in rotation: max(2, frames in flight)
    int cur_nfl = 0;         // frames in flight of the newest frame (a change drains and re-sizes the rotation)
    bool gdirty = false;     // updates since the last frame went into generation next_gen()
    hipStream_t ustream = nullptr;   // geometry updates (skin, transforms, refit)
    hipEvent_t uev = nullptr;        // end of the latest update batch; frames wait on it
    bool uev_valid = false;
    int next_gen() const { return (gcur + 1) % ngens; }
    Geo& G() { return geo[gdirty ? next_gen() : gcur]; }   // the generation updates and builds write
    DevBuf d_rest_pos, d_rest_nrm, d_jidx, d_jw, d_joints;
    DevBuf d_tri_info, d_mat, d_lights, d_halton;
    DevBuf d_tex_texels, d_tex_info, d_mat_tex, d_uv, d_tex_lut;   // texture path (textured scenes)
    bool textured = false;
    DevBuf d_slot_to_tri, d_levels, d_maxabs, d_lbvh_scratch;
    uint32_t num_nodes8 = 0;
    uint32_t* h_lbvh = nullptr;   // pinned word for the device builder's level counts
    // tree quality under refit (rt_tuning.refit_rebuild_pct): the node-area sum (launch_bvh_cost)
    // of the last build and of the last refit, the latter read back asynchronously
    DevBuf d_cost;
    float* h_cost = nullptr;
    hipEvent_t cost_ev = nullptr;
    bool cost_pending = false;
    float cost_built = 0.0f, cost_refit = 0.0f;
    uint64_t auto_rebuilds = 0;
    DevBuf d_random, d_accum[2];
    // Motion vectors rotate over kMaxSlots + 1 targets: a wavefront frame writes d_motion[m + 1]
    // and reads the previous frame's d_motion[m], so it never overwrites a target an older frame
    // still in flight reads (the megakernel reads and rewrites d_motion[m] in place).
    DevBuf d_motion[kMotionTargets];
    int motion_cur = 0;
    int width = 0, height = 0;
    int read_idx = 0;   // accum[read_idx] = history (TextureIndexAccumulation)
    uint32_t last_frame_index = 0;   // Uniforms.frameIndex of the newest frame
    // display output (rt_present): temporal-scaler history at the output size, sRGB thresholds
    DevBuf d_hist[2], d_hdepth[2], d_present_out, d_present_thr;
    DevBuf d_half;   // rt_read_radiance_half staging (RGBA16F)
    int hist_w = 0, hist_h = 0, hist_idx = 0;
    bool hist_valid = false;
    DevBuf d_den[4];   // RT_SCALER_DENOISED scratch at render size: ping, pong, guide, albedo
    size_t den_n = 0;
    rt_stats stats{};

    // frames in flight
    FrameSlot slot[kMaxSlots];
    int max_in_flight = 0;           // rt_opts.frames_in_flight; 0 = by frame size (auto_in_flight)
    int nslots = 1;                  // slots in use (1: megakernel, external stream)
    uint64_t frame_no = 0;           // frames submitted since rt_resize
    int last_slot = 0;               // slot of the newest frame
    hipEvent_t scene_ev = nullptr;   // ctx->stream work a slot-1 frame must follow
    uint64_t ctx_work = 1;           // bumped whenever work that frames must follow is enqueued on ctx->stream
    bool tiles_pending = false;      // a pack / unpack extended the newest frame's `done`
    int last_tiles[3] = {0, 0, 0};   // tile_size, rank, nranks of the newest frame
    rt_stats totals{};   // the running-total fields of rt_stats

    // motion bookkeeping for the extra-sample pass: motion vectors are exactly zero unless the
    // camera, an instance transform or skinned positions differ from their previous copies
    bool inst_moved = false, skin_moved = false, last_moving = false;
};

#define FAIL(ctx, code, msg)                 \
    do {                                     \
        if (ctx) (ctx)->err = (msg);         \
        g_err = (msg);                       \
        return (code);                       \
    } while (0)

#define HIPC(ctx, expr)                                                                            \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            std::string m_ = std::string(#expr) + ": " + hipGetErrorString(e_);                    \
            if (ctx) (ctx)->err = m_;                                                              \
            g_err = m_;                                                                            \
            return e_ == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_HIP;                  \
        }                                                                                          \
    } while (0)

static rt_status dev_alloc(rt_ctx* c, DevBuf& b, size_t bytes) {
    if (b.p && b.bytes >= bytes && bytes > 0) return RT_OK;
    if (b.p) { (void)hipFree(b.p); b.p = nullptr; b.bytes = 0; }
    if (bytes == 0) return RT_OK;
    HIPC(c, hipMalloc(&b.p, bytes));
    b.bytes = bytes;
    return RT_OK;
}
static rt_status dev_upload(rt_ctx* c, DevBuf& b, const void* src, size_t bytes, hipStream_t s = nullptr) {
    rt_status st = dev_alloc(c, b, bytes);
    if (st) return st;
    if (bytes) HIPC(c, hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, s ? s : c->stream));
    if (bytes && !s) c->ctx_work++;
    return RT_OK;
}
static void dev_free(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

static std::vector<HaltonDim> halton_table() {
    std::vector<HaltonDim> t;
    uint32_t n = 2;
    while ((int)t.size() < RT_HALTON_DIMS) {
        bool prime = true;
        for (auto& h : t) {
            if (h.b * h.b > n) break;
            if (n % h.b == 0) { prime = false; break; }
        }
        if (prime) {
            HaltonDim h;
            h.b = n;
            uint32_t l = 0;
            while ((1u << l) < n) ++l;              // 2^(l-1) < b <= 2^l
            h.m = (uint32_t)(((1ull << (31 + l)) + n - 1) / n);
            h.sh = l - 1;
            h.invB = 1.0f / (float)n;
            t.push_back(h);
        }
        ++n;
    }
    return t;
}

// SAH build (one triangle per BVH2 leaf) + SAH-DP 8-wide collapse (c_node 1, c_prim 0.5: the C3g
// sweep of DESIGN.md §3) whose group-stack depth fits the kStackSize LDS stack: the binned-SAH
// builder falls back to median splits past its depth limit, so tighter limits bound the depth.
// false on failure (no depth limit fits, or the builder threw: allocation, internal checks);
// nothing is thrown across the C-ABI.
static bool build_bvh8_fit(const float* world, uint32_t n, BvhResult& b2, Bvh8Result& b8) {
    try {
        for (int limit : {64, 48, 40, 32, 28, 24, 21}) {
            b2 = build_bvh2(world, n, 1, limit);
            b8 = collapse_bvh8_dp(b2, 1.0f, 0.5f);
            if (b8.max_depth <= kStackSize) return true;
        }
    } catch (const std::exception&) {
    }
    return false;
}

// host object->world, identical arithmetic to rt::xform on the device
static void xform_host(const float* m, const float4& p, float* out) {
    for (int r = 0; r < 3; ++r) out[r] = ((m[0 + r] * p.x + m[3 + r] * p.y) + m[6 + r] * p.z) + m[9 + r] * 1.0f;
}

static size_t ctx_bytes(const rt_ctx* c) {
    const DevBuf* all[] = {&c->d_rest_pos, &c->d_rest_nrm, &c->d_jidx, &c->d_jw,
                           &c->d_joints, &c->d_tri_info, &c->d_mat, &c->d_lights,
                           &c->d_halton, &c->d_slot_to_tri, &c->d_levels, &c->d_maxabs, &c->d_random,
                           &c->d_accum[0], &c->d_accum[1], &c->d_lbvh_scratch,
                           &c->d_tex_texels, &c->d_tex_info, &c->d_mat_tex, &c->d_uv, &c->d_tex_lut,
                           &c->d_hist[0], &c->d_hist[1], &c->d_hdepth[0], &c->d_hdepth[1], &c->d_present_out,
                           &c->d_present_thr, &c->d_den[0], &c->d_den[1], &c->d_den[2], &c->d_den[3], &c->d_half, &c->d_cost};
    size_t s = 0;
    for (auto* b : all) s += b->bytes;
    for (const DevBuf& b : c->d_motion) s += b.bytes;
    for (const Geo& g : c->geo)
        for (const DevBuf* b : g.all) s += b->bytes;
    for (const FrameSlot& f : c->slot)
        for (const DevBuf* b : f.bufs) s += b->bytes;
    return s;
}

static rt_status ensure_wavefront(rt_ctx* c, FrameSlot& fs, size_t own_px, int spp, int max_extra) {
    WavefrontBuffers& W = fs.wf;
    size_t paths = own_px * (size_t)(spp + max_extra);
    size_t npix = (size_t)c->width * c->height;
    if (paths >= (1ull << 32)) FAIL(c, RT_ERR_UNSUPPORTED, "too many paths for one frame");
    rt_status st;
    if (W.cap_paths < paths || W.queue_entries < wavefront_queue_entries(paths, max_extra)) {
        size_t qe = wavefront_queue_entries(paths, max_extra);
        if ((st = dev_alloc(c, fs.qc, 2 * qe * 16))) return st;   // both queues' colour arrays
        if ((st = dev_alloc(c, fs.accum, paths * 16))) return st;
        if ((st = dev_alloc(c, fs.meta, paths * 16))) return st;
        if ((st = dev_alloc(c, fs.q0, qe * 32))) return st;
        if ((st = dev_alloc(c, fs.q1, qe * 32))) return st;
        if ((st = dev_alloc(c, fs.hits, qe * 16))) return st;
        if ((st = dev_alloc(c, fs.sq, qe * 48))) return st;
        // hit sort output (4 float4 per hit), only with the sort on
        if (c->sort_bins && (st = dev_alloc(c, fs.sorted, qe * 64))) return st;
        W.cap_paths = paths;
        W.queue_entries = qe;
    }
    if (W.cap_pixels < npix || W.cap_pixels < own_px) {
        size_t px = std::max(npix, own_px);
        if ((st = dev_alloc(c, fs.extra, px * 8))) return st;
        W.cap_pixels = px;
    }
    if (c->sort_bins && !fs.sort_table.p) {
        if ((st = dev_alloc(c, fs.sort_table, (size_t)kSortMaxBins * kSortBlocks * 4))) return st;
        if ((st = dev_alloc(c, fs.sort_total, (size_t)kSortMaxBins * 4))) return st;
    }
    if (!fs.counts.p) {
        if ((st = dev_alloc(c, fs.counts, kWfCountAllocBytes))) return st;
        HIPC(c, hipHostMalloc((void**)&W.h_counts, kWfCountAllocBytes, 0));
        for (auto& e : W.ev) HIPC(c, hipEventCreate(&e));
        for (auto& e : fs.wft.ev) HIPC(c, hipEventCreate(&e));
        for (auto& e : W.param_ev) HIPC(c, hipEventCreate(&e));
        if ((st = dev_alloc(c, fs.params, sizeof(FrameParams)))) return st;
        HIPC(c, hipHostMalloc((void**)&W.h_params, sizeof(FrameParams) * WavefrontBuffers::kParamSlots, 0));
        W.d_params = (FrameParams*)fs.params.p;
    }
    W.qc[0] = (float4*)fs.qc.p;
    W.qc[1] = (float4*)fs.qc.p + W.queue_entries;
    W.p_accum = (float4*)fs.accum.p;
    W.p_meta = (uint4*)fs.meta.p;
    W.q[0] = (float4*)fs.q0.p;
    W.q[1] = (float4*)fs.q1.p;
    W.hits = (float4*)fs.hits.p;
    W.sq = (float4*)fs.sq.p;
    W.counts = (uint32_t*)fs.counts.p;
    W.tstamp = (unsigned long long*)((char*)fs.counts.p + kWfTsOffset);
    W.h_tstamp = (unsigned long long*)((char*)W.h_counts + kWfTsOffset);
    W.px_extra = (uint2*)fs.extra.p;
    W.sorted = (float4*)fs.sorted.p;
    W.sort_table = (uint32_t*)fs.sort_table.p;
    W.sort_total = (uint32_t*)fs.sort_total.p;
    return RT_OK;
}

static hipStream_t slot_stream(rt_ctx* c, int k) { return k == 0 ? c->stream : c->slot[k].own_stream; }

// Waits for every frame in flight.  Everything that changes what frames read (scene, BVH,
// targets, transforms) runs after it, so a frame never sees a half-updated scene.
static rt_status drain_frames(rt_ctx* c) {
    if (c->ustream) HIPC(c, hipStreamSynchronize(c->ustream));
    for (int k = 0; k < kMaxSlots; ++k)
        if (c->slot[k].used) {
            HIPC(c, hipStreamSynchronize(slot_stream(c, k)));
            HIPC(c, hipEventSynchronize(c->slot[k].done));
        }
    return RT_OK;
}

// Before a geometry update: the first one after a frame switches to the other generation, once the
// frames still reading it have finished, seeded with a copy of the current one (on the update
// stream; frames keep reading the current generation meanwhile).
static rt_status begin_update(rt_ctx* c) {
    if (c->gdirty) return RT_OK;
    const int w = c->next_gen();
    for (const FrameSlot& f : c->slot)
        if (f.used && f.gen == w) HIPC(c, hipEventSynchronize(f.done));
    Geo& src = c->geo[c->gcur];
    Geo& dst = c->geo[w];
    for (int i = 0; i < 10; ++i) {
        if (rt_status st = dev_alloc(c, *dst.all[i], src.all[i]->bytes)) return st;
        if (src.all[i]->bytes)
            HIPC(c, hipMemcpyAsync(dst.all[i]->p, src.all[i]->p, src.all[i]->bytes, hipMemcpyDeviceToDevice, c->ustream));
    }
    dst.num_nodes8 = src.num_nodes8;
    c->gdirty = true;
    return RT_OK;
}

extern "C" {

const char* rt_version(void) {
    return "rt_hip 0.4 (gfx950, SAH-DP compressed 8-wide BVH, PLOC device build, wavefront with frames in flight + megakernel, USD + PNG ingest, denoised present)";
}

const char* rt_last_error(const rt_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

rt_status rt_create(const rt_opts* opts, rt_ctx** out) {
    if (!out) FAIL((rt_ctx*)nullptr, RT_ERR_INVALID_ARG, "out is null");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) FAIL((rt_ctx*)nullptr, RT_ERR_NO_DEVICE, "no HIP device");
    rt_ctx* c = new (std::nothrow) rt_ctx();
    if (!c) FAIL((rt_ctx*)nullptr, RT_ERR_OUT_OF_MEMORY, "alloc ctx");
    if (opts) {
        c->device = opts->device;
        c->pipeline = opts->pipeline;
        c->tail_paths = opts->tail_paths;
        c->sort_bins = opts->sort_bins == 0 ? kSortBinsDefault : std::max(opts->sort_bins, 0);
    }
    if (c->device < 0 || c->device >= ndev) { delete c; FAIL((rt_ctx*)nullptr, RT_ERR_INVALID_ARG, "bad device ordinal"); }
    if (c->pipeline != RT_PIPELINE_MEGAKERNEL && c->pipeline != RT_PIPELINE_WAVEFRONT) {
        delete c;
        FAIL((rt_ctx*)nullptr, RT_ERR_INVALID_ARG, "bad pipeline");
    }
    if (c->sort_bins && (c->sort_bins < kSortMinBins || c->sort_bins > kSortMaxBins ||
                         (c->sort_bins & (c->sort_bins - 1)))) {
        delete c;
        FAIL((rt_ctx*)nullptr, RT_ERR_INVALID_ARG, "sort_bins must be a power of two in [1024, 4096]");
    }
    if (opts && opts->frames_in_flight > 0) c->max_in_flight = std::min(opts->frames_in_flight, kMaxSlots);
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    for (FrameSlot& f : c->slot) {
        if (e == hipSuccess) e = hipEventCreate(&f.ev0);
        if (e == hipSuccess) e = hipEventCreate(&f.ev1);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&f.done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipHostMalloc((void**)&f.h_counters, sizeof(unsigned long long) * kCounterWords, 0);
    }
    for (int k = 1; k < kMaxSlots; ++k)
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->slot[k].own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->scene_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->ustream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->uev, hipEventDisableTiming);
    if (e != hipSuccess) {
        g_err = std::string("HIP init: ") + hipGetErrorString(e);
        delete c;
        return RT_ERR_HIP;
    }
    c->stream = c->own_stream;
    auto tab = halton_table();
    rt_status st = dev_upload(c, c->d_halton, tab.data(), tab.size() * sizeof(HaltonDim));
    for (FrameSlot& f : c->slot)
        if (!st) st = dev_alloc(c, f.counters, sizeof(unsigned long long) * kCounterWords);

    if (!st && hipStreamSynchronize(c->stream) != hipSuccess) st = RT_ERR_HIP;
    if (st) {
        g_err = c->err;
        rt_destroy(c);
        return st;
    }
    *out = c;
    return RT_OK;
}

rt_status rt_destroy(rt_ctx* c) {
    if (!c) return RT_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->ustream) (void)hipStreamSynchronize(c->ustream);
    for (FrameSlot& f : c->slot)
        if (f.own_stream) (void)hipStreamSynchronize(f.own_stream);
    DevBuf* all[] = {&c->d_rest_pos, &c->d_rest_nrm, &c->d_jidx, &c->d_jw,
                     &c->d_joints, &c->d_tri_info, &c->d_mat, &c->d_lights, &c->d_halton,
                     &c->d_slot_to_tri, &c->d_levels, &c->d_maxabs, &c->d_random, &c->d_accum[0],
                     &c->d_accum[1], &c->d_lbvh_scratch, &c->d_tex_texels, &c->d_tex_info,
                     &c->d_mat_tex, &c->d_uv, &c->d_tex_lut, &c->d_hist[0], &c->d_hist[1], &c->d_hdepth[0],
                     &c->d_hdepth[1], &c->d_present_out, &c->d_present_thr, &c->d_den[0], &c->d_den[1],
                     &c->d_den[2], &c->d_den[3], &c->d_half, &c->d_cost};
    for (auto* b : all) dev_free(*b);
    for (DevBuf& b : c->d_motion) dev_free(b);
    for (Geo& g : c->geo)
        for (DevBuf* b : g.all) dev_free(*b);
    if (c->uev) (void)hipEventDestroy(c->uev);
    if (c->ustream) (void)hipStreamDestroy(c->ustream);
    if (c->h_lbvh) (void)hipHostFree(c->h_lbvh);
    if (c->h_cost) (void)hipHostFree(c->h_cost);
    if (c->cost_ev) (void)hipEventDestroy(c->cost_ev);
    if (c->scene_ev) (void)hipEventDestroy(c->scene_ev);
    for (FrameSlot& f : c->slot) {
        for (DevBuf* b : f.bufs) dev_free(*b);
        if (f.h_counters) (void)hipHostFree(f.h_counters);
        if (f.wf.h_counts) (void)hipHostFree(f.wf.h_counts);
        for (auto& e : f.wf.ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : f.wft.ev)
            if (e) (void)hipEventDestroy(e);
        for (hipGraphExec_t x : f.wft.exec)
            if (x) (void)hipGraphExecDestroy(x);
        for (auto& e : f.wf.param_ev)
            if (e) (void)hipEventDestroy(e);
        if (f.wf.h_params) (void)hipHostFree(f.wf.h_params);
        for (hipEvent_t ev : {f.ev0, f.ev1, f.done})
            if (ev) (void)hipEventDestroy(ev);
        if (f.own_stream) (void)hipStreamDestroy(f.own_stream);
    }
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return RT_OK;
}

rt_status rt_set_stream(rt_ctx* c, void* s) {
    if (!c) FAIL(c, RT_ERR_INVALID_ARG, "null ctx");
    rt_status st = drain_frames(c);
    if (st) return st;
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return RT_OK;
}

// Texture path: the texel pool, its table, every material slot's texture
// ids and the per-vertex UVs (Model.vertexDescriptor's zero default when a mesh has none,
// Model.swift:329-333).  Nothing is uploaded for an untextured scene.
static rt_status upload_textures(rt_ctx* c, const rt_scene_desc* sd) {
    const uint32_t slots = (uint32_t)c->max_sub * sd->mesh_count;
    std::vector<int4> mt(2 * (size_t)slots, make_int4(0, -1, -1, -1));
    bool textured = false;
    for (uint32_t m = 0; m < sd->mesh_count; ++m)
        for (uint32_t s = 0; s < sd->meshes[m].submesh_count; ++s) {
            const rt_submesh_desc& sm = sd->meshes[m].submeshes[s];
            uint32_t flags = sm.material.textureFlags & ~(1u << 4);   // ENABLE_AO = 0
            if (!flags) continue;
            textured = true;
            int t[8];
            for (int k = 0; k < 8; ++k) t[k] = (k < RT_TEXTURE_SLOTS && (flags >> k & 1u)) ? sm.textures[k] : -1;
            const size_t slot = (size_t)m * c->max_sub + s;
            mt[2 * slot] = make_int4((int)flags, t[0], t[1], t[2]);
            mt[2 * slot + 1] = make_int4(t[3], t[4], t[5], t[6]);
        }
    c->textured = textured;
    if (!textured) return RT_OK;
    std::vector<uint4> info(sd->texture_count);
    std::vector<uint8_t> texels;
    uint64_t off = 0;
    for (uint32_t t = 0; t < sd->texture_count; ++t) {
        const rt_texture_desc& td = sd->textures[t];
        info[t] = make_uint4((uint32_t)off, td.width, td.height, 0u);
        off += (uint64_t)td.width * td.height;
    }
    texels.resize(off * 4);
    for (uint32_t t = 0; t < sd->texture_count; ++t)
        std::memcpy(&texels[4 * (size_t)info[t].x], sd->textures[t].rgba8, 4 * (size_t)info[t].y * info[t].z);
    std::vector<float2> uv(c->num_verts, make_float2(0.0f, 0.0f));
    uint32_t vbase = 0;
    for (uint32_t m = 0; m < sd->mesh_count; ++m) {
        const rt_mesh_desc& md = sd->meshes[m];
        if (md.uvs)
            for (uint32_t v = 0; v < md.vertex_count; ++v) uv[vbase + v] = make_float2(md.uvs[v].x, md.uvs[v].y);
        vbase += md.vertex_count;
    }
    // texel byte -> float: [0, 256) linear b / 255, [256, 512) sRGB EOTF (MTKTextureLoader .SRGB)
    float lut[512];
    for (int b = 0; b < 256; ++b) {
        const double v = b / 255.0;
        lut[b] = (float)v;
        lut[256 + b] = (float)(v <= 0.04045 ? v / 12.92 : std::pow((v + 0.055) / 1.055, 2.4));
    }
    rt_status st;
    if ((st = dev_upload(c, c->d_tex_texels, texels.data(), texels.size()))) return st;
    if ((st = dev_upload(c, c->d_tex_info, info.data(), info.size() * sizeof(uint4)))) return st;
    if ((st = dev_upload(c, c->d_mat_tex, mt.data(), mt.size() * sizeof(int4)))) return st;
    if ((st = dev_upload(c, c->d_uv, uv.data(), uv.size() * sizeof(float2)))) return st;
    if ((st = dev_upload(c, c->d_tex_lut, lut, sizeof lut))) return st;
    return RT_OK;
}

rt_status rt_scene_upload(rt_ctx* c, const rt_scene_desc* sd) {
    if (!c || !sd) FAIL(c, RT_ERR_INVALID_ARG, "null argument");
    if (rt_status dst = drain_frames(c)) return dst;
    HIPC(c, hipSetDevice(c->device));
    if (sd->mesh_count == 0) FAIL(c, RT_ERR_INVALID_ARG, "scene has no meshes");
    if (sd->light_count == 0 || !sd->lights) FAIL(c, RT_ERR_INVALID_ARG, "scene has no lights");
    if (sd->mesh_count >= (1u << 24)) FAIL(c, RT_ERR_UNSUPPORTED, "too many meshes");
    int max_sub = 1;
    uint64_t nv = 0, nt = 0;
    for (uint32_t m = 0; m < sd->mesh_count; ++m) {
        const rt_mesh_desc& md = sd->meshes[m];
        if (!md.positions || !md.normals) FAIL(c, RT_ERR_INVALID_ARG, "mesh without positions/normals");
        if (md.submesh_count == 0 || !md.submeshes) FAIL(c, RT_ERR_INVALID_ARG, "mesh without submeshes");
        if (md.submesh_count > 256) FAIL(c, RT_ERR_UNSUPPORTED, "more than 256 submeshes in a mesh");
        if (md.joint_count && (!md.joint_indices || !md.joint_weights)) FAIL(c, RT_ERR_INVALID_ARG, "skinned mesh without joint streams");
        max_sub = std::max(max_sub, (int)md.submesh_count);
        nv += md.vertex_count;
        for (uint32_t s = 0; s < md.submesh_count; ++s) {
            const rt_submesh_desc& sm = md.submeshes[s];
            if (sm.index_count % 3) FAIL(c, RT_ERR_INVALID_ARG, "index count not a multiple of 3");
            if (sm.index_count && !sm.indices) FAIL(c, RT_ERR_INVALID_ARG, "null indices");
            for (int k = 0; k < RT_TEXTURE_SLOTS; ++k)
                if (k != 4 && (sm.material.textureFlags >> k & 1u) &&   // the AO slot is never sampled
                    (sm.textures[k] < 0 || (uint32_t)sm.textures[k] >= sd->texture_count || !sd->textures))
                    FAIL(c, RT_ERR_INVALID_ARG, "textured material without a valid texture for a flagged slot");
            for (uint32_t i = 0; i < sm.index_count; ++i)
                if (sm.indices[i] >= md.vertex_count) FAIL(c, RT_ERR_INVALID_ARG, "index out of range");
            nt += sm.index_count / 3;
        }
    }
    if (nt >= (1ull << 31) || nv >= (1ull << 32)) FAIL(c, RT_ERR_UNSUPPORTED, "scene too large");
    uint64_t ntexels = 0;
    for (uint32_t t = 0; t < sd->texture_count; ++t) {
        const rt_texture_desc& td = sd->textures[t];
        if (!td.rgba8 || td.width == 0 || td.height == 0) FAIL(c, RT_ERR_INVALID_ARG, "bad texture");
        ntexels += (uint64_t)td.width * td.height;
    }
    if (ntexels >= (1ull << 32)) FAIL(c, RT_ERR_UNSUPPORTED, "texture pool above 2^32 texels");
    c->max_sub = max_sub;
    c->num_inst = sd->mesh_count;
    c->num_tris = (uint32_t)nt;
    c->num_verts = (uint32_t)nv;
    c->h_pos.assign(nv, make_float4(0, 0, 0, 0));
    c->h_nrm.assign(nv, make_float4(0, 0, 0, 0));
    c->h_tri_info.resize(nt);
    c->h_inst.assign(12 * (size_t)sd->mesh_count, 0.0f);
    Material zero_mat;
    std::memset(&zero_mat, 0, sizeof zero_mat);
    c->h_mat.assign((size_t)max_sub * sd->mesh_count, zero_mat);
    c->meshes.assign(sd->mesh_count, MeshInfo());
    c->h_world.resize(9 * nt);
    uint32_t vbase = 0, tri = 0;
    std::vector<uint16_t> jidx;
    std::vector<float> jw;
    bool any_skin = false;
    for (uint32_t m = 0; m < sd->mesh_count; ++m) {
        const rt_mesh_desc& md = sd->meshes[m];
        MeshInfo& mi = c->meshes[m];
        mi.vbase = vbase;
        mi.vcount = md.vertex_count;
        mi.tbase = tri;
        mi.joint_count = md.joint_count;
        mi.skinned = md.joint_count > 0;
        any_skin |= mi.skinned;
        std::memcpy(&c->h_inst[12 * m], &md.transform, 48);
        for (uint32_t v = 0; v < md.vertex_count; ++v) {
            const rt_float3& p = md.positions[v];
            const rt_float3& n = md.normals[v];
            c->h_pos[vbase + v] = make_float4(p.x, p.y, p.z, 0.0f);
            c->h_nrm[vbase + v] = make_float4(n.x, n.y, n.z, 0.0f);
        }
        for (uint32_t s = 0; s < md.submesh_count; ++s) {
            const rt_submesh_desc& sm = md.submeshes[s];
            c->h_mat[(size_t)m * max_sub + s] = sm.material;
            for (uint32_t k = 0; k < sm.index_count / 3; ++k) {
                uint4 ti;
                ti.x = vbase + sm.indices[3 * k + 0];
                ti.y = vbase + sm.indices[3 * k + 1];
                ti.z = vbase + sm.indices[3 * k + 2];
                ti.w = (m << 8) | s;
                c->h_tri_info[tri] = ti;
                const float* M = &c->h_inst[12 * m];
                xform_host(M, c->h_pos[ti.x], &c->h_world[9 * (size_t)tri + 0]);
                xform_host(M, c->h_pos[ti.y], &c->h_world[9 * (size_t)tri + 3]);
                xform_host(M, c->h_pos[ti.z], &c->h_world[9 * (size_t)tri + 6]);
                ++tri;
            }
        }
        vbase += md.vertex_count;
        mi.tcount = tri - mi.tbase;
    }
    c->h_lights.assign(sd->lights, sd->lights + sd->light_count);
    rt_status st;
    if ((st = upload_textures(c, sd))) return st;
    if ((st = dev_upload(c, c->G().pos, c->h_pos.data(), nv * 16))) return st;
    if ((st = dev_upload(c, c->G().prev_pos, c->h_pos.data(), nv * 16))) return st;  // previousPositions = positions (SubMesh.swift:60)
    if ((st = dev_upload(c, c->G().nrm, c->h_nrm.data(), nv * 16))) return st;
    if ((st = dev_upload(c, c->d_tri_info, c->h_tri_info.data(), nt * 16))) return st;
    if ((st = dev_alloc(c, c->G().tri_nrm, nt * 64))) return st;
    launch_tri_nrm((const uint4*)c->d_tri_info.p, (const float4*)c->G().nrm.p, (float4*)c->G().tri_nrm.p, 0,
                   (uint32_t)nt, c->stream);
    c->ctx_work++;
    HIPC(c, hipGetLastError());
    if ((st = dev_upload(c, c->G().inst, c->h_inst.data(), c->h_inst.size() * 4))) return st;
    if ((st = dev_upload(c, c->G().prev_inst, c->h_inst.data(), c->h_inst.size() * 4))) return st;
    if ((st = dev_upload(c, c->d_mat, c->h_mat.data(), c->h_mat.size() * sizeof(Material)))) return st;
    if ((st = dev_upload(c, c->d_lights, c->h_lights.data(), c->h_lights.size() * sizeof(Light)))) return st;
    if (any_skin) {
        // rest pose + joint streams of every skinned mesh (positions of static meshes unused)
        jidx.assign(4 * (size_t)nv, 0);
        jw.assign(4 * (size_t)nv, 0.0f);
        uint32_t maxj = 0;
        for (uint32_t m = 0; m < sd->mesh_count; ++m) {
            const rt_mesh_desc& md = sd->meshes[m];
            if (!md.joint_count) continue;
            maxj = std::max(maxj, md.joint_count);
            std::memcpy(&jidx[4 * (size_t)c->meshes[m].vbase], md.joint_indices, 8 * (size_t)md.vertex_count);
            std::memcpy(&jw[4 * (size_t)c->meshes[m].vbase], md.joint_weights, 16 * (size_t)md.vertex_count);
        }
        if ((st = dev_upload(c, c->d_rest_pos, c->h_pos.data(), nv * 16))) return st;
        if ((st = dev_upload(c, c->d_rest_nrm, c->h_nrm.data(), nv * 16))) return st;
        if ((st = dev_upload(c, c->d_jidx, jidx.data(), jidx.size() * 2))) return st;
        if ((st = dev_upload(c, c->d_jw, jw.data(), jw.size() * 4))) return st;
        if ((st = dev_alloc(c, c->d_joints, (size_t)maxj * 64))) return st;
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    c->scene_ready = true;
    c->bvh_ready = false;
    c->inst_moved = c->skin_moved = c->last_moving = false;
    return RT_OK;
}

// The node-area sum of the current generation's tree (launch_bvh_cost) on the update stream: read
// back at once (sync = true, after a build) or into the pinned word with an event (after a refit).
static rt_status bvh_cost(rt_ctx* c, bool sync) {
    if (rt_status st = dev_alloc(c, c->d_cost, 4)) return st;
    if (!c->h_cost) HIPC(c, hipHostMalloc((void**)&c->h_cost, 16, 0));
    if (!c->cost_ev) HIPC(c, hipEventCreateWithFlags(&c->cost_ev, hipEventDisableTiming));
    launch_bvh_cost((const float*)c->G().node_box.p, c->num_nodes8, (float*)c->d_cost.p, c->ustream);
    HIPC(c, hipGetLastError());
    HIPC(c, hipMemcpyAsync(c->h_cost, c->d_cost.p, 4, hipMemcpyDeviceToHost, c->ustream));
    if (sync) {
        HIPC(c, hipStreamSynchronize(c->ustream));
        c->cost_built = *c->h_cost;   // cost_refit keeps the last refit's figure (rt_stats)
        c->cost_pending = false;
    } else {
        HIPC(c, hipEventRecord(c->cost_ev, c->ustream));
        c->cost_pending = true;
    }
    return RT_OK;
}

// rt_tuning.refit_rebuild_pct: 0 = the default, < 0 = never
constexpr int kRefitRebuildPctDefault = 150;
static int refit_rebuild_pct(const rt_ctx* c) {
    const int p = c->tuning_req.refit_rebuild_pct;
    return p == 0 ? kRefitRebuildPctDefault : p;
}

// Once the last refit's node-area sum has arrived: if it grew past refit_rebuild_pct percent of
// the last build's, rebuild on the device from the current geometry (the reference rebuilds its
// acceleration structures where a refit is not enough, Renderer.swift:1252-1277).  Images do not
// depend on the tree (conservative boxes): this only restores traversal speed.
static rt_status check_refit_quality(rt_ctx* c, bool* rebuilt) {
    *rebuilt = false;
    if (!c->cost_pending || hipEventQuery(c->cost_ev) != hipSuccess) return RT_OK;
    c->cost_pending = false;
    c->cost_refit = *c->h_cost;
    const int pct = refit_rebuild_pct(c);
    if (pct <= 0 || !(c->cost_built > 0.0f) || !(c->cost_refit * 100.0f > c->cost_built * (float)pct)) return RT_OK;
    if (rt_status st = rt_bvh_build_device(c)) return st;
    c->auto_rebuilds++;
    *rebuilt = true;
    return RT_OK;
}

rt_status rt_bvh_build(rt_ctx* c) {
    if (!c) FAIL(c, RT_ERR_INVALID_ARG, "null ctx");
    if (!c->scene_ready) FAIL(c, RT_ERR_STATE, "rt_bvh_build before rt_scene_upload");
    HIPC(c, hipSetDevice(c->device));
    // into the update generation: frames in flight keep theirs (and their tree)
    if (rt_status ust = begin_update(c)) return ust;
    HIPC(c, hipStreamSynchronize(c->ustream));
    // current world-space triangles (may have been skinned / re-transformed on the device)
    if (c->world_dirty) {
        HIPC(c, hipMemcpy(c->h_pos.data(), c->G().pos.p, (size_t)c->num_verts * 16, hipMemcpyDeviceToHost));
        for (uint32_t t = 0; t < c->num_tris; ++t) {
            const uint4& ti = c->h_tri_info[t];
            const float* M = &c->h_inst[12 * (ti.w >> 8)];
            xform_host(M, c->h_pos[ti.x], &c->h_world[9 * (size_t)t + 0]);
            xform_host(M, c->h_pos[ti.y], &c->h_world[9 * (size_t)t + 3]);
            xform_host(M, c->h_pos[ti.z], &c->h_world[9 * (size_t)t + 6]);
        }
        c->world_dirty = false;
    }
    // the size the host and device builders are tested to (the device build's 64-bit Morton keys
    // carry the triangle id beside the Morton bits)
    if (c->num_tris >= (1u << 26)) FAIL(c, RT_ERR_UNSUPPORTED, "more than 2^26 triangles");
    if (!build_bvh8_fit(c->h_world.data(), c->num_tris, c->bvh, c->bvh8))
        FAIL(c, RT_ERR_UNSUPPORTED, "BVH deeper than the traversal stack at every depth limit");
    if (c->bvh8.nodes.size() >= (1u << 23)) FAIL(c, RT_ERR_UNSUPPORTED, "BVH too large (2^23 nodes)");
    const uint32_t n = c->num_tris;
    std::vector<float> tris((size_t)kTriFloats * n);   // 64-B records (rt_device.h)
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t id = c->bvh8.tri_order[k];
        tri_store(&tris[(size_t)kTriFloats * k], &c->h_world[9 * (size_t)id], id);
    }
    // nodes grouped by depth for the level-synchronous refit (BFS order: parent < child)
    const size_t nn = c->bvh8.nodes.size();
    std::vector<int> depth(nn, 0);
    int maxd = 0;
    for (size_t k = 1; k < nn; ++k) {
        depth[k] = depth[c->bvh8.parent[k]] + 1;
        maxd = std::max(maxd, depth[k]);
    }
    c->level_off.assign(maxd + 2, 0);
    for (int d : depth) c->level_off[d + 1]++;
    for (int d = 0; d <= maxd; ++d) c->level_off[d + 1] += c->level_off[d];
    c->level_nodes.assign(nn, 0);
    std::vector<uint32_t> fill(c->level_off.begin(), c->level_off.end() - 1);
    for (size_t k = 0; k < nn; ++k) c->level_nodes[fill[depth[k]]++] = (uint32_t)k;
    rt_status st;
    Geo& g = c->G();
    hipStream_t us = c->ustream;
    if ((st = dev_upload(c, g.tris, tris.data(), tris.size() * 4, us))) return st;
    if ((st = dev_upload(c, g.nodes, c->bvh8.nodes.data(), nn * sizeof(Bvh8Node), us))) return st;
    if ((st = dev_upload(c, g.node_box, c->bvh8.node_box.data(), c->bvh8.node_box.size() * 4, us))) return st;
    if ((st = dev_upload(c, c->d_slot_to_tri, c->bvh8.tri_order.data(), (size_t)n * 4, us))) return st;
    if ((st = dev_upload(c, c->d_levels, c->level_nodes.data(), c->level_nodes.size() * 4, us))) return st;
    // hit-sort keys: the leaf-order bin of every triangle (DevScene::tri_bin)
    std::vector<uint16_t> tri_bin(n);
    for (uint32_t k = 0; k < n; ++k) tri_bin[c->bvh8.tri_order[k]] = (uint16_t)(((uint64_t)k * kSortMaxBins) / n);
    if ((st = dev_upload(c, g.tri_bin, tri_bin.data(), (size_t)n * 2, us))) return st;
    c->num_nodes8 = (uint32_t)nn;
    if ((st = bvh_cost(c, true))) return st;
    HIPC(c, hipStreamSynchronize(us));   // the host arrays are the copies' sources
    g.num_nodes8 = (uint32_t)nn;
    c->num_nodes8 = (uint32_t)nn;
    c->bvh_ready = true;
    return RT_OK;
}

rt_status rt_bvh_build_device(rt_ctx* c) {
    if (!c) FAIL(c, RT_ERR_INVALID_ARG, "null ctx");
    if (!c->scene_ready) FAIL(c, RT_ERR_STATE, "rt_bvh_build_device before rt_scene_upload");
    if (c->num_tris < 2) return rt_bvh_build(c);   // nothing to sort: the host path is exact and instant
    if (c->num_tris >= (1u << 26)) FAIL(c, RT_ERR_UNSUPPORTED, "more than 2^26 triangles");
    HIPC(c, hipSetDevice(c->device));
    // into the update generation on the update stream: frames in flight keep their tree
    rt_status st = begin_update(c);
    if (st) return st;
    const uint32_t n = c->num_tris;
    hipStream_t us = c->ustream;
    if ((st = dev_alloc(c, c->d_lbvh_scratch, lbvh_scratch_bytes(n)))) return st;
    Geo& g = c->G();
    if ((st = dev_alloc(c, g.nodes, (size_t)n * sizeof(Bvh8Node)))) return st;
    if ((st = dev_alloc(c, g.node_box, (size_t)n * 6 * sizeof(float)))) return st;
    if ((st = dev_alloc(c, c->d_slot_to_tri, (size_t)n * 4))) return st;
    if ((st = dev_alloc(c, g.tri_bin, (size_t)n * 2))) return st;
    if ((st = dev_alloc(c, c->d_levels, (size_t)n * 4))) return st;
    if ((st = dev_alloc(c, g.tris, (size_t)n * kTriFloats * 4))) return st;
    if ((st = dev_alloc(c, c->d_maxabs, 4))) return st;
    if (!c->h_lbvh) HIPC(c, hipHostMalloc((void**)&c->h_lbvh, 16, 0));
    LbvhInput in{(const float4*)g.pos.p, (const uint4*)c->d_tri_info.p, (const float*)g.inst.p, n};
    // PLOC topology + SAH-DP collapse by default; RT_DEVICE_BVH=lbvh selects the radix tree, whose
    // faster build wins for a small scene rebuilt every frame
    in.ploc = c->tuning_req.device_bvh == 1 ? 0 : 1;   // rt_tuning.device_bvh: 1 = the LBVH radix tree
    LbvhOutput out{(Bvh8Node*)g.nodes.p, (float*)g.node_box.p, (uint32_t*)c->d_slot_to_tri.p,
                   (uint16_t*)g.tri_bin.p, (uint32_t*)c->d_levels.p, c->h_lbvh};
    LbvhResult res;
    const char* err = nullptr;
    if (!lbvh_build(in, out, c->d_lbvh_scratch.p, us, &res, &err)) {
        c->bvh_ready = false;
        FAIL(c, RT_ERR_UNSUPPORTED, std::string("device BVH build: ") + (err ? err : "?"));
    }
    // world-space triangles in the new slot order
    HIPC(c, hipMemsetAsync(c->d_maxabs.p, 0, 4, us));
    launch_flatten((const uint4*)c->d_tri_info.p, (const uint32_t*)c->d_slot_to_tri.p, (const float4*)g.pos.p,
                   (const float*)g.inst.p, (float*)g.tris.p, n, (unsigned*)c->d_maxabs.p, us);
    HIPC(c, hipGetLastError());
    HIPC(c, hipStreamSynchronize(us));
    if (res.num_nodes >= (1u << 23)) FAIL(c, RT_ERR_UNSUPPORTED, "BVH too large (2^23 nodes)");
    c->level_off = res.level_off;
    c->bvh8 = Bvh8Result();            // the host copy describes the host builder's trees only
    c->bvh8.pad = res.pad;
    c->bvh8.max_depth = res.max_depth;
    c->num_nodes8 = res.num_nodes;
    g.num_nodes8 = res.num_nodes;
    c->bvh_ready = true;
    return bvh_cost(c, true);
}

rt_status rt_bvh_refit(rt_ctx* c) {
    if (!c) FAIL(c, RT_ERR_INVALID_ARG, "null ctx");
    if (!c->bvh_ready) FAIL(c, RT_ERR_STATE, "rt_bvh_refit before rt_bvh_build");
    HIPC(c, hipSetDevice(c->device));
    bool rebuilt = false;
    if (rt_status qst = check_refit_quality(c, &rebuilt)) return qst;
    if (rebuilt) return RT_OK;         // the new tree is built from the current geometry
    rt_status st = begin_update(c);   // frames in flight keep their generation
    if (!st) st = dev_alloc(c, c->d_maxabs, 4);
    if (st) return st;
    Geo& g = c->G();
    HIPC(c, hipMemsetAsync(c->d_maxabs.p, 0, 4, c->ustream));
    launch_flatten((const uint4*)c->d_tri_info.p, (const uint32_t*)c->d_slot_to_tri.p, (const float4*)g.pos.p,
                   (const float*)g.inst.p, (float*)g.tris.p, c->num_tris, (unsigned*)c->d_maxabs.p, c->ustream);
    for (int d = (int)c->level_off.size() - 2; d >= 0; --d) {
        uint32_t off = c->level_off[d], cnt = c->level_off[d + 1] - off;
        launch_refit8_level((Bvh8Node*)g.nodes.p, (float*)g.node_box.p, (const float*)g.tris.p,
                            (const uint32_t*)c->d_levels.p + off, cnt, c->bvh8.pad, (const unsigned*)c->d_maxabs.p,
                            c->ustream);
    }
    HIPC(c, hipGetLastError());
    // the refitted tree's node-area sum, read back without a host wait (check_refit_quality)
    if (refit_rebuild_pct(c) > 0) return bvh_cost(c, false);
    return RT_OK;
}

rt_status rt_set_instance_transforms(rt_ctx* c, const rt_packed_float4x3* t, uint32_t count) {
    if (!c || !t) FAIL(c, RT_ERR_INVALID_ARG, "null argument");
    if (!c->scene_ready || count != c->num_inst) FAIL(c, RT_ERR_INVALID_ARG, "transform count != mesh count");
    HIPC(c, hipSetDevice(c->device));
    if (rt_status st = begin_update(c)) return st;   // frames in flight keep their generation
    Geo& g = c->G();
    // prev <- cur (Renderer.swift:939-944), then the new transforms
    HIPC(c, hipMemcpyAsync(g.prev_inst.p, g.inst.p, c->h_inst.size() * 4, hipMemcpyDeviceToDevice, c->ustream));
    c->inst_moved = std::memcmp(c->h_inst.data(), t, (size_t)count * 48) != 0;
    std::memcpy(c->h_inst.data(), t, (size_t)count * 48);
    HIPC(c, hipMemcpyAsync(g.inst.p, c->h_inst.data(), c->h_inst.size() * 4, hipMemcpyHostToDevice, c->ustream));
    HIPC(c, hipStreamSynchronize(c->ustream));   // h_inst is the copy's source
    c->world_dirty = true;
    return RT_OK;
}

rt_status rt_skin(rt_ctx* c, uint32_t mesh_index, const float* joints, uint32_t joint_count) {
    if (!c || !joints) FAIL(c, RT_ERR_INVALID_ARG, "null argument");
    if (!c->scene_ready || mesh_index >= c->meshes.size()) FAIL(c, RT_ERR_INVALID_ARG, "bad mesh index");
    const MeshInfo& mi = c->meshes[mesh_index];
    if (!mi.skinned) FAIL(c, RT_ERR_INVALID_ARG, "mesh is not skinned");
    if (joint_count != mi.joint_count) FAIL(c, RT_ERR_INVALID_ARG, "joint count mismatch");
    HIPC(c, hipSetDevice(c->device));
    if (rt_status st = begin_update(c)) return st;   // frames in flight keep their generation
    Geo& g = c->G();
    HIPC(c, hipMemcpyAsync(c->d_joints.p, joints, (size_t)joint_count * 64, hipMemcpyHostToDevice, c->ustream));
    // previousPositions <- positions (Renderer.swift:1290-1303)
    HIPC(c, hipMemcpyAsync((float4*)g.prev_pos.p + mi.vbase, (float4*)g.pos.p + mi.vbase, (size_t)mi.vcount * 16,
                           hipMemcpyDeviceToDevice, c->ustream));
    launch_skin((const float4*)c->d_rest_pos.p + mi.vbase, (const float4*)c->d_rest_nrm.p + mi.vbase,
                (const ushort4*)c->d_jidx.p + mi.vbase, (const float4*)c->d_jw.p + mi.vbase, (const float*)c->d_joints.p,
                (float4*)g.pos.p + mi.vbase, (float4*)g.nrm.p + mi.vbase, mi.vcount, c->ustream);
    launch_tri_nrm((const uint4*)c->d_tri_info.p, (const float4*)g.nrm.p, (float4*)g.tri_nrm.p, mi.tbase, mi.tcount,
                   c->ustream);
    HIPC(c, hipGetLastError());
    HIPC(c, hipStreamSynchronize(c->ustream));  // joint upload buffer is reused next call
    c->world_dirty = true;
    c->skin_moved = true;   // conservative: positions may now differ from previousPositions
    return RT_OK;
}

rt_status rt_resize(rt_ctx* c, int32_t w, int32_t h, const uint32_t* offsets) {
    if (!c || !offsets) FAIL(c, RT_ERR_INVALID_ARG, "null argument");
    if (rt_status dst = drain_frames(c)) return dst;
    if (w <= 0 || h <= 0 || (int64_t)w * h > (1ll << 30)) FAIL(c, RT_ERR_INVALID_ARG, "bad size");
    HIPC(c, hipSetDevice(c->device));
    size_t n = (size_t)w * h;
    rt_status st;
    if ((st = dev_upload(c, c->d_random, offsets, n * 4))) return st;
    for (int i = 0; i < 2; ++i) {
        if ((st = dev_alloc(c, c->d_accum[i], n * 16))) return st;
        HIPC(c, hipMemsetAsync(c->d_accum[i].p, 0, n * 16, c->stream));
        c->ctx_work++;
    }
    for (DevBuf& m : c->d_motion) {
        if ((st = dev_alloc(c, m, n * 8))) return st;
        HIPC(c, hipMemsetAsync(m.p, 0, n * 8, c->stream));
    }
    c->motion_cur = 0;
    for (FrameSlot& f : c->slot) {
        if ((st = dev_alloc(c, f.depth, n * 4))) return st;
        HIPC(c, hipMemsetAsync(f.depth.p, 0, n * 4, c->stream));
        dev_free(f.gbuffer);
        dev_free(f.prim_hit);
        f.used = false;
        f.pending = false;
    }
    c->frame_no = 0;
    c->last_slot = 0;
    c->hist_valid = false;
    HIPC(c, hipStreamSynchronize(c->stream));
    c->width = w;
    c->height = h;
    c->read_idx = 0;
    c->last_moving = false;   // motion target cleared
    return RT_OK;
}

int32_t rt_tile_count(int32_t w, int32_t h, const rt_tile_set* t) {
    int ts = (t && t->tile_size > 0) ? t->tile_size : 64;
    int nr = (t && t->nranks > 0) ? t->nranks : 1;
    int rk = (t && t->nranks > 0) ? t->rank : 0;
    int tx = (w + ts - 1) / ts, ty = (h + ts - 1) / ts;
    int total = tx * ty;
    if (rk >= total) return 0;
    return (total - rk + nr - 1) / nr;
}

static rt_status resolve_tiles(rt_ctx* c, const rt_tile_set* t, int& ts, int& rank, int& nranks, int& tiles_x, int& own) {
    ts = (t && t->tile_size > 0) ? t->tile_size : 64;
    nranks = (t && t->nranks > 0) ? t->nranks : 1;
    rank = (t && t->nranks > 0) ? t->rank : 0;
    if (ts % 16 != 0) FAIL(c, RT_ERR_INVALID_ARG, "tile_size must be a multiple of 16");
    if (rank < 0 || rank >= nranks) FAIL(c, RT_ERR_INVALID_ARG, "bad rank");
    tiles_x = (c->width + ts - 1) / ts;
    own = rt_tile_count(c->width, c->height, t);
    return RT_OK;
}

// Folds a finished frame of slot k into rt_stats (its per-frame fields) and the running totals.
// Waits for that frame: called before the slot is reused and from rt_wait, oldest frame first.
static rt_status harvest(rt_ctx* c, int k) {
    FrameSlot& f = c->slot[k];
    if (!f.pending) return RT_OK;
    f.pending = false;
    HIPC(c, hipEventSynchronize(f.done));
    float ms = 0.0f;
    HIPC(c, hipEventElapsedTime(&ms, f.ev0, f.ev1));
    rt_stats& S = c->stats;
    S.last_frame_ms = ms;
    for (float& km : S.kernel_ms) km = 0.0f;
    if (f.wavefront) {
        const char* err = nullptr;
        if (!wavefront_collect(f.wf, f.wft, &f.wfs, &err))
            FAIL(c, RT_ERR_HIP, std::string("wavefront stats: ") + (err ? err : "?"));
        std::memcpy(S.kernel_ms, f.wfs.stage_ms, sizeof S.kernel_ms);
    } else {
        S.kernel_ms[0] = ms;
    }
    S.pipeline = f.wavefront ? RT_PIPELINE_WAVEFRONT : RT_PIPELINE_MEGAKERNEL;
    S.iterations = f.wavefront ? f.wfs.iterations : 0;
    S.trace_rays = f.wavefront ? f.wfs.trace_rays : 0;
    S.trace_launches = f.wavefront ? f.wfs.trace_launches : 0;
    S.trace_ms = f.wavefront ? f.wfs.trace_ms : 0.0f;
    S.trace_dev_ms = f.wavefront ? f.wfs.trace_dev_ms : 0.0f;
    S.trace_dev_launches = f.wavefront ? f.wfs.trace_dev_launches : 0;
    S.finish_dev_ms = f.wavefront ? f.wfs.finish_dev_ms : 0.0f;
    S.finish_dev_launches = f.wavefront ? f.wfs.finish_dev_launches : 0;
    S.trace_closest_rays = f.wavefront ? f.wfs.trace_closest_rays : 0;
    S.finish_launches = f.wavefront ? f.wfs.finish_launches : 0;
    auto total = [&f](int w) {
        unsigned long long t = 0;
        for (int r = 0; r < kCntReplicas; ++r) t += f.h_counters[cnt_word(w, r)];
        return t;
    };
    S.closest_rays = total(kCntClosest);
    S.shadow_rays = total(kCntShadow);
    S.node_visits = total(kCntNodes);
    S.node_visits_lds = 0;
    S.tri_tests = total(kCntTris);
    S.paths = total(kCntPaths);
    S.trace_nodes = f.wavefront ? total(kCntTraceNodes) : 0;
    S.trace_tris = f.wavefront ? total(kCntTraceTris) : 0;
    S.trace_nodes_lds = 0;
    rt_stats& T = c->totals;
    T.frames_total += 1;
    T.total_closest_rays += S.closest_rays;
    T.total_shadow_rays += S.shadow_rays;
    T.total_paths += S.paths;
    T.total_frame_ms += S.last_frame_ms;
    for (int i = 0; i < 7; ++i) T.total_kernel_ms[i] += S.kernel_ms[i];
    T.total_trace_rays += S.trace_rays;
    T.total_trace_closest_rays += S.trace_closest_rays;
    T.total_trace_ms += S.trace_ms;
    T.total_trace_launches += (uint64_t)S.trace_launches;
    T.total_trace_dev_ms += S.trace_dev_ms;
    T.total_trace_dev_launches += (uint64_t)S.trace_dev_launches;
    T.total_finish_dev_ms += S.finish_dev_ms;
    T.total_finish_dev_launches += (uint64_t)S.finish_dev_launches;
    T.total_finish_launches += (uint64_t)S.finish_launches;
    if (f.wavefront) {
        const int gm = f.wfs.graph_mode;   // host-driven frames (run_wavefront without a timeline) count as eager
        (gm == kGraphReplay ? T.total_graph_replays : gm == kGraphCapture ? T.total_graph_captures
         : gm == kGraphFallback ? T.total_graph_fallbacks : T.total_graph_eager) += 1;
    }
    if (total(kCntOverflow)) FAIL(c, RT_ERR_STATE, "traversal stack overflow");
    return RT_OK;
}

rt_status rt_render_frame(rt_ctx* c, const Uniforms* U, const rt_tile_set* tiles) {
    if (!c || !U) FAIL(c, RT_ERR_INVALID_ARG, "null argument");
    if (!c->bvh_ready) FAIL(c, RT_ERR_STATE, "rt_render_frame before rt_bvh_build");
    if (!c->width) FAIL(c, RT_ERR_STATE, "rt_render_frame before rt_resize");
    if (U->width != c->width || U->height != c->height) FAIL(c, RT_ERR_INVALID_ARG, "uniforms size != targets size");
    if (U->lightCount < 1 || U->lightCount > (int)c->h_lights.size()) FAIL(c, RT_ERR_INVALID_ARG, "bad lightCount");
    if (U->maxBounces > RT_MAX_BOUNCES) FAIL(c, RT_ERR_UNSUPPORTED, "maxBounces > 12 exceeds the Halton table");
    if (U->samplesPerPixel > 4096 || U->motionSamplingMaxExtraSamples > 4096) FAIL(c, RT_ERR_INVALID_ARG, "bad spp");
    HIPC(c, hipSetDevice(c->device));
    {   // a refit that degraded the tree past rt_tuning.refit_rebuild_pct: rebuild before this frame
        bool rebuilt = false;
        if (rt_status qst = check_refit_quality(c, &rebuilt)) return qst;
    }
    int ts, rank, nranks, tiles_x, own;
    rt_status st = resolve_tiles(c, tiles, ts, rank, nranks, tiles_x, own);
    if (st) return st;
    size_t n = (size_t)c->width * c->height;
    // DebugTextureModeMotion reads sample 0's motion from later samples of the same pixel
    // (Raytracing.metal:483): only the per-pixel kernel orders samples that way.
    bool wavefront = c->pipeline == RT_PIPELINE_WAVEFRONT && U->debugTextureMode != DebugTextureModeMotion;
    // Frames in flight (Renderer.swift:1406-1409): wavefront frames on the context's own stream
    // rotate over the frames-in-flight slots; a caller's stream and the megakernel keep one.
    //  By default one slot per hardware queue the HIP runtime gives the process (four, eight with
    // GPU_MAX_HW_QUEUES >= 8), as many as fit in kSlotBudget, at least two: the finish tail's
    // latency-bound launch and the bulk rounds of the other frames fill each other's gaps (round 3,
    // C3g 1080p x 4 on one MI355X, 2 / 3 / 4 slots: 7.46-7.49 / 7.91-7.94 / 8.36-8.44 Grays/s;
    // 5 / 6 slots on four queues 7.23-7.28 / 7.59-7.67, 6 / 8 slots on eight queues 8.15-8.24 /
    // 8.34-8.37; configs[1] 720p, 3 / 4 slots: 5.95 / 7.38 in round 2)
    const int spp = std::max(U->samplesPerPixel, 1);
    const int max_extra = U->enableMotionAdaptiveSampling ? std::max(U->motionSamplingMaxExtraSamples, 0) : 0;
    int nfl = 1;
    if (wavefront && c->stream == c->own_stream) {
        const uint64_t frame_paths = (uint64_t)own * ts * ts * (uint64_t)(spp + max_extra);
        const uint64_t slots = frame_paths < kSmallFramePaths ? std::min(4, small_frame_slots()) : small_frame_slots();
        nfl = c->max_in_flight > 0 ? c->max_in_flight
                                   : (int)std::max<uint64_t>(2, std::min<uint64_t>(slots,
                                                                              kSlotBudget / (frame_paths * kSlotBytesPerPath + 1)));
    }
    const int k = c->frame_no > 0 ? (c->last_slot + 1) % nfl : 0;
    FrameSlot& F = c->slot[k];
    const hipStream_t stream = slot_stream(c, k);
    if ((st = harvest(c, k))) return st;   // the slot's previous frame (nfl back) has finished
    // the previous frame, when it runs on the other stream: this frame's history inputs (the
    // accumulation target and motion vectors it wrote) are read after it has finished
    const FrameSlot& prev = c->slot[c->last_slot];
    const bool cross = c->frame_no > 0 && prev.used && (c->last_slot != k || c->tiles_pending);
    // a pack / unpack of the previous frame on another stream: the tiles this frame owns are
    // disjoint from the ones it wrote unless the tile set changed
    const bool retile = ts != c->last_tiles[0] || rank != c->last_tiles[1] || nranks != c->last_tiles[2];
    if (c->tiles_pending && retile && prev.used) HIPC(c, hipStreamWaitEvent(stream, prev.done, 0));
    // scene / target updates enqueued on ctx->stream since this slot last waited for them come
    // first.  Only then: an event recorded on ctx->stream also covers the frame slot 0 has in flight
    // there, and waiting on it every frame held each slot-1..3 frame until that frame had finished
    // (the four slots ran in batches; C3g, 20 steps: 3.64 ms per step).
    if (k != 0 && F.ctx_seen != c->ctx_work) {
        HIPC(c, hipEventRecord(c->scene_ev, c->stream));
        HIPC(c, hipStreamWaitEvent(stream, c->scene_ev, 0));
    }
    F.ctx_seen = c->ctx_work;
    if (c->gdirty) {   // this frame reads the updated generation
        HIPC(c, hipEventRecord(c->uev, c->ustream));
        c->uev_valid = true;
        c->gcur = c->next_gen();
        c->gdirty = false;
    }
    if (nfl != c->cur_nfl) {
        // a different number of frames in flight (a new frame size or tile set): finish the frames
        // in flight, then rotate the geometry over max(2, nfl) generations (from the current one)
        if (c->cur_nfl != 0 && (st = drain_frames(c))) return st;
        c->ngens = std::max(std::max(2, nfl), c->gcur + 1);
        for (int g = c->ngens; g < kGens; ++g)
            for (DevBuf* b : c->geo[g].all) dev_free(*b);
        c->cur_nfl = nfl;
    }
    if (c->uev_valid) HIPC(c, hipStreamWaitEvent(stream, c->uev, 0));
    const Geo& geo = c->geo[c->gcur];
    if (U->enableDenoiseGBuffer && !F.gbuffer.p) {
        if ((st = dev_alloc(c, F.gbuffer, 4 * n * 16))) return st;
        HIPC(c, hipMemsetAsync(F.gbuffer.p, 0, 4 * n * 16, stream));
    }
    DevScene S;
    std::memset(&S, 0, sizeof S);   // no stray padding bytes: the frame-graph key compares S byte for byte
    S.tris = (const float*)geo.tris.p;
    S.nodes8 = (const Bvh8Node*)geo.nodes.p;
    S.tri_info = (const uint4*)c->d_tri_info.p;
    S.pos = (const float4*)geo.pos.p;
    S.prev_pos = (const float4*)geo.prev_pos.p;
    S.nrm = (const float4*)geo.nrm.p;
    S.tri_nrm = (const float4*)geo.tri_nrm.p;
    S.inst = (const float*)geo.inst.p;
    S.prev_inst = (const float*)geo.prev_inst.p;
    S.materials = (const Material*)c->d_mat.p;
    S.lights = (const Light*)c->d_lights.p;
    S.halton = (const HaltonDim*)c->d_halton.p;
    S.tri_bin = (const uint16_t*)geo.tri_bin.p;
    S.max_submeshes = c->max_sub;
    S.num_materials = (int)c->h_mat.size();
    S.num_tris = (int)c->num_tris;
    S.num_nodes8 = (int)geo.num_nodes8;
    S.textured = c->textured ? 1 : 0;
    if (c->textured) {
        S.tex_texels = (const uchar4*)c->d_tex_texels.p;
        S.tex_info = (const uint4*)c->d_tex_info.p;
        S.mat_tex = (const int4*)c->d_mat_tex.p;
        S.uv = (const float2*)c->d_uv.p;
        S.tex_lut = (const float*)c->d_tex_lut.p;
    }
    const int m_prev = c->motion_cur, m_out = wavefront ? (c->motion_cur + 1) % kMotionTargets : c->motion_cur;
    FrameParams P;
    std::memset(&P, 0, sizeof P);
    P.U = *U;
    P.random = (const uint32_t*)c->d_random.p;
    P.accum_in = (const float4*)c->d_accum[c->read_idx].p;
    P.accum_out = (float4*)c->d_accum[1 - c->read_idx].p;
    P.depth = (float*)F.depth.p;
    P.motion = (float2*)c->d_motion[m_out].p;
    P.gbuffer = U->enableDenoiseGBuffer ? (float4*)F.gbuffer.p : nullptr;
    P.prim_hit = nullptr;
    P.motion_prev = nullptr;
    P.counters = (unsigned long long*)F.counters.p;
    P.tile_size = ts;
    P.rank = rank;
    P.nranks = nranks;
    P.tiles_x = tiles_x;
    if (wavefront) {
        if ((st = ensure_wavefront(c, F, (size_t)own * ts * ts, spp, max_extra))) return st;
        if ((st = dev_alloc(c, F.prim_hit, n * 16))) return st;
        P.prim_hit = (uint4*)F.prim_hit.p;
        P.motion_prev = (const float2*)c->d_motion[m_prev].p;
    }
    HIPC(c, hipMemsetAsync(F.counters.p, 0, sizeof(unsigned long long) * kCounterWords, stream));
    F.gbuf_written = U->enableDenoiseGBuffer != 0;
    // extra samples can only be non-zero when something moved in this frame or the previous one
    const bool moving = c->inst_moved || c->skin_moved ||
                        std::memcmp(&U->camera, &U->previousCamera, sizeof(Camera)) != 0;
    const bool extra_pass = moving || c->last_moving;
    c->last_moving = moving;
    HIPC(c, hipEventRecord(F.ev0, stream));
    F.wft.pending = false;
    if (wavefront) {
        const char* err = nullptr;
        F.wfs = WfFrameStats{};
        // finish threshold: with frames in flight the next frames' bulk rounds overlap this
        // frame's tail, so more bulk rounds and a shorter tail pay (kTailInFlight: C3g, 2 in
        // flight 1.25M paths against the one-frame-at-a-time optimum of 4M; 3 in flight 1M)
        int tail = c->tail_paths ? c->tail_paths : (nfl > 1 ? kTailInFlight(nfl) : 0);
        // eight frames in flight and a frame of at most 2.5M base paths (a multi-GPU rank's share):
        // 768K (round 5, finish on 12 % of the grid: 8-way share 7.02 -> 7.20, 4-way 8.44 -> 8.54
        // Grays/s; 1M hands the 8-way share's whole frame to the finish: 6.08)
        if (!c->tail_paths && nfl >= 8 && (uint64_t)own * ts * ts * (uint64_t)spp <= kSmallShareBasePaths) tail = kTailShare;
        if (own > 0 && !run_wavefront(S, P, F.wf, c->tuning, own, c->counting, c->spans, tail, c->sort_bins, extra_pass,
                                      nfl, stream, cross ? prev.done : nullptr, &F.wft, &F.wfs, &err, c->graphs))
            FAIL(c, RT_ERR_HIP, std::string("wavefront: ") + (err ? err : "?"));
        if (own == 0 && cross) HIPC(c, hipStreamWaitEvent(stream, prev.done, 0));
    } else {
        if (cross) HIPC(c, hipStreamWaitEvent(stream, prev.done, 0));
        int nblocks = own * (ts / 16) * (ts / 16);
        if (nblocks > 0) launch_megakernel(S, P, nblocks, c->counting, stream);
    }
    HIPC(c, hipGetLastError());
    HIPC(c, hipEventRecord(F.ev1, stream));
    HIPC(c, hipMemcpyAsync(F.h_counters, F.counters.p, sizeof(unsigned long long) * kCounterWords,
                           hipMemcpyDeviceToHost, stream));
    HIPC(c, hipEventRecord(F.done, stream));
    F.wavefront = wavefront;
    F.pending = true;
    F.used = true;
    F.seq = c->frame_no;
    F.gen = c->gcur;
    c->last_slot = k;
    c->frame_no += 1;
    c->tiles_pending = false;
    c->last_tiles[0] = ts;
    c->last_tiles[1] = rank;
    c->last_tiles[2] = nranks;
    c->motion_cur = m_out;
    c->stats.frames_in_flight = nfl;
    c->last_frame_index = U->frameIndex;
    c->read_idx = 1 - c->read_idx;  // swap accumulationTargets (Renderer.swift:1492-1494)
    return RT_OK;
}

rt_status rt_wait(rt_ctx* c) {
    if (!c) FAIL(c, RT_ERR_INVALID_ARG, "null ctx");
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, hipStreamSynchronize(c->stream));
    // oldest frame first, so rt_stats ends on the newest one
    int order[kMaxSlots];
    for (int k = 0; k < kMaxSlots; ++k) order[k] = k;
    std::sort(order, order + kMaxSlots, [c](int a, int b) { return c->slot[a].seq < c->slot[b].seq; });
    for (int k : order)
        if (rt_status st = harvest(c, k)) return st;
    const FrameSlot& f = c->slot[c->last_slot];
    if (f.used) HIPC(c, hipEventSynchronize(f.done));   // and a pack / unpack after it
    return RT_OK;
}

rt_status rt_read_radiance(rt_ctx* c, float* rgba) {
    if (!c || !rgba) FAIL(c, RT_ERR_INVALID_ARG, "null argument");
    if (!c->width) FAIL(c, RT_ERR_STATE, "no targets");
    rt_status st = rt_wait(c);
    if (st) return st;
    HIPC(c, hipMemcpy(rgba, c->d_accum[c->read_idx].p, (size_t)c->width * c->height * 16, hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_read_radiance_half(rt_ctx* c, uint16_t* rgba) {
    if (!c || !rgba) FAIL(c, RT_ERR_INVALID_ARG, "null argument");
    if (!c->width) FAIL(c, RT_ERR_STATE, "no targets");
    rt_status st = rt_wait(c);
    if (st) return st;
    const size_t n = (size_t)c->width * c->height;
    if ((st = dev_alloc(c, c->d_half, n * 8))) return st;
    launch_to_half((const float4*)c->d_accum[c->read_idx].p, (ushort4*)c->d_half.p, n, c->stream);
    HIPC(c, hipGetLastError());
    HIPC(c, hipMemcpyAsync(rgba, c->d_half.p, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

rt_status rt_read_aux(rt_ctx* c, float* depth, float* motion, float* gbuffer) {
    if (!c) FAIL(c, RT_ERR_INVALID_ARG, "null ctx");
    if (!c->width) FAIL(c, RT_ERR_STATE, "no targets");
    rt_status st = rt_wait(c);
    if (st) return st;
    size_t n = (size_t)c->width * c->height;
    const FrameSlot& f = c->slot[c->last_slot];   // the newest frame's targets
    if (depth) HIPC(c, hipMemcpy(depth, f.depth.p, n * 4, hipMemcpyDeviceToHost));
    if (motion) HIPC(c, hipMemcpy(motion, c->d_motion[c->motion_cur].p, n * 8, hipMemcpyDeviceToHost));
    if (gbuffer) {
        if (!f.gbuffer.p || !f.gbuf_written) FAIL(c, RT_ERR_STATE, "the newest frame wrote no G-buffer (enableDenoiseGBuffer off)");
        HIPC(c, hipMemcpy(gbuffer, f.gbuffer.p, 4 * n * 16, hipMemcpyDeviceToHost));
    }
    return RT_OK;
}

// Pack / unpack run on `stream` after the newest frame, without a host wait, and extend that
// frame's `done` event over themselves: the frame that next writes the same accumulation target
// (two frames later) waits for it before its resolve, so the gather of frame f overlaps the
// rendering of frame f+1.
// own_stream: the ctx stream (rt_pack_tiles / rt_unpack_tiles); otherwise `stream` as the caller gave it,
// the null stream included (a collective ordered on PyTorch's default stream must see the pack)
static rt_status tiles_op(rt_ctx* c, const rt_tile_set* t, const void* src, void* dst, hipStream_t stream, bool pack,
                          bool own_stream) {
    if (!c || (pack ? !dst : !src)) FAIL(c, RT_ERR_INVALID_ARG, "null argument");
    if (!c->width) FAIL(c, RT_ERR_STATE, "no targets");
    int ts, rank, nranks, tiles_x, own;
    rt_status st = resolve_tiles(c, t, ts, rank, nranks, tiles_x, own);
    if (st) return st;
    HIPC(c, hipSetDevice(c->device));
    if (own_stream) {
        stream = c->stream;
        c->ctx_work++;
    }
    FrameSlot& f = c->slot[c->last_slot];
    if (f.used) HIPC(c, hipStreamWaitEvent(stream, f.done, 0));
    float4* accum = (float4*)c->d_accum[c->read_idx].p;
    if (pack)
        launch_pack_tiles(accum, (float4*)dst, c->width, c->height, ts, rank, nranks, tiles_x, own, stream);
    else
        launch_unpack_tiles((const float4*)src, accum, c->width, c->height, ts, rank, nranks, tiles_x, own, stream);
    HIPC(c, hipGetLastError());
    if (f.used) {
        HIPC(c, hipEventRecord(f.done, stream));
        c->tiles_pending = true;
    }
    return RT_OK;
}

rt_status rt_present(rt_ctx* c, const rt_present_opts* o, uint8_t* host_rgba8) {
    if (!c || !host_rgba8) FAIL(c, RT_ERR_INVALID_ARG, "null argument");
    if (!c->width) FAIL(c, RT_ERR_STATE, "no targets");
    const int ow = (o && o->out_width > 0) ? o->out_width : c->width;
    const int oh = (o && o->out_height > 0) ? o->out_height : c->height;
    const int scaler = o ? o->scaler : RT_SCALER_NONE;
    const int encode = o ? o->encode : RT_ENCODE_SRGB8;
    const int passes = (o && o->denoise_passes > 0) ? o->denoise_passes : 3;
    if (scaler < RT_SCALER_NONE || scaler > RT_SCALER_DENOISED || (encode != RT_ENCODE_SRGB8 && encode != RT_ENCODE_LINEAR8))
        FAIL(c, RT_ERR_INVALID_ARG, "bad scaler / encode");
    if (scaler == RT_SCALER_DENOISED && passes > 6) FAIL(c, RT_ERR_INVALID_ARG, "denoise_passes > 6");
    if ((int64_t)ow * oh > (1ll << 28)) FAIL(c, RT_ERR_INVALID_ARG, "output too large");
    HIPC(c, hipSetDevice(c->device));
    rt_status st;
    const size_t n = (size_t)ow * oh;
    if (!c->d_present_thr.p) {   // linear value at which the sRGB code reaches k + 1 (k + 0.5 of 255)
        float thr[256];
        for (int k = 0; k < 255; ++k) {
            const double s = (k + 0.5) / 255.0;
            thr[k] = (float)(s <= 0.04045 ? s / 12.92 : std::pow((s + 0.055) / 1.055, 2.4));
        }
        thr[255] = INFINITY;
        if ((st = dev_upload(c, c->d_present_thr, thr, sizeof thr))) return st;
    }
    if ((st = dev_alloc(c, c->d_present_out, n * 4))) return st;
    const bool temporal = scaler == RT_SCALER_TEMPORAL || scaler == RT_SCALER_DENOISED;
    if (temporal && (c->hist_w != ow || c->hist_h != oh || !c->d_hist[0].p)) {
        for (int i = 0; i < 2; ++i) {
            if ((st = dev_alloc(c, c->d_hist[i], n * 16))) return st;
            if ((st = dev_alloc(c, c->d_hdepth[i], n * 4))) return st;
        }
        c->hist_w = ow;
        c->hist_h = oh;
        c->hist_valid = false;
    }
    // after the newest frame (and any pack / unpack of it)
    FrameSlot& f = c->slot[c->last_slot];
    if (!f.used) FAIL(c, RT_ERR_STATE, "rt_present before the first frame");
    const float4* color = (const float4*)c->d_accum[c->read_idx].p;
    if (scaler == RT_SCALER_DENOISED) {   // render-size scratch: two ping-pong images, guide, albedo
        if (!f.gbuffer.p || !f.gbuf_written)
            FAIL(c, RT_ERR_STATE, "RT_SCALER_DENOISED needs the newest frame's G-buffer (enableDenoiseGBuffer)");
        const size_t rn = (size_t)c->width * c->height;
        if (c->den_n != rn || !c->d_den[0].p) {
            for (int i = 0; i < 4; ++i)
                if ((st = dev_alloc(c, c->d_den[i], rn * 16))) return st;
            c->den_n = rn;
        }
    }
    HIPC(c, hipStreamWaitEvent(c->stream, f.done, 0));
    if (scaler == RT_SCALER_DENOISED)
        color = launch_denoise(color, (const float*)f.depth.p, (const float4*)f.gbuffer.p, (float4*)c->d_den[0].p,
                               (float4*)c->d_den[1].p, (float4*)c->d_den[2].p, (float4*)c->d_den[3].p, c->width,
                               c->height, passes, c->stream);
    const int hi = c->hist_idx;
    launch_present(color, (const float*)f.depth.p,
                   (const float2*)c->d_motion[c->motion_cur].p, temporal ? (const float4*)c->d_hist[hi].p : nullptr,
                   temporal ? (const float*)c->d_hdepth[hi].p : nullptr,
                   temporal ? (float4*)c->d_hist[1 - hi].p : nullptr, temporal ? (float*)c->d_hdepth[1 - hi].p : nullptr,
                   (uchar4*)c->d_present_out.p, (const float*)c->d_present_thr.p, c->width, c->height, ow, oh,
                   temporal ? RT_SCALER_TEMPORAL : scaler,
                   encode == RT_ENCODE_SRGB8 ? 1 : 0, (temporal && c->hist_valid && c->last_frame_index > 0) ? 1 : 0,
                   c->stream);
    HIPC(c, hipGetLastError());
    if (temporal) {
        c->hist_idx = 1 - hi;
        c->hist_valid = true;
    }
    HIPC(c, hipMemcpyAsync(host_rgba8, c->d_present_out.p, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

rt_status rt_pack_tiles(rt_ctx* c, const rt_tile_set* t, void* dst) {
    return tiles_op(c, t, nullptr, dst, nullptr, true, true);
}

rt_status rt_unpack_tiles(rt_ctx* c, const rt_tile_set* t, const void* src) {
    return tiles_op(c, t, src, nullptr, nullptr, false, true);
}

rt_status rt_pack_tiles_on(rt_ctx* c, const rt_tile_set* t, void* dst, void* stream) {
    return tiles_op(c, t, nullptr, dst, (hipStream_t)stream, true, false);
}

rt_status rt_unpack_tiles_on(rt_ctx* c, const rt_tile_set* t, const void* src, void* stream) {
    return tiles_op(c, t, src, nullptr, (hipStream_t)stream, false, false);
}

static rt_status host_tiles(int32_t w, int32_t h, const rt_tile_set* t, int& ts, int& rank, int& nranks, int& tiles_x,
                            int& own) {
    ts = (t && t->tile_size > 0) ? t->tile_size : 64;
    nranks = (t && t->nranks > 0) ? t->nranks : 1;
    rank = (t && t->nranks > 0) ? t->rank : 0;
    if (w <= 0 || h <= 0 || rank < 0 || rank >= nranks) FAIL((rt_ctx*)nullptr, RT_ERR_INVALID_ARG, "bad tile set");
    tiles_x = (w + ts - 1) / ts;
    own = rt_tile_count(w, h, t);
    return RT_OK;
}

rt_status rt_pack_tiles_host(int32_t w, int32_t h, const rt_tile_set* t, const float* src, float* dst) {
    if (!src || !dst) FAIL((rt_ctx*)nullptr, RT_ERR_INVALID_ARG, "null argument");
    int ts, rank, nranks, tiles_x, own;
    rt_status st = host_tiles(w, h, t, ts, rank, nranks, tiles_x, own);
    if (st) return st;
    for (size_t i = 0; i < (size_t)ts * ts * own; ++i) {
        int x, y;
        tile_pixel(i, ts, rank, nranks, tiles_x, x, y);
        for (int q = 0; q < 4; ++q) dst[4 * i + q] = (x < w && y < h) ? src[4 * ((size_t)y * w + x) + q] : 0.0f;
    }
    return RT_OK;
}

rt_status rt_unpack_tiles_host(int32_t w, int32_t h, const rt_tile_set* t, const float* src, float* dst) {
    if (!src || !dst) FAIL((rt_ctx*)nullptr, RT_ERR_INVALID_ARG, "null argument");
    int ts, rank, nranks, tiles_x, own;
    rt_status st = host_tiles(w, h, t, ts, rank, nranks, tiles_x, own);
    if (st) return st;
    for (size_t i = 0; i < (size_t)ts * ts * own; ++i) {
        int x, y;
        tile_pixel(i, ts, rank, nranks, tiles_x, x, y);
        if (x < w && y < h)
            for (int q = 0; q < 4; ++q) dst[4 * ((size_t)y * w + x) + q] = src[4 * i + q];
    }
    return RT_OK;
}

rt_status rt_set_counting(rt_ctx* c, int32_t enabled) {
    if (!c) FAIL(c, RT_ERR_INVALID_ARG, "null ctx");
    c->counting = enabled != 0;
    return RT_OK;
}

rt_status rt_set_device_spans(rt_ctx* c, int32_t enabled) {
    if (!c) FAIL(c, RT_ERR_INVALID_ARG, "null ctx");
    c->spans = enabled != 0;
    return RT_OK;
}

// rt_tuning (0 = default) -> the kernels' resolved parameters
static WfTuning resolve_tuning(const rt_tuning& t) {
    WfTuning w;
    if (t.trace_chunk > 0) w.chunk = t.trace_chunk;
    if (t.finish_chunk > 0) w.fchunk = t.finish_chunk;
    if (t.refill_min > 0) w.refill_min = t.refill_min;
    if (t.shade_min > 0) w.shade_min = t.shade_min;
    if (t.shade_min_drained != 0) w.shade_min_x = t.shade_min_drained;
    w.team = t.team == 0 ? -1 : t.team == 1 ? 0 : t.team;
    if (t.finish_grid_pct > 0) w.finish_frac = std::min(t.finish_grid_pct, 100);
    if (t.trace_grid_pct > 0) w.trace_frac = std::min(t.trace_grid_pct, 100);
    if (t.shade_blocks > 0) w.shade_blocks = (unsigned)std::max(8, t.shade_blocks) / 8u * 8u;
    w.host_ctl = t.host_rounds != 0;
    w.log = std::max(0, t.log);
    return w;
}

rt_status rt_set_tuning(rt_ctx* c, const rt_tuning* t) {
    if (!c) FAIL(c, RT_ERR_INVALID_ARG, "null context");
    rt_tuning v{};
    if (t) v = *t;
    if (v.team != 0 && v.team != 1 && v.team != 2 && v.team != 4 && v.team != 8)
        FAIL(c, RT_ERR_INVALID_ARG, "rt_tuning.team must be 0 (default), 1 (off), 2, 4 or 8");
    // chunk grabs are 32-bit atomicAdds of the chunk size by every wave of the grid (and base + chunk
    // is formed in 32 bits): bounded so that neither can wrap for any queue the library allocates
    if (v.trace_chunk < 0 || v.trace_chunk > kMaxTuneChunk || v.finish_chunk < 0 || v.finish_chunk > kMaxTuneChunk ||
        v.refill_min < 0 || v.refill_min > 64 || v.shade_min < 0 || v.shade_min > 64 || v.shade_min_drained > 64 ||
        v.shade_min_drained < -100 || v.finish_grid_pct < 0 || v.finish_grid_pct > 100 || v.trace_grid_pct < 0 ||
        v.trace_grid_pct > 100 || v.shade_blocks < 0 || v.shade_blocks > kMaxTuneShadeBlocks || v.log < 0 || v.log > 2 ||
        v.device_bvh < 0 || v.device_bvh > 1 || (v.refit_rebuild_pct > 0 && v.refit_rebuild_pct < 100))
        FAIL(c, RT_ERR_INVALID_ARG, "rt_tuning field out of range");
    // frames already in flight keep the parameters they were enqueued with (their graphs' keys)
    c->tuning_req = v;
    c->tuning = resolve_tuning(v);
    return RT_OK;
}

rt_status rt_get_tuning(const rt_ctx* c, rt_tuning* out) {
    if (!c || !out) FAIL((rt_ctx*)nullptr, RT_ERR_INVALID_ARG, "null argument");
    const WfTuning& w = c->tuning;
    rt_tuning t{};
    t.trace_chunk = w.chunk;
    t.finish_chunk = w.fchunk;
    t.refill_min = w.refill_min;
    t.shade_min = w.shade_min;
    t.shade_min_drained = w.shade_min_x;
    t.team = c->tuning_req.team;
    t.finish_grid_pct = w.finish_frac;
    t.trace_grid_pct = w.trace_frac;
    t.shade_blocks = (int32_t)w.shade_blocks;
    t.host_rounds = w.host_ctl ? 1 : 0;
    t.log = w.log;
    t.device_bvh = c->tuning_req.device_bvh;
    t.refit_rebuild_pct = refit_rebuild_pct(c);
    *out = t;
    return RT_OK;
}

rt_status rt_set_graphs(rt_ctx* c, int32_t enabled) {
    if (!c) FAIL(c, RT_ERR_INVALID_ARG, "null ctx");
    c->graphs = enabled != 0;
    return RT_OK;
}

rt_status rt_get_stats(rt_ctx* c, rt_stats* out) {
    if (!c || !out) FAIL(c, RT_ERR_INVALID_ARG, "null argument");
    rt_status st = rt_wait(c);
    if (st) return st;
    c->stats.bvh_nodes = c->num_nodes8;
    c->stats.triangles = c->num_tris;
    c->stats.device_bytes = ctx_bytes(c);
    *out = c->stats;
    const rt_stats& T = c->totals;
    out->frames_total = T.frames_total;
    out->total_closest_rays = T.total_closest_rays;
    out->total_shadow_rays = T.total_shadow_rays;
    out->total_paths = T.total_paths;
    out->total_frame_ms = T.total_frame_ms;
    std::memcpy(out->total_kernel_ms, T.total_kernel_ms, sizeof T.total_kernel_ms);
    out->total_trace_rays = T.total_trace_rays;
    out->total_trace_closest_rays = T.total_trace_closest_rays;
    out->total_trace_ms = T.total_trace_ms;
    out->total_trace_launches = T.total_trace_launches;
    out->total_trace_dev_ms = T.total_trace_dev_ms;
    out->total_trace_dev_launches = T.total_trace_dev_launches;
    out->total_finish_dev_ms = T.total_finish_dev_ms;
    out->total_finish_dev_launches = T.total_finish_dev_launches;
    out->total_finish_launches = T.total_finish_launches;
    out->total_graph_replays = T.total_graph_replays;
    out->total_graph_captures = T.total_graph_captures;
    out->total_graph_fallbacks = T.total_graph_fallbacks;
    out->total_graph_eager = T.total_graph_eager;
    out->total_auto_rebuilds = c->auto_rebuilds;
    out->bvh_cost_built = c->cost_built;
    out->bvh_cost_refit = c->cost_refit;
    return RT_OK;
}

rt_status rt_debug_trace_host(const rt_scene_desc* sd, const float* rays, const float* tmax, uint32_t n, int32_t any,
                              float* t_out, uint32_t* id_out, float* u_out, float* v_out, uint32_t* nodes_out,
                              uint32_t* tris_out) {
    if (!sd || !rays || (n && (!t_out || !id_out))) FAIL((rt_ctx*)nullptr, RT_ERR_INVALID_ARG, "null argument");
    // world-space triangles in the original order (same arithmetic as rt_scene_upload)
    std::vector<float> world;
    for (uint32_t m = 0; m < sd->mesh_count; ++m) {
        const rt_mesh_desc& md = sd->meshes[m];
        float M[12];
        std::memcpy(M, &md.transform, 48);
        for (uint32_t s = 0; s < md.submesh_count; ++s) {
            const rt_submesh_desc& sm = md.submeshes[s];
            for (uint32_t i = 0; i < sm.index_count; ++i) {
                const rt_float3& p = md.positions[sm.indices[i]];
                float w[3];
                xform_host(M, make_float4(p.x, p.y, p.z, 0.0f), w);
                world.insert(world.end(), w, w + 3);
            }
        }
    }
    uint32_t nt = (uint32_t)(world.size() / 9);
    BvhResult bvh2;
    Bvh8Result bvh;
    if (!build_bvh8_fit(world.data(), nt, bvh2, bvh)) FAIL((rt_ctx*)nullptr, RT_ERR_UNSUPPORTED, "BVH too deep");
    std::vector<float> tris((size_t)kTriFloats * nt);
    for (uint32_t k = 0; k < nt; ++k) {
        const uint32_t id = bvh.tri_order[k];
        tri_store(&tris[(size_t)kTriFloats * k], &world[9 * (size_t)id], id);
    }
    DevScene S;
    std::memset(&S, 0, sizeof S);
    S.tris = tris.data();
    S.nodes8 = bvh.nodes.data();
    S.num_tris = (int)nt;
    S.num_nodes8 = (int)bvh.nodes.size();
    std::vector<int> stack((size_t)kStackSize * kBlock);
    for (uint32_t r = 0; r < n; ++r) {
        const float* q = rays + 6 * (size_t)r;
        f3 o = mk3(q[0], q[1], q[2]), d = mk3(q[3], q[4], q[5]);
        float tm = tmax ? tmax[r] : INFINITY;
        Hit h;
        TraceCounters tc{0, 0, 0};
        bool overflow = false;
        bool hit = any ? trace8<true, true>(S, o, d, 0.0f, tm, h, stack.data(), tc, overflow)
                       : trace8<false, true>(S, o, d, 0.0f, tm, h, stack.data(), tc, overflow);
        if (overflow) FAIL((rt_ctx*)nullptr, RT_ERR_STATE, "traversal stack overflow");
        t_out[r] = hit ? h.t : INFINITY;
        id_out[r] = hit ? h.id : 0xffffffffu;
        if (u_out) u_out[r] = hit ? h.u : 0.0f;
        if (v_out) v_out[r] = hit ? h.v : 0.0f;
        if (nodes_out) nodes_out[r] = tc.nodes;
        if (tris_out) tris_out[r] = tc.tris;
    }
    return RT_OK;
}

}  // extern "C"
