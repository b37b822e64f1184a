// rt_kernels.h — kernel parameter blocks and launch entry points (device code lives in *.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "rt_device.h"

namespace rt {

constexpr int kHaltonLds = 64;   // first Halton dimensions staged in LDS per block

enum CounterSlot { kCntClosest = 0, kCntShadow = 1, kCntNodes = 2, kCntTris = 3, kCntPaths = 4, kCntOverflow = 5, kCntSlots = 8 };

struct FrameParams {
    Uniforms U;
    const uint32_t* random;
    const float4* accum_in;    // history (TextureIndexAccumulation, read)
    float4* accum_out;         // new accumulation (TextureIndexPreviousAccumulation, write)
    float* depth;
    float2* motion;            // read (previous frame) + write, in place
    float4* gbuffer;           // 4 planes or null
    unsigned long long* counters;
    int tile_size, rank, nranks, tiles_x;
};

__device__ __forceinline__ unsigned long long wave_sum(uint32_t v) {
    unsigned long long s = v;
    #pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

void launch_megakernel(const DevScene& S, const FrameParams& P, int nblocks, bool count, hipStream_t stream);

// Wavefront pipeline (rt_wavefront.hip): path state SoA indexed by path id
// (own pixel index * spp + sample; extra samples after base_paths), ray queues of
// {float4 o (w = path id), float4 d}, hit records {t, tri id, u, v}, shadow queue of
// {float4 o (w = path id), float4 d (w = tmax), float4 contribution}.
constexpr int kShards = 8;        // queue segments (one allocation counter each)
constexpr int kWfCountWords = 32; // [0..7] queue 0, [8..15] queue 1, [16..23] shadow, [24] extra allocator
struct WavefrontBuffers {
    size_t queue_entries = 0;     // kShards segments of queue_entries / kShards
    float4* p_color = nullptr;
    float4* p_accum = nullptr;
    uint4* p_meta = nullptr;      // (pixel, sample, bounce | tpass << 8 | step << 16, halton index)
    float4* q[2] = {nullptr, nullptr};
    float4* hits = nullptr;
    float4* sq = nullptr;
    uint32_t* counts = nullptr;   // device: [0],[1] ray queues, [2] shadow queue, [3] extra-path allocator
    uint32_t* h_counts = nullptr; // pinned host mirror
    float2* motion_prev = nullptr;
    uint2* px_extra = nullptr;    // per own pixel: (first extra path - base_paths, count)
    size_t cap_paths = 0;         // base + extra paths
    size_t cap_pixels = 0;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
};
// Runs one frame; returns false on a HIP error (message in *err). stage_ms: [0] generate,
// [1] extend, [2] shade, [3] connect, [4] resolve (+extra-sample bookkeeping).
bool run_wavefront(const DevScene& S, const FrameParams& P, WavefrontBuffers& W, int own_tiles, bool count,
                   hipStream_t stream, float* stage_ms, int* iterations, const char** err);
size_t wavefront_queue_entries(size_t paths);

// Utility kernels (rt_util.hip)
void launch_pack_tiles(const float4* src, float4* dst, int width, int height, int tile, int rank, int nranks,
                       int tiles_x, int own, hipStream_t s);
void launch_unpack_tiles(const float4* src, float4* dst, int width, int height, int tile, int rank, int nranks,
                         int tiles_x, int own, hipStream_t s);
void launch_skin(const float4* rest_pos, const float4* rest_nrm, const ushort4* jidx, const float4* jw,
                 const float* joints, float4* out_pos, float4* out_nrm, uint32_t n, hipStream_t s);
void launch_flatten(const uint4* tri_info, const uint32_t* slot_to_tri, const float4* pos, const float* inst,
                    float4* tris, uint32_t n, hipStream_t s);
void launch_refit8_level(Bvh8Node* nodes, float* node_box, const float4* tris, const uint32_t* level_nodes,
                         uint32_t count, float pad, hipStream_t s);

}  // namespace rt
