/*
 * rt_api.h — C-ABI of the MI355X path-tracer hot path (librt_hip.so).
 *
 * This is the drop-in boundary for the reference's one GPU hot path, the Metal compute kernel
 * `raytracingKernel` (MetalRaytracing/Raytracing.metal:220-831) and the host code that binds and
 * dispatches it.  Each entry point names the reference interface it replaces:
 *
 *   rt_create / rt_destroy     Renderer.init?(metalView:) device+queue+pipeline setup
 *                              (Renderer.swift:228-341), deinit
 *   rt_scene_upload            createBuffers: Resource argument buffer, material buffers,
 *                              vertex/index buffers, light buffer (Renderer.swift:342-420,
 *                              SubMesh.swift:38-54, Scene.swift:93)
 *   rt_bvh_build               createMTL4AccelerationStructures BLAS+TLAS build
 *                              (Renderer.swift:464-606, Utilities.swift:101-290)
 *   rt_bvh_build_device        the same build on the GPU (LBVH + 8-wide collapse); also the
 *                              legacy full rebuild of a deformed scene (Renderer.swift:1252-1277)
 *   rt_set_instance_transforms updateInstanceDescriptors (Renderer.swift:937-973): current ->
 *                              previous copy, then new transforms
 *   rt_skin                    SkinningPass.dispatchSkinning + prev-position copy
 *                              (SkinningPass.swift:160-211, Renderer.swift:1290-1310)
 *   rt_bvh_refit               refitMTL4AccelerationStructures (Renderer.swift:1084-1202)
 *   rt_resize                  createTextures: accumulation ping-pong, random-offset texture,
 *                              depth/motion/G-buffer targets (Renderer.swift:676-804)
 *   rt_render_frame            Renderer.draw: argument-table binding + 16x16 dispatch of
 *                              raytracingKernel + ping-pong swap (Renderer.swift:1405-1503)
 *   rt_read_radiance/rt_read_aux  (no reference equivalent: the reference never reads back;
 *                              replaces presenting dstTex/depthTex/motionTex to MetalFX)
 *
 * Conventions: every function returns rt_status (0 = OK); rt_last_error(ctx) describes the last
 * failure.  No exceptions or aborts cross this boundary.  The caller owns every host array and
 * may free it once the call returns.  One context per GPU, used from one host thread.  All
 * work is issued on one HIP stream per context (rt_set_stream may substitute the caller's).
 */
#ifndef RT_API_H
#define RT_API_H

#include "rt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t rt_status;
#define RT_OK 0
#define RT_ERR_INVALID_ARG 1
#define RT_ERR_HIP 2
#define RT_ERR_IO 3
#define RT_ERR_OUT_OF_MEMORY 4
#define RT_ERR_STATE 5
#define RT_ERR_UNSUPPORTED 6
#define RT_ERR_NO_DEVICE 7

typedef struct rt_ctx rt_ctx;

/* ---- scene description (caller-owned, copied by rt_scene_upload) ------------------------- */

/* A decoded texture (the MTLTexture of SubMesh.swift:69-241): width x height RGBA8 texels,
 * row-major, row 0 = the image's top row (texcoord v = 0 after the shader's flip,
 * Raytracing.metal:416).  Base color and emission slots decode sRGB, the others are linear
 * (the loader options of SubMesh.swift:80-97). */
typedef struct rt_texture_desc {
    const uint8_t* rgba8;
    uint32_t width;
    uint32_t height;
} rt_texture_desc;

/* Texture slot k of a submesh <-> MATERIAL_TEXTURE_* bit k of its material's textureFlags:
 * 0 base color, 1 tangent-space normal, 2 roughness, 3 metallic, 4 AO, 5 emission, 6 opacity. */
#define RT_TEXTURE_SLOTS 7

/* One Submesh: a material group of one mesh (SubMesh.swift:18-54). Indices are u32
 * (u16 assets are widened, SubMesh.swift:243-265), three per triangle.  textures[k]: index into
 * rt_scene_desc.textures for every slot whose bit is set in material.textureFlags (other
 * entries are ignored); the AO slot is not sampled (ENABLE_AO = 0, ShaderTypes.h:155-156). */
typedef struct rt_submesh_desc {
    const uint32_t* indices;
    uint32_t index_count;
    uint32_t _pad;
    Material material;
    int32_t textures[8];
} rt_submesh_desc;

/* One Mesh = one instance of the two-level acceleration structure (Mesh.swift:17-68). Vertex
 * streams follow Model.vertexDescriptor (Model.swift:304-341): positions and normals float3 at
 * a 16-byte stride, uvs float2 (may be NULL), joint indices ushort4 and weights float4 (NULL
 * unless skinned).  `transform` is the object->world MTLPackedFloat4x3 of the instance
 * descriptor (Renderer.swift:547-556). */
typedef struct rt_mesh_desc {
    const rt_float3* positions;
    const rt_float3* normals;
    const rt_float2* uvs;
    const uint16_t* joint_indices;
    const float* joint_weights;
    uint32_t vertex_count;
    uint32_t submesh_count;
    const rt_submesh_desc* submeshes;
    rt_packed_float4x3 transform;
    uint32_t joint_count;   /* > 0: skinned mesh (rt_skin rewrites its positions/normals) */
    uint32_t _pad;
} rt_mesh_desc;

typedef struct rt_scene_desc {
    uint32_t mesh_count;
    uint32_t light_count;
    const rt_mesh_desc* meshes;
    const Light* lights;
    uint32_t texture_count;
    uint32_t _pad;
    const rt_texture_desc* textures;
} rt_scene_desc;

/* ---- context ------------------------------------------------------------------------------- */

#define RT_PIPELINE_MEGAKERNEL 0  /* one thread per pixel, the reference's kernel shape */
#define RT_PIPELINE_WAVEFRONT 1   /* generate / extend / shade / connect / resolve queues */

typedef struct rt_opts {
    int32_t device;     /* HIP device ordinal */
    int32_t pipeline;   /* RT_PIPELINE_* */
    int32_t tail_paths; /* wavefront: below this many live paths the rest of the frame runs in the
                           persistent finish kernel; 0 = default (4194304 one frame at a time,
                           1310720 / 1048576 / 786432 / 524288 with 2 / 3 / 4 / 5+ frames in flight), 1 = never */
    int32_t sort_bins;  /* wavefront: hits are sorted into this many bins of BVH leaf order between
                           extend and shade (a power of two in [1024, 4096]); 0 = default (no
                           sort), < 0 = no sort.  Never changes the image, only memory locality. */
    int32_t frames_in_flight; /* wavefront on the context's own stream: frames rendered concurrently,
                                 each overlapping the previous one until it needs that frame's
                                 accumulation / motion output; 0 = default (one per hardware
                                 queue: 8 when the process has GPU_MAX_HW_QUEUES >= 8, 4
                                 otherwise, as many as fit in 96 GB, at least 2), 1 = one at a
                                 time, at most 8.  Each slot holds ~300 B per allocated path,
                                 pixels x (spp + extra samples).  With four or
                                 more slots the finish tail takes 20 % of the resident grid,
                                 with two 40 %.
                                 Geometry updates (skinning, transforms, refit, builds) rotate
                                 over max(2, frames in flight) generations, so per-frame updates
                                 keep every slot's overlap.  Images are identical either way. */
    int32_t reserved[3];
} rt_opts;

/* Image-space tile partition for multi-GPU rendering: the image is cut into
 * tile_size x tile_size tiles numbered row-major; this rank renders tiles with
 * tile_id % nranks == rank.  A NULL tile set (or nranks <= 1) renders the whole image. */
typedef struct rt_tile_set {
    int32_t tile_size;
    int32_t rank;
    int32_t nranks;
    int32_t _pad;
} rt_tile_set;

typedef struct rt_stats {
    uint64_t closest_rays;  /* closest-hit queries traced in the last frame (incl. primary) */
    uint64_t shadow_rays;   /* any-hit shadow queries traced in the last frame */
    uint64_t node_visits;   /* BVH node tests (counting frames only, see rt_set_counting) */
    uint64_t tri_tests;     /* triangles tested (counting frames only) */
    uint64_t paths;         /* pixel samples started */
    uint64_t bvh_nodes;     /* nodes in the current BVH */
    uint64_t triangles;     /* triangles in the current scene */
    uint64_t device_bytes;  /* device memory held by the context */
    float last_frame_ms;    /* device time of the last rt_render_frame (HIP events) */
    float kernel_ms[7];     /* per-stage device time of the last frame: megakernel [0];
                               wavefront [0] generate [1] extend [2] shade [3] connect [4] resolve
                               [5] finish (tail) [6] hit sort */
    int32_t pipeline;       /* RT_PIPELINE_* that rendered the last frame */
    int32_t iterations;     /* wavefront: extend/shade/connect rounds of the last frame */
    /* wavefront: the queue traversal kernel (extend + connect launches; the finish tail excluded) */
    uint64_t trace_rays;    /* rays it traced */
    uint64_t trace_nodes;   /* nodes it fetched (counting frames only) */
    uint64_t trace_tris;    /* triangles it tested (counting frames only) */
    int32_t trace_launches; /* its launches */
    float trace_ms;         /* its summed device time (HIP events on the render stream) */
    uint64_t trace_closest_rays; /* the closest-hit (extend) share of trace_rays */
    int32_t finish_launches;     /* wavefront: persistent finish launches (their time: kernel_ms[5]) */
    int32_t frames_in_flight;    /* frames the last rt_render_frame could overlap (1..8) */
    /* running totals over every finished frame since rt_create (frames submitted back to back
       without rt_wait are each counted) */
    uint64_t frames_total;
    uint64_t total_closest_rays;
    uint64_t total_shadow_rays;
    uint64_t total_paths;
    double total_frame_ms;         /* sum of last_frame_ms */
    double total_kernel_ms[7];     /* sums of kernel_ms */
    uint64_t total_trace_rays;     /* sums of trace_rays, trace_closest_rays, trace_ms, trace_launches, */
    uint64_t total_trace_closest_rays;   /* finish_launches */
    double total_trace_ms;
    uint64_t total_trace_launches;
    uint64_t total_finish_launches;
    /* reserved, always 0 (node visits served from an LDS copy of the BVH's top levels: that
       staging was measured and removed) */
    uint64_t node_visits_lds;
    uint64_t trace_nodes_lds;
    /* wavefront, device clock: each launch from its first workgroup's start to its last wave's end
       (s_memrealtime, 100 MHz), what a kernel trace records for a dispatch.  With frames in flight
       the HIP events of trace_ms / kernel_ms also count the time a launch waits for CUs that other
       frames' kernels hold. */
    float trace_dev_ms;            /* extend + connect launches of the last frame */
    int32_t trace_dev_launches;
    float finish_dev_ms;           /* finish launches of the last frame */
    int32_t finish_dev_launches;
    double total_trace_dev_ms;     /* running sums of the four above */
    uint64_t total_trace_dev_launches;
    double total_finish_dev_ms;
    uint64_t total_finish_dev_launches;
    /* wavefront frames (device-driven, the default) by how they were submitted (running totals):
       replayed from the slot's two captured HIP graphs, captured anew and launched (first frame of
       a slot, or a launch argument changed), enqueued eagerly because the runtime refused a
       capture (the slot then stays eager), enqueued eagerly by choice (RT_GRAPH=0, host-driven
       rounds).  The replacement of the reference's per-frame command buffers
       (Renderer.swift:1405-1490). */
    uint64_t total_graph_replays;
    uint64_t total_graph_captures;
    uint64_t total_graph_fallbacks;
    uint64_t total_graph_eager;
    /* tree quality (rt_tuning.refit_rebuild_pct): device rebuilds a degraded refit triggered, and the
       node-area sum (the sum of the 8-wide node boxes' areas: the SAH node term, proportional to the
       node visits of the scene's rays) of the last build and of the last refit read back (0 before
       the first refit; a rebuild leaves the refit figure that triggered it) */
    uint64_t total_auto_rebuilds;
    float bvh_cost_built;
    float bvh_cost_refit;
} rt_stats;

rt_status rt_create(const rt_opts* opts, rt_ctx** out);
rt_status rt_destroy(rt_ctx* ctx);
const char* rt_last_error(const rt_ctx* ctx);   /* ctx may be NULL: last global error */
rt_status rt_set_stream(rt_ctx* ctx, void* hip_stream);  /* NULL restores the own stream */

rt_status rt_scene_upload(rt_ctx* ctx, const rt_scene_desc* scene);
rt_status rt_bvh_build(rt_ctx* ctx);
/* On-device build from the uploaded (and possibly skinned / re-transformed) geometry: Morton
 * sort + radix tree + top-down collapse into the same 8-wide layout.  Milliseconds instead of the
 * host SAH build's seconds; traversal visits more nodes per ray (LBVH quality).  Images are
 * identical to those of a host-built tree (conservative boxes).  Fails with
 * RT_ERR_UNSUPPORTED when the tree is deeper than the traversal stack. */
rt_status rt_bvh_build_device(rt_ctx* ctx);
rt_status rt_bvh_refit(rt_ctx* ctx);
rt_status rt_set_instance_transforms(rt_ctx* ctx, const rt_packed_float4x3* transforms, uint32_t count);
/* Linear-blend skinning of one skinned mesh (Skinning.metal:7-49). `joint_matrices` are
 * column-major float4x4 (host memory). Copies current positions to previous first. */
rt_status rt_skin(rt_ctx* ctx, uint32_t mesh_index, const float* joint_matrices, uint32_t joint_count);

/* (Re)create the per-pixel targets; `random_offsets` is W*H uint32 (row-major). Resets history. */
rt_status rt_resize(rt_ctx* ctx, int32_t width, int32_t height, const uint32_t* random_offsets);

/* Render one frame (asynchronous; rt_wait to block). Reads the history written by the previous
 * call, writes the new accumulation and swaps (Renderer.swift:1492-1494). */
rt_status rt_render_frame(rt_ctx* ctx, const Uniforms* uniforms, const rt_tile_set* tiles);
rt_status rt_wait(rt_ctx* ctx);

/* Copies of the latest outputs into caller host memory: radiance RGBA float32 W*H*4 (the
 * accumulation target just written; the reference stores it as RGBA16F), depth W*H,
 * motion W*H*2 (pixels, +Y down), G-buffer 4 planes of W*H*4 (diffuse, specular, normal,
 * roughness) or NULL. Rows are in the kernel's tid.y order (row 0 = bottom of the view). */
rt_status rt_read_radiance(rt_ctx* ctx, float* rgba);
/* The same radiance as RGBA16F (uint16_t bit patterns, W*H*4), the format the reference's
 * accumulation texture holds (Renderer.swift:685, Raytracing.metal:819): the fp32 target rounded
 * to nearest even on the device (overflow to infinity, fp16 denormals kept); 8 B per pixel read
 * back instead of 16. */
rt_status rt_read_radiance_half(rt_ctx* ctx, uint16_t* rgba);
rt_status rt_read_aux(rt_ctx* ctx, float* depth, float* motion, float* gbuffer);

/* Display output (FramePresenter.swift:103-238, Shaders.metal:39-52): the newest radiance,
 * resampled to out_width x out_height by `scaler`, tone-mapped color / (1 + color) and encoded
 * to 8-bit RGBA rows top-down (alpha 255), written to host memory.  RT_SCALER_NONE samples the
 * nearest render pixel (the presenter's own path); SPATIAL resamples bilinearly; TEMPORAL blends
 * with the previous output reprojected through the motion vectors, clamped to the current
 * neighbourhood, rejected on depth jumps (MetalFX's scalers are unpublished: these are stand-ins
 * consuming the same inputs).  DENOISED (MTLFXTemporalDenoisedScaler's place when
 * useTemporalDenoiser is set, FramePresenter.swift:77-98,179-198) first filters the radiance at
 * render size, guided by the G-buffer (enableDenoiseGBuffer must be on: RT_ERR_STATE otherwise):
 * demodulation by diffuse + specular albedo, `denoise_passes` edge-avoiding a-trous passes over
 * normals and depth, remodulation; then the TEMPORAL path.  DENOISED and TEMPORAL share one
 * history.  encode: RT_ENCODE_SRGB8 (default) or RT_ENCODE_LINEAR8. */
#define RT_SCALER_NONE 0
#define RT_SCALER_SPATIAL 1
#define RT_SCALER_TEMPORAL 2
#define RT_SCALER_DENOISED 3
#define RT_ENCODE_SRGB8 0
#define RT_ENCODE_LINEAR8 1
typedef struct rt_present_opts {
    int32_t out_width;   /* 0 = render width */
    int32_t out_height;  /* 0 = render height */
    int32_t scaler;
    int32_t encode;
    int32_t denoise_passes;   /* RT_SCALER_DENOISED: 0 = 3; at most 6 */
    int32_t reserved[3];
} rt_present_opts;
rt_status rt_present(rt_ctx* ctx, const rt_present_opts* opts, uint8_t* host_rgba8);

/* Multi-GPU: pack this rank's tiles of the latest radiance into a device buffer of
 * rt_tile_count(...) * tile_size^2 * 4 floats, and the inverse on the gathering rank
 * (writing into the latest radiance target). Device pointers; enqueued after the newest frame
 * on the ctx stream (the _on forms: on `hip_stream` exactly as given, e.g. the stream the
 * collective runs on; NULL is HIP's null stream, PyTorch's default stream), without a host wait.  The next frames overlap them (see frames_in_flight); rt_wait waits for
 * them too. */
int32_t rt_tile_count(int32_t width, int32_t height, const rt_tile_set* tiles);
rt_status rt_pack_tiles(rt_ctx* ctx, const rt_tile_set* tiles, void* device_dst);
rt_status rt_unpack_tiles(rt_ctx* ctx, const rt_tile_set* tiles, const void* device_src);
rt_status rt_pack_tiles_on(rt_ctx* ctx, const rt_tile_set* tiles, void* device_dst, void* hip_stream);
rt_status rt_unpack_tiles_on(rt_ctx* ctx, const rt_tile_set* tiles, const void* device_src, void* hip_stream);
/* Host-memory forms of the same layout (RGBA fp32 images of width x height), for gathers that
 * land in host memory and for tests of the tile protocol without a device. */
rt_status rt_pack_tiles_host(int32_t width, int32_t height, const rt_tile_set* tiles, const float* src_rgba,
                             float* dst_packed);
rt_status rt_unpack_tiles_host(int32_t width, int32_t height, const rt_tile_set* tiles, const float* src_packed,
                               float* dst_rgba);

/* Device ray/node counters: when enabled, frames also count BVH node visits / triangle tests
 * (a few percent slower). Ray counts are always collected. */
rt_status rt_set_counting(rt_ctx* ctx, int32_t enabled);
/* Device-clock launch spans of the wavefront traversal and finish launches (rt_stats
 * total_*_dev_ms; block 0's start to the last wave's end, s_memrealtime), for frames submitted
 * while enabled.  Off by default: the stamps cost ~1 % of a C3g frame.  Measurement only (no
 * reference counterpart). */
rt_status rt_set_device_spans(rt_ctx* ctx, int32_t enabled);
/* Wavefront frames captured once per frame slot as HIP graphs and replayed (default: on), or
 * enqueued launch by launch (off) — the
 * replacement of the reference's per-frame command buffers (Renderer.swift:1405-1490).  Under a
 * HIP runtime that takes no timing events inside a graph, replayed frames record no per-stage
 * times (rt_stats kernel_ms); frames submitted with graphs off always do. */
rt_status rt_set_graphs(rt_ctx* ctx, int32_t enabled);
rt_status rt_get_stats(rt_ctx* ctx, rt_stats* out);

/* Scheduling parameters of the wavefront kernels (no reference counterpart: the
 * Metal driver schedules the reference's one kernel).  0 in any field selects the measured default;
 * images are identical for every value.  The library reads no environment variable
 * for these: only this call changes them, per context.  rt_set_tuning(ctx, NULL) restores the
 * defaults; a field outside its stated range is RT_ERR_INVALID_ARG.  rt_get_tuning returns the
 * values in effect for the fields with a fixed default; team, finish_grid_pct and trace_grid_pct
 * read back 0 when left at their default, which is chosen per frame from the frame size and the
 * frames in flight (rt_stats reports the frame's rounds and launches, not these choices). */
typedef struct rt_tuning {
    int32_t trace_chunk;        /* rays per chunk grab of the bulk traversal launches (default 64; <= 4096) */
    int32_t finish_chunk;       /* paths per chunk grab of the finish launch (default 64; <= 4096) */
    int32_t refill_min;         /* traversal / finish waves refill once this many lanes are idle (default 8) */
    int32_t shade_min;          /* the finish kernel shades once this many lanes wait for it (default 24) */
    int32_t shade_min_drained;  /* the same once its queue has run out: > 0 lanes, < 0 that percentage of
                                   the wave's busy lanes (default -50) */
    int32_t team;               /* finish drain, lanes per query once a wave holds <= 64 / team paths:
                                   0 = default (4 for frames of 256K .. 2.5M base paths, else off),
                                   1 = off, 2 / 4 / 8 */
    int32_t finish_grid_pct;    /* percent of the resident grid the finish launch takes (default by
                                   frames in flight: 100 / 40 / 33 / 20 for 1 / 2 / 3 / 4+) */
    int32_t trace_grid_pct;     /* percent of the resident grid the bulk traversal launches take
                                   (default 100; 60 with four to seven frames in flight; with eight,
                                   20 / 30 / 40 for frames of up to 2.5M / 6M / more base paths) */
    int32_t shade_blocks;       /* wf_shade grid, a multiple of 8 (default 2048; <= 65536) */
    int32_t host_rounds;        /* 1: host-driven rounds (each round's queue size read back); default 0:
                                   device-side round control, whole frames as HIP graphs */
    int32_t log;                /* 1: per-round queue sizes, stage times and finish diagnostics on stderr
                                   (host-driven rounds); 2: + per-path segment counts (slower) */
    int32_t device_bvh;         /* rt_bvh_build_device topology: 0 = PLOC clustering (default),
                                   1 = LBVH radix tree */
    int32_t refit_rebuild_pct;  /* rt_bvh_refit keeps the topology and grows the boxes of moved
                                   geometry; once a refit's node-area sum (rt_stats.bvh_cost_refit)
                                   exceeds this percentage of the last build's, the next
                                   rt_bvh_refit or rt_render_frame rebuilds the tree on the device
                                   (rt_bvh_build_device) instead.  0 = default (150), < 0 = never.
                                   Images are the same either way. */
    int32_t reserved[3];
} rt_tuning;
rt_status rt_set_tuning(rt_ctx* ctx, const rt_tuning* tuning);
rt_status rt_get_tuning(const rt_ctx* ctx, rt_tuning* out);

/* Library build identification (kernel code object arch etc). */
const char* rt_version(void);

/* Test hook (host only, no device): build the library's BVH for `scene` and trace `n` rays
 * (6 floats each: origin, direction) with the traversal code the kernels use, compiled for the
 * host.  any = 0: closest hit, 1: any hit; tmax per ray or NULL (= infinity).  Outputs per ray:
 * t (inf on miss), original triangle id (0xffffffff on miss), barycentrics u/v, BVH nodes
 * fetched and triangles tested (u, v, nodes, tris may be NULL). */
rt_status rt_debug_trace_host(const rt_scene_desc* scene, const float* rays, const float* tmax, uint32_t n,
                              int32_t any, float* t, uint32_t* id, float* u, float* v, uint32_t* nodes,
                              uint32_t* tris);

#ifdef __cplusplus
}
#endif
#endif /* RT_API_H */
