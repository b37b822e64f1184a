/*
 * rt_oracle.h — CPU oracle for the path-tracer hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference kernel raytracingKernel
 * (tatsuya-ogawa/metal4-raytracing, MetalRaytracing/Raytracing.metal:220-831) and the skinning
 * kernel (Skinning.metal:7-49).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it — as the checker / CPU baseline, never as the product path.
 *
 * Independence from the product (metal4-raytracing_amd/): this file shares no code with it.
 * It builds its own BVH (object-median split), its own world-space triangle flattening, and
 * states every arithmetic expression itself.  What both sides share is the *specification*
 * written in DESIGN.md §4: evaluation order without FMA contraction, the watertight
 * ray/triangle test (Woop et al. 2013) with closest-hit ties broken by the smaller original
 * triangle id, pinned sin/cos/pow5 formulas, and the 1024-entry Halton prime table.
 *
 * Parity status: the reference itself cannot run here (Swift/Metal absent), so
 * this oracle is pinned by known-answer tests (tests/test_oracle_kat.py) and by the committed
 * fixtures in tests/golden/ which it generated; ray-triangle/BVH semantics of Apple's
 * intersector are "parity unpinned".
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>
#include "../include/rt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_oracle_scene rt_oracle_scene;

typedef struct rt_oracle_frame {
    const Uniforms* uniforms;
    const uint32_t* random;      /* W*H per-pixel offsets */
    const float* accum_in;       /* W*H*4 history, NULL = zeros */
    float* accum_out;            /* W*H*4 */
    float* depth;                /* W*H */
    float* motion;               /* W*H*2, in: previous frame's motion, out: this frame's */
    float* gbuffer;              /* 4 planes of W*H*4, or NULL */
    int32_t row_start;           /* render rows row_start, row_start+row_step, ... */
    int32_t row_step;            /* <= 0 means 1 */
    int32_t threads;             /* worker threads (<= 0: 1) */
    int32_t tile_size;           /* with nranks > 1: render only the pixels of the tiles with */
    int32_t rank;                /* tile_id % nranks == rank (tile_size x tile_size tiles,     */
    int32_t nranks;              /* numbered row-major), as a rank of the multi-GPU split does */
    uint64_t closest_rays;       /* out */
    uint64_t shadow_rays;        /* out */
    uint64_t paths;              /* out */
} rt_oracle_frame;

int rt_oracle_scene_create(const rt_scene_desc* desc, rt_oracle_scene** out);
void rt_oracle_scene_destroy(rt_oracle_scene* s);
/* previous-frame positions / instance transform of mesh m for motion vectors; NULL keeps */
int rt_oracle_scene_set_previous(rt_oracle_scene* s, uint32_t mesh, const rt_float3* prev_positions,
                                 const float* prev_transform);
uint32_t rt_oracle_scene_triangles(const rt_oracle_scene* s);

int rt_oracle_render(const rt_oracle_scene* s, rt_oracle_frame* f);

/* Known-answer hooks */
float rt_oracle_halton(int32_t i, int32_t d);
void rt_oracle_sincos(float x, float* s, float* c);
float rt_oracle_pow5(float x);
/* bilinear LOD-0 repeat sample of scene texture t at (u, v) (v already flipped); srgb: decode
 * RGB through the sRGB table (base color / emission slots).  0 on success. */
int rt_oracle_tex_sample(const rt_oracle_scene* s, int32_t t, float u, float v, int32_t srgb, float out[4]);
/* world-space closest (any=0) / any (any=1) hit; returns 1 on hit */
int rt_oracle_intersect(const rt_oracle_scene* s, const float o[3], const float d[3], float tmin, float tmax, int any,
                        float* t, uint32_t* id, float* u, float* v);
int rt_oracle_intersect_bruteforce(const rt_oracle_scene* s, const float o[3], const float d[3], float tmin,
                                   float tmax, int any, float* t, uint32_t* id, float* u, float* v);
/* Skinning.metal:7-49 on host arrays (positions/normals float4 stride-16 as rt_float3). */
void rt_oracle_skin(const rt_float3* rest_pos, const rt_float3* rest_nrm, const uint16_t* jidx, const float* jw,
                    const float* joints, rt_float3* out_pos, rt_float3* out_nrm, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
