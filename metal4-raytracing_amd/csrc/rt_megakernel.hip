// rt_megakernel.hip — per-pixel path-tracing kernel for gfx950 (the reference's kernel shape).
//
// One thread per pixel runs the sample loop and the bounce loop of raytracingKernel
// (MetalRaytracing/Raytracing.metal:220-831); the Metal intersector is replaced by rt::trace
// (BVH2 + watertight triangle test, rt_device.h) and the per-hit work by rt::shade_step
// (rt_shade.h, shared with the wavefront pipeline).  Each block is a 16x16 pixel tile made of
// four 8x8 wave64 sub-tiles (square packets for coherent primary rays); blocks are remapped so
// every XCD renders a contiguous band of tiles (L2 locality of the BVH working set).
#include "rt_shade.h"

namespace rt {

template <bool COUNT, bool FULL>
__global__ void __launch_bounds__(kBlock)
megakernel(DevScene S, FrameParams P) {
    __shared__ int lds_stack[kStackSize * kBlock];
    __shared__ HaltonDim lds_halton[kHaltonLds];
    __shared__ MatRec lds_mat[kMatLds];
    const ShadeTabs halton = load_tabs(S, lds_halton, lds_mat);

    const Uniforms& U = P.U;
    // block -> tile mapping (XCD-contiguous), 16x16 pixels per block
    int nblk = gridDim.x;
    int b = blockIdx.x;
    int per = nblk / 8;
    if (b < per * 8) b = (b & 7) * per + (b >> 3);
    const int sub_w = P.tile_size / 16;
    const int sub_per_tile = sub_w * sub_w;
    int own_tile = b / sub_per_tile, sub = b % sub_per_tile;
    int tile_id = P.rank + own_tile * P.nranks;
    int tile_x = tile_id % P.tiles_x, tile_y = tile_id / P.tiles_x;
    int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int px = tile_x * P.tile_size + (sub % sub_w) * 16 + (wave & 1) * 8 + (lane & 7);
    int py = tile_y * P.tile_size + (sub / sub_w) * 16 + (wave >> 1) * 8 + (lane >> 3);

    int* stack = &lds_stack[threadIdx.x];
    TraceCounters tc{0, 0, 0};
    uint32_t n_closest = 0, n_shadow = 0, n_paths = 0;
    bool overflow = false;

    if (px < U.width && py < U.height) {                                          // :241
        const size_t pix = (size_t)py * U.width + px;
        unsigned int offset = P.random[pix];                                         // :245
        float2 pm2 = P.motion[pix];                                                  // :248
        f2 prevMotion;
        prevMotion.x = pm2.x;
        prevMotion.y = pm2.y;
        f3 totalColor = mk3(0.0f, 0.0f, 0.0f);
        float primaryDepth = 1.0e8f;
        f2 motionVector;
        motionVector.x = 0.0f;
        motionVector.y = 0.0f;
        bool hadPrimaryHit = false;
        float4 g0 = make_float4(0, 0, 0, 0), g1 = g0, g2 = g0, g3 = g0;
        bool wroteGBuffer = false;

        int baseSamples = max(U.samplesPerPixel, 1);                                  // :263-266
        int maxExtra = (U.enableMotionAdaptiveSampling != 0) ? max(U.motionSamplingMaxExtraSamples, 0) : 0;
        int sampleStride = baseSamples + maxExtra;
        int totalSamples = baseSamples;

        for (int sampleIndex = 0; sampleIndex < totalSamples; sampleIndex++) {     // :269
            n_paths++;
            int frameOffset = (int)U.frameIndex * sampleStride + sampleIndex;
            int hidx = (int)(offset + (unsigned)frameOffset);
            f3 rayO, rayD;
            primary_ray(U, halton, px, py, hidx, rayO, rayD);                        // :270-292
            PathRegs p;
            p.color = mk3(1.0f, 1.0f, 1.0f);
            p.accum = mk3(0.0f, 0.0f, 0.0f);
            p.bounce = 0;
            p.step = 0;
            p.tpass = 0;
            while (p.bounce < U.maxBounces) {                                        // :311
                Hit h;
                n_closest++;
                if (!trace8<false, COUNT>(S, rayO, rayD, 0.0f, INFINITY, h, stack, tc, overflow)) break;  // :318-322
                StepResult r;
                shade_step<FULL>(S, U, halton, hidx, sampleIndex, rayO, rayD, h, p, !wroteGBuffer, prevMotion,
                           hadPrimaryHit, motionVector, r);
                if (r.primary) {
                    primaryDepth = r.depth;
                    motionVector = r.motion;
                    hadPrimaryHit = true;
                }
                if (FULL && r.gbuf) {
                    g0 = r.g0; g1 = r.g1; g2 = r.g2; g3 = r.g3;
                    wroteGBuffer = true;
                }
                if (r.shadow) {                                                       // :716-743
                    Hit sh;
                    n_shadow++;
                    if (!trace8<true, COUNT>(S, r.so, r.sd, 0.0f, r.stmax, sh, stack, tc, overflow))
                        p.accum = p.accum + r.contrib;
                }
                if (!r.next) break;
            }
            totalColor = totalColor + p.accum;                                       // :777
            if (sampleIndex == 0 && maxExtra > 0)                                    // :779-789
                totalSamples = baseSamples + extra_samples(U, maxExtra, motionVector, prevMotion);
        }
        f3 c = resolve_pixel(U, totalColor, totalSamples, motionVector, prevMotion, P.accum_in, pix);  // :792-817
        P.accum_out[pix] = make_float4(c.x, c.y, c.z, 1.0f);                      // :819
        P.depth[pix] = primaryDepth;                                               // :822
        P.motion[pix] = make_float2(motionVector.x, motionVector.y);               // :823
        if (FULL && U.enableDenoiseGBuffer != 0 && P.gbuffer) {                    // :824-829
            size_t plane = (size_t)U.width * U.height;
            P.gbuffer[pix] = g0;
            P.gbuffer[plane + pix] = g1;
            P.gbuffer[2 * plane + pix] = g2;
            P.gbuffer[3 * plane + pix] = g3;
        }
    }
    block_flush_counters(P.counters, n_closest, n_shadow, COUNT ? tc.nodes : 0u, COUNT ? tc.tris : 0u, n_paths, overflow);
}

void launch_megakernel(const DevScene& S, const FrameParams& P, int nblocks, bool count, hipStream_t stream) {
    const bool full = needs_full(P.U, S);
    if (count) {
        if (full) hipLaunchKernelGGL((megakernel<true, true>), dim3(nblocks), dim3(kBlock), 0, stream, S, P);
        else hipLaunchKernelGGL((megakernel<true, false>), dim3(nblocks), dim3(kBlock), 0, stream, S, P);
    } else {
        if (full) hipLaunchKernelGGL((megakernel<false, true>), dim3(nblocks), dim3(kBlock), 0, stream, S, P);
        else hipLaunchKernelGGL((megakernel<false, false>), dim3(nblocks), dim3(kBlock), 0, stream, S, P);
    }
}

}  // namespace rt
