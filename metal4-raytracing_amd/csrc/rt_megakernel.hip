// rt_megakernel.hip — per-pixel path-tracing kernel for gfx950.
//
// One thread per pixel runs the sample loop and the bounce loop of the reference's
// raytracingKernel (MetalRaytracing/Raytracing.metal:220-831) with the Metal intersector
// replaced by rt::trace (BVH2 + watertight triangle test, rt_device.h).  Each block is a 16x16
// pixel tile made of four 8x8 wave64 sub-tiles (square ray packets for coherent primary rays);
// blocks are remapped so that every XCD renders a contiguous band of tiles (L2 locality of the
// BVH working set).  Line references in comments are to Raytracing.metal.
#include "rt_kernels.h"

namespace rt {

struct PathOut {
    f3 total;
};

template <bool COUNT>
__global__ void __launch_bounds__(kBlock)
megakernel(DevScene S, FrameParams P) {
    __shared__ int lds_stack[kStackSize * kBlock];
    __shared__ HaltonDim lds_halton[kHaltonLds];
    for (int i = threadIdx.x; i < kHaltonLds; i += kBlock) lds_halton[i] = S.halton[i];
    __syncthreads();

    const Uniforms& U = P.U;
    // ---- block -> tile mapping (XCD-contiguous), 16x16 pixels per block ----
    int nblk = gridDim.x;
    int b = blockIdx.x;
    int per = nblk / 8;
    if (b < per * 8) b = (b & 7) * per + (b >> 3);
    const int sub_per_tile = (P.tile_size / 16) * (P.tile_size / 16);
    int own_tile = b / sub_per_tile, sub = b % sub_per_tile;
    int tile_id = P.rank + own_tile * P.nranks;
    int tile_x = tile_id % P.tiles_x, tile_y = tile_id / P.tiles_x;
    int sub_w = P.tile_size / 16;
    int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int px = tile_x * P.tile_size + (sub % sub_w) * 16 + (wave & 1) * 8 + (lane & 7);
    int py = tile_y * P.tile_size + (sub / sub_w) * 16 + (wave >> 1) * 8 + (lane >> 3);

    int* stack = &lds_stack[threadIdx.x];
    TraceCounters tc{0, 0};
    uint32_t n_closest = 0, n_shadow = 0, n_paths = 0;
    bool overflow = false;

    auto halton = [&](int i, int d) -> float {
        return d < kHaltonLds ? halton_fast(i, lds_halton[d]) : halton_fast(i, S.halton[d]);
    };

    if (px < U.width && py < U.height) {                                           // :241
        const size_t pix = (size_t)py * U.width + px;
        unsigned int offset = P.random[pix];                                          // :245
        f3 totalColor = mk3(0.0f, 0.0f, 0.0f);
        float2 pm = P.motion[pix];                                                    // :248
        f2 prevMotion; prevMotion.x = pm.x; prevMotion.y = pm.y;
        float primaryDepth = 1.0e8f;
        f2 motionVector; motionVector.x = 0.0f; motionVector.y = 0.0f;
        bool hadPrimaryHit = false;
        float4 outDiffuseAlbedo = make_float4(0, 0, 0, 0), outSpecularAlbedo = make_float4(0, 0, 0, 0);
        float4 outNormal = make_float4(0, 0, 0, 0), outRoughness = make_float4(0, 0, 0, 0);
        bool wroteGBuffer = false;

        int baseSamples = max(U.samplesPerPixel, 1);                                   // :263
        int maxExtraSamples = (U.enableMotionAdaptiveSampling != 0) ? max(U.motionSamplingMaxExtraSamples, 0) : 0;
        int sampleStride = baseSamples + maxExtraSamples;
        int totalSamples = baseSamples;

        for (int sampleIndex = 0; sampleIndex < totalSamples; sampleIndex++) {      // :269
            n_paths++;
            int frameOffset = (int)U.frameIndex * sampleStride + sampleIndex;
            int hidx = (int)(offset + (unsigned)frameOffset);
            float rx = halton(hidx, 0), ry = halton(hidx, 1);                         // :273-274
            float spx = (float)px + rx, spy = (float)py + ry;
            float uvx = spx / (float)U.width, uvy = spy / (float)U.height;            // :278
            uvx = uvx * 2.0f - 1.0f; uvy = uvy * 2.0f - 1.0f;
            const Camera& cam = U.camera;
            f3 cright = mk3(cam.right.x, cam.right.y, cam.right.z);
            f3 cup = mk3(cam.up.x, cam.up.y, cam.up.z);
            f3 cfwd = mk3(cam.forward.x, cam.forward.y, cam.forward.z);
            f3 rayO = mk3(cam.position.x, cam.position.y, cam.position.z);        // :285
            f3 rayD = normalize((uvx * cright + uvy * cup) + cfwd);                   // :287-289

            f3 color = mk3(1.0f, 1.0f, 1.0f);
            f3 accumulatedColor = mk3(0.0f, 0.0f, 0.0f);
            int bounce = 0, step = 0, transparencyPasses = 0;
            while (bounce < U.maxBounces) {                                           // :311
                Hit h;
                n_closest++;
                if (!trace<false, COUNT>(S, rayO, rayD, 0.0f, INFINITY, h, stack, tc, overflow)) break;  // :318-322
                uint4 ti = S.tri_info[h.id];
                int instanceIndex = (int)(ti.w >> 8);
                int geometryIndex = (int)(ti.w & 0xffu);
                const float* M = S.inst + 12 * instanceIndex;                        // :329-333
                f3 P_ = rayO + rayD * h.t;                                            // :336
                int resourceIndex = instanceIndex * S.max_submeshes + geometryIndex;  // :338
                const Material& mat = S.materials[resourceIndex];
                float bu = h.u, bv = h.v, bw = (1.0f - bu) - bv;                      // :63-65

                if (bounce == 0 && sampleIndex == 0) {                                // :342-389
                    f3 op = (bu * ld3(S.pos[ti.y]) + bv * ld3(S.pos[ti.z])) + bw * ld3(S.pos[ti.x]);
                    f3 pp = (bu * ld3(S.prev_pos[ti.y]) + bv * ld3(S.prev_pos[ti.z])) + bw * ld3(S.prev_pos[ti.x]);
                    f3 worldPos = xform(M, op, 1.0f);
                    f3 prevWorldPos = xform(S.prev_inst + 12 * instanceIndex, pp, 1.0f);
                    f3 cpos = rayO;
                    f3 viewPos = worldPos - mk3(cam.position.x, cam.position.y, cam.position.z);
                    (void)cpos;
                    float sx = dot(viewPos, cright), sy = dot(viewPos, cup);
                    float depth = dot(viewPos, cfwd);
                    primaryDepth = fmaxf(depth, 1.0e-3f);
                    float dd = fmaxf(depth, 0.001f);
                    sx = sx / dd; sy = sy / dd;
                    const Camera& pc = U.previousCamera;
                    f3 prevViewPos = prevWorldPos - mk3(pc.position.x, pc.position.y, pc.position.z);
                    float psx = dot(prevViewPos, mk3(pc.right.x, pc.right.y, pc.right.z));
                    float psy = dot(prevViewPos, mk3(pc.up.x, pc.up.y, pc.up.z));
                    float prevDepth = dot(prevViewPos, mk3(pc.forward.x, pc.forward.y, pc.forward.z));
                    float pd = fmaxf(prevDepth, 0.001f);
                    psx = psx / pd; psy = psy / pd;
                    float mnx = sx - psx, mny = sy - psy;
                    float rightScale = fmaxf(length(cright), 1e-5f);
                    float upScale = fmaxf(length(cup), 1e-5f);
                    float mpx = mnx * ((float)U.width / (2.0f * rightScale));
                    float mpy = mny * ((float)U.height / (2.0f * upScale));
                    motionVector.x = mpx; motionVector.y = -mpy;
                    hadPrimaryHit = true;
                }

                f3 objN = (bu * ld3(S.nrm[ti.y]) + bv * ld3(S.nrm[ti.z])) + bw * ld3(S.nrm[ti.x]);  // :391
                f3 Ng = normalize(xform(M, objN, 0.0f));                              // :392-393
                if (length(objN) < 1e-10f) Ng = -rayD;                                // :395-397

                f3 albedo = mk3(mat.baseColor.x, mat.baseColor.y, mat.baseColor.z);  // :399
                // textureFlags are always 0 for uploaded scenes (texture path: SURVEY §8f)
                float roughness = 1.0f, metallic = 0.0f, ao = 1.0f;                   // :431-441
                float opacity = clampf(mat.opacity, 0.0f, 1.0f);                      // :448
                f3 emission = mk3(mat.emission.x, mat.emission.y, mat.emission.z);   // :453

                if (U.debugTextureMode != DebugTextureModeNone) {                     // :459-490
                    f3 dc = mk3(0.0f, 0.0f, 0.0f);
                    int m = U.debugTextureMode;
                    if (m == DebugTextureModeBaseColor) dc = mk3(1.0f, 0.0f, 1.0f);
                    else if (m == DebugTextureModeNormal) dc = Ng * 0.5f + mk3(0.5f, 0.5f, 0.5f);
                    else if (m == DebugTextureModeRoughness) dc = mk3(roughness, roughness, roughness);
                    else if (m == DebugTextureModeMetallic) dc = mk3(metallic, metallic, metallic);
                    else if (m == DebugTextureModeAO) dc = mk3(1.0f, 0.0f, 1.0f);
                    else if (m == DebugTextureModeEmission) dc = emission;
                    else if (m == DebugTextureModeMotion) {
                        f2 mp = hadPrimaryHit ? motionVector : prevMotion;
                        float scx = clampf(mp.x * 0.05f, -1.0f, 1.0f), scy = clampf(mp.y * 0.05f, -1.0f, 1.0f);
                        float mag = clampf(sqrtf(mp.x * mp.x + mp.y * mp.y) * 0.1f, 0.0f, 1.0f);
                        dc = mk3(scx * 0.5f + 0.5f, scy * 0.5f + 0.5f, mag);
                    }
                    accumulatedColor = dc;
                    break;
                }

                f3 shadingNormal = Ng;                                                // :492

                if (U.enableDenoiseGBuffer != 0 && !wroteGBuffer && sampleIndex == 0) {  // :506-515
                    float rr = clampf(roughness, 0.0f, 1.0f);
                    f3 da = albedo * (1.0f - metallic);
                    f3 sa = mix3(mk3(0.04f, 0.04f, 0.04f), albedo, metallic);
                    f3 on = shadingNormal * 0.5f + mk3(0.5f, 0.5f, 0.5f);
                    outDiffuseAlbedo = make_float4(da.x, da.y, da.z, 1.0f);
                    outSpecularAlbedo = make_float4(sa.x, sa.y, sa.z, 1.0f);
                    outNormal = make_float4(on.x, on.y, on.z, 1.0f);
                    outRoughness = make_float4(rr, 0.0f, 0.0f, 1.0f);
                    wroteGBuffer = true;
                }

                float clampedOpacity = clampf(opacity, 0.0f, 1.0f);                  // :517
                float ior = fmaxf(mat.refractionIndex, 1.0f);
                if (clampedOpacity < 0.999f || ior > 1.01f) {                          // :521-576
                    f3 N = shadingNormal, I = rayD;
                    float cosi = clampf(dot(-I, N), -1.0f, 1.0f);
                    float etaI = 1.0f, etaT = ior;
                    if (cosi < 0.0f) { cosi = -cosi; N = -N; float tmp = etaI; etaI = etaT; etaT = tmp; }
                    float eta = etaI / etaT;
                    float k = 1.0f - (eta * eta) * (1.0f - cosi * cosi);
                    float f0 = (etaT - etaI) / (etaT + etaI);
                    f0 = f0 * f0;
                    float F = f0 + (1.0f - f0) * pow5(clampf(1.0f - cosi, 0.0f, 1.0f));
                    float transmission = 1.0f - clampedOpacity;
                    float reflectWeight = F;
                    float refractWeight = (1.0f - F) * transmission;
                    float totalWeight = fmaxf(reflectWeight + refractWeight, 1e-4f);
                    float reflectProb = reflectWeight / totalWeight;
                    float choice = halton(hidx, 2 + step * 6 + 5);
                    bool consumeBounce = true;
                    if (k < 0.0f || choice < reflectProb) {
                        f3 reflectDir = normalize(I - (2.0f * dot(I, N)) * N);
                        rayO = P_ + reflectDir * 1e-3f;
                        rayD = reflectDir;
                        color = color * totalWeight;
                    } else {
                        float cosT = sqrtf(fmaxf(k, 0.0f));
                        f3 refractDir = normalize(eta * I + (eta * cosi - cosT) * N);
                        rayO = P_ + refractDir * 1e-3f;
                        rayD = refractDir;
                        color = color * (totalWeight * albedo);
                        consumeBounce = false;
                    }
                    step++;
                    if (consumeBounce) { bounce++; transparencyPasses = 0; }
                    else {
                        transparencyPasses++;
                        if (transparencyPasses > U.maxBounces) { bounce++; transparencyPasses = 0; }
                    }
                    continue;
                }

                float perceptualRoughness = clampf(roughness, 0.04f, 1.0f);           // :578
                float alpha = perceptualRoughness * perceptualRoughness;
                f3 diffuseColor = albedo;
                f3 F0 = mix3(mk3(0.04f, 0.04f, 0.04f), albedo, metallic);
                f3 V = normalize(-rayD);

                accumulatedColor = accumulatedColor + color * emission;               // :585

                float lightSample = halton(hidx, 2 + step * 6 + 0);                   // :588
                int lightIndex = min((int)(lightSample * (float)U.lightCount), U.lightCount - 1);
                const Light& light = S.lights[lightIndex];
                f3 Ldir, lightColor;
                float lightDistance;
                f3 lpos = mk3(light.position.x, light.position.y, light.position.z);
                f3 lcol = mk3(light.color.x, light.color.y, light.color.z);
                if (light.type == LightTypeAreaLight) {                               // :597-606, :95-129
                    float ux = halton(hidx, 2 + step * 6 + 1), uy = halton(hidx, 2 + step * 6 + 2);
                    ux = ux * 2.0f - 1.0f; uy = uy * 2.0f - 1.0f;
                    f3 sp = (lpos + mk3(light.right.x, light.right.y, light.right.z) * ux) + mk3(light.up.x, light.up.y, light.up.z) * uy;
                    Ldir = sp - P_;
                    lightDistance = length(Ldir);
                    float inv = 1.0f / fmaxf(lightDistance, 1e-3f);
                    Ldir = Ldir * inv;
                    lightColor = lcol * (inv * inv);
                    lightColor = lightColor * saturate(dot(-Ldir, mk3(light.forward.x, light.forward.y, light.forward.z)));
                } else if (light.type == LightTypeSpotlight) {                        // :608-632
                    Ldir = lpos - P_;
                    lightDistance = length(Ldir);
                    float inv = 1.0f / fmaxf(lightDistance, 1e-3f);
                    Ldir = Ldir * inv;
                    lightColor = mk3(0.0f, 0.0f, 0.0f);
                    f3 coneDirection = normalize(mk3(light.direction.x, light.direction.y, light.direction.z));
                    float spotResult = dot(-Ldir, coneDirection);
                    if (spotResult > cos_pinned(light.coneAngle)) lightColor = (lcol * inv) * inv;
                } else if (light.type == LightTypePointlight) {                       // :633-638
                    Ldir = lpos - P_;
                    lightDistance = length(Ldir);
                    float inv = 1.0f / fmaxf(lightDistance, 1e-3f);
                    Ldir = Ldir * inv;
                    lightColor = (lcol * inv) * inv;
                } else {                                                              // :639-643
                    Ldir = -normalize(mk3(light.direction.x, light.direction.y, light.direction.z));
                    lightDistance = INFINITY;
                    lightColor = lcol;
                }
                lightColor = lightColor * (float)U.lightCount;                        // :647

                if (U.shadingMode == ShadingModeLegacy) {                             // :649-690
                    f3 L = normalize(Ldir);
                    float NdotL = saturate(dot(shadingNormal, L));
                    f3 legacyColor = color * albedo;
                    if (length(legacyColor) < 0.001f) break;
                    if (length(lightColor) > 0.0001f && NdotL > 0.0f) {
                        Hit sh;
                        n_shadow++;
                        if (!trace<true, COUNT>(S, P_ + Ng * 1e-3f, Ldir, 0.0f, lightDistance - 1e-3f, sh, stack, tc, overflow))
                            accumulatedColor = accumulatedColor + (legacyColor * lightColor) * NdotL;
                    }
                    color = legacyColor * ao;
                    if (length(color) < 0.001f) break;
                    float r0 = halton(hidx, 2 + step * 5 + 3), r1 = halton(hidx, 2 + step * 5 + 4);
                    f3 dir = alignHemisphereWithNormal(sampleCosineWeightedHemisphere(r0, r1), shadingNormal);
                    rayO = P_ + Ng * 1e-3f;
                    rayD = dir;
                    step++; bounce++; transparencyPasses = 0;
                    continue;
                }

                if (length(lightColor) > 0.0001f) {                                   // :692-744
                    f3 L = normalize(Ldir);
                    f3 H = normalize(V + L);
                    float NdotL = saturate(dot(shadingNormal, L));
                    float NdotV = saturate(dot(shadingNormal, V));
                    float NdotH = saturate(dot(shadingNormal, H));
                    float VdotH = saturate(dot(V, H));
                    f3 F = fresnelSchlick(VdotH, F0);
                    float D = distributionGGX(NdotH, alpha);
                    float kk = perceptualRoughness + 1.0f;
                    kk = (kk * kk) / 8.0f;
                    float G = geometrySmith(NdotV, NdotL, kk);
                    f3 specular = ((D * G) * F) / fmaxf((4.0f * NdotV) * NdotL, 1e-4f);
                    f3 kD = (mk3(1.0f, 1.0f, 1.0f) - F) * (1.0f - metallic);
                    f3 diffuse = (kD * diffuseColor) / RT_PI;
                    f3 direct = ((diffuse + specular) * lightColor) * NdotL;
                    Hit sh;
                    n_shadow++;
                    if (!trace<true, COUNT>(S, P_ + Ng * 1e-3f, Ldir, 0.0f, lightDistance - 1e-3f, sh, stack, tc, overflow))
                        accumulatedColor = accumulatedColor + color * direct;
                }

                color = color * ((diffuseColor * (1.0f - metallic)) * ao);            // :748
                if (length(color) < 0.001f) break;                                    // :751-753
                float r0 = halton(hidx, 2 + step * 5 + 3), r1 = halton(hidx, 2 + step * 5 + 4);  // :763-764
                f3 dir = alignHemisphereWithNormal(sampleCosineWeightedHemisphere(r0, r1), shadingNormal);
                rayO = P_ + Ng * 1e-3f;                                               // :769
                rayD = dir;
                step++; bounce++; transparencyPasses = 0;
            }
            totalColor = totalColor + accumulatedColor;                               // :777

            if (sampleIndex == 0 && maxExtraSamples > 0) {                            // :779-789
                float motionMag = fmaxf(sqrtf(motionVector.x * motionVector.x + motionVector.y * motionVector.y),
                                        sqrtf(prevMotion.x * prevMotion.x + prevMotion.y * prevMotion.y));
                float low = fmaxf(U.motionSamplingLowThresholdPixels, 0.0f);
                float high = fmaxf(U.motionSamplingHighThresholdPixels, low + 1e-3f);
                float t = clampf((motionMag - low) / (high - low), 0.0f, 1.0f);
                int extraSamples = (int)roundf(t * (float)maxExtraSamples);
                extraSamples = min(max(extraSamples, 0), maxExtraSamples);
                totalSamples = baseSamples + extraSamples;
            }
        }

        totalColor = totalColor / (float)max(totalSamples, 1);                       // :793
        if (U.frameIndex > 0) {                                                       // :796-817
            float4 pc = P.accum_in[pix];
            f3 prevColor = mk3(pc.x, pc.y, pc.z);
            float historyWeight = clampf(U.accumulationWeight, 0.0f, 0.95f);
            if (U.enableMotionAdaptiveAccumulation != 0) {
                float motionMag = fmaxf(sqrtf(motionVector.x * motionVector.x + motionVector.y * motionVector.y),
                                        sqrtf(prevMotion.x * prevMotion.x + prevMotion.y * prevMotion.y));
                float low = fmaxf(U.motionAccumulationLowThresholdPixels, 0.0f);
                float high = fmaxf(U.motionAccumulationHighThresholdPixels, low + 1e-3f);
                float t = clampf((motionMag - low) / (high - low), 0.0f, 1.0f);
                float minWeight = clampf(U.motionAccumulationMinWeight, 0.0f, 0.95f);
                minWeight = fminf(minWeight, historyWeight);
                historyWeight = mixf(historyWeight, minWeight, t);
            }
            totalColor = mix3(totalColor, prevColor, historyWeight);
        }
        P.accum_out[pix] = make_float4(totalColor.x, totalColor.y, totalColor.z, 1.0f);  // :819
        P.depth[pix] = primaryDepth;                                                  // :822
        P.motion[pix] = make_float2(motionVector.x, motionVector.y);                  // :823
        if (U.enableDenoiseGBuffer != 0 && P.gbuffer) {                               // :824-829
            size_t plane = (size_t)U.width * U.height;
            P.gbuffer[pix] = outDiffuseAlbedo;
            P.gbuffer[plane + pix] = outSpecularAlbedo;
            P.gbuffer[2 * plane + pix] = outNormal;
            P.gbuffer[3 * plane + pix] = outRoughness;
        }
    }
    // ---- counters: one atomic per wave ----
    unsigned long long c0 = wave_sum(n_closest), c1 = wave_sum(n_shadow), c4 = wave_sum(n_paths);
    unsigned long long c2 = COUNT ? wave_sum(tc.nodes) : 0ull, c3 = COUNT ? wave_sum(tc.tris) : 0ull;
    unsigned long long c5 = __ballot(overflow) != 0ull ? 1ull : 0ull;
    if (lane == 0) {
        atomicAdd(&P.counters[0], c0);
        atomicAdd(&P.counters[1], c1);
        if (COUNT) { atomicAdd(&P.counters[2], c2); atomicAdd(&P.counters[3], c3); }
        atomicAdd(&P.counters[4], c4);
        if (c5) atomicAdd(&P.counters[5], c5);
    }
}

void launch_megakernel(const DevScene& S, const FrameParams& P, int nblocks, bool count, hipStream_t stream) {
    if (count) hipLaunchKernelGGL(megakernel<true>, dim3(nblocks), dim3(kBlock), 0, stream, S, P);
    else hipLaunchKernelGGL(megakernel<false>, dim3(nblocks), dim3(kBlock), 0, stream, S, P);
}

}  // namespace rt
