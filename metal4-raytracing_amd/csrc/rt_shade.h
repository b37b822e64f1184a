// rt_shade.h — one hit-processing step of a path: everything raytracingKernel does between two
// intersector calls (Raytracing.metal:324-774).  Shared by the per-pixel megakernel and the
// wavefront `shade` stage so both pipelines evaluate exactly the same operation sequence.
//
// Given the current ray and its closest hit, shade_step updates the path registers (throughput
// `color`, `accum`, bounce / step / transparencyPasses), optionally emits a shadow ray whose
// contribution the caller adds to `accum` when it is unoccluded (Raytracing.metal:741-743 /
// :667-669), and either rewrites the ray for the next iteration (next = true) or ends the path.
#pragma once
#include "rt_kernels.h"

namespace rt {

// The fields of a Material the kernel reads (Raytracing.metal:399-453), packed for LDS:
// base = (baseColor, opacity), emis = (emission, refractionIndex).
struct MatRec {
    float4 base;
    float4 emis;
};
constexpr int kMatLds = 128;   // material records staged in LDS per block (4 KB)

constexpr int kInstLds = 32;   // instance matrices staged in LDS per block (48 B each, 1.5 KB)
constexpr int kLightLds = 8;   // lights staged in LDS per block (128 B each, 1 KB)

// Per-block lookup tables of the shading code: the first Halton dimensions, the scene's
// material records, instance matrices and lights in LDS (global memory beyond what was staged).
// A hit's instance matrix is the third load of a dependent chain (queue entry -> tri_nrm ->
// matrix) and its light record waits on the Halton light choice; from LDS each costs an LDS round
// trip instead of an L2 one (wf_shade 0.336 -> 0.310 ms per launch).
struct ShadeTabs {
    const HaltonDim* lds;
    const HaltonDim* glob;
    const MatRec* mat_lds;
    const Material* mat_glob;
    int n_mat_lds;             // = number of materials when they fit in LDS, else 0
    const float4* inst_lds;    // 3 float4 per instance: the 12 floats of its packed 4x3
    const float* inst_glob;
    int n_inst_lds;            // = number of instances when they fit in LDS, else 0
    const Light* light_lds;
    const Light* light_glob;
    int n_light_lds;           // = lightCount when the lights fit in LDS, else 0
    __device__ __forceinline__ float operator()(int i, int d) const {
        if (d == 0) return halton_base2(i);   // base 2: closed form (bit-identical, rt_math.h)
        return halton_fast(i, d < kHaltonLds ? lds[d] : glob[d]);
    }
    __device__ __forceinline__ MatRec material(int slot) const {
        if (slot < n_mat_lds) return mat_lds[slot];
        const Material& m = mat_glob[slot];
        MatRec r;
        r.base = make_float4(m.baseColor.x, m.baseColor.y, m.baseColor.z, m.opacity);
        r.emis = make_float4(m.emission.x, m.emission.y, m.emission.z, m.refractionIndex);
        return r;
    }
    // The instance's 12 floats and the light record, from LDS when staged: one pointer that may
    // point to either (flat loads), which measured faster than a branch between an LDS and a
    // global load of the same record (wf_shade 0.310 vs 0.313 ms; both branches' registers)
    __device__ __forceinline__ const float* instance(int k) const {
        return k < n_inst_lds ? reinterpret_cast<const float*>(inst_lds + 3 * k) : inst_glob + 12 * (size_t)k;
    }
    __device__ __forceinline__ const Light& light(int k) const { return k < n_light_lds ? light_lds[k] : light_glob[k]; }
};

// Stages the Halton dimensions and the material records, instance matrices and lights of the
// scene in LDS (each table only when its LDS array is given and the scene's table fits); every
// thread of the block calls it (ends with a barrier).
__device__ __forceinline__ ShadeTabs load_tabs(const DevScene& S, HaltonDim* lds_halton, MatRec* lds_mat,
                                               float4* lds_inst = nullptr, Light* lds_light = nullptr,
                                               int light_count = 0) {
    for (int i = threadIdx.x; i < kHaltonLds; i += blockDim.x) lds_halton[i] = S.halton[i];
    const int n_mat = (lds_mat && S.num_materials <= kMatLds) ? S.num_materials : 0;
    for (int i = threadIdx.x; i < n_mat; i += blockDim.x) {
        const Material& m = S.materials[i];
        lds_mat[i].base = make_float4(m.baseColor.x, m.baseColor.y, m.baseColor.z, m.opacity);
        lds_mat[i].emis = make_float4(m.emission.x, m.emission.y, m.emission.z, m.refractionIndex);
    }
    const int n_inst_all = S.max_submeshes > 0 ? S.num_materials / S.max_submeshes : 0;
    const int n_inst = (lds_inst && n_inst_all <= kInstLds) ? n_inst_all : 0;
    const float4* ig = reinterpret_cast<const float4*>(S.inst);
    for (int i = threadIdx.x; i < 3 * n_inst; i += blockDim.x) lds_inst[i] = ig[i];
    const int n_light = (lds_light && light_count <= kLightLds) ? light_count : 0;
    for (int i = threadIdx.x; i < n_light; i += blockDim.x) lds_light[i] = S.lights[i];
    __syncthreads();
    return ShadeTabs{lds_halton, S.halton, lds_mat, S.materials, n_mat, lds_inst, S.inst, n_inst,
                     lds_light, S.lights, n_light};
}

struct PathRegs {
    f3 color;
    f3 accum;
    int bounce, step, tpass;
};

struct StepResult {
    bool next;             // trace rayO/rayD again
    bool shadow;           // trace shadow ray; add contrib to accum when unoccluded
    f3 so, sd, contrib;
    float stmax;
    bool primary;          // bounce 0 / sample 0 hit: depth + motion (:342-389)
    float depth;
    f2 motion;
    bool gbuf;             // first hit of sample 0 with the G-buffer enabled (:506-515)
    float4 g0, g1, g2, g3;
};

__device__ __forceinline__ f3 ldf3(const rt_float3& v) { return mk3(v.x, v.y, v.z); }

// ---- texture path --------------------------------------------------------
// The reference samples with sampler(linear, linear, mip linear, address::repeat) in a compute
// kernel, i.e. bilinear from LOD 0 (Raytracing.metal:420).  Here: texel centres at integer + 0.5,
// wrap-around neighbours, each corner decoded through the byte table (sRGB for base color and
// emission maps, linear otherwise; alpha always linear), weights applied in a fixed order.
__device__ __forceinline__ float4 tex_sample(const DevScene& S, int t, f2 uv, bool srgb) {
    const uint4 ti = S.tex_info[t];
    const int w = (int)ti.y, h = (int)ti.z;
    float x = uv.x * (float)w - 0.5f, y = uv.y * (float)h - 0.5f;
    if (!(fabsf(x) < 1.0e9f)) x = 0.0f;   // NaN / huge coordinates
    if (!(fabsf(y) < 1.0e9f)) y = 0.0f;
    const float fx = floorf(x), fy = floorf(y);
    const float ax = x - fx, ay = y - fy, bx = 1.0f - ax, by = 1.0f - ay;
    int x0 = (int)((long long)fx % w), y0 = (int)((long long)fy % h);
    if (x0 < 0) x0 += w;
    if (y0 < 0) y0 += h;
    const int x1 = x0 + 1 == w ? 0 : x0 + 1, y1 = y0 + 1 == h ? 0 : y0 + 1;
    const uchar4* T = S.tex_texels + ti.x;
    const uchar4 c00 = T[(size_t)y0 * w + x0], c10 = T[(size_t)y0 * w + x1];
    const uchar4 c01 = T[(size_t)y1 * w + x0], c11 = T[(size_t)y1 * w + x1];
    const float* L = S.tex_lut;
    const float* Lc = L + (srgb ? 256 : 0);
    auto bil = [&](const float* lut, unsigned a, unsigned b, unsigned c, unsigned d) {
        return (lut[a] * bx + lut[b] * ax) * by + (lut[c] * bx + lut[d] * ax) * ay;
    };
    return make_float4(bil(Lc, c00.x, c10.x, c01.x, c11.x), bil(Lc, c00.y, c10.y, c01.y, c11.y),
                       bil(Lc, c00.z, c10.z, c01.z, c11.z), bil(L, c00.w, c10.w, c01.w, c11.w));
}

__device__ __forceinline__ f2 ld2(const float2& v) { return f2{v.x, v.y}; }

// computeTangentBasis (Raytracing.metal:185-218): object-space dP/du, dP/dv of the hit triangle
// from its vertices in the order (indices[3t+1], indices[3t+2], indices[3t]).
__device__ __forceinline__ bool tangent_basis(const DevScene& S, const uint4& ti, f3& tangent, f3& bitangent) {
    const f3 p0 = ld3(S.pos[ti.y]), p1 = ld3(S.pos[ti.z]), p2 = ld3(S.pos[ti.x]);
    const f2 uv0 = ld2(S.uv[ti.y]), uv1 = ld2(S.uv[ti.z]), uv2 = ld2(S.uv[ti.x]);
    const f3 e1 = p1 - p0, e2 = p2 - p0;
    const float d1x = uv1.x - uv0.x, d1y = uv1.y - uv0.y, d2x = uv2.x - uv0.x, d2y = uv2.y - uv0.y;
    const float denom = d1x * d2y - d1y * d2x;
    if (fabsf(denom) < 1e-8f) return false;
    const float r = 1.0f / denom;
    tangent = (e1 * d2y - e2 * d1y) * r;
    bitangent = (e2 * d1x - e1 * d2x) * r;
    return length(tangent) > 1e-8f && length(bitangent) > 1e-8f;
}

__host__ __device__ __forceinline__ bool needs_full(const Uniforms& U, const DevScene& S) {
    return U.debugTextureMode != DebugTextureModeNone || U.enableDenoiseGBuffer != 0 || S.textured != 0;
}

// Depth and motion vector of a bounce-0 hit of sample 0 (Raytracing.metal:342-389): the hit
// point through this frame's and the previous frame's instance transforms and cameras.  Inline in
// the per-pixel kernel; the wavefront kernels record the hit and wf_motion evaluates this once
// per pixel after the pass (the last bounce-0 hit of sample 0 wins either way).
__device__ __forceinline__ void primary_outputs(const DevScene& S, const Uniforms& U, uint32_t id, float bu, float bv,
                                                float& depth_out, f2& motion_out) {
    const uint4 ti = S.tri_info[id];
    const int instanceIndex = (int)(ti.w >> 8);
    const float* M = S.inst + 12 * instanceIndex;
    const float bw = (1.0f - bu) - bv;
    const Camera& cam = U.camera;
    const f3 cright = ldf3(cam.right), cup = ldf3(cam.up), cfwd = ldf3(cam.forward);
    f3 op = (bu * ld3(S.pos[ti.y]) + bv * ld3(S.pos[ti.z])) + bw * ld3(S.pos[ti.x]);
    f3 pp = (bu * ld3(S.prev_pos[ti.y]) + bv * ld3(S.prev_pos[ti.z])) + bw * ld3(S.prev_pos[ti.x]);
    f3 worldPos = xform(M, op, 1.0f);
    f3 prevWorldPos = xform(S.prev_inst + 12 * instanceIndex, pp, 1.0f);
    f3 viewPos = worldPos - ldf3(cam.position);
    float sx = dot(viewPos, cright), sy = dot(viewPos, cup);
    float depth = dot(viewPos, cfwd);
    depth_out = fmaxf(depth, 1.0e-3f);
    float dd = fmaxf(depth, 0.001f);
    sx = sx / dd;
    sy = sy / dd;
    const Camera& pc = U.previousCamera;
    f3 pv = prevWorldPos - ldf3(pc.position);
    float psx = dot(pv, ldf3(pc.right)), psy = dot(pv, ldf3(pc.up));
    float pd = fmaxf(dot(pv, ldf3(pc.forward)), 0.001f);
    psx = psx / pd;
    psy = psy / pd;
    float mnx = sx - psx, mny = sy - psy;
    float rightScale = fmaxf(length(cright), 1e-5f);
    float upScale = fmaxf(length(cup), 1e-5f);
    float mpx = mnx * ((float)U.width / (2.0f * rightScale));
    float mpy = mny * ((float)U.height / (2.0f * upScale));
    motion_out.x = mpx;
    motion_out.y = -mpy;
}

// prevMotion / hadPrimaryHit / motionVector: only read by DebugTextureModeMotion.
// FULL = false compiles out the texture maps, the debug-visualisation and the G-buffer branches
// (the caller selects FULL = true whenever the scene is textured, uniforms.debugTextureMode != 0
// or enableDenoiseGBuffer != 0).
template <bool FULL, bool INLINE_PRIMARY = true>
__device__ __forceinline__ void shade_step(const DevScene& S, const Uniforms& U, const ShadeTabs& halton, int hidx,
                                           int sampleIndex, f3& rayO, f3& rayD, const Hit& h, PathRegs& p,
                                           bool gbuf_pending, f2 prevMotion, bool hadPrimaryHit, f2 motionVector,
                                           StepResult& r) {
    r.next = false;
    r.shadow = false;
    r.primary = false;
    r.gbuf = false;
    const float4* const rec = S.tri_nrm + 4 * (size_t)h.id;   // (n1 | ti.w, n2, n0, ti)
    const float4 rn1 = rec[0], rn2 = rec[1], rn0 = rec[2];
    const uint32_t tw = __float_as_uint(rn1.w);
    int instanceIndex = (int)(tw >> 8);
    int geometryIndex = (int)(tw & 0xffu);
    const float* M = halton.instance(instanceIndex);                                    // :329-333 (LDS)
    f3 P_ = rayO + rayD * h.t;                                                          // :336
    const MatRec mat = halton.material(instanceIndex * S.max_submeshes + geometryIndex); // :337-339 (LDS)
    float bu = h.u, bv = h.v, bw = (1.0f - bu) - bv;                                    // :63-65
    const Camera& cam = U.camera;
    f3 cright = ldf3(cam.right), cup = ldf3(cam.up), cfwd = ldf3(cam.forward);

    if (p.bounce == 0 && sampleIndex == 0) {                                            // :342-389
        if (INLINE_PRIMARY) primary_outputs(S, U, h.id, bu, bv, r.depth, r.motion);
        r.primary = true;   // deferred: the caller records the hit for wf_motion
    }

    f3 objN = (bu * ld3(rn1) + bv * ld3(rn2)) + bw * ld3(rn0);                     // :391
    f3 Ng = normalize(xform(M, objN, 0.0f));                                          // :392-393
    if (length_lt_1e10(objN)) Ng = -rayD;                                             // :395-397

    f3 albedo = ld3(mat.base);                                                        // :399
    float roughness = 1.0f, metallic = 0.0f;                                          // :431-441
    const float ao = 1.0f;                                                            // :443-446 (ENABLE_AO 0)
    float opacity = clampf(mat.base.w, 0.0f, 1.0f);                                   // :448
    f3 emission = ld3(mat.emis);                                                      // :453
    // texture maps (:400-456): FULL kernels only (the caller selects FULL for textured scenes)
    unsigned tflags = 0;
    int tnormal = -1;
    f2 tc = f2{0.0f, 0.0f};
    float4 bsample = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
    uint4 ti = make_uint4(0u, 0u, 0u, tw);
    if (FULL && S.textured) {
        ti = __builtin_bit_cast(uint4, rec[3]);   // vertex indices for the UVs and the tangent basis
        const int slot = instanceIndex * S.max_submeshes + geometryIndex;
        const int4 t0 = S.mat_tex[2 * slot], t1 = S.mat_tex[2 * slot + 1];
        tflags = (unsigned)t0.x;
        tnormal = t0.z;
        if (tflags) {                                                                 // :412-417
            const f2 a = ld2(S.uv[ti.y]), b = ld2(S.uv[ti.z]), c = ld2(S.uv[ti.x]);
            tc.x = (bu * a.x + bv * b.x) + bw * c.x;
            tc.y = (bu * a.y + bv * b.y) + bw * c.y;
            tc.y = 1.0f - tc.y;
        }
        if (tflags & MATERIAL_TEXTURE_BASECOLOR) {                                    // :423-428
            bsample = tex_sample(S, t0.y, tc, true);
            albedo = albedo * mk3(bsample.x, bsample.y, bsample.z);
        }
        if (tflags & MATERIAL_TEXTURE_ROUGHNESS) roughness = tex_sample(S, t0.w, tc, false).x;   // :431-434
        if (tflags & MATERIAL_TEXTURE_METALLIC) metallic = tex_sample(S, t1.x, tc, false).x;     // :436-439
        if (tflags & MATERIAL_TEXTURE_OPACITY) opacity = opacity * tex_sample(S, t1.w, tc, false).x;  // :448-451
        if (tflags & MATERIAL_TEXTURE_EMISSION) {                                     // :453-456
            const float4 e = tex_sample(S, t1.z, tc, true);
            emission = mk3(e.x, e.y, e.z);
        }
    }

    if (FULL && U.debugTextureMode != DebugTextureModeNone) {                         // :459-490
        f3 dc = mk3(0.0f, 0.0f, 0.0f);
        int m = U.debugTextureMode;
        if (m == DebugTextureModeBaseColor)
            dc = (tflags & MATERIAL_TEXTURE_BASECOLOR) ? mk3(bsample.x, bsample.y, bsample.z) : mk3(1.0f, 0.0f, 1.0f);
        else if (m == DebugTextureModeNormal) {
            if (tflags & MATERIAL_TEXTURE_NORMAL) {
                const float4 nm = tex_sample(S, tnormal, tc, false);
                dc = mk3(nm.x, nm.y, nm.z);
            } else {
                dc = Ng * 0.5f + mk3(0.5f, 0.5f, 0.5f);
            }
        }
        else if (m == DebugTextureModeRoughness) dc = mk3(roughness, roughness, roughness);
        else if (m == DebugTextureModeMetallic) dc = mk3(metallic, metallic, metallic);
        else if (m == DebugTextureModeAO) dc = mk3(1.0f, 0.0f, 1.0f);
        else if (m == DebugTextureModeEmission) dc = emission;
        else if (m == DebugTextureModeMotion) {
            f2 mp = r.primary ? r.motion : (hadPrimaryHit ? motionVector : prevMotion);
            float scx = clampf(mp.x * 0.05f, -1.0f, 1.0f), scy = clampf(mp.y * 0.05f, -1.0f, 1.0f);
            float mag = clampf(sqrtf(mp.x * mp.x + mp.y * mp.y) * 0.1f, 0.0f, 1.0f);
            dc = mk3(scx * 0.5f + 0.5f, scy * 0.5f + 0.5f, mag);
        }
        p.accum = dc;
        return;  // break
    }

    f3 shadingNormal = Ng;                                                            // :492
    if (FULL && (tflags & MATERIAL_TEXTURE_NORMAL)) {                                 // :493-504
        f3 tangent, bitangent;
        if (tangent_basis(S, ti, tangent, bitangent)) {
            f3 worldT = xform(M, tangent, 0.0f);
            worldT = normalize(worldT - Ng * dot(worldT, Ng));
            const f3 worldB = normalize(cross(Ng, worldT));
            const float4 nm = tex_sample(S, tnormal, tc, false);
            const f3 n = mk3(nm.x * 2.0f - 1.0f, nm.y * 2.0f - 1.0f, nm.z * 2.0f - 1.0f);
            shadingNormal = normalize((n.x * worldT + n.y * worldB) + n.z * Ng);
        }
    }

    if (FULL && gbuf_pending && U.enableDenoiseGBuffer != 0 && sampleIndex == 0) {   // :506-515
        float rr = clampf(roughness, 0.0f, 1.0f);
        f3 da = albedo * (1.0f - metallic);
        f3 sa = mix3(mk3(0.04f, 0.04f, 0.04f), albedo, metallic);
        f3 on = shadingNormal * 0.5f + mk3(0.5f, 0.5f, 0.5f);
        r.g0 = make_float4(da.x, da.y, da.z, 1.0f);
        r.g1 = make_float4(sa.x, sa.y, sa.z, 1.0f);
        r.g2 = make_float4(on.x, on.y, on.z, 1.0f);
        r.g3 = make_float4(rr, 0.0f, 0.0f, 1.0f);
        r.gbuf = true;
    }

    float clampedOpacity = clampf(opacity, 0.0f, 1.0f);                              // :517-576
    float ior = fmaxf(mat.emis.w, 1.0f);
    if (clampedOpacity < 0.999f || ior > 1.01f) {
        f3 N = shadingNormal, I = rayD;
        float cosi = clampf(dot(-I, N), -1.0f, 1.0f);
        float etaI = 1.0f, etaT = ior;
        if (cosi < 0.0f) {
            cosi = -cosi;
            N = -N;
            float tmp = etaI;
            etaI = etaT;
            etaT = tmp;
        }
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
        float choice = halton(hidx, 2 + p.step * 6 + 5);
        bool consumeBounce = true;
        if (k < 0.0f || choice < reflectProb) {
            f3 reflectDir = normalize(I - (2.0f * dot(I, N)) * N);
            rayO = P_ + reflectDir * 1e-3f;
            rayD = reflectDir;
            p.color = p.color * totalWeight;
        } else {
            float cosT = sqrtf(fmaxf(k, 0.0f));
            f3 refractDir = normalize(eta * I + (eta * cosi - cosT) * N);
            rayO = P_ + refractDir * 1e-3f;
            rayD = refractDir;
            p.color = p.color * (totalWeight * albedo);
            consumeBounce = false;
        }
        p.step++;
        if (consumeBounce) {
            p.bounce++;
            p.tpass = 0;
        } else {
            p.tpass++;
            if (p.tpass > U.maxBounces) {
                p.bounce++;
                p.tpass = 0;
            }
        }
        r.next = p.bounce < U.maxBounces;
        return;
    }

    float perceptualRoughness = clampf(roughness, 0.04f, 1.0f);                       // :578-582
    float alpha = perceptualRoughness * perceptualRoughness;
    f3 diffuseColor = albedo;
    f3 F0 = mix3(mk3(0.04f, 0.04f, 0.04f), albedo, metallic);
    f3 V = normalize(-rayD);

    p.accum = p.accum + p.color * emission;                                           // :585

    float lightSample = halton(hidx, 2 + p.step * 6 + 0);                             // :588-591
    int lightIndex = min((int)(lightSample * (float)U.lightCount), U.lightCount - 1);
    const Light& light = halton.light(lightIndex);                                      // (LDS)
    f3 Ldir, lightColor;
    float lightDistance;
    f3 lpos = ldf3(light.position), lcol = ldf3(light.color);
    if (light.type == LightTypeAreaLight) {                                           // :597-606, :95-129
        float ux = halton(hidx, 2 + p.step * 6 + 1), uy = halton(hidx, 2 + p.step * 6 + 2);
        ux = ux * 2.0f - 1.0f;
        uy = uy * 2.0f - 1.0f;
        f3 sp = (lpos + ldf3(light.right) * ux) + ldf3(light.up) * uy;
        Ldir = sp - P_;
        lightDistance = length(Ldir);
        float inv = 1.0f / fmaxf(lightDistance, 1e-3f);
        Ldir = Ldir * inv;
        lightColor = lcol * (inv * inv);
        lightColor = lightColor * saturate(dot(-Ldir, ldf3(light.forward)));
    } else if (light.type == LightTypeSpotlight) {                                    // :608-632
        Ldir = lpos - P_;
        lightDistance = length(Ldir);
        float inv = 1.0f / fmaxf(lightDistance, 1e-3f);
        Ldir = Ldir * inv;
        lightColor = mk3(0.0f, 0.0f, 0.0f);
        f3 coneDirection = normalize(ldf3(light.direction));
        float spotResult = dot(-Ldir, coneDirection);
        if (spotResult > cos_pinned(light.coneAngle)) lightColor = (lcol * inv) * inv;
    } else if (light.type == LightTypePointlight) {                                   // :633-638
        Ldir = lpos - P_;
        lightDistance = length(Ldir);
        float inv = 1.0f / fmaxf(lightDistance, 1e-3f);
        Ldir = Ldir * inv;
        lightColor = (lcol * inv) * inv;
    } else {                                                                          // :639-643
        Ldir = -normalize(ldf3(light.direction));
        lightDistance = INFINITY;
        lightColor = lcol;
    }
    lightColor = lightColor * (float)U.lightCount;                                    // :647
    f3 origin = P_ + Ng * 1e-3f;                                                      // :660, :683, :720, :769

    if (U.shadingMode == ShadingModeLegacy) {                                         // :649-690
        f3 L = normalize(Ldir);
        float NdotL = saturate(dot(shadingNormal, L));
        f3 legacyColor = p.color * albedo;
        if (length_lt_1e3(legacyColor)) return;
        if (length_gt_1e4(lightColor) && NdotL > 0.0f) {
            r.shadow = true;
            r.so = origin;
            r.sd = Ldir;
            r.stmax = lightDistance - 1e-3f;
            r.contrib = (legacyColor * lightColor) * NdotL;
        }
        p.color = legacyColor * ao;
        if (length_lt_1e3(p.color)) return;
        float r0 = halton(hidx, 2 + p.step * 5 + 3), r1 = halton(hidx, 2 + p.step * 5 + 4);
        rayD = alignHemisphereWithNormal(sampleCosineWeightedHemisphere(r0, r1), shadingNormal);
        rayO = origin;
        p.step++;
        p.bounce++;
        p.tpass = 0;
        r.next = p.bounce < U.maxBounces;
        return;
    }

    if (length_gt_1e4(lightColor)) {                                                  // :692-744
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
        r.shadow = true;
        r.so = origin;
        r.sd = Ldir;
        r.stmax = lightDistance - 1e-3f;
        r.contrib = p.color * direct;
    }

    p.color = p.color * ((diffuseColor * (1.0f - metallic)) * ao);                    // :748
    if (length_lt_1e3(p.color)) return;                                               // :751-753
    float r0 = halton(hidx, 2 + p.step * 5 + 3), r1 = halton(hidx, 2 + p.step * 5 + 4);  // :763-764
    rayD = alignHemisphereWithNormal(sampleCosineWeightedHemisphere(r0, r1), shadingNormal);
    rayO = origin;                                                                    // :769-770
    p.step++;
    p.bounce++;
    p.tpass = 0;
    r.next = p.bounce < U.maxBounces;
}

// Primary ray for (pixel, sample) (Raytracing.metal:270-292).
__device__ __forceinline__ void primary_ray(const Uniforms& U, const ShadeTabs& halton, int px, int py, int hidx,
                                            f3& o, f3& d) {
    float rx = halton(hidx, 0), ry = halton(hidx, 1);
    float spx = (float)px + rx, spy = (float)py + ry;
    float uvx = spx / (float)U.width, uvy = spy / (float)U.height;
    uvx = uvx * 2.0f - 1.0f;
    uvy = uvy * 2.0f - 1.0f;
    const Camera& cam = U.camera;
    o = ldf3(cam.position);
    d = normalize((uvx * ldf3(cam.right) + uvy * ldf3(cam.up)) + ldf3(cam.forward));
}

// Motion-adaptive extra samples after sample 0 (Raytracing.metal:779-789).
__device__ __forceinline__ int extra_samples(const Uniforms& U, int maxExtra, f2 mv, f2 pm) {
    float motionMag = fmaxf(sqrtf(mv.x * mv.x + mv.y * mv.y), sqrtf(pm.x * pm.x + pm.y * pm.y));
    float low = fmaxf(U.motionSamplingLowThresholdPixels, 0.0f);
    float high = fmaxf(U.motionSamplingHighThresholdPixels, low + 1e-3f);
    float t = clampf((motionMag - low) / (high - low), 0.0f, 1.0f);
    int e = (int)roundf(t * (float)maxExtra);
    return min(max(e, 0), maxExtra);
}

// Average + temporal EMA (Raytracing.metal:792-817).
__device__ __forceinline__ f3 resolve_pixel(const Uniforms& U, f3 total, int totalSamples, f2 mv, f2 pm,
                                            const float4* accum_in, size_t pix) {
    total = total / (float)max(totalSamples, 1);
    if (U.frameIndex > 0) {
        float4 pc = accum_in[pix];
        f3 prevColor = mk3(pc.x, pc.y, pc.z);
        float historyWeight = clampf(U.accumulationWeight, 0.0f, 0.95f);
        if (U.enableMotionAdaptiveAccumulation != 0) {
            float motionMag = fmaxf(sqrtf(mv.x * mv.x + mv.y * mv.y), sqrtf(pm.x * pm.x + pm.y * pm.y));
            float low = fmaxf(U.motionAccumulationLowThresholdPixels, 0.0f);
            float high = fmaxf(U.motionAccumulationHighThresholdPixels, low + 1e-3f);
            float t = clampf((motionMag - low) / (high - low), 0.0f, 1.0f);
            float minWeight = clampf(U.motionAccumulationMinWeight, 0.0f, 0.95f);
            minWeight = fminf(minWeight, historyWeight);
            historyWeight = mixf(historyWeight, minWeight, t);
        }
        total = mix3(total, prevColor, historyWeight);
    }
    return total;
}

}  // namespace rt
