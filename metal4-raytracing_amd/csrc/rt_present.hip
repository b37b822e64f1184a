// rt_present.hip — the display side of a frame: what FramePresenter.swift
// (:103-238) and Shaders.metal (:39-52) do with the newest accumulation target, the depth and the
// motion vectors, as one kernel writing 8-bit RGBA rows in display order (row 0 = top).
//
//   scaler NONE      one output pixel per render pixel, nearest (the presenter's fragment shader
//                    with sampler(nearest) over a full-screen quad);
//   scaler SPATIAL   bilinear resampling of the render target to the output size, clamp to edge
//                    (stand-in for MTLFXSpatialScaler, whose filter is unpublished);
//   scaler TEMPORAL  the spatial resample blended with the previous output reprojected through the
//                    motion vectors (MTLFXTemporalScaler's inputs: colour, depth, motion; its
//                    algorithm is unpublished): history sampled bilinearly at the reprojected
//                    position, clamped to the min/max of the 3x3 render-pixel neighbourhood,
//                    blended 0.9 history / 0.1 current; no history (first frame, frameIndex 0,
//                    reprojection off screen, or a depth jump > 10 % against the history depth)
//                    gives the current value.
//
// Then `color / (1 + color)` (Shaders.metal:50) and the encode: sRGB 8-bit through 255 ascending
// thresholds (the linear values whose sRGB code is k + 0.5, computed in double on the host), or
// linear 8-bit round(v * 255).  Every arithmetic step has a fixed order so a numpy restatement
// reproduces the bytes exactly (tests/test_gpu_present.py).
#include "rt_kernels.h"
#include "../../include/rt_api.h"

namespace rt {
namespace {

__device__ __forceinline__ float4 ld_clamped(const float4* img, int w, int h, int x, int y) {
    x = min(max(x, 0), w - 1);
    y = min(max(y, 0), h - 1);
    return img[(size_t)y * w + x];
}

// bilinear, clamp to edge, texel centres at integer coordinates (x, y in texel units)
__device__ __forceinline__ float4 bilinear(const float4* img, int w, int h, float x, float y) {
    const float fx = floorf(x), fy = floorf(y);
    const float ax = x - fx, ay = y - fy, bx = 1.0f - ax, by = 1.0f - ay;
    const int x0 = (int)fx, y0 = (int)fy;
    const float4 c00 = ld_clamped(img, w, h, x0, y0), c10 = ld_clamped(img, w, h, x0 + 1, y0);
    const float4 c01 = ld_clamped(img, w, h, x0, y0 + 1), c11 = ld_clamped(img, w, h, x0 + 1, y0 + 1);
    float4 r;
    r.x = (c00.x * bx + c10.x * ax) * by + (c01.x * bx + c11.x * ax) * ay;
    r.y = (c00.y * bx + c10.y * ax) * by + (c01.y * bx + c11.y * ax) * ay;
    r.z = (c00.z * bx + c10.z * ax) * by + (c01.z * bx + c11.z * ax) * ay;
    r.w = (c00.w * bx + c10.w * ax) * by + (c01.w * bx + c11.w * ax) * ay;
    return r;
}

__device__ __forceinline__ unsigned encode8(float c, const float* thr, int srgb) {
    const float v = c > 0.0f ? c / (1.0f + c) : 0.0f;   // Shaders.metal:50 (NaN / negative -> 0)
    if (!srgb) {
        const float q = floorf(v * 255.0f + 0.5f);
        return (unsigned)fminf(q, 255.0f);
    }
    unsigned lo = 0, hi = 255;   // number of thresholds <= v
    while (lo < hi) {
        const unsigned mid = (lo + hi) >> 1;
        if (thr[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(256) present_k(const float4* __restrict__ accum, const float* __restrict__ depth,
                                                 const float2* __restrict__ motion, const float4* __restrict__ hist_in,
                                                 const float* __restrict__ hdepth_in, float4* __restrict__ hist_out,
                                                 float* __restrict__ hdepth_out, uchar4* __restrict__ out,
                                                 const float* __restrict__ thr, int w, int h, int ow, int oh,
                                                 int scaler, int srgb, int use_hist) {
    const int ox = blockIdx.x * 16 + (threadIdx.x & 15), oyd = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (ox >= ow || oyd >= oh) return;
    const int oy = oh - 1 - oyd;   // render rows run bottom-up (tid.y), display rows top-down
    float4 c;
    if (scaler == RT_SCALER_NONE) {   // nearest at the output pixel's centre
        const int tx = min((int)(((float)ox + 0.5f) / (float)ow * (float)w), w - 1);
        const int ty = min((int)(((float)oy + 0.5f) / (float)oh * (float)h), h - 1);
        c = accum[(size_t)ty * w + tx];
    } else {
        const float sx = (float)w / (float)ow, sy = (float)h / (float)oh;
        const float px = ((float)ox + 0.5f) * sx - 0.5f, py = ((float)oy + 0.5f) * sy - 0.5f;
        c = bilinear(accum, w, h, px, py);
        if (scaler == RT_SCALER_TEMPORAL) {
            const int nx = min(max((int)floorf(px + 0.5f), 0), w - 1), ny = min(max((int)floorf(py + 0.5f), 0), h - 1);
            float4 mn = accum[(size_t)ny * w + nx], mx = mn;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    const float4 q = ld_clamped(accum, w, h, nx + dx, ny + dy);
                    mn.x = fminf(mn.x, q.x), mn.y = fminf(mn.y, q.y), mn.z = fminf(mn.z, q.z);
                    mx.x = fmaxf(mx.x, q.x), mx.y = fmaxf(mx.y, q.y), mx.z = fmaxf(mx.z, q.z);
                }
            const float2 m = motion[(size_t)ny * w + nx];   // render pixels, +y down the screen
            const float d = depth[(size_t)ny * w + nx];
            const float qx = px - m.x, qy = py + m.y;       // previous render position (rows bottom-up)
            const float hx = (qx + 0.5f) / sx - 0.5f, hy = (qy + 0.5f) / sy - 0.5f;
            bool ok = use_hist && qx >= -0.5f && qx <= (float)w - 0.5f && qy >= -0.5f && qy <= (float)h - 0.5f;
            if (ok) {
                const int hnx = min(max((int)floorf(hx + 0.5f), 0), ow - 1), hny = min(max((int)floorf(hy + 0.5f), 0), oh - 1);
                const float hd = hdepth_in[(size_t)hny * ow + hnx];
                ok = fabsf(hd - d) <= 0.1f * fmaxf(d, hd);
            }
            if (ok) {
                float4 hv = bilinear(hist_in, ow, oh, hx, hy);
                hv.x = fminf(fmaxf(hv.x, mn.x), mx.x);
                hv.y = fminf(fmaxf(hv.y, mn.y), mx.y);
                hv.z = fminf(fmaxf(hv.z, mn.z), mx.z);
                c.x = hv.x + (c.x - hv.x) * 0.1f;
                c.y = hv.y + (c.y - hv.y) * 0.1f;
                c.z = hv.z + (c.z - hv.z) * 0.1f;
            }
            const size_t o = (size_t)oy * ow + ox;
            hist_out[o] = make_float4(c.x, c.y, c.z, 1.0f);
            hdepth_out[o] = d;
        }
    }
    uchar4 r;
    r.x = (unsigned char)encode8(c.x, thr, srgb);
    r.y = (unsigned char)encode8(c.y, thr, srgb);
    r.z = (unsigned char)encode8(c.z, thr, srgb);
    r.w = 255;
    out[(size_t)oyd * ow + ox] = r;
}

// ---- RT_SCALER_DENOISED: G-buffer-guided denoise ahead of the temporal scaler ----------------
// Stand-in for MTLFXTemporalDenoisedScaler (FramePresenter.swift:77-98,179-198), which consumes
// colour, depth, motion and the four G-buffer planes of Raytracing.metal:506-515 with an
// unpublished algorithm.  Here: demodulate the radiance by diffuse + specular albedo, run
// `passes` edge-avoiding a-trous passes (5x5 B3-spline taps at step 1, 2, 4, ...; weights
// max(0, n.n')^16 from the decoded G-buffer normals and 1 / (1 + (dz / (0.05 step z))^2) from
// the depth; background only with background), remodulate, then the TEMPORAL path above.  All
// arithmetic is written in a fixed order without contraction (tests/test_gpu_present.py
// restates it in numpy byte for byte).

// illum = radiance / albedo, guide = (normal, depth) on hits, (0, 0, 0, -1) on background,
// alb = the demodulation albedo (1 where diffuse + specular albedo <= 1e-3 or no hit)
__global__ void __launch_bounds__(256) denoise_prep_k(const float4* __restrict__ accum, const float* __restrict__ depth,
                                                      const float4* __restrict__ gbuf, float4* __restrict__ illum,
                                                      float4* __restrict__ guide, float4* __restrict__ alb, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 c = accum[i], g0 = gbuf[i], g1 = gbuf[(size_t)n + i], g2 = gbuf[2 * (size_t)n + i];
    const bool hit = g2.w > 0.5f;
    float ax = g0.x + g1.x, ay = g0.y + g1.y, az = g0.z + g1.z;
    ax = (hit && ax > 1e-3f) ? ax : 1.0f;
    ay = (hit && ay > 1e-3f) ? ay : 1.0f;
    az = (hit && az > 1e-3f) ? az : 1.0f;
    illum[i] = make_float4(c.x / ax, c.y / ay, c.z / az, c.w);
    guide[i] = hit ? make_float4(g2.x * 2.0f - 1.0f, g2.y * 2.0f - 1.0f, g2.z * 2.0f - 1.0f, depth[i])
                   : make_float4(0.0f, 0.0f, 0.0f, -1.0f);
    alb[i] = make_float4(ax, ay, az, 1.0f);
}

__global__ void __launch_bounds__(256) denoise_atrous_k(const float4* __restrict__ in, const float4* __restrict__ guide,
                                                        const float4* __restrict__ alb, float4* __restrict__ out, int w,
                                                        int h, int step, int last) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= w || y >= h) return;
    const size_t i = (size_t)y * w + x;
    const float4 p = guide[i];
    const float kern[5] = {0.0625f, 0.25f, 0.375f, 0.25f, 0.0625f};
    const float zs = 0.05f * (float)step * p.w;
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    for (int dy = -2; dy <= 2; ++dy) {
        const int yy = y + dy * step;
        if (yy < 0 || yy >= h) continue;
        for (int dx = -2; dx <= 2; ++dx) {
            const int xx = x + dx * step;
            if (xx < 0 || xx >= w) continue;
            const size_t j = (size_t)yy * w + xx;
            const float4 q = guide[j];
            float wgt = kern[dy + 2] * kern[dx + 2];
            if (p.w < 0.0f || q.w < 0.0f) {
                if (p.w >= 0.0f || q.w >= 0.0f) continue;   // hit next to background: no weight
            } else {
                float t = fmaxf(p.x * q.x + p.y * q.y + p.z * q.z, 0.0f);
                t = t * t;
                t = t * t;
                t = t * t;
                t = t * t;
                const float dz = fabsf(p.w - q.w) / zs;
                wgt = (wgt * t) / (1.0f + dz * dz);
            }
            const float4 c = in[j];
            sx = sx + c.x * wgt;
            sy = sy + c.y * wgt;
            sz = sz + c.z * wgt;
            sw = sw + wgt;
        }
    }
    const float4 c0 = in[i];
    float4 r = sw > 0.0f ? make_float4(sx / sw, sy / sw, sz / sw, c0.w) : c0;
    if (last) {
        const float4 a = alb[i];
        r.x = r.x * a.x;
        r.y = r.y * a.y;
        r.z = r.z * a.z;
    }
    out[i] = r;
}

}  // namespace

const float4* launch_denoise(const float4* accum, const float* depth, const float4* gbuf, float4* tmp0, float4* tmp1,
                             float4* guide, float4* alb, int w, int h, int passes, hipStream_t stream) {
    const int n = w * h;
    hipLaunchKernelGGL(denoise_prep_k, dim3((n + 255) / 256), dim3(256), 0, stream, accum, depth, gbuf, tmp0, guide,
                       alb, n);
    float4* src = tmp0;
    float4* dst = tmp1;
    dim3 grid((w + 15) / 16, (h + 15) / 16);
    for (int k = 0; k < passes; ++k) {
        hipLaunchKernelGGL(denoise_atrous_k, grid, dim3(256), 0, stream, src, guide, alb, dst, w, h, 1 << k,
                           k == passes - 1 ? 1 : 0);
        float4* t = src;
        src = dst;
        dst = t;
    }
    return src;
}

void launch_present(const float4* accum, const float* depth, const float2* motion, const float4* hist_in,
                    const float* hdepth_in, float4* hist_out, float* hdepth_out, uchar4* out, const float* thr, int w,
                    int h, int ow, int oh, int scaler, int srgb, int use_hist, hipStream_t stream) {
    dim3 grid((ow + 15) / 16, (oh + 15) / 16);
    hipLaunchKernelGGL(present_k, grid, dim3(256), 0, stream, accum, depth, motion, hist_in, hdepth_in, hist_out,
                       hdepth_out, out, thr, w, h, ow, oh, scaler, srgb, use_hist);
}

}  // namespace rt
