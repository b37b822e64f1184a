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

}  // namespace

void launch_present(const float4* accum, const float* depth, const float2* motion, const float4* hist_in,
                    const float* hdepth_in, float4* hist_out, float* hdepth_out, uchar4* out, const float* thr, int w,
                    int h, int ow, int oh, int scaler, int srgb, int use_hist, hipStream_t stream) {
    dim3 grid((ow + 15) / 16, (oh + 15) / 16);
    hipLaunchKernelGGL(present_k, grid, dim3(256), 0, stream, accum, depth, motion, hist_in, hdepth_in, hist_out,
                       hdepth_out, out, thr, w, h, ow, oh, scaler, srgb, use_hist);
}

}  // namespace rt
