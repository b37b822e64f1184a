// rt_math.h — scalar math of the hot path, compiled for gfx950 (device) and x86-64 (host).
//
// Restates the helper functions of MetalRaytracing/Raytracing.metal:28-166 with an exactly
// specified arithmetic order so that the HIP kernels and the CPU oracle (oracle/, an
// independent C restatement of the same reference lines) produce bit-identical floats:
//   * no FMA contraction (-ffp-contract=off on every compile line + the pragma below);
//   * only IEEE-correctly-rounded primitives (+ - * / sqrt, conversions, min/max, rint);
//   * transcendental functions (sin/cos for the cosine-hemisphere sample, cos(coneAngle),
//     pow(x,5) of the Schlick terms) are pinned polynomial / product formulas defined here,
//     because the reference's fast-math Metal library versions are implementation-defined
//     (project.pbxproj MTL_FAST_MATH=YES).
// Vector type f3 is a 3-float value; storage uses 16-byte float4 rows (rt_types.h).
#pragma once

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__) || defined(__HIP_DEVICE_COMPILE__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD static inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace rt {

struct f3 { float x, y, z; };
struct f2 { float x, y; };

RT_HD f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
RT_HD f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD f3 operator-(f3 a) { return mk3(-a.x, -a.y, -a.z); }
RT_HD f3 operator*(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_HD f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
RT_HD f3 operator*(float s, f3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
RT_HD f3 operator/(f3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
RT_HD float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
RT_HD f3 cross(f3 a, f3 b) {
    return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
RT_HD float length(f3 a) { return sqrtf(dot(a, a)); }
// length(a) < c / length(a) > c for the constants the shading code compares against, without the
// square root: sqrtf and round-to-nearest are monotonic, so each comparison is one on dot(a, a)
// against the first / last float on the other side -- the same result for every input (found and
// checked over every non-negative float: tools/sqrt_thresholds.c, tests/test_sqrt_thresholds.py).
RT_HD bool length_lt_1e10(f3 a) { return dot(a, a) < 0x1.79ca1p-67f; }    // length(a) < 1e-10f
RT_HD bool length_lt_1e3(f3 a) { return dot(a, a) < 0x1.0c6f7ap-20f; }    // length(a) < 0.001f
RT_HD bool length_gt_1e4(f3 a) { return dot(a, a) > 0x1.5798eep-27f; }    // length(a) > 0.0001f
// normalize(v) = v * (1/sqrt(dot(v,v)))  (Metal: v * rsqrt(dot(v,v)))
RT_HD f3 normalize(f3 a) { float inv = 1.0f / sqrtf(dot(a, a)); return a * inv; }
RT_HD float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
RT_HD float saturate(float x) { return clampf(x, 0.0f, 1.0f); }
// Metal mix(x, y, a) = x + (y - x) * a
RT_HD float mixf(float x, float y, float a) { return x + (y - x) * a; }
RT_HD f3 mix3(f3 x, f3 y, float a) { return mk3(mixf(x.x, y.x, a), mixf(x.y, y.y, a), mixf(x.z, y.z, a)); }
RT_HD f3 mix3v(f3 x, f3 y, f3 a) { return mk3(mixf(x.x, y.x, a.x), mixf(x.y, y.y, a.y), mixf(x.z, y.z, a.z)); }

static constexpr float RT_PI = 3.14159265358979323846f;  // M_PI_F

// ---- pinned transcendentals ---------------------------------------------------------------
// sin/cos: Cody-Waite reduction by pi/2 (3-part split), then the Cephes single-precision
// minimax polynomials on [-pi/4, pi/4].  Max abs error ~1e-7 on [0, 2pi].
RT_HD void sincos_pinned(float x, float* s, float* c) {
    float j = rintf(x * 0.63661977236758134f);
    int q = (int)j;
    float r = x - j * 1.5703125f;
    r = r - j * 4.837512969970703125e-4f;
    r = r - j * 7.54978995489188216e-8f;
    float z = r * r;
    float sr = r + r * z * (-1.6666654611e-1f + z * (8.3321608736e-3f + z * (-1.9515295891e-4f)));
    float cr = (1.0f - 0.5f * z) + z * z * (4.166664568298827e-2f + z * (-1.388731625493765e-3f + z * 2.443315711809948e-5f));
    switch (q & 3) {
        case 0: *s = sr; *c = cr; break;
        case 1: *s = cr; *c = -sr; break;
        case 2: *s = -sr; *c = -cr; break;
        default: *s = -cr; *c = sr; break;
    }
}
RT_HD float cos_pinned(float x) { float s, c; sincos_pinned(x, &s, &c); return c; }
// pow(x, 5) for x in [0,1] (Raytracing.metal:165, :537): ((x*x)*(x*x))*x
RT_HD float pow5(float x) { float x2 = x * x; return (x2 * x2) * x; }

// ---- Halton (Raytracing.metal:28-57) --------------------------------------------------------
// The reference's primes[] has 100 entries; dimension 2+6*step+5 exceeds it once step >= 16
// (reachable by glass paths, SURVEY.md §7 hard part 3).  Documented extension: the first 1024
// primes (first 100 identical), which covers every dimension for maxBounces <= 12.
static constexpr int RT_HALTON_DIMS = 1024;
static constexpr int RT_MAX_BOUNCES = 12;

// Exact division of 31-bit non-negative ints by prime b: q = (umulhi(n, m) >> sh) with
// m = ceil(2^(31+l)/b), sh = l-1, 2^(l-1) < b <= 2^l (Granlund-Montgomery).  Integer result
// is identical to n / b, so the float sequence is identical to the reference loop.
struct HaltonDim { uint32_t b; uint32_t m; uint32_t sh; float invB; };

RT_HD uint32_t umulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
#endif
}

RT_HD float halton_fast(int i, const HaltonDim& h) {
    float f = 1.0f, r = 0.0f;
    uint32_t n = (uint32_t)i;
    if (i <= 0) return 0.0f;
    while (n > 0) {
        f = f * h.invB;
        uint32_t q = umulhi32(n, h.m) >> h.sh;
        r = r + f * (float)(n - q * h.b);
        n = q;
    }
    return r;
}

// halton_fast for base 2 (dimension 0) in closed form: the loop adds the bits of i, lowest first,
// at weights 2^-1, 2^-2, ...; each sum is exact until 24 significant bits are held, the next bit is
// a tie (exactly half an ulp: round to even) and every later bit is below half an ulp.  So the
// result is the bit-reversed fraction cut to 24 significant bits plus that one tie.  Bit-identical
// to the loop for every int (checked exhaustively over all 2^31 positive i: tools/halton2_check.c).
RT_HD uint32_t bitrev32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bitreverse32(x);
#else
    x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0f0f0f0fu) | ((x & 0x0f0f0f0fu) << 4);
    x = ((x >> 8) & 0x00ff00ffu) | ((x & 0x00ff00ffu) << 8);
    return (x >> 16) | (x << 16);
#endif
}
RT_HD float halton_base2(int i) {
    if (i <= 0) return 0.0f;
    const uint32_t b = bitrev32((uint32_t)i);   // i's bits as a 32-bit fraction (bit 31 = weight 1/2)
    uint32_t r = b;
    const int drop = 8 - __builtin_clz(b);      // bits below the 24 kept from the leading one
    if (drop > 0) {
        const uint32_t half = (b >> (drop - 1)) & 1u, last = (b >> drop) & 1u;
        r = b & ~((1u << drop) - 1u);
        if (half & last) {
            r += 1u << drop;
            if (r == 0u) return 1.0f;           // carried out of the fraction
        }
    }
    return (float)r * 2.3283064365386963e-10f;  // exact: <= 24 significant bits, times 2^-32
}

// ---- sampling helpers ------------------------------------------------------------------------
// Raytracing.metal:79-89
RT_HD f3 sampleCosineWeightedHemisphere(float ux, float uy) {
    float phi = 2.0f * RT_PI * ux;
    float sin_phi, cos_phi;
    sincos_pinned(phi, &sin_phi, &cos_phi);
    float cos_theta = sqrtf(uy);
    float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
    return mk3(sin_theta * cos_phi, cos_theta, sin_theta * sin_phi);
}
// Raytracing.metal:133-148
RT_HD f3 alignHemisphereWithNormal(f3 s, f3 normal) {
    f3 up = normal;
    f3 right = normalize(cross(normal, mk3(0.0072f, 1.0f, 0.0034f)));
    f3 forward = cross(right, up);
    return (s.x * right + s.y * up) + s.z * forward;
}
// Raytracing.metal:150-166
RT_HD float distributionGGX(float NdotH, float alpha) {
    float a2 = alpha * alpha;
    float denom = (NdotH * NdotH) * (a2 - 1.0f) + 1.0f;
    return a2 / fmaxf(RT_PI * denom * denom, 1e-7f);
}
RT_HD float geometrySchlickGGX(float NdotV, float k) {
    return NdotV / fmaxf(NdotV * (1.0f - k) + k, 1e-7f);
}
RT_HD float geometrySmith(float NdotV, float NdotL, float k) {
    return geometrySchlickGGX(NdotV, k) * geometrySchlickGGX(NdotL, k);
}
RT_HD f3 fresnelSchlick(float cosTheta, f3 F0) {
    float p = pow5(clampf(1.0f - cosTheta, 0.0f, 1.0f));
    return mk3(F0.x + (1.0f - F0.x) * p, F0.y + (1.0f - F0.y) * p, F0.z + (1.0f - F0.z) * p);
}

// ---- intersection -----------------------------------------------------------------------------
// Watertight ray/triangle (Woop, Benthin, Wald, JCGT 2013), no culling, t in [tmin, tmax].
// Barycentrics follow Metal's triangle_barycentric_coord (Raytracing.metal:63-73):
// u weights vertex 1, v weights vertex 2, 1-u-v weights vertex 0.
// The axes are cycled, never swapped: kz = the largest |d| component, kx = kz + 1, ky = kz + 2
// (mod 3).  (Woop et al. swap kx / ky when d[kz] < 0 to keep the winding for back-face culling;
// with no culling the swap negates U, V, W, det and T together, which leaves t, u, v and every
// accept / reject decision unchanged up to the sign of exact zeros -- DESIGN.md §4; the oracle
// states the same.)  Without the swap, a vertex's (kz, kx, ky) components are three consecutive
// floats of (x, y, z, x, y) starting at kz: the triangle record stores each vertex that way and a
// lane loads its ray's window directly (rt_device.h tri_window), no per-component selects.
struct RayPre {
    int kz;
    float Sx, Sy, Sz;
};
RT_HD float comp(f3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }
// (v[kz], v[kx], v[ky]) as (x, y, z)
RT_HD f3 rot3(f3 v, int kz) { return kz == 0 ? mk3(v.x, v.y, v.z) : (kz == 1 ? mk3(v.y, v.z, v.x) : mk3(v.z, v.x, v.y)); }
RT_HD RayPre ray_precompute(f3 d) {
    RayPre p;
    float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    int kz = (ax > ay) ? ((ax > az) ? 0 : 2) : ((ay > az) ? 1 : 2);
    const f3 r = rot3(d, kz);   // (d[kz], d[kx], d[ky])
    p.kz = kz;
    p.Sx = r.y / r.x;
    p.Sy = r.z / r.x;
    p.Sz = 1.0f / r.x;
    return p;
}
// Vertices a, b, c and the origin o already in (kz, kx, ky) order (rot3 / tri_window).
// Returns true on hit and writes t and the unnormalised (V, W, det): u = V / det, v = W / det
// (the divisions happen once, for the closest hit, not for every candidate).
RT_HD bool intersect_rot(const RayPre& p, f3 o, f3 a, f3 b, f3 c, float tmin, float tmax,
                         float* t_out, float* V_out, float* W_out, float* det_out) {
    const float Akz = a.x - o.x, Bkz = b.x - o.x, Ckz = c.x - o.x;
    const float Ax = (a.y - o.y) - p.Sx * Akz;
    const float Ay = (a.z - o.z) - p.Sy * Akz;
    const float Bx = (b.y - o.y) - p.Sx * Bkz;
    const float By = (b.z - o.z) - p.Sy * Bkz;
    const float Cx = (c.y - o.y) - p.Sx * Ckz;
    const float Cy = (c.z - o.z) - p.Sy * Ckz;
    float U = Cx * By - Cy * Bx;
    float V = Ax * Cy - Ay * Cx;
    float W = Bx * Ay - By * Ax;
    if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return false;
    float det = (U + V) + W;
    if (det == 0.0f) return false;
    float Az = p.Sz * Akz, Bz = p.Sz * Bkz, Cz = p.Sz * Ckz;
    float T = (U * Az + V * Bz) + W * Cz;
    float t = T / det;
    if (!(t >= tmin && t <= tmax)) return false;
    *t_out = t;
    *V_out = V;
    *W_out = W;
    *det_out = det;
    return true;
}
// The same test on world-space vertices (host tools).
RT_HD bool intersect_triangle_vw(const RayPre& p, f3 o, f3 v0, f3 v1, f3 v2, float tmin, float tmax,
                                 float* t_out, float* V_out, float* W_out, float* det_out) {
    return intersect_rot(p, rot3(o, p.kz), rot3(v0, p.kz), rot3(v1, p.kz), rot3(v2, p.kz), tmin, tmax, t_out, V_out,
                         W_out, det_out);
}

}  // namespace rt
