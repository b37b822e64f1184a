/*
 * rt_oracle.c — CPU restatement of raytracingKernel (Raytracing.metal:220-831).
 * TEST INFRASTRUCTURE ONLY (see rt_oracle.h).  Build: oracle/Makefile
 * (gcc -O3 -std=gnu11 -ffp-contract=off -fno-fast-math -pthread).
 *
 * Every function cites the reference lines it restates.  Arithmetic is written with explicit
 * evaluation order; DESIGN.md §4 is the shared specification with the HIP path.
 */
#include "rt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- vector helpers (float3) */
typedef struct { float x, y, z; } V3;

static inline V3 v3(float x, float y, float z) { V3 r = {x, y, z}; return r; }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 vscl(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline V3 vdivs(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline float vdot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline V3 vcross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static inline float vlen(V3 a) { return sqrtf(vdot(a, a)); }
static inline V3 vnorm(V3 a) { float inv = 1.0f / sqrtf(vdot(a, a)); return vscl(a, inv); }
static inline float clampf_(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
static inline float satf(float x) { return clampf_(x, 0.0f, 1.0f); }
static inline float mixf_(float x, float y, float a) { return x + (y - x) * a; } /* Metal mix */
static inline V3 vmix(V3 x, V3 y, float a) { return v3(mixf_(x.x, y.x, a), mixf_(x.y, y.y, a), mixf_(x.z, y.z, a)); }
static inline V3 f3v(rt_float3 f) { return v3(f.x, f.y, f.z); }
static inline float vcomp(V3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

#define ORC_PI 3.14159265358979323846f /* M_PI_F */

/* ---------------------------------------------------------------- pinned transcendentals */
/* sin/cos of Raytracing.metal:83 and cos of :630, pinned: Cody-Waite pi/2
 * reduction + Cephes sinf/cosf minimax polynomials. */
void rt_oracle_sincos(float x, float* s, float* c) {
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
/* pow(x, 5.0f) of Raytracing.metal:165 and :537, x in [0,1] */
float rt_oracle_pow5(float x) { float x2 = x * x; return (x2 * x2) * x; }

/* ---------------------------------------------------------------- Halton (:28-57) */
static int g_primes[1024];
static pthread_once_t g_primes_once = PTHREAD_ONCE_INIT;
static void init_primes(void) {
    int n = 2, k = 0;
    while (k < 1024) {
        int is = 1;
        for (int i = 0; i < k && g_primes[i] * g_primes[i] <= n; ++i)
            if (n % g_primes[i] == 0) { is = 0; break; }
        if (is) g_primes[k++] = n;
        ++n;
    }
}
/* Raytracing.metal:42-57, primes[] extended from 100 to 1024 entries (first 100 identical). */
float rt_oracle_halton(int32_t i, int32_t d) {
    pthread_once(&g_primes_once, init_primes);
    int b = g_primes[d];
    float f = 1.0f;
    float invB = 1.0f / (float)b;
    float r = 0;
    while (i > 0) {
        f = f * invB;
        r = r + f * (float)(i % b);
        i = i / b;
    }
    return r;
}

/* ---------------------------------------------------------------- scene */
typedef struct {
    float lo[3], hi[3];
    int32_t left, right;   /* left < 0: leaf */
    uint32_t start, count;
} ONode;

typedef struct {
    uint32_t mesh, sub;
    uint32_t i0, i1, i2;   /* mesh-local vertex indices (SubMesh index buffer order) */
} OTri;

struct rt_oracle_scene {
    uint32_t ntri, nmesh, nlight;
    float* world;          /* 9 per triangle, original order */
    OTri* tri;
    uint32_t* order;       /* BVH leaf order -> original id */
    ONode* nodes;
    uint32_t nnodes;
    float pad;
    /* per mesh */
    const rt_float3** pos;
    const rt_float3** nrm;
    float (*xf)[12];
    float (*prev_xf)[12];
    const rt_float3** prev_pos;
    Material** mats;       /* [mesh][sub] */
    Light* lights;
    /* texture path (SubMesh.swift:69-241, Raytracing.metal:399-504) */
    const rt_float2** uv;  /* per mesh, NULL = zero UVs (Model.swift:329-333) */
    int32_t (**mtex)[8];   /* [mesh][sub] texture per slot */
    const rt_texture_desc* tex;
    uint32_t ntex;
    float lut[512];        /* byte -> float: linear, then sRGB */
};

/* object->world: ((c0*x + c1*y) + c2*z) + c3*w with the MTLPackedFloat4x3 columns
 * (Raytracing.metal:329-333, :348, :392) */
static inline V3 oxform(const float* m, V3 p, float w) {
    V3 c0 = v3(m[0], m[1], m[2]), c1 = v3(m[3], m[4], m[5]), c2 = v3(m[6], m[7], m[8]), c3 = v3(m[9], m[10], m[11]);
    return vadd(vadd(vadd(vscl(c0, p.x), vscl(c1, p.y)), vscl(c2, p.z)), vscl(c3, w));
}

/* Binned-SAH BVH over triangle centroids (16 bins per axis, all three axes), leaves of <= 4
 * triangles, iterative.  Its own builder, independent of the product's (rt_bvh.cpp): boxes are
 * padded by 1e-5 * max |coordinate|, so hits do not depend on the tree. */
#define OBINS 16
#define OMEDIAN_DEPTH 48   /* below this depth: object-median splits (bounds the traversal stack) */
typedef struct { float lo[3], hi[3]; uint32_t n; } OBin;

static void bin_grow(OBin* b, const float* w) {
    for (int q = 0; q < 3; ++q)
        for (int a = 0; a < 3; ++a) {
            b->lo[a] = fminf(b->lo[a], w[3 * q + a]);
            b->hi[a] = fmaxf(b->hi[a], w[3 * q + a]);
        }
}
static void bin_merge(OBin* d, const OBin* b) {
    for (int a = 0; a < 3; ++a) { d->lo[a] = fminf(d->lo[a], b->lo[a]); d->hi[a] = fmaxf(d->hi[a], b->hi[a]); }
    d->n += b->n;
}
static float bin_area(const OBin* b) {
    if (b->n == 0) return 0.0f;
    float dx = b->hi[0] - b->lo[0], dy = b->hi[1] - b->lo[1], dz = b->hi[2] - b->lo[2];
    return dx * dy + dy * dz + dz * dx;
}
static void bin_clear(OBin* b) {
    for (int a = 0; a < 3; ++a) { b->lo[a] = INFINITY; b->hi[a] = -INFINITY; }
    b->n = 0;
}

static int cmp_axis;
static const float* cmp_cen;
static int cmp_c(const void* a, const void* b) {
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    float cx = cmp_cen[3 * x + cmp_axis], cy = cmp_cen[3 * y + cmp_axis];
    if (cx < cy) return -1;
    if (cx > cy) return 1;
    return x < y ? -1 : (x > y);
}

static void build_bvh(rt_oracle_scene* s) {
    uint32_t n = s->ntri;
    float* cen = (float*)malloc(sizeof(float) * 3 * (n ? n : 1));
    float maxabs = 1.0f;
    for (uint32_t t = 0; t < n; ++t)
        for (int a = 0; a < 3; ++a) {
            float lo = fminf(fminf(s->world[9 * t + a], s->world[9 * t + 3 + a]), s->world[9 * t + 6 + a]);
            float hi = fmaxf(fmaxf(s->world[9 * t + a], s->world[9 * t + 3 + a]), s->world[9 * t + 6 + a]);
            cen[3 * t + a] = 0.5f * (lo + hi);
            maxabs = fmaxf(maxabs, fmaxf(fabsf(lo), fabsf(hi)));
        }
    s->pad = 1e-5f * maxabs;
    s->order = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    for (uint32_t t = 0; t < n; ++t) s->order[t] = t;
    uint32_t cap = 2 * (n ? n : 1) + 1;
    s->nodes = (ONode*)malloc(sizeof(ONode) * cap);
    s->nnodes = 1;
    /* work stack of (node, start, end, depth) */
    uint32_t* st = (uint32_t*)malloc(sizeof(uint32_t) * 4 * (64 + 2 * (n ? n : 1)));
    int sp = 0;
    st[0] = 0; st[1] = 0; st[2] = n; st[3] = 0; sp = 1;
    while (sp) {
        --sp;
        uint32_t ni = st[4 * sp], s0 = st[4 * sp + 1], e0 = st[4 * sp + 2], depth = st[4 * sp + 3];
        ONode* nd = &s->nodes[ni];
        OBin all;
        bin_clear(&all);
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t k = s0; k < e0; ++k) {
            uint32_t t = s->order[k];
            bin_grow(&all, &s->world[9 * (size_t)t]);
            for (int a = 0; a < 3; ++a) { clo[a] = fminf(clo[a], cen[3 * t + a]); chi[a] = fmaxf(chi[a], cen[3 * t + a]); }
        }
        for (int a = 0; a < 3; ++a) { nd->lo[a] = all.lo[a] - s->pad; nd->hi[a] = all.hi[a] + s->pad; }
        if (e0 - s0 <= 4) {
            nd->left = -1; nd->right = -1; nd->start = s0; nd->count = e0 - s0;
            continue;
        }
        /* best binned split over the three axes: cost = A(left) * n(left) + A(right) * n(right) */
        int best_axis = -1, best_b = 0;
        float best_cost = INFINITY;
        for (int a = 0; a < 3 && depth < OMEDIAN_DEPTH; ++a) {
            float ext = chi[a] - clo[a];
            if (!(ext > 0.0f)) continue;
            OBin bins[OBINS];
            for (int b = 0; b < OBINS; ++b) bin_clear(&bins[b]);
            float scale = (float)OBINS / ext;
            for (uint32_t k = s0; k < e0; ++k) {
                uint32_t t = s->order[k];
                int b = (int)((cen[3 * t + a] - clo[a]) * scale);
                if (b >= OBINS) b = OBINS - 1;
                if (b < 0) b = 0;
                bin_grow(&bins[b], &s->world[9 * (size_t)t]);
                bins[b].n++;
            }
            float right_cost[OBINS];
            OBin acc;
            bin_clear(&acc);
            for (int b = OBINS - 1; b > 0; --b) {
                bin_merge(&acc, &bins[b]);
                right_cost[b] = bin_area(&acc) * (float)acc.n;
            }
            bin_clear(&acc);
            for (int b = 1; b < OBINS; ++b) {   /* split before bin b */
                bin_merge(&acc, &bins[b - 1]);
                if (acc.n == 0 || acc.n == e0 - s0) continue;
                float c = bin_area(&acc) * (float)acc.n + right_cost[b];
                if (c < best_cost) { best_cost = c; best_axis = a; best_b = b; }
            }
        }
        uint32_t mid;
        if (best_axis >= 0) {   /* partition by bin index */
            int a = best_axis;
            float scale = (float)OBINS / (chi[a] - clo[a]);
            uint32_t i = s0, j = e0;
            while (i < j) {
                uint32_t t = s->order[i];
                int b = (int)((cen[3 * t + a] - clo[a]) * scale);
                if (b >= OBINS) b = OBINS - 1;
                if (b < best_b) { ++i; } else { --j; s->order[i] = s->order[j]; s->order[j] = t; }
            }
            mid = i;
        } else {                /* deep (or all centroids coincide): object median on the longest axis */
            int axis = 0;
            for (int a = 1; a < 3; ++a) if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
            cmp_axis = axis; cmp_cen = cen;
            qsort(s->order + s0, e0 - s0, sizeof(uint32_t), cmp_c);
            mid = s0 + (e0 - s0) / 2;
        }
        uint32_t l = s->nnodes++, r = s->nnodes++;
        nd = &s->nodes[ni];
        nd->left = (int32_t)l; nd->right = (int32_t)r; nd->start = 0; nd->count = 0;
        st[4 * sp] = r; st[4 * sp + 1] = mid; st[4 * sp + 2] = e0; st[4 * sp + 3] = depth + 1; ++sp;
        st[4 * sp] = l; st[4 * sp + 1] = s0; st[4 * sp + 2] = mid; st[4 * sp + 3] = depth + 1; ++sp;
    }
    free(st);
    free(cen);
}

int rt_oracle_scene_create(const rt_scene_desc* d, rt_oracle_scene** out) {
    if (!d || !out || d->mesh_count == 0) return 1;
    rt_oracle_scene* s = (rt_oracle_scene*)calloc(1, sizeof *s);
    s->nmesh = d->mesh_count;
    s->nlight = d->light_count;
    s->lights = (Light*)malloc(sizeof(Light) * (d->light_count ? d->light_count : 1));
    memcpy(s->lights, d->lights, sizeof(Light) * d->light_count);
    s->pos = (const rt_float3**)calloc(s->nmesh, sizeof(void*));
    s->nrm = (const rt_float3**)calloc(s->nmesh, sizeof(void*));
    s->prev_pos = (const rt_float3**)calloc(s->nmesh, sizeof(void*));
    s->xf = calloc(s->nmesh, sizeof(float[12]));
    s->prev_xf = calloc(s->nmesh, sizeof(float[12]));
    s->mats = (Material**)calloc(s->nmesh, sizeof(Material*));
    s->uv = (const rt_float2**)calloc(s->nmesh, sizeof(void*));
    s->mtex = calloc(s->nmesh, sizeof(*s->mtex));
    s->tex = d->textures;
    s->ntex = d->texture_count;
    for (int b = 0; b < 256; ++b) {   /* MTKTextureLoader .SRGB true / false (SubMesh.swift:80-97) */
        double v = b / 255.0;
        s->lut[b] = (float)v;
        s->lut[256 + b] = (float)(v <= 0.04045 ? v / 12.92 : pow((v + 0.055) / 1.055, 2.4));
    }
    uint32_t n = 0;
    for (uint32_t m = 0; m < s->nmesh; ++m)
        for (uint32_t k = 0; k < d->meshes[m].submesh_count; ++k) n += d->meshes[m].submeshes[k].index_count / 3;
    s->ntri = n;
    s->world = (float*)malloc(sizeof(float) * 9 * (n ? n : 1));
    s->tri = (OTri*)malloc(sizeof(OTri) * (n ? n : 1));
    uint32_t t = 0;
    for (uint32_t m = 0; m < s->nmesh; ++m) {
        const rt_mesh_desc* md = &d->meshes[m];
        s->pos[m] = md->positions;
        s->prev_pos[m] = md->positions;   /* previousPositions = positions (SubMesh.swift:60) */
        s->nrm[m] = md->normals;
        memcpy(s->xf[m], &md->transform, 48);
        memcpy(s->prev_xf[m], &md->transform, 48);
        s->mats[m] = (Material*)malloc(sizeof(Material) * md->submesh_count);
        s->uv[m] = md->uvs;
        s->mtex[m] = malloc(sizeof(int32_t[8]) * md->submesh_count);
        for (uint32_t k = 0; k < md->submesh_count; ++k) {
            const rt_submesh_desc* sm = &md->submeshes[k];
            s->mats[m][k] = sm->material;
            memcpy(s->mtex[m][k], sm->textures, sizeof(int32_t[8]));
            for (uint32_t q = 0; q < sm->index_count / 3; ++q) {
                OTri* ot = &s->tri[t];
                ot->mesh = m; ot->sub = k;
                ot->i0 = sm->indices[3 * q]; ot->i1 = sm->indices[3 * q + 1]; ot->i2 = sm->indices[3 * q + 2];
                uint32_t iv[3] = {ot->i0, ot->i1, ot->i2};
                for (int c = 0; c < 3; ++c) {
                    V3 w = oxform(s->xf[m], f3v(md->positions[iv[c]]), 1.0f);
                    s->world[9 * t + 3 * c + 0] = w.x;
                    s->world[9 * t + 3 * c + 1] = w.y;
                    s->world[9 * t + 3 * c + 2] = w.z;
                }
                ++t;
            }
        }
    }
    build_bvh(s);
    *out = s;
    return 0;
}

/* Previous-frame state of mesh m for motion vectors (Raytracing.metal:342-389): the positions
 * before the last skinning tick (Renderer.swift:1290-1303) and/or the previous instance
 * transform (Renderer.swift:939-944).  NULL keeps the current value. */
int rt_oracle_scene_set_previous(rt_oracle_scene* s, uint32_t m, const rt_float3* prev_positions,
                                 const float* prev_transform) {
    if (!s || m >= s->nmesh) return 1;
    if (prev_positions) s->prev_pos[m] = prev_positions;
    if (prev_transform) memcpy(s->prev_xf[m], prev_transform, 48);
    return 0;
}

void rt_oracle_scene_destroy(rt_oracle_scene* s) {
    if (!s) return;
    for (uint32_t m = 0; m < s->nmesh; ++m) { free(s->mats[m]); free(s->mtex[m]); }
    free(s->mats); free(s->mtex); free(s->uv); free(s->pos); free(s->nrm); free(s->prev_pos); free(s->xf); free(s->prev_xf);
    free(s->lights); free(s->world); free(s->tri); free(s->order); free(s->nodes);
    free(s);
}

uint32_t rt_oracle_scene_triangles(const rt_oracle_scene* s) { return s ? s->ntri : 0; }

/* ---------------------------------------------------------------- intersection */
/* Watertight ray/triangle test (Woop, Benthin, Wald 2013) standing in for the Metal
 * intersector<triangle_data, instancing> (Raytracing.metal:301-318): opaque, no culling,
 * t in [tmin, tmax]; u weights vertex 1, v weights vertex 2 (:63-73).  The axes are cycled
 * (kx = kz + 1, ky = kz + 2 mod 3) and never swapped: Woop et al. swap kx / ky when d[kz] < 0 to
 * keep the winding for back-face culling; without culling the swap negates U, V, W, det and T
 * together, which leaves t, u, v and every accept / reject decision unchanged up to the sign of
 * exact zeros. */
typedef struct { int kx, ky, kz; float Sx, Sy, Sz; } OPre;

static OPre opre(V3 d) {
    OPre p;
    float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    int kz = (ax > ay) ? ((ax > az) ? 0 : 2) : ((ay > az) ? 1 : 2);
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    float dz = vcomp(d, kz);
    p.kx = kx; p.ky = ky; p.kz = kz;
    p.Sx = vcomp(d, kx) / dz;
    p.Sy = vcomp(d, ky) / dz;
    p.Sz = 1.0f / dz;
    return p;
}

static int otri(const OPre* p, V3 o, const float* w, float tmin, float tmax, float* to, float* uo, float* vo) {
    V3 A = vsub(v3(w[0], w[1], w[2]), o), B = vsub(v3(w[3], w[4], w[5]), o), C = vsub(v3(w[6], w[7], w[8]), o);
    float Akz = vcomp(A, p->kz), Bkz = vcomp(B, p->kz), Ckz = vcomp(C, p->kz);
    float Ax = vcomp(A, p->kx) - p->Sx * Akz, Ay = vcomp(A, p->ky) - p->Sy * Akz;
    float Bx = vcomp(B, p->kx) - p->Sx * Bkz, By = vcomp(B, p->ky) - p->Sy * Bkz;
    float Cx = vcomp(C, p->kx) - p->Sx * Ckz, Cy = vcomp(C, p->ky) - p->Sy * Ckz;
    float U = Cx * By - Cy * Bx;
    float V = Ax * Cy - Ay * Cx;
    float W = Bx * Ay - By * Ax;
    if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return 0;
    float det = (U + V) + W;
    if (det == 0.0f) return 0;
    float Az = p->Sz * Akz, Bz = p->Sz * Bkz, Cz = p->Sz * Ckz;
    float T = (U * Az + V * Bz) + W * Cz;
    float t = T / det;
    if (!(t >= tmin && t <= tmax)) return 0;
    *to = t; *uo = V / det; *vo = W / det;
    return 1;
}

static float safe_inv(float x) { return 1.0f / (fabsf(x) < 1e-30f ? copysignf(1e-30f, x) : x); }

/* slab test; returns the entry distance, or -1 on a miss */
static float obox(const ONode* n, V3 o, V3 inv, float tmin, float tmax) {
    float tx0 = (n->lo[0] - o.x) * inv.x, tx1 = (n->hi[0] - o.x) * inv.x;
    float ty0 = (n->lo[1] - o.y) * inv.y, ty1 = (n->hi[1] - o.y) * inv.y;
    float tz0 = (n->lo[2] - o.z) * inv.z, tz1 = (n->hi[2] - o.z) * inv.z;
    float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin));
    float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax * 1.000001f));
    return tn <= tf ? tn : -1.0f;
}

/* closest hit over the whole BVH (nearer child first); ties broken by the smaller original
 * triangle id, so the result does not depend on the visiting order */
static int otrace(const rt_oracle_scene* s, V3 o, V3 d, float tmin, float tmax, int any,
                  float* to, uint32_t* ido, float* uo, float* vo) {
    if (s->ntri == 0) return 0;
    OPre p = opre(d);
    V3 inv = v3(safe_inv(d.x), safe_inv(d.y), safe_inv(d.z));
    float best = tmax, bu = 0, bv = 0;
    uint32_t bid = 0xffffffffu;
    /* (node, entry distance) pairs; a popped node whose entry lies beyond the closest hit so far
     * is skipped (the same margin as the slab test) */
    uint32_t stack[256];
    float tent[256];
    int sp = 0;
    float t0 = obox(&s->nodes[0], o, inv, tmin, best);
    if (t0 < 0.0f) return 0;
    stack[sp] = 0; tent[sp++] = t0;
    while (sp) {
        --sp;
        if (tent[sp] > best * 1.000001f) continue;
        const ONode* n = &s->nodes[stack[sp]];
        if (n->left < 0) {
            for (uint32_t k = 0; k < n->count; ++k) {
                uint32_t t = s->order[n->start + k];
                float tt, uu, vv;
                if (otri(&p, o, &s->world[9 * (size_t)t], tmin, best, &tt, &uu, &vv)) {
                    if (any) { *to = tt; *ido = t; *uo = uu; *vo = vv; return 1; }
                    if (tt < best || t < bid) { best = tt; bid = t; bu = uu; bv = vv; }
                }
            }
        } else {
            float tl = obox(&s->nodes[n->left], o, inv, tmin, best);
            float tr = obox(&s->nodes[n->right], o, inv, tmin, best);
            if (tl >= 0.0f && tr >= 0.0f) {
                int near_left = tl <= tr;
                stack[sp] = (uint32_t)(near_left ? n->right : n->left); tent[sp++] = near_left ? tr : tl;
                stack[sp] = (uint32_t)(near_left ? n->left : n->right); tent[sp++] = near_left ? tl : tr;
            } else if (tl >= 0.0f) {
                stack[sp] = (uint32_t)n->left; tent[sp++] = tl;
            } else if (tr >= 0.0f) {
                stack[sp] = (uint32_t)n->right; tent[sp++] = tr;
            }
        }
    }
    if (bid == 0xffffffffu) return 0;
    *to = best; *ido = bid; *uo = bu; *vo = bv;
    return 1;
}

int rt_oracle_intersect(const rt_oracle_scene* s, const float o[3], const float d[3], float tmin, float tmax, int any,
                        float* t, uint32_t* id, float* u, float* v) {
    return otrace(s, v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), tmin, tmax, any, t, id, u, v);
}

int rt_oracle_intersect_bruteforce(const rt_oracle_scene* s, const float o[3], const float d[3], float tmin,
                                   float tmax, int any, float* t, uint32_t* id, float* u, float* v) {
    V3 O = v3(o[0], o[1], o[2]), D = v3(d[0], d[1], d[2]);
    OPre p = opre(D);
    float best = tmax, bu = 0, bv = 0;
    uint32_t bid = 0xffffffffu;
    for (uint32_t k = 0; k < s->ntri; ++k) {
        float tt, uu, vv;
        if (otri(&p, O, &s->world[9 * (size_t)k], tmin, best, &tt, &uu, &vv)) {
            if (any) { *t = tt; *id = k; *u = uu; *v = vv; return 1; }
            if (tt < best || k < bid) { best = tt; bid = k; bu = uu; bv = vv; }
        }
    }
    if (bid == 0xffffffffu) return 0;
    *t = best; *id = bid; *u = bu; *v = bv;
    return 1;
}

/* ---------------------------------------------------------------- sampling helpers */
/* :79-89 */
static V3 cosine_hemisphere(float ux, float uy) {
    float phi = 2.0f * ORC_PI * ux;
    float sin_phi, cos_phi;
    rt_oracle_sincos(phi, &sin_phi, &cos_phi);
    float cos_theta = sqrtf(uy);
    float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
    return v3(sin_theta * cos_phi, cos_theta, sin_theta * sin_phi);
}
/* :133-148 */
static V3 align_hemisphere(V3 smp, V3 normal) {
    V3 up = normal;
    V3 right = vnorm(vcross(normal, v3(0.0072f, 1.0f, 0.0034f)));
    V3 forward = vcross(right, up);
    return vadd(vadd(vscl(right, smp.x), vscl(up, smp.y)), vscl(forward, smp.z));
}
/* :150-166 */
static float ggx_d(float NdotH, float alpha) {
    float a2 = alpha * alpha;
    float denom = (NdotH * NdotH) * (a2 - 1.0f) + 1.0f;
    return a2 / fmaxf(ORC_PI * denom * denom, 1e-7f);
}
static float schlick_g(float NdotV, float k) { return NdotV / fmaxf(NdotV * (1.0f - k) + k, 1e-7f); }
static float smith_g(float NdotV, float NdotL, float k) { return schlick_g(NdotV, k) * schlick_g(NdotL, k); }
static V3 fresnel(float cosTheta, V3 F0) {
    float p = rt_oracle_pow5(clampf_(1.0f - cosTheta, 0.0f, 1.0f));
    return v3(F0.x + (1.0f - F0.x) * p, F0.y + (1.0f - F0.y) * p, F0.z + (1.0f - F0.z) * p);
}
/* interpolateVertexAttribute :61-74: u*A[i1] + v*A[i2] + w*A[i0] */
static V3 interp(const rt_float3* A, const OTri* t, float u, float v, float w) {
    return vadd(vadd(vscl(f3v(A[t->i1]), u), vscl(f3v(A[t->i2]), v)), vscl(f3v(A[t->i0]), w));
}

/* ---------------------------------------------------------------- textures */
typedef struct { float x, y, z, w; } V4;

/* sample(sampler(linear, linear, mip linear, repeat), uv) in a compute kernel = bilinear from
 * LOD 0 (Raytracing.metal:420): texel centres at i + 0.5, wrapped neighbours, corners decoded
 * through the byte table (sRGB for base color / emission, alpha linear), weights in this order. */
static V4 osample(const rt_oracle_scene* s, int t, float u, float v, int srgb) {
    const rt_texture_desc* T = &s->tex[t];
    int w = (int)T->width, h = (int)T->height;
    float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    if (!(fabsf(x) < 1.0e9f)) x = 0.0f;
    if (!(fabsf(y) < 1.0e9f)) y = 0.0f;
    float fx = floorf(x), fy = floorf(y);
    float ax = x - fx, ay = y - fy, bx = 1.0f - ax, by = 1.0f - ay;
    long long ix = (long long)fx % w, iy = (long long)fy % h;
    if (ix < 0) ix += w;
    if (iy < 0) iy += h;
    int x0 = (int)ix, y0 = (int)iy, x1 = x0 + 1 == w ? 0 : x0 + 1, y1 = y0 + 1 == h ? 0 : y0 + 1;
    const uint8_t* c00 = T->rgba8 + 4 * ((size_t)y0 * w + x0);
    const uint8_t* c10 = T->rgba8 + 4 * ((size_t)y0 * w + x1);
    const uint8_t* c01 = T->rgba8 + 4 * ((size_t)y1 * w + x0);
    const uint8_t* c11 = T->rgba8 + 4 * ((size_t)y1 * w + x1);
    float r[4];
    for (int c = 0; c < 4; ++c) {
        const float* L = s->lut + ((srgb && c < 3) ? 256 : 0);
        r[c] = (L[c00[c]] * bx + L[c10[c]] * ax) * by + (L[c01[c]] * bx + L[c11[c]] * ax) * ay;
    }
    V4 o = {r[0], r[1], r[2], r[3]};
    return o;
}

int rt_oracle_tex_sample(const rt_oracle_scene* s, int32_t t, float u, float v, int32_t srgb, float out[4]) {
    if (!s || t < 0 || (uint32_t)t >= s->ntex || !out) return 1;
    V4 r = osample(s, t, u, v, srgb);
    out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
    return 0;
}

static void ouv(const rt_oracle_scene* s, int m, uint32_t i, float* u, float* v) {
    if (s->uv[m]) { *u = s->uv[m][i].x; *v = s->uv[m][i].y; }
    else { *u = 0.0f; *v = 0.0f; }
}

/* computeTangentBasis (Raytracing.metal:185-218) */
static int tangent_basis(const rt_oracle_scene* s, const OTri* t, V3* tangent, V3* bitangent) {
    const rt_float3* P = s->pos[t->mesh];
    V3 p0 = f3v(P[t->i1]), p1 = f3v(P[t->i2]), p2 = f3v(P[t->i0]);
    float u0, v0, u1, v1, u2, v2;
    ouv(s, (int)t->mesh, t->i1, &u0, &v0);
    ouv(s, (int)t->mesh, t->i2, &u1, &v1);
    ouv(s, (int)t->mesh, t->i0, &u2, &v2);
    V3 e1 = vsub(p1, p0), e2 = vsub(p2, p0);
    float d1x = u1 - u0, d1y = v1 - v0, d2x = u2 - u0, d2y = v2 - v0;
    float denom = d1x * d2y - d1y * d2x;
    if (fabsf(denom) < 1e-8f) return 0;
    float r = 1.0f / denom;
    *tangent = vscl(vsub(vscl(e1, d2y), vscl(e2, d1y)), r);
    *bitangent = vscl(vsub(vscl(e2, d1x), vscl(e1, d2x)), r);
    return vlen(*tangent) > 1e-8f && vlen(*bitangent) > 1e-8f;
}

/* ---------------------------------------------------------------- the kernel */
typedef struct {
    const rt_oracle_scene* s;
    rt_oracle_frame* f;
    int* next_row;         /* shared: index of the next row of the subset to render */
    uint64_t closest, shadow, paths;
} Job;

static void render_pixel(const rt_oracle_scene* s, rt_oracle_frame* f, int px, int py, uint64_t* nc, uint64_t* ns,
                         uint64_t* np) {
    const Uniforms* U = f->uniforms;
    size_t pix = (size_t)py * U->width + px;
    unsigned int offset = f->random[pix];                                         /* :245 */
    V3 totalColor = v3(0, 0, 0);
    float pmx = f->motion[2 * pix], pmy = f->motion[2 * pix + 1];                /* :248 */
    float primaryDepth = 1.0e8f;
    float mvx = 0.0f, mvy = 0.0f;
    int hadPrimaryHit = 0;
    float gb[4][4] = {{0}};
    int wroteG = 0;
    int baseSamples = U->samplesPerPixel > 1 ? U->samplesPerPixel : 1;           /* :263-266 */
    int maxExtra = (U->enableMotionAdaptiveSampling != 0) ? (U->motionSamplingMaxExtraSamples > 0 ? U->motionSamplingMaxExtraSamples : 0) : 0;
    int sampleStride = baseSamples + maxExtra;
    int totalSamples = baseSamples;
    V3 cright = f3v(U->camera.right), cup = f3v(U->camera.up), cfwd = f3v(U->camera.forward), cpos = f3v(U->camera.position);

    for (int sampleIndex = 0; sampleIndex < totalSamples; sampleIndex++) {       /* :269 */
        (*np)++;
        int frameOffset = (int)(U->frameIndex * (unsigned)sampleStride + (unsigned)sampleIndex);
        int hi = (int)(offset + (unsigned)frameOffset);
        float rx = rt_oracle_halton(hi, 0), ry = rt_oracle_halton(hi, 1);       /* :273-274 */
        float spx = (float)px + rx, spy = (float)py + ry;
        float uvx = spx / (float)U->width, uvy = spy / (float)U->height;        /* :278-279 */
        uvx = uvx * 2.0f - 1.0f; uvy = uvy * 2.0f - 1.0f;
        V3 ro = cpos;                                                           /* :285 */
        V3 rd = vnorm(vadd(vadd(vscl(cright, uvx), vscl(cup, uvy)), cfwd));     /* :287-289 */
        V3 color = v3(1, 1, 1), acc = v3(0, 0, 0);
        int bounce = 0, step = 0, tpass = 0;
        while (bounce < U->maxBounces) {                                        /* :311 */
            float t, bu, bv;
            uint32_t id;
            (*nc)++;
            if (!otrace(s, ro, rd, 0.0f, INFINITY, 0, &t, &id, &bu, &bv)) break;  /* :318-322 */
            const OTri* tr = &s->tri[id];
            int inst = (int)tr->mesh;
            const float* M = s->xf[inst];
            V3 P = vadd(ro, vscl(rd, t));                                       /* :336 */
            const Material* mat = &s->mats[inst][tr->sub];                      /* :337-339 */
            float bw = (1.0f - bu) - bv;                                        /* :65 */

            if (bounce == 0 && sampleIndex == 0) {                              /* :342-389 */
                V3 op = interp(s->pos[inst], tr, bu, bv, bw);
                V3 pp = interp(s->prev_pos[inst], tr, bu, bv, bw);
                V3 worldPos = oxform(M, op, 1.0f);
                V3 prevWorldPos = oxform(s->prev_xf[inst], pp, 1.0f);
                V3 viewPos = vsub(worldPos, cpos);
                float sx = vdot(viewPos, cright), sy = vdot(viewPos, cup);
                float depth = vdot(viewPos, cfwd);
                primaryDepth = fmaxf(depth, 1.0e-3f);
                float dd = fmaxf(depth, 0.001f);
                sx = sx / dd; sy = sy / dd;
                const Camera* pc = &U->previousCamera;
                V3 pv = vsub(prevWorldPos, f3v(pc->position));
                float psx = vdot(pv, f3v(pc->right)), psy = vdot(pv, f3v(pc->up));
                float pd = fmaxf(vdot(pv, f3v(pc->forward)), 0.001f);
                psx = psx / pd; psy = psy / pd;
                float mnx = sx - psx, mny = sy - psy;
                float rs = fmaxf(vlen(cright), 1e-5f), us = fmaxf(vlen(cup), 1e-5f);
                float mpx = mnx * ((float)U->width / (2.0f * rs));
                float mpy = mny * ((float)U->height / (2.0f * us));
                mvx = mpx; mvy = -mpy;
                hadPrimaryHit = 1;
            }

            V3 objN = interp(s->nrm[inst], tr, bu, bv, bw);                     /* :391 */
            V3 Ng = vnorm(oxform(M, objN, 0.0f));                               /* :392-393 */
            if (vlen(objN) < 1e-10f) Ng = vneg(rd);                             /* :395-397 */
            V3 albedo = f3v(mat->baseColor);                                    /* :399 */
            float roughness = 1.0f, metallic = 0.0f, ao = 1.0f;                 /* :431-446 (ENABLE_AO 0) */
            float opacity = clampf_(mat->opacity, 0.0f, 1.0f);                  /* :448 */
            V3 emission = f3v(mat->emission);                                   /* :453 */
            const int32_t* tx = s->mtex[inst][tr->sub];
            unsigned tfl = mat->textureFlags & ~(unsigned)MATERIAL_TEXTURE_AO;
            float tcu = 0.0f, tcv = 0.0f;
            V4 bsm = {1.0f, 1.0f, 1.0f, 1.0f};
            if (tfl) {                                                          /* :412-417 */
                float ua, va, ub, vb, uc, vc;
                ouv(s, inst, tr->i1, &ua, &va);
                ouv(s, inst, tr->i2, &ub, &vb);
                ouv(s, inst, tr->i0, &uc, &vc);
                tcu = (bu * ua + bv * ub) + bw * uc;
                tcv = (bu * va + bv * vb) + bw * vc;
                tcv = 1.0f - tcv;
            }
            if (tfl & MATERIAL_TEXTURE_BASECOLOR) {                             /* :423-428 */
                bsm = osample(s, tx[0], tcu, tcv, 1);
                albedo = vmul(albedo, v3(bsm.x, bsm.y, bsm.z));
            }
            if (tfl & MATERIAL_TEXTURE_ROUGHNESS) roughness = osample(s, tx[2], tcu, tcv, 0).x;  /* :431-434 */
            if (tfl & MATERIAL_TEXTURE_METALLIC) metallic = osample(s, tx[3], tcu, tcv, 0).x;    /* :436-439 */
            if (tfl & MATERIAL_TEXTURE_OPACITY) opacity = opacity * osample(s, tx[6], tcu, tcv, 0).x;  /* :448-451 */
            if (tfl & MATERIAL_TEXTURE_EMISSION) {                              /* :453-456 */
                V4 e = osample(s, tx[5], tcu, tcv, 1);
                emission = v3(e.x, e.y, e.z);
            }

            if (U->debugTextureMode != DebugTextureModeNone) {                  /* :459-490 */
                V3 dc = v3(0, 0, 0);
                int m = U->debugTextureMode;
                if (m == DebugTextureModeBaseColor)
                    dc = (tfl & MATERIAL_TEXTURE_BASECOLOR) ? v3(bsm.x, bsm.y, bsm.z) : v3(1.0f, 0.0f, 1.0f);
                else if (m == DebugTextureModeNormal) {
                    if (tfl & MATERIAL_TEXTURE_NORMAL) {
                        V4 nm = osample(s, tx[1], tcu, tcv, 0);
                        dc = v3(nm.x, nm.y, nm.z);
                    } else {
                        dc = vadd(vscl(Ng, 0.5f), v3(0.5f, 0.5f, 0.5f));
                    }
                }
                else if (m == DebugTextureModeRoughness) dc = v3(roughness, roughness, roughness);
                else if (m == DebugTextureModeMetallic) dc = v3(metallic, metallic, metallic);
                else if (m == DebugTextureModeAO) dc = v3(1.0f, 0.0f, 1.0f);
                else if (m == DebugTextureModeEmission) dc = emission;
                else if (m == DebugTextureModeMotion) {
                    float mx = hadPrimaryHit ? mvx : pmx, my = hadPrimaryHit ? mvy : pmy;
                    float scx = clampf_(mx * 0.05f, -1.0f, 1.0f), scy = clampf_(my * 0.05f, -1.0f, 1.0f);
                    float mag = clampf_(sqrtf(mx * mx + my * my) * 0.1f, 0.0f, 1.0f);
                    dc = v3(scx * 0.5f + 0.5f, scy * 0.5f + 0.5f, mag);
                }
                acc = dc;
                break;
            }
            V3 sn = Ng;                                                         /* :492 */
            if (tfl & MATERIAL_TEXTURE_NORMAL) {                                /* :493-504 */
                V3 T, B;
                if (tangent_basis(s, tr, &T, &B)) {
                    V3 wT = oxform(M, T, 0.0f);
                    wT = vnorm(vsub(wT, vscl(Ng, vdot(wT, Ng))));
                    V3 wB = vnorm(vcross(Ng, wT));
                    V4 nm = osample(s, tx[1], tcu, tcv, 0);
                    V3 n = v3(nm.x * 2.0f - 1.0f, nm.y * 2.0f - 1.0f, nm.z * 2.0f - 1.0f);
                    sn = vnorm(vadd(vadd(vscl(wT, n.x), vscl(wB, n.y)), vscl(Ng, n.z)));
                }
            }
            if (U->enableDenoiseGBuffer != 0 && !wroteG && sampleIndex == 0) {  /* :506-515 */
                V3 da = vscl(albedo, 1.0f - metallic);
                V3 sa = vmix(v3(0.04f, 0.04f, 0.04f), albedo, metallic);
                V3 on = vadd(vscl(sn, 0.5f), v3(0.5f, 0.5f, 0.5f));
                float g[4][4] = {{da.x, da.y, da.z, 1.0f}, {sa.x, sa.y, sa.z, 1.0f}, {on.x, on.y, on.z, 1.0f},
                                 {clampf_(roughness, 0.0f, 1.0f), 0.0f, 0.0f, 1.0f}};
                memcpy(gb, g, sizeof g);
                wroteG = 1;
            }
            float cop = clampf_(opacity, 0.0f, 1.0f);                           /* :517-576 */
            float ior = fmaxf(mat->refractionIndex, 1.0f);
            if (cop < 0.999f || ior > 1.01f) {
                V3 N = sn, I = rd;
                float cosi = clampf_(vdot(vneg(I), N), -1.0f, 1.0f);
                float etaI = 1.0f, etaT = ior;
                if (cosi < 0.0f) { cosi = -cosi; N = vneg(N); float tmp = etaI; etaI = etaT; etaT = tmp; }
                float eta = etaI / etaT;
                float k = 1.0f - (eta * eta) * (1.0f - cosi * cosi);
                float f0 = (etaT - etaI) / (etaT + etaI);
                f0 = f0 * f0;
                float F = f0 + (1.0f - f0) * rt_oracle_pow5(clampf_(1.0f - cosi, 0.0f, 1.0f));
                float transmission = 1.0f - cop;
                float rw = F, tw = (1.0f - F) * transmission;
                float totalWeight = fmaxf(rw + tw, 1e-4f);
                float reflectProb = rw / totalWeight;
                float choice = rt_oracle_halton(hi, 2 + step * 6 + 5);
                int consume = 1;
                if (k < 0.0f || choice < reflectProb) {
                    V3 R = vnorm(vsub(I, vscl(N, 2.0f * vdot(I, N))));
                    ro = vadd(P, vscl(R, 1e-3f)); rd = R;
                    color = vscl(color, totalWeight);
                } else {
                    float cosT = sqrtf(fmaxf(k, 0.0f));
                    V3 T = vnorm(vadd(vscl(I, eta), vscl(N, eta * cosi - cosT)));
                    ro = vadd(P, vscl(T, 1e-3f)); rd = T;
                    color = vmul(color, vscl(albedo, totalWeight));
                    consume = 0;
                }
                step++;
                if (consume) { bounce++; tpass = 0; }
                else { tpass++; if (tpass > U->maxBounces) { bounce++; tpass = 0; } }
                continue;
            }
            float pr = clampf_(roughness, 0.04f, 1.0f);                         /* :578-582 */
            float alpha = pr * pr;
            V3 diffuseColor = albedo;
            V3 F0 = vmix(v3(0.04f, 0.04f, 0.04f), albedo, metallic);
            V3 V = vnorm(vneg(rd));
            acc = vadd(acc, vmul(color, emission));                             /* :585 */
            float ls = rt_oracle_halton(hi, 2 + step * 6 + 0);                  /* :588-589 */
            int li = (int)(ls * (float)U->lightCount);
            if (li > U->lightCount - 1) li = U->lightCount - 1;
            const Light* L = &s->lights[li];
            V3 Ld, lc;
            float ldist;
            if (L->type == LightTypeAreaLight) {                                /* :597-606, :95-129 */
                float ux = rt_oracle_halton(hi, 2 + step * 6 + 1), uy = rt_oracle_halton(hi, 2 + step * 6 + 2);
                ux = ux * 2.0f - 1.0f; uy = uy * 2.0f - 1.0f;
                V3 sp = vadd(vadd(f3v(L->position), vscl(f3v(L->right), ux)), vscl(f3v(L->up), uy));
                Ld = vsub(sp, P);
                ldist = vlen(Ld);
                float inv = 1.0f / fmaxf(ldist, 1e-3f);
                Ld = vscl(Ld, inv);
                lc = vscl(f3v(L->color), inv * inv);
                lc = vscl(lc, satf(vdot(vneg(Ld), f3v(L->forward))));
            } else if (L->type == LightTypeSpotlight) {                         /* :608-632 */
                Ld = vsub(f3v(L->position), P);
                ldist = vlen(Ld);
                float inv = 1.0f / fmaxf(ldist, 1e-3f);
                Ld = vscl(Ld, inv);
                lc = v3(0, 0, 0);
                V3 cd = vnorm(f3v(L->direction));
                float sr = vdot(vneg(Ld), cd);
                float sc, cc;
                rt_oracle_sincos(L->coneAngle, &sc, &cc);
                if (sr > cc) lc = vscl(vscl(f3v(L->color), inv), inv);
            } else if (L->type == LightTypePointlight) {                        /* :633-638 */
                Ld = vsub(f3v(L->position), P);
                ldist = vlen(Ld);
                float inv = 1.0f / fmaxf(ldist, 1e-3f);
                Ld = vscl(Ld, inv);
                lc = vscl(vscl(f3v(L->color), inv), inv);
            } else {                                                            /* :639-643 */
                Ld = vneg(vnorm(f3v(L->direction)));
                ldist = INFINITY;
                lc = f3v(L->color);
            }
            lc = vscl(lc, (float)U->lightCount);                                /* :647 */
            V3 so = vadd(P, vscl(Ng, 1e-3f));                                   /* :660, :720 */
            if (U->shadingMode == ShadingModeLegacy) {                          /* :649-690 */
                V3 Ln = vnorm(Ld);
                float NdotL = satf(vdot(sn, Ln));
                V3 lcol = vmul(color, albedo);
                if (vlen(lcol) < 0.001f) break;
                if (vlen(lc) > 0.0001f && NdotL > 0.0f) {
                    float tt, uu, vv; uint32_t ii;
                    (*ns)++;
                    if (!otrace(s, so, Ld, 0.0f, ldist - 1e-3f, 1, &tt, &ii, &uu, &vv))
                        acc = vadd(acc, vscl(vmul(lcol, lc), NdotL));
                }
                color = vscl(lcol, ao);
                if (vlen(color) < 0.001f) break;
                float r0 = rt_oracle_halton(hi, 2 + step * 5 + 3), r1 = rt_oracle_halton(hi, 2 + step * 5 + 4);
                V3 dir = align_hemisphere(cosine_hemisphere(r0, r1), sn);
                ro = so; rd = dir;
                step++; bounce++; tpass = 0;
                continue;
            }
            if (vlen(lc) > 0.0001f) {                                           /* :692-744 */
                V3 Ln = vnorm(Ld);
                V3 H = vnorm(vadd(V, Ln));
                float NdotL = satf(vdot(sn, Ln)), NdotV = satf(vdot(sn, V));
                float NdotH = satf(vdot(sn, H)), VdotH = satf(vdot(V, H));
                V3 F = fresnel(VdotH, F0);
                float D = ggx_d(NdotH, alpha);
                float kk = pr + 1.0f;
                kk = (kk * kk) / 8.0f;
                float G = smith_g(NdotV, NdotL, kk);
                V3 spec = vdivs(vscl(F, D * G), fmaxf((4.0f * NdotV) * NdotL, 1e-4f));
                V3 kD = vscl(vsub(v3(1, 1, 1), F), 1.0f - metallic);
                V3 diffuse = vdivs(vmul(kD, diffuseColor), ORC_PI);
                V3 direct = vscl(vmul(vadd(diffuse, spec), lc), NdotL);
                float tt, uu, vv; uint32_t ii;
                (*ns)++;
                if (!otrace(s, so, Ld, 0.0f, ldist - 1e-3f, 1, &tt, &ii, &uu, &vv))
                    acc = vadd(acc, vmul(color, direct));
            }
            color = vmul(color, vscl(vscl(diffuseColor, 1.0f - metallic), ao)); /* :748 */
            if (vlen(color) < 0.001f) break;                                    /* :751-753 */
            float r0 = rt_oracle_halton(hi, 2 + step * 5 + 3), r1 = rt_oracle_halton(hi, 2 + step * 5 + 4);
            V3 dir = align_hemisphere(cosine_hemisphere(r0, r1), sn);           /* :763-767 */
            ro = so; rd = dir;                                                  /* :769-770 */
            step++; bounce++; tpass = 0;
        }
        totalColor = vadd(totalColor, acc);                                     /* :777 */
        if (sampleIndex == 0 && maxExtra > 0) {                                 /* :779-789 */
            float mag = fmaxf(sqrtf(mvx * mvx + mvy * mvy), sqrtf(pmx * pmx + pmy * pmy));
            float low = fmaxf(U->motionSamplingLowThresholdPixels, 0.0f);
            float high = fmaxf(U->motionSamplingHighThresholdPixels, low + 1e-3f);
            float tt = clampf_((mag - low) / (high - low), 0.0f, 1.0f);
            int extra = (int)roundf(tt * (float)maxExtra);
            if (extra < 0) extra = 0;
            if (extra > maxExtra) extra = maxExtra;
            totalSamples = baseSamples + extra;
        }
    }
    totalColor = vdivs(totalColor, (float)(totalSamples > 1 ? totalSamples : 1)); /* :793 */
    if (U->frameIndex > 0) {                                                    /* :796-817 */
        V3 prev = f->accum_in ? v3(f->accum_in[4 * pix], f->accum_in[4 * pix + 1], f->accum_in[4 * pix + 2]) : v3(0, 0, 0);
        float hw = clampf_(U->accumulationWeight, 0.0f, 0.95f);
        if (U->enableMotionAdaptiveAccumulation != 0) {
            float mag = fmaxf(sqrtf(mvx * mvx + mvy * mvy), sqrtf(pmx * pmx + pmy * pmy));
            float low = fmaxf(U->motionAccumulationLowThresholdPixels, 0.0f);
            float high = fmaxf(U->motionAccumulationHighThresholdPixels, low + 1e-3f);
            float tt = clampf_((mag - low) / (high - low), 0.0f, 1.0f);
            float mw = clampf_(U->motionAccumulationMinWeight, 0.0f, 0.95f);
            mw = fminf(mw, hw);
            hw = mixf_(hw, mw, tt);
        }
        totalColor = vmix(totalColor, prev, hw);
    }
    f->accum_out[4 * pix] = totalColor.x;                                       /* :819 */
    f->accum_out[4 * pix + 1] = totalColor.y;
    f->accum_out[4 * pix + 2] = totalColor.z;
    f->accum_out[4 * pix + 3] = 1.0f;
    f->depth[pix] = primaryDepth;                                               /* :822 */
    f->motion[2 * pix] = mvx;                                                   /* :823 */
    f->motion[2 * pix + 1] = mvy;
    if (U->enableDenoiseGBuffer != 0 && f->gbuffer) {                           /* :824-829 */
        size_t plane = (size_t)U->width * U->height;
        for (int g = 0; g < 4; ++g) memcpy(&f->gbuffer[4 * (g * plane + pix)], gb[g], 16);
    }
}

static void* worker(void* arg) {
    Job* j = (Job*)arg;
    const rt_oracle_frame* f = j->f;
    const Uniforms* U = f->uniforms;
    const int step = f->row_step > 0 ? f->row_step : 1;
    const int T = f->tile_size > 0 ? f->tile_size : 64;
    const int split = f->nranks > 1;
    const int tiles_x = (U->width + T - 1) / T;
    for (;;) {   /* rows handed out one at a time: balanced whatever the per-row cost */
        int k = __atomic_fetch_add(j->next_row, 1, __ATOMIC_RELAXED);
        int y = f->row_start + k * step;
        if (y >= U->height) break;
        for (int x = 0; x < U->width; ++x) {
            if (split && ((y / T) * tiles_x + x / T) % f->nranks != f->rank) continue;
            render_pixel(j->s, j->f, x, y, &j->closest, &j->shadow, &j->paths);
        }
    }
    return NULL;
}

int rt_oracle_render(const rt_oracle_scene* s, rt_oracle_frame* f) {
    if (!s || !f || !f->uniforms || !f->random || !f->accum_out || !f->depth || !f->motion) return 1;
    const Uniforms* U = f->uniforms;
    if (U->lightCount < 1 || U->lightCount > (int)s->nlight || U->maxBounces > 12) return 2;
    if (f->nranks > 1 && (f->rank < 0 || f->rank >= f->nranks)) return 3;
    pthread_once(&g_primes_once, init_primes);
    int nt = f->threads > 0 ? f->threads : 1;
    int next_row = 0;
    Job* jobs = (Job*)calloc(nt, sizeof(Job));
    pthread_t* th = (pthread_t*)calloc(nt, sizeof(pthread_t));
    for (int i = 0; i < nt; ++i) {
        jobs[i].s = s; jobs[i].f = f; jobs[i].next_row = &next_row;
        if (nt > 1) pthread_create(&th[i], NULL, worker, &jobs[i]);
    }
    if (nt == 1) worker(&jobs[0]);
    f->closest_rays = f->shadow_rays = f->paths = 0;
    for (int i = 0; i < nt; ++i) {
        if (nt > 1) pthread_join(th[i], NULL);
        f->closest_rays += jobs[i].closest; f->shadow_rays += jobs[i].shadow; f->paths += jobs[i].paths;
    }
    free(jobs); free(th);
    return 0;
}

/* ---------------------------------------------------------------- skinning (Skinning.metal:7-49) */
static void m4v(const float* m, float x, float y, float z, float w, float* r) {
    for (int i = 0; i < 4; ++i) r[i] = ((m[0 + i] * x + m[4 + i] * y) + m[8 + i] * z) + m[12 + i] * w;
}
void rt_oracle_skin(const rt_float3* rp, const rt_float3* rn, const uint16_t* ji, const float* jw, const float* J,
                    rt_float3* op, rt_float3* on, uint32_t n) {
    for (uint32_t v = 0; v < n; ++v) {
        float w[4] = {jw[4 * v], jw[4 * v + 1], jw[4 * v + 2], jw[4 * v + 3]};
        float ws = ((w[0] + w[1]) + w[2]) + w[3];
        if (ws < 0.0001f) { w[0] = 1.0f; w[1] = w[2] = w[3] = 0.0f; }
        float sp[4] = {0, 0, 0, 0}, sn[3] = {0, 0, 0}, a[4];
        for (int k = 0; k < 4; ++k) {
            m4v(J + 16 * ji[4 * v + k], rp[v].x, rp[v].y, rp[v].z, 1.0f, a);
            for (int c = 0; c < 4; ++c) sp[c] = sp[c] + w[k] * a[c];
        }
        for (int k = 0; k < 4; ++k) {
            m4v(J + 16 * ji[4 * v + k], rn[v].x, rn[v].y, rn[v].z, 0.0f, a);
            for (int c = 0; c < 3; ++c) sn[c] = sn[c] + w[k] * a[c];
        }
        op[v].x = sp[0]; op[v].y = sp[1]; op[v].z = sp[2]; op[v]._pad = 0.0f;
        on[v].x = sn[0]; on[v].y = sn[1]; on[v].z = sn[2]; on[v]._pad = 0.0f;
    }
}
