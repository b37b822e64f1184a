// sim_trav.cpp — host-side SIMD-efficiency model of the wf_trace traversal schedule (tool, not product).
//
// Builds the C3g scene's 8-wide BVH with the product's host builder, makes extend rays (primary
// rays of a pixel grid, then one diffuse bounce from their hits), and replays the per-lane
// traversal of trav_step (rt_wavefront.hip) wave by wave (64 lanes, per-lane refill from a ray
// stream).  A wave iteration costs the VALU issues of every code block that at least one lane
// executes (block costs from the gfx950 ISA of wf_trace<false,false>); the model reports
// issues per ray and iterations per ray for several schedules, to rank them before a GPU A/B.
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off -Iinclude tools/sim_trav.cpp \
//     -Lmetal4-raytracing_amd -lrt_hip -Wl,-rpath,$PWD/metal4-raytracing_amd -o /tmp/sim_trav
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>
#include <random>
#include <algorithm>
#include "../metal4-raytracing_amd/csrc/rt_device.h"
#include "../include/rt_scene.h"
#include "../include/rt_api.h"

using namespace rt;
static f3 ldf3(const rt_float3& v) { return mk3(v.x, v.y, v.z); }

// VALU issues per block (ISA of wf_trace<false,false>, round 3)
static double C_HEAD = 20, C_TRI1 = 95, C_TRI2 = 92, C_NODE = 194, C_STACK = 25, C_REFILL = 110;
// edge-sharing pair (pair_bvh8_leaves): the second triangle of a flagged pair reuses two sheared
// vertices and the diagonal's products of the first (C_TRI2 less two vertex setups of ~13 issues
// and two load address computations); C_PSEL: the pair-first selection per triangle step
static double C_PAIR2 = 60, C_PSEL = 4;

struct Lane {
    bool active = false;
    RaySetup R;
    f3 o;   // world-space origin (R.o is in the triangle test's rotated frame)
    float best;
    uint32_t best_id, g_base, g_hits, t_base, t_mask, t_valid, t_pair = 0;
    bool g_flip;
    int sp;
    uint32_t stack[64];
    // postponed triangle group (policy P)
    uint32_t p_base = 0, p_mask = 0, p_valid = 0;
    uint32_t r_mask = 0;   // deferred root triangles (policy defer_root)
    float r_tn = 0;
    int ray = -1;
    int steps = 0;
};

struct Ray { f3 o, d; };

struct Policy {
    const char* name;
    int refill_min = 8;
    int tris_per_step = 2;
    int postpone_thr = 0;   // > 0: the triangle block runs only when >= thr lanes want it (or a lane is blocked)
    int defer_root = 0;     // root-node triangles tested after the rest of the tree, if their leaf box is still in reach
    int coop = 0;           // > 0: the wave tests every pending triangle of the tri-phase lanes in batches of 64
                            // (one per lane, owner's ray via LDS / bpermute); coop = per-batch overhead issues
    int pairs = 0;          // 1: edge-sharing pairs of a leaf (Bvh8Node::reserved) tested as one pair step
};

struct Scene8 {
    std::vector<Bvh8Node> nodes;
    std::vector<float4> tris;   // 3 per slot
};

static void start(Lane& L, const Ray& r) {
    L.R = ray_setup(r.o, r.d);
    L.o = r.o;
    L.best = INFINITY;
    L.best_id = 0xffffffffu;
    L.g_base = 0;
    L.g_hits = 1;
    L.g_flip = false;
    L.t_mask = 0;
    L.p_mask = 0;
    L.r_mask = 0;
    L.sp = 0;
    L.active = true;
    L.steps = 0;
}

// Edge-sharing triangle pairs inside the leaves (DESIGN.md §3.1 "Triangle pairs").  Two triangles
// of one leaf with vertices A = (a, b, c) and B = (a, c, d) -- the halves of a quad split along its
// a-c diagonal, the fan split the OBJ loader and the procedural meshes emit -- move to leaf
// positions (0, 1) or (2, 3), A first, and bit 4j + i (i = 0 or 2) of Bvh8Node::reserved (this model only: the product does not pair) is set.
// The traversal tests such a pair with four sheared vertices instead of six and forms the
// diagonal's two edge products once; the order of triangles inside a leaf never changes a
// closest-hit or any-hit result.  tri_info4: per original triangle (i0, i1, i2, inst << 8 | submesh);
// world: 9 floats per original triangle (the shared vertices must be bitwise equal there).
// Returns the number of pairs flagged.
static uint32_t pair_bvh8_leaves(Bvh8Result& b8, const uint32_t* ti, const float* world) {
    // B = (A.v0, A.v2, D): same vertex, same instance, bitwise-equal world coordinates
    auto same_vertex = [&](uint32_t a, int va, uint32_t b, int vb) {
        return ti[4 * (size_t)a + va] == ti[4 * (size_t)b + vb] && (ti[4 * (size_t)a + 3] >> 8) == (ti[4 * (size_t)b + 3] >> 8) &&
               std::memcmp(&world[9 * (size_t)a + 3 * va], &world[9 * (size_t)b + 3 * vb], 12) == 0;
    };
    auto fan = [&](uint32_t a, uint32_t b) { return same_vertex(a, 0, b, 0) && same_vertex(a, 2, b, 1); };
    uint32_t pairs = 0;
    for (Bvh8Node& nd : b8.nodes) {
        nd.reserved = 0u;
        for (int j = 0; j < 8; ++j) {
            const uint32_t cnt = bvh8_leaf_count(nd.tri_valid, j);
            if (cnt < 2) continue;
            uint32_t* t = &b8.tri_order[nd.tri_base + bvh8_leaf_first(nd.tri_valid, j)];
            uint32_t order[4], n = 0;
            bool used[4] = {false, false, false, false};
            for (uint32_t a = 0; a < cnt && n + 1 < cnt; ++a) {   // greedy: pairs first, A before B
                if (used[a]) continue;
                for (uint32_t b = 0; b < cnt; ++b) {
                    if (b == a || used[b] || !fan(t[a], t[b])) continue;
                    nd.reserved |= 1u << (4 * j + n);
                    order[n++] = t[a];
                    order[n++] = t[b];
                    used[a] = used[b] = true;
                    ++pairs;
                    break;
                }
            }
            for (uint32_t a = 0; a < cnt; ++a)
                if (!used[a]) order[n++] = t[a];
            std::memcpy(t, order, 4 * cnt);
        }
    }
    return pairs;
}


static std::vector<uint32_t> g_tri_tests;
static double g_nodes = 0, g_tris = 0;
static bool tri_test(const Scene8& S, Lane& L, uint32_t slot) {
    const float4* tp = &S.tris[3 * (size_t)slot];
    if (!g_tri_tests.empty()) g_tri_tests[slot]++;
    g_tris += 1;
    float t, u, v, dt;
    const int kz = L.R.pre.kz;
    if (intersect_rot(L.R.pre, L.R.o, rot3(ld3(tp[0]), kz), rot3(ld3(tp[1]), kz), rot3(ld3(tp[2]), kz), 0.0f, L.best, &t, &u, &v, &dt)) {
        const uint32_t id = __builtin_bit_cast(uint32_t, tp[0].w);
        if (t < L.best || id < L.best_id) {
            L.best = t;
            L.best_id = id;
        }
    }
    return false;
}

static bool node_work(const Lane& L) { return L.g_hits != 0u || L.sp > 0; }

// min entry distance of the hit leaf children of node ni (the slab math of test_node8_words)
static float leaf_tn(const Scene8& S, uint32_t ni, const RaySetup& R, f3 org, float tmax) {
    const Bvh8Node& n = S.nodes[ni];
    const int k = n.axis_k >> 4;
    float best = INFINITY;
    for (int c = k; c < 8; ++c) {
        float tn = 0.0f, tf = tmax * 1.0000004f;
        const float inv[3] = {R.ix, R.iy, R.iz}, o[3] = {org.x, org.y, org.z};
        for (int a = 0; a < 3; ++a) {
            const float sc = ldexpf(1.0f, (int)n.e[a] - 127);
            const float lo = n.p[a] + n.q[16 * a + c] * sc, hi = n.p[a] + n.q[16 * a + 8 + c] * sc;
            float t0 = (lo - o[a]) * inv[a], t1 = (hi - o[a]) * inv[a];
            if (t0 > t1) std::swap(t0, t1);
            tn = std::max(tn, t0);
            tf = std::min(tf, t1);
        }
        if (tn <= tf) best = std::min(best, tn);
    }
    return best;
}

static int g_defer_root = 0;
static void node_step(const Scene8& S, Lane& L) {
    if (!L.g_hits) {
        --L.sp;
        const uint32_t ent = L.stack[L.sp];
        L.g_base = ent >> 9;
        L.g_flip = (ent >> 8) & 1u;
        L.g_hits = ent & 0xffu;
    }
    const int r = L.g_flip ? highest_bit(L.g_hits) : lowest_bit(L.g_hits);
    L.g_hits &= ~(1u << r);
    if (L.g_hits) L.stack[L.sp++] = pack_group(L.g_base, L.g_flip, L.g_hits);
    const uint32_t ni = L.g_base + (uint32_t)r;
    g_nodes += 1;
    test_node8(S.nodes.data(), ni, L.R, 0.0f, L.best, L.g_hits, L.t_mask, L.t_valid, L.g_base, L.t_base, L.g_flip);
    L.t_pair = S.nodes[ni].reserved;
    if (g_defer_root && ni == 0 && L.t_mask) {
        L.r_mask = L.t_mask;
        L.r_tn = leaf_tn(S, 0, L.R, L.o, L.best);
        L.t_mask = 0;
    }
}

struct Result {
    double issues = 0, iters = 0, rays = 0, lane_valu = 0;
    double blk_iss[5] = {}, blk_lanes[5] = {};   // head, refill, tri (all k), node, stack
};

static Result simulate(const Scene8& S, const std::vector<Ray>& rays, const Policy& P) {
    Result res;
    const int W = 64;
    size_t next = 0;
    const size_t chunk = 64;
    // waves draw chunks of the ray stream in turn (one wave at a time is enough for SIMD efficiency)
    const int nwaves = 64;
    std::vector<std::vector<Lane>> waves(nwaves, std::vector<Lane>(W));
    std::vector<size_t> wnext(nwaves, 0), wend(nwaves, 0);
    std::vector<bool> done(nwaves, false);
    int live = nwaves;
    while (live > 0) {
        for (int w = 0; w < nwaves; ++w) {
            if (done[w]) continue;
            auto& lanes = waves[w];
            double cost = C_HEAD;
            int idle = 0;
            for (auto& L : lanes) idle += !L.active;
            const bool refill = idle >= P.refill_min || idle == W;
            if (refill && wnext[w] >= wend[w] && next < rays.size()) {
                wnext[w] = next;
                wend[w] = std::min(next + chunk, rays.size());
                next = wend[w];
            }
            if (refill && idle > 0 && wnext[w] < wend[w]) {
                int got = 0;
                for (auto& L : lanes)
                    if (!L.active && wnext[w] < wend[w]) {
                        start(L, rays[wnext[w]]);
                        L.ray = (int)wnext[w];
                        ++wnext[w];
                        ++got;
                    }
                if (got) { cost += C_REFILL; res.blk_iss[1] += C_REFILL; res.blk_lanes[1] += got * C_REFILL; }
                res.lane_valu += got * C_REFILL;
            }
            int nact = 0;
            for (auto& L : lanes) nact += L.active;
            if (nact == 0) {
                done[w] = true;
                --live;
                continue;
            }
            // triangle block participation
            int want_tri = 0, blocked = 0;
            for (auto& L : lanes)
                if (L.active && (L.t_mask || L.p_mask)) {
                    ++want_tri;
                    // blocked: cannot take a node (no node work, or both triangle groups in use)
                    if (!node_work(L) || (L.t_mask && L.p_mask) || P.postpone_thr == 0) ++blocked;
                }
            const bool tri_phase = want_tri > 0 && (P.postpone_thr == 0 || want_tri >= P.postpone_thr || blocked > 0);
            bool any_t[8] = {}, any_node = false, any_stack = false, any_pair = false;
            int n_t[8] = {}, n_node = 0, n_pair = 0;
            for (auto& L : lanes) {
                if (!L.active) continue;
                bool did_tri = false;
                if (tri_phase && (L.t_mask || L.p_mask)) {
                    if (!L.t_mask) {   // take the postponed group
                        L.t_mask = L.p_mask; L.t_base = L.p_base; L.t_valid = L.p_valid; L.p_mask = 0;
                    }
                    const int lim = P.coop ? 64 : P.tris_per_step;
                    const uint32_t pm = P.pairs ? (L.t_mask & L.t_pair) : 0u;
                    if (pm) {   // the pair first: the first triangle's block, then the pair block
                        const int b = lowest_bit(pm);
                        L.t_mask &= ~(3u << b);
                        tri_test(S, L, tri_slot(L.t_base, L.t_valid, b));
                        tri_test(S, L, tri_slot(L.t_base, L.t_valid, b + 1));
                        any_t[0] = true;
                        ++n_t[0];
                        any_pair = true;
                        ++n_pair;
                    }
                    for (int k = 0; !pm && k < lim && L.t_mask; ++k) {
                        const int b = lowest_bit(L.t_mask);
                        L.t_mask &= L.t_mask - 1u;
                        tri_test(S, L, tri_slot(L.t_base, L.t_valid, b));
                        any_t[P.coop ? 0 : k] = true;
                        ++n_t[P.coop ? 0 : k];
                    }
                    if (!L.t_mask && L.p_mask) {
                        L.t_mask = L.p_mask; L.t_base = L.p_base; L.t_valid = L.p_valid; L.p_mask = 0;
                    }
                    did_tri = true;
                }
                (void)did_tri;
                // node step: no pending triangles (current) or a free postponed slot (policy P)
                bool can_node = node_work(L) && (L.t_mask == 0u || (P.postpone_thr > 0 && L.p_mask == 0u));
                if (can_node) {
                    if (L.t_mask) {   // postpone the current group
                        L.p_mask = L.t_mask; L.p_base = L.t_base; L.p_valid = L.t_valid; L.t_mask = 0;
                    }
                    const bool pop = !L.g_hits;
                    node_step(S, L);
                    any_node = true;
                    ++n_node;
                    if (pop || L.sp) any_stack = true;
                }
                ++L.steps;
                if (L.t_mask == 0u && L.p_mask == 0u && !node_work(L) && L.r_mask) {
                    if (L.r_tn <= L.best * 1.0000004f) {
                        L.t_mask = L.r_mask;
                        L.t_base = S.nodes[0].tri_base;
                        L.t_valid = S.nodes[0].tri_valid;
                    }
                    L.r_mask = 0;
                }
                if (L.t_mask == 0u && L.p_mask == 0u && !node_work(L)) {
                    L.active = false;
                    res.rays += 1;
                    res.iters += L.steps;
                }
            }
            if (P.coop) {
                const int batches = (n_t[0] + 63) / 64;
                const double c = batches * (C_TRI1 + P.coop);
                cost += c;
                res.blk_iss[2] += c;
                res.blk_lanes[2] += n_t[0] * C_TRI1;
                n_t[0] = 0;
            }
            if (any_pair) { cost += C_PAIR2; res.blk_iss[2] += C_PAIR2; res.blk_lanes[2] += n_pair * C_PAIR2; res.lane_valu += n_pair * C_PAIR2; }
            if (P.pairs && any_t[0]) { cost += C_PSEL; res.blk_iss[2] += C_PSEL; res.blk_lanes[2] += n_t[0] * C_PSEL; res.lane_valu += n_t[0] * C_PSEL; }
            for (int k = 0; k < 8; ++k) if (any_t[k] && n_t[k]) { cost += k ? C_TRI2 : C_TRI1; res.blk_iss[2] += k ? C_TRI2 : C_TRI1; res.blk_lanes[2] += n_t[k] * (k ? C_TRI2 : C_TRI1); }
            res.blk_iss[0] += C_HEAD; res.blk_lanes[0] += nact * C_HEAD;
            if (any_node) { res.blk_iss[3] += C_NODE; res.blk_lanes[3] += n_node * C_NODE; }
            if (any_stack) res.blk_iss[4] += C_STACK;
            if (any_node) cost += C_NODE;
            if (any_stack) cost += C_STACK;
            res.lane_valu += n_node * C_NODE + nact * C_HEAD;
            for (int k = 0; k < 8; ++k) res.lane_valu += n_t[k] * (k ? C_TRI2 : C_TRI1);
            res.issues += cost;
        }
    }
    return res;
}

int main(int argc, char** argv) {
    const char* assets = argc > 1 ? argv[1] : "assets";
    const int stride = argc > 2 ? atoi(argv[2]) : 4;   // pixel subsampling
    rt_scene* sc = nullptr;
    int32_t synth = 0;
    if (rt_scene_preset("c3g", assets, &sc, &synth) != RT_OK) { fprintf(stderr, "preset failed\n"); return 1; }
    rt_scene_desc D;
    rt_scene_get_desc(sc, &D);
    std::vector<float> world;
    std::vector<uint32_t> tinfo;   // per triangle (i0, i1, i2, inst << 8): global vertex indices, as tri_info
    uint32_t vbase = 0;
    for (uint32_t m = 0; m < D.mesh_count; ++m) {
        const rt_mesh_desc& M = D.meshes[m];
        const float* T = &M.transform.columns[0][0];
        for (uint32_t s = 0; s < M.submesh_count; ++s) {
            const rt_submesh_desc& SM = M.submeshes[s];
            for (uint32_t i = 0; i < SM.index_count; ++i) {
                tinfo.push_back(vbase + SM.indices[i]);
                if (i % 3 == 2) tinfo.push_back(m << 8);
                const rt_float3& p = M.positions[SM.indices[i]];
                for (int r = 0; r < 3; ++r)
                    world.push_back(((T[0 + r] * p.x + T[3 + r] * p.y) + T[6 + r] * p.z) + T[9 + r] * 1.0f);
            }
        }
        vbase += M.vertex_count;
    }
    const uint32_t n = (uint32_t)(world.size() / 9);
    fprintf(stderr, "%u triangles; building\n", n);
    BvhResult b2;
    Bvh8Result b8;
    for (int limit : {64, 48, 40, 32, 28, 24, 21}) {
        b2 = build_bvh2(world.data(), n, 1, limit);
        b8 = collapse_bvh8_dp(b2, 1.0f, getenv("SIM_CPRIM") ? (float)atof(getenv("SIM_CPRIM")) : 0.5f);
        if (b8.max_depth <= 16) break;
    }
    uint32_t npairs = 0;
    if (getenv("SIM_PAIRS")) {
        npairs = pair_bvh8_leaves(b8, tinfo.data(), world.data());
        fprintf(stderr, "%u edge-sharing pairs flagged in leaves (%u triangles)\n", npairs, n);
    }
    Scene8 S;
    S.nodes = b8.nodes;
    S.tris.resize(3 * (size_t)b8.tri_order.size());
    fprintf(stderr, "%zu slots for %u triangles\n", b8.tri_order.size(), n);
    for (size_t k = 0; k < b8.tri_order.size(); ++k) {
        const uint32_t id = b8.tri_order[k];
        for (int v = 0; v < 3; ++v) {
            const float* p = &world[9 * (size_t)id + 3 * v];
            S.tris[3 * k + v] = make_float4(p[0], p[1], p[2], v == 0 ? __builtin_bit_cast(float, id) : 0.0f);
        }
    }
    fprintf(stderr, "%zu nodes, depth %d\n", S.nodes.size(), b8.max_depth);
    for (int ni = 0; ni < 3; ++ni) {
        const Bvh8Node& r = S.nodes[ni];
        fprintf(stderr, "node %d: k_int %d tri_base %u tri_valid %08x\n", ni, r.axis_k >> 4, r.tri_base, r.tri_valid);
    }
    // primary rays: every stride-th pixel of 1920x1080, 4 samples each (jittered), queue order
    Camera cam;
    rt_camera_default(1920, 1080, &cam);
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U01(0.0f, 1.0f);
    std::vector<Ray> prim, sec;
    for (int py = 0; py < 1080; py += stride)
        for (int px = 0; px < 1920; px += stride)
            for (int s = 0; s < 4; ++s) {
                float uvx = ((px + U01(rng)) / 1920.0f) * 2.0f - 1.0f, uvy = ((py + U01(rng)) / 1080.0f) * 2.0f - 1.0f;
                f3 d = normalize((uvx * ldf3(cam.right) + uvy * ldf3(cam.up)) + ldf3(cam.forward));
                prim.push_back(Ray{ldf3(cam.position), d});
            }
    // one diffuse bounce from each primary hit (closest hit by a serial trace)
    TraceCounters tc{0, 0, 0};
    std::vector<int> stackbuf(16 * kBlock);
    DevScene DS{};
    std::vector<float> recs((size_t)kTriFloats * b8.tri_order.size());   // the product's 64-B records for trace8
    for (size_t k = 0; k < b8.tri_order.size(); ++k)
        tri_store(&recs[(size_t)kTriFloats * k], &world[9 * (size_t)b8.tri_order[k]], b8.tri_order[k]);
    DS.tris = recs.data();
    DS.nodes8 = S.nodes.data();
    for (const Ray& r : prim) {
        Hit h;
        bool ovf = false;
        if (!trace8<false, false>(DS, r.o, r.d, 0.0f, INFINITY, h, stackbuf.data(), tc, ovf) || h.id == 0xffffffffu) continue;
        const float* p0 = &world[9 * (size_t)h.id];
        f3 a = mk3(p0[0], p0[1], p0[2]), b = mk3(p0[3], p0[4], p0[5]), c = mk3(p0[6], p0[7], p0[8]);
        f3 N = normalize(cross(b - a, c - a));
        if (dot(N, r.d) > 0) N = -N;
        f3 P = r.o + r.d * h.t;
        // cosine hemisphere
        float r1 = U01(rng), r2 = U01(rng), phi = 6.2831853f * r1, sr = sqrtf(r2);
        f3 t = fabsf(N.x) > 0.5f ? mk3(0, 1, 0) : mk3(1, 0, 0);
        f3 X = normalize(cross(t, N)), Y = cross(N, X);
        f3 d = normalize((X * (cosf(phi) * sr) + Y * (sinf(phi) * sr)) + N * sqrtf(1.0f - r2));
        sec.push_back(Ray{P + N * 1e-3f, d});
    }
    fprintf(stderr, "%zu primary, %zu secondary rays\n", prim.size(), sec.size());
    std::vector<Policy> pols;
    pols.push_back(Policy{"current (refill 8, 2 tris)", 8, 2, 0});
    if (getenv("SIM_PAIRS")) pols.push_back(Policy{"edge-sharing pairs", 8, 2, 0, 0, 0, 1});
    pols.push_back(Policy{"refill 16", 16, 2, 0});
    pols.push_back(Policy{"1 tri per step", 8, 1, 0});
    pols.push_back(Policy{"4 tris per step", 8, 4, 0});
    pols.push_back(Policy{"3 tris per step", 8, 3, 0});
    pols.push_back(Policy{"postpone 24 + 3 tris", 8, 3, 24});
    pols.push_back(Policy{"postpone 24 + 4 tris", 8, 4, 24});
    pols.push_back(Policy{"defer root tris", 8, 2, 0, 1, 0});
    pols.push_back(Policy{"defer root + postpone 24", 8, 2, 24, 1, 0});
    pols.push_back(Policy{"coop ovh 40", 8, 2, 0, 0, 40});
    pols.push_back(Policy{"coop ovh 60", 8, 2, 0, 0, 60});
    pols.push_back(Policy{"coop ovh 60 + postpone 24", 8, 2, 24, 0, 60});
    for (int thr : {24}) {
        static char buf[8][64];
        static int bi = 0;
        snprintf(buf[bi], 64, "postpone thr %d", thr);
        pols.push_back(Policy{buf[bi++], 8, 2, thr});
    }
    if (getenv("SIM_TRISTATS")) {
        g_tri_tests.assign(S.tris.size() / 3, 0);
        Policy P0{"x", 8, 2, 0};
        simulate(S, sec, P0);
        std::vector<std::pair<uint32_t, uint32_t>> v;
        double total = 0;
        for (size_t k = 0; k < g_tri_tests.size(); ++k) { v.push_back({g_tri_tests[k], (uint32_t)k}); total += g_tri_tests[k]; }
        std::sort(v.rbegin(), v.rend());
        double acc = 0;
        printf("secondary: %.0f triangle tests, %.2f per ray\n", total, total / sec.size());
        for (int i = 0; i < 40; ++i) {
            acc += v[i].first;
            const float4* t = &S.tris[3 * (size_t)v[i].second];
            f3 a = ld3(t[0]), b = ld3(t[1]), c = ld3(t[2]);
            printf("  slot %u id %u tests %u (cum %.3f) area %.4g\n", v[i].second, __builtin_bit_cast(uint32_t, t[0].w), v[i].first, acc / total, 0.5f * length(cross(b - a, c - a)));
        }
        return 0;
    }
    for (int set = 0; set < 2; ++set) {
        const auto& rays = set ? sec : prim;
        printf("== %s rays (%zu)\n", set ? "secondary (diffuse bounce)" : "primary", rays.size());
        for (const Policy& P : pols) {
            g_nodes = g_tris = 0;
            g_defer_root = P.defer_root;
            Result r = simulate(S, rays, P);
            printf("  %-28s issues/ray %7.2f  iters/ray %6.2f  lane util %.3f  nodes/ray %.2f tris/ray %.2f\n", P.name, r.issues / r.rays,
                   r.iters / r.rays, r.lane_valu / (r.issues * 64.0), g_nodes / r.rays, g_tris / r.rays);
            const char* bn[5] = {"head", "refill", "tri", "node", "stack"};
            printf("     ");
            for (int b = 0; b < 5; ++b) printf(" %s %.2f/ray (util %.2f)", bn[b], r.blk_iss[b] / r.rays, r.blk_iss[b] > 0 ? r.blk_lanes[b] / (64.0 * r.blk_iss[b]) : 0.0);
            printf("\n");
        }
    }
    rt_scene_free(sc);
    return 0;
}
