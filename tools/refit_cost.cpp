// refit_cost.cpp — host tool: how a refit degrades the tree when one instance moves.
// Builds the preset's 8-wide BVH (the product's host builder), translates mesh 0 (the hero) by dx
// along x, refits the node boxes bottom-up (same topology, as rt_bvh_refit does on the device) and
// prints the node-area sum (launch_bvh_cost's metric) of the build, of the refit and of a fresh
// build of the moved scene.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude tools/refit_cost.cpp -Lmetal4-raytracing_amd -lrt_hip \
//     -Wl,-rpath,$PWD/metal4-raytracing_amd -o /tmp/refit_cost && /tmp/refit_cost assets c3g 0.1 1 3
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../metal4-raytracing_amd/csrc/rt_bvh.h"
#include "../include/rt_scene.h"
#include "../include/rt_api.h"

using namespace rt;

static std::vector<float> world_of(const rt_scene_desc& D, float dx) {
    std::vector<float> w;
    for (uint32_t m = 0; m < D.mesh_count; ++m) {
        const rt_mesh_desc& M = D.meshes[m];
        const float* T = &M.transform.columns[0][0];
        for (uint32_t s = 0; s < M.submesh_count; ++s)
            for (uint32_t i = 0; i < M.submeshes[s].index_count; ++i) {
                const rt_float3& p = M.positions[M.submeshes[s].indices[i]];
                for (int r = 0; r < 3; ++r)
                    w.push_back(((T[0 + r] * p.x + T[3 + r] * p.y) + T[6 + r] * p.z) + T[9 + r] * 1.0f + (m == 0 && r == 0 ? dx : 0.0f));
            }
    }
    return w;
}
static double area(const float* lo, const float* hi) {
    const double a = hi[0] - lo[0], b = hi[1] - lo[1], c = hi[2] - lo[2];
    return (a >= 0 && b >= 0 && c >= 0) ? 2.0 * (a * b + b * c + c * a) : 0.0;
}
static Bvh8Result build(const std::vector<float>& w) {
    Bvh8Result b8;
    for (int limit : {64, 48, 40, 32, 28, 24, 21}) {
        BvhResult b2 = build_bvh2(w.data(), (uint32_t)(w.size() / 9), 1, limit);
        b8 = collapse_bvh8_dp(b2, 1.0f, 0.5f);
        if (b8.max_depth <= 16) break;
    }
    return b8;
}
static double node_area_sum(const Bvh8Result& b) {
    double s = 0;
    for (size_t k = 0; k < b.nodes.size(); ++k) s += area(&b.node_box[6 * k], &b.node_box[6 * k + 3]);
    return s;
}
// the boxes of b's topology over the triangles w (children before parents: node k's children > k)
static double refit_sum(const Bvh8Result& b, const std::vector<float>& w) {
    std::vector<float> box(b.node_box.size());
    for (size_t k = b.nodes.size(); k-- > 0;) {
        const Bvh8Node& n = b.nodes[k];
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        const int ki = n.axis_k >> 4;
        for (int c = 0; c < ki; ++c)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::fmin(lo[a], box[6 * (n.child_base + c) + a]);
                hi[a] = std::fmax(hi[a], box[6 * (n.child_base + c) + 3 + a]);
            }
        for (int j = 0; j < 8; ++j) {
            const uint32_t f = n.tri_base + bvh8_leaf_first(n.tri_valid, j), cnt = bvh8_leaf_count(n.tri_valid, j);
            for (uint32_t t = 0; t < cnt; ++t)
                for (int v = 0; v < 3; ++v)
                    for (int a = 0; a < 3; ++a) {
                        const float x = w[9 * (size_t)b.tri_order[f + t] + 3 * v + a];
                        lo[a] = std::fmin(lo[a], x);
                        hi[a] = std::fmax(hi[a], x);
                    }
        }
        for (int a = 0; a < 3; ++a) { box[6 * k + a] = lo[a]; box[6 * k + 3 + a] = hi[a]; }
    }
    double s = 0;
    for (size_t k = 0; k < b.nodes.size(); ++k) s += area(&box[6 * k], &box[6 * k + 3]);
    if (getenv("REFIT_DEBUG"))
        fprintf(stderr, "root refit box %g %g %g / %g %g %g, build %g %g %g / %g %g %g\n", box[0], box[1], box[2], box[3], box[4],
                box[5], b.node_box[0], b.node_box[1], b.node_box[2], b.node_box[3], b.node_box[4], b.node_box[5]);
    return s;
}

int main(int argc, char** argv) {
    const char* assets = argc > 1 ? argv[1] : "assets";
    const char* preset = argc > 2 ? argv[2] : "c3g";
    rt_scene* sc = nullptr;
    int32_t synth = 0;
    if (rt_scene_preset(preset, assets, &sc, &synth) != RT_OK) { fprintf(stderr, "preset failed\n"); return 1; }
    rt_scene_desc D;
    rt_scene_get_desc(sc, &D);
    const std::vector<float> w0 = world_of(D, 0.0f);
    const Bvh8Result b0 = build(w0);
    const double s0 = node_area_sum(b0);
    printf("%s: %zu triangles, %zu nodes, node-area sum at build %.4g\n", preset, w0.size() / 9, b0.nodes.size(), s0);
    for (int i = 3; i < argc; ++i) {
        const float dx = (float)atof(argv[i]);
        const std::vector<float> w = world_of(D, dx);
        const double sr = refit_sum(b0, w), sb = node_area_sum(build(w));
        printf("  hero moved %+.2f along x: refit %.4g (x%.3f of the build), fresh build %.4g (x%.3f)\n", dx, sr, sr / s0, sb,
               sb / s0);
    }
    rt_scene_free(sc);
    return 0;
}
