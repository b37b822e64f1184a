// Mutation fuzzer for the host-side readers of untrusted asset bytes: the USD text / crate / zip
// readers behind rt_scene_add_usd (rt_usd.cpp + the scene mapping in rt_scene.cpp) and the PNG
// decoder (rt_texture.cpp) and the OBJ reader (rt_scene.cpp).  Built with AddressSanitizer + UBSan by tools/fuzz_host.sh; every
// input must end in RT_OK or an error status, never in a sanitizer report or a crash.
//
//   fuzz_host <usda|usdc|usdz|png|obj> <seed file> <iterations> <rng seed>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <unistd.h>

#include "../include/rt_scene.h"

static uint64_t g_rng = 0x9e3779b97f4a7c15ull;
static uint64_t rnd() {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return g_rng;
}

static void mutate(std::vector<uint8_t>& b) {
    static const uint64_t kInteresting[] = {0, 1, 2, 0x7f, 0x80, 0xff, 0x7fff, 0x8000, 0xffff, 0x7fffffffu,
                                            0x80000000u, 0xffffffffu, 0x100000000ull, 0x7fffffffffffffffull,
                                            0xffffffffffffffffull, 0x4000000000000000ull, 0xc000000000000000ull};
    const int n = 1 + (int)(rnd() % 6);
    for (int k = 0; k < n && !b.empty(); ++k) {
        const size_t at = rnd() % b.size();
        switch (rnd() % 7) {
            case 0: b[at] ^= (uint8_t)(1u << (rnd() % 8)); break;
            case 1: b[at] = (uint8_t)rnd(); break;
            case 2: {   // an interesting little-endian integer of 1, 2, 4 or 8 bytes
                const uint64_t v = kInteresting[rnd() % (sizeof kInteresting / sizeof kInteresting[0])];
                const size_t w = (size_t)1 << (rnd() % 4);
                for (size_t i = 0; i < w && at + i < b.size(); ++i) b[at + i] = (uint8_t)(v >> (8 * i));
                break;
            }
            case 3: b.resize(at); break;   // truncate
            case 4: {                      // duplicate a span
                const size_t len = std::min<size_t>(b.size() - at, 1 + rnd() % 64);
                std::vector<uint8_t> span(b.begin() + at, b.begin() + at + len);
                b.insert(b.begin() + rnd() % (b.size() + 1), span.begin(), span.end());
                break;
            }
            case 5: {   // delete a span
                const size_t len = std::min<size_t>(b.size() - at, 1 + rnd() % 16);
                b.erase(b.begin() + at, b.begin() + at + len);
                break;
            }
            default: {   // small add / subtract on a byte (text numbers, counts)
                b[at] = (uint8_t)(b[at] + (int)(rnd() % 5) - 2);
                break;
            }
        }
    }
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s <usda|usdc|usdz|png|obj> <seed> <iterations> <rng seed>\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    FILE* f = std::fopen(argv[2], "rb");
    if (!f) return 2;
    std::vector<uint8_t> seed;
    uint8_t buf[65536];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof buf, f)) > 0) seed.insert(seed.end(), buf, buf + got);
    std::fclose(f);
    const long iters = std::atol(argv[3]);
    g_rng ^= (uint64_t)std::atoll(argv[4]) * 0x2545f4914f6cdd1dull;
    const std::string tmp = "/tmp/fuzz_host_" + std::to_string(getpid()) + "." + mode;
    long ok = 0, fail = 0;
    for (long it = 0; it < iters; ++it) {
        std::vector<uint8_t> b = seed;
        if (it > 0) mutate(b);
        rt_status st;
        if (mode == "png") {
            uint32_t w = 0, h = 0;
            char err[128];
            st = rt_decode_png(b.data(), b.size(), nullptr, &w, &h, err, sizeof err);
            if (st == RT_OK && (uint64_t)w * h <= (1u << 22)) {
                std::vector<uint8_t> rgba((size_t)w * h * 4);
                st = rt_decode_png(b.data(), b.size(), rgba.data(), &w, &h, err, sizeof err);
            }
        } else {
            FILE* o = std::fopen(tmp.c_str(), "wb");
            if (!o) return 2;
            std::fwrite(b.data(), 1, b.size(), o);
            std::fclose(o);
            rt_scene* sc = nullptr;
            rt_scene_new(&sc);
            const float pos[3] = {0, 0, 0}, rot[3] = {0, 0, 0};
            st = mode == "obj" ? rt_scene_add_obj(sc, tmp.c_str(), pos, rot, 1.0f, nullptr)
                               : rt_scene_add_usd(sc, tmp.c_str(), pos, rot, 1.0f, nullptr);
            if (st == RT_OK) {
                rt_scene_desc d;
                if (rt_scene_get_desc(sc, &d) == RT_OK)
                    for (uint32_t m = 0; m < d.mesh_count; ++m)
                        if (d.meshes[m].joint_count > 0 && d.meshes[m].joint_count <= 4096) {
                            std::vector<float> J((size_t)d.meshes[m].joint_count * 16);
                            uint32_t jc = 0;
                            rt_scene_joint_matrices(sc, m, 0.75, J.data(), d.meshes[m].joint_count, &jc);
                        }
            }
            rt_scene_free(sc);
        }
        (st == RT_OK ? ok : fail)++;
    }
    std::remove(tmp.c_str());
    std::printf("%s: %ld inputs, %ld accepted, %ld rejected\n", mode.c_str(), iters, ok, fail);
    return 0;
}
