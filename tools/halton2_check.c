/* halton2_check.c -- the base-2 Halton radical inverse in closed form (rt_math.h halton_base2)
 * against the reference loop (rt_math.h halton_fast, Raytracing.metal:42-57) over a range of
 * indices, bit for bit.  g++ -O2 -ffp-contract=off -std=c++17 -I. -x c++ tools/halton2_check.c -o /tmp/h2;
 * /tmp/h2 [lo hi]  (default: every positive int, ~1 min per 2^29 indices on one core). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "metal4-raytracing_amd/csrc/rt_math.h"

static float loop2(int i) {
    rt::HaltonDim h;
    h.b = 2u;
    h.m = 0x80000000u;   /* ceil(2^32 / 2), l = 1 */
    h.sh = 0u;
    h.invB = 0.5f;
    return rt::halton_fast(i, h);
}

int main(int argc, char** argv) {
    const uint32_t lo = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 0) : 1u;
    const uint32_t hi = argc > 2 ? (uint32_t)strtoul(argv[2], 0, 0) : 0x7fffffffu;
    unsigned long long bad = 0;
    for (uint32_t i = lo;; ++i) {
        const float a = loop2((int)i), b = rt::halton_base2((int)i);
        uint32_t x, y;
        memcpy(&x, &a, 4);
        memcpy(&y, &b, 4);
        if (x != y) {
            if (bad < 5) printf("mismatch %u: loop %a closed %a\n", i, a, b);
            ++bad;
        }
        if (i >= hi) break;
    }
    printf("range %u..%u: %llu mismatches\n", lo, hi, bad);
    return bad != 0;
}
