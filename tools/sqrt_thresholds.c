/* sqrt_thresholds.c -- the exact dot-product bounds behind rt_math.h's length_lt / length_gt:
 * for the three constants the shading code compares a length against (Raytracing.metal:395, :651,
 * :653, :692, :751), sqrtf(d) < c  <=>  d < D(c)  and  sqrtf(d) > c  <=>  d > E(c)  for every
 * non-negative float d (+inf included; NaN is false on both sides).  sqrtf and round-to-nearest are
 * monotonic, so the bounds are the first / last float on the other side.  Default: recompute the
 * bounds and check every non-negative float (~40 s); "band N": only the 2N floats around each bound.
 *   gcc -O2 -ffp-contract=off tools/sqrt_thresholds.c -o /tmp/st -lm && /tmp/st [band N] */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float fb(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char** argv) {
    const float cs[3] = {1e-10f, 0.001f, 0.0001f};
    const uint32_t want_d[3] = {0x1e3ce508u, 0x358637bdu, 0x322bcc76u};   /* rt_math.h */
    const uint32_t want_e[3] = {0x1e3ce509u, 0x358637beu, 0x322bcc77u};
    const uint32_t band = (argc > 2 && !strcmp(argv[1], "band")) ? (uint32_t)strtoul(argv[2], 0, 0) : 0u;
    int fail = 0;
    for (int k = 0; k < 3; ++k) {
        const float c = cs[k];
        const uint32_t lo = band ? want_d[k] - band : 0u, hi = band ? want_e[k] + band : 0x7f800000u;
        uint32_t D = 0xffffffffu, E = 0u;
        unsigned long long bad = 0;
        for (uint32_t u = lo; u <= hi; ++u) {
            const float d = fb(u), s = sqrtf(d);
            if (s >= c && D == 0xffffffffu) D = u;
            if (s <= c) E = u;
            if ((s < c) != (d < fb(want_d[k]))) ++bad;
            if ((s > c) != (d > fb(want_e[k]))) ++bad;
        }
        printf("c=%g: D=0x%08x E=0x%08x (rt_math.h 0x%08x 0x%08x) mismatches %llu\n", c, D, E, want_d[k], want_e[k], bad);
        fail |= bad != 0 || D != want_d[k] || E != want_e[k];
    }
    return fail;
}
