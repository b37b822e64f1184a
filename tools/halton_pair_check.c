/* halton_pair_check.c -- a two-digits-per-step form of the Halton radical inverse against the
 * one-digit loop (rt_math.h halton_fast, Raytracing.metal:42-57), bit for bit.  Round 6 built it
 * into the shading code (verdict item 6) and measured it: bit-exact (397 GPU tests), wf_shade
 * 0.3346 / 0.3350 ms against 0.3347 / 0.3357, one frame 4.662 / 4.643 against 4.632 / 4.633 ms
 * (profiles/r06_experiments.txt), so the product keeps the one-digit loop; this file keeps the form
 * and its exactness check.
 *
 * The form: q = n / b^2 by one multiply-high (Granlund-Montgomery with d = b^2); the pair
 * p = n - q b^2 < 2^24 from one v_mad_u32_u24 modulo 2^24 (n + q (2^24 - b^2)); its digits in fp32
 * exactly: d1 = trunc(p * rb) with rb = 1/b rounded up, d0 = fma(-d1, b, p); then the loop's float
 * operations digit for digit (f = f * invB; r = r + f * d0; f = f * invB; r = r + f * d1).  When the
 * loop would stop after d0 the extra step adds f * 0 = +0.  Bases up to 2896 (b^2 < 2^23).
 *   g++ -O2 -ffp-contract=off -std=c++17 -I. -x c++ tools/halton_pair_check.c -o /tmp/hp
 *   /tmp/hp split            every pair value p < b^2 of every base b <= 2896: the fp32 split gives
 *                            p / b and p % b, and the 24-bit remainder recovers p for the largest q
 *   /tmp/hp dims N SEED      N random indices (and every b^k +- 2 boundary) in each of the 1024
 *                            dimensions: the pair form == halton_fast
 *   /tmp/hp range D LO HI    every index LO..HI in dimension D (all 2^31 for D = 1..79, the
 *                            dimensions maxBounces <= 12 reaches, ~3 min each on one core) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "metal4-raytracing_amd/csrc/rt_math.h"

static const uint32_t kPairMaxB = 2896;
struct PairDim { uint32_t b, m2, sh2; float invB, rb; };
static rt::HaltonDim one_digit(uint32_t b) {
    uint32_t l = 0;
    while ((1u << l) < b) ++l;
    rt::HaltonDim h;
    h.b = b;
    h.m = (uint32_t)(((1ull << (31 + l)) + b - 1) / b);
    h.sh = l - 1;
    h.invB = 1.0f / (float)b;
    return h;
}
static PairDim pair_dim(uint32_t b) {
    const uint64_t d = (uint64_t)b * b;
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    PairDim h;
    h.b = b;
    h.m2 = (uint32_t)(((1ull << (31 + l)) + d - 1) / d);
    h.sh2 = l - 1;
    h.invB = 1.0f / (float)b;
    float r = 1.0f / (float)b;
    if ((double)r * (double)b < 1.0) r = nextafterf(r, 2.0f);   /* exact product: round up */
    h.rb = r;
    return h;
}
static float halton_pair(int i, const PairDim& h) {
    const uint32_t bneg = 0x1000000u - h.b * h.b;
    const float bf = (float)h.b;
    float f = 1.0f, r = 0.0f;
    uint32_t n = (uint32_t)i;
    if (i <= 0) return 0.0f;
    while (n > 0) {
        const uint32_t q = rt::umulhi32(n, h.m2) >> h.sh2;
        const uint32_t x = (uint32_t)((uint64_t)(q & 0xffffffu) * bneg + n);   /* v_mad_u32_u24 */
        const float p = (float)(x & 0xffffffu);
        const float d1 = truncf(p * h.rb);
        const float d0 = fmaf(-d1, bf, p);
        f = f * h.invB;
        r = r + f * d0;
        f = f * h.invB;
        r = r + f * d1;
        n = q;
    }
    return r;
}

static int primes[1024];
static void init_primes(void) {
    int n = 2, k = 0;
    while (k < 1024) {
        int is = 1;
        for (int i = 0; i < k && primes[i] * primes[i] <= n; ++i)
            if (n % primes[i] == 0) { is = 0; break; }
        if (is) primes[k++] = n;
        ++n;
    }
}
static uint32_t bits(float f) { uint32_t x; memcpy(&x, &f, 4); return x; }
static unsigned long long bad = 0;
static void cmp(int d, uint32_t i, const PairDim& h2, const rt::HaltonDim& h1) {
    const float a = h2.b <= kPairMaxB ? halton_pair((int)i, h2) : rt::halton_fast((int)i, h1),
                b = rt::halton_fast((int)i, h1);
    if (bits(a) != bits(b)) {
        if (bad < 5) printf("dim %d i %u: pair %a loop %a\n", d, i, a, b);
        ++bad;
    }
}
static uint64_t rng = 0;
static uint32_t next31(void) {
    rng = rng * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(rng >> 33);
}

int main(int argc, char** argv) {
    init_primes();
    const char* mode = argc > 1 ? argv[1] : "split";
    if (!strcmp(mode, "split")) {
        int nb = 0;
        for (int k = 0; k < 1024; ++k) {
            const uint32_t b = (uint32_t)primes[k];
            if (b > kPairMaxB) continue;
            const PairDim h = pair_dim(b);
            ++nb;
            const float bf = (float)b;
            const uint32_t bneg = 0x1000000u - b * b, qmax = 0x7fffffffu / (b * b);
            for (uint32_t p = 0; p < b * b; ++p) {
                const float pf = (float)p;
                const float d1 = truncf(pf * h.rb), d0 = fmaf(-d1, bf, pf);
                if (d1 != (float)(p / b) || d0 != (float)(p % b)) {
                    if (bad < 5) printf("b %u p %u: %g %g\n", b, p, d1, d0);
                    ++bad;
                }
                const uint32_t n = qmax * b * b + p;   /* the largest quotient with this pair */
                if (n <= 0x7fffffffu) {
                    const uint32_t q = rt::umulhi32(n, h.m2) >> h.sh2;
                    const uint32_t x = (uint32_t)((uint64_t)(q & 0xffffffu) * bneg + n) & 0xffffffu;
                    if (q != qmax || x != p) {
                        if (bad < 5) printf("b %u n %u: q %u x %u\n", b, n, q, x);
                        ++bad;
                    }
                }
            }
        }
        printf("split: %d pair bases, %llu mismatches\n", nb, bad);
    } else if (!strcmp(mode, "dims")) {
        const long n = argc > 2 ? atol(argv[2]) : 100000;
        rng = argc > 3 ? strtoull(argv[3], 0, 0) : 1;
        for (int d = 1; d < 1024; ++d) {
            const uint32_t b = (uint32_t)primes[d];
            const PairDim h2 = pair_dim(b);
            const rt::HaltonDim h1 = one_digit(b);
            for (long k = 0; k < n; ++k) cmp(d, next31(), h2, h1);
            for (uint64_t p = 1; p <= 0x7fffffffull; p *= b)
                for (int e = -2; e <= 2; ++e)
                    if ((int64_t)p + e > 0 && (int64_t)p + e <= 0x7fffffff) cmp(d, (uint32_t)((int64_t)p + e), h2, h1);
            cmp(d, 0x7fffffffu, h2, h1);
        }
        printf("dims: %ld random indices per dimension, %llu mismatches\n", n, bad);
    } else {
        const int d = argc > 2 ? atoi(argv[2]) : 2;
        const uint32_t lo = argc > 3 ? (uint32_t)strtoul(argv[3], 0, 0) : 1u;
        const uint32_t hi = argc > 4 ? (uint32_t)strtoul(argv[4], 0, 0) : 0x7fffffffu;
        const PairDim h2 = pair_dim((uint32_t)primes[d]);
        const rt::HaltonDim h1 = one_digit((uint32_t)primes[d]);
        for (uint32_t i = lo;; ++i) {
            cmp(d, i, h2, h1);
            if (i >= hi) break;
        }
        printf("range dim %d %u..%u: %llu mismatches\n", d, lo, hi, bad);
    }
    return bad != 0;
}
