// valu_rate.hip — VALU issue rate of single instruction kinds on gfx950 (tool, not product).
// Each kernel runs ITER x 64 independent instructions of one kind (8 register chains, inline asm
// so nothing folds) on every lane of W waves per SIMD; prints cycles per wave-instruction per SIMD
// (s_memtime cycles of the launch x SIMDs / wave-instructions).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/valu_rate.hip -o tools/ubench/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int ITER = 2048;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int K>
__global__ void __launch_bounds__(256) k_rate(float* out, unsigned long long* cyc, float seed) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = seed * 0.5f, c = seed * 0.25f;
    typedef float v2f __attribute__((ext_vector_type(2)));
    v2f a2x[8] = {}, b2 = {b, c}, c2 = {c, b};
    for (int q = 0; q < 8; ++q) a2x[q] = v2f{a0 + q, a1 + q};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITER; ++i) {
#define BODY(n)                                                                                  \
        if (K == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a##n) : "v"(b), "v"(c));                \
        if (K == 1) asm volatile("v_cvt_f32_ubyte1 %0, %0" : "+v"(a##n));                                  \
        if (K == 2) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a##n) : "v"(b), "v"(c));               \
        if (K == 3) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##n) : "v"(b) : "vcc");          \
        if (K == 4) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##n) : "v"(b));                         \
        if (K == 5) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##n) : "v"(b), "v"(c));               \
        if (K == 6) asm volatile("v_pk_fma_f16 %0, %0, %1, %2" : "+v"(a##n) : "v"(b), "v"(c));             \
        if (K == 7) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##n) : "v"(b));                            \
        if (K == 8) asm volatile("v_cmp_le_f32 vcc, %0, %1\n v_cndmask_b32 %0, 0, %0, vcc" : "+v"(a##n) : "v"(b) : "vcc");  \
        if (K == 9) asm volatile("v_rcp_f32 %0, %0" : "+v"(a##n));                                       \
        if (K == 10) asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a##n) : "v"(b));                       \
        if (K == 11) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a##n));                                 \
        if (K == 12) asm volatile("v_fma_f32 %0, %0, %1, %2\n v_cvt_f32_ubyte1 %0, %0" : "+v"(a##n) : "v"(b), "v"(c)); \
        if (K == 13) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a##n) : "v"(b));                         \
        if (K == 14) asm volatile("v_fma_mix_f32 %0, %1, %0, %2 op_sel_hi:[1,0,0]" : "+v"(a##n) : "v"(b), "v"(c)); \
        if (K == 15) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(a##n));                                  \
        if (K == 16) asm volatile("v_cmp_le_f32 s[40:41], %0, %1" : : "v"(a##n), "v"(b) : "s40", "s41");  \
        if (K == 17) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(a##n) : "v"(b) : "s40", "s41"); \
        if (K == 18) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a##n) : "v"(b), "v"(c));              \
        if (K == 19) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a##n) : "v"(b));                          \
        if (K == 20) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a##n) : "v"(b));                          \
        if (K == 21) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a2x[n]) : "v"(b2), "v"(c2));         \
        if (K == 22) asm volatile("v_fma_f32 %0, %0, %1, %2\n v_max3_f32 %0, %0, %1, %2" : "+v"(a##n) : "v"(b), "v"(c)); \
        if (K == 23) asm volatile("v_fma_f32 %0, %0, %1, %2\n v_fma_mix_f32 %0, %1, %0, %2 op_sel_hi:[1,0,0]" : "+v"(a##n) : "v"(b), "v"(c)); \
        if (K == 24) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a##n));                               \
        if (K == 25) asm volatile("v_max_f32 %0, %0, %1\n v_max3_f32 %0, %0, %1, %2" : "+v"(a##n) : "v"(b), "v"(c)); \
        if (K == 26) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a##n) : "v"(b), "v"(c));              \
        if (K == 27) asm volatile("v_cvt_f32_ubyte1 %0, %0\n v_max3_f32 %0, %0, %1, %2" : "+v"(a##n) : "v"(b), "v"(c)); \
        if (K == 28) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a##n));                                  \
        if (K == 29) asm volatile("v_cmp_le_f32 vcc, %0, %1\n v_cndmask_b32_e64 %0, 0, 1, vcc" : "+v"(a##n) : "v"(b) : "vcc");
        REP8(BODY) REP8(BODY) REP8(BODY) REP8(BODY) REP8(BODY) REP8(BODY) REP8(BODY) REP8(BODY)
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float z = 0.0f;
    for (int q = 0; q < 8; ++q) z += a2x[q].x + a2x[q].y;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + z;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
static void run(const char* name, int waves_per_simd, int cus) {
    const int blocks = cus * waves_per_simd;   // 256-thread blocks: one wave per SIMD each
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&cyc, (size_t)blocks * 8);
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, 1.0f);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long* h = (unsigned long long*)malloc((size_t)blocks * 8);
    hipMemcpy(h, cyc, (size_t)blocks * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks; ++i) mean += (double)h[i];
    mean /= blocks;
    const int per = (K == 8 || K == 12 || K == 22 || K == 23 || K == 25 || K == 27 || K == 29) ? 2 : 1;
    const double instr_per_wave = (double)ITER * 64 * per;
    // cycles per wave-instruction on one SIMD: each SIMD runs waves_per_simd waves
    printf("%-22s waves/SIMD %d: %.2f cycles per wave-instr per SIMD (in-kernel), %.3f ms, %.2f GHz-equiv\n", name,
           waves_per_simd, mean / (instr_per_wave * waves_per_simd), ms,
           instr_per_wave * waves_per_simd * 2.0 / (ms * 1e-3) / 1e9);
    free(h);
    hipFree(out);
    hipFree(cyc);
}

int main() {
    int dev = 0, cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    for (int w : {4, 8}) {
        run<0>("v_fma_f32", w, cus);
        run<13>("v_max_f32", w, cus);
        run<20>("v_mul_f32", w, cus);
        run<19>("v_and_b32", w, cus);
        run<24>("v_lshlrev_b32", w, cus);
        run<7>("v_add_u32", w, cus);
        run<1>("v_cvt_f32_ubyte1", w, cus);
        run<28>("v_cvt_f32_u32", w, cus);
        run<15>("v_cvt_f32_f16", w, cus);
        run<14>("v_fma_mix_f32", w, cus);
        run<2>("v_max3_f32", w, cus);
        run<26>("v_med3_f32", w, cus);
        run<18>("v_or3_b32", w, cus);
        run<5>("v_perm_b32", w, cus);
        run<11>("v_bfe_u32", w, cus);
        run<4>("v_mul_lo_u32", w, cus);
        run<6>("v_pk_fma_f16", w, cus);
        run<21>("v_pk_fma_f32", w, cus);
        run<16>("v_cmp_le_f32(sgpr)", w, cus);
        run<17>("v_cndmask_e64(sgpr)", w, cus);
        run<29>("v_cmp+cndmask_e64", w, cus);
        run<12>("fma+cvt_ubyte", w, cus);
        run<22>("fma+max3", w, cus);
        run<23>("fma+fma_mix", w, cus);
        run<25>("max+max3", w, cus);
        run<27>("cvt_ubyte+max3", w, cus);
        run<9>("v_rcp_f32", w, cus);
    }
    return 0;
}
