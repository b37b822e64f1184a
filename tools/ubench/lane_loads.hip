// Micro-benchmark: does a scattered global_load_dwordx4 cost the vector-memory pipeline per
// wave-instruction or per active lane?  Every wave issues K independent 16-B loads per iteration
// to random 16-B records of a table (L2 / Infinity-cache resident sizes), with only the first
// `active` lanes of each wave enabled.  Time per iteration vs active lanes answers it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void __launch_bounds__(256) loads(const float4* __restrict__ tab, uint32_t nrec, int iters, int active,
                                             float* out, int stride16, int group, int gap) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
    float4 acc = make_float4(0, 0, 0, 0);
    uint32_t r = 0;
    if (lane < (uint32_t)active) {
        for (int it = 0; it < iters; ++it) {
            float4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                // group > 1: the k-th of `group` consecutive 16-B words of one random record
                if (k % group == 0) {
                    h = h * 1664525u + 1013904223u;
                    r = (h >> 7) % nrec;
                }
                v[k] = tab[(size_t)r * stride16 + (uint32_t)(k % group) * gap];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
            }
        }
    }
    if (acc.x == 1234.5f) out[0] = acc.y + acc.z + acc.w;
}

int main(int argc, char** argv) {
    const size_t bytes = (size_t)((argc > 1 ? atof(argv[1]) : 48.0) * 1048576.0);   // table MB
    const int stride16 = argc > 2 ? atoi(argv[2]) : 1;             // record stride in 16-B units
    const int group = argc > 3 ? atoi(argv[3]) : 1;                // consecutive 16-B loads per random record
    const int gap = argc > 4 ? atoi(argv[4]) : 1;                  // 16-B units between a record's loads
    const uint32_t nrec = (uint32_t)(bytes / 16 / stride16);
    float4* tab;
    float* out;
    hipMalloc(&tab, bytes);
    hipMemset(tab, 0, bytes);
    hipMalloc(&out, 4);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;   // 8 waves / SIMD at 256 threads per block
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 200;
    for (int active : {64, 32, 16}) {
        loads<<<blocks, 256>>>(tab, nrec, 20, active, out, stride16, group, gap);
        hipEventRecord(a);
        loads<<<blocks, 256>>>(tab, nrec, iters, active, out, stride16, group, gap);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double insts = (double)blocks * 4 * iters * 4;   // wave-instructions
        const double lanes = insts * active;
        printf("gap %d group %d table %zu MB stride %d B active %2d: %.3f ms  %.1f G wave-loads/s  %.1f G lane-loads/s  %.2f TB/s useful\n",
               gap, group, bytes >> 20, stride16 * 16, active, ms, insts / ms * 1e-6, lanes / ms * 1e-6, lanes * 16 / ms * 1e-9);
    }
    return 0;
}
