// Issue cost of v_mul_lo_u32 against v_add_u32 / v_mul_u32_u24 on gfx950: 8 independent chains
// per lane, 4096 steps each, one block per CU, 4 waves.  hipcc --offload-arch=gfx950 -O3 mul_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void k(uint32_t *out, uint32_t s) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7u + i + s;
    for (int it = 0; it < 4096; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) a[i] = a[i] + 0x9E3779B1u + (uint32_t)it;
            else if constexpr (OP == 1) a[i] = a[i] * 0x85EBCA6Bu + (uint32_t)it;
            else a[i] = __umul24(a[i], 0x9E3779u) + (uint32_t)it;
        }
    }
    uint32_t x = 0;
    for (int i = 0; i < 8; ++i) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 256 * 4 * 256 * sizeof(uint32_t));
    const char *names[] = {"v_add_u32 (+add)", "v_mul_lo_u32 (+add)", "v_mul_u32_u24 (+add)"};
    for (int op = 0; op < 3; ++op) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(256 * 4), dim3(256), 0, 0, d, 1u);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(256 * 4), dim3(256), 0, 0, d, 1u);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(256 * 4), dim3(256), 0, 0, d, 1u);
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        float ms;
        hipEventElapsedTime(&ms, a, b);
        // wave-instructions per SIMD: (256*4 blocks * 4 waves) / (256 CUs * 4 SIMDs) waves, each 4096*8*2 instructions
        const double winst = 4.0 * 4096 * 8 * 2;
        printf("%-24s %.3f ms  -> %.2f cycles per wave-instruction pair at 2.4 GHz\n", names[op], ms,
               ms * 1e-3 * 2.4e9 / winst * 2);
    }
    return 0;
}
