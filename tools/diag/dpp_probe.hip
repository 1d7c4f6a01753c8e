// Diagnostic: what the DPP wave shifts used by device_util.hpp return on this GPU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "device_util.hpp"
using namespace sdl;
__global__ void k(uint32_t *out) {
    const uint32_t l = threadIdx.x;
    out[l] = wave_prev(l + 100);          // expect l == 0 ? 0 : l + 99
    out[64 + l] = wave_next(l + 100);     // expect l == 63 ? 0 : l + 101
    uint32_t x = (l == 50) ? 7u : 0u;     // inclusive max scan: lanes >= 50 -> 7
#define MX(a, b) ((a) > (b) ? (a) : (b))
    SDL_DPP_SCAN(x, MX);
    out[128 + l] = x;
    out[192 + l] = wave_prev(x);          // lanes >= 51 -> 7
    out[256 + l] = __shfl_up(x, 1, 64);
}
int main() {
    uint32_t *d, h[320];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    const char *names[] = {"wave_prev(l+100)", "wave_next(l+100)", "incl max scan", "wave_prev(scan)", "shfl_up(scan,1)"};
    for (int r = 0; r < 5; ++r) {
        printf("%s:", names[r]);
        for (int l = 44; l < 56; ++l) printf(" %u", h[64 * r + l]);
        printf("  | lanes 0-3: %u %u %u %u\n", h[64 * r], h[64 * r + 1], h[64 * r + 2], h[64 * r + 3]);
    }
    return 0;
}
