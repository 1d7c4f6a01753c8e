// Diagnostic: span_plane's owner scan (pipeline.hip) in isolation.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "device_util.hpp"
using namespace sdl;
__device__ __forceinline__ void st_nt(int32_t *p, int32_t v) { __builtin_nontemporal_store(v, p); }
#define SDL_MAXU(a, b) ((a) > (b) ? (a) : (b))
template <class Val, class Tail>
__device__ __forceinline__ void span_plane(int32_t *__restrict__ o, int W, int end, const uint16_t *mk, Val val,
                                           Tail tail) {
    const int lane = lane_id();
    uint32_t carry = 0;
    const bool vec = (W & 3) == 0;
    for (int b = 0; b < W; b += 256) {
        const int q0 = b + 4 * lane;
        uint32_t own[4], run = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int q = q0 + w;
            const uint32_t m = q < end ? (uint32_t)mk[q] : 0u;
            run = SDL_MAXU(run, m);
            own[w] = run;
        }
        uint32_t x = run;
        SDL_DPP_SCAN(x, SDL_MAXU);
        const uint32_t prev = wave_prev(x), last = (uint32_t)lane_bcast((int)x, 63);
        const uint32_t before = prev > carry ? prev : carry;
        carry = carry > last ? carry : last;
        int32_t v[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int q = q0 + w;
            v[w] = q < end ? val(q, SDL_MAXU(own[w], before)) : tail(q);
        }
        if (vec) {
            typedef int32_t v4i __attribute__((ext_vector_type(4)));
            if (q0 < W) __builtin_nontemporal_store(v4i{v[0], v[1], v[2], v[3]}, reinterpret_cast<v4i *>(o + q0));
        } else {
#pragma unroll
            for (int w = 0; w < 4; ++w)
                if (q0 + w < W) st_nt(o + q0 + w, v[w]);
        }
    }
}
__global__ void k(int32_t *out, int W, int end) {
    __shared__ uint16_t mk[512];
    for (int j = threadIdx.x; j < 512; j += 64) mk[j] = 0;
    __syncthreads();
    if (threadIdx.x == 0) { mk[18] = 1; mk[40] = 2; mk[201] = 3; }
    __syncthreads();
    span_plane(out, W, end, mk, [&](int q, uint32_t o) -> int32_t { return (int32_t)o; }, [&](int) -> int32_t { return -1; });
}
int main() {
    int32_t *d, h[512];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    for (int W : {128, 256, 512}) {
        (void)hipMemset(d, 0x7f, sizeof(h));
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, W, W - 5);
        if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
        printf("W=%d:", W);
        for (int q = 14; q < 46; ++q) printf(" %d", h[q]);
        printf(" | 198-206:");
        for (int q = 198; q < 207 && q < W; ++q) printf(" %d", h[q]);
        printf("\n");
    }
    return 0;
}
