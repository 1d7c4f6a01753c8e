// device_util.hpp -- wave64 / workgroup scan helpers for gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sdl {

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Value of lane l (l wave-uniform) in every lane: v_readlane into a scalar
// register, no ds_bpermute round trip.
template <class T>
__device__ __forceinline__ T lane_bcast(T x, int l) {
    return (T)__builtin_amdgcn_readlane((int)x, l);
}

// DPP data movement for the wave scans below: lanes without a source (or rows
// outside row_mask) read 0, the identity of every scan here.
#define DPP_MOV(v, ctrl, rows) ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(v), (ctrl), (rows), 0xF, false))
// Inclusive wave64 scan of an associative op with identity 0 in six DPP steps.
#define DPP_SCAN(v, COMBINE)                          \
    do {                                                  \
        uint32_t y_;                                      \
        y_ = DPP_MOV(v, 0x111, 0xF); v = COMBINE(y_, v);  \
        y_ = DPP_MOV(v, 0x112, 0xF); v = COMBINE(y_, v);  \
        y_ = DPP_MOV(v, 0x114, 0xF); v = COMBINE(y_, v);  \
        y_ = DPP_MOV(v, 0x118, 0xF); v = COMBINE(y_, v);  \
        y_ = DPP_MOV(v, 0x142, 0xA); v = COMBINE(y_, v);  \
        y_ = DPP_MOV(v, 0x143, 0xC); v = COMBINE(y_, v);  \
    } while (0)
// The same with identity `id` (DPP lanes without a source read `id`).
#define DPP_ID(v, ctrl, rows, id) \
    ((uint32_t)__builtin_amdgcn_update_dpp((int)(id), (int)(v), (ctrl), (rows), 0xF, false))
#define DPP_SCAN_ID(v, COMBINE, id)                              \
    do {                                                             \
        uint32_t y_;                                                 \
        y_ = DPP_ID(v, 0x111, 0xF, id); v = COMBINE(y_, v);      \
        y_ = DPP_ID(v, 0x112, 0xF, id); v = COMBINE(y_, v);      \
        y_ = DPP_ID(v, 0x114, 0xF, id); v = COMBINE(y_, v);      \
        y_ = DPP_ID(v, 0x118, 0xF, id); v = COMBINE(y_, v);      \
        y_ = DPP_ID(v, 0x142, 0xA, id); v = COMBINE(y_, v);      \
        y_ = DPP_ID(v, 0x143, 0xC, id); v = COMBINE(y_, v);      \
    } while (0)
// next lane's value (lane 63: 0): DPP wave_shl:1
__device__ __forceinline__ uint32_t wave_next(uint32_t v) { return DPP_MOV(v, 0x130, 0xF); }
// previous lane's value (lane 0: 0): DPP wave_shr:1
__device__ __forceinline__ uint32_t wave_prev(uint32_t v) { return DPP_MOV(v, 0x138, 0xF); }

// Inclusive wave64 prefix sum in six DPP steps (the GFX9 wave scan): row_shr
// 1, 2, 4, 8 within each 16-lane row (lanes without a source add 0), then
// row_bcast:15 adds row 0's total to row 1 and row 2's to row 3, and
// row_bcast:31 adds lane 31's running total to rows 2 and 3.  DPP moves data
// inside the VALU -- no ds_bpermute round trip through the LDS crossbar per step.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    int v = (int)x;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return (uint32_t)v;
}

// Exclusive prefix sum over a workgroup of NT threads; *total = sum of all.
// `scratch` needs NT/64 words.  Contains two barriers.
template <int NT>
__device__ __forceinline__ uint32_t block_excl_sum(uint32_t v, uint32_t *total, uint32_t *scratch) {
    const int lane = lane_id(), wid = (int)(threadIdx.x >> 6);
    uint32_t x = wave_incl_sum(v);
    if constexpr (NT == 64) {  // one-wave blocks: the total is lane 63's (no LDS round trip);
        (void)lane;              // one barrier is kept -- callers rely on it to order their
        (void)wid;               // LDS writes before other lanes' reads
        (void)scratch;
        *total = lane_bcast(x, 63);
        __syncthreads();
        return x - v;
    }
    if (lane == 63) scratch[wid] = x;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
        uint32_t s = scratch[k];
        wbase += k < wid ? s : 0u;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return wbase + x - v;
}

// "Last set value wins" scan: a value with bit 8 set replaces the carry, 0 is
// pass-through.  Returns the exclusive scan (0 if nothing before was set).
__device__ __forceinline__ uint32_t last_set(uint32_t a, uint32_t b) { return (b & 0x100u) ? b : a; }

template <int NT>
__device__ __forceinline__ uint32_t block_excl_last_scan(uint32_t v, uint32_t *scratch) {
    const int lane = lane_id(), wid = (int)(threadIdx.x >> 6);
    uint32_t x = v;  // (0 = pass-through: the DPP scan's identity)
    DPP_SCAN(x, last_set);
    const uint32_t ex = wave_prev(x);
    if constexpr (NT == 64) {  // one wave: nothing carries in (one barrier kept, as above)
        (void)lane;
        (void)wid;
        (void)scratch;
        __syncthreads();
        return ex;
    }
    if (lane == 63) scratch[wid] = x;
    __syncthreads();
    uint32_t carry = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k)
        if (k < wid) carry = last_set(carry, scratch[k]);
    __syncthreads();
    return last_set(carry, ex);
}

}  // namespace sdl
