// transport_frame.hip -- the Transport's batch serialisation on gfx950
// (SURVEY.md §8(f) row 1).
//
// The reference Transport pickles every finished DataSet on the CPU with
// serde_pickle::to_vec (rust/src/transport/zmq_transmit.rs:71; crate serde-pickle
// 1.1.1) and the consumer reads it with pickle.loads (python/external_dataset.py:52).
// Here the frames are written straight from the packed device row planes, so a
// batch leaves the GPU as the exact bytes the socket sends.  The encoding is the
// one oracle/orc_pickle.c restates: PROTO 3, a dict of the DataSet's fields in
// Serialize order, each a list of row lists (MARK/APPENDS batches of 1000),
// ints as BININT "J"+i32 LE, f32 labels as BINFLOAT "G"+f64 BE.
//
// Every int takes 5 bytes, so a frame's layout is closed-form (no scan): the
// host computes, per plane, the key position, the first row's offset and the
// row size; row r of a plane starts at off + r*row_bytes + 2*(r/1000).
//
// k_frame_rows: one wave per run of rows (rows of <= 1024 ids, as many as fit:
// S=128 -> 8 rows, S=512 -> 2, the 9-wide f32 labels -> 100).  The wave reads its
// rows (16-B loads, one group of 4 ids per lane), composes the 5-byte records of 4 ids as 5 dwords in
// registers, funnel-shifts them to the row's byte alignment and stores them in
// an LDS image whose alignment matches the destination's; the image then goes
// to HBM as aligned 16-B stores (byte stores only at the row's two ends).  The
// bound is HBM: 4 bytes read and 5 written per id.
// k_frame_skeleton: one lane per (frame, plane) writes the key, the list
// opener, the 1000-row APPENDS markers and the closer; lane (frame, n_planes)
// writes the PROTO/dict header and the SETITEMS/STOP trailer.
#include "common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"

namespace sdl {

namespace {

constexpr int FRAME_WAVES = 4;  // rows (waves) per block

__device__ __forceinline__ uint64_t row_pos(uint32_t r, uint32_t row_bytes) {
    return (uint64_t)r * row_bytes + 2ull * (r / 1000u);
}

// position of element k inside its row list: "](" + k records + the "e(" markers before it
__device__ __forceinline__ uint32_t elem_pos(uint32_t k, uint32_t ew) { return 2u + k * ew + 2u * (k / 1000u); }

// 20 bytes (5 dwords, little-endian byte order) at LDS byte address p
__device__ __forceinline__ void lds_put20(uint8_t *L, uint32_t p, const uint32_t d[5]) {
    const uint32_t c = p & 3u;
    uint32_t *W = reinterpret_cast<uint32_t *>(L + (p - c));
    if (c == 0) {
#pragma unroll
        for (int i = 0; i < 5; ++i) W[i] = d[i];
        return;
    }
    const uint32_t sh = 8u * c;
    // e_i = bytes [4i - c, 4i - c + 4) of the 20-byte record, for the aligned dword i
#pragma unroll
    for (int i = 1; i < 5; ++i) W[i] = (d[i] << sh) | (d[i - 1] >> (32u - sh));
    const uint32_t head = d[0] << sh, tail = d[4] >> (32u - sh);
    for (uint32_t b = c; b < 4; ++b) L[p - c + b] = (uint8_t)(head >> (8u * b));
    for (uint32_t b = 0; b < c; ++b) L[p - c + 20 + b] = (uint8_t)(tail >> (8u * b));
}

__device__ __forceinline__ void lds_put_i32(uint8_t *L, uint32_t p, uint32_t v) {
    L[p] = 'J';
    L[p + 1] = (uint8_t)v;
    L[p + 2] = (uint8_t)(v >> 8);
    L[p + 3] = (uint8_t)(v >> 16);
    L[p + 4] = (uint8_t)(v >> 24);
}

__device__ __forceinline__ void lds_put_f64(uint8_t *L, uint32_t p, float f) {
    const uint64_t u = (uint64_t)__double_as_longlong((double)f);
    L[p] = 'G';
#pragma unroll
    for (int i = 0; i < 8; ++i) L[p + 1 + i] = (uint8_t)(u >> (56 - 8 * i));
}

}  // namespace

__global__ __launch_bounds__(64 * FRAME_WAVES) void k_frame_rows(FrameParams fp, int plane0, uint32_t lds_stride) {
    extern __shared__ uint4 lds_raw[];
    const FramePlane &P = fp.plane[plane0 + (int)blockIdx.y];
    const uint32_t rpw = P.rpw;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint8_t *L = reinterpret_cast<uint8_t *>(lds_raw) + wv * lds_stride;
    // a wave writes a run of up to rpw rows of one frame; rpw divides 1000, so a run
    // never contains an APPENDS marker (those sit between runs)
    const uint64_t wpf = (P.rows_full + rpw - 1) / rpw;  // waves per frame
    const uint64_t g = (uint64_t)blockIdx.x * FRAME_WAVES + wv;
    const uint64_t f = g / wpf;
    const uint32_t r0 = (uint32_t)(g - f * wpf) * rpw;
    const bool last = f == fp.n_frames - 1;
    const uint32_t rows_f = last ? P.rows_last : P.rows_full;
    const bool valid = f < fp.n_frames && r0 < rows_f;
    const uint32_t nr = valid ? min(rpw, rows_f - r0) : 0u;
    const uint32_t rb = last ? P.row_bytes_last : P.row_bytes, W = last ? P.width_last : P.width;
    uint8_t *dst = nullptr;
    uint32_t mis = 0;
    if (valid) {
        dst = fp.out + f * fp.frame_bytes + (last ? P.off_last : P.off_full) + row_pos(r0, P.row_bytes);
        mis = (uint32_t)((uintptr_t)dst & 15u);
        const uint64_t e0 = f * P.frame_stride + (uint64_t)r0 * P.width;  // first source element of the run
        if (!P.is_f32) {
            const int32_t *src = static_cast<const int32_t *>(P.src) + e0;
            const uint32_t gpr = (W + 3u) >> 2;  // groups of 4 ids per row
            const bool v16 = ((e0 | W) & 3u) == 0;  // every row of the run starts 16-B aligned
            for (uint32_t q = lane; q < nr * gpr; q += 64u) {
                const uint32_t i = q / gpr, k0 = (q - i * gpr) * 4u;
                const uint32_t p = mis + i * rb + elem_pos(k0, 5u);
                const int32_t *s = src + (size_t)i * W;
                if (k0 + 4u <= W) {
                    uint32_t v0, v1, v2, v3;
                    if (v16) {
                        const uint4 x = *reinterpret_cast<const uint4 *>(s + k0);
                        v0 = x.x, v1 = x.y, v2 = x.z, v3 = x.w;
                    } else {
                        v0 = (uint32_t)s[k0], v1 = (uint32_t)s[k0 + 1], v2 = (uint32_t)s[k0 + 2],
                        v3 = (uint32_t)s[k0 + 3];
                    }
                    // 'J' v0 'J' v1 'J' v2 'J' v3, little-endian dwords
                    const uint32_t d[5] = {0x4Au | v0 << 8, v0 >> 24 | 0x4Au << 8 | v1 << 16,
                                           v1 >> 16 | 0x4Au << 16 | v2 << 24, v2 >> 8 | 0x4Au << 24, v3};
                    lds_put20(L, p, d);
                } else {
                    for (uint32_t k = k0; k < W; ++k) lds_put_i32(L, mis + i * rb + elem_pos(k, 5u), (uint32_t)s[k]);
                }
            }
        } else {
            const float *src = static_cast<const float *>(P.src) + e0;
            for (uint32_t q = lane; q < nr * W; q += 64u) {
                const uint32_t i = q / W, k = q - i * W;
                lds_put_f64(L, mis + i * rb + elem_pos(k, 9u), src[q]);
            }
        }
        for (uint32_t i = lane; i < nr; i += 64u) {  // list opener, inner markers, closer of each row
            uint8_t *R = L + mis + i * rb;
            R[0] = ']';
            if (W) {
                R[1] = '(';
                const uint32_t ew = P.is_f32 ? 9u : 5u;
                for (uint32_t m = 1; m * 1000u <= W; ++m) {
                    const uint32_t q = 2u + m * 1000u * ew + 2u * (m - 1u);
                    R[q] = 'e';
                    R[q + 1] = '(';
                }
                R[rb - 1] = 'e';
            }
        }
    }
    __syncthreads();
    if (valid) {
        uint8_t *A = dst - mis;  // 16-B aligned
        const uint32_t end = mis + nr * rb, nch = (end + 15u) >> 4;
        for (uint32_t c = lane; c < nch; c += 64u) {
            const uint32_t lo = c * 16u, hi = lo + 16u;
            if (lo >= mis && hi <= end) {
                // frames stream out (read next by the D2H copy, not by this pass): non-temporal
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(*reinterpret_cast<const v4u *>(L + lo), reinterpret_cast<v4u *>(A + lo));
            } else {
                const uint32_t b0 = lo > mis ? lo : mis, b1 = hi < end ? hi : end;
                for (uint32_t b = b0; b < b1; ++b) A[b] = L[b];
            }
        }
    }
}

__global__ __launch_bounds__(64) void k_frame_skeleton(FrameParams fp) {
    const uint64_t t = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    const uint32_t per = (uint32_t)fp.n_planes + 1u;
    if (t >= fp.n_frames * per) return;
    const uint64_t f = t / per;
    const uint32_t p = (uint32_t)(t - f * per);
    const bool last = f == fp.n_frames - 1;
    uint8_t *F = fp.out + f * fp.frame_bytes;
    if (p == (uint32_t)fp.n_planes) {
        F[0] = 0x80, F[1] = 3, F[2] = '}', F[3] = '(';
        const uint64_t e = last ? fp.last_frame_bytes : fp.frame_bytes;
        F[e - 2] = 'u', F[e - 1] = '.';
        return;
    }
    const FramePlane &P = fp.plane[p];
    const uint64_t off = last ? P.off_last : P.off_full;
    const uint32_t rows = last ? P.rows_last : P.rows_full;
    uint8_t *K = F + off - P.key_len;
    for (uint32_t i = 0; i < P.key_len; ++i) K[i] = P.key[i];
    if (P.flat) return;  // the value is one list, written whole by k_frame_rows
    for (uint32_t m = 1; m * 1000u <= rows; ++m) {
        uint8_t *q = F + off + (uint64_t)m * 1000u * P.row_bytes + 2ull * (m - 1u);
        q[0] = 'e', q[1] = '(';
    }
    F[off + row_pos(rows, P.row_bytes)] = 'e';
}

hipError_t launch_frames(const FrameParams &fp, hipStream_t st) {
    if (fp.n_frames == 0) return hipSuccess;
    FrameParams q = fp;
    for (int p = 0; p < q.n_planes; ++p) {
        FramePlane &P = q.plane[p];
        const uint32_t w = P.width > 0 ? P.width : 1u;
        P.rpw = 1;  // rows per wave: the largest divisor of 1000 with <= 1024 elements
        for (uint32_t d : {1000u, 500u, 250u, 200u, 125u, 100u, 50u, 40u, 25u, 20u, 10u, 8u, 5u, 4u, 2u})
            if (d * w <= 1024u) {
                P.rpw = d;
                break;
            }
        if (P.flat) P.rpw = 1;
    }
    // the row-list planes in one launch (blockIdx.y), LDS sized to their widest run; a flat
    // list (SingleClass `label`, B items in one run) in a launch of its own so its larger
    // LDS run does not cut the occupancy of the others
    auto launch = [&](int p0, int p1) -> hipError_t {
        uint32_t stride = 16;
        uint64_t max_waves = 0;
        for (int p = p0; p < p1; ++p) {
            const FramePlane &P = q.plane[p];
            const uint32_t rb = P.row_bytes > P.row_bytes_last ? P.row_bytes : P.row_bytes_last;
            const uint32_t st_p = (P.rpw * rb + 15u + 16u) & ~15u;
            stride = st_p > stride ? st_p : stride;
            const uint64_t waves = q.n_frames * ((P.rows_full + P.rpw - 1) / P.rpw);
            max_waves = waves > max_waves ? waves : max_waves;
        }
        const uint64_t nb = (max_waves + FRAME_WAVES - 1) / FRAME_WAVES;
        if ((size_t)stride * FRAME_WAVES > 160u * 1024u) return hipErrorInvalidValue;
        if (!nb || p1 <= p0) return hipSuccess;
        hipLaunchKernelGGL(k_frame_rows, dim3((unsigned)nb, (unsigned)(p1 - p0)), dim3(64 * FRAME_WAVES),
                           (size_t)stride * FRAME_WAVES, st, q, p0, stride);
        return hipGetLastError();
    };
    int p0 = 0;
    while (p0 < q.n_planes) {
        int p1 = p0 + 1;
        if (!q.plane[p0].flat)
            while (p1 < q.n_planes && !q.plane[p1].flat) ++p1;
        hipError_t e = launch(p0, p1);
        if (e != hipSuccess) return e;
        p0 = p1;
    }
    const uint64_t nt = fp.n_frames * (uint64_t)(fp.n_planes + 1);
    hipLaunchKernelGGL(k_frame_skeleton, dim3((unsigned)((nt + 63) / 64)), dim3(64), 0, st, fp);
    return hipGetLastError();
}

}  // namespace sdl
