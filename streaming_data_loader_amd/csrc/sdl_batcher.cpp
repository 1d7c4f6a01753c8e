// sdl_batcher.cpp -- C ABI of the MI355X Batcher (include/sdl_batcher.h).
//
// Host side of the drop-in for the reference's Batcher stage:
//   - sdl_batcher_create  ~ masking_runner::create_generator (masking_runner.rs:55-62)
//                           -> get_tokenizer + GenTokenizer::new (gen_batcher.rs:23-41)
//   - sdl_batcher_push    ~ Batcher::create_sync_batch (gen_batcher.rs:69-94)
//   - sdl_batcher_flush   ~ Batcher::get_working_batch (gen_batcher.rs:96-98)
// The per-record arithmetic runs on the GPU (sdl_process_device); this file
// only moves bytes and keeps GenTokenizer's VecDeque<DataSet> of batches so the
// emission cadence (at most one batch per create_sync_batch call, one flush at
// end of stream) is the reference's.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sdl_batcher.h"
#include "assets.hpp"
#include "kernels.hpp"

using namespace sdl;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) throw HipError(std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct ArgError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct CapacityError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;  // elements
    void ensure(size_t n) {
        if (n <= cap && p) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        size_t want = std::max<size_t>(n + n / 4, 64);
        HIP_TRY(hipMalloc(&p, want * sizeof(T)));
        cap = want;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

template <class T>
struct PinBuf {
    T *p = nullptr;
    size_t cap = 0;
    void ensure(size_t n) {
        if (n <= cap && p) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        size_t want = std::max<size_t>(n + n / 4, 64);
        HIP_TRY(hipHostMalloc(&p, want * sizeof(T), hipHostMallocDefault));
        cap = want;
    }
    ~PinBuf() {
        if (p) (void)hipHostFree(p);
    }
};

// Pinned blocks holding finished batches, recycled: the device rows are copied
// straight into them (one D2H per plane per batch segment, no host re-copy),
// and a block returns here when its batch is released -- possibly after the
// handle is gone, so batches share ownership of the pool.
struct BatchPool {
    struct Block {
        void *host, *dev;  // dev: the device-mapped address (k_rows_to_host writes there)
    };
    std::mutex mu;
    std::vector<Block> free_;
    size_t bytes;
    size_t fresh = 0;  // blocks allocated so far
    explicit BatchPool(size_t b) : bytes(b) {}
    Block get() {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!free_.empty()) {
                const Block b = free_.back();
                free_.pop_back();
                return b;
            }
        }
        Block b{nullptr, nullptr};
        HIP_TRY(hipHostMalloc(&b.host, bytes, hipHostMallocDefault));
        if (hipHostGetDevicePointer(&b.dev, b.host, 0) != hipSuccess) {
            (void)hipHostFree(b.host);
            throw HipError("hipHostGetDevicePointer failed");
        }
        std::lock_guard<std::mutex> g(mu);
        ++fresh;
        return b;
    }
    void put(const Block &b) {
        std::lock_guard<std::mutex> g(mu);
        free_.push_back(b);
    }
    ~BatchPool() {
        for (const Block &b : free_) (void)hipHostFree(b.host);
    }
};

// One DataSet being filled (BertData / GptData), planes in one pinned block.
// Rows [rows, B) get the initial values of BatchConfig::create_vector
// (batcher.rs:17-22) and BertData::new (bert_data.rs:27-38) when the batch is
// handed out (init_tail): filled rows are written once, by the D2H.
struct HostBatch {
    std::shared_ptr<BatchPool> pool;
    void *block = nullptr;
    char *dev = nullptr;  // the block's device-mapped address (k_rows_to_host writes there)
    int32_t *ids = nullptr, *am = nullptr, *tt = nullptr, *lab = nullptr;
    float *f32 = nullptr;  // MultiLabel: [B, number_labels]
    int rows = 0;
    int B, S, LW;
    static size_t block_bytes(int B, int S, int LW, bool with_tt) {
        return 4 * (size_t)B * ((size_t)S * (with_tt ? 3 : 2) + (size_t)LW);
    }
    HostBatch(std::shared_ptr<BatchPool> pl, int B_, int S_, int LW_, bool with_tt, bool multi)
        : pool(std::move(pl)), B(B_), S(S_), LW(LW_) {
        const BatchPool::Block bl = pool->get();
        block = bl.host;
        dev = static_cast<char *>(bl.dev);
        int32_t *q = static_cast<int32_t *>(block);
        const size_t BS = (size_t)B * S;
        ids = q;
        am = q + BS;
        q += 2 * BS;
        if (with_tt) {
            tt = q;
            q += BS;
        }
        if (multi) f32 = reinterpret_cast<float *>(q);
        else lab = q;
    }
    template <class T>
    int32_t *on_dev(T *host_plane) const {
        return host_plane ? reinterpret_cast<int32_t *>(dev + ((char *)host_plane - (char *)block)) : nullptr;
    }
    HostBatch(const HostBatch &) = delete;
    HostBatch &operator=(const HostBatch &) = delete;
    void init_tail() {
        const size_t r0 = (size_t)rows, r1 = (size_t)B;
        if (r0 >= r1) return;
        std::fill(ids + r0 * S, ids + r1 * S, 0);
        std::fill(am + r0 * S, am + r1 * S, 1);
        if (tt) std::fill(tt + r0 * S, tt + r1 * S, 0);
        if (lab) std::fill(lab + r0 * LW, lab + r1 * LW, -100);
        if (f32) std::fill(f32 + r0 * LW, f32 + r1 * LW, 0.f);
    }
    ~HostBatch() { pool->put(BatchPool::Block{block, dev}); }
};

// SDL_HOST_TIMING=1: wall-clock split of the host path on stderr (diagnostic)
struct HostClock {
    bool on;
    std::chrono::steady_clock::time_point t;
    std::string s;
    HostClock() : on(std::getenv("SDL_HOST_TIMING") != nullptr), t(std::chrono::steady_clock::now()) {}
    void lap(const char *name) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        s += std::string(" ") + name + "=" +
             std::to_string(std::chrono::duration<double, std::milli>(n - t).count()) + "ms";
        t = n;
    }
    void report(int64_t N, size_t segs, size_t fresh) const {
        if (on)
            fprintf(stderr, "[host] %lld B, %zu segments, %zu pinned blocks so far:%s\n", (long long)N, segs, fresh,
                    s.c_str());
    }
};

// memcpy of a large host buffer on several threads (pageable -> pinned staging)
void par_copy(void *dst, const void *src, size_t n) {
    const size_t kMin = (size_t)8 << 20;
    unsigned T = std::thread::hardware_concurrency();
    T = T < 1 ? 1 : T > 8 ? 8 : T;
    if (n < kMin || T == 1) {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t per = (n / T + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    for (unsigned t = 1; t < T; ++t) {
        const size_t a = per * t;
        if (a >= n) break;
        const size_t b = std::min(n, a + per);
        th.emplace_back([=] { std::memcpy((char *)dst + a, (const char *)src + a, b - a); });
    }
    std::memcpy(dst, src, std::min(n, per));
    for (auto &x : th) x.join();
}

const char *kStageNames[] = {"chunk_ranges", "tokenize", "scan_chunks", "compact_tokens", "records", "scan_rows", "rows"};
constexpr int kStages = 7;
// pipelined segments: the tokenize launches, then the downstream work left after the last one
const char *kPipedStageNames[] = {"chunk_ranges", "tokenize", "downstream_tail"};
// segments per call (SDL_SEGMENTS) and the fewest 1 KiB chunks a pipelined
// segment holds (SDL_SEG_MIN_CHUNKS, default 16 MiB of text); read when a
// handle is created
int env_int(const char *name, int dflt) {
    const char *e = std::getenv(name);
    return e ? std::max(1, std::atoi(e)) : dflt;
}
// the same for switches and values where 0 means something (env_int reads "0" as 1)
int env_int0(const char *name, int dflt) {
    const char *e = std::getenv(name);
    return e ? std::max(0, std::atoi(e)) : dflt;
}

}  // namespace

struct sdl_batcher {
    sdl_config cfg{};
    RowParams P{};
    HostTokenizer tok;
    DevTok dt{};
    hipStream_t stream = nullptr;
    int device = 0;

    // device-resident tokenizer tables
    DevBuf<uint16_t> d_upage;
    DevBuf<uint32_t> d_uentry, d_ubmp;
    DevBuf<uint8_t> d_upool, d_vpool;
    DevBuf<VSlot> d_slots, d_wslots;
    DevBuf<int32_t> d_ascii_id;
    DevBuf<uint8_t> d_wp_lens;
    DevBuf<uint16_t> d_gpage, d_byte_id;
    DevBuf<uint8_t> d_gblock;
    DevBuf<MSlot> d_mslots;
    // unigram (t5)
    DevBuf<double> d_uscore;
    DevBuf<uint16_t> d_wres, d_cpage;
    DevBuf<uint8_t> d_upfx;
    DevBuf<uint2> d_cent, d_cbmp;
    DevBuf<float> d_uscore32;
    DevBuf<uint8_t> d_tnorm;
    DevBuf<uint32_t> d_trie;
    DevBuf<int32_t> d_extra;
    DevBuf<double> d_zig;  // span rng_mode 1: ZIG_NORM_X then ZIG_NORM_F (257 each)

    // per-call workspace
    DevBuf<uint32_t> ranges, tokc, chunk_cnt, chunk_off, rec_local, tok_ids, rec_tok, rec_cnt, rec_rows, row_off,
        row_rec, scan_tmp;
    DevBuf<int32_t> o_ids, o_am, o_tt, o_lab;
    // rng_mode 1: the swap indices and mask bits of the rows walked beside the tokenizer on stream2
    // (k_mask_rand_rec: chunk 0 of every record, chunk 1 of the spec_list records); k_rows walks the
    // rest in a second pass
    DevBuf<uint16_t> mask_j0;
    DevBuf<uint32_t> mask_bits0, spec_list, spec_pos;
    hipEvent_t rand_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    DevBuf<float> o_f32;
    DevBuf<uint32_t> lab_err;
    // byte-level BPE long pieces
    DevBuf<uint32_t> long_count, bpe_err, chunk_ent;
    DevBuf<BpeLong> long_list;
    DevBuf<uint16_t> long_scratch;
    // unigram long items
    DevBuf<uint32_t> uni_counters, uni_pool, uni_err, span_err;
    // span rows in two phases: per-row pass plans, row meta, overflow rows
    DevBuf<uint2> span_tab, span_meta;
    DevBuf<uint32_t> span_ovf;
    bool span_two_phase = env_int0("SDL_SPAN_TWO_PHASE", 0) != 0;
    // rng_mode 1: chunk-0 rows walked beside the tokenizer (0: every row by its k_rows wave)
    bool rand_rec0 = env_int0("SDL_RAND_REC0", 1) != 0;
    // ... and chunk 1 of records of >= (S - frame + 1) / rho bytes (WordPiece/BPE give ~0.2-0.3 ids
    // per byte; SDL_RAND_SPEC_RHO_PCT=0: chunk 0 only)
    double rand_spec_rho = env_int0("SDL_RAND_SPEC_RHO_PCT", 25) / 100.0;
    // test hook: clamp the Unigram long-item list (0 = its N / 8 + chunks bound), so the capacity
    // flag can be raised through every path that reports it
    uint32_t uni_item_cap = (uint32_t)std::max(0, env_int0("SDL_UNI_ITEM_CAP", 0));
    // JsonText provider step (sdl_json_text_device)
    DevBuf<uint32_t> j_cnt, j_base, j_nl, j_len, j_rec, j_toff, j_ridx, j_inv, j_tail;
    DevBuf<uint2> j_span;
    DevBuf<uint8_t> j_text;
    DevBuf<uint64_t> j_off;
    // gzip inflate provider step (sdl_gzip_inflate_device)
    DevBuf<uint32_t> z_size, z_off, z_tcrc, z_bad;
    DevBuf<uint64_t> z_from, z_mend;  // (sdl_gzip_inflate_first_device) candidate search start, member ends
    DevBuf<int32_t> z_status;
    DevBuf<unsigned long long> z_total;
    DevBuf<uint8_t> z_out;
    // ... large members in chunks (inflate_chunked)
    DevBuf<uint64_t> zc_nominal, zc_found, zc_start, zc_hdr, zc_end, zc_endhdr, zc_pos;
    DevBuf<uint32_t> zc_list, zc_tgt, zc_next, zc_len, zc_flags, zc_order, zc_crc, zc_shift, zc_stats;
    DevBuf<int32_t> zc_status, zc_rstatus;
    DevBuf<uint16_t> zc_slots;
    DevBuf<uint8_t> zc_windows, zc_gwin;
    DevBuf<uint16_t> zc_gmaps;
    // Transport frames (sdl_pickle_frames_device)
    DevBuf<uint8_t> f_out, f_out2;
    DevBuf<uint8_t> *f_target = &f_out;  // where the next frames go
    uint8_t *f_dest = nullptr;           // ... or here (device-visible, e.g. mapped pinned host memory)
    size_t f_dest_cap = 0;
    bool f_dry = false;                  // lay the frames out, launch nothing
    // sdl_json_to_frames: input slots, the rows carried between chunks, streams/events
    DevBuf<uint8_t> x_json[2], x_frames[2];
    PinBuf<uint8_t> x_pin_in[2], x_pin_out[2];
    DevBuf<int32_t> x_ids[2], x_am[2], x_tt[2], x_lab[2];
    hipStream_t x_in = nullptr, x_out = nullptr;
    hipEvent_t x_ev[8] = {};
    std::vector<hipEvent_t> x_in_ev;  // json_to_frames, pinned input: chunk k's H2D done
    DevBuf<uint8_t> x_json_all;       // ... every chunk, 32 zero bytes after each
    DevBuf<uint4> uni_items, uni_items2, uni_huge;
    DevBuf<uint8_t> uni_scratch;

    // host streaming path (GenTokenizer.store + emitted batches)
    std::deque<HostBatch *> store;
    std::deque<HostBatch *> outbox;
    PinBuf<uint8_t> pin_blob;  // staged call input: text | offsets | labels | label offsets
    // a small push's H2D done by k_chunk_ranges from the mapped blob (process_host -> run_device)
    struct FusedH2D {
        const void *src = nullptr;
        void *dst = nullptr;
        size_t bytes = 0;
        const uint64_t *h_off = nullptr;  // the offsets in the mapped blob
    } fused_h2d;
    void *blob_dev = nullptr;               // pin_blob's device address ...
    const uint8_t *blob_dev_host = nullptr;  // ... for this host buffer
    DevBuf<uint8_t> h2d_blob;
    PinBuf<uint32_t> pin_u32;
    PinBuf<uint32_t> pin_stat;  // direct pass: row offsets + error words (mapped)
    uint32_t *stat_dev = nullptr;
    HostBatch *spare = nullptr;  // direct pass: the next batch, allocated ahead
    DirectDst fuse_dd{};          // ... its destinations, for run_device's fused small path
    uint32_t *fuse_stat = nullptr;
    bool fused_done = false;      // run_device wrote the direct rows and the row offsets
    PinBuf<RowSeg> seg_pin;
    DevBuf<RowSeg> seg_dev;
    void ensure_stat(size_t n) {
        const uint32_t *was = pin_stat.p;
        pin_stat.ensure(n);
        if (pin_stat.p != was || !stat_dev) {
            void *d = nullptr;
            HIP_TRY(hipHostGetDevicePointer(&d, pin_stat.p, 0));
            stat_dev = static_cast<uint32_t *>(d);
        }
    }
    uint32_t pin_u32_err = 0;
    uint32_t pin_u32_2[2] = {0, 0};
    uint64_t n_records = 0;
    int64_t first_override = -1;  // sdl_multi: the global index of the next call's first record

    bool profiling = false;
    hipEvent_t ev[kStages + 1] = {};
    float stage_ms[kStages] = {};
    int n_stages = kStages;
    const char **stage_names = kStageNames;
    // pipelined segments: second stream, cross-stream events, record bounds
    hipStream_t stream2 = nullptr;
    hipStream_t stream_u = nullptr;  // unigram: the wide-job Viterbi and the long items beside the narrow jobs
    hipEvent_t uni_ev[2] = {nullptr, nullptr};
    std::vector<hipEvent_t> pipe_ev;
    DevBuf<uint32_t> seg_rb;
    int seg_target = env_int("SDL_SEGMENTS", 1);
    int64_t seg_min_chunks = env_int("SDL_SEG_MIN_CHUNKS", 16384);

#ifdef SDL_STAMPS
    ~sdl_batcher() {
        print_phase_cycles();
        print_uni_cycles();
        print_long_cycles();
        print_vit_cycles();
        print_bpe_cycles();
        if (uni_counters.p) {
            uint32_t c[4] = {0, 0, 0, 0}, e = 0;
            if (hipMemcpy(c, uni_counters.p, 16, hipMemcpyDeviceToHost) == hipSuccess &&
                hipMemcpy(&e, uni_err.p, 4, hipMemcpyDeviceToHost) == hipSuccess)
                fprintf(stderr, "[uni] long items %u, pool words %u, huge %u, err %u\n", c[0], c[2], c[3], e);
        }
        cleanup();
    }
    void cleanup() {
#else
    ~sdl_batcher() {
#endif
        for (auto *b : store) delete b;
        for (auto *b : outbox) delete b;
        delete spare;
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto &e : pipe_ev) (void)hipEventDestroy(e);
        for (auto &e : rand_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto &e : x_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto &e : x_in_ev) (void)hipEventDestroy(e);
        if (x_in) (void)hipStreamDestroy(x_in);
        if (x_out) (void)hipStreamDestroy(x_out);
        if (stream2) (void)hipStreamDestroy(stream2);
        for (auto &e : uni_ev)
            if (e) (void)hipEventDestroy(e);
        if (stream_u) (void)hipStreamDestroy(stream_u);
        if (stream) (void)hipStreamDestroy(stream);
    }

    bool multi() const { return P.task == SDL_TASK_MULTI_LABEL; }
    bool single() const { return P.task == SDL_TASK_SINGLE_CLASS; }
    bool simple() const { return multi() || single(); }  // SimpleBatcher (simple_batcher.rs)
    bool span() const { return P.task == SDL_TASK_SPAN; }
    bool with_tt() const { return P.task == SDL_TASK_MLM || simple(); }

    std::shared_ptr<BatchPool> pool;
    HostBatch *new_batch() {
        if (!pool) pool = std::make_shared<BatchPool>(HostBatch::block_bytes(P.B, P.S, P.label_width, with_tt()));
        return new HostBatch(pool, P.B, P.S, P.label_width, with_tt(), multi());
    }

    int64_t rows_capacity(int64_t N, int64_t R) const {
        // rows <= sum_r ceil((ids_r + frame) / S) with ids_r <= bytes_r
        const int64_t F = P.n_pre + P.n_post;
        // ids <= bytes (WordPiece, BPE); Unigram: <= 2 * bytes + the pool slack
        const int64_t ids = dt.kind == TOK_UNIGRAM ? 2 * N + 1024 * 1024 : N;
        int64_t cap = P.chunk ? (ids + R * (F + P.S - 1)) / P.S + 1 : R;
        return (cap + P.B - 1) / P.B * P.B;
    }

    void run_device(const uint8_t *d_text, int64_t N, const uint64_t *d_off, int64_t R, uint64_t first_record,
                    hipStream_t st, const uint32_t *d_labels = nullptr, const uint64_t *d_label_off = nullptr) {
        const int64_t n_chunks = (N + CHUNK - 1) / CHUNK;
        const int64_t rows_cap = rows_capacity(N, R);
        ranges.ensure((size_t)std::max<int64_t>(n_chunks, 1) * 3);
        tokc.ensure((size_t)std::max<int64_t>(n_chunks, 1) * (dt.kind == TOK_UNIGRAM ? UNI_STAGE : STAGE));
        chunk_cnt.ensure((size_t)n_chunks + 1);
        chunk_off.ensure((size_t)n_chunks + 1);
        rec_local.ensure((size_t)R + 1);
        // ids <= text bytes for WordPiece/BPE; Unigram adds a "▁" piece per word
        // and expanding normalizations: bound by the chunk entries + the pool
        tok_ids.ensure(dt.kind == TOK_UNIGRAM ? (size_t)2 * N + 1024 * 1024 + 1 : (size_t)N + 1);
        rec_tok.ensure((size_t)R + 1);
        rec_cnt.ensure((size_t)R + 1);
        rec_rows.ensure((size_t)R + 1);
        row_off.ensure((size_t)R + 1);
        scan_tmp.ensure((size_t)std::max(scan_tmp_words(n_chunks), scan_tmp_words(R)) + 1);
        const size_t plane = (size_t)std::max<int64_t>(rows_cap, 1) * P.S;
        o_ids.ensure(plane);
        o_am.ensure(plane);
        if (with_tt()) o_tt.ensure(plane);
        if (multi()) {
            o_f32.ensure((size_t)std::max<int64_t>(rows_cap, 1) * P.label_width);
            lab_err.ensure(1);
        } else {
            o_lab.ensure((size_t)std::max<int64_t>(rows_cap, 1) * P.label_width);
            if (single()) lab_err.ensure(1);
        }
        row_rec.ensure((size_t)std::max<int64_t>(rows_cap, 1));
        const bool rm1 = P.task == SDL_TASK_MLM && P.rng_mode == 1;
        const int mask_w = (P.S + 31) / 32;

        RowParams p = P;
        p.first_record = first_record;
        p.mask_w = mask_w;
        p.mask_bits0 = nullptr;
        p.mask_spos = nullptr;
        p.mask_off = d_off;
        p.mask_R = R;
        p.mask_spec1 = 0;
        const bool bpe = dt.kind == TOK_BYTE_BPE;
        const bool uni = dt.kind == TOK_UNIGRAM;
        // Pipelined segments (WordPiece): the tokenize launches of the chunk
        // ranges run back to back on `st` while a second stream runs each
        // finished segment's scans, compaction, records and rows -- the
        // latency-bound tokenizer and the write-bound row assembly overlap.
        // The other tokenizers finish long items in follow-up kernels over the
        // whole call, so they run as one segment.
        SegChunks sc{};
        sc.K = 1;
        if (!bpe && !uni && seg_target > 1 && n_chunks >= 2 * seg_min_chunks) {
            sc.K = (int)std::min<int64_t>(seg_target, n_chunks / seg_min_chunks);
            sc.K = std::min(sc.K, MAX_SEGMENTS);
        }
        for (int k = 0; k <= sc.K; ++k) sc.cb[k] = n_chunks * k / sc.K;
        seg_rb.ensure(MAX_SEGMENTS + 2);
        const bool piped = sc.K > 1;
        n_stages = piped ? 3 : kStages;
        stage_names = piped ? kPipedStageNames : kStageNames;
        auto mark = [&](int i) {
            if (profiling) HIP_TRY(hipEventRecord(ev[i], st));
        };
        const bool small = !piped && !profiling && n_chunks <= SMALL_CHUNKS && R <= 8192;
        mark(0);
        // (one segment: k_chunk_ranges also writes its record bounds and zeroes the label error word)
        const bool fold = sc.K == 1 && n_chunks > 0;
        // (a small push's H2D rides along: fused_h2d, set by process_host)
        HIP_TRY(launch_chunk_ranges(fused_h2d.bytes ? fused_h2d.h_off : d_off, R, N, ranges.p, st,
                                    fold ? seg_rb.p : nullptr, fold && (multi() || single()) ? lab_err.p : nullptr,
                                    fused_h2d.src, fused_h2d.dst, fused_h2d.bytes));
        fused_h2d = FusedH2D{};
        // rng_mode 1: a row's masks depend on (seed, record, chunk) alone, so the rows known before
        // tokenizing -- chunk 0 of every record, chunk 1 of records long enough to need one at
        // <= rand_spec_rho ids per byte -- are walked, and their mask bits made, on stream2 beside
        // the tokenizer (queued after k_chunk_ranges: launched first, their long waves held it back
        // 0.12 ms); k_rows waits for them.  Rows past the guess take the late path (correct either way).
        const bool rec0 = rm1 && !piped && !small && R > 0 && rand_rec0;
        if (rec0) {
            const int64_t F = P.n_pre + P.n_post;
            p.mask_spec1 = P.chunk && rand_spec_rho > 0 ? (int64_t)((double)(P.S - F + 1) / rand_spec_rho) : 0;
            // chunk-1 slots: the records of >= mask_spec1 bytes, at most N / mask_spec1 of them
            const int64_t ns = R + (p.mask_spec1 > 0 ? std::min<int64_t>(R, N / p.mask_spec1 + 1) : 0);
            mask_j0.ensure((size_t)ns * (size_t)P.S);
            mask_bits0.ensure((size_t)ns * (size_t)mask_w);
            spec_list.ensure((size_t)R + 1);
            spec_pos.ensure((size_t)R + 1);
            p.mask_spos = spec_pos.p;
            ensure_stream2();
            for (auto &e : rand_ev)
                if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            HIP_TRY(hipEventRecord(rand_ev[0], st));  // (the last call's rows have read mask_bits0)
            HIP_TRY(hipStreamWaitEvent(stream2, rand_ev[0], 0));
            p.mask_bits0 = mask_bits0.p;
            HIP_TRY(launch_mask_rand_rec(p, spec_list.p, spec_pos.p, mask_j0.p, mask_bits0.p, stream2));
            HIP_TRY(hipEventRecord(rand_ev[1], stream2));
        }
        if (!fold) HIP_TRY(launch_seg_bounds(ranges.p, sc, R, seg_rb.p, st));
        if (!fold && (multi() || single())) HIP_TRY(hipMemsetAsync(lab_err.p, 0, 4, st));
        mark(1);
        RowOut out{o_ids.p, o_am.p, with_tt() ? o_tt.p : nullptr, multi() ? nullptr : o_lab.p,
                   multi() ? o_f32.p : nullptr, DirectDst{}};
        // a small mlm / clm push with its host batches ready (process_host): k_rows writes them
        // and k_downstream_small the row offsets -- no k_rows_direct launch
        fused_done = small && fuse_stat && (P.task == SDL_TASK_MLM || P.task == SDL_TASK_CLM);
        if (fused_done) out.direct = fuse_dd;
        // everything after the tokenizer, for segment k, on stream s
        auto small_down = [&]() {
            SmallDown d{tokc.p, chunk_cnt.p, chunk_off.p, tok_ids.p,
                        uni ? uni_counters.p : bpe ? long_count.p : nullptr,
                        uni || bpe ? chunk_ent.p : nullptr, bpe ? long_list.p : nullptr,
                        bpe ? long_scratch.p : nullptr, uni ? uni_pool.p : nullptr,
                        uni ? (int64_t)UNI_STAGE : (int64_t)STAGE, rec_local.p, rec_tok.p, rec_cnt.p,
                        rec_rows.p, row_off.p, row_rec.p, fused_done ? fuse_stat : nullptr,
                        uni ? uni_err.p : nullptr, 0, out};
            // mlm (Philox) / clm rows in the same workgroup, no k_rows launch
            d.rows = fused_done && !rm1 ? 1 : 0;
            return d;
        };
        auto downstream = [&](int k, hipStream_t s) {
            const SegSel sel{seg_rb.p, k, k == sc.K - 1 ? 1 : 0};
            const int64_t ca = sc.cb[k], cz = sc.cb[k + 1];
            bool rows_done = false;
            if (small) {  // one launch for the five below
                const SmallDown d = small_down();
                rows_done = d.rows != 0;
                HIP_TRY(launch_downstream_small(d, p, d_off, R, N, s));
            } else {
            if (!piped) mark(2);
            HIP_TRY(launch_exclusive_scan(chunk_cnt.p + ca, chunk_off.p + ca, cz - ca, scan_tmp.p, s,
                                          k > 0 ? chunk_off.p + ca : nullptr));
            if (!piped) mark(3);
            if (uni)
                HIP_TRY(launch_compact_tokens(tokc.p, chunk_cnt.p, chunk_off.p, n_chunks, tok_ids.p, uni_counters.p,
                                              chunk_ent.p, nullptr, nullptr, s, uni_pool.p, UNI_STAGE));
            else if (bpe)
                HIP_TRY(launch_compact_tokens(tokc.p, chunk_cnt.p, chunk_off.p, n_chunks, tok_ids.p, long_count.p,
                                              chunk_ent.p, long_list.p, long_scratch.p, s));
            else
                HIP_TRY(launch_compact_tokens(tokc.p + ca * STAGE, chunk_cnt.p + ca, chunk_off.p + ca, cz - ca,
                                              tok_ids.p, nullptr, nullptr, nullptr, nullptr, s));
            if (!piped) mark(4);
            HIP_TRY(launch_records(p, d_off, R, N, chunk_off.p, n_chunks, rec_local.p, rec_tok.p, rec_cnt.p, rec_rows.p,
                                   sel, s));
            if (!piped) mark(5);
            if (piped) HIP_TRY(launch_scan_range(rec_rows.p, row_off.p, seg_rb.p, k, s));
            else HIP_TRY(launch_exclusive_scan(rec_rows.p, row_off.p, R, scan_tmp.p, s));
            HIP_TRY(launch_row_map(row_off.p, R, row_rec.p, sel, s));
            }
            if (!piped) mark(6);
            if (span()) {
                span_err.ensure(1);
                SpanPlan pl{};
                const bool two_phase = span_two_phase;
                if (two_phase) {
                    pl.capr = P.label_width / 2 + 2;
                    span_tab.ensure((size_t)std::max<int64_t>(rows_cap, 1) * (size_t)pl.capr);
                    span_meta.ensure((size_t)std::max<int64_t>(rows_cap, 1));
                    span_ovf.ensure((size_t)std::max<int64_t>(rows_cap, 1) + 1);
                    pl.tab = span_tab.p;
                    pl.meta = span_meta.p;
                    pl.ovf_n = span_ovf.p;
                    pl.ovf_list = span_ovf.p + 1;
                }
                HIP_TRY(launch_rows_span(p, tok_ids.p, rec_tok.p, rec_cnt.p, row_off.p, row_rec.p, sel, rows_cap, out,
                                         span_err.p, s, two_phase ? &pl : nullptr));
            } else {
                // rng_mode 1: k_rows waits for the rows walked beside the tokenizer and walks the rest
                // (and walks the rows past the guess in a second pass)
                if (rm1 && rec0) {
                    HIP_TRY(hipStreamWaitEvent(s, rand_ev[1], 0));
                    HIP_TRY(launch_rows(p, tok_ids.p, rec_tok.p, rec_cnt.p, row_off.p, row_rec.p, sel, rows_cap, out, s));
                } else if (!rows_done) {
                    HIP_TRY(launch_rows(p, tok_ids.p, rec_tok.p, rec_cnt.p, row_off.p, row_rec.p, sel, rows_cap, out, s));
                }
            }
            if (multi())
                HIP_TRY(launch_multi_labels(d_labels, d_label_off, row_rec.p, row_off.p, sel, rows_cap, P.B,
                                            P.label_width, o_f32.p, lab_err.p, s));
            else if (single())
                HIP_TRY(launch_single_labels(d_labels, d_label_off, row_rec.p, row_off.p, sel, rows_cap, P.B, o_lab.p,
                                             lab_err.p, s));
        };
        if (uni) {
            // long items: words > UNI_WMAX bytes (<= N / 25), one per chunk past
            // its window, and medium words whose normalization overflows the
            // chunk's arena: N / 8 + n_chunks bounds every realistic text (an
            // overflow is flagged in d_tokenize_errors); their ids go to the pool
            // long items: one wave each; 256 CUs x 9 resident (k_unigram_long<20>: 17 KB of LDS, 154 VGPRs)
            const int lane_blocks = 2304, huge_blocks = 8;
            uni_counters.ensure(8);
            uni_err.ensure(1);
            uni_items.ensure((size_t)(N / 8 + n_chunks + 64));
            uni_items2.ensure((size_t)(N / 64 + 64));
            uni_huge.ensure((size_t)(N / 256 + 64));
            uni_pool.ensure((size_t)N + 1024 * 1024);
            uni_scratch.ensure(unigram_scratch_bytes(lane_blocks, huge_blocks));
            chunk_ent.ensure((size_t)n_chunks + 1);
            uint32_t item_cap = (uint32_t)std::min<size_t>(uni_items.cap, 0xFFFFFFFFu);
            if (uni_item_cap) item_cap = std::min(item_cap, uni_item_cap);
            if (!stream_u) {
                HIP_TRY(hipStreamCreateWithFlags(&stream_u, hipStreamNonBlocking));
                for (auto &e : uni_ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            }
            UniWork W{uni_counters.p, uni_items.p, item_cap, uni_pool.p,
                      (uint32_t)std::min<size_t>(uni_pool.cap, 0x3FFFFFFF), uni_huge.p, (uint32_t)uni_huge.cap,
                      uni_items2.p, (uint32_t)uni_items2.cap, uni_scratch.p, lane_blocks, huge_blocks, uni_err.p,
                      stream_u, uni_ev[0], uni_ev[1]};
            HIP_TRY(launch_unigram_chunks(dt, d_text, N, d_off, R, ranges.p, tokc.p, chunk_cnt.p, chunk_ent.p,
                                          rec_local.p, W, st));
            downstream(0, st);
        } else if (bpe) {
            // long pieces are > 64 bytes or run past their chunk's window (<= 1 per chunk)
            const uint32_t cap = (uint32_t)(N / 64 + n_chunks + 1);
            long_count.ensure(2);  // (count, k_bpe_long cursor)
            bpe_err.ensure(1);
            long_list.ensure(cap);
            long_scratch.ensure((size_t)N + 64);
            chunk_ent.ensure((size_t)n_chunks + 1);
            HIP_TRY(launch_bpe_chunks(dt, d_text, N, d_off, R, ranges.p, tokc.p, chunk_cnt.p, chunk_ent.p,
                                      rec_local.p, long_count.p, long_list.p, cap, long_scratch.p, bpe_err.p, st));
            downstream(0, st);
        } else if (!piped) {
            HIP_TRY(launch_wordpiece_chunks(dt, d_text, N, d_off, R, ranges.p, tokc.p, chunk_cnt.p, rec_local.p, st, 0,
                                            -1));
            downstream(0, st);
        } else {
            ensure_pipe_events(sc.K);
            for (int k = 0; k < sc.K; ++k) {
                HIP_TRY(launch_wordpiece_chunks(dt, d_text, N, d_off, R, ranges.p, tokc.p, chunk_cnt.p, rec_local.p, st,
                                                sc.cb[k], sc.cb[k + 1]));
                HIP_TRY(hipEventRecord(pipe_ev[k], st));
                HIP_TRY(hipStreamWaitEvent(stream2, pipe_ev[k], 0));
                downstream(k, stream2);
            }
            mark(2);
            HIP_TRY(hipEventRecord(pipe_ev[sc.K], stream2));
            HIP_TRY(hipStreamWaitEvent(st, pipe_ev[sc.K], 0));  // the caller's stream sees every row
        }
        mark(piped ? 3 : 7);
        last_rows_cap = rows_cap;
        last_R = R;
        last_segments = sc.K;
    }
    void ensure_pipe_events(int K) {
        while ((int)pipe_ev.size() < K + 1) {
            hipEvent_t e;
            HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            pipe_ev.push_back(e);
        }
        ensure_stream2();
    }
    // stream2 runs background work (rng_mode 1 mask walks, pipelined segments) at the lowest
    // priority, so the dispatcher hands CUs to the handle's stream first
    void ensure_stream2() {
        if (stream2) return;
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = 0;
        HIP_TRY(hipStreamCreateWithPriority(&stream2, hipStreamNonBlocking, least));
    }
    int64_t last_segments = 1;
    int64_t last_rows_cap = 0, last_R = 0;

    // H2D a host arena, run the device path, bring back the rows; then play
    // GenTokenizer's queue over the per-record row counts.
    void process_host(const uint8_t *arena, const uint64_t *offsets, int64_t R, const uint32_t *labels,
                      const uint64_t *label_off) {
        const int64_t N = (int64_t)offsets[R];
        // one pinned staging blob, one H2D: text | offsets | labels | label offsets
        const bool with_labels = simple() && labels && label_off;  // validated by the caller
        const uint64_t L = with_labels ? label_off[R] - label_off[0] : 0;
        auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t x_off = up((size_t)N + 16), x_lab = up(x_off + 8 * (size_t)(R + 1)),
                     x_loff = up(x_lab + 4 * (size_t)L + 4), blob = x_loff + 8 * (size_t)(R + 1);
        pin_blob.ensure(blob + 16);  // (+16: k_chunk_ranges copies whole 16-B units)
        h2d_blob.ensure(blob + 16);
        HostClock hc;
        par_copy(pin_blob.p, arena, (size_t)N);
        hc.lap("stage");
        std::memcpy(pin_blob.p + x_off, offsets, sizeof(uint64_t) * (size_t)(R + 1));
        const uint32_t *d_labels = nullptr;
        const uint64_t *d_label_off = nullptr;
        size_t h2d_bytes = x_off + 8 * (size_t)(R + 1);
        if (with_labels) {  // Label::Multi indices / Label::Single
            std::memcpy(pin_blob.p + x_lab, labels, sizeof(uint32_t) * (size_t)L);
            uint64_t *lo = reinterpret_cast<uint64_t *>(pin_blob.p + x_loff);
            for (int64_t r = 0; r <= R; ++r) lo[r] = label_off[r] - label_off[0];
            d_labels = reinterpret_cast<const uint32_t *>(h2d_blob.p + x_lab);
            d_label_off = reinterpret_cast<const uint64_t *>(h2d_blob.p + x_loff);
            h2d_bytes = blob;
        }
        // a small push (<= 64 KiB staged): k_chunk_ranges copies the blob itself, so the stream has
        // one operation fewer before the tokenizer (the few KB cross PCIe as the kernel's loads)
        fused_h2d = FusedH2D{};
        const uint8_t *d_text = h2d_blob.p;
        const uint64_t *d_off = reinterpret_cast<const uint64_t *>(h2d_blob.p + x_off);
        if (h2d_bytes <= (64u << 10) && !profiling) {
            if (blob_dev_host != pin_blob.p) {  // (once per staging buffer)
                HIP_TRY(hipHostGetDevicePointer(&blob_dev, pin_blob.p, 0));
                blob_dev_host = pin_blob.p;
            }
            const uint8_t *dsrc = static_cast<const uint8_t *>(blob_dev);
            fused_h2d.src = dsrc;
            fused_h2d.dst = h2d_blob.p;
            fused_h2d.bytes = h2d_bytes;
            fused_h2d.h_off = reinterpret_cast<const uint64_t *>(dsrc + x_off);
        } else {
            HIP_TRY(hipMemcpyAsync(h2d_blob.p, pin_blob.p, h2d_bytes, hipMemcpyHostToDevice, stream));
        }
        // Small calls (a per-record push): the rows go straight to the back batch
        // and a pre-allocated next one in the same pass, and the row offsets and
        // error words come back through mapped memory -- one synchronisation.
        const bool direct = R <= 4096 && N <= ((int64_t)1 << 20) && !store.empty() && !profiling;
        uint32_t cap = 0;
        const uint32_t *stat;
        DirectDst dd{};
        if (direct) {
            if (!spare) spare = new_batch();
            HostBatch *b0 = store.back(), *b1 = spare;
            cap = (uint32_t)(2 * P.B - b0->rows);
            for (int i = 0; i < 2; ++i) {
                HostBatch *b = i ? b1 : b0;
                dd.ids[i] = b->on_dev(b->ids);
                dd.am[i] = b->on_dev(b->am);
                dd.tt[i] = b->on_dev(b->tt);
                dd.lab[i] = b->on_dev(multi() ? (int32_t *)b->f32 : b->lab);
            }
            dd.base = (uint32_t)b0->rows;
            dd.cap = cap;
            dd.B = (uint32_t)P.B;
            ensure_stat((size_t)R + 3);
            fuse_dd = dd;
            fuse_stat = stat_dev;
        }
        fused_done = false;
        struct FuseReset {  // (no other entry point may see this call's destinations, also on a throw)
            uint32_t *&p;
            ~FuseReset() { p = nullptr; }
        } fuse_reset{fuse_stat};
        {
            struct Clear {  // (never left set for a later call, also on a throw)
                FusedH2D &f;
                ~Clear() { f = FusedH2D{}; }
            } clear{fused_h2d};
            run_device(d_text, N, d_off, R, first_override >= 0 ? (uint64_t)first_override : cfg.first_record + n_records,
                       stream, d_labels, d_label_off);
        }
        fuse_stat = nullptr;
        if (direct) {
            if (!fused_done)
                HIP_TRY(launch_rows_direct(dd, row_off.p, R, o_ids.p, o_am.p, with_tt() ? o_tt.p : nullptr,
                                           multi() ? reinterpret_cast<const int32_t *>(o_f32.p) : o_lab.p, P.S,
                                           P.label_width, span() ? span_err.p : nullptr,
                                           dt.kind == TOK_UNIGRAM ? uni_err.p : nullptr, stat_dev, stream));
            hc.lap("enqueue");
            HIP_TRY(hipStreamSynchronize(stream));
            hc.lap("h2d+kernels+rows");
            stat = pin_stat.p;
        } else {
            hc.lap("enqueue");
            pin_u32.ensure((size_t)R + 3);
            HIP_TRY(hipMemcpyAsync(pin_u32.p, row_off.p, sizeof(uint32_t) * (size_t)(R + 1), hipMemcpyDeviceToHost,
                                   stream));
            pin_u32.p[R + 1] = pin_u32.p[R + 2] = 0;
            if (span()) HIP_TRY(hipMemcpyAsync(pin_u32.p + R + 1, span_err.p, 4, hipMemcpyDeviceToHost, stream));
            if (dt.kind == TOK_UNIGRAM)
                HIP_TRY(hipMemcpyAsync(pin_u32.p + R + 2, uni_err.p, 4, hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            hc.lap("h2d+kernels");
            stat = pin_u32.p;
        }
        // where the reference panics (t5_data.rs:205-216: a label past S/4 or a
        // 101st sentinel) the host path fails the call before any batch is queued
        if (stat[R + 1])
            throw ArgError("span: " + std::to_string(stat[R + 1]) +
                           " label/sentinel writes out of range (the reference panics)");
        if (stat[R + 2])
            throw CapacityError("t5 tokenizer capacity exceeded (flags " + std::to_string(stat[R + 2]) + ")");
        // GenTokenizer::create_sync_batch per record (gen_batcher.rs:69-94):
        // rows fill the back batch (handle_internal_batch per chunk), at most
        // one finished batch is emitted per record.  Each run of rows landing
        // contiguously in one batch and not written by the direct pass is one
        // segment, copied D2H below.
        struct Seg {
            HostBatch *b;
            uint32_t dst, g0, n;
        };
        std::vector<Seg> segs;
        for (int64_t r = 0; r < R; ++r) {
            const uint32_t g0 = stat[r], g1 = stat[r + 1];
            if (g1 > g0 && store.empty())  // store.back_mut().unwrap() (gen_batcher.rs:45) panics
                throw ArgError("a record after get_working_batch emptied the batch store (the reference panics)");
            for (uint32_t g = g0; g < g1; ++g) {
                HostBatch *b = store.back();
                if (g >= cap) {
                    if (!segs.empty() && segs.back().b == b && segs.back().g0 + segs.back().n == g) ++segs.back().n;
                    else segs.push_back(Seg{b, (uint32_t)b->rows, g, 1u});
                }
                b->rows++;
                if (b->rows == P.B) {
                    store.push_back(spare ? spare : new_batch());
                    spare = nullptr;
                }
            }
            if (!store.empty() && store.front()->rows == P.B) {  // at most one batch per call
                outbox.push_back(store.front());
                store.pop_front();
            }
        }
        hc.lap("cadence");
        if (!segs.empty()) {
            seg_pin.ensure(segs.size());
            uint32_t nmax = 0;
            for (size_t i = 0; i < segs.size(); ++i) {
                const Seg &q = segs[i];
                HostBatch *b = q.b;
                seg_pin.p[i] = RowSeg{b->on_dev(b->ids), b->on_dev(b->am), b->on_dev(b->tt),
                                      b->on_dev(multi() ? (int32_t *)b->f32 : b->lab), q.g0, q.n, q.dst, 0u};
                nmax = std::max(nmax, q.n);
            }
            seg_dev.ensure(segs.size());
            HIP_TRY(hipMemcpyAsync(seg_dev.p, seg_pin.p, sizeof(RowSeg) * segs.size(), hipMemcpyHostToDevice, stream));
            HIP_TRY(launch_rows_to_host(seg_dev.p, (int)segs.size(), nmax, o_ids.p, o_am.p,
                                        with_tt() ? o_tt.p : nullptr,
                                        multi() ? reinterpret_cast<const int32_t *>(o_f32.p) : o_lab.p, P.S,
                                        P.label_width, stream));
        }
        hc.lap("d2h enqueue");
        if (!segs.empty()) HIP_TRY(hipStreamSynchronize(stream));
        hc.lap("d2h");
        hc.report(N, segs.size(), pool ? pool->fresh : 0);
        n_records += (uint64_t)R;
    }
};

namespace {

void fill_batch(const sdl_batcher *h, HostBatch *b, sdl_batch *out) {
    std::memset(out, 0, sizeof(*out));
    out->rows = b->rows;
    out->batch_size = b->B;
    out->sequence_length = b->S;
    out->label_width = b->LW;
    b->init_tail();
    out->input_ids = b->ids;
    out->attention_mask = b->am;
    out->token_type_ids = b->tt;
    out->labels = b->lab;
    out->labels_f32 = b->f32;
    out->owner_ = b;
    (void)h;
}

// Span draws (RNG contract): v = trunc_sat(avg - z), z ~ N(0,1),
// by CDF inversion on a 32-bit uniform -- thr[j] = floor(2^32 P(v <= kmin + j)),
// P(v <= k) = erfc((avg - k - 1) / sqrt 2) / 2; `lo` folds smaller values in
// (size: max(.., 1)).  oracle/orc_batcher.c:orc_span_table computes the same.
void span_table(double avg, int lo, int32_t *kmin, int32_t *n, uint32_t *thr) {
    double k0 = std::floor(avg - 10.0);
    if (k0 < lo) k0 = lo;
    if (k0 > 1e9) k0 = 1e9;
    *kmin = (int32_t)k0;
    int m = 0;
    for (int j = 0; j < 32; ++j) {
        const double cdf = 0.5 * std::erfc((avg - (k0 + j) - 1.0) / std::sqrt(2.0));
        const double t = std::floor(cdf * 4294967296.0);
        if (t >= 4294967296.0) break;
        thr[m++] = (uint32_t)t;
    }
    *n = m;
    for (int j = m; j < 32; ++j) thr[j] = 0xFFFFFFFFu;
}

// rand_distr 0.4.3's ziggurat tables for StandardNormal (ZIG_NORM_X /
// ZIG_NORM_F) as its ziggurat_tables.py writes them: 256 layers with
// R = 3.6541528853610088, V = 0.00492867323399, x[i] = f^-1(V / x[i-1] +
// f(x[i-1])), f(x) = exp(-x^2 / 2), each value printed with %.18f and read
// back as the Rust literal.  (oracle/orc_batcher.c zig_tables is the checker's
// restatement; tests/test_rand_mode.py pins the printed head of both.)
void zig_norm_tables(double *X, double *F) {
    const double R = 3.6541528853610088, V = 0.00492867323399;
    auto f = [](double x) { return std::exp(-x * x / 2.0); };
    double x[257];
    x[0] = V / f(R);
    x[1] = R;
    for (int i = 2; i < 256; ++i) x[i] = std::sqrt(-2.0 * std::log(V / x[i - 1] + f(x[i - 1])));
    x[256] = 0.0;
    char buf[64];
    for (int i = 0; i < 257; ++i) {
        std::snprintf(buf, sizeof buf, "%.18f", x[i]);
        X[i] = std::strtod(buf, nullptr);
        std::snprintf(buf, sizeof buf, "%.18f", f(x[i]));
        F[i] = std::strtod(buf, nullptr);
    }
}

std::string default_data_dir() {
    Dl_info info;
    if (dladdr((void *)&default_data_dir, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        size_t s = p.rfind('/');
        return (s == std::string::npos ? std::string(".") : p.substr(0, s)) + "/data";
    }
    return "data";
}

}  // namespace

extern "C" {

int sdl_abi_version(void) { return SDL_ABI_VERSION; }
const char *sdl_last_error(void) { return g_err.c_str(); }

void sdl_config_default(sdl_config *c, int32_t task) {
    std::memset(c, 0, sizeof(*c));
    c->task = task;
    c->batch_size = 4096;  // masking_cases.rs:43
    c->sequence_length = 128;
    const bool simple = task == SDL_TASK_MULTI_LABEL || task == SDL_TASK_SINGLE_CLASS;
    c->chunk = simple ? 0 : 1;
    c->min_ids = simple ? 0 : 64;
    if (task == SDL_TASK_SINGLE_CLASS) c->batch_size = 2048;  // single_cases.rs (Imdb)
    c->mask_length = (int32_t)((float)c->sequence_length * 0.15f);  // masking_cases.rs:34-36
    c->mask_id = 103;
    c->number_labels = 9;
    c->avg_span_gap = 16.0;
    c->avg_span_size = 2.0;
    c->seed = 0;
    c->first_record = 0;
    c->device = 0;
}

int sdl_batcher_create(const sdl_config *cfg, const char *tokenizer_path, const char *data_dir, sdl_batcher **out) {
    if (!cfg || !tokenizer_path || !out) return fail(SDL_ERR_ARG, "null argument");
    *out = nullptr;
    if (cfg->task != SDL_TASK_MLM && cfg->task != SDL_TASK_CLM && cfg->task != SDL_TASK_MULTI_LABEL &&
        cfg->task != SDL_TASK_SPAN && cfg->task != SDL_TASK_SINGLE_CLASS)
        return fail(SDL_ERR_UNSUPPORTED, "unknown task");
    if (cfg->task == SDL_TASK_SPAN && (cfg->sequence_length < 4 || !(cfg->avg_span_gap == cfg->avg_span_gap) ||
                                       !(cfg->avg_span_size == cfg->avg_span_size)))
        return fail(SDL_ERR_ARG, "span needs sequence_length >= 4 and finite avg_span_gap / avg_span_size");
    if (cfg->task == SDL_TASK_MULTI_LABEL && (cfg->number_labels <= 0 || cfg->number_labels > 4096))
        return fail(SDL_ERR_ARG, "number_labels must be in [1, 4096]");
    if (cfg->batch_size <= 0 || cfg->sequence_length <= 0 || cfg->sequence_length > 2048)
        return fail(SDL_ERR_ARG, "batch_size must be > 0 and 0 < sequence_length <= 2048");
    if (cfg->task == SDL_TASK_MLM && (cfg->mask_length < 0 || cfg->mask_length > cfg->sequence_length))
        return fail(SDL_ERR_ARG, "mask_length must be in [0, sequence_length]");
    if (cfg->rng_mode != 0 && cfg->rng_mode != 1) return fail(SDL_ERR_ARG, "rng_mode must be 0 or 1");
    if (cfg->task == SDL_TASK_MLM && cfg->rng_mode == 1 && cfg->sequence_length > RAND_MAX_S)
        return fail(SDL_ERR_UNSUPPORTED, "rng_mode 1 supports sequence_length <= 2048");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(SDL_ERR_NODEV, "no HIP device visible: the Batcher runs only on the GPU (no CPU fallback)");
    if (cfg->device < 0 || cfg->device >= ndev) return fail(SDL_ERR_ARG, "device ordinal out of range");
    std::unique_ptr<sdl_batcher> h(new sdl_batcher());
    try {
        h->cfg = *cfg;
        h->device = cfg->device;
        load_tokenizer(tokenizer_path, data_dir ? std::string(data_dir) : default_data_dir(), h->tok);
        HIP_TRY(hipSetDevice(h->device));
        {  // the handle's stream at the highest priority (stream2's background work yields to it)
            int least = 0, greatest = 0;
            if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
            HIP_TRY(hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, greatest));
        }
        for (auto &e : h->ev) HIP_TRY(hipEventCreate(&e));
        auto &t = h->tok;
        h->d_ubmp.ensure(t.ubmp.size());
        HIP_TRY(hipMemcpy(h->d_ubmp.p, t.ubmp.data(), t.ubmp.size() * 4, hipMemcpyHostToDevice));
        h->d_upage.ensure(t.upage.size());
        h->d_uentry.ensure(t.uentry.size());
        h->d_upool.ensure(t.upool.size());
        h->d_slots.ensure(t.slots.size());
        h->d_vpool.ensure(t.vpool.size());
        h->d_ascii_id.ensure(128);
        if (t.ascii_id.size() == 128)
            HIP_TRY(hipMemcpy(h->d_ascii_id.p, t.ascii_id.data(), 128 * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(h->d_upage.p, t.upage.data(), t.upage.size() * 2, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(h->d_uentry.p, t.uentry.data(), t.uentry.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(h->d_upool.p, t.upool.data(), t.upool.size(), hipMemcpyHostToDevice));
        if (t.kind == TOK_UNIGRAM) {
            // the device copy of the pieces table: a piece whose f64 score is one ulp
            // off its f32 has bit 15 of its id set, and the f32 in word 3 negated when
            // the ulp is towards zero (tokenize_unigram.hip uni_score64)
            std::vector<VSlot> ds(t.slots);
            for (VSlot &v : ds) {
                const uint32_t cont = v.key >> 8;
                if (v.id < 0 || (cont != UC_PIECE && cont != UC_META)) continue;
                const int adj = t.uscore_adj[(size_t)v.id];
                if (adj == 0) continue;
                const float f = t.uscore32[(size_t)v.id];
                // (0x7FFF | 0x8000 is the chunk kernel's "no piece" word: tokenize_unigram.hip NO_PIECE)
                if (v.id >= 0x7FFF || !(f < 0.0f))
                    throw std::runtime_error("Unigram: a score off its f32 needs id < 32767 and a negative score");
                v.id |= 0x8000;
                if (adj < 0) {
                    const float g = -f;
                    std::memcpy(&v.hash, &g, 4);
                }
            }
            HIP_TRY(hipMemcpy(h->d_slots.p, ds.data(), ds.size() * sizeof(VSlot), hipMemcpyHostToDevice));
        } else {
            HIP_TRY(hipMemcpy(h->d_slots.p, t.slots.data(), t.slots.size() * sizeof(VSlot), hipMemcpyHostToDevice));
        }
        HIP_TRY(hipMemcpy(h->d_vpool.p, t.vpool.data(), t.vpool.size(), hipMemcpyHostToDevice));
        DevTok &d = h->dt;
        d.kind = t.kind;
        if (t.kind == TOK_BYTE_BPE) {
            h->d_gpage.ensure(t.gpage.size());
            h->d_gblock.ensure(t.gblock.size());
            h->d_mslots.ensure(t.mslots.size());
            h->d_byte_id.ensure(256);
            HIP_TRY(hipMemcpy(h->d_gpage.p, t.gpage.data(), t.gpage.size() * 2, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(h->d_gblock.p, t.gblock.data(), t.gblock.size(), hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(h->d_mslots.p, t.mslots.data(), t.mslots.size() * sizeof(MSlot), hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(h->d_byte_id.p, t.byte_id.data(), 256 * 2, hipMemcpyHostToDevice));
            d.gpage = h->d_gpage.p;
            d.gblock = h->d_gblock.p;
            d.mslots = h->d_mslots.p;
            d.byte_id = h->d_byte_id.p;
            d.mslot_mask = t.mslot_mask;
        }
        if (t.kind == TOK_UNIGRAM) {
            h->d_uscore.ensure(t.uscore.size());
            h->d_wres.ensure(t.wres.size());
            h->d_cpage.ensure(t.cpage.size());
            h->d_cent.ensure(t.cent.size() / 2);
            h->d_uscore32.ensure(t.uscore32.size());
            h->d_trie.ensure(t.trie.size());
            h->d_tnorm.ensure(t.tnorm.size());
            h->d_extra.ensure(100);
            HIP_TRY(hipMemcpy(h->d_uscore.p, t.uscore.data(), t.uscore.size() * 8, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(h->d_wres.p, t.wres.data(), t.wres.size() * 2, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(h->d_cpage.p, t.cpage.data(), t.cpage.size() * 2, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(h->d_cent.p, t.cent.data(), t.cent.size() * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(h->d_uscore32.p, t.uscore32.data(), t.uscore32.size() * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(h->d_trie.p, t.trie.data(), t.trie.size() * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(h->d_tnorm.p, t.tnorm.data(), t.tnorm.size(), hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(h->d_extra.p, t.extra_ids.data(), 100 * 4, hipMemcpyHostToDevice));
            h->d_wslots.ensure(t.wslots.size());
            HIP_TRY(hipMemcpy(h->d_wslots.p, t.wslots.data(), t.wslots.size() * sizeof(VSlot), hipMemcpyHostToDevice));
            d.wslots = h->d_wslots.p;
            d.wslot_mask = t.wslot_mask;
            h->d_upfx.ensure(t.upfx.size());
            HIP_TRY(hipMemcpy(h->d_upfx.p, t.upfx.data(), t.upfx.size(), hipMemcpyHostToDevice));
            d.upfx = h->d_upfx.p;
            d.uscore = h->d_uscore.p;
            d.wres = h->d_wres.p;
            d.cpage = h->d_cpage.p;
            d.cent = h->d_cent.p;
            {  // the BMP entries flattened: one dependent load per char instead of two
                std::vector<uint32_t> flat(2 * 0x10000);
                for (uint32_t cp = 0; cp < 0x10000; ++cp) {
                    const size_t at = 2 * ((size_t)t.cpage[cp >> 8] * 256 + (cp & 255));
                    flat[2 * cp] = t.cent[at];
                    flat[2 * cp + 1] = t.cent[at + 1];
                }
                // the kernels compute White_Space and the ASCII property bytes
                // (uni_white_space / uni_ascii_props): the tables must agree
                for (uint32_t cp = 0; cp < 0x110000; ++cp) {
                    const uint32_t x = t.cent[2 * ((size_t)t.cpage[cp >> 8] * 256 + (cp & 255))] & 0xFFu;
                    if (((x & GP_WS) != 0) != uni_white_space(cp) || (cp < 0x80 && x != uni_ascii_props(cp)))
                        throw std::runtime_error("t5 grapheme table: White_Space / ASCII properties differ from "
                                                 "the kernels' built-in ones at U+" + std::to_string(cp));
                }
                h->d_cbmp.ensure(0x10000);
                HIP_TRY(hipMemcpy(h->d_cbmp.p, flat.data(), flat.size() * 4, hipMemcpyHostToDevice));
                d.cbmp = h->d_cbmp.p;
            }
            d.uscore32 = h->d_uscore32.p;
            d.trie = h->d_trie.p;
            d.tnorm = h->d_tnorm.p;
            d.trie_units = (uint32_t)t.trie.size();
            d.tnorm_len = (uint32_t)t.tnorm.size();
            d.unk_score = t.unk_score;
            d.maxlen_meta = t.maxlen_cont;
            d.maxlen_word = t.max_word;
            d.maxlen_piece = t.maxlen_piece;
        }
        if (cfg->task == SDL_TASK_SPAN && t.kind != TOK_UNIGRAM)
            throw std::runtime_error("task span needs the t5 (Unigram) tokenizer: TokenizerInfo.extra (tokenizer_wrapper.rs:77-80)");
        d.ubmp = reinterpret_cast<const uint2 *>(h->d_ubmp.p);
        d.upage = h->d_upage.p;
        d.uentry = h->d_uentry.p;
        d.upool = h->d_upool.p;
        d.slots = h->d_slots.p;
        d.vpool = h->d_vpool.p;
        d.slot_mask = t.slot_mask;
        d.unk_id = t.unk_id;
        d.maxlen_first = t.maxlen_first;
        d.maxlen_cont = t.maxlen_cont;
        {
            std::vector<uint8_t> all(2 * LW_MAX, 0);
            for (int c = 0; c < 2; ++c) {
                std::vector<uint8_t> lens = t.wp_lens[c];
                std::sort(lens.begin(), lens.end());
                d.wp_nlens[c] = (int32_t)lens.size();
                std::copy(lens.begin(), lens.end(), all.begin() + c * LW_MAX);
            }
            h->d_wp_lens.ensure(all.size());
            HIP_TRY(hipMemcpy(h->d_wp_lens.p, all.data(), all.size(), hipMemcpyHostToDevice));
            d.wp_lens = h->d_wp_lens.p;
        }
        d.wp_long_pieces = t.wp_long_pieces ? 1 : 0;
        d.ascii_id = h->d_ascii_id.p;
        d.n_special = (int)t.added.size();
        d.max_special_len = t.max_special_len;
        d.opener = t.opener;
        for (size_t i = 0; i < t.added.size() && t.kind != TOK_UNIGRAM; ++i) {
            d.special_id[i] = t.added[i].second;
            d.special_len[i] = (uint8_t)t.added[i].first.size();
            std::memcpy(d.special_bytes[i], t.added[i].first.data(), t.added[i].first.size());
        }
        RowParams &P = h->P;
        P.task = cfg->task;
        P.B = cfg->batch_size;
        P.S = cfg->sequence_length;
        P.chunk = cfg->chunk;
        P.min_ids = cfg->min_ids;
        P.mask_length = cfg->mask_length;
        P.mask_id = cfg->mask_id;
        P.label_width = cfg->task == SDL_TASK_MULTI_LABEL    ? cfg->number_labels
                        : cfg->task == SDL_TASK_SINGLE_CLASS ? 1
                        : cfg->task == SDL_TASK_SPAN          ? cfg->sequence_length / 4  // t5_data.rs:44
                                                              : cfg->sequence_length;
        if (cfg->task == SDL_TASK_SPAN) {
            span_table(cfg->avg_span_gap, 0, &P.gap_kmin, &P.gap_n, P.gap_thr);
            span_table(cfg->avg_span_size, 1, &P.size_kmin, &P.size_n, P.size_thr);
            P.extra_ids = h->d_extra.p;
            P.avg_span_gap = cfg->avg_span_gap;
            P.avg_span_size = cfg->avg_span_size;
            if (cfg->rng_mode == 1) {  // random_data_gap / random_data_size on the row's StdRng
                std::vector<double> zt(2 * 257);
                zig_norm_tables(zt.data(), zt.data() + 257);
                h->d_zig.ensure(zt.size());
                HIP_TRY(hipMemcpy(h->d_zig.p, zt.data(), zt.size() * 8, hipMemcpyHostToDevice));
                P.zig_x = h->d_zig.p;
                P.zig_f = h->d_zig.p + 257;
            }
        }
        if (cfg->task == SDL_TASK_MULTI_LABEL || cfg->task == SDL_TASK_SINGLE_CLASS) {  // SimpleBatcher: one row per record, no filter
            P.chunk = 0;
            P.min_ids = 0;
        }
        P.seed = cfg->seed;
        P.rng_mode = cfg->rng_mode;
        if (t.kind == TOK_UNIGRAM) {
            // encode_mask framing for T5 (tokenizer_wrapper.rs:125-131): [eos] + template($A </s>) + [eos]
            P.n_pre = 1;
            P.pre[0] = t.eos_id;
            P.n_post = 2;
            P.post[0] = t.tpl_eos;
            P.post[1] = t.eos_id;
        } else if (t.kind == TOK_BYTE_BPE) {
            // encode_mask framing for Gpt (tokenizer_wrapper.rs:118-124): [eos] + ids + [eos]
            P.n_pre = 1;
            P.pre[0] = t.eos_id;
            P.n_post = 1;
            P.post[0] = t.eos_id;
        } else {
            // encode_mask framing (tokenizer_wrapper.rs:107-116): [CLS] + template([CLS] $A [SEP]) + [SEP] [SEP]
            P.n_pre = 2;
            P.pre[0] = t.cls_id;
            P.pre[1] = t.tpl_cls;
            P.n_post = 3;
            P.post[0] = t.tpl_sep;
            P.post[1] = t.sep_id;
            P.post[2] = t.sep_id;
        }
        h->store.push_back(h->new_batch());  // GenTokenizer::new: first DataSet
    } catch (HipError &e) {
        return fail(SDL_ERR_HIP, e.what());
    } catch (std::exception &e) {
        return fail(SDL_ERR_IO, e.what());
    }
    *out = h.release();
    return SDL_OK;
}

void sdl_batcher_destroy(sdl_batcher *h) { delete h; }

namespace {
// BertData::put_data panics on an index >= number_labels (bert_data.rs:70-72)
int check_labels(const sdl_batcher *h, const uint32_t *labels, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (labels[i] >= (uint32_t)h->P.label_width)
            return fail(SDL_ERR_ARG, "label index " + std::to_string(labels[i]) + " >= number_labels");
    return SDL_OK;
}
}  // namespace

int sdl_batcher_push(sdl_batcher *h, const uint8_t *utf8, size_t len, const uint32_t *labels, size_t n_labels,
                     sdl_batch *out) {
    if (!h || (!utf8 && len) || (!labels && n_labels)) return fail(SDL_ERR_ARG, "null argument");
    if (h->multi()) {
        if (int rc = check_labels(h, labels, n_labels)) return rc;
    }
    if (h->single() && n_labels != 1) return fail(SDL_ERR_ARG, "single-class records carry exactly one label");
    if (len >= (1ull << 32)) return fail(SDL_ERR_CAPACITY, "record too large");
    try {
        uint64_t offs[2] = {0, (uint64_t)len};
        uint64_t loffs[2] = {0, (uint64_t)n_labels};
        const size_t before = h->outbox.size();
        h->process_host(utf8 ? utf8 : (const uint8_t *)"", offs, 1, labels, loffs);
        if (h->outbox.size() > before) {
            HostBatch *b = h->outbox.back();
            h->outbox.pop_back();
            if (out) fill_batch(h, b, out);
            else delete b;
            return 1;
        }
        return 0;
    } catch (HipError &e) {
        return fail(SDL_ERR_HIP, e.what());
    } catch (CapacityError &e) {
        return fail(SDL_ERR_CAPACITY, e.what());
    } catch (std::exception &e) {
        return fail(SDL_ERR_ARG, e.what());
    }
}

int sdl_batcher_push_many(sdl_batcher *h, const uint8_t *arena, const uint64_t *offsets, size_t n_records,
                          const uint32_t *labels, const uint64_t *label_offsets, size_t *n_emitted) {
    if (!h || !offsets || (!arena && n_records && offsets[n_records])) return fail(SDL_ERR_ARG, "null argument");
    if (h->multi() && label_offsets) {
        if (!labels && label_offsets[n_records] != label_offsets[0]) return fail(SDL_ERR_ARG, "null labels");
        for (size_t r = 0; r < n_records; ++r)
            if (label_offsets[r + 1] < label_offsets[r]) return fail(SDL_ERR_ARG, "label_offsets must be non-decreasing");
        if (int rc = check_labels(h, labels + label_offsets[0], label_offsets[n_records] - label_offsets[0])) return rc;
    }
    if (h->single()) {
        if (!label_offsets || !labels) return fail(SDL_ERR_ARG, "single-class records need their labels");
        for (size_t r = 0; r < n_records; ++r)
            if (label_offsets[r + 1] != label_offsets[r] + 1)
                return fail(SDL_ERR_ARG, "single-class records carry exactly one label");
    }
    if (offsets[0] != 0) return fail(SDL_ERR_ARG, "offsets[0] must be 0");
    for (size_t r = 0; r < n_records; ++r)
        if (offsets[r + 1] < offsets[r]) return fail(SDL_ERR_ARG, "offsets must be non-decreasing");
    if (offsets[n_records] >= (1ull << 32)) return fail(SDL_ERR_CAPACITY, "arena must be < 4 GiB per call");
    try {
        const size_t before = h->outbox.size();
        if (n_records)
            h->process_host(arena, offsets, (int64_t)n_records, labels ? labels + (label_offsets ? label_offsets[0] : 0) : nullptr,
                            label_offsets);
        if (n_emitted) *n_emitted = h->outbox.size() - before;
        return SDL_OK;
    } catch (HipError &e) {
        return fail(SDL_ERR_HIP, e.what());
    } catch (CapacityError &e) {
        return fail(SDL_ERR_CAPACITY, e.what());
    } catch (std::exception &e) {
        return fail(SDL_ERR_ARG, e.what());
    }
}

int sdl_batcher_next(sdl_batcher *h, sdl_batch *out) {
    if (!h || !out) return fail(SDL_ERR_ARG, "null argument");
    if (h->outbox.empty()) return 0;
    HostBatch *b = h->outbox.front();
    h->outbox.pop_front();
    fill_batch(h, b, out);
    return 1;
}

int sdl_batcher_flush(sdl_batcher *h, sdl_batch *out) {
    if (!h || !out) return fail(SDL_ERR_ARG, "null argument");
    if (h->store.empty()) return 0;  // GenTokenizer::get_working_batch = store.pop_front()
    HostBatch *b = h->store.front();
    h->store.pop_front();
    // SimpleBatcher::get_working_batch swaps in a fresh DataSet (simple_batcher.rs:46-52)
    if (h->simple() && h->store.empty()) h->store.push_back(h->new_batch());
    fill_batch(h, b, out);
    return 1;
}

void sdl_batch_release(sdl_batch *b) {
    if (!b || !b->owner_) return;
    delete static_cast<HostBatch *>(b->owner_);
    std::memset(b, 0, sizeof(*b));
}

int sdl_process_device(sdl_batcher *h, const uint8_t *d_text, uint64_t text_len, const uint64_t *d_offsets,
                       uint64_t n_records, uint64_t first_record, void *stream, sdl_device_rows *out) {
    return sdl_process_device_labels(h, d_text, text_len, d_offsets, n_records, nullptr, nullptr, first_record, stream,
                                     out);
}

int sdl_process_device_labels(sdl_batcher *h, const uint8_t *d_text, uint64_t text_len, const uint64_t *d_offsets,
                              uint64_t n_records, const uint32_t *d_labels, const uint64_t *d_label_offsets,
                              uint64_t first_record, void *stream, sdl_device_rows *out) {
    if (!h || !out || !d_offsets || (!d_text && text_len)) return fail(SDL_ERR_ARG, "null argument");
    if ((d_labels == nullptr) != (d_label_offsets == nullptr)) return fail(SDL_ERR_ARG, "labels need label offsets");
    if (text_len >= (1ull << 32)) return fail(SDL_ERR_CAPACITY, "arena must be < 4 GiB per call");
    if (((uintptr_t)d_text & 15u) != 0) return fail(SDL_ERR_ARG, "d_text must be 16-byte aligned");
    try {
        hipStream_t st = stream ? (hipStream_t)stream : h->stream;
        h->run_device(d_text, (int64_t)text_len, d_offsets, (int64_t)n_records, first_record, st, d_labels,
                      d_label_offsets);
        std::memset(out, 0, sizeof(*out));
        out->input_ids = h->o_ids.p;
        out->attention_mask = h->o_am.p;
        out->token_type_ids = h->with_tt() ? h->o_tt.p : nullptr;
        out->labels = h->multi() ? nullptr : h->o_lab.p;
        out->labels_f32 = h->multi() ? h->o_f32.p : nullptr;
        out->d_label_errors = h->simple() ? h->lab_err.p : h->span() ? h->span_err.p : nullptr;
        out->d_tokenize_errors = h->dt.kind == TOK_UNIGRAM ? h->uni_err.p : nullptr;
        out->d_rows = h->row_off.p + n_records;
        out->d_record_rows = h->rec_rows.p;
        out->d_tokens = h->chunk_off.p + (text_len + CHUNK - 1) / CHUNK;
        out->rows_capacity = (uint64_t)h->last_rows_cap;
        out->label_width = h->P.label_width;
        return SDL_OK;
    } catch (HipError &e) {
        return fail(SDL_ERR_HIP, e.what());
    } catch (std::exception &e) {
        return fail(SDL_ERR_ARG, e.what());
    }
}

int sdl_json_text_device(sdl_batcher *h, const uint8_t *d_jsonl, uint64_t len, void *stream, sdl_json_text *out) {
    if (!h || !out || (!d_jsonl && len)) return fail(SDL_ERR_ARG, "null argument");
    if (len >= (1ull << 32)) return fail(SDL_ERR_CAPACITY, "JSON buffer must be < 4 GiB per call");
    if (((uintptr_t)d_jsonl & 15u) != 0) return fail(SDL_ERR_ARG, "d_jsonl must be 16-byte aligned");
    try {
        hipStream_t st = stream ? (hipStream_t)stream : h->stream;
        const int64_t N = (int64_t)len, nb = (N + CHUNK - 1) / CHUNK;
        h->j_cnt.ensure((size_t)nb + 1);
        h->j_base.ensure((size_t)nb + 1);
        h->scan_tmp.ensure((size_t)scan_tmp_words(std::max<int64_t>(nb, 1)) + 1);
        // the newline list is sized for JSON lines of >= 64 B on average (a record line is
        // {"text": ...} plus the dump's fields), so the count and the last position come back
        // together in one synchronisation; denser input grows the list and writes it again
        uint32_t n_nl = 0, last_nl = 0;
        const size_t nl_want = std::min<size_t>((size_t)N / 64 + 4096, (size_t)N + 2);
        h->j_nl.ensure(nl_want);
        h->j_tail.ensure(2);
        if (nb) {
            const uint32_t cap = (uint32_t)std::min<size_t>(h->j_nl.cap, 0xFFFFFFFFu);
            HIP_TRY(launch_json_nl_count(d_jsonl, N, h->j_cnt.p, h->j_base.p, h->scan_tmp.p, st));
            HIP_TRY(launch_json_nl_write(d_jsonl, N, h->j_base.p, h->j_nl.p, cap, st));
            HIP_TRY(launch_json_nl_tail(h->j_base.p + nb, h->j_nl.p, cap, h->j_tail.p, st));
            HIP_TRY(hipMemcpyAsync(h->pin_u32_2, h->j_tail.p, 8, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            n_nl = h->pin_u32_2[0];
            last_nl = h->pin_u32_2[1];
            if (n_nl > cap) {  // more lines than the list held: grow it to the count, write again
                h->j_nl.ensure((size_t)n_nl + 2);
                const uint32_t cap2 = (uint32_t)std::min<size_t>(h->j_nl.cap, 0xFFFFFFFFu);
                HIP_TRY(launch_json_nl_write(d_jsonl, N, h->j_base.p, h->j_nl.p, cap2, st));
                HIP_TRY(launch_json_nl_tail(h->j_base.p + nb, h->j_nl.p, cap2, h->j_tail.p, st));
                HIP_TRY(hipMemcpyAsync(h->pin_u32_2, h->j_tail.p, 8, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                last_nl = h->pin_u32_2[1];
            }
        }
        // tokio lines(): a last line without '\n' counts, an empty tail does not
        const int64_t tail0 = n_nl ? (int64_t)last_nl + 1 : 0;
        const int64_t n_lines = (int64_t)n_nl + (N > tail0 ? 1 : 0);
        const size_t L1 = (size_t)n_lines + 1;
        h->j_len.ensure(L1);
        h->j_rec.ensure(L1);
        h->j_toff.ensure(L1);
        h->j_ridx.ensure(L1);
        h->j_span.ensure(L1);
        h->j_off.ensure(L1);
        h->j_inv.ensure(1);
        h->j_text.ensure((size_t)N + 32);
        h->scan_tmp.ensure((size_t)scan_tmp_words(std::max<int64_t>(std::max<int64_t>(nb, n_lines), 1)) + 1);
        HIP_TRY(hipMemsetAsync(h->j_inv.p, 0, 4, st));
        HIP_TRY(hipMemsetAsync(h->j_off.p, 0, 8, st));
        HIP_TRY(launch_json_parse(d_jsonl, N, h->j_nl.p, n_nl, n_lines, h->j_len.p, h->j_rec.p, h->j_span.p,
                                  h->j_inv.p, st));
        uint32_t counts[3] = {0, 0, 0};  // records, text bytes, invalid lines
        if (n_lines) {
            HIP_TRY(launch_exclusive_scan(h->j_len.p, h->j_toff.p, n_lines, h->scan_tmp.p, st));
            HIP_TRY(launch_exclusive_scan(h->j_rec.p, h->j_ridx.p, n_lines, h->scan_tmp.p, st));
            HIP_TRY(launch_json_write(d_jsonl, N, h->j_nl.p, n_nl, n_lines, h->j_rec.p, h->j_span.p, h->j_toff.p, h->j_ridx.p, h->j_text.p,
                                      h->j_off.p, st));
            HIP_TRY(hipMemcpyAsync(&counts[0], h->j_ridx.p + n_lines, 4, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipMemcpyAsync(&counts[1], h->j_toff.p + n_lines, 4, hipMemcpyDeviceToHost, st));
        }
        HIP_TRY(hipMemcpyAsync(&counts[2], h->j_inv.p, 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemsetAsync(h->j_text.p + counts[1], 0, 16, st));  // zero tail for 16-B readers
        std::memset(out, 0, sizeof(*out));
        out->d_text = h->j_text.p;
        out->d_offsets = h->j_off.p;
        out->n_records = counts[0];
        out->text_bytes = counts[1];
        out->n_lines = (uint64_t)n_lines;
        out->n_invalid = counts[2];
        return SDL_OK;
    } catch (HipError &e) {
        return fail(SDL_ERR_HIP, e.what());
    } catch (std::exception &e) {
        return fail(SDL_ERR_ARG, e.what());
    }
}

namespace {

const char *gz_reason(int32_t s) {
    static const char *names[] = {"ok",
                                  "member range outside the buffer",
                                  "truncated",
                                  "not a gzip header (magic, method or reserved flags)",
                                  "header crc mismatch",
                                  "invalid block type",
                                  "invalid stored block lengths",
                                  "invalid code lengths set",
                                  "invalid literal/length or distance code",
                                  "invalid distance too far back",
                                  "more output than the trailer's size",
                                  "incorrect length check",
                                  "bytes after the member's trailer",
                                  "incorrect data check",
                                  "decoder made no progress"};
    return s >= 0 && s < (int32_t)(sizeof(names) / sizeof(names[0])) ? names[s] : "unknown";
}

X2N make_x2n() {  // zlib's x2n_table: x^(2^k) mod P(x), reflected
    auto mult = [](uint32_t a, uint32_t b) {
        uint32_t m = 1u << 31, p = 0;
        for (;;) {
            if (a & m) {
                p ^= b;
                if ((a & (m - 1)) == 0) break;
            }
            m >>= 1;
            b = b & 1u ? (b >> 1) ^ 0xEDB88320u : b >> 1;
        }
        return p;
    };
    X2N x{};
    uint32_t p = 1u << 30;  // x^1
    x.t[0] = p;
    for (int k = 1; k < 32; ++k) x.t[k] = p = mult(p, p);
    return x;
}

}  // namespace

// A gzip member of >= GZ_SPLIT_MIN compressed bytes -- a single-member .json.gz,
// the reference's own input -- is inflated in chunks (kernels.hpp, "chunked
// members"): a header search per chunk, every chunk decoded at once into 16-bit
// slots, each handing over where a later chunk's searched start is a real block
// start (so wrong picks and block starts the search skips -- stored or fixed
// blocks -- are decoded through in the same launch); the host follows the
// hand-overs in stream order and continues a chunk whose slot filled up with a
// new one resuming inside the block (its header parsed again); the window chain,
// bytes, CRC-32 and ISIZE follow on the device.  The member's status gets
// GZ_VERIFIED so the one-wave path skips it.
constexpr uint64_t GZ_SPLIT_MIN = 1u << 20;  // smaller members: one wave each
constexpr uint64_t GZ_CHUNK = 24u << 10;     // compressed bytes per chunk (at least; 16/20/28/32/64 KiB measured slower)
constexpr uint64_t GZ_MAX_CHUNKS = 8192;     // (larger members: larger chunks)
constexpr uint32_t GZ_SLOT_RATIO = 16;       // slot values per compressed byte of a chunk
constexpr uint64_t GZ_FIND_SPAN = 2;         // header search: this many chunk lengths of bits
constexpr uint64_t GZ_EXTRA_CHUNKS = 256;    // chunks appended behind one that stopped for capacity

void inflate_chunked(sdl_batcher *h, const uint8_t *d_gz, uint64_t m, uint64_t ma, uint64_t mz, uint32_t isize,
                     uint32_t ooff_m, hipStream_t st) {
    const uint64_t len = mz - ma;
    uint64_t ch = GZ_CHUNK;
    while ((len + ch - 1) / ch > GZ_MAX_CHUNKS) ch *= 2;
    const uint64_t C0 = (len - 8 + ch - 1) / ch;  // nominal starts ma + c ch < mz - 8
    const uint64_t CT = C0 + GZ_EXTRA_CHUNKS;
    // 16-bit slot values per chunk: GZ_SLOT_RATIO x its compressed bytes, unless the member's
    // slots together would exceed 8x its ISIZE in bytes (~4x the output per chunk on average);
    // a chunk whose slot fills stops at a flush point and is resumed (GZC_SOFT)
    uint64_t cap64 = ch * GZ_SLOT_RATIO;
    const uint64_t slot_budget = std::max<uint64_t>(8ull * isize, 256ull << 20);
    if (CT * cap64 * 2 > slot_budget) cap64 = std::max<uint64_t>(2 * ch, slot_budget / (2 * CT));
    const uint32_t cap = (uint32_t)cap64;
    static const bool dbg = std::getenv("SDL_GZ_DEBUG") != nullptr;  // diagnostic: phase times to stderr
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms_since = [&](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(now() - t).count();
    };
    const auto t_begin = now();
    int redos = 0;
    try {  // device memory for the chunked path; without it the one-wave path decodes the member
    h->zc_nominal.ensure(CT);
    h->zc_found.ensure(CT);
    h->zc_start.ensure(CT);
    h->zc_hdr.ensure(CT);
    h->zc_end.ensure(CT);
    h->zc_endhdr.ensure(CT);
    h->zc_pos.ensure(CT);
    h->zc_list.ensure(CT);
    h->zc_tgt.ensure(CT);
    h->zc_next.ensure(CT);
    h->zc_len.ensure(CT);
    h->zc_flags.ensure(CT);
    h->zc_order.ensure(CT);
    h->zc_crc.ensure(CT);
    h->zc_shift.ensure(CT);
    h->zc_status.ensure(CT);
    h->zc_rstatus.ensure(1);
    h->zc_slots.ensure((size_t)CT * cap);
    } catch (const HipError &) {
        (void)hipGetLastError();  // (clear the allocation failure so later launches do not report it)
        return;
    }
    std::vector<uint64_t> nominal(CT, GZ_NO_BIT), start(CT, GZ_NO_BIT), hdr(CT, GZ_NO_BIT), end(CT, 0),
        endhdr(CT, 0);
    std::vector<uint32_t> clen(CT, 0), flags(CT, 0), tgt(CT, 0), next(CT, ~0u);
    std::vector<int32_t> status(CT, GZ_OK);
    nominal[0] = 0;
    for (uint64_t c = 1; c < C0; ++c) nominal[c] = 8 * (ma + c * ch);
    for (uint64_t c = 0; c < C0; ++c) tgt[c] = (uint32_t)(c + 1);
    HIP_TRY(hipMemcpyAsync(h->zc_nominal.p, nominal.data(), C0 * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(h->zc_tgt.p, tgt.data(), C0 * 4, hipMemcpyHostToDevice, st));
    if (dbg) {
        h->zc_stats.ensure(3 * C0);
        HIP_TRY(hipMemsetAsync(h->zc_stats.p, 0, 3 * C0 * 4, st));
    }
    if (C0 > 1)
        HIP_TRY(launch_gz_find(d_gz, ma, mz, h->zc_nominal.p + 1, C0 - 1, 8 * GZ_FIND_SPAN * ch, h->zc_found.p + 1,
                               dbg ? h->zc_stats.p : nullptr, st));
    HIP_TRY(hipMemcpyAsync(start.data() + 1, h->zc_found.p + 1, (C0 - 1) * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const double t_find = ms_since(t_begin);
    if (dbg && C0 > 1) {
        std::vector<uint32_t> sv(3 * (C0 - 1));
        HIP_TRY(hipMemcpy(sv.data(), h->zc_stats.p, sv.size() * 4, hipMemcpyDeviceToHost));
        double m[4] = {0, 0, 0, 0};
        uint32_t mx[4] = {0, 0, 0, 0};
        uint64_t nf = 0;
        for (uint64_t c = 0; c + 1 < C0; ++c) {
            nf += start[c + 1] == GZ_NO_BIT;
            const uint32_t v[4] = {sv[3 * c], sv[3 * c + 1] & 4095u, sv[3 * c + 1] >> 12, sv[3 * c + 2]};
            for (int k = 0; k < 4; ++k) {
                m[k] += v[k];
                mx[k] = std::max(mx[k], v[k]);
            }
        }
        fprintf(stderr, "[gz find] per chunk: stages mean %.1f max %u, full checks mean %.1f max %u, "
                "scan kticks mean %.0f max %u, check kticks mean %.0f max %u; %llu without a start\n",
                m[0] / (C0 - 1), mx[0], m[1] / (C0 - 1), mx[1], m[2] / (C0 - 1), mx[2], m[3] / (C0 - 1), mx[3],
                (unsigned long long)nf);
    }
    start[0] = GZ_START_HEADER;
    for (uint64_t c = 0; c < C0; ++c) hdr[c] = start[c];  // searched starts are block boundaries
    HIP_TRY(hipMemcpyAsync(h->zc_found.p, start.data(), 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(h->zc_start.p, start.data(), C0 * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(h->zc_hdr.p, hdr.data(), C0 * 8, hipMemcpyHostToDevice, st));
    GzChunkArgs a{};
    a.ma = ma;
    a.mz = mz;
    a.list = h->zc_list.p;
    a.start_bit = h->zc_start.p;
    a.hdr_bit = h->zc_hdr.p;
    a.nominal = h->zc_nominal.p;
    a.found = h->zc_found.p;
    a.n_chunks = (uint32_t)C0;
    a.tgt0 = h->zc_tgt.p;
    a.slots = h->zc_slots.p;
    a.cap = cap;
    a.end_bit = h->zc_end.p;
    a.end_hdr = h->zc_endhdr.p;
    a.next = h->zc_next.p;
    a.len = h->zc_len.p;
    a.flags = h->zc_flags.p;
    a.status = h->zc_status.p;
    // (i) every chunk with a start, at once
    std::vector<uint32_t> list;
    for (uint64_t c = 0; c < C0; ++c)
        if (start[c] != GZ_NO_BIT) list.push_back((uint32_t)c);
    HIP_TRY(hipMemcpyAsync(h->zc_list.p, list.data(), list.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_inflate_chunks(d_gz, a, list.size(), st));
    HIP_TRY(hipMemcpyAsync(end.data(), h->zc_end.p, C0 * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(endhdr.data(), h->zc_endhdr.p, C0 * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(next.data(), h->zc_next.p, C0 * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(clen.data(), h->zc_len.p, C0 * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(flags.data(), h->zc_flags.p, C0 * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(status.data(), h->zc_status.p, C0 * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const double t_decode = ms_since(t_begin);
    // (ii) the hand-overs in stream order; a chunk whose slot filled up is continued
    // by a new chunk from its last flush point
    auto resume_from = [&](uint64_t r, uint64_t from, uint64_t from_hdr) {
        start[r] = from;
        hdr[r] = from_hdr;
        uint32_t d = 1;  // the first searched chunk whose search began past `from`
        while (d < C0 && nominal[d] <= from) ++d;
        tgt[r] = d;
        const uint32_t one = (uint32_t)r;
        HIP_TRY(hipMemcpyAsync(h->zc_start.p + r, &start[r], 8, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(h->zc_hdr.p + r, &hdr[r], 8, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(h->zc_tgt.p + r, &tgt[r], 4, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(h->zc_list.p, &one, 4, hipMemcpyHostToDevice, st));
        HIP_TRY(launch_inflate_chunks(d_gz, a, 1, st));
        ++redos;
        HIP_TRY(hipMemcpyAsync(&end[r], h->zc_end.p + r, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&endhdr[r], h->zc_endhdr.p + r, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&next[r], h->zc_next.p + r, 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&clen[r], h->zc_len.p + r, 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&flags[r], h->zc_flags.p + r, 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&status[r], h->zc_status.p + r, 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    };
    std::vector<uint32_t> order;
    std::vector<uint64_t> pos;
    uint64_t C = C0, total = 0;
    int32_t err = GZ_OK;
    bool done = false;
    for (uint64_t c = 0;;) {
        if (status[c] != GZ_OK) {
            err = status[c];
            break;
        }
        order.push_back((uint32_t)c);
        pos.push_back(total);
        total += clen[c];
        if (flags[c] & GZC_FINAL) {
            done = true;
            break;
        }
        if (flags[c] & GZC_SOFT) {
            if (C >= CT) {
                err = GZ_E_OVER;
                break;
            }
            const uint64_t r = C++;
            resume_from(r, end[c], endhdr[c]);
            c = r;
            continue;
        }
        if (next[c] >= C0) {  // (a chunk stops only at a hand-over, the final block or a full slot)
            err = GZ_E_STALL;
            break;
        }
        c = next[c];
    }
    if (err == GZ_OK && !done) err = GZ_E_TRUNC;
    if (err == GZ_OK) {  // the trailer right behind the final block, and ISIZE
        const uint64_t t = (end[order.back()] + 7) >> 3;
        if (t + 8 > mz) err = GZ_E_TRUNC;
        else if (t + 8 != mz) err = GZ_E_TRAIL;
        else if (total != isize) err = GZ_E_SIZE;
    }
    if (err == GZ_E_OVER || err == GZ_E_STALL) return;  // (chunk slots exhausted: the one-wave path decodes it)
    if (err != GZ_OK) {
        const int32_t v = err | GZ_VERIFIED;
        HIP_TRY(hipMemcpyAsync(h->z_status.p + m, &v, 4, hipMemcpyHostToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));  // (v is on this stack)
        return;
    }
    // (iii) window chain, bytes + CRC per chunk, the member's CRC
    const uint64_t no = order.size();
    h->zc_windows.ensure((size_t)no * 32768);
    const uint64_t ngroups = (no + gz_window_group(no) - 1) / gz_window_group(no);
    h->zc_gmaps.ensure((size_t)ngroups * 32768);
    h->zc_gwin.ensure((size_t)ngroups * 32768);
    HIP_TRY(hipMemcpyAsync(h->zc_order.p, order.data(), no * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(h->zc_pos.p, pos.data(), no * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(h->zc_rstatus.p, 0, 4, st));
    static const X2N x2n = make_x2n();
    const double t_walk = ms_since(t_begin);
    HIP_TRY(launch_gz_windows(h->zc_slots.p, cap, h->zc_order.p, h->zc_len.p, no, h->zc_windows.p, h->zc_gmaps.p,
                              h->zc_gwin.p, st));
    if (dbg) HIP_TRY(hipStreamSynchronize(st));
    const double t_win = ms_since(t_begin);
    HIP_TRY(launch_gz_resolve(h->zc_slots.p, cap, h->zc_order.p, h->zc_len.p, h->zc_pos.p, no, h->zc_windows.p,
                              h->z_out.p + ooff_m, h->zc_crc.p, h->zc_shift.p, x2n, h->zc_rstatus.p, st));
    if (dbg) HIP_TRY(hipStreamSynchronize(st));
    const double t_res = ms_since(t_begin);
    HIP_TRY(launch_gz_crc_fold(h->zc_crc.p, h->zc_shift.p, no, d_gz + mz - 8, h->zc_rstatus.p, h->z_status.p + m, st));
    HIP_TRY(hipStreamSynchronize(st));  // (order / pos are host vectors)
    if (dbg) {
        int soft = 0;
        for (uint32_t c : order) soft += (flags[c] & GZC_SOFT) != 0;
        fprintf(stderr, "[gz chunked] %llu B member: %llu chunks of %llu B, %zu decoded at once, %d resumed, %llu in "
                "order (%d stopped full); ms: find %.2f decode %.2f walk %.2f windows %.2f resolve %.2f fold %.2f\n",
                (unsigned long long)len, (unsigned long long)C0, (unsigned long long)ch, list.size(), redos,
                (unsigned long long)no, soft, t_find, t_decode - t_find, t_walk - t_decode, t_win - t_walk,
                t_res - t_win, ms_since(t_begin) - t_res);
    }
}

namespace {
// sdl_gzip_inflate_device, members [d_member_offsets[m], d_member_ends[m]) when d_member_ends is
// given (device, u64[n]; else [offsets[m], offsets[m + 1]))
int gzip_inflate_impl(sdl_batcher *h, const uint8_t *d_gz, uint64_t gz_len, const uint64_t *d_member_offsets,
                      const uint64_t *d_member_ends, uint64_t n_members, void *stream, sdl_inflated *out) {
    if (!h || !out || (n_members && (!d_gz || !d_member_offsets))) return fail(SDL_ERR_ARG, "null argument");
    if (gz_len >= (1ull << 32)) return fail(SDL_ERR_CAPACITY, "gzip buffer must be < 4 GiB per call");
    if (n_members >= (1ull << 31)) return fail(SDL_ERR_CAPACITY, "too many gzip members in one call");
    if (((uintptr_t)d_gz & 15u) != 0) return fail(SDL_ERR_ARG, "d_gz must be 16-byte aligned");
    try {
        hipStream_t st = stream ? (hipStream_t)stream : h->stream;
        const size_t n = (size_t)n_members;
        h->z_size.ensure(n + 1);
        h->z_off.ensure(n + 1);
        h->z_tcrc.ensure(n + 1);
        h->z_status.ensure(n + 1);
        h->z_total.ensure(1);
        h->z_bad.ensure(2);
        h->scan_tmp.ensure((size_t)scan_tmp_words(std::max<int64_t>((int64_t)n, 1)) + 1);
        HIP_TRY(hipMemsetAsync(h->z_total.p, 0, sizeof(unsigned long long), st));
        unsigned long long total = 0;
        if (n) {
            HIP_TRY(launch_gz_size(d_gz, gz_len, d_member_offsets, n_members, h->z_size.p, h->z_status.p, h->z_total.p, st,
                                   d_member_ends));
            HIP_TRY(launch_exclusive_scan(h->z_size.p, h->z_off.p, (int64_t)n, h->scan_tmp.p, st));
            HIP_TRY(hipMemcpyAsync(&total, h->z_total.p, sizeof(total), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
        }
        // the trailers' sizes are untrusted until decoded: bound the arena, never the kernel's writes
        if (total >= (1ull << 32) - 64) return fail(SDL_ERR_CAPACITY, "gzip members inflate to >= 4 GiB in one call");
        h->z_out.ensure((size_t)total + 48);
        HIP_TRY(hipMemsetAsync(h->z_out.p + total, 0, 32, st));
        uint32_t bad[2] = {0, 0xFFFFFFFFu};
        if (n) {  // large members first, in chunks (they leave GZ_VERIFIED statuses)
            std::vector<uint64_t> mo(n + 1), me(n);
            HIP_TRY(hipMemcpyAsync(mo.data(), d_member_offsets, (d_member_ends ? n : n + 1) * 8, hipMemcpyDeviceToHost, st));
            if (d_member_ends) HIP_TRY(hipMemcpyAsync(me.data(), d_member_ends, n * 8, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            if (!d_member_ends)
                for (size_t m = 0; m < n; ++m) me[m] = mo[m + 1];
            std::vector<uint64_t> big;
            for (size_t m = 0; m < n; ++m)
                if (me[m] > mo[m] && me[m] - mo[m] >= GZ_SPLIT_MIN && me[m] <= gz_len) big.push_back(m);
            if (!big.empty()) {
                std::vector<uint32_t> sz(n), oo(n);
                std::vector<int32_t> zs(n);
                HIP_TRY(hipMemcpyAsync(sz.data(), h->z_size.p, n * 4, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipMemcpyAsync(oo.data(), h->z_off.p, n * 4, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipMemcpyAsync(zs.data(), h->z_status.p, n * 4, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                for (uint64_t m : big)
                    if (zs[m] == GZ_OK) inflate_chunked(h, d_gz, m, mo[m], me[m], sz[m], oo[m], st);
            }
        }
        if (n) {
            HIP_TRY(hipMemcpyAsync(h->z_bad.p, bad, sizeof(bad), hipMemcpyHostToDevice, st));
            HIP_TRY(launch_inflate(d_gz, d_member_offsets, n_members, h->z_off.p, h->z_out.p, h->z_status.p, h->z_tcrc.p, st,
                                   d_member_ends));
            static const X2N x2n = make_x2n();
            HIP_TRY(launch_gz_crc(h->z_off.p, h->z_out.p, n_members, h->z_tcrc.p, x2n, h->z_status.p, h->z_bad.p, st));
            HIP_TRY(hipMemcpyAsync(bad, h->z_bad.p, sizeof(bad), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
#ifdef SDL_STAMPS
            print_gz_cycles();
#endif
        }
        std::memset(out, 0, sizeof(*out));
        out->d_out = h->z_out.p;
        out->d_member_out = h->z_off.p;
        out->d_status = h->z_status.p;
        out->out_bytes = total;
        out->n_members = n_members;
        out->n_bad = bad[0];
        if (bad[0]) {
            int32_t s = 0;
            HIP_TRY(hipMemcpy(&s, h->z_status.p + bad[1], sizeof(s), hipMemcpyDeviceToHost));
            return fail(SDL_ERR_DATA, "gzip member " + std::to_string(bad[1]) + ": " + gz_reason(s) + " (" +
                                          std::to_string(bad[0]) + " of " + std::to_string(n_members) +
                                          " members failed)");
        }
        return SDL_OK;
    } catch (HipError &e) {
        return fail(SDL_ERR_HIP, e.what());
    } catch (std::exception &e) {
        return fail(SDL_ERR_ARG, e.what());
    }
}
}  // namespace

int sdl_gzip_inflate_device(sdl_batcher *h, const uint8_t *d_gz, uint64_t gz_len, const uint64_t *d_member_offsets,
                            uint64_t n_members, void *stream, sdl_inflated *out) {
    return gzip_inflate_impl(h, d_gz, gz_len, d_member_offsets, nullptr, n_members, stream, out);
}

int sdl_gzip_inflate_first_device(sdl_batcher *h, const uint8_t *d_gz, uint64_t gz_len, const uint64_t *d_file_offsets,
                                  uint64_t n_files, void *stream, sdl_inflated *out) {
    if (!h || !out || (n_files && (!d_gz || !d_file_offsets))) return fail(SDL_ERR_ARG, "null argument");
    if (n_files >= (1ull << 31)) return fail(SDL_ERR_CAPACITY, "too many gzip files in one call");
    try {
        hipStream_t st = stream ? (hipStream_t)stream : h->stream;
        const size_t n = (size_t)n_files;
        if (n == 0) return gzip_inflate_impl(h, d_gz, gz_len, d_file_offsets, nullptr, 0, stream, out);
        std::vector<uint64_t> fo(n + 1), from(n), ends(n);
        HIP_TRY(hipMemcpyAsync(fo.data(), d_file_offsets, (n + 1) * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        for (size_t f = 0; f < n; ++f) {
            if (fo[f + 1] < fo[f] || fo[f + 1] > gz_len) return fail(SDL_ERR_ARG, "file offsets out of order or range");
            from[f] = fo[f] + 19;  // a member is >= 20 bytes: header 10, a final block >= 2, trailer 8
        }
        h->z_from.ensure(n);
        h->z_mend.ensure(n);
        // The first member of file f ends at the next offset where a member header could start, or at
        // the file's end.  A candidate inside the member's own DEFLATE data fails its decode (the
        // range ends early); the file then retries from the next candidate.  Every try decodes every
        // file again (such candidates are rare: ~2^-27 per compressed byte).
        for (int attempt = 0;; ++attempt) {
            for (size_t f = 0; f < n; ++f) ends[f] = fo[f + 1];
            HIP_TRY(hipMemcpyAsync(h->z_from.p, from.data(), n * 8, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(h->z_mend.p, ends.data(), n * 8, hipMemcpyHostToDevice, st));
            HIP_TRY(launch_gz_next_header(d_gz, gz_len, d_file_offsets, n, h->z_from.p,
                                          reinterpret_cast<unsigned long long *>(h->z_mend.p), st));
            HIP_TRY(hipMemcpyAsync(ends.data(), h->z_mend.p, n * 8, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            const int rc = gzip_inflate_impl(h, d_gz, gz_len, d_file_offsets, h->z_mend.p, n_files, stream, out);
            if (rc == SDL_ERR_CAPACITY && attempt < 63) {
                // A range that ends at a candidate inside its member's DEFLATE data read its "ISIZE"
                // from 4 arbitrary bytes, which the 1032:1 bound no longer rejects once the range
                // is a few MB: the sizes overflowed the arena.  Advance the candidate-ended files
                // with the largest sizes until the rest fits, and try again (a real first member
                // this large could not be inflated in one call anyway).
                std::vector<uint32_t> sz(n);
                HIP_TRY(hipMemcpy(sz.data(), h->z_size.p, n * 4, hipMemcpyDeviceToHost));
                unsigned long long tot = 0;
                std::vector<size_t> cand;
                for (size_t f = 0; f < n; ++f) {
                    tot += sz[f];
                    if (ends[f] < fo[f + 1]) cand.push_back(f);
                }
                std::sort(cand.begin(), cand.end(), [&](size_t x, size_t y) { return sz[x] > sz[y]; });
                bool moved = false;
                for (size_t f : cand) {
                    if (tot < (1ull << 32) - 64) break;
                    tot -= sz[f];
                    from[f] = ends[f];
                    moved = true;
                }
                if (moved) continue;
            }
            if (rc != SDL_ERR_DATA || attempt >= 63) return rc;
            std::vector<int32_t> zs(n);
            HIP_TRY(hipMemcpy(zs.data(), h->z_status.p, n * 4, hipMemcpyDeviceToHost));
            bool again = false;
            for (size_t f = 0; f < n; ++f) {
                const int32_t s = zs[f] & 0xFFFF;
                // a failure that a later end can change: not the header, and not a stream that ended
                // before the range (trailing bytes with no member header: the limit of this mode)
                if (s != GZ_OK && s != GZ_E_HEADER && s != GZ_E_HCRC && s != GZ_E_RANGE && s != GZ_E_TRAIL &&
                    ends[f] < fo[f + 1]) {
                    from[f] = ends[f];
                    again = true;
                }
            }
            if (!again) return rc;
        }
    } catch (HipError &e) {
        return fail(SDL_ERR_HIP, e.what());
    } catch (std::exception &e) {
        return fail(SDL_ERR_ARG, e.what());
    }
}

int sdl_gzip_split_members(const uint8_t *gz, uint64_t len, uint64_t *offsets, uint64_t cap, uint64_t *n_members) {
    if ((!gz && len) || !n_members) return fail(SDL_ERR_ARG, "null argument");
    // BGZF: FEXTRA with subfield SI1 'B' SI2 'C' SLEN 2 holding the member size - 1
    auto bsize = [&](uint64_t a) -> uint64_t {
        if (a + 18 > len || gz[a] != 0x1f || gz[a + 1] != 0x8b || gz[a + 2] != 8 || !(gz[a + 3] & 4)) return 0;
        const uint64_t xlen = (uint64_t)gz[a + 10] | (uint64_t)gz[a + 11] << 8;
        for (uint64_t q = a + 12; q + 4 <= a + 12 + xlen && q + 4 <= len;) {
            const uint64_t sl = (uint64_t)gz[q + 2] | (uint64_t)gz[q + 3] << 8;
            if (gz[q] == 'B' && gz[q + 1] == 'C' && sl == 2 && q + 6 <= len)
                return ((uint64_t)gz[q + 4] | (uint64_t)gz[q + 5] << 8) + 1;
            q += 4 + sl;
        }
        return 0;
    };
    std::vector<uint64_t> off{0};
    if (len) {
        uint64_t a = 0, b;
        while (a < len && (b = bsize(a)) != 0 && a + b <= len) {
            a += b;
            off.push_back(a);
        }
        if (a < len) {
            if (off.size() > 1) return fail(SDL_ERR_DATA, "BGZF member at byte " + std::to_string(a) + " has no block size");
            off.push_back(len);  // not BGZF: the file is one member
        }
    }
    *n_members = off.size() - 1;
    if (!offsets || cap < off.size()) return fail(SDL_ERR_CAPACITY, "offsets needs n_members + 1 entries");
    std::memcpy(offsets, off.data(), off.size() * sizeof(uint64_t));
    return SDL_OK;
}

namespace {

struct FramePlaneDesc {
    const char *name;
    const void *src;
    uint32_t width;
    bool f32;
    bool filled_rows_only;  // BertData.label: one entry per filled row
    bool flat;              // Vec<u32> (SingleClass `label`): one list of B (filled) items
};

// list of `n` items of `item` bytes each: "](" items ["e(" per 1000] "e", or "]" when empty
uint64_t list_bytes(uint64_t n, uint64_t item) { return n ? 3 + n * item + 2 * (n / 1000) : 1; }

// lays out one frame (the plane_rows rows of each plane); returns its size
uint64_t frame_layout(FrameParams &fp, const FramePlaneDesc *d, int np, const uint32_t *plane_rows, bool last) {
    uint64_t pos = 4;  // PROTO 3, EMPTY_DICT, MARK
    for (int p = 0; p < np; ++p) {
        FramePlane &P = fp.plane[p];
        const uint32_t n = (uint32_t)std::strlen(d[p].name);
        P.key_len = 5 + n + (P.flat ? 0 : 2);
        P.key[0] = 'X';
        for (int i = 0; i < 4; ++i) P.key[1 + i] = (uint8_t)(n >> (8 * i));
        std::memcpy(P.key + 5, d[p].name, n);
        if (!P.flat) {
            P.key[5 + n] = ']';
            P.key[6 + n] = '(';
        }
        (last ? P.off_last : P.off_full) = pos + P.key_len;
        pos += 5 + n + (P.flat ? (last ? P.row_bytes_last : P.row_bytes) : list_bytes(plane_rows[p], P.row_bytes));
    }
    return pos + 2;  // SETITEMS, STOP
}

}  // namespace

int sdl_pickle_frames_device(sdl_batcher *h, const sdl_device_rows *rows, uint64_t n_rows, int flush_partial,
                             void *stream, sdl_frames *out) {
    if (!h || !rows || !out) return fail(SDL_ERR_ARG, "null argument");
    const int task = h->cfg.task;
    const uint64_t B = (uint64_t)h->cfg.batch_size, S = (uint64_t)h->cfg.sequence_length;
    const uint64_t LW = (uint64_t)rows->label_width;
    if (B == 0 || S == 0) return fail(SDL_ERR_ARG, "batch_size and sequence_length must be > 0");
    const uint64_t rem = n_rows % B, n_frames = n_rows / B + (flush_partial && rem ? 1 : 0);
    if (n_frames * B > rows->rows_capacity)
        return fail(SDL_ERR_ARG, "n_rows exceeds the rows the device planes hold");
    const bool bert = task == SDL_TASK_MLM || task == SDL_TASK_MULTI_LABEL || task == SDL_TASK_SINGLE_CLASS;
    FramePlaneDesc d[4];
    int np = 0;
    d[np++] = {"input_ids", rows->input_ids, (uint32_t)S, false, false, false};
    d[np++] = {"attention_mask", rows->attention_mask, (uint32_t)S, false, false, false};
    if (bert) d[np++] = {"token_type_ids", rows->token_type_ids, (uint32_t)S, false, false, false};
    if (task == SDL_TASK_MULTI_LABEL)
        d[np++] = {"labels", rows->labels_f32, (uint32_t)LW, true, true, false};
    else if (task == SDL_TASK_SINGLE_CLASS)  // bert_data.rs:118-121: "label": Vec<u32>
        d[np++] = {"label", rows->labels, 1, false, true, true};
    else
        d[np++] = {"labels", rows->labels, (uint32_t)LW, false, bert, false};
    for (int p = 0; p < np; ++p)
        if (!d[p].src && n_frames) return fail(SDL_ERR_ARG, std::string("device plane missing: ") + d[p].name);
    try {
        FrameParams fp{};
        fp.n_planes = np;
        fp.B = (uint32_t)B;
        fp.n_frames = n_frames;
        uint32_t full_rows[4], last_rows[4];
        const bool partial = n_frames && n_frames * B > n_rows;
        for (int p = 0; p < np; ++p) {
            FramePlane &P = fp.plane[p];
            const uint32_t ew = d[p].f32 ? 9 : 5;
            const uint64_t filled_last = partial && d[p].filled_rows_only ? rem : B;
            P.src = d[p].src;
            P.is_f32 = d[p].f32;
            P.flat = d[p].flat;
            if (P.flat) {  // one list per frame of the B (last: filled) values
                P.width = (uint32_t)B;
                P.width_last = (uint32_t)filled_last;
                P.frame_stride = B;
                full_rows[p] = P.rows_full = 1;
                last_rows[p] = P.rows_last = 1;
            } else {
                P.width = P.width_last = d[p].width;
                P.frame_stride = B * d[p].width;
                full_rows[p] = P.rows_full = (uint32_t)B;
                last_rows[p] = P.rows_last = (uint32_t)filled_last;
            }
            P.row_bytes = (uint32_t)list_bytes(P.width, ew);
            P.row_bytes_last = (uint32_t)list_bytes(P.width_last, ew);
        }
        fp.frame_bytes = frame_layout(fp, d, np, full_rows, false);
        fp.last_frame_bytes = frame_layout(fp, d, np, last_rows, true);
        const uint64_t total = n_frames ? (n_frames - 1) * fp.frame_bytes + fp.last_frame_bytes : 0;
        uint8_t *dst = nullptr;
        if (h->f_dest) {
            if (!h->f_dry && (size_t)total > h->f_dest_cap) return fail(SDL_ERR_CAPACITY, "frames exceed the destination");
            dst = h->f_dest;
        } else if (!h->f_dry) {
            DevBuf<uint8_t> &fo = *h->f_target;
            fo.ensure((size_t)total + 16);
            dst = fo.p;
        }
        fp.out = dst;
        hipStream_t st = stream ? (hipStream_t)stream : h->stream;
        if (!h->f_dry && n_frames) HIP_TRY(launch_frames(fp, st));
        std::memset(out, 0, sizeof(*out));
        out->d_frames = dst;
        out->n_frames = n_frames;
        out->frame_bytes = fp.frame_bytes;
        out->last_frame_bytes = n_frames ? fp.last_frame_bytes : 0;
        out->total_bytes = total;
        return SDL_OK;
    } catch (HipError &e) {
        return fail(SDL_ERR_HIP, e.what());
    } catch (std::exception &e) {
        return fail(SDL_ERR_ARG, e.what());
    }
}

// ---- End to end, host to host (north_star's path) ------------------------------
// Host JSON lines -> H2D -> JsonText -> tokenize + mask -> serde_pickle frames ->
// D2H -> sink, in chunks cut at line ends, on three streams: chunk k's frames
// copy out (x_out) while chunk k + 1 is copied in (x_in) and computed (the
// handle's stream).  Rows short of a batch at the end of a chunk are carried
// (device to device) to the front of the next chunk's rows, so the frames are
// exactly those of the whole buffer in one call: every full batch, then the
// flushed partial one when flush_partial.  Record indices (RNG keys) continue
// across chunks from cfg.first_record.
int sdl_json_to_frames(sdl_batcher *h, const uint8_t *jsonl, uint64_t len, uint64_t chunk_bytes, int flush_partial,
                       sdl_frame_sink sink, void *user, sdl_json_frames_stats *stats) {
    if (!h || (!jsonl && len)) return fail(SDL_ERR_ARG, "null argument");
    const int task = h->cfg.task;
    if (task != SDL_TASK_MLM && task != SDL_TASK_CLM && task != SDL_TASK_SPAN)
        return fail(SDL_ERR_UNSUPPORTED, "sdl_json_to_frames: JSON lines carry text only (mlm, clm, span)");
    if (chunk_bytes == 0) chunk_bytes = (uint64_t)8 << 20;
    if (chunk_bytes >= (1ull << 31)) return fail(SDL_ERR_CAPACITY, "chunk_bytes must be < 2 GiB");
    try {
        const auto t_start = std::chrono::steady_clock::now();
        if (!h->x_in) HIP_TRY(hipStreamCreateWithFlags(&h->x_in, hipStreamNonBlocking));
        if (!h->x_out) HIP_TRY(hipStreamCreateWithFlags(&h->x_out, hipStreamNonBlocking));
        for (auto &e : h->x_ev)
            if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        // per slot (chunk k uses slot k & 1): H2D done, rows of the chunk ready, frames written
        hipEvent_t *e_h2d = h->x_ev, *e_rows = h->x_ev + 2, *e_frames = h->x_ev + 4;
        const hipStream_t sc = h->stream;
        const uint64_t B = (uint64_t)h->cfg.batch_size, S = (uint64_t)h->cfg.sequence_length;
        const uint64_t LW = (uint64_t)h->P.label_width;
        const bool tt = h->with_tt();
        // chunks end at a '\n' (the last one at len); the first is a quarter chunk so the
        // copy-out stream starts early
        std::vector<uint64_t> cut{0};
        constexpr int64_t head_div = 4;
        while (cut.back() < len) {
            uint64_t e = cut.back() + (cut.size() == 1 ? std::max<uint64_t>(chunk_bytes / head_div, 4096) : chunk_bytes);
            if (e >= len) { cut.push_back(len); break; }
            const void *nl = std::memchr(jsonl + e, '\n', (size_t)(len - e));
            cut.push_back(nl ? (uint64_t)((const uint8_t *)nl - jsonl) + 1 : len);
        }
        const size_t nch = cut.size() - 1;
        // pinned input is copied in directly; pageable input is staged through pinned slots
        bool pinned_in = false;
        {
            hipPointerAttribute_t pa;
            if (len && hipPointerGetAttributes(&pa, jsonl) == hipSuccess && pa.type == hipMemoryTypeHost)
                pinned_in = true;
            (void)hipGetLastError();
        }
        // pinned input: every chunk's H2D is queued up front (one copy each, into its own region
        // followed by 32 zero bytes), so no chunk's input waits behind an earlier chunk's D2H
        std::vector<uint64_t> region(nch + 1, 0);
        for (size_t k = 0; k < nch; ++k) region[k + 1] = region[k] + ((cut[k + 1] - cut[k] + 32 + 255) & ~(uint64_t)255);
        if (pinned_in && nch) {
            while (h->x_in_ev.size() < nch) {
                hipEvent_t e;
                HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                h->x_in_ev.push_back(e);
            }
            h->x_json_all.ensure((size_t)region[nch]);
            HIP_TRY(hipMemsetAsync(h->x_json_all.p, 0, (size_t)region[nch], h->x_in));
            for (size_t k = 0; k < nch; ++k) {
                HIP_TRY(hipMemcpyAsync(h->x_json_all.p + region[k], jsonl + cut[k], (size_t)(cut[k + 1] - cut[k]),
                                       hipMemcpyHostToDevice, h->x_in));
                HIP_TRY(hipEventRecord(h->x_in_ev[k], h->x_in));
            }
        }
        uint64_t carry = 0, carry_at = 0, records = 0, lines = 0, invalid = 0, frames_total = 0, bytes_total = 0;
        uint64_t rows_total = 0, text_total = 0;
        struct Pending {
            bool live = false;
            uint64_t n_frames = 0, frame_bytes = 0, last_bytes = 0, total = 0;
        } pend[2];
        bool used[2] = {false, false};
        double hw[4] = {0, 0, 0, 0};
        auto now = [] { return std::chrono::steady_clock::now(); };
        auto since = [&](std::chrono::steady_clock::time_point t) {
            return std::chrono::duration<double>(now() - t).count();
        };
        auto deliver = [&](int slot) -> int {  // frames of the chunk in slot, once written to host memory
            Pending &q = pend[slot];
            if (!q.live) return 0;
            const auto t0 = now();
            HIP_TRY(hipEventSynchronize(e_frames[slot]));
            hw[3] += since(t0);
            const uint8_t *f = h->x_pin_out[slot].p;
            for (uint64_t i = 0; i < q.n_frames; ++i) {
                const uint64_t nb = i + 1 == q.n_frames ? q.last_bytes : q.frame_bytes;
                if (sink && sink(user, f, nb) != 0) return fail(SDL_ERR_STATE, "sdl_json_to_frames: sink stopped");
                f += nb;
            }
            q.live = false;
            return 0;
        };
        for (size_t k = 0; k <= nch; ++k) {
            const bool last = k == nch;  // the final pass only flushes the carried rows
            const int slot = (int)(k & 1);
            const uint64_t a = last ? len : cut[k], n = last ? 0 : cut[k + 1] - cut[k];
            // this slot's previous frames (chunk k - 2) leave first: its buffers are reused
            if (int rc = deliver(slot)) return rc;
            uint64_t G = 0;
            sdl_device_rows rows{};
            if (n) {
                const uint8_t *d_json;
                if (pinned_in) {
                    d_json = h->x_json_all.p + region[k];
                    HIP_TRY(hipStreamWaitEvent(sc, h->x_in_ev[k], 0));
                } else {
                    h->x_json[slot].ensure((size_t)n + 32);
                    if (used[slot]) HIP_TRY(hipEventSynchronize(e_h2d[slot]));
                    h->x_pin_in[slot].ensure((size_t)n + 32);
                    par_copy(h->x_pin_in[slot].p, jsonl + a, (size_t)n);
                    std::memset(h->x_pin_in[slot].p + n, 0, 32);
                    HIP_TRY(hipMemcpyAsync(h->x_json[slot].p, h->x_pin_in[slot].p, (size_t)n + 32,
                                           hipMemcpyHostToDevice, h->x_in));
                    HIP_TRY(hipEventRecord(e_h2d[slot], h->x_in));
                    used[slot] = true;
                    HIP_TRY(hipStreamWaitEvent(sc, e_h2d[slot], 0));
                    d_json = h->x_json[slot].p;
                }
                sdl_json_text jt;
                auto t0 = now();
                if (int rc = sdl_json_text_device(h, d_json, n, sc, &jt)) return rc;  // syncs sc
                hw[0] += since(t0);
                t0 = now();
                lines += jt.n_lines;
                invalid += jt.n_invalid;
                text_total += jt.text_bytes;
                if (int rc = sdl_process_device(h, jt.d_text, jt.text_bytes, jt.d_offsets, jt.n_records,
                                                h->cfg.first_record + records, sc, &rows))
                    return rc;
                records += jt.n_records;
                uint32_t g32 = 0;
                h->pin_u32_err = 0;
                HIP_TRY(hipMemcpyAsync(&g32, rows.d_rows, 4, hipMemcpyDeviceToHost, sc));
                if (rows.d_tokenize_errors)
                    HIP_TRY(hipMemcpyAsync(&h->pin_u32_err, rows.d_tokenize_errors, 4, hipMemcpyDeviceToHost, sc));
                HIP_TRY(hipStreamSynchronize(sc));
                hw[1] += since(t0);
                if (h->pin_u32_err)
                    throw CapacityError("t5 tokenizer capacity exceeded (flags " + std::to_string(h->pin_u32_err) + ")");
                G = g32;
            }
            // this pass's rows in its slot's planes: the carried rows (from the other slot), then the chunk's
            const uint64_t have = carry + G;
            const uint64_t cap = have + B;
            h->x_ids[slot].ensure((size_t)(cap * S));
            h->x_am[slot].ensure((size_t)(cap * S));
            if (tt) h->x_tt[slot].ensure((size_t)(cap * S));
            h->x_lab[slot].ensure((size_t)(cap * LW));
            const int o = slot ^ 1;
            if (carry) {
                HIP_TRY(hipMemcpyAsync(h->x_ids[slot].p, h->x_ids[o].p + carry_at * S, carry * S * 4,
                                       hipMemcpyDeviceToDevice, sc));
                HIP_TRY(hipMemcpyAsync(h->x_am[slot].p, h->x_am[o].p + carry_at * S, carry * S * 4,
                                       hipMemcpyDeviceToDevice, sc));
                if (tt)
                    HIP_TRY(hipMemcpyAsync(h->x_tt[slot].p, h->x_tt[o].p + carry_at * S, carry * S * 4,
                                           hipMemcpyDeviceToDevice, sc));
                HIP_TRY(hipMemcpyAsync(h->x_lab[slot].p, h->x_lab[o].p + carry_at * LW, carry * LW * 4,
                                       hipMemcpyDeviceToDevice, sc));
            }
            if (G) {
                HIP_TRY(hipMemcpyAsync(h->x_ids[slot].p + carry * S, rows.input_ids, G * S * 4, hipMemcpyDeviceToDevice,
                                       sc));
                HIP_TRY(hipMemcpyAsync(h->x_am[slot].p + carry * S, rows.attention_mask, G * S * 4,
                                       hipMemcpyDeviceToDevice, sc));
                if (tt)
                    HIP_TRY(hipMemcpyAsync(h->x_tt[slot].p + carry * S, rows.token_type_ids, G * S * 4,
                                           hipMemcpyDeviceToDevice, sc));
                HIP_TRY(hipMemcpyAsync(h->x_lab[slot].p + carry * LW, rows.labels, G * LW * 4, hipMemcpyDeviceToDevice,
                                       sc));
            }
            rows_total += G;
            uint64_t nframe_rows = have / B * B;
            const bool flush_now = last && flush_partial && have % B;
            if (flush_now) {  // the partial batch: initial values past its rows
                const uint64_t r0 = have, r1 = (have / B + 1) * B;
                HIP_TRY(hipMemsetD32Async(h->x_ids[slot].p + r0 * S, 0, (r1 - r0) * S, sc));
                HIP_TRY(hipMemsetD32Async(h->x_am[slot].p + r0 * S, 1, (r1 - r0) * S, sc));
                if (tt) HIP_TRY(hipMemsetD32Async(h->x_tt[slot].p + r0 * S, 0, (r1 - r0) * S, sc));
                HIP_TRY(hipMemsetD32Async(h->x_lab[slot].p + r0 * LW, -100, (r1 - r0) * LW, sc));
                nframe_rows = have;
            }
            HIP_TRY(hipEventRecord(e_rows[slot], sc));
            if (nframe_rows) {
                const auto t2 = now();
                sdl_device_rows x{};
                x.input_ids = h->x_ids[slot].p;
                x.attention_mask = h->x_am[slot].p;
                x.token_type_ids = tt ? h->x_tt[slot].p : nullptr;
                x.labels = h->x_lab[slot].p;
                x.rows_capacity = (have / B + 1) * B;
                x.label_width = (int32_t)LW;
                // size the frames, write them into this slot's device buffer from the copy-out
                // stream and copy them to pinned host memory there: the next chunk's kernels
                // overlap the copy.  (Writing mapped pinned host memory from the kernel itself
                // measured ~25 GB/s of shader stores over PCIe against ~56 GB/s for the DMA copy.)
                // The frames kernel runs on the compute stream, so the copy-out stream holds
                // nothing but the copies and they run back to back.
                sdl_frames fr;
                h->f_dry = true;
                int rc = sdl_pickle_frames_device(h, &x, nframe_rows, flush_now ? 1 : 0, h->x_out, &fr);
                h->f_dry = false;
                if (rc) return rc;
                h->x_pin_out[slot].ensure((size_t)fr.total_bytes + 16);
                h->x_frames[slot].ensure((size_t)fr.total_bytes + 16);
                h->f_dest = h->x_frames[slot].p;
                h->f_dest_cap = h->x_frames[slot].cap;
                rc = sdl_pickle_frames_device(h, &x, nframe_rows, flush_now ? 1 : 0, sc, &fr);
                h->f_dest = nullptr;
                h->f_dest_cap = 0;
                if (rc) return rc;
                HIP_TRY(hipEventRecord(e_rows[slot], sc));  // frames written
                HIP_TRY(hipStreamWaitEvent(h->x_out, e_rows[slot], 0));
                HIP_TRY(hipMemcpyAsync(h->x_pin_out[slot].p, h->x_frames[slot].p, (size_t)fr.total_bytes,
                                       hipMemcpyDeviceToHost, h->x_out));
                HIP_TRY(hipEventRecord(e_frames[slot], h->x_out));
                pend[slot] = Pending{true, fr.n_frames, fr.frame_bytes, fr.last_frame_bytes, fr.total_bytes};
                frames_total += fr.n_frames;
                bytes_total += fr.total_bytes;
                hw[2] += since(t2);
            }
            // rows short of a batch are carried into the next pass (copied from this slot)
            const uint64_t rem = have - have / B * B;
            carry = last ? 0 : rem;
            carry_at = have - rem;
            // hand over the previous chunk's frames while this one's are written
            if (int rc = deliver(slot ^ 1)) return rc;
        }
        for (int sl = 0; sl < 2; ++sl)
            if (int rc = deliver(sl)) return rc;
        if (stats) {
            std::memset(stats, 0, sizeof(*stats));
            stats->n_lines = lines;
            stats->n_invalid = invalid;
            stats->n_records = records;
            stats->text_bytes = text_total;
            stats->n_rows = rows_total;
            stats->n_frames = frames_total;
            stats->frame_bytes = bytes_total;
            stats->n_chunks = nch;
            stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
            for (int i = 0; i < 4; ++i) stats->host_wait[i] = hw[i];
        }
        return SDL_OK;
    } catch (HipError &e) {
        return fail(SDL_ERR_HIP, e.what());
    } catch (CapacityError &e) {
        return fail(SDL_ERR_CAPACITY, e.what());
    } catch (std::exception &e) {
        return fail(SDL_ERR_ARG, e.what());
    }
}

int sdl_device_to_host(sdl_batcher *h, void *dst, const void *src, size_t bytes, void *stream) {
    if (!h || (bytes && (!dst || !src))) return fail(SDL_ERR_ARG, "null argument");
    if (!bytes) return SDL_OK;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(SDL_ERR_HIP, std::string("sdl_device_to_host: ") + hipGetErrorString(e));
    return SDL_OK;
}

int sdl_tokenizer_info_get(const char *tokenizer_path, const char *data_dir, sdl_tokenizer_info *out) {
    if (!tokenizer_path || !out) return fail(SDL_ERR_ARG, "null argument");
    try {
        HostTokenizer t;
        load_tokenizer(tokenizer_path, data_dir ? std::string(data_dir) : default_data_dir(), t);
        std::memset(out, 0, sizeof(*out));
        out->kind = t.kind;
        out->vocab_size = (int32_t)t.pieces.size();
        out->n_added = (int32_t)t.added.size();
        out->unk_id = t.unk_id;
        out->eos_id = t.eos_id;
        int mx = 0;
        for (auto &p : t.pieces) mx = std::max(mx, (int)p.size());
        out->max_piece_bytes = mx;
        out->word_table_entries = t.kind == TOK_WORDPIECE ? 0 : t.word_table_entries;
        return SDL_OK;
    } catch (std::exception &e) {
        return fail(SDL_ERR_IO, e.what());
    }
}

int sdl_set_profiling(sdl_batcher *h, int enable) {
    if (!h) return fail(SDL_ERR_ARG, "null argument");
    h->profiling = enable != 0;
    return SDL_OK;
}

int sdl_stage_times(sdl_batcher *h, const char **names, float *ms, int cap) {
    if (!h) return fail(SDL_ERR_ARG, "null argument");
    if (!h->profiling) return fail(SDL_ERR_STATE, "profiling not enabled");
    if (hipEventSynchronize(h->ev[h->n_stages]) != hipSuccess) return fail(SDL_ERR_HIP, "event sync failed");
    int n = std::min(cap, h->n_stages);
    for (int i = 0; i < n; ++i) {
        float t = 0.f;
        if (hipEventElapsedTime(&t, h->ev[i], h->ev[i + 1]) != hipSuccess) return fail(SDL_ERR_HIP, "event time");
        if (names) names[i] = h->stage_names[i];
        if (ms) ms[i] = t;
    }
    return n;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Several GPUs, one record stream (the reference runs one Batcher task,
// rust/src/tasks/runner_simple.rs:68-112): byte-balanced contiguous record ranges, one
// handle + stream + host thread per device, masks keyed by the global record index.
// ---------------------------------------------------------------------------
int sdl_shard_records(const uint64_t *offsets, uint64_t n_records, uint32_t n_shards, uint64_t *bounds) {
    if (!offsets || !bounds || n_shards == 0) return fail(SDL_ERR_ARG, "null argument or zero shards");
    for (uint64_t r = 0; r < n_records; ++r)
        if (offsets[r + 1] < offsets[r]) return fail(SDL_ERR_ARG, "offsets must be non-decreasing");
    const uint64_t base = offsets[0], total = offsets[n_records] - base;
    bounds[0] = 0;
    for (uint32_t k = 1; k < n_shards; ++k) {
        // the first record starting at or past k * total / n_shards
        const unsigned __int128 t = (unsigned __int128)total * k / n_shards;
        const uint64_t want = base + (uint64_t)t;
        bounds[k] = (uint64_t)(std::lower_bound(offsets, offsets + n_records, want) - offsets);
        if (bounds[k] < bounds[k - 1]) bounds[k] = bounds[k - 1];
    }
    bounds[n_shards] = n_records;
    return SDL_OK;
}

struct sdl_multi {
    std::vector<sdl_batcher *> h;
    uint64_t next_record = 0;  // global index of the next call's first record
    bool poisoned = false;     // a shard failed: the others committed their part of that push
    ~sdl_multi() {
        for (sdl_batcher *x : h) sdl_batcher_destroy(x);
    }
};

int sdl_multi_create(const sdl_config *cfg, const char *tokenizer_path, const char *data_dir, const int32_t *devices,
                     uint32_t n_devices, sdl_multi **out) {
    if (!cfg || !devices || !out || n_devices == 0) return fail(SDL_ERR_ARG, "null argument or no devices");
    std::unique_ptr<sdl_multi> m(new sdl_multi());
    m->next_record = cfg->first_record;
    for (uint32_t k = 0; k < n_devices; ++k) {
        sdl_config c = *cfg;
        c.device = devices[k];
        sdl_batcher *h = nullptr;
        if (int rc = sdl_batcher_create(&c, tokenizer_path, data_dir, &h)) return rc;
        m->h.push_back(h);
    }
    *out = m.release();
    return SDL_OK;
}

void sdl_multi_destroy(sdl_multi *m) { delete m; }

sdl_batcher *sdl_multi_handle(sdl_multi *m, uint32_t k) { return m && k < m->h.size() ? m->h[k] : nullptr; }

int sdl_multi_push_many(sdl_multi *m, const uint8_t *arena, const uint64_t *offsets, size_t n_records,
                        const uint32_t *labels, const uint64_t *label_offsets, size_t *n_emitted) {
    if (!m || !offsets || (!arena && n_records && offsets[n_records])) return fail(SDL_ERR_ARG, "null argument");
    if (offsets[0] != 0) return fail(SDL_ERR_ARG, "offsets must start at 0");
    if (m->poisoned) return fail(SDL_ERR_STATE, "an earlier push failed on a shard; the stream is not resumable");
    const uint32_t n = (uint32_t)m->h.size();
    std::vector<uint64_t> bounds(n + 1);
    if (int rc = sdl_shard_records(offsets, n_records, n, bounds.data())) return rc;
    std::vector<int> rcs(n, SDL_OK);
    std::vector<std::string> errs(n);
    std::vector<size_t> emitted(n, 0);
    auto run = [&](uint32_t k) {
        const uint64_t r0 = bounds[k], r1 = bounds[k + 1];
        sdl_batcher *h = m->h[k];
        if (hipSetDevice(h->device) != hipSuccess) {
            rcs[k] = SDL_ERR_HIP;
            errs[k] = "hipSetDevice failed";
            return;
        }
        std::vector<uint64_t> off(r1 - r0 + 1);
        for (uint64_t r = r0; r <= r1; ++r) off[r - r0] = offsets[r] - offsets[r0];
        h->first_override = (int64_t)(m->next_record + r0);
        rcs[k] = sdl_batcher_push_many(h, arena ? arena + offsets[r0] : nullptr, off.data(), (size_t)(r1 - r0), labels,
                                       label_offsets ? label_offsets + r0 : nullptr, &emitted[k]);
        h->first_override = -1;
        if (rcs[k] != SDL_OK) errs[k] = g_err;  // (the message is thread-local)
        // the handle's own counter follows its records; the next call's shard starts are global
    };
    std::vector<std::thread> th;
    for (uint32_t k = 1; k < n; ++k) th.emplace_back(run, k);
    run(0);
    for (auto &t : th) t.join();
    if (n_emitted)  // also on failure: the shards that succeeded have queued these
        for (uint32_t k = 0; k < n; ++k) n_emitted[k] = rcs[k] == SDL_OK ? emitted[k] : 0;
    for (uint32_t k = 0; k < n; ++k)
        if (rcs[k] != SDL_OK) {
            m->poisoned = true;
            return fail(rcs[k], "shard " + std::to_string(k) + ": " + errs[k]);
        }
    m->next_record += n_records;
    return SDL_OK;
}
