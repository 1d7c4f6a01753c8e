// kernels.hpp -- host-side launchers of the gfx950 kernels (all asynchronous on `st`).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace sdl {

// pipeline.hip: per chunk, the record ranges touching its window (3 words per chunk)
// (rb1: also write the one-segment record bounds {0, R} there; zero1: a word to zero)
hipError_t launch_chunk_ranges(const uint64_t *off, int64_t R, int64_t N, uint32_t *ranges, hipStream_t st,
                               uint32_t *rb1 = nullptr, uint32_t *zero1 = nullptr, const void *copy_src = nullptr,
                               void *copy_dst = nullptr, size_t copy_bytes = 0);

// tokenize_wordpiece.hip: text arena -> per-chunk token lists + boundary offsets
// (after launch_chunk_ranges), for chunks [c_begin, c_end) (c_end < 0: all).
hipError_t launch_wordpiece_chunks(const DevTok &T, const uint8_t *text, int64_t N, const uint64_t *off, int64_t R,
                                   uint32_t *ranges, uint32_t *tokc, uint32_t *chunk_cnt, uint32_t *rec_local,
                                   hipStream_t st, int64_t c_begin = 0, int64_t c_end = -1);

// tokenize_bpe.hip: same outputs for a byte-level BPE (gpt2) tokenizer.  Pieces
// longer than 64 bytes go through `long_list` (capacity long_cap) and are
// merged by a second kernel in `scratch` (u16 per text byte); their chunk
// entry is LONG_MARK | list index (k_compact_tokens expands it).
struct BpeLong {
    uint64_t pos;   // first byte
    uint32_t len;   // bytes (0 until known)
    uint32_t chunk; // owning chunk
    uint32_t k;     // ids after merging
    uint32_t pad;
};
hipError_t launch_bpe_chunks(const DevTok &T, const uint8_t *text, int64_t N, const uint64_t *off, int64_t R,
                             const uint32_t *ranges, uint32_t *tokc, uint32_t *chunk_cnt, uint32_t *chunk_ent,
                             uint32_t *rec_local, uint32_t *long_count, BpeLong *long_list, uint32_t long_cap,
                             uint16_t *scratch, uint32_t *err, hipStream_t st);

// tokenize_unigram.hip: t5 (Precompiled + Unigram).  Same chunk outputs as the
// other tokenizers; long items (non-ASCII / long words) are finished by two
// follow-up kernels into `pool` ([k, ids...] per item), their chunk entry
// LONG_MARK | pool offset (k_compact_tokens expands it).
struct UniWork {
    uint32_t *counters;   // [0] long items [1] - [2] pool words used [3] huge items [4] stage-2 items
    uint4 *items;         // long items (chunk, tokc entry, prel, raw length or 0)
    uint32_t item_cap;
    uint32_t *pool;
    uint32_t pool_cap;
    uint4 *huge;          // items past a lane's scratch
    uint32_t huge_cap;
    uint4 *items2;        // stage-2 long items (normalized past LONG_NORM1)
    uint32_t items2_cap;
    uint8_t *scratch;     // unigram_scratch_bytes(lane_blocks, huge_blocks)
    int lane_blocks, huge_blocks;
    uint32_t *err;        // bit 1 ids overflow, 2 pool, 3 item lists, 4 item too large
    // (optional) a second stream and two events: the wide-job Viterbi and the long items run
    // there beside the narrow-job Viterbi (they touch other entries; their counts add atomically)
    hipStream_t side;
    hipEvent_t ev_fork, ev_join;
};
size_t unigram_scratch_bytes(int lane_blocks, int huge_blocks);
hipError_t launch_unigram_chunks(const DevTok &T, const uint8_t *text, int64_t N, const uint64_t *off, int64_t R,
                                 const uint32_t *ranges, uint32_t *tokc, uint32_t *chunk_cnt, uint32_t *chunk_ent,
                                 uint32_t *rec_local, const UniWork &W, hipStream_t st);

#ifdef SDL_STAMPS
void print_phase_cycles();  // diagnostic builds only
void print_uni_cycles();
void print_long_cycles();
void print_vit_cycles();
void print_gz_cycles();
void print_bpe_cycles();
#endif

// json_text.hip: the provider's JsonText filter (newline count + scan, newline
// positions, parse and decode: lane per line below JL_MIN bytes, wave per line above)
hipError_t launch_json_nl_count(const uint8_t *buf, int64_t len, uint32_t *cnt, uint32_t *base, uint32_t *scan_tmp,
                                hipStream_t st);
// the newline list holds `cap` positions; the count comes back in full, so a
// caller whose list was too small grows it and writes it again
hipError_t launch_json_nl_write(const uint8_t *buf, int64_t len, const uint32_t *base, uint32_t *nl, uint32_t cap,
                                hipStream_t st);
hipError_t launch_json_nl_tail(const uint32_t *total, const uint32_t *nl, uint32_t cap, uint32_t *out, hipStream_t st);
hipError_t launch_json_parse(const uint8_t *buf, int64_t len, const uint32_t *nl, uint32_t n_nl, int64_t n_lines,
                             uint32_t *out_len, uint32_t *is_rec, uint2 *span, uint32_t *n_invalid, hipStream_t st);
hipError_t launch_json_write(const uint8_t *buf, int64_t len, const uint32_t *nl, uint32_t n_nl, int64_t n_lines,
                             const uint32_t *is_rec, const uint2 *span, const uint32_t *toff, const uint32_t *ridx,
                             uint8_t *text, uint64_t *offsets, hipStream_t st);

// inflate.hip: gzip members -> their bytes back to back (the provider's GzipDecoder).
// Per-member status (GZ_*); the output of member m is [ooff[m], ooff[m+1]).
enum : int32_t {
    GZ_OK = 0,
    GZ_E_RANGE = 1,   // member range outside the buffer
    GZ_E_TRUNC = 2,   // input ends inside the member
    GZ_E_HEADER = 3,  // not a gzip/deflate header, or reserved flags
    GZ_E_HCRC = 4,    // header CRC16 mismatch
    GZ_E_BTYPE = 5,   // block type 3
    GZ_E_STORED = 6,  // stored block LEN != ~NLEN
    GZ_E_CODES = 7,   // bad dynamic code lengths (sets, repeats, symbol counts, no end-of-block)
    GZ_E_CODE = 8,    // invalid literal/length or distance code
    GZ_E_FAR = 9,     // distance too far back
    GZ_E_OVER = 10,   // more output than the trailer's ISIZE
    GZ_E_SIZE = 11,   // output length != ISIZE
    GZ_E_TRAIL = 12,  // bytes after the member's trailer
    GZ_E_CRC = 13,    // CRC-32 mismatch
    GZ_E_STALL = 14,  // the decoder made no progress (a guard: unreachable with the shipped batch size)
    GZ_VERIFIED = 0x100  // (internal) a member finished by the chunked path: k_inflate skips it, k_gz_crc counts it
};
struct X2N {
    uint32_t t[32];  // x^(2^k) mod P (zlib's x2n_table)
};
// mend (or null): member m is [moff[m], mend[m]) instead of [moff[m], moff[m + 1]) -- a file's
// first member inside the file's range (sdl_gzip_inflate_first_device)
hipError_t launch_gz_size(const uint8_t *in, uint64_t in_len, const uint64_t *moff, uint64_t n, uint32_t *size,
                          int32_t *status, unsigned long long *total, hipStream_t st, const uint64_t *mend = nullptr);
hipError_t launch_inflate(const uint8_t *in, const uint64_t *moff, uint64_t n, const uint32_t *ooff, uint8_t *out,
                          int32_t *status, uint32_t *tcrc, hipStream_t st, const uint64_t *mend = nullptr);
// Per file f (bytes [foff[f], foff[f + 1])): next[f] = min(next[f], the first offset p > from[f] in the
// file where a gzip member header could start (1f 8b 08, no reserved flag bits)) -- where the file's
// first member may end; next[] holds the file end on entry
hipError_t launch_gz_next_header(const uint8_t *in, uint64_t in_len, const uint64_t *foff, uint64_t n,
                                 const uint64_t *from, unsigned long long *next, hipStream_t st);
hipError_t launch_gz_crc(const uint32_t *ooff, const uint8_t *out, uint64_t n, const uint32_t *tcrc, const X2N &x2n,
                         int32_t *status, uint32_t *bad, hipStream_t st);

// One large gzip member inflated in parallel (inflate.hip, "chunked members"):
// the deflate stream is cut into chunks of the compressed bytes; each chunk after
// the first starts at the first dynamic-block header a search finds at or past
// its nominal start, decodes into a 16-bit slot (bytes < 256, 256 + w = byte w
// of the 32 KiB window before the chunk), and hands over at the first block start
// that equals a later chunk's searched start (decoding through wrong or missing
// picks); the host follows the hand-overs in stream order (a chunk whose slot
// fills stops at its last flush point, inside a block, and a new chunk resumes
// there), the window chain is resolved, then every chunk's bytes are written and
// CRC'd in parallel.
constexpr uint64_t GZ_NO_BIT = ~0ull;            // chunk: no start found
constexpr uint64_t GZ_START_HEADER = ~0ull - 1;  // chunk: start at the member's gzip header
enum : uint32_t { GZC_FINAL = 1, GZC_SOFT = 2 };  // chunk flags: final block reached; stopped: slot full
struct GzChunkArgs {
    uint64_t ma, mz;            // the member's byte range in `in`
    const uint32_t *list;       // blockIdx.x -> chunk index
    const uint64_t *start_bit;  // per chunk: absolute bit in `in`, or GZ_START_HEADER
    const uint64_t *hdr_bit;    // per chunk: the header of the block it starts in (== start_bit at a boundary)
    const uint64_t *nominal;    // per searched chunk: where its search began (bits)
    const uint64_t *found;      // per searched chunk: its start (GZ_NO_BIT: none)
    uint32_t n_chunks;          // searched chunks
    const uint32_t *tgt0;       // per chunk: the first chunk it may hand over to
    uint16_t *slots;            // per chunk: `cap` values
    uint32_t cap;
    uint64_t *end_bit;          // out: where the chunk stopped: a block boundary, or (GZC_SOFT, slot
                                //      full) a flush point inside a block ...
    uint64_t *end_hdr;          // out: ... with that block's header bit (else == end_bit)
    uint32_t *next;             // out: the chunk it handed over to (~0u: none)
    uint32_t *len;              // out: values produced
    uint32_t *flags;            // out: GZC_*
    int32_t *status;            // out: GZ_*
    const uint64_t *mend;       // (one-wave members) member m ends at mend[m] instead of moff[m + 1], or null
};
// first dynamic-block header at or past nominal[c] (bits), searching `span` bits;
// found[c] = its bit or GZ_NO_BIT
// (stats: null, or per chunk {search steps, full checks, code-length symbols decoded}, zeroed; diagnostic)
hipError_t launch_gz_find(const uint8_t *in, uint64_t ma, uint64_t mz, const uint64_t *nominal, uint64_t n_chunks,
                          uint64_t span, uint64_t *found, uint32_t *stats, hipStream_t st);
hipError_t launch_inflate_chunks(const uint8_t *in, const GzChunkArgs &a, uint64_t n_list, hipStream_t st);
// windows[j] = the 32 KiB before chunk order[j + 1], for the chunks in stream order;
// gmaps (u16) / gwin (u8) hold 32 KiB per group of gz_window_group(n_order) chunks
inline uint64_t gz_window_group(uint64_t n) {
    uint64_t g = 1;
    while (g * g < n) ++g;
    return g;
}
hipError_t launch_gz_windows(const uint16_t *slots, uint32_t cap, const uint32_t *order, const uint32_t *len,
                             uint64_t n_order, uint8_t *windows, uint16_t *gmaps, uint8_t *gwin, hipStream_t st);
// every ordered chunk's bytes to out + pos[j] (markers through windows[j - 1]), its CRC-32
// and x^(8 len) mod P; status[0] = GZ_E_FAR when a marker reaches before the stream
hipError_t launch_gz_resolve(const uint16_t *slots, uint32_t cap, const uint32_t *order, const uint32_t *len,
                             const uint64_t *pos, uint64_t n_order, const uint8_t *windows, uint8_t *out,
                             uint32_t *crc, uint32_t *shift, const X2N &x2n, int32_t *status, hipStream_t st);
// the member's CRC-32 from the chunks' (crc, shift), checked against the trailer's CRC-32 (the
// 4 bytes at `trailer`, the member's end - 8); writes mstatus[0] = (status[0], or GZ_E_CRC) | GZ_VERIFIED
hipError_t launch_gz_crc_fold(const uint32_t *crc, const uint32_t *shift, uint64_t n_order, const uint8_t *trailer,
                              const int32_t *status, int32_t *mstatus, hipStream_t st);

// pipeline.hip
// out[0..n) = exclusive prefix sum of in[0..n) (+ *carry_in when given),
// out[n] = total.  tmp needs scan_tmp_words(n) words.  carry_in may alias out[0].
int64_t scan_tmp_words(int64_t n);
hipError_t launch_exclusive_scan(const uint32_t *in, uint32_t *out, int64_t n, uint32_t *tmp, hipStream_t st,
                                 const uint32_t *carry_in = nullptr);

// Pipelined segments: the arena's chunks are cut into K host-known ranges
// [cb[k], cb[k+1]); record range k is [rb[k], rb[k+1]) -- the records whose ids
// all lie in chunks < cb[k+1] (rb[K] = R) -- computed on the device from the
// chunk ranges, so nothing syncs with the host.
constexpr int MAX_SEGMENTS = 16;
struct SegChunks {
    int64_t cb[MAX_SEGMENTS + 1];
    int K;
};
hipError_t launch_seg_bounds(const uint32_t *ranges, const SegChunks &sc, int64_t R, uint32_t *rb, hipStream_t st);
// out[rb[k] .. rb[k+1]] = exclusive scan of in[rb[k] .. rb[k+1]) carried from out[rb[k]]
// (0 for k == 0); one workgroup.
hipError_t launch_scan_range(const uint32_t *in, uint32_t *out, const uint32_t *rb, int k, hipStream_t st);

// long_count == null: no long-piece markers (WordPiece).  Else chunk_ent holds
// each chunk's entry count (markers count 1; chunk_cnt counts ids).
// long_pool != null (unigram): a marker's ids are long_pool[off + 1 ..], count long_pool[off].
hipError_t launch_compact_tokens(const uint32_t *tokc, const uint32_t *chunk_cnt, const uint32_t *chunk_off,
                                 int64_t n_chunks, uint32_t *tok, const uint32_t *long_count,
                                 const uint32_t *chunk_ent, const BpeLong *long_list, const uint16_t *long_scratch,
                                 hipStream_t st, const uint32_t *long_pool = nullptr, int64_t stride = STAGE);


// Which records / rows a launch covers: records [rb[k], rb[k+1]), rows
// [row_off[rb[k]], row_off[rb[k+1]]); the last segment (last != 0) also writes
// the initial values of the rows up to the next multiple of B.
struct SegSel {
    const uint32_t *rb;
    int k;
    int last;
};

// per record: token offset, token count, rows it yields (gen_batcher.rs:69-94)
hipError_t launch_records(const RowParams &P, const uint64_t *off, int64_t R, int64_t N, const uint32_t *chunk_off,
                          int64_t n_chunks, const uint32_t *rec_local, uint32_t *rec_tok, uint32_t *rec_cnt,
                          uint32_t *rec_rows, SegSel sel, hipStream_t st);

// Small pushes, no second round trip: global row g of the call goes to slot
// base + g of the back batch (slots >= B: the next, pre-allocated one), rows
// g < cap only (cap 0: off).  k_rows_direct copies them there and writes
// row_off[0..R] and the two error words to `stat` (mapped pinned host memory) so
// the host needs no D2H copy; for mlm / clm on the small-call path k_rows writes
// them there itself (RowOut.direct) and k_downstream_small writes `stat`.
struct DirectDst {
    int32_t *ids[2], *am[2], *tt[2], *lab[2];  // back batch, next batch (device-mapped host)
    uint32_t base, cap, B, pad;
};
struct RowOut {
    int32_t *input_ids, *attention_mask, *token_type_ids, *labels;
    float *labels_f32;
    DirectDst direct;  // (k_rows) rows g < direct.cap go to the host batches; padding rows are skipped
};

// Small calls: chunk scan + compaction + records + row scan + row map in one
// single-workgroup launch (one segment, n_chunks <= SMALL_CHUNKS, R <= 8192).
constexpr int64_t SMALL_CHUNKS = 64;
struct SmallDown {
    const uint32_t *tokc, *chunk_cnt;
    uint32_t *chunk_off, *tok;
    const uint32_t *long_count, *chunk_ent;
    const BpeLong *long_list;
    const uint16_t *long_scratch;
    const uint32_t *long_pool;
    int64_t stride;
    const uint32_t *rec_local;
    uint32_t *rec_tok, *rec_cnt, *rec_rows, *row_off, *row_rec;
    uint32_t *stat;  // or null: row_off[0..R], a zero label-error word and the tokenizer's error word
                     // (mapped host memory, DirectDst)
    const uint32_t *tok_err;  // or null: the Unigram capacity flags (uni_err), copied to stat[R + 2]
    int rows;                 // 1: also the call's rows (k_rows' body) into `out` -- mlm (Philox) / clm
    RowOut out;
};
hipError_t launch_downstream_small(const SmallDown &d, const RowParams &P, const uint64_t *off, int64_t R, int64_t N,
                                   hipStream_t st);

// row -> record map (row_rec needs one word per row)
hipError_t launch_row_map(const uint32_t *row_off, int64_t R, uint32_t *row_rec, SegSel sel, hipStream_t st);

// BertData::put_data + mask_batch for every row (models/bert_data.rs:40-89)
// pipeline.hip: device rows -> finished batches in pinned host memory (the
// host path's D2H).  Segment i copies rows [g0, g0 + n) of every plane to row
// dst of its batch's planes (device-visible host pointers; unused planes null).
struct RowSeg {
    int32_t *ids, *am, *tt, *lab;  // batch planes (host memory, device-mapped)
    uint32_t g0, n, dst, pad;
};
hipError_t launch_rows_to_host(const RowSeg *segs, int n_segs, uint32_t rows_per_seg_max, const int32_t *ids,
                               const int32_t *am, const int32_t *tt, const int32_t *lab, int S, int LW,
                               hipStream_t st);

// (DirectDst: see RowOut)
hipError_t launch_rows_direct(const DirectDst &d, const uint32_t *row_off, int64_t R, const int32_t *ids,
                              const int32_t *am, const int32_t *tt, const int32_t *lab, int S, int LW,
                              const uint32_t *err0, const uint32_t *err1, uint32_t *stat, hipStream_t st);

hipError_t launch_rows(const RowParams &P, const uint32_t *tok, const uint32_t *rec_tok, const uint32_t *rec_cnt,
                       const uint32_t *row_off, const uint32_t *row_rec, SegSel sel, int64_t rows_cap, RowOut out,
                       hipStream_t st,
                       hipStream_t st_late = nullptr);
// rng_mode 1 masks (pipeline.hip): the rows rand_pre_slot names (chunk 0 of every record, chunk 1
// of long ones) from (seed, first_record + r, chunk) alone -- launched beside the tokenizer: swap
// indices (lane per row) into jbuf [2 R, S], then the mask bits into P.mask_bits0 slots
hipError_t launch_mask_rand_rec(const RowParams &P, uint32_t *list, uint32_t *spos, uint16_t *jbuf, uint32_t *bits,
                                hipStream_t st);
// ... and the other rows g of the segment, after the row map: listed (list[0] = count, list[1..] =
// rows; rows_cap + 1 words), then 16 lanes per row, bits into bitsg [rows, S/32]
// BertData MultiLabel labels_f32 plane (bert_data.rs:66-78)
hipError_t launch_multi_labels(const uint32_t *labels, const uint64_t *label_off, const uint32_t *row_rec,
                               const uint32_t *row_off, SegSel sel, int64_t rows_cap, int B, int NL, float *out,
                               uint32_t *err, hipStream_t st);

// T5Data::put_data rows for task=span (models/t5_data.rs:162-226).  With a
// plan (pipeline.hip "Span rows in two phases"): rows_cap x capr entries,
// rows_cap meta words, an overflow row list of rows_cap entries and its count;
// without one, the one-pass kernel.
struct SpanPlan {
    uint2 *tab;
    uint2 *meta;
    int32_t capr;  // plan entries per row: LW / 2 + 2
    uint32_t *ovf_list, *ovf_n;
};
hipError_t launch_rows_span(const RowParams &P, const uint32_t *tok, const uint32_t *rec_tok, const uint32_t *rec_cnt,
                            const uint32_t *row_off, const uint32_t *row_rec, SegSel sel, int64_t rows_cap,
                            RowOut out, uint32_t *err, hipStream_t st, const SpanPlan *plan = nullptr);

hipError_t launch_single_labels(const uint32_t *labels, const uint64_t *label_off, const uint32_t *row_rec,
                                const uint32_t *row_off, SegSel sel, int64_t rows_cap, int B, int32_t *out,
                                uint32_t *err, hipStream_t st);

// transport_frame.hip: the Transport's serde_pickle frames of finished batches
// (zmq_transmit.rs:71) written straight from the device row planes.
struct FramePlane {
    const void *src;     // device plane [rows, width] (int32, or f32 when is_f32)
    uint32_t width;      // elements per row
    uint32_t is_f32;
    uint32_t rows_full;  // rows of this plane in a full frame
    uint32_t rows_last;  // rows in the last frame
    uint32_t row_bytes;  // encoded bytes per row list
    uint32_t key_len;    // bytes of the key segment: 'X' + u32 len + name (+ "](" unless flat)
    uint32_t flat;       // the value is one flat list (Vec<u32>): one "row" per frame, no outer list
    uint32_t width_last;      // row width in the last frame (flat: its filled rows)
    uint32_t row_bytes_last;
    uint32_t rpw;             // rows per wave (set by launch_frames)
    uint64_t frame_stride;    // source elements per frame (B * width; flat: B)
    uint64_t off_full;   // frame offset of row 0 (just past the key segment), full frames
    uint64_t off_last;   // the same in the last frame
    uint8_t key[24];
};
struct FrameParams {
    FramePlane plane[4];
    uint8_t *out;
    uint64_t frame_bytes;       // every frame but the last
    uint64_t last_frame_bytes;
    uint64_t n_frames;
    uint32_t B;                 // rows per batch in the source planes
    int n_planes;
};
hipError_t launch_frames(const FrameParams &fp, hipStream_t st);

}  // namespace sdl
