/*
 * sdl_batcher.h -- C ABI of the MI355X-native Batcher (libsdl_batcher.so).
 *
 * Drop-in boundary for the reference's Batcher stage
 * (andywag/streaming_data_loader @ v1, rust/src/batcher.rs:26-31):
 *
 *     pub trait Batcher { type S; type T;
 *         fn create_sync_batch(&mut self, data: Self::S) -> Option<Self::T>;
 *         fn get_working_batch(&mut self) -> Option<Self::T>; }
 *
 * implemented for the masking tasks by GenTokenizer
 * (rust/src/tasks/gen_batcher.rs:65-98, S = String, T = DataSet) and for the
 * multi-label task by SimpleBatcher (rust/src/models/simple_batcher.rs:31-53).
 * INTEGRATION.md shows the Rust `impl Batcher for GpuBatcher` that binds this
 * header through `extern "C"` so the Provider -> Batcher -> Transport channels
 * (rust/src/tasks/runner_simple.rs:68-112) stay unchanged.
 *
 * Conventions: plain pointers and sizes only; every call returns an int
 * status (SDL_OK = 0, < 0 error; never a panic across the FFI; the message is
 * in sdl_last_error()).  One handle per host thread / GPU; handles are not
 * thread-safe.  Input text is copied in (the caller keeps ownership, as the
 * reference moves the String in); batches are owned by the handle until
 * sdl_batch_release().
 */
#ifndef SDL_BATCHER_H
#define SDL_BATCHER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDL_ABI_VERSION 9

enum {
    SDL_OK = 0,
    SDL_ERR_ARG = -1,         /* bad argument / config (reference: panic!/todo!) */
    SDL_ERR_IO = -2,          /* tokenizer asset unreadable */
    SDL_ERR_HIP = -3,         /* HIP runtime error */
    SDL_ERR_UNSUPPORTED = -4, /* task / tokenizer feature not implemented */
    SDL_ERR_NODEV = -5,       /* no HIP device: the product never falls back to the CPU */
    SDL_ERR_STATE = -6,       /* call out of order */
    SDL_ERR_CAPACITY = -7,    /* input larger than one call supports (>= 4 GiB of text) */
    SDL_ERR_DATA = -8         /* corrupt input the reference's unwrap() panics on (gzip) */
};

/* TaskType -> DataSet selection (rust/src/config.rs:20-62). */
enum {
    SDL_TASK_MLM = 0,        /* BertData, DataSetConfig::Mask   (models/bert_data.rs) */
    SDL_TASK_CLM = 1,        /* GptData,  DataSetConfig::Gpt    (models/gpt_data.rs) */
    SDL_TASK_SPAN = 2,       /* T5Data,   DataSetConfig::Span   (models/t5_data.rs) */
    SDL_TASK_MULTI_LABEL = 3, /* BertData, DataSetConfig::MultiLabel via SimpleBatcher */
    SDL_TASK_SINGLE_CLASS = 4 /* BertData, DataSetConfig::SingleClass via SimpleBatcher
                                 (tasks/single_class/runner.rs:40-49): one Label::Single per record */
};

/* Mirrors TrainingConfig.batch + .dataset_config (rust/src/config.rs:64-72,
 * rust/src/batcher.rs:11-14, rust/src/datasets/dataset_config.rs:7-16) plus the
 * RNG seed that replaces the reference's unseedable thread_rng(). */
typedef struct sdl_config {
    int32_t task;            /* SDL_TASK_* */
    int32_t batch_size;      /* BatchConfig.batch_size */
    int32_t sequence_length; /* BatchConfig.sequence_length */
    int32_t chunk;           /* GenTokenizer.chunk (1 for the masking tasks, masking_runner.rs:55-62) */
    int32_t min_ids;         /* records with fewer framed ids are dropped (gen_batcher.rs:74): 64 */
    int32_t mask_length;     /* DataSetConfig::Mask.mask_length = (S as f32 * 0.15) as usize */
    int32_t mask_id;         /* DataSetConfig::Mask.mask = 103 (masking_cases.rs:60) */
    int32_t number_labels;   /* DataSetConfig::MultiLabel.number_labels */
    double avg_span_gap;     /* DataSetConfig::Span.avg_span_gap  (16.0) */
    double avg_span_size;    /* DataSetConfig::Span.avg_span_size (2.0) */
    uint64_t seed;           /* RNG contract seed */
    uint64_t first_record;   /* global index of this handle's first record (sharding) */
    int32_t device;          /* HIP device ordinal */
    int32_t rng_mode;        /* 0 = the Philox contract (default);
                                1 = the reference's own draws on a per-row StdRng::from_seed(
                                seed | record | chunk, little-endian, zero padded):
                                MLM masks = rand 0.8.5 position_base.shuffle (bert_data.rs:40-43;
                                S <= 2048); span gap / size = rand_distr 0.4.3 StandardNormal,
                                gap then size per pass (t5_data.rs:165-176) */
    int32_t reserved[6];
} sdl_config;

/* A finished batch: DataSet's Serialize view (bert_data.rs:106-145,
 * gpt_data.rs:53-62, t5_data.rs:235-249) as int32 row-major planes. */
typedef struct sdl_batch {
    int32_t rows;            /* rows filled (BertData.index); the MLM `labels` list has this length */
    int32_t batch_size;
    int32_t sequence_length;
    int32_t label_width;     /* S (mlm/clm), S/4 (span), number_labels (multi-label), 1 (single-class) */
    const int32_t *input_ids;      /* [batch_size, sequence_length] */
    const int32_t *attention_mask; /* [batch_size, sequence_length] */
    const int32_t *token_type_ids; /* [batch_size, sequence_length] or NULL (clm/span) */
    const int32_t *labels;         /* [batch_size, label_width] or NULL (multi-label); single-class:
                                      [batch_size, 1], the BertData `label` list = the first `rows` */
    const float *labels_f32;       /* [batch_size, number_labels] (multi-label) or NULL */
    void *owner_;                  /* opaque, for sdl_batch_release */
} sdl_batch;

typedef struct sdl_batcher sdl_batcher;

/* Defaults of the reference masking cases (masking_cases.rs:38-94) for `task`:
 * B=4096 S=128 chunk=1 min_ids=64 mask 15%/103, span 16.0/2.0, 9 labels. */
void sdl_config_default(sdl_config *cfg, int32_t task);

/* get_tokenizer(cfg) + GenTokenizer::new / SimpleBatcher::new
 * (tokenizer_wrapper.rs:162-189, gen_batcher.rs:23-41).  `tokenizer_path` is a
 * HF tokenizer.json (or a WordPiece vocab.txt); `data_dir` holds the Unicode
 * tables (NULL = directory of the library's package data). */
int sdl_batcher_create(const sdl_config *cfg, const char *tokenizer_path, const char *data_dir,
                       sdl_batcher **out);
void sdl_batcher_destroy(sdl_batcher *h);

/* Batcher::create_sync_batch(data) for one record (gen_batcher.rs:69-94 /
 * simple_batcher.rs:35-43).  `labels` are the Label::Multi indices for the
 * multi-label task (ignored otherwise).  Returns 1 and fills *out when this
 * call emits a batch (at most one per call, as the reference), 0 when not. */
int sdl_batcher_push(sdl_batcher *h, const uint8_t *utf8, size_t len, const uint32_t *labels,
                     size_t n_labels, sdl_batch *out);

/* Bulk create_sync_batch over n_records records laid out back to back in
 * `arena` (record r = arena[offsets[r] .. offsets[r+1]), offsets[0] = 0,
 * n_records+1 offsets).  Exactly the batches the reference would emit over the
 * same sequence of calls are queued, in order, for sdl_batcher_next().  For the
 * multi-label task record r's Label::Multi indices are
 * labels[label_offsets[r] .. label_offsets[r+1]) (NULL label_offsets = none). */
int sdl_batcher_push_many(sdl_batcher *h, const uint8_t *arena, const uint64_t *offsets,
                          size_t n_records, const uint32_t *labels, const uint64_t *label_offsets,
                          size_t *n_emitted);
/* Pops the next batch queued by sdl_batcher_push_many: 1 = *out filled, 0 = none. */
int sdl_batcher_next(sdl_batcher *h, sdl_batch *out);
/* Batcher::get_working_batch() (gen_batcher.rs:96-98): pops the front batch
 * (possibly partial, possibly empty).  1 = *out filled, 0 = none left. */
int sdl_batcher_flush(sdl_batcher *h, sdl_batch *out);
void sdl_batch_release(sdl_batch *b);

/* ---- Device-resident bulk path (the measured hot path) -------------------
 * Tokenize + label every record of a device-resident arena in one sequence of
 * kernel launches on `stream` (a hipStream_t; NULL = the handle's stream),
 * without any host synchronisation.  Rows are packed densely in record order:
 * batch b is rows [b*B, (b+1)*B); rows >= *d_rows up to the next multiple of B
 * hold the reference's initial values.  Buffers are owned by the handle and
 * stay valid until the next call.  The global record index of record r (RNG
 * key) is first_record + r. */
typedef struct sdl_device_rows {
    int32_t *input_ids;      /* device [rows_capacity, S] */
    int32_t *attention_mask; /* device [rows_capacity, S] */
    int32_t *token_type_ids; /* device [rows_capacity, S] or NULL */
    int32_t *labels;         /* device [rows_capacity, label_width] */
    float *labels_f32;       /* device [rows_capacity, number_labels] or NULL */
    uint32_t *d_rows;        /* device scalar: rows produced */
    uint32_t *d_record_rows; /* device [n_records]: rows each record produced */
    uint32_t *d_tokens;      /* device scalar: tokenizer ids produced (before framing) */
    uint64_t rows_capacity;
    int32_t label_width;
    uint32_t *d_label_errors; /* device scalar: multi-label -- Label::Multi indices >= number_labels
                                 that were skipped; span -- label writes past the S/4 label width or
                                 sentinel indices >= 100 that were clamped (the reference panics on
                                 both: bert_data.rs:70-72, t5_data.rs:205-216) */
    uint32_t *d_tokenize_errors; /* device scalar (t5 tokenizer), 0 = ok; else bit 1: an item's ids
                                    exceeded their scratch, 2: id pool full, 3: long-item list full,
                                    4: a whitespace-free run longer than 256 KiB normalized (dropped) */
} sdl_device_rows;

int sdl_process_device(sdl_batcher *h, const uint8_t *d_text, uint64_t text_len,
                       const uint64_t *d_offsets, uint64_t n_records, uint64_t first_record,
                       void *stream, sdl_device_rows *out);

/* sdl_process_device for the multi-label task with Label::Multi indices per
 * record: record r's indices are d_labels[d_label_offsets[r] .. d_label_offsets[r+1])
 * (device memory, n_records+1 offsets).  SimpleBatcher::create_sync_batch
 * (simple_batcher.rs:35-43) + BertData MultiLabel (bert_data.rs:66-78). */
int sdl_process_device_labels(sdl_batcher *h, const uint8_t *d_text, uint64_t text_len,
                              const uint64_t *d_offsets, uint64_t n_records, const uint32_t *d_labels,
                              const uint64_t *d_label_offsets, uint64_t first_record, void *stream,
                              sdl_device_rows *out);

/* ---- Provider step: the JsonText filter on the device ----------------------
 * SourceFilter::JsonText over inflated JSON lines (gzip_file_provider.rs:30-50
 * -> provider_util.rs:60-64: serde_json::from_str(line).unwrap(),
 * v["text"].as_str()): every '\n'-separated line whose value is an object with
 * a string member "text" (the last one if repeated) becomes one record, that
 * string unescaped to UTF-8, in a device text arena ready for
 * sdl_process_device.  Lines the reference's unwrap() panics on are skipped and
 * counted.  `d_jsonl` is device memory, 16-byte aligned and readable up to the
 * next multiple of 16 bytes past `len` (< 4 GiB).  The arena and offsets are
 * owned by the handle until the next call; the counts are copied to the host
 * (the call synchronises `stream`). */
typedef struct sdl_json_text {
    uint8_t *d_text;       /* device, 16-byte aligned: records back to back, 16 zero bytes after */
    uint64_t *d_offsets;   /* device [n_records + 1] */
    uint64_t n_records;
    uint64_t text_bytes;   /* = offsets[n_records] */
    uint64_t n_lines;      /* lines seen */
    uint64_t n_invalid;    /* lines the reference would panic on (skipped) */
} sdl_json_text;
int sdl_json_text_device(sdl_batcher *h, const uint8_t *d_jsonl, uint64_t len, void *stream, sdl_json_text *out);

/* ---- Provider step: gzip inflate on the device -----------------------------
 * Replaces the GzipDecoder under the provider's lines (gzip_file_provider.rs:
 * 13-28, async-compression 0.3.14 / flate2 1.0.24 / miniz_oxide 0.5.4): every
 * gzip member (RFC 1952; DEFLATE, RFC 1951) in `d_gz` is inflated by one wave,
 * members in parallel, and its CRC-32 and ISIZE are checked.  Member m is bytes
 * [d_member_offsets[m], d_member_offsets[m+1]) of d_gz (device, u64[n + 1]):
 * one file each (the reference decodes a file's first member), or the BGZF
 * blocks sdl_gzip_split_members finds in one file.  The outputs are written
 * back to back -- the JSON lines sdl_json_text_device takes as is.  d_gz is
 * device memory, 16-byte aligned, gz_len < 4 GiB, total output < 4 GiB.  A
 * corrupt member (where the reference's `next_line().await.unwrap()` panics)
 * makes the call return SDL_ERR_DATA with its index and reason; per-member
 * status codes stay readable in d_status.  The buffers are owned by the handle
 * until the next call; the call synchronises `stream` (the output size comes
 * from the members' trailers before anything is decoded). */
typedef struct sdl_inflated {
    uint8_t *d_out;             /* device, 16-byte aligned, 32 zero bytes after out_bytes */
    uint32_t *d_member_out;     /* device [n_members + 1]: member m's output is [d_member_out[m], [m+1]) */
    int32_t *d_status;          /* device [n_members]: 0 ok, else a GZ_* reason code */
    uint64_t out_bytes;
    uint64_t n_members;
    uint64_t n_bad;             /* members that failed */
} sdl_inflated;
int sdl_gzip_inflate_device(sdl_batcher *h, const uint8_t *d_gz, uint64_t gz_len, const uint64_t *d_member_offsets,
                            uint64_t n_members, void *stream, sdl_inflated *out);

/* The reference-exact variant (opt-in): every range [d_file_offsets[f],
 * d_file_offsets[f+1]) is one FILE, and only its first gzip member is inflated --
 * what async-compression's GzipDecoder with multiple_members off returns
 * (gzip_file_provider.rs:18, 64): `cat a.gz b.gz` yields a's lines, a BGZF file its
 * first block's.  The member's end is found on the device (the next offset where a
 * member header could start, else the file's end; a candidate inside the member's
 * own compressed data fails its decode and the next one is tried).  Output and
 * status as sdl_gzip_inflate_device, one member per file.  Limit: a first member
 * followed by bytes that hold no gzip header (trailing garbage) fails with
 * SDL_ERR_DATA (GZ_E_TRAIL) instead of being ignored. */
int sdl_gzip_inflate_first_device(sdl_batcher *h, const uint8_t *d_gz, uint64_t gz_len, const uint64_t *d_file_offsets,
                                  uint64_t n_files, void *stream, sdl_inflated *out);

/* Host only (no GPU): member byte ranges of one gzip file for
 * sdl_gzip_inflate_device.  BGZF files (every member carries the 'BC' extra
 * subfield with its size, as bgzip writes them) split into their members; any
 * other file is one member (async-compression's GzipDecoder reads the first
 * member of a file).  offsets gets *n_members + 1 entries (capacity `cap`
 * entries; SDL_ERR_CAPACITY with *n_members set when too small). */
int sdl_gzip_split_members(const uint8_t *gz, uint64_t len, uint64_t *offsets, uint64_t cap, uint64_t *n_members);

/* ---- Transport step: batches as serde_pickle frames on the device ----------
 * Replaces serde_pickle::to_vec(&dataset, Default::default()) of each finished
 * DataSet (transport/zmq_transmit.rs:71, serde-pickle 1.1.1) that the Python
 * consumer reads with pickle.loads (python/external_dataset.py:52): the planes
 * of `rows` (from the last sdl_process_device[_labels] call of `h`) become one
 * frame per batch -- PROTO 3, the DataSet's fields in Serialize order
 * (bert_data.rs:106-145, gpt_data.rs:53-62, t5_data.rs:235-249), rows as lists
 * of BININT / BINFLOAT, STOP -- back to back in device memory.  Batches are the
 * n_rows / B full ones plus, when flush_partial and n_rows % B != 0, the
 * partial batch get_working_batch() would flush (its BertData `labels` list
 * holds the filled rows only).  `n_rows` is the value of *rows->d_rows (or
 * fewer rows).  The frames are owned by the handle until the next call; no
 * host synchronisation. */
typedef struct sdl_frames {
    uint8_t *d_frames;         /* device: frame f at f * frame_bytes */
    uint64_t n_frames;
    uint64_t frame_bytes;      /* bytes of every frame but the last */
    uint64_t last_frame_bytes; /* bytes of the last frame */
    uint64_t total_bytes;
} sdl_frames;
int sdl_pickle_frames_device(sdl_batcher *h, const sdl_device_rows *rows, uint64_t n_rows, int flush_partial,
                             void *stream, sdl_frames *out);

/* ---- End to end, host to host: JSON lines in, socket bytes out -------------
 * The reference's Provider -> Batcher -> Transport path for a buffer of
 * inflated JSON lines in host memory (gzip_file_provider.rs:30-50 ->
 * provider_util.rs:60-64 -> create_batch, batcher.rs:33-77 -> zmq_transmit.rs:71):
 * JsonText, tokenize + mask and serde_pickle frames on the device, in chunks of
 * about chunk_bytes (cut at line ends; 0 = 8 MiB) on three streams, so one
 * chunk's frames copy out while the next is copied in and computed.  Every
 * frame is handed to sink(user, frame, bytes) in order (sink may be NULL: the
 * frames still reach host memory); a non-zero return stops the call.  The
 * frames are those of the whole buffer in one sdl_json_text_device +
 * sdl_process_device + sdl_pickle_frames_device call: every full batch (rows
 * short of a batch carry into the next chunk), then the partial batch when
 * flush_partial.  Tasks mlm, clm and span (JSON lines carry no labels). */
typedef int (*sdl_frame_sink)(void *user, const uint8_t *frame, uint64_t bytes);
typedef struct sdl_json_frames_stats {
    uint64_t n_lines, n_invalid, n_records, text_bytes, n_rows, n_frames, frame_bytes, n_chunks;
    double seconds;  /* wall time of the call */
    double host_wait[4];  /* host time in: JsonText (its sizing syncs), tokenize + mask to the row count,
                             frames + copy-out issue, waiting for earlier copies out (delivery) */
} sdl_json_frames_stats;
int sdl_json_to_frames(sdl_batcher *h, const uint8_t *jsonl, uint64_t len, uint64_t chunk_bytes, int flush_partial,
                       sdl_frame_sink sink, void *user, sdl_json_frames_stats *stats);

/* ---- Several GPUs, one record stream ---------------------------------------
 * Records are independent (gen_batcher.rs:69-94 touches only the record's ids and
 * the row cursor), so N Batchers on N contiguous record ranges emit what N
 * reference Batchers (runner_simple.rs:68-112 runs one) would on those shards;
 * masks are keyed by the global record index, so every row equals the row one
 * handle would give over the whole stream.  No collective is involved.
 *
 * Host only: cut records [0, n_records) into n_shards contiguous ranges of about
 * equal bytes -- bounds[k] = the first record starting at or past
 * offsets[0] + k * (offsets[n_records] - offsets[0]) / n_shards, bounds[0] = 0,
 * bounds[n_shards] = n_records (n_shards + 1 entries; a range may be empty). */
int sdl_shard_records(const uint64_t *offsets, uint64_t n_records, uint32_t n_shards, uint64_t *bounds);

typedef struct sdl_multi sdl_multi;
/* One handle (own HIP stream) per entry of devices[0 .. n_devices), cfg->device
 * ignored; a device may repeat.  cfg->first_record is the global index of the
 * first record of the first push. */
int sdl_multi_create(const sdl_config *cfg, const char *tokenizer_path, const char *data_dir,
                     const int32_t *devices, uint32_t n_devices, sdl_multi **out);
void sdl_multi_destroy(sdl_multi *m);
/* sdl_batcher_push_many over one record stream: cut by sdl_shard_records into
 * one shard per handle, every shard pushed into its handle on its own host thread
 * (after hipSetDevice of its device; the calling thread runs shard 0 and is left on
 * devices[0]), shard k's records keyed from the global index of its first record.
 * n_emitted[k] (n_devices entries, may be NULL) = batches shard k queued; pop them
 * with sdl_batcher_next / sdl_batcher_flush on sdl_multi_handle(m, k).  The global
 * record index continues across calls.  When a shard fails, the shards that
 * succeeded have queued their batches: n_emitted is written for every shard either
 * way (0 for a failed one), and the multi handle is poisoned -- later pushes return
 * SDL_ERR_STATE -- since re-pushing the records would duplicate the committed
 * shards' rows. */
int sdl_multi_push_many(sdl_multi *m, const uint8_t *arena, const uint64_t *offsets, size_t n_records,
                        const uint32_t *labels, const uint64_t *label_offsets, size_t *n_emitted);
/* Shard k's handle (also for sdl_process_device on a device-resident shard with
 * first_record = its bound); NULL when k >= n_devices. */
sdl_batcher *sdl_multi_handle(sdl_multi *m, uint32_t k);

/* Copies `bytes` from device memory (e.g. sdl_device_rows planes) to host
 * memory with the handle's HIP runtime, ordered after the handle's work on
 * `stream` (NULL = the handle's stream); returns when the copy is complete. */
int sdl_device_to_host(sdl_batcher *h, void *dst, const void *src, size_t bytes, void *stream);

/* Per-stage device time (ms) of the last sdl_process_device call, measured with
 * hipEvents on the stream the kernels ran on, when enabled. */
int sdl_set_profiling(sdl_batcher *h, int enable);
int sdl_stage_times(sdl_batcher *h, const char **names, float *ms, int cap);

/* Loads and checks a tokenizer on the host only (no GPU needed): what
 * sdl_batcher_create would accept.  kind: 0 WordPiece, 1 byte-level BPE,
 * 2 Unigram (t5). */
typedef struct sdl_tokenizer_info {
    int32_t kind;
    int32_t vocab_size;
    int32_t n_added;            /* added tokens matched on the raw text */
    int32_t unk_id;
    int32_t eos_id;             /* </s> / <|endoftext|> (TokenizerInfo.eos), -1 if none */
    int32_t max_piece_bytes;
    uint64_t word_table_entries; /* device word-table / hash entries */
    int32_t reserved[6];
} sdl_tokenizer_info;
int sdl_tokenizer_info_get(const char *tokenizer_path, const char *data_dir, sdl_tokenizer_info *out);

/* Last error message of the calling thread. */
const char *sdl_last_error(void);
int sdl_abi_version(void);
/* sha256 (hex) of the sources, headers and flags this library was built from
 * (streaming_data_loader_amd/build.py source_hash): proves which build ran. */
const char *sdl_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* SDL_BATCHER_H */
