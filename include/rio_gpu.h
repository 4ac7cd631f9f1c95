/*
 * rio_gpu.h — C ABI of the MI355X recordio block decoder.
 *
 * Drop-in boundary for the reference's v2 scan path (grailbio/base recordio):
 * plain pointers and sizes, no C++ or torch types, no exceptions across the ABI.
 * A Go cgo shim binds these symbols one-to-one.
 *
 * Two layers:
 *  1. Scanner layer — mirrors recordio.NewScanner / NewShardScanner / Scanner
 *     (recordio/scannerv2.go:113-235) and ScannerOpts (scannerv2.go:100-111):
 *     rio_scanner_*.
 *  2. Batch layer — decode a 32 KiB-aligned span of chunks (host or device
 *     resident) into records + item offsets in one call: rio_scan_span,
 *     rio_scan_device. This replaces the per-block loop
 *     ChunkScanner.Scan -> TransformFunc -> parseChunksToItems
 *     (recordio/internal/chunk.go:253-345, recordio/scannerv2.go:53-97, 363-388).
 *  Plus the TransformFunc analogue rio_decode_block (recordio/recordio.go:12)
 *  and the transformer-registry lookup rio_codec_for_transformers
 *  (recordio/registry.go:113-148).
 *
 * Threading: one rio_ctx per OS thread / goroutine; a ctx (and every scanner
 * opened on it) is never used concurrently; each ctx owns its HIP stream(s) on
 * one device. Pointers passed in are not retained past the call (cgo rule).
 */
#ifndef RIO_GPU_H
#define RIO_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RIO_ABI_VERSION 2
#define RIO_CHUNK_SIZE 32768        /* internal.ChunkSize, chunk.go:25 */
#define RIO_CHUNK_HEADER_SIZE 28    /* internal.ChunkHeaderSize, chunk.go:22 */
#define RIO_MAX_CHUNK_PAYLOAD 32740 /* internal.MaxChunkPayloadSize, chunk.go:28 */

/* Block codecs: the untransformer named by the file header (registry.go:113). */
enum rio_codec {
    RIO_CODEC_NONE = 0,  /* idTransform, registry.go:31-39 */
    RIO_CODEC_FLATE = 1, /* recordioflate.FlateUncompress, recordioflate.go:54-65 */
    RIO_CODEC_ZSTD = 2,  /* recordiozstd.zstdUncompress, recordiozstd.go:67-78 */
};
/* A chain of transformers (the header's "transformer" values t0 .. tn-1, 2 <=
 * n <= 4, each flate or zstd): blocks were transformed by t0 first, so they
 * are untransformed tn-1 first, t0 last (registry.go:121-146). As a codec
 * argument: RIO_CODEC_CHAIN(n, t0 | t1 << 2 | t2 << 4 | t3 << 6). Each stage
 * is a launch over the previous stage's output and needs its block sizes on
 * the host, so the async entries (rio_scan_device_async,
 * rio_scan_device_segments_async) run a chain's stages at the call and
 * rio_sync returns their batch (per-block segments and file offsets included).
 * Known divergence (parity with the reference unpinned for chains): the
 * reference's combined untransformer passes the same `scratch` to every stage
 * (registry.go:127-140), so a later stage may write its output over the earlier
 * stage's output while still reading it (zstd.Decompress(scratch, in[0]) with
 * in[0] inside scratch, recordiozstd.go:71-72; FlateUncompress into
 * bytes.Buffer(scratch[:0]), recordioflate.go:54-65). The GPU decodes the clean
 * composition of the stages; the chain test cases are oracle-derived. */
#define RIO_CODEC_CHAIN_FLAG 0x10000
#define RIO_CODEC_CHAIN(n, codes) (RIO_CODEC_CHAIN_FLAG | ((n) << 8) | (codes))

/* Error codes carried in rio_error.code (the reference's error conditions). */
enum rio_err_code {
    RIO_OK = 0,
    RIO_ERR_CHUNK_SIZE = 1,     /* "Invalid chunk size %d"                      chunk.go:334 */
    RIO_ERR_CHUNK_CRC = 2,      /* "Chunk checksum mismatch, expect %d, got %d" chunk.go:341 */
    RIO_ERR_MAGIC_CHANGED = 3,  /* "Magic number changed in the middle..."      chunk.go:274 */
    RIO_ERR_CHUNK_INDEX = 4,    /* "Chunk index mismatch, got %v, expect %v..." chunk.go:279 */
    RIO_ERR_CHUNK_TOTAL = 5,    /* "Chunk nchunk mismatch, got %v, expect %v.." chunk.go:284 */
    RIO_ERR_UNEXPECTED_EOF = 6, /* "unexpected EOF" (truncated chunk)          chunk.go:318 */
    RIO_ERR_BAD_MAGIC = 7,      /* "recordio: invalid magic number: %v"        scannerv2.go:386 */
    RIO_ERR_NITEMS = 8,         /* "...failed to read number of packed items"  scannerv2.go:72 */
    RIO_ERR_ITEM_SIZE = 9,      /* "...failed to read size of packed item %v"  scannerv2.go:86 */
    RIO_ERR_BLOCK_SIZE = 10,    /* "...corrupt block header, got block size"   scannerv2.go:94 */
    RIO_ERR_ITEM_RANGE = 11,    /* wrapped item sizes (the reference panics)   DESIGN.md */
    RIO_ERR_FLATE_CORRUPT = 12, /* "flate: corrupt input before offset %d"     klauspost flate */
    RIO_ERR_FLATE_EOF = 13,     /* "unexpected EOF" from the inflater          */
    RIO_ERR_ZSTD = 14,          /* libzstd error name (DataDog/zstd)           zstd_cgo.go:40 */
    RIO_ERR_ZSTD_EMPTY = 15,    /* "Bytes slice is empty"                      DataDog ErrEmptySlice */
    RIO_ERR_HEADER = 16,        /* header block / header KV errors             scannerv2.go:260-306 */
    RIO_ERR_TRAILER = 17,       /* trailer lookup errors                       scannerv2.go:316-342 */
    RIO_ERR_TRANSFORMER = 18,   /* "Transformer %s not found"                  registry.go:58 */
    RIO_ERR_ARG = 19,           /* invalid argument / sharding                 scannerv2.go:226 */
    RIO_ERR_LEGACY = 20,        /* (unused since v1 files decode natively; kept for ABI stability) */
    RIO_ERR_IO = 21,            /* reader callback failed                      */
    RIO_ERR_LOCATION = 22,      /* "Invalid location %+v, block has only %d items" scannerv2.go:358 */
    RIO_ERR_FALLBACK = 23,      /* transformers this library does not decode: a name other than
                                   flate/zstd, or a chain of more than 4 (registry.go:113-148). Decode the file with
                                   recordio.NewShardScanner; msg is the reference's text for the case the
                                   name is not registered there either ("Transformer %s not found") */
    RIO_ERR_V1_RECORD = 24,     /* v1 record header / read errors (InternalScan): "recordio: crc check
                                   failed - corrupt record header (%v != %v)?", "recordio: failed to read
                                   header: unexpected EOF", "recordio: unreasonably large read record
                                   encountered: %d > %d bytes", "recordio: failed to read record: unexpected
                                   EOF", "recordio: short/long record: %d < %d"
                                                                  deprecated/recordio.go:258-300, 324-334 */
    RIO_ERR_V1_PACKED = 25,     /* v1 packed-record errors (Unpack): "recordio: failed to read crc32",
                                   "...number of packed items exceeds the number of bytes in the record
                                   (%v > %v)", "...crc check failed - corrupt packed record header (%v !=
                                   %v)?", "recordio: offset greater than buf size (%v > %v), ..."
                                   (item count / size varint errors use RIO_ERR_NITEMS / RIO_ERR_ITEM_SIZE,
                                   same text as v2)               deprecated/packer.go:214-272 */
    RIO_ERR_CAPACITY = 98,      /* span or output exceeds the ctx capacity      */
    RIO_ERR_HIP = 99,           /* HIP runtime failure                          */
};

typedef struct rio_error {
    int32_t code;       /* enum rio_err_code */
    int32_t reserved;
    uint64_t file_off;  /* file offset of the failing chunk / block */
    uint64_t a, b, c;   /* detail values (expected/actual CRC, got/expect index, ...) */
    char msg[512];      /* the reference's error text, byte for byte where defined */
} rio_error;

/* rio_config.flags */
#define RIO_CFG_ITEM_END 1u  /* device results (rio_scan_device / _async) carry the
                                cumSize-shaped item output: rio_batch.item_end,
                                block_data, block_first_off instead of item_off /
                                item_len (8 B per item instead of 16) */
#define RIO_CFG_FLATE_NO_SPLIT 2u  /* tuning / test: never split a flate block's copy pass into
                                     * segments (by default a span of few large blocks is split,
                                     * see DESIGN.md "split copy pass") */
/* scanners over this ctx decode up to n (0-2) spans ahead of the batch handed
 * out (bits 8-9 hold n + 1; 0 = the default, 2); n above 2 is taken as 2 */
#define RIO_CFG_SPANS_AHEAD(n) (((((uint32_t)(n)) > 2u ? 2u : ((uint32_t)(n))) + 1u) << 8)
#define RIO_CFG_FLATE_TOK_ONLY 4u  /* test: the wave-per-block Huffman pass declines every flate
                                     * block, so the fallback pass (k_flate_tok) decodes them all */
#define RIO_CFG_FLATE_ONE_WAVE 16u /* test: the Huffman pass one wave per block on every span (by
                                     * default a span of few blocks takes its 4-wave variant) */

typedef struct rio_config {
    int32_t device;             /* HIP device ordinal */
    int32_t flags;              /* RIO_CFG_* bits */
    uint64_t max_span_bytes;    /* largest span per call (multiple of 32768); 0 = 256 MiB */
    uint64_t max_out_bytes;     /* straddler-bytes capacity per call (grown on demand); 0 = span/8 + 1 MiB */
    uint64_t max_items;         /* item-view capacity per call (grown on demand); 0 = span/64 + 1024 */
    /* tuning / test parameters of the flate decoder (0 = the defaults): tokens
     * per block and round (a small value forces the yield / resume path across
     * rounds), and Huffman-pass workgroups (a small value makes every wave
     * decode many blocks) */
    uint64_t flate_tok_limit;
    uint64_t flate_grid;
} rio_config;

typedef struct rio_ctx rio_ctx;

/* item_off[i] with this bit set is an offset into rio_batch.records; otherwise
 * it is an offset into rio_batch.span (the caller's chunk bytes). */
#define RIO_ITEM_IN_RECORDS (1ull << 63)

/* Results of one span: views, not copies. Arrays are owned by the ctx and valid
 * until the next call on it (like "Scan will reuse storage",
 * scannerv2.go:124-126). For rio_scan_span they are host (pinned) pointers; for
 * rio_scan_device they are device pointers (block_file_off is then NULL).
 * Item i is the bytes [o, o + item_len[i]) of
 *   records  when item_off[i] & RIO_ITEM_IN_RECORDS (o = item_off[i] without the bit),
 *   span     otherwise (o = item_off[i]).
 * Uncompressed items that sit inside one chunk payload are views into the span;
 * items that straddle a chunk boundary are gathered into records. For flate /
 * zstd every item is a view into the decoded blocks held in records.
 * Block b's items are [block_first_item[b], block_first_item[b+1]). */
typedef struct rio_batch {
    const uint8_t *span;              /* base of span-relative item offsets */
    const uint8_t *records;           /* straddling items / decoded blocks */
    uint64_t records_len;
    const uint64_t *item_off;         /* n_items entries */
    const uint64_t *item_len;         /* n_items entries */
    uint64_t n_items;
    const uint64_t *block_first_item; /* n_blocks + 1 entries */
    const uint64_t *block_file_off;   /* n_blocks entries (ItemLocation.Block) */
    uint64_t n_blocks;
    uint64_t consumed;   /* bytes of the span fully decoded (block boundary) */
    int32_t stop;        /* RIO_STOP_* */
    int32_t reserved;
    uint64_t in_bytes;   /* chunk-stream bytes examined */
    float kernel_ms;     /* device time of the decode pipeline (HIP events) */
    float total_ms;      /* including H2D / D2H for rio_scan_span */
    rio_error err;
    /* RIO_CFG_ITEM_END device results (item_off / item_len are then NULL): the
     * reference's rawItemList shape (scannerv2.go:24-49, 83-91). Block b's items
     * [F, E) = [block_first_item[b], block_first_item[b+1]) are
     *   item i = payload bytes [s, e) of block b,
     *   s = block_first_off[b] + (i > F ? item_end[i-1] : 0), e = block_first_off[b] + item_end[i]
     * (item_end = cumSize: block-relative inclusive prefix of the sizes;
     * block_first_off = firstOff: the packed header's length). With
     * D = block_data[b] & ~RIO_ITEM_IN_RECORDS:
     *   block_data[b] & RIO_ITEM_IN_RECORDS: the payload is contiguous at
     *     records + D (decoded flate / zstd blocks; none blocks with short
     *     middle chunks, gathered) -> records[D + s, D + e);
     *   else (none codec): the payload is the block's chunk payloads in the span,
     *     its first chunk at span + D: with k = s / 32740 and
     *     o = D + k * 32768 + 28 + s % 32740, an item within one chunk payload
     *     ((e - 1) / 32740 == k) is span[o, o + e - s), an item crossing into the
     *     next chunk is records[o, o + e - s) (gathered at its own span offset). */
    const uint64_t *item_end;         /* n_items entries */
    const uint64_t *block_data;       /* n_blocks entries */
    const uint64_t *block_first_off;  /* n_blocks entries */
    /* rio_scan_device_segments_async results: block b belongs to file
     * block_segment[b] (device array, n_blocks entries; block_file_off is then
     * the device array of the blocks' own file offsets), and an error's
     * err.file_off is an offset in file err_segment's bytes (else -1) */
    const uint64_t *block_segment;
    int64_t err_segment;
} rio_batch;

enum rio_stop {
    RIO_STOP_MORE = 0,    /* span exhausted at a block boundary; feed the rest */
    RIO_STOP_EOF = 1,     /* clean end: trailer block, file end or shard limit */
    RIO_STOP_ERROR = 2,   /* err holds the first error in file order */
};

/* ---- context ---- */
rio_ctx *rio_open(const rio_config *cfg);
void rio_close(rio_ctx *ctx);
/* thread-local text of the last rio_open / ABI failure */
const char *rio_last_error(void);
int rio_abi_version(void);
/* build provenance: a hash of the library's sources, this header and its
 * compile flags (16 hex digits; base_amd/build.py tree_build_id) */
const char *rio_build_id(void);
/* the HIP stream the ctx launches on (hipStream_t as void*) */
void *rio_stream(rio_ctx *ctx);

/* Host-path counters of a ctx since rio_open: the end-to-end (PCIe-inclusive)
 * accounting of rio_scan_span / rio_scan_v1_span and the scanner layer's spans
 * (no reference counterpart: the Go scanner reads and copies on the host). */
typedef struct rio_stats {
    uint64_t spans;     /* host spans scanned */
    uint64_t h2d_bytes; /* bytes copied host -> device (the spans) */
    uint64_t d2h_bytes; /* bytes copied device -> host (records, item views, block tables) */
    double device_ms;   /* HIP-event time of those calls: copies in, pipeline, copies out (a
                           scanner's spans ahead run on a second context: included) */
    uint64_t span_cap;  /* the span the device buffers are sized for now (rio_config.max_span_bytes,
                           grown by a block longer than it; a chain's later stages grow it for that
                           call only) */
} rio_stats;
int rio_ctx_stats(rio_ctx *ctx, rio_stats *out);

/* Transformer registry lookup (registry.go:113-148 + recordioflate/zstd Init):
 * resolves the header's "transformer" values to a codec -- none, flate, zstd,
 * or a RIO_CODEC_CHAIN of 2-4 of flate / zstd. Returns 0 and sets *codec, or
 * RIO_ERR_FALLBACK for a name other than flate / zstd (or a chain of more than
 * 4): the caller decodes such a file with the reference scanner, whose
 * registry may hold user transformers (registry.go:166). */
int rio_codec_for_transformers(const char *const *values, int n, int32_t *codec, rio_error *err);

/* ---- batch layer ----
 * span: bytes at file offset file_off (a block boundary, multiple of 32768).
 * is_file_end: the span reaches the end of the file (a tail shorter than 32768
 * bytes then reads as "unexpected EOF"; an unfinished block ends the scan).
 * limit_off: ChunkScanner.limit (chunk.go:259): blocks starting at or after it
 * are not scanned; use UINT64_MAX for none.
 * Returns 0 on success (check out->stop / out->err), <0 on a runtime failure. */
int rio_scan_span(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off,
                  int32_t is_file_end, uint64_t limit_off, int32_t codec, rio_batch *out);
int rio_scan_device(rio_ctx *ctx, const void *dev_span, uint64_t nbytes, uint64_t file_off,
                    int32_t is_file_end, uint64_t limit_off, int32_t codec, rio_batch *out);

/* v1 ("legacy") files (recordio/deprecated; read by the reference through
 * legacyScannerAdapter, legacyscanner.go:84-117): decode the v1 records in
 * span = file bytes at file_off, a record boundary. Blocks are records
 * (block_file_off = the record's offset, ItemLocation.Block for Seek); a
 * packed record's items are its unpacked items, an unpacked record is one
 * item. Every item is a view into span. stop: EOF at the file end, MORE at the
 * last whole record (consumed = its end; when not even the first record fits,
 * consumed is 0 and err.a holds the span size it needs), ERROR at the first
 * failing record. No LegacyTransform: a caller that sets one decodes the file
 * with the reference scanner. */
int rio_scan_v1_span(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off,
                     int32_t is_file_end, rio_batch *out);

/* Device-resident benchmark entry: like rio_scan_device but asynchronous on the
 * ctx stream and with no host copies; call rio_sync to collect the summary. */
int rio_scan_device_async(rio_ctx *ctx, const void *dev_span, uint64_t nbytes, uint64_t file_off,
                          int32_t codec);
int rio_sync(rio_ctx *ctx, rio_batch *out);

/* Many files in one launch (a rank's trailer-indexed
 * files decoded together). The span holds nseg file bodies back to back:
 * segment s is span bytes [seg_end[s-1], seg_end[s]) (seg_end[-1] = 0), every
 * boundary a multiple of 32768 and a block boundary of its file, and begins
 * at byte seg_file_off[s] of its file. As rio_scan_device_async (the span ends
 * at the last file's end), plus, in the rio_sync results, each block's file
 * (block_segment) and its offset in that file (block_file_off: the
 * ItemLocation.Block a Seek in that file takes). The scan stops at the first
 * error in span order, reported with its file (err_segment) -- the files after
 * a failing one are not decoded in that launch: scan them again without it.
 * seg_end / seg_file_off are host arrays, not retained. */
int rio_scan_device_segments_async(rio_ctx *ctx, const void *dev_span, uint64_t nbytes, const uint64_t *seg_end,
                                   const uint64_t *seg_file_off, uint64_t nseg, int32_t codec);

/* Device time (HIP events) of the last completed run, per stage:
 * [0] block parse + item views + straddler gather (second stream, overlaps [2]),
 * [1] codec decode (compressed codecs), [2] k_crc (chunk CRC32 verify),
 * [3] chunk headers + chunk scans, [4] the whole pipeline.
 * Returns the number of stages written. */
int rio_stage_times(rio_ctx *ctx, float *ms, int n);

/* Flate blocks of the last completed run whose copy pass was split into
 * segments (DESIGN.md "split copy pass"; 0 with RIO_CFG_FLATE_NO_SPLIT, for
 * many small blocks, or before the split scratch has been sized). For tests
 * and measurement; no reference counterpart. */
uint64_t rio_flate_split_blocks(rio_ctx *ctx);

/* TransformFunc analogue (recordio.go:12): untransform one block given its
 * chunk payload views (in order, any lengths; their concatenation is the
 * transformed block). none concatenates on the host; flate / zstd decode on the
 * GPU (recordioflate.go:54-65, recordiozstd.go:67-78). Writes into scratch if
 * it fits and returns 0 with the length in *out_len; RIO_ERR_CAPACITY with the
 * needed size in *out_len when it does not fit; the codec's error (code and
 * the reference's text in *err) for a corrupt stream; < 0 on a runtime failure. */
int rio_decode_block(rio_ctx *ctx, const uint8_t *const *payloads, const uint32_t *lens, int n,
                     int32_t codec, uint8_t *scratch, uint64_t cap, uint64_t *out_len,
                     rio_error *err);

/* ---- writer encode path ----
 * The blocks of a v2 file encoded on the GPU, byte for byte what
 * recordio.NewWriter writes for the same items with the none transformer
 * (flate: a valid DEFLATE stream of the same payload):
 * items_per_block items per block (the writer packs MaxItems + 1 per block:
 * its object slice has capacity MaxItems + 1 and is flushed when full,
 * writerv2.go:315, 366-368; the last block takes the rest; 0 = the default
 * MaxItems 16384 + 1), each block generatePackedHeaderv2 + items
 * (writerv2.go:388-442), framed by ChunkWriter.Write (internal/chunk.go:100-141:
 * 28-byte headers, CRC32-IEEE over [12, 28 + size), 0xdeadbeef padding).
 * kind picks the magic: body blocks (MagicPacked), the header block or the
 * trailer block (one item each: the marshalled header / the trailer bytes,
 * writerv2.go:327-335, 510-536). */
enum rio_block_kind { RIO_BLOCK_BODY = 0, RIO_BLOCK_HEADER = 1, RIO_BLOCK_TRAILER = 2 };
typedef struct rio_encode_args {
    const void *data;          /* item bytes back to back */
    const uint64_t *item_end;  /* n_items exclusive ends: item i = data[end[i-1], end[i]) */
    uint64_t n_items;
    uint64_t items_per_block;  /* MaxItems + 1; 0 = 16385 */
    int32_t codec;             /* RIO_CODEC_NONE, or RIO_CODEC_FLATE: a raw DEFLATE stream per
                                  block ("flate N" transformer, recordioflate.go:31-52; any valid
                                  stream decodes alike -- the bytes are not klauspost's), or
                                  RIO_CODEC_ZSTD: one zstd frame per block ("zstd N",
                                  recordiozstd.go:31-52; Huffman-coded literals where
                                  they shrink, predefined sequence codes, <= 16 KiB blocks -- decoded by libzstd alike) */
    int32_t kind;              /* enum rio_block_kind */
    int32_t level;             /* flate: 0 stored blocks (NoCompression), 1 fixed-Huffman
                                  blocks, otherwise (the default -1 included) a dynamic- or
                                  fixed-Huffman block per 32 KiB, whichever is smaller; both
                                  with greedy hash matches.
                                  codec = RIO_CODEC_CHAIN(n, t0 | t1 << 2 | ...) (1 <= n <= 4,
                                  each flate or zstd): the writer's transformers in order,
                                  stage k transforming stage k - 1's output (registry.go:75-111,
                                  writerv2.go:432-441); stage k's level is the signed byte
                                  (level >> 8k) & 0xff (0xff = -1, the default) */
    int32_t reserved;
} rio_encode_args;
/* Host memory in and out: writes the chunk stream to out (out_cap bytes) and
 * each block's offset in it (ItemLocation.Block minus the stream's file
 * offset) to block_off (ceil(n_items / items_per_block) entries, may be NULL).
 * Returns 0 with *out_len; RIO_ERR_CAPACITY with the needed *out_len when out
 * is too small; < 0 on a runtime failure. The stream is encoded once (into
 * device memory the ctx grows to fit; the ctx's span capacity does not apply). */
int rio_encode(rio_ctx *ctx, const rio_encode_args *a, uint8_t *out, uint64_t out_cap, uint64_t *out_len,
               uint64_t *block_off, rio_error *err);
/* The same with data, item_end, out and block_off in device memory (the
 * device-resident producer of a scan: rio_scan_device reads what this wrote).
 * out = NULL only sizes the stream (*out_len). */
int rio_encode_device(rio_ctx *ctx, const rio_encode_args *a, void *out, uint64_t out_cap, uint64_t *out_len,
                      uint64_t *block_off, rio_error *err);

/* ---- scanner layer ---- */
typedef struct rio_reader {
    void *user;
    /* read up to n bytes at offset off into buf; return bytes read (0 at EOF), <0 on error */
    int64_t (*read_at)(void *user, uint8_t *buf, uint64_t n, uint64_t off);
    int64_t size; /* file size in bytes */
} rio_reader;

/* A reader over a file already in host memory (the caller keeps *m alive
 * while scanners use the reader): read_at is a memcpy, safe from any thread. */
typedef struct rio_memory {
    const uint8_t *data;
    uint64_t size;
} rio_memory;
rio_reader rio_memory_reader(const rio_memory *m);

typedef struct rio_scanner rio_scanner;

/* NewScanner / NewShardScanner (scannerv2.go:200-235). The reader is used
 * until rio_scanner_finish. Never returns NULL for valid ctx/reader; errors
 * are reported through rio_scanner_err like errorScanner.
 * Memory: the scanner decodes up to RIO_CFG_SPANS_AHEAD(n) (n 0-2, default 2)
 * spans ahead of the batch it hands out, each on a further context of the ctx (its
 * "siblings", opened with the ctx's configuration and span size on the first
 * scan that needs them). They stay open, and keep their device and pinned
 * buffers, until rio_close(ctx): with the default depth a scanner's ctx holds
 * about three times the device memory of one context. Open the ctx with
 * RIO_CFG_SPANS_AHEAD(0) where that matters, e.g. many ctxs of very large
 * spans per GPU.
 * Span schedule (read from the environment when the scanner is made; results
 * do not depend on it): RIO_SPAN_RAMP=k (default 2, 0 off) -- an uncompressed
 * body's first spans are the ctx's span >> k, >> k-1, ... (spans of at least
 * RIO_SPAN_RAMP_MIN bytes, default 256 MiB), and a compressed body's of small
 * blocks too (RIO_SPAN_RAMP_C=0: not); RIO_SCAN_EARLY=0 -- a compressed body
 * span is no longer staged and followed by the next span's copy in before it
 * is decoded (DESIGN.md "Round 6 in brief"). */
rio_scanner *rio_scanner_new(rio_ctx *ctx, const rio_reader *r, int start, int limit, int nshard);
/* Scan (scannerv2.go:390-404): 1 if a new record is available */
int rio_scanner_scan(rio_scanner *s);
/* Get: view of the current record, valid until the next scan of a new batch */
int rio_scanner_get(rio_scanner *s, const uint8_t **data, uint64_t *len);
/* Batched Scan+Get: up to max records; returns the count (0 at end/error) */
int64_t rio_scanner_next_batch(rio_scanner *s, const uint8_t **data, uint64_t *lens, int64_t max);
/* Err (scannerv2.go:406-412): 0 when nil, else fills err */
int rio_scanner_err(rio_scanner *s, rio_error *err);
/* Header (scannerv2.go:312): key/value i; type 1 bool, 2 int, 3 uint, 4 string */
int rio_scanner_header_len(rio_scanner *s);
int rio_scanner_header_kv(rio_scanner *s, int i, const char **key, int32_t *type, int64_t *ival,
                          const uint8_t **sval, uint64_t *slen);
/* Trailer (scannerv2.go:316-342): 1 and a view when present, 0 = nil */
int rio_scanner_trailer(rio_scanner *s, const uint8_t **data, uint64_t *len);
/* Seek (scannerv2.go:348-361) to ItemLocation{block, item} */
void rio_scanner_seek(rio_scanner *s, uint64_t block, int64_t item);
/* Gather (random access): the items at n ItemLocations
 * {blocks[i], items[i]}, as Seek + Scan + Get would return them
 * (scannerv2.go:348-361, 390-403), the distinct blocks decoded as one batch.
 * Returns n, or the index of the first location that fails (err filled with
 * the error Seek / Scan sets there; views before it are valid), or -1 on bad
 * arguments. The scan position is untouched; views stay valid until the next
 * gather on this scanner. */
int64_t rio_scanner_gather(rio_scanner *s, const uint64_t *blocks, const int64_t *items, int64_t n,
                           const uint8_t **data, uint64_t *lens, rio_error *err);
/* ItemLocation of the current record */
void rio_scanner_location(rio_scanner *s, uint64_t *block, int64_t *item);
/* Version (scannerv2.go:308, legacyscanner.go:45): 2, or 1 for a v1 file */
int rio_scanner_version(rio_scanner *s);
/* Finish (scannerv2.go:414-425): returns Err() code and frees the scanner */
int rio_scanner_finish(rio_scanner *s, rio_error *err);

#ifdef __cplusplus
}
#endif
#endif /* RIO_GPU_H */
