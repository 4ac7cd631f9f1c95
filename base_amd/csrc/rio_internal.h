// Internal layout shared by the HIP kernels and the host pipeline.
// Not part of the ABI (see include/rio_gpu.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rio_gpu.h"

// RIO_SYNC_EACH (debug builds only): every launch is followed by a stream
// synchronize that names the kernel on failure, so a fault is pinned to its
// kernel even when several are queued.
#ifdef RIO_SYNC_EACH
#include <stdio.h>
namespace rio {
inline void dbg_sync(const char *name, hipStream_t st) {
  const hipError_t e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    fprintf(stderr, "RIO_SYNC_EACH: %s failed: %s\n", name, hipGetErrorString(e));
    fflush(stderr);
  }
}
}  // namespace rio
#undef hipLaunchKernelGGL
#define hipLaunchKernelGGL(kernelName, ...)                     \
  do {                                                          \
    hipLaunchKernelGGLInternal((kernelName), __VA_ARGS__);      \
    ::rio::dbg_sync(#kernelName, rio_sync_stream(__VA_ARGS__)); \
  } while (0)
template <class G, class B, class S, class... A>
inline hipStream_t rio_sync_stream(G, B, S, hipStream_t st, A &&...) {
  return st;
}
#endif

namespace rio {

constexpr int kChunk = RIO_CHUNK_SIZE;              // chunk.go:25
constexpr int kChunkHdr = RIO_CHUNK_HEADER_SIZE;    // chunk.go:22
constexpr int kMaxPayload = RIO_MAX_CHUNK_PAYLOAD;  // chunk.go:28
constexpr unsigned long long kItemInRecords = RIO_ITEM_IN_RECORDS;

// Magic classes (magic.go:15-36).
enum MagicClass : uint32_t { kMagicHeader = 0, kMagicPacked = 1, kMagicTrailer = 2, kMagicOther = 3 };

// Per-chunk structural error codes (k_chunk_meta), ordered like readChunk/Scan
// checks (chunk.go:273-287, 333-336).
enum ChunkErr : uint32_t {
  kCkOk = 0,
  kCkSize = 1,          // size > 32740
  kCkMagicChanged = 2,  // magic differs from the block's first chunk
  kCkIndex = 3,         // index != expected
  kCkTotal = 4,         // total != block's total
};

// Block status codes (k_block_parse).
enum BlockStatus : uint32_t {
  kBlkOk = 0,
  kBlkIncomplete = 1,  // extends past the span (or total == 0)
  kBlkBadMagic = 2,    // neither packed nor (mode-appropriate) header/trailer
  kBlkNItems = 3,      // uvarint item count failed: a = n
  kBlkItemSize = 4,    // uvarint size failed: a = item index, b = n
  kBlkBlockSize = 5,   // total + pos != len: a = len, b = total + pos
  kBlkItemRange = 6,   // wrapped sizes (reference panics)
  kBlkTrailer = 7,     // trailer block in body mode: clean end of scan
  kBlkLimit = 8,       // starts at/after the shard limit
  kBlkCodec = 9,       // decompression failed: a = codec error code, b = offset
  kBlkSlow = 10,       // (internal) header left to the general parser, k_parse_slow
};

// blk_a of a kBlkCodec block (codec.hip: codec_error_text)
enum CodecErr : uint32_t {
  kCodecCorrupt = 1,      // flate: CorruptInputError(offset = blk_b)
  kCodecEof = 2,          // flate: io.ErrUnexpectedEOF
  kCodecFull = 3,         // output region too small (internal: retried with a larger bound)
  kCodecZstd = 4,         // zstd: error, blk_b = ZSTD error enum
  kCodecZstdEmpty = 5,    // zstd: empty source
  kCodecUnsupported = 6,
  kCodecPending = 255,    // (internal) left to k_inflate_exact
};

// kModeRaw: rio_decode_block (TransformFunc analogue): chunk headers, scans and
// the codec only -- no CRC, no packed parse, no resolve.
enum Mode : int32_t { kModeBody = 0, kModeHeader = 1, kModeTrailer = 2, kModeLastChunk = 3, kModeRaw = 4 };

// Ablation builds only (tools/ablate.py compiles with -DRIO_ABLATE=n): 1 no CRC
// fold, 2 no parse path, 4 no CRC. The shipped library is built with 0.
#ifndef RIO_ABLATE
#define RIO_ABLATE 0
#endif

// out_overflow bit of a build / layout fault (k_crc's dynamic LDS tables not at
// address 0): reported as an internal error at once, never retried
constexpr unsigned long long kOvfLayout = 1ull << 40;

// Control block written by the kernels, read back by the host (one copy).
struct Ctl {
  unsigned long long first_chunk_err;    // min chunk with size/structural error
  unsigned long long first_crc_err;      // min chunk with CRC mismatch
  unsigned long long first_block_event;  // min over block event keys (2*chunk + 1 / 2*c0)
  unsigned long long first_incomplete;   // min c0 of a block extending past the span
  unsigned long long out_overflow;       // nonzero if side/items exceeded capacity
  unsigned long long dec_need;           // decode regions' total size (when it exceeds dec_cap)
  unsigned long long pad[2];             // [0] (RIO_FLSTAT builds: flate pass counters); [1] zstd blocks on the serial path
  // filled by k_resolve
  unsigned long long stop_key;
  unsigned long long n_valid_blocks;
  unsigned long long n_items;
  unsigned long long rec_bytes;   // side-buffer / decoded bytes used by the valid blocks
  unsigned long long stop_block;  // block index at the stop (or ~0)
  unsigned long long stop_kind;   // 0 more, 1 eof, 2 error
  unsigned long long err_chunk;   // chunk of a chunk-level error (or ~0)
  unsigned long long err_code;    // ChunkErr / CRC(100) / unexpected EOF(101)
  // details of the stop (filled by k_resolve)
  unsigned long long ck_size, ck_total, ck_index, ck_info;
  unsigned long long ck_crc_stored, ck_crc_actual;
  unsigned long long prev_total, prev_index, prev_info;
  unsigned long long blk_status, blk_a, blk_b, blk_c0, blk_payload;
  unsigned long long consumed_chunks;
  unsigned long long mag_cur, mag_prev, mag_blk;  // little-endian magic bytes
  unsigned long long flstat_esc;                  // (RIO_FLSTAT builds: flate escapes)
  unsigned long long n_retry;                     // blocks k_parse_lean left to k_parse (listed in blk_coff)
  unsigned long long zprof[4];                    // (RIO_ZPROF builds: zstd entropy-pass cycles per phase)
  unsigned long long zjob_n;                      // zstd jobs made (k_zstd_ent)
  unsigned long long seg_used;                    // flate split copy: scratch bytes the blocks asked for (k_flate_plan)
  unsigned long long seg_blocks;                  // flate split copy: blocks split
  unsigned long long zx[4];                       // (RIO_ZPROF builds: zstd execution pass groups, parts, ready, rest matches)
  unsigned long long tok_need;                    // zstd: scratch bytes every block's region needs (kOvfZTok)
};

constexpr unsigned long long kNone = ~0ull;

// An item that crosses a chunk payload boundary (the 28-byte chunk header sits
// inside it). Slot = the chunk where the item starts (at most one straddler
// starts in a chunk and crosses its end): logical payload bytes [src, src+len)
// of the block starting at chunk c0, item index `item`. k_strad gathers it into
// side[ck_sbase[slot]] and points item_off[item] there.
struct StradDesc {
  unsigned long long c0, src, len, item;
};

// blk_meta bit fields
constexpr unsigned long long kMetaTotalMask = 0xffffffffull;  // chunks of the block (ck_total)
constexpr int kMetaClsShift = 32;                             // MagicClass (8 bits)
constexpr unsigned long long kMetaRegular = 1ull << 40;       // every chunk but the last is full
constexpr unsigned long long kMetaComplete = 1ull << 41;      // all chunks inside the span

// Two-pass flate decode (codec_flate.hip): per-block state handed from the
// Huffman pass (k_flate_tok, writes LZ77 tokens) to the copy pass (k_flate_lz,
// 32 KiB LDS window) and kept across rounds when a block's token region fills.
enum FlMode : uint32_t {
  kFlHeader = 0,   // next: a DEFLATE block header (BFINAL, BTYPE)
  kFlFixed = 1,    // inside a fixed-Huffman block
  kFlDynamic = 2,  // inside a dynamic-Huffman block (tables rebuilt from hdrpos on resume)
  kFlStored = 3,   // inside a stored block, stored_left bytes to go
  kFlDone = 4,     // final block decoded
  kFlError = 5,    // decode failed (k_inflate_exact classifies it)
  kFlSkip = 6,     // not decoded (incomplete block, header magic, region overflow)
  kFlSplit = 7,    // tokens complete, copy pass split into segments (k_flate_seg; stored_left = segments)
};
struct FlState {
  unsigned long long bitpos;  // logical bit offset of the next symbol / header
  unsigned long long hdrpos;  // kFlDynamic: bit offset of the block's HLIT field
  unsigned long long olen;    // output bytes of all tokens so far
  unsigned long long olen2;   // output bytes the copy pass has written
  uint32_t mode, final_;      // FlMode; the current DEFLATE block has BFINAL set
  uint32_t ntok, round;       // tokens written in `round`
  uint32_t stored_left, pad;
};
constexpr int kFlRounds = 6;          // Huffman/copy rounds launched per span
constexpr int kTokPerChunk = kChunk;  // token region: 32,768 u32 per chunk of the block
// zstd scratch: each block's region (flattened input, literals, execution
// entries | jobs) is sized from its headers by k_zstd_size and placed back to
// back (blk_zoff); the first attempt's buffer is this many bytes per span byte
// (a run that needs more reports it, tok_need, and the host retries)
constexpr uint64_t kZTokInitFactor = 5;
constexpr unsigned long long kOvfZTok = 0x4000;  // out_overflow: the zstd scratch regions exceed tok_cap
constexpr int kZJobsPerChunk = 16;               // zstd job list capacity (a block past it takes the serial path)
// Split copy pass (codec_flate.hip k_flate_plan / k_flate_seg / k_flate_segfix):
// segments per block at most, and the shortest segment
#ifndef RIO_SEG_MAX
#define RIO_SEG_MAX 16
#endif
constexpr int kSegMax = RIO_SEG_MAX;
constexpr uint32_t kSegMin = 65536;

// Device arrays of one context (capacities fixed at rio_open, grown on demand).
struct DevBufs {
  // per chunk
  uint32_t *ck_size, *ck_total, *ck_index, *ck_info;  // info: magic class | err << 8
  uint32_t *ck_crc;                                   // computed CRC32 per chunk
  uint32_t *ck_block;            // block index of the chunk (valid in the consistent prefix)
  unsigned long long *ck_pay;    // exclusive prefix of payload sizes (nchunks + 1)
  unsigned long long *ck_ssz;    // padded size of the straddler starting in the chunk (0: none)
  unsigned long long *ck_sbase;  // exclusive scan of ck_ssz (nchunks + 1): side offsets
  // per block
  unsigned long long *blk_c0;         // first chunk
  unsigned long long *blk_meta;       // total | class | regular | complete (kMeta*)
  unsigned long long *blk_len;        // untransformed payload bytes (none codec)
  unsigned long long *blk_nitems;     // item slots reserved (the header's item count)
  unsigned long long *blk_hdr;        // varint header length
  unsigned long long *blk_item_base;  // exclusive scan of nitems (n + 1)
  unsigned long long *blk_status;     // BlockStatus
  unsigned long long *blk_a, *blk_b;
  unsigned long long *blk_out_len;    // decoded length (compressed codecs)
  unsigned long long *blk_dec_off;    // offset of the block's decoded bytes in dec (n + 1)
  unsigned long long *blk_need;       // decoded size found by the exact pass after a region overflow
  unsigned long long *blk_coff;       // host results: compact offsets of the decoded blocks (n + 1), then a scratch (n + 1)
  unsigned long long *blk_data;       // item-end output: where the block's payload lies (rio_batch.block_data)
  unsigned long long *blk_file_off;   // segment scans: the block's offset in its file
  unsigned long long *blk_seg;        // segment scans: the block's file (segment index)
  unsigned long long *blk_zneed;      // zstd: the block's scratch region bytes (k_zstd_size)
  unsigned long long *blk_zoff;       // zstd: exclusive scan of blk_zneed (n + 1): region offsets in tok
  unsigned long long *blk_zhalf;      // zstd: region bytes below the jobs (input, literals, entries)
  // outputs: item views into the span or the records buffer (side / dec); in
  // item-end mode (ParseArgs::end_mode) item_off holds item_end (cumSize) instead
  unsigned long long *item_off, *item_len;
  uint8_t *side;        // straddling items (none codec)
  StradDesc *strad;     // straddler per chunk slot
  // scratch
  unsigned long long *scan_tmp;  // tile partials
  uint8_t *dec;                  // decoded blocks (compressed codecs)
  uint8_t *cmp;                  // host results: the valid blocks' decoded bytes back to back
  uint64_t cmp_cap;
  uint64_t dec_cap;              // bytes at dec
  FlState *fl;                   // per block (flate)
  uint32_t *tok;                 // flate tokens: block b's region starts at blk_c0[b] * kTokPerChunk;
                                 // zstd: block b's scratch at byte blk_zoff[b]
  uint64_t tok_cap;              // u32 entries at tok
  uint64_t tok_limit;            // tokens per block and round (0: the whole region; rio_config.flate_tok_limit)
  uint64_t fl_grid;              // Huffman-pass workgroups (0: all resident; rio_config.flate_grid)
  uint64_t fl_tok_only;          // RIO_CFG_FLATE_TOK_ONLY: k_flate_sync declines every block (tests)
  uint64_t fl_one_wave;          // RIO_CFG_FLATE_ONE_WAVE: k_flate_sync<1> on every span (tests)
  unsigned long long *fl_more;   // per round: blocks whose token region filled (kFlRounds)
  unsigned long long *fl_ck;     // per chunk: the Huffman pass's (ntok | olen << 32) at the block's input
                                 // chunk k (entry c0 + k; entry c0 = entries written) -- split points
  unsigned long long *fl_seg;    // per block x kSegMax: (tok | out << 32, scratch offset) of each segment
  uint8_t *seg_scr;              // later segments' u16 symbols (0: no split)
  uint64_t seg_cap;              // bytes at seg_scr
  uint64_t seg_items;            // copy-pass waves the split aims to fill (ncu x kL2Waves; 0: no split)
  uint64_t fl_ck_n;              // entries at fl_ck
  uint32_t *fl_stage;            // Huffman pass: per-wave token staging (k_flate_sync), 0: none
  uint64_t fl_stage_waves;       // waves it holds columns for
  uint8_t *zlit;                 // zstd: one literal buffer per decoder wave (codec_zstd.hip)
  unsigned long long *zjob;      // zstd: job header offsets (bytes from tok)
  uint64_t zjob_cap;
  uint64_t zlit_waves;           // decoder waves zlit holds buffers for
  Ctl *ctl;
  // CRC tables (constant)
  uint32_t *crc_fold;   // 4 x 256 fold tables, each replicated x32 (bank-private copies)
  uint32_t *crc_mul;    // 7 x 4 x 256 multiply-by-constant tables
  uint32_t *crc_fix_a;  // per payload size: ~0 shifted over 16+size bytes
  uint32_t *crc_fix_b;  // per payload size: x^(-8*pad)
};

// zstd decoder sizing (codec_zstd.hip)
uint64_t zstd_grid(int ncu);             // decoder waves launched
uint64_t zstd_lit_bytes(uint64_t grid);  // literal buffers for that many waves
uint64_t flate_seg_items(int ncu);       // copy-pass slots the split copy pass fills
uint64_t flate_stage_words(int ncu);     // the Huffman pass's token staging (u32 words)
uint64_t flate_stage_waves(int ncu);     // waves those words hold a staging column set for

// Kernel argument blocks (kernels.hip, codec.hip; filled by pipeline.cpp).
struct ParseArgs {
  const uint8_t *span;
  uint64_t nchunks;
  uint64_t limit_chunk;  // blocks starting at/after it are not scanned
  int32_t mode;
  int32_t codec;
  const unsigned long long *nblocks;  // device count
  uint64_t item_cap, side_cap;
  int32_t sparse;    // straddlers go to a span-shaped side buffer at their own span offset
  int32_t end_mode;  // RIO_CFG_ITEM_END (sparse results only): item_end[i] = cumSize into item_off
  // k_parse over a list of blocks (the ones k_parse_lean declined) instead of all
  const unsigned long long *list;
  const unsigned long long *list_n;
  // a transformer chain's earlier stage: block structure and codec only, no
  // packed-header parse (the decoded bytes are the next stage's input)
  int32_t no_items;
  int32_t pad2;
};
struct CrcArgs {
  int32_t flags;  // RIO_ABLATE of ablation builds (1 no CRC fold); 0 in the shipped library
  int32_t pad;
};
struct ResolveArgs {
  const uint8_t *span;
  uint64_t nchunks;
  int32_t is_file_end;
  int32_t tail_partial;  // bytes after the last whole chunk at file end
  int32_t mode;
  int32_t codec;
  const unsigned long long *nblocks;
  uint64_t limit_chunk;  // ChunkScanner.limit in chunks (a partial tail chunk at/after it is never read)
  int32_t sparse;        // side buffer layout (ParseArgs::sparse)
  int32_t pad;
};

// ---- host helpers: GF(2) arithmetic of the reflected CRC-32 polynomial ----
constexpr uint32_t kPoly = 0xEDB88320u;
#ifndef RIO_FOLD_COPIES
#define RIO_FOLD_COPIES 16  // (round 4: 32 -> 16, so that another kernel's workgroup fits beside k_crc)
#endif
constexpr int kFoldCopies = RIO_FOLD_COPIES;     // replicas of each fold table (lane l reads copy l % copies)
constexpr int kFoldShift = kFoldCopies == 32 ? 7 : (kFoldCopies == 16 ? 6 : 5);  // log2(4 * copies)
constexpr int kFoldWords = 4 * 256 * kFoldCopies;  // 64 KiB at 16 copies
// Byte-row layout (16 copies): entry b of table j, copy c at byte 256 b + 64 j + 4 c, so a
// lookup's address is one v_perm_b32 -- byte 1 the data byte, byte 0 the lane's
// (64 j + 4 c) -- instead of an extract, a shift and an add (crc_fold.h fold_row)
#ifndef RIO_FOLD_PERM
#define RIO_FOLD_PERM 1
#endif
constexpr bool kFoldPerm = RIO_FOLD_PERM && kFoldCopies == 16;
constexpr int kMulTables = 7;                    // x^-32, then x^-(128*2^l), l = 0..5
uint32_t gf_mul(uint32_t a, uint32_t b);         // a*b mod P (reflected; 1 = 0x80000000)
uint32_t gf_xpow8(int64_t nbytes);               // x^(8*nbytes) mod P, nbytes may be negative
void build_crc_tables(uint32_t *fold, uint32_t *mul, uint32_t *fix_a, uint32_t *fix_b);
uint32_t crc32_host(const uint8_t *p, size_t n);  // plain IEEE CRC (for self-checks)

}  // namespace rio
