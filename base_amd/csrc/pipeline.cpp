// Host orchestration of the span decode pipeline and the batch-layer C ABI
// (include/rio_gpu.h). One rio_ctx = one device, two HIP streams, buffers sized
// at rio_open and grown only when a span needs more.
//
// Launch order per span (one stream; the parse beside k_crc on a second stream
// measured slower):
//   none:       memsets, k_chunk_meta, chunk scans, block scan (item slots),
//               k_parse, k_parse_slow, [straddler scan], k_strad, k_crc, k_resolve
//   flate/zstd: memsets, k_chunk_meta, chunk scans, codec decode, item counts,
//               block scan, k_parse, k_parse_slow, k_crc, k_resolve
#include <hip/hip_runtime.h>
#include <inttypes.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "encode.h"
#include "zstd_enc.h"
#include "legacy.h"
#include "pipeline.h"
#include "rio_internal.h"
#include "sdma.h"

namespace rio {
// kernels.hip
void launch_chunk_pass(const uint8_t *span, uint64_t nchunks, const DevBufs &d, unsigned long long *nblocks_dev,
                       int32_t codec, hipStream_t st);
void launch_reset(const DevBufs &d, unsigned long long *nblocks_dev, hipStream_t st);
void launch_chunk_scan(const unsigned long long *in, unsigned long long *out, unsigned long long *tmp, uint64_t n,
                       hipStream_t st);
void launch_block_scan(const unsigned long long *in, unsigned long long *out, unsigned long long *tmp,
                       const unsigned long long *nblocks_dev, uint64_t max_blocks, hipStream_t st);
// blocks.hip
void launch_parse(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st);
void launch_parse_lean(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st);
void launch_lean_end(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st);
void launch_parse_slow(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st);
void launch_dec_nitems(const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks, hipStream_t st);
void launch_strad(const uint8_t *span, const DevBufs &d, uint64_t nslots, uint64_t side_cap, int32_t sparse, int32_t end_mode,
                  hipStream_t st);
void launch_resolve(const DevBufs &d, const ResolveArgs &a, hipStream_t st);
void launch_block_files(const DevBufs &d, const unsigned long long *seg_end, const unsigned long long *seg_file_off,
                        uint64_t nseg, uint64_t max_blocks, hipStream_t st);
// crc.hip
void launch_crc(const uint8_t *span, uint64_t nchunks, const DevBufs &d, const CrcArgs &ca, int ncu,
                hipStream_t st);
// codec.hip
void launch_compact(const DevBufs &d, const unsigned long long *nblocks_dev, uint64_t max_blocks, hipStream_t st);
void launch_codec_prepare(const DevBufs &d, const unsigned long long *nblocks_dev, uint64_t max_blocks,
                          uint32_t factor, hipStream_t st);
void launch_block_scan(const unsigned long long *in, unsigned long long *out, unsigned long long *tmp,
                       const unsigned long long *nblocks_dev, uint64_t max_blocks, hipStream_t st);
// codec_zstd.hip: per-block decode and scratch regions from the headers
void launch_zstd_size(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks,
                      uint32_t factor, hipStream_t st);
void launch_codec_decode(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks_dev,
                         uint64_t max_blocks, uint64_t nchunks, int codec, uint64_t dec_cap, int rounds, int ncu,
                         hipStream_t st);
// codec_flate.hip: the flate decode's two phases (launch_codec_decode runs both)
void launch_inflate_huff(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks,
                         uint64_t max_blocks, uint64_t nchunks, uint64_t dec_cap, int rounds, int ncu, hipStream_t st);
void launch_inflate_plan(const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks, hipStream_t st);
void launch_inflate_copy(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks,
                         uint64_t max_blocks, uint64_t nchunks, uint64_t dec_cap, int rounds, int ncu, hipStream_t st);
}  // namespace rio

using namespace rio;

static thread_local std::string g_last_error;

static void set_last_error(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

#define HIP_OK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      set_last_error("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return -1;                                                                     \
    }                                                                                \
  } while (0)

enum { kEvStart, kEvScans, kEvDec, kEvCrc0, kEvCrc1, kEvParse0, kEvParse1, kEvEnd, kNumEv };

// Pinned host copies of one span's results (records, item views, block table).
// Each owner -- the ctx for rio_scan_span, every rio_scanner for its batches,
// a scanner's trailer read -- has its own, so results of one never alias
// another's (the reference's scanners share no state).
struct rio_results {
  uint8_t *records = nullptr;
  uint64_t records_cap = 0;
  unsigned long long *items = nullptr;  // off | len
  uint64_t items_cap = 0;
  unsigned long long *blk = nullptr;  // first_item (n+1) | file_off (n)
  uint64_t blk_cap = 0;
  void release() {
    if (records) hipHostFree(records);
    if (items) hipHostFree(items);
    if (blk) hipHostFree(blk);
    *this = rio_results();
  }
};

rio_results *rio_results_new() { return new rio_results(); }
void rio_results_free(rio_results *r) {
  if (!r) return;
  r->release();
  delete r;
}

struct rio_ctx {
  int device = 0;
  int ncu = 256;
  hipStream_t st = nullptr;
  // SDMA engines for the copies of host spans (in) and host results (out),
  // sdma.cpp; null when the runtime offers none (hipMemcpyAsync then). The
  // flags: copies of that direction issued and not yet waited for.
  Sdma *sd = nullptr;
  bool sd_in = false, sd_out = false;
  hipEvent_t ev[kNumEv] = {};
  bool last_had_dec = false;
  int ev_parse0 = kEvParse0, ev_crc0 = kEvCrc0;  // the events the last run's parse / CRC stages start at
  bool item_end_mode = false;  // RIO_CFG_ITEM_END: device results carry item_end (cumSize)
  bool flate_split = true;     // not RIO_CFG_FLATE_NO_SPLIT
  bool split_probed = false;   // the first flate run sized the split scratch mid-run (enqueue)
  rio_stats stats{};           // host-path counters (rio_ctx_stats)
  uint64_t seg_want = 0;       // split copy pass: scratch the last flate run asked for
  bool last_cmp = false;  // the last host result's records are the compacted blocks (d.cmp)
  uint64_t max_span = 0, max_chunks = 0, max_blocks = 0;
  uint64_t side_cap = 0, item_cap = 0, dec_cap = 0;
  // growth for one call (a chain's later stages, rio_decode_block's long block):
  // the sizes before it, restored at the next call (settle)
  bool grown_tmp = false;
  uint64_t base_span = 0, base_side = 0, base_item = 0;
  rio_config cfg{};            // as opened (the sibling opens with it)
  rio_ctx *sibling = nullptr;  // a scanner's further context (its spans ahead), opened on first use
  const uint8_t *staged = nullptr;  // rio_scan_span_stage: the span whose H2D copy is enqueued
  uint64_t staged_n = 0;
  hipEvent_t staged_t0{};
  // rio_scan_span_begin: collect enqueues the result copies without waiting;
  // rio_scan_span_end waits for them and finishes the batch
  bool defer_collect = false, pend = false;
  uint64_t pend_nb = 0, pend_file_off = 0, pend_d2h = 0;
  unsigned long long *pend_foff = nullptr;
  hipEvent_t pend_t0 = nullptr, pend_t1 = nullptr;
  uint32_t dec_factor = 8;  // first-attempt decode-region bound: compressed bytes x this
  // zstd: the first attempt's decode buffer (span bytes x this; regions are sized
  // from the frames' content sizes, k_zstd_size) and scratch (kZTokInitFactor),
  // each grown to what a run reported it needed
  uint32_t zdec_factor = 4;
  uint64_t ztok_want = 0;
  int fl_rounds = kFlRounds;  // flate Huffman/copy rounds per span (doubled if a block needs more)
  DevBufs d{};
  unsigned long long *nblocks_dev = nullptr;
  uint8_t *d_span = nullptr;  // staging for host spans (lazy)
  Ctl *h_ctl = nullptr;  // pinned copy of the control block
  rio_results res;       // host results of rio_scan_span (scanners bring their own)
  uint8_t *h_stage = nullptr;  // pinned staging of rio_decode_block's chunk stream
  // v1 (legacy) spans: the record table (host), packed-record headers staged
  // (pinned host + device), jobs, views
  std::vector<V1Rec> v1_recs;
  std::vector<V1Job> v1_jobs;
  std::vector<uint64_t> v1_job_rec;
  std::vector<V1Unp> v1_unp;
  std::vector<V1Res> v1_res;
  uint8_t *h_v1 = nullptr;
  uint64_t h_v1_cap = 0;
  // writer encode path: per-block arrays (6 x (n + 1)), varint headers,
  // transformed payloads; host-path staging of items, ends and output
  unsigned long long *e_blk = nullptr;
  uint64_t e_blk_cap = 0;
  uint8_t *e_hdr = nullptr, *e_comp = nullptr, *e_comp2 = nullptr, *e_data = nullptr, *e_out = nullptr;
  uint64_t e_hdr_cap = 0, e_comp_cap = 0, e_comp2_cap = 0, e_data_cap = 0, e_out_cap = 0;
  unsigned long long *e_zscr = nullptr;  // zstd / dynamic flate encode: the waves' sequence / token lists
  uint64_t e_zscr_cap = 0;
  ZeTabs *e_ztab = nullptr;              // zstd encode: predefined FSE tables (uploaded once)
  unsigned long long *e_ends = nullptr, *e_boff = nullptr;
  uint64_t e_ends_cap = 0, e_boff_cap = 0;
  uint32_t *e_ckmap = nullptr;            // chunk -> block of the encoded stream
  uint64_t e_ckmap_cap = 0;
  unsigned long long *e_scan = nullptr;   // scan scratch of the per-block arrays
  uint64_t e_scan_cap = 0;
  uint8_t *d_v1 = nullptr;
  uint64_t d_v1_cap = 0;
  V1Job *d_v1_jobs = nullptr;
  V1Res *d_v1_res = nullptr;
  uint64_t d_v1_jobs_cap = 0;
  unsigned long long *d_v1_off = nullptr, *d_v1_len = nullptr;
  uint64_t d_v1_items_cap = 0;
  uint64_t h_stage_cap = 0;
  // pools of pinned host buffers and result sets that finished scanners hand
  // back (a scanner per file would otherwise pin and unpin hundreds of MB
  // per file: SURVEY.md §8(f) 2, cf. file/internal/s3bufpool)
  std::mutex pool_mu;
  std::vector<std::pair<uint8_t *, uint64_t>> buf_pool;
  std::vector<rio_results *> res_pool;
  // segment scans: the segment table on the device (seg_end | seg_file_off) and its host copy
  unsigned long long *d_seg = nullptr;
  uint64_t d_seg_cap = 0;
  std::vector<uint64_t> seg_end_h, seg_file_h;
  // transformer chains through the async entries: the stages ran at the call
  // (each needs the previous one's block sizes on the host); rio_sync returns
  // chain_batch. chain_c0: stage 1's block chunk indexes (the file's), on the
  // host and (for segment scans) on the device
  bool chain_async = false;
  rio_batch chain_batch{};
  std::vector<unsigned long long> chain_c0;
  unsigned long long *d_chain_c0 = nullptr;
  uint64_t d_chain_c0_cap = 0;
  // transformer chains: the reframed stage outputs (two, alternating) and their chunk offsets
  uint8_t *d_chain[2] = {nullptr, nullptr};
  uint64_t d_chain_cap[2] = {0, 0};
  unsigned long long *d_chain_meta = nullptr;
  uint64_t d_chain_meta_cap = 0;
  // last async call
  uint64_t last_nchunks = 0, last_file_off = 0, last_in_bytes = 0, last_nseg = 0;
  int32_t last_codec = 0, last_mode = 0;
  const uint8_t *last_span = nullptr;
};

const char *rio_last_error(void) { return g_last_error.c_str(); }
int rio_abi_version(void) { return RIO_ABI_VERSION; }
void *rio_stream(rio_ctx *ctx) { return ctx ? (void *)ctx->st : nullptr; }
uint64_t rio_ctx_max_span(rio_ctx *c) { return c->max_span; }
int rio_ctx_spans_ahead(rio_ctx *c) {
  const uint32_t v = ((uint32_t)c->cfg.flags >> 8) & 3u;
  return v ? (int)v - 1 : 2;
}

template <class T>
static int dalloc(T **p, uint64_t n) {
  if (*p) hipFree(*p);
  *p = nullptr;
  if (n == 0) n = 1;
  HIP_OK(hipMalloc((void **)p, n * sizeof(T)));
  return 0;
}

// A host <-> device copy of n bytes on the ctx's SDMA engine for that
// direction, else (no engine, pageable host memory) hipMemcpyAsync on the
// kernels' stream. SDMA copies are ordered on the host: an outgoing copy is
// issued once the kernels that wrote its bytes have completed (collect runs
// after the control block's sync), and sdma_settle waits for them before
// anything reuses the buffers; an incoming one completes before the kernels
// that read it are enqueued (run_span).
#ifndef RIO_SDMA
#define RIO_SDMA 3  // directions on SDMA (measurement builds): 1 device -> host, 2 host -> device
#endif
static int copy_to_host(rio_ctx *c, void *dst, const void *src, uint64_t n) {
  if (n == 0) return 0;
  if ((RIO_SDMA & 1) && c->sd && sdma_copy(c->sd, dst, src, n, kSdmaOut) == 0) {
    c->sd_out = true;
    return 0;
  }
  HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->st));
  return 0;
}
static int copy_to_device(rio_ctx *c, void *dst, const void *src, uint64_t n) {
  if (n == 0) return 0;
  if ((RIO_SDMA & 2) && c->sd && sdma_copy(c->sd, dst, src, n, kSdmaIn) == 0) {
    c->sd_in = true;
    return 0;
  }
  HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->st));
  return 0;
}
static int sdma_settle(rio_ctx *c, int dir) {
  bool &f = dir == kSdmaOut ? c->sd_out : c->sd_in;
  if (!f) return 0;
  f = false;
  if (sdma_wait(c->sd, dir) != 0) {
    set_last_error("an SDMA copy did not complete");
    return -1;
  }
  return 0;
}

static int alloc_bufs(rio_ctx *c) {
  DevBufs &d = c->d;
  const uint64_t n = c->max_chunks + 1;
  if (dalloc(&d.ck_size, n) || dalloc(&d.ck_total, n) || dalloc(&d.ck_index, n) || dalloc(&d.ck_info, n) ||
      dalloc(&d.ck_crc, n) || dalloc(&d.ck_block, n) || dalloc(&d.ck_pay, n + 1) || dalloc(&d.ck_ssz, n) ||
      dalloc(&d.ck_sbase, n + 1))
    return -1;
  const uint64_t nb = c->max_blocks + 1;
  if (dalloc(&d.blk_c0, nb) || dalloc(&d.blk_meta, nb) || dalloc(&d.blk_len, nb) || dalloc(&d.blk_nitems, nb) ||
      dalloc(&d.blk_hdr, nb) || dalloc(&d.blk_item_base, nb + 1) || dalloc(&d.blk_status, nb) ||
      dalloc(&d.blk_a, nb) || dalloc(&d.blk_b, nb) || dalloc(&d.blk_out_len, nb) || dalloc(&d.blk_dec_off, nb + 1) ||
      dalloc(&d.blk_need, nb) || dalloc(&d.fl, nb) || dalloc(&d.blk_coff, 2 * (nb + 1)) || dalloc(&d.blk_data, nb) ||
      dalloc(&d.blk_file_off, nb) || dalloc(&d.blk_seg, nb) || dalloc(&d.blk_zneed, nb) ||
      dalloc(&d.blk_zoff, nb + 1) || dalloc(&d.blk_zhalf, nb))
    return -1;
  if (dalloc(&d.scan_tmp, 2 * ((n + 2047) / 2048) + 16) || dalloc(&d.strad, n)) return -1;
  if (dalloc(&d.item_off, c->item_cap) || dalloc(&d.item_len, c->item_cap) || dalloc(&d.side, c->side_cap))
    return -1;
  return 0;
}

static void free_all(rio_ctx *c) {
  sdma_close(c->sd);  // (waits for copies in flight)
  c->sd = nullptr;
  DevBufs &d = c->d;
  void *ps[] = {d.ck_size, d.ck_total, d.ck_index, d.ck_info, d.ck_crc, d.ck_block, d.ck_pay, d.ck_ssz, d.ck_sbase,
                d.blk_c0, d.blk_meta, d.blk_len, d.blk_nitems, d.blk_hdr, d.blk_item_base, d.blk_status, d.blk_a, d.blk_b, d.blk_out_len, d.blk_dec_off, d.blk_need, d.blk_coff, d.blk_data, d.blk_file_off, d.blk_seg, d.blk_zneed, d.blk_zoff, d.blk_zhalf, d.cmp, d.item_off, d.item_len, d.side,
                d.strad, d.scan_tmp, d.dec, d.fl, d.tok, d.fl_more, d.fl_ck, d.fl_seg, d.seg_scr, d.fl_stage, d.zlit, d.zjob, d.ctl, d.crc_fold, d.crc_mul, d.crc_fix_a, d.crc_fix_b,
                c->nblocks_dev, c->d_span, c->d_v1, c->d_v1_jobs, c->d_v1_res, c->d_v1_off, c->d_v1_len,
                c->e_blk, c->e_hdr, c->e_comp, c->e_comp2, c->e_data, c->e_out, c->e_ends, c->e_boff, c->e_zscr, c->e_ztab, c->e_ckmap, c->e_scan, c->d_seg, c->d_chain[0], c->d_chain[1], c->d_chain_meta};
  for (void *p : ps)
    if (p) hipFree(p);
  if (c->h_ctl) hipHostFree(c->h_ctl);
  c->res.release();
  if (c->h_stage) hipHostFree(c->h_stage);
  if (c->h_v1) hipHostFree(c->h_v1);
  for (hipEvent_t e : c->ev)
    if (e) hipEventDestroy(e);
  if (c->st) hipStreamDestroy(c->st);
}

static int ctx_init(rio_ctx *c, const rio_config *cfg) {
  if (cfg) c->cfg = *cfg;
  c->device = cfg ? cfg->device : 0;
  HIP_OK(hipSetDevice(c->device));
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, c->device));
  c->ncu = prop.multiProcessorCount;
  // flate tuning / test parameters: a small token region per block and round
  // forces the yield / resume path across rounds (and the host retry with more
  // rounds); few Huffman-pass waves make every stream decode many blocks
  c->d.tok_limit = cfg ? cfg->flate_tok_limit : 0;
  c->d.fl_grid = cfg ? cfg->flate_grid : 0;
  c->d.fl_tok_only = (cfg && (cfg->flags & RIO_CFG_FLATE_TOK_ONLY)) ? 1 : 0;
  c->d.fl_one_wave = (cfg && (cfg->flags & RIO_CFG_FLATE_ONE_WAVE)) ? 1 : 0;
  c->item_end_mode = cfg && (cfg->flags & RIO_CFG_ITEM_END);
  c->flate_split = !(cfg && (cfg->flags & RIO_CFG_FLATE_NO_SPLIT));
  uint64_t span = (cfg && cfg->max_span_bytes) ? cfg->max_span_bytes : (256ull << 20);
  span = (span + kChunk - 1) / kChunk * kChunk;
  c->max_span = span;
  c->max_chunks = span / kChunk;
  c->max_blocks = c->max_chunks;
  c->side_cap = (cfg && cfg->max_out_bytes) ? cfg->max_out_bytes : span / 8 + (1 << 20);
  c->item_cap = (cfg && cfg->max_items) ? cfg->max_items : span / 64 + 1024;
  c->dec_cap = 0;
  HIP_OK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
  for (hipEvent_t &e : c->ev) HIP_OK(hipEventCreate(&e));
  if (alloc_bufs(c)) return -1;
  DevBufs &d = c->d;
  if (dalloc(&d.ctl, 1) || dalloc(&c->nblocks_dev, 2) || dalloc(&d.fl_more, 64)) return -1;
  c->sd = sdma_open(d.ctl);  // (null: no SDMA engine; copies go through hipMemcpyAsync)
  // CRC tables
  std::vector<uint32_t> fold(kFoldWords), mul(kMulTables * 1024), fa(kMaxPayload + 1), fb(kMaxPayload + 1);
  build_crc_tables(fold.data(), mul.data(), fa.data(), fb.data());
  if (dalloc(&d.crc_fold, fold.size()) || dalloc(&d.crc_mul, mul.size()) || dalloc(&d.crc_fix_a, fa.size()) ||
      dalloc(&d.crc_fix_b, fb.size()))
    return -1;
  HIP_OK(hipMemcpy(d.crc_fold, fold.data(), fold.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d.crc_mul, mul.data(), mul.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d.crc_fix_a, fa.data(), fa.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d.crc_fix_b, fb.data(), fb.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipHostMalloc((void **)&c->h_ctl, sizeof(Ctl), hipHostMallocDefault));
  return 0;
}

// every SDMA copy of the ctx complete: they run outside its stream, so a stream
// sync alone does not order them before a buffer they read or write is freed
static int sdma_quiesce(rio_ctx *c) {
  const int a = sdma_settle(c, kSdmaIn), b = sdma_settle(c, kSdmaOut);
  return (a || b) ? -1 : 0;
}

static int reserve(rio_ctx *c, uint64_t bytes) {
  bytes = (bytes + kChunk - 1) / kChunk * kChunk;
  if (bytes <= c->max_span) return 0;
  HIP_OK(hipSetDevice(c->device));
  HIP_OK(hipStreamSynchronize(c->st));
  if (sdma_quiesce(c)) return -1;
  c->max_span = bytes;
  c->max_chunks = bytes / kChunk;
  c->max_blocks = c->max_chunks;
  if (c->side_cap < bytes / 8 + (1 << 20)) c->side_cap = bytes / 8 + (1 << 20);
  if (c->item_cap < bytes / 64 + 1024) c->item_cap = bytes / 64 + 1024;
  if (c->d_span) {  // host-span staging: reallocated at the new size on next use
    hipFree(c->d_span);
    c->d_span = nullptr;
  }
  return alloc_bufs(c);
}

// a lasting reservation (the scanner's header / long block): also the size a
// temporary growth returns to
int rio_ctx_reserve_span(rio_ctx *c, uint64_t bytes) {
  if (c->grown_tmp) {
    const uint64_t r = (bytes + kChunk - 1) / kChunk * kChunk;
    if (r > c->base_span) c->base_span = r;
    if (c->base_side < r / 8 + (1 << 20)) c->base_side = r / 8 + (1 << 20);
    if (c->base_item < r / 64 + 1024) c->base_item = r / 64 + 1024;
  }
  return reserve(c, bytes);
}

// growth for this call only: a chain stage's decoded bytes can be several times
// the file span, and one chain file should not leave a long-lived context that
// large (the results stay valid until the next call, which shrinks it back)
static int reserve_tmp(rio_ctx *c, uint64_t bytes) {
  if ((bytes + kChunk - 1) / kChunk * kChunk <= c->max_span) return 0;
  if (!c->grown_tmp) {
    c->grown_tmp = true;
    c->base_span = c->max_span;
    c->base_side = c->side_cap;
    c->base_item = c->item_cap;
  }
  return reserve(c, bytes);
}

template <class T>
static void dfree(T **p) {
  if (*p) hipFree(*p);
  *p = nullptr;
}

// back to the sizes before a temporary growth (every buffer sized from the
// grown span is released; the demand-sized ones regrow on use)
// a span staged by rio_scan_span_stage and not decoded: forgotten (d_span is
// reused; its copy in may run on an SDMA engine, outside the stream's order, so
// it completes here before anything else writes or frees d_span)
static int unstage(rio_ctx *c) {
  if (!c->staged) return 0;
  c->staged = nullptr;
  hipEventDestroy(c->staged_t0);
  return sdma_settle(c, kSdmaIn);
}

static int settle(rio_ctx *c) {
  if (unstage(c)) return -1;
  if (!c->grown_tmp) return 0;
  c->grown_tmp = false;
  HIP_OK(hipSetDevice(c->device));
  HIP_OK(hipStreamSynchronize(c->st));
  if (sdma_quiesce(c)) return -1;
  c->max_span = c->base_span;
  c->max_chunks = c->max_span / kChunk;
  c->max_blocks = c->max_chunks;
  c->side_cap = c->base_side;
  c->item_cap = c->base_item;
  DevBufs &d = c->d;
  dfree(&c->d_span);
  dfree(&d.dec);
  c->dec_cap = d.dec_cap = 0;
  dfree(&d.tok);
  d.tok_cap = 0;
  dfree(&d.zjob);
  d.zjob_cap = 0;
  dfree(&d.seg_scr);
  d.seg_cap = 0;
  c->seg_want = 0;
  dfree(&d.fl_ck);
  dfree(&d.fl_seg);
  d.fl_ck_n = 0;
  for (int k = 0; k < 2; k++) {
    dfree(&c->d_chain[k]);
    c->d_chain_cap[k] = 0;
  }
  if (c->h_stage) hipHostFree(c->h_stage);
  c->h_stage = nullptr;
  c->h_stage_cap = 0;
  return alloc_bufs(c);
}

rio_ctx *rio_open(const rio_config *cfg) {
  rio_ctx *c = new rio_ctx();
  if (ctx_init(c, cfg) != 0) {
    free_all(c);
    delete c;
    return nullptr;
  }
  return c;
}

constexpr size_t kPoolMax = 8;  // pooled pinned buffers (and result sets) per ctx

int rio_ctx_take_buf(rio_ctx *c, uint64_t need, uint8_t **p, uint64_t *cap) {
  {
    std::lock_guard<std::mutex> g(c->pool_mu);
    size_t best = c->buf_pool.size();
    for (size_t i = 0; i < c->buf_pool.size(); i++)  // the smallest that fits
      if (c->buf_pool[i].second >= need && (best == c->buf_pool.size() || c->buf_pool[i].second < c->buf_pool[best].second))
        best = i;
    if (best < c->buf_pool.size()) {
      *p = c->buf_pool[best].first;
      *cap = c->buf_pool[best].second;
      c->buf_pool.erase(c->buf_pool.begin() + (long)best);
      return 0;
    }
  }
  *p = nullptr;
  *cap = 0;
  if (hipHostMalloc((void **)p, need, hipHostMallocDefault) != hipSuccess) {
    *p = nullptr;
    return -1;
  }
  *cap = need;
  return 0;
}

void rio_ctx_give_buf(rio_ctx *c, uint8_t *p, uint64_t cap) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> g(c->pool_mu);
    if (c->buf_pool.size() < kPoolMax) {
      c->buf_pool.emplace_back(p, cap);
      return;
    }
  }
  hipHostFree(p);
}

rio_results *rio_ctx_take_results(rio_ctx *c) {
  std::lock_guard<std::mutex> g(c->pool_mu);
  if (c->res_pool.empty()) return rio_results_new();
  rio_results *r = c->res_pool.back();
  c->res_pool.pop_back();
  return r;
}

void rio_ctx_give_results(rio_ctx *c, rio_results *r) {
  if (!r) return;
  {
    std::lock_guard<std::mutex> g(c->pool_mu);
    if (c->res_pool.size() < kPoolMax) {
      c->res_pool.push_back(r);
      return;
    }
  }
  rio_results_free(r);
}

void rio_close(rio_ctx *ctx) {
  if (!ctx) return;
  rio_scan_span_end(ctx);
  rio_close(ctx->sibling);
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->st);
  for (auto &b : ctx->buf_pool) hipHostFree(b.first);
  for (rio_results *r : ctx->res_pool) rio_results_free(r);
  free_all(ctx);
  delete ctx;
}

// ------------------------------------------------------------------ launches
static int ensure_dec(rio_ctx *c, uint64_t need) {
  if (c->dec_cap >= need) return 0;
  const uint64_t cap = need + need / 4;
  if (dalloc(&c->d.dec, cap)) return -1;
  c->dec_cap = cap;
  c->d.dec_cap = cap;
  return 0;
}

// flate token regions: kTokPerChunk u32 per chunk of the span (zstd: the
// blocks' scratch regions, sized by k_zstd_size; `need` in u32)
static int ensure_tok_u32(rio_ctx *c, uint64_t need) {
  if (c->d.tok_cap >= need) return 0;
  if (dalloc(&c->d.tok, need)) return -1;
  c->d.tok_cap = need;
  return 0;
}
static int ensure_tok(rio_ctx *c, uint64_t nchunks, uint64_t per_chunk) {
  return ensure_tok_u32(c, nchunks * per_chunk);
}
static int ensure_ztok(rio_ctx *c, uint64_t nchunks) {
  uint64_t want = nchunks * (uint64_t)kChunk * kZTokInitFactor;
  if (want < c->ztok_want) want = c->ztok_want;
  return ensure_tok_u32(c, (want + 3) / 4);
}

// flate split copy pass: checkpoints per chunk, segment table per block, and
// the later segments' scratch -- grown to what the last run asked for (a
// block the scratch cannot hold is copied whole meanwhile), at most 6x the
// span or 2x the decode regions
static int ensure_split(rio_ctx *c, uint64_t nchunks) {
  DevBufs &d = c->d;
  if (!d.fl_ck || c->max_chunks + 1 > d.fl_ck_n) {
    if (dalloc(&d.fl_ck, c->max_chunks + 1) || dalloc(&d.fl_seg, 2 * (uint64_t)kSegMax * (c->max_blocks + 1)))
      return -1;
    d.fl_ck_n = c->max_chunks + 1;
  }
  d.seg_items = c->flate_split ? flate_seg_items(c->ncu) : 0;
  if (!d.fl_stage) {  // the Huffman pass's token staging (a wave decodes once per round, then copies)
    const uint64_t w = flate_stage_words(c->ncu);
    if (hipMalloc((void **)&d.fl_stage, w * 4) == hipSuccess) d.fl_stage_waves = flate_stage_waves(c->ncu);
    else (void)hipGetLastError(), d.fl_stage = nullptr, d.fl_stage_waves = 0;
  }
  uint64_t want = c->seg_want;
  uint64_t lim = 6 * nchunks * (uint64_t)kChunk;  // (or twice the decode regions: highly compressible blocks)
  if (lim < 2 * c->dec_cap) lim = 2 * c->dec_cap;
  if (want > lim) want = lim;
  if (d.seg_items && want > d.seg_cap) {
    want += want / 8;
    if (d.seg_scr) hipFree(d.seg_scr);
    d.seg_scr = nullptr;
    d.seg_cap = 0;
    if (hipMalloc((void **)&d.seg_scr, want) == hipSuccess) d.seg_cap = want;
    else (void)hipGetLastError();  // no scratch: blocks are copied whole
  }
  return 0;
}

// the scratch the last flate run's split asked for (read from its control block)
static void note_split(rio_ctx *c) {
  if (c->h_ctl->seg_used > c->d.seg_cap && c->h_ctl->seg_used > c->seg_want) c->seg_want = c->h_ctl->seg_used;
}

// zstd scratch: what a run's regions needed (+1/8), kept for the next runs
static int grow_ztok(rio_ctx *c, uint64_t need_bytes) {
  const uint64_t want = need_bytes + need_bytes / 8 + 4096;
  if (want > c->ztok_want) c->ztok_want = want;
  return ensure_tok_u32(c, (c->ztok_want + 3) / 4);
}

// zstd job list: kZJobsPerChunk per chunk of the span
static int ensure_zjob(rio_ctx *c, uint64_t nchunks) {
  const uint64_t need = nchunks * (uint64_t)kZJobsPerChunk + 64;
  if (c->d.zjob_cap >= need) return 0;
  if (dalloc(&c->d.zjob, need)) return -1;
  c->d.zjob_cap = need;
  return 0;
}

// zstd literal buffers: one per decoder wave (allocated on first use)
static int ensure_zlit(rio_ctx *c) {
  if (c->d.zlit) return 0;
  const uint64_t g = zstd_grid(c->ncu);
  if (dalloc(&c->d.zlit, zstd_lit_bytes(g))) return -1;
  c->d.zlit_waves = g;
  return 0;
}

// Enqueue the full pipeline for `nchunks` whole chunks at device span `span`.
static int ensure_side(rio_ctx *c, uint64_t need) {
  if (c->side_cap >= need) return 0;
  if (dalloc(&c->d.side, need)) return -1;
  c->side_cap = need;
  return 0;
}

// sparse: straddlers land at their own span offset in a span-sized side buffer
// (device-resident results, no straddler scan); else compacted (host results).
// stage_flags (transformer chains): kStageNoItems -- decode, no packed parse
// (a chain's earlier stage); kStageNoCrc -- the span is a reframed stage
// output, not file chunks (no CRC stored)
enum { kStageNoItems = 1, kStageNoCrc = 2 };

#ifndef RIO_CRC_FIRST
#define RIO_CRC_FIRST 0
#endif
static int enqueue(rio_ctx *c, const uint8_t *span, uint64_t nchunks, uint64_t limit_chunk, int is_file_end,
                   int tail_partial, int32_t codec, int32_t mode, bool sparse, int attempt, int stage_flags = 0,
                   bool may_sync = true) {
  if (sparse && codec == RIO_CODEC_NONE && ensure_side(c, nchunks * (uint64_t)kChunk)) return -1;
  DevBufs &d = c->d;
  hipStream_t st = c->st;
  c->last_nchunks = nchunks;
  c->last_cmp = false;  // records are d.dec / d.side until a host result compacts them
  HIP_OK(hipEventRecord(c->ev[kEvStart], st));
  // control words (min-reduced: ~0; counters: 0) and the block counters, one launch
  launch_reset(d, c->nblocks_dev, st);
  if (attempt == 0 && codec != RIO_CODEC_NONE && nchunks > 0)
    HIP_OK(hipMemsetAsync(d.blk_need, 0, nchunks * sizeof(unsigned long long), st));
  const uint64_t max_blocks = nchunks ? nchunks : 1;
  // the shipped library always runs every stage; RIO_ABLATE (a -D of ablation
  // builds, tools/ablate.py) drops stages for measurement only
  const bool run_parse = !(RIO_ABLATE & 2) && mode != kModeRaw,
             run_crc = !(RIO_ABLATE & 4) && mode != kModeRaw && !(stage_flags & kStageNoCrc);
  const bool no_items = (stage_flags & kStageNoItems) != 0;
  const CrcArgs ca{RIO_ABLATE, 0};
  // order: chunk pass (headers + scans), (decode), parse, k_crc, resolve
  c->ev_crc0 = kEvCrc0;
  if (!run_crc || nchunks == 0) {  // (no CRC pass later: a zero-length interval)
    HIP_OK(hipEventRecord(c->ev[kEvCrc0], st));
    HIP_OK(hipEventRecord(c->ev[kEvCrc1], st));
  }
  if (nchunks > 0) launch_chunk_pass(span, nchunks, d, c->nblocks_dev, codec, st);
  HIP_OK(hipEventRecord(c->ev[kEvScans], st));
  // none codec, RIO_CRC_FIRST builds: the CRC pass before the parse (it needs
  // only the chunk sizes), so that with two spans in flight a span's parse runs
  // beside the next span's CRC pass. Measured slower (C2 3.03 -> 3.47 ms per
  // step, A/B on one box): the parse's scattered loads beside the CRC pass's
  // stream cost more than the overlap gains
  const bool crc_first = RIO_CRC_FIRST && codec == RIO_CODEC_NONE && run_crc && nchunks > 0;
  if (crc_first) {
    c->ev_crc0 = kEvScans;
    launch_crc(span, nchunks, d, ca, c->ncu, st);
    HIP_OK(hipEventRecord(c->ev[kEvCrc1], st));
  }
  c->last_had_dec = false;
  if (codec != RIO_CODEC_NONE && nchunks > 0) {
    // decode regions: factor x the compressed bytes per block (+4 KiB each);
    // zstd: the frames' content sizes (k_zstd_size), a smaller first guess
    if (codec == RIO_CODEC_ZSTD ? ensure_dec(c, (uint64_t)c->zdec_factor * nchunks * kChunk + nchunks * 256ull)
                                : ensure_dec(c, (uint64_t)c->dec_factor * nchunks * kChunk + nchunks * 4352ull))
      return -1;
    // flate tokens / flattened zstd blocks
    if (codec == RIO_CODEC_FLATE && (ensure_tok(c, nchunks, kTokPerChunk) || ensure_split(c, nchunks))) return -1;
    if (codec == RIO_CODEC_ZSTD && ensure_ztok(c, nchunks)) return -1;
    if (codec == RIO_CODEC_ZSTD && (ensure_zlit(c) || ensure_zjob(c, nchunks))) return -1;
    if (codec == RIO_CODEC_ZSTD) {  // decode and scratch regions from the headers, placed back to back
      launch_zstd_size(span, d, c->nblocks_dev, max_blocks, c->dec_factor, st);
      launch_block_scan(d.blk_out_len, d.blk_dec_off, d.scan_tmp, c->nblocks_dev, max_blocks, st);
      launch_block_scan(d.blk_zneed, d.blk_zoff, d.scan_tmp, c->nblocks_dev, max_blocks, st);
    } else {
      launch_codec_prepare(d, c->nblocks_dev, max_blocks, c->dec_factor, st);
    }
    if (codec == RIO_CODEC_FLATE) {
      launch_inflate_huff(span, d, c->nblocks_dev, max_blocks, nchunks, c->dec_cap, c->fl_rounds, c->ncu, st);
      if (d.seg_items && !c->split_probed && d.seg_cap == 0 && may_sync) {
        // a context's first flate run: the split copy pass needs scratch the
        // Huffman pass's output decides. Read what the plan asked for, size the
        // scratch and plan again (seg_used / seg_blocks reset), so the first
        // scan of a span of few large blocks splits too (later runs grow the
        // scratch for the next call instead, without a mid-run sync; the
        // asynchronous entry points never sync here: their first flate run
        // copies whole blocks and sizes the scratch for the next call)
        c->split_probed = true;
        HIP_OK(hipMemcpyAsync(&c->h_ctl->seg_used, &d.ctl->seg_used, sizeof(unsigned long long),
                              hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        if (c->h_ctl->seg_used) {
          c->seg_want = c->h_ctl->seg_used;
          if (ensure_split(c, nchunks)) return -1;
          HIP_OK(hipMemsetAsync(&d.ctl->seg_used, 0, sizeof(unsigned long long), st));
          HIP_OK(hipMemsetAsync(&d.ctl->seg_blocks, 0, sizeof(unsigned long long), st));
          launch_inflate_plan(d, c->nblocks_dev, max_blocks, st);
        }
      }
      launch_inflate_copy(span, d, c->nblocks_dev, max_blocks, nchunks, c->dec_cap, c->fl_rounds, c->ncu, st);
    } else {
      launch_codec_decode(span, d, c->nblocks_dev, max_blocks, nchunks, codec, c->dec_cap, c->fl_rounds, c->ncu, st);
    }
    c->last_had_dec = true;
  }
  // (an event record costs ~5 us of GPU time between kernels: the stage
  // boundaries share events where they coincide -- parse starts at kEvDec or
  // kEvScans, the CRC at kEvParse1)
  if (c->last_had_dec) HIP_OK(hipEventRecord(c->ev[kEvDec], st));
  c->ev_parse0 = c->last_had_dec ? kEvDec : (crc_first ? kEvCrc1 : kEvScans);
  if (nchunks > 0 && run_parse) {
    ParseArgs pa{span, nchunks, limit_chunk, mode, codec, c->nblocks_dev, c->item_cap, c->side_cap, sparse,
                 (c->item_end_mode && sparse) ? 1 : 0};
    pa.no_items = no_items ? 1 : 0;
    if (no_items) HIP_OK(hipMemsetAsync(d.blk_nitems, 0, max_blocks * sizeof(unsigned long long), st));
    else if (codec != RIO_CODEC_NONE) launch_dec_nitems(d, c->nblocks_dev, max_blocks, st);
    launch_block_scan(d.blk_nitems, d.blk_item_base, d.scan_tmp, c->nblocks_dev, max_blocks, st);
    if (codec == RIO_CODEC_NONE && mode == kModeBody && !no_items) {
      // the common block shape in a lean kernel, the rest listed for k_parse
      if (pa.end_mode) launch_lean_end(d, pa, max_blocks, st);  // (item-end device results)
      else launch_parse_lean(d, pa, max_blocks, st);
      ParseArgs pl = pa;
      pl.list = d.blk_coff;
      pl.list_n = &d.ctl->n_retry;
      launch_parse(d, pl, max_blocks, st);
    } else {
      launch_parse(d, pa, max_blocks, st);
    }
    launch_parse_slow(d, pa, max_blocks, st);
    if (codec == RIO_CODEC_NONE) {
      if (!sparse) launch_chunk_scan(d.ck_ssz, d.ck_sbase, d.scan_tmp, nchunks, st);
      launch_strad(span, d, nchunks, c->side_cap, sparse, pa.end_mode, st);
    }
  } else if (nchunks == 0) {
    HIP_OK(hipMemsetAsync(d.blk_item_base, 0, 8, st));
    HIP_OK(hipMemsetAsync(d.ck_sbase, 0, 8, st));
  }
  HIP_OK(hipEventRecord(c->ev[kEvParse1], st));
  if (run_crc && nchunks > 0 && !crc_first) {
    c->ev_crc0 = kEvParse1;
    launch_crc(span, nchunks, d, ca, c->ncu, st);
    HIP_OK(hipEventRecord(c->ev[kEvCrc1], st));
  }
  if (mode != kModeRaw) {
    ResolveArgs ra{span, nchunks, is_file_end, tail_partial, mode, codec, c->nblocks_dev, limit_chunk, sparse, 0};
    launch_resolve(d, ra, st);
  }
  HIP_OK(hipEventRecord(c->ev[kEvEnd], st));
  return 0;
}

static int collect(rio_ctx *c, const uint8_t *span, uint64_t file_off, int32_t codec, int32_t mode,
                   uint64_t in_bytes, rio_batch *out, rio_results *res) {
  const Ctl &k = *c->h_ctl;
  memset(out, 0, sizeof(*out));
  out->err_segment = -1;
  out->in_bytes = in_bytes;
  out->n_blocks = k.n_valid_blocks;
  out->n_items = k.n_items;
  out->records_len = k.rec_bytes;
  out->consumed = k.consumed_chunks * kChunk;
  out->stop = (int32_t)k.stop_kind;
  out->span = span;
  if (k.stop_kind == 2) rio_fill_error(k, file_off, mode, &out->err);
  const uint8_t *d_records = (codec == RIO_CODEC_NONE) ? c->d.side : (c->last_cmp ? c->d.cmp : c->d.dec);
  const uint64_t nb = k.n_valid_blocks;
  if (!res) {  // device results
    out->records = d_records;
    out->block_first_item = reinterpret_cast<const uint64_t *>(c->d.blk_item_base);
    out->block_file_off = nullptr;
    if (c->item_end_mode) {  // the cumSize-shaped output (rio_gpu.h)
      out->item_end = reinterpret_cast<const uint64_t *>(c->d.item_off);
      out->block_data = reinterpret_cast<const uint64_t *>(c->d.blk_data);
      out->block_first_off = reinterpret_cast<const uint64_t *>(c->d.blk_hdr);
    } else {
      out->item_off = reinterpret_cast<const uint64_t *>(c->d.item_off);
      out->item_len = reinterpret_cast<const uint64_t *>(c->d.item_len);
    }
    return 0;
  }
  // host copies of the valid prefix: item views, block table, straddlers / decoded bytes
  rio_results &r = *res;
  if (r.records_cap < k.rec_bytes + 16) {
    if (r.records) hipHostFree(r.records);
    r.records = nullptr;
    r.records_cap = k.rec_bytes + k.rec_bytes / 4 + 4096;
    HIP_OK(hipHostMalloc((void **)&r.records, r.records_cap, hipHostMallocDefault));
  }
  if (r.items_cap < k.n_items + 1) {
    if (r.items) hipHostFree(r.items);
    r.items = nullptr;
    r.items_cap = k.n_items + k.n_items / 4 + 1024;
    HIP_OK(hipHostMalloc((void **)&r.items, r.items_cap * 16, hipHostMallocDefault));
  }
  if (r.blk_cap < 2 * (nb + 1)) {
    if (r.blk) hipHostFree(r.blk);
    r.blk = nullptr;
    r.blk_cap = 2 * (nb + 1) + 2048;
    HIP_OK(hipHostMalloc((void **)&r.blk, r.blk_cap * 8, hipHostMallocDefault));
  }
  unsigned long long *h_off = r.items, *h_len = r.items + r.items_cap;
  unsigned long long *first = r.blk, *foff = r.blk + nb + 1;
  // (the kernels that wrote these bytes have completed: the control block's sync)
  if (copy_to_host(c, r.records, d_records, k.rec_bytes) || copy_to_host(c, h_off, c->d.item_off, k.n_items * 8) ||
      copy_to_host(c, h_len, c->d.item_len, k.n_items * 8) ||
      copy_to_host(c, first, c->d.blk_item_base, (nb + 1) * 8) || copy_to_host(c, foff, c->d.blk_c0, nb * 8))
    return -1;
  const uint64_t d2h = k.rec_bytes + 16 * k.n_items + 8 * (2 * nb + 1);
  if (c->defer_collect) {  // rio_scan_span_end waits and converts the block offsets
    c->pend = true;
    c->pend_nb = nb;
    c->pend_foff = foff;
    c->pend_file_off = file_off;
    c->pend_d2h = d2h;
  } else {
    HIP_OK(hipStreamSynchronize(c->st));
    if (sdma_settle(c, kSdmaOut)) return -1;
    c->stats.d2h_bytes += d2h;
    for (uint64_t b = 0; b < nb; b++) foff[b] = file_off + foff[b] * kChunk;
  }
  out->records = r.records;
  out->item_off = reinterpret_cast<const uint64_t *>(h_off);
  out->item_len = reinterpret_cast<const uint64_t *>(h_len);
  out->block_first_item = reinterpret_cast<const uint64_t *>(first);
  out->block_file_off = reinterpret_cast<const uint64_t *>(foff);
  return 0;
}

// a run whose output did not fit (after the retries), or a layout fault
static void report_overflow(unsigned long long ov, uint64_t file_off, rio_error *err) {
  if (ov & kOvfLayout)
    rio_set_error(err, RIO_ERR_HIP, file_off, "internal error: k_crc's LDS tables are not at address 0 (build fault)");
  else
    rio_set_error(err, RIO_ERR_CAPACITY, file_off, "output capacity exceeded");
}

static int grow_for_overflow(rio_ctx *c, int32_t codec) {
  unsigned long long nb = 0, items = 0, side = 0;
  HIP_OK(hipMemcpy(&nb, c->nblocks_dev, 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&items, c->d.blk_item_base + nb, 8, hipMemcpyDeviceToHost));
  if (codec == RIO_CODEC_NONE) HIP_OK(hipMemcpy(&side, c->d.ck_sbase + c->last_nchunks, 8, hipMemcpyDeviceToHost));
  if (items > c->item_cap) {
    c->item_cap = items + items / 8 + 1024;
    if (dalloc(&c->d.item_off, c->item_cap) || dalloc(&c->d.item_len, c->item_cap)) return -1;
  }
  if (side > c->side_cap) {
    c->side_cap = side + side / 8 + 4096;
    if (dalloc(&c->d.side, c->side_cap)) return -1;
  }
  return 0;
}

// -DRIO_DEBUG_DUMP builds: per-block state of every run on stderr (development aid)
[[maybe_unused]] static void debug_dump(rio_ctx *c) {
  unsigned long long nb = 0;
  hipMemcpy(&nb, c->nblocks_dev, 8, hipMemcpyDeviceToHost);
  std::vector<unsigned long long> a(nb), st(nb), ol(nb), bl(nb), me(nb), doff(nb), ni(nb), ib(nb), ea(nb), eb(nb),
      hd(nb);
  if (nb) {
    hipMemcpy(a.data(), c->d.blk_c0, 8 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(st.data(), c->d.blk_status, 8 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(ol.data(), c->d.blk_out_len, 8 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(bl.data(), c->d.blk_len, 8 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(me.data(), c->d.blk_meta, 8 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(doff.data(), c->d.blk_dec_off, 8 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(ni.data(), c->d.blk_nitems, 8 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(ib.data(), c->d.blk_item_base, 8 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(ea.data(), c->d.blk_a, 8 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(eb.data(), c->d.blk_b, 8 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(hd.data(), c->d.blk_hdr, 8 * nb, hipMemcpyDeviceToHost);
  }
  fprintf(stderr, "rio debug: nblocks=%llu overflow=%llu flstat passes=%llu full=%llu esc=%llu\n", nb,
          (unsigned long long)c->h_ctl->out_overflow, (unsigned long long)c->h_ctl->pad[0],
          (unsigned long long)c->h_ctl->pad[1], (unsigned long long)c->h_ctl->flstat_esc);
  std::vector<FlState> fl(nb);
  if (nb && c->d.fl) hipMemcpy(fl.data(), c->d.fl, sizeof(FlState) * nb, hipMemcpyDeviceToHost);
  int shown = 0;
  for (uint64_t b = 0; b < nb && shown < 24; b++) {
    if (b >= 4 && st[b] == 0) continue;
    shown++;
    fprintf(stderr,
            "  blk %llu c0=%llu status=%llu meta=%llx len=%llu out_len=%llu dec_off=%llu nitems=%llu base=%llu "
            "a=%llu b=%llu hdr=%llx\n",
            (unsigned long long)b, a[b], st[b], me[b], bl[b], ol[b], doff[b], ni[b], ib[b], ea[b], eb[b], hd[b]);
    if (c->d.fl)
      fprintf(stderr, "    fl: mode=%u round=%u ntok=%u olen=%llu olen2=%llu bitpos=%llu hdrpos=%llu fast_err=%d\n", fl[b].mode,
              fl[b].round, fl[b].ntok, fl[b].olen, fl[b].olen2, fl[b].bitpos, fl[b].hdrpos, (int)fl[b].pad);
  }
}

static int run_chain(rio_ctx *c, const uint8_t *dspan, const uint8_t *report_span, uint64_t nbytes,
                     uint64_t file_off, int32_t is_file_end, uint64_t limit_off, int32_t codec, int32_t mode,
                     rio_results *res, rio_batch *out);

static int run_span(rio_ctx *c, const uint8_t *dspan, const uint8_t *report_span, uint64_t nbytes,
                    uint64_t file_off, int32_t is_file_end, uint64_t limit_off, int32_t codec, int32_t mode,
                    rio_results *res, rio_batch *out, int stage_flags = 0) {
  if (sdma_settle(c, kSdmaIn)) return -1;  // a host span's SDMA copy in, before the kernels that read it
  if (codec & RIO_CODEC_CHAIN_FLAG)
    return run_chain(c, dspan, report_span, nbytes, file_off, is_file_end, limit_off, codec, mode, res, out);
  const bool to_host = res != nullptr;
  HIP_OK(hipSetDevice(c->device));
  const uint64_t nchunks = nbytes / kChunk;
  const int tail_partial = (nbytes % kChunk) != 0;
  if (nchunks > c->max_chunks) {
    memset(out, 0, sizeof(*out));
    rio_set_error(&out->err, RIO_ERR_CAPACITY, file_off, "span of %" PRIu64 " bytes exceeds ctx capacity", nbytes);
    out->stop = RIO_STOP_ERROR;
    return 0;
  }
  uint64_t limit_chunk = UINT64_MAX;
  if (limit_off != UINT64_MAX) limit_chunk = limit_off <= file_off ? 0 : (limit_off - file_off + kChunk - 1) / kChunk;
  for (int attempt = 0; attempt < 4; attempt++) {
    if (enqueue(c, dspan, nchunks, limit_chunk, is_file_end, tail_partial, codec, mode, !to_host, attempt,
                stage_flags))
      return -1;
    HIP_OK(hipMemcpyAsync(c->h_ctl, c->d.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->st));
    HIP_OK(hipStreamSynchronize(c->st));
    note_split(c);
    if (c->h_ctl->out_overflow == 0 || (c->h_ctl->out_overflow & kOvfLayout)) break;
    if (grow_for_overflow(c, codec)) return -1;
    // decode regions: blocks that overflowed theirs carry their exact size (blk_need)
    // into the next attempt; a buffer too small for all regions grows to fit
    if (codec != RIO_CODEC_NONE && (c->h_ctl->out_overflow & 0x40) && ensure_dec(c, c->h_ctl->dec_need)) return -1;
    if ((c->h_ctl->out_overflow & kOvfZTok) && grow_ztok(c, c->h_ctl->tok_need)) return -1;
    // a flate block needed more Huffman/copy rounds than were launched
    if ((c->h_ctl->out_overflow & 0x1000) && c->fl_rounds < 64) c->fl_rounds = c->fl_rounds * 2 > 64 ? 64 : c->fl_rounds * 2;
  }
#ifdef RIO_DEBUG_DUMP
  debug_dump(c);
#endif
  float ms = 0;
  hipEventElapsedTime(&ms, c->ev[kEvStart], c->ev[kEvEnd]);
  // host results of a compressed codec: only the decoded record bytes cross PCIe
  c->last_cmp = false;
  if (to_host && codec != RIO_CODEC_NONE && !(stage_flags & kStageNoItems) && c->h_ctl->out_overflow == 0 &&
      c->h_ctl->n_valid_blocks > 0 && c->h_ctl->rec_bytes > 0) {
    if (c->d.cmp_cap < c->h_ctl->rec_bytes + 64) {
      if (dalloc(&c->d.cmp, c->h_ctl->rec_bytes + 64)) return -1;
      c->d.cmp_cap = c->h_ctl->rec_bytes + 64;
    }
    launch_compact(c->d, c->nblocks_dev, nchunks ? nchunks : 1, c->st);
    HIP_OK(hipMemcpyAsync(&c->h_ctl->rec_bytes, &c->d.ctl->rec_bytes, sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, c->st));
    HIP_OK(hipStreamSynchronize(c->st));
    c->last_cmp = true;
  }
  if (collect(c, report_span, file_off, codec, mode, nbytes, out, res)) return -1;
  out->kernel_ms = ms;
  if (c->h_ctl->out_overflow) {  // still short after the retries: report that, not what it garbled
    memset(&out->err, 0, sizeof(out->err));
    report_overflow(c->h_ctl->out_overflow, file_off, &out->err);
    out->stop = RIO_STOP_ERROR;
  }
  return 0;
}

// ------------------------------------------------------------ transformer chains
// registry.GetUntransformer's combined function (registry.go:121-146): the
// chain t0..tn-1 is untransformed tn-1 first. Stage 1 runs the file's chunks
// through everything but the packed parse -- chunk checks, CRC, block
// structure, tn-1's decode -- so its stop (EOF, trailer, shard limit, the first
// chunk or codec error) is the file's. The blocks it decoded are framed again as
// chunks (k_reframe: 32,740-byte payloads, the block's magic) and decoded by
// the next codec, and so on; the last stage also parses the packed headers.
// A later stage's error lies in a block before stage 1's stop, so it comes
// first in file order; it is reported at its block's file offset. (The
// reference hands each stage the same scratch buffer, so a stage whose output
// fits it can overwrite its own input; this implements the composition the
// chain describes.)
namespace rio {
void launch_reframe(const uint8_t *dec, const unsigned long long *dec_off, const unsigned long long *out_len,
                    const unsigned long long *soff, uint64_t nv, uint64_t magic, uint8_t *out, hipStream_t st);
}

static int ensure_dbuf(uint8_t **p, uint64_t *cap, uint64_t n) {
  if (*cap >= n) return 0;
  if (dalloc(p, n)) return -1;
  *cap = n;
  return 0;
}

static int run_chain(rio_ctx *c, const uint8_t *dspan, const uint8_t *report_span, uint64_t nbytes,
                     uint64_t file_off, int32_t is_file_end, uint64_t limit_off, int32_t codec, int32_t mode,
                     rio_results *res, rio_batch *out) {
  const int n = (codec >> 8) & 0xff;
  auto at = [&](int i) { return (codec >> (2 * i)) & 3; };
  // stage 1: the file's chunks, the last transformer's untransform
  if (run_span(c, dspan, report_span, nbytes, file_off, is_file_end, limit_off, at(n - 1), mode, res, out,
               kStageNoItems))
    return -1;
  const Ctl s1 = *c->h_ctl;
  const rio_batch b1 = *out;
  const uint64_t magic = mode == kModeHeader ? 0xf70416c25cd9e1d9ull
                         : mode == kModeTrailer ? 0x3a75dfcbd71abafeull : 0x2e3c0734eb47762eull;  // magic.go
  uint64_t nv = s1.n_valid_blocks;
  std::vector<unsigned long long> c0(nv), olen(nv), doff(nv);
  if (nv) {
    HIP_OK(hipMemcpy(c0.data(), c->d.blk_c0, nv * 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(olen.data(), c->d.blk_out_len, nv * 8, hipMemcpyDeviceToHost));
  }
  c->chain_c0 = c0;
  Ctl last = s1;      // the latest stage's control block
  bool later_err = false;
  for (int k = n - 2; k >= 0 && nv > 0; k--) {
    // reframe the nv blocks decoded by the previous stage
    std::vector<unsigned long long> soff(nv + 1, 0);
    for (uint64_t b = 0; b < nv; b++) soff[b + 1] = soff[b] + (olen[b] ? (olen[b] - 1) / kMaxPayload + 1 : 1);
    const uint64_t sbytes = soff[nv] * kChunk;
    uint8_t *buf = c->d_chain[k & 1];
    if (ensure_dbuf(&c->d_chain[k & 1], &c->d_chain_cap[k & 1], sbytes) ||
        ensure_dbuf(reinterpret_cast<uint8_t **>(&c->d_chain_meta), &c->d_chain_meta_cap, 8 * (nv + 1)))
      return -1;
    buf = c->d_chain[k & 1];
    HIP_OK(hipMemcpy(c->d_chain_meta, soff.data(), 8 * (nv + 1), hipMemcpyHostToDevice));
    launch_reframe(c->d.dec, c->d.blk_dec_off, c->d.blk_out_len, c->d_chain_meta, nv, magic, buf, c->st);
    HIP_OK(hipStreamSynchronize(c->st));
    // the stage's chunks may outnumber the file's (decoded bytes): the span grows
    // for this call
    if (reserve_tmp(c, sbytes)) return -1;
    if (run_span(c, buf, report_span, sbytes, file_off, 1, UINT64_MAX, at(k), mode, res, out,
                 kStageNoCrc | (k > 0 ? kStageNoItems : 0)))
      return -1;
    last = *c->h_ctl;
    if (c->h_ctl->stop_kind == 2) later_err = true;
    nv = c->h_ctl->n_valid_blocks;  // a stage stops at its first error
    if (k > 0 && nv) HIP_OK(hipMemcpy(olen.data(), c->d.blk_out_len, nv * 8, hipMemcpyDeviceToHost));
    if (later_err) break;
  }
  // the chain's result: the last stage's items; the stop is the first stage's
  // unless a later stage failed on a block before it
  if (n < 2 || s1.n_valid_blocks == 0) return 0;  // (no block reached a later stage: stage 1's batch stands)
  out->consumed = b1.consumed;
  out->in_bytes = b1.in_bytes;
  out->span = b1.span;
  if (later_err) {
    Ctl e = last;
    if (e.stop_block != kNone && e.stop_block < c0.size()) e.blk_c0 = c0[e.stop_block];
    rio_fill_error(e, file_off, mode, &out->err);
    out->stop = RIO_STOP_ERROR;
  } else if (out->err.code != RIO_ERR_CAPACITY) {
    out->stop = b1.stop;
    out->err = b1.err;
  }
  // host results: every block's offset in the file (the stages' own chunk
  // indexes are of the reframed spans)
  if (res && out->block_file_off)
    for (uint64_t b = 0; b < out->n_blocks && b < c0.size(); b++)
      const_cast<uint64_t *>(out->block_file_off)[b] = file_off + c0[b] * kChunk;
  return 0;
}

extern "C" int rio_scan_device(rio_ctx *ctx, const void *dev_span, uint64_t nbytes, uint64_t file_off,
                               int32_t is_file_end, uint64_t limit_off, int32_t codec, rio_batch *out) {
  if (!ctx || !out) return -1;
  memset(out, 0, sizeof(*out));
  if (rio_scan_span_end(ctx)) return -1;
  if (unstage(ctx)) return -1;
  if (!(codec & RIO_CODEC_CHAIN_FLAG) && settle(ctx)) return -1;  // (consecutive chain calls keep the growth)
  return run_span(ctx, (const uint8_t *)dev_span, (const uint8_t *)dev_span, nbytes, file_off, is_file_end,
                  limit_off, codec, kModeBody, nullptr, out);
}

static int stage_span(rio_ctx *c, const uint8_t *span, uint64_t nbytes) {
  if (!c->d_span) HIP_OK(hipMalloc((void **)&c->d_span, c->max_span + kChunk));
  // (the ctx's earlier kernels, which read d_span, have completed: a span's
  // batch is finished, rio_scan_span_end, before the next one is staged)
  if (copy_to_device(c, c->d_span, span, nbytes)) return -1;
  c->stats.h2d_bytes += nbytes;
  return 0;
}

extern "C" int rio_ctx_stats(rio_ctx *ctx, rio_stats *out) {
  if (!ctx || !out) return -1;
  *out = ctx->stats;
  out->span_cap = ctx->max_span;
  for (const rio_ctx *sb = ctx->sibling; sb; sb = sb->sibling) {  // (a scanner's spans ahead ran there)
    out->spans += sb->stats.spans;
    out->h2d_bytes += sb->stats.h2d_bytes;
    out->d2h_bytes += sb->stats.d2h_bytes;
    out->device_ms += sb->stats.device_ms;
  }
  return 0;
}

static int scan_span(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off, int32_t is_file_end,
                     uint64_t limit_off, int32_t codec, int32_t mode, rio_results *res, rio_batch *out, bool defer) {
  if (!ctx || !out) return -1;
  // staged by rio_scan_span_stage (its H2D copy enqueued, the ctx settled)
  const bool pre = span && ctx->staged == span && ctx->staged_n == nbytes;
  if (pre) ctx->staged = nullptr;
  else if (unstage(ctx)) return -1;
  hipEvent_t t0, t1;
  if (pre) {
    memset(out, 0, sizeof(*out));
    if (hipSetDevice(ctx->device) != hipSuccess) return -1;
    t0 = ctx->staged_t0;
    hipEventCreate(&t1);
  } else {
    if (rio_scan_span_end(ctx)) return -1;  // (a deferred batch of this ctx: complete before its buffers are reused)
    memset(out, 0, sizeof(*out));
    if (!(codec & RIO_CODEC_CHAIN_FLAG) && settle(ctx)) return -1;
    if (nbytes > ctx->max_span + kChunk) {
      rio_set_error(&out->err, RIO_ERR_CAPACITY, file_off, "span of %" PRIu64 " bytes exceeds ctx capacity", nbytes);
      out->stop = RIO_STOP_ERROR;
      return 0;
    }
    if (hipSetDevice(ctx->device) != hipSuccess) return -1;
    hipEventCreate(&t0);
    hipEventCreate(&t1);
    hipEventRecord(t0, ctx->st);
    if (stage_span(ctx, span, nbytes)) return -1;
  }
  // (a chain's stages read their results on the host: never deferred)
  ctx->defer_collect = defer && !(codec & RIO_CODEC_CHAIN_FLAG);
  const int rc = run_span(ctx, ctx->d_span, span, nbytes, file_off, is_file_end, limit_off, codec, mode,
                          res ? res : &ctx->res, out);
  ctx->defer_collect = false;
  hipEventRecord(t1, ctx->st);
  if (ctx->pend) {
    if (rc) {  // (no batch to finish)
      ctx->pend = false;
      hipEventSynchronize(t1);
    } else {
      ctx->pend_t0 = t0;
      ctx->pend_t1 = t1;
      return 0;
    }
  }
  hipEventSynchronize(t1);
  float ms = 0;
  hipEventElapsedTime(&ms, t0, t1);
  out->total_ms = ms;
  ctx->stats.spans++;
  ctx->stats.device_ms += ms;
  hipEventDestroy(t0);
  hipEventDestroy(t1);
  return rc;
}

int rio_scan_span_mode(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off, int32_t is_file_end,
                       uint64_t limit_off, int32_t codec, int32_t mode, rio_results *res, rio_batch *out) {
  return scan_span(ctx, span, nbytes, file_off, is_file_end, limit_off, codec, mode, res, out, false);
}

int rio_scan_span_stage(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, int32_t codec) {
  if (!ctx || !span) return -1;
  if (unstage(ctx)) return -1;
  if (rio_scan_span_end(ctx)) return -1;
  if ((codec & RIO_CODEC_CHAIN_FLAG) || nbytes > ctx->max_span + kChunk) return 0;  // (staged by the decode)
  if (settle(ctx)) return -1;
  if (hipSetDevice(ctx->device) != hipSuccess) return -1;
  hipEventCreate(&ctx->staged_t0);
  hipEventRecord(ctx->staged_t0, ctx->st);
  if (stage_span(ctx, span, nbytes)) return -1;
  ctx->staged = span;
  ctx->staged_n = nbytes;
  return 0;
}

int rio_ctx_wait_staged(rio_ctx *ctx) {
  if (!ctx || !ctx->staged) return 0;
  if (hipSetDevice(ctx->device) != hipSuccess) return -1;
  if (sdma_settle(ctx, kSdmaIn)) return -1;
  HIP_OK(hipStreamSynchronize(ctx->st));  // (a copy the stream ran: no SDMA engine)
  return 0;
}

int rio_scan_span_begin(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off, int32_t is_file_end,
                        uint64_t limit_off, int32_t codec, rio_results *res, rio_batch *out) {
  return scan_span(ctx, span, nbytes, file_off, is_file_end, limit_off, codec, 0, res, out, true);
}

int rio_scan_span_end(rio_ctx *ctx) {
  if (!ctx || !ctx->pend) return 0;
  ctx->pend = false;
  HIP_OK(hipSetDevice(ctx->device));
  hipError_t e = hipEventSynchronize(ctx->pend_t1);
  if (e == hipSuccess && sdma_settle(ctx, kSdmaOut)) e = hipErrorUnknown;  // the results' SDMA copies
  float ms = 0;
  hipEventElapsedTime(&ms, ctx->pend_t0, ctx->pend_t1);
  hipEventDestroy(ctx->pend_t0);
  hipEventDestroy(ctx->pend_t1);
  if (e != hipSuccess) {
    set_last_error("HIP error %d (%s) waiting for a span's results", (int)e, hipGetErrorString(e));
    return -1;
  }
  for (uint64_t b = 0; b < ctx->pend_nb; b++) ctx->pend_foff[b] = ctx->pend_file_off + ctx->pend_foff[b] * kChunk;
  ctx->stats.d2h_bytes += ctx->pend_d2h;
  ctx->stats.spans++;
  ctx->stats.device_ms += ms;
  return 0;
}

rio_ctx *rio_ctx_sibling(rio_ctx *c) {
  if (!c) return nullptr;
  if (!c->sibling) {
    rio_config cf = c->cfg;
    cf.max_span_bytes = c->max_span;
    c->sibling = rio_open(&cf);
  }
  return c->sibling;
}

extern "C" int rio_scan_span(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off,
                             int32_t is_file_end, uint64_t limit_off, int32_t codec, rio_batch *out) {
  return rio_scan_span_mode(ctx, span, nbytes, file_off, is_file_end, limit_off, codec, kModeBody, nullptr, out);
}

extern "C" int rio_scan_device_async(rio_ctx *ctx, const void *dev_span, uint64_t nbytes, uint64_t file_off,
                                     int32_t codec) {
  if (!ctx) return -1;
  HIP_OK(hipSetDevice(ctx->device));
  if (rio_scan_span_end(ctx)) return -1;
  if (unstage(ctx)) return -1;
  if (!(codec & RIO_CODEC_CHAIN_FLAG) && settle(ctx)) return -1;
  if (codec & RIO_CODEC_CHAIN_FLAG) {
    // a chain's stages run here, one after the other (each needs the previous
    // one's block sizes on the host): the call returns when they are done and
    // rio_sync hands back their batch
    ctx->last_nseg = 0;
    ctx->chain_async = false;
    memset(&ctx->chain_batch, 0, sizeof(ctx->chain_batch));
    if (run_span(ctx, (const uint8_t *)dev_span, (const uint8_t *)dev_span, nbytes, file_off, 1, UINT64_MAX, codec,
                 kModeBody, nullptr, &ctx->chain_batch))
      return -1;
    ctx->chain_async = true;
    ctx->last_codec = codec;
    return 0;
  }
  const uint64_t nchunks = nbytes / kChunk;
  if (nchunks > ctx->max_chunks) {
    set_last_error("span exceeds ctx capacity");
    return -1;
  }
  ctx->last_nchunks = nchunks;
  ctx->last_file_off = file_off;
  ctx->last_in_bytes = nbytes;
  ctx->last_codec = codec;
  ctx->last_mode = kModeBody;
  ctx->last_span = (const uint8_t *)dev_span;
  ctx->last_nseg = 0;
  return enqueue(ctx, (const uint8_t *)dev_span, nchunks, UINT64_MAX, 1, (nbytes % kChunk) != 0, codec, kModeBody,
                 true, 0, 0, /*may_sync=*/false);
}

extern "C" int rio_scan_device_segments_async(rio_ctx *ctx, const void *dev_span, uint64_t nbytes,
                                              const uint64_t *seg_end, const uint64_t *seg_file_off, uint64_t nseg,
                                              int32_t codec) {
  if (!ctx || (nseg && (!seg_end || !seg_file_off))) return -1;
  for (uint64_t s = 0; s < nseg; s++) {
    const uint64_t lo = s ? seg_end[s - 1] : 0;
    if (seg_end[s] < lo || seg_end[s] % kChunk != 0 || seg_file_off[s] % kChunk != 0) {
      set_last_error("segment %" PRIu64 ": ends must ascend, ends and file offsets be multiples of 32768", s);
      return -1;
    }
  }
  if (nseg && seg_end[nseg - 1] != (nbytes + kChunk - 1) / kChunk * kChunk) {
    set_last_error("the segments must cover the span");
    return -1;
  }
  HIP_OK(hipSetDevice(ctx->device));
  if (ctx->d_seg_cap < 2 * nseg + 2) {
    if (dalloc(&ctx->d_seg, 2 * nseg + 2)) return -1;
    ctx->d_seg_cap = 2 * nseg + 2;
  }
  ctx->seg_end_h.assign(seg_end, seg_end + nseg);
  ctx->seg_file_h.assign(seg_file_off, seg_file_off + nseg);
  if (nseg) {  // (the host copies outlive the async copies)
    HIP_OK(hipMemcpyAsync(ctx->d_seg, ctx->seg_end_h.data(), nseg * 8, hipMemcpyHostToDevice, ctx->st));
    HIP_OK(hipMemcpyAsync(ctx->d_seg + nseg, ctx->seg_file_h.data(), nseg * 8, hipMemcpyHostToDevice, ctx->st));
  }
  if (rio_scan_device_async(ctx, dev_span, nbytes, 0, codec)) return -1;
  ctx->last_nseg = nseg;
  if (nseg && ctx->chain_async) {
    // the last stage's blocks are stage 1's, in order: their segments and
    // file offsets from stage 1's chunk indexes (the last stage's are of its
    // reframed span)
    const uint64_t nv = ctx->chain_c0.size();
    if (ctx->d_chain_c0_cap < nv + 1) {
      if (dalloc(&ctx->d_chain_c0, nv + 1)) return -1;
      ctx->d_chain_c0_cap = nv + 1;
    }
    if (nv) HIP_OK(hipMemcpy(ctx->d_chain_c0, ctx->chain_c0.data(), nv * 8, hipMemcpyHostToDevice));
    DevBufs d1 = ctx->d;
    d1.blk_c0 = ctx->d_chain_c0;
    launch_block_files(d1, ctx->d_seg, ctx->d_seg + nseg, nseg, nv ? nv : 1, ctx->st);
  } else if (nseg) {
    launch_block_files(ctx->d, ctx->d_seg, ctx->d_seg + nseg, nseg, ctx->last_nchunks ? ctx->last_nchunks : 1,
                       ctx->st);
  }
  return 0;
}

static int sync_segments(rio_ctx *ctx, rio_batch *out);

extern "C" int rio_sync(rio_ctx *ctx, rio_batch *out) {
  if (!ctx || !out) return -1;
  HIP_OK(hipSetDevice(ctx->device));
  if (ctx->chain_async) {  // a chain's batch (its stages ran at the async call)
    ctx->chain_async = false;
    HIP_OK(hipStreamSynchronize(ctx->st));
    *out = ctx->chain_batch;
    return sync_segments(ctx, out);
  }
  HIP_OK(hipMemcpyAsync(ctx->h_ctl, ctx->d.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, ctx->st));
  HIP_OK(hipStreamSynchronize(ctx->st));
  note_split(ctx);
  // a buffer the launch found too small (decode regions, zstd scratch, items,
  // straddlers, flate rounds): grown to what it reported and the span run
  // again here, synchronously, as run_span's attempts do -- so an asynchronous
  // scan's first span sizes the context instead of failing
  for (int attempt = 1; attempt < 4; attempt++) {
    const unsigned long long ov = ctx->h_ctl->out_overflow;
    if (ov == 0 || (ov & kOvfLayout)) break;
    if (grow_for_overflow(ctx, ctx->last_codec)) return -1;
    if ((ov & 0x40) && ensure_dec(ctx, ctx->h_ctl->dec_need)) return -1;
    if ((ov & kOvfZTok) && grow_ztok(ctx, ctx->h_ctl->tok_need)) return -1;
    if ((ov & 0x1000) && ctx->fl_rounds < 64) ctx->fl_rounds = ctx->fl_rounds * 2 > 64 ? 64 : ctx->fl_rounds * 2;
    if (enqueue(ctx, ctx->last_span, ctx->last_nchunks, UINT64_MAX, 1, (ctx->last_in_bytes % kChunk) != 0,
                ctx->last_codec, ctx->last_mode, true, attempt, 0, false))
      return -1;
    if (ctx->last_nseg)
      launch_block_files(ctx->d, ctx->d_seg, ctx->d_seg + ctx->last_nseg, ctx->last_nseg,
                         ctx->last_nchunks ? ctx->last_nchunks : 1, ctx->st);
    HIP_OK(hipMemcpyAsync(ctx->h_ctl, ctx->d.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, ctx->st));
    HIP_OK(hipStreamSynchronize(ctx->st));
    note_split(ctx);
  }
#ifdef RIO_ZPROF  // profiling builds: where the zstd entropy pass spends its cycles
  if (ctx->last_codec == RIO_CODEC_ZSTD)
    fprintf(stderr, "rio: zstd blocks on the serial path: %llu; entropy-pass cycles lit %llu tables %llu seq %llu block %llu\n",
            (unsigned long long)ctx->h_ctl->pad[1], ctx->h_ctl->zprof[0], ctx->h_ctl->zprof[1], ctx->h_ctl->zprof[2],
            ctx->h_ctl->zprof[3]);
  if (ctx->last_codec == RIO_CODEC_ZSTD)
    fprintf(stderr, "rio: zstd execution parts with matches %llu, matches %llu, copied in order %llu\n",
            ctx->h_ctl->zx[1], ctx->h_ctl->zx[2], ctx->h_ctl->zx[3]);
#endif
#ifdef RIO_FLSTAT  // statistics builds: the flate copy pass's batches
  if (ctx->last_codec == RIO_CODEC_FLATE)
    fprintf(stderr, "rio flstat: batches %llu tokens %llu pending %llu hbm-sourced %llu rounds %llu split-blocks %llu\n",
            ctx->h_ctl->zprof[0], ctx->h_ctl->zprof[1], ctx->h_ctl->zprof[2], ctx->h_ctl->zprof[3],
            ctx->h_ctl->flstat_esc, ctx->h_ctl->seg_blocks);
#endif
  float ms = 0;
  hipEventElapsedTime(&ms, ctx->ev[kEvStart], ctx->ev[kEvEnd]);
  if (collect(ctx, ctx->last_span, ctx->last_file_off, ctx->last_codec, ctx->last_mode, ctx->last_in_bytes, out,
              nullptr))
    return -1;
  out->kernel_ms = ms;
  if (ctx->h_ctl->out_overflow) {
    report_overflow(ctx->h_ctl->out_overflow, 0, &out->err);
    out->stop = RIO_STOP_ERROR;
  }
  return sync_segments(ctx, out);
}

// segment scans: per-block files, and the error's file
static int sync_segments(rio_ctx *ctx, rio_batch *out) {
  if (ctx->last_nseg) {
    out->block_file_off = reinterpret_cast<const uint64_t *>(ctx->d.blk_file_off);
    out->block_segment = reinterpret_cast<const uint64_t *>(ctx->d.blk_seg);
    if (out->stop == RIO_STOP_ERROR) {
      const std::vector<uint64_t> &e = ctx->seg_end_h;
      const uint64_t so = out->err.file_off;  // a span offset (the span starts at 0)
      const uint64_t s = (uint64_t)(std::upper_bound(e.begin(), e.end(), so) - e.begin());
      if (s < e.size()) {
        out->err_segment = (int64_t)s;
        out->err.file_off = ctx->seg_file_h[s] + so - (s ? e[s - 1] : 0);
      }
    }
  }
  return 0;
}

extern "C" uint64_t rio_flate_split_blocks(rio_ctx *ctx) { return ctx ? ctx->h_ctl->seg_blocks : 0; }

extern "C" int rio_stage_times(rio_ctx *ctx, float *ms, int n) {
  if (!ctx || !ms || n <= 0) return 0;
  float t[5] = {0, 0, 0, 0, 0};
  hipEventElapsedTime(&t[0], ctx->ev[ctx->ev_parse0], ctx->ev[kEvParse1]);
  if (ctx->last_had_dec) hipEventElapsedTime(&t[1], ctx->ev[kEvScans], ctx->ev[kEvDec]);
  hipEventElapsedTime(&t[2], ctx->ev[ctx->ev_crc0], ctx->ev[kEvCrc1]);
  hipEventElapsedTime(&t[3], ctx->ev[kEvStart], ctx->ev[kEvScans]);
  hipEventElapsedTime(&t[4], ctx->ev[kEvStart], ctx->ev[kEvEnd]);
  const int k = n < 5 ? n : 5;
  for (int i = 0; i < k; i++) ms[i] = t[i];
  return k;
}

// TransformFunc analogue (recordio.go:12).
//
// none: idTransform, the concatenation of the payloads (registry.go:31-39).
// flate / zstd (recordioflate.go:54-65, recordiozstd.go:67-78): the payload
// views are laid out as one block of whole chunks in pinned staging -- the
// chunk stream the codec kernels read, whose logical payload view is
// recordioiov's gather over the slices (recordioiov.go:14-58) -- copied to the
// device and run through the chunk scans and the codec stage alone (kModeRaw:
// no CRC, no packed parse). The decoded block, varint header included, comes
// back into scratch.
static const uint8_t kPackedMagic[8] = {0x2e, 0x76, 0x47, 0xeb, 0x34, 0x07, 0x3c, 0x2e};  // magic.go:21

static int decode_raw(rio_ctx *c, const uint8_t *const *payloads, const uint32_t *lens, int n, int32_t codec,
                      uint8_t *scratch, uint64_t cap, uint64_t *out_len, rio_error *err) {
  uint64_t total = 0;
  for (int i = 0; i < n; i++) total += lens[i];
  const uint64_t nch = total ? (total + kMaxPayload - 1) / kMaxPayload : 1;
  const uint64_t nbytes = nch * kChunk;
  if (reserve_tmp(c, nbytes)) return -1;  // a block longer than the span: the span grows to it (this call)
  if (c->h_stage_cap < nbytes) {
    if (c->h_stage) hipHostFree(c->h_stage);
    c->h_stage = nullptr;
    c->h_stage_cap = 0;
    HIP_OK(hipHostMalloc((void **)&c->h_stage, nbytes, hipHostMallocDefault));
    c->h_stage_cap = nbytes;
  }
  int pi = 0;
  uint32_t po = 0;  // position in payloads[pi]
  for (uint64_t k = 0; k < nch; k++) {
    uint8_t *ck = c->h_stage + k * kChunk;
    const uint64_t left = total - k * (uint64_t)kMaxPayload;
    const uint32_t sz = (uint32_t)(left < (uint64_t)kMaxPayload ? left : (uint64_t)kMaxPayload);
    const uint32_t hdr[5] = {0u, 0u, sz, (uint32_t)nch, (uint32_t)k};  // crc flag size total index (chunk.go:31-53)
    memcpy(ck, kPackedMagic, 8);
    memcpy(ck + 8, hdr, sizeof(hdr));
    uint32_t o = 0;
    while (o < sz) {
      while (pi < n && po >= lens[pi]) {
        pi++;
        po = 0;
      }
      const uint32_t m = (lens[pi] - po) < (sz - o) ? (lens[pi] - po) : (sz - o);
      memcpy(ck + kChunkHdr + o, payloads[pi] + po, m);
      o += m;
      po += m;
    }
    memset(ck + kChunkHdr + sz, 0, kChunk - kChunkHdr - sz);
  }
  if (!c->d_span) HIP_OK(hipMalloc((void **)&c->d_span, c->max_span + kChunk));
  HIP_OK(hipMemcpyAsync(c->d_span, c->h_stage, nbytes, hipMemcpyHostToDevice, c->st));
  for (int attempt = 0; attempt < 4; attempt++) {
    if (enqueue(c, c->d_span, nch, UINT64_MAX, 1, 0, codec, kModeRaw, false, attempt)) return -1;
    HIP_OK(hipMemcpyAsync(c->h_ctl, c->d.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->st));
    HIP_OK(hipStreamSynchronize(c->st));
    note_split(c);
    const unsigned long long ov = c->h_ctl->out_overflow;
    if (ov == 0) break;
    if ((ov & 0x40) && ensure_dec(c, c->h_ctl->dec_need)) return -1;
    if ((ov & kOvfZTok) && grow_ztok(c, c->h_ctl->tok_need)) return -1;
    if ((ov & 0x1000) && c->fl_rounds < 64) c->fl_rounds = c->fl_rounds * 2 > 64 ? 64 : c->fl_rounds * 2;
  }
  if (c->h_ctl->out_overflow) {
    rio_set_error(err, RIO_ERR_CAPACITY, 0, "output capacity exceeded");
    return RIO_ERR_CAPACITY;
  }
  unsigned long long st = 0, ea = 0, eb = 0, olen = 0, doff = 0;
  HIP_OK(hipMemcpy(&st, c->d.blk_status, 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&ea, c->d.blk_a, 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&eb, c->d.blk_b, 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&olen, c->d.blk_out_len, 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&doff, c->d.blk_dec_off, 8, hipMemcpyDeviceToHost));
  if (st == kBlkCodec) {
    codec_error_text(ea, eb, 0, err);
    *out_len = 0;
    return err->code;
  }
  *out_len = olen;
  if (olen > cap) {
    rio_set_error(err, RIO_ERR_CAPACITY, 0, "scratch too small: need %" PRIu64, (uint64_t)olen);
    return RIO_ERR_CAPACITY;
  }
  if (olen) HIP_OK(hipMemcpy(scratch, c->d.dec + doff, olen, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int rio_decode_block(rio_ctx *ctx, const uint8_t *const *payloads, const uint32_t *lens, int n,
                                int32_t codec, uint8_t *scratch, uint64_t cap, uint64_t *out_len, rio_error *err) {
  if (!ctx || n < 0 || (n > 0 && (!payloads || !lens)) || !out_len) return -1;
  if (rio_scan_span_end(ctx)) return -1;
  if (settle(ctx)) return -1;
  rio_error scratch_err;
  if (!err) err = &scratch_err;
  memset(err, 0, sizeof(*err));
  *out_len = 0;
  uint64_t total = 0;
  for (int i = 0; i < n; i++) total += lens[i];
  if (codec == RIO_CODEC_NONE) {  // idTransform: concatenation (registry.go:31-39)
    *out_len = total;
    if (total > cap) {
      rio_set_error(err, RIO_ERR_CAPACITY, 0, "scratch too small: need %" PRIu64, total);
      return RIO_ERR_CAPACITY;
    }
    uint64_t o = 0;
    for (int i = 0; i < n; i++) {
      memcpy(scratch + o, payloads[i], lens[i]);
      o += lens[i];
    }
    return 0;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return -1;
  if (codec & RIO_CODEC_CHAIN_FLAG) {  // registry.go:121-146: the last transformer's untransform first
    const int m = (codec >> 8) & 0xff;
    if (m < 2 || m > 4) {
      rio_set_error(err, RIO_ERR_ARG, 0, "bad chain codec %d", codec);
      return RIO_ERR_ARG;
    }
    std::vector<uint8_t> cur;
    const uint8_t *const *ps = payloads;
    const uint32_t *ls = lens;
    int np = n;
    const uint8_t *one[1];
    uint32_t one_len[1];
    for (int k = m - 1; k >= 0; k--) {
      const int32_t ck = (codec >> (2 * k)) & 3;
      uint64_t need = 0;
      int rc;
      std::vector<uint8_t> nxt(k ? (size_t)(64 << 10) : 0);
      for (;;) {  // the stage's output: scratch for the last stage, a host buffer before it
        uint8_t *dst = k ? nxt.data() : scratch;
        const uint64_t dcap = k ? nxt.size() : cap;
        rc = decode_raw(ctx, ps, ls, np, ck, dst, dcap, &need, err);
        if (k && rc == RIO_ERR_CAPACITY && need > nxt.size()) {
          nxt.resize((size_t)need);
          continue;
        }
        break;
      }
      if (rc) {
        *out_len = need;
        return rc;
      }
      if (k == 0) {
        *out_len = need;
        return 0;
      }
      if (need > UINT32_MAX) {
        rio_set_error(err, RIO_ERR_CAPACITY, 0, "chain stage output of %" PRIu64 " bytes", need);
        return RIO_ERR_CAPACITY;
      }
      nxt.resize((size_t)need);
      cur.swap(nxt);
      one[0] = cur.data();
      one_len[0] = (uint32_t)cur.size();
      ps = one;
      ls = one_len;
      np = 1;
    }
    return 0;
  }
  if (codec != RIO_CODEC_FLATE && codec != RIO_CODEC_ZSTD) {
    rio_set_error(err, RIO_ERR_ARG, 0, "unknown codec %d", codec);
    return RIO_ERR_ARG;
  }
  return decode_raw(ctx, payloads, lens, n, codec, scratch, cap, out_len, err);
}

// ------------------------------------------------------------ v1 (legacy) spans
// A span of v1 records (recordio/deprecated/recordio.go:80-86: [magic 8][size
// u64][crc32 of size u32][payload]) decoded as legacyScannerAdapter reads them
// (recordio/legacyscanner.go:84-117). The record chain is serial -- each
// record starts where the previous one ends -- so the host walks the 20-byte
// headers (InternalScan, recordio.go:258-300: header CRC, size limit, truncation,
// magic) and checks each packed record's item count; every packed record's
// sizes, header CRC and item views run on the GPU at once (legacy.hip). An
// unpacked record is one item, the record itself.
namespace {

const uint8_t kV1MagicUnpacked[8] = {0xfc, 0xae, 0x95, 0x31, 0xf0, 0xd9, 0xbd, 0x20};
const uint8_t kV1MagicPacked[8] = {0x2e, 0x76, 0x47, 0xeb, 0x34, 0x07, 0x3c, 0x2e};
constexpr uint64_t kV1MaxRecord = 1ull << 29;  // internal.MaxReadRecordSize, magic.go:33

uint64_t v1_uvarint(const uint8_t *p, uint64_t n, int64_t *cnt) {  // binary.Uvarint, Go 1.13
  uint64_t x = 0;
  unsigned s = 0;
  for (uint64_t i = 0; i < n; i++) {
    const uint8_t b = p[i];
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) {
        *cnt = -(int64_t)(i + 1);
        return 0;
      }
      *cnt = (int64_t)i + 1;
      return x | ((uint64_t)b << s);
    }
    if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
  *cnt = 0;
  return 0;
}

// CRC32-IEEE of the 8 bytes of a record header's size field: slicing-by-8
uint32_t v1_crc8(const uint8_t *p) {
  static const std::vector<uint32_t> tab = [] {
    std::vector<uint32_t> t(8 * 256);
    for (uint32_t b = 0; b < 256; b++) {
      uint32_t c = b;
      for (int k = 0; k < 8; k++) c = (c & 1) ? kPoly ^ (c >> 1) : c >> 1;
      t[b] = c;
    }
    for (int s = 1; s < 8; s++)
      for (uint32_t b = 0; b < 256; b++) t[s * 256 + b] = (t[(s - 1) * 256 + b] >> 8) ^ t[t[(s - 1) * 256 + b] & 0xff];
    return t;
  }();
  uint32_t lo, hi;
  memcpy(&lo, p, 4);
  memcpy(&hi, p + 4, 4);
  lo ^= 0xFFFFFFFFu;
  const uint32_t *T = tab.data();
  const uint32_t c = T[7 * 256 + (lo & 0xff)] ^ T[6 * 256 + ((lo >> 8) & 0xff)] ^ T[5 * 256 + ((lo >> 16) & 0xff)] ^
                     T[4 * 256 + (lo >> 24)] ^ T[3 * 256 + (hi & 0xff)] ^ T[2 * 256 + ((hi >> 8) & 0xff)] ^
                     T[1 * 256 + ((hi >> 16) & 0xff)] ^ T[hi >> 24];
  return ~c;
}

int dgrow(uint8_t **p, uint64_t *cap, uint64_t n) {
  if (*cap >= n) return 0;
  const uint64_t c = n + n / 4 + 64;
  if (dalloc(p, c)) return -1;
  *cap = c;
  return 0;
}

int host_results(rio_results &r, uint64_t n_items, uint64_t nb) {
  if (r.items_cap < n_items + 1) {
    if (r.items) hipHostFree(r.items);
    r.items = nullptr;
    r.items_cap = n_items + n_items / 4 + 1024;
    HIP_OK(hipHostMalloc((void **)&r.items, r.items_cap * 16, hipHostMallocDefault));
  }
  if (r.blk_cap < 2 * (nb + 1)) {
    if (r.blk) hipHostFree(r.blk);
    r.blk = nullptr;
    r.blk_cap = 2 * (nb + 1) + 2048;
    HIP_OK(hipHostMalloc((void **)&r.blk, r.blk_cap * 8, hipHostMallocDefault));
  }
  return 0;
}

}  // namespace

int rio_scan_v1_span_mode(rio_ctx *c, const uint8_t *span, uint64_t nbytes, uint64_t file_off, int32_t is_file_end,
                          rio_results *res, rio_batch *out) {
  if (!c || !out) return -1;
  memset(out, 0, sizeof(*out));
  HIP_OK(hipSetDevice(c->device));
  if (rio_scan_span_end(c)) return -1;
  if (settle(c)) return -1;
  rio_results &r = res ? *res : c->res;
  std::vector<V1Rec> &recs = c->v1_recs;
  std::vector<V1Job> &jobs = c->v1_jobs;
  std::vector<uint64_t> &job_rec = c->v1_job_rec;
  std::vector<V1Unp> &unp = c->v1_unp;
  recs.clear();
  jobs.clear();
  job_rec.clear();
  unp.clear();
  rio_error e{};
  bool err = false;
  int32_t stop = RIO_STOP_MORE;
  uint64_t p = 0, items = 0, need = 0, staged = 0;
  for (;;) {
    if (p == nbytes) {
      if (is_file_end) stop = RIO_STOP_EOF;
      break;
    }
    const uint64_t left = nbytes - p;
    const uint64_t at = file_off + p;
    if (left < 20) {
      if (is_file_end) {
        rio_set_error(&e, RIO_ERR_V1_RECORD, at, "recordio: failed to read header: unexpected EOF");
        err = true;
      } else {
        need = 20;
      }
      break;
    }
    const uint8_t *h = span + p;
    uint64_t size;
    uint32_t crc;
    memcpy(&size, h + 8, 8);
    memcpy(&crc, h + 16, 4);
    const uint32_t ncrc = v1_crc8(h + 8);  // unmarshalHeader, recordio.go:324-334
    if (ncrc != crc) {
      rio_set_error(&e, RIO_ERR_V1_RECORD, at, "recordio: crc check failed - corrupt record header (%u != %u)?", ncrc,
                    crc);
      e.a = ncrc;
      e.b = crc;
      err = true;
      break;
    }
    if (size > kV1MaxRecord) {
      rio_set_error(&e, RIO_ERR_V1_RECORD, at,
                    "recordio: unreasonably large read record encountered: %" PRIu64 " > %" PRIu64 " bytes", size,
                    kV1MaxRecord);
      err = true;
      break;
    }
    if (size > left - 20) {
      if (!is_file_end) {
        need = 20 + size;
      } else if (left == 20) {  // io.ReadFull read nothing: (0, io.EOF), then the length check
        rio_set_error(&e, RIO_ERR_V1_RECORD, at, "recordio: short/long record: 0 < %" PRIu64, size);
        err = true;
      } else {
        rio_set_error(&e, RIO_ERR_V1_RECORD, at, "recordio: failed to read record: unexpected EOF");
        err = true;
      }
      break;
    }
    const uint8_t *pay = h + 20;
    if (memcmp(h, kV1MagicPacked, 8) == 0) {  // Unpack's checks before the sizes (packer.go:215-229)
      if (size < 4) {
        rio_set_error(&e, RIO_ERR_V1_PACKED, at, "recordio: failed to read crc32");
        err = true;
        break;
      }
      int64_t n;
      const uint64_t nb = v1_uvarint(pay + 4, size - 4, &n);
      if (n <= 0) {
        rio_set_error(&e, RIO_ERR_NITEMS, at, "recordio: failed to read number of packed items: %" PRId64, n);
        err = true;
        break;
      }
      if (nb > size) {
        rio_set_error(&e, RIO_ERR_V1_PACKED, at,
                      "recordio: likely corrupt data, number of packed items exceeds the number of bytes in the "
                      "record (%" PRIu64 " > %" PRIu64 ")",
                      nb, size);
        err = true;
        break;
      }
      // a valid header fits in crc + count + 10 bytes per size varint
      const uint64_t bound = 4 + (uint64_t)n + 10 * nb;
      const uint64_t hb = bound < size ? bound : size;
      job_rec.push_back(recs.size());
      jobs.push_back(V1Job{staged, size, nb, items, hb, p + 20});
      staged += (hb + 15) & ~15ull;
      recs.push_back(V1Rec{p, items});
      items += nb ? nb : 1;
    } else if (memcmp(h, kV1MagicUnpacked, 8) == 0) {
      unp.push_back(V1Unp{items, p + 20, size});
      recs.push_back(V1Rec{p, items});
      items += 1;
    } else {
      rio_set_error(&e, RIO_ERR_BAD_MAGIC, at, "recordio: invalid magic number: [%u %u %u %u %u %u %u %u]", h[0],
                    h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
      err = true;
      break;
    }
    p += 20 + size;
  }
  if (err) stop = RIO_STOP_ERROR;
  if (host_results(r, items, recs.size())) return -1;
  unsigned long long *h_off = r.items, *h_len = r.items + r.items_cap;
  float kms = 0;
  uint64_t nrec = recs.size(), nitems = items, consumed = p;
  if (!jobs.empty()) {
    if (c->d_v1_jobs_cap < jobs.size()) {
      const uint64_t cap = jobs.size() + jobs.size() / 4 + 64;
      if (dalloc(&c->d_v1_jobs, cap) || dalloc(&c->d_v1_res, cap)) return -1;
      c->d_v1_jobs_cap = cap;
    }
    if (c->d_v1_items_cap < items) {
      const uint64_t cap = items + items / 4 + 1024;
      if (dalloc(&c->d_v1_off, cap) || dalloc(&c->d_v1_len, cap)) return -1;
      c->d_v1_items_cap = cap;
    }
    std::vector<V1Res> &jr = c->v1_res;
    jr.resize(jobs.size());
    // round 0: every packed record's header bound; round 1: the records whose
    // header ran past it, whole (their error is then exact)
    std::vector<V1Job> run;
    std::vector<uint64_t> sel;
    for (int round = 0; round < 2; round++) {
      if (round == 1) {
        run.clear();
        uint64_t at = 0;
        for (size_t k = 0; k < jobs.size(); k++) {
          if (jr[k].status != kV1More) continue;
          V1Job j = jobs[k];
          j.off = at;
          j.hbytes = j.size;
          at += (j.size + 15) & ~15ull;
          run.push_back(j);
          sel.push_back(k);
        }
        if (run.empty()) break;
        staged = at;
      }
      const std::vector<V1Job> &rj = round == 0 ? jobs : run;
      if (c->h_v1_cap < staged + 64) {
        if (c->h_v1) hipHostFree(c->h_v1);
        c->h_v1 = nullptr;
        c->h_v1_cap = staged + staged / 4 + 4096;
        HIP_OK(hipHostMalloc((void **)&c->h_v1, c->h_v1_cap, hipHostMallocDefault));
      }
      if (dgrow(&c->d_v1, &c->d_v1_cap, staged + 64)) return -1;
      for (const V1Job &j : rj) memcpy(c->h_v1 + j.off, span + j.span_off, j.hbytes);
      HIP_OK(hipMemcpyAsync(c->d_v1, c->h_v1, staged, hipMemcpyHostToDevice, c->st));
      HIP_OK(hipMemcpyAsync(c->d_v1_jobs, rj.data(), rj.size() * sizeof(V1Job), hipMemcpyHostToDevice, c->st));
      c->stats.h2d_bytes += staged + rj.size() * sizeof(V1Job);
      HIP_OK(hipEventRecord(c->ev[kEvStart], c->st));
      launch_v1_unpack(c->d_v1, c->d_v1_jobs, rj.size(), c->d_v1_off, c->d_v1_len, c->d_v1_res, c->st);
      HIP_OK(hipGetLastError());
      HIP_OK(hipEventRecord(c->ev[kEvEnd], c->st));
      if (round == 0) {
        HIP_OK(hipMemcpyAsync(jr.data(), c->d_v1_res, jr.size() * sizeof(V1Res), hipMemcpyDeviceToHost, c->st));
        HIP_OK(hipStreamSynchronize(c->st));
      } else {
        std::vector<V1Res> r1(rj.size());
        HIP_OK(hipMemcpyAsync(r1.data(), c->d_v1_res, r1.size() * sizeof(V1Res), hipMemcpyDeviceToHost, c->st));
        HIP_OK(hipStreamSynchronize(c->st));
        for (size_t q = 0; q < sel.size(); q++) jr[sel[q]] = r1[q];
      }
      float ms = 0;
      hipEventElapsedTime(&ms, c->ev[kEvStart], c->ev[kEvEnd]);
      kms += ms;
    }
    HIP_OK(hipMemcpyAsync(h_off, c->d_v1_off, items * 8, hipMemcpyDeviceToHost, c->st));
    HIP_OK(hipMemcpyAsync(h_len, c->d_v1_len, items * 8, hipMemcpyDeviceToHost, c->st));
    HIP_OK(hipStreamSynchronize(c->st));
    c->stats.d2h_bytes += 16 * items;
    for (size_t k = 0; k < jobs.size(); k++) {  // the first packed record that failed ends the batch there
      const V1Res &x = jr[k];
      if (x.status == kV1Ok) continue;
      const V1Rec &rc = recs[job_rec[k]];
      const uint64_t at = file_off + rc.off;
      memset(&e, 0, sizeof(e));
      switch (x.status) {
      case kV1ItemSize:
        rio_set_error(&e, RIO_ERR_ITEM_SIZE, at,
                      "recordio: likely corrupt data, failed to read size of packed item %" PRIu64 ": %" PRId64,
                      (uint64_t)x.a, (int64_t)x.b);
        break;
      case kV1Crc:
        rio_set_error(&e, RIO_ERR_V1_PACKED, at,
                      "recordio: likely corrupt data, crc check failed - corrupt packed record header (%u != %u)?",
                      (uint32_t)x.a, (uint32_t)x.b);
        break;
      case kV1Offset:
        rio_set_error(&e, RIO_ERR_V1_PACKED, at,
                      "recordio: offset greater than buf size (%" PRIu64 " > %" PRIu64
                      "), likely due to a mismatched transform or a truncated file",
                      (uint64_t)x.a, (uint64_t)x.b);
        break;
      case kV1Range:  // the reference panics slicing
        rio_set_error(&e, RIO_ERR_ITEM_RANGE, at, "recordio: corrupt packed record header, item sizes out of range");
        break;
      default:
        rio_set_error(&e, RIO_ERR_HIP, at, "internal: v1 record status %u", x.status);
      }
      e.a = x.a;
      e.b = x.b;
      err = true;
      stop = RIO_STOP_ERROR;
      nrec = job_rec[k];
      nitems = rc.first;
      consumed = rc.off;
      break;
    }
  }
  for (const V1Unp &u : unp) {
    if (u.slot >= nitems) break;
    h_off[u.slot] = u.off;
    h_len[u.slot] = u.len;
  }
  unsigned long long *first = r.blk, *foff = r.blk + nrec + 1;
  for (uint64_t i = 0; i < nrec; i++) {
    first[i] = recs[i].first;
    foff[i] = file_off + recs[i].off;
  }
  first[nrec] = nitems;
  out->span = span;
  out->records = nullptr;
  out->records_len = 0;
  out->item_off = reinterpret_cast<const uint64_t *>(h_off);
  out->item_len = reinterpret_cast<const uint64_t *>(h_len);
  out->n_items = nitems;
  out->block_first_item = reinterpret_cast<const uint64_t *>(first);
  out->block_file_off = reinterpret_cast<const uint64_t *>(foff);
  out->n_blocks = nrec;
  out->consumed = consumed;
  out->stop = stop;
  out->in_bytes = nbytes;
  out->kernel_ms = kms;
  c->stats.spans++;
  c->stats.device_ms += kms;
  if (err) out->err = e;
  else if (stop == RIO_STOP_MORE && nrec == 0) out->err.a = need;  // the next record needs a span this large
  return 0;
}

extern "C" int rio_scan_v1_span(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off,
                                int32_t is_file_end, rio_batch *out) {
  return rio_scan_v1_span_mode(ctx, span, nbytes, file_off, is_file_end, nullptr, out);
}

// ------------------------------------------------------------ writer encode
// the blocks of a v2 file from items, on the GPU (encode.hip).
namespace {

const unsigned long long kMagicBody = 0x2e3c0734eb47762eull;     // MagicPacked, little-endian
const unsigned long long kMagicHdr = 0xf70416c25cd9e1d9ull;      // MagicHeader
const unsigned long long kMagicTrl = 0x3a75dfcbd71abafeull;      // MagicTrailer

template <class T>
int egrow(T **p, uint64_t *cap, uint64_t n) {
  if (*cap >= n) return 0;
  const uint64_t c = n + n / 4 + 256;
  if (dalloc(p, c)) return -1;
  *cap = c;
  return 0;
}

}  // namespace

// out == nullptr: sizing only (*out_len); out == kOwnOut: into the ctx's own
// device buffer e_out (grown to the stream), block offsets into e_boff. The
// per-block arrays, chunk map and scan scratch grow with the stream, so any
// number of blocks / chunks encodes (no ctx span capacity applies).
static uint8_t *const kOwnOut = reinterpret_cast<uint8_t *>(1);

static int encode_dev(rio_ctx *c, const rio_encode_args *a, const uint8_t *data, const unsigned long long *ends,
                      uint8_t *out, uint64_t out_cap, uint64_t *out_len, unsigned long long *boff, rio_error *err) {
  hipStream_t st = c->st;
  const uint64_t per = a->items_per_block ? a->items_per_block : 16385;  // DefaultPackedItems + 1
  const uint64_t nb = a->n_items ? (a->n_items + per - 1) / per : 0;
  *out_len = 0;
  if (nb == 0) return 0;
  if (egrow(&c->e_blk, &c->e_blk_cap, 6 * (nb + 1))) return -1;
  if (egrow(&c->e_scan, &c->e_scan_cap, (nb + 2047) / 2048 + 16)) return -1;
  EncArgs ea{};
  ea.data = data;
  ea.item_end = ends;
  ea.n_items = a->n_items;
  ea.per_block = per;
  ea.nblocks = nb;
  ea.codec = a->kind == RIO_BLOCK_HEADER ? RIO_CODEC_NONE : a->codec;  // the header block is never transformed
  ea.level = a->level;
  ea.magic = a->kind == RIO_BLOCK_HEADER ? kMagicHdr : a->kind == RIO_BLOCK_TRAILER ? kMagicTrl : kMagicBody;
  ea.hdr_len = c->e_blk;
  ea.hdr_off = c->e_blk + (nb + 1);
  ea.pay_len = c->e_blk + 2 * (nb + 1);
  ea.nck = c->e_blk + 3 * (nb + 1);
  ea.ck0 = c->e_blk + 4 * (nb + 1);
  ea.comp_off = c->e_blk + 5 * (nb + 1);
  HIP_OK(hipEventRecord(c->ev[kEvStart], st));
  launch_enc_count(ea, st);
  launch_chunk_scan(ea.hdr_len, ea.hdr_off, c->e_scan, nb, st);
  unsigned long long hdr_total = 0;
  HIP_OK(hipMemcpyAsync(&hdr_total, ea.hdr_off + nb, 8, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  if (egrow(&c->e_hdr, &c->e_hdr_cap, hdr_total + 16)) return -1;
  ea.hdr = c->e_hdr;
  launch_enc_header(ea, st);
  // the transformers in order (writerv2.go:432-441 with registry.go:75-111's
  // combined transform: stage k transforms stage k - 1's output). A stage
  // after the first reads the previous stage's compressed payloads as its
  // blocks' "headers" (hdr_len = their lengths, no item bytes), the mirror of
  // the scan's k_reframe; stages alternate between two compressed buffers.
  int nst = 1;
  int32_t stc[4] = {ea.codec, 0, 0, 0}, stl[4] = {ea.level, 0, 0, 0};
  if (ea.codec & RIO_CODEC_CHAIN_FLAG) {
    nst = (ea.codec >> 8) & 0xff;
    for (int k = 0; k < nst; k++) {
      stc[k] = (ea.codec >> (2 * k)) & 3;
      stl[k] = (int32_t)(int8_t)(uint8_t)((uint32_t)ea.level >> (8 * k));  // a signed byte per stage
    }
  }
  for (int k = 0; k < nst && stc[0] != RIO_CODEC_NONE; k++) {
    uint8_t **buf = (k & 1) ? &c->e_comp2 : &c->e_comp;
    uint64_t *cap = (k & 1) ? &c->e_comp2_cap : &c->e_comp_cap;
    if (k > 0) {  // the previous stage's payloads become this stage's input
      HIP_OK(hipMemcpyAsync(ea.hdr_len, ea.pay_len, (nb + 1) * 8, hipMemcpyDeviceToDevice, st));
      HIP_OK(hipMemcpyAsync(ea.hdr_off, ea.comp_off, (nb + 1) * 8, hipMemcpyDeviceToDevice, st));
      ea.hdr = ea.comp;
    }
    ea.codec = stc[k];
    ea.level = stl[k];
    if (ea.codec == RIO_CODEC_FLATE) {  // the payloads compressed into comp (deflate_enc.hip)
      launch_deflate_bound(ea, st);
    } else {  // one zstd frame per payload (zstd_enc.hip)
      launch_zstd_enc_bound(ea, st);
    }
    launch_chunk_scan(ea.nck, ea.comp_off, c->e_scan, nb, st);
    unsigned long long comp_total = 0;
    HIP_OK(hipMemcpyAsync(&comp_total, ea.comp_off + nb, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (egrow(buf, cap, comp_total + 64)) return -1;
    ea.comp = *buf;
    if (ea.codec == RIO_CODEC_FLATE) {
      if (ea.level != 0 && ea.level != 1 && egrow(&c->e_zscr, &c->e_zscr_cap, deflate_scratch_words(c->ncu)))
        return -1;
      launch_deflate(ea, c->e_zscr, c->ncu, st);
    } else {
      if (egrow(&c->e_zscr, &c->e_zscr_cap, zstd_enc_scratch_words(c->ncu))) return -1;
      if (!c->e_ztab) {
        ZeTabs t;
        ze_build_tabs(t);
        if (dalloc(&c->e_ztab, 1)) return -1;
        HIP_OK(hipMemcpy(c->e_ztab, &t, sizeof(t), hipMemcpyHostToDevice));
      }
      launch_zstd_enc(ea, c->e_ztab, c->e_zscr, c->ncu, st);
    }
  }
  launch_enc_nck(ea, st);
  launch_chunk_scan(ea.nck, ea.ck0, c->e_scan, nb, st);
  unsigned long long nchunks = 0;
  HIP_OK(hipMemcpyAsync(&nchunks, ea.ck0 + nb, 8, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  *out_len = nchunks * kChunk;
  if (!out) return 0;  // sizing only
  if (out == kOwnOut) {
    if (egrow(&c->e_out, &c->e_out_cap, *out_len) || egrow(&c->e_boff, &c->e_boff_cap, nb + 1)) return -1;
    out = c->e_out;
    boff = c->e_boff;
  } else if (*out_len > out_cap) {
    rio_set_error(err, RIO_ERR_CAPACITY, 0, "output too small: need %" PRIu64 " bytes", *out_len);
    return RIO_ERR_CAPACITY;
  }
  if (egrow(&c->e_ckmap, &c->e_ckmap_cap, nchunks + 1)) return -1;
  ea.ck_block = c->e_ckmap;
  ea.out = out;
  launch_enc_ckmap(ea, st);
  launch_enc_chunks(ea, nchunks, CrcTabs{c->d.crc_fold, c->d.crc_mul, c->d.crc_fix_a, c->d.crc_fix_b}, c->ncu, st);
  if (boff) launch_enc_boff(ea.ck0, boff, nb, st);
  HIP_OK(hipEventRecord(c->ev[kEvEnd], st));
  HIP_OK(hipStreamSynchronize(st));
  return 0;
}

static int encode_check(rio_ctx *ctx, const rio_encode_args *a, rio_error *err) {
  if (!ctx || !a) return -1;
  bool codec_ok = a->codec == RIO_CODEC_NONE || a->codec == RIO_CODEC_FLATE || a->codec == RIO_CODEC_ZSTD;
  if (a->codec & RIO_CODEC_CHAIN_FLAG) {  // 1-4 stages, each flate or zstd
    const int n = (a->codec >> 8) & 0xff;
    codec_ok = n >= 1 && n <= 4 && (a->codec & ~(RIO_CODEC_CHAIN_FLAG | 0xffff)) == 0;
    for (int k = 0; codec_ok && k < n; k++) {
      const int ck = (a->codec >> (2 * k)) & 3;
      codec_ok = ck == RIO_CODEC_FLATE || ck == RIO_CODEC_ZSTD;
    }
    if (codec_ok && (a->codec & 0xff) >> (2 * n)) codec_ok = false;  // codes past the n stages
  }
  if (!codec_ok) {
    rio_set_error(err, RIO_ERR_ARG, 0, "encode: codec %d not supported (none, flate, zstd, a chain of 1-4 of those)",
                  a->codec);
    return RIO_ERR_ARG;
  }
  if (a->kind < RIO_BLOCK_BODY || a->kind > RIO_BLOCK_TRAILER) {
    rio_set_error(err, RIO_ERR_ARG, 0, "encode: unknown block kind %d", a->kind);
    return RIO_ERR_ARG;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return -1;
  return 0;
}

extern "C" int rio_encode_device(rio_ctx *ctx, const rio_encode_args *a, void *out, uint64_t out_cap,
                                 uint64_t *out_len, uint64_t *block_off, rio_error *err) {
  rio_error scratch;
  if (!err) err = &scratch;
  memset(err, 0, sizeof(*err));
  if (!out_len) return -1;
  if (int rc = encode_check(ctx, a, err)) return rc;
  return encode_dev(ctx, a, (const uint8_t *)a->data, (const unsigned long long *)a->item_end, (uint8_t *)out,
                    out_cap, out_len, (unsigned long long *)block_off, err);
}

extern "C" int rio_encode(rio_ctx *ctx, const rio_encode_args *a, uint8_t *out, uint64_t out_cap, uint64_t *out_len,
                          uint64_t *block_off, rio_error *err) {
  rio_error scratch;
  if (!err) err = &scratch;
  memset(err, 0, sizeof(*err));
  if (!out_len) return -1;
  if (int rc = encode_check(ctx, a, err)) return rc;
  rio_ctx *c = ctx;
  const uint64_t n = a->n_items;
  const uint64_t bytes = n ? a->item_end[n - 1] : 0;
  if (egrow(&c->e_data, &c->e_data_cap, bytes + 64) || egrow(&c->e_ends, &c->e_ends_cap, n + 1)) return -1;
  if (bytes) HIP_OK(hipMemcpyAsync(c->e_data, a->data, bytes, hipMemcpyHostToDevice, c->st));
  if (n) HIP_OK(hipMemcpyAsync(c->e_ends, a->item_end, n * 8, hipMemcpyHostToDevice, c->st));
  const uint64_t per = a->items_per_block ? a->items_per_block : 16385;
  const uint64_t nb = n ? (n + per - 1) / per : 0;
  // one pass: encoded into the ctx's device output (sized from the chunk
  // counts), then copied back if the caller's buffer holds it
  int rc = encode_dev(c, a, c->e_data, c->e_ends, kOwnOut, 0, out_len, nullptr, err);
  if (rc) return rc;
  if (*out_len > out_cap) {
    rio_set_error(err, RIO_ERR_CAPACITY, 0, "output too small: need %" PRIu64 " bytes", *out_len);
    return RIO_ERR_CAPACITY;
  }
  if (*out_len == 0) return 0;
  HIP_OK(hipMemcpyAsync(out, c->e_out, *out_len, hipMemcpyDeviceToHost, c->st));
  if (block_off) HIP_OK(hipMemcpyAsync(block_off, c->e_boff, nb * 8, hipMemcpyDeviceToHost, c->st));
  HIP_OK(hipStreamSynchronize(c->st));
  return 0;
}
