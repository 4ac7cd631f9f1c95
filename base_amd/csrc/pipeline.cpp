// Host orchestration of the span decode pipeline and the batch-layer C ABI
// (include/rio_gpu.h). One rio_ctx = one device + one HIP stream + fixed-capacity
// device buffers; no allocation on the hot path except capacity growth.
#include <hip/hip_runtime.h>
#include <inttypes.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "pipeline.h"
#include "rio_internal.h"

namespace rio {

// launchers (kernels.hip)
void launch_chunk_meta(const uint8_t *span, uint64_t nchunks, const DevBufs &d, hipStream_t st);
void launch_chunk_scans(uint64_t nchunks, const DevBufs &d, unsigned long long *nblocks_dev, hipStream_t st);
void launch_block_parse(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st);
void launch_block_scans(const DevBufs &d, const unsigned long long *nblocks_dev, uint64_t max_blocks,
                        hipStream_t st);
void launch_scan_totals(const DevBufs &d, const unsigned long long *nblocks_dev, hipStream_t st);
void launch_items(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st);
void launch_crc_copy(const uint8_t *span, uint64_t nchunks, const DevBufs &d, const CopyArgs &ca,
                     int ncu, hipStream_t st);
void launch_resolve(const DevBufs &d, const ResolveArgs &a, hipStream_t st);
// compressed codecs (codec_flate.hip, codec_zstd.hip)
void launch_codec_prepare(const uint8_t *span, uint64_t nchunks, const DevBufs &d,
                          const unsigned long long *nblocks_dev, uint64_t max_blocks, int codec,
                          uint64_t dec_cap, hipStream_t st);
void launch_codec_decode(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks_dev,
                         uint64_t max_blocks, int codec, uint64_t dec_cap, int ncu, hipStream_t st);


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

#define HIP_OK(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      set_last_error("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      return -1;                                                                        \
    }                                                                                   \
  } while (0)

struct rio_ctx {
  int device = 0;
  int ncu = 256;
  hipStream_t st = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t ev_stage[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t ev_dec[2] = {nullptr, nullptr};
  bool last_had_dec = false;
  uint64_t max_span = 0, max_chunks = 0, max_blocks = 0;
  uint64_t rec_cap = 0, item_cap = 0, dec_cap = 0;
  DevBufs d{};
  unsigned long long *nblocks_dev = nullptr;
  uint8_t *d_span = nullptr;  // staging for host spans (lazy)
  // pinned host results (lazy, grown on demand)
  Ctl *h_ctl = nullptr;
  uint8_t *h_records = nullptr;
  uint64_t h_records_cap = 0;
  unsigned long long *h_item_end = nullptr;
  uint64_t h_item_cap = 0;
  unsigned long long *h_blk = nullptr;  // first_item (n+1) | rec_off (n) | file_off (n)
  uint64_t h_blk_cap = 0;
  std::vector<uint64_t> blk_file_off;
  // last async call
  uint64_t last_nchunks = 0, last_file_off = 0, last_in_bytes = 0;
  int32_t last_codec = 0, last_mode = 0;
  const uint8_t *last_span = nullptr;
};

const char *rio_last_error(void) { return g_last_error.c_str(); }
int rio_abi_version(void) { return RIO_ABI_VERSION; }
void *rio_stream(rio_ctx *ctx) { return ctx ? (void *)ctx->st : nullptr; }

template <class T>
static int dalloc(T **p, uint64_t n) {
  if (*p) hipFree(*p);
  *p = nullptr;
  if (n == 0) n = 1;
  HIP_OK(hipMalloc((void **)p, n * sizeof(T)));
  return 0;
}

static int alloc_chunk_bufs(rio_ctx *c) {
  DevBufs &d = c->d;
  const uint64_t n = c->max_chunks + 1;
  if (dalloc(&d.ck_size, n) || dalloc(&d.ck_total, n) || dalloc(&d.ck_index, n) || dalloc(&d.ck_info, n) ||
      dalloc(&d.ck_crc, n) || dalloc(&d.ck_block, n) || dalloc(&d.ck_pay, n + 1))
    return -1;
  const uint64_t nb = c->max_blocks + 1;
  if (dalloc(&d.blk_c0, nb) || dalloc(&d.blk_nitems, nb) || dalloc(&d.blk_hdr, nb) || dalloc(&d.blk_recb, nb) ||
      dalloc(&d.blk_item_base, nb + 1) || dalloc(&d.blk_rec_base, nb + 1) || dalloc(&d.blk_status, nb) ||
      dalloc(&d.blk_a, nb) || dalloc(&d.blk_b, nb) || dalloc(&d.blk_out_len, nb) || dalloc(&d.blk_dec_off, nb + 1))
    return -1;
  if (dalloc(&d.scan_tmp, (n + 2047) / 2048 + 16)) return -1;
  return 0;
}

static void free_all(rio_ctx *c) {
  DevBufs &d = c->d;
  void *ps[] = {d.ck_size, d.ck_total, d.ck_index, d.ck_info, d.ck_crc, d.ck_block, d.ck_pay,
                d.blk_c0, d.blk_nitems, d.blk_hdr, d.blk_recb, d.blk_item_base, d.blk_rec_base,
                d.blk_status, d.blk_a, d.blk_b, d.blk_out_len, d.blk_dec_off, d.records, d.item_end,
                d.scan_tmp, d.dec, d.ctl, d.crc_fold, d.crc_tree, d.crc_fix_a, d.crc_fix_b,
                c->nblocks_dev, c->d_span};
  for (void *p : ps)
    if (p) hipFree(p);
  if (c->h_ctl) hipHostFree(c->h_ctl);
  if (c->h_records) hipHostFree(c->h_records);
  if (c->h_item_end) hipHostFree(c->h_item_end);
  if (c->h_blk) hipHostFree(c->h_blk);
  if (c->ev0) hipEventDestroy(c->ev0);
  if (c->ev1) hipEventDestroy(c->ev1);
  for (hipEvent_t e : c->ev_stage)
    if (e) hipEventDestroy(e);
  for (hipEvent_t e : c->ev_dec)
    if (e) hipEventDestroy(e);
  if (c->st) hipStreamDestroy(c->st);
}

static int ctx_init(rio_ctx *c, const rio_config *cfg) {
  c->device = cfg ? cfg->device : 0;
  HIP_OK(hipSetDevice(c->device));
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, c->device));
  c->ncu = prop.multiProcessorCount;
  uint64_t span = (cfg && cfg->max_span_bytes) ? cfg->max_span_bytes : (256ull << 20);
  span = (span + kChunk - 1) / kChunk * kChunk;
  c->max_span = span;
  c->max_chunks = span / kChunk;
  c->max_blocks = c->max_chunks;
  c->rec_cap = (cfg && cfg->max_out_bytes) ? cfg->max_out_bytes : span;
  c->item_cap = (cfg && cfg->max_items) ? cfg->max_items : span / 64 + 1024;
  c->dec_cap = 0;
  HIP_OK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
  HIP_OK(hipEventCreate(&c->ev0));
  HIP_OK(hipEventCreate(&c->ev1));
  for (hipEvent_t &e : c->ev_stage) HIP_OK(hipEventCreate(&e));
  for (hipEvent_t &e : c->ev_dec) HIP_OK(hipEventCreate(&e));
  if (alloc_chunk_bufs(c)) return -1;
  DevBufs &d = c->d;
  if (dalloc(&d.records, c->rec_cap) || dalloc(&d.item_end, c->item_cap) || dalloc(&d.ctl, 1) ||
      dalloc(&c->nblocks_dev, 2))
    return -1;
  // CRC tables
  std::vector<uint32_t> fold(16 * 256), tree(6 * 4 * 256), fa(kMaxPayload + 1), fb(kMaxPayload + 1);
  build_crc_tables(fold.data(), tree.data(), fa.data(), fb.data());
  if (dalloc(&d.crc_fold, fold.size()) || dalloc(&d.crc_tree, tree.size()) ||
      dalloc(&d.crc_fix_a, fa.size()) || dalloc(&d.crc_fix_b, fb.size()))
    return -1;
  HIP_OK(hipMemcpy(d.crc_fold, fold.data(), fold.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d.crc_tree, tree.data(), tree.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d.crc_fix_a, fa.data(), fa.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d.crc_fix_b, fb.data(), fb.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipHostMalloc((void **)&c->h_ctl, sizeof(Ctl), hipHostMallocDefault));
  return 0;
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

void rio_close(rio_ctx *ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->st);
  free_all(ctx);
  delete ctx;
}

// ------------------------------------------------------------------ launches
static int ensure_dec(rio_ctx *c, uint64_t need) {
  if (c->dec_cap >= need) return 0;
  uint64_t cap = need + need / 4;
  if (dalloc(&c->d.dec, cap)) return -1;
  c->dec_cap = cap;
  return 0;
}

// Enqueue the full pipeline for `nchunks` whole chunks at dev span `span`.
static int enqueue(rio_ctx *c, const uint8_t *span, uint64_t nchunks, uint64_t limit_chunk, int is_file_end,
                   int tail_partial, int32_t codec, int32_t mode) {
  DevBufs &d = c->d;
  hipStream_t st = c->st;
  // reset control words (events are min-reduced)
  HIP_OK(hipMemsetAsync(d.ctl, 0xff, 5 * sizeof(unsigned long long), st));
  HIP_OK(hipMemsetAsync(&d.ctl->out_overflow, 0, sizeof(unsigned long long), st));
  HIP_OK(hipMemsetAsync(c->nblocks_dev, 0, 2 * sizeof(unsigned long long), st));
  if (nchunks > 0) {
    launch_chunk_meta(span, nchunks, d, st);
    launch_chunk_scans(nchunks, d, c->nblocks_dev, st);
  }
  const uint64_t max_blocks = nchunks ? nchunks : 1;
  HIP_OK(hipEventRecord(c->ev_stage[0], st));
  if (codec != RIO_CODEC_NONE && nchunks > 0) {
    // decompressed capacity: prepare sizes each block's region, then decode
    if (ensure_dec(c, c->dec_cap ? c->dec_cap : 4 * (nchunks * (uint64_t)kChunk) + (1 << 20))) return -1;
    launch_codec_prepare(span, nchunks, d, c->nblocks_dev, max_blocks, codec, c->dec_cap, st);
    HIP_OK(hipEventRecord(c->ev_dec[0], st));
    launch_codec_decode(span, d, c->nblocks_dev, max_blocks, codec, c->dec_cap, c->ncu, st);
    HIP_OK(hipEventRecord(c->ev_dec[1], st));
    c->last_had_dec = true;
  } else {
    c->last_had_dec = false;
  }
  ParseArgs pa{span, nchunks, limit_chunk, mode, codec, c->nblocks_dev, c->item_cap, c->rec_cap};
  if (nchunks > 0) {
    launch_block_parse(d, pa, max_blocks, st);
    launch_block_scans(d, c->nblocks_dev, max_blocks, st);
  }
  launch_scan_totals(d, c->nblocks_dev, st);
  if (nchunks > 0) {
    launch_items(d, pa, max_blocks, st);
    if (codec != RIO_CODEC_NONE) launch_codec_gather(d, c->nblocks_dev, max_blocks, c->rec_cap, (void *)st);
  }
  HIP_OK(hipEventRecord(c->ev_stage[1], st));
  if (nchunks > 0) {
    CopyArgs ca{d.records, c->rec_cap, mode, codec == RIO_CODEC_NONE ? 1 : 0};
    launch_crc_copy(span, nchunks, d, ca, c->ncu, st);
  }
  HIP_OK(hipEventRecord(c->ev_stage[2], st));
  ResolveArgs ra{span, nchunks, is_file_end, tail_partial, mode, 0, c->nblocks_dev, limit_chunk};
  launch_resolve(d, ra, st);
  HIP_OK(hipEventRecord(c->ev_stage[3], st));
  return 0;
}

// ------------------------------------------------------------------ messages
static void fmt_magic_v(uint64_t m, char *out) {
  const uint8_t *b = reinterpret_cast<const uint8_t *>(&m);
  sprintf(out, "[%u %u %u %u %u %u %u %u]", b[0], b[1], b[2], b[3], b[4], b[5], b[6], b[7]);
}
static void fmt_magic_x(uint64_t m, char *out) {
  const uint8_t *b = reinterpret_cast<const uint8_t *>(&m);
  for (int i = 0; i < 8; i++) sprintf(out + 2 * i, "%02x", b[i]);
}

void rio_set_error(rio_error *e, int32_t code, uint64_t file_off, const char *fmt, ...) {
  e->code = code;
  e->file_off = file_off;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(e->msg, sizeof(e->msg), fmt, ap);
  va_end(ap);
}

// Build the reference error text for the stop recorded in h_ctl.
static void fill_error(const Ctl &k, uint64_t file_off, int32_t mode, rio_error *e) {
  memset(e, 0, sizeof(*e));
  char a[64], b[64];
  if (k.err_chunk != kNone) {
    const uint64_t off = file_off + k.err_chunk * kChunk;
    const bool prev_end = (k.err_chunk == 0) || ((int64_t)k.prev_index == (int64_t)k.prev_total - 1);
    switch (k.err_code) {
    case kCkSize:
      rio_set_error(e, RIO_ERR_CHUNK_SIZE, off, "Invalid chunk size %" PRIu64, (uint64_t)k.ck_size);
      e->a = k.ck_size;
      break;
    case 100:
      rio_set_error(e, RIO_ERR_CHUNK_CRC, off, "Chunk checksum mismatch, expect %" PRIu64 ", got %" PRIu64,
                    (uint64_t)k.ck_crc_actual, (uint64_t)k.ck_crc_stored);
      e->a = k.ck_crc_actual;
      e->b = k.ck_crc_stored;
      break;
    case kCkMagicChanged:
      fmt_magic_v(k.mag_prev, a);
      fmt_magic_v(k.mag_cur, b);
      rio_set_error(e, RIO_ERR_MAGIC_CHANGED, off,
                    "Magic number changed in the middle of a chunk sequence, got %s, expect %s", a, b);
      break;
    case kCkIndex: {
      const uint64_t expect = prev_end ? 0 : k.prev_index + 1;
      fmt_magic_x(prev_end ? k.mag_cur : k.mag_prev, a);
      rio_set_error(e, RIO_ERR_CHUNK_INDEX, off, "Chunk index mismatch, got %" PRIu64 ", expect %" PRIu64
                    " for magic %s", (uint64_t)k.ck_index, expect, a);
      e->a = k.ck_index;
      e->b = expect;
      break;
    }
    case kCkTotal:
      fmt_magic_x(k.mag_prev, a);
      rio_set_error(e, RIO_ERR_CHUNK_TOTAL, off, "Chunk nchunk mismatch, got %" PRIu64 ", expect %" PRIu64
                    " for magic %s", (uint64_t)k.ck_total, (uint64_t)k.prev_total, a);
      e->a = k.ck_total;
      e->b = k.prev_total;
      break;
    default:
      rio_set_error(e, RIO_ERR_HIP, off, "internal: unknown chunk error %" PRIu64, (uint64_t)k.err_code);
    }
    return;
  }
  if (k.err_code == 101) {
    rio_set_error(e, RIO_ERR_UNEXPECTED_EOF, file_off, "unexpected EOF");
    return;
  }
  if (k.stop_block != kNone) {
    const uint64_t off = file_off + k.blk_c0 * kChunk;
    switch (k.blk_status) {
    case kBlkBadMagic:
      fmt_magic_v(k.mag_blk, a);
      if (mode == kModeHeader) {
        fmt_magic_v(0xf70416c25cd9e1d9ull, b);
        rio_set_error(e, RIO_ERR_HEADER, off, "Failed to read block, expect %s, got %s", b, a);
      } else if (mode == kModeTrailer) {
        rio_set_error(e, RIO_ERR_TRAILER, off, "Missing magic trailer; found %s", a);
      } else {
        rio_set_error(e, RIO_ERR_BAD_MAGIC, off, "recordio: invalid magic number: %s", a);
      }
      break;
    case kBlkNItems:
      rio_set_error(e, RIO_ERR_NITEMS, off, "recordio: failed to read number of packed items: %" PRId64,
                    (int64_t)k.blk_a);
      break;
    case kBlkItemSize:
      rio_set_error(e, RIO_ERR_ITEM_SIZE, off,
                    "recordio: likely corrupt data, failed to read size of packed item %" PRIu64 ": %" PRId64,
                    (uint64_t)k.blk_a, (int64_t)k.blk_b);
      break;
    case kBlkBlockSize:
      rio_set_error(e, RIO_ERR_BLOCK_SIZE, off,
                    "recordio: corrupt block header, got block size %" PRId64 ", expected %" PRId64,
                    (int64_t)k.blk_a, (int64_t)k.blk_b);
      break;
    case kBlkItemRange:
      rio_set_error(e, RIO_ERR_ITEM_RANGE, off, "recordio: corrupt block header, item sizes out of range");
      break;
    case kBlkCodec:
      codec_error_text(k.blk_a, k.blk_b, off, e);
      break;
    default:
      rio_set_error(e, RIO_ERR_HIP, off, "internal: unknown block status %" PRIu64, (uint64_t)k.blk_status);
    }
    e->a = k.blk_a;
    e->b = k.blk_b;
  }
}

static int collect(rio_ctx *c, uint64_t file_off, uint64_t nchunks, int32_t mode, uint64_t in_bytes,
                   rio_batch *out, bool to_host) {
  const Ctl &k = *c->h_ctl;
  memset(out, 0, sizeof(*out));
  out->in_bytes = in_bytes;
  out->n_blocks = k.n_valid_blocks;
  out->n_items = k.n_items;
  out->records_len = k.rec_bytes;
  out->consumed = k.consumed_chunks * kChunk;
  out->stop = (int32_t)k.stop_kind;
  if (k.stop_kind == 2) fill_error(k, file_off, mode, &out->err);
  const uint64_t nb = k.n_valid_blocks;
  if (!to_host) {
    out->records = c->d.records;
    out->item_end = reinterpret_cast<const uint64_t *>(c->d.item_end);
    out->block_first_item = reinterpret_cast<const uint64_t *>(c->d.blk_item_base);
    out->block_rec_off = reinterpret_cast<const uint64_t *>(c->d.blk_rec_base);
    out->block_file_off = nullptr;
    return 0;
  }
  // host copies of the valid prefix
  if (c->h_records_cap < k.rec_bytes + 16) {
    if (c->h_records) hipHostFree(c->h_records);
    c->h_records_cap = k.rec_bytes + k.rec_bytes / 4 + 4096;
    HIP_OK(hipHostMalloc((void **)&c->h_records, c->h_records_cap, hipHostMallocDefault));
  }
  if (c->h_item_cap < k.n_items + 1) {
    if (c->h_item_end) hipHostFree(c->h_item_end);
    c->h_item_cap = k.n_items + k.n_items / 4 + 1024;
    HIP_OK(hipHostMalloc((void **)&c->h_item_end, c->h_item_cap * 8, hipHostMallocDefault));
  }
  if (c->h_blk_cap < 3 * (nb + 1)) {
    if (c->h_blk) hipHostFree(c->h_blk);
    c->h_blk_cap = 3 * (nb + 1) + 3072;
    HIP_OK(hipHostMalloc((void **)&c->h_blk, c->h_blk_cap * 8, hipHostMallocDefault));
  }
  unsigned long long *first = c->h_blk, *recoff = c->h_blk + nb + 1, *foff = c->h_blk + 2 * nb + 1;
  if (k.rec_bytes)
    HIP_OK(hipMemcpyAsync(c->h_records, c->d.records, k.rec_bytes, hipMemcpyDeviceToHost, c->st));
  if (k.n_items)
    HIP_OK(hipMemcpyAsync(c->h_item_end, c->d.item_end, k.n_items * 8, hipMemcpyDeviceToHost, c->st));
  HIP_OK(hipMemcpyAsync(first, c->d.blk_item_base, (nb + 1) * 8, hipMemcpyDeviceToHost, c->st));
  if (nb) {
    HIP_OK(hipMemcpyAsync(recoff, c->d.blk_rec_base, nb * 8, hipMemcpyDeviceToHost, c->st));
    HIP_OK(hipMemcpyAsync(foff, c->d.blk_c0, nb * 8, hipMemcpyDeviceToHost, c->st));
  }
  HIP_OK(hipStreamSynchronize(c->st));
  for (uint64_t b = 0; b < nb; b++) foff[b] = file_off + foff[b] * kChunk;
  out->records = c->h_records;
  out->item_end = reinterpret_cast<const uint64_t *>(c->h_item_end);
  out->block_first_item = reinterpret_cast<const uint64_t *>(first);
  out->block_rec_off = reinterpret_cast<const uint64_t *>(recoff);
  out->block_file_off = reinterpret_cast<const uint64_t *>(foff);
  (void)nchunks;
  return 0;
}

static int grow_for_overflow(rio_ctx *c) {
  // read the totals over all blocks and grow records/items to fit
  unsigned long long nb = 0;
  HIP_OK(hipMemcpy(&nb, c->nblocks_dev, 8, hipMemcpyDeviceToHost));
  unsigned long long items = 0, recs = 0;
  HIP_OK(hipMemcpy(&items, c->d.blk_item_base + nb, 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&recs, c->d.blk_rec_base + nb, 8, hipMemcpyDeviceToHost));
  if (items > c->item_cap) {
    c->item_cap = items + items / 8 + 1024;
    if (dalloc(&c->d.item_end, c->item_cap)) return -1;
  }
  if (recs > c->rec_cap) {
    c->rec_cap = recs + recs / 8 + 4096;
    if (dalloc(&c->d.records, c->rec_cap)) return -1;
  }
  return 0;
}

int rio_run_span(rio_ctx *c, const uint8_t *dspan, uint64_t nbytes, uint64_t file_off, int32_t is_file_end,
                 uint64_t limit_off, int32_t codec, int32_t mode, bool to_host, rio_batch *out) {
  HIP_OK(hipSetDevice(c->device));
  const uint64_t nchunks = nbytes / kChunk;
  const int tail_partial = (nbytes % kChunk) != 0;
  if (nchunks > c->max_chunks) {
    rio_set_error(&out->err, RIO_ERR_CAPACITY, file_off, "span of %" PRIu64 " bytes exceeds ctx capacity",
                  nbytes);
    out->stop = RIO_STOP_ERROR;
    return 0;
  }
  uint64_t limit_chunk = UINT64_MAX;
  if (limit_off != UINT64_MAX) {
    limit_chunk = limit_off <= file_off ? 0 : (limit_off - file_off + kChunk - 1) / kChunk;
  }
  for (int attempt = 0; attempt < 3; attempt++) {
    HIP_OK(hipEventRecord(c->ev0, c->st));
    if (enqueue(c, dspan, nchunks, limit_chunk, is_file_end, tail_partial, codec, mode)) return -1;
    HIP_OK(hipEventRecord(c->ev1, c->st));
    HIP_OK(hipMemcpyAsync(c->h_ctl, c->d.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->st));
    HIP_OK(hipStreamSynchronize(c->st));
    if (c->h_ctl->out_overflow == 0) break;
    if (grow_for_overflow(c)) return -1;
    if (codec != RIO_CODEC_NONE && (c->h_ctl->out_overflow & 4)) {
      if (ensure_dec(c, c->dec_cap * 2)) return -1;
    }
  }
  float ms = 0;
  hipEventElapsedTime(&ms, c->ev0, c->ev1);
  if (collect(c, file_off, nchunks, mode, nbytes, out, to_host)) return -1;
  out->kernel_ms = ms;
  return 0;
}

extern "C" int rio_scan_device(rio_ctx *ctx, const void *dev_span, uint64_t nbytes, uint64_t file_off,
                               int32_t is_file_end, uint64_t limit_off, int32_t codec, rio_batch *out) {
  if (!ctx || !out) return -1;
  memset(out, 0, sizeof(*out));
  return rio_run_span(ctx, (const uint8_t *)dev_span, nbytes, file_off, is_file_end, limit_off, codec, kModeBody,
                      false, out);
}

int rio_stage_span(rio_ctx *c, const uint8_t *span, uint64_t nbytes) {
  if (!c->d_span) HIP_OK(hipMalloc((void **)&c->d_span, c->max_span + kChunk));
  HIP_OK(hipMemcpyAsync(c->d_span, span, nbytes, hipMemcpyHostToDevice, c->st));
  return 0;
}

uint8_t *rio_staging(rio_ctx *c) { return c->d_span; }

extern "C" int rio_scan_span(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off,
                             int32_t is_file_end, uint64_t limit_off, int32_t codec, rio_batch *out) {
  if (!ctx || !out) return -1;
  memset(out, 0, sizeof(*out));
  if (nbytes > ctx->max_span + kChunk) {
    rio_set_error(&out->err, RIO_ERR_CAPACITY, file_off, "span of %" PRIu64 " bytes exceeds ctx capacity",
                  nbytes);
    out->stop = RIO_STOP_ERROR;
    return 0;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return -1;
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  hipEventRecord(t0, ctx->st);
  if (rio_stage_span(ctx, span, nbytes)) return -1;
  int rc = rio_run_span(ctx, ctx->d_span, nbytes, file_off, is_file_end, limit_off, codec, kModeBody, true, out);
  hipEventRecord(t1, ctx->st);
  hipEventSynchronize(t1);
  float ms = 0;
  hipEventElapsedTime(&ms, t0, t1);
  out->total_ms = ms;
  hipEventDestroy(t0);
  hipEventDestroy(t1);
  return rc;
}

int rio_scan_span_mode(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off, int32_t is_file_end,
                       uint64_t limit_off, int32_t codec, int32_t mode, rio_batch *out) {
  memset(out, 0, sizeof(*out));
  if (nbytes > ctx->max_span + kChunk) {
    rio_set_error(&out->err, RIO_ERR_CAPACITY, file_off, "span exceeds ctx capacity");
    out->stop = RIO_STOP_ERROR;
    return 0;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return -1;
  if (rio_stage_span(ctx, span, nbytes)) return -1;
  return rio_run_span(ctx, ctx->d_span, nbytes, file_off, is_file_end, limit_off, codec, mode, true, out);
}

uint64_t rio_ctx_max_span(rio_ctx *c) { return c->max_span; }

extern "C" int rio_scan_device_async(rio_ctx *ctx, const void *dev_span, uint64_t nbytes, uint64_t file_off,
                                     int32_t codec) {
  if (!ctx) return -1;
  HIP_OK(hipSetDevice(ctx->device));
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
  HIP_OK(hipEventRecord(ctx->ev0, ctx->st));
  if (enqueue(ctx, (const uint8_t *)dev_span, nchunks, UINT64_MAX, 1, (nbytes % kChunk) != 0, codec, kModeBody))
    return -1;
  HIP_OK(hipEventRecord(ctx->ev1, ctx->st));
  return 0;
}

extern "C" int rio_sync(rio_ctx *ctx, rio_batch *out) {
  if (!ctx || !out) return -1;
  HIP_OK(hipSetDevice(ctx->device));
  HIP_OK(hipMemcpyAsync(ctx->h_ctl, ctx->d.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, ctx->st));
  HIP_OK(hipStreamSynchronize(ctx->st));
  float ms = 0;
  hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
  if (collect(ctx, ctx->last_file_off, ctx->last_nchunks, ctx->last_mode, ctx->last_in_bytes, out, false))
    return -1;
  out->kernel_ms = ms;
  if (ctx->h_ctl->out_overflow) {
    rio_set_error(&out->err, RIO_ERR_CAPACITY, 0, "output capacity exceeded");
    out->stop = RIO_STOP_ERROR;
  }
  return 0;
}

extern "C" int rio_stage_times(rio_ctx *ctx, float *ms, int n) {
  if (!ctx || !ms || n <= 0) return 0;
  float t[4] = {0, 0, 0, 0};
  float pre = 0, dec = 0;
  hipEventElapsedTime(&pre, ctx->ev_stage[0], ctx->ev_stage[1]);
  if (ctx->last_had_dec) hipEventElapsedTime(&dec, ctx->ev_dec[0], ctx->ev_dec[1]);
  t[0] = pre - dec;
  t[1] = dec;
  hipEventElapsedTime(&t[2], ctx->ev_stage[1], ctx->ev_stage[2]);
  hipEventElapsedTime(&t[3], ctx->ev_stage[2], ctx->ev_stage[3]);
  const int k = n < 4 ? n : 4;
  for (int i = 0; i < k; i++) ms[i] = t[i];
  return k;
}

// TransformFunc analogue (recordio.go:12). The payload views are staged to the
// device as one contiguous block and run through the codec's block decoder.
extern "C" int rio_decode_block(rio_ctx *ctx, const uint8_t *const *payloads, const uint32_t *lens, int n,
                                int32_t codec, uint8_t *scratch, uint64_t cap, uint64_t *out_len, rio_error *err) {
  if (!ctx || (n > 0 && (!payloads || !lens)) || !out_len) return -1;
  uint64_t total = 0;
  for (int i = 0; i < n; i++) total += lens[i];
  if (codec == RIO_CODEC_NONE) {  // idTransform: concatenation
    *out_len = total;
    if (total > cap) {
      if (err) rio_set_error(err, RIO_ERR_CAPACITY, 0, "scratch too small: need %" PRIu64, total);
      return RIO_ERR_CAPACITY;
    }
    uint64_t o = 0;
    for (int i = 0; i < n; i++) {
      memcpy(scratch + o, payloads[i], lens[i]);
      o += lens[i];
    }
    return 0;
  }
  return rio_decode_block_codec(ctx, payloads, lens, n, codec, scratch, cap, out_len, err);
}
