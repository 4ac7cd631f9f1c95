// The reference's error text for a stop recorded by k_resolve. Every format is
// the reference's fmt string (file:line in rio_gpu.h's rio_err_code list).
#include <inttypes.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "pipeline.h"
#include "rio_internal.h"

using namespace rio;

extern "C" void rio_set_error(rio_error *e, int32_t code, uint64_t file_off, const char *fmt, ...) {
  e->code = code;
  e->file_off = file_off;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(e->msg, sizeof(e->msg), fmt, ap);
  va_end(ap);
}

static void fmt_magic_v(uint64_t m, char *out) {  // %v of [8]byte
  const uint8_t *b = reinterpret_cast<const uint8_t *>(&m);
  sprintf(out, "[%u %u %u %u %u %u %u %u]", b[0], b[1], b[2], b[3], b[4], b[5], b[6], b[7]);
}
static void fmt_magic_x(uint64_t m, char *out) {  // %x of [8]byte
  const uint8_t *b = reinterpret_cast<const uint8_t *>(&m);
  for (int i = 0; i < 8; i++) sprintf(out + 2 * i, "%02x", b[i]);
}

void rio::rio_fill_error(const Ctl &k, uint64_t file_off, int32_t mode, rio_error *e) {
  memset(e, 0, sizeof(*e));
  char a[64], b[64];
  if (k.err_chunk != kNone) {
    const uint64_t off = file_off + k.err_chunk * kChunk;
    const bool prev_end = (k.err_chunk == 0) || ((int64_t)k.prev_index == (int64_t)k.prev_total - 1);
    switch (k.err_code) {
    case kCkSize:  // chunk.go:334
      rio_set_error(e, RIO_ERR_CHUNK_SIZE, off, "Invalid chunk size %" PRIu64, (uint64_t)k.ck_size);
      e->a = k.ck_size;
      break;
    case 100:  // chunk.go:341-342 (arguments swapped in the reference)
      rio_set_error(e, RIO_ERR_CHUNK_CRC, off, "Chunk checksum mismatch, expect %" PRIu64 ", got %" PRIu64,
                    (uint64_t)k.ck_crc_actual, (uint64_t)k.ck_crc_stored);
      e->a = k.ck_crc_actual;
      e->b = k.ck_crc_stored;
      break;
    case kCkMagicChanged:  // chunk.go:274-275: got = block magic, expect = chunk magic
      fmt_magic_v(k.mag_prev, a);
      fmt_magic_v(k.mag_cur, b);
      rio_set_error(e, RIO_ERR_MAGIC_CHANGED, off,
                    "Magic number changed in the middle of a chunk sequence, got %s, expect %s", a, b);
      break;
    case kCkIndex: {  // chunk.go:279-280
      const uint64_t expect = prev_end ? 0 : k.prev_index + 1;
      fmt_magic_x(prev_end ? k.mag_cur : k.mag_prev, a);
      rio_set_error(e, RIO_ERR_CHUNK_INDEX, off,
                    "Chunk index mismatch, got %" PRIu64 ", expect %" PRIu64 " for magic %s", (uint64_t)k.ck_index,
                    expect, a);
      e->a = k.ck_index;
      e->b = expect;
      break;
    }
    case kCkTotal:  // chunk.go:284-285
      fmt_magic_x(k.mag_prev, a);
      rio_set_error(e, RIO_ERR_CHUNK_TOTAL, off,
                    "Chunk nchunk mismatch, got %" PRIu64 ", expect %" PRIu64 " for magic %s", (uint64_t)k.ck_total,
                    (uint64_t)k.prev_total, a);
      e->a = k.ck_total;
      e->b = k.prev_total;
      break;
    default:
      rio_set_error(e, RIO_ERR_HIP, off, "internal: unknown chunk error %" PRIu64, (uint64_t)k.err_code);
    }
    return;
  }
  if (k.err_code == 101) {  // io.ErrUnexpectedEOF, chunk.go:318-322
    rio_set_error(e, RIO_ERR_UNEXPECTED_EOF, file_off, "unexpected EOF");
    return;
  }
  if (k.stop_block == kNone) return;
  const uint64_t off = file_off + k.blk_c0 * kChunk;
  switch (k.blk_status) {
  case kBlkBadMagic:
    fmt_magic_v(k.mag_blk, a);
    if (mode == kModeHeader) {  // readSpecialBlock, scannerv2.go:266-268
      fmt_magic_v(0xf70416c25cd9e1d9ull, b);
      rio_set_error(e, RIO_ERR_HEADER, off, "Failed to read block, expect %s, got %s", b, a);
    } else if (mode == kModeTrailer) {  // Trailer, scannerv2.go:327-329
      rio_set_error(e, RIO_ERR_TRAILER, off, "Did not found the trailer, instead found magic %s", a);
    } else {  // scanNextBlock, scannerv2.go:386
      rio_set_error(e, RIO_ERR_BAD_MAGIC, off, "recordio: invalid magic number: %s", a);
    }
    break;
  case kBlkNItems:  // scannerv2.go:72
    rio_set_error(e, RIO_ERR_NITEMS, off, "recordio: failed to read number of packed items: %" PRId64,
                  (int64_t)k.blk_a);
    break;
  case kBlkItemSize:  // scannerv2.go:86
    rio_set_error(e, RIO_ERR_ITEM_SIZE, off,
                  "recordio: likely corrupt data, failed to read size of packed item %" PRIu64 ": %" PRId64,
                  (uint64_t)k.blk_a, (int64_t)k.blk_b);
    break;
  case kBlkBlockSize:  // scannerv2.go:94
    rio_set_error(e, RIO_ERR_BLOCK_SIZE, off,
                  "recordio: corrupt block header, got block size %" PRId64 ", expected %" PRId64, (int64_t)k.blk_a,
                  (int64_t)k.blk_b);
    break;
  case kBlkItemRange:  // the reference would panic slicing a wrapped cumSize
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
