// Internal host-side entry points shared by pipeline.cpp, the codec launchers and
// the scanner layer (scanner.cpp). Not part of the ABI.
#pragma once
#include <stdint.h>

#include "rio_gpu.h"

// decode one span already in host memory; mode: 0 body, 1 header block, 2 trailer
// block, 3 the last chunk alone (size + CRC only)
int rio_scan_span_mode(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off,
                       int32_t is_file_end, uint64_t limit_off, int32_t codec, int32_t mode, rio_batch *out);
uint64_t rio_ctx_max_span(rio_ctx *c);
extern "C" void rio_set_error(rio_error *e, int32_t code, uint64_t file_off, const char *fmt, ...);
int rio_decode_block_codec(rio_ctx *ctx, const uint8_t *const *payloads, const uint32_t *lens, int n,
                           int32_t codec, uint8_t *scratch, uint64_t cap, uint64_t *out_len, rio_error *err);

namespace rio {
struct DevBufs;
struct Ctl;
void rio_fill_error(const Ctl &k, uint64_t file_off, int32_t mode, rio_error *e);
// codec.hip
void codec_error_text(uint64_t code, uint64_t off, uint64_t file_off, rio_error *e);
}  // namespace rio
