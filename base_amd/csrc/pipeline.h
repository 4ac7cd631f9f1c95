// Internal host-side entry points shared by pipeline.cpp, the codec launchers and
// the scanner layer (scanner.cpp). Not part of the ABI.
#pragma once
#include <stdint.h>

#include "rio_gpu.h"

// Pinned host result buffers (pipeline.cpp); one per owner of a result.
struct rio_results;
rio_results *rio_results_new();
void rio_results_free(rio_results *r);

// decode one span already in host memory; mode: 0 body, 1 header block, 2 trailer
// block, 3 the last chunk alone (size + CRC only). Results land in *res (the
// ctx's own when null) and stay valid until the next call with the same res.
int rio_scan_span_mode(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off,
                       int32_t is_file_end, uint64_t limit_off, int32_t codec, int32_t mode, rio_results *res,
                       rio_batch *out);
// the same with the result copies left in flight: *out's counts, stop and error
// are final, its host arrays arrive by rio_scan_span_end (any later call on the
// ctx waits for them first; total_ms is not set). Body mode; a chain codec runs
// as rio_scan_span_mode.
// the H2D copy of a span rio_scan_span_begin will decode next on this ctx,
// enqueued now (a scanner's span ahead: its copy overlaps the decode of the
// span before it); the same span pointer and size to begin skip the staging
int rio_scan_span_stage(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, int32_t codec);
// the staged span's copy in complete (no-op when none is staged)
int rio_ctx_wait_staged(rio_ctx *ctx);
int rio_scan_span_begin(rio_ctx *ctx, const uint8_t *span, uint64_t nbytes, uint64_t file_off,
                        int32_t is_file_end, uint64_t limit_off, int32_t codec, rio_results *res, rio_batch *out);
int rio_scan_span_end(rio_ctx *ctx);  // 0 (also when nothing is in flight) or -1 (rio_last_error)
// a second context opened with this one's configuration on first use (a
// scanner's span ahead) and closed with it
rio_ctx *rio_ctx_sibling(rio_ctx *c);
// v1 records of one span (rio_scan_v1_span) into *res (the ctx's own when null)
int rio_scan_v1_span_mode(rio_ctx *c, const uint8_t *span, uint64_t nbytes, uint64_t file_off, int32_t is_file_end,
                          rio_results *res, rio_batch *out);
uint64_t rio_ctx_max_span(rio_ctx *c);
// spans a scanner decodes ahead (RIO_CFG_SPANS_AHEAD in rio_config.flags; default 2)
int rio_ctx_spans_ahead(rio_ctx *c);
// grow the ctx's span capacity (and the buffers sized by it) to at least
// `bytes`; 0 on success (a no-op when it is already that large)
int rio_ctx_reserve_span(rio_ctx *c, uint64_t bytes);
// the ctx's pools of pinned buffers and result sets (scanners borrow and return them)
int rio_ctx_take_buf(rio_ctx *c, uint64_t need, uint8_t **p, uint64_t *cap);
void rio_ctx_give_buf(rio_ctx *c, uint8_t *p, uint64_t cap);
rio_results *rio_ctx_take_results(rio_ctx *c);
void rio_ctx_give_results(rio_ctx *c, rio_results *r);
extern "C" void rio_set_error(rio_error *e, int32_t code, uint64_t file_off, const char *fmt, ...);

namespace rio {
struct DevBufs;
struct Ctl;
void rio_fill_error(const Ctl &k, uint64_t file_off, int32_t mode, rio_error *e);
// codec.hip
void codec_error_text(uint64_t code, uint64_t off, uint64_t file_off, rio_error *e);
}  // namespace rio
