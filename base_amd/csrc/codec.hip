// Compressed-codec stages (flate / zstd) of the span pipeline: sizing of the
// per-block decompression regions, the decoders, and the gather of decoded
// records. Decoders live in codec_flate.hip / codec_zstd.hip.
#include <hip/hip_runtime.h>
#include <inttypes.h>
#include <stdio.h>

#include "pipeline.h"
#include "rio_internal.h"

namespace rio {

enum CodecErr : uint32_t {
  kCodecCorrupt = 1,      // flate: CorruptInputError(offset)
  kCodecEof = 2,          // flate: io.ErrUnexpectedEOF
  kCodecFull = 3,         // region too small (internal: retried with a larger bound)
  kCodecZstd = 4,         // zstd: error, b = ZSTD error enum
  kCodecZstdEmpty = 5,    // zstd: empty source
  kCodecUnsupported = 6,
};

// per block: decompressed-capacity bound (flate: comp * factor; zstd: frame size)
__global__ void k_codec_prepare(DevBufs d, const unsigned long long *nblocks_dev, uint64_t nchunks, int codec) {
  const uint64_t nb = *nblocks_dev;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c0 = d.blk_c0[b];
    const uint64_t total = d.ck_total[c0];
    uint64_t comp = 0;
    if (total != 0 && c0 + total <= nchunks) comp = d.ck_pay[c0 + total] - d.ck_pay[c0];
    d.blk_out_len[b] = (comp * 8 + 4096 + 255) & ~255ull;  // bound, refined by the decoder
    d.blk_status[b] = kBlkOk;
    d.blk_a[b] = 0;
    d.blk_b[b] = 0;
  }
}

__global__ void k_codec_stub(DevBufs d, const unsigned long long *nblocks_dev) {
  const uint64_t nb = *nblocks_dev;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    d.blk_status[b] = kBlkCodec;
    d.blk_a[b] = kCodecUnsupported;
    d.blk_out_len[b] = 0;
  }
}

void launch_codec_prepare(const uint8_t *span, uint64_t nchunks, const DevBufs &d,
                          const unsigned long long *nblocks_dev, uint64_t max_blocks, int codec, uint64_t dec_cap,
                          hipStream_t st) {
  (void)span;
  (void)dec_cap;
  unsigned g = (unsigned)((max_blocks + 255) / 256);
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(k_codec_prepare, dim3(g ? g : 1), dim3(256), 0, st, d, nblocks_dev, nchunks, codec);
}

void launch_codec_decode(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks_dev,
                         uint64_t max_blocks, int codec, uint64_t dec_cap, int ncu, hipStream_t st) {
  (void)span;
  (void)codec;
  (void)dec_cap;
  (void)ncu;
  unsigned g = (unsigned)((max_blocks + 255) / 256);
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(k_codec_stub, dim3(g ? g : 1), dim3(256), 0, st, d, nblocks_dev);
}

void codec_error_text(uint64_t code, uint64_t off, uint64_t file_off, rio_error *e) {
  switch (code) {
  case kCodecCorrupt:
    rio_set_error(e, RIO_ERR_FLATE_CORRUPT, file_off, "flate: corrupt input before offset %" PRIu64, off);
    break;
  case kCodecEof:
    rio_set_error(e, RIO_ERR_FLATE_EOF, file_off, "unexpected EOF");
    break;
  case kCodecZstdEmpty:
    rio_set_error(e, RIO_ERR_ZSTD_EMPTY, file_off, "Bytes slice is empty");
    break;
  case kCodecZstd:
    rio_set_error(e, RIO_ERR_ZSTD, file_off, "zstd: error %" PRIu64, off);
    break;
  default:
    rio_set_error(e, RIO_ERR_ARG, file_off, "codec not supported by this build");
  }
}

}  // namespace rio

int rio_decode_block_codec(rio_ctx *ctx, const uint8_t *const *payloads, const uint32_t *lens, int n,
                           int32_t codec, uint8_t *scratch, uint64_t cap, uint64_t *out_len, rio_error *err) {
  (void)ctx;
  (void)payloads;
  (void)lens;
  (void)n;
  (void)codec;
  (void)scratch;
  (void)cap;
  *out_len = 0;
  if (err) rio_set_error(err, RIO_ERR_ARG, 0, "codec not supported by this build");
  return RIO_ERR_ARG;
}
