// Compressed-codec stages (flate / zstd) of the span pipeline: sizing of the
// per-block decode regions and decoder dispatch (codec_flate.hip,
// codec_zstd.hip). Decoded blocks stay where they were decoded; items are
// views into them.
#include <hip/hip_runtime.h>
#include <inttypes.h>
#include <stdio.h>

#include "pipeline.h"
#include "rio_internal.h"

namespace rio {

// per block: the decode region's size bound (flate: compressed bytes x factor;
// the exact size is known only after decoding); resets the codec status
__global__ void k_codec_prepare(DevBufs d, const unsigned long long *nblocks_dev, uint32_t factor) {
  const uint64_t nb = *nblocks_dev;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long comp = (d.blk_meta[b] & kMetaComplete) ? d.blk_len[b] : 0;
    unsigned long long bound = comp * factor + 4096;
    if (d.blk_need[b] > bound) bound = d.blk_need[b];  // exact size from a previous attempt
    d.blk_out_len[b] = (bound + 255) & ~255ull;
    d.blk_status[b] = kBlkOk;
    d.blk_a[b] = 0;
    d.blk_b[b] = 0;
  }
}

__global__ void k_codec_unsupported(DevBufs d, const unsigned long long *nblocks_dev) {
  const uint64_t nb = *nblocks_dev;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    d.blk_status[b] = kBlkCodec;
    d.blk_a[b] = kCodecUnsupported;
    d.blk_out_len[b] = 0;
  }
}

void launch_block_scan(const unsigned long long *in, unsigned long long *out, unsigned long long *tmp,
                       const unsigned long long *nblocks_dev, uint64_t max_blocks, hipStream_t st);
void launch_inflate(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks,
                    uint64_t nchunks, uint64_t dec_cap, int rounds, int ncu, hipStream_t st);
void launch_zstd(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks,
                 uint64_t dec_cap, uint64_t grid, hipStream_t st);

static unsigned grid_blocks(uint64_t n) {
  uint64_t g = (n + 255) / 256;
  if (g > 1024) g = 1024;
  return (unsigned)(g ? g : 1);
}

// decode-region bounds and their offsets (exclusive scan into blk_dec_off)
void launch_codec_prepare(const DevBufs &d, const unsigned long long *nblocks_dev, uint64_t max_blocks,
                          uint32_t factor, hipStream_t st) {
  hipLaunchKernelGGL(k_codec_prepare, dim3(grid_blocks(max_blocks)), dim3(256), 0, st, d, nblocks_dev, factor);
  launch_block_scan(d.blk_out_len, d.blk_dec_off, d.scan_tmp, nblocks_dev, max_blocks, st);
}

void launch_codec_decode(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks_dev,
                         uint64_t max_blocks, uint64_t nchunks, int codec, uint64_t dec_cap, int rounds, int ncu,
                         hipStream_t st) {
  if (codec == RIO_CODEC_FLATE) {
    launch_inflate(span, d, nblocks_dev, max_blocks, nchunks, dec_cap, rounds, ncu, st);
    return;
  }
  if (codec == RIO_CODEC_ZSTD && d.zlit) {
    launch_zstd(span, d, nblocks_dev, max_blocks, dec_cap, d.zlit_waves, st);
    return;
  }
  hipLaunchKernelGGL(k_codec_unsupported, dim3(grid_blocks(max_blocks)), dim3(256), 0, st, d, nblocks_dev);
}

// ---------------------------------------------------------------- host results
// The valid blocks' decoded bytes gathered back to back (16-aligned) and their
// item views rebased, so that a host result (rio_scan_span) copies only record
// bytes back over PCIe, not the decode regions with their slack.
__global__ void k_compact_len(DevBufs d, const unsigned long long *nblocks_dev, unsigned long long *padded) {
  const uint64_t nb = *nblocks_dev, nv = d.ctl->n_valid_blocks;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x)
    padded[b] = b < nv ? (d.blk_out_len[b] + 15) & ~15ull : 0ull;
}

// A wave per (block, part): a span of few large blocks (MaxItems = 16384:
// ~250 blocks of 5 MB per 512 MiB span) spreads each block's copy over up to
// 64 waves instead of one.
__global__ void __launch_bounds__(256) k_compact(DevBufs d, const unsigned long long *nblocks_dev) {
  const uint64_t nv = d.ctl->n_valid_blocks;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = __lane_id();
  if (wave == 0 && l == 0) d.ctl->rec_bytes = d.blk_coff[nv];
  if (nv == 0) return;
  uint64_t P = nwaves / nv;  // parts per block
  if (P < 1) P = 1;
  if (P > 64) P = 64;
  for (uint64_t u = wave; u < nv * P; u += nwaves) {
    const uint64_t b = u % nv, part = u / nv;
    const uint64_t off = d.blk_dec_off[b], co = d.blk_coff[b], n = d.blk_out_len[b];
    const uint4 *src = reinterpret_cast<const uint4 *>(d.dec + off);  // regions are 256-aligned
    uint4 *dst = reinterpret_cast<uint4 *>(d.cmp + co);
    const uint64_t n16 = (n + 15) / 16, k0 = n16 * part / P, k1 = n16 * (part + 1) / P;
    for (uint64_t k = k0 + l; k < k1; k += 64) dst[k] = src[k];
    const uint64_t i0 = d.blk_item_base[b], ni = d.blk_item_base[b + 1] - i0;
    for (uint64_t i = i0 + ni * part / P + l; i < i0 + ni * (part + 1) / P; i += 64) {
      const unsigned long long v = d.item_off[i];
      if (v & kItemInRecords) d.item_off[i] = kItemInRecords | ((v & ~kItemInRecords) - off + co);
    }
  }
}

void launch_compact(const DevBufs &d, const unsigned long long *nblocks_dev, uint64_t max_blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_compact_len, dim3(grid_blocks(max_blocks)), dim3(256), 0, st, d, nblocks_dev,
                     d.blk_coff + max_blocks + 1);
  launch_block_scan(d.blk_coff + max_blocks + 1, d.blk_coff, d.scan_tmp, nblocks_dev, max_blocks, st);
  unsigned g = (unsigned)(max_blocks * 16 < 4096 ? max_blocks * 16 : 4096);  // (16 parts per block when few)
  hipLaunchKernelGGL(k_compact, dim3(g < 1 ? 1 : g), dim3(256), 0, st, d, nblocks_dev);
}

// libzstd's error names (ZSTD_getErrorName) for codec_zstd.hip's ZErr codes
static const char *const kZstdErrNames[] = {
    "",
    "Src size is incorrect",
    "Unknown frame descriptor",
    "Corrupted block detected",
    "Restored data doesn't match checksum",
    "Dictionary mismatch",
    "Frame requires too much memory for decoding",
    "Unsupported frame parameter",
    "Dictionary is corrupted",
};

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
    if (off >= 1 && off < sizeof(kZstdErrNames) / sizeof(kZstdErrNames[0]))
      rio_set_error(e, RIO_ERR_ZSTD, file_off, "%s", kZstdErrNames[off]);
    else
      rio_set_error(e, RIO_ERR_ZSTD, file_off, "Corrupted block detected");
    break;
  default:
    rio_set_error(e, RIO_ERR_ARG, file_off, "codec not supported by this build");
  }
}

// ---------------------------------------------------------------- chains
// Transformer chains (registry.go:121-146): the blocks one untransform stage
// decoded, framed again as a chunk stream (chunk.go:31-53 layout: magic, crc 0,
// flag 0, size, total, index; payloads of 32,740 bytes) so the next stage's
// codec reads them like file chunks. Wave per block; block b's chunks start at
// chunk soff[b] of out.
__global__ void __launch_bounds__(256) k_reframe(const uint8_t *__restrict__ dec, const unsigned long long *dec_off,
                                                 const unsigned long long *out_len, const unsigned long long *soff,
                                                 uint64_t nv, uint32_t mlo, uint32_t mhi, uint8_t *__restrict__ out) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = threadIdx.x & 63;
  for (uint64_t b = wave; b < nv; b += nwaves) {
    const uint64_t len = out_len[b], c0 = soff[b], total = soff[b + 1] - c0;
    const uint8_t *src = dec + dec_off[b];
    for (uint64_t j = 0; j < total; j++) {
      uint8_t *ck = out + (c0 + j) * (uint64_t)kChunk;
      const uint64_t lo = j * (uint64_t)kMaxPayload;
      const uint32_t sz = (uint32_t)((len - lo) < (uint64_t)kMaxPayload ? (len - lo) : (uint64_t)kMaxPayload);
      if (l < 7) {
        const uint32_t h[7] = {mlo, mhi, 0u, 0u, sz, (uint32_t)total, (uint32_t)j};
        reinterpret_cast<uint32_t *>(ck)[l] = h[l];
      }
      for (uint32_t k = l; k < sz; k += 64) ck[kChunkHdr + k] = src[lo + k];
    }
  }
}

void launch_reframe(const uint8_t *dec, const unsigned long long *dec_off, const unsigned long long *out_len,
                    const unsigned long long *soff, uint64_t nv, uint64_t magic, uint8_t *out, hipStream_t st) {
  uint64_t g = (nv + 3) / 4;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(k_reframe, dim3((unsigned)(g ? g : 1)), dim3(256), 0, st, dec, dec_off, out_len, soff, nv,
                     (uint32_t)magic, (uint32_t)(magic >> 32), out);
}

}  // namespace rio
