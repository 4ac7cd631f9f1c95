// Writer encode path on the GPU: the mirror of the scan.
// Items -> packed blocks (generatePackedHeaderv2 + items, writerv2.go:388-442)
// -> chunk stream (ChunkWriter.Write, internal/chunk.go:100-141: 28-byte
// headers, payload, 0xdeadbeef padding, CRC32 over [12, 28 + size)).
//
//   k_enc_count   wave per block: header length (uvarints of the count and of
//                 every item size, wave reduction) and payload length
//   (scan)        header scratch offsets
//   k_enc_header  wave per block: the varint header into scratch (positions by
//                 wave prefix sums of the varint lengths)
//   [k_deflate    flate: wave per block, the payload compressed (deflate_enc.hip)]
//   k_enc_nck     chunks per block: (len - 1) / 32740 + 1 (one for an empty payload)
//   (scan)        first chunk per block
//   k_enc_ckmap   chunk -> block
//   k_enc_chunks  wave per chunk: header fields, payload (16 B per lane from
//                 aligned loads + funnel shift), padding; 16 B stores
//   k_crc         the scan's own CRC kernel over the written chunks
//   k_enc_crc     the CRCs into the chunk headers
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "encode.h"
#include "rio_internal.h"

namespace rio {

__device__ __forceinline__ uint32_t uvarint_len(unsigned long long v) {
  uint32_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}

__device__ __forceinline__ uint64_t enc_first(const EncArgs &a, uint64_t b) {
  const uint64_t f = b * a.per_block;
  return f < a.n_items ? f : a.n_items;
}

__device__ __forceinline__ unsigned long long item_start(const EncArgs &a, uint64_t i) {
  return i == 0 ? 0ull : a.item_end[i - 1];
}

__global__ void __launch_bounds__(256) k_enc_count(EncArgs a) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t b = wave; b < a.nblocks; b += nwaves) {
    const uint64_t f = enc_first(a, b), e = enc_first(a, b + 1);
    unsigned long long vl = 0;
    for (uint64_t i = f + l; i < e; i += 64) vl += uvarint_len(a.item_end[i] - item_start(a, i));
    vl = wave_sum<unsigned long long>(vl);
    if (l == 0) {
      const unsigned long long hdr = uvarint_len(e - f) + vl;
      a.hdr_len[b] = hdr;
      a.pay_len[b] = hdr + (e > f ? a.item_end[e - 1] - item_start(a, f) : 0ull);
    }
  }
}

__global__ void __launch_bounds__(256) k_enc_header(EncArgs a) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t b = wave; b < a.nblocks; b += nwaves) {
    const uint64_t f = enc_first(a, b), e = enc_first(a, b + 1);
    uint8_t *h = a.hdr + a.hdr_off[b];
    const unsigned long long n = e - f;
    const uint32_t n0 = uvarint_len(n);
    if (l == 0) {
      unsigned long long v = n;
      for (uint32_t k = 0; k < n0; k++, v >>= 7) h[k] = (uint8_t)((v & 0x7f) | (k + 1 < n0 ? 0x80 : 0));
    }
    unsigned long long pos = n0;
    for (uint64_t i0 = f; i0 < e; i0 += 64) {
      const uint64_t i = i0 + l;
      unsigned long long v = i < e ? a.item_end[i] - item_start(a, i) : 0ull;
      const uint32_t len = i < e ? uvarint_len(v) : 0u;
      const uint32_t incl = wave_incl_sum<uint32_t>(len);
      uint8_t *q = h + pos + (incl - len);
      for (uint32_t k = 0; k < len; k++, v >>= 7) q[k] = (uint8_t)((v & 0x7f) | (k + 1 < len ? 0x80 : 0));
      pos += __shfl(incl, 63, 64);
    }
  }
}

__global__ void k_enc_nck(EncArgs a) {
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < a.nblocks;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long len = a.pay_len[b];
    a.nck[b] = len == 0 ? 1ull : (len - 1) / kMaxPayload + 1;
  }
}

__global__ void __launch_bounds__(256) k_enc_ckmap(EncArgs a) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t b = wave; b < a.nblocks; b += nwaves) {
    const unsigned long long c0 = a.ck0[b], n = a.nck[b];
    for (uint64_t k = l; k < n; k += 64) a.ck_block[c0 + k] = (uint32_t)b;
  }
}

// A block payload's bytes: the varint header scratch, then the block's item
// bytes (none codec), or the transformed payload (flate)
struct PaySrc {
  const uint8_t *hdr;     // none: header bytes (hlen); flate: the whole payload
  unsigned long long hlen;
  const uint8_t *data;    // none: the block's item bytes
  unsigned long long len;  // payload length
};

__device__ __forceinline__ void load16_any(const uint8_t *p, uint32_t (&w)[4]) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  if (sh == 0) {
#pragma unroll
    for (int k = 0; k < 4; k++) w[k] = q[k];
    return;
  }
  uint32_t d[5];
#pragma unroll
  for (int k = 0; k < 5; k++) d[k] = q[k];  // the 5th dword holds byte 15: inside the source
#pragma unroll
  for (int k = 0; k < 4; k++) w[k] = (d[k] >> sh) | (d[k + 1] << (32 - sh));
}

__device__ __forceinline__ uint32_t pay_byte(const PaySrc &s, unsigned long long p) {
  return p < s.hlen ? s.hdr[p] : s.data[p - s.hlen];
}

__global__ void __launch_bounds__(256) k_enc_chunks(EncArgs a, uint64_t nchunks) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t c = wave; c < nchunks; c += nwaves) {
    const uint32_t b = a.ck_block[c];
    const unsigned long long c0 = a.ck0[b], total = a.nck[b], idx = c - c0;
    PaySrc s;
    if (a.codec == RIO_CODEC_NONE) {
      const uint64_t f = enc_first(a, b);
      s.hdr = a.hdr + a.hdr_off[b];
      s.hlen = a.hdr_len[b];
      s.data = a.data + item_start(a, f);
    } else {
      s.hdr = a.comp + a.comp_off[b];
      s.hlen = ~0ull;
      s.data = nullptr;
    }
    s.len = a.pay_len[b];
    const unsigned long long p0 = idx * kMaxPayload;
    const unsigned long long left = s.len - p0;
    const uint32_t size = (uint32_t)(left < (unsigned long long)kMaxPayload ? left : (unsigned long long)kMaxPayload);
    const uint32_t end = kChunkHdr + size;
    uint8_t *ck = a.out + c * kChunk;
    if (l == 0) a.ck_size[c] = size;
    for (uint32_t u = l; u < kChunk / 16; u += 64) {
      const uint32_t q0 = 16 * u;
      uint32_t w[4];
      if (q0 >= kChunkHdr && q0 + 16 <= end) {  // payload only
        const unsigned long long p = p0 + (q0 - kChunkHdr);
        if (p + 16 <= s.hlen) load16_any(s.hdr + p, w);
        else if (p >= s.hlen) load16_any(s.data + (p - s.hlen), w);
        else {
#pragma unroll
          for (int k = 0; k < 4; k++) {
            uint32_t x = 0;
            for (int j = 0; j < 4; j++) x |= pay_byte(s, p + 4 * k + j) << (8 * j);
            w[k] = x;
          }
        }
      } else if (q0 >= end) {  // padding: de ad be ef from the payload end
        const uint32_t r = (q0 - end) & 3;
        const uint32_t pat = 0xefbeaddeu;  // bytes de ad be ef
        const uint32_t v = r ? (pat >> (8 * r)) | (pat << (32 - 8 * r)) : pat;
        w[0] = w[1] = w[2] = w[3] = v;
      } else {  // header fields, the payload's ends, padding start: byte by byte
#pragma unroll
        for (int k = 0; k < 4; k++) {
          uint32_t x = 0;
          for (int j = 0; j < 4; j++) {
            const uint32_t q = q0 + 4 * k + j;
            uint32_t v;
            if (q < 8) v = (uint32_t)(a.magic >> (8 * q)) & 0xff;
            else if (q < 12) v = 0;  // the CRC, written by k_enc_crc
            else if (q < 16) v = 0;  // flag
            else if (q < 20) v = (size >> (8 * (q - 16))) & 0xff;
            else if (q < 24) v = (uint32_t)(total >> (8 * (q - 20))) & 0xff;
            else if (q < 28) v = (uint32_t)(idx >> (8 * (q - 24))) & 0xff;
            else if (q < end) v = pay_byte(s, p0 + (q - kChunkHdr));
            else v = (0xefbeaddeu >> (8 * ((q - end) & 3))) & 0xff;
            x |= v << (8 * j);
          }
          w[k] = x;
        }
      }
      *reinterpret_cast<uint4 *>(ck + q0) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

__global__ void k_enc_crc(uint8_t *out, const uint32_t *ck_crc, uint64_t nchunks) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks;
       c += (uint64_t)gridDim.x * blockDim.x)
    *reinterpret_cast<uint32_t *>(out + c * kChunk + 8) = ck_crc[c];
}

__global__ void k_enc_boff(const unsigned long long *ck0, unsigned long long *boff, uint64_t nblocks) {
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblocks;
       b += (uint64_t)gridDim.x * blockDim.x)
    boff[b] = ck0[b] * kChunk;
}

static unsigned enc_grid(uint64_t n, uint64_t per_wg) {
  uint64_t g = (n + per_wg - 1) / per_wg;
  if (g > 8192) g = 8192;
  return (unsigned)(g ? g : 1);
}

void launch_enc_count(const EncArgs &a, hipStream_t st) {
  hipLaunchKernelGGL(k_enc_count, dim3(enc_grid(a.nblocks, 4)), dim3(256), 0, st, a);
}
void launch_enc_header(const EncArgs &a, hipStream_t st) {
  hipLaunchKernelGGL(k_enc_header, dim3(enc_grid(a.nblocks, 4)), dim3(256), 0, st, a);
}
void launch_enc_nck(const EncArgs &a, hipStream_t st) {
  hipLaunchKernelGGL(k_enc_nck, dim3(enc_grid(a.nblocks, 256)), dim3(256), 0, st, a);
}
void launch_enc_ckmap(const EncArgs &a, hipStream_t st) {
  hipLaunchKernelGGL(k_enc_ckmap, dim3(enc_grid(a.nblocks, 4)), dim3(256), 0, st, a);
}
void launch_enc_chunks(const EncArgs &a, uint64_t nchunks, hipStream_t st) {
  hipLaunchKernelGGL(k_enc_chunks, dim3(enc_grid(nchunks, 4)), dim3(256), 0, st, a, nchunks);
}
void launch_enc_boff(const unsigned long long *ck0, unsigned long long *boff, uint64_t nblocks, hipStream_t st) {
  hipLaunchKernelGGL(k_enc_boff, dim3(enc_grid(nblocks, 256)), dim3(256), 0, st, ck0, boff, nblocks);
}
void launch_enc_crc(uint8_t *out, const uint32_t *ck_crc, uint64_t nchunks, hipStream_t st) {
  hipLaunchKernelGGL(k_enc_crc, dim3(enc_grid(nchunks, 256)), dim3(256), 0, st, out, ck_crc, nchunks);
}

}  // namespace rio
