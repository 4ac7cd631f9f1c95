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
//                 aligned loads + funnel shift), padding; 16 B stores, each row
//                 folded into the chunk CRC on the way (k_crc's tables)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_fold.h"
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

struct ChunkCtx {
  PaySrc s;
  unsigned long long p0, total, idx;
  uint32_t size, end;
};

__device__ __forceinline__ ChunkCtx chunk_ctx(const EncArgs &a, uint64_t c) {
  ChunkCtx x;
  const uint32_t b = a.ck_block[c];
  const unsigned long long c0 = a.ck0[b];
  x.total = a.nck[b];
  x.idx = c - c0;
  if (a.codec == RIO_CODEC_NONE) {
    const uint64_t f = enc_first(a, b);
    x.s.hdr = a.hdr + a.hdr_off[b];
    x.s.hlen = a.hdr_len[b];
    x.s.data = a.data + item_start(a, f);
  } else {
    x.s.hdr = a.comp + a.comp_off[b];
    x.s.hlen = ~0ull;
    x.s.data = nullptr;
  }
  x.s.len = a.pay_len[b];
  x.p0 = x.idx * kMaxPayload;
  const unsigned long long left = x.s.len - x.p0;
  x.size = (uint32_t)(left < (unsigned long long)kMaxPayload ? left : (unsigned long long)kMaxPayload);
  x.end = kChunkHdr + x.size;
  return x;
}

// the 16 chunk bytes at offset q0 byte by byte (header fields with CRC 0, the
// payload's ends, the start of the padding): the few units at a boundary
__device__ __noinline__ uint4 unit_words_slow(const EncArgs &a, const ChunkCtx &x, uint32_t q0) {
  uint32_t w[4];
  for (int k = 0; k < 4; k++) {
    uint32_t v = 0;
    for (int j = 0; j < 4; j++) {
      const uint32_t q = q0 + 4 * k + j;
      uint32_t bv;
      if (q < 8) bv = (uint32_t)(a.magic >> (8 * q)) & 0xff;
      else if (q < 16) bv = 0;  // the CRC (filled in last) and the flag
      else if (q < 20) bv = (x.size >> (8 * (q - 16))) & 0xff;
      else if (q < 24) bv = (uint32_t)(x.total >> (8 * (q - 20))) & 0xff;
      else if (q < 28) bv = (uint32_t)(x.idx >> (8 * (q - 24))) & 0xff;
      else if (q < x.end) bv = pay_byte(x.s, x.p0 + (q - kChunkHdr));
      else bv = (0xefbeaddeu >> (8 * ((q - x.end) & 3))) & 0xff;
      v |= bv << (8 * j);
    }
    w[k] = v;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// the 16 chunk bytes at offset q0: payload (aligned loads + funnel shift),
// padding, or the slow path
__device__ __forceinline__ void unit_words(const EncArgs &a, const ChunkCtx &x, uint32_t q0, uint32_t (&w)[4]) {
  const unsigned long long p = x.p0 + (q0 - kChunkHdr);
  if (q0 >= kChunkHdr && q0 + 16 <= x.end && (p + 16 <= x.s.hlen || p >= x.s.hlen)) {  // one source
    load16_any(p < x.s.hlen ? x.s.hdr + p : x.s.data + (p - x.s.hlen), w);
  } else if (q0 >= x.end) {  // padding: de ad be ef from the payload end
    const uint32_t r = (q0 - x.end) & 3;
    const uint32_t pat = 0xefbeaddeu;  // bytes de ad be ef
    const uint32_t v = r ? (pat >> (8 * r)) | (pat << (32 - 8 * r)) : pat;
    w[0] = w[1] = w[2] = w[3] = v;
  } else {
    const uint4 u = unit_words_slow(a, x, q0);
    w[0] = u.x;
    w[1] = u.y;
    w[2] = u.z;
    w[3] = u.w;
  }
}

// Wave per chunk, k_crc's layout (lane l owns bytes 1024 i + 16 l of row i):
// every row is built, stored (16 B per lane, 1 KiB per instruction) and folded
// into the lane's 4 CRC streams (crc_fold.h) in the same pass, rows
// software-pipelined in groups of 4 (the next group's loads in flight while one
// is stored and folded). The CRC goes into the header at the end: the chunk
// stream is written once and never read back.
constexpr int kEncWaves = 16;
constexpr int kEncGroup = 4;

__global__ void __launch_bounds__(64 * kEncWaves) k_enc_chunks(EncArgs a, uint64_t nchunks, CrcTabs t) {
  __shared__ __attribute__((aligned(16))) uint32_t s_fold[kFoldWords];
  __shared__ __attribute__((aligned(16))) uint32_t s_mul[kMulTables * 1024];
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(t.fold);
    uint4 *dst = reinterpret_cast<uint4 *>(s_fold);
    for (int i = threadIdx.x; i < kFoldWords / 4; i += blockDim.x) dst[i] = src[i];
    for (int i = threadIdx.x; i < kMulTables * 1024; i += blockDim.x) s_mul[i] = t.mul[i];
  }
  __syncthreads();
  const int l = lane_id();
  const uint32_t lb = (uint32_t)(l & (kFoldCopies - 1)) << 2;
  // (lanes 16-31 / 48-63 in rotated table order: conflict-free lookups, crc_fold.h fold_sel)
  const uint32_t rot = (uint32_t)((l >> 4) & 1);
  const uint32_t sel[4] = {fold_sel(0, rot), fold_sel(1, rot), fold_sel(2, rot), fold_sel(3, rot)};
  const char *tab = reinterpret_cast<const char *>(s_fold);
  const uint64_t nwaves = (uint64_t)gridDim.x * kEncWaves;
  for (uint64_t c = (uint64_t)blockIdx.x * kEncWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); c < nchunks;
       c += nwaves) {
    const ChunkCtx x = chunk_ctx(a, c);
    uint8_t *ck = a.out + c * kChunk;
    uint32_t s[4] = {0, 0, 0, 0}, sq[4] = {0, 0, 0, 0};  // (fold_row3: the stream is s ^ sq)
    uint32_t wa[kEncGroup][4], wb[kEncGroup][4];
#pragma unroll
    for (int r = 0; r < kEncGroup; r++) unit_words(a, x, 1024 * r + 16 * l, wa[r]);
#pragma unroll 1
    for (int g = 0; g < 32 / kEncGroup; g++) {
      if (g + 1 < 32 / kEncGroup) {
#pragma unroll
        for (int r = 0; r < kEncGroup; r++) unit_words(a, x, 1024 * (kEncGroup * (g + 1) + r) + 16 * l, wb[r]);
      }
#pragma unroll
      for (int r = 0; r < kEncGroup; r++) {
        const int row = kEncGroup * g + r;
        const uint32_t q0 = 1024 * row + 16 * l;
        *reinterpret_cast<uint4 *>(ck + q0) = make_uint4(wa[r][0], wa[r][1], wa[r][2], wa[r][3]);
        uint4 v = make_uint4(wa[r][0], wa[r][1], wa[r][2], wa[r][3]);
        if (row == 0 && l == 0) v.x = v.y = v.z = 0;  // magic and CRC are not covered
        if (1024 * (row + 1) > (int)x.end) {
          v.x = mask_dword(v.x, q0, x.end);
          v.y = mask_dword(v.y, q0 + 4, x.end);
          v.z = mask_dword(v.z, q0 + 8, x.end);
          v.w = mask_dword(v.w, q0 + 12, x.end);
        }
        if constexpr (kFoldPerm) fold_row3(tab, lb, v, s, sq, sel);
        else fold_row(tab, lb, v, s);
      }
#pragma unroll
      for (int r = 0; r < kEncGroup; r++)
#pragma unroll
        for (int k = 0; k < 4; k++) wa[r][k] = wb[r][k];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) s[k] ^= sq[k];
    // lane: V_t = s0 + s1 x^-32 + s2 x^-64 + s3 x^-96; lanes: V = sum_t V_t x^-128t
    uint32_t v = mul_const(s_mul, s[3]) ^ s[2];
    v = mul_const(s_mul, v) ^ s[1];
    v = mul_const(s_mul, v) ^ s[0];
#pragma unroll
    for (int lv = 0; lv < 6; lv++) {
      const uint32_t m = mul_const(s_mul + (lv + 1) * 1024, v);
      const int step = 1 << lv;
      const uint32_t o = __shfl(m, (l + step) & 63, 64);
      v ^= (l + step < 64) ? o : 0u;
    }
    if (l == 0) {
      const uint32_t fa = t.fix_a[x.size], fb = t.fix_b[x.size];
      const uint32_t crc = ~(fa ^ (x.size == (uint32_t)kMaxPayload ? v : gf_mul_dev(v, fb)));
      *reinterpret_cast<uint32_t *>(ck + 8) = crc;
    }
  }
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
void launch_enc_chunks(const EncArgs &a, uint64_t nchunks, const CrcTabs &t, int ncu, hipStream_t st) {
  uint64_t g = (nchunks + kEncWaves - 1) / kEncWaves;
  const uint64_t cap = (uint64_t)(ncu > 0 ? ncu : 256);
  if (g > cap) g = cap;
  hipLaunchKernelGGL(k_enc_chunks, dim3((unsigned)(g ? g : 1)), dim3(64 * kEncWaves), 0, st, a, nchunks, t);
}
void launch_enc_boff(const unsigned long long *ck0, unsigned long long *boff, uint64_t nblocks, hipStream_t st) {
  hipLaunchKernelGGL(k_enc_boff, dim3(enc_grid(nblocks, 256)), dim3(256), 0, st, ck0, boff, nblocks);
}

}  // namespace rio
