// Zstandard (RFC 8878) block decode: the "zstd" untransformer
// (recordiozstd.zstdUncompress, recordio/recordiozstd/recordiozstd.go:67-78 ->
// compress/zstd.Decompress, compress/zstd/zstd_cgo.go:34-41 -> DataDog/zstd
// v1.4.1, i.e. libzstd ZSTD_decompress over every frame of the block).
//
// One wave per recordio block:
//  - the chunk payloads are flattened into contiguous scratch first, as
//    recordiozstd.flattenIov does (recordiozstd.go:40-52);
//  - frame / block headers, FSE table descriptions and the sequence
//    bitstream are walked by every lane in step (the values are wave-uniform)
//    and the tables are built by lane 0 into LDS; the checks and their order
//    follow the oracle's restatement (oracle/zstd_dec.c), so the first error
//    a block hits -- and so its libzstd error name -- is the same;
//  - Huffman-coded literals: each of the 4 streams is decoded by its own lane
//    into a per-wave literal buffer in HBM (128 KiB, the block maximum);
//  - each sequence is executed by the whole wave: the literal run, then the
//    match copy reading the frame's earlier output from the decode region
//    (zstd windows are MiB-sized, beyond LDS).
// Errors: blk_a = kCodecZstd with blk_b = ZErr (the names are in codec.hip),
// kCodecZstdEmpty, or kCodecFull with the frames' declared content size for
// the host's retry.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "device_common.h"
#include "rio_internal.h"

namespace rio {

// libzstd error names, in codec.hip's table order
enum ZErr : uint32_t {
  kZOk = 0,
  kZSrc = 1,       // "Src size is incorrect"
  kZPrefix = 2,    // "Unknown frame descriptor"
  kZCorrupt = 3,   // "Corrupted block detected"
  kZChecksum = 4,  // "Restored data doesn't match checksum"
  kZDict = 5,      // "Dictionary mismatch"
  kZWindow = 6,    // "Frame requires too much memory for decoding"
  kZNotSup = 7,    // "Unsupported frame parameter"
  kZFull = 100,    // (internal) decode region too small
};

constexpr uint32_t kZMagic = 0xFD2FB528u;
constexpr int kZBlockMax = 128 * 1024;
constexpr uint64_t kZLitStride = kZBlockMax + 256;  // per-wave literal buffer
#ifndef RIO_ZWAVES
#define RIO_ZWAVES 12
#endif
constexpr int kZWaves = RIO_ZWAVES;  // resident zstd waves per CU (LDS ~10 KiB each)
#ifndef RIO_ZFIX_WAVES
// 6 per SIMD (round 2: 8 waves 162.0 ms for C4, 20: 156.1, 28: 159.8; round 6:
// 24 against 20, serial C4 40.8 against 40.0, profiles/r06_zstd_fix_waves_ab.jsonl)
#define RIO_ZFIX_WAVES 24
#endif
constexpr int kZFixWaves = RIO_ZFIX_WAVES;            // k_zstd_fix waves per CU

__constant__ uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,  12,   13,   14,   15,   16,   18,
                                     20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14,  15,  16,  17,   18,   19,   20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32,  33,  34,  35,   37,   39,   41,
                                     43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
// (base | extra bits << 24) per code: one scalar load each in the sequence loop
// (a byte table would be a vector load whose wait drains every load in flight)
struct ZCodes {
  uint32_t ll[36], ml[53];
};
__constant__ ZCodes kZCodes = {
    {0 | 0u << 24,      1 | 0u << 24,      2 | 0u << 24,      3 | 0u << 24,      4 | 0u << 24,      5 | 0u << 24,
     6 | 0u << 24,      7 | 0u << 24,      8 | 0u << 24,      9 | 0u << 24,      10 | 0u << 24,     11 | 0u << 24,
     12 | 0u << 24,     13 | 0u << 24,     14 | 0u << 24,     15 | 0u << 24,     16 | 1u << 24,     18 | 1u << 24,
     20 | 1u << 24,     22 | 1u << 24,     24 | 2u << 24,     28 | 2u << 24,     32 | 3u << 24,     40 | 3u << 24,
     48 | 4u << 24,     64 | 6u << 24,     128 | 7u << 24,    256 | 8u << 24,    512 | 9u << 24,    1024 | 10u << 24,
     2048 | 11u << 24,  4096 | 12u << 24,  8192 | 13u << 24,  16384 | 14u << 24, 32768 | 15u << 24, 65536 | 16u << 24},
    {3 | 0u << 24,     4 | 0u << 24,     5 | 0u << 24,     6 | 0u << 24,     7 | 0u << 24,     8 | 0u << 24,
     9 | 0u << 24,     10 | 0u << 24,    11 | 0u << 24,    12 | 0u << 24,    13 | 0u << 24,    14 | 0u << 24,
     15 | 0u << 24,    16 | 0u << 24,    17 | 0u << 24,    18 | 0u << 24,    19 | 0u << 24,    20 | 0u << 24,
     21 | 0u << 24,    22 | 0u << 24,    23 | 0u << 24,    24 | 0u << 24,    25 | 0u << 24,    26 | 0u << 24,
     27 | 0u << 24,    28 | 0u << 24,    29 | 0u << 24,    30 | 0u << 24,    31 | 0u << 24,    32 | 0u << 24,
     33 | 0u << 24,    34 | 0u << 24,    35 | 1u << 24,    37 | 1u << 24,    39 | 1u << 24,    41 | 1u << 24,
     43 | 2u << 24,    47 | 2u << 24,    51 | 3u << 24,    59 | 3u << 24,    67 | 4u << 24,    83 | 4u << 24,
     99 | 5u << 24,    131 | 7u << 24,   259 | 8u << 24,   515 | 9u << 24,   1027 | 10u << 24, 2051 | 11u << 24,
     4099 | 12u << 24, 8195 | 13u << 24, 16387 | 14u << 24, 32771 | 15u << 24, 65539 | 16u << 24}};

// 29 predefined offset codes; 29..31 (the table's max_sym) have count 0
__constant__ int16_t kOFDef[32] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, 0, 0, 0};

constexpr int kZDesc = 512;  // staged description bytes (an NCount needs < 100, a Huffman tree < 129)
struct ZLds {
  uint32_t ll[1 << 9], ml[1 << 9], of[1 << 8];  // FSE cells: sym | nbits << 8 | base << 16
  uint32_t wt[1 << 6];                           // FSE table of Huffman weights
  uint16_t huf[1 << 11];                         // Huffman: sym << 4 | nbits
  int16_t norm[64];
  uint16_t next[64];
  uint8_t w[256];
  int32_t res[12];  // lane 0's results, broadcast
  uint32_t sring[128];      // the sequence bitstream, two 256 B blocks (ZSeqBr)
  uint8_t hout[4][256];     // Huffman streams' decoded literals, flushed 256 at a time
  // table descriptions (FSE NCount, Huffman tree) staged from HBM by the whole
  // wave: lane 0's serial bit walks over them then cost LDS, not HBM, latency
  uint32_t desc[kZDesc / 4 + 4];
};

__device__ __forceinline__ void zsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// this wave's global stores complete before its next loads of the same bytes
__device__ __forceinline__ void zmem_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ int highbit(uint32_t v) { return 31 - __clz(v); }

// ---------------------------------------------------------------- bit readers
// backward (Huffman and FSE streams): bits [0, bit) of the stream starting at
// byte `start` of src remain; reads go downwards, bits below 0 read as zero
struct ZBwd {
  const uint32_t *w;  // src as dwords (src is 4-aligned)
  int64_t start8;     // 8 * start
  int64_t bit;
  int64_t cq;         // dword index cached in (c0, c1)
  uint32_t c0, c1;
  __device__ __forceinline__ uint32_t get(int64_t b, int nb) {  // bits [b, b+nb) relative, nb <= 32
    if (nb == 0) return 0;
    const int64_t a = start8 + b;
    const int64_t q = a >= 0 ? (a >> 5) : -((31 - a) >> 5);
    if (q != cq) {
      c0 = q >= 0 ? w[q] : 0u;
      c1 = q + 1 >= 0 ? w[q + 1] : 0u;
      cq = q;
    }
    const uint32_t sh = (uint32_t)(a - 32 * q);
    uint64_t v = ((((uint64_t)c1 << 32) | c0) >> sh) & ((nb >= 32) ? 0xffffffffull : ((1ull << nb) - 1));
    if (b < 0) v = (-b >= nb) ? 0 : (v & ~((1ull << (-b)) - 1));  // below the stream: zero
    return (uint32_t)v;
  }
  __device__ __forceinline__ uint32_t read(int nb) {
    bit -= nb;
    return get(bit, nb);
  }
  __device__ __forceinline__ uint32_t peek(int nb) { return get(bit - nb, nb); }
};
// the last byte's highest set bit marks the stream's end; false: empty / no marker
__device__ __forceinline__ bool bwd_init(ZBwd &r, const uint8_t *src, int64_t start, int64_t n) {
  if (n <= 0) return false;
  const uint32_t last = src[start + n - 1];
  if (last == 0) return false;
  r.w = reinterpret_cast<const uint32_t *>(src);
  r.start8 = 8 * start;
  r.bit = n * 8 - (8 - highbit(last));
  r.cq = INT64_MIN;
  r.c0 = r.c1 = 0;
  return true;
}

// forward (FSE table descriptions): bits past byte n read as zero; p is a
// staged description (ZLds::desc), zero-padded, nb <= 16
__device__ __forceinline__ uint32_t fwd_peek(const uint8_t *p, int64_t n, uint64_t pos, int nb) {
  const uint64_t B = pos >> 3;
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) v |= (int64_t)(B + i) < n ? (uint32_t)p[B + i] << (8 * i) : 0u;
  return (v >> (pos & 7)) & ((1u << nb) - 1u);
}

// ---------------------------------------------------------------- FSE
// FSE_readNCount (oracle fse_read_ncount): bytes consumed or -1
__device__ int z_read_ncount(int16_t *norm, int *max_sym, int *log, const uint8_t *src, int64_t n, int max_log) {
  uint64_t pos = 0;
  const int al = (int)fwd_peek(src, n, pos, 4) + 5;
  pos += 4;
  if (al > max_log) return -1;
  *log = al;
  int remaining = (1 << al) + 1;
  int threshold = 1 << al;
  int nbits = al + 1;
  int sym = 0;
  int prev0 = 0;
  while (remaining > 1 && sym <= *max_sym) {
    if (prev0) {
      int n0 = sym;
      while (fwd_peek(src, n, pos, 16) == 0xFFFF) {
        n0 += 24;
        pos += 16;
      }
      while (fwd_peek(src, n, pos, 2) == 3) {
        n0 += 3;
        pos += 2;
      }
      n0 += (int)fwd_peek(src, n, pos, 2);
      pos += 2;
      if (n0 > *max_sym) return -1;
      while (sym < n0) norm[sym++] = 0;
      if (pos > 8 * (uint64_t)n) return -1;
    }
    const int max = (2 * threshold - 1) - remaining;
    int count;
    const int low = (int)fwd_peek(src, n, pos, nbits - 1);
    if (low < max) {
      count = low;
      pos += nbits - 1;
    } else {
      count = (int)fwd_peek(src, n, pos, nbits);
      if (count >= threshold) count -= max;
      pos += nbits;
    }
    count--;
    remaining -= count < 0 ? -count : count;
    norm[sym++] = (int16_t)count;
    prev0 = (count == 0);
    while (remaining < threshold) {
      nbits--;
      threshold >>= 1;
    }
    if (pos > 8 * (uint64_t)n) return -1;
  }
  if (remaining != 1) return -1;
  *max_sym = sym - 1;
  return (int)((pos + 7) >> 3);
}

// FSE decoding table (oracle fse_build); cells sym | nbits << 8 | base << 16
__device__ bool z_fse_build(uint32_t *t, uint16_t *next, const int16_t *norm, int max_sym, int log) {
  const int size = 1 << log;
  int high = size - 1;
  for (int s = 0; s <= max_sym; s++) {
    if (norm[s] == -1) {
      t[high--] = (uint32_t)s;
      next[s] = 1;
    } else {
      next[s] = (uint16_t)norm[s];
    }
  }
  const int step = (size >> 1) + (size >> 3) + 3;
  const int mask = size - 1;
  int pos = 0;
  for (int s = 0; s <= max_sym; s++) {
    for (int i = 0; i < norm[s]; i++) {
      t[pos] = (uint32_t)s;
      do {
        pos = (pos + step) & mask;
      } while (pos > high);
    }
  }
  if (pos != 0) return false;
  for (int u = 0; u < size; u++) {
    const uint32_t s = t[u] & 0xff;
    const uint32_t ns = next[s]++;
    const int nb = log - highbit(ns);
    t[u] = s | ((uint32_t)nb << 8) | (((ns << nb) - size) << 16);
  }
  return true;
}

// ---------------------------------------------------------------- Huffman
// tree description -> table (oracle huf_read); bytes used or -1; *max_bits set
__device__ int z_huf_read(ZLds &L, int *max_bits_out, const uint8_t *src, int64_t start, int64_t n) {
  if (n < 1) return -1;
  uint8_t *w = L.w;
  int nw = 0;
  const int hb = src[start];
  int64_t used;
  if (hb >= 128) {
    nw = hb - 127;
    used = 1 + (nw + 1) / 2;
    if (used > n) return -1;
    for (int i = 0; i < nw; i++) {
      const uint32_t b = src[start + 1 + i / 2];
      w[i] = (uint8_t)((i & 1) ? (b & 15) : (b >> 4));
    }
  } else {
    used = 1 + hb;
    if (used > n || hb == 0) return -1;
    int max_sym = 15, log;
    const int k = z_read_ncount(L.norm, &max_sym, &log, src + start + 1, hb, 6);
    if (k < 0 || k > hb) return -1;
    if (!z_fse_build(L.wt, L.next, L.norm, max_sym, log)) return -1;
    ZBwd r;
    if (!bwd_init(r, src, start + 1 + k, hb - k)) return -1;
    uint32_t s1 = r.read(log), s2 = r.read(log);
    for (;;) {
      if (nw > 254) return -1;
      w[nw++] = (uint8_t)(L.wt[s1] & 0xff);
      s1 = (L.wt[s1] >> 16) + r.read((L.wt[s1] >> 8) & 0xff);
      if (r.bit < 0) {
        w[nw++] = (uint8_t)(L.wt[s2] & 0xff);
        break;
      }
      if (nw > 254) return -1;
      w[nw++] = (uint8_t)(L.wt[s2] & 0xff);
      s2 = (L.wt[s2] >> 16) + r.read((L.wt[s2] >> 8) & 0xff);
      if (r.bit < 0) {
        w[nw++] = (uint8_t)(L.wt[s1] & 0xff);
        break;
      }
    }
  }
  uint32_t total = 0;
  for (int i = 0; i < nw; i++) {
    if (w[i] > 11) return -1;
    if (w[i]) total += 1u << (w[i] - 1);
  }
  if (total == 0) return -1;
  const int max_bits = highbit(total) + 1;
  const uint32_t rest = (1u << max_bits) - total;
  if (rest & (rest - 1)) return -1;
  if (nw + 1 > 256 || max_bits > 11) return -1;
  w[nw++] = (uint8_t)(highbit(rest) + 1);
  uint32_t rank[13];
  for (int i = 0; i < 13; i++) rank[i] = 0;
  for (int i = 0; i < nw; i++) rank[w[i]]++;
  uint32_t start_[13];
  uint32_t acc = 0;
  for (int wt = 1; wt <= max_bits; wt++) {
    start_[wt] = acc;
    acc += rank[wt] << (wt - 1);
  }
  if (acc != (1u << max_bits)) return -1;
  for (int s = 0; s < nw; s++) {
    const int wt = w[s];
    if (!wt) continue;
    const uint32_t len = 1u << (wt - 1);
    const uint16_t e = (uint16_t)((s << 4) | (max_bits + 1 - wt));
    for (uint32_t j = 0; j < len; j++) L.huf[start_[wt] + j] = e;
    start_[wt] += len;
  }
  *max_bits_out = max_bits;
  return (int)used;
}

// Backward bit reader for the hot loops (Huffman literal streams, the sequence
// bitstream): remaining bits are [lo, bit) of the dword array w (w = the
// stream's first byte rounded down to 4; bits below lo read as zero). The
// window is dwords q (c0) and q+1 (c1); the next 4 dwords down are in flight
// (pf[0] = dword q-1 ...) so that stepping down does not wait on memory.
// U: the state is wave-uniform (every lane walks the same stream): a dword is
// made scalar only when it enters the window, never at its load (that would
// wait for the load right there).
template <bool U, int PF = 4>
struct ZBrT {
  static constexpr int kPf = PF;
  const uint32_t *w;
  int32_t bit, lo, q;
  uint32_t c0, c1, pf[kPf];
  __device__ __forceinline__ uint32_t ld(int32_t i) const { return i >= 0 ? w[i] : 0u; }
  __device__ __forceinline__ uint32_t mk(uint32_t v) const { return U ? uni(v) : v; }
  // false: empty stream or no end marker in its last byte
  __device__ __forceinline__ bool init(const uint8_t *src, int64_t start, int64_t n) {
    if (n <= 0) return false;
    const uint32_t last = src[start + n - 1];
    if (last == 0) return false;
    w = reinterpret_cast<const uint32_t *>(src + (start & ~3ll));
    lo = 8 * (int32_t)(start & 3);
    bit = lo + 8 * (int32_t)n - (8 - highbit(last));
    q = INT32_MIN;
    return true;
  }
  __device__ __forceinline__ void seek(int32_t b) {
    const int32_t qq = b >> 5;
    if (qq != q) {
      if (qq == q - 1) {
        c1 = c0;
        c0 = mk(pf[0]);
#pragma unroll
        for (int i = 0; i + 1 < kPf; i++) pf[i] = pf[i + 1];
        pf[kPf - 1] = ld(qq - kPf);
      } else {
        c0 = mk(ld(qq));
        c1 = mk(ld(qq + 1));
#pragma unroll
        for (int i = 0; i < kPf; i++) pf[i] = ld(qq - 1 - i);
      }
      q = qq;
    }
  }
  // bits [b, b + nb), nb <= 32
  __device__ __forceinline__ uint32_t get(int32_t b, int nb) {
    seek(b);
    uint32_t v = __builtin_amdgcn_alignbit(c1, c0, (uint32_t)b & 31u);
    v &= nb >= 32 ? ~0u : ((1u << nb) - 1u);
    if (b < lo) v = (lo - b >= nb) ? 0u : (v & (~0u << (lo - b)));
    return v;
  }
  __device__ __forceinline__ uint32_t read(int nb) {
    bit -= nb;
    return get(bit, nb);
  }
  __device__ __forceinline__ bool overrun() const { return bit < lo; }
  __device__ __forceinline__ bool exact() const { return bit == lo; }
};
using ZBr = ZBrT<false>;

// The sequence bitstream reader (wave-uniform): the stream moves through LDS
// in 256 B blocks, two resident (block B in ring slot B & 1). Every lane
// loads one dword of the block after next when a block is entered, and stores
// it into LDS when that block is entered in turn, so the only wait on memory
// is for a load issued ~80 sequences earlier.
struct ZSeqBr {
  const uint32_t *w;
  uint32_t *ring;
  int32_t bit, lo, q, inst;  // inst: the lowest block in LDS
  uint32_t c0, c1, pre;      // window dwords q, q+1 (scalar); this lane's dword of block inst-1
  __device__ __forceinline__ uint32_t ld(int32_t i) const { return i >= 0 ? w[i] : 0u; }
  __device__ bool init(const uint8_t *src, int64_t start, int64_t n, uint32_t *lds_ring) {
    if (n <= 0) return false;
    const uint32_t last = src[start + n - 1];
    if (last == 0) return false;
    const int l = lane_id();
    w = reinterpret_cast<const uint32_t *>(src + (start & ~3ll));
    ring = lds_ring;
    lo = 8 * (int32_t)(start & 3);
    bit = lo + 8 * (int32_t)n - (8 - highbit(last));
    const int32_t top = ((bit - 1) >> 5) >> 6;  // block of the highest stream dword
    zsync();
    ring[(top & 1) * 64 + l] = ld(top * 64 + l);
    ring[((top - 1) & 1) * 64 + l] = ld((top - 1) * 64 + l);
    pre = ld((top - 2) * 64 + l);
    inst = top - 1;
    q = INT32_MIN;
    zsync();
    return true;
  }
  __device__ __forceinline__ void seek(int32_t b) {
    const int32_t qq = b >> 5;
    if (qq != q) {
      if ((qq >> 6) < inst) {  // entering block inst-1 (one dword down at a time)
        zsync();
        ring[((inst - 1) & 1) * 64 + lane_id()] = pre;
        zsync();
        inst--;
        pre = ld((inst - 1) * 64 + lane_id());
      }
      if (qq == q - 1) {
        c1 = c0;
      } else {
        c1 = uni(ring[(qq + 1) & 127]);
      }
      c0 = uni(ring[qq & 127]);
      q = qq;
    }
  }
  __device__ __forceinline__ uint32_t read(int nb) {  // nb <= 32
    bit -= nb;
    const int32_t b = bit;
    seek(b);
    uint32_t v = __builtin_amdgcn_alignbit(c1, c0, (uint32_t)b & 31u);
    v &= nb >= 32 ? ~0u : ((1u << nb) - 1u);
    if (b < lo) v = (lo - b >= nb) ? 0u : (v & (~0u << (lo - b)));
    return v;
  }
  __device__ __forceinline__ bool overrun() const { return bit < lo; }
  __device__ __forceinline__ bool exact() const { return bit == lo; }
};

// Huffman literal streams (oracle huf_stream): lane t < ns decodes stream t
// (bytes [st, st + sn) of src) into out + t * seg, cnt symbols; true iff every
// stream decodes exactly. A read below a stream's start only ever lowers
// `bit`, so the final exact-consumption check also catches an overrun
// mid-stream. The decoded bytes go to LDS and are written out by the whole
// wave every 256 symbols: the decode loop issues no stores, so its input
// prefetch is never held up behind them.
__device__ bool z_huf_streams(ZLds &L, int max_bits, const uint8_t *src, int64_t st, int64_t sn, int ns, uint8_t *out,
                              int64_t seg, int64_t cnt) {
  const int l = lane_id();
  ZBr r;
  bool ok = true;
  if (l < ns) ok = r.init(src, st, sn);
  const int64_t seg_max = (int64_t)uni((uint32_t)(ns == 1 ? cnt : seg));
  for (int64_t i0 = 0; i0 < seg_max; i0 += 256) {
    if (l < ns && ok) {
      const int64_t m = cnt - i0 < 256 ? cnt - i0 : 256;
      for (int64_t j = 0; j < m; j++) {
        const uint32_t e = L.huf[r.get(r.bit - max_bits, max_bits)];
        L.hout[l][j] = (uint8_t)(e >> 4);
        r.bit -= (int32_t)(e & 15);
      }
    }
    zsync();
    for (int k = l; k < 256 * ns; k += 64) {
      const int t = k >> 8, j = k & 255;
      const int64_t ct = (int64_t)__builtin_amdgcn_readlane((int)cnt, t);
      if (i0 + j < ct) out[t * seg + i0 + j] = L.hout[t][j];
    }
    zsync();
  }
  if (l < ns && ok) ok = r.exact();
  return __ballot(l < ns && !ok) == 0;
}

// The literal streams with every lane decoding (round 3): each stream is cut
// into 64 / ns segments of its bits, lane j of a stream decoding its segment
// downwards from the segment's top -- a guessed symbol boundary; Huffman codes
// self-synchronise (as in k_flate_sync), so a lane restarts from its
// predecessor's exit until no start changes, then a prefix sum of the lanes'
// symbol counts places each lane's bytes and a second decode writes them.
// Valid iff every stream's chain ends exactly at the stream's first bit after
// exactly its count of symbols -- the serial decoder's exact-consumption
// check. Returns 1 ok, 0 a corrupt stream, -1 no convergence (the caller then
// decodes serially).
constexpr int kZHufIters = 8;
__device__ int z_huf_sync(ZLds &L, int max_bits, const uint8_t *src, int64_t st, int64_t sn, int ns, uint8_t *out,
                          int64_t seg, int64_t cnt) {
  const int l = lane_id();
  const int per = 64 / ns;                 // lanes per stream
  const int t = l / per, j = l % per;      // stream, segment
  const int64_t st_t = (int64_t)__shfl((long long)st, t, 64), sn_t = (int64_t)__shfl((long long)sn, t, 64);
  const int64_t cnt_t = (int64_t)__shfl((long long)cnt, t, 64);
  ZBr r;
  bool ok = r.init(src, st_t, sn_t);
  if (__ballot(!ok)) return 0;
  const int32_t lo = r.lo, top = r.bit;
  const int32_t S = (top - lo + per - 1) / per;  // bits per segment
  const int32_t seg_lo = top - (j + 1) * S < lo ? lo : top - (j + 1) * S;
  int32_t start = top - j * S < lo ? lo : top - j * S;
  // one decode of this lane's segment from `from`: symbols whose top is above
  // seg_lo; the exit is the first symbol boundary at or below it
  auto decode = [&](int32_t from, bool write, int64_t at, uint32_t &n, bool &bad) -> int32_t {
    r.bit = from;
    n = 0;
    bad = false;
    while (r.bit > seg_lo) {
      const uint32_t e = L.huf[r.get(r.bit - max_bits, max_bits)];
      const int32_t nb = (int32_t)(e & 15);
      if (nb == 0) {  // (no code: a malformed table or a lane off the chain)
        bad = true;
        r.bit -= 1;
        continue;
      }
      if (write) out[at + n] = (uint8_t)(e >> 4);
      r.bit -= nb;
      n++;
    }
    return r.bit;
  };
  uint32_t n = 0;
  bool bad = false, need = true, conv = false;
  int32_t ex = 0;
  for (int it = 0; it < kZHufIters; it++) {
    if (need) ex = decode(start, false, 0, n, bad);
    const int32_t prev = __shfl_up(ex, 1, 64);
    const int32_t nst = j == 0 ? top : prev;
    need = nst != start;
    if (need) start = nst;
    if (!__ballot(need)) {
      conv = true;
      break;
    }
  }
  if (!conv) return -1;
  // every stream: its last lane's exit at the stream's first bit, its symbols
  // its count, no undecodable code on the chain
  const uint32_t incl = wave_incl_sum_dpp(n);
  const uint32_t before = (uint32_t)__shfl((int)incl, t > 0 ? t * per - 1 : 0, 64);
  const uint32_t pre = t > 0 ? before : 0u;  // the symbols of the streams before this one
  const uint32_t excl = incl - n - pre;
  const uint32_t tot = (uint32_t)__shfl((int)incl, t * per + per - 1, 64) - pre;
  const bool bad_stream = (j == per - 1 && ex != lo) || (j == 0 && (int64_t)tot != cnt_t) || bad;
  if (__ballot(bad_stream)) return 0;
  uint32_t n2 = 0;
  bool bad2 = false;
  decode(start, true, (int64_t)t * seg + excl, n2, bad2);
  return 1;
}

// ---------------------------------------------------------------- sequence tables
// (oracle seq_table) mode 0 predefined, 1 RLE, 2 compressed, 3 repeat; bytes used or -1
__device__ int z_seq_table(uint32_t *t, uint16_t *next, int16_t *norm, int *have, int *log_io, int mode,
                           const uint8_t *src, int64_t start, int64_t n, const int16_t *def, int def_log, int max_sym,
                           int max_log) {
  if (mode == 0) {
    for (int s = 0; s <= max_sym; s++) norm[s] = def[s];
    z_fse_build(t, next, norm, max_sym, def_log);
    *log_io = def_log;
    *have = 1;
    return 0;
  }
  if (mode == 1) {
    if (n < 1 || src[start] > max_sym) return -1;
    t[0] = src[start];  // log 0: nbits 0, base 0
    *log_io = 0;
    *have = 1;
    return 1;
  }
  if (mode == 2) {
    int ms = max_sym, log;
    const int k = z_read_ncount(norm, &ms, &log, src + start, n, max_log);
    if (k < 0 || k > n) return -1;
    if (!z_fse_build(t, next, norm, ms, log)) return -1;
    *log_io = log;
    *have = 1;
    return k;
  }
  if (!*have) return -1;
  return 0;
}

// ---------------------------------------------------------------- frame state
struct ZFrame {
  const uint8_t *src;  // flattened compressed block
  uint8_t *out;        // decode region (serial path)
  int64_t cap, olen, frame_start;  // olen: output bytes so far (whole recordio block)
  uint8_t *lit;        // the current zstd block's literals
  int max_bits, have_huf, have_ll, have_of, have_ml;
  int ll_log, of_log, ml_log;
  uint64_t rep0, rep1, rep2;
};

#ifdef RIO_ZPROF
#define ZPROF_T(v) const uint64_t v = __builtin_readcyclecounter()
#define ZPROF_ADD(i, t0) \
  if (lane_id() == 0) atomicAdd(&zprof_ctl->zprof[i], (unsigned long long)(__builtin_readcyclecounter() - (t0)))
__device__ Ctl *zprof_ctl;
#else
#define ZPROF_T(v)
#define ZPROF_ADD(i, t0)
#endif

constexpr uint32_t kZSlow = 101;  // (internal) the fast path's scratch is too small: serial path

// lane 0's value in every lane
__device__ __forceinline__ int32_t zbcast(ZLds &L, int slot, int32_t v) {
  zsync();
  if (lane_id() == 0) L.res[slot] = v;
  zsync();
  return L.res[slot];
}

// src[start, start + min(n, kZDesc)) into L.desc, zero after; every lane
__device__ __forceinline__ const uint8_t *z_stage(ZLds &L, const uint8_t *src, int64_t start, int64_t n) {
  uint8_t *dsc = reinterpret_cast<uint8_t *>(L.desc);
  zsync();
  for (int k = lane_id(); k < kZDesc + 16; k += 64) dsc[k] = k < n && k < kZDesc ? src[start + k] : 0;
  zsync();
  return dsc;
}

// Literals section of a compressed block (oracle decode_block, first part):
// the block's literals into z.lit, pos advanced past the section. A
// regenerated size above max_regen returns kZSlow before anything is written.
__device__ uint32_t z_literals(ZFrame &z, ZLds &L, int64_t bstart, int64_t n, int64_t &pos, int64_t &regen_out,
                               int64_t max_regen) {
  const int l = lane_id();
  const uint8_t *src = z.src;
  if (n < 1) return kZCorrupt;
  const uint32_t b0 = src[bstart];
  const int lt = b0 & 3, sf = (b0 >> 2) & 3;
  int64_t regen = 0, csize = 0, hsz = 0;
  int streams = 1;
  if (lt == 0 || lt == 1) {
    if (sf == 0 || sf == 2) {
      regen = b0 >> 3;
      hsz = 1;
    } else if (sf == 1) {
      if (n < 2) return kZCorrupt;
      regen = (b0 >> 4) + ((int64_t)src[bstart + 1] << 4);
      hsz = 2;
    } else {
      if (n < 3) return kZCorrupt;
      regen = (b0 >> 4) + ((int64_t)src[bstart + 1] << 4) + ((int64_t)src[bstart + 2] << 12);
      hsz = 3;
    }
  } else {
    if (sf == 0 || sf == 1) {
      if (n < 3) return kZCorrupt;
      const uint32_t v = src[bstart] | (src[bstart + 1] << 8) | (src[bstart + 2] << 16);
      regen = (v >> 4) & 0x3FF;
      csize = (v >> 14) & 0x3FF;
      hsz = 3;
      streams = sf == 0 ? 1 : 4;
    } else if (sf == 2) {
      if (n < 4) return kZCorrupt;
      const uint32_t v =
          src[bstart] | (src[bstart + 1] << 8) | (src[bstart + 2] << 16) | ((uint32_t)src[bstart + 3] << 24);
      regen = (v >> 4) & 0x3FFF;
      csize = (v >> 18) & 0x3FFF;
      hsz = 4;
      streams = 4;
    } else {
      if (n < 5) return kZCorrupt;
      const uint64_t v = (uint64_t)(src[bstart] | (src[bstart + 1] << 8) | (src[bstart + 2] << 16) |
                                    ((uint32_t)src[bstart + 3] << 24)) |
                         ((uint64_t)src[bstart + 4] << 32);
      regen = (v >> 4) & 0x3FFFF;
      csize = (v >> 22) & 0x3FFFF;
      hsz = 5;
      streams = 4;
    }
  }
  if (regen > kZBlockMax) return kZCorrupt;
  pos = hsz;
  if (lt == 0) {
    if (pos + regen > n) return kZCorrupt;
    if (regen > max_regen) return kZSlow;
    for (int64_t k = l; k < regen; k += 64) z.lit[k] = src[bstart + pos + k];
    pos += regen;
  } else if (lt == 1) {
    if (pos + 1 > n) return kZCorrupt;
    if (regen > max_regen) return kZSlow;
    const uint8_t v = src[bstart + pos];
    for (int64_t k = l; k < regen; k += 64) z.lit[k] = v;
    pos += 1;
  } else {
    if (pos + csize > n) return kZCorrupt;
    int64_t hs = bstart + pos, hn = csize;
    if (lt == 2) {
      int mb = 0, k = 0;
      const uint8_t *dsc = z_stage(L, src, hs, hn);  // the tree description: < 129 bytes
      if (l == 0) k = z_huf_read(L, &mb, dsc, 0, hn < kZDesc ? hn : kZDesc);
      k = zbcast(L, 0, k);
      mb = zbcast(L, 1, mb);
      if (k < 0) return kZCorrupt;
      z.have_huf = 1;
      z.max_bits = mb;
      hs += k;
      hn -= k;
    } else if (!z.have_huf) {
      return kZCorrupt;
    }
    bool ok;
    if (streams == 1) {
      if (regen > max_regen) return kZSlow;
      const int sy = z_huf_sync(L, z.max_bits, src, hs, hn, 1, z.lit, 0, regen);
      ok = sy > 0 || (sy < 0 && z_huf_streams(L, z.max_bits, src, hs, hn, 1, z.lit, 0, regen));
    } else {
      if (hn < 6) return kZCorrupt;
      const int64_t s1 = src[hs] | (src[hs + 1] << 8), s2 = src[hs + 2] | (src[hs + 3] << 8),
                    s3 = src[hs + 4] | (src[hs + 5] << 8);
      if (6 + s1 + s2 + s3 > hn) return kZCorrupt;
      const int64_t s4 = hn - 6 - s1 - s2 - s3;
      const int64_t seg = (regen + 3) / 4;
      if (3 * seg > regen) return kZCorrupt;
      if (regen > max_regen) return kZSlow;
      // the four streams at once, one lane each (the oracle stops at the first
      // bad stream; any failure is the same error)
      const int64_t st = hs + 6 + (l > 0 ? s1 : 0) + (l > 1 ? s2 : 0) + (l > 2 ? s3 : 0);
      const int64_t sn = l == 0 ? s1 : l == 1 ? s2 : l == 2 ? s3 : s4;
      const int64_t cnt = l < 3 ? seg : regen - 3 * seg;
      const int sy = z_huf_sync(L, z.max_bits, src, st, sn, 4, z.lit, seg, cnt);
      ok = sy > 0 || (sy < 0 && z_huf_streams(L, z.max_bits, src, st, sn, 4, z.lit, seg, cnt));
    }
    if (!ok) return kZCorrupt;
    pos += csize;
  }
  regen_out = regen;
  return 0;
}

// Sequences section header and its three FSE tables (lane 0 builds them into
// L): nseq, pos advanced to the sequence bitstream.
// FSE decoding table by the whole wave (round 3; z_fse_build's cells): lane 0
// walking the 512 cells twice -- the spread, then each cell's state from a
// per-symbol counter in LDS -- was over half of k_zstd_ent. Here (1) the
// low-probability symbols take the top cells by a ballot rank; (2) the spread
// writes the k-th symbol occurrence (symbols in order, norm[s] each) to the k-th
// valid cell of the sequence i * step mod size (valid: below the low symbols),
// k from a ballot prefix over i, the symbol of k by binary search of the
// counts' inclusive prefix; (3) a cell's occurrence number within its symbol
// comes from ballots over the 64 cells of a chunk, one per distinct symbol,
// with per-symbol running counts. False: the counts do not fill the table.
// cum / cnt: 64 u16 of LDS scratch each.
__device__ bool z_fse_build_wave(uint32_t *t, const int16_t *norm, int max_sym, int log, uint16_t *cum,
                                 uint16_t *cnt) {
  const int l = lane_id();
  const uint32_t size = 1u << log, mask = size - 1;
  const unsigned long long lt = (1ull << l) - 1;
  const int nv = l <= max_sym ? norm[l] : 0;
  const bool low = l <= max_sym && nv == -1;
  const unsigned long long ml = __ballot(low);
  const uint32_t nlow = (uint32_t)__popcll(ml);
  if (low) t[size - 1 - (uint32_t)__popcll(ml & lt)] = (uint32_t)l;
  const uint32_t high = size - 1 - nlow;
  const uint32_t pc = nv > 0 ? (uint32_t)nv : 0u;
  const uint32_t incl = wave_incl_sum_dpp(pc);
  if ((uint32_t)__builtin_amdgcn_readlane(incl, 63) != high + 1) return false;
  cum[l] = (uint16_t)incl;
  cnt[l] = (uint16_t)(low ? 1 : nv);  // the next state's counter (FSE's symbolNext)
  zsync();
  const uint32_t step = (size >> 1) + (size >> 3) + 3;
  uint32_t carry = 0;
  for (uint32_t i0 = 0; i0 < size; i0 += 64) {
    const uint32_t i = i0 + (uint32_t)l, q = (i * step) & mask;
    const bool v = i < size && q <= high;
    const unsigned long long m = __ballot(v);
    const uint32_t k = carry + (uint32_t)__popcll(m & lt);
    carry += (uint32_t)__popcll(m);
    if (v) {  // the first symbol whose inclusive count passes k
      int lo_s = 0, hi_s = max_sym;
      while (lo_s < hi_s) {
        const int mid = (lo_s + hi_s) >> 1;
        if (cum[mid] > k) hi_s = mid;
        else lo_s = mid + 1;
      }
      t[q] = (uint32_t)lo_s;
    }
  }
  zsync();
  for (uint32_t u0 = 0; u0 < size; u0 += 64) {
    const uint32_t u = u0 + (uint32_t)l;
    const bool in = u < size;
    const uint32_t sym = in ? (t[u] & 0xffu) : 0xffffu;
    unsigned long long left = __ballot(in);
    uint32_t ns = 0;
    while (left) {
      const uint32_t s0 = (uint32_t)__builtin_amdgcn_readlane((int)sym, __ffsll((long long)left) - 1);
      const unsigned long long m = __ballot(in && sym == s0);
      const uint32_t c = cnt[s0];
      if (in && sym == s0) ns = c + (uint32_t)__popcll(m & lt);
      zsync();
      if (l == 0) cnt[s0] = (uint16_t)(c + (uint32_t)__popcll(m));
      zsync();
      left &= ~m;
    }
    if (in) {
      const int nb = log - highbit(ns);
      t[u] = sym | ((uint32_t)nb << 8) | (((ns << nb) - size) << 16);
    }
  }
  zsync();
  return true;
}

__device__ uint32_t z_seq_header(ZFrame &z, ZLds &L, int64_t bstart, int64_t n, int64_t &pos, int64_t &nseq_out) {
  const int l = lane_id();
  const uint8_t *src = z.src;
  if (pos >= n) return kZCorrupt;
  int64_t nseq;
  const uint32_t c0 = src[bstart + pos];
  if (c0 == 0) {
    nseq = 0;
    pos += 1;
  } else if (c0 < 128) {
    nseq = c0;
    pos += 1;
  } else if (c0 < 255) {
    if (pos + 2 > n) return kZCorrupt;
    nseq = ((int64_t)(c0 - 128) << 8) + src[bstart + pos + 1];
    pos += 2;
  } else {
    if (pos + 3 > n) return kZCorrupt;
    nseq = src[bstart + pos + 1] + ((int64_t)src[bstart + pos + 2] << 8) + 0x7F00;
    pos += 3;
  }
  nseq_out = nseq;
  if (nseq == 0) return 0;
  if (pos >= n) return kZCorrupt;
  const int modes = src[bstart + pos++];
  if (modes & 3) return kZCorrupt;
  // tables: lane 0 builds them from the staged descriptions (three NCounts:
  // < 300 bytes together), every lane learns the bytes used / a failure
  const int64_t sn = n - pos < kZDesc ? n - pos : kZDesc;
  const uint8_t *dsc = ((modes >> 2) & 0x3f) ? z_stage(L, src, bstart + pos, n - pos) : nullptr;
  // per table (z_seq_table's modes): lane 0 reads the description (predefined
  // counts, RLE symbol, NCount or repeat), the wave builds the decoding table
  uint16_t *cum = reinterpret_cast<uint16_t *>(L.hout[0]), *cnt = reinterpret_cast<uint16_t *>(L.hout[1]);
  int64_t at = 0;
  auto table = [&](uint32_t *t, int &have, int &logv, int mode, const int16_t *def, int def_log, int max_sym,
                   int max_log) -> bool {
    int k = 0, ms = max_sym, lg = logv, build = 0;
    if (l == 0) {
      if (mode == 0) {
        for (int q = 0; q <= max_sym; q++) L.norm[q] = def[q];
        lg = def_log;
        build = 1;
      } else if (mode == 1) {
        if (sn - at < 1 || dsc[at] > max_sym) {
          k = -1;
        } else {
          t[0] = dsc[at];  // log 0: nbits 0, base 0
          lg = 0;
          k = 1;
        }
      } else if (mode == 2) {
        k = z_read_ncount(L.norm, &ms, &lg, dsc + at, sn - at, max_log);
        if (k > sn - at) k = -1;
        build = k >= 0;
      } else if (!have) {
        k = -1;
      }
    }
    k = zbcast(L, 0, k);
    ms = zbcast(L, 1, ms);
    lg = zbcast(L, 2, lg);
    build = zbcast(L, 3, build);
    if (build && !z_fse_build_wave(t, L.norm, ms, lg, cum, cnt)) k = -1;
    if (k < 0) return false;
    if (mode != 3) {
      have = 1;
      logv = lg;
    }
    at += k;
    return true;
  };
  if (!table(L.ll, z.have_ll, z.ll_log, (modes >> 6) & 3, kLLDef, 6, 35, 9) ||
      !table(L.of, z.have_of, z.of_log, (modes >> 4) & 3, kOFDef, 5, 31, 8) ||
      !table(L.ml, z.have_ml, z.ml_log, (modes >> 2) & 3, kMLDef, 6, 52, 9))
    return kZCorrupt;
  pos += at;
  return 0;
}

// FSE sequence decoder (wave-uniform state)
struct ZSeqDec {
  ZSeqBr r;
  uint32_t sll, sof, sml;
};
__device__ __forceinline__ uint32_t z_seq_start(ZSeqDec &q, const ZFrame &z, ZLds &L, int64_t start, int64_t n) {
  if (!q.r.init(z.src, start, n, L.sring)) return kZCorrupt;
  q.sll = q.r.read(z.ll_log);
  q.sof = q.r.read(z.of_log);
  q.sml = q.r.read(z.ml_log);
  return 0;
}
// the next sequence (oracle decode_block's loop body up to execute): ll, ml and
// the resolved offset; `more`: another sequence follows (the states advance)
__device__ __forceinline__ uint32_t z_seq_next(ZSeqDec &q, ZFrame &z, ZLds &L, bool more, uint64_t &ll,
                                               uint64_t &ml, uint64_t &off) {
  const uint32_t cll = uni(L.ll[q.sll]), cml = uni(L.ml[q.sml]), cof = uni(L.of[q.sof]);
  const uint32_t llc = cll & 0xff, mlc = cml & 0xff, ofc = cof & 0xff;
  if (llc > 35 || mlc > 52 || ofc > 31) return kZCorrupt;
  const uint64_t ofv = (1ull << ofc) + q.r.read((int)ofc);
  const uint32_t mlx = kZCodes.ml[mlc], llx = kZCodes.ll[llc];
  ml = (mlx & 0xFFFFFFu) + q.r.read((int)(mlx >> 24));
  ll = (llx & 0xFFFFFFu) + q.r.read((int)(llx >> 24));
  if (ofv > 3) {
    off = ofv - 3;
    z.rep2 = z.rep1;
    z.rep1 = z.rep0;
    z.rep0 = off;
  } else {
    const uint64_t idx = ofv + (ll == 0 ? 1 : 0);
    if (idx == 1) {
      off = z.rep0;
    } else if (idx == 2) {
      off = z.rep1;
      z.rep1 = z.rep0;
      z.rep0 = off;
    } else if (idx == 3) {
      off = z.rep2;
      z.rep2 = z.rep1;
      z.rep1 = z.rep0;
      z.rep0 = off;
    } else {
      off = z.rep0 - 1;
      if (off == 0) return kZCorrupt;
      z.rep2 = z.rep1;
      z.rep1 = z.rep0;
      z.rep0 = off;
    }
  }
  if (more) {
    q.sll = (cll >> 16) + q.r.read((cll >> 8) & 0xff);
    q.sml = (cml >> 16) + q.r.read((cml >> 8) & 0xff);
    q.sof = (cof >> 16) + q.r.read((cof >> 8) & 0xff);
  }
  if (q.r.overrun()) return kZCorrupt;
  return 0;
}

// ---------------------------------------------------------------- serial path
// Execute one sequence (the oracle's "execute"): the literal run from the
// literal buffer, then the match copy from the frame's output, the whole
// wave cooperating. Returns 0 or a ZErr.
__device__ __forceinline__ uint32_t z_exec(ZFrame &z, uint64_t ll, uint64_t ml, uint64_t off, int64_t &lit_pos,
                                           int64_t regen) {
  const int l = lane_id();
  if (lit_pos + (int64_t)ll > regen) return kZCorrupt;
  if (z.olen + (int64_t)(ll + ml) > z.cap) return kZFull;
  for (uint64_t k = l; k < ll; k += 64) z.out[z.olen + k] = z.lit[lit_pos + k];
  z.olen += (int64_t)ll;
  lit_pos += (int64_t)ll;
  const int64_t produced = z.olen - z.frame_start;
  if (off == 0 || (int64_t)off > produced) return kZCorrupt;
  if (ml) {
    zmem_sync();
    const int64_t s0 = z.olen - (int64_t)off;
    for (uint64_t k0 = 0; k0 < ml; k0 += 64) {
      const uint64_t k = k0 + l;
      // a match may overlap itself: byte k repeats byte k mod off
      const uint64_t kk = off >= ml ? k : k % off;
      uint8_t v = 0;
      if (k < ml) v = z.out[s0 + kk];
      if (k < ml) z.out[z.olen + k] = v;
    }
    z.olen += (int64_t)ml;
    zmem_sync();
  }
  return 0;
}

// XXH64 (below)
__device__ uint64_t z_xxh64(const uint8_t *p, uint64_t len);

// The serial decoder's frame content: output written straight to the decode
// region (k_zstd, the exact path for blocks the fast path declines).
struct ZSerialSink {
  __device__ uint32_t raw(ZFrame &z, int64_t at, int64_t size) {
    if (z.olen + size > z.cap) return kZFull;
    for (int64_t k = lane_id(); k < size; k += 64) z.out[z.olen + k] = z.src[at + k];
    z.olen += size;
    zmem_sync();
    return 0;
  }
  __device__ uint32_t rle(ZFrame &z, uint8_t v, int64_t size) {
    if (z.olen + size > z.cap) return kZFull;
    for (int64_t k = lane_id(); k < size; k += 64) z.out[z.olen + k] = v;
    z.olen += size;
    zmem_sync();
    return 0;
  }
  // one compressed block (oracle decode_block)
  __device__ uint32_t block(ZFrame &z, ZLds &L, int64_t bstart, int64_t n) {
    const int l = lane_id();
    int64_t pos = 0, regen = 0, nseq = 0;
    uint32_t e = z_literals(z, L, bstart, n, pos, regen, kZBlockMax);
    if (e) return e;
    zmem_sync();
    e = z_seq_header(z, L, bstart, n, pos, nseq);
    if (e) return e;
    int64_t lit_pos = 0;
    if (nseq > 0) {
      ZSeqDec q;
      if ((e = z_seq_start(q, z, L, bstart + pos, n - pos))) return e;
      for (int64_t i = 0; i < nseq; i++) {
        uint64_t ll, ml, off;
        if ((e = z_seq_next(q, z, L, i + 1 < nseq, ll, ml, off))) return e;
        if ((e = z_exec(z, ll, ml, off, lit_pos, regen))) return e;
      }
      if (!q.r.exact()) return kZCorrupt;
    }
    // remaining literals
    if (z.olen + (regen - lit_pos) > z.cap) return kZFull;
    for (int64_t k = l; k < regen - lit_pos; k += 64) z.out[z.olen + k] = z.lit[lit_pos + k];
    z.olen += regen - lit_pos;
    zmem_sync();
    return 0;
  }
  __device__ void frame_begin(ZFrame &) {}
  __device__ uint32_t frame_fcs(ZFrame &z, int64_t fcs) {
    return (fcs >= 0 && z.olen - z.frame_start != fcs) ? kZCorrupt : 0u;
  }
  __device__ uint32_t frame_end(ZFrame &z, bool checksum, uint32_t want) {
    if (!checksum) return 0;
    const uint32_t got = (uint32_t)z_xxh64(z.out + z.frame_start, (uint64_t)(z.olen - z.frame_start));
    return want != got ? kZChecksum : 0;
  }
};

// ---------------------------------------------------------------- fast path: jobs
// The fast path turns every zstd block of a recordio block into a job
// (k_zstd_ent: frame walk, literals, table descriptions), decodes every job's
// sequence bitstream in its own lane (k_zstd_seq: one vector instruction
// advances 64 jobs), then -- in file order, one wave per recordio block --
// resolves repeat offsets, checks every sequence and writes the execution
// entries (k_zstd_fix). A job's header, its three FSE tables and its raw
// sequences sit
// in the second half of the block's scratch region; DevBufs::zjob lists the
// headers.
//
// Execution entries (u64, k_zstd_fix -> k_zstd_exec): literal count (bits
// 15:0), match length (31:16), offset (63:32); literal runs and matches are
// split so that each is at most kZPiece bytes (copying a long match in pieces
// with the same offset is the same copy). Frame ends are marked: ll = 0xFFFF
// with ml = 0xFFFF (checksum = offset field) or 0xFFFE (no checksum).
#ifndef RIO_ZPIECE
#define RIO_ZPIECE 2048
#endif
constexpr uint32_t kZPiece = RIO_ZPIECE;
constexpr uint32_t kZMark = 0xFFFF;
constexpr uint32_t kZMarkCk = 0xFFFF, kZMarkNoCk = 0xFFFE;

struct ZJob {
  uint64_t seq_off;         // sequence bitstream (byte offset from d.tok)
  uint32_t seq_len, nseq;
  uint32_t regen, flags;    // the block's literals; kJ*
  uint32_t checksum, logs;  // frame checksum (kJCk); ll_log | of_log << 8 | ml_log << 16
  int64_t fcs;              // frame content size, at the frame's last job (-1: none)
  uint64_t tab_off;         // ll, ml, of cells (u32 x 2^log each)
  uint64_t raw_off;         // raw sequences (u64 x nseq): ll | ml << 17 | offset value << 35
  uint64_t next;            // the block's next job header
  uint32_t err, pad;        // k_zstd_seq: 0, kZCorrupt or kZSlow
};
constexpr int64_t kZJobHdr = (sizeof(ZJob) + 15) / 16 * 16;  // header bytes; 16-aligned tables follow
constexpr uint32_t kJFirst = 1, kJLast = 2, kJCk = 4, kJLit = 8;

// k_zstd_ent's frame content: literals into the literal area, every zstd
// block a job (raw / RLE blocks are literal-only jobs)
struct ZJobSink {
  uint8_t *tok8;           // d.tok as bytes
  uint64_t region;         // this block's scratch region (offset from d.tok)
  int64_t lit_w, half;     // next literal byte; the first half's end (region offsets)
  int64_t job_w, job_end;  // next job; region end
  int64_t last;            // the last job's header (-1: none)
  uint32_t njobs, pend_first;
  unsigned long long *zjob;
  uint64_t zjob_cap;
  Ctl *ctl;

  __device__ __forceinline__ ZJob *hdr(int64_t at) const { return reinterpret_cast<ZJob *>(tok8 + region + at); }
  // a job with tabsz bytes of tables and nseq raw sequences: its region offset, or -1
  __device__ int64_t new_job(int64_t tabsz, int64_t nseq, uint32_t regen, uint32_t flags) {
    const int64_t tabr = (tabsz + 15) & ~15ll;
    const int64_t need = (kZJobHdr + tabr + 8 * nseq + 15) & ~15ll;  // raw entries are stored 16 B at a time
    if (job_w + need > job_end) return -1;
    unsigned long long idx = 0;
    if (lane_id() == 0) idx = atomicAdd(&ctl->zjob_n, 1ull);
    idx = uni64(idx);
    if (idx >= zjob_cap) return -1;
    const int64_t at = job_w;
    job_w += need;
    if (lane_id() == 0) {
      zjob[idx] = region + (uint64_t)at;
      ZJob *h = hdr(at);
      h->seq_off = 0;
      h->seq_len = 0;
      h->nseq = (uint32_t)nseq;
      h->regen = regen;
      h->flags = flags | (pend_first ? kJFirst : 0u);
      h->checksum = 0;
      h->logs = 0;
      h->fcs = -1;
      h->tab_off = region + (uint64_t)(at + kZJobHdr);
      h->raw_off = region + (uint64_t)(at + kZJobHdr + tabr);
      h->next = 0;
      h->err = 0;
      h->pad = 0;
      if (last >= 0) hdr(last)->next = region + (uint64_t)at;
    }
    pend_first = 0;
    last = at;
    njobs++;
    return at;
  }
  __device__ void frame_begin(ZFrame &) { pend_first = 1; }
  __device__ uint32_t frame_fcs(ZFrame &, int64_t fcs) {  // checked by k_zstd_fix (the output size is its)
    if (lane_id() == 0) {
      ZJob *h = hdr(last);
      h->flags |= kJLast;
      h->fcs = fcs;
    }
    return 0;
  }
  __device__ uint32_t frame_end(ZFrame &, bool checksum, uint32_t want) {
    if (checksum && lane_id() == 0) {
      ZJob *h = hdr(last);
      h->flags |= kJCk;
      h->checksum = want;
    }
    return 0;
  }
  __device__ uint32_t lits(const uint8_t *from, uint8_t v, int64_t size) {  // raw (from) / RLE (v)
    if (lit_w + size + 64 > half) return kZSlow;
    if (new_job(0, 0, (uint32_t)size, kJLit) < 0) return kZSlow;
    uint8_t *dst = tok8 + region + lit_w;
    for (int64_t k = lane_id(); k < size; k += 64) dst[k] = from ? from[k] : v;
    lit_w += size;
    return 0;
  }
  __device__ uint32_t raw(ZFrame &z, int64_t at, int64_t size) { return lits(z.src + at, 0, size); }
  __device__ uint32_t rle(ZFrame &, uint8_t v, int64_t size) { return lits(nullptr, v, size); }
  __device__ uint32_t block(ZFrame &z, ZLds &L, int64_t bstart, int64_t n) {
    int64_t pos = 0, regen = 0, nseq = 0;
    z.lit = tok8 + region + lit_w;
    ZPROF_T(t0);
    uint32_t e = z_literals(z, L, bstart, n, pos, regen, half - 64 - lit_w);
    if (e) return e;
    ZPROF_ADD(0, t0);
    ZPROF_T(t1);
    e = z_seq_header(z, L, bstart, n, pos, nseq);
    if (e) return e;
    ZPROF_ADD(1, t1);
    const int nll = 1 << z.ll_log, nml = 1 << z.ml_log, nof = 1 << z.of_log;
    const int64_t tabsz = nseq ? 4 * (int64_t)(nll + nml + nof) : 0;
    const int64_t at = new_job(tabsz, nseq, (uint32_t)regen, 0);
    if (at < 0) return kZSlow;
    if (nseq) {
      if (lane_id() == 0) {
        ZJob *h = hdr(at);
        h->seq_off = region + (uint64_t)(bstart + pos);
        h->seq_len = (uint32_t)(n - pos);
        h->logs = (uint32_t)z.ll_log | ((uint32_t)z.of_log << 8) | ((uint32_t)z.ml_log << 16);
      }
      uint32_t *tll = reinterpret_cast<uint32_t *>(tok8 + region + at + kZJobHdr), *tml = tll + nll, *tof = tml + nml;
      for (int u = lane_id(); u < nll; u += 64) tll[u] = L.ll[u];
      for (int u = lane_id(); u < nml; u += 64) tml[u] = L.ml[u];
      for (int u = lane_id(); u < nof; u += 64) tof[u] = L.of[u];
    }
    lit_w += regen;
    return 0;
  }
};

// ---------------------------------------------------------------- XXH64
constexpr uint64_t kP1 = 0x9E3779B185EBCA87ull, kP2 = 0xC2B2AE3D27D4EB4Full, kP3 = 0x165667B19E3779F9ull,
                   kP4 = 0x85EBCA77C2B2AE63ull, kP5 = 0x27D4EB2F165667C5ull;
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t in) { return rotl64(acc + in * kP2, 31) * kP1; }
__device__ __forceinline__ uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * kP1 + kP4; }
__device__ __forceinline__ uint64_t zrd64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}
// XXH64(p, len, 0): every lane computes it (the frame's output is in HBM)
__device__ uint64_t z_xxh64(const uint8_t *p, uint64_t len) {
  const uint8_t *end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = kP1 + kP2, v2 = kP2, v3 = 0, v4 = 0 - kP1;
    const uint8_t *limit = end - 32;
    do {
      v1 = xround(v1, zrd64(p));
      v2 = xround(v2, zrd64(p + 8));
      v3 = xround(v3, zrd64(p + 16));
      v4 = xround(v4, zrd64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xmerge(h, v1);
    h = xmerge(h, v2);
    h = xmerge(h, v3);
    h = xmerge(h, v4);
  } else {
    h = kP5;
  }
  h += len;
  while (p + 8 <= end) {
    h ^= xround(0, zrd64(p));
    h = rotl64(h, 27) * kP1 + kP4;
    p += 8;
  }
  if (p + 4 <= end) {
    const uint64_t v = (uint64_t)p[0] | ((uint64_t)p[1] << 8) | ((uint64_t)p[2] << 16) | ((uint64_t)p[3] << 24);
    h ^= v * kP1;
    h = rotl64(h, 23) * kP2 + kP3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * kP5;
    h = rotl64(h, 11) * kP1;
    p++;
  }
  h ^= h >> 33;
  h *= kP2;
  h ^= h >> 29;
  h *= kP3;
  h ^= h >> 32;
  return h;
}

}  // namespace rio
#include "zstd_exact.h"
namespace rio {

// ---------------------------------------------------------------- frame
__device__ __forceinline__ uint32_t zrd16(const uint8_t *p, int64_t i) { return p[i] | ((uint32_t)p[i + 1] << 8); }
__device__ __forceinline__ uint32_t zrd24(const uint8_t *p, int64_t i) { return zrd16(p, i) | ((uint32_t)p[i + 2] << 16); }
__device__ __forceinline__ uint32_t zrd32(const uint8_t *p, int64_t i) { return zrd16(p, i) | (zrd16(p, i + 2) << 16); }

// one frame at src[in, in + n) (oracle decode_frame): bytes consumed, or -(ZErr)
template <class Sink>
__device__ int64_t z_decode_frame(ZFrame &z, ZLds &L, Sink &k, int64_t in, int64_t n) {
  const uint8_t *src = z.src;
  if (n < 4) return -(int64_t)kZSrc;
  const uint32_t magic = zrd32(src, in);
  if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
    if (n < 8) return -(int64_t)kZSrc;
    const uint64_t sz = zrd32(src, in + 4);
    if (8 + (int64_t)sz > n) return -(int64_t)kZSrc;
    return 8 + (int64_t)sz;
  }
  if (magic != kZMagic) return -(int64_t)kZPrefix;
  int64_t pos = 4;
  if (pos >= n) return -(int64_t)kZSrc;
  const int fhd = src[in + pos++];
  const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, reserved = (fhd >> 3) & 1, checksum = (fhd >> 2) & 1;
  const int did_flag = fhd & 3;
  if (reserved) return -(int64_t)kZNotSup;
  uint64_t window = 0;
  if (!single) {
    if (pos >= n) return -(int64_t)kZSrc;
    const int wd = src[in + pos++];
    const int wlog = 10 + (wd >> 3);
    if (wlog > 31) return -(int64_t)kZWindow;
    const uint64_t base = 1ull << wlog;
    window = base + (base / 8) * (uint64_t)(wd & 7);
  }
  const int did_len = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
  if (pos + did_len > n) return -(int64_t)kZSrc;
  uint64_t did = 0;
  for (int i = 0; i < did_len; i++) did |= (uint64_t)src[in + pos + i] << (8 * i);
  pos += did_len;
  if (did != 0) return -(int64_t)kZDict;
  const int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : (fcs_flag == 2 ? 4 : 8));
  if (pos + fcs_len > n) return -(int64_t)kZSrc;
  int64_t fcs = -1;
  if (fcs_len == 1) fcs = src[in + pos];
  else if (fcs_len == 2) fcs = zrd16(src, in + pos) + 256;
  else if (fcs_len == 4) fcs = zrd32(src, in + pos);
  else if (fcs_len == 8) fcs = (int64_t)(zrd32(src, in + pos) | ((uint64_t)zrd32(src, in + pos + 4) << 32));
  pos += fcs_len;
  if (single) window = (uint64_t)fcs;
  const uint64_t block_max = window < (uint64_t)kZBlockMax ? window : (uint64_t)kZBlockMax;
  z.frame_start = z.olen;
  z.have_huf = z.have_ll = z.have_of = z.have_ml = 0;
  z.rep0 = 1;
  z.rep1 = 4;
  z.rep2 = 8;
  k.frame_begin(z);
  for (;;) {
    if (pos + 3 > n) return -(int64_t)kZSrc;
    const uint32_t bh = zrd24(src, in + pos);
    pos += 3;
    const int last = bh & 1, type = (bh >> 1) & 3;
    const uint64_t size = bh >> 3;
    if (type == 3) return -(int64_t)kZCorrupt;
    if (size > block_max) return -(int64_t)kZCorrupt;
    uint32_t e;
    if (type == 0) {
      if (pos + (int64_t)size > n) return -(int64_t)kZSrc;
      e = k.raw(z, in + pos, (int64_t)size);
      pos += (int64_t)size;
    } else if (type == 1) {
      if (pos + 1 > n) return -(int64_t)kZSrc;
      e = k.rle(z, src[in + pos], (int64_t)size);
      pos += 1;
    } else {
      if (pos + (int64_t)size > n) return -(int64_t)kZSrc;
      e = k.block(z, L, in + pos, (int64_t)size);
      pos += (int64_t)size;
    }
    if (e) return -(int64_t)e;
    if (last) break;
  }
  if (const uint32_t ef = k.frame_fcs(z, fcs)) return -(int64_t)ef;
  uint32_t want = 0;
  if (checksum) {
    if (pos + 4 > n) return -(int64_t)kZSrc;
    want = zrd32(src, in + pos);
    pos += 4;
  }
  const uint32_t e = k.frame_end(z, checksum != 0, want);
  if (e) return -(int64_t)e;
  return pos;
}

// An upper bound of the block's decoded size from its frame and block headers
// alone (the retry's region when a block outgrew its first bound): raw and RLE
// blocks regenerate exactly their size, a compressed block at most
// min(window, 128 KiB). -1 if the headers do not parse (then the block's
// decode error is what the retry reports).
__device__ int64_t z_size_bound(const uint8_t *src, int64_t n) {
  int64_t pos = 0, total = 0;
  while (pos < n) {
    if (n - pos < 4) return -1;
    const uint32_t magic = zrd32(src, pos);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
      if (n - pos < 8) return -1;
      pos += 8 + (int64_t)zrd32(src, pos + 4);
      continue;
    }
    if (magic != kZMagic || n - pos < 5) return -1;
    const int fhd = src[pos + 4];
    const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
    const int did_len = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
    const int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : (fcs_flag == 2 ? 4 : 8));
    int64_t p = pos + 5;
    uint64_t window = 0;
    if (!single) {
      if (p >= n) return -1;
      const int wd = src[p++];
      const int wlog = 10 + (wd >> 3);
      if (wlog > 31) return -1;
      window = (1ull << wlog) + ((1ull << wlog) / 8) * (uint64_t)(wd & 7);
    }
    p += did_len;
    if (p + fcs_len > n) return -1;
    if (single) {
      if (fcs_len == 1) window = src[p];
      else if (fcs_len == 2) window = zrd16(src, p) + 256;
      else if (fcs_len == 4) window = zrd32(src, p);
      else window = zrd32(src, p) | ((uint64_t)zrd32(src, p + 4) << 32);
    }
    p += fcs_len;
    const int64_t block_max = window < (uint64_t)kZBlockMax ? (int64_t)window : kZBlockMax;
    for (;;) {
      if (p + 3 > n) return -1;
      const uint32_t bh = zrd24(src, p);
      p += 3;
      const int type = (bh >> 1) & 3;
      const int64_t size = bh >> 3;
      if (type == 3) return -1;
      total += type == 2 ? block_max : size;
      p += type == 1 ? 1 : size;
      if (p > n) return -1;
      if (bh & 1) break;
    }
    pos = p + (checksum ? 4 : 0);
  }
  return total;
}

// logical compressed dword at byte p (a multiple of 4) of a block's chunk
// payloads; bytes at/after n read 0
__device__ __forceinline__ uint32_t z_flat_dword(const uint8_t *span, const unsigned long long *ck_pay, uint64_t c0,
                                                 uint64_t total, uint64_t pay0, uint64_t n, bool regular, uint64_t p) {
  if (p >= n) return 0u;
  uint32_t v = 0;
  if (regular) {  // 32,740 B payloads: a dword never crosses a chunk
    const uint64_t j = p / kMaxPayload;
    v = *reinterpret_cast<const uint32_t *>(span + (c0 + j) * kChunk + kChunkHdr + (p - j * kMaxPayload));
  } else {
    for (int i = 0; i < 4; i++) {
      const uint64_t q = p + i;
      if (q >= n) break;
      uint64_t a = c0, b = c0 + total;
      while (b - a > 1) {
        const uint64_t m = (a + b) >> 1;
        if (ck_pay[m] - pay0 <= q) a = m;
        else b = m;
      }
      v |= (uint32_t)span[a * kChunk + kChunkHdr + (q - (ck_pay[a] - pay0))] << (8 * i);
    }
  }
  if (p + 4 > n) v &= 0xffffffffu >> (8 * (uint32_t)(p + 4 - n));
  return v;
}

enum ZsMode : uint32_t {
  kZsSkip = 0,   // nothing to decode (not a transformed block, error already reported, capacity retry)
  kZsExec = 1,   // entries ready for k_zstd_exec
  kZsErrCk = 2,  // entropy error after checksummed frames: k_zstd_exec checks those first
  kZsSlow = 3,   // scratch too small for the fast path: k_zstd (serial) decodes it
  kZsJobs = 4,   // jobs made (k_zstd_ent): k_zstd_seq / k_zstd_fix finish them
};

__device__ __forceinline__ void z_init(ZFrame &z, const uint8_t *src, uint8_t *out, int64_t cap, uint8_t *lit) {
  z.src = src;
  z.out = out;
  z.cap = cap;
  z.olen = 0;
  z.frame_start = 0;
  z.lit = lit;
  z.max_bits = 0;
  z.have_huf = z.have_ll = z.have_of = z.have_ml = 0;
  z.ll_log = z.of_log = z.ml_log = 0;
  z.rep0 = 1;
  z.rep1 = 4;
  z.rep2 = 8;
}

// flattenIov: block b's chunk payloads back to back at the start of its token
// region (+8 zero bytes); false if the block is not decoded by the caller
// (state and status written here)
__device__ __forceinline__ void z_flatten(const uint8_t *span, const DevBufs &d, uint64_t c0, unsigned long long meta,
                                          uint64_t n, uint32_t *flat) {
  const int l = lane_id();
  const uint64_t total = meta & kMetaTotalMask, pay0 = uni64(d.ck_pay[c0]);
  const bool regular = (meta & kMetaRegular) != 0;
  for (uint64_t p = 4 * (uint64_t)l; p < n + 8; p += 256)
    flat[p >> 2] = z_flat_dword(span, d.ck_pay, c0, total, pay0, n, regular, p);
  zmem_sync();
}

// ---------------------------------------------------------------- k_zstd_size
// Region sizing, thread per block, from the block's headers alone -- frame
// headers, zstd block headers, each compressed block's literals-section header
// (Regenerated_Size) and the sequences-section header (Number_of_Sequences),
// RFC 8878 3.1.1, 3.1.1.3.1.1, 3.1.1.3.2.1; no entropy decode:
// - the decode region: Frame_Content_Size where every frame declares it (the
//   writer's single-shot ZSTD_compress does, recordiozstd.go:31-38), else each
//   compressed block's bound min(window, 128 KiB); a frame whose content exceeds
//   its declared size is found by the passes and retried at its exact size
//   (blk_need) as before;
// - the scratch region the fast passes fill: the flattened input, the literal
//   area (every block's literals), the execution entries k_zstd_fix reserves
//   (sequences + pieces of runs over kZPiece + per-job / per-frame marks, its
//   own 8 * (... + 132) check), and the jobs (ZJobSink::new_job: header, tables
//   of at most 4 * (512 + 512 + 256) bytes, 8 B per raw sequence) -- or the
//   serial decoder's (input + zx::State), if larger.
// Regions are then placed back to back by an exclusive scan (blk_zoff): a C4
// block needs ~4x its compressed bytes, against the previous fixed 512 KiB per
// input chunk (16x the span). Every writer still checks its region's limits
// (lits / new_job / k_zstd_fix's entry check -> the serial path), so a header
// this walk cannot parse gets a generous region and the passes decide.
struct ZSzIn {
  const uint8_t *span;
  const unsigned long long *ck_pay;
  uint64_t c0, total, pay0, n;
  bool regular;
  __device__ __forceinline__ uint32_t b(uint64_t p) const {  // logical byte p (0 at/after n)
    if (p >= n) return 0u;
    if (regular) {
      const uint64_t j = p / kMaxPayload;
      return span[(c0 + j) * kChunk + kChunkHdr + (p - j * kMaxPayload)];
    }
    uint64_t a = c0, e = c0 + total;
    while (e - a > 1) {
      const uint64_t m = (a + e) >> 1;
      if (ck_pay[m] - pay0 <= p) a = m;
      else e = m;
    }
    return span[a * kChunk + kChunkHdr + (p - (ck_pay[a] - pay0))];
  }
  __device__ __forceinline__ uint32_t le(uint64_t p, int k) const {  // k <= 4 bytes, little-endian
    uint32_t v = 0;
    for (int i = 0; i < k; i++) v |= b(p + i) << (8 * i);
    return v;
  }
};

struct ZSz {
  uint64_t content = 0;  // decoded bytes (declared or bounded)
  uint64_t bound = 0;    // decoded bytes bounded per block (entry pieces)
  uint64_t lits = 0, nseq = 0, njobs = 0, nframes = 0, jobs_bytes = 0;
};

// the walk; false if a header does not parse
__device__ bool z_size_walk(const ZSzIn &in, ZSz &z) {
  const uint64_t n = in.n;
  uint64_t pos = 0;
  while (pos < n) {
    if (n - pos < 4) return false;
    const uint32_t magic = in.le(pos, 4);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (n - pos < 8) return false;
      pos += 8 + (uint64_t)in.le(pos + 4, 4);
      continue;
    }
    if (magic != kZMagic || n - pos < 5) return false;
    const uint32_t fhd = in.b(pos + 4);
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
    uint64_t p = pos + 5;
    uint64_t window = 0;
    if (!single) {
      if (p >= n) return false;
      const uint32_t wd = in.b(p++);
      const uint32_t wlog = 10 + (wd >> 3);
      if (wlog > 31) return false;
      window = (1ull << wlog) + ((1ull << wlog) / 8) * (uint64_t)(wd & 7);
    }
    p += did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
    const uint32_t fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : (fcs_flag == 2 ? 4 : 8));
    if (p + fcs_len > n) return false;
    int64_t fcs = -1;
    if (fcs_len == 1) fcs = in.b(p);
    else if (fcs_len == 2) fcs = in.le(p, 2) + 256;
    else if (fcs_len == 4) fcs = in.le(p, 4);
    else if (fcs_len == 8) fcs = (int64_t)(in.le(p, 4) | ((uint64_t)in.le(p + 4, 4) << 32));
    p += fcs_len;
    if (single) window = (uint64_t)fcs;
    const uint64_t block_max = window < (uint64_t)kZBlockMax ? window : (uint64_t)kZBlockMax;
    uint64_t fb = 0;  // the frame's decoded bytes, bounded per block
    for (;;) {
      if (p + 3 > n) return false;
      const uint32_t bh = in.le(p, 3);
      p += 3;
      const uint32_t type = (bh >> 1) & 3;
      const uint64_t size = bh >> 3;
      if (type == 3 || size > block_max) return false;
      z.njobs++;
      if (type == 0 || type == 1) {  // raw / RLE: literal-only jobs
        z.lits += size;
        fb += size;
        z.jobs_bytes += (uint64_t)kZJobHdr;
        p += type == 0 ? size : 1;
      } else {
        if (size < 1 || p + size > n) return false;
        const uint32_t b0 = in.b(p);
        const uint32_t ltype = b0 & 3, sf = (b0 >> 2) & 3;
        uint64_t regen, lhdr, ldata;
        if (ltype < 2) {  // raw / RLE literals
          if (sf == 1) lhdr = 2, regen = (b0 >> 4) + ((uint64_t)in.b(p + 1) << 4);
          else if (sf == 3) lhdr = 3, regen = (b0 >> 4) + ((uint64_t)in.le(p + 1, 2) << 4);
          else lhdr = 1, regen = b0 >> 3;
          ldata = ltype == 0 ? regen : 1;
          if (lhdr > size) return false;
        } else {  // Huffman-coded literals: 10/10, 14/14 or 18/18 bits of sizes
          lhdr = sf < 2 ? 3 : (sf == 2 ? 4 : 5);
          if (lhdr > size) return false;
          const uint64_t h = (uint64_t)in.le(p, 4) | (lhdr == 5 ? (uint64_t)in.b(p + 4) << 32 : 0ull);
          const uint32_t bits = sf < 2 ? 10 : (sf == 2 ? 14 : 18);
          regen = (h >> 4) & ((1ull << bits) - 1);
          ldata = (h >> (4 + bits)) & ((1ull << bits) - 1);
        }
        const uint64_t q = p + lhdr + ldata;  // the sequences section
        if (q >= p + size) return false;
        const uint32_t s0 = in.b(q);
        uint64_t ns = s0;
        if (s0 >= 128) {
          if (q + 2 > p + size) return false;
          if (s0 < 255) ns = ((uint64_t)(s0 - 128) << 8) + in.b(q + 1);
          else if (q + 3 > p + size) return false;
          else ns = (uint64_t)in.le(q + 1, 2) + 0x7F00;
        }
        z.lits += regen;
        z.nseq += ns;
        z.jobs_bytes += ((uint64_t)kZJobHdr + (ns ? 4 * (512 + 512 + 256) : 0) + 8 * ns + 15) & ~15ull;
        fb += block_max;
        p += size;
      }
      if (p > n) return false;
      if (bh & 1) break;
    }
    if (checksum) p += 4;
    if (p > n) return false;
    z.content += fcs >= 0 ? (uint64_t)fcs : fb;
    z.bound += fb;
    z.nframes++;
    pos = p;
  }
  return true;
}

__global__ void k_zstd_size(const uint8_t *__restrict__ span, DevBufs d, const unsigned long long *nblocks,
                            uint32_t factor) {
  const uint64_t nb = *nblocks;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long meta = d.blk_meta[b];
    const uint32_t cls = (uint32_t)(meta >> kMetaClsShift) & 0xffu;
    const bool dec = (meta & kMetaComplete) && (cls == kMagicPacked || cls == kMagicTrailer);
    const uint64_t n = dec ? d.blk_len[b] : 0;
    uint64_t out = 0, need = 0, half = 0;
    if (n > 0) {
      const uint64_t in_area = (n + 16 + 15) & ~15ull;
      const uint64_t serial = ((n + 64 + 255) & ~255ull) + zx::kStateBytes;
      ZSzIn in{span, d.ck_pay, d.blk_c0[b], meta & kMetaTotalMask, 0, n, (meta & kMetaRegular) != 0};
      in.pay0 = d.ck_pay[in.c0];
      ZSz z;
      if (z_size_walk(in, z)) {
        out = z.content;
        const uint64_t ents = z.nseq + z.bound / kZPiece + 2 * z.njobs + z.nframes + 2 * (kZBlockMax / kZPiece) + 8;
        half = (in_area + z.lits + 64 + 8 * ents + 15) & ~15ull;
        need = half + z.jobs_bytes;
      } else {  // the passes find the error (or decline to the serial decoder)
        out = n * factor + 4096;
        half = (2 * in_area + 65536 + 15) & ~15ull;
        need = 2 * half;
      }
      if (need < serial) need = serial;
      if (half > need) half = need;
    }
    if (d.blk_need[b] > out) out = d.blk_need[b];  // exact size from a previous attempt
    d.blk_out_len[b] = (out + 255) & ~255ull;
    d.blk_zneed[b] = (need + 255) & ~255ull;
    d.blk_zhalf[b] = half;
    d.blk_status[b] = kBlkOk;
    d.blk_a[b] = 0;
    d.blk_b[b] = 0;
  }
}

void launch_zstd_size(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks,
                      uint32_t factor, hipStream_t st) {
  uint64_t g = (max_blocks + 255) / 256;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(k_zstd_size, dim3((unsigned)(g ? g : 1)), dim3(256), 0, st, span, d, nblocks, factor);
}

// ---------------------------------------------------------------- k_zstd_ent
// Frame pass, one wave per recordio block (grid-stride): flattenIov, frames
// and block headers, Huffman literals (4 streams on 4 lanes) into the block's
// literal area, the sequence tables built from their descriptions; every zstd
// block becomes a job (ZJob) for k_zstd_seq. Region of block b (512 KiB per
// chunk): flattened input | literals (up) ... execution entries (down from
// the middle) | jobs (from the middle up).
// Registers for 3 waves per SIMD (12 per CU, the LDS's limit at ~12 KiB each):
// left to itself the compiler takes 205 VGPRs (2 waves per SIMD) and 1/3 of the
// launched waves wait; at 168 VGPRs (28 spilled, cold paths) C4 177.6 -> 161.4 ms.
#ifndef RIO_ZENT_WPE
#define RIO_ZENT_WPE 3
#endif
#define RIO_ZENT_ATTR __attribute__((amdgpu_waves_per_eu(RIO_ZENT_WPE)))
__global__ void __launch_bounds__(64) RIO_ZENT_ATTR k_zstd_ent(const uint8_t *__restrict__ span, DevBufs d,
                                                 const unsigned long long *nblocks, uint64_t dec_cap) {
  __shared__ ZLds L;
  const int l = lane_id();
  const uint64_t nb = uni64(*nblocks);
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    FlState *sp = &d.fl[b];
    const uint64_t c0 = uni64(d.blk_c0[b]);
    const unsigned long long meta = uni64(d.blk_meta[b]);
    const uint32_t cls = (uint32_t)(meta >> kMetaClsShift) & 0xffu;
    // incomplete blocks, and magics that are never untransformed (the header
    // block is idTransform, registry.go:31; others are errors): nothing decoded
    if (!(meta & kMetaComplete) || (cls != kMagicPacked && cls != kMagicTrailer)) {
      if (l == 0) {
        sp->mode = kZsSkip;
        d.blk_out_len[b] = 0;
      }
      continue;
    }
    const uint64_t off = uni64(d.blk_dec_off[b]), cap = uni64(d.blk_out_len[b]);
    if (off + cap > dec_cap) {  // the regions need a larger buffer (host retries)
      if (l == 0) {
        sp->mode = kZsSkip;
        atomicOr(&d.ctl->out_overflow, 0x40ull);
        atomicMax(&d.ctl->dec_need, (unsigned long long)(off + cap));
        d.blk_out_len[b] = 0;
      }
      continue;
    }
    const uint64_t n = uni64(d.blk_len[b]);
    if (n == 0) {  // DataDog Decompress: ErrEmptySlice
      if (l == 0) {
        sp->mode = kZsSkip;
        d.blk_status[b] = kBlkCodec;
        d.blk_a[b] = kCodecZstdEmpty;
        d.blk_b[b] = 0;
        d.blk_out_len[b] = 0;
      }
      continue;
    }
#ifdef RIO_ZPROF
    zprof_ctl = d.ctl;
#endif
    ZPROF_T(tb);
    // the block's scratch region (k_zstd_size): all regions must fit tok (else
    // the host grows it to their total and retries)
    const uint64_t zoff = uni64(d.blk_zoff[b]), rbytes = uni64(d.blk_zneed[b]);
    if (zoff + rbytes > d.tok_cap * 4) {
      if (l == 0) {
        sp->mode = kZsSkip;
        atomicOr(&d.ctl->out_overflow, kOvfZTok);
        atomicMax(&d.ctl->tok_need, d.blk_zoff[nb]);
        d.blk_out_len[b] = 0;
      }
      continue;
    }
    uint32_t *flat = d.tok + zoff / 4;
    z_flatten(span, d, c0, meta, n, flat);
    ZFrame z;
    z_init(z, reinterpret_cast<const uint8_t *>(flat), nullptr, (int64_t)cap, nullptr);
    ZJobSink k;
    k.tok8 = reinterpret_cast<uint8_t *>(d.tok);
    k.region = zoff;
    k.half = (int64_t)uni64(d.blk_zhalf[b]);
    k.lit_w = (int64_t)((n + 16 + 15) & ~15ull);
    k.job_w = k.half;
    k.job_end = (int64_t)rbytes;
    k.last = -1;
    k.njobs = 0;
    k.pend_first = 0;
    k.zjob = d.zjob;
    k.zjob_cap = d.zjob_cap;
    k.ctl = d.ctl;
    const int64_t lit0 = k.lit_w;
    uint32_t zerr = 0;
    int64_t pos = 0;
    while (pos < (int64_t)n) {
      const int64_t r = z_decode_frame(z, L, k, pos, (int64_t)n - pos);
      if (r < 0) {
        zerr = (uint32_t)(-r);
        break;
      }
      pos += r;
    }
    ZPROF_ADD(3, tb);
    if (l == 0) {
      if (zerr == kZSlow) {
        sp->mode = kZsSlow;
        atomicAdd(&d.ctl->pad[1], 1ull);
      } else {  // k_zstd_fix finishes it: the jobs, then this error (if any)
        sp->mode = kZsJobs;
        sp->final_ = zerr;
        sp->ntok = k.njobs;
        sp->olen = k.region + (uint64_t)k.half;  // the first job's header
        sp->olen2 = (unsigned long long)k.lit_w;  // the literal area's end
        sp->bitpos = (unsigned long long)lit0;
        sp->hdrpos = (unsigned long long)k.half;  // execution entries end here
      }
    }
  }
}

// readlane of a u32
__device__ __forceinline__ uint32_t zrl(uint32_t v, uint32_t lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// ---------------------------------------------------------------- k_zstd_seq2
// Sequence pass with the FSE tables in LDS: four waves per CU, each decoding
// kZs2Jobs jobs at a time (a lane per job, lanes kZs2Jobs..63 idle), each job's
// three tables in its own LDS slot as u16 cells. 60 jobs per CU is far fewer
// than the round-1 pass (a lane per job, u32 cells in HBM) kept in flight, but a
// cell load is an LDS access (~100 cycles) instead of an HBM/MALL miss: with
// every job of a span in flight (82k for C4) the tables (up to 5 KiB each)
// outgrew every cache, and each sequence waited on a DRAM access. A cell here is the symbol (6 bits) and
// FSE's nextState (10 bits); nbBits = log - highbit(nextState) and the new
// state's base = (nextState << nbBits) - 2^log are recomputed per use. A job's
// tables are loaded by the whole wave (u32 cells from k_zstd_ent); the lanes
// then decode independently, and a lane whose job ends takes the next one.
// Backward bitstream reader for the sequence pass. Stream dword D_i (i = 0, 1,
// ... from the end) = w[qtop - i]. A 64-bit container holds the bits below the
// read position (`avail` of them); a reload (when avail <= 32) shifts in
// D_cons from the lane's 32-dword LDS ring, which k_zstd_seq2 refills group by
// group. The sequence loop reloads before the offset, before the match /
// literal extras and before the state updates, which bounds every read
// (offset <= 28 bits, extras <= 16 + 16, states <= 9 + 9 + 8), so a sequence
// takes at most 3 dwords.
constexpr int kZs2Ring = 32;
// Measured and kept out (round 3; A/B on one box, C4 ms per step): the ring
// dword of the next reload loaded a reload ahead (150.2 against 147.0) and the
// LL / ML code baselines computed instead of looked up (153.2; both 155.0) --
// this pass's pace is set by where the compiler places its LDS waits. Round 6:
// a sequence's three ring dwords read with its table lookups, so that no
// reload waits on an LDS read of its own: 40.7 GiB/s against 40.7-40.9.
struct ZBr64 {
  const uint32_t *w;
  uint64_t win;
  int32_t avail, qtop, lo;
  int32_t cons, nf;  // D_cons is the next dword into the container; the ring holds [cons, nf)
  __device__ __forceinline__ uint32_t ld(int32_t i) const { return i >= 0 ? w[i] : 0u; }
  __device__ __forceinline__ uint32_t D(int32_t i) const { return ld(qtop - i); }
  // D_i without the zero fill past the stream's start (a clamped address, no
  // select on the loaded value): those bits are only read by an overrun,
  // which is an error whatever they hold
  __device__ __forceinline__ uint32_t Dc(int32_t i) const { return w[max(qtop - i, 0)]; }
  // ring: this lane's kZs2Ring dwords (D_i at i mod kZs2Ring)
  __device__ __forceinline__ void prime(const uint32_t (&)[kZs2Ring]) {}
  __device__ __forceinline__ void reload(const uint32_t (&ring)[kZs2Ring]) {
    if (avail <= 32) {
      // in the ring once retired from the registers (else a direct load: rare)
      // the ring always holds it: >= 24 dwords at the start of every group of
      // 8 sequences. No global load on this path (its wait would drain every
      // load in flight).
      const uint32_t v = ring[cons & (kZs2Ring - 1)];
      win = (win << 32) | v;
      cons++;
      avail += 32;
    }
  }
  // the same from three ring dwords read at the sequence's start (D_c0 ..
  // D_c0+2: a sequence takes at most three), so that no reload waits for an
  // LDS read of its own (k_zstd_seq4)
  // (the sequence's first reload can only take D_c0, its second D_c0 or D_c0+1)
  __device__ __forceinline__ void reload_pf(uint32_t p) {
    const bool rl = avail <= 32;
    const uint64_t nw = (win << 32) | p;
    win = rl ? nw : win;
    cons += rl ? 1 : 0;
    avail += rl ? 32 : 0;
  }
  __device__ __forceinline__ void reload_pf(uint32_t p0, uint32_t p1, int32_t c0) {
    reload_pf(cons == c0 ? p0 : p1);
  }
  __device__ __forceinline__ void reload_pf(uint32_t p0, uint32_t p1, uint32_t p2, int32_t c0) {
    const int32_t k = cons - c0;
    reload_pf(k == 0 ? p0 : (k == 1 ? p1 : p2));
  }
  // nb (<= 31) bits at off above the read position (the container's bit avail), not consumed
  __device__ __forceinline__ uint32_t field(uint32_t off, uint32_t nb) const {
    return (uint32_t)(win >> (avail + (int32_t)off)) & ((1u << nb) - 1u);
  }
  __device__ __forceinline__ uint32_t read(int nb) {  // nb <= 31
    avail -= nb;
    return (uint32_t)(win >> avail) & ((1u << nb) - 1u);
  }
  // bit position above the stream's dword base: the container's low bit is D_(cons-1)'s
  __device__ __forceinline__ int32_t pos() const { return 32 * (qtop - cons + 1) + avail; }
  __device__ __forceinline__ bool overrun() const { return pos() < lo; }
  __device__ __forceinline__ bool exact() const { return pos() == lo; }
};

// An empty asm that reads and rewrites x: the wait for x's load lands here.
template <class T>
__device__ __forceinline__ void zs2_settle(T &x) {
  asm volatile("" : "+v"(x));
}

#ifndef RIO_ZS2_JOBS
#define RIO_ZS2_JOBS 15
#endif
constexpr int kZs2Jobs = RIO_ZS2_JOBS;         // job slots per wave
constexpr int kZs2Groups = 15 / kZs2Jobs;      // 4-wave workgroups per CU (60 slots' tables fill the LDS)
constexpr int kZs2Cells = 512 + 512 + 256;  // ll (log <= 9), ml (<= 9), of (<= 8)
#ifndef RIO_ZS2_QUAD
#define RIO_ZS2_QUAD 1  // the sequence pass with a quad of lanes per job (k_zstd_seq4); 0: k_zstd_seq2
#endif

__device__ __forceinline__ uint16_t zs2_cell(uint32_t c, int log) {
  const uint32_t sym = c & 0xffu, nb = (c >> 8) & 0xffu, base = c >> 16;
  const uint32_t ns = (base + (1u << log)) >> nb;  // FSE's nextState: base = (ns << nb) - 2^log
  return (uint16_t)(sym | (ns << 6));
}
// cell -> symbol; state <- base + bits (read by the caller)
__device__ __forceinline__ uint32_t zs2_nb(uint32_t e, int log) { return (uint32_t)(log - highbit(e >> 6)); }
__device__ __forceinline__ uint32_t zs2_base(uint32_t e, uint32_t nb, int log) {
  return ((e >> 6) << nb) - (1u << log);
}

__global__ void __launch_bounds__(256) k_zstd_seq2(DevBufs d) {
  __shared__ uint16_t tabs[4][kZs2Jobs][kZs2Cells];
  __shared__ uint32_t rings[4][kZs2Jobs][kZs2Ring];
  __shared__ ZCodes codes;
  const int l = lane_id(), wv = (int)(threadIdx.x >> 6);
  for (int u = (int)threadIdx.x; u < 36; u += 256) codes.ll[u] = kZCodes.ll[u];
  for (int u = (int)threadIdx.x; u < 53; u += 256) codes.ml[u] = kZCodes.ml[u];
  __syncthreads();
  uint8_t *tok8 = reinterpret_cast<uint8_t *>(d.tok);
  const uint64_t nj0 = d.ctl->zjob_n, nj = nj0 < d.zjob_cap ? nj0 : d.zjob_cap;
  const bool slot = l < kZs2Jobs;
  const int ls = slot ? l : 0;  // (indices into the __shared__ arrays, not pointers: a
                                // selected pointer becomes a flat access that waits on vmcnt)
  const uint64_t stride = (uint64_t)gridDim.x * 4 * kZs2Jobs;
  uint64_t j = ((uint64_t)blockIdx.x * 4 + (uint64_t)wv) * kZs2Jobs + (uint64_t)l;
  bool active = false, exhausted = !slot;
  ZJob *hp = nullptr;
  uint32_t nseq = 0, i = 0, err = 0, sll = 0, sml = 0, sof = 0;
  int llg = 0, mlg = 0, ofg = 0;
  uint64_t *raw = nullptr;
  ZBr64 r;
  for (;;) {
    // lanes without a job take their next one (literal-only and empty jobs need no pass)
    bool starting = false;
    uint64_t tab_off = 0;
    if (!active && !exhausted) {
      for (;;) {
        if (j >= nj) {
          exhausted = true;
          break;
        }
        hp = reinterpret_cast<ZJob *>(tok8 + d.zjob[j]);
        j += stride;
        const uint32_t flags = hp->flags;
        nseq = hp->nseq;
        if ((flags & kJLit) || nseq == 0) continue;
        const uint32_t logs = hp->logs;
        llg = logs & 0xff;
        ofg = (logs >> 8) & 0xff;
        mlg = (logs >> 16) & 0xff;
        if (llg > 9 || mlg > 9 || ofg > 8) {  // beyond the format's accuracy logs: not from ent
          hp->err = kZSlow;
          continue;
        }
        tab_off = hp->tab_off;
        raw = reinterpret_cast<uint64_t *>(tok8 + hp->raw_off);
        starting = true;
        // the job's values become plain registers here: the hot loop's first
        // use of a value loaded on this rare path would otherwise wait for
        // every load in flight (the loop's vmcnt bookkeeping is conservative)
        zs2_settle(nseq);
        zs2_settle(llg);
        zs2_settle(mlg);
        zs2_settle(ofg);
        break;
      }
    }
    // the starting lanes' tables into their slots, each by the whole wave
    unsigned long long sm = __ballot(starting);
    while (sm) {
      const int s = __ffsll((long long)sm) - 1;
      sm &= sm - 1;
      const uint64_t to = readlane_u64(tab_off, s);
      const int lg = __builtin_amdgcn_readlane(llg, s), mg = __builtin_amdgcn_readlane(mlg, s);
      const int og = __builtin_amdgcn_readlane(ofg, s);
      const uint32_t nll = 1u << lg, nml = 1u << mg, nof = 1u << og, n = nll + nml + nof;
      const uint32_t *src = reinterpret_cast<const uint32_t *>(tok8 + to);
      uint16_t *dst = tabs[wv][s];
      for (uint32_t k0 = 0; k0 < n; k0 += 512) {
        uint32_t c[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const uint32_t k = k0 + 64 * q + (uint32_t)l;
          c[q] = k < n ? src[k] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const uint32_t k = k0 + 64 * q + (uint32_t)l;
          if (k < nll) dst[k] = zs2_cell(c[q], lg);
          else if (k < nll + nml) dst[512 + (k - nll)] = zs2_cell(c[q], mg);
          else if (k < n) dst[1024 + (k - nll - nml)] = zs2_cell(c[q], og);
        }
      }
    }
    if (starting) {  // the bitstream: container, ring, registers
      i = 0;
      err = 0;
      const int64_t start = (int64_t)hp->seq_off, n = (int64_t)hp->seq_len;
      const uint32_t last = n > 0 ? tok8[start + n - 1] : 0u;
      if (last == 0) {  // empty stream or no end marker in its last byte
        err = kZCorrupt;
      } else {
        r.w = reinterpret_cast<const uint32_t *>(tok8 + (start & ~3ll));
        r.lo = 8 * (int32_t)(start & 3);
        const int32_t P = r.lo + 8 * (int32_t)n - (8 - highbit(last));  // first bit not yet read
        r.qtop = (P - 1) >> 5;
        r.win = ((uint64_t)r.D(0) << 32) | r.D(1);
        r.avail = P - 32 * (r.qtop - 1);
        r.cons = 2;
        // D_2 .. D_(kZs2Ring + 1) into the ring
#pragma unroll
        for (int t = 2; t < 2 + kZs2Ring; t++) rings[wv][ls][t & (kZs2Ring - 1)] = r.D(t);
        r.nf = 2 + kZs2Ring;
        sll = r.read(llg);
        sof = r.read(ofg);
        sml = r.read(mlg);
        r.prime(rings[wv][ls]);
        r.reload(rings[wv][ls]);
      }
      active = err == 0;
      if (!active) hp->err = err;
      zs2_settle(r.win);
      zs2_settle(r.avail);
      zs2_settle(r.qtop);
      zs2_settle(r.lo);
      zs2_settle(sll);
      zs2_settle(sml);
      zs2_settle(sof);
    }
    // top up rings below 24 dwords (a lane that outran its feed; rare: waits)
    if (active && r.nf - r.cons < 24) {
      const int32_t nn = r.cons + kZs2Ring;
      for (int32_t t = r.nf; t < nn; t++) rings[wv][ls][t & (kZs2Ring - 1)] = r.D(t);
      r.nf = nn;
    }
    wave_lds_sync();
    if (!__ballot(active) && !__ballot(!exhausted)) break;
    // Groups of 8 unrolled steps, a sequence each, until a lane needs a job
    // or a top-up. A group starts by loading up to 8 dwords to refill the
    // ring (the ring holds >= 24: enough for 8 sequences of <= 3 dwords) and
    // keeps its 8 raw entries in registers; at its end the loads go into the
    // ring and the entries out. So the group's body issues no vector memory
    // operation whose wait would queue behind others (vmcnt counts in order),
    // and nothing in flight crosses the loop's back edge.
    uint64_t E0 = 0, E1 = 0, E2 = 0, E3 = 0, E4 = 0, E5 = 0, E6 = 0, E7 = 0;
    uint32_t pi0 = 0, pne = 0;  // the previous group's entries (stored by the next group)
    do {
      // the previous group's entries out first: registers of a store in
      // flight are rewritten only once it has read them, and issued before
      // this group's loads that wait does not include them
      if (pne > 0) raw[pi0 + 0] = E0;
      if (pne > 1) raw[pi0 + 1] = E1;
      if (pne > 2) raw[pi0 + 2] = E2;
      if (pne > 3) raw[pi0 + 3] = E3;
      if (pne > 4) raw[pi0 + 4] = E4;
      if (pne > 5) raw[pi0 + 5] = E5;
      if (pne > 6) raw[pi0 + 6] = E6;
      if (pne > 7) raw[pi0 + 7] = E7;
      const int32_t c = active ? min(8, kZs2Ring - (r.nf - r.cons)) : 0;
      // (no initial values: writing a register whose previous load may be in
      // flight waits for it; each L_t is read only under the condition that loads it)
      uint32_t L0, L1, L2, L3, L4, L5, L6, L7;
      if (c > 0) L0 = r.Dc(r.nf);
      if (c > 1) L1 = r.Dc(r.nf + 1);
      if (c > 2) L2 = r.Dc(r.nf + 2);
      if (c > 3) L3 = r.Dc(r.nf + 3);
      if (c > 4) L4 = r.Dc(r.nf + 4);
      if (c > 5) L5 = r.Dc(r.nf + 5);
      if (c > 6) L6 = r.Dc(r.nf + 6);
      if (c > 7) L7 = r.Dc(r.nf + 7);
      const uint32_t i0 = i;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if (active) {
          const uint32_t cl = tabs[wv][ls][sll], cm = tabs[wv][ls][512 + sml], cof = tabs[wv][ls][1024 + sof];
          const uint32_t llc = cl & 63u, mlc = cm & 63u, ofc = cof & 63u;
          if (llc > 35 || mlc > 52 || ofc > 31) {
            err = kZCorrupt;
          } else if (ofc > 28) {
            err = kZSlow;
          } else {
            const uint32_t mlx = codes.ml[mlc], llx = codes.ll[llc];
            const uint32_t ofv = (1u << ofc) + r.read((int)ofc);
            r.reload(rings[wv][ls]);
            const uint32_t ml = (mlx & 0xFFFFFFu) + r.read((int)(mlx >> 24));
            const uint32_t ll = (llx & 0xFFFFFFu) + r.read((int)(llx >> 24));
            r.reload(rings[wv][ls]);
            if (i + 1 < nseq) {
              const uint32_t nl = zs2_nb(cl, llg), nm = zs2_nb(cm, mlg), no = zs2_nb(cof, ofg);
              sll = zs2_base(cl, nl, llg) + r.read((int)nl);
              sml = zs2_base(cm, nm, mlg) + r.read((int)nm);
              sof = zs2_base(cof, no, ofg) + r.read((int)no);
              r.reload(rings[wv][ls]);
            }
            if (r.overrun()) {
              err = kZCorrupt;
            } else {
              uint64_t &Ek = k == 0 ? E0 : k == 1 ? E1 : k == 2 ? E2 : k == 3 ? E3 : k == 4 ? E4 : k == 5 ? E5 : k == 6 ? E6 : E7;
              Ek = (uint64_t)ll | ((uint64_t)ml << 17) | ((uint64_t)ofv << 35);
              i++;
              if (i == nseq && !r.exact()) err = kZCorrupt;
            }
          }
          if (err || i == nseq) active = false;
        }
      }
      // the group's loads into the ring, its entries out (entries i0 .. i - 1)
      const uint32_t ne = i - i0;
      if (c > 0) rings[wv][ls][(r.nf + 0) & (kZs2Ring - 1)] = L0;
      if (c > 1) rings[wv][ls][(r.nf + 1) & (kZs2Ring - 1)] = L1;
      if (c > 2) rings[wv][ls][(r.nf + 2) & (kZs2Ring - 1)] = L2;
      if (c > 3) rings[wv][ls][(r.nf + 3) & (kZs2Ring - 1)] = L3;
      if (c > 4) rings[wv][ls][(r.nf + 4) & (kZs2Ring - 1)] = L4;
      if (c > 5) rings[wv][ls][(r.nf + 5) & (kZs2Ring - 1)] = L5;
      if (c > 6) rings[wv][ls][(r.nf + 6) & (kZs2Ring - 1)] = L6;
      if (c > 7) rings[wv][ls][(r.nf + 7) & (kZs2Ring - 1)] = L7;
      if (c > 0) r.nf += c;
      pi0 = i0;
      pne = ne;
      if (hp && !active && (err || (i == nseq && ne > 0))) hp->err = err;  // the job ended in this group
    } while (!__ballot((slot && !active && !exhausted) || (active && r.nf - r.cons < 24)));
    if (pne > 0) raw[pi0 + 0] = E0;
    if (pne > 1) raw[pi0 + 1] = E1;
    if (pne > 2) raw[pi0 + 2] = E2;
    if (pne > 3) raw[pi0 + 3] = E3;
    if (pne > 4) raw[pi0 + 4] = E4;
    if (pne > 5) raw[pi0 + 5] = E5;
    if (pne > 6) raw[pi0 + 6] = E6;
    if (pne > 7) raw[pi0 + 7] = E7;
  }
}

// ---------------------------------------------------------------- k_zstd_seq4
// The sequence pass with a QUAD of lanes per job (round 6). k_zstd_seq2 gives
// each job one lane, so a step decodes the three FSE symbols (literal length,
// match length, offset) one after the other in that lane, with 15 of 64 lanes
// live: ~164 wave instructions per sequence, and with one wave per SIMD (the
// tables fill the LDS) every instruction is on the chain. Here lanes 4q .. 4q+3
// share job q: lane role 0 owns the literal-length state, 1 the match-length
// state, 2 the offset state (3 shadows role 0). Each lane looks up its own
// table cell and code, the quad exchanges the six bit counts by DPP
// quad-broadcasts, and every lane advances the same bit container (the reads'
// positions depend on all six counts) while extracting only its own fields.
// The three ring dwords a sequence may need are read with the table lookups,
// so no reload waits on an LDS read of its own. Same tables, rings, jobs,
// entries, checks and errors as k_zstd_seq2. The step's error and the state
// update are computed by masks (RIO_ZS4_BFERR): C4 44.8 -> 46.3 GiB/s.
// Measured and not kept (profiles/r06_zstd_seq4_err_ab.jsonl): the literal- and
// match-length codes' extra-bit counts computed from the symbol (a nibble
// table in registers), so that the code table's LDS read leaves the state
// chain -- 44.6 alone, 41.7 together with the mask-based step.
#ifndef RIO_ZS4_BFERR
#define RIO_ZS4_BFERR 1  // the step's error and state update by masks (0: by selects, which the compiler branches on)
#endif
template <int kSel>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {  // lane (4q + kSel)'s v, on all four lanes
  constexpr int kCtl = kSel | (kSel << 2) | (kSel << 4) | (kSel << 6);  // quad_perm [k, k, k, k]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kCtl, 0xf, 0xf, false);
}

// The ring with its first three dwords mirrored after its end (RIO_ZS4_MIRROR),
// so that a step's three dwords D_c0 .. D_c0+2 are adjacent: one address, no
// wrap masks (140 wave instructions per step instead of 157; C4 46.3-46.6
// against 46.5-46.5 without, profiles/r06_zstd_seq4_mirror_ab.jsonl: the pass
// is bound by its step's dependency chain, not by issue).
#ifndef RIO_ZS4_MIRROR
#define RIO_ZS4_MIRROR 1
#endif
constexpr int kZs4Ring = kZs2Ring + (RIO_ZS4_MIRROR ? 4 : 0);
__global__ void __launch_bounds__(256) k_zstd_seq4(DevBufs d) {
  __shared__ uint16_t tabs[4][kZs2Jobs][kZs2Cells];
  __shared__ uint32_t rings[4][kZs2Jobs][kZs4Ring];
  __shared__ uint32_t codes[36 + 53];  // ZCodes: ll at 0, ml at 36
  const int l = lane_id(), wv = (int)(threadIdx.x >> 6);
  const int q = l >> 2, role = l & 3;
  for (int u = (int)threadIdx.x; u < 36; u += 256) codes[u] = kZCodes.ll[u];
  for (int u = (int)threadIdx.x; u < 53; u += 256) codes[36 + u] = kZCodes.ml[u];
  __syncthreads();
  uint8_t *tok8 = reinterpret_cast<uint8_t *>(d.tok);
  const uint64_t nj0 = d.ctl->zjob_n, nj = nj0 < d.zjob_cap ? nj0 : d.zjob_cap;
  const bool slot = q < kZs2Jobs;
  const int qs = slot ? q : 0;
  // this lane's table: cells at toff, codes at cbase, accuracy log (set per job)
  const uint32_t toff = role == 1 ? 512u : (role == 2 ? 1024u : 0u);
  const uint32_t cbase = role == 1 ? 36u : 0u;
  const uint32_t slim = role == 1 ? 52u : (role == 2 ? 31u : 35u);  // the format's largest code
  const uint64_t stride = (uint64_t)gridDim.x * 4 * kZs2Jobs;
  uint64_t j = ((uint64_t)blockIdx.x * 4 + (uint64_t)wv) * kZs2Jobs + (uint64_t)q;
  bool active = false, exhausted = !slot;
  // ring dword D_t in, D_(c0 + k) out (k <= 2)
  auto rput = [&](int32_t t, uint32_t v) {
    const int32_t sl = t & (kZs2Ring - 1);
    rings[wv][qs][sl] = v;
    if (RIO_ZS4_MIRROR && sl < 3) rings[wv][qs][kZs2Ring + sl] = v;
  };
  auto rget = [&](int32_t c0, int k) -> uint32_t {
    return RIO_ZS4_MIRROR ? rings[wv][qs][(c0 & (kZs2Ring - 1)) + k] : rings[wv][qs][(c0 + k) & (kZs2Ring - 1)];
  };
  ZJob *hp = nullptr;
  uint32_t nseq = 0, i = 0, err = 0, st = 0;
  int llg = 0, mlg = 0, ofg = 0, lg = 0;
  uint64_t *raw = nullptr;
  ZBr64 r;
  for (;;) {
    bool starting = false;
    uint64_t tab_off = 0;
    if (!active && !exhausted) {  // (the quad's four lanes take the same job)
      for (;;) {
        if (j >= nj) {
          exhausted = true;
          break;
        }
        hp = reinterpret_cast<ZJob *>(tok8 + d.zjob[j]);
        j += stride;
        const uint32_t flags = hp->flags;
        nseq = hp->nseq;
        if ((flags & kJLit) || nseq == 0) continue;
        const uint32_t logs = hp->logs;
        llg = logs & 0xff;
        ofg = (logs >> 8) & 0xff;
        mlg = (logs >> 16) & 0xff;
        if (llg > 9 || mlg > 9 || ofg > 8) {
          if (role == 0) hp->err = kZSlow;
          continue;
        }
        tab_off = hp->tab_off;
        raw = reinterpret_cast<uint64_t *>(tok8 + hp->raw_off);
        starting = true;
        zs2_settle(nseq);
        zs2_settle(llg);
        zs2_settle(mlg);
        zs2_settle(ofg);
        break;
      }
    }
    // the starting quads' tables into their slots, each by the whole wave
    unsigned long long sm = __ballot(starting && role == 0);
    while (sm) {
      const int s = __ffsll((long long)sm) - 1;  // (lane 4 qq of quad qq)
      sm &= sm - 1;
      const uint64_t to = readlane_u64(tab_off, s);
      const int lg0 = __builtin_amdgcn_readlane(llg, s), mg = __builtin_amdgcn_readlane(mlg, s);
      const int og = __builtin_amdgcn_readlane(ofg, s);
      const uint32_t nll = 1u << lg0, nml = 1u << mg, nof = 1u << og, n = nll + nml + nof;
      const uint32_t *src = reinterpret_cast<const uint32_t *>(tok8 + to);
      uint16_t *dst = tabs[wv][s >> 2];
      for (uint32_t k0 = 0; k0 < n; k0 += 512) {
        uint32_t c[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const uint32_t k = k0 + 64 * u + (uint32_t)l;
          c[u] = k < n ? src[k] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const uint32_t k = k0 + 64 * u + (uint32_t)l;
          if (k < nll) dst[k] = zs2_cell(c[u], lg0);
          else if (k < nll + nml) dst[512 + (k - nll)] = zs2_cell(c[u], mg);
          else if (k < n) dst[1024 + (k - nll - nml)] = zs2_cell(c[u], og);
        }
      }
    }
    if (starting) {  // the bitstream: container and ring (shared by the quad), this lane's state
      i = 0;
      err = 0;
      lg = role == 1 ? mlg : (role == 2 ? ofg : llg);
      const int64_t start = (int64_t)hp->seq_off, n = (int64_t)hp->seq_len;
      const uint32_t last = n > 0 ? tok8[start + n - 1] : 0u;
      if (last == 0) {
        err = kZCorrupt;
      } else {
        r.w = reinterpret_cast<const uint32_t *>(tok8 + (start & ~3ll));
        r.lo = 8 * (int32_t)(start & 3);
        const int32_t P = r.lo + 8 * (int32_t)n - (8 - highbit(last));
        r.qtop = (P - 1) >> 5;
        r.win = ((uint64_t)r.D(0) << 32) | r.D(1);
        r.avail = P - 32 * (r.qtop - 1);
        r.cons = 2;
        // D_2 .. D_(kZs2Ring + 1) into the ring, a quarter per lane of the quad
#pragma unroll
        for (int t = 2; t < 2 + kZs2Ring; t += 4) rput(t + role, r.D(t + role));
        r.nf = 2 + kZs2Ring;
        const uint32_t sll = r.read(llg), sof = r.read(ofg), sml = r.read(mlg);  // RFC 8878 3.1.1.3.2.2
        st = role == 1 ? sml : (role == 2 ? sof : sll);
      }
      if (err == 0) {
        wave_lds_sync();
        r.reload(*reinterpret_cast<const uint32_t(*)[kZs2Ring]>(rings[wv][qs]));
      }
      active = err == 0;
      if (!active && role == 0) hp->err = err;
      zs2_settle(r.win);
      zs2_settle(r.avail);
      zs2_settle(r.qtop);
      zs2_settle(r.lo);
      zs2_settle(st);
    }
    // top up rings below 24 dwords (a quad that outran its feed; rare: waits)
    if (active && r.nf - r.cons < 24) {
      const int32_t nn = r.cons + kZs2Ring;
      for (int32_t t = r.nf; t < nn; t += 4)
        if (t + role < nn) rput(t + role, r.D(t + role));
      r.nf = nn;
    }
    wave_lds_sync();
    if (!__ballot(active) && !__ballot(!exhausted)) break;
    // Groups of 8 steps as k_zstd_seq2's; the group's ring refill split over
    // the quad (lane role k loads dwords k and k + 4 of the group's up to 8)
    uint64_t E0 = 0, E1 = 0, E2 = 0, E3 = 0, E4 = 0, E5 = 0, E6 = 0, E7 = 0;
    uint32_t pi0 = 0, pne = 0;
    do {
      if (role == 0) {
        if (pne > 0) raw[pi0 + 0] = E0;
        if (pne > 1) raw[pi0 + 1] = E1;
        if (pne > 2) raw[pi0 + 2] = E2;
        if (pne > 3) raw[pi0 + 3] = E3;
        if (pne > 4) raw[pi0 + 4] = E4;
        if (pne > 5) raw[pi0 + 5] = E5;
        if (pne > 6) raw[pi0 + 6] = E6;
        if (pne > 7) raw[pi0 + 7] = E7;
      }
      const int32_t c = active ? min(8, kZs2Ring - (r.nf - r.cons)) : 0;
      uint32_t La, Lb;
      if (role < c) La = r.Dc(r.nf + role);
      if (role + 4 < c) Lb = r.Dc(r.nf + role + 4);
      const uint32_t i0 = i;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if (active) {
          const int32_t c0 = r.cons;  // the ring holds D_c0 .. D_c0+2 (>= 24 - 3k dwords at step k)
          const uint32_t cell = tabs[wv][qs][toff + st];
          const uint32_t p0 = rget(c0, 0), p1 = rget(c0, 1),
                         p2 = rget(c0, 2);
          const uint32_t sym = cell & 63u;
          const uint32_t cx = codes[cbase + (sym < 53u ? sym : 0u)];
          const uint32_t nbs = zs2_nb(cell, lg);
          // extra bits and value base of this lane's code (offset: code bits, 1 << code)
          const uint32_t E = role == 2 ? (sym & 31u) : (cx >> 24);
          const uint32_t V = role == 2 ? (1u << (sym & 31u)) : (cx & 0xFFFFFFu);
          const uint32_t flag = (sym > slim ? 1u : 0u) | ((role == 2 && sym > 28u) ? 2u : 0u);
          const uint32_t pk = E | (nbs << 8) | (flag << 16);
          const uint32_t pll = quad_bcast<0>(pk), pml = quad_bcast<1>(pk), pof = quad_bcast<2>(pk);
          // Branch-free: the reads run whatever the checks say (a bad code ends
          // the job, so what its reads did to the container does not matter),
          // the state reads with 0 bits after the job's last sequence (a no-op,
          // as skipping them was), the reloads by selects.
          const bool more = i + 1 < nseq;
          // Each of the three groups of reads (offset extra | match + literal
          // extras | the three states) moves the container once; a lane
          // extracts only its own field of the group, at its offset in it.
          const uint32_t eof = pof & 31u, eml = pml & 31u, ell = pll & 31u;
          const uint32_t nll = more ? (pll >> 8) & 15u : 0u, nml = more ? (pml >> 8) & 15u : 0u,
                         nof = more ? (pof >> 8) & 15u : 0u;
          r.avail -= (int32_t)eof;
          const uint32_t x1 = r.field(0, eof);  // (the offset lane's)
          r.reload_pf(p0);
          r.avail -= (int32_t)(eml + ell);
          const uint32_t x2 = r.field(role == 1 ? ell : 0u, role == 1 ? eml : ell);  // (match / literal lanes')
          r.reload_pf(p0, p1, c0);
          r.avail -= (int32_t)(nll + nml + nof);
          const uint32_t x3 = r.field(role == 1 ? nof : (role == 2 ? 0u : nml + nof), role == 1 ? nml : (role == 2 ? nof : nll));
          r.reload_pf(p0, p1, p2, c0);
          const uint32_t val = V + (role == 2 ? x1 : x2);
          const uint32_t st2 = zs2_base(cell, nbs, lg) + x3;
          const uint32_t ll = val, ml = quad_bcast<1>(val), ofv = quad_bcast<2>(val);  // (role 0's entry is the one stored)
          uint64_t &Ek = k == 0 ? E0 : k == 1 ? E1 : k == 2 ? E2 : k == 3 ? E3 : k == 4 ? E4 : k == 5 ? E5 : k == 6 ? E6 : E7;
          Ek = (uint64_t)ll | ((uint64_t)ml << 17) | ((uint64_t)ofv << 35);
#if RIO_ZS4_BFERR
          // the step's error, in the serial decoder's order (a bad code, then an
          // offset code the fast path declines, then an overrun; after the last
          // sequence, a stream not consumed exactly), by masks: the compiler
          // branches on a chain of selects, and the state update waited on it
          const uint32_t bad = (((pll | pml | pof) >> 16) & 1u), slow = (pof >> 17) & 1u;
          const uint32_t ovr = r.overrun() ? 1u : 0u;
          const uint32_t isc = bad | (ovr & (slow ^ 1u)), iss = slow & (bad ^ 1u);
          const uint32_t e2 = ((uint32_t)kZCorrupt & (0u - isc)) | ((uint32_t)kZSlow & (0u - iss));
          const uint32_t ok = (isc | iss) ^ 1u, mv = more ? 1u : 0u;
          st = (ok & mv) ? st2 : st;
          i += ok;
          err = e2 | ((uint32_t)kZCorrupt & (0u - (ok & (mv ^ 1u) & (r.exact() ? 0u : 1u))));
#else
          const uint32_t e2 = ((pll | pml | pof) & (1u << 16)) ? kZCorrupt
                              : (pof & (2u << 16))             ? kZSlow
                              : r.overrun()                    ? kZCorrupt
                                                               : 0u;
          if (e2 == 0) {
            if (more) st = st2;
            i++;
            if (!more && !r.exact()) err = kZCorrupt;
          } else {
            err = e2;
          }
#endif
          if (err || i == nseq) active = false;
        }
      }
      const uint32_t ne = i - i0;
      if (role < c) rput(r.nf + role, La);
      if (role + 4 < c) rput(r.nf + role + 4, Lb);
      if (c > 0) r.nf += c;
      pi0 = i0;
      pne = ne;
      if (role == 0 && hp && !active && (err || (i == nseq && ne > 0))) hp->err = err;
    } while (!__ballot((slot && !active && !exhausted) || (active && r.nf - r.cons < 24)));
    if (role == 0) {
      if (pne > 0) raw[pi0 + 0] = E0;
      if (pne > 1) raw[pi0 + 1] = E1;
      if (pne > 2) raw[pi0 + 2] = E2;
      if (pne > 3) raw[pi0 + 3] = E3;
      if (pne > 4) raw[pi0 + 4] = E4;
      if (pne > 5) raw[pi0 + 5] = E5;
      if (pne > 6) raw[pi0 + 6] = E6;
      if (pne > 7) raw[pi0 + 7] = E7;
    }
  }
}

// One step of the repeat-offset history scan (k_zstd_fix): compose this
// lane's op (src, c) after the op of the DPP source lane (g o f); lanes the
// DPP pattern gives no source keep the identity op (slot k <- slot k, + 0).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void z_hist_step(uint32_t &src, uint32_t &c0, uint32_t &c1, uint32_t &c2) {
  constexpr int kIdSrc = 0 | (1 << 2) | (2 << 4);
  const uint32_t fs = (uint32_t)__builtin_amdgcn_update_dpp(kIdSrc, (int)src, kCtrl, kRowMask, 0xf, false);
  const uint32_t f0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c0, kCtrl, kRowMask, 0xf, false);
  const uint32_t f1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c1, kCtrl, kRowMask, 0xf, false);
  const uint32_t f2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c2, kCtrl, kRowMask, 0xf, false);
  uint32_t ns = 0, nc[3];
  const uint32_t cc[3] = {c0, c1, c2};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t gs = (src >> (2 * k)) & 3u;
    const uint32_t fsel = gs == 0 ? f0 : (gs == 1 ? f1 : f2);
    ns |= (gs == 3 ? 3u : (fs >> (2 * gs)) & 3u) << (2 * k);
    nc[k] = gs == 3 ? cc[k] : fsel + cc[k];
  }
  src = ns;
  c0 = nc[0];
  c1 = nc[1];
  c2 = nc[2];
}

// ---------------------------------------------------------------- k_zstd_fix
// In file order, one wave per recordio block: every job's raw sequences 64 at
// a time -- repeat offsets resolved by a wave scan of history ops, the serial decoder's
// per-sequence checks made lane-parallel from prefix sums (literals left,
// offset within the frame's output), execution entries written -- then the
// frame checks (content size), then the frame walk's own error if it stopped
// early. The result: entries for k_zstd_exec, an error, the exact size for
// the host's retry, or the serial path.
__global__ void __launch_bounds__(64) k_zstd_fix(DevBufs d, const unsigned long long *nblocks) {
  const int l = lane_id();
  uint8_t *tok8 = reinterpret_cast<uint8_t *>(d.tok);
  const uint64_t nb = uni64(*nblocks);
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    FlState *sp = &d.fl[b];
    if (uni(sp->mode) != kZsJobs) continue;
    const uint64_t region = uni64(d.blk_zoff[b]);
    const int64_t half = (int64_t)uni64(sp->hdrpos), lit_end = (int64_t)uni64(sp->olen2);
    uint8_t *ents = tok8 + region + half;  // entry e at ents - 8 (e + 1)
    const int64_t cap = (int64_t)uni64(d.blk_out_len[b]);
    const uint32_t njobs = uni(sp->ntok);
    uint64_t jo = uni64(sp->olen);
    uint32_t zerr = 0;
    bool ck_done = false;
    int64_t ent = 0, ent_mark = 0, olen = 0, fstart = 0;
    uint32_t rep0 = 1, rep1 = 4, rep2 = 8;
    auto put = [&](uint64_t e) {
      if (l == 0) *reinterpret_cast<uint64_t *>(ents - 8 * (ent + 1)) = e;
      ent++;
    };
    auto pieces = [&](uint64_t ll, uint64_t ml, uint64_t off) {
      while (ll > kZPiece) {
        put(kZPiece);
        ll -= kZPiece;
      }
      uint64_t m = ml < kZPiece ? ml : kZPiece;
      put(ll | (m << 16) | (off << 32));
      ml -= m;
      while (ml) {
        m = ml < kZPiece ? ml : kZPiece;
        put((m << 16) | (off << 32));
        ml -= m;
      }
    };
    for (uint32_t j = 0; j < njobs && !zerr; j++) {
      const ZJob *hp = reinterpret_cast<const ZJob *>(tok8 + jo);
      const uint32_t flags = uni(hp->flags), regen = uni(hp->regen), nseq = uni(hp->nseq), jerr = uni(hp->err);
      const uint64_t raw_off = uni64(hp->raw_off), next = uni64(hp->next);
      const int64_t fcs = (int64_t)uni64((uint64_t)hp->fcs);
      const uint32_t cks = uni(hp->checksum);
      if (flags & kJFirst) {
        fstart = olen;
        rep0 = 1;
        rep1 = 4;
        rep2 = 8;
      }
      // entries grow down towards the literal area's end
      if (lit_end + 64 > half - 8 * (ent + (int64_t)nseq + 2 * (kZBlockMax / kZPiece) + 4)) {
        zerr = kZSlow;
        break;
      }
      int64_t lp = 0;
      if (!(flags & kJLit) && nseq) {
        if (jerr) {
          zerr = jerr;
          break;
        }
        const uint64_t *raw = reinterpret_cast<const uint64_t *>(tok8 + raw_off);
        // raw sequences three groups ahead: a group's work (~200 instructions)
        // is far shorter than a load's latency under load, so with one group in
        // flight each wave waited out most of every load
        auto ld = [&](uint32_t at) { return at + (uint32_t)l < nseq ? raw[at + l] : 0ull; };
        uint64_t rv_1 = ld(0), rv_2 = ld(64), rv_3 = ld(128);
        for (uint32_t g0 = 0; g0 < nseq; g0 += 64) {
          const uint32_t cnt = nseq - g0 < 64 ? nseq - g0 : 64;
          const bool v = (uint32_t)l < cnt;
          const uint64_t rv = rv_1;
          rv_1 = rv_2;
          rv_2 = rv_3;
          if (g0 + 192 < nseq) rv_3 = ld(g0 + 192);
          const uint32_t ll = (uint32_t)rv & 0x1FFFFu, ml = (uint32_t)(rv >> 17) & 0x3FFFFu;
          const uint32_t ofv = (uint32_t)(rv >> 35);
          // Repeat offsets: a sequence maps the offset history (rep0, rep1, rep2)
          // by an op "slot k <- slot src_k + c_k, or the constant c_k when
          // src_k = 3" (RFC 8878 3.1.2.5); an inclusive scan of the composed ops
          // gives each sequence the history after it, whose slot 0 is its offset.
          uint32_t src, c0, c1 = 0, c2 = 0;
          {
            const uint32_t idx = ofv > 3 ? 0u : ofv + (ll == 0 ? 1u : 0u);
            if (!v || idx == 1) {  // offset = rep0, history unchanged
              src = 0u | (1u << 2) | (2u << 4);
              c0 = 0;
            } else if (idx == 0) {  // a new offset
              src = 3u | (0u << 2) | (1u << 4);
              c0 = ofv - 3;
            } else if (idx == 2) {
              src = 1u | (0u << 2) | (2u << 4);
              c0 = 0;
            } else if (idx == 3) {
              src = 2u | (0u << 2) | (1u << 4);
              c0 = 0;
            } else {  // rep0 - 1 (0 is the error below)
              src = 0u | (0u << 2) | (1u << 4);
              c0 = ~0u;
            }
          }
          // inclusive scan by DPP (row shifts, then the row broadcasts, as
          // wave_incl_sum_dpp); lanes without a source lane compose the identity
          z_hist_step<0x111, 0xf>(src, c0, c1, c2);  // row_shr:1
          z_hist_step<0x112, 0xf>(src, c0, c1, c2);  // row_shr:2
          z_hist_step<0x114, 0xf>(src, c0, c1, c2);  // row_shr:4
          z_hist_step<0x118, 0xf>(src, c0, c1, c2);  // row_shr:8
          z_hist_step<0x142, 0xa>(src, c0, c1, c2);  // row_bcast:15
          z_hist_step<0x143, 0xc>(src, c0, c1, c2);  // row_bcast:31
          auto apply = [&](uint32_t sk, uint32_t ck) {
            return sk == 3 ? ck : (sk == 0 ? rep0 : (sk == 1 ? rep1 : rep2)) + ck;
          };
          const uint32_t off = apply(src & 3u, c0);
          {  // the history after the group (lanes past cnt hold the identity)
            const uint32_t ls = zrl(src, 63), l0 = zrl(c0, 63), l1 = zrl(c1, 63), l2 = zrl(c2, 63);
            const uint32_t n0 = apply(ls & 3u, l0), n1 = apply((ls >> 2) & 3u, l1), n2 = apply((ls >> 4) & 3u, l2);
            rep0 = n0;
            rep1 = n1;
            rep2 = n2;
          }
          // z_exec's checks per sequence: literals left, offset within the frame's output
          const uint32_t lin = wave_incl_sum_dpp(v ? ll : 0u), tin = wave_incl_sum_dpp(v ? ll + ml : 0u);
          const int64_t my_lp = lp + (int64_t)(lin - ll);
          const int64_t prod = olen - fstart + (int64_t)(tin - ml);  // output before its match
          const bool bad = v && (my_lp + (int64_t)ll > (int64_t)regen || off == 0 || (int64_t)off > prod);
          if (__ballot(bad)) {
            zerr = kZCorrupt;
            break;
          }
          if (__ballot(v && (ll > kZPiece || ml > kZPiece))) {
            for (uint32_t f = 0; f < cnt; f++) pieces(zrl(ll, f), zrl(ml, f), zrl(off, f));
          } else {
            if (v)
              *reinterpret_cast<uint64_t *>(ents - 8 * (ent + l + 1)) =
                  (uint64_t)ll | ((uint64_t)ml << 16) | ((uint64_t)off << 32);
            ent += cnt;
          }
          lp += zrl(lin, cnt - 1);
          olen += zrl(tin, cnt - 1);
        }
        if (zerr) break;
      }
      if ((int64_t)regen > lp) pieces((uint64_t)((int64_t)regen - lp), 0, 0);  // the block's last literals
      olen += (int64_t)regen - lp;
      if (flags & kJLast) {
        if (fcs >= 0 && olen - fstart != fcs) {
          zerr = kZCorrupt;
          break;
        }
        put((flags & kJCk) ? (kZMark | ((uint64_t)kZMarkCk << 16) | ((uint64_t)cks << 32))
                           : (kZMark | ((uint64_t)kZMarkNoCk << 16)));
        ent_mark = ent;
        ck_done |= (flags & kJCk) != 0;
      }
      jo = next;
    }
    if (!zerr) zerr = uni(sp->final_);                // the frame walk stopped there
    if (!zerr && olen >= (1ll << 31)) zerr = kZSlow;  // the execution pass counts in u32
    if (l == 0) {
      if (zerr) {  // declined or corrupt: the exact decoder decides (libzstd's semantics)
        sp->mode = kZsSlow;
        atomicAdd(&d.ctl->pad[1], 1ull);
      } else if (olen > cap) {  // exact size: the host retries with it
        sp->mode = kZsSkip;
        d.blk_need[b] = (unsigned long long)olen;
        atomicOr(&d.ctl->out_overflow, 8ull);
        d.blk_status[b] = kBlkCodec;
        d.blk_a[b] = kCodecFull;
        d.blk_out_len[b] = 0;
      } else {
        sp->mode = kZsExec;
        sp->stored_left = 0;
        sp->ntok = (uint32_t)ent;
      }
    }
  }
}

// ---------------------------------------------------------------- k_zstd_exec
// Execution pass, one wave per block: the entries in groups of 64, cut into
// parts of at most kZPart output bytes (and at frame ends); per part the
// literals are staged from the literal area into LDS, literal runs written,
// then matches -- a parallel round for short ones whose source precedes the
// part's first match, the rest in order, each by the whole wave -- into an LDS
// ring holding the last kZHist bytes; completed 1 KiB units are flushed to the
// decode region 16 B per lane. Sources further back than the ring are read
// from the decode region: a group's far sources are loaded a group ahead
// (visible by vmcnt's in-order retirement, see the loop), the rest after a
// vmcnt(0) drain. Round 6: with far sources prefetched, an 8 KiB ring at 12
// waves per CU beats 20 KiB at 6 (C4 33.2 -> 40.8 GiB/s pipelined, 29.6 -> 35.1
// serial, A/B on one box, profiles/r06_zstd_ring_ab.jsonl).
#ifndef RIO_ZRING_K
#define RIO_ZRING_K 2
#endif
#ifndef RIO_ZEXEC_READY_MAX
// longest match a lane copies on its own in the parallel round (longer ones: the
// whole wave, in order). Round 6, with far sources prefetched and 12 waves per
// CU: 16 -> C4 47.5-47.7 / 40.1-40.3 serial, 12 the same, 8 46.7-46.9, 24
// 46.8-47.0, 32 (rounds 2-5) 46.6-46.9, 48 45.5-46.1
// (profiles/r06_zstd_ready_max_ab.jsonl)
#define RIO_ZEXEC_READY_MAX 16
#endif
constexpr uint32_t kZRingK = RIO_ZRING_K;  // ring = kZRingK x 4 KiB
static_assert(kZRingK >= 2, "zr_slot's multiply-high reciprocal needs kZRingK >= 2");
constexpr uint32_t kZRing = kZRingK * 4096;
constexpr uint32_t kZPart = 2 * kZPiece;
constexpr uint32_t kZHist = kZRing - kZPart;
#ifndef RIO_ZEXEC_WAVES
#define RIO_ZEXEC_WAVES 12
#endif
constexpr int kZExecWaves = RIO_ZEXEC_WAVES;  // per CU (~12 KiB LDS each at the default ring)

// x mod kZRing: (x >> 12) / kZRingK by a multiply-high, exact below 2^20
__device__ __forceinline__ uint32_t zr_slot(uint32_t x) {
  return x - __umulhi(x >> 12, 0xFFFFFFFFu / kZRingK + 1u) * kZRing;
}
__device__ __forceinline__ uint8_t zr_src(const uint8_t *ring, const uint8_t *out, uint32_t pos, uint32_t base) {
  return pos + kZHist >= base ? ring[zr_slot(pos)] : out[pos];
}
// k mod d for k < 2^20, d >= 1
__device__ __forceinline__ uint32_t z_umod(uint32_t k, uint32_t dv) {
  uint32_t q = (uint32_t)((float)k * __builtin_amdgcn_rcpf((float)dv));
  int32_t r = (int32_t)(k - q * dv);
  if (r < 0) r += (int32_t)dv;
  if (r >= (int32_t)dv) r -= (int32_t)dv;
  return (uint32_t)r;
}
// completed 1 KiB units of [flushed, olen) to HBM (a unit never wraps: the ring is whole KiB)
__device__ __forceinline__ void zr_flush(const uint8_t *ring, uint8_t *out, uint32_t &flushed, uint32_t olen) {
  const int l = lane_id();
  for (uint32_t u0 = flushed; u0 + 1024 <= olen; u0 += 1024) {
    const uint4 v = *reinterpret_cast<const uint4 *>(ring + zr_slot(u0) + 16 * l);
    *reinterpret_cast<uint4 *>(out + u0 + 16 * l) = v;
    flushed = u0 + 1024;
  }
}

__global__ void __launch_bounds__(64) k_zstd_exec(DevBufs d, const unsigned long long *nblocks) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[kZRing];
  __shared__ __attribute__((aligned(16))) uint32_t litbuf[kZPart / 4 + 8];
  const int l = lane_id();
  const uint64_t nb = uni64(*nblocks);
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    FlState *sp = &d.fl[b];
    const uint32_t mode = uni(sp->mode);
    if (mode != kZsExec && mode != kZsErrCk) continue;
    const uint8_t *region = reinterpret_cast<const uint8_t *>(d.tok) + uni64(d.blk_zoff[b]);
    const uint64_t lit0 = uni64(sp->bitpos), ent_end = uni64(sp->hdrpos);
    const uint32_t ntok = uni(sp->ntok);
    const uint64_t *ents = reinterpret_cast<const uint64_t *>(region + ent_end);  // entry e at ents[-1 - e]
    const uint32_t *lit32 = reinterpret_cast<const uint32_t *>(region + lit0);    // 16-aligned
    uint8_t *out = d.dec + uni64(d.blk_dec_off[b]);
    uint32_t olen = 0, litpos = 0, flushed = 0, fstart = 0, zerr = 0;
    uint32_t synced = 0;  // bytes below it: flushed and visible to this wave
    // one group ahead: its 64 entries and the first 256 bytes of its literals
    // (from dword-aligned pf_nx; ~0: not prefetched), so a group usually
    // starts without waiting for memory; entries two groups ahead, so that the
    // next group's far match sources are loaded a group ahead too (below)
    uint64_t e_nx = (uint32_t)l < ntok ? ents[-1 - (int64_t)l] : 0ull;
    uint64_t e_n2 = 64 + (uint32_t)l < ntok ? ents[-1 - (int64_t)(64 + l)] : 0ull;
    uint32_t fl_e2 = 0;  // `flushed` when e_n2's load was issued
    uint32_t pf0 = 0, pf1 = 0, pf2 = 0;  // this lane's far match source in this group: its first 12 dword-aligned bytes
    bool pfv = false;
    uint32_t pf_nx = ~0u, lit_nx = 0;
    if (lit0 + 256 <= ent_end) {
      pf_nx = 0;
      lit_nx = lit32[l];
    }
    wave_lds_sync();
    for (uint32_t g0 = 0; g0 < ntok && !zerr; g0 += 64) {
      const uint32_t n = ntok - g0 < 64 ? ntok - g0 : 64;
      const uint64_t e = e_nx;
      const uint32_t q0 = pf0, q1 = pf1, q2 = pf2;  // (loaded a group ago)
      const bool qv = pfv;
      uint32_t lit_at = ~0u;  // litbuf holds literal bytes [lit_at, lit_at + 256)
      if (pf_nx != ~0u) {
        wave_lds_sync();
        litbuf[l] = lit_nx;
        lit_at = pf_nx;
      }
      // The next group's entries were loaded a group ago, before any of the
      // previous group's flush stores; vmcnt retires a wave's vector memory
      // operations in issue order, so once their load is waited for (its first
      // use, below), every byte flushed before it -- fl_e2 -- is visible to
      // this wave without a vmcnt(0) drain.
      e_nx = e_n2;
      const uint32_t vis = fl_e2;
      fl_e2 = flushed;
      if (g0 + 128 < ntok)
        e_n2 = (uint32_t)l < ntok - g0 - 128 ? ents[-1 - (int64_t)(g0 + 128 + l)] : 0ull;
      const uint32_t ll0 = (uint32_t)e & 0xffffu, ml0 = (uint32_t)(e >> 16) & 0xffffu, off = (uint32_t)(e >> 32);
      const bool mark = ll0 == kZMark;
      const uint32_t len = mark ? 0u : ll0 + ml0, lits = mark ? 0u : ll0;
      const uint32_t incl = wave_incl_sum_dpp(len), lincl = wave_incl_sum_dpp(lits);
      const uint32_t excl = incl - len, lexcl = lincl - lits;
      const unsigned long long marks = __ballot(mark);
      pfv = false;
      if (g0 + 64 < ntok) {
        // the next group's far match sources (more than kZHist back, every byte
        // visible): their first 12 dword-aligned bytes loaded now, used by its
        // parallel round a group later -- the loads' latency hides behind this
        // group's work instead of stalling that round (39 % of C4's sequences
        // reach past the ring, each its own 128-B line: tools/zstd_seqstat.c)
        const uint32_t l1 = (uint32_t)e_nx & 0xffffu, m1 = (uint32_t)(e_nx >> 16) & 0xffffu, o1 = (uint32_t)(e_nx >> 32);
        const bool v1 = g0 + 64 + (uint32_t)l < ntok && l1 != kZMark;
        const uint32_t len1 = v1 ? l1 + m1 : 0u;
        const uint32_t dst1 = olen + zrl(incl, n - 1) + wave_incl_sum_dpp(len1) - len1 + l1;
        const uint32_t src1 = dst1 - o1;
        pfv = v1 && m1 != 0 && o1 > kZHist && o1 <= dst1 && src1 + m1 <= vis;
        if (pfv) {
          const uint32_t *w = reinterpret_cast<const uint32_t *>(out + (src1 & ~3u));
          pf0 = w[0];
          pf1 = w[1];
          pf2 = w[2];
        }
        if (vis > synced) synced = vis;
      }
      {  // the next group's literals start where this group's end
        const uint32_t na = (litpos + zrl(lincl, n - 1)) & ~3u;
        pf_nx = ~0u;
        if (g0 + 64 < ntok && lit0 + na + 256 <= ent_end) {
          pf_nx = na;
          lit_nx = lit32[(na >> 2) + l];
        }
      }
      uint32_t s = 0;
      while (s < n) {
        const uint32_t bs = zrl(excl, s), ls = zrl(lexcl, s);
        const unsigned long long over = __ballot((uint32_t)l >= s && (uint32_t)l < n && incl - bs > kZPart);
        const unsigned long long mk = marks & (~0ull << s);
        uint32_t e1 = n;
        if (over) e1 = min(e1, (uint32_t)(__ffsll((long long)over) - 1));
        if (mk) e1 = min(e1, (uint32_t)(__ffsll((long long)mk) - 1));
        if (e1 > s) {
          const uint32_t T = zrl(incl, e1 - 1) - bs, Ls = zrl(lincl, e1 - 1) - ls;
          const bool mine = (uint32_t)l >= s && (uint32_t)l < e1;
          const uint32_t base = olen;
          const uint32_t p = excl - bs;  // part-relative output position
          const uint32_t myll = mine ? ll0 : 0u, myml = mine ? ml0 : 0u;
          if (Ls) {  // literals: stage the part's run of the literal area, then scatter
            const uint32_t a0 = litpos & ~3u, nd = (litpos + Ls - a0 + 3) >> 2;
            if (a0 != lit_at || nd > 64) {  // not the prefetched bytes
              wave_lds_sync();
              for (uint32_t j = l; j < nd; j += 64) litbuf[j] = lit32[(a0 >> 2) + j];
              lit_at = ~0u;
            }
            wave_lds_sync();
            const uint8_t *lb = reinterpret_cast<const uint8_t *>(litbuf) + (litpos - a0);
            const uint32_t lp = lexcl - ls;
            if (myll && myll <= 32) {
              const uint32_t q0 = base + p;
              for (uint32_t k = 0; k < myll; k++) ring[zr_slot(q0 + k)] = lb[lp + k];
            }
            unsigned long long rem = __ballot(myll > 32);
            while (rem) {
              const uint32_t f = (uint32_t)(__ffsll((long long)rem) - 1);
              rem &= rem - 1;
              const uint32_t N = zrl(myll, f), P = base + zrl(p, f), LP = zrl(lp, f);
              for (uint32_t k0 = 0; k0 < N; k0 += 64) {
                const uint32_t k = k0 + (uint32_t)l;
                if (k < N) ring[zr_slot(P + k)] = lb[LP + k];
              }
            }
          }
          wave_lds_sync();
          const bool m = myml != 0;
          const unsigned long long mm = __ballot(m);
          if (mm) {
            const uint32_t dst = base + p + myll, src = dst - off;
            {  // bytes read from the decode region (pos + kZHist < base) visible first: drain
               // the wave's stores only when one of them lies at or above the last drain's mark
              const uint32_t hi = min(src + (myml < off ? myml : off), base - kZHist);
              if (__ballot(m && src + kZHist < base && hi > synced)) {
                zmem_sync();
                synced = flushed;
              }
            }
            // one parallel round: short matches whose source ends before the
            // part's first match, each by its own lane ...
            const uint32_t R = zrl(dst, (uint32_t)(__ffsll((long long)mm) - 1));
            const uint32_t src_end = src + (myml < off ? myml : off);
            const bool ready = m && src_end <= R && myml <= (uint32_t)RIO_ZEXEC_READY_MAX;
            if (ready) {
              // the source wholly in the ring or wholly flushed (src + kZHist vs base is
              // monotone in the byte), neither ring range wrapping: 12 aligned bytes per
              // 8-byte piece, two funnel shifts, byte stores at immediate offsets
              const bool all_ring = src + kZHist >= base, all_far = src + myml - 1 + kZHist < base;
              const uint32_t ss = zr_slot(src), ds = zr_slot(dst);
              if ((off >= 8 || myml <= off) && (all_far || (all_ring && ss + myml + 12 <= kZRing)) &&
                  ds + myml <= kZRing) {
                // (measured and not kept, round 6: a far match's pieces' source dwords
                // all loaded before any is used -- 44.6 / 37.6 GiB/s against 46.5 /
                // 39.5, profiles/r06_zstd_exec_unroll_ab.jsonl)
                for (uint32_t k = 0; k < myml; k += 8) {
                  uint32_t w0, w1, w2;
                  if (k == 0 && qv && all_far) {  // prefetched a group ago
                    w0 = q0;
                    w1 = q1;
                    w2 = q2;
                  } else {
                    const uint32_t *w = all_ring ? reinterpret_cast<const uint32_t *>(ring + ((ss + k) & ~3u))
                                                 : reinterpret_cast<const uint32_t *>(out + ((src + k) & ~3u));
                    w0 = w[0];
                    w1 = w[1];
                    w2 = w[2];
                  }
                  const uint32_t sh = (src + k) & 3u;  // ss = src (mod 4)
                  const uint32_t x0 = __builtin_amdgcn_alignbyte(w1, w0, sh), x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
                  uint8_t *dp = ring + ds + k;
#pragma unroll
                  for (int jj = 0; jj < 8; jj++)
                    if (k + jj < myml) dp[jj] = (uint8_t)((jj < 4 ? x0 : x1) >> (8 * (jj & 3)));
                }
              } else if (off >= 8 || myml <= off) {  // no byte of an 8-byte piece depends on another
                for (uint32_t k = 0; k < myml; k += 8) {
                  uint8_t v[8];
#pragma unroll
                  for (int jj = 0; jj < 8; jj++) v[jj] = k + jj < myml ? zr_src(ring, out, src + k + jj, base) : 0;
#pragma unroll
                  for (int jj = 0; jj < 8; jj++)
                    if (k + jj < myml) ring[zr_slot(dst + k + jj)] = v[jj];
                }
              } else {  // overlapping run: byte by byte, each reads one written before it
                for (uint32_t k = 0; k < myml; k++) ring[zr_slot(dst + k)] = ring[zr_slot(src + k)];
              }
            }
            // ... then the rest in order, each by the whole wave (every byte it
            // reads precedes it and is final by then)
            unsigned long long rest = mm & ~__ballot(ready);
#ifdef RIO_ZPROF
            if (l == 0) {
              atomicAdd(&d.ctl->zx[1], 1ull);
              atomicAdd(&d.ctl->zx[2], (unsigned long long)__popcll(mm));
              atomicAdd(&d.ctl->zx[3], (unsigned long long)__popcll(rest));
            }
#endif
            while (rest) {
              const uint32_t f = (uint32_t)(__ffsll((long long)rest) - 1);
              rest &= rest - 1;
              wave_lds_sync();
              const uint32_t P = zrl(dst, f), D = zrl(off, f), N = zrl(myml, f), S = P - D;
              for (uint32_t k0 = 0; k0 < N; k0 += 64) {
                const uint32_t k = k0 + (uint32_t)l;
                const uint32_t kk = D >= N ? k : z_umod(k, D);
                const uint8_t v = k < N ? zr_src(ring, out, S + kk, base) : 0;
                if (k < N) ring[zr_slot(P + k)] = v;
              }
            }
          }
          olen += T;
          litpos += Ls;
          if ((olen & ~1023u) > flushed) {
            wave_lds_sync();
            zr_flush(ring, out, flushed, olen);
          }
        }
        if (e1 < n && ((marks >> e1) & 1ull)) {  // frame end
          if (zrl(ml0, e1) == kZMarkCk) {
            wave_lds_sync();
            zr_flush(ring, out, flushed, olen);
            for (uint32_t k = flushed + l; k < olen; k += 64) out[k] = ring[zr_slot(k)];
            zmem_sync();
            const uint32_t got = (uint32_t)z_xxh64(out + fstart, olen - fstart);
            if (got != zrl(off, e1)) {
              zerr = kZChecksum;
              break;
            }
          }
          fstart = olen;
          e1++;
        }
        s = e1;
      }
    }
    wave_lds_sync();
    zr_flush(ring, out, flushed, olen);
    for (uint32_t k = flushed + l; k < olen; k += 64) out[k] = ring[zr_slot(k)];
    if (l == 0) {
      if (!zerr && mode == kZsExec) {
        d.blk_out_len[b] = olen;
      } else {  // a checksum mismatch: the exact decoder re-decodes the block and names the error
        sp->mode = kZsSlow;
        atomicAdd(&d.ctl->pad[1], 1ull);
      }
    }
  }
}

// ---------------------------------------------------------------- k_zstd (serial path)
// The exact decoder (zstd_exact.h: libzstd's semantics, lane 0 of a wave per
// block) for every block the fast passes declined or found corrupt: its result
// -- bytes, or the error and its name -- is the block's. Runs after
// k_zstd_exec, which hands checksum failures here too.
__global__ void __launch_bounds__(64) k_zstd(const uint8_t *__restrict__ span, DevBufs d,
                                             const unsigned long long *nblocks, uint64_t dec_cap) {
  const int l = lane_id();
  const uint64_t nb = uni64(*nblocks);
  uint8_t *lit = d.zlit + (uint64_t)blockIdx.x * kZLitStride;
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    if (uni(d.fl[b].mode) != kZsSlow) continue;
    const uint64_t c0 = uni64(d.blk_c0[b]);
    const unsigned long long meta = uni64(d.blk_meta[b]);
    const uint32_t cls = (uint32_t)(meta >> kMetaClsShift) & 0xffu;
    // incomplete blocks, and magics that are never untransformed (the header
    // block is idTransform, registry.go:31; others are errors): nothing decoded
    if (!(meta & kMetaComplete) || (cls != kMagicPacked && cls != kMagicTrailer)) {
      if (l == 0) d.blk_out_len[b] = 0;
      continue;
    }
    const uint64_t off = uni64(d.blk_dec_off[b]), cap = uni64(d.blk_out_len[b]);
    if (off + cap > dec_cap) {  // the regions need a larger buffer (host retries)
      if (l == 0) {
        atomicOr(&d.ctl->out_overflow, 0x40ull);
        atomicMax(&d.ctl->dec_need, (unsigned long long)(off + cap));
        d.blk_out_len[b] = 0;
      }
      continue;
    }
    const uint64_t n = uni64(d.blk_len[b]);
    uint32_t code = 0, zerr = 0;
    int64_t olen = 0;
    if (n == 0) {  // DataDog Decompress: ErrEmptySlice
      code = kCodecZstdEmpty;
    } else {
      uint32_t *flat = d.tok + uni64(d.blk_zoff[b]) / 4;
      z_flatten(span, d, c0, meta, n, flat);
      if (l == 0) {
        // decoder state after the flattened input in the block's region (k_zstd_size)
        uint8_t *region = reinterpret_cast<uint8_t *>(flat);
        zx::Ctx z;
        z.s = reinterpret_cast<zx::State *>(region + ((n + 64 + 255) & ~255ull));
        z.in = region;
        z.out = d.dec + off;
        z.cap = (int64_t)cap;
        z.lit = lit;
        zerr = zx::decompress(z, (int64_t)n);
        olen = z.olen;
      }
      zerr = (uint32_t)__builtin_amdgcn_readfirstlane(zerr);
      olen = (int64_t)readlane_u64((unsigned long long)olen, 0);
      if (zerr == zx::kFull) {  // size the retry from the declared content size
        int64_t need = z_size_bound(reinterpret_cast<const uint8_t *>(flat), (int64_t)n);
        if (need <= (int64_t)cap) need = 4 * (int64_t)cap + 4096;
        if (l == 0) {
          d.blk_need[b] = (unsigned long long)need;
          atomicOr(&d.ctl->out_overflow, 8ull);
        }
        code = kCodecFull;
      } else if (zerr) {
        code = kCodecZstd;
      }
    }
    if (l == 0) {
      if (code) {
        d.blk_status[b] = kBlkCodec;
        d.blk_a[b] = code;
        d.blk_b[b] = zerr;
        d.blk_out_len[b] = 0;
      } else {
        d.blk_out_len[b] = (unsigned long long)olen;
      }
    }
  }
}


uint64_t zstd_grid(int ncu) { return (uint64_t)ncu * kZWaves; }
uint64_t zstd_lit_bytes(uint64_t grid) { return grid * kZLitStride; }

// entropy pass -> sequence pass -> fix-up pass -> execution pass -> exact serial
// decoder (blocks declined or found corrupt on the way)
void launch_zstd(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks,
                 uint64_t dec_cap, uint64_t grid, hipStream_t st) {
  uint64_t g = max_blocks < grid ? max_blocks : grid;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(k_zstd_ent, dim3((unsigned)g), dim3(64), 0, st, span, d, nblocks, dec_cap);
  // 4-wave workgroups sharing the CU's LDS (kZs2Groups per CU)
  if (RIO_ZS2_QUAD)
    hipLaunchKernelGGL(k_zstd_seq4, dim3((unsigned)(grid / kZWaves * kZs2Groups)), dim3(256), 0, st, d);
  else
    hipLaunchKernelGGL(k_zstd_seq2, dim3((unsigned)(grid / kZWaves * kZs2Groups)), dim3(256), 0, st, d);
  uint64_t g3 = grid / kZWaves * kZFixWaves;
  if (g3 > max_blocks) g3 = max_blocks;
  if (g3 < 1) g3 = 1;
  hipLaunchKernelGGL(k_zstd_fix, dim3((unsigned)g3), dim3(64), 0, st, d, nblocks);
  uint64_t g2 = grid / kZWaves * kZExecWaves;
  if (g2 > max_blocks) g2 = max_blocks;
  if (g2 < 1) g2 = 1;
  hipLaunchKernelGGL(k_zstd_exec, dim3((unsigned)g2), dim3(64), 0, st, d, nblocks);
  hipLaunchKernelGGL(k_zstd, dim3((unsigned)g), dim3(64), 0, st, span, d, nblocks, dec_cap);
}

}  // namespace rio
