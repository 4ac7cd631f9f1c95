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
constexpr int kZWaves = 12;                          // resident zstd waves per CU (LDS ~10 KiB each)

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
// 29 predefined offset codes; 29..31 (the table's max_sym) have count 0
__constant__ int16_t kOFDef[32] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, 0, 0, 0};

struct ZLds {
  uint32_t ll[1 << 9], ml[1 << 9], of[1 << 8];  // FSE cells: sym | nbits << 8 | base << 16
  uint32_t wt[1 << 6];                           // FSE table of Huffman weights
  uint16_t huf[1 << 11];                         // Huffman: sym << 4 | nbits
  int16_t norm[64];
  uint16_t next[64];
  uint8_t w[256];
  int32_t res[12];  // lane 0's results, broadcast
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

// forward (FSE table descriptions): bits past byte n read as zero
__device__ __forceinline__ uint32_t fwd_peek(const uint8_t *p, int64_t n, uint64_t pos, int nb) {
  uint32_t v = 0;
  for (int i = 0; i < nb; i++) {
    const uint64_t b = pos + i;
    const uint32_t bit = (int64_t)(b >> 3) < n ? (p[b >> 3] >> (b & 7)) & 1u : 0u;
    v |= bit << i;
  }
  return v;
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

// one Huffman stream -> out[0, count); true iff it decodes exactly (oracle huf_stream)
__device__ bool z_huf_stream(const ZLds &L, int max_bits, const uint8_t *src, int64_t start, int64_t n, uint8_t *out,
                             int64_t count) {
  ZBwd r;
  if (!bwd_init(r, src, start, n)) return false;
  for (int64_t i = 0; i < count; i++) {
    const uint32_t e = L.huf[r.peek(max_bits)];
    out[i] = (uint8_t)(e >> 4);
    r.read((int)(e & 15));
    if (r.bit < 0) return false;
  }
  return r.bit == 0;
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
  uint8_t *out;        // decode region
  int64_t cap, olen, frame_start;
  uint8_t *lit;        // this wave's literal buffer
  int max_bits, have_huf, have_ll, have_of, have_ml;
  int ll_log, of_log, ml_log;
  uint64_t rep0, rep1, rep2;
};

// lane 0's value in every lane
__device__ __forceinline__ int32_t zbcast(ZLds &L, int slot, int32_t v) {
  zsync();
  if (lane_id() == 0) L.res[slot] = v;
  zsync();
  return L.res[slot];
}

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

// one compressed block (oracle decode_block): 0 or a ZErr
__device__ uint32_t z_decode_block(ZFrame &z, ZLds &L, int64_t bstart, int64_t n) {
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
  int64_t pos = hsz;
  if (lt == 0) {
    if (pos + regen > n) return kZCorrupt;
    for (int64_t k = l; k < regen; k += 64) z.lit[k] = src[bstart + pos + k];
    pos += regen;
  } else if (lt == 1) {
    if (pos + 1 > n) return kZCorrupt;
    const uint8_t v = src[bstart + pos];
    for (int64_t k = l; k < regen; k += 64) z.lit[k] = v;
    pos += 1;
  } else {
    if (pos + csize > n) return kZCorrupt;
    int64_t hs = bstart + pos, hn = csize;
    if (lt == 2) {
      int mb = 0, k = 0;
      if (l == 0) k = z_huf_read(L, &mb, src, hs, hn);
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
      int r = 0;
      if (l == 0) r = z_huf_stream(L, z.max_bits, src, hs, hn, z.lit, regen) ? 1 : 0;
      ok = zbcast(L, 2, r) != 0;
    } else {
      if (hn < 6) return kZCorrupt;
      const int64_t s1 = src[hs] | (src[hs + 1] << 8), s2 = src[hs + 2] | (src[hs + 3] << 8),
                    s3 = src[hs + 4] | (src[hs + 5] << 8);
      if (6 + s1 + s2 + s3 > hn) return kZCorrupt;
      const int64_t s4 = hn - 6 - s1 - s2 - s3;
      const int64_t seg = (regen + 3) / 4;
      if (3 * seg > regen) return kZCorrupt;
      // the four streams at once, one lane each (the oracle stops at the first
      // bad stream; any failure is the same error)
      int r = 1;
      if (l < 4) {
        const int64_t st = hs + 6 + (l > 0 ? s1 : 0) + (l > 1 ? s2 : 0) + (l > 2 ? s3 : 0);
        const int64_t sn = l == 0 ? s1 : l == 1 ? s2 : l == 2 ? s3 : s4;
        const int64_t cnt = l < 3 ? seg : regen - 3 * seg;
        r = z_huf_stream(L, z.max_bits, src, st, sn, z.lit + l * seg, cnt) ? 1 : 0;
      }
      ok = __ballot(r == 0) == 0;
    }
    if (!ok) return kZCorrupt;
    pos += csize;
  }
  zmem_sync();
  // sequences section
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
  int64_t lit_pos = 0;
  if (nseq > 0) {
    if (pos >= n) return kZCorrupt;
    const int modes = src[bstart + pos++];
    if (modes & 3) return kZCorrupt;
    // tables: lane 0 builds them, every lane learns the bytes used / a failure
    int u = 0, uo = 0, um = 0;
    if (l == 0) {
      u = z_seq_table(L.ll, L.next, L.norm, &z.have_ll, &z.ll_log, (modes >> 6) & 3, src, bstart + pos, n - pos,
                      kLLDef, 6, 35, 9);
      if (u >= 0)
        uo = z_seq_table(L.of, L.next, L.norm, &z.have_of, &z.of_log, (modes >> 4) & 3, src, bstart + pos + u,
                         n - pos - u, kOFDef, 5, 31, 8);
      if (u >= 0 && uo >= 0)
        um = z_seq_table(L.ml, L.next, L.norm, &z.have_ml, &z.ml_log, (modes >> 2) & 3, src, bstart + pos + u + uo,
                         n - pos - u - uo, kMLDef, 6, 52, 9);
    }
    u = zbcast(L, 0, u);
    uo = zbcast(L, 1, uo);
    um = zbcast(L, 2, um);
    z.have_ll = zbcast(L, 3, z.have_ll);
    z.have_of = zbcast(L, 4, z.have_of);
    z.have_ml = zbcast(L, 5, z.have_ml);
    z.ll_log = zbcast(L, 6, z.ll_log);
    z.of_log = zbcast(L, 7, z.of_log);
    z.ml_log = zbcast(L, 8, z.ml_log);
    if (u < 0 || uo < 0 || um < 0) return kZCorrupt;
    pos += u + uo + um;
    // the sequence bitstream, walked by every lane in step
    ZBwd r;
    if (!bwd_init(r, src, bstart + pos, n - pos)) return kZCorrupt;
    uint32_t sll = r.read(z.ll_log), sof = r.read(z.of_log), sml = r.read(z.ml_log);
    for (int64_t i = 0; i < nseq; i++) {
      const uint32_t cll = L.ll[sll], cml = L.ml[sml], cof = L.of[sof];
      const uint32_t llc = cll & 0xff, mlc = cml & 0xff, ofc = cof & 0xff;
      if (llc > 35 || mlc > 52 || ofc > 31) return kZCorrupt;
      const uint64_t ofv = (1ull << ofc) + r.read((int)ofc);
      const uint64_t ml = kMLBase[mlc] + r.read(kMLBits[mlc]);
      const uint64_t ll = kLLBase[llc] + r.read(kLLBits[llc]);
      uint64_t off;
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
      if (i + 1 < nseq) {
        sll = (cll >> 16) + r.read((cll >> 8) & 0xff);
        sml = (cml >> 16) + r.read((cml >> 8) & 0xff);
        sof = (cof >> 16) + r.read((cof >> 8) & 0xff);
      }
      if (r.bit < 0) return kZCorrupt;
      const uint32_t e = z_exec(z, ll, ml, off, lit_pos, regen);
      if (e) return e;
    }
    if (r.bit != 0) return kZCorrupt;
  }
  // remaining literals
  if (z.olen + (regen - lit_pos) > z.cap) return kZFull;
  for (int64_t k = l; k < regen - lit_pos; k += 64) z.out[z.olen + k] = z.lit[lit_pos + k];
  z.olen += regen - lit_pos;
  zmem_sync();
  return 0;
}

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

// ---------------------------------------------------------------- frame
__device__ __forceinline__ uint32_t zrd16(const uint8_t *p, int64_t i) { return p[i] | ((uint32_t)p[i + 1] << 8); }
__device__ __forceinline__ uint32_t zrd24(const uint8_t *p, int64_t i) { return zrd16(p, i) | ((uint32_t)p[i + 2] << 16); }
__device__ __forceinline__ uint32_t zrd32(const uint8_t *p, int64_t i) { return zrd16(p, i) | (zrd16(p, i + 2) << 16); }

// one frame at src[in, in + n) (oracle decode_frame): bytes consumed, or -(ZErr)
__device__ int64_t z_decode_frame(ZFrame &z, ZLds &L, int64_t in, int64_t n) {
  const int l = lane_id();
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
  for (;;) {
    if (pos + 3 > n) return -(int64_t)kZSrc;
    const uint32_t bh = zrd24(src, in + pos);
    pos += 3;
    const int last = bh & 1, type = (bh >> 1) & 3;
    const uint64_t size = bh >> 3;
    if (type == 3) return -(int64_t)kZCorrupt;
    if (size > block_max) return -(int64_t)kZCorrupt;
    if (type == 0) {
      if (pos + (int64_t)size > n) return -(int64_t)kZSrc;
      if (z.olen + (int64_t)size > z.cap) return -(int64_t)kZFull;
      for (uint64_t k = l; k < size; k += 64) z.out[z.olen + k] = src[in + pos + k];
      z.olen += (int64_t)size;
      pos += (int64_t)size;
      zmem_sync();
    } else if (type == 1) {
      if (pos + 1 > n) return -(int64_t)kZSrc;
      if (z.olen + (int64_t)size > z.cap) return -(int64_t)kZFull;
      const uint8_t v = src[in + pos];
      for (uint64_t k = l; k < size; k += 64) z.out[z.olen + k] = v;
      z.olen += (int64_t)size;
      pos += 1;
      zmem_sync();
    } else {
      if (pos + (int64_t)size > n) return -(int64_t)kZSrc;
      const uint32_t e = z_decode_block(z, L, in + pos, (int64_t)size);
      if (e) return -(int64_t)e;
      pos += (int64_t)size;
    }
    if (last) break;
  }
  if (fcs >= 0 && z.olen - z.frame_start != fcs) return -(int64_t)kZCorrupt;
  if (checksum) {
    if (pos + 4 > n) return -(int64_t)kZSrc;
    const uint32_t want = zrd32(src, in + pos);
    const uint32_t got = (uint32_t)z_xxh64(z.out + z.frame_start, (uint64_t)(z.olen - z.frame_start));
    if (want != got) return -(int64_t)kZChecksum;
    pos += 4;
  }
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

__global__ void __launch_bounds__(64) k_zstd(const uint8_t *__restrict__ span, DevBufs d,
                                             const unsigned long long *nblocks, uint64_t dec_cap) {
  __shared__ ZLds L;
  const int l = lane_id();
  const uint64_t nb = uni64(*nblocks);
  uint8_t *lit = d.zlit + (uint64_t)blockIdx.x * kZLitStride;
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
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
      // flattenIov: the chunk payloads back to back, in this block's token region
      const uint64_t total = meta & kMetaTotalMask, pay0 = uni64(d.ck_pay[c0]);
      const bool regular = (meta & kMetaRegular) != 0;
      uint32_t *flat = d.tok + c0 * (uint64_t)kTokPerChunk;
      for (uint64_t p = 4 * (uint64_t)l; p < n + 8; p += 256)
        flat[p >> 2] = z_flat_dword(span, d.ck_pay, c0, total, pay0, n, regular, p);
      zmem_sync();
      ZFrame z;
      z.src = reinterpret_cast<const uint8_t *>(flat);
      z.out = d.dec + off;
      z.cap = (int64_t)cap;
      z.olen = 0;
      z.frame_start = 0;
      z.lit = lit;
      z.max_bits = 0;
      z.have_huf = z.have_ll = z.have_of = z.have_ml = 0;
      z.ll_log = z.of_log = z.ml_log = 0;
      z.rep0 = 1;
      z.rep1 = 4;
      z.rep2 = 8;
      int64_t pos = 0;
      while (pos < (int64_t)n) {
        const int64_t k = z_decode_frame(z, L, pos, (int64_t)n - pos);
        if (k < 0) {
          zerr = (uint32_t)(-k);
          break;
        }
        pos += k;
      }
      olen = z.olen;
      if (zerr == kZFull) {  // size the retry from the declared content size
        int64_t need = z_size_bound(z.src, (int64_t)n);
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

void launch_zstd(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks,
                 uint64_t dec_cap, uint64_t grid, hipStream_t st) {
  uint64_t g = max_blocks < grid ? max_blocks : grid;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(k_zstd, dim3((unsigned)g), dim3(64), 0, st, span, d, nblocks, dec_cap);
}

}  // namespace rio
