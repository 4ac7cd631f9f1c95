// The exact zstd decoder of the serial path (k_zstd, codec_zstd.hip): every
// block the fast passes decline or find corrupt is decoded here, by lane 0 of
// its wave, with the semantics of the library the reference links --
// libzstd's one-shot ZSTD_decompress (DataDog/zstd v1.4.1 through
// compress/zstd/zstd_cgo.go:34-41) -- so that accept / reject, the bytes of an
// accepted frame and the error name are libzstd's, not the strictest reading
// of RFC 8878:
//  - the multi-frame loop (trailing bytes < 5 / garbage after a frame read as
//    srcSize_wrong), skippable frames, a frame needs >= 9 bytes;
//  - no block-size or window limits in one-shot decoding; compressed blocks of
//    >= 128 KiB are srcSize_wrong;
//  - the bit reader as a 64-bit container (BIT_DStream_t): reads below the
//    stream start are zero bits, reads after an over-read use libzstd's
//    getMiddleBits / lookBitsFast shift arithmetic;
//  - Huffman table logs up to 12 with libzstd's weight checks; single-stream
//    literals with the single-symbol decoder; four-stream literals with the
//    single- or double-symbol decoder picked by HUF_selectDecoder, the double
//    decoder's 12-bit table, its last-symbol clamp and lockstep checks;
//  - FSE table descriptions read by FSE_readNCount's byte-window arithmetic;
//  - sequences: the modes byte's reserved bits ignored, a block without
//    sequences must end at its count, every FSE state updated after every
//    sequence (the last included), the stream accepted once exhausted or
//    over-read, a repeat offset of 0 forced to 1; the long-offset decoder's
//    stop rule for windows above 16 MiB.
// It restates the same behaviour as the CPU oracle (oracle/zstd_dec.c, the
// checker), which tests/test_zstd_libzstd.py pins against libzstd 1.4.9.
// Throughput is irrelevant here (corrupt or unusual blocks only); all large
// state lives in the block's scratch region in HBM.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rio {
namespace zx {

constexpr int kBlockMax = 128 * 1024;
constexpr int kHufLog = 12;  // HUF_TABLELOG_MAX (the DCtx's HufLog)
constexpr uint32_t kMagic = 0xFD2FB528u;

// error results (codec.hip names them; kFull: the decode region is too small)
enum : uint32_t { kOk = 0, kSrc = 1, kPrefix = 2, kCorrupt = 3, kChecksum = 4, kDict = 5, kWindow = 6, kNotSup = 7,
                  kDictCorrupted = 8, kFull = 100 };

struct SeqCell {
  uint16_t next;
  uint8_t nbits, nb_add;
  uint32_t base;
};
struct SeqTab {
  uint32_t log;
  SeqCell t[1 << 9];
};
struct Huf {
  uint32_t type, log;  // type 0: single-symbol (log = code log), 1: double-symbol (log = 12)
  uint8_t s1[1 << kHufLog], nb1[1 << kHufLog];
  uint8_t seq0[1 << kHufLog], seq1[1 << kHufLog], nb2[1 << kHufLog], len2[1 << kHufLog];
};
struct Sorted {
  uint8_t symbol, weight;
};
// decoder state (~64 KiB), in the block's scratch region
struct State {
  Huf huf;
  SeqTab ll_t, of_t, ml_t, ll_def, of_def, ml_def;
  // scratch of the table builders
  uint8_t w[260];
  Sorted sorted[256];
  uint32_t rank_val[kHufLog][kHufLog + 1];
  uint8_t sym[1 << 9], nb[1 << 9];
  uint16_t ns[1 << 9];
  uint16_t next[256];
  int16_t norm[256];
};
constexpr uint64_t kStateBytes = (sizeof(State) + 255) & ~255ull;

struct Ctx {
  State *s;
  const uint8_t *in;
  uint8_t *out;
  int64_t cap, olen, frame_start;
  uint64_t window;
  uint8_t *lit;  // kBlockMax + slack
  int lit_entropy, fse_entropy;
  const SeqTab *ll, *of, *ml;
  uint32_t rep[3];
  uint32_t err;
};

__device__ __forceinline__ uint32_t rd16(const uint8_t *p) { return p[0] | ((uint32_t)p[1] << 8); }
__device__ __forceinline__ uint32_t rd24(const uint8_t *p) { return rd16(p) | ((uint32_t)p[2] << 16); }
__device__ __forceinline__ uint32_t rd32(const uint8_t *p) { return rd16(p) | (rd16(p + 2) << 16); }
__device__ __forceinline__ uint64_t rd64(const uint8_t *p) { return rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
__device__ __forceinline__ int hb32(uint32_t v) { return 31 - __clz(v); }

// ---------------------------------------------------------------- BIT_DStream_t
struct Bit {
  uint64_t c;
  uint32_t bc;
  const uint8_t *ptr, *start, *limit;
};
enum { kUnfinished = 0, kEndOfBuffer = 1, kCompleted = 2, kOverflow = 3 };

__device__ bool bit_init(Bit &b, const uint8_t *src, uint64_t n) {
  b.c = 0;
  b.bc = 0;
  b.ptr = b.start = b.limit = src;
  if (n < 1) return false;
  b.limit = src + 8;
  const uint8_t last = src[n - 1];
  if (n >= 8) {
    b.ptr = src + n - 8;
    b.c = rd64(b.ptr);
    b.bc = last ? 8 - (uint32_t)hb32(last) : 0;
  } else {
    for (uint64_t k = 0; k < n; k++) b.c |= (uint64_t)src[k] << (8 * k);
    b.bc = last ? 8 - (uint32_t)hb32(last) + (uint32_t)(8 - n) * 8 : 0;
  }
  return last != 0;
}
__device__ __forceinline__ uint64_t bit_look(const Bit &b, uint32_t nb) {  // BIT_getMiddleBits
  const uint32_t st = 64u - b.bc - nb;
  return (b.c >> (st & 63)) & ((1ull << nb) - 1);
}
__device__ __forceinline__ uint64_t bit_look_fast(const Bit &b, uint32_t nb) {
  return (b.c << (b.bc & 63)) >> ((64 - nb) & 63);
}
__device__ __forceinline__ uint64_t bit_read(Bit &b, uint32_t nb) {
  const uint64_t v = bit_look(b, nb);
  b.bc += nb;
  return v;
}
__device__ __forceinline__ uint64_t bit_read_fast(Bit &b, uint32_t nb) {
  const uint64_t v = bit_look_fast(b, nb);
  b.bc += nb;
  return v;
}
__device__ int bit_reload(Bit &b) {
  if (b.bc > 64) return kOverflow;
  if (b.ptr >= b.limit) {
    b.ptr -= b.bc >> 3;
    b.bc &= 7;
    b.c = rd64(b.ptr);
    return kUnfinished;
  }
  if (b.ptr == b.start) return b.bc < 64 ? kEndOfBuffer : kCompleted;
  uint32_t nbytes = b.bc >> 3;
  int r = kUnfinished;
  if (b.ptr - nbytes < b.start) {
    nbytes = (uint32_t)(b.ptr - b.start);
    r = kEndOfBuffer;
  }
  b.ptr -= nbytes;
  b.bc -= nbytes * 8;
  b.c = rd64(b.ptr);
  return r;
}
__device__ __forceinline__ int bit_reload_fast(Bit &b) {
  if (b.ptr < b.limit) return kOverflow;
  b.ptr -= b.bc >> 3;
  b.bc &= 7;
  b.c = rd64(b.ptr);
  return kUnfinished;
}
__device__ __forceinline__ bool bit_end(const Bit &b) { return b.ptr == b.start && b.bc == 64; }

// ---------------------------------------------------------------- FSE_readNCount
__device__ int64_t read_ncount_body(int16_t *norm, uint32_t *max_sv, uint32_t *tlog, const uint8_t *src, uint64_t n) {
  const int64_t iend = (int64_t)n;
  int64_t ip = 0;
  for (uint32_t s = 0; s <= *max_sv; s++) norm[s] = 0;
  uint32_t bs = rd32(src);
  int nbits = (int)(bs & 0xF) + 5;
  if (nbits > 15) return -1;
  bs >>= 4;
  int bit_count = 4;
  *tlog = (uint32_t)nbits;
  int remaining = (1 << nbits) + 1;
  int threshold = 1 << nbits;
  nbits++;
  uint32_t charnum = 0;
  int previous0 = 0;
  while ((remaining > 1) & (charnum <= *max_sv)) {
    if (previous0) {
      uint32_t n0 = charnum;
      while ((bs & 0xFFFF) == 0xFFFF) {
        n0 += 24;
        if (ip < iend - 5) {
          ip += 2;
          bs = rd32(src + ip) >> bit_count;
        } else {
          bs >>= 16;
          bit_count += 16;
        }
      }
      while ((bs & 3) == 3) {
        n0 += 3;
        bs >>= 2;
        bit_count += 2;
      }
      n0 += bs & 3;
      bit_count += 2;
      if (n0 > *max_sv) return -1;
      while (charnum < n0) norm[charnum++] = 0;
      if ((ip <= iend - 7) || (ip + (bit_count >> 3) <= iend - 4)) {
        ip += bit_count >> 3;
        bit_count &= 7;
        bs = rd32(src + ip) >> bit_count;
      } else {
        bs >>= 2;
      }
    }
    const int max = (2 * threshold - 1) - remaining;
    int count;
    if ((int)(bs & (uint32_t)(threshold - 1)) < max) {
      count = (int)(bs & (uint32_t)(threshold - 1));
      bit_count += nbits - 1;
    } else {
      count = (int)(bs & (uint32_t)(2 * threshold - 1));
      if (count >= threshold) count -= max;
      bit_count += nbits;
    }
    count--;
    remaining -= count < 0 ? -count : count;
    norm[charnum++] = (int16_t)count;
    previous0 = !count;
    while (remaining < threshold) {
      nbits--;
      threshold >>= 1;
    }
    if ((ip <= iend - 7) || (ip + (bit_count >> 3) <= iend - 4)) {
      ip += bit_count >> 3;
      bit_count &= 7;
    } else {
      bit_count -= (int)(8 * (iend - 4 - ip));
      ip = iend - 4;
    }
    bs = rd32(src + ip) >> (bit_count & 31);
  }
  if (remaining != 1) return -1;
  if (bit_count > 32) return -1;
  *max_sv = charnum - 1;
  ip += (bit_count + 7) >> 3;
  return ip;
}
__device__ int64_t read_ncount(int16_t *norm, uint32_t *max_sv, uint32_t *tlog, const uint8_t *src, uint64_t n) {
  if (n >= 4) return read_ncount_body(norm, max_sv, tlog, src, n);
  uint8_t pad[4];  // fewer than 4 bytes: read a zero-padded copy
  for (int i = 0; i < 4; i++) pad[i] = (uint64_t)i < n ? src[i] : 0;
  const int64_t k = read_ncount_body(norm, max_sv, tlog, pad, 4);
  return (k < 0 || (uint64_t)k > n) ? -1 : k;
}

// symbol spread + next states (FSE_buildDTable / ZSTD_buildFSETable); false if the spread does not close
__device__ bool spread(State *s, const int16_t *norm, uint32_t max_sv, uint32_t tlog) {
  const uint32_t size = 1u << tlog;
  uint32_t high = size - 1;
  for (uint32_t k = 0; k <= max_sv; k++) {
    if (norm[k] == -1) {
      s->sym[high--] = (uint8_t)k;
      s->next[k] = 1;
    } else {
      s->next[k] = (uint16_t)norm[k];
    }
  }
  const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  uint32_t pos = 0;
  for (uint32_t k = 0; k <= max_sv; k++)
    for (int i = 0; i < norm[k]; i++) {
      s->sym[pos] = (uint8_t)k;
      pos = (pos + step) & mask;
      while (pos > high) pos = (pos + step) & mask;
    }
  for (uint32_t u = 0; u < size; u++) {
    const uint32_t ns = s->next[s->sym[u]]++;
    s->nb[u] = (uint8_t)(tlog - (uint32_t)hb32(ns));
    s->ns[u] = (uint16_t)((ns << s->nb[u]) - size);
  }
  return pos == 0;
}

// ---------------------------------------------------------------- Huffman
// HUF_readStats; bytes consumed or -1
__device__ int64_t read_stats(State *s, uint32_t *rank, uint32_t *nsym, uint32_t *tlog, const uint8_t *src,
                              uint64_t n) {
  uint8_t *w = s->w;
  if (!n) return -1;
  uint64_t isize = src[0], osize;
  if (isize >= 128) {
    osize = isize - 127;
    isize = (osize + 1) / 2;
    if (isize + 1 > n || osize >= 256) return -1;
    for (uint64_t k = 0; k < osize; k += 2) {
      w[k] = src[1 + k / 2] >> 4;
      w[k + 1] = src[1 + k / 2] & 15;
    }
  } else {
    if (isize + 1 > n) return -1;
    const uint8_t *c = src + 1;
    uint64_t cn = isize;
    uint32_t max_sv = 255, log;
    const int64_t k = read_ncount(s->norm, &max_sv, &log, c, cn);
    if (k < 0 || log > 6) return -1;
    c += k;
    cn -= (uint64_t)k;
    if (!spread(s, s->norm, max_sv, log)) return -1;
    Bit b;
    if (!bit_init(b, c, cn)) return -1;
    uint32_t st1 = (uint32_t)bit_read(b, log);
    bit_reload(b);
    uint32_t st2 = (uint32_t)bit_read(b, log);
    bit_reload(b);
    uint64_t op = 0;
    const uint64_t omax = 255, olimit = omax - 3;
    auto sym = [&](uint32_t &st) -> uint8_t {
      const uint8_t v = s->sym[st];
      st = s->ns[st] + (uint32_t)bit_read(b, s->nb[st]);
      return v;
    };
    for (; (bit_reload(b) == kUnfinished) & (op < olimit); op += 4) {
      w[op] = sym(st1);
      w[op + 1] = sym(st2);
      w[op + 2] = sym(st1);
      w[op + 3] = sym(st2);
    }
    for (;;) {
      if (op > omax - 2) return -1;
      w[op++] = sym(st1);
      if (bit_reload(b) == kOverflow) {
        w[op++] = sym(st2);
        break;
      }
      if (op > omax - 2) return -1;
      w[op++] = sym(st2);
      if (bit_reload(b) == kOverflow) {
        w[op++] = sym(st1);
        break;
      }
    }
    osize = op;
  }
  for (int k = 0; k <= kHufLog; k++) rank[k] = 0;
  uint32_t total = 0;
  for (uint64_t k = 0; k < osize; k++) {
    if (w[k] >= kHufLog) return -1;
    rank[w[k]]++;
    total += (1u << w[k]) >> 1;
  }
  if (total == 0) return -1;
  const uint32_t log = (uint32_t)hb32(total) + 1;
  if (log > kHufLog) return -1;
  *tlog = log;
  const uint32_t rest = (1u << log) - total;
  if ((1u << hb32(rest)) != rest) return -1;
  const uint32_t lastw = (uint32_t)hb32(rest) + 1;
  w[osize] = (uint8_t)lastw;
  rank[lastw]++;
  if (rank[1] < 2 || (rank[1] & 1)) return -1;
  *nsym = (uint32_t)osize + 1;
  return (int64_t)isize + 1;
}

__device__ int64_t read_x1(State *s, const uint8_t *src, uint64_t n) {
  uint32_t rank[kHufLog + 1], nsym, log;
  const int64_t isize = read_stats(s, rank, &nsym, &log, src, n);
  if (isize < 0) return -1;
  Huf &h = s->huf;
  h.type = 0;
  h.log = log;
  uint32_t next = 0;
  for (uint32_t k = 1; k < log + 1; k++) {
    const uint32_t cur = next;
    next += rank[k] << (k - 1);
    rank[k] = cur;
  }
  for (uint32_t sy = 0; sy < nsym; sy++) {
    const uint32_t wt = s->w[sy], len = (1u << wt) >> 1, st = rank[wt];
    for (uint32_t u = st; u < st + len; u++) {
      h.s1[u] = (uint8_t)sy;
      h.nb1[u] = (uint8_t)(log + 1 - wt);
    }
    rank[wt] = st + len;
  }
  return isize;
}

__device__ void x2_level2(Huf &h, uint32_t base, uint32_t size_log, uint32_t consumed, const uint32_t *rank_origin,
                          int min_weight, const Sorted *sorted, uint32_t nsorted, uint32_t nb_baseline,
                          uint8_t base_seq) {
  uint32_t rv[kHufLog + 1];
  for (int k = 0; k <= kHufLog; k++) rv[k] = rank_origin[k];
  if (min_weight > 1) {
    const uint32_t skip = rv[min_weight];
    for (uint32_t i = 0; i < skip; i++) {
      h.seq0[base + i] = base_seq;
      h.seq1[base + i] = 0;
      h.nb2[base + i] = (uint8_t)consumed;
      h.len2[base + i] = 1;
    }
  }
  for (uint32_t k = 0; k < nsorted; k++) {
    const uint32_t nb = nb_baseline - sorted[k].weight;
    const uint32_t len = 1u << (size_log - nb), st = rv[sorted[k].weight];
    for (uint32_t i = st; i < st + len; i++) {
      h.seq0[base + i] = base_seq;
      h.seq1[base + i] = sorted[k].symbol;
      h.nb2[base + i] = (uint8_t)(nb + consumed);
      h.len2[base + i] = 2;
    }
    rv[sorted[k].weight] += len;
  }
}

__device__ int64_t read_x2(State *s, const uint8_t *src, uint64_t n) {
  uint32_t rank_stats[kHufLog + 1], nsym, log;
  const int64_t isize = read_stats(s, rank_stats, &nsym, &log, src, n);
  if (isize < 0) return -1;
  const uint32_t max_log = kHufLog;
  uint32_t max_w = log;
  while (rank_stats[max_w] == 0) max_w--;
  uint32_t rank_start0[kHufLog + 2];
  for (int k = 0; k < kHufLog + 2; k++) rank_start0[k] = 0;
  uint32_t *rank_start = rank_start0 + 1;
  uint32_t next = 0;
  for (uint32_t k = 1; k < max_w + 1; k++) {
    const uint32_t cur = next;
    next += rank_stats[k];
    rank_start[k] = cur;
  }
  rank_start[0] = next;
  const uint32_t nsort = next;
  for (uint32_t sy = 0; sy < nsym; sy++) {
    const uint32_t r = rank_start[s->w[sy]]++;
    s->sorted[r].symbol = (uint8_t)sy;
    s->sorted[r].weight = s->w[sy];
  }
  rank_start[0] = 0;
  for (int a = 0; a < kHufLog; a++)
    for (int k = 0; k <= kHufLog; k++) s->rank_val[a][k] = 0;
  {
    const int rescale = (int)(max_log - log) - 1;
    uint32_t nrv = 0;
    for (uint32_t k = 1; k < max_w + 1; k++) {
      const uint32_t cur = nrv;
      nrv += rank_stats[k] << (k + rescale);
      s->rank_val[0][k] = cur;
    }
    const uint32_t min_bits = log + 1 - max_w;
    for (uint32_t consumed = min_bits; consumed < max_log - min_bits + 1; consumed++)
      for (uint32_t k = 1; k < max_w + 1; k++) s->rank_val[consumed][k] = s->rank_val[0][k] >> consumed;
  }
  Huf &h = s->huf;
  const uint32_t nb_baseline = log + 1;
  const int scale_log = (int)nb_baseline - (int)max_log;
  const uint32_t min_bits = nb_baseline - max_w;
  uint32_t rv[kHufLog + 1];
  for (int k = 0; k <= kHufLog; k++) rv[k] = s->rank_val[0][k];
  for (uint32_t k = 0; k < nsort; k++) {
    const uint8_t symbol = s->sorted[k].symbol;
    const uint32_t weight = s->sorted[k].weight;
    const uint32_t nb = nb_baseline - weight;
    const uint32_t start = rv[weight];
    const uint32_t len = 1u << (max_log - nb);
    if (max_log - nb >= min_bits) {
      int min_weight = (int)nb + scale_log;
      if (min_weight < 1) min_weight = 1;
      const uint32_t sorted_rank = rank_start0[min_weight];
      x2_level2(h, start, max_log - nb, nb, s->rank_val[nb], min_weight, s->sorted + sorted_rank,
                nsort - sorted_rank, nb_baseline, symbol);
    } else {
      for (uint32_t u = start; u < start + len; u++) {
        h.seq0[u] = symbol;
        h.seq1[u] = 0;
        h.nb2[u] = (uint8_t)nb;
        h.len2[u] = 1;
      }
    }
    rv[weight] += len;
  }
  h.type = 1;
  h.log = max_log;
  return isize;
}

// HUF_selectDecoder's timing model (Q: compression ratio in 16ths)
__constant__ uint16_t kAlgoTime[16][2][2] = {
      {{0, 0}, {1, 1}},           {{0, 0}, {1, 1}},           {{38, 130}, {1313, 74}},    {{448, 128}, {1353, 74}},
      {{556, 128}, {1353, 74}},   {{714, 128}, {1418, 74}},   {{883, 128}, {1437, 74}},   {{897, 128}, {1515, 75}},
      {{926, 128}, {1613, 75}},   {{947, 128}, {1729, 77}},   {{1107, 128}, {2083, 81}},  {{1177, 128}, {2379, 87}},
      {{1242, 128}, {2415, 93}},  {{1349, 128}, {2644, 106}}, {{1455, 128}, {2422, 124}}, {{722, 128}, {1891, 145}},
};
__device__ bool select_x2(uint64_t dst, uint64_t csrc) {
  const uint16_t(*t)[2][2] = kAlgoTime;
  const uint32_t q = csrc >= dst ? 15 : (uint32_t)(csrc * 16 / dst);
  const uint32_t d256 = (uint32_t)(dst >> 8);
  const uint32_t t0 = t[q][0][0] + t[q][0][1] * d256;
  uint32_t t1 = t[q][1][0] + t[q][1][1] * d256;
  t1 += t1 >> 3;
  return t1 < t0;
}

__device__ __forceinline__ void x1_sym(const Huf &h, Bit &b, uint8_t *lit, int64_t &p) {
  const uint64_t v = bit_look_fast(b, h.log);
  lit[p] = h.s1[v];
  b.bc += h.nb1[v];
  p++;
}
__device__ __forceinline__ void x2_sym(const Huf &h, Bit &b, uint8_t *lit, int64_t &p) {
  const uint64_t v = bit_look_fast(b, h.log);
  lit[p] = h.seq0[v];
  lit[p + 1] = h.seq1[v];
  b.bc += h.nb2[v];
  p += h.len2[v];
}
__device__ void x1_stream(const Huf &h, Bit &b, uint8_t *lit, int64_t p, int64_t end) {
  while ((bit_reload(b) == kUnfinished) & (p < end - 3)) {
    x1_sym(h, b, lit, p);
    x1_sym(h, b, lit, p);
    x1_sym(h, b, lit, p);
    x1_sym(h, b, lit, p);
  }
  while (p < end) x1_sym(h, b, lit, p);
}
__device__ void x2_stream(const Huf &h, Bit &b, uint8_t *lit, int64_t p, int64_t end) {
  while ((bit_reload(b) == kUnfinished) & (p < end - 7)) {
    x2_sym(h, b, lit, p);
    x2_sym(h, b, lit, p);
    x2_sym(h, b, lit, p);
    x2_sym(h, b, lit, p);
  }
  while ((bit_reload(b) == kUnfinished) & (p <= end - 2)) x2_sym(h, b, lit, p);
  while (p <= end - 2) x2_sym(h, b, lit, p);
  if (p < end) {
    const uint64_t v = bit_look_fast(b, h.log);
    lit[p] = h.seq0[v];
    if (h.len2[v] == 1) {
      b.bc += h.nb2[v];
    } else if (b.bc < 64) {
      b.bc += h.nb2[v];
      if (b.bc > 64) b.bc = 64;
    }
  }
}
__device__ bool huf_1x(const Huf &h, uint8_t *lit, uint64_t dst, const uint8_t *src, uint64_t n) {
  Bit b;
  if (!bit_init(b, src, n)) return false;
  if (h.type == 0) x1_stream(h, b, lit, 0, (int64_t)dst);
  else x2_stream(h, b, lit, 0, (int64_t)dst);
  return bit_end(b);
}
__device__ bool huf_4x(const Huf &h, uint8_t *lit, uint64_t dst, const uint8_t *src, uint64_t n) {
  if (n < 10) return false;
  const uint64_t l1 = rd16(src), l2 = rd16(src + 2), l3 = rd16(src + 4);
  const uint64_t l4 = n - (l1 + l2 + l3 + 6);
  if (l4 > n) return false;
  const uint8_t *i1 = src + 6, *i2 = i1 + l1, *i3 = i2 + l2, *i4 = i3 + l3;
  const int64_t seg = (int64_t)(dst + 3) / 4, oend = (int64_t)dst;
  int64_t op[4] = {0, seg, 2 * seg, 3 * seg};
  const int64_t ost[5] = {0, seg, 2 * seg, 3 * seg, oend};
  Bit b[4];
  if (!bit_init(b[0], i1, l1) || !bit_init(b[1], i2, l2) || !bit_init(b[2], i3, l3) || !bit_init(b[3], i4, l4))
    return false;
  if (h.type == 0) {
    int sig = 1;
    for (; sig & (op[3] < oend - 3);) {
      for (int k = 0; k < 4; k++)
        for (int j = 0; j < 4; j++) x1_sym(h, b[k], lit, op[k]);
      for (int k = 0; k < 4; k++) sig &= bit_reload_fast(b[k]) == kUnfinished;
    }
    for (int k = 0; k < 3; k++)
      if (op[k] > ost[k + 1]) return false;
    for (int k = 0; k < 4; k++) x1_stream(h, b[k], lit, op[k], ost[k + 1]);
  } else {
    int sig = 1;
    for (; sig & (op[3] < oend - 7);) {
      for (int j = 0; j < 4; j++)  // the streams interleaved symbol by symbol (2-byte writes may spill)
        for (int k = 0; k < 4; k++) x2_sym(h, b[k], lit, op[k]);
      int all = 1;
      for (int k = 0; k < 4; k++) all &= bit_reload_fast(b[k]) == kUnfinished;
      sig = all;
    }
    for (int k = 0; k < 3; k++)
      if (op[k] > ost[k + 1]) return false;
    for (int k = 0; k < 4; k++) x2_stream(h, b[k], lit, op[k], ost[k + 1]);
  }
  return bit_end(b[0]) & bit_end(b[1]) & bit_end(b[2]) & bit_end(b[3]);
}

// ---------------------------------------------------------------- sequences
// the code tables: kLLBase / kLLBits / kMLBase / kMLBits (codec_zstd.hip, __constant__)
__device__ __forceinline__ uint32_t ll_base(uint32_t s) { return kLLBase[s]; }
__device__ __forceinline__ uint8_t ll_bits(uint32_t s) { return kLLBits[s]; }
__device__ __forceinline__ uint32_t ml_base(uint32_t s) { return kMLBase[s]; }
__device__ __forceinline__ uint8_t ml_bits(uint32_t s) { return kMLBits[s]; }
enum { kLL = 0, kOF = 1, kML = 2 };
__device__ __forceinline__ void cell_value(SeqCell &c, uint32_t s, int kind) {
  if (kind == kOF) {
    c.nb_add = (uint8_t)s;
    c.base = s < 2 ? s : (1u << s) - 3;
  } else if (kind == kLL) {
    c.nb_add = ll_bits(s);
    c.base = ll_base(s);
  } else {
    c.nb_add = ml_bits(s);
    c.base = ml_base(s);
  }
}
__device__ void seq_build(State *s, SeqTab &t, const int16_t *norm, uint32_t max_sv, uint32_t tlog, int kind) {
  spread(s, norm, max_sv, tlog);  // (ZSTD_buildFSETable does not check the spread)
  t.log = tlog;
  for (uint32_t u = 0; u < (1u << tlog); u++) {
    t.t[u].next = s->ns[u];
    t.t[u].nbits = s->nb[u];
    cell_value(t.t[u], s->sym[u], kind);
  }
}
__device__ void build_defaults(State *s) {  // the predefined distributions (kLLDef / kOFDef / kMLDef)
  for (int k = 0; k < 36; k++) s->norm[k] = kLLDef[k];
  seq_build(s, s->ll_def, s->norm, 35, 6, kLL);
  for (int k = 0; k < 29; k++) s->norm[k] = kOFDef[k];
  seq_build(s, s->of_def, s->norm, 28, 5, kOF);
  for (int k = 0; k < 53; k++) s->norm[k] = kMLDef[k];
  seq_build(s, s->ml_def, s->norm, 52, 6, kML);
}

// ZSTD_buildSeqTable; false = corruption
__device__ bool seq_table(Ctx &z, SeqTab &space, const SeqTab &def, const SeqTab *&cur, int type, const uint8_t *src,
                          uint64_t n, uint64_t &used, uint32_t max, uint32_t max_log, int kind) {
  used = 0;
  if (type == 1) {
    if (!n || src[0] > max) return false;
    space.log = 0;
    space.t[0].next = 0;
    space.t[0].nbits = 0;
    cell_value(space.t[0], src[0], kind);
    cur = &space;
    used = 1;
    return true;
  }
  if (type == 0) {
    cur = &def;
    return true;
  }
  if (type == 3) return z.fse_entropy != 0;
  uint32_t ms = max, log;
  const int64_t k = read_ncount(z.s->norm, &ms, &log, src, n);
  if (k < 0 || log > max_log) return false;
  seq_build(z.s, space, z.s->norm, ms, log, kind);
  cur = &space;
  used = (uint64_t)k;
  return true;
}

struct Seq {
  uint64_t ll, ml, off;
};
__device__ Seq decode_seq(Ctx &z, Bit &b, uint32_t &sll, uint32_t &sml, uint32_t &sof, uint64_t *rep) {
  const SeqCell lli = z.ll->t[sll], mli = z.ml->t[sml], ofi = z.of->t[sof];
  Seq q;
  const uint32_t llb = lli.nb_add, mlb = mli.nb_add, ofb = ofi.nb_add;
  uint64_t off;
  if (ofb > 1) {
    off = ofi.base + bit_read_fast(b, ofb);
    rep[2] = rep[1];
    rep[1] = rep[0];
    rep[0] = off;
  } else {
    const uint32_t ll0 = lli.base == 0;
    if (ofb == 0) {
      if (!ll0) {
        off = rep[0];
      } else {
        off = rep[1];
        rep[1] = rep[0];
        rep[0] = off;
      }
    } else {
      off = ofi.base + ll0 + bit_read_fast(b, 1);
      uint64_t t = (off == 3) ? rep[0] - 1 : rep[off];
      t += !t;
      if (off != 1) rep[2] = rep[1];
      rep[1] = rep[0];
      rep[0] = off = t;
    }
  }
  q.off = off;
  q.ml = mli.base + (mlb ? bit_read_fast(b, mlb) : 0);
  if (llb + mlb + ofb >= 57 - (9 + 9 + 8)) bit_reload(b);
  q.ll = lli.base + (llb ? bit_read_fast(b, llb) : 0);
  sll = lli.next + (uint32_t)bit_read(b, lli.nbits);
  sml = mli.next + (uint32_t)bit_read(b, mli.nbits);
  sof = ofi.next + (uint32_t)bit_read(b, ofi.nbits);
  return q;
}
// ZSTD_execSequence with a buffer that grows as needed (DataDog retries
// dstSize_tooSmall with larger buffers): false = corruption. Output past `cap`
// is not written (full: the host retries with more room) but still counted,
// so that the checks of later sequences see the unlimited buffer's positions.
__device__ bool exec_seq(Ctx &z, const Seq &q, uint64_t &lit_pos, uint64_t lit_size, bool &full) {
  if (q.ll > lit_size - lit_pos) return false;
  const int64_t produced = z.olen + (int64_t)q.ll - z.frame_start;
  if (q.off > (uint64_t)produced) return false;
  if (q.ll + q.ml < q.ll || z.olen + (int64_t)(q.ll + q.ml) > z.cap) full = true;
  if (!full) {
    for (uint64_t k = 0; k < q.ll; k++) z.out[z.olen + (int64_t)k] = z.lit[lit_pos + k];
    const int64_t m = z.olen + (int64_t)q.ll;
    for (uint64_t k = 0; k < q.ml; k++) z.out[m + (int64_t)k] = z.out[m - (int64_t)q.off + (int64_t)k];
  }
  z.olen += (int64_t)(q.ll + q.ml);
  lit_pos += q.ll;
  return true;
}

// ZSTD_decompressBlock_internal: kOk, an error, or kFull
__device__ uint32_t decode_block(Ctx &z, const uint8_t *src, uint64_t n) {
  if (n >= (uint64_t)kBlockMax) return kSrc;
  if (n < 3) return kCorrupt;
  const int lt = src[0] & 3, lhl = (src[0] >> 2) & 3;
  uint64_t lit_size, lit_csize;
  if (lt == 2 || lt == 3) {
    if (lt == 3 && !z.lit_entropy) return kDictCorrupted;
    if (n < 5) return kCorrupt;
    uint64_t lh;
    bool single = false;
    const uint32_t lhc = rd32(src);
    if (lhl < 2) {
      single = !lhl;
      lh = 3;
      lit_size = (lhc >> 4) & 0x3FF;
      lit_csize = (lhc >> 14) & 0x3FF;
    } else if (lhl == 2) {
      lh = 4;
      lit_size = (lhc >> 4) & 0x3FFF;
      lit_csize = lhc >> 18;
    } else {
      lh = 5;
      lit_size = (lhc >> 4) & 0x3FFFF;
      lit_csize = (lhc >> 22) + ((uint64_t)src[4] << 10);
    }
    if (lit_size > (uint64_t)kBlockMax || lit_csize + lh > n) return kCorrupt;
    const uint8_t *hs = src + lh;
    bool ok;
    if (lt == 3) {
      ok = single ? huf_1x(z.s->huf, z.lit, lit_size, hs, lit_csize) : huf_4x(z.s->huf, z.lit, lit_size, hs, lit_csize);
    } else if (single) {
      const int64_t k = read_x1(z.s, hs, lit_csize);
      ok = k >= 0 && (uint64_t)k < lit_csize && huf_1x(z.s->huf, z.lit, lit_size, hs + k, lit_csize - (uint64_t)k);
    } else {
      ok = false;
      if (lit_size != 0 && lit_csize != 0) {
        const int64_t k = select_x2(lit_size, lit_csize) ? read_x2(z.s, hs, lit_csize) : read_x1(z.s, hs, lit_csize);
        ok = k >= 0 && (uint64_t)k < lit_csize && huf_4x(z.s->huf, z.lit, lit_size, hs + k, lit_csize - (uint64_t)k);
      }
    }
    if (!ok) return kCorrupt;
    z.lit_entropy = 1;
    lit_csize += lh;
  } else {
    uint64_t lh;
    if (lhl == 1) {
      lh = 2;
      lit_size = rd16(src) >> 4;
    } else if (lhl == 3) {
      lh = 3;
      lit_size = rd24(src) >> 4;
    } else {
      lh = 1;
      lit_size = src[0] >> 3;
    }
    if (lt == 0) {
      if (lit_size + lh > n) return kCorrupt;
      for (uint64_t k = 0; k < lit_size; k++) z.lit[k] = src[lh + k];
      lit_csize = lh + lit_size;
    } else {
      if (lh == 3 && n < 4) return kCorrupt;
      if (lit_size > (uint64_t)kBlockMax) return kCorrupt;
      for (uint64_t k = 0; k < lit_size; k++) z.lit[k] = src[lh];
      lit_csize = lh + 1;
    }
  }
  // ZSTD_decodeSeqHeaders
  const uint8_t *ip = src + lit_csize, *iend = src + n;
  if (ip >= iend) return kSrc;
  int nseq = *ip++;
  if (!nseq) {
    if (iend != ip) return kSrc;
  } else {
    if (nseq > 0x7F) {
      if (nseq == 0xFF) {
        if (ip + 2 > iend) return kSrc;
        nseq = (int)rd16(ip) + 0x7F00;
        ip += 2;
      } else {
        if (ip >= iend) return kSrc;
        nseq = ((nseq - 0x80) << 8) + *ip++;
      }
    }
    if (ip + 1 > iend) return kSrc;
    const int types = *ip++;
    uint64_t used;
    State *s = z.s;
    if (!seq_table(z, s->ll_t, s->ll_def, z.ll, types >> 6, ip, (uint64_t)(iend - ip), used, 35, 9, kLL)) return kCorrupt;
    ip += used;
    if (!seq_table(z, s->of_t, s->of_def, z.of, (types >> 4) & 3, ip, (uint64_t)(iend - ip), used, 31, 8, kOF))
      return kCorrupt;
    ip += used;
    if (!seq_table(z, s->ml_t, s->ml_def, z.ml, (types >> 2) & 3, ip, (uint64_t)(iend - ip), used, 52, 9, kML))
      return kCorrupt;
    ip += used;
  }
  uint64_t lit_pos = 0;
  if (nseq) {
    uint32_t share = 0;  // ZSTD_getLongOffsetsShare
    for (uint32_t u = 0; u < (1u << z.of->log); u++) share += z.of->t[u].nb_add > 22;
    share <<= (8 - z.of->log);
    const bool long_dec = z.window > (1u << 24) && nseq > 4 && share >= 7;
    z.fse_entropy = 1;
    uint64_t rep[3] = {z.rep[0], z.rep[1], z.rep[2]};
    Bit b;
    if (!bit_init(b, ip, (uint64_t)(iend - ip))) return kCorrupt;
    uint32_t sll = (uint32_t)bit_read(b, z.ll->log);
    bit_reload(b);
    uint32_t sof = (uint32_t)bit_read(b, z.of->log);
    bit_reload(b);
    uint32_t sml = (uint32_t)bit_read(b, z.ml->log);
    bit_reload(b);
    bool full = false;
    if (!long_dec) {  // every sequence decoded and executed; errors reported after the loop
      bool err = false;
      for (int i = 0; i < nseq; i++) {
        const Seq q = decode_seq(z, b, sll, sml, sof, rep);
        const int64_t olen0 = z.olen;
        const uint64_t lp0 = lit_pos;
        if (!exec_seq(z, q, lit_pos, lit_size, full)) {  // op and the literals do not advance
          err = true;
          z.olen = olen0;
          lit_pos = lp0;
        }
        bit_reload(b);
      }
      if (err || bit_reload(b) < kCompleted) return kCorrupt;
    } else {
      Seq qs[4];
      const int adv = nseq < 4 ? nseq : 4;
      int i;
      for (i = 0; (bit_reload(b) <= kCompleted) && i < adv; i++) qs[i] = decode_seq(z, b, sll, sml, sof, rep);
      if (i < adv) return kCorrupt;
      for (; (bit_reload(b) <= kCompleted) && i < nseq; i++) {
        const Seq q = decode_seq(z, b, sll, sml, sof, rep);
        if (!exec_seq(z, qs[(i - 4) & 3], lit_pos, lit_size, full)) return kCorrupt;
        qs[i & 3] = q;
      }
      if (i < nseq) return kCorrupt;
      for (i -= adv; i < nseq; i++)
        if (!exec_seq(z, qs[i & 3], lit_pos, lit_size, full)) return kCorrupt;
    }
    if (full) return kFull;
    for (int k = 0; k < 3; k++) z.rep[k] = (uint32_t)rep[k];
  }
  if (z.olen + (int64_t)(lit_size - lit_pos) > z.cap) return kFull;
  for (uint64_t k = lit_pos; k < lit_size; k++) z.out[z.olen++] = z.lit[k];
  return kOk;
}


// ZSTD_decompressFrame: bytes consumed (>= 0) or -(error)
__device__ int64_t decode_frame(Ctx &z, const uint8_t *in, int64_t n) {
  if (n < 9) return -(int64_t)kSrc;
  const int fhd = in[4];
  const int single = (fhd >> 5) & 1, fcs_id = fhd >> 6, did_id = fhd & 3;
  const int did_len = did_id == 0 ? 0 : (did_id == 1 ? 1 : (did_id == 2 ? 2 : 4));
  const int fcs_len = fcs_id == 0 ? 0 : (fcs_id == 1 ? 2 : (fcs_id == 2 ? 4 : 8));
  const int64_t fhs = 5 + !single + did_len + fcs_len + (single && !fcs_id);
  if (n < fhs + 3) return -(int64_t)kSrc;
  if (rd32(in) != kMagic) return -(int64_t)kPrefix;
  if (fhd & 0x08) return -(int64_t)kNotSup;
  int64_t pos = 5;
  uint64_t window = 0;
  if (!single) {
    const int wd = in[pos++];
    const int wlog = 10 + (wd >> 3);
    if (wlog > 31) return -(int64_t)kWindow;
    window = 1ull << wlog;
    window += (window >> 3) * (uint64_t)(wd & 7);
  }
  uint64_t did = 0;
  for (int i = 0; i < did_len; i++) did |= (uint64_t)in[pos + i] << (8 * i);
  pos += did_len;
  uint64_t fcs = ~0ull;
  if (fcs_id == 0) {
    if (single) fcs = in[pos];
  } else if (fcs_id == 1) {
    fcs = (uint64_t)rd16(in + pos) + 256;
  } else if (fcs_id == 2) {
    fcs = rd32(in + pos);
  } else {
    fcs = rd64(in + pos);
  }
  pos = fhs;
  if (single) window = fcs;
  if (did != 0) return -(int64_t)kDict;
  const int checksum = (fhd >> 2) & 1;
  z.window = window;
  z.frame_start = z.olen;
  z.lit_entropy = z.fse_entropy = 0;
  z.rep[0] = 1;
  z.rep[1] = 4;
  z.rep[2] = 8;
  for (;;) {
    if (n - pos < 3) return -(int64_t)kSrc;
    const uint32_t bh = rd24(in + pos);
    const int last = bh & 1, type = (bh >> 1) & 3;
    const uint64_t size = bh >> 3, csize = type == 1 ? 1 : size;
    if (type == 3) return -(int64_t)kCorrupt;
    pos += 3;
    if (csize > (uint64_t)(n - pos)) return -(int64_t)kSrc;
    if (type == 0 || type == 1) {
      if (z.olen + (int64_t)size > z.cap) return -(int64_t)kFull;
      for (uint64_t k = 0; k < size; k++) z.out[z.olen + (int64_t)k] = type == 0 ? in[pos + (int64_t)k] : in[pos];
      z.olen += (int64_t)size;
    } else {
      const uint32_t e = decode_block(z, in + pos, size);
      if (e) return -(int64_t)e;
    }
    pos += (int64_t)csize;
    if (last) break;
  }
  if (fcs != ~0ull && (uint64_t)(z.olen - z.frame_start) != fcs) return -(int64_t)kCorrupt;
  if (checksum) {
    if (n - pos < 4) return -(int64_t)kChecksum;
    const uint32_t got = (uint32_t)z_xxh64(z.out + z.frame_start, (uint64_t)(z.olen - z.frame_start));
    if (rd32(in + pos) != got) return -(int64_t)kChecksum;
    pos += 4;
  }
  return pos;
}

// ZSTD_decompress (ZSTD_decompressMultiFrame) of in[0, n), n > 0: kOk, an error or kFull
__device__ uint32_t decompress(Ctx &z, int64_t n) {
  build_defaults(z.s);
  z.ll = &z.s->ll_def;
  z.of = &z.s->of_def;
  z.ml = &z.s->ml_def;
  z.olen = 0;
  int64_t pos = 0;
  bool more_than_one = false;
  while (n - pos >= 5) {
    const uint32_t magic = rd32(z.in + pos);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // readSkippableFrameSize
      if (n - pos < 8) return kSrc;
      const uint32_t sz = rd32(z.in + pos + 4);
      if ((uint32_t)(sz + 8) < sz) return kNotSup;
      if ((int64_t)sz + 8 > n - pos) return kSrc;
      pos += (int64_t)sz + 8;
      continue;
    }
    const int64_t k = decode_frame(z, z.in + pos, n - pos);
    if (k < 0) {
      const uint32_t e = (uint32_t)(-k);
      return (e == kPrefix && more_than_one) ? kSrc : e;
    }
    pos += k;
    more_than_one = true;
  }
  return n - pos != 0 ? kSrc : kOk;
}

}  // namespace zx
}  // namespace rio
