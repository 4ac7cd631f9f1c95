// zstd frame encoding for the writer's "zstd" transformer (SURVEY.md §8(f) 1:
// the mirror of recordiozstd's zstdUncompress; the reference compresses with
// DataDog/zstd v1.4.1 = libzstd's ZSTD_compress, recordiozstd.go:31-52). Any
// valid zstd frame that libzstd decodes to the payload is a correct "zstd"
// block; these are the pieces shared by the GPU encoder (zstd_enc.hip) and its
// host checks:
//   - FSE compression tables of the three predefined sequence distributions
//     (RFC 8878 3.1.1.3.2.2; built as libzstd's FSE_buildCTable: the same
//     symbol spread as the decoder's tables, next states sorted by symbol,
//     per symbol deltaNbBits / deltaFindState);
//   - the sequence codes and extra bits (RFC 8878 3.1.1.3.2.1.1, with
//     libzstd's value-masking: every baseline is aligned to its bit range);
//   - the sequences' backward bitstream: states initialised from the last
//     sequence, then for sequences n-2 .. 0 the OF, ML, LL state transitions
//     and the LL, ML, OF extra bits, the ML, OF, LL final states and the end
//     mark -- so the decoder, reading from the end, meets the first sequence
//     first.
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

namespace rio {

constexpr int kZeLLLog = 6, kZeMLLog = 6, kZeOFLog = 5;
constexpr int kZeLLSyms = 36, kZeMLSyms = 53, kZeOFSyms = 29;
// RFC 8878 3.1.1.3.2.2 default distributions
constexpr int16_t kZeLLNorm[kZeLLSyms] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                          2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kZeMLNorm[kZeMLSyms] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                          1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                          1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kZeOFNorm[kZeOFSyms] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                          1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

__host__ __device__ __forceinline__ uint32_t ze_highbit_h(uint32_t v) { return v ? 31u - (uint32_t)__builtin_clz(v) : 0u; }

// FSE compression table of one distribution (predefined, or fitted: <= 256 cells)
constexpr int kZeMaxLog = 8;
struct ZeFse {
  uint16_t state[1 << kZeMaxLog];  // next state values (tableSize + position), sorted by symbol
  int32_t dfind[53];               // deltaFindState
  uint32_t dnb[53];                // deltaNbBits
  int32_t log;
};
struct ZeTabs {
  ZeFse ll, ml, of;
};
// scratch of one table build (the GPU encoder keeps it in LDS)
struct ZeFseWork {
  uint8_t sym_at[1 << kZeMaxLog];
  uint16_t cumul[56];
  int16_t norm[56];
};

// FSE_buildCTable for a normalized distribution (host and device, one lane)
__host__ __device__ inline void ze_build_fse(const int16_t *norm, int nsym, int log, ZeFse &t, ZeFseWork &w) {
  const int ts = 1 << log;
  uint8_t *sym_at = w.sym_at;
  uint16_t *cumul = w.cumul;
  int high = ts - 1;
  cumul[0] = 0;
  for (int u = 1; u <= nsym; u++) {
    if (norm[u - 1] == -1) {  // low-probability symbols take the table's end
      cumul[u] = (uint16_t)(cumul[u - 1] + 1);
      sym_at[high--] = (uint8_t)(u - 1);
    } else {
      cumul[u] = (uint16_t)(cumul[u - 1] + norm[u - 1]);
    }
  }
  const int step = (ts >> 1) + (ts >> 3) + 3, mask = ts - 1;
  int pos = 0;
  for (int s = 0; s < nsym; s++)
    for (int k = 0; k < norm[s]; k++) {
      sym_at[pos] = (uint8_t)s;
      pos = (pos + step) & mask;
      while (pos > high) pos = (pos + step) & mask;
    }
  for (int u = 0; u < ts; u++) t.state[cumul[sym_at[u]]++] = (uint16_t)(ts + u);
  int total = 0;
  for (int s = 0; s < nsym; s++) {
    const int n = norm[s];
    if (n == 0) {
      t.dnb[s] = (uint32_t)(((log + 1) << 16) - ts);
      t.dfind[s] = 0;
    } else if (n == -1 || n == 1) {
      t.dnb[s] = (uint32_t)((log << 16) - ts);
      t.dfind[s] = total - 1;
      total++;
    } else {
      int hb = 31;
      while (!((uint32_t)(n - 1) >> hb)) hb--;
      const int max_out = log - hb;
      const int min_plus = n << max_out;
      t.dnb[s] = (uint32_t)((max_out << 16) - min_plus);
      t.dfind[s] = total - n;
      total += n;
    }
  }
  for (int s = nsym; s < 53; s++) {
    t.dnb[s] = 0;
    t.dfind[s] = 0;
  }
  t.log = log;
}

// ---- FSE tables fitted to a block (Compressed_Mode, RFC 8878 3.1.1.3.2.1 and
// 4.1.1): counts normalized to 2^log cells, the table description written as
// the decoder reads it, the compression table built as for the predefined ones.
// Accuracy 8 (the largest every one of LL / OF / ML allows): on C3-style records
// it beats 6 by ~5 % of the output and lower accuracies never won a block.
constexpr int kZeFitLog = 8;

// counts -> normalized counts summing to 2^log, every present symbol >= 1 (no
// "less than 1" probabilities); false when more symbols are present than
// cells, or only one (the caller keeps the predefined table then)
__host__ __device__ inline bool ze_normalize(const uint32_t *cnt, int nsym, int log, int16_t *norm) {
  uint32_t total = 0, present = 0;
  for (int s = 0; s < nsym; s++) {
    total += cnt[s];
    present += cnt[s] ? 1 : 0;
  }
  const int cells = 1 << log;
  if (present < 2 || (int)present > cells) return false;
  int sum = 0, big = -1;
  for (int s = 0; s < nsym; s++) {
    if (!cnt[s]) {
      norm[s] = 0;
      continue;
    }
    // round to nearest, at least 1
    int v = (int)(((uint64_t)cnt[s] * (uint64_t)cells * 2 + total) / (2ull * total));
    if (v < 1) v = 1;
    norm[s] = (int16_t)v;
    sum += v;
    if (big < 0 || cnt[s] > cnt[big]) big = s;
  }
  // the sum back to 2^log: the difference goes to (or comes from) the largest
  // symbols, never below 1
  while (sum != cells) {
    if (sum < cells) {
      norm[big] = (int16_t)(norm[big] + (cells - sum));
      sum = cells;
    } else {
      int t = -1;  // the symbol with the most cells above 1
      for (int s = 0; s < nsym; s++)
        if (norm[s] > 1 && (t < 0 || norm[s] > norm[t])) t = s;
      if (t < 0) return false;
      const int take = (sum - cells) < norm[t] - 1 ? (sum - cells) : norm[t] - 1;
      norm[t] = (int16_t)(norm[t] - take);
      sum -= take;
    }
  }
  return true;
}

// the FSE table description (RFC 8878 4.1.1) of norm[0..nsym) at accuracy log:
// 4 bits of log - 5, then per symbol its count + 1 in a variable bit width that
// shrinks as the remaining probability does (the small values take one bit
// fewer), and after a zero-probability symbol a 2-bit repeat count of further
// zeros (3 = three more, and another repeat field). Little-endian bit order.
// Returns the bytes written.
__host__ __device__ inline uint32_t ze_write_ncount(const int16_t *norm, int nsym, int log, uint8_t *o) {
  uint64_t acc = (uint64_t)(log - 5);
  uint32_t nb = 4, pos = 0;
  auto flush = [&]() {
    while (nb >= 8) {
      o[pos++] = (uint8_t)acc;
      acc >>= 8;
      nb -= 8;
    }
  };
  int remaining = (1 << log) + 1, threshold = 1 << log, bits = log + 1;
  int s = 0;
  bool prev0 = false;
  while (s < nsym && remaining > 1) {
    if (prev0) {  // the zeros after a zero-probability symbol: 2-bit repeat counts
      int start = s;
      while (s < nsym && norm[s] == 0) s++;
      int run = s - start;
      while (run >= 3) {
        acc |= (uint64_t)3 << nb;
        nb += 2;
        run -= 3;
        flush();
      }
      acc |= (uint64_t)run << nb;
      nb += 2;
      flush();
      if (s >= nsym) break;
    }
    int c = norm[s++];
    const int mx = (2 * threshold - 1) - remaining;
    remaining -= c < 0 ? -c : c;
    c += 1;
    if (c >= threshold) c += mx;
    acc |= (uint64_t)(uint32_t)c << nb;
    nb += (uint32_t)bits;
    if (c < mx) nb -= 1;
    prev0 = c == 1;
    flush();
    while (remaining < threshold) {
      bits--;
      threshold >>= 1;
    }
  }
  if (nb) o[pos++] = (uint8_t)acc;
  return pos;
}

// cost in bits of coding cnt[] with a table of normalized counts (log cells):
// symbol s costs about log - log2(norm[s]) bits (1/256-bit steps)
__host__ __device__ inline uint64_t ze_table_cost(const uint32_t *cnt, const int16_t *norm, int nsym, int log) {
  uint64_t c = 0;
  for (int s = 0; s < nsym; s++) {
    if (!cnt[s]) continue;
    const int n = norm[s] < 0 ? 1 : norm[s];
    if (n == 0) return ~0ull;  // not codable with this table
    // 256 * (log - log2 n): log2 by the highest bit plus a linear fraction
    const uint32_t hb = ze_highbit_h((uint32_t)n);
    const uint32_t frac = (((uint32_t)n << 8) >> hb) - 256;  // 0..255
    c += (uint64_t)cnt[s] * (uint64_t)((uint32_t)log * 256 - (hb * 256 + frac));
  }
  return c;
}

// the table one block's sequence codes cnt[0..nsym) cost less with: fitted to
// them (the description at desc, its length returned, t built) or the
// predefined distribution (0 returned, t untouched). Cost = the codes' bits
// (ze_table_cost) + the description's.
__host__ __device__ inline uint32_t ze_fit_table(const uint32_t *cnt, int nsym, const int16_t *pre, int pre_nsym,
                                                 int pre_log, ZeFse &t, ZeFseWork &w, uint8_t *desc) {
  uint64_t cpre = ~0ull;
  bool pre_ok = true;
  for (int s = pre_nsym; s < nsym; s++)
    if (cnt[s]) pre_ok = false;
  if (pre_ok) cpre = ze_table_cost(cnt, pre, pre_nsym, pre_log);
  if (!ze_normalize(cnt, nsym, kZeFitLog, w.norm)) return 0;
  const uint32_t dl = ze_write_ncount(w.norm, nsym, kZeFitLog, desc);
  const uint64_t cfit = ze_table_cost(cnt, w.norm, nsym, kZeFitLog) + 256ull * 8 * dl;
  if (cfit >= cpre) return 0;
  ze_build_fse(w.norm, nsym, kZeFitLog, t, w);
  return dl;
}
// description bytes of one table at most (53 symbols of <= 9 bits + repeat fields + the log)
constexpr uint32_t kZeDescMax = 80;

inline void ze_build_tabs(ZeTabs &t) {
  ZeFseWork w;
  t = ZeTabs{};
  ze_build_fse(kZeLLNorm, kZeLLSyms, kZeLLLog, t.ll, w);
  ze_build_fse(kZeMLNorm, kZeMLSyms, kZeMLLog, t.ml, w);
  ze_build_fse(kZeOFNorm, kZeOFSyms, kZeOFLog, t.of, w);
}

__host__ __device__ __forceinline__ uint32_t ze_highbit(uint32_t v) { return v ? 31u - (uint32_t)__builtin_clz(v) : 0u; }
// literal length -> code (libzstd ZSTD_LLcode)
__host__ __device__ __forceinline__ uint32_t ze_ll_code(uint32_t ll) {
  if (ll < 16) return ll;
  if (ll < 24) return 16 + ((ll - 16) >> 1);
  if (ll < 32) return 20 + ((ll - 24) >> 2);
  if (ll < 48) return 22 + ((ll - 32) >> 3);
  if (ll < 64) return 24;
  return ze_highbit(ll) + 19;
}
// match length - 3 -> code (libzstd ZSTD_MLcode)
__host__ __device__ __forceinline__ uint32_t ze_ml_code(uint32_t mb) {
  if (mb < 32) return mb;
  if (mb < 40) return 32 + ((mb - 32) >> 1);
  if (mb < 48) return 36 + ((mb - 40) >> 2);
  if (mb < 64) return 38 + ((mb - 48) >> 3);
  if (mb < 96) return 40 + ((mb - 64) >> 4);
  if (mb < 128) return 42;
  return ze_highbit(mb) + 36;
}
// extra bits of a code (= the decoder's kZCodes ... >> 24)
__host__ __device__ __forceinline__ uint32_t ze_ll_bits(uint32_t c) {
  return c < 16 ? 0u : (c < 25 ? (uint32_t)(0x433221111ull >> (4 * (c - 16))) & 15u : c - 19);
}
__host__ __device__ __forceinline__ uint32_t ze_ml_bits(uint32_t c) {
  return c < 32 ? 0u : (c < 43 ? (uint32_t)(0x54433221111ull >> (4 * (c - 32))) & 15u : c - 36);
}

// forward bit writer, bytes out as they complete
struct ZeBits {
  uint64_t acc;
  uint32_t nb;
  uint8_t *out;
  uint64_t pos;
  __host__ __device__ __forceinline__ void add(uint32_t v, uint32_t n) {
    acc |= (uint64_t)(v & (uint32_t)((1ull << n) - 1)) << nb;
    nb += n;
    while (nb >= 8) {
      out[pos++] = (uint8_t)acc;
      acc >>= 8;
      nb -= 8;
    }
  }
  __host__ __device__ __forceinline__ void close() {  // end mark, then the last partial byte
    add(1, 1);
    if (nb) out[pos++] = (uint8_t)acc;
    acc = 0;
    nb = 0;
  }
};

__host__ __device__ __forceinline__ uint32_t ze_init(const ZeFse &t, uint32_t sym) {
  const uint32_t nbo = (t.dnb[sym] + (1u << 15)) >> 16;
  const uint32_t v = (nbo << 16) - t.dnb[sym];
  return t.state[(int32_t)(v >> nbo) + t.dfind[sym]];
}
__host__ __device__ __forceinline__ void ze_encode(ZeBits &w, const ZeFse &t, uint32_t &st, uint32_t sym) {
  const uint32_t nbo = (st + t.dnb[sym]) >> 16;
  w.add(st, nbo);
  st = t.state[(int32_t)(st >> nbo) + t.dfind[sym]];
}

// One sequence: literal length, match length (>= 3), offset (>= 1)
struct ZeSeq {
  uint32_t ll, ml, off;
};

// The sequences section's bitstream of seqs[0..n) (n >= 1) at w.out + w.pos
template <class GetSeq>
__host__ __device__ void ze_sequences(ZeBits &w, const ZeTabs &T, uint32_t n, GetSeq get) {
  ZeSeq q = get(n - 1);
  uint32_t ofv = q.off + 3, mb = q.ml - 3;
  uint32_t llc = ze_ll_code(q.ll), mlc = ze_ml_code(mb), ofc = ze_highbit(ofv);
  uint32_t s_ml = ze_init(T.ml, mlc), s_of = ze_init(T.of, ofc), s_ll = ze_init(T.ll, llc);
  w.add(q.ll, ze_ll_bits(llc));
  w.add(mb, ze_ml_bits(mlc));
  w.add(ofv, ofc);
  for (uint32_t i = n - 1; i-- > 0;) {
    q = get(i);
    ofv = q.off + 3;
    mb = q.ml - 3;
    llc = ze_ll_code(q.ll);
    mlc = ze_ml_code(mb);
    ofc = ze_highbit(ofv);
    ze_encode(w, T.of, s_of, ofc);
    ze_encode(w, T.ml, s_ml, mlc);
    ze_encode(w, T.ll, s_ll, llc);
    w.add(q.ll, ze_ll_bits(llc));
    w.add(mb, ze_ml_bits(mlc));
    w.add(ofv, ofc);
  }
  w.add(s_ml, T.ml.log);
  w.add(s_of, T.of.log);
  w.add(s_ll, T.ll.log);
  w.close();
}

// ---- Huffman-coded literals (RFC 8878 3.1.1.3.1, 4.2.1; libzstd HUF_*)
constexpr uint32_t kZeHufMax = 11;  // the format allows 11-bit codes

// Code lengths (<= maxlen) of a complete prefix code for the symbols with
// cnt > 0 (>= 2 of them): Huffman by repeated minimum pairs, then lengths
// clamped to maxlen and the Kraft sum brought back to exactly 1 (zstd's decoder
// deduces the last symbol's weight from it; Go's inflater accepts only complete
// codes). len[s] = 0 for absent symbols. Serial (one lane); w / parent hold
// 2 * nsym nodes. Shared by the zstd (maxlen 11) and DEFLATE (15, 7) encoders.
__host__ __device__ inline void huf_lengths(const uint32_t *cnt, uint32_t nsym, uint32_t maxlen, uint8_t *len,
                                            uint32_t *w, uint16_t *parent) {
  // nodes 0..nsym-1 leaves, nsym.. internal; w = weight (~0: consumed)
  uint32_t n = nsym;
  for (uint32_t s = 0; s < nsym; s++) w[s] = cnt[s] ? cnt[s] : 0xffffffffu;
  uint32_t live = 0;
  for (uint32_t s = 0; s < nsym; s++) live += cnt[s] ? 1 : 0;
  if (live < 2) {  // (callers pass two symbols or more; a lone one gets 1 bit)
    for (uint32_t s = 0; s < nsym; s++) len[s] = cnt[s] ? 1 : 0;
    return;
  }
  while (live > 1) {
    uint32_t a = 0xffffffffu, b = 0xffffffffu;
    for (uint32_t k = 0; k < n; k++) {
      if (w[k] == 0xffffffffu) continue;
      if (a == 0xffffffffu || w[k] < w[a]) {
        b = a;
        a = k;
      } else if (b == 0xffffffffu || w[k] < w[b]) {
        b = k;
      }
    }
    w[n] = w[a] + w[b];
    parent[a] = (uint16_t)n;
    parent[b] = (uint16_t)n;
    w[a] = w[b] = 0xffffffffu;
    n++;
    live--;
  }
  const uint32_t root = n - 1;
  for (uint32_t s = 0; s < nsym; s++) {
    uint32_t d = 0;
    if (cnt[s]) {
      for (uint32_t k = s; k != root; k = parent[k]) d++;
    }
    len[s] = (uint8_t)(d > maxlen ? maxlen : d);
  }
  // Kraft sum in units of 2^-maxlen: make it exactly 2^maxlen
  const uint32_t one = 1u << maxlen;
  uint32_t kraft = 0;
  for (uint32_t s = 0; s < nsym; s++)
    if (len[s]) kraft += 1u << (maxlen - len[s]);
  while (kraft > one) {  // lengthen the longest code below the cap
    uint32_t best = 0xffffffffu;
    for (uint32_t s = 0; s < nsym; s++)
      if (len[s] && len[s] < maxlen &&
          (best == 0xffffffffu || len[s] > len[best] || (len[s] == len[best] && cnt[s] < cnt[best])))
        best = s;
    kraft -= 1u << (maxlen - len[best] - 1);
    len[best]++;
  }
  while (kraft < one) {  // shorten the longest code that still fits
    uint32_t best = 0xffffffffu;
    for (uint32_t s = 0; s < nsym; s++)
      if (len[s] > 1 && kraft + (1u << (maxlen - len[s])) <= one &&
          (best == 0xffffffffu || len[s] > len[best] || (len[s] == len[best] && cnt[s] > cnt[best])))
        best = s;
    kraft += 1u << (maxlen - len[best]);
    len[best]--;
  }
}
__host__ __device__ inline void ze_huf_lengths(const uint32_t *cnt, uint32_t nsym, uint8_t *len, uint32_t *w,
                                               uint16_t *parent) {
  huf_lengths(cnt, nsym, kZeHufMax, len, w, parent);
}

// canonical code values of HUF_buildCTable: longest codes first from 0, each
// shorter rank starting at (previous start + count) / 2, symbols ascending
__host__ __device__ inline uint32_t ze_huf_codes(const uint8_t *len, uint32_t nsym, uint16_t *val) {
  uint32_t maxb = 0;
  uint16_t nper[kZeHufMax + 2] = {0}, vper[kZeHufMax + 2] = {0};
  for (uint32_t s = 0; s < nsym; s++) {
    nper[len[s]]++;
    if (len[s] > maxb) maxb = len[s];
  }
  uint32_t mn = 0;
  for (uint32_t b = maxb; b > 0; b--) {
    vper[b] = (uint16_t)mn;
    mn += nper[b];
    mn >>= 1;
  }
  for (uint32_t s = 0; s < nsym; s++) val[s] = len[s] ? vper[len[s]]++ : 0;
  return maxb;
}

// the tree description, direct representation (max symbol <= 128): header
// byte 127 + N, then the 4-bit weights of symbols 0..N-1 (the last symbol's
// is deduced); weight = maxb + 1 - len. Returns the bytes written.
__host__ __device__ inline uint32_t ze_huf_weights(const uint8_t *len, uint32_t last, uint32_t maxb, uint8_t *o) {
  o[0] = (uint8_t)(127 + last);
  for (uint32_t s = 0; s < last; s += 2) {
    const uint32_t w0 = len[s] ? maxb + 1 - len[s] : 0;
    const uint32_t w1 = (s + 1 < last && len[s + 1]) ? maxb + 1 - len[s + 1] : 0;
    o[1 + s / 2] = (uint8_t)((w0 << 4) | w1);
  }
  return 1 + (last + 1) / 2;
}

// Compressed_Literals_Block header (4 streams): the smallest size format that
// holds both sizes; returns its bytes (3, 4 or 5)
__host__ __device__ inline uint32_t ze_lit_header(uint8_t *o, uint32_t regen, uint32_t comp) {
  uint64_t v;
  uint32_t n;
  if (regen <= 1023 && comp <= 1023) {
    v = 2u | (1u << 2) | ((uint64_t)regen << 4) | ((uint64_t)comp << 14);
    n = 3;
  } else if (regen <= 16383 && comp <= 16383) {
    v = 2u | (2u << 2) | ((uint64_t)regen << 4) | ((uint64_t)comp << 18);
    n = 4;
  } else {
    v = 2u | (3u << 2) | ((uint64_t)regen << 4) | ((uint64_t)comp << 22);
    n = 5;
  }
  for (uint32_t k = 0; k < n; k++) o[k] = (uint8_t)(v >> (8 * k));
  return n;
}
// the 4 streams' symbol ranges: (n + 3) / 4 each, the last the rest
__host__ __device__ __forceinline__ uint32_t ze_seg(uint32_t n) { return (n + 3) / 4; }

// frame header: magic, single segment, 8-byte content size, no checksum
constexpr uint32_t kZeFrameHdr = 13;
__host__ __device__ __forceinline__ void ze_frame_header(uint8_t *o, uint64_t content) {
  o[0] = 0x28;
  o[1] = 0xB5;
  o[2] = 0x2F;
  o[3] = 0xFD;
  o[4] = 0xE0;  // FCS field 8 bytes, Single_Segment_Flag
  for (int k = 0; k < 8; k++) o[5 + k] = (uint8_t)(content >> (8 * k));
}
constexpr uint32_t kZeBlock = 16384;  // block content (more blocks, smaller per-block sequence lists)

}  // namespace rio
