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

// FSE compression table of one predefined distribution
struct ZeFse {
  uint16_t state[64];  // next state values (tableSize + position), sorted by symbol
  int32_t dfind[53];   // deltaFindState
  uint32_t dnb[53];    // deltaNbBits
  int32_t log;
};
struct ZeTabs {
  ZeFse ll, ml, of;
};

// FSE_buildCTable for a normalized distribution (host)
inline void ze_build_fse(const int16_t *norm, int nsym, int log, ZeFse &t) {
  const int ts = 1 << log;
  int sym_at[64];
  int cumul[54];
  int high = ts - 1;
  cumul[0] = 0;
  for (int u = 1; u <= nsym; u++) {
    if (norm[u - 1] == -1) {  // low-probability symbols take the table's end
      cumul[u] = cumul[u - 1] + 1;
      sym_at[high--] = u - 1;
    } else {
      cumul[u] = cumul[u - 1] + norm[u - 1];
    }
  }
  const int step = (ts >> 1) + (ts >> 3) + 3, mask = ts - 1;
  int pos = 0;
  for (int s = 0; s < nsym; s++)
    for (int k = 0; k < norm[s]; k++) {
      sym_at[pos] = s;
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

inline void ze_build_tabs(ZeTabs &t) {
  ze_build_fse(kZeLLNorm, kZeLLSyms, kZeLLLog, t.ll);
  ze_build_fse(kZeMLNorm, kZeMLSyms, kZeMLLog, t.ml);
  ze_build_fse(kZeOFNorm, kZeOFSyms, kZeOFLog, t.of);
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
