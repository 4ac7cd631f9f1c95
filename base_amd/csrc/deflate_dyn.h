// Dynamic-Huffman DEFLATE blocks (RFC 1951 3.2.7) for the writer's "flate"
// transformer: the three trees of a block from its symbol counts, the header
// (HLIT, HDIST, HCLEN, code-length code lengths, the run-length-coded tree
// lengths) and the codes. Shared by the GPU encoder (deflate_enc.hip: lane 0
// builds the trees, the wave places the token bits) and its host check.
// Every tree is a complete code (Go's inflater, the reference's decoder,
// accepts no other), lengths <= 15 (literal/length, distance) and <= 7 (the
// code-length code).
#pragma once
#include <stdint.h>

#ifndef __HIPCC__  // the host check compiles this with g++
#define __host__
#define __device__
#define __forceinline__ inline
#endif


namespace rio {

constexpr uint32_t kDzLit = 286, kDzDist = 30, kDzCl = 19;
constexpr uint8_t kDzClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__host__ __device__ __forceinline__ uint32_t dz_rev(uint32_t code, uint32_t n) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; i++) r |= ((code >> i) & 1u) << (n - 1 - i);
  return r;
}

// length 3..258 -> symbol 257..285, extra bits and value
__host__ __device__ __forceinline__ void dz_len_sym(uint32_t m, uint32_t &sym, uint32_t &ext, uint32_t &val) {
  const uint32_t x = m - 3;
  ext = 0;
  val = 0;
  if (m == 258) {
    sym = 285;
  } else if (x < 8) {
    sym = 257 + x;
  } else {
    const uint32_t k = 31 - __builtin_clz(x);  // >= 3
    sym = 257 + 4 * (k - 1) + ((x >> (k - 2)) & 3);
    ext = k - 2;
    val = x & ((1u << ext) - 1);
  }
}
// distance 1..32768 -> code 0..29, extra bits and value
__host__ __device__ __forceinline__ void dz_dist_sym(uint32_t d, uint32_t &sym, uint32_t &ext, uint32_t &val) {
  const uint32_t y = d - 1;
  ext = 0;
  val = 0;
  if (y < 4) {
    sym = y;
  } else {
    const uint32_t k = 31 - __builtin_clz(y);  // >= 2
    sym = 2 * k + ((y >> (k - 1)) & 1);
    ext = k - 1;
    val = y & ((1u << ext) - 1);
  }
}

// canonical codes (RFC 1951 3.2.2), bit-reversed for LSB-first packing
__host__ __device__ inline void dz_codes(const uint8_t *len, uint32_t n, uint16_t *code) {
  uint32_t bl[16], next[16];
  for (int b = 0; b < 16; b++) bl[b] = 0;
  for (uint32_t i = 0; i < n; i++) bl[len[i]]++;
  bl[0] = 0;
  uint32_t c = 0;
  next[0] = 0;
  for (int b = 1; b < 16; b++) {
    c = (c + bl[b - 1]) << 1;
    next[b] = c;
  }
  for (uint32_t i = 0; i < n; i++) code[i] = len[i] ? (uint16_t)dz_rev(next[len[i]]++, len[i]) : 0;
}

struct DzTrees {
  uint8_t ll_len[kDzLit], d_len[kDzDist], cl_len[kDzCl];
  uint16_t ll_code[kDzLit], d_code[kDzDist], cl_code[kDzCl];
  uint16_t rle[kDzLit + kDzDist];  // code-length symbol | extra value << 5
  uint16_t ord[kDzLit];            // live symbols by ascending (count, symbol)
  uint32_t nrle, hlit, hdist, hclen, hdr_bits;
};

// Huffman code lengths (<= maxlen, a complete code) of the nlive >= 2 live
// symbols in ord (ascending count, then symbol): the two-queue construction
// (leaves in order, internal nodes in creation order are both sorted), node
// depths from the root down, counts per length clamped to maxlen and the
// Kraft sum brought back to exactly 1, then the lengths handed out longest
// first to the rarest symbols. O(nlive); w: nlive, par: 2 * nlive entries.
__host__ __device__ inline void huf_lengths_q(const uint32_t *cnt, uint32_t nsym, const uint16_t *ord, uint32_t nlive,
                                              uint32_t maxlen, uint8_t *len, uint32_t *w, uint16_t *par) {
  for (uint32_t s = 0; s < nsym; s++) len[s] = 0;
  uint32_t i = 0, j = 0;
  for (uint32_t k = 0; k + 1 < nlive; k++) {
    uint32_t nd[2], wt[2];
    for (int q = 0; q < 2; q++) {
      if (i < nlive && (j >= k || cnt[ord[i]] <= w[j])) {
        wt[q] = cnt[ord[i]];
        nd[q] = i++;
      } else {
        wt[q] = w[j];
        nd[q] = nlive + j++;
      }
    }
    w[k] = wt[0] + wt[1];
    par[nd[0]] = par[nd[1]] = (uint16_t)(nlive + k);
  }
  // depths of the internal nodes (into w), root = nlive - 2
  const uint32_t root = nlive - 2;
  w[root] = 0;
  for (uint32_t k = root; k-- > 0;) w[k] = w[par[nlive + k] - nlive] + 1;
  uint32_t bl[16];
  for (uint32_t b = 0; b < 16; b++) bl[b] = 0;
  for (uint32_t q = 0; q < nlive; q++) {
    const uint32_t d = w[par[q] - nlive] + 1;
    bl[d > maxlen ? maxlen : d]++;
  }
  const uint32_t one = 1u << maxlen;
  uint32_t kraft = 0;
  for (uint32_t b = 1; b <= maxlen; b++) kraft += bl[b] << (maxlen - b);
  while (kraft > one) {  // one code of the longest length below the cap gets a bit longer
    uint32_t b = maxlen - 1;
    while (!bl[b]) b--;
    bl[b]--;
    bl[b + 1]++;
    kraft -= 1u << (maxlen - b - 1);
  }
  while (kraft < one) {  // one code of the longest length that still fits gets a bit shorter
    uint32_t b = maxlen;
    while (b > 1 && (!bl[b] || kraft + (1u << (maxlen - b)) > one)) b--;
    bl[b]--;
    bl[b - 1]++;
    kraft += 1u << (maxlen - b);
  }
  uint32_t q = 0;
  for (uint32_t b = maxlen; b >= 1; b--)
    for (uint32_t c = 0; c < bl[b]; c++) len[ord[q++]] = (uint8_t)b;
}

// live symbols by ascending (count, symbol) into ord (insertion: small alphabets)
__host__ __device__ inline uint32_t dz_sort(const uint32_t *cnt, uint32_t nsym, uint16_t *ord) {
  uint32_t n = 0;
  for (uint32_t s = 0; s < nsym; s++) {
    if (!cnt[s]) continue;
    uint32_t p = n++;
    while (p > 0 && cnt[ord[p - 1]] > cnt[s]) {
      ord[p] = ord[p - 1];
      p--;
    }
    ord[p] = (uint16_t)s;
  }
  return n;
}

// degenerate alphabets: a complete code needs two symbols (absent ones get
// count 1); before the literal/length order is taken
__host__ __device__ inline void dz_fill(uint32_t *ll_cnt, uint32_t *d_cnt) {
  uint32_t used = 0;
  for (uint32_t s = 0; s < kDzLit; s++) used += ll_cnt[s] ? 1 : 0;
  if (used < 2) ll_cnt[ll_cnt[0] ? 1 : 0] = 1;
  used = 0;
  for (uint32_t s = 0; s < kDzDist; s++) used += d_cnt[s] ? 1 : 0;
  if (used < 2) {  // no or one distance code: two of them present (a complete 1-bit code)
    if (!d_cnt[0]) d_cnt[0] = 1;
    if (used == 0 || !d_cnt[1]) d_cnt[d_cnt[1] ? 2 : 1] = 1;
  }
}

// the trees of a block from its counts (ll_cnt includes end-of-block, dz_fill
// applied) and t.ord = the ll_n live literal/length symbols in order; w /
// par: 2 * kDzLit node scratch
__host__ __device__ inline void dz_build(const uint32_t *ll_cnt, const uint32_t *d_cnt, uint32_t ll_n, DzTrees &t,
                                         uint32_t *w, uint16_t *par) {
  uint32_t lastll = 0, lastd = 0;
  huf_lengths_q(ll_cnt, kDzLit, t.ord, ll_n, 15, t.ll_len, w, par);
  const uint32_t dn = dz_sort(d_cnt, kDzDist, t.ord);
  huf_lengths_q(d_cnt, kDzDist, t.ord, dn, 15, t.d_len, w, par);
  lastll = 0;
  for (uint32_t s = 0; s < kDzLit; s++)
    if (t.ll_len[s]) lastll = s;
  lastd = 0;
  for (uint32_t s = 0; s < kDzDist; s++)
    if (t.d_len[s]) lastd = s;
  t.hlit = lastll + 1 < 257 ? 257 : lastll + 1;
  t.hdist = lastd + 1;
  // run-length code of the concatenated lengths (16: repeat the previous 3-6
  // times, 17: 3-10 zeros, 18: 11-138 zeros)
  const uint32_t total = t.hlit + t.hdist;
  uint32_t cl_cnt[kDzCl];
  for (uint32_t k = 0; k < kDzCl; k++) cl_cnt[k] = 0;
  t.nrle = 0;
  auto L = [&](uint32_t i) -> uint32_t { return i < t.hlit ? t.ll_len[i] : t.d_len[i - t.hlit]; };
  auto put = [&](uint32_t sym, uint32_t extra) {
    t.rle[t.nrle++] = (uint16_t)(sym | (extra << 5));
    cl_cnt[sym]++;
  };
  for (uint32_t i = 0; i < total;) {
    const uint32_t cur = L(i);
    uint32_t run = 1;
    while (i + run < total && L(i + run) == cur) run++;
    if (cur == 0) {
      uint32_t r = run;
      while (r >= 11) {
        const uint32_t k = r < 138 ? r : 138;
        put(18, k - 11);
        r -= k;
      }
      if (r >= 3) {
        put(17, r - 3);
        r = 0;
      }
      while (r--) put(0, 0);
    } else {
      put(cur, 0);
      uint32_t r = run - 1;
      while (r >= 3) {
        const uint32_t k = r < 6 ? r : 6;
        put(16, k - 3);
        r -= k;
      }
      while (r--) put(cur, 0);
    }
    i += run;
  }
  uint32_t used = 0;
  for (uint32_t k = 0; k < kDzCl; k++) used += cl_cnt[k] ? 1 : 0;
  if (used < 2) cl_cnt[cl_cnt[0] ? 1 : 0] = 1;
  const uint32_t cn = dz_sort(cl_cnt, kDzCl, t.ord);
  huf_lengths_q(cl_cnt, kDzCl, t.ord, cn, 7, t.cl_len, w, par);
  t.hclen = 19;
  while (t.hclen > 4 && t.cl_len[kDzClOrder[t.hclen - 1]] == 0) t.hclen--;
  dz_codes(t.ll_len, kDzLit, t.ll_code);
  dz_codes(t.d_len, kDzDist, t.d_code);
  dz_codes(t.cl_len, kDzCl, t.cl_code);
  uint32_t bits = 3 + 5 + 5 + 4 + 3 * t.hclen;
  for (uint32_t k = 0; k < t.nrle; k++) {
    const uint32_t sym = t.rle[k] & 31u;
    bits += t.cl_len[sym] + (sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0);
  }
  t.hdr_bits = bits;
}

// the block header: BFINAL, BTYPE 10, HLIT, HDIST, HCLEN, the code-length
// code, the run-length-coded lengths (sink.add(value, nbits), LSB first)
template <class Sink>
__host__ __device__ inline void dz_header(Sink &o, const DzTrees &t, bool final) {
  o.add(final ? 1u : 0u, 1);
  o.add(2, 2);
  o.add(t.hlit - 257, 5);
  o.add(t.hdist - 1, 5);
  o.add(t.hclen - 4, 4);
  for (uint32_t k = 0; k < t.hclen; k++) o.add(t.cl_len[kDzClOrder[k]], 3);
  for (uint32_t k = 0; k < t.nrle; k++) {
    const uint32_t sym = t.rle[k] & 31u, ex = t.rle[k] >> 5;
    o.add(t.cl_code[sym], t.cl_len[sym]);
    if (sym == 16) o.add(ex, 2);
    else if (sym == 17) o.add(ex, 3);
    else if (sym == 18) o.add(ex, 7);
  }
}

}  // namespace rio
