// DEFLATE encoder of the writer's "flate" transformer on the GPU (SURVEY.md
// §8(f) 1: the mirror of recordioflate's FlateUncompress; the reference
// compresses with klauspost/compress flate, recordioflate.go:31-52). The
// output need not equal klauspost's bytes -- any valid raw DEFLATE stream
// that the reference's inflater decodes to the payload is a correct "flate"
// block (decode parity is what tests/test_encode_gpu.py checks, with the GPU
// scanner, the oracle's inflater and zlib).
//
// One wave per block, the block payload (varint header + items, the writer
// transforms the whole payload, writerv2.go:432-441) in rounds of 64
// positions:
//   - a 4,096-entry hash table of 4-byte prefixes in LDS (position of the
//     last occurrence); every lane looks up its position, then inserts it
//     (candidates come from earlier rounds, so a round never matches itself);
//   - lanes at or after the parse cursor extend their candidate's match
//     (4 bytes per step, <= 258, distance <= 32 KiB);
//   - greedy parse of the round by the wave: from the cursor, a match if one
//     was found at that position, else a literal (a scalar walk of <= 64
//     steps over readlane'd lengths);
//   - the chosen tokens' fixed-Huffman codes (RFC 1951 3.2.6: <= 31 bits each)
//     placed by a wave prefix sum of their bit lengths and OR-ed into a
//     128-dword LDS ring (ds_or: tokens share dwords); completed dwords are
//     written out coalesced after every round.
// One final block (BFINAL 1, BTYPE 01), end-of-block code 0000000.
// Level 0 emits stored blocks instead (BTYPE 00, <= 65,535 bytes each), like
// flate.NoCompression.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "deflate_dyn.h"
#include "device_common.h"
#include "encode.h"
#include "rio_internal.h"

namespace rio {

constexpr int kDHashBits = 12;
constexpr uint32_t kDNone = 0xffffffffu;
constexpr int kDRing = 128;        // output staging dwords per wave
constexpr int kDWaves = 4;         // waves per workgroup

// 4 payload bytes at p (p + 4 <= len): hdr scratch then items, or one buffer
struct DSrc {
  const uint8_t *hdr;
  unsigned long long hlen;
  const uint8_t *data;
  unsigned long long len;
  __device__ __forceinline__ uint32_t byte(unsigned long long p) const { return p < hlen ? hdr[p] : data[p - hlen]; }
  __device__ __forceinline__ uint32_t load4(unsigned long long p) const {
    const uint8_t *q;
    if (p + 4 <= hlen) q = hdr + p;
    else if (p >= hlen) q = data + (p - hlen);
    else return byte(p) | (byte(p + 1) << 8) | (byte(p + 2) << 16) | (byte(p + 3) << 24);
    const uintptr_t a = (uintptr_t)q;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    return sh ? (w[0] >> sh) | (w[1] << (32 - sh)) : w[0];
  }
  // 16 bytes at p; bytes at or past len read as 0 (and are never loaded)
  __device__ __forceinline__ void load16(unsigned long long p, uint32_t (&w)[4]) const {
    const uint8_t *q = nullptr;
    if (p + 16 <= len) {
      if (p + 16 <= hlen) q = hdr + p;
      else if (p >= hlen) q = data + (p - hlen);
    }
    if (q) {
      // 5 aligned dwords funnel-shifted by the misalignment (v_alignbyte),
      // branch-free across the wave's lanes (their alignments differ); an
      // aligned q reloads dword 3 as the 5th (the next one may lie past the
      // payload)
      const uintptr_t a = (uintptr_t)q;
      const uint32_t *d = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
      const uint32_t nb = (uint32_t)(a & 3);
      uint32_t e[5];
#pragma unroll
      for (int k = 0; k < 4; k++) e[k] = d[k];
      e[4] = d[nb ? 4 : 3];
#pragma unroll
      for (int k = 0; k < 4; k++) w[k] = __builtin_amdgcn_alignbyte(e[k + 1], e[k], nb);
      return;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t v = 0;
      for (int j = 0; j < 4; j++)
        if (p + 4 * k + j < len) v |= byte(p + 4 * k + j) << (8 * j);
      w[k] = v;
    }
  }
};

// bytes equal from the start of two 16-byte groups (16: all)
__device__ __forceinline__ uint32_t common16(const uint32_t (&a)[4], const uint32_t (&b)[4]) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x = a[k] ^ b[k];
    if (x) return 4 * k + ((__ffs(x) - 1) >> 3);
  }
  return 16;
}

__device__ __forceinline__ uint32_t rev_bits(uint32_t code, uint32_t n) { return __brev(code) >> (32 - n); }

// fixed-Huffman bits (LSB first) of a literal byte
__device__ __forceinline__ void lit_bits(uint32_t b, uint32_t &bits, uint32_t &n) {
  if (b < 144) {
    bits = rev_bits(0x30 + b, 8);
    n = 8;
  } else {
    bits = rev_bits(0x190 + (b - 144), 9);
    n = 9;
  }
}

// fixed-Huffman bits of a match (length 3..258, distance 1..32768): <= 31 bits
__device__ __forceinline__ void match_bits(uint32_t m, uint32_t d, uint32_t &bits, uint32_t &n) {
  uint32_t lcode, lext = 0, lval = 0;
  const uint32_t x = m - 3;
  if (m == 258) {
    lcode = 285;
  } else if (x < 8) {
    lcode = 257 + x;
  } else {
    const uint32_t k = 31 - __clz(x);  // >= 3
    lcode = 257 + 4 * (k - 1) + ((x >> (k - 2)) & 3);
    lext = k - 2;
    lval = x & ((1u << lext) - 1);
  }
  uint32_t hc, hn;
  if (lcode <= 279) {
    hc = lcode - 256;
    hn = 7;
  } else {
    hc = 0xC0 + (lcode - 280);
    hn = 8;
  }
  uint32_t dcode, dext = 0, dval = 0;
  const uint32_t y = d - 1;
  if (y < 4) {
    dcode = y;
  } else {
    const uint32_t k = 31 - __clz(y);  // >= 2
    dcode = 2 * k + ((y >> (k - 1)) & 1);
    dext = k - 1;
    dval = y & ((1u << dext) - 1);
  }
  bits = rev_bits(hc, hn);
  n = hn;
  bits |= lval << n;
  n += lext;
  bits |= rev_bits(dcode, 5) << n;
  n += 5;
  bits |= dval << n;
  n += dext;
}

__device__ __forceinline__ DSrc dsrc_of(const EncArgs &a, uint64_t b) {
  DSrc s;
  const uint64_t f0 = b * a.per_block;
  const uint64_t f = f0 < a.n_items ? f0 : a.n_items;
  s.hdr = a.hdr + a.hdr_off[b];
  s.hlen = a.hdr_len[b];
  s.data = a.data + (f == 0 ? 0ull : a.item_end[f - 1]);
  s.len = a.pay_len[b];
  return s;
}

__global__ void __launch_bounds__(64 * kDWaves) k_deflate(EncArgs a) {
  __shared__ uint32_t s_hash[kDWaves][1 << kDHashBits];
  __shared__ uint32_t s_ring[kDWaves][kDRing];
  const int wv = threadIdx.x >> 6;
  uint32_t *hash = s_hash[wv];
  uint32_t *ring = s_ring[wv];
  const int l = lane_id();
  const uint64_t nwaves = (uint64_t)gridDim.x * kDWaves;
  for (uint64_t b = (uint64_t)blockIdx.x * kDWaves + wv; b < a.nblocks; b += nwaves) {
    const DSrc s = dsrc_of(a, b);
    const unsigned long long L = s.len;
    uint32_t *out = reinterpret_cast<uint32_t *>(a.comp + a.comp_off[b]);
    for (int i = l; i < (1 << kDHashBits); i += 64) hash[i] = kDNone;
    for (int i = l; i < kDRing; i += 64) ring[i] = 0;
    wave_lds_sync();
    if (l == 0) ring[0] = 3;  // BFINAL 1, BTYPE 01 (fixed Huffman)
    unsigned long long bitpos = 3, flushed = 0, cur = 0;
    uint32_t nx[4];  // the next round's 16 bytes at this lane's position (prefetched)
    s.load16(l, nx);
    for (unsigned long long base = 0; base < L; base += 64) {
      const unsigned long long p = base + l;
      uint32_t cw[4] = {nx[0], nx[1], nx[2], nx[3]};
      if (base + 64 < L) s.load16(p + 64, nx);
      const bool has4 = p + 4 <= L;
      const uint32_t v4 = cw[0];
      const uint32_t h = (v4 * 0x9E3779B1u) >> (32 - kDHashBits);
      const uint32_t cand = has4 ? hash[h] : kDNone;
      wave_lds_sync();
      if (has4) hash[h] = (uint32_t)p;  // (positions < 2^32: blocks are smaller)
      // match length at p (only where the parse can land): 16 bytes per step
      uint32_t m = 0;
      if (has4 && p >= cur && cand != kDNone && p - cand <= 32768) {
        const unsigned long long room = L - p;
        const uint32_t maxm = room < 258 ? (uint32_t)room : 258u;
        uint32_t cc[4];
        s.load16(cand, cc);
        m = common16(cc, cw);
        while (m == 16 * ((m + 15) / 16) && m > 0 && m < maxm) {  // all equal so far
          uint32_t a16[4], b16[4];
          s.load16(cand + m, a16);
          s.load16(p + m, b16);
          const uint32_t k = common16(a16, b16);
          m += k;
          if (k < 16) break;
        }
        if (m > maxm) m = maxm;
        if (m < 4) m = 0;
      }
      // greedy parse of this round from the cursor (wave-uniform walk)
      unsigned long long chosen = 0;
      unsigned long long pos = cur;
      const unsigned long long rend = base + 64 < L ? base + 64 : L;
      while (pos < rend) {
        const uint32_t lane = (uint32_t)(pos - base);
        const uint32_t ml = (uint32_t)__builtin_amdgcn_readlane((int)m, (int)lane);
        chosen |= 1ull << lane;
        pos += ml >= 4 ? ml : 1;
      }
      cur = pos;
      // this lane's token
      uint32_t bits = 0, nb = 0;
      if ((chosen >> l) & 1) {
        if (m >= 4) match_bits(m, (uint32_t)(p - cand), bits, nb);
        else lit_bits(cw[0] & 0xff, bits, nb);
      }
      const uint32_t incl = wave_incl_sum<uint32_t>(nb);
      const uint32_t tot = __shfl(incl, 63, 64);
      if (nb) {
        const unsigned long long o = bitpos + (incl - nb);
        const uint32_t k = (uint32_t)(o >> 5), sh = (uint32_t)(o & 31);
        atomicOr(&ring[k & (kDRing - 1)], bits << sh);
        if (sh + nb > 32) atomicOr(&ring[(k + 1) & (kDRing - 1)], bits >> (32 - sh));
      }
      bitpos += tot;
      wave_lds_sync();
      // completed dwords out (coalesced), their ring slots cleared
      const unsigned long long done = bitpos >> 5;
      if (flushed + l < done) {
        const uint32_t slot = (uint32_t)((flushed + l) & (kDRing - 1));
        out[flushed + l] = ring[slot];
        ring[slot] = 0;
      }
      flushed = done;
      wave_lds_sync();
    }
    bitpos += 7;  // end of block: code 256 = 0000000
    const unsigned long long nd = (bitpos + 31) >> 5;
    for (unsigned long long k = flushed + l; k < nd; k += 64) {
      const uint32_t slot = (uint32_t)(k & (kDRing - 1));
      out[k] = ring[slot];
      ring[slot] = 0;
    }
    wave_lds_sync();
    if (l == 0) a.pay_len[b] = (bitpos + 7) >> 3;
  }
}

// flate.NoCompression: stored blocks of <= 65,535 bytes (RFC 1951 3.2.4)
__global__ void __launch_bounds__(256) k_deflate_stored(EncArgs a) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t b = wave; b < a.nblocks; b += nwaves) {
    const DSrc s = dsrc_of(a, b);
    const unsigned long long L = s.len;
    uint8_t *out = a.comp + a.comp_off[b];
    const unsigned long long np = L == 0 ? 1 : (L + 65534) / 65535;
    for (unsigned long long k = 0; k < np; k++) {
      const unsigned long long p0 = k * 65535;
      const uint32_t n = (uint32_t)((L - p0) < 65535 ? (L - p0) : 65535);
      uint8_t *o = out + k * 65540;
      if (l == 0) {
        o[0] = (k + 1 == np) ? 1 : 0;  // BFINAL, BTYPE 00, then the byte boundary
        o[1] = n & 0xff;
        o[2] = n >> 8;
        o[3] = ~n & 0xff;
        o[4] = (~n >> 8) & 0xff;
      }
      for (uint32_t i = l; i < n; i += 64) o[5 + i] = (uint8_t)s.byte(p0 + i);
    }
    if (l == 0) a.pay_len[b] = L + 5 * np;
  }
}

// ---- dynamic Huffman (levels >= 2, the default) ----------------------------
// The same hash/greedy parse, in sub-blocks of kDySub payload bytes, each its
// own DEFLATE block: the round's chosen tokens go to the wave's token list in
// HBM (u32: a literal byte, or 1 << 31 | length << 16 | distance - 1) and
// their symbols into LDS histograms; then the literal/length order (a wave
// rank sort), the trees (lane 0, deflate_dyn.h: O(symbols)), the cost of the
// dynamic block against the fixed one from the histograms, the header (lane 0
// into the ring) and the tokens re-read 64 at a time, coded with the chosen
// trees (<= 48 bits each) and placed by a wave prefix sum like k_deflate's.
constexpr int kDySub = 32768;  // payload bytes per DEFLATE block
constexpr int kDyWaves = 2;    // waves per workgroup (~23 KB LDS each)
constexpr int kDyRing = 256;   // staging dwords: a dynamic header is <= 4,500 bits
constexpr uint16_t kDyNone = 0xffff;

struct alignas(16) DyWave {  // (16: the rank sort reads ll_cnt as uint4)
  uint16_t hash[1 << kDHashBits];  // low 16 bits of the last position (kDyNone: none)
  uint32_t ll_cnt[288], d_cnt[32];
  uint32_t w[kDzLit];
  uint16_t par[2 * kDzLit];
  uint32_t ring[kDyRing];
  DzTrees t;
};

struct DyRingSink {  // lane 0: header bits into the ring
  uint32_t *ring;
  unsigned long long pos;
  __device__ void add(uint32_t v, uint32_t n) {
    if (!n) return;
    const uint32_t k = (uint32_t)(pos >> 5), sh = (uint32_t)(pos & 31);
    ring[k & (kDyRing - 1)] |= v << sh;
    if (sh + n > 32) ring[(k + 1) & (kDyRing - 1)] |= v >> (32 - sh);
    pos += n;
  }
};

__device__ __forceinline__ uint32_t dy_fixlen(uint32_t s) { return s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8; }

__device__ __forceinline__ uint32_t dy_wave_sum(uint32_t v) {
  return __shfl(wave_incl_sum<uint32_t>(v), 63, 64);
}

__device__ __forceinline__ void dy_mem_sync() {  // this wave's global stores visible to its lanes' loads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

#ifndef RIO_DY_ATTR
#define RIO_DY_ATTR
#endif
__global__ void __launch_bounds__(64 * kDyWaves) RIO_DY_ATTR k_deflate_dyn(EncArgs a, uint32_t *scratch) {
  __shared__ DyWave s_w[kDyWaves];
  const int wv = threadIdx.x >> 6;
  DyWave &W = s_w[wv];
  uint16_t *hash = W.hash;
  uint32_t *ring = W.ring;
  DzTrees &t = W.t;
  const int l = lane_id();
  const uint64_t nwaves = (uint64_t)gridDim.x * kDyWaves;
  uint32_t *tok = scratch + ((uint64_t)blockIdx.x * kDyWaves + wv) * kDySub;
  for (uint64_t b = (uint64_t)blockIdx.x * kDyWaves + wv; b < a.nblocks; b += nwaves) {
    const DSrc s = dsrc_of(a, b);
    const unsigned long long L = s.len;
    uint32_t *out = reinterpret_cast<uint32_t *>(a.comp + a.comp_off[b]);
    for (int i = l; i < (1 << kDHashBits); i += 64) hash[i] = kDyNone;
    for (int i = l; i < kDyRing; i += 64) ring[i] = 0;
    unsigned long long bitpos = 0, flushed = 0, cur = 0;
    auto flush = [&]() {
      wave_lds_sync();
      const unsigned long long done = bitpos >> 5;
      for (unsigned long long k = flushed + l; k < done; k += 64) {
        const uint32_t slot = (uint32_t)(k & (kDyRing - 1));
        out[k] = ring[slot];
        ring[slot] = 0;
      }
      flushed = done;
      wave_lds_sync();
    };
    uint32_t nx[4];
    s.load16(l, nx);
    for (unsigned long long b0 = 0;; b0 += kDySub) {
      const unsigned long long b1 = b0 + kDySub < L ? b0 + kDySub : L;
      const bool final = b1 >= L;
      for (int i = l; i < 288; i += 64) W.ll_cnt[i] = 0;
      if (l < 32) W.d_cnt[l] = 0;
      wave_lds_sync();
      uint32_t ntok = 0;
      for (unsigned long long base = b0; base < b1; base += 64) {
        const unsigned long long p = base + l;
        uint32_t cw[4] = {nx[0], nx[1], nx[2], nx[3]};
        if (base + 64 < L) s.load16(p + 64, nx);
        const bool has4 = p + 4 <= L;
        const uint32_t h = (cw[0] * 0x9E3779B1u) >> (32 - kDHashBits);
        // the candidate: the latest position with these low 16 bits (any
        // earlier position of this block; the byte compare below decides)
        const uint32_t e = has4 ? hash[h] : kDyNone;
        const uint32_t delta = (uint32_t)(uint16_t)((uint32_t)p - e);
        const unsigned long long cand = p - delta;
        wave_lds_sync();
        if (has4) hash[h] = (uint16_t)p;
        uint32_t m = 0;
        if (has4 && p >= cur && p < b1 && e != kDyNone && delta != 0 && delta <= 32768) {
          const unsigned long long room = b1 - p;
          const uint32_t maxm = room < 258 ? (uint32_t)room : 258u;
          uint32_t cc[4];
          s.load16(cand, cc);
          m = common16(cc, cw);
          while (m == 16 * ((m + 15) / 16) && m > 0 && m < maxm) {
            uint32_t a16[4], b16[4];
            s.load16(cand + m, a16);
            s.load16(p + m, b16);
            const uint32_t k = common16(a16, b16);
            m += k;
            if (k < 16) break;
          }
          if (m > maxm) m = maxm;
          if (m < 4) m = 0;
        }
        unsigned long long chosen = 0, pos = cur;
        const unsigned long long rend = base + 64 < b1 ? base + 64 : b1;
        while (pos < rend) {
          const uint32_t lane = (uint32_t)(pos - base);
          const uint32_t ml = (uint32_t)__builtin_amdgcn_readlane((int)m, (int)lane);
          chosen |= 1ull << lane;
          pos += ml >= 4 ? ml : 1;
        }
        cur = pos;
        if ((chosen >> l) & 1) {
          const uint32_t idx = ntok + (uint32_t)__popcll(chosen & ((1ull << l) - 1));
          uint32_t tk;
          if (m >= 4) {
            const uint32_t d = (uint32_t)(p - cand);
            uint32_t sym, e, v;
            dz_len_sym(m, sym, e, v);
            atomicAdd(&W.ll_cnt[sym], 1u);
            dz_dist_sym(d, sym, e, v);
            atomicAdd(&W.d_cnt[sym], 1u);
            tk = 0x80000000u | (m << 16) | (d - 1);
          } else {
            tk = cw[0] & 0xff;
            atomicAdd(&W.ll_cnt[tk], 1u);
          }
          tok[idx] = tk;
        }
        ntok += (uint32_t)__popcll(chosen);
      }
      wave_lds_sync();
      if (l == 0) {
        W.ll_cnt[256]++;  // end of block
        dz_fill(W.ll_cnt, W.d_cnt);
      }
      wave_lds_sync();
      {  // literal/length symbols by ascending (count, symbol): rank of each
        uint32_t c[5], r[5] = {0, 0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 5; k++) c[k] = l + 64 * k < (int)kDzLit ? W.ll_cnt[l + 64 * k] : 0u;
        const uint4 *cv = reinterpret_cast<const uint4 *>(W.ll_cnt);
        for (int q = 0; q < 72; q++) {
          const uint4 v = cv[q];
          const uint32_t e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint32_t ts = 4 * q + j;
#pragma unroll
            for (int k = 0; k < 5; k++)
              r[k] += (e[j] != 0) & ((e[j] < c[k]) | ((e[j] == c[k]) & (ts < (uint32_t)(l + 64 * k))));
          }
        }
        uint32_t live = 0;
#pragma unroll
        for (int k = 0; k < 5; k++)
          if (c[k]) {
            t.ord[r[k]] = (uint16_t)(l + 64 * k);
            live++;
          }
        live = dy_wave_sum(live);
        wave_lds_sync();
        if (l == 0) dz_build(W.ll_cnt, W.d_cnt, live, t, W.w, W.par);
        wave_lds_sync();
      }
      uint32_t dyn = 0, fix = 0;
      for (int i = l; i < (int)kDzLit; i += 64) {
        dyn += W.ll_cnt[i] * t.ll_len[i];
        fix += W.ll_cnt[i] * dy_fixlen(i);
      }
      if (l < (int)kDzDist) {
        dyn += W.d_cnt[l] * t.d_len[l];
        fix += W.d_cnt[l] * 5;
      }
      dyn = dy_wave_sum(dyn) + t.hdr_bits;
      fix = dy_wave_sum(fix) + 3;
      const bool use_dyn = dyn < fix;
      if (!use_dyn) {  // the fixed code (RFC 1951 3.2.6; 288 literal/length symbols)
        for (int i = l; i < (int)kDzLit; i += 64) {
          const uint32_t n = dy_fixlen(i);
          const uint32_t c = i < 144 ? 0x30 + i : i < 256 ? 0x190 + (i - 144) : i < 280 ? i - 256 : 0xC0 + (i - 280);
          t.ll_len[i] = (uint8_t)n;
          t.ll_code[i] = (uint16_t)rev_bits(c, n);
        }
        if (l < (int)kDzDist) {
          t.d_len[l] = 5;
          t.d_code[l] = (uint16_t)rev_bits(l, 5);
        }
      }
      wave_lds_sync();
      if (l == 0) {
        DyRingSink o{ring, bitpos};
        if (use_dyn) {
          dz_header(o, t, final);
        } else {
          o.add(final ? 1u : 0u, 1);
          o.add(1, 2);
        }
        W.w[0] = (uint32_t)(o.pos - bitpos);
      }
      wave_lds_sync();
      bitpos += W.w[0];
      flush();
      dy_mem_sync();  // the token list's stores visible to every lane
      uint32_t tn = l < (int)ntok ? tok[l] : 0;
      for (uint32_t g = 0; g < ntok; g += 64) {
        const uint32_t tk = tn;
        const bool have = g + l < ntok;
        if (g + 64 + l < ntok) tn = tok[g + 64 + l];
        unsigned long long v = 0;
        uint32_t nb = 0;
        if (have) {
          if (tk >> 31) {
            const uint32_t m = (tk >> 16) & 0x1ff, d = (tk & 0xffff) + 1;
            uint32_t sym, e, x;
            dz_len_sym(m, sym, e, x);
            v = t.ll_code[sym];
            nb = t.ll_len[sym];
            v |= (unsigned long long)x << nb;
            nb += e;
            dz_dist_sym(d, sym, e, x);
            v |= (unsigned long long)t.d_code[sym] << nb;
            nb += t.d_len[sym];
            v |= (unsigned long long)x << nb;
            nb += e;
          } else {
            v = t.ll_code[tk];
            nb = t.ll_len[tk];
          }
        }
        const uint32_t incl = wave_incl_sum<uint32_t>(nb);
        const uint32_t tot = __shfl(incl, 63, 64);
        if (nb) {
          const unsigned long long o = bitpos + (incl - nb);
          const uint32_t k = (uint32_t)(o >> 5), sh = (uint32_t)(o & 31);
          const unsigned long long lo = v << sh;
          atomicOr(&ring[k & (kDyRing - 1)], (uint32_t)lo);
          if (sh + nb > 32) atomicOr(&ring[(k + 1) & (kDyRing - 1)], (uint32_t)(lo >> 32));
          if (sh + nb > 64) atomicOr(&ring[(k + 2) & (kDyRing - 1)], (uint32_t)(v >> (64 - sh)));
        }
        bitpos += tot;
        flush();
      }
      if (l == 0) {
        DyRingSink o{ring, bitpos};
        o.add(t.ll_code[256], t.ll_len[256]);
      }
      bitpos += t.ll_len[256];
      if (final) break;
      flush();
    }
    wave_lds_sync();
    const unsigned long long nd = (bitpos + 31) >> 5;
    for (unsigned long long k = flushed + l; k < nd; k += 64) {
      const uint32_t slot = (uint32_t)(k & (kDyRing - 1));
      out[k] = ring[slot];
      ring[slot] = 0;
    }
    wave_lds_sync();
    if (l == 0) a.pay_len[b] = (bitpos + 7) >> 3;
  }
}

#ifndef RIO_DY_WG
#define RIO_DY_WG 4
#endif
// workgroups per CU: 4 (VGPRs: 2 waves per SIMD)
static uint64_t deflate_dyn_grid(int ncu) { return (uint64_t)(ncu > 0 ? ncu : 256) * RIO_DY_WG; }

uint64_t deflate_scratch_words(int ncu) { return deflate_dyn_grid(ncu) * kDyWaves * kDySub / 2; }

// per block: the compressed region's bound (into nck, scanned into comp_off)
__global__ void k_deflate_bound(EncArgs a) {
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < a.nblocks;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long L = a.pay_len[b];
    const unsigned long long stored = L + 5 * (L / 65535 + 1);
    const unsigned long long fixed = L + L / 8 + 16 + 2 * (L / kDySub + 1);  // (a fixed block per kDySub)
    a.nck[b] = ((stored > fixed ? stored : fixed) + 64 + 15) & ~15ull;
  }
}

void launch_deflate_bound(const EncArgs &a, hipStream_t st) {
  uint64_t g = (a.nblocks + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(k_deflate_bound, dim3((unsigned)(g ? g : 1)), dim3(256), 0, st, a);
}

void launch_deflate(const EncArgs &a, unsigned long long *scratch, int ncu, hipStream_t st) {
  uint64_t g = (a.nblocks + kDWaves - 1) / kDWaves;
  if (g > 8192) g = 8192;
  if (a.level == 0) {
    hipLaunchKernelGGL(k_deflate_stored, dim3((unsigned)(g ? g : 1)), dim3(256), 0, st, a);
  } else if (a.level == 1) {
    hipLaunchKernelGGL(k_deflate, dim3((unsigned)(g ? g : 1)), dim3(64 * kDWaves), 0, st, a);
  } else {
    uint64_t gd = (a.nblocks + kDyWaves - 1) / kDyWaves;
    const uint64_t cap = deflate_dyn_grid(ncu);
    if (gd > cap) gd = cap;
    hipLaunchKernelGGL(k_deflate_dyn, dim3((unsigned)(gd ? gd : 1)), dim3(64 * kDyWaves), 0, st, a,
                       reinterpret_cast<uint32_t *>(scratch));
  }
}

}  // namespace rio
