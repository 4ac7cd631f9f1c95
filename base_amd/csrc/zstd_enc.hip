// zstd encoder of the writer's "zstd" transformer on the GPU (SURVEY.md §8(f)
// 1; the reference compresses with DataDog/zstd = libzstd's ZSTD_compress,
// recordiozstd.go:31-52, and any frame libzstd decodes to the payload is a
// correct "zstd" block: tests/test_encode_gpu.py decodes these with libzstd,
// the oracle and the GPU scanner).
//
// One wave per recordio block, its payload (varint header + items, the whole
// of it transformed, writerv2.go:432-441) as one frame (single segment, 8-byte
// content size, no checksum) of blocks of <= 16 KiB:
//   - matches as in the DEFLATE encoder (deflate_enc.hip): rounds of 64
//     positions, a 4,096-entry LDS hash of 4-byte prefixes (lookups, then
//     inserts), lanes at or after the parse cursor extend their candidate 16
//     bytes per step, a wave-uniform greedy walk picks the sequences -- here
//     any distance back in the frame (the window is the frame), lengths up to
//     the block's end; the walk appends (literal length, match length,
//     offset) to the wave's scratch list;
//   - the block: a raw literals section (the runs between matches, copied by
//     a lane per sequence after wave prefix sums place them), the sequences
//     section in predefined mode: the FSE bitstream (zstd_enc.h) written by
//     the wave in step (wave-uniform state, the three tables spread over the
//     lanes and the sequences read back 64 at a time, both taken by
//     readlane), lane 0 storing the bytes;
//   - a block that does not shrink goes out raw (its compressed attempt's
//     writes past the raw size are suppressed).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "encode.h"
#include "rio_internal.h"
#include "zstd_enc.h"

namespace rio {

constexpr int kZeHashBits = 12;                   // buckets of two 16-bit positions (16 KiB per wave)
constexpr int kZeWaves = 4;                      // waves per workgroup
constexpr uint32_t kZeMaxSeq = kZeBlock / 4 + 1;  // sequences per block (matches are >= 4 bytes)
constexpr uint32_t kZeWaveWords = kZeMaxSeq + kZeBlock / 8;  // per wave: the sequence list, then the literals
constexpr int kZeRing = 128;                      // Huffman stream staging dwords per wave

// payload bytes: varint header scratch, then the block's items
struct ZeSrc {
  const uint8_t *hdr;
  unsigned long long hlen;
  const uint8_t *data;
  unsigned long long len;
  __device__ __forceinline__ uint32_t byte(unsigned long long p) const { return p < hlen ? hdr[p] : data[p - hlen]; }
  // 16 bytes at p (bytes at or past len: 0, never loaded)
  __device__ __forceinline__ void load16(unsigned long long p, uint32_t (&w)[4]) const {
    const uint8_t *q = nullptr;
    if (p + 16 <= len) {
      if (p + 16 <= hlen) q = hdr + p;
      else if (p >= hlen) q = data + (p - hlen);
    }
    if (q) {
      // 5 aligned dwords funnel-shifted (v_alignbyte), branch-free across
      // lanes; an aligned q reloads dword 3 as the 5th (the next may lie past
      // the payload)
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

__device__ __forceinline__ uint32_t ze_common16(const uint32_t (&a)[4], const uint32_t (&b)[4]) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x = a[k] ^ b[k];
    if (x) return 4 * k + ((__ffs(x) - 1) >> 3);
  }
  return 16;
}

// bit writer of the wave: every lane keeps the same state, lane 0 stores;
// bytes at or past lim are not stored (a block that grows goes out raw)
struct ZeWaveBits {
  uint64_t acc;
  uint32_t nb;
  uint8_t *out;
  uint64_t pos, lim;
  bool st;
  __device__ __forceinline__ void put(uint32_t byte) {
    if (st && pos < lim) out[pos] = (uint8_t)byte;
    pos++;
  }
  __device__ __forceinline__ void add(uint32_t v, uint32_t n) {  // n <= 31
    acc |= (uint64_t)(v & (uint32_t)((1ull << n) - 1)) << nb;
    nb += n;
    if (nb >= 32) {  // a whole dword out (nb < 63 before)
      const uint32_t x = (uint32_t)acc;
      put(x);
      put(x >> 8);
      put(x >> 16);
      put(x >> 24);
      acc >>= 32;
      nb -= 32;
    }
  }
  __device__ __forceinline__ void close() {
    add(1, 1);
    while (nb > 0) {
      put((uint32_t)acc);
      acc >>= 8;
      nb = nb > 8 ? nb - 8 : 0;
    }
  }
};

// One FSE table held across the wave's lanes (state entries 2l, 2l+1 and
// 128+2l, 129+2l in lane l, symbol k's deltas in lane k): the encoder's state
// is wave-uniform, so every lookup is a readlane -- no memory latency in the
// serial chain
struct ZeLaneFse {
  uint32_t st0, st1, dnb;
  int32_t dfind;
  int32_t log;
  __device__ __forceinline__ void load(const ZeFse &t, int l) {
    const uint32_t *sw = reinterpret_cast<const uint32_t *>(t.state);
    st0 = sw[l];
    st1 = sw[64 + l];
    dnb = l < 53 ? t.dnb[l] : 0u;
    dfind = l < 53 ? t.dfind[l] : 0;
    log = t.log;
  }
  __device__ __forceinline__ uint32_t rd(uint32_t v, uint32_t k) const {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)k);
  }
  __device__ __forceinline__ uint32_t state_at(uint32_t k) const {
    const uint32_t lane = (k >> 1) & 63u;
    const uint32_t a = rd(st0, lane), b = rd(st1, lane);
    const uint32_t v = (k & 128u) ? b : a;
    return (k & 1u) ? (v >> 16) : (v & 0xffffu);
  }
  __device__ __forceinline__ uint32_t init(uint32_t sym) const {
    const uint32_t d = rd(dnb, sym);
    const uint32_t nbo = (d + (1u << 15)) >> 16;
    const uint32_t v = (nbo << 16) - d;
    return state_at((uint32_t)((int32_t)(v >> nbo) + (int32_t)rd((uint32_t)dfind, sym)));
  }
  __device__ __forceinline__ void encode(ZeWaveBits &w, uint32_t &s, uint32_t sym) const {
    const uint32_t nbo = (s + rd(dnb, sym)) >> 16;
    w.add(s, nbo);
    s = state_at((uint32_t)((int32_t)(s >> nbo) + (int32_t)rd((uint32_t)dfind, sym)));
  }
};

// the per-wave LDS a block's two coding phases share: literals (Huffman build,
// stream staging), then sequences (code counts, one table slot)
struct ZeHufLds {
  uint32_t hist[256];  // literal counts
  uint32_t w[260];     // Huffman build: node weights
  uint16_t par[260];   // ... parents
  uint16_t val[132];   // code values of symbols 0..128
  uint8_t len[132];    // code lengths
  uint32_t ring[kZeRing];  // stream bits being assembled
};
struct ZeFseLds {
  uint32_t cnt[3][56];  // LL, OF, ML code counts
  ZeFse t;              // the table being fitted
  ZeFseWork w;
  uint8_t desc[kZeDescMax];
};
constexpr int kZePhaseWords = ((sizeof(ZeHufLds) > sizeof(ZeFseLds) ? sizeof(ZeHufLds) : sizeof(ZeFseLds)) + 15) / 16 * 4;

// the wave's global stores complete (and visible to its other lanes' loads)
__device__ __forceinline__ void ze_mem_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ ZeSeq ze_unpack(unsigned long long v) {
  return ZeSeq{(uint32_t)(v & 0xffffu), (uint32_t)((v >> 16) & 0xffffu), (uint32_t)(v >> 32)};
}

__device__ __forceinline__ ZeSrc zsrc_of(const EncArgs &a, uint64_t b) {
  ZeSrc s;
  const uint64_t f0 = b * a.per_block;
  const uint64_t f = f0 < a.n_items ? f0 : a.n_items;
  s.hdr = a.hdr + a.hdr_off[b];
  s.hlen = a.hdr_len[b];
  s.data = a.data + (f == 0 ? 0ull : a.item_end[f - 1]);
  s.len = a.pay_len[b];
  return s;
}

__global__ void __launch_bounds__(64 * kZeWaves) k_zstd_enc(EncArgs a, const ZeTabs *__restrict__ T,
                                                          unsigned long long *__restrict__ scratch) {
  __shared__ uint32_t s_hash[kZeWaves][1 << kZeHashBits];
  __shared__ __attribute__((aligned(16))) uint32_t s_phase[kZeWaves][kZePhaseWords];
  const int wv = threadIdx.x >> 6;
  uint32_t *hash = s_hash[wv];
  ZeHufLds &H = *reinterpret_cast<ZeHufLds *>(s_phase[wv]);
  ZeFseLds &F = *reinterpret_cast<ZeFseLds *>(s_phase[wv]);
  uint32_t *hist = H.hist;
  uint16_t *hval = H.val;
  uint8_t *hlen = H.len;
  uint32_t *ring = H.ring;
  const int l = lane_id();
  const uint64_t wave = (uint64_t)blockIdx.x * kZeWaves + wv;
  const uint64_t nwaves = (uint64_t)gridDim.x * kZeWaves;
  unsigned long long *seq = scratch + wave * kZeWaveWords;
  uint8_t *lit = reinterpret_cast<uint8_t *>(seq + kZeMaxSeq);
  ZeLaneFse f_ll, f_ml, f_of;
  for (uint64_t b = wave; b < a.nblocks; b += nwaves) {
    const ZeSrc s = zsrc_of(a, b);
    const unsigned long long L = s.len;
    uint8_t *out = a.comp + a.comp_off[b];
    for (int i = l; i < (1 << kZeHashBits); i += 64) hash[i] = 0;  // (stale / empty entries: verified like any)
    wave_lds_sync();
    if (l == 0) ze_frame_header(out, L);
    unsigned long long o = kZeFrameHdr;
    if (L == 0 && l == 0) {  // one empty raw block
      out[o] = 1;
      out[o + 1] = 0;
      out[o + 2] = 0;
    }
    if (L == 0) o += 3;
    for (unsigned long long b0 = 0; b0 < L; b0 += kZeBlock) {
      const unsigned long long b1 = L - b0 < kZeBlock ? L : b0 + kZeBlock;
      const uint32_t bsz = (uint32_t)(b1 - b0);
      // ---- matches: rounds of 64 positions, greedy walk from the cursor
      uint32_t nseq = 0;
      unsigned long long cur = b0, lit_start = b0;
      uint32_t nx[4];
      s.load16(b0 + l, nx);
      for (unsigned long long base = b0; base < b1; base += 64) {
        const unsigned long long p = base + l;
        uint32_t cw[4] = {nx[0], nx[1], nx[2], nx[3]};
        if (base + 64 < b1) s.load16(p + 64, nx);
        const bool has4 = p + 4 <= b1;
        const uint32_t h = (cw[0] * 0x9E3779B1u) >> (32 - kZeHashBits);
        const uint32_t e = has4 ? hash[h] : 0u;
        wave_lds_sync();
        if (has4) hash[h] = (e << 16) | (uint32_t)(p & 0xffffu);  // the newer position in way 0
        // the two candidates: 16-bit positions, up to 64 KiB back (a stale
        // or empty entry is a candidate like any other: bytes decide)
        uint32_t m = 0, cand = 0;
        if (has4 && p >= cur) {
          const uint32_t maxm = (uint32_t)(b1 - p);
#pragma unroll
          for (int way = 0; way < 2; way++) {
            const uint32_t dd = (uint32_t)(p - (e >> (16 * way))) & 0xffffu;
            if (dd == 0 || dd > p) continue;
            const unsigned long long cd = p - dd;
            uint32_t cc[4];
            s.load16(cd, cc);
            uint32_t mk = ze_common16(cc, cw);
            while (mk == 16 * ((mk + 15) / 16) && mk > 0 && mk < maxm) {  // all equal so far
              uint32_t a16[4], b16[4];
              s.load16(cd + mk, a16);
              s.load16(p + mk, b16);
              const uint32_t k = ze_common16(a16, b16);
              mk += k;
              if (k < 16) break;
            }
            if (mk > maxm) mk = maxm;
            if (mk > m) {  // (ties: way 0, the nearer)
              m = mk;
              cand = (uint32_t)cd;
            }
          }
          if (m < 4) m = 0;
        }
        unsigned long long pos = cur;
        const unsigned long long rend = base + 64 < b1 ? base + 64 : b1;
        while (pos < rend) {
          const uint32_t lane = (uint32_t)(pos - base);
          const uint32_t ml = (uint32_t)__builtin_amdgcn_readlane((int)m, (int)lane);
          if (ml >= 4) {
            const uint32_t cd = (uint32_t)__builtin_amdgcn_readlane((int)cand, (int)lane);
            if (l == 0)
              seq[nseq] = (unsigned long long)(pos - lit_start) | ((unsigned long long)ml << 16) |
                          ((unsigned long long)(uint32_t)(pos - cd) << 32);
            nseq++;
            pos += ml;
            lit_start = pos;
          } else {
            pos++;
          }
        }
        cur = pos;
      }
      // ---- the block: header placeholder, raw literals, sequences
      const unsigned long long bh = o, lim = bh + 3 + bsz + 16;
      unsigned long long q = bh + 3;
      ze_mem_sync();  // the list's stores (lane 0) visible to every lane's loads
      unsigned long long nlit = 0;
      {  // literal count: the block minus its matches
        unsigned long long msum = 0;
        for (uint32_t g = 0; g < nseq; g += 64) {
          const uint32_t i = g + (uint32_t)l;
          const ZeSeq z = i < nseq ? ze_unpack(seq[i]) : ZeSeq{0, 0, 0};
          msum += wave_sum<unsigned long long>(z.ml);
        }
        nlit = bsz - msum;
      }
      // literals: the runs before every match (a lane per sequence, placed by
      // prefix sums) and the tail, gathered into the wave's scratch and counted
      for (int i = l; i < 256; i += 64) hist[i] = 0;
      wave_lds_sync();
      {
        unsigned long long src0 = b0, dst0 = 0;
        for (uint32_t g = 0; g < nseq; g += 64) {
          const uint32_t i = g + (uint32_t)l;
          const ZeSeq z = i < nseq ? ze_unpack(seq[i]) : ZeSeq{0, 0, 0};
          const uint32_t lin = wave_incl_sum_dpp(z.ll), tin = wave_incl_sum_dpp(z.ll + z.ml);
          const unsigned long long sp = src0 + (tin - z.ll - z.ml), dp = dst0 + (lin - z.ll);
          for (uint32_t k = 0; k < z.ll; k += 16) {  // 16 source bytes per load round
            uint32_t w16[4];
            s.load16(sp + k, w16);
#pragma unroll
            for (int j = 0; j < 16; j++)
              if (k + j < z.ll) {
                const uint32_t c = (w16[j >> 2] >> (8 * (j & 3))) & 0xffu;
                lit[dp + k + j] = (uint8_t)c;
                atomicAdd(&hist[c], 1u);
              }
          }
          src0 += (uint32_t)__builtin_amdgcn_readlane((int)tin, 63);
          dst0 += (uint32_t)__builtin_amdgcn_readlane((int)lin, 63);
        }
        for (unsigned long long k = l; src0 + k < b1; k += 64) {
          const uint32_t c = s.byte(src0 + k);
          lit[dst0 + k] = (uint8_t)c;
          atomicAdd(&hist[c], 1u);
        }
      }
      ze_mem_sync();  // the literals visible to every lane
      wave_lds_sync();
      // Huffman-coded literals (4 streams, direct weights) when they shrink
      bool huf = false;
      uint32_t hlast = 0, maxb = 0, seg = 0, sb[4] = {0, 0, 0, 0}, comp = 0, hn = 0;
      if (nlit >= 64) {
        uint32_t lmax = 0, ldist = 0;
        for (int k = l; k < 256; k += 64)
          if (hist[k]) {
            lmax = (uint32_t)k;
            ldist++;
          }
        uint32_t dist = ldist;
        for (int o2 = 32; o2 > 0; o2 >>= 1) {
          dist += (uint32_t)__shfl_xor((int)dist, o2, 64);
          const uint32_t t = (uint32_t)__shfl_xor((int)lmax, o2, 64);
          lmax = t > lmax ? t : lmax;
        }
        hlast = lmax;
        if (dist >= 2 && hlast <= 128) {
          if (l == 0) {
            ze_huf_lengths(hist, hlast + 1, hlen, H.w, H.par);
            maxb = ze_huf_codes(hlen, hlast + 1, hval);
          }
          maxb = (uint32_t)__builtin_amdgcn_readfirstlane((int)maxb);
          wave_lds_sync();
          seg = ze_seg((uint32_t)nlit);
          for (int k = 0; k < 4; k++) {  // each stream's bytes: its code bits + the end mark
            const uint32_t a0 = min((uint32_t)k * seg, (uint32_t)nlit);
            const uint32_t a1 = k < 3 ? min((uint32_t)(k + 1) * seg, (uint32_t)nlit) : (uint32_t)nlit;
            uint32_t bits = 0;
            for (uint32_t i = a0 + l; i < a1; i += 64) bits += hlen[lit[i]];
            bits = wave_sum<uint32_t>(bits);
            sb[k] = (bits + 1 + 7) / 8;
          }
          const uint32_t tree = 1 + (hlast + 1) / 2;
          comp = tree + 6 + sb[0] + sb[1] + sb[2] + sb[3];
          hn = (nlit <= 1023 && comp <= 1023) ? 3u : (nlit <= 16383 && comp <= 16383) ? 4u : 5u;
          huf = hn + comp < 3 + nlit && sb[0] < 65536 && sb[1] < 65536 && sb[2] < 65536;
        }
      }
      if (huf) {
        const uint32_t tree = 1 + (hlast + 1) / 2;
        if (l == 0) {
          ze_lit_header(out + q, (uint32_t)nlit, comp);
          ze_huf_weights(hlen, hlast, maxb, out + q + hn);
          uint8_t *jt = out + q + hn + tree;
          for (int k = 0; k < 3; k++) {
            jt[2 * k] = (uint8_t)sb[k];
            jt[2 * k + 1] = (uint8_t)(sb[k] >> 8);
          }
        }
        for (int i = l; i < kZeRing; i += 64) ring[i] = 0;  // (the sequence phase shares this LDS)
        wave_lds_sync();
        unsigned long long sbase = q + hn + tree + 6;
        for (int k = 0; k < 4; k++) {  // stream k: its symbols last to first, bits placed by a wave scan
          const uint32_t a0 = min((uint32_t)k * seg, (uint32_t)nlit);
          const uint32_t a1 = k < 3 ? min((uint32_t)(k + 1) * seg, (uint32_t)nlit) : (uint32_t)nlit;
          const uint32_t ns = a1 - a0;
          uint32_t bitpos = 0, flushed = 0;
          for (uint32_t e0 = 0; e0 <= ns; e0 += 64) {  // (the last round also places the end mark)
            const uint32_t e = e0 + (uint32_t)l;
            uint32_t ln = 0, v = 0;
            if (e < ns) {
              const uint32_t c = lit[a1 - 1 - e];
              ln = hlen[c];
              v = hval[c];
            } else if (e == ns) {
              ln = 1;  // the end mark
              v = 1;
            }
            const uint32_t incl = wave_incl_sum_dpp(ln);
            if (ln) {
              const uint32_t pos = bitpos + incl - ln, wd = pos >> 5, sh = pos & 31u;
              atomicOr(&ring[wd & (kZeRing - 1)], v << sh);
              if (sh + ln > 32) atomicOr(&ring[(wd + 1) & (kZeRing - 1)], v >> (32 - sh));
            }
            bitpos += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            wave_lds_sync();
            const bool fin = e0 + 64 > ns;
            const uint32_t nbytes = (bitpos + 7) >> 3;
            const uint32_t done = fin ? (nbytes + 3) >> 2 : bitpos >> 5;  // dwords complete (all at the end)
            if (flushed + (uint32_t)l < done) {
              const uint32_t d = flushed + (uint32_t)l, slot = d & (kZeRing - 1);
              const uint32_t x = ring[slot];
              ring[slot] = 0;
#pragma unroll
              for (int j = 0; j < 4; j++)
                if (4 * d + j < nbytes && sbase + 4 * d + j < lim) out[sbase + 4 * d + j] = (uint8_t)(x >> (8 * j));
            }
            flushed = done;
            wave_lds_sync();
          }
          sbase += sb[k];
        }
        q = sbase;
      } else {
        if (l == 0) {
          out[q] = (uint8_t)(0 | (3 << 2) | ((nlit & 15) << 4));  // Raw_Literals_Block, 20-bit size
          out[q + 1] = (uint8_t)(nlit >> 4);
          out[q + 2] = (uint8_t)(nlit >> 12);
        }
        for (unsigned long long k = l; k < nlit; k += 64) out[q + 3 + k] = lit[k];
        q += 3 + nlit;
      }
      // Number_of_Sequences, the modes byte, then per table (LL, OF, ML) a
      // fitted distribution's description where it codes the block's
      // sequences cheaper than the predefined one (zstd_enc.h ze_fit_table)
      const uint32_t nsb = nseq < 128 ? 1u : nseq < 0x7F00 ? 2u : 3u;
      if (l == 0) {
        if (nseq < 128) {
          out[q] = (uint8_t)nseq;
        } else if (nseq < 0x7F00) {
          out[q] = (uint8_t)((nseq >> 8) + 0x80);
          out[q + 1] = (uint8_t)nseq;
        } else {
          out[q] = 0xFF;
          out[q + 1] = (uint8_t)(nseq - 0x7F00);
          out[q + 2] = (uint8_t)((nseq - 0x7F00) >> 8);
        }
      }
      q += nsb;
      if (nseq) {
        wave_lds_sync();  // the literal phase's LDS is free
        for (int i = l; i < 3 * 56; i += 64) (&F.cnt[0][0])[i] = 0u;
        wave_lds_sync();
        for (uint32_t g = 0; g < nseq; g += 64) {
          const uint32_t i = g + (uint32_t)l;
          if (i < nseq) {
            const ZeSeq z = ze_unpack(seq[i]);
            atomicAdd(&F.cnt[0][ze_ll_code(z.ll)], 1u);
            atomicAdd(&F.cnt[1][ze_highbit(z.off + 3)], 1u);
            atomicAdd(&F.cnt[2][ze_ml_code(z.ml - 3)], 1u);
          }
        }
        wave_lds_sync();
        const unsigned long long mq = q;
        q += 1;
        uint32_t modes = 0;
#pragma unroll
        for (int t = 0; t < 3; t++) {
          const ZeFse &pre = t == 0 ? T->ll : t == 1 ? T->of : T->ml;
          uint32_t dl = 0;
          if (l == 0)
            dl = t == 0   ? ze_fit_table(F.cnt[0], 36, kZeLLNorm, kZeLLSyms, kZeLLLog, F.t, F.w, F.desc)
                 : t == 1 ? ze_fit_table(F.cnt[1], 32, kZeOFNorm, kZeOFSyms, kZeOFLog, F.t, F.w, F.desc)
                          : ze_fit_table(F.cnt[2], 53, kZeMLNorm, kZeMLSyms, kZeMLLog, F.t, F.w, F.desc);
          dl = (uint32_t)__builtin_amdgcn_readfirstlane((int)dl);
          wave_lds_sync();  // lane 0's table and description visible
          for (uint32_t k = (uint32_t)l; k < dl; k += 64)
            if (q + k < lim) out[q + k] = F.desc[k];
          q += dl;
          ZeLaneFse &f = t == 0 ? f_ll : t == 1 ? f_of : f_ml;
          f.load(dl ? F.t : pre, l);
          modes |= (dl ? 2u : 0u) << (6 - 2 * t);
          wave_lds_sync();  // the slot is free for the next table
        }
        if (l == 0 && mq < lim) out[mq] = (uint8_t)modes;
      }
      if (nseq) {  // the FSE bitstream, the wave in step, sequences from the last
        ZeWaveBits w{0, 0, out, q, lim, l == 0};
        uint32_t chunk = ~0u;
        unsigned long long v = 0;
        auto get = [&](uint32_t i) -> ZeSeq {
          if ((i >> 6) != chunk) {
            chunk = i >> 6;
            const uint32_t k = (chunk << 6) + (uint32_t)l;
            v = k < nseq ? seq[k] : 0ull;
          }
          const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)(i & 63));
          const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)(i & 63));
          return ze_unpack(((unsigned long long)hi << 32) | lo);
        };
        ZeSeq z = get(nseq - 1);
        uint32_t ofv = z.off + 3, mb = z.ml - 3;
        uint32_t llc = ze_ll_code(z.ll), mlc = ze_ml_code(mb), ofc = ze_highbit(ofv);
        uint32_t s_ml = f_ml.init(mlc), s_of = f_of.init(ofc), s_ll = f_ll.init(llc);
        w.add(z.ll, ze_ll_bits(llc));
        w.add(mb, ze_ml_bits(mlc));
        w.add(ofv, ofc);
        for (uint32_t i = nseq - 1; i-- > 0;) {
          z = get(i);
          ofv = z.off + 3;
          mb = z.ml - 3;
          llc = ze_ll_code(z.ll);
          mlc = ze_ml_code(mb);
          ofc = ze_highbit(ofv);
          f_of.encode(w, s_of, ofc);
          f_ml.encode(w, s_ml, mlc);
          f_ll.encode(w, s_ll, llc);
          w.add(z.ll, ze_ll_bits(llc));
          w.add(mb, ze_ml_bits(mlc));
          w.add(ofv, ofc);
        }
        w.add(s_ml, (uint32_t)f_ml.log);
        w.add(s_of, (uint32_t)f_of.log);
        w.add(s_ll, (uint32_t)f_ll.log);
        w.close();
        q = w.pos;
      }
      const bool last = b1 >= L;
      const unsigned long long csz = q - (bh + 3);
      uint32_t bhv;
      if (csz >= bsz) {  // raw block
        for (uint32_t k = l; k < bsz; k += 64) out[bh + 3 + k] = (uint8_t)s.byte(b0 + k);
        bhv = (last ? 1u : 0u) | (0u << 1) | (bsz << 3);
        o = bh + 3 + bsz;
      } else {
        bhv = (last ? 1u : 0u) | (2u << 1) | ((uint32_t)csz << 3);
        o = q;
      }
      if (l == 0) {
        out[bh] = (uint8_t)bhv;
        out[bh + 1] = (uint8_t)(bhv >> 8);
        out[bh + 2] = (uint8_t)(bhv >> 16);
      }
      wave_lds_sync();
    }
    if (l == 0) a.pay_len[b] = o;
  }
}

// per block: the frame's bound (into nck, scanned into comp_off)
__global__ void k_zstd_enc_bound(EncArgs a) {
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < a.nblocks;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long L = a.pay_len[b];
    const unsigned long long nblk = L / kZeBlock + 1;
    a.nck[b] = (kZeFrameHdr + L + 19 * nblk + 64 + 15) & ~15ull;
  }
}

void launch_zstd_enc_bound(const EncArgs &a, hipStream_t st) {
  uint64_t g = (a.nblocks + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(k_zstd_enc_bound, dim3((unsigned)(g ? g : 1)), dim3(256), 0, st, a);
}

static uint64_t zstd_enc_grid(int ncu) { return (uint64_t)(ncu > 0 ? ncu : 256) * 2; }  // 2 workgroups per CU (LDS)

uint64_t zstd_enc_scratch_words(int ncu) { return zstd_enc_grid(ncu) * kZeWaves * kZeWaveWords; }

void launch_zstd_enc(const EncArgs &a, const ZeTabs *tabs, unsigned long long *scratch, int ncu, hipStream_t st) {
  uint64_t g = (a.nblocks + kZeWaves - 1) / kZeWaves;
  const uint64_t cap = zstd_enc_grid(ncu);
  if (g > cap) g = cap;
  hipLaunchKernelGGL(k_zstd_enc, dim3((unsigned)(g ? g : 1)), dim3(64 * kZeWaves), 0, st, a, tabs, scratch);
}

}  // namespace rio
