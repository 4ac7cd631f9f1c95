// Raw DEFLATE (RFC 1951) block decode: the "flate" untransformer
// (recordioflate.FlateUncompress, recordio/recordioflate/recordioflate.go:54-65,
// through github.com/klauspost/compress v1.8.6 flate -- Go's compress/flate
// inflater: go.mod:24). One wave per recordio block.
//
// The compressed block is the concatenation of its chunk payloads (the
// IOVecReader view, recordioiov.go:14-58). The wave stages 2 KiB of it at a time
// into LDS (64 lanes, one coalesced pass), every lane runs the same bit-reader
// and Huffman decode (uniform state: no divergence, LDS reads broadcast), and
// output goes through an 8 KiB LDS window ring: literals and near matches are
// LDS copies (lane-parallel for matches), each completed 1 KiB is flushed to the
// block's decode region in HBM with one 16 B/lane store, and matches further
// back than the ring read the flushed bytes from HBM.
//
// The fast decoder refills the bit buffer greedily. Go's inflater pulls bytes
// lazily (moreBits), which only matters for *where* an error is reported
// (CorruptInputError's offset is its roffset) and for rejecting a truncated
// stream; so on any error the block is re-decoded by inflate_exact, a
// single-lane restatement with Go's lazy byte pulls that produces the
// reference's error and offset (it writes nothing: an erroring block yields no
// records). Decoding stops at the end of the BFINAL block; trailing bytes are
// ignored, as in Go.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "rio_internal.h"

namespace rio {

constexpr int kInflWaves = 1;    // waves per workgroup (LDS-bound residency: one wave per workgroup)
constexpr int kInBuf = 1024;     // input staging bytes
#ifndef RIO_INFL_WIN
#define RIO_INFL_WIN 8192
#endif
constexpr int kWin = RIO_INFL_WIN;  // output window ring
constexpr int kUnit = 1024;      // flush granule
constexpr int kLitBits = 10;     // root table bits: literal/length
constexpr int kDistBits = 8;     // root table bits: distance (and code-length codes)
constexpr int kMaxBits = 15;

struct HuffT {
  uint16_t count[kMaxBits + 1];
  uint16_t sym[288];
  int32_t min, max, empty, ok;
};

struct InflLds {
  uint8_t win[kWin];
  uint32_t in32[kInBuf / 4 + 4];  // staged compressed bytes
  uint16_t lfast[1 << kLitBits];  // (len << 9) | sym for codes <= kLitBits, 0: longer code
  uint16_t dfast[1 << kDistBits];
  HuffT lit, dist;                // code-length codes are decoded through `dist` / dfast
  uint8_t lens[320];
  uint8_t cl[20];
  uint16_t offs[kMaxBits + 2];
};

// wave-uniform value (LDS loads are per lane; this makes them scalar)
// (the builtin returns int: widen through uint32_t, never sign-extend)
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
  return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------------------- tables
__device__ __forceinline__ uint32_t rev_bits(uint32_t code, int len) { return __brev(code) >> (32 - len); }

// huffmanDecoder.init semantics (Go inflate.go): a code set must be complete,
// except the degenerate single code of length 1; all-zero lengths = empty tree.
// Built by lane 0 (a few thousand cycles per DEFLATE block).
__device__ __attribute__((noinline)) void huff_build(HuffT &h, const uint8_t *lens, int n, uint16_t *offs,
                                                     uint16_t *fast, int fbits) {
  for (int i = 0; i <= kMaxBits; i++) h.count[i] = 0;
  int mn = 0, mx = 0;
  for (int i = 0; i < n; i++) {
    const int l = lens[i];
    if (!l) continue;
    if (mn == 0 || l < mn) mn = l;
    if (l > mx) mx = l;
    h.count[l]++;
  }
  h.min = mn;
  h.max = mx;
  h.empty = (mx == 0);
  h.ok = 1;
  if (h.empty) return;
  int code = 0;
  for (int i = mn; i <= mx; i++) code = (code << 1) + h.count[i];
  if (code != (1 << mx) && !(code == 1 && mx == 1)) {
    h.ok = 0;
    return;
  }
  offs[1] = 0;
  for (int l = 1; l <= kMaxBits; l++) offs[l + 1] = offs[l] + h.count[l];
  for (int i = 0; i < n; i++)
    if (lens[i]) h.sym[offs[lens[i]]++] = (uint16_t)i;
  for (int i = 0; i < (1 << fbits); i++) fast[i] = 0;
  int next = 0, k = 0;
  for (int l = 1; l <= kMaxBits; l++) {
    for (int j = 0; j < h.count[l]; j++, k++) {
      if (l <= fbits) {
        const uint32_t r = rev_bits((uint32_t)(next + j), l);
        for (uint32_t f = r; f < (1u << fbits); f += (1u << l)) fast[f] = (uint16_t)((l << 9) | h.sym[k]);
      }
    }
    next = (next + h.count[l]) << 1;
  }
}

// canonical decode of `bits` (LSB first); returns sym, sets len (0: none)
__device__ __forceinline__ int huff_slow(const HuffT &h, uint32_t bits, int &len) {
  int code = 0, first = 0, index = 0;
  for (int l = 1; l <= kMaxBits; l++) {
    code |= (int)((bits >> (l - 1)) & 1u);
    const int cnt = h.count[l];
    if (code - cnt < first) {
      len = l;
      return h.sym[index + (code - first)];
    }
    index += cnt;
    first += cnt;
    first <<= 1;
    code <<= 1;
  }
  len = 0;
  return -1;
}

// ---------------------------------------------------------------- input view
// Logical compressed bytes [0, n): the block's chunk payloads back to back.
struct CompIn {
  const uint8_t *span;
  uint64_t span_bytes;            // RIO_CHECKED bounds
  unsigned long long *flag;       // RIO_CHECKED violation flags (ctl->out_overflow)
  const uint32_t *ck_size;
  const unsigned long long *ck_pay;
  uint64_t c0, total, n, pay0;
  bool regular;
  __device__ __forceinline__ uint64_t phys(uint64_t p) const {
    uint64_t c, lo;
    if (regular) {
      uint64_t j = p / kMaxPayload;
      if (j >= total) j = total - 1;
      c = c0 + j;
      lo = j * kMaxPayload;
    } else {
      uint64_t a = c0, b = c0 + total;
      while (b - a > 1) {
        const uint64_t m = (a + b) >> 1;
        if (ck_pay[m] - pay0 <= p) a = m;
        else b = m;
      }
      c = a;
      lo = ck_pay[a] - pay0;
    }
    return c * kChunk + kChunkHdr + (p - lo);
  }
  __device__ __forceinline__ uint32_t byte(uint64_t p) const {
    if (p >= n) return 0u;
    const uint64_t q = phys(p);
#ifdef RIO_CHECKED
    if (q >= span_bytes) {
      atomicOr(flag, 0x100ull);
      return 0u;
    }
#endif
    return span[q];
  }
};

// ---------------------------------------------------------------- exact mode
// Single-lane restatement of Go's inflater (oracle/inflate.c follows the same
// rules) used only to classify a failing block: lazy byte pulls, so the error
// offset is Go's roffset. No output is written.
struct Exact {
  const CompIn *in;
  uint64_t pos;
  uint64_t bitbuf;
  int nb;
  uint64_t olen, cap;
  int err;
  uint64_t err_off;
  __device__ bool more() {
    if (pos >= in->n) {
      if (!err) err = kCodecEof;
      return false;
    }
    bitbuf |= (uint64_t)in->byte(pos++) << nb;
    nb += 8;
    return true;
  }
  __device__ bool need(int n) {
    while (nb < n)
      if (!more()) return false;
    return true;
  }
  __device__ uint32_t take(int n) {
    const uint32_t v = (uint32_t)(bitbuf & ((1ull << n) - 1));
    bitbuf >>= n;
    nb -= n;
    return v;
  }
  __device__ void corrupt() {
    if (!err) {
      err = kCodecCorrupt;
      err_off = pos;
    }
  }
  __device__ int sym(const HuffT &h, const uint16_t *fast, int fbits) {
    if (h.empty) {
      if (!need(h.min)) return -1;
      corrupt();
      return -1;
    }
    int n = h.min;
    for (;;) {
      if (!need(n)) return -1;
      const int avail = nb < kMaxBits ? nb : kMaxBits;
      const uint32_t bits = (uint32_t)(bitbuf & ((1u << avail) - 1));
      int len = 0, s = -1;
      const uint16_t e = fast[bits & ((1u << fbits) - 1)];
      if (e && (e >> 9) <= avail) {
        len = e >> 9;
        s = e & 511;
      }
      if (s < 0) s = huff_slow(h, bits, len);
      if (s < 0) {
        corrupt();
        return -1;
      }
      if (len <= nb) {
        take(len);
        return s;
      }
      n = len;
    }
  }
};

__device__ void fixed_lens(uint8_t *l) {
  int i = 0;
  for (; i < 144; i++) l[i] = 8;
  for (; i < 256; i++) l[i] = 9;
  for (; i < 280; i++) l[i] = 7;
  for (; i < 288; i++) l[i] = 8;
}

__device__ const uint8_t kClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// lane 0 only; tables in lds (clobbered)
__device__ void inflate_exact(const CompIn &in, InflLds &L, uint64_t cap, uint32_t &err, uint64_t &err_off,
                              uint64_t &olen) {
  Exact s{&in, 0, 0, 0, 0, cap, 0, 0};
  bool fixed_built = false;
  for (;;) {
    if (!s.need(3)) break;
    const int final = (int)s.take(1);
    const int type = (int)s.take(2);
    bool ok = true;
    if (type == 0) {
      s.nb = 0;
      s.bitbuf = 0;
      if (s.pos + 4 > in.n) {
        s.pos = in.n;
        s.err = kCodecEof;
        break;
      }
      const uint32_t len = in.byte(s.pos) | (in.byte(s.pos + 1) << 8);
      const uint32_t nlen = in.byte(s.pos + 2) | (in.byte(s.pos + 3) << 8);
      s.pos += 4;
      if ((uint16_t)nlen != (uint16_t)~len) {
        s.corrupt();
        break;
      }
      if (s.olen + len > s.cap) {
        s.err = kCodecFull;
        break;
      }
      if (s.pos + len > in.n) {
        s.err = kCodecEof;
        break;
      }
      s.olen += len;
      s.pos += len;
    } else if (type == 1 || type == 2) {
      const HuffT *hl = &L.lit, *hd = nullptr;
      if (type == 1) {
        if (!fixed_built) {
          fixed_lens(L.lens);
          huff_build(L.lit, L.lens, 288, L.offs, L.lfast, kLitBits);
        }
        fixed_built = true;
      } else {
        fixed_built = false;
        if (!s.need(14)) break;
        const int nlit = (int)s.take(5) + 257;
        if (nlit > 286) {
          s.corrupt();
          break;
        }
        const int ndist = (int)s.take(5) + 1;
        if (ndist > 30) {
          s.corrupt();
          break;
        }
        const int nclen = (int)s.take(4) + 4;
        for (int i = 0; i < 19; i++) L.cl[i] = 0;
        bool okc = true;
        for (int i = 0; i < nclen; i++) {
          if (!s.need(3)) {
            okc = false;
            break;
          }
          L.cl[kClenOrder[i]] = (uint8_t)s.take(3);
        }
        if (!okc) break;
        huff_build(L.dist, L.cl, 19, L.offs, L.dfast, kDistBits);  // code-length code
        if (!L.dist.ok) {
          s.corrupt();
          break;
        }
        const int n = nlit + ndist;
        int i = 0;
        while (i < n) {
          const int x = s.sym(L.dist, L.dfast, kDistBits);
          if (x < 0) break;
          if (x < 16) {
            L.lens[i++] = (uint8_t)x;
            continue;
          }
          int rep, nbits, b;
          if (x == 16) {
            rep = 3;
            nbits = 2;
            if (i == 0) {
              s.corrupt();
              break;
            }
            b = L.lens[i - 1];
          } else if (x == 17) {
            rep = 3;
            nbits = 3;
            b = 0;
          } else {
            rep = 11;
            nbits = 7;
            b = 0;
          }
          if (!s.need(nbits)) break;
          rep += (int)s.take(nbits);
          if (i + rep > n) {
            s.corrupt();
            break;
          }
          for (int j = 0; j < rep; j++) L.lens[i++] = (uint8_t)b;
        }
        if (s.err || i < n) break;
        huff_build(L.lit, L.lens, nlit, L.offs, L.lfast, kLitBits);
        huff_build(L.dist, L.lens + nlit, ndist, L.offs, L.dfast, kDistBits);
        if (!L.lit.ok || !L.dist.ok) {
          s.corrupt();
          break;
        }
        if (!L.lit.empty && L.lit.min < L.lens[256]) L.lit.min = L.lens[256];  // h1.min = len(EOB)
        hd = &L.dist;
      }
      // huffmanBlock
      for (;;) {
        const int v = s.sym(*hl, L.lfast, kLitBits);
        if (v < 0) {
          ok = false;
          break;
        }
        if (v < 256) {
          if (s.olen >= s.cap) {
            s.err = kCodecFull;
            ok = false;
            break;
          }
          s.olen++;
          continue;
        }
        if (v == 256) break;
        int length, nbits;
        if (v < 265) { length = v - (257 - 3); nbits = 0; }
        else if (v < 269) { length = v * 2 - (265 * 2 - 11); nbits = 1; }
        else if (v < 273) { length = v * 4 - (269 * 4 - 19); nbits = 2; }
        else if (v < 277) { length = v * 8 - (273 * 8 - 35); nbits = 3; }
        else if (v < 281) { length = v * 16 - (277 * 16 - 67); nbits = 4; }
        else if (v < 285) { length = v * 32 - (281 * 32 - 131); nbits = 5; }
        else if (v < 286) { length = 258; nbits = 0; }
        else {
          s.corrupt();
          ok = false;
          break;
        }
        if (nbits > 0) {
          if (!s.need(nbits)) {
            ok = false;
            break;
          }
          length += (int)s.take(nbits);
        }
        int dist;
        if (hd == nullptr) {
          if (!s.need(5)) {
            ok = false;
            break;
          }
          dist = (int)rev_bits(s.take(5), 5);
        } else {
          dist = s.sym(*hd, L.dfast, kDistBits);
          if (dist < 0) {
            ok = false;
            break;
          }
        }
        if (dist < 4) {
          dist++;
        } else if (dist < 30) {
          const int nb = (dist - 2) >> 1;
          int extra = (dist & 1) << nb;
          if (!s.need(nb)) {
            ok = false;
            break;
          }
          extra |= (int)s.take(nb);
          dist = (1 << (nb + 1)) + 1 + extra;
        } else {
          s.corrupt();
          ok = false;
          break;
        }
        const uint64_t hist = s.olen < 32768 ? s.olen : 32768;
        if ((uint64_t)dist > hist) {
          s.corrupt();
          ok = false;
          break;
        }
        if (s.olen + length > s.cap) {
          s.err = kCodecFull;
          ok = false;
          break;
        }
        s.olen += length;
      }
    } else {
      s.corrupt();
      break;
    }
    if (!ok || s.err) break;
    if (final) break;
  }
  err = s.err;
  err_off = s.err_off;
  olen = s.olen;
}

// ---------------------------------------------------------------- fast mode
// Decoder state is wave-uniform: every value read from LDS goes through uni()
// (v_readfirstlane), so the bit reader and the Huffman walk run on the scalar
// unit; the vector lanes do the wave-parallel parts (staging, LZ77 copies,
// flushes).
struct Fast {
  const CompIn *in;
  InflLds *L;
  uint8_t *out;      // the block's decode region in HBM
  uint64_t cap;
  uint64_t out_room; // RIO_CHECKED: bytes addressable from out
  uint64_t base;     // logical offset of the staged bytes (multiple of 4)
  uint64_t pos;      // next logical byte for the bit buffer
  uint64_t bitbuf;
  int nb;
  uint64_t olen, flushed;

  // stage logical bytes [b & ~3, + kInBuf + 16) into LDS, all lanes
  __device__ void stage(uint64_t b) {
    const int l = lane_id();
    base = b & ~3ull;
    wave_lds_sync();
    uint8_t *dst = reinterpret_cast<uint8_t *>(L->in32);
    for (int k = l; k < kInBuf + 16; k += 64) dst[k] = (uint8_t)in->byte(base + k);
    wave_lds_sync();
  }
  __device__ __forceinline__ uint32_t in_byte(uint64_t p) {
    const uint32_t o = (uint32_t)(p - base);
    return (uni(L->in32[o >> 2]) >> (8 * (o & 3))) & 0xffu;
  }
  __device__ __forceinline__ void refill() {
    if (nb > 32) return;
    if (pos < base || pos + 8 > base + kInBuf) stage(pos);
    const uint32_t o = (uint32_t)(pos - base);
    const uint32_t d0 = uni(L->in32[o >> 2]), d1 = uni(L->in32[(o >> 2) + 1]);
    const uint32_t w = (uint32_t)((((uint64_t)d1 << 32) | d0) >> (8 * (o & 3)));
    bitbuf |= (uint64_t)w << nb;
    nb += 32;
    pos += 4;
  }
  __device__ __forceinline__ uint32_t take(int n) {
    const uint32_t v = (uint32_t)(bitbuf & ((1ull << n) - 1));
    bitbuf >>= n;
    nb -= n;
    return v;
  }
  // bits consumed past the end of the input: the stream is truncated
  __device__ __forceinline__ bool overrun() const { return 8 * pos - (uint64_t)nb > 8 * in->n; }
  __device__ __forceinline__ int sym(const HuffT &h, const uint16_t *fast, int fbits) {
    const uint32_t bits = (uint32_t)bitbuf;
    const uint32_t e = uni(fast[bits & ((1u << fbits) - 1)]);
    int len, s;
    if (e) {
      len = (int)(e >> 9);
      s = (int)(e & 511);
    } else {  // canonical walk for codes longer than the root table
      int code = 0, first = 0, index = 0;
      s = -1;
      len = 0;
      for (int l = 1; l <= kMaxBits; l++) {
        code |= (int)((bits >> (l - 1)) & 1u);
        const int cnt = (int)uni(h.count[l]);
        if (code - cnt < first) {
          len = l;
          s = (int)uni(h.sym[index + (code - first)]);
          break;
        }
        index += cnt;
        first += cnt;
        first <<= 1;
        code <<= 1;
      }
      if (s < 0) return -1;
    }
    take(len);
    return s;
  }
  // write completed flush units [flushed, olen rounded down) to HBM
  __device__ void flush_units() {
    const int l = lane_id();
    if (olen - flushed < (uint64_t)kUnit) return;
    wave_lds_sync();
    while (olen - flushed >= (uint64_t)kUnit) {
      const uint32_t r = (uint32_t)(flushed & (kWin - 1));
      const uint4 v = *reinterpret_cast<const uint4 *>(L->win + r + 16 * l);
#ifdef RIO_CHECKED
      if (flushed + 16 * l + 16 > out_room) {
        atomicOr(in->flag, 0x200ull);
      } else
#endif
      *reinterpret_cast<uint4 *>(out + flushed + 16 * l) = v;
      flushed += kUnit;
    }
  }
  __device__ void flush_tail() {
    flush_units();
    wave_lds_sync();
    const int l = lane_id();
    for (uint64_t k = flushed + l; k < olen; k += 64) {
#ifdef RIO_CHECKED
      if (k >= out_room) {
        atomicOr(in->flag, 0x400ull);
        continue;
      }
#endif
      out[k] = L->win[k & (kWin - 1)];
    }
    flushed = olen;
  }
  __device__ __forceinline__ void literal(uint32_t v) {
    if (lane_id() == 0) L->win[olen & (kWin - 1)] = (uint8_t)v;
    olen++;
    if ((olen & (kUnit - 1)) == 0) flush_units();
  }
  // LZ77 copy: every source byte precedes olen, so all lanes copy at once
  __device__ void copy(uint32_t dist, uint32_t length) {
    const int l = lane_id();
    wave_lds_sync();
    if (dist <= (uint32_t)(kWin - kUnit - 258)) {
      for (uint32_t k0 = 0; k0 < length; k0 += 64) {
        const uint32_t k = k0 + l;
        uint8_t v = 0;
        if (k < length) {
          const uint32_t kk = (k < dist) ? k : (k % dist);
          v = L->win[(olen - dist + kk) & (kWin - 1)];
        }
        wave_lds_sync();
        if (k < length) L->win[(olen + k) & (kWin - 1)] = v;
      }
    } else {  // older than the ring: the flushed bytes in HBM
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      for (uint32_t k0 = 0; k0 < length; k0 += 64) {
        const uint32_t k = k0 + l;
        if (k < length) {
          const uint32_t kk = (k < dist) ? k : (k % dist);
#ifdef RIO_CHECKED
          if (olen - dist + kk >= out_room) {
            atomicOr(in->flag, 0x800ull);
            continue;
          }
#endif
          L->win[(olen + k) & (kWin - 1)] = out[olen - dist + kk];
        }
      }
    }
    wave_lds_sync();
    olen += length;
    flush_units();
  }
  __device__ void stored(uint32_t len) {
    const int l = lane_id();
    uint32_t done = 0;
    while (done < len) {
      if (pos < base || pos + 64 > base + kInBuf) stage(pos);
      const uint32_t n = (len - done) < 64u ? (len - done) : 64u;
      const uint32_t room = (uint32_t)(kUnit - (olen & (kUnit - 1)));
      const uint32_t m = n < room ? n : room;
      const uint8_t *src = reinterpret_cast<const uint8_t *>(L->in32) + (pos - base);
      if ((uint32_t)l < m) L->win[(olen + l) & (kWin - 1)] = src[l];
      wave_lds_sync();
      pos += m;
      olen += m;
      done += m;
      if ((olen & (kUnit - 1)) == 0) flush_units();
    }
  }
};

// Returns 0 (ok; olen set) or a CodecErr for the exact pass to classify.
__device__ int inflate_fast(Fast &f) {
  InflLds &L = *f.L;
  const int l = lane_id();
  bool fixed_built = false;
  for (;;) {
    f.refill();
    const int final = (int)f.take(1);
    const int type = (int)f.take(2);
    if (f.overrun()) return kCodecEof;
    if (type == 0) {
      // discard the rest of the current byte; whole bytes read ahead go back
      f.take(f.nb & 7);
      f.pos -= (uint64_t)(f.nb >> 3);
      f.nb = 0;
      f.bitbuf = 0;
      if (f.pos + 4 > f.in->n) return kCodecEof;
      // the bytes given back may precede the staged window
      if (f.pos < f.base || f.pos + 8 > f.base + kInBuf) f.stage(f.pos);
      const uint32_t len = f.in_byte(f.pos) | (f.in_byte(f.pos + 1) << 8);
      const uint32_t nlen = f.in_byte(f.pos + 2) | (f.in_byte(f.pos + 3) << 8);
      f.pos += 4;
      if ((uint16_t)nlen != (uint16_t)~len) return kCodecCorrupt;
      if (f.olen + len > f.cap) return kCodecFull;
      if (f.pos + len > f.in->n) return kCodecEof;
      f.stored(len);
    } else if (type == 1 || type == 2) {
      bool has_dist = true;
      if (type == 1) {
        if (!fixed_built) {
          wave_lds_sync();
          if (l == 0) {
            fixed_lens(L.lens);
            huff_build(L.lit, L.lens, 288, L.offs, L.lfast, kLitBits);
          }
          wave_lds_sync();
        }
        fixed_built = true;
        has_dist = false;
      } else {
        fixed_built = false;
        f.refill();
        const int nlit = (int)f.take(5) + 257;
        const int ndist = (int)f.take(5) + 1;
        const int nclen = (int)f.take(4) + 4;
        if (nlit > 286 || ndist > 30) return kCodecCorrupt;
        wave_lds_sync();
        if (l == 0)
          for (int i = 0; i < 19; i++) L.cl[i] = 0;
        for (int i = 0; i < nclen; i++) {
          f.refill();
          const uint32_t v = f.take(3);
          if (l == 0) L.cl[kClenOrder[i]] = (uint8_t)v;
        }
        wave_lds_sync();
        if (l == 0) huff_build(L.dist, L.cl, 19, L.offs, L.dfast, kDistBits);
        wave_lds_sync();
        if (!uni(L.dist.ok) || uni(L.dist.empty)) return kCodecCorrupt;
        const int n = nlit + ndist;
        int i = 0, prev = 0;
        while (i < n) {
          f.refill();
          const int x = f.sym(L.dist, L.dfast, kDistBits);
          if (x < 0) return kCodecCorrupt;
          if (x < 16) {
            if (l == 0) L.lens[i] = (uint8_t)x;
            prev = x;
            i++;
            continue;
          }
          int rep, b;
          if (x == 16) {
            if (i == 0) return kCodecCorrupt;
            b = prev;
            rep = 3 + (int)f.take(2);
          } else if (x == 17) {
            b = 0;
            rep = 3 + (int)f.take(3);
          } else {
            b = 0;
            rep = 11 + (int)f.take(7);
          }
          if (i + rep > n) return kCodecCorrupt;
          for (int j = l; j < rep; j += 64) L.lens[i + j] = (uint8_t)b;
          prev = b;
          i += rep;
        }
        if (f.overrun()) return kCodecEof;
        wave_lds_sync();
        if (l == 0) {
          huff_build(L.lit, L.lens, nlit, L.offs, L.lfast, kLitBits);
          huff_build(L.dist, L.lens + nlit, ndist, L.offs, L.dfast, kDistBits);
        }
        wave_lds_sync();
        if (!uni(L.lit.ok) || !uni(L.dist.ok) || uni(L.lit.empty)) return kCodecCorrupt;
      }
      const bool dist_empty = has_dist && uni(L.dist.empty);
      // huffmanBlock
      for (;;) {
        f.refill();
        const int v = f.sym(L.lit, L.lfast, kLitBits);
        if (v < 0) return kCodecCorrupt;
        if (v < 256) {
          if (f.olen >= f.cap) return kCodecFull;
          f.literal((uint32_t)v);
          continue;
        }
        if (f.overrun()) return kCodecEof;
        if (v == 256) break;
        int length, nbits;
        if (v < 265) { length = v - (257 - 3); nbits = 0; }
        else if (v < 269) { length = v * 2 - (265 * 2 - 11); nbits = 1; }
        else if (v < 273) { length = v * 4 - (269 * 4 - 19); nbits = 2; }
        else if (v < 277) { length = v * 8 - (273 * 8 - 35); nbits = 3; }
        else if (v < 281) { length = v * 16 - (277 * 16 - 67); nbits = 4; }
        else if (v < 285) { length = v * 32 - (281 * 32 - 131); nbits = 5; }
        else if (v < 286) { length = 258; nbits = 0; }
        else return kCodecCorrupt;
        if (nbits > 0) length += (int)f.take(nbits);
        f.refill();
        int dist;
        if (!has_dist) {
          dist = (int)rev_bits(f.take(5), 5);
        } else {
          if (dist_empty) return kCodecCorrupt;
          dist = f.sym(L.dist, L.dfast, kDistBits);
          if (dist < 0) return kCodecCorrupt;
        }
        if (dist < 4) {
          dist++;
        } else if (dist < 30) {
          const int nb = (dist - 2) >> 1;
          const int extra = ((dist & 1) << nb) | (int)f.take(nb);
          dist = (1 << (nb + 1)) + 1 + extra;
        } else {
          return kCodecCorrupt;
        }
        if (f.overrun()) return kCodecEof;
        const uint64_t hist = f.olen < 32768 ? f.olen : 32768;
        if ((uint64_t)dist > hist) return kCodecCorrupt;
        if (f.olen + length > f.cap) return kCodecFull;
        f.copy((uint32_t)dist, (uint32_t)length);
      }
    } else {
      return kCodecCorrupt;
    }
    if (f.overrun()) return kCodecEof;
    if (final) break;
  }
  f.flush_tail();
  return 0;
}

__global__ void __launch_bounds__(64 * kInflWaves) k_inflate(const uint8_t *__restrict__ span, DevBufs d,
                                                             const unsigned long long *nblocks, uint64_t nchunks,
                                                             uint64_t dec_cap) {
  __shared__ InflLds s_lds[kInflWaves];
  InflLds &L = s_lds[threadIdx.x >> 6];
  const int l = lane_id();
  const uint64_t nb = *nblocks;
  // one wave per workgroup: the block index is wave-uniform, so the decoder
  // state derived from it lives in scalar registers (no exec-mask branches)
  static_assert(kInflWaves == 1, "k_inflate assumes one wave per workgroup");
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
    CompIn in;
    in.span = span;
    in.span_bytes = nchunks * (uint64_t)kChunk;
    in.flag = &d.ctl->out_overflow;
    in.ck_size = d.ck_size;
    in.ck_pay = d.ck_pay;
    in.c0 = c0;
    in.total = meta & kMetaTotalMask;
    in.n = uni64(d.blk_len[b]);
    in.pay0 = uni64(d.ck_pay[c0]);
    in.regular = (meta & kMetaRegular) != 0;
    const uint64_t off = uni64(d.blk_dec_off[b]);
    const uint64_t cap = uni64(d.blk_out_len[b]);  // the bound from k_codec_prepare
    if (off + cap > dec_cap) {  // the regions need a larger buffer (host retries)
      if (l == 0) {
        atomicOr(&d.ctl->out_overflow, 0x40ull);
        atomicMax(&d.ctl->dec_need, (unsigned long long)(off + cap));
        d.blk_out_len[b] = 0;
      }
      continue;
    }
    Fast f;
    f.in = &in;
    f.L = &L;
    f.out = d.dec + off;
    f.out_room = dec_cap - off;
    f.cap = cap;
    f.base = 0;
    f.pos = 0;
    f.bitbuf = 0;
    f.nb = 0;
    f.olen = 0;
    f.flushed = 0;
    f.stage(0);
    const int err = inflate_fast(f);
    if (l == 0) {
      if (err) {  // k_inflate_exact classifies it (Go's lazy byte pulls) or sizes it
        d.blk_status[b] = kBlkCodec;
        d.blk_a[b] = kCodecPending;
        d.blk_b[b] = (unsigned long long)err;
        d.blk_hdr[b] = f.olen | ((unsigned long long)f.pos << 32);  // where the fast pass stopped (debug)
      }
      d.blk_out_len[b] = err ? 0 : f.olen;
    }
  }
}

// The blocks k_inflate failed on: the exact restatement gives the reference's
// error (and CorruptInputError offset). One wave per failing block, lane 0.
__global__ void __launch_bounds__(64) k_inflate_exact(const uint8_t *__restrict__ span, DevBufs d,
                                                      const unsigned long long *nblocks) {
  __shared__ InflLds L;
  const int l = lane_id();
  const uint64_t nb = *nblocks;
  for (uint64_t g = (uint64_t)blockIdx.x * 64; g < nb; g += (uint64_t)gridDim.x * 64) {
    const bool pend = (g + l < nb) && d.blk_status[g + l] == kBlkCodec && d.blk_a[g + l] == kCodecPending;
    unsigned long long pm = __ballot(pend);
    while (pm) {
      const uint64_t b = g + __ffsll((long long)pm) - 1;
      pm &= pm - 1;
      if (l == 0) {
        const unsigned long long meta = d.blk_meta[b];
        CompIn in;
        in.span = span;
        in.span_bytes = ~0ull;
        in.flag = &d.ctl->out_overflow;
        in.ck_size = d.ck_size;
        in.ck_pay = d.ck_pay;
        in.c0 = d.blk_c0[b];
        in.total = meta & kMetaTotalMask;
        in.n = d.blk_len[b];
        in.pay0 = d.ck_pay[in.c0];
        in.regular = (meta & kMetaRegular) != 0;
        uint32_t e = 0;
        uint64_t eo = 0, olen = 0;
        inflate_exact(in, L, ~0ull >> 1, e, eo, olen);
        if (e == 0 && d.blk_b[b] == kCodecFull) {
          // a valid stream larger than its decode region: the retry sizes it exactly
          d.blk_need[b] = olen;
          atomicOr(&d.ctl->out_overflow, 8ull);
          e = kCodecFull;
        } else if (e == 0 || e == kCodecFull) {
          e = kCodecCorrupt;  // fast and exact disagree: never pass silently
        }
        d.blk_a[b] = e;
        d.blk_b[b] = eo;
      }
    }
  }
}

void launch_inflate(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks,
                    uint64_t nchunks, uint64_t dec_cap, hipStream_t st) {
  uint64_t g = (max_blocks + kInflWaves - 1) / kInflWaves;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(k_inflate, dim3((unsigned)g), dim3(64 * kInflWaves), 0, st, span, d, nblocks, nchunks, dec_cap);
  uint64_t ge = (max_blocks + 63) / 64;
  if (ge > 1024) ge = 1024;
  if (ge < 1) ge = 1;
  hipLaunchKernelGGL(k_inflate_exact, dim3((unsigned)ge), dim3(64), 0, st, span, d, nblocks);
}

}  // namespace rio
