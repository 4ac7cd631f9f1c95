// Raw DEFLATE (RFC 1951) block decode: the "flate" untransformer
// (recordioflate.FlateUncompress, recordio/recordioflate/recordioflate.go:54-65,
// through github.com/klauspost/compress v1.8.6 flate -- Go's compress/flate
// inflater: go.mod:24).
//
// The compressed block is the concatenation of its chunk payloads (the
// IOVecReader view, recordioiov.go:14-58); decoding stops at the end of the
// BFINAL block and trailing bytes are ignored, as in Go.
//
// The fast path (k_flate_sync / k_flate_tok + k_flate_lz2, below) decodes valid streams. Go's
// inflater pulls bytes lazily (moreBits), which only matters for *where* an
// error is reported (CorruptInputError's offset is its roffset) and for
// rejecting a truncated stream; so on any error the block is re-decoded by
// inflate_exact, a single-lane restatement with Go's lazy byte pulls that
// produces the reference's error and offset (it writes nothing: an erroring
// block yields no records).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "rio_internal.h"
#include "lz_ring.h"

namespace rio {

// RIO_TOK_TRACE (debug builds only): every global access of the fallback
// Huffman pass is logged, per lane, into host-coherent memory before it is
// made (a 16-entry ring per lane: seq | site << 48, address), so that after a
// memory fault the host can read each lane's last access.
#ifdef RIO_TOK_TRACE
#include <stdio.h>
#include <string.h>
__device__ unsigned long long *g_tok_trace;
__device__ __forceinline__ void tok_trace(uint32_t site, const volatile void *p) {
  unsigned long long *t = g_tok_trace;
  if (!t) return;
  const uint64_t slot = ((uint64_t)blockIdx.x * 64 + (threadIdx.x & 63)) * 34;
  const unsigned long long seq =
      __hip_atomic_load(&t[slot + 33], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
  __hip_atomic_store(&t[slot + 33], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t e = slot + 2 * (seq & 15);
  __hip_atomic_store(&t[e + 1], (unsigned long long)(uintptr_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&t[e], seq | ((unsigned long long)site << 48), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_s_waitcnt(0);
}
#define RIO_TT(site, p) tok_trace((site), (p))
#else
#define RIO_TT(site, p) ((void)0)
#endif

constexpr int kLitBits = 10;     // root table bits: literal/length
constexpr int kDistBits = 8;     // root table bits: distance (and code-length codes)
constexpr int kMaxBits = 15;

struct HuffT {
  uint16_t count[kMaxBits + 1];
  uint16_t sym[288];
  int32_t min, max, empty, ok;
};

// LDS of the exact (error-classifying) pass
struct InflLds {
  uint16_t lfast[1 << kLitBits];  // (len << 9) | sym for codes <= kLitBits, 0: longer code
  uint16_t dfast[1 << kDistBits];
  HuffT lit, dist;                // code-length codes are decoded through `dist` / dfast
  uint8_t lens[320];
  uint8_t cl[20];
  uint16_t offs[kMaxBits + 2];
};

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
        RIO_TT(11, &ck_pay[m]);
        if (ck_pay[m] - pay0 <= p) a = m;
        else b = m;
      }
      c = a;
      RIO_TT(12, &ck_pay[a]);
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
    RIO_TT(10, &span[q]);
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


// ================================================================ fast path
// Two passes per round (SURVEY.md §7 "DEFLATE kernel"):
//
// k_flate_tok -- Huffman pass, on the vector ALU: a wave decodes 8 recordio
//   blocks at once, 8 lanes per block (a "stream"; its state is the same in
//   all 8 lanes), so every VALU instruction advances 8 streams. Per stream,
//   ~4.7 KiB of LDS: the two Huffman tables (literal/length 10-bit root of
//   u16 entries, distance 8-bit root of u32 entries with base and extra bits
//   precomputed), canonical data for longer codes, a 512 B input ring
//   refilled every 8 steps from a 16 B/lane prefetch issued 8 steps earlier,
//   and a 16-token buffer stored to HBM at the same point. Rare events -- a
//   DEFLATE block header, the table build for a dynamic block, picking up the
//   next recordio block, writing a block's result -- "escape" to wave-uniform
//   scalar code for that one stream (readlane in, cndmask back).
// k_flate_lz2 -- copy pass (below): one wave per block, the 32 KiB history in
//   HBM (the block's own decode region) and a 4 KiB LDS ring per batch of up
//   to 256 tokens.
//
// A block whose token region fills yields (FlState) and resumes in the next
// round: the Huffman pass re-reads the current block header to rebuild its
// tables, the copy pass reloads the last 32 KiB it wrote.
//
// Token (u32):
//   bit 31 = 0: 1-3 literals, count in bits 25:24, bytes in 7:0, 15:8, 23:16
//   bit 31 = 1: match, length-3 in bits 23:16, distance-1 in bits 14:0

// Table entries. Literal/length (u16): code length (3:0; 0 = not decodable
// from the root), bit 4 set for a length or end-of-block, length extra bits
// (7:5; 7 = end-of-block), literal byte or length base - 3 (15:8).
// Distance (u16): code length (3:0), m (6:5), extra bits (10:7), with
// base = (m << extra) + 1. Code-length alphabet (u16): code length (3:0),
// symbol (12:8).
// Code length 0 with bit 4 set (kLongMark) marks a code longer than the root
// (canonical walk); an all-zero entry is a bit pattern no code has or a
// symbol DEFLATE never assigns (literal/length 286-287, distance 30-31):
// decoding it is a corrupt stream (Go: CorruptInputError).
constexpr uint32_t kEnLenBit = 0x10;
constexpr uint32_t kLongMark = kEnLenBit;
constexpr uint32_t kEobExtra = 7;
enum : int { kTabLit = 0, kTabDist = 1, kTabClen = 2 };
enum : int { kTokDone = 0, kTokYield = -1 };
#ifndef RIO_LIT_ROOT
#define RIO_LIT_ROOT 10  // (round 3: 9 -> 10, C3 49.8 -> 51.2 GiB/s A/B; 11 and 12, or a 9-bit distance root: ~40)
#endif
constexpr int kTokLitRoot = RIO_LIT_ROOT;  // literal/length root table bits
#ifndef RIO_DIST_ROOT
#define RIO_DIST_ROOT 8
#endif
constexpr int kTokDistRoot = RIO_DIST_ROOT;  // distance root table bits

// RFC 1951 §3.2.5 length / distance bases and extra bits
__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,    65,    97,    129,
                                       193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

__device__ __forceinline__ uint32_t tab_entry(int kind, uint32_t s, uint32_t len) {
  if (kind == kTabLit) {
    if (s < 256) return len | (s << 8);
    if (s == 256) return len | kEnLenBit | (kEobExtra << 5);
    if (s < 286)
      return len | kEnLenBit | ((uint32_t)kLenExtra[s - 257] << 5) | ((uint32_t)(kLenBase[s - 257] - 3) << 8);
    return 0;
  }
  if (kind == kTabDist) {  // base = (m << extra) + 1
    if (s >= 30) return 0u;
    const uint32_t m = s < 4 ? s : 2u | (s & 1), ex = s < 4 ? 0u : (s >> 1) - 1;
    return len | (m << 5) | (ex << 7);
  }
  return len | (s << 8);
}

#ifndef RIO_FL_LANES
#define RIO_FL_LANES 8
#endif
constexpr int kVG = RIO_FL_LANES;  // lanes per stream (its state is the same in all of them)
constexpr int kVS = 64 / kVG;      // streams per wave
constexpr int kPf = 16 / kVG;      // prefetched ring dwords per lane (16 per stream)
// Input ring per stream: 32 dwords, refilled with 16 (a 2-dword prefetch per
// lane) whenever at most 16 are left. A pass decodes at most kPass symbols,
// <= 48 bits = 1.5 dwords each, so at most 12 dwords: a ring that starts a
// pass with >= 14 dwords never runs dry (the two ahead of rpos stay valid),
// and after the refill it holds >= 17 again (18 after a seek). A refill
// replaces dwords [rhi - 32, rhi - 16), all consumed.
constexpr int kRingDw = 32;
constexpr int kTbuf = 10;      // tokens per stream per pass: 1 per step + 2 slack (a failed hot step's write)
constexpr int kPass = 8;       // decode steps between input passes

// Canonical code data per code length (first code 15:0, count 31:16, index
// of its first entry in canonical order 47:32); streams keep the lengths
// longer than their root tables, for the canonical walk.
struct __attribute__((aligned(16))) StreamLds {
  uint32_t ring[kRingDw];
  uint32_t tbuf[kTbuf];
  uint64_t lfco[15 - kTokLitRoot], dfco[15 - kTokDistRoot];
  uint16_t lit[1 << kTokLitRoot];
  uint16_t dst[1 << kTokDistRoot];  // also the code-length table while a header is read
  uint16_t lent[288], dent[32];     // entries of codes longer than the root, canonical order (code length 0)
};
// per wave: scratch of the header reads and table builds (escapes work on
// one stream at a time)
struct WaveLds {
  uint64_t fco[16];
  uint8_t lens[320];
  uint8_t cl[24];
};

// Wave-cooperative table build with huffmanDecoder.init's rules (Go
// compress/flate inflate.go): returns 0 ok, 1 empty (no codes: decoding with
// it fails), 2 incomplete or oversubscribed (corrupt), except that a single
// code of length 1 is accepted (its other half decodes as a zero entry).
// Ranks within a length come from ballots, so every lane places its own
// symbol; entries of codes up to `root` bits are replicated by their lanes.
template <class TT>
__device__ __forceinline__ int build_table(const uint8_t *lens, int n, TT *tab, int root, uint64_t *sfco,
                                           uint64_t *lfco, TT *sorted, int kind) {
  const int l = lane_id();
  uint32_t cnt[16];
#pragma unroll
  for (int i = 0; i < 16; i++) cnt[i] = 0;
  uint32_t myl[5], rank[5];
#pragma unroll
  for (int c = 0; c < 5; c++) {
    myl[c] = 0;
    rank[c] = 0;
    if (c * 64 < n) {
      const int s = c * 64 + l;
      myl[c] = s < n ? lens[s] : 0u;
#pragma unroll
      for (int L = 1; L <= 15; L++) {
        const unsigned long long m = __ballot(myl[c] == (uint32_t)L);
        if (myl[c] == (uint32_t)L)
          rank[c] = cnt[L] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        cnt[L] += (uint32_t)__popcll(m);
      }
    }
  }
  int mn = 0, mx = 0;
#pragma unroll
  for (int L = 1; L <= 15; L++)
    if (cnt[L]) {
      if (!mn) mn = L;
      mx = L;
    }
  for (int i = l; i < (1 << root); i += 64) tab[i] = (TT)0;
  if (mx == 0) {
    wave_lds_sync();
    return 1;
  }
  uint32_t code = 0;
#pragma unroll
  for (int L = 1; L <= 15; L++)
    if (L >= mn && L <= mx) code = (code << 1) + cnt[L];
  if (code != (1u << mx) && !(code == 1 && mx == 1)) return 2;
  uint32_t c = 0, o = 0;
  uint32_t first[16], offs[16];
  first[0] = offs[0] = 0;
#pragma unroll
  for (int L = 1; L <= 15; L++) {
    c = (c + cnt[L - 1]) << 1;
    first[L] = c;
    offs[L] = o;
    o += cnt[L];
  }
  if (l < 16) {
    uint32_t fc = 0, oc = 0, cc = 0;
#pragma unroll
    for (int L = 0; L < 16; L++)
      if (l == L) {
        fc = first[L];
        oc = offs[L];
        cc = cnt[L];
      }
    const uint64_t v = (uint64_t)(fc & 0xffffu) | ((uint64_t)cc << 16) | ((uint64_t)oc << 32);
    sfco[l] = v;
    if (l > root) lfco[l - root - 1] = v;
  }
  wave_lds_sync();
#pragma unroll
  for (int k = 0; k < 5; k++) {
    if (k * 64 < n) {
      const uint32_t L = myl[k];
      if (L) {
        const uint32_t s = (uint32_t)(k * 64 + l);
        const uint64_t fco = sfco[L];
        const uint32_t cd = (uint32_t)(fco & 0xffffu) + rank[k];
        const uint32_t rev = __brev(cd) >> (32 - L);
        if ((int)L <= root) {
          const TT e = (TT)tab_entry(kind, s, L);
          for (uint32_t f = rev; f < (1u << root); f += (1u << L)) tab[f] = e;
        } else {
#ifdef RIO_CHECKED
          if ((uint32_t)(fco >> 32) + rank[k] >= (root == kTokLitRoot ? 288u : 32u)) {
            printf("build_table: sorted %u out of range (root %d, kind %d, n %d)\n", (uint32_t)(fco >> 32) + rank[k],
                   root, kind, n);
            continue;
          }
#endif
          sorted[(uint32_t)(fco >> 32) + rank[k]] = (TT)tab_entry(kind, s, 0);
          tab[rev & ((1u << root) - 1)] = (TT)kLongMark;
        }
      }
    }
  }
  wave_lds_sync();
  return 0;
}

// entry of a code longer than the root table (canonical walk; per lane): the
// canonical data of every longer length is read at once, then one entry
template <int kRoot, class TT>
__device__ __forceinline__ uint32_t slow_walk(const uint64_t *lfco, const TT *sorted, uint32_t bits) {
  constexpr int kN = 15 - kRoot;
  uint64_t f[kN];
#pragma unroll
  for (int i = 0; i < kN; i++) f[i] = lfco[i];
  const uint32_t rb = __brev(bits);
  uint32_t idx = 0xffffffffu, len = 0;
#pragma unroll
  for (int i = kN - 1; i >= 0; i--) {  // the shortest match wins (codes are prefix-free)
    const uint32_t L = kRoot + 1 + i;
    const uint32_t c = rb >> (32 - L);
    const uint32_t d = c - (uint32_t)(f[i] & 0xffffu);
    if (d < (uint32_t)((f[i] >> 16) & 0xffffu)) {
      idx = (uint32_t)(f[i] >> 32) + d;
      len = L;
    }
  }
#ifdef RIO_CHECKED
  if (idx != 0xffffffffu && idx >= (kRoot == kTokLitRoot ? 288u : 32u)) {
    printf("slow_walk: entry %u out of range (root %d, bits %08x)\n", idx, kRoot, bits);
    return 0u;
  }
#endif
  return idx == 0xffffffffu ? 0u : ((uint32_t)sorted[idx] | len);
}

// logical compressed dword at byte p (a multiple of 4); bytes at/after n read 0
__device__ __forceinline__ uint32_t fetch_dword(const CompIn &in, uint64_t p) {
  if (p >= in.n) return 0u;
  uint32_t v;
  if (in.regular) {  // chunk payloads of 32,740 B = 8,185 dwords: a dword never crosses a chunk
    const uint32_t q = (uint32_t)(p >> 2);
    const uint32_t jj = q / (kMaxPayload / 4);
    const uint64_t w = (in.c0 + jj) * (uint64_t)(kChunk / 4) + kChunkHdr / 4 + (q - jj * (kMaxPayload / 4));
#ifdef RIO_CHECKED
    if (4 * w + 4 > in.span_bytes) {
      atomicOr(in.flag, 0x100ull);
      return 0u;
    }
#endif
    RIO_TT(13, &reinterpret_cast<const uint32_t *>(in.span)[w]);
    v = reinterpret_cast<const uint32_t *>(in.span)[w];
  } else {
    v = in.byte(p) | (in.byte(p + 1) << 8) | (in.byte(p + 2) << 16) | (in.byte(p + 3) << 24);
  }
  if (p + 4 > in.n) v &= 0xffffffffu >> (8 * (uint32_t)(p + 4 - in.n));
  return v;
}

// Wave-uniform bit reader over one stream (block headers, in escapes): the
// stream's bytes through two 512 B VGPR windows (lane l holds dwords l and
// 64+l), read with v_readlane.
struct TokDec {
  CompIn in;
  StreamLds *T;
  WaveLds *W;
  uint32_t c0, c1, n0, n1;
  uint64_t wbase;
  uint32_t wi;
  uint64_t bitbuf;
  int nb;

  __device__ __forceinline__ uint32_t win_dword(uint64_t b, int k) const {
    return fetch_dword(in, b + 4 * (uint64_t)(64 * k + lane_id()));
  }
  __device__ __forceinline__ void seek(uint64_t bit) {
    const uint64_t byte = (bit >> 5) << 2;
    wbase = byte;
    wi = 0;
    c0 = win_dword(byte, 0);
    c1 = win_dword(byte, 1);
    n0 = win_dword(byte + 512, 0);
    n1 = win_dword(byte + 512, 1);
    bitbuf = 0;
    nb = 0;
    refill();
    take((int)(bit & 31));
  }
  __device__ __forceinline__ void refill() {
    if (wi >= 128) {
      c0 = n0;
      c1 = n1;
      wbase += 512;
      wi -= 128;
      n0 = win_dword(wbase + 512, 0);
      n1 = win_dword(wbase + 512, 1);
    }
    const uint32_t v = (wi & 64) ? c1 : c0;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readlane(v, wi & 63);
    bitbuf |= (uint64_t)w << nb;
    nb += 32;
    wi++;
    // wave-uniform by construction; re-assert it so the state stays in SGPRs
    bitbuf = uni64(bitbuf);
    nb = (int)uni((uint32_t)nb);
    wi = uni(wi);
    wbase = uni64(wbase);
  }
  __device__ __forceinline__ uint32_t take(int k) {
    const uint32_t v = (uint32_t)(bitbuf & ((1ull << k) - 1));
    bitbuf >>= k;
    nb -= k;
    return v;
  }
  __device__ __forceinline__ uint64_t bitpos() const { return 8 * (wbase + 4 * (uint64_t)wi) - (uint64_t)nb; }
  __device__ __forceinline__ bool overrun() const { return bitpos() > 8 * in.n; }
};

__device__ __forceinline__ void fixed_tables(StreamLds &T, WaveLds &W) {
  const int l = lane_id();
  wave_lds_sync();
  for (int i = l; i < 288; i += 64) W.lens[i] = (uint8_t)(i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8);
  wave_lds_sync();
  build_table(W.lens, 288, T.lit, kTokLitRoot, W.fco, T.lfco, T.lent, kTabLit);
  for (int i = l; i < 32; i += 64) W.lens[i] = 5;
  wave_lds_sync();
  build_table(W.lens, 32, T.dst, kTokDistRoot, W.fco, T.dfco, T.dent, kTabDist);
}

// dynamic block header (RFC 1951 §3.2.7; Go inflate.go readHuffman)
__device__ __forceinline__ int read_dynamic(TokDec &t) {
  StreamLds &T = *t.T;
  WaveLds &W = *t.W;
  const int l = lane_id();
  if (t.nb < 32) t.refill();
  const uint32_t nlit = t.take(5) + 257, ndist = t.take(5) + 1, nclen = t.take(4) + 4;
  if (nlit > 286 || ndist > 30) return kCodecCorrupt;
  wave_lds_sync();
  if (l < 19) W.cl[l] = 0;
  wave_lds_sync();
  for (uint32_t i = 0; i < nclen; i++) {
    if (t.nb < 32) t.refill();
    const uint32_t v = t.take(3);
    if (l == 0) W.cl[kClenOrder[i]] = (uint8_t)v;
  }
  wave_lds_sync();
  if (build_table(W.cl, 19, T.dst, kTokDistRoot, W.fco, T.dfco, T.dent, kTabClen) != 0) return kCodecCorrupt;
  const uint32_t n = nlit + ndist;
  uint32_t i = 0, prev = 0;
  while (i < n) {
    if (t.nb < 32) t.refill();
    const uint32_t e = uni(T.dst[t.bitbuf & ((1u << kTokDistRoot) - 1)]);
    const uint32_t L = e & 15;
    if (!L) return kCodecCorrupt;
    t.take((int)L);
    const uint32_t x = e >> 8;
    if (x < 16) {
      if (l == 0) W.lens[i] = (uint8_t)x;
      prev = x;
      i++;
      continue;
    }
    uint32_t rep, b;
    if (x == 16) {
      if (i == 0) return kCodecCorrupt;
      b = prev;
      rep = 3 + t.take(2);
    } else if (x == 17) {
      b = 0;
      rep = 3 + t.take(3);
    } else {
      b = 0;
      rep = 11 + t.take(7);
    }
    if (i + rep > n) return kCodecCorrupt;
    for (uint32_t j = l; j < rep; j += 64) W.lens[i + j] = (uint8_t)b;
    prev = b;
    i += rep;
  }
  wave_lds_sync();
  if (build_table(W.lens, (int)nlit, T.lit, kTokLitRoot, W.fco, T.lfco, T.lent, kTabLit) != 0) return kCodecCorrupt;
  if (build_table(W.lens + nlit, (int)ndist, T.dst, kTokDistRoot, W.fco, T.dfco, T.dent, kTabDist) == 2)
    return kCodecCorrupt;
  return 0;
}

// stream modes of k_flate_tok
enum : uint32_t {
  kVHuff = 0,    // decoding symbols of a fixed / dynamic block
  kVStored = 1,  // copying a stored block's bytes into literal tokens
  kVHeader = 2,  // escape: read the next DEFLATE block header
  kVFinish = 3,  // escape: write the block's result (res)
  kVNew = 4,     // escape: pick up the next recordio block
  kVGone = 5,    // no blocks left
};

__device__ __forceinline__ uint32_t rl32(uint32_t v, uint32_t lane) {
  return (uint32_t)__builtin_amdgcn_readlane(v, lane);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t lane) {
  return ((uint64_t)rl32((uint32_t)(v >> 32), lane) << 32) | rl32((uint32_t)v, lane);
}

__device__ __forceinline__ CompIn make_in(const uint8_t *span, const DevBufs &d, uint64_t nchunks, uint64_t c0,
                                          uint64_t total, uint64_t n, bool regular) {
  CompIn in;
  in.span = span;
  in.span_bytes = nchunks * (uint64_t)kChunk;
  in.flag = &d.ctl->out_overflow;
  in.ck_size = d.ck_size;
  in.ck_pay = d.ck_pay;
  in.c0 = c0;
  in.total = total;
  in.n = n;
  RIO_TT(14, &d.ck_pay[c0]);
  in.pay0 = d.ck_pay[c0];
  in.regular = regular;
  return in;
}

__global__ void __launch_bounds__(64) k_flate_tok(const uint8_t *__restrict__ span, DevBufs d,
                                                  const unsigned long long *nblocks, uint64_t nchunks,
                                                  uint64_t dec_cap, int round, int last_round) {
  __shared__ StreamLds S[kVS];
  __shared__ WaveLds W;
  const int l = lane_id();
  const uint32_t g = (uint32_t)l / kVG, j = (uint32_t)l % kVG;
  StreamLds &M = S[g];
  if (round > 0 && uni64(d.fl_more[round - 1]) == 0) return;
  RIO_TT(1, nblocks);
  const uint64_t nblk = uni64(*nblocks);
  const uint64_t stride = (uint64_t)gridDim.x * kVS;

  // stream state (the same in the kVG lanes of a group)
  uint64_t next_b = (uint64_t)blockIdx.x * kVS + g, cur_b = 0;
  uint32_t mode = kVNew, res = 0;
  uint32_t bc0 = 0, bn = 0, btot = 0, breg = 0, tcap = 0, cap = 0;  // block
  // bit reader: stream dwords rpos-2 (lo) and rpos-1 (hi), bit offset o < 32
  // into lo; nw0 / nw1 = ring dwords rpos, rpos+1 (requested one step ahead).
  // The 32-bit window at the read position is alignbit(hi, lo, o): >= 33
  // valid bits, enough for any code plus its extra bits.
  uint32_t lo = 0, hi = 0, o = 0, rpos = 0, rhi = 0, nw0 = 0, nw1 = 0;
  uint32_t pf[kPf];  // next 64 B of the ring
#pragma unroll
  for (int i = 0; i < kPf; i++) pf[i] = 0;
  uint32_t olen = 0, fin = 0, left = 0, fixed_ok = 0;  // decode
  uint64_t hdrpos = 0;
  uint32_t nst = 0, nv = 0;  // tokens stored / buffered in tbuf

  for (;;) {
    // ---------------------------------------------------------- escapes
    unsigned long long esc = __ballot(j == 0 && mode >= kVHeader && mode <= kVNew);
    while (esc) {
#ifdef RIO_FLSTAT
      if (l == 0) atomicAdd(&d.ctl->flstat_esc, 1ull);
#endif
      const uint32_t gl = (uint32_t)__ffsll((long long)esc) - 1;
      esc &= esc - 1;
      const uint32_t gg = gl / kVG;
      const bool mine = g == gg;
      StreamLds &G = S[gg];
      uint32_t sm = rl32(mode, gl);
      uint64_t sb = rl64(cur_b, gl);
      uint32_t s_c0 = rl32(bc0, gl), s_n = rl32(bn, gl), s_tot = rl32(btot, gl), s_reg = rl32(breg, gl);
      uint32_t s_olen = rl32(olen, gl), s_fin = rl32(fin, gl), s_left = rl32(left, gl), s_fixed = rl32(fixed_ok, gl);
      uint32_t s_nst = rl32(nst, gl);
      uint64_t s_hdr = rl64(hdrpos, gl);
      uint64_t s_bit = 32 * ((uint64_t)rl32(rpos, gl) - 2) + rl32(o, gl);
      uint64_t s_next = rl64(next_b, gl);
      uint32_t s_tcap = rl32(tcap, gl), s_cap = rl32(cap, gl);
      bool seek = false;
      int r = 0;
      if (sm == kVFinish) {
        r = (int)rl32(res, gl);
        FlState *sp = &d.fl[sb];
        RIO_TT(20, sp);
        RIO_TT(21, &d.blk_out_len[sb]);
        uint32_t stm = kFlDone;
        if (r == kTokYield) {
          stm = s_left ? kFlStored : (s_fixed ? kFlFixed : kFlDynamic);
          if (last_round) {  // more rounds needed than were launched: the host retries with more
            if (l == 0) atomicOr(&d.ctl->out_overflow, 0x1000ull);
            stm = kFlSkip;
          }
        }
        if (l == 0) {
          sp->round = (uint32_t)round;
          sp->ntok = s_nst;
          if (round == 0) sp->olen2 = 0;
          if (stm == kFlSkip) {
            sp->mode = kFlSkip;
            d.blk_out_len[sb] = 0;
          } else if (r == kTokDone || r == kTokYield) {
            sp->mode = stm;
            sp->olen = s_olen;
            if (r == kTokYield) {
              sp->bitpos = s_bit;
              sp->hdrpos = s_hdr;
              sp->final_ = s_fin;
              sp->stored_left = s_left;
              atomicAdd(&d.fl_more[round], 1ull);
            }
          } else {  // k_inflate_exact classifies it (Go's lazy byte pulls) or sizes it
            sp->bitpos = s_bit;  // where the fast pass stopped and why (RIO_DEBUG)
            sp->olen = s_olen;
            sp->pad = (uint32_t)r;
            sp->mode = kFlError;
            d.blk_status[sb] = kBlkCodec;
            d.blk_a[sb] = r == kCodecUnsupported ? (unsigned long long)kCodecUnsupported : kCodecPending;
            d.blk_b[sb] = (unsigned long long)r;
            d.blk_out_len[sb] = 0;
          }
        }
        sm = kVNew;
        r = 0;
      }
      if (sm == kVNew) {
        for (;;) {
          if (s_next >= nblk) {
            sm = kVGone;
            break;
          }
          sb = s_next;
          s_next += stride;
          FlState *sp = &d.fl[sb];
          RIO_TT(22, sp);
          RIO_TT(23, &d.blk_c0[sb]);
          RIO_TT(24, &d.blk_dec_off[sb]);
          const uint64_t c0 = uni64(d.blk_c0[sb]);
          const unsigned long long meta = uni64(d.blk_meta[sb]);
          uint32_t stm;
          if (round == 0 && uni(sp->mode) != kFlHeader) continue;  // k_flate_sync handled it
          if (round == 0) {
            const uint32_t cls = (uint32_t)(meta >> kMetaClsShift) & 0xffu;
            // incomplete blocks, and magics that are never untransformed (the header
            // block is idTransform, registry.go:31; others are errors): nothing decoded
            bool skip = !(meta & kMetaComplete) || (cls != kMagicPacked && cls != kMagicTrailer);
            const uint64_t off = uni64(d.blk_dec_off[sb]), cp = uni64(d.blk_out_len[sb]);
            if (!skip && off + cp > dec_cap) {  // the regions need a larger buffer (host retries)
              skip = true;
              if (l == 0) {
                atomicOr(&d.ctl->out_overflow, 0x40ull);
                atomicMax(&d.ctl->dec_need, (unsigned long long)(off + cp));
              }
            }
            if (skip) {
              if (l == 0) {
                sp->mode = kFlSkip;
                sp->round = 0;
                d.blk_out_len[sb] = 0;
              }
              continue;
            }
            stm = kFlHeader;
            s_bit = s_hdr = 0;
            s_olen = s_fin = s_left = 0;
          } else {
            stm = uni(sp->mode);
            if (stm >= kFlDone) continue;
            s_bit = uni64(sp->bitpos);
            s_hdr = uni64(sp->hdrpos);
            s_olen = (uint32_t)uni64(sp->olen);
            s_fin = uni(sp->final_);
            s_left = uni(sp->stored_left);
          }
          const uint64_t n = uni64(d.blk_len[sb]);
          const uint64_t total = meta & kMetaTotalMask;
          uint64_t tc = total * (uint64_t)kTokPerChunk;
          if (d.tok_limit && d.tok_limit < tc) tc = d.tok_limit < 64 ? 64 : d.tok_limit;
          const uint64_t cp = uni64(d.blk_out_len[sb]);
          s_c0 = (uint32_t)c0;
          s_n = (uint32_t)n;
          s_tot = (uint32_t)total;
          s_reg = (meta & kMetaRegular) != 0;
          s_tcap = tc > 0xffffff00ull ? 0xffffff00u : (uint32_t)tc;
          s_cap = cp > 0xfffff000ull ? 0xfffff000u : (uint32_t)cp;
          s_nst = 0;
          s_fixed = 0;
          if (n >= (1ull << 28) || c0 >= (1ull << 32)) {  // beyond the 32-bit stream state of this kernel
            r = kCodecUnsupported;
            sm = kVFinish;
            break;
          }
          if (stm == kFlDynamic) {
            TokDec t;
            t.in = make_in(span, d, nchunks, c0, total, n, s_reg != 0);
            t.T = &G;
            t.W = &W;
            t.seek(s_hdr);
            if (read_dynamic(t)) {
              r = kCodecCorrupt;
              sm = kVFinish;
              break;
            }
          } else if (stm == kFlFixed) {
            fixed_tables(G, W);
            s_fixed = 1;
          }
          sm = stm == kFlHeader ? kVHeader : stm == kFlStored ? kVStored : kVHuff;
          seek = sm != kVHeader;
          break;
        }
      }
      // The stream's input view, made from its block fields, which are defined
      // on every path (round 4's fault: a CompIn assigned only on some paths
      // through the loop above was merged by the compiler with an undefined
      // value, and a block header read of an irregular block -- the only reads
      // that take the chunk-payload map from it -- used that as the map's base)
      const CompIn in = make_in(span, d, nchunks, s_c0, s_tot, s_n, s_reg != 0);
      // DEFLATE block headers until a block with content (or the end)
      while (sm == kVHeader) {
        TokDec t;
        t.in = in;
        t.T = &G;
        t.W = &W;
        t.seek(s_bit);
        if (t.nb < 32) t.refill();
        s_fin = t.take(1);
        const uint32_t type = t.take(2);
        if (type == 0) {
          t.take(t.nb & 7);  // to the byte boundary
          if (t.nb < 32) t.refill();
          const uint32_t len = t.take(16), nlen = t.take(16);
          if ((uint16_t)nlen != (uint16_t)~len) r = kCodecCorrupt;
          else if (t.bitpos() / 8 + len > in.n) r = kCodecEof;
          else if (len > s_cap - s_olen) r = kCodecFull;
          s_left = len;
          sm = kVStored;
        } else if (type == 1) {
          if (!s_fixed) fixed_tables(G, W);
          s_fixed = 1;
          sm = kVHuff;
        } else if (type == 2) {
          s_hdr = t.bitpos();
          r = read_dynamic(t);
          s_fixed = 0;
          sm = kVHuff;
        } else {
          r = kCodecCorrupt;
        }
        if (!r && t.overrun()) r = kCodecEof;
        s_bit = t.bitpos();
        if (r) {
          sm = kVFinish;
        } else if (sm == kVStored && s_left == 0) {  // empty stored block
          sm = s_fin ? kVFinish : kVHeader;
          r = kTokDone;
        }
        seek = sm != kVFinish;
      }
      // write the stream state back to its lanes
      if (seek) {  // refill the ring at s_bit: 32 dwords from the 16 B boundary before it
        const uint32_t dw = (uint32_t)(s_bit >> 5), base = dw & ~3u;
        wave_lds_sync();
        if (l < 32) G.ring[(base + l) & (kRingDw - 1)] = fetch_dword(in, 4 * (uint64_t)(base + l));
        wave_lds_sync();
        if (mine) {
          lo = M.ring[dw & (kRingDw - 1)];
          hi = M.ring[(dw + 1) & (kRingDw - 1)];
          o = (uint32_t)(s_bit & 31);
          rpos = dw + 2;
          nw0 = M.ring[rpos & (kRingDw - 1)];
          nw1 = M.ring[(rpos + 1) & (kRingDw - 1)];
          rhi = base + 32;
#pragma unroll
          for (int i = 0; i < kPf; i++) pf[i] = fetch_dword(in, 4 * (uint64_t)(rhi + kPf * j + i));
        }
      }
      if (mine) {
        mode = sm;
        res = (uint32_t)r;
        cur_b = sb;
        next_b = s_next;
        bc0 = s_c0;
        bn = s_n;
        btot = s_tot;
        breg = s_reg;
        tcap = s_tcap;
        cap = s_cap;
        olen = s_olen;
        fin = s_fin;
        left = s_left;
        fixed_ok = s_fixed;
        hdrpos = s_hdr;
        nst = s_nst;
        nv = 0;
      }
    }
    if (!__ballot(mode != kVGone)) break;

    // ---------------------------------------------------------- hot steps
    // The common case, branch-light: a stream decoding a Huffman block with
    // room for this pass's tokens decodes one literal or one match per step.
    // Anything else -- end of block, a corrupt or oversized symbol -- leaves
    // the state untouched and the stream to the full step below.
#ifdef RIO_TOK_NOHOT
    const bool hot0 = false;
#else
    const bool hot0 = mode == kVHuff && tcap - nst - nv >= kPass + 3;
#endif
    bool cold = !hot0;
    uint32_t hs = 0;  // hot steps taken: a pass decodes at most kPass symbols
    if (__ballot(hot0)) {
      for (int step = 0; step < kPass; step++) {
        if (!cold) {
          hs++;
          const uint32_t w = __builtin_amdgcn_alignbit(hi, lo, o);
          uint32_t e = M.lit[w & ((1u << kTokLitRoot) - 1)];
          if ((e & 15) == 0 && (e & kEnLenBit)) e = slow_walk<kTokLitRoot>(M.lfco, M.lent, w);
          const uint32_t L = e & 15, isl = (e >> 4) & 1, E = (e >> 5) & 7;
          const uint32_t len = (e >> 8) + 3 + __builtin_amdgcn_ubfe(w, L, E);
          uint32_t o1 = o + L + E;
          const bool a1 = o1 >= 32;
          const uint32_t lo1 = a1 ? hi : lo, hi1 = a1 ? nw0 : hi;
          o1 -= a1 ? 32u : 0u;
          const uint32_t w2 = __builtin_amdgcn_alignbit(hi1, lo1, o1);
          uint32_t dd = M.dst[w2 & ((1u << kTokDistRoot) - 1)];
          if (isl && (dd & 15) == 0 && (dd & kEnLenBit)) dd = slow_walk<kTokDistRoot>(M.dfco, M.dent, w2);
          const uint32_t L2 = dd & 15, E2 = (dd >> 7) & 15;
          const uint32_t dist = (((dd >> 5) & 3) << E2) + 1 + __builtin_amdgcn_ubfe(w2, L2, E2);
          uint32_t o2 = o1 + (isl ? L2 + E2 : 0u);
          const bool a2 = o2 >= 32;
          const uint32_t lo2 = a2 ? hi1 : lo1, hi2 = a2 ? (a1 ? nw1 : nw0) : hi1;
          o2 -= a2 ? 32u : 0u;
          const uint32_t hist = olen < 32768u ? olen : 32768u;
          const bool ok = L != 0 && (isl ? (E != kEobExtra && L2 != 0 && dist <= hist && len <= cap - olen)
                                         : olen < cap);
          M.tbuf[nv] = isl ? (0x80000000u | ((len - 3) << 16) | (dist - 1)) : ((e >> 8) | (1u << 24));
          if (ok) {
            lo = lo2;
            hi = hi2;
            o = o2;
            rpos += (a1 ? 1u : 0u) + (a2 ? 1u : 0u);
            nv++;
            olen += isl ? len : 1u;
          } else {
            cold = true;
          }
          nw0 = M.ring[rpos & (kRingDw - 1)];
          nw1 = M.ring[(rpos + 1) & (kRingDw - 1)];
        }
      }
    }

    // ---------------------------------------------------------- full steps
#ifdef RIO_FLSTAT
    if (l == 0) {
      atomicAdd(&d.ctl->pad[0], 1ull);
      if (__ballot(cold && mode <= kVStored)) atomicAdd(&d.ctl->pad[1], 1ull);
    }
#endif
#define RIO_ADV(c_)                                    \
  {                                                    \
    o += (c_);                                         \
    if (o >= 32) {                                     \
      lo = hi;                                         \
      hi = nw0;                                        \
      nw0 = nw1;                                       \
      rpos++;                                          \
      nw1 = M.ring[(rpos + 1) & (kRingDw - 1)];        \
      o -= 32;                                         \
    }                                                  \
  }
#define RIO_EMIT(t_)                                   \
  {                                                    \
    M.tbuf[nv] = (t_);                                 \
    nv++;                                              \
  }
    for (uint32_t step = 0; step < kPass && __ballot(cold && mode <= kVStored && step + hs < kPass); step++) {
      if (!cold || step + hs >= kPass) {
      } else if (mode == kVHuff) {
        if (tcap - nst - nv < 3) {
          res = (uint32_t)kTokYield;
          mode = kVFinish;
        } else {
          const uint32_t w = __builtin_amdgcn_alignbit(hi, lo, o);
          uint32_t e = M.lit[w & ((1u << kTokLitRoot) - 1)];
          if ((e & 15) == 0 && (e & kEnLenBit)) e = slow_walk<kTokLitRoot>(M.lfco, M.lent, w);
          const uint32_t L = e & 15, E = (e >> 5) & 7;
          if (L == 0) {
            res = kCodecCorrupt;
            mode = kVFinish;
          } else if (!(e & kEnLenBit)) {
            RIO_ADV(L);
            if (olen >= cap) {
              res = kCodecFull;
              mode = kVFinish;
            } else {
              RIO_EMIT((e >> 8) | (1u << 24));
              olen++;
            }
          } else if (E == kEobExtra) {
            RIO_ADV(L);
            if (fin) {
              res = (32 * (rpos - 2) + o > 8 * bn) ? (uint32_t)kCodecEof : (uint32_t)kTokDone;
              mode = kVFinish;
            } else {
              mode = kVHeader;
            }
          } else {  // length, then the distance code
            const uint32_t len = (e >> 8) + 3 + __builtin_amdgcn_ubfe(w, L, E);
            RIO_ADV(L + E);
            const uint32_t w2 = __builtin_amdgcn_alignbit(hi, lo, o);
            uint32_t dd = M.dst[w2 & ((1u << kTokDistRoot) - 1)];
            if ((dd & 15) == 0 && (dd & kEnLenBit)) dd = slow_walk<kTokDistRoot>(M.dfco, M.dent, w2);
            const uint32_t L2 = dd & 15, E2 = (dd >> 7) & 15;
            if (L2 == 0) {
              res = kCodecCorrupt;
              mode = kVFinish;
            } else {
              const uint32_t dist = (((dd >> 5) & 3) << E2) + 1 + __builtin_amdgcn_ubfe(w2, L2, E2);
              RIO_ADV(L2 + E2);
              const uint32_t hist = olen < 32768u ? olen : 32768u;
              if (dist > hist) {
                res = kCodecCorrupt;
                mode = kVFinish;
              } else if (len > cap - olen) {
                res = kCodecFull;
                mode = kVFinish;
              } else {
                RIO_EMIT(0x80000000u | ((len - 3) << 16) | (dist - 1));
                olen += len;
              }
            }
          }
        }
      } else if (mode == kVStored) {  // stored bytes become literal tokens, 3 at a time
        if (tcap - nst - nv < 3) {
          res = (uint32_t)kTokYield;
          mode = kVFinish;
        } else {
          const uint32_t k = left < 3 ? left : 3;
          const uint32_t v = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(hi, lo, o), 0, 8 * k);
          RIO_ADV(8 * k);
          RIO_EMIT(v | (k << 24));
          olen += k;
          left -= k;
          if (left == 0) {
            if (fin) {
              res = (32 * (rpos - 2) + o > 8 * bn) ? (uint32_t)kCodecEof : (uint32_t)kTokDone;
              mode = kVFinish;
            } else {
              mode = kVHeader;
            }
          }
        }
      }
    }
#undef RIO_ADV
#undef RIO_EMIT

    // ---------------------------------------------------------- input pass
    // (the ring takes the prefetched words first: the loads were issued a
    // pass ago, and no store issued since may sit in front of them in vmcnt)
    {
      if (mode <= kVStored) {
        if (rhi - rpos <= kRingDw - 16) {
          uint32_t *rw = &M.ring[(rhi + kPf * j) & (kRingDw - 1)];
          if (kPf == 4) {
            *reinterpret_cast<uint4 *>(rw) = make_uint4(pf[0], pf[1 % kPf], pf[2 % kPf], pf[3 % kPf]);
          } else if (kPf == 2) {
            *reinterpret_cast<uint2 *>(rw) = make_uint2(pf[0], pf[1 % kPf]);
          } else {
#pragma unroll
            for (int i = 0; i < kPf; i++) rw[i] = pf[i];
          }
          rhi += 16;
          CompIn in = make_in(span, d, nchunks, bc0, btot, bn, breg != 0);
#pragma unroll
          for (int i = 0; i < kPf; i++) pf[i] = fetch_dword(in, 4 * (uint64_t)(rhi + kPf * j + i));
        }
        if (32 * (rpos - 2) + o > 8 * bn + 1024) {  // runaway past the end of the input
          res = kCodecEof;
          mode = kVFinish;
        }
      }
#ifdef RIO_CHECKED
      if (nv && ((uint64_t)bc0 * kTokPerChunk + nst + nv > d.tok_cap || nst + nv > tcap || nv > kTbuf)) {
        if (j == 0)
          printf("k_flate_tok: token store out of range: block %llu c0 %u nst %u nv %u tcap %u tok_cap %llu\n",
                 (unsigned long long)cur_b, bc0, nst, nv, tcap, (unsigned long long)d.tok_cap);
        atomicOr(&d.ctl->out_overflow, 0x200ull);
        nv = 0;
        res = kCodecCorrupt;
        mode = kVFinish;
      }
#endif
      uint32_t *tk = d.tok + (uint64_t)bc0 * kTokPerChunk + nst;
      if (nv) RIO_TT(30, tk + nv - 1);
      for (uint32_t k = j; k < nv; k += kVG) tk[k] = M.tbuf[k];
      nst += nv;
      nv = 0;
      wave_lds_sync();
    }
  }
}

// this wave's global stores complete before its next loads of the same bytes
__device__ __forceinline__ void zmem_sync_dev() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ================================================================ k_flate_sync
// Huffman pass with the whole wave on ONE recordio block (used first; blocks it
// declines go to k_flate_tok). Within a DEFLATE block the compressed bits are
// cut into 64 segments of kSyncSeg bits, one per lane, and every lane decodes
// its segment from a guessed start -- the segment's first bit, which is almost
// never a symbol boundary. Huffman codes self-synchronise: a decode from a wrong
// start falls into step with the true symbol sequence within a few symbols, so
// the position where a lane leaves its segment (the first symbol boundary at or
// after the segment end) is, after a few symbols, the true one. Each lane then
// restarts from its predecessor's exit; when no start changes any more every
// lane is on the true chain (lane 0 starts at a known boundary, and lane i's
// start is lane i-1's exit). A prefix sum of the lanes' token / byte counts
// places each lane's tokens, and a last pass writes them (same token format as
// k_flate_tok, so the copy pass is unchanged). The first lane that decodes the
// end-of-block symbol ends the DEFLATE block; lanes after it were decoding the
// next block's bits and are discarded.
//
// Parallelism is 64 segments of one stream per wave (k_flate_tok: 8 streams per
// wave, each replicated on 8 lanes), with one table set per wave in LDS, so a
// few large recordio blocks (the writer's default MaxItems = 16384: ~5 MB
// blocks) fill the GPU as well as many small ones. Anything unusual -- no
// convergence within kSyncIters rounds, a token region too small, the stream's
// size beyond this kernel's 32-bit positions -- declines the block to
// k_flate_tok; corrupt or oversized streams go to k_inflate_exact as there.
constexpr uint32_t kSyncSeg = 1024;                       // bits per lane per round
constexpr uint32_t kSyncBits = 64 * kSyncSeg;             // bits per round and wave
constexpr int kSyncIters = 8;
#ifndef RIO_SYNC_LEAD
#define RIO_SYNC_LEAD 0
#endif
// bits of a segment's end the first decode of a round covers (0: the whole segment).
// Measured and not kept (round 6, profiles/r06_flate_sync_lead_ab.jsonl): the
// last 128 / 256 / 512 bits only -- serial C3@16k 35.8-36.4 against 37.8, C3
// 49.6-51.8 against 53.6: exits found from a short lead-in are wrong often
// enough that whole waves decode a third time.
constexpr uint32_t kSyncLead = RIO_SYNC_LEAD;
static_assert(kSyncLead < kSyncSeg, "a lead-in within the segment");
#ifndef RIO_SYNC_WAVES
#define RIO_SYNC_WAVES 12
#endif
constexpr int kSyncWaves = RIO_SYNC_WAVES;                 // per CU (launch sizing, one wave per block)
#ifndef RIO_SYNC_W
#define RIO_SYNC_W 4  // waves per block for spans whose blocks all fit at that width (1: never)
#endif
// The kernel is written for kW waves per block (segment g = 64 * wave + lane,
// cross-wave exchanges at barriers); only kW = 1 is instantiated: kW = 2 / 4
// for spans of fewer blocks than one-wave slots measured slower for C3 at
// MaxItems = 16384 (2,158 blocks; round 3): 51.3 ms at 2 waves, 58.1 at 4,
// against 50.0 at one -- only 1,536 two-wave blocks are resident at a time
// (registers), and the barriers cost more than the extra segments gain.

template <int kW>
constexpr uint32_t sync_win_dw() { return kW * kSyncBits / 32 + 32; }  // staged dwords (+ run-out margin)

// cross-wave exchange of a kW-wave block (parity-double-buffered where it is
// written every convergence iteration)
template <int kW>
struct SyncX {
  uint32_t eob[2][kW], ex63[2][kW], need[2][kW];
  uint32_t tsum[kW], osum[kW], bad[kW], fall[kW];
  uint32_t exk;
  uint32_t h_act, h_fin, h_res, h_decl, h_ntok, h_olen;  // the header wave's results
  unsigned long long h_bit;
};
template <>
struct SyncX<1> {};

template <int kW>
struct SyncLdsT {
  StreamLds T;  // the DEFLATE block's tables (ring / tbuf unused)
  WaveLds W;
  uint32_t win[sync_win_dw<kW>() + sync_win_dw<kW>() / 32 + 1];  // skewed: see sync_at
  SyncX<kW> x;
};

// 32 bits of the staged window at relative bit r
// Window dword d lives at d + d/32: the lanes' segments start 32 dwords
// apart, which unskewed would put all 32 lanes of a ds_read_b32 group on one
// LDS bank (a 32-way conflict); skewed, segment i starts on bank i.
__device__ __forceinline__ uint32_t sync_at(uint32_t d) { return d + (d >> 5); }
__device__ __forceinline__ uint32_t sync_bits(const uint32_t *win, uint32_t r) {
  const uint32_t d = r >> 5;
  return __builtin_amdgcn_alignbit(win[sync_at(d + 1)], win[sync_at(d)], r & 31);
}

enum : uint32_t { kSyEob = 1, kSyBad = 2, kSyHist = 4, kSyFull = 8 };
// Literals per token in this pass: one (3, as stored blocks' tokens, cut C3's
// tokens by 8 % without a measurable gain: 50.4 against 51.0 GiB/s, round 3).
constexpr uint32_t kSyncMerge = 1;

// Decode tokens from relative bit r while r < end (or to the end-of-block
// symbol). Counting mode skips an undecodable code by one bit (a lane off the
// true chain); writing mode stops there. Returns the exit position.
// Consecutive literals may share a token (kSyncMerge, up to 3 bytes as stored
// blocks' tokens): both modes group them alike, so the counts place the
// written tokens.
// Bits come through a per-lane 64-bit buffer (bits [r, r + nb) of the window),
// topped up to > 32 bits before the literal/length code (<= 15 + 5 bits) and
// before the distance code (<= 15 + 13): the next window dword is loaded one
// top-up ahead, so a symbol's dependent LDS reads are its table lookups only.
// Counting mode with a stage (sg != nullptr, round 3): the tokens also go to
// the lane's staging column (token i at sg[64 i], the first kSyncStageCap), and
// slack = min over matches of (bytes before it - its distance), so that after
// convergence the counted decode's tokens are copied into place instead of
// decoded a second time.
constexpr uint32_t kSyncStageCap = 256;
template <bool kWrite>
__device__ __forceinline__ uint32_t sync_decode(const StreamLds &T, const uint32_t *win, uint32_t r, uint32_t end,
                                                uint32_t lim, uint32_t &ntok, uint32_t &nout, uint32_t &flags,
                                                uint32_t *tk, uint32_t olen0, uint32_t cap, uint32_t *sg = nullptr,
                                                int32_t *slack = nullptr) {
  uint32_t lacc = 0, lcnt = 0;  // the literal run not yet written
  auto emit = [&](uint32_t tv) {
    if (kWrite) tk[ntok] = tv;
    else if (sg && ntok < kSyncStageCap) sg[64 * ntok] = tv;
  };
  auto flush = [&]() {
    if (lcnt) {
      emit(lacc | (lcnt << 24));
      ntok++;
      lacc = lcnt = 0;
    }
  };
  uint32_t dn = (r >> 5) + 2;  // the next window dword into the buffer
  uint64_t buf = (((uint64_t)win[sync_at(dn - 1)] << 32) | win[sync_at(dn - 2)]) >> (r & 31);
  uint32_t nb = 64 - (r & 31), nxt = win[sync_at(dn)];
  auto top_up = [&]() {
    const bool low = nb <= 32;
    buf |= low ? ((uint64_t)nxt << nb) : 0ull;
    dn += low ? 1u : 0u;
    nb += low ? 32u : 0u;
    nxt = win[sync_at(dn)];  // (the same dword again when nothing was taken)
  };
  auto take = [&](uint32_t k) {
    buf >>= k;
    nb -= k;
    r += k;
  };
  while (r < end && r < lim) {
    top_up();
    const uint32_t w = (uint32_t)buf;
    uint32_t e = T.lit[w & ((1u << kTokLitRoot) - 1)];
    if ((e & 15) == 0 && (e & kEnLenBit)) e = slow_walk<kTokLitRoot>(T.lfco, T.lent, w);
    const uint32_t L = e & 15, E = (e >> 5) & 7;
    if (L == 0) {
      flags |= kSyBad;
      if (kWrite) break;
      take(1);
      continue;
    }
    if (!(e & kEnLenBit)) {
      if (kWrite && olen0 + nout >= cap) {
        flags |= kSyFull;
        break;
      }
      if (lcnt == kSyncMerge) flush();
      lacc |= (e >> 8) << (8 * lcnt);
      lcnt++;
      take(L);
      nout++;
      continue;
    }
    flush();
    if (E == kEobExtra) {
      take(L);
      flags |= kSyEob;
      break;
    }
    const uint32_t len = (e >> 8) + 3 + __builtin_amdgcn_ubfe(w, L, E);
    take(L + E);
    top_up();
    const uint32_t w2 = (uint32_t)buf;
    uint32_t dd = T.dst[w2 & ((1u << kTokDistRoot) - 1)];
    if ((dd & 15) == 0 && (dd & kEnLenBit)) dd = slow_walk<kTokDistRoot>(T.dfco, T.dent, w2);
    const uint32_t L2 = dd & 15, E2 = (dd >> 7) & 15;
    if (L2 == 0) {
      flags |= kSyBad;
      if (kWrite) break;
      continue;
    }
    const uint32_t dist = (((dd >> 5) & 3) << E2) + 1 + __builtin_amdgcn_ubfe(w2, L2, E2);
    if (kWrite) {
      const uint32_t at = olen0 + nout, hist = at < 32768u ? at : 32768u;
      if (dist > hist) {
        flags |= kSyHist;
        break;
      }
      if (len > cap - at) {
        flags |= kSyFull;
        break;
      }
    } else if (sg) {
      const int32_t sl = (int32_t)nout - (int32_t)dist;
      *slack = sl < *slack ? sl : *slack;
    }
    emit(0x80000000u | ((len - 3) << 16) | (dist - 1));
    take(L2 + E2);
    ntok++;
    nout += len;
  }
  flush();
  return r;
}

// Counting decode, one code per step (round 4). sync_decode decodes a whole
// symbol per loop trip -- a literal, or a length code and its distance code --
// so in a wave whose lanes hold both kinds every trip runs the literal path and
// the match path one after the other under exec masks (~170 VALU + 66 SALU per
// trip). Here a trip decodes ONE Huffman code: `sd` says which table (0:
// literal/length, 1: distance), the entry's fields are picked by selects, and
// the token, counts and state follow without branches; a match takes two trips,
// a literal one. Same tokens, counts, staging and exit as sync_decode<false>
// (the writing decode and this one must agree on the true chain): an
// undecodable literal/length code skips one bit, an undecodable distance code
// none (the next trip reads a literal/length code there), a match started
// before `end` is finished past it, and end-of-block ends the segment.
template <bool kCount>
__device__ __forceinline__ uint32_t sync_count(const StreamLds &T, const uint32_t *win, uint32_t r, uint32_t end,
                                               uint32_t lim, uint32_t &ntok, uint32_t &nout, uint32_t &flags,
                                               uint32_t *sg, int32_t &slack) {
  uint32_t dn = (r >> 5) + 2;
  uint64_t buf = (((uint64_t)win[sync_at(dn - 1)] << 32) | win[sync_at(dn - 2)]) >> (r & 31);
  uint32_t nb = 64 - (r & 31), nxt = win[sync_at(dn)];
  uint32_t sd = 0, plen = 0, tn = ntok, on = nout, fl = flags;
  int32_t sl = slack;
  const uint32_t endl = end < lim ? end : lim;
  while ((sd | (uint32_t)(r < endl)) != 0) {
    const uint32_t low = nb <= 32 ? 1u : 0u;
    buf |= (uint64_t)(nxt & (0u - low)) << (nb & 63u);
    dn += low;
    nb += low << 5;
    nxt = win[sync_at(dn)];
    const uint32_t w = (uint32_t)buf;
    const uint32_t idx = w & (sd ? (1u << kTokDistRoot) - 1 : (1u << kTokLitRoot) - 1);
    const uint16_t *tab = sd ? T.dst : T.lit;
    uint32_t e = tab[idx];
    if ((e & 31) == kLongMark)
      e = sd ? slow_walk<kTokDistRoot>(T.dfco, T.dent, w) : slow_walk<kTokLitRoot>(T.lfco, T.lent, w);
    const uint32_t L = e & 15;
    // extra bits: literal/length (7:5; 7 = end-of-block), distance (10:7)
    const uint32_t E = __builtin_amdgcn_ubfe(e, sd ? 7u : 5u, sd ? 4u : 3u);
    const uint32_t lenbit = (e >> 4) & 1u & (sd ^ 1u);  // a length or end-of-block code
    const uint32_t ok = L != 0 ? 1u : 0u;
    const uint32_t eob = lenbit & (E == kEobExtra ? 1u : 0u) & ok;
    const uint32_t lit = (sd | lenbit | (ok ^ 1u)) ^ 1u;
    const uint32_t len = lenbit & (eob ^ 1u) & ok;
    const uint32_t dst = sd & ok;
    const uint32_t k = ok ? (eob ? L : L + E) : (sd ^ 1u);
    buf >>= k;
    nb -= k;
    r += k;
    fl |= ((ok ^ 1u) * (uint32_t)kSyBad) | (eob * (uint32_t)kSyEob);
    if (eob) break;
    // value: literal byte / length - 3 / distance
    const uint32_t base = sd ? (__builtin_amdgcn_ubfe(e, 5, 2) << E) + 1 : e >> 8;
    const uint32_t val = base + __builtin_amdgcn_ubfe(w, L, E);
    if constexpr (kCount) {
      const uint32_t em = lit | dst;
      const uint32_t tm = 0x80000000u | (plen << 16) | (val - 1), tl = val | (1u << 24);
      const uint32_t tv = tm ^ ((tm ^ tl) & (0u - lit));
      if (em && sg && tn < kSyncStageCap) sg[64 * tn] = tv;
      const int32_t s2 = (int32_t)on - (int32_t)val;
      sl = (dst && s2 < sl) ? s2 : sl;
      on += lit + dst * (plen + 3);
      tn += em;
    }
    plen = len ? val : plen;
    sd = len;
  }
  ntok = tn;
  nout = on;
  flags = fl;
  slack = sl;
  return r;
}


// kW waves per block: segment g = 64 * wave + lane. Wave 0 reads the DEFLATE
// block headers and builds the tables; the waves meet at barriers to exchange
// the first end-of-block segment, the exits at their edges, the convergence
// test, token / byte counts and flags (one wave: all within the wave, as before).
// wide_below: the span's block count decides the variant -- the one-wave
// kernel runs spans of >= wide_below blocks, the kSyncW-wave one the others.
template <int kW>
__global__ void __launch_bounds__(64 * kW) k_flate_sync(const uint8_t *__restrict__ span, DevBufs d,
                                                   const unsigned long long *nblocks, uint64_t nchunks,
                                                   uint64_t dec_cap, uint64_t wide_below) {
  constexpr uint32_t kWinDw = sync_win_dw<kW>();
  __shared__ SyncLdsT<kW> S;
  StreamLds &T = S.T;
  const int l = lane_id();
  const int wv = kW == 1 ? 0 : (int)(threadIdx.x >> 6);
  const uint32_t g = (uint32_t)(64 * wv + l);  // this lane's segment
  const bool lead = kW == 1 ? l == 0 : threadIdx.x == 0;
  const uint64_t nb = uni64(*nblocks);
  if ((kW == 1) != (nb >= wide_below)) return;  // the other variant's span
  // this wave's staging columns (kW == 1): lane l's token i at sgl[64 i]
  uint32_t *const sgl = (kW == 1 && d.fl_stage && blockIdx.x < d.fl_stage_waves)
                            ? d.fl_stage + (uint64_t)blockIdx.x * 64 * kSyncStageCap + l
                            : nullptr;
  auto bar = [&]() {
    if constexpr (kW == 1) wave_lds_sync();
    else __syncthreads();
  };
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    FlState *sp = &d.fl[b];
    const uint64_t c0 = uni64(d.blk_c0[b]);
    const unsigned long long meta = uni64(d.blk_meta[b]);
    const uint32_t cls = (uint32_t)(meta >> kMetaClsShift) & 0xffu;
    // incomplete blocks, and magics that are never untransformed (the header
    // block is idTransform, registry.go:31; others are errors): nothing decoded
    bool skip = !(meta & kMetaComplete) || (cls != kMagicPacked && cls != kMagicTrailer);
    const uint64_t doff = uni64(d.blk_dec_off[b]), cp = uni64(d.blk_out_len[b]);
    if (!skip && doff + cp > dec_cap) {  // the regions need a larger buffer (host retries)
      skip = true;
      if (lead) {
        atomicOr(&d.ctl->out_overflow, 0x40ull);
        atomicMax(&d.ctl->dec_need, (unsigned long long)(doff + cp));
      }
    }
    if (skip) {
      if (lead) {
        sp->mode = kFlSkip;
        sp->round = 0;
        d.blk_out_len[b] = 0;
      }
      continue;
    }
    const uint64_t n = uni64(d.blk_len[b]);
    const uint64_t total = meta & kMetaTotalMask;
    uint64_t tcap64 = total * (uint64_t)kTokPerChunk;
    if (d.tok_limit && d.tok_limit < tcap64) tcap64 = d.tok_limit < 64 ? 64 : d.tok_limit;
    const CompIn in = make_in(span, d, nchunks, c0, total, n, (meta & kMetaRegular) != 0);
    // outside this kernel's 32-bit bit positions: k_flate_tok
    bool decline = n >= (1ull << 28) || c0 >= (1ull << 32) || d.fl_tok_only;
    const uint32_t cap = cp > 0xfffff000ull ? 0xfffff000u : (uint32_t)cp;
    const uint32_t tcap = tcap64 > 0xffffff00ull ? 0xffffff00u : (uint32_t)tcap64;
    uint32_t *tok = d.tok + c0 * (uint64_t)kTokPerChunk;
    uint64_t bit = 0;
    uint32_t olen = 0, ntok = 0, res = 0;  // res: 0 ok, else a CodecErr for k_inflate_exact
    uint32_t ck_next = 1;                  // the next input chunk's checkpoint (split copy pass)
    bool fin = false, fixed = false;
    // checkpoints for k_flate_plan: (tokens, output) at the first DEFLATE block
    // header or body round in each input chunk
    auto checkpoint = [&]() {
      const uint64_t kc = (bit >> 3) / (uint64_t)kMaxPayload;
      for (; ck_next <= kc && ck_next < total; ck_next++)
        if (lead) d.fl_ck[c0 + ck_next] = (unsigned long long)ntok | ((unsigned long long)olen << 32);
    };
    while (!decline && !res && !fin) {
      checkpoint();
      // ---- DEFLATE block header (wave 0; wave-uniform). act: 0 a stored
      // block done (next header), 1 a Huffman body follows, 2 stop
      uint32_t act = 2;
      if (wv == 0) {
        TokDec t;
        t.in = in;
        t.T = &T;
        t.W = &S.W;
        t.seek(bit);
        if (t.nb < 32) t.refill();
        fin = t.take(1) != 0;
        const uint32_t type = t.take(2);
        if (type == 0) {  // stored: its bytes become literal tokens, 3 per token
          t.take(t.nb & 7);
          if (t.nb < 32) t.refill();
          const uint32_t len = t.take(16), nlen = t.take(16);
          const uint64_t at = t.bitpos() / 8;
          act = 0;
          if ((uint16_t)nlen != (uint16_t)~len) {
            res = kCodecCorrupt;
          } else if (at + len > n) {
            res = kCodecEof;
          } else if (len > cap - olen) {
            res = kCodecFull;
          } else {
            const uint32_t nt = (len + 2) / 3;
            if ((uint64_t)ntok + nt > tcap) {
              decline = true;
              act = 2;
            } else {
              for (uint32_t k = (uint32_t)l; k < nt; k += 64) {
                const uint32_t c = (len - 3 * k) < 3 ? len - 3 * k : 3u;
                uint32_t v = 0;
                for (uint32_t q = 0; q < c; q++) v |= in.byte(at + 3 * k + q) << (8 * q);
                tok[ntok + k] = v | (c << 24);
              }
              ntok += nt;
              olen += len;
              bit = 8 * (at + len);
            }
          }
        } else {
          if (type == 1) {
            if (!fixed) fixed_tables(T, S.W);
            fixed = true;
          } else if (type == 2) {
            if (read_dynamic(t)) res = kCodecCorrupt;
            fixed = false;
          } else {
            res = kCodecCorrupt;
          }
          if (!res && t.overrun()) res = kCodecEof;
          act = res ? 2u : 1u;
          if (!res) bit = t.bitpos();
        }
      }
      if constexpr (kW > 1) {  // the header wave's results (and its tables) to every wave
        if (lead) {
          S.x.h_act = act;
          S.x.h_fin = fin;
          S.x.h_res = res;
          S.x.h_decl = decline;
          S.x.h_ntok = ntok;
          S.x.h_olen = olen;
          S.x.h_bit = bit;
        }
        __syncthreads();
        act = S.x.h_act;
        fin = S.x.h_fin != 0;
        res = S.x.h_res;
        decline = S.x.h_decl != 0;
        ntok = S.x.h_ntok;
        olen = S.x.h_olen;
        bit = S.x.h_bit;
      }
      if (act == 0) continue;
      if (act == 2) break;
      // ---- the block body, kW * kSyncBits per round
      for (;;) {
        if (bit > 8 * n + 64) {  // ran past the input without an end-of-block
          res = kCodecEof;
          break;
        }
        checkpoint();
        const uint64_t w0 = bit >> 5;  // staged window: dwords [w0, w0 + kWinDw)
        bar();
        for (uint32_t k = (uint32_t)threadIdx.x; k < kWinDw; k += 64 * kW) S.win[sync_at(k)] = fetch_dword(in, 4 * (w0 + k));
        bar();
        const uint32_t r0 = (uint32_t)(bit - 32 * w0), lim = 32 * (kWinDw - 2);
        const uint32_t seg_end = r0 + kSyncSeg * (g + 1);
        uint32_t st = r0 + kSyncSeg * g, ex = 0, nt = 0, no = 0, fl = 0;
        int32_t slack = 0;
        bool need = true, conv = false, stg = false;  // stg: this lane's last decode was staged
        // cnt: this lane's last decode counted its tokens. The first decode of a
        // round (from the guessed starts) only finds each segment's exit: every
        // lane but lane 0 decodes again from its predecessor's exit anyway, so
        // it neither counts nor stages (lane 0 counts in the second iteration)
        bool cnt = false;
        uint32_t ke = 64 * kW - 1, eob_any = 0;  // the first segment that reached end-of-block
        for (int it = 0; it < kSyncIters; it++) {
          if (need && it == 0) {
            nt = no = fl = 0;
            stg = false;
            // only the exit is wanted, and a decode from a wrong start falls into
            // step within a few codes: the segment's last kSyncLead bits suffice
            // (a lane whose exit comes out wrong makes its successor decode again)
            const uint32_t st0 = kSyncLead ? seg_end - kSyncLead : st;
            ex = sync_count<false>(T, S.win, st0, seg_end, lim, nt, no, fl, nullptr, slack);
          } else if (need) {
            nt = no = fl = 0;
            slack = 0x7fffffff;
            cnt = true;
            // every counted decode is staged: staging only the ones that are usually
            // the last (segment 0's first, every later one) left a lane without a
            // staged decode in most rounds (41.0 against 35.4 ms for C3)
            stg = sgl != nullptr;
            ex = sync_count<true>(T, S.win, st, seg_end, lim, nt, no, fl, stg ? sgl : nullptr, slack);
          }
          // the true chain ends at the first segment reaching end-of-block
          const unsigned long long eobm = __ballot((fl & kSyEob) != 0);
          uint32_t prev = __shfl_up(ex, 1, 64);
          bool anyneed;
          if constexpr (kW == 1) {
            eob_any = eobm != 0;
            ke = eobm ? __ffsll((long long)eobm) - 1 : 63;
            const uint32_t nst = l == 0 ? r0 : prev;
            // segments after the end keep their start until the end moves
            need = g <= ke && (nst != st || !cnt);
            if (need) st = nst;
            anyneed = __ballot(need) != 0;
          } else {
            const int par = it & 1;
            if (l == 0) {
              S.x.eob[par][wv] = eobm ? (uint32_t)(64 * wv + __ffsll((long long)eobm) - 1) : 64u * kW;
              S.x.ex63[par][wv] = (uint32_t)__builtin_amdgcn_readlane(ex, 63);
            }
            __syncthreads();
            uint32_t fe = 64u * kW;
#pragma unroll
            for (int w = 0; w < kW; w++) fe = min(fe, S.x.eob[par][w]);
            eob_any = fe < 64u * kW;
            ke = eob_any ? fe : 64u * kW - 1;
            if (l == 0 && wv > 0) prev = S.x.ex63[par][wv - 1];
            const uint32_t nst = g == 0 ? r0 : prev;
            need = g <= ke && (nst != st || !cnt);
            if (need) st = nst;
            const bool wneed = __ballot(need) != 0;  // (the whole wave votes, lane 0 writes)
            if (l == 0) S.x.need[par][wv] = wneed;
            __syncthreads();
            anyneed = false;
#pragma unroll
            for (int w = 0; w < kW; w++) anyneed |= S.x.need[par][w] != 0;
          }
          if (!anyneed) {
            conv = true;
            break;
          }
        }
        if (!conv) {
          decline = true;
          break;
        }
        const bool live = g <= ke;
        const uint32_t tn = live ? nt : 0u, on = live ? no : 0u;
        const uint32_t ti = wave_incl_sum_dpp(tn), oi = wave_incl_sum_dpp(on);
        uint32_t tpre = 0, opre = 0, ttot, otot;
        bool bad = __ballot(live && (fl & kSyBad)) != 0;
        if constexpr (kW == 1) {
          ttot = (uint32_t)__builtin_amdgcn_readlane(ti, 63);
          otot = (uint32_t)__builtin_amdgcn_readlane(oi, 63);
        } else {
          if (l == 0) {
            S.x.tsum[wv] = (uint32_t)__builtin_amdgcn_readlane(ti, 63);
            S.x.osum[wv] = (uint32_t)__builtin_amdgcn_readlane(oi, 63);
            S.x.bad[wv] = bad;
          }
          __syncthreads();
          ttot = otot = 0;
#pragma unroll
          for (int w = 0; w < kW; w++) {
            if (w < wv) {
              tpre += S.x.tsum[w];
              opre += S.x.osum[w];
            }
            ttot += S.x.tsum[w];
            otot += S.x.osum[w];
            bad |= S.x.bad[w] != 0;
          }
        }
        if (bad) {  // an undecodable code on the true chain
          res = kCodecCorrupt;
          break;
        }
        if ((uint64_t)ntok + ttot > tcap) {
          decline = true;
          break;
        }
        uint32_t f2 = 0;
        // the counted decodes' staged tokens into place (every live segment within
        // the stage: the usual case), else a second decode that writes them
        const bool staged = sgl && !__ballot(live && (!stg || nt > kSyncStageCap));
        if (staged) {
          const uint32_t o0 = olen + opre + (oi - on);
          if (live && (int64_t)o0 + slack < 0) f2 |= kSyHist;  // a distance beyond the block's output
          if ((uint64_t)olen + otot > cap) f2 |= kSyFull;
          zmem_sync_dev();  // this wave's staging stores done before its loads of them
          const uint32_t mx = (uint32_t)__reduce_max_sync(~0ull, live ? nt : 0u);
          uint32_t *dst = tok + ntok + tpre + (ti - tn);
          for (uint32_t i = 0; i < mx; i++) {
            if (live && i < nt) dst[i] = __hip_atomic_load(sgl + 64 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        } else if (live) {
          uint32_t wt = 0, wo = 0;
          const uint32_t wx = sync_decode<true>(T, S.win, st, seg_end, lim, wt, wo, f2, tok + ntok + tpre + (ti - tn),
                                                olen + opre + (oi - on), cap);
#ifdef RIO_SYNC_DEBUG
          if (wt != nt || wo != no || wx != ex)
            printf("sync kW=%d b=%llu g=%u st=%u end=%u ke=%u: count nt=%u no=%u ex=%u fl=%u | write wt=%u wo=%u wx=%u f2=%u\n",
                   kW, (unsigned long long)b, g, st, seg_end, ke, nt, no, ex, fl, wt, wo, wx, f2);
#endif
        }
        uint32_t fall = (uint32_t)__reduce_or_sync(~0ull, f2);
        uint32_t exk;
        if constexpr (kW == 1) {
          exk = (uint32_t)__builtin_amdgcn_readlane(ex, ke);
        } else {
          if (l == 0) S.x.fall[wv] = fall;
          if (g == ke) S.x.exk = ex;
          __syncthreads();
#pragma unroll
          for (int w = 0; w < kW; w++) fall |= S.x.fall[w];
          exk = S.x.exk;
        }
        if (fall & kSyHist) {
          res = kCodecCorrupt;
          break;
        }
        if (fall & kSyFull) {
          res = kCodecFull;
          break;
        }
        ntok += ttot;
        olen += otot;
        bit = 32 * w0 + exk;
        if (eob_any) break;  // the DEFLATE block ended
      }
    }
    if (!decline && !res && bit > 8 * n) res = kCodecEof;  // the final block ran past the input
    if (lead) {
      sp->round = 0;
      sp->olen2 = 0;
      if (decline) {
        sp->mode = kFlHeader;  // k_flate_tok decodes it from the start
      } else if (res) {        // k_inflate_exact classifies it (Go's lazy byte pulls) or sizes it
        sp->bitpos = bit;
        sp->olen = olen;
        sp->pad = res;
        sp->ntok = 0;
        sp->mode = kFlError;
        d.blk_status[b] = kBlkCodec;
        d.blk_a[b] = kCodecPending;
        d.blk_b[b] = res;
        d.blk_out_len[b] = 0;
      } else {
        sp->mode = kFlDone;
        sp->ntok = ntok;
        sp->olen = olen;
        d.fl_ck[c0] = ck_next;  // checkpoints 1 .. ck_next - 1
      }
    }
    if constexpr (kW > 1) __syncthreads();  // (S.x and the tables are reused by the next block)
  }
}

// k mod d for k < 2^20, d >= 1 (float reciprocal, one correction step)
__device__ __forceinline__ uint32_t umod_small(uint32_t k, uint32_t d) {
  uint32_t q = (uint32_t)((float)k * __builtin_amdgcn_rcpf((float)d));
  int32_t r = (int32_t)(k - q * d);
  if (r < 0) r += (int32_t)d;
  if (r >= (int32_t)d) r -= (int32_t)d;
  return (uint32_t)r;
}

// ================================================================ k_flate_lz2
// Copy pass with the 32 KiB history in HBM: the block's own output region,
// which the wave has already written. LDS holds only a 4 KiB ring per wave
// (the batch being built plus the 2,544 bytes before it), so ~28 waves fit a
// CU where a 36 KiB window with the whole history (the round-1 pass) fits 4:
// the copy pass is latency-bound, and occupancy is what hides the latency.
//
// A batch is up to 256 tokens (4 per lane, token order k-major) whose output
// fits kL2Span bytes. Its bytes are produced in the ring:
//  - literals, and matches whose source lies wholly before the batch, at once:
//    sources within kL2Near bytes from the ring, older ones from HBM, the
//    four token slots' source dwords loaded together (one memory latency per
//    16 bytes of the longest copy, not one per token);
//  - matches whose source reaches into the batch, in rounds: a round copies
//    every such match whose source ends at or before R, the start of the first
//    match still pending (every byte before R is final), and the first pending
//    match itself (a source overlapping its own output -- dist < len, a run --
//    is copied by the whole wave with period dist).
// Then the batch's complete 16 B units go to HBM (coalesced and aligned:
// decode regions are 256-aligned).
//
// HBM sources are more than kL2Near >= kL2Span + 16 + 258 bytes back, so they
// were flushed two batches ago or earlier; the wave has since waited for the
// token loads it issued after those stores (the tokens of this batch), and a
// gfx9 wave's vector memory operations complete in issue order, so the stores
// are done. Sources are read with agent-scope loads (from L2, never a stale L1
// line).
// Registers for 5 waves per SIMD (96 VGPRs, 4 spilled; the compiler alone takes
// 125: 4 waves): C3 45.6 -> 47.7 GiB/s; 6 waves (80 VGPRs, 31 spilled) 34.3.
#ifndef RIO_LZ2_WPE
#define RIO_LZ2_WPE 5
#endif
#define RIO_LZ2_ATTR __attribute__((amdgpu_waves_per_eu(RIO_LZ2_WPE)))

// The copy pass over one token list (k_flate_lz2; k_flate_seg's segments):
// `ntok` tokens at tk, output from position olen (> 0: resumed) into out
// through a kRingB-byte ring, batches of at most kSpanB bytes. Returns the end
// position. Positions count symbol bytes: kSym = 1, the decoded bytes; kSym =
// 2, a split block's later segment as u16 symbols (k_flate_seg): every length
// and distance doubles, a literal byte b is the symbol (b, 0), and the
// segment's 32 KiB of unknown history are the symbols 256 + i (i = the
// position's offset in that window) -- synthesized in the ring here, written
// before `out` by the caller (syn_a: the segment's start modulo 16, see
// k_flate_seg). Every byte-level step is the same for both widths.
#ifdef RIO_FLSTAT
__device__ Ctl *st_ctl;
#endif
template <int kSym, uint32_t kRingB, uint32_t kSpanB>
__device__ __forceinline__ uint32_t lz2_run(uint8_t *ring, uint8_t *out, const uint32_t *tk, uint32_t ntok,
                                            uint32_t olen, uint32_t syn_a = 0) {
  constexpr uint32_t kMaskB = kRingB - 1, kNearB = kRingB - kSpanB - 16;
  static_assert(kNearB >= kSpanB + 16 + 2 * 258, "HBM sources must be flushed two batches back");
  const int l = lane_id();
  const uint32_t *gw = reinterpret_cast<const uint32_t *>(out);
  wave_lds_sync();
  if (olen > 0) {  // resumed: the history before olen, into the ring
    const uint32_t h0 = (olen > kNearB ? olen - kNearB : 0u) & ~15u;
    for (uint32_t x = h0 + 16 * (uint32_t)l; x < olen; x += 1024) {
      uint4 v;
      if (kSym == 1) {
        v = *reinterpret_cast<const uint4 *>(out + x);
      } else {  // the synthetic window: symbol at x = 256 + x/2 - syn_a
        const uint32_t s0 = 256u + (x >> 1) - syn_a;
        v = make_uint4(s0 | ((s0 + 1) << 16), (s0 + 2) | ((s0 + 3) << 16), (s0 + 4) | ((s0 + 5) << 16),
                       (s0 + 6) | ((s0 + 7) << 16));
      }
      *reinterpret_cast<uint4 *>(ring + (x & kMaskB)) = v;
    }
  }
  uint32_t pre[4];
#pragma unroll
  for (int k = 0; k < 4; k++) pre[k] = (64u * k + (uint32_t)l < ntok) ? tk[64 * k + l] : 0u;
  uint32_t cur = 0;
  while (cur < ntok) {
    uint32_t t[4], len[4], p[4];
#pragma unroll
    for (int k = 0; k < 4; k++) t[k] = pre[k];
    // output positions (relative to the batch) and the tokens this batch takes
    uint32_t carry = 0, take = 0, emax = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const bool valid = cur + 64u * k + (uint32_t)l < ntok;
      len[k] = valid ? kSym * tok_len(t[k]) : 0u;
      const uint32_t incl = wave_incl_sum_dpp(len[k]) + carry;
      p[k] = incl - len[k];
      const bool ok = valid && incl <= kSpanB;  // a prefix of the tokens (positions only grow)
      take += (uint32_t)__popcll(__ballot(ok));
      if (ok) emax = incl;
      else len[k] = 0;
      carry = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
    }
    const uint32_t total = (uint32_t)__reduce_max_sync(~0ull, emax);
    const uint32_t B0 = olen;
#ifdef RIO_FLSTAT  // (statistics builds: batches, tokens, rounds, pending tokens -> ctl->zprof)
    uint32_t st_rounds = 0;
#endif
    {  // zero the batch's ring bytes (their dwords; the history bytes of the first one stay)
      uint32_t *rw = reinterpret_cast<uint32_t *>(ring);
      const uint32_t z0 = (B0 + 3) >> 2, z1 = (B0 + total + 3) >> 2;
      for (uint32_t z = z0 + (uint32_t)l; z < z1; z += 64) rw[z & (kMaskB >> 2)] = 0u;
      if ((B0 & 3) && l == 0) atomicAnd(&rw[(B0 >> 2) & (kMaskB >> 2)], (1u << (8 * (B0 & 3))) - 1);
      wave_lds_sync();
    }
    const uint32_t near = B0 > kNearB ? B0 - kNearB : 0u;  // positions >= near: in the ring
    // literals now; matches sourced before the batch now; the others pending
    bool pend[4];
    uint32_t cs[4], cn[4], glob = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      pend[k] = false;
      cn[k] = 0;
      const uint32_t n = len[k];
      const uint32_t x = B0 + p[k];
      cs[k] = x - kSym * ((t[k] & 0xffffu) + 1);
      if (n == 0) continue;
      if (!(t[k] >> 31)) {  // 1-3 literal bytes
        uint32_t *rw = reinterpret_cast<uint32_t *>(ring);
        const uint32_t v = t[k] & 0xffffffu, o = 8 * (x & 3);
        if (kSym == 1) {
          atomicOr(&rw[(x >> 2) & (kMaskB >> 2)], v << o);
          if ((x & 3) + n > 4) atomicOr(&rw[((x >> 2) + 1) & (kMaskB >> 2)], v >> (32 - o));
        } else {  // bytes b0 0 b1 0 b2 0 at an even x
          const uint64_t w = ((uint64_t)((v & 0xffu) | ((v & 0xff00u) << 8)) | ((uint64_t)(v >> 16) << 32)) << o;
          atomicOr(&rw[(x >> 2) & (kMaskB >> 2)], (uint32_t)w);
          if ((x & 3) + n > 4) atomicOr(&rw[((x >> 2) + 1) & (kMaskB >> 2)], (uint32_t)(w >> 32));
        }
      } else if (cs[k] < near) {
        cn[k] = n;
        glob |= 1u << k;
      } else if (cs[k] + n <= B0) {
        cn[k] = n;
      } else {
        pend[k] = true;
      }
    }
#ifdef RIO_FLSTAT
    {
      uint32_t np = 0, ng = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        np += (uint32_t)__popcll(__ballot(pend[k]));
        ng += (uint32_t)__popcll(__ballot((glob >> k) & 1));
      }
      if (l == 0) {
        atomicAdd(&st_ctl->zprof[0], 1ull);
        atomicAdd(&st_ctl->zprof[1], (unsigned long long)take);
        atomicAdd(&st_ctl->zprof[2], (unsigned long long)np);
        atomicAdd(&st_ctl->zprof[3], (unsigned long long)ng);
      }
    }
#endif
    // the next batch's tokens (issued before this batch's stores: see above)
    const uint32_t nx = cur + take;
#pragma unroll
    for (int k = 0; k < 4; k++) pre[k] = (nx + 64u * k + (uint32_t)l < ntok) ? tk[nx + 64 * k + l] : 0u;
    // the copies above (every slot, ring or HBM sources), then the matches
    // sourced inside the batch in rounds: each round copies only from the ring,
    // slot by slot, and only the slots some lane copies in it (a batch has ~6
    // rounds for ~14 pending tokens: full four-slot copies there were most of
    // the pass's instructions)
    l2_copy4<kMaskB>(ring, gw, cs, B0, p, cn, glob);
    for (;;) {
#ifdef RIO_FLSTAT
      st_rounds++;
#endif
      wave_lds_sync();
      int kf = -1, lf = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const unsigned long long m = __ballot(pend[k]);
        if (kf < 0 && m) {
          kf = k;
          lf = __ffsll((long long)m) - 1;
        }
      }
      if (kf < 0) break;
      // R: the first pending match; every byte before it is final
      const uint32_t R = (uint32_t)__builtin_amdgcn_readlane(pick4(p, kf), lf);
      const uint32_t Df = kSym * (((uint32_t)__builtin_amdgcn_readlane(pick4(t, kf), lf) & 0xffffu) + 1);
      const uint32_t Nf = (uint32_t)__builtin_amdgcn_readlane(pick4(len, kf), lf);
      const bool run = Df < Nf;  // it overlaps its own output: the whole wave copies it
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint32_t n = 0;
        if (pend[k]) {
          const bool first = k == kf && l == lf;
          if (first || cs[k] + len[k] <= B0 + R) {  // source ends at or before R
            if (!first || !run) n = len[k];
            pend[k] = false;
          }
        }
        if (__ballot(n != 0)) l2_copy1_ring<kMaskB>(ring, cs[k], B0 + p[k], n);
      }
      if (run) {  // byte k of the run = byte (k mod dist) of the dist bytes before it (final)
        const uint32_t xs = B0 + R - Df, xd = B0 + R;
        for (uint32_t k0 = 0; k0 < Nf; k0 += 64) {
          const uint32_t k = k0 + (uint32_t)l;
          if (k < Nf) {
            const uint32_t v = ring[(xs + umod_small(k, Df)) & kMaskB];
            atomicOr(reinterpret_cast<uint32_t *>(ring) + (((xd + k) >> 2) & (kMaskB >> 2)), v << (8 * ((xd + k) & 3)));
          }
        }
      }
    }
#ifdef RIO_FLSTAT
    if (l == 0) atomicAdd(&st_ctl->flstat_esc, (unsigned long long)st_rounds);
#endif
    // complete 16 B units of the batch to HBM
    const uint32_t e = B0 + total;
    // (cached stores: the pass reads its far sources back from these bytes; non-temporal
    // ones measured slower, C3 53.3 -> 51.6 GiB/s, profiles/r05_flate_nt_flush_ab.jsonl)
    for (uint32_t x = (B0 & ~15u) + 16 * (uint32_t)l; x + 16 <= e; x += 1024)
      *reinterpret_cast<uint4 *>(out + x) = *reinterpret_cast<const uint4 *>(ring + (x & kMaskB));
    olen = e;
    cur += take;
  }
  // the last partial unit (decode regions and segment scratch are 256-aligned and sized in 256 B steps)
  if ((olen & 15) && l == 0) {
    const uint32_t x = olen & ~15u;
    *reinterpret_cast<uint4 *>(out + x) = *reinterpret_cast<const uint4 *>(ring + (x & kMaskB));
  }
  return olen;
}

__global__ void __launch_bounds__(64) RIO_LZ2_ATTR k_flate_lz2(DevBufs d, const unsigned long long *nblocks, int round) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[kL2Ring];
  const int l = lane_id();
  if (round > 0 && uni64(d.fl_more[round - 1]) == 0) return;
  const uint64_t nb = uni64(*nblocks);
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    FlState *sp = &d.fl[b];
    const uint32_t mode = uni(sp->mode);
    if (uni(sp->round) != (uint32_t)round || mode == kFlError || mode == kFlSkip || mode == kFlSplit) continue;
    uint8_t *out = d.dec + uni64(d.blk_dec_off[b]);
    const uint32_t *tk = d.tok + uni64(d.blk_c0[b]) * (uint64_t)kTokPerChunk;
    const uint32_t olen = lz2_run<1, kL2Ring, kL2Span>(ring, out, tk, uni(sp->ntok), (uint32_t)uni64(sp->olen2));
    if (l == 0) {
      sp->olen2 = olen;
      if (mode == kFlDone) d.blk_out_len[b] = olen;
    }
  }
}

// ================================================================ split copy pass
// A recordio block at the writer's default MaxItems (16,384 records: ~5 MB
// decoded) is one copy-pass wave, so a span of such blocks keeps far fewer
// waves in flight than the pass needs to hide its latency (C3 at MaxItems =
// 16384: 2,158 waves for 5,120 slots). When a span has fewer blocks than
// copy-pass slots, k_flate_plan cuts each block's token list at the Huffman
// pass's checkpoints (the (token, output) position at each input chunk) into
// up to kSegMax segments of >= kSegMin bytes. Segment 0 is copied as usual;
// every later segment is copied at the same time without its history, as u16
// symbols (lz2_run<2>): a byte whose value comes, through any chain of
// matches, from the 32 KiB before the segment is the symbol 256 + its
// position in that window. k_flate_segfix then resolves each block's segments
// in order -- the window is final once the segment before it is -- by one
// lookup per byte. Blocks the scratch cannot hold are copied whole as before.
constexpr uint32_t kSegRing = 8192, kSegSpan = 3072;
#ifndef RIO_SEG_W10
#define RIO_SEG_W10 18  // measured: a u16 segment costs ~1.8x a byte segment per output byte
#endif
constexpr uint32_t kSegW10 = RIO_SEG_W10;
constexpr uint64_t kSegWin = 65536;  // the synthetic window's symbol bytes before a later segment's output

__device__ __forceinline__ uint64_t seg_scratch_bytes(uint32_t o0, uint32_t o1) {
  // window + the segment's symbols from its 16-aligned start to its 16-rounded end (+ slack unit), 256-aligned
  return (kSegWin + 2ull * ((((uint64_t)o1 + 15) & ~15ull) - (o0 & ~15u)) + 32 + 255) & ~255ull;
}

// per block (thread): the split points and each later segment's scratch
__global__ void k_flate_plan(DevBufs d, const unsigned long long *nblocks) {
  const uint64_t nb = *nblocks;
  if (nb == 0) return;
  // as many segments per block as every one gets a copy-pass slot of its own:
  // the pass takes as long as its longest wave, so a second segment on a wave
  // costs more than the split gains
  uint64_t want = d.seg_items / nb;
  if (want > (uint64_t)kSegMax) want = kSegMax;
  if (want < 2) return;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    FlState *sp = &d.fl[b];
    if (sp->mode != kFlDone || sp->round != 0) continue;
    const uint32_t olen = (uint32_t)sp->olen, ntok = sp->ntok;
    uint32_t S = (uint32_t)want;
    if (S > olen / kSegMin) S = olen / kSegMin;
    if (S < 2) continue;
    const uint64_t c0 = d.blk_c0[b];
    const uint32_t K = (uint32_t)d.fl_ck[c0];  // checkpoints 1 .. K-1
    uint32_t tb[kSegMax + 1], ob[kSegMax + 1], n = 1;
    tb[0] = ob[0] = 0;
    uint32_t k = 1;
    for (uint32_t j = 1; j < S; j++) {
      // cut for equal cost: a later segment's byte costs kSegW10 / 10 of segment 0's
      const uint32_t target =
          (uint32_t)((uint64_t)olen * (kSegW10 + 10 * (j - 1)) / (kSegW10 + 10 * (S - 1)));
      unsigned long long e = 0;
      while (k < K) {
        e = d.fl_ck[c0 + k];
        if ((uint32_t)(e >> 32) >= target) break;
        k++;
      }
      if (k >= K) break;
      const uint32_t t = (uint32_t)e, o = (uint32_t)(e >> 32);
      k++;
      if (o - ob[n - 1] >= kSegMin / 2 && olen - o >= kSegMin / 2 && t > tb[n - 1] && t < ntok) {
        tb[n] = t;
        ob[n] = o;
        n++;
      }
    }
    if (n < 2) continue;
    tb[n] = ntok;
    ob[n] = olen;
    uint64_t need = 0;
    for (uint32_t j = 1; j < n; j++) need += seg_scratch_bytes(ob[j], ob[j + 1]);
    const uint64_t off = atomicAdd(&d.ctl->seg_used, (unsigned long long)need);
    if (!d.seg_scr || off + need > d.seg_cap) continue;  // copied whole (the host grows the scratch for next time)
    unsigned long long *e = d.fl_seg + 2 * b * (uint64_t)kSegMax;
    uint64_t so = off;
    for (uint32_t j = 0; j < n; j++) {
      e[2 * j] = (unsigned long long)tb[j] | ((unsigned long long)ob[j] << 32);
      e[2 * j + 1] = j ? so : 0ull;
      if (j) so += seg_scratch_bytes(ob[j], ob[j + 1]);
    }
    sp->stored_left = n;
    sp->mode = kFlSplit;
    atomicAdd(&d.ctl->seg_blocks, 1ull);
  }
}

// segment j of a split block (read by k_flate_seg / k_flate_segfix)
struct SegRef {
  uint32_t t0, t1, o0, o1;
  uint64_t scr;
};
__device__ __forceinline__ SegRef seg_ref(const DevBufs &d, uint64_t b, uint32_t j, uint32_t S, const FlState *sp) {
  const unsigned long long *e = d.fl_seg + 2 * (b * (uint64_t)kSegMax + j);
  SegRef r;
  const uint64_t e0 = uni64(e[0]);
  r.t0 = (uint32_t)e0;
  r.o0 = (uint32_t)(e0 >> 32);
  r.scr = uni64(e[1]);
  if (j + 1 < S) {
    const uint64_t e1 = uni64(e[2]);
    r.t1 = (uint32_t)e1;
    r.o1 = (uint32_t)(e1 >> 32);
  } else {
    r.t1 = uni(sp->ntok);
    r.o1 = (uint32_t)uni64(sp->olen);
  }
  return r;
}

__global__ void __launch_bounds__(64) RIO_LZ2_ATTR k_flate_seg(DevBufs d, const unsigned long long *nblocks) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[kSegRing];
  const int l = lane_id();
  const uint64_t nb = uni64(*nblocks);
  for (uint64_t i = blockIdx.x; i < nb * kSegMax; i += gridDim.x) {
    const uint64_t b = i % nb;
    const uint32_t j = (uint32_t)(i / nb);  // every block's segment 0 first, then segment 1, ...
    const FlState *sp = &d.fl[b];
    if (uni(sp->mode) != kFlSplit) continue;
    const uint32_t S = uni(sp->stored_left);
    if (j >= S) continue;
    const SegRef r = seg_ref(d, b, j, S, sp);
    const uint32_t *tk = d.tok + uni64(d.blk_c0[b]) * (uint64_t)kTokPerChunk + r.t0;
    if (j == 0) {
      lz2_run<1, kSegRing, kSegSpan>(ring, d.dec + uni64(d.blk_dec_off[b]), tk, r.t1, 0);
      continue;
    }
    // position p of the segment is symbol byte x = kSegWin + 2 (p - (o0 & ~15)):
    // 16-aligned positions at 32-aligned symbol bytes. The window before it
    // holds the symbols 256 + i for positions o0 - 32768 + i.
    uint8_t *out = d.seg_scr + r.scr;
    const uint32_t a = r.o0 & 15u;
    const uint32_t x0 = (uint32_t)kSegWin + 2 * a;
    for (uint32_t x = 16 * (uint32_t)l; x < x0; x += 1024) {
      const uint32_t s0 = 256u + (x >> 1) - a;  // (below 2a: never read)
      *reinterpret_cast<uint4 *>(out + x) = make_uint4(s0 | ((s0 + 1) << 16), (s0 + 2) | ((s0 + 3) << 16),
                                                       (s0 + 4) | ((s0 + 5) << 16), (s0 + 6) | ((s0 + 7) << 16));
    }
    zmem_sync_dev();  // the window's stores complete before the copies read it back (agent-scope loads)
    lz2_run<2, kSegRing, kSegSpan>(ring, out, tk, r.t1 - r.t0, x0, a);
  }
}

// Resolve a split block's later segments in order (workgroup per block): the
// final 32 KiB before segment j into LDS, then each 16 B output unit from its
// 16 symbols (< 256: the byte; else the window's byte).
constexpr int kSegFixThreads = 256;
__global__ void __launch_bounds__(kSegFixThreads) k_flate_segfix(DevBufs d, const unsigned long long *nblocks) {
  __shared__ uint32_t win[8192 + 4];
  const uint64_t nb = *nblocks;
  const int tid = (int)threadIdx.x;
  const uint8_t *wb = reinterpret_cast<const uint8_t *>(win);
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    FlState *sp = &d.fl[b];
    if (sp->mode != kFlSplit) continue;  // (the same for every thread of the workgroup)
    const uint32_t S = sp->stored_left;
    uint8_t *dec = d.dec + d.blk_dec_off[b];
    for (uint32_t j = 1; j < S; j++) {
      const unsigned long long *e = d.fl_seg + 2 * (b * (uint64_t)kSegMax + j);
      const uint32_t o0 = (uint32_t)(e[0] >> 32);
      const uint32_t o1 = j + 1 < S ? (uint32_t)(e[2] >> 32) : (uint32_t)sp->olen;
      const uint8_t *scr = d.seg_scr + e[1] + kSegWin;
      const uint32_t w0 = o0 - 32768u, sh = w0 & 3u;  // (o0 >= kSegMin / 2)
      const uint32_t *src = reinterpret_cast<const uint32_t *>(dec + (w0 - sh));
      __syncthreads();  // the previous segment's window reads are done
      for (int k = tid; k < 8193; k += kSegFixThreads)
        win[k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const uint32_t U0 = o0 & ~15u, nu = (o1 - U0 + 15) >> 4;
      for (uint32_t u = (uint32_t)tid; u < nu; u += kSegFixThreads) {
        const uint32_t U = U0 + 16 * u;
        const uint4 s0 = *reinterpret_cast<const uint4 *>(scr + 32 * (size_t)u);
        const uint4 s1 = *reinterpret_cast<const uint4 *>(scr + 32 * (size_t)u + 16);
        const uint32_t sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        uint32_t ov[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          uint32_t w = 0;
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const uint32_t pair = sv[2 * q + h];
#pragma unroll
            for (int m = 0; m < 2; m++) {
              const uint32_t v = (pair >> (16 * m)) & 0xffffu;
              const uint32_t byte = v < 256u ? v : (uint32_t)wb[sh + (v - 256u)];
              w |= byte << (8 * (2 * h + m));
            }
          }
          ov[q] = w;
        }
        uint4 *dp = reinterpret_cast<uint4 *>(dec + U);
        if (U < o0 || U + 16 > o1) {  // bytes of the neighbouring segments stay
          const uint32_t *cw = reinterpret_cast<const uint32_t *>(dp);
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const uint32_t cur = __hip_atomic_load(cw + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint32_t keep = 0;
#pragma unroll
            for (int m = 0; m < 4; m++) {
              const uint32_t p = U + 4 * q + m;
              if (p < o0 || p >= o1) keep |= 0xffu << (8 * m);
            }
            ov[q] = (ov[q] & ~keep) | (cur & keep);
          }
        }
        *dp = make_uint4(ov[0], ov[1], ov[2], ov[3]);
      }
      __threadfence();  // this segment's bytes visible before the next window is read
    }
    __syncthreads();
    if (tid == 0) {
      const uint32_t olen = (uint32_t)sp->olen;
      sp->olen2 = olen;
      d.blk_out_len[b] = olen;
      sp->mode = kFlDone;
    }
  }
}

// The blocks the fast path failed on: the exact restatement gives the
// reference's error (and CorruptInputError offset). One wave per failing block, lane 0.
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

uint64_t flate_seg_items(int ncu) { return (uint64_t)(ncu > 0 ? ncu : 256) * kL2Waves; }
uint64_t flate_stage_waves(int ncu) { return (uint64_t)(ncu > 0 ? ncu : 256) * kSyncWaves; }
uint64_t flate_stage_words(int ncu) { return flate_stage_waves(ncu) * 64 * kSyncStageCap; }

static unsigned grid256(uint64_t n) {
  uint64_t g = (n + 255) / 256;
  if (g > 1024) g = 1024;
  return (unsigned)(g ? g : 1);
}

void launch_inflate_plan(const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks, hipStream_t st);

// The flate decode in two phases, so that the host can size the split copy
// pass's scratch between them (pipeline.cpp: a context's first split plan).
// Phase 1: the Huffman pass (k_flate_sync) and the split plan.
void launch_inflate_huff(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks,
                         uint64_t max_blocks, uint64_t nchunks, uint64_t dec_cap, int rounds, int ncu, hipStream_t st) {
  (void)hipMemsetAsync(d.fl_more, 0, sizeof(unsigned long long) * rounds, st);
  {  // the wave-per-block Huffman pass first; k_flate_tok takes what it declines
    const uint64_t rs = (uint64_t)ncu * kSyncWaves;
    const uint64_t gs = max_blocks < rs ? max_blocks : rs;
#if RIO_SYNC_W > 1
    // a span of few blocks (every block resident with kSyncW waves each, e.g. a
    // scanner's 512 MiB span at MaxItems = 16384: ~250 blocks) runs the
    // kSyncW-wave variant; the device-side block count picks (each returns
    // at once on the other's spans)
    // (workgroups per CU: a function-local static, initialised once and thread-safe)
    static const int wide_per_cu = [] {
      int per_cu = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_flate_sync<RIO_SYNC_W>, 64 * RIO_SYNC_W, 0) !=
              hipSuccess ||
          per_cu < 1)
        per_cu = 1;
      return per_cu;
    }();
    // (RIO_CFG_FLATE_ONE_WAVE: 0, the one-wave kernel on every span)
    const uint64_t wide_below = d.fl_one_wave ? 0 : (uint64_t)wide_per_cu * (uint64_t)(ncu > 0 ? ncu : 256) + 1;
    {
      const uint64_t gw = wide_below == 0 ? 1 : (max_blocks < wide_below - 1 ? max_blocks : wide_below - 1);
      hipLaunchKernelGGL(k_flate_sync<RIO_SYNC_W>, dim3((unsigned)(gw ? gw : 1)), dim3(64 * RIO_SYNC_W), 0, st, span,
                         d, nblocks, nchunks, dec_cap, wide_below);
    }
    hipLaunchKernelGGL(k_flate_sync<1>, dim3((unsigned)(gs ? gs : 1)), dim3(64), 0, st, span, d, nblocks, nchunks,
                       dec_cap, wide_below);
#else
    hipLaunchKernelGGL(k_flate_sync<1>, dim3((unsigned)(gs ? gs : 1)), dim3(64), 0, st, span, d, nblocks, nchunks,
                       dec_cap, 0);
#endif
  }
#ifdef RIO_FLSTAT
  {
    Ctl *p = d.ctl;
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(st_ctl), &p, sizeof(p), 0, hipMemcpyHostToDevice, st);
  }
#endif
  launch_inflate_plan(d, nblocks, max_blocks, st);
}

// few blocks: the copy pass split into segments (k_flate_plan marks the blocks;
// the copy rounds skip them). Relaunched by the host after it sized the scratch
// (with ctl->seg_used / seg_blocks reset): blocks it marks are planned once.
void launch_inflate_plan(const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks, hipStream_t st) {
  if (d.seg_items > 0)
    hipLaunchKernelGGL(k_flate_plan, dim3(grid256(max_blocks)), dim3(256), 0, st, d, nblocks);
}

// Phase 2: the fallback Huffman pass and copy rounds, the split copy pass, and
// the exact pass for failing blocks.
void launch_inflate_copy(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks,
                         uint64_t max_blocks, uint64_t nchunks, uint64_t dec_cap, int rounds, int ncu, hipStream_t st) {
  uint64_t g1 = (max_blocks + kVS - 1) / kVS;
  // resident waves of 8 streams per CU: LDS-bound
  const uint64_t r1 = (uint64_t)ncu * (163840 / (sizeof(StreamLds) * kVS + sizeof(WaveLds)));
  if (g1 > r1) g1 = r1;
  if (d.fl_grid && g1 > d.fl_grid) g1 = d.fl_grid;
  if (g1 < 1) g1 = 1;
  uint64_t g3 = max_blocks;
  if (g3 > (uint64_t)ncu * kL2Waves) g3 = (uint64_t)ncu * kL2Waves;
  if (g3 < 1) g3 = 1;
  const bool split = d.seg_items > 0;
#ifdef RIO_TOK_TRACE
  static unsigned long long *h_trace = nullptr;
  const size_t trace_words = (size_t)g1 * 64 * 34;
  if (!h_trace) {
    (void)hipHostMalloc((void **)&h_trace, (size_t)(r1 > g1 ? r1 : g1) * 64 * 34 * 8, hipHostMallocCoherent);
    if (h_trace) memset(h_trace, 0, (size_t)(r1 > g1 ? r1 : g1) * 64 * 34 * 8);
  }
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_tok_trace), &h_trace, sizeof(h_trace), 0, hipMemcpyHostToDevice, st);
#endif
  for (int r = 0; r < rounds; r++) {
    hipLaunchKernelGGL(k_flate_tok, dim3((unsigned)g1), dim3(64), 0, st, span, d, nblocks, nchunks,
                       dec_cap, r, (int)(r == rounds - 1));
#ifdef RIO_TOK_TRACE
    if (hipStreamSynchronize(st) != hipSuccess && h_trace) {
      fprintf(stderr, "RIO_TOK_TRACE: k_flate_tok round %d failed; span %p..+%llu tok %p..+%llu fl %p ck_pay %p\n", r,
              (const void *)span, (unsigned long long)(nchunks * kChunk), (void *)d.tok,
              (unsigned long long)(d.tok_cap * 4), (void *)d.fl, (void *)d.ck_pay);
      for (size_t w = 0; w < trace_words / (64 * 34); w++)
        for (int ln = 0; ln < 64; ln++) {
          const unsigned long long *t = h_trace + (w * 64 + ln) * 34;
          const unsigned long long n = t[33];
          if (n <= 1) continue;
          fprintf(stderr, "wave %zu lane %d: %llu accesses; last:", w, ln, n);
          for (unsigned long long q = n > 6 ? n - 6 : 1; q <= n; q++) {
            const unsigned long long *e = t + 2 * (q & 15);
            fprintf(stderr, " [%llu site %llu %p]", e[0] & 0xffffffffffffull, e[0] >> 48, (void *)e[1]);
          }
          fprintf(stderr, "\n");
        }
      fflush(stderr);
    }
#endif
    hipLaunchKernelGGL(k_flate_lz2, dim3((unsigned)g3), dim3(64), 0, st, d, nblocks, r);
  }
#ifdef RIO_TOK_TRACE
  {
    unsigned long long *z = nullptr;
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_tok_trace), &z, sizeof(z), 0, hipMemcpyHostToDevice, st);
  }
#endif
  if (split) {
    uint64_t gs = max_blocks * kSegMax;
    if (gs > (uint64_t)ncu * kL2Waves) gs = (uint64_t)ncu * kL2Waves;
    hipLaunchKernelGGL(k_flate_seg, dim3((unsigned)(gs ? gs : 1)), dim3(64), 0, st, d, nblocks);
    uint64_t gf = max_blocks;
    if (gf > (uint64_t)ncu * 4) gf = (uint64_t)ncu * 4;
    hipLaunchKernelGGL(k_flate_segfix, dim3((unsigned)(gf ? gf : 1)), dim3(kSegFixThreads), 0, st, d, nblocks);
  }
  uint64_t ge = (max_blocks + 63) / 64;
  if (ge > 1024) ge = 1024;
  if (ge < 1) ge = 1;
  hipLaunchKernelGGL(k_inflate_exact, dim3((unsigned)ge), dim3(64), 0, st, span, d, nblocks);
}

void launch_inflate(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks,
                    uint64_t nchunks, uint64_t dec_cap, int rounds, int ncu, hipStream_t st) {
  launch_inflate_huff(span, d, nblocks, max_blocks, nchunks, dec_cap, rounds, ncu, st);
  launch_inflate_copy(span, d, nblocks, max_blocks, nchunks, dec_cap, rounds, ncu, st);
}

}  // namespace rio
