// Device helpers shared by the scan kernels and the codec kernels: wave-level
// scans, the block payload accessor and the uvarint header parser of
// parseChunksToItems (recordio/scannerv2.go:53-97).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rio_internal.h"

#ifndef RIO_VIEW_NT
#define RIO_VIEW_NT 1  // (round 5: C2 two-context step 3.05 -> 2.98 ms, A/B on one box)
#endif

namespace rio {

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// wave-uniform value (LDS loads are per lane; this makes them scalar)
// (the builtin returns int: widen through uint32_t, never sign-extend)
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
  return ((uint64_t)hi << 32) | lo;
}

// lane j's value, as a wave-uniform (scalar) value
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int j) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, j);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), j);
  return ((unsigned long long)hi << 32) | lo;
}

// ---------------------------------------------------------------- chunk headers
// little-endian u32 words of the magics (magic.go:15-36)
constexpr uint32_t kHdrLo = 0x5cd9e1d9u, kHdrHi = 0xf70416c2u;
constexpr uint32_t kPkdLo = 0xeb47762eu, kPkdHi = 0x2e3c0734u;
constexpr uint32_t kTrlLo = 0xd71abafeu, kTrlHi = 0x3a75dfcbu;

__device__ __forceinline__ uint32_t magic_class(uint32_t lo, uint32_t hi) {
  if (lo == kPkdLo && hi == kPkdHi) return kMagicPacked;
  if (lo == kHdrLo && hi == kHdrHi) return kMagicHeader;
  if (lo == kTrlLo && hi == kTrlHi) return kMagicTrailer;
  return kMagicOther;
}

// A chunk header's checks, in the order readChunk / ChunkScanner.Scan make
// them (chunk.go:273-287, 333-336): the size limit, then -- against the previous
// chunk of the span (none: the span starts on a block boundary) -- the index of
// a block's first chunk, the magic, the index and the total inside a block.
struct ChunkMeta {
  uint32_t info;  // magic class | error << 8
  uint32_t err;
};
__device__ __forceinline__ ChunkMeta chunk_meta(uint32_t mlo, uint32_t mhi, uint32_t size, uint32_t total,
                                                uint32_t index, bool has_prev, uint32_t plo, uint32_t phi,
                                                uint32_t ptotal, uint32_t pindex) {
  uint32_t err = kCkOk;
  if (size > (uint32_t)kMaxPayload) {
    err = kCkSize;
  } else {
    const bool prev_end = !has_prev || (int64_t)pindex == (int64_t)ptotal - 1;
    if (prev_end) {
      if (index != 0) err = kCkIndex;
    } else if (mlo != plo || mhi != phi) {
      err = kCkMagicChanged;
    } else if ((uint64_t)index != (uint64_t)pindex + 1) {
      err = kCkIndex;
    } else if (total != ptotal) {
      err = kCkTotal;
    }
  }
  return ChunkMeta{magic_class(mlo, mhi) | (err << 8), err};
}

// ---------------------------------------------------------------- wave scans
template <class T>
__device__ __forceinline__ T wave_incl_sum(T v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T t = __shfl_up(v, o, 64);
    if (l >= o) v += t;
  }
  return v;
}

// inclusive prefix sum of a u32 over the wave with DPP: row shifts inside
// each 16-lane row, then the row broadcasts (GFX9 row_bcast:15 / row_bcast:31)
__device__ __forceinline__ uint32_t wave_incl_sum_dpp(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ long long wave_incl_max(long long v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    long long t = __shfl_up(v, o, 64);
    if (l >= o && t > v) v = t;
  }
  return v;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long t = __shfl_xor(v, o, 64);
    v = t < v ? t : v;
  }
  return v;
}

// ---------------------------------------------------------------- payload
// Logical bytes [0, len) of one block's untransformed payload: the chunk
// payloads of the block in the span (none codec; the IOVecReader view of
// recordioiov.go:14-58) or one contiguous decoded buffer.
struct Payload {
  const uint8_t *span;
  const uint32_t *ck_size;
  const unsigned long long *ck_pay;  // exclusive prefix of chunk payload sizes
  uint64_t c0, total;                // chunks of the block
  uint64_t pay0;                     // ck_pay[c0]
  bool regular;                      // every chunk but the last carries 32740 bytes
  const uint8_t *contig;             // decoded buffer (compressed codecs) or null
  uint64_t len;

  __device__ __forceinline__ void chunk_of(uint64_t p, uint64_t &c, uint64_t &lo) const {
    if (regular) {
      uint64_t j = p / kMaxPayload;
      if (j >= total) j = total - 1;
      c = c0 + j;
      lo = j * kMaxPayload;
      return;
    }
    uint64_t a = c0, b = c0 + total;  // last chunk with ck_pay[c] - pay0 <= p
    while (b - a > 1) {
      const uint64_t m = (a + b) >> 1;
      if (ck_pay[m] - pay0 <= p) a = m;
      else b = m;
    }
    c = a;
    lo = ck_pay[a] - pay0;
  }
  // offset of logical byte p in the span (none codec)
  __device__ __forceinline__ uint64_t phys(uint64_t p) const {
    uint64_t c, lo;
    chunk_of(p, c, lo);
    return c * kChunk + kChunkHdr + (p - lo);
  }
  __device__ __forceinline__ uint32_t byte_at(uint64_t p) const {
    if (contig) return contig[p];
    return span[phys(p)];
  }
  // does [s, s+n) (n > 0) cross a chunk payload boundary?
  __device__ __forceinline__ bool straddles(uint64_t s, uint64_t n) const {
    if (contig || n == 0 || total <= 1) return false;
    if (regular) return (s / kMaxPayload) != ((s + n - 1) / kMaxPayload);
    uint64_t c1, l1, c2, l2;
    chunk_of(s, c1, l1);
    chunk_of(s + n - 1, c2, l2);
    return c1 != c2;
  }
  // 16 bytes at logical p, bytes at or beyond `len` read as 0x80 (no terminator)
  __device__ __forceinline__ void fetch16(uint64_t p, uint32_t w[4]) const {
    if (p >= len) {
      w[0] = w[1] = w[2] = w[3] = 0x80808080u;
      return;
    }
    if (contig) {
      if (p + 16 <= len) {
        const uint4 v = *reinterpret_cast<const uint4 *>(contig + p);
        w[0] = v.x;
        w[1] = v.y;
        w[2] = v.z;
        w[3] = v.w;
        return;
      }
    } else if (p + 16 <= len) {
      uint64_t c, lo;
      chunk_of(p, c, lo);
      const uint64_t o = p - lo;
      if (o + 16 <= ck_size[c]) {  // 4-byte aligned: 28 + 16k - 4j
        const uint32_t *q = reinterpret_cast<const uint32_t *>(span + c * kChunk + kChunkHdr + o);
        w[0] = q[0];
        w[1] = q[1];
        w[2] = q[2];
        w[3] = q[3];
        return;
      }
    }
    for (int k = 0; k < 4; k++) {
      uint32_t x = 0;
      for (int i = 0; i < 4; i++) {
        const uint64_t q = p + 4 * k + i;
        const uint32_t b = q < len ? byte_at(q) : 0x80u;
        x |= b << (8 * i);
      }
      w[k] = x;
    }
  }
};

__device__ __forceinline__ Payload make_chunk_payload(const uint8_t *span, const DevBufs &d, uint64_t c0,
                                                      uint64_t total) {
  Payload pl;
  pl.span = span;
  pl.ck_size = d.ck_size;
  pl.ck_pay = d.ck_pay;
  pl.c0 = c0;
  pl.total = total;
  pl.pay0 = d.ck_pay[c0];
  pl.len = d.ck_pay[c0 + total] - pl.pay0;
  pl.regular = (d.ck_pay[c0 + total - 1] - pl.pay0) == (total - 1) * (uint64_t)kMaxPayload;
  pl.contig = nullptr;
  return pl;
}

__device__ __forceinline__ Payload make_contig_payload(const uint8_t *p, uint64_t len) {
  Payload pl;
  pl.span = nullptr;
  pl.ck_size = nullptr;
  pl.ck_pay = nullptr;
  pl.c0 = pl.total = pl.pay0 = 0;
  pl.regular = true;
  pl.contig = p;
  pl.len = len;
  return pl;
}

// ---------------------------------------------------------------- header parse
enum ParseMode : int { kParseCount = 0, kParseWrite = 2 };

struct HdrResult {
  uint32_t status;  // BlockStatus
  unsigned long long a, b;
  unsigned long long nitems, hdr_len;
};

// where kParseWrite puts item views and straddler descriptors
struct ParseOut {
  unsigned long long *item_off, *item_len;
  unsigned long long *item_end;  // item-end mode: cumSize per item here (item_off / item_len unused)
  bool whole;                    // item-end mode: the block's payload is gathered whole (no straddlers)
  uint64_t item_base, item_cap;
  unsigned long long view_base;  // compressed: kItemInRecords | offset of the decoded block
  StradDesc *strad;              // per chunk slot
  unsigned long long *ssz;       // per chunk slot: padded straddler size
  uint64_t c0;
  unsigned long long *overflow;
};

// terminator bits (byte < 0x80) of 4 little-endian bytes as a 4-bit mask
__device__ __forceinline__ uint32_t term4(uint32_t w) {
  const uint32_t t = ~w & 0x80808080u;
  return ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t w[4], int i) {
  return (w[i >> 2] >> (8 * (i & 3))) & 0xffu;
}

__device__ __forceinline__ unsigned long long pad16(unsigned long long n) { return (n + 15) & ~15ull; }

// one item view (kParseWrite): a view into the span / decoded block, or, for an
// item crossing a chunk payload boundary, a straddler descriptor in the slot of
// the chunk it starts in (k_strad fills item_off)
__device__ __forceinline__ void emit_item(const Payload &pl, const ParseOut &po, uint64_t o, unsigned long long st,
                                          unsigned long long v, unsigned long long cum) {
  const uint64_t slot = po.item_base + (o - 1);
  if (slot >= po.item_cap) {
    atomicOr(po.overflow, 1ull);
    return;
  }
  if (po.item_end) {  // cumSize (scannerv2.go:83-91); a straddler still needs its bytes gathered
    po.item_end[slot] = cum;
    if (po.whole || !(v > 0 && pl.straddles(st, v))) return;
    uint64_t c, lo;
    pl.chunk_of(st, c, lo);
    StradDesc dsc;
    dsc.c0 = pl.c0;
    dsc.src = st;
    dsc.len = v;
    dsc.item = slot;
    po.strad[c] = dsc;
    po.ssz[c] = pad16(v);
    return;
  }
  po.item_len[slot] = v;
  if (pl.contig) {
    po.item_off[slot] = po.view_base + st;
    return;
  }
  if (v == 0 && st >= pl.len) {
    po.item_off[slot] = 0;
    return;
  }
  uint64_t c, lo;
  pl.chunk_of(st, c, lo);
  if (v > 0 && pl.straddles(st, v)) {
    StradDesc dsc;
    dsc.c0 = pl.c0;
    dsc.src = st;
    dsc.len = v;
    dsc.item = slot;
    po.strad[c] = dsc;
    po.ssz[c] = pad16(v);
    return;
  }
  po.item_off[slot] = c * kChunk + kChunkHdr + (st - lo);
}

// parseChunksToItems' header loop with Go 1.13 binary.Uvarint semantics: varint
// 0 is the item count, varints 1..n are item sizes. One wave; each lane owns
// 16 consecutive payload bytes of a 1 KiB window; terminator ordinals come from
// a wave prefix sum, varints crossing lanes read their earlier bytes back.
//  kParseCount: item count, header length and the reference's error checks.
//  kParseWrite: (header known valid) item views and straddler descriptors.
template <int MODE>
__device__ HdrResult parse_header(const Payload &pl, const HdrResult &known, const ParseOut &po) {
  const int l = lane_id();
  HdrResult r{kBlkOk, 0, 0, 0, 0};
  const uint64_t plen = pl.len;
  uint64_t ord_base = 0;       // terminators before this window
  long long prev_term = -1;    // position of the last terminator before this window
  bool have_n = MODE != kParseCount;
  unsigned long long nitems = known.nitems;
  const unsigned long long hdr = known.hdr_len;
  unsigned long long sum = 0;  // Go int arithmetic: wraps
  bool range = false;
  for (uint64_t base = 0; base < plen; base += 1024) {
    const uint64_t pos = base + 16ull * l;
    uint32_t w[4];
    pl.fetch16(pos, w);
    const uint32_t tmask = term4(w[0]) | (term4(w[1]) << 4) | (term4(w[2]) << 8) | (term4(w[3]) << 12);
    const uint32_t cnt = __popc(tmask);
    const uint32_t cnt_incl = wave_incl_sum<uint32_t>(cnt);
    const uint32_t ex = cnt_incl - cnt;
    const uint32_t wtotal = __shfl(cnt_incl, 63, 64);
    const long long mylast = tmask ? (long long)(pos + 31 - __clz(tmask)) : -1;
    const long long lmax = wave_incl_max(mylast);
    long long before = __shfl_up(lmax, 1, 64);
    if (l == 0) before = -1;
    if (before < prev_term) before = prev_term;
    const uint64_t ord0 = ord_base + ex;
    if (!have_n && wtotal > 0) {
      // item count: the first terminator overall, always at offset < 16 when valid
      const unsigned long long has = __ballot(cnt > 0);
      const int L = __ffsll((long long)has) - 1;
      const long long p0 = __shfl(mylast >= 0 ? (long long)(pos + __ffs(tmask) - 1) : -1, L, 64);
      const uint32_t b0 = __shfl(tmask ? byte_of(w, __ffs(tmask) - 1) : 0u, L, 64);
      if (p0 > 9 || (p0 == 9 && b0 > 1)) {
        r.status = kBlkNItems;
        r.a = (unsigned long long)(-(p0 + 1));
        return r;
      }
      unsigned long long v = 0;
      if (l == 0) {
        for (int i = 0; i <= (int)p0; i++) v |= (unsigned long long)(byte_of(w, i) & 0x7f) << (7 * i);
      }
      nitems = __shfl(v, 0, 64);
      have_n = true;
    }
    if (have_n) {
      // Walk this lane's terminators with ordinals 1..nitems. pass 0: value
      // sums (+ Go 1.13 overflow checks); pass 1: item views.
      unsigned long long first_bad = ~0ull;
      long long bad_len = 0;
      bool lrange = false;
      auto walk = [&](int pass, unsigned long long run) -> unsigned long long {
        unsigned long long lsum = 0;
        uint32_t m = tmask;
        long long prev = before;
        uint64_t ord = ord0;
        while (m) {
          const int i = __ffs(m) - 1;
          m &= m - 1;
          const long long e = (long long)pos + i;
          const long long s = prev + 1;
          prev = e;
          const uint64_t o = ord++;
          if (o == 0 || o > nitems) continue;
          const long long len = e - s + 1;
          const uint32_t be = byte_of(w, i);
          if (len - 1 > 9 || (len - 1 == 9 && be > 1)) {
            if (pass == 0 && o < first_bad) {
              first_bad = o;
              bad_len = len;
            }
            break;  // later varints of this lane come after the failure
          }
          unsigned long long v = 0;
          for (long long q = s; q <= e; q++) {
            const uint32_t b =
                (q >= (long long)pos) ? byte_of(w, (int)(q - (long long)pos)) : pl.byte_at((uint64_t)q);
            v |= (unsigned long long)(b & 0x7f) << (7 * (q - s));
          }
          if (pass == 0) {
            if (v > plen) lrange = true;
          } else {
            emit_item(pl, po, o, hdr + run + lsum, v, run + lsum + v);
          }
          lsum += v;
        }
        return lsum;
      };
      const unsigned long long lsum = walk(0, 0);
      if (MODE == kParseCount) {
        // the first overflow in the wave (and in file order) stops the header
        const unsigned long long wbad = wave_min_u64(first_bad);
        if (wbad != ~0ull) {
          const unsigned long long bl = __ballot(first_bad == wbad);
          const long long blen = __shfl(bad_len, __ffsll((long long)bl) - 1, 64);
          r.status = kBlkItemSize;
          r.a = wbad - 1;
          r.b = (unsigned long long)(-blen);
          return r;
        }
        if (__ballot(lrange)) range = true;
      } else {
        const unsigned long long incl = wave_incl_sum<unsigned long long>(lsum);
        walk(1, sum + incl - lsum);
      }
      sum += wave_sum<unsigned long long>(lsum);
      // the header ends at the terminator with ordinal nitems
      if (ord_base + wtotal > nitems) {
        const bool mine = (nitems >= ord0) && (nitems < ord0 + cnt);
        long long endp = -1;
        if (mine) {
          uint32_t mm = tmask;
          for (uint64_t k = ord0; k < nitems; k++) mm &= mm - 1;
          endp = (long long)pos + __ffs(mm) - 1;
        }
        const unsigned long long eb = __ballot(mine);
        const long long hend = __shfl(endp, __ffsll((long long)eb) - 1, 64) + 1;
        r.nitems = nitems;
        r.hdr_len = (unsigned long long)hend;
        if (MODE == kParseCount) {
          if (sum + r.hdr_len != plen) {
            r.status = kBlkBlockSize;
            r.a = plen;
            r.b = sum + r.hdr_len;
          } else if (range) {
            r.status = kBlkItemRange;
          }
        }
        return r;
      }
    }
    ord_base += wtotal;
    const long long wl = __shfl(lmax, 63, 64);
    if (wl > prev_term) prev_term = wl;
  }
  // payload exhausted: binary.Uvarint returns n == 0
  if (!have_n) {
    r.status = kBlkNItems;
    r.a = 0;
  } else {
    r.status = kBlkItemSize;
    r.a = ord_base == 0 ? 0 : ord_base - 1;
    r.b = 0;
  }
  return r;
}

// ---------------------------------------------------------------- fast path
// The common block shape -- the whole header inside the first 1 KiB of the
// payload, every varint shorter than 11 bytes, sizes consistent with the block,
// a regular chunk layout -- parsed item-parallel from one prefetched window:
// the window and the terminator positions go to the wave's LDS, then lane t
// decodes items t, t+64, ... and writes their views coalesced. Anything else
// returns false before writing and the block goes through parse_header, which
// also produces the reference's error values.

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// bytes [s, e] of the LDS window as a uvarint (e - s < 10)
__device__ __forceinline__ unsigned long long lds_uvarint(const uint8_t *lwin, uint32_t s, uint32_t e) {
  unsigned long long v = 0;
  for (uint32_t q = s; q <= e; q++) v |= (unsigned long long)(lwin[q] & 0x7fu) << (7 * (q - s));
  return v;
}

// Wave-cooperative copy of n bytes, src and dst congruent mod 4.
__device__ __forceinline__ void wave_copy(uint8_t *dst, const uint8_t *src, uint64_t n) {
  const int l = lane_id();
  const uint64_t head = (4 - ((uintptr_t)src & 3)) & 3;
  const uint64_t h = head < n ? head : n;
  if ((uint64_t)l < h) dst[l] = src[l];
  const uint64_t nw = (n - h) >> 2;
  const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src + h);
  uint32_t *d4 = reinterpret_cast<uint32_t *>(dst + h);
  for (uint64_t k = l; k < nw; k += 64) d4[k] = s4[k];
  const uint64_t t0 = h + (nw << 2);
  if (t0 + l < n) dst[t0 + l] = src[t0 + l];
}

// Straddler of a regular block into the span-shaped side buffer: it starts at
// its own span offset there and runs contiguously (the chunk headers it crosses
// are squeezed out), so straddlers never overlap and src == dst (mod 4).
__device__ __forceinline__ void copy_straddler(const Payload &pl, uint8_t *side, uint64_t st, uint64_t v,
                                               uint64_t dst0) {
  uint64_t p = st, done = 0;
  while (done < v) {
    const uint64_t j = p / kMaxPayload, in = p - j * kMaxPayload;
    const uint64_t room = kMaxPayload - in;
    const uint64_t n = (v - done) < room ? (v - done) : room;
    wave_copy(side + dst0 + done, pl.span + (pl.c0 + j) * kChunk + kChunkHdr + in, n);
    p += n;
    done += n;
  }
}

// 4 bytes of the LDS window from byte s (the window is dword-aligned, with room
// for one dword past its 1 KiB)
__device__ __forceinline__ uint32_t lds_bytes4(const uint8_t *lwin, uint32_t s) {
  const uint32_t *w32 = reinterpret_cast<const uint32_t *>(lwin);
  const uint32_t a = s >> 2;
  return __builtin_amdgcn_alignbyte(w32[a + 1], w32[a], s & 3u);
}

// the uvarint of the n <= 4 bytes in x (only its last byte is a terminator)
__device__ __forceinline__ uint32_t uvarint4(uint32_t x, uint32_t n) {
  const uint32_t v = (x & 0x7fu) | ((x >> 1) & 0x3f80u) | ((x >> 2) & 0x1fc000u) | ((x >> 3) & 0xfe00000u);
  return n >= 4 ? v : v & ((1u << (7 * n)) - 1u);
}

// The fast path's passes for a header of at most 256 sizes (C2's 253, C4's
// ~100): lane l owns items 4l+1 .. 4l+4, so one wave scan places them all; the
// sizes stay in registers between the checks and the writes, sums are u32
// (every valid prefix is below plen < 2^32). Returns 1 (views written), 0 (not
// a valid header: nothing written, the caller declines) or -1 (a size varint
// longer than 4 bytes: the generic passes below take the block).
// kBnd: `bnd` holds payload bytes [kBndW0 + 16 l, +16) -- 512 bytes either side of
// the first chunk boundary, loaded with the header window (k_parse_lean) --
// and a straddler inside that range is written from it, with no load.
constexpr uint32_t kBndW0 = (uint32_t)kMaxPayload - 512;

// straddler [S, S + v) (payload bytes, inside the boundary window) to side + phys,
// in whole dwords: phys = S (mod 4), so every dword lands aligned; the up to 3
// bytes before / after it belong to no straddler (the next one starts a chunk
// later), and side bytes outside straddlers are never read
__device__ __forceinline__ void straddler_from_regs(const uint32_t (&bnd)[4], uint8_t *side, uint32_t S, uint32_t v,
                                                    unsigned long long phys) {
  const int l = lane_id();
  const uint32_t E = S + v;
  uint32_t *dst = reinterpret_cast<uint32_t *>(side + (phys - (S & 3u)));  // the dword holding byte S
  const uint32_t S4 = S & ~3u;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t P = kBndW0 + 16u * (uint32_t)l + 4u * i;
    if (P + 4 > S && P < E) dst[(P - S4) >> 2] = bnd[i];
  }
}

// item view stores of the fast path: written once, read by the caller (not
// by this pass), so they stream past the caches (RIO_VIEW_NT, on since round 5:
// the C2 step beside the other context's CRC pass 3.05 -> 2.98 ms)
typedef unsigned long long u64x2_a8 __attribute__((ext_vector_type(2), aligned(8)));
__device__ __forceinline__ void view_store2(unsigned long long *p, unsigned long long v0, unsigned long long v1) {
  const u64x2_a8 v = {v0, v1};
#if RIO_VIEW_NT
  __builtin_nontemporal_store(v, reinterpret_cast<u64x2_a8 *>(p));
#else
  *reinterpret_cast<u64x2_a8 *>(p) = v;
#endif
}

__device__ __forceinline__ void view_store(unsigned long long *p, unsigned long long v) {
#if RIO_VIEW_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

template <bool kBnd>
__device__ __forceinline__ int small_header(const Payload &pl, const ParseOut &po, const uint8_t *lwin,
                                            const uint16_t *ltpos, uint32_t nitems, uint32_t hdr,
                                            uint8_t *sparse_side, const uint32_t (&bnd)[4]) {
  const int l = lane_id();
  const uint32_t plen = (uint32_t)pl.len;
  uint32_t v[4], st[4];
  bool lng = false, bad = false;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    v[k] = 0;
    const uint32_t o = 64u * k + (uint32_t)l + 1;
    if (o <= nitems) {
      const uint32_t e = ltpos[o], n = e - ltpos[o - 1];  // varint o: bytes e-n+1 .. e
      if (n > 4) {
        lng = true;
      } else {
        v[k] = uvarint4(lds_bytes4(lwin, e + 1 - n), n);
        if (v[k] > plen) bad = true;
      }
    }
  }
  if (__ballot(lng)) return -1;
  if (__ballot(bad)) return 0;
  // item starts: one u32 scan per 64 items; steps are below 2^28, so the first
  // wrap of a scan leaves incl < v, and a carry past plen is already invalid
  unsigned long long carry = hdr;
  bool wrap = false;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t incl = wave_incl_sum_dpp(v[k]);
    wrap |= incl < v[k];
    st[k] = (uint32_t)carry + incl - v[k];
    carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (carry > pl.len) break;
  }
  if (__ballot(wrap) || carry != pl.len) return 0;
  const bool chunks = !pl.contig && pl.total > 1;
  if (kBnd && chunks) {  // every straddler must lie in the boundary window (else: declined, untouched)
    bool far = false;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t st_ = st[k], vk = v[k];
      if (64u * k + (uint32_t)l + 1 <= nitems && vk > 0 && st_ / (uint32_t)kMaxPayload != (st_ + vk - 1) / (uint32_t)kMaxPayload)
        far |= !(st_ >= kBndW0 && st_ + vk <= kBndW0 + 1024);
    }
    if (__ballot(far)) return 0;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t o = 64u * k + (uint32_t)l + 1, sk = st[k], vk = v[k];
    bool sd = false;
    unsigned long long phys = 0;
    if (o <= nitems) {
      const uint64_t slot = po.item_base + (o - 1);
      if (slot < po.item_cap && po.item_end) {  // cumSize: the item's end past the header
        view_store(po.item_end + slot, (unsigned long long)(sk + vk - hdr));
        if (chunks) {
          const uint32_t j = sk / (uint32_t)kMaxPayload;
          sd = vk > 0 && j != (sk + vk - 1) / (uint32_t)kMaxPayload;
          phys = (pl.c0 + j) * (unsigned long long)kChunk + kChunkHdr + (sk - j * (uint32_t)kMaxPayload);
          if (sd && !sparse_side) {
            StradDesc dsc;
            dsc.c0 = pl.c0;
            dsc.src = sk;
            dsc.len = vk;
            dsc.item = slot;
            po.strad[pl.c0 + j] = dsc;
            po.ssz[pl.c0 + j] = pad16(vk);
          }
        }
      } else if (slot < po.item_cap) {
        view_store(po.item_len + slot, vk);
        if (pl.contig) {
          view_store(po.item_off + slot, po.view_base + sk);
        } else {
          const uint32_t j = sk / (uint32_t)kMaxPayload;
          phys = (pl.c0 + j) * (unsigned long long)kChunk + kChunkHdr + (sk - j * (uint32_t)kMaxPayload);
          sd = chunks && vk > 0 && j != (sk + vk - 1) / (uint32_t)kMaxPayload;
          if (sd && sparse_side) {
            view_store(po.item_off + slot, kItemInRecords | phys);
          } else if (sd) {
            StradDesc dsc;
            dsc.c0 = pl.c0;
            dsc.src = sk;
            dsc.len = vk;
            dsc.item = slot;
            po.strad[pl.c0 + j] = dsc;
            po.ssz[pl.c0 + j] = pad16(vk);
          } else {
            view_store(po.item_off + slot, (vk == 0 && sk >= plen) ? 0ull : phys);
          }
        }
      } else {
        atomicOr(po.overflow, 1ull);
      }
    }
    if (sparse_side) {
      unsigned long long sm = __ballot(sd);
      while (sm) {
        const int L = __ffsll((long long)sm) - 1;
        sm &= sm - 1;
        const uint32_t S = (uint32_t)__shfl(sk, L, 64), V = (uint32_t)__shfl(vk, L, 64);
        const unsigned long long ph = __shfl(phys, L, 64);
        if (kBnd)
          straddler_from_regs(bnd, sparse_side, S, V, ph);  // (checked above: inside the window)
        else
          copy_straddler(pl, sparse_side, S, V, ph);
      }
    }
  }
  return 1;
}

// window w = payload bytes [16*lane, 16*lane + 16) (0x80 past the payload);
// writes the block's item views like parse_header<kParseWrite> and returns
// nitems / hdr_len in r, or returns false (nothing written).
// sparse_side != null: straddlers are copied here (span-shaped side buffer);
// else they get descriptors for k_strad.
__device__ bool fast_header(const Payload &pl, const uint32_t (&w)[4], HdrResult &r, const ParseOut &po,
                            uint8_t *lwin, uint16_t *ltpos, uint8_t *sparse_side) {
  const int l = lane_id();
  const uint64_t plen = pl.len;
  if (plen >= (1ull << 32)) return false;
  if (!pl.contig && !pl.regular) return false;
  const uint32_t tmask = term4(w[0]) | (term4(w[1]) << 4) | (term4(w[2]) << 8) | (term4(w[3]) << 12);
  const uint32_t cnt = __popc(tmask);
  const uint32_t incl = wave_incl_sum_dpp(cnt);
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  if (total == 0) return false;
  *reinterpret_cast<uint4 *>(lwin + 16 * l) = make_uint4(w[0], w[1], w[2], w[3]);
  {
    uint32_t m = tmask, o = incl - cnt;
    while (m) {
      const uint32_t i = __ffs(m) - 1;
      m &= m - 1;
      ltpos[o++] = (uint16_t)(16 * l + i);
    }
  }
  wave_lds_sync();
  // item count: the first varint
  const uint32_t p0 = ltpos[0];
  if (p0 > 9 || (p0 == 9 && lwin[9] > 1)) return false;
  const unsigned long long nitems = lds_uvarint(lwin, 0, p0);
  if (nitems >= total) return false;  // header not inside the window
  const uint32_t hdr = (uint32_t)ltpos[nitems] + 1;
  if (nitems <= 256) {
    const uint32_t none[4] = {0, 0, 0, 0};
    const int res = small_header<false>(pl, po, lwin, ltpos, (uint32_t)nitems, hdr, sparse_side, none);
    if (res >= 0) {
      if (!res) return false;
      r.status = kBlkOk;
      r.nitems = nitems;
      r.hdr_len = hdr;
      return true;
    }
  }
  // pass A: validity, range, sum
  int bad = 0;
  unsigned long long lsum = 0;
  for (unsigned long long g = 0; g < nitems; g += 64) {
    const unsigned long long o = g + l + 1;
    if (o <= nitems) {
      const uint32_t s = (uint32_t)ltpos[o - 1] + 1, e = ltpos[o];
      if (e - s > 9 || (e - s == 9 && lwin[e] > 1)) {
        bad = 1;
      } else {
        const unsigned long long v = lds_uvarint(lwin, s, e);
        if (v > plen) bad = 1;
        lsum += v;
      }
    }
  }
  if (__ballot(bad)) return false;
  if (wave_sum<unsigned long long>(lsum) + hdr != plen) return false;
  // pass B: views, coalesced (lane t: slot base + g + t)
  const bool chunks = !pl.contig && pl.total > 1;
  unsigned long long carry = hdr;
  for (unsigned long long g = 0; g < nitems; g += 64) {
    const unsigned long long o = g + l + 1;
    const bool have = o <= nitems;
    unsigned long long v = 0;
    if (have) v = lds_uvarint(lwin, (uint32_t)ltpos[o - 1] + 1, ltpos[o]);
    const unsigned long long vi = wave_incl_sum<unsigned long long>(v);
    const uint32_t st = (uint32_t)(carry + vi - v);
    carry += __shfl(vi, 63, 64);
    bool sd = false;
    unsigned long long phys = 0;
    if (have) {
      const uint64_t slot = po.item_base + (o - 1);
      if (slot < po.item_cap && po.item_end) {  // cumSize
        po.item_end[slot] = st + v - hdr;
        if (chunks) {
          const uint32_t j = st / (uint32_t)kMaxPayload;
          sd = v > 0 && j != (st + (uint32_t)v - 1) / (uint32_t)kMaxPayload;
          phys = (pl.c0 + j) * (unsigned long long)kChunk + kChunkHdr + (st - j * (uint32_t)kMaxPayload);
          if (sd && !sparse_side) {
            StradDesc dsc;
            dsc.c0 = pl.c0;
            dsc.src = st;
            dsc.len = v;
            dsc.item = slot;
            po.strad[pl.c0 + j] = dsc;
            po.ssz[pl.c0 + j] = pad16(v);
          }
        }
      } else if (slot < po.item_cap) {
        po.item_len[slot] = v;
        if (pl.contig) {
          po.item_off[slot] = po.view_base + st;
        } else {
          const uint32_t j = st / (uint32_t)kMaxPayload;
          phys = (pl.c0 + j) * (unsigned long long)kChunk + kChunkHdr + (st - j * (uint32_t)kMaxPayload);
          sd = chunks && v > 0 && j != (st + (uint32_t)v - 1) / (uint32_t)kMaxPayload;
          if (sd && sparse_side) {
            po.item_off[slot] = kItemInRecords | phys;
          } else if (sd) {
            StradDesc dsc;
            dsc.c0 = pl.c0;
            dsc.src = st;
            dsc.len = v;
            dsc.item = slot;
            po.strad[pl.c0 + j] = dsc;
            po.ssz[pl.c0 + j] = pad16(v);
          } else {
            po.item_off[slot] = (v == 0 && st >= plen) ? 0ull : phys;
          }
        }
      } else {
        atomicOr(po.overflow, 1ull);
      }
    }
    if (sparse_side) {
      unsigned long long sm = __ballot(sd);
      while (sm) {
        const int L = __ffsll((long long)sm) - 1;
        sm &= sm - 1;
        copy_straddler(pl, sparse_side, (uint64_t)__shfl(st, L, 64), __shfl(v, L, 64), __shfl(phys, L, 64));
      }
    }
  }
  r.status = kBlkOk;
  r.nitems = nitems;
  r.hdr_len = hdr;
  return true;
}

}  // namespace rio
