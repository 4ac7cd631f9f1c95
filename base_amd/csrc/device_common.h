// Device helpers shared by the scan kernels and the codec kernels: wave-level
// scans, the block payload accessor and the uvarint header parser of
// parseChunksToItems (recordio/scannerv2.go:53-97).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rio_internal.h"

namespace rio {

__device__ __forceinline__ int lane_id() { return __lane_id(); }

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
enum ParseMode : int { kParseCount = 0, kParseStrad = 1, kParseWrite = 2 };

struct HdrResult {
  uint32_t status;  // BlockStatus
  unsigned long long a, b;
  unsigned long long nitems, hdr_len;
  unsigned long long strad_bytes, strad_count;  // kParseStrad
};

// where kParseWrite puts item views and straddler descriptors
struct ParseOut {
  unsigned long long *item_off, *item_len;
  uint64_t item_base, item_cap;
  unsigned long long view_base;  // compressed: kItemInRecords | offset of the decoded block
  StradDesc *strad;
  uint64_t strad_idx;            // first descriptor slot of the block
  unsigned long long side_base;  // first side-buffer byte of the block
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

// parseChunksToItems' header loop with Go 1.13 binary.Uvarint semantics: varint
// 0 is the item count, varints 1..n are item sizes. One wave; each lane owns
// 16 consecutive payload bytes of a 1 KiB window; terminator ordinals come from
// a wave prefix sum, varints crossing lanes read their earlier bytes back.
//  kParseCount: item count, header length and the reference's error checks.
//  kParseStrad: (header known valid) bytes/count of items crossing a chunk
//               payload boundary -- those are copied to the side buffer.
//  kParseWrite: item views (offset, length) and straddler descriptors.
template <int MODE>
__device__ HdrResult parse_header(const Payload &pl, const HdrResult &known, const ParseOut &po) {
  const int l = lane_id();
  HdrResult r{kBlkOk, 0, 0, 0, 0, 0, 0};
  const uint64_t plen = pl.len;
  uint64_t ord_base = 0;       // terminators before this window
  long long prev_term = -1;    // position of the last terminator before this window
  bool have_n = MODE != kParseCount;
  unsigned long long nitems = known.nitems;
  const unsigned long long hdr = known.hdr_len;
  unsigned long long sum = 0;  // Go int arithmetic: wraps
  unsigned long long strad_b = 0, strad_n = 0;
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
      // sums (+ Go 1.13 overflow checks); pass 1: straddler bytes/count at the
      // item positions; pass 2: item views and straddler descriptors.
      unsigned long long first_bad = ~0ull;
      long long bad_len = 0;
      bool lrange = false;
      auto walk = [&](int pass, unsigned long long run, unsigned long long sb, unsigned long long sn,
                      unsigned long long &o_sb, unsigned long long &o_sn) -> unsigned long long {
        unsigned long long lsum = 0;
        uint32_t m = tmask;
        long long prev = before;
        uint64_t ord = ord0;
        o_sb = 0;
        o_sn = 0;
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
            const unsigned long long st = hdr + run + lsum;  // logical start of item o
            const bool sd = pl.straddles(st, v);
            if (pass == 2) {
              const uint64_t slot = po.item_base + (o - 1);
              if (slot < po.item_cap) {
                unsigned long long off;
                if (pl.contig) off = po.view_base + st;
                else if (sd) off = kItemInRecords | (po.side_base + sb + o_sb);
                else off = (v == 0 && st >= plen) ? 0 : pl.phys(st);
                po.item_off[slot] = off;
                po.item_len[slot] = v;
              } else {
                atomicOr(po.overflow, 1ull);
              }
              if (sd) {
                StradDesc dsc;
                dsc.c0 = po.c0;
                dsc.src = st;
                dsc.len = v;
                dsc.dst = po.side_base + sb + o_sb;
                po.strad[po.strad_idx + sn + o_sn] = dsc;
              }
            }
            if (sd) {
              o_sb += pad16(v);
              o_sn += 1;
            }
          }
          lsum += v;
        }
        return lsum;
      };
      unsigned long long t0, t1;
      const unsigned long long lsum = walk(0, 0, 0, 0, t0, t1);
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
        const unsigned long long run = sum + incl - lsum;
        unsigned long long lsb, lsn;
        walk(1, run, 0, 0, lsb, lsn);
        if (MODE == kParseWrite) {
          const unsigned long long ib = wave_incl_sum<unsigned long long>(lsb);
          const unsigned long long in = wave_incl_sum<unsigned long long>(lsn);
          walk(2, run, strad_b + ib - lsb, strad_n + in - lsn, t0, t1);
        }
        strad_b += wave_sum<unsigned long long>(lsb);
        strad_n += wave_sum<unsigned long long>(lsn);
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
        r.strad_bytes = strad_b;
        r.strad_count = strad_n;
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
// payload, every varint shorter than 11 bytes, sizes consistent with the block
// -- parsed from one 16 B/lane window with fully unrolled byte loops (no
// dynamic register indexing). Anything else returns false and the block goes
// through parse_header, which also produces the reference's error values.

// lane's terminators in byte order: f(k, i, value, varint_len, last_byte);
// the lane's first varint continues the previous lane's trailing bytes
template <class F>
__device__ __forceinline__ void walk_lane(const uint32_t w[4], uint32_t tmask, unsigned long long c_acc, int c_len,
                                          F &&f) {
  unsigned long long acc = 0;
  int len = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t b = (w[i >> 2] >> (8 * (i & 3))) & 0xffu;
    const int sh = 7 * len;
    if (sh < 64) acc |= (unsigned long long)(b & 0x7fu) << sh;
    len++;
    if ((tmask >> i) & 1u) {
      unsigned long long v = acc;
      int vl = len;
      if (k == 0) {
        const int csh = 7 * c_len;
        v = c_acc | (csh < 64 ? (acc << csh) : 0ull);
        vl = c_len + len;
      }
      f(k, v, vl, b);
      acc = 0;
      len = 0;
      k++;
    }
  }
}

__device__ __forceinline__ bool uvarint_ok(int vl, uint32_t last) { return vl < 10 || (vl == 10 && last <= 1); }

// MODE kParseCount: r gets nitems, hdr_len, straddler bytes/count.
// MODE kParseWrite: item views and straddler descriptors as parse_header.
template <int MODE>
__device__ bool fast_header(const Payload &pl, HdrResult &r, const ParseOut &po) {
  const int l = lane_id();
  const uint64_t plen = pl.len;
  if (plen >= (1ull << 32)) return false;
  if (!pl.contig && !pl.regular) return false;
  const uint32_t pos = 16u * (uint32_t)l;
  uint32_t w[4];
  pl.fetch16(pos, w);
  const uint32_t tmask = term4(w[0]) | (term4(w[1]) << 4) | (term4(w[2]) << 8) | (term4(w[3]) << 12);
  // the item count: lane 0's first varint
  unsigned long long n0 = 0;
  bool n0_ok = false;
  if (l == 0 && tmask) {
    walk_lane(w, tmask & (0u - tmask), 0ull, 0, [&](int, unsigned long long v, int vl, uint32_t b) {
      n0 = v;
      n0_ok = uvarint_ok(vl, b);
    });
  }
  const unsigned long long nitems = __shfl(n0, 0, 64);
  if (!__shfl((int)n0_ok, 0, 64)) return false;
  const uint32_t cnt = __popc(tmask);
  const uint32_t incl = wave_incl_sum<uint32_t>(cnt);
  const uint32_t ex = incl - cnt;
  const uint32_t total = __shfl(incl, 63, 64);
  if (nitems >= total) return false;  // header not inside the window
  // header end: the terminator with ordinal nitems
  const bool mine = nitems >= ex && nitems < incl;
  int endbit = -1;
  if (mine) {
    uint32_t mm = tmask;
    for (uint32_t k = ex; k < (uint32_t)nitems; k++) mm &= mm - 1;
    endbit = __ffs(mm) - 1;
  }
  const unsigned long long eb = __ballot(mine);
  const uint32_t hdr = (uint32_t)__shfl((int)pos + endbit, __ffsll((long long)eb) - 1, 64) + 1;
  // carry-in: the previous lane's bytes after its last terminator
  const int t_last = tmask ? 31 - __clz(tmask) : -1;
  unsigned long long tacc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t b = (w[i >> 2] >> (8 * (i & 3))) & 0xffu;
    const int sh = 7 * (i - t_last - 1);
    if (i > t_last && sh < 64) tacc |= (unsigned long long)(b & 0x7fu) << sh;
  }
  int c_len = __shfl_up(15 - t_last, 1, 64);
  unsigned long long c_acc = __shfl_up(tacc, 1, 64);
  if (l == 0) {
    c_len = 0;
    c_acc = 0;
  }
  // sizes: validity, range, lane sums
  bool bad = false;
  unsigned long long lsum = 0;
  walk_lane(w, tmask, c_acc, c_len, [&](int k, unsigned long long v, int vl, uint32_t b) {
    const uint32_t o = ex + (uint32_t)k;
    if (o >= 1 && o <= nitems) {
      if (!uvarint_ok(vl, b) || v > plen) bad = true;
      lsum += v;
    }
  });
  if (__ballot(bad)) return false;
  if (wave_sum<unsigned long long>(lsum) + hdr != plen) return false;
  const unsigned long long run0 = hdr + wave_incl_sum<unsigned long long>(lsum) - lsum;
  const bool chunks = !pl.contig && pl.total > 1;
  // straddlers (items crossing a chunk payload boundary)
  unsigned long long sb = 0, sn = 0;
  if (chunks) {
    unsigned long long run = run0;
    walk_lane(w, tmask, c_acc, c_len, [&](int k, unsigned long long v, int, uint32_t) {
      const uint32_t o = ex + (uint32_t)k;
      if (o >= 1 && o <= nitems) {
        const uint32_t st = (uint32_t)run;
        if (v > 0 && st / (uint32_t)kMaxPayload != (st + (uint32_t)v - 1) / (uint32_t)kMaxPayload) {
          sb += pad16(v);
          sn += 1;
        }
        run += v;
      }
    });
  }
  if (MODE == kParseCount) {
    r.status = kBlkOk;
    r.nitems = nitems;
    r.hdr_len = hdr;
    r.strad_bytes = chunks ? wave_sum<unsigned long long>(sb) : 0;
    r.strad_count = chunks ? wave_sum<unsigned long long>(sn) : 0;
    return true;
  }
  unsigned long long sbx = 0, snx = 0;
  if (chunks) {
    sbx = wave_incl_sum<unsigned long long>(sb) - sb;
    snx = wave_incl_sum<unsigned long long>(sn) - sn;
  }
  unsigned long long run = run0;
  walk_lane(w, tmask, c_acc, c_len, [&](int k, unsigned long long v, int, uint32_t) {
    const uint32_t o = ex + (uint32_t)k;
    if (o >= 1 && o <= nitems) {
      const uint32_t st = (uint32_t)run;
      const uint64_t slot = po.item_base + (o - 1);
      unsigned long long off;
      bool sd = false;
      if (pl.contig) {
        off = po.view_base + st;
      } else {
        const uint32_t j = st / (uint32_t)kMaxPayload;
        sd = chunks && v > 0 && j != (st + (uint32_t)v - 1) / (uint32_t)kMaxPayload;
        if (sd) off = kItemInRecords | (po.side_base + sbx);
        else if (v == 0 && st >= plen) off = 0;
        else off = (pl.c0 + j) * (unsigned long long)kChunk + kChunkHdr + (st - j * (uint32_t)kMaxPayload);
      }
      if (slot < po.item_cap) {
        po.item_off[slot] = off;
        po.item_len[slot] = v;
      } else {
        atomicOr(po.overflow, 1ull);
      }
      if (sd) {
        StradDesc dsc;
        dsc.c0 = po.c0;
        dsc.src = st;
        dsc.len = v;
        dsc.dst = po.side_base + sbx;
        po.strad[po.strad_idx + snx] = dsc;
        sbx += pad16(v);
        snx += 1;
      }
      run += v;
    }
  });
  return true;
}

}  // namespace rio
