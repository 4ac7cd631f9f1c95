// v1 ("legacy") packed-record unpack on the GPU: Unpacker.Unpack
// (recordio/deprecated/packer.go:214-272) for every packed record of a span at
// once, as the v2 scanner's legacy adapter calls it per record
// (recordio/legacyscanner.go:84-117).
//
// A packed record's payload is [crc32 u32][uvarint n][n uvarint sizes][items].
// The host walks the 20-byte record headers (a serial chain: each record's
// offset is the previous one's end) and checks the item count varint; this
// kernel does the per-item work, one wave per record:
//   pass 0: the header varints from payload byte 4 on, in 1 KiB windows (lane
//           t owns bytes 16t..16t+15; terminator ordinals from a wave prefix
//           sum, as parse_header does for v2 blocks) -> the header end, the
//           first size varint that fails binary.Uvarint, and the CRC32 of
//           bytes [4, end) folded window by window (per-lane byte-table CRC of
//           16 bytes, a 6-level shuffle tree with x^(128*2^l) multipliers);
//   pass 1: (header valid) the sizes again -> item offsets by a wave prefix
//           sum with a running carry, Unpack's bounds checks, item views
//           written coalesced-ish (consecutive items -> consecutive slots).
// Only each packed record's header bound (crc, count, 10 bytes per size
// varint) is staged to the device; a header that runs past it (a size varint
// of more than 10 bytes, an error) is restaged whole and run again. Item views
// are span offsets: items stay in the caller's host span.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "legacy.h"
#include "rio_internal.h"

namespace rio {

// GF(2) product in the reflected CRC-32 representation (crc_tables.cpp)
__device__ __forceinline__ uint32_t v1_gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 31; i >= 0; i--) {
    p ^= b & (0u - ((a >> i) & 1u));
    b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
  }
  return p;
}

__device__ uint32_t v1_gf_pow(uint32_t base, uint64_t e) {
  uint32_t r = 1u << 31;  // 1
  while (e) {
    if (e & 1) r = v1_gf_mul(r, base);
    base = v1_gf_mul(base, base);
    e >>= 1;
  }
  return r;
}

// x^(8n) and x^(-8n)
__device__ __forceinline__ uint32_t v1_xpow8(uint64_t n) { return v1_gf_pow(1u << 30, 8 * n); }
__device__ __forceinline__ uint32_t v1_xpow8_inv(uint64_t n) {
  const uint32_t xinv = (((1u << 31) ^ kPoly) << 1) | 1u;
  return v1_gf_pow(xinv, 8 * n);
}

// 16 bytes at p[rel..rel+16) from aligned dword loads; bytes at or past hlen
// read as 0x80 (never a varint terminator). The staging buffer has >= 64
// bytes of tail room, so the 5th dword never leaves it.
__device__ __forceinline__ void v1_load16(const uint8_t *p, int64_t rel, int64_t hlen, uint32_t (&w)[4]) {
  if (rel >= hlen) {
    w[0] = w[1] = w[2] = w[3] = 0x80808080u;
    return;
  }
  const uintptr_t a = (uintptr_t)(p + rel);
  const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  uint32_t d[5];
#pragma unroll
  for (int k = 0; k < 5; k++) d[k] = q[k];
#pragma unroll
  for (int k = 0; k < 4; k++) w[k] = sh ? (d[k] >> sh) | (d[k + 1] << (32 - sh)) : d[k];
  if (rel + 16 > hlen) {
#pragma unroll
    for (int j = 0; j < 16; j++)
      if (rel + j >= hlen) w[j >> 2] = (w[j >> 2] & ~(0xffu << (8 * (j & 3)))) | (0x80u << (8 * (j & 3)));
  }
}

__device__ __forceinline__ uint32_t v1_term_mask(const uint32_t (&w)[4]) {
  return term4(w[0]) | (term4(w[1]) << 4) | (term4(w[2]) << 8) | (term4(w[3]) << 12);
}

__global__ void __launch_bounds__(256) k_v1_unpack(const uint8_t *__restrict__ dstage,
                                                   const V1Job *__restrict__ jobs, uint64_t njobs,
                                                   unsigned long long *__restrict__ item_off,
                                                   unsigned long long *__restrict__ item_len, V1Res *res) {
  __shared__ uint32_t tab[256];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? kPoly ^ (c >> 1) : c >> 1;
    tab[i] = c;
  }
  __syncthreads();
  const int l = lane_id();
  // lane-tree multipliers x^(8*16*2^lv) and the window step x^(8*1024)
  uint32_t cm[6];
  cm[0] = v1_xpow8(16);
#pragma unroll
  for (int lv = 1; lv < 6; lv++) cm[lv] = v1_gf_mul(cm[lv - 1], cm[lv - 1]);
  const uint32_t x1024 = v1_gf_mul(cm[5], cm[5]);
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t j = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; j < njobs; j += nwaves) {
    const V1Job jb = jobs[j];
    const uint8_t *p = dstage + jb.off;  // the record payload's staged prefix
    const int64_t len = (int64_t)jb.size;
    const uint64_t nb = jb.nbufs;
    const uint8_t *h = p + 4;  // header varints: ordinal 0 = item count, 1..nb = sizes
    const int64_t hlen = (int64_t)jb.hbytes - 4;
    V1Res r{kV1Ok, 0, 0, 0, 0};
    // ---- pass 0: header end, first bad size varint, CRC of h[0, hend)
    uint64_t ord_base = 0;
    long long prev_term = -1;
    long long hend = -1;
    uint32_t R = 0;
    int64_t covered = 0;
    for (int64_t base = 0; base < hlen; base += 1024) {
      const int64_t pos = base + 16ll * l;
      uint32_t w[4];
      v1_load16(h, pos, hlen, w);
      const uint32_t tmask = v1_term_mask(w);
      const uint32_t cnt = __popc(tmask);
      const uint32_t incl = wave_incl_sum<uint32_t>(cnt);
      const uint32_t wtotal = __shfl(incl, 63, 64);
      const long long mylast = tmask ? (long long)(pos + 31 - __clz(tmask)) : -1;
      const long long lmax = wave_incl_max(mylast);
      long long before = __shfl_up(lmax, 1, 64);
      if (l == 0) before = -1;
      if (before < prev_term) before = prev_term;
      const uint64_t ord0 = ord_base + (incl - cnt);
      unsigned long long bad = ~0ull;
      long long badlen = 0, endp = -1;
      {
        uint32_t m = tmask;
        long long prev = before;
        uint64_t o = ord0;
        while (m) {
          const int i = __ffs(m) - 1;
          m &= m - 1;
          const long long e = (long long)pos + i, s = prev + 1;
          prev = e;
          const uint64_t oo = o++;
          if (oo == nb) endp = e + 1;
          if (oo == 0 || oo > nb) continue;
          const long long L = e - s + 1;
          const uint32_t be = byte_of(w, i);
          if (L > 10 || (L == 10 && be > 1)) {
            bad = oo;
            badlen = L;
            break;
          }
        }
      }
      const unsigned long long wbad = wave_min_u64(bad);
      if (wbad != ~0ull) {  // binary.Uvarint overflow: n = -(bytes read)
        const unsigned long long bl = __ballot(bad == wbad);
        r.status = kV1ItemSize;
        r.a = wbad - 1;
        r.b = (unsigned long long)(-__shfl(badlen, __ffsll((long long)bl) - 1, 64));
        break;
      }
      const unsigned long long eb = __ballot(endp >= 0);
      if (eb) hend = __shfl(endp, __ffsll((long long)eb) - 1, 64);
      // CRC of this window's header bytes (bytes from hend on count as 0)
      uint32_t c = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        uint32_t b = byte_of(w, k);
        if (hend >= 0 && pos + k >= hend) b = 0;
        c = tab[(c ^ b) & 0xffu] ^ (c >> 8);
      }
#pragma unroll
      for (int lv = 0; lv < 6; lv++) {
        const int step = 1 << lv;
        const uint32_t o = __shfl(c, (l + step) & 63, 64);
        c = v1_gf_mul(c, cm[lv]) ^ (l + step < 64 ? o : 0u);
      }
      R = v1_gf_mul(R, x1024) ^ __shfl(c, 0, 64);
      covered = base + 1024;
      if (hend >= 0) break;
      ord_base += wtotal;
      const long long wl = __shfl(lmax, 63, 64);
      if (wl > prev_term) prev_term = wl;
    }
    if (r.status == kV1Ok && hend < 0) {
      if (jb.hbytes < jb.size) {  // (a varint longer than 10 bytes) past the staged bound
        r.status = kV1More;
      } else {  // the record ended first: n == 0
        r.status = kV1ItemSize;
        r.a = ord_base == 0 ? 0 : ord_base - 1;
        r.b = 0;
      }
    }
    if (r.status == kV1Ok) {
      const uint64_t m = (uint64_t)hend;
      const uint32_t rm = v1_gf_mul(R, v1_xpow8_inv((uint64_t)covered - m));  // drop the zero tail
      const uint32_t ncrc = ~(v1_gf_mul(0xFFFFFFFFu, v1_xpow8(m)) ^ rm);
      uint32_t w0[4];
      v1_load16(p, 0, 4, w0);
      if (ncrc != w0[0]) {
        r.status = kV1Crc;
        r.a = ncrc;
        r.b = w0[0];
      }
    }
    // ---- pass 1: item views and Unpack's bounds checks
    if (r.status == kV1Ok) {
      const uint64_t pend = 4 + (uint64_t)hend;  // packed = payload[pend:]
      const uint64_t max = (uint64_t)len - pend;
      const uint64_t vbase = jb.span_off + pend;
      if (nb == 0) {  // packed[0:0]: one empty item
        if (l == 0) {
          item_off[jb.item_base] = vbase;
          item_len[jb.item_base] = 0;
        }
      }
      ord_base = 0;
      prev_term = -1;
      unsigned long long carry = 0;
      for (int64_t base = 0; nb > 0 && base < hend; base += 1024) {
        const int64_t pos = base + 16ll * l;
        uint32_t w[4];
        v1_load16(h, pos, hend, w);
        const uint32_t tmask = v1_term_mask(w);
        const uint32_t cnt = __popc(tmask);
        const uint32_t incl = wave_incl_sum<uint32_t>(cnt);
        const uint32_t wtotal = __shfl(incl, 63, 64);
        const long long mylast = tmask ? (long long)(pos + 31 - __clz(tmask)) : -1;
        const long long lmax = wave_incl_max(mylast);
        long long before = __shfl_up(lmax, 1, 64);
        if (l == 0) before = -1;
        if (before < prev_term) before = prev_term;
        const uint64_t ord0 = ord_base + (incl - cnt);
        // two walks of the lane's terminators: value sum, then views
        unsigned long long lsum = 0, bad = ~0ull, ba = 0, bkind = 0;
        for (int walk = 0; walk < 2; walk++) {
          unsigned long long run = 0;
          if (walk == 1) {
            const unsigned long long inc = wave_incl_sum<unsigned long long>(lsum);
            run = carry + inc - lsum;
          }
          uint32_t m = tmask;
          long long prev = before;
          uint64_t o = ord0;
          while (m) {
            const int i = __ffs(m) - 1;
            m &= m - 1;
            const long long e = (long long)pos + i, s = prev + 1;
            prev = e;
            const uint64_t oo = o++;
            if (oo == 0 || oo > nb) continue;
            unsigned long long v = 0;
            for (long long q = s; q <= e; q++) {
              const uint32_t b = q >= (long long)pos ? byte_of(w, (int)(q - pos)) : (uint32_t)h[q];
              v |= (unsigned long long)(b & 0x7fu) << (7 * (q - s));
            }
            if (walk == 0) {
              lsum += v;
              continue;
            }
            const uint64_t it = oo - 1;
            const unsigned long long end = run + v;  // Go: prev+size in uint64 (wraps)
            if (bad == ~0ull) {
              if (it + 1 < nb && end > max) {
                bad = it;
                bkind = kV1Offset;
                ba = end;
              } else if (end < run || (it + 1 == nb && end > max)) {
                bad = it;  // Go panics slicing (or reads past the record)
                bkind = kV1Range;
              }
            }
            item_off[jb.item_base + it] = vbase + run;
            item_len[jb.item_base + it] = v;
            run = end;
          }
        }
        const unsigned long long wbad = wave_min_u64(bad);
        if (wbad != ~0ull) {
          const int src = __ffsll((long long)__ballot(bad == wbad)) - 1;
          r.status = (uint32_t)__shfl((int)bkind, src, 64);
          r.a = __shfl(ba, src, 64);
          r.b = max;
          break;
        }
        carry += wave_sum<unsigned long long>(lsum);
        ord_base += wtotal;
        const long long wl = __shfl(lmax, 63, 64);
        if (wl > prev_term) prev_term = wl;
      }
    }
    if (l == 0) res[j] = r;
  }
}

void launch_v1_unpack(const uint8_t *dstage, const V1Job *jobs, uint64_t njobs,
                      unsigned long long *item_off, unsigned long long *item_len, V1Res *res, hipStream_t st) {
  uint64_t g = (njobs + 3) / 4;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(k_v1_unpack, dim3((unsigned)g), dim3(256), 0, st, dstage, jobs, njobs, item_off, item_len,
                     res);
}

}  // namespace rio
