// Copy-pass machinery shared by the flate and zstd execution passes
// (k_flate_lz2, k_zstd_exec2): a 4 KiB LDS ring per wave, history older than
// the ring read back from the decode region in HBM. See k_flate_lz2.
#pragma once
#include "device_common.h"

namespace rio {

constexpr uint32_t kL2Ring = 4096, kL2Mask = kL2Ring - 1;
constexpr uint32_t kL2Span = 1536;                   // output bytes per batch at most
constexpr uint32_t kL2Near = kL2Ring - kL2Span - 16;  // bytes before the batch kept in the ring (the
                                                       // batch's zeroing may round up one dword)
#ifndef RIO_ABL_FAR
#define RIO_ABL_FAR 0
#endif
#ifndef RIO_L2_WAVES
#define RIO_L2_WAVES 20  // 5 per SIMD: k_flate_lz2 is register-allocated for that (RIO_LZ2_WPE)
#endif
constexpr int kL2Waves = RIO_L2_WAVES;                          // per CU (launch sizing)
static_assert(kL2Near >= kL2Span + 16 + 258, "HBM sources must be flushed two batches back");

__device__ __forceinline__ uint32_t tok_len(uint32_t t) {
  return (t >> 31) ? ((t >> 16) & 0xffu) + 3 : (t >> 24) & 3u;
}

__device__ __forceinline__ uint32_t pick4(const uint32_t (&a)[4], int k) {
  return k == 0 ? a[0] : k == 1 ? a[1] : k == 2 ? a[2] : a[3];
}

// Four copies at once (one per token slot; n[k] == 0: none): n[k] bytes from
// position s[k] to t[k] = B0 + p[k] (t - s >= n: no overlap), sources in HBM
// where bit k of glob is set (the decode region gw, or the literal area gl
// where bit k of litm is set -- zstd), else in the ring. The batch's ring bytes are zeroed first and
// every byte belongs to one token, so a token ORs its bytes into the
// destination dwords (an LDS atomic, in any order) -- no byte stores, no races
// with the neighbours sharing its end dwords. Source dwords are read aligned
// and funnel-shifted; each step issues every slot's loads before using any.
// kMask: the ring's size - 1 (k_flate_seg's rings are 8 KiB).
template <uint32_t kMask = kL2Mask>
__device__ __forceinline__ void l2_copy4(uint8_t *ring, const uint32_t *gw, const uint32_t (&s)[4], uint32_t B0,
                                         const uint32_t (&p)[4], const uint32_t (&n)[4], uint32_t glob,
                                         const uint32_t *gl = nullptr, uint32_t litm = 0) {
  uint32_t *rw = reinterpret_cast<uint32_t *>(ring);
#if RIO_ABL_FAR  // measurement-only builds: far sources read from the ring (wrong bytes; what their loads cost)
  glob = 0;
#endif
  // per slot (recomputed where used, to keep registers for occupancy): the
  // destination t = B0 + p, its dwords [t/4, (t+n+3)/4), and the source dword
  // under the first one, floor((s - t%4) / 4) (~0 for -1)
  for (uint32_t D = 0;; D += 4) {
    bool any = false;
    uint32_t w[4][5];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t t = B0 + p[k];
      const bool act = n[k] != 0 && (t >> 2) + D < (t + n[k] + 3) >> 2;
      any |= act;
      const uint32_t q = (s[k] >> 2) - ((s[k] & 3) < (t & 3) ? 1u : 0u) + D;
#pragma unroll
      for (int i = 0; i < 5; i++) w[k][i] = 0;
      if (act && ((glob >> k) & 1)) {
        // the decode region, or (bit k of litm) a literal area
        const uint8_t *g = reinterpret_cast<const uint8_t *>(((litm >> k) & 1) ? gl : gw);
        // dword -1 (a source at position < 3) only feeds bytes before the
        // destination, which are masked off: any dword will do (dword 0)
        w[k][0] = __hip_atomic_load(reinterpret_cast<const uint32_t *>(g + (q == 0xffffffffu ? 0u : q << 2)),
                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint8_t *g1 = g + ((q + 1) << 2);
#pragma unroll
        for (int i = 1; i < 5; i++)
          w[k][i] = __hip_atomic_load(reinterpret_cast<const uint32_t *>(g1 + 4 * (i - 1)), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
      } else if (act) {
#pragma unroll
        for (int i = 0; i < 5; i++) w[k][i] = rw[(q + i) & (kMask >> 2)];
      }
    }
    if (!__builtin_amdgcn_ballot_w64(any)) break;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t t = B0 + p[k], d0 = t >> 2, d1 = n[k] ? (t + n[k] + 3) >> 2 : d0;
      const uint32_t sh = 8 * ((s[k] - t) & 3);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t Dj = d0 + D + j;
        if (Dj < d1) {
          const uint32_t v = __builtin_amdgcn_alignbit(w[k][j + 1], w[k][j], sh);
          const uint32_t x0 = 4 * Dj;
          const uint32_t lo = t > x0 ? t - x0 : 0u;                         // 0..3
          const uint32_t hi = t + n[k] < x0 + 4 ? t + n[k] - x0 : 4u;      // 1..4
          const uint32_t m = (0xffffffffu << (8 * lo)) & (0xffffffffu >> (8 * (4 - hi)));
          atomicOr(&rw[Dj & (kMask >> 2)], v & m);
        }
      }
    }
  }
}

// One copy per lane, ring to ring (the pending rounds: sources inside the
// batch, every byte final by then): n bytes from position s to t (t - s >= n),
// the same aligned reads, funnel shifts and OR-writes as l2_copy4.
template <uint32_t kMask = kL2Mask>
__device__ __forceinline__ void l2_copy1_ring(uint8_t *ring, uint32_t s, uint32_t t, uint32_t n) {
  uint32_t *rw = reinterpret_cast<uint32_t *>(ring);
  const uint32_t d0 = t >> 2, d1 = n ? (t + n + 3) >> 2 : d0, sh = 8 * ((s - t) & 3);
  const uint32_t q0 = (s >> 2) - ((s & 3) < (t & 3) ? 1u : 0u);
  for (uint32_t D = 0; __builtin_amdgcn_ballot_w64(d0 + D < d1); D += 4) {
    uint32_t w[5];
#pragma unroll
    for (int i = 0; i < 5; i++) w[i] = rw[(q0 + D + i) & (kMask >> 2)];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t Dj = d0 + D + j;
      if (Dj < d1) {
        const uint32_t v = __builtin_amdgcn_alignbit(w[j + 1], w[j], sh);
        const uint32_t x0 = 4 * Dj;
        const uint32_t lo = t > x0 ? t - x0 : 0u;
        const uint32_t hi = t + n < x0 + 4 ? t + n - x0 : 4u;
        const uint32_t m = (0xffffffffu << (8 * lo)) & (0xffffffffu >> (8 * (4 - hi)));
        atomicOr(&rw[Dj & (kMask >> 2)], v & m);
      }
    }
  }
}

}  // namespace rio
