// The chunk CRC fold of k_crc (crc.hip) as device helpers, shared with the
// writer's fused chunk encoder (encode.hip): GF(2) products in the reflected
// CRC-32 representation, masking of a dword to the covered bytes, one row
// step of a lane's 4 dword streams through the bank-private LDS fold tables,
// and multiply-by-constant through the 4-byte multiply tables.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rio_internal.h"

#ifndef RIO_FOLD_XOR3
#define RIO_FOLD_XOR3 1
#endif

namespace rio {

__device__ __forceinline__ uint32_t gf_mul_dev(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 31; i >= 0; i--) {
    p ^= b & (0u - ((a >> i) & 1u));
    b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
  }
  return p;
}

// keep the bytes of dword v (at chunk offset off) that lie below chunk offset hi
__device__ __forceinline__ uint32_t mask_dword(uint32_t v, int off, int hi) {
  int keep = hi - off;
  keep = keep < 0 ? 0 : (keep > 4 ? 4 : keep);
  const uint32_t m = keep >= 4 ? 0xffffffffu : ((1u << (8 * keep)) - 1u);
  return v & m;
}

// one Horner step of the lane's 4 dword streams: 16 independent lookups in the
// lane's private table copies
// kAbs: the tables start at LDS address 0 (k_crc: dynamic LDS and no static
// LDS, checked at its start) -- the lookup address is the v_perm result itself
// (with a base pointer the compiler adds the dynamic-LDS base, 0, per lookup)
// The byte-row (v_perm) fold with its XORs as v_bitop3_b32 (3-input XOR): the
// state of stream k is s[k] ^ s2[k] (s2: the fourth lookup, not yet folded in),
// so a step is 4 permutes, 4 lookups and 2 XOR3s per dword -- the data XOR
// joins the previous step's last one. Callers start with s2 = 0 and take
// s ^ s2 at the end.
// sel: lookup j's v_perm selector (byte j of the data and of L, the table offset).
// With the 16 table copies banked (16 j + copy) mod 32, a ds_read_b32's 32-lane
// group put lanes l and l + 16 (one copy) on one bank: 2-way conflicts on every
// lookup (k_crc: 596 M conflict cycles of 1,163 M LDS cycles per C2 launch). A
// caller whose lanes 16-31 / 48-63 take lookup (j + 1) & 3 as their j-th
// (fold_sel) spreads the group over 32 banks; the XOR of the four is the same.
__device__ __forceinline__ uint32_t fold_sel(int j, uint32_t rot) {
  const uint32_t jj = ((uint32_t)j + rot) & 3u;
  return 0x0c0c0000u | (jj << 8) | (4u + jj);
}
template <bool kAbs = false>
__device__ __forceinline__ void fold_row3(const char *__restrict__ tab, uint32_t lb, uint4 v, uint32_t (&s)[4],
                                          uint32_t (&s2)[4], const uint32_t (&sel)[4]) {
  static_assert(kFoldPerm, "the byte-row layout");
  const uint32_t L = lb * 0x01010101u + 0xC0804000u;
  const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t d = __builtin_amdgcn_bitop3_b32(vv[k], s[k], s2[k], 0x96);
    uint32_t t[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t a = __builtin_amdgcn_perm(L, d, sel[j]);
      typedef const __attribute__((address_space(3))) uint32_t lds_u32;
      if constexpr (kAbs) t[j] = *(lds_u32 *)(uintptr_t)a;
      else t[j] = *reinterpret_cast<const uint32_t *>(tab + a);
    }
    s[k] = __builtin_amdgcn_bitop3_b32(t[0], t[1], t[2], 0x96);
    s2[k] = t[3];
  }
}
template <bool kAbs = false>
__device__ __forceinline__ void fold_row3(const char *__restrict__ tab, uint32_t lb, uint4 v, uint32_t (&s)[4],
                                          uint32_t (&s2)[4]) {
  const uint32_t sel[4] = {fold_sel(0, 0), fold_sel(1, 0), fold_sel(2, 0), fold_sel(3, 0)};
  fold_row3<kAbs>(tab, lb, v, s, s2, sel);
}

template <bool kAbs = false>
__device__ __forceinline__ void fold_row(const char *__restrict__ tab, uint32_t lb, uint4 v, uint32_t (&s)[4]) {
  if constexpr (kFoldPerm) {
    // lookup j's byte address (256 b + 64 j + lb): byte 1 = data byte j, byte 0 =
    // byte j of L = (lb, 64 + lb, 128 + lb, 192 + lb); bytes 2, 3 zero (selector 0x0c)
    const uint32_t L = lb * 0x01010101u + 0xC0804000u;
    const uint32_t d[4] = {v.x ^ s[0], v.y ^ s[1], v.z ^ s[2], v.w ^ s[3]};
    uint32_t t[4][4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t a = __builtin_amdgcn_perm(L, d[k], 0x0c0c0000u | ((uint32_t)j << 8) | (4u + (uint32_t)j));
        typedef const __attribute__((address_space(3))) uint32_t lds_u32;
        if constexpr (kAbs) t[k][j] = *(lds_u32 *)(uintptr_t)a;
        else t[k][j] = *reinterpret_cast<const uint32_t *>(tab + a);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) s[k] = t[k][0] ^ t[k][1] ^ t[k][2] ^ t[k][3];
    return;
  }
  const uint32_t d[4] = {v.x ^ s[0], v.y ^ s[1], v.z ^ s[2], v.w ^ s[3]};
  uint32_t t[4][4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t a = (((d[k] >> (8 * j)) & 0xffu) << kFoldShift) | lb;
      t[k][j] = *reinterpret_cast<const uint32_t *>(tab + j * (256 * 4 * kFoldCopies) + a);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; k++) s[k] = t[k][0] ^ t[k][1] ^ t[k][2] ^ t[k][3];
}

__device__ __forceinline__ uint32_t mul_const(const uint32_t *__restrict__ T, uint32_t v) {
  return T[v & 0xff] ^ T[256 + ((v >> 8) & 0xff)] ^ T[512 + ((v >> 16) & 0xff)] ^ T[768 + (v >> 24)];
}

}  // namespace rio
