// Chunk CRC32-IEEE verify (readChunk, recordio/internal/chunk.go:338-343) at
// HBM read speed, no carry-less multiply.
//
// One wave per 32 KiB chunk, 16 waves per workgroup, one workgroup per CU.
// Lane t loads the 16-byte units at chunk offsets 1024*i + 16*t (i = 0..31): every
// load instruction is 1 KiB contiguous. Each of the lane's 4 dwords (k = 0..3)
// is its own CRC stream with one dword per 1 KiB row; the 1020-byte gap to the
// stream's next dword is folded into the tables, so one step is
//   S_k <- fold0[b0] ^ fold1[b1] ^ fold2[b2] ^ fold3[b3],  b = bytes of (u_k ^ S_k),
//   fold_j[b] = R(b || 0^(1023-j))     (R = raw CRC: zero init, no final xor).
// Only 4 fold tables exist, so each is replicated 32x in LDS (128 KiB): lane l
// reads copy l & 31 and every ds_read_b32 is bank-conflict free.
// After row 31, stream (t, k) holds R(message) * x^(8(16t + 4k)); the lane
// combines its streams with x^-32 (Horner), a 6-level shuffle tree with
// x^-(128*2^l) combines the lanes (multiply-by-constant = 4 byte lookups).
// Bytes outside [12, 28+size) are zeroed, so V = R(0^12 || covered || 0^pad) and
// crc = ~(~0 * x^(8(16+size)) ^ V * x^(-8 pad)).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "rio_internal.h"

namespace rio {

constexpr int kCrcWaves = 16;  // waves per workgroup (one workgroup per CU: 156 KiB LDS)

__device__ __forceinline__ uint32_t gf_mul_dev(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 31; i >= 0; i--) {
    p ^= b & (0u - ((a >> i) & 1u));
    b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
  }
  return p;
}

__device__ __forceinline__ uint32_t mask_dword(uint32_t v, int off, int hi) {
  // keep bytes with chunk offset < hi
  if (off + 4 <= hi) return v;
  if (off >= hi) return 0u;
  return v & (0xffffffffu >> (8 * (off + 4 - hi)));
}

// one Horner step of a dword stream: lookups in the lane's private table copies
__device__ __forceinline__ uint32_t fold_step(const char *__restrict__ tab, uint32_t lb, uint32_t d) {
  const uint32_t a0 = ((d & 0xffu) << 7) | lb;
  const uint32_t a1 = (((d >> 8) & 0xffu) << 7) | lb;
  const uint32_t a2 = (((d >> 16) & 0xffu) << 7) | lb;
  const uint32_t a3 = ((d >> 24) << 7) | lb;
  return *reinterpret_cast<const uint32_t *>(tab + a0) ^ *reinterpret_cast<const uint32_t *>(tab + 32768 + a1) ^
         *reinterpret_cast<const uint32_t *>(tab + 65536 + a2) ^ *reinterpret_cast<const uint32_t *>(tab + 98304 + a3);
}

__device__ __forceinline__ uint32_t mul_const(const uint32_t *__restrict__ T, uint32_t v) {
  return T[v & 0xff] ^ T[256 + ((v >> 8) & 0xff)] ^ T[512 + ((v >> 16) & 0xff)] ^ T[768 + (v >> 24)];
}

__global__ void __launch_bounds__(64 * kCrcWaves) k_crc(const uint8_t *__restrict__ span, uint64_t nchunks,
                                                       DevBufs d, CrcArgs ca) {
  __shared__ __attribute__((aligned(16))) uint32_t s_fold[kFoldWords];
  __shared__ __attribute__((aligned(16))) uint32_t s_mul[kMulTables * 1024];
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(d.crc_fold);
    uint4 *dst = reinterpret_cast<uint4 *>(s_fold);
    for (int i = threadIdx.x; i < kFoldWords / 4; i += blockDim.x) dst[i] = src[i];
    for (int i = threadIdx.x; i < kMulTables * 1024; i += blockDim.x) s_mul[i] = d.crc_mul[i];
  }
  __syncthreads();
  const int l = lane_id();
  const uint32_t lb = (uint32_t)(l & 31) << 2;
  const char *tab = reinterpret_cast<const char *>(s_fold);
  const bool fold = !(ca.flags & 1);
  const uint64_t wave = (uint64_t)blockIdx.x * kCrcWaves + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kCrcWaves;
  for (uint64_t c = wave; c < nchunks; c += nwaves) {
    const uint8_t *ck = span + c * kChunk;
    const uint32_t size = d.ck_size[c];
    if (size > (uint32_t)kMaxPayload) continue;  // "Invalid chunk size": no CRC
    const int end = kChunkHdr + (int)size;
    const bool full = (size == (uint32_t)kMaxPayload);
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    const uint4 *row = reinterpret_cast<const uint4 *>(ck) + l;
#pragma unroll 8
    for (int i = 0; i < 32; i++) {
      uint4 u = row[64 * i];
      if (i == 0 && l == 0) {  // magic[0:8] and crc[8:12] are not covered
        u.x = 0;
        u.y = 0;
        u.z = 0;
      }
      if (!full) {
        const int o = 1024 * i + 16 * l;
        u.x = mask_dword(u.x, o, end);
        u.y = mask_dword(u.y, o + 4, end);
        u.z = mask_dword(u.z, o + 8, end);
        u.w = mask_dword(u.w, o + 12, end);
      }
      if (fold) {
        s0 = fold_step(tab, lb, u.x ^ s0);
        s1 = fold_step(tab, lb, u.y ^ s1);
        s2 = fold_step(tab, lb, u.z ^ s2);
        s3 = fold_step(tab, lb, u.w ^ s3);
      } else {  // ablation: keep the loads live
        s0 ^= u.x;
        s1 ^= u.y;
        s2 ^= u.z;
        s3 ^= u.w;
      }
    }
    // lane: V_t = s0 + s1 x^-32 + s2 x^-64 + s3 x^-96
    uint32_t v = mul_const(s_mul, s3) ^ s2;
    v = mul_const(s_mul, v) ^ s1;
    v = mul_const(s_mul, v) ^ s0;
    // lanes: V = sum_t V_t x^-128t
#pragma unroll
    for (int lv = 0; lv < 6; lv++) {
      const uint32_t m = mul_const(s_mul + (lv + 1) * 1024, v);
      const int step = 1 << lv;
      const uint32_t o = __shfl(m, (l + step) & 63, 64);
      v ^= (l + step < 64) ? o : 0u;
    }
    if (l == 0) {
      const uint32_t t = full ? v : gf_mul_dev(v, d.crc_fix_b[size]);
      const uint32_t crc = ~(d.crc_fix_a[size] ^ t);
      d.ck_crc[c] = crc;
      const uint32_t stored = *reinterpret_cast<const uint32_t *>(ck + 8);
      if (crc != stored) atomicMin(&d.ctl->first_crc_err, (unsigned long long)c);
    }
  }
}

void launch_crc(const uint8_t *span, uint64_t nchunks, const DevBufs &d, const CrcArgs &ca, int ncu,
                hipStream_t st) {
  uint64_t g = (nchunks + kCrcWaves - 1) / kCrcWaves;
  const uint64_t cap = (uint64_t)(ncu > 0 ? ncu : 256);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(k_crc, dim3((unsigned)g), dim3(64 * kCrcWaves), 0, st, span, nchunks, d, ca);
}

}  // namespace rio
