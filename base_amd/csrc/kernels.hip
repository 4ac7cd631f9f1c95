// CDNA4 (gfx950) kernels of the recordio scan path: chunk layer, block
// enumeration, header parse, fused CRC32 + record copy, and the first-error
// resolve. Host orchestration in pipeline.cpp.
//
// Pipeline for one span of whole chunks:
//   k_chunk_meta   per chunk: header fields, size check, the structural checks of
//                  ChunkScanner.Scan against the previous chunk (chunk.go:253-294,
//                  333-336), block-start flags.
//   scans          block enumeration (index == 0) and the payload prefix ck_pay.
//   k_crc_copy     wave per chunk: CRC32-IEEE over [12, 28+size) (chunk.go:338-343)
//                  fused with idTransform (registry.go:31-39): chunk c's payload
//                  lands at records + ck_pay[c], so a block's bytes are contiguous
//                  (the reference's rawItems.bytes) and no copy waits on parsing.
//   k_block_parse  wave per block: block magic handling (scannerv2.go:374-387) and
//                  the varint header of parseChunksToItems (scannerv2.go:53-97).
//   scan           item bases per block.
//   k_items        wave per block: cumSize -> item_end (scannerv2.go:83-91).
//   k_resolve      the first event in file order (errors.Once) -> summary.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "rio_internal.h"

namespace rio {

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

constexpr uint32_t kNoBlock = 0xffffffffu;

// ---------------------------------------------------------------- k_chunk_meta
__global__ void __launch_bounds__(256) k_chunk_meta(const uint8_t *__restrict__ span, uint64_t nchunks,
                                                    DevBufs d) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks; c += stride) {
    const uint32_t *h = reinterpret_cast<const uint32_t *>(span + c * kChunk);
    const uint4 a = *reinterpret_cast<const uint4 *>(h);      // magic lo, hi, crc, flag
    const uint4 b = *reinterpret_cast<const uint4 *>(h + 4);  // size, total, index, data
    const uint32_t size = b.x, total = b.y, index = b.z;
    const uint32_t cls = magic_class(a.x, a.y);
    uint32_t err = kCkOk;
    if (size > (uint32_t)kMaxPayload) {
      err = kCkSize;
    } else {
      bool prev_end = true;  // the span starts on a block boundary
      uint32_t plo = 0, phi = 0, ptotal = 0, pindex = 0;
      if (c > 0) {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(span + (c - 1) * kChunk);
        const uint4 pa = *reinterpret_cast<const uint4 *>(p);
        const uint4 pb = *reinterpret_cast<const uint4 *>(p + 4);
        plo = pa.x;
        phi = pa.y;
        ptotal = pb.y;
        pindex = pb.z;
        prev_end = (int64_t)pindex == (int64_t)ptotal - 1;
      }
      if (prev_end) {
        if (index != 0) err = kCkIndex;
      } else if (a.x != plo || a.y != phi) {
        err = kCkMagicChanged;
      } else if ((uint64_t)index != (uint64_t)pindex + 1) {
        err = kCkIndex;
      } else if (total != ptotal) {
        err = kCkTotal;
      }
    }
    d.ck_size[c] = size;
    d.ck_total[c] = total;
    d.ck_index[c] = index;
    d.ck_info[c] = cls | (err << 8);
    if (err != kCkOk) atomicMin(&d.ctl->first_chunk_err, (unsigned long long)c);
  }
}

// ---------------------------------------------------------------- scans
// Exclusive scan over n values (n read from *n_dev when non-null, else n_host),
// tiles of 2048 (256 threads x 8). Value and output are functors.
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

// block-wide exclusive scan of one value per thread (blockDim multiple of 64, <= 1024)
__device__ unsigned long long block_excl_scan(unsigned long long v, unsigned long long *total,
                                              unsigned long long *lds /* >= 17 */) {
  const int w = threadIdx.x >> 6, l = lane_id(), nw = blockDim.x >> 6;
  const unsigned long long inc = wave_incl_sum<unsigned long long>(v);
  if (l == 63) lds[w] = inc;
  __syncthreads();
  if (w == 0) {
    const unsigned long long s = (l < nw) ? lds[l] : 0;
    const unsigned long long si = wave_incl_sum<unsigned long long>(s);
    if (l < nw) lds[l] = si - s;
    if (l == nw - 1) lds[16] = si;
  }
  __syncthreads();
  const unsigned long long r = inc - v + lds[w];
  *total = lds[16];
  __syncthreads();
  return r;
}

template <class F>
__global__ void __launch_bounds__(kScanThreads) k_scan_reduce(F f, const unsigned long long *n_dev,
                                                              uint64_t n_host, unsigned long long *partial) {
  __shared__ unsigned long long lds[17];
  const uint64_t n = n_dev ? *n_dev : n_host;
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  if (base >= n) return;
  unsigned long long s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    const uint64_t i = base + threadIdx.x + (uint64_t)kScanThreads * k;
    if (i < n) s += f(i);
  }
  unsigned long long tot;
  block_excl_scan(s, &tot, lds);
  if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(1024) k_scan_partials(const unsigned long long *n_dev, uint64_t n_host,
                                                        unsigned long long *partial,
                                                        unsigned long long *total_out,
                                                        unsigned long long *total_at /* out[n] */) {
  __shared__ unsigned long long lds[17];
  const uint64_t n = n_dev ? *n_dev : n_host;
  const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
  unsigned long long carry = 0;
  for (uint64_t base = 0; base < ntiles; base += blockDim.x) {
    const uint64_t i = base + threadIdx.x;
    const unsigned long long v = (i < ntiles) ? partial[i] : 0;
    unsigned long long tot;
    const unsigned long long ex = block_excl_scan(v, &tot, lds);
    if (i < ntiles) partial[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    if (total_out) *total_out = carry;
    if (total_at) total_at[n] = carry;
  }
}

template <class F, class O>
__global__ void __launch_bounds__(kScanThreads) k_scan_apply(F f, O o, const unsigned long long *n_dev,
                                                             uint64_t n_host, const unsigned long long *partial) {
  __shared__ unsigned long long lds[17];
  const uint64_t n = n_dev ? *n_dev : n_host;
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  if (base >= n) return;
  const uint64_t i0 = base + (uint64_t)threadIdx.x * kScanItems;
  unsigned long long v[kScanItems];
  unsigned long long s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    v[k] = (i0 + k < n) ? f(i0 + k) : 0;
    s += v[k];
  }
  unsigned long long tot;
  unsigned long long ex = block_excl_scan(s, &tot, lds) + partial[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    if (i0 + k < n) o(i0 + k, ex, v[k]);
    ex += v[k];
  }
}

struct FlagLoad {  // block starts: index == 0
  const uint32_t *ck_index;
  __device__ unsigned long long operator()(uint64_t i) const { return ck_index[i] == 0 ? 1ull : 0ull; }
};
struct FlagOut {
  unsigned long long *blk_c0;
  uint32_t *ck_block;
  __device__ void operator()(uint64_t i, unsigned long long ex, unsigned long long v) const {
    if (v) blk_c0[ex] = i;
    ck_block[i] = (ex + v == 0) ? kNoBlock : (uint32_t)(ex + v - 1);  // chunks before any start: none
  }
};
struct SizeLoad {
  const uint32_t *ck_size;
  __device__ unsigned long long operator()(uint64_t i) const {
    const uint32_t s = ck_size[i];
    return s > (uint32_t)kMaxPayload ? 0ull : (unsigned long long)s;
  }
};
struct U64Out {
  unsigned long long *out;
  __device__ void operator()(uint64_t i, unsigned long long ex, unsigned long long) const { out[i] = ex; }
};
struct U64Load {
  const unsigned long long *in;
  __device__ unsigned long long operator()(uint64_t i) const { return in[i]; }
};

// ---------------------------------------------------------------- launchers
static inline unsigned grid_for(uint64_t n, unsigned per, unsigned cap) {
  uint64_t g = (n + per - 1) / per;
  if (g < 1) g = 1;
  return (unsigned)(g > cap ? cap : g);
}

void launch_chunk_meta(const uint8_t *span, uint64_t nchunks, const DevBufs &d, hipStream_t st) {
  hipLaunchKernelGGL(k_chunk_meta, dim3(grid_for(nchunks, 256, 4096)), dim3(256), 0, st, span, nchunks, d);
}

template <class F, class O>
static void scan(F f, O o, const unsigned long long *n_dev, uint64_t n_host, uint64_t n_max,
                 unsigned long long *partial, unsigned long long *total_out, unsigned long long *total_at,
                 hipStream_t st) {
  const unsigned tiles = (unsigned)((n_max + kScanTile - 1) / kScanTile);
  const unsigned g = tiles ? tiles : 1;
  hipLaunchKernelGGL(k_scan_reduce<F>, dim3(g), dim3(kScanThreads), 0, st, f, n_dev, n_host, partial);
  hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(1024), 0, st, n_dev, n_host, partial, total_out, total_at);
  hipLaunchKernelGGL((k_scan_apply<F, O>), dim3(g), dim3(kScanThreads), 0, st, f, o, n_dev, n_host, partial);
}

void launch_chunk_scans(uint64_t nchunks, const DevBufs &d, unsigned long long *nblocks_dev, hipStream_t st) {
  scan(FlagLoad{d.ck_index}, FlagOut{d.blk_c0, d.ck_block}, nullptr, nchunks, nchunks, d.scan_tmp, nblocks_dev,
       nullptr, st);
  scan(SizeLoad{d.ck_size}, U64Out{d.ck_pay}, nullptr, nchunks, nchunks, d.scan_tmp, nullptr, d.ck_pay, st);
}

// exclusive scan of a per-block u64 array into out (n + 1 entries), n on device
void launch_block_scan(const unsigned long long *in, unsigned long long *out, unsigned long long *tmp,
                       const unsigned long long *nblocks_dev, uint64_t max_blocks, hipStream_t st) {
  scan(U64Load{in}, U64Out{out}, nblocks_dev, 0, max_blocks, tmp, nullptr, out, st);
}

}  // namespace rio
