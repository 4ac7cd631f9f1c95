// CDNA4 (gfx950) kernels of the recordio chunk layer: per-chunk header checks
// and the scans that enumerate blocks. Host orchestration in pipeline.cpp.
//
// Pipeline for one span of whole chunks (none codec):
//   chunk pass     per chunk: header fields, size check, the structural checks of
//                  ChunkScanner.Scan against the previous chunk (chunk.go:253-294,
//                  333-336); payload prefix ck_pay; block enumeration (index == 0)
//                  with a descriptor per block and its item count (first header
//                  varint). Three launches (k_chunk_tiles / _partials / _apply).
//   block scan     item slots per block.
//   k_parse        (blocks.hip) wave per block: magic handling, header parse,
//                  item views (parseChunksToItems, scannerv2.go:53-97, 363-388).
//   k_strad        (blocks.hip) gather of items that cross a chunk boundary.
//   k_crc          (crc.hip) CRC32 of every chunk (chunk.go:338-343).
//   k_resolve      (blocks.hip) the first event in file order (errors.Once).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "rio_internal.h"

namespace rio {

constexpr uint32_t kNoBlock = 0xffffffffu;

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

// (1024 threads: a 16-wave workgroup does not fit on a CU beside k_crc's 12
// waves, so with two contexts the next step's parse waits for the CRC pass's
// tail. Round 5 measured 4-wave workgroups, which let the whole parse run beside
// k_crc: 3.05 -> 3.37 ms per C2 step -- the two passes' concurrent HBM streams
// lose more than the overlap gains)
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

// Go 1.13 binary.Uvarint of the block's first payload bytes: the item count
// (parseChunksToItems, scannerv2.go:65), used to reserve item slots before the
// headers are parsed. 0 when it does not decode or cannot fit the block.
__device__ unsigned long long first_uvarint(const uint8_t *span, const DevBufs &d, uint64_t c0, uint32_t total,
                                            unsigned long long len) {
  uint64_t c = c0;
  uint32_t off = 0, csz = d.ck_size[c0];
  unsigned long long v = 0;
  for (int k = 0; k < 10 && (unsigned long long)k < len; k++) {
    while (off >= csz && c + 1 < c0 + total) {
      c++;
      off = 0;
      csz = d.ck_size[c];
    }
    if (off >= csz) return 0;
    const uint32_t b = span[c * kChunk + kChunkHdr + off];
    off++;
    v |= (unsigned long long)(b & 0x7f) << (7 * k);
    if (b < 0x80) {
      if (k == 9 && b > 1) return 0;
      return v <= len ? v : 0;
    }
  }
  return 0;
}

struct U64Out {
  unsigned long long *out;
  __device__ void operator()(uint64_t i, unsigned long long ex, unsigned long long) const { out[i] = ex; }
};
struct U64Load {
  const unsigned long long *in;
  __device__ unsigned long long operator()(uint64_t i) const { return in[i]; }
};

// ---------------------------------------------------------------- chunk pass
// The chunk headers and both per-chunk scans (payload prefix, block starts) in
// three launches. Thread t of a tile owns chunks base + 8t .. base + 8t + 7.
//   k_chunk_tiles    the headers (each thread's 8 and the one before them:
//                    chunk_meta checks against the predecessor), the per-chunk
//                    fields, the tile's sums of payload sizes and block starts;
//   k_chunk_partials the two columns of tile sums scanned (one workgroup);
//   k_chunk_apply    ck_pay, ck_block and the block descriptors (FlagOut).
__global__ void __launch_bounds__(kScanThreads) k_chunk_tiles(const uint8_t *__restrict__ span, uint64_t nchunks,
                                                              DevBufs d, unsigned long long *psize,
                                                              unsigned long long *pflag) {
  __shared__ unsigned long long lds[17];
  const uint64_t i0 = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  uint4 a[kScanItems], b[kScanItems], pa = make_uint4(0, 0, 0, 0), pb = make_uint4(0, 0, 0, 0);
  if (i0 > 0 && i0 < nchunks) {
    const uint4 *h = reinterpret_cast<const uint4 *>(span + (i0 - 1) * kChunk);
    pa = h[0];
    pb = h[1];
  }
#pragma unroll
  for (int k = 0; k < kScanItems; k++)
    if (i0 + k < nchunks) {
      const uint4 *h = reinterpret_cast<const uint4 *>(span + (i0 + k) * kChunk);
      a[k] = h[0];  // magic lo, hi, crc, flag
      b[k] = h[1];  // size, total, index, data
    }
  unsigned long long ss = 0, sf = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    const uint64_t i = i0 + k;
    if (i >= nchunks) break;
    const ChunkMeta m = chunk_meta(a[k].x, a[k].y, b[k].x, b[k].y, b[k].z, i > 0, pa.x, pa.y, pb.y, pb.z);
    d.ck_size[i] = b[k].x;
    d.ck_total[i] = b[k].y;
    d.ck_index[i] = b[k].z;
    d.ck_info[i] = m.info;
    d.ck_ssz[i] = 0;  // straddler slots, filled by the parse
    if (m.err) atomicMin(&d.ctl->first_chunk_err, (unsigned long long)i);
    ss += b[k].x > (uint32_t)kMaxPayload ? 0ull : (unsigned long long)b[k].x;
    sf += b[k].z == 0 ? 1ull : 0ull;
    pa = a[k];
    pb = b[k];
  }
  unsigned long long ts, tf;
  block_excl_scan(ss, &ts, lds);
  block_excl_scan(sf, &tf, lds);
  if (threadIdx.x == 0) {
    psize[blockIdx.x] = ts;
    pflag[blockIdx.x] = tf;
  }
}

__global__ void __launch_bounds__(1024) k_chunk_partials(uint64_t nchunks, unsigned long long *psize,
                                                         unsigned long long *pflag, unsigned long long *pay_total,
                                                         unsigned long long *nblocks) {
  __shared__ unsigned long long lds[17];
  const uint64_t ntiles = (nchunks + kScanTile - 1) / kScanTile;
  unsigned long long cs = 0, cf = 0;
  for (uint64_t base = 0; base < ntiles; base += blockDim.x) {
    const uint64_t i = base + threadIdx.x;
    const bool in = i < ntiles;
    unsigned long long ts, tf;
    const unsigned long long es = block_excl_scan(in ? psize[i] : 0ull, &ts, lds);
    const unsigned long long ef = block_excl_scan(in ? pflag[i] : 0ull, &tf, lds);
    if (in) {
      psize[i] = cs + es;
      pflag[i] = cf + ef;
    }
    cs += ts;
    cf += tf;
  }
  if (threadIdx.x == 0) {
    *pay_total = cs;  // ck_pay[nchunks]
    *nblocks = cf;
  }
}

__global__ void __launch_bounds__(kScanThreads) k_chunk_apply(const uint8_t *__restrict__ span, uint64_t nchunks,
                                                              DevBufs d, int32_t codec,
                                                              const unsigned long long *psize,
                                                              const unsigned long long *pflag) {
  __shared__ unsigned long long lds[17];
  const uint64_t i0 = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  uint32_t sz[kScanItems], st[kScanItems];
  unsigned long long ss = 0, sf = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    const bool in = i0 + k < nchunks;
    const uint32_t s = in ? d.ck_size[i0 + k] : 0u;
    sz[k] = s > (uint32_t)kMaxPayload ? 0u : s;
    st[k] = in && d.ck_index[i0 + k] == 0 ? 1u : 0u;
    ss += sz[k];
    sf += st[k];
  }
  unsigned long long ts, tf;
  unsigned long long es = block_excl_scan(ss, &ts, lds) + psize[blockIdx.x];
  unsigned long long ef = block_excl_scan(sf, &tf, lds) + pflag[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    const uint64_t i = i0 + k;
    if (i >= nchunks) break;
    d.ck_pay[i] = es;
    d.ck_block[i] = (ef + st[k] == 0) ? kNoBlock : (uint32_t)(ef + st[k] - 1);  // chunks before any start: none
    if (st[k]) {  // a block starts here: its descriptor (block ef)
      const uint32_t total = d.ck_total[i];
      const uint32_t cls = d.ck_info[i] & 0xffu;
      unsigned long long meta = (unsigned long long)total | ((unsigned long long)cls << kMetaClsShift);
      unsigned long long len = 0, nres = 0;
      if (total != 0 && i + total <= nchunks) {
        meta |= kMetaComplete;
        // the block's payload bytes (its chunks' sizes, as the payload prefix
        // counts them) and whether every chunk but the last is full
        bool regular = true, overlap = false;
        for (uint32_t q = 0; q < total; q++) {
          const uint32_t s = d.ck_size[i + q];
          const uint32_t v = s > (uint32_t)kMaxPayload ? 0u : s;
          len += v;
          if (q + 1 < total && v != (uint32_t)kMaxPayload) regular = false;
          overlap = overlap || (q > 0 && d.ck_index[i + q] == 0);
        }
        // Another block starting inside this one's chunks (a `total` rewritten
        // with its CRC): a chunk error comes before this block's end, so it is
        // never delivered, but its decode must not write into the other
        // block's regions (token slots, straddlers): it decodes as empty.
        if (overlap) len = 0, regular = false;
        if (regular) meta |= kMetaRegular;
        if (codec == RIO_CODEC_NONE && len) nres = first_uvarint(span, d, i, total, len);
      }
      d.blk_c0[ef] = i;
      d.blk_meta[ef] = meta;
      d.blk_len[ef] = len;
      d.blk_nitems[ef] = nres;
    }
    es += sz[k];
    ef += st[k];
  }
}

// ---------------------------------------------------------------- launchers
static inline unsigned grid_for(uint64_t n, unsigned per, unsigned cap) {
  uint64_t g = (n + per - 1) / per;
  if (g < 1) g = 1;
  return (unsigned)(g > cap ? cap : g);
}

// the control words a pipeline run reduces into, and the block counters, reset
// in one launch (min-reduced words to ~0, counters to 0)
__global__ void k_reset(Ctl *ctl, unsigned long long *nblocks) {
  const int t = threadIdx.x;
  if (t < 4) (&ctl->first_chunk_err)[t] = kNone;   // first_chunk_err .. first_incomplete
  else if (t < 8) (&ctl->out_overflow)[t - 4] = 0;  // out_overflow, dec_need, pad[2]
  else if (t < 10) (&ctl->flstat_esc)[t - 8] = 0;   // flstat_esc, n_retry
  else if (t < 14) ctl->zprof[t - 10] = 0;
  else if (t == 14) ctl->zjob_n = 0;
  else if (t < 17) nblocks[t - 15] = 0;
  else if (t == 17) ctl->seg_used = 0;
  else if (t == 18) ctl->seg_blocks = 0;
  else if (t < 23) ctl->zx[t - 19] = 0;
  else if (t == 23) ctl->tok_need = 0;
}

void launch_reset(const DevBufs &d, unsigned long long *nblocks_dev, hipStream_t st) {
  hipLaunchKernelGGL(k_reset, dim3(1), dim3(64), 0, st, d.ctl, nblocks_dev);
}

void launch_chunk_pass(const uint8_t *span, uint64_t nchunks, const DevBufs &d, unsigned long long *nblocks_dev,
                       int32_t codec, hipStream_t st) {
  const uint64_t tiles = (nchunks + kScanTile - 1) / kScanTile;
  const unsigned g = (unsigned)(tiles ? tiles : 1);
  unsigned long long *psize = d.scan_tmp, *pflag = d.scan_tmp + g;
  hipLaunchKernelGGL(k_chunk_tiles, dim3(g), dim3(kScanThreads), 0, st, span, nchunks, d, psize, pflag);
  hipLaunchKernelGGL(k_chunk_partials, dim3(1), dim3(1024), 0, st, nchunks, psize, pflag, d.ck_pay + nchunks,
                     nblocks_dev);
  hipLaunchKernelGGL(k_chunk_apply, dim3(g), dim3(kScanThreads), 0, st, span, nchunks, d, codec, psize, pflag);
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

// exclusive scan of a per-chunk u64 array into out (n + 1 entries)
void launch_chunk_scan(const unsigned long long *in, unsigned long long *out, unsigned long long *tmp, uint64_t n,
                       hipStream_t st) {
  scan(U64Load{in}, U64Out{out}, nullptr, n, n, tmp, nullptr, out, st);
}

// exclusive scan of a per-block u64 array into out (n + 1 entries), n on device
void launch_block_scan(const unsigned long long *in, unsigned long long *out, unsigned long long *tmp,
                       const unsigned long long *nblocks_dev, uint64_t max_blocks, hipStream_t st) {
  scan(U64Load{in}, U64Out{out}, nblocks_dev, 0, max_blocks, tmp, nullptr, out, st);
}

}  // namespace rio
