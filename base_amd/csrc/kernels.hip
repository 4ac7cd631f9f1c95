// CDNA4 (gfx950) kernels of the recordio scan path, none codec + shared stages.
//
// Pipeline for one span of chunks (host orchestration in pipeline.cpp):
//   k_chunk_meta   per chunk: header parse, size check, the structural checks of
//                  ChunkScanner.Scan against the previous chunk (chunk.go:253-294,
//                  333-336), block-start flags.
//   scans          block enumeration (index==0 flags) and payload prefix sums.
//   k_block_parse  wave per block: block-level magic handling (scannerv2.go:
//                  374-387) and the varint header of parseChunksToItems
//                  (scannerv2.go:53-97): item count, header length, record bytes.
//   scans          item/record bases per block.
//   k_items        wave per block: cumSize -> item_end (scannerv2.go:83-91).
//   k_crc_copy     wave per chunk: CRC32-IEEE over bytes [12, 28+size) of the chunk
//                  (chunk.go:338-343) fused with the idTransform copy of the payload
//                  into the records buffer (registry.go:31-39), header bytes skipped.
//   k_resolve      first event in file order (errors.Once semantics) -> summary.
#include <hip/hip_runtime.h>
#include <stdint.h>

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

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// ---------------------------------------------------------------- k_chunk_meta
__global__ void __launch_bounds__(256) k_chunk_meta(const uint8_t *__restrict__ span, uint64_t nchunks,
                                                    DevBufs d) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks; c += stride) {
    const uint32_t *h = reinterpret_cast<const uint32_t *>(span + c * kChunk);
    uint4 a = *reinterpret_cast<const uint4 *>(h);      // magic lo, hi, crc, flag
    uint4 b = *reinterpret_cast<const uint4 *>(h + 4);  // size, total, index, data
    uint32_t size = b.x, total = b.y, index = b.z;
    uint32_t cls = magic_class(a.x, a.y);
    uint32_t err = kCkOk;
    if (size > (uint32_t)kMaxPayload) {
      err = kCkSize;
    } else {
      bool prev_end = true;
      uint32_t plo = 0, phi = 0, ptotal = 0, pindex = 0;
      if (c > 0) {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(span + (c - 1) * kChunk);
        uint4 pa = *reinterpret_cast<const uint4 *>(p);
        uint4 pb = *reinterpret_cast<const uint4 *>(p + 4);
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

__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    unsigned long long t = __shfl_up(v, o, 64);
    if (l >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide exclusive scan of one value per thread (blockDim multiple of 64, <= 1024)
__device__ unsigned long long block_excl_scan(unsigned long long v, unsigned long long *total,
                                              unsigned long long *lds /* >= 16 */) {
  const int w = threadIdx.x >> 6, l = lane_id(), nw = blockDim.x >> 6;
  unsigned long long inc = wave_incl_scan(v);
  if (l == 63) lds[w] = inc;
  __syncthreads();
  if (w == 0) {
    unsigned long long s = (l < nw) ? lds[l] : 0;
    unsigned long long si = wave_incl_scan(s);
    if (l < nw) lds[l] = si - s;
    if (l == nw - 1) lds[16] = si;
  }
  __syncthreads();
  unsigned long long r = inc - v + lds[w];
  *total = lds[16];
  __syncthreads();
  return r;
}

template <class F>
__global__ void __launch_bounds__(kScanThreads) k_scan_reduce(F f, const unsigned long long *n_dev,
                                                              uint64_t n_host,
                                                              unsigned long long *partial) {
  __shared__ unsigned long long lds[17];
  const uint64_t n = n_dev ? *n_dev : n_host;
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  if (base >= n) return;
  unsigned long long s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    uint64_t i = base + threadIdx.x + (uint64_t)kScanThreads * k;
    if (i < n) s += f(i);
  }
  unsigned long long tot;
  block_excl_scan(s, &tot, lds);
  if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(1024) k_scan_partials(const unsigned long long *n_dev, uint64_t n_host,
                                                        unsigned long long *partial,
                                                        unsigned long long *total_out) {
  __shared__ unsigned long long lds[17];
  const uint64_t n = n_dev ? *n_dev : n_host;
  const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
  unsigned long long carry = 0;
  for (uint64_t base = 0; base < ntiles; base += blockDim.x) {
    uint64_t i = base + threadIdx.x;
    unsigned long long v = (i < ntiles) ? partial[i] : 0;
    unsigned long long tot;
    unsigned long long ex = block_excl_scan(v, &tot, lds);
    if (i < ntiles) partial[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && total_out) *total_out = carry;
}

template <class F, class O>
__global__ void __launch_bounds__(kScanThreads) k_scan_apply(F f, O o, const unsigned long long *n_dev,
                                                             uint64_t n_host,
                                                             const unsigned long long *partial) {
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
    ck_block[i] = (uint32_t)(ex + v - 1);
  }
};
struct SizeLoad {
  const uint32_t *ck_size;
  __device__ unsigned long long operator()(uint64_t i) const {
    uint32_t s = ck_size[i];
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

// ---------------------------------------------------------------- varint parse
// Byte source of one block's (untransformed) payload: either the chunk payloads
// in the span (none codec) or one contiguous decompressed buffer.
struct Payload {
  const uint8_t *span;      // chunked: span base
  const uint32_t *ck_size;  // chunked: payload sizes
  uint64_t c0;              // chunked: first chunk
  uint64_t nseg;            // number of segments
  const uint8_t *contig;    // contiguous payload (nseg == 1) when non-null
  uint64_t contig_len;
  __device__ __forceinline__ void seg(uint64_t k, const uint8_t *&p, uint64_t &len) const {
    if (contig) {
      p = contig;
      len = contig_len;
    } else {
      p = span + (c0 + k) * kChunk + kChunkHdr;
      uint32_t s = ck_size[c0 + k];
      len = s > (uint32_t)kMaxPayload ? 0 : s;
    }
  }
};

struct VarintResult {
  int status;           // 0 ok, 1 truncated/overflow
  int64_t n;            // Go's n for the failing varint
  uint64_t count;       // varints completed
  uint64_t end_pos;     // logical position after the last needed varint
  uint64_t first_val;   // value of the first varint decoded (the item count in phase A)
  unsigned long long sum;
  int range_flag;
};

// Decode `need` consecutive uvarints (Go 1.13 binary.Uvarint semantics) starting
// at logical position `start` of the payload, one byte per lane per window.
// WRITE: also store item_end[item_base + k] = rec_base + running sum.
template <bool WRITE>
__device__ VarintResult parse_varints(const Payload &pl, uint64_t start, uint64_t need,
                                      uint64_t payload_len, unsigned long long *item_end,
                                      uint64_t item_base, uint64_t item_cap,
                                      unsigned long long rec_base, unsigned long long *overflow) {
  const int l = lane_id();
  const unsigned long long lt_mask = (l == 0) ? 0ull : (~0ull >> (64 - l));
  VarintResult r;
  r.status = 0;
  r.n = 0;
  r.count = 0;
  r.end_pos = start;
  r.first_val = 0;
  r.sum = 0;
  r.range_flag = 0;
  if (need == 0) return r;
  uint64_t carry_len = 0;
  unsigned long long carry_val = 0;
  uint64_t seg_lo = 0;
  for (uint64_t k = 0; k < pl.nseg; k++) {
    const uint8_t *p;
    uint64_t len;
    pl.seg(k, p, len);
    if (seg_lo + len <= start) {
      seg_lo += len;
      continue;
    }
    uint64_t x = start > seg_lo ? start - seg_lo : 0;
    for (; x < len; x += 64) {
      const bool valid = x + l < len;
      const uint32_t b = valid ? p[x + l] : 0u;
      const bool term = valid && b < 0x80;
      const unsigned long long tmask = __ballot(term);
      const unsigned long long lt = tmask & lt_mask;
      const int last_before = lt ? 63 - __clzll(lt) : -1;
      const uint64_t vpos = (last_before < 0) ? carry_len + (uint64_t)l : (uint64_t)(l - last_before - 1);
      const unsigned long long contrib =
          (valid && vpos < 10) ? ((unsigned long long)(b & 0x7f) << (7 * vpos)) : 0ull;
      // gather this varint's bytes (at most 9 earlier lanes matter)
      unsigned long long val = contrib;
      const int seg_start = last_before + 1;
#pragma unroll
      for (int j = 1; j <= 9; j++) {
        unsigned long long t = __shfl(contrib, l - j < 0 ? 0 : l - j, 64);
        if (l - j >= seg_start) val |= t;
      }
      if (last_before < 0) val |= carry_val;
      const int ord = __popcll(lt);  // ordinal of this terminator in the window
      const int nterm = __popcll(tmask);
      const uint64_t remaining = need - r.count;
      const int take = (uint64_t)nterm < remaining ? nterm : (int)remaining;
      const bool active = term && ord < take;
      // Go 1.13 overflow rule on the terminating byte
      const bool ovf = active && (vpos > 9 || (vpos == 9 && b > 1));
      const unsigned long long ovf_mask = __ballot(ovf);
      int stop_ord = take;
      if (ovf_mask) {
        const int fl = __ffsll((long long)ovf_mask) - 1;
        const int ford = __popcll(tmask & ((fl == 0) ? 0ull : (~0ull >> (64 - fl))));
        const uint64_t fvpos = __shfl(vpos, fl, 64);
        r.status = 1;
        r.n = -(int64_t)(fvpos + 1);
        stop_ord = ford;
      }
      const bool use = active && ord < stop_ord;
      // the first varint overall (item count in phase A)
      if (r.count == 0) {
        const unsigned long long fm = __ballot(use && ord == 0);
        if (fm) r.first_val = __shfl(val, __ffsll((long long)fm) - 1, 64);
      }
      unsigned long long v = use ? val : 0ull;
      if (WRITE) {
        unsigned long long inc = wave_incl_scan(v);
        if (use) {
          uint64_t slot = item_base + r.count + (uint64_t)ord;
          if (slot < item_cap) item_end[slot] = rec_base + r.sum + inc;
          else atomicOr(overflow, 1ull);
        }
      }
      r.sum += wave_sum(v);
      if (__ballot(use && v > payload_len)) r.range_flag = 1;
      r.count += (uint64_t)stop_ord;
      if (r.status) return r;
      if (r.count == need) {
        // header ends after the take-th terminator
        const unsigned long long em = __ballot(term && ord == take - 1);
        const int el = __ffsll((long long)em) - 1;
        r.end_pos = seg_lo + x + (uint64_t)el + 1;
        return r;
      }
      // carry the trailing partial varint into the next window
      const int nvalid = (int)((len - x) < 64 ? (len - x) : 64);
      if (tmask) {
        const int last = 63 - __clzll(tmask);
        const bool tail = valid && l > last;
        unsigned long long cv = tail ? contrib : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cv |= __shfl_xor(cv, o, 64);
        carry_val = cv;
        carry_len = (uint64_t)(nvalid - last - 1);
      } else {
        unsigned long long cv = contrib;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cv |= __shfl_xor(cv, o, 64);
        carry_val |= cv;
        carry_len += (uint64_t)nvalid;
      }
    }
    seg_lo += len;
  }
  // payload exhausted before `need` varints: binary.Uvarint returns n == 0
  r.status = 1;
  r.n = 0;
  return r;
}


__device__ __forceinline__ bool block_complete(const DevBufs &d, uint64_t c0, uint64_t nchunks,
                                               uint64_t &total) {
  total = d.ck_total[c0];
  return total != 0 && c0 + total <= nchunks;
}

__device__ __forceinline__ Payload block_payload(const DevBufs &d, const ParseArgs &a, uint64_t b,
                                                 uint64_t c0, uint64_t total) {
  Payload pl;
  pl.span = a.span;
  pl.ck_size = d.ck_size;
  pl.c0 = c0;
  pl.nseg = total;
  pl.contig = nullptr;
  pl.contig_len = 0;
  if (a.codec != RIO_CODEC_NONE) {
    pl.contig = d.dec + d.blk_dec_off[b];
    pl.contig_len = d.blk_out_len[b];
    pl.nseg = 1;
  }
  return pl;
}

// wave per block: magic handling + varint header -> counts
__global__ void __launch_bounds__(256) k_block_parse(DevBufs d, ParseArgs a) {
  const uint64_t nb = *a.nblocks;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t b = wave; b < nb; b += nwaves) {
    const uint64_t c0 = d.blk_c0[b];
    uint64_t total;
    unsigned long long status = kBlkOk, ea = 0, eb = 0;
    unsigned long long nitems = 0, hdr = 0, recb = 0;
    const uint32_t cls = d.ck_info[c0] & 0xff;
    bool complete = block_complete(d, c0, a.nchunks, total);
    const uint64_t end = c0 + total - 1;
    unsigned long long event = kNone;
    if (c0 >= a.limit_chunk) {
      status = kBlkLimit;
      event = 2 * c0;
    } else if (!complete) {
      status = kBlkIncomplete;
      if (l == 0) atomicMin(&d.ctl->first_incomplete, (unsigned long long)c0);
    } else {
      bool parse = false;
      if (a.mode == kModeBody) {
        if (cls == kMagicPacked) parse = true;
        else if (cls == kMagicTrailer) status = kBlkTrailer;
        else status = kBlkBadMagic;
      } else if (a.mode == kModeHeader) {
        parse = (cls == kMagicHeader);
        if (!parse) status = kBlkBadMagic;
      } else {
        parse = (cls == kMagicTrailer);
        if (!parse) status = kBlkBadMagic;
      }
      if (parse && a.codec != RIO_CODEC_NONE && d.blk_status[b] == kBlkCodec) {
        parse = false;
        status = kBlkCodec;
        ea = d.blk_a[b];
        eb = d.blk_b[b];
      }
      if (parse) {
        const uint64_t plen = (a.codec == RIO_CODEC_NONE) ? d.ck_pay[c0 + total] - d.ck_pay[c0]
                                                          : d.blk_out_len[b];
        Payload pl = block_payload(d, a, b, c0, total);
        VarintResult r0 = parse_varints<false>(pl, 0, 1, plen, nullptr, 0, 0, 0, nullptr);
        if (r0.status) {
          status = kBlkNItems;
          ea = (unsigned long long)r0.n;
        } else {
          VarintResult r1 = parse_varints<false>(pl, r0.end_pos, r0.first_val, plen, nullptr, 0, 0, 0,
                                                 nullptr);
          if (r1.status) {
            status = kBlkItemSize;
            ea = r1.count;
            eb = (unsigned long long)r1.n;
          } else if (r1.sum + r1.end_pos != plen) {
            status = kBlkBlockSize;
            ea = plen;
            eb = r1.sum + r1.end_pos;
          } else if (r1.range_flag) {
            status = kBlkItemRange;
          } else {
            nitems = r0.first_val;
            hdr = r1.end_pos;
            recb = plen - hdr;
          }
        }
      }
      if (status != kBlkOk && a.mode == kModeBody) event = 2 * end + 1;
    }
    if (l == 0) {
      d.blk_status[b] = status;
      d.blk_a[b] = ea;
      d.blk_b[b] = eb;
      d.blk_nitems[b] = (status == kBlkOk) ? nitems : 0;
      d.blk_hdr[b] = hdr;
      // record regions start 16-byte aligned
      d.blk_recb[b] = (status == kBlkOk) ? ((recb + 15) & ~15ull) : 0;
      if (event != kNone) atomicMin(&d.ctl->first_block_event, event);
    }
  }
}

// wave per block: item_end
__global__ void __launch_bounds__(256) k_items(DevBufs d, ParseArgs a) {
  const uint64_t nb = *a.nblocks;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t b = wave; b < nb; b += nwaves) {
    if (d.blk_status[b] != kBlkOk || d.blk_nitems[b] == 0) continue;
    const uint64_t c0 = d.blk_c0[b];
    const uint64_t total = d.ck_total[c0];
    const uint64_t plen = (a.codec == RIO_CODEC_NONE) ? d.ck_pay[c0 + total] - d.ck_pay[c0]
                                                      : d.blk_out_len[b];
    Payload pl = block_payload(d, a, b, c0, total);
    VarintResult r0 = parse_varints<false>(pl, 0, 1, plen, nullptr, 0, 0, 0, nullptr);
    parse_varints<true>(pl, r0.end_pos, r0.first_val, plen, d.item_end, d.blk_item_base[b], a.item_cap,
                        d.blk_rec_base[b], &d.ctl->out_overflow);
  }
}

// ---------------------------------------------------------------- CRC + copy
// Per chunk (one wave): lane t owns the 16-byte units at chunk offsets
// 1024*i + 16*t (i = 0..31; every load instruction covers 1 KiB contiguous).
// The lane's CRC state is a Horner fold over its units in which the 1008-byte
// gap to its next unit is folded into the slice tables:
//   S <- xor_j fold[j][u_j ^ byte_j(S) (j<4)],  fold[j][b] = R(b || 0^(1023-j)).
// After row 31 lane t's state is R(message) * x^(128 t); a 6-level shuffle tree
// with tables for x^(-128*2^l) combines the lanes. Bytes outside [12, 28+size)
// are zeroed, so V = R(0^12 || crc-bytes || 0^pad); per size
// crc = ~(fix_a[size] ^ V * x^(-8 pad)).
// The same loads feed the copy of the payload to records (idTransform), with
// each lane assembling the 16-byte aligned destination word that starts inside
// its unit (v_alignbyte over the unit and the next one).
constexpr int kCrcWaves = 4;  // waves per workgroup

__device__ __forceinline__ uint32_t gf_mul_dev(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 31; i >= 0; i--) {
    if ((a >> i) & 1u) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

__device__ __forceinline__ uint32_t mask_dword(uint32_t v, int off, int lo, int hi) {
  // keep bytes with chunk offset in [lo, hi)
  uint32_t m = 0xffffffffu;
  if (off < lo) m = (off + 4 <= lo) ? 0u : (0xffffffffu << (8 * (lo - off)));
  if (off + 4 > hi) m &= (off >= hi) ? 0u : (0xffffffffu >> (8 * (off + 4 - hi)));
  return v & m;
}

__device__ __forceinline__ uint32_t fold16(const uint32_t *__restrict__ T, uint32_t s, uint4 u) {
  uint32_t x0 = u.x ^ s;
  uint32_t r = T[0 * 256 + (x0 & 0xff)] ^ T[1 * 256 + ((x0 >> 8) & 0xff)] ^ T[2 * 256 + ((x0 >> 16) & 0xff)] ^
               T[3 * 256 + (x0 >> 24)];
  r ^= T[4 * 256 + (u.y & 0xff)] ^ T[5 * 256 + ((u.y >> 8) & 0xff)] ^ T[6 * 256 + ((u.y >> 16) & 0xff)] ^
       T[7 * 256 + (u.y >> 24)];
  r ^= T[8 * 256 + (u.z & 0xff)] ^ T[9 * 256 + ((u.z >> 8) & 0xff)] ^ T[10 * 256 + ((u.z >> 16) & 0xff)] ^
       T[11 * 256 + (u.z >> 24)];
  r ^= T[12 * 256 + (u.w & 0xff)] ^ T[13 * 256 + ((u.w >> 8) & 0xff)] ^ T[14 * 256 + ((u.w >> 16) & 0xff)] ^
       T[15 * 256 + (u.w >> 24)];
  return r;
}

__device__ __forceinline__ uint32_t tree_mul(const uint32_t *__restrict__ T, uint32_t v) {
  return T[0 * 256 + (v & 0xff)] ^ T[1 * 256 + ((v >> 8) & 0xff)] ^ T[2 * 256 + ((v >> 16) & 0xff)] ^
         T[3 * 256 + (v >> 24)];
}

// bytes [r, r+16) of the 32-byte pair (a, b); r wave-uniform in [0, 16)
__device__ __forceinline__ uint4 funnel16(uint4 a, uint4 b, int r) {
  const int q = r >> 2;
  const uint32_t sh = (uint32_t)(r & 3);
  uint32_t w0, w1, w2, w3, w4;
  if (q == 0) { w0 = a.x; w1 = a.y; w2 = a.z; w3 = a.w; w4 = b.x; }
  else if (q == 1) { w0 = a.y; w1 = a.z; w2 = a.w; w3 = b.x; w4 = b.y; }
  else if (q == 2) { w0 = a.z; w1 = a.w; w2 = b.x; w3 = b.y; w4 = b.z; }
  else { w0 = a.w; w1 = b.x; w2 = b.y; w3 = b.z; w4 = b.w; }
  uint4 o;
  o.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
  o.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
  o.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
  o.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
  return o;
}


__global__ void __launch_bounds__(64 * kCrcWaves) k_crc_copy(const uint8_t *__restrict__ span, uint64_t nchunks,
                                                           DevBufs d, CopyArgs ca) {
  __shared__ uint32_t s_fold[16 * 256];
  __shared__ uint32_t s_tree[6 * 4 * 256];
  for (int i = threadIdx.x; i < 16 * 256; i += blockDim.x) s_fold[i] = d.crc_fold[i];
  for (int i = threadIdx.x; i < 6 * 4 * 256; i += blockDim.x) s_tree[i] = d.crc_tree[i];
  __syncthreads();
  const int l = lane_id();
  const uint64_t wave = (uint64_t)blockIdx.x * kCrcWaves + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kCrcWaves;
  for (uint64_t c = wave; c < nchunks; c += nwaves) {
    const uint8_t *ck = span + c * kChunk;
    const uint32_t size = d.ck_size[c];
    if (size > (uint32_t)kMaxPayload) continue;  // "Invalid chunk size": no CRC
    const int end = kChunkHdr + (int)size;
    // copy window of this chunk (none codec, chunk inside an ok block)
    bool copy = false;
    int64_t D = 0;
    int64_t dlo = 0, dhi = 0;
    if (ca.copy) {
      const uint32_t b = d.ck_block[c];
      const uint64_t c0 = d.blk_c0[b];
      if (d.blk_status[b] == kBlkOk && c >= c0 && c < c0 + d.ck_total[c0]) {
        const uint64_t Lj = d.ck_pay[c] - d.ck_pay[c0];
        const uint64_t hdr = d.blk_hdr[b];
        const uint64_t rb = d.blk_rec_base[b];
        if (Lj + size > hdr && rb + d.blk_recb[b] <= ca.rec_cap) {
          copy = true;
          D = (int64_t)rb + (int64_t)Lj - kChunkHdr - (int64_t)hdr;
          const int64_t plo = (Lj >= hdr) ? kChunkHdr : kChunkHdr + (int64_t)(hdr - Lj);
          dlo = plo + D;
          dhi = end + D;
        } else if (Lj + size > hdr) {
          atomicOr(&d.ctl->out_overflow, 2ull);
        }
      }
    }
    const int r = (int)((-D) & 15);  // source offset of a destination word, mod 16
    uint32_t s = 0;
    const bool full = (size == (uint32_t)kMaxPayload);
#pragma unroll 4
    for (int i = 0; i < 32; i++) {
      const int o = 1024 * i + 16 * l;
      uint4 u = *reinterpret_cast<const uint4 *>(ck + o);
      uint4 v = u;
      if (i == 0 && l == 0) {  // magic[0:8] and crc[8:12] are not covered
        v.x = 0;
        v.y = 0;
        v.z = 0;
      }
      if (!full) {
        v.x = mask_dword(v.x, o, 12, end);
        v.y = mask_dword(v.y, o + 4, 12, end);
        v.z = mask_dword(v.z, o + 8, 12, end);
        v.w = mask_dword(v.w, o + 12, 12, end);
      }
      s = fold16(s_fold, s, v);
      if (copy) {
        const int64_t q = (int64_t)o + r + D;  // destination of bytes [o+r, o+r+16)
        if (q + 16 > dlo && q < dhi) {
          uint4 nx = make_uint4(0, 0, 0, 0);
          if (r != 0 && o + 16 < kChunk) nx = *reinterpret_cast<const uint4 *>(ck + o + 16);
          const uint4 w = funnel16(u, nx, r);
          uint8_t *dst = ca.out + q;
          if (q >= dlo && q + 16 <= dhi) {
            *reinterpret_cast<uint4 *>(dst) = w;
          } else {
            const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int k = 0; k < 16; k++)
              if (q + k >= dlo && q + k < dhi) dst[k] = (uint8_t)(ws[k >> 2] >> (8 * (k & 3)));
          }
        }
      }
    }
    // combine lanes: lane t holds R * x^(128 t)
#pragma unroll
    for (int lv = 0; lv < 6; lv++) {
      const uint32_t m = tree_mul(s_tree + lv * 1024, s);
      const int step = 1 << lv;
      const uint32_t o = __shfl(m, (l + step) & 63, 64);
      s ^= (l + step < 64) ? o : 0u;
    }
    if (l == 0) {
      const uint32_t V = s;
      const uint32_t crc = ~(d.crc_fix_a[size] ^ gf_mul_dev(V, d.crc_fix_b[size]));
      d.ck_crc[c] = crc;
      const uint32_t stored = *reinterpret_cast<const uint32_t *>(ck + 8);
      if (crc != stored) atomicMin(&d.ctl->first_crc_err, (unsigned long long)c);
    }
  }
}

// ---------------------------------------------------------------- resolve

__device__ __forceinline__ void load_magic(const uint8_t *span, uint64_t ch, unsigned long long &m) {
  const uint32_t *h = reinterpret_cast<const uint32_t *>(span + ch * kChunk);
  m = (unsigned long long)h[0] | ((unsigned long long)h[1] << 32);
}

__global__ void k_resolve(DevBufs d, ResolveArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Ctl *c = d.ctl;
  const uint64_t nb = *a.nblocks;
  const unsigned long long ce =
      c->first_chunk_err < c->first_crc_err ? c->first_chunk_err : c->first_crc_err;
  unsigned long long key = (ce == kNone) ? kNone : 2 * ce;
  int kind = (ce == kNone) ? 0 : 2;  // 2 chunk error, 3 block event, 4 tail
  uint64_t nvalid = 0;
  c->stop_block = kNone;
  c->err_chunk = kNone;
  c->err_code = 0;
  c->stop_kind = 0;
  if (a.mode == kModeLastChunk) {
    // ReadLastBlock's first readChunk (chunk.go:387): size, then CRC, of chunk 0
    c->consumed_chunks = a.nchunks;
    c->n_valid_blocks = 0;
    c->n_items = 0;
    c->rec_bytes = 0;
    if (a.nchunks == 0) {
      c->stop_kind = 2;
      c->err_code = 101;
      return;
    }
    const uint32_t cerr = d.ck_info[0] >> 8;
    if (cerr == kCkSize || c->first_crc_err == 0) {
      c->err_chunk = 0;
      c->err_code = (cerr == kCkSize) ? kCkSize : 100;
      c->stop_kind = 2;
      c->ck_size = d.ck_size[0];
      c->ck_crc_stored = *reinterpret_cast<const uint32_t *>(a.span + 8);
      c->ck_crc_actual = d.ck_crc[0];
    } else {
      c->stop_kind = 1;
    }
    return;
  }
  if (a.mode != kModeBody) {
    // header / trailer special block: exactly block 0 (readSpecialBlock,
    // ReadLastBlock); stop after it
    uint64_t total = (nb > 0) ? d.ck_total[0] : 0;
    bool complete = nb > 0 && d.blk_c0[0] == 0 && total != 0 && total <= a.nchunks;
    uint64_t end = complete ? total - 1 : a.nchunks;
    if (ce != kNone && (!complete || ce <= end)) {
      kind = 2;
    } else if (!complete) {
      kind = 4;
      key = 2 * a.nchunks;
    } else {
      kind = 3;
      key = 2 * end + 1;
      c->stop_block = 0;
      nvalid = (d.blk_status[0] == kBlkOk) ? 1 : 0;
    }
  } else {
    const unsigned long long bev = c->first_block_event;
    if (bev < key) {
      key = bev;
      kind = 3;
    }
    unsigned long long tail;
    if (a.is_file_end) tail = 2 * a.nchunks;
    else tail = (c->first_incomplete != kNone) ? 2 * c->first_incomplete : 2 * a.nchunks;
    if (tail < key) {
      key = tail;
      kind = 4;
    }
    // blocks finished strictly before the stop
    uint64_t lo = 0, hi = nb;
    while (lo < hi) {
      uint64_t mid = (lo + hi) / 2;
      if (2 * d.blk_c0[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    nvalid = lo;
    if (nvalid > 0) {
      uint64_t c0 = d.blk_c0[nvalid - 1];
      uint64_t total = d.ck_total[c0];
      if (total == 0 || 2 * (c0 + total - 1) + 1 >= key) nvalid--;
    }
    if (kind == 3) {
      uint64_t chunk = (bev & 1) ? (bev - 1) / 2 : bev / 2;
      uint64_t b = d.ck_block[chunk];
      c->stop_block = (b < nb) ? b : nb - 1;
    }
  }
  c->stop_key = key;
  c->n_valid_blocks = nvalid;
  c->n_items = d.blk_item_base[nvalid];
  c->rec_bytes = d.blk_rec_base[nvalid];
  if (kind == 2) {
    // chunk-level error; within one chunk: size > crc > structural (chunk.go:333-343)
    const uint64_t ch = ce;
    c->err_chunk = ch;
    const uint32_t cerr = d.ck_info[ch] >> 8;
    if (cerr == kCkSize) c->err_code = kCkSize;
    else if (c->first_crc_err == ch) c->err_code = 100;
    else c->err_code = cerr;
    c->stop_kind = 2;
  } else if (kind == 3) {
    const unsigned long long st = d.blk_status[c->stop_block];
    if (a.mode != kModeBody) c->stop_kind = (st == kBlkOk) ? 1 : 2;
    else c->stop_kind = (st == kBlkTrailer || st == kBlkLimit) ? 1 : 2;
  } else if (kind == 4) {
    if (a.is_file_end) {
      // A partial tail chunk is read (io.ErrUnexpectedEOF) only inside an
      // unfinished block, or when a new block may still start there (< limit).
      const bool mid = c->first_incomplete != kNone;
      const bool tail_err = a.tail_partial && (mid || a.nchunks < a.limit_chunk);
      c->stop_kind = tail_err ? 2 : 1;
      if (tail_err) c->err_code = 101;  // "unexpected EOF"
    } else {
      c->stop_kind = 0;
    }
  } else {
    c->stop_kind = a.is_file_end ? 1 : 0;
  }
  c->consumed_chunks = (nvalid < nb) ? d.blk_c0[nvalid] : a.nchunks;
  if (c->first_incomplete != kNone && c->first_incomplete < c->consumed_chunks)
    c->consumed_chunks = c->first_incomplete;
  if (a.mode != kModeBody && nvalid == 1) c->consumed_chunks = d.ck_total[0];
  if (c->err_chunk != kNone) {
    const uint64_t ch = c->err_chunk;
    c->ck_size = d.ck_size[ch];
    c->ck_total = d.ck_total[ch];
    c->ck_index = d.ck_index[ch];
    c->ck_info = d.ck_info[ch];
    c->ck_crc_stored = *reinterpret_cast<const uint32_t *>(a.span + ch * kChunk + 8);
    c->ck_crc_actual = d.ck_crc[ch];
    load_magic(a.span, ch, c->mag_cur);
    if (ch > 0) {
      c->prev_total = d.ck_total[ch - 1];
      c->prev_index = d.ck_index[ch - 1];
      c->prev_info = d.ck_info[ch - 1];
      load_magic(a.span, ch - 1, c->mag_prev);
    }
  }
  if (c->stop_block != kNone) {
    const uint64_t b = c->stop_block;
    c->blk_status = d.blk_status[b];
    c->blk_a = d.blk_a[b];
    c->blk_b = d.blk_b[b];
    c->blk_c0 = d.blk_c0[b];
    load_magic(a.span, c->blk_c0, c->mag_blk);
  }
}

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
                 unsigned long long *partial, unsigned long long *total_out, hipStream_t st) {
  const unsigned tiles = (unsigned)((n_max + kScanTile - 1) / kScanTile);
  const unsigned g = tiles ? tiles : 1;
  hipLaunchKernelGGL(k_scan_reduce<F>, dim3(g), dim3(kScanThreads), 0, st, f, n_dev, n_host, partial);
  hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(1024), 0, st, n_dev, n_host, partial, total_out);
  hipLaunchKernelGGL((k_scan_apply<F, O>), dim3(g), dim3(kScanThreads), 0, st, f, o, n_dev, n_host, partial);
}

void launch_chunk_scans(uint64_t nchunks, const DevBufs &d, unsigned long long *nblocks_dev, hipStream_t st) {
  scan(FlagLoad{d.ck_index}, FlagOut{d.blk_c0, d.ck_block}, nullptr, nchunks, nchunks, d.scan_tmp,
       nblocks_dev, st);
  scan(SizeLoad{d.ck_size}, U64Out{d.ck_pay}, nullptr, nchunks, nchunks, d.scan_tmp, d.ck_pay + nchunks, st);
}

void launch_block_parse(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_block_parse, dim3(grid_for(max_blocks, 4, 2048)), dim3(256), 0, st, d, a);
}

void launch_block_scans(const DevBufs &d, const unsigned long long *nblocks_dev, uint64_t max_blocks,
                        hipStream_t st) {
  scan(U64Load{d.blk_nitems}, U64Out{d.blk_item_base}, nblocks_dev, 0, max_blocks, d.scan_tmp, nullptr, st);
  // totals at [nblocks]: written by a tiny kernel below
  scan(U64Load{d.blk_recb}, U64Out{d.blk_rec_base}, nblocks_dev, 0, max_blocks, d.scan_tmp, nullptr, st);
}

__global__ void k_scan_totals(DevBufs d, const unsigned long long *nblocks_dev) {
  if (threadIdx.x != 0) return;
  const uint64_t n = *nblocks_dev;
  if (n == 0) {
    d.blk_item_base[0] = 0;
    d.blk_rec_base[0] = 0;
    return;
  }
  d.blk_item_base[n] = d.blk_item_base[n - 1] + d.blk_nitems[n - 1];
  d.blk_rec_base[n] = d.blk_rec_base[n - 1] + d.blk_recb[n - 1];
}

void launch_scan_totals(const DevBufs &d, const unsigned long long *nblocks_dev, hipStream_t st) {
  hipLaunchKernelGGL(k_scan_totals, dim3(1), dim3(64), 0, st, d, nblocks_dev);
}

void launch_items(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_items, dim3(grid_for(max_blocks, 4, 2048)), dim3(256), 0, st, d, a);
}

void launch_crc_copy(const uint8_t *span, uint64_t nchunks, const DevBufs &d, const CopyArgs &ca,
                     int ncu, hipStream_t st) {
  const unsigned cap = (unsigned)(ncu > 0 ? ncu : 256) * 4;
  hipLaunchKernelGGL(k_crc_copy, dim3(grid_for(nchunks, kCrcWaves, cap)), dim3(64 * kCrcWaves), 0, st, span,
                     nchunks, d, ca);
}

void launch_resolve(const DevBufs &d, const ResolveArgs &a, hipStream_t st) {
  hipLaunchKernelGGL(k_resolve, dim3(1), dim3(64), 0, st, d, a);
}

}  // namespace rio
