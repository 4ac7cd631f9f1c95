// Block-level kernels of the scan path: header parse (parseChunksToItems,
// recordio/scannerv2.go:53-97), item views, straddler copies and the
// first-error resolve (errors.Once semantics, scannerv2.go:242).
//
// Output contract ("views plus straddler copies"): item i is
// item_len[i] bytes at item_off[i] -- an offset into the input span, or, with
// RIO_ITEM_IN_RECORDS set, into the records buffer, which holds the items that
// cross a chunk payload boundary (none codec) or the decoded blocks (flate,
// zstd). Nothing but straddling items is copied.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "parse_block.h"
#include "rio_internal.h"

namespace rio {

constexpr uint32_t kNoBlockId = 0xffffffffu;
#ifndef RIO_PARSE_BATCH
#define RIO_PARSE_BATCH 4
#endif
#ifndef RIO_PARSE_GRID
#define RIO_PARSE_GRID 2048
#endif
constexpr int kBatch = RIO_PARSE_BATCH;  // blocks per wave iteration: their loads are issued together

// Wave per block, kBatch blocks per iteration: block magic handling
// (scanNextBlock, scannerv2.go:374-387), the header of parseChunksToItems
// (scannerv2.go:53-97) and one view per item (cumSize, scannerv2.go:83-91)
// into the item slots reserved by the block scan.
__global__ void __launch_bounds__(256) k_parse(DevBufs d, ParseArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_win[4][1040];  // 1 KiB window + room for lds_bytes4
  __shared__ __attribute__((aligned(16))) uint16_t s_tpos[4][1024];
  uint8_t *lwin = s_win[threadIdx.x >> 6];
  uint16_t *ltpos = s_tpos[threadIdx.x >> 6];
  const uint64_t nb = a.list ? *a.list_n : *a.nblocks;  // list: the blocks k_parse_lean declined
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t b0 = wave * kBatch; b0 < nb; b0 += nwaves * kBatch) {
    // round 1: descriptors of the batch (lane j: block b0 + j)
    unsigned long long m_b = 0, m_c0 = 0, m_meta = 0, m_len = 0, m_base = 0, m_pay0 = 0;
    if (l < kBatch && b0 + l < nb) {
      const uint64_t b = a.list ? a.list[b0 + l] : b0 + l;
      m_b = b;
      m_c0 = d.blk_c0[b];
      m_meta = d.blk_meta[b];
      m_len = (a.codec == RIO_CODEC_NONE) ? d.blk_len[b] : d.blk_out_len[b];
      m_base = d.blk_item_base[b];
      if (a.codec == RIO_CODEC_NONE) m_pay0 = d.ck_pay[m_c0];
    }
    unsigned long long bs[kBatch], c0s[kBatch], metas[kBatch], lens[kBatch], bases[kBatch], pay0s[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; j++) {  // wave-uniform: scalar registers
      bs[j] = readlane_u64(m_b, j);
      c0s[j] = readlane_u64(m_c0, j);
      metas[j] = readlane_u64(m_meta, j);
      lens[j] = readlane_u64(m_len, j);
      bases[j] = readlane_u64(m_base, j);
      pay0s[j] = readlane_u64(m_pay0, j);
    }
    // round 2: the first 1 KiB of every block payload (16 B per lane)
    uint32_t win[kBatch][4];
#pragma unroll
    for (int j = 0; j < kBatch; j++) {
      win[j][0] = win[j][1] = win[j][2] = win[j][3] = 0x80808080u;
      if (b0 + j >= nb || !(metas[j] & kMetaComplete)) continue;
      const uint64_t p = 16ull * l;
      if (a.codec != RIO_CODEC_NONE) {
        const uint64_t b = bs[j];
        if (p + 16 <= lens[j]) {
#ifdef RIO_CHECKED
          if (d.blk_dec_off[b] + p + 16 > d.dec_cap) {
            atomicOr(&d.ctl->out_overflow, 0x1000ull);
            continue;
          }
#endif
          const uint4 v = *reinterpret_cast<const uint4 *>(d.dec + d.blk_dec_off[b] + p);
          win[j][0] = v.x;
          win[j][1] = v.y;
          win[j][2] = v.z;
          win[j][3] = v.w;
        }
      } else {
        const uint64_t size0 = lens[j] < (uint64_t)kMaxPayload ? lens[j] : (uint64_t)kMaxPayload;
        if (p + 16 <= size0) {  // 4-byte aligned: 28 + 16 l
          const uint32_t *q = reinterpret_cast<const uint32_t *>(a.span + c0s[j] * kChunk + kChunkHdr + p);
          win[j][0] = q[0];
          win[j][1] = q[1];
          win[j][2] = q[2];
          win[j][3] = q[3];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kBatch; j++) {
      if (b0 + j >= nb) break;
      parse_block(d, a, bs[j], c0s[j], metas[j], lens[j], bases[j], pay0s[j], win[j], lwin, ltpos);
    }
  }
}

// The none codec's common block shape in a lean kernel (run before k_parse,
// which then takes only the blocks listed here): a complete packed body block
// of regular chunks, its header inside the first 1 KiB of payload, at most 256
// sizes of at most 4 bytes each, consistent with the block. Wave per block,
// kLeanBatch blocks per iteration with every load of the batch issued
// together: the header window and, for a block of >= 2 chunks, the 1 KiB
// around its first chunk boundary, so the straddler there is written from
// registers. Anything else -- and any header that is not valid -- is appended
// to the list for k_parse, untouched (nothing here writes before the checks).
#ifndef RIO_LEAN_BATCH
#define RIO_LEAN_BATCH 2
#endif
constexpr int kLeanBatch = RIO_LEAN_BATCH;

__global__ void __launch_bounds__(256) k_parse_lean(DevBufs d, ParseArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_win[4][1040];
  __shared__ __attribute__((aligned(16))) uint16_t s_tpos[4][264];
  uint8_t *lwin = s_win[threadIdx.x >> 6];
  uint16_t *ltpos = s_tpos[threadIdx.x >> 6];
  const uint64_t nb = *a.nblocks;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t b0 = wave * kLeanBatch; b0 < nb; b0 += nwaves * kLeanBatch) {
    unsigned long long m_c0 = 0, m_meta = 0, m_len = 0, m_base = 0;
    if (l < kLeanBatch && b0 + l < nb) {
      const uint64_t b = b0 + l;
      m_c0 = d.blk_c0[b];
      m_meta = d.blk_meta[b];
      m_len = d.blk_len[b];
      m_base = d.blk_item_base[b];
    }
    unsigned long long c0s[kLeanBatch], metas[kLeanBatch], lens[kLeanBatch], bases[kLeanBatch];
    bool ok[kLeanBatch];
#pragma unroll
    for (int j = 0; j < kLeanBatch; j++) {
      c0s[j] = readlane_u64(m_c0, j);
      metas[j] = readlane_u64(m_meta, j);
      lens[j] = readlane_u64(m_len, j);
      bases[j] = readlane_u64(m_base, j);
      const uint32_t cls = (uint32_t)(metas[j] >> kMetaClsShift) & 0xffu;
      ok[j] = b0 + j < nb && (metas[j] & kMetaComplete) && (metas[j] & kMetaRegular) && cls == kMagicPacked &&
              c0s[j] < a.limit_chunk && lens[j] < (1ull << 32);
    }
    uint32_t win[kLeanBatch][4], bnd[kLeanBatch][4];
#pragma unroll
    for (int j = 0; j < kLeanBatch; j++) {
      win[j][0] = win[j][1] = win[j][2] = win[j][3] = 0x80808080u;
      bnd[j][0] = bnd[j][1] = bnd[j][2] = bnd[j][3] = 0;
      if (!ok[j]) continue;
      const uint8_t *ck = a.span + c0s[j] * kChunk;
      const uint64_t size0 = lens[j] < (uint64_t)kMaxPayload ? lens[j] : (uint64_t)kMaxPayload;
      if (16ull * l + 16 <= size0) {  // 4-byte aligned: 28 + 16 l
        const uint32_t *q = reinterpret_cast<const uint32_t *>(ck + kChunkHdr + 16 * l);
        win[j][0] = q[0];
        win[j][1] = q[1];
        win[j][2] = q[2];
        win[j][3] = q[3];
      }
      if ((metas[j] & kMetaTotalMask) >= 2) {  // payload kBndW0 + 16 l: chunk c0's tail, then c0 + 1's head
        const uint8_t *src = (l < 32) ? ck + kChunkHdr + kBndW0 + 16 * l : ck + kChunk + kChunkHdr + 16 * (l - 32);
        const uint32_t *q = reinterpret_cast<const uint32_t *>(src);
        bnd[j][0] = q[0];
        bnd[j][1] = q[1];
        bnd[j][2] = q[2];
        bnd[j][3] = q[3];
      }
    }
#pragma unroll
    for (int j = 0; j < kLeanBatch; j++) {
      if (b0 + j >= nb) break;
      const uint64_t b = b0 + j;
      bool done = false;
      uint32_t hdr = 0;
      if (ok[j]) {
        const uint32_t(&w)[4] = win[j];
        const uint32_t tmask = term4(w[0]) | (term4(w[1]) << 4) | (term4(w[2]) << 8) | (term4(w[3]) << 12);
        const uint32_t cnt = __popc(tmask);
        const uint32_t incl = wave_incl_sum_dpp(cnt);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        *reinterpret_cast<uint4 *>(lwin + 16 * l) = make_uint4(w[0], w[1], w[2], w[3]);
        {  // terminator positions of ordinals 0..263 (a header of <= 256 sizes ends by then)
          uint32_t m = (incl - cnt < 264u) ? tmask : 0u, o = incl - cnt;
          while (m && o < 264u) {
            const uint32_t i = __ffs(m) - 1;
            m &= m - 1;
            ltpos[o++] = (uint16_t)(16 * l + i);
          }
        }
        wave_lds_sync();
        const uint32_t p0 = ltpos[0];
        if (total > 0 && p0 < 2) {  // item count: one or two bytes
          const uint32_t nitems = uvarint4(lds_bytes4(lwin, 0), p0 + 1);
          if (nitems <= 256 && nitems < total) {
            hdr = (uint32_t)ltpos[nitems] + 1;
            Payload pl = desc_payload(a.span, d, c0s[j], metas[j], lens[j], 0);
            ParseOut po;
            po.item_off = d.item_off;
            po.item_len = d.item_len;
            po.item_end = a.end_mode ? d.item_off : nullptr;
            po.whole = false;
            po.item_base = bases[j];
            po.item_cap = a.item_cap;
            po.view_base = 0;
            po.strad = d.strad;
            po.ssz = d.ck_ssz;
            po.c0 = c0s[j];
            po.overflow = &d.ctl->out_overflow;
            done = small_header<true>(pl, po, lwin, ltpos, nitems, hdr, a.sparse ? d.side : nullptr, bnd[j]) == 1;
          }
        }
        wave_lds_sync();  // the next block's window reuses lwin / ltpos
      }
      if (l == 0) {
        if (done) {
          d.blk_status[b] = kBlkOk;
          d.blk_a[b] = 0;
          d.blk_b[b] = 0;
          d.blk_hdr[b] = hdr;
          if (a.end_mode) d.blk_data[b] = c0s[j] * (uint64_t)kChunk;
        } else {
          d.blk_coff[atomicAdd(&d.ctl->n_retry, 1ull)] = b;
        }
      }
    }
  }
}

// The lean path in item-end mode (RIO_CFG_ITEM_END device results, the
// none codec): the same block shape as k_parse_lean, one block per wave
// iteration with the next block's descriptor loaded while this one is parsed,
// cumSize per item (8 B) written coalesced, and nothing but the arrays this
// path touches passed in (the full DevBufs costs ~90 scalar registers, whose
// spills dominated the previous kernel's instruction stream). Declined blocks
// go to the list for k_parse, untouched.
struct LeanArgs {
  const uint8_t *span;
  const unsigned long long *blk_c0, *blk_meta, *blk_len, *blk_item_base;
  unsigned long long *blk_status, *blk_hdr, *blk_data, *blk_coff;
  unsigned long long *item_end;
  uint8_t *side;
  Ctl *ctl;
  const unsigned long long *nblocks;
  uint64_t limit_chunk, item_cap;
};

constexpr int kLeanHdrLanes = 32;  // header window lanes loaded (16 B each)
constexpr int kLeanBndLanes = 16;  // boundary window lanes loaded either side of the chunk boundary

// The uvarint of the n <= 4 bytes in x (its last byte the terminator): bytes
// past n masked off first, then the 7-bit groups packed
__device__ __forceinline__ uint32_t uvarint4m(uint32_t x, uint32_t n) {
  x &= 0xffffffffu >> (32u - 8u * n);
  return (x & 0x7fu) | ((x >> 1) & 0x3f80u) | ((x >> 2) & 0x1fc000u) | ((x >> 3) & 0xfe00000u);
}

// k_lean_end (round 5). Lane l owns items 4l .. 4l+3, whose size varints are
// consecutive header bytes: it finds where they start from the terminator of
// rank 4l, decodes them from the window, and one wave scan of the lanes' sums
// places them (the round-4 kernel -- lane l owning items l, l+64, ... with four
// scans and an LDS position per terminator -- issued 19 % more VALU
// instructions at the same time per launch).
// What bounds it (C2, `profiles/r05_lean_end.json`): HBM traffic, not issue --
// 0.36 GB read and 0.60 GB written per launch (0.51 GB of it the 8-byte item
// ends); without the item stores (a measurement-only build) 0.21 ms instead of
// 0.30, and neither 8 waves per SIMD, nor two blocks in flight per wave, nor
// store instructions that never make the loop wait (buffer stores with
// out-of-range offsets for idle lanes, 0.37 ms) shortened it.
__global__ void __launch_bounds__(256) k_lean_end(LeanArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_win[4][1040];
  __shared__ uint32_t s_tm[4][64];  // lane l's terminator mask: window bytes 16 l .. 16 l + 15
  __shared__ uint16_t s_p4[4][64];  // byte of the terminator of rank 4 j (rank 0: the item count's)
  uint32_t *ltm = s_tm[threadIdx.x >> 6];
  uint16_t *lp4 = s_p4[threadIdx.x >> 6];
  uint8_t *lwin = s_win[threadIdx.x >> 6];
  const uint64_t nb = *a.nblocks;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  if (wave >= nb) return;
  // lane j < 4 holds descriptor field j of a block. Software-pipelined: while
  // block b is parsed, block b + nwaves's windows and block b + 2 nwaves's
  // descriptor are in flight
  const unsigned long long *dsrc = l == 0 ? a.blk_c0 : l == 1 ? a.blk_meta : l == 2 ? a.blk_len : a.blk_item_base;
  auto dload = [&](uint64_t x) -> unsigned long long { return dsrc[x < nb ? x : nb - 1]; };  // (x >= nb: unused)
  auto lean_ok = [&](unsigned long long dsc) {
    const uint64_t c0 = readlane_u64(dsc, 0);
    const unsigned long long meta = readlane_u64(dsc, 1), len = readlane_u64(dsc, 2);
    const uint32_t cls = (uint32_t)(meta >> kMetaClsShift) & 0xffu;
    return (meta & kMetaComplete) && (meta & kMetaRegular) && cls == kMagicPacked && c0 < a.limit_chunk &&
           len < (1ull << 32);
  };
  // the header window's first 512 B (lanes 0-31) and 256 B either side of the
  // chunk boundary (lanes 16-47: a C2 block's 508-byte header and 256-byte
  // straddler); a longer header or a straddler outside goes to k_parse
  auto hdr_in = [&](unsigned long long dsc, bool ok) {  // this lane's header piece lies in the payload
    const unsigned long long len = readlane_u64(dsc, 2);
    const uint32_t size0 = len < (uint64_t)kMaxPayload ? (uint32_t)len : (uint32_t)kMaxPayload;
    return ok && l < kLeanHdrLanes && 16u * (uint32_t)l + 16u <= size0;
  };
  auto fetch = [&](unsigned long long dsc, bool ok, uint4 &w, uint4 &bnd) {
    w = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
    bnd = make_uint4(0, 0, 0, 0);
    if (!ok) return;
    const uint64_t c0 = readlane_u64(dsc, 0);
    const unsigned long long meta = readlane_u64(dsc, 1);
    const uint8_t *ck = a.span + c0 * kChunk + kChunkHdr;
    if (hdr_in(dsc, ok)) w = *reinterpret_cast<const uint4 *>(ck + 16 * l);  // 4-byte aligned: 28 + 16 l
    if ((meta & kMetaTotalMask) >= 2 && l >= 32 - kLeanBndLanes && l < 32 + kLeanBndLanes)
      // payload kBndW0 + 16 l: chunk c0's tail, then c0 + 1's head
      bnd = *reinterpret_cast<const uint4 *>(l < 32 ? ck + kBndW0 + 16 * l : ck + kChunk + 16 * (l - 32));
  };
  // one block: parse it from its windows (w, bnd) and write its results
  auto parse_one = [&](uint64_t b, unsigned long long desc, bool ok, const uint4 &wl, const uint4 &bnd4) {
    const uint64_t c0 = readlane_u64(desc, 0);
    const unsigned long long len = readlane_u64(desc, 2);
    const uint64_t base = readlane_u64(desc, 3);
    const uint32_t w[4] = {wl.x, wl.y, wl.z, wl.w}, bnd[4] = {bnd4.x, bnd4.y, bnd4.z, bnd4.w};
    bool done = false;
    uint32_t hdr = 0, nitems = 0, g = 4u * (uint32_t)l, S = 0, E = 0;
    unsigned long long q0 = 0, q1 = 0, q2 = 0, q3 = 0, sm = 0;
    if (ok) {
      const uint32_t tmask = term4(w[0]) | (term4(w[1]) << 4) | (term4(w[2]) << 8) | (term4(w[3]) << 12);
      const uint32_t cnt = __popc(tmask);
      const uint32_t incl = wave_incl_sum_dpp(cnt);
      const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      *reinterpret_cast<uint4 *>(lwin + 16 * l) = make_uint4(w[0], w[1], w[2], w[3]);
      ltm[l] = tmask;
      // the item count: one or two bytes, the window's first terminator
      const uint32_t tm0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)tmask);
      const uint32_t w00 = (uint32_t)__builtin_amdgcn_readfirstlane((int)w[0]);
      nitems = (tm0 & 3u) ? uvarint4m(w00, (tm0 & 1u) ? 1u : 2u) : ~0u;
      const bool hdr_ok = nitems <= 256 && nitems < total;  // every size's terminator inside the window
      if (hdr_ok) {
        // positions of the terminators of ranks 0, 4, 8, ... below nitems
        uint32_t r = incl - cnt, m = tmask;
#pragma unroll
        for (int q = 0; q < 3; q++)
          if (r & 3u) m &= m - 1, r++;
#pragma unroll
        for (int it = 0; it < 4; it++) {
          const bool put = m != 0 && r < nitems;
          if (!__ballot(put)) break;
          if (put) lp4[r >> 2] = (uint16_t)(16u * l + (uint32_t)(__ffs(m) - 1));
          m &= m - 1, m &= m - 1, m &= m - 1, m &= m - 1;
          r += 4;
        }
      }
      wave_lds_sync();
      if (hdr_ok) {
        const bool act = g < nitems;
        const uint32_t s = act ? (uint32_t)lp4[l] + 1u : 0u;  // its size varint's first byte
        const uint32_t tw = ((ltm[s >> 4] | (ltm[(s >> 4) + 1] << 16)) >> (s & 15u));  // terminators from byte s
        uint32_t v[4], e[4];
        bool lng = false;
        uint32_t mm = tw, prev = ~0u, vor = 0;  // prev: the last byte of the previous varint (s-relative)
        // (branch-free: a lane past the last item reads in-window bytes and drops them)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          e[i] = (uint32_t)(__ffs(mm) - 1);  // ~0u when none
          mm &= mm - 1;
          const uint32_t n = e[i] - prev;
          const bool valid = g + i < nitems;
          lng |= valid && n - 1u > 3u;  // a varint longer than 4 bytes (or no terminator)
          const uint32_t x = lds_bytes4(lwin, s + prev + 1u);
          const uint32_t c = (x & 0x7fu) | ((x >> 1) & 0x3f80u) | ((x >> 2) & 0x1fc000u) | ((x >> 3) & 0xfe00000u);
          v[i] = valid ? c & ((1u << (7u * min(n, 4u))) - 1u) : 0u;  // (n > 4 is declined above)
          vor |= v[i];
          prev = e[i];
        }
        // sizes below 2^24: the u32 sums below cannot wrap (4 x 64 of them)
        const uint32_t z0 = v[0], z1 = z0 + v[1], z2 = z1 + v[2], z3 = z2 + v[3];
        const uint32_t inc = wave_incl_sum_dpp(z3);
        const uint32_t ex = inc - z3, sum = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        // the header's end: the terminator of rank nitems (the last item's varint)
        if (nitems > 0) {
          const uint32_t j = (nitems - 1) & 3u;
          const uint32_t ej = j == 0 ? e[0] : j == 1 ? e[1] : j == 2 ? e[2] : e[3];
          hdr = (uint32_t)__builtin_amdgcn_readlane((int)(s + ej), (int)((nitems - 1) >> 2)) + 1u;
        } else {
          hdr = (uint32_t)(__ffs(tm0) - 1) + 1u;
        }
        const uint32_t plen = (uint32_t)len;
        const bool bad = lng || vor >= (1u << 24);
        if (!__ballot(bad) && (uint64_t)hdr + sum == (uint64_t)plen) {
          // chunk crossings (items are payload bytes [hdr + ex + z(i-1), hdr + ex + zi)): only a
          // straddler across the first chunk boundary, inside the loaded part of the
          // boundary window, is taken (written from the registers); any other is declined
          constexpr uint32_t M = (uint32_t)kMaxPayload;
          constexpr uint32_t W0 = M - 16 * kLeanBndLanes, W1 = W0 + 32 * kLeanBndLanes;
          const uint32_t L0 = hdr + ex;
          const bool cross = z3 > 0 && L0 / M != (L0 + z3 - 1) / M;
          bool far = false, sd = false;
          uint32_t Sl = 0, El = 0;
          if (cross) {
            uint32_t st = L0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const uint32_t en = st + v[i];
              if (v[i] > 0 && st / M != (en - 1) / M) {
                const bool here = st < M && en > M && st >= W0 && en <= W1;
                far |= !here;
                if (here) sd = true, Sl = st, El = en;
              }
              st = en;
            }
          }
          if (!__ballot(far)) {
            done = true;
            // cumSize (scannerv2.go:83-91): the item's end past the header
            q0 = ex + z0, q1 = ex + z1, q2 = ex + z2, q3 = ex + z3;
            sm = __ballot(sd);  // the straddler at the boundary (at most one item crosses it)
            if (sm) {
              const int L = __ffsll((long long)sm) - 1;
              S = (uint32_t)__builtin_amdgcn_readlane((int)Sl, L);
              E = (uint32_t)__builtin_amdgcn_readlane((int)El, L);
            }
          }
        }
      }
      wave_lds_sync();  // the next block's window reuses lwin / ltm / lp4
    }
    if (done) {
      const uint64_t cap = a.item_cap, slot = base + g;
      if (g + 3 < nitems && slot + 3 < cap) {
        view_store2(a.item_end + slot, q0, q1);
        view_store2(a.item_end + slot + 2, q2, q3);
      } else if (g < nitems) {
        if (slot < cap) view_store(a.item_end + slot, q0);
        if (g + 1 < nitems && slot + 1 < cap) view_store(a.item_end + slot + 1, q1);
        if (g + 2 < nitems && slot + 2 < cap) view_store(a.item_end + slot + 2, q2);
        if (g + 3 < nitems && slot + 3 < cap) view_store(a.item_end + slot + 3, q3);
      }
      if (base + nitems > cap && l == 0) atomicOr(&a.ctl->out_overflow, 1ull);
      if (sm) straddler_from_regs(bnd, a.side, S, E - S, c0 * (unsigned long long)kChunk + kChunkHdr + S);
    }
    if (l == 0) {
      if (done) {
        a.blk_status[b] = kBlkOk;
        a.blk_hdr[b] = hdr;
        a.blk_data[b] = c0 * (uint64_t)kChunk;
      } else {
        a.blk_coff[atomicAdd(&a.ctl->n_retry, 1ull)] = b;
      }
    }
  };
  unsigned long long desc = dload(wave);
  bool ok_nx = lean_ok(desc);
  uint4 w_nx, bnd_nx;
  fetch(desc, ok_nx, w_nx, bnd_nx);
  unsigned long long desc_nx = dload(wave + nwaves);
  for (uint64_t b = wave; b < nb; b += nwaves) {
    const unsigned long long desc_c = desc;
    const bool ok = ok_nx;
    const uint4 w = w_nx, bnd = bnd_nx;
    // the next block's windows and the one after's descriptor, in flight while this one is parsed
    const uint64_t bn = b + nwaves;
    ok_nx = bn < nb && lean_ok(desc_nx);
    fetch(desc_nx, ok_nx, w_nx, bnd_nx);
    desc = desc_nx;
    desc_nx = dload(bn + nwaves);
    parse_one(b, desc_c, ok, w, bnd);
  }
}

// The blocks k_parse left to the general parser (headers past the first 1 KiB,
// irregular chunk layouts, and every malformed header: parse_header computes
// the reference's error values).
// Teams of kSlowTeam waves share a group of 64 blocks, member m taking the
// group's blocks m, m + kSlowTeam, ... that k_parse marked slow: a run of slow
// blocks (every block of a file written with a large MaxItems) spreads over
// the team. A block's status is read and rewritten by the one member that owns
// its slot -- never ranked among the group's slow blocks, since the other
// members (other workgroups, dispatched at other times when another stream's
// kernels share the GPU) rewrite those statuses as they finish them.
constexpr uint32_t kSlowTeam = 16;

__global__ void __launch_bounds__(256) k_parse_slow(DevBufs d, ParseArgs a) {
  const uint64_t nb = *a.nblocks;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint64_t team = wave / kSlowTeam, nteams = nwaves / kSlowTeam;
  const uint32_t member = (uint32_t)(wave % kSlowTeam);
  const int l = lane_id();
  for (uint64_t g = team * 64; g < nb; g += nteams * 64) {
    // lane j: the member's j-th slot of the group
    const uint64_t slot = g + member + (uint64_t)kSlowTeam * l;
    const bool slow = l < (int)(64 / kSlowTeam) && slot < nb && d.blk_status[slot] == kBlkSlow;
    unsigned long long sm = __ballot(slow);
    while (sm) {
      const uint64_t b = g + member + (uint64_t)kSlowTeam * (uint64_t)(__ffsll((long long)sm) - 1);
      sm &= sm - 1;
      const uint64_t c0 = d.blk_c0[b];
      const unsigned long long meta = d.blk_meta[b];
      const uint64_t total = meta & kMetaTotalMask;
      const unsigned long long len = (a.codec == RIO_CODEC_NONE) ? d.blk_len[b] : d.blk_out_len[b];
      const Payload pl = (a.codec != RIO_CODEC_NONE) ? make_contig_payload(d.dec + d.blk_dec_off[b], len)
                                                     : desc_payload(a.span, d, c0, meta, len, d.ck_pay[c0]);
      // item-end mode, none codec, chunks other than the last short (not what
      // the writer makes, but valid): the payload is gathered whole into the
      // span-shaped side buffer at the block's own offset, where it fits
      const bool whole = a.end_mode && a.codec == RIO_CODEC_NONE && !pl.regular && total > 1;
      ParseOut po;
      po.item_off = d.item_off;
      po.item_len = d.item_len;
      po.item_end = a.end_mode ? d.item_off : nullptr;
      po.whole = whole;
      po.item_base = d.blk_item_base[b];
      po.item_cap = a.item_cap;
      po.view_base = (a.codec != RIO_CODEC_NONE) ? (kItemInRecords | d.blk_dec_off[b]) : 0;
      po.strad = d.strad;
      po.ssz = d.ck_ssz;
      po.c0 = c0;
      po.overflow = &d.ctl->out_overflow;
      const HdrResult none{};
      const HdrResult r = parse_header<kParseCount>(pl, none, po);
      if (r.status == kBlkOk) {
        if (r.nitems != d.blk_nitems[b]) {  // the reservation reads the same varint: internal error
          if (l == 0) atomicOr(&d.ctl->out_overflow, 16ull);
        } else {
          parse_header<kParseWrite>(pl, r, po);
          if (whole) {  // chunk by chunk, back to back
            uint64_t o = 0;
            for (uint64_t c = c0; c < c0 + total; c++) {
              const uint64_t n = d.ck_size[c];
              for (uint64_t k = l; k < n; k += 64) d.side[c0 * kChunk + o + k] = a.span[c * kChunk + kChunkHdr + k];
              o += n;
            }
          }
        }
      }
      if (l == 0) {
        d.blk_status[b] = r.status;
        d.blk_a[b] = r.a;
        d.blk_b[b] = r.b;
        d.blk_hdr[b] = r.hdr_len;
        if (a.end_mode && r.status == kBlkOk)
          d.blk_data[b] = (a.codec != RIO_CODEC_NONE) ? (kItemInRecords | d.blk_dec_off[b])
                          : whole                     ? (kItemInRecords | c0 * (uint64_t)kChunk)
                                                      : c0 * (uint64_t)kChunk;
        if (r.status != kBlkOk && a.mode == kModeBody) atomicMin(&d.ctl->first_block_event, 2 * (c0 + total - 1) + 1);
      }
    }
  }
}

// compressed codecs: item slots from the decoded blocks' first varint
__global__ void __launch_bounds__(256) k_dec_nitems(DevBufs d, const unsigned long long *nblocks) {
  const uint64_t nb = *nblocks;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    unsigned long long v = 0, res = 0;
    const unsigned long long len = d.blk_out_len[b];
    if (d.blk_status[b] != kBlkCodec) {
#ifdef RIO_CHECKED
      if (d.blk_dec_off[b] + (len < 10 ? len : 10) > d.dec_cap) {
        atomicOr(&d.ctl->out_overflow, 0x2000ull);
        d.blk_nitems[b] = 0;
        continue;
      }
#endif
      const uint8_t *p = d.dec + d.blk_dec_off[b];
      for (int k = 0; k < 10 && (unsigned long long)k < len; k++) {
        const uint32_t c = p[k];
        v |= (unsigned long long)(c & 0x7f) << (7 * k);
        if (c < 0x80) {
          if (!(k == 9 && c > 1) && v <= len) res = v;
          break;
        }
      }
    }
    d.blk_nitems[b] = res;
  }
}

// Straddlers recorded by the general parser (and, in compact mode, by the
// fast path): 64 chunk slots per wave, one straddler at a time gathered by the
// whole wave across the chunk header(s) into the side buffer -- at its own span
// offset (sparse) or at ck_sbase[slot] (compact) -- and the item's view set.
__global__ void __launch_bounds__(256) k_strad(const uint8_t *__restrict__ span, DevBufs d, uint64_t nslots,
                                               uint64_t side_cap, int32_t sparse, int32_t end_mode) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t c0 = wave * 64; c0 < nslots; c0 += nwaves * 64) {
    const bool has = (c0 + l < nslots) && d.ck_ssz[c0 + l] != 0;
    unsigned long long sm = __ballot(has);
    while (sm) {
      const uint64_t c = c0 + __ffsll((long long)sm) - 1;
      sm &= sm - 1;
      const StradDesc s = d.strad[c];
      const Payload pl = make_chunk_payload(span, d, s.c0, d.ck_total[s.c0]);
      uint64_t ch, lo;
      pl.chunk_of(s.src, ch, lo);
      const unsigned long long dst = sparse ? ch * kChunk + kChunkHdr + (s.src - lo) : d.ck_sbase[c];
      if (dst + pad16(s.len) > side_cap) {
        if (l == 0) atomicOr(&d.ctl->out_overflow, 4ull);
        continue;
      }
      if (l == 0 && !end_mode) d.item_off[s.item] = kItemInRecords | dst;  // (item-end mode: implied)
      // piecewise: each piece is contiguous in one chunk payload
      unsigned long long p = s.src, o = 0;
      while (o < s.len) {
        pl.chunk_of(p, ch, lo);
        const unsigned long long avail = d.ck_size[ch] - (p - lo);
        const unsigned long long n = (s.len - o) < avail ? (s.len - o) : avail;
        const uint8_t *src = span + ch * kChunk + kChunkHdr + (p - lo);
        for (unsigned long long k = l; k < n; k += 64) d.side[dst + o + k] = src[k];
        p += n;
        o += n;
      }
    }
  }
}

// ---------------------------------------------------------------- resolve
__device__ __forceinline__ void load_magic(const uint8_t *span, uint64_t ch, unsigned long long &m) {
  const uint32_t *h = reinterpret_cast<const uint32_t *>(span + ch * kChunk);
  m = (unsigned long long)h[0] | ((unsigned long long)h[1] << 32);
}

// records-buffer bytes used by the first n of nb blocks
__device__ __forceinline__ unsigned long long rec_end(const DevBufs &d, uint64_t n, uint64_t nb, uint64_t nchunks,
                                                      int codec, int sparse) {
  if (n == 0) return 0;
  if (codec != RIO_CODEC_NONE) return d.blk_dec_off[n - 1] + d.blk_out_len[n - 1];
  const uint64_t c = n < nb ? d.blk_c0[n] : nchunks;  // straddlers of the first n blocks lie before c
  return sparse ? c * kChunk : d.ck_sbase[c];
}

__global__ void k_resolve(DevBufs d, ResolveArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Ctl *c = d.ctl;
  const uint64_t nb = *a.nblocks;
  const unsigned long long ce = c->first_chunk_err < c->first_crc_err ? c->first_chunk_err : c->first_crc_err;
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
    // header / trailer block: exactly block 0 (readSpecialBlock, ReadLastBlock)
    const uint64_t total = (nb > 0) ? d.ck_total[0] : 0;
    const bool complete = nb > 0 && d.blk_c0[0] == 0 && total != 0 && total <= a.nchunks;
    const uint64_t end = complete ? total - 1 : a.nchunks;
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
    // the span running out: after every chunk in it -- the reference reads an
    // unfinished block's chunks one by one, so a chunk error inside the span
    // (a total of 0, a block start where the block goes on) comes first
    const unsigned long long tail = 2 * a.nchunks;
    if (tail < key) {
      key = tail;
      kind = 4;
    }
    // blocks finished strictly before the stop
    uint64_t lo = 0, hi = nb;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) / 2;
      if (2 * d.blk_c0[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    nvalid = lo;
    if (nvalid > 0) {
      const uint64_t c0 = d.blk_c0[nvalid - 1];
      const uint64_t total = d.ck_total[c0];
      if (total == 0 || 2 * (c0 + total - 1) + 1 >= key) nvalid--;
    }
    if (kind == 3) {
      const uint64_t chunk = (bev & 1) ? (bev - 1) / 2 : bev / 2;
      const uint32_t b = d.ck_block[chunk];
      c->stop_block = (b != kNoBlockId && b < nb) ? b : 0;
    }
  }
  c->stop_key = key;
  c->n_valid_blocks = nvalid;
  c->n_items = d.blk_item_base[nvalid];
  c->rec_bytes = rec_end(d, nvalid, nb, a.nchunks, a.codec, a.sparse);
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
  if (c->stop_block != kNone && nb > 0) {
    const uint64_t b = c->stop_block;
    c->blk_status = d.blk_status[b];
    c->blk_a = d.blk_a[b];
    c->blk_b = d.blk_b[b];
    c->blk_c0 = d.blk_c0[b];
    load_magic(a.span, c->blk_c0, c->mag_blk);
  }
}

// ---------------------------------------------------------------- launchers
static inline unsigned grid_of(uint64_t n, unsigned per, unsigned cap) {
  uint64_t g = (n + per - 1) / per;
  if (g < 1) g = 1;
  return (unsigned)(g > cap ? cap : g);
}

void launch_parse(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_parse, dim3(grid_of(max_blocks, 4 * kBatch, RIO_PARSE_GRID)), dim3(256), 0, st, d, a);
}

// one resident round of a kernel: workgroups per CU at this build's occupancy x
// CUs (a function-local static: initialised once, thread-safe -- the scanner's
// span-ahead threads launch concurrently)
template <class K>
static unsigned resident_round(K kernel, int threads) {
  int per_cu = 0, dev = 0, ncu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1) per_cu = 4;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1)
    ncu = 256;
  return (unsigned)(per_cu * ncu);
}

void launch_lean_end(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st) {
  static const unsigned cap = resident_round(k_lean_end, 256);
  LeanArgs la{a.span, d.blk_c0, d.blk_meta, d.blk_len, d.blk_item_base, d.blk_status, d.blk_hdr, d.blk_data,
              d.blk_coff, d.item_off, d.side, d.ctl, a.nblocks, a.limit_chunk, a.item_cap};
  hipLaunchKernelGGL(k_lean_end, dim3(grid_of(max_blocks, 4, cap)), dim3(256), 0, st, la);
}

void launch_parse_lean(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st) {
  static const unsigned cap = resident_round(k_parse_lean, 256);
  hipLaunchKernelGGL(k_parse_lean, dim3(grid_of(max_blocks, 4 * kLeanBatch, cap)), dim3(256), 0, st, d, a);
}

void launch_parse_slow(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st) {
  // whole teams: 4 waves per workgroup, kSlowTeam waves per team
  unsigned g = grid_of(max_blocks, 16, 2048);
  g = (g + kSlowTeam / 4 - 1) / (kSlowTeam / 4) * (kSlowTeam / 4);
  hipLaunchKernelGGL(k_parse_slow, dim3(g), dim3(256), 0, st, d, a);
}

void launch_dec_nitems(const DevBufs &d, const unsigned long long *nblocks, uint64_t max_blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_dec_nitems, dim3(grid_of(max_blocks, 256, 1024)), dim3(256), 0, st, d, nblocks);
}

void launch_strad(const uint8_t *span, const DevBufs &d, uint64_t nslots, uint64_t side_cap, int32_t sparse, int32_t end_mode,
                  hipStream_t st) {
  hipLaunchKernelGGL(k_strad, dim3(grid_of(nslots, 256, 1024)), dim3(256), 0, st, span, d, nslots, side_cap, sparse, end_mode);
}

void launch_resolve(const DevBufs &d, const ResolveArgs &a, hipStream_t st) {
  hipLaunchKernelGGL(k_resolve, dim3(1), dim3(64), 0, st, d, a);
}

// Segment scans (rio_scan_device_segments_async): each valid block's file
// (the segment holding its first chunk) and its offset in that file.
__global__ void __launch_bounds__(256) k_block_files(DevBufs d, const unsigned long long *seg_end,
                                                     const unsigned long long *seg_file_off, uint64_t nseg) {
  const uint64_t nb = d.ctl->n_valid_blocks;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long off = d.blk_c0[b] * (unsigned long long)kChunk;
    uint64_t lo = 0, hi = nseg;  // first segment whose end is past off
    while (lo < hi) {
      const uint64_t m = (lo + hi) >> 1;
      if (seg_end[m] <= off) lo = m + 1;
      else hi = m;
    }
    const unsigned long long s0 = lo ? seg_end[lo - 1] : 0;
    d.blk_seg[b] = lo;
    d.blk_file_off[b] = (lo < nseg ? seg_file_off[lo] : 0) + (off - s0);
  }
}

void launch_block_files(const DevBufs &d, const unsigned long long *seg_end, const unsigned long long *seg_file_off,
                        uint64_t nseg, uint64_t max_blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_block_files, dim3(grid_of(max_blocks, 256, 2048)), dim3(256), 0, st, d, seg_end, seg_file_off,
                     nseg);
}

}  // namespace rio
