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
#include "rio_internal.h"

namespace rio {

constexpr uint32_t kNoBlockId = 0xffffffffu;

__device__ __forceinline__ bool block_complete(const DevBufs &d, uint64_t c0, uint64_t nchunks, uint64_t &total) {
  total = d.ck_total[c0];
  return total != 0 && c0 + total <= nchunks;
}

__device__ __forceinline__ Payload block_payload(const DevBufs &d, const ParseArgs &a, uint64_t b, uint64_t c0,
                                                 uint64_t total) {
  if (a.codec != RIO_CODEC_NONE) return make_contig_payload(d.dec + d.blk_dec_off[b], d.blk_out_len[b]);
  return make_chunk_payload(a.span, d, c0, total);
}

// wave per block: block magic handling (scannerv2.go:374-387) + header counts
__global__ void __launch_bounds__(256) k_block_parse(DevBufs d, ParseArgs a) {
  const uint64_t nb = *a.nblocks;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t b = wave; b < nb; b += nwaves) {
    const uint64_t c0 = d.blk_c0[b];
    uint64_t total;
    unsigned long long status = kBlkOk, ea = 0, eb = 0, nitems = 0, hdr = 0, sb = 0, sn = 0;
    const uint32_t cls = d.ck_info[c0] & 0xff;
    const bool complete = block_complete(d, c0, a.nchunks, total);
    unsigned long long event = kNone;
    if (c0 >= a.limit_chunk && a.mode == kModeBody) {
      status = kBlkLimit;
      event = 2 * c0;
    } else if (!complete) {
      status = kBlkIncomplete;
      if (l == 0) atomicMin(&d.ctl->first_incomplete, (unsigned long long)c0);
    } else {
      const uint64_t end = c0 + total - 1;
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
        const Payload pl = block_payload(d, a, b, c0, total);
        const HdrResult none{};
        const ParseOut po{};
        HdrResult r{};
        if (fast_header<kParseCount>(pl, r, po)) {
          sb = r.strad_bytes;
          sn = r.strad_count;
        } else {
          r = parse_header<kParseCount>(pl, none, po);
          if (r.status == kBlkOk && a.codec == RIO_CODEC_NONE && total > 1 && r.nitems > 0) {
            const HdrResult s = parse_header<kParseStrad>(pl, r, po);
            sb = s.strad_bytes;
            sn = s.strad_count;
          }
        }
        status = r.status;
        ea = r.a;
        eb = r.b;
        nitems = r.nitems;
        hdr = r.hdr_len;
      }
      if (status != kBlkOk && a.mode == kModeBody) event = 2 * end + 1;
    }
    if (l == 0) {
      d.blk_status[b] = status;
      d.blk_a[b] = ea;
      d.blk_b[b] = eb;
      d.blk_nitems[b] = (status == kBlkOk) ? nitems : 0;
      d.blk_hdr[b] = hdr;
      d.blk_sb[b] = (status == kBlkOk) ? sb : 0;
      d.blk_sn[b] = (status == kBlkOk) ? sn : 0;
      if (event != kNone) atomicMin(&d.ctl->first_block_event, event);
    }
  }
}

// wave per block: item views + straddler descriptors (cumSize, scannerv2.go:83-91)
__global__ void __launch_bounds__(256) k_items(DevBufs d, ParseArgs a) {
  const uint64_t nb = *a.nblocks;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t b = wave; b < nb; b += nwaves) {
    if (d.blk_status[b] != kBlkOk || d.blk_nitems[b] == 0) continue;
    const uint64_t c0 = d.blk_c0[b];
    const uint64_t total = d.ck_total[c0];
    const Payload pl = block_payload(d, a, b, c0, total);
    HdrResult known{};
    known.nitems = d.blk_nitems[b];
    known.hdr_len = d.blk_hdr[b];
    ParseOut po;
    po.item_off = d.item_off;
    po.item_len = d.item_len;
    po.item_base = d.blk_item_base[b];
    po.item_cap = a.item_cap;
    po.view_base = (a.codec != RIO_CODEC_NONE) ? (kItemInRecords | d.blk_dec_off[b]) : 0;
    po.strad = d.strad;
    po.strad_idx = d.blk_sn_base[b];
    po.side_base = d.blk_sb_base[b];
    po.c0 = c0;
    po.overflow = &d.ctl->out_overflow;
    if (a.codec == RIO_CODEC_NONE && po.side_base + d.blk_sb[b] > a.side_cap) {
      if (lane_id() == 0) atomicOr(&d.ctl->out_overflow, 4ull);
      continue;
    }
    HdrResult r{};
    if (!fast_header<kParseWrite>(pl, r, po)) parse_header<kParseWrite>(pl, known, po);
  }
}

// wave per straddling item: gather its bytes across the chunk header into side
__global__ void __launch_bounds__(256) k_strad(const uint8_t *__restrict__ span, DevBufs d,
                                               const unsigned long long *nblocks_dev, uint64_t side_cap) {
  const uint64_t n = d.blk_sn_base[*nblocks_dev];  // straddlers of all blocks
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  for (uint64_t i = wave; i < n; i += nwaves) {
    const StradDesc s = d.strad[i];
    if (s.dst + pad16(s.len) > side_cap) continue;
    const Payload pl = make_chunk_payload(span, d, s.c0, d.ck_total[s.c0]);
    for (uint64_t x = 16ull * l; x < s.len; x += 1024) {
      uint32_t w[4] = {0, 0, 0, 0};
      const uint64_t m = (s.len - x) < 16 ? (s.len - x) : 16;
      for (uint64_t k = 0; k < m; k++) w[k >> 2] |= pl.byte_at(s.src + x + k) << (8 * (k & 3));
      *reinterpret_cast<uint4 *>(d.side + s.dst + x) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// ---------------------------------------------------------------- resolve
__device__ __forceinline__ void load_magic(const uint8_t *span, uint64_t ch, unsigned long long &m) {
  const uint32_t *h = reinterpret_cast<const uint32_t *>(span + ch * kChunk);
  m = (unsigned long long)h[0] | ((unsigned long long)h[1] << 32);
}

// records-buffer bytes used by the first n blocks
__device__ __forceinline__ unsigned long long rec_end(const DevBufs &d, uint64_t n, int codec) {
  if (n == 0) return 0;
  if (codec != RIO_CODEC_NONE) return d.blk_dec_off[n - 1] + d.blk_out_len[n - 1];
  return d.blk_sb_base[n];
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
  c->rec_bytes = rec_end(d, nvalid, a.codec);
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

void launch_block_parse(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_block_parse, dim3(grid_of(max_blocks, 4, 4096)), dim3(256), 0, st, d, a);
}

void launch_items(const DevBufs &d, const ParseArgs &a, uint64_t max_blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_items, dim3(grid_of(max_blocks, 4, 4096)), dim3(256), 0, st, d, a);
}

void launch_strad(const uint8_t *span, const DevBufs &d, const unsigned long long *nblocks_dev, uint64_t max_strad,
                  uint64_t side_cap, hipStream_t st) {
  hipLaunchKernelGGL(k_strad, dim3(grid_of(max_strad, 4, 2048)), dim3(256), 0, st, span, d, nblocks_dev, side_cap);
}

void launch_resolve(const DevBufs &d, const ResolveArgs &a, hipStream_t st) {
  hipLaunchKernelGGL(k_resolve, dim3(1), dim3(64), 0, st, d, a);
}

}  // namespace rio
