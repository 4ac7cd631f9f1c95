// The per-block step of parseChunksToItems on the GPU (scannerv2.go:53-97,
// 363-388): block magic handling, the fast header parse and the item views of
// one block by one wave. Shared by k_parse (blocks.hip: compressed codecs,
// after the decode) and the fused k_crc (crc.hip: none codec, the block's
// first chunk is parsed by the wave that has just checksummed it).
#pragma once
#include "device_common.h"

namespace rio {

__device__ __forceinline__ Payload desc_payload(const uint8_t *span, const DevBufs &d, uint64_t c0,
                                                unsigned long long meta, unsigned long long len,
                                                unsigned long long pay0) {
  Payload pl;
  pl.span = span;
  pl.ck_size = d.ck_size;
  pl.ck_pay = d.ck_pay;
  pl.c0 = c0;
  pl.total = meta & kMetaTotalMask;
  pl.pay0 = pay0;
  pl.len = len;
  pl.regular = (meta & kMetaRegular) != 0;
  pl.contig = nullptr;
  return pl;
}

// Block b (first chunk c0, descriptor meta/len, item slots from base): its
// status, and for a packed block whose header fits the 1 KiB window `win`
// (lane l: payload bytes 16l .. 16l+15) its item views. Lane 0 records the
// status and the block's first-event key; headers the fast path declines are
// left to k_parse_slow (kBlkSlow).
__device__ __forceinline__ void parse_block(const DevBufs &d, const ParseArgs &a, uint64_t b, uint64_t c0,
                                            unsigned long long meta, unsigned long long len,
                                            unsigned long long base, unsigned long long pay0,
                                            const uint32_t (&win)[4], uint8_t *lwin, uint16_t *ltpos) {
  const int l = lane_id();
  const uint64_t total = meta & kMetaTotalMask;
  const uint32_t cls = (uint32_t)(meta >> kMetaClsShift) & 0xffu;
  unsigned long long status = kBlkOk, ea = 0, eb = 0, hdr = 0;
  unsigned long long event = kNone;
  if (c0 >= a.limit_chunk && a.mode == kModeBody) {
    status = kBlkLimit;
    event = 2 * c0;
  } else if (!(meta & kMetaComplete)) {
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
    if (parse && a.no_items) {
      parse = false;  // a chain's earlier stage: decoded, not parsed (status ok)
    } else if (parse) {
      Payload pl = (a.codec != RIO_CODEC_NONE) ? make_contig_payload(d.dec + d.blk_dec_off[b], len)
                                               : desc_payload(a.span, d, c0, meta, len, pay0);
      ParseOut po;
      po.item_off = d.item_off;
      po.item_len = d.item_len;
      po.item_end = a.end_mode ? d.item_off : nullptr;
      po.whole = false;
      po.item_base = base;
      po.item_cap = a.item_cap;
      po.view_base = (a.codec != RIO_CODEC_NONE) ? (kItemInRecords | d.blk_dec_off[b]) : 0;
      po.strad = d.strad;
      po.ssz = d.ck_ssz;
      po.c0 = c0;
      po.overflow = &d.ctl->out_overflow;
      HdrResult r{};
      if (fast_header(pl, win, r, po, lwin, ltpos, a.sparse ? d.side : nullptr)) {
        status = r.status;
        hdr = r.hdr_len;
      } else {
        status = kBlkSlow;  // k_parse_slow finishes the block (and its event)
      }
    }
    if (status != kBlkOk && status != kBlkSlow && a.mode == kModeBody) event = 2 * end + 1;
  }
  if (l == 0) {
    d.blk_status[b] = status;
    d.blk_a[b] = ea;
    d.blk_b[b] = eb;
    d.blk_hdr[b] = hdr;
    if (a.end_mode && status == kBlkOk)
      d.blk_data[b] = (a.codec != RIO_CODEC_NONE) ? (kItemInRecords | d.blk_dec_off[b]) : c0 * (uint64_t)kChunk;
    if (event != kNone) atomicMin(&d.ctl->first_block_event, event);
  }
}

}  // namespace rio
