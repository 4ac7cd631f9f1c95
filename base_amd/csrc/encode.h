// Writer encode path (encode.hip, deflate_enc.hip; driver in pipeline.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rio {

struct EncArgs {
  const uint8_t *data;                  // item bytes, back to back
  const unsigned long long *item_end;   // exclusive ends (n_items)
  uint64_t n_items;
  uint64_t per_block;                   // items per block (the writer's MaxItems + 1)
  uint64_t nblocks;
  int32_t codec;
  int32_t level;
  unsigned long long magic;             // block magic, little-endian
  // per block (nblocks + 1)
  unsigned long long *hdr_len, *hdr_off, *pay_len, *nck, *ck0, *comp_off;
  uint8_t *hdr;                         // varint headers
  uint8_t *comp;                        // transformed payloads (flate)
  // per chunk
  uint32_t *ck_block;
  uint8_t *out;
};

void launch_enc_count(const EncArgs &a, hipStream_t st);
void launch_enc_header(const EncArgs &a, hipStream_t st);
void launch_enc_nck(const EncArgs &a, hipStream_t st);
void launch_enc_ckmap(const EncArgs &a, hipStream_t st);
// k_crc's tables (DevBufs::crc_*)
struct CrcTabs {
  const uint32_t *fold, *mul, *fix_a, *fix_b;
};
void launch_enc_chunks(const EncArgs &a, uint64_t nchunks, const CrcTabs &t, int ncu, hipStream_t st);
void launch_deflate_bound(const EncArgs &a, hipStream_t st);
// level 0 stored, 1 fixed Huffman, others (the default -1 included) dynamic
// Huffman, which needs scratch of deflate_scratch_words(ncu) u64
uint64_t deflate_scratch_words(int ncu);
void launch_deflate(const EncArgs &a, unsigned long long *scratch, int ncu, hipStream_t st);
// zstd (zstd_enc.hip): tables of the predefined sequence codes (ZeTabs,
// zstd_enc.h), scratch of zstd_enc_scratch_words(ncu) u64
struct ZeTabs;
void launch_zstd_enc_bound(const EncArgs &a, hipStream_t st);
uint64_t zstd_enc_scratch_words(int ncu);
void launch_zstd_enc(const EncArgs &a, const ZeTabs *tabs, unsigned long long *scratch, int ncu, hipStream_t st);
void launch_enc_boff(const unsigned long long *ck0, unsigned long long *boff, uint64_t nblocks, hipStream_t st);

}  // namespace rio
