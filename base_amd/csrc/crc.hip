// Chunk CRC32-IEEE verify (readChunk, recordio/internal/chunk.go:338-343) at
// HBM read speed, no carry-less multiply.
//
// One wave per 32 KiB chunk, kCrcWaves (16) waves per workgroup, one workgroup per CU.
// Lane t loads the 16-byte units at chunk offsets 1024*i + 16*t (i = 0..31): every
// load instruction is 1 KiB contiguous. Each of the lane's 4 dwords (k = 0..3)
// is its own CRC stream with one dword per 1 KiB row; the 1020-byte gap to the
// stream's next dword is folded into the tables, so one step is
//   S_k <- fold0[b0] ^ fold1[b1] ^ fold2[b2] ^ fold3[b3],  b = bytes of (u_k ^ S_k),
//   fold_j[b] = R(b || 0^(1023-j))     (R = raw CRC: zero init, no final xor).
// Only 4 fold tables exist, so each is replicated 16x in LDS (64 KiB): lane l
// reads copy l & 15 (32 copies, 128 KiB, made every read conflict-free but left
// no room on the CU for anything else). A row's 16
// lookups are independent and issue back to back; only the row-to-row chain
// per stream is serial. Round 5: the tables in byte rows (entry b of table j,
// copy c at byte 256 b + 64 j + 4 c, from LDS address 0), so a lookup's address
// is one v_perm_b32 of the data and the lane's offsets, and the XORs are
// 3-input v_bitop3_b32 (crc_fold.h fold_row3): 24 VALU instructions per 1 KiB
// row where there were 52 (2.84 -> 2.67 ms per C2 launch).
// After row 31, stream (t, k) holds R(message) * x^(8(16t + 4k)); the lane
// combines its streams with x^-32 (Horner), a 6-level shuffle tree with
// x^-(128*2^l) combines the lanes (multiply-by-constant = 4 byte lookups).
// Bytes outside [12, 28+size) are zeroed, so V = R(0^12 || covered || 0^pad) and
// crc = ~(~0 * x^(8(16+size)) ^ V * x^(-8 pad)).
// Loads are software-pipelined in 2 KiB stages through 8 register buffers:
// while one stage is folded the next seven are in flight (16 waves per CU keep
// 224 KiB outstanding). Round 6, with the lookups conflict-free (fold_sel): 16
// waves of 2-row stages, 8 buffers, against 12 waves of 4-row stages, 4 buffers:
// two-context C2 step 2.846-2.857 -> 2.820-2.824 ms, k_crc 2.625-2.635 ->
// 2.615-2.628 (profiles/r06_crc_shape_ab2.jsonl); 12 waves of 2-row stages, 8
// buffers ran k_crc in 2.55-2.58 ms alone but the step in 2.87-2.91.
//
// Room beside it (round 4): the tables are dynamic LDS (92 KiB) and the
// registers are allocated for 4 waves per SIMD (127 VGPRs) while the workgroup
// has 12 waves (3 per SIMD) -- with static LDS the compiler sizes registers for
// the 3 waves per SIMD the LDS allows (167 VGPRs) -- so one workgroup of another
// kernel (k_lean_end: 6 KiB of LDS, 71 VGPRs per wave) fits on each CU beside
// it: with two contexts in flight, step i + 1's parse runs during step i's
// CRC pass (C2, A/B on one box: 3.114 -> 3.043 ms per step; alone k_crc 2.785
// -> 2.75 ms). (Round 6: at 16 waves the registers fill the SIMDs; the parse
// kernels then take CU slots as k_crc's waves finish.)
//
// Fused parse (k_crc<true>, round 2; measured slower and not instantiated:
// DESIGN.md §5; none codec): the wave that checksums a block's
// first chunk also parses the block (parse_block.h: magic handling, the
// varint header, one view per item, straddler copies). The header window --
// payload bytes 0..1023 = chunk bytes 28..1051 -- is taken from the rows the
// wave already holds (row 0 and the first 32 bytes of row 1, staged in LDS),
// and the block descriptor comes through scalar loads, so the parse issues no
// vector load that would wait behind the next chunk's prefetched rows; it runs
// while those rows are in flight. One pass over the span replaces the CRC
// pass + the separate parse pass.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_fold.h"
#include "device_common.h"
#include "parse_block.h"
#include "rio_internal.h"

namespace rio {

#ifndef RIO_CRC_WAVES
#define RIO_CRC_WAVES 16
#endif
constexpr int kCrcWaves = RIO_CRC_WAVES;  // waves per workgroup (one workgroup per CU: 92 KiB LDS at 16 copies, 127 VGPRs)

#ifndef RIO_CRC_MAP
#define RIO_CRC_MAP 0
#endif
#ifndef RIO_CRC_ROWS
#define RIO_CRC_ROWS 2
#endif
constexpr int kRows = RIO_CRC_ROWS;  // rows per pipeline stage (2 KiB per wave)
#ifndef RIO_CRC_BUFS
#define RIO_CRC_BUFS 8
#endif
constexpr int kBufs = RIO_CRC_BUFS;  // register buffers: kBufs - 1 stages in flight during a fold
constexpr int kStages = 32 / kRows;
static_assert(kStages % kBufs == 0, "a chunk's stages must cycle through the buffers evenly");

// the fold tables at LDS address 0 (dynamic LDS, no static LDS in k_crc<false>;
// k_crc checks it): byte-row lookups use their v_perm address as is
#ifndef RIO_CRC_DYN
#define RIO_CRC_DYN 1
#endif
constexpr bool kCrcAbs = kFoldPerm && RIO_CRC_DYN;

// fold stage q (rows kRows*q ..) of a chunk whose covered bytes end at `end`
__device__ __forceinline__ void fold_stage(const uint4 (&u)[kRows], uint32_t (&s)[4], uint32_t (&sq)[4],
                                           const char *__restrict__ tab, uint32_t lb, const uint32_t (&sel)[4],
                                           int l, int q, int end, bool fold, uint32_t &stored) {
#pragma unroll
  for (int r = 0; r < kRows; r++) {
    uint4 v = u[r];
    const int row = kRows * q + r;
    if (row == 0) {  // magic[0:8] and crc[8:12] are not covered
      stored = v.z;  // lane 0: the chunk's stored checksum
      const uint32_t keep = (l == 0) ? 0u : 0xffffffffu;
      v.x &= keep;
      v.y &= keep;
      v.z &= keep;
    }
    if (1024 * (row + 1) > end) {  // wave-uniform: only rows reaching the payload end
      const int o = 1024 * row + 16 * l;
      v.x = mask_dword(v.x, o, end);
      v.y = mask_dword(v.y, o + 4, end);
      v.z = mask_dword(v.z, o + 8, end);
      v.w = mask_dword(v.w, o + 12, end);
    }
    if (fold) {
#if RIO_FOLD_XOR3
      if constexpr (kFoldPerm) fold_row3<kCrcAbs>(tab, lb, v, s, sq, sel);
      else fold_row<kCrcAbs>(tab, lb, v, s);
#else
      fold_row<kCrcAbs>(tab, lb, v, s);
#endif
    } else {  // ablation: keep the loads live
      s[0] ^= v.x;
      s[1] ^= v.y;
      s[2] ^= v.z;
      s[3] ^= v.w;
    }
  }
}

__device__ __forceinline__ void load_stage(uint4 (&u)[kRows], const uint8_t *ck, int q, int l) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 *row = reinterpret_cast<const u32x4 *>(ck) + 64 * kRows * q + l;
#pragma unroll
  for (int r = 0; r < kRows; r++) {
    const u32x4 x = __builtin_nontemporal_load(row + 64 * r);
    u[r] = make_uint4(x.x, x.y, x.z, x.w);
  }
}

// sizes / fix tables (and the fused parse's descriptors) are separate
// restrict-const arguments so that their wave-uniform reads compile to scalar
// loads (a vector load of the next chunk's size would make the wave drain its
// prefetched rows)
struct CrcParseIn {
  const uint32_t *__restrict__ ck_index;
  const uint32_t *__restrict__ ck_block;
  const unsigned long long *__restrict__ blk_meta;
  const unsigned long long *__restrict__ blk_len;
  const unsigned long long *__restrict__ blk_item_base;
  const unsigned long long *__restrict__ ck_pay;
};
constexpr int kStageBytes = 1088;  // payload window staging: row 0 + 32 B of row 1 (then reused as the window)

// the tables in dynamic LDS, so that the compiler sizes registers for
// RIO_CRC_WPE waves per SIMD instead of the occupancy the static LDS allows
#ifndef RIO_CRC_DYN
#define RIO_CRC_DYN 1
#endif
#ifndef RIO_CRC_WPE
#define RIO_CRC_WPE 4
#endif
#if RIO_CRC_DYN
#define RIO_CRC_ATTR __attribute__((amdgpu_waves_per_eu(RIO_CRC_WPE)))
#else
#define RIO_CRC_ATTR
#endif
constexpr size_t kCrcDynLds = RIO_CRC_DYN ? 4 * (size_t)(kFoldWords + kMulTables * 1024) : 0;

template <bool kParse>
__global__ void __launch_bounds__(64 * kCrcWaves) RIO_CRC_ATTR k_crc(const uint8_t *__restrict__ span, uint64_t nchunks,
                                                       const uint32_t *__restrict__ ck_size,
                                                       const uint32_t *__restrict__ fix_a,
                                                       const uint32_t *__restrict__ fix_b, DevBufs d, CrcArgs ca,
                                                       CrcParseIn pin, ParseArgs pa) {
#if RIO_CRC_DYN
  extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
  uint32_t *const s_fold = s_dyn;
  uint32_t *const s_mul = s_dyn + kFoldWords;
#else
  __shared__ __attribute__((aligned(16))) uint32_t s_fold[kFoldWords];
  __shared__ __attribute__((aligned(16))) uint32_t s_mul[kMulTables * 1024];
#endif
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[kParse ? kCrcWaves : 1][kParse ? kStageBytes : 16];
  __shared__ __attribute__((aligned(16))) uint16_t s_tpos[kParse ? kCrcWaves : 1][kParse ? 1024 : 1];
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(d.crc_fold);
    uint4 *dst = reinterpret_cast<uint4 *>(s_fold);
    for (int i = threadIdx.x; i < kFoldWords / 4; i += blockDim.x) dst[i] = src[i];
    for (int i = threadIdx.x; i < kMulTables * 1024; i += blockDim.x) s_mul[i] = d.crc_mul[i];
  }
  __syncthreads();
  if constexpr (kCrcAbs) {  // (a static LDS variable would move the tables: fail loudly)
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    if ((uint32_t)(uintptr_t)(lds_u32 *)s_fold != 0u) {
      if (threadIdx.x == 0) atomicOr(&d.ctl->out_overflow, kOvfLayout);
      return;
    }
  }
  const int l = lane_id();
  const uint32_t lb = (uint32_t)(l & (kFoldCopies - 1)) << 2;
  // lanes 16-31 / 48-63 take their lookups in rotated table order (crc_fold.h fold_sel)
#ifndef RIO_CRC_ROT
#define RIO_CRC_ROT 1
#endif
  const uint32_t rot = RIO_CRC_ROT ? (uint32_t)((l >> 4) & 1) : 0u;
  const uint32_t sel[4] = {fold_sel(0, rot), fold_sel(1, rot), fold_sel(2, rot), fold_sel(3, rot)};
  const char *tab = reinterpret_cast<const char *>(s_fold);
  const bool fold = !(ca.flags & 1);
  const uint64_t nwaves = (uint64_t)gridDim.x * kCrcWaves;
  // wave-uniform chunk index: sizes are scalar loads and the FULL test a scalar branch
#if RIO_CRC_MAP  // (wave-major: a CU's waves read chunks gridDim.x apart)
  uint64_t c = (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * gridDim.x + blockIdx.x;
#else
  uint64_t c = (uint64_t)blockIdx.x * kCrcWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#endif
  if (c >= nchunks) return;
  uint4 buf[kBufs][kRows];
  uint8_t *stage = kParse ? s_stage[threadIdx.x >> 6] : nullptr;
  uint16_t *tpos = kParse ? s_tpos[threadIdx.x >> 6] : nullptr;
  uint32_t size = ck_size[c];
#pragma unroll
  for (int q = 0; q < kBufs - 1; q++) load_stage(buf[q], span + c * kChunk, q, l);
  for (;;) {
    const uint8_t *ck = span + c * kChunk;
    const uint64_t cn = c + nwaves;
    const bool more = cn < nchunks;
    const uint32_t size_n = ck_size[more ? cn : c];
    const uint32_t sz = size > (uint32_t)kMaxPayload ? (uint32_t)kMaxPayload : size;
    const int end = kChunkHdr + (int)sz;
    const bool full = (sz == (uint32_t)kMaxPayload);
    // a block starts here: this wave parses it after the checksum (scalar load)
    const bool starts = kParse && pin.ck_index[c] == 0;
    uint32_t s[4] = {0, 0, 0, 0}, sq[4] = {0, 0, 0, 0};
    uint32_t stored = 0;
    const uint32_t fa = fix_a[sz], fb = fix_b[sz];
#pragma unroll
    for (int q = 0; q < kStages; q++) {
      const int nq = q + kBufs - 1;  // stage to prefetch (this chunk or the next)
      if (nq < kStages) load_stage(buf[nq % kBufs], ck, nq, l);
      else if (more) load_stage(buf[nq % kBufs], span + cn * kChunk, nq - kStages, l);
      if (kParse && q == 0 && starts) {  // rows 0..1 raw, before the fold masks them
        *reinterpret_cast<uint4 *>(stage + 16 * l) = buf[0][0];
        if (l < 2) *reinterpret_cast<uint4 *>(stage + 1024 + 16 * l) = buf[0][1];
      }
      fold_stage(buf[q % kBufs], s, sq, tab, lb, sel, l, q, end, fold, stored);
    }
    // lane: V_t = s0 + s1 x^-32 + s2 x^-64 + s3 x^-96
#pragma unroll
    for (int k = 0; k < 4; k++) s[k] ^= sq[k];  // (fold_row3's unfolded part)
    uint32_t v = mul_const(s_mul, s[3]) ^ s[2];
    v = mul_const(s_mul, v) ^ s[1];
    v = mul_const(s_mul, v) ^ s[0];
    // lanes: V = sum_t V_t x^-128t
#pragma unroll
    for (int lv = 0; lv < 6; lv++) {
      const uint32_t m = mul_const(s_mul + (lv + 1) * 1024, v);
      const int step = 1 << lv;
      const uint32_t o = __shfl(m, (l + step) & 63, 64);
      v ^= (l + step < 64) ? o : 0u;
    }
    if (l == 0 && size <= (uint32_t)kMaxPayload) {  // "Invalid chunk size": no CRC
      const uint32_t t = full ? v : gf_mul_dev(v, fb);
      const uint32_t crc = ~(fa ^ t);
      d.ck_crc[c] = crc;
      // (flags & 2: the encode path computes CRCs of chunks it is writing -- no compare)
      if (crc != stored && fold && !(ca.flags & 2)) atomicMin(&d.ctl->first_crc_err, (unsigned long long)c);
    }
    if (kParse && starts) {
      const uint32_t b = pin.ck_block[c];
      const unsigned long long meta = pin.blk_meta[b], len = pin.blk_len[b];
      const unsigned long long base = pin.blk_item_base[b], pay0 = pin.ck_pay[c];
      // the header window: payload bytes 16l .. 16l+15 (0x80: past the first chunk's payload)
      uint32_t win[4] = {0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u};
      const uint64_t size0 = len < (uint64_t)kMaxPayload ? len : (uint64_t)kMaxPayload;
      if ((meta & kMetaComplete) && 16ull * l + 16 <= size0) {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(stage + kChunkHdr + 16 * l);
        win[0] = q[0];
        win[1] = q[1];
        win[2] = q[2];
        win[3] = q[3];
      }
      parse_block(d, pa, b, c, meta, len, base, pay0, win, stage, tpos);
    }
    if (!more) break;
    c = cn;
    size = size_n;
  }
}

void launch_crc(const uint8_t *span, uint64_t nchunks, const DevBufs &d, const CrcArgs &ca, int ncu,
                hipStream_t st) {
  uint64_t g = (nchunks + kCrcWaves - 1) / kCrcWaves;
  const uint64_t cap = (uint64_t)(ncu > 0 ? ncu : 256);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  const CrcParseIn pin{d.ck_index, d.ck_block, d.blk_meta, d.blk_len, d.blk_item_base, d.ck_pay};
  hipLaunchKernelGGL(k_crc<false>, dim3((unsigned)g), dim3(64 * kCrcWaves), kCrcDynLds, st, span, nchunks, d.ck_size,
                       d.crc_fix_a, d.crc_fix_b, d, ca, pin, ParseArgs{});
}

}  // namespace rio
