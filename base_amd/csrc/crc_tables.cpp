// GF(2) arithmetic of the reflected CRC-32 (IEEE, hash/crc32 as used by
// recordio/internal/magic.go:39) and the constant tables of the chunk CRC
// kernel (see kernels.hip: k_crc_copy for the algorithm these tables serve).
//
// Representation: bit 31 is the x^0 coefficient (reflected), polynomial
// 0xEDB88320. R(M) = raw CRC of M with zero init and no final xor; it is
// linear: R(A||B) = R(A)*x^(8|B|) xor R(B), and crc(M) = ~(~0*x^(8|M|) xor R(M)).
#include <stdint.h>
#include <string.h>

#include "rio_internal.h"

namespace rio {

uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    if (m == 0) break;
    b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

static uint32_t gf_pow(uint32_t base, uint64_t e) {
  uint32_t r = 1u << 31;  // 1
  while (e) {
    if (e & 1) r = gf_mul(r, base);
    base = gf_mul(base, base);
    e >>= 1;
  }
  return r;
}

uint32_t gf_xpow8(int64_t nbytes) {
  const uint32_t x = 1u << 30;  // x^1
  // x^-1: undo one multiply-by-x step (bit 31 of the product tells the carry)
  const uint32_t one = 1u << 31;
  const uint32_t xinv = ((one ^ kPoly) << 1) | 1u;
  if (nbytes >= 0) return gf_pow(x, 8ull * (uint64_t)nbytes);
  return gf_pow(xinv, 8ull * (uint64_t)(-nbytes));
}

static uint32_t byte_table(uint32_t b) {
  uint32_t c = b;
  for (int k = 0; k < 8; k++) c = (c & 1) ? kPoly ^ (c >> 1) : c >> 1;
  return c;
}

uint32_t crc32_host(const uint8_t *p, size_t n) {
  uint32_t c = ~0u;
  for (size_t i = 0; i < n; i++) c = byte_table((c ^ p[i]) & 0xff) ^ (c >> 8);
  return ~c;
}

void build_crc_tables(uint32_t *fold, uint32_t *mul, uint32_t *fix_a, uint32_t *fix_b) {
  // fold[j][b] = R(b || 0^(1023-j)): a dword stream with one dword per 1 KiB
  // row, the 1020-byte gap to its next dword folded into the table (one Horner
  // step per lookup set). Each table is stored x32, entry b of copy k at word
  // (j*256 + b)*32 + k, so lane l reading copy (l & 31) always hits bank l & 31.
  for (int j = 0; j < 4; j++) {
    const uint32_t sh = gf_xpow8(1023 - j);
    for (int b = 0; b < 256; b++) {
      const uint32_t v = gf_mul(byte_table((uint32_t)b), sh);
      for (int k = 0; k < kFoldCopies; k++) {
        if (kFoldPerm) fold[64 * b + 16 * j + k] = v;  // (rio_internal.h: byte-row layout)
        else fold[(j * 256 + b) * kFoldCopies + k] = v;
      }
    }
  }
  // mul[m][k][b] = (b << 8k) * c_m: multiply by c_0 = x^-32 (combine the 4
  // dword streams of a lane) and c_{l+1} = x^-(128*2^l) (lane tree, level l).
  for (int m = 0; m < kMulTables; m++) {
    const uint32_t c = (m == 0) ? gf_xpow8(-4) : gf_xpow8(-((int64_t)16 << (m - 1)));
    for (int k = 0; k < 4; k++)
      for (int b = 0; b < 256; b++) mul[(m * 4 + k) * 256 + b] = gf_mul((uint32_t)b << (8 * k), c);
  }
  // per payload size: crc = ~(fix_a[size] ^ V * fix_b[size]) where V is the
  // raw CRC of the whole 32 KiB chunk with bytes outside [12, 28+size) zeroed.
  for (int size = 0; size <= kMaxPayload; size++) {
    int64_t len = 16 + size;
    int64_t pad = kChunk - kChunkHdr - size;
    fix_a[size] = gf_mul(0xFFFFFFFFu, gf_xpow8(len));
    fix_b[size] = gf_xpow8(-pad);
  }
}

}  // namespace rio
