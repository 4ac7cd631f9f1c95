// Host check of the zstd encoding core shared with the GPU encoder
// (base_amd/csrc/zstd_enc.h: predefined FSE compression tables, sequence codes,
// the backward sequence bitstream, frame / block headers): a serial encoder of
// the GPU encoder's format (<= 16 KiB blocks, raw literals, predefined-mode
// sequences, greedy 4-byte hash matches, raw blocks where a block does not
// shrink) over random, 4-letter, run-heavy and copy-heavy buffers, every frame
// decoded by libzstd (ZSTD_decompress: the library DataDog/zstd wraps) and
// compared. Test infrastructure (tests/test_zstd_enc_core.py builds and runs it).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <string>
#include <zstd.h>
#include "zstd_enc.h"
using namespace rio;

// serial reference of the GPU encoder's format: frame, <=16 KiB blocks, raw literals, predefined sequences
static std::vector<uint8_t> enc(const std::vector<uint8_t> &src, const ZeTabs &T) {
  std::vector<uint8_t> out(src.size() + 64 + 3 * (src.size() / kZeBlock + 2));
  ze_frame_header(out.data(), src.size());
  size_t o = kZeFrameHdr;
  std::vector<int64_t> hash(1 << 12, -1);
  const size_t L = src.size();
  for (size_t b0 = 0; b0 < L || (L == 0 && b0 == 0); b0 += kZeBlock) {
    const size_t b1 = std::min(L, b0 + kZeBlock);
    std::vector<ZeSeq> seqs;
    size_t lit_start = b0, p = b0;
    std::vector<uint8_t> lits;
    while (p < b1) {
      uint32_t m = 0; int64_t cand = -1;
      if (p + 4 <= b1) {
        uint32_t v; memcpy(&v, &src[p], 4);
        uint32_t h = (v * 0x9E3779B1u) >> 20;
        cand = hash[h]; hash[h] = p;
        if (cand >= 0) { while (p + m < b1 && src[cand + m] == src[p + m]) m++; }
      }
      if (m >= 4) {
        for (size_t q = lit_start; q < p; q++) lits.push_back(src[q]);
        seqs.push_back({(uint32_t)(p - lit_start), m, (uint32_t)(p - cand)});
        p += m; lit_start = p;
      } else p++;
    }
    for (size_t q = lit_start; q < b1; q++) lits.push_back(src[q]);
    const bool last = b1 >= L;
    size_t bh = o; o += 3;
    size_t c0 = o;
    const uint32_t nl = lits.size();
    bool huf = false;
    if (nl >= 64) {  // Huffman literals when they shrink (max symbol <= 128, >= 2 symbols)
      uint32_t cnt[256] = {0}, w[512]; uint16_t par[512]; uint8_t len[256]; uint16_t val[256];
      for (uint8_t c : lits) cnt[c]++;
      uint32_t last = 0, distinct = 0;
      for (int k = 0; k < 256; k++) if (cnt[k]) { last = k; distinct++; }
      if (distinct >= 2 && last <= 128) {
        ze_huf_lengths(cnt, last + 1, len, w, par);
        const uint32_t maxb = ze_huf_codes(len, last + 1, val);
        std::vector<uint8_t> sec(nl + 1024);
        uint32_t t = ze_huf_weights(len, last, maxb, sec.data());
        uint32_t jt = t; t += 6;
        const uint32_t seg = ze_seg(nl);
        uint32_t ssz[4];
        for (int k = 0; k < 4; k++) {
          const uint32_t a = k * seg < nl ? k * seg : nl, b = k < 3 ? ((k + 1) * seg < nl ? (k + 1) * seg : nl) : nl;
          ZeBits bw{0, 0, sec.data(), t};
          for (uint32_t i = b; i-- > a;) bw.add(val[lits[i]], len[lits[i]]);
          bw.close();
          ssz[k] = bw.pos - t; t = bw.pos;
        }
        for (int k = 0; k < 3; k++) { sec[jt + 2 * k] = ssz[k]; sec[jt + 2 * k + 1] = ssz[k] >> 8; }
        uint8_t hdr[5];
        const uint32_t hn = ze_lit_header(hdr, nl, t);
        if (hn + t < 3 + nl) {
          memcpy(&out[o], hdr, hn); o += hn; memcpy(&out[o], sec.data(), t); o += t;
          huf = true;
        }
      }
    }
    if (!huf) {
      out[o++] = (uint8_t)(0 | (3 << 2) | ((nl & 15) << 4));
      out[o++] = (uint8_t)(nl >> 4); out[o++] = (uint8_t)(nl >> 12);
      memcpy(&out[o], lits.data(), nl); o += nl;
    }
    const uint32_t n = seqs.size();
    if (n < 128) out[o++] = n;
    else if (n < 0x7F00) { out[o++] = (n >> 8) + 0x80; out[o++] = n & 0xff; }
    else { out[o++] = 0xff; out[o++] = (n - 0x7F00) & 0xff; out[o++] = (n - 0x7F00) >> 8; }
    if (n) {
      out[o++] = 0;  // predefined modes
      ZeBits w{0, 0, out.data(), o};
      ze_sequences(w, T, n, [&](uint32_t i) { return seqs[i]; });
      o = w.pos;
    }
    size_t csz = o - c0;
    uint32_t bsz = b1 - b0;
    if (csz >= bsz) {  // raw block
      o = c0; memcpy(&out[o], &src[b0], bsz); o += bsz;
      uint32_t h = (last ? 1 : 0) | (0 << 1) | (bsz << 3);
      out[bh] = h; out[bh+1] = h >> 8; out[bh+2] = h >> 16;
    } else {
      uint32_t h = (last ? 1 : 0) | (2 << 1) | ((uint32_t)csz << 3);
      out[bh] = h; out[bh+1] = h >> 8; out[bh+2] = h >> 16;
    }
    if (L == 0) break;
  }
  out.resize(o);
  return out;
}

int main() {
  ZeTabs T; ze_build_tabs(T);
  srand(1);
  int fails = 0; size_t tin = 0, tout = 0;
  for (int t = 0; t < 40; t++) {
    size_t n = (t < 5) ? (size_t)(t * 7) : (size_t)(rand() % 300000);
    std::vector<uint8_t> s(n);
    int kind = t % 4;
    std::string alpha = "ACGT";
    for (size_t i = 0; i < n; i++) {
      if (kind == 0) s[i] = rand() & 255;
      else if (kind == 1) s[i] = alpha[rand() & 3];
      else if (kind == 2) s[i] = (i % 97 < 50) ? 'x' : alpha[rand() & 3];
      else s[i] = (i > 1000 && rand() % 5) ? s[i - 1 - rand() % 1000] : rand() & 255;
    }
    auto c = enc(s, T); tin += n; tout += c.size();
    std::vector<uint8_t> d(n + 1);
    size_t r = ZSTD_decompress(d.data(), n + 1, c.data(), c.size());
    bool ok = !ZSTD_isError(r) && r == n && memcmp(d.data(), s.data(), n) == 0;
    if (!ok) { fails++; printf("FAIL t=%d n=%zu kind=%d err=%s\n", t, n, kind, ZSTD_isError(r) ? ZSTD_getErrorName(r) : "mismatch"); }
    
  }
  printf("fails=%d total_in=%zu total_out=%zu\n", fails, tin, tout);
  return fails != 0;
}
