// Host check of the zstd encoding core shared with the GPU encoder
// (base_amd/csrc/zstd_enc.h: FSE compression tables -- predefined and fitted to
// a block, with their descriptions --, sequence codes, the backward sequence
// bitstream, Huffman literals, frame / block headers): a serial encoder of the
// GPU encoder's format (<= 16 KiB blocks; matches from rounds of 64 positions
// against a 4,096-bucket hash of two 16-bit positions, as k_zstd_enc finds
// them; per table the cheaper of predefined and fitted; raw blocks where a
// block does not shrink) over random, 4-letter, run-heavy and copy-heavy
// buffers, every frame decoded by libzstd (ZSTD_decompress: the library
// DataDog/zstd wraps) and compared. Test infrastructure
// (tests/test_zstd_enc_core.py builds and runs it).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <string>
#include <zstd.h>
#include "zstd_enc.h"
using namespace rio;

// the GPU encoder's matches of [b0, b1): per round of 64 positions every
// position looks up its bucket (4-byte prefix hash) before any of the round
// inserts; two 16-bit positions per bucket, the longer match wins (ties: the
// newer); a greedy walk from the parse cursor takes matches >= 4
static void match_block(const std::vector<uint8_t> &src, size_t b0, size_t b1, std::vector<uint32_t> &hash,
                        std::vector<ZeSeq> &seqs, std::vector<uint8_t> &lits) {
  size_t cur = b0, lit_start = b0;
  for (size_t base = b0; base < b1; base += 64) {
    uint32_t hv[64], e[64], mm[64] = {0};
    size_t cd[64] = {0};
    for (int l = 0; l < 64; l++) {
      const size_t p = base + l;
      if (p + 4 > b1) continue;
      uint32_t v;
      memcpy(&v, &src[p], 4);
      hv[l] = (v * 0x9E3779B1u) >> 20;
      e[l] = hash[hv[l]];
      if (p < cur) continue;
      for (int way = 0; way < 2; way++) {
        const uint32_t d = (uint32_t)(p - (e[l] >> (16 * way))) & 0xffffu;
        if (d == 0 || d > p) continue;
        uint32_t m = 0;
        while (p + m < b1 && src[p - d + m] == src[p + m]) m++;
        if (m > mm[l]) { mm[l] = m; cd[l] = p - d; }
      }
    }
    for (int l = 0; l < 64; l++)
      if (base + l + 4 <= b1) hash[hv[l]] = (e[l] << 16) | (uint32_t)((base + l) & 0xffff);
    const size_t rend = std::min(base + 64, b1);
    size_t pos = cur;
    while (pos < rend) {
      const int l = (int)(pos - base);
      if (mm[l] >= 4) {
        for (size_t q = lit_start; q < pos; q++) lits.push_back(src[q]);
        seqs.push_back({(uint32_t)(pos - lit_start), mm[l], (uint32_t)(pos - cd[l])});
        pos += mm[l];
        lit_start = pos;
      } else {
        pos++;
      }
    }
    cur = pos;
  }
  lit_start = std::min(lit_start, b1);
  for (size_t q = lit_start; q < b1; q++) lits.push_back(src[q]);
}

static size_t g_fitted, g_tables;

// serial reference of the GPU encoder's format
static std::vector<uint8_t> enc(const std::vector<uint8_t> &src, const ZeTabs &T) {
  std::vector<uint8_t> out(src.size() + 64 + 3 * (src.size() / kZeBlock + 2) + 512);
  ze_frame_header(out.data(), src.size());
  size_t o = kZeFrameHdr;
  std::vector<uint32_t> hash(1 << 12, 0);
  const size_t L = src.size();
  for (size_t b0 = 0; b0 < L || (L == 0 && b0 == 0); b0 += kZeBlock) {
    const size_t b1 = std::min(L, b0 + kZeBlock);
    std::vector<ZeSeq> seqs;
    std::vector<uint8_t> lits;
    match_block(src, b0, b1, hash, seqs, lits);
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
    if (n) {  // per table (LL, OF, ML) the cheaper of predefined and fitted
      uint32_t cnt[3][56] = {{0}};
      for (auto &q : seqs) {
        cnt[0][ze_ll_code(q.ll)]++;
        cnt[1][ze_highbit(q.off + 3)]++;
        cnt[2][ze_ml_code(q.ml - 3)]++;
      }
      ZeTabs B = T;
      ZeFseWork wk;
      const size_t mq = o++;
      uint8_t modes = 0;
      uint8_t desc[kZeDescMax];
      uint32_t dl;
      dl = ze_fit_table(cnt[0], 36, kZeLLNorm, kZeLLSyms, kZeLLLog, B.ll, wk, desc);
      memcpy(&out[o], desc, dl); o += dl; modes |= (dl ? 2 : 0) << 6; g_fitted += dl != 0;
      dl = ze_fit_table(cnt[1], 32, kZeOFNorm, kZeOFSyms, kZeOFLog, B.of, wk, desc);
      memcpy(&out[o], desc, dl); o += dl; modes |= (dl ? 2 : 0) << 4; g_fitted += dl != 0;
      dl = ze_fit_table(cnt[2], 53, kZeMLNorm, kZeMLSyms, kZeMLLog, B.ml, wk, desc);
      memcpy(&out[o], desc, dl); o += dl; modes |= (dl ? 2 : 0) << 2; g_fitted += dl != 0;
      g_tables += 3;
      out[mq] = modes;
      ZeBits w{0, 0, out.data(), o};
      ze_sequences(w, B, n, [&](uint32_t i) { return seqs[i]; });
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
  for (int t = 0; t < 50; t++) {
    size_t n = (t < 5) ? (size_t)(t * 7) : (size_t)(rand() % 300000);
    std::vector<uint8_t> s(n);
    int kind = t % 5;
    std::string alpha = "ACGT";
    int qv = 30;
    for (size_t i = 0; i < n; i++) {
      if (kind == 0) s[i] = rand() & 255;
      else if (kind == 1) s[i] = alpha[rand() & 3];
      else if (kind == 2) s[i] = (i % 97 < 50) ? 'x' : alpha[rand() & 3];
      else if (kind == 3) s[i] = (i > 1000 && rand() % 5) ? s[i - 1 - rand() % 1000] : rand() & 255;
      else {  // FASTQ-like: 150 bases, then 150 qualities of a bounded walk
        const size_t k = i % 306;
        if (k < 150) s[i] = alpha[rand() & 3];
        else if (k < 153) s[i] = "\n+\n"[k - 150];
        else if (k < 303) { qv += rand() % 7 - 3; qv = qv < 2 ? 2 : qv > 41 ? 41 : qv; s[i] = 33 + qv; }
        else s[i] = "\n@r"[k - 303];
      }
    }
    auto c = enc(s, T); tin += n; tout += c.size();
    std::vector<uint8_t> d(n + 1);
    size_t r = ZSTD_decompress(d.data(), n + 1, c.data(), c.size());
    bool ok = !ZSTD_isError(r) && r == n && memcmp(d.data(), s.data(), n) == 0;
    if (!ok) { fails++; printf("FAIL t=%d n=%zu kind=%d err=%s\n", t, n, kind, ZSTD_isError(r) ? ZSTD_getErrorName(r) : "mismatch"); }
    
  }
  printf("fails=%d total_in=%zu total_out=%zu fitted_tables=%zu/%zu\n", fails, tin, tout, g_fitted, g_tables);
  return fails != 0;
}
