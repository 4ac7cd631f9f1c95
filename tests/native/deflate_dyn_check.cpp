// Host check of the dynamic-Huffman DEFLATE core shared with the GPU encoder
// (base_amd/csrc/deflate_dyn.h: trees from counts, complete length-limited
// codes, the run-length-coded header): a serial encoder of the GPU encoder's
// format (16 KiB sub-blocks, greedy 4-byte hash matches within 32 KiB, each
// sub-block dynamic or fixed, whichever is shorter) over random, 4-letter,
// run-heavy and copy-heavy buffers, every stream inflated by zlib (raw) and
// compared. Test infrastructure (tests/test_deflate_dyn_core.py runs it).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <zlib.h>
#include "zstd_enc.h"  // ZeBits
#include "deflate_dyn.h"
using namespace rio;

struct Tok { uint32_t lit, len, dist; };  // len 0: literal

static void fixed_bits(uint32_t sym, uint32_t &code, uint32_t &n) {
  if (sym < 144) { code = dz_rev(0x30 + sym, 8); n = 8; }
  else if (sym < 256) { code = dz_rev(0x190 + sym - 144, 9); n = 9; }
  else if (sym < 280) { code = dz_rev(sym - 256, 7); n = 7; }
  else { code = dz_rev(0xC0 + sym - 280, 8); n = 8; }
}

static std::vector<uint8_t> enc(const std::vector<uint8_t> &s) {
  std::vector<uint8_t> out(s.size() * 2 + 1024);
  ZeBits w{0, 0, out.data(), 0};
  std::vector<int64_t> hash(1 << 12, -1);
  const size_t L = s.size();
  size_t p = 0;
  for (size_t b0 = 0; b0 < L || (L == 0 && b0 == 0); b0 += 16384) {
    const size_t b1 = std::min(L, b0 + 16384);
    std::vector<Tok> toks;
    uint32_t llc[kDzLit] = {0}, dc[kDzDist] = {0};
    while (p < b1) {
      uint32_t m = 0; int64_t cand = -1;
      if (p + 4 <= L) {
        uint32_t v; memcpy(&v, &s[p], 4);
        uint32_t h = (v * 0x9E3779B1u) >> 20;
        cand = hash[h]; hash[h] = p;
        if (cand >= 0 && p - cand <= 32768) while (p + m < L && m < 258 && s[cand + m] == s[p + m]) m++;
      }
      if (m >= 4) {
        toks.push_back({0, m, (uint32_t)(p - cand)});
        uint32_t sym, e, v; dz_len_sym(m, sym, e, v); llc[sym]++;
        dz_dist_sym(p - cand, sym, e, v); dc[sym]++;
        p += m;
      } else { toks.push_back({s[p], 0, 0}); llc[s[p]]++; p++; }
    }
    llc[256]++;
    const bool final = p >= L;
    DzTrees t; uint32_t wk[2 * kDzLit]; uint16_t par[2 * kDzLit];
    uint32_t lc2[kDzLit], dc2[kDzDist];
    memcpy(lc2, llc, sizeof lc2); memcpy(dc2, dc, sizeof dc2);
    dz_fill(lc2, dc2);
    const uint32_t ln = dz_sort(lc2, kDzLit, t.ord);
    dz_build(lc2, dc2, ln, t, wk, par);
    uint64_t dyn = t.hdr_bits, fix = 3;
    for (auto &k : toks) {
      uint32_t c, n, sym, e, v;
      if (!k.len) { dyn += t.ll_len[k.lit]; fixed_bits(k.lit, c, n); fix += n; }
      else {
        dz_len_sym(k.len, sym, e, v); dyn += t.ll_len[sym] + e; fixed_bits(sym, c, n); fix += n + e;
        dz_dist_sym(k.dist, sym, e, v); dyn += t.d_len[sym] + e; fix += 5 + e;
      }
    }
    dyn += t.ll_len[256]; fix += 7;
    const bool use_dyn = dyn < fix;
    if (use_dyn) dz_header(w, t, final); else { w.add(final, 1); w.add(1, 2); }
    for (auto &k : toks) {
      uint32_t c, n, sym, e, v;
      if (!k.len) { if (use_dyn) w.add(t.ll_code[k.lit], t.ll_len[k.lit]); else { fixed_bits(k.lit, c, n); w.add(c, n); } }
      else {
        dz_len_sym(k.len, sym, e, v);
        if (use_dyn) w.add(t.ll_code[sym], t.ll_len[sym]); else { fixed_bits(sym, c, n); w.add(c, n); }
        w.add(v, e);
        dz_dist_sym(k.dist, sym, e, v);
        if (use_dyn) w.add(t.d_code[sym], t.d_len[sym]); else w.add(dz_rev(sym, 5), 5);
        w.add(v, e);
      }
    }
    if (use_dyn) w.add(t.ll_code[256], t.ll_len[256]); else w.add(0, 7);
    if (L == 0) break;
  }
  if (w.nb) out[w.pos++] = (uint8_t)w.acc;
  out.resize(w.pos);
  return out;
}

int main() {
  srand(3);
  int fails = 0; size_t tin = 0, tout = 0;
  std::string alpha = "ACGT";
  for (int t = 0; t < 40; t++) {
    size_t n = (t < 5) ? (size_t)(t * 7) : (size_t)(rand() % 200000);
    std::vector<uint8_t> s(n);
    int kind = t % 4;
    for (size_t i = 0; i < n; i++) {
      if (kind == 0) s[i] = rand() & 255;
      else if (kind == 1) s[i] = alpha[rand() & 3];
      else if (kind == 2) s[i] = (i % 97 < 50) ? 'x' : alpha[rand() & 3];
      else s[i] = (i > 1000 && rand() % 5) ? s[i - 1 - rand() % 1000] : 'a' + rand() % 20;
    }
    auto c = enc(s); tin += n; tout += c.size();
    std::vector<uint8_t> d(n + 16);
    z_stream zs{}; inflateInit2(&zs, -15);
    zs.next_in = c.data(); zs.avail_in = c.size(); zs.next_out = d.data(); zs.avail_out = d.size();
    int r = inflate(&zs, Z_FINISH); size_t got = zs.total_out; inflateEnd(&zs);
    bool ok = r == Z_STREAM_END && got == n && memcmp(d.data(), s.data(), n) == 0;
    if (!ok) { fails++; printf("FAIL t=%d n=%zu kind=%d r=%d got=%zu\n", t, n, kind, r, got); }
  }
  printf("fails=%d total_in=%zu total_out=%zu\n", fails, tin, tout);
  return fails != 0;
}
