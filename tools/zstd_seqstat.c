/* Sequence statistics of zstd frames (development aid for k_zstd_exec, DESIGN.md
 * §5 C4): the oracle decoder with a hook on every executed sequence. Reads
 * frames from a file of [u32 length][frame] records; prints match-distance and
 * length histograms and how many distinct 128-B lines the far sources of each
 * 64-sequence group touch.
 *   gcc -O2 -o /tmp/zstd_seqstat tools/zstd_seqstat.c -Ioracle && /tmp/zstd_seqstat frames.bin */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct seq_stat {
  uint64_t nseq, match_bytes, lit_bytes, far_seq, far_bytes, rep_like;
  uint64_t dist_hist[8], ml_hist[8];
  uint64_t groups, group_far_lines, group_far_seqs;
  uint64_t gi, lines[64];
  int nl;
} seq_stat;
static seq_stat S;
static uint64_t last_off;

static void hook(int64_t olen, uint64_t ll, uint64_t ml, uint64_t off) {
  S.nseq++;
  S.lit_bytes += ll;
  S.match_bytes += ml;
  const uint64_t lim[8] = {64, 1024, 4096, 16384, 65536, 262144, 1048576, ~0ull};
  for (int i = 0; i < 8; i++)
    if (off <= lim[i]) { S.dist_hist[i]++; break; }
  const uint64_t mlim[8] = {4, 6, 8, 16, 32, 128, 2048, ~0ull};
  for (int i = 0; i < 8; i++)
    if (ml <= mlim[i]) { S.ml_hist[i]++; break; }
  if (off == last_off) S.rep_like++;
  last_off = off;
  const uint64_t src = (uint64_t)olen + ll - off;
  if (off > 16384) {
    S.far_seq++;
    S.far_bytes += ml;
    S.group_far_seqs++;
    for (uint64_t a = src >> 7; a <= (src + ml - 1) >> 7; a++) {
      int seen = 0;
      for (int k = 0; k < S.nl; k++) seen |= S.lines[k] == a;
      if (!seen && S.nl < 64) S.lines[S.nl++] = a;
    }
  }
  if (++S.gi == 64) {
    S.groups++;
    S.group_far_lines += S.nl;
    S.gi = 0;
    S.nl = 0;
  }
}
#define ORC_SEQ_HOOK(z, s) hook((z)->olen, (s)->ll, (s)->ml, (s)->off)
#include "../oracle/zstd_dec.c"

int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 1;
  uint8_t *out = malloc(1 << 24);
  uint32_t n;
  while (fread(&n, 4, 1, f) == 1) {
    uint8_t *in = malloc(n);
    if (fread(in, 1, n, f) != n) return 1;
    int64_t ol = 0;
    const char *msg = 0;
    orc_zstd_decompress(in, n, out, 1 << 24, &ol, &msg);
    free(in);
  }
  printf("seqs %llu lit_bytes %llu match_bytes %llu (%.2f B/seq) rep-offset-like %.3f\n", (unsigned long long)S.nseq,
         (unsigned long long)S.lit_bytes, (unsigned long long)S.match_bytes,
         (double)(S.lit_bytes + S.match_bytes) / S.nseq, (double)S.rep_like / S.nseq);
  const char *dn[8] = {"<=64", "<=1K", "<=4K", "<=16K", "<=64K", "<=256K", "<=1M", ">1M"};
  for (int i = 0; i < 8; i++) printf("dist %-7s %.3f\n", dn[i], (double)S.dist_hist[i] / S.nseq);
  const char *mn[8] = {"<=4", "<=6", "<=8", "<=16", "<=32", "<=128", "<=2048", ">2048"};
  for (int i = 0; i < 8; i++) printf("ml %-7s %.3f\n", mn[i], (double)S.ml_hist[i] / S.nseq);
  printf("far (>16K) seqs %.3f of all, far match bytes %llu; per 64-seq group: %.1f far seqs, %.1f distinct 128-B lines\n",
         (double)S.far_seq / S.nseq, (unsigned long long)S.far_bytes, (double)S.group_far_seqs / S.groups,
         (double)S.group_far_lines / S.groups);
  return 0;
}
