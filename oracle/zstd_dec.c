/*
 * ORACLE — test infrastructure only. Never linked into the product path.
 *
 * CPU restatement of Zstandard frame decoding as used by the reference's
 * "zstd" transformer: recordiozstd.zstdUncompress
 * (recordio/recordiozstd/recordiozstd.go:67-78) -> compress/zstd.Decompress
 * (compress/zstd/zstd_cgo.go:34-41) -> github.com/DataDog/zstd v1.4.1
 * (go.mod:7; not vendored under /root/reference), i.e. libzstd's one-shot
 * ZSTD_decompress over every frame of the block.
 *
 * Valid input decodes per the format (RFC 8878). Invalid input is decoded the
 * way libzstd's implementation handles it, not the RFC's strictest reading, so
 * that accept / reject, the bytes of an accepted frame and the error name
 * match the library the reference links. Restated from libzstd 1.4.x (the
 * 1.4.9 build in this image is the checker: tests/test_zstd_libzstd.py fuzzes
 * the restatement against it):
 *  - multi-frame loop: trailing bytes < 5 or garbage after a frame read as
 *    "Src size is incorrect"; a frame needs >= 9 bytes; skippable frames;
 *  - no block-size / window limits in one-shot decoding (a compressed block of
 *    >= 128 KiB is "Src size is incorrect");
 *  - the bit reader as a 64-bit container (bitstream.h): reads past the start
 *    return zero bits, and past an overflow wrap around the container;
 *  - Huffman: table logs up to 12, libzstd's weight checks, single-stream
 *    literals with the single-symbol decoder, four-stream literals with the
 *    single- or double-symbol decoder chosen by libzstd's timing model (the
 *    double-symbol decoder's last-symbol clamp and lockstep checks included);
 *  - FSE table descriptions read with libzstd's FSE_readNCount;
 *  - sequences: the reserved bits of the modes byte ignored, a block without
 *    sequences must end right after its count, every state updated after every
 *    sequence (the last included), the stream accepted once it is exhausted or
 *    over-read, a repeat offset of 0 forced to 1; the long-offset decoder's
 *    end rule for windows > 16 MiB.
 * Error names are libzstd's (ZSTD_getErrorName).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define ZMAGIC 0xFD2FB528u
#define BLOCK_MAX (128 * 1024)

static const char *E_PREFIX = "Unknown frame descriptor";
static const char *E_CORRUPT = "Corrupted block detected";
static const char *E_SRC = "Src size is incorrect";
static const char *E_CHECKSUM = "Restored data doesn't match checksum";
static const char *E_DICT = "Dictionary mismatch";
static const char *E_WINDOW = "Frame requires too much memory for decoding";
static const char *E_TABLELOG = "tableLog requires too much memory : unsupported";
static const char *E_NOTSUP = "Unsupported frame parameter";

static uint32_t rd16(const uint8_t *p) { return p[0] | ((uint32_t)p[1] << 8); }
static uint32_t rd24(const uint8_t *p) { return p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16); }
static uint32_t rd32(const uint8_t *p) { return rd16(p) | (rd16(p + 2) << 16); }
static uint64_t rd64(const uint8_t *p) { return rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

static int highbit32(uint32_t v) { return 31 - __builtin_clz(v); }

/* ---------------------------------------------------------------- XXH64 */
#define P64_1 0x9E3779B185EBCA87ull
#define P64_2 0xC2B2AE3D27D4EB4Full
#define P64_3 0x165667B19E3779F9ull
#define P64_4 0x85EBCA77C2B2AE63ull
#define P64_5 0x27D4EB2F165667C5ull
static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t xxh_round(uint64_t acc, uint64_t in) {
    acc += in * P64_2;
    acc = rotl64(acc, 31);
    return acc * P64_1;
}
static uint64_t xxh_merge(uint64_t acc, uint64_t v) {
    acc ^= xxh_round(0, v);
    return acc * P64_1 + P64_4;
}
static uint64_t xxh64(const uint8_t *p, size_t len, uint64_t seed) {
    const uint8_t *end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed, v4 = seed - P64_1;
        const uint8_t *limit = end - 32;
        do {
            v1 = xxh_round(v1, rd64(p));
            v2 = xxh_round(v2, rd64(p + 8));
            v3 = xxh_round(v3, rd64(p + 16));
            v4 = xxh_round(v4, rd64(p + 24));
            p += 32;
        } while (p <= limit);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xxh_merge(h, v1);
        h = xxh_merge(h, v2);
        h = xxh_merge(h, v3);
        h = xxh_merge(h, v4);
    } else {
        h = seed + P64_5;
    }
    h += (uint64_t)len;
    while (p + 8 <= end) {
        h ^= xxh_round(0, rd64(p));
        h = rotl64(h, 27) * P64_1 + P64_4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)rd32(p) * P64_1;
        h = rotl64(h, 23) * P64_2 + P64_3;
        p += 4;
    }
    while (p < end) {
        h ^= (*p) * P64_5;
        h = rotl64(h, 11) * P64_1;
        p++;
    }
    h ^= h >> 33;
    h *= P64_2;
    h ^= h >> 29;
    h *= P64_3;
    h ^= h >> 32;
    return h;
}

/* ---------------------------------------------------------------- error names */
static const char *E_DICTC = "Dictionary is corrupted";

/* ---------------------------------------------------------------- bit reader
 * BIT_DStream_t: a 64-bit container read backwards; `bc` bits of it consumed. */
typedef struct {
    uint64_t c;
    unsigned bc;
    const uint8_t *ptr, *start, *limit;
} bitd_t;
enum { BIT_UNFINISHED = 0, BIT_END_OF_BUFFER = 1, BIT_COMPLETED = 2, BIT_OVERFLOW = 3 };

/* 0 ok, -1 error (empty stream, no end mark) */
static int bitd_init(bitd_t *b, const uint8_t *src, size_t n) {
    memset(b, 0, sizeof(*b));
    if (n < 1) return -1;
    b->start = src;
    b->limit = src + 8;
    const uint8_t last = src[n - 1];
    if (n >= 8) {
        b->ptr = src + n - 8;
        b->c = rd64(b->ptr);
        b->bc = last ? 8 - (unsigned)highbit32(last) : 0;
        if (!last) return -1;
    } else {
        b->ptr = src;
        b->c = 0;
        for (size_t k = 0; k < n; k++) b->c |= (uint64_t)src[k] << (8 * k);
        if (!last) return -1;
        b->bc = 8 - (unsigned)highbit32(last) + (unsigned)(8 - n) * 8;
    }
    return 0;
}
static uint64_t bitd_look(const bitd_t *b, unsigned nb) { /* BIT_lookBits = BIT_getMiddleBits (nb may be 0) */
    const uint32_t start = 64u - b->bc - nb; /* U32 arithmetic: wraps once the reader over-reads */
    return (b->c >> (start & 63)) & ((1ull << nb) - 1);
}
static uint64_t bitd_look_fast(const bitd_t *b, unsigned nb) { /* BIT_lookBitsFast (nb >= 1) */
    return (b->c << (b->bc & 63)) >> ((64 - nb) & 63);
}
static uint64_t bitd_read(bitd_t *b, unsigned nb) {
    uint64_t v = bitd_look(b, nb);
    b->bc += nb;
    return v;
}
static uint64_t bitd_read_fast(bitd_t *b, unsigned nb) {
    uint64_t v = bitd_look_fast(b, nb);
    b->bc += nb;
    return v;
}
static int bitd_reload(bitd_t *b) {
    if (b->bc > 64) return BIT_OVERFLOW;
    if (b->ptr >= b->limit) {
        b->ptr -= b->bc >> 3;
        b->bc &= 7;
        b->c = rd64(b->ptr);
        return BIT_UNFINISHED;
    }
    if (b->ptr == b->start) return b->bc < 64 ? BIT_END_OF_BUFFER : BIT_COMPLETED;
    unsigned nbytes = b->bc >> 3;
    int r = BIT_UNFINISHED;
    if (b->ptr - nbytes < b->start) {
        nbytes = (unsigned)(b->ptr - b->start);
        r = BIT_END_OF_BUFFER;
    }
    b->ptr -= nbytes;
    b->bc -= nbytes * 8;
    b->c = rd64(b->ptr);
    return r;
}
static int bitd_reload_fast(bitd_t *b) { /* BIT_reloadDStreamFast */
    if (b->ptr < b->limit) return BIT_OVERFLOW;
    b->ptr -= b->bc >> 3;
    b->bc &= 7;
    b->c = rd64(b->ptr);
    return BIT_UNFINISHED;
}
static int bitd_end(const bitd_t *b) { return b->ptr == b->start && b->bc == 64; }

/* ---------------------------------------------------------------- FSE_readNCount */
/* returns bytes consumed, -1 on error; *max_sv in: capacity, out: last symbol */
static int64_t fse_read_ncount(int16_t *norm, unsigned *max_sv, unsigned *tlog, const uint8_t *src, size_t n) {
    if (n < 4) { /* works on a zero-padded copy */
        uint8_t buf[4] = {0, 0, 0, 0};
        memcpy(buf, src, n);
        int64_t k = fse_read_ncount(norm, max_sv, tlog, buf, 4);
        if (k < 0 || (size_t)k > n) return -1;
        return k;
    }
    const int64_t iend = (int64_t)n;
    int64_t ip = 0;
    memset(norm, 0, (*max_sv + 1) * sizeof(int16_t));
    uint32_t bs = rd32(src);
    int nbits = (int)(bs & 0xF) + 5;
    if (nbits > 15) return -1;
    bs >>= 4;
    int bit_count = 4;
    *tlog = (unsigned)nbits;
    int remaining = (1 << nbits) + 1;
    int threshold = 1 << nbits;
    nbits++;
    unsigned charnum = 0;
    int previous0 = 0;
    while ((remaining > 1) & (charnum <= *max_sv)) {
        if (previous0) {
            unsigned n0 = charnum;
            while ((bs & 0xFFFF) == 0xFFFF) {
                n0 += 24;
                if (ip < iend - 5) {
                    ip += 2;
                    bs = rd32(src + ip) >> bit_count;
                } else {
                    bs >>= 16;
                    bit_count += 16;
                }
            }
            while ((bs & 3) == 3) {
                n0 += 3;
                bs >>= 2;
                bit_count += 2;
            }
            n0 += bs & 3;
            bit_count += 2;
            if (n0 > *max_sv) return -1;
            while (charnum < n0) norm[charnum++] = 0;
            if ((ip <= iend - 7) || (ip + (bit_count >> 3) <= iend - 4)) {
                ip += bit_count >> 3;
                bit_count &= 7;
                bs = rd32(src + ip) >> bit_count;
            } else {
                bs >>= 2;
            }
        }
        {
            const int max = (2 * threshold - 1) - remaining;
            int count;
            if ((int)(bs & (uint32_t)(threshold - 1)) < max) {
                count = (int)(bs & (uint32_t)(threshold - 1));
                bit_count += nbits - 1;
            } else {
                count = (int)(bs & (uint32_t)(2 * threshold - 1));
                if (count >= threshold) count -= max;
                bit_count += nbits;
            }
            count--;
            remaining -= count < 0 ? -count : count;
            norm[charnum++] = (int16_t)count;
            previous0 = !count;
            while (remaining < threshold) {
                nbits--;
                threshold >>= 1;
            }
            if ((ip <= iend - 7) || (ip + (bit_count >> 3) <= iend - 4)) {
                ip += bit_count >> 3;
                bit_count &= 7;
            } else {
                bit_count -= (int)(8 * (iend - 4 - ip));
                ip = iend - 4;
            }
            bs = rd32(src + ip) >> (bit_count & 31);
        }
    }
    if (remaining != 1) return -1;
    if (bit_count > 32) return -1;
    *max_sv = charnum - 1;
    ip += (bit_count + 7) >> 3;
    return ip;
}

/* symbol spread (FSE_buildDTable / ZSTD_buildFSETable): cell -> symbol, the
 * next-state counters; 0 if the spread does not close (FSE_buildDTable's GENERIC) */
static int fse_spread(uint8_t *sym, uint16_t *next_state, uint8_t *nbits_out, const int16_t *norm, unsigned max_sv,
                      unsigned tlog) {
    const uint32_t size = 1u << tlog;
    uint32_t high = size - 1;
    uint16_t next[256];
    for (unsigned s = 0; s <= max_sv; s++) {
        if (norm[s] == -1) {
            sym[high--] = (uint8_t)s;
            next[s] = 1;
        } else {
            next[s] = (uint16_t)norm[s];
        }
    }
    const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    uint32_t pos = 0;
    for (unsigned s = 0; s <= max_sv; s++)
        for (int i = 0; i < norm[s]; i++) {
            sym[pos] = (uint8_t)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    const int closed = pos == 0;
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t ns = next[sym[u]]++;
        nbits_out[u] = (uint8_t)(tlog - (unsigned)highbit32(ns));
        next_state[u] = (uint16_t)((ns << nbits_out[u]) - size);
    }
    return closed;
}

/* ---------------------------------------------------------------- Huffman */
#define HUF_MAXLOG 12 /* HUF_TABLELOG_MAX: the DCtx's Huffman table (HufLog) */

typedef struct {
    int type;          /* 0: single-symbol (X1), 1: double-symbol (X2) */
    unsigned log;      /* X1: the code's table log; X2: HUF_MAXLOG */
    uint8_t s1[1 << HUF_MAXLOG], nb1[1 << HUF_MAXLOG];          /* X1 */
    uint8_t seq0[1 << HUF_MAXLOG], seq1[1 << HUF_MAXLOG];       /* X2 */
    uint8_t nb2[1 << HUF_MAXLOG], len2[1 << HUF_MAXLOG];
} huf_t;

/* HUF_readStats: weights of the symbols (the last implied), rank counts,
 * table log; bytes consumed or -1 */
static int64_t huf_read_stats(uint8_t *w, uint32_t *rank, unsigned *nsym, unsigned *tlog, const uint8_t *src,
                              size_t n) {
    if (!n) return -1;
    size_t isize = src[0], osize;
    if (isize >= 128) {
        osize = isize - 127;
        isize = (osize + 1) / 2;
        if (isize + 1 > n) return -1;
        if (osize >= 256) return -1;
        for (size_t k = 0; k < osize; k += 2) {
            w[k] = src[1 + k / 2] >> 4;
            w[k + 1] = src[1 + k / 2] & 15;
        }
    } else {
        /* FSE_decompress_wksp(w, 255, src+1, isize, maxLog 6) */
        if (isize + 1 > n) return -1;
        const uint8_t *c = src + 1;
        size_t cn = isize;
        int16_t norm[256];
        unsigned max_sv = 255, log;
        int64_t k = fse_read_ncount(norm, &max_sv, &log, c, cn);
        if (k < 0) return -1;
        if (log > 6) return -1;
        c += k;
        cn -= (size_t)k;
        uint8_t sym[64], nb[64];
        uint16_t ns[64];
        if (max_sv > 255 || log > 12) return -1;
        if (!fse_spread(sym, ns, nb, norm, max_sv, log)) return -1;
        bitd_t b;
        if (bitd_init(&b, c, cn) != 0) return -1;
        uint32_t st1 = (uint32_t)bitd_read(&b, log);
        bitd_reload(&b);
        uint32_t st2 = (uint32_t)bitd_read(&b, log);
        bitd_reload(&b);
        size_t op = 0;
        const size_t omax = 255, olimit = omax - 3;
#define FSE_SYM(st) (tmp_ = sym[st], st = ns[st] + (uint32_t)bitd_read(&b, nb[st]), tmp_)
        uint8_t tmp_;
        for (; (bitd_reload(&b) == BIT_UNFINISHED) & (op < olimit); op += 4) {
            w[op] = FSE_SYM(st1);
            w[op + 1] = FSE_SYM(st2);
            w[op + 2] = FSE_SYM(st1);
            w[op + 3] = FSE_SYM(st2);
        }
        for (;;) {
            if (op > omax - 2) return -1;
            w[op++] = FSE_SYM(st1);
            if (bitd_reload(&b) == BIT_OVERFLOW) {
                w[op++] = FSE_SYM(st2);
                break;
            }
            if (op > omax - 2) return -1;
            w[op++] = FSE_SYM(st2);
            if (bitd_reload(&b) == BIT_OVERFLOW) {
                w[op++] = FSE_SYM(st1);
                break;
            }
        }
#undef FSE_SYM
        osize = op;
    }
    memset(rank, 0, (HUF_MAXLOG + 1) * sizeof(uint32_t));
    uint32_t total = 0;
    for (size_t k = 0; k < osize; k++) {
        if (w[k] >= HUF_MAXLOG) return -1;
        rank[w[k]]++;
        total += (1u << w[k]) >> 1;
    }
    if (total == 0) return -1;
    const unsigned log = (unsigned)highbit32(total) + 1;
    if (log > HUF_MAXLOG) return -1;
    *tlog = log;
    const uint32_t rest = (1u << log) - total;
    const uint32_t verif = 1u << highbit32(rest);
    const unsigned lastw = (unsigned)highbit32(rest) + 1;
    if (verif != rest) return -1;
    w[osize] = (uint8_t)lastw;
    rank[lastw]++;
    if (rank[1] < 2 || (rank[1] & 1)) return -1;
    *nsym = (unsigned)osize + 1;
    return (int64_t)isize + 1;
}

/* HUF_readDTableX1_wksp */
static int64_t huf_read_x1(huf_t *h, const uint8_t *src, size_t n) {
    uint8_t w[257];
    uint32_t rank[HUF_MAXLOG + 1];
    unsigned nsym, log;
    int64_t isize = huf_read_stats(w, rank, &nsym, &log, src, n);
    if (isize < 0) return -1;
    h->type = 0;
    h->log = log;
    uint32_t next = 0;
    for (unsigned k = 1; k < log + 1; k++) {
        const uint32_t cur = next;
        next += rank[k] << (k - 1);
        rank[k] = cur;
    }
    for (unsigned s = 0; s < nsym; s++) {
        const unsigned wt = w[s];
        const uint32_t len = (1u << wt) >> 1, st = rank[wt];
        for (uint32_t u = st; u < st + len; u++) {
            h->s1[u] = (uint8_t)s;
            h->nb1[u] = (uint8_t)(log + 1 - wt);
        }
        rank[wt] = st + len;
    }
    return isize;
}

/* HUF_readDTableX2_wksp + HUF_fillDTableX2(Level2): a 12-bit table whose cells
 * hold one symbol or two (when the second's code fits the remaining bits) */
typedef struct {
    uint8_t symbol, weight;
} sorted_t;

static void x2_fill_level2(huf_t *h, uint32_t base, unsigned size_log, unsigned consumed, const uint32_t *rank_origin,
                           int min_weight, const sorted_t *sorted, uint32_t nsorted, unsigned nb_baseline,
                           uint8_t base_seq) {
    uint32_t rv[HUF_MAXLOG + 1];
    memcpy(rv, rank_origin, sizeof(rv));
    if (min_weight > 1) {
        const uint32_t skip = rv[min_weight];
        for (uint32_t i = 0; i < skip; i++) {
            h->seq0[base + i] = base_seq;
            h->seq1[base + i] = 0;
            h->nb2[base + i] = (uint8_t)consumed;
            h->len2[base + i] = 1;
        }
    }
    for (uint32_t s = 0; s < nsorted; s++) {
        const unsigned nb = nb_baseline - sorted[s].weight;
        const uint32_t len = 1u << (size_log - nb), st = rv[sorted[s].weight];
        for (uint32_t i = st; i < st + len; i++) {
            h->seq0[base + i] = base_seq;
            h->seq1[base + i] = sorted[s].symbol;
            h->nb2[base + i] = (uint8_t)(nb + consumed);
            h->len2[base + i] = 2;
        }
        rv[sorted[s].weight] += len;
    }
}

static int64_t huf_read_x2(huf_t *h, const uint8_t *src, size_t n) {
    uint8_t w[257];
    uint32_t rank_stats[HUF_MAXLOG + 1];
    unsigned nsym, log;
    int64_t isize = huf_read_stats(w, rank_stats, &nsym, &log, src, n);
    if (isize < 0) return -1;
    const unsigned max_log = HUF_MAXLOG;
    unsigned max_w = log;
    while (rank_stats[max_w] == 0) max_w--;
    uint32_t rank_start0[HUF_MAXLOG + 2] = {0};
    uint32_t *rank_start = rank_start0 + 1;
    uint32_t next = 0;
    for (unsigned k = 1; k < max_w + 1; k++) {
        const uint32_t cur = next;
        next += rank_stats[k];
        rank_start[k] = cur;
    }
    rank_start[0] = next;
    const uint32_t nsort = next;
    sorted_t sorted[256];
    for (unsigned s = 0; s < nsym; s++) {
        const uint32_t r = rank_start[w[s]]++;
        sorted[r].symbol = (uint8_t)s;
        sorted[r].weight = w[s];
    }
    rank_start[0] = 0;
    uint32_t rank_val[HUF_MAXLOG][HUF_MAXLOG + 1];
    memset(rank_val, 0, sizeof(rank_val));
    {
        const int rescale = (int)(max_log - log) - 1;
        uint32_t nrv = 0;
        for (unsigned k = 1; k < max_w + 1; k++) {
            const uint32_t cur = nrv;
            nrv += rank_stats[k] << (k + rescale);
            rank_val[0][k] = cur;
        }
        const unsigned min_bits = log + 1 - max_w;
        for (unsigned consumed = min_bits; consumed < max_log - min_bits + 1; consumed++)
            for (unsigned k = 1; k < max_w + 1; k++) rank_val[consumed][k] = rank_val[0][k] >> consumed;
    }
    /* HUF_fillDTableX2(dt, max_log, sorted, nsort, rank_start0, rank_val, max_w, log + 1) */
    const unsigned nb_baseline = log + 1;
    const int scale_log = (int)nb_baseline - (int)max_log;
    const unsigned min_bits = nb_baseline - max_w;
    uint32_t rv[HUF_MAXLOG + 1];
    memcpy(rv, rank_val[0], sizeof(rv));
    for (uint32_t s = 0; s < nsort; s++) {
        const uint8_t symbol = sorted[s].symbol;
        const unsigned weight = sorted[s].weight;
        const unsigned nb = nb_baseline - weight;
        const uint32_t start = rv[weight];
        const uint32_t len = 1u << (max_log - nb);
        if (max_log - nb >= min_bits) {
            int min_weight = (int)nb + scale_log;
            if (min_weight < 1) min_weight = 1;
            const uint32_t sorted_rank = rank_start0[min_weight];
            x2_fill_level2(h, start, max_log - nb, nb, rank_val[nb], min_weight, sorted + sorted_rank,
                           nsort - sorted_rank, nb_baseline, symbol);
        } else {
            for (uint32_t u = start; u < start + len; u++) {
                h->seq0[u] = symbol;
                h->seq1[u] = 0;
                h->nb2[u] = (uint8_t)nb;
                h->len2[u] = 1;
            }
        }
        rv[weight] += len;
    }
    h->type = 1;
    h->log = max_log;
    return isize;
}

/* HUF_selectDecoder: libzstd's decoder timing model (Q = compression ratio in 16ths) */
static const uint32_t kAlgoTime[16][2][2] = {
    {{0, 0}, {1, 1}},           {{0, 0}, {1, 1}},           {{38, 130}, {1313, 74}},    {{448, 128}, {1353, 74}},
    {{556, 128}, {1353, 74}},   {{714, 128}, {1418, 74}},   {{883, 128}, {1437, 74}},   {{897, 128}, {1515, 75}},
    {{926, 128}, {1613, 75}},   {{947, 128}, {1729, 77}},   {{1107, 128}, {2083, 81}},  {{1177, 128}, {2379, 87}},
    {{1242, 128}, {2415, 93}},  {{1349, 128}, {2644, 106}}, {{1455, 128}, {2422, 124}}, {{722, 128}, {1891, 145}},
};
static int huf_select_x2(size_t dst, size_t csrc) {
    const uint32_t q = csrc >= dst ? 15 : (uint32_t)(csrc * 16 / dst);
    const uint32_t d256 = (uint32_t)(dst >> 8);
    const uint32_t t0 = kAlgoTime[q][0][0] + kAlgoTime[q][0][1] * d256;
    uint32_t t1 = kAlgoTime[q][1][0] + kAlgoTime[q][1][1] * d256;
    t1 += t1 >> 3;
    return t1 < t0;
}

/* output of a Huffman decode: lit[0 .. n), written with libzstd's slack */
#define LIT_SLACK 64

static inline void x1_sym(const huf_t *h, bitd_t *b, uint8_t *lit, int64_t *p) {
    const uint64_t v = bitd_look_fast(b, h->log);
    lit[*p] = h->s1[v];
    b->bc += h->nb1[v];
    (*p)++;
}
static inline void x2_sym(const huf_t *h, bitd_t *b, uint8_t *lit, int64_t *p) {
    const uint64_t v = bitd_look_fast(b, h->log);
    lit[*p] = h->seq0[v];
    lit[*p + 1] = h->seq1[v];
    b->bc += h->nb2[v];
    *p += h->len2[v];
}

/* HUF_decodeStreamX1 over [p, end) */
static void x1_stream(const huf_t *h, bitd_t *b, uint8_t *lit, int64_t p, int64_t end) {
    while ((bitd_reload(b) == BIT_UNFINISHED) & (p < end - 3)) {
        x1_sym(h, b, lit, &p);
        x1_sym(h, b, lit, &p);
        x1_sym(h, b, lit, &p);
        x1_sym(h, b, lit, &p);
    }
    while (p < end) x1_sym(h, b, lit, &p);
}
/* HUF_decodeStreamX2 over [p, end), with HUF_decodeLastSymbolX2 */
static void x2_stream(const huf_t *h, bitd_t *b, uint8_t *lit, int64_t p, int64_t end) {
    while ((bitd_reload(b) == BIT_UNFINISHED) & (p < end - 7)) {
        x2_sym(h, b, lit, &p);
        x2_sym(h, b, lit, &p);
        x2_sym(h, b, lit, &p);
        x2_sym(h, b, lit, &p);
    }
    while ((bitd_reload(b) == BIT_UNFINISHED) & (p <= end - 2)) x2_sym(h, b, lit, &p);
    while (p <= end - 2) x2_sym(h, b, lit, &p);
    if (p < end) {
        const uint64_t v = bitd_look_fast(b, h->log);
        lit[p] = h->seq0[v];
        if (h->len2[v] == 1) {
            b->bc += h->nb2[v];
        } else if (b->bc < 64) {
            b->bc += h->nb2[v];
            if (b->bc > 64) b->bc = 64;
        }
    }
}

/* one stream of dst bytes (HUF_decompress1X*_usingDTable) */
static int huf_1x(const huf_t *h, uint8_t *lit, size_t dst, const uint8_t *src, size_t n) {
    bitd_t b;
    if (bitd_init(&b, src, n) != 0) return 0;
    if (h->type == 0) x1_stream(h, &b, lit, 0, (int64_t)dst);
    else x2_stream(h, &b, lit, 0, (int64_t)dst);
    return bitd_end(&b);
}

/* four streams (HUF_decompress4X*_usingDTable) */
static int huf_4x(const huf_t *h, uint8_t *lit, size_t dst, const uint8_t *src, size_t n) {
    if (n < 10) return 0;
    const size_t l1 = rd16(src), l2 = rd16(src + 2), l3 = rd16(src + 4);
    const size_t l4 = n - (l1 + l2 + l3 + 6); /* size_t: wraps when the jump table overstates */
    if (l4 > n) return 0;
    const uint8_t *i1 = src + 6, *i2 = i1 + l1, *i3 = i2 + l2, *i4 = i3 + l3;
    const int64_t seg = (int64_t)(dst + 3) / 4, oend = (int64_t)dst;
    int64_t op[4] = {0, seg, 2 * seg, 3 * seg};
    const int64_t ostart[5] = {0, seg, 2 * seg, 3 * seg, oend};
    bitd_t b[4];
    if (bitd_init(&b[0], i1, l1) || bitd_init(&b[1], i2, l2) || bitd_init(&b[2], i3, l3) ||
        bitd_init(&b[3], i4, l4))
        return 0;
    if (h->type == 0) {
        const int64_t olimit = oend - 3;
        int end_signal = 1;
        for (; end_signal & (op[3] < olimit);) {
            for (int k = 0; k < 4; k++)
                for (int j = 0; j < 4; j++) x1_sym(h, &b[k], lit, &op[k]);
            for (int k = 0; k < 4; k++) end_signal &= bitd_reload_fast(&b[k]) == BIT_UNFINISHED;
        }
        for (int k = 0; k < 3; k++)
            if (op[k] > ostart[k + 1]) return 0;
        for (int k = 0; k < 4; k++) x1_stream(h, &b[k], lit, op[k], ostart[k + 1]);
    } else {
        const int64_t olimit = oend - 7;
        int end_signal = 1;
        for (; end_signal & (op[3] < olimit);) {
            for (int j = 0; j < 4; j++) /* the streams interleaved symbol by symbol (their 2-byte writes may spill) */
                for (int k = 0; k < 4; k++) x2_sym(h, &b[k], lit, &op[k]);
            int all = 1;
            for (int k = 0; k < 4; k++) all &= bitd_reload_fast(&b[k]) == BIT_UNFINISHED;
            end_signal = all;
        }
        for (int k = 0; k < 3; k++)
            if (op[k] > ostart[k + 1]) return 0;
        for (int k = 0; k < 4; k++) x2_stream(h, &b[k], lit, op[k], ostart[k + 1]);
    }
    return bitd_end(&b[0]) & bitd_end(&b[1]) & bitd_end(&b[2]) & bitd_end(&b[3]);
}

/* ---------------------------------------------------------------- sequences */
static const uint32_t LL_BASE[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,   10,   11,   12,   13,   14,    15,    16,    18,
                                     20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
static const uint8_t LL_BITS[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const uint32_t ML_BASE[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,  14,  15,  16,   17,   18,   19,   20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,  32,  33,  34,   35,   37,   39,   41,
                                     43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
static const uint8_t ML_BITS[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const int16_t LL_DEF[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const int16_t ML_DEF[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const int16_t OF_DEF[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

/* a decoding cell (ZSTD_seqSymbol) */
typedef struct {
    uint16_t next;
    uint8_t nbits, nb_add;
    uint32_t base;
} seqcell_t;
typedef struct {
    unsigned log;
    seqcell_t t[1 << 9];
} seqtab_t;

/* ZSTD_buildFSETable: value = base[symbol], extra bits = bits[symbol] */
static void seq_build(seqtab_t *t, const int16_t *norm, unsigned max_sv, unsigned tlog, const uint32_t *base,
                      const uint8_t *bits, unsigned of) {
    uint8_t sym[1 << 9], nb[1 << 9];
    uint16_t ns[1 << 9];
    fse_spread(sym, ns, nb, norm, max_sv, tlog);
    t->log = tlog;
    for (uint32_t u = 0; u < (1u << tlog); u++) {
        const unsigned s = sym[u];
        t->t[u].next = ns[u];
        t->t[u].nbits = nb[u];
        t->t[u].nb_add = of ? (uint8_t)s : bits[s];
        t->t[u].base = of ? (s < 2 ? s : ((1u << s) - 3)) : base[s];
    }
}
static void seq_rle(seqtab_t *t, unsigned s, const uint32_t *base, const uint8_t *bits, unsigned of) {
    t->log = 0;
    t->t[0].next = 0;
    t->t[0].nbits = 0;
    t->t[0].nb_add = of ? (uint8_t)s : bits[s];
    t->t[0].base = of ? (s < 2 ? s : ((1u << s) - 3)) : base[s];
}

typedef struct {
    uint8_t *out;
    int64_t cap, olen;
    int64_t frame_start;
    uint64_t window;
    int full;
    /* entropy state of the frame (ZSTD_DCtx) */
    huf_t huf;
    int lit_entropy, fse_entropy;
    seqtab_t ll_t, of_t, ml_t;                    /* the compressed / RLE tables */
    seqtab_t ll_def, of_def, ml_def;              /* the predefined ones */
    const seqtab_t *ll, *of, *ml;                 /* the tables in use (repeat: these) */
    uint32_t rep[3];
    const char *err;
} zctx;

static uint8_t g_lit[BLOCK_MAX + LIT_SLACK];

/* ZSTD_buildSeqTable; 0 ok, -1 corruption (srcSize_wrong / table errors) */
static int seq_table(zctx *z, seqtab_t *space, const seqtab_t *def, const seqtab_t **cur, int type,
                     const uint8_t *src, size_t n, size_t *used, unsigned max, unsigned max_log, const uint32_t *base,
                     const uint8_t *bits, unsigned of) {
    *used = 0;
    if (type == 1) { /* set_rle */
        if (!n || src[0] > max) return -1;
        seq_rle(space, src[0], base, bits, of);
        *cur = space;
        *used = 1;
        return 0;
    }
    if (type == 0) { /* set_basic */
        *cur = def;
        return 0;
    }
    if (type == 3) { /* set_repeat */
        if (!z->fse_entropy) return -1;
        return 0;
    }
    int16_t norm[64];
    unsigned ms = max, log;
    int64_t k = fse_read_ncount(norm, &ms, &log, src, n);
    if (k < 0 || log > max_log) return -1;
    seq_build(space, norm, ms, log, base, bits, of);
    *cur = space;
    *used = (size_t)k;
    return 0;
}

typedef struct {
    uint64_t ll, ml, off;
} seq_t;

/* ZSTD_decodeSequence (64-bit, no long-offset split) */
static seq_t decode_seq(zctx *z, bitd_t *b, uint32_t *sll, uint32_t *sml, uint32_t *sof, uint64_t *rep) {
    const seqcell_t lli = z->ll->t[*sll], mli = z->ml->t[*sml], ofi = z->of->t[*sof];
    seq_t s;
    const unsigned llb = lli.nb_add, mlb = mli.nb_add, ofb = ofi.nb_add;
    const unsigned total = llb + mlb + ofb;
    uint64_t off;
    if (ofb > 1) {
        off = ofi.base + bitd_read_fast(b, ofb);
        rep[2] = rep[1];
        rep[1] = rep[0];
        rep[0] = off;
    } else {
        const unsigned ll0 = lli.base == 0;
        if (ofb == 0) {
            if (!ll0) {
                off = rep[0];
            } else {
                off = rep[1];
                rep[1] = rep[0];
                rep[0] = off;
            }
        } else {
            off = ofi.base + ll0 + bitd_read_fast(b, 1);
            uint64_t t = (off == 3) ? rep[0] - 1 : rep[off];
            t += !t;
            if (off != 1) rep[2] = rep[1];
            rep[1] = rep[0];
            rep[0] = off = t;
        }
    }
    s.off = off;
    s.ml = mli.base + (mlb ? bitd_read_fast(b, mlb) : 0);
    if (total >= 57 - (9 + 9 + 8)) bitd_reload(b); /* STREAM_ACCUMULATOR_MIN_64 - (LLFSELog+MLFSELog+OffFSELog) */
    s.ll = lli.base + (llb ? bitd_read_fast(b, llb) : 0);
    *sll = lli.next + (uint32_t)bitd_read(b, lli.nbits);
    *sml = mli.next + (uint32_t)bitd_read(b, mli.nbits);
    *sof = ofi.next + (uint32_t)bitd_read(b, ofi.nbits);
    return s;
}

/* ZSTD_execSequence with a buffer that grows as needed (DataDog retries
 * dstSize_tooSmall with larger buffers): 0 ok, -1 corruption. Output past
 * `cap` is not written (*full is set: the caller retries with more room) but
 * still counted, so that the checks of later sequences see the unlimited
 * buffer's positions. */
static int exec_seq(zctx *z, const seq_t *s, size_t *lit_pos, size_t lit_size, int *full) {
#ifdef ORC_SEQ_HOOK /* (tools/zstd_seqstat.c: sequence statistics; never in the oracle build) */
    ORC_SEQ_HOOK(z, s);
#endif
    if (s->ll > lit_size - *lit_pos) return -1;
    const int64_t produced = z->olen + (int64_t)s->ll - z->frame_start;
    if (s->off > (uint64_t)produced) return -1;
    if (s->ll + s->ml < s->ll || z->olen + (int64_t)(s->ll + s->ml) > z->cap) *full = 1;
    if (!*full) {
        memcpy(z->out + z->olen, g_lit + *lit_pos, s->ll);
        for (uint64_t k = 0; k < s->ml; k++)
            z->out[z->olen + (int64_t)s->ll + (int64_t)k] = z->out[z->olen + (int64_t)s->ll - (int64_t)s->off + (int64_t)k];
    }
    z->olen += (int64_t)(s->ll + s->ml);
    *lit_pos += s->ll;
    return 0;
}

static int g_line;
#define CORRUPT do { g_line = __LINE__; z->err = E_CORRUPT; return 0; } while (0)
#define SRCSIZE do { g_line = __LINE__; z->err = E_SRC; return 0; } while (0)

/* ZSTD_decompressBlock_internal; 1 ok, 0 error (z->err, or z->full) */
static int decode_block(zctx *z, const uint8_t *src, size_t n) {
    if (n >= BLOCK_MAX) SRCSIZE;
    /* ZSTD_decodeLiteralsBlock */
    if (n < 3) CORRUPT;
    const int lt = src[0] & 3, lhl = (src[0] >> 2) & 3;
    size_t lit_size, lit_csize;
    const uint8_t *lit = g_lit;
    if (lt == 2 || lt == 3) { /* compressed / repeat */
        if (lt == 3 && !z->lit_entropy) {
            z->err = E_DICTC;
            return 0;
        }
        if (n < 5) CORRUPT;
        size_t lh;
        int single = 0;
        const uint32_t lhc = rd32(src);
        if (lhl < 2) {
            single = !lhl;
            lh = 3;
            lit_size = (lhc >> 4) & 0x3FF;
            lit_csize = (lhc >> 14) & 0x3FF;
        } else if (lhl == 2) {
            lh = 4;
            lit_size = (lhc >> 4) & 0x3FFF;
            lit_csize = lhc >> 18;
        } else {
            lh = 5;
            lit_size = (lhc >> 4) & 0x3FFFF;
            lit_csize = (lhc >> 22) + ((size_t)src[4] << 10);
        }
        if (lit_size > BLOCK_MAX) CORRUPT;
        if (lit_csize + lh > n) CORRUPT;
        const uint8_t *hs = src + lh;
        int ok;
        if (lt == 3) {
            ok = single ? huf_1x(&z->huf, g_lit, lit_size, hs, lit_csize) : huf_4x(&z->huf, g_lit, lit_size, hs, lit_csize);
        } else if (single) { /* HUF_decompress1X1_DCtx_wksp */
            int64_t k = huf_read_x1(&z->huf, hs, lit_csize);
            ok = k >= 0 && (size_t)k < lit_csize && huf_1x(&z->huf, g_lit, lit_size, hs + k, lit_csize - (size_t)k);
        } else { /* HUF_decompress4X_hufOnly_wksp */
            ok = 0;
            if (lit_size != 0 && lit_csize != 0) {
                const int x2 = huf_select_x2(lit_size, lit_csize);
                int64_t k = x2 ? huf_read_x2(&z->huf, hs, lit_csize) : huf_read_x1(&z->huf, hs, lit_csize);
                ok = k >= 0 && (size_t)k < lit_csize && huf_4x(&z->huf, g_lit, lit_size, hs + k, lit_csize - (size_t)k);
            }
        }
        if (!ok) CORRUPT;
        z->lit_entropy = 1;
        lit_csize += lh;
    } else {
        size_t lh;
        if (lhl == 1) {
            lh = 2;
            lit_size = rd16(src) >> 4;
        } else if (lhl == 3) {
            lh = 3;
            lit_size = rd24(src) >> 4;
        } else {
            lh = 1;
            lit_size = src[0] >> 3;
        }
        if (lt == 0) { /* raw */
            if (lit_size + lh > n) CORRUPT;
            lit = src + lh;
            lit_csize = lh + lit_size;
        } else { /* RLE */
            if (lh == 3 && n < 4) CORRUPT;
            if (lit_size > BLOCK_MAX) CORRUPT;
            memset(g_lit, src[lh], lit_size);
            lit_csize = lh + 1;
        }
    }
    if (lit != g_lit) {
        memcpy(g_lit, lit, lit_size);
        lit = g_lit;
    }
    /* ZSTD_decodeSeqHeaders */
    const uint8_t *ip = src + lit_csize;
    const uint8_t *iend = src + n;
    if (ip >= iend) SRCSIZE; /* MIN_SEQUENCES_SIZE */
    int nseq = *ip++;
    if (!nseq) {
        if (iend - ip != 0) SRCSIZE;
    } else {
        if (nseq > 0x7F) {
            if (nseq == 0xFF) {
                if (ip + 2 > iend) SRCSIZE;
                nseq = (int)rd16(ip) + 0x7F00;
                ip += 2;
            } else {
                if (ip >= iend) SRCSIZE;
                nseq = ((nseq - 0x80) << 8) + *ip++;
            }
        }
        if (ip + 1 > iend) SRCSIZE;
        const int types = *ip++;
        size_t used;
        if (seq_table(z, &z->ll_t, &z->ll_def, &z->ll, types >> 6, ip, (size_t)(iend - ip), &used, 35, 9, LL_BASE,
                      LL_BITS, 0))
            CORRUPT;
        ip += used;
        if (seq_table(z, &z->of_t, &z->of_def, &z->of, (types >> 4) & 3, ip, (size_t)(iend - ip), &used, 31, 8, NULL,
                      NULL, 1))
            CORRUPT;
        ip += used;
        if (seq_table(z, &z->ml_t, &z->ml_def, &z->ml, (types >> 2) & 3, ip, (size_t)(iend - ip), &used, 52, 9,
                      ML_BASE, ML_BITS, 0))
            CORRUPT;
        ip += used;
    }
    /* ZSTD_decompressSequences(Long) */
    size_t lit_pos = 0;
    if (nseq) {
        uint32_t share = 0; /* ZSTD_getLongOffsetsShare */
        for (uint32_t u = 0; u < (1u << z->of->log); u++) share += z->of->t[u].nb_add > 22;
        share <<= (8 - z->of->log);
        const int long_dec = z->window > (1u << 24) && nseq > 4 && share >= 7;
        z->fse_entropy = 1;
        uint64_t rep[3] = {z->rep[0], z->rep[1], z->rep[2]};
        bitd_t b;
        if (bitd_init(&b, ip, (size_t)(iend - ip)) != 0) CORRUPT;
        uint32_t sll = (uint32_t)bitd_read(&b, z->ll->log);
        bitd_reload(&b);
        uint32_t sof = (uint32_t)bitd_read(&b, z->of->log);
        bitd_reload(&b);
        uint32_t sml = (uint32_t)bitd_read(&b, z->ml->log);
        bitd_reload(&b);
        int full = 0;
        if (!long_dec) { /* every sequence decoded and executed; errors reported after the loop */
            int err = 0;
            for (int i = 0; i < nseq; i++) {
                const seq_t s = decode_seq(z, &b, &sll, &sml, &sof, rep);
                const int64_t olen0 = z->olen;
                const size_t lp0 = lit_pos;
                if (exec_seq(z, &s, &lit_pos, lit_size, &full)) { /* op and the literals do not advance */
                    err = 1;
                    z->olen = olen0;
                    lit_pos = lp0;
                }
                bitd_reload(&b);
            }
            if (err) CORRUPT;
            if (bitd_reload(&b) < BIT_COMPLETED) CORRUPT;
        } else { /* decode 4 ahead; stop on an over-read before the last; no end check */
            seq_t q[4];
            const int adv = nseq < 4 ? nseq : 4;
            int i;
            for (i = 0; (bitd_reload(&b) <= BIT_COMPLETED) && i < adv; i++) q[i] = decode_seq(z, &b, &sll, &sml, &sof, rep);
            if (i < adv) CORRUPT;
            for (; (bitd_reload(&b) <= BIT_COMPLETED) && i < nseq; i++) {
                const seq_t s = decode_seq(z, &b, &sll, &sml, &sof, rep);
                if (exec_seq(z, &q[(i - 4) & 3], &lit_pos, lit_size, &full)) CORRUPT;
                q[i & 3] = s;
            }
            if (i < nseq) CORRUPT;
            for (i -= adv; i < nseq; i++)
                if (exec_seq(z, &q[i & 3], &lit_pos, lit_size, &full)) CORRUPT;
        }
        if (full) {
            z->full = 1;
            return 0;
        }
        for (int k = 0; k < 3; k++) z->rep[k] = (uint32_t)rep[k];
    }
    /* last literals */
    if (z->olen + (int64_t)(lit_size - lit_pos) > z->cap) {
        z->full = 1;
        return 0;
    }
    memcpy(z->out + z->olen, g_lit + lit_pos, lit_size - lit_pos);
    z->olen += (int64_t)(lit_size - lit_pos);
    return 1;
}
int orc_zstd_last_line(void) { return g_line; }

static const uint8_t kDidLen[4] = {0, 1, 2, 4}, kFcsLen[4] = {0, 2, 4, 8};

/* ZSTD_decompressFrame: bytes consumed, -1 on error */
static int64_t decode_frame(zctx *z, const uint8_t *in, int64_t n) {
    if (n < 6 + 3) {
        z->err = E_SRC;
        return -1;
    }
    const int fhd = in[4];
    const int single = (fhd >> 5) & 1, fcs_id = fhd >> 6, did_id = fhd & 3;
    const int64_t fhs = 5 + !single + kDidLen[did_id] + kFcsLen[fcs_id] + (single && !fcs_id);
    if (n < fhs + 3) {
        z->err = E_SRC;
        return -1;
    }
    if (rd32(in) != ZMAGIC) {
        z->err = E_PREFIX;
        return -1;
    }
    if (fhd & 0x08) {
        z->err = E_NOTSUP;
        return -1;
    }
    int64_t pos = 5;
    uint64_t window = 0;
    if (!single) {
        const int wd = in[pos++];
        const int wlog = 10 + (wd >> 3);
        if (wlog > 31) {
            z->err = E_WINDOW;
            return -1;
        }
        window = (uint64_t)1 << wlog;
        window += (window >> 3) * (uint64_t)(wd & 7);
    }
    uint64_t did = 0;
    for (int i = 0; i < kDidLen[did_id]; i++) did |= (uint64_t)in[pos + i] << (8 * i);
    pos += kDidLen[did_id];
    uint64_t fcs = UINT64_MAX; /* ZSTD_CONTENTSIZE_UNKNOWN (a declared 2^64-1 reads the same) */
    if (fcs_id == 0) {
        if (single) fcs = in[pos];
    } else if (fcs_id == 1) {
        fcs = (uint64_t)rd16(in + pos) + 256;
    } else if (fcs_id == 2) {
        fcs = rd32(in + pos);
    } else {
        fcs = rd64(in + pos);
    }
    pos = fhs;
    if (single) window = fcs;
    if (did != 0) {
        z->err = E_DICT;
        return -1;
    }
    const int checksum = (fhd >> 2) & 1;
    z->window = window;
    z->frame_start = z->olen;
    z->lit_entropy = z->fse_entropy = 0;
    z->rep[0] = 1;
    z->rep[1] = 4;
    z->rep[2] = 8;
    for (;;) {
        if (n - pos < 3) {
            z->err = E_SRC;
            return -1;
        }
        const uint32_t bh = rd24(in + pos);
        const int last = bh & 1, type = (bh >> 1) & 3;
        const uint64_t size = bh >> 3;
        const uint64_t csize = type == 1 ? 1 : size;
        if (type == 3) {
            z->err = E_CORRUPT;
            return -1;
        }
        pos += 3;
        if (csize > (uint64_t)(n - pos)) {
            z->err = E_SRC;
            return -1;
        }
        if (type == 0) {
            if (z->olen + (int64_t)size > z->cap) {
                z->full = 1;
                return -1;
            }
            memcpy(z->out + z->olen, in + pos, size);
            z->olen += (int64_t)size;
        } else if (type == 1) {
            if (z->olen + (int64_t)size > z->cap) {
                z->full = 1;
                return -1;
            }
            memset(z->out + z->olen, in[pos], size);
            z->olen += (int64_t)size;
        } else if (!decode_block(z, in + pos, size)) {
            return -1;
        }
        pos += (int64_t)csize;
        if (last) break;
    }
    if (fcs != UINT64_MAX && (uint64_t)(z->olen - z->frame_start) != fcs) {
        z->err = E_CORRUPT;
        return -1;
    }
    if (checksum) {
        if (n - pos < 4) {
            z->err = E_CHECKSUM;
            return -1;
        }
        const uint32_t want = rd32(in + pos);
        const uint32_t got = (uint32_t)xxh64(z->out + z->frame_start, (size_t)(z->olen - z->frame_start), 0);
        if (want != got) {
            z->err = E_CHECKSUM;
            return -1;
        }
        pos += 4;
    }
    return pos;
}

static void build_defaults(zctx *z) {
    seq_build(&z->ll_def, LL_DEF, 35, 6, LL_BASE, LL_BITS, 0);
    seq_build(&z->of_def, OF_DEF, 28, 5, NULL, NULL, 1);
    seq_build(&z->ml_def, ML_DEF, 52, 6, ML_BASE, ML_BITS, 0);
}

/* ZSTD_decompress = ZSTD_decompressMultiFrame */
int orc_zstd_decompress(const uint8_t *in, int64_t n, uint8_t *out, int64_t cap, int64_t *out_len,
                        const char **msg) {
    static zctx z;
    memset(&z, 0, sizeof(z));
    build_defaults(&z);
    z.ll = &z.ll_def;
    z.of = &z.of_def;
    z.ml = &z.ml_def;
    z.out = out;
    z.cap = cap;
    *msg = "";
    *out_len = 0;
    if (n <= 0) { /* DataDog: ErrEmptySlice before libzstd is called (the scanner maps it) */
        *msg = E_SRC;
        return ORC_ZSTD_ERROR;
    }
    int64_t pos = 0;
    int more_than_one = 0;
    while (n - pos >= 5) {
        const uint32_t magic = rd32(in + pos);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) { /* readSkippableFrameSize */
            if (n - pos < 8) {
                z.err = E_SRC;
                goto fail;
            }
            const uint32_t sz = rd32(in + pos + 4);
            if ((uint32_t)(sz + 8) < sz) {
                z.err = E_NOTSUP;
                goto fail;
            }
            if ((int64_t)sz + 8 > n - pos) {
                z.err = E_SRC;
                goto fail;
            }
            pos += (int64_t)sz + 8;
            continue;
        }
        const int64_t k = decode_frame(&z, in + pos, n - pos);
        if (k < 0) {
            if (z.err == E_PREFIX && more_than_one) z.err = E_SRC;
            goto fail;
        }
        pos += k;
        more_than_one = 1;
    }
    if (n - pos != 0) {
        z.err = E_SRC;
        goto fail;
    }
    *out_len = z.olen;
    (void)E_TABLELOG;
    return ORC_ZSTD_OK;
fail:
    *out_len = z.olen;
    if (z.full) return ORC_ZSTD_OUTPUT_FULL;
    *msg = z.err ? z.err : E_CORRUPT;
    return ORC_ZSTD_ERROR;
}

/* ZSTD_getDecompressedSize-like bound: the sum of declared frame sizes, -1 if
 * any frame does not declare one */
int64_t orc_zstd_content_size(const uint8_t *in, int64_t n) {
    if (n < 6 || rd32(in) != ZMAGIC) return -1;
    int fhd = in[4];
    int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, did_flag = fhd & 3;
    static const int did_len[4] = {0, 1, 2, 4};
    int64_t pos = 5 + (single ? 0 : 1) + did_len[did_flag];
    int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : (fcs_flag == 2 ? 4 : 8));
    if (fcs_len == 0 || pos + fcs_len > n) return -1;
    if (fcs_len == 1) return in[pos];
    if (fcs_len == 2) return rd16(in + pos) + 256;
    if (fcs_len == 4) return rd32(in + pos);
    return (int64_t)rd64(in + pos);
}
