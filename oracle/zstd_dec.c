/*
 * ORACLE — test infrastructure only. Never linked into the product path.
 *
 * CPU restatement of Zstandard frame decoding (RFC 8878) as used by the
 * reference's "zstd" transformer: recordiozstd.zstdUncompress
 * (recordio/recordiozstd/recordiozstd.go:67-78) -> compress/zstd.Decompress
 * (compress/zstd/zstd_cgo.go:34-41) -> github.com/DataDog/zstd v1.4.1
 * (go.mod:7; not vendored under /root/reference), i.e. libzstd's
 * ZSTD_decompress over every frame of the block. Restated from the format
 * specification: frame header (3.1.1.1), blocks (3.1.1.2), literals section
 * (3.1.1.3.1) with Huffman trees (4.2) whose weights may be FSE-coded (4.2.1.2),
 * sequences section (3.1.1.3.2) with FSE tables (4.1), the predefined
 * distributions (3.1.1.3.2.2), sequence execution with repeat offsets
 * (3.1.1.4-5), skippable frames, and the XXH64 content checksum.
 * Errors carry libzstd-style names; only error-versus-success parity is
 * claimed for them.
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

/* ---------------------------------------------------------------- bit readers */
/* forward reader (FSE table descriptions) */
typedef struct {
    const uint8_t *p;
    size_t n;
    uint64_t pos; /* bits */
} fwd_t;
static uint32_t fwd_peek(const fwd_t *r, int nb) {
    uint32_t v = 0;
    for (int i = 0; i < nb; i++) {
        uint64_t b = r->pos + i;
        uint32_t bit = (b >> 3) < r->n ? (r->p[b >> 3] >> (b & 7)) & 1u : 0u;
        v |= bit << i;
    }
    return v;
}
static uint32_t fwd_read(fwd_t *r, int nb) {
    uint32_t v = fwd_peek(r, nb);
    r->pos += nb;
    return v;
}

/* backward reader (Huffman streams, FSE streams): the last byte's highest set
 * bit marks the start; bits are consumed from the top down */
typedef struct {
    const uint8_t *p;
    int64_t bit; /* bits remaining above position 0 (may go negative: overflow) */
} bwd_t;
static int bwd_init(bwd_t *r, const uint8_t *p, size_t n) {
    if (n == 0) return 0;
    uint8_t last = p[n - 1];
    if (last == 0) return 0;
    r->p = p;
    r->bit = (int64_t)n * 8 - (8 - highbit32(last));
    return 1;
}
static uint64_t bwd_read(bwd_t *r, int nb) {
    if (nb == 0) return 0;
    r->bit -= nb;
    uint64_t v = 0;
    for (int i = 0; i < nb; i++) {
        int64_t b = r->bit + i;
        uint64_t bit = (b >= 0) ? (r->p[b >> 3] >> (b & 7)) & 1u : 0u;
        v |= bit << i;
    }
    return v;
}
static uint64_t bwd_peek(const bwd_t *r, int nb) {
    bwd_t t = *r;
    return bwd_read(&t, nb);
}

/* ---------------------------------------------------------------- FSE */
typedef struct {
    uint8_t sym;
    uint8_t nbits;
    uint16_t base;
} fse_cell;
typedef struct {
    int log;
    fse_cell t[1 << 9];
} fse_t;

/* FSE_readNCount: returns bytes consumed, -1 on error */
static int fse_read_ncount(int16_t *norm, int *max_sym, int *log, const uint8_t *src, size_t n, int max_log) {
    fwd_t r = {src, n, 0};
    int al = (int)fwd_read(&r, 4) + 5;
    if (al > max_log) return -1;
    *log = al;
    int remaining = (1 << al) + 1;
    int threshold = 1 << al;
    int nbits = al + 1;
    int sym = 0;
    int prev0 = 0;
    while (remaining > 1 && sym <= *max_sym) {
        if (prev0) {
            int n0 = sym;
            while (fwd_peek(&r, 16) == 0xFFFF) {
                n0 += 24;
                r.pos += 16;
            }
            while (fwd_peek(&r, 2) == 3) {
                n0 += 3;
                r.pos += 2;
            }
            n0 += (int)fwd_read(&r, 2);
            if (n0 > *max_sym) return -1;
            while (sym < n0) norm[sym++] = 0;
            if (r.pos > 8 * (uint64_t)n) return -1;
        }
        int max = (2 * threshold - 1) - remaining;
        int count;
        int low = (int)fwd_peek(&r, nbits - 1);
        if (low < max) {
            count = low;
            r.pos += nbits - 1;
        } else {
            count = (int)fwd_peek(&r, nbits);
            if (count >= threshold) count -= max;
            r.pos += nbits;
        }
        count--;
        remaining -= count < 0 ? -count : count;
        norm[sym++] = (int16_t)count;
        prev0 = (count == 0);
        while (remaining < threshold) {
            nbits--;
            threshold >>= 1;
        }
        if (r.pos > 8 * (uint64_t)n) return -1;
    }
    if (remaining != 1) return -1;
    *max_sym = sym - 1;
    return (int)((r.pos + 7) >> 3);
}

static int fse_build(fse_t *f, const int16_t *norm, int max_sym, int log) {
    int size = 1 << log;
    int high = size - 1;
    uint16_t next[256];
    f->log = log;
    for (int s = 0; s <= max_sym; s++) {
        if (norm[s] == -1) {
            f->t[high--].sym = (uint8_t)s;
            next[s] = 1;
        } else {
            next[s] = (uint16_t)norm[s];
        }
    }
    int step = (size >> 1) + (size >> 3) + 3;
    int mask = size - 1;
    int pos = 0;
    for (int s = 0; s <= max_sym; s++) {
        for (int i = 0; i < norm[s]; i++) {
            f->t[pos].sym = (uint8_t)s;
            do {
                pos = (pos + step) & mask;
            } while (pos > high);
        }
    }
    if (pos != 0) return 0;
    for (int u = 0; u < size; u++) {
        int s = f->t[u].sym;
        uint32_t ns = next[s]++;
        int nb = log - highbit32(ns);
        f->t[u].nbits = (uint8_t)nb;
        f->t[u].base = (uint16_t)((ns << nb) - size);
    }
    return 1;
}

static void fse_rle(fse_t *f, int sym) {
    f->log = 0;
    f->t[0].sym = (uint8_t)sym;
    f->t[0].nbits = 0;
    f->t[0].base = 0;
}

/* ---------------------------------------------------------------- Huffman */
typedef struct {
    int max_bits;
    uint8_t sym[1 << 11];
    uint8_t nbits[1 << 11];
} huf_t;

/* Huffman tree description -> table; returns bytes consumed or -1 */
static int huf_read(huf_t *h, const uint8_t *src, size_t n) {
    if (n < 1) return -1;
    uint8_t w[256];
    int nw = 0;
    int hb = src[0];
    size_t used;
    if (hb >= 128) {
        nw = hb - 127;
        used = 1 + (size_t)(nw + 1) / 2;
        if (used > n) return -1;
        for (int i = 0; i < nw; i++) {
            uint8_t b = src[1 + i / 2];
            w[i] = (i & 1) ? (b & 15) : (b >> 4);
        }
    } else {
        used = 1 + (size_t)hb;
        if (used > n || hb == 0) return -1;
        int16_t norm[16];
        int max_sym = 15, log;
        int k = fse_read_ncount(norm, &max_sym, &log, src + 1, hb, 6);
        if (k < 0 || k > hb) return -1;
        static fse_t f;
        if (!fse_build(&f, norm, max_sym, log)) return -1;
        bwd_t r;
        if (!bwd_init(&r, src + 1 + k, hb - k)) return -1;
        uint32_t s1 = (uint32_t)bwd_read(&r, log), s2 = (uint32_t)bwd_read(&r, log);
        for (;;) {
            if (nw > 254) return -1;
            w[nw++] = f.t[s1].sym;
            s1 = f.t[s1].base + (uint32_t)bwd_read(&r, f.t[s1].nbits);
            if (r.bit < 0) {
                w[nw++] = f.t[s2].sym;
                break;
            }
            if (nw > 254) return -1;
            w[nw++] = f.t[s2].sym;
            s2 = f.t[s2].base + (uint32_t)bwd_read(&r, f.t[s2].nbits);
            if (r.bit < 0) {
                w[nw++] = f.t[s1].sym;
                break;
            }
        }
    }
    /* implied last weight */
    uint32_t total = 0;
    for (int i = 0; i < nw; i++) {
        if (w[i] > 11) return -1;
        if (w[i]) total += 1u << (w[i] - 1);
    }
    if (total == 0) return -1;
    int max_bits = highbit32(total) + 1;
    uint32_t rest = (1u << max_bits) - total;
    if (rest & (rest - 1)) return -1;
    if (nw + 1 > 256 || max_bits > 11) return -1;
    w[nw++] = (uint8_t)(highbit32(rest) + 1);
    h->max_bits = max_bits;
    uint32_t rank[13] = {0};
    for (int i = 0; i < nw; i++) rank[w[i]]++;
    uint32_t start[13];
    uint32_t acc = 0;
    for (int wt = 1; wt <= max_bits; wt++) {
        start[wt] = acc;
        acc += rank[wt] << (wt - 1);
    }
    if (acc != (1u << max_bits)) return -1;
    for (int s = 0; s < nw; s++) {
        int wt = w[s];
        if (!wt) continue;
        uint32_t len = 1u << (wt - 1);
        for (uint32_t j = 0; j < len; j++) {
            h->sym[start[wt] + j] = (uint8_t)s;
            h->nbits[start[wt] + j] = (uint8_t)(max_bits + 1 - wt);
        }
        start[wt] += len;
    }
    return (int)used;
}

static int huf_stream(const huf_t *h, const uint8_t *src, size_t n, uint8_t *out, size_t count) {
    bwd_t r;
    if (!bwd_init(&r, src, n)) return 0;
    for (size_t i = 0; i < count; i++) {
        uint32_t v = (uint32_t)bwd_peek(&r, h->max_bits);
        out[i] = h->sym[v];
        bwd_read(&r, h->nbits[v]);
        if (r.bit < 0) return 0;
    }
    return r.bit == 0;
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
/* 29 predefined offset codes; codes 29..31 (seq_table's max_sym) have count 0 */
static const int16_t OF_DEF[32] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, 0, 0, 0};

typedef struct {
    /* output */
    uint8_t *out;
    int64_t cap, olen;
    int64_t frame_start;
    /* persistent across blocks of a frame */
    huf_t huf;
    int have_huf;
    fse_t ll, of, ml;
    int have_ll, have_of, have_ml;
    uint64_t rep[3];
    uint64_t window;
    const char *err;
    int full;
} zctx;

static uint8_t g_lit[BLOCK_MAX + 64];
static int g_line;
#define CORRUPT do { g_line = __LINE__; goto corrupt; } while (0)

/* returns 1 ok, 0 error (err set) */
static int seq_table(zctx *z, fse_t *f, int *have, int mode, const uint8_t *src, size_t n, size_t *used,
                     const int16_t *def, int def_log, int max_sym, int max_log) {
    *used = 0;
    if (mode == 0) {
        fse_build(f, def, max_sym, def_log);
        *have = 1;
        return 1;
    }
    if (mode == 1) {
        if (n < 1 || src[0] > max_sym) {
            z->err = E_CORRUPT;
            return 0;
        }
        fse_rle(f, src[0]);
        *used = 1;
        *have = 1;
        return 1;
    }
    if (mode == 2) {
        int16_t norm[64];
        int ms = max_sym, log;
        int k = fse_read_ncount(norm, &ms, &log, src, n, max_log);
        if (k < 0 || (size_t)k > n) {
            z->err = E_CORRUPT;
            return 0;
        }
        if (!fse_build(f, norm, ms, log)) {
            z->err = E_CORRUPT;
            return 0;
        }
        *used = (size_t)k;
        *have = 1;
        return 1;
    }
    if (!*have) { /* repeat without a previous table */
        z->err = E_CORRUPT;
        return 0;
    }
    return 1;
}

static int decode_block(zctx *z, const uint8_t *src, size_t n) {
    if (n < 1) {
        z->err = E_CORRUPT;
        return 0;
    }
    /* literals section */
    int lt = src[0] & 3, sf = (src[0] >> 2) & 3;
    size_t regen = 0, csize = 0, hsz = 0;
    int streams = 1;
    if (lt == 0 || lt == 1) {
        if (sf == 0 || sf == 2) {
            regen = src[0] >> 3;
            hsz = 1;
        } else if (sf == 1) {
            if (n < 2) CORRUPT;
            regen = (src[0] >> 4) + ((size_t)src[1] << 4);
            hsz = 2;
        } else {
            if (n < 3) CORRUPT;
            regen = (src[0] >> 4) + ((size_t)src[1] << 4) + ((size_t)src[2] << 12);
            hsz = 3;
        }
    } else {
        if (sf == 0 || sf == 1) {
            if (n < 3) CORRUPT;
            uint32_t v = rd24(src);
            regen = (v >> 4) & 0x3FF;
            csize = (v >> 14) & 0x3FF;
            hsz = 3;
            streams = sf == 0 ? 1 : 4;
        } else if (sf == 2) {
            if (n < 4) CORRUPT;
            uint32_t v = rd32(src);
            regen = (v >> 4) & 0x3FFF;
            csize = (v >> 18) & 0x3FFF;
            hsz = 4;
            streams = 4;
        } else {
            if (n < 5) CORRUPT;
            uint64_t v = rd32(src) | ((uint64_t)src[4] << 32);
            regen = (v >> 4) & 0x3FFFF;
            csize = (v >> 22) & 0x3FFFF;
            hsz = 5;
            streams = 4;
        }
    }
    if (regen > BLOCK_MAX) CORRUPT;
    size_t pos = hsz;
    if (lt == 0) {
        if (pos + regen > n) CORRUPT;
        memcpy(g_lit, src + pos, regen);
        pos += regen;
    } else if (lt == 1) {
        if (pos + 1 > n) CORRUPT;
        memset(g_lit, src[pos], regen);
        pos += 1;
    } else {
        if (pos + csize > n) CORRUPT;
        const uint8_t *hs = src + pos;
        size_t hn = csize;
        if (lt == 2) {
            int k = huf_read(&z->huf, hs, hn);
            if (k < 0) CORRUPT;
            z->have_huf = 1;
            hs += k;
            hn -= (size_t)k;
        } else if (!z->have_huf) {
            CORRUPT;
        }
        if (streams == 1) {
            if (!huf_stream(&z->huf, hs, hn, g_lit, regen)) CORRUPT;
        } else {
            if (hn < 6) CORRUPT;
            size_t s1 = rd16(hs), s2 = rd16(hs + 2), s3 = rd16(hs + 4);
            if (6 + s1 + s2 + s3 > hn) CORRUPT;
            size_t s4 = hn - 6 - s1 - s2 - s3;
            size_t seg = (regen + 3) / 4;
            if (3 * seg > regen) CORRUPT;
            const uint8_t *p = hs + 6;
            if (!huf_stream(&z->huf, p, s1, g_lit, seg)) CORRUPT;
            if (!huf_stream(&z->huf, p + s1, s2, g_lit + seg, seg)) CORRUPT;
            if (!huf_stream(&z->huf, p + s1 + s2, s3, g_lit + 2 * seg, seg)) CORRUPT;
            if (!huf_stream(&z->huf, p + s1 + s2 + s3, s4, g_lit + 3 * seg, regen - 3 * seg)) CORRUPT;
        }
        pos += csize;
    }
    /* sequences section */
    if (pos >= n) CORRUPT;
    size_t nseq;
    int b0 = src[pos];
    if (b0 == 0) {
        nseq = 0;
        pos += 1;
    } else if (b0 < 128) {
        nseq = (size_t)b0;
        pos += 1;
    } else if (b0 < 255) {
        if (pos + 2 > n) CORRUPT;
        nseq = ((size_t)(b0 - 128) << 8) + src[pos + 1];
        pos += 2;
    } else {
        if (pos + 3 > n) CORRUPT;
        nseq = src[pos + 1] + ((size_t)src[pos + 2] << 8) + 0x7F00;
        pos += 3;
    }
    size_t lit_pos = 0;
    if (nseq > 0) {
        if (pos >= n) CORRUPT;
        int modes = src[pos++];
        if (modes & 3) CORRUPT;
        size_t used;
        if (!seq_table(z, &z->ll, &z->have_ll, (modes >> 6) & 3, src + pos, n - pos, &used, LL_DEF, 6, 35, 9))
            return 0;
        pos += used;
        if (!seq_table(z, &z->of, &z->have_of, (modes >> 4) & 3, src + pos, n - pos, &used, OF_DEF, 5, 31, 8))
            return 0;
        pos += used;
        if (!seq_table(z, &z->ml, &z->have_ml, (modes >> 2) & 3, src + pos, n - pos, &used, ML_DEF, 6, 52, 9))
            return 0;
        pos += used;
        bwd_t r;
        if (!bwd_init(&r, src + pos, n - pos)) CORRUPT;
        uint32_t sll = (uint32_t)bwd_read(&r, z->ll.log);
        uint32_t sof = (uint32_t)bwd_read(&r, z->of.log);
        uint32_t sml = (uint32_t)bwd_read(&r, z->ml.log);
        for (size_t i = 0; i < nseq; i++) {
            int llc = z->ll.t[sll].sym, mlc = z->ml.t[sml].sym, ofc = z->of.t[sof].sym;
            if (llc > 35 || mlc > 52 || ofc > 31) CORRUPT;
            uint64_t ofv = ((uint64_t)1 << ofc) + bwd_read(&r, ofc);
            uint64_t ml = ML_BASE[mlc] + bwd_read(&r, ML_BITS[mlc]);
            uint64_t ll = LL_BASE[llc] + bwd_read(&r, LL_BITS[llc]);
            uint64_t off;
            if (ofv > 3) {
                off = ofv - 3;
                z->rep[2] = z->rep[1];
                z->rep[1] = z->rep[0];
                z->rep[0] = off;
            } else {
                uint64_t idx = ofv + (ll == 0 ? 1 : 0);
                if (idx == 1) {
                    off = z->rep[0];
                } else if (idx == 2) {
                    off = z->rep[1];
                    z->rep[1] = z->rep[0];
                    z->rep[0] = off;
                } else if (idx == 3) {
                    off = z->rep[2];
                    z->rep[2] = z->rep[1];
                    z->rep[1] = z->rep[0];
                    z->rep[0] = off;
                } else {
                    off = z->rep[0] - 1;
                    if (off == 0) CORRUPT;
                    z->rep[2] = z->rep[1];
                    z->rep[1] = z->rep[0];
                    z->rep[0] = off;
                }
            }
            if (i + 1 < nseq) {
                sll = z->ll.t[sll].base + (uint32_t)bwd_read(&r, z->ll.t[sll].nbits);
                sml = z->ml.t[sml].base + (uint32_t)bwd_read(&r, z->ml.t[sml].nbits);
                sof = z->of.t[sof].base + (uint32_t)bwd_read(&r, z->of.t[sof].nbits);
            }
            if (r.bit < 0) CORRUPT;
            /* execute */
            if (lit_pos + ll > regen) CORRUPT;
            if (z->olen + (int64_t)(ll + ml) > z->cap) {
                z->full = 1;
                return 0;
            }
            memcpy(z->out + z->olen, g_lit + lit_pos, ll);
            z->olen += (int64_t)ll;
            lit_pos += ll;
            int64_t produced = z->olen - z->frame_start;
            if (off == 0 || (int64_t)off > produced) CORRUPT;
            for (uint64_t k = 0; k < ml; k++) z->out[z->olen + k] = z->out[z->olen - (int64_t)off + k];
            z->olen += (int64_t)ml;
        }
        if (r.bit != 0) CORRUPT;
    }
    /* remaining literals */
    if (z->olen + (int64_t)(regen - lit_pos) > z->cap) {
        z->full = 1;
        return 0;
    }
    memcpy(z->out + z->olen, g_lit + lit_pos, regen - lit_pos);
    z->olen += (int64_t)(regen - lit_pos);
    return 1;
corrupt:
    z->err = E_CORRUPT;
    return 0;
}
int orc_zstd_last_line(void) { return g_line; }

/* one frame at in[0..n); returns bytes consumed, -1 on error */
static int64_t decode_frame(zctx *z, const uint8_t *in, int64_t n) {
    if (n < 4) {
        z->err = E_SRC;
        return -1;
    }
    uint32_t magic = rd32(in);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) { /* skippable frame */
        if (n < 8) {
            z->err = E_SRC;
            return -1;
        }
        uint64_t sz = rd32(in + 4);
        if (8 + (int64_t)sz > n) {
            z->err = E_SRC;
            return -1;
        }
        return 8 + (int64_t)sz;
    }
    if (magic != ZMAGIC) {
        z->err = E_PREFIX;
        return -1;
    }
    int64_t pos = 4;
    if (pos >= n) {
        z->err = E_SRC;
        return -1;
    }
    int fhd = in[pos++];
    int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, reserved = (fhd >> 3) & 1, checksum = (fhd >> 2) & 1;
    int did_flag = fhd & 3;
    if (reserved) {
        z->err = E_NOTSUP;
        return -1;
    }
    uint64_t window = 0;
    if (!single) {
        if (pos >= n) {
            z->err = E_SRC;
            return -1;
        }
        int wd = in[pos++];
        int wlog = 10 + (wd >> 3);
        if (wlog > 31) {
            z->err = E_WINDOW;
            return -1;
        }
        uint64_t base = (uint64_t)1 << wlog;
        window = base + (base / 8) * (uint64_t)(wd & 7);
    }
    static const int did_len[4] = {0, 1, 2, 4};
    if (pos + did_len[did_flag] > n) {
        z->err = E_SRC;
        return -1;
    }
    uint64_t did = 0;
    for (int i = 0; i < did_len[did_flag]; i++) did |= (uint64_t)in[pos + i] << (8 * i);
    pos += did_len[did_flag];
    if (did != 0) {
        z->err = E_DICT;
        return -1;
    }
    int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : (fcs_flag == 2 ? 4 : 8));
    if (pos + fcs_len > n) {
        z->err = E_SRC;
        return -1;
    }
    int64_t fcs = -1;
    if (fcs_len == 1) fcs = in[pos];
    else if (fcs_len == 2) fcs = rd16(in + pos) + 256;
    else if (fcs_len == 4) fcs = rd32(in + pos);
    else if (fcs_len == 8) fcs = (int64_t)rd64(in + pos);
    pos += fcs_len;
    if (single) window = (uint64_t)fcs;
    z->window = window;
    uint64_t block_max = window < BLOCK_MAX ? window : BLOCK_MAX;
    z->frame_start = z->olen;
    z->have_huf = z->have_ll = z->have_of = z->have_ml = 0;
    z->rep[0] = 1;
    z->rep[1] = 4;
    z->rep[2] = 8;
    for (;;) {
        if (pos + 3 > n) {
            z->err = E_SRC;
            return -1;
        }
        uint32_t bh = rd24(in + pos);
        pos += 3;
        int last = bh & 1, type = (bh >> 1) & 3;
        uint64_t size = bh >> 3;
        if (type == 3) {
            z->err = E_CORRUPT;
            return -1;
        }
        if (type == 0) {
            if (size > block_max) {
                z->err = E_CORRUPT;
                return -1;
            }
            if (pos + (int64_t)size > n) {
                z->err = E_SRC;
                return -1;
            }
            if (z->olen + (int64_t)size > z->cap) {
                z->full = 1;
                return -1;
            }
            memcpy(z->out + z->olen, in + pos, size);
            z->olen += (int64_t)size;
            pos += (int64_t)size;
        } else if (type == 1) {
            if (size > block_max) {
                z->err = E_CORRUPT;
                return -1;
            }
            if (pos + 1 > n) {
                z->err = E_SRC;
                return -1;
            }
            if (z->olen + (int64_t)size > z->cap) {
                z->full = 1;
                return -1;
            }
            memset(z->out + z->olen, in[pos], size);
            z->olen += (int64_t)size;
            pos += 1;
        } else {
            if (size > block_max) {
                z->err = E_CORRUPT;
                return -1;
            }
            if (pos + (int64_t)size > n) {
                z->err = E_SRC;
                return -1;
            }
            if (!decode_block(z, in + pos, size)) return -1;
            pos += (int64_t)size;
        }
        if (last) break;
    }
    if (fcs >= 0 && z->olen - z->frame_start != fcs) {
        z->err = E_CORRUPT;
        return -1;
    }
    if (checksum) {
        if (pos + 4 > n) {
            z->err = E_SRC;
            return -1;
        }
        uint32_t want = rd32(in + pos);
        uint32_t got = (uint32_t)xxh64(z->out + z->frame_start, (size_t)(z->olen - z->frame_start), 0);
        if (want != got) {
            z->err = E_CHECKSUM;
            return -1;
        }
        pos += 4;
    }
    return pos;
}

int orc_zstd_decompress(const uint8_t *in, int64_t n, uint8_t *out, int64_t cap, int64_t *out_len,
                        const char **msg) {
    static zctx z;
    memset(&z, 0, sizeof(z));
    z.out = out;
    z.cap = cap;
    *msg = "";
    int64_t pos = 0;
    if (n <= 0) {
        *out_len = 0;
        *msg = E_SRC;
        return ORC_ZSTD_ERROR;
    }
    while (pos < n) {
        int64_t k = decode_frame(&z, in + pos, n - pos);
        if (k < 0) {
            *out_len = z.olen;
            if (z.full) return ORC_ZSTD_OUTPUT_FULL;
            *msg = z.err ? z.err : E_CORRUPT;
            return ORC_ZSTD_ERROR;
        }
        pos += k;
    }
    *out_len = z.olen;
    (void)E_TABLELOG;
    return ORC_ZSTD_OK;
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
