/*
 * ORACLE — test infrastructure only. Never linked into or called by the product
 * path; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * it, as the checker.
 *
 * Single-threaded C restatement of the reference v2 scan path (pure Go; no Go
 * toolchain exists here, so the reference itself cannot be built — DESIGN.md):
 *   bytes.Reader / io.ReadFull semantics        (Go stdlib)
 *   errors.Once{Ignored: io.EOF}                errors/once.go:21-54, scannerv2.go:242
 *   ChunkScanner.{Scan,readChunk,LimitShard,ReadLastBlock,readChunkHeader}
 *                                               recordio/internal/chunk.go:180-407
 *   parseChunksToItems, rawItemList.item        recordio/scannerv2.go:24-97
 *   NewShardScanner/newScanner/readSpecialBlock/readHeader/Trailer/Seek/
 *   scanNextBlock/Scan/Err                      recordio/scannerv2.go:200-412
 *   ParsedHeader.unmarshal + headerDecoder      recordio/header.go:140-254
 *   registry getTransformers/GetUntransformer   recordio/registry.go:31-148
 *   idTransform / FlateUncompress / zstdUncompress
 *        registry.go:31-39, recordioflate/recordioflate.go:54-65,
 *        recordiozstd/recordiozstd.go:67-78, compress/zstd/zstd_cgo.go:34-41
 *   binary.Uvarint (Go 1.13-1.15, go.mod:3)
 * Error strings are the reference's fmt formats, byte for byte.
 */
#include <inttypes.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define CHUNK_SIZE 32768
#define CHUNK_HDR 28
#define MAX_PAYLOAD (CHUNK_SIZE - CHUNK_HDR)

static const uint8_t kMagicPacked[8] = {0x2e, 0x76, 0x47, 0xeb, 0x34, 0x07, 0x3c, 0x2e};
static const uint8_t kMagicHeader[8] = {0xd9, 0xe1, 0xd9, 0x5c, 0xc2, 0x16, 0x04, 0xf7};
static const uint8_t kMagicTrailer[8] = {0xfe, 0xba, 0x1a, 0xd7, 0xcb, 0xdf, 0x75, 0x3a};
static const uint8_t kMagicInvalid[8] = {0xe4, 0xe7, 0x9a, 0xc1, 0xb3, 0xf6, 0xb7, 0xa2};

/* ---------------------------------------------------------------- crc32 */
static uint32_t crc_tab[8][256];
static int crc_ready = 0;
static void crc_init(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_tab[0][i] = c;
    }
    for (int t = 1; t < 8; t++)
        for (int i = 0; i < 256; i++)
            crc_tab[t][i] = (crc_tab[t - 1][i] >> 8) ^ crc_tab[0][crc_tab[t - 1][i] & 0xff];
    crc_ready = 1;
}
/* hash/crc32 IEEE (slice-by-8 restatement), crc = running value (0 to start) */
uint32_t orc_crc32(uint32_t crc, const uint8_t *p, size_t n) {
    if (!crc_ready) crc_init();
    crc = ~crc;
    while (n >= 8) {
        uint32_t a = crc ^ (p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
        uint32_t b = p[4] | (uint32_t)p[5] << 8 | (uint32_t)p[6] << 16 | (uint32_t)p[7] << 24;
        crc = crc_tab[7][a & 0xff] ^ crc_tab[6][(a >> 8) & 0xff] ^ crc_tab[5][(a >> 16) & 0xff] ^
              crc_tab[4][a >> 24] ^ crc_tab[3][b & 0xff] ^ crc_tab[2][(b >> 8) & 0xff] ^
              crc_tab[1][(b >> 16) & 0xff] ^ crc_tab[0][b >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) crc = crc_tab[0][(crc ^ *p++) & 0xff] ^ (crc >> 8);
    return ~crc;
}

/* ---------------------------------------------------------------- helpers */
typedef struct {
    int set;
    char msg[1024];
} once_t; /* errors.Once with Ignored = {io.EOF}: callers never Set EOF */

static void once_set(once_t *e, const char *fmt, ...) {
    if (e->set) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(e->msg, sizeof(e->msg), fmt, ap);
    va_end(ap);
    e->set = 1;
}

static void fmt_magic_v(const uint8_t *m, char *out) { /* %v of [8]byte */
    sprintf(out, "[%u %u %u %u %u %u %u %u]", m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7]);
}
static void fmt_magic_x(const uint8_t *m, char *out) { /* %x of [8]byte */
    for (int i = 0; i < 8; i++) sprintf(out + 2 * i, "%02x", m[i]);
}

static uint32_t le32(const uint8_t *p) {
    return p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

/* binary.Uvarint, Go 1.13-1.15 */
static uint64_t uvarint(const uint8_t *buf, int64_t len, int64_t *n) {
    uint64_t x = 0;
    unsigned s = 0;
    for (int64_t i = 0; i < len; i++) {
        uint8_t b = buf[i];
        if (b < 0x80) {
            if (i > 9 || (i == 9 && b > 1)) {
                *n = -(i + 1);
                return 0;
            }
            *n = i + 1;
            return x | ((uint64_t)b << s);
        }
        if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
        s += 7;
    }
    *n = 0;
    return 0;
}

typedef struct {
    uint8_t *p;
    int64_t n, cap;
} vec_t;
static void vec_reserve(vec_t *v, int64_t cap) {
    if (v->cap >= cap) return;
    int64_t nc = v->cap ? v->cap : 64;
    while (nc < cap) nc *= 2;
    v->p = (uint8_t *)realloc(v->p, (size_t)nc);
    v->cap = nc;
}
static void vec_append(vec_t *v, const void *d, int64_t n) {
    vec_reserve(v, v->n + n);
    if (n) memcpy(v->p + v->n, d, (size_t)n);
    v->n += n;
}

/* ---------------------------------------------------------------- bytes.Reader */
typedef struct {
    const uint8_t *p;
    int64_t n, pos;
} rdr_t;

enum { RD_OK = 0, RD_EOF = 1, RD_UNEXPECTED = 2 };

/* io.ReadFull into a view; returns bytes read */
static int64_t read_full(rdr_t *r, int64_t k, const uint8_t **view, int *st) {
    int64_t avail = r->n - r->pos;
    if (avail < 0) avail = 0;
    int64_t got = k < avail ? k : avail;
    *view = r->p + (got ? r->pos : 0);
    r->pos += got;
    if (got == k) *st = RD_OK;
    else if (got == 0) *st = RD_EOF;
    else *st = RD_UNEXPECTED;
    return got;
}

/* Seek; returns 0 on success, -1 with *err message on negative position */
static int rdr_seek(rdr_t *r, int64_t off, int whence, int64_t *newpos) {
    int64_t abs = off;
    if (whence == 1) abs = r->pos + off;
    else if (whence == 2) abs = r->n + off;
    if (abs < 0) {
        *newpos = 0;
        return -1;
    }
    r->pos = abs;
    *newpos = abs;
    return 0;
}
#define SEEK_NEG_MSG "bytes.Reader.Seek: negative position"

/* internal.Seek (chunk.go:66-75) */
static void seek_abs(rdr_t *r, int64_t off, once_t *err) {
    int64_t np;
    if (rdr_seek(r, off, 0, &np) != 0) {
        once_set(err, SEEK_NEG_MSG);
        return;
    }
}

/* ---------------------------------------------------------------- ChunkScanner */
typedef struct {
    rdr_t *r;
    once_t *err;
    int64_t file_size, off, limit;
    uint8_t magic[8];
    const uint8_t **chunk_p;
    int64_t *chunk_n;
    int64_t nchunks, cap;
} cs_t;

static void cs_init(cs_t *c, rdr_t *r, once_t *err) {
    memset(c, 0, sizeof(*c));
    c->r = r;
    c->err = err;
    int64_t np;
    rdr_seek(r, 0, 2, &np);
    c->file_size = np;
    seek_abs(r, 0, err);
    c->limit = INT64_MAX;
    memcpy(c->magic, kMagicInvalid, 8);
}

static void cs_free(cs_t *c) {
    free(c->chunk_p);
    free(c->chunk_n);
}

static void cs_append(cs_t *c, const uint8_t *p, int64_t n) {
    if (c->nchunks == c->cap) {
        c->cap = c->cap ? c->cap * 2 : 16;
        c->chunk_p = (const uint8_t **)realloc(c->chunk_p, sizeof(*c->chunk_p) * (size_t)c->cap);
        c->chunk_n = (int64_t *)realloc(c->chunk_n, sizeof(*c->chunk_n) * (size_t)c->cap);
    }
    c->chunk_p[c->nchunks] = p;
    c->chunk_n[c->nchunks] = n;
    c->nchunks++;
}

/* readChunk (chunk.go:316-345); returns 0 for MagicInvalid */
static int cs_read_chunk(cs_t *c, uint8_t magic[8], int64_t *total, int64_t *index,
                         const uint8_t **payload, int64_t *plen) {
    const uint8_t *buf;
    int st;
    int64_t got = read_full(c->r, CHUNK_SIZE, &buf, &st);
    c->off += got;
    if (st != RD_OK) {
        if (st == RD_UNEXPECTED) once_set(c->err, "unexpected EOF");
        return 0;
    }
    memcpy(magic, buf, 8);
    uint32_t expected = le32(buf + 8);
    uint32_t size = le32(buf + 16);
    *total = le32(buf + 20);
    *index = le32(buf + 24);
    if (size > MAX_PAYLOAD) {
        once_set(c->err, "Invalid chunk size %u", size);
        return 0;
    }
    *payload = buf + CHUNK_HDR;
    *plen = size;
    uint32_t actual = orc_crc32(0, buf + 12, 16 + (size_t)size);
    if (expected != actual)
        once_set(c->err, "Chunk checksum mismatch, expect %u, got %u", actual, expected);
    return 1;
}

/* Scan (chunk.go:253-294) */
static int cs_scan(cs_t *c) {
    c->nchunks = 0;
    memcpy(c->magic, kMagicInvalid, 8);
    if (c->err->set) return 0;
    if (c->off >= c->limit) return 0; /* io.EOF, ignored */
    int64_t total_chunks = -1;
    for (;;) {
        uint8_t m[8];
        int64_t nch, index, plen;
        const uint8_t *payload;
        int ok = cs_read_chunk(c, m, &nch, &index, &payload, &plen);
        if (!ok || memcmp(m, kMagicInvalid, 8) == 0 || c->err->set) return 0;
        if (c->nchunks == 0) {
            memcpy(c->magic, m, 8);
            total_chunks = nch;
        }
        char a[64], b[64];
        if (memcmp(m, c->magic, 8) != 0) {
            fmt_magic_v(c->magic, a);
            fmt_magic_v(m, b);
            once_set(c->err,
                     "Magic number changed in the middle of a chunk sequence, got %s, expect %s", a, b);
            return 0;
        }
        if (c->nchunks != index) {
            fmt_magic_x(c->magic, a);
            once_set(c->err, "Chunk index mismatch, got %" PRId64 ", expect %" PRId64 " for magic %s",
                     index, c->nchunks, a);
            return 0;
        }
        if (nch != total_chunks) {
            fmt_magic_x(c->magic, a);
            once_set(c->err, "Chunk nchunk mismatch, got %" PRId64 ", expect %" PRId64 " for magic %s",
                     nch, total_chunks, a);
            return 0;
        }
        cs_append(c, payload, plen);
        if (index == total_chunks - 1) break;
    }
    return 1;
}

static void cs_seek(cs_t *c, int64_t off) {
    c->off = off;
    seek_abs(c->r, off, c->err);
}

/* readChunkHeader (chunk.go:303-312) */
static int cs_read_chunk_header(cs_t *c, uint8_t hdr[CHUNK_HDR]) {
    const uint8_t *v;
    int st;
    read_full(c->r, CHUNK_HDR, &v, &st);
    if (st != RD_OK) {
        if (st == RD_UNEXPECTED) once_set(c->err, "unexpected EOF");
        return 0;
    }
    memcpy(hdr, v, CHUNK_HDR);
    int64_t np;
    rdr_seek(c->r, -CHUNK_HDR, 1, &np);
    c->off = np;
    return 1;
}

void orc_shard_range(int64_t file_size, int64_t off, int start, int limit, int nshard,
                     int64_t *o_off, int64_t *o_limit) {
    int64_t num_chunks = (file_size - off) / CHUNK_SIZE;
    double cps = (double)num_chunks / (double)nshard;
    *o_off = off + (int64_t)((double)start * cps) * CHUNK_SIZE;
    *o_limit = off + (int64_t)((double)limit * cps) * CHUNK_SIZE;
}

/* LimitShard (chunk.go:198-236) */
static void cs_limit_shard(cs_t *c, int start, int limit, int nshard) {
    int64_t start_off = c->off;
    orc_shard_range(c->file_size, start_off, start, limit, nshard, &c->off, &c->limit);
    if (start == 0) return;
    seek_abs(c->r, c->off, c->err);
    if (c->err->set) return;
    uint8_t hdr[CHUNK_HDR];
    if (!cs_read_chunk_header(c, hdr)) return;
    if (c->err->set) return;
    int64_t index = le32(hdr + 24);
    if (index == 0) return;
    int64_t total = le32(hdr + 20);
    if (total <= index) {
        once_set(c->err, "invalid chunk header");
        return;
    }
    c->off += CHUNK_SIZE * (total - index);
    seek_abs(c->r, c->off, c->err);
}

/* ReadLastBlock (chunk.go:380-407); returns 1 with c->magic/chunks set */
static int cs_read_last_block(cs_t *c) {
    int64_t np;
    if (rdr_seek(c->r, -CHUNK_SIZE, 2, &np) != 0) {
        c->off = 0;
        once_set(c->err, SEEK_NEG_MSG);
        return 0;
    }
    c->off = np;
    uint8_t m[8];
    int64_t total, index, plen;
    const uint8_t *payload;
    if (!cs_read_chunk(c, m, &total, &index, &payload, &plen)) memcpy(m, kMagicInvalid, 8);
    if (memcmp(m, kMagicTrailer, 8) != 0) {
        char a[64];
        fmt_magic_v(m, a);
        once_set(c->err, "Missing magic trailer; found %s", a);
        return 0;
    }
    if (index == 0 && total == 1) {
        c->nchunks = 0;
        cs_append(c, payload, plen);
        memcpy(c->magic, m, 8);
        return 1;
    }
    if (rdr_seek(c->r, -(index + 1) * CHUNK_SIZE, 2, &np) != 0) {
        c->off = 0;
        once_set(c->err, SEEK_NEG_MSG);
        return 0;
    }
    c->off = np;
    if (!cs_scan(c)) {
        once_set(c->err, "Failed to read trailer");
        return 0;
    }
    return 1;
}

/* ---------------------------------------------------------------- transformers */
enum { TR_ID = 0, TR_FLATE = 1, TR_ZSTD = 2 };

/* apply one untransformer to `in` (concatenated), result into *out */
static int untransform_one(int kind, const uint8_t *in, int64_t n, vec_t *out, once_t *err,
                           int nchunks_in) {
    if (kind == TR_ID) {
        out->n = 0;
        vec_append(out, in, n);
        return 1;
    }
    if (kind == TR_FLATE) {
        int64_t cap = n * 4 + 1024;
        for (;;) {
            vec_reserve(out, cap);
            int64_t olen = 0, eoff = 0;
            int rc = orc_inflate(in, n, out->p, cap, &olen, &eoff);
            if (rc == ORC_INFLATE_OUTPUT_FULL) {
                cap *= 2;
                continue;
            }
            if (rc == ORC_INFLATE_CORRUPT) {
                once_set(err, "flate: corrupt input before offset %" PRId64, eoff);
                return 0;
            }
            if (rc == ORC_INFLATE_UNEXPECTED_EOF) {
                once_set(err, "unexpected EOF");
                return 0;
            }
            out->n = olen;
            return 1;
        }
    }
    /* zstd: DataDog Decompress errors on an empty source (ErrEmptySlice) */
    if (nchunks_in == 0 || n == 0) {
        once_set(err, "Bytes slice is empty");
        return 0;
    }
    int64_t cs = orc_zstd_content_size(in, n);
    int64_t cap = cs >= 0 ? cs : n * 3;
    if (cap < 64) cap = 64;
    for (;;) {
        vec_reserve(out, cap);
        int64_t olen = 0;
        const char *msg = "";
        int rc = orc_zstd_decompress(in, n, out->p, cap, &olen, &msg);
        if (rc == ORC_ZSTD_OUTPUT_FULL) {
            cap *= 2;
            continue;
        }
        if (rc != ORC_ZSTD_OK) {
            once_set(err, "%s", msg);
            return 0;
        }
        out->n = olen;
        return 1;
    }
}

/* ---------------------------------------------------------------- header */
typedef struct {
    char *key;
    int type; /* 1 bool 2 int 3 uint 4 string */
    int64_t ival;
    uint8_t *s;
    int64_t slen;
} kv_t;

typedef struct {
    const uint8_t *p;
    int64_t n;
    once_t err;
} hdec_t;

/* getRawValue (header.go:155-198); returns type or 0 on error */
static int hdec_value(hdec_t *d, int64_t *ival, const uint8_t **s, int64_t *slen) {
    if (d->n <= 0) {
        once_set(&d->err, "Failed to read byte in header");
        return 0;
    }
    uint8_t vt = *d->p++;
    d->n--;
    switch (vt) {
    case 1: {
        if (d->n <= 0) {
            once_set(&d->err, "Failed to read byte in header");
            *ival = 0;
            return 1;
        }
        uint8_t b = *d->p++;
        d->n--;
        *ival = b != 0;
        return 1;
    }
    case 3: {
        int64_t n;
        uint64_t v = uvarint(d->p, d->n, &n);
        if (n <= 0) {
            once_set(&d->err, "Failed to parse uint");
            *ival = 0;
            return 3;
        }
        d->p += n;
        d->n -= n;
        *ival = (int64_t)v;
        return 3;
    }
    case 2: {
        int64_t n;
        uint64_t ux = uvarint(d->p, d->n, &n);
        if (n <= 0) {
            once_set(&d->err, "Failed to parse uint");
            *ival = 0;
            return 2;
        }
        d->p += n;
        d->n -= n;
        int64_t x = (int64_t)(ux >> 1);
        if (ux & 1) x = ~x;
        *ival = x;
        return 2;
    }
    case 4: {
        int64_t ln;
        const uint8_t *ds;
        int64_t dl;
        int t = hdec_value(d, &ln, &ds, &dl);
        if (d->err.set) return 4;
        if (t != 3) {
            once_set(&d->err, "failed to read string key");
            return 4;
        }
        if ((uint64_t)d->n < (uint64_t)ln) {
            once_set(&d->err, "header invalid string (%" PRIu64 ")", (uint64_t)ln);
            return 4;
        }
        *s = d->p;
        *slen = ln;
        d->p += ln;
        d->n -= ln;
        return 4;
    }
    default:
        once_set(&d->err, "illegal header type uint8");
        return 0;
    }
}

/* ---------------------------------------------------------------- scanner */
struct orc_result {
    vec_t items;
    uint64_t *ends, *blocks;
    int64_t *idx;
    int64_t n_items, cap_items;
    char err[1024];
    int has_trailer;
    vec_t trailer;
    kv_t *kvs;
    int nkv;
    int legacy;
};

typedef struct {
    once_t err;
    rdr_t r;
    cs_t cs;
    kv_t *kvs;
    int nkv;
    int tr[64];
    int ntr;
    vec_t bytes;
    int64_t first_off;
    int64_t *cum;
    int64_t ncum, capcum;
    int64_t next_item;
    int64_t block_off;
    int error_scanner; /* errorScanner */
    int legacy;
} sc_t;

static void res_push_item(orc_result *r, const uint8_t *p, int64_t n, uint64_t block, int64_t idx) {
    if (r->n_items == r->cap_items) {
        r->cap_items = r->cap_items ? r->cap_items * 2 : 256;
        r->ends = (uint64_t *)realloc(r->ends, 8 * (size_t)r->cap_items);
        r->blocks = (uint64_t *)realloc(r->blocks, 8 * (size_t)r->cap_items);
        r->idx = (int64_t *)realloc(r->idx, 8 * (size_t)r->cap_items);
    }
    vec_append(&r->items, p, n);
    r->ends[r->n_items] = (uint64_t)r->items.n;
    r->blocks[r->n_items] = block;
    r->idx[r->n_items] = idx;
    r->n_items++;
}

/* parseChunksToItems (scannerv2.go:53-97); untransform chain applied in reverse */
static int parse_chunks(sc_t *s, cs_t *c, const int *tr, int ntr, vec_t *bytes, int64_t *first_off,
                        int64_t **cum, int64_t *ncum, int64_t *capcum, once_t *err) {
    vec_t cat = {0};
    for (int64_t i = 0; i < c->nchunks; i++) vec_append(&cat, c->chunk_p[i], c->chunk_n[i]);
    int nin = (int)c->nchunks;
    (void)s;
    if (ntr == 0) {
        bytes->n = 0;
        vec_append(bytes, cat.p, cat.n);
    } else {
        vec_t cur = cat;
        cat.p = NULL;
        for (int k = ntr - 1; k >= 0; k--) {
            vec_t out = {0};
            if (!untransform_one(tr[k], cur.p, cur.n, &out, err, nin)) {
                free(cur.p);
                free(out.p);
                return 0;
            }
            free(cur.p);
            cur = out;
            nin = 1;
        }
        bytes->n = 0;
        vec_append(bytes, cur.p, cur.n);
        free(cur.p);
    }
    free(cat.p);
    const uint8_t *block = bytes->p;
    int64_t blen = bytes->n;
    int64_t n;
    uint64_t un = uvarint(block, blen, &n);
    if (n <= 0) {
        once_set(err, "recordio: failed to read number of packed items: %" PRId64, n);
        return 0;
    }
    int64_t pos = n;
    uint64_t utotal = 0; /* Go int arithmetic wraps */
    int64_t total = 0;
    *ncum = 0;
    for (uint64_t i = 0; i < un; i++) {
        uint64_t size = uvarint(block + pos, blen - pos, &n);
        if (n <= 0) {
            once_set(err, "recordio: likely corrupt data, failed to read size of packed item %" PRIu64
                          ": %" PRId64, i, n);
            return 0;
        }
        utotal += size;
        total = (int64_t)utotal;
        if (*ncum == *capcum) {
            *capcum = *capcum ? *capcum * 2 : 256;
            *cum = (int64_t *)realloc(*cum, 8 * (size_t)*capcum);
        }
        (*cum)[(*ncum)++] = total;
        pos += n;
    }
    *first_off = pos;
    if ((int64_t)(utotal + (uint64_t)pos) != blen) {
        once_set(err, "recordio: corrupt block header, got block size %" PRId64 ", expected %" PRId64,
                 blen, (int64_t)(utotal + (uint64_t)pos));
        return 0;
    }
    /* Go would panic slicing a wrapped cumSize; report it instead */
    for (int64_t i = 0; i < *ncum; i++) {
        int64_t st = i ? (*cum)[i - 1] : 0;
        if ((*cum)[i] < st || pos + (*cum)[i] > blen) {
            once_set(err, "recordio: corrupt block header, item sizes out of range");
            return 0;
        }
    }
    return 1;
}

static const uint8_t *item_at(sc_t *s, int64_t i, int64_t *len) {
    int64_t st = s->first_off + (i > 0 ? s->cum[i - 1] : 0);
    int64_t en = s->first_off + s->cum[i];
    *len = en - st;
    return s->bytes.p + st;
}

static int has_trailer(sc_t *s) { /* header.go:242-254 */
    for (int i = 0; i < s->nkv; i++) {
        if (strcmp(s->kvs[i].key, "trailer") != 0) continue;
        return s->kvs[i].type == 1 && s->kvs[i].ival;
    }
    return 0;
}

static void read_header(sc_t *s) {
    /* readSpecialBlock(MagicHeader, idTransform) */
    char a[64], b[64];
    if (!cs_scan(&s->cs)) {
        fmt_magic_v(kMagicHeader, a);
        once_set(&s->err, "Failed to read block %s", a);
        return;
    }
    if (memcmp(s->cs.magic, kMagicHeader, 8) != 0) {
        fmt_magic_v(kMagicHeader, a);
        fmt_magic_v(s->cs.magic, b);
        once_set(&s->err, "Failed to read block, expect %s, got %s", a, b);
        return;
    }
    vec_t bytes = {0};
    int64_t first_off = 0, ncum = 0, capcum = 0;
    int64_t *cum = NULL;
    if (!parse_chunks(s, &s->cs, NULL, 0, &bytes, &first_off, &cum, &ncum, &capcum, &s->err)) {
        free(bytes.p);
        free(cum);
        return;
    }
    if (ncum != 1) {
        once_set(&s->err, "Wrong # of items in header block, %" PRId64, ncum);
        free(bytes.p);
        free(cum);
        return;
    }
    hdec_t d;
    memset(&d, 0, sizeof(d));
    d.p = bytes.p + first_off;
    d.n = cum[0];
    /* ParsedHeader.unmarshal (header.go:211-239) */
    int64_t nkv;
    const uint8_t *sv;
    int64_t sl;
    int t = hdec_value(&d, &nkv, &sv, &sl);
    if (!d.err.set && t != 3) once_set(&d.err, "Failed to read # header entries");
    if (!d.err.set) {
        for (uint64_t i = 0; i < (uint64_t)nkv; i++) {
            int64_t kiv;
            const uint8_t *ks = NULL;
            int64_t kl = 0;
            int kt = hdec_value(&d, &kiv, &ks, &kl);
            if (d.err.set) break;
            if (kt != 4) {
                once_set(&d.err, "failed to read string key");
                break;
            }
            kv_t kv;
            memset(&kv, 0, sizeof(kv));
            kv.key = (char *)malloc((size_t)kl + 1);
            memcpy(kv.key, ks, (size_t)kl);
            kv.key[kl] = 0;
            const uint8_t *vs = NULL;
            int64_t vl = 0;
            kv.type = hdec_value(&d, &kv.ival, &vs, &vl);
            if (d.err.set) {
                free(kv.key);
                break;
            }
            if (kv.type == 4) {
                kv.s = (uint8_t *)malloc((size_t)vl + 1);
                memcpy(kv.s, vs, (size_t)vl);
                kv.slen = vl;
            }
            s->kvs = (kv_t *)realloc(s->kvs, sizeof(kv_t) * (size_t)(s->nkv + 1));
            s->kvs[s->nkv++] = kv;
        }
    }
    free(bytes.p);
    free(cum);
    if (d.err.set) {
        once_set(&s->err, "%s", d.err.msg);
        return;
    }
    /* registry.GetUntransformer over the "transformer" values */
    for (int i = 0; i < s->nkv; i++) {
        kv_t *kv = &s->kvs[i];
        if (strcmp(kv->key, "transformer") != 0) continue;
        if (kv->type != 4) {
            char v[64];
            if (kv->type == 1) sprintf(v, "%s", kv->ival ? "true" : "false");
            else if (kv->type == 3) sprintf(v, "%" PRIu64, (uint64_t)kv->ival);
            else sprintf(v, "%" PRId64, kv->ival);
            once_set(&s->err, "Expect string value for key %s, but found %s", kv->key, v);
            return;
        }
        char name[256];
        int64_t k = 0;
        while (k < kv->slen && k < 255 && kv->s[k] != ' ') {
            name[k] = (char)kv->s[k];
            k++;
        }
        name[k] = 0;
        int kind;
        if (k == kv->slen || kv->s[k] == ' ') {
            if (strcmp(name, "flate") == 0) kind = TR_FLATE;
            else if (strcmp(name, "zstd") == 0) kind = TR_ZSTD;
            else kind = -1;
        } else {
            kind = -1;
        }
        if (kind < 0) {
            once_set(&s->err, "Transformer %.*s not found", (int)kv->slen, (const char *)kv->s);
            return;
        }
        if (s->ntr < 64) s->tr[s->ntr++] = kind;
    }
}

static void sc_open(sc_t *s, const uint8_t *f, int64_t n, int start, int limit, int nshard) {
    memset(s, 0, sizeof(*s));
    s->r.p = f;
    s->r.n = n;
    const uint8_t *v;
    int st;
    read_full(&s->r, 8, &v, &st);
    if (st != RD_OK) {
        s->error_scanner = 1;
        if (st == RD_UNEXPECTED) once_set(&s->err, "unexpected EOF");
        return;
    }
    uint8_t magic[8];
    memcpy(magic, v, 8);
    s->r.pos = 0;
    if (start >= limit || limit > nshard || start < 0 || nshard <= 0) {
        s->error_scanner = 1;
        once_set(&s->err, "invalid sharding [%d,%d) of %d", start, limit, nshard);
        return;
    }
    if (memcmp(magic, kMagicHeader, 8) != 0) {
        s->error_scanner = 1;
        if (start != 0 || limit != 1 || nshard != 1)
            once_set(&s->err, "legacy record IOs do not support sharding");
        else
            s->legacy = 1;
        return;
    }
    cs_init(&s->cs, &s->r, &s->err);
    read_header(s);
    if (s->err.set) return;
    cs_limit_shard(&s->cs, start, limit, nshard);
}

static void sc_close(sc_t *s) {
    if (!s->error_scanner) cs_free(&s->cs);
    free(s->bytes.p);
    free(s->cum);
    for (int i = 0; i < s->nkv; i++) {
        free(s->kvs[i].key);
        free(s->kvs[i].s);
    }
    free(s->kvs);
}

/* Trailer (scannerv2.go:316-342); returns 1 and fills out when non-nil */
static int sc_trailer(sc_t *s, vec_t *out) {
    if (s->error_scanner) return 0;
    if (!has_trailer(s)) return 0;
    int64_t cur = s->cs.off;
    int ret = 0;
    if (!cs_read_last_block(&s->cs) || s->err.set) goto done;
    if (memcmp(s->cs.magic, kMagicTrailer, 8) != 0) {
        char a[64];
        fmt_magic_v(s->cs.magic, a);
        once_set(&s->err, "Did not found the trailer, instead found magic %s", a);
        goto done;
    }
    {
        vec_t bytes = {0};
        int64_t first_off = 0, ncum = 0, capcum = 0;
        int64_t *cum = NULL;
        if (!parse_chunks(s, &s->cs, s->tr, s->ntr, &bytes, &first_off, &cum, &ncum, &capcum,
                          &s->err)) {
            free(bytes.p);
            free(cum);
            goto done;
        }
        if (ncum != 1) {
            once_set(&s->err, "Expect exactly one trailer item, but found %" PRId64, ncum);
        } else {
            out->n = 0;
            vec_append(out, bytes.p + first_off, cum[0]);
            ret = 1;
        }
        free(bytes.p);
        free(cum);
    }
done:
    cs_seek(&s->cs, cur);
    return ret;
}

/* scanNextBlock (scannerv2.go:363-388) */
static int sc_next_block(sc_t *s) {
    s->ncum = 0;
    s->bytes.n = 0;
    s->next_item = 0;
    if (s->err.set) return 0;
    s->block_off = s->cs.off;
    if (!cs_scan(&s->cs)) return 0;
    if (memcmp(s->cs.magic, kMagicPacked, 8) == 0) {
        if (!parse_chunks(s, &s->cs, s->tr, s->ntr, &s->bytes, &s->first_off, &s->cum, &s->ncum,
                          &s->capcum, &s->err)) {
            s->ncum = 0;
            return 0;
        }
        s->next_item = 0;
        return 1;
    }
    if (memcmp(s->cs.magic, kMagicTrailer, 8) == 0) return 0;
    char a[64];
    fmt_magic_v(s->cs.magic, a);
    once_set(&s->err, "recordio: invalid magic number: %s", a);
    return 0;
}

/* Scan (scannerv2.go:390-404); p and n receive Get() */
static int sc_scan(sc_t *s, const uint8_t **p, int64_t *n) {
    if (s->error_scanner) return 0;
    while (s->next_item >= s->ncum)
        if (!sc_next_block(s)) return 0;
    *p = item_at(s, s->next_item, n);
    s->next_item++;
    return 1;
}

static orc_result *res_new(void) { return (orc_result *)calloc(1, sizeof(orc_result)); }

static void res_take_header(orc_result *r, sc_t *s) {
    r->nkv = s->nkv;
    r->kvs = s->kvs;
    s->kvs = NULL;
    s->nkv = 0;
    r->legacy = s->legacy;
}

/* oracle/legacy.c: the v1 adapter (legacyscanner.go) */
typedef void (*v1_item_fn)(void *u, const uint8_t *p, int64_t n, uint64_t block, int64_t idx);
void orc_v1_run(const uint8_t *f, int64_t n, int seek, uint64_t block, int64_t item, v1_item_fn fn, void *u,
                char *err, size_t errcap);
static void v1_collect(void *u, const uint8_t *p, int64_t n, uint64_t block, int64_t idx) {
    res_push_item((orc_result *)u, p, n, block, idx);
}

orc_result *orc_scan(const uint8_t *f, int64_t n, int start, int limit, int nshard, int flags) {
    sc_t s;
    sc_open(&s, f, n, start, limit, nshard);
    orc_result *r = res_new();
    if (s.legacy) { /* newLegacyScannerAdapter (scannerv2.go:232): Trailer() is nil */
        orc_v1_run(f, n, 0, 0, 0, v1_collect, r, r->err, sizeof(r->err));
        res_take_header(r, &s);
        sc_close(&s);
        return r;
    }
    if ((flags & 1) && !s.error_scanner) r->has_trailer = sc_trailer(&s, &r->trailer);
    const uint8_t *p;
    int64_t len;
    while (sc_scan(&s, &p, &len)) res_push_item(r, p, len, (uint64_t)s.block_off, s.next_item - 1);
    if (s.err.set) snprintf(r->err, sizeof(r->err), "%s", s.err.msg);
    res_take_header(r, &s);
    sc_close(&s);
    return r;
}

orc_result *orc_seek_get(const uint8_t *f, int64_t n, uint64_t block, int64_t item) {
    sc_t s;
    sc_open(&s, f, n, 0, 1, 1);
    orc_result *r = res_new();
    if (s.legacy) {
        orc_v1_run(f, n, 1, block, item, v1_collect, r, r->err, sizeof(r->err));
    } else if (!s.error_scanner) {
        /* Seek (scannerv2.go:348-361) */
        cs_seek(&s.cs, (int64_t)block);
        if (sc_next_block(&s)) {
            if (item >= s.ncum) {
                once_set(&s.err, "Invalid location {Block:%" PRIu64 " Item:%" PRId64
                                 "}, block has only %" PRId64 " items", block, item, s.ncum);
            }
            s.next_item = item;
        }
        const uint8_t *p;
        int64_t len;
        if (sc_scan(&s, &p, &len)) res_push_item(r, p, len, (uint64_t)s.block_off, s.next_item - 1);
    }
    if (s.err.set) snprintf(r->err, sizeof(r->err), "%s", s.err.msg);
    res_take_header(r, &s);
    sc_close(&s);
    return r;
}

int64_t orc_scan_count(const uint8_t *f, int64_t n, int64_t *bytes_out, int start, int limit,
                       int nshard) {
    sc_t s;
    sc_open(&s, f, n, start, limit, nshard);
    if (s.legacy) {
        orc_result *r = res_new();
        orc_v1_run(f, n, 0, 0, 0, v1_collect, r, r->err, sizeof(r->err));
        int64_t items = r->n_items, bad = r->err[0] != 0;
        *bytes_out = (int64_t)r->items.n;
        orc_free(r);
        sc_close(&s);
        return bad ? -1 : items;
    }
    const uint8_t *p;
    int64_t len, items = 0, bytes = 0;
    while (sc_scan(&s, &p, &len)) {
        items++;
        bytes += len;
    }
    *bytes_out = bytes;
    int bad = s.err.set;
    sc_close(&s);
    return bad ? -1 : items;
}

void orc_free(orc_result *r) {
    if (!r) return;
    free(r->items.p);
    free(r->ends);
    free(r->blocks);
    free(r->idx);
    free(r->trailer.p);
    for (int i = 0; i < r->nkv; i++) {
        free(r->kvs[i].key);
        free(r->kvs[i].s);
    }
    free(r->kvs);
    free(r);
}

int64_t orc_n_items(const orc_result *r) { return r->n_items; }
const uint8_t *orc_items(const orc_result *r) { return r->items.p; }
const uint64_t *orc_item_ends(const orc_result *r) { return r->ends; }
const uint64_t *orc_item_block(const orc_result *r) { return r->blocks; }
const int64_t *orc_item_index(const orc_result *r) { return r->idx; }
const char *orc_err(const orc_result *r) { return r->err; }
int orc_has_trailer(const orc_result *r) { return r->has_trailer; }
const uint8_t *orc_trailer(const orc_result *r, int64_t *len) {
    *len = r->trailer.n;
    return r->trailer.p;
}
int orc_header_len(const orc_result *r) { return r->nkv; }
int orc_header_kv(const orc_result *r, int i, const char **key, int *type, int64_t *ival,
                  const uint8_t **sval, int64_t *slen) {
    if (i < 0 || i >= r->nkv) return 0;
    *key = r->kvs[i].key;
    *type = r->kvs[i].type;
    *ival = r->kvs[i].ival;
    *sval = r->kvs[i].s;
    *slen = r->kvs[i].slen;
    return 1;
}
int orc_is_legacy(const orc_result *r) { return r->legacy; }
