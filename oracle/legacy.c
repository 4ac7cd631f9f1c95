/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg). Never linked into or called by the product path.
 *
 * CPU restatement of the reference's v1 ("legacy") read path, which
 * recordio.NewScanner selects for any file whose first 8 bytes are not the v2
 * header magic (scannerv2.go:228-233):
 *   legacyScannerAdapter          recordio/legacyscanner.go:18-152
 *   LegacyScannerImpl.InternalScan recordio/deprecated/recordio.go:258-300
 *   unmarshalHeader               recordio/deprecated/recordio.go:324-334
 *   Unpacker.Unpack               recordio/deprecated/packer.go:214-272
 * with no LegacyTransform (ScannerOpts.LegacyTransform nil). Pinned by the
 * reference's own v1 vectors and error tables (tests/test_legacy.py):
 * deprecated/recordio_test.go:41-110, 138-221, deprecated/packer_test.go:283-318,
 * v2_test.go:49-72.
 */
#include <inttypes.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef void (*v1_item_fn)(void *u, const uint8_t *p, int64_t n, uint64_t block, int64_t idx);

static const uint8_t kMagicLegacyUnpacked[8] = {0xfc, 0xae, 0x95, 0x31, 0xf0, 0xd9, 0xbd, 0x20};
static const uint8_t kMagicPacked[8] = {0x2e, 0x76, 0x47, 0xeb, 0x34, 0x07, 0x3c, 0x2e};
static const uint64_t kMaxReadRecordSize = 1ull << 29; /* internal/magic.go:33 */

/* binary.Uvarint, Go 1.13 (the reference's go.mod) */
static uint64_t v1_uvarint(const uint8_t *p, int64_t n, int64_t *cnt) {
    uint64_t x = 0;
    unsigned s = 0;
    for (int64_t i = 0; i < n; i++) {
        uint8_t b = p[i];
        if (b < 0x80) {
            if (i > 9 || (i == 9 && b > 1)) {
                *cnt = -(i + 1);
                return 0;
            }
            *cnt = i + 1;
            return x | ((uint64_t)b << s);
        }
        if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
        s += 7;
    }
    *cnt = 0;
    return 0;
}

static uint32_t le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static uint64_t le64(const uint8_t *p) { return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32); }

typedef struct {
    int set;
    char msg[512];
} v1_once;

static void v1_set(v1_once *o, const char *fmt, ...) {
    if (o->set) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(o->msg, sizeof(o->msg), fmt, ap);
    va_end(ap);
    o->set = 1;
}

typedef struct {
    const uint8_t *p;
    int64_t n;
} v1_view;

typedef struct {
    const uint8_t *f;
    int64_t n, pos;
    /* LegacyScannerImpl.err: eof = io.EOF (Err() hides it) */
    v1_once sc_err;
    int sc_eof;
    v1_once ad_err; /* legacyScannerAdapter.err */
    const uint8_t *rec;
    int64_t rec_n;
    v1_view *buf;
    int64_t nbuf, capbuf, next;
    uint64_t block; /* file offset of the buffered record */
} v1_t;

static int v1_err(const v1_t *s) { return s->ad_err.set || s->sc_err.set; }

/* InternalScan (deprecated/recordio.go:258-300) on a bytes.Reader */
static int v1_internal_scan(v1_t *s, const uint8_t **magic) {
    *magic = NULL;
    if (s->sc_err.set || s->sc_eof) return 0;
    const int64_t avail = s->n - s->pos;
    if (avail <= 0) { /* io.ReadFull: n == 0 && io.EOF */
        s->sc_eof = 1;
        return 0;
    }
    if (avail < 20) {
        s->pos = s->n;
        v1_set(&s->sc_err, "recordio: failed to read header: unexpected EOF");
        return 0;
    }
    const uint8_t *h = s->f + s->pos;
    s->pos += 20;
    *magic = h;
    /* unmarshalHeader (recordio.go:324-334): crc over the 8 size bytes */
    const uint64_t size = le64(h + 8);
    const uint32_t crc = le32(h + 16), ncrc = orc_crc32(0, h + 8, 8);
    if (ncrc != crc) {
        v1_set(&s->sc_err, "recordio: crc check failed - corrupt record header (%u != %u)?", ncrc, crc);
        return 0;
    }
    if (size == 0) {
        s->rec = h + 20;
        s->rec_n = 0;
        return 1;
    }
    if (size > kMaxReadRecordSize) {
        v1_set(&s->sc_err, "recordio: unreasonably large read record encountered: %" PRIu64 " > %" PRIu64 " bytes",
               size, kMaxReadRecordSize);
        return 0;
    }
    const int64_t left = s->n - s->pos;
    if (left == 0) { /* io.ReadFull returns (0, io.EOF): not isErr, then the length check */
        v1_set(&s->sc_err, "recordio: short/long record: 0 < %" PRIu64, size);
        return 0;
    }
    if ((uint64_t)left < size) {
        s->pos = s->n;
        v1_set(&s->sc_err, "recordio: failed to read record: unexpected EOF");
        return 0;
    }
    s->rec = s->f + s->pos;
    s->rec_n = (int64_t)size;
    s->pos += (int64_t)size;
    return 1;
}

static void v1_push(v1_t *s, const uint8_t *p, int64_t n) {
    if (s->nbuf == s->capbuf) {
        s->capbuf = s->capbuf ? 2 * s->capbuf : 64;
        s->buf = (v1_view *)realloc(s->buf, sizeof(v1_view) * (size_t)s->capbuf);
    }
    s->buf[s->nbuf].p = p;
    s->buf[s->nbuf].n = n;
    s->nbuf++;
}

/* Unpacker.Unpack (deprecated/packer.go:214-272), no transform. Returns 0 and
 * sets ad_err on failure. Where Go would panic slicing (item sizes that wrap,
 * or a last item past the record), this reports the error text below
 * (RIO_ERR_ITEM_RANGE on the GPU path). */
static int v1_unpack(v1_t *s, const uint8_t *buf, int64_t len) {
    s->nbuf = 0;
    if (len < 4) {
        v1_set(&s->ad_err, "recordio: failed to read crc32");
        return 0;
    }
    const uint32_t crc = le32(buf);
    int64_t pos = 4, n;
    const uint64_t nbufs = v1_uvarint(buf + pos, len - pos, &n);
    if (n <= 0) {
        v1_set(&s->ad_err, "recordio: failed to read number of packed items: %" PRId64, n);
        return 0;
    }
    pos += n;
    if (nbufs > (uint64_t)len) {
        v1_set(&s->ad_err,
               "recordio: likely corrupt data, number of packed items exceeds the number of bytes in the record "
               "(%" PRIu64 " > %" PRId64 ")",
               nbufs, len);
        return 0;
    }
    const int64_t start = pos;
    uint64_t total = 0; /* Go int arithmetic wraps */
    for (uint64_t i = 0; i < nbufs; i++) {
        const uint64_t tmp = v1_uvarint(buf + pos, len - pos, &n);
        if (n <= 0) {
            v1_set(&s->ad_err, "recordio: likely corrupt data, failed to read size of packed item %" PRIu64
                               ": %" PRId64, i, n);
            return 0;
        }
        total += tmp;
        pos += n;
    }
    const uint32_t ncrc = orc_crc32(0, buf + 4, (size_t)(pos - 4));
    if (crc != ncrc) {
        v1_set(&s->ad_err, "recordio: likely corrupt data, crc check failed - corrupt packed record header (%u != %u)?",
               ncrc, crc);
        return 0;
    }
    const uint8_t *packed = buf + pos;
    const uint64_t max = (uint64_t)(len - pos);
    uint64_t prev = 0;
    int64_t sp = start;
    for (uint64_t i = 0; i + 1 < nbufs; i++) {
        const uint64_t size = v1_uvarint(buf + sp, pos - sp, &n);
        sp += n;
        const uint64_t end = prev + size; /* uint64: wraps as in Go */
        if (end > max) {
            v1_set(&s->ad_err,
                   "recordio: offset greater than buf size (%" PRIu64 " > %" PRIu64
                   "), likely due to a mismatched transform or a truncated file",
                   end, max);
            s->nbuf = 0;
            return 0;
        }
        if (end < prev) { /* packed[prev:prev+size] with high < low: Go panics */
            v1_set(&s->ad_err, "recordio: corrupt packed record header, item sizes out of range");
            s->nbuf = 0;
            return 0;
        }
        v1_push(s, packed + prev, (int64_t)size);
        prev = end;
    }
    /* the last item is packed[prev:total] (also the one empty item of nbufs == 0) */
    if (total < prev || total > max) { /* Go: a panic, or bytes past the record */
        v1_set(&s->ad_err, "recordio: corrupt packed record header, item sizes out of range");
        s->nbuf = 0;
        return 0;
    }
    v1_push(s, packed + prev, (int64_t)(total - prev));
    return 1;
}

/* scanNextBlock (legacyscanner.go:84-117) */
static int v1_next_block(v1_t *s) {
    s->nbuf = 0;
    s->next = 0;
    if (v1_err(s)) return 0;
    s->block = (uint64_t)s->pos;
    const uint8_t *magic;
    if (!v1_internal_scan(s, &magic)) return 0;
    if (memcmp(magic, kMagicPacked, 8) == 0) return v1_unpack(s, s->rec, s->rec_n);
    if (memcmp(magic, kMagicLegacyUnpacked, 8) == 0) {
        v1_push(s, s->rec, s->rec_n);
        return 1;
    }
    v1_set(&s->ad_err, "recordio: invalid magic number: [%u %u %u %u %u %u %u %u]", magic[0], magic[1], magic[2],
           magic[3], magic[4], magic[5], magic[6], magic[7]);
    return 0;
}

/* Scan (legacyscanner.go:119-133) with idUnmarshal */
static int v1_scan(v1_t *s, v1_item_fn fn, void *u) {
    while (s->next >= s->nbuf)
        if (!v1_next_block(s)) return 0;
    fn(u, s->buf[s->next].p, s->buf[s->next].n, s->block, s->next);
    s->next++;
    return 1;
}

/* Err (legacyscanner.go:135-144) */
static void v1_err_text(const v1_t *s, char *err, size_t cap) {
    if (s->ad_err.set) snprintf(err, cap, "%s", s->ad_err.msg);
    else if (s->sc_err.set) snprintf(err, cap, "%s", s->sc_err.msg);
    else if (cap) err[0] = 0;
}

/* The whole adapter run used by orc_scan / orc_seek_get for a v1 file:
 * seek == 0: Scan until false; seek == 1: Seek(ItemLocation{block, item})
 * (legacyscanner.go:67-82), then one Scan. Items go to fn; err receives Err(). */
void orc_v1_run(const uint8_t *f, int64_t n, int seek, uint64_t block, int64_t item, v1_item_fn fn, void *u,
                char *err, size_t errcap) {
    v1_t s;
    memset(&s, 0, sizeof(s));
    s.f = f;
    s.n = n;
    if (!seek) {
        while (v1_scan(&s, fn, u)) {
        }
    } else {
        /* seekRaw: bytes.Reader.Seek rejects a negative offset */
        if ((int64_t)block < 0) {
            v1_set(&s.ad_err, "bytes.Reader.Seek: negative position");
        } else {
            s.pos = (int64_t)block; /* then sc.Reset clears the scanner's error */
            if (v1_next_block(&s)) {
                if (item < 0 || item >= s.nbuf) /* (Go panics on a negative item) */
                    v1_set(&s.ad_err, "Invalid location {Block:%" PRIu64 " Item:%" PRId64 "}, block has only %" PRId64
                                      " items", block, item, s.nbuf);
                s.next = item < 0 ? s.nbuf : item;
            }
            v1_scan(&s, fn, u);
        }
    }
    v1_err_text(&s, err, errcap);
    free(s.buf);
}
