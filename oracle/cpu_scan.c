/*
 * ORACLE — CPU baseline only (bench.py's cpu_baseline leg). Never linked into
 * the product path.
 *
 * The reference's scan loop over an in-memory file, shaped like its own
 * sharded read test (recordio/v2_test.go:483-509: one NewShardScanner(i, i+1,
 * n) per thread, bytes.NewReader input as in BenchmarkRead,
 * recordio/recordio_test.go:51-71):
 *   LimitShard                 recordio/internal/chunk.go:198-236
 *   ChunkScanner.Scan/readChunk chunk.go:253-345 (size check, CRC32-IEEE over
 *                              [12, 28+size), magic/index/total consistency)
 *   scanNextBlock / Scan       recordio/scannerv2.go:363-404
 *   parseChunksToItems         scannerv2.go:53-97 (uvarint count, sizes, length check)
 * with tuned C decoders standing in for the reference's third-party ones (the
 * Go toolchain is absent, so the reference itself cannot run here):
 *   CRC32-IEEE  carry-less-multiply folding (PCLMULQDQ) like Go's hash/crc32
 *               IEEE path on amd64 (ieeeCLMUL), zlib crc32 for < 16 B tails
 *   flate       zlib raw inflate     (reference: klauspost/compress v1.8.6 flate,
 *                                     fed chunk by chunk like IOVecReader)
 *   zstd        libzstd ZSTD_decompress (reference: DataDog/zstd v1.4.1, which
 *                                     is libzstd through cgo; flattenIov first)
 * Errors only count; their text is the oracle's business (scanner.c).
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>
#include <zstd.h>
#include <zstd_errors.h>

#define CK 32768
#define CKH 28
#define MAXPAY 32740

static const uint8_t MAGIC_PACKED[8] = {0x2e, 0x76, 0x47, 0xeb, 0x34, 0x07, 0x3c, 0x2e};
static const uint8_t MAGIC_TRAILER[8] = {0xfe, 0xba, 0x1a, 0xd7, 0xcb, 0xdf, 0x75, 0x3a};

static uint32_t rd32(const uint8_t *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

static uint64_t uvarint(const uint8_t *p, int64_t n, int64_t *cnt) {
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
            return x | (uint64_t)b << s;
        }
        x |= (uint64_t)(b & 0x7f) << s;
        s += 7;
    }
    *cnt = 0;
    return 0;
}

/* CRC32-IEEE by folding 4 x 128-bit lanes with carry-less multiplies (Intel,
 * "Fast CRC Computation for Generic Polynomials Using PCLMULQDQ"): the fold
 * constants are x^(k) mod P for the reflected polynomial, then a Barrett
 * reduction to 32 bits. len >= 64 and a multiple of 16; raw (no inversion). */
__attribute__((target("pclmul,sse4.1"))) static uint32_t crc32_fold(uint32_t crc, const uint8_t *p, size_t len) {
    const __m128i k1k2 = _mm_set_epi64x(0x1c6e41596LL, 0x154442bd4LL);
    const __m128i k3k4 = _mm_set_epi64x(0x0ccaa009eLL, 0x1751997d0LL);
    const __m128i k5 = _mm_set_epi64x(0, 0x163cd6124LL);
    const __m128i poly = _mm_set_epi64x(0x1f7011641LL, 0x1db710641LL);
    const __m128i mask32 = _mm_set_epi32(0, 0, 0, -1);
    __m128i x0 = _mm_loadu_si128((const __m128i *)p), x1 = _mm_loadu_si128((const __m128i *)(p + 16));
    __m128i x2 = _mm_loadu_si128((const __m128i *)(p + 32)), x3 = _mm_loadu_si128((const __m128i *)(p + 48));
    x0 = _mm_xor_si128(x0, _mm_cvtsi32_si128((int)crc));
    p += 64;
    len -= 64;
#define FOLD(x, k, d) \
    x = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), d)
    while (len >= 64) {
        FOLD(x0, k1k2, _mm_loadu_si128((const __m128i *)p));
        FOLD(x1, k1k2, _mm_loadu_si128((const __m128i *)(p + 16)));
        FOLD(x2, k1k2, _mm_loadu_si128((const __m128i *)(p + 32)));
        FOLD(x3, k1k2, _mm_loadu_si128((const __m128i *)(p + 48)));
        p += 64;
        len -= 64;
    }
    FOLD(x0, k3k4, x1);
    FOLD(x0, k3k4, x2);
    FOLD(x0, k3k4, x3);
    while (len >= 16) {
        FOLD(x0, k3k4, _mm_loadu_si128((const __m128i *)p));
        p += 16;
        len -= 16;
    }
#undef FOLD
    __m128i t = _mm_clmulepi64_si128(x0, k3k4, 0x10); /* 128 -> 64 */
    x0 = _mm_xor_si128(_mm_srli_si128(x0, 8), t);
    t = _mm_clmulepi64_si128(_mm_and_si128(x0, mask32), k5, 0x00); /* 64 -> 32 */
    x0 = _mm_xor_si128(_mm_srli_si128(x0, 4), t);
    t = _mm_clmulepi64_si128(_mm_and_si128(x0, mask32), poly, 0x10); /* Barrett */
    t = _mm_clmulepi64_si128(_mm_and_si128(t, mask32), poly, 0x00);
    x0 = _mm_xor_si128(x0, t);
    return (uint32_t)_mm_extract_epi32(x0, 1);
}

/* crc32.ChecksumIEEE semantics (= zlib crc32(0, p, len)) */
static uint32_t crc32_ieee(const uint8_t *p, size_t len) {
    if (len < 64) return (uint32_t)crc32(0, p, (uInt)len);
    const size_t body = len & ~(size_t)15;
    const uint32_t c = ~crc32_fold(~0u, p, body);
    return (uint32_t)crc32(c, p + body, (uInt)(len - body));
}

/* self-check of the folding CRC against zlib (bench.py calls it once) */
int cpu_crc_selftest(void) {
    uint8_t b[4096];
    for (int i = 0; i < 4096; i++) b[i] = (uint8_t)(i * 131 + (i >> 5));
    for (size_t len = 0; len <= 4096; len += 7)
        if (crc32_ieee(b + (len & 3), len - (len & 3) * (len >= 4)) !=
            (uint32_t)crc32(0, b + (len & 3), (uInt)(len - (len & 3) * (len >= 4))))
            return 0;
    return 1;
}

typedef struct {
    const uint8_t *f;
    int64_t n;
    int codec; /* 0 none, 1 flate, 2 zstd */
    int shard, nshard;
    int64_t items, bytes; /* out; items = -1 on error */
    uint8_t *buf, *dec;
    int64_t buf_cap, dec_cap;
    z_stream zs;
    int zs_ready;
} job_t;

static int grow(uint8_t **p, int64_t *cap, int64_t need) {
    if (*cap >= need) return 1;
    int64_t c = need + need / 2 + 4096;
    uint8_t *q = (uint8_t *)realloc(*p, (size_t)c);
    if (!q) return 0;
    *p = q;
    *cap = c;
    return 1;
}

/* untransform one block (payload views) into a contiguous buffer; returns its length, -1 on error */
static int64_t untransform(job_t *j, const uint8_t **pay, const uint32_t *len, int np, const uint8_t **out) {
    int64_t tot = 0;
    for (int i = 0; i < np; i++) tot += len[i];
    if (j->codec == 0 || (j->codec == 2 && np > 1)) { /* idTransform / flattenIov: one copy */
        if (!grow(&j->buf, &j->buf_cap, tot + 1)) return -1;
        int64_t o = 0;
        for (int i = 0; i < np; i++) {
            memcpy(j->buf + o, pay[i], len[i]);
            o += len[i];
        }
        if (j->codec == 0) {
            *out = j->buf;
            return tot;
        }
    }
    if (j->codec == 2) {
        const uint8_t *src = np > 1 ? j->buf : pay[0];
        if (tot == 0) return -1; /* ErrEmptySlice */
        unsigned long long fcs = ZSTD_getFrameContentSize(src, (size_t)tot);
        int64_t want = (fcs != ZSTD_CONTENTSIZE_UNKNOWN && fcs != ZSTD_CONTENTSIZE_ERROR) ? (int64_t)fcs : 3 * tot;
        for (int tries = 0; tries < 8; tries++) {
            if (!grow(&j->dec, &j->dec_cap, want + 1)) return -1;
            size_t r = ZSTD_decompress(j->dec, (size_t)j->dec_cap, src, (size_t)tot);
            if (!ZSTD_isError(r)) {
                *out = j->dec;
                return (int64_t)r;
            }
            if (ZSTD_getErrorCode(r) != ZSTD_error_dstSize_tooSmall) return -1;
            want = 2 * j->dec_cap;
        }
        return -1;
    }
    /* flate: raw inflate fed one chunk payload at a time */
    if (!j->zs_ready) {
        memset(&j->zs, 0, sizeof(j->zs));
        if (inflateInit2(&j->zs, -15) != Z_OK) return -1;
        j->zs_ready = 1;
    } else if (inflateReset(&j->zs) != Z_OK) {
        return -1;
    }
    if (!grow(&j->dec, &j->dec_cap, 8 * tot + 65536)) return -1;
    int64_t olen = 0;
    int done = 0;
    for (int i = 0; i < np && !done; i++) {
        j->zs.next_in = (Bytef *)pay[i];
        j->zs.avail_in = len[i];
        while (!done) {
            if (j->dec_cap - olen < 65536 && !grow(&j->dec, &j->dec_cap, 2 * j->dec_cap)) return -1;
            j->zs.next_out = j->dec + olen;
            j->zs.avail_out = (uInt)(j->dec_cap - olen);
            int r = inflate(&j->zs, Z_NO_FLUSH);
            olen = j->dec_cap - j->zs.avail_out;
            if (r == Z_STREAM_END) done = 1;
            else if (r == Z_BUF_ERROR && j->zs.avail_in == 0) break; /* next payload */
            else if (r != Z_OK) return -1;
            if (j->zs.avail_in == 0 && j->zs.avail_out != 0) break;
        }
    }
    if (!done) return -1; /* unexpected EOF */
    *out = j->dec;
    return olen;
}

static void *run(void *arg) {
    job_t *j = (job_t *)arg;
    const uint8_t *f = j->f;
    const int64_t n = j->n;
    j->items = -1;
    j->bytes = 0;
    if (n < CK) return NULL;
    /* header block (readHeader): skip its chunks */
    int64_t off = (int64_t)rd32(f + 20) * CK;
    /* LimitShard (chunk.go:198-236) */
    const int64_t num = (n - off) / CK;
    const double cps = (double)num / (double)j->nshard;
    const int64_t start = off;
    off = start + (int64_t)((double)j->shard * cps) * CK;
    const int64_t limit = start + (int64_t)((double)(j->shard + 1) * cps) * CK;
    if (j->shard > 0 && off + CKH <= n) {
        const uint32_t total = rd32(f + off + 20), index = rd32(f + off + 24);
        if (index != 0) off += (int64_t)CK * (total - index);
    }
    const uint8_t *pay[4096];
    uint32_t len[4096];
    int64_t items = 0, bytes = 0;
    while (off < limit && off + CK <= n) {
        /* one block: readChunk until index == total - 1 */
        int np = 0;
        const uint8_t *magic = f + off;
        uint32_t total0 = 0;
        for (;;) {
            if (off + CK > n) return NULL; /* unexpected EOF */
            const uint8_t *c = f + off;
            const uint32_t size = rd32(c + 16), total = rd32(c + 20), index = rd32(c + 24);
            if (size > MAXPAY) return NULL;
            if (crc32_ieee(c + 12, 16 + size) != rd32(c + 8)) return NULL;
            if (np == 0) total0 = total;
            if (memcmp(c, magic, 8) != 0 || index != (uint32_t)np || total != total0 || np >= 4096) return NULL;
            pay[np] = c + CKH;
            len[np] = size;
            np++;
            off += CK;
            if (index + 1 == total) break;
        }
        if (memcmp(magic, MAGIC_TRAILER, 8) == 0) break;
        if (memcmp(magic, MAGIC_PACKED, 8) != 0) return NULL;
        const uint8_t *blk;
        const int64_t blen = untransform(j, pay, len, np, &blk);
        if (blen < 0) return NULL;
        int64_t k;
        const uint64_t nitems = uvarint(blk, blen, &k);
        if (k <= 0) return NULL;
        int64_t pos = k;
        uint64_t sum = 0;
        for (uint64_t i = 0; i < nitems; i++) {
            sum += uvarint(blk + pos, blen - pos, &k);
            if (k <= 0) return NULL;
            pos += k;
        }
        if ((int64_t)sum + pos != blen) return NULL;
        items += (int64_t)nitems;
        bytes += (int64_t)sum;
    }
    j->items = items;
    j->bytes = bytes;
    return NULL;
}

/* Scan `f` on nthreads threads, thread i taking NewShardScanner(i, i+1,
 * nthreads); returns the records found (or -1 on any error), *bytes_out their
 * bytes. */
int64_t cpu_scan(const uint8_t *f, int64_t n, int codec, int nthreads, int64_t *bytes_out) {
    if (nthreads < 1) nthreads = 1;
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int i = 0; i < nthreads; i++) {
        jobs[i].f = f;
        jobs[i].n = n;
        jobs[i].codec = codec;
        jobs[i].shard = i;
        jobs[i].nshard = nthreads;
    }
    for (int i = 1; i < nthreads; i++) pthread_create(&th[i], NULL, run, &jobs[i]);
    run(&jobs[0]);
    for (int i = 1; i < nthreads; i++) pthread_join(th[i], NULL);
    int64_t items = 0, bytes = 0;
    for (int i = 0; i < nthreads; i++) {
        if (jobs[i].items < 0) items = -1;
        if (items >= 0) items += jobs[i].items;
        bytes += jobs[i].bytes;
        free(jobs[i].buf);
        free(jobs[i].dec);
        if (jobs[i].zs_ready) inflateEnd(&jobs[i].zs);
    }
    free(jobs);
    free(th);
    *bytes_out = bytes;
    return items;
}
