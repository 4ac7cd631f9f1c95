/*
 * ORACLE — test infrastructure only. Never linked into the product path.
 *
 * CPU restatement of raw DEFLATE (RFC 1951) decoding with the acceptance rules
 * and error conditions of Go's compress/flate inflater, which the reference's
 * "flate" transformer uses through github.com/klauspost/compress v1.8.6
 * (go.mod:24; call site recordio/recordioflate/recordioflate.go:54-65). That
 * dependency is not vendored under /root/reference; its published algorithm is
 * Go's inflate.go (klauspost/compress/flate is a fork of it):
 *   - huffmanDecoder.init: codes must be complete, except the degenerate single
 *     code of length 1; an all-zero length set is an "empty" tree that fails when
 *     used;
 *   - readHuffman: HLIT <= 286, HDIST <= 30, repeat code 16 needs a previous
 *     length, repeats may not run past HLIT+HDIST; h1.min raised to len(EOB);
 *   - huffmanBlock: literal/length symbols 286/287 and distance codes 30/31 are
 *     corrupt; a distance beyond the bytes produced so far (capped at the 32 KiB
 *     window) is corrupt;
 *   - stored blocks: discard buffered bits, LEN must equal ~NLEN;
 *   - decoding stops at the end of the BFINAL block; trailing bytes are ignored;
 *   - input exhausted mid-stream -> "unexpected EOF".
 * Bytes are pulled from the input one at a time only when more bits are needed
 * (Go's moreBits), so the corrupt-input offset follows Go's f.roffset.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define MAXBITS 15
#define FASTBITS 10

typedef struct {
    int min, max;          /* shortest/longest code length (0 = empty tree) */
    int empty;
    uint16_t count[MAXBITS + 1];
    uint16_t symbol[320];   /* symbols in canonical order */
    uint16_t fast[1 << FASTBITS]; /* (len << 9 | sym) for codes <= FASTBITS, 0 = slow */
} huff_t;

typedef struct {
    const uint8_t *in;
    int64_t n, pos;         /* pos == Go's roffset */
    uint64_t bitbuf;
    int nb;
    uint8_t *out;
    int64_t cap, olen;
    int err;                /* ORC_INFLATE_* */
    int64_t err_off;
} inf_t;

static const uint8_t kCodeOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static int more_bits(inf_t *s) {
    if (s->pos >= s->n) {
        if (!s->err) s->err = ORC_INFLATE_UNEXPECTED_EOF;
        return 0;
    }
    s->bitbuf |= (uint64_t)s->in[s->pos++] << s->nb;
    s->nb += 8;
    return 1;
}

static int need(inf_t *s, int n) {
    while (s->nb < n)
        if (!more_bits(s)) return 0;
    return 1;
}

static uint32_t take(inf_t *s, int n) {
    uint32_t v = (uint32_t)(s->bitbuf & ((1ull << n) - 1));
    s->bitbuf >>= n;
    s->nb -= n;
    return v;
}

static void corrupt(inf_t *s) {
    if (!s->err) {
        s->err = ORC_INFLATE_CORRUPT;
        s->err_off = s->pos;
    }
}

static uint32_t rev(uint32_t code, int len) {
    uint32_t r = 0;
    for (int i = 0; i < len; i++) r |= ((code >> i) & 1u) << (len - 1 - i);
    return r;
}

/* huffmanDecoder.init semantics: returns 0 when the code set is rejected. */
static int huff_init(huff_t *h, const uint8_t *lengths, int n) {
    memset(h, 0, sizeof(*h));
    for (int i = 0; i < n; i++) {
        int l = lengths[i];
        if (!l) continue;
        if (h->min == 0 || l < h->min) h->min = l;
        if (l > h->max) h->max = l;
        h->count[l]++;
    }
    if (h->max == 0) {
        h->empty = 1;
        return 1;
    }
    int code = 0;
    for (int i = h->min; i <= h->max; i++) {
        code <<= 1;
        code += h->count[i];
    }
    if (code != (1 << h->max) && !(code == 1 && h->max == 1)) return 0;
    uint16_t offs[MAXBITS + 2];
    offs[1] = 0;
    for (int l = 1; l <= MAXBITS; l++) offs[l + 1] = offs[l] + h->count[l];
    for (int i = 0; i < n; i++)
        if (lengths[i]) h->symbol[offs[lengths[i]]++] = (uint16_t)i;
    /* fast table: canonical codes assigned in (length, symbol) order */
    int nextcode = 0, k = 0;
    for (int l = 1; l <= MAXBITS; l++) {
        for (int j = 0; j < h->count[l]; j++, k++) {
            if (l <= FASTBITS) {
                uint32_t r = rev((uint32_t)(nextcode + j), l);
                for (uint32_t f = r; f < (1u << FASTBITS); f += (1u << l))
                    h->fast[f] = (uint16_t)((l << 9) | h->symbol[k]);
            }
        }
        nextcode = (nextcode + h->count[l]) << 1;
    }
    return 1;
}

/* huffSym: read the minimum number of bytes that covers the symbol's code. */
static int huff_sym(inf_t *s, const huff_t *h) {
    if (h->empty) {
        /* Go: lookup yields n == 0 once h.min bits are present */
        if (!need(s, h->min)) return -1;
        corrupt(s);
        return -1;
    }
    int n = h->min;
    for (;;) {
        if (!need(s, n)) return -1;
        /* decode against available bits (bits above nb are zero, as in Go) */
        int avail = s->nb < MAXBITS ? s->nb : MAXBITS;
        uint32_t bits = (uint32_t)(s->bitbuf & ((1u << avail) - 1));
        int len = 0, sym = -1;
        if (avail >= 1) {
            uint16_t e = h->fast[bits & ((1u << FASTBITS) - 1)];
            if (e && (e >> 9) <= avail) {
                len = e >> 9;
                sym = e & 511;
            }
        }
        if (sym < 0) {
            /* canonical walk over all lengths, using zeros beyond nb */
            int code = 0, first = 0, index = 0;
            for (int l = 1; l <= MAXBITS; l++) {
                code |= (int)((bits >> (l - 1)) & 1u);
                int cnt = h->count[l];
                if (code - cnt < first) {
                    len = l;
                    sym = h->symbol[index + (code - first)];
                    break;
                }
                index += cnt;
                first += cnt;
                first <<= 1;
                code <<= 1;
            }
        }
        if (sym < 0) { /* cannot happen for a complete code */
            corrupt(s);
            return -1;
        }
        if (len <= s->nb) {
            take(s, len);
            return sym;
        }
        n = len;
    }
}

static int emit(inf_t *s, uint8_t b) {
    if (s->olen >= s->cap) {
        s->err = ORC_INFLATE_OUTPUT_FULL;
        return 0;
    }
    s->out[s->olen++] = b;
    return 1;
}

static void fixed_tables(huff_t *lit) {
    uint8_t l[288];
    int i = 0;
    for (; i < 144; i++) l[i] = 8;
    for (; i < 256; i++) l[i] = 9;
    for (; i < 280; i++) l[i] = 7;
    for (; i < 288; i++) l[i] = 8;
    huff_init(lit, l, 288);
}

static int huffman_block(inf_t *s, const huff_t *hl, const huff_t *hd) {
    for (;;) {
        int v = huff_sym(s, hl);
        if (v < 0) return 0;
        if (v < 256) {
            if (!emit(s, (uint8_t)v)) return 0;
            continue;
        }
        if (v == 256) return 1;
        int length, nbits;
        if (v < 265) { length = v - (257 - 3); nbits = 0; }
        else if (v < 269) { length = v * 2 - (265 * 2 - 11); nbits = 1; }
        else if (v < 273) { length = v * 4 - (269 * 4 - 19); nbits = 2; }
        else if (v < 277) { length = v * 8 - (273 * 8 - 35); nbits = 3; }
        else if (v < 281) { length = v * 16 - (277 * 16 - 67); nbits = 4; }
        else if (v < 285) { length = v * 32 - (281 * 32 - 131); nbits = 5; }
        else if (v < 286) { length = 258; nbits = 0; }
        else { corrupt(s); return 0; }
        if (nbits > 0) {
            if (!need(s, nbits)) return 0;
            length += (int)take(s, nbits);
        }
        int dist;
        if (hd == NULL) {
            if (!need(s, 5)) return 0;
            dist = (int)rev(take(s, 5), 5);
        } else {
            dist = huff_sym(s, hd);
            if (dist < 0) return 0;
        }
        if (dist < 4) {
            dist++;
        } else if (dist < 30) {
            int nb = (dist - 2) >> 1;
            int extra = (dist & 1) << nb;
            if (!need(s, nb)) return 0;
            extra |= (int)take(s, nb);
            dist = (1 << (nb + 1)) + 1 + extra;
        } else {
            corrupt(s);
            return 0;
        }
        int64_t hist = s->olen < 32768 ? s->olen : 32768;
        if (dist > hist) {
            corrupt(s);
            return 0;
        }
        if (s->olen + length > s->cap) {
            s->err = ORC_INFLATE_OUTPUT_FULL;
            return 0;
        }
        for (int i = 0; i < length; i++) s->out[s->olen + i] = s->out[s->olen - dist + i];
        s->olen += length;
    }
}

static int read_dynamic(inf_t *s, huff_t *hl, huff_t *hd) {
    if (!need(s, 5 + 5 + 4)) return 0;
    int nlit = (int)take(s, 5) + 257;
    if (nlit > 286) { corrupt(s); return 0; }
    int ndist = (int)take(s, 5) + 1;
    if (ndist > 30) { corrupt(s); return 0; }
    int nclen = (int)take(s, 4) + 4;
    uint8_t cl[19] = {0};
    for (int i = 0; i < nclen; i++) {
        if (!need(s, 3)) return 0;
        cl[kCodeOrder[i]] = (uint8_t)take(s, 3);
    }
    huff_t hc;
    if (!huff_init(&hc, cl, 19)) { corrupt(s); return 0; }
    uint8_t bits[286 + 30];
    int n = nlit + ndist;
    for (int i = 0; i < n;) {
        int x = huff_sym(s, &hc);
        if (x < 0) return 0;
        if (x < 16) {
            bits[i++] = (uint8_t)x;
            continue;
        }
        int rep, nb, b;
        switch (x) {
        case 16:
            rep = 3; nb = 2;
            if (i == 0) { corrupt(s); return 0; }
            b = bits[i - 1];
            break;
        case 17: rep = 3; nb = 3; b = 0; break;
        case 18: rep = 11; nb = 7; b = 0; break;
        default: corrupt(s); return 0; /* Go: InternalError, unreachable */
        }
        if (!need(s, nb)) return 0;
        rep += (int)take(s, nb);
        if (i + rep > n) { corrupt(s); return 0; }
        for (int j = 0; j < rep; j++) bits[i++] = (uint8_t)b;
    }
    if (!huff_init(hl, bits, nlit) || !huff_init(hd, bits + nlit, ndist)) {
        corrupt(s);
        return 0;
    }
    if (!hl->empty && hl->min < bits[256]) hl->min = bits[256];
    return 1;
}

int orc_inflate(const uint8_t *in, int64_t n, uint8_t *out, int64_t cap, int64_t *out_len,
                int64_t *err_off) {
    inf_t s;
    memset(&s, 0, sizeof(s));
    s.in = in;
    s.n = n;
    s.out = out;
    s.cap = cap;
    static huff_t fixed_lit;
    static int fixed_ready = 0;
    if (!fixed_ready) {
        fixed_tables(&fixed_lit);
        fixed_ready = 1;
    }
    huff_t hl, hd;
    for (;;) {
        if (!need(&s, 3)) break;
        int final = (int)take(&s, 1);
        int type = (int)take(&s, 2);
        int ok = 1;
        if (type == 0) {
            s.nb = 0;
            s.bitbuf = 0;
            if (s.pos + 4 > s.n) {
                s.pos = s.n;
                s.err = ORC_INFLATE_UNEXPECTED_EOF;
                break;
            }
            uint32_t len = s.in[s.pos] | ((uint32_t)s.in[s.pos + 1] << 8);
            uint32_t nlen = s.in[s.pos + 2] | ((uint32_t)s.in[s.pos + 3] << 8);
            s.pos += 4;
            if ((uint16_t)nlen != (uint16_t)~len) {
                corrupt(&s);
                break;
            }
            if (s.olen + len > s.cap) {
                s.err = ORC_INFLATE_OUTPUT_FULL;
                break;
            }
            if (s.pos + len > s.n) {
                s.err = ORC_INFLATE_UNEXPECTED_EOF;
                break;
            }
            memcpy(s.out + s.olen, s.in + s.pos, len);
            s.olen += len;
            s.pos += len;
        } else if (type == 1) {
            ok = huffman_block(&s, &fixed_lit, NULL);
        } else if (type == 2) {
            ok = read_dynamic(&s, &hl, &hd) && huffman_block(&s, &hl, &hd);
        } else {
            corrupt(&s);
            break;
        }
        if (!ok || s.err) break;
        if (final) break;
    }
    *out_len = s.olen;
    if (err_off) *err_off = s.err_off;
    return s.err;
}
