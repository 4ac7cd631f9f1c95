/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg). Never linked into or called by the product path.
 */
#ifndef RIO_ORACLE_H
#define RIO_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORC_INFLATE_OK = 0,
    ORC_INFLATE_CORRUPT = 1,
    ORC_INFLATE_UNEXPECTED_EOF = 2,
    ORC_INFLATE_OUTPUT_FULL = 3,
};

enum {
    ORC_ZSTD_OK = 0,
    ORC_ZSTD_ERROR = 1,
    ORC_ZSTD_OUTPUT_FULL = 3,
};

int orc_inflate(const uint8_t *in, int64_t n, uint8_t *out, int64_t cap, int64_t *out_len,
                int64_t *err_off);
/* returns ORC_ZSTD_*; *msg receives a libzstd-style error name */
int orc_zstd_decompress(const uint8_t *in, int64_t n, uint8_t *out, int64_t cap,
                        int64_t *out_len, const char **msg);
/* upper bound of the decompressed size declared by the frames, -1 if unknown */
int64_t orc_zstd_content_size(const uint8_t *in, int64_t n);

uint32_t orc_crc32(uint32_t crc, const uint8_t *p, size_t n);

typedef struct orc_result orc_result;

/* Scan a whole in-memory recordio file the way the reference does:
 *   sc := NewShardScanner(bytes.NewReader(f), opts, start, limit, nshard)
 *   if flags&1: sc.Trailer()      (as readAllV2 / doShardedReads do)
 *   for sc.Scan() { collect sc.Get() }
 */
orc_result *orc_scan(const uint8_t *f, int64_t n, int start, int limit, int nshard, int flags);
/* Scanner.Seek(ItemLocation{block, item}) then one Scan()+Get() on a fresh scanner */
orc_result *orc_seek_get(const uint8_t *f, int64_t n, uint64_t block, int64_t item);
void orc_free(orc_result *r);

int64_t orc_n_items(const orc_result *r);
const uint8_t *orc_items(const orc_result *r);       /* concatenated item bytes */
const uint64_t *orc_item_ends(const orc_result *r);  /* exclusive ends */
const uint64_t *orc_item_block(const orc_result *r); /* ItemLocation.Block per item */
const int64_t *orc_item_index(const orc_result *r);  /* ItemLocation.Item per item */
const char *orc_err(const orc_result *r);            /* "" when Err() == nil */
int orc_has_trailer(const orc_result *r);            /* Trailer() returned non-nil */
const uint8_t *orc_trailer(const orc_result *r, int64_t *len);
int orc_header_len(const orc_result *r);
/* type: 1 bool, 2 int, 3 uint, 4 string; ival holds bool/int/uint */
int orc_header_kv(const orc_result *r, int i, const char **key, int *type, int64_t *ival,
                  const uint8_t **sval, int64_t *slen);
int orc_is_legacy(const orc_result *r);

/* LimitShard arithmetic (chunk.go:202-206), exposed for the shard table */
void orc_shard_range(int64_t file_size, int64_t off, int start, int limit, int nshard,
                     int64_t *o_off, int64_t *o_limit);

/* CPU baseline helper: decode every item of a file; returns items, bytes */
int64_t orc_scan_count(const uint8_t *f, int64_t n, int64_t *bytes_out, int start, int limit,
                       int nshard);

#ifdef __cplusplus
}
#endif
#endif
