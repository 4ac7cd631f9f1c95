/* ORACLE — placeholder until the RFC 8878 restatement lands. */
#include "oracle.h"
int orc_zstd_decompress(const uint8_t *in, int64_t n, uint8_t *out, int64_t cap, int64_t *out_len,
                        const char **msg) {
    (void)in; (void)n; (void)out; (void)cap;
    *out_len = 0;
    *msg = "zstd: oracle decoder not built";
    return ORC_ZSTD_ERROR;
}
int64_t orc_zstd_content_size(const uint8_t *in, int64_t n) { (void)in; (void)n; return -1; }
