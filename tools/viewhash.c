/* Record hashes for the benchmarks' parity checks (test infrastructure, not
 * product code): a 64-bit hash of each record, given either as views (pointer,
 * length) -- the scanner's rio_scanner_next_batch output -- or as one buffer with
 * exclusive end offsets -- the generator's records. Equal records give equal
 * hashes in both forms, so a scan's records are checked against the generator's
 * without materialising them in Python. Built by base_amd/build.py into
 * tools/_build/libviewhash.so. */
#include <stdint.h>
#include <string.h>

static inline uint64_t mix(uint64_t h, uint64_t w) {
  h ^= w * 0x9E3779B97F4A7C15ull;
  h = (h << 27) | (h >> 37);
  return h * 0xBF58476D1CE4E5B9ull + 0x94D049BB133111EBull;
}

static inline uint64_t rec_hash(const uint8_t *p, uint64_t n) {
  uint64_t h = 0x5EED0004ull ^ (n * 0xD6E8FEB86659FD93ull);
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    h = mix(h, w);
  }
  if (i < n) {
    uint64_t w = 0;
    memcpy(&w, p + i, n - i);
    h = mix(h, w ^ 0xFFull << 56);
  }
  return h ^ (h >> 31);
}

void view_hash(const uint8_t *const *ptrs, const uint64_t *lens, uint64_t n, uint64_t *out) {
  for (uint64_t k = 0; k < n; k++) out[k] = rec_hash(ptrs[k], lens[k]);
}

void buf_hash(const uint8_t *data, const uint64_t *ends, uint64_t n, uint64_t *out) {
  uint64_t lo = 0;
  for (uint64_t k = 0; k < n; k++) {
    out[k] = rec_hash(data + lo, ends[k] - lo);
    lo = ends[k];
  }
}
