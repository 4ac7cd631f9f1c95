// Scanner layer of the C ABI: the host-side mirror of recordio.NewScanner /
// NewShardScanner / Scanner (recordio/scannerv2.go:100-425) on top of the GPU
// batch decoder. Control flow (header, LimitShard, Trailer, Seek, sticky first
// error) is host logic on a few bytes; every chunk CRC, block parse and
// untransform runs in the HIP pipeline.
#include <hip/hip_runtime.h>
#include <inttypes.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <future>
#include <string>
#include <thread>
#include <vector>

#include "pipeline.h"
#include "rio_internal.h"

namespace {

constexpr uint64_t kCk = RIO_CHUNK_SIZE;
const uint8_t kMagicHeaderBytes[8] = {0xd9, 0xe1, 0xd9, 0x5c, 0xc2, 0x16, 0x04, 0xf7};
const uint8_t kMagicTrailerBytes[8] = {0xfe, 0xba, 0x1a, 0xd7, 0xcb, 0xdf, 0x75, 0x3a};

// host view of item i of a collected batch (rio_gpu.h: span view or records)
inline const uint8_t *batch_item(const rio_batch &b, uint64_t i, uint64_t *len) {
  const uint64_t o = b.item_off[i];
  *len = b.item_len[i];
  return (o & RIO_ITEM_IN_RECORDS) ? b.records + (o & ~RIO_ITEM_IN_RECORDS) : b.span + o;
}

struct KV {
  std::string key;
  int32_t type = 0;  // 1 bool 2 int 3 uint 4 string
  int64_t ival = 0;
  std::string sval;
};

void fmt_magic_v(const uint8_t *m, char *out) {
  sprintf(out, "[%u %u %u %u %u %u %u %u]", m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7]);
}

// binary.Uvarint (Go 1.13-1.15)
uint64_t uvarint(const uint8_t *p, uint64_t n, int64_t *cnt) {
  uint64_t x = 0;
  unsigned s = 0;
  for (uint64_t i = 0; i < n; i++) {
    const uint8_t b = p[i];
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) {
        *cnt = -(int64_t)(i + 1);
        return 0;
      }
      *cnt = (int64_t)i + 1;
      return x | ((uint64_t)b << s);
    }
    if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
  *cnt = 0;
  return 0;
}

// headerDecoder (header.go:140-198)
struct HeaderDecoder {
  const uint8_t *p;
  uint64_t n;
  std::string err;
  void set(const char *m) {
    if (err.empty()) err = m;
  }
  int value(KV &v) {
    if (n == 0) {
      set("Failed to read byte in header");
      return 0;
    }
    const uint8_t t = *p++;
    n--;
    switch (t) {
    case 1:
      v.type = 1;
      if (n == 0) {
        set("Failed to read byte in header");
        return 1;
      }
      v.ival = *p++ != 0;
      n--;
      return 1;
    case 2:
    case 3: {
      int64_t c;
      uint64_t u = uvarint(p, n, &c);
      v.type = t;
      if (c <= 0) {
        set("Failed to parse uint");
        return t;
      }
      p += c;
      n -= (uint64_t)c;
      if (t == 2) {
        int64_t x = (int64_t)(u >> 1);
        if (u & 1) x = ~x;
        v.ival = x;
      } else {
        v.ival = (int64_t)u;
      }
      return t;
    }
    case 4: {
      KV len;
      int lt = value(len);
      v.type = 4;
      if (!err.empty()) return 4;
      if (lt != 3) {
        set("failed to read string key");
        return 4;
      }
      if (n < (uint64_t)len.ival) {
        char m[96];
        snprintf(m, sizeof(m), "header invalid string (%" PRIu64 ")", (uint64_t)len.ival);
        set(m);
        return 4;
      }
      v.sval.assign((const char *)p, (size_t)len.ival);
      p += len.ival;
      n -= (uint64_t)len.ival;
      return 4;
    }
    default:
      set("illegal header type uint8");
      return 0;
    }
  }
};

}  // namespace

struct rio_scanner {
  rio_ctx *ctx = nullptr;
  rio_reader r{};
  uint64_t file_size = 0;
  // errors.Once{Ignored: io.EOF}
  bool err_set = false;
  rio_error err{};
  bool pending_set = false;  // error found in a batch, visible once its items are consumed
  rio_error pending{};
  bool error_scanner = false;
  std::vector<KV> header;
  int32_t codec = RIO_CODEC_NONE;
  // a v1 file (legacyScannerAdapter, legacyscanner.go): body spans decode as v1
  // records (rio_scan_v1_span); off is the next record's offset
  bool v1 = false;
  // ChunkScanner position
  uint64_t off = 0, limit = UINT64_MAX;
  // current batch: the span (pinned host staging; none-codec items are views
  // into it) and the result buffers, both owned by this scanner
  uint8_t *span = nullptr;
  uint64_t span_cap = 0;
  rio_results *res = nullptr;
  rio_batch batch{};
  bool have_batch = false;
  bool done = false;  // no further batches (EOF or error)
  uint64_t blk = 0, item = 0;  // next item to deliver (global index in batch), its block
  uint64_t skip = 0;           // items to skip in the first block of the next batch
  const uint8_t *cur = nullptr;
  uint64_t cur_len = 0;
  uint64_t cur_block = 0;
  int64_t cur_item = 0;
  std::vector<uint8_t> trailer;
  int shard_start = 0, shard_limit = 1, shard_n = 1;
  // Read-ahead: while the caller consumes a batch, a
  // thread reads the file bytes after its span into the other pinned buffer
  // (kRaRoom bytes of room in front of them); the next span is the previous
  // span's unconsumed tail (a partial block, copied into that room) followed
  // by those bytes. Only file reads run on the thread, never the ctx.
  static constexpr uint64_t kRaRoom = 8ull << 20;
  uint8_t *ra_buf = nullptr;
  uint64_t ra_cap = 0;
  std::thread ra_th;
  bool ra_running = false, ra_valid = false;
  uint64_t ra_at = 0, ra_len = 0, ra_got = 0;  // prefetched file bytes [ra_at, ra_at + ra_got)
  int ra_st = 0;
  const uint8_t *span_data = nullptr;  // the current batch's span bytes (views point into them)
  uint64_t span_at = 0, span_n = 0;    // its file offset and length
  void ra_join() {
    if (ra_running) {
      ra_th.join();
      ra_running = false;
    }
  }
  void ra_drop() {
    ra_join();
    ra_valid = false;
  }
  void ra_start(uint64_t at, uint64_t len) {  // read [at, at + len) into ra_buf + kRaRoom
    ra_drop();
    if (len == 0 || ensure_buf(&ra_buf, &ra_cap, kRaRoom + rio_ctx_max_span(ctx))) return;
    ra_at = at;
    ra_len = len;
    ra_got = 0;
    ra_st = 0;
    ra_valid = true;
    ra_running = true;
    ra_th = std::thread([this] { ra_got = read_full(ra_buf + kRaRoom, ra_len, ra_at, &ra_st); });
  }
  // Spans ahead: the body's next spans are decoded on further contexts (the
  // ctx's siblings), kSlots - 1 of them in flight beside the current batch, each
  // begun on a thread of its own so that no span's H2D copy and decode waits
  // for the caller. A span's result copies come back while the caller consumes
  // the batches before it, and the copies of different spans overlap on the
  // full-duplex link. A span ahead starts where the span before it will stop:
  // for the first, the current batch's extent (known); for the next, the end of
  // the last complete block of the span before it, read from that span's last
  // chunk header on the host (a prediction: when the GPU's extent differs --
  // a corrupt header, an error, a limit -- the span is dropped and the batch is
  // decoded when it is asked for). A slot is a (context, results) pair: the
  // current batch's is `slot`, each span ahead holds another. Staging buffers
  // rotate: the current batch's span (its views point there), one per span
  // ahead, and the read-ahead's, with spares from batches consumed.
  static constexpr int kSlots = 3;
  // Span ramp: an uncompressed body's first spans are smaller (the ctx's span
  // >> ramp_steps, then twice that, ... up to the ctx's span), so that the
  // first span's copy in is short and the next span's copy follows it at once
  // (the next span's start is known only once a span is decoded). Only for
  // spans of at least ramp_min bytes (RIO_SPAN_RAMP_MIN; RIO_SPAN_RAMP: the
  // steps, 0 off). A span that holds no whole block turns the ramp off.
  // End to end, A/B (profiles/r06_span_ramp_ab.jsonl): C2 42.3 -> 46.0 GiB/s;
  // flate and zstd spans measured slower ramped (C4 13.6 -> 12.8, C3 at
  // MaxItems = 16384 11.6 -> 11.4): a short span of large blocks decodes
  // almost as long as a whole one, so compressed bodies are not ramped.
  int ramp_steps = 2;
  uint64_t ramp_min = 256ull << 20;
  bool ramp_off = false;
  // compressed bodies of small blocks (the first block under kEarlyChunks
  // chunks) ramp too, and stage their next span early (RIO_SPAN_RAMP_C=0: not):
  // their spans decode in proportion to their size
  bool ramp_c = true;
  int ramp_blk = -1;  // the body's first block: 1 small, 0 large, -1 not yet read
  uint64_t body_next = 0;  // the index of the next body span to become the current batch
  uint64_t span_size(uint64_t idx) const {
    const uint64_t maxspan = rio_ctx_max_span(ctx);
    if (ramp_off || v1 || (codec != RIO_CODEC_NONE && !(ramp_c && ramp_blk == 1)) || ramp_steps <= 0 ||
        maxspan < ramp_min || idx >= (uint64_t)ramp_steps)
      return maxspan;
    const uint64_t sz = (maxspan >> (ramp_steps - (int)idx)) / kCk * kCk;
    return sz < 4 * kCk ? maxspan : sz;
  }
  int depth = 0;  // spans ahead (the ctx's RIO_CFG_SPANS_AHEAD: 0 .. kSlots - 1, default kSlots - 1)
  // Early first span ahead (RIO_SCAN_EARLY, default on): a body span read by
  // the main thread (the first, or after a dropped prediction) is staged, and
  // once its copy in is complete -- not once it is decoded -- the span after it
  // is begun from the host's prediction of where it stops. That span's copy in
  // then runs during this span's decode instead of after it; its decode still
  // waits for this one (cur_done).
  // Only for compressed bodies of large blocks (the span's first block at least
  // kEarlyChunks chunks): their spans decode slowly for their size (few blocks
  // to spread over the GPU), so the next copy in waited on a long decode. End to
  // end, A/B (profiles/r06_e2e_early_stage_ab.jsonl): C4 13.5 -> 14.7-14.8 GiB/s,
  // C3 at MaxItems = 16384 11.4-11.5 -> 12.4; C3 at 1,024 items per block 15.1-15.4
  // -> 14.7-15.1 and C2 45.1-46.3 -> 43.4-43.6, hence not for those.
  static constexpr uint32_t kEarlyChunks = 8;
  static uint32_t first_block_chunks(const uint8_t *base, uint64_t n) {
    if (n < kCk) return 0;
    uint32_t total;
    memcpy(&total, base + 20, 4);  // its first chunk's total (chunk.go:31-53)
    return total;
  }
  bool early = true;
  std::promise<void> cur_done;
  std::shared_future<void> cur_done_f;
  rio_ctx *cx[kSlots] = {};
  rio_results *rs[kSlots] = {};
  int slot = 0;
  struct Ahead {
    int slot = 0;
    uint64_t at = 0, n = 0;
    const uint8_t *base = nullptr;
    uint8_t *buf = nullptr;
    uint64_t cap = 0;
    bool ok = false;  // begun (the context held the span)
    int rc = 0;
    std::string msg;  // rio_last_error() of the beginning thread, when rc != 0
    rio_batch b{};
    std::thread th;
    std::promise<void> begun;          // set when the thread is done (begun or not)
    std::shared_future<void> begun_f;  // (the next span's thread waits for it before its decode)
    // set once the span's file bytes are in buf (or the read failed: read_ok
    // false); the main thread waits for it before it reads the span's last
    // chunk header and copies its tail into the next span ahead
    std::promise<void> read;
    std::shared_future<void> read_f;
    bool read_ok = false;
  };
  std::deque<Ahead> aq;
  std::vector<std::pair<uint8_t *, uint64_t>> spare;  // staging buffers free for reuse
  std::string ahead_msg;                               // the taken span's error text
  void ahead_drop() {
    for (Ahead &e : aq) {
      if (e.th.joinable()) e.th.join();
      if (e.ok) rio_scan_span_end(cx[e.slot]);
      spare.emplace_back(e.buf, e.cap);
    }
    aq.clear();
  }
  // the current batch's result copies (rio_scan_span_begin) in place
  int finish_cur() { return rio_scan_span_end(cx[slot]); }
  // A span ahead will be begun: every slot's context opened now, while no
  // span-ahead thread runs (a sibling is opened from the context before it,
  // which such a thread would otherwise be using; rio_gpu.h: a scanner's spans
  // ahead hold `depth` further contexts of the ctx's size until rio_close). A
  // file that fits one span never opens them.
  bool open_siblings() {
    for (int i = 1; i <= depth; i++)
      if (!cx[i]) {
        cx[i] = rio_ctx_sibling(cx[i - 1]);
        if (!cx[i]) return false;
        rs[i] = rio_ctx_take_results(ctx);
      }
    return true;
  }
  // a body span in host memory, decoded into the current slot (results deferred)
  int scan_body(const uint8_t *base, uint64_t n, uint64_t at, rio_batch *out) {
    const int is_end = (at + n >= file_size);
    // (a sibling: as large as the ctx, which a block longer than the span grew)
    if (cx[slot] != ctx && rio_ctx_reserve_span(cx[slot], n) != 0) return -1;
    if (v1) return rio_scan_v1_span_mode(cx[slot], base, n, at, is_end, rs[slot], out);
    return rio_scan_span_begin(cx[slot], base, n, at, is_end, limit, codec, rs[slot], out);
  }
  // the oldest span ahead, if it starts at `at` and spans n bytes
  bool ahead_matches(uint64_t at, uint64_t n) {
    if (aq.empty() || aq.front().at != at || aq.front().n != n) return false;
    Ahead &e = aq.front();
    if (e.th.joinable()) e.th.join();
    return e.ok;
  }
  // the oldest span ahead becomes the current batch
  int take_ahead(rio_batch *out) {
    Ahead &e = aq.front();
    spare.emplace_back(span, span_cap);  // (the previous batch's buffer is free now)
    span = e.buf;
    span_cap = e.cap;
    span_data = e.base;
    span_at = e.at;
    span_n = e.n;
    slot = e.slot;
    *out = e.b;
    const int rc = e.rc;
    ahead_msg = e.msg;
    aq.pop_front();
    return rc;
  }
  // where the span [at, at + n) in host memory will stop: after its last
  // complete block (its last chunk's index and total, chunk.go:31-53); 0 when
  // that cannot be told (the block runs past the span, or a header is not sane)
  static uint64_t predict_consumed(const uint8_t *base, uint64_t n) {
    const uint64_t nck = n / kCk;
    if (nck == 0) return 0;
    uint32_t total, index;
    memcpy(&total, base + (nck - 1) * kCk + 20, 4);
    memcpy(&index, base + (nck - 1) * kCk + 24, 4);
    if (total == 0 || index >= total || index >= nck) return 0;
    return (index + 1 == total ? nck : nck - 1 - index) * kCk;
  }
  // fill the spans ahead: each next span is the unconsumed tail of the span
  // before it (copied here) and the file bytes after that span: the read-ahead's
  // when it holds them, else read by the span's own thread before its decode
  void begin_ahead(bool early_first = false) {
    if (v1 || done || err_set || depth == 0) return;
    const uint64_t maxspan = rio_ctx_max_span(ctx);
    while ((int)aq.size() < depth) {
      // the span before the new one: the last one ahead, or the current batch
      const bool first = aq.empty();
      const uint8_t *pdata = first ? span_data : aq.back().base;
      const uint64_t pat = first ? span_at : aq.back().at, pn = first ? span_n : aq.back().n;
      const uint64_t pend = pat + pn;
      if (!pdata || pend >= file_size) return;
      uint64_t at = off;
      if (first && early_first) {  // (the current span is still to be decoded: predicted as the later ones)
        const uint64_t c = predict_consumed(pdata, pn);
        if (c == 0) return;
        at = pat + c;
      } else if (!first) {
        // the span before this one is still being read by its own thread: its
        // last chunk header and its tail are only there once that read is done
        aq.back().read_f.wait();
        if (!aq.back().read_ok) return;
        const uint64_t c = predict_consumed(pdata, pn);
        if (c == 0) return;
        at = pat + c;
      }
      if (at >= limit || at >= file_size || at < pat || at > pend || pend - at > kRaRoom) return;
      // (the index of this span: body_next counts the current batch once it is decoded)
      const uint64_t want = span_size(body_next + aq.size() + (early_first ? 1 : 0));
      const uint64_t n = file_size - at < want ? file_size - at : want;
      if (at + n <= pend) return;  // (a span inside the one before it: not a body's next span)
      if (first && !open_siblings()) return;
      int sl = -1;  // a slot neither the current batch nor a span ahead holds
      for (int i = 0; i < kSlots && sl < 0; i++) {
        bool used = (i == slot);
        for (const Ahead &e : aq) used = used || e.slot == i;
        if (!used) sl = i;
      }
      if (sl < 0 || !cx[sl]) return;  // (opened above)
      // the staging: the read-ahead's buffer when it holds [pend, at + n), else a spare
      bool from_ra = false;
      if (ra_valid && ra_at == pend) {
        ra_join();
        from_ra = ra_st == 0 && at + n <= pend + ra_got;
      }
      uint8_t *buf = nullptr;
      uint64_t cap = 0;
      if (from_ra) {
        buf = ra_buf;
        cap = ra_cap;
        ra_buf = nullptr;
        ra_cap = 0;
        ra_valid = false;
      } else if (!spare.empty() && spare.back().second >= kRaRoom + maxspan) {
        buf = spare.back().first;
        cap = spare.back().second;
        spare.pop_back();
      } else if (ensure_buf(&buf, &cap, kRaRoom + maxspan)) {
        return;
      }
      const uint64_t t = pend - at;
      // the span ahead of this one: its decode first (the kernels of two spans
      // sharing the GPU would delay the older span's result copies); this
      // span's H2D copy is enqueued before that wait
      std::shared_future<void> prev = first ? (early_first ? cur_done_f : std::shared_future<void>()) : aq.back().begun_f;
      aq.emplace_back();
      Ahead &e = aq.back();
      e.begun_f = e.begun.get_future().share();
      e.read_f = e.read.get_future().share();
      e.slot = sl;
      e.at = at;
      e.n = n;
      e.buf = buf;
      e.cap = cap;
      e.base = buf + kRaRoom - t;
      if (t) memcpy(buf + kRaRoom - t, pdata + (at - pat), t);
      rio_ctx *c = cx[sl];
      rio_results *r = rs[sl];
      const uint64_t need = from_ra ? 0 : at + n - pend;
      const int is_end = at + n >= file_size ? 1 : 0;
      const uint64_t lim = limit;
      const int32_t cdc = codec;
      e.th = std::thread([this, &e, c, r, need, pend, is_end, lim, cdc, prev] {
        struct Signal {
          std::promise<void> &p;
          bool on = true;
          void set() {
            if (on) p.set_value();
            on = false;
          }
          ~Signal() { set(); }
        } signal{e.begun}, read_signal{e.read};
        if (need) {  // (an io error or a short read: the batch decodes when asked for, and reports it)
          int st;
          const uint64_t got = read_full(const_cast<uint8_t *>(e.base) + (pend - e.at), need, pend, &st);
          if (st != 0 || got != need) return;
        }
        e.read_ok = true;
        read_signal.set();
        if (rio_ctx_reserve_span(c, e.n) != 0 || rio_scan_span_stage(c, e.base, e.n, cdc) != 0) return;
        if (prev.valid()) prev.wait();
        e.rc = rio_scan_span_begin(c, e.base, e.n, e.at, is_end, lim, cdc, r, &e.b);
        if (e.rc != 0) e.msg = rio_last_error();
        e.ok = true;
      });
    }
  }
  // rio_scanner_gather: staging, results and the gathered items' bytes
  uint8_t *gspan = nullptr;
  uint64_t gspan_cap = 0;
  rio_results *gres = nullptr;
  std::vector<uint8_t> gbytes;
  std::vector<uint64_t> goff;

  void set_err(const rio_error &e) {
    if (!err_set) {
      err = e;
      err_set = true;
    }
  }
  void set_errf(int32_t code, uint64_t file_off, const char *fmt, ...) {
    if (err_set) return;
    err.code = code;
    err.file_off = file_off;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err.msg, sizeof(err.msg), fmt, ap);
    va_end(ap);
    err_set = true;
  }
  // io.ReadFull at off: returns bytes read; *st 0 ok, 1 EOF, 2 unexpected EOF, 3 io error
  uint64_t read_serial(uint8_t *buf, uint64_t n, uint64_t at, int *st) const {
    uint64_t got = 0;
    while (got < n) {
      int64_t k = r.read_at(r.user, buf + got, n - got, at + got);
      if (k < 0) {
        *st = 3;
        return got;
      }
      if (k == 0) break;
      got += (uint64_t)k;
    }
    *st = (got == n) ? 0 : (got == 0 ? 1 : 2);
    return got;
  }
  // Large reads run as parallel range reads of kPiece bytes (the reader is an
  // io.ReaderAt: concurrent ReadAt calls are allowed), like the reference's
  // S3 reader's parallel chunk reads (file/s3file/file_chunk_read.go:72-102).
  static constexpr uint64_t kPiece = 16ull << 20;
  static constexpr int kReaders = 16;
  uint64_t read_full(uint8_t *buf, uint64_t n, uint64_t at, int *st) const {
    if (n < 2 * kPiece) return read_serial(buf, n, at, st);
    const uint64_t np = (n + kPiece - 1) / kPiece;
    std::vector<uint64_t> got(np, 0);
    std::vector<int> pst(np, 0);
    std::vector<std::thread> th;
    const int nt = (int)(np < (uint64_t)kReaders ? np : (uint64_t)kReaders);
    for (int t = 0; t < nt; t++)
      th.emplace_back([&, t] {
        for (uint64_t i = (uint64_t)t; i < np; i += (uint64_t)nt) {
          const uint64_t o = i * kPiece, len = n - o < kPiece ? n - o : kPiece;
          got[i] = read_serial(buf + o, len, at + o, &pst[i]);
        }
      });
    for (auto &x : th) x.join();
    uint64_t total = 0;  // the bytes read contiguously from `at`, and why they stop
    for (uint64_t i = 0; i < np; i++) {
      total += got[i];
      if (pst[i] == 3) {
        *st = 3;
        return total;
      }
      const uint64_t len = n - i * kPiece < kPiece ? n - i * kPiece : kPiece;
      if (got[i] < len) break;
    }
    *st = (total == n) ? 0 : (total == 0 ? 1 : 2);
    return total;
  }
  // pinned staging of at least n bytes, from (and back to) the ctx's pool
  int ensure_buf(uint8_t **buf, uint64_t *cap, uint64_t n) {
    if (*cap >= n) return 0;
    rio_ctx_give_buf(ctx, *buf, *cap);
    *buf = nullptr;
    *cap = 0;
    return rio_ctx_take_buf(ctx, n, buf, cap);
  }
  void give_buf(uint8_t **buf, uint64_t *cap) {
    if (*buf) rio_ctx_give_buf(ctx, *buf, *cap);
    *buf = nullptr;
    *cap = 0;
  }
  // read [at, at+n) into *buf and decode it on the GPU into *rs (ahead: the
  // read-ahead of the bytes after it starts before the GPU decode)
  int decode_into(uint8_t **buf, uint64_t *cap, rio_results *res_, uint64_t at, uint64_t n, int32_t cdc,
                  int32_t mode, uint64_t lim, rio_batch *out, bool body = false) {
    if (ensure_buf(buf, cap, n ? n : 1)) {
      memset(out, 0, sizeof(*out));
      rio_set_error(&out->err, RIO_ERR_HIP, at, "pinned allocation failed");
      out->stop = RIO_STOP_ERROR;
      return 0;
    }
    int st;
    uint64_t got = read_full(*buf, n, at, &st);
    if (st == 3) {
      memset(out, 0, sizeof(*out));
      rio_set_error(&out->err, RIO_ERR_IO, at, "read error at offset %" PRIu64, at + got);
      out->stop = RIO_STOP_ERROR;
      return 0;
    }
    const int is_end = (at + got >= file_size);
    if (body) {  // the body's span (the current slot; the bytes after it read meanwhile)
      if (early && depth > 0 && !v1 && !is_end && at + got < limit && codec != RIO_CODEC_NONE &&
          (first_block_chunks(*buf, got) >= kEarlyChunks || (ramp_c && ramp_blk == 1))) {
        // staged; the span after it begun once this copy in is done (see `early`)
        rio_ctx *c = cx[slot];
        if (c != ctx && rio_ctx_reserve_span(c, got) != 0) return -1;
        if (rio_scan_span_stage(c, *buf, got, codec) != 0) return -1;
        open_siblings();  // (the first time: while the copy in runs, not after it; a failure is seen below)
        if (rio_ctx_wait_staged(c) != 0) return -1;
        span_data = *buf;
        span_at = at;
        span_n = got;
        cur_done = std::promise<void>();
        cur_done_f = cur_done.get_future().share();
        struct Done {  // (set on every return: the span ahead's thread waits for it)
          std::promise<void> &p;
          ~Done() { p.set_value(); }
        } done_signal{cur_done};
        begin_ahead(true);
        return scan_body(*buf, got, at, out);
      }
      read_ahead(at + got);
      return scan_body(*buf, got, at, out);
    }
    if (v1 && mode == 0) return rio_scan_v1_span_mode(ctx, *buf, got, at, is_end, res_, out);
    // a header / trailer block longer than the ctx's span: the span grows to it
    if (mode != 0 && rio_ctx_reserve_span(ctx, got) != 0) return -1;
    return rio_scan_span_mode(ctx, *buf, got, at, is_end, lim, cdc, mode, res_, out);
  }
  int decode(uint64_t at, uint64_t n, int32_t cdc, int32_t mode, uint64_t lim, rio_batch *out) {
    ra_drop();
    ahead_drop();
    slot = 0;
    span_data = nullptr;
    return decode_into(&span, &span_cap, res, at, n, cdc, mode, lim, out);
  }
  // The file bytes from `end` (the span being decoded ends there), read on the
  // thread while the GPU decodes the span and the caller consumes its batch.
  // Only when the next span certainly starts there or earlier: a shard's
  // spans end once one reaches its limit.
  void read_ahead(uint64_t end) {
    if (end < file_size && end < limit) {
      // (the span after the one being decoded: index body_next + 1)
      const uint64_t left = file_size - end, want = span_size(body_next + 1);
      ra_start(end, left < want ? left : want);
    }
  }
  // the body's next span [at, at + n): from the read-ahead when it holds it
  int decode_body(uint64_t at, uint64_t n, rio_batch *out) {
    ra_join();
    const uint64_t pend = span_at + span_n;  // where the previous span ended
    if (ra_valid && span_data && ra_at == pend && at >= span_at && at <= pend && pend - at <= kRaRoom &&
        ra_st == 0 && at + n <= pend + ra_got) {
      const uint64_t t = pend - at;  // the previous span's unconsumed tail
      uint8_t *base = ra_buf + kRaRoom - t;
      if (t) memcpy(base, span_data + (at - span_at), t);
      ra_valid = false;
      std::swap(span, ra_buf);  // the batch's views will point into this buffer
      std::swap(span_cap, ra_cap);
      read_ahead(at + n);  // (into the previous span's buffer: its batch is consumed)
      const int rc = scan_body(base, n, at, out);
      span_data = base;
      span_at = at;
      span_n = n;
      return rc;
    }
    ra_valid = false;
    const int rc = decode_into(&span, &span_cap, res, at, n, codec, 0, limit, out, true);
    span_data = span;
    span_at = at;
    span_n = n;
    return rc;
  }
};

namespace {

bool has_trailer(const rio_scanner *s) {  // header.go:242-254
  for (const KV &kv : s->header) {
    if (kv.key != "trailer") continue;
    return kv.type == 1 && kv.ival;
  }
  return false;
}

void read_header(rio_scanner *s) {
  // readSpecialBlock(MagicHeader, idTransform) (scannerv2.go:260-306): the
  // header block's chunks (its first chunk's `total`), not a whole span
  const uint64_t maxspan = rio_ctx_max_span(s->ctx);
  uint64_t n = s->file_size < maxspan ? s->file_size : maxspan;
  {
    uint8_t hdr[RIO_CHUNK_HEADER_SIZE];
    int st;
    s->read_serial(hdr, sizeof(hdr), 0, &st);
    uint32_t total;
    memcpy(&total, hdr + 20, 4);
    if (st == 0 && total > 0) {
      // the header block's chunks as far as their own headers confirm them (same
      // magic and total, index i at chunk i: ChunkScanner.Scan's checks,
      // chunk.go:273-286), plus the first chunk that does not -- the GPU pass
      // reports its error as the reference does. A corrupt `total` (or a file
      // that is not recordio) thus reads one or two chunks, not the whole file
      // into the span (the span only grows to a header the headers confirm).
      uint64_t nck = 1;
      for (uint64_t i = 1; i < total; i++) {
        if (i * kCk >= s->file_size) break;
        nck = i + 1;
        if ((i + 1) * kCk > s->file_size) break;  // a truncated chunk (unexpected EOF)
        uint8_t h[RIO_CHUNK_HEADER_SIZE];
        s->read_serial(h, sizeof(h), i * kCk, &st);
        if (st != 0) break;
        uint32_t t2, ix;
        memcpy(&t2, h + 20, 4);
        memcpy(&ix, h + 24, 4);
        if (memcmp(h, hdr, 8) != 0 || t2 != total || ix != i) break;
      }
      n = nck * kCk;
      if (n > s->file_size) n = s->file_size;
    }
  }
  rio_batch b;
  if (s->decode(0, n, RIO_CODEC_NONE, 1, UINT64_MAX, &b) != 0) {
    s->set_errf(RIO_ERR_HIP, 0, "%s", rio_last_error());
    return;
  }
  char a[64];
  if (b.stop == RIO_STOP_ERROR) {
    s->set_err(b.err);
    return;
  }
  if (b.n_blocks == 0) {
    if (b.stop == RIO_STOP_MORE) {  // (n is the header block's own extent: not reached)
      s->set_errf(RIO_ERR_CAPACITY, 0, "header block larger than the GPU span (%" PRIu64 " bytes)", maxspan);
      return;
    }
    fmt_magic_v(kMagicHeaderBytes, a);
    s->set_errf(RIO_ERR_HEADER, 0, "Failed to read block %s", a);
    return;
  }
  if (b.n_items != 1) {
    s->set_errf(RIO_ERR_HEADER, 0, "Wrong # of items in header block, %" PRIu64, b.n_items);
    return;
  }
  uint64_t ilen = 0;
  const uint8_t *item = batch_item(b, 0, &ilen);
  // ParsedHeader.unmarshal (header.go:211-239)
  HeaderDecoder d{item, ilen, {}};
  KV cnt;
  int t = d.value(cnt);
  if (d.err.empty() && t != 3) d.set("Failed to read # header entries");
  if (d.err.empty()) {
    for (uint64_t i = 0; i < (uint64_t)cnt.ival; i++) {
      KV key;
      int kt = d.value(key);
      if (!d.err.empty()) break;
      if (kt != 4) {
        d.set("failed to read string key");
        break;
      }
      KV v;
      d.value(v);
      if (!d.err.empty()) break;
      v.key = key.sval;
      s->header.push_back(v);
    }
  }
  if (!d.err.empty()) {
    s->set_errf(RIO_ERR_HEADER, 0, "%s", d.err.c_str());
    return;
  }
  std::vector<const char *> vals;
  for (const KV &kv : s->header) {
    if (kv.key != "transformer") continue;
    if (kv.type != 4) {
      char v[64];
      if (kv.type == 1) snprintf(v, sizeof(v), "%s", kv.ival ? "true" : "false");
      else if (kv.type == 3) snprintf(v, sizeof(v), "%" PRIu64, (uint64_t)kv.ival);
      else snprintf(v, sizeof(v), "%" PRId64, kv.ival);
      s->set_errf(RIO_ERR_HEADER, 0, "Expect string value for key %s, but found %s", kv.key.c_str(), v);
      return;
    }
    vals.push_back(kv.sval.c_str());
  }
  rio_error e{};
  if (rio_codec_for_transformers(vals.data(), (int)vals.size(), &s->codec, &e) != 0) {
    s->set_err(e);
    return;
  }
  s->off = b.consumed;  // end of the header block
}

// LimitShard (chunk.go:198-236)
void limit_shard(rio_scanner *s, int start, int limit, int nshard) {
  const int64_t num_chunks = ((int64_t)s->file_size - (int64_t)s->off) / (int64_t)kCk;
  const double cps = (double)num_chunks / (double)nshard;
  const uint64_t start_off = s->off;
  s->off = start_off + (uint64_t)((int64_t)((double)start * cps) * (int64_t)kCk);
  s->limit = start_off + (uint64_t)((int64_t)((double)limit * cps) * (int64_t)kCk);
  if (start == 0) return;
  uint8_t hdr[RIO_CHUNK_HEADER_SIZE];
  int st;
  s->read_full(hdr, sizeof(hdr), s->off, &st);
  if (st == 1) return;  // io.EOF: ignored
  if (st == 2) {
    s->set_errf(RIO_ERR_UNEXPECTED_EOF, s->off, "unexpected EOF");
    return;
  }
  if (st == 3) {
    s->set_errf(RIO_ERR_IO, s->off, "read error");
    return;
  }
  uint32_t total, index;
  memcpy(&total, hdr + 20, 4);
  memcpy(&index, hdr + 24, 4);
  if (index == 0) return;
  if (total <= index) {
    s->set_errf(RIO_ERR_ARG, s->off, "invalid chunk header");
    return;
  }
  s->off += kCk * (uint64_t)(total - index);
}

// scanNextBatch: decode blocks from s->off until a batch with items or a stop
bool next_batch(rio_scanner *s) {
  for (;;) {
    if (s->err_set || s->done) return false;
    if (s->off >= s->limit || s->off >= s->file_size) {  // chunk.go:259-262 / EOF
      s->done = true;
      return false;
    }
    if (s->ramp_blk < 0 && s->codec != RIO_CODEC_NONE && !s->v1) {  // the body's first block: small or large
      uint8_t hdr[RIO_CHUNK_HEADER_SIZE];
      int st = 0;
      s->read_full(hdr, sizeof(hdr), s->off, &st);
      uint32_t total = 0;
      if (st == 0) memcpy(&total, hdr + 20, 4);
      s->ramp_blk = (st == 0 && total > 0 && total < rio_scanner::kEarlyChunks) ? 1 : 0;
    }
    const uint64_t want = s->span_size(s->body_next);
    uint64_t n = s->file_size - s->off;
    if (n > want) n = want;
    rio_batch &b = s->batch;
    int rc;
    s->ahead_msg.clear();
    if (s->ahead_matches(s->off, n)) {
      rc = s->take_ahead(&b);
    } else {
      s->ahead_drop();
      rc = s->decode_body(s->off, n, &b);
    }
    if (rc != 0) {
      s->set_errf(RIO_ERR_HIP, s->off, "%s", s->ahead_msg.empty() ? rio_last_error() : s->ahead_msg.c_str());
      s->finish_cur();
      return false;
    }
    s->have_batch = true;
    s->blk = 0;
    s->item = 0;
    if (s->skip && b.n_blocks > 0) {
      const uint64_t n0 = b.block_first_item[1];
      s->item = s->skip < n0 ? s->skip : n0;
    }
    s->skip = 0;
    if (b.stop == RIO_STOP_ERROR) {
      s->pending = b.err;
      s->pending_set = true;
      s->done = true;
    } else if (b.stop == RIO_STOP_EOF) {
      s->done = true;
    } else {
      if (b.consumed == 0 && s->v1 && b.err.a > n) {
        // a v1 record larger than the span (records run to MaxReadRecordSize,
        // 512 MiB): the record alone, in a staging buffer of its size
        const uint64_t need = b.err.a;
        if (s->decode(s->off, need, RIO_CODEC_NONE, 0, UINT64_MAX, &b) != 0) {
          s->set_errf(RIO_ERR_HIP, s->off, "%s", rio_last_error());
          return false;
        }
        s->span_data = s->span;
        s->span_at = s->off;
        s->span_n = need;
        if (b.stop == RIO_STOP_ERROR) {
          s->pending = b.err;
          s->pending_set = true;
          s->done = true;
        } else if (b.stop == RIO_STOP_EOF) {
          s->done = true;
        }
      }
      if (b.stop == RIO_STOP_MORE && b.consumed == 0 && s->v1) {
        s->set_errf(RIO_ERR_CAPACITY, s->off, "record at offset %" PRIu64 " larger than the GPU span",
                    s->off);
        return false;
      }
      if (b.stop == RIO_STOP_MORE && b.consumed == 0 && want < rio_ctx_max_span(s->ctx)) {
        s->ramp_off = true;  // a ramped span shorter than a block: the ctx's span
        s->finish_cur();
        continue;
      }
      if (b.stop == RIO_STOP_MORE && b.consumed == 0) {
        // a block longer than the ctx's span (the reference reads any block):
        // the span grows to the block's extent (its first chunk's total) and
        // the block decodes alone
        uint8_t hdr[RIO_CHUNK_HEADER_SIZE];
        int st;
        s->read_full(hdr, sizeof(hdr), s->off, &st);
        uint32_t total = 0;
        if (st == 0) memcpy(&total, hdr + 20, 4);
        uint64_t need = (uint64_t)total * kCk;
        if (need > s->file_size - s->off) need = s->file_size - s->off;
        if (need <= n || rio_ctx_reserve_span(s->ctx, need) != 0) {
          s->set_errf(RIO_ERR_CAPACITY, s->off, "block at offset %" PRIu64 " larger than the GPU span",
                      s->off);
          return false;
        }
        continue;  // again, at the grown span
      }
      s->off += b.consumed;
      s->body_next++;
      // the spans after this one, begun while its result copies come back and
      // the caller consumes it (the read-ahead of the bytes after the last one
      // ahead -- or after this span -- started when that span was begun)
      s->begin_ahead();
    }
    if (s->finish_cur() != 0) {
      s->set_errf(RIO_ERR_HIP, s->off, "%s", rio_last_error());
      return false;
    }
    if (b.n_items > 0) return true;
    if (s->pending_set) {
      s->set_err(s->pending);
      s->pending_set = false;
      return false;
    }
  }
}

}  // namespace

extern "C" {

static int64_t memory_read_at(void *user, uint8_t *buf, uint64_t n, uint64_t off) {
  const rio_memory *m = static_cast<const rio_memory *>(user);
  if (off >= m->size) return 0;
  const uint64_t k = n < m->size - off ? n : m->size - off;
  memcpy(buf, m->data + off, k);
  return (int64_t)k;
}

rio_reader rio_memory_reader(const rio_memory *m) {
  rio_reader r;
  r.user = const_cast<rio_memory *>(m);
  r.read_at = memory_read_at;
  r.size = m ? (int64_t)m->size : 0;
  return r;
}

int rio_codec_for_transformers(const char *const *values, int n, int32_t *codec, rio_error *err) {
  // registry.getTransformers (registry.go:51-73): split on the first space
  int found = 0;
  int32_t c = RIO_CODEC_NONE;
  for (int i = 0; i < n; i++) {
    const char *v = values[i];
    const char *sp = strchr(v, ' ');
    size_t len = sp ? (size_t)(sp - v) : strlen(v);
    if (len == 5 && strncmp(v, "flate", 5) == 0) c = RIO_CODEC_FLATE;
    else if (len == 4 && strncmp(v, "zstd", 4) == 0) c = RIO_CODEC_ZSTD;
    else {  // not decoded here: the reference registry may hold it (registry.go:166)
      rio_set_error(err, RIO_ERR_FALLBACK, 0, "Transformer %s not found", v);
      return RIO_ERR_FALLBACK;
    }
    found++;
  }
  if (found > 4) {  // longer chains than RIO_CODEC_CHAIN encodes
    rio_set_error(err, RIO_ERR_FALLBACK, 0, "transformer chain of %d: decode with recordio.NewScanner", found);
    return RIO_ERR_FALLBACK;
  }
  if (found > 1) {  // a chain, untransformed in reverse order (registry.go:121-146)
    int32_t codes = 0;
    for (int i = 0; i < n; i++) {
      const int32_t ci = strncmp(values[i], "flate", 5) == 0 ? RIO_CODEC_FLATE : RIO_CODEC_ZSTD;
      codes |= ci << (2 * i);
    }
    *codec = RIO_CODEC_CHAIN(found, codes);
    return 0;
  }
  *codec = c;
  return 0;
}

rio_scanner *rio_scanner_new(rio_ctx *ctx, const rio_reader *r, int start, int limit, int nshard) {
  rio_scanner *s = new rio_scanner();
  s->ctx = ctx;
  s->depth = ctx ? rio_ctx_spans_ahead(ctx) : 0;
  if (s->depth > rio_scanner::kSlots - 1) s->depth = rio_scanner::kSlots - 1;
  if (const char *e = getenv("RIO_SCAN_EARLY")) s->early = atoi(e) != 0;
  if (const char *e = getenv("RIO_SPAN_RAMP_C")) s->ramp_c = atoi(e) != 0;
  if (const char *e = getenv("RIO_SPAN_RAMP")) s->ramp_steps = std::min(std::max(atoi(e), 0), 6);
  if (const char *e = getenv("RIO_SPAN_RAMP_MIN")) s->ramp_min = strtoull(e, nullptr, 0);
  s->res = ctx ? rio_ctx_take_results(ctx) : rio_results_new();
  s->cx[0] = ctx;
  s->rs[0] = s->res;
  s->shard_start = start;
  s->shard_limit = limit;
  s->shard_n = nshard;
  s->r = *r;
  s->file_size = r->size < 0 ? 0 : (uint64_t)r->size;
  // NewShardScanner (scannerv2.go:211-235)
  uint8_t magic[8];
  int st;
  s->read_full(magic, 8, 0, &st);
  if (st != 0) {
    s->error_scanner = true;
    if (st == 2) s->set_errf(RIO_ERR_UNEXPECTED_EOF, 0, "unexpected EOF");
    if (st == 3) s->set_errf(RIO_ERR_IO, 0, "read error");
    return s;
  }
  if (start >= limit || limit > nshard || start < 0 || nshard <= 0) {
    s->error_scanner = true;
    s->set_errf(RIO_ERR_ARG, 0, "invalid sharding [%d,%d) of %d", start, limit, nshard);
    return s;
  }
  if (memcmp(magic, kMagicHeaderBytes, 8) != 0) {
    if (start != 0 || limit != 1 || nshard != 1) {
      s->error_scanner = true;
      s->set_errf(RIO_ERR_ARG, 0, "legacy record IOs do not support sharding");
      return s;
    }
    // newLegacyScannerAdapter (scannerv2.go:232): Header() empty, Trailer() nil
    if (!ctx) {
      s->error_scanner = true;
      s->set_errf(RIO_ERR_ARG, 0, "nil rio_ctx");
      return s;
    }
    s->v1 = true;
    s->off = 0;
    s->limit = UINT64_MAX;
    return s;
  }
  if (!ctx) {
    s->set_errf(RIO_ERR_ARG, 0, "nil rio_ctx");
    return s;
  }
  read_header(s);
  if (s->err_set) return s;
  limit_shard(s, start, limit, nshard);
  return s;
}

int rio_scanner_scan(rio_scanner *s) {
  if (!s || s->error_scanner) return 0;
  for (;;) {
    if (s->have_batch && s->item < s->batch.n_items) {
      const rio_batch &b = s->batch;
      // a sticky error set meanwhile (Trailer, Seek) ends the scan at the end of
      // the current block: the reference only re-checks it in scanNextBlock
      // (scannerv2.go:363-368, 390-395)
      if (s->err_set && s->item >= b.block_first_item[s->blk + 1]) return 0;
      while (s->item >= b.block_first_item[s->blk + 1]) s->blk++;
      const uint64_t first = b.block_first_item[s->blk];
      s->cur = batch_item(b, s->item, &s->cur_len);
      s->cur_block = b.block_file_off[s->blk];
      s->cur_item = (int64_t)(s->item - first);
      s->item++;
      return 1;
    }
    if (s->pending_set) {
      s->set_err(s->pending);
      s->pending_set = false;
    }
    if (!next_batch(s)) return 0;
  }
}

int rio_scanner_get(rio_scanner *s, const uint8_t **data, uint64_t *len) {
  if (!s || !s->cur) return 0;
  *data = s->cur;
  *len = s->cur_len;
  return 1;
}

int64_t rio_scanner_next_batch(rio_scanner *s, const uint8_t **data, uint64_t *lens, int64_t max) {
  int64_t n = 0;
  while (n < max) {
    // do not cross into a new GPU batch: views stay valid for the whole call
    if (n > 0 && !(s->have_batch && s->item < s->batch.n_items)) break;
    if (s && !s->error_scanner && !s->err_set && s->have_batch && s->item < s->batch.n_items) {
      // the current batch's next items in one pass (what rio_scanner_scan would
      // return one by one: a view per item, then the scanner positioned on the
      // last one -- its block and index for Location)
      const rio_batch &b = s->batch;
      const uint64_t k = std::min<uint64_t>(b.n_items - s->item, (uint64_t)(max - n));
      for (uint64_t i = 0; i < k; i++) data[n + i] = batch_item(b, s->item + i, &lens[n + i]);
      const uint64_t last = s->item + k - 1;
      while (last >= b.block_first_item[s->blk + 1]) s->blk++;
      s->cur = data[n + k - 1];
      s->cur_len = lens[n + k - 1];
      s->cur_block = b.block_file_off[s->blk];
      s->cur_item = (int64_t)(last - b.block_first_item[s->blk]);
      s->item = last + 1;
      n += (int64_t)k;
      continue;
    }
    if (!rio_scanner_scan(s)) break;
    data[n] = s->cur;
    lens[n] = s->cur_len;
    n++;
  }
  return n;
}

int rio_scanner_err(rio_scanner *s, rio_error *err) {
  if (!s || !s->err_set) return 0;
  if (err) *err = s->err;
  return s->err.code ? s->err.code : -1;
}

int rio_scanner_header_len(rio_scanner *s) { return s ? (int)s->header.size() : 0; }

int rio_scanner_header_kv(rio_scanner *s, int i, const char **key, int32_t *type, int64_t *ival,
                          const uint8_t **sval, uint64_t *slen) {
  if (!s || i < 0 || i >= (int)s->header.size()) return 0;
  const KV &kv = s->header[(size_t)i];
  *key = kv.key.c_str();
  *type = kv.type;
  *ival = kv.ival;
  *sval = (const uint8_t *)kv.sval.data();
  *slen = kv.sval.size();
  return 1;
}

// Trailer (scannerv2.go:316-342) + ReadLastBlock (chunk.go:380-407). The
// trailer is read into its own staging and result buffers, so the current
// batch -- and the scan position -- are untouched, like the reference's
// deferred Seek(curOff) (scannerv2.go:320-321).
int rio_scanner_trailer(rio_scanner *s, const uint8_t **data, uint64_t *len) {
  if (!s || s->error_scanner || !has_trailer(s)) return 0;
  if (s->err_set) return 0;
  if (s->file_size < kCk) {
    s->set_errf(RIO_ERR_TRAILER, 0, "bytes.Reader.Seek: negative position");
    return 0;
  }
  uint8_t *tspan = nullptr;
  uint64_t tcap = 0;
  rio_results *tres = rio_ctx_take_results(s->ctx);
  struct Cleanup {
    rio_scanner *s;
    uint8_t *&p;
    uint64_t &cap;
    rio_results *r;
    ~Cleanup() {
      s->give_buf(&p, &cap);
      rio_ctx_give_results(s->ctx, r);
    }
  } cleanup{s, tspan, tcap, tres};
  const uint64_t last = s->file_size - kCk;
  rio_batch b;
  // the last chunk alone: its size/CRC first (readChunk), then its magic
  if (s->decode_into(&tspan, &tcap, tres, last, kCk, RIO_CODEC_NONE, 3, UINT64_MAX, &b) != 0) {
    s->set_errf(RIO_ERR_HIP, last, "%s", rio_last_error());
    return 0;
  }
  if (b.stop == RIO_STOP_ERROR) {
    s->set_err(b.err);
    return 0;
  }
  uint8_t hdr[RIO_CHUNK_HEADER_SIZE];
  int st;
  s->read_full(hdr, sizeof(hdr), last, &st);
  if (memcmp(hdr, kMagicTrailerBytes, 8) != 0) {
    char a[64];
    fmt_magic_v(hdr, a);
    s->set_errf(RIO_ERR_TRAILER, last, "Missing magic trailer; found %s", a);
    return 0;
  }
  uint32_t total, index;
  memcpy(&total, hdr + 20, 4);
  memcpy(&index, hdr + 24, 4);
  uint64_t start = last;
  if (!(index == 0 && total == 1)) {
    const uint64_t back = ((uint64_t)index + 1) * kCk;
    if (back > s->file_size) {
      s->set_errf(RIO_ERR_TRAILER, 0, "bytes.Reader.Seek: negative position");
      return 0;
    }
    start = s->file_size - back;
    if (start >= s->limit) {  // ChunkScanner.Scan honours the shard limit
      s->set_errf(RIO_ERR_TRAILER, start, "Failed to read trailer");
      return 0;
    }
  }
  if (s->decode_into(&tspan, &tcap, tres, start, s->file_size - start, s->codec, 2, UINT64_MAX, &b) != 0) {
    s->set_errf(RIO_ERR_HIP, start, "%s", rio_last_error());
    return 0;
  }
  if (b.stop == RIO_STOP_ERROR) {
    s->set_err(b.err);
    return 0;
  }
  if (b.n_blocks == 0) {
    s->set_errf(RIO_ERR_TRAILER, start, "Failed to read trailer");
    return 0;
  }
  if (b.n_items != 1) {
    s->set_errf(RIO_ERR_TRAILER, start, "Expect exactly one trailer item, but found %" PRIu64, b.n_items);
    return 0;
  }
  uint64_t tlen = 0;
  const uint8_t *t0 = batch_item(b, 0, &tlen);
  s->trailer.assign(t0, t0 + tlen);
  *data = s->trailer.data();
  *len = s->trailer.size();
  return 1;
}

void rio_scanner_seek(rio_scanner *s, uint64_t block, int64_t item) {
  if (!s || s->error_scanner) return;
  // v1 Seek (legacyscanner.go:67-82): seekRaw + sc.Reset clear the record
  // scanner's error (InternalScan's); the adapter's own (Unpack, magic,
  // location) stays
  if (s->v1 && s->err_set && s->err.code == RIO_ERR_V1_RECORD) {
    s->err_set = false;
    memset(&s->err, 0, sizeof(s->err));
  }
  if (s->v1 && !s->err_set && (int64_t)block < 0) {
    s->set_errf(RIO_ERR_ARG, block, "bytes.Reader.Seek: negative position");
  }
  if (s->err_set) {  // scanNextBlock clears rawItems, then fails on the sticky error
    s->have_batch = false;
    s->cur = nullptr;
    return;
  }
  // Seek (scannerv2.go:348-361): restart at the block, skip `item` items
  s->ra_drop();
  s->ahead_drop();
  s->have_batch = false;
  s->pending_set = false;
  s->done = false;
  s->off = block;
  s->cur = nullptr;
  if (!next_batch(s)) return;
  const uint64_t nfirst = s->batch.block_first_item[1] - s->batch.block_first_item[0];
  if (item < 0 || (uint64_t)item >= nfirst) {
    s->set_errf(RIO_ERR_LOCATION, block, "Invalid location {Block:%" PRIu64 " Item:%" PRId64
                "}, block has only %" PRIu64 " items", block, item, nfirst);
  }
  s->item = (uint64_t)(item < 0 ? 0 : item);
}

void rio_scanner_location(rio_scanner *s, uint64_t *block, int64_t *item) {
  *block = s ? s->cur_block : 0;
  *item = s ? s->cur_item : 0;
}

int rio_scanner_version(rio_scanner *s) { return (s && s->v1) ? 1 : 2; }

// Gather: the items at n ItemLocations, as n Seek + Scan +
// Get calls would return them (scannerv2.go:348-361, 390-403), with the
// distinct blocks read and decoded as one batch: each block's chunks (its
// first chunk header gives their count, chunk.go:31-53) are staged back to
// back and run through the pipeline at once. A location whose block did not
// decode cleanly in the batch, or whose item index is out of range, is
// resolved exactly as Seek + Scan on a scanner of the same file and shard
// (its error is the one Seek / Scan would set). The scan position is
// untouched. Views stay valid until the next gather on this scanner.
int64_t rio_scanner_gather(rio_scanner *s, const uint64_t *blocks, const int64_t *items, int64_t n,
                           const uint8_t **data, uint64_t *lens, rio_error *err) {
  rio_error err_local;
  if (!err) err = &err_local;
  memset(err, 0, sizeof(*err));
  if (!s || n < 0 || (n > 0 && (!blocks || !items || !data || !lens))) return -1;
  if (s->error_scanner || s->err_set) {  // a scanner that failed to open: its error
    *err = s->err;
    return 0;
  }
  if (!s->gres) s->gres = rio_ctx_take_results(s->ctx);
  s->gbytes.clear();
  s->goff.assign((size_t)n, UINT64_MAX);
  std::vector<uint64_t> uniq(blocks, blocks + n);
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  // per distinct block: its extent, then (after decoding) its items
  struct Blk {
    uint64_t off = 0, bytes = 0, span_at = 0;
    bool ok = false;
    std::vector<uint64_t> item_pos;  // offsets into gbytes, and lengths
    std::vector<uint64_t> item_len;
  };
  std::vector<Blk> bl(uniq.size());
  for (size_t i = 0; i < uniq.size(); i++) {
    bl[i].off = uniq[i];
    uint8_t hdr[RIO_CHUNK_HEADER_SIZE];
    int st;
    // the exact path reports these; a block at or past the shard's limit is EOF
    // there (ChunkScanner.Scan, chunk.go:259-262), not an item
    if (s->v1 || uniq[i] % kCk != 0 || uniq[i] >= s->file_size || uniq[i] >= s->limit) continue;
    s->read_full(hdr, sizeof(hdr), uniq[i], &st);
    if (st != 0) continue;
    uint32_t total, index;
    memcpy(&total, hdr + 20, 4);
    memcpy(&index, hdr + 24, 4);
    if (index != 0 || total == 0) continue;
    const uint64_t bytes = (uint64_t)total * kCk;
    if (uniq[i] + bytes > s->file_size || bytes > rio_ctx_max_span(s->ctx)) continue;
    bl[i].bytes = bytes;
  }
  // batches of blocks up to the ctx's span capacity
  const uint64_t maxspan = rio_ctx_max_span(s->ctx);
  size_t i0 = 0;
  while (i0 < bl.size()) {
    uint64_t used = 0;
    size_t i1 = i0;
    while (i1 < bl.size() && (bl[i1].bytes == 0 || used + bl[i1].bytes <= maxspan)) used += bl[i1++].bytes;
    if (used) {
      if (s->ensure_buf(&s->gspan, &s->gspan_cap, used)) {
        rio_set_error(err, RIO_ERR_HIP, 0, "pinned allocation failed");
        return 0;
      }
      uint64_t at = 0;
      bool io_ok = true;
      for (size_t k = i0; k < i1 && io_ok; k++) {
        if (!bl[k].bytes) continue;
        int st;
        s->read_full(s->gspan + at, bl[k].bytes, bl[k].off, &st);
        if (st != 0) bl[k].bytes = 0;  // short read: the exact path reports it
        bl[k].span_at = at;
        at += bl[k].bytes;
      }
      rio_batch b;
      if (at && rio_scan_span_mode(s->ctx, s->gspan, at, 0, 1, UINT64_MAX, s->codec, 0, s->gres, &b) != 0) {
        rio_set_error(err, RIO_ERR_HIP, 0, "%s", rio_last_error());
        return 0;
      }
      if (at) {
        // blocks decoded before the batch's first error (if any) are good
        size_t k = i0;
        for (uint64_t j = 0; j < b.n_blocks; j++) {
          const uint64_t so = b.block_file_off[j];
          while (k < i1 && (bl[k].bytes == 0 || bl[k].span_at < so)) k++;
          if (k >= i1 || bl[k].span_at != so) break;  // a block the batch split: not trusted
          Blk &B = bl[k];
          const uint64_t f = b.block_first_item[j], e = b.block_first_item[j + 1];
          for (uint64_t it = f; it < e; it++) {
            uint64_t len = 0;
            const uint8_t *p = batch_item(b, it, &len);
            B.item_pos.push_back(s->gbytes.size());
            B.item_len.push_back(len);
            s->gbytes.insert(s->gbytes.end(), p, p + len);
          }
          B.ok = true;  // (the batch's blocks end before its first error)
        }
      }
    }
    i0 = i1 > i0 ? i1 : i0 + 1;
  }
  // the locations, in order
  for (int64_t i = 0; i < n; i++) {
    const size_t k = (size_t)(std::lower_bound(uniq.begin(), uniq.end(), blocks[i]) - uniq.begin());
    const Blk &B = bl[k];
    if (B.ok && items[i] >= 0 && (uint64_t)items[i] < B.item_pos.size()) {
      s->goff[(size_t)i] = B.item_pos[(size_t)items[i]];
      lens[i] = B.item_len[(size_t)items[i]];
      continue;
    }
    // exact: Seek + Scan + Get on a scanner of the same file and shard
    rio_scanner *t = rio_scanner_new(s->ctx, &s->r, s->shard_start, s->shard_limit, s->shard_n);
    rio_error te{};
    bool got = false;
    if (!rio_scanner_err(t, &te)) {
      rio_scanner_seek(t, blocks[i], items[i]);
      if (!rio_scanner_err(t, &te) && rio_scanner_scan(t)) {
        const uint8_t *p = nullptr;
        uint64_t len = 0;
        rio_scanner_get(t, &p, &len);
        s->goff[(size_t)i] = s->gbytes.size();
        lens[i] = len;
        s->gbytes.insert(s->gbytes.end(), p, p + len);
        got = true;
      } else if (!rio_scanner_err(t, &te)) {  // Scan found nothing (EOF / a trailer): no item
        rio_set_error(&te, RIO_ERR_LOCATION, blocks[i], "no item at {Block:%" PRIu64 " Item:%" PRId64 "}",
                      blocks[i], items[i]);
      }
    }
    rio_scanner_finish(t, nullptr);
    if (!got) {
      *err = te;
      for (int64_t q = 0; q < i; q++) data[q] = s->gbytes.data() + s->goff[(size_t)q];
      return i;
    }
  }
  for (int64_t q = 0; q < n; q++) data[q] = s->gbytes.data() + s->goff[(size_t)q];
  return n;
}

int rio_scanner_finish(rio_scanner *s, rio_error *err) {
  if (!s) return 0;
  int rc = rio_scanner_err(s, err);
  s->ra_drop();
  s->ahead_drop();
  for (rio_ctx *c : s->cx) rio_scan_span_end(c);  // (nothing of this scanner's left in flight)
  if (s->ctx) {  // buffers and result sets back to the ctx's pools
    s->give_buf(&s->span, &s->span_cap);
    s->give_buf(&s->ra_buf, &s->ra_cap);
    for (auto &b : s->spare) s->give_buf(&b.first, &b.second);
    s->give_buf(&s->gspan, &s->gspan_cap);
    rio_ctx_give_results(s->ctx, s->gres);
    rio_ctx_give_results(s->ctx, s->res);
    for (int i = 1; i < rio_scanner::kSlots; i++) rio_ctx_give_results(s->ctx, s->rs[i]);
  } else {
    rio_results_free(s->res);
  }
  delete s;
  return rc;
}

}  // extern "C"
