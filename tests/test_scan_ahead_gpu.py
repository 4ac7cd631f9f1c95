"""The scanner's spans ahead (scanner.cpp begin_ahead): with a file of many
spans, spans i + 1 and i + 2 are decoded on the ctx's sibling contexts (each
begun on a thread of its own; the second from a host prediction of where span
i + 1 stops) while batch i's result copies come back, and batches rotate over
the three contexts. Every record, error and location must be what the oracle's
scanner (scannerv2.go's restated) gives, whichever context decoded it: many
spans for each codec, a corrupt chunk in a later span, wrong predictions,
Seek in the middle of a scan, shards, and the byte accounting across the
contexts."""
import random
import struct
import zlib

import pytest

from conftest import oracle_has_zstd

pytestmark = pytest.mark.gpu

SPAN = 8 * 32768  # small spans: a few MB file is dozens of them


def _file(trs, n, seed):
    from base_amd.recordio.writer import WriterOpts, write_file
    rng = random.Random(seed)
    recs = [rng.randbytes(rng.choice([0, 5, 300, 2000])) * rng.choice([1, 1, 6]) for _ in range(n)]
    return recs, write_file(recs, WriterOpts(Transformers=trs, MaxItems=23), trailer=b"AHEAD")


def _scan(data, ctx, start=0, limit=1, nshard=1):
    from base_amd.recordio import gpu
    sc = gpu.NewShardScanner(data, gpu.ScannerOpts(), start, limit, nshard, ctx=ctx)
    items = []
    while sc.Scan():
        items.append(sc.Get())
    e = sc.Finish()
    return items, ("" if e is None else str(e))


@pytest.mark.parametrize("trs", [[], ["flate"], ["zstd"], ["zstd", "flate"]])
def test_many_spans_every_record(oracle, trs):
    from base_amd.recordio import gpu
    if "zstd" in trs and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    recs, data = _file(trs, 2500, 1)
    ref = oracle.scan(data)
    assert ref.err == "" and ref.items == recs
    ctx = gpu.Context(0, max_span_bytes=SPAN)
    try:
        for _ in range(2):  # (the second scan reuses the sibling and the pools)
            items, err = _scan(data, ctx)
            assert err == "" and items == recs, trs
        st = ctx.stats()
        body = len(data) - 32768  # the spans cover the body at least once per scan
        assert st["spans"] >= 2 * (body // SPAN) and st["h2d_bytes"] >= 2 * body
    finally:
        ctx.close()


@pytest.mark.parametrize("trs", [[], ["flate"], ["zstd"]])
def test_corrupt_later_span_matches_oracle(oracle, trs):
    """A bad chunk deep in the file (CRC left stale, or fixed so the codec or the
    packed parse must notice): the same records before it and the same error."""
    from base_amd.recordio import gpu
    if "zstd" in trs and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    recs, data = _file(trs, 2500, 2)
    nck = len(data) // 32768
    rng = random.Random(3)
    ctx = gpu.Context(0, max_span_bytes=SPAN)
    try:
        for trial in range(6):
            b = bytearray(data)
            c = rng.randrange(nck // 2, nck - 2)
            o = c * 32768
            size = struct.unpack_from("<I", b, o + 16)[0]
            if size == 0:
                continue
            b[o + 28 + rng.randrange(size)] ^= 1 << rng.randrange(8)
            if trial % 2:
                struct.pack_into("<I", b, o + 8, zlib.crc32(bytes(b[o + 12:o + 28 + size])))
            d = bytes(b)
            ref = oracle.scan(d, read_trailer=False)
            items, err = _scan(d, ctx)
            assert err == ref.err and items == ref.items, (trs, trial, c)
    finally:
        ctx.close()


@pytest.mark.parametrize("depth", [0, 1, 2])
@pytest.mark.parametrize("trs", [[], ["flate"], ["zstd"]])
def test_wrong_span_prediction_matches_oracle(oracle, trs, depth):
    """The second span ahead starts where the host reads the span before it will
    stop (its last chunk header): a chunk header whose index or total was
    rewritten (CRC fixed, so only the block structure is wrong) makes that
    prediction wrong, or the GPU's extent differ from it. The spans begun on it
    are dropped: the same records and error as the oracle's, at every depth of
    spans ahead (RIO_CFG_SPANS_AHEAD). A rewritten total or index also makes blocks
    overlap (a block start inside another block's chunks): the decode of the
    overlapping block must stay inside its own regions (kernels.hip k_chunk_apply)."""
    from base_amd.recordio import gpu
    if "zstd" in trs and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    recs, data = _file(trs, 2500, 6)
    nck = len(data) // 32768
    rng = random.Random(7)
    ctx = gpu.Context(0, max_span_bytes=SPAN, spans_ahead=depth)
    try:
        for trial in range(12):
            b = bytearray(data)
            # the last chunk of a span (the predicted one) or any chunk
            c = rng.randrange(nck // 4, nck - 2)
            if trial % 2 == 0:
                c = c - c % 8 + 7 if c - c % 8 + 7 < nck - 1 else c
            o = c * 32768
            field = 20 + 4 * rng.randrange(2)  # total or index: + 1, 2 or 5, or index 0
            v = struct.unpack_from("<I", b, o + field)[0] + rng.choice([1, 2, 5])
            struct.pack_into("<I", b, o + field, 0 if field == 24 and trial % 3 == 2 else v)
            struct.pack_into("<I", b, o + 8, zlib.crc32(bytes(b[o + 12:o + 28 + struct.unpack_from("<I", b, o + 16)[0]])))
            d = bytes(b)
            ref = oracle.scan(d, read_trailer=False)
            items, err = _scan(d, ctx)
            assert err == ref.err and items == ref.items, (trs, trial, c, field)
    finally:
        ctx.close()


def test_seek_mid_scan_and_shards(oracle):
    """Seek while a span ahead is in flight, then scan on; shards with small spans."""
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import ItemLocation
    recs, data = _file(["flate"], 3000, 4)
    ref = oracle.scan(data)
    ctx = gpu.Context(0, max_span_bytes=SPAN)
    try:
        sc = gpu.NewScanner(data, ctx=ctx)
        for _ in range(700):  # some spans in: the next one has been begun ahead
            assert sc.Scan()
        for i in (2900, 10, 1500, 2999, 0):
            sc.Seek(ItemLocation(*ref.locations[i]))
            got = []
            while len(got) < 300 and sc.Scan():
                got.append(sc.Get())
            assert got == recs[i:i + 300], i
        assert sc.Finish() is None
        parts = []
        for s in range(4):
            items, err = _scan(data, ctx, s, s + 1, 4)
            assert err == ""
            parts.extend(items)
        assert parts == recs
    finally:
        ctx.close()


@pytest.mark.parametrize("trs", [[], ["zstd"]])
def test_scan_batch_views_and_location(oracle, trs):
    """rio_scanner_next_batch (ScanBatch) hands a batch's items over in one pass:
    the same items as Scan/Get, mixed with plain Scans, odd batch sizes, across
    spans, and Location afterwards is the last item's (the reference's)."""
    from base_amd.recordio import gpu
    if "zstd" in trs and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    recs, data = _file(trs, 2500, 5)
    ref = oracle.scan(data)
    ctx = gpu.Context(0, max_span_bytes=SPAN)
    try:
        sc = gpu.NewScanner(data, ctx=ctx)
        got, sizes, i = [], [7, 1000, 1, 333, 1 << 16], 0
        while True:
            if i % 3 == 2:  # a plain Scan between batches
                if not sc.Scan():
                    break
                got.append(sc.Get())
            else:
                part = sc.ScanBatch(sizes[i % len(sizes)])
                if not part:
                    break
                got.extend(part)
            loc = sc.Location()
            assert (loc.Block, loc.Item) == tuple(ref.locations[len(got) - 1]), (i, len(got))
            i += 1
        assert sc.Finish() is None and got == recs
    finally:
        ctx.close()


class _SlowFile:
    """A file object whose reads past the first span return late, so that the
    threads of spans ahead are still reading when the scanner plans the next
    span (scanner.cpp begin_ahead waits for the read of the span before it)."""

    def __init__(self, data, delay):
        import io
        self._b = io.BytesIO(data)
        self.delay = delay

    def seek(self, off, whence=0):
        return self._b.seek(off, whence)

    def tell(self):
        return self._b.tell()

    def read(self, n=-1):
        import time
        if self._b.tell() > SPAN:
            time.sleep(self.delay)
        return self._b.read(n)


@pytest.mark.parametrize("trs", [[], ["flate"]])
def test_slow_reader_spans_ahead(oracle, trs):
    """Spans ahead over a reader that is slow to return: every record as the
    oracle's, twice on one ctx (the second scan's staging buffers are recycled
    ones that still hold the first scan's chunks)."""
    from base_amd.recordio import gpu
    recs, data = _file(trs, 1500, 7)
    ctx = gpu.Context(0, max_span_bytes=SPAN)
    try:
        for _ in range(2):
            sc = gpu.NewScanner(_SlowFile(data, 0.01), ctx=ctx)
            items = []
            while sc.Scan():
                items.append(sc.Get())
            e = sc.Finish()
            assert e is None and items == recs, trs
    finally:
        ctx.close()


@pytest.mark.parametrize("trs,max_items", [([], 23), (["flate"], 23), (["zstd"], 23), ([], 4000), (["flate"], 4000)])
def test_span_ramp(oracle, trs, max_items, monkeypatch):
    """The span ramp (scanner.cpp span_size): a body's first spans smaller than
    the ctx's, forced here at small sizes (RIO_SPAN_RAMP_MIN=0, 3 steps: 4, 4,
    8, then 16-chunk spans at a 16-chunk ctx span). Every record and the error
    as the oracle's. Compressed bodies of small blocks (MaxItems = 23) ramp and
    stage each next span early too; with MaxItems = 4000 an uncompressed block
    is longer than the first spans, which turns the ramp off (the ctx's span
    from there on), and a compressed one is large, so it is not ramped."""
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import WriterOpts, write_file
    if "zstd" in trs and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    rng = random.Random(11)
    recs = [rng.randbytes(rng.choice([0, 5, 300, 2000])) * rng.choice([1, 1, 6]) for _ in range(2500)]
    data = write_file(recs, WriterOpts(Transformers=trs, MaxItems=max_items), trailer=b"RAMP")
    monkeypatch.setenv("RIO_SPAN_RAMP", "3")
    monkeypatch.setenv("RIO_SPAN_RAMP_MIN", "0")
    ctx = gpu.Context(0, max_span_bytes=16 * 32768)
    try:
        for shard in [(0, 1, 1), (1, 3, 4)]:
            want = oracle.scan(data, *shard)
            items, err = _scan(data, ctx, *shard)
            assert err == want.err and items == want.items, (trs, max_items, shard)
    finally:
        ctx.close()
