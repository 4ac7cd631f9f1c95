"""BASELINE.json configs at full size on the GPU (pytest -m gpu), plus the
reference's randomized sharding tests restated (recordio/v2_test.go:458-591).

- C1 (configs[0]): 1M x 256 B at the writer's default MaxItems = 16384 (16,385 per block)
  (130-chunk blocks, 32 KiB varint headers: the general parser's path), every
  record byte-exact against the generator and against the oracle's scan;
- C4 (configs[3]): the zstd workload's base file (tools/c4_data.py: record sizes
  log-uniform 64 B-64 KiB, >= 1 MiB blocks, level 5), records by SHA-256 and
  lengths against the generator, a few blocks against the oracle;
- TestRandomLargeWrites (v2_test.go:574-591): 100k records, 10 shards, and
  nshard = 1e9 with stride 1e8: the shards concatenate to the input and the
  largest holds 8,000 < n < 12,000 records -- bounds from the reference test;
- TestV2Random-shaped cases (v2_test.go:544-572): up to 2,000 shards, none and
  zstd, Seek to every record's ItemLocation.

The reference generates its records with Go's math/rand; these use Python's
random with the same shapes (lengths rnd.Intn(datasize)+1 of 'A'+Intn(64)
characters, flush probability, trailer "Trailer"), so the bounds, not the exact
byte streams, are the reference's.
"""
import ctypes
import hashlib
import io
import os
import random
import sys

import numpy as np
import pytest

from conftest import ROOT, oracle_has_zstd

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _views_to_array(b, span, nrec, rec_len):
    """Materialise a host batch of fixed-size records (rio_scan_span views)."""
    off = np.ctypeslib.as_array(b.item_off, shape=(b.n_items,)).copy()
    ln = np.ctypeslib.as_array(b.item_len, shape=(b.n_items,))
    assert np.all(ln == rec_len)
    side = np.frombuffer(ctypes.string_at(b.records, b.records_len), dtype=np.uint8) if b.records_len else None
    in_rec = (off >> np.uint64(63)).astype(bool)
    off = (off & np.uint64((1 << 63) - 1)).astype(np.int64)
    ar = np.arange(rec_len, dtype=np.int64)
    out = np.empty((nrec, rec_len), dtype=np.uint8)
    for lo in range(0, nrec, 100000):
        hi = min(nrec, lo + 100000)
        idx = off[lo:hi, None] + ar
        m = in_rec[lo:hi]
        blk = np.empty((hi - lo, rec_len), dtype=np.uint8)
        blk[~m] = span[idx[~m]]
        if m.any():
            blk[m] = side[idx[m]]
        out[lo:hi] = blk
    return out


def test_full_size_c1(oracle):
    """configs[0] at full size: 1,000,000 x 256 B, MaxItems 16384 -> 62 blocks of
    16,385 items (MaxItems + 1, writerv2.go:315, 366-368) in 130 chunks (last
    block 515 items in 5 chunks), SURVEY.md §8(a)."""
    import bench
    from base_amd.recordio import gpu
    data, nrec = bench.make_c1_file()
    assert len(data) == 260046848
    ctx = gpu.Context(0, max_span_bytes=len(data) + 32768)
    b = ctx.scan_span(data[32768:], file_off=32768, is_file_end=True)
    assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
    assert b.n_items == nrec and b.n_blocks == 62
    first = np.ctypeslib.as_array(b.block_first_item, shape=(b.n_blocks + 1,)).astype(np.int64)
    assert np.all(np.diff(first)[:-1] == 16385) and first[-1] - first[-2] == 515
    span = np.frombuffer(data, dtype=np.uint8)[32768:]
    got = _views_to_array(b, span, nrec, 256)
    recs = bench.c2_records()
    assert np.array_equal(got, recs)
    ctx.close()
    # the oracle reads the same file to the same records (and through the scanner API)
    ref = oracle.scan(data)
    assert ref.err == "" and len(ref.items) == nrec
    assert b"".join(ref.items) == recs.tobytes()
    sc = gpu.NewScanner(data, ctx=gpu.Context(0, max_span_bytes=64 << 20))
    h = hashlib.sha256()
    n = 0
    while True:
        got = sc.ScanBatch(1 << 16)
        if not got:
            break
        for r in got:
            h.update(r)
        n += len(got)
    assert sc.Finish() is None and n == nrec
    assert h.hexdigest() == hashlib.sha256(recs.tobytes()).hexdigest()


def test_c4_base_file(oracle):
    """configs[3]'s base file through the device path and the scanner API."""
    from base_amd.recordio import gpu
    from base_amd.recordio.codecs import have_zstd
    if not have_zstd() or not oracle_has_zstd(oracle):
        pytest.skip("libzstd not present to write the fixture")
    import c4_data
    import torch
    data, nblk, nrec, rec_bytes = c4_data.make_file(24 << 20)
    want = c4_data.all_records(nblk)
    assert len(want) == nrec and sum(map(len, want)) == rec_bytes
    body = data[32768:]
    dev = torch.frombuffer(bytearray(body), dtype=torch.uint8).to("cuda:0")
    ctx = gpu.Context(0, max_span_bytes=len(body) + 32768)
    b = ctx.scan_device(dev.data_ptr(), len(body), file_off=32768, is_file_end=True, codec=gpu.RIO_CODEC_ZSTD)
    assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
    got = gpu.device_batch_items(b, body)
    assert [len(x) for x in got] == [len(x) for x in want]
    assert hashlib.sha256(b"".join(got)).digest() == hashlib.sha256(b"".join(want)).digest()
    ctx.close()
    # a few blocks against the oracle, file-shaped (header + block)
    hdr = data[:32768]
    pos, blocks = 32768, []
    while pos < len(data):
        total = int.from_bytes(data[pos + 20:pos + 24], "little")
        blocks.append(data[pos:pos + total * 32768])
        pos += total * 32768
    assert len(blocks) == nblk
    for k in (0, nblk // 2, nblk - 1):
        ref = oracle.scan(hdr + blocks[k])
        assert ref.err == ""
        sc = gpu.NewScanner(hdr + blocks[k])
        items = []
        while sc.Scan():
            items.append(sc.Get())
        assert sc.Finish() is None and items == ref.items


def random_string(n, rnd):
    return bytes(65 + rnd.randrange(64) for _ in range(n))


def generate_random_recordio(rnd, flush_p, n_records, datasize, transformers=()):
    """generateRandomRecordio (v2_test.go:458-481): KeyTrailer header, random
    flushes, trailer "Trailer", the ItemLocation index of every record."""
    from base_amd.recordio.writer import Writer, WriterOpts
    buf = io.BytesIO()
    index = {}
    w = Writer(buf, WriterOpts(Transformers=list(transformers),
                               Index=lambda loc, v: index.__setitem__(bytes(v), loc)))
    w.AddHeader("trailer", True)
    items = []
    for _ in range(n_records):
        d = random_string(rnd.randrange(datasize) + 1, rnd)
        w.Append(d)
        items.append(d)
        if rnd.random() < flush_p:
            w.Flush()
    w.SetTrailer(b"Trailer")
    w.Finish()
    return buf.getvalue(), items, index


def do_sharded_reads(data, stride, nshard, items, ctx):
    """doShardedReads (v2_test.go:483-509): shards [s, s+stride) of nshard, each
    with Trailer() == "Trailer"; returns the largest shard's record count."""
    from base_amd.recordio import gpu
    expected = list(items)
    pos = 0
    max_shard = 0
    for shard in range(0, nshard, stride):
        limit = min(shard + stride, nshard)
        sc = gpu.NewShardScanner(data, gpu.ScannerOpts(), shard, limit, nshard, ctx=ctx)
        assert sc.Trailer() == b"Trailer", (shard, nshard, sc.Err())
        n = 0
        while sc.Scan():
            assert sc.Get() == expected[pos], (pos, shard, nshard)
            pos += 1
            n += 1
        assert sc.Finish() is None
        max_shard = max(max_shard, n)
    assert pos == len(expected)
    return max_shard


def test_random_large_writes(gpu_ctx):
    """TestRandomLargeWrites (v2_test.go:574-591)."""
    rnd = random.Random(0)
    data, items, _ = generate_random_recordio(rnd, 0.01, 100000, 1024)
    m = do_sharded_reads(data, 1, 10, items, gpu_ctx)
    assert 8000 < m < 12000, m
    n = 1000000000  # a large absolute shard count: rounding of the float64 shard math
    m = do_sharded_reads(data, n // 10, n, items, gpu_ctx)
    assert 8000 < m < 12000, m


@pytest.mark.parametrize("codec", ["", "zstd"])
@pytest.mark.parametrize("flush_p,nshard,maxrecords,datasize", [
    (0.001, 2000, 2000, 10 << 10),  # blocks big enough that shards straddle them
    (0.1, 1000, 2000, 30),
    (1.0, 3, 2000, 30),
    (0.0, 2, 2000, 30),
    (0.001, 2000, 1, 30),           # many shards, a single record
    (0.001, 2000, 0, 30),           # an empty file
])
def test_v2_random(gpu_ctx, oracle, codec, flush_p, nshard, maxrecords, datasize):
    """doRandomTest (v2_test.go:511-542) as TestV2Random runs it (544-572)."""
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import ItemLocation
    if codec == "zstd" and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    rnd = random.Random(0)
    n = rnd.randrange(maxrecords) + 1 if maxrecords > 0 else 0
    data, items, index = generate_random_recordio(rnd, flush_p, n, datasize, [codec] if codec else [])
    do_sharded_reads(data, 1, nshard, items, gpu_ctx)
    sc = gpu.NewScanner(data, ctx=gpu_ctx)
    for v in items[:300]:
        loc = index[v]
        sc.Seek(ItemLocation(loc.Block, loc.Item))
        assert sc.Err() is None
        assert sc.Scan() and sc.Get() == v
    sc.Finish()


def test_c5_shaped_file_set(gpu_ctx, oracle):
    """C5 (configs[4]) in miniature: trailer-indexed flate files of FASTQ-like
    records (tools/c5_data.py, 2 MiB of records each instead of 64 MiB). Each
    file's trailer index (read through the GPU scanner's Trailer, ReadLastBlock
    from EOF) equals the writer's block offsets; the file bodies placed back to
    back on the device decode in one rio_scan_device launch to every file's
    records in file-set order; and a two-rank index split of one file
    (shard.split_blocks) covers its records exactly once."""
    import torch
    import c5_data
    from base_amd.recordio import gpu, shard
    rb = 2 << 20
    files = [c5_data.make_base(k, record_bytes=rb, workers=4) for k in range(3)]
    want, bodies = [], []
    for k, (data, nrec, rec_bytes, offsets) in enumerate(files):
        recs = c5_data.base_records(k, record_bytes=rb)
        assert len(recs) == nrec
        sc = gpu.NewScanner(data, ctx=gpu_ctx)
        assert c5_data.parse_index(sc.Trailer()) == offsets
        got = []
        while sc.Scan():
            got.append(sc.Get())
        assert sc.Finish() is None and got == recs
        want.extend(recs)
        bodies.append(data[offsets[0]:shard.trailer_offset(data)])
        if k == 0:  # the index split: rank r decodes blocks [lo, hi) of the body
            body_end = shard.trailer_offset(data)
            parts = []
            for r in range(2):
                lo, hi = shard.split_blocks(offsets, body_end, r, 2)
                if hi > lo:
                    b = gpu_ctx.scan_span(data[lo:hi], file_off=lo, is_file_end=True, codec=gpu.RIO_CODEC_FLATE)
                    assert b.err.code == 0, b.err.msg
                    parts.extend(gpu.batch_items(b))
            assert parts == recs
        ref = oracle.scan(data)
        assert ref.err == "" and ref.items == recs
    span = b"".join(bodies)
    dev = torch.frombuffer(bytearray(span), dtype=torch.uint8).to("cuda:0")
    b = gpu_ctx.scan_device(dev.data_ptr(), len(span), file_off=0, is_file_end=True, codec=gpu.RIO_CODEC_FLATE)
    assert b.err.code == 0, b.err.msg
    assert gpu.device_batch_items(b, span) == want


def test_c5_segments_scan(gpu_ctx, oracle):
    """rio_scan_device_segments_async over C5-shaped file bodies back to back:
    every block's file (block_segment) and its offset in that file
    (block_file_off == the file's trailer index, ItemLocation.Block), the
    records of each file through the item_end output; a corrupt chunk in the
    second file stops the batch there, reported in that file's coordinates
    (err_segment, err.file_off) with the first file's records delivered."""
    import torch
    import c5_data
    from base_amd.recordio import gpu, shard
    rb = 1 << 20
    files = [c5_data.make_base(k, record_bytes=rb, workers=4) for k in range(3)]
    recs = [c5_data.base_records(k, record_bytes=rb) for k in range(3)]
    bodies, ends, foffs = [], [], []
    for data, nrec, rec_bytes, offsets in files:
        bodies.append(data[offsets[0]:shard.trailer_offset(data)])
        ends.append(sum(map(len, bodies)))
        foffs.append(offsets[0])
    span = b"".join(bodies)
    dev = torch.frombuffer(bytearray(span), dtype=torch.uint8).to("cuda:0")
    ctx = gpu.Context(0, max_span_bytes=len(span) + 32768, item_end=True)
    try:
        ctx.scan_device_segments_async(dev.data_ptr(), len(span), ends, foffs, gpu.RIO_CODEC_FLATE)
        b = ctx.sync()
        assert b.err.code == 0 and b.stop == gpu.RIO_STOP_EOF and b.err_segment == -1, b.err.msg
        nb = int(b.n_blocks)
        seg = np.frombuffer(gpu.dev_to_host(ctypes.cast(b.block_segment, ctypes.c_void_p).value, 8 * nb),
                            dtype=np.uint64)
        boff = np.frombuffer(gpu.dev_to_host(ctypes.cast(b.block_file_off, ctypes.c_void_p).value, 8 * nb),
                             dtype=np.uint64)
        first = np.frombuffer(gpu.dev_to_host(ctypes.cast(b.block_first_item, ctypes.c_void_p).value, 8 * (nb + 1)),
                              dtype=np.uint64)
        items = gpu.device_batch_items(b, span)
        for k, (data, nrec, rec_bytes, offsets) in enumerate(files):
            sel = np.nonzero(seg == k)[0]
            assert boff[sel].tolist() == offsets  # ItemLocation.Block of every block of file k
            got = items[int(first[sel[0]]):int(first[sel[-1] + 1])]
            assert got == recs[k]
        # a corrupt chunk in file 1: the error in file 1's coordinates
        bad = bytearray(span)
        at = ends[0] + 5 * 32768 + 1000
        bad[at] ^= 0x40
        dev.copy_(torch.frombuffer(bad, dtype=torch.uint8))
        ctx.scan_device_segments_async(dev.data_ptr(), len(span), ends, foffs, gpu.RIO_CODEC_FLATE)
        b = ctx.sync()
        assert b.stop == gpu.RIO_STOP_ERROR and b.err_segment == 1
        assert b.err.file_off == foffs[1] + 5 * 32768
        data1 = files[1][0]
        ref = oracle.scan(bytes(data1[:foffs[1]]) + bytes(bad[ends[0]:ends[1]]), read_trailer=False)
        assert b.err.msg.decode() == ref.err
        items = gpu.device_batch_items(b, bytes(bad))
        assert items == recs[0] + ref.items
    finally:
        ctx.close()
