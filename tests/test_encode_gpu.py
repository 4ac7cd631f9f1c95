"""Writer encode path on the GPU (rio_encode): the chunk
stream must be byte-identical to the writer restatement (base_amd/recordio/
writer.py: writerv2.go + chunk.go) for the none transformer -- the writer is
deterministic there -- and scan back through both the GPU scanner and the
oracle to the records written."""
import io
import random

import numpy as np
import pytest

from base_amd.recordio import format as F
from base_amd.recordio.writer import WriterOpts, write_file, Writer


def gpu_write(records, opts, header=(), trailer=None, flush_every=0, ctx=None, batch_bytes=64 << 20):
    from base_amd.recordio.gpu_writer import GpuWriter
    import dataclasses
    buf = io.BytesIO()
    opts = dataclasses.replace(opts)
    if trailer is not None:
        opts.KeyTrailer = True
    w = GpuWriter(buf, opts, ctx=ctx, batch_bytes=batch_bytes)
    for k, v in header:
        w.AddHeader(k, v)
    for i, r in enumerate(records):
        w.Append(r)
        if flush_every and i % flush_every == flush_every - 1:
            w.Flush()
    if trailer is not None:
        w.SetTrailer(trailer)
    assert w.Finish() is None
    return buf.getvalue()


def records(rng, n, sizes=(0, 1, 7, 100, 256, 3000, 40000)):
    return [bytes(rng.getrandbits(8) for _ in range(rng.choice(sizes))) if rng.random() < 0.3 else
            rng.randbytes(rng.choice(sizes)) for _ in range(n)]


@pytest.mark.gpu
def test_encode_matches_writer(gpu_ctx, oracle):
    rng = random.Random(3)
    cases = [
        (records(rng, 0), WriterOpts(), {}),
        (records(rng, 1), WriterOpts(), {}),
        (records(rng, 200), WriterOpts(MaxItems=7), {}),
        (records(rng, 500), WriterOpts(MaxItems=1), {"trailer": b"T" * 70000}),
        (records(rng, 300, (0,)), WriterOpts(MaxItems=100), {}),  # empty items only
        (records(rng, 120, (33000, 70000)), WriterOpts(MaxItems=3), {}),  # items over chunks
        (records(rng, 700), WriterOpts(MaxItems=64), {"flush_every": 13}),
        (records(rng, 400), WriterOpts(SkipHeader=True, MaxItems=50), {}),
        (records(rng, 50), WriterOpts(MaxItems=5), {"header": [("k", "v"), ("n", -3), ("b", False)]}),
        (records(rng, 5000, (0, 1, 2, 200)), WriterOpts(), {}),  # one block of 5000 items
    ]
    for i, (recs, opts, kw) in enumerate(cases):
        want = write_file(recs, opts, header=kw.get("header", ()), trailer=kw.get("trailer"),
                          flush_every=kw.get("flush_every", 0))
        got = gpu_write(recs, opts, header=kw.get("header", ()), trailer=kw.get("trailer"),
                        flush_every=kw.get("flush_every", 0), ctx=gpu_ctx, batch_bytes=1 << 16)
        assert got == want, i
        if not opts.SkipHeader:
            ref = oracle.scan(got)
            assert ref.err == "" and ref.items == recs, i


@pytest.mark.gpu
def test_encode_index_locations(gpu_ctx):
    """IndexFunc (writerv2.go:40-43): every item's ItemLocation, as the writer reports it."""
    from base_amd.recordio import gpu
    rng = random.Random(4)
    recs = records(rng, 400)
    got_w, got_g = [], []
    opts = WriterOpts(MaxItems=9, Index=lambda loc, v: got_w.append((loc, v)))
    write_file(recs, opts, flush_every=31)
    opts = WriterOpts(MaxItems=9, Index=lambda loc, v: got_g.append((loc, v)))
    data = gpu_write(recs, opts, flush_every=31, ctx=gpu_ctx, batch_bytes=1 << 12)
    assert got_g == got_w and len(got_g) == len(recs)
    sc = gpu.NewScanner(data, ctx=gpu_ctx)
    for loc, v in got_g[::17]:
        sc.Seek(loc)
        assert sc.Scan() and sc.Get() == v
    assert sc.Finish() is None


@pytest.mark.gpu
def test_encode_c2_round_trip(gpu_ctx):
    """The C2 record set (1e6 x 256 B, 253 per block): encode equals the bench's
    C2 file byte for byte, and the GPU scan of the encoded bytes gives the records."""
    import bench
    from base_amd.recordio import gpu
    recs = bench.c2_records()
    want, n = bench.make_c2_file()
    ctx = gpu.Context(0, max_span_bytes=len(want) + (1 << 20))
    try:
        hdr, _ = ctx.encode([F.marshal_header([])], 1, gpu.RIO_BLOCK_HEADER)
        ends = np.arange(1, n + 1, dtype=np.uint64) * 256
        body, boff = ctx.encode_arrays(recs.tobytes(), ends, 253)
        assert hdr + body == want
        assert boff[:3] == [0, 65536, 131072] and len(boff) == 3953
        b = ctx.scan_span(body, file_off=len(hdr), is_file_end=True)
        assert b.stop == gpu.RIO_STOP_EOF and b.n_items == n
    finally:
        ctx.close()


@pytest.mark.gpu
def test_encode_past_ctx_span(gpu_ctx):
    """rio_encode grows its own buffers: a stream longer than the ctx's span
    encodes (no RIO_ERR_CAPACITY), and a scanner on that small ctx reads a block
    longer than its span (the span grows to the block, as the reference reads
    any block)."""
    from base_amd.recordio import gpu
    ctx = gpu.Context(0, max_span_bytes=1 << 20)  # 32 chunks
    try:
        data, boff = ctx.encode([b"x" * 200000] * 10, 1)  # 10 blocks x 7 chunks
        assert len(data) == 70 * 32768 and boff == [7 * 32768 * i for i in range(10)]
        recs = [bytes([i]) * 150000 for i in range(20)]  # one block of 3 MB
        got = gpu_write(recs, WriterOpts(), ctx=ctx)
        assert got == write_file(recs, WriterOpts())
        sc = gpu.NewScanner(got, ctx=ctx)
        items = []
        while sc.Scan():
            items.append(sc.Get())
        assert sc.Finish() is None and items == recs
    finally:
        ctx.close()


@pytest.mark.gpu
def test_writer_block_larger_than_default_span(gpu_ctx):
    """16,385 items of 20 KiB at the default MaxItems: one block of 336 MB, more
    than the default ctx's 256 MiB span. The writer encodes it, and
    it scans back through a 64 MiB-span ctx."""
    import hashlib
    import os
    from base_amd.recordio import gpu
    blob = os.urandom(16385 * 20480)
    recs = [blob[i * 20480:(i + 1) * 20480] for i in range(16385)]
    buf = io.BytesIO()
    from base_amd.recordio.gpu_writer import GpuWriter
    w = GpuWriter(buf, WriterOpts(KeyTrailer=True))
    for r in recs:
        w.Append(r)
    w.SetTrailer(b"end")
    assert w.Finish() is None
    data = buf.getvalue()
    sc = gpu.NewScanner(data, ctx=gpu_ctx)
    assert sc.Trailer() == b"end"
    h, n = hashlib.sha256(), 0
    while True:
        got = sc.ScanBatch(1 << 14)
        if not got:
            break
        for r in got:
            assert len(r) == 20480
            h.update(r)
        n += len(got)
    assert sc.Finish() is None and n == 16385
    assert h.digest() == hashlib.sha256(blob).digest()


@pytest.mark.gpu
def test_writer_config_errors(gpu_ctx):
    """Transformer configs as the reference's factories parse them: a config
    that is not a decimal int fails NewWriter (strconv.Atoi's error, nothing
    written); a flate level outside [-2, 9] fails the first transformed block
    (klauspost flate.NewWriter's error: the header is written, the block is not),
    and the error sticks (Err, Finish)."""
    from base_amd.recordio.gpu_writer import GpuWriter
    for cfg in ("flate x", "zstd 1.5", "flate  3"):
        buf = io.BytesIO()
        w = GpuWriter(buf, WriterOpts(Transformers=[cfg]), ctx=gpu_ctx)
        w.Append(b"abc")
        arg = cfg.split(" ", 1)[1]
        assert str(w.Err()) == 'strconv.Atoi: parsing "%s": invalid syntax' % arg
        assert str(w.Finish()) == str(w.Err()) and buf.getvalue() == b""
    for lvl in (10, -3, 42):
        buf = io.BytesIO()
        w = GpuWriter(buf, WriterOpts(Transformers=["flate %d" % lvl], MaxItems=2), ctx=gpu_ctx)
        assert w.Err() is None
        for i in range(7):
            w.Append(b"item %d" % i)
        msg = "flate: invalid compression level %d: want value in range [-2, 9]" % lvl
        assert str(w.Finish()) == msg
        assert len(buf.getvalue()) == 32768  # the header block alone
    for cfg in ("flate -2", "flate +9", "flate 0", "zstd -7", "zstd 30"):
        recs = [b"r%d" % i * 40 for i in range(100)]
        got = gpu_write(recs, WriterOpts(Transformers=[cfg], MaxItems=13), ctx=gpu_ctx)
        from base_amd.recordio import gpu
        sc = gpu.NewScanner(got, ctx=gpu_ctx)
        items = []
        while sc.Scan():
            items.append(sc.Get())
        assert sc.Finish() is None and items == recs, cfg


def fastq_records(rng, n):
    """C3-style text records: compressible, with repeats at all distances."""
    bases = b"ACGT"
    out = []
    for i in range(n):
        seq = bytes(rng.choice(bases) for _ in range(rng.randrange(50, 150)))
        qual = bytes(rng.choice(b"FFFF:,") for _ in range(len(seq)))
        out.append(b"@read%d/1\n" % i + seq + b"\n+\n" + qual + b"\n")
    return out


@pytest.mark.gpu
def test_encode_flate_decodes(gpu_ctx, oracle):
    """flate blocks from the GPU encoder (dynamic Huffman by default, fixed
    Huffman at level 1, both with greedy matches; level 0 stored blocks)
    decode -- GPU scanner, the oracle's Go-semantics inflater, zlib -- to the
    records written; text compresses, better with dynamic trees."""
    import zlib
    from base_amd.recordio import gpu
    rng = random.Random(5)
    sets = [fastq_records(rng, 3000), records(rng, 300), [b""] * 50, [b"x" * 100000] * 3,
            [bytes([i % 7]) * rng.randrange(0, 600) for i in range(2000)]]
    sets.append([bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40000))) for _ in range(20)])
    sets.append([b"ACGT"[rng.randrange(4):][:1] * rng.randrange(1, 70000) for _ in range(12)])
    for level in ("flate", "flate 0", "flate 1", "flate 5"):
        for i, recs in enumerate(sets):
            data = gpu_write(recs, WriterOpts(Transformers=[level], MaxItems=rng.choice([1, 50, 1000])),
                             trailer=b"trail" * 3, ctx=gpu_ctx, batch_bytes=1 << 18)
            ref = oracle.scan(data)
            assert ref.err == "" and ref.items == recs and ref.trailer == b"trail" * 3, (level, i)
            sc = gpu.NewScanner(data, ctx=gpu_ctx)
            got = []
            while sc.Scan():
                got.append(sc.Get())
            assert sc.Finish() is None and got == recs, (level, i)
    # every block's payload is a raw DEFLATE stream zlib inflates to the packed payload
    recs = fastq_records(rng, 500)
    sizes = {}
    for level in ("flate 1", "flate"):
        sizes[level] = _zlib_check_blocks(gpu_write(recs, WriterOpts(Transformers=[level], MaxItems=99), ctx=gpu_ctx),
                                          recs)
    assert sizes["flate"] < sizes["flate 1"], sizes  # dynamic trees beat the fixed code on FASTQ text


def _zlib_check_blocks(data, recs):
    import zlib
    off, k, comp, plain = 32768, 0, 0, 0
    while off < len(data):
        total = int.from_bytes(data[off + 20:off + 24], "little")
        pay = b"".join(data[off + c * 32768 + 28: off + c * 32768 + 28 +
                            int.from_bytes(data[off + c * 32768 + 16:off + c * 32768 + 20], "little")]
                       for c in range(total))
        blk = recs[k * 100:(k + 1) * 100]
        assert zlib.decompress(pay, -15) == F.packed_block_payload(blk)
        comp += len(pay)
        plain += len(F.packed_block_payload(blk))
        off += total * 32768
        k += 1
    assert k == 5
    assert comp < 0.75 * plain, (comp, plain)  # greedy matches + Huffman on FASTQ-like text
    return comp


@pytest.mark.gpu
def test_encode_zstd_decodes(gpu_ctx, oracle):
    """zstd blocks from the GPU encoder (one frame per block payload: raw
    literals, predefined sequence codes, <= 16 KiB blocks, raw blocks where
    they do not shrink) decode -- GPU scanner, the oracle's libzstd-semantics
    decoder, libzstd itself (the library DataDog/zstd wraps) -- to the records
    written; text compresses."""
    from base_amd.recordio import gpu
    from base_amd.recordio.codecs import have_zstd, zstd_decompress_ref
    from conftest import oracle_has_zstd
    if not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    rng = random.Random(6)
    sets = [fastq_records(rng, 3000), records(rng, 300), [b""] * 50, [b"x" * 100000] * 3,
            [bytes([i % 7]) * rng.randrange(0, 600) for i in range(2000)], [rng.randbytes(70000)]]
    for tr in ("zstd", "zstd 5"):
        for i, recs in enumerate(sets):
            data = gpu_write(recs, WriterOpts(Transformers=[tr], MaxItems=rng.choice([1, 50, 1000])),
                             trailer=b"trail" * 3, ctx=gpu_ctx, batch_bytes=1 << 18)
            ref = oracle.scan(data)
            assert ref.err == "" and ref.items == recs and ref.trailer == b"trail" * 3, (tr, i)
            sc = gpu.NewScanner(data, ctx=gpu_ctx)
            got = []
            while sc.Scan():
                got.append(sc.Get())
            assert sc.Finish() is None and got == recs, (tr, i)
    if not have_zstd():
        return
    # every block's payload is a zstd frame libzstd decodes to the packed payload
    recs = fastq_records(rng, 800)
    data = gpu_write(recs, WriterOpts(Transformers=["zstd"], MaxItems=199), ctx=gpu_ctx)
    off, k, comp, plain = 32768, 0, 0, 0
    while off < len(data):
        total = int.from_bytes(data[off + 20:off + 24], "little")
        pay = b"".join(data[off + c * 32768 + 28: off + c * 32768 + 28 +
                            int.from_bytes(data[off + c * 32768 + 16:off + c * 32768 + 20], "little")]
                       for c in range(total))
        blk = recs[k * 200:(k + 1) * 200]
        want = F.packed_block_payload(blk)
        assert zstd_decompress_ref(pay, len(want) + 1) == want
        comp += len(pay)
        plain += len(want)
        off += total * 32768
        k += 1
    assert k == 4
    assert comp < 0.75 * plain, (comp, plain)


def _undo_payload(pay, chain):
    """A block payload with the chain's stages undone last first (zlib raw
    inflate, libzstd) -- the reference's GetUntransformer order (registry.go:121-146)."""
    import zlib
    from base_amd.recordio.codecs import zstd_decompress_ref
    for t in reversed(chain):
        if t.split(" ")[0] == "flate":
            pay = zlib.decompress(pay, -15)
        else:
            pay = zstd_decompress_ref(pay, 64 * len(pay) + (1 << 20))
    return pay


@pytest.mark.gpu
def test_encode_chains_decode(gpu_ctx, oracle):
    """Write-side transformer chains (registry.go:75-111, applied in order at
    writerv2.go:432-441): 2- and 3-stage files written on the GPU (one
    RIO_CODEC_CHAIN encode per batch) read back identical through the oracle and
    the GPU scanner; every block payload is the stages applied in order (zlib /
    libzstd undo them, last first)."""
    from base_amd.recordio import gpu
    from base_amd.recordio.codecs import have_zstd
    from conftest import oracle_has_zstd
    if not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    rng = random.Random(11)
    sets = [fastq_records(rng, 2000), records(rng, 200), [b""] * 30, [b"y" * 90000] * 3]
    chains = (["zstd", "flate"], ["flate 1", "zstd", "flate"], ["flate", "flate 0"], ["zstd 5", "zstd"],
              ["flate", "zstd", "flate 1", "zstd"])
    for chain in chains:
        for i, recs in enumerate(sets):
            data = gpu_write(recs, WriterOpts(Transformers=chain, MaxItems=rng.choice([1, 60, 700])),
                             trailer=b"chain-trailer", ctx=gpu_ctx, batch_bytes=1 << 18)
            ref = oracle.scan(data)
            assert ref.err == "" and ref.items == recs and ref.trailer == b"chain-trailer", (chain, i)
            sc = gpu.NewScanner(data, ctx=gpu_ctx)
            got = []
            while sc.Scan():
                got.append(sc.Get())
            assert sc.Finish() is None and got == recs, (chain, i)
    if not have_zstd():
        return
    recs = fastq_records(rng, 600)
    for chain in (["zstd", "flate"], ["flate 1", "zstd", "flate"]):
        data = gpu_write(recs, WriterOpts(Transformers=chain, MaxItems=149), ctx=gpu_ctx)
        off, k = 32768, 0
        while off < len(data):
            total = int.from_bytes(data[off + 20:off + 24], "little")
            pay = b"".join(data[off + c * 32768 + 28: off + c * 32768 + 28 +
                                int.from_bytes(data[off + c * 32768 + 16:off + c * 32768 + 20], "little")]
                           for c in range(total))
            assert _undo_payload(pay, chain) == F.packed_block_payload(recs[k * 150:(k + 1) * 150]), (chain, k)
            off += total * 32768
            k += 1
        assert k == 4


@pytest.mark.gpu
def test_writer_transformer_list_errors(gpu_ctx):
    """NewWriter's transformer errors go to err (writerv2.go:318-320), not raised:
    a name the registry does not hold ("Transformer %s not found",
    registry.go:58, the whole value), a config that does not parse, anywhere in
    a chain; nothing is written. A chain's flate stage with a level outside
    [-2, 9] fails the first transformed block (the header is written)."""
    from base_amd.recordio.gpu_writer import GpuWriter
    for tl, msg in ((["snappy"], "Transformer snappy not found"),
                    (["zstd", "lz4 3"], "Transformer lz4 3 not found"),
                    (["flate", "zstd x"], 'strconv.Atoi: parsing "x": invalid syntax')):
        buf = io.BytesIO()
        w = GpuWriter(buf, WriterOpts(Transformers=tl), ctx=gpu_ctx)
        assert str(w.Err()) == msg
        w.Append(b"abc")
        assert str(w.Finish()) == msg and buf.getvalue() == b"", tl
    buf = io.BytesIO()
    w = GpuWriter(buf, WriterOpts(Transformers=["zstd", "flate 12"], MaxItems=3), ctx=gpu_ctx)
    assert w.Err() is None
    for i in range(10):
        w.Append(b"item %d" % i)
    assert str(w.Finish()) == "flate: invalid compression level 12: want value in range [-2, 9]"
    assert len(buf.getvalue()) == 32768
