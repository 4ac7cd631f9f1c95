"""GPU zstd decoder stress parity (pytest -m gpu): k_zstd (codec_zstd.hip) on
inputs chosen for its edge paths -- compression levels, frame parameters
(checksum, content size, window), several and skippable frames per recordio
block, raw / RLE / multi-block frames, decode-region retries -- bit-exact
against the records the writer compressed, and for corrupt frames against the
CPU oracle's error text (recordiozstd.go:67-78 -> libzstd ZSTD_decompress)."""
import random

import pytest

from conftest import oracle_has_zstd

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(gpu_lib):
    from base_amd.recordio import gpu
    from base_amd.recordio.codecs import have_zstd
    if not have_zstd():
        pytest.skip("libzstd not present to write the fixtures")
    c = gpu.Context(0, max_span_bytes=64 << 20)
    yield c
    c.close()


def scan_all(data, ctx):
    from base_amd.recordio import gpu
    sc = gpu.NewScanner(data, ctx=ctx)
    items = []
    while sc.Scan():
        items.append(sc.Get())
    err = sc.Err()
    sc.Finish()
    return items, ("" if err is None else str(err))


def mixed_records(seed, n, big=3000):
    rng = random.Random(seed)
    words = [bytes(rng.choice(b"ACGTN@+\n") for _ in range(rng.randrange(1, 12))) for _ in range(200)]
    out = []
    for _ in range(n):
        k = rng.random()
        if k < 0.3:
            out.append(bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 400))))
        elif k < 0.9:
            out.append(b"".join(rng.choice(words) for _ in range(rng.randrange(0, 80))))
        else:
            out.append(bytes([rng.randrange(256)]) * rng.randrange(0, big))
    return out


def zstd_file(blocks, header_transformer="zstd"):
    """A recordio file whose body blocks carry the given compressed payloads
    verbatim (header names the zstd transformer)."""
    from base_amd.recordio import format as F
    hdr = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", header_transformer)])]))
    return hdr + b"".join(F.chunk_block(F.MAGIC_PACKED, b) for b in blocks)


def skippable(payload):
    import struct
    return struct.pack("<II", 0x184D2A53, len(payload)) + payload


@pytest.mark.parametrize("level", [1, 3, 5, 9, 19])
def test_levels(ctx, level):
    from base_amd.recordio.writer import write_file, WriterOpts
    recs = mixed_records(level, 900)
    data = write_file(recs, WriterOpts(Transformers=["zstd %d" % level], MaxItems=120))
    items, err = scan_all(data, ctx)
    assert err == "" and items == recs


@pytest.mark.parametrize("checksum", [False, True])
@pytest.mark.parametrize("content_size", [False, True])
@pytest.mark.parametrize("window_log", [0, 10, 17, 23])
def test_frame_parameters(ctx, checksum, content_size, window_log):
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import zstd_compress_ex
    blocks, want = [], []
    for i in range(4):
        recs = mixed_records(window_log * 10 + i, 150 + 200 * i)
        blocks.append(zstd_compress_ex(F.packed_block_payload(recs), 3 + 4 * i, checksum, content_size, window_log))
        want.extend(recs)
    items, err = scan_all(zstd_file(blocks), ctx)
    assert err == "" and items == want


def test_several_and_skippable_frames(ctx):
    # ZSTD_decompress decodes every frame of its input back to back and skips
    # skippable frames; a recordio block's payload is their concatenation
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import zstd_compress_ex
    recs = mixed_records(5, 400)
    payload = F.packed_block_payload(recs)
    cuts = [0, 1, 777, len(payload) // 2, len(payload) - 5, len(payload)]
    parts = []
    for k, (a, b) in enumerate(zip(cuts, cuts[1:])):
        parts.append(zstd_compress_ex(payload[a:b], 1 + 2 * k, checksum=k % 2 == 0, content_size=k % 3 != 0))
        if k % 2:
            parts.append(skippable(bytes(range(k * 7))))
    blob = b"".join(parts)
    items, err = scan_all(zstd_file([skippable(b"lead") + blob, blob]), ctx)
    assert err == "" and items == recs + recs


def test_raw_rle_and_multiblock_frames(ctx):
    from base_amd.recordio.writer import write_file, WriterOpts
    rng = random.Random(8)
    recs = [bytes(rng.getrandbits(8) for _ in range(300000)),  # raw blocks
            b"\x07" * 700000,                                    # RLE blocks
            bytes(rng.getrandbits(8) for _ in range(5)) * 90000,  # rep-offset matches across 128 KiB blocks
            b""]
    data = write_file(recs, WriterOpts(Transformers=["zstd 19"]))
    items, err = scan_all(data, ctx)
    assert err == "" and items == recs


def test_long_distance_matches(ctx):
    # matches reaching back MiB-far inside one frame (window 2^23)
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import zstd_compress_ex
    rng = random.Random(12)
    a = bytes(rng.getrandbits(8) for _ in range(1 << 20))
    recs = [a, bytes(rng.getrandbits(8) for _ in range(3 << 20)), a[:500000], a[600000:]]
    comp = zstd_compress_ex(F.packed_block_payload(recs), 19, True, True, 23)
    items, err = scan_all(zstd_file([comp]), ctx)
    assert err == "" and items == recs


def test_high_ratio_blocks_retry(ctx):
    # decoded size ~ 30,000x the compressed bytes: beyond the first decode
    # region bound (8x); sized from the frame's content size, or without one by
    # the host's growing retry
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import zstd_compress_ex
    recs = [b"\0" * (3 << 20), b"ab" * 100000, b""]
    payload = F.packed_block_payload(recs)
    blocks = [zstd_compress_ex(payload, 5, False, True), zstd_compress_ex(payload, 5, True, False)]
    items, err = scan_all(zstd_file(blocks), ctx)
    assert err == "" and items == recs + recs


def test_async_scan_grows_zstd_scratch(gpu_lib):
    # an asynchronous device scan whose zstd scratch regions (k_zstd_size: the
    # literal area holds every block's literals, RLE blocks included) outgrow the
    # context's first allocation (5x the span): rio_sync grows it and runs the
    # span again, and the records come back whole -- on the first scan of a
    # fresh context and on the next one
    import torch
    from base_amd.recordio import format as F
    from base_amd.recordio import gpu
    from base_amd.recordio.codecs import have_zstd, zstd_compress_ex
    if not have_zstd():
        pytest.skip("libzstd not present to write the fixtures")
    recs = [b"\0" * (3 << 20), b"ab" * 100000, bytes(range(256)) * 64, b""]
    payload = F.packed_block_payload(recs)
    blocks = [zstd_compress_ex(payload, 5, False, True), zstd_compress_ex(payload, 1, True, False)]
    data = zstd_file(blocks)
    body = data[32768:]
    dev = torch.frombuffer(bytearray(body), dtype=torch.uint8).to("cuda:0")
    ctx = gpu.Context(0, max_span_bytes=len(body) + 32768, item_end=True)
    try:
        for _ in range(2):
            ctx.scan_device_async(dev.data_ptr(), len(body), 32768, gpu.RIO_CODEC_ZSTD)
            b = ctx.sync()
            assert b.err.code == 0 and b.stop == gpu.RIO_STOP_EOF, b.err.msg
            assert gpu.device_batch_items(b, body) == recs + recs
    finally:
        ctx.close()


def test_many_small_blocks(ctx, oracle):
    from base_amd.recordio.writer import write_file, WriterOpts
    recs = mixed_records(21, 3000, big=200)
    data = write_file(recs, WriterOpts(Transformers=["zstd"], MaxItems=3))
    items, err = scan_all(data, ctx)
    assert err == "" and items == recs


def test_corrupt_frames_match_oracle(ctx, oracle):
    # corrupt compressed bytes (the chunk CRC is computed over them, so only
    # the decoder can notice): the oracle's error (libzstd's error name) and the
    # items before it
    if not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import zstd_compress_ex
    rng = random.Random(19)
    errs = set()
    for trial in range(80):
        recs = mixed_records(300 + trial, 60)
        payload = F.packed_block_payload(recs)
        comp = bytearray(zstd_compress_ex(payload, rng.choice([1, 5, 19]), rng.random() < 0.5, rng.random() < 0.7))
        kind = rng.randrange(4)
        if kind == 0:  # bit flips anywhere
            for _ in range(rng.randrange(1, 4)):
                i = rng.randrange(len(comp))
                comp[i] ^= 1 << rng.randrange(8)
        elif kind == 1:  # truncation
            del comp[rng.randrange(len(comp)):]
        elif kind == 2:  # frame header byte
            comp[rng.randrange(min(14, len(comp)))] ^= 1 << rng.randrange(8)
        else:  # trailing garbage after the frame
            comp += bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 9)))
        good = zstd_compress_ex(F.packed_block_payload(recs[:5]), 3)
        data = zstd_file([good, bytes(comp)])
        items, err = scan_all(data, ctx)
        ref = oracle.scan(data)
        assert err == ref.err, (trial, kind, err, ref.err)
        assert items == ref.items, trial
        errs.add(err)
    assert len(errs) >= 3, errs


def test_empty_payload(ctx, oracle):
    # DataDog Decompress of an empty slice: ErrEmptySlice ("Bytes slice is empty")
    data = zstd_file([b""])
    items, err = scan_all(data, ctx)
    ref = oracle.scan(data)
    assert err == ref.err and err != "" and items == ref.items == []
