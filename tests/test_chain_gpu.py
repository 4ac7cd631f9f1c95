"""Transformer chains on the GPU (registry.go:121-146): a file written with
Transformers [t0, t1, ...] is untransformed tn-1 first. The golden chain cases
run in test_gpu_parity.test_golden_cases; here the other entry points: the
batch layer (host and device results, both output shapes), rio_decode_block,
Seek / Gather, sharded scans, corrupt streams against the oracle, and the async
entries (rio_scan_device_async, rio_scan_device_segments_async: a chain's
stages run at the call, rio_sync returns the batch)."""
import os
import random
import struct
import sys

import pytest

from conftest import ROOT, golden_bytes, oracle_has_zstd

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def chain_files(oracle):
    from base_amd.recordio.writer import WriterOpts, write_file
    if not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    rng = random.Random(17)
    recs = [rng.randbytes(rng.choice([0, 3, 200, 3000])) * rng.choice([1, 1, 20]) for _ in range(900)]
    out = {}
    for trs in (["zstd", "flate"], ["flate 1", "zstd"], ["flate", "flate 9"], ["zstd", "flate", "zstd 1", "flate"]):
        out[tuple(trs)] = write_file(recs, WriterOpts(Transformers=list(trs), MaxItems=41), trailer=b"TT")
    return recs, out


def _codec(trs):
    from base_amd.recordio import gpu
    return gpu.codec_chain(*[gpu.RIO_CODEC_FLATE if t.startswith("flate") else gpu.RIO_CODEC_ZSTD for t in trs])


def _body(data):
    hdr_chunks = struct.unpack_from("<I", data, 20)[0]
    return hdr_chunks * 32768


def test_chain_scanner_and_seek(gpu_ctx, oracle, chain_files):
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import ItemLocation
    recs, files = chain_files
    for trs, data in files.items():
        ref = oracle.scan(data)
        assert ref.err == "" and ref.items == recs and ref.trailer == b"TT", trs
        sc = gpu.NewScanner(data, ctx=gpu_ctx)
        assert sc.Trailer() == b"TT"
        got = []
        while sc.Scan():
            got.append(sc.Get())
        assert sc.Finish() is None and got == recs, trs
        sc = gpu.NewScanner(data, ctx=gpu_ctx)
        pick = list(range(0, len(recs), 37))
        assert sc.Gather([ItemLocation(*ref.locations[i]) for i in pick]) == [recs[i] for i in pick]
        for i in pick[:5]:
            sc.Seek(ItemLocation(*ref.locations[i]))
            assert sc.Scan() and sc.Get() == recs[i]
        sc.Finish()
        # shards concatenate to the file
        parts = []
        for s in range(3):
            sc = gpu.NewShardScanner(data, gpu.ScannerOpts(), s, s + 1, 3, ctx=gpu_ctx)
            while sc.Scan():
                parts.append(sc.Get())
            assert sc.Finish() is None
        assert parts == recs


@pytest.mark.parametrize("item_end", [False, True])
def test_chain_batch_layer(oracle, chain_files, item_end):
    """rio_scan_span (host results, block offsets in the file) and
    rio_scan_device (device results) over a chain file's body."""
    import torch
    from base_amd.recordio import gpu
    recs, files = chain_files
    ctx = gpu.Context(0, max_span_bytes=8 << 20, item_end=item_end)
    try:
        for trs, data in files.items():
            body = data[_body(data):]
            b = ctx.scan_span(body, file_off=_body(data), is_file_end=True, codec=_codec(trs))
            assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, (trs, b.err.msg)
            assert gpu.batch_items(b) == recs
            ref = oracle.scan(data)
            blocks = sorted({loc[0] for loc in ref.locations})
            assert [b.block_file_off[i] for i in range(b.n_blocks)] == blocks
            dev = torch.frombuffer(bytearray(body), dtype=torch.uint8).to("cuda:0")
            bd = ctx.scan_device(dev.data_ptr(), len(body), file_off=_body(data), is_file_end=True,
                                 codec=_codec(trs))
            assert bd.stop == gpu.RIO_STOP_EOF and bd.err.code == 0, (trs, bd.err.msg)
            assert gpu.device_batch_items(bd, body) == recs
            ctx.scan_device_async(dev.data_ptr(), len(body), _body(data), _codec(trs))
            ba = ctx.sync()
            assert ba.stop == gpu.RIO_STOP_EOF and ba.err.code == 0, (trs, ba.err.msg)
            assert gpu.device_batch_items(ba, body) == recs
    finally:
        ctx.close()


def test_chain_growth_is_temporary(chain_files):
    """A chain's later stages decode spans larger than the file's (the decoded
    bytes, reframed): the context grows for that call only. Consecutive chain
    calls keep the growth; the next plain call (here a none-codec span, checked)
    returns the device buffers to the configured span."""
    import torch
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import WriterOpts, write_file
    recs = chain_files[0]
    trs = ("flate 0", "zstd")  # stored DEFLATE under zstd: stage 2's span is ~the records' size
    data = write_file(recs, WriterOpts(Transformers=list(trs), MaxItems=41))
    body = data[_body(data):]
    cap0 = (len(body) + 32767) // 32768 * 32768
    assert sum(map(len, recs)) > 2 * cap0
    plain_recs = [bytes([k % 251]) * (k * 7 % 900) for k in range(500)]
    plain = write_file(plain_recs, WriterOpts(MaxItems=50))
    ctx = gpu.Context(0, max_span_bytes=cap0)
    try:
        assert ctx.stats()["span_cap"] == cap0
        for _ in range(2):
            b = ctx.scan_span(body, file_off=_body(data), is_file_end=True, codec=_codec(trs))
            assert b.err.code == 0 and gpu.batch_items(b) == recs, b.err.msg
            assert ctx.stats()["span_cap"] > cap0
        pb = plain[_body(plain):]
        dev = torch.frombuffer(bytearray(pb), dtype=torch.uint8).to("cuda:0")
        bd = ctx.scan_device(dev.data_ptr(), len(pb), file_off=_body(plain), is_file_end=True,
                             codec=gpu.RIO_CODEC_NONE)
        assert bd.err.code == 0 and gpu.device_batch_items(bd, pb) == plain_recs
        assert ctx.stats()["span_cap"] == cap0
        b = ctx.scan_span(body, file_off=_body(data), is_file_end=True, codec=_codec(trs))
        assert b.err.code == 0 and gpu.batch_items(b) == recs  # grows again
    finally:
        ctx.close()


def test_decode_block_growth_is_temporary():
    """rio_decode_block of a block longer than the context's span grows it for
    that call; the next plain call returns it to the configured size."""
    import os as _os
    import torch
    from base_amd.recordio import gpu
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import make_compressor
    from base_amd.recordio.writer import WriterOpts, write_file
    recs = [_os.urandom(3000) for _ in range(400)]  # ~1.2 MB, incompressible
    payload = F.packed_block_payload(recs)
    comp = make_compressor("flate 1")(payload)
    cap0 = 4 * 32768
    ctx = gpu.Context(0, max_span_bytes=cap0)
    try:
        assert len(comp) > 2 * cap0
        pays = [comp[i:i + 30000] for i in range(0, len(comp), 30000)]
        assert ctx.decode_block(pays, gpu.RIO_CODEC_FLATE) == payload
        assert ctx.stats()["span_cap"] > cap0
        plain_recs = [bytes([k % 251]) * 100 for k in range(300)]
        plain = write_file(plain_recs, WriterOpts(MaxItems=1000))  # one block: a chunk
        pb = plain[32768:]
        assert len(pb) <= cap0
        dev = torch.frombuffer(bytearray(pb), dtype=torch.uint8).to("cuda:0")
        bd = ctx.scan_device(dev.data_ptr(), len(pb), file_off=32768, is_file_end=True,
                             codec=gpu.RIO_CODEC_NONE)
        assert bd.err.code == 0 and gpu.device_batch_items(bd, pb) == plain_recs, bd.err.msg
        assert ctx.stats()["span_cap"] == cap0
    finally:
        ctx.close()


def test_chain_decode_block(gpu_ctx, oracle, chain_files):
    """rio_decode_block with a chain codec: the combined untransform of one block."""
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import make_compressor
    recs, files = chain_files
    for trs in files:
        payload = F.packed_block_payload(recs[:60])
        comp = payload
        for t in trs:
            comp = make_compressor(t)(comp)
        pays = [comp[i:i + 1000] for i in range(0, len(comp), 1000)]
        assert gpu_ctx.decode_block(pays, _codec(trs)) == payload


def test_chain_corruption_matches_oracle(gpu_ctx, oracle, chain_files):
    """Bit flips inside the compressed streams (chunk CRCs fixed, so only the
    codecs and the packed parse can notice): the same items and error text as
    the oracle's chain."""
    import zlib
    recs, files = chain_files
    rng = random.Random(5)
    for trs, data in files.items():
        for trial in range(8):
            b = bytearray(data)
            c = rng.randrange(_body(data) // 32768, len(data) // 32768 - 1)  # not the trailer
            o = c * 32768
            size = struct.unpack_from("<I", b, o + 16)[0]
            if size == 0:
                continue
            b[o + 28 + rng.randrange(size)] ^= 1 << rng.randrange(8)
            struct.pack_into("<I", b, o + 8, zlib.crc32(bytes(b[o + 12:o + 28 + size])))
            d = bytes(b)
            ref = oracle.scan(d, read_trailer=False)
            from base_amd.recordio import gpu
            sc = gpu.NewScanner(d, ctx=gpu_ctx)
            got = []
            while sc.Scan():
                got.append(sc.Get())
            e = sc.Finish()
            assert ("" if e is None else str(e)) == ref.err and got == ref.items, (trs, trial)


def test_golden_chain_cases_decode(gpu_ctx, manifest):
    """The committed chain fixtures (tests/golden/make_golden.py) through the
    device batch path, against the manifest."""
    import hashlib
    import torch
    from base_amd.recordio import gpu
    for case in manifest:
        if not case["name"].startswith("chain"):
            continue
        data = golden_bytes(case)
        trs = [v for k, t, v in case["header"] if k == "transformer"]
        body = data[_body(data):]
        if case["trailer"] is not None:  # the body ends where the trailer block starts
            body = body[:-32768 * (struct.unpack_from("<I", data, len(data) - 32768 + 24)[0] + 1)]
        dev = torch.frombuffer(bytearray(body), dtype=torch.uint8).to("cuda:0")
        b = gpu_ctx.scan_device(dev.data_ptr(), len(body), file_off=_body(data), is_file_end=True,
                                codec=_codec(trs))
        assert b.err.code == 0, b.err.msg
        items = gpu.device_batch_items(b, body)
        h = hashlib.sha256()
        for it in items:
            h.update(struct.pack("<Q", len(it)))
            h.update(it)
        assert len(items) == case["n_items"] and h.hexdigest() == case["items_sha256"]


def test_chain_segments_scan(oracle, chain_files):
    """Chained files through the many-file launch (rio_scan_device_segments_async,
    configs[4]'s path): the bodies of every chain file of one chain back to back
    with different records each; every block's file (block_segment) and its
    ItemLocation.Block in that file (block_file_off, the oracle's locations), the
    records of each file; a corrupt stream in the second file stops the batch
    there in that file's coordinates, the first file's records delivered."""
    import ctypes
    import zlib
    import numpy as np
    import torch
    from base_amd.recordio import gpu, shard
    from base_amd.recordio.writer import WriterOpts, write_file
    rng = random.Random(23)
    for trs in (("zstd", "flate"), ("flate", "zstd", "flate 1")):
        recs = [[rng.randbytes(rng.choice([5, 90, 2000])) * rng.choice([1, 8]) for _ in range(n)]
                for n in (300, 77, 410)]
        datas = [write_file(r, WriterOpts(Transformers=list(trs), MaxItems=29), trailer=b"T%d" % k)
                 for k, r in enumerate(recs)]
        bodies, ends, foffs = [], [], []
        for d in datas:
            bodies.append(d[_body(d):shard.trailer_offset(d)])
            ends.append(sum(map(len, bodies)))
            foffs.append(_body(d))
        span = b"".join(bodies)
        dev = torch.frombuffer(bytearray(span), dtype=torch.uint8).to("cuda:0")
        ctx = gpu.Context(0, max_span_bytes=len(span) + 32768, item_end=True)
        try:
            ctx.scan_device_segments_async(dev.data_ptr(), len(span), ends, foffs, _codec(trs))
            b = ctx.sync()
            assert b.err.code == 0 and b.stop == gpu.RIO_STOP_EOF and b.err_segment == -1, b.err.msg
            nb = int(b.n_blocks)
            u64 = lambda p, n: np.frombuffer(gpu.dev_to_host(ctypes.cast(p, ctypes.c_void_p).value, 8 * n),
                                             dtype=np.uint64)
            seg, boff, first = u64(b.block_segment, nb), u64(b.block_file_off, nb), u64(b.block_first_item, nb + 1)
            items = gpu.device_batch_items(b, span)
            for k, d in enumerate(datas):
                ref = oracle.scan(d)
                assert ref.err == "" and ref.items == recs[k]
                sel = np.nonzero(seg == k)[0]
                assert boff[sel].tolist() == sorted({loc[0] for loc in ref.locations}), (trs, k)
                assert items[int(first[sel[0]]):int(first[sel[-1] + 1])] == recs[k], (trs, k)
            # file 1's middle chunk: a bit flip with its CRC fixed (the chain decodes or
            # rejects it as the oracle's does), then the same flip with the CRC left
            # stale (stage 1's chunk error); both in file 1's coordinates
            o = ends[0] + (ends[1] - ends[0]) // 32768 // 2 * 32768
            size = struct.unpack_from("<I", span, o + 16)[0]
            for fix_crc in (True, False):
                bad = bytearray(span)
                bad[o + 28 + size // 2] ^= 0x10
                if fix_crc:
                    struct.pack_into("<I", bad, o + 8, zlib.crc32(bytes(bad[o + 12:o + 28 + size])))
                ref = oracle.scan(bytes(datas[1][:foffs[1]]) + bytes(bad[ends[0]:ends[1]]), read_trailer=False)
                assert fix_crc or ref.err.startswith("Chunk checksum mismatch"), ref.err
                dev.copy_(torch.frombuffer(bad, dtype=torch.uint8))
                ctx.scan_device_segments_async(dev.data_ptr(), len(span), ends, foffs, _codec(trs))
                b = ctx.sync()
                got = gpu.device_batch_items(b, bytes(bad))
                if ref.err:
                    assert b.stop == gpu.RIO_STOP_ERROR and b.err_segment == 1, (trs, fix_crc, b.err.msg)
                    assert b.err.msg.decode() == ref.err, (trs, b.err.msg, ref.err)
                    assert got == recs[0] + ref.items
                else:
                    assert b.err.code == 0 and b.stop == gpu.RIO_STOP_EOF, (trs, b.err.msg)
                    assert got == recs[0] + ref.items + recs[2]
        finally:
            ctx.close()
