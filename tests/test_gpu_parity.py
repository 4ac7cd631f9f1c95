"""GPU parity: the HIP scan path (through the C ABI) against the CPU oracle and
the committed golden fixtures. Bit-exact items, identical header/trailer and the
reference's error text. Run on an MI355X: pytest -m gpu."""
import hashlib
import os
import random
import struct

import numpy as np
import pytest

from conftest import golden_bytes, oracle_has_zstd

pytestmark = pytest.mark.gpu

# codecs with a GPU decoder in this build; RIO_TEST_CODECS overrides
DEFAULT_CODECS = "none,flate,zstd"


def sha(items):
    h = hashlib.sha256()
    for it in items:
        h.update(struct.pack("<Q", len(it)))
        h.update(it)
    return h.hexdigest()


def hdr_json(header):
    from base_amd.recordio.format import Uint
    out = []
    for k, v in header:
        if isinstance(v, bool):
            out.append([k, "bool", v])
        elif isinstance(v, Uint):
            out.append([k, "uint", int(v)])
        elif isinstance(v, int):
            out.append([k, "int", v])
        else:
            out.append([k, "string", v])
    return out


def gpu_scan(data, ctx, start=0, limit=1, nshard=1, read_trailer=True):
    """readAllV2 (v2_test.go:34-47) over the GPU scanner."""
    from base_amd.recordio import gpu
    sc = gpu.NewShardScanner(data, gpu.ScannerOpts(), start, limit, nshard, ctx=ctx)
    header = sc.Header()
    trailer = sc.Trailer() if read_trailer else None
    items = []
    while sc.Scan():
        items.append(sc.Get())
    assert not sc.Scan()  # Scan after EOF stays false
    err = sc.Err()
    sc.Finish()
    return header, items, trailer, ("" if err is None else str(err)), err


def codec_supported(case):
    """RIO_TEST_CODECS (default all) limits the codecs under test."""
    enabled = os.environ.get("RIO_TEST_CODECS", DEFAULT_CODECS).split(",")
    for k, t, v in case["header"]:
        if k == "transformer" and v.split()[0] in ("flate", "zstd"):
            return v.split()[0] in enabled
    return True


def test_golden_cases(gpu_ctx, manifest, oracle):
    failures = []
    for case in manifest:
        if not codec_supported(case):
            continue
        data = golden_bytes(case)
        header, items, trailer, err, e = gpu_scan(data, gpu_ctx, read_trailer=case["read_trailer"])
        if case["name"] == "legacy_magic":  # decoded as v1 (legacyscanner.go): the oracle's v1 result
            ref = oracle.scan(data)
            assert ref.legacy and e is not None and e.code == 24 and err == ref.err and items == ref.items
            continue
        want_tr = bytes.fromhex(case["trailer"]) if case["trailer"] is not None else None
        got = (err, len(items), sha(items), trailer, hdr_json(header))
        want = (case["err"], case["n_items"], case["items_sha256"], want_tr, case["header"])
        if got != want:
            failures.append((case["name"], got[0], want[0], got[1], want[1]))
    assert failures == []


def test_seek_locations(gpu_ctx, manifest):
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import ItemLocation
    case = [c for c in manifest if c["name"] == "write_read"][0]
    data = golden_bytes(case)
    sc = gpu.NewScanner(data, ctx=gpu_ctx)
    for value, block, item in case["locations"]:
        sc.Seek(ItemLocation(block, item))
        assert sc.Err() is None
        assert sc.Scan()
        assert sc.Get() == value.encode()
    sc.Seek(ItemLocation(case["locations"][0][1], 7))
    assert str(sc.Err()).startswith("Invalid location {Block:32768 Item:7}, block has only 2 items")
    sc.Finish()


def test_shard_tables(gpu_ctx, manifest):
    for case in manifest:
        if "shards" not in case or not case["shards"] or not codec_supported(case):
            continue
        data = golden_bytes(case)
        for nshard, tab in case["shards"].items():
            nshard = int(nshard)
            counts = []
            for s in range(0, nshard, tab["stride"]):
                _, items, trailer, err, _ = gpu_scan(data, gpu_ctx, s, min(s + tab["stride"], nshard), nshard)
                assert err == "" and trailer == b"Trailer", (case["name"], nshard, s, err)
                counts.append(len(items))
            assert counts == tab["counts"], (case["name"], nshard)


def _random_file(rng, codec, nrec, maxlen, trailer=True):
    from base_amd.recordio.writer import Writer, WriterOpts
    import io
    buf = io.BytesIO()
    w = Writer(buf, WriterOpts(Transformers=[codec] if codec else [], KeyTrailer=trailer,
                               MaxItems=rng.choice([1, 3, 17, 253, 1000, 16384])))
    recs = []
    for i in range(nrec):
        n = rng.choice([0, 1, 2, rng.randrange(maxlen + 1), rng.randrange(128, 300)])
        x = os.urandom(n)
        recs.append(x)
        w.Append(x)
        if rng.random() < 0.02:
            w.Flush()
    if trailer:
        w.SetTrailer(b"Trailer")
    w.Finish()
    return buf.getvalue(), recs


@pytest.mark.parametrize("codec", ["", "flate", "zstd"])
def test_random_files_match_oracle(gpu_ctx, oracle, codec):
    if codec and codec not in os.environ.get("RIO_TEST_CODECS", DEFAULT_CODECS).split(","):
        pytest.skip("codec disabled")
    if codec == "zstd" and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    rng = random.Random(hash(codec) & 0xFFFF)
    for trial in range(12):
        data, recs = _random_file(rng, codec, rng.randrange(0, 3000), rng.choice([10, 300, 5000, 70000]))
        _, items, trailer, err, _ = gpu_scan(data, gpu_ctx)
        assert err == "" and items == recs and trailer == b"Trailer", (trial, err)
        ref = oracle.scan(data)
        assert ref.items == items


@pytest.mark.parametrize("codec", ["", "flate"])
def test_corruption_sweep_matches_oracle(gpu_ctx, oracle, codec):
    """Random single-byte corruptions: the GPU reports the oracle's first error
    (same text) after delivering the same items (errors.Once, first in file order)."""
    if codec and codec not in os.environ.get("RIO_TEST_CODECS", DEFAULT_CODECS).split(","):
        pytest.skip("codec disabled")
    rng = random.Random(77)
    data, recs = _random_file(rng, codec, 800, 3000)
    n = len(data)
    for trial in range(60):
        b = bytearray(data)
        kind = rng.randrange(4)
        c = rng.randrange(n // 32768)
        if kind == 0:  # payload byte
            o = c * 32768 + 28 + rng.randrange(32740)
        elif kind == 1:  # header field byte (crc/size/total/index)
            o = c * 32768 + 8 + rng.randrange(20)
        elif kind == 2:  # magic byte
            o = c * 32768 + rng.randrange(8)
        else:
            o = rng.randrange(n)
        b[o] ^= 1 << rng.randrange(8)
        d = bytes(b)
        _, items, trailer, err, e = gpu_scan(d, gpu_ctx, read_trailer=False)
        ref = oracle.scan(d, read_trailer=False)
        # (header magic destroyed: both read the file as v1, legacyscanner.go)
        assert err == ref.err, (trial, kind, o)
        assert items == ref.items, (trial, kind, o)


def test_span_boundaries(oracle):
    """Blocks larger than / straddling the span size: the scanner re-feeds spans."""
    from base_amd.recordio import gpu
    ctx = gpu.Context(0, max_span_bytes=4 * 32768)
    rng = random.Random(4)
    data, recs = _random_file(rng, "", 400, 20000)
    _, items, trailer, err, _ = gpu_scan(data, ctx)
    ref = oracle.scan(data)
    if ref.err == "":
        assert items == recs
    else:  # a block larger than the span is a capacity error, never wrong data
        assert items == recs[:len(items)]
    ctx.close()


def test_batch_api_c2_like(gpu_ctx, oracle):
    """rio_scan_span on a C2-shaped file (256 B records, 253 per block)."""
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import write_file, WriterOpts
    rng = np.random.default_rng(1)
    recs = [bytes(r) for r in rng.integers(0, 256, size=(20000, 256), dtype=np.uint8)]
    data = write_file(recs, WriterOpts(MaxItems=252))  # 253 per block (MaxItems + 1)
    hdr = 32768
    b = gpu_ctx.scan_span(data[hdr:], file_off=hdr, is_file_end=True)
    assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0
    items = gpu.batch_items(b)
    assert items == recs
    assert b.n_blocks == (20000 + 252) // 253


def test_full_size_c2_property(oracle):
    """C2 at its full 1x size (259 MB file): item count and checksum of checksums."""
    import bench
    from base_amd.recordio import gpu
    data, nrec = bench.make_c2_file()
    ctx = gpu.Context(0, max_span_bytes=len(data) + 32768)
    b = ctx.scan_span(data[32768:], file_off=32768, is_file_end=True)
    assert b.stop == gpu.RIO_STOP_EOF and b.n_items == nrec == 1000000
    recs = bench.c2_records()
    import ctypes
    span = np.frombuffer(data, dtype=np.uint8)[32768:]
    side = np.frombuffer(ctypes.string_at(b.records, b.records_len), dtype=np.uint8) if b.records_len else None
    off = np.ctypeslib.as_array(b.item_off, shape=(b.n_items,)).copy()
    ln = np.ctypeslib.as_array(b.item_len, shape=(b.n_items,))
    assert np.all(ln == 256)
    in_rec = (off >> np.uint64(63)).astype(bool)
    off &= np.uint64((1 << 63) - 1)
    off = off.astype(np.int64)
    ar = np.arange(256, dtype=np.int64)
    for lo in range(0, nrec, 100000):
        hi = min(nrec, lo + 100000)
        idx = off[lo:hi, None] + ar
        m = in_rec[lo:hi]
        got = np.empty((hi - lo, 256), dtype=np.uint8)
        got[~m] = span[idx[~m]]
        if m.any():
            got[m] = side[idx[m]]
        assert np.array_equal(got, recs[lo:hi])
    first = np.ctypeslib.as_array(b.block_first_item, shape=(b.n_blocks + 1,))
    assert first[0] == 0 and first[-1] == nrec
    assert np.all(np.diff(first.astype(np.int64))[:-1] == 253)
    ctx.close()


@pytest.mark.parametrize("codec", ["", "flate", "zstd"])
@pytest.mark.parametrize("item_end", [False, True])
def test_device_path_views(oracle, codec, item_end):
    """rio_scan_device (device-resident span), in both output shapes: item views
    into the span plus straddlers at their own span offset in the records
    buffer, or item_end (cumSize) + block_data / block_first_off
    (RIO_CFG_ITEM_END) -- the headline's output."""
    import torch
    from base_amd.recordio import gpu
    if codec == "zstd" and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    cid = {"": gpu.RIO_CODEC_NONE, "flate": gpu.RIO_CODEC_FLATE, "zstd": gpu.RIO_CODEC_ZSTD}[codec]
    ctx = gpu.Context(0, max_span_bytes=64 << 20, item_end=item_end)
    rng = random.Random(11)
    for trial in range(10):
        data, recs = _random_file(rng, codec, rng.randrange(1, 2500), rng.choice([10, 300, 5000, 70000]))
        hdr_chunks = struct.unpack_from("<I", data, 20)[0]
        body = data[hdr_chunks * 32768:]
        dev = torch.frombuffer(bytearray(body), dtype=torch.uint8).to("cuda:0")
        b = ctx.scan_device(dev.data_ptr(), len(body), file_off=hdr_chunks * 32768, is_file_end=True, codec=cid)
        assert b.err.code == 0, (trial, b.err.msg)
        assert bool(b.item_end) == item_end
        assert gpu.device_batch_items(b, body) == recs, trial
    ctx.close()


@pytest.mark.parametrize("item_end", [False, True])
def test_device_path_corruption(oracle, item_end):
    """The corruption sweep through rio_scan_device: the items before the first
    error (both output shapes) and the oracle's error text."""
    import torch
    from base_amd.recordio import gpu
    rng = random.Random(78)
    data, recs = _random_file(rng, "", 800, 3000, trailer=False)
    hdr_chunks = struct.unpack_from("<I", data, 20)[0]
    h = hdr_chunks * 32768
    ctx = gpu.Context(0, max_span_bytes=64 << 20, item_end=item_end)
    n = len(data)
    for trial in range(40):
        b = bytearray(data)
        o = rng.randrange(h, n) if rng.random() < 0.5 else rng.randrange(h // 32768, n // 32768) * 32768 + rng.randrange(28)
        b[o] ^= 1 << rng.randrange(8)
        d = bytes(b)
        ref = oracle.scan(d, read_trailer=False)
        body = d[h:]
        dev = torch.frombuffer(bytearray(body), dtype=torch.uint8).to("cuda:0")
        r = ctx.scan_device(dev.data_ptr(), len(body), file_off=h, is_file_end=True)
        got_err = r.err.msg.decode() if r.stop == gpu.RIO_STOP_ERROR else ""
        assert got_err == ref.err, (trial, o)
        assert gpu.device_batch_items(r, body) == ref.items, (trial, o)
    ctx.close()


def test_unsupported_codec_fails_loudly(gpu_ctx):
    """A transformer this build has no decoder for is an error -- never a CPU
    fallback and never silent data (registry.go:54-64: "Transformer %s not found")."""
    from base_amd.recordio.writer import write_file
    # the body is written untransformed; the header names an unknown codec
    data = write_file([b"a" * 100] * 10, header=[("transformer", "snappy")])
    _, items, _, err, e = gpu_scan(data, gpu_ctx, read_trailer=False)
    assert items == [] and e is not None and err == "Transformer snappy not found"
