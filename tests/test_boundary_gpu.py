"""The drop-in boundary on the GPU (pytest -m gpu), through the C ABI:

- rio_decode_block, the TransformFunc analogue (recordio/recordio.go:12): every
  flate / zstd body block of the golden fixtures, as one payload per chunk and
  re-split at arbitrary points (recordioiov gather semantics,
  recordioiov.go:14-58), against the oracle's untransform; corrupt blocks
  against the oracle's error text;
- RIO_ERR_FALLBACK for transformer chains and other transformer names
  (registry.go:113-148): the shim's cue to use recordio.NewShardScanner;
- scanners sharing one ctx never see each other's records (the reference's
  scanners share no state);
- Trailer() in the middle of a scan leaves the scan where it was; a Trailer()
  error ends the scan after the current block (scannerv2.go:316-342, 363-404);
- a failing Unmarshal stops the scan with a sticky error (scannerv2.go:396-400).
"""
import random
import struct

import pytest

from conftest import golden_bytes, oracle_has_zstd

pytestmark = pytest.mark.gpu

CHUNK = 32768


def body_blocks(data):
    """(magic, [payload per chunk]) of every block of a v2 file, in order."""
    out, cur = [], None
    for c in range(len(data) // CHUNK):
        h = data[c * CHUNK:c * CHUNK + 28]
        size, total, index = struct.unpack_from("<III", h, 16)
        pay = data[c * CHUNK + 28:c * CHUNK + 28 + size]
        if index == 0:
            cur = (h[:8], [pay])
            out.append(cur)
        else:
            cur[1].append(pay)
    return out


def codec_of(case):
    for k, t, v in case["header"]:
        if k == "transformer":
            return v.split()[0]
    return ""


def resplit(payloads, rng):
    """The same bytes as slices of arbitrary lengths (including empty ones)."""
    cat = b"".join(payloads)
    cuts = sorted(rng.randrange(len(cat) + 1) for _ in range(rng.randrange(0, 6)))
    out, a = [], 0
    for b in cuts + [len(cat)]:
        out.append(cat[a:b])
        a = b
    return out


def oracle_untransform(oracle, codec, comp):
    """The oracle's untransform of one block, through a one-block file: (bytes, error text)."""
    from base_amd.recordio import format as F
    hdr = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", codec)])]))
    if codec == "flate":
        rc, out, _ = oracle.inflate(comp)
    else:
        rc, out, _ = oracle.zstd_decompress(comp)
    ref = oracle.scan(hdr + F.chunk_block(F.MAGIC_PACKED, comp), read_trailer=False)
    return (out if rc == 0 else None), ref.err


def test_decode_block_golden(gpu_ctx, manifest, oracle):
    """Every flate / zstd body block of the golden fixtures (chains: the
    combined untransform, the last transformer first -- registry.go:121-146)."""
    from base_amd.recordio import gpu
    from base_amd.recordio.format import MAGIC_PACKED
    rng = random.Random(5)
    checked = 0
    for case in manifest:
        trs = [v.split()[0] for k, t, v in case["header"] if k == "transformer"]
        if not trs or any(t not in ("flate", "zstd") for t in trs) or case["err"]:
            continue
        if "zstd" in trs and not oracle_has_zstd(oracle):
            continue
        ids = [gpu.RIO_CODEC_FLATE if t == "flate" else gpu.RIO_CODEC_ZSTD for t in trs]
        cid = ids[0] if len(ids) == 1 else gpu.codec_chain(*ids)
        for magic, pays in body_blocks(golden_bytes(case)):
            if magic != MAGIC_PACKED:
                continue
            want, err = b"".join(pays), ""
            for t in reversed(trs):
                want, err = oracle_untransform(oracle, t, want)
                if want is None:
                    break
            assert want is not None, (case["name"], err)
            assert gpu_ctx.decode_block(pays, cid) == want, case["name"]
            assert gpu_ctx.decode_block(resplit(pays, rng), cid, cap=16) == want, case["name"]
            checked += 1
    assert checked >= 20


@pytest.mark.parametrize("codec", ["flate", "zstd"])
def test_decode_block_corrupt(gpu_ctx, oracle, codec):
    from base_amd.recordio import gpu
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import make_compressor
    if codec == "zstd" and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    cid = gpu.RIO_CODEC_FLATE if codec == "flate" else gpu.RIO_CODEC_ZSTD
    rng = random.Random(31)
    comp = make_compressor(codec)
    nerr = 0
    for trial in range(40):
        recs = [bytes(rng.choice(b"ACGT") for _ in range(rng.randrange(0, 300))) for _ in range(50)]
        blob = bytearray(comp(F.packed_block_payload(recs)))
        if trial % 4 == 3:
            del blob[rng.randrange(len(blob)):]
        else:
            blob[rng.randrange(len(blob))] ^= 1 << rng.randrange(8)
        want, err = oracle_untransform(oracle, codec, bytes(blob))
        try:
            got = gpu_ctx.decode_block([bytes(blob)], cid)
            assert want is not None and got == want, (trial, err)
        except gpu.RecordioError as e:
            assert want is None and str(e) == err, (trial, str(e), err)
            nerr += 1
    assert nerr >= 10
    # empty input: Go's inflater reports unexpected EOF, DataDog zstd ErrEmptySlice
    want, err = oracle_untransform(oracle, codec, b"")
    with pytest.raises(gpu.RecordioError) as ei:
        gpu_ctx.decode_block([], cid)
    assert str(ei.value) == err != ""


def test_decode_block_none(gpu_ctx):
    from base_amd.recordio import gpu
    pays = [b"abc", b"", b"defgh" * 1000]
    assert gpu_ctx.decode_block(pays, gpu.RIO_CODEC_NONE, cap=2) == b"".join(pays)


@pytest.mark.parametrize("transformers,msg", [
    (["testplus 3", "testxor 111"], None),                  # v2_test.go:307-372
    (["flate", "testxor 111"], None),                       # a chain with a name not decoded here
    (["snappy"], "Transformer snappy not found"),           # registry.go:58
])
def test_fallback_code(gpu_ctx, transformers, msg):
    """Files this library does not untransform report RIO_ERR_FALLBACK before any
    record, so that the shim hands them to recordio.NewShardScanner."""
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import write_file
    data = write_file([b"a" * 100] * 10, header=[("transformer", t) for t in transformers])
    sc = gpu.NewScanner(data, ctx=gpu_ctx)
    assert not sc.Scan()
    e = sc.Finish()
    assert e is not None and e.code == gpu.RIO_ERR_FALLBACK
    if msg:
        assert str(e) == msg


def _scan_all(sc):
    out = []
    while sc.Scan():
        out.append(sc.Get())
    return out


@pytest.mark.parametrize("codec", ["", "flate", "zstd"])
def test_interleaved_scanners_share_ctx(gpu_ctx, oracle, codec):
    """Two scanners on one ctx, Scan calls interleaved item by item, plus a third
    opened (header read) in the middle: each returns exactly its own file."""
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import write_file, WriterOpts
    if codec == "zstd" and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    rng = random.Random(len(codec))
    tr = [codec] if codec else []
    files = []
    for k in range(3):
        recs = [bytes([k]) * rng.randrange(0, 2000) + bytes(rng.getrandbits(8) for _ in range(8))
                for _ in range(rng.randrange(400, 900))]
        files.append((write_file(recs, WriterOpts(Transformers=tr, MaxItems=rng.choice([7, 50, 300])),
                                 trailer=b"T%d" % k), recs))
    a = gpu.NewScanner(files[0][0], ctx=gpu_ctx)
    b = gpu.NewScanner(files[1][0], ctx=gpu_ctx)
    got_a, got_b, c = [], [], None
    more_a = more_b = True
    while more_a or more_b:
        if more_a:
            more_a = a.Scan()
            if more_a:
                got_a.append(a.Get())
        if more_b:
            more_b = b.Scan()
            if more_b:
                got_b.append(b.Get())
        if c is None and len(got_a) == 100:
            c = gpu.NewScanner(files[2][0], ctx=gpu_ctx)  # header + trailer decode on the shared ctx
            assert c.Trailer() == b"T2"
            assert a.Trailer() == b"T0"
    assert a.Finish() is None and b.Finish() is None
    assert got_a == files[0][1] and got_b == files[1][1]
    assert _scan_all(c) == files[2][1] and c.Finish() is None


@pytest.mark.parametrize("codec", ["", "flate"])
def test_trailer_mid_scan(gpu_ctx, codec):
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import write_file, WriterOpts
    rng = random.Random(3)
    recs = [bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 5000))) for _ in range(600)]
    data = write_file(recs, WriterOpts(Transformers=[codec] if codec else [], MaxItems=40), trailer=b"tail" * 9000)
    sc = gpu.NewScanner(data, ctx=gpu_ctx)
    got = []
    for i in range(len(recs)):
        assert sc.Scan()
        got.append(sc.Get())
        if i in (0, 39, 40, 333):
            assert sc.Trailer() == b"tail" * 9000
    assert not sc.Scan() and sc.Finish() is None
    assert got == recs


def test_trailer_error_mid_scan(gpu_ctx):
    """Header says trailer=true but the file has no trailer block (Writer with
    KeyTrailer and no SetTrailer, writerv2.go:562-587): Trailer() fails with
    ReadLastBlock's error; Scan delivers the rest of the current block only."""
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import Writer, WriterOpts
    import io
    recs = [b"r%05d" % i for i in range(100)]
    buf = io.BytesIO()
    w = Writer(buf, WriterOpts(KeyTrailer=True, MaxItems=30))
    for r in recs:
        w.Append(r)
    w.Finish()
    sc = gpu.NewScanner(buf.getvalue(), ctx=gpu_ctx)
    got = []
    for _ in range(35):  # into the second block (items 31..61: MaxItems + 1 per block)
        assert sc.Scan()
        got.append(sc.Get())
    assert sc.Trailer() is None
    err = str(sc.Err())
    assert err.startswith("Missing magic trailer; found ["), err
    got += _scan_all(sc)
    assert got == recs[:62]  # the rest of block 2, then the sticky error
    assert str(sc.Finish()) == err


def test_unmarshal_error_is_sticky(gpu_ctx):
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import write_file, WriterOpts
    recs = [b"%d" % i for i in range(50)]
    data = write_file(recs, WriterOpts(MaxItems=7))

    def unmarshal(b):
        if b == b"20":
            raise ValueError("bad record 20")
        return int(b)
    sc = gpu.NewScanner(data, gpu.ScannerOpts(Unmarshal=unmarshal), ctx=gpu_ctx)
    got = _scan_all(sc)
    assert got == list(range(20))
    assert not sc.Scan()  # stays false
    assert str(sc.Finish()) == "bad record 20"


@pytest.mark.parametrize("codec", ["flate", "zstd"])
def test_async_device_path_after_host_result(gpu_ctx, oracle, codec):
    """rio_scan_device_async + rio_sync on a ctx whose previous call was a host
    result of a compressed codec (rio_scan_span compacts the decoded blocks):
    the device batch's records are this call's decode regions, not the previous
    call's compacted bytes (pipeline.cpp resets last_cmp per enqueue)."""
    import struct
    import torch
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import write_file, WriterOpts
    if codec == "zstd" and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    rng = random.Random(91)
    code = gpu.RIO_CODEC_FLATE if codec == "flate" else gpu.RIO_CODEC_ZSTD
    files = []
    for k in range(2):
        recs = [bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 600))) for _ in range(700)]
        files.append((write_file(recs, WriterOpts(Transformers=[codec], MaxItems=64)), recs))
    for data, recs in files:
        h = struct.unpack_from("<I", data, 20)[0] * 32768
        b = gpu_ctx.scan_span(data[h:], file_off=h, is_file_end=True, codec=code)  # host result: compacted
        assert gpu.batch_items(b) == recs
    data, recs = files[0]
    h = struct.unpack_from("<I", data, 20)[0] * 32768
    body = data[h:]
    dev = torch.frombuffer(bytearray(body), dtype=torch.uint8).to("cuda:0")
    gpu_ctx.scan_device_async(dev.data_ptr(), len(body), file_off=h, codec=code)
    b = gpu_ctx.sync()
    assert b.err.code == 0, b.err.msg
    assert gpu.device_batch_items(b, body) == recs


def test_file_objects(gpu_ctx, oracle, tmp_path):
    """NewScanner over file objects (the reference takes an io.ReadSeeker): a
    raw and a buffered OS file are read with pread; a gzip.GzipFile (whose
    fileno() is the compressed file's descriptor) through its own seek + read,
    so the decompressed bytes are scanned."""
    import gzip
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import WriterOpts, write_file
    rng = random.Random(9)
    recs = [rng.randbytes(rng.randrange(0, 3000)) for _ in range(800)]
    data = write_file(recs, WriterOpts(MaxItems=31), trailer=b"tr")
    plain = tmp_path / "f.rio"
    plain.write_bytes(data)
    gz = tmp_path / "f.rio.gz"
    with gzip.open(gz, "wb") as f:
        f.write(data)
    for opener in (lambda: open(plain, "rb"), lambda: open(plain, "rb", buffering=0), lambda: gzip.open(gz, "rb")):
        with opener() as f:
            sc = gpu.NewScanner(f, ctx=gpu_ctx)
            assert sc.Trailer() == b"tr"
            got = []
            while sc.Scan():
                got.append(sc.Get())
            assert sc.Finish() is None and got == recs
