"""CPU tests: the oracle (C restatement) pinned against the golden fixtures, the
reference's known answers and independent codecs (zlib, libzstd)."""
import hashlib
import os
import random
import struct
import zlib

import pytest

from conftest import golden_bytes, oracle_has_zstd


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


def test_golden_manifest_cases(oracle, manifest):
    zstd_ok = oracle_has_zstd(oracle)
    checked = 0
    for case in manifest:
        if case["zstd"] and not zstd_ok:
            continue
        if case["name"] == "legacy_magic":  # a v2 chunk read as a v1 record: its header CRC fails
            r = oracle.scan(golden_bytes(case))
            assert r.legacy and r.items == []
            assert r.err.startswith("recordio: crc check failed - corrupt record header (")
            continue
        data = golden_bytes(case)
        r = oracle.scan(data, read_trailer=case["read_trailer"])
        assert r.err == case["err"], case["name"]
        assert len(r.items) == case["n_items"], case["name"]
        assert sha(r.items) == case["items_sha256"], case["name"]
        assert [len(x) for x in r.items][:4096] == case["lengths"], case["name"]
        assert hdr_json(r.header) == case["header"], case["name"]
        want_tr = bytes.fromhex(case["trailer"]) if case["trailer"] is not None else None
        assert r.trailer == want_tr, case["name"]
        checked += 1
    assert checked >= 40


def test_known_answer_sizes(manifest):
    """v2_test.go:80-124: empty body = 1 chunk, empty body + trailer = 2 chunks."""
    by = {c["name"]: c for c in manifest}
    assert by["empty_body"]["size"] == 32768
    assert by["header_only"]["size"] == 32768
    assert by["empty_body_trailer"]["size"] == 65536


def test_seek_locations(oracle, manifest):
    case = [c for c in manifest if c["name"] == "write_read"][0]
    data = golden_bytes(case)
    for value, block, item in case["locations"]:
        r = oracle.seek_get(data, block, item)
        assert r.err == "" and r.items == [value.encode()]
    r = oracle.seek_get(data, case["locations"][0][1], 7)
    assert r.err.startswith("Invalid location {Block:32768 Item:7}, block has only 2 items")


def test_shard_tables(oracle, manifest):
    """doShardedReads (v2_test.go:483-509) over the golden random files."""
    zstd_ok = oracle_has_zstd(oracle)
    for case in manifest:
        if "shards" not in case or (case["zstd"] and not zstd_ok):
            continue
        data = golden_bytes(case)
        for nshard, tab in case["shards"].items():
            nshard = int(nshard)
            stride = tab["stride"]
            counts = []
            for s in range(0, nshard, stride):
                r = oracle.scan(data, s, min(s + stride, nshard), nshard)
                assert r.err == "" and r.trailer == b"Trailer"
                counts.append(len(r.items))
            assert counts == tab["counts"], (case["name"], nshard)


def test_shard_range_float_math(oracle):
    """LimitShard uses float64 chunk math (chunk.go:202-206); check against Python floats."""
    rng = random.Random(3)
    for _ in range(2000):
        fsize = rng.randrange(0, 1 << 40) // 32768 * 32768 + rng.choice([0, 17])
        off = rng.randrange(0, 64) * 32768
        nshard = rng.choice([1, 2, 3, 7, 1000, 10 ** 9, rng.randrange(1, 5000)])
        start = rng.randrange(0, nshard)
        limit = rng.randrange(start + 1, nshard + 1)
        nc = (fsize - off) // 32768 if fsize >= off else -((off - fsize) // 32768)
        cps = float(nc) / float(nshard)
        want = (off + int(float(start) * cps) * 32768, off + int(float(limit) * cps) * 32768)
        assert oracle.shard_range(fsize, off, start, limit, nshard) == want


def test_crc32_matches_zlib(oracle):
    rng = random.Random(5)
    for n in [0, 1, 7, 8, 9, 1000, 32756]:
        b = bytes(rng.getrandbits(8) for _ in range(n))
        assert oracle.crc32(b) == zlib.crc32(b)


@pytest.mark.parametrize("level,strategy", [(0, zlib.Z_DEFAULT_STRATEGY), (1, zlib.Z_DEFAULT_STRATEGY),
                                            (6, zlib.Z_DEFAULT_STRATEGY), (9, zlib.Z_DEFAULT_STRATEGY),
                                            (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_RLE), (6, zlib.Z_FIXED)])
def test_inflate_matches_zlib(oracle, level, strategy):
    rng = random.Random(level * 10 + strategy)
    for n in [0, 1, 100, 5000, 70000, 300000]:
        kind = rng.randrange(3)
        if kind == 0:
            data = bytes(rng.getrandbits(8) for _ in range(n))
        elif kind == 1:
            data = bytes(rng.choice(b"ACGT") for _ in range(n))
        else:
            data = (b"@read\nACGTTGCA\n+\nIIIIHHHH\n" * (n // 25 + 1))[:n]
        c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
        comp = c.compress(data) + c.flush()
        rc, out, _ = oracle.inflate(comp, max(len(data), 1))
        assert rc == 0 and out == data
        # truncation -> unexpected EOF (or corrupt), never success with wrong bytes
        if len(comp) > 4:
            rc, out, _ = oracle.inflate(comp[:len(comp) // 2], len(data) + 1)
            assert rc in (1, 2)


def test_inflate_rejects_go_invalid_codes(oracle):
    # BTYPE=3 is corrupt before offset 1
    rc, _, off = oracle.inflate(b"\x07\x00", 16)
    assert rc == 1 and off == 1
    # stored block with NLEN != ~LEN
    rc, _, off = oracle.inflate(b"\x01\x05\x00\x00\x00hello", 16)
    assert rc == 1 and off == 5


def test_zstd_oracle_against_libzstd(oracle):
    from base_amd.recordio.codecs import have_zstd, zstd_compress
    if not have_zstd():
        pytest.skip("libzstd not present")
    if not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle restatement not built yet")
    rng = random.Random(11)
    for level in (1, 3, 5, 19):
        for n in (0, 1, 100, 5000, 200000):
            data = bytes(rng.choice(b"ACGTN") for _ in range(n))
            comp = zstd_compress(data, level)
            rc, out, msg = oracle.zstd_decompress(comp, max(n, 1))
            assert rc == 0 and out == data, msg


def test_writer_round_trips_through_oracle(oracle):
    from base_amd.recordio.writer import write_file, WriterOpts
    rng = random.Random(9)
    for tr in ([], ["flate"], ["flate 9"]):
        recs = [os.urandom(rng.randrange(0, 5000)) for _ in range(300)]
        data = write_file(recs, WriterOpts(Transformers=tr, MaxItems=rng.randrange(1, 60)), trailer=b"T")
        r = oracle.scan(data)
        assert r.err == "" and r.items == recs and r.trailer == b"T"


def test_random_large_writes_bounds(oracle):
    """TestRandomLargeWrites (recordio/v2_test.go:574-591) against the oracle:
    100k records (lengths 1..1024, flush probability 0.01) in 10 shards, then
    nshard = 1e9 with stride 1e8; the shards concatenate to the input and the
    largest holds 8,000 < n < 12,000 records. The bounds are the reference's --
    this pins the oracle's LimitShard (float64) math independently of itself."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_configs_gpu import generate_random_recordio
    rnd = random.Random(0)
    data, items, _ = generate_random_recordio(rnd, 0.01, 100000, 1024)
    for nshard, stride in ((10, 1), (1000000000, 100000000)):
        got, biggest = [], 0
        for s in range(0, nshard, stride):
            r = oracle.scan(data, s, min(s + stride, nshard), nshard)
            assert r.err == "" and r.trailer == b"Trailer"
            got += r.items
            biggest = max(biggest, len(r.items))
        assert got == items
        assert 8000 < biggest < 12000, (nshard, biggest)
