"""Generate the committed golden fixtures under tests/golden/.

Run here (not on the GPU box): python tests/golden/make_golden.py

Each fixture is a small recordio file written by base_amd.recordio.writer (a
restatement of writerv2.go / chunk.go) with independent encoders (zlib raw
DEFLATE, libzstd), plus the expected scan result. Expectations come from the
records handed to the writer (valid files) or from the reference's error
formats (corrupt files), and are checked against the CPU oracle at generation
time. The reference's own known-answer tests are restated as cases too
(recordio/v2_test.go:74-188, 544-591; transformer_test.go:20-62).
"""
from __future__ import annotations

import hashlib
import io
import json
import os
import random
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from base_amd.recordio import format as F  # noqa: E402
from base_amd.recordio.codecs import have_zstd, zstd_compress  # noqa: E402
from base_amd.recordio.writer import Writer, WriterOpts, write_file  # noqa: E402
from oracle import oracle as O  # noqa: E402

CASES = []
# whether the CPU oracle's zstd restatement is built (oracle/zstd_dec.c)
ORACLE_ZSTD = have_zstd() and O.zstd_decompress(zstd_compress(b"probe", 1))[0] == 0


def sha(items):
    h = hashlib.sha256()
    for it in items:
        h.update(struct.pack("<Q", len(it)))
        h.update(it)
    return h.hexdigest()


def hdr_json(header):
    out = []
    for k, v in header:
        if isinstance(v, bool):
            out.append([k, "bool", v])
        elif isinstance(v, F.Uint):
            out.append([k, "uint", int(v)])
        elif isinstance(v, int):
            out.append([k, "int", v])
        else:
            out.append([k, "string", v])
    return out


def add(name, data, items=None, header=(), trailer=None, err="", shards=None, locations=None, note="",
        read_trailer=True, oracle_check=True):
    """Register a fixture; `items` is what the reference scanner returns."""
    path = os.path.join(HERE, name + ".rio")
    with open(path, "wb") as f:
        f.write(data)
    exp = {"name": name, "file": name + ".rio", "size": len(data), "n_items": len(items or []),
           "items_sha256": sha(items or []), "lengths": [len(x) for x in (items or [])][:4096],
           "header": hdr_json(header), "trailer": (trailer.hex() if trailer is not None else None), "err": err,
           "read_trailer": read_trailer, "note": note}
    if locations is not None:
        exp["locations"] = locations
    if shards is not None:
        exp["shards"] = shards
    uses_zstd = any(k == "transformer" and str(v).startswith("zstd") for k, v in header)
    exp["zstd"] = uses_zstd
    if oracle_check and (ORACLE_ZSTD or not uses_zstd):
        r = O.scan(data, read_trailer=read_trailer)
        got = (len(r.items), sha(r.items), r.err, r.trailer, hdr_json(r.header))
        want = (len(items or []), exp["items_sha256"], err, trailer if read_trailer else None, exp["header"])
        if got != want:
            raise SystemExit(f"oracle disagrees on {name}:\n got  {got[0]} {got[2]!r} {got[3]!r} {got[4]}\n"
                             f" want {want[0]} {want[2]!r} {want[3]!r} {want[4]}")
    CASES.append(exp)


def rnd_bytes(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def rnd_letters(rng, n):
    return bytes(ord("A") + rng.randrange(64) for _ in range(n))


def main():
    rng = random.Random(0x5EED)
    for f in os.listdir(HERE):
        if f.endswith(".rio"):
            os.remove(os.path.join(HERE, f))

    # --- v2_test.go known answers -------------------------------------------
    add("empty_file", b"", [], note="TestEmptyFile v2_test.go:74-78")
    d = write_file([])
    assert len(d) == F.CHUNK_SIZE
    add("empty_body", d, [], note="TestEmptyBody v2_test.go:80-89 (one header chunk)")
    buf = io.BytesIO()
    w = Writer(buf)
    w.Flush()
    w.Finish()
    add("flush_empty", buf.getvalue(), [], note="TestFlushEmpty v2_test.go:91-100")
    buf = io.BytesIO()
    w = Writer(buf)
    w.AddHeader("Foo", "Hah")
    w.Finish()
    assert len(buf.getvalue()) == F.CHUNK_SIZE
    add("header_only", buf.getvalue(), [], header=[("Foo", "Hah")], note="v2_test.go:102-112")
    buf = io.BytesIO()
    w = Writer(buf, WriterOpts(KeyTrailer=True))
    w.SetTrailer(b"TTT")
    w.Finish()
    assert len(buf.getvalue()) == 2 * F.CHUNK_SIZE
    add("empty_body_trailer", buf.getvalue(), [], header=[("trailer", True)], trailer=b"TTT",
        note="v2_test.go:114-124 (header+trailer = 65536 B)")
    large = rnd_letters(rng, F.CHUNK_SIZE * 10 + 100)
    buf = io.BytesIO()
    w = Writer(buf, WriterOpts(KeyTrailer=True))
    w.Append(b"XX")
    w.SetTrailer(large)
    w.Finish()
    add("large_trailer", buf.getvalue(), [b"XX"], header=[("trailer", True)], trailer=large,
        note="TestV2LargeTrailer v2_test.go:126-139 (10 chunks + 100 B)")
    # TestV2WriteRead with typed header and Index locations
    buf = io.BytesIO()
    locs = {}
    w = Writer(buf, WriterOpts(KeyTrailer=True, Index=lambda loc, v: locs.__setitem__(v, loc)))
    w.AddHeader("hh0", "vv0")
    w.AddHeader("hh1", 12345)
    w.AddHeader("hh2", F.Uint(234))
    for x in (b"F0", b"F1"):
        w.Append(x)
    w.Flush()
    w.Append(b"F2")
    w.Flush()
    w.Append(b"F3")
    w.SetTrailer(b"Trailer2")
    w.Finish()
    add("write_read", buf.getvalue(), [b"F0", b"F1", b"F2", b"F3"],
        header=[("trailer", True), ("hh0", "vv0"), ("hh1", 12345), ("hh2", F.Uint(234))], trailer=b"Trailer2",
        locations=[[k.decode(), v.Block, v.Item] for k, v in sorted(locs.items())],
        note="TestV2WriteRead v2_test.go:141-188")
    # transformer_test.go: 300 x 4 KiB compressible items
    items = [bytes([(ord("A") + i) % 256]) * (16 << 8) for i in range(300)]
    for name in (["flate", "zstd"] if have_zstd() else ["flate"]):
        d = write_file(items, WriterOpts(Transformers=[name]))
        assert len(d) / (300 * 4096) < 0.2
        add(f"transformer_{name}", d, items, header=[("transformer", name)],
            note="transformer_test.go:20-62 (ratio < 0.2)")
    # Example_basic (example_basic_test.go:41-48)
    d = write_file([b"Item0", b"Item1"], WriterOpts(Transformers=["flate"]))
    add("example_basic", d, [b"Item0", b"Item1"], header=[("transformer", "flate")])

    # --- record-size mixes across codecs --------------------------------------
    sizes = [0, 1, 127, 128, 255, 256, 32739, 32740, 32741, 65536, 3, 0, 40000]
    mix = [rnd_bytes(rng, s) for s in sizes]
    codecs = [[], ["flate"], ["flate 1"], ["flate 9"], ["flate 0"]]
    if have_zstd():
        codecs += [["zstd"], ["zstd 1"], ["zstd 19"]]
    for tr in codecs:
        tag = (tr[0].replace(" ", "") if tr else "none")
        d = write_file(mix, WriterOpts(Transformers=list(tr), MaxItems=5))
        add(f"mix_{tag}", d, mix, header=[("transformer", t) for t in tr])
    # one record per block, straddling chunk boundaries
    strad = [rnd_bytes(rng, rng.choice([1, 500, 32700, 32760, 40000, 70000])) for _ in range(12)]
    d = write_file(strad, WriterOpts(MaxItems=1))
    add("straddle_none", d, strad)

    # --- flate block types ------------------------------------------------------
    text = b"".join(b"@r%d\nACGTACGTNNACGT\n+\nIIIIHHHGGG\n" % i for i in range(400))
    flate_variants = {
        "stored": dict(level=0, strategy=zlib.Z_DEFAULT_STRATEGY),
        "huffman_only": dict(level=6, strategy=zlib.Z_HUFFMAN_ONLY),
        "rle": dict(level=6, strategy=zlib.Z_RLE),
        "fixed": dict(level=6, strategy=zlib.Z_FIXED),
        "lvl1": dict(level=1, strategy=zlib.Z_DEFAULT_STRATEGY),
        "lvl9": dict(level=9, strategy=zlib.Z_DEFAULT_STRATEGY),
    }
    for vname, kw in flate_variants.items():
        for style in ("go", "zlib"):
            recs = [text[i:i + 97] for i in range(0, len(text), 97)]
            payload = F.packed_block_payload(recs)
            c = zlib.compressobj(kw["level"], zlib.DEFLATED, -15, 8, kw["strategy"])
            if style == "go":
                comp = c.compress(payload) + c.flush(zlib.Z_SYNC_FLUSH) + b"\x01\x00\x00\xff\xff"
            else:
                comp = c.compress(payload) + c.flush(zlib.Z_FINISH)
            assert zlib.decompress(comp, -15) == payload
            data = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", "flate")])]))
            data += F.chunk_block(F.MAGIC_PACKED, comp)
            add(f"flate_{vname}_{style}", data, recs, header=[("transformer", "flate")])
    # trailing garbage after the final block is ignored (Go inflater stops at BFINAL)
    recs = [b"abc", b"defg"]
    comp = zlib.compressobj(6, zlib.DEFLATED, -15)
    comp = comp.compress(F.packed_block_payload(recs)) + comp.flush(zlib.Z_FINISH) + b"GARBAGE"
    data = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", "flate")])]))
    data += F.chunk_block(F.MAGIC_PACKED, comp)
    add("flate_trailing_garbage", data, recs, header=[("transformer", "flate")])

    if have_zstd():
        # two frames in one block payload
        payload = F.packed_block_payload(mix[:6])
        comp = zstd_compress(payload[:len(payload) // 2], 3) + zstd_compress(payload[len(payload) // 2:], 3)
        data = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", "zstd")])]))
        data += F.chunk_block(F.MAGIC_PACKED, comp)
        add("zstd_two_frames", data, mix[:6], header=[("transformer", "zstd")], oracle_check=False)
        rle = [b"\x07" * 100000, b"x" * 5000]
        d = write_file(rle, WriterOpts(Transformers=["zstd"]))
        add("zstd_rle", d, rle, header=[("transformer", "zstd")], oracle_check=False)

    # --- random files with flushes (generateRandomRecordio, v2_test.go:458-481) ---
    for tr in ([[], ["flate"]] + ([["zstd"]] if have_zstd() else [])):
        r2 = random.Random(7)
        recs = []
        buf = io.BytesIO()
        w = Writer(buf, WriterOpts(Transformers=list(tr), KeyTrailer=True))
        for i in range(500):
            x = rnd_letters(r2, r2.randrange(1500) + 1)
            recs.append(x)
            w.Append(x)
            if r2.random() < 0.05:
                w.Flush()
        w.SetTrailer(b"Trailer")
        w.Finish()
        data = buf.getvalue()
        tag = tr[0] if tr else "none"
        hdr = [("transformer", t) for t in tr] + [("trailer", True)]
        # shard table (doShardedReads, v2_test.go:483-509): per-shard item counts
        shards = {}
        for nshard in ((1, 2, 3, 7, 1000, 1000000000) if (tag != "zstd" or ORACLE_ZSTD) else ()):
            stride = max(1, nshard // 10) if nshard >= 1000 else 1
            counts = []
            got = []
            for s in range(0, nshard, stride) if nshard < 1000 else range(0, nshard, stride):
                lim = min(s + stride, nshard)
                rr = O.scan(data, s, lim, nshard)
                assert rr.err == "" and rr.trailer == b"Trailer", (nshard, s, rr.err)
                counts.append(len(rr.items))
                got += rr.items
            assert got == recs, (tag, nshard)
            shards[str(nshard)] = {"stride": stride, "counts": counts}
        add(f"random_{tag}", data, recs, header=hdr, trailer=b"Trailer", shards=shards,
            oracle_check=(tag != "zstd"))

    # --- corruption cases (Appendix B of SURVEY.md) ---------------------------
    base = write_file([rnd_bytes(rng, 3000) for _ in range(40)], WriterOpts(MaxItems=12))
    recs40 = O.scan(base).items
    assert len(recs40) == 40
    nchunks = len(base) // F.CHUNK_SIZE  # header + 4 blocks of 1-2 chunks

    def chunk_hdr(data, c):
        o = c * F.CHUNK_SIZE
        return struct.unpack_from("<8sIIIII", data, o)

    def blocks_of(data):
        out = []
        c = 0
        while c * F.CHUNK_SIZE < len(data):
            total = chunk_hdr(data, c)[4]
            out.append((c, total))
            c += total
        return out

    blks = blocks_of(base)
    items_before = [0]
    for (c0, tot) in blks[1:]:
        r = O.scan(base[:(c0 + tot) * F.CHUNK_SIZE])
        items_before.append(len(r.items))

    def set_field(data, c, off, val):
        b = bytearray(data)
        struct.pack_into("<I", b, c * F.CHUNK_SIZE + off, val)
        return bytes(b)

    def fix_crc(data, c):
        b = bytearray(data)
        o = c * F.CHUNK_SIZE
        size = struct.unpack_from("<I", b, o + 16)[0]
        struct.pack_into("<I", b, o + 8, zlib.crc32(bytes(b[o + 12:o + 28 + size])))
        return bytes(b)

    c_last = blks[2][0]  # first chunk of block 2 (items of blocks 0,1 survive)
    # CRC flip in a payload byte
    b = bytearray(base)
    b[c_last * F.CHUNK_SIZE + 100] ^= 0x40
    stored = struct.unpack_from("<I", b, c_last * F.CHUNK_SIZE + 8)[0]
    size = struct.unpack_from("<I", b, c_last * F.CHUNK_SIZE + 16)[0]
    actual = zlib.crc32(bytes(b[c_last * F.CHUNK_SIZE + 12:c_last * F.CHUNK_SIZE + 28 + size]))
    add("err_crc", bytes(b), recs40[:items_before[1]],
        err=f"Chunk checksum mismatch, expect {actual}, got {stored}")
    # size > 32740
    d = set_field(base, c_last, 16, 40000)
    add("err_size", d, recs40[:items_before[1]], err="Invalid chunk size 40000")
    # index mismatch (CRC fixed so the structural check fires)
    two = [c for c, t in blks if t >= 2]
    cc = two[0] + 1
    d = fix_crc(set_field(base, cc, 24, 5), cc)
    bi = [i for i, (c0, t) in enumerate(blks) if c0 == two[0]][0]
    add("err_index", d, recs40[:items_before[bi - 1]] if bi > 1 else [],
        err="Chunk index mismatch, got 5, expect 1 for magic 2e7647eb34073c2e")
    # nchunk mismatch
    d = fix_crc(set_field(base, cc, 20, 9), cc)
    add("err_total", d, recs40[:items_before[bi - 1]] if bi > 1 else [],
        err=f"Chunk nchunk mismatch, got 9, expect {blks[bi][1]} for magic 2e7647eb34073c2e")
    # magic change in the middle of a block
    bb = bytearray(base)
    bb[cc * F.CHUNK_SIZE:cc * F.CHUNK_SIZE + 8] = F.MAGIC_TRAILER
    d = fix_crc(bytes(bb), cc)
    add("err_magic_changed", d, recs40[:items_before[bi - 1]] if bi > 1 else [],
        err="Magic number changed in the middle of a chunk sequence, got [46 118 71 235 52 7 60 46], "
            "expect [254 186 26 215 203 223 117 58]")
    # invalid block magic (legacy magic as a body block)
    bb = bytearray(base)
    for k in range(blks[2][1]):
        c = blks[2][0] + k
        bb[c * F.CHUNK_SIZE:c * F.CHUNK_SIZE + 8] = F.MAGIC_LEGACY_UNPACKED
    d = bytes(bb)
    for k in range(blks[2][1]):
        d = fix_crc(d, blks[2][0] + k)
    add("err_bad_magic", d, recs40[:items_before[1]],
        err="recordio: invalid magic number: [252 174 149 49 240 217 189 32]")
    # a header block inside the body is an invalid magic too
    d = base + F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([])]))
    add("err_header_in_body", d, recs40, err="recordio: invalid magic number: [217 225 217 92 194 22 4 247]")
    # a partial tail chunk that would start a new block lies past LimitShard's
    # whole-chunk limit (chunk.go:202-206): clean end, no error
    assert blks[-1][1] == 1
    d = base[:-1000]
    add("eof_truncated_tail", d, recs40[:items_before[len(blks) - 2]], err="",
        note="partial last chunk beyond ChunkScanner.limit is never read")
    # a partial chunk inside a block -> unexpected EOF (chunk.go:318-322)
    recs2 = [rnd_bytes(rng, 20000) for _ in range(4)]
    d2 = write_file(recs2, WriterOpts(MaxItems=1))  # 2 items (MaxItems + 1) = 2 chunks per block
    add("err_truncated", d2[:-5000], recs2[:2], err="unexpected EOF")
    # file ending at a chunk boundary inside a block: silent end (io.EOF ignored)
    last_c0, last_t = blks[-1]
    if last_t >= 2:
        d = base[:(last_c0 + 1) * F.CHUNK_SIZE]
        add("eof_mid_block", d, recs40[:items_before[len(blks) - 2]], err="")
    # bad varints / header length mismatch inside a valid chunk
    hdrblock = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([])]))
    ok_block = F.chunk_block(F.MAGIC_PACKED, F.packed_block_payload([b"ok"]))
    add("err_nitems_overflow", hdrblock + ok_block + F.chunk_block(F.MAGIC_PACKED, b"\xff" * 10 + b"\x02"),
        [b"ok"], err="recordio: failed to read number of packed items: -11")
    add("err_nitems_empty", hdrblock + ok_block + F.chunk_block(F.MAGIC_PACKED, b""), [b"ok"],
        err="recordio: failed to read number of packed items: 0")
    add("err_item_size_trunc", hdrblock + F.chunk_block(F.MAGIC_PACKED, b"\x03\x01\x01"), [],
        err="recordio: likely corrupt data, failed to read size of packed item 2: 0")
    add("err_item_size_ovf", hdrblock + F.chunk_block(F.MAGIC_PACKED, b"\x02\x01" + b"\x80" * 9 + b"\x02"), [],
        err="recordio: likely corrupt data, failed to read size of packed item 1: -10")
    add("err_block_size", hdrblock + ok_block + F.chunk_block(F.MAGIC_PACKED, b"\x02\x01\x05abcdefgh"), [b"ok"],
        err="recordio: corrupt block header, got block size 11, expected 9")
    add("zero_items_block", hdrblock + F.chunk_block(F.MAGIC_PACKED, b"\x00") + ok_block, [b"ok"])
    add("long_varint_item_count", hdrblock + F.chunk_block(F.MAGIC_PACKED, b"\x81\x80\x80\x80\x00" + b"\x00"),
        [b""])
    # flate errors
    fl_hdr = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", "flate")])]))
    good = F.chunk_block(F.MAGIC_PACKED, zlib.compressobj(6, zlib.DEFLATED, -15).compress(b"\x01\x02hi") +
                         b"")  # incomplete stream -> unexpected EOF
    add("err_flate_eof", fl_hdr + good, [], header=[("transformer", "flate")], err="unexpected EOF")
    add("err_flate_btype3", fl_hdr + F.chunk_block(F.MAGIC_PACKED, b"\x07\x00"), [], header=[("transformer", "flate")],
        err="flate: corrupt input before offset 1")
    add("err_flate_nlen", fl_hdr + F.chunk_block(F.MAGIC_PACKED, b"\x01\x05\x00\x00\x00hello"), [],
        header=[("transformer", "flate")], err="flate: corrupt input before offset 5")
    # legacy file (first block not a v2 header): the GPU scanner defers to the reference
    legacy = F.chunk_block(F.MAGIC_PACKED, F.packed_block_payload([b"Foo", b"Baz"]))
    add("legacy_magic", legacy, [], err="", note="v1-style magic: oracle reports legacy", oracle_check=False)
    # unknown transformer
    d = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", "nonexistent")])]))
    add("err_unknown_transformer", d, [], header=[("transformer", "nonexistent")],
        err="Transformer nonexistent not found")

    # transformer chains (registry.go:121-146: t0 applied first by the writer,
    # untransformed last): two and three stages, a trailer (transformed too),
    # and a corrupt inner stream whose chunk CRCs are valid
    if have_zstd():
        crecs = [rnd_bytes(rng, rng.choice([0, 1, 5, 300, 4000])) * rng.choice([1, 1, 30]) for _ in range(500)]
        for name, trs, tr in (("chain_zstd_flate", ["zstd", "flate"], b"chain trailer"),
                              ("chain_flate_zstd", ["flate 1", "zstd 3"], None),
                              ("chain3_flate_zstd_flate", ["flate", "zstd", "flate 9"], b"T3")):
            opts = WriterOpts(Transformers=list(trs), MaxItems=36, KeyTrailer=tr is not None)
            d = write_file(crecs, opts, trailer=tr)
            hdr = [("transformer", t) for t in trs] + ([("trailer", True)] if tr is not None else [])
            add(name, d, crecs, header=hdr, trailer=tr)
        # block 3 of chain_zstd_flate: one bit of its raw-DEFLATE stream flipped
        d = bytearray(write_file(crecs, WriterOpts(Transformers=["zstd", "flate"], MaxItems=36)))
        bl = blocks_of(bytes(d))
        c0, _ = bl[3]
        d[c0 * F.CHUNK_SIZE + 28 + 40] ^= 0x10
        d = fix_crc(bytes(d), c0)
        r = O.scan(d, read_trailer=False)
        assert r.err and r.items == crecs[:len(r.items)], r.err
        add("err_chain_inner", d, r.items, header=[("transformer", "zstd"), ("transformer", "flate")], err=r.err,
            read_trailer=False, note="error text from the oracle (the chain's flate stage)")

    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": CASES}, f, indent=1)
    total = sum(c["size"] for c in CASES)
    print(f"{len(CASES)} fixtures, {total / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
