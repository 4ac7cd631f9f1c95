"""Chunk headers rewritten with their CRC recomputed, so that only the chunk and
block structure is wrong (chunk.go:253-294, 316-345 checks it): size, total,
index, magic and flag fields set to other values, for each codec, with the
whole file in one span and with 256 KiB spans (blocks cut at span ends, the
scanner's spans ahead); and payload splices (bytes swapped between chunks of
different blocks, CRCs recomputed) for flate, zstd and multi-frame zstd. Every case must give the oracle's records and error,
and no kernel may read or write outside its block's regions (a GPU fault here
shows as a HIP error in place of the oracle's message)."""
import random
import struct
import zlib

import pytest

from conftest import oracle_has_zstd

pytestmark = pytest.mark.gpu

CK = 32768
MAX_PAYLOAD = CK - 28
MAGICS = [bytes.fromhex("2e7647eb34073c2e"),  # packed
          bytes.fromhex("d9e1d95cc21604f7"),  # header
          bytes.fromhex("feba1ad7cbdf753a")]  # trailer


def _file(trs, seed, multi_frame=False, text=False):
    from base_amd.recordio.writer import WriterOpts, write_file
    rng = random.Random(seed)
    if text:  # compressible records: Huffman / FSE-coded streams, long matches
        words = [rng.randbytes(rng.randrange(2, 9)).hex().encode() for _ in range(40)]
        recs = [b" ".join(rng.choice(words) for _ in range(rng.choice([0, 2, 60, 400, 3000]))) for _ in range(600)]
    else:
        recs = [rng.randbytes(rng.choice([0, 7, 500, 3000, 40000])) for _ in range(600)]
    opts = WriterOpts(Transformers=trs, MaxItems=rng.choice([5, 19, 60]))
    if not multi_frame:
        return write_file(recs, opts, trailer=b"FUZZ")
    # zstd blocks of several frames (ZSTD_decompress decodes concatenated frames,
    # recordiozstd.go:67-78): the writer's transform swapped for one that cuts
    # each block's payload into up to three frames
    import base_amd.recordio.writer as W
    from base_amd.recordio.codecs import zstd_compress
    orig = W.make_compressor

    def frames(b):
        k = len(b) // 3
        cuts = [0, k, 2 * k, len(b)] if k else [0, len(b)]
        return b"".join(zstd_compress(b[cuts[i]:cuts[i + 1]], 3) for i in range(len(cuts) - 1))
    W.make_compressor = lambda spec, style="go": frames
    try:
        return write_file(recs, opts, trailer=b"FUZZ")
    finally:
        W.make_compressor = orig


def _mutate(data, rng):
    b = bytearray(data)
    nck = len(b) // CK
    c = rng.randrange(1, nck)
    o = c * CK
    kind = rng.randrange(6)
    if kind == 0:  # size: smaller, larger, 0, or past the payload limit
        v = rng.choice([0, 1, rng.randrange(MAX_PAYLOAD + 1), MAX_PAYLOAD, MAX_PAYLOAD + 1])
        struct.pack_into("<I", b, o + 16, v)
    elif kind == 1:  # total
        v = rng.choice([0, 1, 2, rng.randrange(1, 40), struct.unpack_from("<I", b, o + 20)[0] + 1, 0xFFFFFFFF])
        struct.pack_into("<I", b, o + 20, v)
    elif kind == 2:  # index
        v = rng.choice([0, 1, rng.randrange(40), struct.unpack_from("<I", b, o + 24)[0] + 1, 0xFFFFFFFF])
        struct.pack_into("<I", b, o + 24, v)
    elif kind == 3:  # magic of another chunk kind
        b[o:o + 8] = rng.choice(MAGICS)
    elif kind == 4:  # total and index both (a block start claiming a long block)
        struct.pack_into("<I", b, o + 24, 0)
        struct.pack_into("<I", b, o + 20, rng.randrange(1, 60))
    else:  # flag word
        struct.pack_into("<I", b, o + 12, rng.getrandbits(32))
    size = struct.unpack_from("<I", b, o + 16)[0]
    if size <= MAX_PAYLOAD:
        struct.pack_into("<I", b, o + 8, zlib.crc32(bytes(b[o + 12:o + 28 + size])))
    return bytes(b), (c, kind)


def _scan(data, ctx):
    from base_amd.recordio import gpu
    sc = gpu.NewScanner(data, ctx=ctx)
    items = []
    while sc.Scan():
        items.append(sc.Get())
    e = sc.Finish()
    return items, ("" if e is None else str(e))


def _splice(data, rng):
    """Chunk payload bytes swapped between two chunks (usually of different
    blocks) with both CRCs recomputed: the chunk structure stays valid and only
    the compressed streams are wrong (a payload-level splice)."""
    b = bytearray(data)
    nck = len(b) // CK
    c1, c2 = rng.randrange(1, nck), rng.randrange(1, nck)
    s1 = struct.unpack_from("<I", b, c1 * CK + 16)[0]
    s2 = struct.unpack_from("<I", b, c2 * CK + 16)[0]
    n = min(s1, s2)
    if c1 != c2 and n > 0:
        ln = rng.randrange(1, n + 1)
        o1, o2 = rng.randrange(0, s1 - ln + 1), rng.randrange(0, s2 - ln + 1)
        a, z = c1 * CK + 28 + o1, c2 * CK + 28 + o2
        b[a:a + ln], b[z:z + ln] = bytes(b[z:z + ln]), bytes(b[a:a + ln])
    for c, sz in ((c1, s1), (c2, s2)):
        o = c * CK
        struct.pack_into("<I", b, o + 8, zlib.crc32(bytes(b[o + 12:o + 28 + sz])))
    return bytes(b), (c1, c2)


def _check(oracle, d, ctxs, what):
    ref = oracle.scan(d, read_trailer=False)
    for ctx in ctxs:
        items, err = _scan(d, ctx)
        assert err == ref.err, what
        assert items == ref.items, what


def test_flate_spliced_chunk_regression(oracle):
    """The case that made k_flate_tok fault (round 4): flate file 2, trial 11 --
    chunk 42's size rewritten to 1 with its CRC recomputed, so an 18-chunk block
    becomes irregular and its stream spliced; the reference reports the
    CorruptInputError (recordioflate.go:54-65). Every block also through the
    fallback Huffman pass."""
    from base_amd.recordio import gpu
    rng = random.Random(12)
    d = None
    for f in range(3):
        data = _file(["flate"], 100 * f + 1)
        for trial in range(25):
            dd, what = _mutate(data, rng)
            if (f, trial) == (2, 11):
                d = dd
                assert what == (42, 0)
    ctxs = [gpu.Context(0, max_span_bytes=64 << 20), gpu.Context(0, max_span_bytes=8 * CK),
            gpu.Context(0, max_span_bytes=64 << 20, flate_tok_only=True),
            gpu.Context(0, max_span_bytes=64 << 20, flate_one_wave=True)]
    try:
        _check(oracle, d, ctxs, "flate (42, 0)")
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("trs,multi", [(["flate"], False), (["zstd"], False), (["zstd"], True)])
def test_payload_splices_match_oracle(oracle, trs, multi):
    from base_amd.recordio import gpu
    if "zstd" in trs and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    rng = random.Random(31 + len(trs) + multi)
    ctxs = [gpu.Context(0, max_span_bytes=64 << 20), gpu.Context(0, max_span_bytes=8 * CK)]
    if trs == ["flate"]:  # (and the one-wave Huffman pass, which small spans do not take by default)
        ctxs.append(gpu.Context(0, max_span_bytes=64 << 20, flate_tok_only=True))
        ctxs.append(gpu.Context(0, max_span_bytes=64 << 20, flate_one_wave=True))
    try:
        for f in range(3):
            data = _file(trs, 300 * f + 7, multi_frame=multi, text=f > 0)
            for trial in range(25):
                d, what = _splice(data, rng)
                _check(oracle, d, ctxs, (trs, multi, f, trial, what))
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("trs", [[], ["flate"], ["zstd"]])
def test_structural_rewrites_match_oracle(oracle, trs):
    from base_amd.recordio import gpu
    if "zstd" in trs and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    rng = random.Random(11 + len(trs))
    small = gpu.Context(0, max_span_bytes=8 * CK)
    big = gpu.Context(0, max_span_bytes=64 << 20)
    # flate: also the one-wave Huffman pass (these small files take its 4-wave variant)
    one = gpu.Context(0, max_span_bytes=64 << 20, flate_one_wave=True) if trs == ["flate"] else None
    try:
        for f in range(3):
            data = _file(trs, 100 * f + len(trs))
            for trial in range(25):
                d, what = _mutate(data, rng)
                ref = oracle.scan(d, read_trailer=False)
                for ctx in (big, small) + ((one,) if one else ()):
                    items, err = _scan(d, ctx)
                    assert err == ref.err, (trs, f, trial, what, ctx is small)
                    assert items == ref.items, (trs, f, trial, what, ctx is small)
    finally:
        small.close()
        big.close()
        if one:
            one.close()
