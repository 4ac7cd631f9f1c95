"""Chunk headers rewritten with their CRC recomputed, so that only the chunk and
block structure is wrong (chunk.go:253-294, 316-345 checks it): size, total,
index, magic and flag fields set to other values, for each codec, with the
whole file in one span and with 256 KiB spans (blocks cut at span ends, the
scanner's spans ahead). Every case must give the oracle's records and error,
and no kernel may read or write outside its block's regions (a GPU fault here
shows as a HIP error in place of the oracle's message)."""
import os
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


def _file(trs, seed):
    from base_amd.recordio.writer import WriterOpts, write_file
    rng = random.Random(seed)
    recs = [rng.randbytes(rng.choice([0, 7, 500, 3000, 40000])) for _ in range(600)]
    return write_file(recs, WriterOpts(Transformers=trs, MaxItems=rng.choice([5, 19, 60])), trailer=b"FUZZ")


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


@pytest.mark.parametrize("trs", [[], ["flate"], ["zstd"]])
def test_structural_rewrites_match_oracle(oracle, trs):
    from base_amd.recordio import gpu
    if "zstd" in trs and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle not built")
    if trs and os.environ.get("RIO_FUZZ_CODECS") != "1":
        # Known open fault: a flate block whose middle chunk's size
        # was rewritten with its CRC makes k_flate_tok fault (file 2, trial 11),
        # which ends the process's GPU context for every later test.
        pytest.skip("codec cases: RIO_FUZZ_CODECS=1 (an open GPU fault, DESIGN.md §7)")
    rng = random.Random(11 + len(trs))
    small = gpu.Context(0, max_span_bytes=8 * CK)
    big = gpu.Context(0, max_span_bytes=64 << 20)
    try:
        for f in range(3):
            data = _file(trs, 100 * f + len(trs))
            for trial in range(25):
                d, what = _mutate(data, rng)
                ref = oracle.scan(d, read_trailer=False)
                for ctx in (big, small):
                    items, err = _scan(d, ctx)
                    assert err == ref.err, (trs, f, trial, what, ctx is small)
                    assert items == ref.items, (trs, f, trial, what, ctx is small)
    finally:
        small.close()
        big.close()
