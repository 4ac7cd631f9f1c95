"""zstd decode parity against libzstd itself -- the library the reference's
"zstd" transformer links (recordiozstd.go:67-78 -> compress/zstd/zstd_cgo.go
:34-41 -> DataDog/zstd v1.4.1, a cgo wrapper of libzstd's ZSTD_decompress).
This image holds libzstd 1.4.9 (/opt/conda/lib/libzstd.so.1), loaded with
ctypes as the checker.

Valid frames decode identically by the format; corrupt frames are where
implementations differ, so both the CPU oracle (oracle/zstd_dec.c) and the GPU
path (codec_zstd.hip's fast passes, then zstd_exact.h for every block they
decline or find corrupt) are held to libzstd's outcome on mutated frames: the
same accept / reject, the same bytes when accepted, the same error name
(ZSTD_getErrorName) when rejected.

Mutations: bit flips and byte replacements anywhere in the frame, truncation,
spliced garbage; frames from levels 1-19 with and without checksum / content
size, over FASTQ-like text, small and large alphabets and incompressible data
(single- and four-stream literals, both Huffman decoders of libzstd)."""
import ctypes
import os
import random

import pytest

from conftest import oracle_has_zstd


def _lib():
    from base_amd.recordio import codecs as C
    L = C._libzstd()
    L.ZSTD_getErrorName.restype = ctypes.c_char_p
    L.ZSTD_getErrorName.argtypes = [ctypes.c_size_t]
    return L


def libzstd(data: bytes, cap: int = 1 << 24):
    """(bytes, "") or (None, ZSTD_getErrorName)."""
    L = _lib()
    dst = ctypes.create_string_buffer(cap)
    n = L.ZSTD_decompress(dst, cap, data, len(data))
    if L.ZSTD_isError(n):
        return None, L.ZSTD_getErrorName(n).decode()
    return dst.raw[:n], ""


def _payload(rng):
    from base_amd.recordio import format as F
    k = rng.randrange(5)
    if k == 0:
        words = [bytes(rng.choice(b"ACGTN@+\n") for _ in range(rng.randrange(1, 12))) for _ in range(50)]
        return F.packed_block_payload([b"".join(rng.choice(words) for _ in range(rng.randrange(0, 60)))
                                       for _ in range(rng.randrange(5, 120))])
    if k == 1:
        return bytes(rng.choice(b"ACGT") for _ in range(rng.randrange(10, 40000)))
    if k == 2:
        alpha = bytes(rng.randrange(256) for _ in range(rng.randrange(2, 60)))
        return bytes(rng.choice(alpha) for _ in range(rng.randrange(10, 140000)))
    if k == 3:
        return os.urandom(rng.randrange(1, 3000)) * rng.randrange(1, 20)
    return bytes(rng.randrange(40, 48) for _ in range(rng.randrange(100, 300000)))


def mutated_frames(seed: int, n: int):
    """(frame bytes) x n: compressed then mutated (never empty)."""
    from base_amd.recordio.codecs import zstd_compress_ex
    rng = random.Random(seed)
    out = []
    while len(out) < n:
        comp = bytearray(zstd_compress_ex(_payload(rng), rng.choice([1, 3, 5, 9, 19]), rng.random() < 0.3,
                                          rng.random() < 0.7))
        kind = rng.randrange(6)
        if kind <= 2:
            for _ in range(rng.choice([1, 1, 2, 3])):
                i = rng.randrange(6, len(comp)) if len(comp) > 6 else 0
                comp[i] ^= 1 << rng.randrange(8)
        elif kind == 3:
            del comp[rng.randrange(len(comp)):]
        elif kind == 4:
            comp[rng.randrange(len(comp))] = rng.randrange(256)
        else:
            i = rng.randrange(len(comp))
            comp[i:i + rng.randrange(1, 6)] = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 6)))
        if comp:
            out.append(bytes(comp))
    return out


def oracle_decompress(oracle, comp):
    """The oracle with DataDog's growing output buffer (OUTPUT_FULL -> retry)."""
    cap = 1 << 22
    while True:
        rc, got, gerr = oracle.zstd_decompress(comp, cap)
        if rc != 3 or cap >= 1 << 28:
            return rc, got, gerr
        cap *= 4


def test_oracle_matches_libzstd(oracle):
    """The CPU oracle against libzstd on 500 mutated frames (a 48,000-frame run
    of the same generator with other seeds found no difference)."""
    if not oracle_has_zstd(oracle):
        pytest.skip("libzstd / zstd oracle unavailable")
    outcomes = set()
    for i, comp in enumerate(mutated_frames(101, 500)):
        want, werr = libzstd(comp)
        rc, got, gerr = oracle_decompress(oracle, comp)
        if want is None:
            assert rc != 0 and gerr == werr, (i, gerr, werr)
        else:
            assert rc == 0 and got == want, (i, rc, gerr)
        outcomes.add(werr)
    assert len(outcomes) >= 4, outcomes  # accepted + several error kinds


@pytest.mark.gpu
def test_gpu_decode_block_matches_libzstd(gpu_ctx, oracle):
    """rio_decode_block (GPU) against libzstd on 400 mutated frames, each split
    into chunk-sized payloads as the scanner would hand them over."""
    from base_amd.recordio import gpu
    if not oracle_has_zstd(oracle):
        pytest.skip("libzstd unavailable")
    seen = set()
    for i, comp in enumerate(mutated_frames(202, 400)):
        want, werr = libzstd(comp)
        pays = [comp[k:k + 32740] for k in range(0, len(comp), 32740)]
        try:
            got = gpu_ctx.decode_block(pays, gpu.RIO_CODEC_ZSTD)
            assert want is not None and got == want, (i, werr)
            seen.add("ok")
        except gpu.RecordioError as e:
            assert want is None and str(e) == werr, (i, str(e), werr)
            seen.add(werr)
    assert len(seen) >= 4, seen


@pytest.mark.gpu
def test_gpu_scan_corrupt_zstd_blocks(gpu_ctx, oracle):
    """The scanner path: a good block, then a mutated one. Items and the error
    text equal the oracle's, whose zstd decode equals libzstd's."""
    from base_amd.recordio import format as F
    from base_amd.recordio import gpu
    from base_amd.recordio.codecs import zstd_compress
    if not oracle_has_zstd(oracle):
        pytest.skip("libzstd unavailable")
    hdr = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", "zstd")])]))
    good = F.chunk_block(F.MAGIC_PACKED, zstd_compress(F.packed_block_payload([b"a" * 10, b"bc" * 50]), 5))
    errs = set()
    for i, comp in enumerate(mutated_frames(303, 150)):
        want, werr = libzstd(comp)
        rc, got, gerr = oracle_decompress(oracle, comp)
        assert (rc == 0) == (want is not None) and (got == want if rc == 0 else gerr == werr), i
        data = hdr + good + F.chunk_block(F.MAGIC_PACKED, comp)
        sc = gpu.NewScanner(data, ctx=gpu_ctx)
        items = []
        while sc.Scan():
            items.append(sc.Get())
        e = sc.Finish()
        ref = oracle.scan(data)
        assert ("" if e is None else str(e)) == ref.err and items == ref.items, (i, e, ref.err)
        errs.add(ref.err)
    assert len(errs) >= 3, errs
