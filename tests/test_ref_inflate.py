"""The oracle's DEFLATE restatement (oracle/inflate.c, Go compress/flate
semantics -- the decoder klauspost/compress v1.8.6 forks, which the reference's
FlateUncompress calls, recordioflate.go:54-65) against a DEFLATE decoder that
ships inside the reference: its vendored libdeflate v1.0
(compress/libdeflate/deflate_decompress.c), compiled from the reference tree
into oracle/_ref/ by `make -C oracle ref` (tests only; never shipped).

Two independent implementations of RFC 1951 must agree byte for byte on every
stream one of them accepts as a complete stream: every flate block of the
golden fixtures, C3-style and edge-case payloads compressed by zlib and in
Go's Writer.Close framing at levels 0, 1, 6, 9 and HuffmanOnly, and random
corruptions of a level-6 stream. Where they may legitimately
differ is Go-specific error behaviour (the inflater reports the offset of
the first bad symbol, a truncated stream is io.ErrUnexpectedEOF): those
parts are pinned by the Go-framed fixtures, not here.
"""
import os
import random
import struct
import sys
import zlib

import pytest

from conftest import ROOT, golden_bytes

sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def ref(oracle):
    if not oracle.build_ref():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    return oracle


def _flate_blocks(data):
    out = []
    c = struct.unpack_from("<I", data, 20)[0] if len(data) >= 32768 else 0
    while (c + 1) * 32768 <= len(data):
        size, total, index = struct.unpack_from("<III", data, c * 32768 + 16)
        if index != 0 or total == 0:
            break
        if data[c * 32768:c * 32768 + 8] == bytes.fromhex("2e7647eb34073c2e"):
            out.append(b"".join(data[(c + k) * 32768 + 28:(c + k) * 32768 + 28 +
                                     struct.unpack_from("<I", data, (c + k) * 32768 + 16)[0]]
                                for k in range(total)))
        c += total
    return out


def _agree(ref, comp, seen):
    rc_o, out_o, _ = ref.inflate(comp, cap=1 << 22)
    rc_r, out_r, _ = ref.ref_inflate(comp, cap=1 << 22)
    if rc_o == 0 or rc_r == 0:
        seen["ok"] += 1
        assert rc_o == 0 and rc_r == 0 and out_o == out_r
    else:
        seen["err"] += 1


def test_golden_flate_streams(ref, manifest):
    seen = {"ok": 0, "err": 0}
    for case in manifest:
        if not any(k == "transformer" and v.split()[0] == "flate" for k, t, v in case["header"]):
            continue
        if len([1 for k, t, v in case["header"] if k == "transformer"]) != 1:
            continue
        for comp in _flate_blocks(golden_bytes(case)):
            _agree(ref, comp, seen)
    assert seen["ok"] >= 20


def test_encoder_and_zlib_streams(ref):
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import flate_compress
    import c3_data
    rng = random.Random(3)
    seen = {"ok": 0, "err": 0}
    payloads = [F.packed_block_payload(c3_data.records(i * 300, 300)) for i in range(4)]
    payloads += [bytes(rng.getrandbits(8) for _ in range(n)) for n in (0, 1, 100, 70000)]
    payloads += [b"ab" * 50000, b"\0" * 100000]
    for p in payloads:
        for lvl in (0, 1, 6, 9, -2):
            for style in ("go", "zlib"):
                _agree(ref, flate_compress(p, lvl, style), seen)
    assert seen["ok"] == len(payloads) * 10


def test_corruptions_agree_on_accepted_streams(ref):
    """Random bit flips and truncations: whenever either decoder accepts the
    stream, both do and produce the same bytes."""
    import c3_data
    from base_amd.recordio import format as F
    rng = random.Random(11)
    base = zlib.compressobj(6, zlib.DEFLATED, -15)
    payload = F.packed_block_payload(c3_data.records(0, 200))
    comp = base.compress(payload) + base.flush()
    seen = {"ok": 0, "err": 0}
    for trial in range(400):
        b = bytearray(comp)
        if trial % 5 == 4:
            del b[rng.randrange(len(b)):]
        else:
            for _ in range(rng.randrange(1, 3)):
                i = rng.randrange(len(b))
                b[i] ^= 1 << rng.randrange(8)
        _agree(ref, bytes(b), seen)
    assert seen["err"] > 100 and seen["ok"] > 0
