"""GPU parity of the block parse's fast paths (k_parse_lean, k_parse's small
header path) on crafted block shapes at their edges: item counts around the
256-size cap, straddlers at the edges of the chunk-boundary window, Go's
non-minimal uvarint encodings, empty blocks, and header corruptions whose chunk
CRCs are recomputed (so the parse, not the CRC check, meets them). Every case
against the oracle (parseChunksToItems, recordio/scannerv2.go:53-97), through
the host path (straddler descriptors) and the device path (straddlers written
into the span-shaped records buffer). Run on an MI355X: pytest -m gpu."""
import random
import struct

import pytest

from base_amd.recordio.format import (MAGIC_HEADER, MAGIC_PACKED, MAX_CHUNK_PAYLOAD, chunk_block, crc32_ieee,
                                      marshal_header, packed_block_payload, put_uvarint)

pytestmark = pytest.mark.gpu

W0 = MAX_CHUNK_PAYLOAD - 512  # kBndW0: the boundary window is payload [W0, W0 + 1024)


def nonmin(v, n):
    """v as an n-byte uvarint (Go's Uvarint accepts non-minimal encodings)."""
    out = bytearray()
    for i in range(n):
        b = (v >> (7 * i)) & 0x7F
        out.append(b | (0x80 if i < n - 1 else 0))
    assert v >> (7 * n) == 0
    return bytes(out)


def block(items, count_enc=None, size_enc=None):
    """Packed payload; count_enc / size_enc override the varint encodings."""
    hdr = bytearray(count_enc if count_enc is not None else put_uvarint(len(items)))
    for i, it in enumerate(items):
        hdr += size_enc(i, len(it)) if size_enc else put_uvarint(len(it))
    return bytes(hdr) + b"".join(items)


def make_file(payloads):
    return chunk_block(MAGIC_HEADER, packed_block_payload([marshal_header([])])) + b"".join(chunk_block(MAGIC_PACKED, p) for p in payloads)


def rnd(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def straddle_block(rng, S, V, tail=5000):
    """Three items: a filler, then X = payload [S, S + V), then a tail."""
    hv = 1 + 3 + len(put_uvarint(V)) + len(put_uvarint(tail))
    F = S - hv
    assert len(put_uvarint(F)) == 3
    return block([rnd(rng, F), rnd(rng, V), rnd(rng, tail)])  # X starts at hv + F = S


def valid_payloads(rng):
    ps = []
    for n in (1, 64, 65, 128, 192, 255, 256, 257, 300):  # around the lean path's 256-size cap
        ps.append(block([rnd(rng, rng.choice([0, 1, 7, 100, 127, 128, 300])) for _ in range(n)]))
    ps.append(block([rnd(rng, 256) for _ in range(253)]))  # C2's shape
    for S, V in ((W0, 1024), (W0, 1025), (W0 - 1, 600), (W0 - 1, 2), (MAX_CHUNK_PAYLOAD - 1, 2),
                 (MAX_CHUNK_PAYLOAD - 300, 300), (MAX_CHUNK_PAYLOAD, 10), (MAX_CHUNK_PAYLOAD - 3, 1027),
                 (MAX_CHUNK_PAYLOAD - 4, 8), (MAX_CHUNK_PAYLOAD - 2, 40000)):
        ps.append(straddle_block(rng, S, V))
    # a straddler at the second chunk boundary (outside the window: k_parse copies it)
    ps.append(block([rnd(rng, 2 * MAX_CHUNK_PAYLOAD - 100), rnd(rng, 300), rnd(rng, 10)]))
    items = [rnd(rng, 50) for _ in range(40)]
    ps.append(block(items, size_enc=lambda i, v: nonmin(v, 4)))  # 4-byte sizes: lean path
    ps.append(block(items, size_enc=lambda i, v: nonmin(v, 5 if i == 7 else 1 + i % 2)))  # one 5-byte size
    ps.append(block(items, count_enc=nonmin(40, 2)))  # count in 2 bytes
    ps.append(block(items, count_enc=nonmin(40, 3)))  # count in 3 bytes: k_parse
    ps.append(block([]))  # no items
    ps.append(block([b""] * 30))  # empty items
    ps.append(block([b""] * 5 + [rnd(rng, 40000)] + [b""] * 5))  # empty items after a straddler
    return ps


def device_items(ctx, data):
    import torch
    from base_amd.recordio import gpu
    hdr_chunks = struct.unpack_from("<I", data, 20)[0]
    body = data[hdr_chunks * 32768:]
    dev = torch.frombuffer(bytearray(body), dtype=torch.uint8).to("cuda:0")
    b = ctx.scan_device(dev.data_ptr(), len(body), file_off=hdr_chunks * 32768, is_file_end=True)
    return b, gpu.device_batch_items(b, body)


def scan_items(ctx, data):
    from base_amd.recordio import gpu
    sc = gpu.NewScanner(data, ctx=ctx)
    items = []
    while sc.Scan():
        items.append(sc.Get())
    err = sc.Err()
    sc.Finish()
    return items, "" if err is None else str(err)


def test_lean_shapes_match_oracle(gpu_ctx, oracle):
    from base_amd.recordio import gpu
    rng = random.Random(2026)
    ps = valid_payloads(rng)
    for order in range(3):  # each shape at several block positions (batch slots, waves)
        rng.shuffle(ps)
        data = make_file(ps)
        ref = oracle.scan(data, read_trailer=False)
        assert ref.err == ""
        items, err = scan_items(gpu_ctx, data)
        assert err == "" and items == ref.items, order
        b, ditems = device_items(gpu_ctx, data)
        assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
        assert ditems == ref.items, order


def fix_crcs(buf):
    for c in range(len(buf) // 32768):
        o = c * 32768
        size = struct.unpack_from("<I", buf, o + 16)[0]
        if size <= MAX_CHUNK_PAYLOAD:
            struct.pack_into("<I", buf, o + 8, crc32_ieee(bytes(buf[o + 12:o + 28 + size])))


def test_header_corruptions_match_oracle(gpu_ctx, oracle):
    """Single-byte changes inside packed headers, CRCs recomputed: the parse
    meets every malformed header (sizes vs block length, varint lengths, counts)
    and must give the reference's first error after the same items."""
    rng = random.Random(5)
    ps = [block([rnd(rng, 256) for _ in range(253)]) for _ in range(6)]
    ps += [block([rnd(rng, rng.choice([1, 90, 200])) for _ in range(rng.choice([10, 255, 256, 257]))])
           for _ in range(6)]
    data = make_file(ps)
    starts, off = [], 32768
    for p in ps:
        starts.append(off)
        off += ((len(p) - 1) // MAX_CHUNK_PAYLOAD + 1) * 32768
    for trial in range(80):
        buf = bytearray(data)
        bi = rng.randrange(len(ps))
        o = starts[bi] + 28 + rng.randrange(min(600, len(ps[bi])))
        if rng.random() < 0.5:
            buf[o] ^= 1 << rng.randrange(8)
        else:
            buf[o] = rng.choice([0x00, 0x7F, 0x80, 0xFF])
        fix_crcs(buf)
        d = bytes(buf)
        ref = oracle.scan(d, read_trailer=False)
        items, err = scan_items(gpu_ctx, d)
        assert err == ref.err, (trial, bi, o)
        assert items == ref.items, (trial, bi, o)
