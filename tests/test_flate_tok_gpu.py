"""The fallback Huffman pass (k_flate_tok) under load on valid data.

k_flate_sync (a wave per block) decodes almost every block of a real file; the
blocks it declines -- no self-synchronisation in 8 rounds (near-uniform codes,
e.g. compressed random bytes), a full token column, > 2^28 bits -- go to
k_flate_tok. RIO_CFG_FLATE_TOK_ONLY makes k_flate_sync decline every block, so
the whole C3 base file (tools/c3_data.py, configs[2]'s records, level-6 Go-framed
DEFLATE) runs through k_flate_tok at 1,024 and 16,385 records per block (the
writer's default MaxItems, writerv2.go:28-29): every record against the
generator, and three blocks against the oracle (recordioflate.go:54-65).
"""
import hashlib
import os
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.parametrize("per_block", [1024, 16385])
def test_c3_every_block_through_k_flate_tok(oracle, per_block):
    import c3_data
    import torch
    from base_amd.recordio import gpu
    data, nrec, rec_bytes = c3_data.make_file(128 << 20, per_block, workers=16)
    want = []
    for first in range(0, nrec, per_block):
        want.extend(c3_data.records(first, min(per_block, nrec - first)))
    body = data[32768:]
    dev = torch.frombuffer(bytearray(body), dtype=torch.uint8).to("cuda:0")
    ctx = gpu.Context(0, max_span_bytes=len(body) + 32768, flate_tok_only=True)
    try:
        b = ctx.scan_device(dev.data_ptr(), len(body), file_off=32768, is_file_end=True, codec=gpu.RIO_CODEC_FLATE)
        assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
        got = gpu.device_batch_items(b, body)
        assert len(got) == nrec
        assert [len(x) for x in got] == [len(x) for x in want]
        assert hashlib.sha256(b"".join(got)).digest() == hashlib.sha256(b"".join(want)).digest()
        assert sum(map(len, got)) == rec_bytes
        # three blocks file-shaped (header + block) through the scanner, against the oracle
        hdr = data[:32768]
        pos, blocks = 32768, []
        while pos < len(data):
            total = int.from_bytes(data[pos + 20:pos + 24], "little")
            blocks.append(data[pos:pos + total * 32768])
            pos += total * 32768
        for k in (0, len(blocks) // 2, len(blocks) - 1):
            ref = oracle.scan(hdr + blocks[k])
            assert ref.err == ""
            sc = gpu.NewScanner(hdr + blocks[k], ctx=ctx)
            items = []
            while sc.Scan():
                items.append(sc.Get())
            assert sc.Finish() is None and items == ref.items
    finally:
        ctx.close()
