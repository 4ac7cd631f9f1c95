"""Split copy pass (DESIGN.md "split copy pass"): a span of few large flate
blocks -- the writer's default MaxItems = 16384 (recordio/writerv2.go:28-29)
gives ~5 MB blocks -- has its blocks' copy passes cut into segments that are
copied at the same time, the later ones as u16 symbols resolved afterwards.
Every record must equal the generator's and the unsplit decode's, for DEFLATE
streams of every block type (stored, fixed, dynamic; levels 0-9) and for long
runs that cross the segment boundaries.

A context's first flate scan sizes the split scratch between the Huffman pass
and the copy pass (round 4; before, the first scan copied its blocks whole and
only later scans split), so the first scan splits as well as the second. Both
are checked, and the split count is read back (rio_flate_split_blocks) so the
test fails if nothing was split.
"""
import os
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, "tools"))

CH = 32768


def _deflate(raw, level):
    """Go Writer.Close framing; level "fixed": fixed-Huffman blocks only (zlib Z_FIXED)."""
    import zlib
    from base_amd.recordio.codecs import flate_compress
    if level != "fixed":
        return flate_compress(raw, level, "go")
    c = zlib.compressobj(6, zlib.DEFLATED, -15, 8, zlib.Z_FIXED)
    return c.compress(raw) + c.flush(zlib.Z_SYNC_FLUSH) + b"\x01\x00\x00\xff\xff"


def _file(blocks):
    """A flate recordio file of the given blocks (lists of records), level per block."""
    from base_amd.recordio import format as F
    out = [F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", "flate")])]))]
    for recs, level in blocks:
        out.append(F.chunk_block(F.MAGIC_PACKED, _deflate(F.packed_block_payload(recs), level)))
    return b"".join(out)


def _scans(data, nrec, split, runs=2):
    """The items of `runs` scans of the file's body on one context, and the split
    block counts."""
    import torch
    from base_amd.recordio import gpu
    body = data[CH:]
    dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda:0")
    ctx = gpu.Context(0, max_span_bytes=len(data), max_items=nrec + 1024, flate_split=split)
    items, nsplit = [], []
    try:
        for _ in range(runs):
            b = ctx.scan_device(dev.data_ptr() + CH, len(body), file_off=CH, is_file_end=True,
                                codec=gpu.RIO_CODEC_FLATE)
            assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
            items.append(gpu.device_batch_items(b, body))
            nsplit.append(ctx.flate_split_blocks())
    finally:
        ctx.close()
    return items, nsplit


def _check(blocks):
    want = [r for recs, _ in blocks for r in recs]
    data = _file(blocks)
    got, nsplit = _scans(data, len(want), True)
    assert nsplit[0] > 0 and nsplit[1] > 0, nsplit  # the first run sizes the scratch mid-run and splits
    for items in got:
        assert len(items) == len(want)
        assert items == want
    whole, n0 = _scans(data, len(want), False, runs=1)
    assert n0 == [0] and whole[0] == want
    return nsplit[1]


@pytest.mark.parametrize("level", [1, 6, 9])
def test_split_default_maxitems(level):
    """Blocks of MaxItems + 1 = 16,385 FASTQ records (~5 MB), a short last block."""
    import c3_data
    per = 16385
    blocks = [(c3_data.records(first, per), level) for first in range(0, 3 * per, per)]
    blocks.append((c3_data.records(3 * per, 1000), level))
    assert _check(blocks) >= 3


def test_split_stored_and_fixed():
    """Stored blocks (level 0: 3-byte literal tokens) and fixed-Huffman streams
    split the same way."""
    import c3_data
    blocks = [(c3_data.records(0, 6000), 0), (c3_data.records(6000, 6000), "fixed"),
              (c3_data.records(12000, 6000), 6)]
    assert _check(blocks) >= 2


def test_split_runs_across_segments():
    """Long runs and near matches: a match's bytes chain back through the
    segment boundary (a run of dist 1 starting before it, 258-byte matches)."""
    import random
    import c3_data
    rnd = random.Random(7)
    recs = []
    for i in range(12000):
        r = rnd.random()
        if r < 0.3:
            recs.append(bytes([65 + i % 26]) * rnd.randrange(200, 3000))  # runs
        elif r < 0.5:
            recs.append(recs[-1] if recs else b"x")  # whole-record repeats
        else:
            recs.extend(c3_data.records(i, 1))
    assert _check([(recs, 6), (recs[::-1], 9)]) >= 1
