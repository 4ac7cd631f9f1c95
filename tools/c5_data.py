"""Synthetic trailer-indexed flate recordio files for the multi-GPU workload
(BASELINE.json configs[4]).

C5 is 1024 files, each 64 MiB of C3 FASTQ-like records (tools/c3_data.py) in
flate blocks of 1024 records, written with KeyTrailer. The trailer's content is
application-defined in the reference (recordio/README.md:69-75); here it is a
block index: uvarint(nblocks) followed by uvarint deltas of the blocks' file
offsets (the first delta is the header block's size). N_BASE distinct base files
are generated; file f of the set is base f % N_BASE (its bytes are what a
reader sees; only the decode is timed, and generating 64 GiB of distinct FASTQ
would dominate the bench).
"""
from __future__ import annotations

import os
import sys
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

N_FILES = 1024
FILE_RECORD_BYTES = 64 << 20
PER_BLOCK = 1024
N_BASE = 8
SEED = 0x5EED0005


def file_nrec(record_bytes: int = FILE_RECORD_BYTES) -> int:
    return max(1, record_bytes // 320)


def make_index(offsets) -> bytes:
    """The trailer item: uvarint(nblocks) + uvarint offset deltas."""
    from base_amd.recordio import format as F
    out = bytearray(F.put_uvarint(len(offsets)))
    prev = 0
    for o in offsets:
        out += F.put_uvarint(o - prev)
        prev = o
    return bytes(out)


def parse_index(trailer: bytes):
    """Block file offsets from a trailer index (raises on a malformed one)."""
    from base_amd.recordio import format as F
    n, k = F.uvarint(trailer, 0)
    if k <= 0:
        raise ValueError("bad block count")
    pos = k
    offs, cur = [], 0
    for _ in range(n):
        d, k = F.uvarint(trailer, pos)
        if k <= 0:
            raise ValueError("bad block offset")
        pos += k
        cur += d
        offs.append(cur)
    if pos != len(trailer):
        raise ValueError("trailing bytes in the block index")
    return offs


def make_base(k: int, record_bytes: int = FILE_RECORD_BYTES, workers: int = 16):
    """Base file k: (bytes, n_records, record_bytes, block_offsets)."""
    import c3_data
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import flate_compress
    nrec = file_nrec(record_bytes)
    first0 = k * nrec
    jobs = [(first0 + b, min(PER_BLOCK, nrec - b), SEED) for b in range(0, nrec, PER_BLOCK)]
    hdr = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload(
        [F.marshal_header([("transformer", "flate"), ("trailer", True)])]))
    out = [hdr]
    offsets = []
    pos = len(hdr)
    rec_bytes = 0
    with ProcessPoolExecutor(max_workers=workers) as ex:
        for blk, nb, _ in ex.map(c3_data._block, jobs, chunksize=4):
            offsets.append(pos)
            out.append(blk)
            pos += len(blk)
            rec_bytes += nb
    index = make_index(offsets)
    out.append(F.chunk_block(F.MAGIC_TRAILER, flate_compress(F.packed_block_payload([index]), 6, "go")))
    return b"".join(out), nrec, rec_bytes, offsets


def base_records(k: int, record_bytes: int = FILE_RECORD_BYTES):
    import c3_data
    nrec = file_nrec(record_bytes)
    out = []
    for b in range(0, nrec, PER_BLOCK):
        out.extend(c3_data.records(k * nrec + b, min(PER_BLOCK, nrec - b), SEED))
    return out
