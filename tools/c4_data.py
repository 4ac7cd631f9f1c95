"""Synthetic zstd recordio for the zstd workload.

Record sizes are log-uniform on [64 B, 64 KiB] (seed 0x5EED0004); the content is
C3-style FASTQ text (tools/c3_data.py) cut to each size. The writer flushes a
block once it holds >= 1 MiB of record bytes; each block payload is one zstd
frame at level 5 (the DataDog default, compress/zstd/zstd_cgo.go:20-22) written
by ZSTD_compress, as recordiozstd does (recordiozstd.go:23-36).
Every block is deterministic in (seed, block index).
"""
from __future__ import annotations

import math
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

SEED = 0x5EED0004
BLOCK_BYTES = 1 << 20
LEVEL = 5


def block_records(b: int, seed: int = SEED):
    """The records of block b: sizes log-uniform in [64, 65536] until the block
    holds >= 1 MiB, content cut from a FASTQ text stream."""
    import c3_data
    rng = np.random.default_rng([seed, b])
    sizes = []
    tot = 0
    while tot < BLOCK_BYTES:
        s = int(math.exp(rng.uniform(math.log(64), math.log(65536))))
        sizes.append(s)
        tot += s
    text = b"\n".join(c3_data.records(b * 4096, tot // 300 + 2, seed=seed))
    out = []
    pos = 0
    for s in sizes:
        out.append(text[pos:pos + s])
        pos += s
    return out


def _block(args):
    b, seed = args
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import zstd_compress
    recs = block_records(b, seed)
    comp = zstd_compress(F.packed_block_payload(recs), LEVEL)
    return F.chunk_block(F.MAGIC_PACKED, comp), sum(len(r) for r in recs), len(recs)


def make_file(target_bytes: int, seed: int = SEED, workers: int = 8):
    """A zstd recordio file of about target_bytes of records.
    Returns (bytes, n_blocks, n_records, record_bytes)."""
    from base_amd.recordio import format as F
    nblk = max(1, target_bytes // BLOCK_BYTES)
    out = [F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", "zstd")])]))]
    rec_bytes = nrec = 0
    jobs = [(b, seed) for b in range(nblk)]
    if workers <= 1:  # in-process (e.g. under a profiler that cannot follow a process pool)
        results = map(_block, jobs)
    else:
        ex = ProcessPoolExecutor(max_workers=workers)
        results = ex.map(_block, jobs, chunksize=2)
    for blk, nb, ni in results:
        out.append(blk)
        rec_bytes += nb
        nrec += ni
    if workers > 1:
        ex.shutdown()
    return b"".join(out), nblk, nrec, rec_bytes


def all_records(nblk: int, seed: int = SEED):
    out = []
    for b in range(nblk):
        out.extend(block_records(b, seed))
    return out
