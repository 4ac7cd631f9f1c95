"""Synthetic FASTQ-like recordio for the flate workload.

Record: b"@r<id>\\n" + 150 bases from {A,C,G,T} (N at 0.1 %) + b"\\n+\\n" + 150
Phred+33 quality characters from a first-order Markov walk, ~320 B. Blocks of
`per_block` records (the reference benchmark's --records-per-block default,
1024), each block payload raw-DEFLATE compressed at level 6 ending like Go's
flate Writer.Close (sync flush + empty final stored block). Seed 0x5EED0003.
"""
from __future__ import annotations

import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SEED = 0x5EED0003
READ_LEN = 150


def records(first: int, n: int, seed: int = SEED):
    """Records first .. first+n-1 (deterministic per record range)."""
    rng = np.random.default_rng([seed, first])
    bases = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=(n, READ_LEN))]
    bases[rng.random((n, READ_LEN)) < 0.001] = ord("N")
    steps = rng.integers(-3, 4, size=(n, READ_LEN))
    q0 = rng.integers(20, 41, size=n)
    q = np.clip(q0[:, None] + np.cumsum(steps, axis=1), 2, 41).astype(np.uint8) + 33
    out = []
    for i in range(n):
        out.append(b"@r%d\n" % (first + i) + bases[i].tobytes() + b"\n+\n" + q[i].tobytes())
    return out


def _block(args):
    first, n, seed = args
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import flate_compress
    recs = records(first, n, seed)
    comp = flate_compress(F.packed_block_payload(recs), 6, "go")
    return F.chunk_block(F.MAGIC_PACKED, comp), sum(len(r) for r in recs), n


def make_file(target_bytes: int, per_block: int = 1024, seed: int = SEED, workers: int = 8):
    """A flate recordio file of about target_bytes of records.
    Returns (bytes, n_records, record_bytes)."""
    from base_amd.recordio import format as F
    nrec = max(1, target_bytes // 320)
    jobs = [(b, min(per_block, nrec - b), seed) for b in range(0, nrec, per_block)]
    out = [F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", "flate")])]))]
    rec_bytes = 0
    with ProcessPoolExecutor(max_workers=workers) as ex:
        for blk, nb, _ in ex.map(_block, jobs, chunksize=4):
            out.append(blk)
            rec_bytes += nb
    return b"".join(out), nrec, rec_bytes
