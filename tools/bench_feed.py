"""Host feed: end-to-end scanner rates with the read-ahead.

The scanner layer (rio_scanner_*) reads the file through its reader callback
into pinned staging, decodes span by span and hands back record views; with
the read-ahead a thread reads the next span's bytes while the GPU decodes and
the caller consumes the current one.

  C2 (none, 259 MB file): one scanner, spans of --span-mib (several spans:
  the read-ahead overlaps), and one span holding the whole file (nothing to
  overlap) for comparison. Records are taken with rio_scanner_next_batch
  (views, no Python copy).
  C3 many files (flate, the C5 base files, 64 MiB of records each): T threads,
  each with its own rio_ctx (own HIP stream) and scanner, files round-robin.
Output: one JSON line. GiB/s of file bytes in.

  python tools/bench_feed.py [--span-mib 64] [--threads 1,4,8] [--files 8]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def scan_count(gpu, data, ctx, batch=1 << 16):
    """Scan a whole file through the scanner; (records, record bytes)."""
    import numpy as np
    L = ctx.L
    sc = gpu.NewScanner(data if isinstance(data, gpu.MemorySource) else gpu.MemorySource(data), ctx=ctx)
    ptrs = (ctypes.c_void_p * batch)()
    lens = (ctypes.c_uint64 * batch)()
    lv = np.ctypeslib.as_array(lens)
    n = tot = 0
    while True:
        k = L.rio_scanner_next_batch(sc.h, ptrs, lens, batch)
        if k <= 0:
            break
        n += k
        tot += int(lv[:k].sum())
    err = sc.Finish()
    assert err is None, err
    return n, tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--span-mib", type=int, default=64)
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--files-per-batch", type=int, default=8)
    ap.add_argument("--ctx-threads", default="1,2")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import bench
    import c5_data
    from base_amd.recordio import gpu

    out = {"metric": "recordio scan GiB/s end-to-end (host file bytes in, record views out)", "unit": "GiB/s"}
    data = gpu.MemorySource(bench.make_c2_file()[0])
    c2 = {}
    for name, span in (("spans", args.span_mib << 20), ("one_span", data.size + (1 << 20))):
        ctx = gpu.Context(0, max_span_bytes=span)
        scan_count(gpu, data, ctx)  # warm: buffers sized
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            n, tot = scan_count(gpu, data, ctx)
            ts.append(time.perf_counter() - t0)
        t = sorted(ts)[len(ts) // 2]
        c2[name] = {"GiBs": round(data.size / t / 2 ** 30, 2), "wall_ms": round(t * 1e3, 1), "records": n,
                    "span_bytes": span}
        ctx.close()
    out["c2_file_bytes"] = data.size
    out["c2"] = c2
    files = [gpu.MemorySource(c5_data.make_base(k % c5_data.N_BASE)[0]) for k in range(args.files)]
    c3 = {}
    for T in [int(x) for x in args.threads.split(",")]:
        ctxs = [gpu.Context(0) for _ in range(T)]
        for c in ctxs:  # warm
            scan_count(gpu, files[0], c)
        res = [0] * T

        def work(w):
            for i in range(w, len(files), T):
                res[w] += scan_count(gpu, files[i], ctxs[w])[0]
        t0 = time.perf_counter()
        th = [threading.Thread(target=work, args=(w,)) for w in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        t = time.perf_counter() - t0
        c3["threads_%d" % T] = {"GiBs": round(sum(f.size for f in files) / t / 2 ** 30, 2), "wall_ms": round(t * 1e3, 1),
                                "records": sum(res)}
        for c in ctxs:
            c.close()
    out["c3_many_files"] = {"files": len(files), "file_bytes": sum(f.size for f in files), **c3}
    # the same files as batches of whole file bodies (each body: the blocks
    # between the header and the trailer, from the file's trailer index), one
    # rio_scan_span (H2D, decode, D2H) per batch, two ctx threads alternating
    from base_amd.recordio import shard
    import numpy as np
    import torch
    bodies = []
    for f in files:
        raw = f._arr.tobytes()
        sc = gpu.NewScanner(f, ctx=gpu.default_context(0))
        lo = c5_data.parse_index(sc.Trailer())[0]
        assert sc.Finish() is None
        bodies.append(raw[lo:shard.trailer_offset(raw)])
    per = max(1, args.files_per_batch)
    batches = [bodies[i:i + per] for i in range(0, len(bodies), per)]
    pinned = [torch.frombuffer(bytearray(b"".join(bt)), dtype=torch.uint8).pin_memory() for bt in batches]
    span = max(p.numel() for p in pinned)
    nrec_b = [None] * len(batches)
    c3b = {}
    for T in [int(x) for x in args.ctx_threads.split(",")]:
        ctxs = [gpu.Context(0, max_span_bytes=span + (1 << 20), max_items=4 << 20) for _ in range(T)]
        for c in ctxs:
            for i, p_ in enumerate(pinned):  # warm (buffers sized); record counts
                bt = c.scan_host_ptr(p_.data_ptr(), p_.numel(), 0, True, codec=gpu.RIO_CODEC_FLATE)
                assert bt.err.code == 0, bt.err.msg
                nrec_b[i] = bt.n_items

        def work(w):
            for i in range(w, len(pinned), T):
                bt = ctxs[w].scan_host_ptr(pinned[i].data_ptr(), pinned[i].numel(), 0, True, codec=gpu.RIO_CODEC_FLATE)
                assert bt.err.code == 0 and bt.n_items == nrec_b[i]
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            th = [threading.Thread(target=work, args=(w,)) for w in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            ts.append(time.perf_counter() - t0)
        t = sorted(ts)[len(ts) // 2]
        c3b["ctx_threads_%d" % T] = {"GiBs": round(sum(f.size for f in files) / t / 2 ** 30, 2),
                                     "wall_ms": round(t * 1e3, 1), "records": sum(nrec_b)}
        for c in ctxs:
            c.close()
    out["c3_batched_bodies"] = {"files": len(files), "files_per_batch": per, **c3b}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
