"""End-to-end (PCIe-inclusive) scan rate through the drop-in path: host file in,
host records out.

The north star's path starts and ends in host memory (an io.Reader feeding
chunks in, []byte records handed back to Go). This measures the path a Go user
of the shim takes -- gpurecordio.NewScanner (recordio/scannerv2.go:200-235 is
the reference's): the scanner layer (rio_scanner_*) reads the file through
rio_memory_reader (a memcpy per range read, 16 MiB pieces in parallel) into
pinned staging, with a read-ahead thread filling the next span while the GPU
decodes the current one; each span is copied to HBM, decoded by the same
pipeline as the device-resident bench, and its results (record bytes, 16 B
views, block tables) copied back into pinned result buffers; records are taken
with rio_scanner_next_batch (views, no copy).

Workloads (~2 GiB files, the configs' base files with their bodies replicated:
blocks are independent, so the file is a valid recordio file of R x the base's
records):
  C2 none (1e6 x 256 B records, 253 per block), C3 flate at 1,024 and at
  16,385 records per block (the writer's default MaxItems, writerv2.go:28-29),
  C4 zstd.
Parity: an untimed scan hashes every record (tools/viewhash.c) against the
generator's records repeated R times. Timed: `reps` whole-file scans; GiB/s of
file bytes, plus the bytes copied each way (rio_ctx_stats) and device time.

  python tools/bench_e2e.py [--gib 2] [--span-mib 512] [--reps 2]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import struct
import sys
import time

_T0 = time.perf_counter()

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

CH = 32768


def _replicate(data: bytes, target: int):
    """The base file's header block + its body replicated to >= target bytes
    (a numpy array: the host file). Returns (array, replicas)."""
    import numpy as np
    hdr = struct.unpack_from("<I", data, 20)[0] * CH  # the header block's chunks
    body = np.frombuffer(data, dtype=np.uint8)[hdr:]
    reps = max(1, -(-(target - hdr) // body.size))
    out = np.empty(hdr + reps * body.size, dtype=np.uint8)
    out[:hdr] = np.frombuffer(data, dtype=np.uint8)[:hdr]
    for r in range(reps):
        out[hdr + r * body.size:hdr + (r + 1) * body.size] = body
    return out, reps


def _scan(gpu, src, ctx, hashes=None, batch=1 << 16):
    """One whole-file scan through the scanner; (records, record bytes, parity
    mismatches). hashes: the expected record hashes in file order (checked)."""
    import numpy as np
    import viewhash
    L = ctx.L
    sc = gpu.NewScanner(src, ctx=ctx)
    ptrs = (ctypes.c_void_p * batch)()
    lens = (ctypes.c_uint64 * batch)()
    lv = np.ctypeslib.as_array(lens)
    n = tot = bad = 0
    while True:
        k = L.rio_scanner_next_batch(sc.h, ptrs, lens, batch)
        if k <= 0:
            break
        if hashes is not None:
            got = viewhash.hash_views(ptrs, lens, k)
            want = hashes[n:n + k] if n + k <= hashes.size else None
            bad += k if want is None or want.size != k else int(np.count_nonzero(got != want))
        n += k
        tot += int(lv[:k].sum())
    err = sc.Finish()
    if err is not None:
        raise RuntimeError(f"scan error: {err}")
    return n, tot, bad


def _log(msg):
    print("[bench_e2e %7.1fs] %s" % (time.perf_counter() - _T0, msg), file=sys.stderr, flush=True)


def _workload(gpu, name, data, base_hashes, base_bytes, target, span, reps, device):
    import numpy as np
    _log("scan " + name)
    arr, R = _replicate(data, target)
    src = gpu.MemorySource(arr)
    want = np.tile(base_hashes, R)
    ctx = gpu.Context(device, max_span_bytes=span)
    try:
        t0 = time.perf_counter()
        n, tot, bad = _scan(gpu, src, ctx, want)  # parity pass (also sizes every buffer)
        first_s = time.perf_counter() - t0
        parity = bad == 0 and n == want.size and tot == base_bytes * R
        s0 = ctx.stats()
        walls = []
        for _ in range(reps):
            t0 = time.perf_counter()
            n2, tot2, _ = _scan(gpu, src, ctx)
            walls.append(time.perf_counter() - t0)
            parity = parity and n2 == n and tot2 == tot
        s1 = ctx.stats()
    finally:
        ctx.close()
    w = float(np.median(walls))
    d = {k: (s1[k] - s0[k]) / reps for k in s0 if k != "span_cap"}
    return {"workload": name, "file_bytes": int(arr.size), "replicas": R, "records": n, "record_bytes": tot,
            "GiBs": round(arr.size / w / 2 ** 30, 3), "wall_ms": round(w * 1e3, 1),
            "records_GiBs": round(tot / w / 2 ** 30, 3),
            "bytes_in_h2d": int(d["h2d_bytes"]), "bytes_back_d2h": int(d["d2h_bytes"]),
            "spans": int(d["spans"]), "device_ms": round(d["device_ms"], 1),
            "first_scan_ms": round(first_s * 1e3, 1), "parity": bool(parity), "records_mismatched": bad}


def run_e2e(device: int = 0, gib: float = 2.0, span_mib: int = 512, reps: int = 2, only=None):
    """The four end-to-end workloads; returns the bench sub-line dict."""
    import numpy as np
    import bench
    import c3_data
    import c4_data
    import viewhash
    from base_amd.recordio import gpu
    target = int(gib * 2 ** 30)
    span = span_mib << 20
    out = []
    t_all = time.perf_counter()
    if only is None or "c2" in only:
        data, nrec = bench.make_c2_file()
        recs = bench.c2_records()
        ends = np.arange(1, nrec + 1, dtype=np.uint64) * np.uint64(bench.RECORD_SIZE)
        h = np.empty(nrec, dtype=np.uint64)
        viewhash.lib().buf_hash(recs.ctypes.data, ends.ctypes.data, nrec, h.ctypes.data)
        out.append(_workload(gpu, "C2 none, 253 records per block", data, h, nrec * bench.RECORD_SIZE, target,
                             span, reps, device))
    for per in (1024, 16384):
        if only is not None and ("c3_%d" % per) not in only:
            continue
        _log("C3 file, %d per block" % per)
        data, nrec, rb = c3_data.make_file(128 << 20, per, workers=16)
        recs = []
        for first in range(0, nrec, per):
            recs.extend(c3_data.records(first, min(per, nrec - first)))
        out.append(_workload(gpu, "C3 flate, %d records per block" % (per if per == 1024 else per + 1),
                             data, viewhash.hash_records(recs), rb, target, span, reps, device))
    if only is None or "c4" in only:
        import bench_zstd
        _log("C4 file")
        data, nblk, nrec, rb = bench_zstd.load_or_make(128, 16, "/tmp/c4.bin")
        out.append(_workload(gpu, "C4 zstd, 64 B-64 KiB records, 1 MiB blocks", data,
                             viewhash.hash_records(c4_data.all_records(nblk)), rb, target, span, reps, device))
    return {"metric": "recordio scan GiB/s end-to-end: host file in (rio_memory_reader), records out "
                      "(rio_scanner_next_batch), PCIe copies included", "unit": "GiB/s",
            "path": "rio_scanner_new + rio_scanner_next_batch (the gpurecordio.NewScanner path), pinned staging, "
                    "read-ahead, span %d MiB" % span_mib,
            "parity": all(w["parity"] for w in out), "workloads": out,
            "bench_s": round(time.perf_counter() - t_all, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--span-mib", type=int, default=512)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--only", default=None, help="comma list of c2,c3_1024,c3_16384,c4")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    only = set(args.only.split(",")) if args.only else None
    print(json.dumps(run_e2e(args.device, args.gib, args.span_mib, args.reps, only)), flush=True)


if __name__ == "__main__":
    main()
