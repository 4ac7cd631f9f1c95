"""CPU baselines for bench.py (the cpu_baseline leg; test infrastructure).

oracle/cpu_scan.c runs the reference's scan loop (NewShardScanner -> Scan,
chunk CRC, untransform, parseChunksToItems) over an in-memory file with tuned C
decoders standing in for the reference's Go / cgo ones: PCLMUL CRC32 (as Go's
hash/crc32 on amd64), zlib raw inflate for flate (reference: klauspost
compress/flate), libzstd for zstd (reference: DataDog/zstd = libzstd). One core
= one scanner; all cores = one NewShardScanner(i, i+1, n) per thread, as in
recordio/v2_test.go:483-509. The Go reference cannot be built here (no Go
toolchain), so these are labelled by the decoder they run.
"""
from __future__ import annotations

import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

KIND = {0: "port", 1: "zlib", 2: "libzstd"}
DECODER = {0: "C restatement of the scan loop, PCLMUL CRC32",
           1: "scan loop + zlib raw inflate (stand-in for klauspost flate)",
           2: "scan loop + libzstd ZSTD_decompress (the library DataDog/zstd wraps)"}


def host_cores() -> int:
    """Cores this process may use, capped at the GPU box's 16-core share."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown CPU"


def time_cpu(data: bytes, codec: int, threads: int, budget_s: float, expect_items: int, label: str):
    """Repeat the CPU scan of `data` for about budget_s; GiB/s of file bytes in
    (the metric's unit: the on-disk chunk stream)."""
    from oracle import oracle as O
    O.build()
    n, _ = O.cpu_scan(data, codec, threads)  # warm (page cache, allocator)
    assert n == expect_items, (n, expect_items)
    t0 = time.perf_counter()
    passes = 0
    while True:
        n, _ = O.cpu_scan(data, codec, threads)
        assert n == expect_items
        passes += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(passes * len(data) / dt / 2 ** 30, 3), "unit": "GiB/s", "cores": threads,
            "kind": KIND[codec],
            "sample": "%d x %s (%d B, %d records), %s, %d thread(s) on %s; the Go reference cannot be "
                      "built here" % (passes, label, len(data), expect_items, DECODER[codec], threads, cpu_model())}


def baselines(data: bytes, codec: int, expect_items: int, label: str, budget_s: float):
    """(one core, all cores) dicts."""
    one = time_cpu(data, codec, 1, budget_s, expect_items, label)
    allc = time_cpu(data, codec, host_cores(), budget_s, expect_items, label)
    return one, allc
