"""v1 (legacy) scan throughput: the C1/C2 record set --
1e6 x 256 B records -- written by the reference's v1 writers with their
defaults (packed: deprecated/packed.go:18-24, 16384 items / 16 MiB per record;
unpacked: one record per item), read
  (a) through the batch layer (rio_scan_v1_span over a host-resident span:
      H2D of the packed records, k_v1_unpack, D2H of the item views),
  (b) through the scanner (rio_scanner_* over rio_memory_reader: read-ahead,
      staging, batch, Scan/Get views),
  (c) by the oracle's v1 restatement on one core (the CPU sample).
Prints one JSON line."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_files(n_items=1_000_000, size=256, seed=7):
    import numpy as np
    from base_amd.recordio import format as F
    rng = np.random.default_rng(seed)
    per = F.LEGACY_DEFAULT_PACKED_ITEMS
    blob = rng.integers(0, 256, size=per * size, dtype=np.uint8).tobytes()
    items = [blob[i * size:(i + 1) * size] for i in range(per)]
    full = F.legacy_record(F.MAGIC_PACKED, F.legacy_packed_payload(items))
    nfull, rest = divmod(n_items, per)
    packed = full * nfull + (F.legacy_record(F.MAGIC_PACKED, F.legacy_packed_payload(items[:rest])) if rest else b"")
    one = b"".join(F.legacy_record(F.MAGIC_LEGACY_UNPACKED, it) for it in items)
    unpacked = one * nfull + b"".join(F.legacy_record(F.MAGIC_LEGACY_UNPACKED, it) for it in items[:rest])
    return packed, unpacked, n_items * size


def bench_batch(ctx, data, reps):
    from base_amd.recordio import gpu
    buf = (ctypes.c_char * len(data)).from_buffer_copy(data)
    H = gpu._hip()
    pinned = ctypes.c_void_p()
    assert H.hipHostMalloc(ctypes.byref(pinned), ctypes.c_size_t(len(data)), 0) == 0
    ctypes.memmove(pinned, buf, len(data))
    out = gpu.RioBatch()
    best, kms = 1e9, 0.0
    for r in range(reps + 1):
        t = time.perf_counter()
        rc = ctx.L.rio_scan_v1_span(ctx.h, pinned, len(data), 0, 1, ctypes.byref(out))
        dt = time.perf_counter() - t
        assert rc == 0 and out.stop == gpu.RIO_STOP_EOF, (rc, out.stop, out.err.msg)
        if r and dt < best:
            best, kms = dt, out.kernel_ms
    n = int(out.n_items)
    H.hipHostFree(pinned)
    return best, kms, n


def bench_scanner(ctx, data, reps):
    from base_amd.recordio import gpu
    src = gpu.MemorySource(data)
    best, n = 1e9, 0
    ptrs = (ctypes.c_void_p * 65536)()
    lens = (ctypes.c_uint64 * 65536)()
    for r in range(reps + 1):
        t = time.perf_counter()
        sc = gpu.NewScanner(src, ctx=ctx)
        k = 0
        while True:
            m = ctx.L.rio_scanner_next_batch(sc.h, ptrs, lens, 65536)
            if m <= 0:
                break
            k += m
        assert sc.Finish() is None
        dt = time.perf_counter() - t
        if r and dt < best:
            best, n = dt, k
    return best, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--cpu", type=int, default=1)
    a = ap.parse_args()
    from base_amd.recordio import gpu
    packed, unpacked, rec_bytes = make_files(a.items)
    ctx = gpu.Context(0, max_span_bytes=512 << 20)
    GiB = float(1 << 30)
    res = {"workload": "v1: %d x 256 B records, reference v1 writer defaults" % a.items,
           "record_bytes": rec_bytes, "packed_file": len(packed), "unpacked_file": len(unpacked)}
    for name, data in (("packed", packed), ("unpacked", unpacked)):
        dt, kms, n = bench_batch(ctx, data, a.reps)
        assert n == a.items
        res[name + "_batch_GiBps"] = round(len(data) / dt / GiB, 2)
        res[name + "_batch_ms"] = round(dt * 1e3, 2)
        res[name + "_kernel_ms"] = round(kms, 3)
        dt, n = bench_scanner(ctx, data, a.reps)
        assert n == a.items
        res[name + "_scanner_GiBps"] = round(len(data) / dt / GiB, 2)
        if a.cpu:
            from oracle import oracle as O
            t = time.perf_counter()
            items, nbytes = O.scan_count(data)
            dt = time.perf_counter() - t
            assert items == a.items
            res[name + "_cpu_oracle_1core_GiBps"] = round(len(data) / dt / GiB, 3)
    ctx.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
