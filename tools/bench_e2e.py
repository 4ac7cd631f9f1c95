"""End-to-end (PCIe-inclusive) scan rate: host bytes in, host results out.

The north star's path starts and ends in host memory (an io.Reader feeding
chunks, []byte records handed back). rio_scan_span takes a host span of whole
chunks, copies it to HBM (hipMemcpyAsync), runs the same pipeline as the
device-resident bench, and copies the results back into library-owned pinned
buffers: 16 B of item view per record plus, for 'none', the chunk-straddling
records (the other records are views into the caller's span), and for flate /
zstd every decoded record byte.

Measured per workload, from pageable (numpy) and pinned (hipHostMalloc via
torch pin_memory) host spans: wall-clock GiB/s of file bytes in, and the split
into H2D / pipeline / D2H from the batch's HIP-event times.

  python tools/bench_e2e.py [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

CH = 32768


def _run(name, data, codec, nrec, reps, device, out_bytes):
    import numpy as np
    import torch
    from base_amd.recordio import gpu

    import struct
    hdr = struct.unpack_from("<I", data, 20)[0] * CH  # the header block (read by the scanner layer)
    data = data[hdr:]
    ctx = gpu.Context(device, max_span_bytes=len(data) + CH, max_items=nrec + 1024)
    res = {}
    page = np.frombuffer(bytearray(data), dtype=np.uint8)
    pin = torch.frombuffer(bytearray(data), dtype=torch.uint8).pin_memory()
    for kind, ptr in (("pageable", page.ctypes.data), ("pinned", pin.data_ptr())):
        b = ctx.scan_host_ptr(ptr, len(data), hdr, True, codec=codec)  # warm: buffers sized
        assert b.err.code == 0 and b.n_items == nrec, (name, kind, b.err.msg, b.n_items, nrec)
        walls, tot, kern = [], [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            b = ctx.scan_host_ptr(ptr, len(data), hdr, True, codec=codec)
            walls.append(time.perf_counter() - t0)
            tot.append(b.total_ms)
            kern.append(b.kernel_ms)
            assert b.err.code == 0 and b.n_items == nrec
        w = float(np.median(walls))
        res[kind] = {"GiBs_in": round(len(data) / w / 2 ** 30, 2), "wall_ms": round(w * 1e3, 2),
                     "device_timeline_ms": round(float(np.median(tot)), 2),
                     "pipeline_ms": round(float(np.median(kern)), 2),
                     "back_bytes": int(b.records_len) + 16 * int(b.n_items)}
    ctx.close()
    return {"workload": name, "span_bytes": len(data), "records": nrec, "record_bytes": out_bytes, **res}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args()
    import bench
    import c3_data
    import c4_data
    from base_amd.recordio import gpu

    out = []
    data, nrec = bench.make_c2_file()
    out.append(_run("C2 none (1x file, 1e6 x 256 B)", data, gpu.RIO_CODEC_NONE, nrec, args.reps, args.device,
                    nrec * 256))
    data, nrec, rb = c3_data.make_file(128 << 20, 1024, workers=16)
    out.append(_run("C3 flate base file (128 MiB of records)", data, gpu.RIO_CODEC_FLATE, nrec, args.reps,
                    args.device, rb))
    data, nblk, nrec, rb = c4_data.make_file(128 << 20, workers=16)
    out.append(_run("C4 zstd base file (128 MiB of records)", data, gpu.RIO_CODEC_ZSTD, nrec, args.reps,
                    args.device, rb))
    print(json.dumps({"end_to_end": out}), flush=True)


if __name__ == "__main__":
    main()
