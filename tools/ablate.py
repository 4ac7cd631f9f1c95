"""Measurement-only ablations of the none-codec pipeline on the C2 workload.

Runs the scan with RIO_KERNEL_FLAGS = 0 (full), 2 (CRC alone), 3 (CRC loads
only, no fold), 4 (parse path alone) and times a plain device-to-device copy of the same bytes (the
copy ceiling quoted in DESIGN.md). One JSON line per variant.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from base_amd.recordio import gpu

    reps = int(os.environ.get("REPLICAS", "64"))
    data, nrec = bench.make_c2_file()
    body = data[bench.CHUNK:]
    total = bench.CHUNK + reps * len(body)
    dev = torch.empty(total, dtype=torch.uint8, device="cuda:0")
    dev[:len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    for r in range(1, reps):
        dev[bench.CHUNK + r * len(body):bench.CHUNK + (r + 1) * len(body)].copy_(dev[bench.CHUNK:len(data)])
    torch.cuda.synchronize()
    span_len = total - bench.CHUNK
    for flags in [int(x) for x in os.environ.get("FLAGS", "0,2,3,4").split(",")]:
        os.environ["RIO_KERNEL_FLAGS"] = str(flags)
        ctx = gpu.Context(0, max_span_bytes=total, max_items=nrec * reps + 1024)
        times = []
        for i in range(6):
            ctx.scan_device_async(dev.data_ptr() + bench.CHUNK, span_len, bench.CHUNK, gpu.RIO_CODEC_NONE)
            b = ctx.sync()
            if i:
                times.append(ctx.stage_times())
        t = np.mean(np.array(times), axis=0)
        print(json.dumps({"flags": flags, "stage_ms": [round(x, 3) for x in t],
                          "crc_GBs": round(span_len / (t[2] * 1e-3) / 1e9, 1) if t[2] > 0 else None,
                          "stop": b.stop, "n_items": b.n_items}), flush=True)
        ctx.close()
    # device-to-device copy ceiling on the same byte count
    dst = torch.empty(span_len, dtype=torch.uint8, device="cuda:0")
    src = dev[bench.CHUNK:]
    for _ in range(2):
        dst.copy_(src)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 5
    for _ in range(n):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(json.dumps({"d2d_copy_ms": round(ms, 3), "d2d_copy_GBs": round(2 * span_len / (ms * 1e-3) / 1e9, 1)}))
    # read-only ceiling: a reduction over the same bytes
    v = src.view(torch.int64)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        s = torch.bitwise_xor(v[: v.numel() // 2], v[v.numel() // 2: 2 * (v.numel() // 2)]).sum()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    print(json.dumps({"xor_reduce_ms": round(ms, 3), "read_GBs": round(span_len / (ms * 1e-3) / 1e9, 1),
                      "dummy": int(s.item()) & 1}))


if __name__ == "__main__":
    main()
