"""Writer encode path throughput: the C2 record set
(1e6 x 256 B, 253 per block) replicated R times device-resident, encoded by
rio_encode_device into a chunk stream (packed headers, framing, padding,
CRC32), then scanned back by rio_scan_device as the parity check (item count,
and the first replica's views against the records). --codec 1 / 2: the C3
FASTQ-like records through the GPU flate / zstd encoders. Prints one JSON line."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--codec", type=int, default=0)  # 0 none (C2 records), 1 flate / 2 zstd (C3 records)
    ap.add_argument("--level", type=int, default=6)  # flate: 0 stored, 1 fixed Huffman, else dynamic
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from base_amd.recordio import gpu
    R = a.replicas
    if a.codec == 0:  # C2: 1e6 x 256 B, 253 per block
        recs = bench.c2_records()
        n1 = recs.shape[0]
        n = n1 * R
        data = torch.from_numpy(np.ascontiguousarray(recs).reshape(-1)).cuda().repeat(R)
        ends = (torch.arange(1, n + 1, dtype=torch.int64, device="cuda") * 256)
        per = 253
    else:  # C3: FASTQ-like records (tools/c3_data.py), 1,024 per block, flate or zstd
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import c3_data
        recs = c3_data.records(0, 1 << 17)
        n1 = len(recs)
        n = n1 * R
        blob = np.frombuffer(b"".join(recs), dtype=np.uint8)
        lens = np.fromiter((len(r) for r in recs), dtype=np.int64, count=n1)
        data = torch.from_numpy(blob.copy()).cuda().repeat(R)
        e1 = torch.from_numpy(np.cumsum(lens)).cuda()
        ends = torch.cat([e1 + k * int(blob.size) for k in range(R)])
        per = 1024
    nb = (n + per - 1) // per
    cap = 32768 * (nb * 2 + int(data.numel()) * 9 // 8 // 32740 + 16)  # >= any stream (flate: <= 9/8)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    boff = torch.empty(nb, dtype=torch.int64, device="cuda")
    ctx = gpu.Context(0, max_span_bytes=cap)
    args = gpu.RioEncodeArgs(data.data_ptr(), ends.data_ptr(), n, per, a.codec, gpu.RIO_BLOCK_BODY, a.level, 0)
    err = gpu.RioError()
    olen = ctypes.c_uint64()
    times = []
    for r in range(a.reps + 1):
        torch.cuda.synchronize()
        t = time.perf_counter()
        rc = ctx.L.rio_encode_device(ctx.h, ctypes.byref(args), out.data_ptr(), cap, ctypes.byref(olen),
                                     boff.data_ptr(), ctypes.byref(err))
        torch.cuda.synchronize()
        if rc != 0:
            raise RuntimeError("rio_encode_device rc=%d %s %s" % (rc, err.msg, ctx.L.rio_last_error()))
        if r:
            times.append(time.perf_counter() - t)
    dt = min(times)
    out_len = olen.value
    # parity: scan the encoded stream back on the device
    b = ctx.scan_device(out.data_ptr(), out_len, 32768, True, a.codec)
    ok = b.stop == gpu.RIO_STOP_EOF and b.n_items == n
    # transformed payload bytes: the chunk headers' size fields (offset 16 of every chunk)
    sizes = out[:out_len].view(-1, 32768)[:, 16:20].contiguous().view(torch.int32)
    pay = int(sizes.sum().item())
    detail = {"stop": int(b.stop), "n_items": int(b.n_items), "err": b.err.msg.decode(),
              "ratio": round(int(data.numel()) / out_len, 3), "payload_bytes": pay,
              "payload_ratio": round(int(data.numel()) / pay, 3)}
    if a.codec == 0:  # the first 3,952 blocks (whole 253-record blocks) equal the bench's C2 file
        want = bench.make_c2_file()[0][32768:32768 + 3952 * 65536]
        detail["bytes_equal"] = out[:len(want)].cpu().numpy().tobytes() == want
        ok = ok and detail["bytes_equal"]
    rec_bytes = int(data.numel())
    GiB = float(1 << 30)
    res = {"workload": "encode %s records x %d (%d records, %d per block), codec %d level %d" %
           ("C2" if a.codec == 0 else "C3", R, n, per, a.codec, a.level),
           "record_bytes": rec_bytes, "out_bytes": out_len, "ms": round(dt * 1e3, 3),
           "records_GiBps": round(rec_bytes / dt / GiB, 1),
           "hbm_alg_GBps": round((rec_bytes + out_len) / dt / 1e9, 1),  # records read + stream written
           "scan_back_ok": bool(ok), "scan_back": detail, "blocks": nb, "chunks": out_len // 32768}
    print(json.dumps(res))
    ctx.close()


if __name__ == "__main__":
    main()
