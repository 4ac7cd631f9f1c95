"""Benchmark: recordio scan GiB/s, device-resident, compressed bytes in.

Workload (BASELINE.json configs[1]): uncompressed ('none')
recordio, 1,000,000 x 256 B records (splitmix64 bytes, seed 0x5EED0001),
MaxItems=253 -> 3,953 blocks of exactly 2 chunks (64 KiB); the 7,906 body
chunks are replicated 64x device-resident (~16.1 GiB, 64M records) behind one
header chunk. One step = one pass of the scan hot path over that whole file:
chunk CRC32 verify + block structure + varint unpack -> one (offset, length)
view per record, chunk-crossing records gathered (k_chunk_meta, scans, k_parse,
k_strad, k_crc, k_resolve).

N GPUs (torchrun, one process per GPU): every rank scans its own replica set
(weak scaling, no data-path collective); value = all ranks' input bytes / max
time over ranks.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_RECORDS = 1_000_000
RECORD_SIZE = 256
MAX_ITEMS = 253
SEED = 0x5EED0001
REPLICAS = 64
CHUNK = 32768
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, GB/s (MI355X_MICROARCH.md)


def splitmix64(seed: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def c2_records() -> np.ndarray:
    """(1e6, 256) uint8 record bytes."""
    return splitmix64(SEED, N_RECORDS * RECORD_SIZE // 8).view(np.uint8).reshape(N_RECORDS, RECORD_SIZE)


def make_c2_file(max_items: int = MAX_ITEMS):
    """C2 file bytes (header chunk + 3,953 two-chunk blocks) and the record count.
    max_items=16384 (the writer default, writerv2.go:28-29) gives the C1 file:
    62 blocks of 130 chunks."""
    from base_amd.recordio import format as F
    recs = c2_records()
    out = [F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([])]))]
    # every block: uvarint(n) + n x uvarint(256) + n x 256 bytes (writerv2.go:388-441)
    for b0 in range(0, N_RECORDS, max_items):
        blk = recs[b0:b0 + max_items]
        hdr = F.put_uvarint(len(blk)) + F.put_uvarint(RECORD_SIZE) * len(blk)
        out.append(F.chunk_block(F.MAGIC_PACKED, hdr + blk.tobytes()))
    data = b"".join(out)
    return data, N_RECORDS


def make_c1_file():
    """C1 (configs[0]): the same records at the default MaxItems = 16384."""
    return make_c2_file(16384)


PMC_FILE = os.path.join(ROOT, "profiles", "r01_c2_pmc.json")


def pmc_traffic(kernel: str, replicas: int):
    """HBM bytes per launch of `kernel` from the committed PMC pass (tools/pmc.sh:
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over this same bench command, FETCH_SIZE
    doubled per MI355X_MICROARCH.md). Only valid for the default replica count."""
    if replicas != REPLICAS or not os.path.exists(PMC_FILE):
        return None
    with open(PMC_FILE) as f:
        e = json.load(f).get("rio::" + kernel)
    if not e:
        return None
    return int(e.get("fetch_bytes", 0) + e.get("write_bytes", 0))


def _shard_worker(args):
    """One core of the all-cores CPU baseline: NewShardScanner(start=i, limit=i+1,
    nshard=n) over the file, repeated for `budget_s` (v2_test.go:483-509 shape)."""
    data_path, i, n, budget_s = args
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    with open(data_path, "rb") as f:
        data = f.read()
    t0 = time.perf_counter()
    items = passes = 0
    while True:
        k, _ = O.scan_count(data, i, i + 1, n)
        assert k >= 0
        items += k
        passes += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    return passes, items, time.perf_counter() - t0


def cpu_baseline_all_cores(data: bytes, budget_s: float = 8.0):
    """The C oracle on every host core this process may use (at most 16, the GPU
    box's CPU share): one shard per core, each core rescanning its shard."""
    import tempfile
    from concurrent.futures import ProcessPoolExecutor
    from oracle import oracle as O
    O.build()
    try:
        ncores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        ncores = os.cpu_count() or 1
    ncores = max(1, min(ncores, 16))
    with tempfile.NamedTemporaryFile(suffix=".rio", delete=False) as f:
        f.write(data)
        path = f.name
    try:
        with ProcessPoolExecutor(max_workers=ncores) as ex:
            res = list(ex.map(_shard_worker, [(path, i, ncores, budget_s) for i in range(ncores)]))
    finally:
        os.unlink(path)
    # each core covers 1/ncores of the file per pass
    gib = sum(p * len(data) / ncores for p, _, _ in res) / 2 ** 30
    wall = max(t for _, _, t in res)
    return {"value": round(gib / wall, 3), "unit": "GiB/s", "cores": ncores, "kind": "port",
            "sample": "C2 1x file split into %d shards (NewShardScanner shape), C oracle, one process per "
                      "core, %.0f s" % (ncores, budget_s)}


def cpu_baseline(data: bytes, budget_s: float = 10.0):
    """The C oracle (restatement of recordio.NewScanner's loop) on one host core."""
    from oracle import oracle as O
    O.build()
    t0 = time.perf_counter()
    passes = 0
    nbytes = 0
    while True:
        n, _ = O.scan_count(data)
        assert n == N_RECORDS
        passes += 1
        nbytes += len(data)
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    cpu = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(nbytes / dt / 2 ** 30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{passes} x C2 1x file ({len(data)} B, {N_RECORDS} records), C oracle "
                      f"(oracle/scanner.c) single thread on {cpu}; the Go reference cannot be built here"}


def c3_flate(args, local, world, dist):
    """BASELINE.json configs[2] beside the headline: ~10 GiB of FASTQ-like records in
    flate blocks (1,024 records per block) per GPU, device-resident, one pass =
    chunk CRC + two-pass DEFLATE decode + packed unpack (tools/bench_flate.py).
    Whole-job GiB/s of compressed input over the max time across ranks."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_flate
    cpu_s = 8.0 if (world == 1 and not args.no_cpu_baseline) else 0.0
    r = bench_flate.run_c3(replicas=args.flate_replicas, steps=max(2, min(args.steps, 5)), warmup=1,
                           device=local, check=True, cpu_s=cpu_s)
    if dist is not None:
        t = torch.tensor([r["ms_per_step"]], device=f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        r["value"] = round(r["config"]["span_bytes"] * world / (ms * 1e-3) / 2 ** 30, 2)
        r["ms_per_step"] = round(ms, 3)
    r["n_gpus"] = world
    r["target_GiBs"] = 40.0  # BASELINE.json north_star: >= 40 GiB/s compressed-in on flate at 1 GPU
    # HBM roofline of the decode pipeline: compressed bytes read + decoded bytes written
    moved = (r["config"]["span_bytes"] + r["config"]["records_bytes"]) * world
    r["hbm_frac"] = round(moved / (r["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    return r


def c4_zstd(args, local, world, dist):
    """BASELINE.json configs[3] beside the headline: ~10 GiB of records (sizes
    log-uniform 64 B-64 KiB, 1 MiB blocks, zstd level 5) per GPU, device-resident,
    one pass = chunk CRC + zstd entropy/execution passes + packed unpack
    (tools/bench_zstd.py). Whole-job GiB/s of compressed input."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_zstd
    cpu_s = 6.0 if (world == 1 and not args.no_cpu_baseline) else 0.0
    r = bench_zstd.run_c4(replicas=args.zstd_replicas, steps=max(2, min(args.steps, 3)), warmup=1, device=local,
                          check=True, cpu_s=cpu_s)
    if dist is not None:
        t = torch.tensor([r["ms_per_step"]], device=f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        r["value"] = round(r["config"]["span_bytes"] * world / (ms * 1e-3) / 2 ** 30, 2)
        r["ms_per_step"] = round(ms, 3)
    r["n_gpus"] = world
    moved = (r["config"]["span_bytes"] + r["config"]["records_bytes"]) * world
    r["hbm_frac"] = round(moved / (r["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--replicas", type=int, default=REPLICAS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-flate", action="store_true", help="skip the C3 flate measurement (configs[2])")
    ap.add_argument("--flate-replicas", type=int, default=80)
    ap.add_argument("--no-zstd", action="store_true", help="skip the C4 zstd measurement (configs[3])")
    ap.add_argument("--zstd-replicas", type=int, default=80)
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

    from base_amd import build as B
    if not os.path.exists(B.LIB):
        B.build()
    from base_amd.recordio import gpu

    data, nrec = make_c2_file()
    body = data[CHUNK:]
    nbody = len(body)
    total = CHUNK + args.replicas * nbody
    dev = torch.empty(total, dtype=torch.uint8, device=f"cuda:{local}")
    host = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    dev[:len(data)].copy_(host)
    body_dev = dev[CHUNK:CHUNK + nbody]
    for r in range(1, args.replicas):
        dev[CHUNK + r * nbody:CHUNK + (r + 1) * nbody].copy_(body_dev)
    torch.cuda.synchronize()
    n_items = nrec * args.replicas
    # items are views into the span; only chunk-straddling items are gathered (side buffer)
    ctx = gpu.Context(local, max_span_bytes=total, max_items=n_items + 1024)
    span_ptr = dev.data_ptr() + CHUNK
    span_len = total - CHUNK

    def step():
        ctx.scan_device_async(span_ptr, span_len, CHUNK, gpu.RIO_CODEC_NONE)
        return ctx.sync()

    b = step()
    assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
    assert b.n_items == n_items, (b.n_items, n_items)
    for _ in range(args.warmup):
        step()

    crc_ms, stage_sum = [], np.zeros(5)
    kern_ms = []
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        bb = step()
        st = ctx.stage_times()
        crc_ms.append(st[2])
        stage_sum += np.array(st)
        kern_ms.append(bb.kernel_ms)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device=f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / args.steps * 1e3
    in_bytes = span_len * world
    value = in_bytes * args.steps / dt / 2 ** 30

    # roofline of the dominant kernel (k_crc): it reads every chunk byte once
    # (B_in per launch; DESIGN.md "Roofline")
    crc_avg = float(np.mean(crc_ms))
    alg = span_len
    achieved = alg / (crc_avg * 1e-3) / 1e9
    # whole pipeline: chunk bytes in + item views (16 B) + block table out (straddlers,
    # ~1 per block here, are ~0.4 % of the bytes and not counted)
    pipe_alg = span_len + 16 * n_items + 8 * int(b.n_blocks)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("k_crc", args.replicas),
            "kernel": "k_crc", "kernel_ms": round(crc_avg, 3),
            "alg_bytes_per_launch": alg,
            "pipeline_ms": round(float(np.mean(kern_ms)), 3),
            "pipeline_alg_GBs": round(pipe_alg / (np.mean(kern_ms) * 1e-3) / 1e9, 1),
            "stage_ms": [round(x / args.steps, 3) for x in stage_sum]}

    out = {"metric": "recordio scan GiB/s device-resident (compressed in) at 1/2/4/8 MI355X",
           "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "config": {"workload": "C2: none codec, 1e6 x 256 B records x %d replicas, MaxItems=253 "
                                  "(64 KiB blocks), chunk CRC32 + packed-unpack" % args.replicas,
                      "records_per_gpu": int(n_items), "record_bytes": RECORD_SIZE,
                      "parallelism": f"{world} GPU(s), independent replica sets",
                      "bytes_in_per_gpu": span_len},
           "roofline": roof}
    ctx.close()
    del dev
    torch.cuda.empty_cache()
    if not args.no_flate:
        out["c3_flate"] = c3_flate(args, local, world, dist)
    if not args.no_zstd:
        out["c4_zstd"] = c4_zstd(args, local, world, dist)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(data)
        out["cpu_baseline_all_cores"] = cpu_baseline_all_cores(data)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
