"""Benchmark: recordio scan GiB/s, device-resident, compressed bytes in.

Workload (BASELINE.json configs[1]): uncompressed ('none')
recordio, 1,000,000 x 256 B records (splitmix64 bytes, seed 0x5EED0001),
253 records per block (the writer packs MaxItems + 1 per block,
writerv2.go:315, 366-368: MaxItems=252) -> 3,953 blocks of exactly 2 chunks
(64 KiB); the 7,906 body
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
import ctypes
import json
import os
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
    max_items = records per block = the writer's MaxItems + 1 (writerv2.go:315,
    366-368); 16385 (the default MaxItems = 16384, writerv2.go:28-29) gives the
    C1 file: 62 blocks of 130 chunks."""
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
    return make_c2_file(16385)


PMC_FILE = os.path.join(ROOT, "profiles", "r06_c2_pmc.json")


def pmc_traffic(kernel: str, replicas: int):
    """HBM bytes per launch of `kernel` from the committed PMC pass (tools/gpu_r06.sh pmcc2:
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over this same bench command, FETCH_SIZE
    doubled per MI355X_MICROARCH.md). Only valid for the default replica count."""
    if replicas != REPLICAS or not os.path.exists(PMC_FILE):
        return None
    with open(PMC_FILE) as f:
        pm = json.load(f)
    e = (pm.get("rio::" + kernel) or pm.get("rio::%s<false>" % kernel)  # k_crc is a template
         or pm.get("rio::%s<false, false>" % kernel))
    if not e:
        return None
    return int(e.get("fetch_bytes", 0) + e.get("write_bytes", 0))


REHEARSE = os.environ.get("RIO_BENCH_REHEARSE") == "1"  # N ranks on one GPU over gloo (rehearsal only)


def mem_share(args, world):
    """Fraction of the per-GPU workload sizes a rank runs: 1 (every rank has its
    own GPU); in a rehearsal (RIO_BENCH_REHEARSE=1, every rank on GPU 0) 1/world
    unless --mem-share says otherwise, so that the ranks' buffers together fit
    the one GPU's HBM. Only the auto-sized defaults scale (C2 replicas, C3 / C4
    replicas, C5 batch size); explicit sizes are kept."""
    if args.mem_share > 0:
        return args.mem_share
    return 1.0 / world if REHEARSE else 1.0
_T0 = time.perf_counter()


def progress(rank, msg):
    """A progress line on stderr (rank 0): stdout carries only the result line."""
    if rank == 0:
        print("[bench %7.1fs] %s" % (time.perf_counter() - _T0, msg), file=sys.stderr, flush=True)


def coll_dev(local):
    """Device of the collectives' tensors: the rank's GPU under RCCL, the CPU under gloo."""
    return "cpu" if REHEARSE else f"cuda:{local}"


def cpu_baselines(args):
    """cpu_baseline legs (rank 0, N=1 only; tools/cpu_base.py): the C2 file (the
    headline's workload) and the C1 file (configs[0], the reference's own
    CPU-runnable case: default MaxItems), one core and all cores."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import cpu_base
    d2, n2 = make_c2_file()
    one, allc = cpu_base.baselines(d2, 0, n2, "C2 1x file", args.cpu_s)
    d1, n1 = make_c1_file()
    c1_one, c1_all = cpu_base.baselines(d1, 0, n1, "C1 file", args.cpu_s)
    return one, allc, {"config": "C1 (configs[0]): 1e6 x 256 B, MaxItems=16384", "cpu_baseline": c1_one,
                       "cpu_baseline_all_cores": c1_all}


def c3_flate(args, local, world, dist):
    """BASELINE.json configs[2] beside the headline: ~10 GiB of FASTQ-like records in
    flate blocks (1,024 records per block) per GPU, device-resident, one pass =
    chunk CRC + two-pass DEFLATE decode + packed unpack (tools/bench_flate.py).
    Whole-job GiB/s of compressed input over the max time across ranks. Steps
    rotate over --flate-pipeline context sets (a scanner's read-ahead: the next
    spans are launched before this one is collected); `serial` is the same steps
    one at a time (with --flate-pipeline 1, `value` is)."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_flate
    cpu_s = args.cpu_s if (world == 1 and not args.no_cpu_baseline) else 0.0
    r = bench_flate.run_c3(replicas=args.flate_replicas, steps=max(2, min(args.steps, 5)), warmup=1,
                           device=local, check=True, cpu_s=cpu_s, pipeline=args.flate_pipeline,
                           share=mem_share(args, world))
    if dist is not None:
        t = torch.tensor([r["ms_per_step"]], device=coll_dev(local), dtype=torch.float64)
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


def c3_flate_16k(args, local, world, dist):
    """BASELINE.json configs[2] at the reference writer's default block size:
    MaxItems = 16384 (recordio/writerv2.go:28-29), i.e. 16,385 records per block
    (~5 MB blocks; SURVEY.md §8(d) C3's sensitivity point), the same ~10 GiB of
    records. Steps rotate over three contexts (--flate16k-pipeline), each
    launched before the previous steps are collected -- a scanner's read-ahead of
    its next spans: one step's copy pass runs beside the next steps' Huffman
    passes (a span of 2,158 blocks fills neither pass alone; three in flight
    measured 43.4-44.2 GiB/s against 42.0-42.3 for two,
    profiles/r05_flate_depth_ab.jsonl). `serial` is the same steps
    one at a time. Every record of the last timed step is checked."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_flate
    r = bench_flate.run_c3(replicas=args.flate_replicas, steps=max(2, min(args.steps, 5)), warmup=2,
                           per_block=16384, device=local, check=True, pipeline=args.flate16k_pipeline,
                           share=mem_share(args, world))
    if dist is not None:
        t = torch.tensor([r["ms_per_step"]], device=coll_dev(local), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        r["value"] = round(r["config"]["span_bytes"] * world / (ms * 1e-3) / 2 ** 30, 2)
        r["ms_per_step"] = round(ms, 3)
    r["n_gpus"] = world
    r["target_GiBs"] = 40.0
    moved = (r["config"]["span_bytes"] + r["config"]["records_bytes"]) * world
    r["hbm_frac"] = round(moved / (r["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    return r


def c4_zstd(args, local, world, dist):
    """BASELINE.json configs[3] beside the headline: ~10 GiB of records (sizes
    log-uniform 64 B-64 KiB, 1 MiB blocks, zstd level 5) per GPU, device-resident,
    one pass = chunk CRC + zstd entropy/execution passes + packed unpack
    (tools/bench_zstd.py). Whole-job GiB/s of compressed input. The span is cut at
    replica boundaries into --zstd-contexts parts, each scanned by its own context
    and all in flight together (the passes' tails and LDS-bound phases overlap);
    every record of every part is checked after the timed steps."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_zstd
    cpu_s = args.cpu_s if (world == 1 and not args.no_cpu_baseline) else 0.0
    # (6 steps: with two in flight the first step's fill weighs on a 3-step average --
    # 92.3 ms per step at 3 against 86.0-86.3 at 4-6, profiles/r06_c4_depth_ab.jsonl)
    r = bench_zstd.run_c4(replicas=args.zstd_replicas, steps=max(2, min(args.steps, 6)), warmup=1, device=local,
                          check=True, cpu_s=cpu_s, contexts=args.zstd_contexts, pipeline=args.zstd_pipeline,
                          share=mem_share(args, world))
    if dist is not None:
        t = torch.tensor([r["ms_per_step"]], device=coll_dev(local), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        r["value"] = round(r["config"]["span_bytes"] * world / (ms * 1e-3) / 2 ** 30, 2)
        r["ms_per_step"] = round(ms, 3)
    r["n_gpus"] = world
    moved = (r["config"]["span_bytes"] + r["config"]["records_bytes"]) * world
    r["hbm_frac"] = round(moved / (r["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    return r


def c5_flate(args, local, rank, world, dist):
    """BASELINE.json configs[4]: 1024 trailer-indexed flate files (64 MiB of C3
    records each, tools/c5_data.py) over the ranks -- files assigned by
    size-balanced greedy assignment (shard.assign_files), every rank's files
    device-resident, decoded as batches of whole file bodies back to back, one
    rio_scan_device_segments_async launch per batch (each body a segment: its
    blocks' ItemLocation.Block offsets are their own file's). The 1024 files are
    made from c5_data.N_BASE generated base files (generating 1024 distinct 64 MiB
    files would take ~10 minutes per run): file f is base f mod N_BASE with its
    blocks rotated by a file-specific count (blocks are independent, so it is a
    valid recordio file of the same records in another order), so every file
    has its own block layout, record order and trailer index; every file is
    decoded and checked on its own. Strong scaling: the 1024 files are fixed as N grows; value = all
    files' bytes / max time over ranks. No record byte crosses xGMI; the one
    collective is the ordered-output prefix (RCCL).

    Parity (untimed pass, every file of the rank): each file's records -- its
    blocks' item bytes by the item_end output -- equal its base's records, and
    its blocks' file offsets equal its trailer index. Timed pass: the batches
    alternate between two contexts (two streams), each batch's result checked
    (no error, its record count) when its context is next used or at the end."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import c5_data
    from base_amd.recordio import gpu, shard
    cache = os.path.join(args.c5_cache, "rio_c5_%d" % (c5_data.FILE_RECORD_BYTES >> 20))
    os.makedirs(cache, exist_ok=True)
    t0 = time.perf_counter()
    for k in range(c5_data.N_BASE):  # bases generated in parallel across ranks, cached on the host
        path = os.path.join(cache, "base%d.rio" % k)
        if k % world == rank and not os.path.exists(path):
            data, nrec, rec_bytes, offsets = c5_data.make_base(k, workers=16 if world == 1 else 4)
            with open(path + ".tmp", "wb") as f:
                f.write(data)
            with open(path + ".json", "w") as f:
                json.dump({"nrec": nrec, "rec_bytes": rec_bytes}, f)
            os.replace(path + ".tmp", path)
    if dist is not None:
        dist.barrier()
    bases, metas = [], []
    for k in range(c5_data.N_BASE):
        path = os.path.join(cache, "base%d.rio" % k)
        with open(path, "rb") as f:
            bases.append(f.read())
        with open(path + ".json") as f:
            metas.append(json.load(f))
    gen_s = time.perf_counter() - t0
    # each base's block index (its trailer item, read through the GPU scanner)
    spans, index = [], []
    for k, data in enumerate(bases):
        sc = gpu.NewScanner(data, ctx=gpu.default_context(local))
        offs = c5_data.parse_index(sc.Trailer())
        assert sc.Finish() is None and len(offs) == -(-metas[k]["nrec"] // c5_data.PER_BLOCK)
        spans.append((offs[0], shard.trailer_offset(data)))
        index.append(offs)
    sizes = [len(bases[f % c5_data.N_BASE]) for f in range(c5_data.N_FILES)]
    mine = shard.assign_files(sizes, world)[rank]
    body_len = [spans[k][1] - spans[k][0] for k in range(c5_data.N_BASE)]
    rel = [[o - index[k][0] for o in index[k]] for k in range(c5_data.N_BASE)]  # body-relative block starts

    def rot(f):  # file f's first block (of its base's): its blocks are base blocks rot, rot + 1, ..., rot - 1
        k = f % c5_data.N_BASE
        return (f // c5_data.N_BASE) * 37 % len(index[k])

    def file_index(f):  # file f's trailer index: its blocks' file offsets, in its block order
        k, r = f % c5_data.N_BASE, rot(f)
        nb_, n, cut = len(index[k]), body_len[k], rel[k][rot(f)]
        return [spans[k][0] + (rel[k][(r + j) % nb_] - cut) % n for j in range(nb_)]
    # batches of whole file bodies, <= args.c5_batch_gib each
    cap = int(args.c5_batch_gib * mem_share(args, world) * 2 ** 30)
    batches, cur, cur_b = [], [], 0
    for f in mine:
        n = body_len[f % c5_data.N_BASE]
        if cur and cur_b + n > cap:
            batches.append(cur)
            cur, cur_b = [], 0
        cur.append(f)
        cur_b += n
    if cur:
        batches.append(cur)
    total = sum(body_len[f % c5_data.N_BASE] for f in mine)
    dev = torch.empty(max(total, 1), dtype=torch.uint8, device=f"cuda:{local}")
    dbase = [torch.frombuffer(bytearray(bases[k][spans[k][0]:spans[k][1]]), dtype=torch.uint8).to(dev.device)
             for k in range(c5_data.N_BASE)]
    layout, pos = [], 0  # per batch: (span offset, bytes, records, segment ends, segment file offsets)
    for bt in batches:
        lo = pos
        ends, foffs = [], []
        for f in bt:
            k = f % c5_data.N_BASE
            n, cut = body_len[k], rel[k][rot(f)]
            dev[pos:pos + n - cut].copy_(dbase[k][cut:])  # blocks rot .. end, then 0 .. rot - 1
            dev[pos + n - cut:pos + n].copy_(dbase[k][:cut])
            pos += n
            ends.append(pos - lo)
            foffs.append(spans[k][0])
        layout.append((lo, pos - lo, sum(metas[f % c5_data.N_BASE]["nrec"] for f in bt), ends, foffs))
    del dbase
    torch.cuda.synchronize()
    biggest = max((n for _, n, _, _, _ in layout), default=0)
    max_items = max((k for _, _, k, _, _ in layout), default=0)
    ctxs = [gpu.Context(local, max_span_bytes=max(biggest, 32768), max_items=max_items + 1024, item_end=True)
            for _ in range(2)]

    def launch(ctx, i):
        lo, nbytes, _, ends, foffs = layout[i]
        ctx.scan_device_segments_async(dev.data_ptr() + lo, nbytes, ends, foffs, gpu.RIO_CODEC_FLATE)

    def done(r, i):
        assert r.err.code == 0 and r.stop == gpu.RIO_STOP_EOF and r.n_items == layout[i][2], \
            (r.err.msg, r.n_items, layout[i][2])
        return int(r.n_items)

    # parity pass: every file of the rank against its base's records and index
    files_ok = 0
    if mine:
        want, blk_bytes = {}, {}
        for k in range(c5_data.N_BASE):
            recs = c5_data.base_records(k)
            w = b"".join(recs)
            want[k] = torch.frombuffer(bytearray(w), dtype=torch.uint8).to(dev.device)
            lens = np.fromiter((len(x) for x in recs), dtype=np.int64, count=len(recs))
            cum = np.concatenate([[0], np.cumsum(lens)])
            blk_bytes[k] = cum[np.minimum(np.arange(len(index[k])) * c5_data.PER_BLOCK, len(recs))]
        for i, bt in enumerate(batches):
            launch(ctxs[0], i)
            r = ctxs[0].sync()
            done(r, i)
            nb = int(r.n_blocks)
            u64 = lambda p, n: np.frombuffer(gpu.dev_to_host(ctypes.cast(p, ctypes.c_void_p).value, 8 * n),
                                             dtype=np.uint64).astype(np.int64)
            first = u64(r.block_first_item, nb + 1)
            end = u64(r.item_end, int(r.n_items))
            data_ = u64(r.block_data, nb) & ((1 << 63) - 1)  # (bit 63: in records)
            foff = u64(r.block_first_off, nb)
            seg = u64(r.block_segment, nb)
            boff = u64(r.block_file_off, nb)
            rec = devcheck_copy(r.records, int(r.records_len), dev.device)
            nbytes = np.where(first[1:] > first[:-1], end[np.maximum(first[1:] - 1, 0)], 0)
            bounds = np.searchsorted(seg, np.arange(len(bt) + 1))
            for j, f in enumerate(bt):
                k = f % c5_data.N_BASE
                b0, b1 = bounds[j], bounds[j + 1]
                got = torch.cat([rec[int(data_[b] + foff[b]):int(data_[b] + foff[b] + nbytes[b])]
                                 for b in range(b0, b1)])
                br = int(blk_bytes[k][rot(f)])  # the records of the base's blocks before rot
                tail = want[k].numel() - br
                if (got.numel() == want[k].numel() and torch.equal(got[:tail], want[k][br:])
                        and torch.equal(got[tail:], want[k][:br]) and boff[b0:b1].tolist() == file_index(f)):
                    files_ok += 1
            del rec
        del want
    parity = files_ok == len(mine)

    steps = max(1, min(args.steps, 3))

    def step():
        n, pending = 0, [None, None]
        for i in range(len(layout)):
            c = i % 2
            if pending[c] is not None:
                n += done(ctxs[c].sync(), pending[c])
            launch(ctxs[c], i)
            pending[c] = i
        for c in range(2):
            if pending[c] is not None:
                n += done(ctxs[c].sync(), pending[c])
        return n

    step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        n_items = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = (time.perf_counter() - t0) / steps
    all_bytes = sum(sizes)
    ok = parity
    if dist is not None:
        t = torch.tensor([dt, 0.0 if ok else 1.0], device=coll_dev(local), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, ok = float(t[0].item()), t[1].item() == 0.0
    # the ordered-output prefix: where this rank's records land in the file-set
    # order (RCCL all_gather; at N = 1 through a one-rank RCCL group of its own)
    import torch.distributed as tdist
    own = not tdist.is_initialized()
    if own:
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        tdist.init_process_group("gloo" if REHEARSE else "nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                 world_size=1, device_id=None if REHEARSE else torch.device("cuda", local))
    my_bytes = sum(metas[f % c5_data.N_BASE]["rec_bytes"] for f in mine)
    pre = shard.ordered_prefix(n_items, my_bytes)
    prefix = {"backend": tdist.get_backend(), "world": tdist.get_world_size(), "item_offset": pre[0],
              "byte_offset": pre[1], "total_items": pre[2], "total_bytes": pre[3]}
    if own:
        tdist.destroy_process_group()
    for c in ctxs:
        c.close()
    del dev
    torch.cuda.empty_cache()
    return {"metric": "recordio scan GiB/s device-resident (compressed in), C5 1024 trailer-indexed flate files",
            "value": round(all_bytes / dt / 2 ** 30, 2), "unit": "GiB/s", "n_gpus": world,
            "scaling": "strong", "ms_per_step": round(dt * 1e3, 3), "steps": steps, "parity": ok,
            "parity_files_checked": len(mine), "parity_files_ok": files_ok, "ordered_prefix": prefix,
            "config": {"files": c5_data.N_FILES, "file_record_bytes": c5_data.FILE_RECORD_BYTES,
                       "records_per_block": c5_data.PER_BLOCK, "distinct_base_files": c5_data.N_BASE,
                       "note": "file f is base f mod %d with its blocks rotated by a file-specific count: "
                               "1024 distinct block layouts and indexes (each decoded and checked on its own)"
                               % c5_data.N_BASE,
                       "files_bytes_total": all_bytes, "files_this_rank": len(mine),
                       "batches_this_rank": len(batches), "launch": "rio_scan_device_segments_async, "
                       "one per batch, batches alternating over 2 contexts (streams)", "gen_s": round(gen_s, 1)}}


def devcheck_copy(ptr, nbytes, device):
    import devcheck
    return devcheck.dev_copy(ptr, nbytes, device)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--replicas", type=int, default=0, help="C2 replicas (0: %d x the rank's memory share)" % REPLICAS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-flate", action="store_true", help="skip the C3 flate measurement (configs[2])")
    ap.add_argument("--flate-replicas", type=int, default=0, help="0: enough for 10 GiB of records")
    ap.add_argument("--no-zstd", action="store_true", help="skip the C4 zstd measurement (configs[3])")
    ap.add_argument("--zstd-replicas", type=int, default=0, help="0: enough for 10 GiB of records")
    ap.add_argument("--zstd-contexts", type=int, default=1,
                    help="C4: the span's parts scanned by their own contexts, in flight together (1: one context)")
    ap.add_argument("--zstd-pipeline", type=int, default=2,
                    help="C4: steps alternate over this many contexts, each launched before the previous is "
                         "collected (1: one step at a time; the line reports that rate as `serial` too)")
    ap.add_argument("--no-flate16k", action="store_true", help="skip C3 at MaxItems 16384 (configs[2] sensitivity)")
    ap.add_argument("--flate-pipeline", type=int, default=3,
                    help="C3: context sets steps rotate over (n - 1 in flight beside the one collected; 1: serial)")
    ap.add_argument("--flate16k-pipeline", type=int, default=3,
                    help="C3 at MaxItems 16384: context sets steps rotate over (n - 1 in flight beside the one collected)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host file in, records out) line")
    ap.add_argument("--e2e-gib", type=float, default=2.0, help="end-to-end: file size per workload")
    ap.add_argument("--cpu-s", type=float, default=4.0, help="seconds per CPU-baseline measurement")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 many-file measurement (configs[4])")
    ap.add_argument("--c2-contexts", type=int, default=2, help="C2: contexts the steps rotate over (1-3; n > 1: n - 1 steps in flight beside the one collected)")
    ap.add_argument("--c5-batch-gib", type=float, default=4.0, help="file bodies per decode batch")
    ap.add_argument("--c5-cache", default="/tmp", help="host directory caching the C5 base files")
    ap.add_argument("--mem-share", type=float, default=0.0,
                    help="scale of the auto-sized workloads per rank (0: 1, or 1/world in a RIO_BENCH_REHEARSE run)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start torchrun as a child before anything touches
        # the GPU here, and exit with its status (never exec over this process)
        import socket
        import subprocess
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 and REHEARSE:  # every rank on GPU 0, collectives over gloo
        import faulthandler
        faulthandler.dump_traceback_later(100, repeat=True)  # (a stalled rehearsal shows where)
        import torch.distributed as dist
        local = 0
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    elif world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

    from base_amd.recordio import gpu
    gpu.load()  # refuses a library whose build id is not this tree's (base_amd/build.py)
    if args.replicas <= 0:
        args.replicas = max(1, int(round(REPLICAS * mem_share(args, world))))

    progress(rank, "C2: %d GPU(s)" % world)
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
    # items are views into the span (RIO_CFG_ITEM_END: the cumSize-shaped output,
    # 8 B per item); only chunk-straddling items are gathered (side buffer)
    # double-buffered: step i runs on context i % 2 (its own stream and result
    # buffers), launched before step i - 1's results are collected, so the
    # host's per-step work (sync, result read-back, the next enqueue) overlaps
    # the GPU's -- a scanner's read-ahead pipeline (--c2-contexts 1: one context,
    # each step synchronous)
    nctx = max(1, min(3, args.c2_contexts))
    ctxs = [gpu.Context(local, max_span_bytes=total, max_items=n_items + 1024, item_end=True)
            for _ in range(nctx)]
    span_ptr = dev.data_ptr() + CHUNK
    span_len = total - CHUNK

    def launch(c):
        ctxs[c].scan_device_async(span_ptr, span_len, CHUNK, gpu.RIO_CODEC_NONE)

    launch(0)
    b = ctxs[0].sync()
    assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
    assert b.n_items == n_items, (b.n_items, n_items)
    bb = b
    crc_ms, stage_sum = [], np.zeros(5)
    kern_ms = []

    def run(steps, record):
        out, pending = None, None

        def collect(c):
            r = ctxs[c].sync()
            if record:
                st = ctxs[c].stage_times()
                crc_ms.append(st[2])
                stage_sum[:] += np.array(st)
                kern_ms.append(r.kernel_ms)
            return r

        inflight = []  # contexts with a step launched and not yet collected, oldest first
        for i in range(steps):
            c = i % nctx
            if nctx == 1 and inflight:
                out = collect(inflight.pop(0))
            launch(c)
            inflight.append(c)
            if nctx > 1 and len(inflight) >= nctx:
                out = collect(inflight.pop(0))
        while inflight:
            out = collect(inflight.pop(0))
        return out

    run(args.warmup, False)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bb = run(args.steps, True)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    # parity of the timed path: the last step's output, every record of every
    # replica gathered on the GPU against the generator's records (tools/devcheck.py)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import devcheck
    want, want_len = devcheck.records_tensors(c2_records(), dev.device)
    chk = devcheck.check_replicated(bb, dev[CHUNK:], want, want_len, args.replicas)
    del want, want_len
    ok = bool(chk["ok"])
    if dist is not None:
        t = torch.tensor([dt, 0.0 if ok else 1.0], device=coll_dev(local), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, ok = float(t[0].item()), t[1].item() == 0.0
    ms_per_step = dt / args.steps * 1e3
    in_bytes = span_len * world
    value = in_bytes * args.steps / dt / 2 ** 30

    # k_crc alone: with two contexts its launches share the GPU with the other
    # context's parse, so its launch time is not its own. A few steps on one
    # context, each synchronous (after the timed region), time it alone -- the
    # roofline's kernel_ms -- and give the one-context step beside the timed one.
    one_crc, one_ms = [], []
    for i in range(max(3, min(args.steps, 10))):
        t1 = time.perf_counter()
        launch(0)
        ctxs[0].sync()
        one_ms.append((time.perf_counter() - t1) * 1e3)
        one_crc.append(ctxs[0].stage_times()[2])
    one_step = float(np.median(one_ms))
    # roofline of the dominant kernel (k_crc): it reads every chunk byte once
    # (B_in per launch; DESIGN.md "Roofline")
    crc_two = float(np.mean(crc_ms))
    crc_avg = float(np.mean(one_crc)) if nctx > 1 else crc_two
    alg = span_len
    achieved = alg / (crc_avg * 1e-3) / 1e9
    # whole pipeline (SURVEY.md §8(d) B_alg): chunk bytes in + item_end (8 B per
    # item) + block metadata (block_first_item, block_data, block_first_off: 24 B
    # per block) + the straddlers gathered (one ~256 B record per 2-chunk block)
    pipe_alg = span_len + 8 * n_items + 24 * int(b.n_blocks) + 256 * int(b.n_blocks)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("k_crc", args.replicas),
            "kernel": "k_crc", "kernel_ms": round(crc_avg, 3),
            "kernel_ms_source": "HIP events around k_crc on its stream, one context, steps synchronous",
            "kernel_ms_two_contexts": round(crc_two, 3),
            "alg_bytes_per_launch": alg,
            # per-step latency, first kernel's start to the last's end (with two
            # contexts, two steps are in flight: the latency spans both)
            "pipeline_latency_ms": round(float(np.mean(kern_ms)), 3),
            "pipeline_alg_GBs": round(pipe_alg / (ms_per_step * 1e-3) / 1e9, 1),
            # the whole step against the peak (k_crc's launches run beside the other
            # context's parse -- k_lean_end fits on each CU beside it, DESIGN.md
            # k_crc design -- so its launch time includes that sharing)
            "step_frac": round(pipe_alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "stage_ms": [round(x / args.steps, 3) for x in stage_sum]}

    out = {"metric": "recordio scan GiB/s device-resident (compressed in) at 1/2/4/8 MI355X",
           "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "config": {"workload": "C2: none codec, 1e6 x 256 B records x %d replicas, 253 per block (MaxItems=252) "
                                  "(64 KiB blocks), chunk CRC32 + packed-unpack" % args.replicas,
                      "records_per_gpu": int(n_items), "record_bytes": RECORD_SIZE,
                      "parallelism": f"{world} GPU(s), independent replica sets",
                      "bytes_in_per_gpu": span_len},
           "roofline": roof,
           "contexts": nctx,
           # the same step on one context, each step synchronous (host sync and
           # enqueue included): the serial rate beside the pipelined one
           "one_context": {"ms_per_step": round(one_step, 3),
                           "value": round(in_bytes / world / (one_step * 1e-3) / 2 ** 30, 2)},
           "parity": {"ok": ok, "checked": "every record of every replica of the last timed step vs the "
                                           "generator (on the GPU)", "items_checked": chk["items_checked"],
                      "bytes_checked": chk["bytes_checked"], "output": "item_end (RIO_CFG_ITEM_END)"},
           "build_id": gpu.build_id(), "lib": os.path.relpath(gpu.LIB_PATH, ROOT)}
    for c in ctxs:
        c.close()
    del dev
    torch.cuda.empty_cache()
    progress(rank, "C2 %.2f GiB/s" % value)
    # the end-to-end scans first among the sub-lines: after the device-resident
    # workloads (tens of GB of generated files and pinned staging allocated and
    # freed) the same scans measured ~10 % slower (C2 40 against 45-47 GiB/s,
    # C3 13.7 against 15-16) than in a process of their own
    if world == 1 and not args.no_e2e:  # the drop-in path, PCIe included (north_star)
        progress(rank, "end-to-end scans")
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_e2e
        out["e2e"] = bench_e2e.run_e2e(local, args.e2e_gib)
    if not args.no_flate:
        progress(rank, "C3 flate")
        out["c3_flate"] = c3_flate(args, local, world, dist)
    if not args.no_flate16k:
        progress(rank, "C3 flate at MaxItems 16384")
        out["c3_flate_16k"] = c3_flate_16k(args, local, world, dist)
    if not args.no_zstd:
        progress(rank, "C4 zstd")
        out["c4_zstd"] = c4_zstd(args, local, world, dist)
    if not args.no_c5:
        progress(rank, "C5 1024 files")
        out["c5_flate"] = c5_flate(args, local, rank, world, dist)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress(rank, "CPU baselines")
        out["cpu_baseline"], out["cpu_baseline_all_cores"], out["c1_cpu"] = cpu_baselines(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
