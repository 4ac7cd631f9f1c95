"""Flate workload (BASELINE.json configs[2]) on one MI355X.

A FASTQ-like flate recordio file (tools/c3_data.py; 1024 records per block) is
built on the host, copied to HBM and its body replicated to ~10 GiB of records;
one step = the scan pipeline over the whole device-resident span (chunk CRC +
DEFLATE decode + packed unpack). Parity: the base file's items (device path)
against the generator's records. Prints one JSON line.

  python tools/bench_flate.py [--base-mib 128] [--replicas 80] [--steps 5]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md), as bench.py


def pmc_decode_traffic(pmc_file, kernels, replicas):
    """HBM bytes per step of the decode stage's kernels from a committed PMC pass
    (tools/gpu_r06.sh pmcc4 / pmc16k: rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE over
    a one-step run of `pmc_replicas` replicas, FETCH_SIZE doubled per
    MI355X_MICROARCH.md), scaled to this run's replica count; None without it."""
    if not pmc_file or not os.path.exists(pmc_file):
        return None
    with open(pmc_file) as f:
        pm = json.load(f)
    n = pm.get("pmc_replicas")
    tot = 0.0
    if not n:
        return None
    for k in kernels:  # (a kernel the run did not launch -- e.g. no block took that path -- adds nothing)
        e = pm.get("per_kernel", {}).get(k)
        if e:
            tot += e["fetch_bytes"] + e["write_bytes"]
    return int(tot * replicas / n)


def dominant_kernel(trace_summary, name):
    """A kernel's median launch time from a committed one-context kernel-trace
    summary (tools/ktrace_summary.py --json over rocprofv3 --kernel-trace of the
    workload's own bench command): {kernel, ms, source}, or None."""
    if not os.path.exists(trace_summary):
        return None
    with open(trace_summary) as f:
        tr = json.load(f)
    for k, v in tr.items():
        if name in k:
            return {"kernel": name, "median_ms": v["median_ms"], "launches": v["calls"],
                    "source": os.path.relpath(trace_summary, ROOT)}
    return None


FLATE_DECODE_KERNELS = ["rio::k_codec_prepare", "rio::k_flate_sync<1>", "rio::k_flate_sync<4>", "rio::k_flate_plan",
                        "rio::k_flate_tok", "rio::k_flate_lz2", "rio::k_flate_seg", "rio::k_flate_segfix",
                        "rio::k_inflate_exact"]
ZSTD_DECODE_KERNELS = ["rio::k_zstd_size", "rio::k_zstd_ent", "rio::k_zstd_seq4", "rio::k_zstd_seq2", "rio::k_zstd_fix", "rio::k_zstd_exec",
                       "rio::k_zstd"]


def measure(data, nrec, rec_bytes, want_fn, codec, workload, replicas, steps, warmup, device=0, check=True,
            flate_split=True, contexts=1, pipeline=1, roof=None):
    """One compressed workload on cuda:`device`: the base file `data` copied to
    HBM, its body replicated `replicas` times; one step = the scan pipeline over
    the whole device-resident span. Parity: the base file's items (device path)
    against want_fn() by SHA-256 and lengths. Returns the measurement dict.
    contexts > 1: the span is cut at replica boundaries into that many parts, each
    scanned by its own context (own stream), all launched before any is collected
    -- a scanner's consecutive spans in flight together."""
    import numpy as np
    import torch
    from base_amd.recordio import gpu

    CH = 32768
    body = data[CH:]
    total = CH + replicas * len(body)
    dev = torch.empty(total, dtype=torch.uint8, device=f"cuda:{device}")
    dev[:len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    for r in range(1, replicas):
        dev[CH + r * len(body):CH + (r + 1) * len(body)].copy_(dev[CH:len(data)])
    torch.cuda.synchronize()

    parity = None
    if check:  # the base file's items (device path, views into the decoded blocks)
        ctx1 = gpu.Context(device, max_span_bytes=len(body) + CH)
        b = ctx1.scan_device(dev.data_ptr() + CH, len(body), file_off=CH, is_file_end=True, codec=codec)
        assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
        items = gpu.device_batch_items(b, body)
        want = want_fn()  # (kept for the timed-output check)
        h_got = hashlib.sha256(b"".join(items)).hexdigest()
        h_want = hashlib.sha256(b"".join(want)).hexdigest()
        parity = (len(items) == nrec and h_got == h_want and [len(x) for x in items] == [len(x) for x in want])
        ctx1.close()

    span_len = total - CH
    nctx = max(1, min(contexts, replicas))
    cuts = [replicas * k // nctx for k in range(nctx + 1)]  # replica ranges of the parts
    parts = [(CH + a * len(body), (z - a) * len(body), z - a) for a, z in zip(cuts[:-1], cuts[1:])]
    npipe = max(1, pipeline)
    # pipeline > 1: consecutive steps alternate over that many context sets, step i
    # launched before step i - 1 is collected (a scanner's read-ahead: one span's
    # copy pass beside the next span's Huffman pass)
    sets = [[gpu.Context(device, max_span_bytes=n + CH, max_items=nrec * r + 1024, item_end=True,
                         flate_split=flate_split) for _, n, r in parts] for _ in range(npipe)]
    ctxs = sets[0]
    base = dev.data_ptr()

    def launch(cs):
        for c, (o, n, _) in zip(cs, parts):
            c.scan_device_async(base + o, n, o, codec)

    for cs in sets:  # (every context's first scan sizes its buffers)
        launch(cs)
        bbs = [c.sync() for c in cs]
        for bb, (_, _, r) in zip(bbs, parts):
            assert bb.stop == gpu.RIO_STOP_EOF and bb.err.code == 0, bb.err.msg
            assert bb.n_items == nrec * r

    def run(n, record):
        out, last = None, ctxs
        inflight = []  # context sets with a step launched and not yet collected, oldest first

        def collect():
            nonlocal out, last
            last = inflight.pop(0)
            out = [c.sync() for c in last]
            if record:
                stages.append(last[0].stage_times())

        for i in range(n):
            cs = sets[i % npipe]
            if cs in inflight:  # (the oldest: npipe steps in flight)
                collect()
            launch(cs)
            inflight.append(cs)
            if npipe == 1:
                collect()
            elif len(inflight) == npipe:  # collect the oldest once the next set is in flight
                collect()
        while inflight:
            collect()
        return out, last

    stages = []
    run(warmup, False)
    serial = None
    if npipe > 1:  # the same steps one at a time on one context set, for comparison
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            launch(ctxs)
            for c in ctxs:
                c.sync()
        serial = (time.perf_counter() - t0) / steps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bbs, last = run(steps, True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    stages = stages or [[0.0] * 5]
    st = np.mean(np.array(stages), axis=0)
    # the decode stage alone: a few steps on one context set, each synchronous
    # (after the timed region), its HIP events around the codec's kernels --
    # the roofline's kernel_ms, as bench.py times k_crc for C2
    dec_one = []
    if roof is not None and len(parts) == 1:
        for _ in range(3):
            launch(ctxs)
            ctxs[0].sync()
            dec_one.append(ctxs[0].stage_times()[1])
    timed_parity = None
    if check:  # the last timed step's output: every record of every replica, on the GPU
        import devcheck
        w, wl = devcheck.records_tensors(want, dev.device)
        timed_parity = {"ok": True, "items_checked": 0, "bytes_checked": 0}
        for bb, (o, n, r) in zip(bbs, parts):
            chk = devcheck.check_replicated(bb, dev[o:o + n], w, wl, r)
            timed_parity["ok"] = timed_parity["ok"] and bool(chk["ok"])
            timed_parity["items_checked"] += chk["items_checked"]
            timed_parity["bytes_checked"] += chk["bytes_checked"]
        del w, wl
    out_bytes = rec_bytes * replicas
    roofline = None
    if dec_one:
        # algorithmic bytes of the decode stage per launch: the compressed span
        # read once + the decoded records written once (SURVEY.md §8(d) B_in + B_rec)
        alg = span_len + out_bytes
        ms = float(np.median(dec_one))
        ach = alg / (ms * 1e-3) / 1e9
        roofline = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": pmc_decode_traffic(roof.get("pmc"), roof["kernels"], replicas),
                    "kernel": "decode stage (%s)" % ", ".join(roof["kernels"]), "kernel_ms": round(ms, 3),
                    "kernel_ms_source": "HIP events around the decode stage on its stream, one context set, steps "
                                        "synchronous",
                    "alg_bytes_per_launch": alg, "dominant_kernel": roof.get("dominant"),
                    "note": roof.get("note")}
    split_blocks = sum(c.flate_split_blocks() for c in last) if codec == gpu.RIO_CODEC_FLATE else 0
    for cs in sets:
        for c in cs:
            c.close()
    del dev
    torch.cuda.empty_cache()
    return {
        "value": round(span_len / dt / 2 ** 30, 2), "unit": "GiB/s",
        "out_GiBs": round(out_bytes / dt / 2 ** 30, 2),
        "ms_per_step": round(dt * 1e3, 3),
        "stage_ms": {"parse": round(st[0], 3), "decode": round(st[1], 3), "crc": round(st[2], 3),
                     "meta": round(st[3], 3), "total": round(st[4], 3)},
        "decode_in_GiBs": round(span_len / (st[1] * 1e-3) / 2 ** 30, 2) if st[1] > 0 else None,
        "config": {"workload": workload, "base_file_bytes": len(data), "base_records": nrec,
                   "base_record_bytes": rec_bytes, "replicas": replicas, "span_bytes": span_len,
                   "records_bytes": out_bytes},
        "parity": parity and bool(timed_parity and timed_parity["ok"]),
        "parity_timed_output": timed_parity,
        "roofline": roofline,
        "split_blocks": split_blocks, "contexts": nctx, "pipeline": npipe,
        "serial": None if serial is None else {
            "value": round(span_len / serial / 2 ** 30, 2), "ms_per_step": round(serial * 1e3, 3),
            "note": "the same steps one at a time (each collected before the next is launched)"}}


TARGET_RECORD_BYTES = 10 << 30  # configs[2]: 10 GiB of uncompressed records


def replicas_for(rec_bytes: int) -> int:
    """Replicas of the base file that reach >= 10 GiB of records."""
    return -(-TARGET_RECORD_BYTES // rec_bytes)


def run_c3(base_mib=128, replicas=0, steps=5, warmup=1, per_block=1024, device=0, check=True, cpu_s=0.0,
           flate_split=True, contexts=1, pipeline=1, share=1.0):
    """The C3 workload on cuda:`device` (replicas=0: enough for 10 GiB of records);
    returns the measurement dict (no print). cpu_s > 0 adds the one-core and
    all-core CPU baselines (zlib inflate) on the base file."""
    import c3_data
    from base_amd.recordio import gpu

    t0 = time.perf_counter()
    data, nrec, rec_bytes = c3_data.make_file(base_mib << 20, per_block, workers=16)
    gen_s = time.perf_counter() - t0

    def want():
        w = []
        for first in range(0, nrec, per_block):
            w.extend(c3_data.records(first, min(per_block, nrec - first)))
        return w

    if replicas <= 0:
        replicas = max(1, int(round(replicas_for(rec_bytes) * share)))
    tag = "c3_16k" if per_block >= 16384 else "c3"
    roof = {"kernels": FLATE_DECODE_KERNELS, "pmc": os.path.join(ROOT, "profiles", "r06_%s_pmc.json" % tag),
            "dominant": dominant_kernel(os.path.join(ROOT, "profiles", "r06_%s_kernel_trace_summary.json" % tag),
                                        "k_flate_seg" if per_block >= 16384 else "k_flate_sync<1>"),
            "note": "compressed bytes in + decoded records out over the decode stage; the Huffman and copy "
                    "passes are instruction-issue and latency bound (DESIGN.md §4), so frac is far below 1"}
    res = measure(data, nrec, rec_bytes, want, gpu.RIO_CODEC_FLATE,
                  "C3-like flate FASTQ, %d records/block" % per_block, replicas, steps, warmup, device, check,
                  flate_split, contexts, pipeline, roof=roof)
    res["config"]["gen_s"] = round(gen_s, 1)
    if cpu_s > 0:
        import cpu_base
        res["cpu_baseline"], res["cpu_baseline_all_cores"] = cpu_base.baselines(
            data, 1, nrec, "C3 base file", cpu_s)
    return dict({"metric": "recordio scan GiB/s device-resident (compressed in), flate"}, **res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base-mib", type=int, default=128)
    ap.add_argument("--replicas", type=int, default=0, help="0: enough for 10 GiB of records")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--per-block", type=int, default=1024)
    ap.add_argument("--cpu-s", type=float, default=0.0)
    ap.add_argument("--no-split", action="store_true", help="copy every block whole (RIO_CFG_FLATE_NO_SPLIT)")
    ap.add_argument("--contexts", type=int, default=1, help="parts of the span scanned by their own contexts, in flight together")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="steps alternate over this many context sets, each launched before the previous is collected")
    args = ap.parse_args()
    print(json.dumps(run_c3(args.base_mib, args.replicas, args.steps, args.warmup, args.per_block,
                            cpu_s=args.cpu_s, flate_split=not args.no_split, contexts=args.contexts,
                            pipeline=args.pipeline)), flush=True)


if __name__ == "__main__":
    main()
