"""Zstd workload (BASELINE.json configs[3]) on one MI355X.

A zstd recordio file (tools/c4_data.py: record sizes log-uniform 64 B-64 KiB,
>= 1 MiB blocks, level 5) is built on the host, copied to HBM and its body
replicated to ~10 GiB of records; one step = the scan pipeline over the whole
device-resident span (chunk CRC + zstd decode + packed unpack). Parity: the base
file's items against the generator's records. Prints one JSON line.

  python tools/bench_zstd.py [--base-mib 128] [--replicas 80] [--steps 5]
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


def load_or_make(base_mib, workers, path=None):
    """The C4 base file; with `path`, cached there (a profiled run loads it: libzstd
    cannot be called under rocprofv3, whose own zstd symbols interpose)."""
    import c4_data
    if path and os.path.exists(path):
        with open(path + ".json") as f:
            m = json.load(f)
        with open(path, "rb") as f:
            return f.read(), m["nblk"], m["nrec"], m["rec_bytes"]
    data, nblk, nrec, rec_bytes = c4_data.make_file(base_mib << 20, workers=workers)
    if path:
        with open(path, "wb") as f:
            f.write(data)
        with open(path + ".json", "w") as f:
            json.dump({"nblk": nblk, "nrec": nrec, "rec_bytes": rec_bytes}, f)
    return data, nblk, nrec, rec_bytes


def run_c4(base_mib=128, replicas=0, steps=5, warmup=1, device=0, check=True, cpu_s=0.0, workers=16, data_path=None,
           contexts=1, pipeline=1, share=1.0):
    """The C4 workload (replicas=0: enough for 10 GiB of records); cpu_s > 0 adds
    the one-core and all-core CPU baselines (libzstd) on the base file."""
    import bench_flate
    import c4_data
    from base_amd.recordio import gpu

    t0 = time.perf_counter()
    data, nblk, nrec, rec_bytes = load_or_make(base_mib, workers, data_path)
    gen_s = time.perf_counter() - t0
    if replicas <= 0:
        replicas = max(1, int(round(bench_flate.replicas_for(rec_bytes) * share)))
    roof = {"kernels": bench_flate.ZSTD_DECODE_KERNELS,
            "pmc": os.path.join(ROOT, "profiles", "r06_c4_pmc.json"),
            "dominant": bench_flate.dominant_kernel(
                os.path.join(ROOT, "profiles", "r06_c4_kernel_trace_summary.json"), "k_zstd_seq4"),
            "note": "compressed bytes in + decoded records out over the decode stage; the sequence pass is bound "
                    "by its FSE chains' instruction issue and the execution pass by far-source loads (DESIGN.md §4)"}
    res = bench_flate.measure(data, nrec, rec_bytes, lambda: c4_data.all_records(nblk), gpu.RIO_CODEC_ZSTD,
                              "C4-like zstd level 5, records 64 B-64 KiB log-uniform, 1 MiB blocks",
                              replicas, steps, warmup, device, check, contexts=contexts,
                              pipeline=pipeline, roof=roof)
    res["config"]["gen_s"] = round(gen_s, 1)
    if cpu_s > 0:
        import cpu_base
        res["cpu_baseline"], res["cpu_baseline_all_cores"] = cpu_base.baselines(
            data, 2, nrec, "C4 base file", cpu_s)
    return dict({"metric": "recordio scan GiB/s device-resident (compressed in), zstd"}, **res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base-mib", type=int, default=128)
    ap.add_argument("--replicas", type=int, default=0, help="0: enough for 10 GiB of records")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-s", type=float, default=0.0)
    ap.add_argument("--workers", type=int, default=16, help="generator processes (1: in-process)")
    ap.add_argument("--data", default=None, help="cache the base file here (load it if present)")
    ap.add_argument("--make-data", action="store_true", help="only write --data, no GPU")
    ap.add_argument("--contexts", type=int, default=1, help="parts of the span scanned by their own contexts, in flight together")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="steps alternate over this many context sets, each launched before the previous is collected")
    args = ap.parse_args()
    if args.make_data:
        load_or_make(args.base_mib, args.workers, args.data)
        return
    print(json.dumps(run_c4(args.base_mib, args.replicas, args.steps, args.warmup, cpu_s=args.cpu_s,
                            workers=args.workers, data_path=args.data, contexts=args.contexts,
                            pipeline=args.pipeline)), flush=True)


if __name__ == "__main__":
    main()
