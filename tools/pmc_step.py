"""Per-kernel HBM bytes of one pipeline step from rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE in separate runs, tools/gpu_r06.sh pmcc4 / pmc16k /
pmcc3), for the bench lines' roofline `traffic` (tools/bench_flate.py
pmc_decode_traffic).

Each kernel's value is its largest dispatch (the runs do one step of
`--replicas` replicas after smaller parity / sizing scans). FETCH_SIZE and
WRITE_SIZE are in KB (1024 B); on gfx950 FETCH_SIZE reports half the bytes of
wide streaming reads (MI355X_MICROARCH.md, HBM section), so fetch_bytes is the
doubled counter and fetch_bytes_raw the counter as read.

  python tools/pmc_step.py --replicas 8 --fetch DIR --write DIR > profiles/r06_c4_pmc.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def per_kernel_max(d):
    best = defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                if not k.startswith("rio::"):  # (torch's parity-check kernels)
                    continue
                best[k] = max(best[k], float(r["Counter_Value"]) * 1024)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--cmd", default="")
    a = ap.parse_args()
    fe, wr = per_kernel_max(a.fetch), per_kernel_max(a.write)
    out = {"pmc_replicas": a.replicas, "cmd": a.cmd,
           "note": "per kernel, its largest dispatch; fetch_bytes = 2 x FETCH_SIZE (gfx950 correction)",
           "per_kernel": {}}
    for k in sorted(set(fe) | set(wr)):
        out["per_kernel"][k] = {"fetch_bytes_raw": int(fe.get(k, 0)), "fetch_bytes": int(2 * fe.get(k, 0)),
                                "write_bytes": int(wr.get(k, 0))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
