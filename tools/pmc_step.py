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


def per_kernel_max(d, last_step=None):
    """Per rio kernel: its largest dispatch, or (last_step = the name of a
    step's first kernel) the sum of its dispatches from that kernel's last
    dispatch on -- one whole step, whatever its kernels' launch counts."""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                rows.append((int(r["Dispatch_Id"]), k, float(r["Counter_Value"]) * 1024))
    best = defaultdict(float)
    if last_step:
        starts = [i for i, k, _ in rows if k == last_step]
        first = max(starts) if starts else 0
        for i, k, v in rows:
            if i >= first and k.startswith("rio::"):
                best[k] += v
        return best
    for _, k, v in rows:
        if k.startswith("rio::"):  # (torch's parity-check kernels)
            best[k] = max(best[k], v)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--cmd", default="")
    ap.add_argument("--last-step", default=None,
                    help="sum each kernel's dispatches of the run's last step, from this kernel's last dispatch on")
    a = ap.parse_args()
    fe, wr = per_kernel_max(a.fetch, a.last_step), per_kernel_max(a.write, a.last_step)
    how = ("per kernel, the sum of its dispatches in the run's last step (from the last %s)" % a.last_step
           if a.last_step else "per kernel, its largest dispatch")
    out = {"pmc_replicas": a.replicas, "cmd": a.cmd,
           "note": how + "; fetch_bytes = 2 x FETCH_SIZE (gfx950 correction)",
           "per_kernel": {}}
    for k in sorted(set(fe) | set(wr)):
        out["per_kernel"][k] = {"fetch_bytes_raw": int(fe.get(k, 0)), "fetch_bytes": int(2 * fe.get(k, 0)),
                                "write_bytes": int(wr.get(k, 0))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
